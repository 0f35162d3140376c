// Feasibility check for the value-indexed SpMV's wave-uniform path: does
// v_fmac_f64_dpp with row_newbcast:q give every lane of a 16-lane row src0 from lane q of that
// row on gfx950?  Prints one line per q and exits non-zero on a mismatch.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int Q>
__global__ void k_bcast(const double* __restrict__ a, const double* __restrict__ x, double* __restrict__ y) {
  const int l = threadIdx.x;
  const double av = a[l];
  const double xv = x[l];
  double acc = 1.0;
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc) : "v"(av), "v"(xv), "i"(Q));
  y[l] = acc;
}

int main() {
  double ha[64], hx[64], hy[64];
  for (int l = 0; l < 64; l++) { ha[l] = 100.0 + l; hx[l] = 0.5 * l + 1.0; }
  double *a, *x, *y;
  (void)hipMalloc(&a, 512); (void)hipMalloc(&x, 512); (void)hipMalloc(&y, 512);
  (void)hipMemcpy(a, ha, 512, hipMemcpyHostToDevice);
  (void)hipMemcpy(x, hx, 512, hipMemcpyHostToDevice);
  int bad = 0;
#define RUNQ(Q)                                                              \
  hipLaunchKernelGGL(k_bcast<Q>, dim3(1), dim3(64), 0, 0, a, x, y);          \
  (void)hipMemcpy(hy, y, 512, hipMemcpyDeviceToHost);                        \
  {                                                                          \
    int b = 0;                                                               \
    for (int l = 0; l < 64; l++) {                                           \
      const double want = 1.0 + ha[(l & ~15) + Q] * hx[l];                   \
      if (hy[l] != want) b++;                                                \
    }                                                                        \
    printf("row_newbcast:%d mismatching lanes %d (lane 17: %g, want %g)\n", Q, b, hy[17], \
           1.0 + ha[16 + Q] * hx[17]);                                       \
    bad += b;                                                                \
  }
  RUNQ(0) RUNQ(3) RUNQ(9) RUNQ(15)
  printf(bad ? "DPP row_newbcast f64: MISMATCH\n" : "DPP row_newbcast f64: ok\n");
  return bad ? 1 : 0;
}
