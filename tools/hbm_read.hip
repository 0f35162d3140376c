// hbm_read.hip — streaming-read ceiling of this MI355X: sum a large fp64 buffer with 16-B
// loads in the shapes the SpMV kernels use (per-wave contiguous chunks vs grid-stride, default
// vs non-temporal policy).  Calibrates "achievable" next to the 8 TB/s spec.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

// each wave reads CH consecutive 1-KB rows (the AIJ AoSoA group shape: CH = 122)
template <bool NT, int CH>
__global__ __launch_bounds__(256) void k_chunk(const double2* __restrict__ a, long nwaves, double* out) {
  const long w = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= nwaves) return;
  const double2* p = a + w * CH * 64 + (threadIdx.x & 63);
  double s0 = 0, s1 = 0;
#pragma unroll 16
  for (int q = 0; q < CH; q++) {
    double2 v;
    if (NT) {
      v.x = __builtin_nontemporal_load(&p[q * 64].x);
      v.y = __builtin_nontemporal_load(&p[q * 64].y);
    } else {
      v = p[q * 64];
    }
    s0 += v.x;
    s1 += v.y;
  }
  if (s0 + s1 == 12345.678) out[0] = s0;  // keep the loads
}

// same, block -> chunk permuted the way the SpMV maps XCDs to y-slabs (block b on XCD b&7
// reads slab b&7, step b>>3); STORE adds the SpMV's 3-double-per-lane y store
template <bool NT, int CH, int STORE>
__global__ __launch_bounds__(256) void k_chunk_xcd(const double2* __restrict__ a, long nblocks, double* out,
                                                   double* y) {
  const long b = blockIdx.x;
  const long per = (nblocks + 7) / 8;
  const long blk = (b & 7) * per + (b >> 3);
  if (blk >= nblocks) return;
  const long w = blk * 4 + (threadIdx.x >> 6);
  const double2* p = a + w * CH * 64 + (threadIdx.x & 63);
  double s0 = 0, s1 = 0;
#pragma unroll 16
  for (int q = 0; q < CH; q++) {
    double2 v;
    if (NT) {
      v.x = __builtin_nontemporal_load(&p[q * 64].x);
      v.y = __builtin_nontemporal_load(&p[q * 64].y);
    } else {
      v = p[q * 64];
    }
    s0 += v.x;
    s1 += v.y;
  }
  if (STORE == 1) {
    const long n = w * 64 + (threadIdx.x & 63);
    y[3 * n] = s0;
    y[3 * n + 1] = s1;
    y[3 * n + 2] = s0 - s1;
  } else if (STORE == 2) {  // through LDS: the wave's 192 doubles as 3 contiguous 512-B stores
    __shared__ double st[4][192];
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    st[wv][3 * l] = s0;
    st[wv][3 * l + 1] = s1;
    st[wv][3 * l + 2] = s0 - s1;
    __builtin_amdgcn_wave_barrier();
    double* yw = y + w * 192;
    yw[l] = st[wv][l];
    yw[64 + l] = st[wv][64 + l];
    yw[128 + l] = st[wv][128 + l];
  } else if (STORE == 4) {
    const long n = w * 64 + (threadIdx.x & 63);
    y[n] = s0 + s1;
  } else if (STORE == 3) {
    const long n = w * 64 + (threadIdx.x & 63);
    __builtin_nontemporal_store(s0, &y[3 * n]);
    __builtin_nontemporal_store(s1, &y[3 * n + 1]);
    __builtin_nontemporal_store(s0 - s1, &y[3 * n + 2]);
  } else if (s0 + s1 == 12345.678) {
    out[0] = s0;
  }
}

__global__ __launch_bounds__(256) void k_write(double* y, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = (double)i;
}

// grid-stride over 16-B elements
template <bool NT>
__global__ __launch_bounds__(256) void k_stride(const double2* __restrict__ a, long n, double* out) {
  double s0 = 0, s1 = 0;
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    double2 v;
    if (NT) {
      v.x = __builtin_nontemporal_load(&a[i].x);
      v.y = __builtin_nontemporal_load(&a[i].y);
    } else {
      v = a[i];
    }
    s0 += v.x;
    s1 += v.y;
  }
  if (s0 + s1 == 12345.678) out[0] = s0;
}

template <class F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; r++) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  return best;
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? std::atof(argv[1]) : 32.0;
  const int CH = 122;
  const long nwaves = (long)(gb * 1e9 / (CH * 1024.0));
  const long n16 = nwaves * CH * 64;
  const double bytes = 16.0 * n16;
  double2* a;
  double* out;
  CK(hipMalloc(&a, (size_t)bytes));
  CK(hipMalloc(&out, 8));
  CK(hipMemset(a, 0, (size_t)bytes));
  const int blocks = (int)((nwaves + 3) / 4);
  auto report = [&](const char* name, float ms) {
    std::printf("%-32s %8.3f ms  %7.0f GB/s\n", name, ms, bytes / ms / 1e6);
  };
  report("chunk122 default", timeit([&] { k_chunk<false, 122><<<blocks, 256>>>(a, nwaves, out); }, 10));
  report("chunk122 nt", timeit([&] { k_chunk<true, 122><<<blocks, 256>>>(a, nwaves, out); }, 10));
  double* y;
  CK(hipMalloc(&y, sizeof(double) * 3 * 64 * (size_t)nwaves));
  const long nblk = (nwaves + 3) / 4;
  const int nbx = (int)(((nblk + 7) / 8) * 8);
  report("chunk122 xcd-slab nt", timeit([&] { k_chunk_xcd<true, 122, 0><<<nbx, 256>>>(a, nblk, out, y); }, 10));
  report("chunk122 xcd-slab nt +y", timeit([&] { k_chunk_xcd<true, 122, 1><<<nbx, 256>>>(a, nblk, out, y); }, 10));
  report("chunk122 xcd-slab nt +y lds", timeit([&] { k_chunk_xcd<true, 122, 2><<<nbx, 256>>>(a, nblk, out, y); }, 10));
  report("chunk122 xcd-slab nt +y nt", timeit([&] { k_chunk_xcd<true, 122, 3><<<nbx, 256>>>(a, nblk, out, y); }, 10));
  report("chunk122 xcd-slab nt +y1", timeit([&] { k_chunk_xcd<true, 122, 4><<<nbx, 256>>>(a, nblk, out, y); }, 10));
  {
    const long ny = 3 * 64 * nwaves;
    float ms = timeit([&] { k_write<<<(int)((ny + 255) / 256), 256>>>(y, ny); }, 10);
    std::printf("%-32s %8.3f ms  %7.0f GB/s (%.0f MB)\n", "write y only", ms, 8.0 * ny / ms / 1e6, 8e-6 * ny);
  }
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  for (int per : {8, 16, 32}) {
    char nm[64];
    std::snprintf(nm, sizeof nm, "stride %d blk/CU default", per);
    report(nm, timeit([&] { k_stride<false><<<ncu * per, 256>>>(a, n16, out); }, 10));
    std::snprintf(nm, sizeof nm, "stride %d blk/CU nt", per);
    report(nm, timeit([&] { k_stride<true><<<ncu * per, 256>>>(a, n16, out); }, 10));
  }
  CK(hipFree(a));
  return 0;
}
