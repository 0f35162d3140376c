// testlaw.hip — TEST FIXTURE (not product): constitutive laws that live OUTSIDE libmacroc_amd
// and plug into its Gauss-point callback boundary (-mat_law external, include/macroc_amd.h):
//  * testlaw_elastic_device(): an mcx_device_law whose homogenize launches its own kernel
//    (sigma = C eps, ctan = C per Gauss point) on the context's stream;
//  * micropp_C_*: a host library with the MicroPP C-wrapper call shapes the reference uses
//    (src/init.c:196-213, src/assembly.c:59,92,149, src/main.c:62,83, src/util.c:71,96),
//    isotropic elastic only, so the C driver can be linked against "a MicroPP" exactly as the
//    reference is (make driver-micropp).
// The isotropic tangent is formed as src/init.c's material values feed MicroPP's linear law:
// lambda = E nu / ((1+nu)(1-2nu)), mu = E / (2(1+nu)); sigma_k = sum_l C_kl eps_l, l ascending.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/macroc_amd.h"

namespace {

struct Iso {
  double C[36];
};

Iso iso(double E, double nu) {
  Iso m;
  const double lam = E * nu / ((1. + nu) * (1. - 2. * nu));
  const double mu = E / (2. * (1. + nu));
  for (int q = 0; q < 36; q++) m.C[q] = 0.;
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) m.C[a * 6 + b] = lam + (a == b ? 2. * mu : 0.);
  for (int a = 3; a < 6; a++) m.C[a * 6 + a] = mu;
  return m;
}

__global__ void k_testlaw(int64_t ngp, Iso m, const double* __restrict__ eps, double* __restrict__ sig,
                          double* __restrict__ ctan) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= ngp) return;
  double e[6];
  for (int l = 0; l < 6; l++) e[l] = eps[l * ngp + q];
  for (int k = 0; k < 6; k++) {
    double s = 0.;
    for (int l = 0; l < 6; l++) s += m.C[k * 6 + l] * e[l];
    sig[k * ngp + q] = s;
  }
  for (int kl = 0; kl < 36; kl++) ctan[kl * ngp + q] = m.C[kl];
}

struct DevState {
  Iso m;
  int calls = 0;
  int updates = 0;
};

int dev_homogenize(void* user, const mcx_gp_batch* b) {
  auto* st = static_cast<DevState*>(user);
  const unsigned blocks = (unsigned)((b->ngp + 255) / 256);
  hipLaunchKernelGGL(k_testlaw, dim3(blocks), dim3(256), 0, (hipStream_t)b->stream, b->ngp, st->m, b->eps, b->sig,
                     b->ctan);
  st->calls++;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

int dev_update(void* user) {
  static_cast<DevState*>(user)->updates++;
  return 0;
}

int dev_stats(void* user, int64_t* n, double* f) {
  (void)user;
  *n = 0;
  *f = -1.;
  return 0;
}

// host MicroPP stand-in state (one instance per process, like MicroPP's singleton)
struct Micro {
  double mat[2][4] = {};
  int ngp = 0;
  Iso m{};
  std::vector<double> eps, sig;
  int homog_calls = 0, updates = 0;
} g_micro;

}  // namespace

extern "C" {

int testlaw_elastic_device(mcx_device_law* out, double E, double nu) {
  auto* st = new DevState();
  st->m = iso(E, nu);
  out->homogenize = dev_homogenize;
  out->update_vars = dev_update;
  out->nonlinear_stats = dev_stats;
  out->user = st;
  return 0;
}

int testlaw_device_calls(const mcx_device_law* law, int* updates) {
  auto* st = static_cast<DevState*>(law->user);
  if (updates) *updates = st->updates;
  return st->calls;
}

// ---- micropp_c_wrapper.h call shapes (the reference's call sites)
void micropp_C_material_set(int id, double E, double nu, double Sy, double Ka, int type) {
  (void)type;
  if (id < 0 || id > 1) return;
  const double v[4] = {E, nu, Sy, Ka};
  std::memcpy(g_micro.mat[id], v, sizeof(v));
}
void micropp_C_material_print(int id) {
  std::printf("E = %e nu = %e Sy = %e Ka = %e\n", g_micro.mat[id][0], g_micro.mat[id][1], g_micro.mat[id][2],
              g_micro.mat[id][3]);
}
void micropp_C_create3(int ngp, int size[3], int micro_type, double params[4]) {
  (void)size;
  (void)micro_type;
  (void)params;
  g_micro.ngp = ngp;
  g_micro.m = iso(g_micro.mat[0][0], g_micro.mat[0][1]);
  g_micro.eps.assign((size_t)ngp * 6, 0.);
  g_micro.sig.assign((size_t)ngp * 6, 0.);
}
void micropp_C_print_info(void) { std::printf("micropp stand-in (test fixture): %d Gauss points\n", g_micro.ngp); }
void micropp_C_set_strain3(int gp, double strain[6]) {
  if (gp < 0 || gp >= g_micro.ngp) std::abort();
  std::memcpy(&g_micro.eps[(size_t)gp * 6], strain, 6 * sizeof(double));
}
void micropp_C_homogenize(void) {
  for (int q = 0; q < g_micro.ngp; q++)
    for (int k = 0; k < 6; k++) {
      double s = 0.;
      for (int l = 0; l < 6; l++) s += g_micro.m.C[k * 6 + l] * g_micro.eps[(size_t)q * 6 + l];
      g_micro.sig[(size_t)q * 6 + k] = s;
    }
  g_micro.homog_calls++;
}
void micropp_C_get_stress3(int gp, double stress[6]) {
  if (gp < 0 || gp >= g_micro.ngp) std::abort();
  std::memcpy(stress, &g_micro.sig[(size_t)gp * 6], 6 * sizeof(double));
}
void micropp_C_get_ctan3(int gp, double ctan[36]) {
  if (gp < 0 || gp >= g_micro.ngp) std::abort();
  std::memcpy(ctan, g_micro.m.C, 36 * sizeof(double));
}
void micropp_C_update_vars(void) { g_micro.updates++; }
int micropp_C_get_non_linear_gps(void) { return 0; }
double micropp_C_get_f_trial_max(void) { return -1.0; }
int micropp_C_homogenize_calls(void) { return g_micro.homog_calls; }

}  // extern "C"
