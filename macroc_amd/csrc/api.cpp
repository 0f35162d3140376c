// api.cpp — C-ABI (include/macroc_amd.h) of the MI355X MacroC Newton inner loop.
// Host control mirrors the reference driver (src/main.c:49-109); all numerics run in the
// HIP kernels of kernels.hip on the context's stream.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "mcx_internal.h"

namespace mcx {

static thread_local std::string g_err;
void set_error(const std::string& s) { g_err = s; }

int exc_return(const char* fn, const char* what) {
  try {
    g_err = std::string(fn) + ": internal exception: " + what;
  } catch (...) {
  }
  return MCX_EXC;
}

// MCX_TEST_THROW (a comma list of entry names) is read once, when the library is loaded: no
// getenv per call (not thread-safe against a concurrent setenv), nothing to do when it is unset
static const std::string g_test_throw = [] {
  const char* e = std::getenv("MCX_TEST_THROW");
  return e ? "," + std::string(e) + "," : std::string();
}();

void test_inject(const char* fn) {
  if (!g_test_throw.empty() && g_test_throw.find("," + std::string(fn) + ",") != std::string::npos)
    throw std::bad_alloc();
}

// padded node vectors (u, p and its buffers): the allocation is shifted by pad_off bytes so that
// with a 16-node row pitch (pad_align) every interior row's first owned node starts a 128-B line
// (DESIGN §3); the base pointers are kept for hipFree
static int dalloc_pad(Ctx& c, double** p, int64_t n) {
  char* base = nullptr;
  MCX_HIP(hipMalloc((void**)&base, sizeof(double) * n + 256));
  MCX_HIP(hipMemsetAsync(base, 0, sizeof(double) * n + 256, c.stream));
  c.pad_bases.push_back(base);
  c.device_bytes += (int64_t)sizeof(double) * n + 256;
  *p = reinterpret_cast<double*>(base + c.pad_off);
  return 0;
}

template <class T>
static int dalloc(Ctx& c, T** p, int64_t n) {
  if (n <= 0) n = 1;
  MCX_HIP(hipMalloc((void**)p, sizeof(T) * n));
  MCX_HIP(hipMemsetAsync(*p, 0, sizeof(T) * n, c.stream));
  c.device_bytes += (int64_t)sizeof(T) * n;
  return 0;
}

static void elastic_C(double E, double nu, double C[36]) {
  const double lam = E * nu / ((1. + nu) * (1. - 2. * nu));
  const double mu = E / (2. * (1. + nu));
  for (int q = 0; q < 36; q++) C[q] = 0.;
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) C[a * 6 + b] = lam + (a == b ? 2. * mu : 0.);
  for (int a = 3; a < 6; a++) C[a * 6 + a] = mu;
}

// phase timer: an event pair on the compute stream, recorded without any host wait (the
// timed steps are not serialised by the instrumentation); mcx_get_timing resolves the last pair
enum { PH_STRAINS, PH_HOMOG, PH_RES, PH_JAC, PH_SOLVE, PH_UPDATE };
struct PhaseTimer {
  Ctx& c;
  int k;
  PhaseTimer(Ctx& cc, int kk) : c(cc), k(kk) {
    if (c.timing && c.ev_phase[k][0]) (void)hipEventRecord(c.ev_phase[k][0], c.stream);
  }
  ~PhaseTimer() {
    if (!c.timing || !c.ev_phase[k][1]) return;
    (void)hipEventRecord(c.ev_phase[k][1], c.stream);
    c.phase_rec[k] = true;
  }
};

static int free_ctx(Ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
  if (c->x_stream) (void)hipStreamSynchronize(c->x_stream);
  if (c->f_stream) (void)hipStreamSynchronize(c->f_stream);
  void* ptrs[] = {c->hist_old, c->hist_new, c->ftrial, c->b, c->du, c->r, c->z, c->w, c->jix, c->jdd, c->V, c->U, c->D, c->d_mask, c->vi_idx, c->wd, c->vi_dict, c->vi_keys, c->vi_slot, c->vi_ctl, c->vi_bdict, c->eps, c->sig, c->ctan, c->Ke,
                  c->vib_keys, c->vib_ctl, c->vib_pos, c->ke_uni, c->xdone, c->esc_node, c->esc_res, c->esc_slot, c->elem_plain, c->cref, c->vi_xslot,
                  c->vi_xlist, c->vi_xcnt, c->vi_exc, c->st_coef, c->st_ids, c->st_slot, c->st_list, c->st_cnt, c->st_mask,
                  c->partials, c->red, c->red_loc, c->cg, c->hist, c->tmp, c->halo.d_send_idx,
                  c->halo.d_recv_idx, c->halo.d_sendbuf, c->halo.d_recvbuf, c->halo.d_bnd};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  for (void* p : c->pad_bases) (void)hipFree(p);  // u and the p buffers (dalloc_pad)
  if (c->h_cg) (void)hipHostFree(c->h_cg);
  for (void* h : {(void*)c->h_vib_keys, (void*)c->h_vib_map, (void*)c->h_vib_dict})
    if (h) (void)hipHostFree(h);
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  if (c->ev_a) (void)hipEventDestroy(c->ev_a);
  if (c->ev_b) (void)hipEventDestroy(c->ev_b);
  for (auto& pr : c->ev_phase)
    for (hipEvent_t e : pr)
      if (e) (void)hipEventDestroy(e);
  for (int q = 0; q < 2; q++)
    if (c->ev_chunk[q]) (void)hipEventDestroy(c->ev_chunk[q]);
  comm_destroy(*c);
  if (c->ev_pack) (void)hipEventDestroy(c->ev_pack);
  if (c->ev_comm) (void)hipEventDestroy(c->ev_comm);
  if (c->comm_stream) (void)hipStreamDestroy(c->comm_stream);
  if (c->x_stream) (void)hipStreamDestroy(c->x_stream);
  if (c->f_stream) (void)hipStreamDestroy(c->f_stream);
  for (hipEvent_t e : {c->ev_xp, c->ev_xd[0], c->ev_xd[1], c->ev_fx, c->ev_fd})
    if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

// largest SpMV grid over the selectable kernels (mcx_set_option may switch between them)
static int64_t max_spmv_blocks(Ctx& c) {
  const int keep = c.spmv_kernel, keep_fmt = c.fmt, keep_bits = c.vi_bits;
  int64_t m = 0;
  for (int f : {FMT_V, FMT_U, FMT_SPLIT, FMT_VI})
    for (int k = 0; k <= 11; k++)
      for (int bits : {4, 8}) {
        c.fmt = f;
        c.spmv_kernel = k;
        c.vi_bits = bits;
        m = std::max(m, spmv_grid_blocks(c));
      }
  c.spmv_kernel = keep;
  c.fmt = keep_fmt;
  c.vi_bits = keep_bits;
  return m;
}

static int init_ctx(Ctx& c, const mcx_opts* o, int rank, int nranks, const void* comm_id, LocalGroup* lg) {
  c.o = *o;
  c.lg = lg;
  c.rank = rank;
  c.nranks = nranks;
  c.comm_timeout = comm_timeout_default();
  if (const char* e = std::getenv("MCX_PAD_ALIGN")) c.pad_align = std::atoi(e);  // A/B of the padded layout
  int ndev = 0;
  MCX_HIP(hipGetDeviceCount(&ndev));
  if (ndev <= 0) {
    set_error("no HIP device visible");
    return 11;
  }
  c.device = lg ? lg->device : (o->device >= 0 ? o->device : rank % ndev);
  MCX_HIP(hipSetDevice(c.device));
  int rc = setup_decomposition(c);
  if (rc) return rc;
  if (lg && (rc = group_setup(c))) return rc;
  int ncu = 0;
  MCX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c.device));
  // z-marching tiles (sbaij and AIJ-split): one resident round of blocks, 256x4 phased tiles
  // where the subdomain is that wide — tools/spmv_ab.py sweeps, DESIGN.md §4
  c.ncu = std::max(ncu, 1);
  c.g.ncu = c.ncu;
  c.aij_split = o->mat_type == MCX_MAT_AIJ && o->mat_aij_split;
  c.aij_vi = o->mat_type == MCX_MAT_AIJ && o->mat_aij_vi;
  c.vi_fma = o->mat_vi_fma != 0;
  if (o->mat_type == MCX_MAT_SBAIJ) {
    // phased z-march 256x4 / 128x4 / 64x4 (128^3: 0.436 vs 0.502 ms for symz 128x2; 64^3:
    // 0.0555 vs 0.0625 ms for symz 64x4; profiles/old/r02_ab_sbaij{128,64}.log)
    c.spmv_kernel = c.g.nx >= 256 ? 11 : (c.g.nx >= 128 ? 7 : 8);
    c.fmt = FMT_U;
  }
  MCX_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
  MCX_HIP(hipStreamCreateWithFlags(&c.comm_stream, hipStreamNonBlocking));
  MCX_HIP(hipEventCreateWithFlags(&c.ev_pack, hipEventDisableTiming));
  MCX_HIP(hipEventCreateWithFlags(&c.ev_comm, hipEventDisableTiming));
  MCX_HIP(hipEventCreate(&c.ev_a));
  MCX_HIP(hipEventCreate(&c.ev_b));
  for (auto& pr : c.ev_phase)
    for (hipEvent_t& e : pr) MCX_HIP(hipEventCreate(&e));
  for (int q = 0; q < 2; q++) MCX_HIP(hipEventCreateWithFlags(&c.ev_chunk[q], hipEventDisableTiming));
  if ((rc = comm_init(c, comm_id))) return rc;
  if ((rc = build_halo_plan(c))) return rc;
  if ((rc = upload_constants(c))) return rc;
  const Geo& g = c.g;
  const int64_t npad = (int64_t)g.PX * g.PY * g.PZ * 3, nown3 = 3 * (int64_t)g.nown, E = g.nelem;
  // matrix storage: AIJ blocks V only for -mat_aij_split 0 (the AIJ-split path allocates it
  // lazily if a correction is not exact, mcx_assembly_jac); U for sbaij and AIJ-split; the
  // AIJ-split corrections D are sized by build_split to the active slots
  // jdd [VI_MAX][3] and the Jacobi vector dinv behind it in one buffer: the block-indexed CG
  // kernels read an exception node's (jix 255) inverse diagonal at jdd + 3 VI_MAX + 3n
  if ((rc = dalloc_pad(c, &c.u_pad, npad)) || (rc = dalloc_pad(c, &c.p_pad, npad)) || (rc = dalloc(c, &c.b, nown3)) ||
      (rc = dalloc(c, &c.du, nown3)) || (rc = dalloc(c, &c.r, nown3)) || (rc = dalloc(c, &c.z, nown3)) ||
      (rc = dalloc(c, &c.w, nown3)) || (rc = dalloc(c, &c.jdd, 3 * VI_MAX + nown3)) ||
      (rc = dalloc(c, &c.jix, (int64_t)g.nown)) || (rc = dalloc(c, &c.tmp, nown3)) ||
      (c.o.mat_type == MCX_MAT_SBAIJ && (rc = dalloc(c, &c.U, c.npgroups * UPAIR * 128))) ||
      (c.o.mat_type == MCX_MAT_AIJ && !c.aij_split && (rc = dalloc(c, &c.V, c.ngroups * NPAIR * 128))) ||
      (rc = dalloc(c, &c.eps, 6 * 8 * E)) || (rc = dalloc(c, &c.sig, 6 * 8 * E)) ||
      (rc = dalloc(c, &c.partials, c.partials_cap = 6 * std::max(max_spmv_blocks(c), node_blocks(c)) + 64)) ||
      (rc = dalloc(c, &c.red, 16)) || (rc = dalloc(c, &c.red_loc, 16)) || (rc = dalloc(c, &c.cg, 2)) ||
      (rc = dalloc(c, &c.hist, (int64_t)o->ksp_max_it + 2)) || (rc = dalloc(c, &c.ke_uni, 576)) ||
      (rc = dalloc_pad(c, &c.p_pad2, npad)) || (rc = dalloc(c, &c.xdone, 1)))  // p's second buffer (cg_pdb, cg_fusep)
    return rc;
  c.dinv = c.jdd + 3 * VI_MAX;
  // per-GP tangent: only laws that hand one over (the isotropic elastic C is a kernel argument)
  c.partials2 = c.partials + c.partials_cap / 2;
  if (o->mat_law != MCX_LAW_ELASTIC &&
      ((rc = dalloc(c, &c.ctan, 36 * 8 * E)) || (rc = dalloc(c, &c.Ke, (int64_t)576 * E))))
    return rc;
  if (o->mat_law == MCX_LAW_PLASTIC &&
      ((rc = dalloc(c, &c.hist_old, 7 * 8 * E)) || (rc = dalloc(c, &c.hist_new, 7 * 8 * E)) ||
       (rc = dalloc(c, &c.ftrial, 8 * E))))
    return rc;
  if (c.aij_split) MCX_HIP(hipMalloc(&c.d_mask, 16 * sizeof(unsigned)));
  MCX_HIP(hipHostMalloc((void**)&c.h_cg, sizeof(CgState) * 2, hipHostMallocDefault));
  std::memset(c.h_cg, 0, sizeof(CgState) * 2);
  if (o->micro_n != 2 && o->mat_law != MCX_LAW_EXTERNAL && rank == 0)
    std::fprintf(stderr,
                 "WARNING! -micro_n %d has no effect: the device Gauss-point laws have no micro-scale FE problem "
                 "(MicroPP's FE2 solver is out of scope); it sizes an external MicroPP (-mat_law external, "
                 "micropp_C_create3, src/init.c:210-213)\n",
                 o->micro_n);
  c.mat.law = o->mat_law;
  c.mat.E = o->micro_mat_1[0];
  c.mat.nu = o->micro_mat_1[1];
  c.mat.Sy = o->micro_mat_1[2];
  c.mat.Ka = o->micro_mat_1[3];
  elastic_C(c.mat.E, c.mat.nu, c.mat.C);
  c.nnz_local = count_nnz_rows(c, g.xs, g.ys, g.zs, g.nx, g.ny, g.nz);
  c.nnz_global = count_nnz_rows(c, 0, 0, 0, o->NX, o->NY, o->NZ);
  c.nupper_local = count_upper_values(c);
  MCX_HIP(hipStreamSynchronize(c.stream));
  if (lg) {
    lg->members[rank] = &c;
    MCX_HIP(hipMemcpy(lg->d_red_ptrs + rank, &c.red_loc, sizeof(double*), hipMemcpyHostToDevice));
    if ((rc = group_barrier(lg, rank, BAR_INIT, c.comm_timeout))) {
      lg->members[rank] = nullptr;
      return rc;
    }
  }
  return 0;
}

// ---------------------------------------------------------------- phases
static int cg_solve(Ctx& c, int* its, double* rnorm, int* reason) {
  launch_jacobi(c);  // PCSetUp_Jacobi happens inside KSPSolve in the reference
  c.fusep_used = false;  // set by cg_iteration when the p update runs inside the SpMV
  c.pdb_used = cg_pdb(c);
  c.pqb_used = c.pdb_used && c.cg_pdb == 4;
  c.xs_used = c.pqb_used && c.cg_xs;
  if (c.pqb_used && !c.p_pad3) {  // the quad-buffered p update's third and fourth buffers
    const int64_t npad = (int64_t)c.g.PX * c.g.PY * c.g.PZ * 3;
    int rc = 0;
    if ((rc = dalloc_pad(c, &c.p_pad3, npad)) || (rc = dalloc_pad(c, &c.p_pad4, npad))) return rc;
  }
  if (c.xs_used) {  // cg_xs: buffers 5-8, the side stream and its events (each made once; a setup
                    // that failed part-way completes at the next solve instead of running without them)
    const int64_t npad = (int64_t)c.g.PX * c.g.PY * c.g.PZ * 3;
    int rc = 0;
    for (int q = 0; q < 4; q++)
      if (!c.p_pad58[q] && (rc = dalloc_pad(c, &c.p_pad58[q], npad))) return rc;
    if (!c.x_stream) MCX_HIP(hipStreamCreateWithFlags(&c.x_stream, hipStreamNonBlocking));
    for (hipEvent_t* e : {&c.ev_xp, &c.ev_xd[0], &c.ev_xd[1]})
      if (!*e) MCX_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
  }
  if (c.pdb_used) MCX_HIP(hipMemsetAsync(c.xdone, 0, sizeof(int), c.stream));
  CgState s{};
  s.rtol = c.o.ksp_rtol;
  s.abstol = c.o.ksp_abstol;
  s.dtol = c.o.ksp_dtol;
  s.maxits = c.o.ksp_max_it;
  s.hist_on = c.o.ksp_monitor ? 1 : 0;
  s.xp = -1;
  c.h_cg[0] = s;
  MCX_HIP(hipMemcpyAsync(c.cg, &c.h_cg[0], sizeof(CgState), hipMemcpyHostToDevice, c.stream));
  launch_cg_init(c);
  int rc = cg_finish_init(c);
  if (rc) return rc;
  // spmv event pairs (timing mode): every 8th iteration (spread over the solve), at most kTimed
  const int kTimed = 512;
  if (c.timing && c.ev_pool.empty()) {
    c.ev_pool.resize(2 * kTimed);
    for (auto& e : c.ev_pool) MCX_HIP(hipEventCreate(&e));
  }
  // chunks of CH iterations; the host polls the previous chunk's CgState while the next chunk
  // runs (kernels of a converged solve return at once)
  const int CH = 8;
  int issued = 0, slot = 0, pending = -1, npairs = 0;
  std::vector<int> pair_it;
  const int cap = c.o.ksp_max_it + 4 * CH;
  while (true) {
    for (int q = 0; q < CH; q++, issued++) {
      hipEvent_t e0 = nullptr, e1 = nullptr;
      if (c.timing && (issued & 7) == 4 && npairs < kTimed) {
        e0 = c.ev_pool[2 * npairs];
        e1 = c.ev_pool[2 * npairs + 1];
        pair_it.push_back(issued);
        npairs++;
      }
      c.cg_it = issued;
      if ((rc = cg_iteration(c, e0, e1, q == 0, q == CH - 1))) return rc;
    }
    MCX_HIP(hipMemcpyAsync(&c.h_cg[slot], c.cg, sizeof(CgState), hipMemcpyDeviceToHost, c.stream));
    MCX_HIP(hipEventRecord(c.ev_chunk[slot], c.stream));
    if (pending >= 0) {
      if ((rc = comm_wait(c, c.ev_chunk[pending], "CG chunk poll (all-reduced CG scalars)"))) return rc;
      if (c.h_cg[pending].reason) break;
    }
    pending = slot;
    slot ^= 1;
    if (issued > cap) break;
  }
  if ((rc = launch_cg_xfinal(c))) return rc;  // the owed VecAXPY(x, alpha, p) terms, deferred by k_cg_pupdate
  MCX_HIP(hipEventRecord(c.ev_chunk[slot], c.stream));  // after the last chunk's (gated) all-reduces
  if ((rc = comm_wait(c, c.ev_chunk[slot], "CG solve end"))) return rc;
  CgState fin;
  MCX_HIP(hipMemcpy(&fin, c.cg, sizeof(CgState), hipMemcpyDeviceToHost));
  if (!fin.reason) {
    set_error("CG loop ended without a converged reason");
    return 30;
  }
  *its = fin.its;
  *rnorm = fin.dp;
  *reason = fin.reason;
  c.last_its = fin.its;
  if (c.o.ksp_monitor) {
    c.last_hist.resize(fin.its + 1);
    MCX_HIP(hipMemcpy(c.last_hist.data(), c.hist, sizeof(double) * (fin.its + 1), hipMemcpyDeviceToHost));
  }
  if (c.timing) {
    int n = 0;  // pairs around iterations that ran (later launches of the last chunk return at once)
    double tot = 0.;
    for (int q = 0; q < npairs; q++) {
      if (pair_it[q] >= fin.its) break;
      float ms = 0.f;
      MCX_HIP(hipEventElapsedTime(&ms, c.ev_pool[2 * q], c.ev_pool[2 * q + 1]));
      tot += ms;
      n++;
    }
    c.t.spmv_launches = n;
    c.t.spmv_ms_total = tot;
  }
  return 0;
}

}  // namespace mcx

using namespace mcx;

#define CTX(p) Ctx& c = *reinterpret_cast<Ctx*>(p)
#define GUARD(p)                      \
  if (!(p)) {                         \
    set_error("null context");        \
    return 1;                         \
  }                                   \
  MCX_HIP(hipSetDevice(reinterpret_cast<Ctx*>(p)->device))

extern "C" {

const char* mcx_last_error(void) { return g_err.c_str(); }
const char* mcx_version(void) { return "macroc_amd 0.3 (gfx950, abi 3)"; }
int mcx_abi_version(void) { return MCX_ABI_VERSION; }

void mcx_default_opts(mcx_opts* o) {
  std::memset(o, 0, sizeof(*o));
  o->NX = 40;  // include/macroc.h:44-46
  o->NY = 3;
  o->NZ = 40;
  o->lx = 50.0;  // include/macroc.h:47-49
  o->ly = 1.0;
  o->lz = 50.0;
  o->dt = 0.001;
  o->final_time = 1.0;
  o->ts = 1;
  o->vtu_freq = -1;
  o->bc_type = MCX_BC_CIRCLE;  // src/init.c:64
  o->rad = 1.0;
  o->newton_max_its = 5;
  o->newton_min_tol = 1.0e-1;
  o->newton_rel_tol = 1.0e-4;
  o->ksp_rtol = 1.0e-5;  // src/init.c:147-148
  o->ksp_abstol = 1.0e-50;
  o->ksp_dtol = 1.0e4;
  o->ksp_max_it = 10000;
  o->micro_n = 2;
  o->micro_type = 1;
  const double mat[4] = {1.0e7, 0.25, 1.0e4, 1.0e7};  // src/init.c:31-32
  std::memcpy(o->micro_mat_1, mat, sizeof(mat));
  std::memcpy(o->micro_mat_2, mat, sizeof(mat));
  o->device = -1;
  o->mat_aij_split = 1;
  o->mat_aij_vi = 1;
  o->mat_vi_fma = 1;
}

int mcx_parse_args(mcx_opts* o, int argc, const char* const* argv) try {
  MCX_ENTRY();
  for (int a = 0; a < argc; a++) {
    const char* k = argv[a];
    const char* v = (a + 1 < argc) ? argv[a + 1] : nullptr;
    auto I = [&](const char* name, auto* f) {
      if (std::strcmp(k, name)) return false;
      if (!v) return false;
      *f = (std::remove_reference_t<decltype(*f)>)std::atoll(v);
      a++;
      return true;
    };
    auto D = [&](const char* name, double* f) {
      if (std::strcmp(k, name)) return false;
      if (!v) return false;
      *f = std::atof(v);
      a++;
      return true;
    };
    auto A4 = [&](const char* name, double* f) {
      if (std::strcmp(k, name)) return false;
      if (!v) return false;
      std::string s(v);
      size_t pos = 0;
      for (int q = 0; q < 4 && pos <= s.size(); q++) {
        size_t e = s.find(',', pos);
        f[q] = std::atof(s.substr(pos, e == std::string::npos ? std::string::npos : e - pos).c_str());
        if (e == std::string::npos) break;
        pos = e + 1;
      }
      a++;
      return true;
    };
    if (I("-da_grid_x", &o->NX) || I("-da_grid_y", &o->NY) || I("-da_grid_z", &o->NZ) ||
        I("-da_processors_x", &o->px) || I("-da_processors_y", &o->py) || I("-da_processors_z", &o->pz) ||
        D("-lx", &o->lx) || D("-ly", &o->ly) || D("-lz", &o->lz) || D("-dt", &o->dt) || I("-ts", &o->ts) ||
        I("-vtu_freq", &o->vtu_freq) || I("-bc_type", &o->bc_type) || I("-newton_max_its", &o->newton_max_its) ||
        D("-newton_min_tol", &o->newton_min_tol) || D("-newton_rel_tol", &o->newton_rel_tol) ||
        D("-ksp_rtol", &o->ksp_rtol) || D("-ksp_atol", &o->ksp_abstol) || D("-ksp_divtol", &o->ksp_dtol) ||
        I("-ksp_max_it", &o->ksp_max_it) || I("-micro_n", &o->micro_n) || I("-micro_type", &o->micro_type) ||
        A4("-micro_mat_1", o->micro_mat_1) || A4("-micro_mat_2", o->micro_mat_2) || I("-device", &o->device) ||
        I("-mat_aij_split", &o->mat_aij_split) || I("-mat_aij_vi", &o->mat_aij_vi) ||
        I("-mat_vi_fma", &o->mat_vi_fma))
      continue;
    if (!std::strcmp(k, "-dm_mat_type")) {
      if (!v || (std::strcmp(v, "aij") && std::strcmp(v, "sbaij"))) {
        set_error(std::string("-dm_mat_type: aij or sbaij, got ") + (v ? v : "(none)"));
        return 2;
      }
      o->mat_type = std::strcmp(v, "sbaij") ? MCX_MAT_AIJ : MCX_MAT_SBAIJ;
      a++;
      continue;
    }
    if (!std::strcmp(k, "-mat_ignore_lower_triangular")) continue;
    if (!std::strcmp(k, "-mat_law")) {
      if (!v || (std::strcmp(v, "elastic") && std::strcmp(v, "plastic") && std::strcmp(v, "external"))) {
        set_error(std::string("-mat_law: elastic, plastic or external, got ") + (v ? v : "(none)"));
        return 2;
      }
      o->mat_law = !std::strcmp(v, "plastic") ? MCX_LAW_PLASTIC
                   : !std::strcmp(v, "external") ? MCX_LAW_EXTERNAL : MCX_LAW_ELASTIC;
      a++;
      continue;
    }
    if (!std::strcmp(k, "-ksp_monitor")) {
      o->ksp_monitor = 1;
      continue;
    }
    if (!std::strcmp(k, "-ksp_type") || !std::strcmp(k, "-pc_type")) {
      if (v && std::strcmp(v, !std::strcmp(k, "-ksp_type") ? "cg" : "jacobi")) {
        set_error(std::string("only -ksp_type cg / -pc_type jacobi are implemented, got ") + v);
        return 2;
      }
      a++;
      continue;
    }
    std::fprintf(stderr, "WARNING! There are options you set that were not used: %s\n", k);
  }
  return 0;
} MCX_CATCH

int mcx_init(const mcx_opts* o, int rank, int nranks, const void* comm_id, void** ctx) try {
  MCX_ENTRY();
  if (!o || !ctx || nranks < 1 || rank < 0 || rank >= nranks) {
    set_error("mcx_init: bad arguments");
    return 1;
  }
  Ctx* c = new Ctx();
  int rc = init_ctx(*c, o, rank, nranks, comm_id, nullptr);
  if (rc) {
    std::string e = g_err;
    free_ctx(c);
    g_err = e;
    *ctx = nullptr;
    return rc;
  }
  *ctx = c;
  return 0;
} MCX_CATCH

int mcx_init_local(const mcx_opts* o, int rank, void* group, void** ctx) try {
  MCX_ENTRY();
  auto* lg = static_cast<LocalGroup*>(group);
  if (!o || !ctx || !lg || rank < 0 || rank >= lg->nranks) {
    set_error("mcx_init_local: bad arguments");
    return 1;
  }
  Ctx* c = new Ctx();
  int rc = init_ctx(*c, o, rank, lg->nranks, nullptr, lg);
  if (rc) {
    std::string e = g_err;
    free_ctx(c);
    g_err = e;
    *ctx = nullptr;
    return rc;
  }
  *ctx = c;
  return 0;
} MCX_CATCH

int mcx_finalize(void* ctx) try {
  MCX_ENTRY();
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  int rc = 0;
  if (c && c->lg) {
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    // no member still copies from this context's buffers: every member drained its streams
    // before crossing.  If the group broke (a member stopped, or reached another collective),
    // the members' enqueued copies may still read these buffers: wait for the whole device.
    if ((rc = group_barrier(c->lg, c->rank, BAR_FINALIZE, c->comm_timeout))) (void)hipDeviceSynchronize();
    c->lg->members[c->rank] = nullptr;
  }
  const std::string e = g_err;
  free_ctx(c);
  if (rc) g_err = e;
  return rc;
} MCX_CATCH

static void fill_info(const Ctx& c, mcx_info* in) {
  const Geo& g = c.g;
  std::memset(in, 0, sizeof(*in));
  in->NX = g.NX;
  in->NY = g.NY;
  in->NZ = g.NZ;
  in->px = c.m;
  in->py = c.n;
  in->pz = c.p;
  in->rank = c.rank;
  in->nranks = c.nranks;
  in->xs = g.xs;
  in->ys = g.ys;
  in->zs = g.zs;
  in->nx = g.nx;
  in->ny = g.ny;
  in->nz = g.nz;
  in->Xs = std::max(g.xs - 1, 0);
  in->Ys = std::max(g.ys - 1, 0);
  in->Zs = std::max(g.zs - 1, 0);
  in->Nx = std::min(g.xs + g.nx + 1, g.NX) - in->Xs;
  in->Ny = std::min(g.ys + g.ny + 1, g.NY) - in->Ys;
  in->Nz = std::min(g.zs + g.nz + 1, g.NZ) - in->Zs;
  in->ndofs_global = 3 * c.rank_node_off[c.nranks];
  in->ndofs_local = 3 * (int64_t)g.nown;
  in->dof_offset = 3 * c.rank_node_off[c.rank];
  in->nnz_local = c.nnz_local;
  in->nnz_global = c.nnz_global;
  int64_t cnt[3];
  int s[3] = {g.xs, g.ys, g.zs}, w[3] = {g.nx, g.ny, g.nz};
  for (int d = 0; d < 3; d++) {
    int lo = s[d] > 0 ? s[d] - 1 : s[d];
    cnt[d] = std::max(0, s[d] + w[d] - 1 - lo);
  }
  in->nelem_local = cnt[0] * cnt[1] * cnt[2];
  in->nelem_ext = g.nelem;
  in->dx = g.dx;
  in->dy = c.dy;
  in->dz = g.dz;
  in->wg = g.wg;
  in->device_bytes = c.device_bytes;
  in->device = c.device;
  in->storage = c.fmt;
  in->split_slots = c.fmt == FMT_SPLIT ? c.dsl.L : 0;
  in->split_bits = c.fmt == FMT_SPLIT ? (c.dsl.wide ? 32 : 16) : 0;
  in->vi_values = c.fmt == FMT_VI ? c.vi_n : 0;
  in->vi_bits = c.fmt == FMT_VI ? c.vi_bits : 0;
  in->vi_blocks = c.fmt == FMT_VI && c.vi_block ? c.vi_nblocks : 0;
  in->vi_exc_nodes = c.fmt == FMT_VI && c.vi_block ? c.vi_nexc : 0;
  in->split_escapes = c.fmt == FMT_SPLIT && c.dsl.esc ? c.dsl.nesc : 0;
  in->st_listed = c.device >= 0 && st_used(c) ? c.st_n : -1;
  if (c.device >= 0) spmv_tile(c, &in->spmv_tx, &in->spmv_ty, &in->spmv_kc);
  in->ex0 = g.ex0;
  in->ey0 = g.ey0;
  in->ez0 = g.ez0;
  in->nex = g.nex;
  in->ney = g.ney;
  in->nez = g.nez;
}


int mcx_get_info(void* ctx, mcx_info* in) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  fill_info(c, in);
  return 0;
} MCX_CATCH

int mcx_comm_info(void* ctx, int* comm_ranks, int* comm_rank, int* device) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  int n = 1, r = 0, d = c.device;
  if (c.lg) {
    n = c.lg->nranks;
    r = c.rank;
  } else if (int rc = comm_query(c, &n, &r, &d)) {
    return rc;
  }
  if (comm_ranks) *comm_ranks = n;
  if (comm_rank) *comm_rank = r;
  if (device) *device = d;
  return 0;
} MCX_CATCH

int mcx_plan(const mcx_opts* o, int rank, int nranks, mcx_info* in) try {
  MCX_ENTRY();
  if (!o || !in || nranks < 1 || rank < 0 || rank >= nranks) {
    set_error("mcx_plan: bad arguments");
    return 1;
  }
  Ctx c;
  c.o = *o;
  c.rank = rank;
  c.nranks = nranks;
  c.device = -1;
  int rc = setup_decomposition(c);
  if (rc) return rc;
  c.nnz_local = count_nnz_rows(c, c.g.xs, c.g.ys, c.g.zs, c.g.nx, c.g.ny, c.g.nz);
  c.nnz_global = count_nnz_rows(c, 0, 0, 0, o->NX, o->NY, o->NZ);
  fill_info(c, in);
  return 0;
} MCX_CATCH

int mcx_plan_halo(const mcx_opts* o, int rank, int nranks, int* nnbr, int* nbr_rank, int64_t* send_cnt,
                  int64_t* recv_cnt, int64_t* send_nat, int64_t* recv_nat, int64_t* nsend, int64_t* nrecv) try {
  MCX_ENTRY();
  if (!o || nranks < 1 || rank < 0 || rank >= nranks) {
    set_error("mcx_plan_halo: bad arguments");
    return 1;
  }
  Ctx c;
  c.o = *o;
  c.rank = rank;
  c.nranks = nranks;
  int rc = setup_decomposition(c);
  if (rc) return rc;
  std::vector<int> sidx, ridx;
  plan_halo(c, sidx, ridx);
  const HaloPlan& h = c.halo;
  if (nnbr) *nnbr = (int)h.nbr_rank.size();
  if (nsend) *nsend = h.nsend;
  if (nrecv) *nrecv = h.nrecv;
  for (size_t q = 0; q < h.nbr_rank.size(); q++) {
    if (nbr_rank) nbr_rank[q] = h.nbr_rank[q];
    if (send_cnt) send_cnt[q] = h.send_cnt[q];
    if (recv_cnt) recv_cnt[q] = h.recv_cnt[q];
  }
  if (send_nat)
    for (int64_t t = 0; t < h.nsend; t++) send_nat[t] = pad_to_natural(c, sidx[t]);
  if (recv_nat)
    for (int64_t t = 0; t < h.nrecv; t++) recv_nat[t] = pad_to_natural(c, ridx[t]);
  return 0;
} MCX_CATCH

int mcx_material_set(void* ctx, int id, double E, double nu, double Sy, double Ka, int type) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  (void)Sy;
  (void)Ka;
  (void)type;
  if (id == 0) {
    c.mat.E = E;
    c.mat.nu = nu;
    c.mat.Sy = Sy;
    c.mat.Ka = Ka;
    elastic_C(E, nu, c.mat.C);
  } else if (id == 1 && (E != c.mat.E || nu != c.mat.nu || Sy != c.mat.Sy || Ka != c.mat.Ka)) {
    set_error("two distinct materials need the MicroPP micro-structure (out of scope); use equal materials");
    return 3;
  }
  return 0;
} MCX_CATCH

double mcx_get_displacement(void* ctx, int time_s) {
  Ctx& c = *reinterpret_cast<Ctx*>(ctx);
  // src/bcs.c:52-58 with the missing `return` restored
  double time = time_s * c.o.dt;
  return -1.0 * (time / c.o.final_time);
}

int mcx_zero_u(void* ctx) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  MCX_HIP(hipMemsetAsync(c.u_pad, 0, sizeof(double) * 3 * (size_t)c.g.PX * c.g.PY * c.g.PZ, c.stream));
  return 0;
} MCX_CATCH

int mcx_apply_bc_u(void* ctx, double U) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  launch_apply_bc_u(c, U);
  MCX_HIP(hipGetLastError());
  return 0;
} MCX_CATCH

int mcx_set_strains(void* ctx) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  PhaseTimer t(c, PH_STRAINS);
  int rc = halo_exchange(c, c.u_pad);  // DMGlobalToLocal (src/assembly.c:40-41)
  if (rc) return rc;
  launch_strains(c);
  MCX_HIP(hipGetLastError());
  return 0;
} MCX_CATCH

// -mat_law external: the registered law fills sig and ctan from eps (see macroc_amd.h)
static int external_homogenize(Ctx& c) {
  const int64_t E = c.g.nelem, ngp = 8 * E;
  if (c.has_dlaw) {
    mcx_gp_batch b{E, ngp, c.eps, c.sig, c.ctan, (void*)c.stream};
    const int rc = c.dlaw.homogenize(c.dlaw.user, &b);
    if (rc) {
      set_error("external device law: homogenize returned " + std::to_string(rc));
      return 6;
    }
    MCX_HIP(hipGetLastError());
    return 0;
  }
  if (!c.has_mpp) return 0;  // values injected with mcx_set_gp_stress / mcx_set_gp_ctan
  // host MicroPP: strains out, per-GP calls in gpi = ie*8 + gp order, stress + tangent back
  c.h_gp.resize((size_t)ngp * 36);
  double* h = c.h_gp.data();
  MCX_HIP(hipMemcpyAsync(h, c.eps, sizeof(double) * 6 * ngp, hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  std::vector<double> soa((size_t)ngp * 6);
  for (int64_t e = 0; e < E; e++)
    for (int gp = 0; gp < 8; gp++) {
      double eps6[6];
      for (int k = 0; k < 6; k++) eps6[k] = h[(int64_t)k * ngp + gp * E + e];
      c.mpp.set_strain3((int)(e * 8 + gp), eps6);
    }
  c.mpp.homogenize();
  for (int64_t e = 0; e < E; e++)
    for (int gp = 0; gp < 8; gp++) {
      double s6[6];
      c.mpp.get_stress3((int)(e * 8 + gp), s6);
      for (int k = 0; k < 6; k++) soa[(size_t)k * ngp + gp * E + e] = s6[k];
    }
  MCX_HIP(hipMemcpyAsync(c.sig, soa.data(), sizeof(double) * 6 * ngp, hipMemcpyHostToDevice, c.stream));
  for (int64_t e = 0; e < E; e++)
    for (int gp = 0; gp < 8; gp++) {
      double c36[36];
      c.mpp.get_ctan3((int)(e * 8 + gp), c36);
      for (int kl = 0; kl < 36; kl++) h[(size_t)kl * ngp + gp * E + e] = c36[kl];
    }
  MCX_HIP(hipMemcpyAsync(c.ctan, h, sizeof(double) * 36 * ngp, hipMemcpyHostToDevice, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));  // the staging buffers are reused
  return 0;
}

int mcx_homogenize(void* ctx) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  PhaseTimer t(c, PH_HOMOG);
  if (c.mat.law == MCX_LAW_EXTERNAL) return external_homogenize(c);
  launch_homogenize(c);
  MCX_HIP(hipGetLastError());
  return 0;
} MCX_CATCH

static int need_external(Ctx& c, const char* fn) {
  if (c.mat.law == MCX_LAW_EXTERNAL) return 0;
  set_error(std::string(fn) + ": the context was created without -mat_law external");
  return 7;
}

int mcx_set_micropp(void* ctx, const mcx_micropp_api* api) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  if (int rc = need_external(c, "mcx_set_micropp")) return rc;
  if (api && (!api->set_strain3 || !api->homogenize || !api->get_stress3 || !api->get_ctan3)) {
    set_error("mcx_set_micropp: set_strain3, homogenize, get_stress3 and get_ctan3 are required");
    return 2;
  }
  c.has_mpp = api != nullptr;
  if (api) c.mpp = *api;
  if (api) c.has_dlaw = false;
  return 0;
} MCX_CATCH

int mcx_set_device_law(void* ctx, const mcx_device_law* law) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  if (int rc = need_external(c, "mcx_set_device_law")) return rc;
  if (law && !law->homogenize) {
    set_error("mcx_set_device_law: homogenize is required");
    return 2;
  }
  c.has_dlaw = law != nullptr;
  if (law) c.dlaw = *law;
  if (law) c.has_mpp = false;
  return 0;
} MCX_CATCH

// host [ngp][ncomp] (gpi order) <-> device [ncomp][8][nelem]
static int gp_upload(Ctx& c, const double* host, double* dev, int ncomp) {
  const int64_t E = c.g.nelem, ngp = 8 * E;
  std::vector<double> soa((size_t)ngp * ncomp);
  for (int64_t e = 0; e < E; e++)
    for (int gp = 0; gp < 8; gp++)
      for (int k = 0; k < ncomp; k++) soa[(size_t)k * ngp + gp * E + e] = host[(e * 8 + gp) * ncomp + k];
  MCX_HIP(hipMemcpyAsync(dev, soa.data(), sizeof(double) * soa.size(), hipMemcpyHostToDevice, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  return 0;
}

int mcx_set_gp_stress(void* ctx, const double* host) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  if (int rc = need_external(c, "mcx_set_gp_stress")) return rc;
  return gp_upload(c, host, c.sig, 6);
} MCX_CATCH

int mcx_set_gp_ctan(void* ctx, const double* host) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  if (int rc = need_external(c, "mcx_set_gp_ctan")) return rc;
  return gp_upload(c, host, c.ctan, 36);
} MCX_CATCH

int mcx_get_gp_strain(void* ctx, double* host) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  const int64_t E = c.g.nelem, ngp = 8 * E;
  std::vector<double> soa((size_t)ngp * 6);
  MCX_HIP(hipMemcpyAsync(soa.data(), c.eps, sizeof(double) * soa.size(), hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  for (int64_t e = 0; e < E; e++)
    for (int gp = 0; gp < 8; gp++)
      for (int k = 0; k < 6; k++) host[(e * 8 + gp) * 6 + k] = soa[(size_t)k * ngp + gp * E + e];
  return 0;
} MCX_CATCH

int mcx_assembly_res(void* ctx, double* norm2) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  {
    PhaseTimer t(c, PH_RES);
    launch_residual(c);
    launch_reduce(c, 1, (int)node_blocks(c), c.red);
    MCX_HIP(hipGetLastError());
  }
  double nrm = 0.;
  MCX_HIP(hipMemcpyAsync(&c.h_cg[0].dp, c.red, sizeof(double), hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipEventRecord(c.ev_chunk[0], c.stream));
  if (int rc = comm_wait(c, c.ev_chunk[0], "assembly_res (all-reduced |RES|)")) return rc;
  nrm = c.h_cg[0].dp;
  if (norm2) *norm2 = nrm;
  return 0;
} MCX_CATCH

// the AIJ stencil-block storage, allocated on first use when the context started with AIJ-split
static int ensure_V(Ctx& c) {
  if (c.V) return 0;
  return dalloc(c, &c.V, c.ngroups * NPAIR * 128);
}

// the value-indexed storage, allocated on first use
static int ensure_VI(Ctx& c) {
  if (c.vi_dict) return 0;
  const int64_t idx_bytes = 0;  // the index array is sized by build_vi to the mode it picks
  const int64_t nd = std::max(VI_MAX, NSLOT * 16), nk = 2 * VI_HASH + NSLOT * 32;
  MCX_HIP(hipMalloc(&c.vi_dict, nd * sizeof(double)));
  MCX_HIP(hipMalloc(&c.vi_bdict, VI_MAX * VIB_STRIDE * sizeof(double)));
  MCX_HIP(hipMalloc(&c.vi_keys, nk * sizeof(unsigned long long)));
  MCX_HIP(hipMalloc(&c.vi_slot, nk));
  MCX_HIP(hipMalloc(&c.vi_ctl, (5 + NSLOT) * sizeof(unsigned)));
  MCX_HIP(hipMalloc(&c.vib_keys, (NSLOT * VB_GSV + VI_HASH) * sizeof(unsigned long long)));
  MCX_HIP(hipMalloc(&c.vib_ctl, 4 * sizeof(unsigned)));
  MCX_HIP(hipHostMalloc((void**)&c.h_vib_keys, (NSLOT * VB_GSV + VI_HASH + 2) * sizeof(unsigned long long),
                        hipHostMallocDefault));
  MCX_HIP(hipHostMalloc((void**)&c.h_vib_map, VI_HASH, hipHostMallocDefault));
  MCX_HIP(hipHostMalloc((void**)&c.h_vib_dict, VI_MAX * VIB_STRIDE * sizeof(double), hipHostMallocDefault));
  c.device_bytes += idx_bytes + nd * 8 + VI_MAX * VIB_STRIDE * 8 + nk * 9 + (5 + NSLOT) * 4 +
                    (NSLOT * VB_GSV + VI_HASH) * 8 + 16;
  return 0;
}

int mcx_assembly_jac(void* ctx) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  PhaseTimer t(c, PH_JAC);
  int rc;
  const bool table = c.mat.law != MCX_LAW_ELASTIC;
  const bool try_vi = c.o.mat_type == MCX_MAT_AIJ && c.aij_vi && !c.vi_declined;
  // a per-GP-tangent law headed for the value-indexed storage with exception nodes: kref and the
  // non-plain elements' matrices only (the value-indexed build needs no other element matrix)
  c.plain_ke = false;
  if (table && try_vi && c.vi_exc_max > 0 && c.vi_block_on && c.vi_bits_max == 4 && c.vib_onepass) {
    if ((rc = launch_plain_ke(c))) return rc;
  } else if (table) {
    launch_element_ke(c);  // per-GP tangent: element matrices first
  } else {
    launch_elastic_ke(c);  // one material, one element shape: one element matrix
  }
  if (try_vi) {
    // value-indexed AIJ when the matrix has at most VI_MAX distinct values (the elastic law's
    // matrices; per-GP-tangent laws with few exception nodes); otherwise the next storage below
    bool ok = false;
    if ((rc = ensure_VI(c)) || (rc = build_vi(c, &ok))) return rc;
    if (ok) {
      c.fmt = FMT_VI;
      if ((rc = build_wdesc(c)) || (rc = build_st(c))) return rc;
      c.assembled = true;
      MCX_HIP(hipGetLastError());
      return 0;
    }
    c.vi_declined = table;  // a per-GP tangent stays varied: skip the attempt
    if (c.plain_ke) {       // the storages below sum every element's matrix
      launch_element_ke(c);
      c.plain_ke = false;
    }
  }
  if (c.o.mat_type == MCX_MAT_SBAIJ) {
    launch_gather_matrix_sym(c);
    c.fmt = FMT_U;
  } else if (c.aij_split && !c.split_declined) {
    if (!c.U && (rc = dalloc(c, &c.U, c.npgroups * UPAIR * 128))) return rc;  // first AIJ-split assembly
    launch_gather_matrix_sym(c);
    bool exact = false;
    if ((rc = build_split(c, &exact))) return rc;
    c.fmt = exact ? FMT_SPLIT : FMT_V;
    if (!exact) {  // a correction is not exact, or they are too many: plain AIJ blocks
      if ((rc = ensure_V(c))) return rc;
      launch_gather_matrix(c);
      // a per-GP-tangent law keeps its inexact (or refused dense) corrections: later assemblies
      // go straight to blocks
      c.split_declined = c.mat.law != MCX_LAW_ELASTIC;
    }
  } else {
    if ((rc = ensure_V(c))) return rc;
    launch_gather_matrix(c);
    c.fmt = FMT_V;
  }
  c.assembled = true;
  MCX_HIP(hipGetLastError());
  return 0;
} MCX_CATCH

int mcx_solve(void* ctx, int* its, double* rnorm, int* reason) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  if (!c.assembled) {
    set_error("mcx_solve: no matrix assembled (call mcx_assembly_jac first)");
    return 5;
  }
  int i0 = 0, r0 = 0;
  double n0 = 0.;
  int rc;
  {
    PhaseTimer t(c, PH_SOLVE);
    rc = cg_solve(c, &i0, &n0, &r0);
  }
  if (rc) return rc;
  MCX_HIP(hipGetLastError());
  if (its) *its = i0;
  if (rnorm) *rnorm = n0;
  if (reason) *reason = r0;
  return 0;
} MCX_CATCH

int mcx_update_u(void* ctx) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  PhaseTimer t(c, PH_UPDATE);
  launch_update_u(c);
  MCX_HIP(hipGetLastError());
  return 0;
} MCX_CATCH

int mcx_update_vars(void* ctx) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  if (c.hist_old) std::swap(c.hist_old, c.hist_new);
  if (c.has_mpp && c.mpp.update_vars) c.mpp.update_vars();
  if (c.has_dlaw && c.dlaw.update_vars) {
    MCX_HIP(hipStreamSynchronize(c.stream));
    if (int rc = c.dlaw.update_vars(c.dlaw.user)) {
      set_error("external device law: update_vars returned " + std::to_string(rc));
      return 6;
    }
  }
  return 0;
} MCX_CATCH

int mcx_get_nonlinear_stats(void* ctx, int64_t* n_nonlinear, double* f_trial_max) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  int64_t n = 0;
  double fm = 0.;
  if (c.has_mpp) {  // the external MicroPP's own counts (over its Gauss points)
    if (c.mpp.get_non_linear_gps) n = c.mpp.get_non_linear_gps();
    if (c.mpp.get_f_trial_max) fm = c.mpp.get_f_trial_max();
  } else if (c.has_dlaw) {
    if (c.dlaw.nonlinear_stats) {
      MCX_HIP(hipStreamSynchronize(c.stream));
      if (int rc = c.dlaw.nonlinear_stats(c.dlaw.user, &n, &fm)) {
        set_error("external device law: nonlinear_stats returned " + std::to_string(rc));
        return 6;
      }
    }
  } else if (c.ftrial) {
    const Geo& g = c.g;
    std::vector<double> ft(8 * g.nelem);
    MCX_HIP(hipMemcpyAsync(ft.data(), c.ftrial, sizeof(double) * ft.size(), hipMemcpyDeviceToHost, c.stream));
    MCX_HIP(hipStreamSynchronize(c.stream));
    int lo[3], hi[3], s[3] = {g.xs, g.ys, g.zs}, w[3] = {g.nx, g.ny, g.nz};
    for (int d = 0; d < 3; d++) {
      lo[d] = s[d] > 0 ? s[d] - 1 : s[d];
      hi[d] = s[d] + w[d] - 2;
    }
    fm = -1e300;
    for (int ez = lo[2]; ez <= hi[2]; ez++)
      for (int ey = lo[1]; ey <= hi[1]; ey++)
        for (int ex = lo[0]; ex <= hi[0]; ex++) {
          int64_t le = (ex - g.ex0) + (int64_t)(ey - g.ey0) * g.nex + (int64_t)(ez - g.ez0) * g.nex * g.ney;
          for (int gp = 0; gp < 8; gp++) {
            double f = ft[gp * g.nelem + le];
            if (f > 0.) n++;
            if (f > fm) fm = f;
          }
        }
  }
  if (n_nonlinear) *n_nonlinear = n;
  if (f_trial_max) *f_trial_max = fm;
  return 0;
} MCX_CATCH

}  // extern "C"

// all-reduce of a few host doubles through red_loc / red (collective; op 0 sum, 1 max)
static int host_allreduce(Ctx& c, double* v, int n, int op) {
  if (c.nranks <= 1 && !c.comm) return 0;
  int rc;
  if ((rc = allreduce_prepare(c))) return rc;
  MCX_HIP(hipMemcpyAsync(c.red_loc, v, sizeof(double) * n, hipMemcpyHostToDevice, c.stream));
  rc = op ? allreduce_max(c, c.red_loc, c.red, n) : allreduce_sum(c, c.red_loc, c.red, n);
  if (rc) return rc;
  MCX_HIP(hipMemcpyAsync(v, c.red, sizeof(double) * n, hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipEventRecord(c.ev_chunk[0], c.stream));
  return comm_wait(c, c.ev_chunk[0], op ? "host all-reduce (max)" : "host all-reduce (sum)");
}

extern "C" {

int mcx_reduce_nonlinear(void* ctx, int64_t* n_local, int64_t* n_total, double* f_trial_max) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  int64_t n = 0;
  double fm = 0.;
  int rc = mcx_get_nonlinear_stats(ctx, &n, &fm);
  if (rc) return rc;
  double s = (double)n;  // exact: at most 8 x elements GPs
  if ((rc = host_allreduce(c, &s, 1, 0)) || (rc = host_allreduce(c, &fm, 1, 1))) return rc;
  if (n_local) *n_local = n;
  if (n_total) *n_total = (int64_t)s;
  if (f_trial_max) *f_trial_max = fm;
  return 0;
} MCX_CATCH

int mcx_calc_force(void* ctx, double* force) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  const Geo& g = c.g;
  // the rank's own elements as PETSc lists them (DMDAGetElements): [s - (s > 0), s + w - 1)
  int lo[3], cnt[3];
  const int s[3] = {g.xs, g.ys, g.zs}, w[3] = {g.nx, g.ny, g.nz};
  for (int d = 0; d < 3; d++) {
    lo[d] = s[d] > 0 ? s[d] - 1 : s[d];
    cnt[d] = std::max(0, s[d] + w[d] - 1 - lo[d]);
  }
  double mpi_force = 0.0;
  std::vector<double> ave;
  auto layer = [&](int comp, int fa, int fixed, int a0, int na, int b0, int nb) -> int {
    ave.assign((size_t)na * nb, 0.);
    if (ave.empty()) return 0;
    launch_force_layer(c, comp, fa, fixed, a0, na, b0, nb, c.tmp);
    MCX_HIP(hipMemcpyAsync(ave.data(), c.tmp, sizeof(double) * ave.size(), hipMemcpyDeviceToHost, c.stream));
    MCX_HIP(hipStreamSynchronize(c.stream));
    return 0;
  };
  int rc;
  if (g.bc_type == MCX_BC_BENDING) {
    // calc_force_bending src/forces.c:58-106: ranks owning x = NX-1 (owned corner, :75),
    // their last x layer of elements, ey outer / ez inner, stress_ave[3] * dy * dz
    if (g.xs + g.nx == g.NX && cnt[0] > 0) {
      if ((rc = layer(3, 0, lo[0] + cnt[0] - 1, lo[1], cnt[1], lo[2], cnt[2]))) return rc;
      for (int ey = 0; ey < cnt[1]; ++ey)
        for (int ez = 0; ez < cnt[2]; ++ez) mpi_force += ave[(size_t)ey * cnt[2] + ez] * c.dy * g.dz;
    }
  } else {
    // calc_force_circle src/forces.c:115-166: ghost corners si, sj, sk with the owned ny
    // (:130-133), top element layer, ex outer / ez inner, elements whose centre is inside
    // the radius, stress_ave[1] * dx * dz
    const int si = lo[0], sj = lo[1], sk = lo[2];
    if (sj + g.ny == g.NY && cnt[1] > 0) {
      if ((rc = layer(1, 1, lo[1] + cnt[1] - 1, lo[0], cnt[0], lo[2], cnt[2]))) return rc;
      for (int ex = 0; ex < cnt[0]; ++ex)
        for (int ez = 0; ez < cnt[2]; ++ez) {
          const double x = g.lx / 2. - ((si + ex) * g.dx + g.dx / 2.);
          const double z = g.lz / 2. - ((sk + ez) * g.dz + g.dz / 2.);
          if ((x * x + z * z) < 1 * (g.rad * g.rad)) mpi_force += ave[(size_t)ex * cnt[2] + ez] * g.dx * g.dz;
        }
    }
  }
  // MPI_Reduce(SUM) src/forces.c:47 (here every rank receives the total)
  if ((rc = host_allreduce(c, &mpi_force, 1, 0))) return rc;
  if (force) *force = mpi_force;
  return 0;
} MCX_CATCH

int mcx_time_step(void* ctx, int time_s, int* newton_its, double* res, int* ksp_its, double* ksp_rnorm) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  int rc;
  double U = mcx_get_displacement(ctx, time_s);
  if ((rc = mcx_apply_bc_u(ctx, U))) return rc;
  double norm = 0., norm_0 = 0.;
  int it = 0;
  while (it < c.o.newton_max_its) {
    if ((rc = mcx_set_strains(ctx)) || (rc = mcx_homogenize(ctx)) || (rc = mcx_assembly_res(ctx, &norm))) return rc;
    if (res) res[it] = norm;
    if (it == 0) norm_0 = norm;
    if (norm < c.o.newton_min_tol || norm < norm_0 * c.o.newton_rel_tol) break;
    int kits = 0, reason = 0;
    double rn = 0.;
    if ((rc = mcx_assembly_jac(ctx)) || (rc = mcx_solve(ctx, &kits, &rn, &reason)) || (rc = mcx_update_u(ctx)))
      return rc;
    if (ksp_its) ksp_its[it] = kits;
    if (ksp_rnorm) ksp_rnorm[it] = rn;
    it++;
  }
  if (newton_its) *newton_its = it;
  if ((rc = mcx_update_vars(ctx))) return rc;  // src/main.c:83
  MCX_HIP(hipEventRecord(c.ev_chunk[0], c.stream));
  return comm_wait(c, c.ev_chunk[0], "time step end");
} MCX_CATCH

// ---------------------------------------------------------------- data access
int mcx_get_u(void* ctx, double* host) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  launch_copy_pad_to_owned(c, c.u_pad, c.tmp);
  MCX_HIP(hipMemcpyAsync(host, c.tmp, sizeof(double) * 3 * c.g.nown, hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  return 0;
} MCX_CATCH

int mcx_set_u(void* ctx, const double* host) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  MCX_HIP(hipMemcpyAsync(c.tmp, host, sizeof(double) * 3 * c.g.nown, hipMemcpyHostToDevice, c.stream));
  launch_copy_owned_to_pad(c, c.tmp, c.u_pad);
  MCX_HIP(hipStreamSynchronize(c.stream));
  return 0;
} MCX_CATCH

static int get_owned(Ctx& c, const double* d, double* host) {
  MCX_HIP(hipMemcpyAsync(host, d, sizeof(double) * 3 * c.g.nown, hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  return 0;
}

int mcx_get_b(void* ctx, double* host) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  return get_owned(c, c.b, host);
} MCX_CATCH

int mcx_get_du(void* ctx, double* host) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  return get_owned(c, c.du, host);
} MCX_CATCH

static int get_gp(Ctx& c, const double* d, double* host) {
  const Geo& g = c.g;
  const int64_t E = g.nelem;
  std::vector<double> all(6 * 8 * E);
  MCX_HIP(hipMemcpyAsync(all.data(), d, sizeof(double) * all.size(), hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  // PETSc-owned elements: lower-left node in [xs - (xs>0), xe - 2] per direction
  int lo[3], hi[3], s[3] = {g.xs, g.ys, g.zs}, w[3] = {g.nx, g.ny, g.nz};
  for (int dd = 0; dd < 3; dd++) {
    lo[dd] = s[dd] > 0 ? s[dd] - 1 : s[dd];
    hi[dd] = s[dd] + w[dd] - 2;
  }
  int64_t ie = 0;
  for (int ez = lo[2]; ez <= hi[2]; ez++)
    for (int ey = lo[1]; ey <= hi[1]; ey++)
      for (int ex = lo[0]; ex <= hi[0]; ex++, ie++) {
        int64_t le = (ex - g.ex0) + (int64_t)(ey - g.ey0) * g.nex + (int64_t)(ez - g.ez0) * g.nex * g.ney;
        for (int gp = 0; gp < 8; gp++)
          for (int k = 0; k < 6; k++) host[(ie * 8 + gp) * 6 + k] = all[((int64_t)k * 8 + gp) * E + le];
      }
  return 0;
}

int mcx_get_strain(void* ctx, double* host) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  return get_gp(c, c.eps, host);
} MCX_CATCH

int mcx_get_stress(void* ctx, double* host) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  return get_gp(c, c.sig, host);
} MCX_CATCH

int mcx_owned_dofs(void* ctx, int64_t* petsc, int64_t* natural) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  const Geo& g = c.g;
  const int64_t off = 3 * c.rank_node_off[c.rank];
  for (int64_t n = 0; n < g.nown; n++) {
    int64_t i = n % g.nx, j = (n / g.nx) % g.ny, k = n / ((int64_t)g.nx * g.ny);
    int64_t nat = (g.xs + i) + (g.ys + j) * (int64_t)g.NX + (g.zs + k) * (int64_t)g.NX * g.NY;
    for (int d = 0; d < 3; d++) {
      if (petsc) petsc[3 * n + d] = off + 3 * n + d;
      if (natural) natural[3 * n + d] = 3 * nat + d;
    }
  }
  return 0;
} MCX_CATCH

int mcx_dump_csr(void* ctx, int64_t* rowptr, int64_t* colidx, double* vals) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  if (vals && !c.assembled) {
    set_error("mcx_dump_csr: no matrix assembled (call mcx_assembly_jac first)");
    return 5;
  }
  const Geo& g = c.g;
  const bool up = c.fmt == FMT_U || c.fmt == FMT_SPLIT;  // values from the upper blocks
  std::vector<double> V;
  std::vector<uint16_t> Dh;
  std::vector<unsigned char> Ih;
  std::vector<double> dict;
  std::vector<double> Xh;  // exception nodes' blocks
  if (vals && c.fmt == FMT_VI && c.vi_block && c.vi_nexc) {  // AoSoA (exc_base)
    Xh.resize((size_t)c.g.xld * 27 * 9);
    MCX_HIP(hipMemcpyAsync(Xh.data(), c.vi_exc, Xh.size() * sizeof(double), hipMemcpyDeviceToHost, c.stream));
  }
  if (vals && c.fmt == FMT_VI) {
    Ih.resize((size_t)c.vi_idx_bytes);
    dict.resize(c.vi_block ? VI_MAX * VIB_STRIDE : std::max(VI_MAX, NSLOT * 16));
    MCX_HIP(hipMemcpyAsync(Ih.data(), c.vi_idx, Ih.size(), hipMemcpyDeviceToHost, c.stream));
    MCX_HIP(hipMemcpyAsync(dict.data(), c.vi_block ? c.vi_bdict : c.vi_dict, dict.size() * sizeof(double),
                           hipMemcpyDeviceToHost, c.stream));
    MCX_HIP(hipStreamSynchronize(c.stream));
  } else if (vals) {
    V.resize(up ? c.npgroups * UPAIR * 128 : c.ngroups * NPAIR * 128);
    MCX_HIP(hipMemcpyAsync(V.data(), up ? c.U : c.V, sizeof(double) * V.size(), hipMemcpyDeviceToHost, c.stream));
    if (c.fmt == FMT_SPLIT && c.dsl.L) {
      Dh.resize((size_t)c.npgroups * c.dsl.Lq * 64 * 8);
      MCX_HIP(hipMemcpyAsync(Dh.data(), c.D, sizeof(uint16_t) * Dh.size(), hipMemcpyDeviceToHost, c.stream));
    }
    MCX_HIP(hipStreamSynchronize(c.stream));
  }
  // AIJ-split escapes: residual of (owned node, slot) added to its bf16 hi
  std::unordered_map<int64_t, double> escmap;
  if (vals && c.fmt == FMT_SPLIT && c.dsl.esc && c.dsl.nesc) {
    std::vector<unsigned> en(g.nown);
    std::vector<double> er(c.dsl.nesc);
    std::vector<unsigned char> es(c.dsl.nesc);
    MCX_HIP(hipMemcpyAsync(en.data(), c.esc_node, sizeof(unsigned) * en.size(), hipMemcpyDeviceToHost, c.stream));
    MCX_HIP(hipMemcpyAsync(er.data(), c.esc_res, sizeof(double) * er.size(), hipMemcpyDeviceToHost, c.stream));
    MCX_HIP(hipMemcpyAsync(es.data(), c.esc_slot, es.size(), hipMemcpyDeviceToHost, c.stream));
    MCX_HIP(hipStreamSynchronize(c.stream));
    for (int64_t n = 0; n < g.nown; n++)
      if (en[n]) {
        const unsigned m = en[n] >> 24, base = (en[n] & 0xffffffu) - 1u;
        for (unsigned t = 0; t < m; t++) escmap[n * 128 + es[base + t]] = er[base + t];
      }
  }
  auto escres = [&](int64_t n, int s, double& v) -> bool {
    if (escmap.empty()) return false;
    auto it = escmap.find(n * 128 + s);
    if (it == escmap.end()) return false;
    v = it->second;
    return true;
  };
  // AIJ-split: packed position of each correction slot (-1: no correction stored), stored with
  // the row node (u_of index): nb*9 + r*3 + c
  int dpos[126];
  for (int s = 0; s < 126; s++) dpos[s] = -1;
  for (int p = 0; p < c.dsl.L; p++) dpos[c.dsl.s[p]] = p;
  auto corr = [&](int64_t u, int s) -> double {
    const int p = dpos[s];
    if (p < 0) return 0.;
    const int per = c.dsl.wide ? 4 : 8;
    const int64_t q = ((u >> 6) * c.dsl.Lq + p / per) * 64 + (u & 63);
    uint32_t f = c.dsl.wide ? (uint32_t)Dh[q * 8 + 2 * (p % 4)] | ((uint32_t)Dh[q * 8 + 2 * (p % 4) + 1] << 16)
                            : (uint32_t)Dh[q * 8 + p % 8] << 16;
    float fv;
    std::memcpy(&fv, &f, 4);
    return (double)fv;
  };
  auto uval = [&](int64_t p, int s) { return V[(p >> 6) * (UPAIR * 128) + (int64_t)(s >> 1) * 128 + 2 * (p & 63) + (s & 1)]; };
  int64_t pos = 0;
  if (rowptr) rowptr[0] = 0;
  std::vector<std::pair<int64_t, double>> row;
  for (int64_t n = 0; n < g.nown; n++) {
    int64_t i = n % g.nx, j = (n / g.nx) % g.ny, k = n / ((int64_t)g.nx * g.ny);
    int64_t gi = g.xs + i, gj = g.ys + j, gk = g.zs + k;
    for (int r = 0; r < 3; r++) {
      row.clear();
      for (int nb = 0; nb < 27; nb++) {
        int64_t hi = gi + nb % 3 - 1, hj = gj + (nb / 3) % 3 - 1, hk = gk + nb / 9 - 1;
        if (hi < 0 || hj < 0 || hk < 0 || hi >= g.NX || hj >= g.NY || hk >= g.NZ) continue;
        int64_t col0 = 3 * petsc_node(c, hi, hj, hk);
        for (int cc = 0; cc < 3; cc++) {
          double v = 0.;
          if (vals && up) {
            // storage index u_of (kernels.hip): 64-aligned rows of UX nodes
            const int64_t pc = 64 + i + (j + 1) * (int64_t)g.UX + (k + 1) * (int64_t)g.UXY;
            const int64_t q = pc + (nb % 3 - 1) + ((nb / 3) % 3 - 1) * (int64_t)g.UX + (nb / 9 - 1) * (int64_t)g.UXY;
            static const int dsl[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
            double er = 0.;
            if (nb < 13) {
              v = uval(q, 6 + 9 * (12 - nb) + cc * 3 + r);
              if (c.fmt == FMT_SPLIT) {  // exact AIJ lower value (an escape: mirror + (hi + residual))
                const int s = nb * 9 + r * 3 + cc;
                v = escres(n, s, er) ? v + (corr(pc, s) + er) : v + corr(pc, s);
              }
            }
            else if (nb == 13) {
              v = uval(pc, dsl[r][cc]);
              if (c.fmt == FMT_SPLIT && r > cc) {  // lower triangle
                const int s = 13 * 9 + r * 3 + cc;
                v = escres(n, s, er) ? v + (corr(pc, s) + er) : v + corr(pc, s);
              }
            }
            else v = uval(pc, 6 + 9 * (nb - 14) + r * 3 + cc);
          } else if (vals && c.fmt == FMT_VI) {
            const int s = nb * 9 + r * 3 + cc;
            if (c.vi_block) {  // byte nb of 2 chunks of 16 B: the block's dictionary entry
              uint32_t xs = 0;  // exception slot + 1 in bytes 28-31
              std::memcpy(&xs, &Ih[(((n >> 6) * 2 + 1) * 64 + (n & 63)) * 16 + 12], 4);
              if (xs && !Xh.empty()) v = Xh[exc_base(xs - 1) + (nb * 9 + r * 3 + cc) * 64];
              else v = dict[Ih[(((n >> 6) * 2 + (nb >> 4)) * 64 + (n & 63)) * 16 + (nb & 15)] * VIB_STRIDE + r * 3 + cc];
            } else if (c.vi_bits == 8) {
              v = dict[Ih[(((n >> 6) * VI_CHUNKS + (s >> 4)) * 64 + (n & 63)) * 16 + (s & 15)]];
            } else {  // nibble s of 8 chunks of 16 B, low nibble first
              const unsigned char byte = Ih[(((n >> 6) * 8 + (s >> 5)) * 64 + (n & 63)) * 16 + ((s & 31) >> 1)];
              v = dict[s * 16 + ((s & 1) ? byte >> 4 : byte & 15)];
            }
          } else if (vals) {
            int s = nb * 9 + r * 3 + cc;
            v = V[(n >> 6) * (NPAIR * 128) + (int64_t)(s >> 1) * 128 + 2 * (n & 63) + (s & 1)];
          }
          row.emplace_back(col0 + cc, v);
        }
      }
      std::sort(row.begin(), row.end(), [](auto& a, auto& b) { return a.first < b.first; });
      for (auto& e : row) {
        if (colidx) colidx[pos] = e.first;
        if (vals) vals[pos] = e.second;
        pos++;
      }
      if (rowptr) rowptr[3 * n + r + 1] = pos;
    }
  }
  return 0;
} MCX_CATCH

int mcx_dump_dirichlet(void* ctx, int64_t* idx, int64_t* n) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  const Geo& g = c.g;
  const int64_t off = 3 * c.rank_node_off[c.rank];
  int64_t cnt = 0;
  for (int64_t q = 0; q < g.nown; q++) {
    int i = (int)(q % g.nx), j = (int)((q / g.nx) % g.ny), k = (int)(q / ((int64_t)g.nx * g.ny));
    int m = dirichlet_mask_host(g, g.xs + i, g.ys + j, g.zs + k);
    for (int d = 0; d < 3; d++)
      if (m >> d & 1) {
        if (idx && cnt < *n) idx[cnt] = off + 3 * q + d;
        cnt++;
      }
  }
  if (idx && cnt > *n) {
    *n = cnt;
    set_error("mcx_dump_dirichlet: capacity too small");
    return 4;
  }
  *n = cnt;
  return 0;
} MCX_CATCH

int mcx_spmv(void* ctx, const double* x_host, double* y_host) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  if (!c.assembled) {
    set_error("mcx_spmv: no matrix assembled (call mcx_assembly_jac first)");
    return 5;
  }
  MCX_HIP(hipMemcpyAsync(c.tmp, x_host, sizeof(double) * 3 * c.g.nown, hipMemcpyHostToDevice, c.stream));
  launch_copy_owned_to_pad(c, c.tmp, c.p_pad);
  int rc = halo_exchange(c, c.p_pad);
  if (rc) return rc;
  launch_spmv(c, c.p_pad, c.tmp, false, false);
  MCX_HIP(hipGetLastError());
  MCX_HIP(hipMemcpyAsync(y_host, c.tmp, sizeof(double) * 3 * c.g.nown, hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  return 0;
} MCX_CATCH

int mcx_get_ksp_history(void* ctx, double* hist, int64_t* n) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  int64_t have = (int64_t)c.last_hist.size();
  int64_t k = std::min(have, *n);
  if (hist) std::memcpy(hist, c.last_hist.data(), sizeof(double) * k);
  *n = have;
  return 0;
} MCX_CATCH

int mcx_set_timing(void* ctx, int on) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  c.timing = on != 0;
  return 0;
} MCX_CATCH

int mcx_get_timing(void* ctx, mcx_timing* t) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  MCX_HIP(hipStreamSynchronize(c.stream));
  double* ph[6] = {&c.t.strains_ms, &c.t.homogenize_ms, &c.t.residual_ms, &c.t.jacobian_ms, &c.t.solve_ms,
                   &c.t.update_ms};
  for (int k = 0; k < 6; k++)
    if (c.phase_rec[k]) {
      float ms = 0.f;
      MCX_HIP(hipEventElapsedTime(&ms, c.ev_phase[k][0], c.ev_phase[k][1]));
      *ph[k] = ms;
    }
  *t = c.t;
  // algorithmic bytes of one SpMV in this format: the stencil-block values actually present
  // (AIJ nonzeros of the owned rows x 8 B), x read once, y written once
  // (value-indexed: vi_bits per nonzero; the pad up to whole 16-B chunks per node is not counted)
  t->spmv_bytes_per_launch =
      (c.fmt == FMT_V    ? c.nnz_local * 8
       : c.fmt == FMT_VI ? (c.vi_block ? c.nnz_local / 9 : (c.nnz_local * c.vi_bits + 7) / 8)
                         : c.nupper_local * 8) +
      2 * 3 * (int64_t)c.g.nown * 8;
  if (c.fmt == FMT_SPLIT) t->spmv_bytes_per_launch += (int64_t)c.g.nown * c.dsl.Lq * 16;
  if (c.fmt == FMT_VI && c.vi_block) t->spmv_bytes_per_launch += c.vi_nexc * 27 * 9 * 8;  // exception blocks
  if (st_used(c)) {  // default stencil: no index bytes but the listed nodes'; the patch masks
    t->spmv_bytes_per_launch += c.st_n * 32 - c.nnz_local / 9 + (int64_t)c.st_npx * c.st_npy * c.g.nz * 8;
  } else if (wd_used(c)) {  // wave descriptors: 128 B per wave and plane, index bytes for the waves that still read per-lane words
    const int64_t nwp = (int64_t)c.wd_npx * c.wd_npy * c.g.nz;
    t->spmv_bytes_per_launch += nwp * 128 - c.nnz_local / 9 +
                                (!c.vi_fma ? c.wd_blocks_exact : c.vi_wdesc == 2 ? c.wd_blocks_two : c.wd_blocks_fma);
  }
  // the fused p update (cg_fusep): r and the diagonal index read, p(i) written
  if (c.fusep_used) t->spmv_bytes_per_launch += (int64_t)c.g.nown * (24 + 1 + 24);
  t->cg_vec_bytes_per_iter = cg_vec_bytes_per_node(c) * (int64_t)c.g.nown;
  return 0;
} MCX_CATCH

int mcx_set_option(void* ctx, const char* name, double value) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  if (!std::strcmp(name, "spmv_subl")) {
    const int old = c.spmv_subl;
    c.spmv_subl = (int)value;
    if (!partials_fit(c)) {
      c.spmv_subl = old;
      set_error("spmv_subl: partials buffer too small");
      return 2;
    }
    return 0;
  }
  if (!std::strcmp(name, "spmv_zblocks")) {
    const int old = c.spmv_zblocks;
    c.spmv_zblocks = (int)value;
    if (!partials_fit(c)) {
      c.spmv_zblocks = old;
      set_error("spmv_zblocks: partials buffer too small");
      return 2;
    }
    return 0;
  }
  if (!std::strcmp(name, "split_wide")) {  // testing: f32 corrections even when bf16 is exact
    c.split_wide = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "split_maxq")) {  // takes effect at the next mcx_assembly_jac
    c.split_declined = false;
    c.split_maxq = std::max(0, std::min(30, (int)value));
    return 0;
  }
  if (!std::strcmp(name, "split_dense")) {  // takes effect at the next mcx_assembly_jac
    c.split_declined = false;
    c.split_dense = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "split_dbg")) {
    c.split_dbg = std::max(0, std::min(2047, (int)value));  // (k_spmv_sp DBG: bits, see the kernel)
    return 0;
  }
  if (!std::strcmp(name, "face_dbg")) {  // timing-only (wrong products): bits 1 listed rows, 2 x faces, 4 y/z faces dropped
    c.face_dbg = std::max(0, std::min(7, (int)value));
    return 0;
  }
  if (!std::strcmp(name, "split_tx")) {
    const int v = (int)value;
    if (v != 0 && v != 64 && v != 128 && v != 256) {
      set_error("split_tx: 0, 64, 128 or 256");
      return 2;
    }
    const int old = c.split_tx;
    c.split_tx = v;
    if (!partials_fit(c)) {
      c.split_tx = old;
      set_error("split_tx: partials buffer too small");
      return 2;
    }
    return 0;
  }
  if (!std::strcmp(name, "cg_fuse")) {
    c.fuse = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "comm_timeout")) {  // seconds a host wait on collective work may take
    if (!(value > 0.)) {
      set_error("comm_timeout: seconds > 0");
      return 1;
    }
    c.comm_timeout = value;
    return 0;
  }
  if (!std::strcmp(name, "halo_overlap")) {
    c.overlap = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "split_ty")) {
    const int v = (int)value;
    if (v != 0 && v != 2 && v != 4 && v != 8 && v != 16) {
      set_error("split_ty: 0, 2, 4, 8 or 16");
      return 2;
    }
    const int old = c.split_ty;
    c.split_ty = v;
    if (!partials_fit(c)) {
      c.split_ty = old;
      set_error("split_ty: partials buffer too small");
      return 2;
    }
    return 0;
  }
  if (!std::strcmp(name, "vi_bits")) {  // takes effect at the next mcx_assembly_jac
    const int v = (int)value;
    if (v != 4 && v != 8) {
      set_error("vi_bits: 4 (per-slot nibbles where every slot has <= 16 values) or 8");
      return 2;
    }
    c.vi_bits_max = v;
    return 0;
  }
  if (!std::strcmp(name, "vi_block")) {  // takes effect at the next mcx_assembly_jac
    c.vi_block_on = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "cg_pdb")) {  // 0 | 1 (two p buffers) | 4 (four, the default)
    if (!(value == 0. || value == 1. || value == 4.)) {
      set_error("cg_pdb: 0, 1 (two p buffers) or 4 (four)");
      return 1;
    }
    c.cg_pdb = (int)value;
    return 0;
  }
  if (!std::strcmp(name, "cg_rev")) {
    c.cg_rev = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "cg_par")) {  // 0 | 1 (the host's parity hint) | 2 (a skewed hint: testing)
    if (!(value == 0. || value == 1. || value == 2.)) {
      set_error("cg_par: 0, 1 or 2 (testing: a wrong hint)");
      return 1;
    }
    c.cg_par = (int)value;
    return 0;
  }
  if (!std::strcmp(name, "vi_exc_list")) {
    if (value < 0. || value > VI_EXC_LIST) {
      set_error("vi_exc_list: 0 .. 2048");
      return 1;
    }
    c.vi_exc_list = (int)value;
    return 0;
  }
  if (!std::strcmp(name, "split_esc")) {  // takes effect at the next mcx_assembly_jac
    c.split_esc = value != 0.;
    c.split_declined = false;
    return 0;
  }
  if (!std::strcmp(name, "vi_lg")) {
    if (!(value == 1. || value == 2. || value == 3.)) {
      set_error("vi_lg: 1, 2 or 3");
      return 1;
    }
    c.vi_lg = (int)value;
    return 0;
  }
  if (!std::strcmp(name, "cg_p2d")) {
    c.cg_p2d = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "vi_st_faces")) {  // rebuilds the default-stencil structures if built
    const int old = c.vi_st_faces;
    c.vi_st_faces = (int)value & 0x7f;  // 1: all 6 faces; else bit c = face class c (1..6)
    if ((c.st_ok || c.st_pending) && build_st(c)) return 1;
    if (!partials_fit(c)) {
      c.vi_st_faces = old;
      set_error("vi_st_faces: partials buffer too small");
      return (c.st_ok || c.st_pending) && build_st(c) ? 1 : 2;
    }
    return 0;
  }
  if (!std::strcmp(name, "vi_st_pair")) {
    const int old = c.vi_st_pair;
    c.vi_st_pair = value != 0.;
    if (!partials_fit(c)) {
      c.vi_st_pair = old;
      set_error("vi_st_pair: partials buffer too small");
      return 2;
    }
    return 0;
  }
  if (!std::strcmp(name, "vi_st_fstream")) {
    c.vi_st_fstream = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "vi_st_l16")) {
    if (!(value == -1. || value == 0. || value == 1.)) {
      set_error("vi_st_l16: -1 (by the list's length), 0 or 1");
      return 1;
    }
    const int old = c.vi_st_l16;
    c.vi_st_l16 = (int)value;
    if (!partials_fit(c)) {
      c.vi_st_l16 = old;
      set_error("vi_st_l16: partials buffer too small");
      return 2;
    }
    return 0;
  }
  if (!std::strcmp(name, "vi_st_pf")) {
    if (!(value == 1. || value == 2. || value == 3.)) {  // 3: timing-only, the ring never refilled (wrong rows)
      set_error("vi_st_pf: 1 or 2");
      return 1;
    }
    c.vi_st_pf = (int)value;
    return 0;
  }
  if (!std::strcmp(name, "vi_st_ty")) {
    if (!(value == 8. || value == 16.)) {
      set_error("vi_st_ty: 8 or 16");
      return 1;
    }
    const int old = c.vi_st_ty;
    c.vi_st_ty = (int)value;
    if (!partials_fit(c)) {
      c.vi_st_ty = old;
      set_error("vi_st_ty: partials buffer too small");
      return 2;
    }
    return 0;
  }
  if (!std::strcmp(name, "vi_st_tail")) {
    const int old = c.vi_st_tail;
    c.vi_st_tail = value != 0.;
    if (!partials_fit(c)) {
      c.vi_st_tail = old;
      set_error("vi_st_tail: partials buffer too small");
      return 2;
    }
    return 0;
  }
  if (!std::strcmp(name, "vi_st")) {  // takes effect at once if the structures were built (they are by default)
    if (!(value == -1. || value == 0. || value == 1.)) {
      set_error("vi_st: -1 (by size), 0 or 1");
      return 1;
    }
    const int old = c.vi_st;
    c.vi_st = (int)value;
    if (c.st_pending && st_wanted(c) && build_st(c)) return 1;  // built lazily: the path turned on
    if (!partials_fit(c)) {
      c.vi_st = old;
      set_error("vi_st: partials buffer too small");
      return 2;
    }
    return 0;
  }
  if (!std::strcmp(name, "vi_exc_kernel")) {
    const bool old = c.vi_exc_kernel;
    c.vi_exc_kernel = value != 0.;
    if (!partials_fit(c)) {
      c.vi_exc_kernel = old;
      set_error("vi_exc_kernel: partials buffer too small");
      return 2;
    }
    return 0;
  }
  if (!std::strcmp(name, "vi_lg_exc")) {
    c.vi_lg_exc = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "cg_xs")) {  // takes effect at the next solve (with cg_pdb 4)
    c.cg_xs = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "cg_ublocks")) {
    if (value < 0 || value > (1 << 30) || value != (double)(int)value) {
      set_error("cg_ublocks: 0 (uncapped) or a block count");
      return 1;
    }
    c.cg_ublocks = (int)value;
    return 0;
  }
  if (!std::strcmp(name, "vi_wdesc")) {
    if (!(value == 0. || value == 1. || value == 2.)) {
      set_error("vi_wdesc: 0, 1 or 2");
      return 1;
    }
    c.vi_wdesc = (int)value;
    return 0;
  }
  if (!std::strcmp(name, "vi_ypair")) {
    c.vi_ypair = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "vi_wmap")) {
    c.vi_wmap = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "vi_ring3")) {
    c.vi_ring3 = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "vi_tx")) {  // validated before it is stored: a refused width leaves the tiling as it was
    const int v = (int)value;
    if (!(v == 0 || v == 64 || v == 128 || v == 256) || (double)v != value) {
      set_error("vi_tx: 0 (default), 64, 128 or 256");
      return 1;
    }
    const int old = c.vi_tx;
    c.vi_tx = v;
    if (!partials_fit(c)) {
      c.vi_tx = old;
      set_error("vi_tx: partials buffer too small");
      return 7;
    }
    return 0;
  }
  if (!std::strcmp(name, "cg_fusep")) {
    c.cg_fusep = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "vi_exc_max")) {  // takes effect at the next mcx_assembly_jac
    c.vi_exc_max = std::max(0, std::min(1000, (int)value));
    c.vi_declined = false;
    return 0;
  }
  if (!std::strcmp(name, "vib_onepass")) {  // takes effect at the next mcx_assembly_jac
    c.vib_onepass = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "vi_fma")) {
    c.vi_fma = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "vi_patch")) {
    c.vi_patch = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "vi_uni")) {
    c.vi_uni = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "vi_xread")) {
    c.vi_xread = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "vi_stage")) {
    const int old = c.vi_stage;
    c.vi_stage = value < 0. ? -1 : (value != 0. ? 1 : 0);
    if (!partials_fit(c)) {
      c.vi_stage = old;
      set_error("vi_stage: partials buffer too small");
      return 2;
    }
    return 0;
  }
  if (!std::strcmp(name, "aij_vi")) {  // takes effect at the next mcx_assembly_jac
    if (c.o.mat_type != MCX_MAT_AIJ) {
      set_error("aij_vi: -dm_mat_type aij only");
      return 2;
    }
    c.vi_declined = false;
    c.aij_vi = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "aij_split")) {  // takes effect at the next mcx_assembly_jac
    c.split_declined = false;
    if (value != 0. && !c.d_mask) {
      set_error("aij_split: context created with -mat_aij_split 0 (no split storage)");
      return 2;
    }
    c.aij_split = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "cg_dix")) {
    c.cg_dix = value != 0.;
    return 0;
  }
  if (!std::strcmp(name, "cg_nt")) {
    c.cg_nt = (int)value;
    return 0;
  }
  if (!std::strcmp(name, "spmv_nt")) {
    c.spmv_nt = (int)value;
    return 0;
  }
  if (!std::strcmp(name, "spmv_kernel")) {
    const int old = c.spmv_kernel;
    c.spmv_kernel = (int)value;
    if (!partials_fit(c)) {
      c.spmv_kernel = old;
      set_error("spmv_kernel: partials buffer too small");
      return 2;
    }
    return 0;
  }
  set_error(std::string("unknown option ") + name);
  return 2;
} MCX_CATCH

int mcx_time_spmv(void* ctx, int iters, double* avg_ms) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  if (!c.assembled) {
    set_error("mcx_time_spmv: no matrix assembled");
    return 5;
  }
  launch_spmv(c, c.p_pad, c.w, true, false);  // warm
  MCX_HIP(hipEventRecord(c.ev_a, c.stream));
  for (int q = 0; q < iters; q++) launch_spmv(c, c.p_pad, c.w, true, false);
  MCX_HIP(hipEventRecord(c.ev_b, c.stream));
  MCX_HIP(hipEventSynchronize(c.ev_b));
  float ms = 0.f;
  MCX_HIP(hipEventElapsedTime(&ms, c.ev_a, c.ev_b));
  *avg_ms = ms / std::max(iters, 1);
  return 0;
} MCX_CATCH

int mcx_synchronize(void* ctx) try {
  MCX_ENTRY();
  GUARD(ctx);
  CTX(ctx);
  MCX_HIP(hipEventRecord(c.ev_chunk[0], c.stream));  // the stream may hold collectives: bounded wait
  return comm_wait(c, c.ev_chunk[0], "mcx_synchronize");
} MCX_CATCH

}  // extern "C"
