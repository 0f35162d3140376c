// mcx_internal.h — context, geometry and kernel-launcher declarations of the MI355X
// MacroC hot path.  See DESIGN.md for the HBM layout; include/macroc_amd.h for the ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/macroc_amd.h"

namespace mcx {

constexpr int NGP = 8, NPE = 8, NVOI = 6;
constexpr int NSLOT = 243;   // 27 neighbour blocks x 3x3
constexpr int NPAIR = 122;   // slots stored as double2 pairs (slot 243 = zero pad)
constexpr int GROUP = 64;    // nodes per AoSoA group (= one wavefront)
constexpr int USLOT = 123;   // sbaij: 6 upper-triangle diagonal values + 13 upper blocks x 9
constexpr int UPAIR = 62;

void set_error(const std::string& s);

// Geometry of one rank's subdomain, passed by value to every kernel.
struct Geo {
  int NX, NY, NZ;          // global node counts
  int xs, ys, zs;          // first owned node (global)
  int nx, ny, nz;          // owned node counts
  int PX, PY, PZ;          // padded box = owned + 1 ghost layer each side
  int UX, UXY;             // sbaij storage pitch: rows of UX = roundup(nx+2, 64) nodes (u_of)
  int ncu;                 // compute units (z-marching grid sizing)
  int nown;                // nx*ny*nz
  int ex0, ey0, ez0;       // first element evaluated on this device (global)
  int nex, ney, nez;       // extended element counts (owned + upper ghost layer)
  int64_t nelem;           // nex*ney*nez
  int64_t xld;             // value-indexed exception blocks: slot capacity of exc (a multiple of 64, exc_base)
  int bc_type;
  double lx, lz, dx, dz, rad, wg;
};

// device-side state of the CG loop (PETSc KSPSolve_CG scalars)
struct CgState {
  double beta, betaold, dpi, dpiold, alpha, dp, ttol, rnorm0, bcoef;
  double rtol, abstol, dtol;
  int i, its, reason, maxits, hist_on;
  int xpend;  // x += alpha p of the last iteration not yet applied (k_cg_pupdate / k_cg_xfinal apply it)
  int xp;     // the last iteration whose alpha step succeeded (-1: none); the fused path's pending x update
  double alpha_prev;  // alpha of the iteration before (the fused path's every-second-iteration x update)
  double ah[8];       // alpha of iteration j at ah[j & 7] (quad-buffered p: x every fourth iteration)
};

struct Material {
  int law;                 // MCX_LAW_ELASTIC | MCX_LAW_PLASTIC
  double E, nu, Sy, Ka;
  double C[36];            // isotropic elastic tangent (Voigt, engineering shear)
};

struct HaloPlan {
  std::vector<int> nbr_rank;          // neighbour ranks (<= 26)
  std::vector<int64_t> send_off, send_cnt, recv_off, recv_cnt;  // in nodes
  int* d_send_idx = nullptr;          // padded node index of each sent node
  int* d_recv_idx = nullptr;          // padded node index of each received node
  double* d_sendbuf = nullptr;
  double* d_recvbuf = nullptr;
  int64_t nsend = 0, nrecv = 0;
  int* d_bnd = nullptr;               // owned node index of every sent node, each once
  int64_t nbnd = 0;
};

struct Ctx;

// value-indexed exception blocks, AoSoA: groups of 64 slots, each group value-major (243 runs of 64
// doubles, one per value (nb, r, c)), so a wave of 64 consecutive slots reads one 512-B run per value
// and a group's values are contiguous (124 KB); value v of slot s at exc[exc_base(s) + v * 64]
__host__ __device__ inline int64_t exc_base(int64_t s) { return (s >> 6) * (243 * 64) + (s & 63); }

// Matrix storage of a context.  FMT_V: AIJ stencil blocks (all 27 blocks per node, every row
// summed in the reference's MatMult order (inode column pairs)).  FMT_U: MATSBAIJ (upper blocks, lower mirrored).  FMT_SPLIT:
// the AIJ matrix held exactly as its upper blocks U plus, per owned node, the bf16 correction
// lower - mirror(upper) of the correction slots that are non-zero somewhere in the matrix
// (every AIJ value reconstructs bit for bit; rows summed in the z-marching order).
// FMT_VI: the AIJ matrix held exactly as small indices into dictionaries of its distinct values
// (value-indexed CSR, Kourtis et al. 2008): a nibble per value into the slot's own dictionary
// (every slot takes at most 16 values) or a byte per value into one dictionary (at most 256),
// all 27 blocks per node in FMT_V's slot order — every row summed in the reference's MatMult order (inode column pairs).
enum Fmt { FMT_V = 0, FMT_U = 1, FMT_SPLIT = 2, FMT_VI = 3 };
constexpr int VI_MAX = 256;     // dictionary entries (one index byte per value)
constexpr int VI_EXC_LIST = 2048;  // staged value-indexed SpMV: exception nodes a tile defers to its block-wide pass
constexpr int VI_HASH = 4096;   // open-addressing set of the distinct values (bit patterns)
constexpr int VI_CHUNKS = 16;   // 16-B index chunks per node: 243 slots + 13 zero pad bytes
// vi_st -1: the default-stencil SpMV from this many owned nodes (at 256^3 it saves 2 % of a CG
// iteration, at 128^3 the faces' share makes it 6 % slower: profiles/r05p_*)
constexpr int64_t ST_MIN_NODES = int64_t(1) << 23;
constexpr int ST_CLASSES = 7;   // default-stencil SpMV: the interior + the 6 domain faces (k_st_setup)
struct StFaces {  // the face phase of the default-stencil SpMV: class c's patches (64 x 4 nodes) are [u[c-1], u[c])
  int64_t u[7];
};
constexpr int VIB_STRIDE = 10;  // doubles per dictionary block (9 values + pad: 16-B aligned)
constexpr int VB_GSV = 64;      // single-pass block build: entries of each slot's global value set (6-bit positions)

// AIJ-split correction slots, passed by value: slot = nb*9 + r*3 + c of the row node's lower
// block nb < 13 holds A(n, nb)[r][c] - U(m, 26-nb)[c][r], m = n + off(nb); nb = 13 (the
// diagonal block, stored as its upper triangle) holds A(n,n)[r][c] - A(n,n)[c][r] for r > c
struct DSlots {
  int L = 0, Lq = 0;        // active slots; 16-B quads per node ([u_of/64][Lq][64])
  int wide = 0;             // 0: 8 bf16 per quad; 1: 4 f32 per quad (some correction not exact in bf16)
  unsigned char s[120];     // ascending active slot ids (at most 117 + 3)
  unsigned short m9[14];    // per lower block nb (13: diagonal): active (r*3+c) bits
  unsigned char pos[14];    // per block: index of its first active slot
  int xc[24];               // slot p < 24: (x offset from 3 * padded index of the row node) * 4 + row
  int dense = 0;            // 1: all 120 slots stored in canonical order (nb*9 + r*3 + c, then the diagonal's
                            // (1,0) (2,0) (2,1)) and applied by a second pass, k_split_dense
  int esc = 0;              // dense bf16 with escapes: a correction not exact in bf16 keeps its truncated bf16
                            // hi in D plus the exact residual d - hi in the escape arrays (Ctx::esc_*)
  int nesc = 0;             // escaped corrections of the current matrix
};

// In-process transport: several contexts (one host thread each) exchanging halos and partial
// sums by device copies + events.  Used to run the multi-rank path on one GPU (tests) and for
// a single process driving several GPUs; the RCCL transport is the multi-process path.
struct LocalGroup {
  int nranks = 0;
  std::vector<Ctx*> members;
  std::vector<hipEvent_t> ev_packed, ev_halo_done, ev_red, ev_sum;
  double** d_red_ptrs = nullptr;   // device array: red_loc of every member
  int device = 0;
  bool dev_ready = false;          // events + d_red_ptrs created (by the first mcx_init_local)
  // host barrier: every crossing is tagged with the collective it belongs to, so members that
  // reach different collectives (one rank finalizing while another exchanges a halo) fail
  // instead of pairing up; a member that never arrives fails the others after timeout_s
  void* mtx = nullptr;
  void* cv = nullptr;
  int count = 0, generation = 0;
  int cur_tag = 0, cur_rank = -1;  // the first arrival of the open generation
  double timeout_s = 300.;         // MCX_COMM_TIMEOUT (seconds) at creation
  bool broken = false;             // a mismatch or a timeout happened: every later crossing fails
  std::string why;                 // ... and what it was
};
// barrier tags (which collective a crossing belongs to)
enum { BAR_INIT = 1, BAR_HALO_PACKED, BAR_HALO_DONE, BAR_RED_IN, BAR_RED_SUM, BAR_FINALIZE, BAR_USER };
int group_barrier(LocalGroup* g, int rank, int tag, double timeout_s);  // 0, or 23 with the reason in mcx_last_error
double comm_timeout_default();                       // MCX_COMM_TIMEOUT, default 300 s

struct Ctx {
  mcx_opts o;
  int rank = 0, nranks = 1, device = 0;
  int m = 1, n = 1, p = 1, pi = 0, pj = 0, pk = 0;
  std::vector<int64_t> wx, wy, wz, sx, sy, sz;  // ownership widths / starts per rank column
  std::vector<int64_t> rank_node_off;           // nranks + 1
  Geo g{};
  double dy = 0;
  Material mat{};
  hipStream_t stream = nullptr;
  hipStream_t comm_stream = nullptr;            // halo exchange (overlaps interior work on `stream`)
  hipEvent_t ev_pack = nullptr, ev_comm = nullptr;
  int overlap = 1;                              // CG: interior p update overlaps the halo (option halo_overlap)
  void* comm = nullptr;                         // ncclComm_t when nranks > 1 (RCCL transport)
  LocalGroup* lg = nullptr;                     // in-process transport
  double comm_timeout = 300.;                   // seconds a host wait on collective work may take (option comm_timeout)
  bool comm_broken = false;                     // the communicator was aborted (timeout / async error): collectives fail
  std::string comm_why;
  HaloPlan halo;

  // device arrays
  double* u_pad = nullptr;   // displacement, padded ghosted box [PX*PY*PZ][3]
  int pad_align = 1;         // padded box: 1 = row pitch PX a multiple of 16 nodes and node (0, j, k) of
                             // every row at a 128-B line (pad_off 104), 2 = the same pitch with the
                             // ghost column (-1, j, k) at a line (pad_off 0), 0 = PX = nx + 2 (round 4)
  int pad_off = 104;         // bytes from an allocation's base to padded node 0
  std::vector<void*> pad_bases;  // allocations of the padded vectors (freed by base)
  double* p_pad = nullptr;   // CG search direction, padded
  double* p_pad2 = nullptr;  // its second buffer (single rank: the p update fused into the SpMV, cg_fusep)
  double* p_pad3 = nullptr;  // third and fourth buffers (cg_pdb 4), allocated at the first solve that uses them
  double* p_pad4 = nullptr;
  double* p_pad58[4] = {nullptr, nullptr, nullptr, nullptr};  // buffers 5-8 (cg_xs)
  int cg_xs = 0;             // quad-buffered p: the four owed VecAXPY(x) terms on a side stream (option cg_xs)
  bool xs_used = false;      // this solve: eight p buffers, k_cg_xwin on x_stream
  hipStream_t x_stream = nullptr;
  hipStream_t f_stream = nullptr;                  // k_spmv_face beside the march (vi_st_fstream)
  hipEvent_t ev_fx = nullptr, ev_fd = nullptr;     // p ready for the face stream / the faces done
  int vi_st_fstream = 0;                           // option vi_st_fstream
  hipEvent_t ev_xp = nullptr, ev_xd[2] = {nullptr, nullptr};
  int cg_fusep = 0;          // option cg_fusep: fuse the CG p update into the value-indexed SpMV (single rank; A/B: no gain)
  bool fusep_used = false;   // the last solve ran the fused kernel (timing: its bytes per launch)
  int cg_pdb = 4;            // option cg_pdb: 1 = p double-buffered (p_pad / p_pad2), VecAXPY(x) every second
                             // iteration; 4 = four buffers, x every fourth iteration; 0 = one buffer, x every iteration
  bool pdb_used = false;     // the current solve runs the double-buffered p update
  bool pqb_used = false;     // ... the quad-buffered one (cg_pdb 4; pdb_used too)
  int cg_rev = 1;            // option cg_rev: PDB p update from the last node down (the update kernel's last r writes hit the Infinity Cache)
  int cg_par = 1;            // option cg_par: PDB p update specialised per iteration parity (host count cg_it)
  int* xdone = nullptr;      // PDB: the last odd iteration whose p update applied the x terms owed
  int cg_it = 0;             // iteration index of the cg_iteration being launched
  double* b = nullptr;       // residual (owned, PETSc-local order)
  double* du = nullptr;      // CG solution x
  double* r = nullptr;
  double* z = nullptr;
  double* w = nullptr;
  double* dinv = nullptr;    // Jacobi inverse diagonal (inside the jdd buffer: jdd + 3 VI_MAX)
  unsigned char* jix = nullptr;  // block-indexed storage: each owned node's diagonal-block index
  double* jdd = nullptr;         // block-indexed storage: the dictionary's inverse diagonals [VI_MAX][3]
  int cg_dix = 1;                // CG kernels: Jacobi from jix/jdd, z recomputed from r (option cg_dix)
  double* V = nullptr;       // aij stencil-block matrix, AoSoA [ngroups][NPAIR][64] double2
  double* U = nullptr;       // sbaij upper stencil blocks over the padded box [npgroups][UPAIR][64] double2
  uint16_t* D = nullptr;     // AIJ-split: bf16 corrections of the padded box [u_of/64][dsl.Lq][64] x 8
  int64_t D_bytes = 0;       // allocated bytes of D (grown to the active slots' quads)
  unsigned* esc_node = nullptr;   // AIJ-split escapes: per owned node count << 24 | (first entry + 1), 0 = none
  double* esc_res = nullptr;      // escaped corrections' residuals d - hi, a node's entries in slot order
  unsigned char* esc_slot = nullptr;  // their slots (nb*9 + r*3 + c)
  int64_t esc_cap = 0;            // allocated escape entries
  int split_esc = 1;              // option split_esc: dense corrections as bf16 + escapes when some are not bf16-exact
  unsigned* d_mask = nullptr;  // AIJ-split assembly: [0..13] slot masks per lower block, [14] inexact
  // value-indexed AIJ (FMT_VI): index bytes [ngroups][VI_CHUNKS][64] x 16 B, the dictionary
  // (VI_MAX doubles, ascending bit pattern), the build's value set and its slot -> index map
  unsigned char* vi_idx = nullptr;
  int64_t vi_idx_bytes = 0;               // allocated bytes of vi_idx (grown to the mode's 32 / 128 / 256 B per node)
  double* vi_dict = nullptr;
  unsigned long long* vi_keys = nullptr;  // [VI_HASH] the value set, [NSLOT][32] the slots' sets, [VI_HASH] the block set
  unsigned char* vi_slot = nullptr;       // index of every set entry ([VI_HASH] or [NSLOT][32]), then the blocks'
  unsigned* vi_ctl = nullptr;             // [0] distinct values, [1] > VI_MAX, [2] a slot > 16, [3 + S] per slot, blocks'
                                          // [3 + NSLOT] count, [4 + NSLOT] > VI_MAX
  int vi_n = 0;                           // distinct values of the current matrix
  int vi_bits = 8;                        // 4: per-slot nibble indices, 8: one byte per value
  int vi_bits_max = 4;                    // option vi_bits: 8 = never use nibble indices
  bool vi_block = false;                  // one byte per 3x3 block into a dictionary of blocks (k_spmv_vib)
  int vi_block_on = 1;                    // option vi_block: try the block dictionary (needs nibbles)
  int vi_nblocks = 0;                     // distinct blocks of the current matrix (block mode)
  double* vi_bdict = nullptr;             // [VI_MAX][VIB_STRIDE] dictionary blocks
  // single-pass block build (k_vib_build + k_vib_remap): per-slot value sets [NSLOT][VB_GSV] and
  // the block-code set [VI_HASH] (one buffer), its control words, every (block position, owned
  // node)'s block-set position [27][nown], and the pinned host images of what crosses PCIe
  unsigned long long* vib_keys = nullptr;
  unsigned* vib_ctl = nullptr;
  unsigned short* vib_pos = nullptr;
  int64_t vib_pos_bytes = 0;
  unsigned long long* h_vib_keys = nullptr;  // readback: sets + ctl
  unsigned char* h_vib_map = nullptr;        // upload: block-set position -> dictionary index [VI_HASH]
  double* h_vib_dict = nullptr;              // upload: [VI_MAX][VIB_STRIDE]
  int vib_onepass = 1;       // option vib_onepass: the single-pass block build (0: round 2's three passes)
  // exception nodes (per-GP-tangent laws, one-pass block build): an owned node touching an
  // element whose tangent differs from the law's reference tangent at some Gauss point keeps its
  // 27 blocks as plain values, [slot][27][9]; its index chunk carries slot + 1 in bytes 28-31
  unsigned char* elem_plain = nullptr;  // [nelem] 1 = every GP tangent equals cref bit for bit
  double* cref = nullptr;               // [36] the reference tangent (plastic: the elastic branch's C)
  unsigned* vi_xslot = nullptr;         // [nown] exception slot + 1, 0 = indexed node
  int* vi_xlist = nullptr;              // [nown] exception slot -> owned node
  unsigned* vi_xcnt = nullptr;          // [node blocks + 1] exception nodes per block, then their exclusive scan
  double* vi_exc = nullptr;             // block values [slot/64][27 x 9][slot%64] (exc_base)
  int64_t vi_exc_bytes = 0;             // allocated bytes of vi_exc
  int64_t vi_nexc = 0;                  // exception nodes of the current matrix
  bool plain_ke = false;                // this assembly formed kref + the non-plain elements' Ke only
  int vi_exc_max = 300;                 // option vi_exc_max: per-mille of owned nodes beyond which the
                                        // assembly falls back to AIJ-split (0: no exceptions)
  double* ke_uni = nullptr;  // elastic law: the element matrix [8 a][8 b][9], the same for every element
  int aij_vi = 1;            // aij: assemble in FMT_VI when the matrix has at most VI_MAX distinct values
  int vi_fma = 1;            // staged block-indexed SpMV: fused multiply-add rows (-mat_vi_fma, option vi_fma;
                             // rounding-level, not bit-exact); implies vi_uni + vi_patch
  int vi_patch = 1;          // with vi_uni: 16 x 4 node patches per wave (option vi_patch)
  int vi_ring3 = 0;          // A/B: the 3-slot x ring (two barriers per plane) for 64x16 tiles (option vi_ring3)
  int vi_exc_list = VI_EXC_LIST;  // staged block-indexed SpMV: exception nodes per tile deferred to its block pass (option vi_exc_list)
  int vi_wmap = 1;           // staged block-indexed SpMV: 16x4 patches on SIMDs as a Latin square (option vi_wmap; 0: row-major)
  int vi_tx = 0;             // staged block-indexed SpMV tile width 256 | 128 | 64 (0: 64; option vi_tx)
  int vi_uni = 1;            // staged block-indexed SpMV: wave-uniform blocks from scalar loads (option vi_uni)
  int vi_ypair = 0;          // with vi_uni: y of lane pairs as 16-B stores (option vi_ypair; A/B)
  int cg_ublocks = 0;        // k_cg_update grid cap (grid-stride; option cg_ublocks, 0 = one node per thread; A/B)
  int vi_lg = 2;             // staged block-indexed SpMV, LDS-dictionary waves: blocks whose reads are issued together (option vi_lg: 1, 2, 3)
  int cg_p2d = 0;            // quad-buffered p update on a (rows, x chunks) grid: no per-node divisions (option cg_p2d; A/B)
  int vi_lg_exc = 1;         // vi_lg 2 also in the exception-node kernel (option vi_lg_exc; 0: per-block waits)
  int vi_st = -1;            // default-stencil SpMV (k_spmv_st + k_spmv_face, option vi_st; FMA rows, 64 x 16 tiles):
                             // -1 (default) from ST_MIN_NODES owned nodes up or with <= 10 % exception nodes, 0 off, 1 on
  int vi_st_faces = 1;       // the domain faces as stencil classes of their own (option vi_st_faces: 1 all, 0 none (listed), else bit c = class c)
  int vi_st_l16 = -1;        // k_spmv_face's listed rows: 16 lanes per node, loads in parallel (option vi_st_l16 1; 0: one
                             // thread per node, st_tail; -1: 16 lanes while the list is short, kernels.hip st_l16)
  int vi_st_pf = 1;          // k_spmv_st's prefetch distance in steps (option vi_st_pf 1 | 2)
  int vi_st_ty = 16;         // k_spmv_sp's tile height (option vi_st_ty: 8 = 512-thread blocks, two per CU; 16 = 1024)
  int vi_st_pair = 0;        // the march as k_spmv_sp (x-pair lanes, round 6; option vi_st_pair 1; the fused p update
                             // on this path needs it): 0.2920 vs 0.2757 ms for k_spmv_st + k_spmv_face (r06t)
  int vi_st_tail = 0;        // its faces and listed rows in the march's blocks after the march (option vi_st_tail; 0: k_spmv_face)
  double* st_coef = nullptr;            // [ST_CLASSES][27][VIB_STRIDE] the stencil classes' blocks
  unsigned* st_ids = nullptr;           // [ST_CLASSES][8] their 7 index words, [7] = class usable
  unsigned* st_slot = nullptr;          // [nown] list position + 1 of a non-default node, 0 = default
  int* st_list = nullptr;               // [nown] non-default nodes in owned-node order
  unsigned* st_cnt = nullptr;           // [node blocks + 1] scan scratch
  unsigned long long* st_mask = nullptr;  // [nz][npy][npx] 16 x 4 patch masks (bit = the march leaves the lane: faces, listed rows)
  int64_t st_mask_bytes = 0, st_n = 0;
  int st_npx = 0, st_npy = 0;
  bool st_ok = false;                   // built for the current block indices
  bool st_pending = false;              // not built: the last assembly's SpMV did not want the path
  unsigned st_fm = 0;                   // bit c: stencil class c usable (k_st_setup)
  StFaces st_faces = {};                // the face phase's units per class
  int vi_exc_kernel = 1;     // staged SpMV: exception rows in their own kernel after the march (k_spmv_exc, option
                             // vi_exc_kernel; 0: round 4's block-wide pass in each tile's tail)
  int vi_wdesc = 1;          // staged block-indexed SpMV: wave descriptors (option vi_wdesc): 1 = uniform waves (default since round 5: -2.1 % per CG iteration), 2 = also two-set waves (FMA rows), 0 = per-lane index words
  unsigned* wd = nullptr;    // wave descriptors [plane][npy][npx][8] + 2 counters (build_wdesc)
  int64_t wd_bytes = 0;
  bool wd_ok = false;        // descriptors built for the current block indices
  int wd_npx = 0, wd_npy = 0;
  int64_t wd_blocks_fma = 0, wd_blocks_exact = 0, wd_blocks_two = 0;  // present blocks of the nodes in waves that read per-lane words
  int vi_xread = 1;          // staged block-indexed SpMV: x as unpaired 8-B LDS reads (option vi_xread; 0: compiler's pairs)
  int vi_stage = -1;         // FMT_VI SpMV: 1 = x staged in LDS, z-marching tiles; 0 = x gathered; -1 = by grid (vi_staged)
  bool vi_declined = false;  // a per-GP-tangent law overflowed the dictionary: skip the attempt
  int fmt = FMT_V;           // storage the matrix is currently assembled in
  bool assembled = false;    // a matrix has been assembled (mcx_assembly_jac)
  int aij_split = 1;         // aij: assemble in FMT_SPLIT when every correction is exact in bf16
  int split_maxq = 4;        // AIJ-split only while the corrections fit this many 16-B quads per node
  int split_dense = 1;       // corrections beyond split_maxq quads: 1 = all 120 slots + a second pass, 0 = AIJ blocks
  bool split_declined = false;  // a correction was not exact (or dense ones are refused): assemble AIJ blocks directly
  int split_dbg = 0;         // timing-only diagnostics of the split SpMV (option split_dbg)
  int face_dbg = 0;          // timing-only: k_spmv_face without (1) listed rows, (2) x-face, (4) y/z-face patches
  int split_wide = 0;        // force f32 corrections (testing the wide path)
  int split_tx = 0;          // AIJ-split tile width (0: by subdomain width, 4 rows; else 1024 / split_tx rows)
  int split_ty = 0;          // AIJ-split: 2 with split_tx 256 selects 256x2 tiles (option split_ty)
  DSlots dsl;
  int64_t npgroups = 0;
  int64_t nupper_local = 0;  // sbaij: stored upper values of the owned rows
  int spmv_subl = 0;         // SpMV sweep: lines per sub-slab of an XCD's slab (0 = whole slab, -1 = linear order)
  int spmv_kernel = 0;       // sbaij: 0 = pull, 1..4 = z-marching push/pull tiles (shapes, see z_shape)
  int cg_nt = 0;             // CG vector kernels: non-temporal stores of x, r, z, p
  int spmv_zblocks = 0;      // z-marching: target block count (0: one resident round, CUs x blocks/CU)
  int ncu = 0;               // compute units of the device
  int spmv_nt = 2;           // aij: 1 = non-temporal matrix loads, 2 = + non-temporal y stores (-3 %, spmv_ab)
  int64_t partials_cap = 0;
  double* eps = nullptr;     // [6][8][nelem]
  double* sig = nullptr;     // [6][8][nelem]
  double* ctan = nullptr;    // [36][8][nelem] per-GP tangent (plastic / external laws only)
  double* Ke = nullptr;      // [576][nelem] element matrices (plastic / external laws only)
  double* hist_old = nullptr; // plastic law: [7][8][nelem] plastic strain (tensor comps) + alpha
  double* hist_new = nullptr;
  double* ftrial = nullptr;  // [8][nelem]
  double* partials = nullptr;
  double* partials2 = nullptr;  // second half of partials: the CG update's z.z / z.r partial sums
  int fuse = 1;              // single rank: CG scalar steps folded into the vector kernels (option cg_fuse)
  double* red = nullptr;     // reduction results (device)
  double* red_loc = nullptr; // local sums before all-reduce
  CgState* cg = nullptr;     // [2]: cg[0] the state the host polls; cg[1] the fused path's post-alpha state
  double* hist = nullptr;
  double* tmp = nullptr;     // owned-vector scratch for host copies
  CgState* h_cg = nullptr;   // pinned mirror
  int64_t ngroups = 0;
  int64_t device_bytes = 0;
  int64_t nnz_local = 0, nnz_global = 0;

  // external Gauss-point law (-mat_law external): host MicroPP-shaped callbacks or a device law
  mcx_micropp_api mpp{};
  bool has_mpp = false;
  mcx_device_law dlaw{};
  bool has_dlaw = false;
  std::vector<double> h_gp;  // host staging of eps / sig / ctan for the host callbacks

  // timing
  bool timing = false;
  mcx_timing t{};
  std::vector<hipEvent_t> ev_pool;
  hipEvent_t ev_a = nullptr, ev_b = nullptr;
  // per-phase event pairs (strains, homogenize, residual, jacobian, solve, update): recorded
  // without a host wait, resolved by mcx_get_timing
  hipEvent_t ev_phase[6][2] = {};
  bool phase_rec[6] = {};
  hipEvent_t ev_chunk[2] = {nullptr, nullptr};
  int last_its = 0;
  std::vector<double> last_hist;
};

// ---- decomposition (dmda.cpp)
int dmda_decide(int64_t M, int64_t N, int64_t P, int size, int* m, int* n, int* p);
int setup_decomposition(Ctx& c);
int64_t petsc_node(const Ctx& c, int64_t i, int64_t j, int64_t k);
int build_halo_plan(Ctx& c);
void plan_halo(Ctx& c, std::vector<int>& sidx, std::vector<int>& ridx);
int64_t pad_to_natural(const Ctx& c, int p);
int64_t count_nnz_rows(const Ctx& c, int64_t xs, int64_t ys, int64_t zs, int64_t nx, int64_t ny, int64_t nz);
void compute_B_table(double B[8][6][24]);
int64_t count_upper_values(const Ctx& c);

// ---- communication (comm.cpp)
int comm_init(Ctx& c, const void* id);
void comm_destroy(Ctx& c);
int halo_exchange(Ctx& c, double* xpad);   // halo_start + halo_finish
int halo_start(Ctx& c, double* xpad);      // pack + exchange on the comm stream
int halo_finish(Ctx& c, double* xpad);     // compute stream waits, unpacks
int allreduce_sum(Ctx& c, const double* in, double* out, int count);
int allreduce_max(Ctx& c, const double* in, double* out, int count);
int allreduce_prepare(Ctx& c);
// host wait for work that depends on other ranks (CG chunk polls, all-reduced norms): the RCCL
// transport polls the event and the communicator's asynchronous error against c.comm_timeout and
// aborts the communicator on either; one rank without a communicator waits plainly
int comm_wait(Ctx& c, hipEvent_t ev, const char* what);
int comm_check(Ctx& c);  // a communicator aborted earlier: fail the collective
int comm_query(Ctx& c, int* n, int* r, int* dev);  // ncclCommCount / UserRank / CuDevice (1, 0, device: none)
int group_setup(Ctx& c);  // the in-process group's events (first member on the device)
void launch_group_sum(Ctx& c, const double* const* ptrs, int nranks, int count, double* out, int op = 0);
void launch_vtu_cells(Ctx& c, const int* lo, const int* cnt, double* out);
void launch_force_layer(Ctx& c, int comp, int fa, int fixed, int a0, int na, int b0, int nb, double* out);

// ---- kernel launchers (kernels.hip)
int upload_constants(Ctx& c);
void launch_apply_bc_u(Ctx& c, double U);
void launch_strains(Ctx& c);
void launch_homogenize(Ctx& c);
void launch_residual(Ctx& c);          // b + partial sums of b.b
void launch_element_ke(Ctx& c);        // Ke of a per-GP-tangent law
int launch_plain_ke(Ctx& c);           // plain elements, kref, the other elements' Ke (exception-node build)
void launch_elastic_ke(Ctx& c);        // the elastic law's one element matrix (ke_uni)
void launch_gather_matrix(Ctx& c);
void launch_gather_matrix_sym(Ctx& c);
int build_split(Ctx& c, bool* exact);  // AIJ-split corrections from U (exact = usable)
int build_vi(Ctx& c, bool* ok);        // value-indexed AIJ (ok = at most VI_MAX distinct values)
void launch_jacobi(Ctx& c);
void launch_spmv(Ctx& c, const double* xpad, double* y, bool dot, bool gated);
void launch_update_u(Ctx& c);
int launch_cg_xfinal(Ctx& c);
void launch_cg_pupdate(Ctx& c, int part);  // 0 all owned nodes, 1 the sent (subdomain-face) nodes, 2 the rest
void launch_reduce(Ctx& c, int nvals, int nparts, double* out);
void launch_cg_init(Ctx& c);
int cg_iteration(Ctx& c, hipEvent_t spmv_start, hipEvent_t spmv_stop, bool first, bool last);
int cg_finish_init(Ctx& c);
void launch_pack(Ctx& c, const double* xpad);
void launch_unpack(Ctx& c, double* xpad);
void launch_copy_owned_to_pad(Ctx& c, const double* owned, double* pad);
void launch_copy_pad_to_owned(Ctx& c, const double* pad, double* owned);
int64_t spmv_grid_blocks(const Ctx& c);
int64_t spmv_nparts(const Ctx& c);
bool partials_fit(const Ctx& c);     // the SpMV's and the node blocks' partials fit half the buffer
bool st_wanted(const Ctx& c);        // option vi_st asks for the default-stencil SpMV   // partial sums the CG's SpMV leaves (its own grid, or the dense pass's)
int64_t node_blocks(const Ctx& c);
bool vi_staged(const Ctx& c);
int build_wdesc(Ctx& c);    // wave descriptors of the block-indexed storage (after build_vi)
bool wd_used(const Ctx& c);  // the staged SpMV reads them
int build_st(Ctx& c);       // default-stencil SpMV structures (after build_vi)
bool st_used(const Ctx& c);  // the SpMV runs k_spmv_st + k_spmv_face
bool fusep(const Ctx& c);  // the CG's p update runs inside the value-indexed SpMV
bool cg_pdb(const Ctx& c);  // the CG's p update double-buffered (x every second iteration)
int64_t cg_vec_bytes_per_node(const Ctx& c);  // the last solve's CG vector kernels, bytes per owned node and iteration
// z-marching SpMV tile of the current storage (tx, ty, planes per chunk); all 0 for gathered kernels
void spmv_tile(const Ctx& c, int* tx, int* ty, int* kc);
int dirichlet_mask_host(const Geo& g, int gi, int gj, int gk);

}  // namespace mcx

// Every extern "C" entry is a function-try-block: no C++ exception (std::bad_alloc from a host
// vector, std::system_error from the group barrier's mutex, ...) crosses the C ABI.  The handler
// stores the message for mcx_last_error and returns MCX_EXC (the PetscErrorCode contract of the
// functions the entries replace).  MCX_ENTRY is the test hook: MCX_TEST_THROW=<entry name> in the
// environment makes that entry throw std::bad_alloc at its start (tests/test_abi.py).
namespace mcx {
constexpr int MCX_EXC = 90;
int exc_return(const char* fn, const char* what);
void test_inject(const char* fn);
}  // namespace mcx
#define MCX_ENTRY() mcx::test_inject(__func__)
#define MCX_CATCH                                                                      \
  catch (const std::exception& e_) {                                                   \
    return mcx::exc_return(__func__, e_.what());                                       \
  }                                                                                    \
  catch (...) {                                                                        \
    return mcx::exc_return(__func__, "unknown exception");                             \
  }

#define MCX_HIP(call)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      mcx::set_error(std::string(#call) + ": " + hipGetErrorString(e_) + " @" +        \
                     __FILE__ + ":" + std::to_string(__LINE__));                       \
      return 10;                                                                       \
    }                                                                                  \
  } while (0)
