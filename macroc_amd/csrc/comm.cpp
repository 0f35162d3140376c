// comm.cpp — RCCL transport of the MI355X MacroC path (one communicator per context).
//
// Replaces the MPI traffic PETSc generates on the hot path: the
// DMGlobalToLocal / MatMult ghost scatter becomes one grouped ncclSend/ncclRecv per
// neighbour (each neighbour of a 2x2x2 box is one direct xGMI link) on a comm stream that
// overlaps interior work (halo_start / halo_finish), and the 1-double MPI_Allreduce of
// VecTDot/VecNorm becomes ncclAllReduce on the compute stream, so the CG loop never returns to
// the host between iterations.  Collective order is identical on every rank: each halo is
// finished (waited for by the compute stream) before the next all-reduce is enqueued.
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "mcx_internal.h"

namespace mcx {

#define MCX_NCCL(call)                                                                          \
  do {                                                                                          \
    ncclResult_t r_ = (call);                                                                   \
    if (r_ != ncclSuccess) {                                                                    \
      set_error(std::string(#call) + ": " + ncclGetErrorString(r_));                            \
      return 20;                                                                                \
    }                                                                                           \
  } while (0)

// One rank with an id given: an RCCL communicator of one, so the all-reduces take the multi-rank
// path (k_reduce partial sums, ncclAllReduce, k_cg_logic) — the RCCL transport on one GPU.
int comm_init(Ctx& c, const void* id) {
  if (c.lg || (c.nranks <= 1 && !id)) return 0;
  if (!id) {
    set_error("nranks > 1 needs a communicator id from mcx_comm_unique_id");
    return 21;
  }
  ncclUniqueId uid;
  static_assert(sizeof(ncclUniqueId) == MCX_COMM_ID_BYTES, "ncclUniqueId size");
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t comm;
  MCX_NCCL(ncclCommInitRank(&comm, c.nranks, uid, c.rank));
  c.comm = comm;
  return 0;
}

void comm_destroy(Ctx& c) {
  if (c.comm) {
    ncclCommDestroy((ncclComm_t)c.comm);
    c.comm = nullptr;
  }
}

// the communicator as RCCL reports it (ncclCommCount / ncclCommUserRank / ncclCommCuDevice):
// what the ranks actually joined, not what the caller asked for; no communicator: 1, 0, c.device
int comm_query(Ctx& c, int* n, int* r, int* dev) {
  *n = 1, *r = 0, *dev = c.device;
  if (int rc = comm_check(c)) return rc;
  if (!c.comm) return 0;
  MCX_NCCL(ncclCommCount((ncclComm_t)c.comm, n));
  MCX_NCCL(ncclCommUserRank((ncclComm_t)c.comm, r));
  MCX_NCCL(ncclCommCuDevice((ncclComm_t)c.comm, dev));
  return 0;
}

double comm_timeout_default() {
  const char* e = std::getenv("MCX_COMM_TIMEOUT");
  const double v = e ? std::atof(e) : 0.;
  return v > 0. ? v : 300.;
}

static const char* bar_name(int tag) {
  switch (tag) {
    case BAR_INIT: return "mcx_init_local";
    case BAR_HALO_PACKED: return "halo exchange (packed)";
    case BAR_HALO_DONE: return "halo exchange (copied)";
    case BAR_RED_IN: return "all-reduce (partials)";
    case BAR_RED_SUM: return "all-reduce (summed)";
    case BAR_FINALIZE: return "mcx_finalize";
    default: return "mcx_local_group_barrier";
  }
}

// The in-process group's host barrier.  Members must cross the same sequence of collectives; a
// crossing carries the collective's tag, and a member arriving with another tag than the first
// arrival of the open generation breaks the group (the RCCL analogue is a mismatched collective,
// which hangs).  A generation still open after timeout_s breaks it too (a member that stopped,
// e.g. after an error of its own).  A broken group fails every later crossing at once, so no
// member proceeds to read a peer's buffers on an exchange the peer is not part of.  timeout_s <= 0:
// the group's own deadline (MCX_COMM_TIMEOUT at creation); the collective entry points pass their
// context's comm_timeout option.
int group_barrier(LocalGroup* g, int rank, int tag, double timeout_s) {
  if (timeout_s <= 0.) timeout_s = g->timeout_s;
  auto* m = static_cast<std::mutex*>(g->mtx);
  auto* cv = static_cast<std::condition_variable*>(g->cv);
  std::unique_lock<std::mutex> lk(*m);
  auto fail = [&]() {
    set_error("in-process group: " + g->why);
    return 23;
  };
  if (g->broken) return fail();
  if (g->count == 0) {
    g->cur_tag = tag;
    g->cur_rank = rank;
  } else if (g->cur_tag != tag) {
    g->broken = true;
    g->why = "mismatched collectives: rank " + std::to_string(rank) + " entered " + bar_name(tag) + ", rank " +
             std::to_string(g->cur_rank) + " " + bar_name(g->cur_tag);
    cv->notify_all();
    return fail();
  }
  const int gen = g->generation;
  if (++g->count == g->nranks) {
    g->count = 0;
    g->generation++;
    cv->notify_all();
    return 0;
  }
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  if (!cv->wait_until(lk, deadline, [&] { return g->generation != gen || g->broken; })) {
    g->broken = true;
    g->why = "rank " + std::to_string(rank) + " waited " + std::to_string((int)timeout_s) + " s in " +
             bar_name(tag) + ": " + std::to_string(g->count) + " of " + std::to_string(g->nranks) +
             " members arrived (a member stopped or skipped the collective)";
    cv->notify_all();
    return fail();
  }
  if (g->generation == gen) return fail();  // broken while waiting
  return 0;
}

// events and the partial-sum pointer table of the group (first mcx_init_local; the group itself
// is host-only, so it can be created and its barrier exercised without a GPU)
static int group_device_setup(LocalGroup* g) {
  std::lock_guard<std::mutex> lk(*static_cast<std::mutex*>(g->mtx));
  if (g->dev_ready) return 0;
  for (auto* v : {&g->ev_packed, &g->ev_halo_done, &g->ev_red, &g->ev_sum}) {
    v->assign(g->nranks, nullptr);
    for (auto& e : *v) MCX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  MCX_HIP(hipMalloc(&g->d_red_ptrs, sizeof(double*) * g->nranks));
  g->dev_ready = true;
  return 0;
}
int group_setup(Ctx& c) { return group_device_setup(c.lg); }

int comm_check(Ctx& c) {
  if (!c.comm_broken) return 0;
  set_error("rank " + std::to_string(c.rank) + ": communicator aborted earlier: " + c.comm_why);
  return 24;
}

static void comm_abort(Ctx& c, const std::string& why) {
  c.comm_broken = true;
  c.comm_why = why;
  if (c.comm) {
    (void)ncclCommAbort((ncclComm_t)c.comm);  // RCCL kernels waiting on peers return
    c.comm = nullptr;
  }
  set_error("rank " + std::to_string(c.rank) + ": " + why);
}

int comm_wait(Ctx& c, hipEvent_t ev, const char* what) {
  if (int rc = comm_check(c)) return rc;
  if (c.nranks <= 1 && !c.comm) {
    MCX_HIP(hipEventSynchronize(ev));
    return 0;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (int spin = 0;; spin++) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return 0;
    if (e != hipErrorNotReady) {
      comm_abort(c, std::string(what) + ": hipEventQuery: " + hipGetErrorString(e));
      return 10;
    }
    if (c.comm) {
      ncclResult_t ar = ncclSuccess;
      const ncclResult_t r = ncclCommGetAsyncError((ncclComm_t)c.comm, &ar);
      if (r != ncclSuccess || (ar != ncclSuccess && ar != ncclInProgress)) {
        comm_abort(c, std::string(what) + ": RCCL asynchronous error: " +
                          ncclGetErrorString(r != ncclSuccess ? r : ar) + " (communicator aborted)");
        return 25;
      }
    }
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (dt > c.comm_timeout) {
      comm_abort(c, std::string(what) + " not complete after " + std::to_string((int)c.comm_timeout) +
                        " s (a peer rank stopped, or the ranks issued different collectives); communicator aborted");
      return 24;
    }
    if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

// Forward halo in two halves so interior work can run while the bytes move:
//   halo_start:  pack the sent nodes (compute stream), then the exchange on the comm stream
//                (grouped ncclSend/ncclRecv, or device copies from the neighbours' send buffers
//                for the in-process transport);
//   halo_finish: the compute stream waits for the exchange and unpacks into the ghost layer.
// halo_exchange = start + finish.  Anything enqueued on the compute stream in between overlaps
// the exchange (cg_iteration: the interior p update).
int halo_start(Ctx& c, double* xpad) {
  if (c.nranks <= 1 || c.halo.nbr_rank.empty()) return 0;
  if (int rc = comm_check(c)) return rc;
  HaloPlan& h = c.halo;
  if (c.lg) {
    LocalGroup* g = c.lg;
    // neighbours finished reading my previous send buffer
    for (int q : h.nbr_rank) MCX_HIP(hipStreamWaitEvent(c.stream, g->ev_halo_done[q], 0));
    launch_pack(c, xpad);
    MCX_HIP(hipEventRecord(g->ev_packed[c.rank], c.stream));
    // the copies below overwrite my receive buffer: order them after my compute stream's last
    // reader of it (the previous halo's k_unpack), as the RCCL branch does
    MCX_HIP(hipStreamWaitEvent(c.comm_stream, g->ev_packed[c.rank], 0));
    if (int rc = group_barrier(g, c.rank, BAR_HALO_PACKED, c.comm_timeout)) return rc;
    for (size_t t = 0; t < h.nbr_rank.size(); t++) {
      const Ctx& q = *g->members[h.nbr_rank[t]];
      size_t idx = 0;
      while (idx < q.halo.nbr_rank.size() && q.halo.nbr_rank[idx] != c.rank) idx++;
      if (idx == q.halo.nbr_rank.size() || q.halo.send_cnt[idx] != h.recv_cnt[t]) {
        set_error("local halo: inconsistent neighbour plans");
        return 22;
      }
      MCX_HIP(hipStreamWaitEvent(c.comm_stream, g->ev_packed[h.nbr_rank[t]], 0));
      MCX_HIP(hipMemcpyAsync(h.d_recvbuf + 3 * h.recv_off[t], q.halo.d_sendbuf + 3 * q.halo.send_off[idx],
                             sizeof(double) * 3 * h.recv_cnt[t], hipMemcpyDeviceToDevice, c.comm_stream));
    }
    MCX_HIP(hipEventRecord(g->ev_halo_done[c.rank], c.comm_stream));
    MCX_HIP(hipEventRecord(c.ev_comm, c.comm_stream));
    // every member recorded ev_halo_done before anyone waits on it again
    if (int rc = group_barrier(g, c.rank, BAR_HALO_DONE, c.comm_timeout)) return rc;
    return 0;
  }
  launch_pack(c, xpad);
  MCX_HIP(hipEventRecord(c.ev_pack, c.stream));
  MCX_HIP(hipStreamWaitEvent(c.comm_stream, c.ev_pack, 0));
  MCX_NCCL(ncclGroupStart());
  for (size_t q = 0; q < h.nbr_rank.size(); q++) {
    MCX_NCCL(ncclSend(h.d_sendbuf + 3 * h.send_off[q], 3 * h.send_cnt[q], ncclDouble, h.nbr_rank[q],
                      (ncclComm_t)c.comm, c.comm_stream));
    MCX_NCCL(ncclRecv(h.d_recvbuf + 3 * h.recv_off[q], 3 * h.recv_cnt[q], ncclDouble, h.nbr_rank[q],
                      (ncclComm_t)c.comm, c.comm_stream));
  }
  MCX_NCCL(ncclGroupEnd());
  MCX_HIP(hipEventRecord(c.ev_comm, c.comm_stream));
  return 0;
}

int halo_finish(Ctx& c, double* xpad) {
  if (c.nranks <= 1 || c.halo.nbr_rank.empty()) return 0;
  MCX_HIP(hipStreamWaitEvent(c.stream, c.ev_comm, 0));
  launch_unpack(c, xpad);
  return 0;
}

int halo_exchange(Ctx& c, double* xpad) {
  int rc = halo_start(c, xpad);
  return rc ? rc : halo_finish(c, xpad);
}

static int allreduce_op(Ctx& c, const double* in, double* out, int count, int op) {
  if (int rc = comm_check(c)) return rc;
  if (c.nranks <= 1 && !c.comm) {
    if (in != out) MCX_HIP(hipMemcpyAsync(out, in, sizeof(double) * count, hipMemcpyDeviceToDevice, c.stream));
    return 0;
  }
  if (c.lg) {
    LocalGroup* g = c.lg;
    MCX_HIP(hipEventRecord(g->ev_red[c.rank], c.stream));
    if (int rc = group_barrier(g, c.rank, BAR_RED_IN, c.comm_timeout)) return rc;
    for (int q = 0; q < g->nranks; q++) MCX_HIP(hipStreamWaitEvent(c.stream, g->ev_red[q], 0));
    launch_group_sum(c, (const double* const*)g->d_red_ptrs, g->nranks, count, out, op);
    MCX_HIP(hipEventRecord(g->ev_sum[c.rank], c.stream));
    if (int rc = group_barrier(g, c.rank, BAR_RED_SUM, c.comm_timeout)) return rc;
    return 0;
  }
  MCX_NCCL(ncclAllReduce(in, out, count, ncclDouble, op ? ncclMax : ncclSum, (ncclComm_t)c.comm, c.stream));
  return 0;
}

// in must be red_loc (the in-process transport sums every member's red_loc)
int allreduce_sum(Ctx& c, const double* in, double* out, int count) { return allreduce_op(c, in, out, count, 0); }
int allreduce_max(Ctx& c, const double* in, double* out, int count) { return allreduce_op(c, in, out, count, 1); }

// before overwriting red_loc: every member has summed the previous partials
int allreduce_prepare(Ctx& c) {
  if (!c.lg) return 0;
  for (int q = 0; q < c.lg->nranks; q++) MCX_HIP(hipStreamWaitEvent(c.stream, c.lg->ev_sum[q], 0));
  return 0;
}

}  // namespace mcx

extern "C" int mcx_local_group_create(int nranks, int device, void** group) try {
  MCX_ENTRY();
  using namespace mcx;
  if (nranks < 1 || !group) {
    set_error("mcx_local_group_create: bad arguments");
    return 1;
  }
  auto* g = new LocalGroup();
  g->nranks = nranks;
  g->device = device;
  g->members.assign(nranks, nullptr);
  g->mtx = new std::mutex();
  g->cv = new std::condition_variable();
  g->timeout_s = comm_timeout_default();
  *group = g;
  return 0;
} MCX_CATCH

extern "C" int mcx_local_group_destroy(void* group) try {
  MCX_ENTRY();
  using namespace mcx;
  auto* g = static_cast<LocalGroup*>(group);
  if (!g) return 0;
  if (g->dev_ready) {
    (void)hipSetDevice(g->device);
    for (auto* v : {&g->ev_packed, &g->ev_halo_done, &g->ev_red, &g->ev_sum})
      for (auto& e : *v)
        if (e) (void)hipEventDestroy(e);
    if (g->d_red_ptrs) (void)hipFree(g->d_red_ptrs);
  }
  delete static_cast<std::mutex*>(g->mtx);
  delete static_cast<std::condition_variable*>(g->cv);
  delete g;
  return 0;
} MCX_CATCH

extern "C" int mcx_local_group_barrier(void* group, int rank) try {
  MCX_ENTRY();
  using namespace mcx;
  auto* g = static_cast<LocalGroup*>(group);
  if (!g || rank < 0 || rank >= g->nranks) {
    set_error("mcx_local_group_barrier: bad arguments");
    return 1;
  }
  return group_barrier(g, rank, BAR_USER, 0.);
} MCX_CATCH

extern "C" int mcx_comm_unique_id(void* id) try {
  MCX_ENTRY();
  ncclUniqueId uid;
  ncclResult_t r = ncclGetUniqueId(&uid);
  if (r != ncclSuccess) {
    mcx::set_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    return 20;
  }
  std::memcpy(id, &uid, sizeof(uid));
  return 0;
} MCX_CATCH
