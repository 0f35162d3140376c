// comm.cpp — RCCL transport of the MI355X MacroC path (one communicator per context).
//
// Replaces the MPI traffic PETSc generates on the hot path: the
// DMGlobalToLocal / MatMult ghost scatter becomes one grouped ncclSend/ncclRecv per
// neighbour (each neighbour of a 2x2x2 box is one direct xGMI link), and the 1-double
// MPI_Allreduce of VecTDot/VecNorm becomes ncclAllReduce on the compute stream, so the CG
// loop never returns to the host between iterations.
#include <rccl/rccl.h>

#include <cstring>

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

int comm_init(Ctx& c, const void* id) {
  if (c.nranks <= 1) return 0;
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

int halo_exchange(Ctx& c, double* xpad) {
  if (c.nranks <= 1 || c.halo.nbr_rank.empty()) return 0;
  HaloPlan& h = c.halo;
  launch_pack(c, xpad);
  MCX_NCCL(ncclGroupStart());
  for (size_t q = 0; q < h.nbr_rank.size(); q++) {
    MCX_NCCL(ncclSend(h.d_sendbuf + 3 * h.send_off[q], 3 * h.send_cnt[q], ncclDouble, h.nbr_rank[q],
                      (ncclComm_t)c.comm, c.stream));
    MCX_NCCL(ncclRecv(h.d_recvbuf + 3 * h.recv_off[q], 3 * h.recv_cnt[q], ncclDouble, h.nbr_rank[q],
                      (ncclComm_t)c.comm, c.stream));
  }
  MCX_NCCL(ncclGroupEnd());
  launch_unpack(c, xpad);
  return 0;
}

int allreduce_sum(Ctx& c, const double* in, double* out, int count) {
  if (c.nranks <= 1) {
    if (in != out) MCX_HIP(hipMemcpyAsync(out, in, sizeof(double) * count, hipMemcpyDeviceToDevice, c.stream));
    return 0;
  }
  MCX_NCCL(ncclAllReduce(in, out, count, ncclDouble, ncclSum, (ncclComm_t)c.comm, c.stream));
  return 0;
}

}  // namespace mcx

extern "C" int mcx_comm_unique_id(void* id) {
  ncclUniqueId uid;
  ncclResult_t r = ncclGetUniqueId(&uid);
  if (r != ncclSuccess) {
    mcx::set_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    return 20;
  }
  std::memcpy(id, &uid, sizeof(uid));
  return 0;
}
