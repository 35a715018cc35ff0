#include "rccl_comm.h"

#include <rccl/rccl.h>
#include <stdexcept>
#include <cstring>
#include "../runtime/runtime.h"

namespace gk {

#define RCCL_CHECK(x)                                                                          \
  do {                                                                                         \
    ncclResult_t _r = (x);                                                                     \
    if (_r != ncclSuccess)                                                                     \
      throw std::runtime_error("[rank " + std::to_string(global_rank()) + "] RCCL error '" +   \
                               ncclGetErrorString(_r) + "' at " + __FILE__ + ":" +             \
                               std::to_string(__LINE__) + ": " #x);                            \
  } while (0)

static ncclComm_t C(void* p) { return reinterpret_cast<ncclComm_t>(p); }

std::string RcclComm::unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

RcclComm::RcclComm(const std::string& uid, int rank, int world) : rank_(rank), world_(world) {
  if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::runtime_error("RcclComm: bad unique id size");
  ncclUniqueId id;
  std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c;
  RCCL_CHECK(ncclCommInitRank(&c, world, id, rank));
  comm_ = c;
}

RcclComm::~RcclComm() {
  if (void* c = comm_.exchange(nullptr)) (void)ncclCommDestroy(C(c));
}

void* RcclComm::live() const {
  void* c = comm_.load();
  if (!c) throw std::runtime_error("[rank " + std::to_string(rank_) + "] RCCL communicator was aborted");
  return c;
}

void RcclComm::allreduce_avg_f32(float* p, long n, hipStream_t s) {
  RCCL_CHECK(ncclAllReduce(p, p, (size_t)n, ncclFloat32, ncclAvg, C(live()), s));
}
void RcclComm::allreduce_sum_f32(float* p, long n, hipStream_t s) {
  RCCL_CHECK(ncclAllReduce(p, p, (size_t)n, ncclFloat32, ncclSum, C(live()), s));
}
void RcclComm::allreduce_max_u32(unsigned* p, long n, hipStream_t s) {
  RCCL_CHECK(ncclAllReduce(p, p, (size_t)n, ncclUint32, ncclMax, C(live()), s));
}
void RcclComm::allreduce_avg_f32_err(float* p, long n, unsigned* err, hipStream_t s) {
  RCCL_CHECK(ncclGroupStart());
  if (n > 0) RCCL_CHECK(ncclAllReduce(p, p, (size_t)n, ncclFloat32, ncclAvg, C(live()), s));
  RCCL_CHECK(ncclAllReduce(err, err, 1, ncclUint32, ncclMax, C(live()), s));
  RCCL_CHECK(ncclGroupEnd());
}
void RcclComm::broadcast_f32(float* p, long n, int root, hipStream_t s) {
  RCCL_CHECK(ncclBroadcast(p, p, (size_t)n, ncclFloat32, root, C(live()), s));
}
void RcclComm::allgather_u8(const unsigned char* send, unsigned char* recv, long n, hipStream_t s) {
  RCCL_CHECK(ncclAllGather(send, recv, (size_t)n, ncclUint8, C(live()), s));
}
void RcclComm::reduce_scatter_avg_f32(const float* send, float* recv, long n, hipStream_t s) {
  RCCL_CHECK(ncclReduceScatter(send, recv, (size_t)n, ncclFloat32, ncclAvg, C(live()), s));
}
void RcclComm::allgather_u16(const unsigned short* send, unsigned short* recv, long n, hipStream_t s) {
  RCCL_CHECK(ncclAllGather(send, recv, (size_t)n, ncclBfloat16, C(live()), s));
}
void RcclComm::allgather_u16_sum_u32(const unsigned short* send, unsigned short* recv, long n, unsigned* pack,
                                     long np, hipStream_t s) {
  RCCL_CHECK(ncclGroupStart());
  if (n > 0) RCCL_CHECK(ncclAllGather(send, recv, (size_t)n, ncclBfloat16, C(live()), s));
  if (np > 0) RCCL_CHECK(ncclAllReduce(pack, pack, (size_t)np, ncclUint32, ncclSum, C(live()), s));
  RCCL_CHECK(ncclGroupEnd());
}
void RcclComm::allgather_f32(const float* send, float* recv, long n, hipStream_t s) {
  RCCL_CHECK(ncclAllGather(send, recv, (size_t)n, ncclFloat32, C(live()), s));
}
void RcclComm::scatterv_f32(const float* send, const long* count, const long* displ, float* recv, int root,
                            hipStream_t s) {
  ncclComm_t c = C(live());
  RCCL_CHECK(ncclGroupStart());
  if (rank_ == root) {
    for (int r = 0; r < world_; ++r)
      if (r != root && count[r] > 0) RCCL_CHECK(ncclSend(send + displ[r], (size_t)count[r], ncclFloat32, r, c, s));
  } else if (count[rank_] > 0) {
    RCCL_CHECK(ncclRecv(recv, (size_t)count[rank_], ncclFloat32, root, c, s));
  }
  RCCL_CHECK(ncclGroupEnd());
}
void RcclComm::gatherv_u8(const unsigned char* send, const long* count, const long* displ, unsigned char* recv,
                          int root, hipStream_t s) {
  ncclComm_t c = C(live());
  RCCL_CHECK(ncclGroupStart());
  if (rank_ == root) {
    for (int r = 0; r < world_; ++r)
      if (r != root && count[r] > 0) RCCL_CHECK(ncclRecv(recv + displ[r], (size_t)count[r], ncclUint8, r, c, s));
  } else if (count[rank_] > 0) {
    RCCL_CHECK(ncclSend(send, (size_t)count[rank_], ncclUint8, root, c, s));
  }
  RCCL_CHECK(ncclGroupEnd());
}
int RcclComm::count() const {
  int n = 0;
  RCCL_CHECK(ncclCommCount(C(live()), &n));
  return n;
}
void RcclComm::check_async_error() {
  ncclResult_t r = ncclSuccess;
  RCCL_CHECK(ncclCommGetAsyncError(C(live()), &r));
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error("[rank " + std::to_string(rank_) + "] RCCL async error: " + ncclGetErrorString(r));
}
void RcclComm::abort() {
  if (void* c = comm_.exchange(nullptr)) (void)ncclCommAbort(C(c));
}

}  // namespace gk
