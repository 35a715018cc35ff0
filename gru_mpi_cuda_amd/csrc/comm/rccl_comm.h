// RCCL communicator over xGMI: one per process/GPU.
//
// Replaces the reference's MPI layer (MPI_Comm_rank/size, MPI_Barrier, MPI_Scatter,
// MPI_Gather on host buffers: /root/reference/namegensf.cu:360-366,615,636,889) with
// device-buffer collectives on HIP streams.  Bootstrap: rank 0 makes an ncclUniqueId, the
// Python side ships its 128 bytes through the torch.distributed TCP store, every rank calls
// ncclCommInitRank.  Collectives issued on a stream that is being captured become graph
// nodes, so gradient all-reduce can live inside the training step's hipGraph.
#pragma once
#include <atomic>
#include <string>
#include <hip/hip_runtime.h>

namespace gk {

class RcclComm {
 public:
  static std::string unique_id();
  RcclComm(const std::string& uid, int rank, int world);
  ~RcclComm();
  void allreduce_avg_f32(float* p, long n, hipStream_t s);
  void allreduce_sum_f32(float* p, long n, hipStream_t s);
  void allreduce_max_u32(unsigned* p, long n, hipStream_t s);
  // the step's last gradient collective grouped (one launch) with a max-reduction of the step error
  // word: every rank then sees a spin timeout of ANY rank and skips the update together
  void allreduce_avg_f32_err(float* p, long n, unsigned* err, hipStream_t s);
  void broadcast_f32(float* p, long n, int root, hipStream_t s);
  void allgather_u8(const unsigned char* send, unsigned char* recv, long n, hipStream_t s);
  // sharded optimiser (ZeRO-1 style): recv[n] = mean over ranks of send[rank*n .. rank*n+n)
  void reduce_scatter_avg_f32(const float* send, float* recv, long n, hipStream_t s);
  // recv[world*n] = concat over ranks of send[n]; bf16 payload moved as 16-bit words
  void allgather_u16(const unsigned short* send, unsigned short* recv, long n, hipStream_t s);
  void allgather_f32(const float* send, float* recv, long n, hipStream_t s);
  // sharded optimiser with bf16 working copies: the owned bf16 slices all-gathered and, in the same
  // group launch, a 32-bit integer sum over `pack` (each rank contributes its own entries, zeros
  // elsewhere: the sum is an exact bitwise exchange of the fp32 values kernels read directly)
  void allgather_u16_sum_u32(const unsigned short* send, unsigned short* recv, long n, unsigned* pack, long np,
                             hipStream_t s);
  // MPI_Scatterv / MPI_Gatherv as grouped point-to-point transfers (one group launch): rank r's
  // slice is [displ[r], displ[r] + count[r]) elements of the root's buffer.  Scatter: the root sends
  // every other rank its slice into that rank's recv (the root's own slice stays where it is);
  // gather: every other rank sends its send[0 .. count[rank]) into the root's recv at displ[r].
  void scatterv_f32(const float* send, const long* count, const long* displ, float* recv, int root, hipStream_t s);
  void gatherv_u8(const unsigned char* send, const long* count, const long* displ, unsigned char* recv, int root,
                  hipStream_t s);
  int count() const;                  // ncclCommCount: ranks the communicator really has
  // watchdog hook: raises if the communicator reported an asynchronous error
  void check_async_error();
  void abort();                       // thread-safe (the watchdog calls it)
  bool aborted() const { return comm_.load() == nullptr; }
  int rank() const { return rank_; }
  int world() const { return world_; }

 private:
  std::atomic<void*> comm_{nullptr};   // ncclComm_t; null once aborted
  void* live() const;
  int rank_ = 0, world_ = 1;
};

}  // namespace gk
