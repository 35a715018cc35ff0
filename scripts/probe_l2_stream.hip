// Per-CU streaming probe for the layer-wavefront questions.
//
// A persistent grid of 256 workgroups x 512 threads (one per CU, forced by a 96 KiB LDS request)
// runs `steps` iterations.  Each iteration a workgroup reads three kinds of bytes and then joins a
// grid-wide hand-off, i.e. the data movement of one persistent-recurrence step with no math:
//   * local  : a region shared by the 32 workgroups of its XCD, the same every step (an XCD-local
//              exchange: after the first reader it is served by the XCD's L2);
//   * remote : a region shared by the workgroups of its XCD but new every step, rotating through
//              `steps` regions (> L2), so each step's first touch comes from the memory side -- the
//              cross-XCD hand-off of a row block spanning XCDs, or another layer's exchange;
//   * slice  : a per-workgroup slice, the same every step: workgroup i of every XCD reads slice i,
//              so each XCD's working set is 32 slices -- streamed weight K-slices (row blocks
//              replicated over XCDs, as in a wavefront that cannot keep its weights resident).
// Two roles: workgroups on XCDs 0-3 use (local, remote, slice) set A, XCDs 4-7 set B, so one launch
// can model a per-layer-workgroup wavefront.  The hand-off is per-producer epoch flags: every workgroup
// waits for its XCD's 32 workgroups (and the partner XCD's when it reads remote bytes), a bounded spin.
// Loads are b128 into registers folded with XOR (all issued before the fold), vmcnt(0) before the
// hand-off.  Output: one JSON line per configuration, us per step (min of 3 launches).
//
//   hipcc -O3 --offload-arch=gfx950 scripts/probe_l2_stream.hip -o scripts/probe_l2_stream
//   ./scripts/probe_l2_stream [steps]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

struct Role { unsigned local_v4, remote_v4, slice_v4; };   // 16-byte vectors per workgroup per step
struct Args {
  const u32x4* local_src;    // [8 XCD][max local]
  const u32x4* remote_src;   // [steps][8 XCD][max remote]
  const u32x4* slice_src;    // [32][max slice]
  unsigned local_max, remote_max, slice_max;
  Role role[2];
  unsigned* flags;   // [256][16]
  unsigned* err;
  u32x4* sink;
  int steps;
};

template <int UNR>
__device__ inline u32x4 stream(const u32x4* p, unsigned n, unsigned tid) {
  u32x4 acc = {0u, 0u, 0u, 0u};
  unsigned i = tid;
  for (; i + (UNR - 1) * 512 < n; i += UNR * 512) {
    u32x4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) v[u] = p[i + u * 512];
#pragma unroll
    for (int u = 0; u < UNR; ++u) acc ^= v[u];
  }
  for (; i < n; i += 512) acc ^= p[i];
  return acc;
}

__global__ void __launch_bounds__(512, 1) probe_kernel(Args a) {
  extern __shared__ u32x4 lds[];
  const unsigned tid = threadIdx.x, b = blockIdx.x, xcd = b % 8, wi = b / 8;
  const Role r = a.role[xcd < 4 ? 0 : 1];
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (int s = 0; s < a.steps; ++s) {
    acc ^= stream<8>(a.local_src + (size_t)xcd * a.local_max, r.local_v4, tid);
    acc ^= stream<8>(a.remote_src + ((size_t)s * 8 + xcd) * a.remote_max, r.remote_v4, tid);
    acc ^= stream<8>(a.slice_src + (size_t)wi * a.slice_max, r.slice_v4, tid);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < 64) {
      // per-producer epoch flags (own 64-B line each), as in the recurrences: lanes 0-31 wait for
      // the 32 workgroups of this XCD, lanes 32-63 for the partner XCD's when remote bytes flow
      // relaxed (sc1) stores and polls after the vmcnt(0) drain above, as the recurrences publish:
      // release / acquire atomics here would add an L2 writeback and invalidate to every step
      if (tid == 0) __hip_atomic_store(a.flags + (size_t)b * 16, (unsigned)(s + 1), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
      const unsigned src = (tid < 32 ? xcd : (r.remote_v4 ? (xcd ^ 4u) : xcd)) + 8u * (tid & 31u);
      unsigned spins = 0;
      while (!__all(__hip_atomic_load(a.flags + (size_t)src * 16, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)(s + 1))) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 22)) {   // bounded: a non-co-resident grid drains instead of hanging
          if (tid == 0) __hip_atomic_fetch_or(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
  }
  lds[tid] = acc;   // keep the loads live
  __syncthreads();
  a.sink[(size_t)b * 512 + tid] = lds[(tid + 1) & 511];
}

int main(int argc, char** argv) {
  const int steps = argc > 1 ? std::atoi(argv[1]) : 64;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  if (cus != 256) { std::fprintf(stderr, "expected 256 CUs, got %d\n", cus); return 2; }
  const size_t lds_bytes = 96 * 1024;
  CK(hipFuncSetAttribute((const void*)probe_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes));
  int nb = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, probe_kernel, 512, lds_bytes));
  if (nb != 1) { std::fprintf(stderr, "occupancy %d != 1\n", nb); return 2; }

  const unsigned KB = 1024 / 16;   // 16-byte vectors per KiB
  const unsigned local_max = 384 * KB, remote_max = 192 * KB, slice_max = 576 * KB;
  u32x4 *local_src, *remote_src, *slice_src, *sink;
  unsigned *flags, *err;
  CK(hipMalloc(&local_src, (size_t)8 * local_max * 16));
  CK(hipMalloc(&remote_src, (size_t)steps * 8 * remote_max * 16));
  CK(hipMalloc(&slice_src, (size_t)32 * slice_max * 16));
  CK(hipMalloc(&sink, (size_t)256 * 512 * 16));
  CK(hipMalloc(&flags, 256 * 16 * 4));
  CK(hipMalloc(&err, 4));
  CK(hipMemset(local_src, 1, (size_t)8 * local_max * 16));
  CK(hipMemset(remote_src, 2, (size_t)steps * 8 * remote_max * 16));
  CK(hipMemset(slice_src, 3, (size_t)32 * slice_max * 16));
  CK(hipMemset(err, 0, 4));

  struct Cfg { const char* name; Role A, B; };
  auto R = [&](unsigned l, unsigned m, unsigned s) { return Role{l * KB, m * KB, s * KB}; };
  const Cfg cfgs[] = {
    {"hand-off only", R(0, 0, 0), R(0, 0, 0)},
    {"local 48K", R(48, 0, 0), R(48, 0, 0)},
    {"local 96K (bwd16 exchange)", R(96, 0, 0), R(96, 0, 0)},
    {"local 192K (32-row exchange)", R(192, 0, 0), R(192, 0, 0)},
    {"local 384K", R(384, 0, 0), R(384, 0, 0)},
    {"remote 96K", R(0, 96, 0), R(0, 96, 0)},
    {"remote 192K (32-row block over 2 XCDs)", R(0, 192, 0), R(0, 192, 0)},
    {"slice 96K (3 MB per XCD)", R(0, 0, 96), R(0, 0, 96)},
    {"slice 192K (6 MB per XCD)", R(0, 0, 192), R(0, 0, 192)},
    {"slice 288K (fwd seq2 weights, streamed)", R(0, 0, 288), R(0, 0, 288)},
    {"slice 576K (16-row fwd wavefront weights)", R(0, 0, 576), R(0, 0, 576)},
    {"fwd16 wave: local 64K + slice 576K", R(64, 0, 576), R(64, 0, 576)},
    {"bwd wave per-layer WGs: L1 local 192K | L0 local 192K + remote 192K + slice 192K",
     R(192, 0, 0), R(192, 192, 192)},
    {"bwd wave same WG: local 96K x2 + remote 0 + slice 192K (W_ih1 streamed)", R(192, 0, 192), R(192, 0, 192)},
  };
  for (const Cfg& c : cfgs) {
    Args a{local_src, remote_src, slice_src, local_max, remote_max, slice_max, {c.A, c.B},
           flags, err, sink, steps};
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipMemset(flags, 0, 256 * 16 * 4));
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(probe_kernel, dim3(256), dim3(512), lds_bytes, 0, a);
      CK(hipGetLastError());
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep > 0 && ms < best) best = ms;   // rep 0 warms up
      CK(hipEventDestroy(e0)); CK(hipEventDestroy(e1));
    }
    unsigned herr = 0;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    const double us = best * 1e3 / steps;
    const double kbA = (c.A.local_v4 + c.A.remote_v4 + c.A.slice_v4) / (double)KB;
    const double kbB = (c.B.local_v4 + c.B.remote_v4 + c.B.slice_v4) / (double)KB;
    std::printf("{\"config\": \"%s\", \"steps\": %d, \"us_per_step\": %.3f, \"kb_per_cu_step\": [%.0f, %.0f], "
                "\"spin_error\": %u}\n", c.name, steps, us, kbA, kbB, herr);
    std::fflush(stdout);
    if (herr) return 3;
  }
  return 0;
}
