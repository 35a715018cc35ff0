// Memory-bound helpers: split-K slab reduction, bf16 cast / transpose of the fp32 master
// weights, column sums, fused Adam/SGD, gradient-norm clipping and deterministic scalar
// reductions.  All vectorised 16 B per lane (cdna_hip_programming.md Guideline 13) and free
// of float atomics, so a training step is bitwise reproducible run to run.
#include <stdexcept>
#include <vector>
#include "kernels.h"
#include "common.h"
#include "optim_dev.h"
#include "../runtime/runtime.h"

namespace gk {

static int nblocks(long n, int per_block, int cap = 4096) {
  long b = (n + per_block - 1) / per_block;
  if (b < 1) b = 1;
  return (int)(b > cap ? cap : b);
}

__global__ void reduce_slabs_kernel(const float* __restrict__ src, int splits, long n, float* __restrict__ dst) {
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 acc = reinterpret_cast<const float4*>(src)[i];
    for (int s = 1; s < splits; ++s) {
      const float4 v = reinterpret_cast<const float4*>(src + (size_t)s * n)[i];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    reinterpret_cast<float4*>(dst)[i] = acc;
  }
  // tail
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < splits; ++s) acc += src[(size_t)s * n + i];
    dst[i] = acc;
  }
}
void reduce_slabs(const float* src, int splits, long n, float* dst, hipStream_t s) {
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3(nblocks(n / 4 + 1, 256, 2048)), dim3(256), 0, s, src, splits, n, dst);
}

__global__ void cast_bf16_kernel(const float* __restrict__ in, long n, u16* __restrict__ out) {
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(in)[i];
    ushort4 o;
    o.x = f2bf(v.x); o.y = f2bf(v.y); o.z = f2bf(v.z); o.w = f2bf(v.w);
    reinterpret_cast<ushort4*>(out)[i] = o;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = f2bf(in[i]);
}
void cast_bf16(const float* in, long n, u16* out, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(nblocks(n / 4 + 1, 256, 2048)), dim3(256), 0, s, in, n, out);
}

// [R][C] fp32 -> [C][R] bf16 through a padded 64x64 LDS tile
__global__ void transpose_bf16_kernel(const float* __restrict__ in, int R, int C, u16* __restrict__ out) {
  __shared__ float tile[64][65];
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 256 threads: 4 rows per pass
  for (int y = ty; y < 64; y += 4) {
    const int r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < R && c < C) ? in[(size_t)r * C + c] : 0.f;
  }
  __syncthreads();
  for (int y = ty; y < 64; y += 4) {
    const int c = c0 + y, r = r0 + tx;
    if (c < C && r < R) out[(size_t)c * R + r] = f2bf(tile[tx][y]);
  }
}
void transpose_bf16(const float* in, int R, int C, u16* outT, hipStream_t s) {
  dim3 grid((C + 63) / 64, (R + 63) / 64);
  hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, s, in, R, C, outT);
}

// [R][C] -> [C]: 64 columns x 4 row groups per block, independent loads, LDS combine (fixed order)
__global__ void colsum_kernel(const float* __restrict__ in, int R, int C, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  float s = 0.f;
  if (c < C)
    for (int r = g; r < R; r += 4) s += in[(size_t)r * C + c];
  red[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && c < C) out[c] = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}
void colsum(const float* in, int R, int C, float* out, hipStream_t s) {
  hipLaunchKernelGGL(colsum_kernel, dim3((C + 63) / 64), dim3(256), 0, s, in, R, C, out);
}

// ---------------------------------------------------------------- multi-tensor launches
// One launch for many independent jobs (the tail of a training step is otherwise a chain of
// tiny kernels, each paying the ~1.6 us graph-node floor).  Blocks are dealt to jobs by a
// prefix sum over their block counts.
__global__ void __launch_bounds__(256) reduce_multi_kernel(SlabJobs j) {
  __shared__ __attribute__((aligned(16))) u16 tile[16][kRedTileP];   // optim_dev.h: conflict-free column reads
  reduce_multi_body(j, blockIdx.x, tile);
}
int reduce_slabs_blocks(SlabJobs& j) {
  int tot = 0;
  for (int k = 0; k < j.n; ++k) {
    const SlabJob& J = j.job[k];
    j.blk_start[k] = tot;
    if (J.bf || J.bfT) {
      if (J.R % 16 || J.C % 64) throw std::runtime_error("reduce_slabs_multi: cast job needs R % 16, C % 64 == 0");
      tot += (J.R / 16) * (J.C / 64);
      continue;
    }
    long b = (J.n / 4 + 255) / 256;
    tot += (int)(b < 1 ? 1 : (b > 512 ? 512 : b));
  }
  j.blk_start[j.n] = tot;
  return tot;
}
void reduce_slabs_multi(SlabJobs& j, hipStream_t s) {
  const int tot = reduce_slabs_blocks(j);
  hipLaunchKernelGGL(reduce_multi_kernel, dim3(tot), dim3(256), 0, s, j);
}

// fp32 [R][C] -> bf16 [R][C] and/or bf16 [C][R], 64x64 tiles through LDS, many tensors per launch
// 64-row tiles where an FT copy needs whole 64 x 64 fragment blocks, else 16-row tiles: 4x the
// workgroups, so a 256 x 1536 tensor (the data-parallel dP cast) reaches every CU
DEV_HOST_INLINE int cast_tile_rows(const CastJob& J) { return (J.dstF || J.dstTF) ? 64 : 16; }
__global__ void cast_multi_kernel(CastJobs j) {
  __shared__ float tile[64][65];
  int b = blockIdx.x, k = 0;
  while (k + 1 < j.n && b >= j.blk_start[k + 1]) ++k;
  const CastJob& J = j.job[k];
  const int th = cast_tile_rows(J);
  const int tiles_c = (J.C + 63) / 64;
  const int t = b - j.blk_start[k];
  const int r0 = (t / tiles_c) * th, c0 = (t % tiles_c) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int y = ty; y < th; y += 4) {
    const int r = r0 + y, c = c0 + tx;
    const float v = (r < J.R && c < J.C) ? (J.src16 ? bf2f(J.src16[(size_t)r * J.C + c]) : J.src[(size_t)r * J.C + c]) : 0.f;
    tile[y][tx] = v;
    if (J.dst && r < J.R && c < J.C) J.dst[(size_t)r * J.C + c] = f2bf(v);
  }
  if (!J.dstT && !J.dstF && !J.dstTF) return;
  __syncthreads();
  if (J.dstT)   // th consecutive threads write one column's th rows (2 th contiguous bytes)
    for (int q = threadIdx.x; q < 64 * th; q += 256) {
      const int y = q / th, x = q % th;
      const int c = c0 + y, r = r0 + x;
      if (c < J.C && r < J.R) J.dstT[(size_t)c * J.R + r] = f2bf(tile[x][y]);
    }
  if (th != 64) return;   // FT copies: whole 64 x 64 tiles only (checked on the host)
  // 512 16-B pieces per tile: (4 row tiles x 2 k-steps) fragments of 64 lanes
  for (int q = threadIdx.x; q < 512; q += 256) {
    const int fl = q & 63, fr = (q >> 6) & 3, fk = q >> 8;   // lane, 16-row tile, 32-k step
    const int rr = fr * 16 + (fl & 15), kk = fk * 32 + 8 * (fl >> 4);
    u16 v[8];
    if (J.dstF) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(tile[rr][kk + e]);
      *reinterpret_cast<uint4*>(J.dstF + ft_offset(r0 + rr, c0 + kk, J.C)) = *reinterpret_cast<const uint4*>(v);
    }
    if (J.dstTF) {   // transpose: rows are columns of the tile, k runs down its rows
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(tile[kk + e][rr]);
      *reinterpret_cast<uint4*>(J.dstTF + ft_offset(c0 + rr, r0 + kk, J.R)) = *reinterpret_cast<const uint4*>(v);
    }
  }
}
void cast_multi(CastJobs& j, hipStream_t s) {
  int tot = 0;
  for (int k = 0; k < j.n; ++k) {
    if ((j.job[k].dstF || j.job[k].dstTF) && (j.job[k].R % 64 || j.job[k].C % 64))
      throw std::runtime_error("cast_multi: FT copies need R, C % 64 == 0");
    j.blk_start[k] = tot;
    const int th = cast_tile_rows(j.job[k]);
    tot += ((j.job[k].R + th - 1) / th) * ((j.job[k].C + 63) / 64);
  }
  j.blk_start[j.n] = tot;
  hipLaunchKernelGGL(cast_multi_kernel, dim3(tot), dim3(256), 0, s, j);
}

__global__ void flat_pack_kernel(float* p, unsigned* pack, FlatRanges r, long lo, long hi, long tail, int unpack) {
  const long tot = r.total();
  for (long k = blockIdx.x * (long)blockDim.x + threadIdx.x; k < tot; k += (long)gridDim.x * blockDim.x) {
    long base = 0, f = -1;
    for (int i = 0; i < r.cnt; ++i) {
      if (k < base + r.n[i]) { f = r.off[i] + (k - base); break; }
      base += r.n[i];
    }
    if (f < 0) continue;
    if (!unpack) pack[k] = (f >= lo && f < hi) ? __float_as_uint(p[f]) : 0u;
    else if (f < tail) p[f] = __uint_as_float(pack[k]);
  }
}
void flat_pack_u32(float* p, unsigned* pack, const FlatRanges& r, long lo, long hi, long tail, int unpack, hipStream_t s) {
  const long tot = r.total();
  if (tot <= 0) return;
  const int blocks = (int)std::min<long>((tot + 255) / 256, 256);
  hipLaunchKernelGGL(flat_pack_kernel, dim3(blocks), dim3(256), 0, s, p, pack, r, lo, hi, tail, unpack);
}

__global__ void adam_kernel(OptimArgs a) {
  if (step_failed(a)) return;
  const int t = *a.step;
  const float lr = sched_lr(a, t);
  const float sc = a.gscale ? *a.gscale : 1.f;
  const float bc1 = 1.f - powf(a.b1, (float)t), bc2 = 1.f - powf(a.b2, (float)t);
  const float ib1 = 1.f / bc1, ib2 = 1.f / bc2;
  const long n4 = a.n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 p = reinterpret_cast<float4*>(a.p)[i];
    const float4 g4 = reinterpret_cast<const float4*>(a.g)[i];
    float pv[4] = {p.x, p.y, p.z, p.w};
    const float gv[4] = {g4.x * sc, g4.y * sc, g4.z * sc, g4.w * sc};
    if (a.sgd) {
#pragma unroll
      for (int e = 0; e < 4; ++e) pv[e] -= lr * (gv[e] + a.wd * pv[e]);
    } else {
      float4 m = reinterpret_cast<float4*>(a.m)[i];
      float4 v = reinterpret_cast<float4*>(a.v)[i];
      float mv[4] = {m.x, m.y, m.z, m.w}, vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        mv[e] = a.b1 * mv[e] + (1.f - a.b1) * gv[e];
        vv[e] = a.b2 * vv[e] + (1.f - a.b2) * gv[e] * gv[e];
        float u = (mv[e] * ib1) / (sqrtf(vv[e] * ib2) + a.eps);
        if (a.wd != 0.f) u += a.wd * pv[e];
        pv[e] -= lr * u;
      }
      reinterpret_cast<float4*>(a.m)[i] = make_float4(mv[0], mv[1], mv[2], mv[3]);
      reinterpret_cast<float4*>(a.v)[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
    }
    reinterpret_cast<float4*>(a.p)[i] = make_float4(pv[0], pv[1], pv[2], pv[3]);
  }
}
void adam_step(const OptimArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(adam_kernel, dim3(nblocks(a.n / 4, 256, 2048)), dim3(256), 0, s, a);
}

__global__ void __launch_bounds__(256) adam_cast_kernel(OptimArgs a, OptCastJobs j) {
  __shared__ __attribute__((aligned(16))) u16 tile[64][kAdamTileP];   // optim_dev.h: conflict-free column reads
  int b = blockIdx.x, k = 0;
  while (k + 1 < j.n && b >= j.blk_start[k + 1]) ++k;
  if (step_failed(a)) return;
  adam_cast_unit<false, false>(a, j.job[k], b - j.blk_start[k], adam_coef(a), tile);
}
void adam_cast_multi(const OptimArgs& a, OptCastJobs& j, hipStream_t s) {
  int tot = 0;
  for (int k = 0; k < j.n; ++k) {
    const OptCastJob& J = j.job[k];
    j.blk_start[k] = tot;
    tot += J.R == 0 ? (J.C + 1023) / 1024 : (J.R / 64) * (J.C / 64);
  }
  j.blk_start[j.n] = tot;
  hipLaunchKernelGGL(adam_cast_kernel, dim3(tot), dim3(256), 0, s, a, j);
}

__global__ void bump_kernel(int* step) { *step += 1; }
void bump_step(int* step, hipStream_t s) { hipLaunchKernelGGL(bump_kernel, dim3(1), dim3(1), 0, s, step); }

__global__ void sumsq_kernel(const float* __restrict__ x, long n, float* __restrict__ parts) {
  __shared__ float red[16];
  float acc = 0.f;
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    acc += x[i] * x[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
    parts[blockIdx.x] = t;
  }
}
void sumsq_partials(const float* x, long n, float* partials, int nparts, hipStream_t s) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(nparts), dim3(256), 0, s, x, n, partials);
}

__global__ void clip_final_kernel(const float* parts, int n, float clip, float* scale) {
  float t = 0.f;
  for (int i = 0; i < n; ++i) t += parts[i];
  const float norm = sqrtf(t);
  scale[0] = fminf(1.f, clip / (norm + 1e-6f));
  scale[1] = norm;
}
void clip_scale_finalize(const float* partials, int nparts, float clip, float* scale, hipStream_t s) {
  hipLaunchKernelGGL(clip_final_kernel, dim3(1), dim3(1), 0, s, partials, nparts, clip, scale);
}

__global__ void sum_partials_kernel(const float* p, int n, float* out, int* step) {
  // one wave, fixed order: deterministic
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += 64) acc += p[i];
  acc = wave_sum(acc);
  if (threadIdx.x == 0) {
    out[0] = acc;
    if (step) *step += 1;
  }
}
void sum_partials(const float* partials, int n, float* out, hipStream_t s, int* bump) {
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(64), 0, s, partials, n, out, bump);
}

// Transpose [B][T] -> [T][Bp] with padding.  `in` may be pinned HOST memory: the kernel reads it
// zero-copy over PCIe on the compute queue (no SDMA engine hand-off in front of the step graph).
// Header: in[0] = B, in[1] = bits of 1/#valid labels (computed by the host).
__global__ void prep_batch_kernel(const int* __restrict__ in, int Bmax, int T, int Bp, int* __restrict__ ids,
                                  int* __restrict__ labels, float* __restrict__ inv_count) {
  prep_batch_body(PrepJob{in, Bmax, T, Bp, ids, labels, inv_count}, blockIdx.x, gridDim.x);
}
void prep_batch(const int* in, int Bmax, int T, int Bp, int* ids, int* labels, float* inv_count, hipStream_t s) {
  const int blocks = prep_batch_blocks(T, Bp);
  hipLaunchKernelGGL(prep_batch_kernel, dim3(blocks), dim3(256), 0, s, in, Bmax, T, Bp, ids, labels, inv_count);
}

__global__ void fill_kernel(float* p, long n, float v) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = v;
}
void fill_f32(float* p, long n, float v, hipStream_t s) {
  hipLaunchKernelGGL(fill_kernel, dim3(nblocks(n, 256, 1024)), dim3(256), 0, s, p, n, v);
}

__global__ void spin_kernel(unsigned long long ticks) {
  // s_memrealtime is a constant 100 MHz counter; the loop always ends
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
void spin_delay(int us, hipStream_t s) {
  const long capped = us < 0 ? 0 : (us > 5000000 ? 5000000 : us);
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, (unsigned long long)capped * 100ull);
}

// CU blocker (fault injection): one 64-thread block per CU holding the CU's whole LDS for `ticks`
// of the 100 MHz clock, so no workgroup that needs LDS can start there meanwhile -- a stand-in for
// an RCCL kernel that holds CUs while it waits for a slow peer.  The loop always ends.
__global__ void block_cu_kernel(unsigned long long ticks) {
  extern __shared__ unsigned char lds_block[];
  if (threadIdx.x == 0) lds_block[0] = 1;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
void block_cus(int nblocks, int us, hipStream_t s) {
  const long capped = us < 0 ? 0 : (us > 5000000 ? 5000000 : us);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)block_cu_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(block_cu_kernel, dim3(nblocks), dim3(64), 160 * 1024, s, (unsigned long long)capped * 100ull);
}

// ---- graph-replay probe: is a memset / memcpy node captured on a stream ordered
// before the kernel captured after it on the same stream, on every replay, with and without host
// syncs between replays?  The kernel counts words that are not the node's value (a node that ran
// late or not at all), then overwrites every word with a pattern so a skipped node shows up on the
// next replay.  Returns the total count over all replays (0 = ordered every time).
__global__ void graph_probe_kernel(unsigned* buf, long n, unsigned want, unsigned pattern, unsigned* bad, long lo, long hi) {
  unsigned cnt = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    if (i >= lo && i < hi) cnt += buf[i] != want;   // words the node covers completely
    buf[i] = pattern;
  }
  cnt = (unsigned)wave_sum((float)cnt);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(bad, cnt);
}
static std::vector<long> g_probe_detail;   // stale words seen per kernel of the chain (last probe)
std::vector<long> graph_node_probe_detail() { return g_probe_detail; }
long graph_node_probe(long words, int reps, int sync_every, int mode) {
  // modes 8 / 9: modes 6 / 7 with the replays (and the copies around them) on the NULL stream --
  // the stream torch's current stream is by default, which the generator launches its graphs on
  const bool null_launch = mode >= 8;
  const bool copy_node = mode == 10;   // 10: mode 9 with a memcpy node in place of the memset
  if (mode == 10) mode = 7;
  else if (null_launch) mode -= 2;
  unsigned *buf = nullptr, *src = nullptr, *bad = nullptr;
  HIP_CHECK(hipMalloc(&buf, words * 4));
  HIP_CHECK(hipMalloc(&src, words * 4));
  HIP_CHECK(hipMalloc(&bad, 72 * 4));
  HIP_CHECK(hipMemset(src, 0x5A, words * 4));
  HIP_CHECK(hipMemset(bad, 0, 72 * 4));
  HIP_CHECK(hipMemset(buf, 0xFF, words * 4));
  hipStream_t s;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const unsigned want = copy_node ? 0x5A5A5A5Au : mode == 0 || mode >= 4 ? 0u : (mode == 3 ? 0x12345678u : 0x5A5A5A5Au);
  long lo = 0, hi = words;
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  HIP_CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  if (mode == 0) HIP_CHECK(hipMemsetAsync(buf, 0, words * 4, s));                                   // memset node
  else if (mode == 1) HIP_CHECK(hipMemcpyAsync(buf, src, words * 4, hipMemcpyDeviceToDevice, s));   // memcpy node
  else if (mode == 2) {
    HIP_CHECK(hipMemcpy2DAsync(buf, 256, src, 256, 256, words * 4 / 256, hipMemcpyDeviceToDevice, s));
    hi = words / 64 * 64;   // whole 256-B rows only
  }
  else if (mode == 3)   // 32-bit pattern memset node (the generator's ids / alive reset of round 2)
    HIP_CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(buf), 0x12345678, words, s));
  else if (mode == 4)   // five back-to-back memset nodes over consecutive fifths (round 2's reset chain)
    for (int q = 0; q < 5; ++q) {
      const long a = words * q / 5, b = words * (q + 1) / 5;
      HIP_CHECK(hipMemsetAsync(buf + a, 0, (b - a) * 4, s));
    }
  else if (copy_node)
    HIP_CHECK(hipMemcpyAsync(buf, src, words * 4, hipMemcpyDeviceToDevice, s));
  else if (mode == 6 || mode == 7)   // memset node first; each replay's result is copied OUT after the launch
    HIP_CHECK(hipMemsetAsync(buf, 0, words * 4, s));
  else {                // a byte memset of odd size and offset (round 2's output-row reset: Bp x (MAX_LEN+1) bytes)
    HIP_CHECK(hipMemsetAsync(reinterpret_cast<unsigned char*>(buf) + 1, 0, words * 4 - 6, s));
    lo = 1; hi = words - 2;
  }
  hipLaunchKernelGGL(graph_probe_kernel, dim3(256), dim3(256), 0, s, buf, words, want, 0xDEADBEEFu, bad, lo, hi);
  // mode 7 mirrors the generator's graph size: 70 more kernel nodes after the check (each leaves
  // the pattern in place), and outside the graph a copy-in + a memset before every replay
  if (mode == 7)
    for (int k = 0; k < 70; ++k)
      hipLaunchKernelGGL(graph_probe_kernel, dim3(64), dim3(256), 0, s, buf, words, 0xDEADBEEFu, 0xDEADBEEFu, bad + 1 + k, lo, hi);
  HIP_CHECK(hipStreamEndCapture(s, &g));
  HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  // mode 6 mirrors Generator::generate(): after each replay the stream copies the result out
  // (hipMemcpyAsync D2D); the NEXT replay's leading memset node must not overtake that copy
  unsigned* outs = nullptr;
  if (mode >= 6) HIP_CHECK(hipMalloc(&outs, (size_t)reps * words * 4));
  hipStream_t ls = null_launch ? nullptr : s;
  for (int r = 0; r < reps; ++r) {
    if (mode == 7) {
      HIP_CHECK(hipMemcpyAsync(src + words / 2, src, words / 2 * 4, hipMemcpyDeviceToDevice, ls));
      HIP_CHECK(hipMemsetAsync(src, 0x5A, 16, ls));
    }
    HIP_CHECK(hipGraphLaunch(ge, ls));
    if (mode >= 6) HIP_CHECK(hipMemcpyAsync(outs + (size_t)r * words, buf, words * 4, hipMemcpyDeviceToDevice, ls));
    if (sync_every > 0 && (r + 1) % sync_every == 0) HIP_CHECK(hipStreamSynchronize(ls));
  }
  HIP_CHECK(hipStreamSynchronize(ls));
  HIP_CHECK(hipStreamSynchronize(s));
  unsigned hb[72];
  HIP_CHECK(hipMemcpy(hb, bad, 72 * 4, hipMemcpyDeviceToHost));
  unsigned h = 0;
  g_probe_detail.assign(72, 0);
  for (int k = 0; k < 72; ++k) { h += hb[k]; g_probe_detail[k] = hb[k]; }
  long copies_bad = 0;
  if (mode >= 6) {   // every copy must hold the kernel's pattern
    std::vector<unsigned> host((size_t)reps * words);
    HIP_CHECK(hipMemcpy(host.data(), outs, host.size() * 4, hipMemcpyDeviceToHost));
    for (unsigned v : host) copies_bad += v != 0xDEADBEEFu;
    (void)hipFree(outs);
  }
  (void)hipGraphExecDestroy(ge);
  (void)hipGraphDestroy(g);
  (void)hipStreamDestroy(s);
  (void)hipFree(buf); (void)hipFree(src); (void)hipFree(bad);
  // low 32 bits: words the checking kernels saw stale; high bits: copied-out words without the pattern
  return (long)h + (copies_bad << 32);
}

// Placement census (diagnostic): out[b] = XCC id of the CU that ran block b (HW_REG_XCC_ID).
__global__ void xcc_census_kernel(unsigned* out) {
  unsigned id;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
  if (threadIdx.x == 0) out[blockIdx.x] = id;
}
void xcc_census(unsigned* out, int nblocks, int threads, hipStream_t s) {
  hipLaunchKernelGGL(xcc_census_kernel, dim3(nblocks), dim3(threads), 0, s, out);
}

}  // namespace gk
