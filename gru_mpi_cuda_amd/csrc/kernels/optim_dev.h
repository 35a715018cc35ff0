// Device-side optimiser pieces of the fused Adam/cast launch (misc.hip): the learning-rate schedule,
// the step error-word gate, the deterministic split-K slab sum and the Adam/SGD update of float4
// groups.
//
// SC1 = true: every gradient / slab load is an L1-bypassing `sc1` buffer load, for a gradient
// produced inside the same launch by other workgroups (sc1 stores published through an agent-scope
// counter: MI355X_MICROARCH.md 'Valid forms' row 1).  The standalone launch uses SC1 = false.
#pragma once
#include "common.h"

namespace gk {

typedef __amdgpu_buffer_rsrc_t brsrc_t;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// raw buffer resource over [p, p + bytes); aux 16 = sc1 on gfx950 (CPol::SCC)
DEV brsrc_t brsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
DEV float4 bld4_sc1(brsrc_t r, unsigned off) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
  return __builtin_bit_cast(float4, v);
}
DEV float bld1_sc1(brsrc_t r, unsigned off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 16));
}
DEV bf16x8 bld8_sc1(brsrc_t r, unsigned off) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);
  return __builtin_bit_cast(bf16x8, v);
}
DEV void bst4_sc1(brsrc_t r, unsigned off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v), r, off, 0, 16);
}
DEV void bst16_sc1(brsrc_t r, unsigned off, u32x4_t v) { __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16); }
DEV void bst8_sc1(brsrc_t r, unsigned off, u32x2_t v) { __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, 16); }
DEV void bst1_sc1(brsrc_t r, unsigned off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 16);
}

// true when the step must not be applied (see OptimArgs::err); uniform over the block
DEV bool step_failed(const OptimArgs& a) {
  if (!a.err) return false;
  const unsigned e = *a.err;
  if (a.err_host && blockIdx.x == 0 && threadIdx.x == 0) *a.err_host = e;
  return e != 0u;
}

// learning rate of update t (1-based): warm-up, then the decay of OptimArgs::sched
DEV float sched_lr(const OptimArgs& a, int t) {
  float lr = a.lr;
  if (a.warmup > 0 && t <= a.warmup) return lr * (float)t / (float)a.warmup;
  if (a.sched == 0 || a.total <= a.warmup) return lr;
  const float p = fminf(1.f, (float)(t - a.warmup) / (float)(a.total - a.warmup));
  const float f = a.sched == 1 ? 0.5f * (1.f + cosf(3.14159265358979f * p)) : 1.f - p;
  return a.lr_min + (lr - a.lr_min) * f;
}

struct AdamCoef { float sc, ib1, ib2, lr; };
// t: the 1-based update number (the step counter after this step's bump)
DEV AdamCoef adam_coef_t(const OptimArgs& a, int t) {
  return AdamCoef{a.gscale ? *a.gscale : 1.f, 1.f / (1.f - powf(a.b1, (float)t)), 1.f / (1.f - powf(a.b2, (float)t)),
                  sched_lr(a, t)};
}
DEV AdamCoef adam_coef(const OptimArgs& a) { return adam_coef_t(a, *a.step); }

// acc = sum over `splits` slabs (stride n floats) of the float4 at src + o, slab order 0,1,2,...
// (deterministic), with the loads of 8 slabs in flight at once instead of one dependent round
// trip per slab
template <bool SC1 = false>
DEV float4 sum_slabs4(const float* __restrict__ src, long n, int splits, size_t o) {
  const brsrc_t r = SC1 ? brsrc(src, (unsigned)((size_t)splits * n * 4)) : brsrc(nullptr, 0u);
  auto ld = [&](size_t e) {
    if constexpr (SC1) return bld4_sc1(r, (unsigned)(e * 4));
    else return *reinterpret_cast<const float4*>(src + e);
  };
  float4 acc = ld(o);
  for (int s0 = 1; s0 < splits; s0 += 8) {
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (s0 + k < splits) v[k] = ld((size_t)(s0 + k) * n + o);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (s0 + k < splits) { acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w; }
  }
  return acc;
}

// gradient float4 i (flat index) of job J: from the gradient buffer, or summed from J's slabs
// (same order as reduce_multi) and written back to the gradient buffer (it stays observable)
template <bool SC1 = false>
DEV float4 job_grad4(const OptimArgs& a, const OptCastJob& J, long i) {
  if (!J.gsl) {
    if constexpr (SC1) return bld4_sc1(brsrc(a.g, (unsigned)(a.n * 4)), (unsigned)(i * 16));
    else return reinterpret_cast<const float4*>(a.g)[i];
  }
  const long n = J.R ? (long)J.R * J.C : (long)J.C;
  const float4 g = sum_slabs4<SC1>(J.gsl, n, J.nsl, (size_t)(i * 4 - J.off));
  if (a.keep_g) reinterpret_cast<float4*>(const_cast<float*>(a.g))[i] = g;
  return g;
}

DEV void adam_update4(const OptimArgs& a, const AdamCoef& k, float4& p, const float4& g4, float4& m, float4& v) {
  float pv[4] = {p.x, p.y, p.z, p.w};
  const float gv[4] = {g4.x * k.sc, g4.y * k.sc, g4.z * k.sc, g4.w * k.sc};
  if (a.sgd) {
#pragma unroll
    for (int e = 0; e < 4; ++e) pv[e] -= k.lr * (gv[e] + a.wd * pv[e]);
  } else {
    float mv[4] = {m.x, m.y, m.z, m.w}, vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      mv[e] = a.b1 * mv[e] + (1.f - a.b1) * gv[e];
      vv[e] = a.b2 * vv[e] + (1.f - a.b2) * gv[e] * gv[e];
      float u = (mv[e] * k.ib1) / (sqrtf(vv[e] * k.ib2) + a.eps);
      if (a.wd != 0.f) u += a.wd * pv[e];
      pv[e] -= k.lr * u;
    }
    m = make_float4(mv[0], mv[1], mv[2], mv[3]);
    v = make_float4(vv[0], vv[1], vv[2], vv[3]);
  }
  p = make_float4(pv[0], pv[1], pv[2], pv[3]);
}

template <bool SC1 = false>
DEV float4 adam4(const OptimArgs& a, const OptCastJob& J, const AdamCoef& k, long i /*float4 index*/) {
  float4 p = reinterpret_cast<float4*>(a.p)[i];
  const float4 g4 = job_grad4<SC1>(a, J, i);
  float4 m = make_float4(0.f, 0.f, 0.f, 0.f), v = m;
  if (!a.sgd) { m = reinterpret_cast<float4*>(a.m)[i]; v = reinterpret_cast<float4*>(a.v)[i]; }
  adam_update4(a, k, p, g4, m, v);
  if (!a.sgd) { reinterpret_cast<float4*>(a.m)[i] = m; reinterpret_cast<float4*>(a.v)[i] = v; }
  reinterpret_cast<float4*>(a.p)[i] = p;
  return p;
}

// adam4 on 4 float4s at element offsets off + q*stride (q = 0..3): every load issued before any
// update, so one memory round trip instead of four.  gradient(q, i) gives float4 q (flat index i).
template <class GradFn>
DEV void adam4x4_g(const OptimArgs& a, const AdamCoef& k, long off, long stride, float4 (&out)[4], GradFn&& gradient) {
  float4 p[4], g[4], m[4], v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long i = (off + q * stride) >> 2;
    p[q] = reinterpret_cast<const float4*>(a.p)[i];
    g[q] = gradient(q, i);
    if (!a.sgd) { m[q] = reinterpret_cast<const float4*>(a.m)[i]; v[q] = reinterpret_cast<const float4*>(a.v)[i]; }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long i = (off + q * stride) >> 2;
    adam_update4(a, k, p[q], g[q], m[q], v[q]);
    if (!a.sgd) { reinterpret_cast<float4*>(a.m)[i] = m[q]; reinterpret_cast<float4*>(a.v)[i] = v[q]; }
    out[q] = p[q];
    reinterpret_cast<float4*>(a.p)[i] = out[q];
  }
}
template <bool SC1 = false>
DEV void adam4x4(const OptimArgs& a, const OptCastJob& J, const AdamCoef& k, long off, long stride,
                 float4 (&out)[4]) {
  adam4x4_g(a, k, off, stride, out, [&](int, long i) { return job_grad4<SC1>(a, J, i); });
}

// One Adam + bf16-refresh work unit: block t of job J.  Matrix job: one 64x64 tile; thread
// (ty = tid/16, tx = tid%16) updates rows ty+16q, columns 4tx..4tx+3 with float4 traffic, writes
// the row-major bf16 copy as 8-B stores, and the transpose / FT copies leave through the LDS tile
// as 16-B stores (8 consecutive rows of one column).  Flat job: 1024 elements.
// GSC1: gradient / slab loads L1-bypassing (the gradient was produced in the same launch).
// DSC1: the row-major bf16 copy (matrix) or the fp32 master (flat) leaves with write-through
// stores (read again later in the same launch).  Uniform over the block (J is).
// gtile (nullable): the tile's fp32 gradient already in LDS ([64][68], this tile's 64 x 64 block);
// it is also written to the gradient buffer (observable) unless store_g is false (the buffer
// holds something still being read, e.g. the all-reduced dP in the W_ih0 slot), and J.gsl is ignored
// bf16 staging tile pitch: 66 u16 = 33 dwords (odd), and element (r, c) sits at column c ^ adam_sw(r)
// (rows 32..63 swap 4-column groups): a 32-lane half of the transposed copies' column reads covers 8
// row segments x 4 columns, and with the pitch alone segments s and s + 4 met in one bank (2-way, 38 %
// LDS conflicts in r5_h512_pmc_summary_final.txt); rows are only 4-B aligned, so the tile is written
// and read in 4-B pieces (the swizzle moves aligned 4-column groups, so pairs stay in one dword)
constexpr int kAdamTileP = 66;
DEV int adam_sw(int r) { return (r & 32) >> 3; }
template <bool GSC1, bool DSC1>
DEV void adam_cast_unit(const OptimArgs& a, const OptCastJob& J, int t, const AdamCoef& co, u16 (*tile)[kAdamTileP],
                        const float (*gtile)[68] = nullptr, bool store_g = true) {
  if (J.R == 0) {   // flat job: 1024 elements per block
    const long i4 = (J.off >> 2) + (long)t * 256 + threadIdx.x;
    if ((long)t * 1024 + threadIdx.x * 4 < J.C) {
      if (J.dst) {   // + the flat bf16 working copy (sharded optimiser, mode 2)
        const float4 p = adam4<GSC1>(a, J, co, i4);
        typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
        const u32x2_ b = {(unsigned)f2bf(p.x) | ((unsigned)f2bf(p.y) << 16), (unsigned)f2bf(p.z) | ((unsigned)f2bf(p.w) << 16)};
        *reinterpret_cast<u32x2_*>(J.dst + (i4 * 4 - J.off)) = b;
      } else if constexpr (!DSC1) {
        adam4<GSC1>(a, J, co, i4);
      } else {
        float4 p = reinterpret_cast<float4*>(a.p)[i4];
        const float4 g4 = job_grad4<GSC1>(a, J, i4);
        float4 m = make_float4(0.f, 0.f, 0.f, 0.f), v = m;
        if (!a.sgd) { m = reinterpret_cast<float4*>(a.m)[i4]; v = reinterpret_cast<float4*>(a.v)[i4]; }
        adam_update4(a, co, p, g4, m, v);
        if (!a.sgd) { reinterpret_cast<float4*>(a.m)[i4] = m; reinterpret_cast<float4*>(a.v)[i4] = v; }
        bst4_sc1(brsrc(a.p, (unsigned)(a.n * 4)), (unsigned)(i4 * 16), p);
      }
    }
    return;
  }
  const int tiles_c = J.C / 64;
  const int r0 = (t / tiles_c) * 64, c0 = (t % tiles_c) * 64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float4 upd[4];
  if (gtile) {
    adam4x4_g(a, co, J.off + (long)(r0 + ty) * J.C + c0 + 4 * tx, 16L * J.C, upd, [&](int q, long i) {
      const float4 g = *reinterpret_cast<const float4*>(&gtile[ty + 16 * q][4 * tx]);
      if (store_g) reinterpret_cast<float4*>(const_cast<float*>(a.g))[i] = g;
      return g;
    });
  } else {
    adam4x4<GSC1>(a, J, co, J.off + (long)(r0 + ty) * J.C + c0 + 4 * tx, 16L * J.C, upd);
  }
  const brsrc_t rd = DSC1 ? brsrc(J.dst, (unsigned)((size_t)J.R * J.C * 2)) : brsrc(nullptr, 0u);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = r0 + ty + 16 * q, c = c0 + 4 * tx;
    const float4 p = upd[q];
    const u16 h0 = f2bf(p.x), h1 = f2bf(p.y), h2 = f2bf(p.z), h3 = f2bf(p.w);
    uint2 w;
    w.x = (unsigned)h0 | ((unsigned)h1 << 16);
    w.y = (unsigned)h2 | ((unsigned)h3 << 16);
    if (J.dst) {
      if constexpr (DSC1) bst8_sc1(rd, (unsigned)(((size_t)r * J.C + c) * 2), u32x2_t{w.x, w.y});
      else *reinterpret_cast<uint2*>(J.dst + (size_t)r * J.C + c) = w;
    }
    if (!J.dstT && !J.dstF && !J.dstTF) continue;
    unsigned* tw = reinterpret_cast<unsigned*>(&tile[ty + 16 * q][(4 * tx) ^ adam_sw(ty + 16 * q)]);
    tw[0] = w.x;
    tw[1] = w.y;
  }
  if (!J.dstT && !J.dstF && !J.dstTF) return;
  __syncthreads();
  if (J.dstT) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int piece = threadIdx.x + 256 * q;          // 64 columns x 8 row segments
      const int col = piece >> 3, seg = piece & 7;
      u16 v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = tile[seg * 8 + e][col ^ adam_sw(seg * 8 + e)];
      *reinterpret_cast<uint4*>(J.dstT + (size_t)(c0 + col) * J.R + r0 + seg * 8) = *reinterpret_cast<const uint4*>(v);
    }
  }
  // FT copies (fragment-tiled, kernels.h ft_offset): 512 16-B pieces per 64 x 64 tile
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int pc = threadIdx.x + 256 * q;
    const int fl = pc & 63, fr = (pc >> 6) & 3, fk = pc >> 8;   // lane, 16-row tile, 32-k step
    const int rr = fr * 16 + (fl & 15), kk = fk * 32 + 8 * (fl >> 4);
    u16 v[8];
    if (J.dstF) {   // 8 consecutive u16 of one row: four 4-B reads (column pairs kk + 2i at (kk + 2i) ^ sw)
      const int sw = adam_sw(rr);
      const unsigned* tr = reinterpret_cast<const unsigned*>(&tile[rr][0]);
      const uint4 v4 = make_uint4(tr[(kk ^ sw) >> 1], tr[((kk + 2) ^ sw) >> 1], tr[((kk + 4) ^ sw) >> 1], tr[((kk + 6) ^ sw) >> 1]);
      *reinterpret_cast<uint4*>(J.dstF + ft_offset(r0 + rr, c0 + kk, J.C)) = v4;
    }
    if (J.dstTF) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = tile[kk + e][rr ^ adam_sw(kk + e)];
      *reinterpret_cast<uint4*>(J.dstTF + ft_offset(c0 + rr, r0 + kk, J.R)) = *reinterpret_cast<const uint4*>(v);
    }
  }
}

// One block's share of a multi-tensor slab reduction (reduce_slabs_multi): block b of the prefix sum
// over the jobs' block counts; tile: 16 x kRedTileP u16 of LDS for the transposed bf16 copies.  Blocks
// past the last job do nothing.
// pitch 66 u16 = 33 dwords: the column reads' two 8-row segments land in different banks (72, 36
// dwords, put them in one: 2-way, 40 % LDS conflicts in r5_h512_pmc_summary_final.txt)
constexpr int kRedTileP = 66;
DEV void reduce_multi_body(const SlabJobs& j, int b, u16 (*tile)[kRedTileP]) {
  if (b >= j.blk_start[j.n]) return;
  int k = 0;
  while (k + 1 < j.n && b >= j.blk_start[k + 1]) ++k;
  if (j.bump && b == 0 && threadIdx.x == 0) *j.bump += 1;
  const SlabJob& J = j.job[k];
  if (J.bf || J.bfT) {   // 16x64 tile (one float4 per thread): slab sum -> fp32 / bf16 / bf16 transposed
    // 16-row tiles: 4x the workgroups of 64x64 ones, so the slab loads of a 256 x 1536 dP reach
    // every CU (96 blocks of 64x64 left most of the chip idle)
    const int tiles_c = J.C / 64, t = b - j.blk_start[k];
    const int r0 = (t / tiles_c) * 16, c0 = (t % tiles_c) * 64;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const size_t o = (size_t)(r0 + ty) * J.C + c0 + 4 * tx;
    const float4 acc = sum_slabs4(J.src, J.n, J.splits, o);
    if (J.dst) *reinterpret_cast<float4*>(J.dst + o) = acc;
    uint2 w;
    w.x = (unsigned)f2bf(acc.x) | ((unsigned)f2bf(acc.y) << 16);
    w.y = (unsigned)f2bf(acc.z) | ((unsigned)f2bf(acc.w) << 16);
    if (J.bf) *reinterpret_cast<uint2*>(J.bf + o) = w;
    if (!J.bfT) return;
    unsigned* tw = reinterpret_cast<unsigned*>(&tile[ty][4 * tx]);   // (4-B aligned rows, see kRedTileP)
    tw[0] = w.x;
    tw[1] = w.y;
    __syncthreads();
    if (threadIdx.x < 128) {   // 64 columns x 2 pieces of 8 rows (16 B)
      const int col = threadIdx.x >> 1, seg = threadIdx.x & 1;
      u16 v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = tile[seg * 8 + e][col];
      *reinterpret_cast<uint4*>(J.bfT + (size_t)(c0 + col) * J.R + r0 + seg * 8) = *reinterpret_cast<const uint4*>(v);
    }
    return;
  }
  const long n4 = J.n / 4;
  const long nb = j.blk_start[k + 1] - j.blk_start[k];
  for (long i = (b - j.blk_start[k]) * (long)blockDim.x + threadIdx.x; i < n4; i += nb * blockDim.x)
    reinterpret_cast<float4*>(J.dst)[i] = sum_slabs4(J.src, J.n, J.splits, (size_t)i * 4);
  if (b == j.blk_start[k]) {
    if (J.n < 4) {   // tiny job (e.g. the loss: many one-float partials): one wave, fixed order
      if (threadIdx.x < 64)
        for (long i = 0; i < J.n; ++i) {
          float acc = 0.f;
          for (int s = threadIdx.x; s < J.splits; s += 64) acc += J.src[(size_t)s * J.n + i];
          acc = wave_sum(acc);
          if (threadIdx.x == 0) J.dst[i] = acc;
        }
    } else {
      for (long i = n4 * 4 + threadIdx.x; i < J.n; i += blockDim.x) {
        float acc = 0.f;
        for (int s = 0; s < J.splits; ++s) acc += J.src[(size_t)s * J.n + i];
        J.dst[i] = acc;
      }
    }
  }
}

}  // namespace gk
