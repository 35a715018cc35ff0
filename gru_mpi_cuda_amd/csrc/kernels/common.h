// Shared device helpers for the gfx950 (CDNA4) kernels.
//
// Everything here is written for wave64 + MFMA 16x16x32 bf16:
//   A fragment: lane l holds A[row l&15][k = 8*(l>>4) + j], j = 0..7   (16 contiguous bytes)
//   B fragment: lane l holds B[k = 8*(l>>4) + j][col l&15]              (stored [N][K]: 16 contiguous bytes)
//   C/D:        lane l, reg i  ->  C[row (l>>4)*4 + i][col l&15]
// so every operand of the "NT" products used by the engine (both operands K-contiguous)
// is a single 16-byte load per lane per 32-deep k-step.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include "kernels.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

#define DEV __device__ __forceinline__

namespace gk {

DEV float bf2f(u16 v) { return __uint_as_float(((unsigned)v) << 16); }

// round-to-nearest-even f32 -> bf16 (hipcc lowers the plain cast to v_cvt_pk_bf16_f32, NaN-safe)
DEV u16 f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(u16, b);
}

DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

DEV bf16x8 ld8(const u16* p) { return *reinterpret_cast<const bf16x8*>(p); }
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
// acc + sum of the 8 bf16 of v: four v_dot2c_f32_bf16 against (1, 1) -- a quarter of the VALU
// issue of eight converts + adds, which beside the MFMAs slowed gemm256's row-sum workgroups 8 %
DEV float add_sum8(const bf16x8& v, float acc) {
  const bf16x2_t one = {(__bf16)1.0f, (__bf16)1.0f};
#pragma unroll
  for (int i = 0; i < 4; ++i) acc = __builtin_amdgcn_fdot2_f32_bf16(bf16x2_t{v[2 * i], v[2 * i + 1]}, one, acc, false);
  return acc;
}

DEV bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (__bf16)0.0f;
  return z;
}

// v_rcp_f32 (1 ulp) instead of the IEEE division sequence (div_scale/fmas/fixup)
DEV float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
DEV float tanhf_(float x) {
  // tanh via exp of a non-positive argument: no overflow, ~1 ulp-level agreement with tanhf
  float e = __expf(-2.0f * fabsf(x));
  float t = (1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e);
  return copysignf(t, x);
}

// Cross-lane reductions.  Within a 16-lane row they use DPP (quad_perm xor 1, xor 2,
// row_half_mirror, row_mirror: four VALU ops, every lane ends with the same value); __shfl_xor
// lowers to ds_bpermute, an LDS round trip with an lgkmcnt(0) wait per step, which serialised
// the FC softmax (profiles/: 3 us of bpermute chains per 32-row block).  Only the steps across
// rows (16, 32) still use shuffles.
template <int CTRL>
DEV float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
DEV float max16(float v) {
  v = fmaxf(v, dppf<0xB1>(v));    // quad_perm [1,0,3,2]
  v = fmaxf(v, dppf<0x4E>(v));    // quad_perm [2,3,0,1]
  v = fmaxf(v, dppf<0x141>(v));   // row_half_mirror
  v = fmaxf(v, dppf<0x140>(v));   // row_mirror
  return v;
}
DEV float sum16(float v) {   // commutative pairings: identical in every lane of the row
  v += dppf<0xB1>(v);
  v += dppf<0x4E>(v);
  v += dppf<0x141>(v);
  v += dppf<0x140>(v);
  return v;
}
DEV float wave_max(float v) {
  v = max16(v);
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}
DEV float wave_sum(float v) {
  v = sum16(v);
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}


// Batch preparation body (see prep_batch in kernels.h): block `blk` of `nblk` 256-thread blocks.
// The staging slot is pinned HOST memory (one round trip ~1.5-2 us): the batch size and the x / y
// words are loaded together (rows up to Bmax >= Bp are always inside the slot) and selected after,
// so a block pays one round trip, not two dependent ones.
DEV void prep_batch_body(const PrepJob& j, int blk, int nblk) {
  const int* x = j.in + 16;
  const int* y = x + (size_t)j.Bmax * j.T;
  const int n = j.T * j.Bp;
  const int B = j.in[0];
  for (int i = blk * 256 + (int)threadIdx.x; i < n; i += nblk * 256) {
    const int b = i / j.T, t = i - b * j.T;       // read in batch-major order (coalesced)
    const int xr = x[i], yr = y[i];
    j.ids[(size_t)t * j.Bp + b] = b < B ? xr : 0;
    j.labels[(size_t)t * j.Bp + b] = b < B ? yr : -1;
  }
  if (blk == 0 && threadIdx.x == 0) j.inv_count[0] = __int_as_float(j.in[1]);
}

// Packed bf16 saves of the large-H / wavefront kernels (a layer's SeqPlan::s16): (r, z, n, gh_n) of one
// (row, unit) item as 4 bf16 in 8 bytes -- one store in the forward, one load in the backward, half the
// bytes of the four fp32 arrays.  h itself stays fp32 (HSf).
DEV void st_save16(u16* p, float r, float z, float n, float g) {
  typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
  const u32x2_ v = {(unsigned)f2bf(r) | ((unsigned)f2bf(z) << 16), (unsigned)f2bf(n) | ((unsigned)f2bf(g) << 16)};
  *reinterpret_cast<u32x2_*>(p) = v;
}
// raw load (the packed words parked in two float registers) and the unpack at the point of use: unpacking
// right after the load made the compiler wait for it there, exposing the latency the early issue hides
// (large-H backward 3.61 -> 3.90 ms at H = 2048)
DEV void ld_save16_raw(const u16* p, float& w0, float& w1) {
  typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
  const u32x2_ v = *reinterpret_cast<const u32x2_*>(p);
  w0 = __uint_as_float(v.x);
  w1 = __uint_as_float(v.y);
}
DEV void unpack_save16(float w0, float w1, float& r, float& z, float& n, float& g) {
  const unsigned x = __float_as_uint(w0), y = __float_as_uint(w1);
  r = __uint_as_float(x << 16); z = __uint_as_float(x & 0xffff0000u);
  n = __uint_as_float(y << 16); g = __uint_as_float(y & 0xffff0000u);
}
DEV void ld_save16(const u16* p, float& r, float& z, float& n, float& g) {
  typedef unsigned u32x2_ __attribute__((ext_vector_type(2)));
  const u32x2_ v = *reinterpret_cast<const u32x2_*>(p);
  r = __uint_as_float(v.x << 16); z = __uint_as_float(v.x & 0xffff0000u);
  n = __uint_as_float(v.y << 16); g = __uint_as_float(v.y & 0xffff0000u);
}

// Workgroup barrier WITHOUT the release fence __syncthreads() carries (that fence is an
// s_waitcnt vmcnt(0), which drains every global load in flight, prefetches included): own LDS
// operations retired, then s_barrier.  For LDS hand-offs between the waves of a workgroup only.
DEV void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

}  // namespace gk
