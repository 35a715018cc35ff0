// fp32 softmax + inverse-CDF sampling of one row by one wave, shared by the batched sampler
// (gen_f32.hip: sample_f32) and the persistent small-batch generator (gen_persist.hip), so both
// paths pick chars by the same arithmetic: max-subtracted expf softmax, the inclusive CDF as
// lane-local sums in index order + a wave scan of the lane totals, and the reference's `psum > r`
// rule (first index whose running sum exceeds r, else V - 1; /root/reference/namegensf.cu:322-333).
//
// Cross-lane steps use DPP inside each 16-lane row and readlane across the four rows, combined in a
// fixed order, so every lane gets bit-identical statistics.  The ds_bpermute shuffles they replace
// are one LDS round trip each: about 30 dependent ones per row made a char's sampling phase in the
// persistent generator 3-8 us (scripts/probe_gen_persist.py).
#pragma once
#include "common.h"

namespace gk {

template <int N> DEV float dpp_shr(float v) {   // row_shr:N, 0 where the source is outside the row
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x110 | N, 0xF, 0xF, false));
}
DEV float rdl(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
DEV float wave_max_dpp(float v) {
  v = max16(v);
  return fmaxf(fmaxf(rdl(v, 0), rdl(v, 16)), fmaxf(rdl(v, 32), rdl(v, 48)));
}
DEV float wave_sum_dpp(float v) {
  v = sum16(v);
  return (rdl(v, 0) + rdl(v, 16)) + (rdl(v, 32) + rdl(v, 48));
}
DEV int wave_min_dpp(int v) {
  v = min(v, __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false));
  v = min(v, __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false));
  return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
// inclusive prefix sum over the 64 lanes: Hillis-Steele inside each row, then the row totals
DEV float wave_scan_incl_dpp(float v) {
  v += dpp_shr<1>(v);
  v += dpp_shr<2>(v);
  v += dpp_shr<4>(v);
  v += dpp_shr<8>(v);
  const float t0 = rdl(v, 15), t1 = rdl(v, 31), t2 = rdl(v, 47);
  const int row = (threadIdx.x & 63) >> 4;
  const float off = row == 0 ? 0.f : row == 1 ? t0 : row == 2 ? t0 + t1 : (t0 + t1) + t2;
  return v + off;
}

// xv[e], e < per (per = V / 64 <= MAXPER): logits V[lane * per + e].  Returns the chosen index
// (identical in every lane).  prow (nullable): the softmax row is written there.
template <int MAXPER>
DEV int softmax_sample_wave(const float (&xv)[MAXPER], int per, int V, float rnd, float* prow) {
  const int lane = threadIdx.x & 63;
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < MAXPER; ++e) mx = fmaxf(mx, xv[e]);
  mx = wave_max_dpp(mx);
  float ex[MAXPER];
  float se = 0.f;
#pragma unroll
  for (int e = 0; e < MAXPER; ++e) {
    ex[e] = e < per ? expf(xv[e] - mx) : 0.f;
    se += ex[e];
  }
  se = wave_sum_dpp(se);
  float p[MAXPER];
  float loc = 0.f;
#pragma unroll
  for (int e = 0; e < MAXPER; ++e) {
    p[e] = e < per ? ex[e] / se : 0.f;
    loc += p[e];
    if (prow && e < per) prow[lane * per + e] = p[e];
  }
  const float inc = wave_scan_incl_dpp(loc);
  float psum = inc - loc;
  int hit = V;
#pragma unroll
  for (int e = 0; e < MAXPER; ++e) {
    psum += p[e];
    if (e < per && hit == V && psum > rnd) hit = lane * per + e;
  }
  hit = wave_min_dpp(hit);
  return hit >= V ? V - 1 : hit;
}

}  // namespace gk
