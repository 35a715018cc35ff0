// fp32 softmax + inverse-CDF sampling of one row by one wave, shared by the batched sampler
// (gen_f32.hip: sample_f32) and the persistent small-batch generator (gen_persist.hip), so both
// paths pick chars by the same arithmetic: max-subtracted expf softmax, the inclusive CDF as
// lane-local sums in index order + a wave scan of the lane totals, and the reference's `psum > r`
// rule (first index whose running sum exceeds r, else V - 1; /root/reference/namegensf.cu:322-333).
#pragma once
#include "common.h"

namespace gk {

// xv[e], e < per (per = V / 64 <= MAXPER): logits V[lane * per + e].  Returns the chosen index
// (identical in every lane).  prow (nullable): the softmax row is written there.
template <int MAXPER>
DEV int softmax_sample_wave(const float (&xv)[MAXPER], int per, int V, float rnd, float* prow) {
  const int lane = threadIdx.x & 63;
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < MAXPER; ++e) mx = fmaxf(mx, xv[e]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float se = 0.f;
#pragma unroll
  for (int e = 0; e < MAXPER; ++e)
    if (e < per) se += expf(xv[e] - mx);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
  float p[MAXPER];
  float loc = 0.f;
#pragma unroll
  for (int e = 0; e < MAXPER; ++e) {
    p[e] = e < per ? expf(xv[e] - mx) / se : 0.f;
    loc += p[e];
    if (prow && e < per) prow[lane * per + e] = p[e];
  }
  float inc = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  float psum = inc - loc;
  int hit = V;
#pragma unroll
  for (int e = 0; e < MAXPER; ++e) {
    psum += p[e];
    if (e < per && hit == V && psum > rnd) hit = lane * per + e;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) hit = min(hit, __shfl_xor(hit, o, 64));
  return hit >= V ? V - 1 : hit;
}

}  // namespace gk
