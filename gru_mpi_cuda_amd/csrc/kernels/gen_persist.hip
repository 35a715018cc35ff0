// Persistent fp32 generation for small batches (<= 64 names): ONE launch runs every char.
//
// The batched fp32 path (gen_f32.hip) launches ~3L + 2 kernels per char, and each one streams fp32
// weights from memory. At 32 names that is 69 us per char, almost all of it launch gaps and
// weight reads of a few rows of work (profiles/r2_generate_modes_splitk.jsonl). Here the weights
// are read once per launch and stay in VGPRs.
//
//   * grid = 256 workgroups of 512 threads, one per CU, all co-resident (checked on the host).
//   * Workgroup b owns units [b U, b U + U) (U = H / 256) of every recurrent matrix (W_hh of each
//     layer, W_ih of layers >= 1) and FC rows [b VR, b VR + VR) (VR = V / 256). That is 2L row
//     tiles of 16 rows (3U gate rows used; VR rows for the FC tile).
//   * Wave w keeps the K-slice [w H/8, (w + 1) H/8) of every tile in registers as fp32 MFMA
//     A-fragments (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulate). Lane (row r,
//     quad q) holds W[r][w H/8 + q H/32 + j] for j < H/32, so its B-fragments of the hidden states
//     are H/32 contiguous floats per name (float4 loads). The 8 wave partials of a 16 x 16
//     (rows x names) tile meet in LDS and are summed in wave order.
//   * Per char t:
//       - Sample char t-1 from the logits of all 256 workgroups. Up to 16 names every workgroup
//         does this redundantly and identically (it needs the ids for layer 0's input). Above 16
//         names workgroup n samples name n alone and publishes id | alive << 16, and every
//         workgroup reads the N ids back: one more hand-off of a word per name, instead of N / 8
//         sequential samples per wave in every workgroup (11.5 us per char at 64 names).
//       - Layer 0: gi = P[id] (the workgroup's slice of the fp32 table, in LDS), then the gates.
//       - Each layer l >= 1: gi_l = h_{l-1}(t) W_ih_l^T + b_ih_l, then the gates.
//       - FC: logits = h_{L-1}(t) W_fc^T + b_fc, on the VALU: a workgroup has VR = V / 256 <= 2
//         rows, which an MFMA tile would compute as 16.
//     The recurrent products gh_l = h_l(t) W_hh_l^T + b_hh_l are only needed by the next char.
//     They reuse the x registers of the product that consumes h_l(t) anyway (gi_{l+1}, or the
//     logits), after that product's publish, so every exchanged state is read once per char and
//     the gh MFMAs overlap the next hand-off.  Padded names are neither loaded nor sampled.  With
//     several name tiles the next tile's x loads are issued before the partial-sum barriers
//     (lds_barrier: no vmcnt drain), so their latency hides behind the cross-wave sums.
//     That is L + 1 hand-offs per char, each an all-to-all of tiny slices (U or VR floats per
//     name per producer). A producer's wave 0 publishes them with write-through (sc1) stores,
//     drains them (vmcnt(0)) and stores its epoch flag. A consumer wave polls only the 32
//     producers of its K-slice (all 256 for the logits), then reads with plain loads that the 32
//     workgroups of an XCD share through its L2 (every char has its own slots).
//   * Small batches hand off without flags (round 5): every slot is filled with kEmpty (a NaN no
//     arithmetic produces) before the launch, producers store write-through with no drain, and
//     consumers re-load (sc1) the pieces they have not seen until none holds kEmpty -- the data is
//     the signal.  The logits up to 16 names (poll_x); the layer states up to 8 names at U = 4
//     (poll_xs), each producer's piece on its own 128-B line (one writer per line, the polls spread
//     over as many lines as flag polls).  Tagged states in the plain [name][H] layout (8 producers
//     per line) measured slower at 8 names (profiles/r5_gen_persist_tagged_all_probe.jsonl); on
//     their own lines 13.1 -> 11.8 us per char at 8 names (r5_gen_persist_tagx_probe.jsonl).
//     Round 2's data-tagged 8-byte granules: 44.6 against 28 us at 8 names
//     (profiles/r2_generate_persistent.jsonl).
//   * One name: the products run on the VALU (KJ FMAs per lane against name 0's x, summed over the
//     K quarters with two shuffles) instead of KJ fp32 MFMAs at 32 cycles of issue each for a
//     16-name tile with one live column: 11.5 -> 10.0 us per char.
//   * Up to 16 names every (name, unit) gate of a workgroup is one lane of wave 0: it sums layer
//     l >= 1's gi from the wave partials itself, computes the gate and stores it at once, and the
//     barrier that protects the partials follows the store (one barrier, a reduce pass and an LDS
//     round trip fewer before each publish); the logits likewise from the FC reduce.  1 name 10.0
//     -> 9.7 us per char, 8 names 12.3 -> 11.7 (profiles/r5_gen_persist_final_probe.jsonl).
//   * Gates use IEEE expf / tanhf, and sampling uses the batched sampler's code (gen_sample.h),
//     i.e. the same arithmetic as the batched fp32 path. Only the order of the fp32 partial sums
//     of each dot product differs.
//   * Spins are bounded. On a timeout, error bit 32 is set and every later wait returns
//     immediately, so the grid drains. The last workgroup to finish zeroes the flags for the next
//     launch.
// Reference: the per-char loop of /root/reference/namegensf.cu:661-884, for all names at once.
#include <stdexcept>
#include "kernels.h"
#include "common.h"
#include "gen_sample.h"

namespace gk {

namespace {
constexpr int kG = 256;        // workgroups
constexpr int kNmax = 64;      // names per launch
constexpr int kFS = 16;        // flag stride in uints (own 64-B line)
constexpr int kVmax = 512;     // V = 256 or 512 (the sampler's instances); LDS: sP is V x 3U floats
constexpr int kDistN = 16;    // more names than this: distributed sampling (workgroup n samples name n)
constexpr int kTagN = 16;     // up to this many names the logits are their own flag (slots pre-filled with kEmpty)
constexpr unsigned kEmpty = 0xFFFFFFFFu;   // a NaN no arithmetic produces from finite operands
constexpr int kTagX = 8;      // up to this many names (U = 4) the layer states are tagged too, one line per producer
constexpr int kXLine = 32;    // floats per producer line of the tagged layer-state layout (128 B)
constexpr int kStampT = 24;   // chars with diagnostic stamps
constexpr int kLgLds = kDistN * kVmax;   // redundant sampling stages names x V <= 8 K floats in LDS
constexpr unsigned kSpin = 1u << 21;   // x s_sleep(1) polls: ~0.3 s
constexpr unsigned kErrBit = 32u;
}

typedef __amdgpu_buffer_rsrc_t prsrc_t;
typedef unsigned int pu32x4 __attribute__((ext_vector_type(4)));

DEV prsrc_t prsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
DEV unsigned flag_load(const unsigned* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a value the compiler cannot hoist out of the char loop: the per-char address math of the sampler
// otherwise becomes loop-invariant VGPRs that the weight-resident register budget spills to scratch
// (a scratch reload on the hand-off's critical path)
DEV int opaque_s(int v) {   // wave-uniform values
  v = __builtin_amdgcn_readfirstlane(v);
  asm volatile("" : "+s"(v));
  return v;
}
DEV int lane_now() {   // the lane id, recomputed where it is used
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

// Wave-level wait: every producer in [lo, lo + cnt) (cnt <= 256) has published epoch `ep` of
// `kind`.  Lane l polls producers l, l + 64, ..., all of a round's flag loads in flight together.
// Two rounds in flight (the next issued before the previous is checked) measured slower: per char
// 12.9 -> 13.3 us at 1 name, 35.9 -> 42.1 at 64 (profiles/r5_gen_persist_v4_probe.jsonl) -- every
// flag line is polled by a wave of each of the 256 workgroups, and doubling that traffic delays
// the producers' own flag stores more than it shortens the detection.
DEV void pwait(const unsigned* flags, int kind, int lo, int cnt, unsigned ep, unsigned* err) {
  const int lane = threadIdx.x & 63;
  const unsigned* f = flags + ((size_t)kind * kG + lo) * kFS;
  const int nq = (cnt + 63) >> 6;   // wave-uniform
  auto issue = [&](unsigned (&v)[4]) {
    const int ln = lane_now();   // recomputed per poll: hoisted flag addresses cost 8 VGPRs for the launch
#pragma unroll
    for (int q = 0; q < 4; ++q)
      v[q] = (q < nq && ln + 64 * q < cnt) ? flag_load(f + (size_t)(ln + 64 * q) * kFS) : ep;
  };
  auto seen = [&](const unsigned (&v)[4]) {
    bool ok = true;
#pragma unroll
    for (int q = 0; q < 4; ++q) ok = ok & (v[q] >= ep);
    return __all(ok);
  };
  unsigned spins = 0;
  auto give_up = [&]() {
    __builtin_amdgcn_s_sleep(1);
    ++spins;
    if ((spins & 255) == 0 && (flag_load(err) & kErrBit)) return true;   // another workgroup gave up
    if (spins > kSpin) {
      if (lane == 0) __hip_atomic_fetch_or(err, kErrBit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
    return false;
  };
  unsigned v[4];
  for (;;) {
    issue(v);
    if (seen(v) || give_up()) break;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the payload loads below the poll
}
DEV void st_sc1(prsrc_t r, unsigned off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 16);   // aux 16 = sc1
}

// this lane's KJ floats of its name from the exchange buffer (b128 loads at byte offset off; a
// padded name, !valid, is not read).  PLAIN loads, cacheable in the XCD's L2, so the 32 workgroups
// of an XCD share one fetch of each line from the last-level cache: every char has its own slots,
// so no line is read before its producer's write-through store and flag (none can be stale in this
// launch; the kernel boundary invalidates the caches between launches).
template <int KJ>
DEV void load_x(prsrc_t r, unsigned off, bool valid, float (&x)[KJ]) {
#pragma unroll
  for (int j = 0; j < KJ; j += 4) {
    pu32x4 v = {0u, 0u, 0u, 0u};
    if (valid) v = __builtin_amdgcn_raw_buffer_load_b128(r, off + j * 4, 0, 0);
    x[j] = __uint_as_float(v.x); x[j + 1] = __uint_as_float(v.y);
    x[j + 2] = __uint_as_float(v.z); x[j + 3] = __uint_as_float(v.w);
  }
}
// tagged hand-off (the logits, <= kTagN names): the slots are filled with kEmpty before the launch and
// the producers store write-through with no drain and no flag; a consumer re-loads (sc1, past the
// non-coherent L2) the pieces it has not seen yet until none holds kEmpty -- one memory round trip
// fewer than flag + payload.  Bounded like pwait (err bit 32 on timeout).  Measured: the logits hop
// + sampling 2.7 -> 1.8 us per char at one name.  The layer-state hand-offs stay on flags: tagged
// as well (every valid lane re-polling its 8 producers' pieces) they cost 12.9 -> 12.4 us per char at
// 1 name but 14.5 -> 17.5 at 8 (profiles/r5_gen_persist_tagged_all_probe.jsonl).
template <int KJ>
DEV void poll_x(prsrc_t r, unsigned off, bool valid, float (&x)[KJ], unsigned* err) {
  constexpr int NP = KJ / 4;
  unsigned need = valid ? (1u << NP) - 1u : 0u;
  unsigned spins = 0;
  for (;;) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
      if ((need >> p) & 1u) {
        const pu32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off + p * 16, 0, 16);
        x[4 * p] = __uint_as_float(v.x); x[4 * p + 1] = __uint_as_float(v.y);
        x[4 * p + 2] = __uint_as_float(v.z); x[4 * p + 3] = __uint_as_float(v.w);
      }
#pragma unroll
    for (int p = 0; p < NP; ++p)
      if (((need >> p) & 1u) && __float_as_uint(x[4 * p]) != kEmpty && __float_as_uint(x[4 * p + 1]) != kEmpty &&
          __float_as_uint(x[4 * p + 2]) != kEmpty && __float_as_uint(x[4 * p + 3]) != kEmpty)
        need &= ~(1u << p);
    if (__all(need == 0u)) break;
    __builtin_amdgcn_s_sleep(1);
    if ((++spins & 255) == 0 && (flag_load(err) & kErrBit)) break;
    if (spins > kSpin) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or(err, kErrBit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
}
// the same over KJ / 4 producers' 16-B pieces `stride` bytes apart (the tagged layer states: each
// producer's piece on its own 128-B line, so a line has one writer and the polls of a consumer wave
// spread over as many lines as its flag polls would)
template <int KJ>
DEV void poll_xs(prsrc_t r, unsigned off, unsigned stride, bool valid, float (&x)[KJ], unsigned* err) {
  constexpr int NP = KJ / 4;
  unsigned need = valid ? (1u << NP) - 1u : 0u;
  if (!valid) {
#pragma unroll
    for (int j = 0; j < KJ; ++j) x[j] = 0.f;
  }
  unsigned spins = 0;
  for (;;) {
#pragma unroll
    for (int p = 0; p < NP; ++p)
      if ((need >> p) & 1u) {
        const pu32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off + p * stride, 0, 16);
        x[4 * p] = __uint_as_float(v.x); x[4 * p + 1] = __uint_as_float(v.y);
        x[4 * p + 2] = __uint_as_float(v.z); x[4 * p + 3] = __uint_as_float(v.w);
      }
#pragma unroll
    for (int p = 0; p < NP; ++p)
      if (((need >> p) & 1u) && __float_as_uint(x[4 * p]) != kEmpty && __float_as_uint(x[4 * p + 1]) != kEmpty &&
          __float_as_uint(x[4 * p + 2]) != kEmpty && __float_as_uint(x[4 * p + 3]) != kEmpty)
        need &= ~(1u << p);
    if (__all(need == 0u)) break;
    __builtin_amdgcn_s_sleep(1);
    if ((++spins & 255) == 0 && (flag_load(err) & kErrBit)) break;
    if (spins > kSpin) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or(err, kErrBit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
}
// one wave's partial of a 16 x 16 (rows x names) tile over its K-slice: A values aval(j), B = x;
// two accumulator chains
template <int KJ, class AVal>
DEV f32x4 tile_mm(AVal&& aval, const float (&x)[KJ]) {
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;
#pragma unroll
  for (int j = 0; j < KJ; j += 2) {
    a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(aval(j), x[j], a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(aval(j + 1), x[j + 1], a1, 0, 0, 0);
  }
  return a0 + a1;
}

// both products of one name tile from the same x (o0: A values av0, o1: av1 when TWO), and, when
// pf, the next name tile's x loaded in place b128 by b128 as soon as the MFMAs of the current
// one have consumed each piece (a rolling prefetch: its latency hides behind the remaining MFMAs
// with no second x register set)
template <int KJ, bool TWO, class A0, class A1>
DEV void tile_mm2(A0&& av0, A1&& av1, float (&x)[KJ], f32x4& o0, f32x4& o1, bool pf, __amdgpu_buffer_rsrc_t r,
                  unsigned off, bool valid) {
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0;   // TWO: a0 accumulates o0, a1 o1 (alternating chains)
#pragma unroll
  for (int j = 0; j < KJ; j += 4) {
    if constexpr (TWO) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av0(j + e), x[j + e], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av1(j + e), x[j + e], a1, 0, 0, 0);
      }
    } else {
      a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av0(j), x[j], a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av0(j + 1), x[j + 1], a1, 0, 0, 0);
      a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av0(j + 2), x[j + 2], a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av0(j + 3), x[j + 3], a1, 0, 0, 0);
    }
    if (pf) {
      pu32x4 v = {0u, 0u, 0u, 0u};
      if (valid) v = __builtin_amdgcn_raw_buffer_load_b128(r, off + j * 4, 0, 0);
      x[j] = __uint_as_float(v.x); x[j + 1] = __uint_as_float(v.y);
      x[j + 2] = __uint_as_float(v.z); x[j + 3] = __uint_as_float(v.w);
    }
  }
  if constexpr (TWO) { o0 = a0; o1 = a1; }
  else o0 = a0 + a1;
}

DEV float sig_ieee(float x) { return 1.f / (1.f + expf(-x)); }
template <int V_> struct ic { static constexpr int value = V_; };
template <int B_, int E_, class F> DEV void static_for(F&& f) {
  if constexpr (B_ < E_) { f(ic<B_>{}); static_for<B_ + 1, E_>(f); }
}

template <int KJ, int L>
__global__ void __launch_bounds__(512, 1) gen_persist_kernel(GenPersistArgs a) {
  constexpr int U = KJ / 8, H = 32 * KJ, KW = H / 8, NT = 2 * L - 1, R3 = 3 * U;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, q4 = lane >> 4;
  const int V = a.V, VR = V / kG, N = a.N, Np = (N + 15) & ~15, nnt = Np / 16, ML = a.ML;

  __shared__ float sP[kVmax * R3];            // P[v][g H + b U + u] -> sP[v][g U + u]
  __shared__ float red[kNmax / 16][2][8][256];   // wave partials of two products, per name tile
  __shared__ float sgh[L][16][kNmax];         // gh rows (incl. b_hh) x names
  __shared__ float sgi[16][kNmax];            // gi rows (incl. b_ih) / logits
  __shared__ float sh[L][kNmax][U];           // own units' hidden states
  __shared__ float sbh[L][16], sbi[L][16], sbf[16];
  __shared__ __attribute__((aligned(16))) float sWf[kVmax / kG][H];   // this workgroup's FC rows
  __shared__ int sid[kNmax], sal[kNmax];
  __shared__ int s_last, s_live;
  __shared__ __attribute__((aligned(16))) float sLG[kLgLds];   // staged logits of the last char
  __shared__ float sRf[kNmax];
  __shared__ unsigned long long sStamp[kStampT][16];   // diagnostic phase stamps (a.dbg)
  __shared__ unsigned long long sClk[kStampT];

  // one slot per char (no reuse inside a launch: see load_x), X_l[t][name][H], LG[t][name][V], then
  // (distributed sampling) ID[t][name] = id | alive-after << 16
  // two sets of exchange buffers, by launch parity: this launch uses set a.par and, after its char loop,
  // refills the other set's tagged slots with kEmpty for the next launch (no fill operations on the
  // stream: two fewer per call, docs/DESIGN.md §4)
  const size_t set_floats = (size_t)L * ML * kNmax * H + (size_t)ML * kNmax * (V + 1);
  const prsrc_t xr = prsrc(a.ws + (size_t)a.par * set_floats, (unsigned)(set_floats * 4));
  const unsigned lg0 = (unsigned)((size_t)L * ML * kNmax * H * 4);
  const unsigned id0 = lg0 + (unsigned)((size_t)ML * kNmax * V * 4);
  const bool dist = N > kDistN;   // flag kinds: 0..L-1 layer states, L logits, L + 1 sampled ids
  const bool tagged = N <= kTagN;  // the logits hand-off without flags (poll_x)
  const bool fastg = N <= 16;      // one name tile, Np U <= 64: gates and publishes by wave 0 alone
  auto xoff = [&](int l, int t, int n, int col) -> unsigned {
    return (unsigned)((((size_t)(l * ML + t) * kNmax + n) * H + col) * 4);
  };
  // tagged layer states (N <= kTagX, U = 4): X_l[t][producer][kXLine], name n's U floats at n U
  const bool tagx = U == 4 && N <= kTagX;
  auto xoffp = [&](int l, int t, int p, int n) -> unsigned {
    return (unsigned)((((size_t)(l * ML + t) * kG + p) * kXLine + n * U) * 4);
  };
  unsigned* flags = a.sync;
  unsigned* done = a.sync + (size_t)(L + 2) * kG * kFS;
  auto publish_flag = [&](int kind, int t) {   // wave 0, after its payload stores
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
      __hip_atomic_store(flags + ((size_t)kind * kG + b) * kFS, (unsigned)(t + 1), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  };

  // (probe: the launch's entry time, before the weights load; kept in a register until the stamps
  // are zeroed)
  const unsigned long long t_entry = a.dbg ? __builtin_amdgcn_s_memrealtime() : 0ull;
  // ---- resident weights: tile ti < L: W_hh_ti; L <= ti < 2L-1: W_ih_(ti-L+1).  The FC rows (VR of
  // the 16 rows of its tile) live in LDS.
  float Wr[NT][KJ];
#pragma unroll
  for (int ti = 0; ti < NT; ++ti) {
    const float* M = ti < L ? a.Whh[ti] : a.Wih[ti - L + 1];
    const bool valid = fr < R3;
    const int row = (fr / U) * H + b * U + fr % U;
    const float* src = M + (size_t)(valid ? row : 0) * H + w * KW + q4 * KJ;
#pragma unroll
    for (int j = 0; j < KJ; j += 4) {
      float4 v = valid ? *reinterpret_cast<const float4*>(src + j) : make_float4(0.f, 0.f, 0.f, 0.f);
      Wr[ti][j] = v.x; Wr[ti][j + 1] = v.y; Wr[ti][j + 2] = v.z; Wr[ti][j + 3] = v.w;
    }
  }
  for (int i = tid; i < VR * H; i += 512) sWf[i / H][i % H] = a.Wfc[(size_t)(b * VR + i / H) * H + i % H];
  for (int i = tid; i < V * R3; i += 512) {
    const int v = i / R3, c = i % R3;
    sP[i] = a.P[(size_t)v * 3 * H + (c / U) * H + b * U + c % U];
  }
  if (tid < 16) {
#pragma unroll
    for (int l = 0; l < L; ++l) {
      sbh[l][tid] = tid < R3 ? a.bhh[l][(tid / U) * H + b * U + tid % U] : 0.f;
      sbi[l][tid] = (l > 0 && tid < R3) ? a.bih[l][(tid / U) * H + b * U + tid % U] : 0.f;
    }
    sbf[tid] = tid < VR ? a.bfc[b * VR + tid] : 0.f;
  }
  for (int i = tid; i < L * kNmax * U; i += 512) (&sh[0][0][0])[i] = 0.f;
  if (a.dbg) {
    for (int i = tid; i < kStampT * 16; i += 512) (&sStamp[0][0])[i] = 0ull;
    __syncthreads();
    if (tid == 0 && ML < kStampT) sStamp[ML][14] = t_entry;   // (row ML has no layer phases)
  }
  if (tid < kNmax) { sid[tid] = a.sos; sal[tid] = tid < N ? 1 : 0; }
  if (dist ? b < N : b == 0)   // each output row has one writer: its sampler (every row: workgroup 0)
    for (int i = tid; i < (dist ? ML + 1 : N * (ML + 1)); i += 512) a.out[(dist ? (size_t)b * (ML + 1) : 0) + i] = 0;
  __syncthreads();

  // cross-wave sum of tile partials -> dst[row][name tile nt] (+ bias), rows < nrows
  // (thread i < 256 of the caller's range: element i of the tile)
  auto reduce_el = [&](float (*dst)[kNmax], int slot, int nt, const float* bias, int nrows, int i) {
    const int row = i >> 4, n = i & 15;
    float s = red[nt][slot][0][i];
#pragma unroll
    for (int k = 1; k < 8; ++k) s += red[nt][slot][k][i];
    if (row < nrows) dst[row][nt * 16 + n] = s + bias[row];
  };
  // the FC rows' partials: wave w, quarter q4 of its K-slice -> red[0][w][(4 q4 + r) 16 + name]; the
  // sum runs over the 8 waves and the 4 quarters
  auto reduce_fc_el = [&](float (*dst)[kNmax], int nt, int i) {   // i < 16 VR
    const int row = i >> 4, n = i & 15;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int q = 0; q < 4; ++q) s += red[nt][0][k][(4 * q + row) * 16 + n];
    dst[row][nt * 16 + n] = s + sbf[row];
  };
  auto stash = [&](int nt, int slot, const f32x4& acc) {
#pragma unroll
    for (int r = 0; r < 4; ++r) red[nt][slot][w][(4 * q4 + r) * 16 + fr] = acc[r];
  };
  // diagnostic phase stamps (100 MHz wall clock), first and last workgroup, thread 0 only:
  // 0 char start, 1 logits seen, 2 sampled, 3 layer 0 published, 4 + 2(l-1) layer l input seen,
  // 5 + 2(l-1) layer l published, 6 + 2(L-2) logits input seen, 7 + 2(L-2) logits published;
  // sampling internals: 8 logits staged, 9 wave 0's first name sampled, 10 wave 0's names done;
  // layer 1's phase: 11 x in, 12 MFMAs stashed, 13 reduced (<= 16 names: partials barrier), 14 gates,
  // 15 gate barrier (<= 16 names: stored); row ML: 14 the launch's entry, 13 the end of the char loop
  // Kept in LDS and copied out after the char loop: a global store per stamp put its write
  // acknowledgement inside the next vmcnt(0) of the timed phase (1 us of phantom time).
  auto stampk = [&](int t, int k) {
    if (!a.dbg || tid != 0 || (b != 0 && b != kG - 1) || k > 15 || t >= kStampT) return;
    sStamp[t][k] = __builtin_amdgcn_s_memrealtime();
    if (k == 0) sClk[t] = __builtin_amdgcn_s_memtime();   // shader clock at char start: the probe's SCLK
  };
  // gates of layer l for all names -> sh[l], then wave 0 publishes h_l(t) and its flag
  auto gates_publish = [&](int l, int t) {
    if (fastg) {
      // <= 16 names: every (name, unit) of the workgroup is one lane of wave 0, which computes its
      // gate (layers >= 1: gi summed straight from the product's wave partials, in reduce_el's
      // order) and stores it at once; the barrier that protects red / sgi / sh comes after the
      // store instead of two barriers and an LDS round trip before it
      if (w == 0) {
        const int ln = lane_now();   // (per use: hoisted lane addresses spill at the weight-resident budget)
        const int n = ln / U, u = ln % U;
        if (ln < Np * U) {
          float gi[3], gh[3];
#pragma unroll
          for (int g = 0; g < 3; ++g) {
            gh[g] = sgh[l][g * U + u][n];
            if (l == 0) {
              gi[g] = sP[sid[n] * R3 + g * U + u];
            } else {
              const int e = (g * U + u) * 16 + n;
              float sum = red[0][0][0][e];
#pragma unroll
              for (int k = 1; k < 8; ++k) sum += red[0][0][k][e];
              gi[g] = sum + sbi[l][g * U + u];
            }
          }
          const float r = sig_ieee(gi[0] + gh[0]);
          const float z = sig_ieee(gi[1] + gh[1]);
          const float nn = tanhf(gi[2] + r * gh[2]);
          const float hv = (1.f - z) * nn + z * sh[l][n][u];
          sh[l][n][u] = hv;
          if (l == 1) stampk(t, 14);   // (probe: gates)
          if (n < N) {
            if (tagx) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(hv), xr, xoffp(l, t, b, n) + 4u * u, 0, 16);
            else st_sc1(xr, xoff(l, t, n, b * U + u), hv);
          }
          if (l == 1) stampk(t, 15);   // (probe: stored)
        }
        if (!tagx) publish_flag(l, t);
      }
      __syncthreads();
      return;
    }
    for (int i = tid; i < Np * U; i += 512) {
      const int n = i / U, u = i % U;
      float gi[3], gh[3];
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        gh[g] = sgh[l][g * U + u][n];
        gi[g] = l == 0 ? sP[sid[n] * R3 + g * U + u] : sgi[g * U + u][n];
      }
      const float r = sig_ieee(gi[0] + gh[0]);
      const float z = sig_ieee(gi[1] + gh[1]);
      const float nn = tanhf(gi[2] + r * gh[2]);
      sh[l][n][u] = (1.f - z) * nn + z * sh[l][n][u];
    }
    if (l == 1) stampk(t, 14);   // (probe: gates)
    __syncthreads();
    if (l == 1) stampk(t, 15);   // (probe: barrier)
    // (wave 0 publishes every exchange; hipcc waits for a store's completion -- vmcnt(0) -- before
    // it reuses the store's data registers, so each publish waits for the previous one's
    // write-through.  A different wave per exchange shortens the publishes and lengthens the
    // consumers' wait by as much: 10.03 -> 10.19 us per char at 1 name, r5_gen_publish_wave_ab.txt)
    if (w == 0) {
      if (lane < Np) {
        if constexpr (U == 4) {
          const pu32x4 v = {__float_as_uint(sh[l][lane][0]), __float_as_uint(sh[l][lane][1]),
                            __float_as_uint(sh[l][lane][2]), __float_as_uint(sh[l][lane][3])};
          if (tagx) {   // its own line, no drain, no flag: the data is the signal
            if (lane < N) __builtin_amdgcn_raw_buffer_store_b128(v, xr, xoffp(l, t, b, lane), 0, 16);
          } else {
            __builtin_amdgcn_raw_buffer_store_b128(v, xr, xoff(l, t, lane, b * U), 0, 16);
          }
        } else {
          for (int u = 0; u < U; ++u) st_sc1(xr, xoff(l, t, lane, b * U + u), sh[l][lane][u]);
        }
      }
      if (!tagx) publish_flag(l, t);
    }
  };

  // gh_l = h_l W_hh_l^T + b_hh_l is only needed by the next char's gates: it is computed beside the
  // product that consumes h_l(t) anyway (gi_{l+1}, or the logits for the top layer), so each
  // exchanged state is read once per char.  At t = 0 (h = 0) it is the bias.
  for (int i = tid; i < L * 16 * kNmax; i += 512) {
    const int l = i / (16 * kNmax), row = (i / kNmax) % 16;
    (&sgh[0][0][0])[i] = sbh[l][row];
  }
  __syncthreads();
  // x = h_src(t) (this wave's K-slice, name tile nt) times W tile TA (-> dst rows < nrows, + bias)
  // and, unless this is the last char, times W_hh_src (-> sgh[src] for the next char)
  float xk[KJ];   // this wave's x of the last name tile, kept for the gh pass after the publish
  // one name (N = 1): lane (row fr, quarter q4) dots its KJ resident weights of tile ti with name
  // 0's x; the quarters' sum lands in name column 0 of the tile's partial slot
  const bool one = N == 1;
  auto vdot_q = [&](auto ti_tag) -> float {
    constexpr int TI = decltype(ti_tag)::value;
    float p = 0.f;
#pragma unroll
    for (int j = 0; j < KJ; ++j) p = fmaf(Wr[TI][j], xk[j], p);
    p += __shfl_xor(p, 16, 64);
    p += __shfl_xor(p, 32, 64);
    return p;
  };
  auto stash_one = [&](int slot, float p) {
    if (q4 == 0) red[0][slot][w][fr * 16] = p;
  };
  auto product = [&](auto ta_tag, auto src_tag, int t, float (*dst)[kNmax], const float* bias, int nrows, int sk) {
    constexpr int TA = decltype(ta_tag)::value, SRC = decltype(src_tag)::value;   // TA = NT: the FC rows
    const int kw0 = w * KW + q4 * KJ;
    // one name: every lane takes name 0's x (the VALU products below need it in all 16 rows)
    const int xn = one ? 0 : fr;
    const bool xv = one || fr < N;
    if (tagx) {
      stampk(t, sk);
      poll_xs<KJ>(xr, xoffp(SRC, t, kw0 / U, xn), kXLine * 4, xv, xk, a.err);
    } else {
      pwait(flags, SRC, w * 32, 32, (unsigned)(t + 1), a.err);
      stampk(t, sk);
      load_x<KJ>(xr, xoff(SRC, t, xn, kw0), xv, xk);
    }
    if (sk == 4 && a.dbg) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); stampk(t, 11); }   // (probe: x in)
    // several name tiles: gh here from the same x (re-reading it after the publish cost more)
    const bool gh = nnt > 1 && t + 1 < ML;
    auto whh = [&](int j) { return Wr[SRC][j]; };
    // every tile's MFMAs back to back (each tile's partials in their own LDS slots), the next tile's
    // x rolling in behind them; one barrier pair per product for all tiles
    for (int nt = 0; nt < nnt; ++nt) {
      // (the last tile's x stays for product_gh).  Without the register room for the in-place
      // prefetch (resident weights NT x KJ > 80 VGPRs: at 96, H = 1024 with L = 2, it fit without spills
      // but measured slower, 64 names 13.7 -> 15.7 us for layer 1) the next tile loads after these MFMAs.
      constexpr bool kRollPF = NT * KJ <= 80;
      const bool pf = kRollPF && nt + 1 < nnt;
      const unsigned noff = xoff(SRC, t, (nt + 1) * 16 + fr, kw0);
      const bool nvalid = (nt + 1) * 16 + fr < N;
      f32x4 o0, o1;
      if constexpr (TA == NT) {
        // the VR <= 2 FC rows on the VALU (an MFMA tile would compute 16 rows for them): KJ fp32
        // FMAs per row from the LDS copy, the sum over quarters and waves in reduce_fc_el
        float p0 = 0.f, p1 = 0.f;
        auto dot = [&](const float* wr, float& p) {
#pragma unroll
          for (int j = 0; j < KJ; j += 8) {
            const float4 u = *reinterpret_cast<const float4*>(wr + j);
            const float4 v = *reinterpret_cast<const float4*>(wr + j + 4);
            p = fmaf(u.x, xk[j], p); p = fmaf(u.y, xk[j + 1], p);
            p = fmaf(u.z, xk[j + 2], p); p = fmaf(u.w, xk[j + 3], p);
            p = fmaf(v.x, xk[j + 4], p); p = fmaf(v.y, xk[j + 5], p);
            p = fmaf(v.z, xk[j + 6], p); p = fmaf(v.w, xk[j + 7], p);
          }
        };
        dot(&sWf[0][kw0], p0);
        if (VR > 1) dot(&sWf[1][kw0], p1);
        red[nt][0][w][(4 * q4) * 16 + fr] = p0;
        red[nt][0][w][(4 * q4 + 1) * 16 + fr] = p1;
        if (gh) {
          tile_mm2<KJ, false>(whh, whh, xk, o1, o0, pf, xr, noff, nvalid);
          stash(nt, 1, o1);
        } else if (pf) {
          load_x<KJ>(xr, noff, nvalid, xk);
        }
      } else if (one) {
        // one name: KJ VALU FMAs per lane (row fr, quarter q4 of the K-slice), summed over the
        // quarters, instead of KJ MFMAs (32 cycles of issue each) for a 16-name tile of one column
        stash_one(0, vdot_q(ic<TA>{}));
      } else {
        auto wta = [&](int j) { return Wr[TA][j]; };
        if (gh) tile_mm2<KJ, true>(wta, whh, xk, o0, o1, pf, xr, noff, nvalid);
        else tile_mm2<KJ, false>(wta, wta, xk, o0, o1, pf, xr, noff, nvalid);
        stash(nt, 0, o0);
        if (gh) stash(nt, 1, o1);
      }
      if (!pf && nt + 1 < nnt) {   // (pf: the next tile's x is already in flight)
        __builtin_amdgcn_sched_barrier(0);   // not hoisted above the MFMAs: one x set live
        load_x<KJ>(xr, noff, nvalid, xk);
      }
    }
    if (sk == 4) stampk(t, 12);   // (probe: MFMAs issued, partials stashed)
    lds_barrier();
    if (fastg && TA != NT) {   // the gates read the partials themselves (gates_publish)
      if (sk == 4) stampk(t, 13);
      return;
    }
    for (int i = tid; i < nnt * 256; i += 512) {
      const int nt = i >> 8, e = i & 255;
      if constexpr (TA == NT) {
        if (e < 16 * nrows) {
          reduce_fc_el(dst, nt, e);
          if (fastg) {   // wave 0 lanes store their logit at once
            const int ln = lane_now(), row = ln >> 4, n = ln & 15;
            if (n < N) st_sc1(xr, lg0 + (unsigned)(((size_t)t * kNmax + n) * V + b * VR + row) * 4, dst[row][n]);
          }
        }
      } else {
        reduce_el(dst, 0, nt, bias, nrows, e);
      }
      if (gh) reduce_el(sgh[SRC], 1, nt, sbh[SRC], R3, e);
    }
    lds_barrier();
    if (sk == 4) stampk(t, 13);   // (probe: partial sums reduced)
  };
  // gh_src of the next char from the same h_src(t), after this phase's publish: with one name tile
  // its MFMAs run while the next hand-off is in flight instead of before the publish (x still in
  // xk): 22 -> 15.6 us per char at 1 name together with the sampler changes
  auto product_gh = [&](auto src_tag, int t) {
    constexpr int SRC = decltype(src_tag)::value;
    if (t + 1 >= ML || nnt > 1) return;   // (several name tiles: done inside product)
    if (one) stash_one(1, vdot_q(ic<SRC>{}));
    else stash(0, 1, tile_mm<KJ>([&](int j) { return Wr[SRC][j]; }, xk));
    lds_barrier();
    if (tid < 256) reduce_el(sgh[SRC], 1, 0, sbh[SRC], R3, tid);
    lds_barrier();
  };

  // one name's sample by one wave: logits from LDS (staged) or straight from the exchange
  auto sample_name = [&](int n, int t, bool staged, float rnd) -> int {
    const int per = V / 64;
    const unsigned base = lg0 + (unsigned)(((size_t)(t - 1) * kNmax + n) * V + lane * per) * 4;
    float* prow = (a.probs && t == ML && (dist || b == 0)) ? a.probs + (size_t)opaque_s(n) * V : nullptr;
    // the sampler instantiated for exactly V / 64 values per lane: a 16-wide instance runs all 16
    // IEEE expf / divides as selects (2.9 us per name and wave, probe_gen_persist.py)
    auto sample = [&](auto per_tag) {
      constexpr int PER = decltype(per_tag)::value;
      float xv[PER];
      if (staged) {
#pragma unroll
        for (int e = 0; e < PER; ++e) xv[e] = sLG[n * V + lane * PER + e];
      } else if (tagged) {   // this name's logits are their own flag (poll_x)
        poll_x<PER>(xr, base, true, xv, a.err);
      } else {
#pragma unroll
        for (int e = 0; e < PER; e += 4) {
          const pu32x4 v = __builtin_amdgcn_raw_buffer_load_b128(xr, base + 4 * e, 0, 0);
          xv[e] = __uint_as_float(v.x); xv[e + 1] = __uint_as_float(v.y);
          xv[e + 2] = __uint_as_float(v.z); xv[e + 3] = __uint_as_float(v.w);
        }
      }
      return softmax_sample_wave(xv, PER, V, rnd, prow);
    };
    return per == 4 ? sample(ic<4>{}) : sample(ic<8>{});
  };

  for (int t = 0; t <= ML; ++t) {
    // the last char is only sampled (workgroup 0 for every name, or each name's own sampler)
    if (t == ML && (dist ? b >= N : b != 0)) break;
    stampk(t, 0);
    // ---- sample char t-1 from the logits of every workgroup
    if (t > 0 && !dist) {   // every workgroup samples every name, redundantly and identically
      if (w == 0 && !tagged) pwait(flags, L, 0, kG, (unsigned)t, a.err);
      __syncthreads();
      stampk(t, 1);
      const unsigned lgt = lg0 + (unsigned)((size_t)(t - 1) * kNmax * V * 4);
      const bool direct = N <= 8;   // one name per wave: its logits straight into its registers
      if (!direct) {
        if (tid < N) {   // this char's uniforms, loaded together
          int tt = tid;
          asm volatile("" : "+v"(tt));   // (address math per char, not a launch-long VGPR pair)
          sRf[tt] = a.rf[(size_t)tt * ML + (t - 1)];
        }
        // every name's logits into LDS with all loads in flight: one memory round trip
        if (tagged) {   // <= 4 pieces per thread, polled two at a time until neither holds kEmpty
          const int np = N * V / 4;
          int ti = tid;
          asm volatile("" : "+v"(ti));   // (per char, not a launch-long VGPR: see opaque_s)
          for (int q0 = 0; q0 < 4 && ti + 512 * q0 < np; q0 += 2) {
            unsigned need = 1u | ((ti + 512 * (q0 + 1) < np) ? 2u : 0u);
            unsigned spins = 0;
            for (;;) {
              pu32x4 v[2];
#pragma unroll
              for (int q = 0; q < 2; ++q)
                if ((need >> q) & 1u) v[q] = __builtin_amdgcn_raw_buffer_load_b128(xr, lgt + 16u * (ti + 512 * (q0 + q)), 0, 16);
#pragma unroll
              for (int q = 0; q < 2; ++q)
                if (((need >> q) & 1u) && v[q].x != kEmpty && v[q].y != kEmpty && v[q].z != kEmpty && v[q].w != kEmpty) {
                  const int i = ti + 512 * (q0 + q);
                  sLG[4 * i] = __uint_as_float(v[q].x); sLG[4 * i + 1] = __uint_as_float(v[q].y);
                  sLG[4 * i + 2] = __uint_as_float(v[q].z); sLG[4 * i + 3] = __uint_as_float(v[q].w);
                  need &= ~(1u << q);
                }
              if (need == 0u) break;
              __builtin_amdgcn_s_sleep(1);
              if ((++spins & 255) == 0 && (flag_load(a.err) & kErrBit)) break;
              if (spins > kSpin) { __hip_atomic_fetch_or(a.err, kErrBit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); break; }
            }
          }
        } else {
          for (int i = tid; i < N * V / 4; i += 512) {
            const pu32x4 v = __builtin_amdgcn_raw_buffer_load_b128(xr, lgt + 16u * i, 0, 0);
            sLG[4 * i] = __uint_as_float(v.x); sLG[4 * i + 1] = __uint_as_float(v.y);
            sLG[4 * i + 2] = __uint_as_float(v.z); sLG[4 * i + 3] = __uint_as_float(v.w);
          }
        }
        __syncthreads();
      }
      stampk(t, 8);
      for (int n = w; n < N; n += 8) {   // real names only: a padded row keeps sid = sos
        const int sel = direct ? sample_name(n, t, false, a.rf[(size_t)n * ML + (t - 1)])
                               : sample_name(n, t, true, sRf[n]);
        if (lane == 0) {
          if (sal[n]) {
            if (b == 0) a.out[(size_t)opaque_s(n) * (ML + 1) + (t - 1)] = (unsigned char)sel;
            if (sel == a.eos) sal[n] = 0;
          }
          sid[n] = sel;
        }
        if (n == w) stampk(t, 9);
      }
      stampk(t, 10);
      __syncthreads();
    } else if (t > 0) {
      // distributed: workgroup n < N samples name n alone (its wave 0), writes its output row and
      // publishes id | alive-after << 16; every workgroup then reads the N ids -- one more hand-off
      // of one word per name instead of N / 8 sequential samples per wave in every workgroup
      if (b < N && w == 0) {
        pwait(flags, L, 0, kG, (unsigned)t, a.err);
        stampk(t, 1);
        const int sel = sample_name(b, t, false, a.rf[(size_t)b * ML + (t - 1)]);
        stampk(t, 9);
        const int alive = sal[b] && sel != a.eos;
        if (lane == 0 && sal[b]) a.out[(size_t)opaque_s(b) * (ML + 1) + (t - 1)] = (unsigned char)sel;
        if (t < ML) {
          if (lane == 0) {
            __builtin_amdgcn_raw_buffer_store_b32((unsigned)(sel | alive << 16), xr,
                                                  id0 + (unsigned)(((t - 1) * kNmax + b) * 4), 0, 16);
          }
          publish_flag(L + 1, t - 1);
        }
      }
      if (t == ML) break;
      if (w == 0) {
        pwait(flags, L + 1, 0, N, (unsigned)t, a.err);
        if (lane < N) {
          const int ln = lane_now();
          const unsigned v = __builtin_amdgcn_raw_buffer_load_b32(xr, id0 + (unsigned)(((t - 1) * kNmax + ln) * 4), 0, 0);
          sid[ln] = (int)(v & 0xFFFFu);
          sal[ln] = (int)(v >> 16);
        }
      }
      stampk(t, 10);
      __syncthreads();
    }
    if (t > 0) {
      if (t == ML) break;
      if (!a.probs) {   // every name ended: all workgroups see the same ids and stop together
        if (tid == 0) {
          int live = 0;
          for (int n = 0; n < N; ++n) live |= sal[n];
          s_live = live;
        }
        __syncthreads();
        if (!s_live) break;
      }
    }
    stampk(t, 2);
    // ---- layer 0: gi = P[id]
    gates_publish(0, t);
    stampk(t, 3);
    // ---- layers >= 1: gi_l = h_{l-1}(t) W_ih_l^T + b_ih_l  (+ gh_{l-1} of the next char)
    static_for<1, L>([&](auto lt) {
      constexpr int l = decltype(lt)::value;
      product(ic<L + l - 1>{}, ic<l - 1>{}, t, sgi, sbi[l], R3, 4 + 2 * (l - 1));
      gates_publish(l, t);
      stampk(t, 5 + 2 * (l - 1));
      product_gh(ic<l - 1>{}, t);
    });
    // ---- FC: logits rows b VR .. b VR + VR  (+ gh_{L-1} of the next char)
    product(ic<NT>{}, ic<L - 1>{}, t, sgi, sbf, VR, 6 + 2 * (L - 2));
    if (w == 0) {
      if (lane < Np && !fastg)   // (fastg: stored inside the product's reduce)
        for (int r = 0; r < VR; ++r)
          st_sc1(xr, lg0 + (unsigned)(((size_t)t * kNmax + lane) * V + b * VR + r) * 4, sgi[r][lane]);
      if (!tagged) publish_flag(L, t);
    }
    stampk(t, 7 + 2 * (L - 2));
    product_gh(ic<L - 1>{}, t);
  }

  if (a.dbg && tid == 0 && ML < kStampT) sStamp[ML][13] = __builtin_amdgcn_s_memrealtime();   // (probe: loop end)
  {   // the other set's tagged slots -> kEmpty (nobody reads that set in this launch; the next one does
      // after the kernel boundary): the layer-state lines and the logits, 1/kG of each per workgroup
    float* other = a.ws + (size_t)(1 - a.par) * set_floats;
    const size_t nst = (size_t)L * ML * kG * kXLine / 4, nlg = (size_t)ML * kNmax * V / 4;
    const pu32x4 e4 = {kEmpty, kEmpty, kEmpty, kEmpty};
    pu32x4* st4 = reinterpret_cast<pu32x4*>(other);
    pu32x4* lg4 = reinterpret_cast<pu32x4*>(other + (size_t)L * ML * kNmax * H);
    for (size_t i = (size_t)b * 512 + tid; i < nst; i += (size_t)kG * 512) st4[i] = e4;
    for (size_t i = (size_t)b * 512 + tid; i < nlg; i += (size_t)kG * 512) lg4[i] = e4;
  }
  if (a.dbg && tid == 0 && (b == 0 || b == kG - 1))
    for (int t = 0; t <= ML && t < kStampT; ++t)
      for (int k = 0; k < 16; ++k)   // slot 15 of the last workgroup's rows: its shader clock at char start
        a.dbg[((size_t)(b == 0 ? 0 : 1) * (ML + 1) + t) * 16 + k] = (b != 0 && k == 15) ? sClk[t] : sStamp[t][k];
  // ---- the last workgroup out zeroes the flags for the next launch (nobody polls them any more)
  __syncthreads();
  if (tid == 0) s_last = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == kG - 1;
  __syncthreads();
  if (s_last) {
    for (long i = tid; i < (long)(L + 2) * kG * kFS; i += 512) flags[i] = 0u;
    if (tid == 0) *done = 0u;
  }
}

#define GP_VARIANTS(X) X(8, 1) X(8, 2) X(8, 3) X(8, 4) X(16, 1) X(16, 2) X(16, 3) X(16, 4) X(32, 1) X(32, 2)

// resident workgroups of the variant on the whole device (0 on any query failure: unsupported)
static int gp_resident(int KJ, int L) {
  int dev = 0, cus = 0, nb = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
#define X(K, LL) \
  if (KJ == K && L == LL && hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, gen_persist_kernel<K, LL>, 512, 0) != hipSuccess) return 0;
  GP_VARIANTS(X)
#undef X
  return cus >= kG ? cus * nb : 0;   // one workgroup per CU is the layout; fewer CUs: unsupported
}

bool gen_persist_supported(int H, int L, int V, int N, int ML) {
  if (N < 1 || N > kNmax || L < 1 || L > 4 || H % 256 || (V != 256 && V != 512) || ML < 1) return false;
  const int KJ = H / 32;
  if (KJ != 8 && KJ != 16 && KJ != 32) return false;
  if (2 * L * KJ > 128) return false;   // resident weight registers per lane
  return gp_resident(KJ, L) >= kG;
}

long gen_persist_ws_floats(int H, int L, int V, int ML) { return 2 * ((long)L * kNmax * H + (long)kNmax * (V + 1)) * ML; }
long gen_persist_sync_words(int L) { return (long)(L + 2) * kG * kFS + 16; }

void gen_persist_fill_ws(float* ws, int H, int L, int V, int ML, hipStream_t s) {
  if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ws), (int)kEmpty, (size_t)gen_persist_ws_floats(H, L, V, ML), s) != hipSuccess)
    throw std::runtime_error("gen_persist_fill_ws: fill failed");
}

void gen_persist_f32(const GenPersistArgs& a, hipStream_t s) {
  if (!gen_persist_supported(a.H, a.L, a.V, a.N, a.ML))
    throw std::runtime_error("gen_persist_f32: unsupported shape or device (see gen_persist_supported)");
  if (!a.ws || !a.sync || !a.err || !a.P || !a.Wfc || !a.bfc || !a.rf || !a.out)
    throw std::runtime_error("gen_persist_f32: missing buffer");
  for (int l = 0; l < a.L; ++l)
    if (!a.Whh[l] || !a.bhh[l] || (l > 0 && (!a.Wih[l] || !a.bih[l])))
      throw std::runtime_error("gen_persist_f32: missing layer weights");
  const int KJ = a.H / 32;
  // tagged slots (poll_x / poll_xs) start as kEmpty: set a.par was refilled by the previous launch;
  // before the first launch the caller fills the whole workspace (gen_persist_fill_ws)
  static_assert((size_t)kG * kXLine <= (size_t)kNmax * 1024, "tagged layout inside the state slots");
  if (a.par != 0 && a.par != 1) throw std::runtime_error("gen_persist_f32: launch parity must be 0 or 1");
#define X(K, LL) \
  if (KJ == K && a.L == LL) { hipLaunchKernelGGL((gen_persist_kernel<K, LL>), dim3(kG), dim3(512), 0, s, a); return; }
  GP_VARIANTS(X)
#undef X
  throw std::runtime_error("gen_persist_f32: no variant");
}

}  // namespace gk
