// One GRU timestep per launch, forward and backward, for gfx950.
//
// Forward replaces the reference's per-layer 23 launches (6 matvec + 9 add + 2 sigmoid
// + 1 tanh + 3 mul + 1 oneminus + ..., /root/reference/namegensf.cu:676-763) with ONE
// launch: the three recurrent gate GEMMs  h_{t-1}·W_h{r,z,n}^T  run on MFMA for a
// 32-row x 16-unit tile *of all three gates at once*, so the epilogue
//     r = σ(Gi_r + Gh_r), z = σ(Gi_z + Gh_z), n = tanh(Gi_n + r ⊙ Gh_n), h = n + z ⊙ (h − n)
// has every operand in the same lane/register and needs no second pass.
//
// The workgroup splits K over KS waves (latency: each wave issues only its K slice's
// loads), reduces the KS partial tiles through LDS, then runs the gate epilogue.
// Backward (BPTT, no reference counterpart) is the mirror: dh_t = dGh_{t+1}·W_hh + carry
// + dy_t as the MFMA product, and the gate-gradient math as its epilogue.
#include <stdexcept>
#include "kernels.h"
#include "mma_tile.h"

namespace gk {

static constexpr int TROWS = 32;   // batch rows per workgroup (2 MFMA row blocks)
static constexpr int TUNITS = 16;  // hidden units per workgroup (x3 gates)

// LDS: partial tiles [KS][NT][4][64] fp32, then transposed staging.
struct FwdEpi { float gi[3], bh[3], hp; };

template <bool FUSE_IN>
DEV void fwd_epi_load(const FwdStepArgs& a, int p, int b0, int j0, FwdEpi& e) {
  const int H = a.H;
  const int rb = p >> 8, reg = (p >> 6) & 3, ln = p & 63;
  const int b = b0 + rb * 16 + (ln >> 4) * 4 + reg, j = j0 + (ln & 15);
#pragma unroll
  for (int g = 0; g < 3; ++g) e.bh[g] = a.bhh[g * H + j];
  if constexpr (FUSE_IN) {
#pragma unroll
    for (int g = 0; g < 3; ++g) e.gi[g] = a.bih[g * H + j];
  } else {
    const float* src = a.ids ? a.P + (size_t)a.ids[b] * 3 * H : a.Gi + (size_t)b * 3 * H;
#pragma unroll
    for (int g = 0; g < 3; ++g) e.gi[g] = src[g * H + j];
  }
  e.hp = a.hprev_f[(size_t)b * H + j];
}

// LDS: partial tiles [KS][NT][4][64] fp32, then transposed staging.
template <int KB, bool FUSE_IN>
__global__ void __launch_bounds__(512) gru_fwd_step_kernel(FwdStepArgs a, int nks_h, int nks_i) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NT = FUSE_IN ? 12 : 6;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int KS = blockDim.x >> 6;
  const int H = a.H;
  const int j0 = blockIdx.x * TUNITS;
  const int b0 = blockIdx.y * TROWS;
  const int lr = lane & 15, lk = 8 * (lane >> 4);

  // epilogue operands of this thread's first item are fetched before the MMA so their
  // latency (a dependent ids -> P gather for layer 0) hides under the recurrent GEMM
  FwdEpi pre;
  fwd_epi_load<FUSE_IN>(a, threadIdx.x, b0, j0, pre);

  f32x4 acc[2][3];
  zero_acc(acc);
  {
    const int k0 = w * nks_h * 32;
    const u16* A = a.hprev_bf + (size_t)(b0 + lr) * H + k0 + lk;
    const u16* B = a.Whh + (size_t)(j0 + lr) * H + k0 + lk;
    MmaLoop<2, 3, KB>::run(acc, A, H, B, H * H, nks_h);
  }
  float* part = smem + (size_t)w * NT * 256;
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[((r * 3 + g) * 4 + i) * 64 + lane] = acc[r][g][i];
  if constexpr (FUSE_IN) {
    f32x4 acci[2][3];
    zero_acc(acci);
    const int K = a.Kin;
    const int k0 = w * nks_i * 32;
    const u16* A = a.x_bf + (size_t)(b0 + lr) * K + k0 + lk;
    const u16* B = a.Wih + (size_t)(j0 + lr) * K + k0 + lk;
    MmaLoop<2, 3, KB>::run(acci, A, K, B, H * K, nks_i);
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) part[((6 + r * 3 + g) * 4 + i) * 64 + lane] = acci[r][g][i];
  }
  __syncthreads();

  // epilogue: 512 (row, unit) pairs; item p = rb*256 + reg*64 + lane
  u16* stage = reinterpret_cast<u16*>(smem + (size_t)KS * NT * 256);   // [16 units][32 rows]
  for (int p = threadIdx.x; p < TROWS * TUNITS; p += blockDim.x) {
    FwdEpi e;
    if (p == (int)threadIdx.x) e = pre; else fwd_epi_load<FUSE_IN>(a, p, b0, j0, e);
    const int rb = p >> 8, reg = (p >> 6) & 3, ln = p & 63;
    const int row = rb * 16 + (ln >> 4) * 4 + reg;
    const int col = ln & 15;
    const int b = b0 + row, j = j0 + col;
    float gh[3], gi[3];
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      float s = 0.f, si = 0.f;
      for (int ww = 0; ww < KS; ++ww) {
        s += smem[(size_t)ww * NT * 256 + ((rb * 3 + g) * 4 + reg) * 64 + ln];
        if constexpr (FUSE_IN) si += smem[(size_t)ww * NT * 256 + ((6 + rb * 3 + g) * 4 + reg) * 64 + ln];
      }
      gh[g] = s + e.bh[g];
      gi[g] = FUSE_IN ? si + e.gi[g] : e.gi[g];
    }
    const float r = sigmoidf_(gi[0] + gh[0]);
    const float z = sigmoidf_(gi[1] + gh[1]);
    const float n = tanhf_(gi[2] + r * gh[2]);
    const size_t o = (size_t)b * H + j;
    const float h = n + z * (e.hp - n);
    a.h_f[o] = h;
    const u16 hb = f2bf(h);
    a.h_bf[o] = hb;
    if (a.sr) { a.sr[o] = r; a.sz[o] = z; a.sn[o] = n; a.sghn[o] = gh[2]; }
    stage[col * TROWS + row] = hb;
  }
  if (a.hT) {
    __syncthreads();
    for (int q = threadIdx.x; q < TROWS * TUNITS; q += blockDim.x) {
      const int col = q >> 5, row = q & 31;
      a.hT[(size_t)(j0 + col) * a.ldT + a.colT + b0 + row] = stage[col * TROWS + row];
    }
  }
}

struct BwdEpi { float dy, carry, r, z, n, ghn, hp; };

DEV void bwd_epi_load(const BwdStepArgs& a, int p, int b0, int j0, BwdEpi& e) {
  const int rb = p >> 8, reg = (p >> 6) & 3, ln = p & 63;
  const int b = b0 + rb * 16 + (ln >> 4) * 4 + reg, j = j0 + (ln & 15);
  const size_t o = (size_t)b * a.H + j;
  e.dy = a.dy[o];
  e.carry = a.carry_in ? a.carry_in[o] : 0.f;
  e.r = a.r[o]; e.z = a.z[o]; e.n = a.n[o]; e.ghn = a.ghn[o]; e.hp = a.hprev[o];
}

template <int KB>
__global__ void __launch_bounds__(512) gru_bwd_step_kernel(BwdStepArgs a, int nks) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NT = 2;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int KS = blockDim.x >> 6;
  const int H = a.H, H3 = 3 * a.H;
  const int j0 = blockIdx.x * TUNITS;
  const int b0 = blockIdx.y * TROWS;
  const int lr = lane & 15, lk = 8 * (lane >> 4);

  BwdEpi pre;
  bwd_epi_load(a, threadIdx.x, b0, j0, pre);
  if (a.dgh_next) {
    f32x4 acc[2][1];
    zero_acc(acc);
    const int k0 = w * nks * 32;
    const u16* A = a.dgh_next + (size_t)(b0 + lr) * H3 + k0 + lk;
    const u16* B = a.WhhT + (size_t)(j0 + lr) * H3 + k0 + lk;
    MmaLoop<2, 1, KB>::run(acc, A, H3, B, 0, nks);
    float* part = smem + (size_t)w * NT * 256;
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[(r * 4 + i) * 64 + lane] = acc[r][0][i];
    __syncthreads();
  }
  // staging for transposed stores: dGh [3][16][32] and dGi_n [16][32]
  u16* st = reinterpret_cast<u16*>(smem + (size_t)KS * NT * 256);
  for (int p = threadIdx.x; p < TROWS * TUNITS; p += blockDim.x) {
    BwdEpi e;
    if (p == (int)threadIdx.x) e = pre; else bwd_epi_load(a, p, b0, j0, e);
    const int rb = p >> 8, reg = (p >> 6) & 3, ln = p & 63;
    const int row = rb * 16 + (ln >> 4) * 4 + reg;
    const int col = ln & 15;
    const int b = b0 + row, j = j0 + col;
    const size_t o = (size_t)b * H + j;
    float dh = e.dy;
    if (a.dgh_next) {
      float s = 0.f;
      for (int ww = 0; ww < KS; ++ww) s += smem[(size_t)ww * NT * 256 + (rb * 4 + reg) * 64 + ln];
      dh += s + e.carry;
    }
    const float r = e.r, z = e.z, n = e.n;
    const float dn = dh * (1.f - z);
    const float dz = dh * (e.hp - n);
    const float dan = dn * (1.f - n * n);
    const float dar = dan * e.ghn * r * (1.f - r);
    const float daz = dz * z * (1.f - z);
    a.carry_out[o] = z * dh;
    const u16 br = f2bf(dar), bz = f2bf(daz), bnh = f2bf(dan * r), bni = f2bf(dan);
    const size_t og = (size_t)b * H3 + j;
    a.dgh[og] = br; a.dgh[og + H] = bz; a.dgh[og + 2 * H] = bnh;
    if (a.dgi) { a.dgi[og] = br; a.dgi[og + H] = bz; a.dgi[og + 2 * H] = bni; }
    st[(0 * TUNITS + col) * TROWS + row] = br;
    st[(1 * TUNITS + col) * TROWS + row] = bz;
    st[(2 * TUNITS + col) * TROWS + row] = bnh;
    st[(3 * TUNITS + col) * TROWS + row] = bni;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < 3 * TROWS * TUNITS; q += blockDim.x) {
    const int g = q / (TROWS * TUNITS);
    const int rem = q - g * TROWS * TUNITS;
    const int col = rem >> 5, row = rem & 31;
    const size_t off = (size_t)(g * H + j0 + col) * a.ldT + a.colT + b0 + row;
    const u16 vh = st[(g * TUNITS + col) * TROWS + row];
    a.dghT[off] = vh;
    if (g == 2) a.dgiT[off] = st[(3 * TUNITS + col) * TROWS + row];
    else if (!a.dgiT_n_only) a.dgiT[off] = vh;
  }
}

// choose (waves per workgroup, k-steps per register batch) so that the K range splits evenly
static void pick_split(int nks_total, int& ks, int& kb) {
  for (int k : {8, 4, 2, 1})
    for (int b : {4, 2, 1})
      if (nks_total % (k * b) == 0) { ks = k; kb = b; return; }
  ks = 1; kb = 1;
}

// auto choice: the big LDS tile once the per-step GEMM is large (H >= 1024); the register tile
// below that, where its 32-row blocks give enough workgroups to fill 256 CUs
bool gru_step_picks_lds(int algo, int H, int Bp) {
  return algo == 2 || (algo == 0 && gru_step_lds_ok(H, Bp) && (H * 2 / 64) * (Bp / 128) >= 128);
}
static bool use_lds(int algo, int H, int Bp, bool fused, int Kin, int ldT, int colT) {
  // fused input projection: a first K phase of Kin (whole 64-deep k-tiles)
  const bool ok = (!fused || (Kin % 64 == 0 && Kin >= 64)) && gru_step_lds_ok(H, Bp) && ldT % 8 == 0 && colT % 8 == 0;
  if (algo == 2 && !ok) throw std::runtime_error("gru step: LDS kernel requested for an unsupported shape");
  return ok && gru_step_picks_lds(algo, H, Bp);
}

void gru_fwd_step(const FwdStepArgs& a, hipStream_t s) {
  if (use_lds(a.algo, a.H, a.Bp, a.x_bf != nullptr, a.Kin, a.ldT, a.colT)) { gru_fwd_step_lds(a, s); return; }
  if (a.s16) throw std::runtime_error("gru_fwd_step: packed bf16 saves need the LDS-staged step kernels");
  const int nks = a.H / 32;
  int ks, kb;
  pick_split(nks, ks, kb);
  const bool fuse = a.x_bf != nullptr;
  int nks_i = 0;
  if (fuse) {
    const int nki = a.Kin / 32;
    // both K ranges must split over the same wave count
    while (ks > 1 && (nki % ks != 0 || (nki / ks) % kb != 0 || (nks / ks) % kb != 0)) ks >>= 1;
    while (kb > 1 && ((nks / ks) % kb != 0 || (nki / ks) % kb != 0)) kb >>= 1;
    nks_i = nki / ks;
  }
  dim3 grid(a.H / TUNITS, a.Bp / TROWS);
  const int NT = fuse ? 12 : 6;
  const size_t shm = (size_t)ks * NT * 256 * 4 + TROWS * TUNITS * 2;
  const int nk = nks / ks;
#define FWD_LAUNCH(KBV, F) hipLaunchKernelGGL((gru_fwd_step_kernel<KBV, F>), grid, dim3(64 * ks), shm, s, a, nk, nks_i)
  if (fuse) {
    if (kb == 4) FWD_LAUNCH(4, true); else if (kb == 2) FWD_LAUNCH(2, true); else FWD_LAUNCH(1, true);
  } else {
    if (kb == 4) FWD_LAUNCH(4, false); else if (kb == 2) FWD_LAUNCH(2, false); else FWD_LAUNCH(1, false);
  }
#undef FWD_LAUNCH
}

void gru_bwd_step(const BwdStepArgs& a, hipStream_t s) {
  if (use_lds(a.algo, a.H, a.Bp, false, 0, a.ldT, a.colT)) { gru_bwd_step_lds(a, s); return; }
  const int nks = 3 * a.H / 32;
  int ks, kb;
  pick_split(nks, ks, kb);
  dim3 grid(a.H / TUNITS, a.Bp / TROWS);
  const size_t shm = (size_t)ks * 2 * 256 * 4 + 4 * TROWS * TUNITS * 2;
  const int nk = nks / ks;
  if (kb == 4) hipLaunchKernelGGL((gru_bwd_step_kernel<4>), grid, dim3(64 * ks), shm, s, a, nk);
  else if (kb == 2) hipLaunchKernelGGL((gru_bwd_step_kernel<2>), grid, dim3(64 * ks), shm, s, a, nk);
  else hipLaunchKernelGGL((gru_bwd_step_kernel<1>), grid, dim3(64 * ks), shm, s, a, nk);
}

}  // namespace gk
