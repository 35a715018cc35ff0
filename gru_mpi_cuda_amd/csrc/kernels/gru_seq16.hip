// Persistent backward with 16-row row blocks (the config-4 shard, L = 2,
// H = 1024, 128 sequences per GPU).
//
// gru_seq.hip's backward tiles a layer as (H/16 unit tiles) x (Bp/32 row blocks).  At Bp = 128 that
// is 4 row blocks of 64 workgroups: a row block spans two XCDs, so its dGh hand-off runs the
// write-through protocol, and every workgroup streams 32 rows x 3H of dGh_{t+1} (192 KB at
// H = 1024) per step -- 5.0-5.2 us per step, twice the 96 KB / 2.8 us of the headline's backward.
// Here a workgroup owns 16 rows x 32 units instead: (H/32) x (Bp/16) = 256 workgroups again, 8 row
// blocks -> one per XCD (the row block is the fast block index, placement verified at run time by
// row_block_local), and half the streamed bytes per step (16 rows x 3H).  The price is a W_hh^T slice
// twice as wide (32 units x 3H = 192 KB at H = 1024): one half stays lane-linear in LDS, the other
// in VGPRs, for the whole sequence.
//
// Per step (as gru_bwd_seq_kernel): each wave streams its K-slice of dGh_{t+1} (one producer per
// 32-column k-step: wave_wait_load1), 2 MFMAs per k-step (one per 16-unit half), partials of the 8
// waves meet in LDS, the gate-gradient epilogue (one element per thread), wave 0 publishes the
// [3 gates][16 rows][32 units] tile (3 KB, whole lines of its own) + flag, waves 1-4 write the
// transposed dGh^T / dGi^T copies, and layer 0 accumulates dP = sum_t onehot(x_t)^T dGi_t on the
// MFMA pipe (K = 16 rows, zero-padded to the 32-deep MFMA).  Bias and dP partials per 16-row block:
// [Bp/16][3H] and [Bp/16][V][3H].  Reference: /root/reference/namegensf.cu:773-854 (the L = 2 model).
#include <stdexcept>
#include "kernels.h"
#include "mma_tile.h"
#include "seq_sync.h"

namespace gk {

template <int NKW3, int NTP>
__global__ void __launch_bounds__(512, 1) gru_bwd_seq16_kernel(SeqBwdArgs a) {
  __shared__ __attribute__((aligned(16))) float part[8][2][256];      // [wave][unit half][4 x 64 lanes]
  __shared__ __attribute__((aligned(16))) u16 srow[3][16][40];        // dGh tile [gate][row][32 units] (80-B rows)
  __shared__ __attribute__((aligned(16))) u16 sgT[4][32][24];         // [dGh r,z,n | dGi n][unit][16 rows] (48-B rows)
  __shared__ __attribute__((aligned(16))) float red[6][32][17];
  __shared__ __attribute__((aligned(16))) bf16x8 bwL[NKW3][512];      // W_hh^T units j0..j0+15, lane-linear
  __shared__ __attribute__((aligned(16))) int idsL[NTP > 0 ? 16 : 1];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, H3 = 3 * a.H, Bp = a.Bp, T = a.T;
  const int nrb = Bp / 16, ut = seq_unit_tile(nrb);
  const int j0 = ut * 32, rbk = seq_row_block(nrb), b0 = rbk * 16;
  const int lr = lane & 15, lk = 8 * (lane >> 4);
  const int k0 = w * NKW3 * 32;
  const unsigned nunit = (unsigned)(H / 32);

  // this wave's K-slice of W_hh^T rows j0..j0+31: the first 16 units in LDS, the second in VGPRs
  bf16x8 bw1[NKW3];
#pragma unroll
  for (int kk = 0; kk < NKW3; ++kk) {
    bwL[kk][tid] = ld8(a.WhhT + (size_t)(j0 + lr) * H3 + k0 + kk * 32 + lk);
    bw1[kk] = ld8(a.WhhT + (size_t)(j0 + 16 + lr) * H3 + k0 + kk * 32 + lk);
  }

  // epilogue element of this thread: unit half uh, accumulator register reg, lane ln
  const int uh = tid >> 8, reg = (tid >> 6) & 3, ln = tid & 63;
  const int row = (ln >> 4) * 4 + reg, col = uh * 16 + (ln & 15);
  const int b = b0 + row, j = j0 + col;
  float carry = 0.f;
  float dbh[3] = {0.f, 0.f, 0.f}, dbi = 0.f;
  f32x4 accP[3][2][NTP > 0 ? NTP : 1];
#pragma unroll
  for (int g = 0; g < 3; ++g) zero_acc(accP[g]);
  // exchange ring: the slot of step t is reused at step t - xr.  Safe for xr >= 2: a producer writes
  // step t only after every producer of its row block published step t + 1, i.e. finished reading
  // the tiles of step t + 2 -- the ones the write replaces when xr = 2.
  const int xr = a.xring >= 2 ? a.xring : T;
  const rsrc_t rX = make_rsrc(a.xbuf, (unsigned)((size_t)T * Bp * H3 * 2));
  const unsigned xlane = (unsigned)((lr * 32 + lk) * 2);   // fragment lane offset in a 1-KB gate block
  zero_next_flags(a.zero_next, a.zero_words);
  const bool loc = a.allow_local && row_block_local(a.cnt + (size_t)rbk * nunit * kFlagStride, ut, (int)nunit, a.err);
  float sv[6];
  int svid = 0;
  auto load_saves = [&](int t) {
    const size_t o = ((size_t)t * Bp + b) * H + j;
    sv[0] = a.dy[o];
    if (a.s16) ld_save16_raw(a.s16 + o * 4, sv[1], sv[2]);   // unpacked at use
    else { sv[1] = a.sr[o]; sv[2] = a.sz[o]; sv[3] = a.sn[o]; sv[4] = a.sghn[o]; }
    sv[5] = a.HSf[o];   // HS[t] = h_{t-1}
    if constexpr (NTP > 0) svid = a.ids[(size_t)t * Bp + b];
  };
  load_saves(T - 1);

  for (int t = T - 1; t >= 0; --t) {
    const int s = T - 1 - t;
    stamp(a.dbg, s, 0);
    f32x4 acc[2];
    acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc[1] = acc[0];
    if (s > 0) {
      // k-step kk: columns c0 = k0 + 32 kk .. +31 = gate c0 / H, units of producer (c0 % H) / 32
      bf16x8 af[NKW3];
      const size_t slot = ((size_t)((t + 1) % xr) * nrb + rbk) * nunit;
      wave_wait_load1<NKW3>(a.cnt + (size_t)rbk * nunit * kFlagStride, lane < NKW3,
                            ((k0 + 32 * lane) % H) / 32, (unsigned)s, a.err, [&](int kk) {
        const int c0 = k0 + kk * 32;
        const int so = (int)((((slot + (size_t)((c0 % H) / 32)) * 3 + (size_t)(c0 / H)) * 512) * 2);
        af[kk] = ld8_sc1s(rX, xlane, so);
      });
      stamp(a.dbg, s, 1);
#pragma unroll
      for (int kk = 0; kk < NKW3; ++kk) {
        acc[0] = mfma16(af[kk], bwL[kk][tid], acc[0]);
        acc[1] = mfma16(af[kk], bw1[kk], acc[1]);
      }
    }
    const int idc = svid;
    float sr = sv[1], sz = sv[2], sn = sv[3], sghn = sv[4];
    if (a.s16) unpack_save16(sv[1], sv[2], sr, sz, sn, sghn);
    const float dy = sv[0], hprev = sv[5];
    if (t > 0) load_saves(t - 1);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 4; ++i) part[w][u][i * 64 + lane] = acc[u][i];
    __syncthreads();
    stamp(a.dbg, s, 2);
    float dh = dy + carry;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) dh += part[ww][uh][reg * 64 + ln];
    const float dn = dh * (1.f - sz);
    const float dz = dh * (hprev - sn);
    const float dan = dn * (1.f - sn * sn);
    const float dar = dan * sghn * sr * (1.f - sr);
    const float daz = dz * sz * (1.f - sz);
    const float dhn = dan * sr;
    carry = sz * dh;
    dbh[0] += dar; dbh[1] += daz; dbh[2] += dhn; dbi += dan;
    const u16 br = f2bf(dar), bz = f2bf(daz), bn = f2bf(dhn), bi = f2bf(dan);
    srow[0][row][col] = br; srow[1][row][col] = bz; srow[2][row][col] = bn;
    sgT[0][col][row] = br; sgT[1][col][row] = bz; sgT[2][col][row] = bn; sgT[3][col][row] = bi;
    if constexpr (NTP > 0) {
      if (col == 0) idsL[row] = idc;
    }
    __syncthreads();
    stamp(a.dbg, s, 3);
    if (w == 0) {
      // publish dGh_t as 3 gate blocks of [16 rows][32 units] (1 KB each, whole lines of its own)
      const size_t tile = (((size_t)(t % xr) * nrb + rbk) * nunit + ut) * (3 * 16 * 32);
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(&srow[g][lane >> 2][(lane & 3) * 8]);
        if (loc) st16_plain(rX, (unsigned)((tile + g * 512 + lane * 8) * 2), v);
        else st16_sc1(rX, (unsigned)((tile + g * 512 + lane * 8) * 2), v);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      unsigned* fl = a.cnt + ((size_t)rbk * nunit + ut) * kFlagStride;
      if (lane == 0) {
        if (loc) signal_flag_local(fl, (unsigned)(s + 1));
        else signal_flag(fl, (unsigned)(s + 1));
      }
      stamp(a.dbg, s, 4);
    } else if (w <= 4 && a.dghT) {
      // transposed copies for the weight-gradient GEMMs: 32 units x 16 rows per kind
      const int g = w - 1;          // 0..3 : dGh r, z, n and dGi n
      const u32x4 v = *reinterpret_cast<const u32x4*>(&sgT[g][lane >> 1][(lane & 1) * 8]);
      const size_t c0 = (size_t)t * Bp + b0 + (lane & 1) * 8;
      const int gg = g < 3 ? g : 2;
      const size_t rowsel = (size_t)(gg * H + j0 + (lane >> 1)) * a.ldG + c0;
      if (g < 3) *reinterpret_cast<u32x4*>(a.dghT + rowsel) = v;
      if (a.dgiT && (g == 3 || (g < 2 && !a.dgiT_n_only))) *reinterpret_cast<u32x4*>(a.dgiT + rowsel) = v;
    }
    if (a.dgi) {   // row-major dGi for the layer below, after the publish
      const size_t og = ((size_t)t * Bp + b) * H3 + j;
      a.dgi[og] = br; a.dgi[og + H] = bz; a.dgi[og + 2 * H] = bi;
    }
    stamp(a.dbg, s, 5);
    if constexpr (NTP > 0) {
      // dP += onehot(x_t)^T dGi_t over this block's 16 rows: A = dGi^T [unit][row] (K = rows, the
      // upper 16 of the 32-deep MFMA zero), B = one-hot [row][vocab column]
      const bool kin = lk < 16;
      int idv[8];
      if (kin) {
        const int4 i0 = *reinterpret_cast<const int4*>(&idsL[lk]), i1 = *reinterpret_cast<const int4*>(&idsL[lk + 4]);
        idv[0] = i0.x; idv[1] = i0.y; idv[2] = i0.z; idv[3] = i0.w;
        idv[4] = i1.x; idv[5] = i1.y; idv[6] = i1.z; idv[7] = i1.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) idv[e] = -1;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        bf16x8 ga[3];
#pragma unroll
        for (int g = 0; g < 3; ++g) {
          const int kind = g < 2 ? g : 3;   // dGi: the n gate without r
          ga[g] = kin ? *reinterpret_cast<const bf16x8*>(&sgT[kind][u * 16 + lr][lk]) : bf16x8{};
        }
#pragma unroll
        for (int nt = 0; nt < NTP; ++nt) {
          const int v = (w * NTP + nt) * 16 + lr;
          bf16x8 oh;
#pragma unroll
          for (int e = 0; e < 8; ++e) oh[e] = (__bf16)(idv[e] == v ? 1.0f : 0.0f);
#pragma unroll
          for (int g = 0; g < 3; ++g) accP[g][u][nt] = mfma16(ga[g], oh, accP[g][u][nt]);
        }
      }
    }
    stamp(a.dbg, s, 6);
  }

  if constexpr (NTP > 0) {
    float* Pp = a.dP_part + (size_t)rbk * a.V * H3;
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int nt = 0; nt < NTP; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            Pp[(size_t)((w * NTP + nt) * 16 + lr) * H3 + g * H + j0 + u * 16 + (lane >> 4) * 4 + i] = accP[g][u][nt][i];
  }
  // ---- bias gradients: reduce the per-thread sums over the 16 rows of the block
  red[0][col][row] = dbh[0]; red[1][col][row] = dbh[1]; red[2][col][row] = dbh[2];
  red[3][col][row] = dbh[0]; red[4][col][row] = dbh[1]; red[5][col][row] = dbi;
  __syncthreads();
  if (tid < 192) {
    const int k = tid >> 5, c = tid & 31;
    float sum = 0.f;
    for (int rr = 0; rr < 16; ++rr) sum += red[k][c][rr];
    float* dst = (k < 3 ? a.dbhh_part : a.dbih_part);
    if (dst) dst[(size_t)rbk * H3 + (k % 3) * H + j0 + c] = sum;
  }
}

// ==================================================================== host side
template <class K>
static int resident16(K kernel) {
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, 512, 0) != hipSuccess) return 0;
  return ncu * per;
}

bool gru_bwd_seq16_supported(int H, int Bp, bool fuse_p) {
  if (H != 1024 || Bp % 16) return false;
  const int cap = fuse_p ? resident16(gru_bwd_seq16_kernel<12, 2>) : resident16(gru_bwd_seq16_kernel<12, 0>);
  return cap >= (H / 32) * (Bp / 16);
}

void gru_bwd_seq16(const SeqBwdArgs& a, hipStream_t s) {
  if (a.H != 1024 || a.Bp % 16 || a.dWhh_part || (a.dP_part && a.V != 256))
    throw std::runtime_error("gru_bwd_seq16: H = 1024, Bp % 16 == 0, no fused dW_hh, V = 256 for the fused dP");
  const dim3 grid((a.H / 32) * (a.Bp / 16)), block(512);
  if (a.dP_part) hipLaunchKernelGGL((gru_bwd_seq16_kernel<12, 2>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((gru_bwd_seq16_kernel<12, 0>), grid, block, 0, s, a);
}

}  // namespace gk
