// The embedding-side table gradient at large H as a streaming kernel:
//     dP[v][c] = sum_k [ids[k] == v] * G[c][k]       (C = onehot(ids)^T . G^T, V = 256 rows)
// G is the transposed gate gradient [3H][B*T] (dGh^T for the r / z rows, dGi^T for the n rows,
// GemmArgs::B / B2), the largest operand of the step at H = 2048 (805 MB of bf16 for 512 x 128
// tokens).  The general one-hot GEMM (gemm_lds.hip, 128 x 128 tiles) reads it twice -- two row tiles
// of the vocabulary -- and spends MFMAs on a 256 x 64 A tile with 64 nonzeros per k-tile: 345 us at
// h2048, 2.3 TB/s (profiles/r6_c5_step_summary.txt).
//
// Here one workgroup covers ALL 256 vocabulary rows for NC columns c of one K-slice, so G streams from
// memory exactly once, through a 4-deep LDS-DMA ring of 16 KiB k-tiles (NC rows x KT tokens; default
// 128 x 64) with the k-tile's KT int32 ids DMA'd behind each G tile; two workgroups per CU.  The ring
// slots are four separate LDS objects and the k loop is unrolled by 4, so every slot is a compile-time
// object, and the ring is read through inline-asm ds_reads (below).  A wave owns 64 vocabulary rows
// (4 tiles of 16) x NC columns; per k-tile four ballots over the ids tell which of its tiles occur,
// and it synthesises the one-hot A fragment and runs the NC / 16 MFMAs per k-step only for those --
// skipping an all-zero A tile is exact (ids outside [0, 256) match nothing, as in the one-hot
// gemm_lds kernel).  Names use a few dozen characters, so most waves skip most k-tiles and the kernel
// runs at the G stream's rate; with uniformly random ids (the tests) every tile is active and the MFMA
// work (1024 cycles per wave per 16 KiB k-tile) still stays under the stream.
// Output: split-K slabs C + sp * M * ldc, summed by the caller's slab reduce (same contract as the
// one-hot gemm_lds launch it replaces).  The reference builds dP's counterpart, the embedding
// gradient, per character on the host side of its loop (namegensf.cu:661-672).
#include <stdexcept>
#include "kernels.h"
#include "common.h"

namespace gk {

typedef __attribute__((address_space(3))) void oh_lds_void;

// LDS reads of the ring through inline asm: hipcc's LDS-DMA alias tracking covers at most 8 DMA
// instructions in flight and, past that, put a vmcnt(0) in front of every ds_read of the ring (the
// 4-deep ring has 15); the reads are ordered by the counted vmcnt + barrier of each k-tile instead,
// and their lgkmcnt is waited for by hand (oh_lgkm_wait ties the results, so no use moves above it)
typedef __attribute__((address_space(3))) const void* oh_lds_cptr;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
DEV u32x4 oh_rd128(const void* p) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"((oh_lds_cptr)p) : "memory");
  return v;
}
DEV int oh_rd32(const void* p) {
  int v;
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"((oh_lds_cptr)p) : "memory");
  return v;
}

template <int N> DEV void oh_vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// wait until the oldest of `ahead + 1` in-flight k-tiles has landed (5 LDS-DMA instructions per wave
// per k-tile; vmcnt retires in order)
template <int A> DEV void oh_wait_ahead(int ahead) {
  if (ahead >= A) { oh_vm_wait<5 * A>(); return; }
  if constexpr (A > 0) oh_wait_ahead<A - 1>(ahead);
}

// NC G rows (columns c of dP) per workgroup, KT tokens per k-tile (2 KT contiguous bytes of each G
// row per fetch); one k-tile = NC x KT bf16 = 16 KiB in every instantiation
template <int NC, int KT> struct OhGeom {
  static_assert(NC * KT == 8192, "16 KiB k-tiles");
  static constexpr int kRowsPerInstr = 512 / KT;   // one wave-instruction: 64 lanes x 16 B = 1 KiB
  static constexpr int kLanesPerRow = KT / 8;
  static constexpr int kIdLanes = KT / 16;         // lanes of a wave's id instruction (KT / 4 ids per wave)
  static constexpr int kSlot = NC * KT + KT * 2;   // u16: the G tile + its KT int32 ids
  static DEV int swz(int r, int c) { return KT == 64 ? c ^ ((r >> 1) & 7) : c ^ (r & 15); }
};

template <int NC, int KT>
__global__ void __launch_bounds__(256, 2) onehot_dp_kernel(GemmArgs a, int ncb, int kper) {
  using Gm = OhGeom<NC, KT>;
  // 4-deep ring, one LDS object per slot (see the header): 4 x ~16.5 KiB, two workgroups per CU
  __shared__ __attribute__((aligned(16))) u16 ring0[Gm::kSlot];
  __shared__ __attribute__((aligned(16))) u16 ring1[Gm::kSlot];
  __shared__ __attribute__((aligned(16))) u16 ring2[Gm::kSlot];
  __shared__ __attribute__((aligned(16))) u16 ring3[Gm::kSlot];
  constexpr int NJ = NC / 16;   // 16-column MFMA tiles per wave
  const int id = blockIdx.x;
  const int cb = id % ncb, sp = id / ncb;
  const int c0 = cb * NC, kbeg = sp * kper, nk = kper / KT;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);   // wave-uniform copy: scalar mask branches
  const int lr = lane & 15, lq = lane >> 4;

  // ---- LDS-DMA staging: wave w, instruction q covers rows (4w + q) * kRowsPerInstr + lane / kLanesPerRow,
  // 16-B chunk slot lane % kLanesPerRow holding the logical chunk swz(row, slot) (conflict-free fragment
  // reads); a fifth instruction (lanes < kIdLanes) brings the wave's quarter of the k-tile's ids
  const int srow = lane / Gm::kLanesPerRow, sslot = lane % Gm::kLanesPerRow;
  const u16* src[4];
  const u16* G = (a.B2 && c0 >= a.b2_row) ? a.B2 : a.B;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = (4 * w + q) * Gm::kRowsPerInstr + srow;
    src[q] = G + (size_t)(c0 + r) * a.ldb + kbeg + Gm::swz(r, sslot) * 8;
  }
  const int* isrc = a.onehot_ids + kbeg + (KT / 4) * w + 4 * (lane % Gm::kIdLanes);
  // (starting each workgroup at its own k-tile, rotated by column block, measured no faster: 64 x 128,
  // 4 K-slices 193.8 -> 200.9 us, profiles/r6_onehot_probe.jsonl; the k order stays the one-hot
  // gemm_lds kernel's, so the two agree bitwise per slab)
  auto stage = [&](u16* slot, int kt) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds(src[q] + kt * KT, (oh_lds_void*)(&slot[(4 * w + q) * Gm::kRowsPerInstr * KT]), 16,
                                       0, 0);
    if (lane < Gm::kIdLanes)
      __builtin_amdgcn_global_load_lds(isrc + kt * KT, (oh_lds_void*)(&slot[NC * KT + (KT / 2) * w]), 16, 0, 0);
  };
#pragma unroll
  for (int s = 0; s < 3; ++s)
    if (s < nk) stage(s == 0 ? ring0 : s == 1 ? ring1 : ring2, s);

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one k-tile from slot R (k-tile kt); k-tile kt + 3 goes into slot N (the one read at kt - 1)
  auto tile = [&](const u16* R, u16* N, int kt) {
    oh_wait_ahead<2>(min(2, nk - 1 - kt));
    // publishes k-tile kt (every wave's DMA share) and proves every wave is done with slot N
    lds_barrier();
    if (kt + 3 < nk) stage(N, kt + 3);
    const int* ids = reinterpret_cast<const int*>(R + NC * KT);
    // the wave's 4 vocabulary tiles that occur among the k-tile's ids (ids outside [0, 256) match no
    // tile and, below, no row)
    int idl[KT / 64];
#pragma unroll
    for (int m = 0; m < KT / 64; ++m) idl[m] = oh_rd32(&ids[lane + 64 * m]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    unsigned mw = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool hit = false;
#pragma unroll
      for (int m = 0; m < KT / 64; ++m) {
        asm volatile("" : "+v"(idl[m]));   // (ordered after the wait above)
        hit |= (unsigned)idl[m] < (unsigned)a.M && (idl[m] >> 4) == 4 * wu + i;
      }
      mw |= __builtin_amdgcn_ballot_w64(hit) ? 1u << i : 0u;
    }
    if (mw == 0) return;   // wave-uniform: no vocabulary row of this wave occurs in the k-tile
#pragma unroll
    for (int ks = 0; ks < KT / 32; ++ks) {
      const int c = ks * 4 + lq;
      u32x4 br[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int r = j * 16 + lr;
        br[j] = oh_rd128(&R[r * KT + Gm::swz(r, c) * 8]);
      }
      u32x4 i0 = oh_rd128(&ids[ks * 32 + lq * 8]), i1 = oh_rd128(&ids[ks * 32 + lq * 8 + 4]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int j = 0; j < NJ; ++j) asm volatile("" : "+v"(br[j]));
      asm volatile("" : "+v"(i0), "+v"(i1));
      const int iv[8] = {(int)i0.x, (int)i0.y, (int)i0.z, (int)i0.w, (int)i1.x, (int)i1.y, (int)i1.z, (int)i1.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (!((mw >> i) & 1u)) continue;
        const int v = (4 * wu + i) * 16 + lr;
        unsigned ow[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) ow[e] = (iv[2 * e] == v ? 0x3F80u : 0u) | (iv[2 * e + 1] == v ? 0x3F800000u : 0u);
        const bf16x8 oh = __builtin_bit_cast(bf16x8, make_uint4(ow[0], ow[1], ow[2], ow[3]));
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(oh, __builtin_bit_cast(bf16x8, br[j]), acc[i][j]);
      }
    }
  };
  for (int kt = 0; kt < nk; kt += 4) {
    tile(ring0, ring3, kt);
    if (kt + 1 < nk) tile(ring1, ring0, kt + 1);
    if (kt + 2 < nk) tile(ring2, ring1, kt + 2);
    if (kt + 3 < nk) tile(ring3, ring2, kt + 3);
  }

  // ---- slab sp: rows v = 16 (4w + i) + 4 lq + e, columns c0 + 16 j + lr
  float* C = a.C + (size_t)sp * a.M * a.ldc;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float* row = C + (size_t)((4 * w + i) * 16 + lq * 4 + e) * a.ldc + c0 + lr;
#pragma unroll
      for (int j = 0; j < NJ; ++j) row[j * 16] = acc[i][j][e];
    }
}

// the instantiation a GemmVariants::onehot value selects: 1 (default) 128 columns x 64-token k-tiles,
// 2 64 x 128, 3 32 x 256.  Standalone at the config-5 shape (805 MB of G, 384 workgroups;
// profiles/r6_onehot_probe.jsonl): 170 / 201 / 246 us against 142 us for a torch row sum over G and
// 349 us for the one-hot gemm_lds kernel -- more rows per k-tile, shorter runs per row, streamed faster
static void oh_geom(int& nc, int& kt) {
  const int v = gemm_variants().onehot;
  nc = v == 2 ? 64 : v == 3 ? 32 : 128;
  kt = 8192 / nc;
}

bool onehot_dp_ok(const GemmArgs& a) {
  int NC, KT;
  oh_geom(NC, KT);
  if (!a.onehot_ids || a.M != 256 || a.N % NC || a.splits < 1 || a.K % a.splits || a.accumulate) return false;
  if (a.bias || a.rowsumA || a.ldc != a.N) return false;
  const int kper = a.K / a.splits;
  if (kper % KT || kper < KT) return false;
  if (a.ldb % 8 || (reinterpret_cast<uintptr_t>(a.B) & 15) || (reinterpret_cast<uintptr_t>(a.onehot_ids) & 15)) return false;
  if (a.B2 && (a.b2_row % NC || (reinterpret_cast<uintptr_t>(a.B2) & 15))) return false;
  return true;
}

// K-slices for an N-column product over K tokens: about 384 workgroups (1.5 per CU, all resident)
int onehot_dp_splits(int N, int K) {
  int NC, KT;
  oh_geom(NC, KT);
  int sp = 1;
  while (sp * 2 * (N / NC) <= 384 && K % (sp * 2 * KT) == 0) sp *= 2;
  return sp;
}

void onehot_dp(const GemmArgs& a, hipStream_t s) {
  if (!onehot_dp_ok(a)) throw std::runtime_error("onehot_dp: unsupported shape (M = 256, N % NC, K-slice % KT)");
  int NC, KT;
  oh_geom(NC, KT);
  const int ncb = a.N / NC, kper = a.K / a.splits;
  dim3 grid(ncb * a.splits), block(256);
  if (NC == 32) hipLaunchKernelGGL((onehot_dp_kernel<32, 256>), grid, block, 0, s, a, ncb, kper);
  else if (NC == 128) hipLaunchKernelGGL((onehot_dp_kernel<128, 64>), grid, block, 0, s, a, ncb, kper);
  else hipLaunchKernelGGL((onehot_dp_kernel<64, 128>), grid, block, 0, s, a, ncb, kper);
}

}  // namespace gk
