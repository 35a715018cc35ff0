// Cross-workgroup hand-off machinery of the persistent sequence kernels (gru_seq.hip, gru_seq16.hip):
// buffer-resource loads / stores with the sc1 bit, wall-clock-bounded spins, per-producer epoch
// flags with per-wave streaming waits, the XCD placement census that picks the L2-local protocol.
// (Protocol: cdna_hip_programming.md §6 Guideline 16, MI355X_MICROARCH.md 'Valid forms' row 1.)
#pragma once
#include "kernels.h"
#include "mma_tile.h"

namespace gk {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

DEV rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
DEV bf16x8 ld8_sc1(rsrc_t r, unsigned off) {
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);   // aux 16 = sc1
  return __builtin_bit_cast(bf16x8, v);
}
DEV void st16_sc1(rsrc_t r, unsigned off, u32x4 v) { __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16); }
// sc1 load with a per-lane offset and a wave-uniform scalar offset: the address math of an
// unrolled k-loop then needs no VGPR temporaries (in the streaming wait, temporaries that alias a
// pending load's destination made the compiler drain vmcnt before every k-step's load)
DEV bf16x8 ld8_sc1s(rsrc_t r, unsigned voff, int soff) {
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 16);
  return __builtin_bit_cast(bf16x8, v);
}

// plain (cached) buffer load, per-lane VGPR offset + wave-uniform scalar offset: read-only operands
DEV bf16x8 ld8_plain_s(rsrc_t r, unsigned voff, int soff) {
  u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  return __builtin_bit_cast(bf16x8, v);
}

// Every cross-workgroup wait is bounded by WALL CLOCK, not by a poll count: workgroups that start
// late because something else holds their CUs (an RCCL kernel of a data-parallel step waiting for a
// slow peer, another process's kernel) delay the wait without tripping it.  5 s of the 100 MHz
// s_memrealtime counter, checked every 64 polls; past it the wait sets bit 1 of the error word and
// gives up (the step's update is skipped on every rank and the watchdog reports it).  Bit 1 is also
// the give-up signal: every later wait of the launch (any workgroup) sees it at its next check and
// returns at once, so a grid that is truly not co-resident drains in one budget, not one per wait.
static constexpr unsigned long long kSpinTicks = 500000000ull;
// s_sleep argument between flag polls (x 64 clocks)
#ifndef GK_POLL_SLEEP
#define GK_POLL_SLEEP 1
#endif
struct SpinBudget {
  const unsigned* err;
  unsigned long long t0 = 0;
  unsigned n = 0;
  DEV explicit SpinBudget(const unsigned* e) : err(e) {}
  // The first check only reads the clock: an error-word load there sits in the poll loop of EVERY
  // wait (a memory round trip before the second poll) -- round 4 measured it at +6 us on the h512
  // backward and +2.5 us on the forward.  From the second check on (64 polls in) it also reads bit 1.
  DEV bool expired() {
    if ((n++ & 63u) != 0u) return false;
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    if (!t0) { t0 = now; return false; }
    if (err && (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1u)) return true;
    return now - t0 > kSpinTicks;
  }
};

// Per-producer epoch flags: producer p of a row block owns flags[p * kFlagStride] (its own 64-B
// line, no read-modify-write contention); after its payload drained it stores the epoch with a
// relaxed agent-scope (sc1) store.  The consumer's wave 0 sweeps all producers' flags -- lane p
// reads flag p with an sc1 load -- until every one has reached the epoch (wave vote), then the
// workgroup barrier releases the other waves.  A single shared counter instead measured ~6.7 us
// per hop (32 atomic adders + 256 pollers on one line; scripts/probe_seq.py).
static constexpr int kFlagStride = 16;   // uints (64 B)

DEV void wait_flags(const unsigned* flags, int nprod, unsigned epoch, unsigned* err) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    SpinBudget spin(err);
    for (;;) {
      bool ok = true;
      if (lane < nprod) ok = __hip_atomic_load(flags + lane * kFlagStride, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT) >= epoch;
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(GK_POLL_SLEEP);
      if (spin.expired()) {
        if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}
// Wave-level variant: a wave's K-slice of the recurrent GEMM only reads the columns produced by
// a few unit-tile workgroups, so each wave waits for exactly those (lane p polls producer
// prod_p) and proceeds on its own -- no workgroup barrier, no coupling to the slowest of all
// H/16 producers.  The acquire-at-wavefront fence only pins the following sc1 loads below
// the poll (no instruction is emitted).
DEV void wave_wait(const unsigned* flags, bool active, int prod, unsigned epoch, unsigned* err) {
  SpinBudget spin(err);
  for (;;) {
    bool ok = true;
    if (active) ok = __hip_atomic_load(flags + prod * kFlagStride, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT) >= epoch;
    if (__all(ok)) break;
    __builtin_amdgcn_s_sleep(GK_POLL_SLEEP);
    if (spin.expired()) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// (Round 5, measured and removed: two flag polls in flight -- the next issued before the previous
// is examined -- in the one-layer forward: 0.2020-0.2029 -> 0.2051-0.2052 ms/step on the same box,
// profiles/r5_poll2_ab.txt; in the persistent generator likewise slower.  Each flag line is polled
// by every consumer workgroup of its row block; doubling that traffic delays the producer's own
// flag store more than it shortens detection.)
// Streaming variant: lane p polls producer p; k-step kk reads the columns of producers 2kk and
// 2kk+1, and its payload loads (loadk(kk): sc1 loads into registers) are issued as soon as BOTH
// have published -- the early producers' data is in flight while the wave still waits for the
// late ones.  The MFMAs run afterwards in fixed k order, so results stay deterministic.  Every
// load follows, in this wave, a poll that saw its producers' flags (R1 hand-off, no acquire).
template <int NK, class LoadK>
DEV void wave_wait_load(const unsigned* flags, bool active, int prod, unsigned epoch, unsigned* err,
                        LoadK&& loadk) {
  constexpr unsigned all = (1u << NK) - 1u;
  unsigned loaded = 0;
  SpinBudget spin(err);
  for (;;) {
    bool ok = true;
    if (active) ok = __hip_atomic_load(flags + prod * kFlagStride, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT) >= epoch;
    const unsigned long long m = __ballot(ok);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the loads below the poll
#pragma unroll
    for (int kk = 0; kk < NK; ++kk)
      if (!((loaded >> kk) & 1u) && ((m >> (2 * kk)) & 3ull) == 3ull) {
        loadk(kk);
        loaded |= 1u << kk;
      }
    if (loaded == all) break;
    __builtin_amdgcn_s_sleep(GK_POLL_SLEEP);
    if (spin.expired()) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int kk = 0; kk < NK; ++kk)
        if (!((loaded >> kk) & 1u)) loadk(kk);   // garbage, flagged: keep the grid draining
      break;
    }
  }
}
// One producer per k-step (the 16-row backward of gru_seq16.hip, whose producers own 32 units):
// lane kk polls producer prod_kk, k-step kk is loaded as soon as its producer published.
template <int NK, class LoadK>
DEV void wave_wait_load1(const unsigned* flags, bool active, int prod, unsigned epoch, unsigned* err,
                         LoadK&& loadk) {
  constexpr unsigned all = (1u << NK) - 1u;
  unsigned loaded = 0;
  SpinBudget spin(err);
  for (;;) {
    bool ok = true;
    if (active) ok = __hip_atomic_load(flags + prod * kFlagStride, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT) >= epoch;
    const unsigned long long m = __ballot(ok);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the loads below the poll
#pragma unroll
    for (int kk = 0; kk < NK; ++kk)
      if (!((loaded >> kk) & 1u) && ((m >> kk) & 1ull)) {
        loadk(kk);
        loaded |= 1u << kk;
      }
    if (loaded == all) break;
    __builtin_amdgcn_s_sleep(GK_POLL_SLEEP);
    if (spin.expired()) {
      if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int kk = 0; kk < NK; ++kk)
        if (!((loaded >> kk) & 1u)) loadk(kk);   // garbage, flagged: keep the grid draining
      break;
    }
  }
}
// Two exchange streams at once (the wavefront forward's h_lo and h_hi): lanes [0, 2NK) poll
// stream a's producers prod0.., lanes [32, 32 + 2NK) stream b's; k-step kk of a stream is loaded
// as soon as both of its producers published.  One poll round trip serves both streams.
template <int NK, class LA, class LB>
DEV void wave_wait_load2(const unsigned* fa, const unsigned* fb, int prod0, unsigned ea, unsigned eb,
                         unsigned* err, LA&& loada, LB&& loadb) {
  static_assert(2 * NK <= 32, "one half-wave of pollers per stream");
  constexpr unsigned all = (1u << NK) - 1u;
  const int lane = threadIdx.x & 63;
  const bool active = (lane & 31) < 2 * NK;
  const unsigned* f = (lane < 32 ? fa : fb) + (size_t)(prod0 + (lane & 31)) * kFlagStride;
  const unsigned ep = lane < 32 ? ea : eb;
  unsigned da = 0, db = 0;
  SpinBudget spin(err);
  for (;;) {
    bool ok = true;
    if (active) ok = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= ep;
    const unsigned long long m = __ballot(ok);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the loads below the poll
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      if (!((da >> kk) & 1u) && ((m >> (2 * kk)) & 3ull) == 3ull) {
        loada(kk);
        da |= 1u << kk;
      }
      if (!((db >> kk) & 1u) && ((m >> (32 + 2 * kk)) & 3ull) == 3ull) {
        loadb(kk);
        db |= 1u << kk;
      }
    }
    if (da == all && db == all) break;
    __builtin_amdgcn_s_sleep(GK_POLL_SLEEP);
    if (spin.expired()) {
      if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {   // garbage, flagged: keep the grid draining
        if (!((da >> kk) & 1u)) loada(kk);
        if (!((db >> kk) & 1u)) loadb(kk);
      }
      break;
    }
  }
}
DEV void signal_flag(unsigned* flag, unsigned epoch) {
  __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Zero the flag block of the sequence kernel that runs NEXT on the stream (it cannot start
// before this launch completes, so plain stores + the kernel boundary order it) -- replaces a
// memset graph node per step.
DEV void zero_next_flags(unsigned* p, long n) {
  if (!p) return;
  const long wg = blockIdx.x, nwg = gridDim.x;
  for (long i = wg * blockDim.x + threadIdx.x; i < n; i += nwg * blockDim.x) p[i] = 0u;
}

// Diagnostic phase stamps (100 MHz wall clock) for the first and last workgroup, thread 0 only.
// Only written when the caller passes a dbg buffer; nothing reads them inside the kernel.
DEV void stamp(unsigned long long* dbg, int t, int k) {
  if (!dbg || threadIdx.x != 0) return;
  const bool first = blockIdx.x == 0;
  const bool last = blockIdx.x == gridDim.x - 1;
  if (!first && !last) return;
  const unsigned long long v = __builtin_amdgcn_s_memrealtime();
  dbg[((last ? 1 : 0) * 4096 + t) * 8 + k] = v;
}

// Workgroup -> (unit tile, row block).  With Bp/32 a multiple of 8 the row block is the fast index
// (block b -> row block b % nrb), so under the dispatcher's observed round-robin placement all unit
// tiles of a row block share one XCD and its L2 (MI355X_MICROARCH.md § placement; a speed choice:
// row_block_local() below checks the placement at run time and picks the protocol from it).
DEV bool seq_rb_fast(int nrb) { return nrb % 8 == 0; }
DEV int seq_unit_tile(int nrb) {
  return seq_rb_fast(nrb) ? (int)(blockIdx.x / nrb) : (int)(blockIdx.x % (gridDim.x / nrb));
}
DEV int seq_row_block(int nrb) {
  return seq_rb_fast(nrb) ? (int)(blockIdx.x % nrb) : (int)(blockIdx.x / (gridDim.x / nrb));
}
// the same map over the first nblk blocks of a larger grid (the recurrence part of gru_fwd_seq_fc)
DEV int seq_unit_tile_n(int nrb, int nblk) {
  return seq_rb_fast(nrb) ? (int)(blockIdx.x / nrb) : (int)(blockIdx.x % (nblk / nrb));
}
DEV int seq_row_block_n(int nrb, int nblk) {
  return seq_rb_fast(nrb) ? (int)(blockIdx.x % nrb) : (int)(blockIdx.x / (nblk / nrb));
}

// Exchange protocol per row block, decided once per launch from where its workgroups actually
// run: each workgroup publishes its XCC id (HW_REG_XCC_ID + 1, agent-scope sc1 store) in word 1
// of its own flag line and reads every producer's word of its row block.  All on one XCD ->
// L2-local hand-off: payload and flag are PLAIN stores (they stay in the shared L2; the producer's
// vmcnt(0) covers them), consumers keep their L1-bypassing sc1 loads, served by that L2.  Any
// producer elsewhere -> the placement-independent write-through (sc1) protocol.  Every member of
// the row block evaluates the same words, so all agree.  The flag block is zeroed before the launch.
DEV bool row_block_local(unsigned* flags /* the row block's producer lines */, int ut, int nunit,
                         unsigned* err) {
  __shared__ int s_local;
  unsigned id;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
  if (threadIdx.x == 0)
    __hip_atomic_store(flags + ut * kFlagStride + 1, id + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    unsigned v = id + 1u;
    SpinBudget spin(err);
    for (;;) {
      if (lane < nunit) v = __hip_atomic_load(flags + lane * kFlagStride + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__all(v != 0u)) break;
      __builtin_amdgcn_s_sleep(GK_POLL_SLEEP);
      if (spin.expired()) {
        if (lane == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    const bool loc = __all(v == id + 1u);
    if (lane == 0) s_local = loc ? 1 : 0;
  }
  __syncthreads();
  return s_local != 0;
}
DEV void st16_plain(rsrc_t r, unsigned off, u32x4 v) { __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0); }
DEV void signal_flag_local(unsigned* flag, unsigned epoch) {
  __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);   // plain store: stays in L2
}

}  // namespace gk
