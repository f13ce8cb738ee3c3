// ldpc_frame.hpp -- the small-code frame decoder (one 64-lane wave, one
// frame), shared by the batch kernels (ldpc_kernels.hip) and the block
// walker's decoders (ldpc_walk.hip).  Device code only.
#pragma once

#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>

#include <algorithm>

#include "ldpc_device.hpp"
#include "ldpc_kernels.hpp"
#include "ldpc_layout.hpp"

namespace ldpc {

// LDS hand-off between lanes of ONE wave.  The LDS executes a wave's DS
// instructions in issue order, so a read issued after a write sees it: only
// the compiler must be kept from reordering the accesses -- no s_waitcnt,
// no s_barrier, waves stay independent.  (LDPC_LDS_FENCE restores the
// wavefront-scope fences for A/B checks.)
__device__ __forceinline__ void wave_lds_sync() {
#ifdef LDPC_LDS_FENCE
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#else
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
#endif
}

#ifdef LDPC_PATH_STATS
// Diagnostic builds only (tools/path_stats.py): per wave-iteration of the
// column-centric sum-product loop, how often the exact arithmetic's rare
// paths run and how often every lane's operands are saturated.
//   [0] wave-iterations  [1] some T = +-1 / NaN  [2] every real T in {+-1, NaN, 0}
//   [3] some nonzero |m| outside [2^-54, 13.5) or NaN  [4] every |m| >= 38.2 or NaN
//   [7] some |m| >= 13.5 (expm1's k >= 20 formula)
//   [8] sum of near-1 log operands per wave-iteration  [9] wave-iterations with > 64 of them
//   [10] sum of those with q == 1 exactly  [11] wave-iterations with > 64 without those
//   [5] every check message equal (bitwise) to the previous iteration's
//   [6] [5] and every bit message too (an exact fixed point)
__device__ unsigned long long g_path_stats[12];
#endif

#ifndef LDPC_TANH_SPLIT
#define LDPC_TANH_SPLIT 16.0  // |m| below which the single-range tanh(m/2) is used
#endif

template <int NW>
__device__ __forceinline__ uint64_t word_at(const uint64_t (&w)[NW], int idx) {
  uint64_t r = w[0];
#pragma unroll
  for (int q = 1; q < NW; ++q) r = idx == q ? w[q] : r;
  return r;
}

// Hides a register value from loop-invariant code motion: the unpacked
// neighbour indices are then recomputed (two ALU ops each) inside the
// iteration loop instead of being hoisted and held live (~30 VGPRs).
template <int W>
__device__ __forceinline__ void opaque(uint32_t (&p)[W]) {
#pragma unroll
  for (int k = 0; k < W; ++k) asm volatile("" : "+v"(p[k]));
}

// 16-bit field k of a packed record held in registers
template <int W>
__device__ __forceinline__ int field(const uint32_t (&p)[W], int k) {
  return (int)((p[k >> 1] >> ((k & 1) * 16)) & 0xffffu);
}

// LDS access by absolute byte address (the relocated tables hold addresses,
// so a gather is one field extract + one ds_read).
template <typename T>
__device__ __forceinline__ T lds_ld(uint32_t addr) {
  typedef const __attribute__((address_space(3))) T *lds_ptr;
  return *(lds_ptr)(uintptr_t)addr;
}
template <typename T>
__device__ __forceinline__ void lds_st(uint32_t addr, T v) {
  typedef __attribute__((address_space(3))) T *lds_ptr;
  *(lds_ptr)(uintptr_t)addr = v;
}
template <typename T>
__device__ __forceinline__ uint32_t lds_addr(const T *p) {
  typedef const __attribute__((address_space(3))) T *lds_ptr;
  return (uint32_t)(uintptr_t)(lds_ptr)p;  // generic -> LDS address-space cast
}

// Rewrites the 16-bit edge/column ids of a packed record (fields 0..nf-1)
// as LDS element indices base/size + id (kNone: the dummy element), i.e.
// LDS byte addresses in units of the element size, so they fit 16 bits for
// every slice (a block's LDS can exceed 64 KiB); lds_at() turns a field back
// into a byte address when the record is unpacked, once per frame.
template <int W>
__device__ __forceinline__ void relocate(uint32_t (&p)[W], int nf, uint32_t base, uint32_t size,
                                         uint32_t dummy) {
#pragma unroll
  for (int k = 0; k < 2 * W; ++k) {
    if (k >= nf) break;
    const uint32_t id = (p[k >> 1] >> ((k & 1) * 16)) & 0xffffu;
    const uint32_t ad = base / size + (id == kNone ? dummy : id);
    p[k >> 1] = (p[k >> 1] & ~(0xffffu << ((k & 1) * 16))) | (ad << ((k & 1) * 16));
  }
}
template <typename Real, int W>
__device__ __forceinline__ uint32_t lds_at(const uint32_t (&p)[W], int k) {
  return (uint32_t)field(p, k) * (uint32_t)sizeof(Real);
}

__host__ __device__ constexpr size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

// Sum-product runs column-centric when that computes no more tanh calls than
// the edge form (64 NW DVN <= 64 S; the reference's H: 192 = 192).
template <int METHOD, int S, int NW, int DVN>
__host__ __device__ constexpr bool cols_kernel() {
#ifdef LDPC_NO_COLS
  return false;
#else
  return METHOD == 1 && NW == 1 && DVN <= S;
#endif
}

// Per-wave LDS slice (the workgroup's waves never share LDS), regions as
// SliceLayout (ldpc_layout.hpp), the host's bank model of the same cells:
//   tb[64S] + 32 identity cells   check-pass operand per edge cell
//   eb[64S] + 32 zero cells       check->variable message per edge cell
//   rb[64 NW], sb[64 NW]          -tx / min-sum column totals per column position
//   nr[64S + 64NW]                sum-product: -r of each edge slot's / position's column
//   jk[64 NW]                     column-centric: sink of missing-edge scatters
template <typename Real, int METHOD, int S, int NW, int DVN>
struct Layout {
  static constexpr SliceLayout L{S, NW, cols_kernel<METHOD, S, NW, DVN>()};
  static constexpr size_t per_wave = align16((size_t)L.end * sizeof(Real));
  static constexpr size_t total = (size_t)kWavesPerBlock * per_wave;
};

// identity cell of 32-lane edge group g (CodeView::dpos)
__device__ __forceinline__ uint32_t dpos_of(const CodeView &code, int g) {
  const uint64_t w = g < 8 ? code.dpos[0] : code.dpos[1];
  return (uint32_t)(w >> (8 * (g & 7))) & 31u;
}

// Per-wave register-resident view of the code (packed 16-bit edge ids).
template <int S, int NW>
struct WaveTables {
  uint32_t rn[S][4];   // rn[0..6] of EdgeRowRec, col in the last half-word
  uint32_t cn[S][2];   // cn[0..2] of EdgeColRec, col in the last half-word
  uint32_t ce[NW][2];  // ColRec.e[0..3]
  uint32_t cr[NW][2];  // ColRec.r[0..3] (bit-flip only)
  uint64_t rowmask[NW][NW];  // rows lane + 64 q, words k (M < N <= 64 NW)
};

// DCN / DVN: row neighbours / column entries the loops visit (compile-time
// degree bounds: DCN >= dc_max - 1, DVN >= dv_max); fewer than the record
// sizes for codes of low degree, e.g. the reference's H (dc <= 6, dv <= 3).
// FIN (sum-product): every sample of the frame is finite, so a missing
// neighbour of a column / variable sum can read -r from the lane's own nr
// slot: its term (-r) + r is exactly +0.0 and adding it is an exact no-op
// (the running sum starts at +0.0 and never becomes -0.0) -- no selects.
// Frames with a non-finite sample keep the selects (FIN = false).
// What decode_frame hands back: the syndrome weight (wave-uniform) and, in
// lanes < KB, packed output byte `lane`.  OUT = false: nothing is stored
// (the block walker's decoders publish these themselves, ldpc_walk.hip).
struct FrameResult {
  int weight;
  uint32_t byte;
  int used;  // iterations executed
};
// FAIR = false: a build that never manages issue priority (the throughput
// build: fair_cycles is 0 there), so the clock reads and the state they need
// are compiled out.
template <int PREC, int METHOD, int S, int NW, int DCN = kDcMax - 1, int DVN = kDvMax,
          bool FIN = false, typename Real = typename Math<PREC>::Real, bool OUT = true,
          bool FAIR = true>
__device__ __forceinline__ FrameResult decode_frame(const CodeView &code, const DecodeArgs &a,
                                             const int64_t b, WaveTables<S, NW> &wt,
                                             Real *tb, Real *eb, Real *rb, Real *sb,
                                             const int lane,
                                             const typename Math<PREC>::Tab *logtab,
                                             const float (&xin)[NW], const int (&colq)[NW],
                                             const uint32_t (&ppos)[2]) {
  const int M = code.M, N = code.N;
  // identity cells tb[64S ..+32] and zero cells eb[64S ..+32] (SliceLayout)
  constexpr int kDummy = 64 * S;
  constexpr SliceLayout L = Layout<Real, METHOD, S, NW, DVN>::L;
  // Channel samples xin = tx = Re(in) * polarity (:149-153, loaded by the
  // caller, 0 past N); r = -tx (:486, :318-321).
  Real post[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const int c = lane + 64 * q;
    rb[c] = -(Real)xin[q];
    post[q] = (Real)xin[q];
  }

  uint64_t hard[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) hard[q] = 0;
  int weight = 0, used = 0;
  // lanes holding a real column / row of each 64-wide slot (wave-uniform):
  // ballots of a compare are masked with these instead of folding the range
  // test into the predicate (that form costs two extra VALU per ballot)
  uint64_t col_ok[NW], row_ok[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    col_ok[q] = __ballot(lane + 64 * q < N);
    row_ok[q] = __ballot(lane + 64 * q < M);
  }

  auto syndrome = [&]() {
    int w = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      int odd = 0;
#pragma unroll
      for (int k = 0; k < NW; ++k) odd ^= __popcll(wt.rowmask[q][k] & hard[k]);
      w += __popcll(__builtin_amdgcn_ballot_w64((odd & 1) != 0) & row_ok[q]);
    }
    return w;
  };

  constexpr bool kCols = cols_kernel<METHOD, S, NW, DVN>();
  if constexpr (kCols) {
    // Column-centric sum-product.  A column lane has all of its column's
    // check messages after one gather, so it computes the posterior
    // (:519-532) and, after the exit test, every bit message of its column,
    // M(j,i) = sum_{k != j} (E(k,i) + r(i)) in ascending k from +0.0
    // (:540-553) -- the same additions in the same order as the edge form --
    // and scatters tanh(M(j,i)/2) to the edges' tb slots.  The edge lanes
    // then only gather row neighbours.  Saves the edge form's per-edge
    // column gathers and repeated (E + r) sums.
    // a missing column entry was relocated to this lane's zero cell
    const uint32_t eb_dummy = lds_addr(eb + kDummy + (lane & 31));
    constexpr uint32_t kTbEb = (uint32_t)(L.eb - L.tb) * sizeof(Real);  // eb - tb in bytes
    if (lane < 32) {
      tb[kDummy + lane] = Real(1);  // product identity (missing row neighbours)
      eb[kDummy + lane] = Real(0);  // padding edge cells' row "neighbours": T = 0
    }
    uint32_t ra[S][DCN], ea[NW][DVN], ta[NW][DVN];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int k = 0; k < DCN; ++k) ra[s][k] = lds_at<Real>(wt.rn[s], k);
    Real *nr = sb + 64 * NW;  // FIN: -r of the lane's column (missing edges' term)
#pragma unroll
    for (int q = 0; q < NW; ++q)
#pragma unroll
      for (int k = 0; k < DVN; ++k) {
        const uint32_t e = lds_at<Real>(wt.ce[q], k);
        // missing edges scatter into the lane's own sink cell (no bank conflict)
        ta[q][k] = e == eb_dummy ? lds_addr(tb + L.jk + lane + 64 * q) : e - kTbEb;
        ea[q][k] = (FIN && e == eb_dummy) ? lds_addr(nr + lane + 64 * q) : e;
      }
    Real rc[NW];
    // F64_FAST only: every check operand in tb is a tanh(m/2) with
    // |m| <= LDPC_TANH_SPLIT (so |T| < 1 and finite): the check messages need
    // no saturation select
    bool open = FIN && PREC == 3 && LDPC_TANH_SPLIT > 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      rc[q] = rb[lane + 64 * q];  // written by this lane above
      if constexpr (FIN) nr[lane + 64 * q] = -rc[q];
      // initial bit messages M(j,i) = r(i) (:489-496)
      const Real t0 = Math<PREC>::tanh_half(rc[q], logtab);
      open = open && __builtin_amdgcn_ballot_w64(!(__builtin_fabs((double)rc[q]) <=
                                                    LDPC_TANH_SPLIT)) == 0;
#pragma unroll
      for (int k = 0; k < DVN; ++k) lds_st<Real>(ta[q][k], t0);
    }
#ifdef LDPC_PATH_STATS
    bool st_same = false;
    double st_prev[NW][DVN];
#pragma unroll
    for (int q = 0; q < NW; ++q)
#pragma unroll
      for (int k = 0; k < DVN; ++k) st_prev[q][k] = __builtin_nan("");
#endif
    const uint32_t fair = FAIR ? a.fair_cycles : 0u;  // 0: no issue-priority management
    uint64_t t_prev = fair ? __builtin_amdgcn_s_memtime() : 0;
    for (int h = 0; h < a.max_iters; ++h) {
      // read here, used once the row gathers below have been waited for (an
      // SMEM result needs lgkmcnt(0), which would otherwise also drain the
      // previous iteration's LDS scatters before any gather could issue)
      const uint64_t now = fair ? __builtin_amdgcn_s_memtime() : 0;
      wave_lds_sync();  // tb complete
      Real nb[S][DCN];
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int k = 0; k < DCN; ++k) nb[s][k] = lds_ld<Real>(ra[s][k]);
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int k = 0; k < DCN; ++k) asm volatile("" ::"v"(nb[s][k]));
      // T = prod_{k != i} tanh(M(j,k)/2), ascending k; E = log((1+T)/(1-T))
      // (:506-513).  Padding neighbours read the 1.0 dummy: exact no-op.
      Real Ts[S];
#pragma unroll
      for (int s = 0; s < S; ++s) {
        Real T = Real(1);
#pragma unroll
        for (int k = 0; k < DCN; ++k) T = T * nb[s][k];
        Ts[s] = T;
      }
      if constexpr (PREC != 3) {
        // the S check messages; modes 0 / 2: glibc's log((1+T)/(1-T)) bit for
        // bit, mode 0 with the S quotients from one reciprocal and the near-1
        // logs packed (tb is free once its gathers above have completed --
        // the products below consume them -- until the variable pass)
        Real Es[S];
        if constexpr (PREC == 0)
          log_ratio_n_packed<S>(Ts, logtab, Es, tb, lane, (uint32_t)(L.ebd - L.tb));
        else
          Math<PREC>::template check_msg_n<S>(Ts, logtab, Es);
#ifdef LDPC_PATH_STATS
        if constexpr (PREC == 0) {
          bool some = false, all = true, same = true;
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const double T = (double)Ts[s];
            const bool sat = !(__builtin_fabs(T) < 1.0);
            some |= sat;
            all &= sat || T == 0.0;
            same &= __builtin_bit_cast(uint64_t, (double)Es[s]) ==
                    __builtin_bit_cast(uint64_t, (double)eb[lane + 64 * s]);
          }
          const bool s1 = __ballot(some) != 0, a1 = __ballot(!all) == 0, e1 = __ballot(!same) == 0;
          st_same = e1;
          int nbase = 0, nunit = 0;
#pragma unroll
          for (int s = 0; s < S; ++s) {
            const double T = (double)Ts[s], q = (1.0 + T) / (1.0 - T);
            const bool near = ex::log_is_near1(q);
            nbase += __popcll(__ballot(near));
            nunit += __popcll(__ballot(near && q == 1.0));
          }
          if (lane == 0) {
            atomicAdd(&g_path_stats[8], (unsigned long long)nbase);
            if (nbase > 64) atomicAdd(&g_path_stats[9], 1ull);
            atomicAdd(&g_path_stats[10], (unsigned long long)nunit);
            if (nbase - nunit > 64) atomicAdd(&g_path_stats[11], 1ull);
            atomicAdd(&g_path_stats[0], 1ull);
            if (s1) atomicAdd(&g_path_stats[1], 1ull);
            if (a1) atomicAdd(&g_path_stats[2], 1ull);
            if (e1) atomicAdd(&g_path_stats[5], 1ull);
          }
        }
#endif
#pragma unroll
        for (int s = 0; s < S; ++s) eb[lane + 64 * s] = Es[s];
      } else if constexpr (FIN && LDPC_TANH_SPLIT > 0) {
        if (open) {
#ifdef LDPC_NO_BATCH_DIV
#pragma unroll
          for (int s = 0; s < S; ++s) eb[lane + 64 * s] = fm::log_ratio_tab_open(Ts[s], logtab);
#else
          // the S quotients (1+T)/(1-T) from one reciprocal: every 1 - T > 0
          // here (|T| <= tanh(8) for real edges of rows of degree >= 2; the
          // padding cells read zero "neighbours", T = 0); a code with a
          // degree-1 row (T = 1, the reference's log(2/0) = inf) divides
          // one quotient at a time
          if (code.dc_min >= 2) {
            Real Es[S];
            fm::log_ratio_tab_open_n<S>(Ts, logtab, Es);
#pragma unroll
            for (int s = 0; s < S; ++s) eb[lane + 64 * s] = Es[s];
          } else {
#pragma unroll
            for (int s = 0; s < S; ++s) eb[lane + 64 * s] = fm::log_ratio_tab_open(Ts[s], logtab);
          }
#endif
        } else {
#pragma unroll
          for (int s = 0; s < S; ++s) eb[lane + 64 * s] = Math<PREC>::check_msg(Ts[s], logtab);
        }
      } else {
#pragma unroll
        for (int s = 0; s < S; ++s) eb[lane + 64 * s] = Math<PREC>::check_msg(Ts[s], logtab);
      }
      if (fair) {
        // Issue priority for starved waves (latency mode, one launch at a
        // time).  A SIMD's waves issue oldest first, and two waves already
        // keep its VALU busy, so the third wave of a SIMD crawls (1.7-2 us
        // per iteration against ~1 us) and a long frame it holds ends the
        // batch.  A wave whose last iteration took more than `fair` core
        // clocks issues first for the next one (-2.6 % per launch).  With
        // launches overlapping (throughput mode) the next batch fills those
        // SIMDs instead, and the priority games cost 2.5 % (same-box A/B,
        // profiles/round2/ab_launch_mode.txt).  Scheduling only: the
        // arithmetic is untouched.
        const uint32_t d = (uint32_t)(now - t_prev);
        t_prev = now;
        if (d > fair)
          __builtin_amdgcn_s_setprio(3);
        else
          __builtin_amdgcn_s_setprio(0);
      }
      wave_lds_sync();  // eb complete
      Real tv[NW][DVN];
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        Real ev[DVN];
#pragma unroll
        for (int k = 0; k < DVN; ++k) ev[k] = lds_ld<Real>(ea[q][k]);
        // L = sum_j (E(j,i) + r(i)), ascending j; 1 iff L <= 0 (:519-532)
#pragma unroll
        for (int k = 0; k < DVN; ++k) tv[q][k] = ev[k] + rc[q];
        Real acc = Real(0);
        if constexpr (FIN) {
          // +0.0 + x == x for every x but -0.0, and no term is -0.0 here: a
          // check message is never -0.0 (E = log(1) = +0.0 at T = +-0), so
          // E + r is -0.0 only if both are, and a missing edge's term is
          // exactly +0.0.  The sums start at their first term instead of the
          // reference's 0.0 seed (the same value, one f64 add fewer).
          acc = tv[q][0];
#pragma unroll
          for (int k = 1; k < DVN; ++k) acc = acc + tv[q][k];
        } else {
#pragma unroll
          for (int k = 0; k < DVN; ++k) acc = ea[q][k] != eb_dummy ? acc + tv[q][k] : acc;
        }
        post[q] = acc;
        hard[q] = __builtin_amdgcn_ballot_w64(acc <= Real(0)) & col_ok[q];
      }
      // the next iteration's operands are computed before the exit test (on
      // the last iteration they are dead stores into this wave's tb), so the
      // syndrome's ballot / scalar chain overlaps the tanh arithmetic
      Real mv[NW][DVN];
#pragma unroll
      for (int q = 0; q < NW; ++q)
#pragma unroll
        for (int k = 0; k < DVN; ++k) {
          Real m = Real(0);
          bool first = true;  // FIN: seeded with the first term (see acc above)
#pragma unroll
          for (int k2 = 0; k2 < DVN; ++k2) {
            if (k2 == k) continue;
            if constexpr (FIN)
              m = first ? tv[q][k2] : m + tv[q][k2];
            else
              m = ea[q][k2] != eb_dummy ? m + tv[q][k2] : m;
            first = false;
          }
          mv[q][k] = m;
        }
#ifdef LDPC_PATH_STATS
      if constexpr (PREC == 0) {
        bool some = false, all = true, same = true, big = false;
#pragma unroll
        for (int q = 0; q < NW; ++q)
#pragma unroll
          for (int k = 0; k < DVN; ++k) {
            const double m = (double)mv[q][k], am = __builtin_fabs(m);
            some |= !(am >= 0x1p-54 && am < 13.5) && am != 0.0;
            big |= am >= 13.5;
            all &= !(am < 38.2);
            same &= __builtin_bit_cast(uint64_t, m) == __builtin_bit_cast(uint64_t, st_prev[q][k]);
            st_prev[q][k] = m;
          }
        const bool s1 = __ballot(some) != 0, a1 = __ballot(!all) == 0, e1 = __ballot(!same) == 0;
        const bool b1 = __ballot(big) != 0;
        if (lane == 0) {
          if (s1) atomicAdd(&g_path_stats[3], 1ull);
          if (b1) atomicAdd(&g_path_stats[7], 1ull);
          if (a1) atomicAdd(&g_path_stats[4], 1ull);
          if (e1 && st_same) atomicAdd(&g_path_stats[6], 1ull);
        }
      }
#endif
      if constexpr (PREC != 3) {
        // tanh(m/2), :509: glibc's, bit for bit; mode 0 forms the column's
        // DVN quotients from one reciprocal
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          Real th[DVN];
          Math<PREC>::template tanh_half_n<DVN>(mv[q], th, logtab);
#pragma unroll
          for (int k = 0; k < DVN; ++k) lds_st<Real>(ta[q][k], th[k]);
        }
      } else if constexpr (LDPC_TANH_SPLIT > 0) {
        // F64_FAST: tanh(m/2), :509.  While every |m| of the frame is below the split,
        // the single-range form (no cap, no range selects) is used: its 1-3 ulp
        // near 1 stay below ~1e-9 in the check messages there.  Otherwise the
        // two-range form, glibc's double near 1 (Math<0>::tanh_half).
        bool wide = false;
#pragma unroll
        for (int q = 0; q < NW; ++q)
#pragma unroll
          for (int k = 0; k < DVN; ++k) wide |= !(__builtin_fabs(mv[q][k]) <= LDPC_TANH_SPLIT);
        if (__builtin_amdgcn_ballot_w64(wide) == 0) {
#pragma unroll
          for (int q = 0; q < NW; ++q) {
#ifdef LDPC_NO_BATCH_DIV
#pragma unroll
            for (int k = 0; k < DVN; ++k) lds_st<Real>(ta[q][k], fm::tanh_half_small(mv[q][k]));
#else
            // the column's DVN quotients -t/(t+2) from one reciprocal
            Real th[DVN];
            fm::tanh_half_small_n<DVN>(mv[q], th);
#pragma unroll
            for (int k = 0; k < DVN; ++k) lds_st<Real>(ta[q][k], th[k]);
#endif
          }
          open = FIN;
        } else {
#pragma unroll
          for (int q = 0; q < NW; ++q)
#pragma unroll
            for (int k = 0; k < DVN; ++k) lds_st<Real>(ta[q][k], Math<PREC>::tanh_half(mv[q][k], logtab));
          open = false;
        }
      } else {
#pragma unroll
        for (int q = 0; q < NW; ++q)
#pragma unroll
          for (int k = 0; k < DVN; ++k) lds_st<Real>(ta[q][k], Math<PREC>::tanh_half(mv[q][k], logtab));
      }
      weight = syndrome();
      used = h + 1;
      if (h + 1 == a.max_iters) break;
      if ((h + 1) % a.et_period == 0 && weight == 0) break;
    }
  } else if constexpr (METHOD == 1 || METHOD == 0) {
    // the tables were relocated to LDS byte addresses (decode_small_kernel):
    // rn -> tb, cn / ce -> eb, rn field 7 -> rb (sb = rb + 64 NW elements);
    // missing neighbours point at identity cells tb[64S + ..] (1.0 for the
    // tanh product, DBL_MAX for the minimum) and zero cells eb[64S + ..]
    // (0.0: an exact no-op for the min-sum column sum, whose running value is
    // never -0.0).
    const uint32_t eb_dummy = lds_addr(eb + kDummy + (lane & 31));
    if (lane < 32) {
      tb[kDummy + lane] = METHOD == 1 ? Real(1) : Math<PREC>::max_();
      eb[kDummy + lane] = Real(0);
    }
    // unpacked once per frame into full registers: a gather is then one
    // ds_read with no address arithmetic in the iteration loop
    uint32_t col[S], ra[S][DCN], ca[S][DVN - 1], ea[NW][DVN];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      col[s] = lds_at<Real>(wt.rn[s], 7);
#pragma unroll
      for (int k = 0; k < DCN; ++k) ra[s][k] = lds_at<Real>(wt.rn[s], k);
#pragma unroll
      for (int k = 0; k < DVN - 1; ++k) ca[s][k] = lds_at<Real>(wt.cn[s], k);
    }
#pragma unroll
    for (int q = 0; q < NW; ++q)
#pragma unroll
      for (int k = 0; k < DVN; ++k) ea[q][k] = lds_at<Real>(wt.ce[q], k);
    if constexpr (METHOD == 1 && FIN) {
      Real *nr = sb + 64 * NW;
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int k = 0; k < DVN - 1; ++k)
          ca[s][k] = ca[s][k] == eb_dummy ? lds_addr(nr + lane + 64 * s) : ca[s][k];
#pragma unroll
      for (int q = 0; q < NW; ++q)
#pragma unroll
        for (int k = 0; k < DVN; ++k)
          ea[q][k] = ea[q][k] == eb_dummy ? lds_addr(nr + 64 * S + lane + 64 * q) : ea[q][k];
    }
    constexpr uint32_t kSb = 64 * NW * sizeof(Real);  // sb - rb in bytes
    wave_lds_sync();  // rb and the dummies visible to every lane
    Real msg[S];      // SP: M(j,i) (:489-496); min-sum: L(q_ij) (:328-331)
    Real lr[S];       // min-sum: L(r_ji)
#pragma unroll
    for (int s = 0; s < S; ++s) {
      msg[s] = lds_ld<Real>(col[s]);
      lr[s] = Real(0);
    }
    if constexpr (METHOD == 1 && FIN) {
      Real *nr = sb + 64 * NW;  // read by later gathers of this wave (in order)
#pragma unroll
      for (int s = 0; s < S; ++s) nr[lane + 64 * s] = -msg[s];
#pragma unroll
      for (int q = 0; q < NW; ++q) nr[64 * S + lane + 64 * q] = -rb[lane + 64 * q];
    }

    for (int h = 0; h < a.max_iters; ++h) {
      // ---- check-pass operand of every edge -> LDS ----------------------
      if constexpr (METHOD == 1) {
        Real th[S];
        Math<PREC>::template tanh_half_n<S>(msg, th, logtab);  // :509
#pragma unroll
        for (int s = 0; s < S; ++s) tb[lane + 64 * s] = th[s];
      } else {
#pragma unroll
        for (int s = 0; s < S; ++s) tb[lane + 64 * s] = msg[s];
      }
      wave_lds_sync();
      // gather the row neighbours of every slot (unconditional loads)
      Real nb[S][DCN];
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int k = 0; k < DCN; ++k) nb[s][k] = lds_ld<Real>(ra[s][k]);
      // all of them in flight before the first use (one LDS wait, not three)
#pragma unroll
      for (int s = 0; s < S; ++s)
#pragma unroll
        for (int k = 0; k < DCN; ++k) asm volatile("" ::"v"(nb[s][k]));
      if constexpr (METHOD == 1) {
        // T = prod_{k != i} tanh(M(j,k)/2), ascending k; E = log((1+T)/(1-T))
        // (:506-513).  Padding neighbours read the 1.0 dummy: exact no-op.
        Real Ts[S], Es[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
          Real T = Real(1);
#pragma unroll
          for (int k = 0; k < DCN; ++k) T = T * nb[s][k];
          Ts[s] = T;
        }
        // tb is free from here to the next iteration's tanh stores
        if constexpr (PREC == 0)
          log_ratio_n_packed<S>(Ts, logtab, Es, tb, lane, (uint32_t)(L.ebd - L.tb));
        else
          Math<PREC>::template check_msg_n<S>(Ts, logtab, Es);
#pragma unroll
        for (int s = 0; s < S; ++s) eb[lane + 64 * s] = Es[s];
      }
#pragma unroll
      for (int s = 0; s < S; ++s) {
        if constexpr (METHOD == 0) {
          // min-sum horizontal step (:350-376): L(r) = p * alpha_self * min,
          // p = prod of every alpha of the row (self included), so
          // p * alpha_self = alpha_self^2 * prod_{others} alpha: 0 when any
          // alpha is sign(0) = 0 (NaN too: neither > 0 nor < 0), else the
          // parity of the others' negative signs -- kept as two masks
          // instead of integer products.  min: fmin against a running value
          // that never holds a NaN equals the reference's `beta < min`
          // (a NaN beta never wins).  Padding neighbours read DBL_MAX: sign
          // +1, never below the running minimum.  +0.0 for a zero product,
          // as (double)0 * min.
          bool zero = !(msg[s] > Real(0)) && !(msg[s] < Real(0));
          bool neg = false;
          Real lo = Math<PREC>::max_();
#pragma unroll
          for (int k = 0; k < DCN; ++k) {
            const bool pos = nb[s][k] > Real(0), ng = nb[s][k] < Real(0);
            zero |= !pos && !ng;
            neg ^= ng;
            lo = __builtin_fmin(Math<PREC>::abs_(nb[s][k]), lo);
          }
          lr[s] = zero ? Real(0) : (neg ? -lo : lo);
          eb[lane + 64 * s] = lr[s];
        }
      }
      wave_lds_sync();
      // the variable pass's gathers go out with the column gathers (one
      // wait); they are simply unused when the frame stops here
      Real cv[S][DVN - 1];
      Real rcs[S];
      if constexpr (METHOD == 1) {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          rcs[s] = lds_ld<Real>(col[s]);
#pragma unroll
          for (int k = 0; k < DVN - 1; ++k) cv[s][k] = lds_ld<Real>(ca[s][k]);
        }
      }
      // ---- per-column totals and the hard decision ----------------------
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const int c = lane + 64 * q;
        Real ev[DVN];
#pragma unroll
        for (int k = 0; k < DVN; ++k) ev[k] = lds_ld<Real>(ea[q][k]);
        const Real rc = rb[c];
        Real acc = Real(0);
        bool bit;
        if constexpr (METHOD == 1) {
          // L = sum_j (E(j,i) + r(i)), ascending j; 1 iff L <= 0 (:519-532)
#pragma unroll
          for (int k = 0; k < DVN; ++k) {
            if constexpr (FIN)
              acc = acc + (ev[k] + rc);
            else
              acc = ea[q][k] != eb_dummy ? acc + (ev[k] + rc) : acc;
          }
          bit = acc <= Real(0);
          post[q] = acc;
        } else {
          // s = sum_i L(r_ji) (:380-385); L(Q) = Lci + s; 1 iff L(Q) < 0 (:395-402).
          // Seeded with the first term, not 0.0: an L(r) is never -0.0 (a zero
          // |beta| sets the zero flag, which yields +0.0) and missing edges read
          // +0.0, so 0.0 + x == x for every term.
          acc = ev[0];
#pragma unroll
          for (int k = 1; k < DVN; ++k) acc = acc + ev[k];
          const Real LQ = rc + acc;
          sb[c] = LQ;
          bit = LQ < Real(0);
          post[q] = LQ;
        }
        hard[q] = __builtin_amdgcn_ballot_w64(bit) & col_ok[q];
      }
      if constexpr (METHOD == 1) {
        // keep the variable pass's gathers above the exit test (the compiler
        // would otherwise sink them below it: one more LDS round trip)
#pragma unroll
        for (int s = 0; s < S; ++s) {
          asm volatile("" ::"v"(rcs[s]));
#pragma unroll
          for (int k = 0; k < DVN - 1; ++k) asm volatile("" ::"v"(cv[s][k]));
        }
      }
      // ---- early exit: SP every iteration (:535-537); min-sum only when
      // h+1 < max_iters (:406-408); et_period > 1 thins the checks.
      weight = syndrome();
      used = h + 1;
      if (h + 1 == a.max_iters) break;
      if ((h + 1) % a.et_period == 0 && weight == 0) break;

      if constexpr (METHOD == 1) {
        // ---- bit messages, :540-553: M(j,i) = sum_{k != j} (E(k,i) + r(i))
#pragma unroll
        for (int s = 0; s < S; ++s) {
          Real acc = Real(0);
#pragma unroll
          for (int k = 0; k < DVN - 1; ++k) {
            if constexpr (FIN)
              acc = acc + (cv[s][k] + rcs[s]);
            else
              acc = ca[s][k] != eb_dummy ? acc + (cv[s][k] + rcs[s]) : acc;
          }
          msg[s] = acc;
        }
      } else {
        wave_lds_sync();  // sb visible
        // L(q_ij) = Lci(j) + s_j - L(r_ji)  (:387-392)
#pragma unroll
        for (int s = 0; s < S; ++s) msg[s] = lds_ld<Real>(col[s] + kSb) - lr[s];
      }
    }
  } else {
    // ---- hard decision y = (tx < 0 ? 0 : 1), :424-431 / :563-569 -----
    uint64_t y[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const int c = lane + 64 * q;
      y[q] = __ballot(c < N && !(post[q] < Real(0)));
      hard[q] = y[q];
    }
    weight = syndrome();
    if constexpr (METHOD == 2) {
      // ---- bit flipping, :439-473 ------------------------------------
      const int half = (int)((unsigned)M / 2u);
      for (int h = 0; h < a.max_iters; ++h) {
        // parity of ci over each row; E(i,j) for an edge = parity ^ ci(j)
        uint64_t rowpar[NW];
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          int odd = 0;
#pragma unroll
          for (int k = 0; k < NW; ++k) odd ^= __popcll(wt.rowmask[q][k] & hard[k]);
          rowpar[q] = __ballot((odd & 1) != 0);
        }
        uint64_t next[NW];
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          const int c = lane + 64 * q;
          const int cib = (int)((hard[q] >> lane) & 1);
          const int yb = (int)((y[q] >> lane) & 1);
          int votes = 0;
#pragma unroll
          for (int k = 0; k < kDvMax; ++k) {
            const int r = field(wt.cr[q], k);
            const int par = (int)((word_at<NW>(rowpar, (r >> 6) & (NW - 1)) >> (r & 63)) & 1);
            votes += (r != kNone && (par ^ cib) != yb) ? 1 : 0;
          }
          const bool nb = votes > half ? (yb == 0) : (cib != 0);
          next[q] = __ballot(nb && c < N);
        }
#pragma unroll
        for (int q = 0; q < NW; ++q) hard[q] = next[q];
        weight = syndrome();
        used = h + 1;
        if (h + 1 == a.max_iters) break;
        if ((h + 1) % a.et_period == 0 && weight == 0) break;
      }
    }
  }

  // ---- outputs (hard / post are by lane position; colq = the column) -----
  if constexpr (OUT) {
    if (lane == 0) {
      if (a.iters) a.iters[b] = used;
      if (a.synd) a.synd[b] = weight;
    }
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const int c = colq[q];
      if (c >= 0) {
        if (a.bits) a.bits[b * N + c] = (uint8_t)((hard[q] >> lane) & 1);
        if (a.llr) a.llr[b * N + c] = (float)post[q];
      }
    }
  }
  // packed info bits M.., MSB first (:207-219): byte `lane` (KB <= 32)
  uint32_t o = 0;
  if (lane < code.KB) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = M + 8 * lane + j;
      const uint32_t p = (ppos[j >> 2] >> (8 * (j & 3))) & 255u;  // position of column c
      if (c < N) o |= (uint32_t)((word_at<NW>(hard, (int)(p >> 6)) >> (p & 63)) & 1) << (7 - j);
    }
    if constexpr (OUT) a.packed[b * code.KB + lane] = (uint8_t)o;
  }
  // the next frame's rb writes must not overtake this frame's LDS reads
  wave_lds_sync();
  return FrameResult{weight, o, used};
}

// Frame b's first sample and polarity (DecodeArgs::pm_half: the second half
// of a both-polarities launch re-reads the first half's windows negated).
__device__ __forceinline__ const float *frame_src(const DecodeArgs &a, int64_t b, float &pol) {
  if (a.win) {
    const int64_t w = a.win[b];
    pol = (w & 1) ? -a.polarity : a.polarity;
    return a.in + (w >> 1) * a.elem_stride;
  }
  pol = a.polarity;
  if (a.pm_half > 0 && b >= a.pm_half) {
    b -= a.pm_half;
    pol = -pol;
  }
  return a.in + b * a.cw_stride;
}

// Per-wave setup of the small-code kernels: the code's tables into registers
// (ids relocated to LDS byte addresses of this wave's slice), the slice's
// regions, the column of each of the lane's positions (colq) and the
// positions of the columns of packed byte `lane` (ppos).
template <int PREC, int METHOD, int S, int NW, int DCN, int DVN,
          typename Real = typename Math<PREC>::Real>
__device__ __forceinline__ void wave_setup(const CodeView &code, unsigned char *smem, int wave,
                                           int lane, WaveTables<S, NW> &wt, Real *&tb, Real *&eb,
                                           Real *&rb, Real *&sb, int (&colq)[NW],
                                           uint32_t (&ppos)[2]) {
  const int M = code.M;
  typedef Layout<Real, METHOD, S, NW, DVN> LW;
  constexpr SliceLayout L = LW::L;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const uint4 r = reinterpret_cast<const uint4 *>(code.erow)[lane + 64 * s];
    wt.rn[s][0] = r.x;
    wt.rn[s][1] = r.y;
    wt.rn[s][2] = r.z;
    wt.rn[s][3] = r.w;
    const uint2 c = reinterpret_cast<const uint2 *>(code.ecol)[lane + 64 * s];
    wt.cn[s][0] = c.x;
    wt.cn[s][1] = c.y;
  }
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const uint4 c = reinterpret_cast<const uint4 *>(code.cols)[lane + 64 * q];
    wt.ce[q][0] = c.x;
    wt.ce[q][1] = c.y;
    wt.cr[q][0] = c.z;
    wt.cr[q][1] = c.w;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int j = lane + 64 * q;
      wt.rowmask[q][k] = j < M ? code.rowmask[j * NW + k] : 0ull;
    }
  }

  tb = reinterpret_cast<Real *>(smem + (size_t)wave * LW::per_wave) + L.tb;
  eb = tb + (L.eb - L.tb);
  rb = tb + (L.rb - L.tb);
  sb = tb + (L.sb - L.tb);
  if constexpr (METHOD <= 1) {
    // ids -> LDS byte addresses of this wave's slice (see decode_frame).
    // Missing row neighbours -> the identity cell of the lane's 32-lane group,
    // missing column entries -> the lane's zero cell: banks no other lane of
    // the group reads (ldpc_layout.hpp)
    constexpr uint32_t R = sizeof(Real), kDummy = 64 * S;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint32_t cid = (uint32_t)field(wt.rn[s], 7);
      // padding cells (no edge) read zero cells, so their product T is 0, not 1
      relocate(wt.rn[s], DCN, lds_addr(tb), R,
               cid == kNone ? (uint32_t)(L.ebd - L.tb) + (lane & 31)
                            : kDummy + dpos_of(code, 2 * s + (lane >> 5)));
      const uint32_t ca = lds_addr(rb) / R + (cid == kNone ? (uint32_t)lane : cid);
      wt.rn[s][3] = (wt.rn[s][3] & 0xffffu) | (ca << 16);
      relocate(wt.cn[s], DVN - 1, lds_addr(eb), R, kDummy + (lane & 31));
    }
#pragma unroll
    for (int q = 0; q < NW; ++q) relocate(wt.ce[q], DVN, lds_addr(eb), R, kDummy + (lane & 31));
  }
  // column of each of the lane's positions, and the positions of the
  // columns of packed byte `lane` (8 bits each; N <= 256)
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const uint32_t c = code.lane_col[lane + 64 * q];
    colq[q] = c == kNone ? -1 : (int)c;
  }
  ppos[0] = 0u;
  ppos[1] = 0u;
  if (lane < code.KB) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = M + 8 * lane + j;
      if (c < code.N) ppos[j >> 2] |= (uint32_t)code.col_lane[c] << (8 * (j & 3));
    }
  }
}

// LDS of the workgroup-per-frame kernels (decode_mw_kernel, serve_mw_kernel):
// tb / eb per edge cell, per-wave rb / sb, the frame slot
template <typename Real, int S, int NW>
struct MwLayout {
  size_t eb, waves, per_wave, fslot, total;
  __host__ __device__ MwLayout() {
    eb = align16((64 * S + 2) * sizeof(Real));           // tb at 0
    waves = eb + align16((64 * S + 2) * sizeof(Real));   // per-wave rb, sb
    per_wave = align16(2 * 64 * NW * sizeof(Real));
    fslot = waves + (size_t)S * per_wave;
    total = fslot + 16;
  }
};

// ---------------------------------------------------------------------------
// Workgroup-per-frame form: one frame on S waves, one edge per lane (thread
// tid owns edge cell tid), two workgroup barriers per iteration.  The cheap
// column phase (posterior, hard decision, syndrome) is computed by every wave
// redundantly from the shared check messages, so every wave reaches the same
// early-exit decision without a third barrier.  Used by the batch kernel
// (decode_mw_kernel) and the block's window server (ldpc_serve.hip).
// ---------------------------------------------------------------------------
template <int NW>
struct MwTables {
  uint32_t rn[4], cn[2], ce[NW][2];  // EdgeRowRec / EdgeColRec of edge tid, ColRec.e per position
  uint64_t rowmask[NW][NW];
  int col;                           // the edge's column position (0 for padding)
  int colq[NW];                      // column at each of the lane's positions (-1: none)
};

template <int NW>
__device__ __forceinline__ void mw_setup(const CodeView &code, int tid, MwTables<NW> &t) {
  const int lane = tid & 63, M = code.M;
  const uint4 r = reinterpret_cast<const uint4 *>(code.erow)[tid];
  t.rn[0] = r.x;
  t.rn[1] = r.y;
  t.rn[2] = r.z;
  t.rn[3] = r.w;
  const uint2 c = reinterpret_cast<const uint2 *>(code.ecol)[tid];
  t.cn[0] = c.x;
  t.cn[1] = c.y;
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const uint4 cc = reinterpret_cast<const uint4 *>(code.cols)[lane + 64 * q];
    t.ce[q][0] = cc.x;
    t.ce[q][1] = cc.y;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int j = lane + 64 * q;
      t.rowmask[q][k] = j < M ? code.rowmask[j * NW + k] : 0ull;
    }
  }
  const int cl = field(t.rn, 7);
  t.col = cl != kNone ? cl : 0;
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const uint32_t cq = code.lane_col[lane + 64 * q];
    t.colq[q] = cq == kNone ? -1 : (int)cq;
  }
}

// One frame: samples src[colq] * pol.  DCN / DVN: row neighbours / column
// entries the loops visit (>= dc_max - 1 / dv_max; the records' unused
// fields are kNone).  Leaves the hard decisions (by lane
// position) and posteriors in every wave; returns the syndrome weight and
// the iterations used.  Starts with a workgroup barrier (the caller's LDS
// reads of the previous frame must be done when it is entered: every caller
// ends a frame with __syncthreads).  tb[64 S] must hold the identity.
template <int PREC, int METHOD, int S, int NW, int DCN = kDcMax - 1, int DVN = kDvMax,
          typename Real = typename Math<PREC>::Real>
__device__ __forceinline__ int mw_frame(const CodeView &code, int max_iters, int et_period,
                                        MwTables<NW> &t, Real *tb, Real *eb, Real *rb, Real *sb,
                                        const typename Math<PREC>::Tab *logtab, const float *src,
                                        float pol, int elem_stride, uint64_t (&hard)[NW],
                                        Real (&post)[NW], int &used) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int M = code.M, N = code.N;
  constexpr int kDummy = 64 * S;
  // channel samples, one private copy per wave (:149-153, :486)
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const int c = lane + 64 * q;
    float x = 0.0f;
    if (t.colq[q] >= 0) x = src[(int64_t)t.colq[q] * elem_stride] * pol;
    rb[c] = -(Real)x;
    post[q] = (Real)x;
  }
  __syncthreads();  // dummy written; previous frame's tb/eb readers done
#pragma unroll
  for (int q = 0; q < NW; ++q) hard[q] = 0;
  int weight = 0;
  used = 0;
  Real msg = rb[t.col], lr = Real(0);
  for (int h = 0; h < max_iters; ++h) {
    opaque(t.rn);
    opaque(t.cn);
    if constexpr (METHOD == 1)
      tb[tid] = Math<PREC>::tanh_half(msg, logtab);  // :509
    else
      tb[tid] = msg;
    __syncthreads();
    Real nb[DCN];
#pragma unroll
    for (int k = 0; k < DCN; ++k) {
      const int n = field(t.rn, k);
      nb[k] = tb[n == kNone ? kDummy : n];
    }
    if constexpr (METHOD == 1) {
      Real T = Real(1);  // ascending column; dummies are exact 1.0 (:506-511)
#pragma unroll
      for (int k = 0; k < DCN; ++k) T = T * nb[k];
      eb[tid] = Math<PREC>::check_msg(T, logtab);  // :513
    } else {
      const int self = sgn(msg);  // :350-376
      int prod = self;
      Real lo = Math<PREC>::max_();
#pragma unroll
      for (int k = 0; k < DCN; ++k) {
        prod *= sgn(nb[k]);
        const Real beta = Math<PREC>::abs_(nb[k]);
        lo = beta < lo ? beta : lo;
      }
      lr = (Real)(prod * self) * lo;
      eb[tid] = lr;
    }
    __syncthreads();
    // column phase, identical in every wave
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      opaque(t.ce[q]);
      const int c = lane + 64 * q;
      Real ev[DVN];
#pragma unroll
      for (int k = 0; k < DVN; ++k) {
        const int n = field(t.ce[q], k);
        ev[k] = eb[n == kNone ? kDummy : n];
      }
      const Real rc = rb[c];
      Real acc = Real(0);
      bool bit;
      if constexpr (METHOD == 1) {  // :519-532
#pragma unroll
        for (int k = 0; k < DVN; ++k)
          acc = field(t.ce[q], k) != kNone ? acc + (ev[k] + rc) : acc;
        bit = acc <= Real(0);
        post[q] = acc;
      } else {  // :379-403
#pragma unroll
        for (int k = 0; k < DVN; ++k)
          acc = field(t.ce[q], k) != kNone ? acc + ev[k] : acc;
        const Real LQ = rc + acc;
        sb[c] = LQ;
        bit = LQ < Real(0);
        post[q] = LQ;
      }
      hard[q] = __ballot(bit && c < N);
    }
    weight = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      int odd = 0;
#pragma unroll
      for (int k = 0; k < NW; ++k) odd ^= __popcll(t.rowmask[q][k] & hard[k]);
      weight += __popcll(__ballot((odd & 1) != 0 && lane + 64 * q < M));
    }
    used = h + 1;
    if (h + 1 == max_iters) break;
    if ((h + 1) % et_period == 0 && weight == 0) break;
    if constexpr (METHOD == 1) {  // :540-553
      const Real rc = rb[t.col];
      Real cv[DVN - 1];
#pragma unroll
      for (int k = 0; k < DVN - 1; ++k) {
        const int n = field(t.cn, k);
        cv[k] = eb[n == kNone ? kDummy : n];
      }
      Real acc = Real(0);
#pragma unroll
      for (int k = 0; k < DVN - 1; ++k)
        acc = field(t.cn, k) != kNone ? acc + (cv[k] + rc) : acc;
      msg = acc;
    } else {
      wave_lds_sync();  // this wave's sb
      msg = sb[t.col] - lr;  // :387-392
    }
  }
  return weight;
}

// packed info byte `lane` (lanes < KB) of a frame's hard decisions (:207-219)
template <int NW>
__device__ __forceinline__ uint32_t mw_packed_byte(const CodeView &code, const uint64_t (&hard)[NW],
                                                   int lane) {
  uint32_t o = 0;
  if (lane < code.KB) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = code.M + 8 * lane + j;
      if (c < code.N) {
        const int x = code.col_lane[c];  // position of column c
        o |= (uint32_t)((word_at<NW>(hard, x >> 6) >> (x & 63)) & 1) << (7 - j);
      }
    }
  }
  return o;
}

}  // namespace ldpc
