// ldpc_kernels.hip -- belief-propagation decode kernels for gfx950 (MI355X).
//
// Hot path of ericdegroot/gr-ldpc_ece535a: the decode call inside
// ldpc_decoder_cb_impl::general_work (lib/ldpc_decoder_cb_impl.cc:155-164).
//
// Mapping ("small code" kernel, N <= 256, E <= 512, dc <= 8, dv <= 4):
//   * one 64-lane wave decodes one frame at a time; 4 independent waves per
//     256-thread workgroup, each with a private LDS slice; a wave leaves its
//     iteration loop on its own syndrome (per-frame early termination exactly
//     as the reference) and pulls the next frame from a launch-wide queue;
//   * lane l owns edges l, l+64, ... (S slots): its variable->check message
//     lives in VGPRs across iterations; the per-iteration exchange goes
//     through LDS (tanh values for the check pass, check->variable messages
//     for the column sums);
//   * every LDS gather is unconditional: unused neighbour entries point at a
//     per-wave dummy element holding the operation's identity (1.0 for the
//     tanh product, DBL_MAX for the min-sum minimum), or their contribution
//     is dropped with a select -- so a lane's loads issue back to back and the
//     wave waits once per phase instead of once per neighbour;
//   * lane l also owns columns l, l+64, ... for the hard decision; the hard
//     decision is a 64-bit wave ballot per 64 columns, the syndrome is
//     popcount(rowmask & hard) per row lane + one more ballot;
//   * per frame the only HBM traffic is its N input samples and its outputs.
// Arithmetic follows the reference operation for operation (same operand
// order, no contraction: built with -ffp-contract=off), in double
// (LDPC_PREC_F64) or float (LDPC_PREC_F32).
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
template <int PREC, int METHOD, int S, int NW, int DCN = kDcMax - 1, int DVN = kDvMax,
          bool FIN = false, typename Real = typename Math<PREC>::Real>
__device__ __forceinline__ void decode_frame(const CodeView &code, const DecodeArgs &a,
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
    const uint32_t fair = a.fair_cycles;  // 0: no issue-priority management
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
          log_ratio_n_packed<S>(Ts, logtab, Es, tb, lane);
        else
          Math<PREC>::template check_msg_n<S>(Ts, logtab, Es);
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
          log_ratio_n_packed<S>(Ts, logtab, Es, tb, lane);
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
  // packed info bits M.., MSB first (:207-219): byte `lane` (KB <= 32)
  if (lane < code.KB) {
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = M + 8 * lane + j;
      const uint32_t p = (ppos[j >> 2] >> (8 * (j & 3))) & 255u;  // position of column c
      if (c < N) o |= (uint32_t)((word_at<NW>(hard, (int)(p >> 6)) >> (p & 63)) & 1) << (7 - j);
    }
    a.packed[b * code.KB + lane] = (uint8_t)o;
  }
  // the next frame's rb writes must not overtake this frame's LDS reads
  wave_lds_sync();
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

// Persistent launch: `a.waves` waves; wave w decodes frame w, then frames
// a.waves + ticket++ until the batch is exhausted.  Frames stop after 1..cap
// iterations, so pulling work keeps every SIMD busy to the end instead of
// leaving it with a fixed share of the batch.
#ifdef LDPC_TIMELINE
// Diagnostic builds only (tools/timeline.py): per frame the 100 MHz realtime
// clock at its start and end and the wave's hardware ids.
constexpr int kTimelineFrames = 65536;
__device__ uint64_t g_timeline[4 * kTimelineFrames];
#endif

#ifndef LDPC_SMALL_MIN_BLOCKS
// occupancy hint: 3 waves per SIMD (for 4-wave workgroups the compiler's
// default, 1, gives the same register budget)
#define LDPC_SMALL_MIN_BLOCKS (kWavesPerBlock >= 4 ? 1 : 12 / kWavesPerBlock)
#endif
// MINB = 4 (four waves per SIMD, <= 128 VGPRs): the throughput build of the
// sum-product f64 kernel (several launches in flight share the CUs); one
// launch at a time runs faster with the larger register budget
// (profiles/round2/layout/ab_min_blocks.txt).
template <int PREC, int METHOD, int S, int NW, int DCN = kDcMax - 1, int DVN = kDvMax,
          int MINB = LDPC_SMALL_MIN_BLOCKS>
__global__ void __launch_bounds__(kThreads, MINB)
    decode_small_kernel(CodeView code, DecodeArgs a) {
  typedef typename Math<PREC>::Real Real;
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int M = code.M;
  typedef Layout<Real, METHOD, S, NW, DVN> LW;
  constexpr SliceLayout L = LW::L;
  __shared__ typename Math<PREC>::Tab logtab[TabLds<PREC>::kN];
  if constexpr (METHOD == 1) stage_tab<PREC>(logtab);

  int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  if (b >= a.waves || b >= a.B) return;

  // the wave's view of the code, in registers
  WaveTables<S, NW> wt;
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

  Real *tb = reinterpret_cast<Real *>(smem + (size_t)wave * LW::per_wave) + L.tb;
  Real *eb = tb + (L.eb - L.tb);
  Real *rb = tb + (L.rb - L.tb);
  Real *sb = tb + (L.sb - L.tb);
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
  int colq[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const uint32_t c = code.lane_col[lane + 64 * q];
    colq[q] = c == kNone ? -1 : (int)c;
  }
  uint32_t ppos[2] = {0u, 0u};
  if (lane < code.KB) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = M + 8 * lane + j;
      if (c < code.N) ppos[j >> 2] |= (uint32_t)code.col_lane[c] << (8 * (j & 3));
    }
  }

#ifndef LDPC_NO_PREFETCH
  // pull the samples of the frames the ticket queue hands out later into L2
  // (one frame per resident wave); the values are consumed by an empty asm
  // after the first frame, when the loads have long completed
  float pf[NW];
  {
    const int64_t pb = (int64_t)a.waves + b;
    float ppol;
    const float *ps = frame_src(a, pb < a.B ? pb : b, ppol);
    (void)ppol;  // the prefetch only pulls the samples into L2
#pragma unroll
    for (int q = 0; q < NW; ++q) pf[q] = colq[q] >= 0 ? ps[(int64_t)colq[q] * a.elem_stride] : 0.0f;
  }
  bool first = true;
#endif
  while (b < a.B) {
#ifdef LDPC_TIMELINE
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const uint64_t c_start = __builtin_amdgcn_s_memtime();
#endif
    // the frame's channel samples, one load per lane and column position
    // (a permutation of the frame's N samples); positions past N are 0
    float xin[NW], pol;
    const float *src = frame_src(a, b, pol);
#pragma unroll
    for (int q = 0; q < NW; ++q)
      xin[q] = colq[q] >= 0 ? src[(int64_t)colq[q] * a.elem_stride] * pol : 0.0f;
    if constexpr (METHOD == 1) {
      bool bad = false;
#pragma unroll
      for (int q = 0; q < NW; ++q) bad |= !__builtin_isfinite(xin[q]);
      if (__ballot(bad) == 0)
        decode_frame<PREC, METHOD, S, NW, DCN, DVN, true>(code, a, b, wt, tb, eb, rb, sb, lane,
                                                           logtab, xin, colq, ppos);
      else
        decode_frame<PREC, METHOD, S, NW, DCN, DVN, false>(code, a, b, wt, tb, eb, rb, sb, lane,
                                                            logtab, xin, colq, ppos);
    } else {
      decode_frame<PREC, METHOD, S, NW, DCN, DVN>(code, a, b, wt, tb, eb, rb, sb, lane, logtab,
                                                  xin, colq, ppos);
    }
#ifndef LDPC_NO_PREFETCH
    if (first) {
#pragma unroll
      for (int q = 0; q < NW; ++q) asm volatile("" ::"v"(pf[q]));
      first = false;
    }
#endif
#ifdef LDPC_TIMELINE
    if (lane == 0 && b < kTimelineFrames) {
      g_timeline[4 * b] = t_start;
      g_timeline[4 * b + 1] = __builtin_amdgcn_s_memrealtime();
      g_timeline[4 * b + 2] = (uint64_t)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) |  // HW_ID
                              ((uint64_t)(uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);  // XCC_ID
      g_timeline[4 * b + 3] = __builtin_amdgcn_s_memtime() - c_start;  // core clocks
    }
#endif
    if (a.static_stride) {
      b += a.waves;
    } else {
      uint32_t t = 0;
      if (lane == 0) t = atomicAdd(a.ticket, 1u) - a.ticket_base;
      b = (int64_t)a.waves + (int64_t)__builtin_amdgcn_readfirstlane((int)t);
    }
  }
}

// ---------------------------------------------------------------------------
// Multi-wave kernel: one frame per S-wave workgroup, one edge per lane.
//
// At small batches the decode time is set by the frames that run to the
// iteration cap, i.e. by one frame's per-iteration latency.  Spreading a
// frame over S waves (on different SIMDs of the CU) divides the edge work of
// an iteration by S; the price is two workgroup barriers per iteration.  The
// cheap column phase (posterior, hard decision, syndrome) is computed by
// every wave redundantly from the shared check messages, so every wave
// reaches the same early-exit decision without a third barrier.
// ---------------------------------------------------------------------------
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

template <int PREC, int METHOD, int S, int NW>
__global__ void __launch_bounds__(64 * S) decode_mw_kernel(CodeView code, DecodeArgs a) {
  typedef typename Math<PREC>::Real Real;
  extern __shared__ __align__(16) unsigned char smem[];
  const MwLayout<Real, S, NW> L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = code.M, N = code.N;
  constexpr int kDummy = 64 * S;
  Real *tb = reinterpret_cast<Real *>(smem);
  Real *eb = reinterpret_cast<Real *>(smem + L.eb);
  Real *rb = reinterpret_cast<Real *>(smem + L.waves + (size_t)wave * L.per_wave);
  Real *sb = rb + 64 * NW;
  int *fslot = reinterpret_cast<int *>(smem + L.fslot);
  __shared__ typename Math<PREC>::Tab logtab[TabLds<PREC>::kN];
  if constexpr (METHOD == 1) stage_tab<PREC>(logtab);
  if (tid == 0) tb[kDummy] = METHOD == 1 ? Real(1) : Math<PREC>::max_();

  // this lane's edge, and (every wave) the columns lane + 64 q
  uint32_t rn[4], cn[2], ce[NW][2];
  {
    const uint4 r = reinterpret_cast<const uint4 *>(code.erow)[tid];
    rn[0] = r.x; rn[1] = r.y; rn[2] = r.z; rn[3] = r.w;
    const uint2 c = reinterpret_cast<const uint2 *>(code.ecol)[tid];
    cn[0] = c.x; cn[1] = c.y;
  }
  uint64_t rowmask[NW][NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const uint4 c = reinterpret_cast<const uint4 *>(code.cols)[lane + 64 * q];
    ce[q][0] = c.x; ce[q][1] = c.y;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int j = lane + 64 * q;
      rowmask[q][k] = j < M ? code.rowmask[j * NW + k] : 0ull;
    }
  }
  int col = field(rn, 7);
  col = col != kNone ? col : 0;
  int colq[NW];  // column at each of the lane's positions (-1: none)
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const uint32_t c = code.lane_col[lane + 64 * q];
    colq[q] = c == kNone ? -1 : (int)c;
  }

  int64_t b = blockIdx.x;
  while (b < a.B) {
    // channel samples, one private copy per wave (:149-153, :486)
    float pol;
    const float *src = frame_src(a, b, pol);
    Real post[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const int c = lane + 64 * q;
      float x = 0.0f;
      if (colq[q] >= 0) x = src[(int64_t)colq[q] * a.elem_stride] * pol;
      rb[c] = -(Real)x;
      post[q] = (Real)x;
    }
    __syncthreads();  // dummy written; previous frame's tb/eb readers done
    uint64_t hard[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) hard[q] = 0;
    int weight = 0, used = 0;
    Real msg = rb[col], lr = Real(0);
    for (int h = 0; h < a.max_iters; ++h) {
      opaque(rn);
      opaque(cn);
      if constexpr (METHOD == 1)
        tb[tid] = Math<PREC>::tanh_half(msg, logtab);  // :509
      else
        tb[tid] = msg;
      __syncthreads();
      Real nb[kDcMax - 1];
#pragma unroll
      for (int k = 0; k < kDcMax - 1; ++k) {
        const int n = field(rn, k);
        nb[k] = tb[n == kNone ? kDummy : n];
      }
      if constexpr (METHOD == 1) {
        Real T = Real(1);  // ascending column; dummies are exact 1.0 (:506-511)
#pragma unroll
        for (int k = 0; k < kDcMax - 1; ++k) T = T * nb[k];
        eb[tid] = Math<PREC>::check_msg(T, logtab);  // :513
      } else {
        const int self = sgn(msg);  // :350-376
        int prod = self;
        Real lo = Math<PREC>::max_();
#pragma unroll
        for (int k = 0; k < kDcMax - 1; ++k) {
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
        opaque(ce[q]);
        const int c = lane + 64 * q;
        Real ev[kDvMax];
#pragma unroll
        for (int k = 0; k < kDvMax; ++k) {
          const int n = field(ce[q], k);
          ev[k] = eb[n == kNone ? kDummy : n];
        }
        const Real rc = rb[c];
        Real acc = Real(0);
        bool bit;
        if constexpr (METHOD == 1) {  // :519-532
#pragma unroll
          for (int k = 0; k < kDvMax; ++k)
            acc = field(ce[q], k) != kNone ? acc + (ev[k] + rc) : acc;
          bit = acc <= Real(0);
          post[q] = acc;
        } else {  // :379-403
#pragma unroll
          for (int k = 0; k < kDvMax; ++k)
            acc = field(ce[q], k) != kNone ? acc + ev[k] : acc;
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
        for (int k = 0; k < NW; ++k) odd ^= __popcll(rowmask[q][k] & hard[k]);
        weight += __popcll(__ballot((odd & 1) != 0 && lane + 64 * q < M));
      }
      used = h + 1;
      if (h + 1 == a.max_iters) break;
      if ((h + 1) % a.et_period == 0 && weight == 0) break;
      if constexpr (METHOD == 1) {  // :540-553
        const Real rc = rb[col];
        Real cv[kDvMax - 1];
#pragma unroll
        for (int k = 0; k < kDvMax - 1; ++k) {
          const int n = field(cn, k);
          cv[k] = eb[n == kNone ? kDummy : n];
        }
        Real acc = Real(0);
#pragma unroll
        for (int k = 0; k < kDvMax - 1; ++k)
          acc = field(cn, k) != kNone ? acc + (cv[k] + rc) : acc;
        msg = acc;
      } else {
        wave_lds_sync();  // this wave's sb
        msg = sb[col] - lr;  // :387-392
      }
    }
    // outputs (wave 0)
    if (wave == 0) {
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
      for (int p = lane; p < code.KB; p += 64) {
        uint32_t o = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = M + 8 * p + j;
          if (c < N) {
            const int x = code.col_lane[c];  // position of column c
            o |= (uint32_t)((word_at<NW>(hard, x >> 6) >> (x & 63)) & 1) << (7 - j);
          }
        }
        a.packed[b * code.KB + p] = (uint8_t)o;
      }
    }
    wave_lds_sync();  // this wave's rb reads done before the next frame's writes
    if (a.static_stride) {
      __syncthreads();
      b += a.waves;
    } else {
      if (tid == 0) *fslot = (int)(atomicAdd(a.ticket, 1u) - a.ticket_base);
      __syncthreads();
      b = (int64_t)a.waves + (int64_t)*fslot;
    }
  }
}

// ---------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------
template <int PREC, int METHOD, int S, int NW, int DCN = kDcMax - 1, int DVN = kDvMax,
          int MINB = LDPC_SMALL_MIN_BLOCKS>
static int launch_one(const CodeView &code, const DecodeArgs &a, hipStream_t st) {
  typedef typename Math<PREC>::Real Real;
  const size_t lds = Layout<Real, METHOD, S, NW, DVN>::total;
  if (lds > 65536 &&
      hipFuncSetAttribute((const void *)decode_small_kernel<PREC, METHOD, S, NW, DCN, DVN, MINB>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -3;
  const dim3 grid((unsigned)((a.waves + kWavesPerBlock - 1) / kWavesPerBlock));
  hipLaunchKernelGGL((decode_small_kernel<PREC, METHOD, S, NW, DCN, DVN, MINB>), grid, dim3(kThreads),
                     lds, st, code, a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int PREC, int METHOD, int S, int NW>
static int launch_mw(const CodeView &code, const DecodeArgs &a, hipStream_t st) {
  typedef typename Math<PREC>::Real Real;
  const size_t lds = MwLayout<Real, S, NW>().total;
  if (lds > 65536 &&
      hipFuncSetAttribute((const void *)decode_mw_kernel<PREC, METHOD, S, NW>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -3;
  hipLaunchKernelGGL((decode_mw_kernel<PREC, METHOD, S, NW>), dim3((unsigned)a.waves),
                     dim3(64 * S), lds, st, code, a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int PREC, int METHOD, int NW>
static int launch_mw_slots(const CodeView &code, const DecodeArgs &a, int slots, hipStream_t st) {
  switch (slots) {
    case 1: return launch_mw<PREC, METHOD, 1, NW>(code, a, st);
    case 2: return launch_mw<PREC, METHOD, 2, NW>(code, a, st);
    case 3: return launch_mw<PREC, METHOD, 3, NW>(code, a, st);
    case 4: return launch_mw<PREC, METHOD, 4, NW>(code, a, st);
    case 5: return launch_mw<PREC, METHOD, 5, NW>(code, a, st);
    case 6: return launch_mw<PREC, METHOD, 6, NW>(code, a, st);
    case 7: return launch_mw<PREC, METHOD, 7, NW>(code, a, st);
    case 8: return launch_mw<PREC, METHOD, 8, NW>(code, a, st);
    default: return -2;
  }
}

#ifndef LDPC_TP_MINB
#define LDPC_TP_MINB 4  // throughput build: waves per SIMD the register budget allows
#endif
template <int PREC, int METHOD, int NW>
static int launch_slots(const CodeView &code, const DecodeArgs &a, int slots, hipStream_t st) {
  // low-degree codes (dc <= 6, dv <= 3: the reference's H) with one column
  // slot get loops sized to their degrees
  if constexpr (NW == 1 && METHOD <= 1) {
    if (code.dc_max <= 6 && code.dv_max <= 3) {
      // throughput mode (no issue-priority management): the 4-waves-per-SIMD build
      if constexpr ((PREC == 0 || PREC == 3) && METHOD == 1)
        if (a.fair_cycles == 0) switch (slots) {
            case 3: return launch_one<PREC, METHOD, 3, NW, 5, 3, LDPC_TP_MINB>(code, a, st);
            case 4: return launch_one<PREC, METHOD, 4, NW, 5, 3, LDPC_TP_MINB>(code, a, st);
            default: break;
          }
      switch (slots) {
        case 1: return launch_one<PREC, METHOD, 1, NW, 5, 3>(code, a, st);
        case 2: return launch_one<PREC, METHOD, 2, NW, 5, 3>(code, a, st);
        case 3: return launch_one<PREC, METHOD, 3, NW, 5, 3>(code, a, st);
        case 4: return launch_one<PREC, METHOD, 4, NW, 5, 3>(code, a, st);
        default: break;
      }
    }
  }
  switch (slots) {
    case 1: return launch_one<PREC, METHOD, 1, NW>(code, a, st);
    case 2: return launch_one<PREC, METHOD, 2, NW>(code, a, st);
    case 3: return launch_one<PREC, METHOD, 3, NW>(code, a, st);
    case 4: return launch_one<PREC, METHOD, 4, NW>(code, a, st);
    case 5: return launch_one<PREC, METHOD, 5, NW>(code, a, st);
    case 6: return launch_one<PREC, METHOD, 6, NW>(code, a, st);
    case 7: return launch_one<PREC, METHOD, 7, NW>(code, a, st);
    case 8: return launch_one<PREC, METHOD, 8, NW>(code, a, st);
    default: return -2;
  }
}

template <int NW>
static int launch_nw(const CodeView &code, const DecodeArgs &a, int method, int prec, int slots,
                     bool mw, hipStream_t st) {
  if (mw && method == 1) {
    if (prec == 1) return launch_mw_slots<1, 1, NW>(code, a, slots, st);
    if (prec == 2) return launch_mw_slots<2, 1, NW>(code, a, slots, st);
    if (prec == 3) return launch_mw_slots<3, 1, NW>(code, a, slots, st);
    return launch_mw_slots<0, 1, NW>(code, a, slots, st);
  }
  if (mw && method == 0)
    return prec == 1 ? launch_mw_slots<1, 0, NW>(code, a, slots, st)
                     : launch_mw_slots<0, 0, NW>(code, a, slots, st);
  if (method == 3) return launch_one<1, 3, 1, NW>(code, a, st);
  if (method == 2) return launch_one<1, 2, 1, NW>(code, a, st);
  if (method == 1) {
    if (prec == 1) return launch_slots<1, 1, NW>(code, a, slots, st);
    if (prec == 2) return launch_slots<2, 1, NW>(code, a, slots, st);
    if (prec == 3) return launch_slots<3, 1, NW>(code, a, slots, st);
    return launch_slots<0, 1, NW>(code, a, slots, st);
  }
  // min-sum has no transcendentals: both f64 modes are the same kernel
  return prec == 1 ? launch_slots<1, 0, NW>(code, a, slots, st)
                   : launch_slots<0, 0, NW>(code, a, slots, st);
}

int launch_decode(const CodeView &code, const DecodeArgs &args, int method, int prec, int slots,
                  int nw, int waves_per_cu, int schedule, void *stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (args.B <= 0) return 0;
  DecodeArgs a = args;
  // CUs of the current device, looked up once per device
  static int cus_of[64] = {0};
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64) {
    if (!cus_of[dev] &&
        hipDeviceGetAttribute(&cus_of[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus_of[dev] = 256;
    cus = cus_of[dev];
  }
#ifndef LDPC_SMALL_WPC
#define LDPC_SMALL_WPC 12
#endif
  if (waves_per_cu <= 0) waves_per_cu = LDPC_SMALL_WPC;
  // schedule: 1 one wave per frame, 2 one workgroup of `slots` waves per
  // frame, 0 auto.  Measured (bench.py --sweep-batch): with round 2's compact
  // arithmetic the one-wave form was as fast as the workgroup form for every
  // method at B = 16..256 and faster from B = 1024 on
  // (profiles/round1/schedules_sweep.txt); with the exact sum-product
  // arithmetic (precision 0 / 2) a frame's iteration is long enough that
  // splitting it over `slots` waves lowers the latency of small launches --
  // 50 iterations of one frame 60.8 vs 88.6 us, B = 256 0.066 vs 0.097 ms --
  // while the one-wave form stays ahead at B = 1024 (0.0995 vs 0.113 ms;
  // profiles/round3/latency_schedules_exact.txt).  Auto therefore takes the
  // workgroup form for exact sum-product launches of <= kMwAutoMax frames
  // (the block's dependent window launches) and the one-wave form otherwise.
  constexpr int kMwAutoMax = 512;
  const bool mw = schedule == 2 || (schedule == 0 && method == 1 && (prec == 0 || prec == 2) &&
                                    a.B <= kMwAutoMax);
  if (mw) {
    const int64_t frames_in_flight = std::max<int64_t>(1, (int64_t)waves_per_cu * cus / slots);
    a.waves = (int)std::min<int64_t>((int64_t)a.B, frames_in_flight);
  } else {
    const int64_t w = std::min<int64_t>((int64_t)a.B, (int64_t)waves_per_cu * cus);
    a.waves = (int)((w + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock);
  }
  if (nw == 1) return launch_nw<1>(code, a, method, prec, slots, mw, st);
  if (nw == 4) return launch_nw<4>(code, a, method, prec, slots, mw, st);
  return -2;
}

}  // namespace ldpc

#ifdef LDPC_TIMELINE
extern "C" int ldpc_debug_timeline(uint64_t *host, int frames) {
  if (frames > ldpc::kTimelineFrames) frames = ldpc::kTimelineFrames;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(ldpc::g_timeline), sizeof(uint64_t) * 4 * frames) ==
                 hipSuccess
             ? frames
             : -1;
}
#endif
