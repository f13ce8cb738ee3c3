// ldpc_graph_msn.hip -- large-code min-sum with the
// gathered state kept in one XCD's L2.
//
// The reference's horizontal and vertical steps (lib/ldpc_decoder_cb_impl.cc:
// 340-403) with a row's L(r) recovered exactly from {m1, m2, i1, P} and a
// 2-bit alpha per edge (the compressed messages of the round-2 64-frame
// pipeline, retired in round 4), laid out for the cache hierarchy:
//
// * Narrow chunks.  A chunk holds F = kF frames (2 since round 4; element x
//   of frame f at (k * n + x) * F + f), so the tables a pass gathers from --
//   LQ in the check pass (8 N F bytes = 1.05 MB for N = 64800 at F = 2), the
//   row state {m1, m2, meta} in the variable pass (17 M F = 1.1 MB) -- fit
//   one XCD's 4 MiB L2.  With 64-frame chunks they were 33-35 MB, every
//   gather went to the Infinity Cache (~8 TB/s) and the passes moved 8.4 MB
//   per frame-iteration.
// * XCD-aware placement.  Workgroup b runs on XCD b mod 8; chunk k's blocks
//   are the ones with b mod 8 == k mod 8, in chunk order, so each XCD works
//   through its chunks one after another and a chunk's table is gathered
//   by the CUs whose L2 holds it.
// * Storage order.  Rows and columns are stored in an order chosen on the
//   host (ldpc_msn_build): for codes with the DVB-S2 structure (IRA, 360-
//   column groups, row r = x + s q mod M) rows by residue class mod q, which
//   makes every circulant a shifted identity, so the 64 rows of a wave read
//   (runs of) consecutive columns for each of their edges and the 64 columns
//   of a wave read consecutive rows.  The arithmetic still visits a row's edges in ascending
//   original column and a column's edges in ascending original row (the
//   reference's scan order); the order only moves where values are stored.
// * One row (column) per lane, 64 per wave, 256 per block; the chunk's F
//   frames sit in the lane as one vector (Vec).  The
//   decisions are the signs of LQ (vhat = LQ < 0, :398-402), so the check
//   pass forms the parities of the last decisions from the LQ values it
//   gathers anyway (no separate hard-decision array), and outputs (packed
//   bytes, bits, posteriors = (float) LQ) are read from LQ when a frame stops.
// * The uncapped syndrome weight of a frame stopped at the cap is counted by
//   the check pass of its last pass (atomic adds per wave, only at the cap).
//
// Per pass: msn_check (the chunk's stop / refill decision taken by the block
// that completes the chunk) -> msn_var (outputs of the stopped frames, the vertical
// step, refills); separate msn_post / msn_cols launches for the outputs only
// for codes outside that fast path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <vector>

#include <stdio.h>
#include <stdlib.h>

#include "ldpc_device.hpp"
#include "ldpc_graph.hpp"

namespace ldpc {
namespace {

constexpr int kF = kMsnFrames;  // frames per chunk
constexpr int kIB = 256;        // rows / columns per 256-thread block (one per lane)
static_assert(kF == 2 || kF == 4, "frames per chunk: 2 or 4");

// Workgroup b -> (chunk, block of the chunk).  With a multiple of 8 chunks,
// chunk k's blocks run on XCD k mod 8 (the dispatcher deals workgroups to the
// XCDs round robin), the XCD's chunks one after another.
// rev: the XCD's chunks in the opposite order.  The variable pass runs them
// backwards and the check pass forwards (a zigzag): each launch starts on the
// chunks whose gathered table -- the row state the check pass just wrote, the
// LQ the variable pass just wrote -- the previous launch wrote last, while it
// is still in the XCD's L2.
__device__ __forceinline__ void map_block(int b, int chunks, int nbpc, int &k, int &bi,
                                          bool rev = false) {
  if ((chunks & 7) == 0) {
    const int idx = b >> 3;
    int c = idx / nbpc;
    bi = idx - c * nbpc;
    if (rev) c = (chunks >> 3) - 1 - c;
    k = (b & 7) + 8 * c;
  } else {
    k = b / nbpc;
    bi = b - k * nbpc;
  }
}

__device__ __forceinline__ int64_t el(int k, int n, int x) { return ((int64_t)k * n + x) * kF; }

// F consecutive values (one vector load / store)
template <typename Real>
struct Vec {
  Real v[kF];
};
template <typename Real>
__device__ __forceinline__ Vec<Real> ldv(const Real *p) {
  return *(const Vec<Real> *)p;
}
template <typename Real>
__device__ __forceinline__ void stv(Real *p, const Vec<Real> &x) {
  *(Vec<Real> *)p = x;
}
// The same, non-temporal, for the state a pass streams once (row state in the
// check pass, L and LQ in the variable pass) -- meant to keep the gathered
// table and the edge tables in L2.  Measured slower (config 4: 1 973 vs
// 2 212 Mbit/s, profiles/round3/msn/ab_nt.txt), so off unless built with
// -DLDPC_MSN_NT=1.
#ifndef LDPC_MSN_NT
#define LDPC_MSN_NT 0
#endif
template <typename Real>
__device__ __forceinline__ Vec<Real> ldv_nt(const Real *p) {
#if LDPC_MSN_NT
  typedef Real V __attribute__((ext_vector_type(kF)));
  const V v = __builtin_nontemporal_load((const V *)p);
  Vec<Real> r;
#pragma unroll
  for (int j = 0; j < kF; ++j) r.v[j] = v[j];
  return r;
#else
  return ldv(p);
#endif
}
template <typename Real>
__device__ __forceinline__ void stv_nt(Real *p, const Vec<Real> &x) {
#if LDPC_MSN_NT
  typedef Real V __attribute__((ext_vector_type(kF)));
  V v;
#pragma unroll
  for (int j = 0; j < kF; ++j) v[j] = x.v[j];
  __builtin_nontemporal_store(v, (V *)p);
#else
  stv(p, x);
#endif
}
typedef uint32_t MetaWord;  // F meta bytes (F <= 4)
__device__ __forceinline__ MetaWord ld_meta(const uint8_t *p) {
  if constexpr (kF == 4) return *(const uint32_t *)p;
  else return *(const uint16_t *)p;
}
__device__ __forceinline__ void st_meta(uint8_t *p, MetaWord m) {
  if constexpr (kF == 4) *(uint32_t *)p = m;
  else *(uint16_t *)p = (uint16_t)m;
}

// alpha of an edge for frame f from the chunk's byte: bit 2f L(q) < 0, bit
// 2f+1 sign 0 (:338, sign(0) = sign(NaN) = 0)
// With 2 frames per chunk an edge's alpha bits take a nibble: slots 2u and
// 2u + 1 of a row share byte u ([u][p] per chunk), half the bytes.
constexpr bool kAlphaNibbles = kF == 2;
__host__ __device__ __forceinline__ int alpha_rows(int dc_max) {
  return kAlphaNibbles ? (dc_max + 1) / 2 : dc_max;
}
__device__ __forceinline__ int alpha_of(uint32_t byte, int f) {
  const uint32_t b = byte >> (2 * f);
  return (b & 2u) ? 0 : ((b & 1u) ? -1 : 1);
}

__device__ __forceinline__ void decide_slots(const MsnWork &w, int k, uint32_t odd, int nb,
                                             int max_iters, int et_period, int B, int32_t *synd);

__device__ __forceinline__ int wave_of_block() {
  return __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
}

// Uniform loads (chunk masks, iteration counts) through the scalar cache:
// issued at the top of a kernel, in parallel with its vector loads, and never
// written by the kernel that reads them (the previous launch's decision wrote
// them).
template <typename T>
__device__ __forceinline__ T ld_uniform(const T *p) {
  return *(const __attribute__((address_space(4))) T *)p;
}

// Descriptor words.  The S descriptors of wave w of item block b sit at
// (4 b + w) S, so one 4-byte load per lane reads 8 of them -- lane l gets
// dword l & 7 of slot 8 g + (l >> 3) -- at an address known from blockIdx
// alone.  Groups 0 .. NW - 1.  Runs with every lane of the wave active:
// slot_value reads the words across the wave, so lanes whose item is past n
// must have loaded theirs.
template <int NW>
__device__ __forceinline__ void desc_words(const MsnDesc *desc, int bi, int S, int (&word)[NW]) {
  const int lane = threadIdx.x & 63;
  const MsnDesc *d = desc + (int64_t)(4 * bi + wave_of_block()) * S;
#pragma unroll
  for (int i = 0; i < NW; ++i)
    word[i] = 8 * i < S && 8 * i + (lane >> 3) < S ? ((const int32_t *)(d + 8 * i))[lane] : 0;
}
// the block's largest degree and whether this wave's values are explicit
__device__ __forceinline__ int desc_degree(int word0) { return __builtin_amdgcn_readlane(word0, 6); }
__device__ __forceinline__ bool desc_explicit(int word0) {
  return __builtin_amdgcn_readlane(word0, 7) != 0;
}

// The lane's value of slot T from its group's word: b[run] + lane (runs and
// bases read across the wave), or the explicit table's value.
template <int T>
__device__ __forceinline__ int slot_value(int word) {
  constexpr int q = 8 * (T & 7);
  const int lane = threadIdx.x & 63;
  const uint32_t thr = (uint32_t)__builtin_amdgcn_readlane(word, q + 4);
  const int b0 = __builtin_amdgcn_readlane(word, q), b1 = __builtin_amdgcn_readlane(word, q + 1),
            b2 = __builtin_amdgcn_readlane(word, q + 2), b3 = __builtin_amdgcn_readlane(word, q + 3);
  int base = lane >= (int)(thr & 0xffu) ? b1 : b0;  // s1 <= s2 <= s3
  base = lane >= (int)((thr >> 8) & 0xffu) ? b2 : base;
  base = lane >= (int)((thr >> 16) & 0xffu) ? b3 : base;
  return base + lane;
}
template <int T>
__device__ __forceinline__ int slot_explicit(int word, const int32_t *x) {
  return x[__builtin_amdgcn_readlane(word, 8 * (T & 7) + 5) + (int)(threadIdx.x & 63)];
}

template <int T0, int I, bool EXPL>
__device__ __forceinline__ void slot_values(const int *word, const int32_t *x, int deg, int *v) {
  if constexpr (I > 0) {
    slot_values<T0, I - 1, EXPL>(word, x, deg, v);
    constexpr int t = T0 + I - 1;
    const int wd = word[t / 8];
    if constexpr (EXPL)
      v[I - 1] = t < deg ? slot_explicit<t>(wd, x) : -1;
    else
      v[I - 1] = t < deg ? slot_value<t>(wd) : -1;
  }
}

// The lane's values of slots T0 .. T0 + D - 1 of its item (negative: no
// edge) from its wave's descriptor words (desc_words).
template <int T0, int D, int NW>
__device__ __forceinline__ void edge_values(const int (&word)[NW], const int32_t *x, int (&v)[D]) {
  static_assert((T0 + D - 1) / 8 < NW, "descriptor group not loaded");
  const int deg = desc_degree(word[0]);
  if (desc_explicit(word[0]))
    slot_values<T0, D, true>(word, x, deg, v);
  else
    slot_values<T0, D, false>(word, x, deg, v);
}


// ---------------------------------------------------------------------------
// Horizontal step (:340-376) of one row (storage position p) for the chunk's
// F frames, D = the block's largest row degree, every load of the row issued
// before the first is used (edges past the row's own degree read column 0
// and are masked).  L(q) of each edge is LQ - L(r_old) (:387-392); a frame's
// first step takes L(q) = Lci (LQ = Lci, no old message).  The parity of the
// last decisions (checkFrame, :236-253) comes from the signs of the same LQ.
// The row's state (om1, om2, omt) and alpha bytes (ab) were loaded by the
// caller with the descriptor words; the block's degree is <= D: the
// straight-line bodies are instantiated at the block degree, the body for
// degrees above 8 at D = DC with slots past the block degree masked.
template <int PREC, int D, int NW, int NA>
__device__ __forceinline__ void check_row(const MsnView &g, const MsnWork &w, int k, int p,
                                          const int (&word)[NW],
                                          const Vec<typename Math<PREC>::Real> &om1,
                                          const Vec<typename Math<PREC>::Real> &om2, MetaWord omt,
                                          const uint32_t (&ab)[NA], const int (&itf)[kF],
                                          bool (&par)[kF]) {
  static_assert(D <= NA, "alpha bytes not loaded");
  typedef typename Math<PREC>::Real Real;
  int cs[D];
  bool ok[D];
  edge_values<0, D>(word, g.rx, cs);
#pragma unroll
  for (int t = 0; t < D; ++t) {
    ok[t] = cs[t] >= 0;
    cs[t] = ok[t] ? cs[t] : 0;
  }
  Real *m1 = (Real *)w.m1, *m2 = (Real *)w.m2;
  const Real *LQ = (const Real *)w.LQ;
  const int64_t ro = el(k, g.M, p);
  uint8_t *alpha = w.alpha + (int64_t)k * alpha_rows(g.dc_max) * g.M + p;  // [t][p] / [t/2][p]
  Vec<Real> lq[D];
#pragma unroll
  for (int t = 0; t < D; ++t) lq[t] = ldv(LQ + el(k, g.N, cs[t]));
  // per frame: L(q) in ascending original column, sign product, smallest and
  // second smallest |L(q)| (strict <, first occurrence, DBL_MAX seeds; NaN
  // never passes), the new alpha bits
  Vec<Real> n1, n2;
  MetaWord nmt = 0;
  uint32_t nb[D];
#pragma unroll
  for (int t = 0; t < D; ++t) nb[t] = 0;
#pragma unroll
  for (int f = 0; f < kF; ++f) {
    const int mt = (int)((omt >> (8 * f)) & 0xffu);
    const int oP = (mt >> 6) - 1, oi1 = (mt & 63) - 1;
    int P = 1, i1 = -1;
    Real a1 = Math<PREC>::max_(), a2 = Math<PREC>::max_();
#pragma unroll
    for (int t = 0; t < D; ++t)
      if (ok[t]) {
        const Real l = lq[t].v[f];
        par[f] ^= l < Real(0);
        const Real r = itf[f] == 0 ? Real(0)
                                   : (Real)(oP * alpha_of(ab[t], f)) * (t == oi1 ? om2.v[f] : om1.v[f]);
        const Real q = l - r;
        P *= sgn(q);
        const Real a = Math<PREC>::abs_(q);
        if (a < a1) {
          a2 = a1;
          a1 = a;
          i1 = t;
        } else if (a < a2) {
          a2 = a;
        }
        const bool neg = q < Real(0);
        const bool zero = !(q > Real(0)) && !neg;
        nb[t] |= ((uint32_t)neg | ((uint32_t)zero << 1)) << (2 * f);
      }
    n1.v[f] = a1;
    n2.v[f] = a2;
    nmt |= (MetaWord)(((P + 1) << 6) | (i1 + 1)) << (8 * f);
  }
  stv_nt(m1 + ro, n1);
  stv_nt(m2 + ro, n2);
  st_meta(w.meta + ro, nmt);
  if constexpr (kAlphaNibbles) {
#pragma unroll
    for (int u = 0; 2 * u < D; ++u)
      if (ok[2 * u])
        alpha[(int64_t)u * g.M] = (uint8_t)(nb[2 * u] | (2 * u + 1 < D ? nb[2 * u + 1] << 4 : 0u));
  } else {
#pragma unroll
    for (int t = 0; t < D; ++t)
      if (ok[t]) alpha[(int64_t)t * g.M] = (uint8_t)nb[t];
  }
}

// One row per lane, the chunk's F frames in the lane.  Frames whose slot is
// not live compute on stale values nobody reads.
// mbuf: this pass's mask buffer (the decision writes the other).  The
// chunk's decision is taken in this launch by the block whose arrival
// completes the chunk: 64-bit atomic adds carry the arrival (bits 0-11) and,
// per frame f, "a row of these blocks is unsatisfied" (bits 12(f+1)..), in
// two levels (8 group words per chunk, then the chunk's word); no fence and
// no waiting (a chunk that is not live decides in its block 0 alone).
#ifndef LDPC_MSN_ZIGZAG
#define LDPC_MSN_ZIGZAG 1  // the variable pass walks each XCD's chunks backwards
#endif
// occupancy hints (waves per SIMD; A/B knobs)
#ifndef LDPC_MSN_CHECK_MINB
#define LDPC_MSN_CHECK_MINB 1
#endif
#ifndef LDPC_MSN_VAR_MINB
#define LDPC_MSN_VAR_MINB 1
#endif
template <int PREC, int DC>
__global__ void __launch_bounds__(256, LDPC_MSN_CHECK_MINB) msn_check(MsnView g, MsnWork w, int mbuf, int max_iters,
                                                 int et_period, int B, int32_t *synd) {
  typedef typename Math<PREC>::Real Real;
  int k, bi;
  map_block(blockIdx.x, w.chunks, w.nb_check, k, bi);
  // every load that does not depend on the descriptors goes out with them:
  // one memory round trip before the gathers (rows past M load row M - 1)
  const int p = bi * kIB + threadIdx.x;  // row storage position
  const int pl = min(p, g.M - 1);
  int word[(DC + 7) / 8];
  desc_words(g.rdesc, bi, g.rs, word);
  const uint32_t live = ld_uniform(&w.live[mbuf * w.chunks + k]);
  int itf[kF];
#pragma unroll
  for (int f = 0; f < kF; ++f) itf[f] = ld_uniform(&w.it[k * kF + f]);
  const int64_t ro = el(k, g.M, pl);
  const Vec<Real> om1 = ldv_nt((const Real *)w.m1 + ro), om2 = ldv_nt((const Real *)w.m2 + ro);
  const MetaWord omt = ld_meta(w.meta + ro);
  uint32_t ab[DC];
  const uint8_t *alpha = w.alpha + (int64_t)k * alpha_rows(g.dc_max) * g.M + pl;
  if constexpr (kAlphaNibbles) {
#pragma unroll
    for (int u = 0; 2 * u < DC; ++u) {
      const uint32_t byte = 2 * u < g.dc_max ? alpha[(int64_t)u * g.M] : 0u;
      ab[2 * u] = byte & 15u;
      if (2 * u + 1 < DC) ab[2 * u + 1] = byte >> 4;
    }
  } else {
#pragma unroll
    for (int t = 0; t < DC; ++t) ab[t] = t < g.dc_max ? alpha[(int64_t)t * g.M] : 0u;
  }
  if (!live) {
    if (bi == 0 && threadIdx.x < 64)
      decide_slots(w, k, 0u, mbuf ^ 1, max_iters, et_period, B, synd);
    return;
  }
  bool par[kF];
#pragma unroll
  for (int f = 0; f < kF; ++f) par[f] = false;
  if (p < g.M) {
    switch (desc_degree(word[0])) {
#define LDPC_MSN_ROW(n) \
  case n:               \
    if constexpr (n <= DC) check_row<PREC, (n <= DC ? n : 1)>(g, w, k, p, word, om1, om2, omt, ab, itf, par); \
    break;
      LDPC_MSN_ROW(1) LDPC_MSN_ROW(2) LDPC_MSN_ROW(3) LDPC_MSN_ROW(4) LDPC_MSN_ROW(5)
      LDPC_MSN_ROW(6) LDPC_MSN_ROW(7) LDPC_MSN_ROW(8)
#undef LDPC_MSN_ROW
      default:
        if constexpr (DC > 8) check_row<PREC, DC>(g, w, k, p, word, om1, om2, omt, ab, itf, par);
        break;
    }
  }
  uint32_t odd = 0;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int f = 0; f < kF; ++f) {
    const bool on = ((live >> f) & 1u) != 0;
    const uint64_t pm = __ballot(par[f]);
    if (on && pm) odd |= 1u << f;
    // a frame at the cap stops in this pass: its uncapped syndrome weight
    // (returning atomic: performed before this block's arrival below)
    if (on && itf[f] >= 1 && itf[f] >= max_iters && pm && lane == 0) {
      const int r = atomicAdd(&w.capsyn[k * kF + f], __popcll(pm));
      asm volatile("" ::"v"(r) : "memory");
    }
  }
  {
    __shared__ uint32_t s_odd[4];
    __shared__ int s_last;
    __shared__ uint32_t s_tot;
    if (lane == 0) s_odd[threadIdx.x >> 6] = odd;
    __syncthreads();
    if (threadIdx.x == 0) {
      // two levels, so no word sees more than ~16 + 8 arrivals: block bi
      // arrives at its group's word (bi mod 8); a group's last block
      // forwards the group's flags to the chunk's word
      const uint32_t bo = s_odd[0] | s_odd[1] | s_odd[2] | s_odd[3];
      uint64_t add = 1;
#pragma unroll
      for (int f = 0; f < kF; ++f)
        if ((bo >> f) & 1u) add += 1ull << (12 * (f + 1));
      const int grp = bi & 7, ngrp = (w.nb_check - grp + 7) >> 3, groups = min(8, w.nb_check);
      unsigned long long *word = (unsigned long long *)&w.arrive[(int64_t)k * 9];
      const uint64_t old = atomicAdd(word + 1 + grp, (unsigned long long)add);
      const uint64_t tot = old + add;
      int last = 0;
      uint32_t o = 0;
      if ((int)(old & 0xfffu) == ngrp - 1) {
        atomicExch(word + 1 + grp, 0ull);
        uint64_t add2 = 1;
#pragma unroll
        for (int f = 0; f < kF; ++f)
          if ((tot >> (12 * (f + 1))) & 0xfffu) add2 += 1ull << (12 * (f + 1));
        const uint64_t old2 = atomicAdd(word, (unsigned long long)add2);
        const uint64_t tot2 = old2 + add2;
        last = (int)(old2 & 0xfffu) == groups - 1;
#pragma unroll
        for (int f = 0; f < kF; ++f)
          if ((tot2 >> (12 * (f + 1))) & 0xfffu) o |= 1u << f;
      }
      s_last = last;
      s_tot = o;
    }
    __syncthreads();
    if (!s_last || threadIdx.x >= 64) return;
    if (threadIdx.x == 0) atomicExch((unsigned long long *)&w.arrive[(int64_t)k * 9], 0ull);
    decide_slots(w, k, s_tot, mbuf ^ 1, max_iters, et_period, B, synd);
  }
}

// The reference's stopping rule for chunk k's slots (one wave, lanes < F):
// at the cap, or (min-sum, :406-408) when it < cap, it % et_period == 0 and
// every check is satisfied (bit f of odd: frame f saw an unsatisfied row);
// freed (and empty) slots take the next frames of the batch.  The new masks
// go to mask buffer `nb` (the pass's check read the other one).
__device__ __forceinline__ void decide_slots(const MsnWork &w, int k, uint32_t odd, int nb,
                                             int max_iters, int et_period, int B, int32_t *synd) {
  const int lane = threadIdx.x;
  const bool on = lane < kF;
  const int slot = k * kF + lane;
  const int it = on ? w.it[slot] : 0, fr = on ? w.frame[slot] : -1;
  const bool running = fr >= 0;
  const bool unsat = ((odd >> lane) & 1u) != 0;
  const bool stop = running && it >= 1 && (it >= max_iters || (it % et_period == 0 && !unsat));
  const bool want = on && (stop || !running);
  const uint64_t wm = __ballot(want);
  int base = 0;
  if (lane == 0 && wm) base = atomicAdd(&w.ctrl[0], __popcll(wm));
  base = __shfl(base, 0);
  const int rank = __popcll(wm & ((1ull << lane) - 1ull));
  const int nf = want && base + rank < B ? base + rank : -1;
  const bool fill = nf >= 0;
  const bool run = running && !stop;
  // the cap's syndrome weight (0 unless stopped at the cap unsatisfied);
  // taken with an atomic: the check pass added it with atomics
  const int cs = on ? atomicExch(&w.capsyn[slot], 0) : 0;
  if (stop) {
    w.used[slot] = it;
    w.out_frame[slot] = fr;  // its outputs go out in this pass
    if (synd) synd[fr] = cs;
  }
  if (on) {
    w.frame[slot] = want ? nf : fr;  // a refilled slot's new frame
    w.it[slot] = run ? it + 1 : 0;
  }
  const uint32_t sw = (uint32_t)__ballot(stop), rw = (uint32_t)__ballot(run),
                 fw = (uint32_t)__ballot(fill);
  if (lane == 0) {
    const int m = nb * w.chunks + k;
    w.stop[m] = sw;
    w.run[m] = rw;
    w.fill[m] = fw;
    w.live[m] = rw | fw;
    if (sw) atomicAdd(&w.ctrl[1], __popc(sw));
  }
}

// Packed info bits (columns M.., MSB first, :207-219) and iterations of the
// frames that stopped in this pass, from the signs of their LQ.
__global__ void __launch_bounds__(256) msn_post(MsnView g, MsnWork w, DecodeArgs a, int nb) {
  const int k = blockIdx.y;
  const uint32_t sel = w.stop[nb * w.chunks + k];
  if (!sel) return;
  const double *LQd = (const double *)w.LQ;
  const float *LQf = (const float *)w.LQ;
  const bool f32 = w.real_bytes == 4;
  for (int q = blockIdx.x * 256 + threadIdx.x; q < g.KB; q += gridDim.x * 256) {
    int xs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = g.M + q * 8 + j;
      xs[j] = c < g.N ? g.cpos[c] : -1;
    }
    for (int f = 0; f < kF; ++f) {
      if (!((sel >> f) & 1u)) continue;
      unsigned o = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (xs[j] >= 0) {
          const int64_t i = el(k, g.N, xs[j]) + f;
          const bool neg = f32 ? LQf[i] < 0.0f : LQd[i] < 0.0;
          o |= (unsigned)neg << (7 - j);
        }
      a.packed[(int64_t)w.out_frame[k * kF + f] * g.KB + q] = (uint8_t)o;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < kF && ((sel >> threadIdx.x) & 1u) && a.iters) {
    const int slot = k * kF + threadIdx.x;
    a.iters[w.out_frame[slot]] = w.used[slot];
  }
}

// Hard decisions (B x N bytes) and posteriors L(Q) as float (B x N) of the
// frames that stopped.
__global__ void __launch_bounds__(256) msn_cols(MsnView g, MsnWork w, uint8_t *bits, float *llr,
                                                int nb) {
  const int k = blockIdx.y;
  const uint32_t sel = w.stop[nb * w.chunks + k];
  if (!sel) return;
  const double *LQd = (const double *)w.LQ;
  const float *LQf = (const float *)w.LQ;
  const bool f32 = w.real_bytes == 4;
  for (int c = blockIdx.x * 256 + threadIdx.x; c < g.N; c += gridDim.x * 256) {
    const int x = g.cpos[c];
    for (int f = 0; f < kF; ++f) {
      if (!((sel >> f) & 1u)) continue;
      const int64_t i = el(k, g.N, x) + f, fr = w.out_frame[k * kF + f];
      const float v = f32 ? LQf[i] : (float)LQd[i];
      const bool neg = f32 ? LQf[i] < 0.0f : LQd[i] < 0.0;
      if (bits) bits[fr * g.N + c] = (uint8_t)neg;
      if (llr) llr[fr * g.N + c] = v;
    }
  }
}

// Edges T0 .. T0 + D - 1 of the lane's column (storage x = the block's
// item): L(r_ji) from the row's state, added to s in ascending original row.
// Every load of the group is issued before the first is used (m1 and m2 both,
// rather than selecting by meta first: one load level less); edges past the
// column's own degree read row 0 and are masked.
template <typename Real, int T0, int D, int NW>
__device__ __forceinline__ void var_edges(const MsnView &g, const MsnWork &w, int k,
                                          const int (&word)[NW], Vec<Real> &s) {
  const Real *m1 = (const Real *)w.m1, *m2 = (const Real *)w.m2;
  const uint8_t *alpha = w.alpha + (int64_t)k * alpha_rows(g.dc_max) * g.M;
  int v[D];
  edge_values<T0, D>(word, g.cx, v);
  bool ok[D];
  int place[D];
  int64_t ro[D];
  uint32_t ai[D];
#pragma unroll
  for (int t = 0; t < D; ++t) {
    ok[t] = v[t] >= 0;
    const int rp = ok[t] ? (v[t] & 0xffffff) : 0;
    place[t] = ok[t] ? (v[t] >> 24) : 0;
    ro[t] = el(k, g.M, rp);
    ai[t] = (uint32_t)(kAlphaNibbles ? place[t] >> 1 : place[t]) * (uint32_t)g.M + (uint32_t)rp;
  }
  MetaWord mt[D];
  uint32_t ab[D];
  Vec<Real> v1[D], v2[D];
#pragma unroll
  for (int t = 0; t < D; ++t) {
    mt[t] = ld_meta(w.meta + ro[t]);
    ab[t] = alpha[ai[t]];
    if constexpr (kAlphaNibbles) ab[t] = (ab[t] >> (4 * (place[t] & 1))) & 15u;
    v1[t] = ldv(m1 + ro[t]);
    v2[t] = ldv(m2 + ro[t]);
  }
#pragma unroll
  for (int t = 0; t < D; ++t)
    if (ok[t]) {
#pragma unroll
      for (int f = 0; f < kF; ++f) {
        const int m = (int)((mt[t] >> (8 * f)) & 0xffu);
        const Real mag = place[t] == (m & 63) - 1 ? v2[t].v[f] : v1[t].v[f];
        s.v[f] = s.v[f] + (Real)(((m >> 6) - 1) * alpha_of(ab[t], f)) * mag;
      }
    }
}

// the same for columns of degree > 8: edges 8 .. deg - 1, four at a time
template <typename Real>
__device__ void var_edges_rt(const MsnView &g, const MsnWork &w, int k, const int (&word)[2],
                             Vec<Real> &s) {
  const int deg = desc_degree(word[0]);
  if (deg > 8) var_edges<Real, 8, 4>(g, w, k, word, s);
  if (deg > 12) var_edges<Real, 12, 4>(g, w, k, word, s);
}

// Vertical step (:379-403), one column per lane, the chunk's F frames in the
// lane: L(r_ji) of each edge from its row's state, s = sum_j L(r_ji) over
// ascending original rows from +0.0, LQ = Lci + s.  Refilled slots:
// Lci = LQ = -tx of their new frame (:318-331; exact in float, tx is a float).
// With out_var (info columns in place, M % 8 == 0) the frames that stopped
// in this pass write their outputs here from the LQ being replaced -- packed
// bytes (8 lanes' decisions, MSB first, :207-219), iterations, and the
// optional bits / posteriors -- instead of in msn_post / msn_cols.
template <typename Real, int DV>
__global__ void __launch_bounds__(256, LDPC_MSN_VAR_MINB) msn_var(MsnView g, MsnWork w, DecodeArgs a, int nb) {
  int k, bi;
  map_block(blockIdx.x, w.chunks, w.nb_var, k, bi, LDPC_MSN_ZIGZAG != 0);
  const int m = nb * w.chunks + k;  // the decision's mask buffer
  const uint32_t run = ld_uniform(&w.run[m]), fill = ld_uniform(&w.fill[m]),
                 stop = ld_uniform(&w.stop[m]);
  const int x = bi * kIB + threadIdx.x;  // column storage position
  const int64_t ci = el(k, g.N, x);
  Real *LQ = (Real *)w.LQ;
  // the descriptor words and Lci go out together (columns past N load the
  // last column's)
  int word[(DV + 7) / 8];
  desc_words(g.cdesc, bi, g.cs, word);
  Vec<float> lci = ldv_nt(w.L + el(k, g.N, min(x, g.N - 1)));
  if (w.out_var && stop) {
    const int lane = threadIdx.x & 63;
    const bool in = x < g.N;
    const Vec<Real> old = in ? ldv((const Real *)LQ + ci) : Vec<Real>{};
    const int c = in ? g.corig[x] : 0;
#pragma unroll
    for (int f = 0; f < kF; ++f) {
      if (!((stop >> f) & 1u)) continue;
      const int64_t fr = w.out_frame[k * kF + f];
      const bool neg = in && old.v[f] < Real(0);
      const uint64_t m = __ballot(neg);
      if (in && c >= g.M && ((c - g.M) & 7) == 0)
        a.packed[fr * g.KB + ((c - g.M) >> 3)] =
            (uint8_t)(__builtin_bitreverse32((uint32_t)(m >> lane) & 0xffu) >> 24);
      if (in && a.bits) a.bits[fr * g.N + c] = (uint8_t)neg;
      if (in && a.llr) a.llr[fr * g.N + c] = (float)old.v[f];
      if (bi == 0 && threadIdx.x == 0 && a.iters) a.iters[fr] = w.used[k * kF + f];
    }
  }
  if (!(run | fill) || x >= g.N) return;
  if (fill) {
    const int64_t src = (int64_t)g.corig[x] * a.elem_stride;
#pragma unroll
    for (int f = 0; f < kF; ++f)
      if ((fill >> f) & 1u)
        lci.v[f] = -(a.in[(int64_t)w.frame[k * kF + f] * a.cw_stride + src] * a.polarity);
    stv(w.L + ci, lci);
  }
  Vec<Real> s;
#pragma unroll
  for (int f = 0; f < kF; ++f) s.v[f] = Real(0);
  if (run) {
    switch (desc_degree(word[0])) {
#define LDPC_MSN_COL(n)                                                    \
  case n:                                                                  \
    if constexpr (n <= DV) var_edges<Real, 0, (n < 4 ? n : 4)>(g, w, k, word, s); \
    if constexpr (n > 4 && n <= DV) var_edges<Real, 4, (n > 4 ? n - 4 : 1)>(g, w, k, word, s); \
    break;
      LDPC_MSN_COL(1) LDPC_MSN_COL(2) LDPC_MSN_COL(3) LDPC_MSN_COL(4) LDPC_MSN_COL(5)
      LDPC_MSN_COL(6) LDPC_MSN_COL(7) LDPC_MSN_COL(8)
#undef LDPC_MSN_COL
      default:
        if constexpr (DV > 8) {
          var_edges<Real, 0, 4>(g, w, k, word, s);
          var_edges<Real, 4, 4>(g, w, k, word, s);
          var_edges_rt<Real>(g, w, k, word, s);
        }
        break;
    }
  }
  // running frames: Lci + s; refilled: Lci; other slots are not read again
  Vec<Real> lq;
#pragma unroll
  for (int f = 0; f < kF; ++f) lq.v[f] = ((fill >> f) & 1u) ? (Real)lci.v[f] : (Real)lci.v[f] + s.v[f];
  stv_nt(LQ + ci, lq);
}

__global__ void msn_init(MsnWork w) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < w.S; i += gridDim.x * blockDim.x) {
    w.frame[i] = -1;
    w.it[i] = 0;
    w.capsyn[i] = 0;
  }
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < 2 * w.chunks; k += gridDim.x * blockDim.x) {
    w.live[k] = w.run[k] = w.stop[k] = w.fill[k] = 0;
    if (k < w.chunks)
      for (int j = 0; j < 9; ++j) w.arrive[(int64_t)k * 9 + j] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    w.ctrl[0] = 0;
    w.ctrl[1] = 0;
  }
}

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// Pass p reads mask buffer p & 1 and decides into the other.
template <int PREC>
void msn_pass(const MsnView &g, const MsnWork &w, const DecodeArgs &a, int par, hipStream_t st) {
  typedef typename Math<PREC>::Real Real;
  const int rblocks = w.nb_check * w.chunks, cblocks = w.nb_var * w.chunks, nb = par ^ 1;
  static_assert(kMsnFrames == kF, "");
#define LDPC_MSN_CHECK(DC) \
  msn_check<PREC, DC><<<rblocks, 256, 0, st>>>(g, w, par, a.max_iters, a.et_period, a.B, a.synd)
  if (g.dc_max <= 8)
    LDPC_MSN_CHECK(8);
  else if (g.dc_max <= 16)
    LDPC_MSN_CHECK(16);
  else
    LDPC_MSN_CHECK(32);
#undef LDPC_MSN_CHECK
  if (!w.out_var) {
    const int pb = std::min(16, (g.KB + 255) / 256);
    msn_post<<<dim3(pb, w.chunks), 256, 0, st>>>(g, w, a, nb);
    if (a.bits || a.llr)
      msn_cols<<<dim3(std::min(64, (g.N + 255) / 256), w.chunks), 256, 0, st>>>(g, w, a.bits, a.llr,
                                                                                nb);
  }
  if (g.dv_max <= 4)
    msn_var<Real, 4><<<cblocks, 256, 0, st>>>(g, w, a, nb);
  else if (g.dv_max <= 8)
    msn_var<Real, 8><<<cblocks, 256, 0, st>>>(g, w, a, nb);
  else
    msn_var<Real, 16><<<cblocks, 256, 0, st>>>(g, w, a, nb);
}

}  // namespace

int msn_default_chunks() {
  const char *e = getenv("LDPC_MSN_CHUNKS");  // A/B knob
  const int v = e ? atoi(e) : 0;
  // 80 chunks of 2 frames = 160 frames in flight, 10 chunks per XCD:
  // 2 518-2 522 Mbit/s against 2 486 for 64, 2 469 for 96 and 2 104 for 112
  // (profiles/round4/msn_chunks/; round 3 at 4 frames per chunk: 40 chunks,
  // profiles/round3/msn/chunks_fused.txt)
  return v >= 1 ? v : 80;
}

size_t msn_work_bytes(const MsnView &g, int chunks, int prec) {
  const size_t real = prec == 1 ? 4 : 8, F = kF, C = chunks;
  size_t n = al256(C * g.N * F * 4) + al256(C * g.N * F * real);  // L, LQ
  n += 2 * al256(C * g.M * F * real) + al256(C * g.M * F);        // m1, m2, meta
  n += al256(C * alpha_rows(g.dc_max) * g.M);                     // alpha
  n += 5 * al256(C * F * 4);                                      // capsyn, it, frame, out_frame, used
  n += 4 * al256(2 * C * 4) + al256(C * 9 * 8) + al256(64);      // masks x 2, arrive, ctrl
  return n;
}

void msn_work_carve(MsnWork &w, void *base, const MsnView &g, int chunks, int prec) {
  const size_t real = prec == 1 ? 4 : 8, F = kF, C = chunks;
  char *p = (char *)base;
  auto take = [&](size_t bytes) {
    char *r = p;
    p += al256(bytes);
    return (void *)r;
  };
  w = MsnWork{};
  w.chunks = chunks;
  w.S = chunks * kF;
  w.real_bytes = (int)real;
  w.nb_check = (g.M + kIB - 1) / kIB;
  w.nb_var = (g.N + kIB - 1) / kIB;
  w.check_waves = w.nb_check * 4;
  w.out_var = g.out_var;
  w.L = (float *)take(C * g.N * F * 4);
  w.LQ = take(C * g.N * F * real);
  w.m1 = take(C * g.M * F * real);
  w.m2 = take(C * g.M * F * real);
  w.meta = (uint8_t *)take(C * g.M * F);
  w.alpha = (uint8_t *)take(C * alpha_rows(g.dc_max) * g.M);
  w.capsyn = (int32_t *)take(C * F * 4);
  w.it = (int32_t *)take(C * F * 4);
  w.frame = (int32_t *)take(C * F * 4);
  w.out_frame = (int32_t *)take(C * F * 4);
  w.used = (int32_t *)take(C * F * 4);
  w.live = (uint32_t *)take(2 * C * 4);
  w.run = (uint32_t *)take(2 * C * 4);
  w.stop = (uint32_t *)take(2 * C * 4);
  w.fill = (uint32_t *)take(2 * C * 4);
  w.arrive = (uint64_t *)take(C * 9 * 8);
  // The decision in the check pass's last block per chunk (12-bit arrival
  // counts: M <= kMsnMaxRows).  One word per chunk made the 127 blocks of a
  // chunk contend (check pass 53.5 us against 40.8 + 4.9 for the check and
  // decision launches, profiles/round3/msn/fused_decide.txt); two levels (8
  // group words, then the chunk's) measured 2 219-2 229 against 2 207-2 212
  // Mbit/s for a separate decision launch (profiles/round3/msn/ab_fuse2.txt),
  // which was then removed
  w.ctrl = (int32_t *)take(64);
}

int launch_graph_decode_msn(const MsnView &g, const MsnWork &w, const DecodeArgs &a, int prec,
                            int32_t *h_ctrl, void *stream) {
  if (g.dc_max > kGraphDcMax || g.dv_max > kGraphDvMax) return -2;
  if (a.B <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  msn_init<<<std::max(1, std::min(64, (w.S + 255) / 256)), 256, 0, st>>>(w);
  // every slot finishes a frame at least every max_iters + 1 passes (as
  // launch_graph_decode_ms); the host stops enqueueing once every frame is done
  const int64_t bound = ((int64_t)(a.B + w.S - 1) / w.S + 1) * (a.max_iters + 1) + 2;
  const int kRound = 8;
  hipEvent_t ev[2] = {nullptr, nullptr};
  for (int i = 0; i < 2; ++i)
    if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return -1;
  int rc = 0;
  int64_t pass = 0;
  for (int round = 0; pass < bound; ++round) {
    for (int i = 0; i < kRound && pass < bound; ++i, ++pass) {
      if (prec == 1)
        msn_pass<1>(g, w, a, (int)(pass & 1), st);
      else
        msn_pass<0>(g, w, a, (int)(pass & 1), st);
    }
    if (hipMemcpyAsync(h_ctrl + 2 * (round & 1), w.ctrl, 8, hipMemcpyDeviceToHost, st) !=
            hipSuccess ||
        hipEventRecord(ev[round & 1], st) != hipSuccess) {
      rc = -1;
      break;
    }
    if (round > 0) {
      if (hipEventSynchronize(ev[(round - 1) & 1]) != hipSuccess) {
        rc = -1;
        break;
      }
      if (h_ctrl[2 * ((round - 1) & 1) + 1] >= a.B) break;  // all frames finished
    }
  }
  for (int i = 0; i < 2; ++i) (void)hipEventDestroy(ev[i]);
  if (rc == 0 && hipGetLastError() != hipSuccess) rc = -1;
  return rc;
}

// ---- storage order (host) --------------------------------------------------

namespace {

// Pairs of neighbouring storage rows (columns) of equal degree whose t-th
// edges land on neighbouring storage columns (rows): the contiguity a wave's
// gathers get from the order.
long contiguity(const MsnTables &t) {
  long s = 0;
  const int M = (int)t.rp.size() - 1, N = (int)t.cp.size() - 1;
  for (int p = 0; p + 1 < M; ++p) {
    const int d = t.rp[p + 1] - t.rp[p];
    if (t.rp[p + 2] - t.rp[p + 1] != d) continue;
    for (int e = 0; e < d; ++e) s += t.rcs[(size_t)e * M + p + 1] == t.rcs[(size_t)e * M + p] + 1;
  }
  for (int x = 0; x + 1 < N; ++x) {
    const int d = t.cp[x + 1] - t.cp[x];
    if (t.cp[x + 2] - t.cp[x + 1] != d) continue;
    for (int e = 0; e < d; ++e)
      s += (t.crs[(size_t)e * N + x + 1] & 0xffffff) == (t.crs[(size_t)e * N + x] & 0xffffff) + 1;
  }
  return s;
}

}  // namespace

// A slot-major table full[t][x] (D x n, -1 past each item's degree) as
// descriptors (MsnDesc: up to 4 runs of consecutive values): S = D per wave
// of the kernels' 256-item blocks, slot t of wave w of block b at
// (4 b + w) S + t; slots past the block's largest degree hold no edge.  Each
// descriptor also carries that degree (pad[0]) and whether its wave's values
// are explicit (pad[1]): a wave with a slot of more than 4 runs keeps every
// slot's 64 values in `x` (at each descriptor's xoff).
void msn_block_tables(const std::vector<int32_t> &full, int D, int n, std::vector<MsnDesc> &desc,
                      std::vector<int32_t> &x) {
  const int nb = (n + kIB - 1) / kIB, nw = kIB / 64, S = D;
  MsnDesc none{};
  for (int r = 0; r < 4; ++r) none.b[r] = kMsnNoEdge;
  none.thr = 64u | 64u << 8 | 64u << 16;
  none.xoff = -1;
  desc.assign((size_t)nb * nw * S, none);
  x.clear();
  for (int b = 0; b < nb; ++b) {
    int deg = 0;
    for (int i = 0; i < kIB; ++i) {
      const int c = b * kIB + i;
      if (c >= n) break;
      for (int t = 0; t < D; ++t)
        if (full[(size_t)t * n + c] != -1) deg = std::max(deg, t + 1);
    }
    for (int w = 0; w < nw; ++w) {
      MsnDesc *mine = &desc[((size_t)b * nw + w) * S];
      std::vector<int32_t> vals((size_t)deg * 64);
      bool explicit_wave = false;
      for (int t = 0; t < deg; ++t) {
        int32_t *v = &vals[(size_t)t * 64];
        for (int l = 0; l < 64; ++l) {
          const int c = b * kIB + w * 64 + l;
          v[l] = c < n ? full[(size_t)t * n + c] : -1;
        }
        int start[64], runs = 0;
        for (int l = 0; l < 64; ++l) {
          const bool cont = l > 0 && ((v[l - 1] < 0 && v[l] < 0) || (v[l - 1] >= 0 && v[l] == v[l - 1] + 1));
          if (!cont) start[runs++] = l;
        }
        MsnDesc &d = mine[t];
        explicit_wave |= runs > 4;
        uint32_t thr = 0;
        for (int r = 0; r < 4; ++r) {
          const int a = r < runs ? start[r] : 64;
          d.b[r] = r < runs ? (v[a] < 0 ? kMsnNoEdge : v[a] - a) : kMsnNoEdge;
          if (r >= 1) thr |= (uint32_t)a << (8 * (r - 1));
        }
        d.thr = thr;
      }
      if (explicit_wave)
        for (int t = 0; t < deg; ++t) mine[t].xoff = (int32_t)(x.size() + (size_t)t * 64);
      if (explicit_wave) x.insert(x.end(), vals.begin(), vals.end());
      for (int t = 0; t < S; ++t) {
        mine[t].pad[0] = deg;
        mine[t].pad[1] = explicit_wave ? 1 : 0;
      }
    }
  }
  // self-check: decode every (block, wave, slot, lane) as the kernels do
  // (desc_words / slot_value / slot_explicit) and compare with the table
  for (int b = 0; b < nb; ++b)
    for (int w = 0; w < nw; ++w)
      for (int t = 0; t < S; ++t) {
        const MsnDesc *mine = &desc[((size_t)b * nw + w) * S];
        const MsnDesc &d = mine[t];
        const int deg = mine[0].pad[0];
        const bool expl = mine[0].pad[1] != 0;
        for (int l = 0; l < 64; ++l) {
          const int c = b * kIB + w * 64 + l;
          const int32_t want = c < n ? full[(size_t)t * n + c] : -1;
          int32_t got;
          if (t >= deg) {
            got = -1;
          } else if (expl) {
            got = x[(size_t)d.xoff + l];
          } else {
            int base = l >= (int)(d.thr & 0xffu) ? d.b[1] : d.b[0];
            base = l >= (int)((d.thr >> 8) & 0xffu) ? d.b[2] : base;
            base = l >= (int)((d.thr >> 16) & 0xffu) ? d.b[3] : base;
            got = base + l;
          }
          if ((want < 0) != (got < 0) || (want >= 0 && want != got))
            throw std::runtime_error("msn_block_tables: descriptor self-check failed");
        }
      }
}

// Storage-ordered tables of H (rows rpos, columns cpos): row offsets and
// column offsets for the degrees, and slot-major edge lists -- rcs[t][p] the
// storage column of row p's t-th edge (ascending original column), crs[t][x]
// the storage row of column x's t-th edge (ascending original row) | the
// edge's place in that row << 24 -- so a wave's t-th edges are one
// coalesced load.
void msn_tables(int M, int N, const std::vector<int32_t> &rp0, const std::vector<int32_t> &ci0,
                const std::vector<int32_t> &rpos, const std::vector<int32_t> &cpos,
                MsnTables &t) {
  std::vector<int32_t> rorig(M), corig(N);
  for (int j = 0; j < M; ++j) rorig[rpos[j]] = j;
  for (int c = 0; c < N; ++c) corig[cpos[c]] = c;
  int dc = 0, dv = 0;
  std::vector<int32_t> cdeg((size_t)N, 0);
  for (int j = 0; j < M; ++j) {
    dc = std::max(dc, rp0[j + 1] - rp0[j]);
    for (int32_t o = rp0[j]; o < rp0[j + 1]; ++o) cdeg[cpos[ci0[o]]]++;
  }
  for (int x = 0; x < N; ++x) dv = std::max(dv, cdeg[x]);
  t.rp.assign((size_t)M + 1, 0);
  t.rcs.assign((size_t)dc * M, -1);
  for (int p = 0; p < M; ++p) {
    const int j = rorig[p];
    t.rp[p + 1] = t.rp[p] + (rp0[j + 1] - rp0[j]);
    for (int32_t o = rp0[j]; o < rp0[j + 1]; ++o) t.rcs[(size_t)(o - rp0[j]) * M + p] = cpos[ci0[o]];
  }
  t.cp.assign((size_t)N + 1, 0);
  for (int x = 0; x < N; ++x) t.cp[x + 1] = t.cp[x] + cdeg[x];
  t.crs.assign((size_t)dv * N, -1);
  std::vector<int32_t> fill((size_t)N, 0);
  for (int j = 0; j < M; ++j)  // original rows ascending
    for (int32_t o = rp0[j]; o < rp0[j + 1]; ++o) {
      const int x = cpos[ci0[o]];
      t.crs[(size_t)fill[x]++ * N + x] = rpos[j] | ((o - rp0[j]) << 24);
    }
  t.corig = corig;
  t.cpos = cpos;
  t.rpos = rpos;
  msn_block_tables(t.rcs, dc, M, t.rdesc, t.rx);
  msn_block_tables(t.crs, dv, N, t.cdesc, t.cx);
  t.rs = dc;
  t.cs = dv;
  // outputs from the variable pass need the info columns in place, 8 per byte
  t.out_var = M % 8 == 0;
  for (int c = M; c < N && t.out_var; ++c) t.out_var = cpos[c] == c;
}

// Chooses the storage order: the identity, or for M a multiple of 360 the
// DVB-S2 residue-class order (row r -> (r mod q) * 360 + r / q, q = M / 360,
// and the staircase's degree <= 2 columns {r, r+1} moved among their own
// positions in the order of r's class position) -- whichever gives the
// kernels' gathers more contiguity.  LDPC_MSN_ORDER=0 / 1 forces one.
void msn_build(int M, int N, const std::vector<int32_t> &rp0, const std::vector<int32_t> &ci0,
               MsnTables &t) {
  std::vector<int32_t> rid(M), cid(N);
  for (int j = 0; j < M; ++j) rid[j] = j;
  for (int c = 0; c < N; ++c) cid[c] = c;
  const char *env = getenv("LDPC_MSN_ORDER");
  const int force = env ? atoi(env) : -1;
  msn_tables(M, N, rp0, ci0, rid, cid, t);
  t.order = 0;
  t.score[0] = contiguity(t);
  t.score[1] = -1;
  if (M % 360 != 0 || force == 0) return;
  const int q = M / 360;
  std::vector<int32_t> rpos(M), cpos(cid);
  for (int j = 0; j < M; ++j) rpos[j] = (j % q) * 360 + j / q;
  // staircase columns: degree 1 or 2 with rows r (and r + 1)
  std::vector<int32_t> cdeg(N, 0), cfirst(N, -1), clast(N, -1);
  for (int j = 0; j < M; ++j)
    for (int32_t o = rp0[j]; o < rp0[j + 1]; ++o) {
      const int c = ci0[o];
      if (cfirst[c] < 0) cfirst[c] = j;
      clast[c] = j;
      cdeg[c]++;
    }
  std::vector<int32_t> stair, slots;
  for (int c = 0; c < N; ++c)
    if ((cdeg[c] == 1) || (cdeg[c] == 2 && clast[c] == cfirst[c] + 1)) {
      stair.push_back(c);
      slots.push_back(c);
    }
  std::stable_sort(stair.begin(), stair.end(),
                   [&](int a, int b) { return rpos[cfirst[a]] < rpos[cfirst[b]]; });
  for (size_t i = 0; i < stair.size(); ++i) cpos[stair[i]] = slots[i];
  MsnTables qc;
  msn_tables(M, N, rp0, ci0, rpos, cpos, qc);
  qc.order = 1;
  const long s_id = contiguity(t), s_qc = contiguity(qc);
  qc.score[0] = s_id;
  qc.score[1] = s_qc;
  t.score[1] = s_qc;
  if (force == 1 || s_qc > s_id) t = std::move(qc);
}

}  // namespace ldpc
