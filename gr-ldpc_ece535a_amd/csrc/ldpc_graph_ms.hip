// ldpc_graph_ms.hip -- min-sum on large codes with
// compressed check messages and a frame pipeline.
//
// The reference's horizontal step (lib/ldpc_decoder_cb_impl.cc:350-376) gives
// every edge of row j the message
//     L(r_ji) = (double)(P_j * alpha_ji) * (i == i1_j ? m2_j : m1_j)
// where alpha = sign(L(q)) (sign(0) = sign(NaN) = 0), P_j = prod of the
// row's alphas, m1 / m2 = the smallest / second smallest |L(q)| of the row
// (strict <, first occurrence, DBL_MAX seeds, NaN never taken) and i1 the
// position of m1.  So a row's messages are exactly recoverable from
// {m1, m2, i1, P} plus one 2-bit alpha per edge, and the vertical step's
// L(q_ij) = (Lci + s) - L(r_ji) (:387-392) is LQ_i - L(r_ji) with
// LQ_i = Lci + s (:395).  This path stores per 64-frame chunk
//   LQ (N) and Lci (N, float: -tx is a float),
//   m1, m2 (M), meta (M bytes: P+1 in bits 6-7, i1+1 in bits 0-5),
//   alpha (2 words per edge: lanes with L(q) < 0, lanes with sign 0),
// instead of the edge messages L(q) and L(r) (2 E values), and recomputes
// L(q) in the check pass and L(r) in the variable pass, operation for
// operation as the reference.  Per frame-iteration that is ~17 M + 12 N
// bytes plus 2 bits per edge of state instead of 16 E -- small enough that a
// few chunks' state stays in the 256 MiB Infinity Cache between the passes.
//
// Frame pipeline: S slots (a few 64-frame chunks) are in flight; every pass
// advances each running slot by one iteration; a slot whose frame stops
// (early exit under the reference's rule, or the cap) writes that frame's
// outputs and loads the next frame of the batch.  Four launches per pass:
//   ms_check     one wave = 4 rows x 64 slots: syndrome parities of the last
//                decisions, L(q) = LQ - L(r_old), the row state of the new L(r)
//   ms_decide    one block per chunk: stop / run / refill per slot
//   ms_post      packed bytes and iterations of the stopped frames, and the
//                syndrome weight of those stopped at the cap
//   (ms_flush_cols  bits / posteriors of the stopped frames, when asked for)
//   ms_var_fill  one wave = 4 columns x 64 slots: running slots: L(r) from the
//                row states, s = sum L(r) ascending rows, LQ = Lci + s, vhat =
//                LQ < 0; refilled slots: Lci = LQ = -tx of their new frame
// A slot refilled in pass p runs its first horizontal step in pass p+1.
#include <hip/hip_runtime.h>

#include <algorithm>

#include <stdlib.h>

#include "ldpc_device.hpp"
#include "ldpc_graph.hpp"

namespace ldpc {
namespace {

#ifndef LDPC_MS_ROWS
#define LDPC_MS_ROWS 8
#endif
#ifndef LDPC_MS_COLS
#define LDPC_MS_COLS 4
#endif
constexpr int kMsRows = LDPC_MS_ROWS;  // check rows per wave
constexpr int kMsCols = LDPC_MS_COLS;  // columns per wave

__device__ __forceinline__ int wave_id() {
  return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}
__device__ __forceinline__ uint64_t lane_bit(uint64_t w, int lane) { return (w >> lane) & 1ull; }
__device__ __forceinline__ int64_t at(int64_t x, int k, int64_t n, int lane) {
  return ((int64_t)k * n + x) * 64 + lane;
}
size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
// lane l's 64-bit value, to every lane (l uniform)
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

// alpha of an edge for this lane from its two words
__device__ __forceinline__ int alpha_of(uint64_t neg, uint64_t zero, int lane) {
  return lane_bit(zero, lane) ? 0 : (lane_bit(neg, lane) ? -1 : 1);
}

// ---------------------------------------------------------------------------
template <int PREC, int DC>
__device__ __forceinline__ void check_rows(const GraphView &g, const MsWork &w, int k) {
  typedef typename Math<PREC>::Real Real;
  const int lane = threadIdx.x & 63;
  const int64_t chunks = w.chunks;
  const bool fresh = w.it[k * 64 + lane] == 0;  // first horizontal step: L(q) = Lci
  const Real *LQ = (const Real *)w.LQ;
  Real *m1 = (Real *)w.m1, *m2 = (Real *)w.m2;
  const int wg = blockIdx.x * 4 + wave_id();
  const int j0 = wg * kMsRows;
  const int j1 = min(j0 + kMsRows, g.M);
  uint64_t odd = 0;  // checkFrame (:236-253) of the last decisions, 64 slots per word
  for (int j = j0; j < j1; ++j) {
    uint64_t par = 0;
    const int e1 = g.rp[j + 1];
    for (int e = g.rp[j]; e < e1; ++e) par ^= w.hard[(int64_t)g.ci[e] * chunks + k];
    odd |= par;
  }
  for (int j = j0; j < j1; ++j) {
    const int e0 = g.rp[j], d = g.rp[j + 1] - e0;
    const int64_t ro = at(j, k, g.M, lane);
    const Real om1 = m1[ro], om2 = m2[ro];
    const int omt = w.meta[ro];
    const int oP = (omt >> 6) - 1, oi1 = (omt & 63) - 1;
    Real q[DC];
#pragma unroll
    for (int t = 0; t < DC; ++t) {
      if (t < d) {
        const Real lq = LQ[at(g.ci[e0 + t], k, g.N, lane)];
        const uint64_t *aw = w.alpha + ((int64_t)(e0 + t) * chunks + k) * 2;
        const int al = alpha_of(aw[0], aw[1], lane);
        // the previous L(r) of the edge (:376), then L(q) = LQ - L(r) (:387-392)
        const Real r = fresh ? Real(0) : (Real)(oP * al) * (t == oi1 ? om2 : om1);
        q[t] = lq - r;
      } else {
        q[t] = Real(0);
      }
    }
    // horizontal step (:340-376): sign product, smallest and second smallest
    // |L(q)| with the reference's strict < (NaN never passes)
    int P = 1, i1 = -1;
    Real a1 = Math<PREC>::max_(), a2 = Math<PREC>::max_();
#pragma unroll
    for (int t = 0; t < DC; ++t)
      if (t < d) {
        P *= sgn(q[t]);
        const Real a = Math<PREC>::abs_(q[t]);
        if (a < a1) {
          a2 = a1;
          a1 = a;
          i1 = t;
        } else if (a < a2) {
          a2 = a;
        }
      }
    m1[ro] = a1;
    m2[ro] = a2;
    w.meta[ro] = (uint8_t)(((P + 1) << 6) | (i1 + 1));
#pragma unroll
    for (int t = 0; t < DC; ++t)
      if (t < d) {
        const uint64_t neg = __ballot(q[t] < Real(0));
        const uint64_t zero = __ballot(!(q[t] > Real(0)) && !(q[t] < Real(0)));
        if (lane == 0) {
          uint64_t *aw = w.alpha + ((int64_t)(e0 + t) * chunks + k) * 2;
          aw[0] = neg;
          aw[1] = zero;
        }
      }
  }
  if (lane == 0) w.odd[(int64_t)wg * chunks + k] = odd;
}

// check_rows for a wave whose rows have at most 64 edges together (8 rows of
// degree <= 8): the rows' edges are consecutive in CSR order, so lane l
// loads edge e_first + l's column, alpha words and hard word with one vector
// load each, and every per-edge value the row loop needs is a readlane --
// instead of three dependent scalar loads per edge (alpha misses the scalar
// cache: 16 B x E x chunks).  The new alpha words go back the same way, one
// vector store per wave.  Same arithmetic, same order as check_rows.
template <int PREC, int DC>
__device__ __forceinline__ void check_rows_lanes(const GraphView &g, const MsWork &w, int k) {
  typedef typename Math<PREC>::Real Real;
  const int lane = threadIdx.x & 63;
  const int64_t chunks = w.chunks;
  const bool fresh = w.it[k * 64 + lane] == 0;  // first horizontal step: L(q) = Lci
  const Real *LQ = (const Real *)w.LQ;
  Real *m1 = (Real *)w.m1, *m2 = (Real *)w.m2;
  const int wg = blockIdx.x * 4 + wave_id();
  const int j0 = wg * kMsRows;
  const int j1 = min(j0 + kMsRows, g.M);
  if (j0 >= j1) {  // a wave past the last row still reports "no row unsatisfied"
    if (lane == 0) w.odd[(int64_t)wg * chunks + k] = 0;
    return;
  }
  const int eb = g.rp[j0], ne = g.rp[j1] - eb;  // <= 64: 8 rows of degree <= 8
  const bool has = lane < ne;
  const int my_c = has ? g.ci[eb + lane] : 0;
  uint64_t my_neg = 0, my_zero = 0, my_h = 0;
  if (has) {
    const uint64_t *aw = w.alpha + ((int64_t)(eb + lane) * chunks + k) * 2;
    my_neg = aw[0];
    my_zero = aw[1];
    my_h = w.hard[(int64_t)my_c * chunks + k];
  }
  uint64_t odd = 0;  // checkFrame (:236-253) of the last decisions, 64 slots per word
  uint64_t new_neg = 0, new_zero = 0;  // this lane's edge's new alpha words
  for (int j = j0; j < j1; ++j) {
    const int e0 = g.rp[j] - eb, d = g.rp[j + 1] - g.rp[j];
    uint64_t par = 0;
    for (int t = 0; t < d; ++t) par ^= readlane64(my_h, e0 + t);
    odd |= par;
    const int64_t ro = at(j, k, g.M, lane);
    const Real om1 = m1[ro], om2 = m2[ro];
    const int omt = w.meta[ro];
    const int oP = (omt >> 6) - 1, oi1 = (omt & 63) - 1;
    Real q[DC];
#pragma unroll
    for (int t = 0; t < DC; ++t) {
      if (t < d) {
        const int c = __builtin_amdgcn_readlane(my_c, e0 + t);
        const Real lq = LQ[at(c, k, g.N, lane)];
        const int al = alpha_of(readlane64(my_neg, e0 + t), readlane64(my_zero, e0 + t), lane);
        // the previous L(r) of the edge (:376), then L(q) = LQ - L(r) (:387-392)
        const Real r = fresh ? Real(0) : (Real)(oP * al) * (t == oi1 ? om2 : om1);
        q[t] = lq - r;
      } else {
        q[t] = Real(0);
      }
    }
    // horizontal step (:340-376): sign product, smallest and second smallest
    // |L(q)| with the reference's strict < (NaN never passes)
    int P = 1, i1 = -1;
    Real a1 = Math<PREC>::max_(), a2 = Math<PREC>::max_();
#pragma unroll
    for (int t = 0; t < DC; ++t)
      if (t < d) {
        P *= sgn(q[t]);
        const Real a = Math<PREC>::abs_(q[t]);
        if (a < a1) {
          a2 = a1;
          a1 = a;
          i1 = t;
        } else if (a < a2) {
          a2 = a;
        }
      }
    m1[ro] = a1;
    m2[ro] = a2;
    w.meta[ro] = (uint8_t)(((P + 1) << 6) | (i1 + 1));
#pragma unroll
    for (int t = 0; t < DC; ++t)
      if (t < d) {
        const uint64_t neg = __ballot(q[t] < Real(0));
        const uint64_t zero = __ballot(!(q[t] > Real(0)) && !(q[t] < Real(0)));
        new_neg = lane == e0 + t ? neg : new_neg;
        new_zero = lane == e0 + t ? zero : new_zero;
      }
  }
  if (has) {
    uint64_t *aw = w.alpha + ((int64_t)(eb + lane) * chunks + k) * 2;
    aw[0] = new_neg;
    aw[1] = new_zero;
  }
  if (lane == 0) w.odd[(int64_t)wg * chunks + k] = odd;
}

template <int PREC, int DC>
__global__ void __launch_bounds__(256) ms_check(GraphView g, MsWork w) {
  const int k = blockIdx.y;
  if (!w.live_w[k]) return;
#ifndef LDPC_MS_SCALAR_META
  if constexpr (DC * kMsRows <= 64) {
    check_rows_lanes<PREC, DC>(g, w, k);
    return;
  }
#endif
  check_rows<PREC, DC>(g, w, k);
}

__device__ void decide_chunk(MsWork w, int k, int max_iters, int et_period, int B, int32_t *synd);

// One block per chunk.  (Deciding in ms_check's last block instead needs
// agent-scope fences in every block, which write back the XCD's L2: slower.)
constexpr int kDecideThreads = 1024;  // the OR over ~4 000 check waves' words: 4 loads each
__global__ void __launch_bounds__(kDecideThreads) ms_decide(MsWork w, int max_iters, int et_period,
                                                            int B, int32_t *synd) {
  decide_chunk(w, blockIdx.x, max_iters, et_period, B, synd);
}

// One kDecideThreads-thread block per chunk.  A running slot that has
// executed `it` iterations stops at the cap, or -- min-sum's rule (:406-408)
// -- when it < cap, it % et_period == 0 and its decision satisfies every
// check.  Freed (and empty) slots take the next frames of the batch in lane
// order.
__device__ void decide_chunk(MsWork w, int k, int max_iters, int et_period, int B, int32_t *synd) {
  constexpr int kWaves = kDecideThreads / 64;
  __shared__ uint64_t part[kWaves];
  const int lane = threadIdx.x & 63;
  const int64_t chunks = w.chunks;
  uint64_t odd = 0;
  if (w.live_w[k])
    for (int i = threadIdx.x; i < w.check_waves; i += kDecideThreads)
      odd |= w.odd[(int64_t)i * chunks + k];
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)odd, off), hi = __shfl_xor((uint32_t)(odd >> 32), off);
    odd |= ((uint64_t)hi << 32) | lo;
  }
  if (lane == 0) part[threadIdx.x >> 6] = odd;
  __syncthreads();
  if (threadIdx.x >= 64) return;
  odd = 0;
#pragma unroll
  for (int i = 0; i < kWaves; ++i) odd |= part[i];
  const int slot = k * 64 + lane;
  const int it = w.it[slot], f = w.frame[slot];
  const bool running = f >= 0;
  const bool unsat = lane_bit(odd, lane) != 0;
  const bool stop = running && it >= 1 &&
                    (it >= max_iters || (it % et_period == 0 && !unsat));
  const bool want = stop || !running;
  const uint64_t wm = __ballot(want);
  int base = 0;
  if (lane == 0 && wm) base = atomicAdd(&w.ctrl[0], __popcll(wm));
  base = __shfl(base, 0);
  const int rank = __popcll(wm & ((1ull << lane) - 1ull));
  const int nf = want && base + rank < B ? base + rank : -1;
  const bool fill = nf >= 0;
  const bool run = running && !stop;
  if (stop) w.used[slot] = it;
  if (stop && synd) synd[f] = 0;  // ms_post adds the weight of frames stopped at the cap
  w.nxt[slot] = want ? nf : f;
  w.it[slot] = run ? it + 1 : 0;
  const uint64_t sw = __ballot(stop), rw = __ballot(run), fw = __ballot(fill);
  const uint64_t cw = __ballot(stop && unsat);
  if (lane == 0) {
    w.stop_w[k] = sw;
    w.run_w[k] = rw;
    w.fill_w[k] = fw;
    w.cap_w[k] = cw;
    w.live_w[k] = rw | fw;
    if (sw) atomicAdd(&w.ctrl[1], __popcll(sw));
  }
}

// Outputs of the frames that stopped in this pass: packed info bits (bits
// M.., MSB first, :207-219) through an LDS transpose and iterations
// (decide_chunk zeroed their syndrome weight; flush_synd adds it for the
// frames stopped at the cap).
__device__ void flush_packed(const GraphView &g, const MsWork &w, const DecodeArgs &a, int bx,
                             int k) {
  const uint64_t sel = w.stop_w[k];
  if (!sel) return;
  __shared__ uint8_t tile[64][65];
  __shared__ uint64_t hw[512];  // hard words of the block's 512 columns (one vector load each)
  const int q0 = bx * 64, lane = threadIdx.x & 63, wv = wave_id();
  const int64_t chunks = w.chunks;
  for (int i = threadIdx.x; i < 512; i += 256) {
    const int c = g.M + q0 * 8 + i;
    hw[i] = c < g.N ? w.hard[(int64_t)c * chunks + k] : 0ull;
  }
  __syncthreads();
  for (int qq = wv; qq < 64; qq += 4) {
    unsigned o = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) o |= (unsigned)lane_bit(hw[qq * 8 + j], lane) << (7 - j);
    tile[lane][qq] = (uint8_t)o;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int f = i >> 6, qq = i & 63, q = q0 + qq;
    if (lane_bit(sel, f) && q < g.KB) a.packed[(int64_t)w.frame[k * 64 + f] * g.KB + q] = tile[f][qq];
  }
  if (bx == 0 && threadIdx.x < 64 && lane_bit(sel, threadIdx.x)) {
    const int slot = k * 64 + threadIdx.x, fr = w.frame[slot];
    if (a.iters) a.iters[fr] = w.used[slot];
  }
}

// Full hard decisions (B x N bytes) and posteriors (B x N floats) of the
// frames that stopped.
__global__ void __launch_bounds__(256) ms_flush_cols(GraphView g, MsWork w, uint8_t *bits,
                                                     float *llr) {
  const int k = blockIdx.y;
  const uint64_t sel = w.stop_w[k];
  if (!sel) return;
  __shared__ float tile[64][65];
  __shared__ uint8_t btile[64][65];
  const int c0 = blockIdx.x * 64, lane = threadIdx.x & 63, wv = wave_id();
  for (int cc = wv; cc < 64; cc += 4) {
    const int c = c0 + cc;
    btile[lane][cc] = c < g.N ? (uint8_t)lane_bit(w.hard[(int64_t)c * w.chunks + k], lane) : 0;
    if (llr) tile[lane][cc] = c < g.N ? w.post[at(c, k, g.N, lane)] : 0.0f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int f = i >> 6, cc = i & 63, c = c0 + cc;
    if (!lane_bit(sel, f) || c >= g.N) continue;
    const int64_t fr = w.frame[k * 64 + f];
    if (bits) bits[fr * g.N + c] = btile[f][cc];
    if (llr) llr[fr * g.N + c] = tile[f][cc];
  }
}

__device__ void flush_synd_rows(const GraphView &g, const MsWork &w, int32_t *synd, int bx, int k);

// Uncapped syndrome weight of the frames that stopped at the cap with
// unsatisfied checks (added to the zero decide_chunk wrote).  nb blocks per
// chunk stride over the check waves' row groups: a pass where no frame
// stopped at the cap (most) costs nb near-empty blocks, not one per group.
__device__ void flush_synd(const GraphView &g, const MsWork &w, int32_t *synd, int bx, int nb,
                           int k) {
  const uint64_t sel = w.cap_w[k];
  if (!sel || !synd) return;
  for (int grp = bx; grp < w.check_waves / 4; grp += nb) flush_synd_rows(g, w, synd, grp, k);
}

__device__ void flush_synd_rows(const GraphView &g, const MsWork &w, int32_t *synd, int bx, int k) {
  const uint64_t sel = w.cap_w[k];
  const int lane = threadIdx.x & 63;
  const int64_t chunks = w.chunks;
  const int j0 = (bx * 4 + wave_id()) * kMsRows;
  const int j1 = min(j0 + kMsRows, g.M);
  if (j0 >= j1) return;
  int cnt = 0;
  const int eb = g.rp[j0], ne = g.rp[j1] - eb;
  if (g.dc_max * kMsRows <= 64) {  // the rows' edges in the wave's lanes (check_rows_lanes)
    const uint64_t my_h = lane < ne ? w.hard[(int64_t)g.ci[eb + lane] * chunks + k] : 0ull;
    for (int j = j0; j < j1; ++j) {
      uint64_t par = 0;
      const int e0 = g.rp[j] - eb, d = g.rp[j + 1] - g.rp[j];
      for (int t = 0; t < d; ++t) par ^= readlane64(my_h, e0 + t);
      cnt += (int)lane_bit(par, lane);
    }
  } else {
    for (int j = j0; j < j1; ++j) {
      uint64_t par = 0;
      const int e1 = g.rp[j + 1];
      for (int e = g.rp[j]; e < e1; ++e) par ^= w.hard[(int64_t)g.ci[e] * chunks + k];
      cnt += (int)lane_bit(par, lane);
    }
  }
  if (cnt && lane_bit(sel, lane)) atomicAdd(&synd[w.frame[k * 64 + lane]], cnt);
}

// blocks [0, nb_flush): flush_packed; the rest: flush_synd
__global__ void __launch_bounds__(256) ms_post(GraphView g, MsWork w, DecodeArgs a, int nb_flush) {
  const int k = blockIdx.y;
  if ((int)blockIdx.x < nb_flush)
    flush_packed(g, w, a, blockIdx.x, k);
  else
    flush_synd(g, w, a.synd, blockIdx.x - nb_flush, (int)gridDim.x - nb_flush, k);
}

// Vertical step (:379-403) for the running slots: L(r_ji) of every edge of
// the column from its row's state, s = sum_j L(r_ji) in ascending j,
// LQ = Lci + s, vhat = LQ < 0.
template <typename Real, int DV>
__global__ void __launch_bounds__(256) ms_var_fill(GraphView g, MsWork w, DecodeArgs a) {
  const int k = blockIdx.y;
  const uint64_t run = w.run_w[k], fill = w.fill_w[k];
  const int lane = threadIdx.x & 63;
  if (blockIdx.x == 0 && threadIdx.x < 64) {  // the slots' frames move on (after ms_post)
    const int slot = k * 64 + threadIdx.x;
    if (lane_bit(w.stop_w[k] | fill, threadIdx.x)) w.frame[slot] = w.nxt[slot];
  }
  if (!(run | fill)) return;
  const bool filling = lane_bit(fill, lane) != 0;
  // a refilled slot's new frame (the decide's choice)
  const float *src = filling ? a.in + (int64_t)w.nxt[k * 64 + lane] * a.cw_stride : nullptr;
  const int64_t chunks = w.chunks;
  const Real *m1 = (const Real *)w.m1, *m2 = (const Real *)w.m2;
  Real *LQ = (Real *)w.LQ;
  const int c0 = (blockIdx.x * 4 + wave_id()) * kMsCols;
  // the wave's columns' CSC edges are consecutive: lane l takes edge cp[c0] + l
  // (its row, its place in the row, its alpha words) with one vector load
  // each, when they fit the wave (as check_rows_lanes)
  int kb = 0, my_j = 0, my_pos = 0;
  uint64_t my_neg = 0, my_zero = 0;
  bool lanes_meta = false;
#ifndef LDPC_MS_SCALAR_META
  if constexpr (DV * kMsCols <= 64) {
    if (run && c0 < g.N) {
      lanes_meta = true;
      kb = g.cp[c0];
      const int ne = g.cp[min(c0 + kMsCols, g.N)] - kb;
      if (lane < ne) {
        const int e = g.ce[kb + lane];
        my_j = g.cr[kb + lane];
        my_pos = e - g.rp[my_j];
        const uint64_t *aw = w.alpha + ((int64_t)e * chunks + k) * 2;
        my_neg = aw[0];
        my_zero = aw[1];
      }
    }
  }
#endif
  for (int cc = 0; cc < kMsCols; ++cc) {
    const int c = c0 + cc;
    if (c >= g.N) break;
    // Lci = -tx as float (exact: tx is a float), LQ = Lci (:318-321, :328-331)
    const float xf = filling ? -(src[(int64_t)c * a.elem_stride] * a.polarity) : 0.0f;
    if (filling) w.L[at(c, k, g.N, lane)] = xf;
    if (!run) {  // only refills in this chunk
      if (filling) LQ[at(c, k, g.N, lane)] = (Real)xf;
      continue;
    }
    const int k0 = g.cp[c], d = g.cp[c + 1] - k0;
    const Real lci = filling ? (Real)xf : (Real)w.L[at(c, k, g.N, lane)];
    Real r[DV];
    if (lanes_meta) {
      // this column's edges are lanes k0 - kb .. of the wave's edge lanes
      const int l0 = k0 - kb;
#pragma unroll
      for (int t = 0; t < DV; ++t) {
        r[t] = Real(0);
        if (t < d) {
          const int j = __builtin_amdgcn_readlane(my_j, l0 + t);
          const int pos = __builtin_amdgcn_readlane(my_pos, l0 + t);
          const int64_t ro = at(j, k, g.M, lane);
          const int mt = w.meta[ro];
          const int al = alpha_of(readlane64(my_neg, l0 + t), readlane64(my_zero, l0 + t), lane);
          r[t] = (Real)(((mt >> 6) - 1) * al) * (pos == (mt & 63) - 1 ? m2[ro] : m1[ro]);
        }
      }
    } else {
#pragma unroll
      for (int t = 0; t < DV; ++t) {
        r[t] = Real(0);
        if (t < d) {
          const int e = g.ce[k0 + t], j = g.cr[k0 + t];
          const int pos = e - g.rp[j];  // the edge's place in its row
          const int64_t ro = at(j, k, g.M, lane);
          const int mt = w.meta[ro];
          const uint64_t *aw = w.alpha + ((int64_t)e * chunks + k) * 2;
          const int al = alpha_of(aw[0], aw[1], lane);
          r[t] = (Real)(((mt >> 6) - 1) * al) * (pos == (mt & 63) - 1 ? m2[ro] : m1[ro]);
        }
      }
    }
    Real s = Real(0);
#pragma unroll
    for (int t = 0; t < DV; ++t)
      if (t < d) s = s + r[t];
    // a refilled lane's row states are stale: its sum is dead, LQ = Lci
    const Real lq = filling ? lci : lci + s;
    LQ[at(c, k, g.N, lane)] = lq;
    const uint64_t bw = __ballot(lq < Real(0));
    if (lane == 0) w.hard[(int64_t)c * chunks + k] = bw;
    if (w.post) w.post[at(c, k, g.N, lane)] = (float)lq;
  }
}

__global__ void ms_init(MsWork w) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < w.S; i += gridDim.x * blockDim.x) {
    w.frame[i] = -1;
    w.it[i] = 0;
  }
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < w.chunks; k += gridDim.x * blockDim.x) {
    w.live_w[k] = 0;
    w.run_w[k] = w.stop_w[k] = w.fill_w[k] = w.cap_w[k] = 0;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    w.ctrl[0] = 0;
    w.ctrl[1] = 0;
  }
}

int ms_check_waves(const GraphView &g) { return 4 * ((g.M + 4 * kMsRows - 1) / (4 * kMsRows)); }

template <int PREC>
void ms_pass(const GraphView &g, const MsWork &w, const DecodeArgs &a, int method_iters,
             hipStream_t st) {
  typedef typename Math<PREC>::Real Real;
  const dim3 rgrid(w.check_waves / 4, w.chunks);
  const dim3 cgrid((g.N + 4 * kMsCols - 1) / (4 * kMsCols), w.chunks);
  const dim3 tgrid((g.N + 63) / 64, w.chunks);
  if (g.dc_max <= 8)
    ms_check<PREC, 8><<<rgrid, 256, 0, st>>>(g, w);
  else if (g.dc_max <= 16)
    ms_check<PREC, 16><<<rgrid, 256, 0, st>>>(g, w);
  else
    ms_check<PREC, 32><<<rgrid, 256, 0, st>>>(g, w);
  ms_decide<<<w.chunks, kDecideThreads, 0, st>>>(w, method_iters, a.et_period, a.B, a.synd);
  if (a.bits || (a.llr && w.post)) ms_flush_cols<<<tgrid, 256, 0, st>>>(g, w, a.bits, a.llr);
  const int nb_flush = (g.KB + 63) / 64;
  const int nb_synd = std::min(64, std::max(1, w.check_waves / 4));
  ms_post<<<dim3(nb_flush + nb_synd, w.chunks), 256, 0, st>>>(g, w, a, nb_flush);
  if (g.dv_max <= 4)
    ms_var_fill<Real, 4><<<cgrid, 256, 0, st>>>(g, w, a);
  else if (g.dv_max <= 8)
    ms_var_fill<Real, 8><<<cgrid, 256, 0, st>>>(g, w, a);
  else
    ms_var_fill<Real, 16><<<cgrid, 256, 0, st>>>(g, w, a);
}

}  // namespace

int ms_default_slots() {
  const char *e = getenv("LDPC_MS_SLOTS");  // A/B knob
  const int v = e ? atoi(e) : 0;
  return v >= 64 ? v / 64 * 64 : 128;
}

size_t ms_work_bytes(const GraphView &g, int S, int prec, bool want_post) {
  const size_t real = prec == 1 ? 4 : 8;
  const size_t chunks = (size_t)S / 64;
  size_t n = al256((size_t)g.N * S * 4) + al256((size_t)g.N * S * real);  // L, LQ
  n += 2 * al256((size_t)g.M * S * real) + al256((size_t)g.M * S);        // m1, m2, meta
  n += al256((size_t)g.E * chunks * 16);                                  // alpha
  n += al256((size_t)g.N * chunks * 8);                                   // hard
  if (want_post) n += al256((size_t)g.N * S * 4);
  n += al256((size_t)ms_check_waves(g) * chunks * 8);                     // odd
  n += 4 * al256((size_t)S * 4);                                          // it, frame, nxt, used
  n += 6 * al256(chunks * 8) + al256(64);                                 // masks, ctrl
  return n;
}

void ms_work_carve(MsWork &w, void *base, const GraphView &g, int S, int prec, bool want_post) {
  const size_t real = prec == 1 ? 4 : 8;
  const size_t chunks = (size_t)S / 64;
  char *p = (char *)base;
  auto take = [&](size_t bytes) {
    char *r = p;
    p += al256(bytes);
    return (void *)r;
  };
  w = MsWork{};
  w.S = S;
  w.chunks = (int)chunks;
  w.check_waves = ms_check_waves(g);
  w.L = (float *)take((size_t)g.N * S * 4);
  w.LQ = take((size_t)g.N * S * real);
  w.m1 = take((size_t)g.M * S * real);
  w.m2 = take((size_t)g.M * S * real);
  w.meta = (uint8_t *)take((size_t)g.M * S);
  w.alpha = (uint64_t *)take((size_t)g.E * chunks * 16);
  w.hard = (uint64_t *)take((size_t)g.N * chunks * 8);
  w.post = want_post ? (float *)take((size_t)g.N * S * 4) : nullptr;
  w.odd = (uint64_t *)take((size_t)w.check_waves * chunks * 8);
  w.it = (int32_t *)take((size_t)S * 4);
  w.frame = (int32_t *)take((size_t)S * 4);
  w.nxt = (int32_t *)take((size_t)S * 4);
  w.used = (int32_t *)take((size_t)S * 4);
  w.live_w = (uint64_t *)take(chunks * 8);
  w.run_w = (uint64_t *)take(chunks * 8);
  w.stop_w = (uint64_t *)take(chunks * 8);
  w.fill_w = (uint64_t *)take(chunks * 8);
  w.cap_w = (uint64_t *)take(chunks * 8);
  take(chunks * 8);
  w.ctrl = (int32_t *)take(64);
}

int launch_graph_decode_ms(const GraphView &g, const MsWork &w, const DecodeArgs &a, int prec,
                           int32_t *h_ctrl, void *stream) {
  if (g.dc_max > kGraphDcMax || g.dv_max > kGraphDvMax) return -2;
  if (a.B <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  ms_init<<<std::max(1, std::min(64, (w.S + 255) / 256)), 256, 0, st>>>(w);
  // a slot finishes a frame at least every max_iters + 1 passes, so the pool
  // drains within ceil(B/S) (max+1) passes and the last frames finish
  // within max+1 more; passes past the end return at once (empty chunks)
  const int64_t bound = ((int64_t)(a.B + w.S - 1) / w.S + 1) * (a.max_iters + 1) + 2;
  // Default: the host reads the progress counter back every kRound passes
  // (one round behind, so the GPU never waits) and stops enqueueing when
  // every frame is done -- the call returns once the decode has finished.
  // LDPC_MS_ASYNC=1: all `bound` passes are enqueued and the call returns at
  // once, like the other ldpc_decode_device paths; the passes after the last
  // frame find no running chunk and return, but with 128 slots the bound is
  // ~3x the passes a 2 dB batch needs and the empty ones cost 11 % of config
  // 4's throughput (profiles/round3/ab_ms_async.txt).
  static const bool async = getenv("LDPC_MS_ASYNC") && getenv("LDPC_MS_ASYNC")[0] == '1';
  if (async) {
    for (int64_t pass = 0; pass < bound; ++pass) {
      if (prec == 1)
        ms_pass<1>(g, w, a, a.max_iters, st);
      else
        ms_pass<0>(g, w, a, a.max_iters, st);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  const int kRound = 8;
  hipEvent_t ev[2] = {nullptr, nullptr};
  for (int i = 0; i < 2; ++i)
    if (hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return -1;
  int rc = 0;
  int64_t pass = 0;
  for (int round = 0; pass < bound; ++round) {
    for (int i = 0; i < kRound && pass < bound; ++i, ++pass) {
      if (prec == 1)
        ms_pass<1>(g, w, a, a.max_iters, st);
      else
        ms_pass<0>(g, w, a, a.max_iters, st);
    }
    // progress of this round, read back when the next round is queued
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

}  // namespace ldpc
