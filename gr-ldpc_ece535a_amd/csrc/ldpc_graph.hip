// ldpc_graph.hip -- large-code decode kernels for gfx950 (MI355X).
//
// The small-code kernel (ldpc_kernels.hip) keeps a whole frame in one wave's
// registers and LDS.  A DVB-S2-size code (E = 226799 edges) does not fit, so
// this path keeps the messages in HBM and runs each iteration of the
// reference's loop as separate grid-wide passes over the Tanner graph
// (lib/ldpc_decoder_cb_impl.cc: sum-product :500-553, bit-flip :439-473;
// min-sum has its own frame pipeline, ldpc_graph_msn.hip):
//
//   g_check   one wave = 8 check rows x 64 frames: reads each row's Q
//             messages, writes its R messages (horizontal step), and -- from
//             the bit-packed hard decision of the previous iteration -- the
//             rows' parities, OR-ed into one 64-bit "odd row seen" word;
//   g_decide  one wave per 64-frame chunk: ORs those words; a frame whose
//             checks are all satisfied stops, under the reference's rule
//             (min-sum / bit-flip only when it+1 < iterations; et_period
//             thins the checks); a chunk whose frames all stopped is skipped
//             from then on;
//   g_var     one wave = 8 columns x 64 frames: column sums, hard decision
//             (a 64-bit ballot per column), new Q messages (vertical step).
//
// Per-frame arrays are chunk-major, frame-minor ((k * n + x) * 64 + lane for
// element x of frame 64k + lane): a wave moves 64 consecutive values of one
// edge per access, a full aligned 512-byte (f64) or 256-byte (f32)
// transaction, and a check row's edges are adjacent blocks.  Inside a chunk that is still running every lane computes and
// stores, stopped frames included (their messages are dead data), so no
// store is a partial line; a stopped frame's hard decision and posterior are
// frozen by masking instead.  Per frame-iteration the sum-product traffic is
// 2E x sizeof(Real) read + 2E x sizeof(Real) written + 4N channel bytes.  A stopped chunk costs one flag read per block.
//
// The per-edge arithmetic is the reference's, in its order, with the same
// Math<PREC> as the small-code kernel (ldpc_device.hpp).
#include <hip/hip_runtime.h>

#include <algorithm>

#include <stdlib.h>

#include "ldpc_device.hpp"
#include "ldpc_graph.hpp"

namespace ldpc {
namespace {

#ifndef LDPC_GRAPH_ROWS_PER_WAVE
#define LDPC_GRAPH_ROWS_PER_WAVE 4
#endif
#ifndef LDPC_GRAPH_COLS_PER_WAVE
#define LDPC_GRAPH_COLS_PER_WAVE 4
#endif
constexpr int kRowsPerWave = LDPC_GRAPH_ROWS_PER_WAVE;
constexpr int kColsPerWave = LDPC_GRAPH_COLS_PER_WAVE;

__device__ __forceinline__ int wave_in_block() {
  return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

__device__ __forceinline__ uint64_t bit_of(uint64_t w, int lane) { return (w >> lane) & 1ull; }

size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

// Element x (an edge or a column) of frame lane in chunk k: chunk-major, so
// one chunk's values of consecutive edges are consecutive 64-lane blocks
// (a check row's messages are one contiguous run).
__device__ __forceinline__ int64_t at(int64_t x, int k, int64_t n, int lane) {
  return ((int64_t)k * n + x) * 64 + lane;
}

// The group's live buffers (compaction swaps them on the device).
__device__ __forceinline__ GraphWork live(GraphWork w) {
  const GraphState *st = w.st;
  w.Q = st->Q;
  w.R = st->R;
  w.L = st->L;
  w.post = st->post;
  w.hard = st->hard;
  w.perm = st->perm;
  return w;
}

// Slot b holds a frame of this group (compaction empties slots).
__device__ __forceinline__ bool valid_slot(const GraphWork &w, int64_t b) { return w.perm[b] >= 0; }

// One wave per chunk: counters, padding frames (b >= B) marked stopped.
__global__ void __launch_bounds__(64) g_reset(GraphWork w, int B, int used0) {
  const int k = blockIdx.x, lane = threadIdx.x;
  const int b = k * 64 + lane;
  w.used[b] = used0;
  w.synd[b] = 0;
  w.perm[b] = b < B ? b : -1;
  const uint64_t pad = __ballot(b >= B);
  if (lane == 0) {
    w.done_w[k] = pad;
    w.chunk_done[k] = 0;
  }
  if (k == 0 && lane == 0) {
    GraphState *st = w.st;
    st->Q = w.Q;
    st->R = w.R;
    st->L = w.L;
    st->post = w.post;
    st->hard = w.hard;
    st->perm = w.perm;
    st->L2 = w.L2;
    st->post2 = w.post2;
    st->hard2 = w.hard2;
    st->perm2 = w.perm2;
    st->slots = w.Bp;
    st->n_new = 0;
    st->flag = 0;
  }
}

// Channel samples -> per-column arrays through an LDS transpose: the block
// reads 64 frames x 64 samples row by row (coalesced along the frame) and
// writes 64 columns x 64 frames.  tx = in * polarity (:149-153).
//   SOFT (methods 0/1): L = -tx (Lci :318-321 / r :486), Q = L on every edge
//        of the column (:328-331, :489-496);
//   else (methods 2/3): y = hard decision of tx (:424-431, :563-569).
template <typename Real, bool SOFT>
__global__ void __launch_bounds__(256) g_load(GraphView g, GraphWork w_, const float *in,
                                              int64_t cw_stride, int elem_stride,
                                              float polarity, int B) {
  const GraphWork w = live(w_);
  __shared__ float tile[64][65];
  const int c0 = blockIdx.x * 64, k = blockIdx.y, b0 = k * 64;
  const int lane = threadIdx.x & 63, wv = wave_in_block();
  for (int f = wv; f < 64; f += 4) {
    const int b = b0 + f, c = c0 + lane;
    float x = 0.0f;
    if (b < B && c < g.N) x = in[(int64_t)b * cw_stride + (int64_t)c * elem_stride] * polarity;
    tile[f][lane] = x;
  }
  __syncthreads();
  for (int cc = wv; cc < 64; cc += 4) {
    const int c = c0 + cc;
    if (c >= g.N) break;
    const float x = tile[lane][cc];
    if (w.post) w.post[at(c, k, g.N, lane)] = x;  // hard / bit-flip report tx
    if constexpr (SOFT) {
      w.L[at(c, k, g.N, lane)] = -x;
      const Real l = -(Real)x;
      Real *Q = (Real *)w.Q;
      const int k1 = g.cp[c + 1];
      for (int e = g.cp[c]; e < k1; ++e) Q[at(g.ce[e], k, g.E, lane)] = l;
    } else {
      const uint64_t yw = __ballot(!(x < 0.0f));
      if (lane == 0) {
        w.hard[(int64_t)c * w.chunks + k] = yw;
        w.y[(int64_t)c * w.chunks + k] = yw;
      }
    }
  }
}

// Horizontal step for kRowsPerWave rows x 64 frames per wave.  For h > 0 the
// same pass evaluates checkFrame's rows (:236-253) on the hard decision of
// iteration h-1: 64 frames per XOR of packed words.
template <int PREC, int DC>
__global__ void __launch_bounds__(256) g_check(GraphView g, GraphWork w_, int h) {
  const GraphWork w = live(w_);
  typedef typename Math<PREC>::Real Real;
  const int k = blockIdx.y;
  __shared__ typename Math<PREC>::Tab logtab[TabLds<PREC>::kN];
  if constexpr (Math<PREC>::kTabN > 0) {
    if (w.chunk_done[k]) return;  // uniform per block: no thread misses the barrier
    stage_tab<PREC>(logtab);
  }
  if (w.chunk_done[k]) return;
  const int lane = threadIdx.x & 63;
  const int64_t chunks = w.chunks;
  const Real *Q = (const Real *)w.Q + at(0, k, g.E, lane);
  Real *R = (Real *)w.R + at(0, k, g.E, lane);
  const int wg = blockIdx.x * 4 + wave_in_block();
  const int j0 = wg * kRowsPerWave;
  // parities first: their scalar loads then issue back to back instead of
  // queueing behind each row's message stores
  uint64_t odd = 0;
  if (h > 0) {
    const int j1 = min(j0 + kRowsPerWave, g.M);
    for (int j = j0; j < j1; ++j) {
      uint64_t par = 0;
      const int e1 = g.rp[j + 1];
      for (int e = g.rp[j]; e < e1; ++e) par ^= w.hard[(int64_t)g.ci[e] * chunks + k];
      odd |= par;
    }
  }
  for (int jj = 0; jj < kRowsPerWave; ++jj) {
    const int j = j0 + jj;
    if (j >= g.M) break;
    const int e0 = g.rp[j], d = g.rp[j + 1] - e0;
    Real q[DC];
#pragma unroll
    for (int t = 0; t < DC; ++t) q[t] = t < d ? Q[(int64_t)(e0 + t) * 64] : Real(0);
    // E(j,i) = log((1+T)/(1-T)), T = prod_{k != i} tanh(M(j,k)/2) in
    // ascending k (:503-516)
#pragma unroll
    for (int t = 0; t < DC; ++t)
      if (t < d) q[t] = Math<PREC>::tanh_half(q[t], logtab);
    for (int e = 0; e < d; ++e) {
      Real T = Real(1);
#pragma unroll
      for (int t = 0; t < DC; ++t) T = (t != e && t < d) ? T * q[t] : T;
      R[(int64_t)(e0 + e) * 64] = Math<PREC>::check_msg(T, logtab);
    }
  }
  if (h > 0 && lane == 0) w.synd_part[(int64_t)wg * chunks + k] = odd;
}

// Bit-flip: parity words of each row over the hard decision of iteration h-1
// (the received y for h == 0), :443-452; E(i,j) of an edge is parity ^ ci(j).
__global__ void __launch_bounds__(256) g_check_bf(GraphView g, GraphWork w_, int h) {
  const GraphWork w = live(w_);
  const int k = blockIdx.y;
  if (w.chunk_done[k]) return;
  const int64_t chunks = w.chunks;
  const int wg = blockIdx.x * 4 + wave_in_block();
  const int j0 = wg * kRowsPerWave;
  uint64_t odd = 0;
  for (int jj = 0; jj < kRowsPerWave; ++jj) {
    const int j = j0 + jj;
    if (j >= g.M) break;
    const int e0 = g.rp[j], d = g.rp[j + 1] - e0;
    uint64_t par = 0;
    for (int t = 0; t < d; ++t) par ^= w.hard[(int64_t)g.ci[e0 + t] * chunks + k];
    if (threadIdx.x % 64 == 0) w.rowpar[(int64_t)j * chunks + k] = par;
    odd |= par;
  }
  if (h > 0 && threadIdx.x % 64 == 0) w.synd_part[(int64_t)wg * chunks + k] = odd;
}

// Early exit after iteration h-1 (:406-408, :470-472, :535-537): a frame
// whose hard decision satisfies every check stops with h iterations
// executed, when h < max_iters (the reference's min-sum / bit-flip rule; for
// sum-product stopping at the last iteration changes nothing) and
// h % et_period == 0.  One wave per 64-frame chunk.
__global__ void __launch_bounds__(256) g_decide(GraphWork w, int h, int max_iters, int et_period) {
  __shared__ uint64_t part[4];
  const int k = blockIdx.x, lane = threadIdx.x & 63;
  if (w.chunk_done[k]) return;
  const int64_t chunks = w.chunks;
  uint64_t odd = 0;
  for (int i = threadIdx.x; i < w.check_waves; i += 256) odd |= w.synd_part[(int64_t)i * chunks + k];
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)odd, off), hi = __shfl_xor((uint32_t)(odd >> 32), off);
    odd |= ((uint64_t)hi << 32) | lo;
  }
  if (lane == 0) part[threadIdx.x >> 6] = odd;
  __syncthreads();
  if (threadIdx.x >= 64) return;
  odd = part[0] | part[1] | part[2] | part[3];
  if (!(h < max_iters && h % et_period == 0)) return;
  const uint64_t done = w.done_w[k];
  const uint64_t newly = ~odd & ~done;
  if (bit_of(newly, lane)) w.used[(int64_t)k * 64 + lane] = h;
  if (lane == 0) {
    w.done_w[k] = done | newly;
    if ((done | newly) == ~0ull) w.chunk_done[k] = 1;
  }
}

// Vertical step for kColsPerWave columns x 64 frames per wave (sum-product):
// L = sum_j (E(j,i) + r) (:519-532), vhat = L <= 0, and
// M(j,i) = sum_{k != j} (E(k,i) + r) (:540-553), both ascending.
template <typename Real, int DV>
__global__ void __launch_bounds__(256) g_var(GraphView g, GraphWork w_) {
  const GraphWork w = live(w_);
  const int k = blockIdx.y;
  if (w.chunk_done[k]) return;
  const int lane = threadIdx.x & 63;
  const int64_t chunks = w.chunks;
  const uint64_t done = w.done_w[k];
  const bool frozen = bit_of(done, lane) != 0;
  const Real *R = (const Real *)w.R + at(0, k, g.E, lane);
  Real *Q = (Real *)w.Q + at(0, k, g.E, lane);
  const int c0 = (blockIdx.x * 4 + wave_in_block()) * kColsPerWave;
  for (int cc = 0; cc < kColsPerWave; ++cc) {
    const int c = c0 + cc;
    if (c >= g.N) break;
    const int k0 = g.cp[c], d = g.cp[c + 1] - k0;
    const Real rc = (Real)w.L[at(c, k, g.N, lane)];
    int e[DV];
    Real r[DV];
#pragma unroll
    for (int t = 0; t < DV; ++t) {
      e[t] = t < d ? g.ce[k0 + t] : 0;
      r[t] = t < d ? R[(int64_t)e[t] * 64] : Real(0);
    }
    Real tot = Real(0);
    bool bit;
#pragma unroll
    for (int t = 0; t < DV; ++t)
      if (t < d) tot = tot + (r[t] + rc);
    bit = tot <= Real(0);
#pragma unroll
    for (int s = 0; s < DV; ++s)
      if (s < d) {
        Real T = Real(0);
#pragma unroll
        for (int t = 0; t < DV; ++t) T = (t != s && t < d) ? T + (r[t] + rc) : T;
        Q[(int64_t)e[s] * 64] = T;
      }
    const uint64_t bw = __ballot(bit);
    if (lane == 0) {
      uint64_t *hw = &w.hard[(int64_t)c * chunks + k];
      *hw = done ? ((*hw & done) | (bw & ~done)) : bw;
    }
    if (w.post) {
      float *pp = &w.post[at(c, k, g.N, lane)];
      const float pv = frozen ? *pp : (float)tot;
      *pp = pv;
    }
  }
}

// Bit-flip vote (:453-467): column i becomes 1 - y(i) when more than M/2 of
// its checks disagree with y(i) (parity ^ vhat(i) != y(i)), else keeps vhat(i).
template <int DV>
__global__ void __launch_bounds__(256) g_var_bf(GraphView g, GraphWork w_) {
  const GraphWork w = live(w_);
  const int k = blockIdx.y;
  if (w.chunk_done[k]) return;
  const int lane = threadIdx.x & 63;
  const int64_t chunks = w.chunks;
  const uint64_t done = w.done_w[k];
  const int half = (int)((unsigned)g.M / 2u);
  const int c0 = (blockIdx.x * 4 + wave_in_block()) * kColsPerWave;
  for (int cc = 0; cc < kColsPerWave; ++cc) {
    const int c = c0 + cc;
    if (c >= g.N) break;
    const int k0 = g.cp[c], d = g.cp[c + 1] - k0;
    const uint64_t hw = w.hard[(int64_t)c * chunks + k], yw = w.y[(int64_t)c * chunks + k];
    int votes = 0;
#pragma unroll
    for (int t = 0; t < DV; ++t)
      if (t < d) votes += (int)bit_of(w.rowpar[(int64_t)g.cr[k0 + t] * chunks + k] ^ hw ^ yw, lane);
    const bool nb = votes > half ? !bit_of(yw, lane) : bit_of(hw, lane) != 0;
    const uint64_t bw = __ballot(nb);
    if (lane == 0) w.hard[(int64_t)c * chunks + k] = (hw & done) | (bw & ~done);
  }
}

// Final syndrome weight (uncapped checkFrame) of every frame's decision.
__global__ void __launch_bounds__(256) g_synd(GraphView g, GraphWork w_, int B) {
  const GraphWork w = live(w_);
  const int k = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int64_t chunks = w.chunks;
  const int64_t b = (int64_t)k * 64 + lane;
  const int j0 = (blockIdx.x * 4 + wave_in_block()) * kRowsPerWave;
  int cnt = 0;
  for (int jj = 0; jj < kRowsPerWave; ++jj) {
    const int j = j0 + jj;
    if (j >= g.M) break;
    const int e0 = g.rp[j], d = g.rp[j + 1] - e0;
    uint64_t par = 0;
    for (int t = 0; t < d; ++t) par ^= w.hard[(int64_t)g.ci[e0 + t] * chunks + k];
    cnt += (int)bit_of(par, lane);
  }
  if (cnt && b < B && valid_slot(w, b)) atomicAdd(&w.synd[b], cnt);
}

// Outputs, transposed back to frame-major through LDS: packed info bytes
// (bits M.., MSB first, :207-219), and the per-frame counters.
// flush = 1: only frames that stopped, written before a compaction drops them.
__global__ void __launch_bounds__(256) g_store_packed(GraphView g, GraphWork w_, DecodeArgs a,
                                                      int flush) {
  const GraphWork w = live(w_);
  if (flush && !w.st->flag) return;
  __shared__ uint8_t tile[64][65];
  const int q0 = blockIdx.x * 64, k = blockIdx.y, b0 = k * 64;
  const uint64_t sel = flush ? w.done_w[k] : ~0ull;
  const int lane = threadIdx.x & 63, wv = wave_in_block();
  const int64_t chunks = w.chunks;
  for (int qq = wv; qq < 64; qq += 4) {
    const int q = q0 + qq;
    unsigned o = 0;
    if (q < g.KB)
      for (int j = 0; j < 8; ++j) {
        const int c = g.M + q * 8 + j;
        if (c < g.N) o |= (unsigned)bit_of(w.hard[(int64_t)c * chunks + k], lane) << (7 - j);
      }
    tile[lane][qq] = (uint8_t)o;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int f = i >> 6, qq = i & 63;
    const int fr = w.perm[b0 + f], q = q0 + qq;
    if (fr >= 0 && bit_of(sel, f) && q < g.KB) a.packed[(int64_t)fr * g.KB + q] = tile[f][qq];
  }
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    const int b = b0 + threadIdx.x, fr = w.perm[b];
    if (fr >= 0 && bit_of(sel, threadIdx.x)) {
      if (a.iters) a.iters[fr] = w.used[b];
      if (a.synd) a.synd[fr] = w.synd[b];  // 0 for a frame that stopped
    }
  }
}

// Full hard decision, B x N bytes.
__global__ void __launch_bounds__(256) g_store_bits(GraphView g, GraphWork w_, uint8_t *dst, int B,
                                                    int flush) {
  const GraphWork w = live(w_);
  if (flush && !w.st->flag) return;
  __shared__ uint8_t tile[64][65];
  const int c0 = blockIdx.x * 64, k = blockIdx.y, b0 = k * 64;
  const uint64_t sel = flush ? w.done_w[k] : ~0ull;
  const int lane = threadIdx.x & 63, wv = wave_in_block();
  for (int cc = wv; cc < 64; cc += 4) {
    const int c = c0 + cc;
    tile[lane][cc] = c < g.N ? (uint8_t)bit_of(w.hard[(int64_t)c * w.chunks + k], lane) : 0;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int f = i >> 6, cc = i & 63;
    const int fr = w.perm[b0 + f], c = c0 + cc;
    if (fr >= 0 && fr < B && bit_of(sel, f) && c < g.N) dst[(int64_t)fr * g.N + c] = tile[f][cc];
  }
}

// Posterior, B x N floats.
__global__ void __launch_bounds__(256) g_store_post(GraphView g, GraphWork w_, float *dst, int B,
                                                    int flush) {
  const GraphWork w = live(w_);
  if (flush && !w.st->flag) return;
  __shared__ float tile[64][65];
  const int c0 = blockIdx.x * 64, b0 = blockIdx.y * 64;
  const uint64_t sel = flush ? w.done_w[blockIdx.y] : ~0ull;
  const int lane = threadIdx.x & 63, wv = wave_in_block();
  for (int cc = wv; cc < 64; cc += 4) {
    const int c = c0 + cc;
    tile[lane][cc] = c < g.N ? w.post[at(c, blockIdx.y, g.N, lane)] : 0.0f;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int f = i >> 6, cc = i & 63;
    const int fr = w.perm[b0 + f], c = c0 + cc;
    if (fr >= 0 && fr < B && bit_of(sel, f) && c < g.N) dst[(int64_t)fr * g.N + c] = tile[f][cc];
  }
}

// ---- compaction --------------------------------------------------------
// A 64-frame chunk runs until its slowest frame stops, so without
// compaction a frame that stopped keeps costing memory traffic.  After an
// iteration's variable pass (Q live, R dead), when the running frames fit in
// fewer chunks and fill at most 3/4 of the occupied slots, they move, in
// order, to the lowest slots of the spare buffers: their outputs are
// unaffected (every frame's arithmetic is independent of its slot), and the
// frames that stopped are flushed to the caller's buffers first.

// One block: count running frames, decide, and list new slot -> old slot.
__global__ void __launch_bounds__(1024) g_plan(GraphWork w) {
  __shared__ int part[16];
  __shared__ int run_base;
  GraphState *st = w.st;
  const int live_chunks = st->slots / 64;
  int mine = 0;
  for (int k = threadIdx.x; k < live_chunks; k += 1024) mine += __popcll(~w.done_w[k]);
  for (int off = 32; off > 0; off >>= 1) mine += __shfl_xor(mine, off);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = mine;
  __syncthreads();
  int active = 0;
  for (int i = 0; i < 16; ++i) active += part[i];
  const int new_chunks = (active + 63) / 64;
  const bool go = active > 0 && new_chunks < live_chunks && 4 * active <= 3 * st->slots;
  __syncthreads();
  if (threadIdx.x == 0) {
    st->flag = go ? 1 : 0;
    st->n_new = active;
    run_base = 0;
  }
  if (!go) return;
  __syncthreads();
  // tiles of 1024 chunks: exclusive scan of per-chunk counts, then scatter
  for (int k0 = 0; k0 < live_chunks; k0 += 1024) {
    const int k = k0 + (int)threadIdx.x;
    const uint64_t act = k < live_chunks ? ~w.done_w[k] : 0ull;
    const int c = __popcll(act);
    int incl = c;  // inclusive scan within the wave
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(incl, off);
      if ((threadIdx.x & 63) >= off) incl += v;
    }
    __syncthreads();
    if ((threadIdx.x & 63) == 63) part[threadIdx.x >> 6] = incl;
    __syncthreads();
    int wave_base = 0;
    for (int i = 0; i < (int)(threadIdx.x >> 6); ++i) wave_base += part[i];
    int pos = run_base + wave_base + incl - c;
    for (uint64_t m = act; m; m &= m - 1) w.src[pos++] = k * 64 + __builtin_ctzll(m);
    __syncthreads();
    if (threadIdx.x == 1023) run_base += wave_base + incl;
    __syncthreads();
  }
}

// Live Q of the running frames -> the R buffer (dead between the variable
// pass and the next check pass), new slot t <- old slot src[t].
template <typename Real>
__global__ void __launch_bounds__(256) g_move_msgs(GraphView g, GraphWork w_) {
  const GraphWork w = live(w_);
  const GraphState *st = w.st;
  if (!st->flag) return;
  const int kn = blockIdx.y, lane = threadIdx.x & 63;
  const int t = kn * 64 + lane;
  if (kn * 64 >= st->n_new) return;
  const bool ok = t < st->n_new;
  const int s = ok ? w.src[t] : 0;
  const Real *Q = (const Real *)w.Q + at(0, s >> 6, g.E, s & 63);
  Real *D = (Real *)w.R + at(0, kn, g.E, lane);
  const int per = (g.E + gridDim.x - 1) / gridDim.x;
  const int e0 = blockIdx.x * per, e1 = min(g.E, e0 + per);
  if (ok)
    for (int e = e0 + wave_in_block(); e < e1; e += 4) D[(int64_t)e * 64] = Q[(int64_t)e * 64];
}

// Channel values, posteriors and hard bits of the running frames -> spares.
__global__ void __launch_bounds__(256) g_move_cols(GraphView g, GraphWork w_) {
  const GraphWork w = live(w_);
  const GraphState *st = w.st;
  if (!st->flag) return;
  const int kn = blockIdx.y, lane = threadIdx.x & 63;
  if (kn * 64 >= st->n_new) return;
  const int t = kn * 64 + lane;
  const bool ok = t < st->n_new;
  const int s = ok ? w.src[t] : 0;
  const int per = (g.N + gridDim.x - 1) / gridDim.x;
  const int c0 = blockIdx.x * per, c1 = min(g.N, c0 + per);
  for (int c = c0 + wave_in_block(); c < c1; c += 4) {
    if (ok) {
      st->L2[at(c, kn, g.N, lane)] = w.L[at(c, s >> 6, g.N, s & 63)];
      if (w.post) st->post2[at(c, kn, g.N, lane)] = w.post[at(c, s >> 6, g.N, s & 63)];
    }
    const bool bit = ok && bit_of(w.hard[(int64_t)c * w.chunks + (s >> 6)], s & 63);
    const uint64_t bw = __ballot(bit);
    if (lane == 0) st->hard2[(int64_t)c * w.chunks + kn] = bw;
  }
}

// Swap to the compacted buffers and rewrite the per-slot state.
__global__ void __launch_bounds__(256) g_commit(GraphWork w, int used0) {
  GraphState *st = w.st;
  if (!st->flag) return;
  const int n = st->n_new;
  // every slot of the spare map: slots past the old occupied range still
  // hold entries from an earlier use of the buffer
  for (int t = threadIdx.x; t < w.Bp; t += 256) {
    st->perm2[t] = t < n ? st->perm[w.src[t]] : -1;
    if (t < n) w.used[t] = used0;  // still running
  }
  for (int k = threadIdx.x; k < w.chunks; k += 256) {
    const int lo = k * 64;
    const uint64_t empty = lo + 64 <= n ? 0ull : (lo >= n ? ~0ull : (~0ull << (n - lo)));
    w.done_w[k] = empty;
    w.chunk_done[k] = lo >= n ? 1 : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    void *q = st->Q;
    st->Q = st->R;
    st->R = q;
    float *l = st->L;
    st->L = st->L2;
    st->L2 = l;
    float *p = st->post;
    st->post = st->post2;
    st->post2 = p;
    uint64_t *hd = st->hard;
    st->hard = st->hard2;
    st->hard2 = hd;
    int32_t *pm = st->perm;
    st->perm = st->perm2;
    st->perm2 = pm;
    st->slots = (n + 63) / 64 * 64;
    st->flag = 0;
  }
}

template <int PREC>
void launch_check(const GraphView &g, const GraphWork &w, int h, dim3 grid, hipStream_t st) {
  if (g.dc_max <= 8)
    g_check<PREC, 8><<<grid, 256, 0, st>>>(g, w, h);
  else if (g.dc_max <= 16)
    g_check<PREC, 16><<<grid, 256, 0, st>>>(g, w, h);
  else
    g_check<PREC, 32><<<grid, 256, 0, st>>>(g, w, h);
}

template <typename Real>
void launch_var(const GraphView &g, const GraphWork &w, dim3 grid, hipStream_t st) {
  if (g.dv_max <= 4)
    g_var<Real, 4><<<grid, 256, 0, st>>>(g, w);
  else if (g.dv_max <= 8)
    g_var<Real, 8><<<grid, 256, 0, st>>>(g, w);
  else
    g_var<Real, 16><<<grid, 256, 0, st>>>(g, w);
}

// LDPC_GRAPH_COMPACT=0 disables compaction (A/B and debugging knob).
bool compaction_enabled() {
  const char *e = getenv("LDPC_GRAPH_COMPACT");
  return !(e && e[0] == '0');
}

// Compaction after the variable pass of iteration h (every other iteration
// from h = 3 while more than one iteration remains; a no-op unless g_plan
// finds the running frames fit in fewer chunks and <= 3/4 of the slots).
template <typename Real>
void launch_compaction(const GraphView &g, const GraphWork &w, const DecodeArgs &a, int used0,
                       hipStream_t st) {
  const int chunks = w.chunks;
  g_plan<<<1, 1024, 0, st>>>(w);
  g_store_packed<<<dim3((g.KB + 63) / 64, chunks), 256, 0, st>>>(g, w, a, 1);
  if (a.bits) g_store_bits<<<dim3((g.N + 63) / 64, chunks), 256, 0, st>>>(g, w, a.bits, a.B, 1);
  if (a.llr && w.post)
    g_store_post<<<dim3((g.N + 63) / 64, chunks), 256, 0, st>>>(g, w, a.llr, a.B, 1);
  const unsigned eb = (unsigned)std::min<int64_t>(128, (g.E + 255) / 256);
  const unsigned cb = (unsigned)std::min<int64_t>(64, (g.N + 255) / 256);
  g_move_msgs<Real><<<dim3(eb, chunks), 256, 0, st>>>(g, w);
  g_move_cols<<<dim3(cb, chunks), 256, 0, st>>>(g, w);
  g_commit<<<1, 256, 0, st>>>(w, used0);
}

template <int PREC>
void run_sp(const GraphView &g, const GraphWork &w, const DecodeArgs &a, dim3 rgrid,
            dim3 cgrid, hipStream_t st) {
  typedef typename Math<PREC>::Real Real;
  for (int h = 0; h < a.max_iters; ++h) {
    launch_check<PREC>(g, w, h, rgrid, st);
    if (h > 0) g_decide<<<w.chunks, 256, 0, st>>>(w, h, a.max_iters, a.et_period);
    launch_var<Real>(g, w, cgrid, st);
    if (compaction_enabled() && w.chunks > 1 && h >= 3 && (h & 1) && h + 1 < a.max_iters)
      launch_compaction<Real>(g, w, a, a.max_iters, st);
  }
}

int check_waves(const GraphView &g) {
  return 4 * ((g.M + 4 * kRowsPerWave - 1) / (4 * kRowsPerWave));
}

}  // namespace

size_t graph_work_bytes(const GraphView &g, int Bp, int prec, int method, bool want_post) {
  const size_t real = prec == 1 ? 4 : 8;
  const bool soft = method == 0 || method == 1;
  const size_t chunks = (size_t)Bp / 64;
  size_t n = 0;
  if (soft) n += 2 * al256((size_t)g.E * Bp * real) + al256((size_t)g.N * Bp * 4);
  n += al256((size_t)g.N * chunks * 8);                                   // hard
  if (!soft) n += al256((size_t)g.N * chunks * 8) + al256((size_t)g.M * chunks * 8);  // y, rowpar
  n += al256((size_t)check_waves(g) * chunks * 8) + al256(chunks * 8) + al256(chunks);
  n += 2 * al256((size_t)Bp * 4);
  if (want_post) n += al256((size_t)g.N * Bp * 4);
  // compaction: state, perm x2, src, spare L / post / hard
  n += al256(sizeof(GraphState)) + 3 * al256((size_t)Bp * 4) + al256((size_t)g.N * chunks * 8);
  if (soft) n += al256((size_t)g.N * Bp * 4) + (want_post ? al256((size_t)g.N * Bp * 4) : 0);
  return n;
}

void graph_work_carve(GraphWork &w, void *base, const GraphView &g, int Bp, int prec, int method,
                      bool want_post) {
  const size_t real = prec == 1 ? 4 : 8;
  const bool soft = method == 0 || method == 1;
  const size_t chunks = (size_t)Bp / 64;
  char *p = (char *)base;
  auto take = [&](size_t bytes) {
    char *r = p;
    p += al256(bytes);
    return (void *)r;
  };
  w = GraphWork{};
  w.Bp = Bp;
  w.chunks = (int)chunks;
  w.check_waves = check_waves(g);
  if (soft) {
    w.Q = take((size_t)g.E * Bp * real);
    w.R = take((size_t)g.E * Bp * real);
    w.L = (float *)take((size_t)g.N * Bp * 4);
  }
  w.hard = (uint64_t *)take((size_t)g.N * chunks * 8);
  if (!soft) {
    w.y = (uint64_t *)take((size_t)g.N * chunks * 8);
    w.rowpar = (uint64_t *)take((size_t)g.M * chunks * 8);
  }
  w.synd_part = (uint64_t *)take((size_t)w.check_waves * chunks * 8);
  w.done_w = (uint64_t *)take(chunks * 8);
  w.chunk_done = (uint8_t *)take(chunks);
  w.used = (int32_t *)take((size_t)Bp * 4);
  w.synd = (int32_t *)take((size_t)Bp * 4);
  w.post = want_post ? (float *)take((size_t)g.N * Bp * 4) : nullptr;
  w.st = (GraphState *)take(sizeof(GraphState));
  w.perm = (int32_t *)take((size_t)Bp * 4);
  w.perm2 = (int32_t *)take((size_t)Bp * 4);
  w.src = (int32_t *)take((size_t)Bp * 4);
  w.hard2 = (uint64_t *)take((size_t)g.N * chunks * 8);
  if (soft) {
    w.L2 = (float *)take((size_t)g.N * Bp * 4);
    w.post2 = want_post ? (float *)take((size_t)g.N * Bp * 4) : nullptr;
  }
}

int launch_graph_decode(const GraphView &g, const GraphWork &w, const DecodeArgs &a, int method,
                        int prec, void *stream) {
  // min-sum runs on the narrow-chunk pipeline (ldpc_graph_msn.hip)
  if (g.dc_max > kGraphDcMax || g.dv_max > kGraphDvMax || method == 0) return -2;
  if (a.B <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int chunks = w.chunks;
  const dim3 rgrid(w.check_waves / 4, chunks);
  const dim3 cgrid((g.N + 4 * kColsPerWave - 1) / (4 * kColsPerWave), chunks);
  const dim3 tgrid((g.N + 63) / 64, chunks);
  const bool soft = method == 0 || method == 1;
  g_reset<<<chunks, 64, 0, st>>>(w, a.B, method == 3 ? 0 : a.max_iters);
  if (soft) {
    if (prec == 1)
      g_load<float, true><<<tgrid, 256, 0, st>>>(g, w, a.in, a.cw_stride, a.elem_stride,
                                                  a.polarity, a.B);
    else
      g_load<double, true><<<tgrid, 256, 0, st>>>(g, w, a.in, a.cw_stride, a.elem_stride,
                                                   a.polarity, a.B);
  } else {
    g_load<float, false><<<tgrid, 256, 0, st>>>(g, w, a.in, a.cw_stride, a.elem_stride,
                                                 a.polarity, a.B);
  }
  if (method == 1) {
    if (prec == 1)
      run_sp<1>(g, w, a, rgrid, cgrid, st);
    else if (prec == 2)
      run_sp<2>(g, w, a, rgrid, cgrid, st);
    else if (prec == 3)
      run_sp<3>(g, w, a, rgrid, cgrid, st);
    else
      run_sp<0>(g, w, a, rgrid, cgrid, st);
  } else if (method == 2) {
    for (int h = 0; h < a.max_iters; ++h) {
      g_check_bf<<<rgrid, 256, 0, st>>>(g, w, h);
      if (h > 0) g_decide<<<chunks, 256, 0, st>>>(w, h, a.max_iters, a.et_period);
      if (g.dv_max <= 4)
        g_var_bf<4><<<cgrid, 256, 0, st>>>(g, w);
      else if (g.dv_max <= 8)
        g_var_bf<8><<<cgrid, 256, 0, st>>>(g, w);
      else
        g_var_bf<16><<<cgrid, 256, 0, st>>>(g, w);
    }
  }
  g_synd<<<rgrid, 256, 0, st>>>(g, w, a.B);
  g_store_packed<<<dim3((g.KB + 63) / 64, chunks), 256, 0, st>>>(g, w, a, 0);
  if (a.bits) g_store_bits<<<tgrid, 256, 0, st>>>(g, w, a.bits, a.B, 0);
  if (a.llr && w.post) g_store_post<<<tgrid, 256, 0, st>>>(g, w, a.llr, a.B, 0);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace ldpc
