// ldpc_kernels.hip -- belief-propagation decode kernels for gfx950 (MI355X).
//
// Hot path of ericdegroot/gr-ldpc_ece535a: the decode call inside
// ldpc_decoder_cb_impl::general_work (lib/ldpc_decoder_cb_impl.cc:155-164).
//
// Mapping ("small code" kernel, N <= 256, E <= 512, dc <= 8, dv <= 4):
//   * one 64-lane wave decodes one frame; 4 independent waves per 256-thread
//     workgroup, each with a private LDS slice, no workgroup barrier after the
//     prologue, so every wave leaves its iteration loop on its own syndrome
//     (per-frame early termination exactly as the reference);
//   * lane l owns edges l, l+64, ... (S slots): its variable->check message
//     lives in VGPRs across iterations, only the per-iteration exchange goes
//     through LDS (tanh values for the check pass, check->variable messages
//     for the column sums);
//   * lane l also owns columns l, l+64, ... for the hard decision; the hard
//     decision vector is a 64-bit wave ballot per 64 columns, and the
//     syndrome is popcount(rowmask & hard) per row lane + one more ballot;
//   * the only HBM traffic per frame is the N input samples, the packed
//     output and the optional per-frame outputs.
// Arithmetic follows the reference operation for operation (same operand
// order, no contraction: build with -ffp-contract=off), in double
// (LDPC_PREC_F64) or float (LDPC_PREC_F32).
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>

#include <algorithm>

#include "ldpc_kernels.hpp"
#include "ldpc_math.hpp"

namespace ldpc {

// LDS hand-off between lanes of ONE wave: the wave's LDS operations execute
// in issue order, so a wavefront-scope fence (compiler ordering + lgkmcnt)
// is all that is needed; no s_barrier, waves stay independent.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename Real>
struct Math;
template <>
struct Math<double> {
#ifdef LDPC_OCML_F64  // A/B switch: ROCm's ocml tanh/log
  static __device__ __forceinline__ double tanh_(double x) { return ::tanh(x); }
  static __device__ __forceinline__ double log_(double x) { return ::log(x); }
#else  // fdlibm (ldpc_math.hpp): tanh bit-identical to glibc's, log < 1 ulp
  static __device__ __forceinline__ double tanh_(double x) { return fm::tanh_f64_bf(x); }
  static __device__ __forceinline__ double log_(double x) { return fm::log_f64_bf(x); }
#endif
  static __device__ __forceinline__ double abs_(double x) { return ::fabs(x); }
  static __device__ __forceinline__ double max_() { return DBL_MAX; }
};
template <>
struct Math<float> {
  static __device__ __forceinline__ float tanh_(float x) { return ::tanhf(x); }
  static __device__ __forceinline__ float log_(float x) { return ::logf(x); }
  static __device__ __forceinline__ float abs_(float x) { return ::fabsf(x); }
  static __device__ __forceinline__ float max_() { return FLT_MAX; }
};

// sign(), lib/ldpc_decoder_cb_impl.cc:574-578 (sign(0) == 0).
template <typename Real>
__device__ __forceinline__ int sgn(Real v) {
  return (v > Real(0)) - (v < Real(0));
}

template <int NW>
__device__ __forceinline__ uint64_t word_at(const uint64_t (&w)[NW], int idx) {
  uint64_t r = w[0];
#pragma unroll
  for (int q = 1; q < NW; ++q)
    if (idx == q) r = w[q];
  return r;
}

__device__ __forceinline__ uint64_t word4_at(const uint64_t (&w)[4], int idx) {
  uint64_t r = w[0];
  r = idx == 1 ? w[1] : r;
  r = idx == 2 ? w[2] : r;
  r = idx == 3 ? w[3] : r;
  return r;
}

// Unsatisfied checks of the hard decision `hard` (checkFrame :236-253 with
// an unreachable threshold): row lane j XORs popcount(rowmask_j & hard),
// one ballot per 64 rows gathers the odd rows.
template <int NW>
__device__ __forceinline__ int syndrome_weight(const uint64_t (&hard)[NW],
                                               const uint64_t *rowmask, int M,
                                               int rs, int lane) {
  int weight = 0;
#pragma unroll
  for (int q = 0; q < kMMax / 64; ++q) {
    if (q < rs) {
      const int j = lane + 64 * q;
      int odd = 0;
      if (j < M) {
#pragma unroll
        for (int w = 0; w < NW; ++w) odd ^= __popcll(rowmask[j * NW + w] & hard[w]);
        odd &= 1;
      }
      weight += __popcll(__ballot(odd));
    }
  }
  return weight;
}

__host__ __device__ constexpr size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

// Block LDS: [rowmask M x NW][row recs 64S][col-neighbour recs 64S]
// [column recs 64 NW] then one slice per wave [tb 64S][eb 64S][rb 64NW][sb 64NW].
template <typename Real, int S, int NW>
struct Layout {
  size_t erow, ecol, cols, waves, per_wave, total;
  __host__ __device__ explicit Layout(int M) {
    erow = align16((size_t)M * NW * 8);
    ecol = erow + (size_t)64 * S * sizeof(EdgeRowRec);
    cols = ecol + (size_t)64 * S * sizeof(EdgeColRec);
    waves = align16(cols + (size_t)64 * NW * sizeof(ColRec));
    per_wave = (2 * 64 * S + 2 * 64 * NW) * sizeof(Real);
    total = waves + (size_t)kWavesPerBlock * per_wave;
  }
};

// Decodes frame b with the wave's resident tables (er/cr) and LDS slice.
template <typename Real, int METHOD, int S, int NW>
__device__ __forceinline__ void decode_frame(const CodeView &code, const DecodeArgs &a,
                                             const int64_t b, const int (&col)[S],
                                             const EdgeRowRec *erow, const EdgeColRec *ecol,
                                             const ColRec *cols, const uint64_t *rowmask,
                                             Real *tb, Real *eb, Real *rb, Real *sb,
                                             const int lane) {
  const int M = code.M, N = code.N;
  // Channel samples: tx = Re(in) * polarity (:149-153); r = -tx (:486,
  // :318-321).  Lane l reads sample l of each 64-column slot (coalesced).
  const float *src = a.in + b * a.cw_stride;
  Real post[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const int c = lane + 64 * q;
    float x = 0.0f;
    if (c < N) x = src[(int64_t)c * a.elem_stride] * a.polarity;
    rb[c] = -(Real)x;
    post[q] = (Real)x;
  }

  uint64_t hard[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) hard[q] = 0;
  int weight = 0, used = 0;

  if constexpr (METHOD == 1 || METHOD == 0) {
    wave_lds_sync();  // rb visible to every lane
    Real msg[S];      // SP: M(j,i) (:489-496); min-sum: L(q_ij) (:328-331)
    Real lr[S];       // min-sum: L(r_ji)
#pragma unroll
    for (int s = 0; s < S; ++s) {
      msg[s] = col[s] != kNone ? rb[col[s]] : Real(0);
      lr[s] = Real(0);
    }

    for (int h = 0; h < a.max_iters; ++h) {
      if constexpr (METHOD == 1) {
        // ---- check pass, :503-516 -----------------------------------
#pragma unroll
        for (int s = 0; s < S; ++s)
          if (col[s] != kNone) tb[lane + 64 * s] = Math<Real>::tanh_(msg[s] / Real(2));
        wave_lds_sync();
#pragma unroll
        for (int s = 0; s < S; ++s) {
          if (col[s] != kNone) {
            const EdgeRowRec er = erow[lane + 64 * s];
            Real T = Real(1);
#pragma unroll
            for (int k = 0; k < kDcMax - 1; ++k) {
              const int n = er.rn[k];
              if (n != kNone) T = T * tb[n];
            }
            eb[lane + 64 * s] = Math<Real>::log_((Real(1) + T) / (Real(1) - T));
          }
        }
        wave_lds_sync();
        // ---- decision, :519-532: L = sum_j (E(j,i) + r(i)), 1 iff L <= 0
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          const int c = lane + 64 * q;
          bool bit = false;
          if (c < N) {
            const ColRec cr = cols[c];
            const Real rc = rb[c];
            Real L = Real(0);
#pragma unroll
            for (int k = 0; k < kDvMax; ++k) {
              const int n = cr.e[k];
              if (n != kNone) L = L + (eb[n] + rc);
            }
            bit = L <= Real(0);
            post[q] = L;
          }
          hard[q] = __ballot(bit);
        }
      } else {
        // ---- min-sum horizontal step, :340-376 ----------------------
#pragma unroll
        for (int s = 0; s < S; ++s)
          if (col[s] != kNone) tb[lane + 64 * s] = msg[s];
        wave_lds_sync();
#pragma unroll
        for (int s = 0; s < S; ++s) {
          if (col[s] != kNone) {
            const EdgeRowRec er = erow[lane + 64 * s];
            const int self = sgn(msg[s]);
            int prod = self;
            Real lo = Math<Real>::max_();
#pragma unroll
            for (int k = 0; k < kDcMax - 1; ++k) {
              const int n = er.rn[k];
              if (n != kNone) {
                const Real v = tb[n];
                prod *= sgn(v);
                const Real beta = Math<Real>::abs_(v);
                if (beta < lo) lo = beta;
              }
            }
            lr[s] = (Real)(prod * self) * lo;
            eb[lane + 64 * s] = lr[s];
          }
        }
        wave_lds_sync();
        // ---- vertical step, :379-403: s = sum_i L(r_ji); L(Q) = Lci + s
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          const int c = lane + 64 * q;
          bool bit = false;
          if (c < N) {
            const ColRec cr = cols[c];
            Real acc = Real(0);
#pragma unroll
            for (int k = 0; k < kDvMax; ++k) {
              const int n = cr.e[k];
              if (n != kNone) acc = acc + eb[n];
            }
            const Real LQ = rb[c] + acc;
            sb[c] = LQ;
            bit = LQ < Real(0);
            post[q] = LQ;
          }
          hard[q] = __ballot(bit);
        }
      }
      // ---- early exit: SP every iteration (:535-537); min-sum only when
      // h+1 < max_iters (:406-408); et_period > 1 thins the checks.
      weight = syndrome_weight<NW>(hard, rowmask, M, code.rs, lane);
      used = h + 1;
      if (h + 1 == a.max_iters) break;
      if ((h + 1) % a.et_period == 0 && weight == 0) break;

      if constexpr (METHOD == 1) {
        // ---- bit messages, :540-553: M(j,i) = sum_{k != j} (E(k,i) + r(i))
#pragma unroll
        for (int s = 0; s < S; ++s) {
          if (col[s] != kNone) {
            const EdgeColRec ec = ecol[lane + 64 * s];
            const Real rc = rb[col[s]];
            Real acc = Real(0);
#pragma unroll
            for (int k = 0; k < kDvMax - 1; ++k) {
              const int n = ec.cn[k];
              if (n != kNone) acc = acc + (eb[n] + rc);
            }
            msg[s] = acc;
          }
        }
      } else {
        wave_lds_sync();  // sb visible
        // L(q_ij) = Lci(j) + s_j - L(r_ji)  (:387-392)
#pragma unroll
        for (int s = 0; s < S; ++s)
          if (col[s] != kNone) msg[s] = sb[col[s]] - lr[s];
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
    weight = syndrome_weight<NW>(hard, rowmask, M, code.rs, lane);
    if constexpr (METHOD == 2) {
      // ---- bit flipping, :439-473 ------------------------------------
      const int half = (int)((unsigned)M / 2u);
      for (int h = 0; h < a.max_iters; ++h) {
        // parity of ci over each row; E(i,j) for an edge = parity ^ ci(j)
        uint64_t rowpar[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          rowpar[q] = 0;
          if (q < code.rs) {
            const int j = lane + 64 * q;
            int odd = 0;
            if (j < M) {
#pragma unroll
              for (int w = 0; w < NW; ++w) odd ^= __popcll(rowmask[j * NW + w] & hard[w]);
              odd &= 1;
            }
            rowpar[q] = __ballot(odd);
          }
        }
        uint64_t next[NW];
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          const int c = lane + 64 * q;
          bool nb = false;
          if (c < N) {
            const ColRec cr = cols[c];
            const int cib = (int)((hard[q] >> lane) & 1);
            const int yb = (int)((y[q] >> lane) & 1);
            int votes = 0;
#pragma unroll
            for (int k = 0; k < kDvMax; ++k) {
              if (cr.e[k] != kNone) {
                const int r = cr.r[k];
                const int par = (int)((word4_at(rowpar, r >> 6) >> (r & 63)) & 1);
                if ((par ^ cib) != yb) ++votes;
              }
            }
            nb = votes > half ? (yb == 0) : (cib != 0);
          }
          next[q] = __ballot(nb);
        }
#pragma unroll
        for (int q = 0; q < NW; ++q) hard[q] = next[q];
        weight = syndrome_weight<NW>(hard, rowmask, M, code.rs, lane);
        used = h + 1;
        if (h + 1 == a.max_iters) break;
        if ((h + 1) % a.et_period == 0 && weight == 0) break;
      }
    }
  }

  // ---- outputs ---------------------------------------------------------
  if (lane == 0) {
    if (a.iters) a.iters[b] = used;
    if (a.synd) a.synd[b] = weight;
  }
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const int c = lane + 64 * q;
    if (c < N) {
      if (a.bits) a.bits[b * N + c] = (uint8_t)((hard[q] >> lane) & 1);
      if (a.llr) a.llr[b * N + c] = (float)post[q];
    }
  }
  // packed info bits M.., MSB first (:207-219)
  for (int p = lane; p < code.KB; p += 64) {
    uint32_t o = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = M + 8 * p + j;
      if (c < N) o |= (uint32_t)((word_at<NW>(hard, c >> 6) >> (c & 63)) & 1) << (7 - j);
    }
    a.packed[b * code.KB + p] = (uint8_t)o;
  }
  // the next frame's rb writes must not overtake this frame's LDS reads
  wave_lds_sync();
}

// Persistent launch: `a.waves` waves; wave w decodes frame w, then frames
// a.waves + ticket++ until the batch is exhausted.  Frames stop after 1..cap
// iterations, so pulling work keeps every SIMD busy to the end instead of
// leaving it with a fixed share of the batch.
template <typename Real, int METHOD, int S, int NW>
__global__ void __launch_bounds__(kThreads)
    decode_small_kernel(CodeView code, DecodeArgs a) {
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int M = code.M;
  const Layout<Real, S, NW> L(M);

  // Code tables into LDS, shared by the block's waves (the only workgroup
  // barrier): row masks, per-edge neighbour records, per-column records.
  uint64_t *rowmask = reinterpret_cast<uint64_t *>(smem);
  EdgeRowRec *erow = reinterpret_cast<EdgeRowRec *>(smem + L.erow);
  EdgeColRec *ecol = reinterpret_cast<EdgeColRec *>(smem + L.ecol);
  ColRec *cols = reinterpret_cast<ColRec *>(smem + L.cols);
  for (int t = threadIdx.x; t < M * NW; t += kThreads) rowmask[t] = code.rowmask[t];
  for (int t = threadIdx.x; t < 64 * S; t += kThreads) {
    erow[t] = code.erow[t];
    ecol[t] = code.ecol[t];
  }
  for (int t = threadIdx.x; t < 64 * NW; t += kThreads) cols[t] = code.cols[t];
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.ticket_next = 0u;  // next launch's queue head
  __syncthreads();

  int64_t b = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  if (b >= a.waves || b >= a.B) return;

  Real *tb = reinterpret_cast<Real *>(smem + L.waves + (size_t)wave * L.per_wave);
  Real *eb = tb + 64 * S;
  Real *rb = eb + 64 * S;
  Real *sb = rb + 64 * NW;
  int col[S];
#pragma unroll
  for (int s = 0; s < S; ++s) col[s] = erow[lane + 64 * s].col;

  while (b < a.B) {
    decode_frame<Real, METHOD, S, NW>(code, a, b, col, erow, ecol, cols, rowmask, tb, eb, rb, sb,
                                      lane);
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(a.ticket, 1u);
    b = (int64_t)a.waves + (int64_t)__builtin_amdgcn_readfirstlane((int)t);
  }
}

// ---------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------
template <typename Real, int METHOD, int S, int NW>
static int launch_one(const CodeView &code, const DecodeArgs &a, hipStream_t st) {
  const size_t lds = Layout<Real, S, NW>(code.M).total;
  if (lds > 65536 &&
      hipFuncSetAttribute((const void *)decode_small_kernel<Real, METHOD, S, NW>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -3;
  const dim3 grid((unsigned)((a.waves + kWavesPerBlock - 1) / kWavesPerBlock));
  hipLaunchKernelGGL((decode_small_kernel<Real, METHOD, S, NW>), grid, dim3(kThreads),
                     lds, st, code, a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <typename Real, int METHOD, int NW>
static int launch_slots(const CodeView &code, const DecodeArgs &a, int slots,
                        hipStream_t st) {
  switch (slots) {
    case 1: return launch_one<Real, METHOD, 1, NW>(code, a, st);
    case 2: return launch_one<Real, METHOD, 2, NW>(code, a, st);
    case 3: return launch_one<Real, METHOD, 3, NW>(code, a, st);
    case 4: return launch_one<Real, METHOD, 4, NW>(code, a, st);
    case 5: return launch_one<Real, METHOD, 5, NW>(code, a, st);
    case 6: return launch_one<Real, METHOD, 6, NW>(code, a, st);
    case 7: return launch_one<Real, METHOD, 7, NW>(code, a, st);
    case 8: return launch_one<Real, METHOD, 8, NW>(code, a, st);
    default: return -2;
  }
}

template <int NW>
static int launch_nw(const CodeView &code, const DecodeArgs &a, int method, int prec,
                     int slots, hipStream_t st) {
  if (method == 3) return launch_one<float, 3, 1, NW>(code, a, st);
  if (method == 2) return launch_one<float, 2, 1, NW>(code, a, st);
  if (method == 1)
    return prec == 1 ? launch_slots<float, 1, NW>(code, a, slots, st)
                     : launch_slots<double, 1, NW>(code, a, slots, st);
  return prec == 1 ? launch_slots<float, 0, NW>(code, a, slots, st)
                   : launch_slots<double, 0, NW>(code, a, slots, st);
}

int launch_decode(const CodeView &code, const DecodeArgs &args, int method, int prec,
                  int slots, int nw, int waves_per_cu, void *stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (args.B <= 0) return 0;
  DecodeArgs a = args;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (waves_per_cu <= 0) waves_per_cu = 8;
  const int64_t w = std::min<int64_t>((int64_t)a.B, (int64_t)waves_per_cu * cus);
  a.waves = (int)((w + kWavesPerBlock - 1) / kWavesPerBlock * kWavesPerBlock);

  if (nw == 1) return launch_nw<1>(code, a, method, prec, slots, st);
  if (nw == 4) return launch_nw<4>(code, a, method, prec, slots, st);
  return -2;
}

}  // namespace ldpc
