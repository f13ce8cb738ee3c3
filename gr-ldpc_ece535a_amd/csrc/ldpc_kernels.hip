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
#include "ldpc_frame.hpp"

namespace ldpc {

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
#ifndef LDPC_TP_MINB
#define LDPC_TP_MINB 4  // throughput build: waves per SIMD the register budget allows
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

  const int64_t w = (int64_t)blockIdx.x * kWavesPerBlock + wave;
  const int64_t c = a.claim;  // frames per claim (1 with static_stride)
  int64_t b = w * c;
  if (w >= a.waves || b >= a.B) return;
  int64_t bend = b + c;  // end of the wave's current claim

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
    int64_t pb = (int64_t)a.waves * c + b;
    pb = pb < a.B ? pb : b;
    float ppol;
    const float *ps = frame_src(a, pb, ppol);
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
    const int64_t f = b;
    // the frame's channel samples, one load per lane and column position
    // (a permutation of the frame's N samples); positions past N are 0
    float xin[NW], pol;
    const float *src = frame_src(a, f, pol);
#pragma unroll
    for (int q = 0; q < NW; ++q)
      xin[q] = colq[q] >= 0 ? src[(int64_t)colq[q] * a.elem_stride] * pol : 0.0f;
    if constexpr (METHOD == 1) {
      bool bad = false;
#pragma unroll
      for (int q = 0; q < NW; ++q) bad |= !__builtin_isfinite(xin[q]);
      // the throughput build runs with fair_cycles 0 (launch_slots)
      constexpr bool kFair = MINB != LDPC_TP_MINB;
      if (__ballot(bad) == 0)
        decode_frame<PREC, METHOD, S, NW, DCN, DVN, true, Real, true, kFair>(
            code, a, f, wt, tb, eb, rb, sb, lane, logtab, xin, colq, ppos);
      else
        decode_frame<PREC, METHOD, S, NW, DCN, DVN, false, Real, true, kFair>(
            code, a, f, wt, tb, eb, rb, sb, lane, logtab, xin, colq, ppos);
    } else {
      decode_frame<PREC, METHOD, S, NW, DCN, DVN>(code, a, f, wt, tb, eb, rb, sb, lane, logtab,
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
    } else if (++b == bend || b >= a.B) {
      // the claim is used up (or cut by the batch's end): the next one
      uint32_t t = 0;
      if (lane == 0) t = atomicAdd(a.ticket, (uint32_t)c) - a.ticket_base;
      b = (int64_t)a.waves * c + (int64_t)__builtin_amdgcn_readfirstlane((int)t);
      bend = b + c;
    }
  }
}

// ---------------------------------------------------------------------------
// Multi-wave kernel: one frame per S-wave workgroup, one edge per lane
// (mw_frame, ldpc_frame.hpp).
//
// At small batches the decode time is set by the frames that run to the
// iteration cap, i.e. by one frame's per-iteration latency.  Spreading a
// frame over S waves (on different SIMDs of the CU) divides the edge work of
// an iteration by S; the price is two workgroup barriers per iteration.
// ---------------------------------------------------------------------------

template <int PREC, int METHOD, int S, int NW>
__global__ void __launch_bounds__(64 * S) decode_mw_kernel(CodeView code, DecodeArgs a) {
  typedef typename Math<PREC>::Real Real;
  extern __shared__ __align__(16) unsigned char smem[];
  const MwLayout<Real, S, NW> L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N = code.N;
  constexpr int kDummy = 64 * S;
  Real *tb = reinterpret_cast<Real *>(smem);
  Real *eb = reinterpret_cast<Real *>(smem + L.eb);
  Real *rb = reinterpret_cast<Real *>(smem + L.waves + (size_t)wave * L.per_wave);
  Real *sb = rb + 64 * NW;
  int *fslot = reinterpret_cast<int *>(smem + L.fslot);
  __shared__ typename Math<PREC>::Tab logtab[TabLds<PREC>::kN];
  if constexpr (METHOD == 1) stage_tab<PREC>(logtab);
  if (tid == 0) tb[kDummy] = METHOD == 1 ? Real(1) : Math<PREC>::max_();
  MwTables<NW> t;
  mw_setup<NW>(code, tid, t);

  int64_t b = blockIdx.x;
  while (b < a.B) {
    float pol;
    const float *src = frame_src(a, b, pol);
    uint64_t hard[NW];
    Real post[NW];
    int used = 0;
    const int weight = mw_frame<PREC, METHOD, S, NW>(code, a.max_iters, a.et_period, t, tb, eb,
                                                     rb, sb, logtab, src, pol, a.elem_stride,
                                                     hard, post, used);
    // outputs (wave 0)
    if (wave == 0) {
      if (lane == 0) {
        if (a.iters) a.iters[b] = used;
        if (a.synd) a.synd[b] = weight;
      }
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        const int c = t.colq[q];
        if (c >= 0) {
          if (a.bits) a.bits[b * N + c] = (uint8_t)((hard[q] >> lane) & 1);
          if (a.llr) a.llr[b * N + c] = (float)post[q];
        }
      }
      for (int p = lane; p < code.KB; p += 64) {
        uint32_t o = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = code.M + 8 * p + j;
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
                  int nw, int waves_per_cu, int schedule, void *stream, uint32_t *advance_out) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  *advance_out = 0;
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
  // the one-wave kernel's fast modes claim several frames per queue add when
  // the batch is several times the resident waves (one counter word serves
  // ~88 adds per us: ring_claim, ldpc_kernels.hpp); smaller batches, the
  // workgroup form and fixed strides take one (every wave's first claim
  // starts at once: claims of several frames would serialise a small batch)
  const int64_t waves_max = (int64_t)waves_per_cu * cus;
  a.claim = mw || a.static_stride || a.B < 4 * waves_max ? 1 : ring_claim(method, prec);
  if (nw != 1 && nw != 4) return -2;
  const int rc = nw == 1 ? launch_nw<1>(code, a, method, prec, slots, mw, st)
                         : launch_nw<4>(code, a, method, prec, slots, mw, st);
  if (rc == 0 && !a.static_stride)
    *advance_out = (uint32_t)(a.claim * ((a.B + a.claim - 1) / a.claim));
  return rc;
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
