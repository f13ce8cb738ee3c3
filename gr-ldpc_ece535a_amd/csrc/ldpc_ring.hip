// ldpc_ring.hip -- the frame ring: one persistent launch for a stream of
// batches (gfx950).
//
// The reference decodes one frame per call (lib/ldpc_decoder_cb_impl.cc:
// 155-164); a throughput caller here hands the GPU whole batches of frames
// (the bench's config 2: 4096 frames of the default H at 2 dB, 50-iteration
// cap with the reference's per-frame early exit :535-537).  Frames stop after
// 1..50 iterations, so a launch per batch ends with most SIMDs idle while its
// last long frames run; round 5 hid that by keeping four launches in flight
// on four hardware queues, and still paid a launch-sized drain at the end of
// every timed window.
//
// Here ONE launch serves every batch posted to the ring (ldpc_ring_post):
//   * the frames of all posted batches form one queue: batch q's frame f is
//     ticket start_q + f, and a wave takes the next ticket from one device
//     counter, whatever batch it falls in -- a SIMD freed by a short frame of
//     batch q starts a frame of batch q + 1, and only the session's end has a
//     tail;
//   * a wave finds its ticket's batch from the descriptors the host writes
//     into mapped host memory: one 64-byte line per batch, every 8-byte word
//     tagged with the batch's sequence number (bits 48..63), read by one
//     instruction and accepted only when all eight tags agree (a line read
//     while the host rewrites it is read again);
//   * each frame is decoded by the batch kernels' one-wave arithmetic
//     (decode_frame, ldpc_frame.hpp: results equal every other decode of the
//     same samples); its outputs are stored write-through (sc1), then the
//     wave adds one to the batch slot's frame counter; the wave whose add
//     completes the batch writes the batch's completion word (q + 1) into
//     mapped host memory, which ldpc_ring_wait polls;
//   * a descriptor with `quit` ends the launch for every ticket past the last
//     batch; a wave that waits `deadline` for a batch that is never posted
//     leaves too (the host relaunches from the first incomplete batch).
// Visibility (MI355X_MICROARCH.md, inter-workgroup visibility): host memory
// is read with system-scope loads; outputs are sc1 stores drained by
// s_waitcnt vmcnt(0) before the agent-scope counter add; the completion word
// is one system-scope 8-byte store.
#include <atomic>

#include "ldpc_frame.hpp"

namespace ldpc {
namespace {

typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) int32_t gi32;
typedef __attribute__((address_space(1))) uint8_t gu8;
typedef __attribute__((address_space(1))) float gf32;

__device__ __forceinline__ uint64_t ticks() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ uint64_t sys_load(const uint64_t *p) {
  return __hip_atomic_load((const gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(uint64_t *p, uint64_t v) {
  __hip_atomic_store((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// write-through (sc1) output stores and input loads
__device__ __forceinline__ void wt_store(int32_t *p, int32_t v) {
  __hip_atomic_store((gi32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wt_store(uint32_t *p, uint32_t v) {
  __hip_atomic_store((gu32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void wt_store(uint8_t *p, uint8_t v) {
  __hip_atomic_store((gu8 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ag_load(const float *p) {
  return __hip_atomic_load((const gf32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}

// The batch a wave is working through, wave-uniform.  q: its sequence number
// (slot q % kRingSlots); [start, end): its tickets.  A batch found complete
// (its slot already reused) keeps end = start, so no ticket falls in it.
struct Batch {
  uint64_t q;
  int64_t start, end;
  const float *in;
  int64_t cw;
  uint8_t *packed;
  int32_t *iters, *synd;
  int B;
  bool quit;
};

constexpr uint64_t kPay = (1ull << 48) - 1;  // payload bits of a descriptor word

#ifdef LDPC_TIMELINE
// Diagnostic builds only (tools/ring_timeline.py): per ticket of the last
// launch, 5 words (ldpc_debug_ring_timeline).
constexpr int64_t kRingTimeline = 131072;
constexpr int kTlWords = 6;
__device__ uint64_t g_ring_timeline[kTlWords * kRingTimeline];
#endif

// How a descriptor line (lane j < 8 holds word j) reads for batch q.
enum LineState { kPosted, kNotYet, kReused, kTorn, kBusy };
__device__ __forceinline__ LineState classify(uint64_t w, uint64_t q, int lane) {
  const uint64_t seq = readlane64(w, 0);
  if (seq < q + 1) return kNotYet;
  if (seq > q + 1) return kReused;
  const uint64_t tag = ((q + 1) & 0xFFFFu) << 48;
  return __ballot(lane >= 1 && lane < 8 && (w & ~kPay) != tag) == 0 ? kPosted : kTorn;
}
__device__ __forceinline__ uint64_t ag_load64(const uint64_t *p) {
  return __hip_atomic_load((const gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ag_store64(uint64_t *p, uint64_t v) {
  __hip_atomic_store((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Batch q's line as posted, or what the slot says instead.  The device
// mirror (sc1 lines, one per slot and XCD) is read first.  A wave that finds it stale
// reads the host's line only if it takes the slot's fetch lock: every wave
// reading the host -- eight 8-byte PCIe reads each -- capped the ring at ~10
// frames/us, and at a launch's start 4 096 waves missing the empty mirror at
// once cost ~0.6 ms.  The lock word is {(q + 1) mod 2^32, time taken};
// it is taken (compare-and-swap, tried only after a plain load found it free)
// when it names another batch, was released, or was taken more than ~20 us
// ago (a mirror line a slower wave overwrote with an older one is fetched
// again).  The holder copies a posted line into the mirror -- with the next
// slot's line when that one is posted too, so the waves that cross into the
// next batch find it there -- or releases the lock when the batch is not
// posted yet, so the next poll can fetch again; the others answer kBusy and
// read the mirror again.  Every word keeps its tag, so a mirror line read
// while it is written is recognised as torn.
constexpr uint32_t kLockHold = 125;  // ~20 us in the lock's 160 ns units
__device__ __forceinline__ LineState fetch(const RingArgs &r, uint64_t q, int lane, uint64_t &w,
                                           int xcd) {
  uint64_t *m = r.mirror + 8 * (kRingSlots * xcd + q % kRingSlots);
  w = lane < 8 ? ag_load64(m + lane) : 0;
  LineState st = classify(w, q, lane);
  if (st == kPosted || st == kReused) return st;
  uint64_t *lk = r.lock + kRingSlots * xcd + q % kRingSlots;
  const uint32_t me = (uint32_t)(q + 1), now = (uint32_t)(ticks() >> 4);
  bool mine = false;
  if (lane == 0) {
    uint64_t cur = ag_load64(lk);
    const bool free_ = (uint32_t)(cur >> 32) != me || (uint32_t)cur == 0u ||
                       now - (uint32_t)cur > kLockHold;
    if (free_)
      mine = __hip_atomic_compare_exchange_strong((gu64 *)lk, &cur, ((uint64_t)me << 32) | (now | 1u),
                                                  __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
  }
  if (__ballot(mine) == 0) return kBusy;  // another wave is fetching it
  const uint64_t *h = reinterpret_cast<const uint64_t *>(r.desc + (q % kRingSlots));
  w = lane < 8 ? sys_load(h + lane) : 0;
  st = classify(w, q, lane);
  if (st == kPosted) {
    if (lane < 8) ag_store64(m + lane, w);
    const uint64_t q1 = q + 1;
    const uint64_t *h1 = reinterpret_cast<const uint64_t *>(r.desc + (q1 % kRingSlots));
    const uint64_t w1 = lane < 8 ? sys_load(h1 + lane) : 0;
    if (classify(w1, q1, lane) == kPosted && lane < 8)
      ag_store64(r.mirror + 8 * (kRingSlots * xcd + q1 % kRingSlots) + lane, w1);
  } else if (lane == 0) {
    // not posted (or torn, or reused): release, so the next poll fetches again
    ag_store64(lk, (uint64_t)me << 32);
  }
  return st;
}

// Moves `bt` forward to the batch holding ticket t.  Returns false when the
// wave must leave: the quit descriptor was reached, or no batch was posted
// for `deadline` ticks.  bt.q starts at the launch's cursor with end =
// start = -1 ("not read yet").
__device__ __forceinline__ bool locate(const RingArgs &r, int64_t t, Batch &bt, int lane, int xcd) {
  bool first = bt.end < 0;  // bt.q itself has not been read yet
  uint64_t t_wait = 0;
  uint32_t nap = 0;
  while (first || t >= bt.end) {
    const uint64_t q = first ? bt.q : bt.q + 1;
    uint64_t w;
    const LineState st = fetch(r, q, lane, w, xcd);
    if (st == kPosted) {
      bt.q = q;
      bt.start = (int64_t)(readlane64(w, 1) & kPay);
      bt.in = reinterpret_cast<const float *>(readlane64(w, 2) & kPay);
      bt.cw = (int64_t)(readlane64(w, 3) & kPay);
      bt.packed = reinterpret_cast<uint8_t *>(readlane64(w, 4) & kPay);
      bt.iters = reinterpret_cast<int32_t *>(readlane64(w, 5) & kPay);
      bt.synd = reinterpret_cast<int32_t *>(readlane64(w, 6) & kPay);
      const uint64_t bq = readlane64(w, 7);
      bt.B = (int)(uint32_t)bq;
      bt.quit = ((bq >> 32) & 1u) != 0;
      bt.end = bt.start + bt.B;
      first = false;
      if (bt.quit) return false;
      t_wait = 0;
      nap = 0;
    } else if (st == kReused) {
      // the slot already holds a later batch: batch q is complete, so it
      // cannot hold the unfinished ticket t
      bt.q = q;
      bt.start = bt.end = t;  // (t >= end: go on to q + 1)
      first = false;
    } else if (st == kNotYet || st == kBusy) {
      // not posted yet, or another wave is fetching the line: read the mirror
      // again after ~0.5 us; once the wait passes ~20 us (the batch is not
      // posted: the ring has nothing to do) back off to ~54 us between polls
      const uint64_t now = ticks();
      if (!t_wait) t_wait = now;
      if (now - t_wait > r.deadline) return false;
      if (now - t_wait < 2000) {
        __builtin_amdgcn_s_sleep(20);
      } else {
        for (uint32_t k = 0; k <= nap; ++k) __builtin_amdgcn_s_sleep(127);  // ~3.4 us each
        nap = nap < 15 ? nap + 1 : nap;
      }
    }  // (kTorn: read again)
  }
  return true;
}

template <int PREC, int METHOD, int S, int NW, int DCN, int DVN, int MINB>
__global__ void __launch_bounds__(kThreads, MINB) ring_kernel(CodeView code, RingArgs r) {
  typedef typename Math<PREC>::Real Real;
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __shared__ typename Math<PREC>::Tab logtab[TabLds<PREC>::kN];
  if constexpr (METHOD == 1) stage_tab<PREC>(logtab);
  WaveTables<S, NW> wt;
  Real *tb, *eb, *rb, *sb;
  int colq[NW];
  uint32_t ppos[2];
  wave_setup<PREC, METHOD, S, NW, DCN, DVN>(code, smem, wave, lane, wt, tb, eb, rb, sb, colq, ppos);
  DecodeArgs a{};
  a.max_iters = r.max_iters;
  a.et_period = r.et_period;
  const int KB = code.KB;

  Batch bt{};
  bt.q = r.cursor0;
  bt.start = bt.end = -1;
  // wave w's first claim is tickets [w c, w c + c) (c = ring_claim); the queue
  // hands out the claims after all the launch's waves' (4 096 first claims
  // on one counter at once took ~46 us: ~88 per us, MI355X_MICROARCH.md
  // "dequeue")
  constexpr int64_t c = ring_claim(METHOD, PREC);
  const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
  int64_t t = r.ticket0 + ((int64_t)blockIdx.x * kWavesPerBlock + wave) * c;
  int64_t tend = t + c;  // end of the current claim
  // frames decoded but not yet counted done: batch pend_q (B = pend_B), count
  uint64_t pend_q = 0;
  int pend_B = 0;
  uint32_t pend_n = 0;
  // counts the pending frames done (their stores drained first); the add that
  // completes a batch resets its counter and signals the host
  auto flush = [&]() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores are out
    if (lane == 0) {
      uint32_t *dn = r.done + (pend_q % kRingSlots) * kRingDoneStride;
      const uint32_t old = __hip_atomic_fetch_add((gu32 *)dn, pend_n, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      if (old + pend_n == (uint32_t)pend_B) {  // the batch's last frames: reset the slot, then signal
        __hip_atomic_store((gu32 *)dn, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        sys_store(r.comp + (pend_q % kRingSlots), pend_q + 1);
      }
    }
    pend_n = 0;
  };
#ifdef LDPC_TIMELINE
  const uint64_t t_wave0 = ticks();
#endif
  // this wave's XCD: its mirror and lock copies live in that XCD's L2 only
  // (an sc1 load polling a line another XCD rewrote kept reading its own
  // L2's copy: at a launch's start every wave off the fetching XCD waited
  // out the ~20 us lock, tools/ring_timeline.py)
  const int xcd = (int)(__builtin_amdgcn_s_getreg((31 << 11) | 20) & (kRingXcds - 1));  // XCC_ID
  while (locate(r, t, bt, lane, xcd)) {
#ifdef LDPC_TIMELINE
    const uint64_t t_f0 = ticks(), c_f0 = __builtin_amdgcn_s_memtime();
#endif
    const int64_t f = t - bt.start;
    const float *src = bt.in + f * bt.cw;
    float xin[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) xin[q] = colq[q] >= 0 ? ag_load(src + colq[q]) : 0.0f;
#ifdef LDPC_TIMELINE
    const uint64_t t_f1 = ticks();  // (samples loaded and the claim issued)
#endif
    FrameResult fr;
    if constexpr (METHOD == 1) {
      bool bad = false;
#pragma unroll
      for (int q = 0; q < NW; ++q) bad |= !__builtin_isfinite(xin[q]);
      if (__ballot(bad) == 0)
        fr = decode_frame<PREC, METHOD, S, NW, DCN, DVN, true, Real, false, false>(
            code, a, f, wt, tb, eb, rb, sb, lane, logtab, xin, colq, ppos);
      else
        fr = decode_frame<PREC, METHOD, S, NW, DCN, DVN, false, Real, false, false>(
            code, a, f, wt, tb, eb, rb, sb, lane, logtab, xin, colq, ppos);
    } else {
      fr = decode_frame<PREC, METHOD, S, NW, DCN, DVN, false, Real, false, false>(
          code, a, f, wt, tb, eb, rb, sb, lane, logtab, xin, colq, ppos);
    }
    // the next claim, taken when the current one's last frame is done: a
    // claim taken at a frame's start waited for the frame (up to 50
    // iterations), and at a session's end the last tickets sat with waves
    // busy on long frames while the others had run out of work
    // (tools/ring_timeline.py: the last frame started 90 us before the end,
    // the queue emptied ~250 us before).  The claim's round trip overlaps the
    // output stores' drain below.
    const bool last = c == 1 || t + 1 == tend;
    uint32_t nt = 0;
    if (last && lane == 0) nt = atomicAdd(r.ticket, (uint32_t)c);
    // outputs, write-through: packed bytes M.. (:207-219) as 32-bit words
    // where the layout allows, iterations, syndrome weight
    uint8_t *pk = bt.packed + f * KB;
    if ((KB & 3) == 0 && (reinterpret_cast<uintptr_t>(pk) & 3) == 0) {
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        word |= ((uint32_t)__shfl((int)fr.byte, (4 * lane + j) & 63) & 255u) << (8 * j);
      if (lane < (KB >> 2)) wt_store(reinterpret_cast<uint32_t *>(pk) + lane, word);
    } else if (lane < KB) {
      wt_store(pk + lane, (uint8_t)fr.byte);
    }
    if (lane == 0) {
      if (bt.iters) wt_store(bt.iters + f, (int32_t)fr.used);
      if (bt.synd) wt_store(bt.synd + f, (int32_t)fr.weight);
    }
    // done counts: one add per claim and batch
    if constexpr (c == 1) {
      pend_q = bt.q;
      pend_B = bt.B;
      pend_n = 1;
      flush();
    } else {
      if (pend_n && pend_q != bt.q) flush();
      pend_q = bt.q;
      pend_B = bt.B;
      pend_n += 1;
    }
#ifdef LDPC_TIMELINE
    {  // per ticket: wave start, frame start, decode start, frame end, wave id |
       // iterations, core clocks of the frame
      const int64_t rel = t - r.ticket0;
      if (lane == 0 && rel >= 0 && rel < kRingTimeline) {
        uint64_t *o = g_ring_timeline + kTlWords * rel;
        o[0] = t_wave0;
        o[1] = t_f0;
        o[2] = t_f1;
        o[3] = ticks();
        o[4] = ((uint64_t)(blockIdx.x * kWavesPerBlock + wave) << 8) | (uint64_t)fr.used;
        o[5] = __builtin_amdgcn_s_memtime() - c_f0;  // core clocks of the frame
      }
    }
#endif
    if (last) {
      t = r.ticket0 + nwaves * c + (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)nt);
      tend = t + c;
    } else {
      t += 1;
    }
    // counted at the claim's end, or before the next ticket leaves the batch
    // (locate may wait there for a batch not posted yet, and the host may be
    // waiting for this one)
    if constexpr (c > 1)
      if (last || t >= bt.end) flush();
  }
  // a claim cut short by the quit descriptor or the deadline: its decoded
  // frames still count
  if constexpr (c > 1)
    if (pend_n) flush();
}

int cus_of(int dev) {
  static std::atomic<int> cus[64];
  if (dev < 0 || dev >= 64) return 256;
  int n = cus[dev].load(std::memory_order_relaxed);
  if (!n) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
    cus[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

template <int PREC, int METHOD, int S, int NW, int DCN, int DVN, int MINB>
int launch_r(const CodeView &code, const RingArgs &r, int dev, hipStream_t st, int *wg) {
  typedef typename Math<PREC>::Real Real;
  const size_t lds = Layout<Real, METHOD, S, NW, DVN>::total;
  const void *fn = (const void *)ring_kernel<PREC, METHOD, S, NW, DCN, DVN, MINB>;
  static std::atomic<int> per_cu_once{0};  // resident workgroups per CU (computed once)
  int per_cu = per_cu_once.load(std::memory_order_relaxed);
  if (!per_cu) {
    if (lds > 65536 &&
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return -3;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kThreads, lds) != hipSuccess || n < 1)
      n = 1;
    // the register budget's waves per SIMD bound the workgroups too (a
    // workgroup past the resident ones only starts when one leaves: a speed
    // matter, never a hang -- no wave waits on another)
    per_cu = std::min(n, std::max(1, 4 * MINB / kWavesPerBlock));
    per_cu_once.store(per_cu, std::memory_order_relaxed);
  }
  const int blocks = per_cu * cus_of(dev);
  *wg = blocks;
  hipLaunchKernelGGL((ring_kernel<PREC, METHOD, S, NW, DCN, DVN, MINB>), dim3((unsigned)blocks),
                     dim3(kThreads), lds, st, code, r);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

#ifndef LDPC_TP_MINB
#define LDPC_TP_MINB 4  // four waves per SIMD (<= 128 VGPRs): the throughput build
#endif

template <int PREC, int METHOD, int NW>
int ring_slots(const CodeView &code, const RingArgs &r, int slots, int dev, hipStream_t st, int *wg) {
  // low-degree codes (the reference's H) get loops sized to their degrees,
  // and four waves per SIMD (ldpc_kernels.hip launch_slots' throughput build)
  if constexpr (NW == 1) {
    if (code.dc_max <= 6 && code.dv_max <= 3) switch (slots) {
        case 1: return launch_r<PREC, METHOD, 1, NW, 5, 3, LDPC_TP_MINB>(code, r, dev, st, wg);
        case 2: return launch_r<PREC, METHOD, 2, NW, 5, 3, LDPC_TP_MINB>(code, r, dev, st, wg);
        case 3: return launch_r<PREC, METHOD, 3, NW, 5, 3, LDPC_TP_MINB>(code, r, dev, st, wg);
        case 4: return launch_r<PREC, METHOD, 4, NW, 5, 3, LDPC_TP_MINB>(code, r, dev, st, wg);
        default: break;
      }
  }
  constexpr int D = kDcMax - 1, V = kDvMax;
  switch (slots) {
    case 1: return launch_r<PREC, METHOD, 1, NW, D, V, 2>(code, r, dev, st, wg);
    case 2: return launch_r<PREC, METHOD, 2, NW, D, V, 2>(code, r, dev, st, wg);
    case 3: return launch_r<PREC, METHOD, 3, NW, D, V, 2>(code, r, dev, st, wg);
    case 4: return launch_r<PREC, METHOD, 4, NW, D, V, 2>(code, r, dev, st, wg);
    case 5: return launch_r<PREC, METHOD, 5, NW, D, V, 2>(code, r, dev, st, wg);
    case 6: return launch_r<PREC, METHOD, 6, NW, D, V, 2>(code, r, dev, st, wg);
    case 7: return launch_r<PREC, METHOD, 7, NW, D, V, 2>(code, r, dev, st, wg);
    case 8: return launch_r<PREC, METHOD, 8, NW, D, V, 2>(code, r, dev, st, wg);
    default: return -2;
  }
}

template <int NW>
int ring_nw(const CodeView &code, const RingArgs &r, int method, int prec, int slots, int dev,
            hipStream_t st, int *wg) {
  if (method == 1) {
    if (prec == 1) return ring_slots<1, 1, NW>(code, r, slots, dev, st, wg);
    if (prec == 2) return ring_slots<2, 1, NW>(code, r, slots, dev, st, wg);
    if (prec == 3) return ring_slots<3, 1, NW>(code, r, slots, dev, st, wg);
    return ring_slots<0, 1, NW>(code, r, slots, dev, st, wg);
  }
  if (method == 0)  // min-sum: both f64 modes are the same arithmetic
    return prec == 1 ? ring_slots<1, 0, NW>(code, r, slots, dev, st, wg)
                     : ring_slots<0, 0, NW>(code, r, slots, dev, st, wg);
  return -2;
}

}  // namespace

int launch_ring(const CodeView &code, const RingArgs &r, int method, int prec, int slots, int nw,
                int device, void *stream, int *workgroups_out) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (nw == 1) return ring_nw<1>(code, r, method, prec, slots, device, st, workgroups_out);
  if (nw == 4) return ring_nw<4>(code, r, method, prec, slots, device, st, workgroups_out);
  return -2;
}

}  // namespace ldpc

#ifdef LDPC_PATH_STATS
extern "C" int ldpc_debug_path_stats(unsigned long long *host, int reset) {
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(ldpc::g_path_stats), 12 * sizeof(unsigned long long)) !=
      hipSuccess)
    return -1;
  if (reset) {
    unsigned long long z[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(ldpc::g_path_stats), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif

#ifdef LDPC_TIMELINE
extern "C" int ldpc_debug_ring_timeline(uint64_t *host, int tickets) {
  if (tickets > ldpc::kRingTimeline) tickets = (int)ldpc::kRingTimeline;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(ldpc::g_ring_timeline),
                             sizeof(uint64_t) * ldpc::kTlWords * tickets) ==
                 hipSuccess
             ? tickets
             : -1;
}
#endif
