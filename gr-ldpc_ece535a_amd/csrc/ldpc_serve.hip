// ldpc_serve.hip -- the decoder block's window server (gfx950).
//
// lib/ldpc_decoder_cb_impl.cc:146-226 decodes one window per step (the N
// samples at the current position, times +-1) and its state machine picks the
// next position from the result.  The block replays that loop on the host over
// decoded windows and asks for the windows a dry run says it will need
// (csrc/block/ldpc_decoder_cb_impl.cc); at the reference's 5 iterations most
// of a call is a chain of such dependent rounds of a few hundred windows, and
// a kernel launch per round costs ~21 us whatever its size: dispatch, the
// kernel's prologue (code tables, the log table into LDS, the window list
// over the bus), completion and the host's wake-up -- against ~6 us for the
// windows' 5 iterations.
//
// Here ONE launch serves every round of a general_work call:
//   * wave 0 of workgroup 0 is the poller: each poll reads the round word in
//     host-mapped memory, {epoch, B}, and the first 511 window keys in one
//     PCIe round trip, and a new round is republished in device memory (the
//     keys of its first 480 windows inside the lines the decoders poll);
//   * every other workgroup is a decoder: tables and the log table are loaded
//     into LDS once, then it waits for a new epoch, decodes windows g, g + G,
//     ... of the round's list (the batch kernels' workgroup-per-frame
//     arithmetic, mw_frame in ldpc_frame.hpp: results equal every other
//     decode of the same samples) and publishes each result as one 8-byte
//     granule {(epoch << 9) | syndrome weight, packed bytes} in host-mapped
//     memory, which the host polls;
//   * B = kServeB ends the launch, and so does a round of a later launch's
//     session (the host overwrote the quit round before the poller saw it);
//     so does a deadline (no round for `deadline` ticks of the 100 MHz
//     clock), after which the host relaunches the server if it still wants a
//     round.
// Visibility: the device reads host memory with system-scope loads (the
// round word and the keys, each key tagged with its round's epoch, so a key
// read before the host wrote it is read again), writes results
// with one system-scope 8-byte store per window, and hands the round word to
// the decoders as one agent-scope (sc1) granule polled with sc1 loads
// (MI355X_MICROARCH.md, inter-workgroup visibility, R2).
#include <atomic>

#include "ldpc_frame.hpp"

namespace ldpc {
namespace {

typedef __attribute__((address_space(1))) uint64_t gu64;

__device__ __forceinline__ uint64_t ticks() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ uint64_t agent_load(const uint64_t *p) {
  return __hip_atomic_load((const gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void agent_store(uint64_t *p, uint64_t v) {
  __hip_atomic_store((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t sys_load(const uint64_t *p) {
  return __hip_atomic_load((const gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(uint64_t *p, uint64_t v) {
  __hip_atomic_store((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The round as the poller publishes it, one 8-byte granule: epoch (bits
// 40..63), the decoders sharing it (20..39), B (0..19).  A decoder takes the
// census (one atomic add, once per launch) when it starts; the windows of a
// round go to the decoders counted when the round was published -- running,
// so no window waits on a workgroup that is not resident.  Host epochs stay
// below 2^23 (ldpc_serve_begin restarts them).  The poller writes the round
// to kCopies lines of ctl, and decoder g polls copy g % kCopies: a thousand
// decoders polling one line queue behind each other for microseconds.
constexpr uint64_t kQuitRound = ~0ull;  // epoch all ones: every decoder leaves
__device__ __forceinline__ uint64_t ctl_word(uint32_t ep, uint32_t live, uint32_t B) {
  return ((uint64_t)ep << 40) | ((uint64_t)(live & 0xFFFFFu) << 20) | (B & 0xFFFFFu);
}
__device__ __forceinline__ uint64_t *ctl_copy(uint64_t *ctl, int i) { return ctl + 16 * i; }
// Where window b's key is published: keys of the first kInlineKeys windows
// ride in the round copies' lines (word 1 + b / 32 of copy b % 32, the line
// decoder b polls, so its poll fetches its key too), the others in dkeys.
// Keys keep the host's epoch tag (bits 40..63): a reader that finds an older
// tag reads again, so no key store has to be ordered before the round word.
constexpr int64_t kInlineKeys = 15 * kServeCopies;
__device__ __forceinline__ uint64_t *key_slot(const ServeArgs &s, int64_t b) {
  return b < kInlineKeys ? s.ctl + 16 * (b % kServeCopies) + 1 + b / kServeCopies
                         : (uint64_t *)s.dkeys + b;
}
// Why a window key must not be gathered (0: it may): no key of this round
// (-1), or a window that reaches past the staged span.  Every decoder checks
// before its gather, whatever the host checked: a persistent kernel that
// polls host memory must not be able to fault on a bad or stale key.
__device__ __forceinline__ uint32_t key_fault(int64_t key, int N, int64_t span) {
  if (key < 0) return kServeLostKey;
  return (key >> 1) + N > span ? kServeBadKey : 0u;
}
__device__ __forceinline__ uint32_t *census_word(uint64_t *ctl) {
  return reinterpret_cast<uint32_t *>(ctl + 16 * kServeCopies);
}
__device__ __forceinline__ uint64_t *diag(uint64_t *ctl, int j) { return ctl + 16 * (kServeCopies + 1) + j; }
// LDPC_SERVE_DEBUG counters; the times are absolute 100 MHz ticks: the
// poller's sight of the round and its publication, the last decoder's key
// read and result store (the host reads them after the round and zeroes the
// last two)
enum { kDiagExit, kDiagExitRound, kDiagStarts, kDiagG0, kDiagResults, kDiagPub, kDiagKey, kDiagDone,
       kDiagSeen };
__device__ __forceinline__ uint32_t census_load(uint64_t *ctl) {
  return __hip_atomic_load((const __attribute__((address_space(1))) uint32_t *)census_word(ctl),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t census_take(uint64_t *ctl) {
  return __hip_atomic_fetch_add((__attribute__((address_space(1))) uint32_t *)census_word(ctl), 1u,
                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void dbg_max(uint64_t *p, uint64_t v) {
  __hip_atomic_fetch_max((__attribute__((address_space(1))) uint64_t *)p, v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void dbg_add(uint64_t *p) {
  __hip_atomic_fetch_add((__attribute__((address_space(1))) uint64_t *)p, (uint64_t)1,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t lane_bcast(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
__device__ __forceinline__ uint64_t wave_uniform(uint64_t v) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}

// The poller (wave 0 of workgroup 0): lane 0 reads the round word, the other
// loads of the same poll the first 511 key slots (host memory, one PCIe
// round trip); a new round's keys -- each tagged with its epoch by the host,
// so a slot read before the host rewrote it is read again -- go to their
// key_slot (agent-scope stores, tags kept), and the round word to the ctl
// copies right behind them.
constexpr int kKeyLoads = 8;
__device__ __forceinline__ void poll_rounds(const ServeArgs &s, int lane) {
  uint32_t last = s.start_epoch;
  const uint64_t t_start = ticks();
  uint64_t t_last = t_start;
  uint32_t live = 0;  // decoders counted by the census
  for (;;) {
    // every poll also reads the first 64 kKeyLoads - 1 key slots (the same
    // PCIe round trip), so a round of up to 511 windows needs no second trip:
    // -0.5..-1.3 us per round of 64..400 windows, +1..2 % on the block at
    // 4 dB / 5 iterations (profiles/round5/serve_preload_ab.txt)
    uint64_t v[kKeyLoads];
#pragma unroll
    for (int j = 0; j < kKeyLoads; ++j)
      v[j] = sys_load(j == 0 && lane == 0 ? s.round : (const uint64_t *)s.keys + (64 * j + lane - 1));
    const uint64_t r = lane_bcast(v[0], 0);
    const uint32_t ep = (uint32_t)(r >> 32);
    if (ep != last) {
      const uint64_t t_seen = ticks();
      // a round of a later launch (this launch's quit round was overwritten
      // before it was seen) ends this launch too
      const bool quit = ((uint32_t)r & kServeB) == kServeB ||
                        (((uint32_t)r >> 20) & 0xFFFu) != (s.session & 0xFFFu);
      const int64_t B = quit ? 0 : (int64_t)((uint32_t)r & kServeB);
      const uint64_t tag = (uint64_t)(ep & 0xFFFFFFu);
      const uint64_t t_keys = ticks();
      bool lost = false;  // a key slot that never showed this epoch (the host is gone)
      // key slot c + 64 j + lane; kKeyLoads loads in flight per lane (the
      // first group, c = -1, is the poll's own read)
      for (int64_t c = -1; c < B && !lost; c += 64 * kKeyLoads) {
        uint64_t k[kKeyLoads];
        bool in[kKeyLoads];
#pragma unroll
        for (int j = 0; j < kKeyLoads; ++j) {
          const int64_t b = c + 64 * j + lane;
          in[j] = b >= 0 && b < B;
          k[j] = c < 0 ? v[j] : (in[j] ? sys_load((const uint64_t *)s.keys + b) : 0);
        }
#pragma unroll
        for (int j = 0; j < kKeyLoads; ++j) {
          const int64_t b = c + 64 * j + lane;
          // (an older tag is read again; a later round's -- the host gave this
          // round up -- is passed on, and the decoders answer it as lost)
          while (!lost && __ballot(in[j] && (k[j] >> 40) < tag)) {
            if (in[j] && (k[j] >> 40) < tag) k[j] = sys_load((const uint64_t *)s.keys + b);
            if (ticks() - t_keys > s.deadline) lost = true;
          }
          if (in[j]) agent_store(key_slot(s, b), k[j]);
        }
      }
      if (lost) {
        if (lane < kServeCopies) agent_store(ctl_copy(s.ctl, lane), kQuitRound);
        if (lane == 0) agent_store(diag(s.ctl, kDiagExit), 3);
        return;
      }
      // the decoders that have started by now share the round: all of them
      // (every workgroup is resident) or, if some never start while this
      // launch runs, those counted 20 us after the launch began -- at least
      // one.  Once all have started the count is not read again, and after
      // the first 20 us only for a round that wants more decoders than were
      // counted (a census load is a trip to memory on the round's path).
      if (live < gridDim.x - 1 && (live == 0 || B > (int64_t)live || ticks() - t_start < 2000)) {
        live = census_load(s.ctl);
        while (!quit && live < gridDim.x - 1 && (live == 0 || ticks() - t_start < 2000)) {
          __builtin_amdgcn_s_sleep(2);
          live = census_load(s.ctl);
          if (ticks() - t_start > s.deadline) break;  // (no decoder at all: give up below)
        }
        live = (uint32_t)__builtin_amdgcn_readfirstlane((int)live);
      }
      const uint64_t w = quit ? kQuitRound : ctl_word(ep, live, (uint32_t)B);
      if (lane < kServeCopies) agent_store(ctl_copy(s.ctl, lane), w);
      if (s.debug && lane == 0) {
        agent_store(diag(s.ctl, kDiagSeen), t_seen);
        agent_store(diag(s.ctl, kDiagPub), ticks());
      }
      last = ep;
      t_last = ticks();
      if (quit) {  // diagnostics: why, and the round word seen
        if (lane == 0) {
          agent_store(diag(s.ctl, kDiagExit), 1);
          agent_store(diag(s.ctl, kDiagExitRound), r);
        }
        return;
      }
    } else if (ticks() - t_last > s.deadline) {
      if (lane < kServeCopies) agent_store(ctl_copy(s.ctl, lane), kQuitRound);
      if (lane == 0) {
        agent_store(diag(s.ctl, kDiagExit), 2);
        agent_store(diag(s.ctl, kDiagExitRound), r);
      }
      return;
    }
  }
}

// Workgroup 0: the poller (wave 0).  Others: decoders.  A round of at most as
// many windows as there are decoders is decoded one window per workgroup
// (mw_frame: S waves, one edge per lane, the lowest latency); a bigger round
// one window per wave (decode_frame, the batch kernels' one-wave form: fewer
// issue slots per window), windows w, w + W, ... for wave w of W.  The two
// forms share the workgroup's LDS (never at the same time).
// Register budget (__launch_bounds__' second operand: waves per SIMD): three
// waves per SIMD (<= 168 VGPRs).  Four (<= 128, the batch kernels' throughput
// build) spill and made every round slower -- one window of 5 iterations 16.9
// against 15.4 us, a round of 4096 windows 107 against 83 us
// (profiles/round5/serve_latency.txt).  Big rounds go to launches instead
// (the block's hybrid, ldpc_decoder_cb_impl.h).
constexpr int kServeWavesPerSimd = 3;
// bytes of the two forms' overlaid frame regions
template <typename Real, int METHOD, int S, int NW, int DVN>
__host__ __device__ size_t serve_lds_main() {
  const size_t a = MwLayout<Real, S, NW>().total, b = (size_t)S * Layout<Real, METHOD, S, NW, DVN>::per_wave;
  return align16(a > b ? a : b);
}  // (__launch_bounds__' second operand: waves per SIMD)
template <int PREC, int METHOD, int S, int NW, int DCN, int DVN>
__global__ void __launch_bounds__(64 * S, kServeWavesPerSimd) serve_kernel(CodeView code, DecodeArgs a, ServeArgs s) {
  typedef typename Math<PREC>::Real Real;
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ int64_t sslot[2];  // the round, the window key (workgroup form)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (blockIdx.x == 0) {
    if (wave == 0) poll_rounds(s, lane);
    return;
  }
  __shared__ typename Math<PREC>::Tab logtab[TabLds<PREC>::kN];
  if constexpr (METHOD == 1) stage_tab<PREC>(logtab);
  // workgroup-per-window form: tables per edge, LDS per MwLayout
  const MwLayout<Real, S, NW> L;
  constexpr int kDummy = 64 * S;
  Real *mtb = reinterpret_cast<Real *>(smem);
  Real *meb = reinterpret_cast<Real *>(smem + L.eb);
  Real *mrb = reinterpret_cast<Real *>(smem + L.waves + (size_t)wave * L.per_wave);
  Real *msb = mrb + 64 * NW;
  MwTables<NW> mt;
  mw_setup<NW>(code, tid, mt);
  // wave-per-window form: the wave's tables in registers, its own LDS slice
  WaveTables<S, NW> wt;
  Real *tb, *eb, *rb, *sb;
  int colq[NW];
  uint32_t ppos[2];
  wave_setup<PREC, METHOD, S, NW, DCN, DVN>(code, smem, wave, lane, wt, tb, eb, rb, sb, colq, ppos);
  if (tid == 0) sslot[1] = (int64_t)census_take(s.ctl);
  __syncthreads();
  const int64_t g = sslot[1];  // this decoder's place among those that started
  const uint64_t *poll = ctl_copy(s.ctl, (int)(g % kServeCopies));
  const uint64_t *my_key = key_slot(s, g);
  // epochs only grow (ctl is zeroed before the launch, below start_epoch)
  uint32_t last = s.start_epoch;
  uint64_t idle = ticks();
  for (;;) {
    if (tid == 0) {  // the next round, and this decoder's key with it
      uint64_t r, k = 0;
      for (int spins = 0;; ++spins) {
        r = agent_load(poll);
        k = agent_load(my_key);
        if ((uint32_t)(r >> 40) > last) break;
        if ((spins & 15) == 15 && ticks() - idle > s.deadline) {
          r = kQuitRound;
          break;
        }
        // every decoder polls every ~0.16 us: with the keys riding in the
        // round lines, a thousand pollers cost the round's sight nothing
        // measurable, and decoders past the first 256 polling 30x less often
        // made rounds of more windows 0.5-1 us slower and the block 2 %
        // slower (profiles/round5/serve_pollers_ab.txt)
        __builtin_amdgcn_s_sleep(6);
      }
      // the workgroup form's key: tagged with the round's epoch (see key_slot).
      // A slot that still holds an older tag is read again; one that never
      // shows this round's tag within the deadline, or already shows a later
      // round's, yields no key (-1: a kServeLostKey granule, no gather).
      if (r != kQuitRound && g < (int64_t)(r & 0xFFFFFu) && (int64_t)(r & 0xFFFFFu) <= (int64_t)((r >> 20) & 0xFFFFFu)) {
        const uint64_t ktag = (r >> 40) & 0xFFFFFFu;
        const uint64_t t_k = ticks();
        while ((k >> 40) < ktag && ticks() - t_k <= s.deadline) k = agent_load(my_key);
        sslot[1] = (k >> 40) == ktag ? (int64_t)(k & ((1ull << 40) - 1)) : -1;
      }
      sslot[0] = (int64_t)r;
    }
    __syncthreads();
    const uint64_t r = (uint64_t)sslot[0];
    if (r == kQuitRound) return;  // every thread of the workgroup
    const uint32_t ep = (uint32_t)(r >> 40), B = (uint32_t)r & 0xFFFFFu;
    const int64_t G = (int64_t)((r >> 20) & 0xFFFFFu);
    const uint64_t tag = (uint64_t)((ep & 0x7FFFFFu) << 9) << 32;
    if (s.debug && tid == 0 && (g & 63) == 0) {  // diagnostics: rounds seen (sampled decoders)
      dbg_add(diag(s.ctl, kDiagStarts));
      if (g == 0) agent_store(diag(s.ctl, kDiagG0), r);
    }
    if ((int64_t)B <= G) {
      // one window per workgroup
      if (g < (int64_t)B) {
        if (tid == 0) {
          mtb[kDummy] = METHOD == 1 ? Real(1) : Math<PREC>::max_();  // (the LDS is shared)
          // (sampled: one decoder in 64, so the counters' atomics do not
          // queue behind each other and time themselves)
          if (s.debug && (g & 63) == 0) dbg_max(diag(s.ctl, kDiagKey), ticks());
        }
        __syncthreads();  // (mw_frame's first barrier orders the key's readers)
        const int64_t key = sslot[1];  // (workgroup-uniform)
        const uint32_t why = key_fault(key, code.N, s.span);
        if (why) {
          if (tid == 0) sys_store(s.res + g, tag | ((uint64_t)why << 32));
        } else {
          uint64_t hard[NW];
          Real post[NW];
          int used = 0;
          const int weight = mw_frame<PREC, METHOD, S, NW, DCN, DVN>(code, a.max_iters, 1, mt, mtb, meb, mrb,
                                                           msb, logtab, a.in + (key >> 1),
                                                           (key & 1) ? -1.0f : 1.0f, 1, hard, post,
                                                           used);
          (void)post;
          if (wave == 0) {  // packed bytes M.. (:207-219), then the granule
            const uint32_t o = mw_packed_byte<NW>(code, hard, lane);
            uint32_t pk = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j)
              pk |= ((uint32_t)__builtin_amdgcn_readlane((int)o, j) & 255u) << (8 * j);
            if (lane == 0) {
              sys_store(s.res + g, tag | ((uint64_t)(uint32_t)weight << 32) | pk);
              if (s.debug && (g & 63) == 0) {
                dbg_add(diag(s.ctl, kDiagResults));
                dbg_max(diag(s.ctl, kDiagDone), ticks());
              }
            }
          }
          wave_lds_sync();
        }
      }
    } else {
      // one window per wave
      const int64_t W = G * S;
      for (int64_t b = g * S + wave; b < (int64_t)B && g < G; b += W) {
        // the key, once it carries this round's tag: an older tag is read
        // again (bounded); a key that never shows this round's tag is not
        // decoded (a kServeLostKey granule), nor is one outside the span
        // (kServeBadKey) -- no gather ever uses a key the checks did not pass
        const uint64_t ktag = ep & 0xFFFFFFu;
        uint64_t kk = wave_uniform(agent_load(key_slot(s, b)));
        const uint64_t t_k = ticks();
        while ((kk >> 40) < ktag && ticks() - t_k <= s.deadline)
          kk = wave_uniform(agent_load(key_slot(s, b)));
        const int64_t key = (kk >> 40) == ktag ? (int64_t)(kk & ((1ull << 40) - 1)) : -1;
        const uint32_t why = key_fault(key, code.N, s.span);
        if (why) {
          if (lane == 0) sys_store(s.res + b, tag | ((uint64_t)why << 32));
          continue;
        }
        const float *src = a.in + (key >> 1);
        const float sgn = (key & 1) ? -1.0f : 1.0f;
        float xin[NW];
#pragma unroll
        for (int q = 0; q < NW; ++q) xin[q] = colq[q] >= 0 ? src[colq[q]] * sgn : 0.0f;
        FrameResult fr;
        if constexpr (METHOD == 1) {
          bool bad = false;
#pragma unroll
          for (int q = 0; q < NW; ++q) bad |= !__builtin_isfinite(xin[q]);
          if (__ballot(bad) == 0)
            fr = decode_frame<PREC, METHOD, S, NW, DCN, DVN, true, Real, false, false>(
                code, a, 0, wt, tb, eb, rb, sb, lane, logtab, xin, colq, ppos);
          else
            fr = decode_frame<PREC, METHOD, S, NW, DCN, DVN, false, Real, false, false>(
                code, a, 0, wt, tb, eb, rb, sb, lane, logtab, xin, colq, ppos);
        } else {
          fr = decode_frame<PREC, METHOD, S, NW, DCN, DVN, false, Real, false, false>(
              code, a, 0, wt, tb, eb, rb, sb, lane, logtab, xin, colq, ppos);
        }
        uint32_t pk = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          pk |= ((uint32_t)__builtin_amdgcn_readlane((int)fr.byte, j) & 255u) << (8 * j);
        if (lane == 0) sys_store(s.res + b, tag | ((uint64_t)(uint32_t)fr.weight << 32) | pk);
      }
    }
    __syncthreads();  // the round's LDS reads done, and every thread has read the round
    last = ep;
    idle = ticks();
  }
}

// CUs of the context's device (not the calling thread's current one: the
// block relaunches a server from its own thread)
int cus_of_device(int dev) {
  static std::atomic<int> cus_of[64];
  if (dev < 0 || dev >= 64) return 256;
  int n = cus_of[dev].load(std::memory_order_relaxed);
  if (!n) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
    cus_of[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

template <int PREC, int METHOD, int S, int NW, int DCN, int DVN>
int launch_s(const CodeView &code, const DecodeArgs &a, const ServeArgs &s, int device,
             hipStream_t st, int *wg) {
  typedef typename Math<PREC>::Real Real;
  // the two forms' LDS, overlaid
  const size_t lds = serve_lds_main<Real, METHOD, S, NW, DVN>();
  const void *fn = (const void *)serve_kernel<PREC, METHOD, S, NW, DCN, DVN>;
  // resident decoder workgroups per CU (the same on every MI355X of a box;
  // computed once, racing threads compute the same value)
  static std::atomic<int> per_cu_once{0};
  int per_cu = per_cu_once.load(std::memory_order_relaxed);
  if (!per_cu) {
    if (lds > 65536 &&
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return -3;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 64 * S, lds) != hipSuccess || n < 1)
      n = 1;
    // the API can count more than the hardware admits (SGPR-limited waves,
    // MI355X_MICROARCH.md "Residency"): workgroups past the resident ones
    // only start once the launch ends, and rounds go to the decoders that
    // started (the census), so this is a speed matter only
    per_cu = std::min(n, 4 * kServeWavesPerSimd / S);
    per_cu_once.store(per_cu, std::memory_order_relaxed);
  }
  const int blocks = (s.blocks_per_cu > 0 ? std::min(per_cu, s.blocks_per_cu) : per_cu) *
                     cus_of_device(device);
  *wg = blocks - 1;
  hipLaunchKernelGGL((serve_kernel<PREC, METHOD, S, NW, DCN, DVN>), dim3((unsigned)blocks),
                     dim3(64 * S), lds, st, code, a, s);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int PREC, int METHOD, int NW>
int serve_slots(const CodeView &code, const DecodeArgs &a, const ServeArgs &s, int slots,
                int dev, hipStream_t st, int *wg) {
  // low-degree codes (the reference's H) get loops sized to their degrees, as
  // the batch kernels (ldpc_kernels.hip launch_slots)
  if constexpr (NW == 1) {
    if (code.dc_max <= 6 && code.dv_max <= 3) switch (slots) {
        case 1: return launch_s<PREC, METHOD, 1, NW, 5, 3>(code, a, s, dev, st, wg);
        case 2: return launch_s<PREC, METHOD, 2, NW, 5, 3>(code, a, s, dev, st, wg);
        case 3: return launch_s<PREC, METHOD, 3, NW, 5, 3>(code, a, s, dev, st, wg);
        case 4: return launch_s<PREC, METHOD, 4, NW, 5, 3>(code, a, s, dev, st, wg);
        default: break;
      }
  }
  constexpr int D = kDcMax - 1, V = kDvMax;
  switch (slots) {
    case 1: return launch_s<PREC, METHOD, 1, NW, D, V>(code, a, s, dev, st, wg);
    case 2: return launch_s<PREC, METHOD, 2, NW, D, V>(code, a, s, dev, st, wg);
    case 3: return launch_s<PREC, METHOD, 3, NW, D, V>(code, a, s, dev, st, wg);
    case 4: return launch_s<PREC, METHOD, 4, NW, D, V>(code, a, s, dev, st, wg);
    default: return -2;  // workgroups of more than 4 waves: launches
  }
}

template <int NW>
int serve_nw(const CodeView &code, const DecodeArgs &a, const ServeArgs &s, int method, int prec,
             int slots, int dev, hipStream_t st, int *wg) {
  if (method == 1) {
    if (prec == 1) return serve_slots<1, 1, NW>(code, a, s, slots, dev, st, wg);
    if (prec == 2) return serve_slots<2, 1, NW>(code, a, s, slots, dev, st, wg);
    if (prec == 3) return serve_slots<3, 1, NW>(code, a, s, slots, dev, st, wg);
    return serve_slots<0, 1, NW>(code, a, s, slots, dev, st, wg);
  }
  if (method == 0)  // min-sum: both f64 modes are the same arithmetic
    return prec == 1 ? serve_slots<1, 0, NW>(code, a, s, slots, dev, st, wg)
                     : serve_slots<0, 0, NW>(code, a, s, slots, dev, st, wg);
  return -2;
}

}  // namespace

int launch_serve(const CodeView &code, const DecodeArgs &a, const ServeArgs &s, int method,
                 int prec, int slots, int nw, int device, void *stream, int *workgroups_out) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (code.KB > 4 || s.start_epoch >= kServeEpochLimit) return -2;
  if (nw == 1) return serve_nw<1>(code, a, s, method, prec, slots, device, st, workgroups_out);
  if (nw == 4) return serve_nw<4>(code, a, s, method, prec, slots, device, st, workgroups_out);
  return -2;
}

}  // namespace ldpc
