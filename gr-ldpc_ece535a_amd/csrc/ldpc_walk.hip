// ldpc_walk.hip -- the decoder block's frame loop on the device (gfx950).
//
// lib/ldpc_decoder_cb_impl.cc:146-226 decodes one window per step -- the N
// samples at the current position, times +-1 -- and a three-state machine
// (out of sync / in sync / in sync inverted) picks the next position from the
// window's syndrome weight.  At the reference's 5 iterations a window is a
// few microseconds of one wave, so a host that plans launches around the
// machine (the block's dry-run replay) spends its time in round trips: ~12
// dependent launches per 4 096-frame call at 4 dB.  Here the machine runs
// inside one persistent launch:
//
//   * wave 0 of workgroup 0 (the walker) steps the machine exactly, 64 frames
//     or search positions per wave instruction (ballots over the window
//     results), writes the output bytes and the sync messages;
//   * ahead of it a speculative cursor in the same wave asks for the windows
//     the loop will probably need -- the frames on the grid, the -tx retry
//     where the 11th failure falls and the sample-by-sample search after it,
//     guessing that the search lands on the same grid -- so results are
//     usually there when the loop arrives;
//   * every other wave of the launch decodes requested windows (the same
//     frame decoder as the batch kernels, ldpc_frame.hpp: results are those of
//     any other decode of the same samples) and publishes each result as one
//     8-byte granule {tag = (epoch << 9) | syndrome weight, packed bytes};
//   * requests are granules too; a decoder claims the next slot of its XCD's
//     queue shard (one atomic add, eight heads) and polls it.
// A window the loop needs that nobody asked for (a false sync's grid, a
// search past the grid position) is requested on the spot and waited for.
//
// Visibility: every hand-off word is written by one agent-scope (sc1) store
// and read by sc1 loads (MI355X_MICROARCH.md, inter-workgroup visibility, R2
// granules); nothing else crosses workgroups.  Every wait is bounded by a
// deadline on the 100 MHz clock: on expiry the walker reports status 1 and the
// host redoes the call on its planner path.
#include "ldpc_frame.hpp"

namespace ldpc {
namespace {

constexpr int kWalkChunks = 4;   // 64-frame chunks one in-sync step of the loop looks at
constexpr int kSpecChunks = 8;   // ... and one of the speculation
constexpr int kVerify = 2;       // guesses settled per speculation step
enum { kProgress = 0, kWait = 1, kEnd = 2 };

// every access goes through global (address space 1) pointers: the sc1
// hand-off loads must be global_, never flat_ (the pointers arrive generic)
typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint8_t gu8;
typedef __attribute__((address_space(3))) uint32_t lu32;  // LDS
__device__ __forceinline__ uint64_t gload(const uint64_t *p) {
  return __hip_atomic_load((const gu64 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gstore(uint64_t *p, uint64_t v) {
  __hip_atomic_store((gu64 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t gload32(const uint32_t *p) {
  return __hip_atomic_load((const gu32 *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gstore32(uint32_t *p, uint32_t v) {
  __hip_atomic_store((gu32 *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ticks() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ uint64_t lowmask(int k) { return k >= 64 ? ~0ull : ((1ull << k) - 1); }
__device__ __forceinline__ int ctz64(uint64_t x) { return x ? __builtin_ctzll(x) : 64; }
// lane index of the n-th (1-based) set bit of x, which has at least n
__device__ __forceinline__ int nth_bit(uint64_t x, int n) {
  for (int i = 1; i < n; ++i) x &= x - 1;
  return __builtin_ctzll(x);
}

// One in-sync look at 64 frames (lane k: frame k) with `err` errors so far:
// R leading frames have results; the loss (the 11th error, :169-176) falls
// on frame kstar if `loss`, else kstar = R; F / P: failing / passing frames
// before kstar.
struct SyncScan {
  int R, kstar;
  bool loss;
  uint64_t F, P;
};

struct Walk {
  const WalkArgs &w;
  const int lane;
  uint32_t *bm;  // LDS bitmap of the windows asked for
  int64_t tail = 0;  // requests posted
  bool full = false;  // the request queue ran out
  // the loop, exactly
  int64_t pos = 0;
  int st = 0, err = 0, prod = 0;
  bool retry = false;  // the -tx retry of a lost frame (:178-198) is pending
  int rpol = 0;
  int lst = 1;   // the in-sync state held last
  int ehst = 1;  // the in-sync state held last on the anchor phase
  int64_t last_pass = 0, anchor_pos = -1;
  int nmsg = 0, gframes = 0, gfails = 0, surprises = 0;
  // the speculative cursor
  bool pon = false, pretry = false;
  int64_t pp = 0;
  int pst = 0, perr = 0, prpol = 0, hst = 1, restarts = 0;
  int64_t pgph = -1, pgc0 = 0, pgc1 = 0;  // grid prefetch: phase, cursor per polarity
  // guess ring: record i in lane i & 63 (loss frame, guessed landing, state)
  int64_t gLp = 0, gland = 0;
  int gst = 0;
  int gh = 0, gt = 0;  // oldest unverified guess, next free
  // diagnostics: surprises at a grid frame / in a search / at a retry,
  // guesses, wrong guesses, restarts because the loop got ahead
  int d_sync = 0, d_out = 0, d_retry = 0, d_guess = 0, d_wrong = 0, d_behind = 0;

  __device__ __forceinline__ Walk(const WalkArgs &a, int l, uint32_t *b) : w(a), lane(l), bm(b) {}

  __device__ __forceinline__ bool ready(uint64_t g) const { return (uint32_t)(g >> 41) == w.epoch; }
  __device__ __forceinline__ static int synd(uint64_t g) { return (int)((g >> 32) & 511u); }
  __device__ __forceinline__ const uint64_t *res(int pol) const { return w.res + (int64_t)pol * w.cap; }
  __device__ __forceinline__ bool fits(int64_t p) const { return p >= 0 && p + w.N <= w.nin; }

  // Which windows were asked for: one bit per (polarity, position) in the
  // walker's LDS (bits = 2 * nin <= 8 * kWalkLdsBytes; the workgroup's other
  // waves have left), set with an atomic OR that also tells whether the bit
  // was already set -- so no window is asked for twice, at LDS latency.
  __device__ __forceinline__ uint32_t bit_index(int64_t p, int pol) const {
    return (uint32_t)(pol ? w.nin + p : p);
  }
  __device__ __forceinline__ bool claim_bit(int64_t p, int pol) {
    const uint32_t i = bit_index(p, pol);
    const uint32_t b = 1u << (i & 31);
    return (__hip_atomic_fetch_or((lu32 *)bm + (i >> 5), b, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP) & b) == 0;
  }
  // ask for window (p, pol) in every lane where `act` (p may differ per
  // lane; no two active lanes name the same window); windows asked for
  // before in this call are skipped
  __device__ __forceinline__ void request(int64_t p, int pol, bool act) {
    act = act && fits(p);
    const bool fresh = act && claim_bit(p, pol);
    const uint64_t m = __ballot(fresh);
    if (!m || !room(__popcll(m))) return;
    if (fresh) {
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      gstore(w.req + tail + below, ((uint64_t)w.epoch << 32) | (uint32_t)((p << 1) | pol));
    }
    tail += __popcll(m);
  }
  __device__ __forceinline__ void request_new(int64_t p, int pol, bool act) { request(p, pol, act); }
  // request slots left?  (the queue ends kWalkClaimSlack slots before its
  // end: decoders claim past the last request.)  Full: nothing more is asked
  // for; a loop that then waits for a window runs into its deadline, and the
  // host redoes the call.  (With the bitmap a window is asked for once, so
  // 2 nin slots always suffice.)
  __device__ __forceinline__ bool room(int n) {
    if (tail + n <= w.req_cap - kWalkClaimSlack) return true;
    full = true;
    return false;
  }
  __device__ __forceinline__ bool requested(int64_t p, int pol) const {
    const uint32_t i = bit_index(p, pol);
    return (((const lu32 *)bm)[i >> 5] >> (i & 31)) & 1u;
  }
  // the search positions a + 1 .. z after a lost frame at a, both polarities
  __device__ __forceinline__ void search(int64_t a, int64_t z) {
    for (int64_t q0 = a + 1; q0 <= z; q0 += 64) {
      const int64_t q = q0 + lane;
      request(q, 0, q <= z);
      request(q, 1, q <= z);
    }
  }
  __device__ __forceinline__ void request_search(int64_t a) { search(a, a + w.N); }
  __device__ __forceinline__ void search_new(int64_t a, int64_t z) { search(a, z); }
  // a position on the stream's grid (this call's newest, else the caller's), -1: none
  __device__ __forceinline__ int64_t anchor() const { return anchor_pos >= 0 ? anchor_pos : w.anchor; }

  // diagnostics: record {ticks | kind << 56, a, b, c}
  int ntr = 0;
  __device__ __forceinline__ void tr(int kind, int64_t a, int64_t b, int64_t c) {
    if (!w.trace || ntr >= w.trace_cap) return;
    if (lane < 4) {
      const uint64_t v = lane == 0 ? (ticks() & ((1ull << 56) - 1)) | ((uint64_t)kind << 56)
                                   : (uint64_t)(lane == 1 ? a : lane == 2 ? b : c);
      ((gu64 *)w.trace)[(int64_t)ntr * 4 + lane] = v;
    }
    ++ntr;
  }
  __device__ __forceinline__ void msg(int code) {
    if (lane == 0) ((gu8 *)w.msgs)[nmsg] = (uint8_t)code;
    ++nmsg;
  }
  // output frame prod + k (:207-219, bytes built by the decoder)
  __device__ __forceinline__ void put(int k, uint32_t packed, bool act) {
    if (!act) return;
    gu8 *o = (gu8 *)w.out + (int64_t)(prod + k) * w.mo;
    if (w.mo == 4) {
      *(gu32 *)o = packed;
    } else {
      for (int b = 0; b < w.mo; ++b) o[b] = (uint8_t)(packed >> (8 * b));
    }
  }

  __device__ __forceinline__ SyncScan scan_sync(uint64_t g, bool val, int e) const {
    const bool rdy = val && ready(g);
    SyncScan s;
    s.R = ctz64(~__ballot(rdy));
    const bool fail = rdy && synd(g) > w.thr;  // checkFrame > M/8 (:166)
    const uint64_t F = __ballot(fail) & lowmask(s.R);
    const int need = 11 - e;
    s.loss = __popcll(F) >= need;
    s.kstar = s.loss ? nth_bit(F, need) : s.R;
    s.F = F & lowmask(s.kstar);
    s.P = __ballot(rdy && !fail) & lowmask(s.kstar);
    return s;
  }

  // -- surprises: windows the loop needs and nobody asked for ---------------
  __device__ __forceinline__ void surprise_sync(int pol) {
    ++surprises;
    ++d_sync;
    tr(1, pos, st, err);
    const int64_t A = anchor();
    if (A < 0 || (pos - A) % w.N == 0) {
      request(pos + lane * w.N, pol, true);  // the grid: the next 64 frames
      return;
    }
    // a grid the speculation did not follow (a false sync): its frames until
    // 11 of them fail, the retries where the 11th may fall, the search after
    detour(pos, pol, err);
  }
  // the windows a grid off the anchor phase needs from frame p on (errors e
  // so far) if every frame fails: up to the 11th failure and a few more, the
  // retries where the 11th may fall, the search from there back to the grid
  __device__ __forceinline__ void detour(int64_t p, int pol, int e) {
    const int64_t N = w.N, A = anchor();
    const int need = 11 - e;
    request_new(p + lane * N, pol, lane < need + 2);
    request_new(p + (int64_t)(need - 1 + lane) * N, pol ^ 1, lane < 3);
    const int64_t L = p + (int64_t)(need - 1) * N;
    search_new(L, A >= 0 ? L + 1 + (((A - L - 1) % N) + N) % N : L + N);
  }
  __device__ __forceinline__ void surprise_out() {
    ++surprises;
    ++d_out;
    tr(2, pos, st, err);
    request(pos + lane, 0, true);
    request(pos + lane, 1, true);
  }

  // -- the loop ---------------------------------------------------------------
  // In sync off the anchor phase (a false sync): the frames up to the 11th
  // error, that frame's -tx retry and the search after it, loaded in one
  // round; if every frame fails and the retry fails -- the usual detour --
  // the loop goes through all of it here.  Anything else: false, and the
  // ordinary steps take the frames one look at a time.
  __device__ __forceinline__ bool e_detour() {
    const int pol = st == 2;
    const int64_t N = w.N;
    const int need = 11 - err;
    const int64_t Lf = pos + (int64_t)(need - 1) * N;
    if (!fits(Lf) || prod + need > w.nout || nmsg + 3 > w.msgs_cap) return false;
    const int64_t f = pos + (int64_t)lane * N;
    const bool in = lane < need;
    const uint64_t gf = in ? gload(res(pol) + f) : 0ull;
    const uint64_t gr = gload(res(pol ^ 1) + Lf);
    const int64_t q = Lf + 1 + lane;
    const bool val = fits(q);
    const uint64_t g0 = val ? gload(res(0) + q) : 0ull;
    const uint64_t g1 = val ? gload(res(1) + q) : 0ull;
    if (__ballot(in && !(ready(gf) && synd(gf) > w.thr))) return false;
    if (!ready(gr) || synd(gr) <= w.thr) return false;
    // frames pos .. Lf - N: in sync, failing, output (:169-176, :207-219)
    put(lane, (uint32_t)gf, lane < need - 1);
    gframes += need;
    gfails += need;
    prod += need - 1;
    pos = Lf;
    msg(kWalkMsgLost);  // the 11th error
    err = 0;
    st = 0;
    lst = pol + 1;
    pos += 1;  // the retry failed: skip one sample (:193-197)
    out_scan(g0, g1, val);
    return true;
  }

  __device__ __forceinline__ int e_sync() {
    const int pol = st == 2;
    const int64_t N = w.N;
    {
      const int64_t A = anchor();
      if (A < 0 || (pos - A) % N == 0)
        ehst = st;
      else if (e_detour())
        return kProgress;
    }
    uint64_t g[kWalkChunks];
    bool val[kWalkChunks];
#pragma unroll
    for (int c = 0; c < kWalkChunks; ++c) {
      const int k = 64 * c + lane;
      const int64_t f = pos + (int64_t)k * N;
      val[c] = f + N <= w.nin && prod + k < w.nout;  // :146-147
      g[c] = val[c] ? gload(res(pol) + f) : 0ull;
    }
    bool moved = false;
#pragma unroll
    for (int c = 0; c < kWalkChunks; ++c) {
      if (!__ballot(val[c])) return moved ? kProgress : kEnd;
      const SyncScan s = scan_sync(g[c], val[c], err);
      if (s.R == 0) {
        if (!moved && !requested(pos, pol)) surprise_sync(pol);
        return moved ? kProgress : kWait;
      }
      put(lane, (uint32_t)g[c], lane < s.kstar);
      if (s.P) {  // two passes N apart in sync: their phase is the stream's grid
        if ((s.P & (s.P << 1)) || ((s.P & 1) && last_pass == pos - N)) anchor_pos = pos;
        last_pass = pos + (int64_t)(63 - __builtin_clzll(s.P)) * N;
      }
      gframes += s.kstar + (s.loss ? 1 : 0);
      gfails += __popcll(s.F) + (s.loss ? 1 : 0);
      err += __popcll(s.F);
      prod += s.kstar;
      pos += (int64_t)s.kstar * N;
      moved = true;
      if (s.loss) {  // :169-176; the -tx retry of this frame follows (e_retry)
        lst = st;
        msg(kWalkMsgLost);
        err = 0;
        st = 0;
        retry = true;
        rpol = pol ^ 1;
        return kProgress;
      }
      if (s.R < 64) return kProgress;
    }
    return kProgress;
  }

  __device__ __forceinline__ int e_retry() {  // :178-198 for the frame at pos, then the search
    const uint64_t g = gload(res(rpol) + pos);
    const int64_t q = pos + 1 + lane;  // the search's first positions, loaded alongside
    const bool val = fits(q);
    const uint64_t g0 = val ? gload(res(0) + q) : 0ull;
    const uint64_t g1 = val ? gload(res(1) + q) : 0ull;
    if (!ready(g)) {
      if (!requested(pos, rpol)) {
        ++surprises;
        ++d_retry;
        tr(3, pos, rpol, 0);
        request(pos, rpol, lane == 0);
      }
      return kWait;
    }
    retry = false;
    if (synd(g) <= w.thr) {
      msg(kWalkMsgInverted);
      st = 2;
      err = 0;
      put(0, (uint32_t)g, lane == 0);
      ++prod;
      pos += w.N;
    } else {
      pos += 1;
      if (prod < w.nout) out_scan(g0, g1, val);
    }
    return kProgress;
  }

  __device__ __forceinline__ int e_out() {  // out of sync: the search, one sample per step
    const int64_t q = pos + lane;
    const bool val = fits(q);
    const uint64_t g0 = val ? gload(res(0) + q) : 0ull;
    const uint64_t g1 = val ? gload(res(1) + q) : 0ull;
    return out_scan(g0, g1, val);
  }
  // positions pos + lane (val), results g0 / g1 at the two polarities
  __device__ __forceinline__ int out_scan(uint64_t g0, uint64_t g1, bool val) {
    const uint64_t vm = __ballot(val);
    if (!vm) return kEnd;
    const bool r0 = ready(g0), r1 = ready(g1);
    const bool p0 = r0 && synd(g0) <= w.thr, p1 = r1 && synd(g1) <= w.thr;
    const bool known = val && (p0 || (r0 && r1));
    const int D = ctz64(~__ballot(known));
    const uint64_t hit = __ballot(known && (p0 || p1)) & lowmask(D);
    if (hit) {
      const int j = ctz64(hit);
      const bool via0 = (__ballot(p0) >> j) & 1;
      const uint32_t pk = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(via0 ? g0 : g1), j);
      pos += j;
      msg(via0 ? kWalkMsgSync : kWalkMsgInverted);  // :201-205 / :187-190
      st = via0 ? 1 : 2;
      err = 0;
      put(0, pk, lane == 0);
      ++prod;
      pos += w.N;
      // a sync off the anchor phase: its detour, asked for now (the
      // speculation finds out as late as this)
      const int64_t A = anchor();
      if (A >= 0 && (pos - A) % w.N != 0) detour(pos, via0 ? 0 : 1, 0);
      return kProgress;
    }
    pos += D;
    if (D < __popcll(vm)) {
      if (!requested(pos, 0) || !requested(pos, 1)) surprise_out();
      return D ? kProgress : kWait;
    }
    return kProgress;
  }

  // -- speculation ------------------------------------------------------------
  // A second cursor (pp, pst, perr, pretry) runs the same loop ahead of the
  // exact one and asks for the windows it touches.  Where a result it needs
  // is not there yet it guesses instead of waiting, logs the guess (one
  // record per lane of a 64-entry ring) and goes on:
  //   S (search): the -tx retry of a lost frame fails (if it is pending) and
  //     the search after it lands on the stream's grid -- the next position
  //     of the anchor phase, else N samples on -- in the home state (the
  //     state last held on that grid);
  //   F (false grid): in sync off the anchor phase (after a false sync, which
  //     most searches meet: a misaligned window passes ~1 % of the time and a
  //     search tries ~126), every frame fails until the 11th error.
  // Each step checks the oldest guesses against the results once they are in;
  // a wrong one rolls the cursor back to the truth at that point and drops
  // the later guesses.  So the cursor follows the loop's real path and asks
  // for a false sync's whole detour (its frames, the retry, the search back)
  // in one go, and the loop rarely finds a window nobody asked for.
  // Frames of the home grid are asked for up to `lead` frames ahead (pg: the
  // next one not asked for).
  __device__ __forceinline__ void p_set(int64_t p, int s_, int e_, bool rt, int rp) {
    pp = p;
    pst = s_;
    perr = e_;
    pretry = rt;
    prpol = rp;
    gt = gh;  // later guesses are void
  }
  __device__ __forceinline__ void p_restart() {
    tr(4, pos, pp, st);
    pon = true;
    ++restarts;
    gh = gt = 0;
    p_set(pos, st, err, retry, rpol);
    hst = ehst;
  }
  __device__ __forceinline__ void p_log(int64_t a, int64_t b, int bits) {
    tr(5, a, b, bits);
    if (lane == (gt & 63)) {
      gLp = a;
      gland = b;
      gst = bits;
    }
    ++gt;
    ++d_guess;
  }
  // Settles the oldest guesses whose results are in (up to kVerify, their
  // results loaded in one round): right ones are dropped, the first wrong one
  // rolls the cursor back
  __device__ __forceinline__ void p_verify() {
    const int n = min(gt - gh, kVerify);
    if (n <= 0) return;
    const int64_t N = w.N;
    int64_t A_[kVerify], Z_[kVerify];
    int W_[kVerify];
    uint64_t ga[kVerify], gb[kVerify], gr[kVerify];
#pragma unroll
    for (int i = 0; i < kVerify; ++i) {
      A_[i] = Z_[i] = 0;
      W_[i] = 0;
      ga[i] = gb[i] = gr[i] = 0ull;
      if (i < n) {
        const int slot = (gh + i) & 63;
        A_[i] = ((int64_t)__builtin_amdgcn_readlane((int)(gLp >> 32), slot) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)gLp, slot);
        Z_[i] = ((int64_t)__builtin_amdgcn_readlane((int)(gland >> 32), slot) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)gland, slot);
        W_[i] = __builtin_amdgcn_readlane(gst, slot);
        const int64_t a = A_[i], z = Z_[i];
        if (W_[i] & 16) {  // F: frames a, a + N, .. z
          const int64_t f = a + (int64_t)lane * N;
          ga[i] = f <= z ? gload(res((W_[i] >> 3) & 1) + f) : 0ull;
        } else {  // S: the retry at a, the search a + 1 .. z
          if (W_[i] & 4) gr[i] = gload(res((W_[i] >> 3) & 1) + a);
          const int64_t q = a + 1 + lane;
          if (q <= z) {
            ga[i] = gload(res(0) + q);
            gb[i] = gload(res(1) + q);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kVerify; ++i) {
      if (i >= n) return;
      const int64_t a = A_[i], z = Z_[i];
      const int gw = W_[i];
      if (gw & 16) {
        const int pol = (gw >> 3) & 1;
        const bool val = a + (int64_t)lane * N <= z;
        if (__ballot(val && !ready(ga[i]))) return;  // not all in yet
        if (!__ballot(val && synd(ga[i]) <= w.thr)) {
          ++gh;
          tr(6, a, z, gw);
          continue;
        }
        ++d_wrong;  // one passes: back to the start, where the cursor now reads them
        tr(7, a, z, gw);
        p_set(a, pol + 1, (gw >> 8) & 15, false, 0);
        return;
      }
      const int gs = gw & 3;  // guessed state after the landing
      if (gw & 4) {
        if (!ready(gr[i])) return;
        if (synd(gr[i]) <= w.thr) {  // the retry passes: in sync inverted at a
          ++d_wrong;
          tr(7, a, z, gw);
          p_set(a + N, 2, 0, false, 0);
          return;
        }
      }
      const bool val = a + 1 + lane <= z;
      const bool r0 = ready(ga[i]), r1 = ready(gb[i]);
      const bool p0 = r0 && synd(ga[i]) <= w.thr, p1 = r1 && synd(gb[i]) <= w.thr;
      const bool known = val && (p0 || (r0 && r1));
      const uint64_t vm = __ballot(val);
      const int D = ctz64(~__ballot(known));
      const uint64_t hit = __ballot(known && (p0 || p1)) & lowmask(D);
      if (hit) {
        const int j = ctz64(hit);
        const int s1 = ((__ballot(p0) >> j) & 1) ? 1 : 2;
        if (a + 1 + j == z && s1 == gs) {
          ++gh;  // right
          tr(6, a, z, gw);
          continue;
        }
        ++d_wrong;
        tr(7, a, a + 1 + j, gw | (s1 << 12));
        p_set(a + 1 + j + N, s1, 0, false, 0);  // a false sync, or another state
        return;
      }
      if (D < __popcll(vm)) return;  // not all in yet
      ++d_wrong;
      tr(7, a, -1, gw);
      p_set(z + 1, 0, 0, false, 0);  // nothing passed up to the guessed landing
      return;
    }
  }
  // guess S from the loss at Lp (retry pending at polarity rp if has_retry)
  __device__ __forceinline__ void p_guess(int64_t Lp, bool has_retry, int rp) {
    const int64_t N = w.N, A = anchor();
    const int64_t land = A >= 0 ? Lp + 1 + (((A - Lp - 1) % N) + N) % N : Lp + N;
    if (has_retry) request_new(Lp, rp, lane == 0);
    search_new(Lp, land);
    p_log(Lp, land, hst | (has_retry ? 4 : 0) | (rp << 3));
    pp = land;  // in sync from the landing frame on (it passes: the scan sees so)
    pst = hst;
    perr = 0;
    pretry = false;
  }
  // waiting: the loop waits for a result (keep the step short, to look again soon)
  __device__ __forceinline__ void p_step(bool waiting) {
    if (pon && pp < pos) ++d_behind;
    if (!pon || pp < pos) p_restart();
    p_verify();
    if (pp < pos) {
      ++d_behind;
      p_restart();
    }
    const int64_t N = w.N;
    const int64_t limit = pos + (int64_t)w.lead * N;
    // several losses per step: the loop takes about three steps per loss
    // while the loop waits and the cursor is ahead (unsettled guesses), the
    // loop is not kept from looking again; behind (after a rollback), the
    // cursor takes a full turn: the windows after the landing it now knows
    // are what the loop will wait for next
    if (waiting && gt - gh >= 2) return;
    for (int it = 0; it < 8; ++it) {
      if (pp >= limit || gt - gh >= 62) {
        tr(11, pp, pst | (pretry << 2), (limit - pos) | ((int64_t)(gt - gh) << 40) | (1ll << 56));
        return;
      }
      if (pretry) {
        const uint64_t g = gload(res(prpol) + pp);
        if (!ready(g)) {
          p_guess(pp, true, prpol);
          continue;
        }
        pretry = false;
        if (synd(g) <= w.thr) {
          pst = 2;
          perr = 0;
          pp += N;
        } else {
          p_guess(pp, false, 0);
        }
        continue;
      }
      if (!pst) {
        // out of sync (a restart in the loop's search, or a wrong landing)
        if (!fits(pp)) {
          tr(11, pp, pst, 3ll << 56);
          return;
        }
        p_guess(pp - 1, false, 0);
        continue;
      }
      const int pol = pst == 2;
      const int64_t A = anchor();
      const bool home = A < 0 || (pp - A) % N == 0;
      uint64_t g[kWalkChunks];
      bool val[kWalkChunks];
      if (home) {
        hst = pst;
        // the grid ahead: one cursor per polarity (pgc[pol], the first frame
        // not asked for), for one phase; only ever moving forward
        const int64_t ph = ((pp % N) + N) % N;
        if (ph != pgph) {
          pgph = ph;
          pgc0 = pgc1 = pp;
        }
        int64_t pg = pol ? pgc1 : pgc0;
        if (pg < pp) pg = pp;
#pragma unroll
        for (int c = 0; c < kWalkChunks; ++c) {
          if (pg >= limit) break;
          const int64_t f = pg + (int64_t)lane * N;
          request_new(f, pol, f < limit);
          pg = min(pg + 64 * N, pg + (limit - pg + N - 1) / N * N);
        }
        if (pol)
          pgc1 = pg;
        else
          pgc0 = pg;
        // kSpecChunks x 64 frames in one round; every loss among them is
        // guessed over (S, landing on this grid) without another load
        uint64_t hg[kSpecChunks];
        const int64_t base = pp;
#pragma unroll
        for (int c = 0; c < kSpecChunks; ++c) {
          const int64_t f = base + (int64_t)(64 * c + lane) * N;
          hg[c] = fits(f) ? gload(res(pol) + f) : 0ull;
        }
        int k = 0;  // frames of the window behind the cursor
        bool stop = false;
#pragma unroll
        for (int c = 0; c < kSpecChunks; ++c) {
          if (!stop && k < 64 * (c + 1)) {
            const bool val = fits(base + (int64_t)(64 * c + lane) * N);
            const uint64_t RM = __ballot(val && ready(hg[c]));
            const uint64_t FM = __ballot(val && ready(hg[c]) && synd(hg[c]) > w.thr) & RM;
            int b = k - 64 * c;
            while (b < 64) {
              const int R = ctz64(~(RM >> b));
              if (R == 0) {
                stop = true;
                break;
              }
              const uint64_t F = (FM >> b) & lowmask(R);
              const int need = 11 - perr;
              if (__popcll(F) < need) {
                perr += __popcll(F);
                b += R;
                continue;
              }
              const int kk = b + nth_bit(F, need);  // the 11th failure
              const int64_t Lp = base + (int64_t)(64 * c + kk) * N;
              // the search lands on the first frame after it known to pass
              // (frames known to fail before it, at most 8, are searched
              // through), else on the next one
              const uint64_t after = kk + 1 < 64 ? RM >> (kk + 1) : 0ull;
              const int run = min(ctz64(~after), 8);
              const uint64_t passes =
                  kk + 1 < 64 ? (after & ~(FM >> (kk + 1))) & lowmask(run) : 0ull;
              const int j = passes ? kk + 1 + ctz64(passes) : kk + 1 + run;
              const int64_t land = base + (int64_t)(64 * c + j) * N;
              request_new(Lp, pol ^ 1, lane == 0);
              search_new(Lp, land);
              p_log(Lp, land, pst | 4 | ((pol ^ 1) << 3));
              perr = 0;
              b = j;
              if (gt - gh >= 62) {
                stop = true;
                break;
              }
            }
            k = 64 * c + b;
          }
        }
        pp = base + (int64_t)k * N;
        return;
      } else {
        // a false grid: its frames up to the 11th error; guess F if they are
        // not all in, else read them like any other
        const int need = 11 - perr;
        const int64_t f = pp + (int64_t)lane * N;
        const bool in = lane < need && fits(f);
        const uint64_t gf = in ? gload(res(pol) + f) : 0ull;
        if (__ballot(in && !ready(gf))) {
          const int64_t Lf = pp + (int64_t)(need - 1) * N;
          if (!fits(Lf)) return;
          request_new(f, pol, in && !ready(gf));
          p_log(pp, Lf, 16 | (pol << 3) | (perr << 8));
          pp = Lf;  // the 11th error: the retry next
          perr = 0;
          pretry = true;
          prpol = pol ^ 1;
          pst = 0;
          continue;
        }
        val[0] = lane < need && fits(f);
        g[0] = gf;
#pragma unroll
        for (int c = 1; c < kWalkChunks; ++c) {
          val[c] = false;
          g[c] = 0ull;
        }
      }
      bool lost = false;
      tr(12, pp, pst | (home << 3), pgc0);
#pragma unroll
      for (int c = 0; c < kWalkChunks; ++c) {
        if (!__ballot(val[c])) {
          tr(11, pp, pst, 4ll << 56);
          return;
        }
        const SyncScan sc = scan_sync(g[c], val[c], perr);
        perr += __popcll(sc.F);
        pp += (int64_t)sc.kstar * N;
        if (sc.loss) {  // the 11th failure: the retry next
          perr = 0;
          pretry = true;
          prpol = pol ^ 1;
          pst = 0;
          lost = true;
          break;
        }
        if (sc.R < 64) {
          tr(11, pp, pst, (5ll << 56) | sc.R);
          return;
        }
      }
      if (!lost) {
        tr(11, pp, pst, 6ll << 56);
        return;
      }
    }
  }
};

// Compiled once (not per decoder instantiation); its arguments are the
// kernel's, copied to LDS by the caller, and its state lives in registers.
__device__ __attribute__((noinline)) void walker_run(const WalkArgs &w, uint32_t *bm) {
  const int lane = threadIdx.x & 63;
  // clear the bitmap: 2 nin bits
  const int words = (int)((2 * w.nin + 31) / 32);
  for (int i = lane; i < words; i += 64) ((lu32 *)bm)[i] = 0u;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  Walk k(w, lane, bm);
  k.st = w.state;
  k.err = w.errors;
  k.last_pass = w.last_pass;
  const uint64_t t0 = ticks();
  uint64_t t_last = t0, t_moved = t0, wait_ticks = 0;
  int status = 0, waits = 0, steps = 0;
  for (;; ++steps) {
    if (!k.retry && (w.nin - k.pos < w.N || k.prod >= w.nout || k.nmsg + 2 > w.msgs_cap)) break;
    int r = kProgress;
    for (int e = 0; e < 4 && r == kProgress; ++e) {
      if (!k.retry && (w.nin - k.pos < w.N || k.prod >= w.nout || k.nmsg + 2 > w.msgs_cap)) {
        r = kEnd;
        break;
      }
      r = k.retry ? k.e_retry() : (k.st ? k.e_sync() : k.e_out());
      k.tr(8 + r, k.pos, k.st, k.pp);
    }
    if (r == kEnd && !k.retry) break;
    k.p_step(r == kWait);
    const uint64_t t = ticks();
    if (r == kWait) {
      ++waits;
      wait_ticks += t - t_last;
      if (t - t_moved > w.deadline || (k.full && t - t_moved > w.deadline / 16)) {
        status = k.full ? 2 : 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    } else {
      t_moved = t;
    }
    t_last = t;
  }
  if (lane == 0) {
    __attribute__((address_space(1))) WalkSummary *s =
        (__attribute__((address_space(1))) WalkSummary *)w.sum;
    s->consumed = k.pos;
    s->last_pass = k.last_pass;
    s->anchor_pos = k.anchor_pos;
    s->produced = k.prod;
    s->state = k.st;
    s->errors = k.err;
    s->status = status;
    s->n_msgs = k.nmsg;
    s->grid_frames = k.gframes;
    s->grid_fails = k.gfails;
    s->requests = (int32_t)k.tail;
    s->surprises = k.surprises;
    s->waits = waits;
    s->steps = steps;
    s->restarts = k.restarts;
    s->diag[0] = k.d_sync;
    s->diag[1] = k.d_out;
    s->diag[2] = k.d_retry;
    s->diag[3] = k.d_guess;
    s->diag[4] = k.d_wrong;
    s->diag[5] = k.d_behind;
    s->wait_ticks = (int64_t)wait_ticks;
    s->total_ticks = (int64_t)(ticks() - t0);
    gstore32(w.ctl + kWalkDone, 1u);
  }
}

// Workgroup 0: the walker (wave 0; its other waves leave).  Every other wave:
// a decoder pulling requests until the walker is done.
template <int PREC, int METHOD, int S, int NW, int DCN, int DVN>
__global__ void __launch_bounds__(kThreads, 1)
    walk_small_kernel(CodeView code, DecodeArgs a, WalkArgs w) {
  typedef typename Math<PREC>::Real Real;
  extern __shared__ __align__(16) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  __shared__ typename Math<PREC>::Tab logtab[TabLds<PREC>::kN];
  if constexpr (METHOD == 1) stage_tab<PREC>(logtab);
  if (blockIdx.x == 0) {
    if (wave == 0) {
      __shared__ WalkArgs wl;
      if (lane == 0) wl = w;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      walker_run(wl, reinterpret_cast<uint32_t *>(smem));
    }
    return;
  }
  WaveTables<S, NW> wt;
  Real *tb, *eb, *rb, *sb;
  int colq[NW];
  uint32_t ppos[2];
  wave_setup<PREC, METHOD, S, NW, DCN, DVN>(code, smem, wave, lane, wt, tb, eb, rb, sb, colq, ppos);
  // the queue shard of this wave's XCD (speed only: any shard is correct)
  const uint32_t x = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;
  uint64_t idle = ticks();
  for (;;) {
    uint32_t c = 0;
    if (lane == 0)
      c = __hip_atomic_fetch_add((gu32 *)(w.ctl + 32 * x), 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    c = (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
    const int64_t i = (int64_t)c * 8 + x;
    uint32_t key = 0;
    for (int spins = 0;; ++spins) {
      const uint64_t g = i < w.req_cap ? gload(w.req + i) : 0ull;
      if ((uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(g >> 32)) == w.epoch) {
        key = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)g);
        break;
      }
      if ((spins & 7) == 7 && (gload32(w.ctl + kWalkDone) != 0u || ticks() - idle > w.deadline))
        return;
      if (spins < 8)
        __builtin_amdgcn_s_sleep(1);
      else
        __builtin_amdgcn_s_sleep(4);
    }
    const uint64_t t_got = ticks();
    // window key: the N samples from position key >> 1, negated when key & 1
    const int64_t p = key >> 1;
    const float sgn = (key & 1) ? -1.0f : 1.0f;
    const __attribute__((address_space(1))) float *src =
        (const __attribute__((address_space(1))) float *)a.in + p;
    float xin[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) xin[q] = colq[q] >= 0 ? src[colq[q]] * sgn : 0.0f;
    FrameResult r;
    if constexpr (METHOD == 1) {
      bool bad = false;
#pragma unroll
      for (int q = 0; q < NW; ++q) bad |= !__builtin_isfinite(xin[q]);
      if (__ballot(bad) == 0)
        r = decode_frame<PREC, METHOD, S, NW, DCN, DVN, true, Real, false>(
            code, a, 0, wt, tb, eb, rb, sb, lane, logtab, xin, colq, ppos);
      else
        r = decode_frame<PREC, METHOD, S, NW, DCN, DVN, false, Real, false>(
            code, a, 0, wt, tb, eb, rb, sb, lane, logtab, xin, colq, ppos);
    } else {
      r = decode_frame<PREC, METHOD, S, NW, DCN, DVN, false, Real, false>(
          code, a, 0, wt, tb, eb, rb, sb, lane, logtab, xin, colq, ppos);
    }
    uint32_t pk = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      pk |= ((uint32_t)__builtin_amdgcn_readlane((int)r.byte, j) & 255u) << (8 * j);
    const uint64_t out = ((uint64_t)((w.epoch << 9) | (uint32_t)r.weight) << 32) | pk;
    if (lane == 0) gstore(w.res + (int64_t)(key & 1) * w.cap + p, out);
    idle = ticks();
    if (w.trace && lane == 0) {  // diagnostics: decode time and count
      __hip_atomic_fetch_add((gu32 *)(w.ctl + 264), (uint32_t)(idle - t_got), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add((gu32 *)(w.ctl + 265), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

int cus_now() {
  static int cus_of[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus_of[dev] &&
      hipDeviceGetAttribute(&cus_of[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus_of[dev] = 256;
  return cus_of[dev];
}

// The decoders in workgroup form (LDPC_WALK_MW, sum-product and min-sum):
// each workgroup of S waves decodes one window at a time, one edge per lane
// -- the decode_mw_kernel arithmetic (ldpc_kernels.hip), whose iteration is
// ~1.1 us against ~2 us for one wave -- so a round of the loop's chain (a
// false sync's detour) waits less.  Workgroup 0 is the walker, as above.
template <int PREC, int METHOD, int S, int NW>
__global__ void __launch_bounds__(64 * S)
    walk_mw_kernel(CodeView code, DecodeArgs a, WalkArgs w) {
  typedef typename Math<PREC>::Real Real;
  extern __shared__ __align__(16) unsigned char smem[];
  const MwLayout<Real, S, NW> L;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = code.M, N = code.N;
  constexpr int kDummy = 64 * S;
  __shared__ typename Math<PREC>::Tab logtab[TabLds<PREC>::kN];
  if constexpr (METHOD == 1) stage_tab<PREC>(logtab);
  if (blockIdx.x == 0) {
    if (wave == 0) {
      __shared__ WalkArgs wl;
      if (lane == 0) wl = w;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      walker_run(wl, reinterpret_cast<uint32_t *>(smem));
    }
    return;
  }
  Real *tb = reinterpret_cast<Real *>(smem);
  Real *eb = reinterpret_cast<Real *>(smem + L.eb);
  Real *rb = reinterpret_cast<Real *>(smem + L.waves + (size_t)wave * L.per_wave);
  Real *sb = rb + 64 * NW;
  int *fslot = reinterpret_cast<int *>(smem + L.fslot);
  if (tid == 0) tb[kDummy] = METHOD == 1 ? Real(1) : Math<PREC>::max_();
  uint32_t rn[4], cn[2], ce[NW][2];
  {
    const uint4 r = reinterpret_cast<const uint4 *>(code.erow)[tid];
    rn[0] = r.x;
    rn[1] = r.y;
    rn[2] = r.z;
    rn[3] = r.w;
    const uint2 c = reinterpret_cast<const uint2 *>(code.ecol)[tid];
    cn[0] = c.x;
    cn[1] = c.y;
  }
  uint64_t rowmask[NW][NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const uint4 c = reinterpret_cast<const uint4 *>(code.cols)[lane + 64 * q];
    ce[q][0] = c.x;
    ce[q][1] = c.y;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const int j = lane + 64 * q;
      rowmask[q][k] = j < M ? code.rowmask[j * NW + k] : 0ull;
    }
  }
  int col = field(rn, 7);
  col = col != kNone ? col : 0;
  int colq[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const uint32_t c = code.lane_col[lane + 64 * q];
    colq[q] = c == kNone ? -1 : (int)c;
  }
  const uint32_t x = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20) & 7u;
  uint64_t idle = ticks();
  for (;;) {
    if (tid == 0) {  // claim a slot of this XCD's shard, wait for its request
      const uint32_t c = __hip_atomic_fetch_add((gu32 *)(w.ctl + 32 * x), 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      const int64_t i = (int64_t)c * 8 + x;
      int key = -1;
      for (int spins = 0;; ++spins) {
        const uint64_t g = i < w.req_cap ? gload(w.req + i) : 0ull;
        if ((uint32_t)(g >> 32) == w.epoch) {
          key = (int)(uint32_t)g;
          break;
        }
        if ((spins & 7) == 7 &&
            (gload32(w.ctl + kWalkDone) != 0u || ticks() - idle > w.deadline))
          break;
        if (spins < 8)
          __builtin_amdgcn_s_sleep(1);
        else
          __builtin_amdgcn_s_sleep(4);
      }
      *fslot = key;
    }
    __syncthreads();
    const int key = *fslot;
    if (key < 0) return;  // the walk is over (every thread of the workgroup)
    const int64_t p = key >> 1;
    const float polv = (key & 1) ? -1.0f : 1.0f;
    const __attribute__((address_space(1))) float *src =
        (const __attribute__((address_space(1))) float *)a.in + p;
    Real post[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      const int c = lane + 64 * q;
      float xv = 0.0f;
      if (colq[q] >= 0) xv = src[colq[q]] * polv;
      rb[c] = -(Real)xv;
      post[q] = (Real)xv;
    }
    __syncthreads();
    uint64_t hard[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) hard[q] = 0;
    int weight = 0;
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
    (void)post;
    if (wave == 0) {  // packed bytes M.. (:207-219), then the granule
      uint32_t o = 0;
      if (lane < code.KB) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = M + 8 * lane + j;
          if (c < N) {
            const int xp = code.col_lane[c];  // position of column c
            o |= (uint32_t)((word_at<NW>(hard, xp >> 6) >> (xp & 63)) & 1) << (7 - j);
          }
        }
      }
      uint32_t pk = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        pk |= ((uint32_t)__builtin_amdgcn_readlane((int)o, j) & 255u) << (8 * j);
      const uint64_t out = ((uint64_t)((w.epoch << 9) | (uint32_t)weight) << 32) | pk;
      if (lane == 0) gstore(w.res + (int64_t)(key & 1) * w.cap + p, out);
    }
    wave_lds_sync();
    __syncthreads();  // the window's LDS reads done before the next window's writes
    idle = ticks();
  }
}

template <int PREC, int METHOD, int S, int NW>
int launch_wmw(const CodeView &code, const DecodeArgs &a, const WalkArgs &w, hipStream_t st) {
  typedef typename Math<PREC>::Real Real;
  const size_t bm = (size_t)((2 * w.nin + 127) / 128) * 16;  // the walker's bitmap
  const size_t lds = std::max(MwLayout<Real, S, NW>().total, bm);
  const void *fn = (const void *)walk_mw_kernel<PREC, METHOD, S, NW>;
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, kWalkLdsBytes) !=
        hipSuccess)
      return -3;
    attr = true;
  }
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 64 * S, lds) != hipSuccess || n < 1)
    n = 1;
  const char *e = getenv("LDPC_WALK_BLOCKS_PER_CU");
  const int blocks = std::min(n, e ? std::max(atoi(e), 1) : 4) * cus_now();
  hipLaunchKernelGGL((walk_mw_kernel<PREC, METHOD, S, NW>), dim3((unsigned)blocks),
                     dim3(64 * S), lds, st, code, a, w);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int PREC, int METHOD, int NW>
int walk_mw_slots(const CodeView &code, const DecodeArgs &a, const WalkArgs &w, int slots,
                  hipStream_t st) {
  switch (slots) {
    case 1: return launch_wmw<PREC, METHOD, 1, NW>(code, a, w, st);
    case 2: return launch_wmw<PREC, METHOD, 2, NW>(code, a, w, st);
    case 3: return launch_wmw<PREC, METHOD, 3, NW>(code, a, w, st);
    case 4: return launch_wmw<PREC, METHOD, 4, NW>(code, a, w, st);
    default: return -2;
  }
}


template <int PREC, int METHOD, int S, int NW, int DCN, int DVN>
int launch_w(const CodeView &code, const DecodeArgs &a, const WalkArgs &w, int blocks,
             hipStream_t st) {
  typedef typename Math<PREC>::Real Real;
  // the decoders' slices, and the walker's bitmap in workgroup 0
  const size_t lds = std::max(Layout<Real, METHOD, S, NW, DVN>::total, (size_t)kWalkLdsBytes);
  const void *fn = (const void *)walk_small_kernel<PREC, METHOD, S, NW, DCN, DVN>;
  static int per_cu = 0;  // resident workgroups per CU (all of them run at once)
  if (!per_cu) {
    // one workgroup per CU by default (LDPC_WALK_BLOCKS_PER_CU): ~1 000
    // decoder waves serve the walk's requests, and the walker's CU is shared
    // with one other workgroup at most
    if (lds > 65536 &&
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return -3;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kThreads, lds) != hipSuccess || n < 1)
      n = 1;
    per_cu = n;
  }
  const char *e = getenv("LDPC_WALK_BLOCKS_PER_CU");
  if (blocks <= 0) blocks = std::min(per_cu, e ? std::max(atoi(e), 1) : 1) * cus_now();
  hipLaunchKernelGGL((walk_small_kernel<PREC, METHOD, S, NW, DCN, DVN>), dim3((unsigned)blocks),
                     dim3(kThreads), lds, st, code, a, w);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int PREC, int METHOD, int NW>
int walk_slots(const CodeView &code, const DecodeArgs &a, const WalkArgs &w, int slots, int blocks,
               hipStream_t st) {
  if constexpr (NW == 1 && METHOD <= 1) {
    if (code.dc_max <= 6 && code.dv_max <= 3) switch (slots) {
        case 1: return launch_w<PREC, METHOD, 1, NW, 5, 3>(code, a, w, blocks, st);
        case 2: return launch_w<PREC, METHOD, 2, NW, 5, 3>(code, a, w, blocks, st);
        case 3: return launch_w<PREC, METHOD, 3, NW, 5, 3>(code, a, w, blocks, st);
        case 4: return launch_w<PREC, METHOD, 4, NW, 5, 3>(code, a, w, blocks, st);
        default: break;
      }
  }
  constexpr int D = kDcMax - 1, V = kDvMax;
  switch (slots) {
    case 1: return launch_w<PREC, METHOD, 1, NW, D, V>(code, a, w, blocks, st);
    case 2: return launch_w<PREC, METHOD, 2, NW, D, V>(code, a, w, blocks, st);
    case 3: return launch_w<PREC, METHOD, 3, NW, D, V>(code, a, w, blocks, st);
    case 4: return launch_w<PREC, METHOD, 4, NW, D, V>(code, a, w, blocks, st);
    case 5: return launch_w<PREC, METHOD, 5, NW, D, V>(code, a, w, blocks, st);
    case 6: return launch_w<PREC, METHOD, 6, NW, D, V>(code, a, w, blocks, st);
    case 7: return launch_w<PREC, METHOD, 7, NW, D, V>(code, a, w, blocks, st);
    case 8: return launch_w<PREC, METHOD, 8, NW, D, V>(code, a, w, blocks, st);
    default: return -2;
  }
}

template <int NW>
int walk_nw(const CodeView &code, const DecodeArgs &a, const WalkArgs &w, int method, int prec,
            int slots, int blocks, hipStream_t st) {
  constexpr int D = kDcMax - 1, V = kDvMax;
  if (method == 3) return launch_w<1, 3, 1, NW, D, V>(code, a, w, blocks, st);
  if (method == 2) return launch_w<1, 2, 1, NW, D, V>(code, a, w, blocks, st);
  if (method == 1) {
    if (prec == 1) return walk_slots<1, 1, NW>(code, a, w, slots, blocks, st);
    if (prec == 2) return walk_slots<2, 1, NW>(code, a, w, slots, blocks, st);
    if (prec == 3) return walk_slots<3, 1, NW>(code, a, w, slots, blocks, st);
    return walk_slots<0, 1, NW>(code, a, w, slots, blocks, st);
  }
  return prec == 1 ? walk_slots<1, 0, NW>(code, a, w, slots, blocks, st)
                   : walk_slots<0, 0, NW>(code, a, w, slots, blocks, st);
}

}  // namespace

int launch_walk(const CodeView &code, const DecodeArgs &a, const WalkArgs &w, int method,
                int prec, int slots, int nw, int blocks, void *stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (w.KB > 4 || w.mo > 4 || w.epoch == 0 || w.epoch >= (1u << 23)) return -2;
  // LDPC_WALK_MW=1: workgroup decoders for sum-product / min-sum (codes with
  // <= 4 edge slots)
  const bool mw = getenv("LDPC_WALK_MW") && getenv("LDPC_WALK_MW")[0] == '1';
  if (mw && method <= 1 && slots <= 4) {
    if (nw == 1) {
      if (method == 1)
        return prec == 1 ? walk_mw_slots<1, 1, 1>(code, a, w, slots, st)
             : prec == 2 ? walk_mw_slots<2, 1, 1>(code, a, w, slots, st)
             : prec == 3 ? walk_mw_slots<3, 1, 1>(code, a, w, slots, st)
                         : walk_mw_slots<0, 1, 1>(code, a, w, slots, st);
      return prec == 1 ? walk_mw_slots<1, 0, 1>(code, a, w, slots, st)
                       : walk_mw_slots<0, 0, 1>(code, a, w, slots, st);
    }
  }
  if (nw == 1) return walk_nw<1>(code, a, w, method, prec, slots, blocks, st);
  if (nw == 4) return walk_nw<4>(code, a, w, method, prec, slots, blocks, st);
  return -2;
}

}  // namespace ldpc
