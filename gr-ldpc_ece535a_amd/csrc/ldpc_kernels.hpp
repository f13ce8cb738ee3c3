// ldpc_kernels.hpp -- shared host/device types of the MI355X decode path.
//
// The decoder's view of H is held as per-edge / per-column records in HBM,
// built once per context (ldpc_capi.hip) from the reordered dense H of
// lib/ldpc_decoder_cb_impl.cc:98-106.  Edges are numbered in CSR order
// (row-major, ascending column), which is the order the reference's dense
// scans visit them.
#pragma once

#include <stdint.h>

namespace ldpc {

// one frame (codeword) per 64-lane wave; waves per workgroup of the one-wave
// kernel (a workgroup's LDS is released when its last wave ends)
#ifndef LDPC_WAVES_PER_BLOCK
#define LDPC_WAVES_PER_BLOCK 4
#endif
constexpr int kWavesPerBlock = LDPC_WAVES_PER_BLOCK;
constexpr int kThreads = 64 * kWavesPerBlock;
constexpr int kDcMax = 8;          // check-degree limit of the small-code kernel
constexpr int kDvMax = 4;          // variable-degree limit
constexpr int kSlotsMax = 8;       // edge slots per lane: E <= 512
constexpr int kNMax = 256;         // 4 x 64-bit hard-decision words
constexpr int kMMax = 256;         // 4 row slots per lane
constexpr uint16_t kNone = 0xFFFF;

// One edge (j, i) of H, split in two 16/8-byte records so each pass reads
// its half with one LDS load.  rn: the other edges of row j in ascending
// column order -- the order of the product T *= tanh(M(j,k)/2) at :507-511
// and of the minimum scan at :363-369.  cn: the other edges of column i in
// ascending row order -- the order of the sum at :544-548.  Unused entries
// are kNone; records of padding edges (index >= E) have col == kNone.
struct alignas(16) EdgeRowRec {
  uint16_t rn[kDcMax - 1];
  uint16_t col;
};  // 16 bytes
struct alignas(8) EdgeColRec {
  uint16_t cn[kDvMax - 1];
  uint16_t col;
};  // 8 bytes

// One column i: its edges and their rows in ascending row order (the sums
// at :521-525 and :381-385, and the bit-flip vote at :457-461).
struct alignas(16) ColRec {
  uint16_t e[kDvMax];
  uint16_t r[kDvMax];
};  // 16 bytes

// Edge records live at their edge's cell (lane slot 64 s + lane) and column
// records at their column's lane position (lane + 64 q), both chosen per H by
// plan_layout (ldpc_layout.hpp) so the kernel's LDS gathers are free of bank
// conflicts; record fields hold cells / positions.  Positions 0..N-1 hold the
// columns (in some order), positions >= N none.
struct CodeView {
  const EdgeRowRec *erow;    // 64 * S records, by cell
  const EdgeColRec *ecol;    // 64 * S records, by cell
  const ColRec *cols;        // 64 * NW records by position; records >= N are all kNone
  const uint64_t *rowmask;   // M x NW words: bit p of row j <=> H(j, column at position p)
  const uint16_t *lane_col;  // 64 * NW: column at position p (kNone past N)
  const uint8_t *col_lane;   // N: position of column c
  uint64_t dpos[2];          // byte g: identity cell (tb[64 S + dpos]) of 32-lane group g
  int M, N, E, KB, rs;       // rs = ceil(M / 64)
  int dc_max, dv_max;        // largest check / variable degree
  int dc_min;                // smallest check degree
};

struct DecodeArgs {
  const float *in;           // frame b, sample i: in[b*cw_stride + i*elem_stride]
  int64_t cw_stride;
  int elem_stride;
  float polarity;
  int B;
  // both polarities in one launch (the block's OUT_OF_SYNC search, :178-198):
  // when pm_half > 0, frames b >= pm_half decode window b - pm_half with
  // -polarity (B = 2 * pm_half)
  int pm_half;
  // windows of one span (ldpc_decode_windows): when set, frame b is the N
  // samples from in + (win[b] >> 1) * elem_stride, negated when win[b] & 1
  // (cw_stride and pm_half unused)
  const int64_t *win;
  int max_iters;
  int et_period;
  uint8_t *packed;           // B x KB
  uint8_t *bits;             // B x N   (optional)
  int32_t *iters;            // B       (optional)
  int32_t *synd;             // B       (optional)
  float *llr;                // B x N   (optional)
  // persistent scheduling: `waves` resident waves take frames 0..waves-1,
  // then pull the next frame index from *ticket, a monotonic counter owned by
  // the (context, stream) pair: frame = waves + (atomicAdd(ticket, 1) -
  // ticket_base).  A launch adds exactly B to its counter (one add per frame
  // decoded, the last add of each wave being the one past the batch), so the
  // host advances ticket_base by B per launch and no launch ever zeroes a
  // counter: launches on different streams use different counters and
  // cannot disturb each other's queues.
  uint32_t *ticket;
  uint32_t ticket_base;
  int waves;
  // 1: no queue -- wave (workgroup) w takes frames w, w + waves, w + 2 waves,
  // ... and the counter is untouched.  For launches of short frames (small
  // iteration caps: the block's windows at the reference's 5 iterations) the
  // one counter's atomics were the bottleneck -- one word serves ~88 adds per
  // us (MI355X_MICROARCH.md), 8 192 frames ~93 us -- while frames of similar
  // length need no balancing.
  int static_stride;
  // issue-priority threshold in core clocks for waves whose last iteration
  // was slow (0: off); see decode_frame
  uint32_t fair_cycles;
  // frames per queue claim of the one-wave kernel (set by launch_decode,
  // ring_claim): wave w takes frames [w claim, (w + 1) claim), then claims
  // `claim` frames at a time from waves * claim on; a launch then adds
  // claim * ceil(B / claim) to its counter
  int claim;
};

// ---------------------------------------------------------------------------
// The block's window server (ldpc_serve.hip): one persistent launch per
// general_work call serves rounds of windows of the staged span.  The host
// writes a round's keys, then the round word (epoch << 32) | B; results come
// back as 8-byte granules {(epoch mod 2^23) << 9 | syndrome weight, packed
// bytes}.  Epochs only grow; a launch serves epochs above start_epoch.
// ---------------------------------------------------------------------------
// Round word: epoch (bits 32..63), the launch's session (20..31, mod 2^12),
// B (0..19; kServeB: the round that ends the launch).
constexpr uint32_t kServeB = 0xFFFFFu;
constexpr int kServeCopies = 32;  // lines of ctl the poller writes the round to
constexpr size_t kServeCtlBytes = 128 * (kServeCopies + 2);  // + census line, diagnostics line
struct alignas(16) ServeArgs {
  const uint64_t *round;  // host-mapped round word
  const int64_t *keys;    // host-mapped window keys (epoch mod 2^24 << 40) | (position << 1) | polarity
  int64_t *dkeys;         // device: the round's keys, copied by the poller
  uint64_t *res;          // host-mapped result granules
  uint64_t *ctl;          // device, kServeCtlBytes: round copies, census, diagnostics (zeroed per launch)
  uint64_t deadline;      // 100 MHz ticks without a new round before the launch ends
  uint32_t start_epoch;   // the last epoch posted before this launch
  uint32_t session;       // this launch's session id (the host's count of launches)
  int blocks_per_cu;      // decoder workgroups per CU (capped by occupancy; 0: occupancy)
  int debug;              // LDPC_SERVE_DEBUG: counters in ctl words 24..28
  // samples of the staged span (DecodeArgs::in): every key is checked on the
  // device, (key >> 1) + N <= span, before its window is gathered
  int64_t span;
};
// Result granules that carry no decode: the syndrome-weight field (9 bits,
// a real weight is <= M <= 256) says why.  The host turns either into an
// error of the round.
constexpr uint32_t kServeBadKey = 511;   // the key's window is outside the staged span
constexpr uint32_t kServeLostKey = 510;  // the key never showed the round's tag (deadline)
// Epochs stay below this (the host restarts a session before it); a round's
// result tag is epoch mod 2^23.
constexpr uint32_t kServeEpochLimit = (1u << 23) - (1u << 16);
// *workgroups_out: the launch's decoder workgroups
int launch_serve(const CodeView &code, const DecodeArgs &a, const ServeArgs &s, int method,
                 int prec, int slots, int nw, int device, void *stream, int *workgroups_out);

// ---------------------------------------------------------------------------
// The frame ring (ldpc_ring.hip, ldpc_ring_*): ONE persistent launch decodes
// every batch posted to it.  Frames of all posted batches form one queue
// (global tickets: batch q's frame f is ticket start_q + f), so a wave that
// ends a short frame takes the next one whatever batch it belongs to -- no
// SIMD idles at a batch's end waiting for its longest frames.
// The host writes batch q's descriptor into slot q % kRingSlots of mapped
// host memory, `seq` (= q + 1) last; the launch's last wave to finish one of
// the batch's frames writes comp[slot] = q + 1.  Outputs are stored
// write-through (sc1), so a batch's outputs are in memory when its comp word
// is.  A slot is reused only once its batch is complete.
// ---------------------------------------------------------------------------
constexpr int kRingSlots = 256;
struct alignas(64) RingDesc {
  uint64_t seq;          // q + 1 once posted (written last)
  int64_t start;         // ticket of the batch's frame 0
  const float *in;       // frame f at in + f * cw_stride (elem_stride 1, polarity +1)
  int64_t cw_stride;
  uint8_t *packed;       // B x KB
  int32_t *iters;        // B (optional)
  int32_t *synd;         // B (optional)
  int32_t B;             // 0 with quit
  int32_t quit;          // 1: the launch ends at this batch (every later ticket)
};
struct RingArgs {
  const RingDesc *desc;  // host-mapped, kRingSlots
  uint64_t *comp;        // host-mapped, kRingSlots completion words
  uint32_t *done;        // device, frames finished per slot (one 256-byte line each)
  uint32_t *ticket;      // device queue head (zeroed before the launch)
  uint64_t *mirror;      // device copies of the descriptor lines, one set per XCD (zeroed)
  uint64_t *lock;        // device, per XCD and slot: fetch lock {seq, time} (zeroed)
  int64_t ticket0;       // ticket of the launch's first frame
  uint64_t cursor0;      // the launch's first batch (seq - 1)
  uint64_t deadline;     // 100 MHz ticks without a posted batch before a wave leaves
  int max_iters, et_period;
};
// One returning atomic word serves ~88 claims per us (MI355X_MICROARCH.md,
// dequeue): frames shorter than ~12 ns of the chip's time per frame (min-sum,
// f32, the compact mode: ~48 us per 4 096-frame batch whatever the iteration
// cap, tools/ring_probe.py ITERS=1..5) wait on the queue head and on their
// batch's done counter, so those modes claim several frames at a time and
// count them done together.  The exact sum-product (~43 frames per us) claims
// one: a wave holding unstarted frames lengthens the session's tail.
constexpr int kRingMaxClaim = 4;
constexpr int ring_claim(int method, int prec) {
  return method == 1 && (prec == 0 || prec == 2) ? 1 : kRingMaxClaim;
}
constexpr int kRingDoneStride = 64;  // u32 words between two slots' done counters
constexpr int kRingXcds = 8;         // mirror / lock copies: one per XCD (its own L2)
int launch_ring(const CodeView &code, const RingArgs &r, int method, int prec, int slots, int nw,
                int device, void *stream, int *workgroups_out);

// Launch one decode (host side, implemented in ldpc_kernels.hip).
// method: 0 min-sum, 1 sum-product, 2 bit-flip, 3 hard; prec 0 f64, 1 f32;
// slots = ceil(E/64); nw = 1 or 4 (hard-decision words).
// waves_per_cu (0 = default) sets the number of persistent waves;
// schedule: 0 auto, 1 one wave per frame, 2 one multi-wave workgroup per frame.
// *advance_out: what the launch adds to its queue counter (0 with static_stride).
int launch_decode(const CodeView &code, const DecodeArgs &args, int method,
                  int prec, int slots, int nw, int waves_per_cu, int schedule, void *stream,
                  uint32_t *advance_out);

}  // namespace ldpc
