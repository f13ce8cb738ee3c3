// ldpc_capi.hip -- the C ABI of include/ldpc_hip.h (libldpc_hip.so).
//
// Host side of the drop-in boundary: H ingestion (the constructor's matrix
// + reorderHMatrix, lib/ldpc_decoder_cb_impl.cc:60-106), the device edge
// tables, staging buffers and kernel dispatch.  Every decode runs on the GPU;
// when no device is usable ldpc_create fails with LDPC_EDEVICE.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <exception>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ldpc_hip.h"
#include "ldpc_aux.hpp"
#include "ldpc_graph.hpp"
#include "ldpc_kernels.hpp"
#include "ldpc_layout.hpp"

using ldpc::ColRec;
using ldpc::EdgeColRec;
using ldpc::EdgeRowRec;
using ldpc::kNone;

// Host threads that gather a span's samples into pinned memory (copy_span):
// the block's spans are gr_complex, and taking the real parts of 4096 frames
// (2 MB read) on one thread is ~100-180 us in front of the call's first round.
// Pieces are handed out by an atomic counter; the calling thread gathers too
// and sends each piece to the device, in order, once it is ready.
struct GatherPool {
  static constexpr int kThreads = 3;      // helpers (plus the calling thread)
  static constexpr int64_t kPiece = 1 << 14;  // samples per piece gathered
  // samples per copy to the device: a copy costs ~8 us of its own (64 KB
  // copies, one per gathered piece, took 16 x 15.6 us for a 1 MB span,
  // profiles/round5/block_trace.txt)
  static constexpr int64_t kCopy = 1 << 18;
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv;
  uint64_t gen = 0;
  bool quit = false;
  const float *in = nullptr;
  float *h = nullptr;
  int64_t S = 0, npieces = 0;
  int stride = 1;
  std::atomic<int64_t> next{0};
  std::unique_ptr<std::atomic<uint64_t>[]> ready;
  int64_t ready_cap = 0;
  void gather(int64_t p) const {
    const int64_t i0 = p * kPiece, i1 = std::min(S, i0 + kPiece);
    if (stride == 1)
      memcpy(h + i0, in + i0, (size_t)(i1 - i0) * 4);
    else if (stride == 2)  // gr_complex real parts: a constant stride vectorises
      for (int64_t i = i0; i < i1; ++i) h[i] = in[2 * i];
    else
      for (int64_t i = i0; i < i1; ++i) h[i] = in[i * stride];
  }
  void worker() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return quit || gen != seen; });
        if (quit) return;
        seen = gen;
      }
      for (;;) {
        const int64_t p = next.fetch_add(1);
        if (p >= npieces) break;
        gather(p);
        ready[p].store(seen, std::memory_order_release);
      }
    }
  }
  ~GatherPool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      quit = true;
    }
    cv.notify_all();
    for (auto &t : th) t.join();
  }
};

struct ldpc_ctx {
  // LDPC_BLOCK_PROFILE=1: also the host time split of ldpc_decode_windows,
  // printed by ldpc_destroy (span staging, window list + launch, wait, result
  // copy); =2 also a line per call
  bool win_profile = getenv("LDPC_BLOCK_PROFILE") != nullptr;
  bool win_trace = win_profile && getenv("LDPC_BLOCK_PROFILE")[0] == '2';  // a line per call
  double win_prof[5] = {0, 0, 0, 0, 0};
  long long win_calls = 0, win_windows = 0;
  int M = 0, N = 0, E = 0, K = 0, KB = 0, dc_max = 0, dv_max = 0, dc_min = 0;
  int slots = 0, nw = 0, rs = 0;
  int device = 0;
  std::vector<uint8_t> H;  // the decoder's (reordered) H
  hipStream_t stream = nullptr;
  EdgeRowRec *d_erow = nullptr;
  EdgeColRec *d_ecol = nullptr;
  ColRec *d_cols = nullptr;
  uint64_t *d_rowmask = nullptr;
  uint16_t *d_lane_col = nullptr;  // small-code LDS layout (ldpc_layout.hpp)
  uint8_t *d_col_lane = nullptr;
  uint64_t dpos[2] = {0, 0};
  int layout_model[5] = {0, 0, 0, 0, 0};  // searched?, modelled cc / ec, plain cc / ec
  void *d_stage = nullptr;
  size_t stage_bytes = 0;
  float *h_stage = nullptr;  // pinned host staging of host-buffer decodes
  std::unique_ptr<GatherPool> gather;  // copy_span's helpers (made on first use)
  size_t h_stage_bytes = 0;
  bool h_stage_busy = false;  // a copy out of h_stage may still be running (ldpc_stage_span)
  int32_t *h_ctrl = nullptr;  // pinned progress words of the min-sum pipeline
  // ldpc_decode_windows: the staged sample span (device), window list and
  // frames; span_samples > 0 while the staged span may be reused
  void *d_wstage = nullptr;
  size_t wstage_bytes = 0;
  int64_t *h_win = nullptr;
  size_t h_win_bytes = 0;
  int64_t span_samples = 0;
  // the window server (ldpc_serve.hip, ldpc_serve_*): mapped pinned memory
  // [round word | keys | result granules] for srv_cap windows, the device
  // copy of the round word, and the running launch's parameters
  bool serving = false;
  uint8_t *h_srv = nullptr;
  int64_t srv_cap = 0;
  uint64_t *d_srv_ctl = nullptr;
  int64_t *d_srv_keys = nullptr;  // the round's keys as the poller copies them
  uint32_t srv_epoch = 0;  // the last round posted (grows across launches)
  int srv_method = 0, srv_iters = 0, srv_prec = 0;
  int srv_launches = 0, srv_rounds = 0;
  int srv_workgroups = 0;  // decoder workgroups of the running launch
  // LDPC_SERVE_DEBUG: rounds, host us, poller's sight -> publication, ->
  // last key read, -> last result stored (us)
  double dbg[6] = {0, 0, 0, 0, 0, 0};  // ... and the host's sight of the first result
  bool srv_debug = false;  // LDPC_SERVE_DEBUG, read when a launch starts
  bool srv_test_skip_check = false;  // ldpc_test_hook(LDPC_TEST_SERVE_UNCHECKED)
  // the frame ring (ldpc_ring_*, ldpc_ring.hip): mapped host memory
  // [kRingSlots descriptors | kRingSlots completion words], device memory
  // [per-slot frame counters | queue head], the launch's own stream and an
  // event recorded behind the launch (complete = the launch has ended)
  bool ring_on = false;  // a session is open (ldpc_ring_begin .. ldpc_ring_end)
  int ring_method = 0, ring_iters = 0, ring_et = 1, ring_prec = 0;
  uint8_t *h_ring = nullptr;
  uint32_t *d_ring = nullptr;
  hipStream_t ring_stream = nullptr;
  hipEvent_t ring_ev = nullptr, ring_user_ev = nullptr;
  void *ring_user_stream = nullptr;
  uint64_t ring_next = 0;      // the next batch's sequence number (grows across sessions)
  int64_t ring_frames = 0;     // tickets posted so far (the next batch's start)
  uint64_t ring_first = 0;     // the session's first batch
  int64_t ring_first_frame = 0;
  int64_t ring_start[ldpc::kRingSlots] = {};  // start ticket of the batch in each slot
  int ring_launches = 0, ring_workgroups = 0;
  bool ring_clean = false;  // d_ring zeroed for the next launch already
  // in-flight stream set for throughput callers (ldpc_ctx_streams): streams
  // verified to run concurrently, i.e. on distinct hardware queues
  std::vector<hipStream_t> tp_streams;
  uint32_t *d_probe = nullptr;
  // large-code min-sum runs on the narrow-chunk pipeline (ldpc_graph_msn.hip)
  bool narrow = false;  // large code with the min-sum pipeline's tables (M <= kMsnMaxRows)
  ldpc::MsnTables msn;  // storage order of the narrow pipeline
  int32_t *d_msn[4] = {nullptr, nullptr, nullptr, nullptr};  // rx cx corig cpos
  ldpc::MsnDesc *d_msnd[2] = {nullptr, nullptr};                               // rdesc cdesc
  // small-code frame queues: one monotonic counter per stream that has
  // launched on this context (ldpc_kernels.hpp DecodeArgs::ticket)
  uint32_t *d_tickets = nullptr;
  struct Queue {
    void *stream;
    uint32_t base;  // counter value at the start of the next launch
  };
  std::vector<Queue> queues;
  // large-code path: the workspace is shared, so launches on a different
  // stream than the previous one first wait for it (graph_done)
  void *graph_stream = nullptr;
  hipEvent_t graph_done = nullptr;
  int waves_per_cu = 0;           // 0: kernel default
  // launch mode (ldpc_set_launch_mode): issue-priority threshold of the
  // small-code kernel, core clocks (profiles/round1/ab_fair_threshold_warm.txt:
  // 1800 is the best of 1200..3000 for one launch at a time); 0 = off
  uint32_t fair_cycles = 1800;
  int schedule = 0;               // 0 auto, 1 wave per frame, 2 workgroup per frame
  // large-code path (ldpc_graph.hip): H as CSR + CSC, messages in a workspace
  bool graph = false;
  std::vector<int32_t> rp, ci;    // host CSR of the decoder's H
  int32_t *d_rp = nullptr, *d_ci = nullptr, *d_cp = nullptr, *d_ce = nullptr, *d_cr = nullptr;
  void *d_work = nullptr;
  size_t work_bytes = 0;
  size_t work_limit = (size_t)8 << 30;
  // device encoder (built on first ldpc_encode_device): 1 small (A = H_p^-1 H_d
  // bit rows in d_encA), 2 IRA staircase, -1 no systematic encoder
  int enc_kind = 0;
  uint64_t *d_encA = nullptr;
  std::string enc_err;
  std::string err;
};

#define LDPC_TICKET_SLOTS 64
// one counter per 256 bytes: the streams' queues never share a cache line
// (atomics on one line serialise in its L2 channel)
#define LDPC_TICKET_STRIDE 64

namespace {

thread_local std::string g_create_error;

// The reference decoder's H, lib/ldpc_decoder_cb_impl.cc:63-96 (32 x 64),
// one 64-bit word per row, bit c = column c.
const uint64_t kDefaultH[32] = {
    0x0000504000000140ull, 0x0000024080100020ull, 0x0020000141004000ull,
    0x000a008000000220ull, 0x0000080400848000ull, 0x0008000401000090ull,
    0x4100400204000000ull, 0x0010301000000001ull, 0x00024c0000000008ull,
    0x9500006000000000ull, 0x0101200080000400ull, 0x1040000000002004ull,
    0x3080080002000002ull, 0x0200800008010010ull, 0x0410018008040000ull,
    0x0000001200005020ull, 0x0080000040802200ull, 0x0020008010480000ull,
    0x0400001000018088ull, 0x2002020000200004ull, 0x0000000300080300ull,
    0xc200000000240080ull, 0x02000000e4000000ull, 0x0800000000301002ull,
    0x2000040008402040ull, 0x8800010400080000ull, 0x0070000000800000ull,
    0x4040010800000840ull, 0x000c02000000c800ull, 0x0000002811000008ull,
    0x0884000010000401ull, 0x0000900902020000ull,
};

int set_err(ldpc_ctx *ctx, int code, const std::string &msg) {
  if (ctx)
    ctx->err = msg;
  else
    g_create_error = msg;
  return code;
}

int hip_err(ldpc_ctx *ctx, hipError_t e, const char *what) {
  return set_err(ctx, LDPC_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

// reorderHMatrix, lib/ldpc_decoder_cb_impl.cc:255-307 ('First' strategy):
// for each row i pick the first column j >= i with F(i,j) != 0 (column 0 if
// none), swap columns i and j of F and H, and clear column i below row i
// with GF(2) row additions.  lower/upper (M x (N-M), optional) receive the
// factors the encoder solves with (lib/ldpc_encoder_bc_impl.cc:259-260).
void reorder_columns(uint8_t *H, int M, int N, int32_t *chosen,
                     std::vector<uint8_t> *lower, std::vector<uint8_t> *upper) {
  std::vector<uint8_t> F(H, H + (size_t)M * N);
  const int K = N - M;
  if (lower) lower->assign((size_t)M * std::max(K, 0), 0);
  if (upper) upper->assign((size_t)M * std::max(K, 0), 0);
  for (int i = 0; i < M; ++i) {
    int pick = 0;
    for (int j = i; j < N; ++j)
      if (F[(size_t)i * N + j]) {
        pick = j;
        break;
      }
    if (chosen) chosen[i] = pick;
    if (pick != i)
      for (int r = 0; r < M; ++r) {
        std::swap(F[(size_t)r * N + i], F[(size_t)r * N + pick]);
        std::swap(H[(size_t)r * N + i], H[(size_t)r * N + pick]);
      }
    if (i < K) {
      if (lower)
        for (int r = i; r < M; ++r) (*lower)[(size_t)r * K + i] = F[(size_t)r * N + i];
      if (upper)
        for (int r = 0; r <= i; ++r) (*upper)[(size_t)r * K + i] = F[(size_t)r * N + i];
    }
    for (int k = i + 1; k < M; ++k)
      if (F[(size_t)k * N + i])
        for (int c = 0; c < N; ++c) F[(size_t)k * N + c] ^= F[(size_t)i * N + c];
  }
}

bool valid_h(const uint8_t *H, int M, int N) {
  if (!H || M <= 0 || N <= 0 || M >= N) return false;
  for (size_t t = 0; t < (size_t)M * N; ++t)
    if (H[t] > 1) return false;
  return true;
}

// The loop lengths the small-code kernel is built with for this code
// (ldpc_kernels.hip launch_slots), and whether sum-product runs its
// column-centric form (cols_kernel).
void kernel_shape(int nw, int slots, int dc_max, int dv_max, int &dcn, int &dvn, bool &cols) {
  const bool low = nw == 1 && dc_max <= 6 && dv_max <= 3 && slots <= 4;
  dcn = low ? 5 : ldpc::kDcMax - 1;
  dvn = low ? 3 : ldpc::kDvMax;
  cols = nw == 1 && dvn <= slots;
}

// Edge / column / row tables of the decoder's H (see ldpc_kernels.hpp), at
// the cells and positions plan_layout chooses (search false: the plain CSR
// layout, LDPC_FLAG_PLAIN_LAYOUT).
int build_tables(ldpc_ctx *ctx, std::vector<EdgeRowRec> &erecs, std::vector<EdgeColRec> &crecs,
                 std::vector<ColRec> &cols, std::vector<uint64_t> &rowmask,
                 std::vector<uint16_t> &lane_col, std::vector<uint8_t> &col_lane,
                 bool search, std::vector<int> *cell_out = nullptr) {
  const int M = ctx->M, N = ctx->N;
  const uint8_t *H = ctx->H.data();
  std::vector<std::vector<int>> row_edges(M), col_edges(N);
  std::vector<int> erow, ecol;
  for (int j = 0; j < M; ++j)
    for (int i = 0; i < N; ++i)
      if (H[(size_t)j * N + i]) {
        const int e = (int)erow.size();
        erow.push_back(j);
        ecol.push_back(i);
        row_edges[j].push_back(e);
        col_edges[i].push_back(e);  // rows ascend because j ascends
      }
  ctx->E = (int)erow.size();
  ctx->dc_max = 0;
  ctx->dv_max = 0;
  for (auto &r : row_edges) ctx->dc_max = std::max(ctx->dc_max, (int)r.size());
  ctx->dc_min = ctx->dc_max;
  for (auto &r : row_edges) ctx->dc_min = std::min(ctx->dc_min, (int)r.size());
  for (auto &c : col_edges) ctx->dv_max = std::max(ctx->dv_max, (int)c.size());
  if (ctx->E == 0) return set_err(ctx, LDPC_EINVAL, "H has no ones");
  if (N > ldpc::kNMax || M > ldpc::kMMax || ctx->E > 64 * ldpc::kSlotsMax ||
      ctx->dc_max > ldpc::kDcMax || ctx->dv_max > ldpc::kDvMax) {
    char buf[256];
    snprintf(buf, sizeof buf,
             "code shape outside the small-code kernel (M=%d N=%d E=%d dc_max=%d dv_max=%d; "
             "limits M,N<=%d E<=%d dc<=%d dv<=%d)",
             M, N, ctx->E, ctx->dc_max, ctx->dv_max, ldpc::kNMax, 64 * ldpc::kSlotsMax,
             ldpc::kDcMax, ldpc::kDvMax);
    return set_err(ctx, LDPC_EUNSUPPORTED, buf);
  }
  ctx->slots = (ctx->E + 63) / 64;
  ctx->nw = N <= 64 ? 1 : 4;
  ctx->rs = (M + 63) / 64;
  ctx->K = N - M;
  ctx->KB = (ctx->K + 7) / 8;

  int dcn, dvn;
  bool cols_k;
  kernel_shape(ctx->nw, ctx->slots, ctx->dc_max, ctx->dv_max, dcn, dvn, cols_k);
  const ldpc::EdgeLayout lay = ldpc::plan_layout(M, N, erow, ecol, ctx->slots, ctx->nw, dcn, dvn,
                                                 cols_k, search);
  const std::vector<int> &cell = lay.slot, &pos = lay.pos;
  if (cell_out) *cell_out = cell;
  ctx->layout_model[0] = lay.searched ? 1 : 0;
  ctx->layout_model[1] = lay.model_cc;
  ctx->layout_model[2] = lay.model_ec;
  ctx->layout_model[3] = lay.plain_cc;
  ctx->layout_model[4] = lay.plain_ec;
  ctx->dpos[0] = ctx->dpos[1] = 0;
  for (int g = 0; g < 2 * ctx->slots; ++g)
    ctx->dpos[g / 8] |= (uint64_t)(lay.dpos[g] & 31) << (8 * (g % 8));

  erecs.assign((size_t)64 * ctx->slots, EdgeRowRec{});
  crecs.assign((size_t)64 * ctx->slots, EdgeColRec{});
  for (auto &r : erecs) {
    std::fill(std::begin(r.rn), std::end(r.rn), kNone);
    r.col = kNone;
  }
  for (auto &r : crecs) {
    std::fill(std::begin(r.cn), std::end(r.cn), kNone);
    r.col = kNone;
  }
  for (int e = 0; e < ctx->E; ++e) {
    EdgeRowRec &er = erecs[cell[e]];
    EdgeColRec &ec = crecs[cell[e]];
    er.col = ec.col = (uint16_t)pos[ecol[e]];
    int k = 0;
    for (int n : row_edges[erow[e]])
      if (n != e) er.rn[k++] = (uint16_t)cell[n];  // ascending column
    k = 0;
    for (int n : col_edges[ecol[e]])
      if (n != e) ec.cn[k++] = (uint16_t)cell[n];  // ascending row
  }
  cols.assign((size_t)64 * ctx->nw, ColRec{});
  for (auto &c : cols) {
    std::fill(std::begin(c.e), std::end(c.e), kNone);
    std::fill(std::begin(c.r), std::end(c.r), kNone);
  }
  lane_col.assign((size_t)64 * ctx->nw, kNone);
  col_lane.assign((size_t)N, 0);
  for (int i = 0; i < N; ++i) {
    lane_col[pos[i]] = (uint16_t)i;
    col_lane[i] = (uint8_t)pos[i];
    for (size_t k = 0; k < col_edges[i].size(); ++k) {
      cols[pos[i]].e[k] = (uint16_t)cell[col_edges[i][k]];
      cols[pos[i]].r[k] = (uint16_t)erow[col_edges[i][k]];
    }
  }
  rowmask.assign((size_t)M * ctx->nw, 0);
  for (int j = 0; j < M; ++j)
    for (int i = 0; i < N; ++i)
      if (H[(size_t)j * N + i])
        rowmask[(size_t)j * ctx->nw + pos[i] / 64] |= 1ull << (pos[i] % 64);
  return LDPC_OK;
}


// ---- the window server (ldpc_serve_*) --------------------------------------
// Mapped pinned memory: the round word (its own 256 bytes), the keys, the
// result granules.
size_t srv_keys_off() { return 256; }
size_t srv_res_off(int64_t cap) { return 256 + (((size_t)cap * 8 + 255) & ~(size_t)255); }
size_t srv_bytes(int64_t cap) { return srv_res_off(cap) + (size_t)cap * 8; }

// Posts round word (epoch << 32) | B after the keys (x86 stores are ordered;
// the device reads the keys only after it has seen the round word).
// Round word (ldpc_kernels.hpp): (epoch << 32) | (session << 20) | B; the
// session tells a launch still polling after its quit round was overwritten
// that the rounds are no longer its own.
void serve_post(ldpc_ctx *ctx, uint32_t B) {
  ++ctx->srv_epoch;  // < 2^23: ldpc_serve_begin restarts the epochs well before
  __atomic_store_n(reinterpret_cast<uint64_t *>(ctx->h_srv),
                   ((uint64_t)ctx->srv_epoch << 32) | ((uint64_t)(ctx->srv_launches & 0xFFF) << 20) |
                       (B & ldpc::kServeB),
                   __ATOMIC_RELEASE);
}

// Ends a running window server: posts its quit round and waits for the
// launch to finish, so whatever the caller enqueues next does not queue
// behind a launch that polls for rounds.
void serve_stop(ldpc_ctx *ctx) {
  if (!ctx || !ctx->serving) return;
  serve_post(ctx, ldpc::kServeB);
  ctx->serving = false;
  (void)hipStreamSynchronize(ctx->stream);
}

int ensure_stage(ldpc_ctx *ctx, size_t bytes) {
  if (bytes <= ctx->stage_bytes) return LDPC_OK;
  if (ctx->d_stage) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->d_stage);
    ctx->d_stage = nullptr;
    ctx->stage_bytes = 0;
  }
  size_t want = std::max(bytes, (size_t)1 << 20);
  hipError_t e = hipMalloc(&ctx->d_stage, want);
  if (e != hipSuccess) return hip_err(ctx, e, "hipMalloc(staging)");
  ctx->stage_bytes = want;
  return LDPC_OK;
}

int ensure_host_stage(ldpc_ctx *ctx, size_t bytes) {
  if (ctx->h_stage_busy) {  // every writer of h_stage comes through here
    (void)hipStreamSynchronize(ctx->stream);
    ctx->h_stage_busy = false;
  }
  if (bytes <= ctx->h_stage_bytes) return LDPC_OK;
  if (ctx->h_stage) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipHostFree(ctx->h_stage);
    ctx->h_stage = nullptr;
    ctx->h_stage_bytes = 0;
  }
  size_t want = std::max(bytes, (size_t)1 << 20);
  hipError_t e = hipHostMalloc((void **)&ctx->h_stage, want, hipHostMallocDefault);
  if (e != hipSuccess) return hip_err(ctx, e, "hipHostMalloc(staging)");
  ctx->h_stage_bytes = want;
  return LDPC_OK;
}

int check_decode_args(ldpc_ctx *ctx, int &method, int max_iters, int et_period, int precision,
                      int B, int elem_stride, int64_t cw_stride) {
  if (!ctx) return LDPC_EINVAL;
  if (method < 0 || method > 3) method = 0;  // general_work :162-164
  if (B < 0) return set_err(ctx, LDPC_EINVAL, "B < 0");
  if ((method == 0 || method == 1) && max_iters < 1)
    return set_err(ctx, LDPC_EINVAL, "max_iters must be >= 1 for min-sum / sum-product");
  if (method == 2 && max_iters < 0) return set_err(ctx, LDPC_EINVAL, "max_iters < 0");
  if (et_period < 1) return set_err(ctx, LDPC_EINVAL, "et_period must be >= 1");
  if (precision != LDPC_PREC_F64 && precision != LDPC_PREC_F32 &&
      precision != LDPC_PREC_F64_LIBM && precision != LDPC_PREC_F64_FAST)
    return set_err(ctx, LDPC_EINVAL, "precision must be one of LDPC_PREC_*");
  if (elem_stride < 1 || cw_stride < 0) return set_err(ctx, LDPC_EINVAL, "bad strides");
  return LDPC_OK;
}

// CSR of a dense H (edges row-major, ascending column).
void dense_to_csr(const uint8_t *H, int M, int N, std::vector<int32_t> &rp,
                  std::vector<int32_t> &ci) {
  rp.assign((size_t)M + 1, 0);
  ci.clear();
  for (int j = 0; j < M; ++j) {
    for (int i = 0; i < N; ++i)
      if (H[(size_t)j * N + i]) ci.push_back(i);
    rp[j + 1] = (int32_t)ci.size();
  }
}

bool valid_csr(int M, int N, const int32_t *rp, const int32_t *ci) {
  if (!rp || M <= 0 || N <= 0 || M >= N || rp[0] != 0) return false;
  for (int j = 0; j < M; ++j) {
    if (rp[j + 1] < rp[j]) return false;
    for (int32_t e = rp[j]; e < rp[j + 1]; ++e) {
      if (!ci || ci[e] < 0 || ci[e] >= N) return false;
      if (e > rp[j] && ci[e] <= ci[e - 1]) return false;  // ascending, no duplicates
    }
  }
  return true;
}

// Degrees and the CSC permutation of the context's CSR; checks the
// large-code kernels' degree limits.
int build_graph(ldpc_ctx *ctx, std::vector<int32_t> &cp, std::vector<int32_t> &ce,
                std::vector<int32_t> &cr) {
  const int M = ctx->M, N = ctx->N;
  ctx->E = ctx->rp[M];
  if (ctx->E == 0) return set_err(ctx, LDPC_EINVAL, "H has no ones");
  cp.assign((size_t)N + 1, 0);
  for (int e = 0; e < ctx->E; ++e) cp[ctx->ci[e] + 1]++;
  ctx->dc_max = 0;
  ctx->dv_max = 0;
  for (int i = 0; i < N; ++i) ctx->dv_max = std::max(ctx->dv_max, cp[i + 1]);
  for (int j = 0; j < M; ++j) ctx->dc_max = std::max(ctx->dc_max, ctx->rp[j + 1] - ctx->rp[j]);
  for (int i = 0; i < N; ++i) cp[i + 1] += cp[i];
  ce.assign((size_t)ctx->E, 0);
  cr.assign((size_t)ctx->E, 0);
  std::vector<int32_t> fill(cp.begin(), cp.end() - 1);
  for (int j = 0; j < M; ++j)
    for (int32_t e = ctx->rp[j]; e < ctx->rp[j + 1]; ++e) {
      const int32_t k = fill[ctx->ci[e]]++;  // rows ascend because j ascends
      ce[k] = e;
      cr[k] = j;
    }
  if (ctx->dc_max > ldpc::kGraphDcMax || ctx->dv_max > ldpc::kGraphDvMax) {
    char buf[160];
    snprintf(buf, sizeof buf,
             "code degrees outside the large-code kernels (dc_max=%d dv_max=%d; limits %d, %d)",
             ctx->dc_max, ctx->dv_max, ldpc::kGraphDcMax, ldpc::kGraphDvMax);
    return set_err(ctx, LDPC_EUNSUPPORTED, buf);
  }
  ctx->K = N - M;
  ctx->KB = (ctx->K + 7) / 8;
  ctx->graph = true;
  return LDPC_OK;
}

ldpc::GraphView graph_view(const ldpc_ctx *ctx) {
  ldpc::GraphView g;
  g.rp = ctx->d_rp;
  g.ci = ctx->d_ci;
  g.cp = ctx->d_cp;
  g.ce = ctx->d_ce;
  g.cr = ctx->d_cr;
  g.M = ctx->M;
  g.N = ctx->N;
  g.E = ctx->E;
  g.KB = ctx->KB;
  g.dc_max = ctx->dc_max;
  g.dv_max = ctx->dv_max;
  return g;
}

ldpc::CodeView code_view(const ldpc_ctx *ctx) {
  ldpc::CodeView v;
  v.erow = ctx->d_erow;
  v.ecol = ctx->d_ecol;
  v.cols = ctx->d_cols;
  v.rowmask = ctx->d_rowmask;
  v.lane_col = ctx->d_lane_col;
  v.col_lane = ctx->d_col_lane;
  v.dpos[0] = ctx->dpos[0];
  v.dpos[1] = ctx->dpos[1];
  v.M = ctx->M;
  v.N = ctx->N;
  v.E = ctx->E;
  v.KB = ctx->KB;
  v.rs = ctx->rs;
  v.dc_max = ctx->dc_max;
  v.dv_max = ctx->dv_max;
  v.dc_min = ctx->dc_min;
  return v;
}

// Large-code path: frames in groups that fit the workspace limit, each group
// decoded by launch_graph_decode on `st`.
int decode_graph(ldpc_ctx *ctx, const ldpc::DecodeArgs &a, int method, int precision, void *st) {
  const ldpc::GraphView g = graph_view(ctx);
  const bool want_post = a.llr != nullptr;
  if (method == 0) {
    // min-sum: narrow chunks, gathered state L2-resident per XCD
    if (!ctx->narrow)
      return set_err(ctx, LDPC_EUNSUPPORTED,
                     "large-code min-sum needs M <= " + std::to_string(ldpc::kMsnMaxRows) +
                         " check rows (the narrow-chunk pipeline's limit)");
    ldpc::MsnView v;
    v.rx = ctx->d_msn[0];
    v.cx = ctx->d_msn[1];
    v.rdesc = ctx->d_msnd[0];
    v.cdesc = ctx->d_msnd[1];
    v.rs = ctx->msn.rs;
    v.cs = ctx->msn.cs;
    v.corig = ctx->d_msn[2];
    v.cpos = ctx->d_msn[3];
    v.M = g.M;
    v.N = g.N;
    v.E = g.E;
    v.KB = g.KB;
    v.dc_max = g.dc_max;
    v.dv_max = g.dv_max;
    v.out_var = ctx->msn.out_var ? 1 : 0;
    int C = ldpc::msn_default_chunks();
    const int need_c = (a.B + ldpc::kMsnFrames - 1) / ldpc::kMsnFrames;
    if (need_c < C) C = need_c >= 8 ? (need_c + 7) / 8 * 8 : need_c;
    // ldpc_set_work_limit caps the chunks in flight (at least one; multiples
    // of 8 keep the XCD placement)
    while (C > 1 && ldpc::msn_work_bytes(v, C, precision) > ctx->work_limit)
      C = C > 8 && C % 8 == 0 ? C - 8 : C - 1;
    const size_t need = ldpc::msn_work_bytes(v, C, precision);
    if (need > ctx->work_bytes) {
      if (ctx->d_work) {
        (void)hipDeviceSynchronize();
        (void)hipFree(ctx->d_work);
        ctx->d_work = nullptr;
        ctx->work_bytes = 0;
      }
      hipError_t e = hipMalloc(&ctx->d_work, need);
      if (e != hipSuccess) return hip_err(ctx, e, "hipMalloc(graph workspace)");
      ctx->work_bytes = need;
    }
    if (!ctx->h_ctrl) {
      hipError_t e = hipHostMalloc((void **)&ctx->h_ctrl, 64, hipHostMallocDefault);
      if (e != hipSuccess) return hip_err(ctx, e, "hipHostMalloc(ctrl)");
    }
    ldpc::MsnWork w;
    ldpc::msn_work_carve(w, ctx->d_work, v, C, precision);
    const int rc = ldpc::launch_graph_decode_msn(v, w, a, precision, ctx->h_ctrl, st);
    if (rc == -2) return set_err(ctx, LDPC_EUNSUPPORTED, "code degrees outside the large-code kernels");
    if (rc != 0) return hip_err(ctx, hipGetLastError(), "graph kernel launch");
    return LDPC_OK;
  }
  const size_t per64 = ldpc::graph_work_bytes(g, 64, precision, method, want_post);
  int group = (int)std::min<size_t>((size_t)1 << 30, std::max<size_t>(1, ctx->work_limit / per64) * 64);
  group = std::min(group, (a.B + 63) / 64 * 64);
  const size_t need = ldpc::graph_work_bytes(g, group, precision, method, want_post);
  if (need > ctx->work_bytes) {
    if (ctx->d_work) {
      (void)hipDeviceSynchronize();  // the old workspace may be in use on any stream
      (void)hipFree(ctx->d_work);
      ctx->d_work = nullptr;
      ctx->work_bytes = 0;
    }
    hipError_t e = hipMalloc(&ctx->d_work, need);
    if (e != hipSuccess) return hip_err(ctx, e, "hipMalloc(graph workspace)");
    ctx->work_bytes = need;
  }
  for (int b0 = 0; b0 < a.B; b0 += group) {
    const int nb = std::min(group, a.B - b0);
    ldpc::GraphWork w;
    ldpc::graph_work_carve(w, ctx->d_work, g, (nb + 63) / 64 * 64, precision, method, want_post);
    ldpc::DecodeArgs s = a;
    s.in = a.in + (int64_t)b0 * a.cw_stride;
    s.B = nb;
    s.packed = a.packed + (int64_t)b0 * ctx->KB;
    if (a.bits) s.bits = a.bits + (int64_t)b0 * ctx->N;
    if (a.iters) s.iters = a.iters + b0;
    if (a.synd) s.synd = a.synd + b0;
    if (a.llr) s.llr = a.llr + (int64_t)b0 * ctx->N;
    const int rc = ldpc::launch_graph_decode(g, w, s, method, precision, st);
    if (rc == -2) return set_err(ctx, LDPC_EUNSUPPORTED, "code degrees outside the large-code kernels");
    if (rc != 0) return hip_err(ctx, hipGetLastError(), "graph kernel launch");
  }
  return LDPC_OK;
}

// Systematic encoder of the context's H (codeword = [parity (M) | data (K)]):
// small codes get A = H_p^-1 H_d by Gauss-Jordan over GF(2) (unique when the
// first M columns are independent, which reorderHMatrix ensures); large codes
// must have the accumulator staircase in columns 0..M-1 (IRA / DVB-S2).
int prepare_encoder(ldpc_ctx *ctx) {
  if (ctx->enc_kind > 0) return LDPC_OK;
  if (ctx->enc_kind < 0) return set_err(ctx, LDPC_EUNSUPPORTED, ctx->enc_err);
  const int M = ctx->M, N = ctx->N, K = N - M;
  if (!ctx->H.empty() && K <= 256) {
    const int W = (N + 63) / 64;
    std::vector<uint64_t> rows((size_t)M * W, 0);
    for (int j = 0; j < M; ++j)
      for (int i = 0; i < N; ++i)
        if (ctx->H[(size_t)j * N + i]) rows[(size_t)j * W + i / 64] |= 1ull << (i % 64);
    for (int c = 0; c < M; ++c) {
      int piv = -1;
      for (int r = c; r < M; ++r)
        if ((rows[(size_t)r * W + c / 64] >> (c % 64)) & 1) {
          piv = r;
          break;
        }
      if (piv < 0) {
        ctx->enc_kind = -1;
        ctx->enc_err = "the first M columns of H are dependent: no systematic encoder";
        return set_err(ctx, LDPC_EUNSUPPORTED, ctx->enc_err);
      }
      if (piv != c)
        for (int w = 0; w < W; ++w) std::swap(rows[(size_t)piv * W + w], rows[(size_t)c * W + w]);
      for (int r = 0; r < M; ++r)
        if (r != c && ((rows[(size_t)r * W + c / 64] >> (c % 64)) & 1))
          for (int w = 0; w < W; ++w) rows[(size_t)r * W + w] ^= rows[(size_t)c * W + w];
    }
    const int KW = (K + 63) / 64;
    std::vector<uint64_t> A((size_t)M * KW, 0);
    for (int j = 0; j < M; ++j)
      for (int i = 0; i < K; ++i)
        if ((rows[(size_t)j * W + (M + i) / 64] >> ((M + i) % 64)) & 1)
          A[(size_t)j * KW + i / 64] |= 1ull << (i % 64);
    hipError_t e = hipMalloc(&ctx->d_encA, A.size() * 8);
    if (e == hipSuccess) e = hipMemcpy(ctx->d_encA, A.data(), A.size() * 8, hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_err(ctx, e, "encoder upload");
    ctx->enc_kind = 1;
    return LDPC_OK;
  }
  for (int j = 0; j < M; ++j) {
    int want[2] = {j - 1, j}, n = 0;
    bool ok = true;
    for (int32_t e = ctx->rp[j]; e < ctx->rp[j + 1] && ctx->ci[e] < M; ++e) {
      const int c = ctx->ci[e];
      if (n >= 2 || (j == 0 ? c != 0 : c != want[n])) ok = false;
      ++n;
    }
    if (!ok || n != (j == 0 ? 1 : 2)) {
      ctx->enc_kind = -1;
      ctx->enc_err =
          "large code without the accumulator staircase in columns 0..M-1: no device encoder";
      return set_err(ctx, LDPC_EUNSUPPORTED, ctx->enc_err);
    }
  }
  ctx->enc_kind = 2;
  return LDPC_OK;
}

}  // namespace

extern "C" {

int ldpc_default_h(uint8_t *H_out) {
  if (!H_out) return LDPC_EINVAL;
  for (int j = 0; j < 32; ++j)
    for (int i = 0; i < 64; ++i) H_out[j * 64 + i] = (uint8_t)((kDefaultH[j] >> i) & 1);
  return LDPC_OK;
}

// MacKay's alist format: "N M", "max_col_deg max_row_deg", the N column
// degrees, the M row degrees, then per column its rows and per row its
// columns (1-based), each list zero-padded to the maximum degree or not
// padded at all (both forms are in use).  The row lists must agree with the
// column lists.
int ldpc_alist_read(const char *path, int *M_out, int *N_out, int32_t *row_ptr_opt,
                    int32_t *col_idx_opt, int64_t col_idx_cap) {
  if (!path || !M_out || !N_out) return set_err(nullptr, LDPC_EINVAL, "null argument");
  FILE *f = fopen(path, "r");
  if (!f) return set_err(nullptr, LDPC_EINVAL, std::string("cannot open ") + path);
  std::vector<long> v;
  long x;
  while (fscanf(f, "%ld", &x) == 1) v.push_back(x);
  const bool clean_eof = feof(f) != 0;
  fclose(f);
  if (!clean_eof) return set_err(nullptr, LDPC_EINVAL, "alist: non-numeric content");
  if (v.size() < 4) return set_err(nullptr, LDPC_EINVAL, "alist: truncated header");
  const long N = v[0], M = v[1], dvm = v[2], dcm = v[3];
  if (N <= 0 || M <= 0 || M >= N || N > (1L << 24) || dvm <= 0 || dcm <= 0 ||
      v.size() < (size_t)(4 + N + M))
    return set_err(nullptr, LDPC_EINVAL, "alist: bad header (need 0 < M < N)");
  long sum_c = 0, sum_r = 0;
  for (long i = 0; i < N; ++i) {
    const long d = v[4 + i];
    if (d < 0 || d > dvm) return set_err(nullptr, LDPC_EINVAL, "alist: bad column degree");
    sum_c += d;
  }
  for (long j = 0; j < M; ++j) {
    const long d = v[4 + N + j];
    if (d < 0 || d > dcm) return set_err(nullptr, LDPC_EINVAL, "alist: bad row degree");
    sum_r += d;
  }
  if (sum_c != sum_r) return set_err(nullptr, LDPC_EINVAL, "alist: degree sums differ");
  const size_t head = 4 + N + M;
  bool padded;
  if (v.size() == head + (size_t)(N * dvm + M * dcm))
    padded = true;
  else if (v.size() == head + (size_t)(sum_c + sum_r))
    padded = false;
  else
    return set_err(nullptr, LDPC_EINVAL, "alist: list length matches neither padded nor unpadded");
  // column lists -> (row, col) pairs; row lists checked against them
  std::vector<std::vector<int32_t>> rows(M);
  size_t at = head;
  for (long i = 0; i < N; ++i) {
    const long d = v[4 + i], width = padded ? dvm : d;
    for (long k = 0; k < width; ++k) {
      const long r = v[at++];
      if (k >= d) {
        if (r != 0) return set_err(nullptr, LDPC_EINVAL, "alist: non-zero padding");
        continue;
      }
      if (r < 1 || r > M) return set_err(nullptr, LDPC_EINVAL, "alist: row index out of range");
      rows[r - 1].push_back((int32_t)i);
    }
  }
  int64_t E = 0;
  for (long j = 0; j < M; ++j) {
    std::vector<int32_t> &c = rows[j];
    std::sort(c.begin(), c.end());
    if (std::adjacent_find(c.begin(), c.end()) != c.end())
      return set_err(nullptr, LDPC_EINVAL, "alist: repeated entry");
    const long d = v[4 + N + j], width = padded ? dcm : d;
    if ((long)c.size() != d) return set_err(nullptr, LDPC_EINVAL, "alist: row degree mismatch");
    std::vector<int32_t> listed;
    for (long k = 0; k < width; ++k) {
      const long cc = v[at++];
      if (k >= d) {
        if (cc != 0) return set_err(nullptr, LDPC_EINVAL, "alist: non-zero padding");
        continue;
      }
      if (cc < 1 || cc > N) return set_err(nullptr, LDPC_EINVAL, "alist: column index out of range");
      listed.push_back((int32_t)(cc - 1));
    }
    std::sort(listed.begin(), listed.end());
    if (listed != c) return set_err(nullptr, LDPC_EINVAL, "alist: row and column lists disagree");
    E += d;
  }
  *M_out = (int)M;
  *N_out = (int)N;
  if (row_ptr_opt) {
    row_ptr_opt[0] = 0;
    for (long j = 0; j < M; ++j) row_ptr_opt[j + 1] = row_ptr_opt[j] + (int32_t)rows[j].size();
  }
  if (col_idx_opt) {
    if (col_idx_cap < E) return set_err(nullptr, LDPC_EINVAL, "alist: col_idx buffer too small");
    int64_t o = 0;
    for (long j = 0; j < M; ++j)
      for (int32_t c : rows[j]) col_idx_opt[o++] = c;
  }
  return (int)E;
}

int ldpc_reorder_h(uint8_t *H, int M, int N, int32_t *chosen_opt) {
  if (!valid_h(H, M, N)) return LDPC_EINVAL;
  reorder_columns(H, M, N, chosen_opt, nullptr, nullptr);
  return LDPC_OK;
}

int ldpc_check_frame(const uint8_t *H, int M, int N, const uint8_t *bits, int threshold) {
  if (!valid_h(H, M, N) || !bits) return LDPC_EINVAL;
  int unsatisfied = 0;
  for (int k = 0; k < M; ++k) {
    int parity = 0;
    for (int j = 0; j < N; ++j) parity ^= (H[(size_t)k * N + j] & (bits[j] & 1));
    if (parity) ++unsatisfied;
    if (unsatisfied > threshold) break;
  }
  return unsatisfied;
}

// makeParityCheck (lib/ldpc_encoder_bc_impl.cc:275-294) over GF(2): the
// reference's two real-valued dgesv solves on the unit-triangular 0/1
// factors are exact integer substitutions, which reduce mod 2 to the
// substitutions below.  The factors come from re-running the reorder on the
// (already reordered) H, which then moves no column.
int ldpc_encode(const uint8_t *Hr, int M, int N, const uint8_t *data_bits, int B,
                uint8_t *codewords_out) {
  if (!valid_h(Hr, M, N) || N != 2 * M || B < 0 || (B > 0 && (!data_bits || !codewords_out)))
    return LDPC_EINVAL;
  std::vector<uint8_t> H(Hr, Hr + (size_t)M * N), L, U;
  std::vector<int32_t> chosen(M);
  reorder_columns(H.data(), M, N, chosen.data(), &L, &U);
  for (int i = 0; i < M; ++i)
    if (chosen[i] != i) return LDPC_EINVAL;  // not the reordered form
  const int K = N - M;
  for (int i = 0; i < M; ++i)
    if (!L[(size_t)i * K + i] || !U[(size_t)i * K + i]) return LDPC_ESINGULAR;
  std::vector<uint8_t> z(M), x(M);
  for (int b = 0; b < B; ++b) {
    const uint8_t *d = data_bits + (size_t)b * K;
    uint8_t *cw = codewords_out + (size_t)b * N;
    for (int i = 0; i < M; ++i) {
      int acc = 0;
      for (int j = 0; j < K; ++j) acc ^= Hr[(size_t)i * N + M + j] & (d[j] & 1);
      z[i] = (uint8_t)acc;
    }
    for (int i = 0; i < M; ++i) {  // L x = z
      int acc = z[i];
      for (int j = 0; j < i; ++j) acc ^= L[(size_t)i * K + j] & x[j];
      x[i] = (uint8_t)acc;
    }
    for (int i = M - 1; i >= 0; --i) {  // U c = x
      int acc = x[i];
      for (int j = i + 1; j < M; ++j) acc ^= U[(size_t)i * K + j] & cw[j];
      cw[i] = (uint8_t)acc;
    }
    for (int j = 0; j < K; ++j) cw[M + j] = d[j] & 1;
  }
  return LDPC_OK;
}

}  // extern "C"

namespace {

template <typename T>
bool upload(ldpc_ctx *ctx, T **dst, const std::vector<T> &src, const char *what,
            const char *&failed, hipError_t &e) {
  if (failed) return false;
  if ((e = hipMalloc((void **)dst, std::max<size_t>(src.size(), 1) * sizeof(T))) != hipSuccess ||
      (!src.empty() &&
       (e = hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice)) !=
           hipSuccess)) {
    failed = what;
    return false;
  }
  return true;
}

// Device setup shared by ldpc_create / ldpc_create_csr: the context's H is
// in ctx->rp / ctx->ci (and ctx->H for small codes).  Picks the small-code
// kernel when the code fits it (unless LDPC_FLAG_GRAPH), else the large-code
// path.  Consumes ctx on failure.
ldpc_ctx *finish_create(ldpc_ctx *ctx, int flags, int device) {
  std::vector<EdgeRowRec> erecs;
  std::vector<EdgeColRec> crecs;
  std::vector<ColRec> cols;
  std::vector<uint64_t> rowmask;
  std::vector<uint16_t> lane_col;
  std::vector<uint8_t> col_lane;
  std::vector<int32_t> cp, ce, cr;
  int rc = LDPC_EUNSUPPORTED;
  if (!(flags & LDPC_FLAG_GRAPH) && !ctx->H.empty())
    rc = build_tables(ctx, erecs, crecs, cols, rowmask, lane_col, col_lane,
                      !(flags & LDPC_FLAG_PLAIN_LAYOUT));
  if (rc == LDPC_EUNSUPPORTED) {
    ctx->err.clear();
    rc = build_graph(ctx, cp, ce, cr);
  }
  if (rc != LDPC_OK) {
    g_create_error = ctx->err;
    delete ctx;
    return nullptr;
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0 || device < 0 || device >= ndev) {
    g_create_error = std::string("no usable HIP device (") +
                     (e != hipSuccess ? hipGetErrorString(e) : "device index out of range") +
                     "); the decode path has no CPU fallback";
    delete ctx;
    return nullptr;
  }
  ctx->device = device;
  {  // large-code min-sum: the narrow-chunk pipeline's tables
    ctx->narrow = ctx->graph && ctx->M <= ldpc::kMsnMaxRows;
    if (ctx->narrow) {
      try {
        ldpc::msn_build(ctx->M, ctx->N, ctx->rp, ctx->ci, ctx->msn);
      } catch (const std::exception &ex) {
        g_create_error = ex.what();
        delete ctx;
        return nullptr;
      }
    }
  }
  const char *what = nullptr;
  if ((e = hipSetDevice(device)) != hipSuccess) what = "hipSetDevice";
  if (!what && (e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) != hipSuccess)
    what = "hipStreamCreate";
  if (ctx->graph) {
    upload(ctx, &ctx->d_rp, ctx->rp, "upload(row_ptr)", what, e);
    upload(ctx, &ctx->d_ci, ctx->ci, "upload(col_idx)", what, e);
    upload(ctx, &ctx->d_cp, cp, "upload(col_ptr)", what, e);
    upload(ctx, &ctx->d_ce, ce, "upload(col_edges)", what, e);
    upload(ctx, &ctx->d_cr, cr, "upload(col_rows)", what, e);
    if (ctx->narrow) {
      const std::vector<int32_t> *t[4] = {&ctx->msn.rx, &ctx->msn.cx, &ctx->msn.corig,
                                          &ctx->msn.cpos};
      for (int i = 0; i < 4; ++i) upload(ctx, &ctx->d_msn[i], *t[i], "upload(storage order)", what, e);
      upload(ctx, &ctx->d_msnd[0], ctx->msn.rdesc, "upload(edge descriptors)", what, e);
      upload(ctx, &ctx->d_msnd[1], ctx->msn.cdesc, "upload(edge descriptors)", what, e);
    }
  } else {
    upload(ctx, &ctx->d_erow, erecs, "upload(erow)", what, e);
    upload(ctx, &ctx->d_ecol, crecs, "upload(ecol)", what, e);
    upload(ctx, &ctx->d_cols, cols, "upload(cols)", what, e);
    upload(ctx, &ctx->d_rowmask, rowmask, "upload(rowmask)", what, e);
    upload(ctx, &ctx->d_lane_col, lane_col, "upload(lane_col)", what, e);
    upload(ctx, &ctx->d_col_lane, col_lane, "upload(col_lane)", what, e);
    std::vector<uint32_t> zeros((size_t)LDPC_TICKET_SLOTS * LDPC_TICKET_STRIDE, 0);
    upload(ctx, &ctx->d_tickets, zeros, "upload(tickets)", what, e);
  }
  if (what) {
    g_create_error = std::string(what) + ": " + hipGetErrorString(e);
    ldpc_destroy(ctx);
    return nullptr;
  }
  return ctx;
}

}  // namespace

extern "C" {

ldpc_ctx *ldpc_create(const uint8_t *H, int M, int N, int flags, int device) {
  g_create_error.clear();
  if (!valid_h(H, M, N)) {
    set_err(nullptr, LDPC_EINVAL, "H must be M x N (M < N) with 0/1 entries");
    return nullptr;
  }
  ldpc_ctx *ctx = new ldpc_ctx();
  ctx->M = M;
  ctx->N = N;
  ctx->H.assign(H, H + (size_t)M * N);
  if (!(flags & LDPC_FLAG_NO_REORDER)) reorder_columns(ctx->H.data(), M, N, nullptr, nullptr, nullptr);
  dense_to_csr(ctx->H.data(), M, N, ctx->rp, ctx->ci);
  return finish_create(ctx, flags, device);
}

ldpc_ctx *ldpc_create_csr(int M, int N, const int32_t *row_ptr, const int32_t *col_idx,
                          int flags, int device) {
  g_create_error.clear();
  if (!valid_csr(M, N, row_ptr, col_idx)) {
    set_err(nullptr, LDPC_EINVAL,
            "CSR H must be M x N (M < N), row_ptr[0] == 0, non-decreasing, columns ascending "
            "and in range");
    return nullptr;
  }
  ldpc_ctx *ctx = new ldpc_ctx();
  ctx->M = M;
  ctx->N = N;
  ctx->rp.assign(row_ptr, row_ptr + M + 1);
  ctx->ci.assign(col_idx, col_idx + row_ptr[M]);
  if (N <= ldpc::kNMax && M <= ldpc::kMMax) {  // small enough for the register kernel
    ctx->H.assign((size_t)M * N, 0);
    for (int j = 0; j < M; ++j)
      for (int32_t e = row_ptr[j]; e < row_ptr[j + 1]; ++e) ctx->H[(size_t)j * N + col_idx[e]] = 1;
  }
  return finish_create(ctx, flags, device);
}

void ldpc_destroy(ldpc_ctx *ctx) {
  if (!ctx) return;
  serve_stop(ctx);
  if (ctx->ring_on) (void)ldpc_ring_end(ctx);
  if (ctx->ring_stream) {
    (void)hipStreamSynchronize(ctx->ring_stream);
    (void)hipStreamDestroy(ctx->ring_stream);
  }
  if (ctx->ring_ev) (void)hipEventDestroy(ctx->ring_ev);
  if (ctx->ring_user_ev) (void)hipEventDestroy(ctx->ring_user_ev);
  if (ctx->h_ring) (void)hipHostFree(ctx->h_ring);
  if (ctx->d_ring) (void)hipFree(ctx->d_ring);
  if (ctx->win_profile && ctx->win_calls)
    fprintf(stderr,
            "ldpc_decode_windows profile: %lld calls, %lld windows; staging %.3f ms, window list + "
            "launch %.3f ms, wait %.3f ms, results %.3f ms\n",
            ctx->win_calls, ctx->win_windows, 1e3 * ctx->win_prof[0], 1e3 * ctx->win_prof[1],
            1e3 * ctx->win_prof[2], 1e3 * ctx->win_prof[3]);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->d_erow) (void)hipFree(ctx->d_erow);
  if (ctx->d_ecol) (void)hipFree(ctx->d_ecol);
  if (ctx->d_cols) (void)hipFree(ctx->d_cols);
  if (ctx->d_rowmask) (void)hipFree(ctx->d_rowmask);
  if (ctx->d_lane_col) (void)hipFree(ctx->d_lane_col);
  if (ctx->d_col_lane) (void)hipFree(ctx->d_col_lane);
  if (ctx->d_stage) (void)hipFree(ctx->d_stage);
  if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
  if (ctx->h_ctrl) (void)hipHostFree(ctx->h_ctrl);
  if (ctx->d_wstage) (void)hipFree(ctx->d_wstage);
  if (ctx->h_win) (void)hipHostFree(ctx->h_win);
  if (ctx->h_srv) (void)hipHostFree(ctx->h_srv);
  for (hipStream_t t : ctx->tp_streams) {
    (void)hipStreamSynchronize(t);
    (void)hipStreamDestroy(t);
  }
  if (ctx->d_probe) (void)hipFree(ctx->d_probe);
  if (ctx->d_srv_ctl) (void)hipFree(ctx->d_srv_ctl);
  if (ctx->d_srv_keys) (void)hipFree(ctx->d_srv_keys);
  if (ctx->d_tickets) (void)hipFree(ctx->d_tickets);
  for (int32_t *p : {ctx->d_rp, ctx->d_ci, ctx->d_cp, ctx->d_ce, ctx->d_cr})
    if (p) (void)hipFree(p);
  for (int32_t *p : ctx->d_msn)
    if (p) (void)hipFree(p);
  for (ldpc::MsnDesc *p : ctx->d_msnd)
    if (p) (void)hipFree(p);
  if (ctx->d_work) {
    (void)hipDeviceSynchronize();  // graph decodes may run on caller streams
    (void)hipFree(ctx->d_work);
  }
  if (ctx->graph_done) (void)hipEventDestroy(ctx->graph_done);
  if (ctx->d_encA) (void)hipFree(ctx->d_encA);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char *ldpc_last_error(const ldpc_ctx *ctx) {
  return ctx ? ctx->err.c_str() : g_create_error.c_str();
}

int ldpc_ctx_info(const ldpc_ctx *ctx, int *M, int *N, int *E, int *K, int *KB, int *dc_max,
                  int *dv_max) {
  if (!ctx) return LDPC_EINVAL;
  if (M) *M = ctx->M;
  if (N) *N = ctx->N;
  if (E) *E = ctx->E;
  if (K) *K = ctx->K;
  if (KB) *KB = ctx->KB;
  if (dc_max) *dc_max = ctx->dc_max;
  if (dv_max) *dv_max = ctx->dv_max;
  return LDPC_OK;
}

int ldpc_ctx_h(const ldpc_ctx *ctx, uint8_t *H_out) {
  if (!ctx || !H_out) return LDPC_EINVAL;
  memset(H_out, 0, (size_t)ctx->M * ctx->N);
  for (int j = 0; j < ctx->M; ++j)
    for (int32_t e = ctx->rp[j]; e < ctx->rp[j + 1]; ++e) H_out[(size_t)j * ctx->N + ctx->ci[e]] = 1;
  return LDPC_OK;
}

int ldpc_ctx_csr(const ldpc_ctx *ctx, int32_t *row_ptr_out, int32_t *col_idx_out) {
  if (!ctx) return LDPC_EINVAL;
  if (row_ptr_out) memcpy(row_ptr_out, ctx->rp.data(), ctx->rp.size() * sizeof(int32_t));
  if (col_idx_out) memcpy(col_idx_out, ctx->ci.data(), ctx->ci.size() * sizeof(int32_t));
  return LDPC_OK;
}

int ldpc_ctx_path(const ldpc_ctx *ctx) {
  if (!ctx) return LDPC_EINVAL;
  return ctx->graph ? 1 : 0;
}

int ldpc_ctx_pipeline(const ldpc_ctx *ctx, int *frames_per_chunk, int *chunks) {
  if (!ctx) return LDPC_EINVAL;
  const bool narrow = ctx->narrow;
  if (frames_per_chunk) *frames_per_chunk = narrow ? ldpc::kMsnFrames : 0;
  if (chunks) *chunks = narrow ? ldpc::msn_default_chunks() : 0;
  return narrow ? 1 : 0;
}

int ldpc_ctx_layout(const ldpc_ctx *ctx, int32_t *model_out) {
  if (!ctx || !model_out) return LDPC_EINVAL;
  if (ctx->graph) return LDPC_EUNSUPPORTED;
  std::copy(ctx->layout_model, ctx->layout_model + 5, model_out);
  return LDPC_OK;
}

int ldpc_plan_storage_order(int M, int N, const int32_t *row_ptr, const int32_t *col_idx,
                            int32_t *rpos_out_opt, int32_t *cpos_out_opt, int64_t *score_out_opt) {
  g_create_error.clear();
  if (!valid_csr(M, N, row_ptr, col_idx))
    return set_err(nullptr, LDPC_EINVAL, "CSR H must be M x N (M < N), columns ascending and in range");
  try {
    std::vector<int32_t> rp(row_ptr, row_ptr + M + 1), ci(col_idx, col_idx + row_ptr[M]);
    ldpc::MsnTables t;
    ldpc::msn_build(M, N, rp, ci, t);
    if (rpos_out_opt) std::copy(t.rpos.begin(), t.rpos.end(), rpos_out_opt);
    if (cpos_out_opt) std::copy(t.cpos.begin(), t.cpos.end(), cpos_out_opt);
    if (score_out_opt) {
      score_out_opt[0] = t.score[0];
      score_out_opt[1] = t.score[1];
    }
    return t.order;
  } catch (const std::exception &e) {
    return set_err(nullptr, LDPC_ENOMEM, e.what());
  }
}

int ldpc_plan_layout(const uint8_t *H, int M, int N, int flags, int32_t *cell_out_opt,
                     int32_t *pos_out_opt, int32_t *model_out_opt) {
  g_create_error.clear();
  if (!valid_h(H, M, N)) return set_err(nullptr, LDPC_EINVAL, "H must be M x N (M < N) with 0/1 entries");
  ldpc_ctx tmp;
  tmp.M = M;
  tmp.N = N;
  tmp.H.assign(H, H + (size_t)M * N);
  if (!(flags & LDPC_FLAG_NO_REORDER)) reorder_columns(tmp.H.data(), M, N, nullptr, nullptr, nullptr);
  std::vector<EdgeRowRec> erecs;
  std::vector<EdgeColRec> crecs;
  std::vector<ColRec> cols;
  std::vector<uint64_t> rowmask;
  std::vector<uint16_t> lane_col;
  std::vector<uint8_t> col_lane;
  std::vector<int> cell;
  const int rc = build_tables(&tmp, erecs, crecs, cols, rowmask, lane_col, col_lane,
                              !(flags & LDPC_FLAG_PLAIN_LAYOUT), &cell);
  if (rc != LDPC_OK) return set_err(nullptr, rc, tmp.err);
  if (cell_out_opt) std::copy(cell.begin(), cell.end(), cell_out_opt);
  if (pos_out_opt)
    for (int i = 0; i < N; ++i) pos_out_opt[i] = col_lane[i];
  if (model_out_opt) std::copy(tmp.layout_model, tmp.layout_model + 5, model_out_opt);
  return tmp.E;
}

int ldpc_encode_device(ldpc_ctx *ctx, const uint8_t *d_data_bits, int B, uint8_t *d_codewords,
                       void *hip_stream) {
  serve_stop(ctx);
  if (!ctx) return LDPC_EINVAL;
  if (B < 0 || (B > 0 && (!d_data_bits || !d_codewords)))
    return set_err(ctx, LDPC_EINVAL, "bad encoder arguments");
  if (B == 0) return LDPC_OK;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  int rc = prepare_encoder(ctx);
  if (rc != LDPC_OK) return rc;
  void *st = hip_stream ? hip_stream : (void *)ctx->stream;
  const int K = ctx->N - ctx->M;
  if (ctx->enc_kind == 1)
    rc = ldpc::launch_encode_small(ctx->d_encA, ctx->M, K, d_data_bits, B, d_codewords, st);
  else
    rc = ldpc::launch_encode_ira(ctx->d_rp ? ctx->d_rp : nullptr, ctx->d_ci, ctx->M, K,
                                 d_data_bits, B, d_codewords, st);
  return rc == 0 ? LDPC_OK : hip_err(ctx, hipGetLastError(), "encoder launch");
}

int ldpc_random_bits(uint8_t *d_out, int64_t n, uint64_t seed, void *hip_stream) {
  if (n < 0 || (n > 0 && !d_out)) return set_err(nullptr, LDPC_EINVAL, "bad arguments");
  return ldpc::launch_random_bits(d_out, n, seed, hip_stream) == 0
             ? LDPC_OK
             : hip_err(nullptr, hipGetLastError(), "random_bits launch");
}

int ldpc_bpsk_awgn(const uint8_t *d_bits, int64_t n, float sigma, uint64_t seed, float *d_out,
                   void *hip_stream) {
  if (n < 0 || (n > 0 && (!d_bits || !d_out)) || !(sigma >= 0.0f))
    return set_err(nullptr, LDPC_EINVAL, "bad arguments");
  return ldpc::launch_bpsk_awgn(d_bits, n, sigma, seed, d_out, hip_stream) == 0
             ? LDPC_OK
             : hip_err(nullptr, hipGetLastError(), "bpsk_awgn launch");
}

int ldpc_count_bit_errors(const uint8_t *d_a, const uint8_t *d_b, int64_t per_frame, int B,
                          int32_t *d_counts, void *hip_stream) {
  if (B < 0 || per_frame < 0 || (B > 0 && (!d_a || !d_b || !d_counts)))
    return set_err(nullptr, LDPC_EINVAL, "bad arguments");
  return ldpc::launch_count_errors(d_a, d_b, per_frame, B, d_counts, hip_stream) == 0
             ? LDPC_OK
             : hip_err(nullptr, hipGetLastError(), "count_errors launch");
}

int ldpc_set_work_limit(ldpc_ctx *ctx, int64_t bytes) {
  if (!ctx || bytes < 0) return set_err(ctx, LDPC_EINVAL, "work limit must be >= 0");
  ctx->work_limit = bytes ? (size_t)bytes : ((size_t)8 << 30);
  return LDPC_OK;
}

}  // extern "C"

namespace {

// Enqueues one decode of device-resident frames.  pm_half > 0: B = 2 pm_half
// and frames pm_half.. re-decode windows 0..pm_half-1 with -polarity
// (DecodeArgs::pm_half), in the same launch on the small-code path.
int decode_device_impl(ldpc_ctx *ctx, int method, int max_iters, int et_period, int precision,
                       const float *d_in, int64_t cw_stride, int elem_stride, float polarity,
                       int B, int pm_half, uint8_t *d_out_packed, uint8_t *d_out_bits_opt,
                       int32_t *d_iters_used_opt, int32_t *d_syn_weight_opt,
                       float *d_llr_out_opt, void *hip_stream,
                       const int64_t *d_win = nullptr) {
  serve_stop(ctx);
  int rc = check_decode_args(ctx, method, max_iters, et_period, precision, B, elem_stride,
                             cw_stride);
  if (rc != LDPC_OK) return rc;
  if (B == 0) return LDPC_OK;
  if (!d_in || !d_out_packed) return set_err(ctx, LDPC_EINVAL, "null device buffer");
  ldpc::DecodeArgs a{};
  a.in = d_in;
  a.cw_stride = cw_stride;
  a.elem_stride = elem_stride;
  a.polarity = polarity;
  a.B = B;
  a.pm_half = 0;
  a.win = d_win;
  a.max_iters = max_iters;
  a.et_period = et_period;
  a.packed = d_out_packed;
  a.bits = d_out_bits_opt;
  a.iters = d_iters_used_opt;
  a.synd = d_syn_weight_opt;
  a.llr = d_llr_out_opt;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  void *st = hip_stream ? hip_stream : (void *)ctx->stream;
  if (ctx->graph) {
    if (d_win) return set_err(ctx, LDPC_EUNSUPPORTED, "window lists: small-code kernels only");
    // one workspace per context: order this decode after the previous one
    // when it was enqueued on another stream
    if (!ctx->graph_done &&
        (e = hipEventCreateWithFlags(&ctx->graph_done, hipEventDisableTiming)) != hipSuccess)
      return hip_err(ctx, e, "hipEventCreate");
    if (ctx->graph_stream && ctx->graph_stream != st &&
        (e = hipStreamWaitEvent((hipStream_t)st, ctx->graph_done, 0)) != hipSuccess)
      return hip_err(ctx, e, "hipStreamWaitEvent");
    if (pm_half > 0) {  // the large-code passes run per polarity
      ldpc::DecodeArgs n = a;
      a.B = n.B = pm_half;
      n.polarity = -polarity;
      n.packed += (int64_t)pm_half * ctx->KB;
      if (n.bits) n.bits += (int64_t)pm_half * ctx->N;
      if (n.iters) n.iters += pm_half;
      if (n.synd) n.synd += pm_half;
      if (n.llr) n.llr += (int64_t)pm_half * ctx->N;
      rc = decode_graph(ctx, a, method, precision, st);
      if (rc == LDPC_OK) rc = decode_graph(ctx, n, method, precision, st);
    } else {
      rc = decode_graph(ctx, a, method, precision, st);
    }
    if (rc != LDPC_OK) return rc;
    if ((e = hipEventRecord(ctx->graph_done, (hipStream_t)st)) != hipSuccess)
      return hip_err(ctx, e, "hipEventRecord");
    ctx->graph_stream = st;
    return LDPC_OK;
  }
  a.pm_half = pm_half;
  // the stream's own frame-queue counter (ldpc_kernels.hpp DecodeArgs::ticket)
  size_t q = 0;
  while (q < ctx->queues.size() && ctx->queues[q].stream != st) ++q;
  if (q == ctx->queues.size()) {
    if (q == LDPC_TICKET_SLOTS) {
      // more streams than counters: drain the device, start every queue over.
      // The memset runs on the null stream, which non-blocking streams are
      // not ordered after: wait for it before any stream launches again.
      if ((e = hipDeviceSynchronize()) != hipSuccess ||
          (e = hipMemset(ctx->d_tickets, 0,
                         (size_t)LDPC_TICKET_SLOTS * LDPC_TICKET_STRIDE * sizeof(uint32_t))) !=
              hipSuccess ||
          (e = hipDeviceSynchronize()) != hipSuccess)
        return hip_err(ctx, e, "ticket reset");
      ctx->queues.clear();
      q = 0;
    }
    // slots are handed out in order from zeroed memory (creation, reset)
    ctx->queues.push_back({st, 0u});
  }
  a.ticket = ctx->d_tickets + q * LDPC_TICKET_STRIDE;
  a.ticket_base = ctx->queues[q].base;
  a.waves = 0;
  // short frames (iteration cap <= 10): fixed frame stride, no queue atomics
  // (ldpc_kernels.hpp DecodeArgs::static_stride)
  a.static_stride = max_iters <= 10 ? 1 : 0;
  a.fair_cycles = ctx->fair_cycles;
  uint32_t advance = 0;
  rc = ldpc::launch_decode(code_view(ctx), a, method, precision, ctx->slots, ctx->nw,
                           ctx->waves_per_cu, ctx->schedule, st, &advance);
  if (rc == -2) return set_err(ctx, LDPC_EUNSUPPORTED, "no kernel for this code shape");
  if (rc != 0) return hip_err(ctx, hipGetLastError(), "kernel launch");
  ctx->queues[q].base += advance;  // what the launch adds to its counter (B with one frame per claim)
  return LDPC_OK;
}

// Host-buffer decode (synchronous).  B_out = B (pm_half 0) or 2B (both
// polarities).  The frames' samples are staged through a pinned buffer; for
// an interleaved gr_complex stream (elem_stride 2, even cw_stride) only the
// real parts are gathered and copied, and the kernel reads them densely.
int decode_host_impl(ldpc_ctx *ctx, int method, int max_iters, int et_period, int precision,
                     const float *in, int64_t n_in_floats, int64_t cw_stride, int elem_stride,
                     float polarity, int B, bool both, uint8_t *out_packed, uint8_t *out_bits_opt,
                     int32_t *iters_used_opt, int32_t *syn_weight_opt, float *llr_out_opt) {
  serve_stop(ctx);
  int rc = check_decode_args(ctx, method, max_iters, et_period, precision, B, elem_stride,
                             cw_stride);
  if (rc != LDPC_OK) return rc;
  if (B == 0) return LDPC_OK;
  if (!in || !out_packed) return set_err(ctx, LDPC_EINVAL, "null buffer");
  const int64_t span = (int64_t)(B - 1) * cw_stride + (int64_t)(ctx->N - 1) * elem_stride + 1;
  if (span > n_in_floats) return set_err(ctx, LDPC_EINVAL, "input shorter than the frames read");
  const bool re_only = elem_stride == 2 && cw_stride % 2 == 0;
  const int64_t n_stage = re_only ? (span + 1) / 2 : span;
  const int64_t cw = re_only ? cw_stride / 2 : cw_stride;
  const int es = re_only ? 1 : elem_stride;
  const int BO = both ? 2 * B : B;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t b_in = al((size_t)n_stage * 4), b_pk = al((size_t)BO * ctx->KB),
               b_bits = out_bits_opt ? al((size_t)BO * ctx->N) : 0,
               b_it = iters_used_opt ? al((size_t)BO * 4) : 0,
               b_sy = syn_weight_opt ? al((size_t)BO * 4) : 0,
               b_llr = llr_out_opt ? al((size_t)BO * ctx->N * 4) : 0;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  rc = ensure_stage(ctx, b_in + b_pk + b_bits + b_it + b_sy + b_llr);
  if (rc != LDPC_OK) return rc;
  // the pinned stage carries the input in and, after the kernel (stream
  // order), every output back in one copy of the adjacent device outputs
  const size_t b_out = b_pk + b_bits + b_it + b_sy + b_llr;
  rc = ensure_host_stage(ctx, std::max((size_t)n_stage * 4, b_out));
  if (rc != LDPC_OK) return rc;
  char *base = (char *)ctx->d_stage;
  float *d_in = (float *)base;
  uint8_t *d_pk = (uint8_t *)(base + b_in);
  uint8_t *d_bits = out_bits_opt ? (uint8_t *)(base + b_in + b_pk) : nullptr;
  int32_t *d_it = iters_used_opt ? (int32_t *)(base + b_in + b_pk + b_bits) : nullptr;
  int32_t *d_sy = syn_weight_opt ? (int32_t *)(base + b_in + b_pk + b_bits + b_it) : nullptr;
  float *d_llr = llr_out_opt ? (float *)(base + b_in + b_pk + b_bits + b_it + b_sy) : nullptr;
  float *h = ctx->h_stage;
  if (re_only)
    for (int64_t i = 0; i < n_stage; ++i) h[i] = in[2 * i];
  else
    memcpy(h, in, (size_t)span * 4);
  if ((e = hipMemcpyAsync(d_in, h, (size_t)n_stage * 4, hipMemcpyHostToDevice, ctx->stream)) !=
      hipSuccess)
    return hip_err(ctx, e, "hipMemcpyAsync(in)");
  rc = decode_device_impl(ctx, method, max_iters, et_period, precision, d_in, cw, es, polarity,
                          BO, both ? B : 0, d_pk, d_bits, d_it, d_sy, d_llr, ctx->stream);
  if (rc != LDPC_OK) return rc;
  if ((e = hipMemcpyAsync(h, d_pk, b_out, hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess)
    return hip_err(ctx, e, "hipMemcpyAsync(out)");
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess)
    return hip_err(ctx, e, "hipStreamSynchronize");
  const char *ho = (const char *)h;
  struct {
    void *dst;
    size_t off, n;
  } back[] = {{out_packed, 0, (size_t)BO * ctx->KB},
              {out_bits_opt, b_pk, (size_t)BO * ctx->N},
              {iters_used_opt, b_pk + b_bits, (size_t)BO * 4},
              {syn_weight_opt, b_pk + b_bits + b_it, (size_t)BO * 4},
              {llr_out_opt, b_pk + b_bits + b_it + b_sy, (size_t)BO * ctx->N * 4}};
  for (auto &c : back)
    if (c.dst) memcpy(c.dst, ho + c.off, c.n);
  return LDPC_OK;
}

// ldpc_decode_windows: span in ctx->d_wstage [0, span), then the window list,
// the gathered frames and the outputs.
// The window-launch staging area: the span at its start, window lists and
// outputs at its end.  A bigger area moves everything: the staged span is gone.
int ensure_window_stage(ldpc_ctx *ctx, size_t need) {
  if (need <= ctx->wstage_bytes) return LDPC_OK;
  if (ctx->d_wstage) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->d_wstage);
    ctx->d_wstage = nullptr;
    ctx->wstage_bytes = 0;
  }
  ctx->span_samples = 0;
  const size_t want = std::max(need + need / 2, (size_t)4 << 20);
  hipError_t e = hipMalloc(&ctx->d_wstage, want);
  if (e != hipSuccess) return hip_err(ctx, e, "hipMalloc(window staging)");
  ctx->wstage_bytes = want;
  return LDPC_OK;
}

// S samples in[i * elem_stride] -> pinned host stage -> d_span (enqueued on
// the context's stream; the launches that read it follow on the same stream).
int copy_span(ldpc_ctx *ctx, const float *in, int64_t S, int elem_stride, float *d_span) {
  int rc = ensure_host_stage(ctx, (size_t)S * 4);
  if (rc != LDPC_OK) return rc;
  float *h = ctx->h_stage;
  if (S >= ((int64_t)1 << 17)) {
    // big spans: gathered by the pool, each piece sent once ready
    if (!ctx->gather) {
      ctx->gather.reset(new GatherPool);
      for (int t = 0; t < GatherPool::kThreads; ++t)
        ctx->gather->th.emplace_back([g = ctx->gather.get()] { g->worker(); });
    }
    GatherPool &g = *ctx->gather;
    const int64_t np = (S + GatherPool::kPiece - 1) / GatherPool::kPiece;
    uint64_t gen;
    {
      std::lock_guard<std::mutex> lk(g.mu);
      if (g.ready_cap < np) {
        g.ready.reset(new std::atomic<uint64_t>[np]);
        for (int64_t p = 0; p < np; ++p) g.ready[p].store(0);
        g.ready_cap = np;
      }
      g.in = in;
      g.h = h;
      g.S = S;
      g.stride = elem_stride;
      g.npieces = np;
      g.next.store(0);
      gen = ++g.gen;
    }
    g.cv.notify_all();
    constexpr int64_t per_copy = GatherPool::kCopy / GatherPool::kPiece;
    for (int64_t p = 0; p < np; ++p) {
      while (g.ready[p].load(std::memory_order_acquire) != gen) {
        const int64_t q = g.next.fetch_add(1);  // help while waiting
        if (q < np) {
          g.gather(q);
          g.ready[q].store(gen, std::memory_order_release);
        } else {
          std::this_thread::yield();
        }
      }
      if ((p + 1) % per_copy != 0 && p + 1 != np) continue;
      const int64_t i0 = (p / per_copy) * GatherPool::kCopy, n = std::min(S - i0, GatherPool::kCopy);
      hipError_t e = hipMemcpyAsync(d_span + i0, h + i0, (size_t)n * 4, hipMemcpyHostToDevice,
                                    ctx->stream);
      if (e != hipSuccess) return hip_err(ctx, e, "hipMemcpyAsync(span)");
    }
    ctx->h_stage_busy = true;
    ctx->span_samples = S;
    return LDPC_OK;
  }
  // in pieces: each piece's copy to the device runs while the next is gathered
  const int64_t piece = S;
  for (int64_t i0 = 0; i0 < S; i0 += piece) {
    const int64_t i1 = std::min(S, i0 + piece);
    if (elem_stride == 1)
      memcpy(h + i0, in + i0, (size_t)(i1 - i0) * 4);
    else if (elem_stride == 2)  // gr_complex real parts (the block): a constant stride vectorises
      for (int64_t i = i0; i < i1; ++i) h[i] = in[2 * i];
    else
      for (int64_t i = i0; i < i1; ++i) h[i] = in[i * elem_stride];
    hipError_t e = hipMemcpyAsync(d_span + i0, h + i0, (size_t)(i1 - i0) * 4,
                                  hipMemcpyHostToDevice, ctx->stream);
    if (e != hipSuccess) return hip_err(ctx, e, "hipMemcpyAsync(span)");
  }
  ctx->h_stage_busy = true;
  ctx->span_samples = S;
  return LDPC_OK;
}

int decode_windows_impl(ldpc_ctx *ctx, int method, int max_iters, int et_period, int precision,
                        const float *in, int64_t n_in_floats, int elem_stride, int reuse_span,
                        const int64_t *win, int B, uint8_t *out_packed, int32_t *syn_weight_opt) {
  serve_stop(ctx);
  int rc = check_decode_args(ctx, method, max_iters, et_period, precision, B, elem_stride,
                             ctx ? ctx->N : 1);
  if (rc != LDPC_OK) return rc;
  if (B == 0) return LDPC_OK;
  if (!in || !win || !out_packed) return set_err(ctx, LDPC_EINVAL, "null buffer");
  const int N = ctx->N;
  const int64_t S = (n_in_floats + elem_stride - 1) / elem_stride;  // samples in the span
  for (int b = 0; b < B; ++b)
    if (win[b] < 0 || (win[b] >> 1) + N > S)
      return set_err(ctx, LDPC_EINVAL, "window outside the input span");
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t b_span = al((size_t)S * 4), b_win = al((size_t)B * 8),
               // gathered frames: only the large-code kernels need them
               b_fr = ctx->graph ? al((size_t)B * N * 4) : 0, b_pk = al((size_t)B * ctx->KB),
               b_sy = al((size_t)B * 4);
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  rc = ensure_window_stage(ctx, b_span + b_win + b_fr + b_pk + b_sy);
  if (rc != LDPC_OK) return rc;
  // pinned: the window list in, then the packed words and syndrome weights
  // out in one copy (d_pk .. d_sy are adjacent in the staging area), so no
  // transfer goes through a pageable bounce
  const size_t h_need = b_win + b_pk + b_sy;
  if (h_need > ctx->h_win_bytes) {
    if (ctx->h_win) {
      (void)hipStreamSynchronize(ctx->stream);
      (void)hipHostFree(ctx->h_win);
      ctx->h_win = nullptr;
    }
    const size_t want = std::max(h_need + h_need / 2, (size_t)1 << 16);
    // mapped and coherent: the small-code kernels read the window list and
    // write their outputs here directly (no copy either way; see below)
    if ((e = hipHostMalloc((void **)&ctx->h_win, want,
                           hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
      return hip_err(ctx, e, "hipHostMalloc(windows)");
    ctx->h_win_bytes = want;
  }
  // the span sits at the start of the staging area; a reused span must be the
  // one staged last, with the same length (then it ends before span_cap)
  char *base = (char *)ctx->d_wstage;
  const size_t span_cap = ctx->wstage_bytes - (b_win + b_fr + b_pk + b_sy);
  float *d_span = (float *)base;
  int64_t *d_win = (int64_t *)(base + span_cap);
  float *d_fr = (float *)(base + span_cap + b_win);
  uint8_t *d_pk = (uint8_t *)(base + span_cap + b_win + b_fr);
  int32_t *d_sy = (int32_t *)(base + span_cap + b_win + b_fr + b_pk);
  const auto tnow = []() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  double t0 = ctx->win_profile ? tnow() : 0.0;
  if (!(reuse_span && ctx->span_samples == S)) {
    rc = copy_span(ctx, in, S, elem_stride, d_span);
    if (rc != LDPC_OK) return rc;
  }
  if (ctx->win_profile) {
    const double t1 = tnow();
    ctx->win_prof[0] += t1 - t0;
    t0 = t1;
  }
  // the previous call's copy out of h_win has completed (it synchronised)
  memcpy(ctx->h_win, win, (size_t)B * 8);
  uint8_t *h_out = (uint8_t *)ctx->h_win + b_win;
  // Small codes: the kernel reads the (pinned, mapped) window list and writes
  // its packed bytes and syndrome weights into pinned memory itself -- a few
  // bytes per window over the bus, and no DMA round trip on a launch whose
  // latency is that of one frame
  const bool direct = !ctx->graph;
  if (direct) {
    void *dv = nullptr;
    if ((e = hipHostGetDevicePointer(&dv, ctx->h_win, 0)) != hipSuccess)
      return hip_err(ctx, e, "hipHostGetDevicePointer(windows)");
    d_win = (int64_t *)dv;
    d_pk = (uint8_t *)dv + b_win;
    d_sy = (int32_t *)((uint8_t *)dv + b_win + b_pk);
  } else if ((e = hipMemcpyAsync(d_win, ctx->h_win, (size_t)B * 8, hipMemcpyHostToDevice,
                                 ctx->stream)) != hipSuccess) {
    return hip_err(ctx, e, "hipMemcpyAsync(windows)");
  }
  if (ctx->graph) {  // the large-code kernels read frames at a fixed stride: gather first
    if (ldpc::launch_gather_windows(d_span, d_win, B, N, d_fr, ctx->stream) != 0)
      return set_err(ctx, LDPC_EDEVICE, "gather_windows launch failed");
    rc = decode_device_impl(ctx, method, max_iters, et_period, precision, d_fr, N, 1, 1.0f, B,
                            0, d_pk, nullptr, nullptr, syn_weight_opt ? d_sy : nullptr, nullptr,
                            ctx->stream);
  } else {  // the small-code kernels read each window in place (DecodeArgs::win)
    rc = decode_device_impl(ctx, method, max_iters, et_period, precision, d_span, N, 1, 1.0f, B,
                            0, d_pk, nullptr, nullptr, syn_weight_opt ? d_sy : nullptr, nullptr,
                            ctx->stream, d_win);
  }
  if (rc != LDPC_OK) return rc;
  const size_t out_bytes = syn_weight_opt ? b_pk + (size_t)B * 4 : (size_t)B * ctx->KB;
  if (!direct && (e = hipMemcpyAsync(h_out, d_pk, out_bytes, hipMemcpyDeviceToHost,
                                     ctx->stream)) != hipSuccess)
    return hip_err(ctx, e, "hipMemcpyAsync(out)");
  if (ctx->win_profile) {
    const double t1 = tnow();
    ctx->win_prof[1] += t1 - t0;
    t0 = t1;
  }
  // wait for the launch (polling measured no faster,
  // profiles/round2/block/window_latency.txt)
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess)
    return hip_err(ctx, e, "hipStreamSynchronize");
  if (ctx->win_profile) {
    const double t1 = tnow();
    ctx->win_prof[2] += t1 - t0;
    t0 = t1;
  }
  memcpy(out_packed, h_out, (size_t)B * ctx->KB);
  if (syn_weight_opt) memcpy(syn_weight_opt, h_out + b_pk, (size_t)B * 4);
  if (ctx->win_profile) {
    ctx->win_prof[3] += tnow() - t0;
    ctx->win_calls += 1;
    ctx->win_windows += B;
    if (ctx->win_trace) {
      static double last[4] = {0, 0, 0, 0};
      fprintf(stderr, "decode_windows B=%d stage %.1f list+launch %.1f wait %.1f results %.1f us\n",
              B, 1e6 * (ctx->win_prof[0] - last[0]), 1e6 * (ctx->win_prof[1] - last[1]),
              1e6 * (ctx->win_prof[2] - last[2]), 1e6 * (ctx->win_prof[3] - last[3]));
      for (int i = 0; i < 4; ++i) last[i] = ctx->win_prof[i];
    }
  }
  return LDPC_OK;
}

// Launches the window server for the context's parameters on its stream
// (ctl zeroed first: it must read below every epoch the launch serves).
// repost_n >= 0 (a relaunch after the old launch's deadline): the round the
// host is waiting on, repost_n windows, is posted again with the NEW session
// before the launch, so the new poller never sees the old session's word for
// it and quits (the host used to post after the launch).
int serve_launch(ldpc_ctx *ctx, int repost_n = -1) {
  hipError_t e;
  if (!ctx->d_srv_ctl || !ctx->d_srv_keys || !ctx->h_srv)
    return set_err(ctx, LDPC_EINVAL, "window server buffers missing");
  if ((e = hipSetDevice(ctx->device)) != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  if ((e = hipMemsetAsync(ctx->d_srv_ctl, 0, ldpc::kServeCtlBytes, ctx->stream)) != hipSuccess)
    return hip_err(ctx, e, "hipMemsetAsync(server ctl)");
  void *dh = nullptr;
  if ((e = hipHostGetDevicePointer(&dh, ctx->h_srv, 0)) != hipSuccess)
    return hip_err(ctx, e, "hipHostGetDevicePointer(server)");
  ldpc::ServeArgs sa{};
  sa.round = (const uint64_t *)dh;
  sa.keys = (const int64_t *)((uint8_t *)dh + srv_keys_off());
  sa.res = (uint64_t *)((uint8_t *)dh + srv_res_off(ctx->srv_cap));
  sa.dkeys = ctx->d_srv_keys;
  sa.ctl = ctx->d_srv_ctl;
  sa.span = ctx->span_samples;
  const char *dl = getenv("LDPC_SERVE_DEADLINE_MS");
  sa.deadline = (uint64_t)((dl ? atof(dl) : 200.0) * 1e5);  // 100 MHz ticks
  ctx->srv_launches += 1;  // this launch's session: the rounds posted from now on
  sa.session = (uint32_t)ctx->srv_launches;
  if (repost_n >= 0) {
    ctx->srv_epoch -= 1;  // the launch serves epochs above start_epoch
    sa.start_epoch = ctx->srv_epoch;
    serve_post(ctx, (uint32_t)repost_n);  // the same round (epoch, key tags), the new session
  } else {
    sa.start_epoch = ctx->srv_epoch;
  }
  // decoder workgroups per CU (capped by occupancy); 0 = as many as fit
  const char *pc = getenv("LDPC_SERVE_BLOCKS_PER_CU");
  sa.blocks_per_cu = pc ? atoi(pc) : 0;
  ctx->srv_debug = getenv("LDPC_SERVE_DEBUG") != nullptr;  // (read per launch)
  sa.debug = ctx->srv_debug ? 1 : 0;
  int wg = 0;
  ldpc::DecodeArgs a{};
  a.in = (const float *)ctx->d_wstage;
  a.cw_stride = ctx->N;
  a.elem_stride = 1;
  a.polarity = 1.0f;
  a.max_iters = ctx->srv_iters;
  a.et_period = 1;
  const int rc = ldpc::launch_serve(code_view(ctx), a, sa, ctx->srv_method, ctx->srv_prec,
                                    ctx->slots, ctx->nw, ctx->device, ctx->stream, &wg);
  ctx->srv_workgroups = wg;
  if (rc == -2) return set_err(ctx, LDPC_EUNSUPPORTED, "no window server for this code shape");
  if (rc != 0) return hip_err(ctx, hipGetLastError(), "window server launch");
  return LDPC_OK;
}

// Starts the epochs over (a new session): the running launch, if any, has
// finished; host keys and results and the device key copies are cleared, so
// no slot carries a tag from before the restart.
int serve_reset_epochs(ldpc_ctx *ctx) {
  hipError_t e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return hip_err(ctx, e, "hipStreamSynchronize(server)");
  memset(ctx->h_srv, 0, srv_bytes(ctx->srv_cap));
  if ((e = hipMemsetAsync(ctx->d_srv_keys, 0, (size_t)ctx->srv_cap * 8, ctx->stream)) != hipSuccess)
    return hip_err(ctx, e, "hipMemsetAsync(server keys)");
  ctx->srv_epoch = 0;
  return LDPC_OK;
}

int serve_begin_impl(ldpc_ctx *ctx, int method, int max_iters, int precision, int max_windows) {
  int rc = check_decode_args(ctx, method, max_iters, 1, precision, 1, 1, ctx ? ctx->N : 1);
  if (rc != LDPC_OK) return rc;
  if (ctx->graph || ctx->KB > 4 || (method != 0 && method != 1))
    return set_err(ctx, LDPC_EUNSUPPORTED,
                   "the window server takes min-sum / sum-product on small codes with KB <= 4");
  if (ctx->span_samples <= 0) return set_err(ctx, LDPC_EINVAL, "no staged span (ldpc_stage_span)");
  if (max_windows < 1 || max_windows > (1 << 19))
    return set_err(ctx, LDPC_EINVAL, "max_windows must be in [1, 2^19]");
  if (ctx->serving) {
    if (ctx->srv_method == method && ctx->srv_iters == max_iters && ctx->srv_prec == precision &&
        ctx->srv_cap >= max_windows)
      return LDPC_OK;
    serve_stop(ctx);
  }
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  if (!ctx->d_srv_ctl && (e = hipMalloc((void **)&ctx->d_srv_ctl, ldpc::kServeCtlBytes)) != hipSuccess)
    return hip_err(ctx, e, "hipMalloc(server ctl)");
  // a new buffer (or epochs near the end of their range) starts the epochs over:
  // the previous launch has finished first
  if (ctx->srv_cap < max_windows || ctx->srv_epoch >= ldpc::kServeEpochLimit) {
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->srv_cap < max_windows) {
      if (ctx->h_srv) (void)hipHostFree(ctx->h_srv);
      if (ctx->d_srv_keys) (void)hipFree(ctx->d_srv_keys);
      ctx->h_srv = nullptr;
      ctx->d_srv_keys = nullptr;
      ctx->srv_cap = 0;
      const int64_t cap = std::max<int64_t>(max_windows, 4096);
      if ((e = hipHostMalloc((void **)&ctx->h_srv, srv_bytes(cap),
                             hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
        return hip_err(ctx, e, "hipHostMalloc(server)");
      if ((e = hipMalloc((void **)&ctx->d_srv_keys, (size_t)cap * 8)) != hipSuccess)
        return hip_err(ctx, e, "hipMalloc(server keys)");
      ctx->srv_cap = cap;
    }
    if ((rc = serve_reset_epochs(ctx)) != LDPC_OK) return rc;
  }
  ctx->srv_method = method;
  ctx->srv_iters = max_iters;
  ctx->srv_prec = precision;
  rc = serve_launch(ctx);
  if (rc != LDPC_OK) return rc;
  ctx->serving = true;
  return LDPC_OK;
}

int serve_windows_impl(ldpc_ctx *ctx, const int64_t *win, int B, uint8_t *out_packed,
                       int32_t *syn_weight_opt) {
  if (!ctx) return LDPC_EINVAL;
  if (!ctx->serving) return set_err(ctx, LDPC_EINVAL, "no window server running (ldpc_serve_begin)");
  if (B < 0) return set_err(ctx, LDPC_EINVAL, "B < 0");
  if (B == 0) return LDPC_OK;
  if (!win || !out_packed) return set_err(ctx, LDPC_EINVAL, "null buffer");
  const int N = ctx->N, KB = ctx->KB;
  // (ldpc_test_hook 1 skips this check once, so that the device's own check
  // of every key -- ldpc_serve.hip key_fault -- can be exercised)
  const bool host_check = !ctx->srv_test_skip_check;
  ctx->srv_test_skip_check = false;
  for (int b = 0; b < B; ++b)
    if (win[b] < 0 || win[b] >= ((int64_t)1 << 40) ||
        (host_check && (win[b] >> 1) + N > ctx->span_samples))
      return set_err(ctx, LDPC_EINVAL, "window outside the staged span");
  int device_fault = 0;  // a granule that carries no decode (kServeBadKey / kServeLostKey)
  int64_t fault_key = 0;
  int64_t *keys = (int64_t *)(ctx->h_srv + srv_keys_off());
  const uint64_t *res = (const uint64_t *)(ctx->h_srv + srv_res_off(ctx->srv_cap));
  const double timeout_s = 10.0;
  for (int b0 = 0; b0 < B; b0 += (int)ctx->srv_cap) {
    const int n = (int)std::min<int64_t>(ctx->srv_cap, B - b0);
    // epochs stay below kServeEpochLimit (result tags are epoch mod 2^23, and a
    // tag that wrapped would match a stale slot): a session that reaches it is
    // ended and started over before this round
    if (ctx->srv_epoch + 2 >= ldpc::kServeEpochLimit) {
      serve_stop(ctx);
      int rc = serve_reset_epochs(ctx);
      if (rc == LDPC_OK) rc = serve_launch(ctx);
      if (rc != LDPC_OK) return rc;
      ctx->serving = true;
    }
    // each key carries the epoch it is posted with (mod 2^24), so the poller
    // can tell a slot it read before this round's write (ldpc_serve.hip)
    const uint64_t ktag = (uint64_t)((ctx->srv_epoch + 1) & 0xFFFFFFu) << 40;
    for (int b = 0; b < n; ++b) keys[b] = (int64_t)((uint64_t)win[b0 + b] | ktag);
    serve_post(ctx, (uint32_t)n);
    ctx->srv_rounds += 1;
    const uint32_t tag = ctx->srv_epoch & 0x7FFFFFu;
    const auto t0 = std::chrono::steady_clock::now();
    auto t_first = t0;
    int relaunches = 0;
    for (int b = 0; b < n; ++b) {
      if (b == 1 && ctx->srv_debug) t_first = std::chrono::steady_clock::now();
      uint64_t g;
      for (uint32_t spins = 1;; ++spins) {
        g = __atomic_load_n(res + b, __ATOMIC_ACQUIRE);
        if ((uint32_t)(g >> 41) == tag) break;
        if ((spins & 0xFFFu) == 0) {
          // the launch ended (its deadline passed between rounds): start another
          const hipError_t q = hipStreamQuery(ctx->stream);
          if (q == hipSuccess) {
            if (ctx->srv_debug) {
              uint64_t c[8] = {0}, c0 = 0;
              uint32_t census = 0;
              (void)hipMemcpy(&c0, ctx->d_srv_ctl, 8, hipMemcpyDeviceToHost);
              (void)hipMemcpy(&census, ctx->d_srv_ctl + 16 * ldpc::kServeCopies, 4, hipMemcpyDeviceToHost);
              (void)hipMemcpy(c, ctx->d_srv_ctl + 16 * (ldpc::kServeCopies + 1), sizeof c,
                              hipMemcpyDeviceToHost);
              fprintf(stderr,
                      "ldpc_serve: launch %d ended before round %u (B %d, result %d of them "
                      "in): ctl %016llx census %u, poller exit %llu on round word %016llx, "
                      "host round word %016llx; decoder round starts %llu (g0 saw %016llx), "
                      "mw results %llu\n",
                      ctx->srv_launches, ctx->srv_epoch, n, b, (unsigned long long)c0, census,
                      (unsigned long long)c[0], (unsigned long long)c[1],
                      (unsigned long long)*(const uint64_t *)ctx->h_srv, (unsigned long long)c[2],
                      (unsigned long long)c[3], (unsigned long long)c[4]);
            }
            if (++relaunches > 4) {
              ctx->serving = false;
              return set_err(ctx, LDPC_ETIMEOUT, "the window server keeps ending before its round");
            }
            const int rc = serve_launch(ctx, n);  // the same round, posted for the new session
            if (rc != LDPC_OK) {
              ctx->serving = false;
              return rc;
            }
          } else if (q != hipErrorNotReady) {
            ctx->serving = false;
            return hip_err(ctx, q, "window server");
          }
          if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
            serve_stop(ctx);
            return set_err(ctx, LDPC_ETIMEOUT, "a window server round passed its timeout");
          }
        }
      }
      const uint32_t pk = (uint32_t)g, wt = (uint32_t)(g >> 32) & 511u;
      if (wt == ldpc::kServeBadKey || wt == ldpc::kServeLostKey) {
        if (!device_fault) {
          device_fault = (int)wt;
          fault_key = win[b0 + b];
        }
        continue;  // (the round's other results are still collected)
      }
      for (int j = 0; j < KB; ++j) out_packed[(size_t)(b0 + b) * KB + j] = (uint8_t)(pk >> (8 * j));
      if (syn_weight_opt) syn_weight_opt[b0 + b] = (int32_t)wt;
    }
    if (ctx->srv_debug) {  // device-side split of the round (100 MHz ticks)
      const double host_us =
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e6;
      const double first_us = std::chrono::duration<double>(t_first - t0).count() * 1e6;
      uint64_t c[9] = {0};
      uint64_t *dg = ctx->d_srv_ctl + 16 * (ldpc::kServeCopies + 1);
      (void)hipMemcpy(c, dg, sizeof c, hipMemcpyDeviceToHost);
      const uint64_t zero[2] = {0, 0};
      (void)hipMemcpy(dg + 6, zero, sizeof zero, hipMemcpyHostToDevice);
      // (only the one-wave form of big rounds does not time its decoders)
      if (c[6] >= c[5] && c[7] >= c[5] && c[5] >= c[8]) {
        ctx->dbg[0] += 1;
        ctx->dbg[1] += host_us;
        ctx->dbg[2] += 1e-2 * (double)(c[5] - c[8]);
        ctx->dbg[3] += 1e-2 * (double)(c[6] - c[5]);
        ctx->dbg[4] += 1e-2 * (double)(c[7] - c[5]);
        ctx->dbg[5] += n > 1 ? first_us : host_us;
      }
    }
  }
  if (device_fault) {
    char buf[200];
    snprintf(buf, sizeof buf,
             "window server: %s (window key %lld, span of %lld samples); the window was not "
             "decoded",
             device_fault == (int)ldpc::kServeBadKey
                 ? "the device refused a window key outside the staged span"
                 : "a window key never reached the device within the deadline",
             (long long)fault_key, (long long)ctx->span_samples);
    return set_err(ctx, LDPC_EDEVICE, buf);
  }
  return LDPC_OK;
}

// ---- the frame ring (ldpc_ring_*) -------------------------------------------
// Mapped host memory: kRingSlots 64-byte descriptors, then kRingSlots
// completion words.  Device memory: kRingSlots frame counters, one 256-byte
// line each, then the queue head on a line of its own.
constexpr size_t kRingCompOff = sizeof(ldpc::RingDesc) * ldpc::kRingSlots;
constexpr size_t kRingHostBytes = kRingCompOff + 8 * ldpc::kRingSlots;
constexpr size_t kRingTicketOff = (size_t)ldpc::kRingSlots * ldpc::kRingDoneStride;  // in u32
constexpr size_t kRingMirrorOff = 4 * (kRingTicketOff + 64);  // bytes: the descriptor mirror
constexpr size_t kRingLockOff =
    kRingMirrorOff + sizeof(ldpc::RingDesc) * ldpc::kRingSlots * ldpc::kRingXcds;
constexpr size_t kRingDevBytes = kRingLockOff + 8 * ldpc::kRingSlots * ldpc::kRingXcds;
constexpr uint64_t kRingDeadlineTicks = 5000000;  // 50 ms without a batch: a wave leaves
constexpr double kRingTimeoutS = 10.0;

bool ring_done(ldpc_ctx *ctx, uint64_t q) {
  return __atomic_load_n(reinterpret_cast<uint64_t *>(ctx->h_ring + kRingCompOff) +
                             q % ldpc::kRingSlots,
                         __ATOMIC_ACQUIRE) >= q + 1;
}

// Writes batch q's descriptor: words 1..7 tagged with (q + 1) mod 2^16 in bits
// 48..63, then word 0 = q + 1 (x86 stores are ordered; the device accepts the
// line only when all eight agree, ldpc_ring.hip locate).
void ring_write_desc(ldpc_ctx *ctx, uint64_t q, int64_t start, const void *in, int64_t cw,
                     void *packed, void *iters, void *synd, int B, int quit) {
  uint64_t *w = reinterpret_cast<uint64_t *>(ctx->h_ring) + 8 * (q % ldpc::kRingSlots);
  const uint64_t tag = ((q + 1) & 0xFFFFu) << 48, pay = (1ull << 48) - 1;
  const uint64_t v[7] = {(uint64_t)start, (uint64_t)(uintptr_t)in, (uint64_t)cw,
                         (uint64_t)(uintptr_t)packed, (uint64_t)(uintptr_t)iters,
                         (uint64_t)(uintptr_t)synd,
                         (uint64_t)(uint32_t)B | ((uint64_t)(quit ? 1 : 0) << 32)};
  for (int j = 0; j < 7; ++j) __atomic_store_n(w + 1 + j, (v[j] & pay) | tag, __ATOMIC_RELAXED);
  __atomic_store_n(w, q + 1, __ATOMIC_RELEASE);
}

// Launches the ring from batch `cursor` (every earlier batch complete), its
// first ticket `ticket0`: counters and queue head zeroed first, on the ring's
// stream, and the event recorded behind the launch.
int ring_launch(ldpc_ctx *ctx, uint64_t cursor, int64_t ticket0) {
  hipError_t e;
  if ((e = hipSetDevice(ctx->device)) != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  // (zeroed behind the previous session's launch by ldpc_ring_end, off the
  // next session's critical path; a relaunch zeroes here)
  if (!ctx->ring_clean &&
      (e = hipMemsetAsync(ctx->d_ring, 0, kRingDevBytes, ctx->ring_stream)) != hipSuccess)
    return hip_err(ctx, e, "hipMemsetAsync(ring)");
  ctx->ring_clean = false;
  void *dh = nullptr;
  if ((e = hipHostGetDevicePointer(&dh, ctx->h_ring, 0)) != hipSuccess)
    return hip_err(ctx, e, "hipHostGetDevicePointer(ring)");
  ldpc::RingArgs r{};
  r.desc = reinterpret_cast<const ldpc::RingDesc *>(dh);
  r.comp = reinterpret_cast<uint64_t *>((uint8_t *)dh + kRingCompOff);
  r.done = ctx->d_ring;
  r.ticket = ctx->d_ring + kRingTicketOff;
  r.mirror = reinterpret_cast<uint64_t *>(reinterpret_cast<uint8_t *>(ctx->d_ring) + kRingMirrorOff);
  r.lock = reinterpret_cast<uint64_t *>(reinterpret_cast<uint8_t *>(ctx->d_ring) + kRingLockOff);
  r.ticket0 = ticket0;
  r.cursor0 = cursor;
  r.deadline = kRingDeadlineTicks;
  r.max_iters = ctx->ring_iters;
  r.et_period = ctx->ring_et;
  int wg = 0;
  const int rc = ldpc::launch_ring(code_view(ctx), r, ctx->ring_method, ctx->ring_prec, ctx->slots,
                                   ctx->nw, ctx->device, ctx->ring_stream, &wg);
  if (rc == -2) return set_err(ctx, LDPC_EUNSUPPORTED, "no frame ring for this code shape");
  if (rc != 0) return hip_err(ctx, hipGetLastError(), "frame ring launch");
  ctx->ring_workgroups = wg;
  ctx->ring_launches += 1;
  if ((e = hipEventRecord(ctx->ring_ev, ctx->ring_stream)) != hipSuccess)
    return hip_err(ctx, e, "hipEventRecord(ring)");
  return LDPC_OK;
}

// A launch whose waves all left on the deadline (no batch for 50 ms) has
// ended: if posted batches are not complete, launch again from the first of
// them.  Its frames are decoded again from frame 0 -- a wave may have left
// holding a ticket of a batch it never saw -- and the frame counters start
// at zero, so a batch completes exactly once.
// `upto`: batches before it are the ones that must complete (a posted quit
// descriptor is not one of them).
int ring_revive(ldpc_ctx *ctx, uint64_t upto) {
  const hipError_t q = hipEventQuery(ctx->ring_ev);
  if (q == hipErrorNotReady) return LDPC_OK;
  if (q != hipSuccess) return hip_err(ctx, q, "frame ring");
  uint64_t first = upto;
  const uint64_t lo = std::max<uint64_t>(
      ctx->ring_first, upto > (uint64_t)ldpc::kRingSlots ? upto - ldpc::kRingSlots : 0);
  for (uint64_t b = lo; b < upto; ++b)
    if (!ring_done(ctx, b)) {
      first = b;
      break;
    }
  if (first == upto) return LDPC_OK;  // nothing outstanding: relaunch on the next post
  return ring_launch(ctx, first, ctx->ring_start[first % ldpc::kRingSlots]);
}

// Waits until batch q is complete (q < ring_next).
int ring_wait_impl(ldpc_ctx *ctx, uint64_t q) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spins = 1; !ring_done(ctx, q); ++spins) {
    if ((spins & 0x3FFu) == 0) {
      const int rc = ring_revive(ctx, q + 1);
      if (rc != LDPC_OK) return rc;
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() >
          kRingTimeoutS)
        return set_err(ctx, LDPC_ETIMEOUT, "a frame ring batch passed its timeout");
    }
  }
  return LDPC_OK;
}

// Posts one descriptor (a batch, or quit): waits for its slot's previous
// batch, writes the line, and relaunches a launch that has ended.
int64_t ring_post_impl(ldpc_ctx *ctx, const float *d_in, int64_t cw, int B, uint8_t *packed,
                       int32_t *iters, int32_t *synd, int quit) {
  const uint64_t q = ctx->ring_next;
  if (q >= ctx->ring_first + ldpc::kRingSlots) {
    const int rc = ring_wait_impl(ctx, q - ldpc::kRingSlots);
    if (rc != LDPC_OK) return rc;
  }
  ctx->ring_start[q % ldpc::kRingSlots] = ctx->ring_frames;
  ring_write_desc(ctx, q, ctx->ring_frames, d_in, cw, packed, iters, synd, B, quit);
  ctx->ring_next = q + 1;
  ctx->ring_frames += B;
  // a launch that has ended meanwhile would never see it
  // (a quit descriptor alone needs no launch: nothing would be decoded)
  const int rc = ring_revive(ctx, quit ? q : q + 1);
  return rc != LDPC_OK ? rc : (int64_t)q;
}
}  // namespace

extern "C" {

int ldpc_stage_span(ldpc_ctx *ctx, const float *in, int64_t n_in_floats, int elem_stride,
                    int max_windows) {
  serve_stop(ctx);
  if (!ctx) return LDPC_EINVAL;
  if (!in || elem_stride < 1 || n_in_floats < 0 || max_windows < 0)
    return set_err(ctx, LDPC_EINVAL, "bad span");
  const int64_t S = (n_in_floats + elem_stride - 1) / elem_stride;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t B = (size_t)max_windows;
  // room for that many windows' lists and outputs behind the span
  const size_t extra = al(B * 8) + (ctx->graph ? al(B * (size_t)ctx->N * 4) : 0) +
                       al(B * (size_t)ctx->KB) + al(B * 4);
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  int rc = ensure_window_stage(ctx, al((size_t)S * 4) + extra);
  if (rc != LDPC_OK) return rc;
  return copy_span(ctx, in, S, elem_stride, (float *)ctx->d_wstage);
}

int ldpc_serve_begin(ldpc_ctx *ctx, int method, int max_iters, int precision, int max_windows) {
  return serve_begin_impl(ctx, method, max_iters, precision, max_windows);
}

int ldpc_serve_windows(ldpc_ctx *ctx, const int64_t *windows, int B, uint8_t *out_packed,
                       int32_t *syn_weight_opt) {
  return serve_windows_impl(ctx, windows, B, out_packed, syn_weight_opt);
}

int ldpc_serve_end(ldpc_ctx *ctx) {
  if (!ctx) return LDPC_EINVAL;
  if (ctx->srv_debug && ctx->dbg[0] > 0) {
    fprintf(stderr,
            "ldpc_serve: %.0f rounds: host %.1f us per round; poller: sight to publication %.1f "
            "us; from the publication: last key read %.1f us, last result stored %.1f us; host: "
            "first result seen %.1f us after the post (mean over rounds)\n",
            ctx->dbg[0], ctx->dbg[1] / ctx->dbg[0], ctx->dbg[2] / ctx->dbg[0],
            ctx->dbg[3] / ctx->dbg[0], ctx->dbg[4] / ctx->dbg[0], ctx->dbg[5] / ctx->dbg[0]);
    for (double &d : ctx->dbg) d = 0;
    uint32_t census = 0;
    (void)hipMemcpy(&census, ctx->d_srv_ctl + 16 * ldpc::kServeCopies, 4, hipMemcpyDeviceToHost);
    fprintf(stderr, "ldpc_serve: %u of %d decoder workgroups started\n", census, ctx->srv_workgroups);
  }
  if (ctx->serving) {  // the launch finishes on its own; the stream orders what follows
    serve_post(ctx, ldpc::kServeB);
    ctx->serving = false;
  }
  return LDPC_OK;
}

int ldpc_ring_begin(ldpc_ctx *ctx, int method, int max_iters, int et_period, int precision,
                    void *hip_stream) {
  if (!ctx) return LDPC_EINVAL;
  int rc = check_decode_args(ctx, method, max_iters, et_period, precision, 1, 1, ctx->N);
  if (rc != LDPC_OK) return rc;
  if (ctx->ring_on) return set_err(ctx, LDPC_EINVAL, "a frame ring session is open (ldpc_ring_end)");
  if (ctx->graph || (method != 0 && method != 1))
    return set_err(ctx, LDPC_EUNSUPPORTED,
                   "the frame ring takes min-sum / sum-product on small codes");
  serve_stop(ctx);
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  if (!ctx->h_ring &&
      (e = hipHostMalloc((void **)&ctx->h_ring, kRingHostBytes,
                         hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
    return hip_err(ctx, e, "hipHostMalloc(ring)");
  if (!ctx->d_ring && (e = hipMalloc((void **)&ctx->d_ring, kRingDevBytes)) != hipSuccess)
    return hip_err(ctx, e, "hipMalloc(ring)");
  if (!ctx->ring_stream &&
      (e = hipStreamCreateWithFlags(&ctx->ring_stream, hipStreamNonBlocking)) != hipSuccess)
    return hip_err(ctx, e, "hipStreamCreate(ring)");
  if (!ctx->ring_ev && (e = hipEventCreateWithFlags(&ctx->ring_ev, hipEventDisableTiming)) != hipSuccess)
    return hip_err(ctx, e, "hipEventCreate(ring)");
  if (!ctx->ring_user_ev &&
      (e = hipEventCreateWithFlags(&ctx->ring_user_ev, hipEventDisableTiming)) != hipSuccess)
    return hip_err(ctx, e, "hipEventCreate(ring)");
  // the previous session's launch has ended before the slots are cleared
  if ((e = hipStreamSynchronize(ctx->ring_stream)) != hipSuccess)
    return hip_err(ctx, e, "hipStreamSynchronize(ring)");
  // sequence numbers and tickets keep growing across the context's sessions,
  // so no line a previous session left anywhere (host slots, the device
  // mirror, a cache) can read as one of this session's batches
  memset(ctx->h_ring, 0, kRingHostBytes);
  ctx->ring_method = method;
  ctx->ring_iters = max_iters;
  ctx->ring_et = et_period;
  ctx->ring_prec = precision;
  ctx->ring_first = ctx->ring_next;
  ctx->ring_first_frame = ctx->ring_frames;
  // the launch follows the work enqueued on the caller's stream so far
  ctx->ring_user_stream = hip_stream ? hip_stream : (void *)ctx->stream;
  if ((e = hipEventRecord(ctx->ring_user_ev, (hipStream_t)ctx->ring_user_stream)) != hipSuccess ||
      (e = hipStreamWaitEvent(ctx->ring_stream, ctx->ring_user_ev, 0)) != hipSuccess)
    return hip_err(ctx, e, "frame ring: stream order");
  rc = ring_launch(ctx, ctx->ring_next, ctx->ring_frames);
  if (rc != LDPC_OK) return rc;
  ctx->ring_on = true;
  return LDPC_OK;
}

int64_t ldpc_ring_post(ldpc_ctx *ctx, const float *d_in, int64_t cw_stride, int B,
                       uint8_t *d_out_packed, int32_t *d_iters_used_opt,
                       int32_t *d_syn_weight_opt) {
  if (!ctx) return LDPC_EINVAL;
  if (!ctx->ring_on) return set_err(ctx, LDPC_EINVAL, "no frame ring session (ldpc_ring_begin)");
  if (B < 1) return set_err(ctx, LDPC_EINVAL, "B must be >= 1");
  if (!d_in || !d_out_packed) return set_err(ctx, LDPC_EINVAL, "null buffer");
  if (cw_stride < ctx->N || cw_stride >= ((int64_t)1 << 40))
    return set_err(ctx, LDPC_EINVAL, "cw_stride must be in [N, 2^40)");
  for (const void *p : {(const void *)d_in, (const void *)d_out_packed, (const void *)d_iters_used_opt,
                        (const void *)d_syn_weight_opt})
    if ((uintptr_t)p >> 48) return set_err(ctx, LDPC_EINVAL, "pointer above 2^48");
  if (ctx->ring_frames - ctx->ring_first_frame + B >= ((int64_t)1 << 31) ||
      ctx->ring_frames + B >= ((int64_t)1 << 47))
    return set_err(ctx, LDPC_EINVAL, "a frame ring session takes < 2^31 frames: end it and begin anew");
  return ring_post_impl(ctx, d_in, cw_stride, B, d_out_packed, d_iters_used_opt, d_syn_weight_opt, 0);
}

int ldpc_ring_wait(ldpc_ctx *ctx, int64_t batch) {
  if (!ctx) return LDPC_EINVAL;
  if (batch < (int64_t)ctx->ring_first || (uint64_t)batch >= ctx->ring_next)
    return set_err(ctx, LDPC_EINVAL, "no such batch in this session");
  return ring_wait_impl(ctx, (uint64_t)batch);
}

int ldpc_ring_end(ldpc_ctx *ctx) {
  if (!ctx) return LDPC_EINVAL;
  if (!ctx->ring_on) return LDPC_OK;
  ctx->ring_on = false;
  const int64_t q = ring_post_impl(ctx, nullptr, 0, 0, nullptr, nullptr, nullptr, 1);
  if (q < 0) return (int)q;
  // work the caller enqueues on its stream from now on follows the launch
  hipError_t e = hipStreamWaitEvent((hipStream_t)ctx->ring_user_stream, ctx->ring_ev, 0);
  if (e != hipSuccess) return hip_err(ctx, e, "frame ring: stream order");
  // the next session's counters, zeroed on the ring's stream once this
  // launch has ended (the caller's stream waits for the launch only)
  if ((e = hipMemsetAsync(ctx->d_ring, 0, kRingDevBytes, ctx->ring_stream)) != hipSuccess)
    return hip_err(ctx, e, "hipMemsetAsync(ring)");
  ctx->ring_clean = true;
  return LDPC_OK;
}

int ldpc_ring_info(const ldpc_ctx *ctx, int *launches_out, int *workgroups_out) {
  if (!ctx) return LDPC_EINVAL;
  if (launches_out) *launches_out = ctx->ring_launches;
  if (workgroups_out) *workgroups_out = ctx->ring_workgroups;
  return LDPC_OK;
}

int ldpc_test_hook(ldpc_ctx *ctx, int op, int64_t arg) {
  if (!ctx) return LDPC_EINVAL;
  switch (op) {
    case LDPC_TEST_SERVE_UNCHECKED:
      ctx->srv_test_skip_check = true;
      return LDPC_OK;
    case LDPC_TEST_SERVE_EPOCH:
      // epochs only grow within a session (a launch serves epochs above its start)
      if (arg < (int64_t)ctx->srv_epoch || arg >= (int64_t)ldpc::kServeEpochLimit)
        return set_err(ctx, LDPC_EINVAL, "epoch must be in [current, kServeEpochLimit)");
      ctx->srv_epoch = (uint32_t)arg;
      return LDPC_OK;
    case LDPC_TEST_SERVE_EPOCH_NOW:
      return (int)ctx->srv_epoch;
    case LDPC_TEST_STREAM_OVERLAP: {
      // streams i = arg >> 8 and j = arg & 255 of the in-flight set: a 0.2 ms
      // spin on each, 1 if the two spins' device-clock intervals intersect
      const size_t i = (size_t)(arg >> 8) & 255u, j = (size_t)arg & 255u;
      if (i >= ctx->tp_streams.size() || j >= ctx->tp_streams.size())
        return set_err(ctx, LDPC_EINVAL, "no such stream in the set");
      hipError_t e;
      if (!ctx->d_probe && (e = hipMalloc((void **)&ctx->d_probe, 256)) != hipSuccess)
        return hip_err(ctx, e, "hipMalloc(probe)");
      uint64_t *st = reinterpret_cast<uint64_t *>(ctx->d_probe) + 8, h[4] = {0, 0, 0, 0};
      if (ldpc::launch_stamp(st, 20000, ctx->tp_streams[i]) != 0 ||
          ldpc::launch_stamp(st + 2, 20000, ctx->tp_streams[j]) != 0 ||
          (e = hipStreamSynchronize(ctx->tp_streams[i])) != hipSuccess ||
          (e = hipStreamSynchronize(ctx->tp_streams[j])) != hipSuccess ||
          (e = hipMemcpy(h, st, sizeof h, hipMemcpyDeviceToHost)) != hipSuccess)
        return set_err(ctx, LDPC_EDEVICE, "stream overlap probe");
      return h[2] < h[1] && h[0] < h[3] ? 1 : 0;
    }
    default:
      return set_err(ctx, LDPC_EINVAL, "unknown test hook");
  }
}

int ldpc_decode_windows(ldpc_ctx *ctx, int method, int max_iters, int et_period, int precision,
                        const float *in, int64_t n_in_floats, int elem_stride, int reuse_span,
                        const int64_t *windows, int B, uint8_t *out_packed,
                        int32_t *syn_weight_opt) {
  return decode_windows_impl(ctx, method, max_iters, et_period, precision, in, n_in_floats,
                             elem_stride, reuse_span, windows, B, out_packed, syn_weight_opt);
}

int ldpc_decode_device(ldpc_ctx *ctx, int method, int max_iters, int et_period, int precision,
                       const float *d_in, int64_t cw_stride, int elem_stride, float polarity,
                       int B, uint8_t *d_out_packed, uint8_t *d_out_bits_opt,
                       int32_t *d_iters_used_opt, int32_t *d_syn_weight_opt,
                       float *d_llr_out_opt, void *hip_stream) {
  return decode_device_impl(ctx, method, max_iters, et_period, precision, d_in, cw_stride,
                            elem_stride, polarity, B, 0, d_out_packed, d_out_bits_opt,
                            d_iters_used_opt, d_syn_weight_opt, d_llr_out_opt, hip_stream);
}

int ldpc_decode_strided(ldpc_ctx *ctx, int method, int max_iters, int et_period, int precision,
                        const float *in, int64_t n_in_floats, int64_t cw_stride, int elem_stride,
                        float polarity, int B, uint8_t *out_packed, uint8_t *out_bits_opt,
                        int32_t *iters_used_opt, int32_t *syn_weight_opt, float *llr_out_opt) {
  return decode_host_impl(ctx, method, max_iters, et_period, precision, in, n_in_floats,
                          cw_stride, elem_stride, polarity, B, false, out_packed, out_bits_opt,
                          iters_used_opt, syn_weight_opt, llr_out_opt);
}

int ldpc_decode_strided_both(ldpc_ctx *ctx, int method, int max_iters, int et_period,
                             int precision, const float *in, int64_t n_in_floats,
                             int64_t cw_stride, int elem_stride, float polarity, int B,
                             uint8_t *out_packed, int32_t *syn_weight_opt) {
  return decode_host_impl(ctx, method, max_iters, et_period, precision, in, n_in_floats,
                          cw_stride, elem_stride, polarity, B, true, out_packed, nullptr,
                          nullptr, syn_weight_opt, nullptr);
}

int ldpc_decode(ldpc_ctx *ctx, int method, int max_iters, int et_period, int precision,
                const float *llr_re, int B, uint8_t *out_packed, uint8_t *out_bits_opt,
                int32_t *iters_used_opt, int32_t *syn_weight_opt) {
  if (!ctx) return LDPC_EINVAL;
  return ldpc_decode_strided(ctx, method, max_iters, et_period, precision, llr_re,
                             (int64_t)B * ctx->N, ctx->N, 1, 1.0f, B, out_packed, out_bits_opt,
                             iters_used_opt, syn_weight_opt, nullptr);
}

int ldpc_ctx_streams(ldpc_ctx *ctx, int n, void **streams_out) {
  if (!ctx || n < 1 || n > 16 || !streams_out)
    return set_err(ctx, LDPC_EINVAL, "n must be in [1, 16] with an output array");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  if (!ctx->d_probe && (e = hipMalloc((void **)&ctx->d_probe, 256)) != hipSuccess)
    return hip_err(ctx, e, "hipMalloc(probe)");
  // Which hardware queue a stream lands on (GPU_MAX_HW_QUEUES of them) depends
  // on every stream the process made before it; two streams on one queue run
  // their launches one after the other.  A candidate joins the set only if a
  // probe pair runs concurrently with every member (both ways round); the
  // others are kept until the set is complete (so the next candidate lands
  // elsewhere), then freed, and the finished set is probed once more.
  // Measured (profiles/round5/inflight_bimodal.txt): a stream's FIRST launch
  // can run beside a launch on a stream that shares its queue, so a probe
  // that is a candidate's first use passed sets whose streams then ran one
  // after the other -- one process in four at 0.72x the in-flight rate.  Every
  // candidate now makes a launch of its own (and waits for it) before it is
  // probed, and a probe waits up to 5 ms.  A new stream lands on the queue
  // fewest streams use, so when the process's streams sit unevenly on its
  // queues (a test process that made dozens) the missing queue is reached
  // only after the others have taken the rejected candidates: up to 16 per
  // wanted stream are tried.
  int rc = LDPC_OK;
  if (ctx->tp_streams.size() < (size_t)n) {
    // the probes should see only each other: the context's own work is waited
    // for (its stream, the frame ring's, the set so far; a window server is
    // ended first) -- not the device: other contexts of the process (other
    // blocks of a flowgraph) keep running.  Their work can hold a probe back
    // past its timeout; the candidate is then rejected and another tried.
    serve_stop(ctx);
    auto own_idle = [&]() {
      hipError_t r = hipStreamSynchronize(ctx->stream);
      if (r == hipSuccess && ctx->ring_stream) r = hipStreamSynchronize(ctx->ring_stream);
      for (hipStream_t t : ctx->tp_streams)
        if (r == hipSuccess) r = hipStreamSynchronize(t);
      return r;
    };
    if ((e = own_idle()) != hipSuccess) return hip_err(ctx, e, "hipStreamSynchronize");
    // total probing is bounded: ~0.5 s, after which the set is what it is
    const auto t_start = std::chrono::steady_clock::now();
    auto over = [&]() {
      return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count() > 0.5;
    };
    auto concurrent = [&](hipStream_t a, hipStream_t c, bool &ok) {
      uint32_t seen = 0;
      if ((e = hipMemset(ctx->d_probe, 0, 8)) != hipSuccess ||
          ldpc::launch_probe_pair(ctx->d_probe, 500000 /* 5 ms */, a, c) != 0 ||
          (e = hipStreamSynchronize(a)) != hipSuccess || (e = hipStreamSynchronize(c)) != hipSuccess ||
          (e = hipMemcpy(&seen, ctx->d_probe + 1, 4, hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_err(ctx, e, "stream probe");
      ok = seen == 1u;
      return LDPC_OK;
    };
    auto both_ways = [&](hipStream_t a, hipStream_t c, bool &ok) {
      int r = concurrent(a, c, ok);
      if (r == LDPC_OK && ok) r = concurrent(c, a, ok);
      return r;
    };
    auto fresh = [&](hipStream_t &c) {
      c = nullptr;
      if ((e = hipStreamCreateWithFlags(&c, hipStreamNonBlocking)) != hipSuccess)
        return hip_err(ctx, e, "hipStreamCreate");
      if (ldpc::launch_probe_touch(ctx->d_probe + 8, c) != 0 ||
          (e = hipStreamSynchronize(c)) != hipSuccess) {
        (void)hipStreamDestroy(c);
        c = nullptr;
        return hip_err(ctx, e, "stream probe");
      }
      return LDPC_OK;
    };
    // members handed out by an earlier call stay (their callers hold them)
    const size_t held = ctx->tp_streams.size();
    for (int attempt = 0; attempt < 3 && rc == LDPC_OK; ++attempt) {
      std::vector<hipStream_t> spare;
      // (more streams than the process has hardware queues cannot all be
      // concurrent: after a few candidates the set's streams are handed out
      // again)
      for (int tries = 0; (int)ctx->tp_streams.size() < n && tries < 16 * n &&
                          (ctx->tp_streams.empty() || !over());
           ++tries) {
        hipStream_t c = nullptr;
        if ((rc = fresh(c)) != LDPC_OK) break;
        bool ok = true;
        for (hipStream_t a : ctx->tp_streams) {
          rc = both_ways(a, c, ok);
          if (rc != LDPC_OK || !ok) break;
        }
        (ok && rc == LDPC_OK ? ctx->tp_streams : spare).push_back(c);
        if (rc != LDPC_OK) break;
      }
      for (hipStream_t t : spare) (void)hipStreamDestroy(t);
      if (rc != LDPC_OK) break;
      // freeing a stream can release its hardware queue, and for a few ms
      // after that probes read concurrent pairs as shared: let it settle
      if ((e = own_idle()) != hipSuccess) return hip_err(ctx, e, "hipStreamSynchronize");
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
      // the finished set, once more; one that fails is made again, and after
      // three tries the last one stays (a set, even a slower one, rather than
      // an error)
      bool all = true;
      for (size_t i = 0; i < ctx->tp_streams.size() && all && rc == LDPC_OK; ++i)
        for (size_t j = i + 1; j < ctx->tp_streams.size() && all && rc == LDPC_OK; ++j)
          rc = both_ways(ctx->tp_streams[i], ctx->tp_streams[j], all);
      if (rc != LDPC_OK || all || attempt == 2 || over()) break;
      for (size_t i = held; i < ctx->tp_streams.size(); ++i) (void)hipStreamDestroy(ctx->tp_streams[i]);
      ctx->tp_streams.resize(held);
    }
    if (rc != LDPC_OK) return rc;
  }
  if (ctx->tp_streams.empty()) return set_err(ctx, LDPC_EDEVICE, "no stream");
  const size_t m = ctx->tp_streams.size();
  for (int i = 0; i < n; ++i) streams_out[i] = (void *)ctx->tp_streams[(size_t)i % m];
  // the distinct streams handed out (the set's concurrent ones, at most n)
  return (int)std::min<size_t>(m, (size_t)n);
}

int ldpc_set_waves_per_cu(ldpc_ctx *ctx, int waves_per_cu) {
  if (!ctx || waves_per_cu < 0 || waves_per_cu > 32)
    return set_err(ctx, LDPC_EINVAL, "waves_per_cu must be in [0, 32]");
  ctx->waves_per_cu = waves_per_cu;
  return LDPC_OK;
}

int ldpc_set_launch_mode(ldpc_ctx *ctx, int mode) {
  if (!ctx || (mode != LDPC_MODE_LATENCY && mode != LDPC_MODE_THROUGHPUT))
    return set_err(ctx, LDPC_EINVAL, "mode must be LDPC_MODE_LATENCY or LDPC_MODE_THROUGHPUT");
  // measured on the config-2 batch (profiles/round2/ab_launch_mode.txt,
  // profiles/round2/layout/): one launch at a time: 12 waves per CU, priority
  // for starved waves; overlapping launches: 4 waves per CU each (4 launches
  // in flight fill the CU's 16 wave slots of the throughput build), no
  // priority games
  ctx->waves_per_cu = mode == LDPC_MODE_THROUGHPUT ? 4 : 0;
  ctx->fair_cycles = mode == LDPC_MODE_THROUGHPUT ? 0 : 1800;
  return LDPC_OK;
}

int ldpc_set_schedule(ldpc_ctx *ctx, int schedule) {
  if (!ctx || schedule < 0 || schedule > 2)
    return set_err(ctx, LDPC_EINVAL, "schedule must be 0 (auto), 1 or 2");
  ctx->schedule = schedule;
  return LDPC_OK;
}

int ldpc_synchronize(ldpc_ctx *ctx) {
  serve_stop(ctx);
  if (!ctx) return LDPC_EINVAL;
  hipError_t e = hipStreamSynchronize(ctx->stream);
  return e == hipSuccess ? LDPC_OK : hip_err(ctx, e, "hipStreamSynchronize");
}

}  // extern "C"
