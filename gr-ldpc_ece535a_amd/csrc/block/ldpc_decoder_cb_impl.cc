/* -*- c++ -*- */
/*
 * LDPC decoder block implementation (MI355X edition).
 *
 * general_work reproduces the control flow of lib/ldpc_decoder_cb_impl.cc:133-234
 * of gr-ldpc_ece535a for any chunking of the input; its outputs equal the
 * reference's as far as the window decodes do (see the end of this comment
 * and DESIGN.md section 3).  The
 * reference loop decodes one window per step -- the N samples at the
 * current position times +-1 -- and its state machine decides the next
 * position.  Here the loop is replayed exactly over a memo of decoded
 * windows; when it reaches a window not decoded yet, a dry run of the same
 * loop goes ahead on guesses and collects every window it touches, and all of
 * them are decoded in ONE round (any positions, either polarity, one staged
 * copy of the input): a round of the call's window server (ldpc_serve_windows:
 * one persistent launch per call, started right behind the span's copy), or
 * one launch (ldpc_decode_windows) for codes and methods the server does not
 * take.  The exact replay then goes on; a wrong guess only means another round.
 *
 * The guesses follow the stream's grid: the phase (mod N) where two frames in
 * a row last passed in sync.  A window on the grid passes, any other fails --
 * a misaligned window passes the M/8 threshold ~1 % of the time.  So after a
 * sync loss the dry run searches one sample at a time up to the next grid
 * position and syncs there; after a false sync on a misaligned window it
 * follows the 11 failing frames (:169-176), the retry and the search back to
 * the grid, instead of decoding the rest of the input on the wrong grid.
 * Frames on the grid are wanted at both polarities, so a sync loss's "-tx"
 * retry (:178-187) is known.  An out-of-sync search that finds nothing within
 * its budget (128 positions) widens x4 per launch.  Measured on one MI355X
 * (profiles/round2/block/block_plans.txt): 4 dB stream 32 -> 75 Mbit/s, 2 dB
 * 11 -> 19 Mbit/s against guessing that every frame in sync passes.
 * A round costs one window's latency plus the host round trip
 * (DESIGN.md section 9), as much as thousands of extra windows.
 *
 * The H is the reference's default (make(method)), or a runtime H (dense,
 * reordered like the reference's constructor; CSR; or an alist file).
 *
 * Decoding is deterministic per window and the replay only ever uses real
 * decode results, so given the window decodes the block emits the same
 * bytes, consumes the same items, prints the same sync messages and leaves
 * the same state as the reference's frame-at-a-time loop.  The window
 * decodes themselves are the reference's arithmetic bit for bit in the
 * default f64 mode (min-sum has no transcendentals;
 * sum-product reproduces glibc's tanh and log -- the __log_fma variant that
 * glibc >= 2.28 selects on FMA-capable x86-64 -- with correctly rounded
 * divisions), so the bytes equal those of the reference built against such a
 * glibc.
 */
#include "ldpc_decoder_cb_impl.h"

#include <gnuradio/io_signature.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstring>
#include <iostream>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace gr {
namespace ldpc_ece535a {

#define STATE_OUT_OF_SYNC 0
#define STATE_IN_SYNC 1
#define STATE_IN_SYNC_INVERTED 2

namespace {
// Per launch at most kWindowSamples samples of windows (1 << 17 windows of
// the reference's N = 64; a DVB-S2-size code gets ~130), which bounds the
// staging memory and the launch for any N; the out-of-sync search starts
// with at most kSearchFirst (128) positions and widens x4 per round.
const int64_t kWindowSamples = (int64_t)64 << 17;
int max_windows(unsigned N) {
  return (int)std::max<int64_t>(16, std::min<int64_t>((int64_t)1 << 17, kWindowSamples / (int64_t)N));
}
const size_t kDenseMax = (size_t)1 << 22;  // alist codes up to M N entries go dense

void print_method(int method) {
  if (method == 3)
    std::cout << "Method: Hard" << std::endl;
  else if (method == 2)
    std::cout << "Method: BitFlip" << std::endl;
  else if (method == 1)
    std::cout << "Method: SumProduct" << std::endl;
  else
    std::cout << "Method: LogDomain" << std::endl;
}
}  // namespace

ldpc_decoder_cb::sptr ldpc_decoder_cb::make(const int method) {
  return gnuradio::get_initial_sptr(new ldpc_decoder_cb_impl(method, 5, LDPC_PREC_F64, 0));
}

ldpc_decoder_cb::sptr ldpc_decoder_cb::make(const int method, const int iterations,
                                            const int precision) {
  return gnuradio::get_initial_sptr(
      new ldpc_decoder_cb_impl(method, iterations, precision, 0));
}

ldpc_decoder_cb::sptr ldpc_decoder_cb::make(const int method, const int iterations,
                                            const int precision,
                                            const std::vector<unsigned char> &H, const int M,
                                            const int N) {
  if (M <= 0 || N <= 0 || H.size() != (size_t)M * (size_t)N)
    throw std::invalid_argument("ldpc_decoder_cb: H must hold M x N entries");
  return gnuradio::get_initial_sptr(
      new ldpc_decoder_cb_impl(method, iterations, precision, 0, H.data(), M, N, 0));
}

ldpc_decoder_cb::sptr ldpc_decoder_cb::make(const int method, const int iterations,
                                            const int precision, const std::string &alist_path) {
  return gnuradio::get_initial_sptr(
      new ldpc_decoder_cb_impl(method, iterations, precision, 0, alist_path));
}

#define LDPC_BLOCK_INIT(method, iterations, precision)                                  \
  gr::block("ldpc_decoder_cb", gr::io_signature::make(1, 1, sizeof(gr_complex)),       \
            gr::io_signature::make(1, 1, sizeof(unsigned char))),                      \
      d_method(method), d_state(STATE_OUT_OF_SYNC), d_M(32), d_N(64),                  \
      d_iterations(iterations), d_errors(0), d_out_bytes(4), d_precision(precision),    \
      d_ctx(nullptr), d_backend(nullptr), d_backend_user(nullptr), d_frames_decoded(0)

ldpc_decoder_cb_impl::ldpc_decoder_cb_impl(int method, int iterations, int precision,
                                           int device, const uint8_t *H, int M, int N,
                                           int flags)
    : LDPC_BLOCK_INIT(method, iterations, precision) {
  ldpc_ctx *ctx;
  if (!H) {
    // The reference's hard-coded 32x64 matrix (:60-102), column-reordered by
    // reorderHMatrix (:104-106) inside ldpc_create.
    uint8_t Hd[32 * 64];
    ldpc_default_h(Hd);
    ctx = ldpc_create(Hd, 32, 64, flags, device);
  } else {
    ctx = ldpc_create(H, M, N, flags, device);
  }
  adopt(ctx);
  print_method(d_method);
}

ldpc_decoder_cb_impl::ldpc_decoder_cb_impl(int method, int iterations, int precision,
                                           int device, int M, int N, const int32_t *row_ptr,
                                           const int32_t *col_idx, int flags)
    : LDPC_BLOCK_INIT(method, iterations, precision) {
  adopt(ldpc_create_csr(M, N, row_ptr, col_idx, flags, device));
  print_method(d_method);
}

ldpc_decoder_cb_impl::ldpc_decoder_cb_impl(int method, int iterations, int precision,
                                           int device, const std::string &alist_path)
    : LDPC_BLOCK_INIT(method, iterations, precision) {
  int M = 0, N = 0;
  const int E = ldpc_alist_read(alist_path.c_str(), &M, &N, nullptr, nullptr, 0);
  if (E < 0) throw std::runtime_error(std::string("ldpc_decoder_cb: ") + ldpc_last_error(nullptr));
  std::vector<int32_t> rp((size_t)M + 1), ci((size_t)std::max(E, 1));
  if (ldpc_alist_read(alist_path.c_str(), &M, &N, rp.data(), ci.data(), E) < 0)
    throw std::runtime_error(std::string("ldpc_decoder_cb: ") + ldpc_last_error(nullptr));
  ldpc_ctx *ctx;
  if ((size_t)M * (size_t)N <= kDenseMax) {  // as the reference treats its H: reordered
    std::vector<uint8_t> H((size_t)M * N, 0);
    for (int j = 0; j < M; ++j)
      for (int32_t e = rp[j]; e < rp[j + 1]; ++e) H[(size_t)j * N + ci[e]] = 1;
    ctx = ldpc_create(H.data(), M, N, 0, device);
  } else {
    ctx = ldpc_create_csr(M, N, rp.data(), ci.data(), 0, device);
  }
  adopt(ctx);
  print_method(d_method);
}

void ldpc_decoder_cb_impl::adopt(ldpc_ctx *ctx) {
  if (!ctx) throw std::runtime_error(std::string("ldpc_decoder_cb: ") + ldpc_last_error(nullptr));
  int M = 0, N = 0, K = 0;
  ldpc_ctx_info(ctx, &M, &N, nullptr, &K, nullptr, nullptr, nullptr);
  // :141 emits M/8 bytes of bits M.. per frame: they must exist
  if (K < 8 * (M / 8)) {
    ldpc_destroy(ctx);
    throw std::invalid_argument(
        "ldpc_decoder_cb: the block emits M/8 bytes of information bits per frame "
        "(lib/ldpc_decoder_cb_impl.cc:141, :209-219); this H has N - M < 8 (M/8)");
  }
  d_ctx = ctx;
  d_M = (unsigned)M;
  d_N = (unsigned)N;
  d_out_bytes = M / 8;
  // the window server: load its kernel now with one round of one window of
  // zeros (a kernel's first launch costs milliseconds); codes or methods it
  // does not take keep a launch per round
  if (d_serve && (d_method == 0 || d_method == 1)) {
    std::vector<float> z((size_t)2 * N, 0.0f);
    int rc = ldpc_stage_span(ctx, z.data(), 2 * (int64_t)N, 2, 1);
    if (rc == LDPC_OK) rc = ldpc_serve_begin(ctx, d_method, (int)d_iterations, d_precision, 1);
    if (rc == LDPC_OK) {
      const int64_t key = 0;
      std::vector<uint8_t> pk((size_t)std::max(1, (N - M + 7) / 8));
      int32_t sy = 0;
      rc = ldpc_serve_windows(ctx, &key, 1, pk.data(), &sy);
      (void)ldpc_serve_end(ctx);
    }
    if (rc == LDPC_EUNSUPPORTED) d_serve = false;
    else if (rc < 0) {
      const std::string why = ldpc_last_error(ctx);
      ldpc_destroy(ctx);
      d_ctx = nullptr;
      throw std::runtime_error("ldpc_decoder_cb: window server: " + why);
    }
  } else {
    d_serve = false;
  }
}

ldpc_decoder_cb_impl::ldpc_decoder_cb_impl(int method, int iterations, ldpc_block_backend_fn fn,
                                           void *user)
    : LDPC_BLOCK_INIT(method, iterations, LDPC_PREC_F64) {
  if (!fn) throw std::runtime_error("ldpc_decoder_cb: null backend");
  d_backend = fn;
  d_backend_user = user;
}

int ldpc_decoder_cb_impl::Stager::run() {
  return ldpc_stage_span(ctx, in, n, 2, max_windows);
}

void ldpc_decoder_cb_impl::stage_async(const float *in, int64_t n_floats, int max_windows) {
  Stager &sg = d_stager;
  if (!sg.th.joinable())
    sg.th = std::thread([&sg]() {
      std::unique_lock<std::mutex> lk(sg.mu);
      for (;;) {
        sg.cv.wait(lk, [&sg]() { return sg.busy || sg.quit; });
        if (sg.quit) return;
        lk.unlock();
        const int rc = sg.run();
        lk.lock();
        sg.rc = rc;
        sg.busy = false;
        sg.cv.notify_all();
      }
    });
  std::lock_guard<std::mutex> lk(sg.mu);
  sg.ctx = d_ctx;
  sg.in = in;
  sg.n = n_floats;
  sg.max_windows = max_windows;
  sg.busy = true;
  sg.cv.notify_all();
}

int ldpc_decoder_cb_impl::stage_wait() {
  Stager &sg = d_stager;
  {
    std::unique_lock<std::mutex> lk(sg.mu);
    sg.cv.wait(lk, [&sg]() { return !sg.busy; });
  }
  return sg.rc;
}

ldpc_decoder_cb_impl::~ldpc_decoder_cb_impl() {
  if (d_stager.th.joinable()) {
    {
      std::lock_guard<std::mutex> lk(d_stager.mu);
      d_stager.quit = true;
      d_stager.cv.notify_all();
    }
    d_stager.th.join();
  }
  if (d_profile)
    fprintf(stderr,
            "ldpc_decoder_cb profile: %lld rounds; general_work %.3f ms = exact replay %.3f + "
            "dry runs %.3f + staging wait %.3f + first rounds %.3f + other rounds %.3f + rest\n",
            (long long)d_launches, 1e3 * d_prof[0], 1e3 * d_prof[1], 1e3 * d_prof[2],
            1e3 * d_prof[3], 1e3 * d_prof[4], 1e3 * d_prof[5]);
  ldpc_destroy(d_ctx);
}

double ldpc_decoder_cb_impl::now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void ldpc_decoder_cb_impl::forecast(int noutput_items, gr_vector_int &ninput_items_required) {
  ninput_items_required[0] = noutput_items * d_N;
}

void ldpc_decoder_cb_impl::decode_wanted(const float *in, int nin, bool first, bool first_round) {
  const int KB = (int)(d_N - d_M + 7) / 8;
  const int B = (int)d_want.size();
  // results land straight at the end of the memo's result arrays
  const size_t base = d_rsynd.size();
  d_rsynd.resize(base + B);
  d_rpacked.resize((base + B) * KB);
  int32_t *synd = d_rsynd.data() + base;
  uint8_t *packed = d_rpacked.data() + base * KB;
  if (d_backend) {
    // the test seam decodes equally spaced windows of one polarity per call
    for (int i = 0; i < B;) {
      const int64_t p0 = d_want[i] >> 1, pol = d_want[i] & 1;
      int j = i + 1;
      int64_t step = 0;
      if (j < B && (d_want[j] & 1) == pol && (d_want[j] >> 1) > p0) {
        step = (d_want[j] >> 1) - p0;
        while (j < B && (d_want[j] & 1) == pol && (d_want[j] >> 1) - (d_want[j - 1] >> 1) == step)
          ++j;
      }
      const int n = j - i;
      const int rc = d_backend(d_backend_user, in + 2 * p0, 2 * ((int64_t)nin - p0),
                               2 * std::max<int64_t>(step, 1), 2, pol ? -1.0f : 1.0f, n,
                               packed + (size_t)i * KB, synd + i);
      if (rc < 0) throw std::runtime_error("ldpc_decoder_cb: decode failed: backend error");
      i = j;
    }
  } else {
    const bool small = d_serve && (int64_t)B * d_iterations <= kServeWork;
    if (small && !d_serving) serve_start();
    if (small && d_serving) {
      const int rc = ldpc_serve_windows(d_ctx, d_want.data(), B, packed, synd);
      if (rc < 0)
        throw std::runtime_error(std::string("ldpc_decoder_cb: decode failed: ") +
                                 ldpc_last_error(d_ctx));
    } else {
      d_serving = false;  // (ldpc_decode_windows ends a running server first)
      const int rc = ldpc_decode_windows(d_ctx, d_method, (int)d_iterations, 1, d_precision, in,
                                         2 * (int64_t)nin, 2, first ? 0 : 1, d_want.data(), B,
                                         packed, synd);
      if (rc < 0)
        throw std::runtime_error(std::string("ldpc_decoder_cb: decode failed: ") +
                                 ldpc_last_error(d_ctx));
      // after a call's first round (the grid, usually big) the rounds are
      // mostly small: the server's launch goes behind this one now and starts
      // while the next round is planned; later, a small round starts it
      if (d_serve && d_serve_mode == 2 && first_round) serve_start();
    }
  }
  for (int b = 0; b < B; ++b) d_memo[(size_t)d_want[b]] = (int32_t)(base + b);
  d_touched.insert(d_touched.end(), d_want.begin(), d_want.end());
  d_frames_decoded += B;
  d_launches += 1;
}

void ldpc_decoder_cb_impl::serve_start() {
  const int rc = ldpc_serve_begin(d_ctx, d_method, (int)d_iterations, d_precision, max_windows(d_N));
  if (rc == LDPC_OK)
    d_serving = true;
  else if (rc == LDPC_EUNSUPPORTED)
    d_serve = false;  // this code / method: launches
  else
    throw std::runtime_error(std::string("ldpc_decoder_cb: window server: ") + ldpc_last_error(d_ctx));
}

void ldpc_decoder_cb_impl::want(int64_t pos, int pol, int nin) {
  if (pos < 0 || pos + (int64_t)d_N > nin || d_want.size() >= (size_t)max_windows(d_N)) return;
  int32_t &m = d_memo[mi(pos, pol)];
  if (m == -1) {
    m = -2;  // pending: wanted by this launch
    d_want.push_back((pos << 1) | pol);
  }
}

int ldpc_decoder_cb_impl::pass_run(int pol, int pos, int nin) {
  // frames pos, pos + N, ... that are decoded at `pol` and pass (:166-168);
  // d_skip jumps over runs found before (memo entries are not removed within
  // a call, so a run stays a run), and the path is compressed to its end
  const int N = (int)d_N, thr = (int)d_M / 8;
  int32_t *skip = d_skip[pol].data();
  int p = pos;
  while (p + N <= nin) {
    const int64_t s = slot(p);
    const int32_t u = d_memo[mi(p, pol)];
    if (u < 0 || d_rsynd[u] > thr) break;
    p = skip[s] > p ? skip[s] : p + N;
  }
  for (int q = pos; q < p;) {
    const int64_t s = slot(q);
    const int nx = skip[s] > q ? skip[s] : q + N;
    if (skip[s] == 0) d_skip_touched.push_back(((int64_t)q << 1) | pol);
    skip[s] = p;
    q = nx;
  }
  return (p - pos) / N;
}

ldpc_decoder_cb_impl::Outcome ldpc_decoder_cb_impl::replay(Replay &r, bool exact, int nin,
                                                           int noutput, unsigned char *out,
                                                           int max_out, size_t max_want) {
  const int N = (int)d_N;
  const int mo = d_out_bytes;                      // :141 (M/8)
  const int thr = (int)d_M / 8;                    // :142
  const int KB = (N - (int)d_M + 7) / 8;
  int out_run = 0;  // dry run: out-of-sync positions in a row with a guessed window
  int searches = 0;  // dry run: runs of such positions so far
  while ((nin - r.consumed) >= N && (noutput - r.produced) >= mo) {  // :146-147
    const int pos = r.consumed;
    const int pol = r.state == STATE_IN_SYNC_INVERTED ? 1 : 0;  // tx = Re * -1 (:149-153)
    if (r.state != STATE_OUT_OF_SYNC) {
      // frames in sync that are decoded and pass change nothing but the
      // position and the output (:207-225): take the whole run at once
      const int k = std::min(pass_run(pol, pos, nin), (noutput - r.produced) / mo);
      if (k > 0) {
        if (exact) {
          d_grid_frames += k;
          for (int i = 0; i < k; ++i)
            std::memcpy(out + r.produced + (size_t)i * mo,
                        &d_rpacked[(size_t)d_memo[mi(pos + i * N, pol)] * KB], (size_t)mo);
          // two frames in a row pass in sync: their grid is the stream's
          if (k > 1 || d_last_pass == d_abs + pos - N) d_anchor = (int)((d_abs + pos) % N);
          d_last_pass = d_abs + pos + (int64_t)(k - 1) * N;
        }
        r.consumed += k * N;
        r.produced += k * mo;
        out_run = 0;
        continue;
      }
      if (!exact && (d_anchor < 0 || (d_abs + pos) % N == d_anchor)) {
        // dry run, in sync on the grid, windows not decoded yet: each is
        // guessed to pass (the general step below), so the run of them goes
        // in one tight loop -- the same wants in the same order, the same
        // position -- up to the first decoded window or one known to pass at
        // the other polarity (those take the general step)
        const bool both = grid_fails_often();
        const size_t maxw = (size_t)max_windows(d_N);
        int32_t *mm = d_memo.data();
        int p = pos, prod = r.produced;
        while (nin - p >= N && noutput - prod >= mo && d_want.size() < max_want) {
          int32_t *m0 = mm + mi(p, pol), *m1 = mm + mi(p, pol ^ 1);
          if (*m0 >= 0) break;
          const int32_t o = *m1;
          if (o >= 0 && d_rsynd[o] <= thr) break;
          if (*m0 == -1 && d_want.size() < maxw) {
            *m0 = -2;
            d_want.push_back(((int64_t)p << 1) | pol);
          }
          if (both && o == -1 && d_want.size() < maxw) {
            *m1 = -2;
            d_want.push_back(((int64_t)p << 1) | (pol ^ 1));
          }
          p += N;
          prod += mo;
        }
        if (p > pos) {
          r.consumed = p;
          r.produced = prod;
          out_run = 0;
          if (d_want.size() >= max_want) return STALLED;
          continue;
        }
      }
    }
    Replay n = r;
    bool guessed_out = false, lost = false, inverted = false, synced = false;
    // checkFrame(vhat, M/8) > M/8 (:166-168); it stops counting past the
    // threshold, so comparing the full weight gives the same decision
    int32_t use = d_memo[mi(pos, pol)];
    // the dry run's guess: a window on the grid the stream was last seen in
    // sync on passes, any other fails (a misaligned window passes ~1 % of the
    // time); with no grid seen yet, frames in sync pass
    bool pass;
    if (use >= 0) {
      pass = d_rsynd[use] <= thr;
    } else {
      if (exact) return STALLED;
      want(pos, pol, nin);
      const bool on_grid = d_anchor < 0 || (d_abs + pos) % N == d_anchor;
      pass = on_grid && (r.state != STATE_OUT_OF_SYNC || d_anchor >= 0);
      // the same samples known to pass at the other polarity: this one fails
      // (the complement of a codeword leaves every odd-weight row unsatisfied:
      // 20 of the default H's 32)
      if (pass) {
        const int32_t o = d_memo[mi(pos, pol ^ 1)];
        if (o >= 0 && d_rsynd[o] <= thr) pass = false;
      }
      guessed_out = !pass;
      // a frame in sync is also wanted at the other polarity when its result
      // decides a sync loss's "-tx" retry (:178-187)
      if (pass && grid_fails_often())
        want(pos, pol ^ 1, nin);
    }
    if (exact && pass && r.state != STATE_OUT_OF_SYNC) {
      // two frames in a row pass in sync: their grid is the stream's (a
      // misaligned pair passes ~1e-4 of the time)
      if (d_last_pass == d_abs + pos - N) d_anchor = (int)((d_abs + pos) % N);
      d_last_pass = d_abs + pos;
    }
    if (exact && r.state != STATE_OUT_OF_SYNC) {  // the grid's failure rate, decayed
      d_grid_frames += 1;
      d_grid_fails += pass ? 0 : 1;
      if (d_grid_frames > 4096) {
        d_grid_frames *= 0.5;
        d_grid_fails *= 0.5;
      }
    }
    if (!pass) {
      if (n.state != STATE_OUT_OF_SYNC) {  // :169-176
        n.errors++;
        if (n.errors > 10) {
          n.errors = 0;
          n.state = STATE_OUT_OF_SYNC;
          lost = true;
        }
      }
      if (n.state == STATE_OUT_OF_SYNC) {  // the "-tx" retry, :178-198
        const int32_t i2 = d_memo[mi(pos, pol ^ 1)];
        bool pass2 = false;
        if (i2 >= 0) {
          pass2 = d_rsynd[i2] <= thr;
        } else {
          if (exact) return STALLED;
          want(pos, pol ^ 1, nin);
          guessed_out = true;  // a retry that fails mostly
        }
        if (pass2) {
          n.state = STATE_IN_SYNC_INVERTED;
          n.errors = 0;
          use = i2;
          inverted = true;
        } else {
          n.consumed += 1;  // skip one sample (:193-197)
        }
      }
    } else if (n.state == STATE_OUT_OF_SYNC) {  // :201-205
      n.state = STATE_IN_SYNC;
      n.errors = 0;
      synced = true;
    }
    if (n.state == STATE_IN_SYNC || n.state == STATE_IN_SYNC_INVERTED) {  // :207-225
      if (exact) std::memcpy(out + n.produced, &d_rpacked[(size_t)use * KB], (size_t)mo);
      n.consumed += N;
      n.produced += mo;
    }
    if (exact) {
      // the reference's messages (:174, :190, :202); flushed once per call
      // (general_work's end), not per line: a flush is a write syscall
      if (lost) std::cout << "MAX ERRORS; OUT OF SYNC\n";
      if (inverted) std::cout << "IN SYNC; PHASE INVERTED\n";
      if (synced) std::cout << "IN SYNC\n";
    }
    if (!exact && d_searches_now > 0 && guessed_out && n.state == STATE_OUT_OF_SYNC &&
        out_run == 0 && searches++ >= d_searches_now)
      return STALLED;  // a later search: the first one likely syncs off the grid first
    r = n;
    if (!exact) {
      out_run = (guessed_out && r.state == STATE_OUT_OF_SYNC) ? out_run + 1 : 0;
      if (out_run >= max_out || d_want.size() >= max_want) return STALLED;
    }
  }
  return DONE;
}

int ldpc_decoder_cb_impl::general_work(int noutput_items, gr_vector_int &ninput_items,
                                       gr_vector_const_void_star &input_items,
                                       gr_vector_void_star &output_items) {
  const double t_call = d_profile ? now_s() : 0.0;
  const float *in = (const float *)input_items[0];  // interleaved re/im
  unsigned char *out = (unsigned char *)output_items[0];
  const int N = (int)d_N;
  const int nin = ninput_items[0];
  const size_t npos = (size_t)std::max(nin - N + 1, 0);
  // the memo and the jump table keep their size between calls: only the
  // entries the last call set go back to "not decoded" (a full reset was
  // 2 x 4 bytes per input sample per call)
  for (int64_t key : d_touched) d_memo[(size_t)key] = -1;
  for (int64_t key : d_skip_touched) d_skip[key & 1][slot(key >> 1)] = 0;
  d_touched.clear();
  d_skip_touched.clear();
  // every entry is clean again; grow the grid-major tables if this call's
  // positions need more rows (a larger layout moves every slot)
  const int64_t rows = (int64_t)npos / N + 2;
  if (rows > d_rows) {
    d_rows = std::max(rows, 2 * d_rows);
    d_nshift = -1;
    for (int sh = 0; sh < 31; ++sh)
      if ((1 << sh) == N) d_nshift = sh;
    d_memo.assign((size_t)2 * N * (size_t)d_rows, -1);
    for (int pl = 0; pl < 2; ++pl) d_skip[pl].assign((size_t)N * (size_t)d_rows, 0);
  }
  d_rsynd.clear();
  d_rpacked.clear();

  Replay r{d_state, d_errors, 0, 0};
  // the span goes to the device while the first dry run plans (every launch
  // of this call then reuses it)
  // (the worker reads `in`: it is joined on every way out of this call)
  struct StageJoin {
    ldpc_decoder_cb_impl *self;
    bool pending = false;
    void operator()() {
      if (pending) {
        pending = false;
        if (self->stage_wait() < 0)
          throw std::runtime_error(std::string("ldpc_decoder_cb: staging failed: ") +
                                   ldpc_last_error(self->d_ctx));
      }
    }
    ~StageJoin() {
      if (pending) self->stage_wait();
    }
  } join_stage{this};
  bool staged = false;
  if (!d_backend && nin >= N && noutput_items >= d_out_bytes) {
    stage_async(in, 2 * (int64_t)nin, max_windows(d_N));
    staged = join_stage.pending = true;
  }
  const int search_first = std::min(kSearchFirst, max_windows(d_N));
  int out_budget = search_first;  // out-of-sync positions one launch may guess past
  bool first = true, last_out = false;
  double t0 = d_profile ? now_s() : 0.0;
  while (replay(r, true, nin, noutput_items, out, 0, 0) == STALLED) {
    if (d_profile) d_prof[1] += now_s() - t0;
    // the loop needs a window not decoded yet: dry-run ahead from here to
    // collect the windows it will probably need, and decode them at once
    const bool now_out = r.state == STATE_OUT_OF_SYNC;
    if (now_out && last_out)
      out_budget = std::min(4 * out_budget, max_windows(d_N));  // the search goes on: wider
    else if (!now_out)
      out_budget = search_first;
    last_out = now_out;
    d_want.clear();
    Replay dry = r;
    if (d_profile) t0 = now_s();
    // how many windows one dry run may collect: a launch of up to ~1024
    // 50-iteration windows costs one window's latency, larger ones more
    // (profiles/round3/window_latency_schedules.txt), so while the grid
    // rarely fails (the high-SNR regime, few windows per sync loss) a dry run
    // stops there; with many grid failures (low SNR) the launches stay whole
    // (profiles/round3/block_plans_maxwant.txt: +7 % at 4 dB, -27 % at 2 dB
    // for a fixed cap)
    int cap = max_windows(d_N);
    if (d_max_want > 0)
      cap = std::min(d_max_want, cap);
    else if (d_max_want == 0 && d_iterations >= 20 && 8 * d_grid_fails <= d_grid_frames)
      cap = std::min(1024, cap);
    d_searches_now = d_searches >= 0 ? d_searches
                                     : (d_iterations <= 10 && !grid_fails_often() ? 4 : 0);
    replay(dry, false, nin, noutput_items, nullptr, out_budget, (size_t)cap);
    if (d_debug)
      std::cerr << "ldpc_decoder_cb: stall at " << r.consumed << " state " << r.state
                << " errors " << r.errors << " grid " << d_anchor << ": launch " << d_want.size()
                << " windows, dry run to " << dry.consumed << " state " << dry.state << std::endl;
    if (d_debug == 2) {  // what the round holds
      int64_t on_grid[2] = {0, 0}, off_grid[2] = {0, 0}, lo = INT64_MAX, hi = -1;
      for (int64_t w : d_want) {
        const int64_t p = w >> 1;
        ((d_anchor >= 0 && (d_abs + p) % (int64_t)d_N == d_anchor) ? on_grid : off_grid)[w & 1]++;
        lo = std::min(lo, p);
        hi = std::max(hi, p);
      }
      std::cerr << "  on grid " << on_grid[0] << "+" << on_grid[1] << " off grid " << off_grid[0]
                << "+" << off_grid[1] << " positions " << lo << ".." << hi << std::endl;
    }
    if (d_profile) {
      const double t1 = now_s();
      d_prof[2] += t1 - t0;
      t0 = t1;
    }
    join_stage();  // the span is on its way to the device before the launch
    if (d_profile) {
      const double t1 = now_s();
      d_prof[3] += t1 - t0;
      t0 = t1;
    }
    decode_wanted(in, nin, first && !staged, first);
    if (d_profile) {
      const double t1 = now_s();
      d_prof[first ? 4 : 5] += t1 - t0;
      t0 = t1;
    }
    first = false;
  }
  if (d_profile) {
    d_prof[1] += now_s() - t0;
    d_prof[0] += now_s() - t_call;
    if (d_profile_calls) {  // a line per call
      static double last[6] = {0, 0, 0, 0, 0, 0};
      fprintf(stderr,
              "general_work call: %.1f us = replay %.1f + dry runs %.1f + staging wait %.1f + "
              "first round %.1f + other rounds %.1f\n",
              1e6 * (d_prof[0] - last[0]), 1e6 * (d_prof[1] - last[1]),
              1e6 * (d_prof[2] - last[2]), 1e6 * (d_prof[3] - last[3]),
              1e6 * (d_prof[4] - last[4]), 1e6 * (d_prof[5] - last[5]));
      for (int i = 0; i < 6; ++i) last[i] = d_prof[i];
    }
  }
  std::cout.flush();
  join_stage();  // no launch this call: the staging must still finish
  if (d_serving) {  // the call's window server may finish (no wait)
    d_serving = false;
    (void)ldpc_serve_end(d_ctx);
  }
  d_state = r.state;
  d_errors = r.errors;
  d_abs += r.consumed;
  consume_each(r.consumed);
  return r.produced;
}

}  // namespace ldpc_ece535a
}  // namespace gr
