/* -*- c++ -*- */
/*
 * LDPC decoder block implementation (MI355X edition).
 *
 * Keeps the reference's block contract (lib/ldpc_decoder_cb_impl.h:22-66):
 * 64 gr_complex in -> 4 bytes out per frame, methods 0..3, the frame-sync /
 * polarity state machine.  What changes is how frames are decoded: instead
 * of one CPU decode per 64-sample window, general_work predicts the windows
 * the reference loop will decode, decodes them in one GPU launch and replays
 * the reference's state machine over the results (see ldpc_decoder_cb_impl.cc).
 */
#ifndef INCLUDED_LDPC_ECE535A_LDPC_DECODER_CB_IMPL_H
#define INCLUDED_LDPC_ECE535A_LDPC_DECODER_CB_IMPL_H

#include <ldpc_block.h>
#include <ldpc_ece535a/ldpc_decoder_cb.h>
#include <ldpc_hip.h>

#include <stdlib.h>

#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace gr {
namespace ldpc_ece535a {

class ldpc_decoder_cb_impl : public ldpc_decoder_cb {
 private:
  int d_method;
  int d_state;
  unsigned int d_M;
  unsigned int d_N;
  unsigned int d_iterations;
  unsigned int d_errors;
  int d_out_bytes;               // per frame: M/8 (:141)
  int d_precision;
  ldpc_ctx *d_ctx;               // GPU context (the block's H, reordered)
  ldpc_block_backend_fn d_backend;  // test seam; null = GPU
  void *d_backend_user;
  int64_t d_frames_decoded;
  int64_t d_launches = 0;
  // A worker thread stages each call's span (ldpc_stage_span: the real parts
  // copied into pinned memory and sent to the device) while general_work
  // plans its first round, and then starts the call's window server
  // (ldpc_serve_begin: one persistent launch serves every round of the call)
  // right behind the span's copy in the context's stream; joined before the
  // first round.
  struct Stager {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    bool busy = false, quit = false;
    int rc = 0;
    ldpc_ctx *ctx = nullptr;
    const float *in = nullptr;
    int64_t n = 0;
    int max_windows = 0;
    int run();                   // stages the span; returns ldpc_stage_span's result
  } d_stager;
  // How a round of windows is decoded: through the window server
  // (ldpc_serve_*: one persistent launch serves the call's rounds) or by a
  // launch of its own (ldpc_decode_windows).  The server answers a small
  // round sooner; a big one (windows x iterations above kServeWork) runs
  // faster as a launch, with the batch kernels' full throughput
  // (profiles/round5/serve_latency*.txt).  LDPC_BLOCK_SERVE=0: launches only
  // (the A/B of the server); default: by round size.  (The server for every
  // round, =1 until round 6, was slower in every regime measured.)  Codes or
  // methods the server does not take: launches.
  int d_serve_mode = getenv("LDPC_BLOCK_SERVE") && getenv("LDPC_BLOCK_SERVE")[0] == '0' ? 0 : 2;
  // windows x iterations of the biggest round the server takes: the
  // crossovers measured at ~700 windows of 5 iterations and ~150 of 50
  // (profiles/round5/serve_latency.txt)
  static const int64_t kServeWork = 4096;
  bool d_serve = d_serve_mode != 0;  // the server takes this code and method (until it says otherwise)
  bool d_serving = false;  // a server is running for this call
  void serve_start();
  void stage_async(const float *in, int64_t n_floats, int max_windows);
  int stage_wait();
  // LDPC_BLOCK_DEBUG: one line per round on stderr (=2: also what it holds);
  // read once, when the block is made
  int d_debug = !getenv("LDPC_BLOCK_DEBUG") ? 0 : getenv("LDPC_BLOCK_DEBUG")[0] == '2' ? 2 : 1;
  // LDPC_BLOCK_PROFILE: host time split of general_work, printed when destroyed
  // (=2: also a line per call)
  bool d_profile = getenv("LDPC_BLOCK_PROFILE") != nullptr;
  bool d_profile_calls = d_profile && getenv("LDPC_BLOCK_PROFILE")[0] == '2';
  // total, exact replay, dry runs, waiting for the span's staging, the
  // call's first round, the other rounds
  double d_prof[6] = {0, 0, 0, 0, 0, 0};
  static double now_s();
  // In-sync frames guessed to pass are also wanted at the other polarity
  // when more than 1 in 4 frames on the grid fail (then sync losses, and
  // their "-tx" retries, are frequent; the reference's 4 dB stream fails 1 in
  // 4..8, 2 dB more than 1 in 2).  (1 in 8 requested every grid frame twice at
  // 4 dB / 5 iterations: 9.1 windows per output frame.)
  bool grid_fails_often() const { return 4 * d_grid_fails > d_grid_frames; }
  double d_grid_frames = 0, d_grid_fails = 0;  // decayed counts of in-sync frames
  // A/B knob: LDPC_BLOCK_SEARCHES=k stops a dry run at its (k+1)-th guessed
  // search (0: no limit).  Each search passes a misaligned window somewhere
  // with high probability (~1 % per window, ~126 windows) and the searches
  // after such a false sync move, yet a limit of 1 or 2 costs more rounds
  // than the windows it saves (tools/block_policy_sim.py)
  // Default (unset): 4 for short windows (iterations <= 10) while the grid
  // rarely fails, no limit otherwise: at 4 dB / 5 iterations 26 launches of
  // 3.7 windows per output frame beat 14 of 9.1 (128 vs 119 and
  // 123 vs 117.5 Mbit/s on two boxes, profiles/round4/block/ab_spec_searches.txt); where a round costs a
  // 50-iteration window's latency, or searches are frequent, the extra
  // rounds cost more than the windows they save
  int d_searches = getenv("LDPC_BLOCK_SEARCHES") ? atoi(getenv("LDPC_BLOCK_SEARCHES")) : -1;
  int d_searches_now = 0;  // this dry run's limit
  // out-of-sync positions a dry run may guess past in a row before the round
  // (x4 per round while the search goes on)
  static const int kSearchFirst = 128;
  // A/B knob: LDPC_BLOCK_MAXWANT=n stops a dry run once it has collected n
  // windows; -1: the round limit, max_windows(N), always; 0 (default): 1024
  // while grid frames rarely fail, else the round limit
  int d_max_want = getenv("LDPC_BLOCK_MAXWANT") ? atoi(getenv("LDPC_BLOCK_MAXWANT")) : 0;
  // grid: absolute sample index of the call's first input item; the phase
  // (mod N) of the last two consecutive frames that passed in sync (-1: none yet)
  int64_t d_abs = 0;
  int d_anchor = -1;
  int64_t d_last_pass = -1;  // absolute position of the last window passing in sync

  // general_work's decode memo for the current call: the result of window
  // (position p, polarity) -- p in samples from the call's first input item,
  // polarity 0 = +tx, 1 = -tx -- is entry d_memo[mi(p, pol)] = d_memo[key] of
  // d_rsynd / d_rpacked (-1: not decoded, -2: wanted by the round being
  // planned), key = (p << 1) | pol: position-major, both polarities of a
  // position side by side, as the out-of-sync search reads them
  std::vector<int32_t> d_memo;
  static size_t mi(int64_t p, int pol) { return (size_t)((p << 1) | pol); }
  std::vector<int32_t> d_rsynd;
  // d_skip[pol][slot(p)] > p: frames p, p + N, ... before it are decoded and
  // pass.  Stored grid-major -- position p at (p mod N) * d_rows + p / N -- so
  // a run of frames on one grid reads consecutive words instead of one word
  // every N
  std::vector<int32_t> d_skip[2];
  int64_t d_rows = 0;
  int d_nshift = -1;  // log2(N) when N is a power of two
  int64_t slot(int64_t p) const {
    return d_nshift >= 0 ? (p & (((int64_t)1 << d_nshift) - 1)) * d_rows + (p >> d_nshift)
                         : (p % (int64_t)d_N) * d_rows + p / (int64_t)d_N;
  }
  // keys whose memo / jump entries this call set (reset at the next call)
  std::vector<int64_t> d_touched, d_skip_touched;
  std::vector<uint8_t> d_rpacked;
  std::vector<int64_t> d_want;   // keys of the next launch

  // The reference loop's progress (:140-234), for exact replay and for the
  // speculative dry run that picks the next launch's windows.
  struct Replay {
    int state;
    unsigned int errors;
    int consumed, produced;
  };
  enum Outcome { DONE, STALLED };
  // Runs the reference loop from r over the memo.  exact: stops (without
  // taking the step) at the first window not decoded yet and commits
  // outputs; dry: guesses missing windows (pass while in sync, fail out of
  // sync), records them in d_want and stops after max_out consecutive
  // out-of-sync positions with missing windows, or max_want keys.
  Outcome replay(Replay &r, bool exact, int nin, int noutput, unsigned char *out, int max_out,
                 size_t max_want);
  // Frames pos, pos + N, ... decoded at pol that pass, counted (jump table)
  int pass_run(int pol, int pos, int nin);
  // Dry run: adds window (pos, pol) to d_want unless decoded or wanted (memo -2)
  void want(int64_t pos, int pol, int nin);
  // Decodes the windows d_want of the call's input into the memo (one
  // launch on the GPU; the test seam decodes runs of equally spaced windows).
  // first: the span is not staged yet (copy it); first_round: the call's first round
  void decode_wanted(const float *in, int nin, bool first, bool first_round);
  void adopt(ldpc_ctx *ctx);  // takes M, N from the context; checks the output shape

 public:
  // H == nullptr: the reference's default 32x64 H.  Otherwise an M x N
  // dense H, reordered (flags: LDPC_FLAG_*).
  ldpc_decoder_cb_impl(int method, int iterations, int precision, int device,
                       const uint8_t *H = nullptr, int M = 0, int N = 0, int flags = 0);
  // CSR H, used as given
  ldpc_decoder_cb_impl(int method, int iterations, int precision, int device, int M, int N,
                       const int32_t *row_ptr, const int32_t *col_idx, int flags);
  // MacKay alist file (see ldpc_decoder_cb::make)
  ldpc_decoder_cb_impl(int method, int iterations, int precision, int device,
                       const std::string &alist_path);
  ldpc_decoder_cb_impl(int method, int iterations, ldpc_block_backend_fn fn, void *user);
  ~ldpc_decoder_cb_impl();

  void forecast(int noutput_items, gr_vector_int &ninput_items_required);
  int general_work(int noutput_items, gr_vector_int &ninput_items,
                   gr_vector_const_void_star &input_items, gr_vector_void_star &output_items);

  int state() const { return d_state; }
  unsigned int errors() const { return d_errors; }
  int64_t frames_decoded() const { return d_frames_decoded; }
  int64_t launches() const { return d_launches; }
  unsigned int frame_samples() const { return d_N; }
  int frame_bytes() const { return d_out_bytes; }
  int frame_checks() const { return (int)d_M; }
};

}  // namespace ldpc_ece535a
}  // namespace gr

#endif
