/* -*- c++ -*- */
/*
 * LDPC decoder block implementation (MI355X edition).
 *
 * general_work reproduces lib/ldpc_decoder_cb_impl.cc:133-234 of
 * gr-ldpc_ece535a output for output, for any chunking of the input:
 *
 *  - IN_SYNC / IN_SYNC_INVERTED: the windows at consumed, consumed+64, ...
 *    that fit the input and output buffers are decoded in ONE GPU launch
 *    with the state's polarity; the reference's per-frame decisions are then
 *    replayed in order.  A frame that fails (syndrome weight > M/8) bumps the
 *    error counter and is still emitted (:168-176, :207-225); the 11th
 *    failure drops sync, retries the same window negated -- with the quirk
 *    that the negation is relative to the polarity the window was decoded
 *    with (:180-191) -- and either re-syncs inverted or skips one sample.
 *    Results past a state change are discarded and re-decoded.
 *  - OUT_OF_SYNC: candidate start positions (1-sample steps, :194-198) are
 *    decoded at both polarities in one launch per batch, in batches of 64,
 *    256, 1024, ... positions; the first position whose +tx or, failing
 *    that, -tx decode passes the frame check wins, exactly as the
 *    reference's serial search would find, and the search stops at the first
 *    batch that holds one (a sync loss costs ~128 decodes when the frame
 *    boundary is near, not two decodes per visible sample).
 *
 * The H is the reference's default (make(method)), or a runtime H (dense,
 * reordered like the reference's constructor; CSR; or an alist file).
 *
 * Decoding is deterministic per window, so the batched schedule emits the
 * same bytes, consumes the same items and leaves the same state as the
 * reference's frame-at-a-time loop.
 */
#include "ldpc_decoder_cb_impl.h"

#include <gnuradio/io_signature.h>

#include <algorithm>
#include <cstring>
#include <iostream>
#include <stdexcept>
#include <string>

namespace gr {
namespace ldpc_ece535a {

#define STATE_OUT_OF_SYNC 0
#define STATE_IN_SYNC 1
#define STATE_IN_SYNC_INVERTED 2

namespace {
const int kMaxWindows = 1 << 16;  // windows per launch (bounds staging memory)
const int kSearchFirst = 64;      // first OUT_OF_SYNC batch; x4 per batch after
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
}

ldpc_decoder_cb_impl::ldpc_decoder_cb_impl(int method, int iterations, ldpc_block_backend_fn fn,
                                           void *user)
    : LDPC_BLOCK_INIT(method, iterations, LDPC_PREC_F64) {
  if (!fn) throw std::runtime_error("ldpc_decoder_cb: null backend");
  d_backend = fn;
  d_backend_user = user;
}

ldpc_decoder_cb_impl::~ldpc_decoder_cb_impl() { ldpc_destroy(d_ctx); }

void ldpc_decoder_cb_impl::forecast(int noutput_items, gr_vector_int &ninput_items_required) {
  ninput_items_required[0] = noutput_items * d_N;
}

void ldpc_decoder_cb_impl::decode_both(const float *in, int64_t n_floats, int B) {
  if (d_backend) {  // the test seam decodes one polarity per call
    decode_windows(in, n_floats, 1, 1.0f, B, 0);
    decode_windows(in, n_floats, 1, -1.0f, B, 1);
    return;
  }
  const int KB = (int)(d_N - d_M + 7) / 8;
  d_packed[0].resize((size_t)2 * B * KB);
  d_synd[0].resize((size_t)2 * B);
  const int rc = ldpc_decode_strided_both(d_ctx, d_method, (int)d_iterations, 1, d_precision, in,
                                          n_floats, 2, 2, 1.0f, B, d_packed[0].data(),
                                          d_synd[0].data());
  if (rc < 0)
    throw std::runtime_error(std::string("ldpc_decoder_cb: decode failed: ") +
                             ldpc_last_error(d_ctx));
  // rows B.. are the -tx decodes
  d_packed[1].assign(d_packed[0].begin() + (size_t)B * KB, d_packed[0].end());
  d_synd[1].assign(d_synd[0].begin() + B, d_synd[0].end());
  d_frames_decoded += 2 * (int64_t)B;
}

void ldpc_decoder_cb_impl::decode_windows(const float *in, int64_t n_floats, int stride,
                                          float polarity, int B, int slot) {
  const int KB = (int)(d_N - d_M + 7) / 8;
  d_packed[slot].resize((size_t)B * KB);
  d_synd[slot].resize((size_t)B);
  int rc;
  if (d_backend)
    rc = d_backend(d_backend_user, in, n_floats, 2 * (int64_t)stride, 2, polarity, B,
                   d_packed[slot].data(), d_synd[slot].data());
  else
    rc = ldpc_decode_strided(d_ctx, d_method, (int)d_iterations, 1, d_precision, in, n_floats,
                             2 * (int64_t)stride, 2, polarity, B, d_packed[slot].data(),
                             nullptr, nullptr, d_synd[slot].data(), nullptr);
  if (rc < 0)
    throw std::runtime_error(std::string("ldpc_decoder_cb: decode failed: ") +
                             (d_ctx ? ldpc_last_error(d_ctx) : "backend error"));
  d_frames_decoded += B;
}

int ldpc_decoder_cb_impl::general_work(int noutput_items, gr_vector_int &ninput_items,
                                       gr_vector_const_void_star &input_items,
                                       gr_vector_void_star &output_items) {
  const float *in = (const float *)input_items[0];  // interleaved re/im
  unsigned char *out = (unsigned char *)output_items[0];
  const int N = (int)d_N;
  const int min_output_required = d_out_bytes;      // :141 (M/8)
  const int frame_error_threshold = (int)d_M / 8;   // :142
  const int KB = (N - (int)d_M + 7) / 8;
  const int nin = ninput_items[0];

  int input_consumed = 0;
  int output_produced = 0;
  int search_batch = kSearchFirst;
  // checkFrame(vhat, threshold) stops counting at threshold+1 (:247-249)
  auto capped = [&](int32_t w) { return std::min<int32_t>(w, frame_error_threshold + 1); };
  auto emit = [&](const uint8_t *bytes) {
    std::memcpy(out + output_produced, bytes, (size_t)min_output_required);
    input_consumed += N;
    output_produced += min_output_required;
  };

  while ((nin - input_consumed) >= N && (noutput_items - output_produced) >= min_output_required) {
    const float *here = in + 2 * (int64_t)input_consumed;
    const int64_t avail = 2 * (int64_t)(nin - input_consumed);
    if (d_state != STATE_OUT_OF_SYNC) {
      const float pol = d_state == STATE_IN_SYNC_INVERTED ? -1.0f : 1.0f;
      int W = (nin - input_consumed) / N;
      if (min_output_required > 0)
        W = std::min(W, (noutput_items - output_produced) / min_output_required);
      W = std::min(W, kMaxWindows);
      decode_windows(here, avail, N, pol, W, 0);
      for (int w = 0; w < W; ++w) {
        const int sNotZero = capped(d_synd[0][w]);
        if (sNotZero > frame_error_threshold) {
          d_errors++;
          if (d_errors > 10) {  // :171-175
            d_errors = 0;
            d_state = STATE_OUT_OF_SYNC;
            std::cout << "MAX ERRORS; OUT OF SYNC" << std::endl;
            // retry this window with -tx, tx taken at the old polarity (:178-191)
            const float *win = in + 2 * (int64_t)input_consumed;
            decode_windows(win, 2 * (int64_t)(nin - input_consumed), N, -pol, 1, 1);
            if (capped(d_synd[1][0]) <= frame_error_threshold) {
              std::cout << "IN SYNC; PHASE INVERTED" << std::endl;
              d_state = STATE_IN_SYNC_INVERTED;
              d_errors = 0;
              emit(d_packed[1].data());
            } else {
              input_consumed += 1;  // :194-198
            }
            break;  // the rest of the batch was decoded for the old state
          }
        }
        emit(&d_packed[0][(size_t)w * KB]);
      }
    } else {
      // start positions with a full window, both polarities in one launch,
      // in growing batches (the first batch is small: the frame boundary is
      // usually near); one failed position consumes one sample (:194-198)
      int P = std::min(nin - input_consumed - N + 1, std::min(search_batch, kMaxWindows));
      search_batch = std::min(4 * search_batch, kMaxWindows);
      decode_both(here, avail, P);
      for (int p = 0; p < P; ++p) {
        if (capped(d_synd[0][p]) <= frame_error_threshold) {  // :201-205
          search_batch = kSearchFirst;
          std::cout << "IN SYNC" << std::endl;
          d_state = STATE_IN_SYNC;
          d_errors = 0;
          emit(&d_packed[0][(size_t)p * KB]);
          break;
        }
        if (capped(d_synd[1][p]) <= frame_error_threshold) {  // :189-192
          search_batch = kSearchFirst;
          std::cout << "IN SYNC; PHASE INVERTED" << std::endl;
          d_state = STATE_IN_SYNC_INVERTED;
          d_errors = 0;
          emit(&d_packed[1][(size_t)p * KB]);
          break;
        }
        input_consumed += 1;  // skip one sample and search on
      }
    }
  }

  consume_each(input_consumed);
  return output_produced;
}

}  // namespace ldpc_ece535a
}  // namespace gr
