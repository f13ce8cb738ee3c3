/* -*- c++ -*- */
/*
 * LDPC decoder block implementation (MI355X edition).
 *
 * Keeps the reference's block contract (lib/ldpc_decoder_cb_impl.h:22-66):
 * 64 gr_complex in -> 4 bytes out per frame, methods 0..3, the frame-sync /
 * polarity state machine.  What changes is how frames are decoded: instead
 * of one CPU decode per 64-sample window, general_work decodes every window
 * it can already see in one GPU launch and then replays the reference's
 * state machine over the results (see ldpc_decoder_cb_impl.cc).
 */
#ifndef INCLUDED_LDPC_ECE535A_LDPC_DECODER_CB_IMPL_H
#define INCLUDED_LDPC_ECE535A_LDPC_DECODER_CB_IMPL_H

#include <ldpc_block.h>
#include <ldpc_ece535a/ldpc_decoder_cb.h>
#include <ldpc_hip.h>

#include <string>
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
  std::vector<uint8_t> d_packed[2];
  std::vector<int32_t> d_synd[2];

  // Decodes B windows of the interleaved complex input starting at `in`
  // (window b starts b*stride samples in), tx = Re * polarity.
  void decode_windows(const float *in, int64_t n_floats, int stride, float polarity, int B,
                      int slot);
  // Decodes B one-sample-step windows at +tx into slot 0 and -tx into slot 1
  // (one launch on the GPU).
  void decode_both(const float *in, int64_t n_floats, int B);
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
  unsigned int frame_samples() const { return d_N; }
  int frame_bytes() const { return d_out_bytes; }
  int frame_checks() const { return (int)d_M; }
};

}  // namespace ldpc_ece535a
}  // namespace gr

#endif
