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
  int d_precision;
  ldpc_ctx *d_ctx;               // GPU context (default H, reordered)
  ldpc_block_backend_fn d_backend;  // test seam; null = GPU
  void *d_backend_user;
  int64_t d_frames_decoded;
  std::vector<uint8_t> d_packed[2];
  std::vector<int32_t> d_synd[2];

  // Decodes B windows of the interleaved complex input starting at `in`
  // (window b starts b*stride samples in), tx = Re * polarity.
  void decode_windows(const float *in, int64_t n_floats, int stride, float polarity, int B,
                      int slot);

 public:
  ldpc_decoder_cb_impl(int method, int iterations, int precision, int device);
  ldpc_decoder_cb_impl(int method, int iterations, ldpc_block_backend_fn fn, void *user);
  ~ldpc_decoder_cb_impl();

  void forecast(int noutput_items, gr_vector_int &ninput_items_required);
  int general_work(int noutput_items, gr_vector_int &ninput_items,
                   gr_vector_const_void_star &input_items, gr_vector_void_star &output_items);

  int state() const { return d_state; }
  unsigned int errors() const { return d_errors; }
  int64_t frames_decoded() const { return d_frames_decoded; }
  unsigned int frame_samples() const { return d_N; }
};

}  // namespace ldpc_ece535a
}  // namespace gr

#endif
