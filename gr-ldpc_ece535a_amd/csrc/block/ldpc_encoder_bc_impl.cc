/* -*- c++ -*- */
/*
 * LDPC encoder block implementation.  Same stream contract as
 * lib/ldpc_encoder_bc_impl.cc:111-178 of gr-ldpc_ece535a; all frames that
 * fit the buffers are encoded in one ldpc_encode call.
 */
#include "ldpc_encoder_bc_impl.h"

#include <gnuradio/io_signature.h>
#include <ldpc_hip.h>

#include <cmath>
#include <stdexcept>

namespace gr {
namespace ldpc_ece535a {

ldpc_encoder_bc::sptr ldpc_encoder_bc::make() {
  return gnuradio::get_initial_sptr(new ldpc_encoder_bc_impl());
}

ldpc_encoder_bc_impl::ldpc_encoder_bc_impl()
    : gr::block("ldpc_encoder_bc", gr::io_signature::make(1, 1, sizeof(unsigned char)),
                gr::io_signature::make(1, 1, sizeof(gr_complex))),
      d_M(32),
      d_N(64),
      d_H(32 * 64) {
  ldpc_default_h(d_H.data());  // :57-99
  ldpc_reorder_h(d_H.data(), (int)d_M, (int)d_N, nullptr);  // :101
}

ldpc_encoder_bc_impl::~ldpc_encoder_bc_impl() {}

void ldpc_encoder_bc_impl::forecast(int noutput_items, gr_vector_int &ninput_items_required) {
  ninput_items_required[0] = (int)std::ceil(noutput_items / 16.0);  // rate 1/2 (:112-116)
}

int ldpc_encoder_bc_impl::general_work(int noutput_items, gr_vector_int &ninput_items,
                                       gr_vector_const_void_star &input_items,
                                       gr_vector_void_star &output_items) {
  const unsigned char *in = (const unsigned char *)input_items[0];
  gr_complex *out = (gr_complex *)output_items[0];
  const int in_per_frame = (int)d_M / 8;  // :127
  const int out_per_frame = (int)d_N;     // :128
  const int frames = std::min(noutput_items / out_per_frame, ninput_items[0] / in_per_frame);
  if (frames <= 0) {
    consume_each(0);
    return 0;
  }
  const int K = (int)(d_N - d_M);
  std::vector<uint8_t> data((size_t)frames * K), cw((size_t)frames * d_N);
  for (int f = 0; f < frames; ++f)  // data bits MSB first (:137-147)
    for (int i = 0; i < in_per_frame; ++i)
      for (int j = 0; j < 8; ++j)
        data[(size_t)f * K + i * 8 + j] = (in[f * in_per_frame + i] >> (7 - j)) & 1;
  if (ldpc_encode(d_H.data(), (int)d_M, (int)d_N, data.data(), frames, cw.data()) != 0)
    throw std::runtime_error("ldpc_encoder_bc: ldpc_encode failed");
  for (size_t t = 0; t < cw.size(); ++t)  // 1 -> +1, 0 -> -1 (:153-165)
    out[t] = gr_complex(cw[t] == 1 ? 1.0f : -1.0f, 0.0f);
  consume_each(frames * in_per_frame);
  return frames * out_per_frame;
}

}  // namespace ldpc_ece535a
}  // namespace gr
