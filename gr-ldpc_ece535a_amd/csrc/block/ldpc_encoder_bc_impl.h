/* -*- c++ -*- */
/*
 * LDPC encoder block implementation (reference:
 * lib/ldpc_encoder_bc_impl.{h,cc}): 4 bytes -> 32 data bits (MSB first)
 * -> [parity(32); data(32)] as BPSK +-1 gr_complex.  The parity comes from
 * ldpc_encode (include/ldpc_hip.h), the GF(2) form of makeParityCheck.
 */
#ifndef INCLUDED_LDPC_ECE535A_LDPC_ENCODER_BC_IMPL_H
#define INCLUDED_LDPC_ECE535A_LDPC_ENCODER_BC_IMPL_H

#include <ldpc_ece535a/ldpc_encoder_bc.h>

#include <vector>

namespace gr {
namespace ldpc_ece535a {

class ldpc_encoder_bc_impl : public ldpc_encoder_bc {
 private:
  unsigned int d_M;
  unsigned int d_N;
  std::vector<uint8_t> d_H;  // reordered default H

 public:
  ldpc_encoder_bc_impl();
  ~ldpc_encoder_bc_impl();
  void forecast(int noutput_items, gr_vector_int &ninput_items_required);
  int general_work(int noutput_items, gr_vector_int &ninput_items,
                   gr_vector_const_void_star &input_items, gr_vector_void_star &output_items);
};

}  // namespace ldpc_ece535a
}  // namespace gr
#endif
