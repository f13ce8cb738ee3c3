/* -*- c++ -*- */
/*
 * LDPC encoder block (reference: include/ldpc_ece535a/ldpc_encoder_bc.h:22-36):
 * packed bytes in, BPSK +-1 gr_complex out, rate 1/2 with the default H.
 */
#ifndef INCLUDED_LDPC_ECE535A_LDPC_ENCODER_BC_H
#define INCLUDED_LDPC_ECE535A_LDPC_ENCODER_BC_H

#include <gnuradio/block.h>
#include <ldpc_ece535a/api.h>

namespace gr {
namespace ldpc_ece535a {

class LDPC_ECE535A_API ldpc_encoder_bc : virtual public gr::block {
 public:
  typedef boost::shared_ptr<ldpc_encoder_bc> sptr;
  static sptr make();
};

}  // namespace ldpc_ece535a
}  // namespace gr

#endif /* INCLUDED_LDPC_ECE535A_LDPC_ENCODER_BC_H */
