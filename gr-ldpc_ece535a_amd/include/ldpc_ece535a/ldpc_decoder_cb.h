/* -*- c++ -*- */
/*
 * LDPC decoder block, MI355X edition.
 *
 * Same public interface as gr-ldpc_ece535a's
 * include/ldpc_ece535a/ldpc_decoder_cb.h:22-36 -- a gr::block taking
 * gr_complex samples and producing packed data bytes, created with
 * make(method) -- so existing flowgraphs, GRC descriptors and SWIG bindings
 * keep working.  The decode itself runs on the GPU through the C ABI of
 * include/ldpc_hip.h.
 */
#ifndef INCLUDED_LDPC_ECE535A_LDPC_DECODER_CB_H
#define INCLUDED_LDPC_ECE535A_LDPC_DECODER_CB_H

#include <gnuradio/block.h>
#include <ldpc_ece535a/api.h>

#include <string>
#include <vector>

namespace gr {
namespace ldpc_ece535a {

/*!
 * \brief LDPC decoder block
 * \ingroup ldpc_ece535a
 *
 * method: 0 LogDomain (min-sum), 1 SumProduct, 2 BitFlip, 3 Hard
 * (grc/ldpc_ece535a_ldpc_decoder_cb.xml:11-29); other values behave as 0.
 */
class LDPC_ECE535A_API ldpc_decoder_cb : virtual public gr::block {
 public:
  typedef boost::shared_ptr<ldpc_decoder_cb> sptr;

  /*! The reference's factory: default 32x64 H, 5 iterations. */
  static sptr make(const int method);

  /*! Additive overload: iteration cap (the reference hard-codes 5) and
   *  arithmetic precision (include/ldpc_hip.h LDPC_PREC_*): 0 = f64, the
   *  reference's arithmetic bit for bit (glibc's tanh / log reproduced,
   *  correctly rounded divisions); 1 = f32; 2 = the same f64 functions one
   *  value at a time (also exact); 3 = f64 with compact tanh / log (within
   *  3 / 1 ulp of glibc, not exact). */
  static sptr make(const int method, const int iterations, const int precision = 0);

  /*! Additive overload: a runtime H in place of the compiled-in matrix
   *  (lib/ldpc_decoder_cb_impl.cc:60-102).  H is M x N, row-major, one byte
   *  per entry; reorderHMatrix is applied as the reference's constructor does
   *  (:104-106).  Per frame N samples in, M/8 bytes (bits M.. of the decision)
   *  out, frame-error threshold M/8 (:141-142); needs N - M >= 8 (M/8). */
  static sptr make(const int method, const int iterations, const int precision,
                   const std::vector<unsigned char> &H, const int M, const int N);

  /*! Additive overload: H from a MacKay alist file.  Codes small enough for a
   *  dense matrix (M N <= 2^22) are reordered like the reference's H; larger
   *  ones are used as given (put the information columns last). */
  static sptr make(const int method, const int iterations, const int precision,
                   const std::string &alist_path);
};

}  // namespace ldpc_ece535a
}  // namespace gr

#endif /* INCLUDED_LDPC_ECE535A_LDPC_DECODER_CB_H */
