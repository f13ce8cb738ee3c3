// Minimal stand-in for GNU Radio 3.7's <gnuradio/gr_complex.h> (GNU Radio is
// not installed in this build environment).  Only what the ldpc_ece535a
// blocks use.  Build against a real GNU Radio 3.7 install by putting its
// include directory ahead of this one.
#ifndef INCLUDED_GR_COMPLEX_H
#define INCLUDED_GR_COMPLEX_H
#include <complex>
typedef std::complex<float> gr_complex;
#endif
