// Minimal stand-in for GNU Radio 3.7's <gnuradio/block.h>: the subset of
// gr::block that a general_work block and its scheduler need (forecast,
// general_work, consume_each, the i/o signatures).  The real runtime
// (scheduler thread, circular buffers) is replaced in tests by the small
// harness in ldpc_ece535a/flowgraph.py.
#ifndef INCLUDED_GR_BLOCK_H
#define INCLUDED_GR_BLOCK_H
#include <memory>
#include <string>
#include <vector>

#include <gnuradio/gr_complex.h>
#include <gnuradio/io_signature.h>

typedef std::vector<int> gr_vector_int;
typedef std::vector<const void *> gr_vector_const_void_star;
typedef std::vector<void *> gr_vector_void_star;

namespace boost {
using std::shared_ptr;  // GR 3.7 uses boost::shared_ptr for sptr
}

namespace gr {
class block {
 public:
  block(const std::string &name, io_signature::sptr input_signature,
        io_signature::sptr output_signature)
      : d_name(name), d_in(input_signature), d_out(output_signature), d_consumed(0) {}
  virtual ~block() {}
  virtual void forecast(int noutput_items, gr_vector_int &ninput_items_required) = 0;
  virtual int general_work(int noutput_items, gr_vector_int &ninput_items,
                           gr_vector_const_void_star &input_items,
                           gr_vector_void_star &output_items) = 0;
  const std::string &name() const { return d_name; }
  io_signature::sptr input_signature() const { return d_in; }
  io_signature::sptr output_signature() const { return d_out; }
  void consume_each(int how_many_items) { d_consumed = how_many_items; }
  // scheduler side: items consumed by the last general_work call
  int last_consumed() const { return d_consumed; }

 private:
  std::string d_name;
  io_signature::sptr d_in, d_out;
  int d_consumed;
};
}  // namespace gr

namespace gnuradio {
template <class T>
std::shared_ptr<T> get_initial_sptr(T *p) {
  return std::shared_ptr<T>(p);
}
}  // namespace gnuradio
#endif
