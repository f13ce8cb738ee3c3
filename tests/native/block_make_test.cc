// A GNU Radio-style caller of the drop-in block, written against the public
// C++ face only (include/ldpc_ece535a/ldpc_decoder_cb.h, the reference's
// include/ldpc_ece535a/ldpc_decoder_cb.h:22-36): the block comes from
// ldpc_decoder_cb::make(method) -- or make(method, iterations, precision,
// alist_path) -- and is driven through the gr::block virtual interface
// (forecast, general_work, consume_each) the way the GR 3.7 scheduler drives
// it: input arrives in chunks, unconsumed input is kept, general_work is
// called again until it consumes nothing.
//
//   block_make_test <method> <in.f32> <out.u8> [chunk] [iterations precision alist]
//
// in.f32: interleaved gr_complex samples (re, im float32).  Built by
// gr-ldpc_ece535a_amd/Makefile (target native); run by tests/test_gpu_block.py.
#include <gnuradio/block.h>
#include <ldpc_ece535a/ldpc_decoder_cb.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <string>
#include <vector>

int main(int argc, char **argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s method in.f32 out.u8 [chunk] [iterations precision alist]\n",
                 argv[0]);
    return 2;
  }
  const int method = std::atoi(argv[1]);
  const int chunk = argc > 4 ? std::atoi(argv[4]) : 1000;
  std::vector<float> in;
  {
    FILE *f = std::fopen(argv[2], "rb");
    if (!f) return 3;
    float buf[4096];
    size_t n;
    while ((n = std::fread(buf, sizeof(float), 4096, f)) > 0) in.insert(in.end(), buf, buf + n);
    std::fclose(f);
  }
  const int total = (int)(in.size() / 2);
  try {
    gr::ldpc_ece535a::ldpc_decoder_cb::sptr blk =
        argc > 7 ? gr::ldpc_ece535a::ldpc_decoder_cb::make(method, std::atoi(argv[5]),
                                                           std::atoi(argv[6]),
                                                           std::string(argv[7]))
                 : gr::ldpc_ece535a::ldpc_decoder_cb::make(method);
    gr::block &b = *blk;  // only the gr::block interface from here on
    std::vector<unsigned char> out;
    std::vector<unsigned char> obuf(1 << 16);
    int pos = 0, avail_end = 0;
    for (;;) {
      avail_end = std::min(total, avail_end + chunk);
      for (;;) {
        const int nin = avail_end - pos;
        gr_vector_int req(1, 0);
        b.forecast((int)obuf.size(), req);  // GR asks; a real scheduler may call anyway
        gr_vector_int ninput(1, nin);
        gr_vector_const_void_star ins(1, in.data() + 2 * (size_t)pos);
        gr_vector_void_star outs(1, obuf.data());
        const int made = b.general_work((int)obuf.size(), ninput, ins, outs);
        const int used = b.last_consumed();
        out.insert(out.end(), obuf.begin(), obuf.begin() + made);
        pos += used;
        if (used == 0) break;
      }
      if (avail_end >= total) break;
    }
    FILE *f = std::fopen(argv[3], "wb");
    if (!f) return 4;
    std::fwrite(out.data(), 1, out.size(), f);
    std::fclose(f);
    std::printf("block %s: %d samples in, %zu bytes out\n", b.name().c_str(), pos, out.size());
  } catch (const std::exception &e) {
    std::fprintf(stderr, "block_make_test: %s\n", e.what());
    return 1;
  }
  return 0;
}
