// Host cost of the decoder block's launch planning (replay + dry run) alone:
// the block is driven through its test seam over a table of window results
// (tools/block_policy_sim.py writes the tables: synd / packed / samples as raw
// .bin), in calls of `chunk` frames, 200 times.  Build and time, or profile
// with -pg and gprof:
//   g++ -O2 -std=c++17 -Igr-ldpc_ece535a_amd/csrc/block -Igr-ldpc_ece535a_amd/include \
//       -Iinclude tools/native/block_plan_cost.cc gr-ldpc_ece535a_amd/csrc/block/*.cc \
//       -Lgr-ldpc_ece535a_amd/lib -lldpc_hip -Wl,-rpath,$PWD/gr-ldpc_ece535a_amd/lib -o /tmp/bpc
//   time /tmp/bpc x.bin synd.bin packed.bin 512
#include <ldpc_block.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <unistd.h>
#include <fcntl.h>
struct T { const float *base; const int32_t *synd; const uint8_t *pk; int64_t npos; };
static std::vector<char> rd(const char *f) { FILE *p = fopen(f, "rb"); fseek(p, 0, SEEK_END); long n = ftell(p); fseek(p, 0, SEEK_SET); std::vector<char> v(n); if (fread(v.data(), 1, n, p)) {} fclose(p); return v; }
static int fn(void *u, const float *in, int64_t, int64_t cw, int, float pol, int B, uint8_t *pk, int32_t *sy) {
  T *t = (T *)u; int64_t p0 = (in - t->base) / 2; int pl = pol < 0;
  for (int b = 0; b < B; ++b) { int64_t p = p0 + (cw / 2) * b; sy[b] = t->synd[pl * t->npos + p]; for (int i = 0; i < 4; ++i) pk[4 * b + i] = t->pk[(pl * t->npos + p) * 4 + i]; }
  return 0;
}
int main(int argc, char **argv) {
  auto x = rd(argv[1]); auto s = rd(argv[2]); auto k = rd(argv[3]); int chunk = atoi(argv[4]) * 64;
  T t{(const float *)x.data(), (const int32_t *)s.data(), (const uint8_t *)k.data(), (int64_t)(s.size() / 8)};
  int dn = open("/dev/null", O_WRONLY); dup2(dn, 1);
  for (int rep = 0; rep < 200; ++rep) {
    ldpc_block *b = ldpc_decoder_cb_make_with_backend(1, 50, fn, &t);
    int64_t nS = x.size() / 8, pos = 0; std::vector<uint8_t> out(chunk / 16 + 16);
    while (pos + 64 <= nS) { int used = 0; int n = (int)std::min<int64_t>(chunk, nS - pos);
      ldpc_decoder_cb_general_work(b, chunk / 16, n, t.base + 2 * pos, out.data(), &used); pos += used; if (!used) break; }
    ldpc_decoder_cb_destroy(b);
  }
}
