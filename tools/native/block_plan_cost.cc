// Host cost of the decoder block's launch planning (replay + dry run) in
// steady state: one block driven through its test seam over a long periodic
// stream (a table stream repeated `reps` times), calls of `chunk` frames.
// The seam's table lookup (fn) is test cost the GPU path does not have.
// Tables: raw synd (int32, 2 x npos), packed (u8, 2 x npos x 4) and samples
// (float re/im) of one stream, e.g. from tools/block_policy_sim.py's cache:
//   np.load(c)["synd"].astype(np.int32).tofile("synd.bin"), ... ["packed"], ["x"]
// Build and run (gprof with -pg):
//   g++ -O2 -std=c++17 -Igr-ldpc_ece535a_amd/csrc/block -Igr-ldpc_ece535a_amd/include \
//       -Iinclude tools/native/block_plan_cost.cc gr-ldpc_ece535a_amd/csrc/block/*.cc \
//       -Lgr-ldpc_ece535a_amd/lib -lldpc_hip -Wl,-rpath,$PWD/gr-ldpc_ece535a_amd/lib -o /tmp/bpc
//   /tmp/bpc x.bin synd.bin packed.bin <chunk frames> <reps> [iterations, default 50]
// one block, a long periodic stream (the table's stream repeated): steady-state planning cost
#include <ldpc_block.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <unistd.h>
#include <fcntl.h>
struct T { const float *base; const int32_t *synd; const uint8_t *pk; int64_t npos, S; };
static std::vector<char> rd(const char *f) { FILE *p = fopen(f, "rb"); fseek(p, 0, SEEK_END); long n = ftell(p); fseek(p, 0, SEEK_SET); std::vector<char> v(n); if (fread(v.data(), 1, n, p)) {} fclose(p); return v; }
static int fn(void *u, const float *in, int64_t, int64_t cw, int, float pol, int B, uint8_t *pk, int32_t *sy) {
  T *t = (T *)u; int64_t p0 = (in - t->base) / 2; int pl = pol < 0;
  for (int b = 0; b < B; ++b) { int64_t p = (p0 + (cw / 2) * b) % t->S;
    if (p >= t->npos) { sy[b] = 32; memset(pk + 4 * b, 0, 4); continue; }
    sy[b] = t->synd[pl * t->npos + p]; memcpy(pk + 4 * b, t->pk + (pl * t->npos + p) * 4, 4); }
  return 0;
}
int main(int argc, char **argv) {
  auto x = rd(argv[1]); auto s = rd(argv[2]); auto k = rd(argv[3]); int chunk = atoi(argv[4]) * 64; int reps = atoi(argv[5]);
  const int64_t S = x.size() / 8;
  std::vector<float> big((size_t)S * 2 * reps);
  for (int r = 0; r < reps; ++r) memcpy(big.data() + (size_t)r * S * 2, x.data(), x.size());
  T t{big.data(), (const int32_t *)s.data(), (const uint8_t *)k.data(), (int64_t)(s.size() / 8), S};
  int dn = open("/dev/null", O_WRONLY); dup2(dn, 1);
  const int iters = argc > 6 ? atoi(argv[6]) : 50;  // the planner's launch cap depends on it
  ldpc_block *b = ldpc_decoder_cb_make_with_backend(1, iters, fn, &t);
  int64_t nS = S * reps, pos = 0; std::vector<uint8_t> out(chunk / 16 + 16); int calls = 0; long long l0 = 0;
  auto t0 = std::chrono::steady_clock::now();
  while (pos + 64 <= nS) { int used = 0; int n = (int)std::min<int64_t>(chunk, nS - pos);
    ldpc_decoder_cb_general_work(b, chunk / 16, n, t.base + 2 * pos, out.data(), &used); pos += used; ++calls;
    if (calls == 2) { t0 = std::chrono::steady_clock::now(); l0 = ldpc_decoder_cb_launches(b); }
    if (!used) break; }
  double tot = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  fprintf(stderr, "%d calls: %.1f us per call, %.1f launches per call, %.1f us per launch\n", calls - 2, tot / (calls - 2) * 1e6, (double)(ldpc_decoder_cb_launches(b) - l0) / (calls - 2), tot / (ldpc_decoder_cb_launches(b) - l0) * 1e6);
}
