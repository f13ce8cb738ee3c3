// The headline's four-in-flight rate in a plain C++ process (no Python, no
// torch), next to what the stream probes say about the context's set: is the
// bimodal four-in-flight rate of bench.py (profiles/round5/inflight_bimodal.txt)
// a property of the stream set, of the process, or of the Python harness?
//
//   hipcc --offload-arch=gfx950 -O2 -Iinclude -o tools/_inflight_diag tools/inflight_diag.cpp \
//       -Lgr-ldpc_ece535a_amd/lib -lldpc_hip -Wl,-rpath,$PWD/gr-ldpc_ece535a_amd/lib
//   tools/_inflight_diag [steps] [extra_streams_first]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ldpc_hip.h"

typedef __attribute__((address_space(1))) unsigned gu32;

__global__ void __launch_bounds__(64) k_wait(unsigned *flag, unsigned long long deadline) {
  extern __shared__ unsigned lds[];
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned v = 0;
  while ((v = __hip_atomic_load((gu32 *)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u &&
         __builtin_amdgcn_s_memrealtime() - t0 < deadline)
    __builtin_amdgcn_s_sleep(2);
  lds[0] = v;
  if (v) __hip_atomic_fetch_or((gu32 *)(flag + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_set(unsigned *flag) {
  if (threadIdx.x == 0) __hip_atomic_store((gu32 *)flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)
#define CL(x)                                                                    \
  do {                                                                           \
    int r_ = (x);                                                                \
    if (r_ < 0) {                                                                \
      fprintf(stderr, "%s:%d %s: %d %s\n", __FILE__, __LINE__, #x, r_, ldpc_last_error(ctx)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

int main(int argc, char **argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 100;
  const int extra = argc > 2 ? atoi(argv[2]) : 0;
  std::vector<hipStream_t> keep(extra);
  for (auto &x : keep) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  std::vector<uint8_t> H(64 * 32);
  ldpc_default_h(H.data());
  ldpc_reorder_h(H.data(), 32, 64, nullptr);
  ldpc_ctx *ctx = ldpc_create(H.data(), 32, 64, 0, 0);
  if (!ctx) {
    fprintf(stderr, "ldpc_create: %s\n", ldpc_last_error(nullptr));
    return 1;
  }
  int K = 0, KB = 0;
  ldpc_ctx_info(ctx, nullptr, nullptr, nullptr, &K, &KB, nullptr, nullptr);
  const int B = 4096, D = 4, N = 64;
  std::vector<float *> y(D);
  std::vector<uint8_t *> pk(D);
  std::vector<int32_t *> it(D);
  uint8_t *bits, *cw;
  CK(hipMalloc(&bits, (size_t)B * K));
  CK(hipMalloc(&cw, (size_t)B * N));
  const float sigma = std::sqrt(std::pow(10.0f, -2.0f / 10.0f));
  for (int d = 0; d < D; ++d) {
    CK(hipMalloc(&y[d], (size_t)B * N * 4));
    CK(hipMalloc(&pk[d], (size_t)B * KB));
    CK(hipMalloc(&it[d], (size_t)B * 4));
    CL(ldpc_random_bits(bits, (int64_t)B * K, 2024 + d, nullptr));
    CL(ldpc_encode_device(ctx, bits, B, cw, nullptr));
    CL(ldpc_bpsk_awgn(cw, (int64_t)B * N, sigma, 77 + d, y[d], nullptr));
  }
  CK(hipDeviceSynchronize());
  CL(ldpc_set_launch_mode(ctx, LDPC_MODE_THROUGHPUT));
  void *sv[4];
  CL(ldpc_ctx_streams(ctx, D, sv));
  std::vector<hipEvent_t> ev(2 * D);
  for (auto &e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  auto run = [&](int method, int n) {
    CK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < n; ++k) {
      const int d = k % D;
      if (k >= 2 * D) CK(hipEventSynchronize(ev[k % (2 * D)]));
      CL(ldpc_decode_device(ctx, method, 50, 1, 0, y[d], N, 1, 1.0f, B, pk[d], nullptr, it[d],
                            nullptr, nullptr, sv[d]));
      CK(hipEventRecord(ev[k % (2 * D)], (hipStream_t)sv[d]));
    }
    CK(hipDeviceSynchronize());
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return (double)n * B * K / s / 1e6;
  };
  run(1, 40);  // warm-up
  const double sp = run(1, steps), ms = run(0, steps), sp2 = run(1, steps);
  printf("sum-product f64 %.1f Mbit/s, min-sum f64 %.1f, sum-product again %.1f; streams", sp, ms, sp2);
  for (int d = 0; d < D; ++d) printf(" %p", sv[d]);
  printf("\n");
  unsigned *flag;
  CK(hipMalloc(&flag, 256));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipFuncSetAttribute((const void *)k_wait, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
  for (int mode = 0; mode < 2; ++mode) {
    printf("%s:", mode ? "stall" : "plain");
    for (int i = 0; i < D; ++i)
      for (int j = 0; j < D; ++j) {
        if (i == j) continue;
        CK(hipMemset(flag, 0, 8));
        CK(hipDeviceSynchronize());
        if (mode == 0)
          hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, (hipStream_t)sv[i], flag, 200000ull);
        else
          hipLaunchKernelGGL(k_wait, dim3(6 * cus), dim3(64), 65536, (hipStream_t)sv[i], flag, 50000ull);
        hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, (hipStream_t)sv[j], flag);
        CK(hipDeviceSynchronize());
        unsigned seen = 0;
        CK(hipMemcpy(&seen, flag + 1, 4, hipMemcpyDeviceToHost));
        printf(" %d%d:%u", i, j, seen);
      }
    printf("\n");
  }
  ldpc_destroy(ctx);
  return 0;
}
