// Which streams can dispatch while another stream's launch is stalled in
// dispatch (more workgroups than fit): a pairwise matrix for n streams made
// back to back, next to the plain concurrency probe (both kernels tiny).
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/_pipe_probe tools/pipe_probe.cpp
//   tools/_pipe_probe [n_streams] [extra_streams_first]
//
// "plain": a one-wave kernel on stream a spins on a flag (2 ms at most) that a
// one-wave kernel on stream b raises.  "stall": the kernel on a has more
// workgroups than the GPU holds (64 KB of LDS each), every one spinning on the
// flag for at most 0.5 ms, so its dispatch is stuck until they time out; the
// flag kernel on b runs in time only if b's queue dispatches independently.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

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

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e_ = (x);                                             \
    if (e_ != hipSuccess) {                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
      exit(1);                                                       \
    }                                                                \
  } while (0)

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 8;
  const int extra = argc > 2 ? atoi(argv[2]) : 0;
  std::vector<hipStream_t> keep(extra), s(n);
  for (auto &x : keep) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  for (auto &x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  unsigned *flag;
  CK(hipMalloc(&flag, 256));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipFuncSetAttribute((const void *)k_wait, hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
  for (int mode = 0; mode < 2; ++mode) {
    printf("%s probe (1 = b ran while a waited)\n   ", mode ? "stall" : "plain");
    for (int j = 0; j < n; ++j) printf(" %2d", j);
    printf("\n");
    for (int i = 0; i < n; ++i) {
      printf("%2d:", i);
      for (int j = 0; j < n; ++j) {
        if (i == j) {
          printf("  -");
          continue;
        }
        CK(hipMemset(flag, 0, 8));
        CK(hipDeviceSynchronize());
        if (mode == 0)
          hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, s[i], flag, 200000ull);
        else  // 3 x the resident workgroups at 64 KB of LDS (2 per CU)
          hipLaunchKernelGGL(k_wait, dim3(6 * cus), dim3(64), 65536, s[i], flag, 50000ull);
        hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, s[j], flag);
        CK(hipDeviceSynchronize());
        unsigned seen = 0;
        CK(hipMemcpy(&seen, flag + 1, 4, hipMemcpyDeviceToHost));
        printf("  %u", seen);
      }
      printf("\n");
    }
  }
  return 0;
}
