// Host <-> persistent-kernel round-trip latency on MI355X, three hand-off
// forms for the host -> device direction (the device -> host direction is
// always a system-scope store into mapped pinned host memory):
//   mode 0: host writes mapped pinned HOST memory, one device lane polls it
//           with system-scope loads (the window server's poller);
//   mode 1: host writes FINE-GRAINED DEVICE memory (hipExtMallocWithFlags,
//           hipDeviceMallocFinegrained) through the BAR, the device lane
//           polls its own memory;
//   mode 2: as 1, but 256 workgroups poll (agent-scope loads) and all answer.
// Usage: pingpong [rounds]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <vector>

typedef __attribute__((address_space(1))) uint64_t gu64;

__global__ void pong(const uint64_t *in, uint64_t *out, int rounds, int sys, uint64_t deadline) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int r = 1; r <= rounds; ++r) {
    uint64_t v;
    for (;;) {
      v = sys ? __hip_atomic_load((const gu64 *)in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
              : __hip_atomic_load((const gu64 *)in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v >= (uint64_t)r) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > deadline) return;
    }
    __hip_atomic_store((gu64 *)(out + 8 * blockIdx.x), (uint64_t)r, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 2000;
  uint64_t *h_in = nullptr, *h_out = nullptr, *d_in = nullptr;
  hipHostMalloc((void **)&h_in, 4096, hipHostMallocMapped | hipHostMallocCoherent);
  hipHostMalloc((void **)&h_out, 1 << 16, hipHostMallocMapped | hipHostMallocCoherent);
  hipError_t e = hipExtMallocWithFlags((void **)&d_in, 4096, hipDeviceMallocFinegrained);
  printf("fine-grained device alloc: %s\n", hipGetErrorString(e));
  void *dh_in = nullptr, *dh_out = nullptr;
  hipHostGetDevicePointer(&dh_in, h_in, 0);
  hipHostGetDevicePointer(&dh_out, h_out, 0);
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  for (int mode = 0; mode < 3; ++mode) {
    if (mode > 0 && e != hipSuccess) break;
    volatile uint64_t *win = mode == 0 ? (volatile uint64_t *)h_in : (volatile uint64_t *)d_in;
    win[0] = 0;
    memset(h_out, 0, 1 << 16);
    const int blocks = mode == 2 ? 256 : 1;
    hipLaunchKernelGGL(pong, dim3(blocks), dim3(64), 0, st, mode == 0 ? (uint64_t *)dh_in : d_in,
                       (uint64_t *)dh_out, rounds, mode == 0 ? 1 : 0, (uint64_t)200000000);
    std::vector<double> t(rounds);
    for (int r = 1; r <= rounds; ++r) {
      const auto a = std::chrono::steady_clock::now();
      __atomic_store_n((uint64_t *)win, (uint64_t)r, __ATOMIC_RELEASE);
      for (int b = 0; b < blocks; ++b) {
        long spins = 0;
        while (__atomic_load_n(h_out + 8 * b, __ATOMIC_ACQUIRE) < (uint64_t)r) {
          if (++spins > 400000000L) { printf("timeout mode %d round %d\n", mode, r); return 1; }
        }
      }
      t[r - 1] = std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count() * 1e6;
    }
    hipStreamSynchronize(st);
    std::vector<double> s(t.begin() + rounds / 4, t.end());
    std::sort(s.begin(), s.end());
    printf("mode %d (%s): round trip median %.2f us, p10 %.2f, p90 %.2f\n", mode,
           mode == 0 ? "host memory + poller" : mode == 1 ? "fine-grained device memory, 1 poller"
                                                          : "fine-grained device memory, 256 pollers",
           s[s.size() / 2], s[s.size() / 10], s[s.size() * 9 / 10]);
  }
  return 0;
}
