// Stream-pair probes as a shared library for in-process diagnostics
// (bench.py LDPC_BENCH_PROBE=1): plain = one-wave kernels; stall = the
// waiting launch has more workgroups than fit (64 KB LDS each), so its
// dispatch is stuck while they spin.  Returns 1 if the set kernel on b ran
// while a waited, 0 if not, negative on a HIP error.
//   hipcc --offload-arch=gfx950 -O2 -shared -fPIC -o tools/_probe_lib.so tools/probe_lib.cpp
#include <hip/hip_runtime.h>

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

extern "C" int probe_pair(void *a, void *b, int stall) {
  static unsigned *flag = nullptr;
  static int cus = 0;
  if (!flag) {
    if (hipMalloc(&flag, 256) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0) != hipSuccess) return -1;
    if (hipFuncSetAttribute((const void *)k_wait, hipFuncAttributeMaxDynamicSharedMemorySize, 65536) != hipSuccess)
      return -1;
  }
  if (hipMemset(flag, 0, 8) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return -2;
  if (stall)
    hipLaunchKernelGGL(k_wait, dim3(6 * cus), dim3(64), 65536, (hipStream_t)a, flag, 50000ull);
  else
    hipLaunchKernelGGL(k_wait, dim3(1), dim3(64), 0, (hipStream_t)a, flag, 2000000ull);
  hipLaunchKernelGGL(k_set, dim3(1), dim3(64), 0, (hipStream_t)b, flag);
  if (hipDeviceSynchronize() != hipSuccess) return -3;
  unsigned seen = 0;
  if (hipMemcpy(&seen, flag + 1, 4, hipMemcpyDeviceToHost) != hipSuccess) return -4;
  return (int)seen;
}
