// Is device memory writable by the host here (large BAR)?  Allocates
// fine-grained / uncached device memory, prints its pointer attributes, and
// if it has a host pointer writes and reads it from the host and has a kernel
// read the host's value back.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <chrono>

__global__ void rd(const uint64_t *p, uint64_t *out) {
  out[0] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
  const unsigned flags[] = {hipDeviceMallocFinegrained, hipDeviceMallocUncached};
  uint64_t *d_out = nullptr, h_out = 0;
  (void)hipMalloc(&d_out, 8);
  for (unsigned f : flags) {
    void *p = nullptr;
    hipError_t e = hipExtMallocWithFlags(&p, 4096, f);
    hipPointerAttribute_t a{};
    hipError_t e2 = hipPointerGetAttributes(&a, p);
    printf("flags %u: malloc %d ptr %p attr %d type %d hostPointer %p devicePointer %p\n", f, (int)e,
           p, (int)e2, (int)a.type, a.hostPointer, a.devicePointer);
    fflush(stdout);
    if (e == hipSuccess) {  // the device address itself (one address space); a fault ends this probe
      volatile uint64_t *hp = (volatile uint64_t *)(a.hostPointer ? a.hostPointer : p);
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < 512; ++i) hp[i] = 0x1234567800000000ull + i;
      auto t1 = std::chrono::steady_clock::now();
      uint64_t s = 0;
      for (int i = 0; i < 8; ++i) s += hp[i];
      auto t2 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(rd, dim3(1), dim3(1), 0, 0, (const uint64_t *)a.devicePointer, d_out);
      (void)hipMemcpy(&h_out, d_out, 8, hipMemcpyDeviceToHost);
      printf("  512 host writes %.2f us, 8 host reads %.2f us (sum %llx); kernel read %llx\n",
             std::chrono::duration<double>(t1 - t0).count() * 1e6,
             std::chrono::duration<double>(t2 - t1).count() * 1e6, (unsigned long long)s,
             (unsigned long long)h_out);
      fflush(stdout);
    }
    (void)hipFree(p);
  }
  return 0;
}
