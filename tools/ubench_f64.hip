// ubench_f64.hip -- diagnostic microbenchmark (not part of the product):
// issue cost and dependent latency of the f64 VALU instructions the
// sum-product loop is made of, on gfx950, by waves per SIMD and chain count.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/ubench_f64 tools/ubench_f64.hip
//   ./ubench_f64          -> one line per (op, waves/SIMD, chains): cycles per
//                            wave-instruction per SIMD (s_memtime shader clocks)
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>

constexpr int kIters = 2048;

template <int OP, int C>
__global__ void __launch_bounds__(1024) kern(double *out, unsigned long long *cyc, double seed) {
  double v[C];
#pragma unroll
  for (int c = 0; c < C; ++c) v[c] = seed + threadIdx.x * 1e-9 + c;
  const double a = 1.0000001, b = 1e-9;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        if constexpr (OP == 0) v[c] = __builtin_fma(v[c], a, b);
        if constexpr (OP == 1) v[c] = v[c] + b;
        if constexpr (OP == 2) v[c] = v[c] * a;
        if constexpr (OP == 3) v[c] = __builtin_amdgcn_rcp(v[c]);
        if constexpr (OP == 4) v[c] = __builtin_ldexp(v[c], 1 - 2 * (u & 1));
      }
    }
    asm volatile("" ::: "memory");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) s += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP, int C>
void run(const char *name, int waves_per_simd) {
  const int cus = 256;
  const int threads = 64 * 4 * waves_per_simd;  // one block per CU
  double *out;
  unsigned long long *cyc;
  hipMalloc(&out, sizeof(double) * cus * threads);
  hipMalloc(&cyc, sizeof(unsigned long long) * cus * threads / 64);
  hipLaunchKernelGGL((kern<OP, C>), dim3(cus), dim3(threads), 0, 0, out, cyc, 1.0);
  hipLaunchKernelGGL((kern<OP, C>), dim3(cus), dim3(threads), 0, 0, out, cyc, 1.0);
  hipDeviceSynchronize();
  const int nw = cus * threads / 64;
  unsigned long long *h = (unsigned long long *)malloc(sizeof(unsigned long long) * nw);
  hipMemcpy(h, cyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost);
  double mean = 0, mx = 0;
  for (int i = 0; i < nw; ++i) {
    mean += (double)h[i];
    mx = (double)h[i] > mx ? (double)h[i] : mx;
  }
  mean /= nw;
  const double insts = (double)kIters * 8 * C;
  // per SIMD: waves_per_simd waves each issued `insts` instructions in ~mx cycles
  printf("%-6s waves/SIMD=%d chains=%d  per-wave cycles/inst=%.2f  SIMD cycles/inst=%.2f\n", name,
         waves_per_simd, C, mean / insts, mx / (insts * waves_per_simd));
  free(h);
  hipFree(out);
  hipFree(cyc);
}

template <int OP>
void sweep(const char *name) {
  for (int w : {1, 2, 3, 4}) {
    run<OP, 1>(name, w);
    run<OP, 2>(name, w);
    run<OP, 4>(name, w);
    run<OP, 8>(name, w);
  }
}

int main() {
  sweep<0>("fma64");
  sweep<1>("add64");
  sweep<2>("mul64");
  sweep<3>("rcp64");
  sweep<4>("ldexp");
  return 0;
}
