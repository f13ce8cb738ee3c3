// ubench_valu.hip -- diagnostic microbenchmark (not part of the product):
// issue cost on gfx950 of the non-FMA VALU instructions the exact
// sum-product loop is made of (integer / select / move / compare / convert),
// measured like tools/ubench_f64.hip: 4 waves per SIMD, 4 independent chains
// per wave, cycles per wave-instruction per SIMD (s_memtime shader clocks).
// The product's roofline weights come from these numbers.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/bin/ubench_valu tools/ubench_valu.hip
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int kIters = 1024;
constexpr int kChains = 4;

#define OP1(INS) asm volatile(INS " %0, %0, %1" : "+v"(v[c]) : "v"(w));
template <int OP>
__global__ void __launch_bounds__(1024) kern(uint64_t *out, unsigned long long *cyc, uint64_t seed) {
  uint64_t v[kChains];
  uint32_t s[kChains];
  double d[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    v[c] = seed + threadIdx.x + c;
    s[c] = (uint32_t)v[c];
    d[c] = 1.0 + threadIdx.x * 1e-9 + c;
  }
  const uint32_t w = (uint32_t)seed | 1u;
  const double dw = 1.5;
  const uint64_t mask = __builtin_amdgcn_ballot_w64(threadIdx.x & 1);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
#pragma unroll
      for (int c = 0; c < kChains; ++c) {
        if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(s[c]) : "v"(w));
        if constexpr (OP == 1) asm volatile("v_and_b32 %0, %0, %1" : "+v"(s[c]) : "v"(w));
        if constexpr (OP == 2)  // mask in an SGPR pair written once before the loop
          asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(s[c]) : "v"(w), "s"(mask));
        if constexpr (OP == 3) asm volatile("v_mov_b64 %0, %1" : "=v"(v[c]) : "v"(v[(c + 1) % kChains]));
        if constexpr (OP == 4) asm volatile("v_lshl_add_u64 %0, %0, 0, -1" : "+v"(v[c]));
        if constexpr (OP == 5) asm volatile("v_cmp_lt_f64 vcc, %0, %1" ::"v"(d[c]), "v"(dw) : "vcc");
        if constexpr (OP == 6) asm volatile("v_max_f64 %0, %0, %1" : "+v"(d[c]) : "v"(dw));
        if constexpr (OP == 7) asm volatile("v_trunc_f64 %0, %0" : "+v"(d[c]));
        if constexpr (OP == 8) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(d[c]) : "v"(s[c]));
        if constexpr (OP == 9) asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(s[c]) : "v"(d[c]));
        if constexpr (OP == 10) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[c]) : "v"(dw));
        if constexpr (OP == 11) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[c]) : "v"(dw));
        if constexpr (OP == 12) asm volatile("v_cmp_gt_u32 vcc, %0, %1" ::"v"(s[c]), "v"(w) : "vcc");
        if constexpr (OP == 13) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(s[c]) : "v"(w));
        if constexpr (OP == 14) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[c]));
        if constexpr (OP == 15)  // compare writing a mask, then a select reading it
          asm volatile("v_cmp_gt_u32_e64 s[40:41], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[40:41]"
                       : "+v"(s[c]) : "v"(w) : "s40", "s41");
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) acc += v[c] + s[c] + (uint64_t)d[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
void run(const char *name, int waves_per_simd) {
  const int cus = 256;
  const int threads = 64 * 4 * waves_per_simd;  // one block per CU
  uint64_t *out;
  unsigned long long *cyc;
  hipMalloc(&out, sizeof(uint64_t) * cus * threads);
  hipMalloc(&cyc, sizeof(unsigned long long) * cus * threads / 64);
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL((kern<OP>), dim3(cus), dim3(threads), 0, 0, out, cyc, 12345ull);
  hipDeviceSynchronize();
  const int nw = cus * threads / 64;
  unsigned long long *h = (unsigned long long *)malloc(sizeof(unsigned long long) * nw);
  hipMemcpy(h, cyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost);
  double mx = 0;
  for (int i = 0; i < nw; ++i) mx = (double)h[i] > mx ? (double)h[i] : mx;
  const double insts = (double)kIters * 8 * kChains * (OP == 15 ? 2 : 1);
  printf("%-16s waves/SIMD=%d chains=%d  SIMD cycles/inst=%.2f\n", name, waves_per_simd, kChains,
         mx / (insts * waves_per_simd));
  free(h);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w : {2, 4}) {
    run<0>("v_add_u32", w);
    run<1>("v_and_b32", w);
    run<13>("v_xor_b32", w);
    run<2>("v_cndmask_b32", w);
    run<15>("v_cmp+v_cndmask", w);
    run<3>("v_mov_b64", w);
    run<4>("v_lshl_add_u64", w);
    run<12>("v_cmp_gt_u32", w);
    run<5>("v_cmp_lt_f64", w);
    run<6>("v_max_f64", w);
    run<7>("v_trunc_f64", w);
    run<8>("v_cvt_f64_i32", w);
    run<9>("v_cvt_i32_f64", w);
    run<10>("v_add_f64", w);
    run<11>("v_fma_f64", w);
    run<14>("v_rcp_f64", w);
  }
  return 0;
}
