// ldpc_aux.hip -- device-side encoder, channel and error counting (SURVEY 8(f)
// rows 2 and 3): what the reference's encoder block (lib/ldpc_encoder_bc_impl.cc)
// and BER program (apps/ldpc_lapack.cpp:533-811) do on the host, so synthetic
// batches and BER sweeps never leave HBM.
//
//   encode_small   codes within the small-code limits: parity = A d over GF(2),
//                  A = H_p^-1 H_d (bit rows, built once on the host); one wave
//                  per frame, lane = parity row, data words from ballots.
//   encode_ira     IRA / DVB-S2-style codes (parity part = accumulator
//                  staircase): s_j = XOR of row j's information bits, parity =
//                  prefix-XOR of s; one 256-thread block per frame (segmented
//                  scan through LDS).
//   random_bits    Philox4x32-10 counter-based bits (seeded, reproducible).
//   bpsk_awgn      x = 2c - 1 + sigma * n, n ~ N(0,1) by Box-Muller on Philox
//                  output; sigma = sqrt(10^(-EbN0/10)) is the reference's
//                  convention (apps/ldpc_lapack.cpp:629-636).
//   count_errors   per-frame count of positions where two 0/1 arrays differ
//                  (biterr, apps/ldpc_lapack.cpp:508-517, before the division).
//   gather_windows the windows a decoder block asks for (any start sample, either
//                  polarity) copied out of one staged sample span into frames.
#include <hip/hip_runtime.h>

#include "ldpc_aux.hpp"

namespace ldpc {
namespace {

struct u4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u4 philox(uint64_t ctr, uint32_t stream, uint64_t seed) {
  u4 c{(uint32_t)ctr, (uint32_t)(ctr >> 32), stream, 0x2545F491u};
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__global__ void __launch_bounds__(256) k_random_bits(uint8_t *out, int64_t n, uint64_t seed) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= n) return;
  const u4 r = philox((uint64_t)(i4 >> 2), 1u, seed);
  const uint32_t v[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (i4 + k < n) out[i4 + k] = (uint8_t)(v[k] >> 31);
}

__global__ void __launch_bounds__(256) k_bpsk_awgn(const uint8_t *bits, int64_t n, float sigma,
                                                   uint64_t seed, float *out) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 >= n) return;
  const u4 r = philox((uint64_t)(i4 >> 2), 2u, seed);
  // two Box-Muller pairs; u1 in (0, 1] keeps the log finite
  const float u1a = ((float)r.x + 1.0f) * 2.3283064e-10f, u2a = (float)r.y * 2.3283064e-10f;
  const float u1b = ((float)r.z + 1.0f) * 2.3283064e-10f, u2b = (float)r.w * 2.3283064e-10f;
  const float ra = sqrtf(-2.0f * logf(fminf(u1a, 1.0f))), rb = sqrtf(-2.0f * logf(fminf(u1b, 1.0f)));
  float sa, ca, sb, cb;
  sincospif(2.0f * u2a, &sa, &ca);
  sincospif(2.0f * u2b, &sb, &cb);
  const float nz[4] = {ra * ca, ra * sa, rb * cb, rb * sb};
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (i4 + k < n) out[i4 + k] = (2.0f * (float)(bits[i4 + k] & 1) - 1.0f) + sigma * nz[k];
}

__global__ void __launch_bounds__(256) k_count_errors(const uint8_t *a, const uint8_t *b,
                                                      int64_t per_frame, int32_t *counts) {
  __shared__ int part[4];
  const int64_t base = (int64_t)blockIdx.x * per_frame;
  int c = 0;
  for (int64_t i = threadIdx.x; i < per_frame; i += 256)
    c += ((a[base + i] ^ b[base + i]) & 1) ? 1 : 0;
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) counts[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// One wave per frame.  A: M rows of KW 64-bit words (bit i of word w = data
// bit 64w + i).  Codeword = [parity (M) | data (K)] in the decoder's column
// order.
template <int KW>
__global__ void __launch_bounds__(64) k_encode_small(const uint64_t *A, int M, int K,
                                                     const uint8_t *data, uint8_t *cw) {
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  const uint8_t *d = data + b * K;
  uint8_t *out = cw + b * (int64_t)(M + K);
  uint64_t dw[KW];
#pragma unroll
  for (int w = 0; w < KW; ++w) {
    const int i = 64 * w + lane;
    const uint8_t bit = i < K ? (d[i] & 1) : 0;
    dw[w] = __ballot(bit != 0);
    if (i < K) out[M + i] = bit;
  }
  for (int j = lane; j < M; j += 64) {
    int par = 0;
#pragma unroll
    for (int w = 0; w < KW; ++w) par ^= __popcll(A[(int64_t)j * KW + w] & dw[w]);
    out[j] = (uint8_t)(par & 1);
  }
}

// One 256-thread block per frame; thread t owns rows [t*seg, (t+1)*seg).
__global__ void __launch_bounds__(256) k_encode_ira(const int32_t *rp, const int32_t *ci, int M,
                                                    int K, const uint8_t *data, uint8_t *cw) {
  __shared__ uint8_t tot[256];
  const int t = threadIdx.x;
  const int64_t b = blockIdx.x;
  const uint8_t *d = data + b * K;
  uint8_t *out = cw + b * (int64_t)(M + K);
  for (int i = t; i < K; i += 256) out[M + i] = d[i] & 1;
  const int seg = (M + 255) / 256;
  const int j0 = min(M, t * seg), j1 = min(M, j0 + seg);
  uint8_t acc = 0;
  for (int j = j0; j < j1; ++j)
    for (int e = rp[j]; e < rp[j + 1]; ++e)
      if (ci[e] >= M) acc ^= d[ci[e] - M] & 1;
  tot[t] = acc;
  __syncthreads();
  // exclusive XOR-scan of the segment totals (256 entries, one thread)
  if (t == 0) {
    uint8_t run = 0;
    for (int i = 0; i < 256; ++i) {
      const uint8_t v = tot[i];
      tot[i] = run;
      run ^= v;
    }
  }
  __syncthreads();
  uint8_t p = tot[t];
  for (int j = j0; j < j1; ++j) {
    uint8_t s = 0;
    for (int e = rp[j]; e < rp[j + 1]; ++e)
      if (ci[e] >= M) s ^= d[ci[e] - M] & 1;
    p ^= s;
    out[j] = p;
  }
}

inline unsigned blocks_for(int64_t n, int per_block) {
  return (unsigned)((n + per_block - 1) / per_block);
}

}  // namespace

int launch_random_bits(uint8_t *out, int64_t n, uint64_t seed, void *stream) {
  if (n <= 0) return 0;
  k_random_bits<<<blocks_for(n, 1024), 256, 0, (hipStream_t)stream>>>(out, n, seed);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_bpsk_awgn(const uint8_t *bits, int64_t n, float sigma, uint64_t seed, float *out,
                     void *stream) {
  if (n <= 0) return 0;
  k_bpsk_awgn<<<blocks_for(n, 1024), 256, 0, (hipStream_t)stream>>>(bits, n, sigma, seed, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_count_errors(const uint8_t *a, const uint8_t *b, int64_t per_frame, int B,
                        int32_t *counts, void *stream) {
  if (B <= 0) return 0;
  k_count_errors<<<B, 256, 0, (hipStream_t)stream>>>(a, b, per_frame, counts);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_encode_small(const uint64_t *A, int M, int K, const uint8_t *data, int B, uint8_t *cw,
                        void *stream) {
  if (B <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int kw = (K + 63) / 64;
  switch (kw) {
    case 1: k_encode_small<1><<<B, 64, 0, st>>>(A, M, K, data, cw); break;
    case 2: k_encode_small<2><<<B, 64, 0, st>>>(A, M, K, data, cw); break;
    case 3: k_encode_small<3><<<B, 64, 0, st>>>(A, M, K, data, cw); break;
    case 4: k_encode_small<4><<<B, 64, 0, st>>>(A, M, K, data, cw); break;
    default: return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_encode_ira(const int32_t *rp, const int32_t *ci, int M, int K, const uint8_t *data,
                      int B, uint8_t *cw, void *stream) {
  if (B <= 0) return 0;
  k_encode_ira<<<B, 256, 0, (hipStream_t)stream>>>(rp, ci, M, K, data, cw);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

namespace {
__global__ void __launch_bounds__(256) k_gather_windows(const float *span, const int64_t *win,
                                                        int64_t total, int N, float *out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  const int64_t b = t / N, i = t - b * N;
  const int64_t w = win[b];
  const float v = span[(w >> 1) + i];
  out[t] = (w & 1) ? -v : v;  // negation is exact: the decoder sees tx = -Re exactly
}
}  // namespace

int launch_gather_windows(const float *span, const int64_t *win, int B, int N, float *out,
                          void *stream) {
  const int64_t total = (int64_t)B * N;
  if (total <= 0) return 0;
  hipLaunchKernelGGL(k_gather_windows, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, span, win, total, N, out);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Stream concurrency probe (ldpc_ctx_streams): k_probe_wait spins on a flag
// for at most `deadline` ticks of the 100 MHz clock and records what it saw;
// k_probe_set raises the flag.  Enqueued on two streams, the wait sees the
// flag only if the two run at the same time -- on one hardware queue the set
// runs after the wait has given up.
namespace {
__global__ void __launch_bounds__(64) k_probe_wait(uint32_t *flag, uint64_t deadline) {
  if (threadIdx.x != 0) return;
  typedef __attribute__((address_space(1))) uint32_t gu32;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t v = 0;
  while ((v = __hip_atomic_load((gu32 *)flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0u &&
         __builtin_amdgcn_s_memrealtime() - t0 < deadline)
    __builtin_amdgcn_s_sleep(2);
  __hip_atomic_store((gu32 *)(flag + 1), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void __launch_bounds__(64) k_probe_set(uint32_t *flag) {
  typedef __attribute__((address_space(1))) uint32_t gu32;
  if (threadIdx.x == 0) __hip_atomic_store((gu32 *)flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace

int launch_probe_touch(uint32_t *flag, void *stream) {
  hipLaunchKernelGGL(k_probe_set, dim3(1), dim3(64), 0, (hipStream_t)stream, flag);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Device timestamps of one spin (tests): out[0] = the 100 MHz clock when the
// kernel starts, out[1] when it has spun `ticks` and ends.  Two of them on
// two streams overlap in time iff the streams run side by side.
namespace {
__global__ void __launch_bounds__(64) k_stamp(uint64_t *out, uint64_t ticks) {
  if (threadIdx.x != 0) return;
  typedef __attribute__((address_space(1))) uint64_t gu64;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  __hip_atomic_store((gu64 *)out, t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((gu64 *)(out + 1), __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace

int launch_stamp(uint64_t *out, uint64_t ticks, void *stream) {
  hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, (hipStream_t)stream, out, ticks);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_probe_pair(uint32_t *flag, uint64_t deadline, void *wait_stream, void *set_stream) {
  hipLaunchKernelGGL(k_probe_wait, dim3(1), dim3(64), 0, (hipStream_t)wait_stream, flag, deadline);
  if (hipGetLastError() != hipSuccess) return -3;
  hipLaunchKernelGGL(k_probe_set, dim3(1), dim3(64), 0, (hipStream_t)set_stream, flag);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace ldpc
