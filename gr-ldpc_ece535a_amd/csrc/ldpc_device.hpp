// ldpc_device.hpp -- device-side arithmetic shared by the small-code
// kernels (ldpc_kernels.hip) and the large-code kernels (ldpc_graph.hip), so
// both repeat the reference's per-edge operations identically.
#pragma once

#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>

#include "ldpc_math.hpp"

namespace ldpc {

// Arithmetic per precision mode (include/ldpc_hip.h LDPC_PREC_*):
//   0 F64       double, compact two-range tanh (glibc's double near 1, <= 3 ulp
//               elsewhere) and table-driven
//               log (<= 1 ulp) of ldpc_math.hpp, reciprocal-based divisions
//   1 F32       float, ROCm libm
//   2 F64_LIBM  double, fdlibm tanh bit-identical to glibc's, fdlibm log
template <int PREC>
struct Math;
// The 512-entry log table of LDPC_PREC_F64's check message (ldpc_logtab.hpp);
// kernels stage it in LDS (stage_logtab) and pass that copy to check_msg.
__device__ const fm::LogTabEntry kLogTab[1 << fm::kLogTabBits] = {LDPC_LOGTAB_ENTRIES};

// Every thread of the block takes part; one __syncthreads.
__device__ __forceinline__ void stage_logtab(fm::LogTabEntry *lds) {
  for (int i = threadIdx.x; i < (1 << fm::kLogTabBits); i += blockDim.x) lds[i] = kLogTab[i];
  __syncthreads();
}

// tanh_half(m) = tanh(m / 2) (:509); check_msg(T, tab) = log((1+T)/(1-T))
// (:513), tab = the LDS copy of kLogTab (used by LDPC_PREC_F64 only).
template <>
struct Math<0> {
  typedef double Real;
#ifdef LDPC_TANH_SINGLE_RANGE  // A/B only: loses parity on large-amplitude frames
  static __device__ __forceinline__ double tanh_half(double m) { return fm::tanh_half_fast(m); }
#else
  static __device__ __forceinline__ double tanh_half(double m) { return fm::tanh_half_acc(m); }
#endif
  static __device__ __forceinline__ double check_msg(double T, const fm::LogTabEntry *tab) {
    return fm::log_ratio_tab(T, tab);
  }
  static __device__ __forceinline__ double abs_(double x) { return ::fabs(x); }
  static __device__ __forceinline__ double max_() { return DBL_MAX; }
};
template <>
struct Math<2> : Math<0> {
  static __device__ __forceinline__ double tanh_half(double m) { return fm::tanh_f64_bf(m / 2.0); }
  static __device__ __forceinline__ double check_msg(double T, const fm::LogTabEntry *) {
    return fm::log_f64_bf((1.0 + T) / (1.0 - T));  // IEEE division
  }
};
template <>
struct Math<1> {
  typedef float Real;
  static __device__ __forceinline__ float tanh_half(float m) { return ::tanhf(m / 2.0f); }
  static __device__ __forceinline__ float check_msg(float T, const fm::LogTabEntry *) {
    return ::logf((1.0f + T) / (1.0f - T));
  }
  static __device__ __forceinline__ float abs_(float x) { return ::fabsf(x); }
  static __device__ __forceinline__ float max_() { return FLT_MAX; }
};

// sign(), lib/ldpc_decoder_cb_impl.cc:574-578 (sign(0) == 0).
template <typename Real>
__device__ __forceinline__ int sgn(Real v) {
  return (v > Real(0)) - (v < Real(0));
}

}  // namespace ldpc
