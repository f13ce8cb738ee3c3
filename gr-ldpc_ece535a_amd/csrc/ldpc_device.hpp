// ldpc_device.hpp -- device-side arithmetic shared by the small-code
// kernels (ldpc_kernels.hip) and the large-code kernels (ldpc_graph.hip), so
// both repeat the reference's per-edge operations identically.
#pragma once

#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>

#include "ldpc_exact.hpp"
#include "ldpc_math.hpp"

namespace ldpc {

// Arithmetic per precision mode (include/ldpc_hip.h LDPC_PREC_*):
//   0 F64       double, glibc's tanh(m/2) and log((1+T)/(1-T)) bit for bit
//               (ldpc_exact.hpp), n quotients per shared reciprocal with
//               correctly rounded results -- the reference's arithmetic
//   2 F64_LIBM  the same functions one value at a time (no shared
//               reciprocal): an independent evaluation of mode 0
//   3 F64_FAST  double, compact approximations (ldpc_math.hpp): tanh within
//               3 ulp of glibc, table log within 1 ulp -- faster, not exact
//   1 F32       float, ROCm libm
// tanh_half(m) = tanh(m / 2) (:509); check_msg(T, tab) = log((1+T)/(1-T))
// (:513); the _n forms take n independent operands (a lane's edge slots /
// column entries) so their divisions can share one reciprocal.  `Tab` is
// the log table the kernels stage in LDS (stage_tab) and pass back in.
template <int PREC>
struct Math;

// glibc's log table and expm1's per-k constants (ldpc_exact.hpp)
__device__ const ex::ExTab kExTab = ex::make_ex_tab();
// The 512-entry table of LDPC_PREC_F64_FAST's log (ldpc_logtab.hpp).
__device__ const fm::LogTabEntry kLogTab[1 << fm::kLogTabBits] = {LDPC_LOGTAB_ENTRIES};

template <>
struct Math<0> {
  typedef double Real;
  typedef ex::ExTab Tab;
  static constexpr int kTabN = 1;
  static __device__ __forceinline__ const Tab *tab_src() { return &kExTab; }
  template <int n>
  static __device__ __forceinline__ void tanh_half_n(const double (&m)[n], double (&z)[n],
                                                     const Tab *tab) {
    ex::tanh_half_n<n>(m, z, tab);
  }
  template <int n>
  static __device__ __forceinline__ void check_msg_n(const double (&T)[n], const Tab *tab,
                                                     double (&E)[n]) {
    ex::log_ratio_n<n>(T, tab, E);
  }
  static __device__ __forceinline__ double tanh_half(double m, const Tab *tab) {
    const double v[1] = {m};
    double z[1];
    ex::tanh_half_n<1>(v, z, tab);
    return z[0];
  }
  static __device__ __forceinline__ double check_msg(double T, const Tab *tab) {
    const double v[1] = {T};
    double e[1];
    ex::log_ratio_n<1>(v, tab, e);
    return e[0];
  }
  static __device__ __forceinline__ double abs_(double x) { return ::fabs(x); }
  static __device__ __forceinline__ double max_() { return DBL_MAX; }
};
template <>
struct Math<2> : Math<0> {
  template <int n>
  static __device__ __forceinline__ void tanh_half_n(const double (&m)[n], double (&z)[n],
                                                     const Tab *tab) {
#pragma unroll
    for (int i = 0; i < n; ++i) z[i] = Math<0>::tanh_half(m[i], tab);
  }
  template <int n>
  static __device__ __forceinline__ void check_msg_n(const double (&T)[n], const Tab *tab,
                                                     double (&E)[n]) {
#pragma unroll
    for (int i = 0; i < n; ++i) E[i] = Math<0>::check_msg(T[i], tab);
  }
};
template <>
struct Math<3> {
  typedef double Real;
  typedef fm::LogTabEntry Tab;
  static constexpr int kTabN = 1 << fm::kLogTabBits;
  static __device__ __forceinline__ const Tab *tab_src() { return kLogTab; }
#ifdef LDPC_TANH_SINGLE_RANGE  // A/B only: loses accuracy on large-amplitude frames
  static __device__ __forceinline__ double tanh_half(double m, const Tab * = nullptr) {
    return fm::tanh_half_fast(m);
  }
#else
  static __device__ __forceinline__ double tanh_half(double m, const Tab * = nullptr) {
    return fm::tanh_half_acc(m);
  }
#endif
  static __device__ __forceinline__ double check_msg(double T, const Tab *tab) {
    return fm::log_ratio_tab(T, tab);
  }
  template <int n>
  static __device__ __forceinline__ void tanh_half_n(const double (&m)[n], double (&z)[n],
                                                     const Tab *) {
#pragma unroll
    for (int i = 0; i < n; ++i) z[i] = tanh_half(m[i]);
  }
  template <int n>
  static __device__ __forceinline__ void check_msg_n(const double (&T)[n], const Tab *tab,
                                                     double (&E)[n]) {
#pragma unroll
    for (int i = 0; i < n; ++i) E[i] = check_msg(T[i], tab);
  }
  static __device__ __forceinline__ double abs_(double x) { return ::fabs(x); }
  static __device__ __forceinline__ double max_() { return DBL_MAX; }
};
template <>
struct Math<1> {
  typedef float Real;
  typedef float Tab;  // no table
  static constexpr int kTabN = 0;
  static __device__ __forceinline__ const Tab *tab_src() { return nullptr; }
  static __device__ __forceinline__ float tanh_half(float m, const Tab * = nullptr) {
    return ::tanhf(m / 2.0f);
  }
  static __device__ __forceinline__ float check_msg(float T, const Tab *) {
    return ::logf((1.0f + T) / (1.0f - T));
  }
  template <int n>
  static __device__ __forceinline__ void tanh_half_n(const float (&m)[n], float (&z)[n],
                                                     const Tab *) {
#pragma unroll
    for (int i = 0; i < n; ++i) z[i] = tanh_half(m[i]);
  }
  template <int n>
  static __device__ __forceinline__ void check_msg_n(const float (&T)[n], const Tab *tab,
                                                     float (&E)[n]) {
#pragma unroll
    for (int i = 0; i < n; ++i) E[i] = check_msg(T[i], tab);
  }
  static __device__ __forceinline__ float abs_(float x) { return ::fabsf(x); }
  static __device__ __forceinline__ float max_() { return FLT_MAX; }
};

// log_ratio_n with glibc's |q - 1| < 1/16 path evaluated once per 64 such
// ratios of the wave instead of once per slot that has any: about a fifth of
// the check messages take that path in steady state, so with per-slot
// branches every slot would run both paths.  The near-1 ratios are packed
// (ballot + mbcnt prefix) into `scratch` -- this wave's LDS, >= 64 n
// doubles, free for the duration of the call --, evaluated densely, and read
// back by their lanes.  Same functions, same results as ex::log_ratio_n.
// A wave's LDS accesses execute in issue order, so only the compiler must be
// kept from reordering them (the empty asm with a memory clobber).
template <int n>
__device__ __forceinline__ void log_ratio_n_packed(const double (&T)[n],
                                                   const ex::ExTab *tab, double (&E)[n],
                                                   double *scratch, int lane, uint32_t zero_at) {
  double q[n];
  // wave-uniform at once (a per-lane flag held across the loop below costs a
  // VGPR and two conversions per call)
  const bool any_special = ex::ratio_n<n>(T, q);  // wave-uniform
  // q = 1 exactly (T = +-0: every padding cell, the rows with a degree-1
  // column; or a tiny |T|) is glibc's log(1) = +0 without evaluating it: those
  // lanes read a +0.0 the caller keeps at scratch[zero_at] (a zero cell,
  // never written during a frame: one address, an LDS broadcast) instead of
  // a packed result.  They are
  // half the near-1 operands of the headline workload, and without them 9 %
  // rather than 60 % of wave-iterations need a second packed pass
  // (tools/path_stats.py).
  uint32_t pos[n];
  bool near[n], packed[n];
  uint32_t base = 0;  // wave-uniform
#pragma unroll
  for (int i = 0; i < n; ++i) {
    E[i] = ex::log_main(q[i], tab->log);
    near[i] = ex::log_is_near1(q[i]);
    const bool unit = q[i] == 1.0;
    packed[i] = near[i] && !unit;
    const uint64_t m = __builtin_amdgcn_ballot_w64(packed[i]);
    pos[i] = unit ? zero_at
                  : base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    base += (uint32_t)__builtin_popcountll(m);
  }
  asm volatile("" ::: "memory");
  if (base != 0) {
#pragma unroll
    for (int i = 0; i < n; ++i)
      if (packed[i]) scratch[pos[i]] = q[i];
    asm volatile("" ::: "memory");
    for (uint32_t p = 0; p < base; p += 64) {
      const uint32_t idx = p + (uint32_t)lane;
      if (idx < base) scratch[idx] = ex::log_near1(scratch[idx]);
    }
    asm volatile("" ::: "memory");
  }
#pragma unroll
  for (int i = 0; i < n; ++i)
    if (near[i]) E[i] = scratch[pos[i]];
  asm volatile("" ::: "memory");
  if (any_special) {
    LDPC_EX_COLD();
    ex::ratio_fix_n<n>(T, E);
  }
}

// LDS copy of mode PREC's log table (sized 1 for modes without one); every
// thread of the block takes part, one __syncthreads.
template <int PREC>
struct TabLds {
  typedef typename Math<PREC>::Tab Tab;
  static constexpr int kN = Math<PREC>::kTabN > 0 ? Math<PREC>::kTabN : 1;
};
template <int PREC>
__device__ __forceinline__ void stage_tab(typename Math<PREC>::Tab *lds) {
  if constexpr (Math<PREC>::kTabN > 0) {
    typedef typename Math<PREC>::Tab Tab;
    static_assert(sizeof(Tab) % 4 == 0, "tables are copied in 32-bit words");
    constexpr int words = (int)(sizeof(Tab) / 4) * Math<PREC>::kTabN;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(Math<PREC>::tab_src());
    uint32_t *dst = reinterpret_cast<uint32_t *>(lds);
    for (int i = threadIdx.x; i < words; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
  }
}

// sign(), lib/ldpc_decoder_cb_impl.cc:574-578 (sign(0) == 0).
template <typename Real>
__device__ __forceinline__ int sgn(Real v) {
  return (v > Real(0)) - (v < Real(0));
}

}  // namespace ldpc
