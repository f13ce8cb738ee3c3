// ldpc_math.hpp -- double-precision tanh / expm1 / log for the decode kernels.
//
// The reference's check-node update calls glibc's tanh and log
// (lib/ldpc_decoder_cb_impl.cc:509, :513).  ROCm's ocml versions cost 165 and
// 98 VALU instructions on gfx950; the ones below are the classic fdlibm
// algorithms (Sun Microsystems, 1993, freely distributable), which is also
// what glibc's double tanh/expm1 are, written as straight-line double
// arithmetic without fused multiply-add so host and device round alike:
//   * tanh_f64 / expm1_f64: fdlibm s_tanh.c / s_expm1.c -- tests/test_math.py
//     checks them bit for bit against the host libm on the decoder's range;
//   * log_f64: fdlibm e_log.c (< 1 ulp).  glibc >= 2.28 uses a table-driven
//     log instead, so results can differ from the oracle's in the last bit.
// Header-only, __host__ __device__ so the CPU tests run the same code.
#pragma once

#include <stdint.h>
#include <string.h>

#ifndef LDPC_HD
#if defined(__HIPCC__)
#define LDPC_HD __host__ __device__ __forceinline__
#else
#define LDPC_HD inline
#endif
#endif

#include "ldpc_logtab.hpp"

namespace ldpc {
namespace fm {

LDPC_HD uint32_t hi_word(double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  return (uint32_t)(u >> 32);
}
LDPC_HD uint32_t lo_word(double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  return (uint32_t)u;
}
LDPC_HD double from_words(uint32_t hi, uint32_t lo) {
  const uint64_t u = ((uint64_t)hi << 32) | lo;
  double x;
  memcpy(&x, &u, 8);
  return x;
}
LDPC_HD double with_hi(double x, uint32_t hi) { return from_words(hi, lo_word(x)); }

// fdlibm s_expm1.c (polynomial grouped as in glibc's copy)
LDPC_HD double expm1_f64(double x) {
  const double o_threshold = 7.09782712893383973096e+02;
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  const double invln2 = 1.44269504088896338700e+00;
  const double Q1 = -3.33333333333331316428e-02;
  const double Q2 = 1.58730158725481460165e-03;
  const double Q3 = -7.93650757867487942473e-05;
  const double Q4 = 4.00821782732936239552e-06;
  const double Q5 = -2.01099218183624371326e-07;
  double y, hi, lo, c = 0.0, t, e, hxs, hfx, r1, twopk;
  int k;
  uint32_t hx = hi_word(x);
  const uint32_t xsb = hx & 0x80000000u;
  hx &= 0x7fffffffu;
  if (hx >= 0x4043687Au) {  // |x| >= 56 ln2
    if (hx >= 0x40862E42u) {  // |x| >= 709.78
      if (hx >= 0x7ff00000u) {
        if (((hx & 0xfffffu) | lo_word(x)) != 0) return x + x;  // NaN
        return xsb == 0 ? x : -1.0;                             // exp(+-inf)-1
      }
      if (x > o_threshold) return __builtin_inf();
    }
    if (xsb != 0) return -1.0;  // x < -56 ln2
  }
  if (hx > 0x3fd62e42u) {  // |x| > 0.5 ln2
    if (hx < 0x3FF0A2B2u) {  // and |x| < 1.5 ln2
      if (xsb == 0) {
        hi = x - ln2_hi;
        lo = ln2_lo;
        k = 1;
      } else {
        hi = x + ln2_hi;
        lo = -ln2_lo;
        k = -1;
      }
    } else {
      k = (int)(invln2 * x + ((xsb == 0) ? 0.5 : -0.5));
      t = k;
      hi = x - t * ln2_hi;  // t*ln2_hi is exact here
      lo = t * ln2_lo;
    }
    x = hi - lo;
    c = (hi - x) - lo;
  } else if (hx < 0x3c900000u) {  // |x| < 2^-54
    return x;
  } else {
    k = 0;
  }
  hfx = 0.5 * x;
  hxs = x * hfx;
  // Estrin form, as glibc evaluates it (a Horner form differs in the last bit)
  const double R1 = 1.0 + hxs * Q1, h2 = hxs * hxs;
  const double R2 = Q2 + hxs * Q3, h4 = h2 * h2;
  const double R3 = Q4 + hxs * Q5;
  r1 = R1 + h2 * R2 + h4 * R3;
  t = 3.0 - r1 * hfx;
  e = hxs * ((r1 - t) / (6.0 - x * t));
  if (k == 0) return x - (x * e - hxs);
  twopk = from_words((uint32_t)(0x3ff + k) << 20, 0);  // 2^k
  e = (x * (e - c) - c);
  e -= hxs;
  if (k == -1) return 0.5 * (x - e) - 0.5;
  if (k == 1) {
    if (x < -0.25) return -2.0 * (e - (x + 0.5));
    return 1.0 + 2.0 * (x - e);
  }
  if (k <= -2 || k > 56) {  // exp(x)-1 suffices
    y = 1.0 - (e - x);
    if (k == 1024)
      y = y * 2.0 * 8.98846567431157953865e+307;  // 2^1023
    else
      y = y * twopk;
    return y - 1.0;
  }
  if (k < 20) {
    t = from_words(0x3ff00000u - (0x200000u >> k), 0);  // 1 - 2^-k
    y = t - (e - x);
    y = y * twopk;
  } else {
    t = from_words((uint32_t)(0x3ff - k) << 20, 0);  // 2^-k
    y = x - (e + t);
    y += 1.0;
    y = y * twopk;
  }
  return y;
}

// fdlibm s_tanh.c
LDPC_HD double tanh_f64(double x) {
  const int32_t jx = (int32_t)hi_word(x);
  const uint32_t ix = (uint32_t)jx & 0x7fffffffu;
  double t, z;
  if (ix >= 0x7ff00000u) {  // inf or NaN
    if (jx >= 0) return 1.0 / x + 1.0;
    return 1.0 / x - 1.0;
  }
  if (ix < 0x40360000u) {  // |x| < 22
    if (ix < 0x3c800000u) return x * (1.0 + x);  // |x| < 2^-55
    if (ix >= 0x3ff00000u) {                       // |x| >= 1
      t = expm1_f64(2.0 * __builtin_fabs(x));
      z = 1.0 - 2.0 / (t + 2.0);
    } else {
      t = expm1_f64(-2.0 * __builtin_fabs(x));
      z = -t / (t + 2.0);
    }
  } else {
    z = 1.0;  // |x| >= 22
  }
  return jx >= 0 ? z : -z;
}

// fdlibm e_log.c
LDPC_HD double log_f64(double x) {
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  const double two54 = 1.80143985094819840000e+16;
  const double Lg1 = 6.666666666666735130e-01;
  const double Lg2 = 3.999999999940941908e-01;
  const double Lg3 = 2.857142874366239149e-01;
  const double Lg4 = 2.222219843214978396e-01;
  const double Lg5 = 1.818357216161805012e-01;
  const double Lg6 = 1.531383769920937332e-01;
  const double Lg7 = 1.479819860511658591e-01;
  int32_t hx = (int32_t)hi_word(x);
  const uint32_t lx = lo_word(x);
  int32_t k = 0;
  if (hx < 0x00100000) {  // x < 2^-1022
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -__builtin_inf();  // log(+-0)
    if (hx < 0) return (x - x) / 0.0;  // log(-#) = NaN
    k -= 54;
    x *= two54;  // subnormal: scale up
    hx = (int32_t)hi_word(x);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  const int32_t i = (hx + 0x95f64) & 0x100000;
  x = with_hi(x, (uint32_t)(hx | (i ^ 0x3ff00000)));  // normalize x or x/2
  k += (i >> 20);
  const double f = x - 1.0;
  const double dk = (double)k;
  if ((0x000fffff & (2 + hx)) < 3) {  // -2^-20 <= f < 2^-20
    if (f == 0.0) return dk * ln2_hi + dk * ln2_lo;
    const double R = f * f * (0.5 - 0.33333333333333333 * f);
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
  const double s = f / (2.0 + f);
  const double z = s * s;
  int32_t ii = hx - 0x6147a;
  const double w = z * z;
  const int32_t j = 0x6b851 - hx;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  ii |= j;
  const double R = t2 + t1;
  if (ii > 0) {
    const double hfsq = 0.5 * f * f;
    return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  }
  return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// ---------------------------------------------------------------------------
// Branch-free restatements for the GPU: every path of the functions above is
// evaluated and the result selected, so divergent lanes do not serialise.
// Same operations in the same order, hence the same results (checked bit for
// bit against the branchy versions by tests/test_math.py).
// ---------------------------------------------------------------------------

LDPC_HD double sel(bool c, double a, double b) { return c ? a : b; }

// expm1 for -56 ln2 < x < 709.78 (the range tanh_f64_bf feeds it; any other
// finite input returns an unspecified value that the caller discards).
LDPC_HD double expm1_f64_bf(double x) {
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  const double invln2 = 1.44269504088896338700e+00;
  const double Q1 = -3.33333333333331316428e-02;
  const double Q2 = 1.58730158725481460165e-03;
  const double Q3 = -7.93650757867487942473e-05;
  const double Q4 = 4.00821782732936239552e-06;
  const double Q5 = -2.01099218183624371326e-07;
  const uint32_t hw = hi_word(x);
  const bool neg = (hw & 0x80000000u) != 0;
  const uint32_t hx = hw & 0x7fffffffu;
  const double x0 = x;
  // argument reduction: k = 0 (|x| <= 0.5 ln2), +-1 (< 1.5 ln2), else round
  const int kgen = (int)(invln2 * x + (neg ? -0.5 : 0.5));
  int k = hx < 0x3FF0A2B2u ? (neg ? -1 : 1) : kgen;
  k = hx > 0x3fd62e42u ? k : 0;
  const double tk = (double)k;
  const double hi = x - tk * ln2_hi;  // k == 0: hi == x, lo == 0, c == 0
  const double lo = tk * ln2_lo;
  x = hi - lo;
  const double c = (hi - x) - lo;
  const double hfx = 0.5 * x;
  const double hxs = x * hfx;
  const double R1 = 1.0 + hxs * Q1, h2 = hxs * hxs;
  const double R2 = Q2 + hxs * Q3, h4 = h2 * h2;
  const double R3 = Q4 + hxs * Q5;
  const double r1 = R1 + h2 * R2 + h4 * R3;
  double t = 3.0 - r1 * hfx;
  double e = hxs * ((r1 - t) / (6.0 - x * t));
  const double res0 = x - (x * e - hxs);  // k == 0
  const int kc = k < -1022 ? -1022 : (k > 1023 ? 1023 : k);
  const double twopk = from_words((uint32_t)(0x3ff + kc) << 20, 0);
  e = (x * (e - c) - c);
  e -= hxs;
  const double resm1 = 0.5 * (x - e) - 0.5;                                   // k == -1
  const double resp1 = sel(x < -0.25, -2.0 * (e - (x + 0.5)), 1.0 + 2.0 * (x - e));  // k == 1
  const double resbig = (1.0 - (e - x)) * twopk - 1.0;  // k <= -2 || k > 56
  const int klo = k < 1 ? 1 : (k > 19 ? 19 : k);
  const double t20 = from_words(0x3ff00000u - (0x200000u >> klo), 0);  // 1 - 2^-k
  const double reslt20 = (t20 - (e - x)) * twopk;                      // 2 <= k < 20
  const int khi = k < 20 ? 20 : (k > 56 ? 56 : k);
  const double tm = from_words((uint32_t)(0x3ff - khi) << 20, 0);  // 2^-k
  double yge = x - (e + tm);
  yge += 1.0;
  const double resge20 = yge * twopk;  // 20 <= k <= 56
  double r = sel(k < 20, reslt20, resge20);
  r = sel(k <= -2 || k > 56, resbig, r);
  r = sel(k == 1, resp1, r);
  r = sel(k == -1, resm1, r);
  r = sel(k == 0, res0, r);
  return sel(hx < 0x3c900000u, x0, r);  // |x| < 2^-54
}

LDPC_HD double tanh_f64_bf(double x) {
  const int32_t jx = (int32_t)hi_word(x);
  const uint32_t ix = (uint32_t)jx & 0x7fffffffu;
  const double a = __builtin_fabs(x);
  const bool big = ix >= 0x3ff00000u;  // |x| >= 1
  // |x| < 22 keeps the expm1 argument inside expm1_f64_bf's range
  const double arg = ix < 0x40360000u ? (big ? 2.0 * a : -2.0 * a) : 0.0;
  const double t = expm1_f64_bf(arg);
  const double q = (big ? 2.0 : -t) / (t + 2.0);
  double z = big ? 1.0 - q : q;
  z = ix < 0x40360000u ? z : 1.0;
  z = jx >= 0 ? z : -z;
  z = ix < 0x3c800000u ? x * (1.0 + x) : z;
  const double special = jx >= 0 ? 1.0 / x + 1.0 : 1.0 / x - 1.0;  // +-inf, NaN
  return ix >= 0x7ff00000u ? special : z;
}

LDPC_HD double log_f64_bf(double x) {
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  const double two54 = 1.80143985094819840000e+16;
  const double Lg1 = 6.666666666666735130e-01;
  const double Lg2 = 3.999999999940941908e-01;
  const double Lg3 = 2.857142874366239149e-01;
  const double Lg4 = 2.222219843214978396e-01;
  const double Lg5 = 1.818357216161805012e-01;
  const double Lg6 = 1.531383769920937332e-01;
  const double Lg7 = 1.479819860511658591e-01;
  const double x_in = x;
  const int32_t hx0 = (int32_t)hi_word(x);
  const uint32_t lx0 = lo_word(x);
  const bool zero = ((hx0 & 0x7fffffff) | (int32_t)lx0) == 0;
  const bool tiny = hx0 < 0x00100000;  // subnormal, zero or negative
  x = tiny ? x * two54 : x;
  int32_t k = tiny ? -54 : 0;
  int32_t hx = (int32_t)hi_word(x);
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  const int32_t i = (hx + 0x95f64) & 0x100000;
  x = with_hi(x, (uint32_t)(hx | (i ^ 0x3ff00000)));
  k += (i >> 20);
  const double f = x - 1.0;
  const double dk = (double)k;
  // |f| < 2^-20
  const double Rs = f * f * (0.5 - 0.33333333333333333 * f);
  double rsmall = dk * ln2_hi - ((Rs - dk * ln2_lo) - f);
  rsmall = f == 0.0 ? dk * ln2_hi + dk * ln2_lo : rsmall;
  // general
  const double s = f / (2.0 + f);
  const double z = s * s;
  int32_t ii = hx - 0x6147a;
  const double w = z * z;
  const int32_t j = 0x6b851 - hx;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  ii |= j;
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double rpos = dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
  const double rneg = dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
  double r = ii > 0 ? rpos : rneg;
  r = (0x000fffff & (2 + hx)) < 3 ? rsmall : r;
  r = hx0 >= 0x7ff00000 ? x_in + x_in : r;       // +inf, NaN
  r = hx0 < 0 && !zero ? (x_in - x_in) / 0.0 : r;  // negative: NaN
  return zero ? -__builtin_inf() : r;
}

// ---------------------------------------------------------------------------
// Compact forms for the default f64 mode: same functions, a fraction of the
// instructions, within a few ulp of glibc (tests/test_math.py bounds them).
// Domain handling is complete (0, +-inf, NaN), but the fast paths assume what
// the decoder feeds them: tanh of a finite or infinite double, log of a
// quotient (1+T)/(1-T) in [0, 2^54] or +inf.
// ---------------------------------------------------------------------------

#if defined(__HIP_DEVICE_COMPILE__)
LDPC_HD double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
LDPC_HD double rint_(double x) { return __builtin_rint(x); }
LDPC_HD double ldexp_(double x, int e) { return __builtin_ldexp(x, e); }
LDPC_HD double frexp_(double x, int *e) { return __builtin_frexp(x, e); }
#else
LDPC_HD double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
LDPC_HD double rint_(double x) { return __builtin_rint(x); }
LDPC_HD double ldexp_(double x, int e) { return __builtin_ldexp(x, e); }
LDPC_HD double frexp_(double x, int *e) { return __builtin_frexp(x, e); }
#endif

// n / d for the divisions inside the compact forms (not the decoder's own
// (1+T)/(1-T), which stays an IEEE division): reciprocal, one Newton step,
// one residual correction -- within 1 ulp for the normal, finite operands
// these functions produce (d in [1, 2^64]).
LDPC_HD double div_fast(double n, double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  double y = __builtin_amdgcn_rcp(d);
#else
  double y = 1.0 / d;
#endif
  y = fma_(fma_(-d, y, 1.0), y, y);
  const double q = n * y;
  return fma_(fma_(-d, q, n), y, q);
}

// n quotients num[i] / den[i] from ONE reciprocal (Montgomery's batch
// inversion): prefix products p_i = den[0]..den[i], y = 1/p_{n-1} (one
// reciprocal + Newton step), then backwards 1/den[i] = y p_{i-1}, y *= den[i].
// Each quotient gets div_fast's residual correction q + (num - den q) / den,
// so it carries div_fast's accuracy (the few-ulp error of the batched
// reciprocal is squared away); a v_rcp_f64 (16 issue cycles) and a Newton
// step are traded for three multiplies per extra quotient.  For operands
// whose product stays normal: den in [1, 2] (tanh_half_small_n) or
// [2^-23, 2] (log_ratio_tab_open_n).
template <int n>
LDPC_HD void div_fast_n(const double (&num)[n], const double (&den)[n], double (&q)[n]) {
  double p[n];
  p[0] = den[0];
  for (int i = 1; i < n; ++i) p[i] = p[i - 1] * den[i];
#if defined(__HIP_DEVICE_COMPILE__)
  double y = __builtin_amdgcn_rcp(p[n - 1]);
#else
  double y = 1.0 / p[n - 1];
#endif
  y = fma_(fma_(-p[n - 1], y, 1.0), y, y);
  for (int i = n - 1; i > 0; --i) {
    const double inv = y * p[i - 1];
    y = y * den[i];
    const double qi = num[i] * inv;
    q[i] = fma_(fma_(-den[i], qi, num[i]), inv, qi);
  }
  const double q0 = num[0] * y;
  q[0] = fma_(fma_(-den[0], q0, num[0]), y, q0);
}

// expm1(z) for z in [-44, 44]: z = n ln2 + r, |r| <= ln2/2, expm1(r) =
// r + r^2 p(r), p the Chebyshev-economised degree-9 fit of (e^r - 1 - r)/r^2
// on [-0.3466, 0.3466] (tools/gen_expm1_poly.py; dropped mass 1.0e-16, within
// 3 ulp of glibc in tanh, tests/test_math.py), then expm1(z) = 2^n expm1(r) +
// (2^n - 1) as one fma (2^n - 1 exact for n <= 53).
LDPC_HD double expm1_mid_f64(double z) {
  const double log2e = 1.4426950408889634;
  const double ln2_hi = 6.93147180369123816490e-01;  // low 21 bits zero
  const double ln2_lo = 1.90821492927058770002e-10;
  // n = round(z log2e) by the shifter: the fma rounds the exact product once
  // and leaves n in the low word, so 2^n needs no float->int conversion
  const double shifter = 0x1.8p52;
  const double nd = fma_(z, log2e, shifter);
  const double n = nd - shifter;
  double r = fma_(-n, ln2_hi, z);
  r = fma_(-n, ln2_lo, r);
  double p = 0x1.af4de76a90952p-26;
  p = fma_(p, r, 0x1.289184013c6bbp-22);
  p = fma_(p, r, 0x1.71de023288d0bp-19);
  p = fma_(p, r, 0x1.a019b90e3c799p-16);
  p = fma_(p, r, 0x1.a01a01abe7b65p-13);
  p = fma_(p, r, 0x1.6c16c1788b9a4p-10);
  p = fma_(p, r, 0x1.11111111100dcp-7);
  p = fma_(p, r, 0x1.5555555553d63p-5);
  p = fma_(p, r, 0x1.5555555555557p-3);
  p = fma_(p, r, 0x1.0000000000001p-1);
  const double em = fma_(r * r, p, r);  // expm1(r)
  const double s = ldexp_(1.0, (int)lo_word(nd));  // 2^n, exact
  return fma_(s, em, s - 1.0);
}

// tanh with fdlibm's two ranges (s_tanh.c), one expm1 and one division:
//   |x| <  1: t = expm1(-2|x|), tanh = -t / (t + 2)
//   |x| >= 1: t = expm1( 2|x|), tanh = 1 - 2 / (t + 2);  |x| >= 22: 1
LDPC_HD double tanh_fast_f64(double x) {
  const double a = __builtin_fabs(x);
  const bool big = a >= 1.0;
  const double z = big ? 2.0 * (a < 22.0 ? a : 22.0) : -2.0 * a;
  const double t = expm1_mid_f64(z);
  const double q = div_fast(big ? 2.0 : -t, t + 2.0);
  double r = big ? 1.0 - q : q;
  r = a >= 22.0 ? 1.0 : r;
  r = x < 0.0 ? -r : r;
  return x != x ? x : r;  // NaN
}

// log(q) for q >= 0: q = 2^k (1 + f), sqrt(1/2) <= 1 + f < sqrt(2);
// s = f / (2 + f); log(1 + f) = f - (hfsq - s (hfsq + R(s^2))) with fdlibm's
// minimax R (e_log.c Lg1..Lg7).
LDPC_HD double log_fast_f64(double q) {
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01;
  const double Lg2 = 3.999999999940941908e-01;
  const double Lg3 = 2.857142874366239149e-01;
  const double Lg4 = 2.222219843214978396e-01;
  const double Lg5 = 1.818357216161805012e-01;
  const double Lg6 = 1.531383769920937332e-01;
  const double Lg7 = 1.479819860511658591e-01;
  int k;
  double m = frexp_(q, &k);  // m in [0.5, 1)
  const bool lo = m < 0.70710678118654752440;
  m = lo ? m + m : m;
  k = lo ? k - 1 : k;
  const double f = m - 1.0;  // exact
  const double s = div_fast(f, 2.0 + f);
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * fma_(w, fma_(w, Lg6, Lg4), Lg2);
  const double t2 = z * fma_(w, fma_(w, fma_(w, Lg7, Lg5), Lg3), Lg1);
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)k;
  double r = dk * ln2_hi - ((hfsq - fma_(s, hfsq + R, dk * ln2_lo)) - f);
  r = q == 0.0 ? -__builtin_inf() : r;
  r = q < 0.0 ? __builtin_nan("") : r;
  return (q == __builtin_inf() || q != q) ? q + q : r;
}

// tanh(m / 2), the sum-product check pass's operand (:509), in one range:
// t = expm1(-|m|), tanh(|m|/2) = -t / (t + 2).  fdlibm switches to
// 1 - 2/(expm1(|m|) + 2) above |m| = 2, but for t in (-1, -0.86] both -t and
// t + 2 are within half an ulp, so the single form stays within 3 ulp of glibc
// (tests/test_math.py) with no range selects.  |m| is capped at 44 (t rounds
// to -1 from 38 on, so the result saturates to 1 as tanh does); NaN
// propagates, and the sign is copied (tanh(-0) = -0 as in glibc).  For
// |m| < 2 this is exactly tanh_fast_f64(m/2).
LDPC_HD double tanh_half_fast(double m) {
  const double a = __builtin_fabs(m);
  const double t = expm1_mid_f64(-(a > 44.0 ? 44.0 : a));
  return __builtin_copysign(div_fast(-t, t + 2.0), m);
}

// tanh_half_fast without its cap: |m| <= 44 (finite) only.
LDPC_HD double tanh_half_small(double m) {
  const double t = expm1_mid_f64(-__builtin_fabs(m));
  return __builtin_copysign(div_fast(-t, t + 2.0), m);
}

// tanh_half_small of n values with one batched division (div_fast_n).
template <int n>
LDPC_HD void tanh_half_small_n(const double (&m)[n], double (&out)[n]) {
  double num[n], den[n];
  for (int i = 0; i < n; ++i) {
    const double t = expm1_mid_f64(-__builtin_fabs(m[i]));
    num[i] = -t;
    den[i] = t + 2.0;
  }
  div_fast_n<n>(num, den, out);
  for (int i = 0; i < n; ++i) out[i] = __builtin_copysign(out[i], m[i]);
}

// tanh(m / 2) with fdlibm's two ranges (s_tanh.c) on x = |m| / 2:
//   |m| <  2: t = expm1(-|m|), tanh = -t / (t + 2)   (as tanh_half_fast)
//   |m| >= 2: t = expm1( |m|), tanh = 1 - 2 / (t + 2)
// Near 1 the single-range form's quotient carries 1-3 ulp of 1.0, i.e. a
// relative error of 1 - tanh, which the check message log((1+T)/(1-T))
// amplifies (a 30x-amplitude frame moved its posteriors by ~1e-2 and its
// decisions).  Here the small q = 2 / (t + 2) is formed first and the result
// is the rounding of 1 - q: q's few-ulp error reaches that rounding only
// with probability ~ q 2^-50, so the result is glibc's double except near
// |m| = 2, where 1 - tanh is not small and the error is harmless.  |m| is
// capped at 44 (tanh = 1 from 38 on); NaN propagates; the sign is copied.
LDPC_HD double tanh_half_acc(double m) {
  const double a = __builtin_fabs(m);
  const bool big = a >= 2.0;
  const double ac = a > 44.0 ? 44.0 : a;  // NaN stays NaN
  const double t = expm1_mid_f64(big ? ac : -ac);
  const double q = div_fast(big ? 2.0 : -t, t + 2.0);
  return __builtin_copysign(big ? 1.0 - q : q, m);
}

// log((1+T)/(1-T)), the sum-product check message (:513), for T in [-1, 1]
// (a product of tanh values) or NaN.  The ratio q is then 0 only for T = -1,
// +inf only for T = 1 and never subnormal or negative, so log_fast_f64's
// special cases reduce to |T| == 1 -> +-inf; NaN propagates through the
// polynomial.  The division is the reciprocal-based div_fast.
LDPC_HD double log_ratio_fast(double T) {
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01;
  const double Lg2 = 3.999999999940941908e-01;
  const double Lg3 = 2.857142874366239149e-01;
  const double Lg4 = 2.222219843214978396e-01;
  const double Lg5 = 1.818357216161805012e-01;
  const double Lg6 = 1.531383769920937332e-01;
  const double Lg7 = 1.479819860511658591e-01;
  const double q = div_fast(1.0 + T, 1.0 - T);
  int k;
  double m = frexp_(q, &k);  // m in [0.5, 1)
  const bool lo = m < 0.70710678118654752440;
  m = lo ? m + m : m;
  k = lo ? k - 1 : k;
  const double f = m - 1.0;  // exact
  const double s = div_fast(f, 2.0 + f);
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * fma_(w, fma_(w, Lg6, Lg4), Lg2);
  const double t2 = z * fma_(w, fma_(w, fma_(w, Lg7, Lg5), Lg3), Lg1);
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)k;
  const double r = dk * ln2_hi - ((hfsq - fma_(s, hfsq + R, dk * ln2_lo)) - f);
  return __builtin_fabs(T) == 1.0 ? __builtin_copysign(__builtin_inf(), T) : r;
}

// log((1+T)/(1-T)) for |T| < 1 (no NaN): log_ratio_tab without its final
// select.  The decode kernels use it for iterations whose check operands are
// all tanh values of |m| <= LDPC_TANH_SPLIT (< 1 - 2e-7 in magnitude), so no
// product can reach 1.
LDPC_HD double log_ratio_tab_open(double T, const LogTabEntry *tab);

// log((1+T)/(1-T)) with a table-driven log (tools/gen_logtab.py): the same
// ratio q as log_ratio_fast, then q = 2^k z, z in [0.6875, 1.375), bucket i
// from the top 9 bits, r = z invc_i - 1 (|r| < 1/512), log(q) = k ln2 +
// logc_i + log1p(r) with log1p(r) - r = r^2 (-1/2 + r/3 - ... - r^4/6).  The
// buckets touching 1.0 use c = 1 (logc = 0, r = z - 1 exact), so results near
// 0 keep full relative accuracy.  `tab` is the 512-entry table (in LDS on the
// GPU).  |T| == 1 -> +-inf, NaN -> NaN.
LDPC_HD double log_ratio_tab(double T, const LogTabEntry *tab) {
  const double ln2_hi = 6.93147180369123816490e-01;  // 21 trailing zero bits
  const double ln2_lo = 1.90821492927058770002e-10;
  const double q = div_fast(1.0 + T, 1.0 - T);
  uint64_t ix;
  __builtin_memcpy(&ix, &q, 8);
  // bucket, exponent and reduced argument from the high word alone (32-bit ops)
  const uint32_t hx = (uint32_t)(ix >> 32);
  const uint32_t th = hx - 0x3FE60000u;
  // byte offset of bucket (th >> (20 - kLogTabBits)) % 2^kLogTabBits in one shift and one mask
#if defined(LDPC_PROBE_LOGTAB_LANE) && defined(__HIP_DEVICE_COMPILE__)
  // diagnostic build only (wrong results): every lane reads its own entry,
  // so the table reads are conflict-free (tools/probe_logtab.sh)
  const uint32_t off = (__builtin_amdgcn_workitem_id_x() & 63u) << 4;
#else
  const uint32_t off = (th >> (20 - kLogTabBits - 4)) & (((1u << kLogTabBits) - 1) << 4);
#endif
  const int k = (int)th >> 20;
  const uint64_t iz = ((uint64_t)(hx - (th & 0xFFF00000u)) << 32) | (ix & 0xFFFFFFFFull);
  double z;
  __builtin_memcpy(&z, &iz, 8);
  static_assert(sizeof(LogTabEntry) == 16, "table entries are 16 bytes");
  const LogTabEntry e = *reinterpret_cast<const LogTabEntry *>(
      reinterpret_cast<const char *>(tab) + off);
  const double r = fma_(z, e.invc, -1.0);
  const double kd = (double)k;
  const double w = fma_(kd, ln2_hi, e.logc);  // kd * ln2_hi is exact
  const double hi = w + r;
  const double lo = fma_(kd, ln2_lo, w - hi + r);
  const double r2 = r * r;
  // log1p(r) - r for |r| < 2^-9 (512 buckets): the r^7 term is below 2^-65
  static_assert(kLogTabBits == 9, "the series length assumes 512 buckets");
  double p = -1.0 / 6.0;
  p = fma_(p, r, 1.0 / 5.0);
  p = fma_(p, r, -1.0 / 4.0);
  p = fma_(p, r, 1.0 / 3.0);
  p = fma_(p, r, -0.5);
  const double y = fma_(r2, p, lo) + hi;
  // |T| == 1 -> T * inf = +-inf; NaN -> NaN
  return __builtin_fabs(T) < 1.0 ? y : T * __builtin_inf();
}

// log(q) of log_ratio_tab_open, q = (1+T)/(1-T) already formed.
LDPC_HD double log_q_tab_open(double q, const LogTabEntry *tab) {
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  uint64_t ix;
  __builtin_memcpy(&ix, &q, 8);
  const uint32_t hx = (uint32_t)(ix >> 32);
  const uint32_t th = hx - 0x3FE60000u;
#if defined(LDPC_PROBE_LOGTAB_LANE) && defined(__HIP_DEVICE_COMPILE__)
  // diagnostic build only (wrong results): every lane reads its own entry,
  // so the table reads are conflict-free (tools/probe_logtab.sh)
  const uint32_t off = (__builtin_amdgcn_workitem_id_x() & 63u) << 4;
#else
  const uint32_t off = (th >> (20 - kLogTabBits - 4)) & (((1u << kLogTabBits) - 1) << 4);
#endif
  const int k = (int)th >> 20;
  const uint64_t iz = ((uint64_t)(hx - (th & 0xFFF00000u)) << 32) | (ix & 0xFFFFFFFFull);
  double z;
  __builtin_memcpy(&z, &iz, 8);
  const LogTabEntry e = *reinterpret_cast<const LogTabEntry *>(
      reinterpret_cast<const char *>(tab) + off);
  const double r = fma_(z, e.invc, -1.0);
  const double kd = (double)k;
  const double w = fma_(kd, ln2_hi, e.logc);
  const double hi = w + r;
  const double lo = fma_(kd, ln2_lo, w - hi + r);
  const double r2 = r * r;
  double p = -1.0 / 6.0;
  p = fma_(p, r, 1.0 / 5.0);
  p = fma_(p, r, -1.0 / 4.0);
  p = fma_(p, r, 1.0 / 3.0);
  p = fma_(p, r, -0.5);
  return fma_(r2, p, lo) + hi;
}

LDPC_HD double log_ratio_tab_open(double T, const LogTabEntry *tab) {
  return log_q_tab_open(div_fast(1.0 + T, 1.0 - T), tab);
}

// log_ratio_tab_open of n products with one batched division (div_fast_n);
// every |T| <= tanh(LDPC_TANH_SPLIT / 2), so each 1 - T >= 2^-23.
template <int n>
LDPC_HD void log_ratio_tab_open_n(const double (&T)[n], const LogTabEntry *tab, double (&out)[n]) {
  double num[n], den[n], q[n];
  for (int i = 0; i < n; ++i) {
    num[i] = 1.0 + T[i];
    den[i] = 1.0 - T[i];
  }
  div_fast_n<n>(num, den, q);
  for (int i = 0; i < n; ++i) out[i] = log_q_tab_open(q[i], tab);
}

}  // namespace fm
}  // namespace ldpc
