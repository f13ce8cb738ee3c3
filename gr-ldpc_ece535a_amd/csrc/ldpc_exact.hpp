// ldpc_exact.hpp -- the sum-product check pass's transcendentals, bit for bit
// what the reference computes (lib/ldpc_decoder_cb_impl.cc:509, :513):
//
//   tanh_half_n(m)  = std::tanh(m / 2.0)              glibc 2.35 s_tanh.c + s_expm1.c
//   log_ratio_n(T)  = std::log((1.0 + T) / (1.0 - T)) IEEE division + glibc e_log.c
//
// "Bit for bit" is the contract: every operation below is one of the
// operations glibc's code performs on the host, with the same operands and
// the same rounding, so the result is the same double -- not an
// approximation that is usually close.  The host's log is glibc's FMA build
// (the x86_64 ifunc selects __log_fma on any CPU with FMA/AVX2): its fused
// operations, read off the disassembly of the host libm, are written here as
// explicit fma_() calls; everything else is a separately rounded operation
// (this header must be compiled with -ffp-contract=off, as the Makefile
// does).  tanh/expm1 have no FMA build in glibc 2.35, so they use none.
//
// What is NOT glibc's code is only the *form* of the work on a wave:
//   * divisions: x / y is formed from a reciprocal shared by n quotients
//     (Montgomery's batch inversion: one v_rcp_f64 for n divisors), refined
//     per quotient by a Newton step and finished by the residual correction
//     q + (x - y q) / y -- the same steps as the IEEE double division the
//     compiler emits for gfx950 (rcp, Newton, q, residual, fma) minus its
//     scaling/fix-up instructions, which only act on operands near the ends
//     of the exponent range (every operand here is a normal number far from
//     them: see the domains below).  tests/test_exact.py checks the batched
//     quotients against the host's IEEE division on tens of millions of
//     operands, with the shared reciprocal perturbed by up to +-8 ulp;
//   * expm1's five result formulas (k = 0, -1, <= -2, 2..19, > 56) are one
//     fused multiply-add with per-lane constants -- each is exactly the
//     glibc formula (the proof is at expm1_n) -- and the sixth (k = 20..56)
//     is evaluated only when some lane of the wave needs it;
//   * log's |x - 1| < 1/16 path is evaluated only when some lane needs it.
//
// Header-only, __host__ __device__: the CPU tests run this same code against
// the host libm (tests/test_exact.py, tests/native/exact_check.cc).
#pragma once

#include <stdint.h>
#include <string.h>

#include "ldpc_glibc_log.hpp"

#ifndef LDPC_HD
#if defined(__HIPCC__)
#define LDPC_HD __host__ __device__ __forceinline__
#else
#define LDPC_HD inline
#endif
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// wave-uniform "does any lane need this": the region is skipped otherwise
#define LDPC_EX_ANY(c) (__builtin_amdgcn_ballot_w64(c) != 0)
// first statement of such a rare region: an empty volatile asm cannot be
// speculated, so the compiler keeps the branch instead of if-converting it
// into selects evaluated on every iteration
#define LDPC_EX_COLD() asm volatile(";ldpc_cold")
#else
#define LDPC_EX_ANY(c) (c)
#define LDPC_EX_COLD() ((void)0)
#endif

namespace ldpc {
namespace ex {

LDPC_HD uint64_t bits(double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  return u;
}
LDPC_HD double dbl(uint64_t u) {
  double x;
  memcpy(&x, &u, 8);
  return x;
}
LDPC_HD uint32_t hiw(double x) { return (uint32_t)(bits(x) >> 32); }
// a double whose low word is zero, from its high word
LDPC_HD double from_hi(uint32_t h) { return dbl((uint64_t)h << 32); }
LDPC_HD double fma_(double a, double b, double c) { return __builtin_fma(a, b, c); }
LDPC_HD double sel(bool c, double a, double b) { return c ? a : b; }

#if !defined(__HIP_DEVICE_COMPILE__)
// host tests only: perturbs the shared reciprocal by this many ulp, standing
// in for the GPU's approximate v_rcp_f64 (tests/native/exact_check.cc)
inline int g_rcp_perturb_ulps = 0;
#endif

LDPC_HD double rcp_seed(double p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcp(p);
#else
  return dbl(bits(1.0 / p) + (int64_t)g_rcp_perturb_ulps);
#endif
}

// a / b, correctly rounded, from yk = y (1 + 2^-40), y ~ 1/b with relative
// error < 2^-45 (so b yk lies in (1 + 2^-41, 1 + 2^-39)).
//  1. q0 = a yk; r = fma(-b, q0, a); q1 = fma(r, yk, q0).  q1 - a/b =
//     (a/b - q0)(b yk - 1) + rounding: q1 is within 1/2 ulp + 2^-26 ulp of
//     a/b (the product is below 2^-78 relative), i.e. faithful -- and
//     RN(a/b) unless a/b lies within 2^-26 ulp of a rounding boundary (the Markstein step alone is not enough there:
//     a = 1, b = 1 - 2^-53 with y = 1 gives 1 instead of 1 + 2^-52).
//  2. The decision is then made exactly.  For faithful q1 the residual
//     r1 = a - b q1 is a double, so fma(-b, q1, a) is exact, and
//     a/b - q1 = r1 / b.  RN(a/b) = q1 iff |r1 / b| is below half the gap
//     to q1's neighbour on a/b's side (a quotient of two doubles is never a
//     midpoint, so there are no ties).  The common path tests that with one
//     fma, q1 + r1 y (1 + 2^-40) rounding back to q1 (see below): a sure
//     pass, or a flag raised only within 2^-39 of a midpoint; a flagged lane
//     is settled from the exact gap, h = 2^(e-53) for q1 in [2^e, 2^e+1)
//     (halved below a power of two), in a branch the wave takes only then.
// Domain: a, b normal (or a = +-0), a / b normal, all far from
// over/underflow (|exponents| < 900).
LDPC_HD double div_core(double a, double b, double yk) {
  const double q0 = a * yk;
  const double r = fma_(-b, q0, a);
  double q1 = fma_(r, yk, q0);
  const double r1 = fma_(-b, q1, a);  // exact: a/b = q1 + r1/b
  // t' = r1 yk, |b yk| in (1 + 2^-41, 1 + 2^-39): t' has r1/b's sign and a
  // larger magnitude, so RN(q1 + t') == q1 implies |r1/b| < |t'| <= half
  // the gap on that side (the addition itself takes the smaller gap below a
  // power of two), i.e. RN(a/b) == q1.  Anything else is flagged.
  const bool flag = fma_(r1, yk, q1) != q1;
  if (LDPC_EX_ANY(flag)) {
    LDPC_EX_COLD();
    // exact decision: a/b is on q1's zero side iff r1 / b and q1 differ in
    // sign; h = half the gap on that side (below a power of two it halves)
    const bool down = ((hiw(r1) ^ hiw(b) ^ hiw(q1)) & 0x80000000u) != 0;
    const uint32_t e = down ? (uint32_t)((bits(q1) - 1) >> 32) : hiw(q1);
    const double h = from_hi((e & 0x7ff00000u) - (53u << 20));
    const bool wrong = fma_(-__builtin_fabs(b), h, __builtin_fabs(r1)) > 0.0;
    q1 = wrong ? dbl(bits(q1) + (down ? ~0ull : 1ull)) : q1;
  }
  return q1;
}

// q[i] = a[i] / b[i], correctly rounded, from ONE reciprocal: prefix products
// p_i = b_0 ... b_i, y = 1 / p_{n-1} (v_rcp_f64 + one Newton step), scaled
// once by 1 + 2^-40 (div_core's yk), then backwards 1/b_i (1 + 2^-40) ~
// y p_{i-1}, y <- y b_i (a few ulp); each quotient then takes div_core.
// Domain: div_core's, and every prefix product normal.
template <int n>
LDPC_HD void div_n(const double (&a)[n], const double (&b)[n], double (&q)[n]) {
  double p[n];
  p[0] = b[0];
#pragma unroll
  for (int i = 1; i < n; ++i) p[i] = p[i - 1] * b[i];
  double y = rcp_seed(p[n - 1]);
  y = fma_(fma_(-p[n - 1], y, 1.0), y, y);
  y = y * (1.0 + 0x1p-40);
#pragma unroll
  for (int i = n - 1; i > 0; --i) {
    const double inv = y * p[i - 1];
    y = y * b[i];
    q[i] = div_core(a[i], b[i], inv);
  }
  q[0] = div_core(a[0], b[0], y);
}

// Per-k constants of expm1 (below), as doubles, for k in [kTailLo,
// kTailLo + kTailN), in two 16-byte tables (a 16-byte stride spreads the
// lanes' lookups over the LDS banks): the argument reduction's k ln2_hi
// (exact: ln2_hi has 32 significant bits) and k ln2_lo (glibc's rounded
// product, the same double), and A, B of the result formula.
struct RedEntry {
  double khi, klo;  // k ln2_hi, RN(k ln2_lo)
};
struct TailEntry {
  double a, b;  // A, B
};
constexpr int kTailLo = -3, kTailN = 68;  // k = -3 .. 64
constexpr double kLn2Hi = 6.93147180369123816490e-01;
constexpr double kLn2Lo = 1.90821492927058770002e-10;
constexpr RedEntry red_entry(int k) { return RedEntry{(double)k * kLn2Hi, (double)k * kLn2Lo}; }
constexpr TailEntry tail_entry(int k) {
  return TailEntry{(k == 0 || k == -1) ? 0.0                                    // A = 0
                   : (k >= 2 && k <= 19) ? 1.0 - 1.0 / (double)(1ull << k)     // 1 - 2^-k
                                         : 1.0,                                 // 1
                   k == -1 ? -0.5 : (k >= 0 && k <= 56) ? -0.0 : -1.0};         // B
}
// Everything the exact functions look up: glibc's log table and the tails.
struct ExTab {
  GlLogEntry log[1 << kGlTabBits];
  RedEntry red[kTailN];
  TailEntry tail[kTailN];
};
constexpr ExTab make_ex_tab() {
  ExTab t{{LDPC_GLIBC_LOG_TAB}, {}, {}};
  for (int k = kTailLo; k < kTailLo + kTailN; ++k) {
    t.red[k - kTailLo] = red_entry(k);
    t.tail[k - kTailLo] = tail_entry(k);
  }
  return t;
}

// ---------------------------------------------------------------------------
// expm1(u) for u in (-2, -2^-54] U [2, 44): the arguments tanh(m/2) passes
// (-2|x| for |x| < 1, 2|x| for 1 <= |x| < 22).  glibc 2.35 s_expm1.c:
//   k = 0 if |u| <= 0.5 ln2 (by the high word), -1 if |u| < 1.5 ln2 (u < 0),
//       else (int)(invln2 u +- 0.5);
//   hi = u - k ln2_hi (exact product), lo = k ln2_lo, x = hi - lo
//   (both products are table entries: hi is one subtraction, lo a load;
//   at k = 0 they are +0.0, so x = u and c = 0 as glibc's k == 0 path),
//   c = (hi - x) - lo; hfx = 0.5 x, hxs = x hfx;
//   r1 = 1 + hxs Q1 + hxs^2 (Q2 + hxs Q3) + hxs^4 (Q4 + hxs Q5)  (this grouping);
//   t = 3 - r1 hfx; e = hxs ((r1 - t) / (6 - x t));
//   k == 0:       x - (x e - hxs)
//   else e' = (x (e - c) - c) - hxs and
//   k == -1:      0.5 (x - e') - 0.5
//   k <= -2, >56: (1 - (e' - x)) 2^k - 1
//   2 <= k < 20:  ((1 - 2^-k) - (e' - x)) 2^k
//   20 <= k <= 56: ((x - (e' + 2^-k)) + 1) 2^k
// With d = e' - x (one rounding) the first four are one fma, fma(A - d, 2^k, B):
//   k == 0:  A = 0, B = -0.  At k = 0, c = 0 and the e' recurrence gives
//            e' = (x e) - hxs exactly as glibc's k == 0 line, and
//            RN(0 - d) = -RN(e' - x) = RN(x - e') (rounding is odd-symmetric;
//            + -0 leaves every value, signed zeros included, unchanged).
//   k == -1: A = 0, B = -0.5: 0.5 (x - e') is exact (scaling by 2), so
//            RN(0.5 RN(x - e') - 0.5) = fma(-d, 0.5, -0.5).
//   k <= -2 / k > 56: A = 1, B = -1: RN(1 - d) 2^k is exact (|k| <= 64).
//   2 <= k < 20: A = 1 - 2^-k (exact), B = -0: the product 2^k RN(A - d) is
//            exact, so the fma's rounding is the product's (none).
// Everything else is glibc's operation sequence, unchanged.
// ---------------------------------------------------------------------------
// mid_possible: false if the caller knows every |u| < 13.5 (k <= 19), so
// the k = 20..56 formula need not be checked for (tanh_half_n folds that
// test into its own rare-case test).  hx[i]: the high word of |u[i]|, or any
// word that is above 0x3fd62e42 exactly when that one is.
template <int n>
LDPC_HD void expm1_n(const double (&u)[n], const uint32_t (&hx)[n], double (&t)[n],
                     const ExTab *tab, bool mid_possible = true) {
  constexpr double invln2 = 1.44269504088896338700e+00;
  constexpr double Q1 = -3.33333333333331316428e-02;
  constexpr double Q2 = 1.58730158725481460165e-03;
  constexpr double Q3 = -7.93650757867487942473e-05;
  constexpr double Q4 = 4.00821782732936239552e-06;
  constexpr double Q5 = -2.01099218183624371326e-07;
  double x[n], c[n], hxs[n], num[n], den[n], q[n];
  int k[n];
  bool edge = false;
#pragma unroll
  for (int i = 0; i < n; ++i) {
    const uint32_t sgn = hiw(u[i]) & 0x80000000u;
    // k = (int)(invln2 * u + (u > 0 ? 0.5 : -0.5)), truncation toward zero
    // (|k| <= 63 here).  glibc takes k = -1 for hx in (0x3fd62e42,
    // 0x3FF0A2B2) instead of this rounding, but on that range (u < 0 here)
    // invln2 u - 0.5 lies in (-2, -1): the conversion gives -1 there too.
    // Only k = 0 needs its own select.
    // Below the 0x3fd62e42 high word (|u| < 0.5 ln2 but for the top of that
    // word) the rounding gives k = 0 as glibc's test does; only |u| in
    // (0.5 ln2, 0x3fd62e42ffffffff] -- high word 0x3fd62e42, where glibc
    // takes k = 0 and the rounding may give -1 -- needs the select, in a
    // branch a wave takes only when one of its lanes has that high word.
    k[i] = (int)(invln2 * u[i] + from_hi(0x3fe00000u | sgn));
    edge |= hx[i] == 0x3fd62e42u;
  }
  if (LDPC_EX_ANY(edge)) {
    LDPC_EX_COLD();
#pragma unroll
    for (int i = 0; i < n; ++i) k[i] = hx[i] > 0x3fd62e42u ? k[i] : 0;
  }
#pragma unroll
  for (int i = 0; i < n; ++i) {
    const RedEntry re = tab->red[k[i] - kTailLo];
    const double hi = u[i] - re.khi;
    const double lo = re.klo;
    x[i] = hi - lo;
    c[i] = (hi - x[i]) - lo;
    const double hfx = 0.5 * x[i];
    hxs[i] = x[i] * hfx;
    const double h = hxs[i];
    const double R1 = 1.0 + h * Q1, h2 = h * h;
    const double R2 = Q2 + h * Q3, h4 = h2 * h2;
    const double R3 = Q4 + h * Q5;
    const double r1 = R1 + h2 * R2 + h4 * R3;
    const double tt = 3.0 - r1 * hfx;
    num[i] = r1 - tt;
    den[i] = 6.0 - x[i] * tt;
  }
  div_n<n>(num, den, q);
  bool any_mid = false;
  double ep[n];
#pragma unroll
  for (int i = 0; i < n; ++i) {
    const double e = hxs[i] * q[i];
    ep[i] = (x[i] * (e - c[i]) - c[i]) - hxs[i];
    const double d = ep[i] - x[i];
    const int kk = k[i];
    // per-lane constants: A, B from the table (tail_entry).  fma(A - d, 2^k,
    // B) with its exact product is the exact scaling (ldexp, |k| <= 64 on
    // moderate values) followed by the one rounded addition
    const TailEntry te = tab->tail[kk - kTailLo];
    t[i] = __builtin_ldexp(te.a - d, kk) + te.b;
  }
  if (mid_possible) {  // (a wave-uniform flag: the test stays in its branch)
#pragma unroll
    for (int i = 0; i < n; ++i) any_mid |= (uint32_t)(k[i] - 20) <= 36u;
  }
  if (mid_possible && LDPC_EX_ANY(any_mid)) {
    LDPC_EX_COLD();
#pragma unroll
    for (int i = 0; i < n; ++i) {
      const int kk = k[i];
      const int km = kk < 20 ? 20 : (kk > 56 ? 56 : kk);
      const double tm = from_hi((uint32_t)(0x3ff - km) << 20);  // 2^-k
      const double y = (x[i] - (ep[i] + tm)) + 1.0;
      const double v = y * from_hi((uint32_t)(0x3ff + km) << 20);
      t[i] = (uint32_t)(kk - 20) <= 36u ? v : t[i];
    }
  }
}

template <int n>
LDPC_HD void expm1_n(const double (&u)[n], double (&t)[n], const ExTab *tab,
                     bool mid_possible = true) {
  uint32_t hx[n];
#pragma unroll
  for (int i = 0; i < n; ++i) hx[i] = hiw(u[i]) & 0x7fffffffu;
  expm1_n<n>(u, hx, t, tab, mid_possible);
}

// ---------------------------------------------------------------------------
// z[i] = tanh(m[i] / 2.0) as glibc 2.35 computes it (s_tanh.c):
//   x = m / 2 (m * 0.5: the same correctly rounded value);
//   NaN / inf: 1/x +- 1 (NaN, +-1);  |x| >= 22: +-(1 - tiny) = +-1;
//   |x| < 2^-55: x (1 + x)  (x = +-0 included: glibc returns x, the same);
//   1 <= |x| < 22: t = expm1(2|x|),  z = 1 - 2 / (t + 2);
//   else:          t = expm1(-2|x|), z = -t / (t + 2);   sign of x restored.
// The n quotients share one reciprocal (div_n); lanes outside the expm1
// range feed it a dummy argument and are selected away.
// ---------------------------------------------------------------------------
template <int n>
LDPC_HD void tanh_half_n(const double (&m)[n], double (&z)[n], const ExTab *tab) {
  static_assert(n <= 8, "the tanh divisors (up to 2^63 each) share one prefix product");
  double u[n], t[n], num[n], den[n], q[n];
  uint32_t hm[n];
  bool special = false;
#pragma unroll
  for (int i = 0; i < n; ++i) {
    // x = m / 2 and glibc's expm1 argument +-2|x| = +-|m| (exact: m / 2 is
    // exact for |m| >= 2^-1021; smaller m are special below), so the
    // thresholds on |x| are thresholds on |m| one binade up
    hm[i] = hiw(m[i]);
    const uint32_t im = hm[i] & 0x7fffffffu;
    // u = |m| for |x| >= 1, else -|m|: the sign bit of im - bits(2.0)
    u[i] = dbl(((uint64_t)(im | ((im - 0x40000000u) & 0x80000000u)) << 32) | (uint32_t)bits(m[i]));
    // outside [2^-54, 13.5): |x| < 2^-55, inf, NaN, or possibly k >= 20 --
    // but for m = +-0, which the general path below gets right (expm1's k = 0
    // reduction of u = -0 gives t = +-0, q = +-0 / 2, and the sign is m's: the
    // +-0 glibc returns for x (1 + x)).  The zeros are not rare: a column of
    // degree 1 has no other edge, so its bit message is the empty sum +0.0
    // every iteration (3 of the reference H's 64 columns), and with them in
    // the special set every wave took the special branches every iteration
    special |= im - 0x3c900000u >= 0x402b0000u - 0x3c900000u && m[i] != 0.0;
  }
  const bool any_special = LDPC_EX_ANY(special);
  if (any_special) {
    LDPC_EX_COLD();
#pragma unroll
    for (int i = 0; i < n; ++i) {
      // |m| clamped into [2^-54, 43] (NaN -> 2^-54): lanes outside glibc's
      // expm1 range are replaced below, and any |m| >= 38.2 gives exactly 1,
      // as glibc's 1 - tiny for |x| >= 22 (2 / (expm1(|m|) + 2) < 2^-54)
      const uint32_t im = hm[i] & 0x7fffffffu;
      const double ac = __builtin_fmin(__builtin_fmax(__builtin_fabs(m[i]), 0x1p-54), 43.0);
      u[i] = dbl(bits(ac) ^ ((uint64_t)((im - 0x40000000u) & 0x80000000u) << 32));
    }
  }
  // im is the high word of |u| except on the clamped lanes, where it gives
  // the same k: |m| < 2^-54 and 2^-54 are both below 0x3fd62e42, |m| > 43
  // (inf) and 43 both above; a NaN is above, but its u = 2^-54 converts to
  // k = 0 all the same
  uint32_t hx[n];
#pragma unroll
  for (int i = 0; i < n; ++i) hx[i] = hm[i] & 0x7fffffffu;
  expm1_n<n>(u, hx, t, tab, any_special);
#pragma unroll
  for (int i = 0; i < n; ++i) {
    const bool big = (hm[i] & 0x7fffffffu) >= 0x40000000u;  // |x| >= 1
    num[i] = big ? 2.0 : -t[i];
    den[i] = t[i] + 2.0;
  }
  div_n<n>(num, den, q);
#pragma unroll
  for (int i = 0; i < n; ++i) {
    // glibc: 1 - q (|x| >= 1) or q, with x's sign.  |RN(q - 1)| = RN(1 - q)
    // (rounding is odd-symmetric, 0 <= q <= 1) and RN(q + 0) = q (q > 0 here),
    // so both are |q + w| with w = -1 or +0 -- one constant select (its low
    // word is 0 either way) instead of a double one -- and the magnitude
    // goes in with the sign transfer
    const bool big = (hm[i] & 0x7fffffffu) >= 0x40000000u;
    const double r = q[i] + from_hi(big ? 0xbff00000u : 0u);
    const uint32_t zh = (hiw(r) & 0x7fffffffu) | (hm[i] & 0x80000000u);
    z[i] = dbl(((uint64_t)zh << 32) | (uint32_t)bits(r));
  }
  if (any_special) {
    LDPC_EX_COLD();
#pragma unroll
    for (int i = 0; i < n; ++i) {
      const double x = m[i] * 0.5;
      const uint32_t ix = hiw(x) & 0x7fffffffu;
      // glibc: x (1 + x) below 2^-55 (x itself at +-0); 1/x +- 1 for NaN
      // (NaN) and +-inf (+-1, as computed above)
      z[i] = ix < 0x3c800000u ? x * (1.0 + x) : (x != x ? x + x : z[i]);
    }
  }
}

// ---------------------------------------------------------------------------
// glibc's log (e_log.c, FMA build), for the decoder's ratios:
// q in {+0} U [2^-60, 2^60] U {+inf, NaN} (no subnormal or negative operand:
// log_glibc below is the full function, for the host tests).
//   |q - 1| < 1/16 (q's bits in [bits(1 - 2^-4), bits(1 + 0x1.09p-4))):
//     r = q - 1 and glibc's B-polynomial path (below);
//   else q = 2^k z, z in [0x1.6p-1, 0x1.6p0), i = 7 bits of z:
//     r = fma(z, invc_i, -1); w = fma(k, ln2hi, logc_i); hi = w + r;
//     lo = fma(k, ln2lo, (w - hi) + r); r2 = r r; r3 = r r2;
//     y = fma(r3, fma(fma(r, A4, A3), r2, fma(r, A2, A1)), fma(r2, A0, lo)) + hi.
// `tab` is glibc's 128-entry (invc, logc) table (LDS on the GPU).
// ---------------------------------------------------------------------------
LDPC_HD double log_main(double q, const GlLogEntry *tab) {
  const uint64_t ix = bits(q);
  const uint32_t th = (uint32_t)(ix >> 32) - 0x3fe60000u;  // high word of ix - OFF
  const int k = (int32_t)th >> 20;
  // glibc's iz = ix - (tmp & 0xfff << 52) is q scaled by 2^-k, exactly (q and
  // z = q 2^-k in [0x1.6p-1, 0x1.6p0) are normal): one ldexp
  const double z = __builtin_ldexp(q, -k);
  // entry i = bits 13..19 of th, as a byte offset (16-byte entries)
  static_assert(sizeof(GlLogEntry) == 16, "16-byte log table entries");
  const uint32_t off = (th >> (20 - kGlTabBits - 4)) & (((1u << kGlTabBits) - 1) << 4);
  const GlLogEntry e = *reinterpret_cast<const GlLogEntry *>(reinterpret_cast<const char *>(tab) + off);
  const double r = fma_(z, e.invc, -1.0);
  const double kd = (double)k;
  const double w = fma_(kd, kGlLn2hi, e.logc);
  const double hi = w + r;
  const double lo = fma_(kd, kGlLn2lo, (w - hi) + r);
  const double r2 = r * r;
  const double r3 = r * r2;
  const double p = fma_(fma_(r, kGlA[4], kGlA[3]), r2, fma_(r, kGlA[2], kGlA[1]));
  return fma_(r3, p, fma_(r2, kGlA[0], lo)) + hi;
}

// the |q - 1| < 1/16 path: r = q - 1 (exact), log1p(r) = r + B0 r^2 + r^3 P(r)
// with r split into rhi (26 bits) + rlo so r + B0 rhi^2 is formed exactly
LDPC_HD double log_near1(double q) {
  const double r = q - 1.0;
  const double r2 = r * r;
  const double r3 = r * r2;
  const double P1 = fma_(r2, kGlB[3], fma_(r, kGlB[2], kGlB[1]));
  const double P2 = fma_(r2, kGlB[6], fma_(r, kGlB[5], kGlB[4]));
  const double P3 = fma_(r3, kGlB[10], fma_(r2, kGlB[9], fma_(r, kGlB[8], kGlB[7])));
  const double poly = fma_(fma_(P3, r3, P2), r3, P1);
  const double W = fma_(r, 0x1p27, r);      // glibc: w = r * 0x1p27; rhi = r + w - w
  const double rhi = fma_(-0x1p27, r, W);   // (contracted by the compiler as here)
  const double rlo = r - rhi;
  const double rh2 = rhi * rhi;             // exact (26-bit halves)
  const double hi = fma_(rh2, kGlB[0], r);  // r + B0 rhi^2
  const double lo = fma_(rh2, kGlB[0], r - hi);
  const double lo2 = fma_(kGlB[0] * rlo, r + rhi, lo);
  return fma_(poly, r3, lo2) + hi;
}

// bits(q) - bits(1 - 2^-4) < bits(1 + 0x1.09p-4) - bits(1 - 2^-4): both bounds
// have zero low words, so the high word decides
LDPC_HD bool log_is_near1(double q) { return hiw(q) - 0x3fee0000u < 0x3ff10900u - 0x3fee0000u; }

// log(q) for q normal in [2^-60, 2^60] (the decoder's open ratios)
LDPC_HD double log_q(double q, const GlLogEntry *tab) {
  double y = log_main(q, tab);
  const bool near = log_is_near1(q);
  if (LDPC_EX_ANY(near)) {
    LDPC_EX_COLD();
    y = near ? log_near1(q) : y;
  }
  return y;
}

// log_main with glibc's own bit arithmetic for the scaling (the ldexp above
// needs a normal q; glibc's subnormal path hands in a pseudo-double whose
// exponent field is below 1)
inline double log_main_bits(uint64_t ix, const GlLogEntry *tab) {
  const uint32_t th = (uint32_t)(ix >> 32) - 0x3fe60000u;
  const uint32_t i = (th >> (20 - kGlTabBits)) & ((1u << kGlTabBits) - 1);
  const int k = (int32_t)th >> 20;
  const uint64_t iz = ((uint64_t)((uint32_t)(ix >> 32) - (th & 0xfff00000u)) << 32) | (uint32_t)ix;
  const GlLogEntry e = tab[i];
  const double z = dbl(iz);
  const double r = fma_(z, e.invc, -1.0);
  const double kd = (double)k;
  const double w = fma_(kd, kGlLn2hi, e.logc);
  const double hi = w + r;
  const double lo = fma_(kd, kGlLn2lo, (w - hi) + r);
  const double r2 = r * r;
  const double r3 = r * r2;
  const double p = fma_(fma_(r, kGlA[4], kGlA[3]), r2, fma_(r, kGlA[2], kGlA[1]));
  return fma_(r3, p, fma_(r2, kGlA[0], lo)) + hi;
}

// glibc's log on every double (host reference for the tests)
inline double log_glibc(double x, const GlLogEntry *tab) {
  uint64_t ix = bits(x);
  if (log_is_near1(x)) return ix == bits(1.0) ? 0.0 : log_near1(x);
  const uint32_t top = (uint32_t)(ix >> 48);
  if (top - 0x0010u >= 0x7ff0u - 0x0010u) {
    if ((ix << 1) == 0) return -__builtin_inf();
    if (ix == bits(__builtin_inf())) return x;
    if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return (x - x) / 0.0;  // NaN
    ix = bits(x * 0x1p52) - (52ull << 52);  // subnormal
    return log_main_bits(ix, tab);
  }
  return log_main(dbl(ix), tab);
}

// ---------------------------------------------------------------------------
// E[i] = log((1 + T[i]) / (1 - T[i])) (:513) for T in [-1, 1] or NaN (a
// product of tanh values): the quotient is +0 at T = -1, +inf at T = 1, and
// otherwise in [2^-54, 2^54] (1 -+ T >= 2^-53), so div_n's domain holds for
// every lane once T = 1 / NaN lanes divide by 1 and are selected away.
// ---------------------------------------------------------------------------
// the quotients (1 + T) / (1 - T) of log_ratio_n; returns whether a lane
// (device: any lane of the wave) holds a T of +-1 or NaN (its q is then a
// placeholder: see ratio_fix_n)
template <int n>
LDPC_HD bool ratio_n(const double (&T)[n], double (&q)[n]) {
  static_assert(n <= 16, "the divisors (>= 2^-53 each) share one prefix product");
  double num[n], den[n];
  bool special = false;  // (device: any lane of the wave; host: this lane)
#pragma unroll
  for (int i = 0; i < n; ++i) {
    num[i] = 1.0 + T[i];
    den[i] = 1.0 - T[i];
    // T = +-1 (2/0, 0/2) or NaN; one ballot per slot, OR-ed as scalar masks
    // (a per-lane flag kept across the slots costs a select and a compare)
    special |= LDPC_EX_ANY(!(__builtin_fabs(T[i]) < 1.0));
  }
  // 1 - T >= 2^-53 unless T = 1 or NaN: when some lane has one, every lane's
  // divisor is raised to >= 2^-60 (a finite quotient in the shared product;
  // the other lanes' divisors are unchanged) and ratio_fix_n replaces them
  if (special) {
    LDPC_EX_COLD();
#pragma unroll
    for (int i = 0; i < n; ++i) den[i] = __builtin_fmax(den[i], 0x1p-60);
  }
  div_n<n>(num, den, q);
  return special;
}

// E for the T = +-1 / NaN lanes: log(2/0) = +inf, log(0/2) = -inf, NaN
template <int n>
LDPC_HD void ratio_fix_n(const double (&T)[n], double (&E)[n]) {
#pragma unroll
  for (int i = 0; i < n; ++i)
    E[i] = __builtin_fabs(T[i]) < 1.0
               ? E[i]
               : (T[i] != T[i] ? T[i] + T[i] : __builtin_copysign(__builtin_inf(), T[i]));
}

template <int n>
LDPC_HD void log_ratio_n(const double (&T)[n], const ExTab *tab, double (&E)[n]) {
  double q[n];
  const bool any_special = ratio_n<n>(T, q);  // (wave-uniform on the device)
#pragma unroll
  for (int i = 0; i < n; ++i) E[i] = log_q(q[i], tab->log);
  if (any_special) {
    LDPC_EX_COLD();
    ratio_fix_n<n>(T, E);
  }
}

}  // namespace ex
}  // namespace ldpc
