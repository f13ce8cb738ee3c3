// Host check of gr-ldpc_ece535a_amd/csrc/ldpc_exact.hpp against the host libm
// (glibc: what the reference and the oracle call).  Built by
// tests/test_exact.py with -ffp-contract=off.  Every function returns the
// number of results whose bits differ (NaN == NaN) in out[0] and the largest
// ulp distance in out[1].
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../../gr-ldpc_ece535a_amd/csrc/ldpc_exact.hpp"

using namespace ldpc::ex;

static const ExTab kEx = make_ex_tab();
static const GlLogEntry *const kTab = kEx.log;

static int64_t ulps(double a, double b) {
  if (a != a && b != b) return 0;
  if (bits(a) == bits(b)) return 0;
  int64_t ia = (int64_t)bits(a), ib = (int64_t)bits(b);
  if (ia < 0) ia = (int64_t)0x8000000000000000ull - ia;
  if (ib < 0) ib = (int64_t)0x8000000000000000ull - ib;
  const int64_t d = ia - ib;
  return d == 0 ? 1 : (d < 0 ? -d : d);  // +0 vs -0 counts as a mismatch
}

static void tally(double a, double b, int64_t *out) {
  const int64_t u = ulps(a, b);
  if (u) ++out[0];
  if (u > out[1]) out[1] = u;
}

extern "C" {

void set_rcp_perturb(int ulps_) { g_rcp_perturb_ulps = ulps_; }

// tanh_half_n<3>(m) vs tanh(m / 2.0), on consecutive triples (n % 3 == 0)
void check_tanh_half(const double *m, int64_t n, int64_t *out) {
  out[0] = out[1] = 0;
  for (int64_t i = 0; i + 3 <= n; i += 3) {
    const double v[3] = {m[i], m[i + 1], m[i + 2]};
    double z[3];
    tanh_half_n<3>(v, z, &kEx);
    for (int j = 0; j < 3; ++j) tally(z[j], tanh(v[j] / 2.0), out);
  }
}

// expm1_n<3>(u) vs expm1(u), u in (-2, -2^-54] U [2, 44)
void check_expm1(const double *u, int64_t n, int64_t *out) {
  out[0] = out[1] = 0;
  for (int64_t i = 0; i + 3 <= n; i += 3) {
    const double v[3] = {u[i], u[i + 1], u[i + 2]};
    double t[3];
    expm1_n<3>(v, t, &kEx);
    for (int j = 0; j < 3; ++j) tally(t[j], expm1(v[j]), out);
  }
}

// mode 0: log_glibc(x) vs log(x) (any double); mode 1: log_q(x) (decoder domain)
void check_log(int mode, const double *x, int64_t n, int64_t *out) {
  out[0] = out[1] = 0;
  for (int64_t i = 0; i < n; ++i)
    tally(mode == 0 ? log_glibc(x[i], kTab) : log_q(x[i], kTab), log(x[i]), out);
}

// log_ratio_n<3>(T) vs log((1 + T) / (1 - T)), T in [-1, 1] or NaN
void check_log_ratio(const double *T, int64_t n, int64_t *out) {
  out[0] = out[1] = 0;
  for (int64_t i = 0; i + 3 <= n; i += 3) {
    const double v[3] = {T[i], T[i + 1], T[i + 2]};
    double e[3];
    log_ratio_n<3>(v, &kEx, e);
    for (int j = 0; j < 3; ++j) tally(e[j], log((1.0 + v[j]) / (1.0 - v[j])), out);
  }
}

// div_n<k>(a, b) vs a / b for k = 1, 2, 3 (consecutive groups)
void check_div(int k, const double *a, const double *b, int64_t n, int64_t *out) {
  out[0] = out[1] = 0;
  for (int64_t i = 0; i + k <= n; i += k) {
    if (k == 1) {
      const double x[1] = {a[i]}, y[1] = {b[i]};
      double q[1];
      div_n<1>(x, y, q);
      tally(q[0], a[i] / b[i], out);
    } else if (k == 2) {
      const double x[2] = {a[i], a[i + 1]}, y[2] = {b[i], b[i + 1]};
      double q[2];
      div_n<2>(x, y, q);
      for (int j = 0; j < 2; ++j) tally(q[j], a[i + j] / b[i + j], out);
    } else {
      const double x[3] = {a[i], a[i + 1], a[i + 2]}, y[3] = {b[i], b[i + 1], b[i + 2]};
      double q[3];
      div_n<3>(x, y, q);
      for (int j = 0; j < 3; ++j) tally(q[j], a[i + j] / b[i + j], out);
    }
  }
}

// the glibc constants this build carries match the libm it runs against:
// log_glibc vs log on a fixed sweep of every table subinterval and both paths
int64_t self_check(void) {
  int64_t out[2] = {0, 0};
  for (int i = 0; i < 1 << 20; ++i) {
    const double x = 0.5 + 1.5 * i / (double)(1 << 20);
    tally(log_glibc(x, kTab), log(x), out);
  }
  return out[0];
}
}
