"""ldpc_exact.hpp -- the arithmetic of the default sum-product mode -- on the
host, against the host libm (glibc: what the reference and the oracle call).

The claim is bit-identity, not closeness: tanh(m/2), expm1, log and
log((1+T)/(1-T)) must return the same double as glibc for every operand the
decoder can produce, and the batched divisions the same double as IEEE
division -- also when the shared reciprocal is off by several ulp (the GPU's
v_rcp_f64 is an approximation; its seed is refined before use).  Each test
sweeps millions of random operands plus the boundaries of every branch of
glibc's code (the k classes of expm1, tanh's |x| = 1 / 22 / 2^-55 switches,
log's |x - 1| < 1/16 window and table subintervals)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "native", "exact_check.cc")


@pytest.fixture(scope="module")
def ec(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("ec") / "exact_check.so")
    flags = ["-O2", "-ffp-contract=off", "-fPIC", "-shared"]
    if "fma" in open("/proc/cpuinfo").read().split():
        flags.append("-mfma")  # speed only: every fused operation is an explicit fma
    subprocess.check_call(["g++"] + flags + ["-o", so, SRC, "-lm"])
    lib = ctypes.CDLL(so)
    lib.self_check.restype = ctypes.c_int64
    return lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _call(fn, *arrays, mode=None):
    arrays = [np.ascontiguousarray(a, np.float64) for a in arrays]
    n = min(a.size for a in arrays)
    out = np.zeros(2, np.int64)
    args = ([ctypes.c_int(mode)] if mode is not None else []) + [_ptr(a) for a in arrays]
    fn(*args, ctypes.c_int64(n), _ptr(out))
    return int(out[0]), int(out[1])


def _triples(x):
    x = np.asarray(x, np.float64).ravel()
    pad = (-x.size) % 3
    return np.concatenate([x, np.full(pad, 0.5)]) if pad else x


def _around(points, width=64):
    """every double within `width` ulp of each point, both signs"""
    pts = np.asarray(points, np.float64)
    b = pts.view(np.int64)[:, None] + np.arange(-width, width + 1)[None, :]
    v = b.view(np.float64).ravel()
    return np.concatenate([v, -v])


def test_constants_match_host_libm(ec):
    """ldpc_glibc_log.hpp holds this libm's __log_data (regenerate with
    tools/gen_glibc_log.py if the image's glibc changes)."""
    assert ec.self_check() == 0
    out = subprocess.run(["python3", os.path.join(ROOT, "tools", "gen_glibc_log.py"), "--check"],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr


def test_log_bit_identical(ec):
    rng = np.random.default_rng(101)
    sets = [rng.uniform(0, 3, 4_000_000), np.exp(rng.uniform(-45, 45, 4_000_000)),
            1 + rng.uniform(-0.07, 0.07, 4_000_000),
            1 + rng.uniform(-1, 1, 2_000_000) * 10.0 ** rng.uniform(-17, -1, 2_000_000),
            10.0 ** rng.uniform(-307, 308, 2_000_000),
            # both ends of the |x - 1| < 1/16 window and every table subinterval edge
            _around([1 - 2.0 ** -4, 1 + float.fromhex("0x1.09p-4"), 1.0], 4096),
            _around(np.arange(0x3FE6000000000000, 0x3FF6000000000000, 1 << 45,
                              dtype=np.int64).view(np.float64), 16),
            np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, 2.0, 0.5, 5e-324, 1e-310, -1.0])]
    for x in sets:
        mism, maxu = _call(ec.check_log, x, mode=0)
        assert mism == 0, (mism, maxu)
    # the decoder's form on its own domain: normal [2^-60, 2^60] (log_ratio_n
    # handles T = +-1 / NaN, i.e. ratios 0 / inf / NaN, itself)
    for x in sets[:4] + [np.array([2.0 ** -60, 2.0 ** 60, 1.0])]:
        x = x[(x >= 2.0 ** -60) & (x <= 2.0 ** 60)]
        assert _call(ec.check_log, x, mode=1)[0] == 0


def test_tanh_half_bit_identical(ec):
    rng = np.random.default_rng(102)
    ln2 = np.log(2.0)
    # expm1's k classes switch at |u| = 0.5 ln2, 1.5 ln2 (high word) and
    # (k + 1/2) ln2; u = |m| (|m| >= 2) or -|m|; tanh's at |m| = 2, 44, 2^-54
    edges = [0.5 * ln2, 1.5 * ln2, 2.0, 44.0, 2.0 ** -54, 2.0 ** -53]
    edges += [(k + 0.5) * ln2 for k in range(2, 64)]
    edges += [float.fromhex("0x1.62e42p-2"), float.fromhex("0x1.0a2b2p0")]
    sets = [rng.uniform(-4, 4, 6_000_000), rng.uniform(-60, 60, 6_000_000),
            rng.normal(0, 12, 6_000_000),
            rng.uniform(-1, 1, 3_000_000) * 10.0 ** rng.uniform(-30, 0, 3_000_000),
            _around(edges, 512),
            # |m| with high word 0x3fd62e42 above 0.5 ln2, where glibc's expm1
            # takes k = 0 by the high word and the rounding alone would not
            # (ldpc_exact.hpp takes that select in a rare branch)
            np.concatenate([v := rng.integers(0x3FD62E42FEFA39EF, 0x3FD62E4300000000, 200_000,
                                               dtype=np.int64).view(np.float64), -v]),
            np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 1e-310, 1e300,
                      -1e300, 2.0, -2.0, 44.0, -44.0])]
    for m in sets:
        mism, maxu = _call(ec.check_tanh_half, _triples(m))
        assert mism == 0, (mism, maxu)


def test_expm1_bit_identical(ec):
    rng = np.random.default_rng(103)
    for u in (-rng.uniform(0, 2, 3_000_000), rng.uniform(2, 44, 3_000_000),
              -10.0 ** rng.uniform(-16, 0.3, 3_000_000)):
        u = u[((u < 0) & (u > -2) & (u <= -2.0 ** -54)) | ((u >= 2) & (u < 44))]
        mism, maxu = _call(ec.check_expm1, _triples(u))
        assert mism == 0, (mism, maxu)


def test_log_ratio_bit_identical(ec):
    rng = np.random.default_rng(104)
    t = np.tanh(rng.normal(0, 6, (2_000_000, 5)) / 2)
    sets = [rng.uniform(-1, 1, 6_000_000), np.prod(t, axis=1), t[:, 0] * t[:, 1],
            1 - 10.0 ** rng.uniform(-16.5, 0, 3_000_000), -1 + 10.0 ** rng.uniform(-16.5, 0, 3_000_000),
            rng.uniform(-0.07, 0.07, 3_000_000),
            rng.uniform(-1, 1, 1_000_000) * 10.0 ** rng.uniform(-300, 0, 1_000_000),
            np.array([1.0, -1.0, 0.0, -0.0, np.nan, 0.5, -0.5, 1 - 2.0 ** -53, -1 + 2.0 ** -53,
                      np.nan, 1.0, 1.0])]
    for T in sets:
        mism, maxu = _call(ec.check_log_ratio, _triples(T))
        assert mism == 0, (mism, maxu)


@pytest.mark.parametrize("perturb", [0, 1, -1, 3, -3, 8, -8, 1 << 20, -(1 << 22)])
def test_batched_division_is_ieee(ec, perturb):
    """div_n<k> for k = 1..3 equals a / b with the shared reciprocal seed off
    by `perturb` ulp (up to 2^22): the residual correction and the exact
    residual test make the result independent of the seed's last bits.  Operands: the
    three divisions of the sum-product pass (expm1's (r1 - t) / (6 - x t) ~
    O(1), tanh's -t/(t+2) or 2/(t+2), (1+T)/(1-T) down to 2^-53) and
    significands with long runs of ones / zeros (the hard cases of division)."""
    rng = np.random.default_rng(105 + abs(perturb))
    ec.set_rcp_perturb(perturb)
    try:
        n = 3_000_000
        hard = (np.int64(0x3FF0000000000000) |
                (rng.integers(0, 2, n) * ((1 << 52) - 1) ^ rng.integers(0, 1 << 20, n))).view(np.float64)
        cases = [(rng.uniform(-2.2, -1.8, n), rng.uniform(5, 7, n)),
                 (rng.uniform(0, 0.87, n), rng.uniform(1.13, 2, n)),
                 (np.full(n, 2.0), 2 + np.exp(rng.uniform(1.8, 44, n))),
                 (1 + rng.uniform(-1, 1, n), 1 - rng.uniform(-1, 1, n) * 10.0 ** -rng.uniform(0, 16, n)),
                 (hard, np.roll(hard, 1)), (rng.uniform(1, 2, n), hard),
                 # 1 / (1 - 2^-53) = 1 + 2^-53 + 2^-106...: just above a midpoint,
                 # where the residual-corrected quotient alone rounds the wrong way
                 (np.ones(n), np.full(n, 1 - 2.0 ** -53)),
                 (1 + rng.integers(0, 1 << 12, n) * 2.0 ** -52,
                  (np.int64(0x3FEFFFFFFFFFFFFF) - rng.integers(0, 1 << 8, n)).view(np.float64)),
                 (1 + rng.uniform(-1, 1, n) * 2.0 ** -53 * rng.integers(0, 3, n),
                  1 - rng.integers(0, 3, n) * 2.0 ** -53)]
        for a, b in cases:
            for k in (1, 2, 3):
                mism, maxu = _call(lambda *args: ec.check_div(ctypes.c_int(k), *args), a, b)
                assert mism == 0, (k, mism, maxu)
    finally:
        ec.set_rcp_perturb(0)
