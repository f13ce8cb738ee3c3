"""ldpc_math.hpp (the f64 tanh/expm1/log the kernels use) on the host:
tanh/expm1 bit-identical to the host libm (glibc, what the reference and the
oracle call); the branch-free GPU forms identical to the branchy fdlibm
forms; log within 1 ulp of glibc."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "math_check.cc")


@pytest.fixture(scope="module")
def mc(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("mc") / "math_check.so")
    subprocess.check_call(["g++", "-O2", "-ffp-contract=off", "-fPIC", "-shared", "-o", so, SRC,
                           "-lm"])
    return ctypes.CDLL(so)


def _run(mc, fname, fn, x):
    x = np.ascontiguousarray(x, np.float64)
    out = np.zeros(2, np.int64)
    getattr(mc, fname)(fn, x.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(x.size),
                       out.ctypes.data_as(ctypes.c_void_p))
    return out


SPECIALS = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 1e-310, 2.0 ** -55,
                     2.0 ** -54, 22.0, -22.0, 21.999, 1.0, -1.0, 0.34657359, 1.0397, 38.8,
                     44.0, 1e300, -1e300])


def _inputs(seed, n=400_000):
    rng = np.random.default_rng(seed)
    return [rng.uniform(-1, 1, n), rng.uniform(-30, 30, n), rng.normal(0, 8, n),
            rng.uniform(-1, 1, n) * 10.0 ** rng.uniform(-20, 0, n), SPECIALS]


def test_tanh_bit_identical_to_libm(mc):
    for x in _inputs(1):
        mism, maxulp = _run(mc, "check_fn", 0, x)
        assert mism == 0, (mism, maxulp)


def test_expm1_bit_identical_to_libm(mc):
    rng = np.random.default_rng(2)
    for x in (rng.uniform(-2, 0, 400_000), rng.uniform(2, 44, 400_000),
              rng.uniform(-60, 300, 400_000), SPECIALS):
        mism, _ = _run(mc, "check_fn", 1, x)
        assert mism == 0


def test_branch_free_forms_identical(mc):
    rng = np.random.default_rng(3)
    for x in _inputs(4):
        assert _run(mc, "check_bf", 0, x)[0] == 0
    for x in (rng.uniform(-2, 0, 400_000), rng.uniform(2, 44, 400_000)):
        assert _run(mc, "check_bf", 1, x)[0] == 0
    for x in (np.exp(rng.uniform(-40, 40, 400_000)), 1 + rng.uniform(-2e-6, 2e-6, 400_000),
              rng.uniform(0, 3, 400_000), SPECIALS):
        assert _run(mc, "check_bf", 2, x)[0] == 0


def test_log_within_one_ulp(mc):
    rng = np.random.default_rng(5)
    for x in (np.exp(rng.uniform(-40, 40, 400_000)), rng.uniform(0, 3, 400_000),
              1 + rng.uniform(-1e-3, 1e-3, 400_000)):
        _, maxulp = _run(mc, "check_fn", 2, x)
        assert maxulp <= 1


def test_compact_tanh_within_3ulp(mc):
    """LDPC_PREC_F64 (compact) tanh: within 3 ulp of glibc."""
    for i, x in enumerate(_inputs(11)):
        _, maxulp = _run(mc, "check_fast", 0, x)
        assert maxulp <= 3, (i, maxulp)


def test_compact_log_within_3ulp(mc):
    rng = np.random.default_rng(12)
    for x in (np.exp(rng.uniform(-40, 40, 400_000)), rng.uniform(0, 3, 400_000),
              1 + rng.uniform(-1e-3, 1e-3, 400_000)):
        _, maxulp = _run(mc, "check_fast", 2, x)
        assert maxulp <= 3


def test_check_pass_forms(mc):
    """tanh_half_fast(m) within 3 ulp of glibc tanh(m/2) (and == the two-range
    tanh_fast_f64(m/2) for normal |m| < 2, where both take the same path);
    log_ratio_fast(T) within 3 ulp of glibc log((1+T)/(1-T)) over T in
    [-1, 1] incl. the +-1 / +-0 / NaN edges."""
    for x in _inputs(13):
        normal = x[np.isfinite(x) & (np.abs(x) > 1e-300) & (np.abs(x) < 2.0)]
        mism, _ = _run(mc, "check_pass", 2, normal)
        assert mism == 0
        _, maxulp = _run(mc, "check_pass", 0, x)
        assert maxulp <= 3
    rng = np.random.default_rng(14)
    Ts = [rng.uniform(-1, 1, 400_000), np.tanh(rng.normal(0, 10, 400_000)),
          1 - 10.0 ** rng.uniform(-16, 0, 200_000), -1 + 10.0 ** rng.uniform(-16, 0, 200_000),
          np.array([1.0, -1.0, 0.0, -0.0, np.nan, 0.5, -0.5, 1 - 2.0 ** -53, -1 + 2.0 ** -53])]
    for T in Ts:
        _, maxulp = _run(mc, "check_pass", 1, T)
        assert maxulp <= 3


def test_two_range_tanh_matches_libm_near_one(mc):
    """The f64 mode's tanh(m/2) (tanh_half_acc, used whenever some |m| of the
    frame reaches the split): glibc's exact double for |m| >= 16 and all but
    ~1e-5 of the values in [8, 16) -- where 1 - tanh is small and
    log((1+T)/(1-T)) would amplify any last-bit difference --, within 1 ulp
    for |m| >= 2 (the single-range form is 1-2 ulp off for most of them) and
    within 3 ulp below (the single-range form there).  The
    uncapped single-range form of the fast path equals tanh_half_fast
    wherever it is used (|m| <= 44)."""
    rng = np.random.default_rng(21)
    far = np.concatenate([rng.uniform(16, 60, 400_000), -rng.uniform(16, 60, 400_000),
                          np.array([np.inf, -np.inf, 44.0, 38.0, 100.0, 1e300])])
    mism, _ = _run(mc, "check_pass", 3, far)
    assert mism == 0
    mid = rng.uniform(8, 16, 400_000) * rng.choice([-1.0, 1.0], 400_000)
    mism, maxulp = _run(mc, "check_pass", 3, mid)
    assert mism <= 8 and maxulp <= 1
    for x in _inputs(22):
        _, maxulp = _run(mc, "check_pass", 3, x)
        assert maxulp <= 3
        _, maxulp = _run(mc, "check_pass", 3, x[np.abs(x) >= 2.0])
        assert maxulp <= 1
        small = x[np.isfinite(x) & (np.abs(x) <= 44.0)]
        mism, _ = _run(mc, "check_pass", 4, small)
        assert mism == 0


def test_table_log_within_1ulp(mc):
    """LDPC_PREC_F64's table-driven log((1+T)/(1-T)) (tools/gen_logtab.py):
    within 1 ulp of glibc over T in [-1, 1], near +-1, near 0 and the edges."""
    rng = np.random.default_rng(15)
    Ts = [rng.uniform(-1, 1, 400_000), np.tanh(rng.normal(0, 10, 400_000)),
          1 - 10.0 ** rng.uniform(-16, 0, 200_000), -1 + 10.0 ** rng.uniform(-16, 0, 200_000),
          10.0 ** rng.uniform(-300, -1, 200_000),
          np.array([1.0, -1.0, 0.0, -0.0, np.nan, 0.5, -0.5, 1 - 2.0 ** -53, -1 + 2.0 ** -53])]
    for T in Ts:
        x = np.ascontiguousarray(T, np.float64)
        out = np.zeros(2, np.int64)
        mc.check_logtab(x.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(x.size),
                        out.ctypes.data_as(ctypes.c_void_p))
        assert out[1] <= 1


def test_logtab_header_is_generated():
    """The committed table equals what tools/gen_logtab.py produces."""
    import importlib.util
    root = os.path.dirname(HERE)
    spec = importlib.util.spec_from_file_location("gen_logtab",
                                                  os.path.join(root, "tools", "gen_logtab.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    hdr = open(os.path.join(root, "gr-ldpc_ece535a_amd", "csrc", "ldpc_logtab.hpp")).read()
    for invc, logc, _, _ in g.table():
        assert "{%s, %s}" % (invc.hex(), logc.hex()) in hdr


def test_batched_divisions(mc):
    """div_fast_n (one reciprocal for the column's three tanh quotients and
    for the slots' three open check-message quotients): the same accuracy as
    the one-at-a-time forms -- within 3 ulp of glibc, and identical to them
    on these 2.4 M host operands (the residual correction squares the batched
    reciprocal's error away); the GPU's v_rcp_f64 seed is checked by the GPU
    parity tests."""
    rng = np.random.default_rng(21)
    m = np.concatenate([rng.uniform(-16, 16, 600_000), rng.normal(0, 3, 600_000),
                        rng.uniform(-1, 1, 300_000) * 10.0 ** rng.uniform(-12, 0, 300_000)])
    mism, maxulp = _run(mc, "check_batch", 0, m)
    assert maxulp <= 1 and mism <= m.size * 1e-3, (mism, maxulp)
    _, maxulp = _run(mc, "check_batch", 2, m)
    assert maxulp <= 3
    # open check operands: products of tanh(m/2) with |m| <= 16
    t = np.tanh(rng.uniform(-8, 8, (1_200_000, 3)) / 1.0)
    T = (t[:, 0] * t[:, 1] * rng.choice([1.0, 0.5, 1e-3], t.shape[0])).astype(np.float64)
    T = np.concatenate([T, np.tanh(rng.uniform(-8, 8, 300_000))])
    mism, maxulp = _run(mc, "check_batch", 1, T)
    assert maxulp <= 1 and mism <= T.size * 1e-3, (mism, maxulp)
    _, maxulp = _run(mc, "check_batch", 3, T)
    assert maxulp <= 3
