"""The window server (ldpc_serve_*, csrc/ldpc_serve.hip): rounds of windows
of one staged span, served by one persistent launch, equal the same windows
through ldpc_decode_windows (a launch per round) and the oracle's decodes of
the same samples -- every polarity, round sizes from 1 to past the host
buffer, both methods the server takes -- and the launch survives its own
deadline between rounds (the next round starts another)."""
import os
import time

import numpy as np
import pytest

import ldpc_ece535a as L
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _span(Hr, frames, seed, ebn0=2.0):
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 2, size=(frames, Hr.shape[1] - Hr.shape[0]), dtype=np.uint8)
    x = 2.0 * L.encode(Hr, data) - 1.0
    y = x + np.sqrt(10 ** (-ebn0 / 10)) * rng.standard_normal(x.shape)
    s = np.concatenate([rng.standard_normal(37), y.ravel()]).astype(np.float32)
    return s


def _windows(rng, n, span_len, N):
    p = rng.integers(0, span_len - N + 1, size=n).astype(np.int64)
    return (p << 1) | rng.integers(0, 2, size=n).astype(np.int64)


def _oracle(method, Hr, s, win, iters):
    N = Hr.shape[1]
    p, neg = win >> 1, (win & 1).astype(bool)
    frames = np.stack([s[q:q + N] for q in p]).astype(np.float32)
    frames[neg] = -frames[neg]
    return orc.decode_batch(method, Hr, frames, iters)


@pytest.mark.parametrize("method,iters", [(1, 5), (1, 50), (0, 5), (0, 50)])
def test_serve_rounds_equal_launches_and_oracle(method, iters):
    dec = L.Decoder()
    Hr = dec.H
    s = _span(Hr, 600, 11 + method + iters)
    rng = np.random.default_rng(3)
    dec.stage_span(s, max_windows=4096)
    dec.serve_begin(method=method, max_iters=iters, max_windows=4096)
    rounds = [_windows(rng, n, s.size, dec.N) for n in (1, 7, 64, 300, 1021, 5000)]
    got = [dec.serve_windows(w) for w in rounds]
    dec.serve_end()
    for w, g in zip(rounds, got):
        ref = _oracle(method, Hr, s, w, iters)
        assert (g["packed"] == ref["packed"]).all()
        assert (g["synd"] == ref["synd"]).all()
        lw = dec.decode_windows(s, w, method=method, max_iters=iters)
        assert (lw["packed"] == g["packed"]).all() and (lw["synd"] == g["synd"]).all()
    dec.close()


@pytest.mark.parametrize("env", [{"LDPC_SERVE_BLOCKS_PER_CU": "1"}, {"LDPC_SERVE_DEBUG": "1"}],
                         ids=["one-workgroup-per-cu", "debug-counters"])
def test_serve_knobs(env):
    """The server's knobs (read per launch): one decoder workgroup per CU --
    rounds of 300 and 5000 windows then take the one-wave form, a round of
    one the workgroup form -- and the debug counters change no result."""
    dec = L.Decoder()
    Hr = dec.H
    s = _span(Hr, 400, 21)
    rng = np.random.default_rng(4)
    os.environ.update(env)
    try:
        dec.stage_span(s, max_windows=8192)
        dec.serve_begin(method=1, max_iters=5, max_windows=8192)
        rounds = [_windows(rng, n, s.size, dec.N) for n in (1, 300, 5000)]
        got = [dec.serve_windows(w) for w in rounds]
        dec.serve_end()
    finally:
        for k in env:
            os.environ.pop(k, None)
    for w, g in zip(rounds, got):
        ref = _oracle(1, Hr, s, w, 5)
        assert (g["packed"] == ref["packed"]).all() and (g["synd"] == ref["synd"]).all()
    dec.close()


def test_serve_survives_its_deadline():
    """A launch that ends on its deadline between rounds is replaced by the
    next round; a decode on the context's stream afterwards is not blocked."""
    dec = L.Decoder()
    Hr = dec.H
    s = _span(Hr, 200, 5)
    rng = np.random.default_rng(8)
    os.environ["LDPC_SERVE_DEADLINE_MS"] = "2"
    try:
        dec.stage_span(s, max_windows=512)
        dec.serve_begin(method=1, max_iters=5, max_windows=512)
        for _ in range(3):
            w = _windows(rng, 200, s.size, dec.N)
            g = dec.serve_windows(w)
            ref = _oracle(1, Hr, s, w, 5)
            assert (g["packed"] == ref["packed"]).all() and (g["synd"] == ref["synd"]).all()
            time.sleep(0.02)  # longer than the deadline: the launch has ended
    finally:
        os.environ.pop("LDPC_SERVE_DEADLINE_MS", None)
    dec.serve_end()
    out = dec.decode(s[37:37 + 64 * 4].reshape(4, 64), method=1, max_iters=5)
    ref = orc.decode_batch(1, Hr, s[37:37 + 64 * 4].reshape(4, 64), 5)
    assert (out["packed"] == ref["packed"]).all()
    dec.close()


def test_serve_errors():
    dec = L.Decoder()
    s = _span(dec.H, 10, 1)
    with pytest.raises(L.LdpcError):  # no server running
        dec.serve_windows(np.array([0], np.int64))
    dec.stage_span(s, max_windows=16)
    dec.serve_begin(method=1, max_iters=5, max_windows=16)
    with pytest.raises(L.LdpcError):  # past the span
        dec.serve_windows(np.array([(s.size - 63) << 1], np.int64))
    with pytest.raises(L.LdpcError):  # bit-flip: launches only
        dec.serve_begin(method=2, max_iters=5, max_windows=16)
    dec.close()


def test_serve_device_refuses_out_of_span_key():
    """The device checks every key against the staged span before it gathers
    (ldpc_serve.hip key_fault): a key past the span, let through the host's
    own check by the test seam, comes back as an error of the round -- not an
    illegal memory access -- in both the workgroup form (a round of a few
    windows) and the one-wave form (a round of more windows than decoders),
    and the server goes on serving correct rounds."""
    from ldpc_ece535a._capi import TEST_SERVE_UNCHECKED
    dec = L.Decoder()
    Hr = dec.H
    s = _span(Hr, 300, 31)
    rng = np.random.default_rng(9)
    dec.stage_span(s, max_windows=8192)
    dec.serve_begin(method=1, max_iters=5, max_windows=8192)
    far = (int(s.size) + (1 << 30)) << 1  # ~4 GB past the span's end
    for n in (3, 6000):
        w = _windows(rng, n, s.size, dec.N)
        w[n // 2] = far
        w[-1] = (s.size - dec.N + 1) << 1  # one sample past the end
        dec.test_hook(TEST_SERVE_UNCHECKED)
        with pytest.raises(L.LdpcError, match="LDPC_EDEVICE.*outside the staged span"):
            dec.serve_windows(w)
        good = _windows(rng, n, s.size, dec.N)
        g = dec.serve_windows(good)
        ref = _oracle(1, Hr, s, good, 5)
        assert (g["packed"] == ref["packed"]).all() and (g["synd"] == ref["synd"]).all()
    dec.serve_end()
    dec.close()


def test_serve_epoch_limit_restarts_the_session():
    """Round epochs stay below 2^23 - 2^16 (result tags are epoch mod 2^23):
    a session that reaches the limit is ended and started over before its
    next round, and every round's results stay right across it."""
    from ldpc_ece535a._capi import (SERVE_EPOCH_LIMIT, TEST_SERVE_EPOCH,
                                    TEST_SERVE_EPOCH_NOW)
    dec = L.Decoder()
    Hr = dec.H
    s = _span(Hr, 200, 41)
    rng = np.random.default_rng(10)
    dec.stage_span(s, max_windows=1024)
    dec.serve_begin(method=0, max_iters=5, max_windows=1024)
    dec.test_hook(TEST_SERVE_EPOCH, SERVE_EPOCH_LIMIT - 6)
    seen = []
    for n in (1, 700, 5, 64, 1, 300, 2, 9):
        w = _windows(rng, n, s.size, dec.N)
        g = dec.serve_windows(w)
        seen.append(dec.test_hook(TEST_SERVE_EPOCH_NOW))
        ref = _oracle(0, Hr, s, w, 5)
        assert (g["packed"] == ref["packed"]).all() and (g["synd"] == ref["synd"]).all()
    dec.serve_end()
    dec.close()
    assert max(seen) < SERVE_EPOCH_LIMIT and min(seen) < 16  # it restarted


@pytest.mark.parametrize("method", [0, 1])
def test_serve_special_samples_vs_oracle(method):
    """Windows over a span holding exact +0.0 / -0.0 samples, +-inf / NaN
    samples and amplitudes from 1e-38 to 1e30, both polarities, in rounds
    of both decode forms (one window per workgroup, one per wave): packed
    bytes and syndrome weights equal the oracle's decodes of the same
    samples."""
    dec = L.Decoder()
    Hr = dec.H
    s = _span(Hr, 400, 515 + method).astype(np.float64)
    rng = np.random.default_rng(808)
    n = s.size
    z = rng.random(n) < 0.08
    s[z & (rng.random(n) < 0.5)] = 0.0
    s[z & (s != 0.0)] = -0.0
    bad = rng.choice(n, size=40, replace=False)
    s[bad] = rng.choice([np.inf, -np.inf, np.nan], size=bad.size)
    seg = n // 8
    s[seg:2 * seg] *= 1e30
    s[2 * seg:3 * seg] *= 1e-38
    s[3 * seg:4 * seg] *= 1e3
    s = s.astype(np.float32)
    dec.stage_span(s, max_windows=4096)
    dec.serve_begin(method=method, max_iters=30, max_windows=4096)
    rounds = [_windows(rng, m, s.size, dec.N) for m in (1, 200, 3000)]
    got = [dec.serve_windows(w) for w in rounds]
    dec.serve_end()
    for w, g in zip(rounds, got):
        ref = _oracle(method, Hr, s, w, 30)
        bad_rows = np.flatnonzero((g["packed"] != ref["packed"]).any(axis=1))
        assert bad_rows.size == 0, (w[bad_rows[:4]], bad_rows[:8])
        assert (g["synd"] == ref["synd"]).all()
    dec.close()
