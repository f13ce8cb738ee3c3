"""The LDS layout search (csrc/ldpc_layout.hpp) moves edges and columns to
other lanes and cells, never the arithmetic: every output of every method,
precision and schedule is identical between the planned layout and the plain
CSR layout (LDPC_FLAG_PLAIN_LAYOUT), on the reference's codes and on random
codes of the small-code kernel's other shapes (two column words, six and
eight edge slots), and matches the oracle in the f64 parity modes."""
import numpy as np
import pytest

import ldpc_ece535a as L

pytestmark = pytest.mark.gpu


def random_code(rng, M, N, dv):
    H = np.zeros((M, N), np.uint8)
    deg = np.zeros(M)
    for i in range(N):
        rows = np.lexsort((rng.random(M), deg))[:dv]
        H[rows, i] = 1
        deg[rows] += 1
    return H


def code(golden, name):
    if name.startswith("rand"):
        M, N, dv = {"rand96x192": (96, 192, 2), "rand64x128": (64, 128, 3),
                    "rand128x256": (128, 256, 2)}[name]
        return random_code(np.random.default_rng(M + N), M, N, dv)
    return golden("reference_data.npz")[name]


def frames(Hr, B, db, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    K = Hr.shape[1] - Hr.shape[0]
    data = rng.integers(0, 2, size=(B, K), dtype=np.uint8)
    try:
        x = 2.0 * L.encode(Hr, data) - 1.0
    except L.LdpcError:  # no systematic encoder (dependent columns): all-zero word
        x = -np.ones((B, Hr.shape[1]))
    return (x + np.sqrt(10 ** (-db / 10)) * rng.standard_normal(x.shape)).astype(np.float32)


NAMES = ["decoder_h", "hData2", "hData5", "qa_h", "rand96x192", "rand64x128", "rand128x256"]


@pytest.mark.parametrize("name", NAMES)
def test_planned_layout_equals_plain_layout(golden, name):
    H = code(golden, name)
    a = L.Decoder(H)
    b = L.Decoder(H, plain_layout=True)
    assert a.path == 0 and b.path == 0
    assert b.layout_model["searched"] == 0
    y = frames(a.H, 256, 2.0, 11)
    for sched in (1, 2):
        a.set_schedule(sched)
        b.set_schedule(sched)
        for method in (0, 1, 2, 3):
            for prec in ((0, 1, 2) if method <= 1 else (0,)):
                ra = a.decode(y, method=method, max_iters=30, precision=prec, want_llr=True)
                rb = b.decode(y, method=method, max_iters=30, precision=prec, want_llr=True)
                for k in ("packed", "bits", "iters", "synd"):
                    assert (ra[k] == rb[k]).all(), (name, sched, method, prec, k)
                assert np.array_equal(ra["llr"], rb["llr"], equal_nan=True), (name, sched, method, prec)


@pytest.mark.parametrize("name", ["decoder_h", "hData2", "rand96x192", "rand128x256"])
@pytest.mark.parametrize("method", [0, 1])
def test_planned_layout_matches_oracle(golden, name, method):
    from oracle import oracle as orc
    H = code(golden, name)
    dec = L.Decoder(H)
    y = frames(dec.H, 512, 1.5, 23)
    out = dec.decode(y, method=method, max_iters=50)
    ref = orc.decode_batch(method, dec.H, y, 50, nthreads=8)
    assert (out["packed"] == ref["packed"]).all()
    assert (out["bits"] == ref["bits"]).all()
    assert (out["iters"] == ref["iters"]).all()
    assert (out["synd"] == ref["synd"]).all()


def test_default_layout_model(golden):
    m = L.Decoder().layout_model
    assert m["searched"] == 1 and m["cc"] == 0 and m["ec"] == 0, m


@pytest.mark.parametrize("prec", [0, 1, 2])
@pytest.mark.parametrize("method", [0, 1])
def test_throughput_build_equals_latency_build(golden, method, prec):
    """The throughput launch mode runs a different build of the kernel (four
    waves per SIMD, no issue priority) on the reference's H: same outputs."""
    from oracle import oracle as orc
    dec = L.Decoder()
    y = frames(dec.H, 2048, 2.0, 31)
    dec.set_launch_mode(0)
    a = dec.decode(y, method=method, max_iters=50, precision=prec, want_llr=True)
    dec.set_launch_mode(1)
    b = dec.decode(y, method=method, max_iters=50, precision=prec, want_llr=True)
    for k in ("packed", "bits", "iters", "synd"):
        assert (a[k] == b[k]).all(), k
    assert np.array_equal(a["llr"], b["llr"], equal_nan=True)
    if prec != 1:
        ref = orc.decode_batch(method, dec.H, y, 50, nthreads=8)
        assert (b["packed"] == ref["packed"]).all() and (b["iters"] == ref["iters"]).all()
