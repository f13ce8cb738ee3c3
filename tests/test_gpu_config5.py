"""Config 5 (BASELINE.json configs[4]) pinned against the oracle: a mixed
Eb/N0 batch -- every frame at its own Eb/N0 in {0,1,2,3,4} dB -- decoded with
the early-termination test every 5 iterations.

The reference tests the syndrome after every iteration (SP :535-537, min-sum
:406-408); et_period 5 is the config-5 extension, restated in the oracle as
orc_decode_batch_et (et_period 1 == the reference, tests/test_oracle.py).
Hard decisions, packed bytes, iteration counts and syndrome weights must be
identical to the oracle for the small-code kernel (sum-product in both f64
parity modes, min-sum f64) and for the large-code (HBM message) kernels on
the same code, at B = 4096 and B = 65536."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EBN0 = (0, 1, 2, 3, 4)


def mixed_frames(Hr, B, seed):
    """Each frame at its own Eb/N0; sigma = sqrt(10^(-EbN0/10))
    (apps/ldpc_lapack.cpp:629-636); returns (frames, per-frame dB)."""
    import ldpc_ece535a as L
    rng = np.random.Generator(np.random.PCG64(seed))
    K = Hr.shape[1] - Hr.shape[0]
    x = 2.0 * L.encode(Hr, rng.integers(0, 2, size=(B, K), dtype=np.uint8)) - 1.0
    db = rng.choice(np.array(EBN0), size=B)
    sigma = np.sqrt(10.0 ** (-db / 10.0))[:, None]
    return (x + sigma * rng.standard_normal(x.shape)).astype(np.float32), db


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


_REF = {}


def reference(Hr, y, method, key):
    """Oracle outputs, cached per (batch, method) across the parametrised tests."""
    from oracle import oracle as orc
    k = (key, method)
    if k not in _REF:
        _REF[k] = orc.decode_batch(method, Hr, y, 50, nthreads=_threads(), et_period=5)
    return _REF[k]


@pytest.fixture(scope="module")
def small():
    import ldpc_ece535a as L
    return L.Decoder()


@pytest.fixture(scope="module")
def graph():
    import ldpc_ece535a as L
    d = L.Decoder(force_graph=True)
    assert d.path == 1
    return d


@pytest.fixture(scope="module")
def batches(small):
    return {B: mixed_frames(small.H, B, 500 + B) for B in (4096, 65536)}


@pytest.mark.parametrize("B", [4096, 65536])
@pytest.mark.parametrize("path,method,prec", [("small", 1, 0), ("small", 1, 2), ("small", 0, 0),
                                              ("graph", 1, 0), ("graph", 0, 0)])
def test_config5_mixed_ebn0_et5(small, graph, batches, B, path, method, prec):
    dec = small if path == "small" else graph
    y, db = batches[B]
    out = dec.decode(y, method=method, max_iters=50, et_period=5, precision=prec)
    ref = reference(small.H, y, method, B)
    bad = (out["bits"] != ref["bits"]).any(axis=1)
    assert bad.sum() == 0, "frames with different hard decisions: %d" % bad.sum()
    assert (out["packed"] == ref["packed"]).all()
    assert (out["iters"] == ref["iters"]).all()
    assert (out["synd"] == ref["synd"]).all()
    it = out["iters"]
    assert ((it % 5 == 0) | (it == 50)).all()
    # every Eb/N0 class is present and the batch really is mixed
    means = [it[db == d].mean() for d in EBN0]
    assert all(np.isfinite(means)) and means[0] > means[-1]


def test_config5_et5_vs_et1_property(small, batches):
    """Frames that converge (zero syndrome) at et_period 1 by iteration i stop
    at et_period 5 no later than the cap, and a stop before the cap always has
    a zero syndrome."""
    y, _ = batches[4096]
    o5 = small.decode(y, method=1, max_iters=50, et_period=5)
    early = o5["iters"] < 50
    assert (o5["synd"][early] == 0).all()
    o1 = small.decode(y, method=1, max_iters=50, et_period=1)
    assert o5["iters"].sum() >= o1["iters"].sum()
