"""Parity at scale: 16384 seeded frames per (method, Eb/N0), f64 parity mode,
against the oracle run on the host's cores.  Hard decisions, packed bytes,
iteration counts and syndrome weights must all be identical."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dec():
    import ldpc_ece535a as L
    return L.Decoder()


def frames(Hr, B, db, seed):
    import ldpc_ece535a as L
    rng = np.random.Generator(np.random.PCG64(seed))
    data = rng.integers(0, 2, size=(B, 32), dtype=np.uint8)
    x = 2.0 * L.encode(Hr, data) - 1.0
    return (x + np.sqrt(10 ** (-db / 10)) * rng.standard_normal(x.shape)).astype(np.float32)


@pytest.mark.parametrize("method,db,sched", [(1, 0.0, 1), (1, 1.0, 2), (1, 2.0, 1), (1, 2.0, 2),
                                             (1, 3.0, 1), (0, 0.0, 2), (0, 2.0, 1), (0, 4.0, 2),
                                             (2, 2.0, 0)])
def test_parity_16k(dec, method, db, sched):
    from oracle import oracle as orc
    y = frames(dec.H, 16384, db, seed=int(100 + 10 * db + method))
    dec.set_schedule(sched)
    out = dec.decode(y, method=method, max_iters=50)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    ref = orc.decode_batch(method, dec.H, y, 50, nthreads=threads)
    bad = (out["bits"] != ref["bits"]).any(axis=1)
    assert bad.sum() == 0, "frames with different hard decisions: %d" % bad.sum()
    assert (out["iters"] == ref["iters"]).all()
    assert (out["synd"] == ref["synd"]).all()
