"""GPU parity: the HIP decode path (through the C ABI) against the golden
fixtures written by the C oracle (tests/golden/make_golden.py)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dec():
    import ldpc_ece535a
    return ldpc_ece535a.Decoder()  # default H, reordered like the block


@pytest.mark.parametrize("db", [0, 2, 4])
@pytest.mark.parametrize("method", [0, 1, 2, 3])
@pytest.mark.parametrize("iters", [5, 50])
def test_default_h_fixtures_f64(dec, golden, db, method, iters):
    fd = golden("frames_default.npz")
    assert (dec.H == fd["H_reordered"]).all()
    llr = fd["db%d_llr" % db]
    out = dec.decode(llr, method=method, max_iters=iters, precision=0, want_llr=True)
    key = "db%d_m%d_i%d" % (db, method, iters)
    np.testing.assert_array_equal(out["bits"], fd[key + "_bits"])
    np.testing.assert_array_equal(out["packed"], fd[key + "_packed"])
    np.testing.assert_array_equal(out["iters"], fd[key + "_iters"])
    np.testing.assert_array_equal(out["synd"], fd[key + "_synd"])
    if method == 0 or method >= 2:
        # min-sum / hard / bit-flip posteriors are exact in f64
        np.testing.assert_array_equal(out["llr"], fd[key + "_post"])
    else:
        np.testing.assert_allclose(out["llr"], fd[key + "_post"], rtol=1e-6, atol=1e-6)
