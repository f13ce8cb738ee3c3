"""GPU parity of the large-code path (ldpc_graph.hip, messages in HBM).

1. Forced onto the reference's own codes (LDPC_FLAG_GRAPH), it must give the
   golden fixtures bit for bit, exactly like the small-code kernel.
2. On the DVB-S2-size code of SURVEY 8(d) config 4 (N = 64800, synthetic
   address table with the rate-1/2 profile, ldpc_ece535a.codes) it is checked
   against the oracle's sparse restatement (oracle/ldpc_oracle.c
   orc_decode_batch_sparse, itself checked against the dense restatement in
   tests/test_oracle.py) and, at full batch size, by encode -> noise ->
   decode round trips.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gdec():
    import ldpc_ece535a as L
    d = L.Decoder(force_graph=True)
    assert d.path == L._capi.PATH_GRAPH
    return d


@pytest.fixture(scope="module")
def dvb():
    import ldpc_ece535a as L
    from ldpc_ece535a import codes
    csr = codes.dvbs2_like(0)
    d = L.Decoder(csr=csr)
    assert d.path == L._capi.PATH_GRAPH and d.E == 226799
    return csr, d


def _noisy(csr, B, db, seed):
    from ldpc_ece535a import codes
    rng = np.random.Generator(np.random.PCG64(seed))
    info = rng.integers(0, 2, size=(B, csr[1] - csr[0]), dtype=np.uint8)
    x = 2.0 * codes.ira_encode(csr, info) - 1.0
    y = (x + np.sqrt(10 ** (-db / 10)) * rng.standard_normal(x.shape)).astype(np.float32)
    return info, y


@pytest.mark.parametrize("prec", [0, 2])
@pytest.mark.parametrize("db", [0, 2, 4])
@pytest.mark.parametrize("method", [0, 1, 2, 3])
@pytest.mark.parametrize("iters", [5, 50])
def test_graph_path_default_h_fixtures(gdec, golden, db, method, iters, prec):
    fd = golden("frames_default.npz")
    assert (gdec.H == fd["H_reordered"]).all()
    out = gdec.decode(fd["db%d_llr" % db], method=method, max_iters=iters, precision=prec,
                      want_llr=True)
    key = "db%d_m%d_i%d" % (db, method, iters)
    np.testing.assert_array_equal(out["bits"], fd[key + "_bits"])
    np.testing.assert_array_equal(out["packed"], fd[key + "_packed"])
    np.testing.assert_array_equal(out["iters"], fd[key + "_iters"])
    np.testing.assert_array_equal(out["synd"], fd[key + "_synd"])
    # every f64 mode here is exact (sum-product: ldpc_exact.hpp)
    np.testing.assert_array_equal(out["llr"], fd[key + "_post"])


@pytest.mark.parametrize("name", ["hData1", "hData2", "hData3", "hData5"])
@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_graph_path_other_h(golden, name, method):
    import ldpc_ece535a as L
    fo = golden("frames_other.npz")
    d = L.Decoder(golden("reference_data.npz")[name], force_graph=True)
    out = d.decode(fo[name + "_llr"], method=method, max_iters=20, precision=0)
    np.testing.assert_array_equal(out["bits"], fo["%s_m%d_bits" % (name, method)])
    np.testing.assert_array_equal(out["iters"], fo["%s_m%d_iters" % (name, method)])
    np.testing.assert_array_equal(out["synd"], fo["%s_m%d_synd" % (name, method)])


def test_graph_path_strided_polarity_groups(gdec, golden):
    """Strided gr_complex windows, polarity -1, a batch that is not a
    multiple of 64, and a workspace cap that forces several groups."""
    from oracle import oracle as orc
    fd = golden("frames_default.npz")
    y = fd["db2_llr"][:60].reshape(-1)
    z = np.zeros(2 * y.size + 10, np.float32)
    z[10::2] = y
    B = 1000  # 1-sample steps through the stream
    n = (z.size - 10 - 128) // 2
    B = min(B, n)
    gdec.set_work_limit(200 * 1024)  # a few 64-frame chunks per group
    try:
        for pol in (1.0, -1.0):
            out = gdec.decode(z[10:], method=1, max_iters=50, polarity=pol, cw_stride=2,
                              elem_stride=2, B=B)
            ref = orc.decode_batch(1, fd["H_reordered"], z[10:], 50, polarity=pol, cw_stride=2,
                                   elem_stride=2, B=B, nthreads=8)
            assert (out["bits"] == ref["bits"]).all()
            assert (out["iters"] == ref["iters"]).all()
            assert (out["synd"] == ref["synd"]).all()
    finally:
        gdec.set_work_limit(0)


def test_graph_path_et_period(gdec, golden):
    from oracle import oracle as orc  # noqa: F401
    fd = golden("frames_default.npz")
    small = __import__("ldpc_ece535a").Decoder()
    a = gdec.decode(fd["db4_llr"], method=1, max_iters=50, et_period=5)
    b = small.decode(fd["db4_llr"], method=1, max_iters=50, et_period=5)
    for k in ("bits", "iters", "synd", "packed"):
        assert (a[k] == b[k]).all()


@pytest.mark.parametrize("db,iters", [(2, 50), (1, 30)])
def test_dvbs2_like_minsum_f64_vs_sparse_oracle(dvb, db, iters):
    from oracle import oracle as orc
    csr, d = dvb
    M, N, rp, ci = csr
    info, y = _noisy(csr, 96, db, seed=10 + db)
    out = d.decode(y, method=0, max_iters=iters, precision=0)
    ref = orc.decode_batch_sparse(0, rp, ci, M, N, y, iters, nthreads=16)
    np.testing.assert_array_equal(out["iters"], ref["iters"])
    np.testing.assert_array_equal(out["synd"], ref["synd"])
    np.testing.assert_array_equal(out["bits"], ref["bits"])
    np.testing.assert_array_equal(out["packed"], ref["packed"])


@pytest.mark.parametrize("prec", [0, 2])
@pytest.mark.parametrize("method", [1, 2, 3])
def test_dvbs2_like_other_methods_vs_sparse_oracle(dvb, method, prec):
    """Sum-product on this code saturates tanh -> log(2/0) = inf -> NaN
    messages, exactly as the reference's unclipped arithmetic does; both
    exact f64 modes (glibc's tanh / log reproduced) must follow the oracle
    through it."""
    from oracle import oracle as orc
    csr, d = dvb
    M, N, rp, ci = csr
    info, y = _noisy(csr, 16, 2, seed=20 + method)
    iters = 12
    out = d.decode(y, method=method, max_iters=iters, precision=prec)
    ref = orc.decode_batch_sparse(method, rp, ci, M, N, y, iters, nthreads=16)
    np.testing.assert_array_equal(out["iters"], ref["iters"])
    np.testing.assert_array_equal(out["synd"], ref["synd"])
    np.testing.assert_array_equal(out["bits"], ref["bits"])


def test_dvbs2_like_full_batch_roundtrip(dvb):
    """Config-4 batch (1024 frames at 2 dB): every frame decodes to its info
    bits with a zero syndrome, f64 and f32; all 1024 f64 frames (packed
    bytes, iterations, syndromes) equal the sparse oracle's."""
    csr, d = dvb
    M, N, rp, ci = csr
    info, y = _noisy(csr, 1024, 2, seed=4)
    want = np.packbits(info, axis=1)
    from oracle import oracle as orc
    ref = orc.decode_batch_sparse(0, rp, ci, M, N, y, 50, nthreads=16, want_bits=False)
    for prec in (0, 1):
        out = d.decode(y, method=0, max_iters=50, precision=prec, want_bits=False)
        assert (out["synd"] == 0).all()
        assert (out["packed"] == want).all()
        if prec == 0:
            for k in ("packed", "iters", "synd"):
                np.testing.assert_array_equal(out[k], ref[k], err_msg=k)


@pytest.mark.parametrize("method,db,compact", [(0, 2, "1"), (1, 2, "1"), (0, 4, "1"), (1, 1, "1"),
                                               (1, 2, "0")])
def test_graph_path_repeated_compaction(method, db, compact, monkeypatch):
    """Thousands of frames on the large-code kernels: running frames are
    compacted several times as others stop (sum-product's edge-message
    passes; LDPC_GRAPH_COMPACT=0: never); every output (bits, iterations,
    syndromes, posteriors) must still be the oracle's."""
    import bench
    import ldpc_ece535a as L
    from oracle import oracle as orc
    monkeypatch.setenv("LDPC_GRAPH_COMPACT", compact)
    d = L.Decoder(force_graph=True)
    y, _ = bench.synth(d.H, 4096, db, 50 + db)
    out = d.decode(y, method=method, max_iters=50, precision=0, want_llr=True)
    ref = orc.decode_batch(method, d.H, y, 50, nthreads=16, want_post=True)
    np.testing.assert_array_equal(out["iters"], ref["iters"])
    np.testing.assert_array_equal(out["synd"], ref["synd"])
    np.testing.assert_array_equal(out["bits"], ref["bits"])
    np.testing.assert_array_equal(out["llr"], ref["post"])
