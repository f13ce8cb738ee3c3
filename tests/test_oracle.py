"""The oracle (oracle/) pinned against the reference's own known-answer
vectors and cross-checked against the independent pure-Python restatement.

KATs: python/qa_ldpc_encoder_bc.py:21-41 and python/qa_ldpc_decoder_cb.py:20-43
of gr-ldpc_ece535a, which assume the 8x16 H (apps/test_data.h:119-131 ==
the commented H at lib/ldpc_decoder_cb_impl.cc:48-57).
"""
import numpy as np
import pytest

from oracle import ldpc_oracle_py as pyo
from oracle import oracle as orc

# columns chosen by reorderHMatrix on the default H
SURVEY_CHOSEN = [6, 5, 14, 9, 15, 7, 26, 26, 9, 37, 10, 13, 25, 15, 18, 20, 18, 19, 23, 21, 22,
                 23, 29, 24, 25, 26, 27, 29, 28, 33, 31, 32]


def test_default_h_is_the_decoders(golden):
    ref = golden("reference_data.npz")
    assert (ref["decoder_h"] == ref["hData4"]).all()
    Hr, chosen, _, _ = orc.reorder_h(ref["decoder_h"])
    assert list(chosen) == SURVEY_CHOSEN
    assert Hr.sum() == 168
    assert sorted(set(Hr.sum(0))) == [1, 2, 3] and sorted(set(Hr.sum(1))) == [4, 5, 6]


def test_encoder_kat_8x16(golden):
    ref = golden("reference_data.npz")
    Hr, _, L, U = orc.reorder_h(ref["qa_h"])
    bits = np.unpackbits(ref["kat_data"]).reshape(8, 8)
    cw = orc.encode(Hr, L, U, bits)
    assert ((2 * cw[:, :8].astype(int) - 1) == ref["kat_mod_check"]).all()
    assert ((2 * cw[:, 8:].astype(int) - 1) == ref["kat_mod_data"]).all()


@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_decoder_kat_8x16(golden, method):
    ref = golden("reference_data.npz")
    Hr, _, _, _ = orc.reorder_h(ref["qa_h"])
    frames = np.concatenate([ref["kat_mod_check"], ref["kat_mod_data"]], 1).astype(np.float32)
    out = orc.decode_batch(method, Hr, frames, 5)
    assert (out["packed"].ravel() == ref["kat_expected"]).all()
    # the stream-level restatement (general_work) recovers the same bytes
    stream = frames.reshape(-1).astype(np.complex64)
    assert (orc.run_stream(method, Hr, stream, iterations=5) == ref["kat_expected"]).all()


@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_c_oracle_matches_python_restatement(golden, method):
    fd = golden("frames_default.npz")
    Hr = fd["H_reordered"]
    y = fd["db2_llr"][:4]
    out = orc.decode_batch(method, Hr, y, 50)
    for b in range(y.shape[0]):
        v, used = pyo.decode(method, Hr.tolist(), [float(x) for x in y[b]], 50)
        assert list(out["bits"][b]) == v
        assert out["iters"][b] == used


def test_oracle_reproduces_fixtures(golden):
    fd = golden("frames_default.npz")
    Hr = fd["H_reordered"]
    for db in (0, 2, 4):
        for m in (0, 1, 2, 3):
            for it in (5, 50):
                key = "db%d_m%d_i%d" % (db, m, it)
                out = orc.decode_batch(m, Hr, fd["db%d_llr" % db], it, nthreads=4)
                assert (out["bits"] == fd[key + "_bits"]).all(), key
                assert (out["iters"] == fd[key + "_iters"]).all(), key


def test_python_reorder_matches_c(golden):
    ref = golden("reference_data.npz")
    for name in ("hData1", "hData2", "hData3", "hData4", "hData5"):
        Hc, chc, Lc, Uc = orc.reorder_h(ref[name])
        Hp, chp, Lp, Up = pyo.reorder_h(ref[name].tolist())
        assert (np.array(Hp) == Hc).all() and list(chc) == chp, name
        assert (np.array(Lp) == Lc).all() and (np.array(Up) == Uc).all(), name


def test_encode_satisfies_checks(golden):
    ref = golden("reference_data.npz")
    Hr, _, L, U = orc.reorder_h(ref["decoder_h"])
    rng = np.random.default_rng(3)
    data = rng.integers(0, 2, size=(200, 32), dtype=np.uint8)
    cw = orc.encode(Hr, L, U, data)
    assert not ((Hr.astype(int) @ cw.T.astype(int)) % 2).any()
    # the reference's own source-bit matrix (apps/test_data.h:180, 32 x frames)
    src = ref["dSourceData4"].T
    cw2 = orc.encode(Hr, L, U, src)
    assert not ((Hr.astype(int) @ cw2.T.astype(int)) % 2).any()


def test_streams_fixture_chunking_invariance(golden):
    st = golden("streams.npz")
    Hr = golden("frames_default.npz")["H_reordered"]
    rng = np.random.default_rng(11)
    for name in ("offset", "burst"):
        s = st[name + "_in"]
        chunks = rng.integers(1, 90, size=len(s))
        got = orc.run_stream(1, Hr, s, iterations=5, chunks=chunks)
        assert (got == st[name + "_m1_out"]).all()


@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_sparse_restatement_equals_dense(golden, method):
    """orc_decode_batch_sparse (CSR/CSC loops, used for codes too large for
    the dense restatement) is bit-identical to the dense restatement."""
    fd = golden("frames_default.npz")
    Hr = fd["H_reordered"]
    rp, ci = orc.dense_to_csr(Hr)
    for db in (0, 2, 4):
        y = fd["db%d_llr" % db]
        a = orc.decode_batch(method, Hr, y, 50, nthreads=4)
        b = orc.decode_batch_sparse(method, rp, ci, 32, 64, y, 50, nthreads=4)
        for k in ("bits", "packed", "iters", "synd"):
            assert (a[k] == b[k]).all(), k
    ref = golden("reference_data.npz")
    fo = golden("frames_other.npz")
    for name in ("hData1", "hData2", "hData3", "hData5"):
        H = fo[name + "_H_reordered"]
        rp, ci = orc.dense_to_csr(H)
        b = orc.decode_batch_sparse(method, rp, ci, H.shape[0], H.shape[1], fo[name + "_llr"], 20)
        assert (b["bits"] == fo["%s_m%d_bits" % (name, method)]).all()
        assert (b["iters"] == fo["%s_m%d_iters" % (name, method)]).all()
    assert ref is not None


def test_dvbs2_like_code_structure():
    """Config 4's code: the DVB-S2 rate-1/2 normal-frame profile, and the
    IRA encoder's codewords satisfy every check."""
    from ldpc_ece535a import codes
    csr = codes.dvbs2_like(0)
    M, N, rp, ci = csr
    assert (M, N, int(rp[-1])) == (32400, 64800, 226799)
    rdeg = np.bincount(np.diff(rp))
    assert rdeg[7] == 32399 and rdeg[6] == 1
    cdeg = np.bincount(np.bincount(ci, minlength=N))
    assert (cdeg[8], cdeg[3], cdeg[2], cdeg[1]) == (12960, 19440, 32399, 1)
    rng = np.random.default_rng(3)
    info = rng.integers(0, 2, (3, 32400), dtype=np.uint8)
    cw = codes.ira_encode(csr, info)
    assert (codes.syndrome_weight(csr, cw) == 0).all()
    assert (cw[:, M:] == info).all()
    # the oracle's sparse checkFrame agrees, and min-sum decodes a 2 dB frame
    x = 2.0 * cw[:1] - 1.0
    y = (x + np.sqrt(10 ** -0.2) * rng.standard_normal(x.shape)).astype(np.float32)
    r = orc.decode_batch_sparse(0, rp, ci, M, N, y, 50, want_bits=False)
    assert r["synd"][0] == 0 and (r["packed"][0] == np.packbits(info[0])).all()


def _mixed_ebn0_frames(Hr, B, seed):
    """Config 5's input: each frame at its own Eb/N0 in {0,1,2,3,4} dB
    (sigma = sqrt(10^(-EbN0/10)), apps/ldpc_lapack.cpp:629-636)."""
    from ldpc_ece535a import encode
    rng = np.random.Generator(np.random.PCG64(seed))
    K = Hr.shape[1] - Hr.shape[0]
    x = 2.0 * encode(Hr, rng.integers(0, 2, size=(B, K), dtype=np.uint8)) - 1.0
    db = rng.integers(0, 5, size=B)
    sigma = np.sqrt(10.0 ** (-db / 10.0))[:, None]
    return (x + sigma * rng.standard_normal(x.shape)).astype(np.float32)


@pytest.mark.parametrize("method", [0, 1, 2])
def test_et_period_c_matches_python_restatement(golden, method):
    """The early-termination period (config 5) restated twice, independently."""
    Hr = golden("frames_default.npz")["H_reordered"]
    y = _mixed_ebn0_frames(Hr, 6, 55)
    for et in (2, 5):
        out = orc.decode_batch(method, Hr, y, 50, et_period=et)
        for b in range(y.shape[0]):
            v, used = pyo.decode(method, Hr.tolist(), [float(x) for x in y[b]], 50, et)
            assert list(out["bits"][b]) == v, (et, b)
            assert out["iters"][b] == used, (et, b)


@pytest.mark.parametrize("method", [0, 1, 2])
def test_et_period_sparse_equals_dense(golden, method):
    Hr = golden("frames_default.npz")["H_reordered"]
    rp, ci = orc.dense_to_csr(Hr)
    y = _mixed_ebn0_frames(Hr, 64, 56)
    M, N = Hr.shape
    for et in (1, 5):
        d = orc.decode_batch(method, Hr, y, 50, nthreads=4, et_period=et)
        s = orc.decode_batch_sparse(method, rp, ci, M, N, y, 50, nthreads=4, et_period=et)
        for k in ("bits", "packed", "iters", "synd"):
            assert (d[k] == s[k]).all(), (et, k)


def test_et_period_stops_only_on_period(golden):
    """With et_period 5 a frame stops at a multiple of 5 or at the cap; with
    et_period 1 the oracle equals its plain entry point (the reference)."""
    Hr = golden("frames_default.npz")["H_reordered"]
    y = _mixed_ebn0_frames(Hr, 128, 57)
    for m in (0, 1, 2):
        o5 = orc.decode_batch(m, Hr, y, 50, nthreads=4, et_period=5)
        assert ((o5["iters"] % 5 == 0) | (o5["iters"] == 50)).all()
        # a frame stopped early has a zero syndrome
        early = o5["iters"] < 50
        assert (o5["synd"][early] == 0).all()
        o1 = orc.decode_batch(m, Hr, y, 50, nthreads=4, et_period=1)
        o1c = orc.decode_batch(m, Hr, y, 50, nthreads=4)
        for k in ("bits", "iters", "synd"):
            assert (o1[k] == o1c[k]).all()


@pytest.mark.parametrize("name", ["offset", "burst"])
def test_sparse_block_restatement_matches_dense(golden, name):
    """orc_block_general_work_sparse (the loop with every window decoded by
    the sparse restatement, for large codes) gives the dense block's bytes --
    and the fixtures' -- on the default H."""
    st = golden("streams.npz")
    Hr = golden("frames_default.npz")["H_reordered"]
    rp, ci = orc.dense_to_csr(Hr)
    s = st[name + "_in"]
    for m in (0, 1, 2, 3):
        sp = orc.run_stream(m, None, s, iterations=5, csr=(Hr.shape[0], Hr.shape[1], rp, ci),
                            chunks=[700, 33, 5000] * 40)
        assert (sp == st["%s_m%d_out" % (name, m)]).all(), m
