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
