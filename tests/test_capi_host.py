"""The C ABI without a GPU: the shared libraries load, export every symbol
their headers declare, and the host helpers (default H, reorderHMatrix,
checkFrame, makeParityCheck) agree with the oracle.  No decode is called
here: decoding needs the GPU (tests/test_gpu_*.py)."""
import ctypes
import os
import re

import numpy as np
import pytest

import ldpc_ece535a as L
from ldpc_ece535a import _capi, blocks
from oracle import oracle as orc

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    txt = open(os.path.join(REPO, "include", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ldpc_\w+)\s*\(", txt)) - {"ldpc_block_backend_fn"})


@pytest.mark.parametrize("header,libpath", [("ldpc_hip.h", _capi.HIP_LIB),
                                            ("ldpc_block.h", blocks.BLOCK_LIB)])
def test_library_exports_every_declared_symbol(header, libpath):
    lib = ctypes.CDLL(libpath)
    names = declared(header)
    assert len(names) >= 8
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_the_header():
    assert set(declared("ldpc_hip.h")) == set(_capi.SIGNATURES)
    assert set(declared("ldpc_block.h")) == set(blocks.SIGNATURES)


def test_default_h(golden):
    assert (L.default_h() == golden("reference_data.npz")["decoder_h"]).all()


@pytest.mark.parametrize("name", ["hData1", "hData2", "hData3", "hData4", "hData5", "qa_h"])
def test_reorder_matches_oracle(golden, name):
    H = golden("reference_data.npz")[name]
    Hr, chosen = L.reorder_h(H)
    Ho, cho, _, _ = orc.reorder_h(H)
    assert (Hr == Ho).all() and (chosen == cho).all()


def test_check_frame_matches_oracle(golden):
    Hr = golden("frames_default.npz")["H_reordered"]
    rng = np.random.default_rng(0)
    for _ in range(200):
        bits = rng.integers(0, 2, 64).astype(np.uint8)
        for thr in (0, 4, 32):
            assert L.check_frame(Hr, bits, thr) == orc.check_frame(Hr, bits, thr)


@pytest.mark.parametrize("name", ["decoder_h", "qa_h", "hData5"])
def test_encode_matches_oracle(golden, name):
    ref = golden("reference_data.npz")
    Hr, _, Lf, Uf = orc.reorder_h(ref[name])
    M, N = Hr.shape
    rng = np.random.default_rng(1)
    data = rng.integers(0, 2, size=(64, N - M), dtype=np.uint8)
    assert (L.encode(Hr, data) == orc.encode(Hr, Lf, Uf, data)).all()


def test_encode_kat_8x16(golden):
    ref = golden("reference_data.npz")
    Hr, _ = L.reorder_h(ref["qa_h"])
    cw = L.encode(Hr, np.unpackbits(ref["kat_data"]).reshape(8, 8))
    assert ((2 * cw[:, :8].astype(int) - 1) == ref["kat_mod_check"]).all()


def test_encode_rejects_unreordered_h(golden):
    H = golden("reference_data.npz")["decoder_h"]
    with pytest.raises(L.LdpcError):
        L.encode(H, np.zeros((1, 32), np.uint8))


def test_bad_h_rejected():
    with pytest.raises(L.LdpcError):
        L.reorder_h(np.full((4, 8), 2, np.uint8))


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(L.LdpcError, match="no CPU fallback"):
        L.Decoder()
    with pytest.raises(L.LdpcError):
        L.ldpc_decoder_cb(1)


def test_create_csr_validates_and_has_no_cpu_fallback():
    import torch
    rp = np.array([0, 2, 4], np.int32)
    bad = [  # (M, N, row_ptr, col_idx)
        (2, 4, rp, np.array([1, 0, 2, 3], np.int32)),   # not ascending
        (2, 4, rp, np.array([0, 1, 2, 4], np.int32)),   # out of range
        (2, 4, np.array([0, 3, 2], np.int32), np.array([0, 1, 2, 3], np.int32)),
        (4, 4, np.array([0, 1, 2, 3, 4], np.int32), np.arange(4, dtype=np.int32)),  # M >= N
    ]
    for csr in bad:
        with pytest.raises(L.LdpcError, match="CSR H must be"):
            L.Decoder(csr=csr)
    if not torch.cuda.is_available():
        with pytest.raises(L.LdpcError, match="no CPU fallback"):
            L.Decoder(csr=(2, 4, rp, np.array([0, 1, 2, 3], np.int32)))
        from ldpc_ece535a import codes
        with pytest.raises(L.LdpcError, match="no CPU fallback"):
            L.Decoder(csr=codes.dvbs2_like(0))


def test_degree_limits_reported_before_device_lookup():
    H = np.zeros((300, 600), np.uint8)
    H[np.arange(300), np.arange(300)] = 1
    H[:, 300] = 1  # column degree 300 > the large-code kernels' 16
    with pytest.raises(L.LdpcError, match="outside the large-code kernels"):
        L.Decoder(H)


def test_ber_octave_format_and_grid():
    from ldpc_ece535a import ber
    g = ber.parse_range("-7:10:0.5")
    assert len(g) == 35 and g[0] == -7.0 and g[-1] == 10.0 and g == ber.DEFAULT_EBN0
    assert abs(ber.sigma_of(2.0) - np.sqrt(10 ** -0.2)) < 1e-15
    res = {n: {"ber": [0.5, 0.25], "fer": [3, 0]} for n, _ in ber.METHODS}
    txt = ber.octave([0.0, 1.5], res)
    lines = txt.splitlines()
    assert lines[0] == "EbN0=[0 1.5 ];" and lines[2] == "ber0=[0.5 0.25 ];"
    assert "fer3=[" in txt and "3, 0" in txt
