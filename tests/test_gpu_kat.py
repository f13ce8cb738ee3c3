"""The reference's own decoder known-answer test, on the GPU.

python/qa_ldpc_decoder_cb.py:20-43 feeds 8 noiseless frames of the 8x16 H
(apps/test_data.h:119-131, the H commented out at
lib/ldpc_decoder_cb_impl.cc:48-57) -- check symbols then data symbols, the
encoder KAT's output (python/qa_ldpc_encoder_bc.py:21-41) -- through the
decoder block and expects the 8 data bytes back (:43, :52-57).  Here the same
frames go through every GPU entry point: the C ABI's Decoder(qa_h) (small-code
kernels under both schedules, and the large-code kernels), the block
ldpc_decoder_cb(method, 5, 0, qa_h) under the scheduler harness, and the
compiled C++ caller make(method, 5, 0, alist) through the gr::block interface.
Every path must yield kat_expected.
"""
import os
import subprocess

import numpy as np
import pytest

import ldpc_ece535a as L
from ldpc_ece535a import flowgraph as fg

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _kat(golden):
    ref = golden("reference_data.npz")
    frames = np.concatenate([ref["kat_mod_check"], ref["kat_mod_data"]], 1).astype(np.float32)
    return ref["qa_h"], frames, ref["kat_expected"]


@pytest.mark.parametrize("prec", [0, 1, 2, 3])
@pytest.mark.parametrize("sched", [1, 2])
@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_kat_decoder_small_code(golden, method, sched, prec):
    qa_h, frames, expected = _kat(golden)
    dec = L.Decoder(qa_h)
    dec.set_schedule(sched)
    out = dec.decode(frames, method=method, max_iters=5, precision=prec)
    assert (out["packed"].ravel() == expected).all()
    assert (out["synd"] == 0).all()


@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_kat_decoder_large_code_path(golden, method):
    qa_h, frames, expected = _kat(golden)
    dec = L.Decoder(qa_h, force_graph=True)
    out = dec.decode(frames, method=method, max_iters=5, precision=0)
    assert (out["packed"].ravel() == expected).all()


@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_kat_block(golden, method):
    """python/qa_ldpc_decoder_cb.py:45-57: vector_source_c -> decoder ->
    vector_sink_b, with the block built on the 8x16 H and 5 iterations."""
    qa_h, frames, expected = _kat(golden)
    blk = L.ldpc_decoder_cb(method, 5, 0, H=qa_h)
    assert (blk.M, blk.N, blk.frame_bytes) == (8, 16, 1)
    for chunk in (None, [5, 16, 3, 40]):
        blk = L.ldpc_decoder_cb(method, 5, 0, H=qa_h)
        tb = fg.top_block(chunk=chunk) if chunk else fg.top_block()
        src, dst = fg.vector_source_c(frames.reshape(-1).astype(np.complex64)), fg.vector_sink_b()
        tb.connect((src, 0), (blk, 0))
        tb.connect((blk, 0), (dst, 0))
        tb.run()
        assert (dst.array() == expected).all()
        assert blk.state == L.STATE_IN_SYNC


@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_kat_native_caller(tmp_path, golden, method):
    """make(method, 5, 0, alist_path) from C++ through the gr::block interface."""
    _, frames, expected = _kat(golden)
    exe = os.path.join(REPO, "gr-ldpc_ece535a_amd", "lib", "block_make_test")
    assert os.path.exists(exe), "build first: make -C gr-ldpc_ece535a_amd native"
    path = os.path.join(REPO, "tests", "golden", "hData3.alist")
    fin, fout = str(tmp_path / "in.f32"), str(tmp_path / "out.u8")
    frames.reshape(-1).astype(np.complex64).view(np.float32).tofile(fin)
    r = subprocess.run([exe, str(method), fin, fout, "7", "5", "0", path], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert (np.fromfile(fout, np.uint8) == expected).all()
