"""The decoder block on the GPU: the golden streams (misaligned start,
inverted polarity, burst -> resync, noisy) decode to the restated
general_work's bytes for every method, under irregular chunking; and the
reference's QA test (python/qa_ldpc_decoder_cb.py), done with the default H:
encoder block -> decoder block recovers the 8 KAT bytes."""
import numpy as np
import pytest

import ldpc_ece535a as L
from ldpc_ece535a import flowgraph as fg

pytestmark = pytest.mark.gpu


PATHS = {"serve": {}, "launch": {"LDPC_BLOCK_SERVE": "0"},
         # the planner's A/B knobs: short dry runs, one search per round
         "plan": {"LDPC_BLOCK_MAXWANT": "64", "LDPC_BLOCK_SEARCHES": "1"},
         # every diagnostic knob on: stderr lines only, the same bytes
         "diag": {"LDPC_BLOCK_DEBUG": "2", "LDPC_BLOCK_PROFILE": "2",
                  "LDPC_SERVE_DEBUG": "1"}}


def _block(method, path, **kw):
    """The block with its small rounds through the window server and big ones
    by launch (default), a launch per round (LDPC_BLOCK_SERVE=0), another
    dry-run plan, or every diagnostic on."""
    import os
    env = PATHS[path]
    os.environ.update(env)
    try:
        return L.ldpc_decoder_cb(method, **kw)
    finally:
        for k in env:
            os.environ.pop(k, None)


@pytest.mark.parametrize("path", sorted(PATHS))
@pytest.mark.parametrize("name", ["aligned", "offset", "inverted", "burst", "noisy"])
@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_gpu_block_streams(golden, name, method, path):
    st = golden("streams.npz")
    s = st[name + "_in"]
    blk = _block(method, path)
    tb = fg.top_block(chunk=[97, 13, 640, 5, 2000] * 4)
    src, dst = fg.vector_source_c(s), fg.vector_sink_b()
    tb.connect((src, 0), (blk, 0))
    tb.connect((blk, 0), (dst, 0))
    tb.run()
    assert (dst.array() == st["%s_m%d_out" % (name, method)]).all()


@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_qa_loopback_default_h(method):
    data = (0b11101101, 0b00000010, 0b00110100, 0b10000000,
            0b01010011, 0b00000110, 0b00110001, 0b11101000)
    tb = fg.top_block()
    src = fg.vector_source_b(data)
    enc = L.ldpc_encoder_bc()
    dec = L.ldpc_decoder_cb(method)
    dst = fg.vector_sink_b()
    tb.connect((src, 0), (enc, 0))
    tb.connect((enc, 0), (dec, 0))
    tb.connect((dec, 0), (dst, 0))
    tb.run()
    assert dst.data() == data
    assert dec.state == L.STATE_IN_SYNC


@pytest.mark.parametrize("iters", [5, 50])
@pytest.mark.parametrize("path", sorted(PATHS))
def test_gpu_block_long_random_stream(golden, path, iters):
    """A longer mixed stream: results equal the restated general_work.  At
    50 iterations the default path decodes its first, big rounds by launch
    and the small ones after them through the window server."""
    import sys
    from oracle import oracle as orc
    Hr = golden("frames_default.npz")["H_reordered"]
    rng = np.random.default_rng(21)
    data = rng.integers(0, 2, size=(300, 32), dtype=np.uint8)
    x = (2.0 * L.encode(Hr, data) - 1.0).astype(np.float32)
    x = x + 0.6 * rng.standard_normal(x.shape).astype(np.float32)
    s = np.concatenate([rng.standard_normal(29).astype(np.float32), x[:150].ravel(),
                        rng.standard_normal(64 * 13).astype(np.float32), -x[150:].ravel()])
    s = s.astype(np.complex64)
    exp = orc.run_stream(1, Hr, s, iterations=iters)
    blk = _block(1, path, iterations=iters)
    tb = fg.top_block(chunk=[1000, 20000] if iters == 50 else 1000,
                      out_space=4096 if iters == 50 else 64)
    src, dst = fg.vector_source_c(s), fg.vector_sink_b()
    tb.connect(src, blk, dst)
    tb.run()
    assert (dst.array() == exp).all()


@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_dump_app_roundtrip(method):
    """apps/ldpc_ece535a_dump's flowgraph (random ASCII -> encoder ->
    decoder -> sink) on this package's blocks: noiseless text comes back
    unchanged with every method; SURVEY config 1 is --chars 4 --iterations 10."""
    import io
    from ldpc_ece535a import dump
    out = io.StringIO()
    sent, got = dump.run(chars=64, method=method, iterations=10, seed=5, stream=out)
    assert bytes(got) == bytes(sent)
    assert out.getvalue() == bytes(sent).decode()


def test_dump_app_noisy_sum_product():
    from ldpc_ece535a import dump
    sent, got = dump.run(chars=400, method=1, iterations=50, ebn0=6.0, seed=9,
                         stream=open("/dev/null", "w"))
    assert len(got) == len(sent)
    assert (got != sent).mean() < 0.02


def _zero_region_stream(Hr, seed):
    """Frames, a region of exact zeros (not a whole number of frames), frames
    again, negative zeros, negated frames.  What a window of +-0 samples
    decodes to (all-zero or all-one bytes, a sync loss or not) is decided by
    each method's sign rule at exactly zero (lib/ldpc_decoder_cb_impl.cc
    :398, :426, :527, :564); the bytes must be the restated
    general_work's, including the resynchronisation after the region."""
    rng = np.random.default_rng(seed)
    x = (2.0 * L.encode(Hr, rng.integers(0, 2, size=(90, 32), dtype=np.uint8)) - 1.0)
    x = (x + 0.7 * rng.standard_normal(x.shape)).astype(np.float32)
    z = np.zeros(64 * 9 + 23, np.float32)
    s = np.concatenate([rng.standard_normal(11).astype(np.float32), x[:30].ravel(), z,
                        x[30:60].ravel(), -z, np.zeros(5, np.float32), -x[60:].ravel()])
    return s.astype(np.complex64)


@pytest.mark.parametrize("path", ["serve", "launch"])
@pytest.mark.parametrize("method,iters", [(0, 5), (1, 5), (1, 50), (2, 5), (3, 5)])
def test_gpu_block_zero_filled_region(golden, method, iters, path):
    from oracle import oracle as orc
    Hr = golden("frames_default.npz")["H_reordered"]
    s = _zero_region_stream(Hr, 31 + method)
    exp = orc.run_stream(method, Hr, s, iterations=iters)
    assert len(exp) > 0
    for chunk in ([97, 13, 640, 5, 2000] * 8, 100000):
        blk = _block(method, path, iterations=iters)
        tb = fg.top_block(chunk=chunk, out_space=61)
        src, dst = fg.vector_source_c(s), fg.vector_sink_b()
        tb.connect(src, blk, dst)
        tb.run()
        assert (dst.array() == exp).all(), chunk
