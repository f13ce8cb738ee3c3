"""The decoder block's frame loop on the device (ldpc_walk_span): one launch
per call, checked against the restated general_work (oracle Block, the loop
of lib/ldpc_decoder_cb_impl.cc:146-226) on the same samples -- output bytes,
items consumed, final state and error count -- for every method, in and
out of sync, at low and high Eb/N0, with short output buffers; and through
the block, against the host-planned path's bytes and printed sync messages."""
import os

import numpy as np
import pytest

import ldpc_ece535a as L
from ldpc_ece535a import flowgraph as fg
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _stream(Hr, frames, ebn0, seed, lead=37, invert_from=None):
    """Encoded random frames with AWGN at ebn0 (rate-1/2 sigma as bench.synth),
    a `lead`-sample noise prefix, the tail negated from frame `invert_from`."""
    import bench
    y, _ = bench.synth(Hr, frames, ebn0, seed)
    y = y.astype(np.float32)
    if invert_from is not None:
        y[invert_from:] *= -1.0
    rng = np.random.default_rng(seed)
    s = np.concatenate([rng.standard_normal(lead).astype(np.float32), y.ravel()])
    return s.astype(np.complex64)


@pytest.fixture(scope="module")
def Hr(golden):
    return golden("frames_default.npz")["H_reordered"]


@pytest.mark.parametrize("method", [0, 1, 2, 3])
@pytest.mark.parametrize("ebn0", [2.0, 4.0])
def test_walk_one_call_matches_loop(Hr, method, ebn0):
    # the restated bit-flip / hard loops are slow on the CPU: shorter streams
    frames = 700 if method <= 1 else 160
    s = _stream(Hr, frames, ebn0, 3 + int(ebn0), invert_from=frames * 4 // 7)
    dec = L.Decoder()
    for iters, state, errors in [(5, 0, 0), (5, 1, 9), (12, 2, 4)]:
        blk = orc.Block(method, Hr, iters)
        blk.s.state, blk.s.errors = state, errors
        exp, used = blk.general_work(1 << 20, s)
        r = dec.walk_span(s.view(np.float32), 1 << 20, method=method, max_iters=iters,
                          elem_stride=2, state=state, errors=errors)
        io = r["io"]
        assert io.consumed == used
        assert r["out"] == exp.tobytes()
        assert (io.state, io.errors) == (blk.state, blk.errors)


@pytest.mark.parametrize("nout_frames", [1, 7, 64, 333])
def test_walk_output_limit(Hr, nout_frames):
    """The loop stops when the output is full (:146-147), mid-search included."""
    s = _stream(Hr, 500, 3.0, 11)
    dec = L.Decoder()
    blk = orc.Block(1, Hr, 5)
    exp, used = blk.general_work(4 * nout_frames, s)
    r = dec.walk_span(s.view(np.float32), 4 * nout_frames, method=1, max_iters=5, elem_stride=2)
    assert r["io"].consumed == used
    assert r["out"] == exp.tobytes()
    assert (r["io"].state, r["io"].errors) == (blk.state, blk.errors)


def test_walk_short_and_empty(Hr):
    dec = L.Decoder()
    for n in [0, 1, 63]:
        r = dec.walk_span(np.zeros(2 * n, np.float32), 64, elem_stride=2)
        assert r["io"].consumed == 0 and r["out"] == b"" and r["msgs"] == []
    # exactly one window, noise: one skip
    x = np.random.default_rng(2).standard_normal(64).astype(np.complex64)
    blk = orc.Block(1, Hr, 5)
    exp, used = blk.general_work(64, x)
    r = dec.walk_span(x.view(np.float32), 64, elem_stride=2)
    assert r["io"].consumed == used and r["out"] == exp.tobytes()


@pytest.mark.parametrize("method", [0, 1])
@pytest.mark.parametrize("chunk", [1000, [97, 13, 640, 5, 2000] * 6])
def test_walk_block_chunked_matches_loop(Hr, method, chunk):
    s = _stream(Hr, 900, 2.5, 5, invert_from=500)
    exp = orc.run_stream(method, Hr, s, iterations=5)  # the loop's output ignores chunking
    os.environ["LDPC_BLOCK_WALK"] = "1"
    try:
        blk = L.ldpc_decoder_cb(method)
    finally:
        os.environ.pop("LDPC_BLOCK_WALK", None)
    tb = fg.top_block(chunk=chunk, out_space=4096)
    src, dst = fg.vector_source_c(s), fg.vector_sink_b()
    tb.connect(src, blk, dst)
    tb.run()
    assert (dst.array() == exp).all()


def test_walk_messages_match_planner(Hr, capfd):
    """Walk and host planner print the same sync messages in the same order."""
    s = _stream(Hr, 800, 2.0, 9, invert_from=300)
    outs, texts = [], []
    for walk in ("1", "0"):
        os.environ["LDPC_BLOCK_WALK"] = walk
        try:
            blk = L.ldpc_decoder_cb(1)
        finally:
            os.environ.pop("LDPC_BLOCK_WALK", None)
        capfd.readouterr()
        tb = fg.top_block(chunk=2048, out_space=4096)
        src, dst = fg.vector_source_c(s), fg.vector_sink_b()
        tb.connect(src, blk, dst)
        tb.run()
        texts.append([l for l in capfd.readouterr().out.splitlines() if "SYNC" in l])
        outs.append(dst.array())
    assert (outs[0] == outs[1]).all()
    assert texts[0] == texts[1]
    assert len(texts[0]) > 3  # the stream does lose and regain sync
