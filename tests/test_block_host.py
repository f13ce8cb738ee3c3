"""Host logic of the decoder block (batched windows, replayed frame-sync
state machine, polarity retry, packing) driven on the CPU through the
block's test seam, with the oracle as the frame decoder.  The expected
streams come from the restated general_work (oracle/, tests/golden).

The product path never takes this seam: ldpc_decoder_cb(method) always
decodes on the GPU (tests/test_gpu_block.py runs the same streams there)."""
import numpy as np
import pytest

import ldpc_ece535a as L
from ldpc_ece535a import flowgraph as fg
from oracle import oracle as orc


def oracle_backend(method, Hr, iterations=5):
    Hr = np.ascontiguousarray(Hr, np.uint8)

    def fn(user, inp, n_floats, cw_stride, elem_stride, polarity, B, packed, synd):
        x = np.ctypeslib.as_array(inp, shape=(int(n_floats),))
        r = orc.decode_batch(method, Hr, x, iterations, polarity=polarity, cw_stride=cw_stride,
                             elem_stride=elem_stride, B=B)
        np.ctypeslib.as_array(packed, shape=(B * r["packed"].shape[1],))[:] = r["packed"].ravel()
        np.ctypeslib.as_array(synd, shape=(B,))[:] = r["synd"]
        return 0
    return fn


@pytest.fixture(scope="module")
def Hr(golden):
    return golden("frames_default.npz")["H_reordered"]


@pytest.mark.parametrize("name", ["aligned", "offset", "inverted", "burst", "noisy"])
@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_block_streams_match_restated_general_work(golden, Hr, name, method):
    st = golden("streams.npz")
    s = st[name + "_in"]
    blk = L.ldpc_decoder_cb(method, _backend=oracle_backend(method, Hr))
    tb = fg.top_block()
    src, dst = fg.vector_source_c(s), fg.vector_sink_b()
    tb.connect((src, 0), (blk, 0))
    tb.connect((blk, 0), (dst, 0))
    tb.run()
    assert (dst.array() == st["%s_m%d_out" % (name, method)]).all()


@pytest.mark.parametrize("chunk,out_space", [(7, 4), (64, 8), (100, 1000), (333, 12)])
def test_block_chunking_and_output_space(golden, Hr, chunk, out_space):
    st = golden("streams.npz")
    s = st["burst_in"]
    blk = L.ldpc_decoder_cb(1, _backend=oracle_backend(1, Hr))
    tb = fg.top_block(chunk=chunk, out_space=out_space)
    src, dst = fg.vector_source_c(s), fg.vector_sink_b()
    tb.connect(src, blk, dst)
    tb.run()
    assert (dst.array() == st["burst_m1_out"]).all()


def test_forecast(Hr):
    blk = L.ldpc_decoder_cb(1, _backend=oracle_backend(1, Hr))
    assert blk.forecast(4) == 256  # noutput * N (:126-130)
    assert L.ldpc_encoder_bc().forecast(64) == 4  # ceil(64/16) (:112-116)


def test_state_machine_inverted_quirk(Hr):
    """Out of sync while INVERTED, the '-tx' retry decodes the un-inverted
    samples yet sets INVERTED again (:150-152 with :180-191)."""
    rng = np.random.default_rng(5)
    data = rng.integers(0, 2, size=(30, 32), dtype=np.uint8)
    cw = L.encode(Hr, data)
    x = (2.0 * cw - 1.0).astype(np.float32)
    frames = np.concatenate([-x[:10], rng.standard_normal((12, 64)).astype(np.float32), x[10:]])
    s = frames.reshape(-1).astype(np.complex64)
    exp = orc.run_stream(1, Hr, s, iterations=5)
    blk = L.ldpc_decoder_cb(1, _backend=oracle_backend(1, Hr))
    out, used = blk.general_work(10 ** 6, s)
    assert (out == exp).all()
    ob = orc.Block(1, Hr, 5)
    ob.general_work(10 ** 6, s)
    assert blk.state == ob.state and blk.errors == ob.errors


def test_encoder_block_roundtrip(Hr):
    rng = np.random.default_rng(9)
    payload = rng.integers(0, 256, 40, dtype=np.uint8)
    enc = L.ldpc_encoder_bc()
    tb = fg.top_block(chunk=3, out_space=200)
    src, dst = fg.vector_source_b(payload), fg.vector_sink_c()
    tb.connect(src, enc, dst)
    tb.run()
    sym = dst.array()
    assert len(sym) == 40 // 4 * 64 and (sym.imag == 0).all()
    bits = (sym.real.reshape(-1, 64) > 0).astype(np.uint8)
    assert not ((Hr.astype(int) @ bits.T.astype(int)) % 2).any()
    assert (np.packbits(bits[:, 32:].reshape(-1)) == payload).all()
    # noiseless frames decode back through the (oracle-backed) block
    blk = L.ldpc_decoder_cb(1, _backend=oracle_backend(1, Hr))
    out, _ = blk.general_work(10 ** 6, sym)
    assert (out == payload).all()


def _hard_stream(Hr, seed, frames=32, db=1.0):
    """Low-SNR frames (sync losses every few frames), a polarity flip, a
    misaligned garbage stretch and frames again: exercises every branch of
    the replayed state machine and the speculative search windows."""
    rng = np.random.default_rng(seed)
    M, N = Hr.shape
    data = rng.integers(0, 2, size=(frames, N - M), dtype=np.uint8)
    x = 2.0 * L.encode(Hr, data) - 1.0
    y = x + np.sqrt(10 ** (-db / 10)) * rng.standard_normal(x.shape)
    half = frames // 2
    s = np.concatenate([rng.standard_normal(17), y[:half].ravel(), rng.standard_normal(N + 29),
                        -y[half:].ravel()]).astype(np.float32)
    return s.astype(np.complex64)


@pytest.mark.parametrize("method,iters", [(0, 5), (1, 5), (1, 20), (2, 5), (3, 1)])
@pytest.mark.parametrize("chunk,out_space", [(None, 1 << 20), (200, 12), (777, 1 << 20)])
def test_block_low_snr_streams_match_restated_general_work(Hr, method, iters, chunk, out_space):
    s = _hard_stream(Hr, 100 + method * 7 + iters, db=1.0 if method <= 1 else 3.0)
    exp = orc.run_stream(method, Hr, s, iterations=iters,
                         chunks=None if chunk is None else [chunk] * (len(s) // chunk + 1),
                         out_space=out_space)
    blk = L.ldpc_decoder_cb(method, iterations=iters, _backend=oracle_backend(method, Hr, iters))
    tb = fg.top_block(chunk=chunk, out_space=out_space)
    src, dst = fg.vector_source_c(s), fg.vector_sink_b()
    tb.connect(src, blk, dst)
    tb.run()
    assert len(exp) > 0
    assert (dst.array() == exp).all()


@pytest.mark.parametrize("ebn0", [1.0, 3.0])
def test_plans_exact_and_windows_bounded(Hr, ebn0, monkeypatch):
    """The dry run's plan (ldpc_decoder_cb_impl.cc header; the A/B knobs
    LDPC_BLOCK_MAXWANT and LDPC_BLOCK_SEARCHES) changes only which windows
    are decoded, never the stream: every plan gives the restated
    general_work's output, and the default plan's grid guesses decode at most
    a few times the reference loop's own decodes."""
    import bench
    y, _ = bench.synth(Hr, 192, ebn0, 31)
    x = np.zeros(2 * y.size, np.float32)
    x[0::2] = y.ravel()
    s = x.view(np.complex64)
    stats = {}
    exp = orc.run_stream(1, Hr, s, iterations=5, chunks=[64 * 48] * 4, stats=stats)
    plans = {"default": {}, "maxwant64": {"LDPC_BLOCK_MAXWANT": "64"},
             "searches1": {"LDPC_BLOCK_SEARCHES": "1"}, "whole": {"LDPC_BLOCK_MAXWANT": "-1",
                                                                 "LDPC_BLOCK_SEARCHES": "0"}}
    decoded = {}
    for plan, env in plans.items():
        for k in ("LDPC_BLOCK_MAXWANT", "LDPC_BLOCK_SEARCHES"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        blk = L.ldpc_decoder_cb(1, _backend=oracle_backend(1, Hr))
        tb = fg.top_block(chunk=64 * 48, out_space=4 * 48)
        src, dst = fg.vector_source_c(s), fg.vector_sink_b()
        tb.connect(src, blk, dst)
        tb.run()
        assert (dst.array() == exp).all(), plan
        decoded[plan] = blk.frames_decoded
    assert decoded["default"] <= 16 * stats["decodes"], (decoded, stats["decodes"])
