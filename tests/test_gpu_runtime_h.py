"""Runtime H on the GPU and the block's new paths.

* A code loaded from an alist file decodes exactly as the oracle decodes the
  same (reordered) H, every method.
* The block built with a runtime H -- from an alist file, a dense H, or the
  default H forced onto the large-code kernels -- turns noisy streams
  (misaligned start, polarity flip, garbage between frames) into the bytes
  of the restated general_work (oracle/ orc_block) on that H.
* ldpc_decode_strided_both (both polarities in one launch, the block's
  OUT_OF_SYNC search) equals two single-polarity decodes.
* The C++ caller of the public factory make(method) (tests/native/
  block_make_test.cc) driving general_work through the gr::block interface
  reproduces the restated general_work."""
import os
import subprocess

import numpy as np
import pytest

import ldpc_ece535a as L
from ldpc_ece535a import codes
from ldpc_ece535a import flowgraph as fg

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")


def _noisy_frames(Hr, B, db, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    K = Hr.shape[1] - Hr.shape[0]
    x = 2.0 * L.encode(Hr, rng.integers(0, 2, size=(B, K), dtype=np.uint8)) - 1.0
    return (x + np.sqrt(10 ** (-db / 10)) * rng.standard_normal(x.shape)).astype(np.float32)


def _stream(Hr, seed):
    """Garbage, frames, garbage, negated frames: exercises sync search,
    polarity inversion and re-sync."""
    rng = np.random.default_rng(seed)
    N = Hr.shape[1]
    x = _noisy_frames(Hr, 60, 5.0, seed)
    s = np.concatenate([rng.standard_normal(N // 2 + 3).astype(np.float32), x[:30].ravel(),
                        rng.standard_normal(N * 14).astype(np.float32), -x[30:].ravel()])
    return s.astype(np.complex64)


@pytest.mark.parametrize("k", [2, 3, 5])
@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_alist_code_decode_parity(k, method):
    from oracle import oracle as orc
    M, N, rp, ci = codes.read_alist(os.path.join(GOLDEN, "hData%d.alist" % k))
    H = np.zeros((M, N), np.uint8)
    for j in range(M):
        H[j, ci[rp[j]:rp[j + 1]]] = 1
    dec = L.Decoder(H)  # reordered as the reference's constructor does
    Hr, _, _, _ = orc.reorder_h(H)
    assert (dec.H == Hr).all()
    y = _noisy_frames(Hr, 512, 2.0, 40 + k)
    out = dec.decode(y, method=method, max_iters=50)
    ref = orc.decode_batch(method, Hr, y, 50, nthreads=8)
    for key in ("bits", "packed", "iters", "synd"):
        assert (out[key] == ref[key]).all(), key


@pytest.mark.parametrize("how", ["alist2", "alist5", "dense5", "graph_default"])
@pytest.mark.parametrize("method", [0, 1])
def test_block_runtime_h_stream(how, method):
    from oracle import oracle as orc
    if how.startswith("alist"):
        path = os.path.join(GOLDEN, "hData%s.alist" % how[-1])
        blk = L.ldpc_decoder_cb(method, iterations=20, alist=path)
        M, N, rp, ci = codes.read_alist(path)
        H = np.zeros((M, N), np.uint8)
        for j in range(M):
            H[j, ci[rp[j]:rp[j + 1]]] = 1
    elif how == "dense5":
        H = np.load(os.path.join(GOLDEN, "reference_data.npz"))["hData5"]
        blk = L.ldpc_decoder_cb(method, iterations=20, H=H)
    else:  # the default H on the large-code (HBM message) kernels: LDPC_FLAG_GRAPH
        H = L.default_h()
        blk = _graph_block(method, H)
    Hr, _, _, _ = orc.reorder_h(H)
    assert (blk.M, blk.N, blk.frame_bytes) == (Hr.shape[0], Hr.shape[1], Hr.shape[0] // 8)
    s = _stream(Hr, 11 + method)
    exp = orc.run_stream(method, Hr, s, iterations=20)
    tb = fg.top_block(chunk=[301, 17, 1200, 64, 999] * 6, out_space=97)
    src, dst = fg.vector_source_c(s), fg.vector_sink_b()
    tb.connect(src, blk, dst)
    tb.run()
    assert len(exp) > 0
    assert (dst.array() == exp).all()


def _graph_block(method, H):
    import ctypes
    from ldpc_ece535a import blocks
    H = np.ascontiguousarray(H, np.uint8)
    b = L.ldpc_decoder_cb.__new__(L.ldpc_decoder_cb)
    b._backend = None
    b._h = blocks.lib().ldpc_decoder_cb_make_h(method, 20, 0, 0, H.ctypes.data_as(blocks._u8p),
                                               H.shape[0], H.shape[1], 2)  # LDPC_FLAG_GRAPH
    assert b._h, blocks._err()
    b.method = method
    m, n, k = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int32(0)
    blocks.lib().ldpc_decoder_cb_frame_shape(b._h, ctypes.byref(m), ctypes.byref(n),
                                             ctypes.byref(k))
    b.M, b.N, b.frame_bytes = m.value, n.value, k.value
    return b


def test_block_rejects_short_information_part():
    H = np.zeros((16, 20), np.uint8)  # K = 4 < 8 (M/8) = 16
    for j in range(16):
        H[j, j] = 1
        H[j, 16 + j % 4] = 1
    with pytest.raises(L.LdpcError):
        L.ldpc_decoder_cb(1, H=H, reorder=False)


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_decode_strided_both(graph, method):
    dec = L.Decoder(force_graph=graph)
    y = _noisy_frames(dec.H, 300, 1.0, 77)
    z = np.zeros(2 * y.size, np.float32)
    z[0::2] = y.ravel()
    B = 200
    both = dec.decode_both(z, method=method, max_iters=30, cw_stride=2, elem_stride=2, B=B)
    for half, pol in ((0, 1.0), (1, -1.0)):
        one = dec.decode(z, method=method, max_iters=30, polarity=pol, cw_stride=2,
                         elem_stride=2, B=B)
        assert (both["packed"][half * B:(half + 1) * B] == one["packed"]).all()
        assert (both["synd"][half * B:(half + 1) * B] == one["synd"]).all()


@pytest.mark.parametrize("method", [0, 1, 2, 3])
def test_native_make_caller(tmp_path, golden, method):
    """ldpc_decoder_cb::make(method) from C++ through the gr::block interface."""
    from oracle import oracle as orc
    exe = os.path.join(REPO, "gr-ldpc_ece535a_amd", "lib", "block_make_test")
    assert os.path.exists(exe), "build first: make -C gr-ldpc_ece535a_amd native"
    st = golden("streams.npz")
    Hr = golden("frames_default.npz")["H_reordered"]
    for name in ("offset", "inverted", "burst"):
        s = np.asarray(st[name + "_in"], np.complex64)
        fin, fout = str(tmp_path / "in.f32"), str(tmp_path / "out.u8")
        s.view(np.float32).tofile(fin)
        r = subprocess.run([exe, str(method), fin, fout, "777"], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr
        got = np.fromfile(fout, np.uint8)
        assert (got == st["%s_m%d_out" % (name, method)]).all(), name
        assert (got == orc.run_stream(method, Hr, s, iterations=5)).all(), name


def test_native_make_caller_alist(tmp_path):
    """make(method, iterations, precision, alist_path) from C++."""
    from oracle import oracle as orc
    exe = os.path.join(REPO, "gr-ldpc_ece535a_amd", "lib", "block_make_test")
    path = os.path.join(GOLDEN, "hData5.alist")
    M, N, rp, ci = codes.read_alist(path)
    H = np.zeros((M, N), np.uint8)
    for j in range(M):
        H[j, ci[rp[j]:rp[j + 1]]] = 1
    Hr, _, _, _ = orc.reorder_h(H)
    s = _stream(Hr, 5)
    fin, fout = str(tmp_path / "in.f32"), str(tmp_path / "out.u8")
    s.view(np.float32).tofile(fin)
    r = subprocess.run([exe, "1", fin, fout, "500", "20", "0", path], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert (np.fromfile(fout, np.uint8) == orc.run_stream(1, Hr, s, iterations=20)).all()


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("method", [0, 1])
def test_decode_windows_any_positions(graph, method):
    """ldpc_decode_windows (the block's launches): windows at arbitrary sample
    positions of one interleaved gr_complex span, either polarity, equal the
    strided single-window decodes of the same samples; a reused span gives
    the same results."""
    dec = L.Decoder(force_graph=graph)
    N = dec.N
    rng = np.random.default_rng(9)
    x = _noisy_frames(dec.H, 24, 2.0, 77).ravel()
    span = np.concatenate([rng.standard_normal(37).astype(np.float32), x])
    cx = np.zeros(2 * span.size, np.float32)
    cx[0::2] = span
    cx[1::2] = rng.standard_normal(span.size)  # imaginary parts are ignored
    pos = np.concatenate([37 + N * np.arange(20), rng.integers(0, span.size - N, 40)])
    neg = rng.integers(0, 2, pos.size)
    win = (pos.astype(np.int64) << 1) | neg
    out = dec.decode_windows(cx, win, method=method, max_iters=20, elem_stride=2)
    again = dec.decode_windows(cx, win[::-1].copy(), method=method, max_iters=20, elem_stride=2,
                               reuse_span=True)
    for b, (p, n) in enumerate(zip(pos, neg)):
        ref = dec.decode(span[p:p + N], method=method, max_iters=20, polarity=-1.0 if n else 1.0)
        assert (out["packed"][b] == ref["packed"][0]).all(), b
        assert out["synd"][b] == ref["synd"][0], b
    assert (again["packed"][::-1] == out["packed"]).all()
    assert (again["synd"][::-1] == out["synd"]).all()
    # a span staged ahead (ldpc_stage_span, the block's first step) serves
    # the launches that reuse it; a host-buffer decode in between waits for
    # its copy before touching the pinned stage
    other = dec.decode(span[37:37 + 4 * N], method=method, max_iters=20)
    dec.stage_span(cx, elem_stride=2, max_windows=win.size)
    mid = dec.decode(span[37:37 + 4 * N], method=method, max_iters=20)
    assert (mid["packed"] == other["packed"]).all()
    dec.stage_span(cx, elem_stride=2, max_windows=win.size)
    pre = dec.decode_windows(cx, win, method=method, max_iters=20, elem_stride=2,
                             reuse_span=True)
    assert (pre["packed"] == out["packed"]).all() and (pre["synd"] == out["synd"]).all()


def test_decode_windows_rejects_out_of_span():
    dec = L.Decoder()
    cx = np.zeros(2 * 100, np.float32)
    with pytest.raises(L.LdpcError):
        dec.decode_windows(cx, np.array([(40 << 1)], np.int64), elem_stride=2)  # 40 + 64 > 100


def _ira_code():
    """A quasi-cyclic IRA code of the config-4 family at N = 720 (the
    large-code kernels: N > 256), [parity | info] as the block emits it."""
    t = codes.dvbs2_like_table(3, K=360, N=720, hi_groups=1, hi_deg=6, lo_deg=3)
    return codes.ira_from_table(t, 360, 720)


@pytest.mark.parametrize("method,ebn0,garbage", [(0, 2.0, True), (1, 4.0, False)])
def test_block_large_csr_stream(method, ebn0, garbage):
    """The block on a large runtime H given as CSR (the min-sum frame pipeline
    / the sum-product graph passes, window limits sized by N): a misaligned
    start, frames, [3 frames of noise then frames off the old grid: 11
    errors, a sync loss and an N-position search,] a polarity flip -- the
    bytes of the restated general_work decoding every window with the sparse
    restatement (orc_block_general_work_sparse)."""
    from oracle import oracle as orc
    csr = _ira_code()
    M, N, rp, ci = csr
    rng = np.random.default_rng(40 + method)
    x = 2.0 * codes.ira_encode(csr, rng.integers(0, 2, size=(36, N - M), dtype=np.uint8)) - 1.0
    x = (x + np.sqrt(10 ** (-ebn0 / 10)) * rng.standard_normal(x.shape)).astype(np.float32)
    parts = [rng.standard_normal(5).astype(np.float32), x[:18].ravel()]
    if garbage:
        parts.append(rng.standard_normal(3 * N + 5).astype(np.float32))
    parts.append(-x[18:].ravel())
    s = np.concatenate(parts).astype(np.complex64)
    exp = orc.run_stream(method, None, s, iterations=5, csr=csr)
    assert len(exp) >= 10 * (M // 8)
    blk = L.ldpc_decoder_cb(method, iterations=5, csr=csr)
    assert (blk.M, blk.N) == (M, N)
    tb = fg.top_block(chunk=[N * 7 + 3, 999, N * 20] * 4, out_space=M // 8 * 5)
    src, dst = fg.vector_source_c(s), fg.vector_sink_b()
    tb.connect(src, blk, dst)
    tb.run()
    assert (dst.array() == exp).all()
