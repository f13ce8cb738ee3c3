"""The frame ring (ldpc_ring_*, csrc/ldpc_ring.hip): one persistent launch
decodes every batch posted to it, frames of all batches from one queue.

Checked here, each through the C ABI (ldpc_ece535a.Decoder.ring_*):
  * 16 384+ frames posted as batches of unequal size -- the second posted
    while the first is being decoded, a later one after the ring has sat
    idle, and one after the launch has ended on its deadline -- equal the
    oracle's decodes (packed bytes, iterations, syndrome weights);
  * every method / precision the ring takes equals ldpc_decode_device on the
    same frames (the same arithmetic);
  * more batches than descriptor slots (slot reuse, the host's wait for the
    oldest batch), and batches of one frame;
  * an input buffer rewritten between two batches of one launch is read
    afresh;
  * signed-zero, +-inf / NaN and extreme finite samples equal the oracle;
  * the reference's other H matrices equal the oracle;
  * the errors of the API."""
import os
import time

import numpy as np
import pytest

import ldpc_ece535a as L

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def frames(Hr, B, db, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    data = rng.integers(0, 2, size=(B, Hr.shape[1] - Hr.shape[0]), dtype=np.uint8)
    x = 2.0 * L.encode(Hr, data) - 1.0
    return (x + np.sqrt(10 ** (-db / 10)) * rng.standard_normal(x.shape)).astype(np.float32)


def outs(dec, B):
    return (torch.zeros((B, dec.KB), dtype=torch.uint8, device="cuda"),
            torch.full((B,), -1, dtype=torch.int32, device="cuda"),
            torch.full((B,), -1, dtype=torch.int32, device="cuda"))


def post(dec, d_y, o, lo=0, hi=None):
    hi = d_y.shape[0] if hi is None else hi
    N = dec.N
    return dec.ring_post(d_y.data_ptr() + 4 * N * lo, hi - lo, o[0].data_ptr() + dec.KB * lo,
                         o[1].data_ptr() + 4 * lo, o[2].data_ptr() + 4 * lo)


def oracle(method, Hr, y, iters=50, et=1):
    from oracle import oracle as orc
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    return orc.decode_batch(method, Hr, y, iters, nthreads=threads, et_period=et)


def test_ring_batches_vs_oracle():
    dec = L.Decoder()
    Hr = dec.H
    sizes = [4096, 4096, 1, 3000, 4096, 1187, 2]
    y = frames(Hr, sum(sizes), 2.0, 606)
    d_y = torch.from_numpy(y).cuda()
    o = outs(dec, y.shape[0])
    torch.cuda.synchronize()
    dec.ring_begin(method=1, max_iters=50)
    cuts = np.cumsum([0] + sizes)
    ids = [post(dec, d_y, o, cuts[0], cuts[1]),
           post(dec, d_y, o, cuts[1], cuts[2])]  # posted while batch 0 is being decoded
    dec.ring_wait(ids[1])
    time.sleep(0.005)  # the ring idles: its waves wait for a post
    for k in range(2, 5):
        ids.append(post(dec, d_y, o, cuts[k], cuts[k + 1]))
    dec.ring_wait(ids[-1])
    time.sleep(0.2)  # past the 50 ms deadline: the launch ends, the next post starts one
    ids.append(post(dec, d_y, o, cuts[5], cuts[6]))
    ids.append(post(dec, d_y, o, cuts[6], cuts[7]))
    for i in ids:
        dec.ring_wait(i)
    info = dec.ring_info()
    dec.ring_end()
    torch.cuda.synchronize()
    assert ids == list(range(ids[0], ids[0] + len(sizes)))
    assert info["launches"] >= 2, info
    ref = oracle(1, Hr, y)
    pk, it, sy = (t.cpu().numpy() for t in o)
    assert (pk == ref["packed"]).all(axis=1).all(), (pk != ref["packed"]).any(axis=1).sum()
    assert (it == ref["iters"]).all()
    assert (sy == ref["synd"]).all()
    dec.close()


@pytest.mark.parametrize("method,prec,et", [(1, 0, 1), (1, 1, 1), (1, 2, 1), (1, 3, 1), (0, 0, 1),
                                            (0, 1, 1), (1, 0, 5)])
def test_ring_equals_decode_device(method, prec, et):
    dec = L.Decoder()
    y = frames(dec.H, 6000, 1.5, 700 + 10 * method + prec)
    d_y = torch.from_numpy(y).cuda()
    B = y.shape[0]
    o = outs(dec, B)
    ref = outs(dec, B)
    dec.decode_device(d_y.data_ptr(), B, ref[0].data_ptr(), method=method, max_iters=50,
                      et_period=et, precision=prec, d_iters=ref[1].data_ptr(),
                      d_synd=ref[2].data_ptr())
    dec.synchronize()
    dec.ring_begin(method=method, max_iters=50, et_period=et, precision=prec)
    last = [post(dec, d_y, o, lo, min(B, lo + 1000)) for lo in range(0, B, 1000)][-1]
    dec.ring_wait(last)
    dec.ring_end()
    torch.cuda.synchronize()
    for a, b in zip(o, ref):
        assert torch.equal(a, b)
    if (method, prec) in ((1, 0), (0, 0)):
        r = oracle(method, dec.H, y, 50, et)
        assert (o[0].cpu().numpy() == r["packed"]).all()
        assert (o[1].cpu().numpy() == r["iters"]).all()
    dec.close()


def test_ring_many_small_batches_reuse_slots():
    """700 batches of 1..7 frames: more than the 256 descriptor slots, so
    slots are reused and posts wait for the oldest batch."""
    dec = L.Decoder()
    rng = np.random.default_rng(5)
    sizes = rng.integers(1, 8, size=700)
    y = frames(dec.H, int(sizes.sum()), 2.0, 77)
    d_y = torch.from_numpy(y).cuda()
    o = outs(dec, y.shape[0])
    torch.cuda.synchronize()
    dec.ring_begin(method=0, max_iters=20)
    cuts = np.cumsum(np.concatenate([[0], sizes]))
    ids = [post(dec, d_y, o, int(cuts[k]), int(cuts[k + 1])) for k in range(len(sizes))]
    dec.ring_wait(ids[-1])
    for i in ids[::37]:
        dec.ring_wait(i)  # long since complete (slot reused): returns at once
    dec.ring_end()
    torch.cuda.synchronize()
    ref = oracle(0, dec.H, y, 20)
    assert (o[0].cpu().numpy() == ref["packed"]).all()
    assert (o[1].cpu().numpy() == ref["iters"]).all()
    assert (o[2].cpu().numpy() == ref["synd"]).all()
    dec.close()


def test_ring_reads_a_rewritten_input_afresh():
    """One input buffer, rewritten by a copy between batches of one launch
    (a receiver reusing its buffers): every batch decodes the data that was
    in the buffer when it was posted."""
    dec = L.Decoder()
    B = 2048
    ys = [frames(dec.H, B, 2.0, 900 + k) for k in range(4)]
    buf = torch.empty((B, dec.N), dtype=torch.float32, device="cuda")
    o = [outs(dec, B) for _ in ys]
    side = torch.cuda.Stream()
    dec.ring_begin(method=1, max_iters=50)
    for y, ok in zip(ys, o):
        with torch.cuda.stream(side):
            buf.copy_(torch.from_numpy(y).pin_memory(), non_blocking=True)
        side.synchronize()
        dec.ring_wait(post(dec, buf, ok))
    dec.ring_end()
    torch.cuda.synchronize()
    for y, ok in zip(ys, o):
        ref = oracle(1, dec.H, y)
        assert (ok[0].cpu().numpy() == ref["packed"]).all()
        assert (ok[1].cpu().numpy() == ref["iters"]).all()
    dec.close()


def test_ring_errors():
    dec = L.Decoder()
    d = torch.zeros((4, dec.N), device="cuda")
    pk = torch.zeros((4, dec.KB), dtype=torch.uint8, device="cuda")
    with pytest.raises(L.LdpcError):  # no session
        dec.ring_post(d.data_ptr(), 4, pk.data_ptr())
    with pytest.raises(L.LdpcError):  # bit-flip: not on the ring
        dec.ring_begin(method=2)
    dec.ring_begin(method=1)
    with pytest.raises(L.LdpcError):  # one session at a time
        dec.ring_begin(method=1)
    with pytest.raises(L.LdpcError):  # B < 1
        dec.ring_post(d.data_ptr(), 0, pk.data_ptr())
    with pytest.raises(L.LdpcError):  # cw_stride < N
        dec.ring_post(d.data_ptr(), 4, pk.data_ptr(), cw_stride=dec.N - 1)
    with pytest.raises(L.LdpcError):  # no such batch
        dec.ring_wait(0)
    i = dec.ring_post(d.data_ptr(), 4, pk.data_ptr())
    dec.ring_wait(i)
    dec.ring_end()
    dec.ring_end()  # (no session: a no-op)
    torch.cuda.synchronize()
    dec.close()


def test_ring_sessions_back_to_back():
    """Consecutive sessions on one context (what bench.py does: a warmup
    session, then the timed one), each batch into outputs of its own: no
    descriptor a previous session left behind is taken for a new batch."""
    dec = L.Decoder()
    B = 1500
    y = frames(dec.H, B, 2.0, 4242)
    d_y = torch.from_numpy(y).cuda()
    ref = oracle(1, dec.H, y)
    for s in range(5):
        o = [outs(dec, B) for _ in range(3)]
        dec.ring_begin(method=1, max_iters=50)
        for ok in o:
            post(dec, d_y, ok)
        dec.ring_end()
        torch.cuda.synchronize()
        for ok in o:
            assert (ok[0].cpu().numpy() == ref["packed"]).all(), s
            assert (ok[1].cpu().numpy() == ref["iters"]).all(), s
    dec.close()


@pytest.mark.parametrize("k", [2, 3, 5])
@pytest.mark.parametrize("method", [0, 1])
def test_ring_other_codes_vs_oracle(k, method):
    """The reference's other H matrices (tests/golden/hData{2,3,5}.alist:
    100 x 50, 16 x 8, 48 x 24): more than one column word (N = 100), and
    packed outputs of 7 / 1 / 3 bytes, which the ring stores byte by byte
    (the default H's 4 go as one 32-bit word)."""
    from ldpc_ece535a import codes
    from oracle import oracle as orc
    M, N, rp, ci = codes.read_alist(os.path.join(os.path.dirname(__file__), "golden",
                                                 "hData%d.alist" % k))
    H = np.zeros((M, N), np.uint8)
    for j in range(M):
        H[j, ci[rp[j]:rp[j + 1]]] = 1
    dec = L.Decoder(H)
    Hr = orc.reorder_h(H)[0]
    assert (dec.H == Hr).all()
    y = frames(Hr, 3000, 2.0, 60 + k)
    d_y = torch.from_numpy(y).cuda()
    o = outs(dec, y.shape[0])
    torch.cuda.synchronize()
    dec.ring_begin(method=method, max_iters=50)
    ids = [post(dec, d_y, o, lo, min(3000, lo + 1100)) for lo in range(0, 3000, 1100)]
    dec.ring_wait(ids[-1])
    dec.ring_end()
    torch.cuda.synchronize()
    ref = oracle(method, Hr, y)
    assert (o[0].cpu().numpy() == ref["packed"]).all()
    assert (o[1].cpu().numpy() == ref["iters"]).all()
    assert (o[2].cpu().numpy() == ref["synd"]).all()
    dec.close()


@pytest.mark.parametrize("method", [0, 1])
def test_ring_special_samples_vs_oracle(golden, method):
    """The headline path on the samples the batch kernels' special-value tests
    use: exact +0.0 / -0.0 samples (every kind of frame the signed-zero test
    builds), +-inf / NaN samples (the select-based sum-product loop), and
    finite amplitudes from 1e-40 to 1e30 (tanh saturating to +-1 inside
    all-finite frames), posted as three batches of one session: bytes,
    iterations and syndrome weights equal the oracle's."""
    from oracle import oracle as orc
    fd = golden("frames_default.npz")
    rng = np.random.default_rng(2606)
    base = np.concatenate([fd["db%d_llr" % db] for db in (0, 2, 4)]).astype(np.float32)
    z = base.copy()
    hit = rng.random(z.shape) < 0.25
    sign = rng.random(z.shape) < 0.5
    z[hit & sign] = 0.0
    z[hit & ~sign] = -0.0
    z[0] = 0.0
    z[1] = -0.0
    nf = fd["db2_llr"].astype(np.float32).copy()
    for b in range(0, nf.shape[0], 3):
        for _ in range(1 + b % 3):
            nf[b, rng.integers(0, 64)] = rng.choice([np.inf, -np.inf, np.nan])
    big = fd["db2_llr"].astype(np.float64)
    ex = np.concatenate([big[:48] * a for a in (8.0, 1e3, 1e30, 1e-30, 1e-40)]).astype(np.float32)
    y = np.ascontiguousarray(np.concatenate([z, nf, ex]))
    dec = L.Decoder()
    d_y = torch.from_numpy(y).cuda()
    o = outs(dec, y.shape[0])
    torch.cuda.synchronize()
    dec.ring_begin(method=method, max_iters=30)
    cuts = [0, z.shape[0], z.shape[0] + nf.shape[0], y.shape[0]]
    ids = [post(dec, d_y, o, cuts[k], cuts[k + 1]) for k in range(3)]
    dec.ring_wait(ids[-1])
    dec.ring_end()
    torch.cuda.synchronize()
    ref = orc.decode_batch(method, dec.H, y, 30)
    pk, it, sy = (t.cpu().numpy() for t in o)
    assert (pk == ref["packed"]).all(axis=1).all(), np.flatnonzero((pk != ref["packed"]).any(axis=1))[:8]
    np.testing.assert_array_equal(it, ref["iters"])
    np.testing.assert_array_equal(sy, ref["synd"])
    dec.close()
