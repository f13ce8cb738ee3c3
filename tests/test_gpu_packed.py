"""GPU parity of the packed sum-product kernel (decode_packed_kernel: F frames
per wave, ldpc_kernels.hip), which throughput mode (ldpc_set_launch_mode 1)
uses for sum-product f64 on codes it takes (the reference's default H: 3
frames x 168 edges in 512 cells) when a context is created with
LDPC_PACKED=1 (opt-in: exact, not yet faster).  Every output -- packed bytes,
bits, iteration counts, syndromes, posteriors' bits -- must equal the oracle's
and the one-frame-per-wave kernel's: frames finish at different iterations,
so slots refill mid-launch; batches that leave slots empty; frames with
non-finite samples (the select form) mixed with finite ones; both
polarities; strided inputs."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def decs():
    import ldpc_ece535a as L
    os.environ["LDPC_PACKED"] = "1"  # opt-in (read when a context is created)
    try:
        tp = L.Decoder()
    finally:
        del os.environ["LDPC_PACKED"]
    tp.set_launch_mode(1)  # throughput: the packed kernel
    lat = L.Decoder()      # latency (default): one frame per wave
    assert tp.packed_frames_per_wave() == 3 and lat.packed_frames_per_wave() == 0
    return tp, lat


def _same_post(a, b):
    return ((a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))).all()


@pytest.mark.parametrize("iters", [1, 5, 50])
@pytest.mark.parametrize("db", [0, 2, 4])
def test_fixtures(decs, golden, db, iters):
    tp, _ = decs
    sys.path.insert(0, REPO)
    from oracle import oracle as orc
    fd = golden("frames_default.npz")
    y = fd["db%d_llr" % db]
    out = tp.decode(y, method=1, max_iters=iters, want_llr=True)
    ref = orc.decode_batch(1, tp.H, y, iters, nthreads=8, want_post=True)
    for k in ("packed", "bits", "iters", "synd"):
        np.testing.assert_array_equal(out[k], ref[k], err_msg=k)
    assert _same_post(out["llr"], ref["post"])


@pytest.mark.parametrize("B", [1, 2, 3, 4, 7, 100, 3073, 20000])
def test_batch_sizes_vs_one_frame_kernel(decs, B):
    """Slots left empty (B < 3 per wave), refills, and a launch with more
    frames than resident slots: identical to the one-frame kernel."""
    import bench
    tp, lat = decs
    y, _ = bench.synth(tp.H, B, 1.5, 300 + B)
    a = tp.decode(y, method=1, max_iters=50, want_llr=True)
    b = lat.decode(y, method=1, max_iters=50, want_llr=True)
    for k in ("packed", "bits", "iters", "synd"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert _same_post(a["llr"], b["llr"])


def test_large_batch_vs_oracle(decs):
    import bench
    tp, _ = decs
    from oracle import oracle as orc
    y, _ = bench.synth(tp.H, 16384, 2.0, 4242)
    out = tp.decode(y, method=1, max_iters=50, et_period=1)
    ref = orc.decode_batch(1, tp.H, y, 50, nthreads=16)
    for k in ("packed", "iters", "synd"):
        np.testing.assert_array_equal(out[k], ref[k], err_msg=k)
    out5 = tp.decode(y[:4096], method=1, max_iters=50, et_period=5)
    ref5 = orc.decode_batch(1, tp.H, y[:4096], 50, nthreads=16, et_period=5)
    for k in ("packed", "iters", "synd"):
        np.testing.assert_array_equal(out5[k], ref5[k], err_msg=k)


def test_non_finite_frames_mixed(decs):
    """Frames with inf / NaN samples take the select form; they share waves
    with finite frames, which must not change."""
    import bench
    tp, _ = decs
    from oracle import oracle as orc
    y, _ = bench.synth(tp.H, 600, 1.0, 77)
    y[5, 3] = np.inf
    y[17, 0] = -np.inf
    y[30, 10] = np.nan
    y[31, :] = np.inf
    y[200, 63] = np.nan
    out = tp.decode(y, method=1, max_iters=30, want_llr=True)
    ref = orc.decode_batch(1, tp.H, y, 30, nthreads=8, want_post=True)
    for k in ("packed", "bits", "iters", "synd"):
        np.testing.assert_array_equal(out[k], ref[k], err_msg=k)
    assert _same_post(out["llr"], ref["post"])


def test_both_polarities_and_strides(decs):
    import bench
    tp, lat = decs
    y, _ = bench.synth(tp.H, 999, 2.0, 5)
    a = tp.decode_both(y, method=1, max_iters=50)
    b = lat.decode_both(y, method=1, max_iters=50)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    # gr_complex-style interleaved input (elem_stride 2) with a row stride
    z = np.zeros((999, 2 * 64 + 6), np.float32)
    z[:, 0:128:2] = y
    c = tp.decode(z, method=1, max_iters=50, cw_stride=z.shape[1], elem_stride=2, B=999)
    d = lat.decode(y, method=1, max_iters=50)
    for k in ("packed", "iters", "synd"):
        np.testing.assert_array_equal(c[k], d[k], err_msg=k)
