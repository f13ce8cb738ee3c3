"""GPU parity on frames holding exact +0.0 / -0.0 samples (a sample of 0.0
makes r = -tx = -0.0, :486 / :318-321): the small-code kernels' column sums
start at their first term instead of a 0.0 seed (csrc/ldpc_kernels.hip,
FIN path), which is the same value only because no term is ever -0.0.  These
frames put signed zeros into every position the argument covers, against the
live oracle (the C restatement of lib/ldpc_decoder_cb_impl.cc:309-557)."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _frames(golden):
    fd = golden("frames_default.npz")
    rng = np.random.default_rng(535)
    base = np.concatenate([fd["db%d_llr" % db] for db in (0, 2, 4)]).astype(np.float32)
    y = np.tile(base, (2, 1))
    # 0: 25 % of samples +0.0, 1: 25 % -0.0, 2: both kinds, 3: untouched
    kind = np.arange(y.shape[0]) % 4
    hit = rng.random(y.shape) < 0.25
    y[(kind == 0)[:, None] & hit] = 0.0
    y[(kind == 1)[:, None] & hit] = -0.0
    sign = rng.random(y.shape) < 0.5
    y[(kind == 2)[:, None] & hit & sign] = 0.0
    y[(kind == 2)[:, None] & hit & ~sign] = -0.0
    # whole frames of zeros of either sign, and one zero column per frame
    y[0] = 0.0
    y[1] = -0.0
    y[4:, 5] = -0.0
    return y


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("prec", [0, 2, 3])
@pytest.mark.parametrize("method", [0, 1])
def test_signed_zero_samples(golden, method, prec, mode):
    """Modes 0 (default) and 2 are the reference's arithmetic bit for bit:
    bytes, iterations, syndromes and the posteriors' bits (sign of zero too)
    equal the oracle's on every frame.  Mode 3 (F64_FAST, compact tanh/log
    within 3 ulp of glibc) is not exact: on these frames -- a quarter of
    their samples exactly 0, posteriors near 0 for 50 iterations -- its last
    bits grow into decisions on 2 of 576 frames (126 and 376) at 50
    iterations (profiles/round2/signed_zero_probe.txt); pinned here so a
    change in either mode shows."""
    import ldpc_ece535a
    sys.path.insert(0, REPO)
    from oracle import oracle as orc
    dec = ldpc_ece535a.Decoder()
    dec.set_launch_mode(mode)
    y = _frames(golden)
    for iters in (5, 50):
        out = dec.decode(y, method=method, max_iters=iters, precision=prec, want_llr=True)
        ref = orc.decode_batch(method, dec.H, y, iters, nthreads=8, want_post=True)
        if method == 1 and prec == 3:
            bad = np.flatnonzero((out["packed"] != ref["packed"]).any(axis=1))
            assert len(bad) <= (0 if iters == 5 else 4), bad
            continue
        np.testing.assert_array_equal(out["packed"], ref["packed"])
        np.testing.assert_array_equal(out["iters"], ref["iters"])
        np.testing.assert_array_equal(out["synd"], ref["synd"])
        # posteriors (float of the f64 sums): bit patterns, NaN == NaN
        a, b = out["llr"], ref["post"]
        same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
        assert same.all(), np.argwhere(~same)[:5]
