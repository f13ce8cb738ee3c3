#!/usr/bin/env python3
"""Latency of one ldpc_decode_windows call (the block's launch unit) against
the number of windows: one staged span of frames at -3 dB (every window runs
the 50-iteration cap), reuse_span=1, median over --reps calls.  The host side
of a launch is what the LDPC_WIN_COPY / LDPC_WIN_SPIN knobs change.

    python tools/window_latency.py [--sizes 1,64,256,1024,4096] [--reps 50]"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,64,256,1024,4096")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--label", default="")
    ap.add_argument("--iters", default="50", help="iteration caps, comma-separated")
    ap.add_argument("--schedules", default="0", help="kernel schedules (ldpc_set_schedule), comma-separated")
    a = ap.parse_args()
    import torch  # noqa: F401
    import bench
    import ldpc_ece535a as L
    dec = L.Decoder()
    Bmax = max(int(v) for v in a.sizes.split(","))
    y, _ = bench.synth(dec.H, Bmax + 1, -3.0, 11)
    span = y.ravel().astype(np.float32)
    for sched, it, B in [(s, int(i), int(b)) for s in a.schedules.split(",")
                         for i in a.iters.split(",") for b in a.sizes.split(",")]:
        dec.set_schedule(int(sched))
        if True:
            rng = np.random.default_rng(B)
            w = (rng.integers(0, span.size - 64, size=B).astype(np.int64) << 1) | \
                rng.integers(0, 2, B)
            dec.decode_windows(span, w, max_iters=it)  # stage the span
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                dec.decode_windows(span, w, max_iters=it, reuse_span=True)
                ts.append(time.perf_counter() - t0)
            print("%s schedule=%s iters=%2d B=%5d median %.1f us  min %.1f us" % (
                a.label, sched, it, B, 1e6 * np.median(ts), 1e6 * np.min(ts)), flush=True)


if __name__ == "__main__":
    main()
