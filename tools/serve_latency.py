#!/usr/bin/env python3
"""Round latency of the window server (ldpc_serve_windows) against a launch
per round (ldpc_decode_windows): B windows of one staged span at random
positions / polarities, sum-product f64, 5 and 50 iterations; median host
time per round over many rounds.

    python tools/serve_latency.py [--sizes 1,64,400,1024,4096] [--rounds 200]"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gr-ldpc_ece535a_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,64,400,1024,4096")
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--iters", default="5,50")
    ap.add_argument("--ebn0", type=float, default=4.0)
    ap.add_argument("--mode", type=int, default=0, help="ldpc_set_launch_mode for the launch path")
    ap.add_argument("--no-serve", action="store_true")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import bench
    import ldpc_ece535a as L
    dec = L.Decoder()
    dec.set_launch_mode(a.mode)
    y, _ = bench.synth(dec.H, 4096, a.ebn0, 3)
    s = y.ravel()
    rng = np.random.default_rng(1)
    for it in [int(x) for x in a.iters.split(",")]:
        for B in [int(x) for x in a.sizes.split(",")]:
            wins = [((rng.integers(0, s.size - 64, B).astype(np.int64)) << 1) |
                    rng.integers(0, 2, B).astype(np.int64) for _ in range(8)]
            dec.stage_span(s, max_windows=max(B, 4096))
            # launch per round
            t = []
            for r in range(a.rounds):
                t0 = time.perf_counter()
                dec.decode_windows(s, wins[r % 8], method=1, max_iters=it, reuse_span=True)
                t.append(time.perf_counter() - t0)
            launch_us = 1e6 * np.median(t[a.rounds // 4:])
            if a.no_serve:
                print("iters %2d B %5d: launch %8.1f us per round (mode %d)" % (it, B, launch_us, a.mode),
                      flush=True)
                continue
            dec.stage_span(s, max_windows=max(B, 4096))
            dec.serve_begin(method=1, max_iters=it, max_windows=max(B, 4096))
            t = []
            for r in range(a.rounds):
                t0 = time.perf_counter()
                dec.serve_windows(wins[r % 8])
                t.append(time.perf_counter() - t0)
            dec.serve_end()
            serve_us = 1e6 * np.median(t[a.rounds // 4:])
            print("iters %2d B %5d: launch %8.1f us  serve %8.1f us per round" % (
                it, B, launch_us, serve_us), flush=True)


if __name__ == "__main__":
    main()
