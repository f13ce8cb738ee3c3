#!/usr/bin/env python3
"""The drop-in block's throughput alone (bench.py's block variant): general_work
over a continuous stream of gr_complex in host memory, fed in calls of B frames
(bench.drive_stream), at several Eb/N0, sum-product f64, 50 iterations; prints
Mbit/s, launches per call and decoded windows per output frame for each launch
plan (the block's LDPC_BLOCK_* knobs, read when a block is made).

    python tools/block_bench.py [--batch 4096] [--reps 4] [--ebn0 4,2]
        [--plans "default:,launch:LDPC_BLOCK_SERVE=0"]
(under rocprofv3 --kernel-trace --stats for the per-kernel split)"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

KNOBS = ("LDPC_BLOCK_SERVE", "LDPC_BLOCK_MAXWANT", "LDPC_BLOCK_SEARCHES")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--ebn0", default="4,2")
    ap.add_argument("--plans", default="default:")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import bench
    import ldpc_ece535a as L
    from ldpc_ece535a import blocks
    Hr = L.Decoder().H
    for db in [float(x) for x in a.ebn0.split(",")]:
        y, _ = bench.synth(Hr, (a.reps + 1) * a.batch, db, 7 + int(db))
        st = np.zeros(2 * y.size, np.float32)
        st[0::2] = y.ravel()
        cx = st.view(np.complex64)
        for spec in a.plans.split(","):
            name, _, kv = spec.partition(":")
            for k in KNOBS:
                os.environ.pop(k, None)
            os.environ.update(dict(p.split("=", 1) for p in kv.split(";") if p))
            blk = blocks.ldpc_decoder_cb(1, iterations=a.iters, precision=0)
            with bench._quiet_stdout():
                dt, made, calls, launches, windows = bench.drive_stream(blk, cx, a.batch)
            print("ebn0 %g %-10s %.2f Mbit/s, %.3f ms/call, %d calls, %.1f launches/call, "
                  "%.2f windows per output frame" % (
                      db, name, made * 8 / dt / 1e6, dt / calls * 1e3, calls, launches / calls,
                      windows / max(1, made / 4)), flush=True)
            del blk  # LDPC_BLOCK_PROFILE prints its split when the block is destroyed
            import gc
            gc.collect()


if __name__ == "__main__":
    main()
