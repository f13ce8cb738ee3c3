#!/usr/bin/env python3
"""The drop-in block's throughput alone (bench.py's block variant): general_work
over a stream of B frames of gr_complex in host memory at Eb/N0 4 and 2 dB,
sum-product f64, 50 iterations; prints Mbit/s, launches and decodes per call.

    python tools/block_bench.py [--batch 4096] [--reps 4] [--ebn0 4,2]
(under rocprofv3 --kernel-trace --stats for the per-kernel split)"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--ebn0", default="4,2")
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import bench
    import ldpc_ece535a as L
    from ldpc_ece535a import blocks
    Hr = L.Decoder().H
    for db in [float(x) for x in a.ebn0.split(",")]:
        y, _ = bench.synth(Hr, a.batch, db, 7 + int(db))
        st = np.zeros(2 * y.size, np.float32)
        st[0::2] = y.ravel()
        cx = st.view(np.complex64)
        blk = blocks.ldpc_decoder_cb(1, iterations=a.iters, precision=0)
        with bench._quiet_stdout():
            blk.general_work(a.batch * 4, cx[:64 * 8])
            l0, f0 = blk.launches, blk.frames_decoded
            made = calls = 0
            t0 = time.perf_counter()
            for _ in range(a.reps):
                pos = 0
                while pos + 64 <= cx.size:
                    o, used = blk.general_work(a.batch * 4, cx[pos:])
                    pos += used
                    made += o.size
                    calls += 1
                    if used == 0:
                        break
            dt = time.perf_counter() - t0
        print("ebn0 %g: %.2f Mbit/s, %.3f ms/call, %d calls, %.1f launches/call, %.0f decodes/call, "
              "%.2f decodes per output frame" % (
                  db, made * 8 / dt / 1e6, dt / calls * 1e3, calls, (blk.launches - l0) / calls,
                  (blk.frames_decoded - f0) / calls, (blk.frames_decoded - f0) / max(1, made / 4)),
              flush=True)


if __name__ == "__main__":
    main()
