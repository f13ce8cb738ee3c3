#!/usr/bin/env python3
"""Diagnostic: per-batch time of the config-2 decode with 1, 2 or 3 batches in
flight (consecutive batches on alternating HIP streams, one context).

    python tools/exp_pipeline.py [--steps 100] [--warmup 20]
"""
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
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096)
    a = ap.parse_args()
    import torch
    import bench
    import ldpc_ece535a as L
    dec = L.Decoder()
    B = a.batch
    bufs = []
    for k in range(3):
        y, _ = bench.synth(dec.H, B, 2.0, 2024 + k)
        bufs.append(dict(inp=torch.from_numpy(y).cuda(),
                         pk=torch.empty((B, dec.KB), dtype=torch.uint8, device="cuda"),
                         it=torch.empty(B, dtype=torch.int32, device="cuda")))
    for depth in (1, 2, 3, 1, 2):
        streams = [torch.cuda.Stream() for _ in range(depth)]

        def step(k):
            st = streams[k % depth]
            b = bufs[k % depth]
            dec.decode_device(b["inp"].data_ptr(), B, b["pk"].data_ptr(), method=1, max_iters=50,
                              d_iters=b["it"].data_ptr(), stream=st.cuda_stream)
        for k in range(a.warmup):
            step(k)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.steps):
            step(k)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        print("depth %d: %.4f ms per batch, %.1f Mbit/s" % (depth, dt * 1e3, B * 32 / dt / 1e6),
              flush=True)


if __name__ == "__main__":
    main()
