#!/usr/bin/env python3
"""Parity sweep (diagnostic): GPU f64 decode vs the C oracle over channel
amplitude x Eb/N0, 2048 frames each; prints mismatching frames per cell."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gr-ldpc_ece535a_amd")]
import torch  # noqa: F401,E402
import ldpc_ece535a as L  # noqa: E402
from oracle import oracle as orc  # noqa: E402

d = L.Decoder()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
# launch mode: 0 latency build (the block), 1 throughput build (bench.py)
mode = int(sys.argv[2]) if len(sys.argv) > 2 else 0
d.set_launch_mode(mode)
print("launch mode %d, %d frames per cell" % (mode, B), flush=True)
threads = max(1, min(16, len(os.sched_getaffinity(0))))
for method in (1, 0):
    for amp in (1.0, 2.0, 4.0, 8.0, 16.0):
        row = []
        for db in (0.0, 2.0, 4.0, 6.0, 8.0):
            rng = np.random.Generator(np.random.PCG64(int(1000 * amp + 10 * db + method)))
            data = rng.integers(0, 2, size=(B, d.K), dtype=np.uint8)
            x = 2.0 * L.encode(d.H, data) - 1.0
            y = (amp * (x + np.sqrt(10 ** (-db / 10)) * rng.standard_normal(x.shape))).astype(np.float32)
            out = d.decode(y, method=method, max_iters=50)
            ref = orc.decode_batch(method, d.H, y, 50, nthreads=threads)
            bad = (out["bits"] != ref["bits"]).any(axis=1) | (out["iters"] != ref["iters"])
            row.append(int(bad.sum()))
        print("method %d amp %5.1f  mismatching frames at 0,2,4,6,8 dB: %s" % (method, amp, row), flush=True)
