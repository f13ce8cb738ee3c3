#!/usr/bin/env python3
"""Cost of the block's window launches (ldpc_decode_windows) against plain
device-resident launches of the same frames (diagnostic): median host-timed
latency per call by batch size and iteration cap, sum-product f64 (exact),
latency launch mode -- which part of a window launch is fixed, which grows
with windows and which with iterations.

    python tools/window_cost.py [--sizes 1,64,512,2048,8192] [--iters 1,5,20]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,64,512,1024,2048,4096,8192")
    ap.add_argument("--iters", default="1,5,20")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--ebn0", type=float, default=4.0)
    a = ap.parse_args()
    import torch  # first: one HIP runtime
    import bench
    import ldpc_ece535a as L
    dec = L.Decoder()
    N = dec.N
    sizes = [int(v) for v in a.sizes.split(",")]
    Bmax = max(sizes)
    y, _ = bench.synth(dec.H, Bmax, a.ebn0, 5)
    cx = np.zeros(2 * y.size, np.float32)
    cx[0::2] = y.ravel()
    d_y = torch.from_numpy(y).cuda()
    st = torch.cuda.Stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    pk = torch.empty((Bmax, dec.KB), dtype=torch.uint8, device="cuda")
    for it in [int(v) for v in a.iters.split(",")]:
        for B in sizes:
            win = (np.arange(B, dtype=np.int64) * N) << 1
            dec.decode_windows(cx, win, method=1, max_iters=it, elem_stride=2)  # stage + warm
            tw = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                dec.decode_windows(cx, win, method=1, max_iters=it, elem_stride=2, reuse_span=True)
                tw.append(time.perf_counter() - t0)
            td = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                dec.decode_device(d_y.data_ptr(), B, pk.data_ptr(), method=1, max_iters=it,
                                  stream=sp)
                st.synchronize()
                td.append(time.perf_counter() - t0)
            print("iters %2d B %5d  windows %8.1f us  device frames %8.1f us" %
                  (it, B, 1e6 * np.median(tw), 1e6 * np.median(td)), flush=True)


if __name__ == "__main__":
    main()
