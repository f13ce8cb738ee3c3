#!/usr/bin/env python3
"""How much does the order frames are handed to the waves matter? (diagnostic)

Decodes the bench workload (config 2: default H, B frames, 2 dB, sum-product
f64) with the frames of every batch permuted on the host before timing:
  random     -- as made (the bench's order)
  weight     -- descending initial syndrome weight (unsatisfied checks of the
                hard decisions of the channel values), a predictor computable
                in one cheap pass
  iters      -- descending true iteration count (from a first decode): the
                longest-processing-time-first bound
and times one batch in flight (latency mode) and D in flight (throughput
mode, K steps after W warmup), printing ms per batch for each order.

    python tools/order_probe.py [--batch 4096] [--steps 20] [--warmup 5]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--inflight", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch  # first: one HIP runtime
    import bench
    import ldpc_ece535a as L
    dev = torch.device("cuda", 0)
    dec = L.Decoder(device=0)
    H = dec.H.astype(np.int64)
    B, D = a.batch, a.inflight
    ins = [bench.synth_device(L, torch, dec, B, 2.0, 2024 + 7919 * j, dev)[0] for j in range(D)]
    hosts = [x.cpu().numpy() for x in ins]
    # true iterations of every frame (one decode per batch, latency mode)
    dec.set_launch_mode(0)
    iters = [bench.time_decoder(dec, torch, [x], B, 1, 50, 1, 0, 1, 0)["iters"] for x in ins]
    orders = {}
    for j, y in enumerate(hosts):
        hard = (y > 0).astype(np.int64)  # bench's BPSK: x = 2c - 1
        w = ((hard @ H.T) & 1).sum(axis=1)
        orders.setdefault("random", []).append(np.arange(B))
        orders.setdefault("weight", []).append(np.argsort(-w, kind="stable"))
        orders.setdefault("iters", []).append(np.argsort(-iters[j], kind="stable"))
        if j == 0:
            long = iters[j] >= 50
            print("weight vs 50-iteration frames: corr(w, iters) %.3f; mean w long %.2f short %.2f"
                  % (np.corrcoef(w, iters[j])[0, 1], w[long].mean(), w[~long].mean()))
    for rnd in range(a.rounds):
        for name, perms in orders.items():
            xs = [torch.from_numpy(np.ascontiguousarray(h[p])).to(dev) for h, p in zip(hosts, perms)]
            dec.set_launch_mode(0)
            r1 = bench.time_decoder(dec, torch, xs[:1], B, 1, 50, 1, 0, 20, 5)
            dec.set_launch_mode(1)
            rD = bench.time_decoder(dec, torch, xs, B, 1, 50, 1, 0, a.steps, a.warmup, inflight=D)
            rL = bench.time_decoder(dec, torch, xs, B, 1, 50, 1, 0, 100, 20, inflight=D)
            print("round %d %-7s latency %.4f ms/batch | %d in flight K=%d: %.4f ms/step "
                  "(%.0f Mbit/s) | K=100: %.4f ms/step (%.0f Mbit/s)" % (
                      rnd, name, r1["per_launch_ms"], D, a.steps, rD["wall"] / a.steps * 1e3,
                      B * 32 * a.steps / rD["wall"] / 1e6, rL["wall"] / 100 * 1e3,
                      B * 32 * 100 / rL["wall"] / 1e6), flush=True)


if __name__ == "__main__":
    main()
