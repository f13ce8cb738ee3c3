#!/usr/bin/env python3
"""Longest-first frame order against queue order on the bench's headline
workload (config 2: the reference's H, 4096 frames, sum-product f64, 50
iterations, 4 batches in flight on the context's streams, throughput launch
mode), interleaved A/B over several repetitions, plus the one-launch-at-a-time
(latency mode) case where a launch's tail is not filled by other batches.

    python tools/order_ab.py [--steps 200] [--reps 5]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gr-ldpc_ece535a_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import bench
    import ldpc_ece535a as L
    dev = torch.device("cuda", 0)
    dec = L.Decoder(device=0)
    B = 4096
    inputs = [bench.synth_device(L, torch, dec, B, 2.0, 2024 + 104729 * j, dev)[0] for j in range(4)]
    res = {}
    for mode, inflight, name in ((1, 4, "4 in flight"), (0, 1, "one at a time")):
        dec.set_launch_mode(mode)
        streams = [torch.cuda.ExternalStream(h, device=dev) for h in dec.streams(inflight)]
        for rep in range(a.reps):
            for order in (0, 1):
                dec.set_frame_order(order)
                r = bench.time_decoder(dec, torch, inputs, B, 1, 50, 1, 0, a.steps, a.warmup,
                                       inflight=inflight, streams=streams)
                mbit = B * dec.K * a.steps / r["wall"] / 1e6
                res.setdefault((name, order), []).append(mbit)
                print("%-14s order %d rep %d: %8.1f Mbit/s  (%.4f ms per launch, device)" % (
                    name, order, rep, mbit, r["per_launch_ms"]), flush=True)
    for name in ("4 in flight", "one at a time"):
        q, lf = res[(name, 0)], res[(name, 1)]
        mq, ml = sorted(q)[len(q) // 2], sorted(lf)[len(lf) // 2]
        print("%-14s median: queue %.1f, longest first %.1f Mbit/s (%+.1f %%)" % (
            name, mq, ml, 100.0 * (ml / mq - 1)), flush=True)


if __name__ == "__main__":
    main()
