#!/usr/bin/env python3
"""Does the headline (config 2, 4 batches in flight on the context's streams)
depend on what the process ran before?  Measures it fresh, then after each of
bench.py's variants in turn (config 5, config 4, the block), with the
context's stream set and with freshly made torch streams.

    python tools/headline_history.py [--steps 100]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gr-ldpc_ece535a_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=100)
    a = ap.parse_args()
    import torch
    import bench
    import ldpc_ece535a as L
    args = bench.parse([])
    args.no_cpu_baseline = True
    dev = torch.device("cuda", 0)
    dec = L.Decoder(device=0)
    dec.set_launch_mode(1)
    B, D = 4096, 4
    inputs = [bench.synth_device(L, torch, dec, B, 2.0, 2024 + 104729 * j, dev)[0] for j in range(D)]
    torch.cuda.synchronize(dev)

    def head(tag):
        r = bench.time_decoder(dec, torch, inputs, B, 1, 50, 1, 0, a.steps, a.warmup, inflight=D)
        ctx = B * dec.K * a.steps / r["wall"] / 1e6
        fresh = [torch.cuda.Stream(dev) for _ in range(D)]
        r = bench.time_decoder(dec, torch, inputs, B, 1, 50, 1, 0, a.steps, a.warmup, inflight=D,
                               streams=fresh)
        fr = B * dec.K * a.steps / r["wall"] / 1e6
        print("%-22s ctx streams %7.1f  fresh torch streams %7.1f Mbit/s" % (tag, ctx, fr), flush=True)

    head("fresh process")
    bench.config5_variant(L, torch, args, dev)
    head("after config 5")
    bench.config4_variant(L, torch, dev, args, args.seed + 31, cpu_sample=0)
    head("after config 4")
    from ldpc_ece535a import blocks
    with bench._quiet_stdout():
        bench.block_variant(L, torch, blocks, dev, args, inputs[0], B)
    head("after the block")


if __name__ == "__main__":
    main()
