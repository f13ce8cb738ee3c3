"""Throughput of K timed steps (the driver times K = 20) against the launch
configuration: batches in flight, persistent waves per CU, launch mode.
After a long warm-up on the same process, so only fill/drain of the K-step
window differs.  Prints one line per (config, K)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gr-ldpc_ece535a_amd"))

import bench  # noqa: E402


def main():
    import torch
    import ldpc_ece535a as L
    dev = torch.device("cuda", 0)
    dec = L.Decoder()
    B = 4096
    ks = [int(k) for k in os.environ.get("KS", "20,50,200").split(",")]
    cfgs = os.environ.get("CFGS", "1:4:0,1:8:0,1:4:8,1:2:0,0:4:0,1:4:16").split(",")
    inputs = [bench.synth_device(L, torch, dec, B, 2.0, 2024 + 7919 * j, dev)[0] for j in range(8)]
    torch.cuda.synchronize()
    bench.time_decoder(dec, torch, inputs[:4], B, 1, 50, 1, 0, 300, 10, inflight=4)
    if os.environ.get("PRE"):  # K=20 W=5 after 30+ ms of another (method, precision)
        for pre in os.environ["PRE"].split(","):
            m, p, W = (int(x) for x in pre.split(":"))
            dec.set_launch_mode(1)
            bench.time_decoder(dec, torch, inputs[:4], B, m, 50, 1, p, 700, 4, inflight=4)
            r = bench.time_decoder(dec, torch, inputs[:4], B, 1, 50, 1, 0, 20, W, inflight=4)
            print("after method %d prec %d, W %d: K 20 %8.1f Mbit/s" % (
                m, p, W, B * dec.K * 20 / r["wall"] / 1e6), flush=True)
    for c in cfgs:
        mode, D, wpc = (int(x) for x in c.split(":"))
        dec.set_launch_mode(mode)
        if wpc:  # 0: the mode's own (throughput: 4)
            dec.set_waves_per_cu(wpc)
        for K in ks:
            r = bench.time_decoder(dec, torch, inputs[:D], B, 1, 50, 1, 0, K, 20, inflight=D)
            print("mode %d inflight %d wpc %2d K %4d: %8.1f Mbit/s (span %.4f ms/launch)" % (
                mode, D, wpc, K, B * dec.K * K / r["wall"] / 1e6, r["per_launch_ms"]), flush=True)


if __name__ == "__main__":
    main()
