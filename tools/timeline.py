#!/usr/bin/env python3
"""Per-SIMD timeline of one headline decode launch (diagnostic).

Needs a library built with -DLDPC_TIMELINE (tools/ab_variants.sh "<args>"
"-DLDPC_TIMELINE" builds one into ab/V1); LDPC_PKG_DIR points at it.  Runs
the bench workload (config 2: default H, B frames, 2 dB, sum-product f64),
reads back every frame's start / end (100 MHz realtime clock) and hardware ids,
and prints: the launch span, the time-weighted share of SIMD-time spent with
0..3 frames resident, per-iteration time by concurrency, and when the last
frames started and ended.

    LDPC_PKG_DIR=$PWD/ab/V1 python tools/timeline.py [--batch 4096] [--json out]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--ebn0", type=float, default=2.0)
    ap.add_argument("--precision", type=int, default=0)
    ap.add_argument("--method", type=int, default=1)
    ap.add_argument("--json", default=None)
    ap.add_argument("--et", type=int, default=1, help="syndrome check period (50: every frame runs 50)")
    ap.add_argument("--launches", type=int, default=0,
                    help="instead: run this many launches from a cold process and print the span "
                         "and median in-kernel clock of selected ones (warmup behaviour)")
    ap.add_argument("--steady", type=int, default=0,
                    help="instead: K steps of the bench's throughput setting (4 batches in flight, "
                         "launch mode 1) after 300 warm ones; print the in-kernel clock of the "
                         "last frames recorded")
    a = ap.parse_args()
    import torch  # first: one HIP runtime
    import bench  # noqa: E402  (sets sys.path from LDPC_PKG_DIR)
    import ldpc_ece535a as L
    lib = L._capi.lib()
    if not hasattr(lib, "ldpc_debug_timeline"):
        sys.exit("library built without -DLDPC_TIMELINE")
    dec = L.Decoder()
    y, _ = bench.synth(dec.H, a.batch, a.ebn0, 2024)
    d_in = torch.from_numpy(y).cuda()
    B = a.batch
    buf = np.zeros(4 * B, np.uint64)
    lib.ldpc_debug_timeline.restype = ctypes.c_int
    if a.steady:
        dec.set_launch_mode(1)
        ins = [torch.from_numpy(bench.synth(dec.H, B, a.ebn0, 2024 + j)[0]).cuda() for j in range(4)]
        for k, steps in (("warm", 300), ("steady", a.steady)):
            r = bench.time_decoder(dec, torch, ins, B, a.method, 50, a.et, a.precision, steps, 10,
                                   inflight=4)
            torch.cuda.synchronize()
            assert lib.ldpc_debug_timeline(buf.ctypes.data_as(ctypes.c_void_p), B) == B
            t = buf.reshape(B, 4)
            dur = np.maximum((t[:, 1] - t[:, 0]).astype(np.float64) / 100.0, 1e-3)
            clk = t[:, 3] / dur / 1e3
            print("%s: %d steps, %.1f Mbit/s, in-kernel clock GHz median %.3f p5 %.3f p95 %.3f" % (
                k, steps, B * dec.K * steps / r["wall"] / 1e6, np.median(clk),
                np.percentile(clk, 5), np.percentile(clk, 95)), flush=True)
        return
    if a.launches:
        show = {0, 1, 2, 5, 10, 20, 50, 100, 150, 200, 300, 400, 600, 800}
        for i in range(a.launches):
            kms = bench.time_decoder(dec, torch, [d_in], B, a.method, 50, a.et, a.precision, 1,
                                     0)["per_launch_ms"]
            torch.cuda.synchronize()
            if i in show or i == a.launches - 1:
                assert lib.ldpc_debug_timeline(buf.ctypes.data_as(ctypes.c_void_p), B) == B
                t = buf.reshape(B, 4)
                st = t[:, 0].astype(np.float64)
                en = t[:, 1].astype(np.float64)
                dur = np.maximum((en - st) / 100.0, 1e-3)
                print("launch %4d: kernel %.4f ms, span %.1f us, in-kernel clock median %.3f GHz" %
                      (i, kms, (en.max() - st.min()) / 100.0, np.median(t[:, 3] / dur / 1e3)), flush=True)
        return
    r = bench.time_decoder(dec, torch, [d_in], a.batch, a.method, 50, a.et, a.precision, 3, 2)
    kern_ms, iters = r["per_launch_ms"], r["iters"]
    torch.cuda.synchronize()
    n = lib.ldpc_debug_timeline(buf.ctypes.data_as(ctypes.c_void_p), B)
    assert n == B, n
    t = buf.reshape(B, 4)
    start = (t[:, 0] - t[:, 0].min()).astype(np.float64) / 100.0  # us
    end = (t[:, 1] - t[:, 0].min()).astype(np.float64) / 100.0
    hw = (t[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    xcc = (t[:, 2] >> np.uint64(32)).astype(np.int64) & 0xF
    clk = t[:, 3].astype(np.float64) / np.maximum(end - start, 1e-3) / 1e3  # GHz
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    span = end.max()
    iters = np.asarray(iters, np.float64)
    print("launch: %d frames, mean kernel %.4f ms (3 launches), timeline span %.1f us, "
          "%d SIMDs used, mean iters %.2f" % (B, kern_ms, span, len(np.unique(key)), iters.mean()))
    # concurrency per SIMD over time
    grid = np.linspace(0, span, 2001)
    occ = np.zeros((4,), np.float64)
    conc_at_frame = np.zeros(B)
    keys = np.unique(key)
    for k in keys:
        idx = np.where(key == k)[0]
        c = np.zeros_like(grid)
        for i in idx:
            c += (grid >= start[i]) & (grid < end[i])
        for j in range(4):
            occ[j] += np.sum(np.minimum(c, 3) == j)
        for i in idx:
            m = (grid >= start[i]) & (grid < end[i])
            conc_at_frame[i] = c[m].mean() if m.any() else 1
    occ /= occ.sum()
    print("SIMD-time with 0/1/2/3 frames resident: %s" % " ".join("%.3f" % x for x in occ))
    dur = end - start
    per_it = dur / np.maximum(iters, 1)
    for lo, hi in ((0.5, 1.5), (1.5, 2.5), (2.5, 3.5)):
        m = (conc_at_frame >= lo) & (conc_at_frame < hi) & (iters >= 10)
        if m.any():
            print("frames at mean concurrency %.1f-%.1f: %4d, us per iteration median %.3f" %
                  (lo, hi, m.sum(), np.median(per_it[m])))
    long_ = iters == 50
    print("50-iteration frames: %d; their duration us: min %.1f median %.1f max %.1f" %
          (long_.sum(), dur[long_].min(), np.median(dur[long_]), dur[long_].max()))
    order = np.argsort(start)
    print("last frame started at %.1f us; 90%% of frames ended by %.1f us; last end %.1f us" %
          (start[order[-1]], np.percentile(end, 90), span))
    late = np.argsort(-end)[:5]
    for i in late:
        print("  frame %4d simd %5d start %.1f end %.1f iters %d conc %.2f" %
              (i, key[i], start[i], end[i], iters[i], conc_at_frame[i]))
    print("in-kernel clock GHz (per frame): median %.3f p5 %.3f p95 %.3f" %
          (np.median(clk), np.percentile(clk, 5), np.percentile(clk, 95)))
    if a.json:
        json.dump({"clk_ghz": clk.tolist(), "start_us": start.tolist(), "end_us": end.tolist(), "simd": key.tolist(),
                   "iters": iters.tolist()}, open(a.json, "w"))


if __name__ == "__main__":
    main()
