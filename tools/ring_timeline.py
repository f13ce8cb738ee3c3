#!/usr/bin/env python3
"""Timeline of one frame-ring session (diagnostic).  Needs a library built
with -DLDPC_TIMELINE (tools/ab_variants.sh "" "-DLDPC_TIMELINE" -> ab/V1;
LDPC_PKG_DIR points at it).  Runs warm sessions of K config-2 batches, then
one more, reads back every ticket's {wave start, frame start, samples
loaded, frame end, wave | iterations} (100 MHz clock), and prints where the
session's time goes: the launch's start, the first frames, the gap a wave
spends between two frames, frames in flight over time, and the tail."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.environ.get("LDPC_PKG_DIR", os.path.join(REPO, "gr-ldpc_ece535a_amd")))
import torch  # noqa: E402
import bench  # noqa: E402
import ldpc_ece535a as L  # noqa: E402


def main():
    lib = L._capi.lib()
    if not hasattr(lib, "ldpc_debug_ring_timeline"):
        sys.exit("library built without -DLDPC_TIMELINE")
    dev = torch.device("cuda", 0)
    dec = L.Decoder()
    B = 4096
    K = int(os.environ.get("K", "20"))
    ins = [bench.synth_device(L, torch, dec, B, 2.0, 2024 + 104729 * j, dev)[0] for j in range(4)]
    st = torch.cuda.Stream(dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    pool = [(torch.empty((B, dec.KB), dtype=torch.uint8, device=dev),
             torch.empty(B, dtype=torch.int32, device=dev),
             torch.empty(B, dtype=torch.int32, device=dev)) for _ in range(K)]

    def session():
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        dec.ring_begin(method=1, max_iters=50, stream=sp)
        for k in range(K):
            pk, it, sy = pool[k]
            dec.ring_post(ins[k % 4].data_ptr(), B, pk.data_ptr(), it.data_ptr(), sy.data_ptr())
        dec.ring_end()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    if os.environ.get("PREROLL") == "serial":  # bench.py's order: 30 ms one batch at a time, 5-batch session
        dec2 = L.Decoder()
        dec2.set_launch_mode(0)
        s1 = torch.cuda.Stream(dev)
        import time
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < 0.03:
                pk, it, sy = pool[0]
                dec2.decode_device(ins[0].data_ptr(), B, pk.data_ptr(), method=1, max_iters=50,
                                   d_iters=it.data_ptr(), d_synd=sy.data_ptr(), stream=s1.cuda_stream)
                s1.synchronize()
            dec.ring_begin(method=1, max_iters=50, stream=sp)
            for k in range(5):
                pk, it, sy = pool[k]
                dec.ring_post(ins[k % 4].data_ptr(), B, pk.data_ptr(), it.data_ptr(), sy.data_ptr())
            dec.ring_end()
            torch.cuda.synchronize()
            span_ms = session()
            print("serial pre-roll: span %.1f us per batch" % (1e3 * span_ms / K))
    else:
        for _ in range(40):
            session()
        span_ms = session()
    n = K * B
    W = 6
    buf = np.zeros(W * n, np.uint64)
    lib.ldpc_debug_ring_timeline.argtypes = [ctypes.c_void_p, ctypes.c_int]
    got = lib.ldpc_debug_ring_timeline(buf.ctypes.data, n)
    tl = buf[:W * got].reshape(got, W).astype(np.int64)
    wave0, f0, f1, f3 = tl[:, 0], tl[:, 1], tl[:, 2], tl[:, 3]
    wid, its = tl[:, 4] >> 8, tl[:, 4] & 255
    T0 = wave0.min()
    us = lambda x: x / 100.0  # noqa: E731  (100 MHz ticks -> us)
    print("host span (events) %.1f us; device: first wave start -> last frame end %.1f us; "
          "%d frames, mean iterations %.2f" % (1e3 * span_ms, us(f3.max() - T0), got, its.mean()))
    nw = len(np.unique(wid))
    print("waves %d; wave starts: last %.1f us after the first" % (nw, us(wave0.max() - T0)))
    first = np.argsort(f0)[:nw]
    print("first frames start: median %.1f us, p99 %.1f, max %.1f (after the first wave start)" % (
        us(np.median(f0[first] - T0)), us(np.percentile(f0[first] - T0, 99)), us((f0[first] - T0).max())))
    print("samples load + claim per frame (f1 - f0): median %.2f us, p99 %.2f" % (
        us(np.median(f1 - f0)), us(np.percentile(f1 - f0, 99))))
    order = np.lexsort((f0, wid))
    w_s, f0_s, f3_s = wid[order], f0[order], f3[order]
    same = w_s[1:] == w_s[:-1]
    gaps = (f0_s[1:] - f3_s[:-1])[same]
    print("gap between a wave's frames (locate + outputs): median %.2f us, p90 %.2f, p99 %.2f, "
          "total %.1f wave-us = %.2f%% of wave time" % (
              us(np.median(gaps)), us(np.percentile(gaps, 90)), us(np.percentile(gaps, 99)),
              us(gaps.sum()), 100.0 * gaps.sum() / ((f3 - f0).sum() + gaps.sum())))
    dur = f3 - f0
    clk = tl[:, 5] / np.maximum(dur, 1) * 100.0  # MHz
    mid = (f0 + f3) // 2
    for lo_, hi_ in ((0.0, 0.1), (0.1, 0.5), (0.5, 0.9), (0.9, 1.0)):
        a_, b_ = T0 + lo_ * (f3.max() - T0), T0 + hi_ * (f3.max() - T0)
        sel_ = (mid >= a_) & (mid < b_)
        print("core clock, frames centred in %3.0f-%3.0f%% of the span: %.0f MHz" % (
            100 * lo_, 100 * hi_, np.median(clk[sel_])))
    print("frame time at full load: %.2f us per iteration (median of frame time / iterations)" % (
        us(np.median(dur / np.maximum(its, 1)))))
    # frames in flight over time
    t_end = f3.max()
    edges = np.arange(T0, t_end + 1000, 1000)  # 10 us bins
    inflight = np.zeros(len(edges))
    ev = np.concatenate([np.stack([f0, np.ones_like(f0)], 1), np.stack([f3, -np.ones_like(f3)], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    cur = np.cumsum(ev[:, 1])
    idx = np.searchsorted(ev[:, 0], edges, side="right") - 1
    inflight = np.where(idx >= 0, cur[np.clip(idx, 0, None)], 0)
    print("frames in flight per 10 us (first 12 bins):", " ".join(str(int(x)) for x in inflight[:12]))
    print("frames in flight per 10 us (last 25 bins):", " ".join(str(int(x)) for x in inflight[-25:]))
    last_start = f0.max()
    print("last frame start -> last frame end: %.1f us; frames ending in the last 100 us: %d" % (
        us(t_end - last_start), int((f3 > t_end - 10000).sum())))
    full = inflight >= 0.98 * nw
    print("time with >= 98%% of waves busy: %.1f us of %.1f" % (10 * full.sum(), us(t_end - T0)))
    busy_wave_us = us(dur.sum())
    print("wave-time busy %.1f%% of waves x device span" % (100.0 * busy_wave_us / (nw * us(t_end - T0))))


if __name__ == "__main__":
    main()
