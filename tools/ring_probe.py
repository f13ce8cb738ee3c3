#!/usr/bin/env python3
"""Frame-ring diagnostics (run on the GPU box, optionally under rocprofv3
--kernel-trace): host cost of ldpc_ring_post, and the ring launch's time for
K config-2 batches when the posts race the launch ("live") and when every
batch is posted before the launch starts ("preposted": the session's stream
first runs a spin kernel, so the ring's launch waits behind it)."""
import ctypes
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.environ.get("LDPC_PKG_DIR", os.path.join(REPO, "gr-ldpc_ece535a_amd")))
import torch  # noqa: E402
import bench  # noqa: E402
import ldpc_ece535a as L  # noqa: E402

ITERS = int(os.environ.get("ITERS", "50"))  # iteration cap of every session
EBN0 = float(os.environ.get("EBN0", "2.0"))


def session_n(dec, ins, pool, sp, st, n):
    """An untimed ring session of n batches (the pool is reused)."""
    dec.ring_begin(method=1, max_iters=ITERS, stream=sp)
    for k in range(n):
        pk, it, sy = pool[k % len(pool)]
        dec.ring_post(ins[k % 4].data_ptr(), pk.shape[0], pk.data_ptr(), it.data_ptr(), sy.data_ptr())
    dec.ring_end()
    torch.cuda.synchronize()


def main():
    dev = torch.device("cuda", 0)
    dec = L.Decoder()
    B = 4096
    ins = [bench.synth_device(L, torch, dec, B, EBN0, 2024 + 104729 * j, dev)[0] for j in range(4)]
    st = torch.cuda.Stream(dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    K = int(os.environ.get("K", "20"))
    pool = [(torch.empty((B, dec.KB), dtype=torch.uint8, device=dev),
             torch.empty(B, dtype=torch.int32, device=dev),
             torch.empty(B, dtype=torch.int32, device=dev)) for _ in range(K)]

    def session(pre_sleep):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(st)
        if pre_sleep:
            with torch.cuda.stream(st):
                torch.cuda._sleep(int(pre_sleep))
        dec.ring_begin(method=1, max_iters=ITERS, stream=sp)
        tp = []
        for k in range(K):
            a = time.perf_counter()
            pk, it, sy = pool[k]
            dec.ring_post(ins[k % 4].data_ptr(), B, pk.data_ptr(), it.data_ptr(), sy.data_ptr())
            tp.append(time.perf_counter() - a)
        dec.ring_end()
        e1.record(st)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        return wall, e0.elapsed_time(e1), np.array(tp) * 1e6

    if os.environ.get("MODE") == "launch":  # the round-5 form: a launch per batch, 4 streams
        dec.set_launch_mode(1)
        sts = [torch.cuda.Stream(dev) for _ in range(4)]
        for rep in range(12):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(K):
                pk, it, sy = pool[k]
                dec.decode_device(ins[k % 4].data_ptr(), B, pk.data_ptr(), method=1, max_iters=50,
                                  d_iters=it.data_ptr(), d_synd=sy.data_ptr(),
                                  stream=sts[k % 4].cuda_stream)
            torch.cuda.synchronize()
            print("launch K=%d wall %.3f ms" % (K, 1e3 * (time.perf_counter() - t0)), flush=True)
        return
    for _ in range(30):
        session(0)
    if os.environ.get("PREROLL"):  # what runs before a timed session (bench.py's order)
        dec2 = L.Decoder()
        dec2.set_launch_mode(0)
        s1 = torch.cuda.Stream(dev)

        def serial(ms):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < ms * 1e-3:
                pk, it, sy = pool[0]
                dec2.decode_device(ins[0].data_ptr(), B, pk.data_ptr(), method=1, max_iters=50,
                                   d_iters=it.data_ptr(), d_synd=sy.data_ptr(), stream=s1.cuda_stream)
                s1.synchronize()

        def short(nb):
            K0 = K
            globals()["K"] = nb
            return K0

        res = {}
        for rep in range(5):
            for mode in ("warm", "serial30+w5", "serial30+w5+idle50ms", "w50"):
                if mode.startswith("serial"):
                    serial(30)
                    session_n(dec, ins, pool, sp, st, 5)
                    if "idle" in mode:
                        time.sleep(0.05)
                elif mode == "w50":
                    session_n(dec, ins, pool, sp, st, 50)
                else:
                    session(0)
                res.setdefault(mode, []).append(1e3 * session(0)[1] / K)
        for m, v in res.items():
            print("preroll %-22s K=%d us/batch: median %.1f  all %s" % (
                m, K, float(np.median(v)), " ".join("%.1f" % x for x in v)), flush=True)
        return
    if os.environ.get("VARIANTS"):  # LDPC_RING_PROBE experiment bits, alternated
        vs = os.environ["VARIANTS"].split(",")
        res = {v: [] for v in vs}
        for rep in range(6):
            for v in vs:
                os.environ["LDPC_RING_PROBE"] = v
                sp_ = sorted(session(0)[1] for _ in range(5))
                res[v].append(sp_[2] * 1e3 / K)
        for v in vs:
            print("probe %-4s K=%d us/batch: median %.1f  all %s" % (
                v, K, float(np.median(res[v])), " ".join("%.1f" % x for x in res[v])), flush=True)
        return
    if os.environ.get("MODE") == "ring":
        for _ in range(10):
            session(0)
        return
    for mode, pre in (("live", 0), ("preposted", 2_000_000), ("live", 0), ("preposted", 2_000_000)):
        walls, spans, posts = [], [], []
        for _ in range(10):
            w, s, tp = session(pre)
            walls.append(w)
            spans.append(s)
            posts.append(tp)
        tp = np.concatenate(posts)
        print("%-9s K=%d wall %.3f ms  span %.3f ms (%.1f us/batch)  post us: median %.1f max %.1f"
              % (mode, K, 1e3 * np.median(walls), np.median(spans), 1e3 * np.median(spans) / K,
                 np.median(tp), tp.max()), flush=True)
    print("ring", dec.ring_info())


if __name__ == "__main__":
    main()
