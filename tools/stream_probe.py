#!/usr/bin/env python3
"""Which streams overlap: the headline's four-in-flight decode rate for
several ways of making its four streams, in one process.

  python tools/stream_probe.py [--steps K] [--patterns torch:0,torch:3,hip:0,...]

torch:k  k throw-away torch.cuda.Stream() objects, then the four streams
prioP:k  k throw-away raw streams, then four made with hipStreamCreateWithPriority(P)
         (P: 0, 1, m1 for -1)
hip:k    k throw-away hipStreamCreateWithFlags streams, then four raw HIP
         streams (wrapped as torch.cuda.ExternalStream for the events)
ctx:k    k throw-away torch streams, then a new decoder context's own in-flight
         set (ldpc_ctx_streams: probe-checked to run on distinct hardware queues)

Each line: pattern, Mbit/s, the four handles.  Run it under
`rocprofv3 --kernel-trace` to see which hardware queue each launch took.
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gr-ldpc_ece535a_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--patterns", default="torch:0,torch:1,torch:2,torch:3,hip:0,hip:1,hip:2,hip:3,torch:0")
    args = ap.parse_args()
    import torch
    import bench
    import ldpc_ece535a as L

    hip = ctypes.CDLL("libamdhip64.so")
    dev = torch.device("cuda", 0)
    dec = L.Decoder(device=0)
    B = 4096
    inputs = [bench.synth_device(L, torch, dec, B, 2.0, 2024 + 104729 * j, dev)[0] for j in range(4)]
    dec.set_launch_mode(1)
    keep = []  # throw-away streams stay alive (a destroyed one frees its queue slot)

    def raw_stream():
        s = ctypes.c_void_p()
        rc = hip.hipStreamCreateWithFlags(ctypes.byref(s), ctypes.c_uint(1))
        assert rc == 0, rc
        return s.value

    for pat in args.patterns.split(","):
        kind, _, k = pat.partition(":")
        k = int(k or 0)
        dd = dec
        if kind == "torch":
            keep += [torch.cuda.Stream(dev) for _ in range(k)]
            streams = [torch.cuda.Stream(dev) for _ in range(4)]
        elif kind == "hip":
            keep += [raw_stream() for _ in range(k)]
            streams = [torch.cuda.ExternalStream(raw_stream(), device=dev) for _ in range(4)]
        elif kind.startswith("prio"):  # prioP:k raw streams made with hipStreamCreateWithPriority
            prio = int(kind[4:].replace("m", "-"))

            def prio_stream():
                h = ctypes.c_void_p()
                rc = hip.hipStreamCreateWithPriority(ctypes.byref(h), ctypes.c_uint(1), ctypes.c_int(prio))
                assert rc == 0, rc
                return h.value
            keep += [prio_stream() for _ in range(k)]
            streams = [torch.cuda.ExternalStream(prio_stream(), device=dev) for _ in range(4)]
        elif kind == "own":  # the measuring context's own in-flight set
            keep += [torch.cuda.Stream(dev) for _ in range(k)]
            streams = [torch.cuda.ExternalStream(h, device=dev) for h in dec.streams(4)]
        elif kind == "newhip":  # a new context, raw HIP streams
            keep += [raw_stream() for _ in range(k)]
            d2 = L.Decoder(device=0)
            d2.set_launch_mode(1)
            keep.append(d2)
            dd = d2
            streams = [torch.cuda.ExternalStream(raw_stream(), device=dev) for _ in range(4)]
        elif kind == "ctx":
            keep += [torch.cuda.Stream(dev) for _ in range(k)]
            d2 = L.Decoder(device=0)
            d2.set_launch_mode(1)
            keep.append(d2)
            dd = d2
            streams = [torch.cuda.ExternalStream(h, device=dev) for h in d2.streams(4)]
        else:
            raise SystemExit("unknown pattern " + pat)
        keep += streams
        r = bench.time_decoder(dd, torch, inputs, B, 1, 50, 1, 0,
                               args.steps, args.warmup, inflight=4, streams=streams)
        mbit = B * dec.K * args.steps / r["wall"] / 1e6
        print("%-9s %8.1f Mbit/s  handles %s" % (pat, mbit, " ".join(hex(x.cuda_stream) for x in streams)),
              flush=True)


if __name__ == "__main__":
    main()
