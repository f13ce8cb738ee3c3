#!/usr/bin/env python3
"""Offline model of the decoder block's launch planning (CPU only).

Decodes every window of one synthetic stream -- each start sample, both
polarities -- once with the oracle (a table), then drives the real block
(csrc/block/ldpc_decoder_cb_impl.cc, through its test seam) over the stream
with the table as the frame decoder, and reports what each launch plan costs:
launches, decoded windows and the iterations they run (the GPU work).  The
block's outputs are compared with the restated general_work.  Planning knobs
are the block's LDPC_BLOCK_* environment variables, so one table serves an A/B
of several plans:

    python tools/block_policy_sim.py --frames 512 --ebn0 4,2 --plans base:,searches1:LDPC_BLOCK_SEARCHES=1
"""
import argparse
import ctypes
import os
import subprocess
import sys
import time
from multiprocessing import Pool

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gr-ldpc_ece535a_amd"))

_G = {}
MODEL_LAUNCH_US, MODEL_SLOTS, MODEL_ROUND_US = 40.0, 3072, 45.0


def _init(Hr, x, iters):
    _G.update(Hr=Hr, x=x, iters=iters)


def _chunk(args):
    from oracle import oracle as orc
    p0, n, pol = args
    x = _G["x"]
    r = orc.decode_batch(1, _G["Hr"], x[2 * p0:], _G["iters"], polarity=-1.0 if pol else 1.0,
                         cw_stride=2, elem_stride=2, B=n)
    return p0, pol, r["packed"], r["synd"], r["iters"]


def table(Hr, x, npos, iters, procs):
    KB = (Hr.shape[1] - Hr.shape[0] + 7) // 8
    packed = np.zeros((2, npos, KB), np.uint8)
    synd = np.zeros((2, npos), np.int32)
    its = np.zeros((2, npos), np.int32)
    C = 512
    jobs = [(p, min(C, npos - p), pol) for pol in (0, 1) for p in range(0, npos, C)]
    with Pool(procs, initializer=_init, initargs=(Hr, x, iters)) as pool:
        for p0, pol, pk, sy, it in pool.imap_unordered(_chunk, jobs):
            n = sy.size
            packed[pol, p0:p0 + n] = pk
            synd[pol, p0:p0 + n] = sy
            its[pol, p0:p0 + n] = it
    return packed, synd, its


def run_plan(env, cache):
    """Child process: the block reads its knobs from the environment at construction."""
    cmd = [sys.executable, os.path.abspath(__file__), "--child", cache]
    e = dict(os.environ)
    e.update(env)
    out = subprocess.run(cmd, env=e, capture_output=True, text=True, check=True)
    if out.stderr.strip():
        sys.stderr.write(out.stderr)
    return [l for l in out.stdout.splitlines() if l.startswith("plan:")][0][5:]


def child(cache):
    import ldpc_ece535a as L
    d = np.load(cache)
    packed, synd, its, x, Hr = d["packed"], d["synd"], d["its"], d["x"], d["Hr"]
    base = x.ctypes.data
    per_launch = {}
    per_launch_it = {}
    st = {"launches": 0, "windows": 0, "iters": 0, "max_iter_sum": 0}

    def fn(user, inp, n_floats, cw_stride, elem_stride, polarity, B, pk, sy):
        p0 = (ctypes.cast(inp, ctypes.c_void_p).value - base) // 8
        pol = 1 if polarity < 0 else 0
        pos = p0 + (cw_stride // 2) * np.arange(B)
        KB = packed.shape[2]
        np.ctypeslib.as_array(pk, shape=(B * KB,))[:] = packed[pol, pos].ravel()
        np.ctypeslib.as_array(sy, shape=(B,))[:] = synd[pol, pos]
        st["windows"] += B
        st["iters"] += int(its[pol, pos].sum())
        k = blk.launches  # the launch this run of windows belongs to
        per_launch[k] = per_launch.get(k, 0) + B
        per_launch_it[k] = per_launch_it.get(k, 0) + int(its[pol, pos].sum())
        return 0

    blk = L.ldpc_decoder_cb(1, _backend=fn)
    cx = x.view(np.complex64)
    import io
    import contextlib
    # the stream arrives in calls of `chunk` frames, unconsumed input carried
    # over as the GR scheduler does; the first call (acquisition) is not counted
    chunk = int(d["chunk"]) * 64
    pos, made, first = 0, [], True
    with contextlib.redirect_stdout(io.StringIO()):
        while pos + 64 <= cx.size:
            if first and pos >= chunk:
                first = False
                l0, w0, i0, m0 = blk.launches, st["windows"], st["iters"], len(made)
                per_launch.clear()
                per_launch_it.clear()
            o, used = blk.general_work(chunk // 16, cx[pos:pos + chunk])
            made.append(o)
            pos += used
            if used == 0:
                break
    out = np.concatenate(made)
    np.save(cache + ".out.npy", out)
    l, w, i, b = (blk.launches - l0, st["windows"] - w0, st["iters"] - i0,
                  sum(m.size for m in made[m0:]))
    # GPU time model: a launch costs its fixed overhead plus one 50-iteration
    # frame latency per round of wave slots its windows fill; or, with
    # LDPC_SIM_MODEL="launch_us,window_ns", a fixed cost per launch (host gap +
    # kernel floor) plus a cost per window (5 iterations on one MI355X:
    # "56,12.8", profiles/round4/block/)
    lin = os.environ.get("LDPC_SIM_MODEL")
    srv = os.environ.get("LDPC_SIM_SERVER")
    if srv:
        # window server: a round costs its latency (fixed + the slowest
        # window's iterations) plus its window-iterations at the decode
        # throughput: "round_us,per_iter_us,window_iter_ns"
        r0, ri, wn = (float(v) for v in srv.split(","))
        t = 0.0
        for k, W in per_launch.items():
            t += r0 + ri * int(d["iters_cap"]) + per_launch_it[k] * wn / 1e3
    elif lin:
        lu, wn = (float(v) for v in lin.split(","))
        t = sum(lu + W * wn / 1e3 for W in per_launch.values())
    else:
        t = sum(MODEL_LAUNCH_US + -(-W // MODEL_SLOTS) * MODEL_ROUND_US for W in per_launch.values())
    if os.environ.get("LDPC_SIM_PER_LAUNCH"):
        sys.stderr.write("windows per launch: %s\n" % [per_launch[k] for k in sorted(per_launch)])
    print("plan:launches %d windows %d iters %d out_frames %d model %.2f ms (%.1f Mbit/s)" % (
        l, w, i, b // 4, t / 1e3, b * 8 / t))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--ebn0", default="4,2")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--chunk", type=int, default=512, help="frames of input per call")
    ap.add_argument("--plans", default="base:,searches1:LDPC_BLOCK_SEARCHES=1")
    ap.add_argument("--child", default="")
    ap.add_argument("--cache", default="/tmp/blkpol")
    a = ap.parse_args()
    if a.child:
        return child(a.child)
    import bench
    from oracle import oracle as orc
    Hr = np.load(os.path.join(REPO, "tests/golden/frames_default.npz"))["H_reordered"]
    for db in [float(v) for v in a.ebn0.split(",")]:
        cache = "%s_%d_%g.npz" % (a.cache, a.frames, db)
        if not os.path.exists(cache):
            y, _ = bench.synth(Hr, a.frames, db, 7 + int(db))
            x = np.zeros(2 * y.size, np.float32)
            x[0::2] = y.ravel()
            t = time.time()
            packed, synd, its = table(Hr, x, x.size // 2 - 64 + 1, a.iters, a.procs)
            ref = orc.run_stream(1, Hr, x.view(np.complex64), iterations=a.iters)
            np.savez(cache, packed=packed, synd=synd, its=its, x=x, Hr=Hr, chunk=a.chunk, ref=ref,
                     iters_cap=a.iters)
            print("table %g dB: %d windows in %.1f s" % (db, synd.size, time.time() - t), flush=True)
        ref = np.load(cache)["ref"]
        for spec in a.plans.split(","):
            name, _, kv = spec.partition(":")
            env = dict(p.split("=", 1) for p in kv.split(";") if p)
            res = run_plan(env, cache)
            out = np.load(cache + ".out.npy")
            same = "same" if out.size == ref.size and (out == ref).all() else "DIFFERENT"
            print("%g dB %-10s %s  [%s]" % (db, name, res, same), flush=True)


if __name__ == "__main__":
    main()
