#!/usr/bin/env python3
"""Scheduling model of the persistent small-code decode kernel (diagnostic).

Feeds the per-frame iteration counts of the bench batch (oracle, config 2)
through a processor-sharing model of the SIMDs: `slots` resident waves per
SIMD; a wave running alone takes `t1` us per iteration (latency-bound), n
busy waves share the SIMD's VALU issue at `tv` us per frame-iteration, so
each takes max(t1, n * tv) per iteration.  Compares the plain frame queue
with the two-phase schedule (a frame still running after `park` iterations
is parked; parked frames are resumed once the frame queue is empty).

    python tools/sched_sim.py [--batch 4096] [--park 4,6,8,10,12]
"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gr-ldpc_ece535a_amd"))


def simulate(iters, simds, slots, t1, tv, park=0, dt=0.02):
    """Makespan (us) of one launch under the model."""
    W = simds * slots
    simd_of = np.arange(W) % simds
    B = len(iters)
    rem = np.zeros(W)            # iterations left in the wave's current run
    busy = np.zeros(W, bool)
    owes = np.zeros(W)           # iterations the current run parks for later
    parked = []
    nxt = 0
    t = 0.0

    def take(w):
        nonlocal nxt
        if nxt < B:
            it = iters[nxt]
            nxt += 1
            if park and it > park:
                rem[w], owes[w] = park, it - park
            else:
                rem[w], owes[w] = it, 0
            busy[w] = True
        elif parked:
            rem[w], owes[w] = parked.pop(0), 0
            busy[w] = True

    for w in range(W):
        take(w)
    while busy.any():
        n = np.bincount(simd_of[busy], minlength=simds)
        per_it = np.maximum(t1, n[simd_of] * tv)
        rem[busy] -= dt / per_it[busy]
        t += dt
        for w in np.where(busy & (rem <= 0))[0]:
            busy[w] = False
            if owes[w] > 0:
                parked.append(owes[w])
                owes[w] = 0
        for w in np.where(~busy)[0]:
            if nxt >= B and not parked:
                break
            take(w)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--park", default="4,6,8,10,12,16")
    ap.add_argument("--t1", type=float, default=0.81)
    ap.add_argument("--tv", type=float, default=0.42)
    ap.add_argument("--slots", type=int, default=3)
    a = ap.parse_args()
    import bench
    import ldpc_ece535a as L
    from oracle import oracle as orc
    Hr, _ = L.reorder_h(L.default_h())
    y, _ = bench.synth(Hr, a.batch, 2.0, 2024)
    ref = orc.decode_batch(1, Hr, y, 50, nthreads=8)
    it = ref["iters"].astype(np.float64)
    h = np.bincount(ref["iters"], minlength=51)
    print("mean iters %.2f; at cap %d; histogram 1..20: %s" % (it.mean(), h[50], h[1:21].tolist()))
    print("frame queue: %.1f us" % simulate(it, 1024, a.slots, a.t1, a.tv))
    for p in [int(x) for x in a.park.split(",")]:
        print("park at %2d: %.1f us" % (p, simulate(it, 1024, a.slots, a.t1, a.tv, park=p)))


if __name__ == "__main__":
    main()
