#!/usr/bin/env python3
"""Scheduling model of the persistent small-code decode kernel (diagnostic).

Feeds the per-frame iteration counts of the bench batch (oracle, config 2)
through a processor-sharing model of the SIMDs: `slots` resident waves per
SIMD; a wave running alone takes `t1` us per iteration (latency-bound), n
busy waves share the SIMD's VALU issue at `tv` us per frame-iteration, so
each takes max(t1, n * tv) per iteration.  Compares the plain frame queue
with the two-phase schedule (a frame still running after `park` iterations
is parked; parked frames are resumed once the frame queue is empty), and
(round 4) the verdict's join schedule: once the frame queue is empty, an idle
wave joins the running frame of a sibling wave of its 4-wave workgroup
(waves of a workgroup sit on the CU's 4 SIMDs; a frame's 3 edge slots allow
at most 3 waves), the frame advancing at the sum of its waves' rates times
an efficiency `e` for the two LDS handshakes per iteration -- with the
batch in queue order and in longest-first order (perfect knowledge).

    python tools/sched_sim.py [--batch 4096] [--park 4,6,8,10,12] [--join-e 0.8,1.0]
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


def simulate_join(iters, cus, slots, t1, tv, e=1.0, join=True):
    """Makespan (us) of one launch, event-driven: `slots` 4-wave workgroups
    per CU, wave p of the grid on CU (p // 4) % cus, SIMD p % 4."""
    B = len(iters)
    W = min(B, slots * cus * 4)
    simd = lambda w: ((w // 4) % cus) * 4 + w % 4
    on_simd = {}
    rem, parts = {}, {}
    nxt = 0
    for w in range(W):
        rem[nxt], parts[nxt] = float(iters[nxt]), [w]
        on_simd.setdefault(simd(w), set()).add(w)
        nxt += 1
    idle = set()
    t = 0.0
    while rem:
        rate = {}
        for f, ws in parts.items():
            r = sum(1.0 / max(t1, len(on_simd[simd(w)]) * tv) for w in ws)
            rate[f] = r * (e if len(ws) > 1 else 1.0)
        dt = min(rem[f] / rate[f] for f in rem)
        t += dt
        done = [f for f in rem if rem[f] - rate[f] * dt <= 1e-9]
        for f in rem:
            rem[f] -= rate[f] * dt
        for f in done:
            ws = parts.pop(f)
            del rem[f]
            for w in ws:
                if nxt < B:
                    rem[nxt], parts[nxt] = float(iters[nxt]), [w]
                    nxt += 1
                else:
                    on_simd[simd(w)].discard(w)
                    idle.add(w)
        if join:
            for w in sorted(idle):
                c = [f for f, ws in parts.items() if ws[0] // 4 == w // 4 and len(ws) < 3]
                if not c:
                    continue
                f = max(c, key=lambda x: rem[x])
                if rem[f] < 3:
                    continue
                parts[f].append(w)
                idle.discard(w)
                on_simd[simd(w)].add(w)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--park", default="4,6,8,10,12,16")
    ap.add_argument("--t1", type=float, default=0.81)
    ap.add_argument("--tv", type=float, default=0.42)
    ap.add_argument("--slots", type=int, default=3)
    ap.add_argument("--join-e", default="0.6,0.8,1.0")
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
    print("mean-work bound (every SIMD saturated to the end): %.1f us" % (it.sum() * a.tv / 1024))
    lpt = np.sort(it)[::-1]
    for name, order in [("queue order", it), ("longest first", lpt)]:
        print("%s, event model: no join %.1f us" % (name, simulate_join(order, 256, a.slots, a.t1, a.tv, join=False)))
        for e in [float(x) for x in a.join_e.split(",")]:
            print("%s, join e=%.1f: %.1f us" % (name, e, simulate_join(order, 256, a.slots, a.t1, a.tv, e=e)))


if __name__ == "__main__":
    main()
