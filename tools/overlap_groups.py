#!/usr/bin/env python3
"""Groups of a kernel's dispatches that ran on one set of streams (a new
group whenever the set of the last 4 streams changes), with the hardware
queues, dispatch count and mean concurrency of each (rocpd sqlite from
rocprofv3 --kernel-trace).

    python tools/overlap_groups.py results.db [--name decode_small_kernel] [--min 20]"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--name", default="decode_small_kernel")
    ap.add_argument("--min", type=int, default=20)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = [r for r in cur.execute("select start, end, queue_id, stream_id, name, grid_x from kernels order by start")
            if a.name in r[4]]
    groups, cur_g, cur_set = [], [], None
    for r in rows:
        key = (r[5],)
        if cur_g and (r[3] not in cur_set and len(cur_set) >= 4 or key != cur_g[-1][6]):
            groups.append(cur_g)
            cur_g, cur_set = [], set()
        if cur_set is None:
            cur_set = set()
        cur_set.add(r[3])
        cur_g.append(r + (key,))
    if cur_g:
        groups.append(cur_g)
    for g in groups:
        if len(g) < a.min:
            continue
        g = g[len(g) // 4:]  # past the warmup
        span = max(r[1] for r in g) - min(r[0] for r in g)
        busy = sum(r[1] - r[0] for r in g)
        q = collections.Counter(r[2] for r in g)
        s = collections.Counter(r[3] for r in g)
        print("%4d dispatches (grid %d): mean %.1f us, concurrency %.2f, queues %s, streams %s" % (
            len(g), g[0][5], busy / len(g) / 1e3, busy / max(span, 1), dict(q), dict(s)))


if __name__ == "__main__":
    main()
