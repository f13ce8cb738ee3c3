#!/usr/bin/env python3
"""Concurrency of one kernel's dispatches in a rocprofv3 --kernel-trace
database (rocpd sqlite): for the last K dispatches whose name matches, the
hardware queues they ran on, the mean number running at once (sum of
durations / wall span) and the span.

    python tools/overlap.py results.db [--name decode_small_kernel] [--last 100]"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--name", default="decode_small_kernel")
    ap.add_argument("--last", type=int, default=100)
    ap.add_argument("--skip-last", type=int, default=0, help="ignore this many final dispatches")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    rows = [r for r in cur.execute("select start, end, queue_id, stream_id, name from kernels order by start")
            if a.name in r[4]]
    if a.skip_last:
        rows = rows[:-a.skip_last]
    rows = rows[-a.last:]
    if not rows:
        print("no dispatches of", a.name)
        return
    span = max(r[1] for r in rows) - min(r[0] for r in rows)
    busy = sum(r[1] - r[0] for r in rows)
    q = collections.Counter(r[2] for r in rows)
    s = collections.Counter(r[3] for r in rows)
    print("%d dispatches: span %.1f us, mean duration %.1f us, mean concurrency %.2f" % (
        len(rows), span / 1e3, busy / len(rows) / 1e3, busy / max(span, 1)))
    print("queues:", dict(q))
    print("streams:", dict(s))


if __name__ == "__main__":
    main()
