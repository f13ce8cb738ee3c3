#!/usr/bin/env python3
"""Timeline of a rocprofv3 --kernel-trace --memory-copy-trace database
(rocpd sqlite): kernels and copies in start order, with gaps, from the Nth
event on.

    python tools/trace_timeline.py results.db [--skip N] [--count M]"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--count", type=int, default=80)
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    ev = [(s, e, "K " + n[:60], g) for s, e, n, g in
          cur.execute("select start, end, name, grid_x from kernels")]
    ev += [(s, e, "C %s %d B" % (n, z), 0) for s, e, n, z in
           cur.execute("select start, end, name, size from memory_copies")]
    ev.sort()
    t0 = ev[a.skip][0] if ev else 0
    prev_end = t0
    for s, e, n, g in ev[a.skip:a.skip + a.count]:
        print("%10.1f us  dur %8.1f  gap %8.1f  %s %s" % ((s - t0) / 1e3, (e - s) / 1e3,
                                                        (s - prev_end) / 1e3, n, g or ""))
        prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
