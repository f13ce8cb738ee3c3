#!/usr/bin/env python3
"""Per-kernel summary and the launch sequence of the last decode from a
rocprofv3 rocpd database (tools/trace_seq.py <dir-with-.db> [marker])."""
import collections
import glob
import re
import sqlite3
import statistics
import sys


def load(path):
    db = glob.glob(path + "/**/*.db", recursive=True)[0] if not path.endswith(".db") else path
    c = sqlite3.connect(db)
    tabs = {re.sub(r"_[0-9a-f]{8}_.*", "", r[0]): r[0]
            for r in c.execute("select name from sqlite_master where type='table'")}
    kd, ks = tabs["rocpd_kernel_dispatch"], tabs["rocpd_info_kernel_symbol"]
    return c.execute(f"select s.kernel_name, d.start, d.end from {kd} d join {ks} s "
                     f"on d.kernel_id=s.id order by d.start").fetchall()


def short(n):
    m = re.search(r"(g_[a-z_]+|decode_\w+?kernel)", n)
    return m.group(1) if m else n[:30]


if __name__ == "__main__":
    rows = load(sys.argv[1])
    marker = sys.argv[2] if len(sys.argv) > 2 else "g_reset"
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, s, e in rows:
        agg[short(n)][0] += 1
        agg[short(n)][1] += (e - s) / 1e6
    tot = sum(v[1] for v in agg.values())
    for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"{k:24s} n={n:6d} total={t:10.3f} ms avg={t / n * 1e3:9.2f} us {t / tot * 100:5.1f}%")
    idx = [i for i, r in enumerate(rows) if marker in r[0]]
    if idx:
        seq = rows[idx[-1]:]
        print(" ".join("%s:%.0f" % (short(n)[2:5], (e - s) / 1e3) for n, s, e in seq))
        print("last decode span ms %.3f" % ((seq[-1][2] - seq[0][1]) / 1e6))
