#!/usr/bin/env python3
"""Per-batch PMC counters of the ring kernel vs the batch kernel from
tools/ring_pmc.sh output (rocprofv3 counter_collection.csv), and kernel
time per batch from the kernel traces."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r6/rpmc"
K = 50


def counters(mode, pas):
    tot = defaultdict(float)
    disp = set()
    for f in glob.glob("%s/%s_%s/*counter_collection.csv" % (root, mode, pas)):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "ring_kernel" not in name and "decode_small_kernel" not in name:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
    return tot, len(disp)


def ktime(mode):
    rows = []
    for f in glob.glob("%s/%s_kt/*kernel_trace.csv" % (root, mode)):
        for r in csv.DictReader(open(f)):
            if "ring_kernel" in r["Kernel_Name"] or "decode_small_kernel" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(rows)


for mode in ("ring", "launch"):
    rows = ktime(mode)
    if mode == "ring":
        per = [(e - s) / K / 1e3 for s, e in rows[-10:]]
        print("ring: %d launches, last 10: %.1f us per batch (min %.1f)" % (len(rows), sum(per) / len(per), min(per)))
    else:
        # sessions of K launches on 4 streams: span of each group of K
        spans = []
        for g in range(len(rows) // K):
            grp = rows[g * K:(g + 1) * K]
            spans.append((max(e for _, e in grp) - min(s for s, _ in grp)) / K / 1e3)
        print("launch: %d launches, last 10 groups: %.1f us per batch (min %.1f)" % (
            len(rows), sum(spans[-10:]) / len(spans[-10:]), min(spans[-10:])))
    for pas in ("p1", "p2"):
        tot, nd = counters(mode, pas)
        batches = nd * (K if mode == "ring" else 1)
        print("  %s %s dispatches=%d batches=%d" % (mode, pas, nd, batches))
        for k in sorted(tot):
            print("    %-24s %14.1f per batch" % (k, tot[k] / batches))
