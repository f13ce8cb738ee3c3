#!/usr/bin/env python3
"""Summarise tools/profile.sh output: per-kernel mean duration (kernel
trace) and mean PMC counters per dispatch.  FETCH_SIZE is doubled per
MI355X_MICROARCH.md (gfx950 reports half of a wide coalesced read); both
FETCH_SIZE and WRITE_SIZE are in KiB.

usage: tools/parse_prof.py gpurun_out/prof/<tag> [--kernel substr] [--json out.json --key K]
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="decode_small_kernel")
    ap.add_argument("--json", default=None)
    ap.add_argument("--steps", type=int, default=0, help="timed launches at the end of the run")
    ap.add_argument("--source", default=None, help="recorded in the json entry")
    ap.add_argument("--key", default=None)
    ap.add_argument("--ring-batches", type=int, default=0,
                    help="frame ring: the kernel's LAST dispatch (the timed session) decoded this "
                         "many batches; its counters and duration are divided by it (per batch)")
    ap.add_argument("--per-decode", default=None,
                    help="large-code path: sum the traffic of every kernel whose name contains "
                         "this substring and divide by the number of decodes (g_reset dispatches)")
    a = ap.parse_args()
    res = {}
    kt = rows(os.path.join(a.dir, "kt", "**", "*kernel_trace.csv"))
    durs = collections.defaultdict(list)
    for r in kt:
        durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print("== kernel trace (ns) ==")
    if a.steps:
        # the last K dispatches of the kernel are the timed steps: their span
        # (first start to last end) / K is the per-launch time bench.py reports
        # (with D batches in flight a launch's own start-to-end is longer)
        mine = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kt
                      if a.kernel in r["Kernel_Name"])[-a.steps:]
        if mine:
            res["span_ns_per_launch"] = (max(e for _, e in mine) - mine[0][0]) / len(mine)
            print("timed launches: %d, span per launch %.1f ns" % (len(mine),
                                                                   res["span_ns_per_launch"]))
    for k, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        print("%-90s n=%4d mean=%10.1f median=%10.1f" % (k[:90], len(v), statistics.mean(v),
                                                          statistics.median(v)))
        if a.kernel in k:
            res["kernel"] = k
            res["mean_ns"] = statistics.mean(v)
            res["median_ns"] = statistics.median(v)
            res["dispatches"] = len(v)
    stats = rows(os.path.join(a.dir, "kt", "**", "*kernel_stats.csv"))
    for r in stats:
        if a.kernel in r.get("Name", ""):
            print("stats:", {k: r[k] for k in r if k in ("Name", "Calls", "AverageNs", "TotalDurationNs",
                                                           "Percentage")})
    counters = collections.defaultdict(list)
    if a.ring_batches:
        last = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in kt
                      if a.kernel in r["Kernel_Name"])[-1]
        res["mean_ns"] = res["span_ns_per_launch"] = (last[1] - last[0]) / a.ring_batches
        res["ring_session_ns"] = last[1] - last[0]
        res["ring_batches"] = a.ring_batches
        print("ring: last dispatch %.1f us, %d batches: %.1f ns per batch" % (
            (last[1] - last[0]) / 1e3, a.ring_batches, res["mean_ns"]))
    for p in ("pmc1", "pmc2", "pmc3", "pmc4", "pmc5"):
        prs = [r for r in rows(os.path.join(a.dir, p, "**", "*counter_collection.csv"))
               if a.kernel in r["Kernel_Name"]]
        if a.ring_batches and prs:
            dmax = max(int(r["Dispatch_Id"]) for r in prs)
            tot = collections.defaultdict(float)
            for r in prs:
                if int(r["Dispatch_Id"]) == dmax:
                    tot[r["Counter_Name"]] += float(r["Counter_Value"])
            for k, v in tot.items():
                counters[k].append(v / a.ring_batches)
            continue
        for r in prs:
            counters[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("== counters (mean per dispatch of %s) ==" % a.kernel)
    pmc = {}
    for k, v in sorted(counters.items()):
        pmc[k] = statistics.mean(v)
        print("%-28s %16.1f  (n=%d)" % (k, pmc[k], len(v)))
    res["pmc"] = pmc
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        fetch = 2.0 * pmc["FETCH_SIZE"] * 1024.0  # gfx950: FETCH_SIZE reads half
        write = pmc["WRITE_SIZE"] * 1024.0
        res["hbm_bytes_per_launch"] = fetch + write
        print("HBM bytes/launch (2*FETCH_SIZE + WRITE_SIZE, KiB->B): %.0f" % (fetch + write))
    if a.per_decode:
        tot = collections.defaultdict(float)
        for p in ("pmc3", "pmc4"):
            for r in rows(os.path.join(a.dir, p, "**", "*counter_collection.csv")):
                if a.per_decode in r["Kernel_Name"]:
                    tot[r["Counter_Name"]] += float(r["Counter_Value"])
        decodes = sum(1 for r in kt if "g_reset" in r["Kernel_Name"] or "ms_init" in r["Kernel_Name"])
        span = collections.defaultdict(float)
        for r in kt:
            if a.per_decode in r["Kernel_Name"]:
                span["ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        nd_pmc = decodes  # each pass re-runs the same bench command
        fetch = 2.0 * tot["FETCH_SIZE"] * 1024.0 / max(1, nd_pmc)
        write = tot["WRITE_SIZE"] * 1024.0 / max(1, nd_pmc)
        res["per_decode"] = {"decodes": decodes, "kernel_ns_per_decode": span["ns"] / max(1, decodes),
                             "fetch_bytes": fetch, "write_bytes": write}
        res["hbm_bytes_per_launch"] = fetch + write
        print("per decode (%d decodes): kernel time %.3f ms, HBM bytes %.4g (fetch %.4g, write %.4g)"
              % (decodes, span["ns"] / max(1, decodes) / 1e6, fetch + write, fetch, write))
    if a.json and a.key:
        try:
            allj = json.load(open(a.json))
        except (OSError, ValueError):
            allj = {}
        if a.source:
            res["source"] = a.source
        allj[a.key] = res
        json.dump(allj, open(a.json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
