#!/usr/bin/env python3
"""Per-kernel time and counters of one rocprofv3 run directory (as written by
tools/profile_msn.sh): total / mean duration per kernel name from the kernel
trace, and the sum and mean per dispatch of every PMC counter per kernel.

usage: tools/kernel_split.py gpurun_out/prof/msn_2 [--decodes N]
"""
import argparse
import collections
import csv
import glob
import os


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def short(name):
    for pre in ("void ", "ldpc::(anonymous namespace)::", "ldpc::"):
        name = name.replace(pre, "")
    return name.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--decodes", type=int, default=0,
                    help="divide totals by this many decodes (default: dispatches of *_init)")
    ap.add_argument("--update-json", default="",
                    help="write the msn_* kernels' memory traffic per decode into this PMC json "
                         "(key --key) with --pipeline F,C and --source")
    ap.add_argument("--key", default="dvb0_f64_b1024_i50_db2")
    ap.add_argument("--pipeline", default="")
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    kt = rows(os.path.join(a.dir, "kt", "**", "*kernel_trace.csv"))
    dur = collections.defaultdict(list)
    for r in kt:
        dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    nd = a.decodes or max(1, sum(len(v) for k, v in dur.items() if k.endswith("_init")))
    tot = sum(sum(v) for v in dur.values())
    print("decodes: %d, kernel time per decode %.3f ms" % (nd, tot / nd / 1e6))
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print("  %-60s n/decode=%7.1f mean=%9.1f ns  total/decode=%8.3f ms  %5.1f %%"
              % (k, len(v) / nd, sum(v) / len(v), sum(v) / nd / 1e6, 100.0 * sum(v) / tot))
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(int))
    for p in sorted(glob.glob(os.path.join(a.dir, "pmc*"))):
        for r in rows(os.path.join(p, "**", "*counter_collection.csv")):
            k = short(r["Kernel_Name"])
            cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k][r["Counter_Name"]] += 1
    if cnt:
        print("counters (sum per decode; FETCH_SIZE doubled, KiB -> MB):")
    for k in sorted(cnt, key=lambda k: -sum(dur.get(k, [0]))):
        c = cnt[k]
        parts = []
        for name, v in sorted(c.items()):
            v = v / nd
            if name == "FETCH_SIZE":
                parts.append("fetch %.1f MB" % (2 * v * 1024 / 1e6))
            elif name == "WRITE_SIZE":
                parts.append("write %.1f MB" % (v * 1024 / 1e6))
            else:
                parts.append("%s %.4g" % (name, v))
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            h, m = c["TCC_HIT_sum"], c["TCC_MISS_sum"]
            parts.append("L2 hit %.3f" % (h / max(1.0, h + m)))
        print("  %-60s %s" % (k, ", ".join(parts)))
    if a.update_json:
        import json
        fetch = write = kns = 0.0
        for k, c in cnt.items():
            if k.startswith("msn_"):
                fetch += 2 * c.get("FETCH_SIZE", 0.0) * 1024 / nd
                write += c.get("WRITE_SIZE", 0.0) * 1024 / nd
                kns += sum(dur.get(k, [0])) / nd
        f, ch = (int(x) for x in a.pipeline.split(","))
        db = json.load(open(a.update_json))
        db[a.key] = {"hbm_bytes_per_launch": fetch + write,
                     "per_decode": {"decodes": nd, "fetch_bytes": fetch, "write_bytes": write,
                                    "kernel_ns_per_decode": kns},
                     "pipeline": {"frames_per_chunk": f, "chunks": ch},
                     "source": a.source}
        json.dump(db, open(a.update_json, "w"), indent=1)
        print("updated %s[%s]: %.1f GB per decode" % (a.update_json, a.key, (fetch + write) / 1e9))


if __name__ == "__main__":
    main()
