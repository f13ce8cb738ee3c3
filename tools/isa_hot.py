#!/usr/bin/env python3
"""VALU issue mix of a kernel's iteration loop, hot path only, from a
`hipcc --cuda-device-only -S` listing.

Regions the wave enters only for rare lanes (bodies of branches whose first
instructions carry the ;ldpc_cold marker that LDPC_EX_COLD() emits, see
csrc/ldpc_exact.hpp) are skipped.  Each instruction is weighted by its
measured issue cost on gfx950 (tools/ubench_valu.hip, tools/ubench_f64.hip,
profiles/round3/ubench_valu.txt, 4 waves per SIMD): 4.31 cycles for f64
add/mul/fma and for any VOP3-encoded or 64-bit instruction (compares, e64
selects, 64-bit moves and shifts, converts, min/max), 2.75 for VOP1/VOP2
32-bit ones, 16.3 for v_rcp_f64.  Prints the per-iteration totals and the
mean weight of the instructions the PMC counts as "other VALU" (everything
but SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64), which bench.py's roofline uses.

usage: tools/isa_hot.py <file.s> <kernel-regex> [--loop-rank K] [--json out --key K]
"""
import argparse
import collections
import json
import re

W_F64, W_VOP3, W_VOP2, W_TRANS = 4.31, 4.31, 2.75, 16.3


def weight(op):
    if "rcp_f64" in op or "rsq_f64" in op or "sqrt_f64" in op:
        return W_TRANS
    if "f64" in op or "_e64" in op or "b64" in op or "u64" in op or "i64" in op:
        return W_VOP3
    if op.startswith(("v_mad", "v_fma", "v_lshl_add", "v_add3", "v_and_or", "v_or3", "v_xor3",
                      "v_bfe", "v_bfi", "v_alignbit", "v_perm", "v_mbcnt", "v_readlane",
                      "v_writelane", "v_cndmask_b32_e64", "v_med3", "v_min3", "v_max3",
                      "v_lshl_or", "v_ldexp")):
        return W_VOP3
    return W_VOP2


def pmc_class(op):
    for k in ("add_f64", "mul_f64", "fma_f64", "fmac_f64"):
        if op.startswith("v_" + k):
            return "f64"
    if "rcp_f64" in op:
        return "trans"
    return "other"


def loops(lines):
    labels = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            labels[m.group(1)] = i
    out = []
    for i, l in enumerate(lines):
        m = re.match(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            out.append((labels[m.group(1)], i))
    return out


def hot_path(lines, full=False):
    hot, i = [], 0
    while i < len(lines):
        l = lines[i]
        m = re.match(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)", l)
        if m:
            tgt = m.group(1) + ":"
            # cold: the marker sits in the first basic block the branch skips
            # (the compiler may schedule instructions of that block ahead of
            # it, but not move it into another block)
            cold, j = False, i + 1
            while j < len(lines) and not re.match(r"^\.LBB\d+_\d+:", lines[j]):
                if "ldpc_cold" in lines[j]:
                    cold = True
                    break
                j += 1
            if cold:
                k = i + 1
                while k < len(lines) and not lines[k].startswith(tgt):
                    k += 1
                i = k
                continue
        hot.append(l)
        i += 1
    keep = [l for l in hot if l and not l.startswith((".", ";")) and not re.match(r"^\S+:", l)]
    return keep if full else [l.split()[0] for l in keep]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--loop-rank", type=int, default=0,
                    help="0: the loop with the most VALU that is not the frame loop")
    ap.add_argument("--json", default=None)
    ap.add_argument("--key", default=None)
    ap.add_argument("--dump", default=None, help="write the hot path's instructions here")
    a = ap.parse_args()
    s = open(a.asm).read()
    m = re.search(r"^(\S*%s\S*):" % a.kernel, s, re.M)
    body = s[m.end():s.index(".Lfunc_end", m.end())]
    lines = [l.strip() for l in body.split("\n")]
    cand = []
    for lo, hi in loops(lines):
        ins = hot_path(lines[lo:hi])
        cand.append((sum(1 for x in ins if x.startswith("v_")), lo, hi, ins))
    # the iteration loops are the ones nested in the frame loop: skip loops
    # that contain another loop of real size (>= 100 VALU)
    inner = [c for c in cand
             if not any(o[1] >= c[1] and o[2] <= c[2] and o != c and o[0] >= 100
                        for o in cand)]
    inner.sort(key=lambda c: -c[0])
    n, lo, hi, ins = inner[min(a.loop_rank, len(inner) - 1)]
    if a.dump:
        open(a.dump, "w").write("\n".join(hot_path(lines[lo:hi], full=True)) + "\n")
    c = collections.Counter(x for x in ins if x.startswith("v_"))
    cyc = {"f64": 0.0, "trans": 0.0, "other": 0.0}
    cnt = {"f64": 0, "trans": 0, "other": 0}
    for op, k in c.items():
        cl = pmc_class(op)
        cyc[cl] += k * weight(op)
        cnt[cl] += k
    total = sum(cyc.values())
    w_other = cyc["other"] / max(1, cnt["other"])
    print("%s lines %d-%d: hot-path VALU %d (f64 add/mul/fma %d, trans %d, other %d), "
          "%.0f issue cycles per iteration; mean 'other' weight %.3f"
          % (m.group(1)[:60], lo, hi, n, cnt["f64"], cnt["trans"], cnt["other"], total, w_other))
    for op, k in sorted(c.items(), key=lambda kv: -kv[1] * weight(kv[0]))[:25]:
        print("  %4d x %-26s %6.0f cycles" % (k, op, k * weight(op)))
    if a.json and a.key:
        try:
            allj = json.load(open(a.json))
        except (OSError, ValueError):
            allj = {}
        e = allj.setdefault(a.key, {})
        e["isa_hot"] = {"valu": n, "f64": cnt["f64"], "trans": cnt["trans"], "other": cnt["other"],
                        "issue_cycles_per_iteration": round(total, 1),
                        "other_weight": round(w_other, 3),
                        "weights": "f64 add/mul/fma and VOP3/64-bit %g, VOP1/VOP2 %g, v_rcp_f64 %g"
                                   % (W_F64, W_VOP2, W_TRANS)}
        json.dump(allj, open(a.json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
