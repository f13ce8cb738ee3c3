#!/usr/bin/env python3
"""Prints the headline numbers of a bench.py JSON line (file argument)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"])
t = d["timing"]
print("span/batch", t["device_span_ms_per_launch"], "ring", t.get("frame_ring"))
r = d["roofline"]
print("roofline", {k: r.get(k) for k in ("achieved", "frac", "frac_nominal", "f64_tflops")})
print("parity", d.get("parity"))
print("serial", d.get("serial_1_batch_in_flight"))
v = d.get("variants_1gpu", {})
for k in v:
    if k.startswith("config") or k.startswith("block"):
        continue
    print(" ", k, v[k])
if "config4" in v:
    c = v["config4"]["min-sum f64"]
    print("config4", c.get("Mbit/s"), c.get("measured_MB_per_frame_iteration"), c.get("parity"))
for k, x in v.get("block general_work (host buffers)", {}).items():
    print("block", k, x["Mbit/s"], x["windows_per_output_frame"])
