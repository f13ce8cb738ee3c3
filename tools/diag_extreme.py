#!/usr/bin/env python3
"""Diagnostic: which amplitude groups / iterations of the extreme-input
parity test differ between the GPU (precision 0) and the oracle."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gr-ldpc_ece535a_amd")]
import torch  # noqa: F401,E402  (one HIP runtime)
import ldpc_ece535a as L  # noqa: E402
from oracle import oracle as orc  # noqa: E402

fd = np.load(os.path.join(REPO, "tests", "golden", "frames_default.npz"))
base = fd["db2_llr"].astype(np.float64)
amps = (8.0, 30.0, 1e3, 1e10, 1e30, 1e-30, 1e-40)
y = np.concatenate([base[:48] * a for a in amps]).astype(np.float32)
d = L.Decoder()
for it in (1, 2, 3, 4, 6, 10, 30):
    for prec in (0, 2):
        out = d.decode(y, method=1, max_iters=it, precision=prec, want_llr=True)
        ref = orc.decode_batch(1, fd["H_reordered"], y, it, want_post=True)
        bad = (out["bits"] != ref["bits"]).any(axis=1)
        pm = ~((out["llr"] == ref["post"]) | (np.isnan(out["llr"]) & np.isnan(ref["post"])))
        print("iters %2d prec %d: frames with different bits per amplitude %s; posterior "
              "mismatching frames %s" % (it, prec, [int(bad[48 * g:48 * g + 48].sum()) for g in range(len(amps))],
                                         [int(pm[48 * g:48 * g + 48].any(axis=1).sum()) for g in range(len(amps))]))
        if prec == 0 and pm.any():
            b = int(np.where(pm.any(axis=1))[0][0])
            c = np.where(pm[b])[0][:4]
            print("   frame", b, "cols", c.tolist(), "gpu", out["llr"][b, c].tolist(), "ref", ref["post"][b, c].tolist())
