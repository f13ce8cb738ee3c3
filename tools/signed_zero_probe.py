"""Mismatch counts vs the oracle on the signed-zero frames of
tests/test_gpu_signed_zero.py, for every (method, precision, launch mode),
with the package build LDPC_PKG_DIR points at (tools/ab.sh A/B runs).
Prints one line per case: frames whose packed bytes / iterations differ."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("LDPC_PKG_DIR", os.path.join(REPO, "gr-ldpc_ece535a_amd")))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import ldpc_ece535a  # noqa: E402
from oracle import oracle as orc  # noqa: E402
import test_gpu_signed_zero as t  # noqa: E402


def main():
    y = t._frames(lambda n: np.load(os.path.join(REPO, "tests", "golden", n), allow_pickle=False))
    for method in (0, 1):
        for prec in (0, 2):
            for mode in (0, 1):
                dec = ldpc_ece535a.Decoder()
                dec.set_launch_mode(mode)
                for iters in (5, 50):
                    out = dec.decode(y, method=method, max_iters=iters, precision=prec)
                    ref = orc.decode_batch(method, dec.H, y, iters, nthreads=8)
                    bad = np.nonzero((out["packed"] != ref["packed"]).any(axis=1))[0]
                    itb = int((out["iters"] != ref["iters"]).sum())
                    print("method %d prec %d mode %d iters %2d: packed %d frames %s, iters %d"
                          % (method, prec, mode, iters, bad.size, bad[:8].tolist(), itb),
                          flush=True)


if __name__ == "__main__":
    main()
