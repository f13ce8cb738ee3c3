#!/usr/bin/env python3
"""Writes the alist fixtures tests/golden/hData{1..5}.alist (zero-padded
MacKay format) and hData2_unpadded.alist from the H matrices in
reference_data.npz (the reference's apps/test_data.h codes, stored as data
by make_golden.py).  Data only: no reference source is read here.

    python tests/golden/make_alist.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "gr-ldpc_ece535a_amd"))

from ldpc_ece535a.codes import write_alist  # noqa: E402


def main():
    ref = np.load(os.path.join(HERE, "reference_data.npz"), allow_pickle=False)
    for k in range(1, 6):
        write_alist(os.path.join(HERE, "hData%d.alist" % k), H=ref["hData%d" % k])
    write_alist(os.path.join(HERE, "hData2_unpadded.alist"), H=ref["hData2"], padded=False)


if __name__ == "__main__":
    main()
