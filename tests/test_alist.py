"""Runtime H source: MacKay alist files read by the C
ABI's ldpc_alist_read (include/ldpc_hip.h), host only.  The fixtures
tests/golden/hData*.alist hold the reference's apps/test_data.h matrices
(written by tests/golden/make_alist.py from reference_data.npz)."""
import os

import numpy as np
import pytest

from ldpc_ece535a import LdpcError, codes

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _dense(M, N, rp, ci):
    H = np.zeros((M, N), np.uint8)
    for j in range(M):
        H[j, ci[rp[j]:rp[j + 1]]] = 1
    return H


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5])
def test_reference_codes_from_alist(golden, k):
    ref = golden("reference_data.npz")["hData%d" % k]
    M, N, rp, ci = codes.read_alist(os.path.join(GOLDEN, "hData%d.alist" % k))
    assert (M, N) == ref.shape
    assert (_dense(M, N, rp, ci) == ref).all()


def test_unpadded_alist(golden):
    a = codes.read_alist(os.path.join(GOLDEN, "hData2.alist"))
    b = codes.read_alist(os.path.join(GOLDEN, "hData2_unpadded.alist"))
    assert a[:2] == b[:2] and (a[2] == b[2]).all() and (a[3] == b[3]).all()


def test_default_h_alist_roundtrip(tmp_path):
    import ldpc_ece535a as L
    H = L.default_h()
    p = str(tmp_path / "default.alist")
    codes.write_alist(p, H=H)
    M, N, rp, ci = codes.read_alist(p)
    assert (_dense(M, N, rp, ci) == H).all()


def test_dvbs2_like_alist_roundtrip(tmp_path):
    csr = codes.dvbs2_like(0)
    p = str(tmp_path / "dvb.alist")
    codes.write_alist(p, csr=csr)
    M, N, rp, ci = codes.read_alist(p)
    assert (M, N) == (csr[0], csr[1])
    assert (rp == csr[2]).all() and (ci == csr[3]).all()


@pytest.mark.parametrize("mutate", ["truncate", "bad_row", "disagree", "degree", "text",
                                    "padding", "missing"])
def test_malformed_alist_rejected(tmp_path, golden, mutate):
    txt = codes.alist_text(H=golden("reference_data.npz")["hData3"])
    lines = txt.splitlines()
    if mutate == "truncate":
        lines = lines[:-2]
    elif mutate == "bad_row":
        lines[4] = "99 0 0"
    elif mutate == "disagree":  # column 1 lists row 2 instead of its own row
        lines[4] = "2 0 0" if lines[4].split()[0] != "2" else "3 0 0"
    elif mutate == "degree":
        lines[2] = "9 " + lines[2].split(" ", 1)[1]
    elif mutate == "text":
        lines[5] = "x y z"
    elif mutate == "padding":
        lines[4] = lines[4].split()[0] + " 7 0"
    elif mutate == "missing":
        lines = []
    p = str(tmp_path / "bad.alist")
    open(p, "w").write("\n".join(lines) + "\n")
    with pytest.raises(LdpcError):
        codes.read_alist(p)
    with pytest.raises(LdpcError):
        codes.read_alist(str(tmp_path / "does_not_exist.alist"))
