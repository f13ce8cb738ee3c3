"""Host logic of the large-code min-sum pipeline's storage order
(ldpc_plan_storage_order, the choice ldpc_create_csr makes; no GPU).

For codes with the DVB-S2 structure (row r = x + s q mod M, q = M / 360) rows
are stored by residue class, r -> (r mod q) * 360 + r / q, and the
staircase's degree-2 columns move among their own positions in that order;
the order is taken only when it gives the kernels' gathers more contiguity.
Any order is correct -- the kernels visit edges in the reference's order
regardless -- so these tests pin the choice and that it is a permutation
(DESIGN §5)."""
import os

import numpy as np

import ldpc_ece535a as L
from ldpc_ece535a import codes


def _perm(a, n):
    return np.array_equal(np.sort(a), np.arange(n))


def test_dvbs2_like_residue_order():
    csr = codes.dvbs2_like(0)
    M, N, rp, ci = csr
    r = L._capi.plan_storage_order(csr)
    assert r["order"] == 1
    s_id, s_qc = r["score"]
    assert s_qc > 3 * s_id > 0
    q = M // 360
    j = np.arange(M)
    assert np.array_equal(r["rpos"], (j % q) * 360 + j // q)
    assert _perm(r["rpos"], M) and _perm(r["cpos"], N)
    # information columns (parity first in codes.py) stay in place; the
    # staircase columns (rows c, c+1) are ordered by their first row's class position
    assert np.array_equal(r["cpos"][M:], np.arange(M, N))
    stair = np.argsort(r["cpos"][:M])
    assert np.all(np.diff(r["rpos"][stair]) > 0)


def test_info_first_column_order():
    """ETSI order ([info | parity]): the same rows, the staircase columns are
    found wherever they are and moved only among their own positions."""
    M, N, rp, ci = codes.dvbs2_like(0)
    K = N - M
    newcol = np.where(ci >= M, ci - M, ci + K).astype(np.int64)  # parity -> K.., info -> 0..
    rows = np.repeat(np.arange(M), np.diff(rp))
    order = np.lexsort((newcol, rows))
    csr2 = (M, N, rp, newcol[order].astype(np.int32))
    r = L._capi.plan_storage_order(csr2)
    assert r["order"] == 1
    assert np.array_equal(r["cpos"][:K], np.arange(K))
    assert _perm(r["cpos"][K:] - K, M)


def test_identity_when_not_quasi_cyclic():
    from oracle import oracle as orc
    Hr, _ = L._capi.reorder_h(L._capi.default_h())
    rp, ci = orc.dense_to_csr(Hr)
    csr = (Hr.shape[0], Hr.shape[1], rp, ci)
    r = L._capi.plan_storage_order(csr)
    assert r["order"] == 0 and r["score"][1] == -1
    assert np.array_equal(r["rpos"], np.arange(csr[0]))
    assert np.array_equal(r["cpos"], np.arange(csr[1]))


def test_forced_identity():
    csr = codes.dvbs2_like(0)
    old = os.environ.get("LDPC_MSN_ORDER")
    os.environ["LDPC_MSN_ORDER"] = "0"
    try:
        r = L._capi.plan_storage_order(csr)
    finally:
        if old is None:
            del os.environ["LDPC_MSN_ORDER"]
        else:
            os.environ["LDPC_MSN_ORDER"] = old
    assert r["order"] == 0
    assert np.array_equal(r["rpos"], np.arange(csr[0]))


def test_edge_descriptor_self_check_high_degree_codes():
    """The edge tables are run-length descriptors per (wave, slot)
    (ldpc_graph.hpp MsnDesc) built with a host self-check that decodes every
    entry the way the kernels do and throws on a mismatch; plan_storage_order
    runs that build.  Codes with row degrees 6-20 and column degrees 1-12,
    in both storage orders."""
    for hg, hd in ((3, 8), (5, 12)):
        csr = codes.ira_from_table(codes.dvbs2_like_table(3, K=5400, N=7200, hi_groups=hg,
                                                          hi_deg=hd, lo_deg=3), 5400, 7200)
        for force in ("0", "1"):
            os.environ["LDPC_MSN_ORDER"] = force
            try:
                assert L._capi.plan_storage_order(csr)["order"] == int(force)
            finally:
                del os.environ["LDPC_MSN_ORDER"]
