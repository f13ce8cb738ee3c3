"""The small-code kernel's LDS layout (csrc/ldpc_layout.hpp), host only.

plan_layout places every edge in a lane slot ("cell") and every column at a
lane position so the kernel's LDS gathers and scatters are free of bank
conflicts.  The layout must be a valid placement (distinct cells, a column
permutation), must never model worse than the plain CSR layout, and must
reach zero modelled conflicts on the reference's default H.  The model itself
is re-derived here, independently, from the bank rules of
cdna_hip_programming.md §2 (ds_read_b64: two 32-lane groups, bank pair =
element mod 32; ds_write_b64: four 16-lane groups, element mod 16) and the
kernel's access lists (ldpc_kernels.hip decode_frame)."""
import numpy as np
import pytest

import ldpc_ece535a as L


def kernel_shape(M, N, E, dc, dv):
    S = (E + 63) // 64
    NW = 1 if N <= 64 else 4
    low = NW == 1 and dc <= 6 and dv <= 3 and S <= 4
    dcn, dvn = (5, 3) if low else (7, 4)
    return S, NW, dcn, dvn, NW == 1 and dvn <= S


def slice_layout(S, NW):
    tb, tbd = 0, 64 * S
    eb = tbd + 32
    ebd = eb + 64 * S
    rb = ebd + 32
    sb = rb + 64 * NW
    nr = sb + 64 * NW
    jk = nr + 64 * (S + NW)
    return dict(tb=tb, tbd=tbd, eb=eb, ebd=ebd, rb=rb, sb=sb, nr=nr, jk=jk)


def group_cost(addrs, mod):
    u = sorted(set(a for a in addrs if a >= 0))
    if not u:
        return 0
    return int(np.bincount(np.array(u) % mod).max()) - 1


def read_cost(a):
    return group_cost(a[:32], 32) + group_cost(a[32:], 32)


def write_cost(a):
    return sum(group_cost(a[g:g + 16], 16) for g in range(0, 64, 16))


def model(Hr, cell, pos, cols):
    """Extra LDS cycles per iteration; identity cells chosen per group as
    the kernel's planner does (the cheapest of the 32)."""
    M, N = Hr.shape
    erow, ecol = np.nonzero(Hr)
    E = len(erow)
    S, NW, dcn, dvn, _ = kernel_shape(M, N, E, Hr.sum(1).max(), Hr.sum(0).max())
    Ls = slice_layout(S, NW)
    rows = [list(np.nonzero(erow == j)[0]) for j in range(M)]
    cole = [list(np.nonzero(ecol == i)[0]) for i in range(N)]
    nbr = [[n for n in rows[erow[e]] if n != e] for e in range(E)]
    edge_at = -np.ones(64 * S, int)
    edge_at[cell] = np.arange(E)
    col_at = -np.ones(64 * NW, int)
    col_at[pos] = np.arange(N)
    cost = 0
    for g in range(2 * S):
        best = None
        for r in range(32):
            c = 0
            for k in range(dcn):
                a = []
                for l in range(32):
                    e = edge_at[32 * g + l]
                    if e < 0:  # padding cell: reads a zero cell (T = 0)
                        a.append(Ls["ebd"] + l)
                    else:
                        a.append(Ls["tb"] + cell[nbr[e][k]] if k < len(nbr[e]) else Ls["tbd"] + r)
                c += group_cost(a, 32)
            best = c if best is None else min(best, c)
        cost += best
    for q in range(NW):
        for k in range(dvn):
            a, w = [], []
            for l in range(64):
                p = 64 * q + l
                c = col_at[p]
                has = c >= 0 and k < len(cole[c])
                if cols:
                    a.append(Ls["eb"] + cell[cole[c][k]] if has else Ls["nr"] + p)
                    w.append(Ls["tb"] + cell[cole[c][k]] if has else Ls["jk"] + p)
                else:
                    a.append(Ls["eb"] + cell[cole[c][k]] if has else Ls["ebd"] + (l & 31))
            cost += read_cost(a)
            if cols:
                cost += write_cost(w)
    if not cols:
        for s in range(S):
            a = [Ls["sb"] + (pos[ecol[edge_at[64 * s + l]]] if edge_at[64 * s + l] >= 0 else l)
                 for l in range(64)]
            cost += read_cost(a)
    return cost


def random_code(rng, M, N, dv):
    """Random H with dv ones per column and near-equal row degrees (each
    column takes the dv least-used rows, ties broken at random)."""
    H = np.zeros((M, N), np.uint8)
    deg = np.zeros(M)
    for i in range(N):
        rows = np.lexsort((rng.random(M), deg))[:dv]
        H[rows, i] = 1
        deg[rows] += 1
    return H


def codes(golden):
    ref = golden("reference_data.npz")
    out = [("default", ref["decoder_h"]), ("qa_h", ref["qa_h"])]
    out += [(n, ref[n]) for n in ("hData1", "hData2", "hData3", "hData4", "hData5")]
    rng = np.random.default_rng(7)
    out += [("rand96x192", random_code(rng, 96, 192, 2)), ("rand64x128", random_code(rng, 64, 128, 3))]
    return out


def test_layout_is_a_placement_and_never_worse(golden):
    for name, H in codes(golden):
        Hr, _ = L.reorder_h(H)
        M, N = Hr.shape
        lay = L.plan_layout(H)
        cell, pos, m = lay["cell"], lay["pos"], lay["model"]
        E = int(Hr.sum())
        S = (E + 63) // 64
        NW = 1 if N <= 64 else 4
        assert len(cell) == E and len(set(cell.tolist())) == E, name
        assert cell.min() >= 0 and cell.max() < 64 * S, name
        assert sorted(pos.tolist()) == list(range(N)), name  # positions 0..N-1: the columns
        assert m["cc"] + m["ec"] <= m["plain_cc"] + m["plain_ec"], (name, m)
        plain = L.plan_layout(H, plain=True)
        assert (plain["cell"] == np.arange(E)).all() and (plain["pos"] == np.arange(N)).all()
        assert plain["model"]["searched"] == 0
        assert NW * 64 >= N


def test_default_h_layout_is_conflict_free(golden):
    lay = L.plan_layout(golden("reference_data.npz")["decoder_h"])
    m = lay["model"]
    assert m["searched"] == 1 and m["cc"] == 0 and m["ec"] == 0, m
    assert m["plain_cc"] > 40 and m["plain_ec"] > 20, m  # the CSR layout it replaces


@pytest.mark.parametrize("name", ["default", "hData4", "hData5", "hData2", "rand64x128"])
def test_model_matches_independent_restatement(golden, name):
    H = dict(codes(golden))[name]
    Hr, _ = L.reorder_h(H)
    M, N = Hr.shape
    E = int(Hr.sum())
    cols = kernel_shape(M, N, E, Hr.sum(1).max(), Hr.sum(0).max())[4]
    for plain in (False, True):
        lay = L.plan_layout(H, plain=plain)
        m = lay["model"]
        ec = model(Hr, lay["cell"], lay["pos"], False)
        key = "plain_" if plain or not m["searched"] else ""
        assert ec == m[key + "ec"], (name, plain, ec, m)
        if cols:
            assert model(Hr, lay["cell"], lay["pos"], True) == m[key + "cc"], (name, plain, m)
