"""Parity-check matrices beyond the reference's hard-coded 32x64 H.

The reference decodes one fixed 32x64 code held as dense uBLAS matrices
(lib/ldpc_decoder_cb_impl.cc:60-106).  SURVEY 8(d) config 4 asks for the
same decode on a DVB-S2-size code (N = 64800, K = 32400, E = 226799), which
only fits as a sparse matrix: this module builds such codes as CSR
(M, N, row_ptr, col_idx) for Decoder(csr=...) / ldpc_create_csr.

IRA codes in the DVB-S2 style (ETSI EN 302 307-1, 5.3.2): information bit m
of group g (360 bits per group) is checked by the rows (x + m*q) mod M for
every address x in row g of the code's address table, q = M / 360; the parity
part is the accumulator staircase (p_j = p_{j-1} ^ row j).  The ETSI tables
are not available offline, so dvbs2_like_table() draws a table with the
rate-1/2 normal frame's exact structure -- q = 90, 36 groups of degree 8 and
54 of degree 3, every residue mod q used 5 times, so every check row has
degree 7 (row 0: 6) and E = 226799 -- from a seed.  Results on it are
labelled "DVB-S2-like (synthetic address table)".

Column order: parity bits first (columns 0..M-1), information bits last
(M..N-1), matching the decoder's packed output (info = columns M..N-1, as
the reference's [parity; data] codewords, lib/ldpc_encoder_bc_impl.cc:153-165).
"""
import numpy as np

GROUP = 360


def dvbs2_like_table(seed=0, K=32400, N=64800, hi_groups=36, hi_deg=8, lo_deg=3):
    """Seeded address table with the DVB-S2 rate-1/2 normal-frame profile."""
    M = N - K
    q = M // GROUP
    groups = K // GROUP
    degs = [hi_deg] * hi_groups + [lo_deg] * (groups - hi_groups)
    total = sum(degs)
    if total % q:
        raise ValueError("degree profile does not spread evenly over the q residues")
    rng = np.random.Generator(np.random.PCG64(seed))
    residues = np.repeat(np.arange(q), total // q)
    rng.shuffle(residues)
    table, pos = [], 0
    for d in degs:
        row = set()
        for r in residues[pos:pos + d]:
            while True:
                x = int(r) + q * int(rng.integers(0, M // q))
                if x not in row:
                    row.add(x)
                    break
        table.append(sorted(row))
        pos += d
    return table


def ira_from_table(table, K, N):
    """CSR (M, N, row_ptr, col_idx) of the IRA code of an address table."""
    M = N - K
    if M % GROUP or K % GROUP or len(table) != K // GROUP:
        raise ValueError("K and N-K must be multiples of 360, one table row per 360 info bits")
    q = M // GROUP
    rows, cols = [], []
    m = np.arange(GROUP, dtype=np.int64)
    for g, addrs in enumerate(table):
        for x in addrs:
            rows.append((x + m * q) % M)
            cols.append(M + g * GROUP + m)
    # accumulator: row j holds parity bits j and j-1
    j = np.arange(M, dtype=np.int64)
    rows += [j, j[1:]]
    cols += [j, j[1:] - 1]
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    order = np.lexsort((c, r))
    r, c = r[order], c[order]
    if np.any((r[1:] == r[:-1]) & (c[1:] == c[:-1])):
        raise ValueError("address table places two ones in the same row and column")
    row_ptr = np.zeros(M + 1, np.int64)
    np.add.at(row_ptr, r + 1, 1)
    return M, N, np.cumsum(row_ptr).astype(np.int32), c.astype(np.int32)


def dvbs2_like(seed=0):
    """The config-4 code: N = 64800, K = 32400, E = 226799 (synthetic table)."""
    return ira_from_table(dvbs2_like_table(seed), 32400, 64800)


def ira_encode(csr, info_bits):
    """Systematic IRA encoding: (B, K) info bits -> (B, N) codewords
    [parity | info] with p_j = p_{j-1} ^ (info part of row j)."""
    M, N, row_ptr, col_idx = csr
    info = np.atleast_2d(np.asarray(info_bits, np.uint8)) & 1
    B = info.shape[0]
    # info part of each row = its ones at columns >= M
    rp = np.asarray(row_ptr, np.int64)
    ci = np.asarray(col_idx, np.int64)
    keep = ci >= M
    row_of = np.repeat(np.arange(M), np.diff(rp))[keep]
    s = np.zeros((B, M), np.uint8)
    vals = info[:, ci[keep] - M]
    for b in range(B):
        s[b] = np.bincount(row_of, weights=vals[b], minlength=M).astype(np.int64) & 1
    p = np.bitwise_xor.accumulate(s, axis=1)
    return np.concatenate([p, info], axis=1)


def syndrome_weight(csr, bits):
    """Unsatisfied checks of each (B, N) hard decision (checkFrame, uncapped)."""
    M, N, row_ptr, col_idx = csr
    bits = np.atleast_2d(np.asarray(bits, np.uint8)) & 1
    rp = np.asarray(row_ptr, np.int64)
    row_of = np.repeat(np.arange(M), np.diff(rp))
    out = np.zeros(bits.shape[0], np.int64)
    for b in range(bits.shape[0]):
        par = np.bincount(row_of, weights=bits[b, col_idx], minlength=M).astype(np.int64) & 1
        out[b] = par.sum()
    return out


def alist_text(H=None, csr=None, padded=True):
    """MacKay alist text of a dense H (M, N) or a CSR (M, N, row_ptr, col_idx):
    "N M", the maximum column / row degrees, the degrees, then each column's
    rows and each row's columns (1-based; zero-padded to the maximum degree
    when `padded`)."""
    if H is not None:
        H = np.asarray(H, np.uint8)
        M, N = H.shape
        rows = [np.nonzero(H[j])[0] for j in range(M)]
    else:
        M, N, rp, ci = csr
        rp = np.asarray(rp, np.int64)
        ci = np.asarray(ci, np.int64)
        rows = [np.sort(ci[rp[j]:rp[j + 1]]) for j in range(M)]
    cols = [[] for _ in range(N)]
    for j, r in enumerate(rows):
        for c in r:
            cols[int(c)].append(j)
    dv = [len(c) for c in cols]
    dc = [len(r) for r in rows]
    dvm, dcm = max(dv), max(dc)

    def line(v, width):
        v = [int(x) + 1 for x in v]
        if padded:
            v += [0] * (width - len(v))
        return " ".join(str(x) for x in v)
    out = ["%d %d" % (N, M), "%d %d" % (dvm, dcm), " ".join(map(str, dv)), " ".join(map(str, dc))]
    out += [line(c, dvm) for c in cols]
    out += [line(r, dcm) for r in rows]
    return "\n".join(out) + "\n"


def write_alist(path, H=None, csr=None, padded=True):
    with open(path, "w") as f:
        f.write(alist_text(H=H, csr=csr, padded=padded))


def read_alist(path):
    """(M, N, row_ptr, col_idx) of a MacKay alist file, read by the C ABI's
    ldpc_alist_read (include/ldpc_hip.h)."""
    from ._capi import alist_read
    return alist_read(path)
