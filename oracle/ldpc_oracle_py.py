"""Pure-Python restatement of the reference decode path (TEST INFRASTRUCTURE ONLY).

A second, independent restatement of lib/ldpc_decoder_cb_impl.cc
(ericdegroot/gr-ldpc_ece535a) used to cross-check the C oracle
(oracle/ldpc_oracle.c) bit for bit.  It walks adjacency lists instead of the
dense M x N scans, keeping the reference's visiting order (ascending column
inside a row, ascending row inside a column), so every floating-point result
is formed by the same operations in the same order.  `math.tanh`/`math.log`
call the C library's tanh/log, exactly as std::tanh/std::log do.

Only for small cases (tests); never imported by the product.
"""
import math

DBL_MAX = 1.7976931348623157e308


def reorder_h(H):
    """reorderHMatrix, lib/ldpc_decoder_cb_impl.cc:255-307.

    H: list of M lists of N ints (0/1).  Returns (Hr, chosen, L, U); Hr is a new
    matrix with the reference's column swaps applied.
    """
    M, N = len(H), len(H[0])
    K = N - M
    F = [row[:] for row in H]
    Hr = [row[:] for row in H]
    L = [[0] * K for _ in range(M)]
    U = [[0] * K for _ in range(M)]
    chosen = []
    for i in range(M):
        pick = 0
        for j in range(i, N):
            if F[i][j] != 0:
                pick = j
                break
        chosen.append(pick)
        for A in (F, Hr):
            for r in range(M):
                A[r][i], A[r][pick] = A[r][pick], A[r][i]
        if i < K:
            for r in range(i, M):
                L[r][i] = F[r][i]
            for r in range(0, i + 1):
                U[r][i] = F[r][i]
        if i < M - 1:
            for k in range(i + 1, M):
                if F[k][i] != 0:
                    F[k] = [(a + b) % 2 for a, b in zip(F[k], F[i])]
    return Hr, chosen, L, U


def check_frame(H, u, threshold):
    """checkFrame, :236-253."""
    bad = 0
    for row in H:
        if sum(a * b for a, b in zip(u, row)) % 2 != 0:
            bad += 1
        if bad > threshold:
            break
    return bad


class _Graph:
    def __init__(self, H):
        self.M, self.N = len(H), len(H[0])
        self.rows = [[c for c in range(self.N) if H[r][c]] for r in range(self.M)]
        self.cols = [[r for r in range(self.M) if H[r][c]] for c in range(self.N)]


def decode_hard(rx):
    """decodeHard, :559-572."""
    return [0 if x < 0 else 1 for x in rx], 0


def decode_bitflip(H, rx, iterations, et_period=1):
    """decodeBitFlipping, :414-476 (E(i,j) for edges = parity of the other
    row members)."""
    g = _Graph(H)
    y = [0 if x < 0.0 else 1 for x in rx]
    ci = y[:]
    used = iterations
    half = g.M // 2
    for it in range(iterations):
        E = {}
        for r in range(g.M):
            for c in g.rows[r]:
                E[(r, c)] = sum(ci[k] for k in g.rows[r] if k != c) % 2
        for c in range(g.N):
            votes = sum(1 for r in g.cols[c] if E[(r, c)] != y[c])
            if votes > half:
                ci[c] = (y[c] + 1) % 2
        if it + 1 < iterations and (it + 1) % et_period == 0 and check_frame(H, ci, 0) == 0:
            used = it + 1
            break
    return ci, used


def _sign(v):
    return (v > 0) - (v < 0)


def decode_minsum(H, rx, iterations, et_period=1):
    """decodeLogDomainSimple, :309-412."""
    g = _Graph(H)
    Lci = [-x for x in rx]
    Lq = {(r, c): Lci[c] for r in range(g.M) for c in g.rows[r]}
    Lr = {}
    vhat = [0] * g.N
    used = iterations
    for it in range(iterations):
        for r in range(g.M):
            sgn = 1
            for c in g.rows[r]:
                sgn *= _sign(Lq[(r, c)])
            for c in g.rows[r]:
                lo = DBL_MAX
                for k in g.rows[r]:
                    if k != c and abs(Lq[(r, k)]) < lo:
                        lo = abs(Lq[(r, k)])
                Lr[(r, c)] = float(sgn * _sign(Lq[(r, c)])) * lo
        for c in range(g.N):
            s = 0.0
            for r in g.cols[c]:
                s += Lr[(r, c)]
            for r in g.cols[c]:
                Lq[(r, c)] = Lci[c] + s - Lr[(r, c)]
            vhat[c] = 1 if (Lci[c] + s) < 0 else 0
        if it + 1 < iterations and (it + 1) % et_period == 0 and check_frame(H, vhat, 0) == 0:
            used = it + 1
            break
    return vhat, used


def decode_sumproduct(H, rx, iterations, et_period=1):
    """decodeSumProductSoft, :478-557."""
    g = _Graph(H)
    r_ = [-x for x in rx]
    Q = {(j, i): r_[i] for j in range(g.M) for i in g.rows[j]}
    E = {}
    vhat = [0] * g.N
    used = iterations
    for it in range(iterations):
        for j in range(g.M):
            for i in g.rows[j]:
                T = 1.0
                for k in g.rows[j]:
                    if k != i:
                        T *= math.tanh(Q[(j, k)] / 2.0)
                # log((1+T)/(1-T)) with the reference's inf/nan behaviour
                num, den = 1.0 + T, 1.0 - T
                if den == 0.0:
                    q = math.copysign(math.inf, num) if num != 0.0 else math.nan
                else:
                    q = num / den
                if q == 0.0:
                    E[(j, i)] = -math.inf
                elif q < 0.0 or q != q:
                    E[(j, i)] = math.nan
                elif q == math.inf:
                    E[(j, i)] = math.inf
                else:
                    E[(j, i)] = math.log(q)
        for i in range(g.N):
            L = 0.0
            for j in g.cols[i]:
                L += E[(j, i)] + r_[i]
            vhat[i] = 1 if L <= 0 else 0
        if (it + 1) % et_period == 0 and check_frame(H, vhat, 0) == 0:
            used = it + 1
            break
        for j in range(g.M):
            for i in g.rows[j]:
                T = 0.0
                for k in g.cols[i]:
                    if k != j:
                        T += E[(k, i)] + r_[i]
                Q[(j, i)] = T
    return vhat, used


def decode(method, H, rx, iterations, et_period=1):
    """general_work's dispatch, :155-164.  et_period > 1 thins the early-exit
    test to iterations it with (it + 1) % et_period == 0 (SURVEY 8(d) config 5;
    1 = the reference)."""
    if method == 3:
        return decode_hard(rx)
    if method == 2:
        return decode_bitflip(H, rx, iterations, et_period)
    if method == 1:
        return decode_sumproduct(H, rx, iterations, et_period)
    return decode_minsum(H, rx, iterations, et_period)
