"""ctypes wrapper around oracle/libldpc_oracle.so (TEST INFRASTRUCTURE ONLY).

Used by tests/, __graft_entry__.smoke() (as the checker) and bench.py's
cpu_baseline leg.  The product (gr-ldpc_ece535a_amd/) never imports this.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libldpc_oracle.so")
_lib = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i32p = ctypes.POINTER(ctypes.c_int32)
_f32p = ctypes.POINTER(ctypes.c_float)
_f64p = ctypes.POINTER(ctypes.c_double)


def build():
    """Compile the oracle in place (gcc; host only)."""
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_reorder_h.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, _i32p, _u8p, _u8p]
        L.orc_reorder_h.restype = None
        L.orc_check_frame.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, _i32p, ctypes.c_int]
        L.orc_check_frame.restype = ctypes.c_int
        L.orc_encode.argtypes = [_u8p, _u8p, _u8p, ctypes.c_int, ctypes.c_int, _i32p, _i32p]
        L.orc_encode.restype = ctypes.c_int
        L.orc_decode.argtypes = [ctypes.c_int, _u8p, ctypes.c_int, ctypes.c_int, _f64p,
                                 ctypes.c_int, _i32p, _f64p]
        L.orc_decode.restype = ctypes.c_int
        L.orc_decode_batch.argtypes = [ctypes.c_int, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       _f32p, ctypes.c_long, ctypes.c_int, ctypes.c_float,
                                       ctypes.c_int, _u8p, _u8p, _i32p, _i32p, _f32p, ctypes.c_int]
        L.orc_decode_batch.restype = ctypes.c_int
        L.orc_decode_batch_et.argtypes = [ctypes.c_int, _u8p, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, _f32p, ctypes.c_long,
                                          ctypes.c_int, ctypes.c_float, ctypes.c_int, _u8p, _u8p,
                                          _i32p, _i32p, _f32p, ctypes.c_int]
        L.orc_decode_batch_et.restype = ctypes.c_int
        L.orc_decode_batch_sparse_et.argtypes = [ctypes.c_int, _i32p, _i32p, ctypes.c_int,
                                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p,
                                                 ctypes.c_long, ctypes.c_int, ctypes.c_float,
                                                 ctypes.c_int, _u8p, _u8p, _i32p, _i32p,
                                                 ctypes.c_int]
        L.orc_decode_batch_sparse_et.restype = ctypes.c_int
        L.orc_decode_batch_sparse.argtypes = [ctypes.c_int, _i32p, _i32p, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, _f32p, ctypes.c_long,
                                              ctypes.c_int, ctypes.c_float, ctypes.c_int, _u8p,
                                              _u8p, _i32p, _i32p, ctypes.c_int]
        L.orc_decode_batch_sparse.restype = ctypes.c_int
        L.orc_block_init.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, _u8p,
                                     ctypes.c_int, ctypes.c_int]
        L.orc_block_init.restype = None
        L.orc_block_general_work.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, _f32p,
                                             _u8p, _i32p]
        L.orc_block_general_work.restype = ctypes.c_int
        L.orc_block_general_work_sparse.argtypes = [ctypes.c_void_p, _i32p, _i32p, ctypes.c_int,
                                                    ctypes.c_int, _f32p, _u8p, _i32p]
        L.orc_block_general_work_sparse.restype = ctypes.c_int
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def reorder_h(H):
    """Returns (Hr, chosen, L, U) like reorderHMatrix (+ encoder L/U)."""
    H = np.ascontiguousarray(H, dtype=np.uint8).copy()
    M, N = H.shape
    chosen = np.zeros(M, np.int32)
    K = N - M
    L = np.zeros((M, K), np.uint8)
    U = np.zeros((M, K), np.uint8)
    lib().orc_reorder_h(_p(H, _u8p), M, N, _p(chosen, _i32p), _p(L, _u8p), _p(U, _u8p))
    return H, chosen, L, U


def check_frame(Hr, bits, threshold):
    Hr = np.ascontiguousarray(Hr, dtype=np.uint8)
    u = np.ascontiguousarray(bits, dtype=np.int32)
    M, N = Hr.shape
    return lib().orc_check_frame(_p(Hr, _u8p), M, N, _p(u, _i32p), int(threshold))


def encode(Hr, L, U, data_bits):
    """makeParityCheck for a batch: data_bits (B, N-M) -> codewords (B, N) as
    [parity; data] (lib/ldpc_encoder_bc_impl.cc:151-165)."""
    Hr = np.ascontiguousarray(Hr, np.uint8)
    L = np.ascontiguousarray(L, np.uint8)
    U = np.ascontiguousarray(U, np.uint8)
    M, N = Hr.shape
    d = np.ascontiguousarray(np.atleast_2d(data_bits), np.int32)
    out = np.zeros((d.shape[0], N), np.uint8)
    par = np.zeros(M, np.int32)
    for b in range(d.shape[0]):
        row = np.ascontiguousarray(d[b])
        rc = lib().orc_encode(_p(Hr, _u8p), _p(L, _u8p), _p(U, _u8p), M, N,
                              _p(row, _i32p), _p(par, _i32p))
        if rc != 0:
            raise ValueError("singular triangular factor")
        out[b, :M] = par
        out[b, M:] = d[b]
    return out


def decode_one(method, Hr, rx, iterations):
    Hr = np.ascontiguousarray(Hr, np.uint8)
    M, N = Hr.shape
    rx = np.ascontiguousarray(rx, np.float64)
    v = np.zeros(N, np.int32)
    post = np.zeros(N, np.float64)
    used = lib().orc_decode(int(method), _p(Hr, _u8p), M, N, _p(rx, _f64p), int(iterations),
                            _p(v, _i32p), _p(post, _f64p))
    return v, used, post


def decode_batch(method, Hr, llr, iterations, polarity=1.0, nthreads=1, cw_stride=None,
                 elem_stride=1, B=None, want_post=False, et_period=1):
    """Decode B frames of float32 samples.  Returns dict with bits (B,N) u8,
    packed (B,KB) u8, iters (B,) i32, synd (B,) i32 [, post (B,N) f32].
    et_period > 1 thins the early-exit test (orc_decode_et; 1 = reference)."""
    Hr = np.ascontiguousarray(Hr, np.uint8)
    M, N = Hr.shape
    llr = np.ascontiguousarray(llr, np.float32)
    if cw_stride is None:
        cw_stride = N * elem_stride
    if B is None:
        B = llr.size // cw_stride if llr.ndim == 1 else llr.shape[0]
    KB = (N - M + 7) // 8
    bits = np.zeros((B, N), np.uint8)
    packed = np.zeros((B, KB), np.uint8)
    iters = np.zeros(B, np.int32)
    synd = np.zeros(B, np.int32)
    post = np.zeros((B, N), np.float32) if want_post else None
    lib().orc_decode_batch_et(int(method), _p(Hr, _u8p), M, N, int(iterations), int(et_period),
                              _p(llr, _f32p), int(cw_stride), int(elem_stride), float(polarity),
                              int(B), _p(bits, _u8p), _p(packed, _u8p), _p(iters, _i32p),
                              _p(synd, _i32p), _p(post, _f32p), int(nthreads))
    out = dict(bits=bits, packed=packed, iters=iters, synd=synd)
    if want_post:
        out["post"] = post
    return out


def decode_batch_sparse(method, row_ptr, col_idx, M, N, llr, iterations, polarity=1.0,
                        nthreads=1, cw_stride=None, elem_stride=1, B=None, want_bits=True,
                        et_period=1):
    """Sparse (CSR) restatement for large codes; same outputs as decode_batch."""
    rp = np.ascontiguousarray(row_ptr, np.int32)
    ci = np.ascontiguousarray(col_idx, np.int32)
    llr = np.ascontiguousarray(llr, np.float32)
    if cw_stride is None:
        cw_stride = N * elem_stride
    if B is None:
        B = llr.size // cw_stride if llr.ndim == 1 else llr.shape[0]
    KB = (N - M + 7) // 8
    bits = np.zeros((B, N), np.uint8) if want_bits else None
    packed = np.zeros((B, KB), np.uint8)
    iters = np.zeros(B, np.int32)
    synd = np.zeros(B, np.int32)
    lib().orc_decode_batch_sparse_et(int(method), _p(rp, _i32p), _p(ci, _i32p), int(M), int(N),
                                     int(iterations), int(et_period), _p(llr, _f32p),
                                     int(cw_stride), int(elem_stride), float(polarity), int(B),
                                     _p(bits, _u8p), _p(packed, _u8p), _p(iters, _i32p),
                                     _p(synd, _i32p), int(nthreads))
    out = dict(packed=packed, iters=iters, synd=synd)
    if want_bits:
        out["bits"] = bits
    return out


def dense_to_csr(H):
    H = np.asarray(H, np.uint8)
    rows, cols = np.nonzero(H)
    row_ptr = np.zeros(H.shape[0] + 1, np.int32)
    np.add.at(row_ptr, rows + 1, 1)
    return np.cumsum(row_ptr).astype(np.int32), cols.astype(np.int32)


class _OrcBlock(ctypes.Structure):
    _fields_ = [("method", ctypes.c_int), ("iterations", ctypes.c_int),
                ("state", ctypes.c_int), ("errors", ctypes.c_uint),
                ("M", ctypes.c_int), ("N", ctypes.c_int), ("H", ctypes.c_void_p),
                ("decodes", ctypes.c_longlong)]


class Block:
    """general_work restatement (lib/ldpc_decoder_cb_impl.cc:126-234)."""

    def __init__(self, method, Hr, iterations=5, csr=None):
        """Hr: the reordered dense H; or csr = (M, N, row_ptr, col_idx) for a
        large code, whose windows the sparse restatement decodes (the same
        loop, orc_block_general_work_sparse)."""
        self.csr = None
        if csr is not None:
            M, N, rp, ci = csr
            self.csr = (np.ascontiguousarray(rp, np.int32), np.ascontiguousarray(ci, np.int32))
            self.H = None
            self.MN = (int(M), int(N))
            hp = None
        else:
            self.H = np.ascontiguousarray(Hr, np.uint8)
            self.MN = self.H.shape
            hp = _p(self.H, _u8p)
        M, N = self.MN
        self.s = _OrcBlock()
        lib().orc_block_init(ctypes.byref(self.s), int(method), int(iterations), hp, M, N)

    @property
    def state(self):
        return self.s.state

    @property
    def errors(self):
        return self.s.errors

    @property
    def decodes(self):
        """Windows decoded so far, each "-tx" retry counted (a measurement)."""
        return self.s.decodes

    def general_work(self, noutput_items, in_complex):
        """in_complex: complex64 array (ninput_items long).  Returns
        (out_bytes, consumed)."""
        x = np.ascontiguousarray(in_complex, np.complex64).view(np.float32)
        M, N = self.MN
        bound = (x.size // 2) // N * (M // 8)  # each output frame consumes N
        noutput_items = min(int(noutput_items), bound)
        out = np.zeros(max(noutput_items, 1), np.uint8)
        used = ctypes.c_int32(0)
        if self.csr is not None:
            made = lib().orc_block_general_work_sparse(
                ctypes.byref(self.s), _p(self.csr[0], _i32p), _p(self.csr[1], _i32p),
                int(noutput_items), int(x.size // 2), _p(x, _f32p), _p(out, _u8p),
                ctypes.byref(used))
        else:
            made = lib().orc_block_general_work(ctypes.byref(self.s), int(noutput_items),
                                                int(x.size // 2), _p(x, _f32p), _p(out, _u8p),
                                                ctypes.byref(used))
        return out[:made].copy(), used.value


def run_stream(method, Hr, samples, iterations=5, chunks=None, out_space=1 << 30, csr=None,
               stats=None):
    """Feed a complex stream through the restated block the way the GR
    scheduler does: input arrives in `chunks` (sizes), unconsumed input is
    kept, and general_work is called again until it consumes nothing.
    Returns the concatenated output bytes.  csr: a large code's (M, N,
    row_ptr, col_idx) instead of Hr (sparse window decodes).  stats: a dict
    that receives the number of windows the loop decoded ("decodes")."""
    blk = Block(method, Hr, iterations, csr=csr)
    samples = np.asarray(samples, np.complex64)
    ends = list(np.cumsum(chunks)) if chunks is not None else []
    ends = [min(int(e), len(samples)) for e in ends] + [len(samples)]
    pos, outs = 0, []
    for end in ends:
        while True:
            out, used = blk.general_work(out_space, samples[pos:end])
            outs.append(out)
            pos += used
            if used == 0:
                break
    if stats is not None:
        stats["decodes"] = int(blk.decodes)
    return np.concatenate(outs) if outs else np.zeros(0, np.uint8)
