"""ctypes binding of the C ABI in include/ldpc_hip.h (lib/libldpc_hip.so).

The shared library is built in-tree (gr-ldpc_ece535a_amd/lib/); importing this
module never falls back to anything else: if the library is missing, loading
fails with an error that says how to build it, and if no GPU is usable,
Decoder() raises.
"""
import ctypes
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(PKG_ROOT, "lib")
HIP_LIB = os.path.join(LIB_DIR, "libldpc_hip.so")

METHOD_LOGDOMAIN, METHOD_SUMPRODUCT, METHOD_BITFLIP, METHOD_HARD = 0, 1, 2, 3
PREC_F64, PREC_F32, PREC_F64_LIBM, PREC_F64_FAST = 0, 1, 2, 3
FLAG_NO_REORDER = 1
FLAG_GRAPH = 2
FLAG_PLAIN_LAYOUT = 4
TEST_SERVE_UNCHECKED, TEST_SERVE_EPOCH, TEST_SERVE_EPOCH_NOW, TEST_STREAM_OVERLAP = 1, 2, 3, 4
SERVE_EPOCH_LIMIT = (1 << 23) - (1 << 16)
PATH_SMALL, PATH_GRAPH = 0, 1
MODE_LATENCY, MODE_THROUGHPUT = 0, 1
ERRORS = {0: "LDPC_OK", -1: "LDPC_EINVAL", -2: "LDPC_EUNSUPPORTED", -3: "LDPC_EDEVICE",
          -4: "LDPC_ESINGULAR", -5: "LDPC_ENOMEM", -6: "LDPC_ETIMEOUT"}


_u8p = ctypes.POINTER(ctypes.c_uint8)
_i32p = ctypes.POINTER(ctypes.c_int32)
_f32p = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_int64)
_i = ctypes.c_int
_i64 = ctypes.c_int64
_vp = ctypes.c_void_p

# name -> (restype, argtypes); the full set the header declares
SIGNATURES = {
    "ldpc_default_h": (_i, [_u8p]),
    "ldpc_reorder_h": (_i, [_u8p, _i, _i, _i32p]),
    "ldpc_check_frame": (_i, [_u8p, _i, _i, _u8p, _i]),
    "ldpc_encode": (_i, [_u8p, _i, _i, _u8p, _i, _u8p]),
    "ldpc_create": (_vp, [_u8p, _i, _i, _i, _i]),
    "ldpc_create_csr": (_vp, [_i, _i, _i32p, _i32p, _i, _i]),
    "ldpc_ctx_csr": (_i, [_vp, _i32p, _i32p]),
    "ldpc_ctx_path": (_i, [_vp]),
    "ldpc_ctx_pipeline": (_i, [_vp, _i32p, _i32p]),
    "ldpc_ctx_layout": (_i, [_vp, _i32p]),
    "ldpc_plan_layout": (_i, [_u8p, _i, _i, _i, _i32p, _i32p, _i32p]),
    "ldpc_plan_storage_order": (_i, [_i, _i, _i32p, _i32p, _i32p, _i32p, _i64p]),
    "ldpc_set_work_limit": (_i, [_vp, _i64]),
    "ldpc_encode_device": (_i, [_vp, _vp, _i, _vp, _vp]),
    "ldpc_random_bits": (_i, [_vp, _i64, ctypes.c_uint64, _vp]),
    "ldpc_bpsk_awgn": (_i, [_vp, _i64, ctypes.c_float, ctypes.c_uint64, _vp, _vp]),
    "ldpc_count_bit_errors": (_i, [_vp, _vp, _i64, _i, _vp, _vp]),
    "ldpc_destroy": (None, [_vp]),
    "ldpc_last_error": (ctypes.c_char_p, [_vp]),
    "ldpc_ctx_info": (_i, [_vp, _i32p, _i32p, _i32p, _i32p, _i32p, _i32p, _i32p]),
    "ldpc_ctx_h": (_i, [_vp, _u8p]),
    "ldpc_decode": (_i, [_vp, _i, _i, _i, _i, _f32p, _i, _u8p, _u8p, _i32p, _i32p]),
    "ldpc_decode_strided": (_i, [_vp, _i, _i, _i, _i, _f32p, _i64, _i64, _i, ctypes.c_float, _i,
                                 _u8p, _u8p, _i32p, _i32p, _f32p]),
    "ldpc_decode_device": (_i, [_vp, _i, _i, _i, _i, _vp, _i64, _i, ctypes.c_float, _i,
                                _vp, _vp, _vp, _vp, _vp, _vp]),
    "ldpc_decode_strided_both": (_i, [_vp, _i, _i, _i, _i, _f32p, _i64, _i64, _i,
                                     ctypes.c_float, _i, _u8p, _i32p]),
    "ldpc_decode_windows": (_i, [_vp, _i, _i, _i, _i, _f32p, _i64, _i, _i,
                                 ctypes.POINTER(ctypes.c_int64), _i, _u8p, _i32p]),
    "ldpc_stage_span": (_i, [_vp, _f32p, _i64, _i, _i]),
    "ldpc_serve_begin": (_i, [_vp, _i, _i, _i, _i]),
    "ldpc_serve_windows": (_i, [_vp, ctypes.POINTER(ctypes.c_int64), _i, _u8p, _i32p]),
    "ldpc_serve_end": (_i, [_vp]),
    "ldpc_ctx_streams": (_i, [_vp, _i, ctypes.POINTER(ctypes.c_void_p)]),
    "ldpc_alist_read": (_i, [ctypes.c_char_p, _i32p, _i32p, _i32p, _i32p, _i64]),
    "ldpc_set_waves_per_cu": (_i, [_vp, _i]),
    "ldpc_set_launch_mode": (_i, [_vp, _i]),
    "ldpc_set_schedule": (_i, [_vp, _i]),
    "ldpc_synchronize": (_i, [_vp]),
    "ldpc_test_hook": (_i, [_vp, _i, _i64]),
    "ldpc_ring_begin": (_i, [_vp, _i, _i, _i, _i, _vp]),
    "ldpc_ring_post": (_i64, [_vp, _vp, _i64, _i, _vp, _vp, _vp]),
    "ldpc_ring_wait": (_i, [_vp, _i64]),
    "ldpc_ring_end": (_i, [_vp]),
    "ldpc_ring_info": (_i, [_vp, _i32p, _i32p]),
}

_lib = None


class LdpcError(RuntimeError):
    pass


def lib():
    """Load lib/libldpc_hip.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(HIP_LIB):
            raise LdpcError("%s is missing: build it with `make -C %s` (or "
                            "__graft_entry__.build()); there is no fallback" % (HIP_LIB, PKG_ROOT))
        L = ctypes.CDLL(HIP_LIB)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a, t):
    return None if a is None else a.ctypes.data_as(t)


def _check(rc, ctx=None):
    if rc < 0:
        msg = lib().ldpc_last_error(ctx)
        raise LdpcError("%s: %s" % (ERRORS.get(rc, rc), (msg or b"").decode()))
    return rc


def default_h():
    """The reference decoder's 32x64 H (lib/ldpc_decoder_cb_impl.cc:63-96)."""
    H = np.zeros((32, 64), np.uint8)
    _check(lib().ldpc_default_h(_p(H, _u8p)))
    return H


def reorder_h(H):
    """reorderHMatrix (lib/ldpc_decoder_cb_impl.cc:255-307) -> (Hr, chosen)."""
    H = np.ascontiguousarray(H, np.uint8).copy()
    M, N = H.shape
    chosen = np.zeros(M, np.int32)
    _check(lib().ldpc_reorder_h(_p(H, _u8p), M, N, _p(chosen, _i32p)))
    return H, chosen


def check_frame(H, bits, threshold):
    """checkFrame (lib/ldpc_decoder_cb_impl.cc:236-253)."""
    H = np.ascontiguousarray(H, np.uint8)
    bits = np.ascontiguousarray(bits, np.uint8)
    M, N = H.shape
    return _check(lib().ldpc_check_frame(_p(H, _u8p), M, N, _p(bits, _u8p), int(threshold)))


def encode(Hr, data_bits):
    """makeParityCheck (lib/ldpc_encoder_bc_impl.cc:275-294): (B, N-M) data
    bits -> (B, N) codewords [parity; data]."""
    Hr = np.ascontiguousarray(Hr, np.uint8)
    M, N = Hr.shape
    d = np.ascontiguousarray(np.atleast_2d(data_bits), np.uint8)
    out = np.zeros((d.shape[0], N), np.uint8)
    _check(lib().ldpc_encode(_p(Hr, _u8p), M, N, _p(d, _u8p), d.shape[0], _p(out, _u8p)))
    return out


def plan_layout(H, reorder=True, plain=False):
    """The small-code kernel's LDS layout for H (host only, no GPU): dict with
    cell (E,) = lane slot of each edge in CSR order of the decoder's H, pos (N,)
    = lane position of each column, and model = {searched, cc, ec, plain_cc,
    plain_ec}: modelled extra LDS bank-conflict cycles per iteration of the
    column-centric sum-product / min-sum kernels for this layout and for the
    plain CSR layout (csrc/ldpc_layout.hpp)."""
    H = np.ascontiguousarray(H, np.uint8)
    M, N = H.shape
    flags = (0 if reorder else FLAG_NO_REORDER) | (FLAG_PLAIN_LAYOUT if plain else 0)
    cell = np.zeros(M * N, np.int32)
    pos = np.zeros(N, np.int32)
    model = np.zeros(5, np.int32)
    E = _check(lib().ldpc_plan_layout(_p(H, _u8p), M, N, flags, _p(cell, _i32p), _p(pos, _i32p),
                                      _p(model, _i32p)))
    return dict(cell=cell[:E].copy(), pos=pos,
                model=dict(zip(("searched", "cc", "ec", "plain_cc", "plain_ec"),
                               (int(v) for v in model))))


def plan_storage_order(csr):
    """The large-code min-sum pipeline's storage order for csr = (M, N,
    row_ptr, col_idx) (host only, no GPU): dict with order (0 identity, 1
    DVB-S2 residue classes), rpos (M,) and cpos (N,) = storage position of
    each original row / column, and score = contiguity of the identity and
    residue-class orders (-1: not tried)."""
    M, N, rp, ci = csr
    rp = np.ascontiguousarray(rp, np.int32)
    ci = np.ascontiguousarray(ci, np.int32)
    rpos = np.zeros(M, np.int32)
    cpos = np.zeros(N, np.int32)
    score = np.zeros(2, np.int64)
    order = _check(lib().ldpc_plan_storage_order(M, N, _p(rp, _i32p), _p(ci, _i32p),
                                                 _p(rpos, _i32p), _p(cpos, _i32p),
                                                 _p(score, _i64p)))
    return dict(order=order, rpos=rpos, cpos=cpos, score=(int(score[0]), int(score[1])))


class Decoder:
    """One decode context (device tables + stream) for one H.

    H: dense (M, N) 0/1 matrix (reorderHMatrix applied unless reorder=False),
    or csr=(M, N, row_ptr, col_idx) for a sparse H used as given.
    force_graph=True selects the large-code (HBM message) kernels even for a
    code the small-code kernel could take; plain_layout=True keeps the
    small-code kernel's edges and columns in CSR order (A/B and tests)."""

    def __init__(self, H=None, reorder=True, device=0, csr=None, force_graph=False,
                 plain_layout=False):
        flags = ((0 if reorder else FLAG_NO_REORDER) | (FLAG_GRAPH if force_graph else 0) |
                 (FLAG_PLAIN_LAYOUT if plain_layout else 0))
        if csr is not None:
            M, N, rp, ci = csr
            rp = np.ascontiguousarray(rp, np.int32)
            ci = np.ascontiguousarray(ci, np.int32)
            self._ctx = lib().ldpc_create_csr(int(M), int(N), _p(rp, _i32p), _p(ci, _i32p),
                                              flags, int(device))
            what = "ldpc_create_csr"
        else:
            if H is None:
                H = default_h()
            H = np.ascontiguousarray(H, np.uint8)
            M, N = H.shape
            self._ctx = lib().ldpc_create(_p(H, _u8p), M, N, flags, int(device))
            what = "ldpc_create"
        if not self._ctx:
            raise LdpcError("%s failed: %s" % (what, lib().ldpc_last_error(None).decode()))
        v = [ctypes.c_int32(0) for _ in range(7)]
        _check(lib().ldpc_ctx_info(self._ctx, *[ctypes.byref(x) for x in v]), self._ctx)
        self.M, self.N, self.E, self.K, self.KB, self.dc_max, self.dv_max = [x.value for x in v]
        self.path = _check(lib().ldpc_ctx_path(self._ctx), self._ctx)
        self.row_ptr = np.zeros(self.M + 1, np.int32)
        self.col_idx = np.zeros(self.E, np.int32)
        _check(lib().ldpc_ctx_csr(self._ctx, _p(self.row_ptr, _i32p), _p(self.col_idx, _i32p)),
               self._ctx)
        self._H = None

    def pipeline(self):
        """ldpc_ctx_pipeline: {frames_per_chunk, chunks} of the large-code
        min-sum pipeline (both 0 when this context does not use it)."""
        f, c = ctypes.c_int32(0), ctypes.c_int32(0)
        _check(lib().ldpc_ctx_pipeline(self._ctx, ctypes.byref(f), ctypes.byref(c)), self._ctx)
        return {"frames_per_chunk": f.value, "chunks": c.value}

    @property
    def layout_model(self):
        """ldpc_ctx_layout: {searched, cc, ec, plain_cc, plain_ec} (see plan_layout)."""
        m = np.zeros(5, np.int32)
        _check(lib().ldpc_ctx_layout(self._ctx, _p(m, _i32p)), self._ctx)
        return dict(zip(("searched", "cc", "ec", "plain_cc", "plain_ec"), (int(v) for v in m)))

    @property
    def H(self):
        """The decoder's (reordered) H as a dense (M, N) array (built on demand)."""
        if self._H is None:
            self._H = np.zeros((self.M, self.N), np.uint8)
            _check(lib().ldpc_ctx_h(self._ctx, _p(self._H, _u8p)), self._ctx)
        return self._H

    def close(self):
        if getattr(self, "_ctx", None):
            lib().ldpc_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._ctx

    def decode(self, llr, method=METHOD_SUMPRODUCT, max_iters=50, et_period=1,
               precision=PREC_F64, polarity=1.0, cw_stride=None, elem_stride=1, B=None,
               want_bits=True, want_llr=False):
        """Decode host float32 frames (synchronous).  Returns a dict with
        packed (B,KB), bits (B,N), iters (B,), synd (B,) [, llr (B,N)]."""
        x = np.ascontiguousarray(llr, np.float32).reshape(-1)
        if cw_stride is None:
            cw_stride = self.N * elem_stride
        if B is None:
            B = x.size // cw_stride if cw_stride else 0
        packed = np.zeros((B, self.KB), np.uint8)
        bits = np.zeros((B, self.N), np.uint8) if want_bits else None
        iters = np.zeros(B, np.int32)
        synd = np.zeros(B, np.int32)
        post = np.zeros((B, self.N), np.float32) if want_llr else None
        _check(lib().ldpc_decode_strided(self._ctx, int(method), int(max_iters), int(et_period),
                                         int(precision), _p(x, _f32p), x.size, int(cw_stride),
                                         int(elem_stride), float(polarity), int(B),
                                         _p(packed, _u8p), _p(bits, _u8p), _p(iters, _i32p),
                                         _p(synd, _i32p), _p(post, _f32p)), self._ctx)
        out = dict(packed=packed, iters=iters, synd=synd)
        if want_bits:
            out["bits"] = bits
        if want_llr:
            out["llr"] = post
        return out

    def decode_both(self, llr, method=METHOD_SUMPRODUCT, max_iters=50, et_period=1,
                    precision=PREC_F64, polarity=1.0, cw_stride=None, elem_stride=1, B=None):
        """ldpc_decode_strided_both: the B windows decoded at +polarity (rows
        0..B-1) and -polarity (rows B..2B-1) in one launch.  Returns dict with
        packed (2B,KB) and synd (2B,)."""
        x = np.ascontiguousarray(llr, np.float32).reshape(-1)
        if cw_stride is None:
            cw_stride = self.N * elem_stride
        if B is None:
            B = x.size // cw_stride if cw_stride else 0
        packed = np.zeros((2 * B, self.KB), np.uint8)
        synd = np.zeros(2 * B, np.int32)
        _check(lib().ldpc_decode_strided_both(self._ctx, int(method), int(max_iters),
                                              int(et_period), int(precision), _p(x, _f32p),
                                              x.size, int(cw_stride), int(elem_stride),
                                              float(polarity), int(B), _p(packed, _u8p),
                                              _p(synd, _i32p)), self._ctx)
        return dict(packed=packed, synd=synd)

    def stage_span(self, samples, elem_stride=1, max_windows=0):
        """ldpc_stage_span: copy a sample span to the device for the
        decode_windows(..., reuse_span=True) calls that follow."""
        x = np.ascontiguousarray(samples, np.float32).reshape(-1)
        self._span = x  # the copy is asynchronous: keep the source alive
        _check(lib().ldpc_stage_span(self._ctx, _p(x, _f32p), x.size, int(elem_stride),
                                     int(max_windows)), self._ctx)

    def decode_windows(self, samples, windows, method=METHOD_SUMPRODUCT, max_iters=50,
                       et_period=1, precision=PREC_F64, elem_stride=1, reuse_span=False):
        """ldpc_decode_windows: windows (B,) int64 = (start << 1) | negate over
        one host sample span.  Returns dict(packed (B,KB), synd (B,))."""
        x = np.ascontiguousarray(samples, np.float32).reshape(-1)
        w = np.ascontiguousarray(windows, np.int64)
        B = w.size
        packed = np.zeros((B, self.KB), np.uint8)
        synd = np.zeros(B, np.int32)
        _check(lib().ldpc_decode_windows(self._ctx, int(method), int(max_iters), int(et_period),
                                         int(precision), _p(x, _f32p), x.size, int(elem_stride),
                                         1 if reuse_span else 0,
                                         w.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), B,
                                         _p(packed, _u8p), _p(synd, _i32p)), self._ctx)
        return dict(packed=packed, synd=synd)

    def serve_begin(self, method=METHOD_SUMPRODUCT, max_iters=5, precision=PREC_F64,
                    max_windows=4096):
        """ldpc_serve_begin: start the window server over the span staged last
        (stage_span); rounds then go through serve_windows."""
        _check(lib().ldpc_serve_begin(self._ctx, int(method), int(max_iters), int(precision),
                                      int(max_windows)), self._ctx)

    def serve_windows(self, windows):
        """ldpc_serve_windows: one round of windows (int64 (start << 1) | negate)
        of the staged span.  Returns dict(packed (B,KB), synd (B,))."""
        w = np.ascontiguousarray(windows, np.int64)
        B = w.size
        packed = np.zeros((B, self.KB), np.uint8)
        synd = np.zeros(B, np.int32)
        _check(lib().ldpc_serve_windows(self._ctx, w.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                        B, _p(packed, _u8p), _p(synd, _i32p)), self._ctx)
        return dict(packed=packed, synd=synd)

    def streams(self, n):
        """ldpc_ctx_streams: n hipStream_t handles (ints) of the context's
        in-flight set (best effort: self.streams_distinct of them distinct)."""
        arr = (ctypes.c_void_p * int(n))()
        self.streams_distinct = _check(lib().ldpc_ctx_streams(self._ctx, int(n), arr), self._ctx)
        return [int(x) for x in arr]

    def ring_begin(self, method=METHOD_SUMPRODUCT, max_iters=50, et_period=1,
                   precision=PREC_F64, stream=None):
        """ldpc_ring_begin: open a frame-ring session (one persistent launch for
        every batch posted until ring_end), after the work on `stream`."""
        _check(lib().ldpc_ring_begin(self._ctx, int(method), int(max_iters), int(et_period),
                                     int(precision), stream), self._ctx)

    def ring_post(self, d_in, B, d_packed, d_iters=None, d_synd=None, cw_stride=None):
        """ldpc_ring_post: post B device-resident frames (raw pointers); returns
        the batch id."""
        if cw_stride is None:
            cw_stride = self.N
        ptr = lambda x: None if x is None else int(x)  # noqa: E731
        return _check(lib().ldpc_ring_post(self._ctx, ptr(d_in), int(cw_stride), int(B),
                                           ptr(d_packed), ptr(d_iters), ptr(d_synd)), self._ctx)

    def ring_wait(self, batch):
        """ldpc_ring_wait: return once batch `batch` is complete."""
        _check(lib().ldpc_ring_wait(self._ctx, int(batch)), self._ctx)

    def ring_end(self):
        """ldpc_ring_end: end the session (work enqueued on the session's
        stream afterwards follows its last batch)."""
        _check(lib().ldpc_ring_end(self._ctx), self._ctx)

    def ring_info(self):
        """ldpc_ring_info: {launches, workgroups} of this context's ring."""
        a, b = ctypes.c_int32(0), ctypes.c_int32(0)
        _check(lib().ldpc_ring_info(self._ctx, ctypes.byref(a), ctypes.byref(b)), self._ctx)
        return {"launches": a.value, "workgroups": b.value}

    def test_hook(self, op, arg=0):
        """ldpc_test_hook (test seam): TEST_SERVE_UNCHECKED, TEST_SERVE_EPOCH,
        TEST_SERVE_EPOCH_NOW."""
        return _check(lib().ldpc_test_hook(self._ctx, int(op), int(arg)), self._ctx)

    def serve_end(self):
        _check(lib().ldpc_serve_end(self._ctx), self._ctx)

    def decode_device(self, d_in, B, d_packed, method=METHOD_SUMPRODUCT, max_iters=50,
                      et_period=1, precision=PREC_F64, polarity=1.0, cw_stride=None,
                      elem_stride=1, d_bits=None, d_iters=None, d_synd=None, d_llr=None,
                      stream=None):
        """Enqueue a decode of device-resident buffers (raw pointers / ints)."""
        if cw_stride is None:
            cw_stride = self.N * elem_stride
        _check(lib().ldpc_decode_device(self._ctx, int(method), int(max_iters), int(et_period),
                                        int(precision), d_in, int(cw_stride), int(elem_stride),
                                        float(polarity), int(B), d_packed, d_bits, d_iters,
                                        d_synd, d_llr, stream), self._ctx)

    def set_launch_mode(self, mode):
        """MODE_LATENCY (default: one decode at a time) or MODE_THROUGHPUT
        (several decodes in flight on different streams)."""
        _check(lib().ldpc_set_launch_mode(self._ctx, int(mode)), self._ctx)

    def set_waves_per_cu(self, n):
        _check(lib().ldpc_set_waves_per_cu(self._ctx, int(n)), self._ctx)

    def encode_device(self, d_data, B, d_codewords, stream=None):
        """Enqueue a systematic encode of B frames (device pointers): (B, K)
        0/1 bytes -> (B, N) codewords [parity | data]."""
        _check(lib().ldpc_encode_device(self._ctx, d_data, int(B), d_codewords, stream),
               self._ctx)

    def set_work_limit(self, nbytes):
        """Large-code path: device workspace cap (0 = default 8 GiB)."""
        _check(lib().ldpc_set_work_limit(self._ctx, int(nbytes)), self._ctx)

    def set_schedule(self, mode):
        """0 auto, 1 one wave per frame, 2 one workgroup per frame."""
        _check(lib().ldpc_set_schedule(self._ctx, int(mode)), self._ctx)

    def synchronize(self):
        _check(lib().ldpc_synchronize(self._ctx), self._ctx)


def alist_read(path):
    """ldpc_alist_read: a MacKay alist file as (M, N, row_ptr, col_idx)."""
    M, N = ctypes.c_int32(0), ctypes.c_int32(0)
    bpath = os.fsencode(path)
    E = lib().ldpc_alist_read(bpath, ctypes.byref(M), ctypes.byref(N), None, None, 0)
    if E < 0:
        raise LdpcError("ldpc_alist_read(%s): %s" % (path, lib().ldpc_last_error(None).decode()))
    rp = np.zeros(M.value + 1, np.int32)
    ci = np.zeros(max(E, 1), np.int32)
    _check(lib().ldpc_alist_read(bpath, ctypes.byref(M), ctypes.byref(N), _p(rp, _i32p),
                                 _p(ci, _i32p), int(E)))
    return M.value, N.value, rp, ci[:E]


def random_bits(d_out, n, seed, stream=None):
    """n seeded random 0/1 bytes into device memory (Philox4x32-10)."""
    _check(lib().ldpc_random_bits(d_out, int(n), int(seed) & 0xFFFFFFFFFFFFFFFF, stream))


def bpsk_awgn(d_bits, n, sigma, seed, d_out, stream=None):
    """d_out = 2 * bits - 1 + sigma * N(0, 1) (float32, device pointers)."""
    _check(lib().ldpc_bpsk_awgn(d_bits, int(n), float(sigma), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                d_out, stream))


def count_bit_errors(d_a, d_b, per_frame, B, d_counts, stream=None):
    """Per-frame count of differing 0/1 bytes (device pointers)."""
    _check(lib().ldpc_count_bit_errors(d_a, d_b, int(per_frame), int(B), d_counts, stream))
