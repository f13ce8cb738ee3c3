"""Python blocks over lib/libgnuradio-ldpc_ece535a.so (include/ldpc_block.h).

`ldpc_decoder_cb(method)` and `ldpc_encoder_bc()` mirror the reference's SWIG
blocks (swig/ldpc_ece535a_swig.i:17-22): construct with the same arguments,
then a scheduler (ldpc_ece535a.flowgraph, or a maintainer's GNU Radio glue)
calls forecast() / general_work() with the GNU Radio meaning of the
arguments.  The decoder decodes on the GPU; constructing it without one
raises LdpcError.
"""
import ctypes
import os

import numpy as np

from ._capi import LIB_DIR, LdpcError

BLOCK_LIB = os.path.join(LIB_DIR, "libgnuradio-ldpc_ece535a.so")

STATE_OUT_OF_SYNC, STATE_IN_SYNC, STATE_IN_SYNC_INVERTED = 0, 1, 2

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_f32p = ctypes.POINTER(ctypes.c_float)
_vp = ctypes.c_void_p
_i = ctypes.c_int

BACKEND_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, _f32p, ctypes.c_int64,
                              ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_int, _u8p,
                              _i32p)

SIGNATURES = {
    "ldpc_decoder_cb_make": (_vp, [_i, _i, _i, _i]),
    "ldpc_decoder_cb_forecast": (None, [_vp, _i, _i32p]),
    "ldpc_decoder_cb_general_work": (_i, [_vp, _i, _i, _f32p, _u8p, _i32p]),
    "ldpc_decoder_cb_state": (_i, [_vp, _u32p]),
    "ldpc_decoder_cb_frames_decoded": (ctypes.c_int64, [_vp]),
    "ldpc_decoder_cb_launches": (ctypes.c_int64, [_vp]),
    "ldpc_decoder_cb_destroy": (None, [_vp]),
    "ldpc_decoder_cb_make_with_backend": (_vp, [_i, _i, BACKEND_FN, _vp]),
    "ldpc_decoder_cb_make_h": (_vp, [_i, _i, _i, _i, _u8p, _i, _i, _i]),
    "ldpc_decoder_cb_make_csr": (_vp, [_i, _i, _i, _i, _i, _i, _i32p, _i32p, _i]),
    "ldpc_decoder_cb_make_alist": (_vp, [_i, _i, _i, _i, ctypes.c_char_p]),
    "ldpc_decoder_cb_frame_shape": (_i, [_vp, _i32p, _i32p, _i32p]),
    "ldpc_encoder_bc_make": (_vp, []),
    "ldpc_encoder_bc_forecast": (None, [_vp, _i, _i32p]),
    "ldpc_encoder_bc_general_work": (_i, [_vp, _i, _i, _u8p, _f32p, _i32p]),
    "ldpc_encoder_bc_destroy": (None, [_vp]),
    "ldpc_block_last_error": (ctypes.c_char_p, []),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(BLOCK_LIB):
            raise LdpcError("%s is missing: build with `make -C %s`" %
                            (BLOCK_LIB, os.path.dirname(LIB_DIR)))
        L = ctypes.CDLL(BLOCK_LIB)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _err():
    return (lib().ldpc_block_last_error() or b"").decode()


class ldpc_decoder_cb:
    """LDPC decoder block: gr_complex in, packed bytes out.

    ldpc_decoder_cb(method) is the reference's make(method) (5 iterations,
    f64 parity arithmetic, the default 32x64 H); iterations / precision are
    additive options, as is a runtime H: `H` (dense M x N, reorderHMatrix
    applied as the reference's constructor does, unless reorder=False), `csr`
    = (M, N, row_ptr, col_idx) used as given, or `alist` = a MacKay alist path.
    """
    in_itemsize = 8   # sizeof(gr_complex)
    out_itemsize = 1

    def __init__(self, method=0, iterations=5, precision=0, device=0, H=None, csr=None,
                 alist=None, reorder=True, _backend=None):
        self._backend = None
        if H is not None:
            H = np.ascontiguousarray(H, np.uint8)
            self._h = lib().ldpc_decoder_cb_make_h(int(method), int(iterations), int(precision),
                                                   int(device), H.ctypes.data_as(_u8p),
                                                   H.shape[0], H.shape[1], 0 if reorder else 1)
        elif csr is not None:
            M, N, rp, ci = csr
            rp = np.ascontiguousarray(rp, np.int32)
            ci = np.ascontiguousarray(ci, np.int32)
            self._h = lib().ldpc_decoder_cb_make_csr(int(method), int(iterations), int(precision),
                                                     int(device), int(M), int(N),
                                                     rp.ctypes.data_as(_i32p),
                                                     ci.ctypes.data_as(_i32p), 0)
        elif alist is not None:
            self._h = lib().ldpc_decoder_cb_make_alist(int(method), int(iterations),
                                                       int(precision), int(device),
                                                       os.fsencode(alist))
        elif _backend is not None:
            # TEST SEAM: host-logic tests only (see include/ldpc_block.h)
            self._backend = BACKEND_FN(_backend)
            self._h = lib().ldpc_decoder_cb_make_with_backend(int(method), int(iterations),
                                                              self._backend, None)
        else:
            self._h = lib().ldpc_decoder_cb_make(int(method), int(iterations), int(precision),
                                                 int(device))
        if not self._h:
            raise LdpcError("ldpc_decoder_cb: %s" % _err())
        self.method = method
        m, n, k = ctypes.c_int32(0), ctypes.c_int32(0), ctypes.c_int32(0)
        lib().ldpc_decoder_cb_frame_shape(self._h, ctypes.byref(m), ctypes.byref(n),
                                          ctypes.byref(k))
        self.M, self.N, self.frame_bytes = m.value, n.value, k.value

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().ldpc_decoder_cb_destroy(h)
            self._h = None

    def forecast(self, noutput_items):
        req = ctypes.c_int32(0)
        lib().ldpc_decoder_cb_forecast(self._h, int(noutput_items), ctypes.byref(req))
        return req.value

    def general_work(self, noutput_items, input_items):
        """input_items: complex64 array (the available input); returns
        (output bytes, consumed)."""
        x = np.ascontiguousarray(input_items, np.complex64).view(np.float32)
        out = np.zeros(max(int(noutput_items), 1), np.uint8)
        used = ctypes.c_int32(0)
        made = lib().ldpc_decoder_cb_general_work(
            self._h, int(noutput_items), int(x.size // 2), x.ctypes.data_as(_f32p),
            out.ctypes.data_as(_u8p), ctypes.byref(used))
        if made < 0:
            raise LdpcError("ldpc_decoder_cb.general_work: %s" % _err())
        return out[:made].copy(), used.value

    @property
    def state(self):
        return lib().ldpc_decoder_cb_state(self._h, None)

    @property
    def errors(self):
        e = ctypes.c_uint32(0)
        lib().ldpc_decoder_cb_state(self._h, ctypes.byref(e))
        return e.value

    @property
    def frames_decoded(self):
        return lib().ldpc_decoder_cb_frames_decoded(self._h)

    @property
    def launches(self):
        return lib().ldpc_decoder_cb_launches(self._h)


class ldpc_encoder_bc:
    """LDPC encoder block: packed bytes in, BPSK gr_complex out (rate 1/2)."""
    in_itemsize = 1
    out_itemsize = 8

    def __init__(self):
        self._h = lib().ldpc_encoder_bc_make()
        if not self._h:
            raise LdpcError("ldpc_encoder_bc: %s" % _err())

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().ldpc_encoder_bc_destroy(h)
            self._h = None

    def forecast(self, noutput_items):
        req = ctypes.c_int32(0)
        lib().ldpc_encoder_bc_forecast(self._h, int(noutput_items), ctypes.byref(req))
        return req.value

    def general_work(self, noutput_items, input_items):
        x = np.ascontiguousarray(input_items, np.uint8)
        out = np.zeros(max(int(noutput_items), 1), np.complex64)
        used = ctypes.c_int32(0)
        made = lib().ldpc_encoder_bc_general_work(
            self._h, int(noutput_items), int(x.size), x.ctypes.data_as(_u8p),
            out.view(np.float32).ctypes.data_as(_f32p), ctypes.byref(used))
        if made < 0:
            raise LdpcError("ldpc_encoder_bc.general_work: %s" % _err())
        return out[:made].copy(), used.value
