"""ldpc_ece535a -- MI355X-native drop-in for gr-ldpc_ece535a's decode path.

Python face of the package, mirroring the reference's SWIG module
(swig/ldpc_ece535a_swig.i:17-22, python/__init__.py:45):

    ldpc_ece535a.ldpc_decoder_cb(method)   # GR-3.7-shaped decoder block
    ldpc_ece535a.ldpc_encoder_bc()         # GR-3.7-shaped encoder block

plus the C-ABI binding (`Decoder`, `encode`, `reorder_h`, ...) of
include/ldpc_hip.h.  Decoding always runs on the GPU through
lib/libldpc_hip.so; there is no CPU fallback.
"""
from ._capi import (  # noqa: F401
    FLAG_NO_REORDER, METHOD_BITFLIP, METHOD_HARD, METHOD_LOGDOMAIN, METHOD_SUMPRODUCT,
    PREC_F32, PREC_F64, PREC_F64_FAST, PREC_F64_LIBM, Decoder, LdpcError, bpsk_awgn, check_frame, count_bit_errors,
    default_h, encode, plan_layout, random_bits, reorder_h,
)
from .blocks import (  # noqa: F401,E402
    STATE_IN_SYNC, STATE_IN_SYNC_INVERTED, STATE_OUT_OF_SYNC, ldpc_decoder_cb, ldpc_encoder_bc,
)
from . import flowgraph  # noqa: F401,E402
