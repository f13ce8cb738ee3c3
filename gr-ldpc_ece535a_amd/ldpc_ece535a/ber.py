"""BER / FER sweep on the GPU.

The reference's BER program (apps/ldpc_lapack.cpp:533-811) draws random
source bits, encodes them, BPSK-modulates (2u - 1), adds white Gaussian noise
with sqrt(N0), N0 = 1 / 10^(EbN0/10) (:629-636), and decodes every frame with
four decoders -- hard BPSK, BitFlip, LogDomainSimple (min-sum) and
SumProduct, 5 iterations -- over Eb/N0 = -7 .. 10 dB in 0.5 dB steps, 30
frames per point.  Per point it reports BER = mean over frames of the
fraction of codeword bits in error (biterr, :508-517) and FER = the number of
frames whose decision fails the parity checks (checkMessage, :519-529).  It
prints an Octave script.

Here every step runs on the device through the C ABI: ldpc_random_bits ->
ldpc_encode_device -> ldpc_bpsk_awgn -> ldpc_decode_device (each method) ->
ldpc_count_bit_errors, with the syndrome weight from the decoder.  The "BPSK"
curve uses the decoder's hard method (decodeHard, which maps an exact 0.0 to
1 where the app's decodeBPSK maps it to 0 -- a probability-zero event).
The decoders are the block's (lib/ldpc_decoder_cb_impl.cc), not the app's
private copies.

    python -m ldpc_ece535a.ber [--frames 30] [--iterations 5]
                               [--ebn0 -7:10:0.5] [--code default|dvbs2] [--json out]
"""
import argparse
import json
import math
import sys

import numpy as np

from . import _capi

DEFAULT_EBN0 = [-7.0 + 0.5 * i for i in range(35)]  # :540
METHODS = (("BPSK", _capi.METHOD_HARD), ("BitFlip", _capi.METHOD_BITFLIP),
           ("LogDomainSimple", _capi.METHOD_LOGDOMAIN), ("SumProduct", _capi.METHOD_SUMPRODUCT))


def sigma_of(ebn0_db):
    """sqrt(N0), N0 = 1 / exp(EbN0 ln(10) / 10) (apps/ldpc_lapack.cpp:629)."""
    return math.sqrt(1.0 / math.exp(ebn0_db * math.log(10.0) / 10.0))


def sweep(dec=None, ebn0=DEFAULT_EBN0, frames=30, iterations=5, seed=0, precision=0, device=0):
    """Returns {method name: {"ber": [...], "fer": [...]}} over `ebn0`."""
    import torch
    if dec is None:
        dec = _capi.Decoder(device=device)
    dev = torch.device("cuda", device)
    B, N, K = int(frames), dec.N, dec.K
    d_data = torch.empty((B, K), dtype=torch.uint8, device=dev)
    d_cw = torch.empty((B, N), dtype=torch.uint8, device=dev)
    d_tx = torch.empty((B, N), dtype=torch.float32, device=dev)
    d_bits = torch.empty((B, N), dtype=torch.uint8, device=dev)
    d_packed = torch.empty((B, dec.KB), dtype=torch.uint8, device=dev)
    d_synd = torch.empty(B, dtype=torch.int32, device=dev)
    d_err = torch.empty(B, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)
    sp = stream.cuda_stream
    out = {name: {"ber": [], "fer": []} for name, _ in METHODS}
    for i, db in enumerate(ebn0):
        s0 = (int(seed) * 1000003 + i) & 0xFFFFFFFF
        _capi.random_bits(d_data.data_ptr(), B * K, s0, sp)
        dec.encode_device(d_data.data_ptr(), B, d_cw.data_ptr(), sp)
        _capi.bpsk_awgn(d_cw.data_ptr(), B * N, sigma_of(db), s0 ^ 0x5DEECE66D, d_tx.data_ptr(),
                        sp)
        for name, m in METHODS:
            dec.decode_device(d_tx.data_ptr(), B, d_packed.data_ptr(), method=m,
                              max_iters=iterations, precision=precision, d_bits=d_bits.data_ptr(),
                              d_synd=d_synd.data_ptr(), stream=sp)
            _capi.count_bit_errors(d_bits.data_ptr(), d_cw.data_ptr(), N, B, d_err.data_ptr(), sp)
            stream.synchronize()
            err = d_err.cpu().numpy().astype(np.float64)
            synd = d_synd.cpu().numpy()
            out[name]["ber"].append(float((err / N).mean()) if B else 0.0)
            out[name]["fer"].append(int((synd > 0).sum()))
    return out


def octave(ebn0, res):
    """The reference program's Octave output (apps/ldpc_lapack.cpp:707-811)."""
    f = lambda v: "%.4g" % v  # noqa: E731  (std::cout.precision(4))
    lines = ["EbN0=[" + " ".join(f(x) for x in ebn0) + " ];", "figure(1);"]
    styles = ["'or--'", "'og-'", "'ob-'", "'om-'"]
    for k, (name, _) in enumerate(METHODS):
        lines.append("ber%d=[" % k + " ".join(f(x) for x in res[name]["ber"]) + " ];")
        lines.append("plot(EbN0, ber%d, %s);" % (k, styles[k]))
        if k == 0:
            lines.append("hold;")
    lines += ["grid on;", "hold off;", "title('Bit Error Rate');",
              "legend('BPSK', 'BitFlip', 'LogDomainSimple', 'SumProduct');",
              "xlabel('EbN0');", "ylabel('BER');", "figure(2);"]
    fstyles = ["'or:'", "'og-'", "'ob-'", "'om-'"]
    for k, (name, _) in enumerate(METHODS):
        lines.append("fer%d=[" % k)
        lines.append(", ".join(str(x) for x in res[name]["fer"]))  # printVector, :71-81
        lines.append("];")
        lines.append("plot(EbN0, fer%d, %s);" % (k, fstyles[k]))
        if k == 0:
            lines.append("hold;")
    lines += ["grid on;", "hold off;", "title('Frame Errors');",
              "legend('BPSK', 'BitFlip', 'LogDomainSimple', 'SumProduct');",
              "xlabel('EbN0');", "ylabel('FER');"]
    return "\n".join(lines) + "\n"


def parse_range(text):
    """'a:b:step' (inclusive) or a comma list."""
    if ":" in text:
        a, b, st = (float(x) for x in text.split(":"))
        n = int(round((b - a) / st)) + 1
        return [a + st * i for i in range(n)]
    return [float(x) for x in text.split(",")]


def main(argv=None):
    ap = argparse.ArgumentParser(prog="ldpc_ber", description=__doc__.split("\n\n")[0])
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--iterations", type=int, default=5)
    ap.add_argument("--ebn0", default="-7:10:0.5")
    ap.add_argument("--code", choices=["default", "dvbs2"], default="default")
    ap.add_argument("--precision", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    # torch first: it then shares its HIP runtime with libldpc_hip.so (see
    # INTEGRATION.md, "One HIP runtime per process")
    import torch  # noqa: F401
    if a.code == "dvbs2":
        from . import codes
        dec = _capi.Decoder(csr=codes.dvbs2_like(0))
    else:
        dec = _capi.Decoder()
    grid = parse_range(a.ebn0)
    res = sweep(dec, grid, a.frames, a.iterations, a.seed, a.precision)
    sys.stdout.write(octave(grid, res))
    if a.json:
        json.dump({"ebn0": grid, "frames": a.frames, "iterations": a.iterations,
                   "code": a.code, "results": res}, open(a.json, "w"), indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
