"""ldpc_dump: the reference's apps/ldpc_ece535a_dump flowgraph on this package.

The reference app (apps/ldpc_ece535a_dump:32-61) builds
    random printable ASCII -> throttle -> ldpc_encoder_bc -> ldpc_decoder_cb -> dump sink
and prints the decoded characters.  Here the same chain runs through this
package's blocks (the decoder on the GPU) in the flowgraph harness; the
throttle is dropped (it only paces a live flowgraph).  Options add what the
app hard-codes or cannot do: the decoder method and iteration cap (SURVEY
config 1: one codeword, 10 sum-product iterations), AWGN with the reference's
sigma = sqrt(10^(-EbN0/10)) convention, a seed, and a check against the sent
text.

    python -m ldpc_ece535a.dump [--chars 4] [--method 1] [--iterations 10]
                                [--ebn0 DB] [--seed S] [--check]

Four characters are 32 bits: one codeword of the reference's 32x64 code.
"""
import argparse
import sys

import numpy as np

from . import flowgraph
from .blocks import ldpc_decoder_cb, ldpc_encoder_bc


class dump_sink(flowgraph.vector_sink_b):
    """Writes every received byte as a character (apps/ldpc_ece535a_dump:17-29)."""

    def __init__(self, stream=None):
        super().__init__()
        self._stream = stream if stream is not None else sys.stdout

    def _push(self, items):
        super()._push(items)
        self._stream.write("".join(chr(int(i)) for i in items))


class _noise:
    """A pass-through block adding AWGN to the complex BPSK symbols."""

    def __init__(self, ebn0, rng):
        self._sigma = float(np.sqrt(10.0 ** (-ebn0 / 10.0)))
        self._rng = rng

    def general_work(self, noutput_items, input_items):
        x = np.asarray(input_items, np.complex64)
        if not len(x):
            return np.zeros(0, np.complex64), 0
        n = self._rng.standard_normal(len(x)) * self._sigma
        return (x + n.astype(np.float32)).astype(np.complex64), len(x)


def run(chars=4, method=1, iterations=10, ebn0=None, seed=None, precision=0, device=0,
        stream=None):
    """Runs the dump flowgraph; returns (sent bytes, received bytes)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    text = rng.integers(32, 127, size=chars, dtype=np.uint8)  # :47 randint(32, 127)
    tb = flowgraph.top_block("LDPC Dump")
    src = flowgraph.vector_source_b(text)
    enc = ldpc_encoder_bc()
    dec = ldpc_decoder_cb(method, iterations, precision, device)
    sink = dump_sink(stream)
    chain = [src, enc] + ([_noise(ebn0, rng)] if ebn0 is not None else []) + [dec, sink]
    tb.connect(*[(b, 0) for b in chain])
    tb.run()
    return text, sink.array()


def main(argv=None):
    ap = argparse.ArgumentParser(prog="ldpc_dump", description=__doc__.split("\n\n")[0])
    ap.add_argument("--chars", type=int, default=4, help="characters (4 per codeword)")
    ap.add_argument("--method", type=int, default=1,
                    help="0 LogDomain (min-sum), 1 SumProduct, 2 BitFlip, 3 Hard")
    ap.add_argument("--iterations", type=int, default=10)
    ap.add_argument("--ebn0", type=float, default=None, help="add AWGN at this Eb/N0 (dB)")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--precision", type=int, default=0, help="0 f64, 1 f32, 2 f64 libm")
    ap.add_argument("--check", action="store_true", help="exit 1 if the text differs")
    a = ap.parse_args(argv)
    sent, got = run(a.chars, a.method, a.iterations, a.ebn0, a.seed, a.precision)
    sys.stdout.write("\n")
    if a.check:
        same = len(got) == len(sent) and bool((got == sent).all())
        sys.stderr.write("sent %r\nrecv %r\n%s\n" % (bytes(sent), bytes(got),
                                                     "OK" if same else "MISMATCH"))
        return 0 if same else 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
