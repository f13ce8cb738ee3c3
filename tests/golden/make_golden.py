#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run in the development container (it reads /root/reference as TEXT to lift
the data the reference holds: its H matrices, source-bit matrices and the QA
known-answer tuples).  The GPU box never runs this; it only loads the .npz
files written here (numpy, allow_pickle=False).

Outputs
  reference_data.npz  H matrices hData1..5 (apps/test_data.h), the decoder's
                      active 32x64 H (lib/ldpc_decoder_cb_impl.cc:63-96),
                      the commented 8x16 QA H (:48-57), dSourceData2..5, and
                      the QA KATs (python/qa_ldpc_encoder_bc.py:21-41,
                      python/qa_ldpc_decoder_cb.py:20-43).
  frames_default.npz  seeded noisy frames for the default (reordered) H at
                      0/2/4 dB with every method's expected hard bits,
                      packed bytes, iterations executed and syndrome weight,
                      at 5 and 50 iterations (C oracle; a subset cross-checked
                      against the pure-Python restatement before writing).
  frames_other.npz    the same for hData1, hData2, hData3, hData5 at 2 dB.
  streams.npz         complex streams (misaligned start, inverted polarity,
                      burst -> resync) with the restated general_work output.
"""
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import oracle as orc  # noqa: E402
from oracle import ldpc_oracle_py as pyo  # noqa: E402

REF = "/root/reference"


def _ints(txt):
    return np.array([int(x) for x in re.findall(r"-?\d+", txt)], dtype=np.int64)


def parse_test_data():
    src = open(os.path.join(REF, "apps/test_data.h")).read()
    out = {}
    dims = {}
    for m in re.finditer(r"const int ([MN]\d) = (\d+);", src):
        dims[m.group(1)] = int(m.group(2))
    for k in range(1, 6):
        M, N = dims["M%d" % k], dims["N%d" % k]
        body = re.search(r"const int hData%d\[\] = \{(.*?)\};" % k, src, re.S).group(1)
        out["hData%d" % k] = _ints(body).reshape(M, N).astype(np.uint8)
        m = re.search(r"const int dSourceData%d\[\] = \{(.*?)\};" % k, src, re.S)
        if m:
            v = _ints(m.group(1))
            out["dSourceData%d" % k] = v.reshape(M, -1).astype(np.uint8)  # M rows x frames
    return out


def parse_decoder_h():
    src = open(os.path.join(REF, "lib/ldpc_decoder_cb_impl.cc")).read()
    # the commented 8x16 block and the active 32x64 block (:48-57, :63-96)
    blocks = re.findall(r"const int h_data\[\] = \{(.*?)\};", src, re.S)
    h8 = _ints(blocks[0]).reshape(8, 16).astype(np.uint8)
    h32 = _ints(blocks[1]).reshape(32, 64).astype(np.uint8)
    return h8, h32


def parse_kats():
    enc = open(os.path.join(REF, "python/qa_ldpc_encoder_bc.py")).read()
    data = [int(x, 2) for x in re.findall(r"0b([01]{8})", enc.split("mod_data")[0])]
    def tuple_block(name, txt):
        body = re.search(name + r"\s*=\s*\((.*?)\)\s*\)", txt, re.S).group(1)
        return _ints(body).reshape(8, 8)
    mod_data = tuple_block("mod_data", enc)
    mod_check = tuple_block("mod_check", enc)
    dec = open(os.path.join(REF, "python/qa_ldpc_decoder_cb.py")).read()
    exp = [int(x, 2) for x in re.findall(r"0b([01]{8})", dec)]
    dmod_data = tuple_block("mod_data", dec)
    dmod_check = tuple_block("mod_check", dec)
    assert (dmod_data == mod_data).all() and (dmod_check == mod_check).all()
    return (np.array(data, np.uint8), mod_check.astype(np.int8), mod_data.astype(np.int8),
            np.array(exp, np.uint8))


def synth_frames(Hr, L, U, B, ebn0_db, seed):
    """Seeded synthetic frames with the reference's noise convention
    (apps/ldpc_lapack.cpp:625-642): BPSK 1->+1, 0->-1, sigma = sqrt(10^(-EbN0/10))."""
    M, N = Hr.shape
    rng = np.random.Generator(np.random.PCG64(seed))
    data = rng.integers(0, 2, size=(B, N - M), dtype=np.uint8)
    cw = orc.encode(Hr, L, U, data)
    x = 2.0 * cw.astype(np.float64) - 1.0
    sigma = np.sqrt(10.0 ** (-ebn0_db / 10.0))
    y = (x + sigma * rng.standard_normal(size=(B, N))).astype(np.float32)
    return data, cw, y


def cross_check(Hr, frames, method, iters, expect, count):
    """Pure-Python restatement must agree bit for bit with the C oracle."""
    for b in range(min(count, frames.shape[0])):
        rx = [float(v) for v in frames[b]]
        v, used = pyo.decode(method, Hr.tolist(), rx, iters)
        assert list(expect["bits"][b]) == v, (method, b)
        assert expect["iters"][b] == used, (method, b, used, expect["iters"][b])


def main():
    td = parse_test_data()
    h8, h32 = parse_decoder_h()
    assert (h32 == td["hData4"]).all(), "decoder H != hData4"
    assert (h8 == td["hData3"]).all(), "commented decoder H != hData3"
    kat_data, kat_check, kat_mdata, kat_expect = parse_kats()
    ref = dict(td)
    ref.update(decoder_h=h32, qa_h=h8, kat_data=kat_data, kat_mod_check=kat_check,
               kat_mod_data=kat_mdata, kat_expected=kat_expect)
    np.savez_compressed(os.path.join(HERE, "reference_data.npz"), **ref)

    # --- default H noisy frames -------------------------------------------
    Hr, chosen, L, U = orc.reorder_h(h32)
    pyHr, pychosen, _, _ = pyo.reorder_h(h32.tolist())
    assert (np.array(pyHr) == Hr).all() and list(chosen) == pychosen
    fd = dict(H_reordered=Hr, chosen=chosen, L=L, U=U)
    B = 96
    for k, db in enumerate((0.0, 2.0, 4.0)):
        data, cw, y = synth_frames(Hr, L, U, B, db, seed=1000 + k)
        tag = "db%d" % int(db)
        fd["%s_llr" % tag] = y
        fd["%s_data" % tag] = data
        for method in (0, 1, 2, 3):
            for iters in (5, 50):
                res = orc.decode_batch(method, Hr, y, iters, want_post=True)
                cross_check(Hr, y, method, iters, res, count=6 if method in (0, 1) else 3)
                key = "%s_m%d_i%d" % (tag, method, iters)
                for f in ("bits", "packed", "iters", "synd", "post"):
                    fd["%s_%s" % (key, f)] = res[f]
    np.savez_compressed(os.path.join(HERE, "frames_default.npz"), **fd)

    # --- the other H matrices of apps/test_data.h ---------------------------
    fo = {}
    for name in ("hData1", "hData2", "hData3", "hData5"):
        H = td[name]
        Hr2, ch2, L2, U2 = orc.reorder_h(H)
        fo["%s_H_reordered" % name] = Hr2
        fo["%s_chosen" % name] = ch2
        try:
            data, cw, y = synth_frames(Hr2, L2, U2, 24, 2.0, seed=77)
        except ValueError:
            # rank-deficient parity block: decode raw noise instead
            rng = np.random.Generator(np.random.PCG64(77))
            y = rng.standard_normal(size=(24, H.shape[1])).astype(np.float32)
        fo["%s_llr" % name] = y
        for method in (0, 1, 2, 3):
            res = orc.decode_batch(method, Hr2, y, 20, want_post=True)
            cross_check(Hr2, y, method, 20, res, count=3)
            for f in ("bits", "packed", "iters", "synd", "post"):
                fo["%s_m%d_%s" % (name, method, f)] = res[f]
    np.savez_compressed(os.path.join(HERE, "frames_other.npz"), **fo)

    # --- streams through the restated general_work -------------------------
    rng = np.random.Generator(np.random.PCG64(4242))
    st = {}

    def make_stream(nframes, db, lead, invert=False, burst_at=None, burst_len=0, shift=0):
        _, _, y = synth_frames(Hr, L, U, nframes, db, seed=int(rng.integers(1 << 30)))
        s = y.reshape(-1).astype(np.float32)
        if invert:
            s = -s
        parts = [rng.standard_normal(lead).astype(np.float32), s[: (burst_at or nframes) * 64]]
        if burst_at is not None:
            parts.append(rng.standard_normal(burst_len).astype(np.float32))
            parts.append(rng.standard_normal(shift).astype(np.float32))
            parts.append(s[burst_at * 64:])
        re_ = np.concatenate(parts)
        im = (0.01 * rng.standard_normal(re_.size)).astype(np.float32)
        return (re_ + 1j * im).astype(np.complex64)

    streams = {
        "aligned": make_stream(24, 6.0, 0),
        "offset": make_stream(24, 6.0, 17),
        "inverted": make_stream(24, 6.0, 5, invert=True),
        "burst": make_stream(40, 6.0, 3, burst_at=12, burst_len=64 * 14, shift=23),
        "noisy": make_stream(24, 1.0, 9),
    }
    for name, s in streams.items():
        st["%s_in" % name] = s
        for method in (0, 1, 2, 3):
            whole = orc.run_stream(method, Hr, s, iterations=5)
            chunks = rng.integers(1, 200, size=len(s) // 50 + 2)
            parts = orc.run_stream(method, Hr, s, iterations=5, chunks=chunks)
            assert (whole == parts).all(), "chunking changed the restated output"
            st["%s_m%d_out" % (name, method)] = whole
    np.savez_compressed(os.path.join(HERE, "streams.npz"), **st)
    print("wrote fixtures to", HERE)


if __name__ == "__main__":
    main()
