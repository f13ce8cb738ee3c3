#!/usr/bin/env python3
"""Benchmark of the decode hot path (BASELINE.json configs[1] / [2]).

One "step" = one pass of the decoder over one batch of synthetic frames
already resident in HBM: B = 4096 frames of the reference's default 32x64 H
(reordered as the block does), sum-product (method 1), 50-iteration cap with
the reference's per-frame early exit, Eb/N0 = 2 dB with the reference noise
convention (sigma = sqrt(10^(-EbN0/10)), apps/ldpc_lapack.cpp:635-642).

  python bench.py [--gpus N --steps K --warmup W] [--inflight D] [--strong]

Data are made on the GPU before timing: Philox bits (ldpc_random_bits) ->
systematic GF(2) encode (ldpc_encode_device) -> BPSK + AWGN
(ldpc_bpsk_awgn); the first frames are cross-checked against the host
encoder.  D distinct batches are made (D = --inflight, default 4); step k
posts batch k mod D to the decoder's frame ring (ldpc_ring_post,
csrc/ldpc_ring.hip): ONE persistent launch per timed region decodes every
posted batch, frames of all batches from one device queue, so the frames of
the next batch fill the SIMDs the previous batch's last long frames leave
idle (a streaming receiver's steady state) and only the region's end has a
tail.  Every step decodes its whole batch into its own outputs; the
single-batch latency (one launch per batch, one at a time) is reported
beside it.

N > 1 runs under torch.distributed.run, one rank per GPU.  Weak scaling
(default): every rank decodes its own B frames.  --strong: one global batch
of B frames is split with ldpc_ece535a.dist.shard_range.  No collective runs
in the data path; after the timed loop ldpc_ece535a.dist.gather_outputs
all-gathers the packed outputs and all-reduces the counters over RCCL (the
"final throughput gather"), and the max over ranks of the timed wall time is
taken.  Rank 0 prints ONE JSON line; `value` = info bits of all frames all
ranks decoded / that max.

roofline (small-code path): the kernel keeps every edge message in LDS /
VGPRs, so HBM does not bound it; f64 VALU issue does.  achieved = VALU issue
cycles per launch (rocprofv3 PMC instruction counts, profiles/pmc_counters.json)
weighted by the issue costs measured on gfx950 at four waves per SIMD
(tools/ubench_valu.hip, profiles/round3/ubench_valu.txt: 4.31 cycles per f64
add/mul/fma wave-instruction, 16.3 per f64 transcendental, the kernel's own
hot-path mix for the other VALU instructions, ~3.5, tools/isa_hot.py) / the
per-launch time; peak = 1024 SIMDs x 2.4 GHz.  frac_nominal is the same with
the ISA's nominal costs (4 / 16 / 2).  The SURVEY 8(d) byte model stays as a
labelled secondary figure (equivalent streaming bandwidth).  Config 4
(--code dvbs2) is memory-bound: measured traffic (PMC, taken at the bench's
own chunk count) over the decode time against the 8 TB/s peak.
cpu_baseline: the C oracle (oracle/, a dense double restatement of the
reference decoder) decoding the same frames on the host's cores.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
# LDPC_PKG_DIR: an alternative build of the package (tools/ab.sh A/B runs)
sys.path.insert(0, os.environ.get("LDPC_PKG_DIR", os.path.join(REPO, "gr-ldpc_ece535a_amd")))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
SIMDS, CLOCK_HZ = 1024, 2.4e9  # 256 CUs x 4 SIMDs, max clock
F64_PEAK_TFLOPS = 78.6         # MI355X FP64 vector spec
# VALU issue cycles per wave64 instruction on gfx950 (profiles/round2/ubench_f64.txt)
# issue cycles per wave64 instruction at 4 waves/SIMD (tools/ubench_f64.hip,
# tools/ubench_valu.hip; profiles/round3/ubench_valu.txt): f64 add/mul/fma
# 4.31, v_rcp_f64 16.3; "other VALU" (the PMC's remainder: 32-bit VOP2 ops at
# 2.75, VOP3 / 64-bit ones -- compares, e64 selects, converts, 64-bit moves --
# at 4.31) takes the kernel's hot-path mix (tools/isa_hot.py, recorded with
# the counters) or this default
ISSUE_F64, ISSUE_TRANS64, ISSUE_OTHER = 4.31, 16.3, 3.5
NOMINAL_F64, NOMINAL_TRANS64, NOMINAL_OTHER = 4.0, 16.0, 2.0  # the ISA's nominal costs
METRIC = "decoded info Mbit/s @ 50 BP iters, batch=4096; achieved HBM GB/s vs peak"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    # the first ~100-200 launches of a fresh process run slower while the clock
    # ramps (profiles/round1/warmup_clock.txt); the default warmup covers them
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--inflight", type=int, default=4,
                    help="batches in flight (consecutive steps on alternating streams)")
    ap.add_argument("--strong", action="store_true",
                    help="N > 1: split one global batch over the ranks (default: weak scaling)")
    ap.add_argument("--code", choices=["default", "dvbs2"], default="default",
                    help="default: the reference's 32x64 H (config 2); dvbs2: the DVB-S2-size "
                         "code of config 4 (synthetic rate-1/2 address table)")
    ap.add_argument("--batch", type=int, default=None, help="default 4096 (1024 for dvbs2)")
    ap.add_argument("--method", type=int, default=None, help="default 1 (0 for dvbs2)")
    ap.add_argument("--no-config4", action="store_true", help="skip the config-4 variant")
    ap.add_argument("--no-block", action="store_true", help="skip the block-throughput variant")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 variant")
    ap.add_argument("--precision", choices=["f64", "f64libm", "f64fast", "f32"], default="f64",
                    help="f64: LDPC_PREC_F64 (default, bit-exact), f64libm: LDPC_PREC_F64_LIBM "
                         "(exact, unbatched divisions), f64fast: LDPC_PREC_F64_FAST (compact "
                         "tanh/log, not exact), f32")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--et-period", type=int, default=1)
    ap.add_argument("--ebn0", type=float, default=2.0)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--waves-per-cu", type=int, default=0)
    ap.add_argument("--schedule", type=int, default=0, help="0 auto, 1 wave/frame, 2 workgroup/frame")
    ap.add_argument("--sweep-batch", default="",
                    help="comma list of B: latency/throughput sweep to stderr")
    ap.add_argument("--sweep-inflight", default="",
                    help="comma list of in-flight depths: per-batch time table to stderr")
    ap.add_argument("--sweep-modes", default="1:f64,1:f32,0:f64",
                    help="method:precision list for the sweeps")
    ap.add_argument("--sweep-config5", default="",
                    help="comma list of B: config 5 (syndrome check every 5 iterations, mixed "
                         "Eb/N0 0..4 dB per frame) latency/throughput table to stderr")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "pmc_counters.json"))
    return ap.parse_args(argv)


# --------------------------------------------------------------------------
# synthetic data
# --------------------------------------------------------------------------
def sigma_of(ebn0):
    """The reference's noise convention (apps/ldpc_lapack.cpp:629-636)."""
    return float(np.sqrt(10.0 ** (-ebn0 / 10.0)))


_STREAMS = {}


def side_stream(torch, dev):
    """The one torch stream the bench makes its data on (every synth_device
    call)."""
    key = str(dev)
    if key not in _STREAMS:
        _STREAMS[key] = torch.cuda.Stream(dev)
    return _STREAMS[key]


def ring_stream(torch, dev):
    """The stream the frame ring's sessions follow and the timing events sit on."""
    key = "ring" + str(dev)
    if key not in _STREAMS:
        _STREAMS[key] = torch.cuda.Stream(dev)
    return _STREAMS[key]


def synth_device(L, torch, dec, B, ebn0, seed, dev, check_frames=64):
    """Frames made on the GPU: Philox bits -> ldpc_encode_device -> BPSK +
    AWGN.  ebn0 may be a scalar or a per-frame array (config 5).  Returns
    (device float32 (B, N), device data bits (B, K)).  The first
    check_frames codewords are compared with the host encoder."""
    K, N = dec.K, dec.N
    # one explicit (non-null) stream for every step: a NULL stream argument
    # would mean the context's own stream for ldpc_encode_device
    st = side_stream(torch, dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    with torch.cuda.stream(st):
        d_bits = torch.empty((B, K), dtype=torch.uint8, device=dev)
        d_cw = torch.empty((B, N), dtype=torch.uint8, device=dev)
        d_y = torch.empty((B, N), dtype=torch.float32, device=dev)
        if B == 0:
            return d_y, d_bits
        L.random_bits(d_bits.data_ptr(), B * K, seed, sp)
        dec.encode_device(d_bits.data_ptr(), B, d_cw.data_ptr(), sp)
        if np.ndim(ebn0) == 0:
            L.bpsk_awgn(d_cw.data_ptr(), B * N, sigma_of(ebn0), seed * 2 + 1, d_y.data_ptr(), sp)
        else:  # unit-variance noise, scaled per frame
            L.bpsk_awgn(d_cw.data_ptr(), B * N, 1.0, seed * 2 + 1, d_y.data_ptr(), sp)
            x = 2.0 * d_cw.to(torch.float32) - 1.0
            s = torch.from_numpy(np.sqrt(10.0 ** (-np.asarray(ebn0, np.float64) / 10.0))
                                 .astype(np.float32)).to(dev)[:, None]
            d_y = x + (d_y - x) * s
    st.synchronize()
    n = min(B, check_frames)
    if n:
        bits = d_bits[:n].cpu().numpy()
        cw = d_cw[:n].cpu().numpy()
        if dec.N <= 4096:  # small enough for the dense host encoder
            host = L.encode(dec.H, bits)
        else:  # large codes: the IRA / DVB-S2 accumulator encoder
            from ldpc_ece535a import codes
            host = codes.ira_encode((dec.M, dec.N, dec.row_ptr, dec.col_idx), bits)
        if not (host == cw).all():
            raise RuntimeError("device encoder disagrees with the host encoder")
        if not (cw[:, dec.M:] == bits).all():
            raise RuntimeError("systematic part of the device codewords is not the data")
    return d_y, d_bits


def synth(Hr, B, ebn0, seed):
    """Host-made frames (tests and tools): data ~ Bernoulli(1/2) (PCG64),
    GF(2) encode through the product's ldpc_encode, BPSK 1->+1, AWGN with the
    reference sigma.  Returns (float32 (B, N), data bits (B, K))."""
    import ldpc_ece535a as L
    M, N = Hr.shape
    rng = np.random.Generator(np.random.PCG64(seed))
    data = rng.integers(0, 2, size=(B, N - M), dtype=np.uint8)
    cw = L.encode(Hr, data)
    y = (2.0 * cw.astype(np.float64) - 1.0 + sigma_of(ebn0) * rng.standard_normal((B, N)))
    return y.astype(np.float32), data


def bytes_per_iter(E, N, prec):
    return 16 * E + 6 * N if prec == 1 else 32 * E + 10 * N


# --------------------------------------------------------------------------
# timing (shared with tests/test_bench_dist.py, which runs it on the CPU)
# --------------------------------------------------------------------------
def timed_steps(step, steps, warmup, sync, dist=None):
    """W untimed steps, then exactly K timed steps bracketed by a barrier
    and a device synchronize on both sides.  Returns the wall time (s)."""
    for k in range(warmup):
        step(k)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(warmup + k)
    sync()
    if dist is not None:
        dist.barrier()
    return time.perf_counter() - t0


def reduce_results(dist, packed, counters, wall, device=None):
    """The final throughput gather: all-gather the packed outputs
    (ldpc_ece535a.dist.gather_outputs), all-reduce the counters, max of the
    wall times.  Single process: returned as is."""
    if dist is None:
        return packed, [float(c) for c in counters], wall
    import torch
    from ldpc_ece535a.dist import gather_outputs
    full, c = gather_outputs(dist, packed, counters, device)
    dev = packed.device if device is None else device
    w = torch.tensor([float(wall)], dtype=torch.float64, device=dev)
    dist.all_reduce(w, op=dist.ReduceOp.MAX)
    return full, c, float(w.item())


def gathered_parity(L, torch, orc, dec, args, dev, full, world, Hr, csr, threads, sample=256):
    """Rank 0, N > 1: the all-gathered outputs (every rank's first batch, in
    rank order) against the oracle.  Each rank's batch is made again here from
    its seed (synth_device is deterministic) and the first `sample` frames of
    every rank are decoded on the CPU."""
    full = full.cpu().numpy()
    pos, frames, bad = 0, 0, 0
    for rk in range(world):
        _, Br = plan_batch(args.batch, world, rk, args.strong)
        y = synth_device(L, torch, dec, Br, args.ebn0, args.seed + 7919 * rk, dev)[0]
        nb = min(Br, sample)
        llr = y[:nb].cpu().numpy()
        if csr is not None:
            ref = orc.decode_batch_sparse(args.method, csr[2], csr[3], csr[0], csr[1], llr,
                                          args.iters, nthreads=threads, want_bits=False)
        else:
            ref = orc.decode_batch(args.method, Hr, llr, args.iters, nthreads=threads,
                                   et_period=args.et_period)
        bad += int((ref["packed"] != full[pos:pos + nb]).any(axis=1).sum())
        frames += nb
        pos += Br
    return {"ranks": world, "frames": frames, "gathered_frames": int(full.shape[0]),
            "packed_mismatch_frames": bad,
            "checker": "first %d frames of every rank's batch (made again from the rank's seed) "
                       "vs the oracle, compared with the all-gathered outputs" % sample}


def plan_batch(B, world, rank, strong):
    """Frames this rank decodes: (offset in the global batch, count).  Weak
    scaling: every rank its own B frames; strong: shard_range of one B."""
    if not strong or world == 1:
        return rank * B, B
    from ldpc_ece535a.dist import shard_range
    lo, hi = shard_range(B, rank, world)
    return lo, hi - lo


def time_ring(dec, torch, inputs, B, method, iters, et, prec, steps, warmup, dist=None,
              inflight=None, streams=None):
    """Decode `steps` batches through the frame ring (ldpc_ring_*): step k
    posts inputs[k % D] with outputs of its own.  One ring session per region
    (the warmup's, the timed steps'): ldpc_ring_begin at the region's first
    step, ldpc_ring_end after its last, so the closing synchronize of the
    region waits for the launch to end, i.e. for every batch of the region.
    Returns dict(wall, span_ms, per_launch_ms, iters, outs) like
    time_decoder: span_ms from a HIP event recorded on the session's stream
    before the timed session begins to one recorded after it ends (the
    launch follows the first and the second follows the launch),
    per_launch_ms = span_ms / steps (per batch), outs[d] = (packed, iters,
    synd) of the last timed batch of inputs[d]."""
    D = len(inputs)
    dev = inputs[0].device
    # the session's stream (torch's default stream is the null stream, which
    # the ring's non-blocking streams do not order against)
    st = ring_stream(torch, dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    # outputs of their own for every step of both regions: a timed batch's
    # outputs can only come from the timed session
    P = max(1, steps + warmup)
    pool = [(torch.empty((B, dec.KB), dtype=torch.uint8, device=dev),
             torch.empty(B, dtype=torch.int32, device=dev),
             torch.empty(B, dtype=torch.int32, device=dev)) for _ in range(P)]
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    for ev in (e0, e1):  # created before the timed region
        ev.record(st)
    last = {}

    def step(k):
        if k == 0 or k == warmup:
            if k == warmup:
                e0.record(st)
            dec.ring_begin(method=method, max_iters=iters, et_period=et, precision=prec, stream=sp)
        pk, it, sy = pool[k]
        dec.ring_post(inputs[k % D].data_ptr(), B, pk.data_ptr(), it.data_ptr(), sy.data_ptr())
        if k >= warmup:
            last[k % D] = k
        if k == warmup - 1 or k == warmup + steps - 1:
            dec.ring_end()
            if k == warmup + steps - 1:
                e1.record(st)

    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    wall = timed_steps(step, steps, warmup, sync, dist)
    span = e0.elapsed_time(e1) if steps else 0.0
    outs = [pool[last[d]] if d in last else pool[0] for d in range(D)]
    return dict(wall=wall, span_ms=span, per_launch_ms=span / max(1, steps),
                iters=outs[0][1].cpu().numpy(), outs=outs, ring=dec.ring_info())


def time_decoder(dec, torch, inputs, B, method, iters, et, prec, steps, warmup, dist=None,
                 inflight=1, streams=None):
    """Decode `steps` batches with `inflight` batches in flight: step k
    decodes inputs[k % D] on stream k % D into that stream's output buffers.
    Returns dict(wall, span_ms, per_launch_ms, iters, outs) where span_ms is
    the device time from the first launch's start (a HIP event on the first
    timed step's stream, which each other stream waits for before its first
    launch) to the last launch's end (one event per stream) and per_launch_ms = span_ms / steps.  outs[d] = (packed, iters,
    synd) of the last decode of batch d."""
    D = max(1, inflight)
    dev = inputs[0].device
    if streams is None:
        streams = [torch.cuda.Stream(dev) for _ in range(D)]
    sps = [ctypes.c_void_p(s.cuda_stream) for s in streams]
    outs = [(torch.empty((B, dec.KB), dtype=torch.uint8, device=dev),
             torch.empty(B, dtype=torch.int32, device=dev),
             torch.empty(B, dtype=torch.int32, device=dev)) for _ in range(D)]

    # at most two launches queued per stream: the host waits for step k - 2D
    # before it enqueues step k (a pipeline's depth, not an unbounded backlog
    # of hundreds of launches)
    done_ev = [torch.cuda.Event() for _ in range(2 * D)]

    def step(k):
        d = k % D
        if k >= 2 * D:
            done_ev[k % (2 * D)].synchronize()
        pk, it, sy = outs[d]
        dec.decode_device(inputs[d % len(inputs)].data_ptr(), B, pk.data_ptr(), method=method,
                          max_iters=iters, et_period=et, precision=prec, d_iters=it.data_ptr(),
                          d_synd=sy.data_ptr(), stream=sps[d])
        done_ev[k % (2 * D)].record(streams[d])

    e0 = torch.cuda.Event(enable_timing=True)
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(D)]
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    marks = {}

    # every event exists before the timed region (a torch event is created at
    # its first record): no event creation inside the timed steps
    for ev in done_ev + [e0] + ends:
        ev.record(streams[0])

    def timed_step(k):
        # first timed step: the start event on its stream; each other stream
        # waits on it right before its own first launch, so the first launch
        # is not queued behind the other streams' waits on the host
        d = k % D
        if k == warmup:
            e0.record(streams[d])
        elif k < warmup + D:
            streams[d].wait_event(e0)
        step(k)
        if k == warmup + steps - 1:
            for s, e in zip(streams, ends):
                e.record(s)
            marks["done"] = True

    wall = timed_steps(timed_step, steps, warmup, sync, dist)
    span = max(e0.elapsed_time(e) for e in ends) if marks else 0.0
    return dict(wall=wall, span_ms=span, per_launch_ms=span / max(1, steps),
                iters=outs[0][1].cpu().numpy(), outs=outs,
                streams_distinct=len(set(s.cuda_stream for s in streams)))


# --------------------------------------------------------------------------
# measurement helpers
# --------------------------------------------------------------------------
def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


def physical_cores(cpus):
    """Distinct (package, core) pairs among the given logical CPUs."""
    seen = set()
    for c in cpus:
        base = "/sys/devices/system/cpu/cpu%d/topology/" % c
        try:
            seen.add((open(base + "physical_package_id").read().strip(),
                      open(base + "core_id").read().strip()))
        except OSError:
            return None
    return len(seen)


def cpu_share():
    """(threads to use, logical CPUs visible).  The GPU box grants each GPU a
    CPU share and exports it as OMP_NUM_THREADS (16 per GPU) while
    sched_getaffinity shows the whole machine; the share is used."""
    try:
        visible = len(os.sched_getaffinity(0))
    except AttributeError:
        visible = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    n = int(share) if share and share.isdigit() and int(share) > 0 else visible
    return max(1, min(n, visible)), visible


def load_pmc(path, key):
    try:
        return json.load(open(path)).get(key)
    except (OSError, ValueError):
        return None


def valu_roofline(pmc, per_launch_ms, w_other=None):
    """VALU issue-cycle roofline from PMC instruction counts per launch."""
    w_other = ISSUE_OTHER if w_other is None else w_other
    f64 = sum(pmc.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                         "SQ_INSTS_VALU_FMA_F64"))
    trans = pmc.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
    other = max(0.0, pmc["SQ_INSTS_VALU"] - f64 - trans)
    cycles = ISSUE_F64 * f64 + ISSUE_TRANS64 * trans + w_other * other
    nominal = NOMINAL_F64 * f64 + NOMINAL_TRANS64 * trans + NOMINAL_OTHER * other
    peak = SIMDS * CLOCK_HZ / 1e9
    ach = cycles / (per_launch_ms * 1e-3) / 1e9
    flop = 64.0 * (2.0 * pmc.get("SQ_INSTS_VALU_FMA_F64", 0.0) +
                   pmc.get("SQ_INSTS_VALU_ADD_F64", 0.0) + pmc.get("SQ_INSTS_VALU_MUL_F64", 0.0))
    return {"bound": "valu", "achieved": round(ach, 1), "peak": peak,
            "unit": "G SIMD-cycles/s of VALU issue (f64-weighted)", "frac": round(ach / peak, 4),
            "issue_cycles_per_launch": round(cycles),
            "frac_nominal": round(nominal / (per_launch_ms * 1e-3) / 1e9 / peak, 4),
            "nominal_weights": "f64 add/mul/fma %g, f64 transcendental %g, other VALU %g cycles "
                               "per wave64 instruction" % (NOMINAL_F64, NOMINAL_TRANS64,
                                                          NOMINAL_OTHER),
            "f64_tflops": round(flop / (per_launch_ms * 1e-3) / 1e12, 2),
            "f64_tflops_frac": round(flop / (per_launch_ms * 1e-3) / 1e12 / F64_PEAK_TFLOPS, 4),
            "weights": "issue cycles per wave64 instruction: f64 add/mul/fma %g, f64 "
                       "transcendental %g, other VALU %g (profiles/round3/ubench_valu.txt; "
                       "'other' = the kernel's hot-path VOP2/VOP3 mix, tools/isa_hot.py)"
                       % (ISSUE_F64, ISSUE_TRANS64, w_other)}


class _quiet_stdout:
    """The block prints the reference's sync messages on stdout
    (lib/ldpc_decoder_cb_impl.cc:171-200); keep them out of the JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        null = os.open(os.devnull, os.O_WRONLY)
        os.dup2(null, 1)
        os.close(null)

    def __exit__(self, *exc):
        os.dup2(self.saved, 1)
        os.close(self.saved)


def drive_stream(blk, cx, B):
    """Feed a continuous stream to the block as a GR scheduler does: calls of
    at most B frames of input, unconsumed input carried over.  The first call
    (acquisition from a fresh block) is not timed.  Returns (seconds, output
    bytes, calls, launches, windows decoded) of the timed calls."""
    chunk = B * 64
    pos = 0
    o, used = blk.general_work(B * 4, cx[:chunk])
    pos += used
    outs = [o]
    l0, f0 = blk.launches, blk.frames_decoded
    made = calls = 0
    t0 = time.perf_counter()
    while pos + 64 <= cx.size:
        o, used = blk.general_work(B * 4, cx[pos:pos + chunk])
        pos += used
        made += o.size
        calls += 1
        outs.append(o)
        if used == 0:
            break
    dt = time.perf_counter() - t0
    drive_stream.last_out = np.concatenate(outs)  # every byte, the untimed first call's too
    return (dt, made, calls, blk.launches - l0, blk.frames_decoded - f0)


def block_variant(L, torch, blocks, dev, args, d_y, B, reps=4, cpu_frames=1024):
    """The drop-in block's own throughput: ldpc_decoder_cb (method 1, f64; the
    bench's iteration cap, and the reference block's own 5) general_work over
    a continuous stream of gr_complex frames in host memory, as a GNU Radio
    scheduler drives it
    (lib/ldpc_decoder_cb_impl.cc:133-234): calls of B frames of input,
    packed bytes out.  Beside each: the reference block restated on the CPU
    (oracle Block, one core: the state machine is sequential) over the
    stream's first `cpu_frames` frames of samples -- its rate, and whether its
    bytes equal the GPU block's for that prefix (the block is causal)."""
    out = {}
    orc = None
    if cpu_frames and not args.no_cpu_baseline:
        sys.path.insert(0, REPO)
        from oracle import oracle as orc
    # (name, Eb/N0, iterations, CPU sample in frames: ~3-15 s of one core each)
    runs = (("in-sync stream (4 dB)", 4.0, args.iters, cpu_frames, None),
            ("2 dB stream (sync losses)", 2.0, args.iters, cpu_frames // 2, None),
            # make(method) as the reference builds it: 5 iterations (:40)
            ("make(1) defaults, 5 iterations, 4 dB", 4.0, 5, cpu_frames, None),
            # the same stream with a launch per round instead of the call's
            # window server (LDPC_BLOCK_SERVE=0: the A/B of the server)
            ("make(1) defaults, 5 iterations, 4 dB, launch per round", 4.0, 5, cpu_frames, "0"))
    last_ref = None
    for name, ebn0, iters, n_cpu, serve in runs:
        dec = L.Decoder(device=dev.index or 0)
        y, _ = synth_device(L, torch, dec, (reps + 1) * B, ebn0, args.seed + 77, dev,
                            check_frames=0)
        Hr = dec.H.copy()  # the block's H: the reference default, reordered (:98-106)
        dec.close()
        stream = np.zeros(2 * y.numel(), np.float32)
        stream[0::2] = y.cpu().numpy().ravel()
        cx = stream.view(np.complex64)
        if serve is not None:
            os.environ["LDPC_BLOCK_SERVE"] = serve
        try:
            blk = blocks.ldpc_decoder_cb(1, iterations=iters, precision=0, device=dev.index or 0)
        finally:
            os.environ.pop("LDPC_BLOCK_SERVE", None)
        dt, made, calls, launches, windows = drive_stream(blk, cx, B)
        out[name] = {"Mbit/s": round(made * 8 / dt / 1e6, 2), "calls": calls,
                     "ms_per_call": round(dt / max(1, calls) * 1e3, 4),
                     "launches_per_call": round(launches / max(1, calls), 2),
                     "windows_per_output_frame": round(windows / max(1, made // 4), 2),
                     "bytes_out": int(made)}
        if serve is not None and last_ref is not None:  # the earlier run's CPU restatement, same stream
            gpu_bytes = drive_stream.last_out
            out[name]["bytes_equal_cpu_prefix"] = bool(
                gpu_bytes.size >= last_ref.size and (gpu_bytes[:last_ref.size] == last_ref).all())
            continue
        if orc is not None:
            gpu_bytes = drive_stream.last_out
            sample = cx[:n_cpu * 64]
            t0 = time.perf_counter()
            stats = {}
            ref = orc.run_stream(1, Hr, sample, iterations=iters, stats=stats)
            cpu_s = time.perf_counter() - t0
            last_ref = ref
            out[name]["cpu_baseline"] = {
                "Mbit/s": round(ref.size * 8 / cpu_s / 1e6, 5), "cores": 1, "kind": "port",
                "sample": "the stream's first %d frames of samples through the restated "
                          "general_work (oracle Block, :133-234), one thread" % n_cpu,
                "bytes": int(ref.size),
                # the yardstick for windows_per_output_frame: the reference
                # loop's own decodes (one per step, two on a "-tx" retry)
                "decodes_per_output_frame": round(stats["decodes"] / max(1, ref.size // 4), 3),
                "bytes_equal_gpu_prefix": bool(gpu_bytes.size >= ref.size and
                                               (gpu_bytes[:ref.size] == ref).all())}
    return out



def config4_variant(L, torch, dev, args, seed, steps=5, warmup=1, cpu_sample=0):
    """DVB-S2-like N=64800 code, min-sum, 1024 frames (config 4) on the
    large-code path.  Returns (results, check): check() runs the parity of
    the first `cpu_sample` frames vs the sparse oracle on the CPU -- called
    after every GPU measurement, so the GPU does not idle between them."""
    from ldpc_ece535a import codes
    csr = codes.dvbs2_like(0)
    dec = L.Decoder(csr=csr, device=dev.index or 0)
    pipe = dec.pipeline()
    B = 1024
    d_y, d_bits = synth_device(L, torch, dec, B, args.ebn0, seed, dev)
    data = d_bits.cpu().numpy()
    out = {}
    kept = {}
    for name, p in (("f64", 0), ("f32", 1)):
        r = time_decoder(dec, torch, [d_y], B, 0, args.iters, 1, p, steps, warmup)
        it = r["iters"]
        k = r["per_launch_ms"]
        alg = float(B * (4 * dec.N + dec.KB + 8) + it.sum() * bytes_per_iter(dec.E, dec.N, p))
        pk = r["outs"][0][0].cpu().numpy()
        out["min-sum " + name] = {
            "Mbit/s": round(B * dec.K * steps / r["wall"] / 1e6, 2), "ms_per_decode": round(k, 4),
            "mean_iters": round(float(it.mean()), 3), "max_iters": int(it.max()),
            "alg_GB/s": round(alg / (k * 1e-3) / 1e9, 1),
            "alg_GB/s_note": "edge-message byte model (SURVEY 8(d)) per decode time; the "
                             "narrow pipeline moves ~0.53x those bytes (DESIGN section 5)",
            "frames_decoded_to_sent_data": int((pk == np.packbits(data, axis=1)).all(axis=1).sum())}
        ent = load_pmc(args.pmc_json, "dvb0_f64_b1024_i50_db2") or {}
        t = ent.get("hbm_bytes_per_launch")
        # the measured traffic applies only to the pipeline configuration it
        # was taken at (frames per chunk, chunks in flight)
        if p == 0 and t and args.iters == 50 and args.ebn0 == 2.0 and ent.get("pipeline") == pipe:
            out["min-sum " + name]["measured_GB/s"] = round(t / (k * 1e-3) / 1e9, 1)
            out["min-sum " + name]["measured_frac_of_8TB/s"] = round(t / (k * 1e-3) / 8e12, 4)
            out["min-sum " + name]["measured_MB_per_frame_iteration"] = round(
                t / float(it.sum()) / 1e6, 3)
            out["min-sum " + name]["pmc_source"] = ent.get("source")
        if p == 0 and cpu_sample:
            kept = dict(y=d_y[:cpu_sample].cpu().numpy(), pk=pk[:cpu_sample],
                        it=it[:cpu_sample], K=dec.K)
    out["code"] = ("DVB-S2-like N=64800 K=32400 E=226799 (synthetic rate-1/2 address table, "
                   "ldpc_ece535a.codes.dvbs2_like(0)), B=1024, %d-iteration cap" % args.iters)
    out["pipeline"] = pipe
    dec.close()

    def check():
        if not kept:
            return
        from oracle import oracle as orc
        threads, _ = cpu_share()
        t0 = time.perf_counter()
        ref = orc.decode_batch_sparse(0, csr[2], csr[3], csr[0], csr[1], kept["y"], args.iters,
                                      nthreads=threads, want_bits=False)
        cpu_s = time.perf_counter() - t0
        out["min-sum f64"]["parity"] = {
            "frames": cpu_sample,
            "packed_mismatch_frames": int((ref["packed"] != kept["pk"]).any(axis=1).sum()),
            "iters_mismatch_frames": int((ref["iters"] != kept["it"]).sum()),
            "checker": "oracle sparse restatement (orc_decode_batch_sparse)",
            "cpu_Mbit/s": round(cpu_sample * kept["K"] / cpu_s / 1e6, 4), "cpu_threads": threads}
    return out, check


def config5_variant(L, torch, args, dev, sizes=(1, 16, 256, 4096, 65536), check_b=4096):
    """Config 5 (BASELINE configs[4]): the syndrome checked every 5
    iterations (et_period 5, the reference checks every iteration,
    lib/ldpc_decoder_cb_impl.cc:535-537 / :406-408), each frame at its own
    Eb/N0 drawn from {0,1,2,3,4} dB, one launch at a time (latency mode):
    latency per launch and Mbit/s per batch size, sum-product f64 (exact) and
    min-sum f64.  Returns (results, check): check() compares the first
    `check_b` frames of the B = check_b and largest launches with the
    oracle's et_period restatement (CPU, after the GPU work)."""
    # its own context (frame queues, streams): the headline's decoder is
    # left exactly as the other variants leave it
    dec = L.Decoder(device=dev.index or 0)
    rng = np.random.Generator(np.random.PCG64(args.seed + 5))
    Bmax = max(sizes)
    dbs = rng.integers(0, 5, size=Bmax).astype(np.float64)
    d_y, _ = synth_device(L, torch, dec, Bmax, dbs, args.seed + 100, dev, check_frames=0)
    dec.set_launch_mode(0)
    out = {"setup": "et_period 5, Eb/N0 per frame uniform over {0,1,2,3,4} dB, 50-iteration "
                    "cap, one launch at a time (latency mode); latency = HIP-event span per "
                    "launch"}
    kept = {}
    # one launch at a time, on a stream of its own
    c5_stream = [torch.cuda.Stream(dev)]
    for name, m in (("sum-product f64 (exact)", 1), ("min-sum f64", 0)):
        rows = {}
        for Bs in sizes:
            r, st = time_variant(time_decoder, dec, torch, [d_y[:Bs]], Bs, m, args.iters, 5, 0,
                                 10, 3, 1, streams=c5_stream)
            it = r["iters"]
            rows["B=%d" % Bs] = {"latency_ms": round(r["per_launch_ms"], 5),
                                 "Mbit/s": round(Bs * dec.K * st / r["wall"] / 1e6, 2),
                                 "mean_iters": round(float(it.mean()), 3), "steps": st}
            if Bs in (check_b, Bmax):
                kept[(m, Bs)] = (r["outs"][0][0][:check_b].cpu().numpy(), it[:check_b])
        out[name] = rows
    Hr = dec.H.copy()
    dec.close()

    def check():
        if not kept or args.no_cpu_baseline:
            return
        from oracle import oracle as orc
        threads, _ = cpu_share()
        llr = d_y[:check_b].cpu().numpy()
        for name, m in (("sum-product f64 (exact)", 1), ("min-sum f64", 0)):
            ref = orc.decode_batch(m, Hr, llr, args.iters, nthreads=threads, et_period=5)
            bad_pk = bad_it = 0
            for (mm, Bs), (pk, it) in kept.items():
                if mm == m:
                    bad_pk += int((ref["packed"] != pk).any(axis=1).sum())
                    bad_it += int((ref["iters"] != it).sum())
            out[name]["parity"] = {"frames": check_b, "launches_checked": 2,
                                   "packed_mismatch_frames": bad_pk,
                                   "iters_mismatch_frames": bad_it,
                                   "checker": "oracle decode_batch, et_period 5"}
    return out, check


def time_variant(timer, dec, torch, inputs, B, m, iters, et, p, steps, warmup, D, min_s=0.03,
                 streams=None):
    """A variant timed over max(steps, enough steps for min_s seconds): a few
    dozen short launches would time the clock ramp and the pipeline's fill and
    drain rather than the decoder, and the last variant's run is what the GPU
    was doing just before the headline's warmup (its clock has ramped).
    Returns (result, steps timed)."""
    r = timer(dec, torch, inputs, B, m, iters, et, p, steps, warmup, inflight=D, streams=streams)
    need = int(np.ceil(min_s / max(r["wall"] / steps, 1e-6)))
    if need > steps:
        steps = need
        r = timer(dec, torch, inputs, B, m, iters, et, p, steps, warmup, inflight=D,
                  streams=streams)
    return r, steps


def gpu_variants(L, torch, dec, args, dev, inputs, B, D, prec, dvb, world, rank):
    """Everything the line reports beside the headline that runs on the GPU:
    config 4, the block, one batch in flight, the other methods / precisions.
    Returns dict(variants, serial, outs, config4_check)."""
    res = dict(variants={}, serial=None, outs={}, config4_check=None, config5_check=None)
    if args.no_variants:
        return res
    var = res["variants"]
    if not dvb and not args.no_config4:
        var["config4"], res["config4_check"] = config4_variant(
            L, torch, dev, args, args.seed + 31,
            cpu_sample=0 if (args.no_cpu_baseline or rank != 0) else 1024)
    if not dvb and not args.no_config5:
        var["config5"], res["config5_check"] = config5_variant(L, torch, args, dev)
    if not dvb and not args.no_block and world == 1:
        from ldpc_ece535a import blocks
        with _quiet_stdout():
            var["block general_work (host buffers)"] = block_variant(L, torch, blocks, dev,
                                                                     args, inputs[0], B)
    if not dvb:
        for name, (m, p) in {"sum-product f32": (1, 1), "sum-product f64": (1, 0),
                             "sum-product f64fast (compact tanh/log, not exact)": (1, 3),
                             "min-sum f64": (0, 0), "min-sum f32": (0, 1)}.items():
            if (m, p) == (args.method, prec):
                continue
            r2, st = time_variant(time_ring, dec, torch, inputs, B, m, args.iters,
                                  args.et_period, p, max(5, args.steps // 2), 4, D)
            it2 = r2["iters"]
            var[name] = {"Mbit/s": round(B * dec.K * st / r2["wall"] / 1e6, 2),
                         "ms_per_batch": round(r2["wall"] / st * 1e3, 5),
                         "mean_iters": round(float(it2.mean()), 3)}
            res["outs"][name] = (m, r2["outs"][0][0].cpu().numpy(), it2)
    # last: one batch in flight of the headline's own method and precision,
    # so the GPU's clock and power state before the headline's warmup are
    # those of this workload (after a lighter kernel the first few ms of f64
    # sum-product run at a transiently lower clock: tools/short_runs.py,
    # profiles/round3/short_runs.txt)
    if D > 1:  # single batch in flight (latency per batch)
        if not dvb:
            dec.set_launch_mode(0)  # one launch at a time: the latency mode
        r1, st = time_variant(time_decoder, dec, torch, inputs[:1], B, args.method, args.iters,
                              args.et_period, prec, max(10, args.steps // 2), 5, 1)
        if not dvb:
            dec.set_launch_mode(1)
        res["serial"] = {"Mbit/s": round(B * dec.K * st / r1["wall"] / 1e6, 2),
                         "latency_ms_per_batch": round(r1["per_launch_ms"], 5)}
    return res


def relaunch_distributed(args):
    """`python bench.py --gpus N` (N > 1) outside torchrun: run torchrun as a
    child process (no exec; nothing has touched the GPU yet) and return its
    exit code.  The driver's own torchrun launch sets WORLD_SIZE and never
    gets here."""
    import random
    import subprocess
    port = str(29500 + random.randint(0, 2000))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", port, os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def sweeps(L, torch, dec, args, dev):
    modes = [(int(m.split(":")[0]), 0 if m.split(":")[1] == "f64" else 1)
             for m in args.sweep_modes.split(",")]
    if args.sweep_batch:
        for Bs in [int(x) for x in args.sweep_batch.split(",")]:
            d_y, _ = synth_device(L, torch, dec, Bs, args.ebn0, args.seed + 17, dev)
            for m, p in modes:
                r = time_decoder(dec, torch, [d_y], Bs, m, args.iters, args.et_period, p,
                                 args.steps, args.warmup)
                k0, it0 = r["per_launch_ms"], r["iters"]
                print("sweepB method=%d prec=%d B=%6d ebn0=%g mean_it=%6.2f max_it=%2d "
                      "kernel_ms=%8.4f Mbit/s=%9.2f" %
                      (m, p, Bs, args.ebn0, it0.mean(), it0.max(), k0,
                       Bs * dec.K / (k0 * 1e-3) / 1e6), file=sys.stderr, flush=True)
    if args.sweep_inflight:
        B = args.batch
        ins = [synth_device(L, torch, dec, B, args.ebn0, args.seed + 300 + j, dev)[0]
               for j in range(8)]
        for m, p in modes:
            for D in [int(x) for x in args.sweep_inflight.split(",")]:
                dec.set_launch_mode(1 if D > 1 else 0)
                r = time_decoder(dec, torch, ins, B, m, args.iters, args.et_period, p,
                                 args.steps, args.warmup, inflight=D)
                print("inflight method=%d prec=%d D=%d ms_per_batch=%8.4f Mbit/s=%9.2f" %
                      (m, p, D, r["wall"] / args.steps * 1e3,
                       B * dec.K * args.steps / r["wall"] / 1e6), file=sys.stderr, flush=True)
    if args.sweep_config5:
        # config 5: et_period 5, each frame at its own Eb/N0 drawn from {0,1,2,3,4} dB
        for Bs in [int(x) for x in args.sweep_config5.split(",")]:
            rng = np.random.Generator(np.random.PCG64(args.seed + 5))
            dbs = rng.integers(0, 5, size=Bs).astype(np.float64)
            d_y, _ = synth_device(L, torch, dec, Bs, dbs, args.seed + 100, dev)
            for m, p in ((1, 0), (1, 1), (0, 0)):
                r = time_decoder(dec, torch, [d_y], Bs, m, args.iters, 5, p, args.steps,
                                 args.warmup)
                k0, it0 = r["per_launch_ms"], r["iters"]
                print("config5 method=%d prec=%d B=%7d et=5 mean_it=%6.2f max_it=%2d "
                      "latency_ms=%8.4f Mbit/s=%9.2f" % (m, p, Bs, it0.mean(), it0.max(), k0,
                                                          Bs * dec.K / (k0 * 1e-3) / 1e6),
                      file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import ldpc_ece535a as L

    dist = None
    # LDPC_BENCH_SHARE_GPU=1: ranks share the visible GPUs (local % count) --
    # a rehearsal of the N-rank path on a one-GPU box, with
    # LDPC_BENCH_DIST_BACKEND=gloo (RCCL wants one GPU per rank).  The driver's
    # runs set neither: one rank per GPU over RCCL.
    if os.environ.get("LDPC_BENCH_SHARE_GPU") == "1":
        local = local % max(1, torch.cuda.device_count())
    backend = os.environ.get("LDPC_BENCH_DIST_BACKEND", "nccl")
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as tdist
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
        dist = tdist
    dev = torch.device("cuda", local)
    prec = {"f64": 0, "f32": 1, "f64libm": 2, "f64fast": 3}[args.precision]
    dvb = args.code == "dvbs2"
    if args.method is None:
        args.method = 0 if dvb else 1
    if args.batch is None:
        args.batch = 1024 if dvb else 4096
    D = max(1, args.inflight)

    csr = None
    if dvb:
        from ldpc_ece535a import codes
        csr = codes.dvbs2_like(0)
        dec = L.Decoder(csr=csr, device=local)
        Hr = None
    else:
        dec = L.Decoder(device=local)  # default H, reorderHMatrix applied
        dec.set_schedule(args.schedule)
        Hr = dec.H
    offset, B = plan_batch(args.batch, world, rank, args.strong)
    # D distinct batches per rank, made on the GPU, resident in HBM before timing
    inputs = [synth_device(L, torch, dec, B, args.ebn0, args.seed + 7919 * rank + 104729 * j,
                           dev)[0] for j in range(D)]
    torch.cuda.synchronize(dev)
    sweeps(L, torch, dec, args, dev)

    # several batches in flight: the throughput launch mode (4 waves per CU per
    # launch, four-waves-per-SIMD build, no issue-priority management;
    # include/ldpc_hip.h ldpc_set_launch_mode)
    if not dvb:
        dec.set_launch_mode(1 if D > 1 else 0)
        if args.waves_per_cu:
            dec.set_waves_per_cu(args.waves_per_cu)
    # The variants (other methods / precisions, latency, the block, config 4)
    # are measured first, on every rank, so the headline's K steps run on a
    # GPU that has been busy for a while (its clock ramps from ~2.0 to
    # ~2.33 GHz over the first ~20 ms of work, profiles/round1/
    # warmup_clock.txt) and every rank arrives in the same state.  Their CPU
    # checks run after the headline.
    pre = gpu_variants(L, torch, dec, args, dev, inputs, B, D, prec, dvb, world, rank)
    # small codes: the frame ring (one launch per timed region, frames of all
    # batches from one queue); large codes (config 4's pipeline): a launch per
    # batch
    timer = time_decoder if dvb else time_ring
    r = timer(dec, torch, inputs, B, args.method, args.iters, args.et_period, prec,
              args.steps, args.warmup, dist, inflight=D)
    wall = r["wall"]
    iters_b = [o[1].cpu().numpy() for o in r["outs"]]
    synd_b = [o[2].cpu().numpy() for o in r["outs"]]
    # per step: batch k % D; counters over the K timed steps
    steps_of = [len(range(j, args.steps, D)) for j in range(D)]
    counters = [sum(steps_of[j] * B for j in range(D)),
                sum(steps_of[j] * B * dec.K for j in range(D)),
                sum(steps_of[j] * int(iters_b[j].sum()) for j in range(D)),
                sum(steps_of[j] * int((synd_b[j] > 0).sum()) for j in range(D))]
    red_dev = dev if backend == "nccl" else torch.device("cpu")
    full, totals, wall_max = reduce_results(
        dist, r["outs"][0][0].to(red_dev), counters, wall, red_dev)

    if rank != 0:
        dist.destroy_process_group()
        return

    frames_all, info_bits = totals[0], totals[1]
    value = info_bits / wall_max / 1e6
    per_launch_ms = wall_max / args.steps * 1e3
    mean_it = totals[2] / max(1.0, frames_all)
    E, N = dec.E, dec.N
    alg_bytes = float(B * (4 * N + dec.KB + 8) + mean_it * B * bytes_per_iter(E, N, prec))
    workload_key = "%s%d_%s_b%d_i%d_db%g" % ("dvb" if dvb else "sp", args.method, args.precision,
                                            args.batch, args.iters, args.ebn0)
    entry = load_pmc(args.pmc_json, workload_key) or {}
    if dvb and entry.get("pipeline") != dec.pipeline():
        entry = {}  # taken at another pipeline configuration: not this run's traffic
    pmc = entry.get("pmc")
    traffic = entry.get("hbm_bytes_per_launch")

    mname = {0: "min-sum", 1: "sum-product", 2: "bit-flip", 3: "hard"}[args.method]
    if dvb:
        workload = ("config4: DVB-S2-like N=64800 K=32400 E=226799 code (synthetic rate-1/2 "
                    "address table), large-code path (messages in HBM), B=%d frames/GPU, "
                    "method %d (%s), %d-iteration cap with per-frame early exit, Eb/N0 %g dB"
                    % (B, args.method, mname, args.iters, args.ebn0))
    else:
        workload = ("config2: reference default 32x64 H (reordered), B=%d frames%s, method %d "
                    "(%s), %d-iteration cap with per-frame early exit, Eb/N0 %g dB"
                    % (args.batch, " split over the ranks" if args.strong and world > 1
                       else "/GPU", args.method, mname, args.iters, args.ebn0))
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mbit/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(per_launch_ms, 4),
        "higher_is_better": True,
        "scaling": "strong" if args.strong and world > 1 else "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.precision == "f32" else "f64",
        "data": "synthetic, made on the GPU: Philox bits, GF(2) systematic encode "
                "(ldpc_encode_device), BPSK, AWGN sigma=sqrt(10^(-EbN0/10))",
        "config": {
            "workload": workload,
            "global_batch": args.batch * (1 if args.strong else world),
            "frames_per_gpu": B,
            "distinct_input_batches": D,
            "decoder": ("one launch per batch" if dvb else
                        "frame ring (ldpc_ring_*): one persistent launch per timed region, "
                        "frames of all posted batches from one queue"),
            "parallelism": "dp%d (independent frames)" % world,
            "mean_iters": round(mean_it, 3),
            "syndrome_fail_frac": round(totals[3] / max(1.0, frames_all), 4),
            "et_period": args.et_period,
        },
    }
    hbm_model = {
        "achieved_equiv_GB/s": round(alg_bytes / (per_launch_ms * 1e-3) / 1e9, 1),
        "model_bytes_per_launch": int(alg_bytes),
        "model": "SURVEY 8(d) algorithmic bytes: sum_b [4N + KB + 8 + iters_b (32E + 10N)] "
                 "(f64; 16E + 6N f32)",
        "traffic": traffic,
    }
    if dvb:
        model_gbs = alg_bytes / (per_launch_ms * 1e-3) / 1e9
        if traffic:
            # the compressed-message pipeline moves ~half the edge-message
            # model's bytes (so the model's rate exceeds the peak): the
            # roofline is the measured memory traffic (PMC, per decode) over
            # the live decode time; the model's rate is reported beside it
            achieved = traffic / (per_launch_ms * 1e-3) / 1e9
            line["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                                "achieved_basis": "measured bytes (traffic) / live decode time",
                                "model_equiv_GB/s": round(model_gbs, 1),
                                "traffic_vs_model": round(traffic / alg_bytes, 3),
                                "model": hbm_model["model"], "traffic_source": entry.get("source")}
        else:
            line["roofline"] = {"bound": "hbm", "achieved": round(model_gbs, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": round(model_gbs / HBM_PEAK_GBS, 4), "traffic": None,
                                "achieved_basis": "edge-message byte model (no PMC entry)",
                                "model": hbm_model["model"]}
    elif pmc and "SQ_INSTS_VALU" in pmc:
        # per batch: the PMC entry's counts per batch over the device span per
        # batch (the ring launch's own time / K)
        line["roofline"] = valu_roofline(pmc, r["per_launch_ms"] or per_launch_ms,
                                         (entry.get("isa_hot") or {}).get("other_weight"))
        line["roofline"]["traffic"] = traffic
        line["roofline"]["pmc_source"] = entry.get("source")
        hbm_model["label"] = ("equivalent streaming bandwidth of a decoder that streams its edge "
                              "messages through HBM; this kernel keeps them on chip (traffic = "
                              "measured HBM bytes per launch), so no HBM fraction applies")
        line["hbm_byte_model"] = hbm_model
    else:
        line["roofline"] = {"bound": "valu", "achieved": None, "peak": SIMDS * CLOCK_HZ / 1e9,
                            "unit": "G SIMD-cycles/s of VALU issue (f64-weighted)", "frac": None,
                            "traffic": traffic,
                            "note": "no PMC instruction counts for %s in %s" % (workload_key,
                                                                              args.pmc_json)}
        line["hbm_byte_model"] = hbm_model
    line["timing"] = {"device_span_ms_per_launch": round(r["per_launch_ms"], 5),
                      "wall_ms_per_step": round(per_launch_ms, 5),
                      "note": ("span = HIP events on the ring session's stream: one before "
                               "the timed session's launch (which waits on it), one after the "
                               "session's end (which waits on the launch), / K batches; the "
                               "roofline's per-batch time" if not dvb else
                               "span = HIP events around the K launches, / K"),
                      "frame_ring": r.get("ring"),
                      "order": "measured after the GPU variants below (same process), so the "
                               "K steps see the GPU's steady clock; --no-variants times a "
                               "cold GPU"}

    if pre["serial"]:
        line["serial_1_batch_in_flight"] = pre["serial"]
    if pre["variants"]:
        line["variants_1gpu"] = pre["variants"]
    variant_outs = pre["outs"]

    # ---- CPU baseline + parity (the oracle as checker) ----------------------
    if not args.no_cpu_baseline:
        sys.path.insert(0, REPO)
        from oracle import oracle as orc
        threads, visible = cpu_share()
        threads = args.cpu_threads or threads
        llr = inputs[0].cpu().numpy()
        packed = r["outs"][0][0].cpu().numpy()
        if dvb:  # the sparse restatement on every frame of rank 0's batch (~2 s)
            nb = B
            t0 = time.perf_counter()
            ref = orc.decode_batch_sparse(args.method, csr[2], csr[3], csr[0], csr[1], llr[:nb],
                                          args.iters, nthreads=threads, want_bits=False)
            cpu_s = time.perf_counter() - t0
            line["cpu_baseline"] = {
                "value": round(nb * dec.K / cpu_s / 1e6, 5), "unit": "Mbit/s", "cores": threads,
                "kind": "port",
                "sample": "%d of rank 0's %d frames, sparse oracle, %d threads on %s"
                          % (nb, B, threads, cpu_model())}
            line["parity"] = {"frames": nb,
                              "packed_mismatch_frames": int((ref["packed"] != packed[:nb]).any(axis=1).sum()),
                              "iters_mismatch_frames": int((ref["iters"] != iters_b[0][:nb]).sum()),
                              "checker": "oracle sparse restatement (orc_decode_batch_sparse)"}
        else:
            t0 = time.perf_counter()
            ref = orc.decode_batch(args.method, Hr, llr, args.iters, nthreads=threads,
                                   et_period=args.et_period)
            cpu_s = time.perf_counter() - t0
            nsample = min(B, 256)
            t1 = time.perf_counter()
            orc.decode_batch(args.method, Hr, llr[:nsample], args.iters, nthreads=1,
                             et_period=args.et_period)
            cpu1 = nsample * dec.K / (time.perf_counter() - t1) / 1e6
            phys = physical_cores(sorted(os.sched_getaffinity(0))) if hasattr(
                os, "sched_getaffinity") else None
            # the same frames on every logical CPU the process may run on (the
            # box's CPU quota, not this count, then sets the rate)
            t2 = time.perf_counter()
            orc.decode_batch(args.method, Hr, llr, args.iters, nthreads=min(visible, 256),
                             et_period=args.et_period)
            cpu_all = B * dec.K / (time.perf_counter() - t2) / 1e6
            line["cpu_baseline"] = {
                "value": round(B * dec.K / cpu_s / 1e6, 5),
                "unit": "Mbit/s",
                "cores": threads,
                "kind": "port",
                "sample": "the same %d frames (rank 0's first batch), %d threads (the GPU box's "
                          "CPU share per GPU) on %s; 1 core: %.5f Mbit/s on the first %d frames; "
                          "host: %d logical CPUs visible, %s physical cores" % (
                              B, threads, cpu_model(), cpu1, nsample, visible, phys),
                "one_core_Mbit/s": round(cpu1, 5),
                "all_visible_cpus": {"threads": min(visible, 256), "Mbit/s": round(cpu_all, 5)},
                "all_physical_cores_Mbit/s_linear_extrapolation":
                    round(cpu1 * phys, 4) if phys else None,
            }
            line["parity"] = {"frames": B,
                              "packed_mismatch_frames": int((ref["packed"] != packed).any(axis=1).sum()),
                              "iters_mismatch_frames": int((ref["iters"] != iters_b[0]).sum()),
                              "synd_mismatch_frames": int((ref["synd"] != synd_b[0]).sum()),
                              "checker": "oracle/ (C restatement of the reference decoder)"}
            refs = {args.method: ref}
            for name, (m, pk, it2) in variant_outs.items():
                if m not in refs:
                    refs[m] = orc.decode_batch(m, Hr, llr, args.iters, nthreads=threads,
                                               et_period=args.et_period)
                line["variants_1gpu"][name]["packed_mismatch_frames"] = int(
                    (refs[m]["packed"] != pk).any(axis=1).sum())
        if world > 1:
            line["parity_all_ranks"] = gathered_parity(L, torch, orc, dec, args, dev, full, world,
                                                       Hr, csr, threads)
    for chk in ("config4_check", "config5_check"):
        if pre[chk] is not None:
            pre[chk]()
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
