#!/usr/bin/env python3
"""Benchmark of the decode hot path (BASELINE.json configs[1] / [2]).

One "step" = one pass of the decoder over one batch of synthetic frames
already resident in HBM: B = 4096 frames of the reference's default 32x64 H
(reordered as the block does), sum-product (method 1), 50-iteration cap with
the reference's per-frame early exit, Eb/N0 = 2 dB with the reference noise
convention (sigma = sqrt(10^(-EbN0/10)), apps/ldpc_lapack.cpp:635-642).

  python bench.py [--gpus N --steps K --warmup W]

N > 1 runs under torch.distributed.run, one rank per GPU: each rank decodes
its own batch (weak scaling, independent frames, no collective in the data
path); after the timed loop RCCL all-gathers the packed outputs and
all-reduces the counters (the "final throughput gather").  Rank 0 prints ONE
JSON line.  `value` = info bits of all frames all ranks decoded / the max
over ranks of the timed wall time.

roofline.achieved uses SURVEY.md 8(d)'s algorithmic byte model per launch:
  sum_b [4N (fp32 Re in) + KB + 8 (packed, iters, syndrome out)
         + iters_b * (32E + 10N)]  (f64 parity mode; 16E + 6N for f32)
divided by the kernel's mean duration: one HIP event pair on the launch
stream around the K timed launches, divided by K.  roofline.traffic is the rocprofv3 PMC measurement
(profiles/) per launch, when a matching entry exists.  roofline_valu: the
bound that actually applies to the small-code kernel (messages never leave
LDS/VGPRs): PMC VALU wave-instructions per launch / kernel time against the
1024-SIMD issue peak.
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

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    # the first ~100-200 launches of a fresh process run ~7 % slower (clock settling,
    # profiles/round1/warmup_dependence.txt); the default warmup covers them
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--code", choices=["default", "dvbs2"], default="default",
                    help="default: the reference's 32x64 H (config 2); dvbs2: the DVB-S2-size "
                         "code of config 4 (synthetic rate-1/2 address table)")
    ap.add_argument("--batch", type=int, default=None, help="default 4096 (1024 for dvbs2)")
    ap.add_argument("--method", type=int, default=None, help="default 1 (0 for dvbs2)")
    ap.add_argument("--no-config4", action="store_true", help="skip the config-4 variant")
    ap.add_argument("--precision", choices=["f64", "f32"], default="f64")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--et-period", type=int, default=1)
    ap.add_argument("--ebn0", type=float, default=2.0)
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--waves-per-cu", type=int, default=0)
    ap.add_argument("--sweep-wpc", default="", help="comma list; prints a table to stderr")
    ap.add_argument("--sweep-batch", default="",
                    help="comma list of B: latency/throughput sweep (config 5) to stderr")
    ap.add_argument("--schedule", type=int, default=0, help="0 auto, 1 wave/frame, 2 workgroup/frame")
    ap.add_argument("--sweep-schedules", default="0", help="comma list for --sweep-batch")
    ap.add_argument("--sweep-modes", default="1:f64,1:f32,0:f64",
                    help="method:precision list for the sweeps")
    ap.add_argument("--sweep-config5", default="",
                    help="comma list of B: config 5 (syndrome check every 5 iterations, mixed "
                         "Eb/N0 0..4 dB per frame) latency/throughput table to stderr")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def synth_csr(csr, B, ebn0, seed):
    """Config 4: PCG64 info bits, IRA encode (ldpc_ece535a.codes), BPSK, AWGN."""
    from ldpc_ece535a import codes
    M, N = csr[0], csr[1]
    rng = np.random.Generator(np.random.PCG64(seed))
    data = rng.integers(0, 2, size=(B, N - M), dtype=np.uint8)
    cw = codes.ira_encode(csr, data)
    sigma = np.sqrt(10.0 ** (-ebn0 / 10.0))
    y = (2.0 * cw.astype(np.float64) - 1.0 + sigma * rng.standard_normal((B, N)))
    return y.astype(np.float32), data


def config4_variant(L, torch, dev, args, seed, steps=5, warmup=1, cpu_sample=0):
    """DVB-S2-like N=64800 code, min-sum f64, 1024 frames (config 4) on the
    large-code path; optional parity of the first frames vs the sparse oracle."""
    from ldpc_ece535a import codes
    csr = codes.dvbs2_like(0)
    dec = L.Decoder(csr=csr, device=dev.index or 0)
    B = 1024
    y, data = synth_csr(csr, B, args.ebn0, seed)
    d_y = torch.from_numpy(y).to(dev)
    out = {}
    for name, p in (("f64", 0), ("f32", 1)):
        w, k, it, o = time_decoder(dec, torch, d_y, B, 0, args.iters, 1, p, steps, warmup)
        alg = float(B * (4 * dec.N + dec.KB + 8) + it.sum() * bytes_per_iter(dec.E, dec.N, p))
        pk = o[0].cpu().numpy()
        out["min-sum " + name] = {
            "Mbit/s": round(B * dec.K * steps / w / 1e6, 2), "ms_per_decode": round(k, 4),
            "mean_iters": round(float(it.mean()), 3), "max_iters": int(it.max()),
            "alg_GB/s": round(alg / (k * 1e-3) / 1e9, 1),
            "frames_decoded_to_sent_data": int((pk == np.packbits(data, axis=1)).all(axis=1).sum())}
        if p == 0 and cpu_sample:
            from oracle import oracle as orc
            t0 = time.perf_counter()
            ref = orc.decode_batch_sparse(0, csr[2], csr[3], csr[0], csr[1], y[:cpu_sample],
                                          args.iters, nthreads=16, want_bits=False)
            cpu_s = time.perf_counter() - t0
            out["min-sum f64"]["parity_sample"] = {
                "frames": cpu_sample,
                "packed_mismatch_frames": int((ref["packed"] != pk[:cpu_sample]).any(axis=1).sum()),
                "iters_mismatch_frames": int((ref["iters"] != it[:cpu_sample]).sum()),
                "checker": "oracle sparse restatement (orc_decode_batch_sparse)",
                "cpu_Mbit/s_16_threads": round(cpu_sample * dec.K / cpu_s / 1e6, 4)}
    out["code"] = ("DVB-S2-like N=64800 K=32400 E=226799 (synthetic rate-1/2 address table, "
                   "ldpc_ece535a.codes.dvbs2_like(0)), B=1024, %d-iteration cap" % args.iters)
    dec.close()
    return out


def synth(Hr, B, ebn0, seed):
    """Seeded frames: data ~ Bernoulli(1/2) (PCG64), GF(2) encode through the
    product's ldpc_encode, BPSK 1->+1, AWGN with the reference sigma."""
    import ldpc_ece535a as L
    M, N = Hr.shape
    rng = np.random.Generator(np.random.PCG64(seed))
    data = rng.integers(0, 2, size=(B, N - M), dtype=np.uint8)
    cw = L.encode(Hr, data)
    sigma = np.sqrt(10.0 ** (-ebn0 / 10.0))
    y = (2.0 * cw.astype(np.float64) - 1.0 + sigma * rng.standard_normal((B, N)))
    return y.astype(np.float32), data


def bytes_per_iter(E, N, prec):
    return 32 * E + 10 * N if prec == 0 else 16 * E + 6 * N


def time_decoder(dec, torch, d_in, B, method, iters, et, prec, steps, warmup, dist=None):
    """Returns (wall_s, mean_kernel_ms, per-frame iters, outputs).

    One HIP event pair on the launch stream brackets the K timed launches;
    mean_kernel_ms = that span / K (it includes the short gaps between
    back-to-back launches, so it is slightly conservative).  Per-launch event
    records are avoided: they perturb the launches they bracket (measured:
    +5 % per step)."""
    dev = d_in.device
    d_packed = torch.empty((B, dec.KB), dtype=torch.uint8, device=dev)
    d_iters = torch.empty(B, dtype=torch.int32, device=dev)
    d_synd = torch.empty(B, dtype=torch.int32, device=dev)
    # a dedicated (non-null) stream: the kernel and the timing events share it
    stream = torch.cuda.Stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)

    def step():
        dec.decode_device(d_in.data_ptr(), B, d_packed.data_ptr(), method=method, max_iters=iters,
                          et_period=et, precision=prec, d_iters=d_iters.data_ptr(),
                          d_synd=d_synd.data_ptr(), stream=sp)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    kern_ms = e0.elapsed_time(e1) / max(1, steps)
    return wall, kern_ms, d_iters.cpu().numpy(), (d_packed, d_iters, d_synd)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown CPU"


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
    if world > 1:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = tdist
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    prec = 0 if args.precision == "f64" else 1
    dvb = args.code == "dvbs2"
    if args.method is None:
        args.method = 0 if dvb else 1
    if args.batch is None:
        args.batch = 1024 if dvb else 4096

    csr = None
    if dvb:
        from ldpc_ece535a import codes
        csr = codes.dvbs2_like(0)
        dec = L.Decoder(csr=csr, device=local)
        Hr = None
    else:
        dec = L.Decoder(device=local)  # default H, reorderHMatrix applied
        dec.set_waves_per_cu(args.waves_per_cu)
        dec.set_schedule(args.schedule)
        Hr = dec.H
    B = args.batch
    if dvb:
        llr, data = synth_csr(csr, B, args.ebn0, args.seed + 7919 * rank)
    else:
        llr, data = synth(Hr, B, args.ebn0, args.seed + 7919 * rank)
    d_in = torch.from_numpy(llr).to(dev)  # resident in HBM before timing

    if args.sweep_batch:
        modes = [(int(m.split(":")[0]), 0 if m.split(":")[1] == "f64" else 1)
                 for m in args.sweep_modes.split(",")]
        for Bs in [int(x) for x in args.sweep_batch.split(",")]:
            y, _ = synth(Hr, Bs, args.ebn0, args.seed + 17)
            d_y = torch.from_numpy(y).to(dev)
            for sched in [int(x) for x in args.sweep_schedules.split(",")]:
                dec.set_schedule(sched)
                for m, p in modes:
                    w0, k0, it0, _ = time_decoder(dec, torch, d_y, Bs, m, args.iters,
                                                  args.et_period, p, args.steps, args.warmup)
                    print("sweepB sched=%d method=%d prec=%d B=%6d ebn0=%g mean_it=%6.2f "
                          "max_it=%2d kernel_ms=%8.4f Mbit/s=%9.2f us/iter(max-frame)=%7.3f" %
                          (sched, m, p, Bs, args.ebn0, it0.mean(), it0.max(), k0,
                           Bs * dec.K / (k0 * 1e-3) / 1e6, k0 * 1e3 / max(1, it0.max())),
                          file=sys.stderr, flush=True)
            dec.set_schedule(args.schedule)

    if args.sweep_config5:
        # config 5: et_period 5, each frame at its own Eb/N0 drawn from {0,1,2,3,4} dB
        for Bs in [int(x) for x in args.sweep_config5.split(",")]:
            rng = np.random.Generator(np.random.PCG64(args.seed + 5))
            dbs = rng.integers(0, 5, size=Bs)
            parts = []
            for db in range(5):
                n = int((dbs == db).sum())
                parts.append(synth(Hr, n, float(db), args.seed + 100 + db)[0] if n else
                             np.zeros((0, Hr.shape[1]), np.float32))
            y = np.zeros((Bs, Hr.shape[1]), np.float32)
            for db in range(5):
                y[dbs == db] = parts[db]
            d_y = torch.from_numpy(y).to(dev)
            for m, p in ((1, 0), (1, 1), (0, 0)):
                w0, k0, it0, _ = time_decoder(dec, torch, d_y, Bs, m, args.iters, 5, p,
                                              args.steps, args.warmup)
                print("config5 method=%d prec=%d B=%7d et=5 mean_it=%6.2f max_it=%2d "
                      "latency_ms=%8.4f Mbit/s=%9.2f" % (m, p, Bs, it0.mean(), it0.max(), k0,
                                                          Bs * dec.K / (k0 * 1e-3) / 1e6),
                      file=sys.stderr, flush=True)

    if args.sweep_wpc:
        for m, p in ((args.method, prec), (1, 1), (0, 0)):
            for wpc in [int(x) for x in args.sweep_wpc.split(",")]:
                dec.set_waves_per_cu(wpc)
                w0, k0, it0, _ = time_decoder(dec, torch, d_in, B, m, args.iters,
                                              args.et_period, p, args.steps, args.warmup)
                print("sweep method=%d prec=%d wpc=%2d kernel_ms=%.4f wall_ms/step=%.4f" %
                      (m, p, wpc, k0, w0 / args.steps * 1e3), file=sys.stderr, flush=True)
        dec.set_waves_per_cu(args.waves_per_cu)

    wall, kern_ms, iters_b, outs = time_decoder(dec, torch, d_in, B, args.method, args.iters,
                                                args.et_period, prec, args.steps, args.warmup,
                                                dist)
    packed = outs[0].cpu().numpy()
    synd = outs[2].cpu().numpy()

    # ---- final gather (RCCL): outputs to every rank + counters ------------
    totals = np.array([B, B * dec.K, int(iters_b.sum()), int((synd > 0).sum())], np.float64)
    wall_max = wall
    if dist is not None:
        g = [torch.empty_like(outs[0]) for _ in range(world)]
        dist.all_gather(g, outs[0])
        t = torch.tensor(totals, device=dev)
        dist.all_reduce(t)
        totals = t.cpu().numpy()
        w = torch.tensor([wall], device=dev, dtype=torch.float64)
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall_max = float(w.item())

    if rank != 0:
        dist.destroy_process_group()
        return

    frames_all = totals[0] * args.steps
    info_bits = totals[1] * args.steps
    value = info_bits / wall_max / 1e6
    E, N = dec.E, dec.N
    alg_bytes = float(B * (4 * N + dec.KB + 8) + iters_b.sum() * bytes_per_iter(E, N, prec))
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    pmc = None
    workload_key = "%s%d_%s_b%d_i%d_db%g" % ("dvb" if dvb else "sp", args.method, args.precision, B,
                                            args.iters, args.ebn0)
    try:
        tj = json.load(open(args.traffic_json))
        if workload_key in tj:
            traffic = tj[workload_key]["hbm_bytes_per_launch"]
            pmc = tj[workload_key].get("pmc")
    except (OSError, ValueError, KeyError):
        pass

    mname = {0: "min-sum", 1: "sum-product", 2: "bit-flip", 3: "hard"}[args.method]
    if dvb:
        workload = ("config4: DVB-S2-like N=64800 K=32400 E=226799 code (synthetic rate-1/2 "
                    "address table), large-code path (messages in HBM), B=%d frames/GPU, "
                    "method %d (%s), %d-iteration cap with per-frame early exit, Eb/N0 %g dB"
                    % (B, args.method, mname, args.iters, args.ebn0))
    else:
        workload = ("config2: reference default 32x64 H (reordered), B=%d frames/GPU, "
                    "method %d (%s), %d-iteration cap with per-frame early exit, "
                    "Eb/N0 %g dB" % (B, args.method, mname, args.iters, args.ebn0))
    line = {
        "metric": "decoded info Mbit/s @ 50 BP iters, batch=4096; achieved HBM GB/s vs peak",
        "value": round(value, 3),
        "unit": "Mbit/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (PCG64 bits, GF(2) encode, BPSK, AWGN sigma=sqrt(10^(-EbN0/10)))",
        "config": {
            "workload": workload,
            "global_batch": int(totals[0]),
            "frames_per_gpu": B,
            "parallelism": "dp%d (independent frames)" % world,
            "mean_iters": round(float(iters_b.mean()), 3),
            "syndrome_fail_frac": round(float((synd > 0).mean()), 4),
            "et_period": args.et_period,
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel_ms": round(kern_ms, 5),
            "model": "SURVEY 8(d) algorithmic bytes per launch = %d" % int(alg_bytes),
            "label": ("equivalent streaming bandwidth: the small-code kernel keeps every message "
                      "in LDS/VGPRs (traffic = measured HBM bytes per launch); roofline_valu is "
                      "the bound that applies") if not dvb else "HBM-resident messages",
        },
    }
    if pmc and "SQ_INSTS_VALU" in pmc and not dvb:
        # The small-code kernel keeps every message in LDS / VGPRs (traffic is
        # ~0.2 % of the byte model), so HBM does not bound it: VALU issue does.
        # achieved = PMC VALU wave-instructions per launch (profiles/) / the
        # live kernel time; peak = 1024 SIMDs x 2.4 GHz / 4 cycles per wave64
        # VALU instruction (f64 FMA is full rate on gfx950).
        valu_peak = 256 * 4 * 2.4e9 / 4 / 1e9
        valu_ach = pmc["SQ_INSTS_VALU"] / (kern_ms * 1e-3) / 1e9
        line["roofline_valu"] = {
            "bound": "valu", "achieved": round(valu_ach, 1), "peak": valu_peak,
            "unit": "G wave-instr/s", "frac": round(valu_ach / valu_peak, 4),
            "f64_fma_per_launch": pmc.get("SQ_INSTS_VALU_FMA_F64"),
            "source": "SQ_INSTS_VALU per launch from the rocprofv3 PMC pass (profiles/pmc_traffic.json)"}

    # ---- variants measured in the same process (not the headline) ----------
    variant_outs = {}
    if not args.no_variants and not dvb:
        var = {}
        for name, (m, p) in {"sum-product f32": (1, 1), "sum-product f64": (1, 0),
                             "min-sum f64": (0, 0), "min-sum f32": (0, 1)}.items():
            if (m, p) == (args.method, prec):
                continue
            st = max(5, args.steps // 2)
            w2, k2, it2, o2 = time_decoder(dec, torch, d_in, B, m, args.iters, args.et_period, p,
                                           st, 2)
            alg2 = float(B * (4 * dec.N + dec.KB + 8) + it2.sum() * bytes_per_iter(dec.E, dec.N, p))
            var[name] = {"Mbit/s": round(B * dec.K * st / w2 / 1e6, 2),
                         "kernel_ms": round(k2, 5), "mean_iters": round(float(it2.mean()), 3),
                         "alg_GB/s": round(alg2 / (k2 * 1e-3) / 1e9, 1)}
            variant_outs[name] = (m, o2[0].cpu().numpy(), it2)
        line["variants_1gpu"] = var

    # ---- CPU baseline + parity (the oracle as checker) ----------------------
    if not args.no_cpu_baseline:
        sys.path.insert(0, REPO)
        from oracle import oracle as orc
        try:
            ncpu = len(os.sched_getaffinity(0))
        except AttributeError:
            ncpu = os.cpu_count() or 1
        threads = args.cpu_threads or max(1, min(16, ncpu))
        if dvb:  # bounded sample: the sparse restatement on the first 128 frames
            nb = min(B, 128)
            t0 = time.perf_counter()
            ref = orc.decode_batch_sparse(args.method, csr[2], csr[3], csr[0], csr[1], llr[:nb],
                                          args.iters, nthreads=threads, want_bits=False)
            cpu_s = time.perf_counter() - t0
            line["cpu_baseline"] = {
                "value": round(nb * dec.K / cpu_s / 1e6, 5), "unit": "Mbit/s", "cores": threads,
                "kind": "port",
                "sample": "first %d of rank 0's %d frames, sparse oracle, %d threads on %s"
                          % (nb, B, threads, cpu_model())}
            line["parity"] = {"frames": nb,
                              "packed_mismatch_frames": int((ref["packed"] != packed[:nb]).any(axis=1).sum()),
                              "iters_mismatch_frames": int((ref["iters"] != iters_b[:nb]).sum()),
                              "checker": "oracle sparse restatement (orc_decode_batch_sparse)"}
            print(json.dumps(line), flush=True)
            if dist is not None:
                dist.destroy_process_group()
            return
        t0 = time.perf_counter()
        ref = orc.decode_batch(args.method, Hr, llr, args.iters, nthreads=threads)
        cpu_s = time.perf_counter() - t0
        nsample = min(B, 128)
        t1 = time.perf_counter()
        orc.decode_batch(args.method, Hr, llr[:nsample], args.iters, nthreads=1)
        cpu1_s = time.perf_counter() - t1
        mism = int((ref["packed"] != packed).any(axis=1).sum()) if rank == 0 else None
        line["cpu_baseline"] = {
            "value": round(B * dec.K / cpu_s / 1e6, 5),
            "unit": "Mbit/s",
            "cores": threads,
            "kind": "port",
            "sample": "the same %d frames (rank 0's batch), %d threads on %s; 1-core: %.5f "
                      "Mbit/s on the first %d frames" % (B, threads, cpu_model(),
                                                          nsample * dec.K / cpu1_s / 1e6, nsample),
        }
        line["parity"] = {"frames": B, "packed_mismatch_frames": mism,
                          "iters_mismatch_frames": int((ref["iters"] != iters_b).sum()),
                          "checker": "oracle/ (C restatement of the reference decoder)"}
        refs = {args.method: ref}
        for name, (m, pk, it2) in variant_outs.items():
            if m not in refs:
                refs[m] = orc.decode_batch(m, Hr, llr, args.iters, nthreads=threads)
            line["variants_1gpu"][name]["packed_mismatch_frames"] = int(
                (refs[m]["packed"] != pk).any(axis=1).sum())
    if not args.no_variants and not dvb and not args.no_config4:
        line.setdefault("variants_1gpu", {})["config4"] = config4_variant(
            L, torch, dev, args, args.seed + 31, cpu_sample=0 if args.no_cpu_baseline else 64)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
