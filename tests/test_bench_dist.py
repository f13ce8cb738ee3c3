"""bench.py's multi-GPU path, rehearsed on the CPU with gloo at world size 2.

The GPU decode is replaced by the oracle (a stub decoder: the data path under
test here is bench.py's own -- plan_batch's weak / strong shards,
timed_steps' barrier-bracketed loop, reduce_results' gather through
ldpc_ece535a.dist.gather_outputs and the max-over-ranks wall time -- and the
headline formula value = all ranks' info bits / max wall)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, strong, B, steps, out_path):
    import sys
    import time
    sys.path[:0] = [REPO, os.path.join(REPO, "gr-ldpc_ece535a_amd")]
    import torch
    import bench
    from oracle import oracle as orc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fd = np.load(os.path.join(REPO, "tests", "golden", "frames_default.npz"))
    Hr = fd["H_reordered"]
    allframes = np.concatenate([fd["db2_llr"], fd["db0_llr"], fd["db4_llr"]])
    off, n = bench.plan_batch(B, world, rank, strong)
    y = allframes[off:off + n]
    res = {}

    def step(k):
        res["out"] = orc.decode_batch(1, Hr, y, 50)
        if rank == 1:
            time.sleep(0.05)  # the slower rank sets the wall time

    wall = bench.timed_steps(step, steps, 1, lambda: None, dist)
    o = res["out"]
    counters = [steps * n, steps * n * 32, steps * int(o["iters"].sum()),
                steps * int((o["synd"] > 0).sum())]
    full, totals, wall_max = bench.reduce_results(dist, torch.from_numpy(o["packed"]), counters,
                                                  wall)
    if rank == 0:
        np.savez(out_path, packed=full.numpy(), totals=np.array(totals), wall=wall,
                 wall_max=wall_max, value=totals[1] / wall_max / 1e6)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("strong", [False, True])
def test_bench_distributed_path_gloo(tmp_path, strong):
    world, B, steps = 2, 48, 3
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(world, port, strong, B, steps, out), nprocs=world, join=True)
    from oracle import oracle as orc
    fd = np.load(os.path.join(REPO, "tests", "golden", "frames_default.npz"))
    allframes = np.concatenate([fd["db2_llr"], fd["db0_llr"], fd["db4_llr"]])
    total = B if strong else world * B  # frames per step, all ranks
    ref = orc.decode_batch(1, fd["H_reordered"], allframes[:total], 50)
    got = np.load(out)
    assert (got["packed"] == ref["packed"]).all()
    t = got["totals"]
    assert t[0] == steps * total and t[1] == steps * total * 32
    assert t[2] == steps * ref["iters"].sum() and t[3] == steps * (ref["synd"] > 0).sum()
    # the max over ranks: rank 1 sleeps 50 ms per step
    assert got["wall_max"] >= got["wall"] and got["wall_max"] >= steps * 0.05
    assert np.isclose(got["value"], t[1] / got["wall_max"] / 1e6)


def test_plan_batch():
    import sys
    sys.path[:0] = [REPO]
    import bench
    assert bench.plan_batch(4096, 1, 0, True) == (0, 4096)
    assert bench.plan_batch(4096, 8, 3, False) == (3 * 4096, 4096)
    parts = [bench.plan_batch(4097, 8, r, True) for r in range(8)]
    assert sum(n for _, n in parts) == 4097 and parts[0][0] == 0
    assert all(parts[i][0] + parts[i][1] == parts[i + 1][0] for i in range(7))


@pytest.mark.parametrize("strong", [False, True])
def test_gathered_parity(monkeypatch, strong):
    """bench.gathered_parity (rank 0, N > 1): every rank's batch is made again
    from its seed and checked against the all-gathered outputs.  The device
    synthesis is replaced by fixture frames chosen by the rank the seed
    encodes; one corrupted frame of rank 1 must be counted."""
    import sys
    import types
    import torch
    sys.path[:0] = [REPO, os.path.join(REPO, "gr-ldpc_ece535a_amd")]
    import bench
    from oracle import oracle as orc
    fd = np.load(os.path.join(REPO, "tests", "golden", "frames_default.npz"))
    Hr = fd["H_reordered"]
    allframes = np.concatenate([fd["db2_llr"], fd["db0_llr"], fd["db4_llr"]])
    world, B = 2, 48
    args = types.SimpleNamespace(batch=B, strong=strong, ebn0=2.0, seed=2024, method=1,
                                 iters=50, et_period=1)

    def fake_synth(L, torch_, dec, Br, ebn0, seed, dev):
        rk = (seed - args.seed) // 7919
        off, n = bench.plan_batch(B, world, rk, strong)
        assert n == Br
        return torch.from_numpy(allframes[off:off + n].copy()), None

    monkeypatch.setattr(bench, "synth_device", fake_synth)
    total = B if strong else world * B
    full = torch.from_numpy(orc.decode_batch(1, Hr, allframes[:total], 50)["packed"])
    r = bench.gathered_parity(None, torch, orc, None, args, None, full, world, Hr, None, 2,
                              sample=16)
    assert r["ranks"] == world and r["frames"] == 2 * 16 and r["gathered_frames"] == total
    assert r["packed_mismatch_frames"] == 0
    _, n0 = bench.plan_batch(B, world, 0, strong)
    full[n0 + 3] ^= 1  # rank 1's fourth frame
    r = bench.gathered_parity(None, torch, orc, None, args, None, full, world, Hr, None, 2,
                              sample=16)
    assert r["packed_mismatch_frames"] == 1
