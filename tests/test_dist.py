"""Sharding across ranks: world_size 2 with gloo on the CPU.
Each rank decodes its contiguous slice (here with the oracle as the decoder:
the GPU path is covered by bench.py on the box); gather_outputs must
reassemble exactly the unsharded result."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from ldpc_ece535a.dist import shard_range

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_range_partitions():
    for B in (0, 1, 7, 4096, 4097):
        for world in (1, 2, 3, 8):
            parts = [shard_range(B, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == B
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
            assert max(h - l for l, h in parts) - min(h - l for l, h in parts) <= 1


def _worker(rank, world, port, B, result_path):
    import sys
    sys.path[:0] = [REPO, os.path.join(REPO, "gr-ldpc_ece535a_amd")]
    import torch
    from ldpc_ece535a.dist import gather_outputs
    from oracle import oracle as orc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fd = np.load(os.path.join(REPO, "tests", "golden", "frames_default.npz"))
    Hr, y = fd["H_reordered"], fd["db2_llr"][:B]
    lo, hi = shard_range(B, rank, world)
    r = orc.decode_batch(1, Hr, y[lo:hi], 50)
    full, c = gather_outputs(dist, torch.from_numpy(r["packed"]),
                             [hi - lo, int(r["iters"].sum()), int((r["synd"] > 0).sum())])
    if rank == 0:
        np.savez(result_path, packed=full.numpy(), counters=np.array(c))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,B", [(2, 37), (2, 96)])
def test_gloo_sharded_decode_equals_unsharded(tmp_path, world, B):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(world, port, B, out), nprocs=world, join=True)
    from oracle import oracle as orc
    fd = np.load(os.path.join(REPO, "tests", "golden", "frames_default.npz"))
    ref = orc.decode_batch(1, fd["H_reordered"], fd["db2_llr"][:B], 50)
    got = np.load(out)
    assert (got["packed"] == ref["packed"]).all()
    assert list(got["counters"]) == [B, ref["iters"].sum(), (ref["synd"] > 0).sum()]
