"""The multi-GPU gather over RCCL, executed.

bench.py's N-rank path initialises `init_process_group("nccl", device_id=...)`
(RCCL on ROCm) and, after the timed loop, all-gathers the packed outputs
(uint8 device tensors) and all-reduces the counters (f64) and the wall time
(f64, MAX) through ldpc_ece535a.dist.gather_outputs / bench.reduce_results.
The box has one GPU, so this runs that exact code over RCCL at world size 1
in a child process (its own RCCL communicator, torn down at exit): ragged
gathers and multi-rank reductions are covered by the gloo tests
(tests/test_dist.py, tests/test_bench_dist.py); what only hardware can show
-- the nccl backend, device_id binding, device-tensor collectives of these
dtypes -- is shown here."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
sys.path[:0] = [@@REPO@@, os.path.join(@@REPO@@, "gr-ldpc_ece535a_amd")]
import numpy as np
import torch
import torch.distributed as dist
import bench
import ldpc_ece535a as L
from oracle import oracle as orc

os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=@@PORT@@, RANK="0", WORLD_SIZE="1")
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=dev)
assert dist.get_backend() == "nccl"
dec = L.Decoder(device=0)
B = 1000
y, _ = bench.synth(dec.H, B, 2.0, 77)
d_y = torch.from_numpy(y).to(dev)
packed = torch.empty((B, dec.KB), dtype=torch.uint8, device=dev)
iters = torch.empty(B, dtype=torch.int32, device=dev)
dec.decode_device(d_y.data_ptr(), B, packed.data_ptr(), method=1, max_iters=50,
                  d_iters=iters.data_ptr())
dec.synchronize()
counters = [B, int(iters.sum().item()), 0.5]
full, c, wall = bench.reduce_results(dist, packed, counters, 0.125, dev)
assert full.device.type == "cuda" and full.dtype == torch.uint8
ref = orc.decode_batch(1, dec.H, y, 50, nthreads=8)
# a second, explicit collective of each dtype the bench uses
x = torch.arange(7, dtype=torch.float64, device=dev)
dist.all_reduce(x, op=dist.ReduceOp.MAX)
parts = [torch.empty(5, dtype=torch.uint8, device=dev)]
dist.all_gather(parts, torch.full((5,), 9, dtype=torch.uint8, device=dev))
torch.cuda.synchronize()
out = dict(backend=dist.get_backend(), gathered=int(full.shape[0]),
           packed_equal=bool((full.cpu().numpy() == packed.cpu().numpy()).all()),
           oracle_equal=bool((full.cpu().numpy() == ref["packed"]).all()),
           counters=c, expect=[float(B), float(ref["iters"].sum()), 0.5], wall=wall,
           f64_ok=x.cpu().tolist() == list(range(7)), u8_ok=parts[0].cpu().tolist() == [9] * 5)
dist.destroy_process_group()
print("RESULT " + json.dumps(out))
"""


def test_rccl_world1_gather_and_reduce():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    code = CHILD.replace("@@REPO@@", repr(REPO)).replace("@@PORT@@", repr(str(port)))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                       env=env, cwd=REPO)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")][-1]
    r = json.loads(line[7:])
    assert r["backend"] == "nccl"
    assert r["gathered"] == 1000 and r["packed_equal"] and r["oracle_equal"]
    assert r["counters"] == r["expect"] and r["wall"] == 0.125
    assert r["f64_ok"] and r["u8_ok"]
