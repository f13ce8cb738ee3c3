"""Host cost of enqueueing decodes: per-call time of the bench's step loop
(ldpc_decode_device on four streams) against the device time of the same
launches, for a fast variant (min-sum f64) and the headline (SP f64).  If
the enqueue loop is as slow as the batches it enqueues, the variant's
Mbit/s is a host figure, not a kernel one."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gr-ldpc_ece535a_amd"))

import bench  # noqa: E402


def main():
    import ctypes
    import torch
    import ldpc_ece535a as L
    dev = torch.device("cuda", 0)
    dec = L.Decoder()
    dec.set_launch_mode(1)
    B = 4096
    ins = [bench.synth_device(L, torch, dec, B, 2.0, 2024 + j, dev)[0] for j in range(4)]
    streams = [torch.cuda.Stream(dev) for _ in range(4)]
    sps = [ctypes.c_void_p(s.cuda_stream) for s in streams]
    outs = [torch.empty((B, dec.KB), dtype=torch.uint8, device=dev) for _ in range(4)]
    for m, p in ((0, 0), (1, 1), (1, 0)):
        for rep in range(2):
            K = 400
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(K):
                d = k % 4
                dec.decode_device(ins[d].data_ptr(), B, outs[d].data_ptr(), method=m, max_iters=50,
                                  precision=p, stream=sps[d])
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print("method %d prec %d: enqueue %.1f us/call, wall %.1f us/batch -> %.0f Mbit/s"
                  % (m, p, (t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6,
                     B * dec.K * K / (t2 - t0) / 1e6), flush=True)
    # the C call alone, no Python wrapper: ctypes straight into the ABI
    lib = L._capi.lib()
    for rep in range(2):
        K = 400
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            d = k % 4
            lib.ldpc_decode_device(dec._ctx, 0, 50, 1, 0, ins[d].data_ptr(), dec.N, 1, 1.0, B,
                                   outs[d].data_ptr(), None, None, None, None, sps[d])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("raw ctypes min-sum: enqueue %.1f us/call, wall %.1f us/batch" %
              ((t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6), flush=True)


if __name__ == "__main__":
    main()
