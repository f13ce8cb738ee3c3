#!/usr/bin/env python3
"""How often the exact arithmetic's rare paths run in the headline workload
(diagnostic).  Needs a library built with -DLDPC_PATH_STATS (tools/mkv.sh PS
-DLDPC_PATH_STATS; LDPC_PKG_DIR points at it).  Decodes K config-2 batches
through one ring session and prints, per wave-iteration of the column-centric
sum-product loop (csrc/ldpc_frame.hpp g_path_stats): the share where some
lane's check product T is +-1 / NaN (log's special path), where every real T
is +-1 / NaN / 0, where some |m| leaves [2^-54, 13.5) (tanh's special path),
where every |m| >= 38.2 or NaN (every tanh exactly +-1 or NaN), where every
check message repeats the previous iteration's bit for bit, and where every
check and bit message does (an exact fixed point of the iteration)."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.environ.get("LDPC_PKG_DIR", os.path.join(REPO, "gr-ldpc_ece535a_amd")))
import torch  # noqa: E402
import bench  # noqa: E402
import ldpc_ece535a as L  # noqa: E402

NAMES = ["wave-iterations", "some T = +-1 / NaN", "every real T in {+-1, NaN, 0}",
         "some nonzero |m| outside [2^-54, 13.5)", "every |m| >= 38.2 or NaN",
         "check messages repeat", "check and bit messages repeat (fixed point)",
         "some |m| >= 13.5 (expm1 k >= 20)", "near-1 log operands (sum)",
         "wave-iterations with > 64 near-1 operands", "near-1 operands with q == 1 (sum)",
         "wave-iterations with > 64 near-1 operands other than q == 1"]


def main():
    lib = L._capi.lib()
    if not hasattr(lib, "ldpc_debug_path_stats"):
        sys.exit("library built without -DLDPC_PATH_STATS")
    lib.ldpc_debug_path_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    dec = L.Decoder()
    B = 4096
    K = int(os.environ.get("K", "20"))
    for db in [float(x) for x in os.environ.get("EBN0", "2").split(",")]:
        ins = [bench.synth_device(L, torch, dec, B, db, 2024 + 104729 * j, dev)[0] for j in range(4)]
        pool = [(torch.empty((B, dec.KB), dtype=torch.uint8, device=dev),
                 torch.empty(B, dtype=torch.int32, device=dev),
                 torch.empty(B, dtype=torch.int32, device=dev)) for _ in range(K)]
        st = torch.cuda.Stream(dev)
        buf = np.zeros(12, np.uint64)
        torch.cuda.synchronize()
        lib.ldpc_debug_path_stats(buf.ctypes.data, 1)
        dec.ring_begin(method=1, max_iters=50, stream=ctypes.c_void_p(st.cuda_stream))
        for k in range(K):
            pk, it, sy = pool[k]
            dec.ring_post(ins[k % 4].data_ptr(), B, pk.data_ptr(), it.data_ptr(), sy.data_ptr())
        dec.ring_end()
        torch.cuda.synchronize()
        lib.ldpc_debug_path_stats(buf.ctypes.data, 1)
        iters = np.concatenate([p[1].cpu().numpy() for p in pool])
        n = float(buf[0])
        print("Eb/N0 %g dB: %d frames, mean iterations %.2f, %.1f%% at the cap" %
              (db, iters.size, iters.mean(), 100.0 * (iters >= 50).mean()))
        print("  %-46s %12d" % (NAMES[0], int(buf[0])))
        for i in range(1, 12):
            print("  %-46s %12d  %6.2f%%" % (NAMES[i], int(buf[i]), 100.0 * buf[i] / max(n, 1)))


if __name__ == "__main__":
    main()
