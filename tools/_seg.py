import os, sys, faulthandler
faulthandler.enable()
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "gr-ldpc_ece535a_amd"))
import torch  # noqa
import numpy as np
print("imported torch", flush=True)
import ldpc_ece535a as L
from ldpc_ece535a import flowgraph as fg
from oracle import oracle as orc
st = np.load(os.path.join(REPO, "tests/golden/streams.npz"))
paths = {"serve": {}, "launch": {"LDPC_BLOCK_SERVE": "0"},
         "plan": {"LDPC_BLOCK_MAXWANT": "64", "LDPC_BLOCK_SEARCHES": "1"},
         "diag": {"LDPC_BLOCK_DEBUG": "2", "LDPC_BLOCK_PROFILE": "2",
                  "LDPC_SERVE_DEBUG": "1"}}
for path in sys.argv[1].split(","):
    for name in ["aligned", "offset"]:
        for method in [0, 1]:
            os.environ.update(paths[path])
            print("make", path, name, method, flush=True)
            blk = L.ldpc_decoder_cb(method)
            for k in paths[path]:
                os.environ.pop(k, None)
            s = st[name + "_in"]
            tb = fg.top_block(chunk=[97, 13, 640, 5, 2000] * 4)
            src, dst = fg.vector_source_c(s), fg.vector_sink_b()
            tb.connect((src, 0), (blk, 0)); tb.connect((blk, 0), (dst, 0))
            print("run", flush=True)
            tb.run()
            print(path, name, method, dst.array().size, (dst.array() == st[name + "_m%d_out" % method]).all(), flush=True)
