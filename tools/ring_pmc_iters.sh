#!/bin/bash
# Per-frame against per-iteration VALU of the ring: PMC instruction counts of
# 50-batch ring sessions with the iteration cap at 1, 2 and 50 (2 dB: at caps 1
# and 2 every frame runs the cap).  Output: gpurun_out/r6/rpmc_iters/
set -o pipefail
out=gpurun_out/r6/rpmc_iters
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for it in 1 2 50; do
  ITERS=$it MODE=ring K=50 timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_SALU \
    -d "$out/it$it" -o p1 --output-format csv -- python3 tools/ring_probe.py > "$out/it$it.log" 2>&1 || { echo "iters $it failed"; exit 1; }
done
echo done
