#!/bin/bash
# The drop-in block at the reference's own make(method) settings (5
# iterations, 4 dB stream): host split (LDPC_BLOCK_PROFILE: exact replay /
# dry runs / decode round trips) and a rocprofv3 kernel trace of the same
# run.  Output under gpurun_out/blk5 (copy what is kept to profiles/).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/blk5
mkdir -p "$out"
cd "$R"
ITERS=${ITERS:-5}
DB=${DB:-4}
LDPC_BLOCK_PROFILE=1 timeout -k 10 180 python tools/block_bench.py --iters $ITERS --ebn0 $DB \
  --reps 4 > "$out/split.txt" 2>&1
export TMPDIR=/tmp
LDPC_BLOCK_PROFILE=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o blk \
  -- python3 tools/block_bench.py --iters $ITERS --ebn0 $DB --reps 4 > "$out/kt.log" 2>&1
