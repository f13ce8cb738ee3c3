#!/bin/bash
# tools/ab_block.sh: the block, make(1) at 4 dB / 5 iterations: HEAD build (ab/OLD) vs the working tree, alternated
# (ab/OLD: tools/mkv.sh OLD built from the baseline revision's checkout)
set -o pipefail
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for v in OLD NEW; do
    if [ $v = NEW ]; then unset LDPC_PKG_DIR; else export LDPC_PKG_DIR=$PWD/ab/$v; fi
    timeout -k 10 200 python tools/block_bench.py --iters 5 --ebn0 4 --reps 6 > gpurun_out/ab/blk_$v.$r.txt 2>&1 || { tail -5 gpurun_out/ab/blk_$v.$r.txt; exit 1; }
    echo "$v $r $(grep -i 'mbit' gpurun_out/ab/blk_$v.$r.txt | head -1)"
  done
done
unset LDPC_PKG_DIR
LDPC_SERVE_DEBUG=1 timeout -k 10 200 python tools/block_bench.py --iters 5 --ebn0 4 --reps 4 2>&1 | grep "rounds: host" | head -4
