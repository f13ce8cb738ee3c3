#!/bin/bash
# tools/ab_ring.sh V1 V2 ...: headline ring throughput (tools/ring_probe.py, 20-batch
# sessions) of the working tree (NEW) and of variant builds ab/V (tools/mkv.sh), alternated
set -o pipefail
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for v in NEW "$@"; do
    if [ $v = NEW ]; then unset LDPC_PKG_DIR; else export LDPC_PKG_DIR=$PWD/ab/$v; fi
    K=20 VARIANTS=0 timeout -k 10 200 python -u tools/ring_probe.py > gpurun_out/ab/ring_$v.$r.txt 2>&1 || { tail -5 gpurun_out/ab/ring_$v.$r.txt; exit 1; }
    echo "$v $r $(grep 'probe 0' gpurun_out/ab/ring_$v.$r.txt)"
  done
done
