#!/bin/bash
# rocprofv3 evidence for the config-4 min-sum pipelines (DVB-S2-like code,
# B = 1024): kernel trace, then one PMC pass per counter group (L2 hits /
# misses; memory-side fetch / write bytes).  MSN_MODES lists the
# LDPC_MS_PIPELINE values to profile (2 narrow chunks, 1 64-frame chunks).
# Output: gpurun_out/prof/msn_<mode>/...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
args="--code dvbs2 --steps 2 --warmup 0 --inflight 1 --no-cpu-baseline --no-variants"
for m in ${MSN_MODES:-2 1}; do
  out=gpurun_out/prof/msn_$m
  mkdir -p $out
  export LDPC_MS_PIPELINE=$m LDPC_MSN_DEBUG=1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- python3 bench.py $args > $out/kt.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $out/pmc1 -o pmc1 --output-format csv -- python3 bench.py $args > $out/pmc1.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/pmc2 -o pmc2 --output-format csv -- python3 bench.py $args > $out/pmc2.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/pmc3 -o pmc3 --output-format csv -- python3 bench.py $args > $out/pmc3.log 2>&1 || exit 1
  echo "mode $m ok"
done
