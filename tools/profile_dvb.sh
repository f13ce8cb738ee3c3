#!/bin/bash
# rocprofv3 evidence for config 4 (DVB-S2-like code, min-sum f64, B = 1024):
# kernel trace + FETCH_SIZE / WRITE_SIZE passes, for the default min-sum
# pipeline (compressed check messages) and, with LDPC_MS_PIPELINE=0, the
# edge-message passes.  Output: gpurun_out/prof/dvb_{ms,edge}/...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
args="--code dvbs2 --steps 2 --warmup 0 --inflight 1 --no-cpu-baseline"
for v in ${DVB_VARIANTS:-ms edge}; do
  out=gpurun_out/prof/dvb_$v
  mkdir -p $out
  if [ $v = edge ]; then export LDPC_MS_PIPELINE=0; else unset LDPC_MS_PIPELINE; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/kt -o kt --output-format csv -- python3 bench.py $args > $out/kt.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/pmc3 -o pmc3 --output-format csv -- python3 bench.py $args > $out/pmc3.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/pmc4 -o pmc4 --output-format csv -- python3 bench.py $args > $out/pmc4.log 2>&1 || exit 1
  echo "$v ok"
done
