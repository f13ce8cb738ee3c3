#!/bin/bash
# One PMC pass of the bench workload per layout (planned vs LDPC_LAYOUT=0):
# LDS bank conflicts, LDS instructions, dependency waits, wave cycles.
# Run from the repo root via gpurun; output gpurun_out/pmc_ab/<variant>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
args="--no-cpu-baseline --no-variants --steps 50 --warmup 50 $*"
ctr="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES"
for v in planned plain; do
  out=gpurun_out/pmc_ab/$v
  mkdir -p "$out"
  if [ $v = plain ]; then export LDPC_LAYOUT=0; else unset LDPC_LAYOUT; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctr -d "$out" -o pmc --output-format csv \
    -- python3 bench.py $args > "$out/bench.log" 2>&1 || exit 1
  echo "$v done"
done
