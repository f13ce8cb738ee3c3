#!/bin/bash
# Collects the rocprofv3 evidence for the bench workload on the GPU box:
#   1. --kernel-trace --stats (kernel durations)
#   2. separate --pmc passes (SQ instruction mix, LDS conflicts, waits;
#      FETCH_SIZE; WRITE_SIZE), each within the per-block counter limits
# Run from the repo root, via gpurun.  Output: gpurun_out/prof/<tag>/...
# usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
tag=${1:-run}; shift
out=gpurun_out/prof/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
args="--no-cpu-baseline --no-variants --steps 100 --warmup 200 $*"
run() {  # name, rocprof options...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$out/$name" -o "$name" --output-format csv \
    -- python3 bench.py $args > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run kt --kernel-trace --stats &&
run pmc1 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT &&
run pmc2 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE &&
run pmc3 --kernel-trace --pmc FETCH_SIZE &&
run pmc4 --kernel-trace --pmc WRITE_SIZE
