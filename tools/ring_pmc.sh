#!/bin/bash
# PMC passes over tools/ring_probe.py, ring vs a launch per batch (MODE),
# K batches per session.  Output: gpurun_out/r6/rpmc/<mode>_<pass>/
set -o pipefail
out=gpurun_out/r6/rpmc
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for mode in ring launch; do
  for pass in "kt --kernel-trace --stats" \
              "p1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_SALU" \
              "p2 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM" ; do
    set -- $pass
    name=$1; shift
    MODE=$mode K=50 timeout -k 10 120 rocprofv3 "$@" -d "$out/${mode}_$name" -o "$name" --output-format csv \
      -- python3 tools/ring_probe.py > "$out/${mode}_$name.log" 2>&1 || { echo "$mode $name failed"; exit 1; }
  done
done
echo done
