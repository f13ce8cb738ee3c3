#!/bin/bash
# Diagnostic: how much of the small-code kernel's LDS bank conflict count
# comes from the data-dependent log-table reads.  ab/P is the package built
# with -DLDPC_PROBE_LOGTAB_LANE (every lane reads its own table entry: the
# results are wrong, the other LDS traffic keeps its pattern); the in-tree
# build is the product.  One --pmc pass each, per dispatch means.
set -o pipefail
out=gpurun_out/probe_logtab
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
args="--no-cpu-baseline --no-variants --no-config4 --no-block --steps 20 --warmup 5"
LDPC_PKG_DIR=$PWD/ab/P timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU \
  -d "$out/P" -o P --output-format csv -- python3 bench.py $args > "$out/P.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU \
  -d "$out/T" -o T --output-format csv -- python3 bench.py $args > "$out/T.log" 2>&1
