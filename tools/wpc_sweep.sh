#!/bin/bash
# bench.py headline over persistent waves per CU x batches in flight (A/B aid)
for w in ${WPC:-2 3 4 6}; do for d in ${INFLIGHT:-4 8}; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --no-config4 --no-block \
    --steps 200 --warmup 100 --waves-per-cu $w --inflight $d > gpurun_out/wpc_${w}_${d}.json \
    2> gpurun_out/wpc_${w}_${d}.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/wpc_${w}_${d}.json'));print('wpc $w inflight $d', d['value'])"
done; done
