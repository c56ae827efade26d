#!/bin/bash
# Same-box A/B of the C5 K2 variants inside the bench itself (its prewarm and per-launch events):
# OMR_K2_EVAL_CPT=-2 (pipelined, default) vs 2 (plain grid stride), alternating.
set -o pipefail
O=gpurun_out/c5bench; mkdir -p $O
for i in 1 2; do
  for v in -2 2; do
    OMR_K2_EVAL_CPT=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-jpeg --no-latency \
        > $O/b_$v$i.json 2> $O/b_$v$i.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('$O/b_$v$i.json').read().strip().splitlines()[-1])['c5_float']; print('cpt $v run $i', d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
  done
done
