#!/bin/bash
# C5 K2 chunk/pipeline variants on one box (OMR_K2_EVAL_CPT: -1 / -2 pipelined, 2 / 4 plain
# grid stride), alternating, after the render GPU tests; one JSON line per run.
set -o pipefail
O=gpurun_out/${1:-c5cpt}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_render_gpu.py tests/test_semantics_gpu.py tests/test_render_sweep_gpu.py > $O/tests.log 2>&1 \
    || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in -1 -2 2; do
    echo -n "cpt $v run $i: "; OMR_K2_EVAL_CPT=$v C5_TILES=64 timeout -k 10 120 python3 tools/c5_probe.py 2> $O/c5_$v$i.err || exit $?
  done
done
