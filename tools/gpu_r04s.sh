#!/bin/bash
# Round-4 session s: the new mixed int8 / int16 coefficient-block tests (batch and fused paths).
set -o pipefail
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_jpeg_batch_gpu.py tests/test_render_jpeg_gpu.py -k "int8_and_int16" > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo R04S OK
