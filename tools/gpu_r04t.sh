#!/bin/bash
# Round-4 session t: batcher with two dispatchers (OMR_BATCHER_WORKERS, default 2): batcher / pool /
# JNI GPU tests, then the serving legs with 1 and 2 dispatchers (bench host_fed section only).
set -o pipefail
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_batcher_gpu.py \
    tests/test_jni_shim_gpu.py tests/test_request_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in 1 2 1 2; do
  OMR_BATCHER_WORKERS=$w timeout -k 10 300 python -u tools/serving_probe.py > $O/serve_$w.json 2> $O/serve.err || { tail $O/serve.err; exit 1; }
  echo "workers $w: $(cat $O/serve_$w.json | cut -c1-400)"
done
echo R04T OK
