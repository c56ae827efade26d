#!/bin/bash
# Round-4 session e: multi-row SWAR PNG filter, HBM stack cache, serving legs for projection and
# shape masks: PNG / batcher / JNI GPU tests, traced batched-PNG probe, bench without the JPEG leg.
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
R=$PWD
timeout -k 10 500 python -u -m pytest tests/test_png_batch_gpu.py tests/test_encode_gpu.py tests/test_batcher_gpu.py \
    tests/test_jni_shim_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/$O/pngtrace -o png -- \
    python3 $R/tools/png_batch_probe.py > $R/$O/png_probe_traced.json 2> $R/$O/png_trace.err ) || { tail $O/png_trace.err; exit 1; }
f=$(find $O/pngtrace -name '*kernel_trace.csv' | head -1)
python3 tools/trace_kernels.py $f $O/png_probe_kernels.csv && rm -rf $O/pngtrace
grep -E "pngb" $O/png_probe_kernels.csv | cut -c1-110
cat $O/png_probe_traced.json
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-jpeg --no-latency > $O/bench.json \
    2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(json.dumps(d['png'])); print(json.dumps(d['host_fed']['serving']))"
echo R04E OK
