#!/bin/bash
# Round-4 session c: batcher projection / mask jobs, batched PNG (single path's stored blocks now
# carry the filtered rows), multi-stack projection; the batched-PNG kernel trace; the bench's C3
# gated-burst K3 timing; then the whole GPU suite.
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_png_batch_gpu.py tests/test_batcher_gpu.py tests/test_project_gpu.py \
    tests/test_encode_gpu.py -x -v --timeout 120 --timeout-method thread > $O/new_tests.log 2>&1 \
    || { tail -60 $O/new_tests.log; exit 1; }
tail -2 $O/new_tests.log
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/$O/pngtrace -o png -- \
    python3 $R/tools/png_batch_probe.py > $R/$O/png_probe_traced.json 2> $R/$O/png_trace.err ) || { tail $O/png_trace.err; exit 1; }
f=$(find $O/pngtrace -name '*kernel_trace.csv' | head -1)
python3 tools/trace_kernels.py $f $O/png_probe_kernels.csv && rm -rf $O/pngtrace
head -20 $O/png_probe_kernels.csv | cut -c1-160
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-jpeg --no-latency > $O/bench_c3c5.json \
    2> $O/bench_c3c5.err || { tail $O/bench_c3c5.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c3c5.json').read().strip().splitlines()[-1]); print(json.dumps(d['c3_projection'])[:1500]); print(json.dumps(d['c5_float']['roofline']))"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 \
    || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
echo R04C OK
