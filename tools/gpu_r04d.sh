#!/bin/bash
# Round-4 session d: PNG filter (dword LDS, staged output) + mask-based LZ parse + packed tokens:
# every PNG test (decoded pixels, batch == single path), then the traced batched-PNG probe.
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
R=$PWD
timeout -k 10 400 python -u -m pytest tests/test_png_batch_gpu.py tests/test_encode_gpu.py tests/test_batcher_gpu.py \
    -x -q --timeout 120 --timeout-method thread > $O/png_tests.log 2>&1 || { tail -60 $O/png_tests.log; exit 1; }
tail -2 $O/png_tests.log
timeout -k 10 180 python -u tools/png_batch_probe.py > $O/png_probe.json 2> $O/png_probe.err || { tail $O/png_probe.err; exit 1; }
cat $O/png_probe.json
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/$O/pngtrace -o png -- \
    python3 $R/tools/png_batch_probe.py > $R/$O/png_probe_traced.json 2> $R/$O/png_trace.err ) || { tail $O/png_trace.err; exit 1; }
f=$(find $O/pngtrace -name '*kernel_trace.csv' | head -1)
python3 tools/trace_kernels.py $f $O/png_probe_kernels.csv && rm -rf $O/pngtrace
grep -E "pngb|k_png" $O/png_probe_kernels.csv | cut -c1-130
echo R04D OK
