#!/bin/bash
# Round-4 session b: the batched PNG tests (new kernels first, short limit), the full GPU suite,
# the batched PNG probe, C3 K3 event timing with and without the system-scope fence against a
# rocprofv3 kernel trace of the same probe, then the all-sections profile (tools/profile_r04.sh).
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_png_batch_gpu.py -x -v --timeout 120 --timeout-method thread \
    > $O/png_batch_tests.log 2>&1 || { tail -40 $O/png_batch_tests.log; exit 1; }
tail -2 $O/png_batch_tests.log
timeout -k 10 180 python -u tools/png_batch_probe.py > $O/png_probe.json 2> $O/png_probe.err || { tail $O/png_probe.err; exit 1; }
cat $O/png_probe.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 \
    || { tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 120 python -u tools/c3_probe.py > $O/c3_nofence.json 2> $O/c3.err || exit 1
OMR_TIMING_FENCE=1 timeout -k 10 120 python -u tools/c3_probe.py > $O/c3_fence.json 2>> $O/c3.err || exit 1
cat $O/c3_nofence.json $O/c3_fence.json
R=$PWD
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $R/$O/c3trace -o c3 -- \
    python3 $R/tools/c3_probe.py > $R/$O/c3_traced.json 2> $R/$O/c3_trace.err ) || exit 1
f=$(find $O/c3trace -name '*kernel_trace.csv' | head -1)
python3 tools/trace_kernels.py $f $O/c3_probe_kernels.csv && rm -rf $O/c3trace
timeout -k 10 900 bash tools/profile_r04.sh r04b_prof || exit $?
echo R04B OK
