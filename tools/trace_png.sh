#!/bin/bash
# Kernel trace of tools/png_probe.py (PNG encode pipeline), per-kernel medians in png_kernels.txt.
set -o pipefail
R=$PWD; O=$R/gpurun_out/${TRACE_TAG:-png_trace}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O -o t -- python3 $R/tools/png_probe.py > $O/probe.log 2>&1 || exit $?
find $O -name '*kernel_trace.csv' -exec cp {} $O/kernel_trace.csv \;
find $O -name '*memory_copy_trace.csv' -exec cp {} $O/copy_trace.csv \; || true
echo done
