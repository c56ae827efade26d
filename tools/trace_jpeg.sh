set -o pipefail
R=$PWD; O=$R/gpurun_out/${TRACE_TAG:-jpeg_trace0}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
JPEG_PROBE_ITERS=10 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o t -- python3 $R/tools/jpeg_probe.py > $O/c2.log 2>&1 || exit $?
find $O -name '*kernel_stats.csv' -exec cp {} $O/c2_stats.csv \;
find $O -name '*kernel_trace.csv' -exec cp {} $O/c2_trace.csv \;
echo done
