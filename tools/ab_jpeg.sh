#!/bin/bash
# A/B of the JPEG kernels on one box: kernel traces of tools/jpeg_probe.py with the in-tree
# libomr.so and with ab/libomr_old.so (OMR_LIB), alternating, per-kernel medians.
set -o pipefail
R=$PWD; O=$R/gpurun_out/ab_jpeg; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export OMR_LIB=$R/ab/libomr_old.so; else unset OMR_LIB; fi
    JPEG_PROBE_ITERS=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/$v$i -o t -- python3 $R/tools/jpeg_probe.py > $O/$v$i.log 2>&1 || exit $?
    f=$(find $O/$v$i -name '*kernel_trace.csv' | head -1)
    echo "== $v $i"; python3 $R/tools/trace_summary.py $f | grep -E "fdct|huff|block_bits|stuff|group_scan|tile_scan"
    rm -rf $O/$v$i
  done
done
