#!/bin/bash
# Same-box A/B/n of the JPEG kernels: the in-tree libomr.so ("new") and ab/libomr_<v>.so for each
# argument v (OMR_LIB), alternating twice; per-kernel medians of tools/jpeg_probe.py traces.
set -o pipefail
R=$PWD; O=$R/gpurun_out/ab_jpeg_n; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
  for v in new "$@"; do
    if [ $v = new ]; then unset OMR_LIB; else export OMR_LIB=$R/ab/libomr_$v.so; fi
    JPEG_PROBE_ITERS=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/$v$i -o t -- python3 $R/tools/jpeg_probe.py > $O/$v$i.log 2>&1 || exit $?
    f=$(find $O/$v$i -name '*kernel_trace.csv' | head -1)
    echo "== $v $i"; python3 $R/tools/trace_summary.py $f | grep -E "fdct|huff|block_bits|stuff|group_scan|tile_scan"
    rm -rf $O/$v$i
  done
done
