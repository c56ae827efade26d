#!/bin/bash
# A/B of the C5 threshold-mode K2 on one box: tools/c5_probe.py with the in-tree libomr.so and the
# variants under ab/ (OMR_LIB), alternating; one JSON line per run (per-launch K2 median, checksum).
set -o pipefail
R=$PWD; O=$R/gpurun_out/ab_c5; mkdir -p $O
for i in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset OMR_LIB; else export OMR_LIB=$R/ab/libomr_$v.so; fi
    echo -n "$v $i "; C5_TILES=64 timeout -k 10 120 python3 $R/tools/c5_probe.py 2> $O/$v$i.err || exit $?
  done
done
