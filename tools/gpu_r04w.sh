#!/bin/bash
# Round-4 session w: B1/F1 MCUs per wave (kB1McuPerWave) 8 (in-tree) vs 4 vs 10, same-box C2/C1 rates.
set -o pipefail
O=gpurun_out/r04w; mkdir -p $O
R=$PWD
for i in 1 2; do
  for v in m8 m4 m10; do
    if [ $v = m8 ]; then unset OMR_LIB; else export OMR_LIB=$R/ab/libomr_$v.so; fi
    for c in c2 c1; do
      JPEG_PROBE_CASE=$c timeout -k 10 120 python3 tools/jpeg_rate.py > $O/rate_${c}_${v}$i.json 2> $O/rate.err || { tail $O/rate.err; exit 1; }
      echo "$c $v run $i: $(cut -c1-100 $O/rate_${c}_${v}$i.json)"
    done
  done
done
echo R04W OK
