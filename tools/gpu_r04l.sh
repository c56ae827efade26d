#!/bin/bash
# Round-4 session l: F1 store variants, same-box C2/C1 rate A/B (tools/jpeg_rate.py):
# head = committed (int16/int8 store per block in a branch, 64 VGPRs forced); v1 = int8 stores
# unconditional + one int16 branch, 65 VGPRs (7 waves); v2 = v1 held to 64 VGPRs (12 B spill).
set -o pipefail
O=gpurun_out/r04l; mkdir -p $O
R=$PWD
for i in 1 2; do
  for v in head v1 v2; do
    export OMR_LIB=$R/ab/libomr_$v.so
    for c in c2 c1; do
      JPEG_PROBE_CASE=$c timeout -k 10 120 python3 tools/jpeg_rate.py > $O/rate_${c}_${v}$i.json 2> $O/rate.err || { tail $O/rate.err; exit 1; }
      echo "$c $v run $i: $(cut -c1-100 $O/rate_${c}_${v}$i.json)"
    done
  done
done
echo R04L OK
