#!/bin/bash
# Round-4 session k: B2a/B3 coefficient loads no longer wait for the block record (B2a loads the int8 form with
# the record; B3 learns the form from B2a's bits word): JPEG GPU tests, rate A/B against ab/libomr_n1.so (previous
# commit) and ab/libomr_dot2.so, the C2 256-tile kernel trace, FETCH/WRITE passes for the JPEG kernels.
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
R=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_jpeg_batch_gpu.py tests/test_render_jpeg_gpu.py tests/test_encode_gpu.py tests/test_request_gpu.py \
    > $O/jpeg_tests.log 2>&1 || { tail -30 $O/jpeg_tests.log; exit 1; }
tail -1 $O/jpeg_tests.log
for i in 1 2; do
  for v in new n1 dot2; do
    case $v in dot2) export OMR_LIB=$R/ab/libomr_dot2.so ;; n1) export OMR_LIB=$R/ab/libomr_n1.so ;; *) unset OMR_LIB ;; esac
    for c in c2 c1; do
      JPEG_PROBE_CASE=$c timeout -k 10 120 python3 tools/jpeg_rate.py > $O/rate_${c}_${v}$i.json 2> $O/rate.err || { tail $O/rate.err; exit 1; }
      echo "$c $v run $i: $(cut -c1-110 $O/rate_${c}_${v}$i.json)"
    done
  done
done
unset OMR_LIB
( cd /tmp && export TMPDIR=/tmp && JPEG_PROBE_TILES=256 JPEG_PROBE_ITERS=6 timeout -k 10 240 rocprofv3 --kernel-trace \
    --output-format csv -d $R/$O/jtrace -o j -- python3 $R/tools/jpeg_probe.py > $R/$O/jpeg_trace.log 2>&1 ) \
    || { tail $O/jpeg_trace.log; exit 1; }
f=$(find $O/jtrace -name '*kernel_trace.csv' | head -1)
python3 tools/trace_kernels.py $f $O/jpeg_c2_256_kernels.csv && rm -rf $O/jtrace
grep -E "jpeg|k_render|k_build" $O/jpeg_c2_256_kernels.csv | cut -c1-120
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  JPEG_PROBE_TILES=256 JPEG_PROBE_ITERS=2 timeout -s KILL 180 rocprofv3 --pmc $c --kernel-include-regex "k_jpeg|k_render" \
      --output-format csv -d $R/$O/pmc_jpeg_$c -o p -- python3 $R/tools/jpeg_probe.py > /dev/null 2> $R/$O/pmc_jpeg_$c.err \
      || { echo "pmc $c failed"; tail -5 $R/$O/pmc_jpeg_$c.err; exit 1; }
done
python3 $R/tools/pmc_traffic.py $R/$O/pmc_traffic_jpeg.json $(find $R/$O -path "*pmc_jpeg_*" -name '*counter_collection.csv') \
    > $R/$O/pmc_traffic_jpeg.txt || exit 1
find $R/$O -path "*pmc_jpeg_*" -name '*counter_collection.csv' -delete
cat $R/$O/pmc_traffic_jpeg.txt | cut -c1-150
echo R04I OK
