#!/bin/bash
# Round-4 session g: host -> HBM copy shapes (tools/pcie_probe); JPEG B1/F1 colour transform on
# v_dot2 + DC records by v_writelane: JPEG GPU tests, same-box rate A/B against ab/libomr_old.so
# (and ab/libomr_b3pf.so: B3 reading the next coefficient's code entry ahead);
# C5 buckets holding their code's contribution: render GPU tests, bench A/B.
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 120 ./tools/pcie_probe > $O/pcie_probe.json 2> $O/pcie_probe.err || { cat $O/pcie_probe.err; exit 1; }
cat $O/pcie_probe.json
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_jpeg_batch_gpu.py tests/test_render_jpeg_gpu.py tests/test_request_gpu.py tests/test_batcher_gpu.py > $O/jpeg_tests.log 2>&1 || { tail -30 $O/jpeg_tests.log; exit 1; }
tail -1 $O/jpeg_tests.log
for i in 1 2; do
  for v in new b3pf old; do
    case $v in old) export OMR_LIB=$PWD/ab/libomr_old.so ;; b3pf) export OMR_LIB=$PWD/ab/libomr_b3pf.so ;; *) unset OMR_LIB ;; esac
    for c in c2 c1; do
      JPEG_PROBE_CASE=$c timeout -k 10 120 python3 tools/jpeg_rate.py > $O/rate_${c}_${v}$i.json 2> $O/rate.err || { tail $O/rate.err; exit 1; }
      echo "$c $v run $i: $(cut -c1-110 $O/rate_${c}_${v}$i.json)"
    done
  done
done
unset OMR_LIB
timeout -k 10 900 bash tools/c5_lib_ab.sh || exit $?
echo R04G OK
