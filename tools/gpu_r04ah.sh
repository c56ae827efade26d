#!/bin/bash
# Round-4 session ah: F1 Fast16FU (unsigned, unchecked fast16-f32: sign bias and domain check compiled out; 84 SGPRs, 8 waves; loop VALU 423 -> 382)
# workgroup barrier) + B6 held to 8 waves per SIMD (77 -> 60 VGPRs): JPEG GPU tests, then a
# same-box rate A/B/n (in-tree = both, ab/libomr_b6.so = B6 only, ab/libomr_head.so = committed),
# then the C2 256-tile kernel trace.
set -o pipefail
O=gpurun_out/r04ah; mkdir -p $O
R=$PWD
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_jpeg_batch_gpu.py tests/test_render_jpeg_gpu.py tests/test_encode_gpu.py > $O/jpeg_tests.log 2>&1 \
    || { tail -30 $O/jpeg_tests.log; exit 1; }
tail -1 $O/jpeg_tests.log
for i in 1 2; do
  for v in new head; do
    if [ $v = new ]; then unset OMR_LIB; else export OMR_LIB=$R/ab/libomr_$v.so; fi
    for c in c2 c1; do
      JPEG_PROBE_CASE=$c timeout -k 10 120 python3 tools/jpeg_rate.py > $O/rate_${c}_${v}$i.json 2> $O/rate.err || { tail $O/rate.err; exit 1; }
      echo "$c $v run $i: $(cut -c1-100 $O/rate_${c}_${v}$i.json)"
    done
  done
done
unset OMR_LIB
( cd /tmp && export TMPDIR=/tmp && JPEG_PROBE_TILES=256 JPEG_PROBE_ITERS=6 timeout -k 10 240 rocprofv3 --kernel-trace \
    --output-format csv -d $R/$O/jtrace -o j -- python3 $R/tools/jpeg_probe.py > $R/$O/jpeg_trace.log 2>&1 ) \
    || { tail $O/jpeg_trace.log; exit 1; }
f=$(find $O/jtrace -name '*kernel_trace.csv' | head -1)
python3 tools/trace_kernels.py $f $O/jpeg_c2_256_kernels.csv && rm -rf $O/jtrace
grep -E "jpeg|k_render<" $O/jpeg_c2_256_kernels.csv | cut -c1-120
echo R04AH OK
