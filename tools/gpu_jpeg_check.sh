#!/bin/bash
# JPEG iteration step on the GPU box: the JPEG / render-JPEG GPU tests (byte identity against the
# CPU restatement), then a same-box A/B of the JPEG kernels against ab/libomr_old.so.
set -o pipefail
O=gpurun_out/${1:-jpegcheck}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_jpeg_batch_gpu.py tests/test_render_jpeg_gpu.py tests/test_encode_gpu.py tests/test_batcher_gpu.py \
    > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
[ -f ab/libomr_old.so ] && { bash tools/ab_jpeg.sh > $O/ab.txt 2>&1 || exit $?; cat $O/ab.txt; }
exit 0
