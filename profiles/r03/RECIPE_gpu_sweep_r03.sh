#!/bin/bash
# Wider randomised parity sweeps on the GPU (render incl. the fused render -> JPEG batch, JPEG
# sizes/qualities, projection glue) at OMR_SWEEP_SEEDS seeds each; log under gpurun_out/<tag>/.
set -o pipefail
O=gpurun_out/${1:-sweep_r03}; mkdir -p $O
OMR_SWEEP_SEEDS=${SEEDS:-600} timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_render_sweep_gpu.py tests/test_jpeg_batch_gpu.py::test_jpeg_sweep_sizes_qualities \
    tests/test_project_gpu.py::test_projection_glue_sweep > $O/sweep.log 2>&1 || { tail -30 $O/sweep.log; exit 1; }
tail -1 $O/sweep.log
