#!/bin/bash
# Round-4 session p: host-fed bands merged into file-order copies, group-size variants
# (tools/hostfed_probe.py, 64 and 256 tiles per call), pixel-buffer GPU tests; then the JPEG SQ
# profile of the current build (tools/profile_jpeg_r04.sh).
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_request_gpu.py \
    tests/test_batcher_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for n in 64 256; do
  HOSTFED_TILES=$n timeout -k 10 240 python3 tools/hostfed_probe.py > $O/hostfed_$n.json 2> $O/hostfed.err \
      || { tail $O/hostfed.err; exit 1; }
  cat $O/hostfed_$n.json
done
timeout -k 10 700 bash tools/profile_jpeg_r04.sh r04p_jpeg || exit 1
echo R04P OK
