#!/bin/bash
# Ablation study of the JPEG first kernels (B1 k_jpeg_fdct_batch, F1 k_jpeg_render_fdct): libomr
# variants with one part of the MCU body removed (-DOMR_ABL=<mask>, see omr_jpeg.hip; their
# outputs are wrong) timed by rocprofv3 kernel traces of tools/jpeg_probe.py (64 C2 tiles).
#   build (CPU, here):  tools/ablate_jpeg.sh build
#   run (GPU box):      tools/ablate_jpeg.sh run
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
MASKS=${ABL_MASKS:-"0 2 4 8 16 32 64 127"}
if [ "$1" = build ]; then
  cd $R/omero-ms-image-region_amd
  for m in $MASKS; do
    mkdir -p $R/ab/abl$m
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -I../include \
        -Icsrc -Wall -Wno-unused-function -Wno-pass-failed -DOMR_ABL=$m -c -x hip csrc/omr_jpeg.hip \
        -o $R/ab/abl$m/omr_jpeg.o || exit 1
    objs=$(ls build/*.o | grep -v omr_jpeg.o)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/ab/libomr_abl$m.so $objs $R/ab/abl$m/omr_jpeg.o || exit 1
    rm -rf $R/ab/abl$m
  done
  exit 0
fi
O=$R/gpurun_out/ablate_jpeg; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in $MASKS; do
  export OMR_LIB=$R/ab/libomr_abl$m.so
  JPEG_PROBE_ITERS=10 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/a$m -o t -- \
      python3 $R/tools/jpeg_probe.py > $O/a$m.log 2>&1 || exit $?
  f=$(find $O/a$m -name '*kernel_trace.csv' | head -1)
  echo "== mask $m"; python3 $R/tools/trace_summary.py $f | grep -E "fdct"
  rm -rf $O/a$m
done
