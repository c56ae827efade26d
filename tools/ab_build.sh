#!/bin/bash
# Build a variant of libomr.so for a same-box A/B (runs here, on the CPU; the GPU side is
# `tools/gpu.sh <tag> ab=<probe>:<name>[,<name>...]`, which alternates the in-tree library with
# ab/libomr_<name>.so through OMR_LIB).
#
#   tools/ab_build.sh <name> [extra hipcc flags, e.g. -DOMR_ABL=4 -DOMR_F1_DEPTH=1]
#
# Every HIP source is recompiled with the extra flags (AB_SOURCES="omr_png ..." limits that to the
# named sources, the rest coming from the in-tree build); the host C++ objects come from the
# in-tree build (make first).  The current working tree is what gets built: to A/B against an older
# revision, `git stash` / checkout it, build the variant, and restore.
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=${1:?variant name}; shift
P=$R/omero-ms-image-region_amd
make -C $P -s -j8 || exit 1
T=$R/ab/build_$NAME; rm -rf $T; mkdir -p $T
FLAGS="-O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -I$R/include -I$P/csrc -Wall -Wno-unused-function -Wno-pass-failed"
pids=""
SRCS=$P/csrc/*.hip
[ -n "$AB_SOURCES" ] && SRCS=$(for n in $AB_SOURCES; do echo $P/csrc/$n.hip; done)
for s in $SRCS; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 $FLAGS "$@" -c -x hip $s -o $T/$(basename $s .hip).o &
    pids="$pids $!"
done
for p in $pids; do wait $p || exit 1; done
skip=$(for s in $SRCS; do basename $s .hip; done | paste -sd'|')
objs="$T/*.o $(ls $P/build/*.o | grep -v -E "^$P/build/($skip)\.o$")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/ab/libomr_$NAME.so $objs || exit 1
rm -rf $T
echo "ab/libomr_$NAME.so"
