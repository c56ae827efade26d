#!/bin/bash
# Round-4 session f: the C2 render -> JPEG pipeline per kernel (256 tiles, fused + unfused trace),
# a same-box A/B of the B4a / B6 grid sizing (OMR_JPEG_EST_CENTIBPP), then the bench without the
# JPEG leg (host-fed: PCIe probe, two copy queues).
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
R=$PWD
( cd /tmp && export TMPDIR=/tmp && JPEG_PROBE_TILES=256 JPEG_PROBE_ITERS=6 timeout -k 10 240 rocprofv3 --kernel-trace \
    --output-format csv -d $R/$O/jtrace -o j -- python3 $R/tools/jpeg_probe.py > $R/$O/jpeg_trace.log 2>&1 ) \
    || { tail $O/jpeg_trace.log; exit 1; }
f=$(find $O/jtrace -name '*kernel_trace.csv' | head -1)
python3 tools/trace_kernels.py $f $O/jpeg_c2_256_kernels.csv && rm -rf $O/jtrace
grep -E "jpeg|k_render|k_build" $O/jpeg_c2_256_kernels.csv | cut -c1-120
for i in 1 2; do
  for e in 100 50 40; do
    OMR_JPEG_EST_CENTIBPP=$e timeout -k 10 120 python3 tools/jpeg_rate.py > $O/rate_${e}_$i.json 2> $O/rate.err \
        || { tail $O/rate.err; exit 1; }
    echo "est $e run $i: $(cat $O/rate_${e}_$i.json | cut -c1-120)"
  done
done
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-jpeg --no-latency > $O/bench.json \
    2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); h=d['host_fed']; h.pop('serving'); print(json.dumps(h))"
echo R04F OK
