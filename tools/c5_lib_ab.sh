#!/bin/bash
# C5 K2: render GPU tests, then the in-tree libomr.so vs ab/libomr_old.so (OMR_LIB) inside the
# bench (prewarm + per-launch events), alternating.
set -o pipefail
O=gpurun_out/c5lib; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_render_gpu.py tests/test_semantics_gpu.py tests/test_render_sweep_gpu.py > $O/tests.log 2>&1 \
    || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export OMR_LIB=$PWD/ab/libomr_old.so; else unset OMR_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-jpeg --no-latency \
        > $O/b_$v$i.json 2> $O/b_$v$i.err || exit $?
    python3 -c "import json; d=json.loads(open('$O/b_$v$i.json').read().strip().splitlines()[-1])['c5_float']; print('$v run $i', d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
    python3 -c "import json; h=json.loads(open('$O/b_$v$i.json').read().strip().splitlines()[-1])['host_fed']; print('  host_fed', {k: h[k]['tiles_per_s'] for k in h if k.startswith('device_out') and isinstance(h[k], dict)}, h.get('device_out_vs_pcie_probe'))"
  done
done
