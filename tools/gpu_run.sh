#!/bin/bash
# One GPU-box session: probes, bench, GPU tests.  Usage: tools/gpu_run.sh TAG [steps...]
# steps: info series bench bench2 tests (default: all).  Each GPU step has its own time limit;
# the first failing step ends the script.
set -o pipefail
TAG=${1:-run}; shift
STEPS=${*:-info series bench tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for s in $STEPS; do
  case $s in
    info)
      (grep -m1 "model name" /proc/cpuinfo; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null;
       grep -m1 -o -w avx512f /proc/cpuinfo; rocm-smi --showclocks 2>/dev/null | head -30) > $OUT/info.txt 2>&1 ;;
    series)
      OMR_K2_NT_STORE=1 timeout -k 10 180 python -u tools/k2_series.py > $OUT/k2_series_nt1.json 2> $OUT/k2_series_nt1.err || exit $?
      OMR_K2_NT_STORE=0 timeout -k 10 180 python -u tools/k2_series.py > $OUT/k2_series_nt0.json 2> $OUT/k2_series_nt0.err || exit $? ;;
    bench)
      timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $? ;;
    bench2)
      timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_g2.json 2> $OUT/bench_g2.err || exit $? ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || exit $? ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $? ;;
  esac
  echo "step $s done" 
done
