#!/bin/bash
# Round-3 profiling of the bench workload on the GPU box (run from the repo root):
#  1. rocprofv3 --kernel-trace --stats of the headline bench command (C2 K2);
#  2. one PMC counter per pass (FETCH_SIZE, WRITE_SIZE) over the same launches -> traffic summary;
#  3. kernel trace + stats of the other sections (JPEG, PNG, C3, C5) without the CPU legs.
# Raw per-dispatch CSVs are summarised and deleted on the box so gpurun_out/ stays small.
set -o pipefail
R=$PWD
O=$R/gpurun_out/${1:-r03prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
HEAD="--steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-jpeg --no-configs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o k2 -- \
    python3 $R/bench.py $HEAD > $O/headline_traced_bench.json 2> $O/trace.err || exit $?
find $O/trace -name '*kernel_trace.csv' -delete
echo TRACE OK
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o p -- \
      python3 $R/bench.py --steps 4 --warmup 1 --prewarm-ms 100 --no-cpu-baseline --no-latency --no-jpeg --no-configs \
      > /dev/null 2> $O/pmc_$c.err || exit $?
  echo PMC $c OK
done
python3 $R/tools/pmc_summary.py $O/pmc_render_c2.json "k_render<2, 8, true, false, 3, 4" 256 12582912 \
    $(find $O -name '*counter_collection.csv') || exit $?
find $O -name '*counter_collection.csv' -delete
if [ "${2:-}" = "all" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_all -o all -- \
      python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/all_sections_traced_bench.json 2> $O/trace_all.err || exit $?
  find $O/trace_all -name '*kernel_trace.csv' -delete
  echo TRACE ALL OK
fi
du -sh $O
