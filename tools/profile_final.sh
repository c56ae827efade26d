#!/bin/bash
# Round profile of the bench workload: kernel trace + stats of the full bench (every section),
# FETCH_SIZE / WRITE_SIZE PMC passes over the headline K2 launches only, then the default bench
# line.  Raw traces are summarised and dropped on the box so the merged gpurun_out/ stays small.
set -e
R=$PWD
O=$R/gpurun_out/final
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o k -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-latency > $O/bench_traced.json 2> $O/trace.err
find $O/trace -name '*kernel_trace.csv' -delete
echo TRACE OK
# headline only (the bench line's K2 launches, 256 C2 tiles each): its K2 average is the one the
# bench's HIP-event roofline must agree with
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_headline -o k -- python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-latency --no-jpeg --no-configs > $O/bench_headline_traced.json 2> $O/trace_headline.err
find $O/trace_headline -name '*kernel_trace.csv' -delete
echo TRACE HEADLINE OK
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_render" --output-format csv -d $O/pmc_$c -o p -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-latency --no-jpeg --no-configs > /dev/null 2> $O/pmc_$c.err
  echo PMC $c OK
done
python3 $R/tools/pmc_summary.py $O/pmc_render_c2.json "k_render<2, 8, true, false, 3, 4" 256 12582912 $(find $O -name '*counter_collection.csv')
find $O -name '*counter_collection.csv' -delete
cd $R
timeout -k 10 400 python3 bench.py > $O/bench_full.json 2> $O/bench_full.err
echo BENCH OK
du -sh $R/gpurun_out
