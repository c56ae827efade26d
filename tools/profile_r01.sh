#!/bin/bash
# Round-1 profiling of the bench workload (C2 K2): kernel trace + stats, one PMC counter per
# pass, then the default bench line.  Raw CSVs are summarised and dropped on the box so the
# merged gpurun_out/ stays small.
set -e
R=$PWD
O=$R/gpurun_out/r01prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o k2 -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-latency > $O/bench_traced.json 2> $O/trace.err
find $O/trace -name '*kernel_trace.csv' -delete
echo TRACE OK
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o p -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-latency > /dev/null 2> $O/pmc_$c.err
  echo PMC $c OK
done
ls -R $O | head -40; python3 $R/tools/pmc_summary.py $O/pmc_render_c2.json "k_render<2, 8, true, false, 3, 4" 256 12582912 $(find $O -name '*counter_collection.csv')
find $O -name '*counter_collection.csv' -delete
cd $R
timeout -k 10 300 python3 bench.py > $O/bench_full.json 2> $O/bench_full.err
echo BENCH OK
cat $O/bench_full.json
du -sh $R/gpurun_out
