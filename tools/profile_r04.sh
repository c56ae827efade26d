#!/bin/bash
# Round-4 profile of every bench section (run from the repo root on the GPU box):
#  1. rocprofv3 --kernel-trace --stats over the full driver bench command (all sections, CPU legs
#     off): the per-(kernel, grid) launch table every section's roofline fraction is recomputed
#     from (tools/trace_kernels.py -> all_sections_kernels.csv) + the traced bench line;
#  2. FETCH_SIZE / WRITE_SIZE passes (one counter per pass) over the C3 projection (K3), the C5
#     threshold-mode K2 (k_render_pipe) and 256-tile C2 -> JPEG (B1, F1, B2a, B3, ...)
#     -> pmc_traffic_{c3,c5,jpeg}.json (tools/pmc_traffic.py).
# Raw per-dispatch CSVs are summarised and deleted on the box so gpurun_out/ stays small.
set -o pipefail
R=$PWD
O=$R/gpurun_out/${1:-r04prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_all -o all -- \
    python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/all_sections_traced_bench.json \
    2> $O/trace_all.err || exit $?
f=$(find $O/trace_all -name '*kernel_trace.csv' | head -1)
python3 $R/tools/trace_kernels.py $f $O/all_sections_kernels.csv || exit $?
find $O/trace_all -name '*kernel_stats.csv' -exec cp {} $O/all_sections_kernel_stats.csv \;
rm -rf $O/trace_all
echo TRACE ALL OK
for probe in c3 c5 jpeg; do
  case $probe in
    c3) cmd="python3 $R/tools/c3_probe.py"; rx="k_project" ;;
    c5) cmd="python3 $R/tools/c5_probe.py"; rx="k_render" ;;
    jpeg) cmd="python3 $R/tools/jpeg_probe.py"; rx="k_jpeg|k_render" ;;
  esac
  for c in FETCH_SIZE WRITE_SIZE; do
    C5_TILES=64 JPEG_PROBE_TILES=256 JPEG_PROBE_ITERS=2 timeout -s KILL 180 rocprofv3 --pmc $c \
        --kernel-include-regex "$rx" --output-format csv -d $O/pmc_${probe}_$c -o p -- $cmd \
        > /dev/null 2> $O/pmc_${probe}_$c.err || { echo "pmc $probe $c failed"; tail -5 $O/pmc_${probe}_$c.err; exit 1; }
    echo PMC $probe $c OK
  done
  python3 $R/tools/pmc_traffic.py $O/pmc_traffic_$probe.json $(find $O -path "*pmc_${probe}_*" -name '*counter_collection.csv') \
      > $O/pmc_traffic_$probe.txt || exit $?
  find $O -path "*pmc_${probe}_*" -name '*counter_collection.csv' -delete
done
du -sh $O
