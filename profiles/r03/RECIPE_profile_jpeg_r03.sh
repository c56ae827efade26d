#!/bin/bash
# Round-3 JPEG profile (run from the repo root on the GPU box):
#  1. rocprofv3 --kernel-trace --stats of tools/jpeg_probe.py (64 C2 tiles, unfused + fused);
#  2. SQ counters of B1 / F1 / B3, one --pmc pass per group (<= 8 SQ counters), including the
#     f64 and transcendental VALU counts that bench.py's issue-cycle roofline charges at their
#     real cost.  Summary text + jpeg_valu_pmc.json.
set -o pipefail
R=$PWD
O=$R/gpurun_out/${1:-jpeg_r03}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
JPEG_PROBE_ITERS=10 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- \
    python3 $R/tools/jpeg_probe.py > $O/trace.log 2>&1 || exit $?
find $O/trace -name '*kernel_stats.csv' -exec cp {} $O/c2_kernel_stats.csv \;
f=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python3 $R/tools/trace_summary.py $f > $O/c2_trace_summary.txt || exit $?
rm -rf $O/trace
echo TRACE OK
for case in ${JPEG_CASES:-c2 c1}; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_VALU_CVT" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32"; do
    i=$((i+1))
    JPEG_PROBE_CASE=$case timeout -s KILL 120 rocprofv3 --pmc $grp \
        --kernel-include-regex "k_jpeg_(fdct_batch|render_fdct|huff_thread)" \
        --output-format csv -d $O/$case/p$i -o p -- python3 $R/tools/jpeg_probe.py > /dev/null 2> $O/$case.p$i.err \
        || { echo "pass $case $i failed"; tail -5 $O/$case.p$i.err; exit 1; }
    echo PMC $case $i OK
  done
  python3 $R/tools/pmc_kernels.py --json $O/jpeg_valu_pmc.json --case $case --mcus 262144 \
      $(find $O/$case -name '*counter_collection.csv') > $O/summary_$case.txt || exit $?
  find $O/$case -name '*counter_collection.csv' -delete
done
cat $O/summary_c2.txt
