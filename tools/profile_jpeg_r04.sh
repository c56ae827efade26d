#!/bin/bash
# Round-4 JPEG SQ profile (run from the repo root on the GPU box), the r03 recipe on the current
# build: SQ counters of B1 / F1 / B2a / B3 (64 C2 and C1 tiles, one --pmc pass per counter group),
# including the f64 and transcendental VALU counts bench.py's issue-cycle roofline charges at their
# real cost -> summary_<case>.txt + jpeg_valu_pmc.json (bench.py VALU_PMC).
set -o pipefail
R=$PWD
O=$R/gpurun_out/${1:-jpeg_r04}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for case in c2 c1; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_VALU_CVT" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32"; do
    i=$((i+1))
    JPEG_PROBE_CASE=$case timeout -s KILL 120 rocprofv3 --pmc $grp \
        --kernel-include-regex "k_jpeg_(fdct_batch|render_fdct|block_bits|huff_thread)" \
        --output-format csv -d $O/$case/p$i -o p -- python3 $R/tools/jpeg_probe.py > /dev/null 2> $O/$case.p$i.err \
        || { echo "pass $case $i failed"; tail -5 $O/$case.p$i.err; exit 1; }
    echo PMC $case $i OK
  done
  python3 $R/tools/pmc_kernels.py --json $O/jpeg_valu_pmc.json --case $case --mcus 262144 \
      $(find $O/$case -name '*counter_collection.csv') > $O/summary_$case.txt || exit $?
  find $O/$case -name '*counter_collection.csv' -delete
done
cat $O/summary_c2.txt | grep -E "==|VALU/wave|WAIT|BANK|IDX"
echo JPEG PROFILE OK
