#!/bin/bash
# SQ counters of B1 (k_jpeg_fdct_batch), F1 (k_jpeg_render_fdct) and B3 (k_jpeg_huff_thread) on 64
# C2 tiles and 64 C1 tiles (tools/jpeg_probe.py): one --pmc pass per counter group (<= 8 SQ
# counters each), per case.  Summary text + jpeg_valu_pmc.json (bench.py's JPEG VALU roofline).
set -o pipefail
R=$PWD
O=$R/gpurun_out/${1:-jpeg_pmc_r02}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for case in ${JPEG_CASES:-c2 c1}; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FP64 SQ_INSTS_SMEM" \
             "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    JPEG_PROBE_CASE=$case timeout -s KILL 120 rocprofv3 --pmc $grp \
        --kernel-include-regex "k_jpeg_(fdct_batch|render_fdct|huff_thread)" \
        --output-format csv -d $O/$case/p$i -o p -- python3 $R/tools/jpeg_probe.py > /dev/null 2> $O/$case.p$i.err \
        || { echo "pass $case $i failed"; tail -5 $O/$case.p$i.err; exit 1; }
    echo PMC $case $i OK
  done
  # 64 tiles of 1024^2 -> 64 * 4096 MCUs (16x16 pixels, 4:2:0) per launch
  python3 $R/tools/pmc_kernels.py --json $O/jpeg_valu_pmc.json --case $case --mcus 262144 \
      $(find $O/$case -name '*counter_collection.csv') > $O/summary_$case.txt || exit $?
  find $O/$case -name '*counter_collection.csv' -delete
done
cat $O/summary_c2.txt
