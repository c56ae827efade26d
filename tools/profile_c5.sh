#!/bin/bash
# SQ counters of the C5 K2 (threshold mode) kernel on 64 tiles (tools/c5_probe.py): one --pmc
# pass per counter group; summary in gpurun_out/<tag>/summary.txt.
set -o pipefail
R=$PWD
O=$R/gpurun_out/${1:-c5_pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FP64 SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  C5_TILES=64 timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_render" \
      --output-format csv -d $O/p$i -o p -- python3 $R/tools/c5_probe.py > /dev/null 2> $O/p$i.err \
      || { echo "pass $i failed"; tail -5 $O/p$i.err; exit 1; }
  echo PMC $i OK
done
python3 $R/tools/pmc_kernels.py $(find $O -name '*counter_collection.csv') > $O/summary.txt || exit $?
find $O -name '*counter_collection.csv' -delete
cat $O/summary.txt
