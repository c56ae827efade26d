#!/bin/bash
# SQ counters for the batched JPEG kernels (B1 k_jpeg_fdct_batch, B3 k_jpeg_huff_thread) over the
# bench's jpeg section: one --pmc pass per counter group, summarised per kernel.
set -e
R=$PWD
O=$R/gpurun_out/${1:-jpeg_pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_jpeg_(fdct_batch|huff_thread|block_bits|stuff)" --output-format csv -d $O/p$i -o p -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-latency --no-configs --jpeg-steps 2 > /dev/null 2> $O/p$i.err
  echo PMC $i OK
done
python3 $R/tools/pmc_kernels.py $(find $O -name '*counter_collection.csv') > $O/summary.txt
find $O -name '*counter_collection.csv' -delete
cat $O/summary.txt
