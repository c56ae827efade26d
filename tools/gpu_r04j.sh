#!/bin/bash
# Round-4 session j: SQ counters of the C2 -> JPEG kernels F1, B2a, B3 (256 tiles, one pass per
# counter group) -> summary (tools/pmc_kernels.py).
set -o pipefail
R=$PWD
O=$R/gpurun_out/r04j; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_VALU_CVT" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  JPEG_PROBE_TILES=256 JPEG_PROBE_ITERS=2 timeout -s KILL 150 rocprofv3 --pmc $grp \
      --kernel-include-regex "k_jpeg_(render_fdct|block_bits|huff_thread)" \
      --output-format csv -d $O/p$i -o p -- python3 $R/tools/jpeg_probe.py > /dev/null 2> $O/p$i.err \
      || { echo "pass $i failed"; tail -5 $O/p$i.err; exit 1; }
  echo PMC $i OK
done
python3 $R/tools/pmc_kernels.py $(find $O -name '*counter_collection.csv') > $O/summary_c2.txt || exit 1
find $O -name '*counter_collection.csv' -delete
cat $O/summary_c2.txt
echo R04J OK
