#!/bin/bash
# C5 K2 A/B on the GPU box: the c5 probe under each (bucket count, chunks per lane) setting, two
# alternating passes, one JSON line each (checksums must agree).  tools/gpu.sh py= cannot set env
# per run, hence this script.   tools/c5_ab.sh <out-dir>
O=${1:?out}; mkdir -p $O
for pass in 1 2; do
  for lg in ${LGS:-11 10}; do
    for cpt in ${CPTS:--2 -1}; do
      OMR_K2_BUCKETS_LG=$lg OMR_K2_EVAL_CPT=$cpt timeout -k 10 120 python3 tools/c5_probe.py > $O/c5_lg${lg}_cpt${cpt}_p$pass.json \
        || { echo "c5 probe failed lg=$lg cpt=$cpt"; exit 1; }
      echo "lg=$lg cpt=$cpt pass=$pass $(cat $O/c5_lg${lg}_cpt${cpt}_p$pass.json)"
    done
  done
done
