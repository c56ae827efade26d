#!/bin/bash
# C5 K2 A/B over bucket counts (OMR_K2_BUCKETS, any multiple of 256 in 1024..2048): the c5 probe
# per count, two alternating passes, one JSON line each (checksums must agree).
#   tools/c5_ab_n.sh <out-dir> [counts...]
O=${1:?out}; shift; mkdir -p $O
NS=${*:-2048 1792 1536 1280}
for pass in 1 2; do
  for n in $NS; do
    OMR_K2_BUCKETS=$n timeout -k 10 120 python3 tools/c5_probe.py > $O/c5_n${n}_p$pass.json \
      || { echo "c5 probe failed n=$n"; exit 1; }
    echo "n=$n pass=$pass $(cat $O/c5_n${n}_p$pass.json)"
  done
done
