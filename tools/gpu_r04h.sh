#!/bin/bash
# Round-4 session h: host-fed copy modes alternated on one box (tools/hostfed_probe.py) at 64 and
# 256 tiles per call, then the PCIe probe.
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
for n in 64 256; do
  HOSTFED_TILES=$n timeout -k 10 240 python3 tools/hostfed_probe.py > $O/hostfed_$n.json 2> $O/hostfed.err \
      || { tail $O/hostfed.err; exit 1; }
  cat $O/hostfed_$n.json
done
timeout -k 10 120 ./tools/pcie_probe > $O/pcie_probe.json 2> $O/pcie_probe.err || { cat $O/pcie_probe.err; exit 1; }
cat $O/pcie_probe.json
echo R04H OK
