#!/bin/bash
# Round-4 final measurement on the committed build: the driver's bench command (N=1, defaults),
# then the all-sections rocprofv3 trace + FETCH/WRITE PMC passes (tools/profile_r04.sh).
set -o pipefail
O=gpurun_out/${1:-r04final}; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['ms_per_step'])"
timeout -k 10 1000 bash tools/profile_r04.sh ${1:-r04final}_prof || exit 1
echo R04FINAL OK
