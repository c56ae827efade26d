#!/bin/bash
# Round-4 session r: the multi-rank bench paths on one GPU (ranks share the device, gloo control):
# under torch.distributed.run as the driver launches it, and bench.py's own rank spawner.
set -o pipefail
O=gpurun_out/r04r; mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-jpeg --no-cpu-baseline --no-latency --no-configs \
    > $O/torchrun2.json 2> $O/torchrun2.err || { tail -20 $O/torchrun2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/torchrun2.json').read().strip().splitlines()[-1]); print('torchrun', d['n_gpus'], d['value'], d['config'].get('ranks'), d['config'].get('control_backend'), d['config'].get('ranks_share_devices'))"
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --no-jpeg --no-cpu-baseline --no-latency --no-configs \
    > $O/spawn2.json 2> $O/spawn2.err || { tail -20 $O/spawn2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/spawn2.json').read().strip().splitlines()[-1]); print('spawn', d['n_gpus'], d['value'], d['config'].get('ranks'), d['config'].get('control_backend'))"
echo R04R OK
