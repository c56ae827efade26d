"""C2 at the bench's exact instantiation and C4 (BASELINE.json configs[1] and [3]) on the GPU.

* The headline launch: 256 strided big-endian 4-channel uint16 1024^2 tiles, C2 windows and
  colours, rgb model (bench.py `step`, omr_render_batch_strided_device) — every output tile
  compared with the CPU restatement, word for word.
* C4: a 4096-tile batch (a 64x64-tile pyramid level) sharded over 8 ranks by omr/shard.py, each
  shard rendered on cuda:{rank % device_count} through the same C ABI call, every tile
  compared with the CPU restatement; the shards cover the batch exactly once.
* `bench.py --gpus 2` starts two rank processes itself and reports the node-wide batch.

Tile t's planes are unique source tile src(t) (8 distinct microscopy tiles), so the oracle
renders 8 tiles and every GPU tile is checked against the expected tile of its source.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from omr import _lib
from omr.context import make_bindings, make_qdef
from omr.shard import ShardPlan
from omr.synthetic import c2_channels, torch_tiles_u16

TILE, C, U = 1024, 4, 8
PLANE = TILE * TILE * 2
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def c2_sources(oracle):
    import torch
    torch.manual_seed(20261015)
    native = torch_tiles_u16(U, C, TILE, TILE, "cuda:0")
    be = native.view(torch.uint8).view(U, C, TILE, TILE, 2).flip(-1).contiguous().view(torch.int16).view(
        U, C, TILE, TILE)
    host = be.cpu().numpy().view(np.uint16)
    tiles = [[np.ascontiguousarray(host[t, c]) for c in range(C)] for t in range(U)]
    _, exp = oracle.render_tiles_mt(c2_channels(C), tiles, U, _lib.PIXELS_UINT16, TILE, TILE, big_endian=True,
                                    n_threads=min(8, os.cpu_count() or 1))
    return be, torch.from_numpy(exp.view(np.int32)).to("cuda:0")


def _render_shard(ctx, be, exp, src_of, n, device):
    import torch
    data = torch.empty((n, C, TILE, TILE), dtype=torch.int16, device=device)
    be_d, exp_d = be.to(device), exp.to(device)
    for i in range(n):
        data[i].copy_(be_d[src_of(i)])
    out = torch.empty((n, TILE, TILE), dtype=torch.int32, device=device)
    out.fill_(0x55)
    status = torch.full((n,), -1, dtype=torch.int32, device=device)
    torch.cuda.synchronize(device)      # torch's stream -> the context's own stream
    chans = c2_channels(C)
    ctx.render_batch_strided_device(make_qdef("rgb"), chans, data, C * PLANE, PLANE, n, _lib.PIXELS_UINT16,
                                    TILE, TILE, out, status=status, big_endian=True, bindings=make_bindings(chans))
    ctx.synchronize()
    assert int(status.abs().sum()) == 0
    bad = [i for i in range(n) if not torch.equal(out[i], exp_d[src_of(i)])]
    return bad


@pytest.mark.gpu
def test_bench_headline_instantiation_bit_exact(ctx, c2_sources):
    """bench.py's timed launch (build_batch: tile t = source t % 8), 256 tiles, vs the oracle."""
    be, exp = c2_sources
    bad = _render_shard(ctx, be, exp, lambda i: i % U, 256, "cuda:0")
    assert not bad, f"{len(bad)} of 256 tiles differ from the CPU restatement (first {bad[:5]})"


@pytest.mark.gpu
def test_c4_4096_tiles_sharded_over_8_ranks(c2_sources):
    import omr
    import torch
    be, exp = c2_sources
    n_total, world = 4096, 8
    ndev = torch.cuda.device_count()
    covered = []
    ctxs = {}
    try:
        for rank in range(world):
            plan = ShardPlan(n_total, world, rank)
            dev = rank % ndev
            if dev not in ctxs:
                ctxs[dev] = omr.Context(dev)
            src_of = lambda i, lo=plan.lo: ((lo + i) * 5 + (lo + i) // 64) % U   # noqa: E731
            bad = _render_shard(ctxs[dev], be, exp, src_of, plan.count, f"cuda:{dev}")
            assert not bad, f"rank {rank}: {len(bad)} tiles differ (first {[plan.lo + b for b in bad[:5]]})"
            covered.extend(plan.indices())
            torch.cuda.empty_cache()
    finally:
        for c in ctxs.values():
            c.close()
    assert sorted(covered) == list(range(n_total))


@pytest.mark.gpu
def test_bench_gpus_2_spawns_two_ranks():
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--batch", "8", "--unique", "2", "--no-cpu-baseline", "--no-jpeg", "--no-configs", "--no-latency"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["config"]["tiles_per_node_per_step"] == 16
    assert d["config"]["ranks"] == 2
    assert d["value"] > 0 and d["roofline"]["launches"] == 3
