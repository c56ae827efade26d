"""Multi-process sharding of a tile batch: world_size 2 over gloo.

Each rank renders only its contiguous shard of the batch, with no collective on the data path;
the test then gathers per-tile digests (verification only) and checks that the union equals a
single-process render of the whole batch, with every tile rendered exactly once.  The CPU test
uses the CPU restatement as the per-rank renderer (no GPU here); the gpu-marked test runs the
same plan through libomr.so with both ranks on cuda:0.
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from omr.shard import ShardPlan, pyramid_tiles, render_shard, shard_range

N_TILES, W, H = 12, 48, 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    for n in (0, 1, 7, 4096):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[r][1] == spans[r + 1][0] for r in range(world - 1))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1
    assert shard_range(4096, 8, 3) == (1536, 2048)        # C4: 512 tiles per GPU
    assert len(pyramid_tiles(64, 64)) == 4096
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _tile_planes(i):
    from omr.synthetic import tile_u16, to_big_endian
    return [to_big_endian(p) for p in tile_u16(i, 4, H, W)]


def _digest(argb):
    return hashlib.sha256(np.ascontiguousarray(argb).tobytes()).hexdigest()


def _render_cpu(i):
    import oracle_lib
    from omr import _lib
    from omr.synthetic import c2_channels
    st, out = oracle_lib.render(c2_channels(4), _tile_planes(i), _lib.PIXELS_UINT16, W, H,
                                big_endian=True)
    assert st == 0
    return _digest(out)


def _render_gpu(ctx, i):
    import torch
    from omr import _lib
    from omr.context import make_qdef
    from omr.synthetic import c2_channels
    planes = [torch.from_numpy(np.ascontiguousarray(p).view(np.uint8).reshape(-1)).to("cuda:0")
              for p in _tile_planes(i)]
    out = torch.empty((H, W), dtype=torch.int32, device="cuda:0")
    ctx.render_packed_int_device(make_qdef("rgb"), c2_channels(4), planes, _lib.PIXELS_UINT16, W, H,
                                 out, big_endian=True)
    ctx.synchronize()
    return _digest(out.cpu().numpy().view(np.uint32))


def _worker(rank, world, port, out_dir, use_gpu):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.join(os.path.dirname(here), "omero-ms-image-region_amd"), here):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = ShardPlan.from_env(N_TILES)
    if use_gpu:
        import omr
        ctx = omr.Context(0)
        mine = render_shard(plan, lambda i: _render_gpu(ctx, i))
        ctx.close()
    else:
        mine = render_shard(plan, _render_cpu)
    gathered = [None] * world
    dist.all_gather_object(gathered, {"rank": rank, "tiles": mine})   # verification only
    if rank == 0:
        import json
        with open(os.path.join(out_dir, "gathered.json"), "w") as fh:
            json.dump(gathered, fh)
    dist.barrier()
    dist.destroy_process_group()


def _run(tmp_path, use_gpu):
    import json
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, str(tmp_path), use_gpu), nprocs=2, join=True,
                       start_method="spawn")
    gathered = json.load(open(tmp_path / "gathered.json"))
    seen = {}
    for g in gathered:
        lo, hi = shard_range(N_TILES, 2, g["rank"])
        assert sorted(int(k) for k in g["tiles"]) == list(range(lo, hi))
        for k, v in g["tiles"].items():
            assert int(k) not in seen
            seen[int(k)] = v
    assert sorted(seen) == list(range(N_TILES))
    return seen


def test_two_rank_gloo_shards_match_single_process(tmp_path):
    seen = _run(tmp_path, use_gpu=False)
    single = {i: _render_cpu(i) for i in range(N_TILES)}
    assert seen == single


@pytest.mark.gpu
def test_two_rank_gpu_shards_match_cpu_restatement(tmp_path):
    seen = _run(tmp_path, use_gpu=True)
    assert seen == {i: _render_cpu(i) for i in range(N_TILES)}
