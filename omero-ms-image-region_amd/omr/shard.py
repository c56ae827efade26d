"""Multi-GPU sharding of tile batches.

The reference's only parallelism is request-level: N Vert.x worker instances, each rendering
whole requests (ImageRegionMicroserviceVerticle.java:84-85,149-165).  Tiles are independent, so
the MI355X node runs one process per GPU and hands each rank a contiguous shard of the tile
batch (C4: 4096 tiles of a 64x64-tile pyramid level over 8 GPUs).  There is no exchange step:
no collective touches pixel data.  Ranks only meet for timing barriers, and the node-level
"gather" is each rank answering its own requests.
"""


def shard_range(n_units, world, rank):
    """[lo, hi) of rank's contiguous shard; sizes differ by at most one (the first n % world
    ranks take one extra)."""
    if world <= 0 or not 0 <= rank < world or n_units < 0:
        raise ValueError(f"bad shard request: n={n_units} world={world} rank={rank}")
    base, extra = divmod(n_units, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def pyramid_tiles(grid_x, grid_y):
    """Tile coordinates of one pyramid level in row-major order (the `tile=res,x,y` requests a
    whole-slide viewer issues)."""
    return [(tx, ty) for ty in range(grid_y) for tx in range(grid_x)]


class ShardPlan:
    """Which tiles of a batch this rank renders."""

    def __init__(self, n_tiles, world, rank):
        self.n_tiles, self.world, self.rank = n_tiles, world, rank
        self.lo, self.hi = shard_range(n_tiles, world, rank)

    @property
    def count(self):
        return self.hi - self.lo

    def indices(self):
        return range(self.lo, self.hi)

    @classmethod
    def from_env(cls, n_tiles):
        import os
        return cls(n_tiles, int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")))


def render_shard(plan, render_tile):
    """Render this rank's tiles with render_tile(index) -> result; {index: result}.  Each rank
    runs this independently on its own GPU (no communication)."""
    return {i: render_tile(i) for i in plan.indices()}
