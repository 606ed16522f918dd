"""Multi-GPU decomposition of a frame: 8x8 pixel tiles (or row blocks)
interleaved over ranks.

The reference renders a frame as 32x32 blocks handed to worker threads
(BlockedRenderProcess, src/librender/renderproc.cpp:40-149) and merges every
finished block into one film (Film::put).  Here one process drives one MI355X:
rank r renders the rows y with (y // row_block) % world == r -- neighbouring
rows cost about the same, so the interleave balances without a work queue --
into its own HBM film, and the films are summed onto rank 0 with one reduce
over RCCL/xGMI (or gloo in the CPU tests).  Pixels of different ranks never
overlap, so the sum is the reference's merge; the only shared pixels are the
filter-border splats, which the reference also accumulates by addition.

TileSharding (the bench's decomposition) deals the window's 8x8 tiles
round-robin: rank r renders tiles t with t % world == r (row-major tile order,
MTSGPU_FLAG_TILE_SHARD), so each rank keeps whole tiles -- the unit whose 64
neighbouring pixels share a wave and BVH nodes in an XCD's L2 -- at any rank
count.  RowSharding keeps whole rows (row blocks of 8 down to 1 as the rank
count grows, which at 8 ranks leaves a rank's 8x8 work tiles spanning 2-row
strips 16 image rows apart).
"""
ROW_BLOCK = 8


def balanced_row_block(height, world, preferred=ROW_BLOCK):
    """The largest row block <= `preferred` (8, 4, 2, 1) whose block count divides
    evenly over the ranks, so that every rank renders the same number of rows
    (720 rows: 8 for 1-2 ranks, 4 for 4, 2 for 8); 1 when none does."""
    b = preferred
    while b > 1:
        if -(-height // b) % world == 0:
            return b
        b //= 2
    return 1


class RowSharding:
    tile_shard = False

    def __init__(self, rank=0, world=1, row_block=ROW_BLOCK):
        if world < 1 or not (0 <= rank < world) or row_block < 1:
            raise ValueError('bad sharding rank=%r world=%r row_block=%r' % (rank, world, row_block))
        self.rank, self.world, self.row_block = rank, world, row_block

    @classmethod
    def for_frame(cls, rank, world, height):
        return cls(rank, world, balanced_row_block(height, world))

    def row_params(self):
        """(row_block, row_stride, row_phase) of mtsgpu_render_params."""
        return (self.row_block, self.world, self.rank)

    def rows(self, height, y0=0):
        """Image rows of this rank inside a window starting at row y0."""
        return [y0 + r for r in range(height) if (r // self.row_block) % self.world == self.rank]

    def reduce(self, film, dist=None, dst=0):
        """Sum the ranks' films onto rank `dst` (in place on `film`, a torch tensor)."""
        if self.world > 1:
            if dist is None:
                import torch.distributed as dist
            dist.reduce(film, dst=dst, op=dist.ReduceOp.SUM)
        return film


class TileSharding:
    """Rank r renders the window's 8x8 tiles t with t % world == r (tiles in
    row-major order over the window, t = (y // 8) * ceil(width / 8) + x // 8)."""
    tile_shard = True

    def __init__(self, rank=0, world=1):
        if world < 1 or not (0 <= rank < world):
            raise ValueError('bad sharding rank=%r world=%r' % (rank, world))
        self.rank, self.world = rank, world
        self.row_block = 8

    @classmethod
    def for_frame(cls, rank, world, height=None):
        return cls(rank, world)

    def row_params(self):
        """(row_block, row_stride, row_phase) of mtsgpu_render_params (with MTSGPU_FLAG_TILE_SHARD)."""
        return (8, self.world, self.rank)

    def pixels(self, width, height):
        """Boolean (height, width) mask of this rank's pixels."""
        import numpy as np
        ty, tx = np.meshgrid(np.arange(height) // 8, np.arange(width) // 8, indexing='ij')
        return (ty * (-(-width // 8)) + tx) % self.world == self.rank

    reduce = RowSharding.reduce
