"""Multi-GPU decomposition of a frame: row blocks interleaved over ranks.

The reference renders a frame as 32x32 blocks handed to worker threads
(BlockedRenderProcess, src/librender/renderproc.cpp:40-149) and merges every
finished block into one film (Film::put).  Here one process drives one MI355X:
rank r renders the rows y with (y // row_block) % world == r -- neighbouring
rows cost about the same, so the interleave balances without a work queue --
into its own HBM film, and the films are summed onto rank 0 with one reduce
over RCCL/xGMI (or gloo in the CPU tests).  Pixels of different ranks never
overlap, so the sum is the reference's merge; the only shared pixels are the
filter-border splats, which the reference also accumulates by addition.
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
