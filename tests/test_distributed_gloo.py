"""The N>1 decomposition on CPU (gloo), world sizes 2, 4 and 8: each rank
renders its 8x8 tiles (TileSharding, as bench.py does on the GPUs; RowSharding
at world size 2), the films are summed onto rank 0 with one reduce, and the
result equals the single-process frame (bit for bit with the box filter).  The
per-rank renderer here is the CPU oracle; on the GPUs bench.py calls the HIP
path with the same tile parameters and RCCL (the same imageproc.cpp:28-80
partition of the frame into independent blocks, merged by Film::put's sum)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pkgimport import mitsuba_amd  # noqa: E402  (spawned workers re-import this module)

mitsuba_amd()
from mitsuba_amd.distributed import RowSharding, TileSharding  # noqa: E402


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_row_sharding_partitions_rows():
    for h in (1, 7, 8, 9, 64, 720, 723):
        for world in (1, 2, 3, 4, 8):
            rows = [RowSharding(r, world, 8).rows(h) for r in range(world)]
            flat = sorted(sum(rows, []))
            assert flat == list(range(h)), (h, world)
    with pytest.raises(ValueError):
        RowSharding(2, 2)


def test_tile_sharding_partitions_tiles():
    for w, h in ((1, 1), (7, 9), (40, 36), (1280, 720), (1283, 723)):
        for world in (1, 2, 3, 4, 8):
            masks = [TileSharding(r, world).pixels(w, h) for r in range(world)]
            cover = np.sum(masks, axis=0)
            assert cover.shape == (h, w) and (cover == 1).all(), (w, h, world)
            # whole 8x8 tiles per rank
            for m in masks:
                blocks = m[:h // 8 * 8, :w // 8 * 8].reshape(h // 8, 8, w // 8, 8)
                assert (blocks.all(axis=(1, 3)) | ~blocks.any(axis=(1, 3))).all()
    # 1280x720 = 14400 tiles: equal shares at 1, 2, 4 and 8 ranks
    for world in (1, 2, 4, 8):
        counts = [TileSharding(r, world).pixels(1280, 720).sum() for r in range(world)]
        assert len(set(counts)) == 1
    with pytest.raises(ValueError):
        TileSharding(2, 2)


def _worker(rank, world, port, rfilter, out_path, tiles=True):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from mitsuba_amd import scenes
    import oracle.binding as ob
    sc, it = scenes.build('C1', width=40, height=36, spp=4, rfilter=rfilter)
    shard = TileSharding(rank, world) if tiles else RowSharding(rank, world, 8)
    film, _, st = ob.render(sc, it, row=shard.row_params(), tile_shard=shard.tile_shard)
    t = torch.from_numpy(film.reshape(-1).copy())
    n = torch.tensor([st['samples']], dtype=torch.float64)
    shard.reduce(t, dist)
    dist.all_reduce(n)
    if rank == 0:
        np.save(out_path, t.numpy().reshape(film.shape))
        assert int(n.item()) == 40 * 36 * 4
    dist.destroy_process_group()


@pytest.mark.parametrize('world,rfilter,tiles', [(2, 'box', False), (2, 'gaussian', False), (2, 'box', True),
                                                 (2, 'gaussian', True), (4, 'box', True), (8, 'box', True),
                                                 (8, 'gaussian', True)])
def test_sharded_frame_equals_single_process(tmp_path, world, rfilter, tiles, oracle):
    from mitsuba_amd import scenes
    out = str(tmp_path / 'film.npy')
    mp.spawn(_worker, args=(world, _port(), rfilter, out, tiles), nprocs=world, join=True)
    sharded = np.load(out)
    sc, it = scenes.build('C1', width=40, height=36, spp=4, rfilter=rfilter)
    full, _, _ = oracle.render(sc, it)
    if rfilter == 'box':
        # box splats never leave their pixel with non-zero weight: the merge is exact
        np.testing.assert_array_equal(sharded.view(np.uint32), full.view(np.uint32))
    else:
        # gaussian border splats from both ranks are summed in another order
        np.testing.assert_allclose(sharded, full, rtol=2e-6, atol=1e-7)
