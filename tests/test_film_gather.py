"""The gather-mode film (filters whose footprint covers neighbours: gaussian,
Mitsuba's default, film.cpp:89-95) on the CPU.

The oracle (oracle/mts_oracle.c film_gather) and the GPU (path_kernel.hip
film_gather<H>) form each film pixel's sum in one fixed order: for each sample
index j ascending, the source pixels of the (2H+1)^2 neighbourhood in row-major
order, each adding weight * value[k] with ImageBlock::put's footprint and
weights (imageblock.h:124-204: the block bitmap's clip, the discretised filter
of rfilter.cpp:37-55).  Here that order is restated independently in numpy from
the oracle's per-sample records and the oracle's film must equal it bit for bit.
"""
import numpy as np
import pytest

from mitsuba_amd import scenes
from mitsuba_amd.distributed import TileSharding

BLOCK = 32


def gather_ref(smp, spp, window, W, H, rfilter, param, ob, shard=None):
    """numpy restatement of the gather order; smp = the oracle's records of `window`."""
    radius, scale, b, values = ob.filter_table(rfilter, param)
    r32 = np.float32(radius)
    Hh = max(b, int(np.floor(np.float32(radius) + np.float32(0.5))))
    x0, y0, w, h = window
    fw, fh = W + 2 * b, H + 2 * b
    film = np.zeros((fh, fw, 5), np.float32)
    rec = smp.reshape(h, w, spp, 8)
    gy, gx = np.meshgrid(np.arange(max(0, y0 + b - Hh), min(fh, y0 + h + b + Hh)),
                         np.arange(max(0, x0 + b - Hh), min(fw, x0 + w + b + Hh)), indexing='ij')
    acc = np.zeros(gx.shape + (5,), np.float32)
    bw = BLOCK + 2 * b

    def disc(x):
        i = np.abs((x * scale).astype(np.float32)).astype(np.int64)
        return values[np.minimum(i, 31)]

    for j in range(spp):
        for dy in range(-Hh, Hh + 1):
            for dx in range(-Hh, Hh + 1):
                qx, qy = gx - b + dx, gy - b + dy
                lx, ly = qx - x0, qy - y0
                m = (lx >= 0) & (ly >= 0) & (lx < w) & (ly < h)
                if shard is not None:
                    m &= shard.pixels(w, h)[np.clip(ly, 0, h - 1), np.clip(lx, 0, w - 1)]
                r = rec[np.clip(ly, 0, h - 1), np.clip(lx, 0, w - 1), j]
                L = r[..., :3]
                m &= np.all(np.isfinite(L) & (L >= 0), axis=-1)
                sx, sy = r[..., 4].astype(np.float32), r[..., 5].astype(np.float32)
                bx, by = (np.maximum(qx, 0) // BLOCK) * BLOCK, (np.maximum(qy, 0) // BLOCK) * BLOCK
                posx = (sx - np.float32(0.5)) - (bx - b).astype(np.float32)
                posy = (sy - np.float32(0.5)) - (by - b).astype(np.float32)
                minx = np.maximum(np.ceil(posx - r32).astype(np.int64), 0)
                miny = np.maximum(np.ceil(posy - r32).astype(np.int64), 0)
                maxx = np.minimum(np.floor(posx + r32).astype(np.int64), bw - 1)
                maxy = np.minimum(np.floor(posy + r32).astype(np.int64), bw - 1)
                x, y = gx - bx, gy - by
                m &= (x >= minx) & (x <= maxx) & (y >= miny) & (y <= maxy)
                wgt = (disc(x.astype(np.float32) - posx) * disc(y.astype(np.float32) - posy)).astype(np.float32)
                val = np.concatenate([L, r[..., 3:4], np.ones_like(L[..., :1])], axis=-1).astype(np.float32)
                acc = np.where(m[..., None], acc + wgt[..., None] * val, acc)
    film[gy, gx] = acc
    return film


@pytest.mark.parametrize('window', [None, (17, 9, 40, 33)])
def test_oracle_gather_equals_numpy_order(oracle, window):
    sc, it = scenes.build('C1', width=96, height=80, spp=4, rfilter='gaussian')
    W, H = sc.sensor.width, sc.sensor.height
    win = window or (0, 0, W, H)
    film, smp, st = oracle.render(sc, it, window=win, samples=True, threads=8)
    assert st['samples'] == win[2] * win[3] * 4
    ref = gather_ref(smp, 4, win, W, H, 'gaussian', 0.5, oracle)
    bad = np.argwhere(np.any(film.view(np.uint32) != ref.view(np.uint32), axis=-1))
    assert bad.size == 0, (bad[:4].tolist(), film[tuple(bad[0])].tolist(), ref[tuple(bad[0])].tolist())
    assert np.count_nonzero(film[..., 4]) > win[2] * win[3]   # the footprints reach the border pixels


def test_oracle_gather_tile_shard_and_wide_filter(oracle):
    """A shard renders only its 8x8 tiles (sources outside them contribute nothing),
    and a wider gaussian (stddev 0.8: radius 3.2, H = 3) takes the same order."""
    sc, it = scenes.build('C1', width=48, height=40, spp=2, rfilter='gaussian')
    it.rfilterParam = 0.8
    W, H = sc.sensor.width, sc.sensor.height
    sh = TileSharding(1, 3)
    film, smp, _ = oracle.render(sc, it, samples=True, row=sh.row_params(), tile_shard=True, threads=8)
    ref = gather_ref(smp, 2, (0, 0, W, H), W, H, 'gaussian', 0.8, oracle, shard=sh)
    assert np.array_equal(film.view(np.uint32), ref.view(np.uint32))

