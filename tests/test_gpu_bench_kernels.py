"""The kernels bench.py times, checked against the oracle.

Every per-sample parity test renders with records on, which launches the
instrumented instantiation path_kernel<INSTR=true, ...>.  bench.py renders
without records (`Context.render_device`, path_kernel<false, ...>): a separate
compile of the same source with its own register allocation.  Here that
instantiation is compared with the oracle directly:

- a row band of each benchmark configuration (C2-C5 at 1280x720 and their
  configured spp), rendered without records through the bench's decomposition
  (8x8 tiles, MTSGPU_FLAG_TILE_SHARD at world size 1): the box-filter film bit
  for bit against the oracle's film of the same band, and the sample / ray /
  shadow-ray / path-length counters equal;
- the whole frame rendered exactly as bench.py's timed step does
  (`render_device` into a torch film on torch's stream): its rows of the band
  equal the oracle's bit for bit (the oracle band carries one filter-border row
  above and below, so every splat those rows receive is rendered);
- debug counter 15 names the instantiation that ran; it must be the
  uninstrumented kernel the bench profiles name (profiles/*_bench_<cfg>_
  kernel_stats.csv), e.g. path_kernel<false, false, 336, 4> for C4;
- C1 (512x512, 64 spp) as a whole frame the same way.

Film order: film_reduce sums a pixel's own splats in sample order,
the reference's `*dest += weight * value[k]` sequence (imageblock.h:124-204),
and film_finalize adds the (rare, box radius 0.5 + 1e-5) neighbour splats.
Reference: integrator.cpp:140-188 (renderBlock), renderproc.cpp:142-149.
"""
import glob
import os

import numpy as np
import pytest

import bench
from mitsuba_amd import film_border
from mitsuba_amd.distributed import TileSharding

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)
BANDS = {'C2': (352, 16), 'C3': (356, 8), 'C4': (300, 4), 'C5': (360, 4), 'C2g': (360, 16)}
KERNELS = {'C1': 'path_kernel<false, true, 8, 4>', 'C2': 'path_kernel<false, true, 8, 4>',
           'C2g': 'path_kernel<false, true, 8, 4>',
           'C3': 'path_kernel<false, false, 817, 4>', 'C4': 'path_kernel<false, false, 336, 4>',
           'C5': 'path_kernel<false, false, 883, 4>'}
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _films_equal(fg, fo, what):
    diff = np.any(_bits(fg) != _bits(fo), axis=-1)
    bad = np.argwhere(diff)
    assert not diff.any(), '%s: %d of %d film pixels differ, first %s: %s vs %s' % (
        what, bad.shape[0], diff.size, bad[:3].tolist(), fg[tuple(bad[0])].tolist(), fo[tuple(bad[0])].tolist())


def _bench_frame(ctx, integ, H, W, b):
    """One timed step of bench.py at world size 1 (run_workload's step())."""
    import torch
    shard = TileSharding.for_frame(0, 1, H)
    film = torch.zeros(((H + 2 * b) * (W + 2 * b) * 5,), dtype=torch.float32, device='cuda')
    stream = torch.cuda.current_stream().cuda_stream
    st = ctx.render_device(integ, film.data_ptr(), stream, row=shard.row_params(), tile_shard=shard.tile_shard)
    torch.cuda.synchronize()
    return film.cpu().numpy().reshape(H + 2 * b, W + 2 * b, 5), st


def _profiled_kernel(cfg):
    """The dominant kernel of the newest committed bench kernel-stats profile of cfg."""
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_bench_%s_kernel_stats.csv' % cfg)))
    if not files:
        return None
    import csv
    rows = list(csv.DictReader(open(files[-1])))
    top = max(rows, key=lambda r: float(r['TotalDurationNs']))
    return top['Name'].replace('void ', '').replace('(MtsgLaunch)', '')


def _check_variant(ctx, cfg):
    v = ctx.kernel_variant()
    assert v is not None and not v['instr'], v
    assert v['name'] == KERNELS[cfg], (cfg, v)
    return v


def _reach(it):
    """The farthest film pixel a sample's splat reaches from its own: the band's margin."""
    b = film_border(it.rfilter, it.rfilterParam)
    r = np.float32(it.rfilterParam) + np.float32(1e-5) if it.rfilter == 'box' else np.float32(4) * np.float32(it.rfilterParam)
    return max(b, int(np.floor(r + np.float32(0.5))))


@pytest.mark.parametrize('cfg', ['C2', 'C3', 'C4', 'C5', 'C2g'])
def test_bench_kernel_row_band_bitexact(gpu_ctx, oracle, cfg):
    """C2g: C2 with Mitsuba's default gaussian filter (film.cpp:89-95), the film
    gathered in one fixed order (film_gather), bit-exact as the box films."""
    sc, it = bench.build_scene(cfg)
    W, H = sc.sensor.width, sc.sensor.height
    assert (W, H) == (1280, 720)
    b = film_border(it.rfilter, it.rfilterParam)
    y0, h = BANDS[cfg]
    m = _reach(it)
    win = (0, y0 - m, W, h + 2 * m)
    gpu_ctx.upload(sc)
    # the band through the uninstrumented kernel and the bench's tile decomposition
    film_g, smp, st_g = gpu_ctx.render(it, window=win, row=(8, 1, 0), tile_shard=True)
    assert smp is None
    _check_variant(gpu_ctx, cfg)
    film_o, _, st_o = oracle.render(sc, it, window=win, libm_mode=0, threads=THREADS)
    assert st_g['samples'] == st_o['samples'] == W * (h + 2 * m) * it.sampleCount
    for k in ('rays', 'shadow_rays', 'path_length_sum'):
        assert st_g[k] == st_o[k], (k, st_g[k], st_o[k])
    _films_equal(film_g, film_o, '%s band (uninstrumented kernel)' % cfg)
    # the bench's own call on the whole frame: the band's rows equal the oracle's
    film_f, st_f = _bench_frame(gpu_ctx, it, H, W, b)
    assert st_f['samples'] == W * H * it.sampleCount
    _check_variant(gpu_ctx, cfg)
    rows = slice(y0 + b, y0 + b + h)
    _films_equal(film_f[rows], film_o[rows], '%s whole frame, rows %d-%d' % (cfg, y0, y0 + h - 1))
    prof = _profiled_kernel(cfg)
    if prof is not None:
        assert prof == KERNELS[cfg], ('the committed bench profile timed another kernel', prof)


def test_bench_kernel_c1_full_frame_bitexact(gpu_ctx, oracle):
    sc, it = bench.build_scene('C1')
    W, H = sc.sensor.width, sc.sensor.height
    assert (W, H, it.sampleCount) == (512, 512, 64)
    b = film_border(it.rfilter, it.rfilterParam)
    gpu_ctx.upload(sc)
    film_g, _, st_g = gpu_ctx.render(it, row=(8, 1, 0), tile_shard=True)
    _check_variant(gpu_ctx, 'C1')
    film_o, _, st_o = oracle.render(sc, it, libm_mode=0, threads=THREADS)
    assert st_g['samples'] == st_o['samples'] == W * H * 64
    for k in ('rays', 'shadow_rays', 'path_length_sum'):
        assert st_g[k] == st_o[k], k
    _films_equal(film_g, film_o, 'C1 (uninstrumented kernel)')
    film_f, st_f = _bench_frame(gpu_ctx, it, H, W, b)
    _check_variant(gpu_ctx, 'C1')
    assert st_f['samples'] == W * H * 64
    _films_equal(film_f, film_o, 'C1 bench call')
