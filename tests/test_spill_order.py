"""Box-filter neighbour splats (the spill film) sum in double on both sides
(dpath.h film_splat, oracle film_put), so a pixel's spill total does not depend
on the order its contributions land: float atomics made it schedule-dependent
once three or more samples splat into one pixel (one pixel of C3 at 1/4 rows
changed with the megakernel's sample-run length, profiles/r06_rounds/).

A box of radius 1 makes every sample splat into its neighbours, so most film
pixels receive many spills: the oracle's film must not change with its thread
count (dynamic OpenMP schedule), and the GPU's must equal it bit for bit.
Reference: ImageBlock::put (imageblock.h:124-204), rfilters/box.cpp."""
import numpy as np
import pytest

from mitsuba_amd import scenes


def _scene():
    sc, it = scenes.build('C1', width=48, height=40, spp=8)
    it.rfilterParam = 1.0
    return sc, it


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_oracle_spill_film_independent_of_threads(oracle):
    sc, it = _scene()
    f1, _, _ = oracle.render(sc, it, threads=1)
    f8, _, _ = oracle.render(sc, it, threads=8)
    assert f1.shape[0] == 40 + 2 and f1[1:-1, 1:-1, 4].min() > 0
    assert np.array_equal(_bits(f1), _bits(f8))


@pytest.mark.gpu
def test_gpu_wide_box_film_bitexact(gpu_ctx, oracle):
    sc, it = _scene()
    gpu_ctx.upload(sc)
    fg, _, _ = gpu_ctx.render(it)
    fo, _, _ = oracle.render(sc, it, threads=8)
    d = np.any(_bits(fg) != _bits(fo), axis=-1)
    assert not d.any(), '%d pixels differ, first %s' % (d.sum(), np.argwhere(d)[:3].tolist())
