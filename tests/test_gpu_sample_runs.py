"""Megakernel sample runs (dmega.h): a lane renders 2^s consecutive samples of one
pixel (s = MtsgLaunch::round_shift, chosen per chunk by capi.cpp run_shift, or
forced with MTSGPU_ROUND_SHIFT).  The work decomposition must not change a
single bit: every (pixel, sample) is rendered exactly once, whatever s, the
chunk's spp (13: not a multiple of 2^s; 3: fewer samples than a run) and the
film's padding pixels (a 44x28 window: partial 8x8 tiles).  Films, per-sample
records and counters are compared with the oracle (integrator.cpp:140-188,
path.cpp:119-294)."""
import os

import numpy as np
import pytest

from mitsuba_amd import scenes

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.fixture
def shift_env():
    saved = os.environ.get('MTSGPU_ROUND_SHIFT')
    yield
    if saved is None:
        os.environ.pop('MTSGPU_ROUND_SHIFT', None)
    else:
        os.environ['MTSGPU_ROUND_SHIFT'] = saved


@pytest.mark.parametrize('cfg', ['C1', 'C3'])
@pytest.mark.parametrize('spp', [13, 3])
def test_sample_runs_bitexact(gpu_ctx, oracle, shift_env, cfg, spp):
    sc, it = scenes.build(cfg, width=44, height=28, spp=spp)
    gpu_ctx.upload(sc)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0, threads=8)
    for s in (0, 1, 2, 4):
        os.environ['MTSGPU_ROUND_SHIFT'] = str(s)
        film_i, smp_i, st_i = gpu_ctx.render(it, samples=True)        # path_kernel<true, ...>
        film_u, _, st_u = gpu_ctx.render(it)                          # path_kernel<false, ...>
        same = np.all(_bits(smp_i) == _bits(smp_o), axis=1)
        assert same.all(), (s, int((~same).sum()))
        for name, f, st in (('instrumented', film_i, st_i), ('uninstrumented', film_u, st_u)):
            assert np.array_equal(_bits(f), _bits(film_o)), (s, name)
            for k in ('samples', 'rays', 'shadow_rays', 'path_length_sum'):
                assert st[k] == st_o[k], (s, name, k, st[k], st_o[k])
