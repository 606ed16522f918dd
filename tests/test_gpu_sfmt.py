"""The SFMT replay samplers on the GPU.

* The device generator (gen_rand_all / nextULong in HBM, csrc/sfmt.h) reproduces
  the reference's SFMT19937 known-answer vector (src/tests/test_random.cpp:
  433-508) and the oracle's clone streams (Random(Random *) seeding on the host).
* 'independent-sfmt' (one worker over every block, `mitsuba -p 1`) and
  'independent-sfmt-blocks' (clone k renders spiral block k) render bit for bit
  what the oracle renders: every per-sample record and ray count."""
import json
import os

import numpy as np
import pytest

from mitsuba_amd import scenes
from mitsuba_amd.scene import PathIntegrator, VolpathIntegrator

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden', 'sfmt19937_kat.json')


def test_device_sfmt_known_answer(gpu_ctx):
    kat = json.load(open(GOLDEN))
    ref = np.array([int(v, 16) for v in kat['next_ulong']], np.uint64)
    assert np.array_equal(gpu_ctx.debug_sfmt(kat['seed'], ref.size), ref)


@pytest.mark.parametrize('clone', [1, 2, 7])
def test_device_sfmt_clones_match_oracle(gpu_ctx, oracle, clone):
    n = 1000   # three state refills
    assert np.array_equal(gpu_ctx.debug_sfmt(5489, n, clone=clone), oracle.sfmt_u64(5489, n, clone=clone))


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize('sampler', ['independent-sfmt', 'independent-sfmt-blocks'])
@pytest.mark.parametrize('case', ['diffuse', 'rough', 'shapes', 'envmap-volpath'])
def test_sfmt_replay_bitexact(gpu_ctx, oracle, sampler, case):
    if case == 'envmap-volpath':
        sc, _ = scenes.build('C3', width=40, height=24, spp=4, env_size=(128, 64), blob=(48, 30), area_light=True)
        it = VolpathIntegrator(sampleCount=4, rfilter='box', sampler=sampler)
    else:
        W, H = (72, 40) if sampler == 'independent-sfmt-blocks' else (40, 32)
        sc, _ = scenes.build('C1', width=W, height=H, spp=4, materials=case)
        it = PathIntegrator(sampleCount=4, rfilter='box', sampler=sampler)
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0, threads=8)
    same = np.all(_bits(smp_g) == _bits(smp_o), axis=1)
    bad = np.nonzero(~same)[0]
    assert same.all(), '%d of %d records differ, first %s: %s vs %s' % (
        bad.size, same.size, bad[:3].tolist(), smp_g[bad[:3]].tolist(), smp_o[bad[:3]].tolist())
    for k in ('samples', 'rays', 'shadow_rays', 'path_length_sum'):
        assert st_g[k] == st_o[k], k
    np.testing.assert_allclose(film_g, film_o, rtol=1e-6, atol=1e-7)


def test_sfmt_replay_rejects_row_shards(gpu_ctx):
    from mitsuba_amd.integrator import MtsgpuError
    sc, _ = scenes.build('C1', width=32, height=32, spp=2)
    gpu_ctx.upload(sc)
    it = PathIntegrator(sampleCount=2, rfilter='box', sampler='independent-sfmt')
    with pytest.raises(MtsgpuError):
        gpu_ctx.render(it, row=(8, 2, 0))
