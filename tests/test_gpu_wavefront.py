"""The wavefront engine (wf_shade + wf_trace, per-bounce ray queues) against the
CPU oracle and against the megakernel.

Both engines run the same PathShader code per bounce, so every per-sample
record (Li, alpha, position, depth, sampler flag) and every ray count must be
bit-identical to the oracle's whatever the engine; only the order in which
the slots pick up (sample, pixel) items differs.  The cases cover each kernel
variant the engine dispatches: linear-scan and LDS-BVH small scenes, HBM BVHs,
the environment emitters, EXT BSDFs, analytic shapes, volpath, the independent
sampler, and a render with more samples than path slots (slot regeneration
over several generations)."""
import os

import numpy as np
import pytest

from mitsuba_amd import scenes

pytestmark = pytest.mark.gpu

THREADS = min(32, os.cpu_count() or 1)


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _records_equal(a, b, what):
    assert a.shape == b.shape
    same = np.all(_bits(a) == _bits(b), axis=1)
    bad = np.nonzero(~same)[0]
    assert same.all(), '%s: per-sample mismatch at %d of %d records, first %s: %s vs %s' % (
        what, bad.size, same.size, bad[:3].tolist(), a[bad[:3]].tolist(), b[bad[:3]].tolist())


def _check(gpu_ctx, oracle, sc, it, what, window=None):
    gpu_ctx.upload(sc)
    film_w, smp_w, st_w = gpu_ctx.render(it, window=window, samples=True, engine='wavefront')
    film_m, smp_m, st_m = gpu_ctx.render(it, window=window, samples=True, engine='megakernel')
    film_o, smp_o, st_o = oracle.render(sc, it, window=window, samples=True, libm_mode=0, threads=THREADS)
    _records_equal(smp_w, smp_o, what + ' wavefront vs oracle')
    _records_equal(smp_m, smp_o, what + ' megakernel vs oracle')
    for k in ('samples', 'rays', 'shadow_rays', 'path_length_sum'):
        assert st_w[k] == st_o[k] == st_m[k], (what, k, st_w[k], st_m[k], st_o[k])
    # box: ordered own-pixel sums (+ rare neighbour splats); gaussian: the fixed gather order
    assert np.array_equal(_bits(film_w), _bits(film_o)), (what, np.argwhere(_bits(film_w) != _bits(film_o))[:4])
    return film_w, film_m


def _c3_small(**kw):
    return scenes.build('C3', width=kw.pop('width', 40), height=kw.pop('height', 24), spp=kw.pop('spp', 8),
                        env_size=kw.pop('env_size', (128, 64)), blob=kw.pop('blob', (48, 30)), **kw)


@pytest.mark.parametrize('materials', ['diffuse', 'rough', 'smooth', 'plastic', 'shapes'])
def test_wavefront_cornell_variants(gpu_ctx, oracle, materials):
    sc, it = scenes.build('C1', width=48, height=40, spp=8, materials=materials)
    film_w, film_m = _check(gpu_ctx, oracle, sc, it, materials)
    # box filter: own-pixel splats only, ordered reduction -> the films are identical too
    assert np.array_equal(_bits(film_w), _bits(film_m))


def test_wavefront_hbm_bvh_small_scene(gpu_ctx, oracle, monkeypatch):
    """The Cornell box with its BVH in HBM (no LDS staging): the global-memory traversal."""
    monkeypatch.setenv('MTSGPU_NO_SCENE_LDS', '1')
    sc, it = scenes.build('C1', width=40, height=32, spp=8, materials='rough')
    _check(gpu_ctx, oracle, sc, it, 'hbm-bvh')


def test_wavefront_lds_bvh_no_scan(gpu_ctx, oracle, monkeypatch):
    """SCENE_LDS with the BVH traversal instead of the linear scan (wf_trace stages the BVH)."""
    monkeypatch.setenv('MTSGPU_NO_SCAN', '1')
    sc, it = scenes.build('C1', width=40, height=32, spp=8)
    _check(gpu_ctx, oracle, sc, it, 'lds-bvh')


def test_wavefront_envmap_and_area(gpu_ctx, oracle):
    for kw, hide in (({}, False), ({'area_light': True, 'env_weight': 2.0}, False), ({}, True)):
        sc, it = _c3_small(**kw)
        it.hideEmitters = hide
        _check(gpu_ctx, oracle, sc, it, repr((kw, hide)))


def test_wavefront_atrium(gpu_ctx, oracle):
    sc, it = scenes.build('C4', width=48, height=27, spp=4)
    _check(gpu_ctx, oracle, sc, it, 'C4')


def test_wavefront_textured_roughplastic(gpu_ctx, oracle):
    sc, it = scenes.build('C5', width=48, height=27, spp=8, env_size=(128, 64), blob=(60, 38))
    _check(gpu_ctx, oracle, sc, it, 'C5')


def test_wavefront_volpath_independent_gaussian(gpu_ctx, oracle):
    from mitsuba_amd.scene import PathIntegrator, VolpathIntegrator
    sc, _ = _c3_small(area_light=True)
    _check(gpu_ctx, oracle, sc, VolpathIntegrator(sampleCount=8, rfilter='box', strictNormals=True), 'volpath')
    sc, _ = scenes.build('C1', width=40, height=32, spp=8, materials='shapes')
    _check(gpu_ctx, oracle, sc, PathIntegrator(sampleCount=8, rfilter='box', sampler='independent'), 'independent')
    sc, it = scenes.build('C1', width=96, height=80, spp=4)
    it.rfilter = 'gaussian'
    _check(gpu_ctx, oracle, sc, it, 'gaussian window', window=(17, 9, 40, 33))


def test_wavefront_slot_regeneration(gpu_ctx, oracle):
    """More (sample, pixel) items than path slots: every slot runs several paths,
    items come from all 8 pixel bands (band stealing at the end)."""
    sc, it = scenes.build('C1', width=160, height=120, spp=32, materials='rough')
    film_w, film_m = _check(gpu_ctx, oracle, sc, it, 'regeneration')
    assert np.array_equal(_bits(film_w), _bits(film_m))


def test_wavefront_row_shards_sum(gpu_ctx):
    sc, it = _c3_small(width=64, height=48, spp=4)
    gpu_ctx.upload(sc)
    full, _, _ = gpu_ctx.render(it, engine='wavefront')
    acc = np.zeros_like(full)
    for k in range(3):
        acc += gpu_ctx.render(it, row=(8, 3, k), engine='wavefront')[0]
    np.testing.assert_allclose(acc, full, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('case', ['shapes', 'C4', 'C5', 'kdtree'])
def test_wavefront_hit_records(gpu_ctx, oracle, monkeypatch, case):
    """MTSGPU_WF_HITREC=1: the trace kernel forms each closest hit's whole record
    (fill_hit: position, normals, shading frame, wi, UVs) and the shade kernels
    load it instead of re-deriving it from the primitive.  Analytic shapes, a
    large HBM-BVH scene, textures (UVs in the record) and the kd-tree trace."""
    monkeypatch.setenv('MTSGPU_WF_HITREC', '1')
    if case == 'shapes':
        sc, it = scenes.build('C1', width=48, height=40, spp=8, materials='shapes')
    elif case == 'C4':
        sc, it = scenes.build('C4', width=48, height=27, spp=4)
    elif case == 'C5':
        sc, it = scenes.build('C5', width=48, height=27, spp=8, env_size=(128, 64), blob=(60, 38))
    else:
        sc, it = scenes.build('C1', width=40, height=32, spp=8, materials='rough')
        gpu_ctx.upload(sc)
        _, smp_k, st_k = gpu_ctx.render(it, samples=True, engine='kdtree')
        monkeypatch.delenv('MTSGPU_WF_HITREC')
        _, smp_r, st_r = gpu_ctx.render(it, samples=True, engine='kdtree')
        _records_equal(smp_k, smp_r, 'kd-tree hit records vs kd-tree')
        assert st_k['rays'] == st_r['rays']
        return
    _check(gpu_ctx, oracle, sc, it, case + ' hit records')
