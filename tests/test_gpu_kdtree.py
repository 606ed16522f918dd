"""GPU traversal of the reference's SAH kd-tree (mtsgpu_trace_rays_ex with
MTSGPU_TRACE_KDTREE: the host builder of kdtree_build.cpp, the device
SAHKDTree3D::rayIntersectHavran with its mailbox) against the oracle's Havran
traversal of the same tree: every hit record {t, u, v, prim} bit-identical,
shadow queries identical; and the kd-tree's closest distances equal the BVH
path's (tests/test_kdtree.py for the CPU side)."""
import numpy as np
import pytest

from mitsuba_amd import scenes

from test_kdtree import _rays

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('cfg,kw', [('C1', dict(width=16, height=16, spp=1)),
                                    ('C3', dict(width=16, height=16, spp=1, env_size=(16, 8))),
                                    ('C4', dict(width=16, height=16, spp=1))])
def test_kdtree_trace_bitexact(gpu_ctx, oracle, cfg, kw):
    sc, _ = scenes.build(cfg, **kw)
    gpu_ctx.upload(sc)
    nodes, idx, info = gpu_ctx.kdtree()
    o, d = _rays(sc, 100000, 11)
    g, _ = gpu_ctx.trace_rays(o, d, kdtree=True)
    c = oracle.trace_rays_kd(sc, nodes, idx, o, d)
    same = np.all(g.view(np.uint32) == c.view(np.uint32), axis=1)
    assert same.all(), (np.nonzero(~same)[0][:5], g[~same][:3], c[~same][:3])
    b, _ = gpu_ctx.trace_rays(o, d)
    assert np.array_equal(g[:, 0].view(np.uint32), b[:, 0].view(np.uint32))
    gs, _ = gpu_ctx.trace_rays(o, d, maxt=1.5, shadow=True, kdtree=True)
    cs = oracle.trace_rays_kd(sc, nodes, idx, o, d, maxt=1.5, shadow=True)
    assert np.array_equal(gs[:, 0], cs[:, 0])


@pytest.mark.parametrize('cfg,kw', [('C1', dict(width=48, height=32, spp=4)),
                                    ('C4', dict(width=48, height=32, spp=2))])
def test_path_render_over_kdtree_bitexact(gpu_ctx, oracle, cfg, kw):
    """A whole path render with every ray traced through the reference's kd-tree
    (MTSGPU_FLAG_KDTREE) against the oracle render over the same tree: per-sample
    records bit-identical, ray counts equal."""
    sc, it = scenes.build(cfg, **kw)
    gpu_ctx.upload(sc)
    nodes, idx, _ = gpu_ctx.kdtree()
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True, engine='kdtree')
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0, kdtree=(nodes, idx))
    same = np.all(smp_g.view(np.uint32) == smp_o.view(np.uint32), axis=1)
    assert same.all(), (np.nonzero(~same)[0][:5], smp_g[~same][:2], smp_o[~same][:2])
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']
    np.testing.assert_allclose(film_g, film_o, rtol=1e-6, atol=1e-7)
