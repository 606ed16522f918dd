"""The tiny-scene linear scan (path_kernel.hip scan_pair / scan_tris: records
grouped by projection axis, a bounce's shadow and closest-hit rays tested in
one pass) on a scene built to stress it: the Cornell box plus an exact copy of
the short block's faces with another BSDF (every hit on the block is an
exact-t tie, which the larger primitive index must win) and a
degenerate triangle (TriAccel k = 3, never hit).  Still <= MTSG_SCAN_MAX
triangles, so the GPU renders it with the scan; the oracle traverses its BVH.
Per-sample records must be bit-identical."""
import numpy as np
import pytest

from mitsuba_amd import scenes
from mitsuba_amd.scene import BSDF, Mesh

pytestmark = pytest.mark.gpu


def _tie_scene(width, height, spp, dup_bsdf):
    sc, it = scenes.build('C1', width=width, height=height, spp=spp)
    short = sc.meshes[5]
    sc.bsdfs = list(sc.bsdfs) + [BSDF('diffuse', reflectance=(0.1, 0.3, 0.9))]
    dup = Mesh(short.positions.copy(), short.indices.copy(), bsdf=len(sc.bsdfs) - 1 if dup_bsdf else short.bsdf,
               faceNormals=True)
    p = np.array([[0.5, 0.5, 0.5], [1.0, 1.0, 1.0], [1.5, 1.5, 1.5]], np.float32)
    degen = Mesh(p, np.array([[0, 1, 2]], np.uint32), bsdf=0, faceNormals=True)
    sc.meshes = list(sc.meshes) + [dup, degen]
    return sc, it


def test_scan_ties_and_degenerate_bitexact(gpu_ctx, oracle):
    sc, it = _tie_scene(64, 48, 8, True)
    assert sc.num_triangles <= 64
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0)
    same = np.all(smp_g.view(np.uint32) == smp_o.view(np.uint32), axis=1)
    assert same.all(), (np.nonzero(~same)[0][:5], smp_g[~same][:2], smp_o[~same][:2])
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']
    np.testing.assert_allclose(film_g, film_o, rtol=1e-6, atol=1e-7)
    # the ties decide what is seen: with the copy's BSDF equal to the block's
    # the image changes, so the larger primitive (the copy) won them
    sc2, it2 = _tie_scene(64, 48, 8, False)
    gpu_ctx.upload(sc2)
    film_2, _, _ = gpu_ctx.render(it2, samples=True)
    assert not np.array_equal(film_g, film_2)
