"""GPU parity at the configured sizes (BASELINE.json configs), not just the
small cases of test_gpu_parity.py.

- C1 (Cornell box, 512x512, 64 spp: 16.8 M samples) whole frame: every
  per-sample record (Li, alpha, sample position, path depth) bit-identical to
  the oracle, and the ray / shadow-ray / path-length counters equal.
- C2 (Cornell box 1280x720, 512 spp), C3 (matpreview + envmap, 512 spp),
  C4 (atrium, 256 spp) and C5 (textured roughplastic, 1024 spp): a
  full-resolution row band at the configured spp,
  rendered by the full-frame launch geometry (window = whole rows).

Same bar as test_gpu_parity.py.  The oracle runs on the
box's CPU share (16 threads).
"""
import os

import numpy as np
import pytest

from mitsuba_amd import scenes

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _records_equal(smp_g, smp_o):
    assert smp_g.shape == smp_o.shape
    same = np.all(_bits(smp_g) == _bits(smp_o), axis=1)
    bad = np.nonzero(~same)[0]
    assert same.all(), 'per-sample mismatch at %d of %d records, first %s: %s vs %s' % (
        bad.size, same.size, bad[:3].tolist(), smp_g[bad[:3]].tolist(), smp_o[bad[:3]].tolist())


def test_c1_full_frame_bitexact(gpu_ctx, oracle):
    sc, it = scenes.build('C1')
    assert (sc.sensor.width, sc.sensor.height, it.sampleCount) == (512, 512, 64)
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0, threads=THREADS)
    assert st_g['samples'] == st_o['samples'] == 512 * 512 * 64
    _records_equal(smp_g, smp_o)
    for k in ('rays', 'shadow_rays', 'path_length_sum'):
        assert st_g[k] == st_o[k], k
    np.testing.assert_allclose(film_g, film_o, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('cfg,rows', [('C2', (352, 8)), ('C3', (356, 4)), ('C4', (300, 2)), ('C5', (360, 1))])
def test_full_resolution_row_band_bitexact(gpu_ctx, oracle, cfg, rows):
    sc, it = scenes.build(cfg)
    W = sc.sensor.width
    assert W == 1280 and sc.sensor.height == 720
    win = (0, rows[0], W, rows[1])
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, window=win, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, window=win, samples=True, libm_mode=0, threads=THREADS)
    assert st_g['samples'] == st_o['samples'] == W * rows[1] * it.sampleCount
    _records_equal(smp_g, smp_o)
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']


def test_c5_row_band_on_reference_table_layers(gpu_ctx, oracle, c5_reference_tables):
    """C5's configuration (1280 wide, 1024 spp, full envmap and blob) on the
    reference's own ggx.dat values at C5's eta (conftest.c5_reference_tables):
    the row band bit-exact against the oracle on the same table."""
    from mitsuba_amd import rtrans
    sc, it = scenes.build('C5')
    for b in sc.bsdfs:
        if b.type == 'roughplastic':
            b.rtransDir = c5_reference_tables
    rtrans._cache.clear()
    win = (0, 360, sc.sensor.width, 1)
    gpu_ctx.upload(sc)
    _, smp_g, st_g = gpu_ctx.render(it, window=win, samples=True)
    _, smp_o, st_o = oracle.render(sc, it, window=win, samples=True, libm_mode=0, threads=THREADS)
    rtrans._cache.clear()
    assert st_g['samples'] == st_o['samples'] == 1280 * 1024
    _records_equal(smp_g, smp_o)
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']


@pytest.mark.parametrize('cfg', ['C3', 'C4', 'C5'])
def test_bsdf_set_variant_equals_generic(gpu_ctx, cfg, monkeypatch):
    """C3-C5 render through a megakernel specialised to the scene's BSDF set
    (dbsdf.h BSet: GGX only, no roughdielectric / roughconductor); with
    MTSGPU_NO_BSDF_SETS=1 the generic all-BSDF variant runs.  Both give the same
    per-sample records bit for bit (the rows above check the specialised
    variant against the oracle)."""
    sc, it = scenes.build(cfg)
    win = (0, 200, sc.sensor.width, 2)
    gpu_ctx.upload(sc)
    _, smp_s, st_s = gpu_ctx.render(it, window=win, samples=True)
    assert gpu_ctx.debug_counters()[15] & (FEAT_GGX | FEAT_NORD | FEAT_NORC), 'no BSDF-set kernel ran'
    monkeypatch.setenv('MTSGPU_NO_BSDF_SETS', '1')
    _, smp_g, st_g = gpu_ctx.render(it, window=win, samples=True)
    _records_equal(smp_s, smp_g)
    assert st_s['rays'] == st_g['rays'] and st_s['shadow_rays'] == st_g['shadow_rays']


FEAT_ENV, FEAT_EXT, FEAT_GGX, FEAT_NORD, FEAT_NORC = 1, 2, 16, 32, 64   # csrc/layout.h MTSG_FEAT_*


def _beckmann_conductor_box():
    """The Cornell box with Beckmann rough conductors on the two blocks and area
    light only: no GGX, no roughdielectric -- none of the three benchmark sets."""
    from mitsuba_amd.scene import BSDF
    sc, it = scenes.build('C1', width=96, height=72, spp=8)
    sc.bsdfs.append(BSDF('roughconductor', distribution='beckmann', alpha=0.3, material='Al'))
    sc.bsdfs.append(BSDF('roughconductor', distribution='beckmann', alpha=0.12, material='Au'))
    sc.meshes[5].bsdf = len(sc.bsdfs) - 2
    sc.meshes[6].bsdf = len(sc.bsdfs) - 1
    return sc, it


def test_bsdf_set_beckmann_conductor_scene(gpu_ctx, oracle, monkeypatch):
    """every (feature set x BSDF set) combination has a
    specialised megakernel (path_f.hip), so a Beckmann roughconductor scene with
    an area light runs the NORD set (no GGX bit, roughconductors present): its
    records equal the generic kernel's and the oracle's bit for bit, and debug
    counter 15 shows which kernel ran."""
    monkeypatch.setenv('MTSGPU_NO_SCENE_LDS', '1')   # the sets serve large scenes (BVH in HBM)
    sc, it = _beckmann_conductor_box()
    gpu_ctx.upload(sc)
    _, smp_s, st_s = gpu_ctx.render(it, samples=True)
    ran = gpu_ctx.debug_counters()[15]
    assert ran & 0xff == FEAT_NORD, hex(ran)
    monkeypatch.setenv('MTSGPU_NO_BSDF_SETS', '1')
    _, smp_g, st_g = gpu_ctx.render(it, samples=True)
    assert gpu_ctx.debug_counters()[15] & 0xff == 0
    _records_equal(smp_s, smp_g)
    _, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0, threads=THREADS)
    _records_equal(smp_s, smp_o)
    assert st_s['rays'] == st_g['rays'] == st_o['rays']


def test_strict_normals_runs_generic_kernel_bitexact(gpu_ctx, oracle):
    """The BSDF-set megakernels are built without strictNormals (MTSG_FEAT_NOSTRICT,
    round 5): a large scene with strictNormals runs the generic kernel (counter 15
    shows no set bits) and stays bit-exact against the oracle, path and volpath
    (path.cpp:158-160, 196-197, 243-246; volpath.cpp:214-221)."""
    from mitsuba_amd.scene import VolpathIntegrator
    sc, it = scenes.build('C4')
    win = (0, 300, 320, 1)
    gpu_ctx.upload(sc)
    it.strictNormals = True
    for integ in (it, VolpathIntegrator(sampleCount=64, rfilter='box', strictNormals=True)):
        _, smp_g, st_g = gpu_ctx.render(integ, window=win, samples=True)
        assert gpu_ctx.debug_counters()[15] & (FEAT_GGX | FEAT_NORD | FEAT_NORC) == 0, 'a BSDF-set kernel ran'
        _, smp_o, st_o = oracle.render(sc, integ, window=win, samples=True, libm_mode=0, threads=THREADS)
        _records_equal(smp_g, smp_o)
        assert st_g['rays'] == st_o['rays'] and st_g['path_length_sum'] == st_o['path_length_sum']
    it.strictNormals = False
    _, smp_s, _ = gpu_ctx.render(it, window=win, samples=True)
    assert gpu_ctx.debug_counters()[15] & (FEAT_GGX | FEAT_NORD | FEAT_NORC), 'no BSDF-set kernel ran'
