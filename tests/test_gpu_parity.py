"""GPU parity: libmtsgpu.so (HIP, gfx950) vs the CPU oracle on identical Sobol
sample sequences.

Bar: per-sample Li (RGB), alpha, sample position and path
depth bit-identical to the oracle run with glibc's transcendentals
(libm_mode=0, as the reference calls them; the device computes glibc's
algorithms, csrc/glibc_f32.h); the film bit-identical except pixels that
received spill splats (|u| within 1e-5 of a pixel edge), which match to 1e-6
relative (float atomics change the summation order).
"""
import numpy as np
import pytest

from mitsuba_amd import scenes

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _assert_records_equal(smp_g, smp_o, what=''):
    """Every per-sample record (Li, alpha, position, depth, flags) bit-identical."""
    assert smp_g.shape == smp_o.shape
    same = np.all(_bits(smp_g) == _bits(smp_o), axis=1)
    bad = np.nonzero(~same)[0]
    assert same.all(), '%s: per-sample mismatch at %d of %d records, first %s: %s vs %s' % (
        what, bad.size, same.size, bad[:3].tolist(), smp_g[bad[:3]].tolist(), smp_o[bad[:3]].tolist())


def _compare(film_g, smp_g, film_o, smp_o):
    _assert_records_equal(smp_g, smp_o)
    np.testing.assert_allclose(film_g, film_o, rtol=1e-6, atol=1e-7)
    frac = np.mean(_bits(film_g) == _bits(film_o))
    assert frac > 0.999, frac


def test_cornell_small_bitexact(gpu_ctx, oracle):
    sc, it = scenes.build('C1', width=64, height=48, spp=8)
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0)
    _compare(film_g, smp_g, film_o, smp_o)
    assert st_g['samples'] == st_o['samples'] == 64 * 48 * 8
    assert st_g['rays'] == st_o['rays']
    assert st_g['shadow_rays'] == st_o['shadow_rays']
    assert st_g['path_length_sum'] == st_o['path_length_sum']


def test_cornell_window_and_gaussian(gpu_ctx, oracle):
    sc, it = scenes.build('C1', width=96, height=80, spp=4)
    it.rfilter = 'gaussian'
    gpu_ctx.upload(sc)
    win = (17, 9, 40, 33)
    film_g, smp_g, _ = gpu_ctx.render(it, window=win, samples=True)
    film_o, smp_o, _ = oracle.render(sc, it, window=win, samples=True, libm_mode=0)
    assert np.all(_bits(smp_g) == _bits(smp_o))
    # gather mode (film_gather): the gaussian film's sums in one fixed order, bit-exact
    assert np.array_equal(_bits(film_g), _bits(film_o)), np.argwhere(_bits(film_g) != _bits(film_o))[:4]


def test_row_interleave_sums_to_full(gpu_ctx):
    sc, it = scenes.build('C1', width=64, height=64, spp=4)
    gpu_ctx.upload(sc)
    full, _, _ = gpu_ctx.render(it)
    parts = [gpu_ctx.render(it, row=(8, 4, k))[0] for k in range(4)]
    acc = np.zeros_like(full)
    for p in parts:
        acc += p
    np.testing.assert_allclose(acc, full, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('world', [3, 8])
def test_tile_shards_bitexact_and_sum_to_full(gpu_ctx, oracle, world):
    """MTSGPU_FLAG_TILE_SHARD (the multi-GPU bench's decomposition): each shard's
    per-sample records equal the oracle's for the same tiles, the shards cover
    every sample once, and the box-filter films sum to the full frame bit for bit
    (a 67x45 window: partial tiles at the right and bottom edges)."""
    sc, it = scenes.build('C1', width=80, height=56, spp=4)
    gpu_ctx.upload(sc)
    win = (5, 3, 67, 45)
    full, smp_full, _ = gpu_ctx.render(it, window=win, samples=True)
    acc = np.zeros_like(full)
    seen = np.zeros(smp_full.shape[0], bool)
    for k in range(world):
        f, smp, st = gpu_ctx.render(it, window=win, samples=True, row=(8, world, k), tile_shard=True)
        fo, smpo, _ = oracle.render(sc, it, window=win, samples=True, row=(8, world, k), tile_shard=True)
        assert np.all(_bits(smp) == _bits(smpo))
        mine = np.any(smp != 0, axis=1)
        assert not (seen & mine).any()
        seen |= mine
        acc += f
    assert seen.sum() == np.any(smp_full != 0, axis=1).sum()
    np.testing.assert_array_equal(acc.view(np.uint32), full.view(np.uint32))


def test_rough_bsdfs_bitexact(gpu_ctx, oracle):
    """roughconductor (GGX/Beckmann/Phong, visible and all-normal sampling) and
    roughdielectric (incl. the extra lobe-choice sample) on the Cornell blocks."""
    sc, it = scenes.build('C1', width=48, height=40, spp=16, materials='rough')
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0)
    _compare(film_g, smp_g, film_o, smp_o)
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']


def test_rough_bsdfs_all_materials(gpu_ctx, oracle):
    """Every entry of rough_materials() on the tall block, one render each."""
    from mitsuba_amd.scenes import rough_materials
    for mi in range(len(rough_materials())):
        sc, it = scenes.build('C1', width=24, height=24, spp=8, materials='rough')
        sc.meshes[6].bsdf = 3 + mi
        gpu_ctx.upload(sc)
        film_g, smp_g, _ = gpu_ctx.render(it, samples=True)
        film_o, smp_o, _ = oracle.render(sc, it, samples=True, libm_mode=0)
        _assert_records_equal(smp_g, smp_o, repr(mi))


def _c3_small(**kw):
    sc, it = scenes.build('C3', width=kw.pop('width', 40), height=kw.pop('height', 24), spp=kw.pop('spp', 8),
                          env_size=kw.pop('env_size', (128, 64)), blob=kw.pop('blob', (48, 30)), **kw)
    return sc, it


def test_envmap_bitexact(gpu_ctx, oracle):
    """envmap emitter: EWA-filtered camera misses, bilinear BSDF-sampled misses
    with MIS, importance-sampled NEE through the bounding sphere."""
    sc, it = _c3_small()
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0)
    _compare(film_g, smp_g, film_o, smp_o)
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']


def test_envmap_variants(gpu_ctx, oracle):
    """envmap + area light (emitter PDF over both), odd-sized pyramid, hideEmitters."""
    for kw, hide in (({'area_light': True, 'env_weight': 2.0}, False), ({'env_size': (100, 37)}, False),
                     ({}, True)):
        sc, it = _c3_small(**kw)
        it.hideEmitters = hide
        gpu_ctx.upload(sc)
        film_g, smp_g, _ = gpu_ctx.render(it, samples=True)
        film_o, smp_o, _ = oracle.render(sc, it, samples=True, libm_mode=0)
        _assert_records_equal(smp_g, smp_o, repr((kw, hide)))


def test_atrium_bitexact(gpu_ctx, oracle):
    """C4 at small size: ~195k triangles in HBM (no LDS staging), roughdielectric columns,
    four area lights -- the global-memory traversal path."""
    sc, it = scenes.build('C4', width=48, height=27, spp=4)
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0, threads=8)
    _compare(film_g, smp_g, film_o, smp_o)
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']


def test_xml_scene_bitexact(gpu_ctx, oracle, tmp_path):
    """A scene written to Mitsuba XML (+PLY/PFM) and loaded back renders on the
    GPU bit-identically to the oracle."""
    from mitsuba_amd.xmlscene import load_scene, save_scene
    sc, it = scenes.build('C3', width=32, height=18, spp=4, env_size=(64, 32), blob=(24, 16), area_light=True)
    sc2, it2 = load_scene(save_scene(sc, it, str(tmp_path)))
    gpu_ctx.upload(sc2)
    film_g, smp_g, _ = gpu_ctx.render(it2, samples=True)
    film_o, smp_o, _ = oracle.render(sc2, it2, samples=True, libm_mode=0)
    _compare(film_g, smp_g, film_o, smp_o)


def test_roughplastic_and_textures_bitexact(gpu_ctx, oracle):
    """roughplastic (GGX / Beckmann / Phong, nonlinear, visible and all-normal
    sampling) with the rough-transmittance slices, checkerboard-textured roughness
    (2D alpha x theta slice), textured diffuse and textured roughconductor."""
    sc, it = scenes.build('C1', width=48, height=40, spp=16, materials='plastic')
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0)
    _compare(film_g, smp_g, film_o, smp_o)
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']


def test_c5_textured_roughplastic_bitexact(gpu_ctx, oracle):
    """C5 at small size: the matpreview object in roughplastic GGX with a
    checkerboard roughness over spherical UVs, under the environment map."""
    sc, it = scenes.build('C5', width=48, height=27, spp=8, env_size=(128, 64), blob=(60, 38))
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0)
    _compare(film_g, smp_g, film_o, smp_o)


def test_c5_reference_table_layers_bitexact(gpu_ctx, oracle, c5_reference_tables):
    """C5 on the reference's own rough-transmittance values: ggx.dat with the eta
    layers C5's roughplastic reads taken from data/microfacet/ggx.dat
    (tests/golden/rtrans_c5_ggx_layers.npz; the host test
    test_c5_layer_fixture_equals_reference_file shows the oracle renders it as it
    renders the full reference file).  GPU = oracle bit for bit, and the records
    differ from the generated table's: the values reached the device."""
    from mitsuba_amd import rtrans
    recs = []
    for d in (c5_reference_tables, rtrans.GENERATED_DIR):
        sc, it = scenes.build('C5', width=48, height=27, spp=8, env_size=(128, 64), blob=(60, 38))
        for b in sc.bsdfs:
            if b.type == 'roughplastic':
                b.rtransDir = d
        rtrans._cache.clear()
        gpu_ctx.upload(sc)
        film_g, smp_g, _ = gpu_ctx.render(it, samples=True)
        recs.append(_bits(smp_g))
        if d == c5_reference_tables:
            film_o, smp_o, _ = oracle.render(sc, it, samples=True, libm_mode=0)
            _compare(film_g, smp_g, film_o, smp_o)
    rtrans._cache.clear()
    assert not np.array_equal(recs[0], recs[1])


def test_smooth_bsdfs_bitexact(gpu_ctx, oracle):
    """Delta BSDFs (conductor, dielectric, plastic with textured nonlinear base) and
    twosided (one nested BSDF; two nested with the back side in view): no NEE on
    purely specular vertices, MIS weight 1 after delta bounces, eta tracking."""
    sc, it = scenes.build('C1', width=48, height=40, spp=16, materials='smooth')
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0)
    _compare(film_g, smp_g, film_o, smp_o)
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']


def test_smooth_bsdfs_all_materials(gpu_ctx, oracle):
    """Every entry of smooth_materials() on the tall block, one render each."""
    from mitsuba_amd.scenes import smooth_materials
    for mi in range(len(smooth_materials())):
        sc, it = scenes.build('C1', width=24, height=24, spp=8, materials='smooth')
        sc.meshes[6].bsdf = 3 + mi
        gpu_ctx.upload(sc)
        film_g, smp_g, _ = gpu_ctx.render(it, samples=True)
        film_o, smp_o, _ = oracle.render(sc, it, samples=True, libm_mode=0)
        _assert_records_equal(smp_g, smp_o, repr(mi))


def test_analytic_shapes_bitexact(gpu_ctx, oracle):
    """rectangle / disk / sphere shapes (exact intersection in double for spheres,
    plugin hit records and UVs), a rectangle area light, an emitting sphere
    (cone sampling and its solid-angle pdf), flipNormals with twosided."""
    sc, it = scenes.build('C1', width=48, height=48, spp=16, materials='shapes')
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0)
    _compare(film_g, smp_g, film_o, smp_o)
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']


def test_analytic_shapes_under_envmap(gpu_ctx, oracle):
    """The ENV | EXT | ANA kernel: spheres and a disk in the envmap scene."""
    from mitsuba_amd.scene import BSDF, Mesh
    from mitsuba_amd.transform import Transform
    sc, it = _c3_small()
    sc.bsdfs.append(BSDF('plastic', diffuseReflectance=(0.7, 0.2, 0.2)))
    b = len(sc.bsdfs) - 1
    sc.meshes.append(Mesh(shape='sphere', center=(1.6, 0.6, 0.4), radius=0.6, bsdf=b))
    sc.meshes.append(Mesh(shape='disk', toWorld=Transform().scale(0.8).rotate((1, 0, 0), -90).translate(-1.5, 0.01, 0.5),
                          bsdf=b))
    gpu_ctx.upload(sc)
    film_g, smp_g, _ = gpu_ctx.render(it, samples=True)
    film_o, smp_o, _ = oracle.render(sc, it, samples=True, libm_mode=0)
    _assert_records_equal(smp_g, smp_o)


def test_constant_emitter_bitexact(gpu_ctx, oracle):
    """constant.cpp: uniform environment on the scene's bounding sphere -- camera and
    BSDF-sampled misses, cosine-sampled NEE (uniform-sphere NEE where refN = 0:
    the roughdielectric sphere), its solid-angle pdf in MIS; with an area light."""
    from mitsuba_amd.scene import BSDF, Emitter, Mesh
    sc, it = _c3_small(area_light=True)
    sc.emitters[0] = Emitter('constant', radiance=(0.8, 0.9, 1.1), samplingWeight=1.5)
    sc.bsdfs.append(BSDF('roughdielectric', distribution='ggx', alpha=0.2, intIOR=1.5))
    sc.meshes.append(Mesh(shape='sphere', center=(-1.6, 0.7, 0.3), radius=0.7, bsdf=len(sc.bsdfs) - 1))
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0)
    _compare(film_g, smp_g, film_o, smp_o)
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']


@pytest.mark.parametrize('counts', [(1, 1), (4, 2), (2, 3)])
def test_direct_integrator_bitexact(gpu_ctx, oracle, counts):
    """direct.cpp on the GPU: emitter and BSDF samples per shading point, the
    sampler's 2D arrays for counts > 1, MIS fractions and weights."""
    from mitsuba_amd.scene import DirectIntegrator
    sc, _ = scenes.build('C1', width=40, height=32, spp=8, materials='smooth')
    d = DirectIntegrator(sampleCount=8, rfilter='box', emitterSamples=counts[0], bsdfSamples=counts[1])
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(d, samples=True)
    film_o, smp_o, st_o = oracle.render(sc, d, samples=True, libm_mode=0)
    _compare(film_g, smp_g, film_o, smp_o)
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']


@pytest.mark.parametrize('materials', ['rough', 'shapes'])
def test_independent_sampler_bitexact(gpu_ctx, oracle, materials):
    """The independent sampler's per-(pixel, sample) streams: path (no dimension
    limit, RR) and direct with 2D sample arrays, bit-exact against the oracle."""
    from mitsuba_amd.scene import DirectIntegrator, PathIntegrator
    sc, _ = scenes.build('C1', width=40, height=32, spp=8, materials=materials)
    gpu_ctx.upload(sc)
    for it in (PathIntegrator(sampleCount=8, rfilter='box', sampler='independent'),
               DirectIntegrator(sampleCount=8, rfilter='box', sampler='independent', emitterSamples=3,
                                bsdfSamples=2)):
        film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
        film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0)
        _assert_records_equal(smp_g, smp_o)
        assert st_g['rays'] == st_o['rays']


def test_volpath_bitexact(gpu_ctx, oracle):
    """volpath without media: evalTransmittance shadow segments (shadow epsilon on
    every emitter, re-normalised env / sphere-light directions), strictNormals and
    path-length accounting, on the envmap scene and the analytic-shape box."""
    from mitsuba_amd.scene import VolpathIntegrator
    for sc, _ in (_c3_small(area_light=True), scenes.build('C1', width=32, height=32, spp=8, materials='shapes')):
        v = VolpathIntegrator(sampleCount=8, rfilter='box', strictNormals=True)
        gpu_ctx.upload(sc)
        film_g, smp_g, st_g = gpu_ctx.render(v, samples=True)
        film_o, smp_o, st_o = oracle.render(sc, v, samples=True, libm_mode=0)
        _assert_records_equal(smp_g, smp_o)
        assert st_g['path_length_sum'] == st_o['path_length_sum']


def test_direct_integrator_envmap_and_shapes(gpu_ctx, oracle):
    from mitsuba_amd.scene import DirectIntegrator
    for sc, _ in (_c3_small(area_light=True), scenes.build('C1', width=32, height=32, spp=4, materials='shapes')):
        d = DirectIntegrator(sampleCount=4, rfilter='box', emitterSamples=2, bsdfSamples=2)
        gpu_ctx.upload(sc)
        film_g, smp_g, _ = gpu_ctx.render(d, samples=True)
        film_o, smp_o, _ = oracle.render(sc, d, samples=True, libm_mode=0)
        _assert_records_equal(smp_g, smp_o)


def _random_rays(sc, n, seed):
    rng = np.random.default_rng(seed)
    lo = np.min([m.positions.min(0) for m in sc.meshes if not m.analytic], 0)
    hi = np.max([m.positions.max(0) for m in sc.meshes if not m.analytic], 0)
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d


@pytest.mark.parametrize('cfg', ['C3', 'C4', 'shapes'])
def test_trace_rays_bitexact(gpu_ctx, oracle, cfg):
    """mtsgpu_trace_rays (Scene::rayIntersect / occlusion in batch) == the oracle's
    kd-tree-semantics query: same t, barycentrics (an analytic shape's object-space
    hit) and primitive, bit for bit."""
    sc, _ = scenes.build('C1', materials='shapes') if cfg == 'shapes' else scenes.build(cfg)
    gpu_ctx.upload(sc)
    o, d = _random_rays(sc, 100000, 5)
    for shadow, maxt in ((False, np.inf), (True, 3.0)):
        hg, _ = gpu_ctx.trace_rays(o, d, maxt=maxt, shadow=shadow)
        ho = oracle.trace_rays(sc, o, d, maxt=maxt, shadow=shadow)
        assert np.array_equal(_bits(hg), _bits(ho)), (cfg, shadow, np.argwhere(_bits(hg) != _bits(ho))[:5])
        assert 0.05 < np.mean(hg[:, 3].view(np.uint32) != 0xffffffff if not shadow else hg[:, 0] > 0) < 1.0


@pytest.mark.parametrize('env', [False, True])
def test_analytic_shapes_bsdf_set_kernels(gpu_ctx, oracle, monkeypatch, env):
    """the megakernel's shadow rays run the inlined any-hit traversal
    (traverse<ANY=true>, the code GVN-PRE miscompiled inside direct_kernel).
    Cross-check it where round 3 did not: the BSDF-set megakernels of large
    scenes (BVH in HBM) with analytic spheres, disks and rectangles, with and
    without an environment emitter -- every record against the oracle, and
    counter 15 shows that a set kernel with the ANA bit ran."""
    monkeypatch.setenv('MTSGPU_NO_SCENE_LDS', '1')
    if env:
        from mitsuba_amd.scene import BSDF, Mesh
        from mitsuba_amd.transform import Transform
        sc, it = _c3_small()
        sc.bsdfs.append(BSDF('diffuse', reflectance=(0.7, 0.2, 0.2)))
        b = len(sc.bsdfs) - 1
        sc.meshes.append(Mesh(shape='sphere', center=(1.6, 0.6, 0.4), radius=0.6, bsdf=b))
        sc.meshes.append(Mesh(shape='sphere', center=(-1.4, 0.5, 0.9), radius=0.5, bsdf=b))
        sc.meshes.append(Mesh(shape='disk', toWorld=Transform().scale(0.8).rotate((1, 0, 0), -90)
                              .translate(-1.5, 0.01, 0.5), bsdf=b))
    else:
        sc, it = scenes.build('C1', width=48, height=48, spp=16, materials='shapes')
    gpu_ctx.upload(sc)
    film_g, smp_g, st_g = gpu_ctx.render(it, samples=True)
    ran = gpu_ctx.debug_counters()[15]
    assert ran & 4 and ran & (16 | 32 | 64), hex(ran)      # MTSG_FEAT_ANA + a BSDF-set bit
    film_o, smp_o, st_o = oracle.render(sc, it, samples=True, libm_mode=0)
    _assert_records_equal(smp_g, smp_o)
    assert st_g['rays'] == st_o['rays'] and st_g['shadow_rays'] == st_o['shadow_rays']
