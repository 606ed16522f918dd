"""XML scene loading: the reference's scene format
(scenehandler.cpp semantics) into the same Scene the programmatic builders
make -- round trips are bit-identical through the oracle -- plus OBJ /
serialized / cube shapes, $parameters, refs, transforms and errors."""
import os
import textwrap

import numpy as np
import pytest

from mitsuba_amd import scenes
from mitsuba_amd.serialized import load_serialized, write_serialized
from mitsuba_amd.transform import Transform
from mitsuba_amd.xmlscene import SceneError, cube_mesh, load_scene, read_pfm, save_scene, write_pfm


@pytest.mark.parametrize('cfg,kw', [('C1', dict(width=40, height=30, spp=4)),
                                    ('C1', dict(width=24, height=24, spp=4, materials='rough')),
                                    ('C1', dict(width=24, height=24, spp=4, materials='smooth')),
                                    ('C1', dict(width=24, height=24, spp=4, materials='shapes')),
                                    ('C3', dict(width=32, height=18, spp=4, env_size=(64, 32), blob=(24, 16)))])
def test_round_trip_renders_identically(tmp_path, oracle, cfg, kw):
    sc, it = scenes.build(cfg, **kw)
    path = save_scene(sc, it, str(tmp_path))
    sc2, it2 = load_scene(path)
    f1, s1, _ = oracle.render(sc, it, samples=True, threads=4)
    f2, s2, _ = oracle.render(sc2, it2, samples=True, threads=4)
    np.testing.assert_array_equal(s1.view(np.uint32), s2.view(np.uint32))
    np.testing.assert_array_equal(f1.view(np.uint32), f2.view(np.uint32))


OBJ = """\
# a quad and a triangle in two groups, with normals, uvs, negative indices
mtllib m.mtl
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
vt 0 0
vt 1 0
vt 1 1
vt 0 1
vn 0 0 1
g quad
usemtl red
f 1/1/1 2/2/1 3/3/1 4/4/1
g tri
usemtl grey
f -4//-1 -3//-1 -2//-1
"""
MTL = """\
newmtl red
Kd 0.8 0.1 0.1
illum 1
newmtl grey
Kd 0.5 0.5 0.5
"""


def _write_scene(tmp, body, extra_files=()):
    for name, text in extra_files:
        open(os.path.join(tmp, name), 'w').write(text)
    path = os.path.join(tmp, 'scene.xml')
    open(path, 'w').write(textwrap.dedent(body))
    return path


SENSOR = """
  <integrator type="path"><integer name="maxDepth" value="$depth"/></integrator>
  <sensor type="perspective">
    <float name="fov" value="45"/>
    <transform name="toWorld"><lookat origin="0.5, 0.5, 3" target="0.5, 0.5, 0" up="0, 1, 0"/></transform>
    <sampler type="sobol"><integer name="sampleCount" value="4"/></sampler>
    <film type="hdrfilm"><integer name="width" value="16"/><integer name="height" value="12"/>
      <rfilter type="gaussian"/></film>
  </sensor>
"""


def test_obj_groups_materials_and_refs(tmp_path, oracle):
    body = """\
    <scene version="0.6.0">
      <default name="depth" value="3"/>
      %s
      <bsdf type="roughconductor" id="metal"><string name="distribution" value="ggx"/>
        <float name="alpha" value="0.2"/></bsdf>
      <shape type="obj"><string name="filename" value="m.obj"/>
        <ref name="grey" id="metal"/>
      </shape>
      <shape type="cube">
        <transform name="toWorld"><scale value="0.2"/><translate x="0.5" y="0.5" z="1"/></transform>
        <emitter type="area"><rgb name="radiance" value="5, 5, 4"/></emitter>
      </shape>
    </scene>""" % SENSOR
    path = _write_scene(str(tmp_path), body, [('m.obj', OBJ), ('m.mtl', MTL)])
    sc, it = load_scene(path)
    assert it.maxDepth == 3 and it.sampleCount == 4 and it.rfilter == 'gaussian'
    assert [m.name for m in sc.meshes][:2] == ['quad', 'tri']
    quad, tri, cube = sc.meshes
    assert quad.indices.tolist() == [[0, 1, 2], [0, 2, 3]]          # fan triangulation
    np.testing.assert_array_equal(quad.texcoords[2], [1, 0])         # v flipped (flipTexCoords)
    assert sc.bsdfs[quad.bsdf].type == 'diffuse'                      # from the MTL, sRGB -> linear
    np.testing.assert_allclose(sc.bsdfs[quad.bsdf].reflectance, (0.6038, 0.01002, 0.01002), rtol=1e-3)
    assert sc.bsdfs[tri.bsdf].type == 'roughconductor'               # <ref name="grey"> overrides the MTL
    assert cube.emitter == 0 and sc.emitters[0].radiance == (5.0, 5.0, 4.0)
    np.testing.assert_allclose(cube.positions.min(0), [0.3, 0.3, 0.8], atol=1e-6)
    film, _, st = oracle.render(sc, it)
    assert st['samples'] == 16 * 12 * 4 and np.isfinite(film).all()
    assert load_scene(path, depth=7)[1].maxDepth == 7                # $depth overridden


def test_serialized_round_trip(tmp_path):
    P = np.random.default_rng(1).random((10, 3)).astype(np.float32)
    I = np.array([[0, 1, 2], [3, 4, 5], [6, 7, 8]], np.uint32)
    N = np.tile(np.float32([0, 0, 1]), (10, 1))
    for version in (3, 4):
        fn = str(tmp_path / ('m%d.serialized' % version))
        write_serialized(fn, [('a', P, I, None, None), ('b', P[::-1].copy(), I, N, None)], version=version)
        m0 = load_serialized(fn, 0)
        m1 = load_serialized(fn, 1, toWorld=Transform().scale(-1, 1, 1))
        np.testing.assert_array_equal(m0.positions, P)
        assert m0.normals is None and m1.normals is not None
        np.testing.assert_array_equal(m1.indices, I[:, [1, 0, 2]])   # det < 0 swaps idx[0], idx[1]


def test_pfm_and_cube(tmp_path):
    img = np.random.default_rng(2).random((5, 7, 3)).astype(np.float32)
    write_pfm(str(tmp_path / 'e.pfm'), img)
    np.testing.assert_array_equal(read_pfm(str(tmp_path / 'e.pfm')), img)
    c = cube_mesh()
    assert c.positions.shape == (24, 3) and c.indices.shape == (12, 3)
    # every face is counter-clockwise around its outward normal
    for t in c.indices:
        p0, p1, p2 = c.positions[t]
        assert np.dot(np.cross(p1 - p0, p2 - p0), c.normals[t[0]]) > 0


def test_unsupported_plugins_raise(tmp_path):
    for shape in ('<shape type="cylinder"/>', '<shape type="hair"/>'):
        path = _write_scene(str(tmp_path), '<scene version="0.6.0">%s%s</scene>' % (SENSOR.replace('$depth', '2'), shape))
        with pytest.raises(NotImplementedError):
            load_scene(path)
    path = _write_scene(str(tmp_path), '<scene version="0.6.0">%s</scene>' % SENSOR)
    with pytest.raises(SceneError):
        load_scene(path)       # $depth has no value
