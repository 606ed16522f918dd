"""Host data formats and transforms: the PLY loader (src/shapes/ply.cpp) on
synthetic files in every body format, and Transform (core/transform.cpp)."""
import numpy as np
import pytest

from mitsuba_amd.ply import load_ply
from mitsuba_amd.transform import Transform

VERTS = np.array([(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0.5, 0.5, 1)], np.float32)
NRMS = np.array([(0, 0, 2), (0, 0, 1), (0, 0, 1), (0, 0, 1), (1, 1, 1)], np.float32)
UVS = np.array([(0, 0), (1, 0), (1, 1), (0, 1), (0.5, 0.5)], np.float32)
FACES = [(0, 1, 2, 3), (0, 1, 4), (1, 2, 4)]


def _write(path, fmt, normals=True, uv=True, index_type='int'):
    props = ['x', 'y', 'z'] + (['nx', 'ny', 'nz'] if normals else []) + (['u', 'v'] if uv else [])
    head = ['ply', 'format %s 1.0' % fmt, 'comment synthetic', 'element vertex %d' % len(VERTS)]
    head += ['property float %s' % p for p in props]
    head += ['element face %d' % len(FACES), 'property list uchar %s vertex_indices' % index_type, 'end_header']
    rows = [np.concatenate([VERTS[i]] + ([NRMS[i]] if normals else []) + ([UVS[i]] if uv else [])) for i in range(len(VERTS))]
    with open(path, 'wb') as f:
        f.write(('\n'.join(head) + '\n').encode())
        if fmt == 'ascii':
            for r in rows:
                f.write((' '.join('%r' % float(x) for x in r) + '\n').encode())
            for fc in FACES:
                f.write((' '.join(str(x) for x in (len(fc),) + fc) + '\n').encode())
        else:
            e = '<' if fmt == 'binary_little_endian' else '>'
            it = {'int': 'i4', 'uint': 'u4', 'int32': 'i4'}[index_type]
            for r in rows:
                f.write(np.asarray(r, e + 'f4').tobytes())
            for fc in FACES:
                f.write(np.uint8(len(fc)).tobytes() + np.asarray(fc, e + it).tobytes())


@pytest.mark.parametrize('fmt', ['ascii', 'binary_little_endian', 'binary_big_endian'])
def test_ply_formats(tmp_path, fmt):
    p = tmp_path / 'm.ply'
    _write(p, fmt)
    m = load_ply(str(p))
    np.testing.assert_array_equal(m.positions, VERTS)
    # quad (0,1,2,3) -> (0,1,2), (3,0,2) (ply.cpp:275-287)
    np.testing.assert_array_equal(m.indices, np.array([(0, 1, 2), (3, 0, 2), (0, 1, 4), (1, 2, 4)], np.uint32))
    np.testing.assert_allclose(np.linalg.norm(m.normals, axis=1), 1.0, rtol=1e-6)   # normalised on load
    np.testing.assert_array_equal(m.texcoords, UVS)


def test_ply_triangles_only_fast_path(tmp_path):
    global FACES
    saved = FACES
    FACES = [(0, 1, 4), (1, 2, 4), (2, 3, 4)]
    try:
        p = tmp_path / 't.ply'
        _write(p, 'binary_little_endian', normals=False, uv=False, index_type='uint')
        m = load_ply(str(p))
        np.testing.assert_array_equal(m.indices, np.array(FACES, np.uint32))
        assert m.normals is None and m.texcoords is None
    finally:
        FACES = saved


def test_ply_to_world(tmp_path):
    p = tmp_path / 'm.ply'
    _write(p, 'binary_little_endian')
    T = Transform().scale(2.0).translate(1, 2, 3)
    m = load_ply(str(p), toWorld=T)
    np.testing.assert_allclose(m.positions, VERTS * 2 + np.float32([1, 2, 3]), rtol=1e-6)


def test_ply_rejects_polygons(tmp_path):
    global FACES
    saved = FACES
    FACES = [(0, 1, 2, 3, 4)]
    try:
        p = tmp_path / 'bad.ply'
        _write(p, 'ascii')
        with pytest.raises(ValueError):
            load_ply(str(p))
    finally:
        FACES = saved


def test_transform_inverse_and_composition():
    T = Transform().scale(2, 3, 4).rotate((1, 2, 3), 37.0).translate(0.5, -1, 2)
    np.testing.assert_allclose(T.m.astype(np.float64) @ T.inv.astype(np.float64), np.eye(4), atol=1e-5)
    R = Transform.rotate_((0, 1, 0), 90.0)
    np.testing.assert_allclose(R.m @ R.inv, np.eye(4), atol=1e-6)
    np.testing.assert_allclose(R.apply_points(np.float32([[1, 0, 0]])), [[0, 0, -1]], atol=1e-6)
    L = Transform.look_at_((0, 0, -5), (0, 0, 0), (0, 1, 0))
    np.testing.assert_allclose(L.m.astype(np.float64) @ L.inv.astype(np.float64), np.eye(4), atol=1e-6)
    np.testing.assert_array_equal(L.m[:3, 3], np.float32([0, 0, -5]))
