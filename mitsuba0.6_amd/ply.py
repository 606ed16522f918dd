"""PLY shape loader: the host side of the reference's `ply` shape plugin.

Follows PLYLoader (src/shapes/ply.cpp:65-498): vertex x/y/z (+ nx/ny/nz,
u/v texture coordinates), triangle and quad faces (a quad (0,1,2,3) becomes
(0,1,2), (3,0,2)), `toWorld` applied to positions (Transform on points) and
normals (inverse transpose, then normalized), binary little/big endian and
ascii bodies.  Faces with another vertex count are an error, as in the
reference.  Returns a `Mesh`; normals left to TriMesh::computeNormals when the
file has none (faceNormals=False).
"""
import numpy as np

from .scene import Mesh
from .transform import Transform, normalize_rows

_TYPES = {'char': 'i1', 'int8': 'i1', 'uchar': 'u1', 'uint8': 'u1', 'short': 'i2', 'int16': 'i2',
          'ushort': 'u2', 'uint16': 'u2', 'int': 'i4', 'int32': 'i4', 'uint': 'u4', 'uint32': 'u4',
          'float': 'f4', 'float32': 'f4', 'double': 'f8', 'float64': 'f8'}
_U_NAMES = ('u', 's', 'texture_u', 'texture_s')
_V_NAMES = ('v', 't', 'texture_v', 'texture_t')


def _parse_header(f):
    if f.readline().strip() != b'ply':
        raise ValueError('not a PLY file')
    fmt, elements = None, []
    while True:
        line = f.readline()
        if not line:
            raise ValueError('unexpected end of PLY header')
        tok = line.decode('ascii', 'replace').split()
        if not tok or tok[0] in ('comment', 'obj_info'):
            continue
        if tok[0] == 'format':
            fmt = tok[1]
        elif tok[0] == 'element':
            elements.append({'name': tok[1], 'count': int(tok[2]), 'props': []})
        elif tok[0] == 'property':
            if tok[1] == 'list':
                elements[-1]['props'].append((tok[4], 'list', _TYPES[tok[2]], _TYPES[tok[3]]))
            else:
                elements[-1]['props'].append((tok[2], 'scalar', _TYPES[tok[1]], None))
        elif tok[0] == 'end_header':
            return fmt, elements


def _read_binary(f, elements, endian):
    data = {}
    buf = f.read()
    off = 0
    for el in elements:
        n = el['count']
        if all(p[1] == 'scalar' for p in el['props']):
            dt = np.dtype([(p[0], endian + p[2]) for p in el['props']])
            arr = np.frombuffer(buf, dt, count=n, offset=off)
            off += dt.itemsize * n
            data[el['name']] = {p[0]: arr[p[0]] for p in el['props']}
            continue
        props = el['props']
        if len(props) == 1 and props[0][1] == 'list':
            # one list property (the usual `vertex_indices`): vectorised if every face is a triangle
            name, _, t0, t1 = props[0]
            cs, isz = np.dtype(t0).itemsize, np.dtype(t1).itemsize
            rec = cs + 3 * isz
            if n and len(buf) >= off + rec * n:
                dt = np.dtype([('c', endian + t0), ('i', endian + t1, (3,))])
                arr = np.frombuffer(buf, dt, count=n, offset=off)
                if np.all(arr['c'] == 3):
                    data[el['name']] = {name: arr['i'].astype(np.int64)}
                    off += rec * n
                    continue
        # generic path
        cols = {p[0]: [] for p in el['props']}
        for _ in range(n):
            for name, kind, t0, t1 in el['props']:
                if kind == 'scalar':
                    v = np.frombuffer(buf, endian + t0, 1, off)[0]
                    off += np.dtype(t0).itemsize
                    cols[name].append(v)
                else:
                    cnt = int(np.frombuffer(buf, endian + t0, 1, off)[0])
                    off += np.dtype(t0).itemsize
                    cols[name].append(np.frombuffer(buf, endian + t1, cnt, off))
                    off += np.dtype(t1).itemsize * cnt
        data[el['name']] = cols
    return data


def _read_ascii(f, elements):
    data = {}
    tokens = f.read().split()
    pos = 0
    for el in elements:
        cols = {p[0]: [] for p in el['props']}
        for _ in range(el['count']):
            for name, kind, t0, t1 in el['props']:
                if kind == 'scalar':
                    cols[name].append(float(tokens[pos]))
                    pos += 1
                else:
                    cnt = int(tokens[pos])
                    pos += 1
                    cols[name].append(np.array([float(x) for x in tokens[pos:pos + cnt]]))
                    pos += cnt
        data[el['name']] = cols
    return data


def load_ply(path, toWorld=None, bsdf=-1, emitter=-1, faceNormals=False, flipNormals=False, name=''):
    toWorld = toWorld or Transform()
    with open(path, 'rb') as f:
        fmt, elements = _parse_header(f)
        if fmt == 'ascii':
            data = _read_ascii(f, elements)
        elif fmt in ('binary_little_endian', 'binary_big_endian'):
            data = _read_binary(f, elements, '<' if fmt == 'binary_little_endian' else '>')
        else:
            raise ValueError('unsupported PLY format %r' % fmt)
    if 'vertex' not in data or 'face' not in data:
        raise ValueError('Unable to load "%s" (no triangles or vertices found)!' % path)
    V = data['vertex']
    pos = np.stack([np.asarray(V[k], np.float32) for k in ('x', 'y', 'z')], 1)
    pos = toWorld.apply_points(pos)
    nrm = None
    if all(k in V for k in ('nx', 'ny', 'nz')):
        nrm = np.stack([np.asarray(V[k], np.float32) for k in ('nx', 'ny', 'nz')], 1)
        nrm = normalize_rows(toWorld.apply_normals(nrm))
    uv = None
    un = next((k for k in _U_NAMES if k in V), None)
    vn = next((k for k in _V_NAMES if k in V), None)
    if un is not None and vn is not None:
        uv = np.stack([np.asarray(V[un], np.float32), np.asarray(V[vn], np.float32)], 1)
    F = data['face']
    key = 'vertex_indices' if 'vertex_indices' in F else ('vertex_index' if 'vertex_index' in F else None)
    if key is None:
        raise ValueError('PLY face element has no vertex_indices')
    nv = pos.shape[0]
    faces = F[key]
    if isinstance(faces, np.ndarray) and faces.ndim == 2:     # all triangles (vectorised read)
        if np.any(faces < 0) or np.any(faces >= nv):
            raise ValueError('PLY face index out of range')
        return Mesh(pos, faces.astype(np.uint32), normals=nrm, texcoords=uv, bsdf=bsdf, emitter=emitter,
                    faceNormals=faceNormals, flipNormals=flipNormals, name=name)
    tris = []
    for face in faces:
        face = np.asarray(face, np.int64)
        if len(face) not in (3, 4):
            raise ValueError('Encountered a face with %d vertices! Only triangle and quad-based PLY '
                             'meshes are supported for now.' % len(face))
        if np.any(face < 0) or np.any(face >= nv):
            raise ValueError('PLY face index out of range')
        tris.append((face[0], face[1], face[2]))
        if len(face) == 4:
            tris.append((face[3], face[0], face[2]))
    if not tris or nv == 0:
        raise ValueError('Unable to load "%s" (no triangles or vertices found)!' % path)
    idx = np.asarray(tris, np.uint32)
    return Mesh(pos, idx, normals=nrm, texcoords=uv, bsdf=bsdf, emitter=emitter, faceNormals=faceNormals,
                flipNormals=flipNormals, name=name)


def write_ply(path, mesh):
    """Binary little-endian PLY of a Mesh (positions, optional normals/texcoords, triangles)."""
    P = np.asarray(mesh.positions, '<f4')
    cols = [P]
    props = ['x', 'y', 'z']
    if mesh.normals is not None:
        cols.append(np.asarray(mesh.normals, '<f4'))
        props += ['nx', 'ny', 'nz']
    if mesh.texcoords is not None:
        cols.append(np.asarray(mesh.texcoords, '<f4'))
        props += ['u', 'v']
    V = np.ascontiguousarray(np.concatenate(cols, axis=1), '<f4')
    idx = np.asarray(mesh.indices, '<i4')
    head = ['ply', 'format binary_little_endian 1.0', 'element vertex %d' % len(P)]
    head += ['property float %s' % p for p in props]
    head += ['element face %d' % len(idx), 'property list uchar int vertex_indices', 'end_header']
    faces = np.empty(len(idx), np.dtype([('c', 'u1'), ('i', '<i4', (3,))]))
    faces['c'] = 3
    faces['i'] = idx
    with open(path, 'wb') as fh:
        fh.write(('\n'.join(head) + '\n').encode())
        fh.write(V.tobytes())
        fh.write(faces.tobytes())
