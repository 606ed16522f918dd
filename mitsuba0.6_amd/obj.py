"""Wavefront OBJ shape loader: the host side of the reference's `obj` plugin.

Follows WavefrontOBJ (src/shapes/obj.cpp:190-720):
- `v`/`vn`/`vt` records. Texture v is flipped (v = 1 - v) unless flipTexCoords=False.
- `f` records with v, v/vt, v//vn and v/vt/vn forms, negative (relative) indices,
  and n-gons fanned as (p0, p_prev, p_new).
- One mesh per `g` group or `usemtl` switch (collapse=True keeps one mesh).
- Each mesh keeps its own vertex buffer: (p, n, uv) triples are merged in order
  of first use, as the reference's std::map keyed on the exact values does.
- Positions go through toWorld (points); normals go through its inverse
  transpose and are normalised when non-zero.

Materials from an `mtllib` are honoured for the BSDFs on the GPU path. A `Kd`
colour with illum 0/1 becomes `diffuse`, converted by Spectrum::fromSRGB
(spectrum.cpp). Other MTL models raise NotImplementedError.
"""
import ctypes
import ctypes.util
import os

import numpy as np

from .scene import BSDF, Mesh
from .transform import Transform, normalize_rows

f32 = np.float32
_libm = None


def _powf(x, y):
    global _libm
    if _libm is None:
        _libm = ctypes.CDLL(ctypes.util.find_library('m') or 'libm.so.6')
        _libm.powf.restype = ctypes.c_float
        _libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]
    return f32(_libm.powf(float(x), float(y)))


_libc = None


def strtof(text):
    """Correctly rounded decimal -> float32 (what `istream >> float` yields);
    numpy's str -> float32 goes through double and can round twice."""
    global _libc
    if _libc is None:
        _libc = ctypes.CDLL(ctypes.util.find_library('c') or 'libc.so.6')
        _libc.strtof.restype = ctypes.c_float
        _libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    return f32(_libc.strtof(text.encode() if isinstance(text, str) else text, None))


def srgb_to_linear(v):
    """Spectrum::fromSRGB component (spectrum.cpp): value <= 0.04045 ? value/12.92
    : powf((value + 0.055) / 1.055, 2.4), in single precision."""
    v = f32(v)
    if v <= f32(0.04045):
        return f32(v / f32(12.92))
    return _powf(f32(f32(v + f32(0.055)) / f32(1.055)), f32(2.4))


def _fetch_lines(path):
    """fetch_line (obj.cpp:152-175): strip trailing whitespace, join '\\'-continued lines."""
    with open(path, 'r', errors='replace') as fh:
        raw = fh.read().split('\n')
    out, i = [], 0
    while i < len(raw):
        line = raw[i].rstrip('\r\n\t ')
        while line.endswith('\\') and i + 1 < len(raw):
            i += 1
            line = line[:-1] + raw[i].rstrip('\r\n\t ')
        out.append(line)
        i += 1
    return out


def _parse_index(tok):
    parts = [p for p in tok.split('/') if p != '']
    if len(parts) == 1:
        return int(parts[0]), 0, 0
    if len(parts) == 2:
        if '//' not in tok:
            return int(parts[0]), int(parts[1]), 0
        return int(parts[0]), 0, int(parts[1])
    if len(parts) == 3:
        return int(parts[0]), int(parts[1]), int(parts[2])
    raise ValueError('Invalid OBJ face format!')


def _load_mtl(path):
    """MTL materials -> BSDF (obj.cpp:420-560, addMaterial: illum 0/1/other -> diffuse(Kd))."""
    mats, name, kd, illum, other = {}, '', (0.0, 0.0, 0.0), 0, False

    def flush():
        if name:
            model = illum
            if model in (2, 4, 5, 6, 7, 8, 9) or other:
                mats[name] = NotImplementedError('MTL material "%s" (illum %d) needs a BSDF outside the GPU path'
                                                 % (name, illum))
            else:
                mats[name] = BSDF('diffuse', reflectance=tuple(float(srgb_to_linear(c)) for c in kd))

    if not os.path.exists(path):
        return mats
    for line in _fetch_lines(path):
        tok = line.split()
        if not tok:
            continue
        if tok[0] == 'newmtl':
            flush()
            name, kd, illum, other = line[6:].strip(), (0.0, 0.0, 0.0), 0, False
        elif tok[0] == 'Kd':
            kd = tuple(float(x) for x in tok[1:4])
        elif tok[0] == 'illum':
            illum = int(tok[1])
        elif tok[0] in ('map_Kd', 'map_Ks', 'bump', 'map_d'):
            other = True
    flush()
    return mats


def load_obj(path, toWorld=None, faceNormals=False, flipNormals=False, flipTexCoords=True, collapse=False,
             shapeIndex=-1, loadMaterials=True, name=''):
    """Returns a list of (Mesh, material_name, mtl BSDF or None) in file order."""
    toWorld = toWorld or Transform()
    V, N, T = [], [], []
    tris = []                      # [(p[3], uv[3], n[3])]
    out = []
    geom_names, geom_index = set(), 0
    name_before_geometry = False
    cur_name = name or os.path.splitext(os.path.basename(path))[0]
    material = ''
    mtllib = None

    def create(mesh_name):
        if not tris:
            return
        vmap, vbuf = {}, []
        idx = np.empty((len(tris), 3), np.uint32)
        has_n = has_uv = False
        P = np.asarray(V, f32) if V else np.zeros((0, 3), f32)
        Pw = toWorld.apply_points(P) if len(P) else P
        Nw = None
        if N:
            Nw = toWorld.apply_normals(np.asarray(N, f32))
        for ti, (p, uv, n) in enumerate(tris):
            for j in range(3):
                vi, ni, ui = p[j], n[j], uv[j]
                if vi < 0:
                    vi += len(V) + 1
                if ni < 0:
                    ni += len(N) + 1
                if ui < 0:
                    ui += len(T) + 1
                if vi > len(V) or vi <= 0:
                    raise ValueError('Out of bounds: tried to access vertex %d (max: %d)' % (vi, len(V)))
                pos = tuple(float(x) for x in Pw[vi - 1])
                if ni != 0:
                    if ni > len(N) or ni < 0:
                        raise ValueError('Out of bounds: tried to access normal %d (max: %d)' % (ni, len(N)))
                    nv = Nw[ni - 1]
                    if np.any(nv != 0):
                        nv = normalize_rows(nv[None, :])[0]
                    nrm = tuple(float(x) for x in nv)
                    has_n = True
                else:
                    nrm = (0.0, 0.0, 0.0)
                if ui != 0:
                    if ui > len(T) or ui < 0:
                        raise ValueError('Out of bounds: tried to access uv %d (max: %d)' % (ui, len(T)))
                    tex = T[ui - 1]
                    has_uv = True
                else:
                    tex = (0.0, 0.0)
                key = pos + nrm + tex
                k = vmap.get(key)
                if k is None:
                    k = len(vbuf)
                    vmap[key] = k
                    vbuf.append(key)
                idx[ti, j] = k
        vb = np.asarray(vbuf, f32).reshape(-1, 8)
        m = Mesh(vb[:, 0:3].copy(), idx, normals=vb[:, 3:6].copy() if has_n else None,
                 texcoords=vb[:, 6:8].copy() if has_uv else None, faceNormals=faceNormals,
                 flipNormals=flipNormals, name=mesh_name)
        out.append((m, material))

    def flush_named(n):
        nonlocal geom_index
        if n in geom_names:
            n = '%s_%d' % (n, geom_index)
        geom_index += 1
        geom_names.add(n)
        if shapeIndex < 0 or geom_index - 1 == shapeIndex:
            create(n)
        tris.clear()

    for line in _fetch_lines(path):
        tok = line.split()
        if not tok:
            continue
        key = tok[0]
        if key == 'v':
            V.append(tuple(strtof(x) for x in tok[1:4]))
        elif key == 'vn':
            N.append(tuple(strtof(x) for x in tok[1:4]))
        elif key == 'vt':
            u = strtof(tok[1])
            v = strtof(tok[2]) if len(tok) > 2 else f32(0)
            if flipTexCoords:
                v = f32(f32(1) - v)
            T.append((float(u), float(v)))
        elif key == 'g' and not collapse:
            new_name = line[1:].strip()
            target = cur_name if name_before_geometry else new_name
            if tris:
                flush_named(target)
            else:
                name_before_geometry = True
            cur_name = new_name
        elif key == 'usemtl':
            if tris and not collapse:
                flush_named(cur_name)
                cur_name = name or os.path.splitext(os.path.basename(path))[0]
            material = line[6:].strip()
        elif key == 'mtllib':
            mtllib = os.path.join(os.path.dirname(os.path.abspath(path)), line[6:].strip())
        elif key == 'f':
            fs = [_parse_index(t) for t in tok[1:]]
            if len(fs) < 3:
                raise ValueError('Invalid OBJ face format!')
            p = [fs[0][0], fs[1][0], fs[2][0]]
            uv = [fs[0][1], fs[1][1], fs[2][1]]
            n = [fs[0][2], fs[1][2], fs[2][2]]
            tris.append((tuple(p), tuple(uv), tuple(n)))
            for extra in fs[3:]:
                p[1], uv[1], n[1] = p[2], uv[2], n[2]
                p[2], uv[2], n[2] = extra
                tris.append((tuple(p), tuple(uv), tuple(n)))
    final = cur_name
    if final in geom_names:
        final = '%s_%d' % (name or os.path.splitext(os.path.basename(path))[0], geom_index)
    if shapeIndex < 0 or geom_index - 1 == shapeIndex:
        create(final)
    mats = _load_mtl(mtllib) if (loadMaterials and mtllib) else {}
    return [(m, matname, mats.get(matname)) for m, matname in out]
