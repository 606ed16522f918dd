"""`Transform` -- the reference's 4x4 transform pair (matrix + inverse).

Mirrors include/mitsuba/core/transform.h and src/libcore/transform.cpp in
float32 with the reference's evaluation order (Matrix4x4 product
matrix.h:744-756: `sum += a[i][k] * b[k][j]`), and the XML loader's
composition rule (src/librender/scenehandler.cpp:352-439: every nested
<translate>/<rotate>/<scale>/<lookat>/<matrix> left-multiplies the transform
built so far).  Only host-side scene construction uses this module.
"""
import ctypes
import ctypes.util

import numpy as np

f32 = np.float32

_libm = None


def _sincosf(x):
    """math::sincos(float) -> glibc sincosf, as the reference calls it (math.h:218-222)."""
    global _libm
    if _libm is None:
        _libm = ctypes.CDLL(ctypes.util.find_library('m') or 'libm.so.6')
        _libm.sinf.restype = ctypes.c_float
        _libm.sinf.argtypes = [ctypes.c_float]
        _libm.cosf.restype = ctypes.c_float
        _libm.cosf.argtypes = [ctypes.c_float]
    return f32(_libm.sinf(float(x))), f32(_libm.cosf(float(x)))


def _matmul(a, b):
    r = np.zeros((4, 4), f32)
    for i in range(4):
        for j in range(4):
            s = f32(0)
            for k in range(4):
                s = f32(s + f32(a[i, k] * b[k, j]))
            r[i, j] = s
    return r


def _normalize(v):
    v = np.asarray(v, f32)
    ln = f32(np.sqrt(f32(f32(f32(v[0] * v[0]) + f32(v[1] * v[1])) + f32(v[2] * v[2]))))
    r = f32(f32(1) / ln)
    return (v * r).astype(f32)


def _cross(a, b):
    return np.array([f32(a[1] * b[2]) - f32(a[2] * b[1]), f32(a[2] * b[0]) - f32(a[0] * b[2]),
                     f32(a[0] * b[1]) - f32(a[1] * b[0])], f32)


class Transform:
    def __init__(self, m=None, inv=None):
        self.m = np.eye(4, dtype=f32) if m is None else np.asarray(m, f32).copy()
        self.inv = np.eye(4, dtype=f32) if inv is None else np.asarray(inv, f32).copy()
        # XML steps that built this transform (None once composed arbitrarily);
        # lets the scene writer reproduce the exact matrix *and* inverse
        self.steps = [] if m is None and inv is None else None

    def _then(self, t, step):
        r = t * self
        r.steps = None if self.steps is None else self.steps + [step]
        return r

    def __mul__(self, t):                           # transform.cpp:28-31
        return Transform(_matmul(self.m, t.m), _matmul(t.inv, self.inv))

    @staticmethod
    def translate_(x, y, z):                        # transform.cpp:33-47
        m = np.eye(4, dtype=f32)
        inv = np.eye(4, dtype=f32)
        m[:3, 3] = (x, y, z)
        inv[:3, 3] = (-f32(x), -f32(y), -f32(z))
        return Transform(m, inv)

    @staticmethod
    def scale_(x, y, z):                            # transform.cpp:49-63
        m = np.diag([x, y, z, 1]).astype(f32)
        inv = np.diag([f32(1) / f32(x), f32(1) / f32(y), f32(1) / f32(z), 1]).astype(f32)
        return Transform(m, inv)

    @staticmethod
    def rotate_(axis, angle):                       # transform.cpp:65-97
        n = _normalize(axis)
        s, c = _sincosf(f32(angle) * f32(f32(np.pi) / f32(180)))  # degToRad (util.h:297), M_PI = M_PI_FLT
        one = f32(1)
        m = np.eye(4, dtype=f32)
        m[0, 0] = f32(n[0] * n[0]) + f32(f32(one - f32(n[0] * n[0])) * c)
        m[0, 1] = f32(f32(n[0] * n[1]) * f32(one - c)) - f32(n[2] * s)
        m[0, 2] = f32(f32(n[0] * n[2]) * f32(one - c)) + f32(n[1] * s)
        m[1, 0] = f32(f32(n[0] * n[1]) * f32(one - c)) + f32(n[2] * s)
        m[1, 1] = f32(n[1] * n[1]) + f32(f32(one - f32(n[1] * n[1])) * c)
        m[1, 2] = f32(f32(n[1] * n[2]) * f32(one - c)) - f32(n[0] * s)
        m[2, 0] = f32(f32(n[0] * n[2]) * f32(one - c)) - f32(n[1] * s)
        m[2, 1] = f32(f32(n[1] * n[2]) * f32(one - c)) + f32(n[0] * s)
        m[2, 2] = f32(n[2] * n[2]) + f32(f32(one - f32(n[2] * n[2])) * c)
        return Transform(m, m.T.copy())

    @staticmethod
    def look_at_(origin, target, up):               # transform.cpp:191-214
        p = np.asarray(origin, f32)
        d = _normalize((np.asarray(target, f32) - p).astype(f32))
        left = _normalize(_cross(np.asarray(up, f32), d))
        new_up = _cross(d, left)
        m = np.zeros((4, 4), f32)
        m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = left, new_up, d, p
        m[3, 3] = 1
        q = [f32(f32(f32(m[0, k] * p[0]) + f32(m[1, k] * p[1])) + f32(m[2, k] * p[2])) for k in range(3)]
        inv = np.zeros((4, 4), f32)
        inv[0, :3], inv[1, :3], inv[2, :3] = left, new_up, d
        inv[:3, 3] = (-q[0], -q[1], -q[2])
        inv[3, 3] = 1
        return Transform(m, inv)

    # XML-style builders: each step left-multiplies (scenehandler.cpp:352-439)
    def translate(self, x, y, z):
        return self._then(Transform.translate_(x, y, z), ('translate', {'x': x, 'y': y, 'z': z}))

    def scale(self, x, y=None, z=None):
        if y is None:
            y = z = x
        return self._then(Transform.scale_(x, y, z), ('scale', {'x': x, 'y': y, 'z': z}))

    def rotate(self, axis, angle):
        return self._then(Transform.rotate_(axis, angle),
                          ('rotate', {'x': axis[0], 'y': axis[1], 'z': axis[2], 'angle': angle}))

    def look_at(self, origin, target, up):
        return self._then(Transform.look_at_(origin, target, up),
                          ('lookat', {'origin': tuple(origin), 'target': tuple(target), 'up': tuple(up)}))

    def apply_points(self, p):
        """Transform::operator()(Point) (transform.h:108-125), row-wise over (n, 3)."""
        p = np.asarray(p, f32)
        m = self.m
        x = ((m[0, 0] * p[:, 0] + m[0, 1] * p[:, 1]) + m[0, 2] * p[:, 2]) + m[0, 3]
        y = ((m[1, 0] * p[:, 0] + m[1, 1] * p[:, 1]) + m[1, 2] * p[:, 2]) + m[1, 3]
        z = ((m[2, 0] * p[:, 0] + m[2, 1] * p[:, 1]) + m[2, 2] * p[:, 2]) + m[2, 3]
        w = ((m[3, 0] * p[:, 0] + m[3, 1] * p[:, 1]) + m[3, 2] * p[:, 2]) + m[3, 3]
        out = np.stack([x, y, z], 1).astype(f32)
        sel = w != f32(1)
        if np.any(sel):
            r = (f32(1) / w[sel]).astype(f32)
            out[sel] = out[sel] * r[:, None]
        return out

    def apply_normals(self, n):
        """Transform::operator()(Normal) (transform.h:203-211): inverse transpose."""
        n = np.asarray(n, f32)
        v = self.inv
        x = (v[0, 0] * n[:, 0] + v[1, 0] * n[:, 1]) + v[2, 0] * n[:, 2]
        y = (v[0, 1] * n[:, 0] + v[1, 1] * n[:, 1]) + v[2, 1] * n[:, 2]
        z = (v[0, 2] * n[:, 0] + v[1, 2] * n[:, 1]) + v[2, 2] * n[:, 2]
        return np.stack([x, y, z], 1).astype(f32)


def normalize_rows(v):
    v = np.asarray(v, f32)
    ln = np.sqrt(((v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]).astype(f32)).astype(f32)
    r = (f32(1) / ln).astype(f32)
    return (v * r[:, None]).astype(f32)
