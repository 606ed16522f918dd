"""TEST INFRASTRUCTURE: ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, '_build', 'liboracle.so')
# the same source built with the reference's release flags (Makefile REFFLAGS)
LIB_REFFLAGS = os.path.join(HERE, '_build', 'liboracle_refflags.so')
_lib = None
_libs = {}


def _stale(path=LIB):
    if not os.path.exists(path):
        return True
    t = os.path.getmtime(path)
    srcs = [os.path.join(HERE, f) for f in ('mts_oracle.c', 'mts_oracle.h', 'Makefile')]
    srcs.append(os.path.join(os.path.dirname(HERE), 'include', 'mtsgpu.h'))
    return any(os.path.getmtime(f) > t for f in srcs if os.path.exists(f))


def lib(variant='strict'):
    """The oracle library: 'strict' (source order, the parity checker) or
    'refflags' (the reference's -funsafe-math-optimizations release flags)."""
    global _lib
    path = LIB if variant == 'strict' else LIB_REFFLAGS
    if variant != 'strict' and variant != 'refflags':
        raise ValueError('unknown oracle variant %r' % variant)
    if variant == 'strict' and _lib is not None:
        return _lib
    if variant in _libs:
        return _libs[variant]
    if True:
        if _stale(path):   # a stale checker silently compares against old semantics: rebuild it
            import subprocess
            subprocess.run(['make', '-s', '-C', HERE], check=True)
        import sys
        sys.path.insert(0, os.path.dirname(HERE))
        from pkgimport import mitsuba_amd
        m = mitsuba_amd()
        abi = m.abi
        L = C.CDLL(path)
        L.oracle_sobol_init.argtypes = [C.c_char_p]
        L.oracle_render.argtypes = [C.POINTER(abi.SceneDesc), C.POINTER(abi.RenderParams),
                                    C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(abi.Stats),
                                    C.c_int, C.c_int]
        L.oracle_sobol_sample.restype = C.c_float
        L.oracle_sobol_sample.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32]
        L.oracle_sobol_lookup.restype = C.c_uint64
        L.oracle_sobol_lookup.argtypes = [C.c_uint32] * 4 + [C.c_uint64]
        L.oracle_sobol_matrix.restype = C.c_uint32
        L.oracle_sobol_matrix.argtypes = [C.c_uint32, C.c_uint32]
        L.oracle_triaccel_load.argtypes = [C.POINTER(C.c_float)] * 4
        L.oracle_triaccel_intersect.argtypes = [C.POINTER(C.c_float)] * 3 + [C.c_float, C.c_float, C.POINTER(C.c_float)]
        L.oracle_camera.argtypes = [C.POINTER(abi.SensorDesc), C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.oracle_bsdf_sample.argtypes = [C.POINTER(abi.BsdfDesc)] + [C.POINTER(C.c_float)] * 6 + [C.c_int]
        L.oracle_bsdf_eval.argtypes = [C.POINTER(abi.BsdfDesc)] + [C.POINTER(C.c_float)] * 4 + [C.c_int]
        L.oracle_fresnel_diffuse_reflectance.restype = C.c_float
        L.oracle_fresnel_diffuse_reflectance.argtypes = [C.c_float]
        L.oracle_configure.argtypes = [C.POINTER(abi.SceneDesc)]
        L.oracle_trace_rays.argtypes = [C.POINTER(abi.SceneDesc), C.POINTER(C.c_float), C.c_uint32, C.c_int,
                                        C.POINTER(C.c_float)]
        L.oracle_rdiel_trans_weight.argtypes = [C.c_int, C.c_float, C.c_float, C.POINTER(C.c_float), C.c_float,
                                                C.c_float, C.c_int]
        L.oracle_rdiel_trans_weight.restype = C.c_float
        L.oracle_set_kdtree.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        L.oracle_trace_rays_kd.argtypes = [C.POINTER(abi.SceneDesc), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                           C.POINTER(C.c_float), C.c_uint32, C.c_int, C.POINTER(C.c_float)]
        L.oracle_intersect.argtypes = [C.POINTER(abi.SceneDesc), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                       C.POINTER(C.c_float)]
        L.oracle_filter.argtypes = [C.c_int, C.c_float, C.POINTER(C.c_float)]
        L.oracle_sfmt_u64.argtypes = [C.c_uint64, C.POINTER(C.c_uint64), C.c_int, C.c_int]
        L.oracle_render_order.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                          C.POINTER(C.c_int)]
        rc = L.oracle_sobol_init(m.SOBOL_PARAMS.encode())
        if rc != 0:
            raise RuntimeError('oracle_sobol_init failed: %d' % rc)
        _libs[variant] = L
        if variant == 'strict':
            _lib = L
    return L


def trace_rays(scene, o, d, mint=1e-4, maxt=np.inf, shadow=False):
    """The oracle's Scene::rayIntersect / occlusion for a batch (same layout as Context.trace_rays)."""
    o = np.asarray(o, np.float32).reshape(-1, 3)
    d = np.asarray(d, np.float32).reshape(-1, 3)
    n = o.shape[0]
    rays = np.empty((n, 8), np.float32)
    rays[:, 0:3], rays[:, 3], rays[:, 4:7], rays[:, 7] = o, mint, d, maxt
    hits = np.empty((n, 4), np.float32)
    desc = scene.desc()
    fp = C.POINTER(C.c_float)
    rc = lib().oracle_trace_rays(C.byref(desc), rays.ctypes.data_as(fp), n, int(shadow), hits.ctypes.data_as(fp))
    if rc != 0:
        raise RuntimeError('oracle_trace_rays failed: %d' % rc)
    return hits


def trace_rays_kd(scene, nodes, indices, o, d, mint=1e-4, maxt=np.inf, shadow=False):
    """The same batch over a given kd-tree (KDNode words `nodes`, primitive lists
    `indices`) with SAHKDTree3D::rayIntersectHavran (sahkdtree3.h:178-308)."""
    o = np.asarray(o, np.float32).reshape(-1, 3)
    d = np.asarray(d, np.float32).reshape(-1, 3)
    n = o.shape[0]
    rays = np.empty((n, 8), np.float32)
    rays[:, 0:3], rays[:, 3], rays[:, 4:7], rays[:, 7] = o, mint, d, maxt
    hits = np.empty((n, 4), np.float32)
    nodes = np.ascontiguousarray(nodes, np.uint32)
    indices = np.ascontiguousarray(indices, np.uint32)
    desc = scene.desc()
    fp, up = C.POINTER(C.c_float), C.POINTER(C.c_uint32)
    rc = lib().oracle_trace_rays_kd(C.byref(desc), nodes.ctypes.data_as(up), indices.ctypes.data_as(up),
                                    rays.ctypes.data_as(fp), n, int(shadow), hits.ctypes.data_as(fp))
    if rc != 0:
        raise RuntimeError('oracle_trace_rays_kd failed: %d' % rc)
    return hits


def configure_rc(scene):
    """The oracle's configure() status for `scene` (0 = accepted)."""
    d = scene.desc()
    return lib().oracle_configure(C.byref(d))


def render(scene, integ, window=None, libm_mode=0, threads=1, samples=False, row=(0, 1, 0), variant='strict',
           kdtree=None, tile_shard=False):
    """Render with the oracle; returns (film (H+2b, W+2b, 5), samples or None, stats dict).
    variant='refflags' renders with the reference-flags build (lib()).
    kdtree=(nodes, indices): every ray query traverses that kd-tree (Havran).
    tile_shard: row = (-, stride, phase) selects 8x8 tiles t % stride == phase."""
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    from pkgimport import mitsuba_amd
    m = mitsuba_amd()
    L = lib(variant)
    W, H = scene.sensor.width, scene.sensor.height
    x0, y0, w, h = window if window else (getattr(integ, 'crop', None) or (0, 0, W, H))
    p = integ.params(W, H, x0, y0, w, h, row[0], row[1], row[2])
    if tile_shard:
        p.flags |= m.abi.FLAG_TILE_SHARD
    b = m.film_border(integ.rfilter, integ.rfilterParam)
    film = np.zeros((H + 2 * b, W + 2 * b, 5), np.float32)
    smp = np.zeros((w * h * integ.sampleCount, m.abi.SAMPLE_RECORD_FLOATS), np.float32) if samples else None
    st = m.abi.Stats()
    d = scene.desc()
    up = C.POINTER(C.c_uint32)
    if kdtree is not None:
        kn = np.ascontiguousarray(kdtree[0], np.uint32)
        ki = np.ascontiguousarray(kdtree[1], np.uint32)
        L.oracle_set_kdtree(kn.ctypes.data_as(up), ki.ctypes.data_as(up))
    try:
        rc = L.oracle_render(C.byref(d), C.byref(p), film.ctypes.data_as(C.POINTER(C.c_float)),
                             smp.ctypes.data_as(C.POINTER(C.c_float)) if samples else None,
                             C.byref(st), libm_mode, threads)
    finally:
        if kdtree is not None:
            L.oracle_set_kdtree(None, None)
    if rc != 0:
        raise RuntimeError('oracle_render failed: %d' % rc)
    return film, smp, st.as_dict()


def sfmt_u64(seed, n, clone=0):
    """The first n outputs of the reference's Random(seed)::nextULong (SFMT19937), or
    of the clone-th Random(&master) made from it (clone >= 1)."""
    out = np.zeros(n, np.uint64)
    lib().oracle_sfmt_u64(C.c_uint64(seed), out.ctypes.data_as(C.POINTER(C.c_uint64)), n, clone)
    return out


def filter_table(rfilter, param):
    """The oracle's configured filter: (radius, scale, border, values (FILTER_RES + 1,) float32)."""
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    from pkgimport import mitsuba_amd
    abi = mitsuba_amd().abi
    out = np.zeros(64, np.float32)
    t = {'box': abi.RFILTER_BOX, 'gaussian': abi.RFILTER_GAUSSIAN}[rfilter] if isinstance(rfilter, str) else rfilter
    rc = lib().oracle_filter(t, param, out.ctypes.data_as(C.POINTER(C.c_float)))
    if rc:
        raise ValueError('oracle_filter failed (%d)' % rc)
    return float(out[0]), np.float32(out[1]), int(out[2]), out[3:3 + 32].copy()


def render_order(width, height, block=32):
    """The reference's pixel order over a crop: (pixels (n, 2) int32 relative to the
    crop, block_start (num_blocks + 1,)) -- spiral blocks, Hilbert pixels."""
    nb = -(-width // block) * -(-height // block)
    pts = np.zeros((width * height, 2), np.int32)
    bs = np.zeros(nb + 1, np.int32)
    cnt = C.c_int(0)
    ip = C.POINTER(C.c_int)
    n = lib().oracle_render_order(width, height, block, pts.ctypes.data_as(ip), bs.ctypes.data_as(ip), C.byref(cnt))
    assert n == width * height and cnt.value == nb
    return pts, bs


def rdiel_trans_weight(distr, alpha, eta, wi, sx, sy, walter=False):
    """Rough-transmittance integrand (oracle_rdiel_trans_weight) at one point:
    distr 0/1/2 = beckmann/ggx/phong."""
    L = lib()
    w = (C.c_float * 3)(*[float(x) for x in wi])
    return L.oracle_rdiel_trans_weight(int(distr), alpha, eta, w, sx, sy, int(bool(walter)))

