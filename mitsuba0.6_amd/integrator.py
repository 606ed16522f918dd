"""`PathTracer`: the host-side mirror of the reference's `path` Integrator plugin.

Mirrors MIPathTracer / MonteCarloIntegrator (src/integrators/path/path.cpp:110-
117, src/librender/integrator.cpp:190-225): same property names and the same
errors (raised as ValueError where the reference calls Log(EError)).  Rendering
goes through libmtsgpu.so's C-ABI; there is no CPU fallback -- without the HIP
library or a gfx950 device every call raises `NativeUnavailable`.
"""
import ctypes as C
import os

import numpy as np

from . import LIB_PATH, abi
from .scene import PathIntegrator, film_border


class NativeUnavailable(RuntimeError):
    pass


class MtsgpuError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__('%s (%d): %s' % (abi.STATUS_NAMES.get(code, '?'), code, msg))
        self.code = code


EXPORTS = ['mtsgpu_create', 'mtsgpu_upload_scene', 'mtsgpu_film_border', 'mtsgpu_render',
           'mtsgpu_render_device', 'mtsgpu_last_error', 'mtsgpu_destroy', 'mtsgpu_abi_version',
           'mtsgpu_debug_arith', 'mtsgpu_debug_scene_info', 'mtsgpu_debug_counters', 'mtsgpu_debug_sfmt', 'mtsgpu_develop', 'mtsgpu_develop_device', 'mtsgpu_check_scene',
           'mtsgpu_trace_rays', 'mtsgpu_group_create', 'mtsgpu_group_size', 'mtsgpu_group_upload_scene',
           'mtsgpu_group_render', 'mtsgpu_group_render_device', 'mtsgpu_group_member', 'mtsgpu_group_last_error',
           'mtsgpu_group_destroy', 'mtsgpu_trace_rays_ex', 'mtsgpu_debug_kdtree', 'mtsgpu_kdtree_host', 'mtsgpu_debug_libm',
           'mtsgpu_bvh_host', 'mtsgpu_group_member_params', 'mtsgpu_render_pixels',
           'mtsgpu_xml_bsdf', 'mtsgpu_xml_bsdf_ex']

_lib = None


def load_library(path=None):
    """Load libmtsgpu.so (the in-tree build).  Raises NativeUnavailable if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise NativeUnavailable('libmtsgpu.so not built: %s (run __graft_entry__.build())' % p)
    # PyTorch ships its own libamdhip64: load it first, so that libmtsgpu binds
    # to the same HIP runtime and device pointers / streams from torch are valid
    # in both (two runtimes in one process hide the GPU from the second one).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(p)
    P = C.POINTER
    L.mtsgpu_create.argtypes = [C.c_int, P(C.c_void_p)]
    L.mtsgpu_upload_scene.argtypes = [C.c_void_p, P(abi.SceneDesc)]
    L.mtsgpu_film_border.argtypes = [C.c_int32, C.c_float]
    L.mtsgpu_group_member_params.argtypes = [P(abi.RenderParams), C.c_int, C.c_int, P(abi.RenderParams)]
    L.mtsgpu_render_pixels.argtypes = [P(abi.RenderParams)]
    L.mtsgpu_render_pixels.restype = C.c_uint64
    L.mtsgpu_xml_bsdf.argtypes = [C.c_char_p, C.c_char_p, P(abi.XmlNode), C.c_int, P(abi.XmlProp), C.c_int,
                                  P(C.c_int), P(C.c_int), C.c_char_p, C.c_size_t]
    L.mtsgpu_xml_bsdf_ex.argtypes = [C.c_char_p, C.c_char_p, C.c_int32, P(C.c_char_p), P(C.c_char_p), C.c_int32,
                                     P(abi.XmlNode), C.c_int, P(abi.XmlProp), C.c_int, P(C.c_int), P(C.c_int),
                                     C.c_char_p, C.c_size_t]
    L.mtsgpu_render.argtypes = [C.c_void_p, P(abi.RenderParams), P(C.c_float), P(C.c_float), P(abi.Stats)]
    L.mtsgpu_render_device.argtypes = [C.c_void_p, P(abi.RenderParams), C.c_void_p, C.c_void_p, P(abi.Stats)]
    L.mtsgpu_last_error.argtypes = [C.c_void_p]
    L.mtsgpu_last_error.restype = C.c_char_p
    L.mtsgpu_destroy.argtypes = [C.c_void_p]
    L.mtsgpu_debug_arith.argtypes = [C.c_void_p, P(C.c_float), P(C.c_float), P(C.c_float), C.c_int]
    L.mtsgpu_debug_scene_info.argtypes = [C.c_void_p, P(C.c_uint32)]
    L.mtsgpu_debug_counters.argtypes = [C.c_void_p, P(C.c_uint64)]
    L.mtsgpu_debug_sfmt.argtypes = [C.c_void_p, C.c_uint64, C.c_int, P(C.c_uint64), C.c_int]
    L.mtsgpu_debug_libm.argtypes = [C.c_void_p, C.c_int, P(C.c_float), P(C.c_float), P(C.c_float), C.c_size_t,
                                    C.c_uint32]
    L.mtsgpu_trace_rays.argtypes = [C.c_void_p, P(C.c_float), C.c_uint32, C.c_int, P(C.c_float), P(C.c_double)]
    L.mtsgpu_check_scene.argtypes = [P(abi.SceneDesc), C.c_char_p, C.c_size_t]
    L.mtsgpu_develop.argtypes = [C.c_void_p, P(abi.DevelopParams), P(C.c_float), C.c_void_p]
    L.mtsgpu_develop_device.argtypes = [C.c_void_p, P(abi.DevelopParams), C.c_void_p, C.c_void_p, C.c_void_p]
    L.mtsgpu_trace_rays_ex.argtypes = [C.c_void_p, P(C.c_float), C.c_uint32, C.c_uint32, P(C.c_float), P(C.c_double)]
    L.mtsgpu_debug_kdtree.argtypes = [C.c_void_p, P(C.c_uint32), C.c_size_t, P(C.c_uint32), C.c_size_t, P(C.c_uint32)]
    L.mtsgpu_kdtree_host.argtypes = [P(abi.SceneDesc), P(C.c_uint32), C.c_size_t, P(C.c_uint32), C.c_size_t,
                                     P(C.c_uint32), C.c_char_p, C.c_size_t]
    L.mtsgpu_bvh_host.argtypes = [P(abi.SceneDesc), P(C.c_uint32), C.c_size_t, P(C.c_uint32), C.c_size_t,
                                  P(C.c_uint32), C.c_size_t, P(C.c_uint32), C.c_char_p, C.c_size_t]
    L.mtsgpu_group_create.argtypes = [P(C.c_int), C.c_int, P(C.c_void_p)]
    L.mtsgpu_group_size.argtypes = [C.c_void_p]
    L.mtsgpu_group_upload_scene.argtypes = [C.c_void_p, P(abi.SceneDesc)]
    L.mtsgpu_group_render.argtypes = [C.c_void_p, P(abi.RenderParams), P(C.c_float), P(abi.Stats)]
    L.mtsgpu_group_render_device.argtypes = [C.c_void_p, P(abi.RenderParams), C.c_void_p, P(abi.Stats)]
    L.mtsgpu_group_member.argtypes = [C.c_void_p, C.c_int]
    L.mtsgpu_group_member.restype = C.c_void_p
    L.mtsgpu_group_last_error.argtypes = [C.c_void_p]
    L.mtsgpu_group_last_error.restype = C.c_char_p
    L.mtsgpu_group_destroy.argtypes = [C.c_void_p]
    if L.mtsgpu_abi_version() != abi.ABI_VERSION:
        raise NativeUnavailable('ABI version mismatch')
    if path is None:
        _lib = L
    return L


def check_scene(scene):
    """Host-only configure of `scene` (mtsgpu_check_scene): raises MtsgpuError with
    the reference's configure() error message, or returns None."""
    L = load_library()
    d = scene.desc()
    buf = C.create_string_buffer(1024)
    rc = L.mtsgpu_check_scene(C.byref(d), buf, 1024)
    if rc != 0:
        raise MtsgpuError(rc, buf.value.decode())


KD_KEYS = ('nodes', 'indices', 'inner', 'leaves', 'nonempty_leaves', 'retracted', 'pruned', 'max_depth')


def bvh_host(scene):
    """The BVH the kernels traverse, built on the host without a device
    (mtsgpu_bvh_host): (nodes (N, 16) uint32 MtsgNode words, hnodes (N, 8) MtsgHNode
    words, qnodes (M, 16) MtsgQNode words, 4-wide inner-node levels)."""
    L = load_library()
    d = scene.desc()
    info = (C.c_uint32 * 4)()
    buf = C.create_string_buffer(512)
    rc = L.mtsgpu_bvh_host(C.byref(d), None, 0, None, 0, None, 0, info, buf, 512)
    if rc != 0:
        raise MtsgpuError(rc, buf.value.decode())
    n = np.zeros((info[0], 16), np.uint32)
    h = np.zeros((info[1], 8), np.uint32)
    q = np.zeros((info[2], 16), np.uint32)
    up = C.POINTER(C.c_uint32)
    rc = L.mtsgpu_bvh_host(C.byref(d), n.ctypes.data_as(up), n.size, h.ctypes.data_as(up), h.size,
                           q.ctypes.data_as(up), q.size, info, buf, 512)
    if rc != 0:
        raise MtsgpuError(rc, buf.value.decode())
    return n, h, q, int(info[3])


def kdtree_host(scene):
    """The reference's SAH kd-tree of `scene`, built on the host without a device
    (mtsgpu_kdtree_host): (nodes (N, 2) uint32 KDNode words, indices, info dict)."""
    L = load_library()
    d = scene.desc()
    info = (C.c_uint32 * 8)()
    buf = C.create_string_buffer(512)
    rc = L.mtsgpu_kdtree_host(C.byref(d), None, 0, None, 0, info, buf, 512)
    if rc != 0:
        raise MtsgpuError(rc, buf.value.decode())
    nodes = np.zeros((info[0], 2), np.uint32)
    idx = np.zeros(max(1, info[1]), np.uint32)
    up = C.POINTER(C.c_uint32)
    rc = L.mtsgpu_kdtree_host(C.byref(d), nodes.ctypes.data_as(up), nodes.size, idx.ctypes.data_as(up), idx.size,
                              info, buf, 512)
    if rc != 0:
        raise MtsgpuError(rc, buf.value.decode())
    return nodes, idx[:info[1]], dict(zip(KD_KEYS, list(info)))


class Context:
    """One libmtsgpu context (one HIP device)."""

    def __init__(self, device=-1, lib_path=None):
        self.L = load_library(lib_path)
        h = C.c_void_p()
        rc = self.L.mtsgpu_create(device, C.byref(h))
        if rc != 0:
            raise NativeUnavailable('mtsgpu_create failed: %s' % self.L.mtsgpu_last_error(None).decode())
        self.h = h
        self.scene = None

    def _check(self, rc):
        if rc != 0:
            raise MtsgpuError(rc, self.L.mtsgpu_last_error(self.h).decode())

    def upload(self, scene):
        d = scene.desc()
        self._check(self.L.mtsgpu_upload_scene(self.h, C.byref(d)))
        self.scene = scene

    def debug_counters(self):
        """The 16 raw device counters of the last render (include/mtsgpu.h)."""
        out = (C.c_uint64 * 16)()
        self._check(self.L.mtsgpu_debug_counters(self.h, out))
        return list(out)

    def kernel_variant(self):
        """The megakernel instantiation the last render launched, decoded from debug
        counter 15 (capi.cpp): {'instr', 'scene_lds', 'feat', 'waves', 'name'}, where
        name is the template as rocprofv3 reports it, e.g.
        'path_kernel<false, false, 336, 4>'; None after a wavefront-engine render."""
        c = self.debug_counters()[15]
        if c & (1 << 16):
            return None
        feat = (c & 0xff) | (256 if c & (1 << 14) else 0) | (512 if c & (1 << 15) else 0)
        instr, lds, waves = bool(c & (1 << 13)), bool(c & (1 << 12)), (c >> 8) & 0xf
        b = lambda v: 'true' if v else 'false'
        return {'instr': instr, 'scene_lds': lds, 'feat': feat, 'waves': waves,
                'name': 'path_kernel<%s, %s, %d, %d>' % (b(instr), b(lds), feat, waves)}

    def debug_sfmt(self, seed, n, clone=0):
        """n nextULong draws of the device's SFMT19937 from Random(seed) (or its clone-th clone)."""
        out = np.zeros(n, np.uint64)
        self._check(self.L.mtsgpu_debug_sfmt(self.h, C.c_uint64(seed), clone, out.ctypes.data_as(C.POINTER(C.c_uint64)), n))
        return out

    def scene_info(self):
        info = (C.c_uint32 * 4)()
        self._check(self.L.mtsgpu_debug_scene_info(self.h, info))
        return {'nodes': info[0], 'prims': info[1], 'depth': info[2], 'cus': info[3]}

    @staticmethod
    def _engine_flags(engine):
        if engine is None:
            return 0
        if engine == 'wavefront':
            return abi.FLAG_WAVEFRONT
        if engine == 'megakernel':
            return abi.FLAG_MEGAKERNEL
        if engine == 'kdtree':       # the wavefront engine over the reference's kd-tree
            return abi.FLAG_KDTREE
        raise ValueError('engine must be None, "wavefront", "megakernel" or "kdtree"')

    def render(self, integ, window=None, samples=False, row=(0, 1, 0), traversal_stats=False, engine=None,
               tile_shard=False):
        """Returns (film (H+2b, W+2b, 5) float32, per-sample records or None, stats dict).
        engine: None (the library's default), 'wavefront', 'megakernel' or 'kdtree'
        (the wavefront engine tracing through the reference's kd-tree).
        row = (row_block, row_stride, row_phase); tile_shard: row_stride/row_phase
        select 8x8 tiles (MTSGPU_FLAG_TILE_SHARD) instead of row blocks."""
        sc = self.scene
        W, H = sc.sensor.width, sc.sensor.height
        x0, y0, w, h = window if window else (integ.crop or (0, 0, W, H))
        p = integ.params(W, H, x0, y0, w, h, row[0], row[1], row[2])
        if traversal_stats:
            p.flags |= abi.FLAG_TRAVERSAL_STATS
        if tile_shard:
            p.flags |= abi.FLAG_TILE_SHARD
        p.flags |= self._engine_flags(engine)
        b = film_border(integ.rfilter, integ.rfilterParam)
        film = np.zeros((H + 2 * b, W + 2 * b, 5), np.float32)
        smp = np.zeros((w * h * integ.sampleCount, abi.SAMPLE_RECORD_FLOATS), np.float32) if samples else None
        st = abi.Stats()
        self._check(self.L.mtsgpu_render(self.h, C.byref(p), film.ctypes.data_as(C.POINTER(C.c_float)),
                                          smp.ctypes.data_as(C.POINTER(C.c_float)) if samples else None,
                                          C.byref(st)))
        return film, smp, st.as_dict()

    def render_device(self, integ, film_ptr, stream_ptr=None, window=None, row=(0, 1, 0), engine=None,
                      tile_shard=False):
        sc = self.scene
        W, H = sc.sensor.width, sc.sensor.height
        x0, y0, w, h = window if window else (integ.crop or (0, 0, W, H))
        p = integ.params(W, H, x0, y0, w, h, row[0], row[1], row[2])
        if tile_shard:
            p.flags |= abi.FLAG_TILE_SHARD
        p.flags |= self._engine_flags(engine)
        st = abi.Stats()
        self._check(self.L.mtsgpu_render_device(self.h, C.byref(p), C.c_void_p(film_ptr),
                                                 C.c_void_p(stream_ptr) if stream_ptr else None, C.byref(st)))
        return st.as_dict()

    def develop(self, film, border, hdrfilm):
        """hdrfilm develop on the device (mtsgpu_develop): `film` (H+2b, W+2b, 5)
        float32 host array -> (H, W, C) in hdrfilm's component dtype."""
        film = np.ascontiguousarray(film, np.float32)
        if film.ndim != 3 or film.shape[2] != 5:
            raise ValueError('develop: film must be (H+2b, W+2b, 5) float32')
        p = hdrfilm.develop_params(film.shape, border)
        out = hdrfilm.output_array(film.shape, border)
        self._check(self.L.mtsgpu_develop(self.h, C.byref(p), abi.fptr(film), out.ctypes.data_as(C.c_void_p)))
        return out

    def develop_device(self, film_ptr, film_shape, border, hdrfilm, out_ptr, stream_ptr=None):
        """Same on device buffers (e.g. torch tensors' data_ptr()); the output
        holds hdrfilm.output_array(film_shape, border).nbytes bytes."""
        p = hdrfilm.develop_params(film_shape, border)
        self._check(self.L.mtsgpu_develop_device(self.h, C.byref(p), C.c_void_p(film_ptr), C.c_void_p(out_ptr),
                                                  C.c_void_p(stream_ptr) if stream_ptr else None))

    def kdtree(self):
        """The reference's SAH kd-tree of the uploaded scene (mtsgpu_debug_kdtree):
        (nodes (N, 2) uint32 KDNode words, indices uint32, info dict)."""
        info = (C.c_uint32 * 8)()
        self._check(self.L.mtsgpu_debug_kdtree(self.h, None, 0, None, 0, info))
        nodes = np.zeros((info[0], 2), np.uint32)
        idx = np.zeros(max(1, info[1]), np.uint32)
        up = C.POINTER(C.c_uint32)
        self._check(self.L.mtsgpu_debug_kdtree(self.h, nodes.ctypes.data_as(up), nodes.size, idx.ctypes.data_as(up),
                                               idx.size, info))
        return nodes, idx[:info[1]], dict(zip(KD_KEYS, list(info)))

    def trace_rays(self, o, d, mint=1e-4, maxt=np.inf, shadow=False, kdtree=False):
        """Scene::rayIntersect (shadow=False) / occlusion (shadow=True) for a batch of
        rays: o, d (n, 3); mint, maxt scalars or (n,).  kdtree=True traverses the
        reference's own kd-tree (MTSGPU_TRACE_KDTREE).  Returns (hits (n, 4) float32
        {t, u, v, prim bits}, kernel ms)."""
        o = np.asarray(o, np.float32).reshape(-1, 3)
        d = np.asarray(d, np.float32).reshape(-1, 3)
        n = o.shape[0]
        rays = np.empty((n, 8), np.float32)
        rays[:, 0:3], rays[:, 3], rays[:, 4:7], rays[:, 7] = o, mint, d, maxt
        hits = np.empty((n, 4), np.float32)
        ms = C.c_double()
        flags = (abi.TRACE_SHADOW if shadow else 0) | (abi.TRACE_KDTREE if kdtree else 0)
        self._check(self.L.mtsgpu_trace_rays_ex(self.h, abi.fptr(rays), n, flags, abi.fptr(hits), C.byref(ms)))
        return hits, ms.value

    LIBM_FNS = ('sin', 'cos', 'expf', 'acosf', 'atanf', 'tanf', 'atan2f', 'powf', 'fastexp', 'fastlog')

    def debug_libm(self, fn, a=None, b=None, first=0, n=None):
        """The device's transcendental `fn` (LIBM_FNS name or id) over a (and b),
        or over the n floats whose bits are first, first+1, ..."""
        fid = self.LIBM_FNS.index(fn) if isinstance(fn, str) else int(fn)
        P = C.POINTER(C.c_float)
        if a is not None:
            a = np.ascontiguousarray(a, np.float32)
            n = a.size
        if b is not None:
            b = np.ascontiguousarray(b, np.float32)
        out = np.empty(n, np.float32)
        self._check(self.L.mtsgpu_debug_libm(self.h, fid, abi.fptr(a) if a is not None else P(),
                                             abi.fptr(b) if b is not None else P(), abi.fptr(out), n,
                                             C.c_uint32(first)))
        return out

    def debug_arith(self, a, b):
        a = np.ascontiguousarray(a, np.float32)
        b = np.ascontiguousarray(b, np.float32)
        out = np.zeros((a.size, 8), np.float32)
        self._check(self.L.mtsgpu_debug_arith(self.h, abi.fptr(a), abi.fptr(b), abi.fptr(out), a.size))
        return out

    def close(self):
        if self.h:
            self.L.mtsgpu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceGroup:
    """One render over several GPUs of this node (mtsgpu_group_*): the library
    shards the 8x8 tiles over the devices, one host thread each, and merges the films
    on the first device over xGMI (include/mtsgpu.h).  A device may be listed
    twice (two contexts on one GPU)."""

    def __init__(self, devices, lib_path=None):
        self.L = load_library(lib_path)
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        rc = self.L.mtsgpu_group_create(devs, len(devices), C.byref(h))
        if rc != 0:
            raise NativeUnavailable('mtsgpu_group_create failed: %s' % self.L.mtsgpu_group_last_error(None).decode())
        self.h = h
        self.devices = list(devices)
        self.scene = None

    def _check(self, rc):
        if rc != 0:
            raise MtsgpuError(rc, self.L.mtsgpu_group_last_error(self.h).decode())

    def __len__(self):
        return self.L.mtsgpu_group_size(self.h)

    def upload(self, scene):
        d = scene.desc()
        self._check(self.L.mtsgpu_group_upload_scene(self.h, C.byref(d)))
        self.scene = scene

    def render(self, integ, window=None, engine=None, row_block=8):
        """Returns (film (H+2b, W+2b, 5) float32, stats dict) of the whole window."""
        sc = self.scene
        W, H = sc.sensor.width, sc.sensor.height
        x0, y0, w, h = window if window else (integ.crop or (0, 0, W, H))
        p = integ.params(W, H, x0, y0, w, h, row_block, 1, 0)
        p.flags |= Context._engine_flags(engine)
        b = film_border(integ.rfilter, integ.rfilterParam)
        film = np.zeros((H + 2 * b, W + 2 * b, 5), np.float32)
        st = abi.Stats()
        self._check(self.L.mtsgpu_group_render(self.h, C.byref(p), film.ctypes.data_as(C.POINTER(C.c_float)),
                                                C.byref(st)))
        return film, st.as_dict()

    def close(self):
        if self.h:
            self.L.mtsgpu_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PathTracer(PathIntegrator):
    """The `path` integrator (MIPathTracer) running on MI355X."""

    def render(self, scene, ctx=None):
        ctx = ctx or Context()
        if ctx.scene is not scene:
            ctx.upload(scene)
        film, _, stats = ctx.render(self)
        return film, stats
