"""ctypes mirror of include/mtsgpu.h (the C-ABI of libmtsgpu.so).

Plain data layouts only: the structs below are what a Mitsuba-side caller
hands across the boundary.  Keep in sync with include/mtsgpu.h.
"""
import ctypes as C

import numpy as np

OK, EINVAL, EHIP, ENOMEM, ESTATE, EDIM, ECANCEL, ENODEV, ENOENT = 0, -1, -2, -3, -4, -5, -6, -7, -8
STATUS_NAMES = {OK: 'OK', EINVAL: 'EINVAL', EHIP: 'EHIP', ENOMEM: 'ENOMEM', ESTATE: 'ESTATE',
                EDIM: 'EDIM', ECANCEL: 'ECANCEL', ENODEV: 'ENODEV', ENOENT: 'ENOENT'}

BSDF_DIFFUSE, BSDF_ROUGHCONDUCTOR, BSDF_ROUGHDIELECTRIC, BSDF_ROUGHPLASTIC = 0, 1, 2, 3
BSDF_CONDUCTOR, BSDF_DIELECTRIC, BSDF_PLASTIC, BSDF_TWOSIDED = 4, 5, 6, 7
TEX_NONE, TEX_CHECKERBOARD = 0, 1
ABI_VERSION = 8
TRACE_SHADOW, TRACE_KDTREE = 1, 2           # mtsgpu_trace_rays_ex flags
DISTR_BECKMANN, DISTR_GGX, DISTR_PHONG = 0, 1, 2
EMITTER_AREA, EMITTER_ENVMAP, EMITTER_CONSTANT = 0, 1, 2
SHAPE_TRIMESH, SHAPE_RECTANGLE, SHAPE_DISK, SHAPE_SPHERE = 0, 1, 2, 3
FOV_X, FOV_Y, FOV_DIAGONAL, FOV_SMALLER, FOV_LARGER = 0, 1, 2, 3, 4
RFILTER_BOX, RFILTER_GAUSSIAN = 0, 1
INTEGRATOR_PATH, INTEGRATOR_DIRECT, INTEGRATOR_VOLPATH = 0, 1, 2
SAMPLER_SOBOL, SAMPLER_INDEPENDENT, SAMPLER_SFMT_REPLAY, SAMPLER_SFMT_BLOCKS = 0, 1, 2, 3
SAMPLE_RECORD_FLOATS = 8
PIX_LUMINANCE, PIX_LUMINANCE_ALPHA, PIX_RGB, PIX_RGBA, PIX_XYZ, PIX_XYZA = 0, 1, 2, 3, 4, 5
COMP_FLOAT16, COMP_FLOAT32, COMP_UINT32 = 0, 1, 2

_f3 = C.c_float * 3
_f16 = C.c_float * 16


class TextureDesc(C.Structure):
    _fields_ = [('type', C.c_int32), ('color0', _f3), ('color1', _f3), ('uoffset', C.c_float),
                ('voffset', C.c_float), ('uscale', C.c_float), ('vscale', C.c_float)]


class BsdfDesc(C.Structure):
    _fields_ = [('type', C.c_int32), ('distribution', C.c_int32), ('sample_visible', C.c_int32),
                ('ensure_energy_conservation', C.c_int32),
                ('alpha_u', C.c_float), ('alpha_v', C.c_float),
                ('reflectance', _f3), ('specular_reflectance', _f3), ('specular_transmittance', _f3),
                ('eta', _f3), ('k', _f3), ('ext_eta', C.c_float),
                ('int_ior', C.c_float), ('ext_ior', C.c_float),
                ('diffuse_reflectance', _f3), ('nonlinear', C.c_int32),
                ('rtrans_data', C.c_void_p), ('rtrans_bytes', C.c_uint64),
                ('reflectance_tex', TextureDesc), ('alpha_tex', TextureDesc),
                ('nested', C.c_int32 * 2)]


class EmitterDesc(C.Structure):
    _fields_ = [('type', C.c_int32), ('radiance', _f3), ('sampling_weight', C.c_float),
                ('env_rgb', C.POINTER(C.c_float)), ('env_width', C.c_uint32), ('env_height', C.c_uint32),
                ('env_scale', C.c_float), ('env_to_world', _f16), ('env_to_world_inv', _f16)]


class MeshDesc(C.Structure):
    _fields_ = [('positions', C.POINTER(C.c_float)), ('normals', C.POINTER(C.c_float)),
                ('texcoords', C.POINTER(C.c_float)), ('indices', C.POINTER(C.c_uint32)),
                ('num_vertices', C.c_uint32), ('num_triangles', C.c_uint32),
                ('bsdf', C.c_int32), ('emitter', C.c_int32),
                ('face_normals', C.c_int32), ('flip_normals', C.c_int32),
                ('shape_type', C.c_int32), ('has_to_world', C.c_int32), ('to_world', _f16),
                ('to_world_inv', _f16), ('center', _f3), ('radius', C.c_float)]


class SensorDesc(C.Structure):
    _fields_ = [('fov', C.c_float), ('fov_axis', C.c_int32), ('near_clip', C.c_float),
                ('far_clip', C.c_float), ('to_world', _f16),
                ('film_width', C.c_uint32), ('film_height', C.c_uint32)]


class SceneDesc(C.Structure):
    _fields_ = [('meshes', C.POINTER(MeshDesc)), ('num_meshes', C.c_uint32),
                ('bsdfs', C.POINTER(BsdfDesc)), ('num_bsdfs', C.c_uint32),
                ('emitters', C.POINTER(EmitterDesc)), ('num_emitters', C.c_uint32),
                ('sensor', SensorDesc)]


class RenderParams(C.Structure):
    _fields_ = [('spp', C.c_uint32), ('scramble', C.c_uint64), ('max_depth', C.c_int32),
                ('rr_depth', C.c_int32), ('strict_normals', C.c_int32), ('hide_emitters', C.c_int32),
                ('has_alpha', C.c_int32), ('rfilter', C.c_int32), ('rfilter_param', C.c_float),
                ('x0', C.c_uint32), ('y0', C.c_uint32), ('width', C.c_uint32), ('height', C.c_uint32),
                ('row_block', C.c_uint32), ('row_stride', C.c_uint32), ('row_phase', C.c_uint32),
                ('cancel', C.POINTER(C.c_int32)), ('flags', C.c_uint32),
                ('integrator', C.c_int32), ('emitter_samples', C.c_uint32), ('bsdf_samples', C.c_uint32),
                ('sampler', C.c_int32)]


FLAG_TRAVERSAL_STATS = 1
FLAG_WAVEFRONT = 2
FLAG_MEGAKERNEL = 4
FLAG_KDTREE = 8                          # trace through the reference's kd-tree (wavefront engine)
FLAG_TILE_SHARD = 16                     # row_stride/row_phase interleave 8x8 tiles, not row blocks


class DevelopParams(C.Structure):
    _fields_ = [('film_width', C.c_uint32), ('film_height', C.c_uint32), ('border', C.c_uint32),
                ('pixel_format', C.c_int32), ('component_format', C.c_int32), ('multiplier', C.c_float)]


class Stats(C.Structure):
    _fields_ = [('samples', C.c_uint64), ('rays', C.c_uint64), ('shadow_rays', C.c_uint64),
                ('path_length_sum', C.c_uint64), ('node_visits', C.c_uint64),
                ('tri_tests', C.c_uint64), ('hits', C.c_uint64), ('nee_samples', C.c_uint64),
                ('sobol_reads', C.c_uint64), ('kernel_ms', C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def fptr(a):
    """float32 C-contiguous numpy array -> POINTER(c_float) (None passes NULL)."""
    if a is None:
        return None
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_float))


def uptr(a):
    assert a.dtype == np.uint32 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


XML_BSDF, XML_TEXTURE = 0, 1
XML_BY_ID, XML_BY_SHAPE = 0, 1                # mtsgpu_xml_bsdf_ex lookup
XML_PROP_PARAM, XML_PROP_DEFAULT, XML_PROP_UNSUPPORTED = 1, 2, 4   # mtsgpu_xml_prop.flags


class XmlNode(C.Structure):
    """mtsgpu_xml_node (include/mtsgpu.h)."""
    _fields_ = [('kind', C.c_int32), ('parent', C.c_int32), ('plugin', C.c_char * 32), ('name', C.c_char * 64),
                ('id', C.c_char * 64), ('first_prop', C.c_int32), ('num_props', C.c_int32)]


class XmlProp(C.Structure):
    """mtsgpu_xml_prop (include/mtsgpu.h)."""
    _fields_ = [('tag', C.c_char * 16), ('name', C.c_char * 64), ('value', C.c_char * 128), ('flags', C.c_int32)]
