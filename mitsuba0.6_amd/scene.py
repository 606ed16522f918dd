"""Host-side scene model mirroring the reference's plugin properties.

A `Scene` holds what Mitsuba 0.6 has after parsing and plugin construction
(SceneHandler -> PluginManager::createObject, src/librender/scenehandler.cpp):
world-space triangle meshes (the TriMesh that the obj/ply/serialized/cube shape
plugins produce, with their `toWorld` already applied), BSDF and emitter
parameters under the reference's property names, the perspective sensor, the
film and the sampler.  `Scene.desc()` packs it into the C-ABI structs of
include/mtsgpu.h; everything the reference derives in configure() is derived
behind the ABI by libmtsgpu.so.
"""
import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import abi

# IOR table entries used by the configs (src/bsdfs/ior.h:40-67)
IOR = {'vacuum': 1.0, 'air': 1.000277, 'water': 1.3330, 'bk7': 1.5046, 'glass': 1.5046,
       'diamond': 2.419, 'polypropylene': 1.49, 'acrylic glass': 1.49, 'fused quartz': 1.458}


def lookup_ior(v):
    if isinstance(v, str):
        return IOR[v.lower()]
    return float(v)


# sampler plugin names -> MTSGPU_SAMPLER_* (include/mtsgpu.h)
SAMPLERS = {'sobol': abi.SAMPLER_SOBOL, 'independent': abi.SAMPLER_INDEPENDENT,
            'independent-sfmt': abi.SAMPLER_SFMT_REPLAY, 'independent-sfmt-blocks': abi.SAMPLER_SFMT_BLOCKS}

@dataclass
class Checkerboard:
    """`checkerboard` texture (src/textures/checkerboard.cpp) with Texture2D's
    uv transform (src/librender/texture.cpp:81-121): uv' = uv * scale + offset,
    color0 where (2 (floor-mod of int(2u')) - 1) (2 (.. v') - 1) == 1."""
    color0: tuple = (0.4, 0.4, 0.4)
    color1: tuple = (0.2, 0.2, 0.2)
    uoffset: float = 0.0
    voffset: float = 0.0
    uscale: float = 1.0
    vscale: float = 1.0

    def fill(self, t):
        t.type = abi.TEX_CHECKERBOARD
        t.color0[:] = _spec(self.color0)
        t.color1[:] = _spec(self.color1)
        t.uoffset, t.voffset, t.uscale, t.vscale = self.uoffset, self.voffset, self.uscale, self.vscale

    def average(self):
        c0, c1 = np.asarray(_spec(self.color0), np.float32), np.asarray(_spec(self.color1), np.float32)
        return tuple(float(x) for x in ((c0 + c1) * np.float32(0.5)))


def _spec(v):
    """A Spectrum property: a float is Spectrum(value), a 3-tuple RGB."""
    if isinstance(v, (int, float, np.floating)):
        return (float(v),) * 3
    return tuple(float(x) for x in v)


BSDF_TYPES = {'diffuse': abi.BSDF_DIFFUSE, 'roughconductor': abi.BSDF_ROUGHCONDUCTOR,
              'roughdielectric': abi.BSDF_ROUGHDIELECTRIC, 'roughplastic': abi.BSDF_ROUGHPLASTIC,
              'conductor': abi.BSDF_CONDUCTOR, 'dielectric': abi.BSDF_DIELECTRIC,
              'plastic': abi.BSDF_PLASTIC, 'twosided': abi.BSDF_TWOSIDED}


@dataclass
class BSDF:
    """One of diffuse / roughconductor / roughdielectric / roughplastic /
    conductor / dielectric / plastic / twosided with Mitsuba property names.
    `reflectance` (diffuse), `diffuseReflectance` ((rough)plastic) and `alpha`
    (rough BSDFs, isotropic) may be a Checkerboard.  A twosided BSDF holds its
    one or two nested BSDFs in `nested` (twosided.cpp:63-103)."""
    type: str = 'diffuse'
    reflectance: object = (0.5, 0.5, 0.5)
    distribution: str = 'beckmann'
    alpha: object = None
    alphaU: Optional[float] = None
    alphaV: Optional[float] = None
    sampleVisible: bool = True
    specularReflectance: tuple = (1.0, 1.0, 1.0)
    specularTransmittance: tuple = (1.0, 1.0, 1.0)
    eta: Optional[tuple] = None        # roughconductor: explicit RGB eta/k override `material`
    k: Optional[tuple] = None
    material: Optional[str] = 'Cu'     # roughconductor.cpp:174 default
    extEta: object = 'air'
    intIOR: object = None              # roughdielectric: bk7 (roughdielectric.cpp:186); roughplastic: polypropylene
    extIOR: object = 'air'
    diffuseReflectance: object = (0.5, 0.5, 0.5)   # roughplastic.cpp:201
    nonlinear: bool = False
    rtransDir: Optional[str] = None    # where data/microfacet/<distribution>.dat is looked up first (rtrans.py)
    ensureEnergyConservation: bool = True
    nested: list = field(default_factory=list)   # twosided: [front] or [front, back]

    def int_ior(self):
        if self.intIOR is not None:
            return self.intIOR
        return 'polypropylene' if self.type in ('roughplastic', 'plastic') else 'bk7'

    def to_desc(self):
        d = abi.BsdfDesc()
        if self.type not in BSDF_TYPES:
            raise NotImplementedError('BSDF plugin "%s" is not on the GPU path' % self.type)
        d.type = BSDF_TYPES[self.type]
        d.nested[0] = d.nested[1] = -1
        d.distribution = {'beckmann': abi.DISTR_BECKMANN, 'ggx': abi.DISTR_GGX,
                          'phong': abi.DISTR_PHONG, 'as': abi.DISTR_PHONG}[self.distribution.lower()]
        d.sample_visible = int(self.sampleVisible)
        d.ensure_energy_conservation = int(self.ensureEnergyConservation)
        # MicrofacetDistribution(props) defaults alphaU = alphaV = 0.1 (microfacet.h:99-101,117-130)
        if isinstance(self.alpha, Checkerboard):
            if self.alphaU is not None or self.alphaV is not None:
                raise ValueError("Microfacet model: please specify either 'alpha' or 'alphaU'/'alphaV'.")
            au = av = 0.1
            self.alpha.fill(d.alpha_tex)
        elif self.alpha is not None:
            au = av = float(self.alpha)
        elif self.alphaU is not None or self.alphaV is not None:
            if self.alphaU is None or self.alphaV is None:
                raise ValueError("Microfacet model: both 'alphaU' and 'alphaV' must be specified.")
            au, av = float(self.alphaU), float(self.alphaV)
        else:
            au = av = 0.1
        d.alpha_u, d.alpha_v = au, av
        if isinstance(self.reflectance, Checkerboard):
            if self.type == 'diffuse':
                self.reflectance.fill(d.reflectance_tex)
        else:
            d.reflectance[:] = _spec(self.reflectance)
        d.specular_reflectance[:] = _spec(self.specularReflectance)
        d.specular_transmittance[:] = _spec(self.specularTransmittance)
        if self.type in ('roughconductor', 'conductor'):
            # intEta/intK from the material, overridden by explicit 'eta'/'k' (roughconductor.cpp:172-190)
            from .conductors import conductor_rgb
            eta, k = conductor_rgb(self.material or 'Cu')
            d.eta[:] = self.eta if self.eta is not None else eta
            d.k[:] = self.k if self.k is not None else k
        if self.type in ('roughplastic', 'plastic'):
            if isinstance(self.diffuseReflectance, Checkerboard):
                self.diffuseReflectance.fill(d.reflectance_tex)
            else:
                d.diffuse_reflectance[:] = _spec(self.diffuseReflectance)
            d.nonlinear = int(self.nonlinear)
        if self.type == 'roughplastic':
            from .rtrans import table_bytes
            data = table_bytes(self.distribution, [self.rtransDir])
            buf = C.create_string_buffer(data, len(data))
            d.rtrans_data = C.cast(buf, C.c_void_p)
            d.rtrans_bytes = len(data)
            d._keep = buf                  # the buffer lives as long as the descriptor
        d.ext_eta = lookup_ior(self.extEta)
        d.int_ior = lookup_ior(self.int_ior())
        d.ext_ior = lookup_ior(self.extIOR)
        return d


@dataclass
class Emitter:
    """`area` (src/emitters/area.cpp), `envmap` (src/emitters/envmap.cpp) or
    `constant` (src/emitters/constant.cpp: a uniform `radiance` environment).

    envmap: `bitmap` is the decoded lat-long image, (H, W, 3) linear RGB float32
    (what Bitmap(EAuto, stream) yields for an RGB EXR/PFM/HDR file), `scale` and
    `toWorld` (a transform.Transform) as in the XML."""
    type: str = 'area'
    radiance: tuple = (1.0, 1.0, 1.0)
    samplingWeight: float = 1.0
    bitmap: Optional[np.ndarray] = None
    scale: float = 1.0
    toWorld: object = None

    def to_desc(self):
        d = abi.EmitterDesc()
        d.type = {'area': abi.EMITTER_AREA, 'envmap': abi.EMITTER_ENVMAP, 'constant': abi.EMITTER_CONSTANT}[self.type]
        d.radiance[:] = self.radiance
        d.sampling_weight = self.samplingWeight
        d.env_scale = self.scale
        if self.toWorld is not None:
            d.env_to_world[:] = [float(x) for x in np.asarray(self.toWorld.m, np.float32).reshape(-1)]
            d.env_to_world_inv[:] = [float(x) for x in np.asarray(self.toWorld.inv, np.float32).reshape(-1)]
        else:
            d.env_to_world[:] = [float(x) for x in np.eye(4, dtype=np.float32).reshape(-1)]
            d.env_to_world_inv[:] = [float(x) for x in np.eye(4, dtype=np.float32).reshape(-1)]
        return d


@dataclass
class Mesh:
    """A shape: a world-space triangle mesh (obj/ply/serialized/cube) or, with
    `shape` = 'rectangle' / 'disk' / 'sphere', an analytic shape intersected
    exactly (src/shapes/{rectangle,disk,sphere}.cpp) -- then positions/indices
    are None and toWorld (+ its carried inverse), center and radius apply."""
    positions: Optional[np.ndarray] = None   # (n,3) float32, world space
    indices: Optional[np.ndarray] = None     # (m,3) uint32
    normals: Optional[np.ndarray] = None
    texcoords: Optional[np.ndarray] = None
    bsdf: int = -1
    emitter: int = -1
    faceNormals: bool = False
    flipNormals: bool = False
    name: str = ''
    shape: str = 'trimesh'
    toWorld: object = None                   # 'toWorld': transform.Transform or 4x4 (rectangle / disk / sphere)
    toWorldInv: Optional[np.ndarray] = None  # its inverse as the reference's Transform carries it
    center: tuple = (0.0, 0.0, 0.0)          # sphere
    radius: float = 1.0                      # sphere

    @property
    def analytic(self):
        return self.shape != 'trimesh'


@dataclass
class Sensor:
    fov: float = 39.3077
    fovAxis: str = 'x'
    nearClip: float = 1e-2
    farClip: float = 1e4
    toWorld: np.ndarray = field(default_factory=lambda: np.eye(4, dtype=np.float32))
    width: int = 768
    height: int = 576


def look_at(origin, target, up):
    """Transform::lookAt (src/libcore/transform.cpp:191-214), float32."""
    p = np.asarray(origin, np.float32)
    t = np.asarray(target, np.float32)
    up = np.asarray(up, np.float32)

    def normalize(v):
        ln = np.float32(np.sqrt(np.float32(v[0] * v[0] + v[1] * v[1]) + np.float32(v[2] * v[2])))
        r = np.float32(1.0) / ln
        return (v * r).astype(np.float32)

    def cross(a, b):
        return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2],
                         a[0] * b[1] - a[1] * b[0]], np.float32)
    d = normalize((t - p).astype(np.float32))
    left = normalize(cross(up, d))
    new_up = cross(d, left)
    m = np.zeros((4, 4), np.float32)
    m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = left, new_up, d, p
    m[3, 3] = 1
    return m


class Scene:
    """Scene after plugin construction (the C-ABI scene description)."""

    def __init__(self, sensor: Sensor, meshes: List[Mesh], bsdfs: List[BSDF], emitters: List[Emitter], name=''):
        self.sensor, self.meshes, self.bsdfs, self.emitters, self.name = sensor, meshes, bsdfs, emitters, name

    @property
    def num_triangles(self):
        """Primitives of the acceleration structure (an analytic shape counts one)."""
        return sum(1 if m.analytic else int(m.indices.shape[0]) for m in self.meshes)

    def desc(self):
        """Pack into abi.SceneDesc; the returned object keeps every buffer alive."""
        keep = []
        md = (abi.MeshDesc * len(self.meshes))()
        for i, m in enumerate(self.meshes):
            if m.analytic:
                md[i].shape_type = {'rectangle': abi.SHAPE_RECTANGLE, 'disk': abi.SHAPE_DISK,
                                    'sphere': abi.SHAPE_SPHERE}[m.shape]
                md[i].bsdf, md[i].emitter = m.bsdf, m.emitter
                md[i].flip_normals = int(m.flipNormals)
                md[i].has_to_world = int(m.toWorld is not None)
                tw, twi = m.toWorld, m.toWorldInv
                if hasattr(tw, 'inv'):           # a transform.Transform: matrix + carried inverse
                    tw, twi = tw.m, tw.inv
                T = np.eye(4, dtype=np.float32) if tw is None else np.asarray(tw, np.float32)
                md[i].to_world[:] = [float(x) for x in T.reshape(-1)]
                if twi is not None:
                    md[i].to_world_inv[:] = [float(x) for x in np.asarray(twi, np.float32).reshape(-1)]
                elif tw is None:
                    md[i].to_world_inv[:] = [float(x) for x in T.reshape(-1)]
                md[i].center[:] = [float(x) for x in m.center]
                md[i].radius = float(m.radius)
                continue
            pos = np.ascontiguousarray(m.positions, np.float32)
            idx = np.ascontiguousarray(m.indices, np.uint32)
            nrm = None if m.normals is None else np.ascontiguousarray(m.normals, np.float32)
            uv = None if m.texcoords is None else np.ascontiguousarray(m.texcoords, np.float32)
            keep += [pos, idx, nrm, uv]
            md[i].positions = abi.fptr(pos)
            md[i].normals = abi.fptr(nrm)
            md[i].texcoords = abi.fptr(uv)
            md[i].indices = abi.uptr(idx)
            md[i].num_vertices = pos.shape[0]
            md[i].num_triangles = idx.shape[0]
            md[i].bsdf, md[i].emitter = m.bsdf, m.emitter
            md[i].face_normals, md[i].flip_normals = int(m.faceNormals), int(m.flipNormals)
        # twosided's nested BSDFs go after the scene's own (mesh indices stay valid)
        flat = list(self.bsdfs)
        nested_idx = {}
        for i, b in enumerate(self.bsdfs):
            if b.type == 'twosided':
                if not 1 <= len(b.nested) <= 2:
                    raise ValueError('twosided: one or two nested BSDFs (twosided.cpp:82-87, 161-170)')
                nested_idx[i] = []
                for nb in b.nested:
                    nested_idx[i].append(len(flat))
                    flat.append(nb)
        bd = (abi.BsdfDesc * max(1, len(flat)))()
        for i, b in enumerate(flat):
            bdi = b.to_desc()
            keep.append(getattr(bdi, '_keep', None))
            if i in nested_idx:
                for k, j in enumerate(nested_idx[i]):
                    bdi.nested[k] = j
            bd[i] = bdi
        ed = (abi.EmitterDesc * max(1, len(self.emitters)))()
        for i, e in enumerate(self.emitters):
            ed[i] = e.to_desc()
            if e.type == 'envmap':
                if e.bitmap is None:
                    raise ValueError('envmap emitter needs a bitmap')
                img = np.ascontiguousarray(e.bitmap, np.float32)
                keep.append(img)
                ed[i].env_rgb = abi.fptr(img)
                ed[i].env_height, ed[i].env_width = img.shape[0], img.shape[1]
        d = abi.SceneDesc()
        d.meshes, d.num_meshes = md, len(self.meshes)
        d.bsdfs, d.num_bsdfs = bd, len(flat)
        d.emitters, d.num_emitters = ed, len(self.emitters)
        s = self.sensor
        d.sensor.fov = s.fov
        d.sensor.fov_axis = {'x': abi.FOV_X, 'y': abi.FOV_Y, 'diagonal': abi.FOV_DIAGONAL,
                             'smaller': abi.FOV_SMALLER, 'larger': abi.FOV_LARGER}[s.fovAxis]
        d.sensor.near_clip, d.sensor.far_clip = s.nearClip, s.farClip
        d.sensor.to_world[:] = [float(x) for x in np.asarray(s.toWorld, np.float32).reshape(-1)]
        d.sensor.film_width, d.sensor.film_height = s.width, s.height
        d._keep = (keep, md, bd, ed)
        return d


@dataclass
class PathIntegrator:
    """Properties of the reference `path` plugin (MonteCarloIntegrator ctor,
    src/librender/integrator.cpp:190-225) plus sampler/film settings."""
    maxDepth: int = -1
    rrDepth: int = 5
    strictNormals: bool = False
    hideEmitters: bool = False
    sampleCount: int = 4           # sobol 'sampleCount' (sobol.cpp:87)
    scramble: int = 0
    rfilter: str = 'gaussian'      # film default (film.cpp:93)
    rfilterParam: float = 0.5      # box radius / gaussian stddev
    hasAlpha: bool = False         # hdrfilm pixelFormat default "rgb" (hdrfilm.cpp:216)
    crop: Optional[tuple] = None   # hdrfilm crop window (x0, y0, w, h) (film.cpp:35-43); None = whole film
    film: Optional['HDRFilm'] = None   # hdrfilm output format (film.py); None = the hdrfilm defaults
    # 'sobol', 'independent' (counter-based streams), 'independent-sfmt' (the reference's
    # SFMT19937 stream of a one-worker render, replayed) or 'independent-sfmt-blocks' (one
    # SFMT clone per 32x32 block): include/mtsgpu.h MTSGPU_SAMPLER_*
    sampler: str = 'sobol'

    def __post_init__(self):
        if self.sampler not in SAMPLERS:
            raise ValueError('sampler "%s" (%s)' % (self.sampler, ', '.join(SAMPLERS)))
        if self.rrDepth <= 0:
            raise ValueError("'rrDepth' must be set to a value greater than zero!")
        if self.maxDepth <= 0 and self.maxDepth != -1:
            raise ValueError("'maxDepth' must be set to -1 (infinite) or a value greater than zero!")
        if self.film is None:
            from .film import HDRFilm
            self.film = HDRFilm()

    def params(self, width, height, x0=0, y0=0, w=None, h=None, row_block=0, row_stride=1, row_phase=0):
        p = abi.RenderParams()
        p.spp = self.sampleCount
        p.scramble = self.scramble
        p.max_depth, p.rr_depth = self.maxDepth, self.rrDepth
        p.strict_normals, p.hide_emitters = int(self.strictNormals), int(self.hideEmitters)
        p.has_alpha = int(self.hasAlpha)
        p.rfilter = {'box': abi.RFILTER_BOX, 'gaussian': abi.RFILTER_GAUSSIAN}[self.rfilter]
        p.rfilter_param = self.rfilterParam
        p.x0, p.y0 = x0, y0
        p.width = width - x0 if w is None else w
        p.height = height - y0 if h is None else h
        p.row_block, p.row_stride, p.row_phase = row_block, row_stride, row_phase
        p.integrator = abi.INTEGRATOR_PATH
        p.sampler = SAMPLERS[self.sampler]
        return p


@dataclass
class VolpathIntegrator(PathIntegrator):
    """The reference `volpath` plugin (MIVolumetricPathTracer,
    src/integrators/path/volpath.cpp) on scenes without participating media:
    path's properties; shadow rays are Scene::evalTransmittance segments to the
    sampled emitter point, the strictNormals test and the path-length count
    follow volpath.cpp.  Media are out of scope."""

    def params(self, *a, **kw):
        p = super().params(*a, **kw)
        p.integrator = abi.INTEGRATOR_VOLPATH
        return p


@dataclass
class DirectIntegrator(PathIntegrator):
    """Properties of the reference `direct` plugin (MIDirectIntegrator,
    src/integrators/direct/direct.cpp:90-135): `shadingSamples` sets both
    `emitterSamples` and `bsdfSamples` unless given; strictNormals/hideEmitters
    as in `path`.  Sampler and film settings as PathIntegrator (maxDepth and
    rrDepth are unused)."""
    shadingSamples: int = 1
    emitterSamples: Optional[int] = None
    bsdfSamples: Optional[int] = None

    def __post_init__(self):
        super().__post_init__()
        if self.emitterSamples is None:
            self.emitterSamples = self.shadingSamples
        if self.bsdfSamples is None:
            self.bsdfSamples = self.shadingSamples
        if self.emitterSamples + self.bsdfSamples <= 0 or min(self.emitterSamples, self.bsdfSamples) < 0:
            raise ValueError('direct: emitterSamples + bsdfSamples must be positive (direct.cpp:106)')

    def params(self, *a, **kw):
        p = super().params(*a, **kw)
        p.integrator = abi.INTEGRATOR_DIRECT
        p.emitter_samples, p.bsdf_samples = self.emitterSamples, self.bsdfSamples
        return p


def film_border(rfilter, param):
    """ReconstructionFilter border size (rfilter.cpp:50)."""
    import math
    radius = np.float32(param) + np.float32(1e-5) if rfilter == 'box' else np.float32(4) * np.float32(param)
    return int(math.ceil(np.float32(radius - np.float32(0.5))))
