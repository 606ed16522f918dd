"""Mitsuba 0.6 XML scene loader for the `path` GPU hot path.

This reads the subset of the reference's scene format (data/schema/scene.xsd)
that maps onto the path this library accelerates, with SceneHandler's
semantics (src/librender/scenehandler.cpp):
- `$name` parameters: keyword arguments override `<default>` values.
- `<include>` (the included file is parsed in place).
- `<ref id>` to named top-level objects.
- nested `<transform>` steps, each left-multiplying (translate, rotate, scale,
  lookat, matrix).
- properties: `<float>`, `<integer>`, `<boolean>`, `<string>`, `<rgb>`, `<srgb>`,
  `<spectrum>` (constant values), `<point>`, `<vector>`.

Plugins:
- integrators `path` and `volpath` (maxDepth, rrDepth, strictNormals,
  hideEmitters; volpath without media) and
  `direct` (shadingSamples, emitterSamples, bsdfSamples, strictNormals,
  hideEmitters).
- sensor `perspective` (fov/fovAxis or focalLength, near/farClip, toWorld),
  with sampler `sobol` (sampleCount, scramble) or `independent` (sampleCount;
  the default without a <sampler>), film `hdrfilm` or `mfilm` (size, crop
  window, pixel/file formats), whose rfilter is `box` or `gaussian`.
- shapes `obj`, `ply`, `serialized`, `cube` (triangle meshes) and the analytic
  `rectangle`, `disk`, `sphere`.
- BSDFs `diffuse`, `roughconductor`, `roughdielectric`, `roughplastic`,
  `conductor`, `dielectric`, `plastic`, `twosided`; `checkerboard` textures.
- emitters `area` (inside a shape), `envmap` (PFM/EXR/RGBE files) and `constant`.

Anything else raises NotImplementedError naming the plugin (e.g. `cylinder`,
`hair`, media).
"""
import math
import os
import re
import xml.etree.ElementTree as ET

import numpy as np

from .film import HDRFilm, MFilm, load_bitmap, read_pfm, write_pfm  # noqa: F401  (Bitmap readers/writers)
from .obj import load_obj, srgb_to_linear, strtof
from .ply import load_ply
from .scene import (BSDF, Checkerboard, DirectIntegrator, Emitter, Mesh, PathIntegrator, Scene, Sensor,
                    VolpathIntegrator)
from .serialized import load_serialized
from .transform import Transform, _cross, _normalize, normalize_rows

f32 = np.float32


class SceneError(ValueError):
    pass


# ---------------------------------------------------------------------------
# property parsing
# ---------------------------------------------------------------------------
def _xfloat(text):
    """SceneHandler::parseFloat (scenehandler.cpp:182-195): (Float) strtod(...)."""
    return f32(float(text))


def _floats(text):
    return [_xfloat(t) for t in re.split(r'[\s,]+', text.strip()) if t]


class _Props(dict):
    """Properties of one plugin (name -> python value), with the reference's
    getters' defaults and type errors."""

    def __init__(self, plugin, tag):
        super().__init__()
        self.plugin, self.tag, self.children = plugin, tag, []

    def get(self, name, default=None):
        return dict.get(self, name, default)


def _parse_transform(el, params):
    t = Transform()
    for step in el:
        a = {k: _subst(v, params) for k, v in step.attrib.items()}
        if step.tag == 'translate':
            t = t.translate(_xfloat(a.get('x', '0')), _xfloat(a.get('y', '0')), _xfloat(a.get('z', '0')))
        elif step.tag == 'rotate':
            t = t.rotate((_xfloat(a.get('x', '0')), _xfloat(a.get('y', '0')), _xfloat(a.get('z', '0'))),
                         _xfloat(a['angle']))
        elif step.tag == 'scale':
            if 'value' in a:
                v = _xfloat(a['value'])
                t = t.scale(v, v, v)
            else:
                t = t.scale(_xfloat(a.get('x', '1')), _xfloat(a.get('y', '1')), _xfloat(a.get('z', '1')))
        elif step.tag == 'lookat':
            o = _floats(a['origin'])
            tg = _floats(a['target'])
            up = _floats(a.get('up', '0 0 0'))
            if not any(up):
                # scenehandler.cpp:383-396: an unspecified 'up' picks one perpendicular to the direction
                d = _normalize((np.asarray(tg, f32) - np.asarray(o, f32)).astype(f32))
                if abs(d[0]) > abs(d[1]):
                    inv = f32(1) / f32(np.sqrt(f32(f32(d[0] * d[0]) + f32(d[2] * d[2]))))
                    c = np.array([d[2] * inv, 0, -d[0] * inv], f32)
                else:
                    inv = f32(1) / f32(np.sqrt(f32(f32(d[1] * d[1]) + f32(d[2] * d[2]))))
                    c = np.array([0, d[2] * inv, -d[1] * inv], f32)
                up = _cross(c, d)
            t = t.look_at(o, tg, up)
        elif step.tag == 'matrix':
            m = np.asarray(_floats(a['value']), f32).reshape(4, 4)
            t = Transform(m, _invert(m)) * t
        else:
            raise SceneError('unsupported transform step <%s>' % step.tag)
    return t


def _invert(m):
    """Matrix4x4::invert (core/matrix.inl:138-193), Gauss-Jordan in float32."""
    t = np.asarray(m, f32).copy()
    indxc, indxr, ipiv = [0] * 4, [0] * 4, [0] * 4
    for i in range(4):
        irow = icol = -1
        big = f32(0)
        for j in range(4):
            if ipiv[j] != 1:
                for k in range(4):
                    if ipiv[k] == 0:
                        if abs(t[j, k]) >= big:
                            big = abs(t[j, k])
                            irow, icol = j, k
                    elif ipiv[k] > 1:
                        raise SceneError('Singular matrix in Matrix::invert')
        ipiv[icol] += 1
        if irow != icol:
            t[[irow, icol]] = t[[icol, irow]]
        indxr[i], indxc[i] = irow, icol
        if t[icol, icol] == 0:
            raise SceneError('Singular matrix in Matrix::invert')
        pivinv = f32(f32(1) / t[icol, icol])
        t[icol, icol] = 1
        for j in range(4):
            t[icol, j] = f32(t[icol, j] * pivinv)
        for j in range(4):
            if j != icol:
                save = t[j, icol]
                t[j, icol] = 0
                for k in range(4):
                    t[j, k] = f32(t[j, k] - f32(t[icol, k] * save))
    for j in range(3, -1, -1):
        if indxr[j] != indxc[j]:
            t[:, [indxr[j], indxc[j]]] = t[:, [indxc[j], indxr[j]]]
    return t


def _subst(value, params):
    """$name substitution (scenehandler.cpp:123-149)."""
    def rep(mo):
        key = mo.group(1)
        if key not in params:
            raise SceneError('Unable to supply a value for the parameter "%s"' % key)
        return str(params[key])
    return re.sub(r'\$([A-Za-z_][A-Za-z0-9_]*)', rep, value)


def _spectrum(el, params):
    tag = el.tag
    v = _subst(el.attrib.get('value', ''), params)
    if tag == 'rgb':
        if len(v) == 7 and v.startswith('#'):
            return tuple(float(f32(f32(int(v[i:i + 2], 16)) / f32(255))) for i in (1, 3, 5))
        c = _floats(v)
        if len(c) == 1:
            c = c * 3
        return tuple(float(x) for x in c[:3])
    if tag == 'srgb':
        if v.startswith('#'):
            c = [f32(f32(int(v[i:i + 2], 16)) / f32(255)) for i in (1, 3, 5)]
        else:
            c = _floats(v)
            if len(c) == 1:
                c = c * 3
        return tuple(float(srgb_to_linear(x)) for x in c[:3])
    if tag == 'spectrum':
        if ':' in v or 'filename' in el.attrib:
            raise NotImplementedError('sampled <spectrum> values (wavelength:value lists, .spd files): '
                                      'give an <rgb> value')
        c = _floats(v)
        if len(c) == 1:
            return (float(c[0]),) * 3
        raise NotImplementedError('<spectrum> with %d values in the RGB build' % len(c))
    raise SceneError('not a spectrum: <%s>' % tag)


class XMLSceneLoader:
    def __init__(self, path, params):
        self.path = os.path.abspath(path)
        self.base = os.path.dirname(self.path)
        self.params = dict(params)
        self.named = {}

    def resolve(self, fn):
        p = fn if os.path.isabs(fn) else os.path.join(self.base, fn)
        if not os.path.exists(p):
            raise SceneError('file "%s" not found' % fn)
        return p

    # -- generic object parsing ------------------------------------------------
    def parse_object(self, el):
        props = _Props(el.attrib.get('type', ''), el.tag)
        for ch in el:
            tag = ch.tag
            name = ch.attrib.get('name', '')
            if tag in ('float', 'integer', 'boolean', 'string'):
                v = _subst(ch.attrib['value'], self.params)
                if tag == 'float':
                    props[name] = _xfloat(v)
                elif tag == 'integer':
                    props[name] = int(v)
                elif tag == 'boolean':
                    if v.lower() not in ('true', 'false'):
                        raise SceneError('could not parse boolean "%s"' % v)
                    props[name] = v.lower() == 'true'
                else:
                    props[name] = v
            elif tag in ('rgb', 'srgb', 'spectrum'):
                props[name] = _spectrum(ch, self.params)
            elif tag in ('point', 'vector'):
                a = {k: _subst(v, self.params) for k, v in ch.attrib.items()}
                if 'value' in a:
                    props[name] = tuple(_floats(a['value']))
                else:
                    props[name] = (_xfloat(a.get('x', '0')), _xfloat(a.get('y', '0')), _xfloat(a.get('z', '0')))
            elif tag == 'transform':
                props[name] = _parse_transform(ch, self.params)
            elif tag == 'ref':
                rid = ch.attrib['id']
                if rid not in self.named:
                    raise SceneError('Unable to find object with id "%s"' % rid)
                props.children.append((name, self.named[rid]))
            elif tag in ('bsdf', 'emitter', 'sampler', 'film', 'rfilter', 'shape', 'texture', 'sensor', 'medium',
                         'subsurface', 'phase', 'integrator'):
                props.children.append((name, self.parse_object(ch)))
            elif tag == 'animation':
                raise NotImplementedError('<animation> transforms')
            else:
                raise SceneError('unexpected tag <%s> inside <%s>' % (tag, el.tag))
        if 'id' in el.attrib and el.tag != 'scene':
            self.named[el.attrib['id']] = props
        return props

    # -- plugins ------------------------------------------------------------------
    def make_texture(self, p):
        """checkerboard (textures/checkerboard.cpp) with the Texture2D uv transform (texture.cpp:81-95)."""
        if p.plugin != 'checkerboard':
            raise NotImplementedError('texture "%s" (checkerboard is on the GPU path)' % p.plugin)
        if p.get('coordinates', 'uv') != 'uv':
            raise SceneError('Only UV coordinates are supported at the moment!')
        uvscale = float(p.get('uvscale', 1.0))
        return Checkerboard(color0=p.get('color0', 0.4), color1=p.get('color1', 0.2),
                            uoffset=float(p.get('uoffset', 0.0)), voffset=float(p.get('voffset', 0.0)),
                            uscale=float(p.get('uscale', uvscale)), vscale=float(p.get('vscale', uvscale)))

    def _tex_params(self, p, allowed):
        """Texture children (nested or <ref>) by parameter name; BSDF::addChild semantics."""
        out = {}
        for name, ch in p.children:
            if ch.tag != 'texture':
                continue
            if name not in allowed:
                raise SceneError('%s: unsupported texture parameter "%s"' % (p.plugin, name))
            out[name] = self.make_texture(ch)
        return out

    def make_bsdf(self, p):
        if p.tag != 'bsdf':
            raise SceneError('expected a BSDF')
        t = p.plugin
        if t == 'diffuse':
            tex = self._tex_params(p, ('reflectance',))
            return BSDF('diffuse', reflectance=tex.get('reflectance', p.get('reflectance', (0.5, 0.5, 0.5))),
                        ensureEnergyConservation=p.get('ensureEnergyConservation', True))
        if t in ('roughconductor', 'roughdielectric', 'roughplastic'):
            tex = self._tex_params(p, ('alpha', 'diffuseReflectance') if t == 'roughplastic' else ('alpha',))
            kw = dict(distribution=p.get('distribution', 'beckmann'), sampleVisible=p.get('sampleVisible', True),
                      specularReflectance=p.get('specularReflectance', (1.0, 1.0, 1.0)),
                      ensureEnergyConservation=p.get('ensureEnergyConservation', True))
            if 'alpha' in p:
                kw['alpha'] = float(p['alpha'])
            if 'alphaU' in p or 'alphaV' in p:
                kw['alphaU'], kw['alphaV'] = p.get('alphaU'), p.get('alphaV')
            if 'alpha' in tex:
                kw['alpha'] = tex['alpha']
            if t == 'roughconductor':
                kw.update(material=p.get('material', 'Cu'), eta=p.get('eta'), k=p.get('k'),
                          extEta=p.get('extEta', 'air'))
            elif t == 'roughdielectric':
                kw.update(intIOR=p.get('intIOR', 'bk7'), extIOR=p.get('extIOR', 'air'),
                          specularTransmittance=p.get('specularTransmittance', (1.0, 1.0, 1.0)))
            else:
                kw.update(intIOR=p.get('intIOR', 'polypropylene'), extIOR=p.get('extIOR', 'air'),
                          diffuseReflectance=tex.get('diffuseReflectance', p.get('diffuseReflectance', (0.5, 0.5, 0.5))),
                          nonlinear=p.get('nonlinear', False), rtransDir=os.path.dirname(os.path.abspath(self.path)))
            return BSDF(t, **kw)
        if t == 'conductor':                       # conductor.cpp:164-181
            self._tex_params(p, ())
            return BSDF('conductor', material=p.get('material', 'Cu'), eta=p.get('eta'), k=p.get('k'),
                        extEta=p.get('extEta', 'air'),
                        specularReflectance=p.get('specularReflectance', (1.0, 1.0, 1.0)),
                        ensureEnergyConservation=p.get('ensureEnergyConservation', True))
        if t == 'dielectric':                      # dielectric.cpp:146-165
            self._tex_params(p, ())
            return BSDF('dielectric', intIOR=p.get('intIOR', 'bk7'), extIOR=p.get('extIOR', 'air'),
                        specularReflectance=p.get('specularReflectance', (1.0, 1.0, 1.0)),
                        specularTransmittance=p.get('specularTransmittance', (1.0, 1.0, 1.0)),
                        ensureEnergyConservation=p.get('ensureEnergyConservation', True))
        if t == 'plastic':                         # plastic.cpp:144-165
            tex = self._tex_params(p, ('diffuseReflectance',))
            return BSDF('plastic', intIOR=p.get('intIOR', 'polypropylene'), extIOR=p.get('extIOR', 'air'),
                        specularReflectance=p.get('specularReflectance', (1.0, 1.0, 1.0)),
                        diffuseReflectance=tex.get('diffuseReflectance', p.get('diffuseReflectance', (0.5, 0.5, 0.5))),
                        nonlinear=p.get('nonlinear', False),
                        ensureEnergyConservation=p.get('ensureEnergyConservation', True))
        if t == 'twosided':                        # twosided.cpp:63-103, 193-205 (addChild)
            nested = [self.make_bsdf(c) for _, c in p.children if c.tag == 'bsdf']
            for _, c in p.children:
                if c.tag != 'bsdf':
                    raise SceneError('twosided: unexpected <%s> child' % c.tag)
            if not nested:
                raise SceneError('A nested one-sided material is required!')
            if len(nested) > 2:
                raise SceneError('No more than two nested BRDFs can be added!')
            return BSDF('twosided', nested=nested)
        raise NotImplementedError('BSDF plugin "%s" is not on the GPU path (diffuse, roughconductor, '
                                  'roughdielectric, roughplastic, conductor, dielectric, plastic, '
                                  'twosided)' % t)

    def make_area(self, p):
        if p.plugin != 'area':
            raise NotImplementedError('shape-attached emitter "%s"' % p.plugin)
        return Emitter('area', radiance=p.get('radiance', (1.0, 1.0, 1.0)), samplingWeight=p.get('samplingWeight', 1.0))

    def make_envmap(self, p):
        if p.plugin == 'constant':   # constant.cpp:46-49; Spectrum::getD65() is 1 in the RGB build (spectrum.cpp:163-165)
            return Emitter('constant', radiance=p.get('radiance', (1.0, 1.0, 1.0)),
                           samplingWeight=float(p.get('samplingWeight', 1.0)))
        fn = p.get('filename')
        if fn is None:
            raise SceneError('envmap: missing filename')
        path = self.resolve(fn)
        if p.get('gamma', 0) not in (0, 1):
            raise NotImplementedError('envmap gamma override')
        return Emitter('envmap', bitmap=load_bitmap(path), scale=float(p.get('scale', 1.0)),
                       samplingWeight=float(p.get('samplingWeight', 1.0)), toWorld=p.get('toWorld'))

    def make_shapes(self, p):
        t = p.plugin
        tw = p.get('toWorld')
        fn, flip = p.get('faceNormals', False), p.get('flipNormals', False)
        if t == 'obj':
            items = load_obj(self.resolve(p['filename']), toWorld=tw, faceNormals=fn, flipNormals=flip,
                             flipTexCoords=p.get('flipTexCoords', True), collapse=p.get('collapse', False),
                             shapeIndex=p.get('shapeIndex', -1), loadMaterials=p.get('loadMaterials', True))
            meshes = [(m, mat, mb) for m, mat, mb in items]
        elif t == 'ply':
            meshes = [(load_ply(self.resolve(p['filename']), toWorld=tw, faceNormals=fn, flipNormals=flip), '', None)]
        elif t == 'serialized':
            meshes = [(load_serialized(self.resolve(p['filename']), shapeIndex=p.get('shapeIndex', 0), toWorld=tw,
                                       faceNormals=fn, flipNormals=flip), '', None)]
        elif t == 'cube':
            meshes = [(cube_mesh(tw, flip), '', None)]
        elif t in ('rectangle', 'disk'):            # rectangle.cpp:80-85, disk.cpp:83-88
            meshes = [(Mesh(shape=t, toWorld=tw, flipNormals=flip), '', None)]
        elif t == 'sphere':                          # sphere.cpp:108-130
            c = p.get('center', (0.0, 0.0, 0.0))
            meshes = [(Mesh(shape='sphere', center=tuple(float(x) for x in c), radius=float(p.get('radius', 1.0)),
                            toWorld=tw, flipNormals=flip), '', None)]
        else:
            raise NotImplementedError('shape plugin "%s": the GPU path has obj, ply, serialized, cube, '
                                      'rectangle, disk and sphere' % t)
        return meshes

    # -- scene --------------------------------------------------------------------
    def load(self):
        root = ET.parse(self.path).getroot()
        if root.tag != 'scene':
            raise SceneError('root element must be <scene>')
        return self._scene(root)

    def _expand(self, root):
        """defaults and includes, in document order."""
        out = []
        for el in root:
            if el.tag == 'default':
                self.params.setdefault(el.attrib['name'], el.attrib['value'])
            elif el.tag == 'include':
                inc = ET.parse(self.resolve(_subst(el.attrib['filename'], self.params))).getroot()
                out.extend(self._expand(inc))
            else:
                out.append(el)
        return out

    def _scene(self, root):
        elements = self._expand(root)
        integ_props = sensor_props = None
        shape_props, env_props = [], []
        for el in elements:
            if el.tag == 'integrator':
                integ_props = self.parse_object(el)
            elif el.tag == 'sensor':
                sensor_props = self.parse_object(el)
            elif el.tag == 'shape':
                shape_props.append(self.parse_object(el))
            elif el.tag in ('bsdf', 'texture'):
                self.parse_object(el)       # named object for later <ref>
            elif el.tag == 'emitter':
                p = self.parse_object(el)
                if p.plugin not in ('envmap', 'constant'):
                    raise NotImplementedError('emitter plugin "%s" (area lights on shapes, envmap and constant '
                                              'are supported)' % p.plugin)
                env_props.append(p)
            elif el.tag in ('medium', 'subsurface'):
                raise NotImplementedError('<%s>: participating media / subsurface are not on the path' % el.tag)
            elif el.tag == 'alias':
                self.named[el.attrib['as']] = self.named[el.attrib['id']]
            else:
                raise SceneError('unexpected <%s> in <scene>' % el.tag)
        integ = self._integrator(integ_props)
        sensor, integ = self._sensor(sensor_props, integ)
        bsdfs, emitters, meshes = [], [], []
        bsdf_index = {}

        def bsdf_id(b):
            k = id(b)
            if k not in bsdf_index:
                bsdf_index[k] = len(bsdfs)
                bsdfs.append(b)
            return bsdf_index[k]

        made = {}
        for sp in shape_props:
            if sp.plugin in ('shapegroup', 'instance'):
                raise NotImplementedError('shape instancing')
            bsdf_children = [(n, c) for n, c in sp.children if c.tag == 'bsdf']
            em_children = [c for _, c in sp.children if c.tag == 'emitter']
            for n, c in sp.children:
                if c.tag not in ('bsdf', 'emitter'):
                    raise NotImplementedError('<%s> inside a shape' % c.tag)
            items = self.make_shapes(sp)
            if em_children and len(items) > 1:
                raise SceneError('Cannot attach an emitter to an OBJ file containing multiple objects!')
            for mesh, matname, mtlbsdf in items:
                b = None
                for n, c in bsdf_children:     # unnamed -> all meshes; named -> OBJ material (obj.cpp:736-760)
                    if n == '' or n == matname:
                        if id(c) not in made:
                            made[id(c)] = self.make_bsdf(c)
                        b = made[id(c)]
                if b is None and isinstance(mtlbsdf, Exception):
                    raise mtlbsdf
                if b is None and mtlbsdf is not None:
                    b = mtlbsdf
                mesh.bsdf = bsdf_id(b) if b is not None else -1
                for c in em_children:
                    mesh.emitter = len(emitters)
                    emitters.append(self.make_area(c))
                meshes.append(mesh)
        # the environment emitter comes after the shapes' emitters (Scene::addChild order)
        for ep in env_props:
            emitters.append(self.make_envmap(ep))
        if not meshes:
            raise SceneError('the scene has no triangle meshes')
        return Scene(sensor, meshes, bsdfs, emitters, name=os.path.basename(self.path)), integ

    def _integrator(self, p):
        if p is None:
            raise SceneError('no <integrator> (the GPU path implements "path")')
        if p.plugin == 'direct':                     # direct.cpp:92-107
            n = int(p.get('shadingSamples', 1))
            return DirectIntegrator(shadingSamples=n, emitterSamples=int(p.get('emitterSamples', n)),
                                    bsdfSamples=int(p.get('bsdfSamples', n)),
                                    strictNormals=p.get('strictNormals', False),
                                    hideEmitters=p.get('hideEmitters', False))
        if p.plugin not in ('path', 'volpath'):
            raise NotImplementedError('integrator "%s" (the GPU path implements "path", "volpath" and "direct")'
                                      % p.plugin)
        cls = VolpathIntegrator if p.plugin == 'volpath' else PathIntegrator
        return cls(maxDepth=p.get('maxDepth', -1), rrDepth=p.get('rrDepth', 5),
                   strictNormals=p.get('strictNormals', False), hideEmitters=p.get('hideEmitters', False))

    def _sensor(self, p, integ):
        if p is None:
            raise SceneError('no <sensor>')
        if p.plugin != 'perspective':
            raise NotImplementedError('sensor "%s" (only "perspective")' % p.plugin)
        film = next((c for _, c in p.children if c.tag == 'film'), None)
        sampler = next((c for _, c in p.children if c.tag == 'sampler'), None)
        width, height = 768, 576
        rfilter, rparam, has_alpha, crop, hdr = 'gaussian', 0.5, False, None, HDRFilm()
        if film is not None:
            if film.plugin not in ('hdrfilm', 'mfilm'):
                raise NotImplementedError('film "%s" (hdrfilm, mfilm)' % film.plugin)
            mf = film.plugin == 'mfilm'
            width, height = film.get('width', 1 if mf else 768), film.get('height', 1 if mf else 576)   # film.cpp:27-33
            try:
                if mf:
                    hdr = MFilm(fileFormat=film.get('fileFormat', 'matlab'), pixelFormat=film.get('pixelFormat',
                                                                                                   'luminance'),
                                digits=film.get('digits', 4), variable=film.get('variable', 'data'))
                    rfilter, rparam = 'box', 0.5            # mfilm.cpp:156-165: box by default
                else:
                    hdr = HDRFilm(fileFormat=film.get('fileFormat', 'openexr'),
                                  pixelFormat=film.get('pixelFormat', 'rgb'),
                                  componentFormat=film.get('componentFormat', 'float16'),
                                  channelNames=film.get('channelNames', ''), banner=film.get('banner', True),
                                  attachLog=film.get('attachLog', True))
            except ValueError as e:
                raise SceneError(str(e))
            if film.get('highQualityEdges', False):
                raise NotImplementedError('highQualityEdges=true (renders the border pixels outside the crop)')
            has_alpha = hdr.hasAlpha
            crop = (film.get('cropOffsetX', 0), film.get('cropOffsetY', 0), film.get('cropWidth', width),
                    film.get('cropHeight', height))
            if (crop[0] < 0 or crop[1] < 0 or crop[2] <= 0 or crop[3] <= 0 or crop[0] + crop[2] > width
                    or crop[1] + crop[3] > height):     # film.cpp:44-48
                raise SceneError('Invalid crop window specification!')
            rf = next((c for _, c in film.children if c.tag == 'rfilter'), None)
            if rf is not None:
                if rf.plugin == 'box':
                    rfilter, rparam = 'box', float(rf.get('radius', 0.5))
                elif rf.plugin == 'gaussian':
                    rfilter, rparam = 'gaussian', float(rf.get('stddev', 0.5))
                else:
                    raise NotImplementedError('rfilter "%s" (box, gaussian)' % rf.plugin)
        spp, scramble = 4, 0
        # no <sampler>: an independent sampler with 4 samples per pixel (sensor.cpp:92-97)
        kind = 'independent' if sampler is None else sampler.plugin
        if kind not in ('sobol', 'independent'):
            raise NotImplementedError('sampler "%s" (sobol, independent)' % kind)
        if sampler is not None:
            spp = sampler.get('sampleCount', 4)
            scramble = sampler.get('scramble', 0) if kind == 'sobol' else 0
        if 'fov' in p and 'focalLength' in p:
            raise SceneError("Please specify either a focal length ('focalLength') or a field of view ('fov')!")
        if 'fov' in p:
            fov, axis = float(p['fov']), p.get('fovAxis', 'x').lower()
        else:
            f = p.get('focalLength', '50mm')
            f = f[:-2] if f.endswith('mm') else f
            value = f32(float(f))
            # setDiagonalFov(2 * 180/M_PI * atan(sqrt(36*36+24*24) / (2*value))) (sensor.cpp:265-276)
            from .obj import _powf  # noqa: F401  (ensures libm is loaded)
            import ctypes
            import ctypes.util
            libm = ctypes.CDLL(ctypes.util.find_library('m') or 'libm.so.6')
            libm.atanf.restype = ctypes.c_float
            libm.atanf.argtypes = [ctypes.c_float]
            arg = f32(f32(np.sqrt(f32(1872))) / f32(f32(2) * value))
            fov = float(f32(f32(f32(360) / f32(math.pi)) * f32(libm.atanf(float(arg)))))
            axis = 'diagonal'
        tw = p.get('toWorld', Transform())
        sensor = Sensor(fov=fov, fovAxis=axis, nearClip=float(p.get('nearClip', 1e-2)),
                        farClip=float(p.get('farClip', 1e4)), toWorld=tw.m, width=width, height=height)
        integ.sampleCount, integ.scramble, integ.sampler = spp, scramble, kind
        integ.rfilter, integ.rfilterParam, integ.hasAlpha = rfilter, rparam, has_alpha
        integ.crop = crop
        integ.film = hdr
        return sensor, integ


# Cube shape data (src/shapes/cube.cpp): 24 vertices, faces -y, +y, +x, +z, -x, -z,
# each face (a, b, c, d) triangulated (a, b, c), (d, a, c); uv (0,1),(1,1),(1,0),(0,0)
_CUBE_FACES = [((1, -1, -1), (1, -1, 1), (-1, -1, 1), (-1, -1, -1), (0, -1, 0)),
               ((1, 1, -1), (-1, 1, -1), (-1, 1, 1), (1, 1, 1), (0, 1, 0)),
               ((1, -1, -1), (1, 1, -1), (1, 1, 1), (1, -1, 1), (1, 0, 0)),
               ((1, -1, 1), (1, 1, 1), (-1, 1, 1), (-1, -1, 1), (0, 0, 1)),
               ((-1, -1, 1), (-1, 1, 1), (-1, 1, -1), (-1, -1, -1), (-1, 0, 0)),
               ((1, 1, -1), (1, -1, -1), (-1, -1, -1), (-1, 1, -1), (0, 0, -1))]


def cube_mesh(toWorld=None, flipNormals=False):
    toWorld = toWorld or Transform()
    P, N, T, I = [], [], [], []
    for f, (a, b, c, d, n) in enumerate(_CUBE_FACES):
        P += [a, b, c, d]
        N += [n] * 4
        T += [(0, 1), (1, 1), (1, 0), (0, 0)]
        I += [(4 * f, 4 * f + 1, 4 * f + 2), (4 * f + 3, 4 * f, 4 * f + 2)]
    P = toWorld.apply_points(np.asarray(P, f32))
    N = normalize_rows(toWorld.apply_normals(np.asarray(N, f32)))
    return Mesh(P, np.asarray(I, np.uint32), normals=N, texcoords=np.asarray(T, f32), flipNormals=flipNormals,
                name='cube')


def load_scene(path, **params):
    """Load a Mitsuba 0.6 XML scene: returns (Scene, PathIntegrator); `params`
    supply $name values (like `mitsuba -Dname=value`)."""
    return XMLSceneLoader(path, params).load()


# ---------------------------------------------------------------------------
# writer (round trips programmatic scenes through the loader; PLY + PFM payloads)
# ---------------------------------------------------------------------------
def _fmt(x):
    """Shortest decimal that parses back to the same float32 through strtod + cast."""
    v = f32(x)
    for digits in range(6, 12):
        s = '%.*g' % (digits, float(v))
        if f32(float(s)) == v:
            return s
    return repr(float(v))


def _rgb(name, c):
    return '<rgb name="%s" value="%s"/>' % (name, ', '.join(_fmt(x) for x in _spec3(c)))


def _checker_xml(name, t):
    return ('<texture type="checkerboard" name="%s">%s%s<float name="uoffset" value="%s"/>'
            '<float name="voffset" value="%s"/><float name="uscale" value="%s"/><float name="vscale" value="%s"/>'
            '</texture>' % (name, _rgb('color0', _spec3(t.color0)), _rgb('color1', _spec3(t.color1)), _fmt(t.uoffset),
                            _fmt(t.voffset), _fmt(t.uscale), _fmt(t.vscale)))


def _spec3(v):
    return (v,) * 3 if isinstance(v, (int, float, np.floating)) else v


def _spec_xml(name, v):
    return _checker_xml(name, v) if isinstance(v, Checkerboard) else _rgb(name, _spec3(v))


def _matrix(m):
    return '<matrix value="%s"/>' % ' '.join(_fmt(x) for x in np.asarray(m, f32).reshape(-1))


def _transform_xml(t):
    """The construction steps when known (exact matrix and inverse), else a <matrix>."""
    if getattr(t, 'steps', None) is None:
        return _matrix(t.m)
    out = []
    for tag, a in t.steps:
        if tag == 'lookat':
            out.append('<lookat origin="%s" target="%s" up="%s"/>' % tuple(
                ', '.join(_fmt(x) for x in a[k]) for k in ('origin', 'target', 'up')))
        else:
            out.append('<%s %s/>' % (tag, ' '.join('%s="%s"' % (k, _fmt(v)) for k, v in a.items())))
    return ''.join(out)


def _ior_xml(nm, v, ind):
    return ind + '<%s name="%s" value="%s"/>' % (('string', nm, v) if isinstance(v, str) else ('float', nm, _fmt(v)))


def _bsdf_xml(b, ind, bid=None):
    """One <bsdf> element (nested BSDFs of twosided inline)."""
    L = ['%s<bsdf type="%s"%s>' % (ind, b.type, ' id="%s"' % bid if bid else '')]
    i2 = ind + '  '
    if b.type == 'twosided':
        for nb in b.nested:
            L += _bsdf_xml(nb, i2)
    elif b.type == 'diffuse':
        L.append(i2 + _spec_xml('reflectance', b.reflectance))
    else:
        if b.type.startswith('rough'):
            L.append(i2 + '<string name="distribution" value="%s"/>' % b.distribution)
            if isinstance(b.alpha, Checkerboard):
                L.append(i2 + _checker_xml('alpha', b.alpha))
            elif b.alpha is not None:
                L.append(i2 + '<float name="alpha" value="%s"/>' % _fmt(b.alpha))
            elif b.alphaU is not None:
                L.append(i2 + '<float name="alphaU" value="%s"/><float name="alphaV" value="%s"/>'
                         % (_fmt(b.alphaU), _fmt(b.alphaV)))
            L.append(i2 + '<boolean name="sampleVisible" value="%s"/>' % str(bool(b.sampleVisible)).lower())
        L.append(i2 + _rgb('specularReflectance', b.specularReflectance))
        if b.type in ('roughconductor', 'conductor'):
            if b.material:                    # None: the plugin default (Cu)
                L.append(i2 + '<string name="material" value="%s"/>' % b.material)
            if b.eta is not None:
                L.append(i2 + _rgb('eta', b.eta))
            if b.k is not None:
                L.append(i2 + _rgb('k', b.k))
            L.append(_ior_xml('extEta', b.extEta, i2))
        else:
            L.append(_ior_xml('intIOR', b.int_ior(), i2))
            L.append(_ior_xml('extIOR', b.extIOR, i2))
            if b.type in ('roughdielectric', 'dielectric'):
                L.append(i2 + _rgb('specularTransmittance', b.specularTransmittance))
            else:
                L.append(i2 + _spec_xml('diffuseReflectance', b.diffuseReflectance))
                L.append(i2 + '<boolean name="nonlinear" value="%s"/>' % str(bool(b.nonlinear)).lower())
    L.append(ind + '</bsdf>')
    return L


def save_scene(scene, integ, directory, name='scene.xml'):
    """Write `scene` as a Mitsuba 0.6 XML scene (meshes as PLY, envmap as PFM)."""
    os.makedirs(directory, exist_ok=True)
    from .ply import write_ply
    L = ['<?xml version="1.0" encoding="utf-8"?>', '<scene version="0.6.0">']
    if isinstance(integ, DirectIntegrator):
        L.append('  <integrator type="direct">')
        L.append('    <integer name="emitterSamples" value="%d"/>' % integ.emitterSamples)
        L.append('    <integer name="bsdfSamples" value="%d"/>' % integ.bsdfSamples)
    else:
        L.append('  <integrator type="%s">' % ('volpath' if isinstance(integ, VolpathIntegrator) else 'path'))
        L.append('    <integer name="maxDepth" value="%d"/>' % integ.maxDepth)
        L.append('    <integer name="rrDepth" value="%d"/>' % integ.rrDepth)
    L.append('    <boolean name="strictNormals" value="%s"/>' % str(bool(integ.strictNormals)).lower())
    L.append('    <boolean name="hideEmitters" value="%s"/>' % str(bool(integ.hideEmitters)).lower())
    L.append('  </integrator>')
    s = scene.sensor
    L.append('  <sensor type="perspective">')
    L.append('    <float name="fov" value="%s"/>' % _fmt(s.fov))
    L.append('    <string name="fovAxis" value="%s"/>' % s.fovAxis)
    L.append('    <float name="nearClip" value="%s"/>' % _fmt(s.nearClip))
    L.append('    <float name="farClip" value="%s"/>' % _fmt(s.farClip))
    L.append('    <transform name="toWorld">%s</transform>' % _matrix(s.toWorld))
    if integ.sampler == 'independent':
        L.append('    <sampler type="independent"><integer name="sampleCount" value="%d"/></sampler>'
                 % integ.sampleCount)
    else:
        L.append('    <sampler type="sobol"><integer name="sampleCount" value="%d"/>'
                 '<integer name="scramble" value="%d"/></sampler>' % (integ.sampleCount, integ.scramble))
    hf = integ.film or HDRFilm()
    mf = isinstance(hf, MFilm)
    L.append('    <film type="%s">' % ('mfilm' if mf else 'hdrfilm'))
    L.append('      <integer name="width" value="%d"/><integer name="height" value="%d"/>' % (s.width, s.height))
    fmt = hf.pixel_format if hf.hasAlpha == bool(integ.hasAlpha) else ('rgba' if integ.hasAlpha else 'rgb')
    L.append('      <string name="pixelFormat" value="%s"/>' % fmt)
    if mf:
        L.append('      <string name="fileFormat" value="%s"/><integer name="digits" value="%d"/>'
                 '<string name="variable" value="%s"/>' % (hf.fileFormat, hf.digits, hf.variable))
    else:
        L.append('      <string name="fileFormat" value="%s"/><string name="componentFormat" value="%s"/>'
                 % (hf.fileFormat, hf.componentFormat))
        L.append('      <boolean name="banner" value="%s"/>' % str(bool(hf.banner)).lower())
    if integ.crop:
        x0, y0, w, h = integ.crop
        L.append('      <integer name="cropOffsetX" value="%d"/><integer name="cropOffsetY" value="%d"/>'
                 '<integer name="cropWidth" value="%d"/><integer name="cropHeight" value="%d"/>' % (x0, y0, w, h))
    pname = 'radius' if integ.rfilter == 'box' else 'stddev'
    L.append('      <rfilter type="%s"><float name="%s" value="%s"/></rfilter>' % (integ.rfilter, pname,
                                                                                 _fmt(integ.rfilterParam)))
    L.append('    </film>')
    L.append('  </sensor>')
    for i, b in enumerate(scene.bsdfs):
        L += _bsdf_xml(b, '  ', 'bsdf%d' % i)
    for i, m in enumerate(scene.meshes):
        if m.analytic:
            L.append('  <shape type="%s">' % m.shape)
            if m.shape == 'sphere':
                L.append('    <point name="center" x="%s" y="%s" z="%s"/>' % tuple(_fmt(x) for x in m.center))
                L.append('    <float name="radius" value="%s"/>' % _fmt(m.radius))
            if m.toWorld is not None:
                t = m.toWorld if hasattr(m.toWorld, 'inv') else Transform(m.toWorld, m.toWorldInv)
                L.append('    <transform name="toWorld">%s</transform>' % _transform_xml(t))
        else:
            fn = 'mesh%03d.ply' % i
            write_ply(os.path.join(directory, fn), m)
            L.append('  <shape type="ply">')
            L.append('    <string name="filename" value="%s"/>' % fn)
            L.append('    <boolean name="faceNormals" value="%s"/>' % str(bool(m.faceNormals)).lower())
        L.append('    <boolean name="flipNormals" value="%s"/>' % str(bool(m.flipNormals)).lower())
        if m.bsdf >= 0:
            L.append('    <ref id="bsdf%d"/>' % m.bsdf)
        if m.emitter >= 0:
            e = scene.emitters[m.emitter]
            L.append('    <emitter type="area">%s<float name="samplingWeight" value="%s"/></emitter>'
                     % (_rgb('radiance', e.radiance), _fmt(e.samplingWeight)))
        L.append('  </shape>')
    for j, e in enumerate(scene.emitters):
        if e.type == 'constant':
            L.append('  <emitter type="constant">%s<float name="samplingWeight" value="%s"/></emitter>'
                     % (_rgb('radiance', e.radiance), _fmt(e.samplingWeight)))
            continue
        if e.type != 'envmap':
            continue
        fn = 'envmap%d.pfm' % j
        write_pfm(os.path.join(directory, fn), e.bitmap)
        L.append('  <emitter type="envmap">')
        L.append('    <string name="filename" value="%s"/>' % fn)
        L.append('    <float name="scale" value="%s"/>' % _fmt(e.scale))
        L.append('    <float name="samplingWeight" value="%s"/>' % _fmt(e.samplingWeight))
        if e.toWorld is not None:
            L.append('    <transform name="toWorld">%s</transform>' % _transform_xml(e.toWorld))
        L.append('  </emitter>')
    L.append('</scene>')
    path = os.path.join(directory, name)
    open(path, 'w').write('\n'.join(L) + '\n')
    return path
