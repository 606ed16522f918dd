"""Synthetic benchmark scenes.

The reference ships no Cornell box or matpreview scene;
these are authored here, deterministically (seed 0x5EED), as the Mitsuba
scene a user would write: per-shape meshes with BSDFs and area emitters.
"""
import numpy as np

from .scene import BSDF, Emitter, Mesh, PathIntegrator, Scene, Sensor, look_at

S = 0.01  # classic Cornell box data is in millimetres; scene units are 10 cm

# Classic Cornell box geometry (Cornell University Program of Computer Graphics
# measurements); quads listed counter-clockwise as seen from inside the box.
_FLOOR = [(552.8, 0, 0), (0, 0, 0), (0, 0, 559.2), (549.6, 0, 559.2)]
_CEIL = [(556, 548.8, 0), (556, 548.8, 559.2), (0, 548.8, 559.2), (0, 548.8, 0)]
_BACK = [(549.6, 0, 559.2), (0, 0, 559.2), (0, 548.8, 559.2), (556, 548.8, 559.2)]
_GREEN = [(0, 0, 559.2), (0, 0, 0), (0, 548.8, 0), (0, 548.8, 559.2)]
_RED = [(552.8, 0, 0), (549.6, 0, 559.2), (556, 548.8, 559.2), (556, 548.8, 0)]
_LIGHT = [(343, 548.7, 227), (343, 548.7, 332), (213, 548.7, 332), (213, 548.7, 227)]
_SHORT = [[(130, 165, 65), (82, 165, 225), (240, 165, 272), (290, 165, 114)],
          [(290, 0, 114), (290, 165, 114), (240, 165, 272), (240, 0, 272)],
          [(130, 0, 65), (130, 165, 65), (290, 165, 114), (290, 0, 114)],
          [(82, 0, 225), (82, 165, 225), (130, 165, 65), (130, 0, 65)],
          [(240, 0, 272), (240, 165, 272), (82, 165, 225), (82, 0, 225)]]
_TALL = [[(423, 330, 247), (265, 330, 296), (314, 330, 456), (472, 330, 406)],
         [(423, 0, 247), (423, 330, 247), (472, 330, 406), (472, 0, 406)],
         [(472, 0, 406), (472, 330, 406), (314, 330, 456), (314, 0, 456)],
         [(314, 0, 456), (314, 330, 456), (265, 330, 296), (265, 0, 296)],
         [(265, 0, 296), (265, 330, 296), (423, 330, 247), (423, 0, 247)]]
_CENTER = np.array([278.0, 274.4, 279.6])


def _quads_mesh(quads, inward=True, center=_CENTER, uv=False):
    """Triangulate quads (0,1,2),(0,2,3); orient each so its normal faces `center`
    (inside of the room) or away from it (outside of a block).  uv=True also
    returns per-vertex texcoords (0,0),(1,0),(1,1),(0,1) per quad."""
    pos, idx = [], []
    for q in quads:
        q = np.asarray(q, np.float64)
        n = np.cross(q[1] - q[0], q[2] - q[0])
        to_c = center - q.mean(axis=0)
        facing = np.dot(n, to_c) > 0
        if facing != inward:
            q = q[::-1]
        base = len(pos)
        pos.extend(q)
        idx += [(base, base + 1, base + 2), (base, base + 2, base + 3)]
    p, i = (np.asarray(pos, np.float64) * S).astype(np.float32), np.asarray(idx, np.uint32)
    if uv:
        return p, i, np.tile(np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float32), (len(quads), 1))
    return p, i


# RGB complex IOR of copper (linear sRGB primaries; used as explicit 'eta'/'k'
# properties -- the reference's named-material .spd -> RGB conversion is a
# host-side step outside the hot path)
CU_ETA = (0.200438, 0.924033, 1.10221)
CU_K = (3.91295, 2.45285, 2.14219)


def rough_materials():
    """BSDF set exercising every rough-BSDF code path of the kernel."""
    return [
        BSDF('roughconductor', distribution='ggx', alpha=0.2, material=None, eta=CU_ETA, k=CU_K),
        BSDF('roughdielectric', distribution='beckmann', alpha=0.15, intIOR=1.5, extIOR='air'),
        BSDF('roughconductor', distribution='beckmann', alpha=0.35, material=None, eta=CU_ETA, k=CU_K),
        BSDF('roughdielectric', distribution='ggx', alpha=0.3, intIOR='bk7', extIOR='air'),
        BSDF('roughconductor', distribution='phong', alpha=0.25, material=None, eta=CU_ETA, k=CU_K),
        BSDF('roughconductor', distribution='ggx', alpha=0.1, sampleVisible=False, material='none'),
        BSDF('roughdielectric', distribution='ggx', alpha=0.2, sampleVisible=False, intIOR=1.33),
        BSDF('roughconductor', distribution='ggx', alphaU=0.05, alphaV=0.4, material=None, eta=CU_ETA, k=CU_K),
        BSDF('roughdielectric', distribution='beckmann', alphaU=0.3, alphaV=0.08, intIOR=1.5),
        BSDF('roughconductor', distribution='phong', alphaU=0.1, alphaV=0.3, material=None, eta=CU_ETA, k=CU_K),
    ]


def cornell_box(width=512, height=512, spp=64, rfilter='box', max_depth=-1, materials='diffuse'):
    """Config C1 (512x512, 64 spp) / C2 (1280x720, 512 spp): diffuse Cornell box
    with a rectangular area light.  materials='rough' swaps the
    blocks and floor for rough conductors/dielectrics (parity coverage)."""
    white = BSDF('diffuse', reflectance=(0.725, 0.71, 0.68))
    red = BSDF('diffuse', reflectance=(0.63, 0.065, 0.05))
    green = BSDF('diffuse', reflectance=(0.14, 0.45, 0.091))
    bsdfs = [white, red, green]
    meshes = []
    # room surfaces: vertex normals left to TriMesh::computeNormals (trimesh.cpp:608-681)
    floor_b, short_b, tall_b = 0, 0, 0
    if materials == 'rough':
        rough = rough_materials()
        base = len(bsdfs)
        bsdfs += rough
        floor_b, short_b, tall_b = base + 7, base + 0, base + 1
    uv = materials == 'rough'    # UV tangents on every rough surface (anisotropic ones require them)
    for quad, b in ((_FLOOR, floor_b), (_CEIL, 0), (_BACK, 0), (_GREEN, 2), (_RED, 1)):
        m = _quads_mesh([quad], inward=True, uv=uv)
        meshes.append(Mesh(m[0], m[1], texcoords=m[2] if uv else None, bsdf=b))
    for quads, b in ((_SHORT, short_b), (_TALL, tall_b)):
        m = _quads_mesh(quads, inward=False, center=np.mean(np.asarray(quads, np.float64).reshape(-1, 3), 0), uv=uv)
        meshes.append(Mesh(m[0], m[1], texcoords=m[2] if uv else None, bsdf=b, faceNormals=True))
    p, i = _quads_mesh([_LIGHT], inward=True)
    meshes.append(Mesh(p, i, bsdf=-1, emitter=0, faceNormals=True))
    emitters = [Emitter('area', radiance=(17.0, 12.0, 4.0))]
    cam = look_at(np.array([278, 273, -800]) * S, np.array([278, 273, -799]) * S, (0, 1, 0))
    sensor = Sensor(fov=39.3077, fovAxis='smaller', nearClip=10 * S, farClip=2800 * S,
                    toWorld=cam, width=width, height=height)
    scene = Scene(sensor, meshes, bsdfs, emitters, name='cornell-box')
    integ = PathIntegrator(maxDepth=max_depth, rrDepth=5, sampleCount=spp, rfilter=rfilter,
                           rfilterParam=0.5)
    return scene, integ


CONFIGS = {
    'C1': dict(builder='cornell_box', width=512, height=512, spp=64),
    'C2': dict(builder='cornell_box', width=1280, height=720, spp=512),
}


def build(config, **overrides):
    c = dict(CONFIGS[config])
    c.update(overrides)
    builder = globals()[c.pop('builder')]
    return builder(**c)
