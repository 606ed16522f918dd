"""Synthetic benchmark scenes.

The reference ships no Cornell box or matpreview scene;
these are authored here, deterministically (seed 0x5EED), as the Mitsuba
scene a user would write: per-shape meshes with BSDFs and area emitters.
"""
import numpy as np

from .scene import BSDF, Checkerboard, Emitter, Mesh, PathIntegrator, Scene, Sensor, look_at
from .transform import Transform

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


# an explicit RGB complex IOR (the 'eta'/'k' override path); named materials
# come from conductors.py
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
        BSDF('roughconductor', distribution='ggx', alpha=0.15, material='Au'),
        BSDF('roughconductor', distribution='beckmann', alpha=0.2, material='Al', extEta=1.33),
    ]


def plastic_materials():
    """roughplastic (with the rough-transmittance tables) and checkerboard-textured
    BSDFs: constant and textured roughness, the three distributions, nonlinear,
    a textured diffuse reflectance."""
    chk_alpha = Checkerboard(color0=0.05, color1=0.4, uscale=3.0, vscale=3.0)
    return [
        BSDF('roughplastic', distribution='ggx', alpha=0.15, diffuseReflectance=(0.1, 0.3, 0.7)),
        BSDF('roughplastic', distribution='beckmann', alpha=chk_alpha, diffuseReflectance=(0.6, 0.2, 0.1),
             intIOR=1.6),
        BSDF('roughplastic', distribution='phong', alpha=0.3, nonlinear=True, diffuseReflectance=(0.7, 0.7, 0.2)),
        BSDF('roughplastic', distribution='ggx', alpha=chk_alpha, sampleVisible=False,
             diffuseReflectance=Checkerboard(color0=(0.8, 0.1, 0.1), color1=(0.1, 0.1, 0.8), uscale=4, vscale=4)),
        BSDF('diffuse', reflectance=Checkerboard(color0=(0.75, 0.75, 0.7), color1=(0.2, 0.25, 0.3), uscale=6,
                                                 vscale=6, uoffset=0.1)),
        BSDF('roughconductor', distribution='ggx', alpha=Checkerboard(color0=0.02, color1=0.3, uscale=2,
                                                                      vscale=2), material='Au'),
    ]


def smooth_materials():
    """Delta BSDFs and twosided: conductor (named and 'none'), dielectric
    (glass, water-like with a tinted transmittance), plastic (linear, and
    nonlinear with a textured diffuse base), twosided with one and with two
    nested BSDFs."""
    return [
        BSDF('conductor', material='Cu'),
        BSDF('dielectric', intIOR=1.5, extIOR='air'),
        BSDF('plastic', diffuseReflectance=(0.1, 0.3, 0.7)),
        BSDF('plastic', intIOR=1.6, nonlinear=True,
             diffuseReflectance=Checkerboard(color0=(0.8, 0.1, 0.1), color1=(0.1, 0.1, 0.8), uscale=4, vscale=4)),
        BSDF('twosided', nested=[BSDF('diffuse', reflectance=(0.14, 0.45, 0.091))]),
        BSDF('twosided', nested=[BSDF('plastic', diffuseReflectance=(0.7, 0.6, 0.2)),
                                 BSDF('roughconductor', distribution='ggx', alpha=0.2, material='Au')]),
        BSDF('conductor', material='none', specularReflectance=0.8),
        BSDF('dielectric', intIOR=1.33, extIOR=1.0, specularTransmittance=(0.9, 0.8, 0.7)),
        # roughplastic inside twosided: its per-vertex transmittance terms are
        # formed for the nested BSDF and the side's wi (path_kernel rpPre)
        BSDF('twosided', nested=[BSDF('roughplastic', distribution='ggx', alpha=0.2,
                                      diffuseReflectance=(0.6, 0.3, 0.2))]),
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
    back_b = 0
    if materials == 'rough':
        rough = rough_materials()
        base = len(bsdfs)
        bsdfs += rough
        floor_b, short_b, tall_b = base + 7, base + 0, base + 1
    elif materials == 'plastic':
        base = len(bsdfs)
        bsdfs += plastic_materials()
        floor_b, short_b, tall_b, back_b = base + 4, base + 1, base + 0, base + 5
    if materials == 'shapes':
        return _cornell_shapes(width, height, spp, rfilter, max_depth)
    green_b, red_b, flip_back = 2, 1, False
    if materials == 'smooth':
        # the back wall shows its back side (flipped normals) through twosided
        base = len(bsdfs)
        bsdfs += smooth_materials()
        floor_b, short_b, tall_b, back_b, green_b, flip_back = base + 3, base + 0, base + 1, base + 5, base + 4, True
        red_b = base + 8
    uv = materials in ('rough', 'plastic', 'smooth')   # UV tangents (anisotropic BSDFs) and texture coordinates
    for quad, b in ((_FLOOR, floor_b), (_CEIL, 0), (_BACK, back_b), (_GREEN, green_b), (_RED, red_b)):
        m = _quads_mesh([quad], inward=True, uv=uv)
        meshes.append(Mesh(m[0], m[1], texcoords=m[2] if uv else None, bsdf=b,
                           flipNormals=flip_back and quad is _BACK))
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


def _cornell_shapes(width, height, spp, rfilter, max_depth):
    """The Cornell room with analytic shapes (rectangle.cpp, disk.cpp, sphere.cpp):
    a rectangle area light in place of the light quad, a gold sphere and a glass
    sphere in place of the blocks, a small emitting sphere (cone sampling), a
    disk on the floor and a flipped, twosided mirror rectangle on the green wall."""
    sc, integ = cornell_box(width, height, spp, rfilter, max_depth)
    walls = sc.meshes[:5]
    bsdfs = sc.bsdfs + [
        BSDF('roughconductor', distribution='ggx', alpha=0.15, material='Au'),
        BSDF('dielectric', intIOR=1.5),
        BSDF('diffuse', reflectance=(0.2, 0.6, 0.8)),
        BSDF('twosided', nested=[BSDF('conductor', material='none', specularReflectance=0.9)]),
    ]
    gold, glass, blue, mirror = 3, 4, 5, 6
    T = Transform
    light = T().scale(65 * S, 52.5 * S, 1).rotate((1, 0, 0), 90).translate(278 * S, 548.7 * S, 279.5 * S)
    disk = T().scale(0.6).rotate((1, 0, 0), -90).translate(450 * S, 1 * S, 120 * S)
    mir = T().scale(1.2, 1.0, 1).rotate((0, 1, 0), 90).translate(1 * S, 2.5, 3.2)
    meshes = walls + [
        Mesh(shape='rectangle', toWorld=light, bsdf=-1, emitter=0),
        Mesh(shape='sphere', center=(370 * S, 90 * S, 350 * S), radius=0.9, bsdf=gold),
        Mesh(shape='sphere', center=(185 * S, 80 * S, 170 * S), radius=0.8, bsdf=glass),
        Mesh(shape='sphere', toWorld=T().scale(0.3).translate(1.5, 4.0, 4.0), bsdf=-1, emitter=1),
        Mesh(shape='disk', toWorld=disk, bsdf=blue),
        Mesh(shape='rectangle', toWorld=mir, flipNormals=True, bsdf=mirror),
    ]
    emitters = [Emitter('area', radiance=(17.0, 12.0, 4.0)), Emitter('area', radiance=(4.0, 4.0, 8.0))]
    return Scene(sc.sensor, meshes, bsdfs, emitters, name='cornell-shapes'), integ


def procedural_envmap(width=1024, height=512, seed=0x5EED):
    """Deterministic lat-long sky (the 'procedural 1024x512 PFM envmap' of BASELINE.md C3):
    elevation gradient, warm horizon, dark ground, a small bright sun and three
    rectangular soft boxes, with mild multiplicative noise.  (H, W, 3) float32."""
    rng = np.random.default_rng(seed)
    v = (np.arange(height, dtype=np.float64) + 0.5) / height          # 0 = zenith (envmap.cpp:384-388)
    u = (np.arange(width, dtype=np.float64) + 0.5) / width
    theta = v * np.pi
    phi = u * 2 * np.pi
    elev = (np.pi / 2 - theta)[:, None] * np.ones((1, width))
    t = np.clip(elev / (np.pi / 2), -1, 1)
    sky = np.where(t[..., None] >= 0,
                   (1 - t[..., None]) * np.array([1.2, 1.05, 0.9]) + t[..., None] * np.array([0.25, 0.45, 1.0]),
                   np.array([0.18, 0.16, 0.13]) * (1 + 0.5 * t[..., None]))
    # sun: 3 degree disk at elevation 35, azimuth 60 (radiance 400)
    sd = np.array([np.cos(np.radians(35)) * np.sin(np.radians(60)), np.sin(np.radians(35)),
                   -np.cos(np.radians(35)) * np.cos(np.radians(60))])
    st, sp = np.sin(theta)[:, None], phi[None, :]
    dirs = np.stack([np.sin(sp) * st, np.cos(theta)[:, None] * np.ones_like(sp), -np.cos(sp) * st], -1)
    cosang = dirs @ sd
    sky = sky + (cosang > np.cos(np.radians(3.0)))[..., None] * np.array([400.0, 380.0, 330.0])
    # soft boxes
    for (u0, u1, v0, v1, rad) in ((0.05, 0.12, 0.30, 0.40, 12.0), (0.55, 0.70, 0.20, 0.28, 8.0),
                                  (0.80, 0.84, 0.35, 0.47, 15.0)):
        uu, vv = u[None, :], v[:, None]
        box = (uu >= u0) & (uu < u1) & (vv >= v0) & (vv < v1)
        sky = sky + box[..., None] * rad
    sky = sky * rng.uniform(0.9, 1.1, size=(height, width, 1))
    return sky.astype(np.float32)


def blob_mesh(nu=236, nv=148, radius=1.0, center=(0.0, 1.0, 0.0), uv=False):
    """Procedural stand-in for data/tests/bunny.ply (~69k triangles, closed,
    smooth vertex normals left to computeNormals): a displaced UV sphere.
    uv=True also returns spherical texture coordinates (u = phi / 2pi, v = theta / pi)."""
    th = np.linspace(0, np.pi, nv)
    ph = np.linspace(0, 2 * np.pi, nu, endpoint=False)
    T, P = np.meshgrid(th, ph, indexing='ij')
    r = radius * (1 + 0.12 * np.sin(5 * T) * np.sin(4 * P) + 0.05 * np.cos(9 * P + 3 * T))
    pos = np.stack([r * np.sin(T) * np.cos(P), r * np.cos(T), r * np.sin(T) * np.sin(P)], -1).reshape(-1, 3)
    pos = (pos + np.asarray(center)).astype(np.float32)
    idx = []
    for i in range(nv - 1):
        for j in range(nu):
            a, b = i * nu + j, i * nu + (j + 1) % nu
            c, d = (i + 1) * nu + j, (i + 1) * nu + (j + 1) % nu
            if i > 0:
                idx.append((a, b, d))
            if i < nv - 2:
                idx.append((a, d, c))
    if uv:
        tc = np.stack([(P / (2 * np.pi)), T / np.pi], -1).reshape(-1, 2).astype(np.float32)
        return pos, np.asarray(idx, np.uint32), tc
    return pos, np.asarray(idx, np.uint32)


def matpreview(width=1280, height=720, spp=512, rfilter='box', max_depth=-1, env_size=(1024, 512),
               blob=(236, 148), area_light=False, env_weight=1.0, plastic=False, object_mesh=None):
    """Config C3: a ~69k-triangle object in roughconductor GGX alpha=0.1 (copper) on a
    diffuse checker ground, lit only by a 1024x512 environment map.
    plastic=True is config C5: the object in roughplastic GGX whose roughness is a
    checkerboard texture over spherical UVs (alpha 0.05 / 0.3), so every shading
    point interpolates the 2D (alpha x theta) rough-transmittance slice.
    object_mesh: a Mesh (e.g. Mitsuba's data/tests/bunny.ply through ply.load_ply,
    already in world space) in place of the procedural object."""
    if plastic:
        obj = BSDF('roughplastic', distribution='ggx', diffuseReflectance=(0.2, 0.35, 0.6),
                   alpha=Checkerboard(color0=0.05, color1=0.3, uscale=8.0, vscale=4.0))
    else:
        obj = BSDF('roughconductor', distribution='ggx', alpha=0.1, material='Cu')
    g0 = BSDF('diffuse', reflectance=(0.4, 0.4, 0.4))
    g1 = BSDF('diffuse', reflectance=(0.15, 0.15, 0.15))
    bsdfs = [obj, g0, g1]
    meshes = []
    if object_mesh is not None:
        object_mesh.bsdf = 0
        meshes.append(object_mesh)
    elif plastic:
        p, i, tc = blob_mesh(*blob, uv=True)
        meshes.append(Mesh(p, i, texcoords=tc, bsdf=0, name='object'))
    else:
        p, i = blob_mesh(*blob)
        meshes.append(Mesh(p, i, bsdf=0, name='object'))
    # 12x12 checker of quads, y = 0 (two meshes, one per colour)
    n, half = 12, 6.0
    for col in (0, 1):
        pos, idx = [], []
        for a in range(n):
            for b in range(n):
                if (a + b) % 2 != col:
                    continue
                x0, z0 = -half + a * (2 * half / n), -half + b * (2 * half / n)
                x1, z1 = x0 + 2 * half / n, z0 + 2 * half / n
                base = len(pos)
                pos += [(x0, 0, z0), (x0, 0, z1), (x1, 0, z1), (x1, 0, z0)]
                idx += [(base, base + 1, base + 2), (base, base + 2, base + 3)]
        meshes.append(Mesh(np.asarray(pos, np.float32), np.asarray(idx, np.uint32), bsdf=1 + col,
                           faceNormals=True, name='ground%d' % col))
    env = Emitter('envmap', bitmap=procedural_envmap(*env_size), scale=1.0, samplingWeight=env_weight,
                  toWorld=Transform().rotate((0, 1, 0), 30.0))
    emitters = [env]
    if area_light:   # parity coverage: an area light next to the environment (emitter PDF over both)
        meshes.append(Mesh(np.array([(-1, 3.5, -1), (1, 3.5, -1), (1, 3.5, 1), (-1, 3.5, 1)], np.float32),
                           np.array([(0, 1, 2), (0, 2, 3)], np.uint32), emitter=1, faceNormals=True, name='lamp'))
        emitters.append(Emitter('area', radiance=(6.0, 6.0, 5.0)))
    cam = Transform.look_at_((0.0, 2.6, 7.6), (0.0, 0.9, 0.0), (0, 1, 0)).m
    sensor = Sensor(fov=35.0, fovAxis='x', nearClip=0.01, farClip=100.0, toWorld=cam, width=width, height=height)
    scene = Scene(sensor, meshes, bsdfs, emitters, name='matpreview')
    integ = PathIntegrator(maxDepth=max_depth, rrDepth=5, sampleCount=spp, rfilter=rfilter, rfilterParam=0.5)
    return scene, integ


def _box_mesh(lo, hi, n=1, inward=False):
    """Axis-aligned box, each face an n x n grid of quads (2n^2 triangles per face)."""
    lo, hi = np.asarray(lo, np.float64), np.asarray(hi, np.float64)
    pos, idx = [], []
    for axis in range(3):
        for side in (0, 1):
            u, v = [a for a in range(3) if a != axis]
            base = len(pos)
            for i in range(n + 1):
                for j in range(n + 1):
                    p = np.empty(3)
                    p[axis] = hi[axis] if side else lo[axis]
                    p[u] = lo[u] + (hi[u] - lo[u]) * i / n
                    p[v] = lo[v] + (hi[v] - lo[v]) * j / n
                    pos.append(p)
            outward_sign = 1 if side else -1
            # (u, v, axis) right-handed? orient so the normal points outward (or inward)
            flip = (np.cross(np.eye(3)[u], np.eye(3)[v])[axis] * outward_sign < 0) != inward
            for i in range(n):
                for j in range(n):
                    a, b = base + i * (n + 1) + j, base + (i + 1) * (n + 1) + j
                    c, d = b + 1, a + 1
                    tris = [(a, b, c), (a, c, d)]
                    if flip:
                        tris = [(a, c, b), (a, d, c)]
                    idx += tris
    return np.asarray(pos, np.float32), np.asarray(idx, np.uint32)


def _column_mesh(cx, cz, radius, height, seg, rings, rng):
    """Fluted column: a cylinder with a sinusoidal flute profile, capped top and bottom."""
    th = np.linspace(0, 2 * np.pi, seg, endpoint=False)
    ys = np.linspace(0.0, height, rings + 1)
    flute = 1 + 0.06 * np.cos(16 * th + rng.uniform(0, 2 * np.pi))
    pos = []
    for y in ys:
        taper = 1 - 0.12 * y / height
        for t, f in zip(th, flute):
            r = radius * f * taper
            pos.append((cx + r * np.cos(t), y, cz + r * np.sin(t)))
    idx = []
    for k in range(rings):
        for i in range(seg):
            a, b = k * seg + i, k * seg + (i + 1) % seg
            c, d = a + seg, b + seg
            idx += [(a, c, d), (a, d, b)]
    # caps (fans around a centre vertex)
    for y, top in ((0.0, False), (height, True)):
        ci = len(pos)
        pos.append((cx, y, cz))
        ring0 = rings * seg if top else 0
        for i in range(seg):
            a, b = ring0 + i, ring0 + (i + 1) % seg
            idx.append((ci, b, a) if top else (ci, a, b))
    return np.asarray(pos, np.float32), np.asarray(idx, np.uint32)


def atrium(width=1280, height=720, spp=256, rfilter='box', max_depth=-1, columns=(4, 6), seg=96, rings=40,
           seed=0x5EED):
    """Config C4: procedural ~200k-triangle atrium -- a hall with 24 fluted columns,
    tiled floor, four ceiling lights; roughdielectric GGX alpha=0.2 eta=1.5 on ~30%
    of the meshes, diffuse elsewhere."""
    rng = np.random.default_rng(seed)
    glass = BSDF('roughdielectric', distribution='ggx', alpha=0.2, intIOR=1.5, extIOR=1.0)
    bsdfs = [BSDF('diffuse', reflectance=(0.7, 0.68, 0.62)),     # 0 walls
             BSDF('diffuse', reflectance=(0.35, 0.3, 0.25)),     # 1 floor
             glass]                                              # 2
    meshes, emitters = [], []
    W, D, H = 16.0, 28.0, 9.0
    p, i = _box_mesh((-W / 2, 0, -D / 2), (W / 2, H, D / 2), n=12, inward=True)
    meshes.append(Mesh(p, i, bsdf=0, faceNormals=True, name='hall'))
    p, i = _box_mesh((-W / 2 + 0.2, 0.0, -D / 2 + 0.2), (W / 2 - 0.2, 0.05, D / 2 - 0.2), n=20)
    meshes.append(Mesh(p, i, bsdf=1, faceNormals=True, name='floor'))
    nx, nz = columns
    k = 0
    for a in range(nx):
        for b in range(nz):
            cx = -W / 2 + (a + 0.5) * W / nx
            cz = -D / 2 + (b + 0.5) * D / nz
            if abs(cx) < 1.0 and cz > 4:
                cz += 0.0
            c = rng.uniform(0.2, 0.8, 3)
            if rng.random() < 0.3:
                bi = 2
            else:
                bsdfs.append(BSDF('diffuse', reflectance=tuple(float(x) for x in c)))
                bi = len(bsdfs) - 1
            p, i = _column_mesh(cx, cz, 0.45, H - 0.5, seg, rings, rng)
            meshes.append(Mesh(p, i, bsdf=bi, name='column%d' % k))
            k += 1
    for lx, lz in ((-3.5, -7), (3.5, -7), (-3.5, 7), (3.5, 7)):
        q = np.array([(lx - 1, H - 0.01, lz - 1.5), (lx + 1, H - 0.01, lz - 1.5), (lx + 1, H - 0.01, lz + 1.5),
                      (lx - 1, H - 0.01, lz + 1.5)], np.float32)
        meshes.append(Mesh(q, np.array([(0, 1, 2), (0, 2, 3)], np.uint32), emitter=len(emitters),
                           faceNormals=True, name='light'))
        emitters.append(Emitter('area', radiance=(14.0, 13.0, 11.0)))
    cam = Transform.look_at_((0.0, 3.2, -13.0), (0.0, 3.0, 4.0), (0, 1, 0)).m
    sensor = Sensor(fov=60.0, fovAxis='x', nearClip=0.01, farClip=100.0, toWorld=cam, width=width, height=height)
    scene = Scene(sensor, meshes, bsdfs, emitters, name='atrium')
    integ = PathIntegrator(maxDepth=max_depth, rrDepth=5, sampleCount=spp, rfilter=rfilter, rfilterParam=0.5)
    return scene, integ


CONFIGS = {
    'C1': dict(builder='cornell_box', width=512, height=512, spp=64),
    'C2': dict(builder='cornell_box', width=1280, height=720, spp=512),
    'C3': dict(builder='matpreview', width=1280, height=720, spp=512),
    'C4': dict(builder='atrium', width=1280, height=720, spp=256),
    'C5': dict(builder='matpreview', width=1280, height=720, spp=1024, plastic=True),
}


def build(config, **overrides):
    c = dict(CONFIGS[config])
    c.update(overrides)
    builder = globals()[c.pop('builder')]
    return builder(**c)
