#!/usr/bin/env python3
"""Diagnostics: per-sample GPU-vs-oracle mismatch census for the parity scenes.

For every scene of tests/test_gpu_parity.py that is not yet asserted bit-exact,
print how many per-sample records differ, and for the first few: pixel, sample
index, both records and the max ulp distance per field.  Optional variant
libraries (name=path) are run on the same scenes.
usage: diag_parity.py [--only=case,case] [name=lib.so ...]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()
from mitsuba_amd import scenes  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402
from mitsuba_amd.scene import BSDF, DirectIntegrator, Emitter, Mesh, PathIntegrator, VolpathIntegrator  # noqa: E402
from mitsuba_amd.transform import Transform  # noqa: E402
import oracle.binding as ob  # noqa: E402


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.int32)


def c3_small(**kw):
    return scenes.build('C3', width=kw.pop('width', 40), height=kw.pop('height', 24), spp=kw.pop('spp', 8),
                        env_size=kw.pop('env_size', (128, 64)), blob=kw.pop('blob', (48, 30)), **kw)


def cases():
    from mitsuba_amd.scenes import rough_materials, smooth_materials
    for mi in range(len(rough_materials())):
        sc, it = scenes.build('C1', width=24, height=24, spp=8, materials='rough')
        sc.meshes[6].bsdf = 3 + mi
        yield 'rough_mat%d' % mi, sc, it
    for kw, hide in (({'area_light': True, 'env_weight': 2.0}, False), ({'env_size': (100, 37)}, False), ({}, True)):
        sc, it = c3_small(**kw)
        it.hideEmitters = hide
        yield 'env_%s_%s' % ('_'.join(kw) or 'plain', hide), sc, it
    for mi in range(len(smooth_materials())):
        sc, it = scenes.build('C1', width=24, height=24, spp=8, materials='smooth')
        sc.meshes[6].bsdf = 3 + mi
        yield 'smooth_mat%d' % mi, sc, it
    sc, it = c3_small()
    sc.bsdfs.append(BSDF('plastic', diffuseReflectance=(0.7, 0.2, 0.2)))
    b = len(sc.bsdfs) - 1
    sc.meshes.append(Mesh(shape='sphere', center=(1.6, 0.6, 0.4), radius=0.6, bsdf=b))
    sc.meshes.append(Mesh(shape='disk', toWorld=Transform().scale(0.8).rotate((1, 0, 0), -90).translate(-1.5, 0.01, 0.5),
                          bsdf=b))
    yield 'shapes_under_env', sc, it
    for materials in ('rough', 'shapes'):
        sc, _ = scenes.build('C1', width=40, height=32, spp=8, materials=materials)
        yield 'indep_path_' + materials, sc, PathIntegrator(sampleCount=8, rfilter='box', sampler='independent')
        yield 'indep_direct_' + materials, sc, DirectIntegrator(sampleCount=8, rfilter='box', sampler='independent',
                                                               emitterSamples=3, bsdfSamples=2)
    for name, (sc, _) in (('env', c3_small(area_light=True)),
                          ('shapes', scenes.build('C1', width=32, height=32, spp=8, materials='shapes'))):
        yield 'volpath_' + name, sc, VolpathIntegrator(sampleCount=8, rfilter='box', strictNormals=True)
    for name, (sc, _) in (('env', c3_small(area_light=True)),
                          ('shapes', scenes.build('C1', width=32, height=32, spp=4, materials='shapes'))):
        yield 'direct_' + name, sc, DirectIntegrator(sampleCount=4, rfilter='box', emitterSamples=2, bsdfSamples=2)


def report(name, sc, it, smp_g, smp_o):
    bg, bo = bits(smp_g), bits(smp_o)
    same = np.all(bg == bo, axis=1)
    n = int((~same).sum())
    print('%-28s %6d / %6d differ' % (name, n, same.size), flush=True)
    if n:
        spp = it.sampleCount
        W = sc.sensor.width
        for r in np.nonzero(~same)[0][:4]:
            pix, j = divmod(int(r), spp)
            ulp = np.abs(bg[r].astype(np.int64) - bo[r].astype(np.int64))
            print('    px=(%d,%d) j=%d ulp=%s\n      gpu=%s\n      ora=%s' % (
                pix % W, pix // W, j, ulp.tolist(), smp_g[r].tolist(), smp_o[r].tolist()), flush=True)
        # ulp histogram of the Li fields of differing records
        d = np.abs(bg[~same, :3].astype(np.int64) - bo[~same, :3].astype(np.int64)).max(1)
        print('    max-ulp(Li) histogram: <=1: %d, <=16: %d, >16: %d; depth differs: %d' % (
            (d <= 1).sum(), ((d > 1) & (d <= 16)).sum(), (d > 16).sum(),
            int((smp_g[~same, 6] != smp_o[~same, 6]).sum())), flush=True)
    return n


def main():
    only = [a.split('=', 1)[1].split(',') for a in sys.argv[1:] if a.startswith('--only=')]
    only = only[0] if only else None
    variants = [('base', None)] + [tuple(a.split('=', 1)) for a in sys.argv[1:] if not a.startswith('--')]
    ctxs = {n: Context(0, lib_path=p) for n, p in variants}
    total = {n: 0 for n, _ in variants}
    for name, sc, it in cases():
        if only and name not in only:
            continue
        _, smp_o, _ = ob.render(sc, it, samples=True, libm_mode=0, threads=8)
        for vn, _ in variants:
            c = ctxs[vn]
            c.upload(sc)
            _, smp_g, _ = c.render(it, samples=True)
            total[vn] += report('%s[%s]' % (name, vn), sc, it, smp_g, smp_o)
    print('TOTAL differing records:', total)


if __name__ == '__main__':
    main()
