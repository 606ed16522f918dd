#!/usr/bin/env python3
"""C4's diverging sample (pixel 1215, row 299, j 176; tests/test_gpu_bench_kernels.py):
its last closest-hit ray, which the oracle answers with prim 4445 at t = 0.0693
(ORACLE_TRACE=1215,299,176), through the GPU's batch query (full-precision
BVH nodes) and the kd traversal, and the sample's row rendered by the BSDF-set
kernel (half-float node boxes) and by the generic kernel (MTSGPU_NO_BSDF_SETS=1)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
sc, it = bench.build_scene('C4')
import oracle.binding as ob  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402

f = float.fromhex
o = np.array([[f('-0x1.2114dp+1'), 0.0, f('0x1.652fc6p+3')]], np.float32)
d = np.array([[f('0x1.873b5p-3'), f('0x1.718456p-1'), f('0x1.54a38ep-1')]], np.float32)
eps = np.float32(f('0x1.a36e2ep-14'))
ctx = Context(0)
ctx.upload(sc)
print('oracle ', ob.trace_rays(sc, o, d, mint=eps)[0].tolist(), 'prim bits', ob.trace_rays(sc, o, d, mint=eps)[:, 3].view(np.uint32))
hg, _ = ctx.trace_rays(o, d, mint=eps)
print('gpu bvh', hg[0].tolist(), 'prim bits', hg[:, 3].view(np.uint32))
hk, _ = ctx.trace_rays(o, d, mint=eps, kdtree=True)
print('gpu kd ', hk[0].tolist(), 'prim bits', hk[:, 3].view(np.uint32))
win = (0, 299, 1280, 1)
_, so, sto = ob.render(sc, it, window=win, samples=True, libm_mode=0, threads=16)
for env in (None, '1'):
    if env:
        os.environ['MTSGPU_NO_BSDF_SETS'] = env
    _, sg, stg = ctx.render(it, window=win, samples=True)
    bad = np.nonzero(np.any(sg.view(np.uint32) != so.view(np.uint32), axis=1))[0]
    print('render', ctx.kernel_variant()['name'], 'rays', stg['rays'], 'oracle', sto['rays'], 'differing records', bad.tolist()[:10])
    for e in ('wavefront', 'kdtree'):
        _, sw, stw = ctx.render(it, window=win, samples=True, engine=e)
        badw = np.nonzero(np.any(sw.view(np.uint32) != so.view(np.uint32), axis=1))[0]
        print('  engine', e, 'rays', stw['rays'], 'differing records', badw.tolist()[:10])
