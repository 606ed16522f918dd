#!/usr/bin/env python3
"""Diagnose a mismatch between the uninstrumented megakernel (the one bench.py
times) and the oracle on a window: renders the window with records
(path_kernel<true,...>) and without (path_kernel<false,...>), each with and
without the 8x8 tile decomposition, and reports counters, record and film
differences against the oracle.
usage: diag_bench_kernel.py CFG Y0 H"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
bench.build_scene("C1", "8x8x1")   # puts the package on sys.path
import oracle.binding as ob  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402

cfg, y0, h = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
sc, it = bench.build_scene(cfg)
W = sc.sensor.width
win = (0, y0, W, h)
ctx = Context(0)
ctx.upload(sc)
bits = lambda a: np.ascontiguousarray(a, np.float32).view(np.uint32)
fo, so, sto = ob.render(sc, it, window=win, samples=True, libm_mode=0, threads=16)
print('oracle', {k: sto[k] for k in ('samples', 'rays', 'shadow_rays', 'path_length_sum')})
for tile in (False, True):
    row = (8, 1, 0)
    fi, si, sti = ctx.render(it, window=win, samples=True, row=row, tile_shard=tile)
    vi = ctx.kernel_variant()
    fu, _, stu = ctx.render(it, window=win, row=row, tile_shard=tile)
    vu = ctx.kernel_variant()
    bad = np.nonzero(np.any(bits(si) != bits(so), axis=1))[0]
    print('tile_shard=%s' % tile)
    print('  instr  ', vi['name'], {k: sti[k] for k in ('samples', 'rays', 'shadow_rays', 'path_length_sum')},
          'records differing:', bad.size)
    for i in bad[:8]:
        print('    rec', i, 'pixel', i // it.sampleCount, 'j', i % it.sampleCount, si[i].tolist(), so[i].tolist())
    print('  uninstr', vu['name'], {k: stu[k] for k in ('samples', 'rays', 'shadow_rays', 'path_length_sum')})
    for name, f in (('instr', fi), ('uninstr', fu)):
        d = np.argwhere(np.any(bits(f) != bits(fo), axis=-1))
        print('  film %s vs oracle: %d pixels differ' % (name, d.shape[0]), d[:6].tolist())
        for p in d[:4]:
            print('     ', tuple(p), f[tuple(p)].tolist(), fo[tuple(p)].tolist())
    d = np.argwhere(np.any(bits(fi) != bits(fu), axis=-1))
    print('  film instr vs uninstr: %d pixels differ' % d.shape[0], d[:6].tolist())
