#!/usr/bin/env python3
"""Throughput of the batch ray query kernel (mtsgpu_trace_rays): incoherent
random rays inside the scene bounds, closest hit and occlusion; compare with
the path kernel's effective ray rate.  usage: trace_bench.py C3[,C4] [n]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()
from mitsuba_amd import scenes  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402

n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 23
for cfg in sys.argv[1].split(','):
    sc, _ = scenes.build(cfg)
    ctx = Context(0)
    ctx.upload(sc)
    rng = np.random.default_rng(1)
    lo = np.min([m.positions.min(0) for m in sc.meshes], 0)
    hi = np.max([m.positions.max(0) for m in sc.meshes], 0)
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    for shadow in (False, True):
        ctx.trace_rays(o[:65536], d[:65536], shadow=shadow)
        best = min(ctx.trace_rays(o, d, maxt=np.inf, shadow=shadow)[1] for _ in range(3))
        print('%s %s: %.0f Mrays/s (%d rays, %.2f ms)' % (cfg, 'shadow ' if shadow else 'closest', n / best / 1e3, n, best))
