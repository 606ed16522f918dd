#!/usr/bin/env python3
"""Film determinism across megakernel sample-run lengths (MTSGPU_ROUND_SHIFT):
renders CFG at 1/STRIDE rows twice per shift and reports, per pair of films, how
many pixels differ and by how much, split by whether the pixel's neighbour-splat
(spill) share is involved.
usage: diag_rounds.py CFG STRIDE SHIFT..."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()
from mitsuba_amd import scenes  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402

cfg, stride, shifts = sys.argv[1], int(sys.argv[2]), [int(s) for s in sys.argv[3:]]
sc, it = scenes.build(cfg.rstrip('g'), rfilter='gaussian' if cfg.endswith('g') else 'box')
ctx = Context(0)
ctx.upload(sc)
bits = lambda a: np.ascontiguousarray(a, np.float32).view(np.uint32)
films = {}
for s in shifts:
    os.environ['MTSGPU_ROUND_SHIFT'] = str(s)
    for rep in range(2):
        f, _, st = ctx.render(it, row=(8, stride, 0))
        films[(s, rep)] = f
        print('s%d rep%d' % (s, rep), {k: st[k] for k in ('samples', 'rays', 'shadow_rays', 'path_length_sum')},
              ctx.kernel_variant()['name'], flush=True)
keys = list(films)
ref = films[keys[0]]
for k in keys[1:]:
    f = films[k]
    d = np.any(bits(f) != bits(ref), axis=-1)
    n = int(d.sum())
    msg = 's%d rep%d vs s%d rep%d: %d pixels differ' % (k + keys[0] + (n,))
    if n:
        idx = np.argwhere(d)
        rel = np.max(np.abs(f[d] - ref[d]) / np.maximum(np.abs(ref[d]), 1e-30))
        msg += ', max rel diff %.3g, first %s' % (rel, idx[:4].tolist())
        p = tuple(idx[0])
        msg += ' %s vs %s' % (f[p].tolist(), ref[p].tolist())
    print(msg, flush=True)
