#!/usr/bin/env python3
"""Interleaved A/B timing of libmtsgpu variants in one process (guide rule 24).
usage: ab_variants.py <config> <rounds> <rows_stride> name=path ..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()
from mitsuba_amd import scenes  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402

cfg, rounds, stride = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
variants = [a.split('=', 1) for a in sys.argv[4:]]
sc, it = scenes.build(cfg, rfilter='box')
ctxs = {}
for name, path in variants:
    c = Context(0, lib_path=path)
    c.upload(sc)
    c.render(it, row=(8, stride, 0))   # warm up
    ctxs[name] = c
res = {n: [] for n, _ in variants}
for r in range(rounds):
    for name, _ in variants:
        _, _, st = ctxs[name].render(it, row=(8, stride, 0))
        res[name].append(st['samples'] / st['kernel_ms'] / 1e3)
for name, v in res.items():
    v = sorted(v)
    print('%-14s median %8.1f  min %8.1f  max %8.1f Msamples/s' % (name, v[len(v) // 2], v[0], v[-1]))
