#!/usr/bin/env python3
"""Interleaved A/B timing of libmtsgpu variants in one process (guide rule 24).
usage: ab_variants.py <config> <rounds> <rows_stride> name=path[,ENV=VAL...] ...
(environment overrides are applied around each variant's render calls;
AB_ENGINE=wavefront|megakernel|kdtree picks the engine of every variant, ENGINE=... in a
variant's list that variant's)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()
from mitsuba_amd import scenes  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402

cfg, rounds, stride = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
engine = os.environ.get('AB_ENGINE') or None
variants, envs = [], {}
for a in sys.argv[4:]:
    name, rest = a.split('=', 1)
    parts = rest.split(',')
    variants.append((name, parts[0]))
    envs[name] = dict(p.split('=', 1) for p in parts[1:])
engines = {n: envs[n].pop('ENGINE', engine) for n, _ in variants}   # per-variant engine: name=path,ENGINE=wavefront


def with_env(name, fn):
    saved = {k: os.environ.get(k) for k in envs[name]}
    os.environ.update(envs[name])
    try:
        return fn()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


sc, it = scenes.build(cfg.rstrip('g'), rfilter='gaussian' if cfg.endswith('g') else 'box')   # C2g: gaussian
ctxs = {}
for name, path in variants:
    c = Context(0, lib_path=path)
    with_env(name, lambda: c.upload(sc))
    with_env(name, lambda: c.render(it, row=(8, stride, 0), engine=engines[name]))   # warm up
    ctxs[name] = c
res = {n: [] for n, _ in variants}
films = {}
stats = {}
for r in range(rounds):
    for name, _ in variants:
        film, _, st = with_env(name, lambda: ctxs[name].render(it, row=(8, stride, 0), engine=engines[name]))
        films.setdefault(name, film)
        stats.setdefault(name, {k: st.get(k) for k in ('samples', 'rays', 'shadow_rays', 'path_length_sum', 'errors')})
        res[name].append(st['samples'] / st['kernel_ms'] / 1e3)
first = variants[0][0]
for name, v in res.items():
    v = sorted(v)
    same = films[name].tobytes() == films[first].tobytes()
    print('%-14s median %8.1f  min %8.1f  max %8.1f Msamples/s  film bit-identical to %s: %s  counters equal: %s' % (
        name, v[len(v) // 2], v[0], v[-1], first, same, stats[name] == stats[first]))
print('counters', stats[first])
