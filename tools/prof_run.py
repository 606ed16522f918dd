#!/usr/bin/env python3
"""Profiling driver: renders a config through libmtsgpu (no torch) for rocprofv3.
usage: prof_run.py [config] [frames] [rows_stride] [engine]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()
from mitsuba_amd import scenes  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'C2'
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 1
stride = int(sys.argv[3]) if len(sys.argv) > 3 else 1
engine = sys.argv[4] if len(sys.argv) > 4 else None
# C2g: C2 with the gaussian filter (bench.py's secondary block)
sc, it = scenes.build(cfg.rstrip('g'), rfilter='gaussian' if cfg.endswith('g') else 'box')
ctx = Context(0, lib_path=os.environ.get('PROF_LIB'))   # PROF_LIB: a variant build (A/B traffic passes)
ctx.upload(sc)
print('scene', ctx.scene_info())
for f in range(frames):
    _, _, st = ctx.render(it, row=(8, stride, 0), engine=engine)
    print('frame', f, 'kernel_ms %.2f' % st['kernel_ms'], 'Msamples/s %.1f' % (st['samples'] / st['kernel_ms'] / 1e3))
