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


def full_frame_shift(cfg, pixels, spp, lanes=256 * 4 * 256):
    """The megakernel's sample-run length for the whole frame (capi.cpp run_shift): tiny
    LDS scenes 1; else the longest run <= 64 samples leaving every lane >= 100 runs.
    lanes: 256 CUs x 4 resident blocks of 256 (every benchmark kernel runs 4 waves/SIMD)."""
    if cfg in ('C1', 'C2', 'C2g'):
        return 1
    per_lane, s = pixels * spp // lanes, 6
    while s > 0 and ((1 << s) > spp or (per_lane >> s) < 100):
        s -= 1
    return s


# PROF_FULL_RUNS=1: a pass over a fraction of the rows keeps the full frame's run length
# (fewer samples per lane would otherwise pick shorter runs), so its per-sample counters
# describe the kernel bench.py times
if stride > 1 and os.environ.get('PROF_FULL_RUNS') == '1' and 'MTSGPU_ROUND_SHIFT' not in os.environ:
    os.environ['MTSGPU_ROUND_SHIFT'] = str(full_frame_shift(cfg, sc.sensor.width * sc.sensor.height, it.sampleCount))
    print('MTSGPU_ROUND_SHIFT', os.environ['MTSGPU_ROUND_SHIFT'])
ctx = Context(0, lib_path=os.environ.get('PROF_LIB'))   # PROF_LIB: a variant build (A/B traffic passes)
ctx.upload(sc)
print('scene', ctx.scene_info())
for f in range(frames):
    _, _, st = ctx.render(it, row=(8, stride, 0), engine=engine)
    print('frame', f, 'kernel_ms %.2f' % st['kernel_ms'], 'Msamples/s %.1f' % (st['samples'] / st['kernel_ms'] / 1e3))
