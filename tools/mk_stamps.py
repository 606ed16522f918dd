#!/usr/bin/env python3
"""Section shares of the megakernel from a -DMTSG_MK_STAMPS build (diagnostic:
wave cycles per section summed over waves; read shares, not times).
usage: mk_stamps.py <lib.so> <config>[,config...] [rows_stride]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()
from mitsuba_amd import scenes  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402

lib, cfgs = sys.argv[1], sys.argv[2].split(',')
stride = int(sys.argv[3]) if len(sys.argv) > 3 else 4
names = ['start', 'shadow trace', 'closest trace', 'shade']
for cfg in cfgs:
    sc, it = scenes.build(cfg, rfilter='box')
    ctx = Context(0, lib_path=lib)
    ctx.upload(sc)
    _, _, st = ctx.render(it, row=(8, stride, 0), engine='megakernel')
    c = ctx.debug_counters()
    tot = sum(c[11:15]) or 1
    print('%s: %.1f ms, %s' % (cfg, st['kernel_ms'], ', '.join('%s %.1f%%' % (n, 100.0 * v / tot)
                                                              for n, v in zip(names, c[11:15]))))
