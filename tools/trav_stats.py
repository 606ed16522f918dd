#!/usr/bin/env python3
"""Traversal statistics of one frame slice (INSTR kernel): rays, shadow rays,
node visits and triangle tests per ray, path length; usage: trav_stats.py C3 [stride]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()
from mitsuba_amd import scenes  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402

for cfg in sys.argv[1].split(','):
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    sc, it = scenes.build(cfg)
    ctx = Context(0)
    ctx.upload(sc)
    _, _, st = ctx.render(it, row=(8, stride, 0), traversal_stats=True)
    rays = st['rays'] + st['shadow_rays']
    print('%s info %s' % (cfg, ctx.scene_info()))
    print('%s samples %d rays/sample %.2f shadow/sample %.2f nodes/ray %.1f tests/ray %.1f pathlen %.2f' % (
        cfg, st['samples'], st['rays'] / st['samples'], st['shadow_rays'] / st['samples'],
        st['node_visits'] / rays, st['tri_tests'] / rays, st['path_length_sum'] / st['samples']))
