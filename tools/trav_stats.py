#!/usr/bin/env python3
"""Traversal statistics per configuration: node visits and triangle tests per
traced ray (closest-hit and shadow rays together), rays per sample, from the
kernel's own counters (MTSGPU_FLAG_TRAVERSAL_STATS) over every <stride>-th
8-row band.  usage: trav_stats.py <stride> C3 C4 ..."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()
from mitsuba_amd import scenes  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402

stride = int(sys.argv[1])
for cfg in sys.argv[2:]:
    sc, it = scenes.build(cfg, rfilter='box')
    c = Context(0)
    c.upload(sc)
    info = c.scene_info() if hasattr(c, 'scene_info') else {}
    _, _, st = c.render(it, row=(8, stride, 0), traversal_stats=True)
    rays = st['rays'] + st['shadow_rays']
    print('%s: %s | samples %d, rays/sample %.2f (closest %.2f, shadow %.2f), nodes/ray %.1f, tri tests/ray %.1f, '
          'hits/sample %.2f' % (cfg, info, st['samples'], rays / st['samples'], st['rays'] / st['samples'],
                                st['shadow_rays'] / st['samples'], st['node_visits'] / max(1, rays),
                                st['tri_tests'] / max(1, rays), st['hits'] / st['samples']), flush=True)
