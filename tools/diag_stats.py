"""Per-ray traversal statistics of each config (INSTR pass over 1/16 of the rows)."""
import sys
sys.path.insert(0, '.')
from pkgimport import mitsuba_amd
mitsuba_amd()
from mitsuba_amd import scenes
from mitsuba_amd.integrator import Context

ctx = Context()
for cfg in sys.argv[1:] or ['C2', 'C3', 'C4']:
    sc, it = scenes.build(cfg, rfilter='box')
    ctx.upload(sc)
    info = ctx.scene_info()
    _, _, st = ctx.render(it, row=(8, 16, 0), traversal_stats=True)
    _, _, st2 = ctx.render(it, row=(8, 16, 0))
    rays = st['rays'] + st['shadow_rays']
    print(cfg, info, 'samples', st['samples'], 'rays/sample %.2f shadow/sample %.2f' % (st['rays'] / st['samples'], st['shadow_rays'] / st['samples']),
          'nodes/ray %.1f tests/ray %.1f' % (st['node_visits'] / rays, st['tri_tests'] / rays),
          'pathlen %.2f' % (st['path_length_sum'] / st['samples']),
          'plain Msamples/s %.1f' % (st2['samples'] / st2['kernel_ms'] / 1e3), flush=True)
