#!/usr/bin/env python3
"""Diagnostics: which shadow rays does direct_kernel's inlined any-hit query get wrong?

  anyhit_xc.py render LIB > xc.log   renders diag_parity's `direct_shapes` case with a
                                     library built with -DMTSG_ANYHIT_CROSSCHECK: every
                                     shadow ray is answered by the inlined any-hit
                                     traversal and by the __noinline__ call, and each
                                     disagreement is printed (bit patterns of o, d, dist
                                     and the clipped [mint, maxt]) as an `XC` line;
                                     -DMTSG_ANYHIT_XC_SLOT adds the test that accepted
                                     the ray (which perturbs the code generated).
  anyhit_xc.py check xc.log          replays those rays through the oracle's occlusion
                                     test and closest hit, and through trace_kernel's
                                     any-hit and closest-hit queries (the same
                                     traverse<ANY> inlined into another kernel).
"""
import os
import re
import struct
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()
from mitsuba_amd import scenes  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402
from mitsuba_amd.scene import DirectIntegrator  # noqa: E402
import oracle.binding as ob  # noqa: E402

XC = re.compile(r'XC (\d+) inl (\d) call (\d) o (\w+) (\w+) (\w+) d (\w+) (\w+) (\w+) dist (\w+) mint (\w+) maxt (\w+) lane \d+ slot (\w+) a (\S+) (\S+) (\S+)')


def scene():
    sc, _ = scenes.build('C1', width=32, height=32, spp=4, materials='shapes')
    return sc, DirectIntegrator(sampleCount=4, rfilter='box', emitterSamples=2, bsdfSamples=2)


def f(h):
    return struct.unpack('<f', struct.pack('<I', int(h, 16)))[0]


def main():
    mode, arg = sys.argv[1], sys.argv[2]
    sc, it = scene()
    if mode == 'render':
        c = Context(0, lib_path=arg)
        c.upload(sc)
        c.render(it, samples=True)
        sys.stdout.flush()
        return
    rows = [XC.search(l) for l in open(arg)]
    rows = [m for m in rows if m]
    if not rows:
        print('no XC lines')
        return
    inl = np.array([int(m.group(2)) for m in rows])
    call = np.array([int(m.group(3)) for m in rows])
    v = np.array([[f(m.group(k)) for k in range(4, 13)] for m in rows], np.float32)
    o, d, dist = v[:, 0:3], v[:, 3:6], v[:, 6]
    mint = np.float32(1e-4)
    maxt = (dist * np.float32(1 - 1e-3)).astype(np.float32)   # Ray(ref, d, Epsilon, dist*(1-ShadowEpsilon))
    occ_o = ob.trace_rays(sc, o, d, mint, maxt, shadow=True)[:, 0]
    hit_o = ob.trace_rays(sc, o, d, mint, maxt, shadow=False)
    c = Context(0)
    c.upload(sc)
    occ_g = c.trace_rays(o, d, mint, maxt, shadow=True)[0][:, 0]
    hit_g = c.trace_rays(o, d, mint, maxt, shadow=False)[0]
    print('%d disagreements (inlined vs call) in direct_kernel' % len(rows))
    print('inlined answer == oracle: %d, call answer == oracle: %d, trace_kernel any-hit == oracle: %d' % (
        int((inl == occ_o).sum()), int((call == occ_o).sum()), int((occ_g == occ_o).sum())))
    for k in range(len(rows)):
        slot = int(rows[k].group(13), 16)
        kind = 'none' if slot == 0xffffffff else ('analytic' if slot & 0x80000000 else 'triangle')
        if slot != 0xffffffff:   # -DMTSG_ANYHIT_XC_SLOT builds report the accepting test
          print('  accepted by %s slot %d: %s %s %s (triangle: t u v; analytic: nearT farT maxt)' % (
              kind, slot & 0x7fffffff, rows[k].group(14), rows[k].group(15), rows[k].group(16)))
        prim = struct.unpack('<I', struct.pack('<f', hit_o[k, 3]))[0]
        print('  inl %d call %d oracle %d trace_kernel %d | closest t %.9g prim %d (gpu t %.9g) maxt %.9g | '
              'clipped [%.9g, %.9g]' % (inl[k], call[k], int(occ_o[k]), int(occ_g[k]), hit_o[k, 0],
                                       prim if prim != 0xffffffff else -1, hit_g[k, 0], maxt[k], v[k, 7], v[k, 8]))


if __name__ == '__main__':
    main()
