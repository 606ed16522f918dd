#!/usr/bin/env python3
"""Diagnostics for the direct integrator's any-hit shadow rays: a variant
library (built with -DMTSG_DIRECT_ANYHIT_DEBUG) runs both traversals on every
shadow ray and stores the first ray per sample where they disagree in the
sample record; those rays are then replayed through mtsgpu_trace_rays and
the oracle."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from pkgimport import mitsuba_amd  # noqa: E402

mitsuba_amd()
from mitsuba_amd import scenes  # noqa: E402
from mitsuba_amd.integrator import Context  # noqa: E402
from mitsuba_amd.scene import DirectIntegrator  # noqa: E402
import oracle.binding as ob  # noqa: E402

dbg_lib = sys.argv[1]
sc, _ = scenes.build('C1', width=32, height=32, spp=4, materials='shapes')
d = DirectIntegrator(sampleCount=4, rfilter='box', emitterSamples=2, bsdfSamples=2)
cd = Context(0, lib_path=dbg_lib)
cd.upload(sc)
_, smp, _ = cd.render(d, samples=True)
rays = smp[smp[:, 6] != 1.0]
print('disagreeing shadow rays (first per sample):', len(rays), 'of', len(smp), 'samples')
if len(rays):
    o, dd, mint, maxt = rays[:, 0:3], rays[:, 3:6], rays[:, 6], rays[:, 7]
    base = Context(0)
    base.upload(sc)
    for k in range(min(8, len(rays))):
        print('  o=%s d=%s mint=%r maxt=%r' % (o[k].tolist(), dd[k].tolist(), float(mint[k]), float(maxt[k])))
    for shadow in (True, False):
        hits = np.stack([base.trace_rays(o[k:k + 1], dd[k:k + 1], mint=float(mint[k]), maxt=float(maxt[k]),
                                         shadow=shadow)[0][0] for k in range(len(rays))])
        ho = np.stack([ob.trace_rays(sc, o[k:k + 1], dd[k:k + 1], mint=float(mint[k]), maxt=float(maxt[k]),
                                     shadow=shadow)[0] for k in range(len(rays))])
        print('trace_rays shadow=%s: gpu %s | oracle %s' % (shadow, hits[:8].tolist(), ho[:8].tolist()))
        if shadow:
            print('  gpu occluded: %d / %d, oracle occluded: %d' % ((hits[:, 0] > 0).sum(), len(hits), (ho[:, 0] > 0).sum()))
        else:
            print('  gpu hit: %d, oracle hit: %d, prims %s' % ((hits[:, 3].view(np.uint32) != 0xffffffff).sum(),
                  (ho[:, 3].view(np.uint32) != 0xffffffff).sum(), np.unique(ho[:, 3].view(np.uint32)).tolist()))
