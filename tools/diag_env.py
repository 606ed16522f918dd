"""GPU diagnostic: mismatch pattern of the envmap scene vs the oracle."""
import sys
import numpy as np
sys.path.insert(0, '.')
from pkgimport import mitsuba_amd
mitsuba_amd()
from mitsuba_amd import scenes
from mitsuba_amd.integrator import Context
import oracle.binding as ob

ctx = Context()
prev = None
for kw in ({'md': -1}, {'md': -1}, {'md': 2}, {'md': 3}, {'md': -1, 'hide': True}, {'md': -1, 'rr': 1}):
    sc, it = scenes.build('C3', width=40, height=24, spp=8, env_size=(128, 64), blob=(48, 30))
    it.hideEmitters = kw.get('hide', False)
    it.maxDepth = kw['md']
    if 'rr' in kw:
        it.rrDepth = kw['rr']
    ctx.upload(sc)
    fg, sg, _ = ctx.render(it, samples=True)
    fo, so, _ = ob.render(sc, it, samples=True, libm_mode=0)
    bad = ~np.all(sg.view(np.uint32) == so.view(np.uint32), axis=1)
    print(kw, 'mismatch', bad.sum(), 'of', len(bad))
    if prev is not None and kw == {'md': -1}:
        print('  gpu self-consistent:', np.array_equal(prev.view(np.uint32), sg.view(np.uint32)))
    if kw == {'md': -1}:
        prev = sg.copy()
    if bad.any():
        d = sg[bad, 6]
        print('  depth hist', np.unique(d, return_counts=True))
        ulp = np.abs(sg[bad, :3].view(np.int32).astype(np.int64) - so[bad, :3].view(np.int32).astype(np.int64))
        print('  ulp hist', np.unique(ulp, return_counts=True))
        for r in np.nonzero(bad)[0][:4]:
            print('  ', r, sg[r].tolist(), so[r].tolist())
