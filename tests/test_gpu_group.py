"""Device groups (mtsgpu_group_*): one render call sharded over several GPUs,
films merged on the first device (include/mtsgpu.h).

A one-GPU box lists device 0 more than once: the members are separate
contexts with their own films, so the 8x8 tile sharding (the bench's
decomposition, tests/test_group_plan.py checks its balance on the host), the
per-member renders on parallel host threads and the in-order merge all run as
on a node.  Bar: with the box filter the merged film equals the single-context
film bit for bit (disjoint tiles, Film::put sums of zeros elsewhere); with the
gaussian filter the overlapping borders of neighbouring tiles are summed in
another order (rtol 2e-6, as the row-shard test of test_gpu_parity.py)."""
import numpy as np
import pytest

from mitsuba_amd import scenes
from mitsuba_amd.integrator import DeviceGroup

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('n', [1, 2, 3])
def test_group_film_equals_single_context(gpu_ctx, n):
    sc, it = scenes.build('C1', width=96, height=72, spp=8)
    gpu_ctx.upload(sc)
    film_1, _, st_1 = gpu_ctx.render(it)
    g = DeviceGroup([0] * n)
    assert len(g) == n
    g.upload(sc)
    film_g, st_g = g.render(it)
    assert np.array_equal(film_g.view(np.uint32), film_1.view(np.uint32))
    for k in ('samples', 'rays', 'shadow_rays', 'path_length_sum'):
        assert st_g[k] == st_1[k], k
    g.close()


def test_group_gaussian_window(gpu_ctx):
    sc, it = scenes.build('C1', width=80, height=64, spp=4)
    it.rfilter = 'gaussian'
    gpu_ctx.upload(sc)
    win = (5, 3, 61, 49)
    film_1, _, _ = gpu_ctx.render(it, window=win)
    g = DeviceGroup([0, 0])
    g.upload(sc)
    for n in (1, 3):   # row_block is ignored: the group shards 8x8 tiles
        film_g, st = g.render(it, window=win, row_block=n)
        np.testing.assert_allclose(film_g, film_1, rtol=2e-6, atol=1e-6)
        assert st['samples'] == 61 * 49 * 4
    g.close()


def test_group_rejects_row_stride_and_render_before_upload():
    import ctypes as C
    from mitsuba_amd import abi
    g = DeviceGroup([0, 0])
    sc, it = scenes.build('C1', width=16, height=16, spp=1)
    from mitsuba_amd.scene import film_border
    b = film_border(it.rfilter, it.rfilterParam)
    film = np.zeros((16 + 2 * b, 16 + 2 * b, 5), np.float32)    # the (W+2b)(H+2b)x5 layout the library writes

    def call(p):
        return g.L.mtsgpu_group_render(g.h, C.byref(p), film.ctypes.data_as(C.POINTER(C.c_float)), C.byref(abi.Stats()))
    assert call(it.params(16, 16, 0, 0, 16, 16, 8, 1, 0)) == abi.ESTATE
    assert b'before upload' in g.L.mtsgpu_group_last_error(g.h)
    g.upload(sc)
    assert call(it.params(16, 16, 0, 0, 16, 16, 8, 2, 0)) == abi.EINVAL
    assert b'row_stride' in g.L.mtsgpu_group_last_error(g.h)
    assert call(it.params(16, 16, 0, 0, 16, 16, 8, 1, 0)) == abi.OK
    g.close()


_FRESH_GROUP = r'''
import sys
sys.path.insert(0, sys.argv[1])
from pkgimport import mitsuba_amd
mitsuba_amd()
import numpy as np
from mitsuba_amd import scenes
from mitsuba_amd.integrator import Context, DeviceGroup
sc, it = scenes.build('C1', width=64, height=48, spp=4)
g = DeviceGroup([0, 0, 0, 0])      # first upload of the process: four members build the tables at once
g.upload(sc)
film_g, st_g = g.render(it)
ctx = Context(0)
ctx.upload(sc)
film_1, _, _ = ctx.render(it)
assert np.array_equal(film_g.view(np.uint32), film_1.view(np.uint32)), 'group film differs'
g.close()
print('fresh group ok')
'''


def test_group_first_upload_in_fresh_process():
    """the first upload of a process going through a group builds
    the Sobol tables on several host threads at once (capi.cpp
    sobol_nibble_tables, scene_build.cpp mtsg_sobol_matrices).  Run it in a
    fresh child process, with no prior single-context upload."""
    import os
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, '-c', _FRESH_GROUP, repo], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert 'fresh group ok' in r.stdout
