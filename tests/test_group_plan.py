"""The device group's decomposition on the host (no GPU): mtsgpu_group_member_params
deals the window's 8x8 tiles round-robin (MTSGPU_FLAG_TILE_SHARD, the bench's
decomposition, cf. BlockedImageProcess, src/librender/imageproc.cpp:28-80) and
mtsgpu_render_pixels counts what each member then renders, by the kernels'
item -> pixel rule.  Bar: the members cover the window exactly once and their
shares differ by at most one tile; at 1280x720 and N = 2, 4, 8 they are equal."""
import ctypes as C

import pytest

from mitsuba_amd import abi, integrator, scenes
from mitsuba_amd.distributed import TileSharding


def _member_pixels(w, h, n):
    L = integrator.load_library()
    _, it = scenes.build('C1', width=16, height=16, spp=1)
    base = it.params(w, h, 0, 0, w, h, 8, 1, 0)
    out = []
    for k in range(n):
        q = abi.RenderParams()
        assert L.mtsgpu_group_member_params(C.byref(base), n, k, C.byref(q)) == abi.OK
        assert q.flags & 16 and q.row_stride == n and q.row_phase == k
        out.append(L.mtsgpu_render_pixels(C.byref(q)))
    return out


@pytest.mark.parametrize('n', [2, 4, 8])
def test_group_members_equal_at_bench_frame(n):
    px = _member_pixels(1280, 720, n)
    assert sum(px) == 1280 * 720
    assert len(set(px)) == 1, px     # 14400 tiles divide evenly over 2, 4, 8 members


@pytest.mark.parametrize('w,h,n', [(1280, 720, 3), (1280, 720, 7), (517, 301, 8), (20, 12, 5), (5, 3, 4)])
def test_group_members_balanced_within_one_tile(w, h, n):
    px = _member_pixels(w, h, n)
    assert sum(px) == w * h
    assert max(px) - min(px) <= 64, px
    for k in range(n):
        assert px[k] == int(TileSharding(k, n).pixels(w, h).sum())


def test_member_pixels_match_rank_sharding():
    """The group's member k renders what bench.py's rank k renders (distributed.TileSharding)."""
    w, h, n = 1280, 720, 8
    px = _member_pixels(w, h, n)
    for k in range(n):
        s = TileSharding(k, n)
        assert s.row_params() == (8, n, k)
        assert px[k] == int(s.pixels(w, h).sum())


def test_member_params_reject_bad_arguments():
    L = integrator.load_library()
    _, it = scenes.build('C1', width=16, height=16, spp=1)
    p = it.params(16, 16, 0, 0, 16, 16, 8, 1, 0)
    q = abi.RenderParams()
    assert L.mtsgpu_group_member_params(C.byref(p), 0, 0, C.byref(q)) == abi.EINVAL
    assert L.mtsgpu_group_member_params(C.byref(p), 2, 2, C.byref(q)) == abi.EINVAL
    assert L.mtsgpu_group_member_params(None, 2, 0, C.byref(q)) == abi.EINVAL
