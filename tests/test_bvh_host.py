"""The BVH the kernels traverse, checked on the host (no device): the 32 B
half-box nodes (MtsgHNode) and the 4-wide nodes (MtsgQNode) must be
conservative copies of the BVH2 (MtsgNode) -- every half box contains the
float box it replaces, and the 4-wide tree reaches exactly the BVH2's leaves --
so that the exact triangle / shape tests, and with them every hit, are the same
whichever node format a kernel traverses."""
import numpy as np
import pytest

from conftest import mitsuba_amd
from mitsuba_amd import scenes
from mitsuba_amd.integrator import bvh_host


def halves(words):
    """uint32 words -> (lo, hi) float32 arrays of the two packed IEEE halves."""
    w = np.ascontiguousarray(words, np.uint32)
    lo = (w & 0xFFFF).astype(np.uint16).view(np.float16).astype(np.float32)
    hi = (w >> 16).astype(np.uint16).view(np.float16).astype(np.float32)
    return lo, hi


def float_boxes(n):
    """MtsgNode words -> child boxes (N, 2, 3) lo and hi and child refs (N, 2)."""
    f = n.view(np.float32)
    lo = np.stack([np.stack([f[:, 0], f[:, 2], f[:, 8]], 1), np.stack([f[:, 4], f[:, 6], f[:, 10]], 1)], 1)
    hi = np.stack([np.stack([f[:, 1], f[:, 3], f[:, 9]], 1), np.stack([f[:, 5], f[:, 7], f[:, 11]], 1)], 1)
    return lo, hi, n[:, 12:14].view(np.int32)


def collapse(lo, hi, refs):
    """The 4-wide tree the host must have built from the BVH2: node 0 is the
    root; an inner BVH2 child is replaced by its two children; nodes are
    numbered in depth-first preorder (scene_build.cpp QCollapse).  Returns, per
    4-wide node, its children as (box lo, box hi, ref) with inner refs renumbered."""
    out = []

    def emit(ref):
        kids = []
        for c in range(2):
            r = int(refs[ref, c])
            if r >= 0:
                kids += [(lo[r, g], hi[r, g], int(refs[r, g])) for g in range(2)]
            else:
                kids.append((lo[ref, c], hi[ref, c], r))
        k = len(out)
        out.append(None)
        out[k] = [(a, b, emit(r) if r >= 0 else r) for a, b, r in kids]
        return k

    emit(0)
    return out


@pytest.mark.parametrize('cfg,kw', [('C1', dict(width=16, height=16, spp=1)),
                                    ('C4', dict(width=16, height=16, spp=1, columns=(2, 3), seg=24, rings=10))])
def test_half_and_wide_nodes_are_conservative(cfg, kw):
    sc, _ = scenes.build(cfg, **kw)
    n, h, q, depth4 = bvh_host(sc)
    assert len(n) == len(h) > 0 and len(q) > 0 and depth4 >= 1
    lo, hi, refs = float_boxes(n)
    # half-box nodes: same children, every bound widened outward (or equal)
    assert np.array_equal(h[:, 6:8].view(np.int32), refs)
    hl, hh = halves(h[:, :6])
    # box word order: {c0x}{c0y}{c1x}{c1y}{c0z}{c1z}
    hlo = np.stack([np.stack([hl[:, 0], hl[:, 1], hl[:, 4]], 1), np.stack([hl[:, 2], hl[:, 3], hl[:, 5]], 1)], 1)
    hhi = np.stack([np.stack([hh[:, 0], hh[:, 1], hh[:, 4]], 1), np.stack([hh[:, 2], hh[:, 3], hh[:, 5]], 1)], 1)
    assert np.all(hlo <= lo) and np.all(hhi >= hi)
    # and no wider than one half ulp beyond (the rounding is directed, not sloppy)
    step = np.spacing(np.abs(np.concatenate([lo, hi])).astype(np.float16)).astype(np.float32)
    widen = np.concatenate([lo - hlo, hhi - hi])
    assert np.all(widen <= step * 1.0001 + 1e-7)
    # 4-wide nodes: exactly the collapse of the BVH2, each box widened outward
    ql, qh = halves(q[:, :12])
    qref = q[:, 12:16].view(np.int32)
    want = collapse(lo, hi, refs)
    assert len(want) == len(q)
    for k, kids in enumerate(want):
        assert len(kids) >= 2
        for j in range(4):
            if j >= len(kids):
                assert qref[k, j] == 0
                continue
            blo, bhi, r = kids[j]
            assert qref[k, j] == r
            assert np.all(ql[k, 3 * j:3 * j + 3] <= blo) and np.all(qh[k, 3 * j:3 * j + 3] >= bhi)
