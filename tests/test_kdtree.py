"""The reference's SAH kd-tree (kdtree_build.cpp, after gkdtree.h:959-2592) on
the host, without a device: structural invariants of the KDNode array, and
the oracle's Havran traversal over it (sahkdtree3.h:178-308) against the
oracle's BVH traversal on the same rays -- the closest hit distance must
agree everywhere, the primitive wherever the hit is not an exact tie.

Parity with the reference's own tree is unpinned: the reference cannot be
built in this image; the builder follows its source step by
step and the GPU traversal is checked against the oracle's
(tests/test_gpu_kdtree.py)."""
import numpy as np
import pytest

from mitsuba_amd import scenes
from mitsuba_amd.integrator import kdtree_host


def _walk(nodes, idx):
    """Depth-first walk of the KDNode array: (leaf count, max depth, primitives seen)."""
    seen, leaves, depth = set(), 0, 0
    stack = [(0, 1)]
    while stack:
        n, dep = stack.pop()
        depth = max(depth, dep)
        a, b = int(nodes[n, 0]), int(nodes[n, 1])
        if a & 0x80000000:
            s = a & 0x7fffffff
            assert s <= b <= idx.size
            seen.update(idx[s:b].tolist())
            leaves += 1
        else:
            assert not (a & 0x40000000)                     # no indirections in the final layout
            left = n + ((a & ~(3 | 0x40000000)) >> 2)
            assert left > n and left + 1 < nodes.shape[0] and (a & 3) < 3
            stack += [(left + 1, dep + 1), (left, dep + 1)]
    return leaves, depth, seen


@pytest.mark.parametrize('cfg,kw', [('C1', dict(width=16, height=16, spp=1)),
                                    ('C3', dict(width=16, height=16, spp=1, blob=(60, 40), env_size=(16, 8))),
                                    ('C3', dict(width=16, height=16, spp=1, env_size=(16, 8)))])   # > 65536: min-max binning
def test_kdtree_structure(cfg, kw):
    sc, _ = scenes.build(cfg, **kw)
    nodes, idx, info = kdtree_host(sc)
    prims = sc.num_triangles
    assert info['nodes'] == nodes.shape[0] and info['indices'] == idx.size
    assert info['max_depth'] == min(48, int(8 + 1.3 * int(np.log2(prims))))
    leaves, depth, seen = _walk(nodes, idx)
    assert depth <= info['max_depth']
    assert leaves == nodes.shape[0] - (nodes.shape[0] - 1) // 2       # a full binary tree
    assert idx.max() < prims
    # every triangle with a non-degenerate box is in some leaf (pruning drops only empty clips)
    assert len(seen) >= prims - info['pruned']
    if prims > 65536:
        assert info['inner'] > 0


def _rays(sc, n, seed):
    rng = np.random.default_rng(seed)
    lo = np.min([m.positions.min(0) for m in sc.meshes], axis=0)
    hi = np.max([m.positions.max(0) for m in sc.meshes], axis=0)
    o = lo + (hi - lo) * rng.random((n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    # a share of axis-parallel rays (zero direction components, planar splits)
    d[: n // 8] = np.eye(3)[rng.integers(0, 3, n // 8)] * rng.choice([-1, 1], (n // 8, 1))
    return o.astype(np.float32), d.astype(np.float32)


@pytest.mark.parametrize('cfg,kw', [('C1', dict(width=16, height=16, spp=1)),
                                    ('C4', dict(width=16, height=16, spp=1)),
                                    ('C3', dict(width=16, height=16, spp=1, env_size=(16, 8)))])
def test_oracle_kd_traversal_matches_bvh(oracle, cfg, kw):
    sc, _ = scenes.build(cfg, **kw)
    nodes, idx, _ = kdtree_host(sc)
    o, d = _rays(sc, 20000, 7)
    kd = oracle.trace_rays_kd(sc, nodes, idx, o, d)
    bvh = oracle.trace_rays(sc, o, d)
    assert np.array_equal(kd[:, 0].view(np.uint32), bvh[:, 0].view(np.uint32))      # closest distance, bit for bit
    same_prim = kd[:, 3].view(np.uint32) == bvh[:, 3].view(np.uint32)
    assert same_prim.mean() > 0.999
    kd_s = oracle.trace_rays_kd(sc, nodes, idx, o, d, maxt=2.0, shadow=True)
    bvh_s = oracle.trace_rays(sc, o, d, maxt=2.0, shadow=True)
    assert np.array_equal(kd_s[:, 0], bvh_s[:, 0])


def test_oracle_render_over_kdtree_matches_bvh(oracle):
    """The oracle's path render over the kd-tree equals its BVH render wherever no
    exact-t tie decides a hit (the Cornell box has none at these samples)."""
    sc, it = scenes.build('C1', width=32, height=24, spp=4)
    nodes, idx, _ = kdtree_host(sc)
    f_kd, s_kd, st_kd = oracle.render(sc, it, samples=True, libm_mode=0, kdtree=(nodes, idx))
    f_bvh, s_bvh, st_bvh = oracle.render(sc, it, samples=True, libm_mode=0)
    same = np.all(s_kd.view(np.uint32) == s_bvh.view(np.uint32), axis=1)
    assert same.mean() > 0.999
    assert st_kd['samples'] == st_bvh['samples']
