// kdtree.h -- host side of the reference's SAH kd-tree (kdtree_build.cpp).
#pragma once
#include <cstdint>
#include <vector>

struct KdStats {
    uint32_t inner = 0, leaves = 0, nonempty_leaves = 0, retracted = 0, pruned = 0;
    uint32_t nodes = 0, max_depth = 0;
};

// KDNode array in the reference's final layout (gkdtree.h:453-601): two words
// per node; inner: {axis | relOffset << 2, split bits}, leaf: {1 << 31 | start,
// end}; `indices` the primitive lists (global primitive numbers: meshes in scene
// order, triangles in mesh order).
struct KdTree {
    std::vector<uint32_t> nodes;
    std::vector<uint32_t> indices;
    float aabb_min[3] = {0, 0, 0}, aabb_max[3] = {0, 0, 0};   // tight bounds (before the 1e-3 enlargement)
    KdStats stats;
};

// tri_positions: 9 floats per primitive (v0, v1, v2, world space), global order.
// multicore: the reference machine builds above 65536 primitives in parallel
// (subtrees handed to workers are never retracted).
// false: a child offset exceeds KDNode's 28-bit relative field (the reference
// then inserts indirection nodes, which are not restated here)
bool mtsg_build_kdtree(const float *tri_positions, uint32_t prims, KdTree &out, bool multicore = true);
