// kdtree_build.cpp -- Mitsuba's SAH kd-tree over the scene's triangles, built
// on the host as the reference builds ShapeKDTree (src/librender/skdtree.cpp:
// 68-110 -> SAHKDTree3D::buildInternal -> GenericKDTree::buildInternal,
// include/mitsuba/render/gkdtree.h:959-1264), so that the GPU can traverse
// the reference's own tree (rayIntersectHavran, sahkdtree3.h:178-308) and
// reproduce its closest-hit choice among exactly tied primitives.
//
// Followed step by step, in single precision where the reference's Float is
// single (SINGLE_PRECISION) and in double where it computes in double:
//   defaults                 gkdtree.h:733-746 (traversal 15, query 20, empty-space
//                            bonus 0.9, perfect splits, retraction, stop 6 prims,
//                            3 bad refines, exact threshold 65536, 128 min-max bins)
//   depth cutoff             :986-989 (8 + 1.3 log2i(n), at most MTS_KD_MAXDEPTH 48)
//   min-max binning          :1793-1924 (MinMaxBins :2406-2592) above the threshold
//   O(n log n) sweep         :1955-2398 (edge events ordered by axis, pos, type,
//                            index :1332-1342; planar split sides; classification,
//                            clipping of straddling triangles, merge)
//   event lists              :1552-1592; leaves :1608-1700 (event order / retraction
//                            collapses to a sorted unique list)
//   parallel build           :1036-1047, 1730-1762: above the threshold subtrees go to
//                            worker threads and report cost -inf (never retracted);
//                            the result does not depend on the thread count, so the
//                            subtrees are built here in order with that cost
//   final layout             :1105-1182 (depth-first rewrite, children pairs)
//   perfect splits           Triangle::getClippedAABB (src/libcore/triangle.cpp:71-147,
//                            Sutherland-Hodgman in double, castflt_down/up)
//   SAH                      SurfaceAreaHeuristic3 (sahkdtree3.h:39-84)
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "kdtree.h"

namespace {

constexpr float kTraversalCost = 15, kQueryCost = 20, kEmptySpaceBonus = 0.9f;
constexpr uint32_t kStopPrims = 6, kMaxBadRefines = 3, kExactPrimThreshold = 65536, kMinMaxBins = 128;
constexpr uint32_t kMaxDepthLimit = 48;   // MTS_KD_MAXDEPTH (gkdtree.h:38)
const float kInf = std::numeric_limits<float>::infinity();

struct Box {   // TAABB<Point> with reset() bounds (aabb.h:101-104)
    float mn[3] = {kInf, kInf, kInf}, mx[3] = {-kInf, -kInf, -kInf};
    bool valid() const { return !(mx[0] < mn[0] || mx[1] < mn[1] || mx[2] < mn[2]); }
    float area() const {   // AABB::getSurfaceArea (aabb.h:464-467)
        const float dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
        return 2.0f * (dx * dy + dx * dz + dy * dz);
    }
    void expand(const Box &b) {
        for (int i = 0; i < 3; ++i) { mn[i] = std::min(mn[i], b.mn[i]); mx[i] = std::max(mx[i], b.mx[i]); }
    }
    void expand(const float *p) {
        for (int i = 0; i < 3; ++i) { mn[i] = std::min(mn[i], p[i]); mx[i] = std::max(mx[i], p[i]); }
    }
    void clip(const Box &b) {   // aabb.h:87-92
        for (int i = 0; i < 3; ++i) { mn[i] = std::max(mn[i], b.mn[i]); mx[i] = std::min(mx[i], b.mx[i]); }
    }
};

// math::castflt_down / castflt_up (math.h:284-310)
float castflt_up(double v) {
    float a = (float)v;
    if ((double)a < v) a = std::nextafter(a, kInf);
    return a;
}
float castflt_down(double v) {
    float a = (float)v;
    if ((double)a > v) a = std::nextafter(a, -kInf);
    return a;
}

// SurfaceAreaHeuristic3 (sahkdtree3.h:48-73)
struct SAH {
    float t0[3], t1[3];
    explicit SAH(const Box &b) {
        const float ex = b.mx[0] - b.mn[0], ey = b.mx[1] - b.mn[1], ez = b.mx[2] - b.mn[2];
        const float temp = 1.0f / (ex * ey + ey * ez + ex * ez);
        t0[0] = ey * ez * temp; t0[1] = ex * ez * temp; t0[2] = ex * ey * temp;
        t1[0] = (ey + ez) * temp; t1[1] = (ex + ez) * temp; t1[2] = (ex + ey) * temp;
    }
    void operator()(int axis, float lw, float rw, float &pl, float &pr) const {
        pl = t0[axis] + t1[axis] * lw;
        pr = t0[axis] + t1[axis] * rw;
    }
};

enum { EEnd = 0, EPlanar = 1, EStart = 2 };
struct Event {
    float pos;
    uint32_t index;
    uint8_t type, axis;
};
inline bool ev_less(const Event &a, const Event &b) {   // EdgeEventOrdering (gkdtree.h:1332-1342)
    if (a.axis != b.axis) return a.axis < b.axis;
    if (a.pos != b.pos) return a.pos < b.pos;
    if (a.type != b.type) return a.type < b.type;
    return a.index < b.index;
}

enum { EBothSides = 0, ELeftSide = 1, ERightSide = 2, EBothSidesProcessed = 3 };

// preliminary node: the reference's KDNode before the rewrite (children in pairs)
struct PNode {
    bool leaf = false;
    int axis = 0;
    float split = 0;
    uint32_t left = 0;            // index of the children pair in `nodes`
    uint32_t primStart = 0, primEnd = 0;
};

struct Builder {
    const float *P;               // 9 floats per primitive: v0, v1, v2 (world space)
    uint32_t primCount;
    uint32_t maxDepth;
    bool parallel;
    std::vector<PNode> nodes;
    std::vector<uint32_t> indices;
    std::vector<uint8_t> cls;
    KdStats st;

    Box prim_aabb(uint32_t i) const {   // Triangle::getAABB
        Box b;
        for (int v = 0; v < 3; ++v) b.expand(P + 9 * (size_t)i + 3 * v);
        return b;
    }

    // Triangle::getClippedAABB (triangle.cpp:71-147)
    static int sutherland_hodgman(const double (*in)[3], int inCount, double (*out)[3], int axis, double splitPos,
                                  bool isMinimum) {
        if (inCount < 3) return 0;
        double cur[3] = {in[0][0], in[0][1], in[0][2]};
        const double sign = isMinimum ? 1.0 : -1.0;
        double distance = sign * (cur[axis] - splitPos);
        bool curIsInside = distance >= 0;
        int outCount = 0;
        for (int i = 0; i < inCount; ++i) {
            int nextIdx = i + 1;
            if (nextIdx == inCount) nextIdx = 0;
            const double next[3] = {in[nextIdx][0], in[nextIdx][1], in[nextIdx][2]};
            distance = sign * (next[axis] - splitPos);
            const bool nextIsInside = distance >= 0;
            if (curIsInside && nextIsInside) {
                std::memcpy(out[outCount++], next, sizeof next);
            } else if (curIsInside != nextIsInside) {
                const double t = (splitPos - cur[axis]) / (next[axis] - cur[axis]);
                double *p = out[outCount++];
                for (int k = 0; k < 3; ++k) p[k] = cur[k] + (next[k] - cur[k]) * t;
                p[axis] = splitPos;
                if (nextIsInside) std::memcpy(out[outCount++], next, sizeof next);
            }
            std::memcpy(cur, next, sizeof cur);
            curIsInside = nextIsInside;
        }
        return outCount;
    }
    Box clipped_aabb(uint32_t i, const Box &box) const {
        double v1[10][3], v2[10][3];
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 3; ++k) v1[v][k] = (double)P[9 * (size_t)i + 3 * v + k];
        int n = 3;
        for (int axis = 0; axis < 3; ++axis) {
            n = sutherland_hodgman(v1, n, v2, axis, (double)box.mn[axis], true);
            n = sutherland_hodgman(v2, n, v1, axis, (double)box.mx[axis], false);
        }
        Box r;
        for (int v = 0; v < n; ++v)
            for (int k = 0; k < 3; ++k) {
                r.mn[k] = std::min(r.mn[k], castflt_down(v1[v][k]));
                r.mx[k] = std::max(r.mx[k], castflt_up(v1[v][k]));
            }
        r.clip(box);
        return r;
    }

    static void push_events(std::vector<Event> &ev, const Box &b, uint32_t index) {
        for (int axis = 0; axis < 3; ++axis) {
            const float mn = b.mn[axis], mx = b.mx[axis];
            if (mn == mx) {
                ev.push_back({mn, index, EPlanar, (uint8_t)axis});
            } else {
                ev.push_back({mn, index, EStart, (uint8_t)axis});
                ev.push_back({mx, index, EEnd, (uint8_t)axis});
            }
        }
    }

    // createLeaf (gkdtree.h:1608-1651)
    void leaf_from_events(PNode &node, const std::vector<Event> &ev, uint32_t primCount) {
        node.leaf = true;
        node.primStart = (uint32_t)indices.size();
        if (primCount > 0) {
            for (const Event &e : ev) {
                if (e.axis != 0) break;
                if (e.type == EStart || e.type == EPlanar) indices.push_back(e.index);
            }
            st.nonempty_leaves++;
        }
        node.primEnd = (uint32_t)indices.size();
        st.leaves++;
    }
    void leaf_from_indices(PNode &node, const uint32_t *idx, uint32_t primCount) {
        node.leaf = true;
        node.primStart = (uint32_t)indices.size();
        if (primCount > 0) {
            indices.insert(indices.end(), idx, idx + primCount);
            st.nonempty_leaves++;
        }
        node.primEnd = (uint32_t)indices.size();
        st.leaves++;
    }
    // createLeafAfterRetraction (gkdtree.h:1666-1700)
    void leaf_after_retraction(PNode &node, uint32_t start) {
        std::vector<uint32_t> tmp(indices.begin() + start, indices.end());
        std::sort(tmp.begin(), tmp.end());
        tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
        indices.resize(start);
        indices.insert(indices.end(), tmp.begin(), tmp.end());
        node.leaf = true;
        node.primStart = start;
        node.primEnd = (uint32_t)indices.size();
        st.nonempty_leaves++;
        st.leaves++;
    }

    uint32_t alloc_pair() {
        nodes.emplace_back();
        nodes.emplace_back();
        return (uint32_t)nodes.size() - 2;
    }

    // createEventList + transitionToNLogN (gkdtree.h:1552-1592, 1730-1762)
    float transition(uint32_t depth, uint32_t node, const Box &nodeAABB, const std::vector<uint32_t> &prims,
                     uint32_t badRefines) {
        std::vector<Event> ev;
        ev.reserve(prims.size() * 6);
        uint32_t actual = 0;
        for (uint32_t index : prims) {
            const Box b = clipped_aabb(index, nodeAABB);   // m_clip
            if (!b.valid() || b.area() == 0) continue;
            push_events(ev, b, index);
            ++actual;
        }
        std::sort(ev.begin(), ev.end(), ev_less);
        const float cost = build(depth, node, nodeAABB, ev, actual, badRefines);
        return parallel ? -kInf : cost;   // a worker's subtree is never torn down
    }

    // buildTreeMinMax (gkdtree.h:1793-1924)
    float build_minmax(uint32_t depth, uint32_t node, const Box &nodeAABB, const Box &tightAABB,
                       std::vector<uint32_t> &prims, uint32_t badRefines) {
        const uint32_t primCount = (uint32_t)prims.size();
        const float leafCost = primCount * kQueryCost;
        if (primCount <= kStopPrims || depth >= maxDepth) {
            leaf_from_indices(nodes[node], prims.data(), primCount);
            return leafCost;
        }
        if (primCount <= kExactPrimThreshold) return transition(depth, node, nodeAABB, prims, badRefines);

        // MinMaxBins::setAABB / bin (:2420-2458)
        float bmin[3], binSize[3], invBin[3];
        Box binBox;
        for (int a = 0; a < 3; ++a) {
            const float mn = tightAABB.mn[a], mx = tightAABB.mx[a];   // castflt of floats: unchanged
            bmin[a] = mn; binBox.mn[a] = mn; binBox.mx[a] = mx;
            binSize[a] = (mx - mn) / (float)kMinMaxBins;
            invBin[a] = 1 / binSize[a];
        }
        auto computeIndex = [&](float pos, int axis) -> uint32_t {
            return (uint32_t)std::min((float)(kMinMaxBins - 1), std::max(0.0f, (pos - bmin[axis]) * invBin[axis]));
        };
        std::vector<uint32_t> minBins(3 * kMinMaxBins, 0), maxBins(3 * kMinMaxBins, 0);
        for (uint32_t i = 0; i < primCount; ++i) {
            const Box b = prim_aabb(prims[i]);
            for (int a = 0; a < 3; ++a) {
                minBins[a * kMinMaxBins + computeIndex(b.mn[a], a)]++;
                maxBins[a * kMinMaxBins + computeIndex(b.mx[a], a)]++;
            }
        }
        // MinMaxBins::minimizeCost (:2466-2504)
        float bestCost = kInf;
        int bestAxis = 0, leftBin = -1;
        uint32_t bestL = 0, bestR = 0;
        {
            const SAH tch(binBox);
            int binIdx = 0;
            for (int axis = 0; axis < 3; ++axis) {
                uint32_t numLeft = 0, numRight = primCount;
                float leftWidth = 0, rightWidth = binBox.mx[axis] - binBox.mn[axis];
                const float bs = binSize[axis];
                for (int i = 0; i < (int)kMinMaxBins - 1; ++i) {
                    numLeft += minBins[binIdx];
                    numRight -= maxBins[binIdx];
                    leftWidth += bs;
                    rightWidth -= bs;
                    float pl, pr;
                    tch(axis, leftWidth, rightWidth, pl, pr);
                    const float cost = kTraversalCost + kQueryCost * (pl * numLeft + pr * numRight);
                    if (cost < bestCost) {
                        bestCost = cost; bestAxis = axis; bestL = numLeft; bestR = numRight; leftBin = i;
                    }
                    binIdx++;
                }
                binIdx++;
            }
        }
        if (bestCost == kInf) return transition(depth, node, nodeAABB, prims, badRefines);
        if (bestCost >= leafCost) {   // "bad refines" (PBRT)
            if ((bestCost > 4 * leafCost && primCount < 16) || badRefines >= kMaxBadRefines) {
                leaf_from_indices(nodes[node], prims.data(), primCount);
                return leafCost;
            }
            ++badRefines;
        }
        // MinMaxBins::partition (:2523-2582)
        std::vector<uint32_t> li, ri;
        li.reserve(bestL); ri.reserve(bestR);
        Box lb, rb;
        const int axis = bestAxis;
        for (uint32_t i = 0; i < primCount; ++i) {
            const uint32_t p = prims[i];
            const Box b = prim_aabb(p);
            const int s = (int)computeIndex(b.mn[axis], axis), e = (int)computeIndex(b.mx[axis], axis);
            if (e <= leftBin) { lb.expand(b); li.push_back(p); }
            else if (s > leftBin) { rb.expand(b); ri.push_back(p); }
            else { lb.expand(b); rb.expand(b); li.push_back(p); ri.push_back(p); }
        }
        lb.clip(binBox);
        rb.clip(binBox);
        const float pos = bmin[axis] + binSize[axis] * (float)(leftBin + 1);
        lb.mx[axis] = std::min(lb.mx[axis], pos);
        rb.mn[axis] = std::max(rb.mn[axis], pos);
        std::vector<uint32_t>().swap(prims);

        const uint32_t children = alloc_pair();
        const uint32_t nodePos = (uint32_t)nodes.size(), indexPos = (uint32_t)indices.size();
        const KdStats saved = st;
        nodes[node].leaf = false; nodes[node].axis = axis; nodes[node].split = pos; nodes[node].left = children;
        st.inner++;
        Box childAABB = nodeAABB;
        childAABB.mx[axis] = pos;
        const float leftCost = build_minmax(depth + 1, children, childAABB, lb, li, badRefines);
        childAABB.mn[axis] = pos;
        childAABB.mx[axis] = nodeAABB.mx[axis];
        const float rightCost = build_minmax(depth + 1, children + 1, childAABB, rb, ri, badRefines);
        const SAH tch(nodeAABB);
        float pl, pr;
        tch(axis, pos - nodeAABB.mn[axis], nodeAABB.mx[axis] - pos, pl, pr);
        const float finalCost = kTraversalCost + (pl * leftCost + pr * rightCost);
        if (finalCost < primCount * kQueryCost) return finalCost;
        nodes.resize(nodePos);   // retract (:1911-1923)
        st.leaves = saved.leaves; st.nonempty_leaves = saved.nonempty_leaves; st.inner = saved.inner;
        st.retracted++;
        leaf_after_retraction(nodes[node], indexPos);
        return leafCost;
    }

    // buildTree (gkdtree.h:1955-2398)
    float build(uint32_t depth, uint32_t node, const Box &nodeAABB, std::vector<Event> &ev, uint32_t primCount,
                uint32_t badRefines) {
        const float leafCost = primCount * kQueryCost;
        if (primCount <= kStopPrims || depth >= maxDepth) {
            leaf_from_events(nodes[node], ev, primCount);
            return leafCost;
        }
        float bCost = kInf, bPos = 0;
        int bAxis = 0;
        uint32_t bNL = 0, bNR = 0;
        bool bPlanarLeft = false;
        uint32_t numLeft[3] = {0, 0, 0}, numRight[3] = {primCount, primCount, primCount};
        size_t byAxis[3] = {0, 0, 0};
        int byAxisCtr = 1;
        const SAH tch(nodeAABB);
        const size_t n = ev.size();
        for (size_t e = 0; e < n;) {
            const int axis = ev[e].axis;
            const float pos = ev[e].pos;
            uint32_t numStart = 0, numEnd = 0, numPlanar = 0;
            while (e < n && ev[e].pos == pos && ev[e].axis == axis && ev[e].type == EEnd) { ++numEnd; ++e; }
            while (e < n && ev[e].pos == pos && ev[e].axis == axis && ev[e].type == EPlanar) { ++numPlanar; ++e; }
            while (e < n && ev[e].pos == pos && ev[e].axis == axis && ev[e].type == EStart) { ++numStart; ++e; }
            if (e < n && ev[e].axis != axis) byAxis[byAxisCtr++] = e;
            numRight[axis] -= numPlanar + numEnd;
            if (pos > nodeAABB.mn[axis] && pos < nodeAABB.mx[axis]) {
                const uint32_t nL = numLeft[axis], nR = numRight[axis];
                const float nLF = (float)nL, nRF = (float)nR;
                float pl, pr;
                tch(axis, pos - nodeAABB.mn[axis], nodeAABB.mx[axis] - pos, pl, pr);
                if (numPlanar == 0) {
                    float cost = kTraversalCost + kQueryCost * (pl * nLF + pr * nRF);
                    if (nL == 0 || nR == 0) cost *= kEmptySpaceBonus;
                    if (cost < bCost) { bPos = pos; bAxis = axis; bCost = cost; bNL = nL; bNR = nR; }
                } else {
                    float cL = kTraversalCost + kQueryCost * (pl * (float)(nL + numPlanar) + pr * nRF);
                    float cR = kTraversalCost + kQueryCost * (pl * nLF + pr * (float)(nR + numPlanar));
                    if (nL + numPlanar == 0 || nR == 0) cL *= kEmptySpaceBonus;
                    if (nL == 0 || nR + numPlanar == 0) cR *= kEmptySpaceBonus;
                    if (cL < bCost || cR < bCost) {
                        bPos = pos; bAxis = axis;
                        if (cL < cR) { bCost = cL; bNL = nL + numPlanar; bNR = nR; bPlanarLeft = true; }
                        else { bCost = cR; bNL = nL; bNR = nR + numPlanar; bPlanarLeft = false; }
                    }
                }
            }
            numLeft[axis] += numStart + numPlanar;
        }
        if (bCost >= leafCost) {
            if ((bCost > 4 * leafCost && primCount < 16) || badRefines >= kMaxBadRefines || bCost == kInf) {
                leaf_from_events(nodes[node], ev, primCount);
                return leafCost;
            }
            ++badRefines;
        }
        // classification (:2121-2166)
        uint32_t primsLeft = 0, primsRight = 0, primsBoth = primCount;
        const size_t a0 = byAxis[bAxis];
        for (size_t e = a0; e < n && ev[e].axis == bAxis; ++e) cls[ev[e].index] = EBothSides;
        for (size_t e = a0; e < n && ev[e].axis == bAxis; ++e) {
            const Event &E = ev[e];
            if (E.type == EEnd && E.pos <= bPos) {
                cls[E.index] = ELeftSide; primsBoth--; primsLeft++;
            } else if (E.type == EStart && E.pos >= bPos) {
                cls[E.index] = ERightSide; primsBoth--; primsRight++;
            } else if (E.type == EPlanar) {
                if (E.pos < bPos || (E.pos == bPos && bPlanarLeft)) { cls[E.index] = ELeftSide; primsBoth--; primsLeft++; }
                else { cls[E.index] = ERightSide; primsBoth--; primsRight++; }
            }
        }
        Box lAABB = nodeAABB, rAABB = nodeAABB;
        lAABB.mx[bAxis] = bPos;
        rAABB.mn[bAxis] = bPos;
        uint32_t prunedLeft = 0, prunedRight = 0;
        // partitioning with perfect splits (:2197-2303)
        std::vector<Event> lTmp, rTmp, nL, nR;
        lTmp.reserve((size_t)primsLeft * 6); rTmp.reserve((size_t)primsRight * 6);
        nL.reserve((size_t)primsBoth * 6); nR.reserve((size_t)primsBoth * 6);
        for (size_t e = 0; e < n; ++e) {
            const Event &E = ev[e];
            const int c = cls[E.index];
            if (c == ELeftSide) lTmp.push_back(E);
            else if (c == ERightSide) rTmp.push_back(E);
            else if (c == EBothSides) {
                const Box cl = clipped_aabb(E.index, lAABB), cr = clipped_aabb(E.index, rAABB);
                if (cl.valid() && cl.area() > 0) push_events(nL, cl, E.index);
                else prunedLeft++;
                if (cr.valid() && cr.area() > 0) push_events(nR, cr, E.index);
                else prunedRight++;
                cls[E.index] = EBothSidesProcessed;
            }
        }
        st.pruned += prunedLeft + prunedRight;
        std::sort(nL.begin(), nL.end(), ev_less);
        std::sort(nR.begin(), nR.end(), ev_less);
        std::vector<Event> lEv(lTmp.size() + nL.size()), rEv(rTmp.size() + nR.size());
        std::merge(lTmp.begin(), lTmp.end(), nL.begin(), nL.end(), lEv.begin(), ev_less);
        std::merge(rTmp.begin(), rTmp.end(), nR.begin(), nR.end(), rEv.begin(), ev_less);
        std::vector<Event>().swap(lTmp); std::vector<Event>().swap(rTmp);
        std::vector<Event>().swap(nL); std::vector<Event>().swap(nR);
        std::vector<Event>().swap(ev);

        const uint32_t children = alloc_pair();
        const uint32_t nodePos = (uint32_t)nodes.size(), indexPos = (uint32_t)indices.size();
        const KdStats saved = st;
        nodes[node].leaf = false; nodes[node].axis = bAxis; nodes[node].split = bPos; nodes[node].left = children;
        st.inner++;
        const float leftCost = build(depth + 1, children, lAABB, lEv, bNL - prunedLeft, badRefines);
        const float rightCost = build(depth + 1, children + 1, rAABB, rEv, bNR - prunedRight, badRefines);
        float pl, pr;
        tch(bAxis, bPos - nodeAABB.mn[bAxis], nodeAABB.mx[bAxis] - bPos, pl, pr);
        const float finalCost = kTraversalCost + (pl * leftCost + pr * rightCost);
        if (finalCost < primCount * kQueryCost) return finalCost;
        nodes.resize(nodePos);
        st.leaves = saved.leaves; st.nonempty_leaves = saved.nonempty_leaves; st.inner = saved.inner;
        st.retracted++;
        leaf_after_retraction(nodes[node], indexPos);
        return leafCost;
    }
};

int log2i(uint32_t v) {   // math::log2i: floor(log2 v)
    int r = 0;
    while (v >>= 1) ++r;
    return r;
}

}  // namespace

bool mtsg_build_kdtree(const float *tri_positions, uint32_t prims, KdTree &out, bool multicore) {
    out = KdTree();
    Builder B;
    B.P = tri_positions;
    B.primCount = prims;
    B.cls.assign(prims, 0);
    if (prims == 0) {   // gkdtree.h:973-979
        out.nodes = {0x80000000u, 0u};
        return true;
    }
    // m_parallelBuild: on above the exact threshold, with more than one core (:981-982, 1036-1038)
    B.parallel = multicore && prims > kExactPrimThreshold;
    B.maxDepth = std::min((uint32_t)(int)(8 + 1.3f * log2i(prims)), kMaxDepthLimit);
    Box aabb;
    std::vector<uint32_t> idx(prims);
    for (uint32_t i = 0; i < prims; ++i) {
        aabb.expand(B.prim_aabb(i));
        idx[i] = i;
    }
    B.nodes.emplace_back();   // prelimRoot
    B.build_minmax(1, 0, aabb, aabb, idx, 0);

    // depth-first rewrite into the final node array (gkdtree.h:1105-1182)
    out.nodes.clear();
    out.indices.clear();
    struct Item { uint32_t node, target; };
    std::vector<Item> stack;
    out.nodes.resize(2 * B.nodes.size());
    uint32_t nodePtr = 0;
    stack.push_back({0, nodePtr++});
    while (!stack.empty()) {
        const Item it = stack.back();
        stack.pop_back();
        const PNode &pn = B.nodes[it.node];
        uint32_t *t = &out.nodes[2 * it.target];
        if (pn.leaf) {
            const uint32_t start = (uint32_t)out.indices.size();
            for (uint32_t k = pn.primStart; k < pn.primEnd; ++k) out.indices.push_back(B.indices[k]);
            t[0] = 0x80000000u | start;                        // initLeafNode
            t[1] = start + (pn.primEnd - pn.primStart);
        } else {
            const uint32_t children = nodePtr;
            nodePtr += 2;
            const uint32_t rel = children - it.target;
            // KDNode's 28-bit relative offset (gkdtree.h:489-505, ERelOffsetLimit); the
            // reference's indirection nodes past it are not restated: refuse the tree
            if (rel > (1u << 28) - 1) return false;
            t[0] = (uint32_t)pn.axis | (rel << 2);              // initInnerNode
            std::memcpy(&t[1], &pn.split, 4);
            stack.push_back({pn.left + 1, children + 1});
            stack.push_back({pn.left, children});
        }
    }
    out.nodes.resize(2 * (size_t)nodePtr);
    out.stats = B.st;
    out.stats.nodes = nodePtr;
    out.stats.max_depth = B.maxDepth;
    for (int a = 0; a < 3; ++a) { out.aabb_min[a] = aabb.mn[a]; out.aabb_max[a] = aabb.mx[a]; }
    return true;
}
