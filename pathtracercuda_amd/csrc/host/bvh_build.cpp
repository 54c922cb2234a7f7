// Binned-SAH BVH of the C++ drop-in API (reference src/pathtracer/BVH.cpp:5-255).
// The node layout is the traversal contract of the GPU kernel (depth-first, left child = node+1,
// right child = m_offset, leaves point at a contiguous run of the reordered elements), and the
// build is deterministic given the libstdc++ std::partition / std::nth_element algorithms; the
// test suite checks it node-for-node against the oracle's independent restatement.
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <future>
#include <limits>
#include <thread>

#include "pathtracer_amd.hpp"

namespace {

float calcSurfaceArea(const vec3& minCorner, const vec3& maxCorner)   // BVH.cpp:54-64
{
    const vec3 extent = maxCorner - minCorner;
    if (extent.x <= 0.0f || extent.y <= 0.0f || extent.z <= 0.0f) return 0.0f;
    return (extent[0] * extent[1] + extent[0] * extent[2] + extent[1] * extent[2]) * 2.0f;
}

// int(float) as an x86 build of the reference executes it (cvttss2si: out of range -> INT_MIN)
inline int toIntX86(float f)
{
    if (!(f > -2147483904.0f && f < 2147483648.0f)) return INT_MIN;
    return (int)f;
}

inline AABB merge(const AABB& a, const AABB& b) { return AABB{min(a.m_min, b.m_min), max(a.m_max, b.m_max)}; }

} // namespace

void BVH::build(size_t elementCount, const CpuHittable* elements, uint32_t maxLeafElements)
{
    m_maxLeafElements = maxLeafElements;
    m_nodes.clear();
    m_elements.assign(elements, elements + elementCount);
    if (elementCount == 0) return;
    m_nodes.reserve(2 * elementCount - 1);
    // Subtrees are independent (disjoint element ranges, per-node arithmetic only), so large
    // subtrees build on worker threads into their own node arrays, which are then concatenated in
    // depth-first order with interior offsets rebased: the result is the sequential layout exactly.
    // (SAH splits can be very uneven, so threads go to nodes whose *smaller* side is large.)
    unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    if (const char* env = getenv("PT_BVH_THREADS")) hw = std::max(1, atoi(env));   // 1 = sequential
    std::atomic<int> spare((int)std::min(hw, 64u) - 1);
    m_spareThreads = &spare;
    buildInto(m_nodes, 0, elementCount);
    m_spareThreads = nullptr;
}

// Appends a subtree built into its own array (root at index 0) at the end of `out`.
static void appendSubtree(std::vector<BVHNode>& out, const std::vector<BVHNode>& sub)
{
    const uint32_t base = static_cast<uint32_t>(out.size());
    for (BVHNode n : sub) {
        if ((n.m_primitiveCountAxis >> 16) == 0) n.m_offset += base;   // interior: node index; leaf: element index
        out.push_back(n);
    }
}

uint32_t BVH::getDepth(uint32_t node) const
{
    // iterative (the reference recurses, BVH.cpp:27-34); deep degenerate trees must not blow the stack
    uint32_t best = 0;
    std::vector<std::pair<uint32_t, uint32_t>> st{{node, 1u}};
    while (!st.empty()) {
        auto [n, d] = st.back();
        st.pop_back();
        if (m_nodes[n].m_primitiveCountAxis >> 16) {
            best = std::max(best, d);
        } else {
            st.push_back({n + 1, d + 1});
            st.push_back({m_nodes[n].m_offset, d + 1});
        }
    }
    return best;
}

bool BVH::validate()
{
    std::vector<char> reached(m_elements.size(), 0);
    if (m_nodes.empty()) return m_elements.empty();
    bool ok = validateRecursive(0, reached);
    for (char r : reached)
        if (!r) return false;
    return ok;
}

bool BVH::validateRecursive(uint32_t node, std::vector<char>& reached)
{
    const uint32_t count = m_nodes[node].m_primitiveCountAxis >> 16;
    if (count) {
        for (uint32_t i = 0; i < count; ++i) {
            const size_t e = (size_t)m_nodes[node].m_offset + i;
            if (e >= reached.size() || reached[e]) return false;
            reached[e] = 1;
        }
        return true;
    }
    if (node + 1 >= m_nodes.size() || m_nodes[node].m_offset >= m_nodes.size()) return false;
    return validateRecursive(node + 1, reached) && validateRecursive(m_nodes[node].m_offset, reached);
}

uint32_t BVH::buildInto(std::vector<BVHNode>& out, size_t begin, size_t end)
{
    const uint32_t nodeIndex = static_cast<uint32_t>(out.size());
    out.push_back({});
    BVHNode node = {};
    node.m_aabb.m_min = vec3(std::numeric_limits<float>::max());
    node.m_aabb.m_max = vec3(std::numeric_limits<float>::lowest());
    for (size_t i = begin; i < end; ++i) node.m_aabb = merge(node.m_aabb, m_elements[i].getAABB());

    if ((end - begin) > m_maxLeafElements) {
        struct Bin {
            uint32_t count = 0;
            AABB aabb = AABB{vec3(std::numeric_limits<float>::max()), vec3(std::numeric_limits<float>::lowest())};
        };
        Bin bins[3][8];
        const vec3 extent = max(node.m_aabb.m_max - node.m_aabb.m_min, vec3(0.00000001f));

        // bin by centroid (relative offset uses the reciprocal-multiply vec3 division, BVH.cpp:109)
        for (size_t i = begin; i < end; ++i) {
            const AABB e = m_elements[i].getAABB();
            const vec3 centroid = (e.m_min + e.m_max) * 0.5f;
            const vec3 rel = (centroid - node.m_aabb.m_min) / extent;
            for (int j = 0; j < 3; ++j) {
                int bin = toIntX86(rel[j] * 8.0f);
                bin = bin < 0 ? 0 : bin > 7 ? 7 : bin;
                bins[j][bin].count += 1;
                bins[j][bin].aabb = merge(bins[j][bin].aabb, e);
            }
        }

        const float invArea = 1.0f / std::max(calcSurfaceArea(node.m_aabb.m_min, node.m_aabb.m_max), 0.000000001f);
        float lowestCost = std::numeric_limits<float>::max();
        uint32_t bestAxis = 0, bestBin = 0;
        for (uint32_t i = 0; i < 3; ++i) {
            for (uint32_t j = 0; j < 7; ++j) {
                AABB a0{vec3(std::numeric_limits<float>::max()), vec3(std::numeric_limits<float>::lowest())};
                AABB a1 = a0;
                uint32_t c0 = 0, c1 = 0;
                for (uint32_t k = 0; k <= j; ++k) { a0 = merge(a0, bins[i][k].aabb); c0 += bins[i][k].count; }
                for (uint32_t k = j + 1; k < 8; ++k) { a1 = merge(a1, bins[i][k].aabb); c1 += bins[i][k].count; }
                const float s0 = calcSurfaceArea(a0.m_min, a0.m_max);
                const float s1 = calcSurfaceArea(a1.m_min, a1.m_max);
                float cost = 0.125f + ((float)c0 * s0 + (float)c1 * s1) * invArea;
                cost = (c0 == 0 || c1 == 0) ? std::numeric_limits<float>::max() : cost;
                if (cost < lowestCost) {   // strict: the first minimum (axis-major) wins
                    lowestCost = cost;
                    bestAxis = i;
                    bestBin = j;
                }
            }
        }

        // partition (true division here, BVH.cpp:180, unlike the binning pass)
        const float nodeMin = node.m_aabb.m_min[(int)bestAxis];
        const float ext = extent[(int)bestAxis];
        const int axis = (int)bestAxis;
        CpuHittable* mid = std::partition(m_elements.data() + begin, m_elements.data() + end, [&](const CpuHittable& item) {
            const AABB e = item.getAABB();
            const vec3 centroid = (e.m_min + e.m_max) * 0.5f;
            const float rel = ((centroid[axis] - nodeMin) / ext);
            int bin = toIntX86(8.0f * rel);
            bin = bin < 0 ? 0 : bin > 7 ? 7 : bin;
            return static_cast<uint32_t>(bin) <= bestBin;
        });
        size_t split = static_cast<size_t>(mid - m_elements.data());

        if (split == begin || split == end) {
            // median fallback; the axis rule is the reference's (not the largest extent), BVH.cpp:193
            bestAxis = (extent[0] < extent[1]) ? 0 : (extent[1] < extent[2]) ? 1 : 2;
            split = (begin + end) / 2;
            const int ax = (int)bestAxis;
            std::nth_element(m_elements.data() + begin, m_elements.data() + split, m_elements.data() + end,
                             [ax](const CpuHittable& lhs, const CpuHittable& rhs) {
                                 const vec3 lc = (lhs.getAABB().m_min + lhs.getAABB().m_max) * 0.5f;
                                 const vec3 rc = (rhs.getAABB().m_min + rhs.getAABB().m_max) * 0.5f;
                                 return lc[ax] < rc[ax];
                             });
        }
        bool spawn = false;
        if (m_spareThreads && std::min(split - begin, end - split) >= 4096) {
            spawn = m_spareThreads->fetch_sub(1) > 0;
            if (!spawn) m_spareThreads->fetch_add(1);
        }
        if (spawn) {
            std::vector<BVHNode> left;
            left.reserve(2 * (split - begin));
            auto job = std::async(std::launch::async, [&] {
                buildInto(left, begin, split);
                m_spareThreads->fetch_add(1);
            });
            std::vector<BVHNode> right;
            right.reserve(2 * (end - split));
            buildInto(right, split, end);
            job.get();
            appendSubtree(out, left);                    // left child = nodeIndex + 1
            node.m_offset = static_cast<uint32_t>(out.size());
            appendSubtree(out, right);
        } else {
            buildInto(out, begin, split);
            node.m_offset = buildInto(out, split, end);
        }
        node.m_primitiveCountAxis |= (bestAxis << 8);
    } else {
        node.m_offset = static_cast<uint32_t>(begin);
        node.m_primitiveCountAxis |= static_cast<uint32_t>(end - begin) << 16;
    }
    out[nodeIndex] = node;
    return nodeIndex;
}
