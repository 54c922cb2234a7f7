// Internal helpers shared by the host sources of libpt_host.so.
#pragma once
#include <stdexcept>
#include <string>

#include "pathtracer_amd.hpp"

namespace ptamd {

// When set (the C ABI of pt_host.h does), Pathtracer errors throw instead of terminating.
extern thread_local bool g_throwOnError;

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline pt_bvh_node toDeviceNode(const BVHNode& n)
{
    pt_bvh_node d;
    for (int i = 0; i < 3; ++i) {
        d.aabb_min[i] = n.m_aabb.m_min[i];
        d.aabb_max[i] = n.m_aabb.m_max[i];
    }
    d.offset = n.m_offset;
    d.primitive_count_axis = n.m_primitiveCountAxis;
    return d;
}

} // namespace ptamd
