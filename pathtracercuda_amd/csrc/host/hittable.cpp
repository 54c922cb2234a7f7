// CpuHittable: object transform and world AABB (reference src/pathtracer/Hittable.cpp:6-190).
// The 3x4 world->object rows computed here are what the GPU intersects against, so the
// quaternion construction, its inverse and every product follow the reference's order.
#include <cfloat>
#include <cmath>
#include <cstring>

#include "pathtracer_amd.hpp"

namespace {

struct Quat { float x, y, z, w; };

void quatToRotMat(const Quat& q, float (&m)[3][3])
{
    const float qxx = q.x * q.x, qyy = q.y * q.y, qzz = q.z * q.z;
    const float qxz = q.x * q.z, qxy = q.x * q.y, qyz = q.y * q.z;
    const float qwx = q.w * q.x, qwy = q.w * q.y, qwz = q.w * q.z;
    m[0][0] = 1.0f - 2.0f * (qyy + qzz);
    m[0][1] = 2.0f * (qxy + qwz);
    m[0][2] = 2.0f * (qxz - qwy);
    m[1][0] = 2.0f * (qxy - qwz);
    m[1][1] = 1.0f - 2.0f * (qxx + qzz);
    m[1][2] = 2.0f * (qyz + qwx);
    m[2][0] = 2.0f * (qxz + qwy);
    m[2][1] = 2.0f * (qyz - qwx);
    m[2][2] = 1.0f - 2.0f * (qxx + qyy);
}

// world = T * R * S; returns its inverse rows S^-1 R^-1 T^-1 and the forward rows
void worldTransform(const vec3& position, const vec3& rotation, const vec3& scale, float (&l2w)[3][4], float (&w2l)[3][4])
{
    Quat q;
    {
        const vec3 c = vec3(cosf(rotation.x * 0.5f), cosf(rotation.y * 0.5f), cosf(rotation.z * 0.5f));
        const vec3 s = vec3(sinf(rotation.x * 0.5f), sinf(rotation.y * 0.5f), sinf(rotation.z * 0.5f));
        q.w = c.x * c.y * c.z + s.x * s.y * s.z;
        q.x = s.x * c.y * c.z - c.x * s.y * s.z;
        q.y = c.x * s.y * c.z + s.x * c.y * s.z;
        q.z = c.x * c.y * s.z - s.x * s.y * c.z;
    }
    Quat iq;
    {
        const float invDot = (1.0f / (q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w));
        iq.x = -q.x * invDot;
        iq.y = -q.y * invDot;
        iq.z = -q.z * invDot;
        iq.w = q.w * invDot;
    }
    {
        float ir[3][3];
        quatToRotMat(iq, ir);
        const vec3 invScale = 1.0f / scale;
        const vec3 np = -position;
        for (int k = 0; k < 3; ++k) {
            w2l[k][0] = invScale[k] * ir[0][k];
            w2l[k][1] = invScale[k] * ir[1][k];
            w2l[k][2] = invScale[k] * ir[2][k];
            w2l[k][3] = invScale[k] * dot(vec3(ir[0][k], ir[1][k], ir[2][k]), np);
        }
    }
    {
        float r[3][3];
        quatToRotMat(q, r);
        for (int k = 0; k < 3; ++k) {
            l2w[k][0] = scale.x * r[0][k];
            l2w[k][1] = scale.y * r[1][k];
            l2w[k][2] = scale.z * r[2][k];
            l2w[k][3] = position[k];
        }
    }
}

} // namespace

CpuHittable::CpuHittable()
    : m_invTransformRows{{1.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 1.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 1.0f, 0.0f}},
      m_material(),
      m_aabb{vec3(-1.0f), vec3(1.0f)},
      m_type(HittableType::SPHERE)
{
}

CpuHittable::CpuHittable(HittableType type, const vec3& position, const vec3& rotation, const vec3& scale,
                         const Material& material)
    : m_invTransformRows{{1.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 1.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 1.0f, 0.0f}},
      m_material(material),
      m_aabb{vec3(-1.0f), vec3(1.0f)},
      m_type(type)
{
    // 2-D primitives do not inflate their box along y (Hittable.cpp:124-128)
    vec3 adjustedScale = scale;
    if (m_type == HittableType::DISK || m_type == HittableType::QUAD) adjustedScale.y = 1.0f;

    float l2w[3][4], w2l[3][4];
    worldTransform(position, rotation, adjustedScale, l2w, w2l);
    memcpy(m_invTransformRows, w2l, sizeof(w2l));

    m_aabb.m_min = vec3(FLT_MAX);
    m_aabb.m_max = vec3(-FLT_MAX);
    float xe[2] = {-1.0f, 1.0f}, ye[2] = {-1.0f, 1.0f}, ze[2] = {-1.0f, 1.0f};
    if (m_type == HittableType::DISK || m_type == HittableType::QUAD) {
        ye[0] = -0.01f;
        ye[1] = 0.01f;
    } else if (m_type == HittableType::PARABOLOID) {
        ye[0] = 0.0f;
    }
    for (int z = 0; z < 2; ++z)
        for (int y = 0; y < 2; ++y)
            for (int x = 0; x < 2; ++x) {
                const vec3 corner(xe[x], ye[y], ze[z]);
                vec3 p;
                p.x = dot(corner, vec3(l2w[0][0], l2w[0][1], l2w[0][2])) + l2w[0][3];
                p.y = dot(corner, vec3(l2w[1][0], l2w[1][1], l2w[1][2])) + l2w[1][3];
                p.z = dot(corner, vec3(l2w[2][0], l2w[2][1], l2w[2][2])) + l2w[2][3];
                m_aabb.m_min = min(m_aabb.m_min, p);
                m_aabb.m_max = max(m_aabb.m_max, p);
            }
}

pt_hittable CpuHittable::getGpuHittable() const
{
    pt_hittable h;
    memset(&h, 0, sizeof(h));
    memcpy(h.inv_transform_rows, m_invTransformRows, sizeof(h.inv_transform_rows));
    for (int i = 0; i < 3; ++i) {
        h.base_color[i] = m_material.m_baseColor[i];
        h.emissive[i] = m_material.m_emissive[i];
    }
    h.roughness = m_material.m_roughness;
    h.metalness = m_material.m_metalness;
    h.texture_index = m_material.m_textureIndex;
    h.material_type = (uint32_t)m_material.m_materialType;
    h.type = (uint32_t)m_type;
    return h;
}
