// Host math, Camera and Material of the C++ drop-in API (include/pathtracer_amd.hpp).
// Reference: src/pathtracer/vec3.inl:210-254, Camera.inl:4-62, Material.inl:9-18,
// SceneLoader.cpp:193-196.  Built with -ffp-contract=off: the camera computed here is passed
// bit-for-bit to the GPU, and must equal the reference's host-side construction.
#include <cmath>

#include "pathtracer_amd.hpp"

float length(const vec3& v) { return sqrtf(v.e[0] * v.e[0] + v.e[1] * v.e[1] + v.e[2] * v.e[2]); }

vec3 rotateAroundVector(const vec3& v, const vec3& axis, float cosAngle, float sinAngle)
{
    // vec3.inl:244-247 (Rodrigues)
    return v * cosAngle + cross(axis, v) * sinAngle + axis * dot(axis, v) * (1.0f - cosAngle);
}

Camera::Camera(const vec3& position, const vec3& lookat, const vec3& up, float fovy, float aspectRatio)
    : m_tanHalfFovy(tanf(fovy * 0.5f)),
      m_aspectRatio(aspectRatio),
      m_origin(position),
      m_lowerLeftCorner(-1.0f, -1.0f, -1.0f),
      m_horizontal(2.0f, 0.0f, 0.0f),
      m_vertical(0.0f, 2.0f, 0.0f)
{
    m_backward = normalize(m_origin - lookat);
    m_right = normalize(cross(up, m_backward));
    m_up = cross(m_backward, m_right);
    update();
}

void Camera::rotate(float pitch, float yaw, float /*roll*/)
{
    const float cosPitch = cosf(-pitch);
    const float sinPitch = sinf(-pitch);
    m_up = rotateAroundVector(m_up, m_right, cosPitch, sinPitch);
    m_backward = rotateAroundVector(m_backward, m_right, cosPitch, sinPitch);
    const float cosYaw = cosf(-yaw);
    const float sinYaw = sinf(-yaw);
    m_right = rotateAroundVector(m_right, vec3(0.0f, 1.0f, 0.0f), cosYaw, sinYaw);
    m_up = rotateAroundVector(m_up, vec3(0.0f, 1.0f, 0.0f), cosYaw, sinYaw);
    m_backward = rotateAroundVector(m_backward, vec3(0.0f, 1.0f, 0.0f), cosYaw, sinYaw);
    update();
}

void Camera::translate(float x, float y, float z)
{
    m_origin += x * m_right + y * m_up + z * m_backward;
    update();
}

void Camera::update()
{
    const float halfHeight = m_tanHalfFovy;
    const float halfWidth = m_aspectRatio * halfHeight;
    m_lowerLeftCorner = -halfWidth * m_right + -halfHeight * m_up - m_backward;
    m_horizontal = 2.0f * halfWidth * m_right;
    m_vertical = 2.0f * halfHeight * m_up;
}

pt_camera Camera::toDevice() const
{
    pt_camera c;
    c.tan_half_fovy = m_tanHalfFovy;
    c.aspect_ratio = m_aspectRatio;
    for (int i = 0; i < 3; ++i) {
        c.origin[i] = m_origin[i];
        c.lower_left_corner[i] = m_lowerLeftCorner[i];
        c.horizontal[i] = m_horizontal[i];
        c.vertical[i] = m_vertical[i];
        c.right[i] = m_right[i];
        c.up[i] = m_up[i];
        c.backward[i] = m_backward[i];
    }
    return c;
}

Material::Material(MaterialType type, const vec3& baseColor, const vec3& emissive, float roughness, float metalness,
                   uint32_t textureIndex)
    : m_baseColor(baseColor),
      m_roughness(roughness < 0.04f ? 0.04f : roughness), // minimum roughness (Material.inl:12)
      m_emissive(emissive),
      m_metalness(metalness),
      m_textureIndex(textureIndex),
      m_materialType(type)
{
}

namespace ptamd {
float radians(float degree) { return degree * (1.0f / 180.0f) * 3.14159265358979323846f; }
} // namespace ptamd
