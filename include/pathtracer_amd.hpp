// pathtracer_amd.hpp -- C++ drop-in API of the MI355X path tracer (libpt_host.so).
//
// Mirrors the public host surface of DoerriesT/PathtracerCUDA so its callers (SceneLoader.cpp,
// main.cpp) build unchanged against this library:
//   vec3 ops                 src/pathtracer/vec3.h:7-57
//   Camera                   src/pathtracer/Camera.h:4-23
//   Material / MaterialType  src/pathtracer/Material.h:9-32
//   CpuHittable / HittableType src/pathtracer/Hittable.h:9-56
//   BVHNode / BVH            src/pathtracer/BVH.h:6-31
//   Pathtracer               src/pathtracer/Pathtracer.h:12-68
//   Params                   src/Params.h:4-13
//   loadScene                src/SceneLoader.h:9, SceneLoader.cpp:124-348
// Differences (all additive): a Pathtracer can own a row-band tile of a larger image or span
// several GPUs of the process (RCCL gather), a device index can be chosen, and renderChunks()
// runs several render() calls in one launch.
// All host arithmetic follows the reference operation for operation (built with
// -ffp-contract=off) so BVHs, transforms and cameras are bit-identical to the reference's.
#pragma once

#include <cstddef>
#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

#include "pt_hip.h"

// ------------------------------------------------------------------------------------------------
// vec3 (vec3.h / vec3.inl semantics: v / s == (1 / s) * v, min uses <, max uses >=)
// ------------------------------------------------------------------------------------------------
#define PT_PI (3.14159265358979323846f)

struct vec3 {
    union {
        struct { float x, y, z; };
        struct { float r, g, b; };
        float e[3];
    };
    vec3() : e{0.0f, 0.0f, 0.0f} {}
    vec3(float e0, float e1, float e2) : e{e0, e1, e2} {}
    vec3(float s) : e{s, s, s} {}
    vec3 operator-() const { return vec3(-e[0], -e[1], -e[2]); }
    float operator[](int i) const { return e[i]; }
    float& operator[](int i) { return e[i]; }
    vec3& operator+=(const vec3& v) { e[0] += v.e[0]; e[1] += v.e[1]; e[2] += v.e[2]; return *this; }
    vec3& operator*=(float t) { e[0] *= t; e[1] *= t; e[2] *= t; return *this; }
    vec3& operator*=(const vec3& t) { e[0] *= t.x; e[1] *= t.y; e[2] *= t.z; return *this; }
    vec3& operator/=(float t) { return *this *= 1 / t; }
};

inline vec3 operator+(const vec3& u, const vec3& v) { return vec3(u.e[0] + v.e[0], u.e[1] + v.e[1], u.e[2] + v.e[2]); }
inline vec3 operator+(const vec3& u, float v) { return vec3(u.e[0] + v, u.e[1] + v, u.e[2] + v); }
inline vec3 operator+(float u, const vec3& v) { return v + u; }
inline vec3 operator-(const vec3& u, const vec3& v) { return vec3(u.e[0] - v.e[0], u.e[1] - v.e[1], u.e[2] - v.e[2]); }
inline vec3 operator-(const vec3& u, float v) { return vec3(u.e[0] - v, u.e[1] - v, u.e[2] - v); }
inline vec3 operator-(float u, const vec3& v) { return -v + u; }
inline vec3 operator*(const vec3& u, const vec3& v) { return vec3(u.e[0] * v.e[0], u.e[1] * v.e[1], u.e[2] * v.e[2]); }
inline vec3 operator*(float t, const vec3& v) { return vec3(t * v.e[0], t * v.e[1], t * v.e[2]); }
inline vec3 operator*(const vec3& v, float t) { return t * v; }
inline vec3 operator/(const vec3& v, const vec3& t) { return vec3(1.0f / t.x, 1.0f / t.y, 1.0f / t.z) * v; }
inline vec3 operator/(const vec3& v, float t) { return (1.0f / t) * v; }
inline vec3 operator/(float v, const vec3& t) { return vec3(1.0f / t.x, 1.0f / t.y, 1.0f / t.z) * v; }
inline bool operator==(const vec3& u, const vec3& v) { return u.x == v.x && u.y == v.y && u.z == v.z; }
inline float dot(const vec3& u, const vec3& v) { return u.e[0] * v.e[0] + u.e[1] * v.e[1] + u.e[2] * v.e[2]; }
inline vec3 cross(const vec3& u, const vec3& v)
{
    return vec3(u.e[1] * v.e[2] - u.e[2] * v.e[1], u.e[2] * v.e[0] - u.e[0] * v.e[2], u.e[0] * v.e[1] - u.e[1] * v.e[0]);
}
float length(const vec3& v);
inline vec3 min(const vec3& a, const vec3& b)
{
    return vec3(a.x < b.x ? a.x : b.x, a.y < b.y ? a.y : b.y, a.z < b.z ? a.z : b.z);
}
inline vec3 max(const vec3& a, const vec3& b)
{
    return vec3(a.x >= b.x ? a.x : b.x, a.y >= b.y ? a.y : b.y, a.z >= b.z ? a.z : b.z);
}
inline vec3 normalize(const vec3& v) { return v / length(v); }
vec3 rotateAroundVector(const vec3& v, const vec3& axis, float cosAngle, float sinAngle);

// ------------------------------------------------------------------------------------------------
// Camera (Camera.h / Camera.inl); fovy in radians
// ------------------------------------------------------------------------------------------------
class Camera {
public:
    Camera(const vec3& position, const vec3& lookat, const vec3& up, float fovy, float aspectRatio);
    void rotate(float pitch, float yaw, float roll);
    void translate(float x, float y, float z);
    void update();
    pt_camera toDevice() const;

    float m_tanHalfFovy;
    float m_aspectRatio;
    vec3 m_origin;
    vec3 m_lowerLeftCorner;
    vec3 m_horizontal;
    vec3 m_vertical;
    vec3 m_right;
    vec3 m_up;
    vec3 m_backward;
};

// ------------------------------------------------------------------------------------------------
// Material, shapes
// ------------------------------------------------------------------------------------------------
enum class MaterialType : uint32_t { LAMBERT, GGX, LAMBERT_GGX };
enum class HittableType : uint32_t { SPHERE, CYLINDER, DISK, CONE, PARABOLOID, QUAD, CUBE };

class Material {
public:
    Material(MaterialType type = MaterialType::LAMBERT, const vec3& baseColor = vec3(1.0f), const vec3& emissive = vec3(0.0f),
             float roughness = 0.5f, float metalness = 0.0f, uint32_t textureIndex = 0);

    vec3 m_baseColor;
    float m_roughness;
    vec3 m_emissive;
    float m_metalness;
    uint32_t m_textureIndex;
    MaterialType m_materialType;
};

struct AABB {
    vec3 m_min;
    vec3 m_max;
};

// Scene object with the data needed to build the BVH (Hittable.h:40-56); rotation in radians.
class CpuHittable {
public:
    CpuHittable();
    CpuHittable(HittableType type, const vec3& position, const vec3& rotation, const vec3& scale, const Material& material);
    const AABB& getAABB() const { return m_aabb; }
    pt_hittable getGpuHittable() const;
    HittableType type() const { return m_type; }
    const float* invTransformRows() const { return &m_invTransformRows[0][0]; }
    const Material& material() const { return m_material; }

private:
    float m_invTransformRows[3][4];
    Material m_material;
    AABB m_aabb;
    HittableType m_type;
};

// ------------------------------------------------------------------------------------------------
// BVH (BVH.h): binned SAH, 8 bins x 3 axes, depth-first layout, left child = node + 1
// ------------------------------------------------------------------------------------------------
struct BVHNode {
    AABB m_aabb;
    uint32_t m_offset;
    uint32_t m_primitiveCountAxis;
};

class BVH {
public:
    void build(size_t elementCount, const CpuHittable* elements, uint32_t maxLeafElements);
    const std::vector<BVHNode>& getNodes() const { return m_nodes; }
    const std::vector<CpuHittable>& getElements() const { return m_elements; }
    uint32_t getDepth(uint32_t node = 0) const;
    bool validate();

private:
    uint32_t m_maxLeafElements = 1;
    std::vector<BVHNode> m_nodes;
    std::vector<CpuHittable> m_elements;
    uint32_t buildInto(std::vector<BVHNode>& out, size_t begin, size_t end);
    std::atomic<int>* m_spareThreads = nullptr;   // worker-thread budget during build()
    bool validateRecursive(uint32_t node, std::vector<char>& reached);
};

// ------------------------------------------------------------------------------------------------
// Pathtracer (Pathtracer.h:12-68)
// ------------------------------------------------------------------------------------------------
class Pathtracer {
public:
    // openglPixelBuffer is accepted for source compatibility; GL interop is not supported (must be 0).
    explicit Pathtracer(uint32_t width, uint32_t height, unsigned int openglPixelBuffer = 0);
    // Row tile of a width x height image on `device`: rows y = rowOffset + k * rowStride.
    Pathtracer(uint32_t width, uint32_t height, int device, uint32_t rowOffset, uint32_t rowStride);
    // Band tile on `device`: the bands of bandRows rows b = bandOffset + k * bandStride
    // (pt_create_banded); bandRows = 1 is the row tile above.
    struct Tile {
        int device;
        uint32_t bandRows, bandOffset, bandStride;
    };
    Pathtracer(uint32_t width, uint32_t height, const Tile& tile);
    // The whole image on several GPUs of this process (the CLI's -gpus N): device i renders the row
    // bands i, i + N, ... and getHDRImageData / getImageData return the full image, gathered on
    // devices[0] over RCCL (pt_group_*).  Bit-identical to a single-device render.
    Pathtracer(uint32_t width, uint32_t height, const std::vector<int>& devices, uint32_t bandRows = 8);
    Pathtracer(const Pathtracer&) = delete;
    Pathtracer(const Pathtracer&&) = delete;
    Pathtracer& operator=(const Pathtracer&) = delete;
    Pathtracer& operator=(const Pathtracer&&) = delete;
    ~Pathtracer();

    void setScene(size_t count, const CpuHittable* hittables);
    void render(const Camera& camera, uint32_t spp, bool ignoreHistory);
    // `chunks` successive render(camera, spp, ...) calls in one launch (first one honours
    // ignoreHistory); bit-identical to the loop.  Timing covers the whole launch.
    void renderChunks(const Camera& camera, uint32_t spp, uint32_t chunks, bool ignoreHistory);
    float getTiming() const;
    uint32_t loadTexture(const char* path);
    void setSkyboxTextureHandle(uint32_t handle);
    float* getHDRImageData();
    char* getImageData();

    // additions
    uint32_t width() const { return m_width; }
    uint32_t height() const { return m_height; }
    uint32_t localRows() const;     // rows of the image data this object returns
    uint32_t accumulatedFrames() const { return m_accumulatedFrames; }
    pt_context* context() const { return m_ctx; }    // device context (devices[0]'s for a group)
    pt_group* group() const { return m_group; }      // null unless multi-device
    int deviceCount() const { return m_group ? pt_group_size(m_group) : 1; }
    float lastGatherMs() const { return m_gatherMs; }
    const BVH& bvh() const { return m_bvh; }

private:
    uint32_t m_width;
    uint32_t m_height;
    uint32_t m_hittableCount = 0;
    uint32_t m_nodeCount = 0;
    float m_timing = 0.0f;
    uint32_t m_accumulatedFrames = 0;
    uint32_t m_textureCount = 0;
    uint32_t m_skyboxTextureHandle = 0;
    std::vector<float> m_cpuAccumBuffer;
    std::vector<char> m_cpuResultBuffer;
    pt_context* m_ctx = nullptr;
    pt_group* m_group = nullptr;
    float m_gatherMs = 0.0f;
    BVH m_bvh;
    void allocHostBuffers();
    void check(int rc, const char* what) const;
};

// ------------------------------------------------------------------------------------------------
// CLI parameters and scene loading (Params.h, SceneLoader.h)
// ------------------------------------------------------------------------------------------------
struct Params {
    unsigned int m_width = 1024;
    unsigned int m_height = 1024;
    unsigned int m_spp = 1024;
    const char* m_inputFilepath = nullptr;
    const char* m_outputFilepath = nullptr;
    bool m_showWindow = false;
    bool m_enableControls = false;
    bool m_outputHdr = false;
    // additions
    unsigned int m_chunk = 8;        // samples per render() call of the headless loop (main.cpp:272)
    bool m_singleLaunch = true;      // run all chunks in one launch (bit-identical; CLI -call_loop: false)
};

Camera loadScene(Pathtracer& pathtracer, const Params& params);

namespace ptamd {

// Scene description produced by the JSON loader without touching a GPU.
struct SceneDesc {
    std::vector<CpuHittable> objects;
    std::vector<std::string> texturePaths;   // index = handle - 1 of successfully loaded textures
    uint32_t skyboxHandle = 0;
    bool hasObjects = false;                 // "objects" array present (setScene is called)
    bool hasSkybox = false;                  // "skybox" string present
    vec3 cameraPosition = vec3(0.0f);
    vec3 cameraLookAt = vec3(0.0f, 0.0f, -1.0f);
    float cameraFovyDegrees = 60.0f;
};

// Parses a scene file (SceneLoader.cpp:124-348 semantics).  `textureLoader` is called for each
// distinct texture path in order of first use and returns the handle (0 = failure).
bool parseSceneFile(const std::string& path, SceneDesc& out, std::string& error,
                    uint32_t (*textureLoader)(void* user, const std::string& path), void* user);

float radians(float degree);   // SceneLoader.cpp:193-196

// Image I/O (stb_image / stb_image_write semantics for the formats the project uses).
bool isHdrFile(const std::string& path);
bool loadImageRGBA32F(const std::string& path, std::vector<float>& rgba, uint32_t& w, uint32_t& h, std::string& error);
bool writePNG(const std::string& path, uint32_t w, uint32_t h, const uint8_t* rgba, bool flipVertically);
bool writeHDR(const std::string& path, uint32_t w, uint32_t h, const float* rgba, bool flipVertically);

} // namespace ptamd
