// C ABI of the host layer (include/pt_host.h).
#include <chrono>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "host_internal.h"
#include "pathtracer_amd.hpp"
#include "pt_host.h"

namespace {

thread_local std::string g_lastError;

int setError(int code, const std::string& msg)
{
    g_lastError = msg;
    return code;
}

struct HostTexture {
    uint32_t w = 0, h = 0;
    std::vector<float> rgba;
};

} // namespace

struct pth_scene {
    ptamd::SceneDesc desc;
    BVH bvh;
    std::vector<HostTexture> textures;
    std::string path;
    pt_camera camera;
    double parseMs = 0.0, bvhMs = 0.0;
};

struct pth_renderer {
    std::unique_ptr<Pathtracer> pt;
};

static std::string resolvePath(const std::string& scene, const std::string& p)
{
    FILE* f = fopen(p.c_str(), "rb");
    if (f) { fclose(f); return p; }
    const size_t slash = scene.find_last_of('/');
    if (slash == std::string::npos) return p;
    std::string alt = scene.substr(0, slash + 1) + p;
    f = fopen(alt.c_str(), "rb");
    if (f) { fclose(f); return alt; }
    return p;
}

static uint32_t hostTextureLoader(void* user, const std::string& path)
{
    pth_scene* s = (pth_scene*)user;
    if (s->textures.size() >= PT_MAX_TEXTURES) return 0;
    HostTexture t;
    std::string err;
    if (!ptamd::loadImageRGBA32F(resolvePath(s->path, path), t.rgba, t.w, t.h, err)) return 0;
    s->textures.push_back(std::move(t));
    return (uint32_t)s->textures.size();
}

extern "C" {

PT_API const char* pth_last_error(void) { return g_lastError.c_str(); }

PT_API int pth_scene_load(const char* path, uint32_t width, uint32_t height, pth_scene** out)
{
    if (!path || !out || width == 0 || height == 0) return setError(PT_ERR_ARG, "pth_scene_load: invalid argument");
    *out = nullptr;
    auto s = std::make_unique<pth_scene>();
    s->path = path;
    std::string err;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    if (!ptamd::parseSceneFile(path, s->desc, err, hostTextureLoader, s.get())) return setError(PT_ERR_ARG, err);
    const auto t1 = clk::now();
    if (!s->desc.objects.empty()) {
        s->bvh.build(s->desc.objects.size(), s->desc.objects.data(), 4);
        s->bvhMs = std::chrono::duration<double, std::milli>(clk::now() - t1).count();
        if (!s->bvh.validate()) return setError(PT_ERR_STATE, "BVH validation failed");
    }
    s->parseMs = std::chrono::duration<double, std::milli>(t1 - t0).count();
    const Camera cam(s->desc.cameraPosition, s->desc.cameraLookAt, vec3(0.0f, 1.0f, 0.0f),
                     ptamd::radians(s->desc.cameraFovyDegrees), (float)width / height);
    s->camera = cam.toDevice();
    *out = s.release();
    return PT_OK;
}

PT_API void pth_scene_free(pth_scene* scene) { delete scene; }

PT_API int pth_scene_timing(const pth_scene* s, double* parse_ms, double* bvh_ms)
{
    if (!s) return setError(PT_ERR_ARG, "null scene");
    if (parse_ms) *parse_ms = s->parseMs;
    if (bvh_ms) *bvh_ms = s->bvhMs;
    return PT_OK;
}

PT_API uint32_t pth_scene_object_count(const pth_scene* s) { return s ? (uint32_t)s->desc.objects.size() : 0; }
PT_API uint32_t pth_scene_node_count(const pth_scene* s) { return s ? (uint32_t)s->bvh.getNodes().size() : 0; }
PT_API uint32_t pth_scene_bvh_depth(const pth_scene* s)
{
    return (s && !s->bvh.getNodes().empty()) ? s->bvh.getDepth(0) : 0;
}

PT_API int pth_scene_objects(const pth_scene* s, pt_hittable* objects, float* aabbs)
{
    if (!s) return setError(PT_ERR_ARG, "null scene");
    for (size_t i = 0; i < s->desc.objects.size(); ++i) {
        const CpuHittable& h = s->desc.objects[i];
        if (objects) objects[i] = h.getGpuHittable();
        if (aabbs)
            for (int k = 0; k < 3; ++k) {
                aabbs[6 * i + k] = h.getAABB().m_min[k];
                aabbs[6 * i + 3 + k] = h.getAABB().m_max[k];
            }
    }
    return PT_OK;
}

PT_API int pth_scene_bvh(const pth_scene* s, pt_bvh_node* nodes, pt_hittable* prims)
{
    if (!s) return setError(PT_ERR_ARG, "null scene");
    const auto& n = s->bvh.getNodes();
    const auto& e = s->bvh.getElements();
    if (nodes)
        for (size_t i = 0; i < n.size(); ++i) nodes[i] = ptamd::toDeviceNode(n[i]);
    if (prims)
        for (size_t i = 0; i < e.size(); ++i) prims[i] = e[i].getGpuHittable();
    return PT_OK;
}

PT_API int pth_scene_camera(const pth_scene* s, pt_camera* camera)
{
    if (!s || !camera) return setError(PT_ERR_ARG, "invalid argument");
    *camera = s->camera;
    return PT_OK;
}

PT_API uint32_t pth_scene_skybox(const pth_scene* s) { return s ? s->desc.skyboxHandle : 0; }
PT_API uint32_t pth_scene_texture_count(const pth_scene* s) { return s ? (uint32_t)s->textures.size() : 0; }

PT_API int pth_scene_texture_info(const pth_scene* s, uint32_t handle, uint32_t* w, uint32_t* h)
{
    if (!s || handle == 0 || handle > s->textures.size()) return setError(PT_ERR_ARG, "invalid texture handle");
    if (w) *w = s->textures[handle - 1].w;
    if (h) *h = s->textures[handle - 1].h;
    return PT_OK;
}

PT_API int pth_scene_texture_data(const pth_scene* s, uint32_t handle, float* rgba)
{
    if (!s || !rgba || handle == 0 || handle > s->textures.size()) return setError(PT_ERR_ARG, "invalid texture handle");
    const auto& t = s->textures[handle - 1];
    memcpy(rgba, t.rgba.data(), t.rgba.size() * sizeof(float));
    return PT_OK;
}

PT_API int pth_camera_make(const float* position, const float* lookat, const float* up, float fovy, float aspect,
                           pt_camera* out)
{
    if (!position || !lookat || !up || !out) return setError(PT_ERR_ARG, "invalid argument");
    const Camera c(vec3(position[0], position[1], position[2]), vec3(lookat[0], lookat[1], lookat[2]),
                   vec3(up[0], up[1], up[2]), fovy, aspect);
    *out = c.toDevice();
    return PT_OK;
}

static Camera camera_from_device(const pt_camera& d)
{
    Camera c(vec3(0.0f, 0.0f, 0.0f), vec3(0.0f, 0.0f, -1.0f), vec3(0.0f, 1.0f, 0.0f), 1.0f, 1.0f);
    c.m_tanHalfFovy = d.tan_half_fovy;
    c.m_aspectRatio = d.aspect_ratio;
    c.m_origin = vec3(d.origin[0], d.origin[1], d.origin[2]);
    c.m_lowerLeftCorner = vec3(d.lower_left_corner[0], d.lower_left_corner[1], d.lower_left_corner[2]);
    c.m_horizontal = vec3(d.horizontal[0], d.horizontal[1], d.horizontal[2]);
    c.m_vertical = vec3(d.vertical[0], d.vertical[1], d.vertical[2]);
    c.m_right = vec3(d.right[0], d.right[1], d.right[2]);
    c.m_up = vec3(d.up[0], d.up[1], d.up[2]);
    c.m_backward = vec3(d.backward[0], d.backward[1], d.backward[2]);
    return c;
}

PT_API int pth_camera_rotate(pt_camera* cam, float pitch, float yaw, float roll)
{
    if (!cam) return setError(PT_ERR_ARG, "invalid argument");
    Camera c = camera_from_device(*cam);
    c.rotate(pitch, yaw, roll);
    *cam = c.toDevice();
    return PT_OK;
}

PT_API int pth_camera_translate(pt_camera* cam, float x, float y, float z)
{
    if (!cam) return setError(PT_ERR_ARG, "invalid argument");
    Camera c = camera_from_device(*cam);
    c.translate(x, y, z);
    *cam = c.toDevice();
    return PT_OK;
}

PT_API float pth_radians(float degrees) { return ptamd::radians(degrees); }

#define PTH_GUARD_BEGIN                      \
    ptamd::g_throwOnError = true;            \
    try {
#define PTH_GUARD_END                                        \
    } catch (const ptamd::Error& e) {                        \
        return setError(e.code, e.what());                   \
    } catch (const std::exception& e) {                     \
        return setError(PT_ERR_STATE, e.what());             \
    }

PT_API int pth_renderer_create(uint32_t width, uint32_t height, int device, uint32_t row_offset, uint32_t row_stride,
                               pth_renderer** out)
{
    if (!out) return setError(PT_ERR_ARG, "invalid argument");
    *out = nullptr;
    PTH_GUARD_BEGIN
    auto r = std::make_unique<pth_renderer>();
    r->pt = std::make_unique<Pathtracer>(width, height, device, row_offset, row_stride);
    *out = r.release();
    return PT_OK;
    PTH_GUARD_END
}

PT_API int pth_renderer_create_banded(uint32_t width, uint32_t height, int device, uint32_t band_rows,
                                      uint32_t band_offset, uint32_t band_stride, pth_renderer** out)
{
    if (!out) return setError(PT_ERR_ARG, "invalid argument");
    *out = nullptr;
    PTH_GUARD_BEGIN
    auto r = std::make_unique<pth_renderer>();
    r->pt = std::make_unique<Pathtracer>(width, height, Pathtracer::Tile{device, band_rows, band_offset, band_stride});
    *out = r.release();
    return PT_OK;
    PTH_GUARD_END
}

PT_API int pth_renderer_create_group(uint32_t width, uint32_t height, int ndev, const int* devices, uint32_t band_rows,
                                     pth_renderer** out)
{
    if (!out || ndev < 1 || !devices) return setError(PT_ERR_ARG, "invalid argument");
    *out = nullptr;
    PTH_GUARD_BEGIN
    auto r = std::make_unique<pth_renderer>();
    r->pt = std::make_unique<Pathtracer>(width, height, std::vector<int>(devices, devices + ndev), band_rows);
    *out = r.release();
    return PT_OK;
    PTH_GUARD_END
}

PT_API float pth_renderer_gather_ms(const pth_renderer* r) { return r ? r->pt->lastGatherMs() : 0.0f; }

PT_API void pth_renderer_destroy(pth_renderer* r) { delete r; }

PT_API int pth_renderer_load_scene(pth_renderer* r, const char* path, pt_camera* camera)
{
    if (!r || !path) return setError(PT_ERR_ARG, "invalid argument");
    PTH_GUARD_BEGIN
    Params p;
    p.m_width = r->pt->width();
    p.m_height = r->pt->height();
    p.m_inputFilepath = path;
    // loadScene() terminates on unreadable / malformed files like the reference; check first.
    ptamd::SceneDesc probe;
    std::string err;
    if (!ptamd::parseSceneFile(path, probe, err, nullptr, nullptr)) return setError(PT_ERR_ARG, err);
    const Camera cam = loadScene(*r->pt, p);
    if (camera) *camera = cam.toDevice();
    return PT_OK;
    PTH_GUARD_END
}

PT_API int pth_renderer_render(pth_renderer* r, const pt_camera* camera, uint32_t spp, uint32_t chunks, int ignore_history)
{
    if (!r || !camera) return setError(PT_ERR_ARG, "invalid argument");
    PTH_GUARD_BEGIN
    Camera cam(vec3(0.0f), vec3(0.0f, 0.0f, -1.0f), vec3(0.0f, 1.0f, 0.0f), 1.0f, 1.0f);
    cam.m_tanHalfFovy = camera->tan_half_fovy;
    cam.m_aspectRatio = camera->aspect_ratio;
    for (int i = 0; i < 3; ++i) {
        cam.m_origin[i] = camera->origin[i];
        cam.m_lowerLeftCorner[i] = camera->lower_left_corner[i];
        cam.m_horizontal[i] = camera->horizontal[i];
        cam.m_vertical[i] = camera->vertical[i];
        cam.m_right[i] = camera->right[i];
        cam.m_up[i] = camera->up[i];
        cam.m_backward[i] = camera->backward[i];
    }
    r->pt->renderChunks(cam, spp, chunks, ignore_history != 0);
    return PT_OK;
    PTH_GUARD_END
}

PT_API float pth_renderer_timing(const pth_renderer* r) { return r ? r->pt->getTiming() : 0.0f; }
PT_API uint32_t pth_renderer_frames(const pth_renderer* r) { return r ? r->pt->accumulatedFrames() : 0; }
PT_API uint32_t pth_renderer_local_rows(const pth_renderer* r) { return r ? r->pt->localRows() : 0; }

PT_API const float* pth_renderer_hdr(pth_renderer* r)
{
    if (!r) return nullptr;
    ptamd::g_throwOnError = true;
    try { return r->pt->getHDRImageData(); } catch (const std::exception& e) { setError(PT_ERR_HIP, e.what()); }
    return nullptr;
}

PT_API const uint8_t* pth_renderer_image(pth_renderer* r)
{
    if (!r) return nullptr;
    ptamd::g_throwOnError = true;
    try { return (const uint8_t*)r->pt->getImageData(); } catch (const std::exception& e) { setError(PT_ERR_HIP, e.what()); }
    return nullptr;
}

PT_API pt_context* pth_renderer_context(pth_renderer* r) { return r ? r->pt->context() : nullptr; }
PT_API pt_group* pth_renderer_group(pth_renderer* r) { return r ? r->pt->group() : nullptr; }

PT_API int pth_write_png(const char* path, uint32_t w, uint32_t h, const uint8_t* rgba, int flip)
{
    if (!path || !rgba) return setError(PT_ERR_ARG, "invalid argument");
    return ptamd::writePNG(path, w, h, rgba, flip != 0) ? PT_OK : setError(PT_ERR_STATE, "failed to write PNG");
}

PT_API int pth_write_hdr(const char* path, uint32_t w, uint32_t h, const float* rgba, int flip)
{
    if (!path || !rgba) return setError(PT_ERR_ARG, "invalid argument");
    return ptamd::writeHDR(path, w, h, rgba, flip != 0) ? PT_OK : setError(PT_ERR_STATE, "failed to write HDR");
}

} // extern "C"
