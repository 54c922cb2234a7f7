// Pathtracer: host owner of one device context (reference src/pathtracer/Pathtracer.cpp:30-339).
// Host side keeps the reference's responsibilities: BVH build + validation on setScene, texture
// decode on loadTexture, the accumulated-frame counter and the two normalisations of
// getHDRImageData / getImageData.  Device work goes through the C ABI of include/pt_hip.h.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>

#include "host_internal.h"
#include "pathtracer_amd.hpp"

namespace ptamd {
thread_local bool g_throwOnError = false;
}

void Pathtracer::check(int rc, const char* what) const
{
    if (rc == PT_OK) return;
    char buf[1024];
    const char* detail = m_group ? pt_group_last_error(m_group) : (m_ctx ? pt_last_error(m_ctx) : "");
    snprintf(buf, sizeof(buf), "HIP error = %d at %s '%s'", rc, what, detail);
    if (ptamd::g_throwOnError) throw ptamd::Error(rc, buf);
    // reference behaviour (Pathtracer.cpp:17-28): report and terminate
    fprintf(stderr, "%s\n", buf);
    exit(EXIT_FAILURE);
}

Pathtracer::Pathtracer(uint32_t width, uint32_t height, unsigned int openglPixelBuffer)
    : Pathtracer(width, height, 0, 0u, 1u)
{
    if (openglPixelBuffer != 0) {
        const char* msg = "OpenGL pixel-buffer interop is not supported (headless renderer)";
        if (ptamd::g_throwOnError) throw ptamd::Error(PT_ERR_ARG, msg);
        fprintf(stderr, "%s\n", msg);
        exit(EXIT_FAILURE);
    }
}

Pathtracer::Pathtracer(uint32_t width, uint32_t height, int device, uint32_t rowOffset, uint32_t rowStride)
    : Pathtracer(width, height, Tile{device, 1u, rowOffset, rowStride})
{
}

Pathtracer::Pathtracer(uint32_t width, uint32_t height, const Tile& tile)
    : m_width(width), m_height(height)
{
    check(pt_create_banded(tile.device, width, height, tile.bandRows, tile.bandOffset, tile.bandStride, &m_ctx),
          "pt_create_banded");
    allocHostBuffers();
}

Pathtracer::Pathtracer(uint32_t width, uint32_t height, const std::vector<int>& devices, uint32_t bandRows)
    : m_width(width), m_height(height)
{
    // the reference hard-codes device 0 (Pathtracer.cpp:40); here every listed device renders a
    // share of the row bands and RCCL assembles the image on devices[0]
    check(pt_group_create((int)devices.size(), devices.data(), width, height, bandRows, &m_group), "pt_group_create");
    m_ctx = pt_group_context(m_group, 0);
    allocHostBuffers();
}

void Pathtracer::allocHostBuffers()
{
    const size_t npix = (size_t)localRows() * m_width;
    m_cpuAccumBuffer.resize(npix * 4);
    m_cpuResultBuffer.resize(npix * 4);
}

Pathtracer::~Pathtracer()
{
    if (m_group) pt_group_destroy(m_group);
    else pt_destroy(m_ctx);
}

uint32_t Pathtracer::localRows() const { return m_group ? m_height : pt_local_rows(m_ctx); }

void Pathtracer::setScene(size_t count, const CpuHittable* hittables)
{
    if (count == 0) {
        printf("Setting an empty scene is not allowed!\n");
        return;
    }
    m_bvh = BVH();
    m_bvh.build(count, hittables, 4);
    if (!m_bvh.validate()) check(PT_ERR_STATE, "BVH::validate");   // reference: assert(bvh.validate())
    const auto& nodes = m_bvh.getNodes();
    const auto& elems = m_bvh.getElements();
    std::vector<pt_bvh_node> dn(nodes.size());
    for (size_t i = 0; i < nodes.size(); ++i) dn[i] = ptamd::toDeviceNode(nodes[i]);
    std::vector<pt_hittable> dp(elems.size());
    for (size_t i = 0; i < elems.size(); ++i) dp[i] = elems[i].getGpuHittable();
    if (m_group)
        check(pt_group_set_scene(m_group, dn.data(), (uint32_t)dn.size(), dp.data(), (uint32_t)dp.size()), "pt_group_set_scene");
    else
        check(pt_set_scene(m_ctx, dn.data(), (uint32_t)dn.size(), dp.data(), (uint32_t)dp.size()), "pt_set_scene");
    m_nodeCount = (uint32_t)dn.size();
    m_hittableCount = (uint32_t)dp.size();
}

void Pathtracer::render(const Camera& camera, uint32_t spp, bool ignoreHistory)
{
    renderChunks(camera, spp, 1, ignoreHistory);
}

void Pathtracer::renderChunks(const Camera& camera, uint32_t spp, uint32_t chunks, bool ignoreHistory)
{
    if (ignoreHistory) m_accumulatedFrames = 0;
    m_timing = 0.0f;
    const pt_camera cam = camera.toDevice();
    float ms = 0.0f;
    if (m_group) check(pt_group_render(m_group, &cam, spp, chunks, ignoreHistory ? 1 : 0, &ms), "pt_group_render");
    else check(pt_render(m_ctx, &cam, spp, chunks, ignoreHistory ? 1 : 0, &ms), "pt_render");
    m_timing = ms;
    m_accumulatedFrames += chunks;
}

float Pathtracer::getTiming() const { return m_timing; }

uint32_t Pathtracer::loadTexture(const char* path)
{
    if (m_textureCount >= PT_MAX_TEXTURES) return 0;
    std::vector<float> rgba;
    uint32_t w = 0, h = 0;
    std::string err;
    if (!ptamd::loadImageRGBA32F(path, rgba, w, h, err)) return 0;     // failure -> null handle
    if (m_group) check(pt_group_set_texture(m_group, m_textureCount + 1, rgba.data(), w, h), "pt_group_set_texture");
    else check(pt_set_texture(m_ctx, m_textureCount + 1, rgba.data(), w, h), "pt_set_texture");
    ++m_textureCount;
    return m_textureCount;
}

void Pathtracer::setSkyboxTextureHandle(uint32_t handle)
{
    m_skyboxTextureHandle = handle;
    if (m_group) check(pt_group_set_skybox(m_group, handle), "pt_group_set_skybox");
    else check(pt_set_skybox(m_ctx, handle), "pt_set_skybox");
}

float* Pathtracer::getHDRImageData()
{
    if (m_group) {
        check(pt_group_gather(m_group, &m_gatherMs), "pt_group_gather");
        check(pt_group_read_accum(m_group, m_cpuAccumBuffer.data()), "pt_group_read_accum");
    } else {
        check(pt_read_accum(m_ctx, m_cpuAccumBuffer.data()), "pt_read_accum");
    }
    const float inv = 1.0f / fmaxf((float)m_accumulatedFrames, 1.0f);   // Pathtracer.cpp:307
    for (float& v : m_cpuAccumBuffer) v *= inv;
    return m_cpuAccumBuffer.data();
}

char* Pathtracer::getImageData()
{
    if (m_group) check(pt_group_tonemap(m_group, m_accumulatedFrames, (uint8_t*)m_cpuResultBuffer.data()), "pt_group_tonemap");
    else check(pt_tonemap(m_ctx, m_accumulatedFrames, (uint8_t*)m_cpuResultBuffer.data()), "pt_tonemap");
    return m_cpuResultBuffer.data();
}
