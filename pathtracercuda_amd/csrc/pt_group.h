// Multi-device group (pt_group_*): one context per device, one RCCL communicator.
// Part of the trace kernel's single translation unit: included by pt_kernels.hip after the C ABI
// definitions (pt_context, render_impl); not a standalone header.
#pragma once

// =============================================================================================
// Multi-device group: one context per device over interleaved row bands, one RCCL communicator
// per device (ncclCommInitAll, single process), and the framebuffer gather -- each device sends
// its rows to device 0 with grouped ncclSend/ncclRecv over xGMI, device 0 scatters them into the
// full image (unpermute_rows_kernel).  Replaces the reference's single hard-coded device
// (Pathtracer.cpp:40) behind the same Pathtracer interface (include/pathtracer_amd.hpp).
// =============================================================================================
struct pt_group {
    std::vector<int> devices;
    std::vector<pt_context*> ctx;
    std::vector<ncclComm_t> comms;
    std::vector<size_t> stageOff;     // float4 offset of each device's rows in `stage`
    uint32_t width = 0, height = 0, bandRows = 1;
    float4* stage = nullptr;          // device 0: the received rows of every device, concatenated
    float4* full = nullptr;           // device 0: the assembled image, height x width
    uchar4* ldr = nullptr;            // device 0: tonemap staging
    // `full` holds the accumulation as of these context epochs (every launch on a context, through
    // the group or directly on pt_group_context(i), bumps its epoch and so invalidates `full`)
    std::vector<uint64_t> gatherEpoch;
    std::string err;
};

static bool group_gathered(const pt_group* g)
{
    if (g->gatherEpoch.size() != g->ctx.size()) return false;
    for (size_t i = 0; i < g->ctx.size(); ++i)
        if (g->gatherEpoch[i] != g->ctx[i]->epoch) return false;
    return true;
}

static int gfail(pt_group* g, int code, const std::string& msg)
{
    if (g) g->err = msg;
    return code;
}

#define PT_NCCL_CHECK(g, expr)                                                                   \
    do {                                                                                         \
        ncclResult_t r_ = (expr);                                                                \
        if (r_ != ncclSuccess)                                                                   \
            return gfail((g), PT_ERR_HIP, std::string("RCCL error ") + ncclGetErrorString(r_) + \
                                              " at '" #expr "'");                                \
    } while (0)

#define PT_GHIP_CHECK(g, expr)                                                                   \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return gfail((g), PT_ERR_HIP, std::string("HIP error ") + hipGetErrorString(e_) +    \
                                              " at '" #expr "'");                                \
    } while (0)

// first failing context's status, with its message
static int gctx_rc(pt_group* g, const std::vector<int>& rc)
{
    for (size_t i = 0; i < rc.size(); ++i)
        if (rc[i] != PT_OK) return gfail(g, rc[i], "device " + std::to_string(g->devices[i]) + ": " + g->ctx[i]->err);
    return PT_OK;
}

extern "C" {

PT_API void pt_group_destroy(pt_group* g)
{
    if (!g) return;
    for (ncclComm_t c : g->comms)
        if (c) (void)ncclCommDestroy(c);
    if (!g->devices.empty()) (void)hipSetDevice(g->devices[0]);
    (void)hipFree(g->stage);
    (void)hipFree(g->full);
    (void)hipFree(g->ldr);
    for (pt_context* c : g->ctx) pt_destroy(c);
    delete g;
}

PT_API int pt_group_create(int ndev, const int* devices, uint32_t width, uint32_t height, uint32_t band_rows,
                           pt_group** out)
{
    if (!out || ndev < 1 || !devices) return PT_ERR_ARG;
    *out = nullptr;
    pt_group* g = new pt_group();
    g->devices.assign(devices, devices + ndev);
    g->width = width;
    g->height = height;
    g->bandRows = band_rows;
    auto bail = [&](int rc) { pt_group_destroy(g); return rc; };
    for (int i = 0; i < ndev; ++i)
        for (int j = 0; j < i; ++j)
            if (devices[i] == devices[j]) return bail(PT_ERR_ARG);      // one rank per device (RCCL)
    size_t staged = 0;
    for (int i = 0; i < ndev; ++i) {
        pt_context* c = nullptr;
        const int rc = pt_create_banded(devices[i], width, height, band_rows, (uint32_t)i, (uint32_t)ndev, &c);
        if (rc != PT_OK) return bail(rc);
        g->ctx.push_back(c);
        g->stageOff.push_back(staged);
        staged += (size_t)c->rows * width;
    }
    g->comms.assign(ndev, nullptr);
    if (ncclCommInitAll(g->comms.data(), ndev, devices) != ncclSuccess) {
        g->comms.clear();
        return bail(PT_ERR_HIP);
    }
    if (hipSetDevice(devices[0]) != hipSuccess) return bail(PT_ERR_HIP);
    if (hipMalloc(&g->stage, std::max<size_t>(staged, 1) * sizeof(float4)) != hipSuccess) return bail(PT_ERR_HIP);
    if (hipMalloc(&g->full, (size_t)width * height * sizeof(float4)) != hipSuccess) return bail(PT_ERR_HIP);
    *out = g;
    return PT_OK;
}

PT_API int pt_group_size(const pt_group* g) { return g ? (int)g->ctx.size() : 0; }

PT_API pt_context* pt_group_context(pt_group* g, int index)
{
    return (g && index >= 0 && index < (int)g->ctx.size()) ? g->ctx[index] : nullptr;
}

PT_API int pt_group_set_scene(pt_group* g, const pt_bvh_node* nodes, uint32_t node_count, const pt_hittable* prims,
                              uint32_t prim_count)
{
    if (!g) return PT_ERR_ARG;
    std::vector<int> rc;
    for (pt_context* c : g->ctx) rc.push_back(pt_set_scene(c, nodes, node_count, prims, prim_count));
    return gctx_rc(g, rc);
}

PT_API int pt_group_set_texture(pt_group* g, uint32_t handle, const float* rgba, uint32_t width, uint32_t height)
{
    if (!g) return PT_ERR_ARG;
    std::vector<int> rc;
    for (pt_context* c : g->ctx) rc.push_back(pt_set_texture(c, handle, rgba, width, height));
    return gctx_rc(g, rc);
}

PT_API int pt_group_set_skybox(pt_group* g, uint32_t handle)
{
    if (!g) return PT_ERR_ARG;
    std::vector<int> rc;
    for (pt_context* c : g->ctx) rc.push_back(pt_set_skybox(c, handle));
    return gctx_rc(g, rc);
}

PT_API int pt_group_render(pt_group* g, const pt_camera* camera, uint32_t spp, uint32_t chunks, int ignore_history,
                           float* gpu_ms)
{
    if (!g || !camera) return PT_ERR_ARG;
    const size_t n = g->ctx.size();
    std::vector<int> rc(n, PT_OK);
    std::vector<float> ms(n, 0.0f);
    auto one = [&](size_t i) { rc[i] = pt_render(g->ctx[i], camera, spp, chunks, ignore_history, &ms[i]); };
    if (n == 1) {
        one(0);
    } else {                                   // one host thread per device: the launches overlap
        std::vector<std::thread> th;
        for (size_t i = 0; i < n; ++i) th.emplace_back(one, i);
        for (auto& t : th) t.join();
    }
    if (gpu_ms) *gpu_ms = *std::max_element(ms.begin(), ms.end());
    return gctx_rc(g, rc);
}

PT_API int pt_group_gather(pt_group* g, float* host_ms)
{
    if (!g) return PT_ERR_ARG;
    const auto t0 = std::chrono::steady_clock::now();
    const size_t n = g->ctx.size();
    pt_context* root = g->ctx[0];
    // every context's stream is idle (pt_render is synchronous); one RCCL group: device i sends
    // its rows (rows_i x width float4, contiguous) to device 0, which receives them into `stage`
    PT_NCCL_CHECK(g, ncclGroupStart());
    for (size_t i = 0; i < n; ++i) {
        const size_t count = (size_t)g->ctx[i]->rows * g->width * 4;
        if (count == 0) continue;
        PT_NCCL_CHECK(g, ncclSend(g->ctx[i]->accum, count, ncclFloat, 0, g->comms[i], g->ctx[i]->stream));
        PT_NCCL_CHECK(g, ncclRecv(g->stage + g->stageOff[i], count, ncclFloat, (int)i, g->comms[0], root->stream));
    }
    PT_NCCL_CHECK(g, ncclGroupEnd());
    PT_GHIP_CHECK(g, hipSetDevice(root->device));
    for (size_t i = 0; i < n; ++i) {
        const size_t npix = (size_t)g->ctx[i]->rows * g->width;
        if (npix == 0) continue;
        unpermute_rows_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, root->stream>>>(
            g->full, g->stage + g->stageOff[i], g->width, g->ctx[i]->rows, (uint32_t)i, (uint32_t)n, root->bandShift);
        PT_GHIP_CHECK(g, hipGetLastError());
    }
    for (size_t i = 0; i < n; ++i) {
        PT_GHIP_CHECK(g, hipSetDevice(g->ctx[i]->device));
        PT_GHIP_CHECK(g, hipStreamSynchronize(g->ctx[i]->stream));
    }
    g->gatherEpoch.clear();
    for (pt_context* c : g->ctx) g->gatherEpoch.push_back(c->epoch);
    if (host_ms) *host_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return PT_OK;
}

PT_API int pt_group_read_accum(pt_group* g, float* dst)
{
    if (!g || !dst) return PT_ERR_ARG;
    if (!group_gathered(g)) {
        const int rc = pt_group_gather(g, nullptr);
        if (rc != PT_OK) return rc;
    }
    PT_GHIP_CHECK(g, hipSetDevice(g->devices[0]));
    PT_GHIP_CHECK(g, hipMemcpy(dst, g->full, (size_t)g->width * g->height * sizeof(float4), hipMemcpyDeviceToHost));
    return PT_OK;
}

PT_API int pt_group_tonemap(pt_group* g, uint32_t frames, uint8_t* dst)
{
    if (!g || !dst) return PT_ERR_ARG;
    if (!group_gathered(g)) {
        const int rc = pt_group_gather(g, nullptr);
        if (rc != PT_OK) return rc;
    }
    pt_context* root = g->ctx[0];
    const size_t npix = (size_t)g->width * g->height;
    PT_GHIP_CHECK(g, hipSetDevice(root->device));
    if (!g->ldr) PT_GHIP_CHECK(g, hipMalloc(&g->ldr, npix * sizeof(uchar4)));
    tonemap_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, root->stream>>>(g->ldr, g->full, npix, frames);
    PT_GHIP_CHECK(g, hipGetLastError());
    PT_GHIP_CHECK(g, hipMemcpyAsync(dst, g->ldr, npix * sizeof(uchar4), hipMemcpyDeviceToHost, root->stream));
    PT_GHIP_CHECK(g, hipStreamSynchronize(root->stream));
    return PT_OK;
}

PT_API const char* pt_group_last_error(const pt_group* g) { return g ? g->err.c_str() : "null group"; }

} // extern "C"
