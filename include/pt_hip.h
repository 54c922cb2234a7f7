/*
 * pt_hip.h -- C ABI of the MI355X (gfx950) path-tracing device layer, libpt_hip.so.
 *
 * This is the drop-in boundary below the reference's `Pathtracer` class: it replaces the CUDA
 * resource management and kernel launches of PathtracerCUDA/src/pathtracer/Pathtracer.cpp and the
 * three kernels of src/pathtracer/kernels/ (trace.cu, initRandState.cu, tonemap.cu).  Plain C:
 * POD structs, pointers and sizes only; no C++ or torch types.  The host C++ layer
 * (include/pt_host.h, libpt_host.so) owns scene loading, the SAH BVH build and the frame counter,
 * exactly as the reference's host code does, and calls down into these entry points.
 *
 * Every call returns PT_OK (0) or a PT_ERR_* code; pt_last_error() gives the message.  All calls
 * on one context must come from one host thread (reference: single thread, Pathtracer.cpp:40).
 */
#ifndef PT_HIP_H
#define PT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_API __attribute__((visibility("default")))

enum {
    PT_OK = 0,
    PT_ERR_HIP = 1,        /* a HIP runtime call failed (reference: checkCudaErrors -> exit) */
    PT_ERR_ARG = 2,        /* invalid argument */
    PT_ERR_STATE = 3,      /* call not valid in the current state */
    PT_ERR_DEPTH = 4,      /* BVH deeper than the 32-entry traversal stack (trace.cu:39) allows */
    PT_ERR_NO_DEVICE = 5   /* no GPU visible */
};

#define PT_MAX_TEXTURES 64 /* Pathtracer.cpp:15 MAX_TEXTURE_COUNT */

/* Camera (reference Camera.h:14-22, 92 B, passed by value to traceKernel, trace.h:20) */
typedef struct pt_camera {
    float tan_half_fovy;
    float aspect_ratio;
    float origin[3];
    float lower_left_corner[3];
    float horizontal[3];
    float vertical[3];
    float right[3];
    float up[3];
    float backward[3];
} pt_camera;

/* BVH node (reference BVH.h:6-11, 32 B): interior nodes have primitive count 0 in bits 16-31 and
 * the split axis in bits 8-15; left child = index + 1, right child = offset; leaves hold the first
 * primitive index in offset. */
typedef struct pt_bvh_node {
    float aabb_min[3];
    float aabb_max[3];
    uint32_t offset;
    uint32_t primitive_count_axis;
} pt_bvh_node;

/* Device hittable (reference Hittable.h:23-27 + Material.h:22-27, 96 B): world->object 3x4 rows,
 * material, shape type (0 SPHERE .. 6 CUBE, Hittable.h:9-12); material_type 0 LAMBERT, 1 GGX,
 * 2 LAMBERT_GGX (Material.h:9-12); texture_index is a 1-based handle, 0 = none. */
typedef struct pt_hittable {
    float inv_transform_rows[3][4];
    float base_color[3];
    float roughness;
    float emissive[3];
    float metalness;
    uint32_t texture_index;
    uint32_t material_type;
    uint32_t type;
    uint32_t pad;
} pt_hittable;

/* Traversal statistics of an instrumented render (for the algorithmic-byte count of DESIGN.md). */
typedef struct pt_render_stats {
    uint64_t node_tests;   /* AABB::hit calls                         */
    uint64_t prim_tests;   /* Hittable::hit calls                     */
    uint64_t hits;         /* segments that hit a primitive           */
    uint64_t sky_lookups;  /* misses that sampled the skybox texture  */
    uint64_t segments;     /* hitBVH calls                            */
    uint64_t samples;      /* camera paths                            */
    /* wave-level executions of the same events: SIMD efficiency of a phase = lane count / (64 x
     * wave count) */
    uint64_t wave_node_iters;
    uint64_t wave_prim_iters;
    uint64_t wave_hits;
    uint64_t wave_sky;
    uint64_t wave_segments;
    /* shader-clock cycles summed over waves (s_memtime stamps; while-while variants): interior
     * walk, leaf tests, shading, whole lane loop */
    uint64_t cycles_node_walk;
    uint64_t cycles_leaf_tests;
    uint64_t cycles_shading;
    uint64_t cycles_total;
    uint64_t cycles_lane_idle;  /* resumable variants: lane cycles spent done while the tile still ran */
    /* leaf tests by shape family (plane = disk/quad, cube, quadric: the three code paths of the
     * primitive test), resumable variants: leaf rounds (the wave's pending leaves after an interior
     * walk), family-path executions as run (per leaf position, one per family present), and as a
     * perfect cross-lane compaction would run them (per leaf round, ceil(pairs of the family / 64)) */
    uint64_t leaf_rounds;
    uint64_t family_execs;
    uint64_t family_execs_compacted;
    /* per leaf round: the lanes taking part and their (lane, primitive) pairs, summed; and the
     * family-path executions a compaction over only those lanes would need (the pairs in
     * family-major order, batches of as many pairs as lanes, one execution per batch and family) */
    uint64_t leaf_round_lanes;
    uint64_t leaf_pairs;
    uint64_t family_execs_compacted_in_round;
    /* child-box walks: leaf rounds that ended with t_max above its value at the leaf's start (the
     * sphere's far-root quirk, Hittable.inl:152-158) and rebuilt the reference's pending far
     * children (trace.cu:48-98; repair_pending in pt_kernels.hip) */
    uint64_t repairs;
} pt_render_stats;

typedef struct pt_context pt_context;

/* Number of visible GPUs. */
PT_API int pt_device_count(int *count);

/* Pathtracer ctor (Pathtracer.cpp:30-68): allocates the accumulation buffer and the per-pixel
 * XORWOW state and seeds it with curand_init(1984 + x + y * width, 0, 0) (initRandState.cu:16).
 * The context covers rows y = row_offset + k * row_stride (k = 0 .. local rows - 1) of a
 * width x height image, so an image can be tiled across GPUs (row_offset = rank, row_stride = N);
 * seeds and camera coordinates always use global pixel coordinates. */
PT_API int pt_create(int device, uint32_t width, uint32_t height, uint32_t row_offset, uint32_t row_stride,
                     pt_context **out);

/* Same, tiling the image in bands of band_rows rows (a power of two, 1..256): the context covers
 * the bands b = band_offset + k * band_stride, i.e. global row
 *     y(ly) = (band_offset + (ly / band_rows) * band_stride) * band_rows + ly % band_rows
 * for local row ly.  band_rows = 1 is pt_create's row interleave; band_rows = 8 (the multi-GPU
 * default) keeps each 8x8 tile of a context a spatially coherent 8x8 tile of the image. */
PT_API int pt_create_banded(int device, uint32_t width, uint32_t height, uint32_t band_rows, uint32_t band_offset,
                            uint32_t band_stride, pt_context **out);

/* Number of local rows of such a context (0 if it owns no band or the arguments are invalid). */
PT_API uint32_t pt_band_rows(uint32_t height, uint32_t band_rows, uint32_t band_offset, uint32_t band_stride);
/* Scatter one tile's rows (pt_band_rows(height, ...) x width float4, local row order, device memory
 * `part`) into the full image (height x width float4, device memory `full`) on `device`: the
 * unpermute step of pt_group_gather, for callers that gathered the tiles themselves (the
 * one-process-per-GPU path over torch.distributed / RCCL, pathtracercuda_amd/distributed.py).
 * Synchronises the device before and after. */
PT_API int pt_unpermute_bands(int device, void *full, const void *part, uint32_t width, uint32_t height,
                              uint32_t band_rows, uint32_t band_offset, uint32_t band_stride);
PT_API void pt_destroy(pt_context *ctx);

/* Pathtracer::setScene upload half (Pathtracer.cpp:137-159): nodes and primitives as produced by
 * the host BVH build (elements already reordered).  Replaces the previous scene.  Returns
 * PT_ERR_DEPTH if a traversal could overflow the reference's 32-entry stack. */
PT_API int pt_set_scene(pt_context *ctx, const pt_bvh_node *nodes, uint32_t node_count, const pt_hittable *prims,
                        uint32_t prim_count);

/* Pathtracer::loadTexture upload half (Pathtracer.cpp:258-288): RGBA float texels (LDR textures
 * already normalised to [0,1]), row 0 = first image row; handle is 1-based (1..64).  Sampled with
 * bilinear filtering, wrap in u, clamp in v, normalised coordinates. */
PT_API int pt_set_texture(pt_context *ctx, uint32_t handle, const float *rgba, uint32_t width, uint32_t height);

/* Pathtracer::setSkyboxTextureHandle (Pathtracer.cpp:294-297); 0 = no skybox (black). */
PT_API int pt_set_skybox(pt_context *ctx, uint32_t handle);

/* traceKernel launch (Pathtracer.cpp:162-199, trace.cu:158-199).  Equivalent to `chunks`
 * successive reference render(camera, spp, ignore) calls where the first call uses
 * ignore = ignore_history and the others ignore = false (the headless loop, main.cpp:275-279).
 * Synchronous.  gpu_ms (optional) receives the kernel time measured with hipEvents on the
 * context's stream (it includes the cost pre-pass below).  No launch (and no error) when no scene
 * is set or spp == 0, as in the reference (Pathtracer.cpp:174).
 * Tiles are dispatched most expensive first.  When no cost order is known yet for the scene and
 * camera and spp * chunks >= 16, a 2-spp pre-pass that writes nothing back measures the tile
 * costs first; results never depend on the order. */
PT_API int pt_render(pt_context *ctx, const pt_camera *camera, uint32_t spp, uint32_t chunks, int ignore_history,
                     float *gpu_ms);

/* Same as pt_render with the instrumented kernel variant: identical results plus counters. */
PT_API int pt_render_instrumented(pt_context *ctx, const pt_camera *camera, uint32_t spp, uint32_t chunks,
                           int ignore_history, float *gpu_ms, pt_render_stats *stats);

/* Raw accumulation sums (float4 per local pixel, rows x width, y-up), the data behind
 * getHDRImageData (Pathtracer.cpp:299-315) before the division by the frame count. */
PT_API int pt_read_accum(pt_context *ctx, float *dst);

/* Device-to-device copy of the raw accumulation buffer (rows * width * 16 bytes) into memory of
 * the same device, e.g. a send buffer for the multi-GPU framebuffer gather. */
PT_API int pt_copy_accum_device(pt_context *ctx, void *dst_device, size_t bytes);

/* tonemap kernel (tonemap.cu:4-27) over the local rows: accum / frames, Reinhard, gamma 2.2,
 * truncation to 8 bits, alpha 255 (RGBA8, rows x width). */
PT_API int pt_tonemap(pt_context *ctx, uint32_t frames, uint8_t *dst);
/* Same, into a device buffer of >= rows*width*4 bytes (RGBA8): the replacement of render()'s
 * OpenGL pixel-buffer tonemap (Pathtracer.cpp:207-221) for a progressive viewer. */
PT_API int pt_tonemap_device(pt_context *ctx, uint32_t frames, void *dst, size_t dst_bytes);

/* Per-pixel XORWOW state (d, v0..v4 as uint32, rows x width x 6) -- for tests/checkpoints. */
PT_API int pt_read_rng(pt_context *ctx, uint32_t *dst);
PT_API int pt_write_rng(pt_context *ctx, const uint32_t *src);

PT_API uint32_t pt_local_rows(const pt_context *ctx);

/* Shader-clock cycles each 8x8 tile took in the last launch (row-major over the context's tiles,
 * count = ceil(width / 8) * ceil(rows / 8)); the input of the cost order. */
PT_API int pt_read_tile_costs(pt_context *ctx, uint32_t *dst, uint32_t count);
/* Diagnostics: per tile (row-major, same count), the mean over its lanes of the shader-clock cycles
 * between a lane finishing its pixel and the tile's end, from the last pt_render_instrumented launch
 * (resumable variants).  Divided by the tile's cycles (pt_read_tile_costs) it is the tile's
 * idle-lane fraction. */
PT_API int pt_read_tile_idle(pt_context *ctx, uint32_t *dst, uint32_t count);
/* Diagnostics: schedule trace.  With enabled != 0 every instrumented launch (pt_render_instrumented;
 * the plain kernel carries no trace code) also records per tile (row-major) two words: the
 * shader-clock cycle (low 32 bits; the counter is per CU) at which its wave started it, and the
 * wave's hardware ids (XCC_ID << 16 | HW_ID bits 0-15: wave, SIMD, pipe, CU, SH, SE).
 * pt_read_tile_trace reads the last such launch's 2 x tiles words.  Results are unchanged. */
PT_API int pt_set_tile_trace(pt_context *ctx, int enabled);
PT_API int pt_read_tile_trace(pt_context *ctx, uint32_t *dst, uint32_t count);

/* Tuning knob for A/B measurements: 0 = automatic (default); otherwise one of the shipped
 * trace-kernel variants (traversal loop shape, deferred shading, BVH staged in LDS or read through
 * the caches, occupancy target; see pt_kernels.hip).  All variants produce bit-identical results.
 *   picked automatically (0):   60 and 40 (records in LDS, six / five waves per SIMD), 61 and 41
 *                               (records through the caches), 46 (deep BVHs, four waves), 47 / 48
 *                               (small grids);
 *   fallbacks the automatic choice also uses: 4 and 6 (node-at-a-time walks for scenes outside the
 *                               child-box encoding or whose leaves are not in DFS order);
 *   reference / counting:       1 (the reference's control flow), 20 (counts the reference's node and
 *                               primitive tests; the bench's algorithmic bytes);
 *   test / A-B only:            39 (no deferred shading), 91 (48 without the rising-t_max rebuild;
 *                               not the reference's results -- its cost A/B only).
 * Other numbers return PT_ERR_ARG. */
PT_API int pt_set_kernel_variant(pt_context *ctx, int variant);

/* Tile dispatch order: 0 = by the measured cost of each 8x8 tile, most expensive first (default:
 * every launch records the tile costs, and after a scene, texture or camera change the order is
 * rebuilt on the device from the latest launch), 1 = always row-major.  Results are identical;
 * only the launch tail changes. */
PT_API int pt_set_schedule(pt_context *ctx, int mode);

/* Tuning knob for measurements: persistent trace-kernel grids hold at most workgroups_per_cu
 * workgroups (of four waves, one per SIMD) per CU, i.e. that many waves per SIMD (0 = as many as
 * fit, the default).  Results are identical. */
PT_API int pt_set_occupancy(pt_context *ctx, uint32_t workgroups_per_cu);

/* Issue priority by position in the cost order (s_setprio): mode 0 = automatic (default: graded by
 * quarter of the order, the first band raised to every position a persistent plain launch deals at
 * its start), 1 = off, 2 = explicit -- positions < level3 run at wave priority 3, < level2 at 2,
 * < level1 at 1, the rest at 0 (level3 <= level2 <= level1).  Results are identical. */
PT_API int pt_set_issue_priority(pt_context *ctx, int mode, uint32_t level3, uint32_t level2, uint32_t level1);

/* Speculative sample groups.  A pixel's samples are one serial XORWOW stream
 * (trace.cu:183-193), so a launch with fewer 8x8 tiles than about four per wave slot of the chip
 * (multi-GPU strong scaling, small images) lasts as long as its slowest tile's whole chain.  With
 * groups, each pixel's chain is cut into G pieces started at guessed draw offsets and stitched where
 * the guessed parse meets the true one; results stay bit-identical.  mode: 0 = automatic (default),
 * 1 = never, G >= 2 = always G groups (tests).  pt_last_sample_groups: groups of the last launch
 * (0 = plain).  pt_read_group_stats fills 10 words: G, patch rounds run, and the pixels at a dead end
 * after fold rounds 0..7.  pt_read_group_log_counts: samples each (tile, item) logged per lane
 * ([tile][2G - 1][64], tiles in dispatch (cost) order; item 0 = group 0, items 2g - 1 and 2g =
 * group g at its guessed offset and one draw pair later).  pt_set_patch_rounds: patch rounds before
 * the remaining dead ends run as a plain resume launch (default 6; 0 exercises the resume path).
 * pt_set_group_lookback: a second phase (the item one pair later) also stops where its first
 * phase's parse holds the second phase's sample start `far` or `near` samples back -- the first
 * phase may run behind on the parse the two share (defaults 64 and 16; 0 = off: only the current
 * start).  Scheduling only: results are identical for every setting. */
/* Tuning knob: tiles per dispatch unit of launches with few samples per pixel (a row strip of K
 * tiles; a lane whose pixel is done takes the same position in the next tile of its strip).
 * 0 = automatic (K = 4 at <= 2 samples per pixel on large images), 1 = off, K = 2..16 = always K
 * (resumable variants).  Results are identical for every setting. */
PT_API int pt_set_strip_units(pt_context *ctx, int mode);
/* Test knob (negative control): enabled = 0 skips the child-box walks' rebuild of the pending far
 * children after a leaf raised t_max (the sphere's far-root quirk, Hittable.inl:152-158), so those
 * walks drop boxes the reference would test (trace.cu:48-98) and results are NOT the reference's on
 * rays that meet the quirk.  Default 1.  Exists so a test can show that a scene exercises the rebuild. */
PT_API int pt_set_rise_repair(pt_context *ctx, int enabled);
/* Run-ahead across render() calls: a launch of 3..64 samples per pixel (the reference's
 * render(camera, 8, ...) calls, main.cpp:272-279) lets the lanes whose pixels are done go on with the
 * pixel's next call (same XORWOW stream) until their tile ends, and keeps per pixel the colour sum,
 * count and state after the last finished sample; the next pt_render with the same camera, scene,
 * textures, sky and RNG state starts every pixel from there.  Any other next launch ignores the
 * stash: the stored RNG state and accumulation are always those of the calls made, so results are
 * the reference's either way.
 * 0 = automatic (the default; stops while the camera or scene changes at every launch),
 * 1 = off, 2 = make a stash at every launch (tests), 3 = make stashes but never use them
 * (diagnostic: the cost of the run-ahead work alone). */
PT_API int pt_set_run_ahead(pt_context *ctx, int mode);
/* Tuning knob of the cold start (the first launch after a scene, texture or camera change, which has
 * no tile costs yet).  prepass_spp = 0 (default): a launch of several render() calls runs its first
 * call alone in row-major order and the rest in the cost order of that call (a one-call launch runs a
 * discarded 2-spp cost pre-pass); prepass_spp > 0 (at most 64): always a discarded pre-pass of that
 * many spp.  priority: issue priority on that order (1, the default) or not (0).  Scheduling only:
 * results are identical for every setting. */
PT_API int pt_set_cold_start(pt_context *ctx, uint32_t prepass_spp, int priority);
PT_API int pt_set_sample_groups(pt_context *ctx, int mode);
PT_API int pt_set_patch_rounds(pt_context *ctx, uint32_t rounds);
PT_API int pt_set_group_lookback(pt_context *ctx, uint32_t far, uint32_t near);
PT_API int pt_last_sample_groups(const pt_context *ctx);
/* The trace-kernel variant the last launch ran (its main pass; diagnostics and tests). */
PT_API int pt_last_variant(const pt_context *ctx);
PT_API int pt_read_group_stats(const pt_context *ctx, uint32_t *dst);
PT_API int pt_read_group_log_counts(pt_context *ctx, uint32_t *dst, size_t count);
/* Diagnostics: one word plane of the per-pixel fold state (rows x width; word 16 = dead-end flag,
 * 7 = samples done, 8 = draw-pair offset), or with words 19 / 20 / 21 the statistics the next
 * launch's guesses use (float): draw pairs per sample, odd-length fraction, variance. */
PT_API int pt_read_group_fold(pt_context *ctx, uint32_t word, uint32_t *dst);
PT_API const char *pt_last_error(const pt_context *ctx);

/* ---- Multi-device group (one process, one context per GPU, RCCL over xGMI) -------------------
 * Replaces the reference's hard-coded single device (Pathtracer.cpp:40: cudaSetDevice(0)) behind
 * the same Pathtracer interface: device i renders the row bands b = i, i + N, ... of the image
 * (pt_create_banded with band_offset = i, band_stride = N), and pt_group_gather assembles the
 * accumulation buffer on devices[0] with one grouped ncclSend/ncclRecv (communicators from
 * ncclCommInitAll) plus an unpermute kernel.  Seeds use global pixel indices, so the assembled
 * image is bit-identical to a single-device render.  Devices must be distinct. */
typedef struct pt_group pt_group;

PT_API int pt_group_create(int ndev, const int *devices, uint32_t width, uint32_t height, uint32_t band_rows,
                           pt_group **out);
PT_API void pt_group_destroy(pt_group *g);
PT_API int pt_group_size(const pt_group *g);
/* The context of device index i (for per-device calls such as pt_set_kernel_variant). */
PT_API pt_context *pt_group_context(pt_group *g, int index);
PT_API int pt_group_set_scene(pt_group *g, const pt_bvh_node *nodes, uint32_t node_count, const pt_hittable *prims,
                              uint32_t prim_count);
PT_API int pt_group_set_texture(pt_group *g, uint32_t handle, const float *rgba, uint32_t width, uint32_t height);
PT_API int pt_group_set_skybox(pt_group *g, uint32_t handle);
/* pt_render on every device concurrently (one host thread each); gpu_ms = the slowest device. */
PT_API int pt_group_render(pt_group *g, const pt_camera *camera, uint32_t spp, uint32_t chunks, int ignore_history,
                           float *gpu_ms);
/* RCCL gather of every device's accumulation rows to devices[0] + unpermute into the full image;
 * host_ms (optional) = wall time of the gather. */
PT_API int pt_group_gather(pt_group *g, float *host_ms);
/* Full-image raw accumulation (height x width float4, y-up) / tonemap (RGBA8), gathering first if
 * the image changed since the last gather. */
PT_API int pt_group_read_accum(pt_group *g, float *dst);
PT_API int pt_group_tonemap(pt_group *g, uint32_t frames, uint8_t *dst);
PT_API const char *pt_group_last_error(const pt_group *g);

#ifdef __cplusplus
}
#endif

#endif /* PT_HIP_H */
