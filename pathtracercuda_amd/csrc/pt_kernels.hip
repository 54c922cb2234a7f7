// pt_kernels.hip -- gfx950 path-tracing megakernel, RNG seeding and tonemap kernels, and the C ABI
// of include/pt_hip.h.
//
// Reference behaviour (PathtracerCUDA/src/pathtracer/):
//   traceKernel  kernels/trace.cu:158-199 (+ getColor :101-156, hitBVH :28-98)
//   intersection Hittable.inl:88-358, AABB.inl:22-69
//   shading      Material.inl:20-144, MonteCarlo.h:5-114, brdf.h:4-62
//   seeding      kernels/initRandState.cu:4-17
//   tonemap      kernels/tonemap.cu:4-27
//
// MI355X design (DESIGN.md has the full rationale):
//   * one wave64 = one 8x8 pixel tile, one lane = one pixel: the per-pixel XORWOW stream is serial
//     (SURVEY.md fact 3), so pixels are the only parallel unit;
//   * the lane runs a flat state machine (segment = traverse + shade) and starts its pixel's next
//     sample as soon as a path ends, so a wave stays busy until its lanes have finished all
//     samples of all chunks of the launch, instead of idling at every path end;
//   * all `chunks` render() calls of the headless loop run in one launch; the per-chunk summation
//     (color = sum of spp paths, then color + accum) is reproduced exactly (the colour sum in LDS,
//     the accumulation value in registers);
//   * RNG state (24 B/pixel) and accum (16 B/pixel) are read once and written once per launch, SoA;
//   * the BVH node test hoists the per-ray reciprocals (bit-identical to recomputing them) and the
//     hit record is reconstructed once for the closest hit instead of for every candidate hit.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rccl/rccl.h>
#include <stdint.h>
#include <cmath>
#include <string.h>
#include <stdio.h>
#include <string>
#include <vector>
#include <algorithm>
#include <atomic>
#include <thread>
#include <chrono>

#include "pt_math.h"
#include "../../include/pt_hip.h"

using namespace pt;

namespace {

// The kernel's dynamic LDS (layout: trace_kernel).  Declared here so device functions address it
// directly (ds_* instructions; a generic pointer kept in a struct would compile to flat_*).
extern __shared__ float4 lds4[];

__device__ __forceinline__ float* lds_f() { return reinterpret_cast<float*>(lds4); }

struct DevTex {
    const float4* texels;
    uint32_t width, height;
    float fwidth, fheight;      // (float)width, (float)height, converted once on the host: a uniform
                                // conversion in the kernel would be a VALU result held in a VGPR
};

struct DevCamera {
    f3 origin, llc, horizontal, vertical;
};

struct TraceParams {
    float4* accum;              // rows x width, local
    uint32_t* rng;              // 6 planes of rows x width (d, v0..v4)
    const float4* nodes;        // 2 per node: (min.xyz, max.x), (max.yz, offset bits, pca bits)
    const float4* prims;        // 4 per prim: row0, row1, row2, (type bits, 0, 0, 0)
    const float4* mats;         // 3 per prim: (base.xyz, roughness), (emissive.xyz, metal), (tex, type)
    const DevTex* textures;     // 64 entries
    unsigned long long* stats;  // 6 counters (instrumented variant only)
    uint32_t skybox;
    DevTex skyTex;              // the skybox's descriptor itself (kernel argument: scalar loads, no
                                // dependent fetch from the texture table per miss)
    uint32_t width, height, rowOffset, rowStride, rows;
    float fwidth, fheight;      // (float)width, (float)height (host-converted, see DevTex)
    uint32_t bandShift;         // rows are tiled in bands of 1 << bandShift rows (global_row)
    uint32_t spp, chunks, ignoreFirst;
    uint32_t tilesX, tilesY;
    uint32_t nodeCount, primCount, stackDepth, slabFast;
    const float4* cnodes;       // child-box records (4 per interior node), see traverse_cb
    uint32_t cnodeCount, rootWord;
    float rootBox[6];           // (min.x, max.x, min.y, max.y, min.z, max.z) of the root
    const uint32_t* order;      // tile dispatch order as packed tile coordinates (tileY << 16 | tileX),
                                // see "Tile scheduling"; null only with scatterWaves
    uint32_t scatterWaves;      // != 0: scattered pixel mapping over this many waves (pixel_of)
    uint32_t* tileCursor;       // persistent variants: {next dispatch slot, waves finished}, rewound by the last wave
    uint32_t numSlots;          // dispatch slots = 8x8 tiles
    uint32_t* tileCost;         // per-tile shader-clock cycles of this launch (null: not recorded)
    uint32_t* tileIdle;         // instrumented launches: per tile, the lanes' mean cycles between finishing
                                // their pixel and the tile's end (zeroed before the launch)
    uint32_t discard;           // != 0: cost pre-pass -- pixel state (RNG, accum) is read, never written
    float* pairsOut;            // cost pre-pass: per-pixel draw pairs per sample (speculative groups' guess)
    // Speculative sample groups (0 = off).  A tile has J = 2G - 1 work items: item 0 =
    // group 0; items 2g - 1 and 2g = group g >= 1 started at its guessed draw offset and, for pixels
    // whose sample starts sit on the even lattice with rare odd shifts, one pair later (else that
    // lane is idle).  Slot s runs tile order[s / J], item s % J; item index = (s / J) * J + j, i.e. the
    // per-item buffers are indexed by the tile's position in the order (ssgTiles = the grouped
    // positions 0 .. ssgTiles - 1).  Patch rounds (ssgPatch):
    // one carrier per grouped tile, lanes = the pixels the fold left at a dead end.
    uint32_t ssgG;              // groups per pixel
    uint32_t ssgTiles;          // grouped tiles: order positions 0 .. ssgTiles - 1
    uint32_t ssgCap;            // sample-log capacity per item
    uint32_t ssgPatch;          // != 0: patch round
    float* ssgLog;              // [item][cap][3][64] path colours
    uint16_t* ssgEnd;           // [item][cap][64] end of each sample, in draw pairs from the item's start
    const uint32_t* ssgStart;   // [item][8][64] start offset (draw pairs; ~0 = idle lane), d, v0..v4, stop offset
    unsigned long long* ssgBits;// [item][ssgWin][64] the item's sample starts in its window
    uint32_t ssgWin;            // window words per lane (64 draw pairs each) after an item's start
    uint32_t* ssgCount;         // [item][64] samples logged
    uint32_t ssgLook[2];        // a second phase also stops where its first phase's parse holds its
                                // sample start this many samples back (lag tolerance; 0 = off)
    uint32_t* fold;             // [kFoldWords][rows*width] fold state (ssg_fold_kernel); AUX resume input
    DevCamera cam;
    uint32_t occCap;            // host only: persistent grids hold at most this many workgroups per CU (0 = all)
    uint32_t prio[3];           // issue priority by order position: < prio[0] -> 3, < prio[1] -> 2, < prio[2] -> 1
    uint32_t strip;             // MODE 3: tiles per dispatch unit (a row strip of `strip` tiles; see trace_kernel)
    // MODE 4 (run-ahead across render() calls, see trace_kernel): per-pixel stash of the NEXT call's
    // first samples, kAheadWords planes of rows x width u32 (ahead_store).
    uint32_t* ahead;
    uint32_t aheadUse;          // != 0: the stash was made under this launch's camera and scene: consume it
    uint32_t aheadMake;         // != 0: lanes whose pixel is done go on with the next call's samples
};

// Speculative sample groups: window of a group's start offset in which an earlier group's parse can
// join it (draw pairs; 16 x 64-bit words per lane), and the fold state kept per pixel between rounds.
constexpr uint32_t kWinWords = 16;        // G >= 3: groups <= n samples apart, the window covers a group's start
// With G = 2 the window covers the second group's whole range (up to 6 draw pairs per sample): in
// long multi-bounce pixels two parses can take hundreds of samples to meet, and a first group that
// never meets the second runs the whole chain (measured: every lane of a tile).
static inline uint32_t ssg_window_words(uint32_t G, uint32_t n)
{
    return G == 2 ? (n * 6u + 256u + 63u) / 64u : kWinWords;
}
constexpr uint32_t kFoldBatch = 16;       // samples the fold loads at once
constexpr uint32_t kStatWords = 23;       // counters of an instrumented launch (pt_render_stats)
constexpr uint32_t kStartWords = 8;       // start record: offset, d, v0..v4, stop offset (last group)
constexpr uint32_t kAheadWords = 10;      // run-ahead stash: colour sum x3, samples, XORWOW state x6
enum : uint32_t { F_ACC = 0, F_COL = 3, F_SC = 6, F_DONE = 7, F_OFF = 8, F_H = 9, F_ST = 10, F_FLAG = 16, F_ODD = 17,
                  F_SQ = 18, kFoldWords = 19 };

// Row tiling of an image across contexts (multi-GPU): the image is cut into bands of
// B = 1 << shift rows, and a context owns bands b = offset + k * stride.  Local row ly lies in the
// context's band ly / B at row ly % B.  B = 1 is plain row interleaving (y = offset + ly * stride);
// B = 8 keeps every 8x8 tile of a context a spatially coherent 8x8 tile of the image.  Seeds and
// camera coordinates always use the global row, so every tiling reproduces the 1-GPU image.
__host__ __device__ inline uint32_t global_row(uint32_t ly, uint32_t offset, uint32_t stride, uint32_t shift)
{
    return ((offset + (ly >> shift) * stride) << shift) + (ly & ((1u << shift) - 1u));
}

// ---------------------------------------------------------------------------------------------
// texture sampling: CUDA 2-D linear fetch, normalised coordinates, wrap (u) / clamp (v),
// weights quantised to 1/256 (sampler of Pathtracer.cpp:276-283)
// ---------------------------------------------------------------------------------------------
PT_DEV f3 tex2d(const DevTex& t, float u, float v)
{
    const float W = t.fwidth, H = t.fheight;
    const float uw = u - floorf(u);
    const float x = uw * W - 0.5f;
    const float y = v * H - 0.5f;
    const float fx = floorf(x), fy = floorf(y);
    float a = x - fx, b = y - fy;
    a = floorf(a * 256.0f + 0.5f) * (1.0f / 256.0f);
    b = floorf(b * 256.0f + 0.5f) * (1.0f / 256.0f);
    const int32_t w = (int32_t)t.width, h = (int32_t)t.height;
    int32_t i0 = (fx > -1.0e9f && fx < 1.0e9f) ? (int32_t)fx : 0;
    int32_t j0 = (fy > -1.0e9f && fy < 1.0e9f) ? (int32_t)fy : (fy > 0.0f ? h : -1);
    int32_t i1 = i0 + 1, j1 = j0 + 1;
    // wrap: u - floor(u) lies in [0, 1] (or is NaN, giving i0 = 0), so fx lies in [-1, w - 1] and
    // i0 in [-1, w - 1], i1 in [0, w]: one conditional add/subtract equals ((i % w) + w) % w here
    i0 = i0 < 0 ? i0 + w : i0;
    i1 = i1 >= w ? i1 - w : i1;
    j0 = j0 < 0 ? 0 : (j0 > h - 1 ? h - 1 : j0);
    j1 = j1 < 0 ? 0 : (j1 > h - 1 ? h - 1 : j1);
    const float4 T00 = t.texels[(size_t)j0 * t.width + (size_t)i0];
    const float4 T10 = t.texels[(size_t)j0 * t.width + (size_t)i1];
    const float4 T01 = t.texels[(size_t)j1 * t.width + (size_t)i0];
    const float4 T11 = t.texels[(size_t)j1 * t.width + (size_t)i1];
    const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    return mk(w00 * T00.x + w10 * T10.x + w01 * T01.x + w11 * T11.x,
              w00 * T00.y + w10 * T10.y + w01 * T01.y + w11 * T11.y,
              w00 * T00.z + w10 * T10.z + w01 * T01.z + w11 * T11.z);
}

// ---------------------------------------------------------------------------------------------
// intersection
// ---------------------------------------------------------------------------------------------
enum : uint32_t { SPHERE = 0, CYLINDER = 1, DISK = 2, CONE = 3, PARABOLOID = 4, QUAD = 5, CUBE = 6 };

struct LocalRay { f3 o, d; };

typedef float f2v __attribute__((ext_vector_type(2)));   // lowers to v_pk_{add,mul}_f32 on gfx950

PT_DEV f2v f2(float a, float b) { return (f2v){a, b}; }

// Hittable.inl:91-98: world -> object space with the 3x4 inverse rows (origin gets +w).  Device
// layout of the rows (pt_set_scene): P0 = (r0.x, r1.x, r0.y, r1.y), P1 = (r0.z, r1.z, r0.w, r1.w),
// P2 = row 2, so the x and y components are evaluated pairwise with packed FP32 ops -- the same
// products and sums in the same order as the reference's dot products, two lanes of a
// v_pk_mul/v_pk_add at a time (exactly rounded per element; no FMA contraction).
PT_DEV LocalRay to_local(const float4& P0, const float4& P1, const float4& r2, f3 o, f3 d)
{
    LocalRay l;
    f2v oxy = f2(P0.x, P0.y) * f2(o.x, o.x);
    oxy = oxy + f2(P0.z, P0.w) * f2(o.y, o.y);
    oxy = oxy + f2(P1.x, P1.y) * f2(o.z, o.z);
    oxy = oxy + f2(P1.z, P1.w);
    f2v dxy = f2(P0.x, P0.y) * f2(d.x, d.x);
    dxy = dxy + f2(P0.z, P0.w) * f2(d.y, d.y);
    dxy = dxy + f2(P1.x, P1.y) * f2(d.z, d.z);
    l.o.x = oxy.x;
    l.o.y = oxy.y;
    l.o.z = (o.x * r2.x + o.y * r2.y + o.z * r2.z) + r2.w;
    l.d.x = dxy.x;
    l.d.y = dxy.y;
    l.d.z = d.x * r2.x + d.y * r2.y + d.z * r2.z;
    return l;
}

// Quadric coefficients of the four quadric shapes (Hittable.inl:152,176,242,273): all have
// A = C = 1 and D = E = F = G = I = 0; B, H, J vary.  Evaluated with the nonzero terms in the
// template's order; dropping the exact +-0 terms of D..G and I cannot change a, b or c except for
// the sign of a zero, which no later operation observes (DESIGN.md "Quadric terms").
PT_DEV bool quadric_roots(uint32_t type, const LocalRay& r, float& t0, float& t1)
{
    const float B = (type == SPHERE) ? 1.0f : (type == CONE ? -1.0f : 0.0f);
    const float Hc = (type == PARABOLOID) ? -1.0f : 0.0f;
    const float J = (type == SPHERE || type == CYLINDER) ? -1.0f : 0.0f;
    const f3 o = r.o, d = r.d;
    const float a = (d.x * d.x + (B * d.y) * d.y) + d.z * d.z;
    const float b = (((2.0f * o.x) * d.x + ((2.0f * B) * o.y) * d.y) + (2.0f * o.z) * d.z) + Hc * d.y;
    const float c = (((o.x * o.x + (B * o.y) * o.y) + o.z * o.z) + Hc * o.y) + J;
    // quadratic (Hittable.inl:7-39)
    const float disc = b * b - 4.0f * a * c;
    if (disc < 0.0f) return false;
    const float rt = sqrt_rn(disc);
    const float q = b < 0.0f ? -0.5f * (b - rt) : -0.5f * (b + rt);
    float x0 = q / a;
    float x1 = c / q;
    t0 = x0 > x1 ? x1 : x0;
    t1 = x0 > x1 ? x0 : x1;
    return true;
}

// A primitive's record as the test reads it: the inverse-transform rows and the shape type.
struct PrimRec {
    float4 r0, r1, r2;
    uint32_t type;
};

PT_DEV PrimRec load_prim(const float4* __restrict__ prims, uint32_t p)
{
    PrimRec q;
    q.r0 = prims[4 * p + 0];
    q.r1 = prims[4 * p + 1];
    q.r2 = prims[4 * p + 2];
    q.type = __float_as_uint(prims[4 * p + 3].x);
    return q;
}

// Hittable::hit without the hit-record side effects: returns the hit distance of the primitive.
PT_DEV bool prim_hit_rec(const PrimRec& q, f3 o, f3 d, float tMin, float tMax, float& tOut)
{
    const uint32_t type = q.type;
    const LocalRay r = to_local(q.r0, q.r1, q.r2, o, d);
    if (type == DISK || type == QUAD) {                    // Hittable.inl:205-235, 299-329
        if (r.d.y == 0.0f) return false;
        const float t = -r.o.y / r.d.y;
        if (t <= tMin || t > tMax) return false;
        const float hx = r.o.x + r.d.x * t;
        const float hz = r.o.z + r.d.z * t;
        if (type == QUAD) {
            if (fabsf(hx) > 1.0f || fabsf(hz) > 1.0f) return false;
        } else {
            if ((hx * hx + hz * hz) >= 1.0f) return false;
        }
        tOut = t;
        return true;
    }
    if (type == CUBE) {                                     // Hittable.inl:331-358, AABB.inl:46-69
        float lo = tMin, hi = tMax;
        const float ox[3] = {r.o.x, r.o.y, r.o.z};
        const float dx[3] = {r.d.x, r.d.y, r.d.z};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float invD = rcp_rn(dx[a]);
            float t0 = (-1.0f - ox[a]) * invD;
            float t1 = (1.0f - ox[a]) * invD;
            if (invD < 0.0f) { const float tmp = t0; t0 = t1; t1 = tmp; }
            lo = t0 > lo ? t0 : lo;
            hi = t1 < hi ? t1 : hi;
        }
        if (hi <= lo) return false;
        tOut = lo;
        return true;
    }
    float t0 = 0.0f, t1 = 0.0f;                             // quadrics
    if (!quadric_roots(type, r, t0, t1) || t0 > tMax || t1 <= tMin) return false;
    if (type == SPHERE) {                                   // Hittable.inl:158 (far-root quirk kept)
        tOut = t0 > tMin ? t0 : t1;
        return true;
    }
    const float h0 = r.d.y * t0 + r.o.y;                    // Hittable.inl:182-185
    const float h1 = r.d.y * t1 + r.o.y;
    const bool v0 = t0 > tMin && t0 <= tMax && h0 >= -1.0f && h0 <= 1.0f;
    const bool v1 = t1 > tMin && t1 <= tMax && h1 >= -1.0f && h1 <= 1.0f;
    if (!v0 && !v1) return false;
    tOut = v0 ? t0 : t1;
    return true;
}

PT_DEV bool prim_hit(const float4* __restrict__ prims, uint32_t p, f3 o, f3 d, float tMin, float tMax, float& tOut)
{
    return prim_hit_rec(load_prim(prims, p), o, d, tMin, tMax, tOut);
}

struct Counters {
    uint32_t node_tests, prim_tests, hits, sky, segments, samples;
    // wave-level executions of the same points (SIMD efficiency = lane count / (64 * wave count))
    uint32_t w_node, w_prim, w_hits, w_sky, w_segments;
    // wave-level shader-clock cycles per phase (instrumented variant only)
    uint64_t cyc_node, cyc_leaf, cyc_shade, cyc_total;
    uint64_t cyc_lane_idle;     // per lane: cycles between finishing its pixel and the tile's end
    uint32_t w_leaf_rounds, w_fam_exec, w_fam_ideal;   // leaf tests by shape family (pt_render_stats)
    uint32_t w_leaf_lanes, w_leaf_pairs, w_fam_inplace;  // lanes and (lane, primitive) pairs per leaf round
    uint32_t repairs;           // leaf rounds that raised t_max and rebuilt the pending set (repair_pending)
};

// Shape family of a primitive test's code path in prim_hit: 0 plane (disk, quad), 1 cube, 2 quadric.
PT_DEV uint32_t shape_family(uint32_t type) { return (type == DISK || type == QUAD) ? 0u : (type == CUBE ? 1u : 2u); }

// Instrumented variants: one leaf round, counted once per wave -- the family-path executions a
// perfect cross-lane compaction over all 64 lanes would need (ceil(pairs of the family / 64) per
// family), and the ones a compaction over the lanes that are in the round would need: its pairs in
// family-major order cut into batches of as many pairs as there are such lanes, one execution per
// (batch, family) segment.  Also the round's lanes and pairs.
PT_DEV void leaf_round_stats(const float4* __restrict__ prims, uint32_t off, uint32_t count, Counters& cnt)
{
    uint32_t nf[3] = {0u, 0u, 0u};
    for (uint32_t k = 0; k < count; ++k) nf[shape_family(__float_as_uint(prims[4 * (off + k) + 3].x))]++;
    const unsigned long long m = __ballot(1);
    const uint32_t lanes = (uint32_t)__popcll(m);
    uint32_t ideal = 0, inplace = 0, start = 0;
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        uint32_t total = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b) total += (uint32_t)__popcll(__ballot((nf[f] >> b) & 1u)) << b;
        ideal += (total + 63u) / 64u;
        if (total) inplace += (start + total - 1u) / lanes - start / lanes + 1u;
        start += total;
    }
    if ((threadIdx.x & 63u) == (uint32_t)(__ffsll((long long)m) - 1)) {
        cnt.w_leaf_rounds++;
        cnt.w_fam_ideal += ideal;
        cnt.w_leaf_lanes += lanes;
        cnt.w_leaf_pairs += start;
        cnt.w_fam_inplace += inplace;
    }
}

// One leaf position: the family paths the wave runs (one per family among its active lanes).
PT_DEV void leaf_position_stats(const float4* __restrict__ prims, uint32_t p, Counters& cnt)
{
    const uint32_t f = shape_family(__float_as_uint(prims[4 * p + 3].x));
    const uint32_t execs = (__ballot(f == 0u) != 0ull) + (__ballot(f == 1u) != 0ull) + (__ballot(f == 2u) != 0ull);
    const unsigned long long m = __ballot(1);
    if ((threadIdx.x & 63u) == (uint32_t)(__ffsll((long long)m) - 1)) cnt.w_fam_exec += execs;
}

// Adds the cycles since `t0` to `acc` once per wave and restarts the stamp.
PT_DEV void wave_time(uint64_t& acc, uint64_t& t0)
{
    const uint64_t t = __builtin_amdgcn_s_memtime();
    const unsigned long long m = __ballot(1);
    if ((threadIdx.x & 63u) == (uint32_t)(__ffsll((long long)m) - 1)) acc += t - t0;
    t0 = t;
}

// Counts one per wave that executes this point (instrumented variant only).
PT_DEV void wave_tick(uint32_t& c)
{
    const unsigned long long m = __ballot(1);
    if ((threadIdx.x & 63u) == (uint32_t)(__ffsll((long long)m) - 1)) c++;
}

// hitBVH (trace.cu:28-98): identical visit order, node culling with the current t_max, and
// in-order leaf tests (later equal-t primitives win).  Returns the closest primitive or ~0u.
// `stack` points at this lane's column of the wave's LDS stack ([depth][64 lanes] u32: entry k of
// lane l is stack[64 * k], so one wave-wide push/pop touches 64 distinct banks-pairs, conflict-free).
// Slab test of node `cur` against the ray's running interval (AABB.inl:22-44).  The reference
// recomputes 1/d per node and axis, a function of the ray only, so it is hoisted (bit-identical);
// the early returns are dropped because both bounds are monotone and never NaN.  Device node
// layout (pt_set_scene): A = (min.x, max.x, min.y, max.y), B = (min.z, max.z, offset, pca).
struct NodeHit {
    bool hit;
    uint32_t offset, pca;
};

// Exact form for any ray: swap on negative 1/d, NaN products ignored by the selects.
PT_DEV NodeHit node_test(const float4* __restrict__ nodes, uint32_t cur, f3 o, float ix, float iy, float iz, float tMin,
                         float tMax)
{
    const float4 A = nodes[2 * cur];
    const float4 Bq = nodes[2 * cur + 1];
    float lo = tMin, hi = tMax;
    {
        float t0 = (A.x - o.x) * ix, t1 = (A.y - o.x) * ix;
        if (ix < 0.0f) { const float tmp = t0; t0 = t1; t1 = tmp; }
        lo = t0 > lo ? t0 : lo;
        hi = t1 < hi ? t1 : hi;
    }
    {
        float t0 = (A.z - o.y) * iy, t1 = (A.w - o.y) * iy;
        if (iy < 0.0f) { const float tmp = t0; t0 = t1; t1 = tmp; }
        lo = t0 > lo ? t0 : lo;
        hi = t1 < hi ? t1 : hi;
    }
    {
        float t0 = (Bq.x - o.z) * iz, t1 = (Bq.y - o.z) * iz;
        if (iz < 0.0f) { const float tmp = t0; t0 = t1; t1 = tmp; }
        lo = t0 > lo ? t0 : lo;
        hi = t1 < hi ? t1 : hi;
    }
    return NodeHit{hi > lo, __float_as_uint(Bq.z), __float_as_uint(Bq.w)};
}

// Fast form, exact when 1/d is finite on all axes and the box is not inverted (checked per ray
// and per scene): then no product is NaN, the swap on a negative 1/d is min/max of the two slab
// distances, and the running max/min over the axes is order-independent, so v_max3/v_min3 and
// packed subtract/multiply give the reference's values.
PT_DEV NodeHit node_test_fast(const float4* __restrict__ nodes, uint32_t cur, f2v ox2, f2v oy2, f2v oz2, f2v ix2,
                              f2v iy2, f2v iz2, float tMin, float tMax)
{
    const float4 A = nodes[2 * cur];
    const float4 Bq = nodes[2 * cur + 1];
    const f2v tx = (f2(A.x, A.y) - ox2) * ix2;
    const f2v ty = (f2(A.z, A.w) - oy2) * iy2;
    const f2v tz = (f2(Bq.x, Bq.y) - oz2) * iz2;
    const float lo = __builtin_fmaxf(__builtin_fmaxf(tMin, __builtin_fminf(tx.x, tx.y)),
                                     __builtin_fmaxf(__builtin_fminf(ty.x, ty.y), __builtin_fminf(tz.x, tz.y)));
    const float hi = __builtin_fminf(__builtin_fminf(tMax, __builtin_fmaxf(tx.x, tx.y)),
                                     __builtin_fminf(__builtin_fmaxf(ty.x, ty.y), __builtin_fmaxf(tz.x, tz.y)));
    return NodeHit{hi > lo, __float_as_uint(Bq.z), __float_as_uint(Bq.w)};
}

// hitBVH (trace.cu:28-98): identical per-lane visit order, node culling with the current t_max,
// and in-order leaf tests (later equal-t primitives win).  Returns the closest primitive or ~0u.
// `stack` points at this lane's column of the wave's LDS stack ([depth][64 lanes] u32: entry k of
// lane l is stack[64 * k], so a wave-wide push/pop is bank-conflict free).
//
// WW = false: one loop, a visited leaf is tested immediately (the reference's control flow).
// WW = true ("while-while"): each lane walks interior nodes until it reaches a leaf to test (or
// finishes); then the wave tests the pending leaves together.  The per-lane sequence of node and
// primitive tests is unchanged -- only the SIMD schedule differs -- so results are bit-identical,
// but the expensive primitive tests run with most lanes active instead of once per node step.
template <bool STATS, int WW>
PT_DEV uint32_t traverse(const float4* __restrict__ nodes, const float4* __restrict__ prims, uint32_t* stack, f3 o,
                         f3 d, bool slabFast, float& tHit, Counters& cnt)
{
    const float tMin = 0.001f;
    float tMax = kFltMax;
    const float ix = rcp_rn(d.x), iy = rcp_rn(d.y), iz = rcp_rn(d.z);
    // trace.cu:31-36: dirIsNeg from 1/(d != 0 ? d : 1e-7) < 0, i.e. d < 0
    const uint32_t negMask = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
    const bool fast = slabFast && __builtin_isfinite(ix) && __builtin_isfinite(iy) && __builtin_isfinite(iz);
    const f2v ox2 = f2(o.x, o.x), oy2 = f2(o.y, o.y), oz2 = f2(o.z, o.z);
    const f2v ix2 = f2(ix, ix), iy2 = f2(iy, iy), iz2 = f2(iz, iz);
    auto test = [&](uint32_t node) {
        return fast ? node_test_fast(nodes, node, ox2, oy2, oz2, ix2, iy2, iz2, tMin, tMax)
                    : node_test(nodes, node, o, ix, iy, iz, tMin, tMax);
    };
    uint32_t sp = 0, cur = 0, elem = 0xffffffffu;
    if (WW == 0) {
        for (;;) {
            if (STATS) { cnt.node_tests++; wave_tick(cnt.w_node); }
            const NodeHit nh = test(cur);
            if (nh.hit) {
                const uint32_t count = nh.pca >> 16;
                if (count > 0) {
                    for (uint32_t i = 0; i < count; ++i) {
                        if (STATS) { cnt.prim_tests++; wave_tick(cnt.w_prim); }
                        float t;
                        if (prim_hit(prims, nh.offset + i, o, d, tMin, tMax, t)) {
                            tMax = t;
                            elem = nh.offset + i;
                        }
                    }
                    if (sp == 0) break;
                    cur = stack[64u * (--sp)];
                } else {
                    const bool isNeg = (negMask >> ((nh.pca >> 8) & 0xffu)) & 1u;
                    stack[64u * (sp++)] = isNeg ? (cur + 1) : nh.offset;
                    cur = isNeg ? nh.offset : (cur + 1);
                }
            } else {
                if (sp == 0) break;
                cur = stack[64u * (--sp)];
            }
        }
    } else if (WW == 1) {
        uint32_t leafOff = 0, leafCnt = 0;
        bool done = false;
        uint64_t tPhase = STATS ? __builtin_amdgcn_s_memtime() : 0;
        while (!done) {
            while (leafCnt == 0 && !done) {                     // interior walk
                if (STATS) { cnt.node_tests++; wave_tick(cnt.w_node); }
                const NodeHit nh = test(cur);
                const uint32_t count = nh.pca >> 16;
                const bool isNeg = (negMask >> ((nh.pca >> 8) & 0xffu)) & 1u;
                const uint32_t nearC = isNeg ? nh.offset : cur + 1;
                const uint32_t farC = isNeg ? cur + 1 : nh.offset;
                if (nh.hit) {
                    if (count > 0) {
                        leafOff = nh.offset;
                        leafCnt = count;
                    } else {
                        stack[64u * sp] = farC;
                        ++sp;
                        cur = nearC;
                    }
                } else {
                    if (sp == 0) done = true;
                    else cur = stack[64u * (--sp)];
                }
            }
            if (STATS) wave_time(cnt.cyc_node, tPhase);
            while (leafCnt > 0) {                                // pending leaf, in order
                if (STATS) { cnt.prim_tests++; wave_tick(cnt.w_prim); }
                float t;
                if (prim_hit(prims, leafOff, o, d, tMin, tMax, t)) {
                    tMax = t;
                    elem = leafOff;
                }
                ++leafOff;
                --leafCnt;
            }
            if (STATS) wave_time(cnt.cyc_leaf, tPhase);
            if (!done) {
                if (sp == 0) done = true;
                else cur = stack[64u * (--sp)];
            }
        }
    }
    tHit = tMax;
    return elem;
}

// ---------------------------------------------------------------------------------------------
// Child-box traversal (WW == 3).  Device layout "cnodes": one 64-byte record per INTERIOR node of
// the reference BVH holding both children's boxes and references:
//   Q0 = (L.min.x, L.max.x, L.min.y, L.max.y)   Q1 = (L.min.z, L.max.z, R.min.z, R.max.z)
//   Q2 = (R.min.x, R.max.x, R.min.y, R.max.y)   Q3 = (L word, R word, 1 << split axis, 0)
// L = first child (node + 1), R = second child (node.offset); a child word is (count << 24 | prim
// offset) for a leaf and the child's record index for an interior node.
//
// Why it is exact: the slab test of AABB.inl:22-44 (node_test) starts its running upper bound at
// the ray's t_max and every update is a min that skips NaN, so for any ray
//     hit(t_max) = (X > lo) && (t_max > lo)
// with lo and X (the same test started from +inf) independent of t_max.  hitBVH tests a node's
// near child right after the node (t_max unchanged) and its far child when it is popped, after
// the near subtree may have lowered t_max.  Here both children are tested when their parent is
// visited; the far child is pushed with its lo and, when popped, re-tested as t_max > lo with the
// then-current t_max -- the reference's verdict.  Visit order, node tests and primitive tests per
// lane are unchanged; a visit costs one dependent fetch instead of two, and leaves cost none.
// ---------------------------------------------------------------------------------------------
struct SlabRay {
    f2v ox2, oy2, oz2, ix2, iy2, iz2;
    f3 o;
    float ix, iy, iz;
    bool fast;
};

// lo and X of one box (see above); the fast form under the same conditions as node_test_fast.
template <bool ALLFAST = false>
PT_DEV float slab_lo_x(const SlabRay& R, f2v bx, f2v by, f2v bz, float tMin, float& X)
{
    if (ALLFAST || R.fast) {
        const f2v tx = (bx - R.ox2) * R.ix2;
        const f2v ty = (by - R.oy2) * R.iy2;
        const f2v tz = (bz - R.oz2) * R.iz2;
        X = __builtin_fminf(__builtin_fmaxf(tx.x, tx.y), __builtin_fminf(__builtin_fmaxf(ty.x, ty.y), __builtin_fmaxf(tz.x, tz.y)));
        return __builtin_fmaxf(__builtin_fmaxf(tMin, __builtin_fminf(tx.x, tx.y)),
                               __builtin_fmaxf(__builtin_fminf(ty.x, ty.y), __builtin_fminf(tz.x, tz.y)));
    }
    float lo = tMin, hi = __builtin_inff();
    const float inv[3] = {R.ix, R.iy, R.iz};
    const float org[3] = {R.o.x, R.o.y, R.o.z};
    const f2v b[3] = {bx, by, bz};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float t0 = (b[k].x - org[k]) * inv[k], t1 = (b[k].y - org[k]) * inv[k];
        if (inv[k] < 0.0f) { const float tmp = t0; t0 = t1; t1 = tmp; }
        lo = t0 > lo ? t0 : lo;
        hi = t1 < hi ? t1 : hi;
    }
    X = hi;
    return lo;
}

// Both children of interior record `cur`, in the reference's visit order (trace.cu:66-77: near =
// second child when the ray direction is negative along the split axis).  Only the choice of
// the next node and of the pushed (far) child depends on the order: "both hit" and "any hit" are
// symmetric, so the hit flags stay compare results (wave masks, combined on the SALU) and three
// selects pick the next node, the far node and its entry distance.
// t_max can RISE during a traversal: the sphere's far-root quirk (Hittable.inl:158, prim_hit_rec)
// accepts t1 > t_max when t0 <= t_min, and the reference then tests the boxes it pops with that
// larger t_max (trace.cu:48-98).  The child-box walks keep a far child only if it is hit at the
// current t_max (`push`) -- exact while t_max only falls -- and rebuild the pending set when a leaf
// raises it (repair_pending).  A BVH whose leaves do not hold their primitives in DFS order (a
// caller's, pt_set_scene) cannot be descended by the rebuild and runs the node-at-a-time walks,
// which push every far child as the reference does.
struct ChildPair {
    bool push, any;             // push: keep the far child (both children hit); any: a child is hit
    uint32_t wNext, wF;         // next node (the near one when both hit), far node
    float loNext, loF;          // their slab entry distances
};

template <bool ALLFAST = false>
PT_DEV ChildPair cb_pair(const float4& Q0, const float4& Q1, const float4& Q2, const float4& Q3, const SlabRay& R,
                         uint32_t negMask, float tMin, float tMax)
{
    float XL, XR;
    const float loL = slab_lo_x<ALLFAST>(R, f2(Q0.x, Q0.y), f2(Q0.z, Q0.w), f2(Q1.x, Q1.y), tMin, XL);
    const float loR = slab_lo_x<ALLFAST>(R, f2(Q2.x, Q2.y), f2(Q2.z, Q2.w), f2(Q1.z, Q1.w), tMin, XR);
    const bool isNeg = (negMask & __float_as_uint(Q3.z)) != 0u;
    const uint32_t wL = __float_as_uint(Q3.x), wR = __float_as_uint(Q3.y);
    const bool hL = XL > loL && tMax > loL;
    const bool hR = XR > loR && tMax > loR;
    const bool takeL = hL && (!hR || !isNeg);
    ChildPair c;
    c.push = hL && hR;
    c.any = hL || hR;
    c.wNext = takeL ? wL : wR;
    c.loNext = takeL ? loL : loR;
    c.wF = isNeg ? wL : wR;
    c.loF = isNeg ? loL : loR;
    return c;
}

template <bool ALLFAST = false>
PT_DEV ChildPair cb_children(const float4* __restrict__ cnodes, uint32_t cur, const SlabRay& R, uint32_t negMask,
                             float tMin, float tMax)
{
    return cb_pair<ALLFAST>(cnodes[4 * cur], cnodes[4 * cur + 1], cnodes[4 * cur + 2], cnodes[4 * cur + 3], R, negMask,
                            tMin, tMax);
}

// The reference's pending far children at leaf `leafOff` (after a leaf raised t_max): its stack
// holds, for every interior node on the path to the leaf where the path took the near child, the
// far child (trace.cu:75) -- bottom to top in path order.  The path is found from the root by the
// first primitive of each second child (child-box record Q3.w; leaves hold their primitives in DFS
// order, host-checked), and a far child whose box the ray does not meet at all (X <= lo) is left out
// (no t_max makes it pass).  Rebuilt entries include every one the walk kept, so the lane resumes
// exactly where the reference stands.
PT_DEV void repair_pending(const float4* __restrict__ cnodes, uint2* stack, const SlabRay& R, uint32_t negMask, float tMin,
                           uint32_t rootWord, uint32_t leafOff, uint32_t& sp)
{
    sp = 0;
    uint32_t n = rootWord;
    while ((n >> 24) == 0u) {
        const float4 Q0 = cnodes[4 * n], Q1 = cnodes[4 * n + 1], Q2 = cnodes[4 * n + 2], Q3 = cnodes[4 * n + 3];
        const bool inR = leafOff >= __float_as_uint(Q3.w);
        const bool isNeg = (negMask & __float_as_uint(Q3.z)) != 0u;   // near child = second when negative
        float X;                                                     // the other child's box (Q0..Q2 layout)
        const float lo = slab_lo_x(R, inR ? f2(Q0.x, Q0.y) : f2(Q2.x, Q2.y), inR ? f2(Q0.z, Q0.w) : f2(Q2.z, Q2.w),
                                   inR ? f2(Q1.x, Q1.y) : f2(Q1.z, Q1.w), tMin, X);
        if (inR == isNeg && X > lo) {                                // the path took the near child
            stack[64u * sp] = make_uint2(__float_as_uint(inR ? Q3.x : Q3.y), __float_as_uint(lo));
            ++sp;
        }
        n = __float_as_uint(inR ? Q3.y : Q3.x);
    }
}

// The interior walk of the resumable traversal (trace.cu:66-77 per visited node): descend until a
// leaf is reached (returns false, cur = leaf word) or the stack holds no entry that passes its
// re-test (returns true).  Written for few exec-mask operations (the CU's one scalar unit serves
// all its waves): ALLFAST (wave-uniform, decided by the caller) drops the per-lane exact-form
// branch of the slab test, and the far child is written to the stack unconditionally -- the slot
// above the top, inside the lane's column since an interior node has at most depth - 2 pending
// entries -- with the stack pointer advanced only when the far child is to be kept (ChildPair).
template <bool STATS, bool ALLFAST>
PT_DEV bool walk_interior(const float4* __restrict__ cnodes, uint2* stack, const SlabRay& R, uint32_t negMask,
                          float tMin, float tMax, uint32_t& cur, uint32_t& sp, Counters& cnt)
{
    while ((cur >> 24) == 0u) {
        if (STATS) { cnt.node_tests += 2; wave_tick(cnt.w_node); }
        const ChildPair ch = cb_children<ALLFAST>(cnodes, cur, R, negMask, tMin, tMax);
        stack[64u * sp] = make_uint2(ch.wF, __float_as_uint(ch.loF));
        sp += ch.push ? 1u : 0u;
        if (ch.any) {
            cur = ch.wNext;
        } else {
            bool found = false;
            while (sp > 0) {
                const uint2 e = stack[64u * (--sp)];
                if (tMax > __uint_as_float(e.y)) { cur = e.x; found = true; break; }
            }
            if (!found) return true;
        }
    }
    return false;
}

template <bool STATS>
PT_DEV uint32_t traverse_cb(const float4* __restrict__ cnodes, const float4* __restrict__ prims, uint2* stack,
                            const TraceParams& P, f3 o, f3 d, float& tHit, Counters& cnt)
{
    const float tMin = 0.001f;
    float tMax = kFltMax;
    SlabRay R;
    R.o = o;
    R.ix = rcp_rn(d.x);
    R.iy = rcp_rn(d.y);
    R.iz = rcp_rn(d.z);
    R.fast = P.slabFast && __builtin_isfinite(R.ix) && __builtin_isfinite(R.iy) && __builtin_isfinite(R.iz);
    R.ox2 = f2(o.x, o.x);
    R.oy2 = f2(o.y, o.y);
    R.oz2 = f2(o.z, o.z);
    R.ix2 = f2(R.ix, R.ix);
    R.iy2 = f2(R.iy, R.iy);
    R.iz2 = f2(R.iz, R.iz);
    const uint32_t negMask = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
    uint32_t sp = 0, elem = 0xffffffffu, cur = P.rootWord;
    // pops the next pending far child that still passes its box test under the current t_max
    auto pop = [&]() -> bool {
        while (sp > 0) {
            const uint2 e = stack[64u * (--sp)];
            if (tMax > __uint_as_float(e.y)) { cur = e.x; return true; }
        }
        return false;
    };
    if (STATS) { cnt.node_tests++; wave_tick(cnt.w_node); }
    float X;
    const float lo0 = slab_lo_x(R, f2(P.rootBox[0], P.rootBox[1]), f2(P.rootBox[2], P.rootBox[3]),
                                f2(P.rootBox[4], P.rootBox[5]), tMin, X);
    bool done = !(X > lo0 && tMax > lo0);
    uint64_t tPhase = STATS ? __builtin_amdgcn_s_memtime() : 0;
    while (!done) {
        while ((cur >> 24) == 0u) {                               // interior walk
            if (STATS) { cnt.node_tests += 2; wave_tick(cnt.w_node); }
            const ChildPair ch = cb_children(cnodes, cur, R, negMask, tMin, tMax);   // trace.cu:66-77
            if (ch.push) {
                stack[64u * sp] = make_uint2(ch.wF, __float_as_uint(ch.loF));
                ++sp;
            }
            if (ch.any) {
                cur = ch.wNext;
            } else if (!pop()) {
                done = true;
                break;
            }
        }
        if (STATS) wave_time(cnt.cyc_node, tPhase);
        if (done) break;
        uint32_t leafOff = cur & 0xffffffu, leafCnt = cur >> 24;  // in-order leaf tests
        const uint32_t leaf0 = leafOff;
        const float tLeaf = tMax;
        if (STATS) leaf_round_stats(prims, leafOff, leafCnt, cnt);
        while (leafCnt > 0) {
            if (STATS) { cnt.prim_tests++; wave_tick(cnt.w_prim); leaf_position_stats(prims, leafOff, cnt); }
            float t;
            if (prim_hit(prims, leafOff, o, d, tMin, tMax, t)) {
                tMax = t;
                elem = leafOff;
            }
            ++leafOff;
            --leafCnt;
        }
        // t_max ended the leaf above where it started (the sphere's far-root quirk, ChildPair): boxes
        // dropped for failing an earlier, smaller t_max may pass now.  (A rise undone within the leaf
        // needs nothing: every dropped box failed a t_max at least as large as the one left.)
        const bool rose = tMax > tLeaf;
        if (__ballot(rose) != 0ull && rose) {                  // rare: a uniform test first
            repair_pending(cnodes, stack, R, negMask, tMin, P.rootWord, leaf0, sp);
            if (STATS) cnt.repairs++;
        }
        if (STATS) wave_time(cnt.cyc_leaf, tPhase);
        if (!pop()) done = true;
    }
    tHit = tMax;
    return elem;
}

// ---------------------------------------------------------------------------------------------
// Resumable child-box traversal (WW = 100 + Q).  The wave leaves the traversal as soon as at most
// Q/64 of the lanes that entered are still walking, shades the finished ones, and resumes the stragglers'
// traversals -- node, stack pointer, t_max, closest primitive; the stack itself stays in LDS --
// together with the new rays of the shaded lanes.  The long tail of a wave's traversal (a few
// lanes with deep walks while the rest idle) then overlaps other lanes' next segments.  Every
// lane performs exactly the same sequence of tests as traverse_cb; only when differs.
// ---------------------------------------------------------------------------------------------
struct TravState {
    uint32_t cur, sp, elem;
    float tMax;
};

// The interior walk is walk_interior (the lean form: wave-uniform slab-form choice, unconditional
// far-child write).  WW = 200 + EXITQ selects this traversal.  NOREPAIR (a test-only instantiation,
// pt_set_rise_repair) skips repair_pending: the negative control that shows a scene exercises it.
template <bool STATS, int EXITQ, bool NOREPAIR = false>
PT_DEV bool traverse_cb_phase(const float4* __restrict__ cnodes, const float4* __restrict__ prims, uint2* stack,
                              const TraceParams& P, f3 o, f3 d, bool fresh, TravState& ts, Counters& cnt)
{
    const float tMin = 0.001f;
    SlabRay R;
    R.o = o;
    R.ix = rcp_rn(d.x);
    R.iy = rcp_rn(d.y);
    R.iz = rcp_rn(d.z);
    R.fast = P.slabFast && __builtin_isfinite(R.ix) && __builtin_isfinite(R.iy) && __builtin_isfinite(R.iz);
    R.ox2 = f2(o.x, o.x);
    R.oy2 = f2(o.y, o.y);
    R.oz2 = f2(o.z, o.z);
    R.ix2 = f2(R.ix, R.ix);
    R.iy2 = f2(R.iy, R.iy);
    R.iz2 = f2(R.iz, R.iz);
    const uint32_t negMask = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
    const uint32_t nAct = (uint32_t)__popcll(__ballot(1));
    bool done = false;
    if (fresh) {
        ts.tMax = kFltMax;
        ts.sp = 0;
        ts.elem = 0xffffffffu;
        ts.cur = P.rootWord;
        if (STATS) { cnt.node_tests++; wave_tick(cnt.w_node); }
        float X;
        const float lo0 = slab_lo_x(R, f2(P.rootBox[0], P.rootBox[1]), f2(P.rootBox[2], P.rootBox[3]),
                                    f2(P.rootBox[4], P.rootBox[5]), tMin, X);
        done = !(X > lo0 && ts.tMax > lo0);
    }
    uint32_t sp = ts.sp, cur = ts.cur, elem = ts.elem;
    float tMax = ts.tMax;
    auto pop = [&]() -> bool {
        while (sp > 0) {
            const uint2 e = stack[64u * (--sp)];
            if (tMax > __uint_as_float(e.y)) { cur = e.x; return true; }
        }
        return false;
    };
    uint64_t tPhase = STATS ? __builtin_amdgcn_s_memtime() : 0;
    const bool allFast = __ballot(!R.fast) == 0;                         // wave-uniform
    while (!done) {
        done = allFast ? walk_interior<STATS, true>(cnodes, stack, R, negMask, tMin, tMax, cur, sp, cnt)
                       : walk_interior<STATS, false>(cnodes, stack, R, negMask, tMin, tMax, cur, sp, cnt);
        if (STATS) wave_time(cnt.cyc_node, tPhase);
        if (done) break;
        uint32_t leafOff = cur & 0xffffffu, leafCnt = cur >> 24;
        const uint32_t leaf0 = leafOff;
        const float tLeaf = tMax;
        if (STATS) leaf_round_stats(prims, leafOff, leafCnt, cnt);
        while (leafCnt > 0) {
            if (STATS) { cnt.prim_tests++; wave_tick(cnt.w_prim); leaf_position_stats(prims, leafOff, cnt); }
            float t;
            if (prim_hit(prims, leafOff, o, d, tMin, tMax, t)) {
                tMax = t;
                elem = leafOff;
            }
            ++leafOff;
            --leafCnt;
        }
        // t_max ended the leaf above where it started (the sphere's far-root quirk, ChildPair): boxes
        // dropped for failing an earlier, smaller t_max may pass now.  (A rise undone within the leaf
        // needs nothing: every dropped box failed a t_max at least as large as the one left.)
        const bool rose = tMax > tLeaf;
        if (!NOREPAIR && __ballot(rose) != 0ull && rose) {     // rare: a uniform test first
            repair_pending(cnodes, stack, R, negMask, tMin, P.rootWord, leaf0, sp);
            if (STATS) cnt.repairs++;
        }
        if (STATS) wave_time(cnt.cyc_leaf, tPhase);
        if (!pop()) { done = true; break; }
        // early exit once at most EXITQ/64 of the lanes that entered are still walking
        if ((uint32_t)__popcll(__ballot(1)) * 64u <= nAct * (uint32_t)EXITQ) break;
    }
    ts.sp = sp;
    ts.cur = cur;
    ts.elem = elem;
    ts.tMax = tMax;
    return done;
}

// Surface data of the closest hit (Hittable.inl:126-144 + the shape's normal/uv), rebuilt once.
struct Surface {
    f3 p, n;
    float u, v;
};

PT_DEV Surface surface_of(const float4& r0, const float4& r1, const float4& r2, uint32_t type, f3 o, f3 d, float t,
                          bool needUV)
{
    const LocalRay r = to_local(r0, r1, r2, o, d);
    const f3 lp = add(r.o, scale(t, r.d));                 // r.at(t) in object space
    f3 n;
    float u = 0.0f, v = 0.0f;
    switch (type) {
    case SPHERE:
        n = normalize(lp);
        if (needUV) {
            const float theta = acos_sel(n.y);
            const float phi = atan2_sel(n.z, n.x);
            u = 1.0f - div_two_pi(phi);
            v = div_pi(theta);
        }
        break;
    case CYLINDER:
        n = mk(lp.x, 0.0f, lp.z);
        if (needUV) {
            const float phi = atan2_sel(n.z, n.x);
            u = 1.0f - div_two_pi(phi);
            v = 1.0f - (lp.y * 0.5f + 0.5f);
        }
        break;
    case DISK:
    case QUAD: {
        n = mk(0.0f, 1.0f, 0.0f);
        const float hx = r.o.x + r.d.x * t;
        const float hz = r.o.z + r.d.z * t;
        u = hx * 0.5f + 0.5f;
        v = 1.0f - (hz * 0.5f + 0.5f);
        break;
    }
    case CONE:        // quadricNormal<1,-1,1>: the trailing "+ G/H/I" (int 0) turns -0 into +0
        n = mk(2.0f * lp.x + 0.0f, 2.0f * (-lp.y) + 0.0f, 2.0f * lp.z + 0.0f);
        break;
    case PARABOLOID:  // quadricNormal<1,0,1,0,0,0,0,-1>
        n = mk(2.0f * lp.x + 0.0f, -1.0f, 2.0f * lp.z + 0.0f);
        break;
    default: {        // CUBE: Hittable.inl:345-357
        const float ax = fabsf(lp.x), ay = fabsf(lp.y), az = fabsf(lp.z);
        if (ax > ay && ax > az) n = mk(lp.x > 0.0f ? 1.0f : -1.0f, 0.0f, 0.0f);
        else if (ay > ax && ay > az) n = mk(0.0f, lp.y > 0.0f ? 1.0f : -1.0f, 0.0f);
        else n = mk(0.0f, 0.0f, lp.z > 0.0f ? 1.0f : -1.0f);
        break;
    }
    }
    f3 tmp;                                                 // Hittable.inl:131-134
    tmp.x = n.x * r0.x + n.y * r0.y + n.z * r2.x;           // (r0.x, r1.x, r2.x)
    tmp.y = n.x * r0.z + n.y * r0.w + n.z * r2.y;           // (r0.y, r1.y, r2.y)
    tmp.z = n.x * r1.x + n.y * r1.y + n.z * r2.z;           // (r0.z, r1.z, r2.z)
    Surface s;
    s.p = add(o, scale(t, d));
    const f3 on = normalize(tmp);
    s.n = dot(d, on) < 0.0f ? on : neg(on);                 // HitRecord.h:18-24
    s.u = u;
    s.v = v;
    return s;
}

// MonteCarlo.h:5-22 tangent frame
PT_DEV void tangent_frame(f3 N, f3& t, f3& b)
{
    const f3 up = fabsf(N.z) < 0.999f ? mk(0.0f, 0.0f, 1.0f) : mk(1.0f, 0.0f, 0.0f);
    t = normalize(cross(up, N));
    b = cross(N, t);
}

PT_DEV float d_ggx(float NdotH, float a2)     // brdf.h:11-15
{
    const float dd = (NdotH * a2 - NdotH) * NdotH + 1.0f;
    return a2 / (kPi * dd * dd);
}

// importanceSampleGGXVNDF (MonteCarlo.h:73-101) with r = sqrt(u0) and (sin, cos)(2 pi u1) supplied
// by the caller (shared with the cosine lobe, MonteCarlo.h:24-30, see shade)
PT_DEV f3 vndf_sample_rsc(f3 V, float r, float s, float c, float a)
{
    const f3 Vh = normalize(mk(a * V.x, a * V.y, V.z));
    const float lensq = Vh.x * Vh.x + Vh.y * Vh.y;
    const f3 T1 = lensq > 0.0f ? scale(rcp_sqrt_rn(lensq), mk(-Vh.y, Vh.x, 0.0f)) : mk(1.0f, 0.0f, 0.0f);
    const f3 T2 = cross(Vh, T1);
    const float t1 = r * c;
    float t2 = r * s;
    const float sv = 0.5f * (1.0f + Vh.z);
    t2 = (1.0f - sv) * sqrt_rn(1.0f - t1 * t1) + sv * t2;
    const f3 Nh = add(add(scale(t1, T1), scale(t2, T2)), scale(sqrt_rn(clamp01(1.0f - t1 * t1 - t2 * t2)), Vh));
    return normalize(mk(a * Nh.x, a * Nh.y, clamp01(Nh.z)));
}

PT_DEV float vndf_pdf(f3 H, f3 V, float a)    // MonteCarlo.h:104-114
{
    const float a2 = a * a;
    const float NdotH = H.z;
    const float VdotH = clamp01(dot(V, H));
    const float G1 = (2.0f * V.z) / (V.z + sqrt_rn(a2 + (1.0f - a2) * (V.z * V.z)));
    const float Dv = (G1 * VdotH * d_ggx(NdotH, a2)) / V.z;
    return Dv / (4.0f * VdotH);
}

PT_DEV f3 specular_ggx(f3 F0, float NdotV, float NdotL, float NdotH, float VdotH, float a2)  // brdf.h:56-62
{
    const float D = d_ggx(NdotH, a2);
    float sv, sl;                                                          // brdf.h:18-24
    sqrt2_rn((-NdotV * a2 + NdotV) * NdotV + a2, (-NdotL * a2 + NdotL) * NdotL + a2, sv, sl);
    const float lv = NdotL * sv;
    const float ll = NdotV * sl;
    const float Vis = 0.5f / (lv + ll + 1e-5f);
    const float v = 1.0f - VdotH;                                          // brdf.h:27-32
    const float v2 = v * v;
    const float p = v2 * v2 * v;
    const f3 F = adds(scale(1.0f - p, F0), p);
    return scale(D * Vis, F);
}

// Per-lane path state of the megakernel (trace.cu:158-199 + getColor's loop variables).
struct PathState {
    f3 o, d;          // current ray
    f3 L, T;          // radiance and throughput of the current path (trace.cu:104-105)
    f3 sum;           // CL builds: the running accumulation value (trace.cu:196); else the sum of the
                      // finished paths of the current render() call (trace.cu:186) -- see get_color
    uint32_t slot;    // float index of this lane's slice of the dynamic LDS holding the other of the
                      // two: x, y, z at lds_f()[slot], [slot + 64], [slot + 128]
    uint32_t s, c, bounce;
    bool alive;
};

// camera ray of one sample (trace.cu:190-192, Camera.inl:25-28): two uniforms, x then y
PT_DEV void camera_ray(const TraceParams& P, float fx, float fy, Xorwow& rng, f3& o, f3& d)
{
    const float u = (fx + uniform(rng)) / P.fwidth;
    const float v = (fy + uniform(rng)) / P.fheight;
    o = P.cam.origin;
    d = normalize(add(add(P.cam.llc, scale(u, P.cam.horizontal)), scale(v, P.cam.vertical)));
}

// One iteration of getColor's bounce loop after hitBVH (trace.cu:114-152): miss -> sky, hit ->
// emission + Material::sample + throughput update.  Returns true when the path ends.
template <bool STATS>
PT_DEV bool shade(const TraceParams& P, const float4* __restrict__ prims, uint32_t e, float t, PathState& ps,
                  Xorwow& rng, Counters& cnt)
{
    if (e == 0xffffffffu) {                                                   // trace.cu:115-134
        f3 sky = splat(0.0f);
        if (P.skybox != 0) {
            if (STATS) { cnt.sky++; wave_tick(cnt.w_sky); }
            const float theta = acos_sel(ps.d.y);
            const float phi = atan2_sel(ps.d.z, ps.d.x);
            const float v = div_pi(theta);
            const float u = div_two_pi(phi);
            sky = tex2d(P.skyTex, u, v);
        }
        ps.L = add(ps.L, mul(ps.T, sky));
        return true;
    }
    if (STATS) { cnt.hits++; wave_tick(cnt.w_hits); }
    // every load the hit needs is issued here, together: material, then the primitive's rows for
    // rebuilding the hit record (the shading chain is latency-bound)
    const float4 m0 = P.mats[3 * e + 0];
    const float4 m1 = P.mats[3 * e + 1];
    const float4 m2 = P.mats[3 * e + 2];
    const float4 q0 = prims[4 * e + 0];
    const float4 q1 = prims[4 * e + 1];
    const float4 q2 = prims[4 * e + 2];
    const uint32_t ptype = __float_as_uint(prims[4 * e + 3].x);
    ps.L = add(ps.L, mul(ps.T, mk(m1.x, m1.y, m1.z)));                      // trace.cu:139
    if (ps.bounce == 4) {
        // 5th segment: its scattered ray is discarded (trace.cu:109); only the two uniforms of
        // Material.inl:40-41 are observable.
        (void)uniform(rng);
        (void)uniform(rng);
        return true;
    }
    const uint32_t texIdx = __float_as_uint(m2.x);
    const uint32_t mtype = __float_as_uint(m2.y);
    const Surface sf = surface_of(q0, q1, q2, ptype, ps.o, ps.d, t, texIdx != 0);
    f3 tg, bt;
    tangent_frame(sf.n, tg, bt);
    const f3 wo = neg(ps.d);                                                  // MonteCarlo.h:15-22
    const f3 V = normalize(add(add(scale(wo.x, mk(tg.x, bt.x, sf.n.x)), scale(wo.y, mk(tg.y, bt.y, sf.n.y))),
                               scale(wo.z, mk(tg.z, bt.z, sf.n.z))));
    f3 base = mk(m0.x, m0.y, m0.z);
    if (texIdx != 0) {                                                        // Material.inl:26-35
        const f3 tap = tex2d(P.textures[texIdx - 1], sf.u, sf.v);
        base = mk(pow_(tap.x, 2.2f), pow_(tap.y, 2.2f), pow_(tap.z, 2.2f));
    }
    float rnd0 = uniform(rng);
    const float rnd1 = uniform(rng);
    const float rough = m0.w, metal = m1.w;
    const float a = rough * rough;
    const float a2 = a * a;
    f3 dir = splat(0.0f), att = splat(0.0f);
    float pdf = 0.0f;
    bool killed = false;
    // Lobe sampling.  cosine_sample(u0, u1) needs sincos(2 pi u0) and sqrt(u1); vndf_sample(u0, u1)
    // needs sqrt(u0) and sincos(2 pi u1): one shared sincos and sqrt with per-lane operands serve
    // both lobes (a wave shading LAMBERT_GGX runs both), each lane computing exactly its own lobe.
    bool specular = mtype == 1u;
    if (mtype == 2u) {                                                        // LAMBERT_GGX (:101-144)
        if (rnd0 < 0.5f) rnd0 = 2.0f * rnd0;
        else { rnd0 = 2.0f * (rnd0 - 0.5f); specular = true; }
    }
    float sn, cs;
    sincos_pos(kTwoPi * (specular ? rnd1 : rnd0), sn, cs);
    // sqrt of the lobe's radius uniform and the cosine lobe's sin(theta) behind one range guard
    float sq, sinTheta;
    sqrt2_rn(specular ? rnd0 : rnd1, 1.0f - rnd1, sq, sinTheta);
    if (mtype == 0u) {                                                        // LAMBERT (Material.inl:67-72)
        dir = mk(cs * sinTheta, sn * sinTheta, sq);                            // cosine_sample
        pdf = div_pi(dir.z);
        att = scale(kInvPi, base);
    } else if (mtype <= 2u) {
        if (specular) {
            dir = reflect(neg(V), vndf_sample_rsc(V, sq, sn, cs, a));
        } else {
            dir = mk(cs * sinTheta, sn * sinTheta, sq);
        }
        if (dir.z < 0.0f) {
            killed = true;                                                    // pdf = 1, attenuation 0
        } else {
            const float NdotV = fabsf(V.z) + 1e-5f;
            const f3 H = normalize(add(V, dir));
            const float VdotH = clamp01(dot(V, H));
            const float NdotH = clamp01(H.z);
            const float NdotL = clamp01(dir.z);
            const float ggxPdf = vndf_pdf(H, V, a);
            const f3 F0 = lerp(splat(0.04f), base, metal);
            const f3 kS = specular_ggx(F0, NdotV, NdotL, NdotH, VdotH, a2);
            if (mtype == 1u) {                                                // GGX (:74-99)
                pdf = ggxPdf;
                att = kS;
            } else {
                const float cosinePdf = div_pi(dir.z);
                pdf = (ggxPdf + cosinePdf) * 0.5f;
                att = add(scale(1.0f - metal, scale(kInvPi, base)), kS);
            }
        }
    }
    if (killed || is_zero(att) || pdf == 0.0f) return true;                  // trace.cu:145-148
    // Material.inl:57: normalize(tangentToWorld(...)), which itself normalizes
    const f3 sd = normalize(normalize(add(add(scale(dir.x, tg), scale(dir.y, bt)), scale(dir.z, sf.n))));
    const f3 w = divs(scale(fabsf(dot(sd, sf.n)), att), pdf);                 // trace.cu:150
    ps.T = mul(ps.T, w);
    ps.o = sf.p;
    ps.d = sd;
    ++ps.bounce;
    return false;
}

struct PixelCtx {
    bool valid;
    uint32_t px, py;
    uint32_t li;      // local pixel index: contexts hold < 2^30 pixels (pt_create_banded)
    size_t npix;      // (plane offsets k * npix + li reach past 2^32 in the 10-plane run-ahead stash)
};

PT_DEV PixelCtx pixel_of(const TraceParams& P, uint32_t tile, uint32_t lane)
{
    PixelCtx pc;
    pc.npix = (size_t)P.rows * P.width;
    if (P.scatterWaves) {
        // scattered mapping: lane k of wave w takes local pixel k * waves + w, so every wave holds
        // pixels from the whole tile of rows and all waves cost about the same
        const size_t li = (size_t)lane * P.scatterWaves + tile;
        pc.valid = tile < P.scatterWaves && li < pc.npix;
        pc.li = pc.valid ? li : 0;
        const uint32_t ly = (uint32_t)(pc.li / P.width);
        pc.px = (uint32_t)(pc.li - (size_t)ly * P.width);
        pc.py = global_row(ly, P.rowOffset, P.rowStride, P.bandShift);
        return pc;
    }
    const uint32_t tileX = tile & 0xffffu, tileY = tile >> 16;   // packed (order entries)
    pc.px = tileX * 8u + (lane & 7u);
    const uint32_t ly = tileY * 8u + (lane >> 3);
    pc.valid = tileY < P.tilesY && pc.px < P.width && ly < P.rows;
    pc.py = global_row(ly, P.rowOffset, P.rowStride, P.bandShift);
    pc.li = (size_t)ly * P.width + pc.px;
    return pc;
}

// Where the current render() call's colour sum (touched once per sample) and the running
// accumulation value (touched once per call) live.  CL (the six-wave builds, 80 VGPRs): the colour
// sum in the wave's LDS slice, the accumulation value in registers -- the register allocator spills
// the value used least often, and a per-call spill costs an eighth of a per-sample one at the
// reference's 8 spp per call (C3 224.2 -> 221.7 ms).  Otherwise the reverse: the five- and four-wave
// builds have the registers, and an LDS round trip per sample cost the deep-BVH build (4 waves/SIMD)
// 2.6 % (profiles/r05_six_waves.json).
PT_DEV f3 slice_get(const PathState& ps)
{
    const float* c = lds_f() + ps.slot;
    return mk(c[0], c[64], c[128]);
}

PT_DEV void slice_set(const PathState& ps, const f3& v)
{
    float* c = lds_f() + ps.slot;
    c[0] = v.x;
    c[64] = v.y;
    c[128] = v.z;
}

template <bool CL> PT_DEV f3 get_color(const PathState& ps) { return CL ? slice_get(ps) : ps.sum; }
template <bool CL> PT_DEV f3 get_accum(const PathState& ps) { return CL ? ps.sum : slice_get(ps); }

template <bool CL> PT_DEV void set_color(PathState& ps, const f3& v)
{
    if (CL) slice_set(ps, v);
    else ps.sum = v;
}

template <bool CL> PT_DEV void set_accum(PathState& ps, const f3& v)
{
    if (CL) ps.sum = v;
    else slice_set(ps, v);
}

template <bool AUX, bool CL>
PT_DEV void load_pixel(const TraceParams& P, const PixelCtx& pc, Xorwow& rng, PathState& ps, uint32_t accL)
{
    // AUX: resume launches (see ssg_fold_kernel; pixels the fold finished are skipped by the caller)
    rng.d = P.rng[pc.li];
    rng.v0 = P.rng[pc.npix + pc.li];
    rng.v1 = P.rng[2 * pc.npix + pc.li];
    rng.v2 = P.rng[3 * pc.npix + pc.li];
    rng.v3 = P.rng[4 * pc.npix + pc.li];
    rng.v4 = P.rng[5 * pc.npix + pc.li];
    ps.slot = accL;
    if (!P.ignoreFirst || (AUX && P.fold)) {     // the first call of an ignoreHistory launch overwrites it
        const float4 a = P.accum[pc.li];
        set_accum<CL>(ps, mk(a.x, a.y, a.z));
    } else if (CL) {
        ps.sum = splat(0.0f);
    }
    f3 color = splat(0.0f);
    ps.L = splat(0.0f);
    ps.T = splat(1.0f);
    ps.s = ps.c = ps.bounce = 0;
    ps.alive = P.chunks > 0 && P.spp > 0;
    if (AUX && P.fold) {                         // mid-launch state left by ssg_fold_kernel
        const uint32_t* F = P.fold;
        color = mk(__uint_as_float(F[(F_COL + 0) * pc.npix + pc.li]), __uint_as_float(F[(F_COL + 1) * pc.npix + pc.li]),
                   __uint_as_float(F[(F_COL + 2) * pc.npix + pc.li]));
        const uint32_t sc = F[F_SC * pc.npix + pc.li];
        ps.s = sc & 0xffffu;
        ps.c = sc >> 16;
        ps.alive = ps.c < P.chunks;
    }
    set_color<CL>(ps, color);
}

// Run-ahead (MODE 4): the previous launch's stash of this call's first k samples (same camera, scene,
// textures, sky and RNG state: the host checked the key) -- their colour sum in sample order from 0
// and the XORWOW state after them.  A stash longer than this call's spp cannot be split: dropped.
template <bool CL>
PT_DEV void ahead_load(const TraceParams& P, const PixelCtx& pc, Xorwow& rng, PathState& ps)
{
    const uint32_t* A = P.ahead;
    const size_t n = pc.npix, li = pc.li;
    const uint32_t k = A[3 * n + li];
    if (k == 0u || k > P.spp) return;
    set_color<CL>(ps, mk(__uint_as_float(A[li]), __uint_as_float(A[n + li]), __uint_as_float(A[2 * n + li])));
    ps.s = k;
    rng.d = A[4 * n + li];
    rng.v0 = A[5 * n + li];
    rng.v1 = A[6 * n + li];
    rng.v2 = A[7 * n + li];
    rng.v3 = A[8 * n + li];
    rng.v4 = A[9 * n + li];
}

template <bool CL>
PT_DEV void store_pixel(const TraceParams& P, const PixelCtx& pc, const Xorwow& rng, const PathState& ps)
{
    // The pixel index passes through an empty asm so the store addresses are recomputed here from
    // one 32-bit register: otherwise the compiler reuses the seven 64-bit addresses of load_pixel and
    // keeps them live (spilled) across the whole tile.  Contexts hold < 2^30 pixels (pt_create).
    uint32_t li = (uint32_t)pc.li;
    asm volatile("" : "+v"(li));
    P.rng[li] = rng.d;
    P.rng[pc.npix + li] = rng.v0;
    P.rng[2 * pc.npix + li] = rng.v1;
    P.rng[3 * pc.npix + li] = rng.v2;
    P.rng[4 * pc.npix + li] = rng.v3;
    P.rng[5 * pc.npix + li] = rng.v4;
    const f3 acc = get_accum<CL>(ps);
    P.accum[li] = make_float4(acc.x, acc.y, acc.z, 1.0f);   // trace.cu:198, once per launch
}

// Run-ahead (MODE 4): after every sample of the NEXT call a lane stashes the call's colour sum so far
// (in sample order from 0), the sample count and the XORWOW state -- the state at a sample start, from
// which the next launch continues (a sample in progress when the tile ends is redone there, from a
// fresh camera ray like its neighbours').
PT_DEV void ahead_store(const TraceParams& P, const PixelCtx& pc, const f3& color, uint32_t k, const Xorwow& rng)
{
    uint32_t li = (uint32_t)pc.li;
    asm volatile("" : "+v"(li));                 // addresses from one register (store_pixel)
    uint32_t* A = P.ahead;
    const size_t n = pc.npix;
    A[li] = __float_as_uint(color.x);
    A[n + li] = __float_as_uint(color.y);
    A[2 * n + li] = __float_as_uint(color.z);
    A[3 * n + li] = k;
    A[4 * n + li] = rng.d;
    A[5 * n + li] = rng.v0;
    A[6 * n + li] = rng.v1;
    A[7 * n + li] = rng.v2;
    A[8 * n + li] = rng.v3;
    A[9 * n + li] = rng.v4;
}

// End of a path: sum it into the render() call's color; at the end of a call fold the call into
// the accumulation value (trace.cu:193-198); start the next sample while any remain.  The running
// accumulation value lives in the wave's LDS slice for the whole launch (loaded by load_pixel,
// stored once by store_pixel), so a launch of many render() calls writes each pixel once instead of
// once per call -- the fold and its order (color + accum) are unchanged.
// The end of a render() call's samples (ps.s == spp): fold the call into the accumulation value
// (trace.cu:193-198).  AHEAD: a lane already in run-ahead (ps.c == chunks) has done a whole next call:
// it stashes it and stops; a lane finishing its last call stores its pixel now (the call's RNG state
// and accumulation are final here) and, when the launch makes a stash, goes on with the next call.
template <bool AHEAD, bool CL>
PT_DEV void end_call(const TraceParams& P, const PixelCtx& pc, PathState& ps, const Xorwow& rng)
{
    const f3 color = get_color<CL>(ps);
    if (AHEAD && ps.c == P.chunks) {
        ahead_store(P, pc, color, ps.s, rng);
        ps.alive = false;
        return;
    }
    const bool ignore = (ps.c == 0) && P.ignoreFirst;
    set_accum<CL>(ps, ignore ? color : add(color, get_accum<CL>(ps)));
    set_color<CL>(ps, splat(0.0f));
    ps.s = 0;
    if (++ps.c == P.chunks) {
        ps.alive = false;
        if (AHEAD) {
            store_pixel<CL>(P, pc, rng, ps);
            if (P.aheadMake) P.ahead[3 * pc.npix + (uint32_t)pc.li] = 0u;   // no stash until a next-call sample ends
            ps.alive = P.aheadMake != 0;
        }
    }
}

template <bool STATS, bool AHEAD, bool CL>
PT_DEV void finish_path(const TraceParams& P, PathState& ps, Xorwow& rng, float fx, float fy, Counters& cnt,
                        const PixelCtx& pc)
{
    const f3 color = add(get_color<CL>(ps), ps.L);
    set_color<CL>(ps, color);
    if (STATS) cnt.samples++;
    if (++ps.s == P.spp) end_call<AHEAD, CL>(P, pc, ps, rng);
    else if (AHEAD && ps.c == P.chunks) ahead_store(P, pc, color, ps.s, rng);   // a next-call sample
    if (ps.alive) {
        camera_ray(P, fx, fy, rng, ps.o, ps.d);
        ps.L = splat(0.0f);
        ps.T = splat(1.0f);
        ps.bounce = 0;
    }
}

template <bool STATS>
PT_DEV void flush_counters(const TraceParams& P, const Counters& cnt)
{
    if (!STATS) return;
    atomicAdd(&P.stats[0], (unsigned long long)cnt.node_tests);
    atomicAdd(&P.stats[1], (unsigned long long)cnt.prim_tests);
    atomicAdd(&P.stats[2], (unsigned long long)cnt.hits);
    atomicAdd(&P.stats[3], (unsigned long long)cnt.sky);
    atomicAdd(&P.stats[4], (unsigned long long)cnt.segments);
    atomicAdd(&P.stats[5], (unsigned long long)cnt.samples);
    atomicAdd(&P.stats[6], (unsigned long long)cnt.w_node);
    atomicAdd(&P.stats[7], (unsigned long long)cnt.w_prim);
    atomicAdd(&P.stats[8], (unsigned long long)cnt.w_hits);
    atomicAdd(&P.stats[9], (unsigned long long)cnt.w_sky);
    atomicAdd(&P.stats[10], (unsigned long long)cnt.w_segments);
    atomicAdd(&P.stats[11], (unsigned long long)cnt.cyc_node);
    atomicAdd(&P.stats[12], (unsigned long long)cnt.cyc_leaf);
    atomicAdd(&P.stats[13], (unsigned long long)cnt.cyc_shade);
    atomicAdd(&P.stats[14], (unsigned long long)cnt.cyc_total);
    atomicAdd(&P.stats[15], (unsigned long long)cnt.cyc_lane_idle);
    atomicAdd(&P.stats[16], (unsigned long long)cnt.w_leaf_rounds);
    atomicAdd(&P.stats[17], (unsigned long long)cnt.w_fam_exec);
    atomicAdd(&P.stats[18], (unsigned long long)cnt.w_fam_ideal);
    atomicAdd(&P.stats[19], (unsigned long long)cnt.w_leaf_lanes);
    atomicAdd(&P.stats[20], (unsigned long long)cnt.w_leaf_pairs);
    atomicAdd(&P.stats[21], (unsigned long long)cnt.w_fam_inplace);
    atomicAdd(&P.stats[22], (unsigned long long)cnt.repairs);
}

// One atomic per wave: the first active lane adds n to *cursor; the old value is read back from
// that lane into a scalar register (readfirstlane), so the slot and everything derived from it --
// tile, pixel base, priority -- is wave-uniform for the compiler too (SGPRs, scalar loads).
PT_DEV uint32_t wave_fetch(uint32_t* cursor, uint32_t n)
{
    const unsigned long long m = __ballot(1);
    const uint32_t leader = (uint32_t)(__ffsll((long long)m) - 1);
    uint32_t base = 0;
    if ((threadIdx.x & 63u) == leader) base = atomicAdd(cursor, n);
    return __builtin_amdgcn_readfirstlane(base);
}

// ---------------------------------------------------------------------------------------------
// Speculative sample groups.  A pixel's samples are one serial XORWOW stream, so
// a tile costs as long as its slowest pixel's whole chain.  When a launch holds too few tiles to
// fill the chip (multi-GPU strong scaling, small images), each pixel's chain is cut into G groups:
// group g >= 1 starts at a guessed draw offset (the pixel's measured draw pairs per sample x g x n)
// with the XORWOW state of that offset, and logs each sample's colour and end offset.  A sample
// starts wherever the previous one ended, so two parses of one stream that share a sample start
// coincide from there on: a group's parse becomes the true one where the true parse reaches one of
// its sample starts (a junction).  Each item records its sample starts near its own start; an
// earlier item stops at its first junction with a later one.  ssg_fold_kernel then walks the true
// parse through the logs, folds colours in the reference's order (trace.cu:186-198) and sets the
// final state; whatever the logs do not cover runs in a resume launch.  Results are bit-identical.
// ---------------------------------------------------------------------------------------------
struct SsgLane {
    uint32_t logItem;   // index into the log arrays: pos * J + j, or pos in a patch round (pos: order position)
    uint32_t grp0;      // pos * J: the items of this tile
    uint32_t g;         // group index; G in a patch round (no window of its own)
    uint32_t k;         // samples logged
    uint32_t h;         // next group whose window this parse may reach (G: none)
    uint32_t hStart;    // its start offset
    uint32_t limit;     // samples before the item stops regardless
    // the item's start state word, start offset and (last group) stop offset: ssg_item_start
};

PT_DEV uint32_t ssg_start_word(const TraceParams& P, uint32_t item, uint32_t w, uint32_t lane)
{
    return P.ssgStart[((size_t)item * kStartWords + w) * 64 + lane];
}

// `pos`: the tile's position in the order (the per-item buffers' index), `g`: the item within it.
PT_DEV void ssg_load(const TraceParams& P, uint32_t pos, uint32_t g, uint32_t lane, size_t li, size_t npix,
                     Xorwow& rng, PathState& ps, SsgLane& sl)
{
    const uint32_t G = P.ssgG;
    sl.grp0 = pos * (2 * G - 1);
    sl.k = 0;
    ps.L = splat(0.0f);
    ps.T = splat(1.0f);
    ps.bounce = 0;
    if (P.ssgPatch) {
        // a carrier from the fold's dead end: the true state there, the fold's next candidate group
        const uint32_t* F = P.fold;
        sl.logItem = pos;
        sl.g = G;
        if (!(F[F_FLAG * npix + li] & 1u)) {       // finished pixel: its other fold words are stale
            sl.limit = 0;
            ps.alive = false;
            sl.h = G;
            sl.hStart = 0xffffffffu;
            return;
        }
        rng.d = F[(F_ST + 0) * npix + li];
        rng.v0 = F[(F_ST + 1) * npix + li];
        rng.v1 = F[(F_ST + 2) * npix + li];
        rng.v2 = F[(F_ST + 3) * npix + li];
        rng.v3 = F[(F_ST + 4) * npix + li];
        rng.v4 = F[(F_ST + 5) * npix + li];
        sl.h = min(F[F_H * npix + li], G);
        sl.limit = min(P.ssgCap, P.spp * P.chunks - F[F_DONE * npix + li]);
    } else {
        const uint32_t j = g;                      // item index within the tile
        g = (j + 1) >> 1;
        sl.logItem = sl.grp0 + j;
        sl.g = g;
        if (g == 0) {
            rng.d = P.rng[li];
            rng.v0 = P.rng[npix + li];
            rng.v1 = P.rng[2 * npix + li];
            rng.v2 = P.rng[3 * npix + li];
            rng.v3 = P.rng[4 * npix + li];
            rng.v4 = P.rng[5 * npix + li];
        } else {
            if (ssg_start_word(P, sl.logItem, 0, lane) == 0xffffffffu) {   // the second phase of a pixel that has none
                sl.limit = 0;
                ps.alive = false;
                sl.h = G;
                sl.hStart = 0xffffffffu;
                return;
            }
            rng.d = ssg_start_word(P, sl.logItem, 1, lane);
            rng.v0 = ssg_start_word(P, sl.logItem, 2, lane);
            rng.v1 = ssg_start_word(P, sl.logItem, 3, lane);
            rng.v2 = ssg_start_word(P, sl.logItem, 4, lane);
            rng.v3 = ssg_start_word(P, sl.logItem, 5, lane);
            rng.v4 = ssg_start_word(P, sl.logItem, 6, lane);
            // the group's own start is its first sample start
            __hip_atomic_fetch_or(&P.ssgBits[(size_t)sl.logItem * P.ssgWin * 64 + lane], 1ull, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        }
        sl.h = g + 1;
        sl.limit = P.ssgCap;
    }
    sl.hStart = sl.h < G ? ssg_start_word(P, sl.grp0 + 2 * sl.h - 1, 0, lane) : 0xffffffffu;
    ps.alive = sl.limit > 0;
}

// The item's start (Weyl word d0, draw-pair offset base) and, for the last group, its stop offset:
// constant for the whole item, so they are re-read from the start records (L1/L2) when a sample
// ends instead of being held in registers across the kernel's loop (they pushed the grouped
// instantiation into spills).
PT_DEV void ssg_item_start(const TraceParams& P, const SsgLane& sl, uint32_t lane, size_t li, uint32_t& d0, uint32_t& base,
                           uint32_t& stopOff)
{
    const size_t npix = (size_t)P.rows * P.width;
    if (P.ssgPatch) {
        d0 = P.fold[(F_ST + 0) * npix + li];
        base = P.fold[F_OFF * npix + li];
        stopOff = 0xffffffffu;
    } else if (sl.g == 0) {
        d0 = P.rng[li];
        base = 0;
        stopOff = sl.g + 1 == P.ssgG ? ssg_start_word(P, sl.logItem, 7, lane) : 0xffffffffu;
    } else {
        d0 = ssg_start_word(P, sl.logItem, 1, lane);
        base = ssg_start_word(P, sl.logItem, 0, lane);
        stopOff = sl.g + 1 == P.ssgG ? ssg_start_word(P, sl.logItem, 7, lane) : 0xffffffffu;
    }
}

// End of a path in a speculative item: log it, record the sample start that follows (in the group's
// own window), stop at a junction with a later group or at the item's limit, else start the next
// sample.
template <bool STATS>
PT_DEV void ssg_finish(const TraceParams& P, PathState& ps, Xorwow& rng, float fx, float fy, SsgLane& sl,
                       uint32_t lane, size_t li, Counters& cnt)
{
    uint32_t d0, base, stopOff;
    ssg_item_start(P, sl, lane, li, d0, base, stopOff);
    if (STATS) cnt.samples++;
    const size_t rec = (size_t)sl.logItem * P.ssgCap + sl.k;
    P.ssgLog[(rec * 3 + 0) * 64 + lane] = ps.L.x;
    P.ssgLog[(rec * 3 + 1) * 64 + lane] = ps.L.y;
    P.ssgLog[(rec * 3 + 2) * 64 + lane] = ps.L.z;
    const uint32_t rel = ((rng.d - d0) * kInvWeyl) >> 1;             // draw pairs since the item's start
    P.ssgEnd[rec * 64 + lane] = (uint16_t)rel;
    ++sl.k;
    bool stop = sl.k >= sl.limit;
    if (sl.g - 1u < P.ssgG - 1u && rel < (P.ssgWin * 64u))                    // groups 1 .. G-1
        __hip_atomic_fetch_or(&P.ssgBits[((size_t)sl.logItem * P.ssgWin + rel / 64) * 64 + lane], 1ull << (rel % 64),
                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t off = base + rel;
    stop = stop || off >= stopOff;                                     // the last group: past the expected end
    const uint32_t j = sl.logItem - sl.grp0;
    if (!stop && j >= 2 && !(j & 1u) && !P.ssgPatch && rel + 1 < (P.ssgWin * 64u)) {
        // the second phase has joined the first one's parse (a sample start of item j - 1): from here
        // the two are the same parse, the first carries on
        const uint32_t wa = rel + 1;
        const unsigned long long* bitsA = P.ssgBits + (size_t)(sl.logItem - 1) * P.ssgWin * 64 + lane;
        stop = (__hip_atomic_load(&bitsA[(wa / 64) * 64], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (wa % 64)) & 1ull;
        // the first phase may run behind on the parse the two share: a start ssgLook samples back
        // that it holds means the two coincide from there (the fold continues in its log)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint32_t L = P.ssgLook[q];
            if (!stop && L && sl.k > L) {
                const uint32_t wb = (uint32_t)P.ssgEnd[(rec - L) * 64 + lane] + 1u;
                stop = wb < (P.ssgWin * 64u) &&
                       ((__hip_atomic_load(&bitsA[(wb / 64) * 64], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (wb % 64)) & 1ull);
            }
        }
    }
    while (sl.h < P.ssgG && off > sl.hStart + (P.ssgWin * 64u)) {           // passed that group's windows
        ++sl.h;
        sl.hStart = sl.h < P.ssgG ? ssg_start_word(P, sl.grp0 + 2 * sl.h - 1, 0, lane) : 0xffffffffu;
    }
    // reached the next group's start without meeting group h (the windows overlap the following
    // groups): the candidate becomes the latest group started, whose two phases are still fresh
    while (sl.h + 1 < P.ssgG) {
        const uint32_t nx = ssg_start_word(P, sl.grp0 + 2 * sl.h + 1, 0, lane);
        if (off < nx) break;
        ++sl.h;
        sl.hStart = nx;
    }
    if (!stop && sl.h < P.ssgG && off >= sl.hStart) {
        // junction: a sample start of group h's parse (either phase; an idle phase has no bits)
        const uint32_t w = off - sl.hStart;
        const size_t itA = sl.grp0 + 2 * sl.h - 1;
        if (w < (P.ssgWin * 64u))
            stop = (__hip_atomic_load(&P.ssgBits[(itA * P.ssgWin + w / 64) * 64 + lane], __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT) >> (w % 64)) & 1ull;
        if (!stop && w >= 1)
            stop = (__hip_atomic_load(&P.ssgBits[((itA + 1) * P.ssgWin + (w - 1) / 64) * 64 + lane], __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT) >> ((w - 1) % 64)) & 1ull;
    }
    if (stop) {
        ps.alive = false;
        return;
    }
    camera_ray(P, fx, fy, rng, ps.o, ps.d);
    ps.L = splat(0.0f);
    ps.T = splat(1.0f);
    ps.bounce = 0;
}

// ---------------------------------------------------------------------------------------------
// Kernel A: lane-synchronous segments (traverse, then shade), per-lane path regeneration.
// LDS layout per workgroup: [scene nodes (2 float4 each) | scene prims (4 float4 each)] when
// SCENE_LDS, then WPB wave stacks of stackDepth x 64 u32.
// ---------------------------------------------------------------------------------------------
// The scene copied into the workgroup's LDS (SL >= 1), once per workgroup.
template <int SL, int WPB, int WW>
PT_DEV void stage_scene_impl(const TraceParams& P)
{
    if (SL < 1) return;
    const float4* gnodes = WW >= 3 ? P.cnodes : P.nodes;
    const uint32_t nodeF4 = WW >= 3 ? 4u * P.cnodeCount : 2u * P.nodeCount;
    for (uint32_t i = threadIdx.x; i < nodeF4; i += WPB * 64) lds4[i] = gnodes[i];
    if (SL >= 2)
        for (uint32_t i = threadIdx.x; i < 4u * P.primCount; i += WPB * 64) lds4[nodeF4 + i] = P.prims[i];
    __syncthreads();
}

// The LDS of a wave (trace_kernel's layout): the scene (SL >= 1: child-box records or nodes, SL >= 2:
// primitives too), WPB wave stacks of stackDepth x 64 entries (u32 node index, or uint2 (word, lo) for
// WW >= 3), then one accumulation slice per wave (3 planes of 64 floats).  Recomputed by every user
// from threadIdx, so the pointers stay LDS pointers even in a non-inlined item function.
template <int SL, int WPB, int WW>
struct WaveLds {
    const float4* nodes;
    const float4* prims;
    uint32_t* stack;
    uint32_t accL;            // float index of this lane's accumulation value in the dynamic LDS
};

template <int SL, int WPB, int WW>
PT_DEV WaveLds<SL, WPB, WW> wave_lds(const TraceParams& P)
{
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const float4* gnodes = WW >= 3 ? P.cnodes : P.nodes;
    const uint32_t nodeF4 = WW >= 3 ? 4u * P.cnodeCount : 2u * P.nodeCount;
    const uint32_t sceneF4 = (SL >= 1 ? nodeF4 : 0u) + (SL >= 2 ? 4u * P.primCount : 0u);
    WaveLds<SL, WPB, WW> L;
    L.nodes = SL >= 1 ? lds4 : gnodes;
    L.prims = SL >= 2 ? lds4 + nodeF4 : P.prims;
    const uint32_t stackWords = (WW >= 3 ? 2u : 1u) * P.stackDepth * 64u;
    L.stack = reinterpret_cast<uint32_t*>(lds4 + sceneF4) + wave * stackWords + (WW >= 3 ? 2u : 1u) * lane;
    L.accL = 4u * sceneF4 + WPB * stackWords + wave * 192u + lane;
    return L;
}

// One work item of trace_kernel: the tile at dispatch slot `slot` (MODE 1: the (tile, group) item).
template <bool STATS, int SL, int WPB, int WW, int MINW, bool PERSIST, int MODE>
PT_DEV void run_item(const TraceParams& P, uint32_t slot, Counters& cnt)
{
    // MODE 4 (AHEAD): run-ahead across render() calls.  A launch of one or a few render() calls ends a
    // tile when its slowest pixel has finished; the lanes whose pixels finished first would idle until
    // then (28 % of lane time at 8 spp per call).  Here a lane whose pixel has finished
    // its last call stores the pixel (the call's final RNG state and accumulation value) and goes on
    // with the pixel's NEXT call -- the same XORWOW stream -- stashing after every sample the colour
    // sum so far, the sample count and the state (ahead_store), until the tile ends or a whole next
    // call is done.  A wave leaves the tile as soon as no lane has samples of this launch left.  The
    // next launch continues from the stash when its camera and scene are the ones it was made with
    // (host key, render_impl); otherwise the stored state is the exact one to continue from.
    constexpr bool SSG = MODE == 1, AUX = MODE == 2, STRIP = MODE == 3, AHEAD = MODE == 4;
    // the call's colour sum in LDS (get_color): the plain six-wave launch only (measured there; the
    // run-ahead build was 0.9 % slower with it on the reference's call loop)
    constexpr bool CL = MINW >= 6 && MODE == 0;
    const uint32_t lane = threadIdx.x & 63u;
    const WaveLds<SL, WPB, WW> Lw = wave_lds<SL, WPB, WW>(P);
    const float4* __restrict__ nodes = Lw.nodes;
    const float4* __restrict__ prims = Lw.prims;
    uint32_t* stack = Lw.stack;
    const uint32_t accL = Lw.accL;
    uint32_t tile, grp = 0, pos = slot;              // pos: the tile's position in the order
    if (SSG && !P.ssgPatch) {
        const uint32_t J = 2 * P.ssgG - 1;
        pos = slot / J;
        grp = slot - pos * J;                        // item within the tile (ssg_load)
    }
    tile = P.order ? P.order[pos] : pos;          // packed coordinates (scatter mode: wave index)
    // Issue priority: the cost order puts the most expensive tiles first, and at full occupancy
    // such a tile's chain runs ~3x slower than alone (tools/occupancy_probe.py) -- long enough to
    // end the launch.  Waves on the head of the order take issue slots first (s_setprio), the rest
    // fill the gaps.  pos is wave-uniform (an SGPR), so only one s_setprio executes.  Scheduling
    // only: results are identical.
    if (pos < P.prio[0]) __builtin_amdgcn_s_setprio(3);
    else if (pos < P.prio[1]) __builtin_amdgcn_s_setprio(2);
    else if (pos < P.prio[2]) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
    PixelCtx pc = pixel_of(P, tile, lane);
    const uint64_t tWave = __builtin_amdgcn_s_memtime();
    const bool run = pc.valid && (!AUX || !P.fold || (P.fold[F_FLAG * pc.npix + pc.li] & 1u));
    if (run) {
        Xorwow rng;
        PathState ps;
        SsgLane sl;
        if (SSG) ssg_load(P, pos, grp, lane, pc.li, pc.npix, rng, ps, sl);
        else load_pixel<AUX, CL>(P, pc, rng, ps, accL);
        if (AHEAD && P.aheadUse) {
            ahead_load<CL>(P, pc, rng, ps);
            if (ps.s == P.spp) end_call<true, CL>(P, pc, ps, rng);     // a whole call was stashed
        }
        float fx = (float)(int32_t)pc.px, fy = (float)(int32_t)pc.py;
        camera_ray(P, fx, fy, rng, ps.o, ps.d);
        uint32_t stripK = 0;                     // STRIP: this lane's tile within the unit
        uint64_t tAll = STATS ? __builtin_amdgcn_s_memtime() : 0;
        uint64_t tDone = 0;
        if (WW >= 100) {
            // DEFERQ (WW / 1000, eighths; 0 = off): a wave shades its pending hits only once they are at
            // least DEFERQ/8 of its live lanes.  A lane whose hit is held back skips the traversal
            // rounds until then (its closest hit stays in ts), so hit shading -- the longest branch
            // -- runs for more lanes at once and in fewer rounds.  Every lane still performs its own
            // sequence of operations in order; only the round in which it shades changes.
            // SKYQ (WW / 10000): the same for misses (sky lookup, end of path, next camera ray).
            // DEFERQ + SKYQ <= 8, so when every live lane is ready one class always runs.
            constexpr int DEFERQ = (WW / 1000) % 10, SKYQ = (WW / 10000) % 10;
            constexpr bool NOREPAIR = (WW / 100000) % 10 != 0;     // test-only (pt_set_rise_repair)
            static_assert(DEFERQ + SKYQ <= 8, "a wave whose lanes are all ready must shade one class");
            bool fresh = true, held = false;
            TravState ts = {0u, 0u, 0xffffffffu, kFltMax};
            while (ps.alive) {
                if (AHEAD && __ballot(ps.c < P.chunks) == 0ull) break;   // only run-ahead lanes left
                if (STATS && fresh && !held) { cnt.segments++; wave_tick(cnt.w_segments); }
                bool tdone = true;
                if (!held) {
                    tdone = traverse_cb_phase<STATS, WW % 100, NOREPAIR>(nodes, prims, reinterpret_cast<uint2*>(stack), P,
                                                                ps.o, ps.d, fresh, ts, cnt);
                    fresh = tdone;
                }
                if (DEFERQ > 0 || SKYQ > 0) {
                    const bool hitReady = tdone && ts.elem != 0xffffffffu;
                    const bool missReady = tdone && ts.elem == 0xffffffffu;
                    const uint32_t na = (uint32_t)__popcll(__ballot(1));
                    bool hold = false;
                    if (DEFERQ > 0) hold = hitReady && (uint32_t)__popcll(__ballot(hitReady)) * 8u < na * (uint32_t)DEFERQ;
                    if (SKYQ > 0 && P.skybox != 0)     // without a sky texture a miss costs next to nothing
                        hold = hold || (missReady && (uint32_t)__popcll(__ballot(missReady)) * 8u < na * (uint32_t)SKYQ);
                    held = hold;
                    if (held) continue;
                }
                if (!tdone) continue;                              // suspended: resumes next round
                uint64_t tS = STATS ? __builtin_amdgcn_s_memtime() : 0;
                if (shade<STATS>(P, prims, ts.elem, ts.tMax, ps, rng, cnt)) {
                    if (SSG) ssg_finish<STATS>(P, ps, rng, fx, fy, sl, lane, pc.li, cnt);
                    else finish_path<STATS, AHEAD, CL>(P, ps, rng, fx, fy, cnt, pc);
                    if (STRIP && !ps.alive && stripK + 1 < P.strip) {
                        // Strip units (launches of few samples per pixel): a lane whose pixel is done
                        // stores it and takes the same position in the unit's next tile -- the tile to
                        // the right, so the wave's rays stay spatially coherent -- instead of idling
                        // until the slowest pixel of its tile is done.  Pixels are independent
                        // (their own RNG stream and accumulation value): results are unchanged.
                        const PixelCtx nx = pixel_of(P, tile + stripK + 1, lane);
                        if (nx.valid) {
                            if (!P.discard) store_pixel<CL>(P, pc, rng, ps);   // a cost pre-pass writes nothing
                            pc = nx;
                            ++stripK;
                            load_pixel<false, CL>(P, pc, rng, ps, accL);
                            fx = (float)(int32_t)pc.px;
                            fy = (float)(int32_t)pc.py;
                            camera_ray(P, fx, fy, rng, ps.o, ps.d);
                        }
                    }
                }
                if (STATS) wave_time(cnt.cyc_shade, tS);
                if (STATS && !ps.alive) tDone = __builtin_amdgcn_s_memtime();
            }
        }
        while (WW < 100 && ps.alive) {
            if (STATS) { cnt.segments++; wave_tick(cnt.w_segments); }
            float t;
            const uint32_t e = WW >= 3 ? traverse_cb<STATS>(nodes, prims, reinterpret_cast<uint2*>(stack), P, ps.o, ps.d, t, cnt)
                                       : traverse<STATS, WW>(nodes, prims, stack, ps.o, ps.d, P.slabFast != 0, t, cnt);
            uint64_t tS = STATS ? __builtin_amdgcn_s_memtime() : 0;
            if (shade<STATS>(P, prims, e, t, ps, rng, cnt)) {
                if (SSG) ssg_finish<STATS>(P, ps, rng, fx, fy, sl, lane, pc.li, cnt);
                else finish_path<STATS, false, CL>(P, ps, rng, fx, fy, cnt, pc);
            }
            if (STATS) wave_time(cnt.cyc_shade, tS);
        }
        if (STATS && WW >= 100 && tDone) {
            const uint64_t idle = __builtin_amdgcn_s_memtime() - tDone;
            cnt.cyc_lane_idle += idle;
            if (P.tileIdle && (tile >> 16) < P.tilesY)
                atomicAdd(&P.tileIdle[(tile >> 16) * P.tilesX + (tile & 0xffffu)], (uint32_t)min(idle >> 6, (uint64_t)0x3ffffffu));
        }
        if (STATS) wave_time(cnt.cyc_total, tAll);
        if (SSG) P.ssgCount[(size_t)sl.logItem * 64 + lane] = sl.k;
        else if (AHEAD) {}                    // stored when its last call ended (end_call)
        else if (!P.discard) store_pixel<CL>(P, pc, rng, ps);
        else if (AUX && P.pairsOut)           // cost pre-pass: draw pairs per sample of this pixel
        {
            P.pairsOut[pc.li] = (float)(((rng.d - P.rng[pc.li]) * kInvWeyl) >> 1) / (float)(P.spp * P.chunks);
            P.pairsOut[pc.npix + pc.li] = -1.0f;      // odd-length fraction unknown
        }
    }
    if (P.tileCost && lane == 0 && (tile >> 16) < P.tilesY) {
        const uint32_t cyc = (uint32_t)min(__builtin_amdgcn_s_memtime() - tWave, (uint64_t)0xffffffffu);
        const uint32_t lin = (tile >> 16) * P.tilesX + (tile & 0xffffu);
        // SSG: zeroed before the launch (idle items add ~0)
        if (SSG) atomicAdd(&P.tileCost[lin], cyc / P.ssgG);
        else P.tileCost[lin] = cyc;
        // STRIP: the unit's cost sits at its first tile, the other tiles' entries are 0, so a sort of
        // the tile costs lists the units first (pt_render: the order of a strip launch)
        if (STRIP)
            for (uint32_t k = 1; k < P.strip && (tile & 0xffffu) + k < P.tilesX; ++k) P.tileCost[lin + k] = 0u;
    }
}

// SL = 0: scene read through the caches; 1: BVH nodes staged in LDS; 2: nodes and primitives in LDS.
// One wave = one 8x8 tile.  PERSIST: the grid holds only the resident waves, and each wave takes
// the next dispatch slot from a global counter when its tile is done, so a wave never waits for
// the other waves of its workgroup (which would keep the group's LDS and slots idle).
// MODE 0: plain; 1 (SSG): speculative sample groups (ssg_load / ssg_finish), one work item per
// (tile, group); 2: auxiliary launches -- the resume pass after a grouped launch, and the cost
// pre-pass that also measures draw pairs per sample; 3: strip units; 4: run-ahead across render()
// calls (run_item).  Separate instantiations keep the plain kernel's register allocation free of
// their code.
template <bool STATS, int SL, int WPB, int WW, int MINW, bool PERSIST = false, int MODE = 0>
__global__ void __launch_bounds__(WPB * 64, MINW) trace_kernel(TraceParams P)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    stage_scene_impl<SL, WPB, WW>(P);
    Counters cnt = {};
    uint32_t slot = PERSIST ? wave_fetch(P.tileCursor, 1u) : __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)WPB + wave);
    for (;;) {
    if (slot >= P.numSlots) break;               // also the grid's spare slots past the last item
    run_item<STATS, SL, WPB, WW, MINW, PERSIST, MODE>(P, slot, cnt);
    if (!PERSIST) break;
    slot = wave_fetch(P.tileCursor, 1u);
    }
    if (PERSIST) {
        // the last wave to leave rewinds the cursor for the next launch (every wave has made its
        // final fetch before it counts itself out), so no memset precedes the launch
        if (wave_fetch(P.tileCursor + 1, 1u) == gridDim.x * (uint32_t)WPB - 1 && lane == 0) {
            P.tileCursor[0] = 0;
            P.tileCursor[1] = 0;
        }
    }
    flush_counters<STATS>(P, cnt);
}

// initRandState (initRandState.cu:4-17): curand_init(1984 + x + y * width, 0, 0)
__global__ void __launch_bounds__(256) init_rng_kernel(uint32_t* rng, uint32_t width, uint32_t rows, uint32_t rowOffset,
                                                       uint32_t rowStride, uint32_t bandShift)
{
    const size_t npix = (size_t)rows * width;
    const size_t li = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= npix) return;
    const uint32_t x = (uint32_t)(li % width);
    const uint32_t ly = (uint32_t)(li / width);
    const uint32_t y = global_row(ly, rowOffset, rowStride, bandShift);
    const uint32_t idx = x + y * width;
    const Xorwow s = xorwow_init((uint64_t)(uint32_t)(1984u + idx));
    rng[li] = s.d;
    rng[npix + li] = s.v0;
    rng[2 * npix + li] = s.v1;
    rng[3 * npix + li] = s.v2;
    rng[4 * npix + li] = s.v3;
    rng[5 * npix + li] = s.v4;
}

// tonemap (tonemap.cu:4-27)
__global__ void __launch_bounds__(256) tonemap_kernel(uchar4* out, const float4* accum, size_t npix, uint32_t frames)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    const float4 a = accum[i];
    f3 c = divs(mk(a.x, a.y, a.z), (float)frames);
    c = mul(mk(1.0f / (c.x + 1.0f), 1.0f / (c.y + 1.0f), 1.0f / (c.z + 1.0f)), c);
    const float g = 1.0f / 2.2f;
    const float ch[3] = {pow_(c.x, g), pow_(c.y, g), pow_(c.z, g)};
    unsigned char q[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float f = ch[k] * 255.0f;
        const int32_t v = (f != f) ? 0 : f2i_x86(f);
        q[k] = (unsigned char)(v & 0xff);
    }
    out[i] = make_uchar4(q[0], q[1], q[2], 255);
}

// ---- speculative sample groups: start states and the fold ---------------------
// Both run one lane per pixel, indexed like the trace kernel's items (tile, lane), so the per-item
// buffers ([item][..][64]) are read and written in whole 256-B rows.
PT_DEV bool ssg_pixel(const TraceParams& P, size_t gid, uint32_t& pos, uint32_t& lane, size_t& li)
{
    pos = (uint32_t)(gid >> 6);                      // position in the order: the per-item buffers' index
    lane = (uint32_t)(gid & 63u);
    if (pos >= P.ssgTiles) return false;
    const uint32_t tile = P.order[pos];              // packed tile coordinates
    const uint32_t tileX = tile & 0xffffu, tileY = tile >> 16;
    const uint32_t px = tileX * 8u + (lane & 7u), ly = tileY * 8u + (lane >> 3);
    li = (size_t)ly * P.width + px;
    return tileY < P.tilesY && px < P.width && ly < P.rows;
}

// Group g >= 1 of a pixel starts at draw pair round(g * n * m), m = the pixel's draw pairs per
// sample (the previous launch's, or the cost pre-pass's), strictly increasing in g; its state is
// the pixel's current state advanced that far.
__global__ void __launch_bounds__(256) ssg_guess_kernel(TraceParams P, const float* __restrict__ pairs, uint32_t n,
                                                        uint32_t* __restrict__ start)
{
    uint32_t tile, lane;
    size_t li;
    if (!ssg_pixel(P, (size_t)blockIdx.x * 256 + threadIdx.x, tile, lane, li)) return;
    const size_t npix = (size_t)P.rows * P.width;
    Xorwow st = {P.rng[li], P.rng[npix + li], P.rng[2 * npix + li], P.rng[3 * npix + li], P.rng[4 * npix + li],
                 P.rng[5 * npix + li]};
    const size_t npixAll = (size_t)P.rows * P.width;
    float m = pairs ? pairs[li] : 2.0f;
    m = (m >= 1.0f) ? fminf(m, 6.0f) : 1.0f;       // 1..6 pairs per sample (jitter + up to 5 hits)
    const float podd = pairs ? pairs[npixAll + li] : -1.0f;   // fraction of odd-length samples (< 0: unknown)
    const float var = (pairs && podd >= 0.0f) ? pairs[2 * npixAll + li] : 1.0f;   // variance of pairs per sample
    // the last group stops once its parse passes the expected end of the pixel's chain plus three
    // standard deviations (a short tail is finished by a patch round)
    const float total = (float)(P.spp * P.chunks);
    const uint32_t stopOff = (uint32_t)(total * m + 3.0f * sqrtf(total * fmaxf(var, 0.05f)) + 2.0f);
    // A pixel whose samples rarely take an odd number of pairs (< 6 %; ground under open sky: 2, or
    // 2 and 4) keeps its true sample starts on one parity for long stretches; a rare odd sample
    // flips it.  Its guesses sit on even offsets, and a second item starts one pair later, so the
    // parse that joins exists whatever the parity of the true one.  Other near-integer means q >= 3
    // use their own lattice (single item).
    const bool parityStable = podd >= 0.0f ? podd < 0.06f : fabsf(m - 2.0f) < 0.25f;
    const float q = parityStable ? 2.0f : rintf(m);
    const bool lattice = parityStable || (q >= 3.0f && fabsf(m - q) < 0.02f);
    const bool dual = parityStable && m > 1.5f;
    const uint32_t J = 2 * P.ssgG - 1;
    uint32_t off = 0;
    for (uint32_t g = 1; g < P.ssgG; ++g) {
        uint32_t o = lattice ? (uint32_t)q * (uint32_t)((float)(g * n) * (m / q) + 0.5f)
                             : (uint32_t)((float)(g * n) * m + 0.5f);
        if (o <= off) o = off + 1;
        xorwow_skip(st, 2u * (o - off));
        off = o;
        uint32_t* w = start + ((size_t)tile * J + 2 * g - 1) * kStartWords * 64 + lane;
        w[0] = o;
        w[64] = st.d;
        w[128] = st.v0;
        w[192] = st.v1;
        w[256] = st.v2;
        w[320] = st.v3;
        w[384] = st.v4;
        w[448] = g + 1 == P.ssgG ? stopOff : 0xffffffffu;
        uint32_t* w2 = w + kStartWords * 64;       // the item one pair later
        if (dual) {
            Xorwow s2 = st;
            xorwow_skip(s2, 2u);
            w2[0] = o + 1;
            w2[64] = s2.d;
            w2[128] = s2.v0;
            w2[192] = s2.v1;
            w2[256] = s2.v2;
            w2[320] = s2.v3;
            w2[384] = s2.v4;
            w2[448] = g + 1 == P.ssgG ? stopOff : 0xffffffffu;
        } else {
            w2[0] = 0xffffffffu;
        }
    }
}

// Walk each pixel's true parse through the logs.  Round 0 starts at group 0 (the pixel's own state);
// a later round starts in the patch log of the carrier that ran from the previous round's dead end.
// At every sample start the walk checks whether a later group's parse has a sample start there (its
// window bits) and, if that group logged samples from there, continues in its log.  Colours are summed
// per render() call and folded into the accumulation value exactly as trace.cu:186-198 does.  Where
// the logs end first (a dead end), the state is kept for the next round: the exact XORWOW state there
// (the item's start state advanced by the draws since), the partial sums, the next candidate group.
__global__ void __launch_bounds__(256) ssg_fold_kernel(TraceParams P, uint32_t round, const float* __restrict__ patchLog,
                                                       const uint16_t* __restrict__ patchEnd,
                                                       const uint32_t* __restrict__ patchCount, uint32_t patchCap,
                                                       float* __restrict__ pairs, uint32_t* __restrict__ deadCount)
{
    uint32_t tile, lane;
    size_t li;
    if (!ssg_pixel(P, (size_t)blockIdx.x * 256 + threadIdx.x, tile, lane, li)) return;
    const size_t npix = (size_t)P.rows * P.width;
    uint32_t* F = P.fold;
    const uint32_t G = P.ssgG, item0 = tile * (2 * G - 1), total = P.spp * P.chunks;
    f3 acc, color;
    uint32_t sIdx, c, done, off, h, odd = 0, prevRel = 0, sq = 0;
    bool inPatch;
    uint32_t cur, k, base, cnt;
    if (round == 0) {
        acc = splat(0.0f);
        if (!P.ignoreFirst) {
            const float4 a = P.accum[li];
            acc = mk(a.x, a.y, a.z);
        }
        color = splat(0.0f);
        sIdx = c = done = off = 0;
        h = 1;
        inPatch = false;
        cur = 0;
        k = 0;
        base = 0;
        cnt = P.ssgCount[(size_t)item0 * 64 + lane];
    } else {
        if (!(F[F_FLAG * npix + li] & 1u)) return;
        acc = mk(__uint_as_float(F[(F_ACC + 0) * npix + li]), __uint_as_float(F[(F_ACC + 1) * npix + li]),
                 __uint_as_float(F[(F_ACC + 2) * npix + li]));
        color = mk(__uint_as_float(F[(F_COL + 0) * npix + li]), __uint_as_float(F[(F_COL + 1) * npix + li]),
                   __uint_as_float(F[(F_COL + 2) * npix + li]));
        const uint32_t sc = F[F_SC * npix + li];
        sIdx = sc & 0xffffu;
        c = sc >> 16;
        done = F[F_DONE * npix + li];
        off = F[F_OFF * npix + li];
        h = min(F[F_H * npix + li], G);
        odd = F[F_ODD * npix + li];
        sq = F[F_SQ * npix + li];
        inPatch = true;
        cur = G;
        k = 0;
        base = off;
        cnt = patchCount[(size_t)tile * 64 + lane];
    }
    uint32_t hStart = h < G ? ssg_start_word(P, item0 + 2 * h - 1, 0, lane) : 0xffffffffu;
    while (done < total) {
        while (h < G && off > hStart + (P.ssgWin * 64u)) {
            ++h;
            hStart = h < G ? ssg_start_word(P, item0 + 2 * h - 1, 0, lane) : 0xffffffffu;
        }
        while (h + 1 < G) {                                  // the latest group started (ssg_finish)
            const uint32_t nx = ssg_start_word(P, item0 + 2 * h + 1, 0, lane);
            if (off < nx) break;
            ++h;
            hStart = nx;
        }
        if (h < G && off >= hStart) {
            bool joined = false;
            for (uint32_t ph = 0; ph < 2 && !joined; ++ph) {        // both phases of group h
                const uint32_t it = item0 + 2 * h - 1 + ph;
                if (off < hStart + ph) continue;
                const uint32_t w = off - hStart - ph;
                if (w >= (P.ssgWin * 64u)) continue;
                const unsigned long long* bits = P.ssgBits + (size_t)it * P.ssgWin * 64 + lane;
                if (!((bits[(w / 64) * 64] >> (w % 64)) & 1ull)) continue;
                uint32_t kh = __popcll(bits[(w / 64) * 64] & ((1ull << (w % 64)) - 1ull));
                for (uint32_t j = 0; j < w / 64; ++j) kh += __popcll(bits[j * 64]);
                const uint32_t ch = P.ssgCount[(size_t)it * 64 + lane];
                if (kh < ch) {                                // continue in this item's log
                    inPatch = false;
                    cur = 2 * h - 1 + ph;
                    k = kh;
                    base = hStart + ph;
                    cnt = ch;
                    joined = true;
                    prevRel = kh ? P.ssgEnd[((size_t)it * P.ssgCap + kh - 1) * 64 + lane] : 0u;
                }
            }
            if (joined) {
                ++h;
                hStart = h < G ? ssg_start_word(P, item0 + 2 * h - 1, 0, lane) : 0xffffffffu;
                continue;
            }
        }
        if (k >= cnt && !inPatch && cur >= 2 && !(cur & 1u)) {
            // a second-phase item ends where it joined its first phase: continue in that one's log
            const uint32_t it = item0 + cur - 1;
            const uint32_t w = off - (base - 1);
            const unsigned long long* bits = P.ssgBits + (size_t)it * P.ssgWin * 64 + lane;
            if (w < (P.ssgWin * 64u) && ((bits[(w / 64) * 64] >> (w % 64)) & 1ull)) {
                uint32_t kh = __popcll(bits[(w / 64) * 64] & ((1ull << (w % 64)) - 1ull));
                for (uint32_t q = 0; q < w / 64; ++q) kh += __popcll(bits[q * 64]);
                const uint32_t ch = P.ssgCount[(size_t)it * 64 + lane];
                if (kh < ch) {
                    cur -= 1;
                    k = kh;
                    base -= 1;
                    cnt = ch;
                    prevRel = kh ? P.ssgEnd[((size_t)it * P.ssgCap + kh - 1) * 64 + lane] : 0u;
                    continue;
                }
            }
        }
        if (k >= cnt) break;
        // up to 16 samples at once (their loads issued together, the sums in order); the batch ends
        // at the first sample start inside it that may be a junction or that passes group h's window,
        // which the top of the loop then handles
        uint32_t m = min(min(cnt - k, total - done), kFoldBatch);
        const float* lg = inPatch ? patchLog : P.ssgLog;
        const uint16_t* le = inPatch ? patchEnd : P.ssgEnd;
        const size_t rec = inPatch ? (size_t)tile * patchCap + k : (size_t)(item0 + cur) * P.ssgCap + k;
        float cx[kFoldBatch], cy[kFoldBatch], cz[kFoldBatch];
        uint32_t er[kFoldBatch];
#pragma unroll
        for (uint32_t j = 0; j < kFoldBatch; ++j) {
            if (j < m) {
                cx[j] = lg[((rec + j) * 3 + 0) * 64 + lane];
                cy[j] = lg[((rec + j) * 3 + 1) * 64 + lane];
                cz[j] = lg[((rec + j) * 3 + 2) * 64 + lane];
                er[j] = le[(rec + j) * 64 + lane];
            }
        }
        if (h < G && m > 1 && base + er[m - 2] >= hStart) {
            // bit words of both phases around the batch's first start at or past hStart
            const uint32_t p0 = max(base + er[0], hStart) - hStart;
            const uint32_t i0 = min(p0 / 64, P.ssgWin - 1);
            const unsigned long long* bA = P.ssgBits + (size_t)(item0 + 2 * h - 1) * P.ssgWin * 64 + lane;
            const unsigned long long* bB = bA + (size_t)P.ssgWin * 64;
            const unsigned long long a0 = bA[i0 * 64], a1 = i0 + 1 < P.ssgWin ? bA[(i0 + 1) * 64] : 0ull;
            const uint32_t iB = p0 ? min((p0 - 1) / 64, P.ssgWin - 1) : 0u;
            const unsigned long long c0 = bB[iB * 64], c1 = iB + 1 < P.ssgWin ? bB[(iB + 1) * 64] : 0ull;
            auto bit = [&](unsigned long long w0, unsigned long long w1, uint32_t i, const unsigned long long* b,
                           uint32_t w) -> bool {
                const uint32_t idx = w / 64;
                const unsigned long long word = idx == i ? w0 : (idx == i + 1 ? w1 : (idx < P.ssgWin ? b[idx * 64] : 0ull));
                return (word >> (w % 64)) & 1ull;
            };
            const uint32_t hNext = h + 1 < G ? ssg_start_word(P, item0 + 2 * h + 1, 0, lane) : 0xffffffffu;
            for (uint32_t j = 0; j + 1 < m; ++j) {
                const uint32_t pos = base + er[j];
                if (pos < hStart) continue;
                const uint32_t w = pos - hStart;
                if (w > (P.ssgWin * 64u) || pos >= hNext || (w < (P.ssgWin * 64u) && bit(a0, a1, i0, bA, w)) ||
                    (w >= 1 && bit(c0, c1, iB, bB, w - 1))) {
                    m = j + 1;
                    break;
                }
            }
        }
        uint32_t endRel = prevRel;
#pragma unroll
        for (uint32_t j = 0; j < kFoldBatch; ++j) {
            if (j < m) {
                odd += (er[j] - endRel) & 1u;               // odd-length sample (guess statistics)
                sq += (er[j] - endRel) * (er[j] - endRel);
                endRel = er[j];
            }
        }
        prevRel = endRel;
#pragma unroll
        for (uint32_t j = 0; j < kFoldBatch; ++j) {
            if (j < m) {
                color = add(color, mk(cx[j], cy[j], cz[j]));
                if (++sIdx == P.spp) {                                  // trace.cu:196
                    acc = (c == 0 && P.ignoreFirst) ? color : add(color, acc);
                    color = splat(0.0f);
                    sIdx = 0;
                    ++c;
                }
            }
        }
        off = base + endRel;
        k += m;
        done += m;
    }
    // the exact state at `off`: the current item's start state advanced by the draws since
    Xorwow st;
    if (inPatch) {
        st = {F[(F_ST + 0) * npix + li], F[(F_ST + 1) * npix + li], F[(F_ST + 2) * npix + li],
              F[(F_ST + 3) * npix + li], F[(F_ST + 4) * npix + li], F[(F_ST + 5) * npix + li]};
    } else if (cur == 0) {
        st = {P.rng[li], P.rng[npix + li], P.rng[2 * npix + li], P.rng[3 * npix + li], P.rng[4 * npix + li],
              P.rng[5 * npix + li]};
    } else {
        const uint32_t it = item0 + cur;
        st = {ssg_start_word(P, it, 1, lane), ssg_start_word(P, it, 2, lane), ssg_start_word(P, it, 3, lane),
              ssg_start_word(P, it, 4, lane), ssg_start_word(P, it, 5, lane), ssg_start_word(P, it, 6, lane)};
    }
    xorwow_skip(st, 2u * (off - base));
    P.rng[li] = st.d;
    P.rng[npix + li] = st.v0;
    P.rng[2 * npix + li] = st.v1;
    P.rng[3 * npix + li] = st.v2;
    P.rng[4 * npix + li] = st.v3;
    P.rng[5 * npix + li] = st.v4;
    P.accum[li] = make_float4(acc.x, acc.y, acc.z, 1.0f);
    if (done == total) {
        if (done > 0) {
            pairs[li] = (float)off / (float)done;
            pairs[npix + li] = (float)odd / (float)done;
            const float mean = (float)off / (float)done;
            pairs[2 * npix + li] = fmaxf((float)sq / (float)done - mean * mean, 0.0f);
        }
        F[F_FLAG * npix + li] = round << 8;      // finished (bit 0 clear), in this fold round (diagnostics)
        return;
    }
    if (done > 0) pairs[li] = (float)off / (float)done;   // the next launch's guess for this pixel
    F[(F_ACC + 0) * npix + li] = __float_as_uint(acc.x);
    F[(F_ACC + 1) * npix + li] = __float_as_uint(acc.y);
    F[(F_ACC + 2) * npix + li] = __float_as_uint(acc.z);
    F[(F_COL + 0) * npix + li] = __float_as_uint(color.x);
    F[(F_COL + 1) * npix + li] = __float_as_uint(color.y);
    F[(F_COL + 2) * npix + li] = __float_as_uint(color.z);
    F[F_SC * npix + li] = sIdx | (c << 16);
    F[F_DONE * npix + li] = done;
    F[F_OFF * npix + li] = off;
    F[F_H * npix + li] = h;
    F[F_ODD * npix + li] = odd;
    F[F_SQ * npix + li] = sq;
    F[(F_ST + 0) * npix + li] = st.d;
    F[(F_ST + 1) * npix + li] = st.v0;
    F[(F_ST + 2) * npix + li] = st.v1;
    F[(F_ST + 3) * npix + li] = st.v2;
    F[(F_ST + 4) * npix + li] = st.v3;
    F[(F_ST + 5) * npix + li] = st.v4;
    F[F_FLAG * npix + li] = 1u;
    atomicAdd(deadCount, 1u);
}

// Multi-device gather, second half: scatter one device's received rows (its bands, in local row
// order) into the full image.  A band is band-rows consecutive image rows in both buffers, so every
// lane copies one float4 of a coalesced row.
__global__ void __launch_bounds__(256) unpermute_rows_kernel(float4* __restrict__ full, const float4* __restrict__ part,
                                                             uint32_t width, uint32_t rows, uint32_t offset,
                                                             uint32_t stride, uint32_t shift)
{
    const size_t li = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (li >= (size_t)rows * width) return;
    const uint32_t ly = (uint32_t)(li / width);
    const uint32_t x = (uint32_t)(li - (size_t)ly * width);
    full[(size_t)global_row(ly, offset, stride, shift) * width + x] = part[li];
}

} // namespace

// =============================================================================================
// C ABI
// =============================================================================================
struct pt_context {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    uint32_t width = 0, height = 0, rowOffset = 0, rowStride = 1, rows = 0, bandShift = 0;
    float4* accum = nullptr;
    uint32_t* rng = nullptr;
    float4* nodes = nullptr;
    float4* prims = nullptr;
    float4* mats = nullptr;
    float4* cnodes = nullptr;   // child-box records (traverse_cb); null when the scene exceeds its encoding
    uint32_t cnodeCount = 0, rootWord = 0;
    bool dfsOrder = true;             // leaves hold their primitives in DFS order (repair_pending)
    bool riseRepair = true;           // pt_set_rise_repair (tests' negative control only)
    // run-ahead across render() calls (MODE 4): the stash and the key it was made under
    uint32_t* ahead = nullptr;        // [kAheadWords][pixels]
    bool aheadValid = false;          // the last launch made a stash
    pt_camera aheadCam = {};
    uint64_t aheadState = 0;          // stateEpoch when it was made
    uint32_t aheadMisses = 0;         // consecutive launches that could not use the previous stash
    int aheadMode = 0;                // pt_set_run_ahead: 0 automatic, 1 off, 2 always make a stash, 3 make but never use
    uint32_t prepassSpp = 0;          // pt_set_cold_start: 0 = first call split off (pre-pass of kPrepassSpp for
                                      // one-call launches), > 0 = a discarded pre-pass of that many spp
    bool coldPriority = true;         // pt_set_cold_start: issue priority on the cold start's order
    uint64_t stateEpoch = 0;          // bumped by every change of scene, textures, sky or RNG state
    uint64_t lastState = 0;           // stateEpoch at the last launch
    bool launched = false;
    float rootBox[6] = {};
    uint32_t nodeCount = 0, primCount = 0, stackDepth = 1;
    bool slabFast = true;
    int variant = 0;
    DevTex* texTable = nullptr;
    DevTex hostTex[PT_MAX_TEXTURES] = {};
    uint32_t skybox = 0;
    unsigned long long* stats = nullptr;
    // tile scheduling: per-tile cost of the last launch and the cost-sorted dispatch order
    uint32_t* tileCost = nullptr;
    uint32_t* tileIdle = nullptr;     // instrumented launches: per-tile mean lane idle cycles (pt_read_tile_idle)
    uint32_t* order = nullptr;
    uint32_t* rowMajor = nullptr;     // the row-major order (packed coordinates), before costs are known
    uint32_t* tileCursor = nullptr;   // persistent variants
    uint32_t* sortKeys = nullptr; // radix-sort scratch: sorted costs, tile ids, temp storage
    uint32_t* tileIds = nullptr;
    void* sortTemp = nullptr;
    size_t sortTempBytes = 0;
    uchar4* ldr = nullptr;        // tonemap staging buffer (pt_tonemap)
    uint32_t orderTiles = 0;      // tiles the device buffers hold
    bool orderValid = false;      // `order` holds a cost-sorted permutation
    bool orderStale = true;       // rebuild it after the next launch (scene, texture or camera changed)
    uint64_t orderSamples = 0;    // samples per pixel of the launch whose tile costs built `order`
    int schedule = 0;             // 0 = cost-sorted tiles (default), 1 = row-major
    int stripMode = 0;            // strip units: 0 = automatic, 1 = off, K >= 2 = always K tiles per unit
    uint32_t orderStrip = 1;      // tiles per unit of the launch whose costs built `order`
    uint32_t* unitMajor = nullptr;    // row-major order of strip units (packed first tiles), for unitK
    uint32_t unitK = 0, unitTiles = 0;
    uint32_t occupancy = 0;       // tuning knob: workgroups per CU of persistent grids (0 = all that fit)
    int prioMode = 0;             // issue priority: 0 = automatic, 1 = off, 2 = explicit bounds prioBounds
    uint32_t prioBounds[3] = {0, 0, 0};
    // speculative sample groups
    int ssgMode = 0;              // 0 = automatic, 1 = off, G >= 2 = always G groups (tests)
    uint32_t patchRounds = 6;     // patch rounds before the remaining dead ends run plain
    uint32_t ssgLook[2] = {64, 16}; // second-phase lag tolerances in samples (TraceParams::ssgLook)
    float* pairs = nullptr;       // per-pixel draw pairs per sample (start-offset guesses)
    bool pairsValid = false;
    uint32_t* ssgStart = nullptr;
    unsigned long long* ssgBits = nullptr;
    uint32_t* ssgCount = nullptr;
    float* ssgLog = nullptr;
    uint16_t* ssgEnd = nullptr;
    uint32_t* fold = nullptr;     // [kFoldWords][pixels] fold state between rounds
    uint32_t* deadCount = nullptr;
    float* patchLog = nullptr;    // patch-round carriers: [tile][patchCap][3][64]
    uint16_t* patchEnd = nullptr;
    uint32_t* patchCount = nullptr;
    size_t ssgItems = 0, ssgSamples = 0, patchSamples = 0;   // allocated capacities (records)
    size_t ssgBitsWords = 0;
    uint32_t lastGroups = 0;      // groups of the last launch (0 = plain launch)
    int lastVariant = 0;          // trace-kernel variant of the last launch's main pass
    uint32_t groupStats[10] = {}; // G, patch rounds, dead-end pixels after fold rounds 0..7
    pt_camera lastCam = {};
    uint64_t epoch = 0;           // launches that wrote the accumulation (a group's gather cache key)
    std::string err;
};

#define PT_HIP_CHECK(ctx, expr)                                                              \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) {                                                              \
            if (ctx) {                                                                       \
                char b_[512];                                                                \
                snprintf(b_, sizeof(b_), "HIP error = %u (%s) at %s:%d '%s'", (unsigned)e_,  \
                         hipGetErrorString(e_), __FILE__, __LINE__, #expr);                  \
                (ctx)->err = b_;                                                             \
            }                                                                                \
            return PT_ERR_HIP;                                                               \
        }                                                                                    \
    } while (0)

static inline float u2f(uint32_t u)
{
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static inline f3 hf3(const float* v) { f3 r; r.x = v[0]; r.y = v[1]; r.z = v[2]; return r; }

static int fail(pt_context* ctx, int code, const char* msg)
{
    if (ctx) ctx->err = msg;
    return code;
}

// Kernel variants (workgroup size, scene staged in LDS or read through the caches).
template <bool STATS, int SL, int WPB, int WW, int MINW, bool PERSIST = false, int MODE = 0>
static hipError_t launch_one(const TraceParams& P, hipStream_t stream)
{
    const size_t nodeF4 = WW >= 3 ? 4 * (size_t)P.cnodeCount : 2 * (size_t)P.nodeCount;
    const size_t sceneBytes = ((SL >= 1 ? nodeF4 : 0) + (SL >= 2 ? 4 * (size_t)P.primCount : 0)) * sizeof(float4);
    const size_t lds = sceneBytes + (size_t)WPB * P.stackDepth * 64 * (WW >= 3 ? 8 : 4) + (size_t)WPB * 64 * 12;
    // no child-box layout: the node-at-a-time walk -- except for grouped and strip launches, whose
    // item and strip hand-off logic lives only in the resumable walk (pick_variant never sends them here)
    if (WW >= 3 && P.cnodes == nullptr) {
        if constexpr (MODE == 1 || MODE >= 3) return hipErrorInvalidValue;
        else return launch_one<STATS, SL, WPB, 1, MINW, PERSIST, MODE>(P, stream);
    }
    if (lds > 160 * 1024) {
        // scene too large to stage in LDS: the same variant reading the scene through the caches
        if (SL > 0) return launch_one<STATS, 0, WPB, WW, MINW, PERSIST, MODE>(P, stream);
        return hipErrorInvalidValue;                   // the stacks alone exceed the LDS
    }
    // the dynamic-LDS limit is raised once per device (contexts on several devices may run on
    // several host threads, as the CLI's -gpus mode does)
    static std::atomic<uint64_t> attrSet{0};
    int dev = 0;
    (void)hipGetDevice(&dev);
    const uint64_t bit = 1ull << (dev & 63);
    if (!(attrSet.load() & bit)) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&trace_kernel<STATS, SL, WPB, WW, MINW, PERSIST, MODE>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attrSet.fetch_or(bit);
    }
    unsigned blocks = (P.numSlots + WPB - 1) / WPB;    // numSlots = tiles, or tiles x groups (SSG)
    if (PERSIST) {
        // resident workgroups per device, cached per instantiation; a grid that fits in one
        // pass gains nothing from the cursor and runs the plain kernel
        static std::atomic<int> resident[64];
        int cap = resident[dev & 63].load();
        if (cap == 0) {
            int cus = 0, perCu = 0;
            hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            if (e == hipSuccess)
                e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                    &perCu, reinterpret_cast<const void*>(&trace_kernel<STATS, SL, WPB, WW, MINW, PERSIST, MODE>), WPB * 64, lds);
            if (e != hipSuccess) return e;
            cap = std::max(cus, 1) * std::max(perCu, 1);
            resident[dev & 63].store(cap);
        }
        if (P.occCap) {                                // tuning knob (pt_set_occupancy): fewer waves per SIMD
            int cus = 0;
            if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0)
                cap = cus * std::min(cap / cus, (int)P.occCap);
            trace_kernel<STATS, SL, WPB, WW, MINW, PERSIST, MODE><<<(unsigned)cap, WPB * 64, lds, stream>>>(P);
            return hipGetLastError();
        }
        if (blocks <= (unsigned)cap) return launch_one<STATS, SL, WPB, WW, MINW, false, MODE>(P, stream);
        blocks = (unsigned)cap;
    }
    trace_kernel<STATS, SL, WPB, WW, MINW, PERSIST, MODE><<<blocks, WPB * 64, lds, stream>>>(P);
    return hipGetLastError();
}

// Shipped variants (all bit-identical).  Measured-and-rejected variants of earlier rounds (single
// loop with LDS nodes, other exit thresholds, 2/8/16-wave groups, 6-8 waves/SIMD, speculative
// traversal, select-form primitive tests, a ballot-driven phase scheduler) are recorded in DESIGN.md
// and git history, not shipped.
//   1   reference control flow (one loop, node at a time), scene read through the caches
//   4   node-at-a-time while-while, caches, 5 waves/SIMD   (scenes outside the child-box encoding)
//   6   node-at-a-time while-while, nodes in LDS           (idem, small BVH)
//   20  child-box traversal, one tile per wave             (counts the reference's node/prim tests)
// The WW parameter of the resumable walk encodes 100000 * NOREPAIR + 10000 * SKYQ + 1000 * DEFERQ + 200 + EXITQ
// (deferred shading and the traversal's exit threshold, see trace_kernel).
//   39  variant 40 without deferred shading, exit <= 24/64 (the round-1 default; A/B reference)
//   40  default: resumable lean child-box walk, records in LDS, persistent waves, deferred shading
//       (hits >= 4/8, misses >= 1/8 with a sky texture), exit <= 12/64
//   41  default for cache-read scenes: same, records through the caches
//   46  default for deep cache-read BVHs: variant 41 compiled for 4 waves/SIMD (128 VGPRs)
//   47  small grids (<= 4 tiles per SIMD): variant 39 compiled for 4 waves/SIMD (128 VGPRs); no
//       deferral, which costs a single pass of latency-bound waves 2.8 %
//   48  small grids whose primitives fit in LDS too: records and primitives in LDS, 4 waves/SIMD,
//       deferred hits
// Variants 50/51 (leaf tests compacted across a round's lanes by shape family, -14.6 % on C3) were
// measured in round 3 and removed in round 4; commit 1b0d322 has them.
constexpr int kV40Walk = 14212;     // variant 40's walk parameters (SKYQ 1, DEFERQ 4, exit <= 12/64;
                                    // retuned in round 3, profiles/r03_walk_params_ab.json)
template <bool STATS, int MODE = 0>
static hipError_t launch_variant(int v, const TraceParams& P, hipStream_t stream)
{
    switch (v) {
    case 1: return launch_one<STATS, 0, 4, 0, 1, false, MODE>(P, stream);
    case 4: return launch_one<STATS, 0, 4, 1, 5, false, MODE>(P, stream);
    case 6: return launch_one<STATS, 1, 4, 1, 5, false, MODE>(P, stream);
    case 20: return launch_one<STATS, 0, 4, 3, 5, false, MODE>(P, stream);
    case 39: return launch_one<STATS, 1, 4, 224, 5, true, MODE>(P, stream);
    case 40: return launch_one<STATS, 1, 4, kV40Walk, 5, true, MODE>(P, stream);
    case 41: return launch_one<STATS, 0, 4, 14212, 5, true, MODE>(P, stream);
    case 46: return launch_one<STATS, 0, 4, 14212, 4, true, MODE>(P, stream);
    case 47: return launch_one<STATS, 1, 4, 224, 4, true, MODE>(P, stream);
    case 48: return launch_one<STATS, 2, 4, 13216, 4, true, MODE>(P, stream);
    case 60:
        if constexpr (STATS) return launch_one<STATS, 1, 4, kV40Walk, 5, true, MODE>(P, stream);
        else return launch_one<false, 1, 8, kV40Walk, 6, true, MODE>(P, stream);
    case 61:
        if constexpr (STATS) return launch_one<STATS, 0, 4, 14212, 5, true, MODE>(P, stream);
        else return launch_one<false, 0, 4, 14212, 6, true, MODE>(P, stream);
    case 90: return launch_one<false, 1, 4, 100000 + kV40Walk, 5, true, 0>(P, stream);   // test only: 40, no repair
    case 91: return launch_one<false, 2, 4, 113216, 4, true, 0>(P, stream);              // A/B only: 48, no repair
    default: return hipErrorInvalidValue;
    }
}

// Speculative-group launches (MODE 1) and their resume / pre-pass launches (MODE 2) exist for the
// default variants only.
template <int MODE>
static hipError_t launch_grouped(int v, const TraceParams& P, hipStream_t stream)
{
    switch (v) {
    case 39: return launch_one<false, 1, 4, 224, 5, true, MODE>(P, stream);
    case 40: return launch_one<false, 1, 4, kV40Walk, 5, true, MODE>(P, stream);
    case 41: return launch_one<false, 0, 4, 14212, 5, true, MODE>(P, stream);
    case 46: return launch_one<false, 0, 4, 14212, 4, true, MODE>(P, stream);
    case 60: return launch_one<false, 1, 8, kV40Walk, 6, true, MODE>(P, stream);
    case 61: return launch_one<false, 0, 4, 14212, 6, true, MODE>(P, stream);
    default: return hipErrorInvalidValue;
    }
}

// Strip-unit launches (MODE 3) of the resumable persistent variants.
static hipError_t launch_strip(int v, const TraceParams& P, hipStream_t stream)
{
    switch (v) {
    case 40: return launch_one<false, 1, 4, kV40Walk, 5, true, 3>(P, stream);
    case 41: return launch_one<false, 0, 4, 14212, 5, true, 3>(P, stream);
    case 46: return launch_one<false, 0, 4, 14212, 4, true, 3>(P, stream);
    case 60: return launch_one<false, 1, 8, kV40Walk, 6, true, 3>(P, stream);
    case 61: return launch_one<false, 0, 4, 14212, 6, true, 3>(P, stream);
    default: return hipErrorInvalidValue;
    }
}

static bool strip_capable(int v) { return v == 40 || v == 41 || v == 46 || v == 60 || v == 61; }

// Waves per SIMD a persistent variant is compiled for (its wave slots: CUs x 4 SIMDs x this).
static uint32_t variant_waves(int v) { return v == 60 || v == 61 ? 6u : (v == 46 || v == 47 || v == 48 || v == 91) ? 4u : 5u; }

// Run-ahead launches (MODE 4) of the resumable persistent variants.
static hipError_t launch_ahead(int v, const TraceParams& P, hipStream_t stream)
{
    switch (v) {
    case 40: return launch_one<false, 1, 4, kV40Walk, 5, true, 4>(P, stream);
    case 41: return launch_one<false, 0, 4, 14212, 5, true, 4>(P, stream);
    case 46: return launch_one<false, 0, 4, 14212, 4, true, 4>(P, stream);
    case 60: return launch_one<false, 1, 8, kV40Walk, 6, true, 4>(P, stream);
    case 61: return launch_one<false, 0, 4, 14212, 6, true, 4>(P, stream);
    default: return hipErrorInvalidValue;
    }
}

// Tiles per dispatch unit.  A launch of few samples per pixel idles the lanes whose pixels finish
// first for the rest of their tile; strips of K tiles let those lanes go on with the next tile.
// Measured at 1080p (tools/call_loop.py, profiles/r04_call_loop.json): 1-spp progressive frames
// 0.673 -> 0.646 ms (K = 2) -> 0.592 ms (K = 4); the reference's 8-spp calls 316 -> 320 ms (K = 2)
// -> 466 ms (K = 4) per 128 calls -- units of several tiles are too few to balance the launch's tail
// there.  Automatic: K = 4 for launches of at most 2 samples per pixel with at least ~6 tiles per
// wave slot; the variant must be a strip-capable one.
constexpr uint64_t kStripMaxSamples = 2;

// `variant` is the one that runs (pick_variant's result, which already replaces a forced child-box
// variant by a node-at-a-time one on scenes without the child-box layout or DFS leaf order).
static uint32_t strip_tiles(const pt_context* ctx, int variant, uint32_t tiles, uint64_t samples)
{
    if (ctx->stripMode == 1 || !strip_capable(variant) || !ctx->cnodes) return 1;
    if (ctx->stripMode >= 2) return (uint32_t)ctx->stripMode;
    if (samples > kStripMaxSamples) return 1;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess) return 1;
    const uint64_t slots = (uint64_t)cus * 4 * 5;       // (the threshold was measured at five waves)
    return (uint64_t)tiles >= 6 * slots ? 4u : 1u;
}

static bool variant_shipped(int v)
{
    return v == 0 || v == 1 || v == 4 || v == 6 || v == 20 || v == 40 || v == 41 || v == 46 || v == 47 || v == 48 || v == 39 ||
           v == 60 || v == 61 || v == 91;   // 91: variant 48 without the rising-t_max rebuild (A/B of its cost only; not the reference's bits)
}

// Run-ahead (MODE 4): launches of kAheadMinSamples..kAheadMaxSamples samples per pixel make a stash
// of the next call's first samples (the reference's render(cam, 8, ...) calls, main.cpp:272-279);
// 1-2 spp progressive frames use strip units instead.
constexpr uint64_t kAheadMinSamples = 3, kAheadMaxSamples = 64;
// Cost pre-pass of a cold-start launch (render_impl): samples per pixel, and the smallest launch
// (spp x chunks) that gets one.
constexpr uint32_t kPrepassSpp = 2;
constexpr uint64_t kPrepassMinSpp = 16;

static int pick_variant(const pt_context* ctx)
{
    const size_t nodeBytes = 2 * (size_t)ctx->nodeCount * sizeof(float4);
    if (ctx->variant > 0) {
        // a child-box walk needs the child-box layout (leaf counts < 256) and leaves in DFS primitive
        // order (repair_pending, ChildPair); without them the node-at-a-time walk runs, so grouped and
        // strip launches (which exist only for the child-box walks) are never chosen for such scenes
        const bool childBox = ctx->variant != 1 && ctx->variant != 4 && ctx->variant != 6;
        return (childBox && (!ctx->dfsOrder || !ctx->cnodes)) ? (nodeBytes <= 48 * 1024 ? 6 : 4) : ctx->variant;
    }
    // measured on MI355X (tools/ab_variants.py, profiles/): child-box traversal (one dependent
    // fetch per interior visit, leaves inline) with while-while leaf batching and 5 waves/SIMD
    // wins on every scene; the child-box records are staged in LDS when they fit in 48 KB
    // (cornell, the 484-object scene) and read through the caches otherwise (100k objects).
    // Scenes outside the child-box encoding fall back to the node-at-a-time walk (launch_one).
    // The resumable form wins everywhere (the wave shades its finished lanes once at most 12/64
    // still walk), and so do persistent waves pulling tiles from a cursor (variants 30/34: +6% on
    // the 484-object scene, +11% on 100k objects over the one-tile-per-wave grid, variants 28/26).
    // A cache-read scene whose four LDS stacks per workgroup leave room for fewer than five
    // workgroups per CU (BVH depth > 16) runs at 4 waves/SIMD anyway: variant 46 is variant 41
    // compiled for that occupancy (128 VGPRs, no spill), +1% on the 100k-object scene (depth 19).
    // Six waves per SIMD (variants 60 / 61: the same walks compiled for 80 VGPRs) when the LDS holds
    // them: with the records in LDS as three 8-wave workgroups per CU (the records staged once per
    // eight waves), with cache-read records as six 4-wave workgroups.  Measured on C3
    // (profiles/r05_six_waves.json): 60 224.2 ms against 40 231.2; 61 237.5 against 41 245.7.
    const size_t cbBytes = 4 * (size_t)ctx->cnodeCount * sizeof(float4);
    const size_t waveBytes = (size_t)ctx->stackDepth * 64 * 8 + 64 * 12;   // a wave's stack + accumulation slice
    const size_t ldsCap = 160 * 1024;
    // (a BVH whose leaves are not in DFS primitive order cannot be descended by repair_pending: the
    // node-at-a-time walks, which push every far child as the reference does)
    if (!ctx->cnodes || !ctx->dfsOrder) return nodeBytes <= 48 * 1024 ? 6 : 4;
    if (cbBytes <= 48 * 1024 && 3 * (cbBytes + 8 * waveBytes) <= ldsCap) return 60;
    if (cbBytes <= 48 * 1024 && 5 * (cbBytes + 4 * waveBytes) <= ldsCap) return 40;
    if (6 * 4 * waveBytes <= ldsCap) return 61;
    return cbBytes <= 48 * 1024 ? 40 : (5 * 4 * waveBytes > ldsCap ? 46 : 41);
}

extern "C" {

PT_API int pt_device_count(int* count)
{
    if (!count) return PT_ERR_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return PT_OK;
}

PT_API uint32_t pt_band_rows(uint32_t height, uint32_t band_rows, uint32_t band_offset, uint32_t band_stride)
{
    if (band_rows == 0 || band_stride == 0 || (band_rows & (band_rows - 1)) != 0) return 0;
    const uint32_t nb = (height + band_rows - 1) / band_rows;
    if (band_offset >= nb) return 0;
    const uint32_t own = (nb - band_offset + band_stride - 1) / band_stride;
    const uint32_t last = band_offset + (own - 1) * band_stride;
    return (own - 1) * band_rows + std::min(band_rows, height - last * band_rows);
}

PT_API int pt_unpermute_bands(int device, void* full, const void* part, uint32_t width, uint32_t height, uint32_t band_rows,
                              uint32_t band_offset, uint32_t band_stride)
{
    if (!full || !part || width == 0 || band_stride == 0 || band_rows == 0 || band_rows > 256 ||
        (band_rows & (band_rows - 1)) != 0)
        return PT_ERR_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return PT_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return PT_ERR_ARG;
    const uint32_t rows = pt_band_rows(height, band_rows, band_offset, band_stride);
    const size_t npix = (size_t)rows * width;
    if (npix == 0) return PT_OK;
    if (hipSetDevice(device) != hipSuccess) return PT_ERR_HIP;
    // the caller's buffers may be in use on any stream of the device: synchronise around the copy
    if (hipDeviceSynchronize() != hipSuccess) return PT_ERR_HIP;
    unpermute_rows_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, 0>>>(
        static_cast<float4*>(full), static_cast<const float4*>(part), width, rows, band_offset, band_stride,
        (uint32_t)__builtin_ctz(band_rows));
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return PT_ERR_HIP;
    return PT_OK;
}

PT_API int pt_create(int device, uint32_t width, uint32_t height, uint32_t row_offset, uint32_t row_stride,
                     pt_context** out)
{
    return pt_create_banded(device, width, height, 1, row_offset, row_stride, out);
}

PT_API int pt_create_banded(int device, uint32_t width, uint32_t height, uint32_t band_rows, uint32_t band_offset,
                            uint32_t band_stride, pt_context** out)
{
    if (!out || width == 0 || height == 0 || band_stride == 0) return PT_ERR_ARG;
    *out = nullptr;
    if (band_rows == 0 || band_rows > 256 || (band_rows & (band_rows - 1)) != 0) return PT_ERR_ARG;
    // tiles are addressed by packed 16-bit coordinates (tileY << 16 | tileX), pixels by 32-bit indices
    {
        const uint64_t r = pt_band_rows(height, band_rows, band_offset, band_stride);
        if (width > 8u * 0xffffu || r > 8u * 0xfffeu || r * width >= (1ull << 30)) return PT_ERR_ARG;
    }
    const uint32_t row_offset = band_offset, row_stride = band_stride;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return PT_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return PT_ERR_ARG;
    pt_context* ctx = new pt_context();
    ctx->device = device;
    ctx->width = width;
    ctx->height = height;
    ctx->rowOffset = row_offset;
    ctx->rowStride = row_stride;
    ctx->bandShift = (uint32_t)__builtin_ctz(band_rows);
    ctx->rows = pt_band_rows(height, band_rows, band_offset, band_stride);
    auto bail = [&](int code) { pt_destroy(ctx); return code; };
    if (hipSetDevice(device) != hipSuccess) return bail(PT_ERR_HIP);
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) return bail(PT_ERR_HIP);
    if (hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) return bail(PT_ERR_HIP);
    const size_t npix = (size_t)ctx->rows * width;
    const size_t nalloc = npix ? npix : 1;
    if (hipMalloc(&ctx->accum, nalloc * sizeof(float4)) != hipSuccess) return bail(PT_ERR_HIP);
    if (hipMalloc(&ctx->rng, nalloc * 6 * sizeof(uint32_t)) != hipSuccess) return bail(PT_ERR_HIP);
    if (hipMalloc(&ctx->texTable, PT_MAX_TEXTURES * sizeof(DevTex)) != hipSuccess) return bail(PT_ERR_HIP);
    if (hipMalloc(&ctx->stats, kStatWords * sizeof(unsigned long long)) != hipSuccess) return bail(PT_ERR_HIP);
    if (hipMemsetAsync(ctx->accum, 0, nalloc * sizeof(float4), ctx->stream) != hipSuccess) return bail(PT_ERR_HIP);
    if (hipMemcpyAsync(ctx->texTable, ctx->hostTex, sizeof(ctx->hostTex), hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
        return bail(PT_ERR_HIP);
    if (npix) {
        const unsigned blocks = (unsigned)((npix + 255) / 256);
        init_rng_kernel<<<blocks, 256, 0, ctx->stream>>>(ctx->rng, width, ctx->rows, row_offset, row_stride,
                                                                ctx->bandShift);
        if (hipGetLastError() != hipSuccess) return bail(PT_ERR_HIP);
    }
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return bail(PT_ERR_HIP);
    *out = ctx;
    return PT_OK;
}

PT_API void pt_destroy(pt_context* ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->accum);
    (void)hipFree(ctx->rng);
    (void)hipFree(ctx->nodes);
    (void)hipFree(ctx->prims);
    (void)hipFree(ctx->mats);
    (void)hipFree(ctx->cnodes);
    (void)hipFree(ctx->tileCost);
    (void)hipFree(ctx->tileIdle);
    (void)hipFree(ctx->order);
    (void)hipFree(ctx->rowMajor);
    (void)hipFree(ctx->unitMajor);
    (void)hipFree(ctx->tileCursor);
    (void)hipFree(ctx->ldr);
    (void)hipFree(ctx->sortKeys);
    (void)hipFree(ctx->tileIds);
    (void)hipFree(ctx->sortTemp);
    (void)hipFree(ctx->texTable);
    (void)hipFree(ctx->stats);
    (void)hipFree(ctx->pairs);
    (void)hipFree(ctx->ssgStart);
    (void)hipFree(ctx->ssgBits);
    (void)hipFree(ctx->ssgCount);
    (void)hipFree(ctx->ssgLog);
    (void)hipFree(ctx->ssgEnd);
    (void)hipFree(ctx->fold);
    (void)hipFree(ctx->deadCount);
    (void)hipFree(ctx->patchLog);
    (void)hipFree(ctx->patchEnd);
    (void)hipFree(ctx->patchCount);
    (void)hipFree(ctx->ahead);
    for (auto& t : ctx->hostTex) (void)hipFree((void*)t.texels);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

// Host-side validation of the BVH so a malformed scene can never make the kernel read out of
// bounds or overflow its 32-entry stack (the reference does not check, trace.cu:39).
static int validate_scene(pt_context* ctx, const pt_bvh_node* nodes, uint32_t nn, const pt_hittable* prims, uint32_t np,
                          uint32_t& maxDepthOut)
{
    for (uint32_t i = 0; i < np; ++i) {
        if (prims[i].type > 6u) return fail(ctx, PT_ERR_ARG, "pt_set_scene: invalid hittable type");
        if (prims[i].texture_index > PT_MAX_TEXTURES) return fail(ctx, PT_ERR_ARG, "pt_set_scene: invalid texture index");
    }
    // iterative DFS computing the depth (number of nodes on the root-to-node path)
    std::vector<std::pair<uint32_t, uint32_t>> st;
    st.push_back({0u, 1u});
    uint32_t maxDepth = 0, visited = 0;
    while (!st.empty()) {
        auto [i, depth] = st.back();
        st.pop_back();
        if (i >= nn) return fail(ctx, PT_ERR_ARG, "pt_set_scene: node index out of range");
        if (++visited > nn) return fail(ctx, PT_ERR_ARG, "pt_set_scene: BVH is not a tree");
        maxDepth = std::max(maxDepth, depth);
        const uint32_t pca = nodes[i].primitive_count_axis;
        const uint32_t count = pca >> 16;
        if (count > 0) {
            if ((uint64_t)nodes[i].offset + count > np) return fail(ctx, PT_ERR_ARG, "pt_set_scene: leaf range out of bounds");
        } else {
            if (((pca >> 8) & 0xffu) > 2u) return fail(ctx, PT_ERR_ARG, "pt_set_scene: invalid split axis");
            if (nodes[i].offset <= i + 1 || nodes[i].offset >= nn || i + 1 >= nn)
                return fail(ctx, PT_ERR_ARG, "pt_set_scene: invalid child index");
            st.push_back({i + 1, depth + 1});
            st.push_back({nodes[i].offset, depth + 1});
        }
    }
    if (maxDepth > 33) return fail(ctx, PT_ERR_DEPTH, "pt_set_scene: BVH depth exceeds the 32-entry traversal stack");
    maxDepthOut = maxDepth;
    return PT_OK;
}

PT_API int pt_set_scene(pt_context* ctx, const pt_bvh_node* nodes, uint32_t node_count, const pt_hittable* prims,
                        uint32_t prim_count)
{
    if (!ctx) return PT_ERR_ARG;
    if (node_count == 0 || prim_count == 0 || !nodes || !prims) return fail(ctx, PT_ERR_ARG, "pt_set_scene: empty scene");
    uint32_t maxDepth = 1;
    int rc = validate_scene(ctx, nodes, node_count, prims, prim_count, maxDepth);
    if (rc != PT_OK) return rc;
    std::vector<float4> hn(2 * (size_t)node_count), hp(4 * (size_t)prim_count), hm(3 * (size_t)prim_count);
    bool slabFast = true;
    for (uint32_t i = 0; i < node_count; ++i) {
        const pt_bvh_node& n = nodes[i];
        hn[2 * i] = make_float4(n.aabb_min[0], n.aabb_max[0], n.aabb_min[1], n.aabb_max[1]);
        hn[2 * i + 1] = make_float4(n.aabb_min[2], n.aabb_max[2], u2f(n.offset), u2f(n.primitive_count_axis));
        for (int k = 0; k < 3; ++k)   // the fast slab test needs ordered, non-NaN bounds
            if (!(n.aabb_min[k] <= n.aabb_max[k])) slabFast = false;
    }
    // child-box records: interior nodes renumbered in order; a child word is (count << 24 | prim
    // offset) for a leaf, the record index otherwise (needs counts < 256 and offsets < 2^24)
    std::vector<uint32_t> rec(node_count, 0xffffffffu);
    uint32_t interior = 0;
    bool cbOk = node_count < (1u << 24) && prim_count < (1u << 24);
    for (uint32_t i = 0; i < node_count; ++i) {
        const uint32_t count = nodes[i].primitive_count_axis >> 16;
        if (count == 0) rec[i] = interior++;
        else if (count > 255) cbOk = false;
    }
    auto word = [&](uint32_t i) {
        const uint32_t count = nodes[i].primitive_count_axis >> 16;
        return count ? (count << 24) | nodes[i].offset : rec[i];
    };
    // first and last primitive under each node (children follow their parent in the array); the
    // rising-t_max rebuild (repair_pending) finds a leaf's path by the first primitive of each
    // second child, which needs every left subtree's primitives below the right subtree's
    std::vector<uint32_t> firstPrim(node_count), lastPrim(node_count);
    bool dfsOrder = true;
    for (uint32_t i = node_count; i-- > 0;) {
        const uint32_t count = nodes[i].primitive_count_axis >> 16;
        if (count) {
            firstPrim[i] = nodes[i].offset;
            lastPrim[i] = nodes[i].offset + count - 1;
        } else {
            const uint32_t a = i + 1, b = nodes[i].offset;
            firstPrim[i] = std::min(firstPrim[a], firstPrim[b]);
            lastPrim[i] = std::max(lastPrim[a], lastPrim[b]);
            if (!(lastPrim[a] < firstPrim[b])) dfsOrder = false;
        }
    }
    std::vector<float4> hc(4 * (size_t)std::max(interior, 1u), make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (uint32_t i = 0; cbOk && i < node_count; ++i) {
        if (rec[i] == 0xffffffffu) continue;
        const pt_bvh_node& L = nodes[i + 1];
        const pt_bvh_node& R = nodes[nodes[i].offset];
        float4* q = &hc[4 * (size_t)rec[i]];
        q[0] = make_float4(L.aabb_min[0], L.aabb_max[0], L.aabb_min[1], L.aabb_max[1]);
        q[1] = make_float4(L.aabb_min[2], L.aabb_max[2], R.aabb_min[2], R.aabb_max[2]);
        q[2] = make_float4(R.aabb_min[0], R.aabb_max[0], R.aabb_min[1], R.aabb_max[1]);
        q[3] = make_float4(u2f(word(i + 1)), u2f(word(nodes[i].offset)), u2f(1u << ((nodes[i].primitive_count_axis >> 8) & 0xffu)),
                           u2f(firstPrim[nodes[i].offset]));
    }
    for (uint32_t i = 0; i < prim_count; ++i) {
        const pt_hittable& h = prims[i];
        const float(&R)[3][4] = h.inv_transform_rows;
        hp[4 * i + 0] = make_float4(R[0][0], R[1][0], R[0][1], R[1][1]);
        hp[4 * i + 1] = make_float4(R[0][2], R[1][2], R[0][3], R[1][3]);
        hp[4 * i + 2] = make_float4(R[2][0], R[2][1], R[2][2], R[2][3]);
        hp[4 * i + 3] = make_float4(u2f(h.type), 0.0f, 0.0f, 0.0f);
        hm[3 * i] = make_float4(h.base_color[0], h.base_color[1], h.base_color[2], h.roughness);
        hm[3 * i + 1] = make_float4(h.emissive[0], h.emissive[1], h.emissive[2], h.metalness);
        hm[3 * i + 2] = make_float4(u2f(h.texture_index), u2f(h.material_type), 0.0f, 0.0f);
    }
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    PT_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    (void)hipFree(ctx->nodes);
    (void)hipFree(ctx->prims);
    (void)hipFree(ctx->mats);
    (void)hipFree(ctx->cnodes);
    ctx->nodes = ctx->prims = ctx->mats = ctx->cnodes = nullptr;
    ctx->nodeCount = ctx->primCount = ctx->cnodeCount = 0;
    PT_HIP_CHECK(ctx, hipMalloc(&ctx->nodes, hn.size() * sizeof(float4)));
    PT_HIP_CHECK(ctx, hipMalloc(&ctx->prims, hp.size() * sizeof(float4)));
    PT_HIP_CHECK(ctx, hipMalloc(&ctx->mats, hm.size() * sizeof(float4)));
    PT_HIP_CHECK(ctx, hipMemcpy(ctx->nodes, hn.data(), hn.size() * sizeof(float4), hipMemcpyHostToDevice));
    PT_HIP_CHECK(ctx, hipMemcpy(ctx->prims, hp.data(), hp.size() * sizeof(float4), hipMemcpyHostToDevice));
    PT_HIP_CHECK(ctx, hipMemcpy(ctx->mats, hm.data(), hm.size() * sizeof(float4), hipMemcpyHostToDevice));
    if (cbOk) {
        PT_HIP_CHECK(ctx, hipMalloc(&ctx->cnodes, hc.size() * sizeof(float4)));
        PT_HIP_CHECK(ctx, hipMemcpy(ctx->cnodes, hc.data(), hc.size() * sizeof(float4), hipMemcpyHostToDevice));
        ctx->cnodeCount = interior;
    }
    ctx->dfsOrder = dfsOrder;
    ctx->orderStale = true;
    ++ctx->stateEpoch;
    ctx->rootWord = word(0);
    for (int k = 0; k < 3; ++k) {
        ctx->rootBox[2 * k] = nodes[0].aabb_min[k];
        ctx->rootBox[2 * k + 1] = nodes[0].aabb_max[k];
    }
    ctx->nodeCount = node_count;
    ctx->primCount = prim_count;
    ctx->slabFast = slabFast;
    // LDS stack rows.  A lane visiting node v holds at most pend(v) pending entries: the ancestors
    // whose near child (trace.cu:69-76, by the sign of the ray direction along their split axis) is
    // on the path to v -- their far child is pushed (and repair_pending rebuilds exactly these).
    // The walks write one entry unconditionally above the top at an interior visit (walk_interior;
    // the node-at-a-time walks push there), so the rows needed are the maximum over the 8 direction
    // octants of pend(v) + 1 over interior v; pend(v) <= depth(v) - 1, the reference's bound.  pend is
    // carried down the same root DFS validate_scene runs (only reachable nodes; an orphan node that
    // names a reachable child cannot overwrite that child's value).
    {
        uint32_t need = 1;
        std::vector<std::pair<uint32_t, uint32_t>> st;
        for (uint32_t o = 0; o < 8; ++o) {
            st.assign(1, {0u, 0u});
            while (!st.empty()) {
                const auto [i, pend] = st.back();
                st.pop_back();
                const uint32_t pca = nodes[i].primitive_count_axis;
                if ((pca >> 16) != 0) continue;
                need = std::max(need, pend + 1u);
                const bool neg = (o >> ((pca >> 8) & 0xffu)) & 1u;
                const uint32_t a = i + 1, b = nodes[i].offset;
                st.push_back({neg ? b : a, pend + 1u});    // near child: its sibling is pending
                st.push_back({neg ? a : b, pend});
            }
        }
        ctx->stackDepth = std::min(need, maxDepth > 1 ? maxDepth - 1 : 1u);
    }
    return PT_OK;
}

PT_API int pt_set_texture(pt_context* ctx, uint32_t handle, const float* rgba, uint32_t width, uint32_t height)
{
    if (!ctx) return PT_ERR_ARG;
    if (handle == 0 || handle > PT_MAX_TEXTURES || !rgba || width == 0 || height == 0)
        return fail(ctx, PT_ERR_ARG, "pt_set_texture: invalid argument");
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    PT_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    DevTex& t = ctx->hostTex[handle - 1];
    (void)hipFree((void*)t.texels);
    t = DevTex{};
    float4* mem = nullptr;
    const size_t bytes = (size_t)width * height * sizeof(float4);
    PT_HIP_CHECK(ctx, hipMalloc(&mem, bytes));
    PT_HIP_CHECK(ctx, hipMemcpy(mem, rgba, bytes, hipMemcpyHostToDevice));
    t.texels = mem;
    t.width = width;
    t.height = height;
    t.fwidth = (float)width;
    t.fheight = (float)height;
    ctx->orderStale = true;
    ++ctx->stateEpoch;
    PT_HIP_CHECK(ctx, hipMemcpy(ctx->texTable, ctx->hostTex, sizeof(ctx->hostTex), hipMemcpyHostToDevice));
    return PT_OK;
}

PT_API int pt_set_skybox(pt_context* ctx, uint32_t handle)
{
    if (!ctx) return PT_ERR_ARG;
    if (handle > PT_MAX_TEXTURES) return fail(ctx, PT_ERR_ARG, "pt_set_skybox: invalid handle");
    if (ctx->skybox != handle) ++ctx->stateEpoch;
    ctx->skybox = handle;
    return PT_OK;
}

// Speculative sample groups: how many groups a launch uses (0 = a plain launch).  A launch of
// `tiles` 8x8 tiles on a chip with `resident` wave slots gets enough groups for about six work items
// per slot (at most 8, each at least 64 samples long), and runs plain when that is fewer than 4
// (1.5 tiles per slot or more: the cost-sorted list schedule balances well enough).
static uint32_t ssg_groups(const pt_context* ctx, int variant, uint32_t tiles, uint32_t total)
{
    if (ctx->ssgMode == 1 || !(variant == 39 || strip_capable(variant))) return 0;
    if (ctx->ssgMode >= 2) return std::min<uint32_t>((uint32_t)ctx->ssgMode, std::max(total, 1u));
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess) return 0;
    const uint64_t resident = (uint64_t)cus * 4 * variant_waves(variant);
    uint64_t g = (6 * resident + tiles - 1) / tiles;
    g = std::min<uint64_t>({g, 8, total / 64});
    // measured (tools/ssg_probe.py): with 2 or 3 groups the logging, the fold and the
    // extra samples cost more than the shorter tail returns; from 4 groups on the tail wins
    return g >= 4 ? (uint32_t)g : 0;
}

// A plain launch with at most four tiles per SIMD runs every tile in one pass at four waves per
// SIMD, so the fifth wave slot the default kernels are compiled for (96 VGPRs, with spills) buys
// nothing: the same walk compiled for four waves (128 VGPRs, no spill) shortens every wave's chain,
// and when the primitives fit in LDS next to the child-box records, four workgroups per CU still
// fit and leaf tests read LDS instead of L1/L2.  Measured (tools/ab_variants.py, MI355X): cornell
// 512x512x64 +5.5 % (48), one rank's share of 1080p x 1024 at N = 8 +4 % (47).
static int small_grid_variant(const pt_context* ctx, int variant, uint32_t tiles)
{
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess) return variant;
    if ((uint64_t)tiles > (uint64_t)cus * 4 * 4) return variant;
    if (variant == 41 || variant == 61) return 46;
    if (variant != 40 && variant != 60) return variant;
    const size_t group = 4 * (size_t)ctx->cnodeCount * sizeof(float4) + 4 * (size_t)ctx->primCount * sizeof(float4) +
                         4 * (size_t)ctx->stackDepth * 64 * 8 + 4 * 64 * 12;
    return 4 * group <= 160 * 1024 ? 48 : 47;
}

// Grow-only device buffers of the speculative groups; false if the device is out of memory (the
// launch then runs plain).
static bool ssg_reserve(pt_context* ctx, size_t tiles, size_t items, size_t samples, size_t patchSamples,
                        size_t bitsWords = 0)
{
    const size_t npix = (size_t)ctx->rows * ctx->width;
    auto fail_ = [] { (void)hipGetLastError(); return false; };
    if (!ctx->pairs) {
        if (hipMalloc(&ctx->pairs, 3 * npix * sizeof(float)) != hipSuccess ||
            hipMalloc(&ctx->fold, kFoldWords * npix * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&ctx->deadCount, sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&ctx->patchCount, tiles * 64 * sizeof(uint32_t)) != hipSuccess)
            return fail_();
        // guess statistics until a pre-pass or fold measures them: 2 pairs per sample, odd-length
        // fraction unknown (< 0), variance 1
        if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ctx->pairs), 0x40000000, npix, ctx->stream) != hipSuccess ||
            hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ctx->pairs + npix), 0xbf800000, npix, ctx->stream) != hipSuccess ||
            hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ctx->pairs + 2 * npix), 0x3f800000, npix, ctx->stream) != hipSuccess)
            return fail_();
    }
    if (items > ctx->ssgItems) {
        (void)hipFree(ctx->ssgStart);
        (void)hipFree(ctx->ssgCount);
        ctx->ssgStart = nullptr;
        ctx->ssgCount = nullptr;
        ctx->ssgItems = 0;
        if (hipMalloc(&ctx->ssgStart, items * kStartWords * 64 * sizeof(uint32_t)) != hipSuccess ||
            hipMalloc(&ctx->ssgCount, items * 64 * sizeof(uint32_t)) != hipSuccess)
            return fail_();
        ctx->ssgItems = items;
    }
    if (bitsWords > ctx->ssgBitsWords) {           // [item][window words][64 lanes]
        (void)hipFree(ctx->ssgBits);
        ctx->ssgBits = nullptr;
        ctx->ssgBitsWords = 0;
        if (hipMalloc(&ctx->ssgBits, bitsWords * 64 * sizeof(unsigned long long)) != hipSuccess) return fail_();
        ctx->ssgBitsWords = bitsWords;
    }
    if (samples > ctx->ssgSamples) {
        (void)hipFree(ctx->ssgLog);
        (void)hipFree(ctx->ssgEnd);
        ctx->ssgLog = nullptr;
        ctx->ssgEnd = nullptr;
        ctx->ssgSamples = 0;
        if (hipMalloc(&ctx->ssgLog, samples * 64 * 3 * sizeof(float)) != hipSuccess ||
            hipMalloc(&ctx->ssgEnd, samples * 64 * sizeof(uint16_t)) != hipSuccess)
            return fail_();
        ctx->ssgSamples = samples;
    }
    if (patchSamples > ctx->patchSamples) {
        (void)hipFree(ctx->patchLog);
        (void)hipFree(ctx->patchEnd);
        ctx->patchLog = nullptr;
        ctx->patchEnd = nullptr;
        ctx->patchSamples = 0;
        if (hipMalloc(&ctx->patchLog, patchSamples * 64 * 3 * sizeof(float)) != hipSuccess ||
            hipMalloc(&ctx->patchEnd, patchSamples * 64 * sizeof(uint16_t)) != hipSuccess)
            return fail_();
        ctx->patchSamples = patchSamples;
    }
    return true;
}

// The sample-group logs of a context that launches plain again (up to ~15 GB at a 1080p rank share
// at N = 8) are released; the per-pixel statistics (pairs, fold state) stay for the next guesses.
static void ssg_release(pt_context* ctx)
{
    if (!ctx->ssgItems && !ctx->ssgSamples && !ctx->patchSamples && !ctx->ssgBitsWords) return;
    (void)hipStreamSynchronize(ctx->stream);
    for (void* q : {(void*)ctx->ssgStart, (void*)ctx->ssgCount, (void*)ctx->ssgBits, (void*)ctx->ssgLog,
                    (void*)ctx->ssgEnd, (void*)ctx->patchLog, (void*)ctx->patchEnd})
        (void)hipFree(q);
    ctx->ssgStart = nullptr;
    ctx->ssgCount = nullptr;
    ctx->ssgBits = nullptr;
    ctx->ssgLog = nullptr;
    ctx->ssgEnd = nullptr;
    ctx->patchLog = nullptr;
    ctx->patchEnd = nullptr;
    ctx->ssgItems = ctx->ssgSamples = ctx->patchSamples = ctx->ssgBitsWords = 0;
}

// Stable radix sort of (cost, tile) pairs, descending, into the dispatch order: deterministic, ties
// in tile order.
static int sort_order(pt_context* ctx, uint32_t tiles, uint64_t samples, uint32_t strip)
{
    ctx->orderSamples = samples;
    ctx->orderStrip = strip;
    size_t bytes = ctx->sortTempBytes;
    PT_HIP_CHECK(ctx, rocprim::radix_sort_pairs_desc(ctx->sortTemp, bytes, ctx->tileCost, ctx->sortKeys, ctx->tileIds,
                                                     ctx->order, tiles, 0, 32, ctx->stream));
    PT_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    ctx->orderValid = true;
    ctx->orderStale = false;
    return PT_OK;
}

// Guess, grouped launch, fold, patch rounds and resume of speculative sample groups over the first
// `groupTiles` tiles of P.order (all tiles when P.order is null), on `s`.
static int run_groups(pt_context* ctx, int variant, const TraceParams& P0, uint32_t G, uint32_t groupTiles,
                      uint32_t ssgCap, hipStream_t s)
{
    TraceParams P = P0;
    const uint32_t total = P.spp * P.chunks;
    const uint32_t ssgN = total / G;
    const size_t items = (size_t)groupTiles * (2 * G - 1);
    const unsigned pixBlocks = (unsigned)(((size_t)groupTiles * 64 + 255) / 256);
    P.ssgG = G;
    P.ssgTiles = groupTiles;
    P.ssgCap = ssgCap;
    P.ssgLog = ctx->ssgLog;
    P.ssgEnd = ctx->ssgEnd;
    P.ssgStart = ctx->ssgStart;
    P.ssgBits = ctx->ssgBits;
    P.ssgCount = ctx->ssgCount;
    P.ssgWin = ssg_window_words(G, ssgN);
    P.fold = ctx->fold;
    P.numSlots = (uint32_t)items;
    ctx->groupStats[0] = G;
    PT_HIP_CHECK(ctx, hipMemsetAsync(ctx->ssgBits, 0, items * P.ssgWin * 64 * sizeof(unsigned long long), s));
    PT_HIP_CHECK(ctx, hipMemsetAsync(ctx->deadCount, 0, sizeof(uint32_t), s));
    ssg_guess_kernel<<<pixBlocks, 256, 0, s>>>(P, ctx->pairs, ssgN, ctx->ssgStart);
    PT_HIP_CHECK(ctx, hipGetLastError());
    P.ssgLook[0] = ctx->ssgLook[0];
    P.ssgLook[1] = ctx->ssgLook[1];
    PT_HIP_CHECK(ctx, launch_grouped<1>(variant, P, s));
    ssg_fold_kernel<<<pixBlocks, 256, 0, s>>>(P, 0, ctx->patchLog, ctx->patchEnd, ctx->patchCount, ssgCap, ctx->pairs,
                                              ctx->deadCount);
    PT_HIP_CHECK(ctx, hipGetLastError());
    ctx->pairsValid = true;
    // Patch rounds: a carrier from each dead end (the exact state there) runs until it meets a
    // later group's parse, and the fold continues; what is left after them runs plain.
    TraceParams Q = P;
    Q.ssgPatch = 1;
    Q.ssgLog = ctx->patchLog;
    Q.ssgEnd = ctx->patchEnd;
    Q.ssgCount = ctx->patchCount;
    Q.numSlots = groupTiles;
    Q.tileCost = nullptr;
    uint32_t dead = 0;
    for (uint32_t r = 1;; ++r) {
        PT_HIP_CHECK(ctx, hipMemcpyAsync(&dead, ctx->deadCount, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        PT_HIP_CHECK(ctx, hipStreamSynchronize(s));
        if (r - 1 < 8) ctx->groupStats[2 + r - 1] = dead;
        if (dead == 0 || r > ctx->patchRounds) break;
        ctx->groupStats[1] = r;
        PT_HIP_CHECK(ctx, hipMemsetAsync(ctx->deadCount, 0, sizeof(uint32_t), s));
        PT_HIP_CHECK(ctx, launch_grouped<1>(variant, Q, s));
        ssg_fold_kernel<<<pixBlocks, 256, 0, s>>>(P, r, ctx->patchLog, ctx->patchEnd, ctx->patchCount, ssgCap, ctx->pairs,
                                                  ctx->deadCount);
        PT_HIP_CHECK(ctx, hipGetLastError());
    }
    if (dead) {
        TraceParams R = P;
        R.ssgG = 0;
        R.numSlots = groupTiles;
        R.tileCost = nullptr;
        PT_HIP_CHECK(ctx, launch_grouped<2>(variant, R, s));
    }
    return PT_OK;
}

// Issue priority of a launch over `tiles` order positions (pt_set_issue_priority): position bounds of
// priority levels 3, 2, 1; the rest run at 0.
static void issue_priority(const pt_context* ctx, uint32_t tiles, uint32_t* prio)
{
    if (ctx->prioMode == 2) {
        for (int i = 0; i < 3; ++i) prio[i] = ctx->prioBounds[i];
        return;
    }
    for (int i = 0; i < 3; ++i) prio[i] = 0;
    if (ctx->prioMode == 1) return;
    // automatic: graded by quarter of the order -- the most expensive quarter of the tiles at
    // priority 3, the next at 2, then 1, the cheapest quarter at 0.  Measured on the refined cost
    // order (tools/sched_probe.py, profiles/r03_priority_policies.json): C3 N = 1 239.7 -> 235.8 ms,
    // its N = 2 share 141.6 -> 128.6 ms, the C4 N = 8 share 552.6 -> 496.2 ms; no setting was slower.
    prio[0] = tiles / 4;
    prio[1] = tiles / 2;
    prio[2] = tiles - tiles / 4;
}

static int render_impl(pt_context* ctx, const pt_camera* cam, uint32_t spp, uint32_t chunks, int ignore, float* gpu_ms,
                       pt_render_stats* stats)
{
    if (!ctx || !cam) return PT_ERR_ARG;
    if (gpu_ms) *gpu_ms = 0.0f;
    if (stats) memset(stats, 0, sizeof(*stats));
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    if (ctx->nodeCount < 1 || ctx->primCount < 1 || spp == 0 || chunks == 0 || ctx->rows == 0) return PT_OK;
    // textures referenced by the launch must exist (the reference would read an invalid object)
    if (ctx->skybox != 0 && ctx->hostTex[ctx->skybox - 1].texels == nullptr)
        return fail(ctx, PT_ERR_STATE, "pt_render: skybox handle has no texture");
    TraceParams P;
    memset(&P, 0, sizeof(P));
    P.accum = ctx->accum;
    P.rng = ctx->rng;
    P.nodes = ctx->nodes;
    P.prims = ctx->prims;
    P.mats = ctx->mats;
    P.textures = ctx->texTable;
    P.stats = ctx->stats;
    P.skybox = ctx->skybox;
    if (ctx->skybox != 0) P.skyTex = ctx->hostTex[ctx->skybox - 1];
    P.width = ctx->width;
    P.height = ctx->height;
    P.fwidth = (float)ctx->width;
    P.fheight = (float)ctx->height;
    P.rowOffset = ctx->rowOffset;
    P.rowStride = ctx->rowStride;
    P.rows = ctx->rows;
    P.bandShift = ctx->bandShift;
    P.spp = spp;
    P.chunks = chunks;
    P.ignoreFirst = ignore ? 1u : 0u;
    P.tilesX = (ctx->width + 7) / 8;
    P.tilesY = (ctx->rows + 7) / 8;
    P.cam.origin = hf3(cam->origin);
    P.cam.llc = hf3(cam->lower_left_corner);
    P.cam.horizontal = hf3(cam->horizontal);
    P.cam.vertical = hf3(cam->vertical);
    P.nodeCount = ctx->nodeCount;
    P.primCount = ctx->primCount;
    P.stackDepth = ctx->stackDepth;
    P.slabFast = ctx->slabFast ? 1u : 0u;
    P.cnodes = ctx->cnodes;
    P.cnodeCount = ctx->cnodeCount;
    P.rootWord = ctx->rootWord;
    for (int k = 0; k < 6; ++k) P.rootBox[k] = ctx->rootBox[k];
    // Tile scheduling: a pixel's samples are sequential (one XORWOW stream), so a tile is the
    // smallest unit of work, and tiles differ several-fold in cost (sky vs geometry).  Every
    // launch records each tile's cycle count; after a scene, texture or camera change the
    // dispatch order is rebuilt on the device from the latest costs (most expensive first, a
    // stable radix sort), so
    // the launch tail consists of cheap tiles and the waves of a workgroup (which hold the
    // group's LDS until the last one ends) have similar lengths.  A camera move keeps using the
    // previous order for one launch.  The order changes which wave renders a tile, never how:
    // results are identical.
    const uint32_t tiles = P.tilesX * P.tilesY;
    if (ctx->orderTiles != tiles) {
        (void)hipFree(ctx->tileCost);
        (void)hipFree(ctx->order);
        (void)hipFree(ctx->tileIdle);
        ctx->tileCost = nullptr;
        ctx->order = nullptr;
        ctx->tileIdle = nullptr;
        ctx->orderTiles = 0;
        ctx->orderValid = false;
        PT_HIP_CHECK(ctx, hipMalloc(&ctx->tileCost, (size_t)tiles * sizeof(uint32_t)));
        PT_HIP_CHECK(ctx, hipMalloc(&ctx->order, ((size_t)tiles + 64) * sizeof(uint32_t)));
        (void)hipFree(ctx->sortKeys);
        (void)hipFree(ctx->tileIds);
        (void)hipFree(ctx->sortTemp);
        ctx->sortKeys = ctx->tileIds = nullptr;
        ctx->sortTemp = nullptr;
        PT_HIP_CHECK(ctx, hipMalloc(&ctx->sortKeys, (size_t)tiles * sizeof(uint32_t)));
        PT_HIP_CHECK(ctx, hipMalloc(&ctx->tileIds, (size_t)tiles * sizeof(uint32_t)));
        ctx->sortTempBytes = 0;
        PT_HIP_CHECK(ctx, rocprim::radix_sort_pairs_desc(nullptr, ctx->sortTempBytes, ctx->tileCost, ctx->sortKeys,
                                                         ctx->tileIds, ctx->order, tiles, 0, 32, ctx->stream));
        PT_HIP_CHECK(ctx, hipMalloc(&ctx->sortTemp, ctx->sortTempBytes ? ctx->sortTempBytes : 4));
        PT_HIP_CHECK(ctx, hipMemsetAsync(ctx->tileCost, 0, (size_t)tiles * sizeof(uint32_t), ctx->stream));
        // tiles as packed coordinates (tileY << 16 | tileX: the kernel needs no division by tilesX);
        // slots past the last tile stay invalid (tileY = tilesY)
        std::vector<uint32_t> ident((size_t)tiles + 64);
        for (size_t i = 0; i < ident.size(); ++i)
            ident[i] = i < tiles ? ((uint32_t)(i / P.tilesX) << 16) | (uint32_t)(i % P.tilesX) : P.tilesY << 16;
        (void)hipFree(ctx->rowMajor);
        ctx->rowMajor = nullptr;
        PT_HIP_CHECK(ctx, hipMalloc(&ctx->rowMajor, ident.size() * sizeof(uint32_t)));
        PT_HIP_CHECK(ctx, hipMemcpy(ctx->rowMajor, ident.data(), ident.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        PT_HIP_CHECK(ctx, hipMemcpy(ctx->order, ident.data(), ident.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        PT_HIP_CHECK(ctx, hipMemcpy(ctx->tileIds, ident.data(), (size_t)tiles * sizeof(uint32_t), hipMemcpyHostToDevice));
        ctx->orderTiles = tiles;
        ctx->orderStale = true;
    }
    // Run-ahead across render() calls (MODE 4): a stash made by the previous launch is valid when
    // this launch has its camera, scene, textures, sky and RNG state (stateEpoch); a context whose
    // camera or state changed on the last two launches (a moving progressive camera) stops making
    // stashes until it holds still again.
    const bool sameKey = ctx->launched && memcmp(&ctx->lastCam, cam, sizeof(pt_camera)) == 0 &&
                         ctx->lastState == ctx->stateEpoch;
    ctx->aheadMisses = sameKey ? 0u : std::min(ctx->aheadMisses + 1u, 1000u);
    const bool stashMatches = ctx->aheadValid && sameKey;
    ctx->aheadValid = false;              // consumed or dropped; a making launch sets it again
    ctx->launched = true;
    ctx->lastState = ctx->stateEpoch;
    if (memcmp(&ctx->lastCam, cam, sizeof(pt_camera)) != 0) {
        ctx->orderStale = true;
        ctx->lastCam = *cam;
    }
    const bool sorted = ctx->schedule == 0;
    // Strip units (MODE 3, trace_kernel): launches of few samples per pixel dispatch row strips of K
    // tiles, and a lane whose pixel is done moves on to the next tile of its strip.  The cost order
    // is over units, so it is rebuilt when K changes.
    const bool noRepair = !ctx->riseRepair;           // test knob: plain launches of variant 90 only
    const uint64_t launchSamples = (uint64_t)spp * chunks;
    // (strip units or sample groups forced by their knobs take precedence over automatic run-ahead)
    const bool aheadCapable = !stats && !noRepair && ctx->cnodes && strip_capable(pick_variant(ctx)) && ctx->aheadMode != 1 &&
                              (ctx->aheadMode == 2 || (ctx->stripMode < 2 && ctx->ssgMode < 2));
    const bool aheadUse = aheadCapable && stashMatches && ctx->aheadMode != 3;   // 3: diagnostic, never consume
    const bool aheadMake = aheadCapable && (ctx->aheadMode == 2 ||
        (launchSamples >= kAheadMinSamples && launchSamples <= kAheadMaxSamples && ctx->aheadMisses < 2));
    const bool ahead = aheadUse || aheadMake;
    const uint32_t K = (sorted && !stats && !noRepair && !ahead) ? strip_tiles(ctx, pick_variant(ctx), tiles, launchSamples) : 1u;
    const uint32_t unitsX = (P.tilesX + K - 1) / K, units = unitsX * P.tilesY;
    if (K != ctx->orderStrip) {
        ctx->orderValid = false;
        ctx->orderStale = true;
    }
    if (K > 1 && (ctx->unitK != K || ctx->unitTiles != tiles)) {
        (void)hipFree(ctx->unitMajor);
        ctx->unitMajor = nullptr;
        std::vector<uint32_t> um((size_t)units + 64);
        for (size_t i = 0; i < um.size(); ++i)
            um[i] = i < units ? ((uint32_t)(i / unitsX) << 16) | (uint32_t)(i % unitsX * K) : P.tilesY << 16;
        PT_HIP_CHECK(ctx, hipMalloc(&ctx->unitMajor, um.size() * sizeof(uint32_t)));
        PT_HIP_CHECK(ctx, hipMemcpy(ctx->unitMajor, um.data(), um.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        ctx->unitK = K;
        ctx->unitTiles = tiles;
    }
    uint32_t* const firstOrder = K > 1 ? ctx->unitMajor : ctx->rowMajor;
    P.strip = K;
    P.order = (sorted && ctx->orderValid) ? ctx->order : firstOrder;
    P.tileCost = sorted ? ctx->tileCost : nullptr;
    P.scatterWaves = ctx->schedule == 2 ? (uint32_t)(((size_t)ctx->rows * ctx->width + 63) / 64) : 0u;
    if (P.scatterWaves) P.order = nullptr;          // scattered mapping: slot = wave index
    if (!ctx->tileCursor) {
        PT_HIP_CHECK(ctx, hipMalloc(&ctx->tileCursor, 2 * sizeof(uint32_t)));
        PT_HIP_CHECK(ctx, hipMemset(ctx->tileCursor, 0, 2 * sizeof(uint32_t)));
    }
    P.tileCursor = ctx->tileCursor;
    P.numSlots = units;
    P.occCap = ctx->occupancy;
    // Issue priority follows the order position, so it is meaningful only on a current cost order.
    // A launch whose tile costs will rebuild the order (stale order, or this launch measures >= 4x
    // the samples the order came from; see the rebuild below) runs without it: graded priority
    // shortens the head quarter's tiles, and costs measured under it would rank those tiles lower
    // on every rebuild (a feedback the order would carry over camera moves).
    const bool rebuilds = ctx->schedule == 0 &&
                          (ctx->orderStale || !ctx->orderValid || (uint64_t)spp * chunks >= 4 * ctx->orderSamples);
    if (!rebuilds || ctx->prioMode == 2) issue_priority(ctx, units, P.prio);   // explicit bounds: always
    if (stats) {
        PT_HIP_CHECK(ctx, hipMemsetAsync(ctx->stats, 0, kStatWords * sizeof(unsigned long long), ctx->stream));
        if (!ctx->tileIdle) PT_HIP_CHECK(ctx, hipMalloc(&ctx->tileIdle, (size_t)tiles * sizeof(uint32_t)));
        PT_HIP_CHECK(ctx, hipMemsetAsync(ctx->tileIdle, 0, (size_t)tiles * sizeof(uint32_t), ctx->stream));
        P.tileIdle = ctx->tileIdle;
    }
    int variant = pick_variant(ctx);
    // speculative sample groups
    const uint32_t total = spp * chunks;
    // the fold state packs (sample in call, call) into one word as sIdx | c << 16 (ssg_fold_kernel)
    const bool groupable = !stats && sorted && (uint64_t)spp * chunks < (1ull << 31) && spp <= 0xffffu && chunks <= 0xffffu;
    uint32_t G = groupable && K == 1 && !noRepair && !ahead ? ssg_groups(ctx, variant, tiles, total) : 0;
    if (!G && ctx->variant == 0 && K == 1 && !noRepair && !ahead) variant = small_grid_variant(ctx, variant, tiles);
    // The sixth wave slot (variants 60 / 61) raises throughput but gives each wave a smaller share of
    // the SIMD's issue: a plain launch of few tiles per slot, whose end is its heaviest tiles' sample
    // chains, runs longer with it (the C4 N = 8 share, 2.6 tiles per six-wave slot: 532 against 498 ms;
    // C3, 5.3 tiles per slot: 224.2 against 231.2; profiles/r05_six_waves.json).  Plain launches of
    // fewer than 4 dispatch units per six-wave slot (also 1-spp strip-unit frames) run the five-wave build.
    if (!G && ctx->variant == 0 && (variant == 60 || variant == 61)) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess ||
            (uint64_t)units < 4ull * cus * 4 * 6)
            variant = variant == 60 ? 40 : 41;
    }
    if (ahead) {
        if (!ctx->ahead) {
            const size_t n = std::max<size_t>((size_t)ctx->rows * ctx->width, 1);
            PT_HIP_CHECK(ctx, hipMalloc(&ctx->ahead, kAheadWords * n * sizeof(uint32_t)));
        }
        P.ahead = ctx->ahead;
        P.aheadUse = aheadUse ? 1u : 0u;
        P.aheadMake = aheadMake ? 1u : 0u;
    }
    if (noRepair) {
        if (variant == 60) variant = 40;              // (the no-repair build exists at five waves only)
        if (variant != 40 || stats)
            return fail(ctx, PT_ERR_STATE, "pt_set_rise_repair(0): only plain launches of variant 40 have a no-repair build");
        variant = 90;
    }
    // Grouped launches of at most one tile per wave slot (one rank's 1080p share at N = 8) are
    // short items whose latency sets the launch: deferred shading, which trades a lane's latency for
    // fuller hit-shading rounds, measured bimodal there (median 57.7-62.6 ms against 57.8-58.2 ms
    // without; at N = 4, two tiles per slot, 96.8 against 103.9), so they run the undeferred walk.
    if (G && ctx->variant == 0 && (variant == 40 || variant == 60)) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) == hipSuccess &&
            (uint64_t)tiles <= (uint64_t)cus * 4 * variant_waves(variant))
            variant = 39;
    }
    ctx->lastGroups = 0;
    ctx->lastVariant = variant;
    memset(ctx->groupStats, 0, sizeof(ctx->groupStats));
    ++ctx->epoch;
    uint32_t ssgCap = 0;
    if (G) {
        const uint32_t ssgN = total / G;
        // an item runs its group and, where the next group's guess missed, into the group after it;
        // further dead ends go to patch rounds
        ssgCap = std::min<uint32_t>({total, 2 * ssgN + 64, 10000u});   // end offsets: 16-bit draw pairs (<= 6 per sample)
        const size_t J = 2 * (size_t)G - 1;
        if (!ssg_reserve(ctx, tiles, (size_t)tiles * J, (size_t)tiles * J * ssgCap, (size_t)tiles * ssgCap,
                         (size_t)tiles * J * ssg_window_words(G, ssgN)))
            G = 0;
    }
    // a plain launch after grouped ones releases the group logs (a stream synchronisation and frees
    // of up to ~15 GB): before the timed region starts
    if (!G) ssg_release(ctx);
    PT_HIP_CHECK(ctx, hipEventRecord(ctx->ev0, ctx->stream));
    // Cold start (first launch, or the scene, a texture or the camera changed): no tile costs yet.
    // Progressive 1-spp frames reuse the previous order for one launch.  A launch of several render()
    // calls runs its FIRST call as a launch of its own in row-major order, sorts the tiles by that
    // call's costs on the device and runs the other calls in that order -- nothing is computed twice,
    // and two launches of 1 and chunks - 1 calls are the reference's calls exactly as one launch is
    // (each call folds into the accumulation, ignoreHistory applies to the first).  Other launches
    // (one call, or sample groups, which take their draw-pair guesses from it) run a short discarded
    // pre-pass instead.  Either way the launch then runs with issue priority on that order
    // (pt_set_cold_start; measured: one-shot C3 251-255 -> 238-240 ms, tools/cold_start.py); as its
    // tile costs are measured under priority, the order rebuilt from them is biased toward the head's
    // tiles, so the next launch rebuilds it again without priority (orderSamples = 0 below).
    const bool cold = sorted && (ctx->orderStale || !ctx->orderValid) && (uint64_t)spp * chunks >= kPrepassMinSpp && !stats;
    const bool splitCall = cold && chunks >= 2 && !G && K == 1 && !ahead && ctx->prepassSpp == 0;
    bool biasedOrder = false;
    if (splitCall) {
        TraceParams Q = P;
        Q.chunks = 1;
        Q.order = firstOrder;
        for (int i = 0; i < 3; ++i) Q.prio[i] = 0;        // row-major positions: no priority grading
        PT_HIP_CHECK(ctx, launch_variant<false>(variant, Q, ctx->stream));
        const int rs = sort_order(ctx, tiles, spp, K);
        if (rs != PT_OK) return rs;
        P.order = ctx->order;
        P.chunks = chunks - 1;
        P.ignoreFirst = 0;                               // the first call is done
        if (ctx->coldPriority && ctx->prioMode == 0) {
            issue_priority(ctx, units, P.prio);
            biasedOrder = true;
        }
    } else if (cold) {
        // pre-pass: kPrepassSpp samples per pixel from the pixels' current RNG state, nothing
        // written back (discard)
        TraceParams Q = P;
        const bool guesses = G != 0;           // speculative groups also take their offset guesses from it
        Q.spp = guesses ? 8u : (ctx->prepassSpp ? ctx->prepassSpp : kPrepassSpp);
        Q.chunks = 1;
        Q.ignoreFirst = 1;
        Q.discard = 1;
        Q.order = firstOrder;
        for (int i = 0; i < 3; ++i) Q.prio[i] = 0;        // row-major positions: no priority grading
        Q.pairsOut = guesses && ssg_reserve(ctx, tiles, 0, 0, 0) ? ctx->pairs : nullptr;
        if (Q.pairsOut) ctx->pairsValid = true;
        PT_HIP_CHECK(ctx, Q.pairsOut ? launch_grouped<2>(variant, Q, ctx->stream)
                                     : (K > 1 ? launch_strip(variant, Q, ctx->stream) : launch_variant<false>(variant, Q, ctx->stream)));
        const int rs = sort_order(ctx, tiles, Q.spp, K);
        if (rs != PT_OK) return rs;
        P.order = ctx->order;
        if (ctx->coldPriority && ctx->prioMode == 0) {
            issue_priority(ctx, units, P.prio);
            biasedOrder = true;
        }
    }
    if (G && P.tileCost) PT_HIP_CHECK(ctx, hipMemsetAsync(P.tileCost, 0, (size_t)tiles * sizeof(uint32_t), ctx->stream));
    if (G) {
        const int rc = run_groups(ctx, variant, P, G, tiles, ssgCap, ctx->stream);
        if (rc != PT_OK) return rc;
        ctx->lastGroups = G;
    } else {
        PT_HIP_CHECK(ctx, stats ? launch_variant<true>(variant, P, ctx->stream)
                                : ahead ? launch_ahead(variant, P, ctx->stream)
                                : (K > 1 ? launch_strip(variant, P, ctx->stream) : launch_variant<false>(variant, P, ctx->stream)));
    }
    if (aheadMake) {
        ctx->aheadValid = true;
        ctx->aheadCam = *cam;
        ctx->aheadState = ctx->stateEpoch;
    }
    PT_HIP_CHECK(ctx, hipGetLastError());
    PT_HIP_CHECK(ctx, hipEventRecord(ctx->ev1, ctx->stream));
    PT_HIP_CHECK(ctx, hipEventSynchronize(ctx->ev1));
    float ms = 0.0f;
    PT_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    if (gpu_ms) *gpu_ms = ms;
    // The order is rebuilt from this launch's tile costs when it is stale, or when this launch
    // measured every tile over at least 4x as many samples as the costs the order came from (a cold
    // start's 2-spp pre-pass, an 8-spp first launch): short launches rank tiles noisily, and a heavy
    // tile ranked light is dispatched late and becomes the launch's tail.
    if (sorted && (ctx->orderStale || !ctx->orderValid || total >= 4 * ctx->orderSamples)) {
        const int rs = sort_order(ctx, tiles, total, K);
        if (rs != PT_OK) return rs;
        if (biasedOrder) ctx->orderSamples = 0;          // costs measured under priority: rebuild once more
    }
    if (stats) {
        unsigned long long h[kStatWords];
        PT_HIP_CHECK(ctx, hipMemcpy(h, ctx->stats, sizeof(h), hipMemcpyDeviceToHost));
        stats->node_tests = h[0];
        stats->prim_tests = h[1];
        stats->hits = h[2];
        stats->sky_lookups = h[3];
        stats->segments = h[4];
        stats->samples = h[5];
        stats->wave_node_iters = h[6];
        stats->wave_prim_iters = h[7];
        stats->wave_hits = h[8];
        stats->wave_sky = h[9];
        stats->wave_segments = h[10];
        stats->cycles_node_walk = h[11];
        stats->cycles_leaf_tests = h[12];
        stats->cycles_shading = h[13];
        stats->cycles_total = h[14];
        stats->cycles_lane_idle = h[15];
        stats->leaf_rounds = h[16];
        stats->family_execs = h[17];
        stats->family_execs_compacted = h[18];
        stats->leaf_round_lanes = h[19];
        stats->leaf_pairs = h[20];
        stats->family_execs_compacted_in_round = h[21];
        stats->repairs = h[22];
    }
    return PT_OK;
}

PT_API int pt_set_cold_start(pt_context* ctx, uint32_t prepass_spp, int priority)
{
    if (!ctx || prepass_spp > 64 || priority < 0 || priority > 1) return PT_ERR_ARG;
    ctx->prepassSpp = prepass_spp;
    ctx->coldPriority = priority != 0;
    return PT_OK;
}

PT_API int pt_set_run_ahead(pt_context* ctx, int mode)
{
    if (!ctx || mode < 0 || mode > 3) return PT_ERR_ARG;
    ctx->aheadMode = mode;
    return PT_OK;
}

PT_API int pt_set_rise_repair(pt_context* ctx, int enabled)
{
    if (!ctx || enabled < 0 || enabled > 1) return PT_ERR_ARG;
    ctx->riseRepair = enabled != 0;
    return PT_OK;
}

PT_API int pt_set_strip_units(pt_context* ctx, int mode)
{
    if (!ctx || mode < 0 || mode > 16) return PT_ERR_ARG;
    ctx->stripMode = mode;
    return PT_OK;
}

PT_API int pt_set_sample_groups(pt_context* ctx, int mode)
{
    if (!ctx || mode < 0 || mode > 4096) return PT_ERR_ARG;
    ctx->ssgMode = mode;
    return PT_OK;
}

PT_API int pt_set_group_lookback(pt_context* ctx, uint32_t far, uint32_t near)
{
    if (!ctx || far > 256 || near > 256) return PT_ERR_ARG;
    ctx->ssgLook[0] = far;
    ctx->ssgLook[1] = near;
    return PT_OK;
}

PT_API int pt_set_patch_rounds(pt_context* ctx, uint32_t rounds)
{
    if (!ctx || rounds > 64) return PT_ERR_ARG;
    ctx->patchRounds = rounds;
    return PT_OK;
}

PT_API int pt_last_sample_groups(const pt_context* ctx)
{
    return ctx ? (int)ctx->lastGroups : 0;
}

PT_API int pt_last_variant(const pt_context* ctx) { return ctx ? ctx->lastVariant : 0; }


PT_API int pt_read_group_log_counts(pt_context* ctx, uint32_t* dst, size_t count)
{
    if (!ctx || !dst) return PT_ERR_ARG;
    if (!ctx->ssgCount || ctx->lastGroups == 0) return PT_ERR_STATE;
    const size_t tiles = (size_t)((ctx->width + 7) / 8) * ((ctx->rows + 7) / 8);
    const size_t n = tiles * (2 * ctx->lastGroups - 1) * 64;
    if (count < n) return PT_ERR_ARG;
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    PT_HIP_CHECK(ctx, hipMemcpy(dst, ctx->ssgCount, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return PT_OK;
}

PT_API int pt_read_group_fold(pt_context* ctx, uint32_t word, uint32_t* dst)
{
    if (!ctx || !dst || word >= kFoldWords + 3) return PT_ERR_ARG;
    if (!ctx->fold) return PT_ERR_STATE;
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    const size_t npix = (size_t)ctx->rows * ctx->width;
    const void* src = word >= kFoldWords ? (const void*)(ctx->pairs + (word - kFoldWords) * npix)
                                         : (const void*)(ctx->fold + (size_t)word * npix);
    PT_HIP_CHECK(ctx, hipMemcpy(dst, src, npix * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return PT_OK;
}

PT_API int pt_read_group_stats(const pt_context* ctx, uint32_t* dst)
{
    if (!ctx || !dst) return PT_ERR_ARG;
    memcpy(dst, ctx->groupStats, sizeof(ctx->groupStats));
    return PT_OK;
}

PT_API int pt_set_issue_priority(pt_context* ctx, int mode, uint32_t level3, uint32_t level2, uint32_t level1)
{
    if (!ctx || mode < 0 || mode > 2 || (mode == 2 && !(level3 <= level2 && level2 <= level1))) return PT_ERR_ARG;
    ctx->prioMode = mode;
    ctx->prioBounds[0] = level3;
    ctx->prioBounds[1] = level2;
    ctx->prioBounds[2] = level1;
    return PT_OK;
}

PT_API int pt_set_occupancy(pt_context* ctx, uint32_t workgroups_per_cu)
{
    if (!ctx || workgroups_per_cu > 16) return PT_ERR_ARG;
    ctx->occupancy = workgroups_per_cu;
    return PT_OK;
}

PT_API int pt_set_schedule(pt_context* ctx, int mode)
{
    if (!ctx || mode < 0 || mode > 2) return PT_ERR_ARG;
    ctx->schedule = mode;
    ctx->orderStale = true;
    return PT_OK;
}

PT_API int pt_render(pt_context* ctx, const pt_camera* camera, uint32_t spp, uint32_t chunks, int ignore_history,
                     float* gpu_ms)
{
    return render_impl(ctx, camera, spp, chunks, ignore_history, gpu_ms, nullptr);
}

PT_API int pt_render_instrumented(pt_context* ctx, const pt_camera* camera, uint32_t spp, uint32_t chunks, int ignore_history,
                           float* gpu_ms, pt_render_stats* stats)
{
    if (!stats) return PT_ERR_ARG;
    return render_impl(ctx, camera, spp, chunks, ignore_history, gpu_ms, stats);
}

PT_API int pt_read_accum(pt_context* ctx, float* dst)
{
    if (!ctx || !dst) return PT_ERR_ARG;
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    PT_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    PT_HIP_CHECK(ctx, hipMemcpy(dst, ctx->accum, (size_t)ctx->rows * ctx->width * sizeof(float4), hipMemcpyDeviceToHost));
    return PT_OK;
}

PT_API int pt_copy_accum_device(pt_context* ctx, void* dst_device, size_t bytes)
{
    if (!ctx || !dst_device) return PT_ERR_ARG;
    const size_t need = (size_t)ctx->rows * ctx->width * sizeof(float4);
    if (bytes < need) return fail(ctx, PT_ERR_ARG, "pt_copy_accum_device: destination too small");
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    PT_HIP_CHECK(ctx, hipMemcpyAsync(dst_device, ctx->accum, need, hipMemcpyDeviceToDevice, ctx->stream));
    PT_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    return PT_OK;
}

PT_API int pt_tonemap_device(pt_context* ctx, uint32_t frames, void* dst, size_t dst_bytes)
{
    if (!ctx || !dst) return PT_ERR_ARG;
    const size_t npix = (size_t)ctx->rows * ctx->width;
    if (dst_bytes < npix * sizeof(uchar4)) return fail(ctx, PT_ERR_ARG, "pt_tonemap_device: destination too small");
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    if (npix == 0) return PT_OK;
    tonemap_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, ctx->stream>>>(static_cast<uchar4*>(dst), ctx->accum, npix,
                                                                             frames);
    PT_HIP_CHECK(ctx, hipGetLastError());
    PT_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    return PT_OK;
}

PT_API int pt_tonemap(pt_context* ctx, uint32_t frames, uint8_t* dst)
{
    if (!ctx || !dst) return PT_ERR_ARG;
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    const size_t npix = (size_t)ctx->rows * ctx->width;
    if (npix == 0) return PT_OK;
    if (!ctx->ldr) PT_HIP_CHECK(ctx, hipMalloc(&ctx->ldr, npix * sizeof(uchar4)));   // kept for per-frame use
    tonemap_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, ctx->stream>>>(ctx->ldr, ctx->accum, npix, frames);
    PT_HIP_CHECK(ctx, hipGetLastError());
    PT_HIP_CHECK(ctx, hipMemcpyAsync(dst, ctx->ldr, npix * sizeof(uchar4), hipMemcpyDeviceToHost, ctx->stream));
    PT_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    return PT_OK;
}

PT_API int pt_read_rng(pt_context* ctx, uint32_t* dst)
{
    if (!ctx || !dst) return PT_ERR_ARG;
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    PT_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    const size_t npix = (size_t)ctx->rows * ctx->width;
    std::vector<uint32_t> soa(6 * npix);
    PT_HIP_CHECK(ctx, hipMemcpy(soa.data(), ctx->rng, soa.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < npix; ++i)
        for (int k = 0; k < 6; ++k) dst[6 * i + k] = soa[k * npix + i];
    return PT_OK;
}

PT_API int pt_write_rng(pt_context* ctx, const uint32_t* src)
{
    if (!ctx || !src) return PT_ERR_ARG;
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    PT_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    const size_t npix = (size_t)ctx->rows * ctx->width;
    std::vector<uint32_t> soa(6 * npix);
    for (size_t i = 0; i < npix; ++i)
        for (int k = 0; k < 6; ++k) soa[k * npix + i] = src[6 * i + k];
    PT_HIP_CHECK(ctx, hipMemcpy(ctx->rng, soa.data(), soa.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    ++ctx->stateEpoch;                    // a run-ahead stash continues the old streams: void
    return PT_OK;
}

PT_API uint32_t pt_local_rows(const pt_context* ctx) { return ctx ? ctx->rows : 0; }

PT_API int pt_read_tile_costs(pt_context* ctx, uint32_t* dst, uint32_t count)
{
    if (!ctx || !dst) return PT_ERR_ARG;
    if (!ctx->tileCost || count != ctx->orderTiles) return fail(ctx, PT_ERR_STATE, "pt_read_tile_costs: no costs of that size");
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    PT_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    PT_HIP_CHECK(ctx, hipMemcpy(dst, ctx->tileCost, (size_t)count * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return PT_OK;
}

PT_API int pt_read_tile_idle(pt_context* ctx, uint32_t* dst, uint32_t count)
{
    if (!ctx || !dst) return PT_ERR_ARG;
    if (!ctx->tileIdle || count != ctx->orderTiles) return fail(ctx, PT_ERR_STATE, "pt_read_tile_idle: no instrumented launch of that size");
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    PT_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    PT_HIP_CHECK(ctx, hipMemcpy(dst, ctx->tileIdle, (size_t)count * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return PT_OK;
}

PT_API int pt_set_kernel_variant(pt_context* ctx, int variant)
{
    if (!ctx) return PT_ERR_ARG;
    if (!variant_shipped(variant)) return fail(ctx, PT_ERR_ARG, "pt_set_kernel_variant: not a shipped variant");
    ctx->variant = variant;
    return PT_OK;
}

PT_API const char* pt_last_error(const pt_context* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

} // extern "C"

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
