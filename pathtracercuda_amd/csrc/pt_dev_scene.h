// Launch parameters, textures, primitives and their intersection tests, the counters of the
// instrumented launches and the node-at-a-time BVH walks.
// Part of the trace kernel's single translation unit: included by pt_kernels.hip inside its anonymous
// namespace, in this order: pt_dev_scene.h, pt_dev_walk.h, pt_dev_path.h, pt_dev_groups.h,
// pt_dev_fold.h; not a standalone header.
#pragma once


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
    uint32_t* tileTrace;        // instrumented launches, pt_set_tile_trace: per tile {start cycles, XCC << 16 | HW_ID}
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
    uint32_t spreadCU;          // persistent grids of CU-count multiples: the CU count (spread_slot), else 0
    uint32_t prioDealt;         // host only: persistent grids raise the first band to every position dealt
                                // at the start (launch_one; automatic priority)
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
