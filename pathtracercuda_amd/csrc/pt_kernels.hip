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
#include "pt_dev_scene.h"

#include "pt_dev_walk.h"

#include "pt_dev_path.h"

#include "pt_dev_groups.h"

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
        if (STATS && P.tileTrace) {              // schedule trace (pt_set_tile_trace): start, hardware ids
            P.tileTrace[2 * lin] = (uint32_t)tWave;
            P.tileTrace[2 * lin + 1] = (__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20) << 16) |
                                       (__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4) & 0xffffu);
        }
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
// First dispatch slot of wave `w` of workgroup `b` in a persistent grid of nCU x k workgroups.  The
// hardware places workgroups 0..nCU-1 on distinct CUs (round robin over the XCDs) and a workgroup's
// waves on distinct SIMDs, four apart (tools/hwid_probe.hip), so the slots -- positions in the cost
// order -- are dealt one per SIMD per round, every other round in reverse: a SIMD holds one of the
// heaviest tiles next to lighter ones of the later rounds.  A shared cursor instead hands the head to
// whichever waves start first, which cluster on a few CUs (208 distinct SIMDs among the first 1,024
// waves to start).  A bijection onto [0, grid x WPB); later slots come from the cursor after that range.
template <int WPB>
PT_DEV uint32_t spread_slot(uint32_t b, uint32_t w, uint32_t nCU)
{
    const uint32_t per = 4u * nCU;
    const uint32_t r = (b / nCU) * (uint32_t)(WPB / 4) + (w >> 2);
    const uint32_t idx = (w & 3u) * nCU + b % nCU;
    return r * per + ((r & 1u) ? per - 1u - idx : idx);
}

template <bool STATS, int SL, int WPB, int WW, int MINW, bool PERSIST = false, int MODE = 0>
__global__ void __launch_bounds__(WPB * 64, MINW) trace_kernel(TraceParams P)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    stage_scene_impl<SL, WPB, WW>(P);
    Counters cnt = {};
    const bool spread = PERSIST && P.spreadCU != 0;
    const uint32_t base = spread ? gridDim.x * (uint32_t)WPB : 0u;
    uint32_t slot = !PERSIST ? __builtin_amdgcn_readfirstlane(blockIdx.x * (uint32_t)WPB + wave)
                  : spread   ? spread_slot<WPB>(blockIdx.x, __builtin_amdgcn_readfirstlane(wave), P.spreadCU)
                             : wave_fetch(P.tileCursor, 1u);
    for (;;) {
    if (slot >= P.numSlots) break;               // also the grid's spare slots past the last item
    run_item<STATS, SL, WPB, WW, MINW, PERSIST, MODE>(P, slot, cnt);
    if (!PERSIST) break;
    slot = base + wave_fetch(P.tileCursor, 1u);
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

#include "pt_dev_fold.h"

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
    uint32_t* tileTrace = nullptr;    // pt_set_tile_trace: per tile {start cycles, hardware ids} of the last launch
    bool traceTiles = false;
    uint32_t traceCap = 0;
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
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 0;
        if (P.occCap && cus > 0)                       // tuning knob (pt_set_occupancy): fewer waves per SIMD
            cap = cus * std::min(cap / cus, (int)P.occCap);
        else if (P.occCap)
            cap = 0;
        if (!P.occCap && blocks <= (unsigned)cap) return launch_one<STATS, SL, WPB, WW, MINW, false, MODE>(P, stream);
        if (cap <= 0) return hipErrorInvalidValue;
        TraceParams Q = P;                             // first slots dealt per SIMD (spread_slot)
        Q.spreadCU = (cus > 0 && WPB % 4 == 0 && cap % cus == 0) ? (uint32_t)cus : 0u;
        if (P.prioDealt) {
            // Every position dealt at the start runs in the first priority band.  Waves of equal
            // priority issue oldest first (the resident grid's dispatch order: tools/tile_trace.py shows
            // the dealing rounds' tiles at 164 / 175 / 235 / 273 ms median and the last round's, at level
            // 2 below the others, at 373 ms -- the launch's end on the C4 N = 8 share); in one band the
            // order of the rounds follows the cost order.  C4 N = 8 share 464-481 -> 446-456 ms
            // (tools/prio_probe.py, profiles/r06_schedule_trace.json).
            const uint32_t dealt = std::min<uint32_t>(P.numSlots, (uint32_t)cap * WPB);
            Q.prio[0] = std::max(Q.prio[0], dealt);
            Q.prio[1] = std::max(Q.prio[1], Q.prio[0]);
            Q.prio[2] = std::max(Q.prio[2], Q.prio[1]);
        }
        trace_kernel<STATS, SL, WPB, WW, MINW, PERSIST, MODE><<<(unsigned)cap, WPB * 64, lds, stream>>>(Q);
        return hipGetLastError();
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
    // 60 / 61 instrumented: the six-wave builds themselves, so the counters of an
    // instrumented launch (lane utilisation, repairs) come from the kernel that is timed
    case 60: return launch_one<STATS, 1, 8, kV40Walk, 6, true, MODE>(P, stream);
    case 61: return launch_one<STATS, 0, 4, 14212, 6, true, MODE>(P, stream);
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
    (void)hipFree(ctx->tileTrace);
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
                          uint32_t& maxDepthOut, std::vector<uint8_t>& reach)
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
        reach[i] = 1;
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
    // nodes reachable from the root: only they are validated, so only they are read below (an
    // unreachable node may hold any offset; the reference never visits it either)
    std::vector<uint8_t> reach(node_count, 0);
    int rc = validate_scene(ctx, nodes, node_count, prims, prim_count, maxDepth, reach);
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
        else if (count > 255 && reach[i]) cbOk = false;
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
        if (!reach[i]) {
            firstPrim[i] = lastPrim[i] = 0;
        } else if (count) {
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
        if (rec[i] == 0xffffffffu || !reach[i]) continue;   // an unreachable record stays zero
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
// `tiles` 8x8 tiles on a chip with `resident` wave slots is grouped when six work items per slot
// would take at least 4 groups (under ~1.5 tiles per slot; with more, the cost-sorted list schedule
// balances well enough), and then gets 3.5 items per slot, at least 4 groups, at most 8, each at
// least 64 samples long.  Measured at six waves per SIMD (profiles/r05_six_waves.json, C3 rank-0
// shares): N = 4 G = 4 / 5 / 6 / 8 78.4 / 79.5 / 80.6 / 83.7 ms; N = 8 G = 4 / 5 / 6 / 8 46.8 / 44.5 /
// 44.5 / 46.0 ms (the six-items rule gave 5 and 8).
static uint32_t ssg_groups(const pt_context* ctx, int variant, uint32_t tiles, uint32_t total)
{
    if (ctx->ssgMode == 1 || !(variant == 39 || strip_capable(variant))) return 0;
    if (ctx->ssgMode >= 2) return std::min<uint32_t>((uint32_t)ctx->ssgMode, std::max(total, 1u));
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess) return 0;
    const uint64_t resident = (uint64_t)cus * 4 * variant_waves(variant);
    // measured (tools/ssg_probe.py): with 2 or 3 groups the logging, the fold and the
    // extra samples cost more than the shorter tail returns; from 4 groups on the tail wins
    if ((6 * resident + tiles - 1) / tiles < 4) return 0;
    uint64_t g = std::max<uint64_t>(4, (7 * resident + 2 * (uint64_t)tiles - 1) / (2 * (uint64_t)tiles));
    g = std::min<uint64_t>({g, 8, total / 64});
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
    // Automatic run-ahead only where tiles wait for a wave slot: a grid that holds every tile in one
    // pass (cornell 512x512: 4,096 tiles, 5,120-6,144 slots) has no next tile for a finished lane's
    // wave to delay, and run-ahead measured neutral there (4.37-4.42 vs 4.35-4.36 ms)
    // while it keeps the small-grid build from running.
    bool aheadFits = true;
    if (ctx->aheadMode == 0 && aheadCapable) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) == hipSuccess)
            aheadFits = (uint64_t)tiles > (uint64_t)cus * 4 * variant_waves(pick_variant(ctx));
    }
    const bool aheadMake = aheadCapable && (ctx->aheadMode == 2 ||
        (launchSamples >= kAheadMinSamples && launchSamples <= kAheadMaxSamples && ctx->aheadMisses < 2 && aheadFits));
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
    P.prioDealt = ctx->prioMode == 0 && P.prio[0] != 0;
    if (ctx->traceTiles && stats && P.tileCost) {
        if (ctx->tileTrace && ctx->traceCap < tiles) {
            (void)hipFree(ctx->tileTrace);
            ctx->tileTrace = nullptr;
        }
        if (!ctx->tileTrace) {
            PT_HIP_CHECK(ctx, hipMalloc(&ctx->tileTrace, 2 * (size_t)tiles * sizeof(uint32_t)));
            ctx->traceCap = tiles;
        }
        P.tileTrace = ctx->tileTrace;
    }
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
    // (Round 3 sent grouped launches of at most one tile per wave slot to the undeferred walk, 39;
    // measured again on the C3 N = 8 share it costs 8-10 %: 52.9 ms against 47.1 (40) and 47.8-48.9
    // (60) with deferred shading, profiles/r05_six_waves.json.  Grouped launches keep the picked walk.)
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
        Q.prioDealt = 0;
        PT_HIP_CHECK(ctx, launch_variant<false>(variant, Q, ctx->stream));
        const int rs = sort_order(ctx, tiles, spp, K);
        if (rs != PT_OK) return rs;
        P.order = ctx->order;
        P.chunks = chunks - 1;
        P.ignoreFirst = 0;                               // the first call is done
        if (ctx->coldPriority && ctx->prioMode == 0) {
            issue_priority(ctx, units, P.prio);
            P.prioDealt = 1;
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
        Q.prioDealt = 0;
        Q.pairsOut = guesses && ssg_reserve(ctx, tiles, 0, 0, 0) ? ctx->pairs : nullptr;
        if (Q.pairsOut) ctx->pairsValid = true;
        PT_HIP_CHECK(ctx, Q.pairsOut ? launch_grouped<2>(variant, Q, ctx->stream)
                                     : (K > 1 ? launch_strip(variant, Q, ctx->stream) : launch_variant<false>(variant, Q, ctx->stream)));
        const int rs = sort_order(ctx, tiles, Q.spp, K);
        if (rs != PT_OK) return rs;
        P.order = ctx->order;
        if (ctx->coldPriority && ctx->prioMode == 0) {
            issue_priority(ctx, units, P.prio);
            P.prioDealt = 1;
            biasedOrder = true;
        }
    }
    if (G && P.tileCost) PT_HIP_CHECK(ctx, hipMemsetAsync(P.tileCost, 0, (size_t)tiles * sizeof(uint32_t), ctx->stream));
    if (G) {
        P.prioDealt = 0;           // (grouped positions are (tile, group) items: measured slower with it)
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

PT_API int pt_set_tile_trace(pt_context* ctx, int enabled)
{
    if (!ctx) return PT_ERR_ARG;
    ctx->traceTiles = enabled != 0;
    return PT_OK;
}

PT_API int pt_read_tile_trace(pt_context* ctx, uint32_t* dst, uint32_t count)
{
    if (!ctx || !dst) return PT_ERR_ARG;
    if (!ctx->tileTrace || count != 2 * ctx->orderTiles || ctx->traceCap < ctx->orderTiles)
        return fail(ctx, PT_ERR_STATE, "pt_read_tile_trace: no traced launch of that size");
    PT_HIP_CHECK(ctx, hipSetDevice(ctx->device));
    PT_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));
    PT_HIP_CHECK(ctx, hipMemcpy(dst, ctx->tileTrace, (size_t)count * sizeof(uint32_t), hipMemcpyDeviceToHost));
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

#include "pt_group.h"
