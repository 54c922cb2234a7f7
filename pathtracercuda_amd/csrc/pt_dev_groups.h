// Speculative sample groups, lane side: item start states, logs and junctions.
// Part of the trace kernel's single translation unit: included by pt_kernels.hip inside its anonymous
// namespace, in this order: pt_dev_scene.h, pt_dev_walk.h, pt_dev_path.h, pt_dev_groups.h,
// pt_dev_fold.h; not a standalone header.
#pragma once

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
