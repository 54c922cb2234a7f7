// The child-box BVH walks (traverse_cb, the resumable traverse_cb_phase) and the rebuild of the
// pending set after a rising t_max (repair_pending).
// Part of the trace kernel's single translation unit: included by pt_kernels.hip inside its anonymous
// namespace, in this order: pt_dev_scene.h, pt_dev_walk.h, pt_dev_path.h, pt_dev_groups.h,
// pt_dev_fold.h; not a standalone header.
#pragma once

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

// The one-pass child-box walk (variant 20: counts the reference's node and primitive tests).
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

// The resumable walk's control flow (round 6).  Round 5's form left the interior loop by reaching a
// leaf OR by an empty pop (`return true` from inside the pop loop), and the phase loop by four
// breaks; each extra exit is an exec mask the structurizer keeps and updates with scalar
// instructions on every iteration (~26 SALU against ~40 VALU per interior visit in the ISA of
// variant 60).  Here the end of the traversal is a node word, kWalkDone, that no leaf or record can
// have (a leaf word with 255 primitives at offset 2^24 - 1 would end past any scene, pt_set_scene
// caps both), so every loop has one exit condition, a property of `cur` (~15 SALU per visit).  The
// per-lane sequence of node tests, stack operations, leaf tests and repairs is unchanged.
// Measured same-box (profiles/r06_single_exit_ab.json): C3 221.7 -> 211.7 ms (variant 60), the C4
// N = 8 rank-2 share 486.8 -> 454.4 ms (variant 40).
//
// The interior walk (trace.cu:66-77 per visited node) descends until a leaf is reached or the stack
// holds no entry that passes its re-test (cur = kWalkDone).  ALLFAST (wave-uniform, decided by the
// caller) drops the per-lane exact-form branch of the slab test, and the far child is written to the
// stack unconditionally -- the slot above the top, inside the lane's column since an interior node
// has at most depth - 2 pending entries -- with the stack pointer advanced only when the far child
// is to be kept (ChildPair).
constexpr uint32_t kWalkDone = 0xffffffffu;

template <bool STATS, bool ALLFAST>
PT_DEV void walk_interior(const float4* __restrict__ cnodes, uint2* stack, const SlabRay& R, uint32_t negMask,
                          float tMin, float tMax, uint32_t& cur, uint32_t& sp, Counters& cnt)
{
    while ((cur >> 24) == 0u) {                       // interior record (kWalkDone >> 24 == 255)
        if (STATS) { cnt.node_tests += 2; wave_tick(cnt.w_node); }
        const ChildPair ch = cb_children<ALLFAST>(cnodes, cur, R, negMask, tMin, tMax);
        stack[64u * sp] = make_uint2(ch.wF, __float_as_uint(ch.loF));
        sp += ch.push ? 1u : 0u;
        cur = ch.any ? ch.wNext : kWalkDone;
        if (!ch.any) {                                // pop the next far child still hit at t_max
            bool more = sp > 0;
            while (more) {
                const uint2 e = stack[64u * (--sp)];
                const bool pass = tMax > __uint_as_float(e.y);
                cur = pass ? e.x : cur;
                more = !pass && sp > 0;
            }
        }
    }
}

// WW = 200 + EXITQ selects this traversal (the wave leaves it once at most EXITQ/64 of the lanes
// that entered still walk, see above).  NOREPAIR (a test-only instantiation, pt_set_rise_repair)
// skips repair_pending: the negative control that shows a scene exercises it.
template <bool STATS, int EXITQ, bool NOREPAIR = false>
PT_DEV bool traverse_cb_phase(const float4* __restrict__ cnodes, const float4* __restrict__ prims, uint2* stack,
                              const TraceParams& P, f3 o, f3 d, bool fresh, TravState& ts, Counters& cnt)
{
    const float tMin = 0.001f;
    SlabRay R;
    R.o = o;
    // The three reciprocals behind ONE wave-uniform guard: the fast sequences for every lane, the
    // general 1/x for the wave only when some lane has a component outside [2^-125, 2^125] (an
    // axis-aligned direction); the values are rcp_rn's.  Three divergent guards cost the scalar unit
    // an exec-mask save, flip and restore each, on every phase entry (same-box: C3 -0.4 %, the C4
    // N = 8 share -0.4 %, profiles/r06_shading_ab.json).
    R.ix = rcp_fast(d.x);
    R.iy = rcp_fast(d.y);
    R.iz = rcp_fast(d.z);
    {
        const float ax = __builtin_fabsf(d.x), ay = __builtin_fabsf(d.y), az = __builtin_fabsf(d.z);
        const bool ok = ax >= 0x1p-125f && ax <= 0x1p125f && ay >= 0x1p-125f && ay <= 0x1p125f &&
                        az >= 0x1p-125f && az <= 0x1p125f;
        if (__ballot(!ok) != 0ull) {
            const float gx = 1.0f / d.x, gy = 1.0f / d.y, gz = 1.0f / d.z;
            R.ix = ok ? R.ix : gx;
            R.iy = ok ? R.iy : gy;
            R.iz = ok ? R.iz : gz;
        }
    }
    R.fast = P.slabFast && __builtin_isfinite(R.ix) && __builtin_isfinite(R.iy) && __builtin_isfinite(R.iz);
    R.ox2 = f2(o.x, o.x);
    R.oy2 = f2(o.y, o.y);
    R.oz2 = f2(o.z, o.z);
    R.ix2 = f2(R.ix, R.ix);
    R.iy2 = f2(R.iy, R.iy);
    R.iz2 = f2(R.iz, R.iz);
    const uint32_t negMask = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
    const uint32_t nAct = (uint32_t)__popcll(__ballot(1));
    if (fresh) {
        ts.tMax = kFltMax;
        ts.sp = 0;
        ts.elem = 0xffffffffu;
        if (STATS) { cnt.node_tests++; wave_tick(cnt.w_node); }
        float X;
        const float lo0 = slab_lo_x(R, f2(P.rootBox[0], P.rootBox[1]), f2(P.rootBox[2], P.rootBox[3]),
                                    f2(P.rootBox[4], P.rootBox[5]), tMin, X);
        ts.cur = (X > lo0 && ts.tMax > lo0) ? P.rootWord : kWalkDone;
    }
    uint32_t sp = ts.sp, cur = ts.cur, elem = ts.elem;
    float tMax = ts.tMax;
    uint64_t tPhase = STATS ? __builtin_amdgcn_s_memtime() : 0;
    const bool allFast = __ballot(!R.fast) == 0;                         // wave-uniform
    bool go = cur != kWalkDone;
    while (go) {
        if (allFast) walk_interior<STATS, true>(cnodes, stack, R, negMask, tMin, tMax, cur, sp, cnt);
        else walk_interior<STATS, false>(cnodes, stack, R, negMask, tMin, tMax, cur, sp, cnt);
        if (STATS) wave_time(cnt.cyc_node, tPhase);
        if (cur != kWalkDone) {                       // a leaf: in-order tests, repair, next pop
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
            // t_max ended the leaf above where it started (the sphere's far-root quirk, ChildPair):
            // boxes dropped for failing an earlier, smaller t_max may pass now.  (A rise undone within
            // the leaf needs nothing: every dropped box failed a t_max at least as large as the one left.)
            const bool rose = tMax > tLeaf;
            if (!NOREPAIR && __ballot(rose) != 0ull && rose) {     // rare: a uniform test first
                repair_pending(cnodes, stack, R, negMask, tMin, P.rootWord, leaf0, sp);
                if (STATS) cnt.repairs++;
            }
            if (STATS) wave_time(cnt.cyc_leaf, tPhase);
            cur = kWalkDone;
            bool more = sp > 0;
            while (more) {
                const uint2 e = stack[64u * (--sp)];
                const bool pass = tMax > __uint_as_float(e.y);
                cur = pass ? e.x : cur;
                more = !pass && sp > 0;
            }
        }
        // early exit once at most EXITQ/64 of the lanes that entered are still walking
        const bool walking = cur != kWalkDone;
        go = walking && (uint32_t)__popcll(__ballot(walking)) * 64u > nAct * (uint32_t)EXITQ;
    }
    ts.sp = sp;
    ts.cur = cur;
    ts.elem = elem;
    ts.tMax = tMax;
    return cur == kWalkDone;
}
