// Shading, the per-lane path state, pixel load/store, the render() call fold and the run-ahead
// stash.
// Part of the trace kernel's single translation unit: included by pt_kernels.hip inside its anonymous
// namespace, in this order: pt_dev_scene.h, pt_dev_walk.h, pt_dev_path.h, pt_dev_groups.h,
// pt_dev_fold.h; not a standalone header.
#pragma once

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
        n = normalize_dom(lp);                              // a point on the unit sphere
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
    t = normalize_dom(cross(up, N));           // N unit, |up . N| < 0.999 or up = x: |up x N|^2 >= 0.001
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
    // sqrt_dom: |t1| = |r c| <= 1, so 1 - t1^2 is +0 or >= 2^-24; (1 - t1^2) - t2^2 is NaN (t2 NaN),
    // <= 0 (clamped to +0) or >= 2^-48 (exact difference of floats >= 2^-25 where they are close)
    t2 = (1.0f - sv) * sqrt_dom(1.0f - t1 * t1) + sv * t2;
    const f3 Nh = add(add(scale(t1, T1), scale(t2, T2)), scale(sqrt_dom(clamp01(1.0f - t1 * t1 - t2 * t2)), Vh));
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
    // brdf.h:18-24.  NdotV = |V.z| + 1e-5, so the first operand, NdotV^2 (1 - a2) + a2 with a2 in
    // [0, 1], is NaN or >= 1e-10 (sqrt_dom); NdotL may be any value in [0, 1], so the second keeps
    // the guarded root
    const float sv = sqrt_dom((-NdotV * a2 + NdotV) * NdotV + a2);
    const float sl = sqrt_rn((-NdotL * a2 + NdotL) * NdotL + a2);
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
    // (normalize_dom: a unit vector in the orthonormal frame (tg, bt, n))
    const f3 V = normalize_dom(add(add(scale(wo.x, mk(tg.x, bt.x, sf.n.x)), scale(wo.y, mk(tg.y, bt.y, sf.n.y))),
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
    // sqrt of the lobe's radius uniform and the cosine lobe's sin(theta) with no range guard
    // (sqrt_dom): uniforms lie in [2^-33, 1], LAMBERT_GGX's 2 (u - 0.5) is +0 or >= 2^-23, and 1 - u is
    // +0 or >= 2^-25
    const float sq = sqrt_dom(specular ? rnd0 : rnd1);
    const float sinTheta = sqrt_dom(1.0f - rnd1);
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
    // Material.inl:57: normalize(tangentToWorld(...)), which itself normalizes (normalize_dom: the
    // sampled direction is a unit vector -- cosine sample or mirror of the unit V -- in the frame)
    const f3 sd = normalize_dom(normalize_dom(add(add(scale(dir.x, tg), scale(dir.y, bt)), scale(dir.z, sf.n))));
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
