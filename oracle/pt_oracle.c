/*
 * pt_oracle.c -- TEST INFRASTRUCTURE ONLY.  Never linked into, imported by or called from the
 * product path (pathtracercuda_amd/, include/).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it, and only as the checker / the timed CPU baseline.
 *
 * A plain-C restatement of the hot path of DoerriesT/PathtracerCUDA (reference @ /root/reference,
 * paths below are relative to PathtracerCUDA/src/).  Every function follows the cited reference
 * function in exact floating-point operation order (no FMA contraction: build with
 * -ffp-contract=off), so the HIP megakernel can be compared with it bit for bit.
 *
 * PARITY STATUS vs the original CUDA binary: UNPINNED.  The reference has no tests, golden vectors
 * or KATs; compiling/executing the reference's own sources in this container
 * was refused (binding).  Three third-party behaviours are restated, not pinned:
 *   - cuRAND XORWOW (curand_init / curand_uniform, CUDA 10.2);
 *   - CUDA libdevice acosf/atan2f/sinf/cosf/powf: replaced by the Cephes-style single-precision
 *     routines below (the HIP kernel implements the same routines);
 *   - CUDA texture-unit bilinear filtering: the fixed rule of SURVEY.md Appendix C (weights
 *     quantised to 1/256, round-to-nearest), implemented identically on the GPU.
 * The oracle is pinned statistically against the reference's own published render
 * (cornell_box_4096spp.png block means, tests/golden/) and by analytic known-answer tests.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <float.h>
#include <limits.h>
#include <pthread.h>

#define OR_EXPORT __attribute__((visibility("default")))

/* vec3.h:5 */
#define PI_F 3.14159265358979323846f

/* ------------------------------------------------------------------------------------------ */
/* float bit helpers                                                                           */
/* ------------------------------------------------------------------------------------------ */
static inline uint32_t f_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float bits_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* float -> int32 with x86 cvttss2si semantics (NaN / out of range -> INT_MIN), as an MSVC or gcc
 * x86 build of the reference's int(float) casts behaves (BVH.cpp:114,183). */
static inline int32_t f2i_x86(float f)
{
    if (!(f > -2147483904.0f && f < 2147483648.0f)) return INT32_MIN;
    return (int32_t)f;
}

/* ------------------------------------------------------------------------------------------ */
/* vec3 (vec3.h:7-57, vec3.inl)                                                                */
/* ------------------------------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;

static inline v3 V(float x, float y, float z) { v3 r = { x, y, z }; return r; }
static inline v3 Vs(float s) { return V(s, s, s); }
static inline float v3_get(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
static inline v3 v3_neg(v3 a) { return V(-a.x, -a.y, -a.z); }                         /* :79-82 */
static inline v3 v3_add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }    /* :126-129 */
static inline v3 v3_adds(v3 a, float s) { return V(a.x + s, a.y + s, a.z + s); }      /* :131-134 */
static inline v3 v3_sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }    /* :141-144 */
static inline v3 v3_mul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }    /* :156-159 */
static inline v3 v3_scale(float t, v3 v) { return V(t * v.x, t * v.y, t * v.z); }     /* :161-169 */
static inline v3 v3_divs(v3 v, float t) { return v3_scale(1.0f / t, v); }           /* :176-179 */
static inline v3 v3_divv(v3 v, v3 t) { return v3_mul(V(1.0f / t.x, 1.0f / t.y, 1.0f / t.z), v); } /* :171-174 */
static inline int v3_eq(v3 a, v3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; } /* :186-189 */
static inline float v3_dot(v3 u, v3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }  /* :191-196 */
static inline v3 v3_cross(v3 u, v3 v)                                                  /* :198-203 */
{
    return V(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
static inline float v3_length(v3 v) { return sqrtf(v.x * v.x + v.y * v.y + v.z * v.z); } /* :205-213 */
static inline v3 v3_min(v3 a, v3 b)                                                    /* :215-222 */
{
    return V(a.x < b.x ? a.x : b.x, a.y < b.y ? a.y : b.y, a.z < b.z ? a.z : b.z);
}
static inline v3 v3_max(v3 a, v3 b)                                                    /* :224-231 */
{
    return V(a.x >= b.x ? a.x : b.x, a.y >= b.y ? a.y : b.y, a.z >= b.z ? a.z : b.z);
}
static inline v3 v3_normalize(v3 v) { return v3_divs(v, v3_length(v)); }               /* :233-236 */
static inline v3 v3_reflect(v3 v, v3 n) { return v3_sub(v, v3_scale(2.0f * v3_dot(v, n), n)); } /* :238-241 */
static inline v3 v3_lerp(v3 x, v3 y, float a)                                          /* :261-264 */
{
    return v3_add(v3_scale(1.0f - a, x), v3_scale(a, y));
}
static inline float clampf01(float x)                                                  /* :271-276 */
{
    x = x < 0.0f ? 0.0f : x;
    x = x > 1.0f ? 1.0f : x;
    return x;
}

/* ------------------------------------------------------------------------------------------ */
/* Single-precision transcendentals (stand-ins for CUDA libdevice; identical in the HIP kernel) */
/* Cephes-style argument reduction + minimax polynomials, evaluated without FMA.               */
/* ------------------------------------------------------------------------------------------ */
#define PM_FOPI 1.27323954473516f
#define PM_DP1 0.78515625f
#define PM_DP2 2.4187564849853515625e-4f
#define PM_DP3 3.77489497744594108e-8f
#define PM_PIO2 1.5707963267948966192f
#define PM_PIO4 0.7853981633974483096f

static inline float pm_sin_poly(float z, float zz)
{
    return ((-1.9515295891E-4f * zz + 8.3321608736E-3f) * zz - 1.6666654611E-1f) * zz * z + z;
}
static inline float pm_cos_poly(float zz)
{
    float y = ((2.443315711809948E-5f * zz - 1.388731625493765E-3f) * zz + 4.166664568298827E-2f) * zz * zz;
    y = y - 0.5f * zz;
    return y + 1.0f;
}

OR_EXPORT float pm_sinf(float xx)
{
    int neg = xx < 0.0f;
    float x = fabsf(xx);
    if (!(x <= 65536.0f)) return (x != x) ? x : (xx - xx); /* NaN / huge: not reached on the path */
    int32_t j = (int32_t)(x * PM_FOPI);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    if (j > 3) { neg = !neg; j -= 4; }
    float z = ((x - y * PM_DP1) - y * PM_DP2) - y * PM_DP3;
    float zz = z * z;
    float r = (j == 1 || j == 2) ? pm_cos_poly(zz) : pm_sin_poly(z, zz);
    return neg ? -r : r;
}

OR_EXPORT float pm_cosf(float xx)
{
    int neg = 0;
    float x = fabsf(xx);
    if (!(x <= 65536.0f)) return (x != x) ? x : (xx - xx);
    int32_t j = (int32_t)(x * PM_FOPI);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    if (j > 3) { j -= 4; neg = !neg; }
    if (j > 1) neg = !neg;
    float z = ((x - y * PM_DP1) - y * PM_DP2) - y * PM_DP3;
    float zz = z * z;
    float r = (j == 1 || j == 2) ? pm_sin_poly(z, zz) : pm_cos_poly(zz);
    return neg ? -r : r;
}

static inline float pm_asin_core(float a /* |x| <= 1 */)
{
    float x, z;
    int flag;
    if (a > 0.5f) { z = 0.5f * (1.0f - a); x = sqrtf(z); flag = 1; }
    else { x = a; z = x * x; flag = 0; }
    float r;
    if (a < 1.0e-4f) r = a;
    else r = ((((4.2163199048E-2f * z + 2.4181311049E-2f) * z + 4.5470025998E-2f) * z + 7.4953002686E-2f) * z + 1.6666752422E-1f) * z * x + x;
    if (flag) { r = r + r; r = PM_PIO2 - r; }
    return r;
}

OR_EXPORT float pm_acosf(float x)
{
    if (!(x >= -1.0f && x <= 1.0f)) return (x != x) ? x : bits_f(0x7fc00000u);
    if (x < -0.5f) return PI_F - 2.0f * pm_asin_core(sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * pm_asin_core(sqrtf(0.5f * (1.0f - x)));
    float r = pm_asin_core(fabsf(x));
    return x < 0.0f ? PM_PIO2 + r : PM_PIO2 - r;
}

static inline float pm_atan_pos(float x /* >= 0, finite or inf */)
{
    float y, z;
    if (x > 2.414213562373095f) { y = PM_PIO2; x = -1.0f / x; }
    else if (x > 0.4142135623730950f) { y = PM_PIO4; x = (x - 1.0f) / (x + 1.0f); }
    else y = 0.0f;
    z = x * x;
    y = y + ((((8.05374449538e-2f * z - 1.38776856032E-1f) * z + 1.99777106478E-1f) * z - 3.33329491539E-1f) * z * x + x);
    return y;
}

OR_EXPORT float pm_atan2f(float y, float x)
{
    if (x != x || y != y) return x + y;
    if (y == 0.0f) {
        if (f_bits(x) >> 31) return (f_bits(y) >> 31) ? -PI_F : PI_F; /* x < 0 or x == -0 */
        return y;                                                    /* +-0 */
    }
    if (x == 0.0f) return y < 0.0f ? -PM_PIO2 : PM_PIO2;
    float ay = fabsf(y), ax = fabsf(x);
    if (isinf(ax)) {
        float r;
        if (isinf(ay)) r = (x > 0.0f) ? PM_PIO4 : 3.0f * PM_PIO4;
        else r = (x > 0.0f) ? 0.0f : PI_F;
        return y < 0.0f ? -r : r;
    }
    float r = pm_atan_pos(ay / ax);
    if (x < 0.0f) r = PI_F - r;
    return y < 0.0f ? -r : r;
}

/* natural log for x > 0 finite (Cephes logf) */
static inline float pm_logf(float x)
{
    uint32_t b = f_bits(x);
    int32_t e = 0;
    if ((b >> 23) == 0) { x = x * 8388608.0f; b = f_bits(x); e = -23; } /* denormal */
    e += (int32_t)((b >> 23) & 0xffu) - 126;
    x = bits_f((b & 0x807fffffu) | 0x3f000000u); /* [0.5, 1) */
    if (x < 0.707106781186547524f) { e -= 1; x = x + x - 1.0f; }
    else x = x - 1.0f;
    float z = x * x;
    float y = ((((((((7.0376836292E-2f * x - 1.1514610310E-1f) * x + 1.1676998740E-1f) * x - 1.2420140846E-1f) * x
                   + 1.4249322787E-1f) * x - 1.6668057665E-1f) * x + 2.0000714765E-1f) * x - 2.4999993993E-1f) * x
              + 3.3333331174E-1f) * x * z;
    float fe = (float)e;
    y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    z = x + y;
    z = z + 0.693359375f * fe;
    return z;
}

/* exp for finite x (Cephes expf); result scaled exactly by powers of two */
static inline float pm_expf(float x)
{
    if (x > 88.7228391f) return bits_f(0x7f800000u);
    if (x < -103.972084f) return 0.0f;
    float z = floorf(1.44269504088896341f * x + 0.5f);
    x = x - z * 0.693359375f;
    x = x - z * -2.12194440e-4f;
    int32_t n = (int32_t)z;
    z = x * x;
    float r = ((((( 1.9875691500E-4f * x + 1.3981999507E-3f) * x + 8.3334519073E-3f) * x + 4.1665795894E-2f) * x
               + 1.6666665459E-1f) * x + 5.0000001201E-1f) * z + x + 1.0f;
    /* r * 2^n in two exact steps */
    int32_t n1 = n / 2, n2 = n - n1;
    r = r * bits_f((uint32_t)(n1 + 127) << 23);
    r = r * bits_f((uint32_t)(n2 + 127) << 23);
    return r;
}

/* pow for the two uses on the path: tonemap.cu:19-21 (x in [0,1], y = 1/2.2) and
 * Material.inl:30-32 (texel in [0,1], y = 2.2). */
OR_EXPORT float pm_powf(float x, float y)
{
    if (x != x || y != y) return x + y;
    if (y == 0.0f || x == 1.0f) return 1.0f;
    if (x == 0.0f) return y > 0.0f ? 0.0f : bits_f(0x7f800000u);
    if (x < 0.0f) return bits_f(0x7fc00000u);
    if (isinf(x)) return y > 0.0f ? x : 0.0f;
    return pm_expf(y * pm_logf(x));
}

/* ------------------------------------------------------------------------------------------ */
/* cuRAND XORWOW as used (initRandState.cu:16, trace.cu:190-191,         */
/* Material.inl:40-41)                                                                          */
/* ------------------------------------------------------------------------------------------ */
typedef struct { uint32_t d, v[5]; } xorwow_t; /* the 24 B of curandState that are used */

OR_EXPORT void or_xorwow_init(uint64_t seed, xorwow_t *s)
{
    uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    s->d = 6615241u + t1 + t0;
    s->v[0] = 123456789u + t0;
    s->v[1] = 362436069u ^ t0;
    s->v[2] = 521288629u + t1;
    s->v[3] = 88675123u ^ t1;
    s->v[4] = 5783321u + t0;
}

static inline uint32_t xorwow_next(xorwow_t *s)
{
    uint32_t t = s->v[0] ^ (s->v[0] >> 2);
    s->v[0] = s->v[1];
    s->v[1] = s->v[2];
    s->v[2] = s->v[3];
    s->v[3] = s->v[4];
    s->v[4] = (s->v[4] ^ (s->v[4] << 4)) ^ (t ^ (t << 1));
    s->d += 362437u;
    return s->v[4] + s->d;
}

static inline float xorwow_uniform(xorwow_t *s)
{
    return (float)xorwow_next(s) * 2.3283064e-10f + (2.3283064e-10f / 2.0f);
}

OR_EXPORT uint32_t or_xorwow_next(xorwow_t *s) { return xorwow_next(s); }
OR_EXPORT float or_xorwow_uniform(xorwow_t *s) { return xorwow_uniform(s); }

/* ------------------------------------------------------------------------------------------ */
/* Scene records                                                                               */
/* ------------------------------------------------------------------------------------------ */
enum { SPHERE = 0, CYLINDER, DISK, CONE, PARABOLOID, QUAD, CUBE };   /* Hittable.h:9-12 */
enum { LAMBERT = 0, GGX, LAMBERT_GGX };                               /* Material.h:9-12 */

typedef struct {            /* Material.h:22-27 (40 B) */
    v3 baseColor;
    float roughness;
    v3 emissive;
    float metalness;
    uint32_t textureIndex;
    uint32_t materialType;
} or_material;

typedef struct {            /* Hittable.h:23-27 (96 B) */
    float rows[3][4];
    or_material mat;
    uint32_t type;
    uint32_t pad;
} or_hittable;

typedef struct {            /* Hittable.h:50-55 */
    float rows[3][4];
    or_material mat;
    v3 aabbMin, aabbMax;
    uint32_t type;
} or_cpu_hittable;

typedef struct {            /* BVH.h:6-11 (32 B) */
    v3 bmin, bmax;
    uint32_t offset;
    uint32_t primitiveCountAxis;
} or_bvh_node;

typedef struct {            /* Camera.h:14-22 (92 B) */
    float tanHalfFovy, aspectRatio;
    v3 origin, lowerLeftCorner, horizontal, vertical, right, up, backward;
} or_camera;

typedef struct {
    uint32_t width, height;
    const float *texels;    /* RGBA f32, row-major, row 0 = first row of the image file */
} or_texture;

/* Material ctor (Material.inl:9-18): roughness clamp */
OR_EXPORT void or_material_make(uint32_t type, const float *baseColor, const float *emissive, float roughness,
                                float metalness, uint32_t textureIndex, or_material *m)
{
    m->baseColor = V(baseColor[0], baseColor[1], baseColor[2]);
    m->emissive = V(emissive[0], emissive[1], emissive[2]);
    m->roughness = roughness < 0.04f ? 0.04f : roughness;
    m->metalness = metalness;
    m->textureIndex = textureIndex;
    m->materialType = type;
}

/* SceneLoader.cpp:193-196 */
OR_EXPORT float or_radians(float degree) { return degree * (1.0f / 180.0f) * 3.14159265358979323846f; }

/* Hittable.cpp:6-103 worldTransform */
static void world_transform(v3 position, v3 rotation, v3 scale, float l2w[3][4], float w2l[3][4])
{
    float q[4]; /* x y z w */
    {
        v3 c = V(cosf(rotation.x * 0.5f), cosf(rotation.y * 0.5f), cosf(rotation.z * 0.5f));
        v3 s = V(sinf(rotation.x * 0.5f), sinf(rotation.y * 0.5f), sinf(rotation.z * 0.5f));
        q[3] = c.x * c.y * c.z + s.x * s.y * s.z;
        q[0] = s.x * c.y * c.z - c.x * s.y * s.z;
        q[1] = c.x * s.y * c.z + s.x * c.y * s.z;
        q[2] = c.x * c.y * s.z - s.x * s.y * c.z;
    }
    float iq[4];
    {
        float invDot = (1.0f / (q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]));
        iq[0] = -q[0] * invDot;
        iq[1] = -q[1] * invDot;
        iq[2] = -q[2] * invDot;
        iq[3] = q[3] * invDot;
    }
#define QUAT_TO_ROT(Q, M)                                                     \
    do {                                                                      \
        float qxx = Q[0] * Q[0], qyy = Q[1] * Q[1], qzz = Q[2] * Q[2];        \
        float qxz = Q[0] * Q[2], qxy = Q[0] * Q[1], qyz = Q[1] * Q[2];        \
        float qwx = Q[3] * Q[0], qwy = Q[3] * Q[1], qwz = Q[3] * Q[2];        \
        M[0][0] = 1.0f - 2.0f * (qyy + qzz);                                  \
        M[0][1] = 2.0f * (qxy + qwz);                                         \
        M[0][2] = 2.0f * (qxz - qwy);                                         \
        M[1][0] = 2.0f * (qxy - qwz);                                         \
        M[1][1] = 1.0f - 2.0f * (qxx + qzz);                                  \
        M[1][2] = 2.0f * (qyz + qwx);                                         \
        M[2][0] = 2.0f * (qxz + qwy);                                         \
        M[2][1] = 2.0f * (qyz - qwx);                                         \
        M[2][2] = 1.0f - 2.0f * (qxx + qyy);                                  \
    } while (0)
    {
        float ir[3][3];
        QUAT_TO_ROT(iq, ir);
        v3 is = v3_mul(V(1.0f / scale.x, 1.0f / scale.y, 1.0f / scale.z), Vs(1.0f)); /* 1.0f / scale */
        v3 np = v3_neg(position);
        for (int k = 0; k < 3; ++k) {
            float sk = v3_get(is, k);
            w2l[k][0] = sk * ir[0][k];
            w2l[k][1] = sk * ir[1][k];
            w2l[k][2] = sk * ir[2][k];
            w2l[k][3] = sk * v3_dot(V(ir[0][k], ir[1][k], ir[2][k]), np);
        }
    }
    {
        float r[3][3];
        QUAT_TO_ROT(q, r);
        float pos[3] = { position.x, position.y, position.z };
        for (int k = 0; k < 3; ++k) {
            l2w[k][0] = scale.x * r[0][k];
            l2w[k][1] = scale.y * r[1][k];
            l2w[k][2] = scale.z * r[2][k];
            l2w[k][3] = pos[k];
        }
    }
#undef QUAT_TO_ROT
}

/* CpuHittable ctor (Hittable.cpp:115-179); rotation in radians */
OR_EXPORT void or_cpu_hittable_make(uint32_t type, const float *position, const float *rotation, const float *scale,
                                    const or_material *mat, or_cpu_hittable *h)
{
    memset(h, 0, sizeof(*h));
    h->mat = *mat;
    h->type = type;
    v3 adj = V(scale[0], scale[1], scale[2]);
    if (type == DISK || type == QUAD) adj.y = 1.0f;
    float w2l[3][4], l2w[3][4];
    world_transform(V(position[0], position[1], position[2]), V(rotation[0], rotation[1], rotation[2]), adj, l2w, w2l);
    memcpy(h->rows, w2l, sizeof(w2l));

    v3 mn = Vs(FLT_MAX), mx = Vs(-FLT_MAX);
    float xe[2] = { -1.0f, 1.0f }, ye[2] = { -1.0f, 1.0f }, ze[2] = { -1.0f, 1.0f };
    if (type == DISK || type == QUAD) { ye[0] = -0.01f; ye[1] = 0.01f; }
    else if (type == PARABOLOID) { ye[0] = 0.0f; }
    for (int z = 0; z < 2; ++z)
        for (int y = 0; y < 2; ++y)
            for (int x = 0; x < 2; ++x) {
                v3 c = V(xe[x], ye[y], ze[z]);
                v3 p;
                p.x = v3_dot(c, V(l2w[0][0], l2w[0][1], l2w[0][2])) + l2w[0][3];
                p.y = v3_dot(c, V(l2w[1][0], l2w[1][1], l2w[1][2])) + l2w[1][3];
                p.z = v3_dot(c, V(l2w[2][0], l2w[2][1], l2w[2][2])) + l2w[2][3];
                mn = v3_min(mn, p);
                mx = v3_max(mx, p);
            }
    h->aabbMin = mn;
    h->aabbMax = mx;
}

/* getGpuHittable (Hittable.cpp:186-190) */
OR_EXPORT void or_gpu_hittable(const or_cpu_hittable *c, or_hittable *g)
{
    memset(g, 0, sizeof(*g));
    memcpy(g->rows, c->rows, sizeof(g->rows));
    g->mat = c->mat;
    g->type = c->type;
}

/* Camera ctor + update (Camera.inl:4-23, 54-62); fovy in radians */
OR_EXPORT void or_camera_make(const float *position, const float *lookat, const float *up, float fovy, float aspect,
                              or_camera *c)
{
    c->tanHalfFovy = tanf(fovy * 0.5f);
    c->aspectRatio = aspect;
    c->origin = V(position[0], position[1], position[2]);
    c->backward = v3_normalize(v3_sub(c->origin, V(lookat[0], lookat[1], lookat[2])));
    c->right = v3_normalize(v3_cross(V(up[0], up[1], up[2]), c->backward));
    c->up = v3_cross(c->backward, c->right);
    float hh = c->tanHalfFovy;
    float hw = c->aspectRatio * hh;
    c->lowerLeftCorner = v3_sub(v3_add(v3_scale(-hw, c->right), v3_scale(-hh, c->up)), c->backward);
    c->horizontal = v3_scale(2.0f * hw, c->right);
    c->vertical = v3_scale(2.0f * hh, c->up);
}

/* Camera::rotate / translate / update (Camera.inl:30-62), rotateAroundVector (vec3.inl:184-187) */
static v3 rotate_around(v3 v, v3 axis, float c, float s)
{
    return v3_add(v3_add(v3_scale(c, v), v3_scale(s, v3_cross(axis, v))),
                  v3_scale(1.0f - c, v3_scale(v3_dot(axis, v), axis)));
}

static void camera_update(or_camera *c)
{
    float hh = c->tanHalfFovy;
    float hw = c->aspectRatio * hh;
    c->lowerLeftCorner = v3_sub(v3_add(v3_scale(-hw, c->right), v3_scale(-hh, c->up)), c->backward);
    c->horizontal = v3_scale(2.0f * hw, c->right);
    c->vertical = v3_scale(2.0f * hh, c->up);
}

OR_EXPORT void or_camera_rotate(or_camera *c, float pitch, float yaw, float roll)
{
    (void)roll;
    const float cp = cosf(-pitch), sp = sinf(-pitch);
    c->up = rotate_around(c->up, c->right, cp, sp);
    c->backward = rotate_around(c->backward, c->right, cp, sp);
    const float cy = cosf(-yaw), sy = sinf(-yaw);
    const v3 Y = V(0.0f, 1.0f, 0.0f);
    c->right = rotate_around(c->right, Y, cy, sy);
    c->up = rotate_around(c->up, Y, cy, sy);
    c->backward = rotate_around(c->backward, Y, cy, sy);
    camera_update(c);
}

OR_EXPORT void or_camera_translate(or_camera *c, float x, float y, float z)
{
    c->origin = v3_add(c->origin, v3_add(v3_add(v3_scale(x, c->right), v3_scale(y, c->up)), v3_scale(z, c->backward)));
    camera_update(c);
}

/* ------------------------------------------------------------------------------------------ */
/* BVH build (BVH.cpp:5-15, 54-228) with libstdc++'s std::partition / std::nth_element        */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    or_cpu_hittable *e;
    or_bvh_node *nodes;
    uint32_t nodeCount;
    uint32_t maxLeaf;
} bvh_builder;

static float calc_surface_area(v3 mn, v3 mx) /* BVH.cpp:54-64 */
{
    v3 ext = v3_sub(mx, mn);
    if (ext.x <= 0.0f || ext.y <= 0.0f || ext.z <= 0.0f) return 0.0f;
    return (ext.x * ext.y + ext.x * ext.z + ext.y * ext.z) * 2.0f;
}

static inline v3 centroid_of(const or_cpu_hittable *h)
{
    return v3_scale(0.5f, v3_add(h->aabbMin, h->aabbMax));
}

static inline void swap_h(or_cpu_hittable *a, or_cpu_hittable *b)
{
    or_cpu_hittable t = *a; *a = *b; *b = t;
}

/* predicate of BVH.cpp:176-186 */
typedef struct { int axis; uint32_t bestBin; float nmin, ext; } part_pred;
static inline int pred_eval(const part_pred *p, const or_cpu_hittable *h)
{
    v3 c = centroid_of(h);
    float rel = ((v3_get(c, p->axis) - p->nmin) / p->ext);
    int32_t bin = f2i_x86(8.0f * rel);
    bin = bin < 0 ? 0 : bin > 7 ? 7 : bin;
    return (uint32_t)bin <= p->bestBin;
}

/* libstdc++ std::__partition, bidirectional form (also MSVC's algorithm) */
static or_cpu_hittable *std_partition(or_cpu_hittable *first, or_cpu_hittable *last, const part_pred *p)
{
    for (;;) {
        for (;;) {
            if (first == last) return first;
            if (pred_eval(p, first)) ++first;
            else break;
        }
        --last;
        for (;;) {
            if (first == last) return first;
            if (!pred_eval(p, last)) --last;
            else break;
        }
        swap_h(first, last);
        ++first;
    }
}

/* comparator of BVH.cpp:195-206 */
static inline int cmp_less(int axis, const or_cpu_hittable *a, const or_cpu_hittable *b)
{
    return v3_get(centroid_of(a), axis) < v3_get(centroid_of(b), axis);
}

/* libstdc++ heap helpers (for __heap_select when the introselect depth limit is hit) */
static void adjust_heap(or_cpu_hittable *first, ptrdiff_t hole, ptrdiff_t len, or_cpu_hittable value, int axis)
{
    const ptrdiff_t top = hole;
    ptrdiff_t child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (cmp_less(axis, &first[child], &first[child - 1])) child--;
        first[hole] = first[child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        first[hole] = first[child - 1];
        hole = child - 1;
    }
    /* __push_heap */
    ptrdiff_t parent = (hole - 1) / 2;
    while (hole > top && cmp_less(axis, &first[parent], &value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

static void make_heap(or_cpu_hittable *first, or_cpu_hittable *last, int axis)
{
    ptrdiff_t len = last - first;
    if (len < 2) return;
    ptrdiff_t parent = (len - 2) / 2;
    for (;;) {
        or_cpu_hittable value = first[parent];
        adjust_heap(first, parent, len, value, axis);
        if (parent == 0) return;
        parent--;
    }
}

static void heap_select(or_cpu_hittable *first, or_cpu_hittable *middle, or_cpu_hittable *last, int axis)
{
    make_heap(first, middle, axis);
    for (or_cpu_hittable *i = middle; i < last; ++i)
        if (cmp_less(axis, i, first)) {
            /* __pop_heap(first, middle, i) */
            or_cpu_hittable value = *i;
            *i = *first;
            adjust_heap(first, 0, middle - first, value, axis);
        }
}

static void move_median_to_first(or_cpu_hittable *result, or_cpu_hittable *a, or_cpu_hittable *b,
                                 or_cpu_hittable *c, int axis)
{
    if (cmp_less(axis, a, b)) {
        if (cmp_less(axis, b, c)) swap_h(result, b);
        else if (cmp_less(axis, a, c)) swap_h(result, c);
        else swap_h(result, a);
    } else if (cmp_less(axis, a, c)) swap_h(result, a);
    else if (cmp_less(axis, b, c)) swap_h(result, c);
    else swap_h(result, b);
}

static or_cpu_hittable *unguarded_partition(or_cpu_hittable *first, or_cpu_hittable *last,
                                            or_cpu_hittable *pivot, int axis)
{
    for (;;) {
        while (cmp_less(axis, first, pivot)) ++first;
        --last;
        while (cmp_less(axis, pivot, last)) --last;
        if (!(first < last)) return first;
        swap_h(first, last);
        ++first;
    }
}

static void insertion_sort(or_cpu_hittable *first, or_cpu_hittable *last, int axis)
{
    if (first == last) return;
    for (or_cpu_hittable *i = first + 1; i != last; ++i) {
        if (cmp_less(axis, i, first)) {
            or_cpu_hittable val = *i;
            memmove(first + 1, first, (size_t)(i - first) * sizeof(*first));
            *first = val;
        } else {
            or_cpu_hittable val = *i;
            or_cpu_hittable *l = i, *next = i - 1;
            while (cmp_less(axis, &val, next)) { *l = *next; l = next; --next; }
            *l = val;
        }
    }
}

static void std_nth_element(or_cpu_hittable *first, or_cpu_hittable *nth, or_cpu_hittable *last, int axis)
{
    if (first == last || nth == last) return;
    ptrdiff_t n = last - first;
    int lg = 63 - __builtin_clzll((unsigned long long)n);
    ptrdiff_t depth = (ptrdiff_t)lg * 2;
    while (last - first > 3) {
        if (depth == 0) {
            heap_select(first, nth + 1, last, axis);
            swap_h(first, nth);
            return;
        }
        --depth;
        or_cpu_hittable *mid = first + (last - first) / 2;
        move_median_to_first(first, first + 1, mid, last - 1, axis);
        or_cpu_hittable *cut = unguarded_partition(first + 1, last, first, axis);
        if (cut <= nth) first = cut;
        else last = cut;
    }
    insertion_sort(first, last, axis);
}

static uint32_t build_recursive(bvh_builder *b, size_t begin, size_t end) /* BVH.cpp:66-228 */
{
    uint32_t nodeIndex = b->nodeCount++;
    or_bvh_node node;
    memset(&node, 0, sizeof(node));
    node.bmin = Vs(FLT_MAX);
    node.bmax = Vs(-FLT_MAX);
    for (size_t i = begin; i < end; ++i) {
        node.bmin = v3_min(node.bmin, b->e[i].aabbMin);
        node.bmax = v3_max(node.bmax, b->e[i].aabbMax);
    }
    if ((end - begin) > b->maxLeaf) {
        struct { uint32_t count; v3 mn, mx; } bins[3][8];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 8; ++j) { bins[i][j].count = 0; bins[i][j].mn = Vs(FLT_MAX); bins[i][j].mx = Vs(-FLT_MAX); }
        const v3 ext = v3_max(v3_sub(node.bmax, node.bmin), Vs(0.00000001f));
        for (size_t i = begin; i < end; ++i) {
            const or_cpu_hittable *h = &b->e[i];
            v3 c = v3_scale(0.5f, v3_add(h->aabbMin, h->aabbMax));
            v3 rel = v3_divv(v3_sub(c, node.bmin), ext);
            for (int j = 0; j < 3; ++j) {
                int32_t bin = f2i_x86(v3_get(rel, j) * 8.0f);
                bin = bin < 0 ? 0 : bin > 7 ? 7 : bin;
                bins[j][bin].count += 1;
                bins[j][bin].mn = v3_min(bins[j][bin].mn, h->aabbMin);
                bins[j][bin].mx = v3_max(bins[j][bin].mx, h->aabbMax);
            }
        }
        float sa = calc_surface_area(node.bmin, node.bmax);
        const float invSA = 1.0f / ((sa < 0.000000001f) ? 0.000000001f : sa);
        float lowest = FLT_MAX;
        uint32_t bestAxis = 0, bestBin = 0;
        for (uint32_t i = 0; i < 3; ++i)
            for (uint32_t j = 0; j < 7; ++j) {
                v3 mn0 = Vs(FLT_MAX), mx0 = Vs(-FLT_MAX), mn1 = Vs(FLT_MAX), mx1 = Vs(-FLT_MAX);
                uint32_t c0 = 0, c1 = 0;
                for (uint32_t k = 0; k <= j; ++k) {
                    mn0 = v3_min(mn0, bins[i][k].mn); mx0 = v3_max(mx0, bins[i][k].mx); c0 += bins[i][k].count;
                }
                for (uint32_t k = j + 1; k < 8; ++k) {
                    mn1 = v3_min(mn1, bins[i][k].mn); mx1 = v3_max(mx1, bins[i][k].mx); c1 += bins[i][k].count;
                }
                float a0 = calc_surface_area(mn0, mx0);
                float a1 = calc_surface_area(mn1, mx1);
                float cost = 0.125f + ((float)c0 * a0 + (float)c1 * a1) * invSA;
                cost = (c0 == 0 || c1 == 0) ? FLT_MAX : cost;
                if (cost < lowest) { lowest = cost; bestAxis = i; bestBin = j; }
            }
        part_pred p = { (int)bestAxis, bestBin, v3_get(node.bmin, (int)bestAxis), v3_get(ext, (int)bestAxis) };
        or_cpu_hittable *mid = std_partition(b->e + begin, b->e + end, &p);
        size_t split = (size_t)(mid - b->e);
        if (split == begin || split == end) {
            bestAxis = (ext.x < ext.y) ? 0 : (ext.y < ext.z) ? 1 : 2;
            split = (begin + end) / 2;
            std_nth_element(b->e + begin, b->e + split, b->e + end, (int)bestAxis);
        }
        build_recursive(b, begin, split);
        node.offset = build_recursive(b, split, end);
        node.primitiveCountAxis |= (bestAxis << 8);
    } else {
        node.offset = (uint32_t)begin;
        node.primitiveCountAxis |= (uint32_t)(end - begin) << 16;
    }
    b->nodes[nodeIndex] = node;
    return nodeIndex;
}

/* BVH::build (BVH.cpp:5-15): elements reordered in place; nodes must hold 2n-1 entries */
OR_EXPORT uint32_t or_bvh_build(size_t count, or_cpu_hittable *elements, uint32_t maxLeaf, or_bvh_node *nodes)
{
    bvh_builder b = { elements, nodes, 0, maxLeaf };
    if (count == 0) return 0;
    build_recursive(&b, 0, count);
    return b.nodeCount;
}

/* ------------------------------------------------------------------------------------------ */
/* Intersection (Hittable.inl, AABB.inl)                                                       */
/* ------------------------------------------------------------------------------------------ */
typedef struct { v3 o, d; } ray_t; /* Ray.h */
static inline v3 ray_at(const ray_t *r, float t) { return v3_add(r->o, v3_scale(t, r->d)); }

typedef struct {                   /* HitRecord.h:8-16 */
    v3 p, normal;
    const or_material *mat;
    float t, u, v;
    int frontFace;
} hit_rec;

/* Hittable.inl:7-39 */
static inline int quadratic(float a, float b, float c, float *t0, float *t1)
{
    const float disc = b * b - 4.0f * a * c;
    if (disc < 0.0f) return 0;
    const float r = sqrtf(disc);
    const float q = b < 0.0f ? -0.5f * (b - r) : -0.5f * (b + r);
    *t0 = q / a;
    *t1 = c / q;
    if (*t0 > *t1) { float tmp = *t0; *t0 = *t1; *t1 = tmp; }
    return 1;
}

/* Hittable.inl:42-55, with the template's int coefficients converted exactly as C++ does */
static inline int hit_quadric(const int K[10], v3 o, v3 d, float *t0, float *t1)
{
    const float A = (float)K[0], B = (float)K[1], C = (float)K[2], D = (float)K[3], E = (float)K[4];
    const float F = (float)K[5], G = (float)K[6], H = (float)K[7], I = (float)K[8], J = (float)K[9];
    float a = (A * d.x * d.x) + (B * d.y * d.y) + (C * d.z * d.z) + (D * d.x * d.y) + (E * d.x * d.z) + (F * d.y * d.z);
    float b = (2.0f * A * o.x * d.x) + (2.0f * B * o.y * d.y) + (2.0f * C * o.z * d.z) + (D * (o.x * d.y + o.y * d.x))
            + (E * (o.x * d.z + o.z * d.x)) + (F * (o.y * d.z + d.y * o.z)) + (G * d.x) + (H * d.y) + (I * d.z);
    float c = (A * o.x * o.x) + (B * o.y * o.y) + (C * o.z * o.z) + (D * o.x * o.y) + (E * o.x * o.z) + (F * o.y * o.z)
            + (G * o.x) + (H * o.y) + (I * o.z) + J;
    return quadratic(a, b, c, t0, t1);
}

/* Hittable.inl:58-67 */
static inline v3 quadric_normal(const int K[10], v3 p)
{
    const float A = (float)K[0], B = (float)K[1], C = (float)K[2], D = (float)K[3], E = (float)K[4];
    const float F = (float)K[5], G = (float)K[6], H = (float)K[7], I = (float)K[8];
    v3 n;
    n.x = 2.0f * (A * p.x) + (D * p.y) + (E * p.z) + G;
    n.y = 2.0f * (B * p.y) + (D * p.x) + (F * p.z) + H;
    n.z = 2.0f * (C * p.z) + (E * p.x) + (F * p.y) + I;
    return n;
}

static const int Q_SPHERE[10] = { 1, 1, 1, 0, 0, 0, 0, 0, 0, -1 };
static const int Q_CYLINDER[10] = { 1, 0, 1, 0, 0, 0, 0, 0, 0, -1 };
static const int Q_CONE[10] = { 1, -1, 1, 0, 0, 0, 0, 0, 0, 0 };
static const int Q_PARABOLOID[10] = { 1, 0, 1, 0, 0, 0, 0, -1, 0, 0 };

#define TWO_PI_F (2.0f * PI_F)

/* Hittable.inl:147-169 */
static int hit_sphere(const ray_t *r, float tMin, float tMax, float *t, v3 *n, float *u, float *v)
{
    float t0 = 0.0f, t1 = 0.0f;
    if (!hit_quadric(Q_SPHERE, r->o, r->d, &t0, &t1) || t0 > tMax || t1 <= tMin) return 0;
    *t = t0 > tMin ? t0 : t1;
    *n = v3_normalize(ray_at(r, *t));
    float theta = pm_acosf(n->y);
    float phi = pm_atan2f(n->z, n->x);
    *u = 1.0f - phi / TWO_PI_F;
    *v = theta / PI_F;
    return 1;
}

/* Hittable.inl:171-203 / 237-266 / 268-297: quadrics limited to |y| <= 1 */
static int quadric_valid_t(const ray_t *r, float tMin, float tMax, float t0, float t1, float *t)
{
    const float h0 = r->d.y * t0 + r->o.y;
    const float h1 = r->d.y * t1 + r->o.y;
    const int v0 = t0 > tMin && t0 <= tMax && h0 >= -1.0f && h0 <= 1.0f;
    const int v1 = t1 > tMin && t1 <= tMax && h1 >= -1.0f && h1 <= 1.0f;
    if (!v0 && !v1) return 0;
    *t = v0 ? t0 : t1;
    return 1;
}

static int hit_cylinder(const ray_t *r, float tMin, float tMax, float *t, v3 *n, float *u, float *v)
{
    float t0 = 0.0f, t1 = 0.0f;
    if (!hit_quadric(Q_CYLINDER, r->o, r->d, &t0, &t1) || t0 > tMax || t1 <= tMin) return 0;
    if (!quadric_valid_t(r, tMin, tMax, t0, t1, t)) return 0;
    v3 p = ray_at(r, *t);
    *n = V(p.x, 0.0f, p.z);
    float phi = pm_atan2f(n->z, n->x);
    *u = 1.0f - phi / TWO_PI_F;
    *v = 1.0f - (p.y * 0.5f + 0.5f);
    return 1;
}

/* Hittable.inl:205-235 (disk) and 299-329 (quad) */
static int hit_planar(int isQuad, const ray_t *r, float tMin, float tMax, float *t, v3 *n, float *u, float *v)
{
    if (r->d.y == 0.0f) return 0;
    *t = -r->o.y / r->d.y;
    if (*t <= tMin || *t > tMax) return 0;
    float hx = r->o.x + r->d.x * *t;
    float hz = r->o.z + r->d.z * *t;
    if (isQuad) { if (fabsf(hx) > 1.0f || fabsf(hz) > 1.0f) return 0; }
    else { if ((hx * hx + hz * hz) >= 1.0f) return 0; }
    *n = V(0.0f, 1.0f, 0.0f);
    *u = hx * 0.5f + 0.5f;
    *v = 1.0f - (hz * 0.5f + 0.5f);
    return 1;
}

static int hit_cone(const ray_t *r, float tMin, float tMax, float *t, v3 *n, float *u, float *v)
{
    float t0 = 0.0f, t1 = 0.0f;
    if (!hit_quadric(Q_CONE, r->o, r->d, &t0, &t1) || t0 > tMax || t1 <= tMin) return 0;
    if (!quadric_valid_t(r, tMin, tMax, t0, t1, t)) return 0;
    *n = quadric_normal(Q_CONE, ray_at(r, *t));
    *u = 0.0f; /* uninitialised in the reference (Appendix B.5): defined as 0 here */
    *v = 0.0f;
    return 1;
}

static int hit_paraboloid(const ray_t *r, float tMin, float tMax, float *t, v3 *n, float *u, float *v)
{
    float t0 = 0.0f, t1 = 0.0f;
    if (!hit_quadric(Q_PARABOLOID, r->o, r->d, &t0, &t1) || t0 > tMax || t1 <= tMin) return 0;
    if (!quadric_valid_t(r, tMin, tMax, t0, t1, t)) return 0;
    *n = quadric_normal(Q_PARABOLOID, ray_at(r, *t));
    *u = 0.0f;
    *v = 0.0f;
    return 1;
}

/* AABB.inl:22-44 */
static inline int aabb_hit(v3 mn, v3 mx, const ray_t *r, float tMin, float tMax)
{
    for (int a = 0; a < 3; ++a) {
        float invD = 1.0f / v3_get(r->d, a);
        float t0 = (v3_get(mn, a) - v3_get(r->o, a)) * invD;
        float t1 = (v3_get(mx, a) - v3_get(r->o, a)) * invD;
        if (invD < 0.0f) { float tmp = t0; t0 = t1; t1 = tmp; }
        tMin = t0 > tMin ? t0 : tMin;
        tMax = t1 < tMax ? t1 : tMax;
        if (tMax <= tMin) return 0;
    }
    return 1;
}

/* AABB.inl:46-69 */
static inline int aabb_intersect(v3 mn, v3 mx, const ray_t *r, float tMin, float tMax, float *t)
{
    for (int a = 0; a < 3; ++a) {
        float invD = 1.0f / v3_get(r->d, a);
        float t0 = (v3_get(mn, a) - v3_get(r->o, a)) * invD;
        float t1 = (v3_get(mx, a) - v3_get(r->o, a)) * invD;
        if (invD < 0.0f) { float tmp = t0; t0 = t1; t1 = tmp; }
        tMin = t0 > tMin ? t0 : tMin;
        tMax = t1 < tMax ? t1 : tMax;
        if (tMax <= tMin) return 0;
    }
    *t = tMin;
    return 1;
}

/* Hittable.inl:331-358 */
static int hit_box(const ray_t *r, float tMin, float tMax, float *t, v3 *n, float *u, float *v)
{
    if (!aabb_intersect(Vs(-1.0f), Vs(1.0f), r, tMin, tMax, t)) return 0;
    v3 p = ray_at(r, *t);
    v3 an = V(fabsf(p.x), fabsf(p.y), fabsf(p.z));
    if (an.x > an.y && an.x > an.z) *n = V(p.x > 0.0f ? 1.0f : -1.0f, 0.0f, 0.0f);
    else if (an.y > an.x && an.y > an.z) *n = V(0.0f, p.y > 0.0f ? 1.0f : -1.0f, 0.0f);
    else *n = V(0.0f, 0.0f, p.z > 0.0f ? 1.0f : -1.0f);
    *u = 0.0f; /* uninitialised in the reference: defined as 0 */
    *v = 0.0f;
    return 1;
}

/* Hittable::hit (Hittable.inl:88-145) */
static int hittable_hit(const or_hittable *h, const ray_t *r, float tMin, float tMax, hit_rec *rec)
{
    ray_t lr;
    lr.o.x = v3_dot(r->o, V(h->rows[0][0], h->rows[0][1], h->rows[0][2])) + h->rows[0][3];
    lr.o.y = v3_dot(r->o, V(h->rows[1][0], h->rows[1][1], h->rows[1][2])) + h->rows[1][3];
    lr.o.z = v3_dot(r->o, V(h->rows[2][0], h->rows[2][1], h->rows[2][2])) + h->rows[2][3];
    lr.d.x = v3_dot(r->d, V(h->rows[0][0], h->rows[0][1], h->rows[0][2]));
    lr.d.y = v3_dot(r->d, V(h->rows[1][0], h->rows[1][1], h->rows[1][2]));
    lr.d.z = v3_dot(r->d, V(h->rows[2][0], h->rows[2][1], h->rows[2][2]));
    int res = 0;
    float t = 0.0f, u = 0.0f, v = 0.0f;
    v3 n = Vs(0.0f);
    switch (h->type) {
    case SPHERE: res = hit_sphere(&lr, tMin, tMax, &t, &n, &u, &v); break;
    case CYLINDER: res = hit_cylinder(&lr, tMin, tMax, &t, &n, &u, &v); break;
    case DISK: res = hit_planar(0, &lr, tMin, tMax, &t, &n, &u, &v); break;
    case CONE: res = hit_cone(&lr, tMin, tMax, &t, &n, &u, &v); break;
    case PARABOLOID: res = hit_paraboloid(&lr, tMin, tMax, &t, &n, &u, &v); break;
    case QUAD: res = hit_planar(1, &lr, tMin, tMax, &t, &n, &u, &v); break;
    case CUBE: res = hit_box(&lr, tMin, tMax, &t, &n, &u, &v); break;
    default: break;
    }
    if (res) {
        v3 tmp;
        tmp.x = v3_dot(n, V(h->rows[0][0], h->rows[1][0], h->rows[2][0]));
        tmp.y = v3_dot(n, V(h->rows[0][1], h->rows[1][1], h->rows[2][1]));
        tmp.z = v3_dot(n, V(h->rows[0][2], h->rows[1][2], h->rows[2][2]));
        rec->t = t;
        rec->p = ray_at(r, rec->t);
        v3 on = v3_normalize(tmp);
        rec->frontFace = v3_dot(r->d, on) < 0.0f;          /* HitRecord.h:18-24 */
        rec->normal = rec->frontFace ? on : v3_neg(on);
        rec->mat = &h->mat;
        rec->u = u;
        rec->v = v;
    }
    return res;
}

/* ------------------------------------------------------------------------------------------ */
/* Scene + statistics                                                                           */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    const or_hittable *prims;
    uint32_t primCount;
    const or_bvh_node *nodes;
    uint32_t nodeCount;
    uint32_t skyboxHandle;
    const or_texture *textures;  /* textures[handle-1] */
    uint32_t textureCount;
} or_scene;

typedef struct {               /* counters for SURVEY.md §8(d) algorithmic bytes */
    uint64_t node_tests, prim_tests, hits, sky_lookups, segments, samples, max_stack;
    uint64_t rises;            /* leaf visits that end with t_max above its value at the leaf's start
                                  (hit_sphere's far root t1 > t_max, Hittable.inl:152-158) */
} or_stats;

/* hitBVH (trace.cu:28-98) */
static int hit_bvh(const or_scene *s, const ray_t *r, float tMin, float tMax, hit_rec *rec, or_stats *st)
{
    /* trace.cu:31-36: invRayDir is only used for the sign test */
    int dirIsNeg[3];
    for (int i = 0; i < 3; ++i) {
        float d = v3_get(r->d, i);
        float inv = 1.0f / (d != 0.0f ? d : 1e-7f);
        dirIsNeg[i] = inv < 0.0f;
    }
    uint32_t stack[32];
    uint32_t sp = 0, cur = 0, elem = UINT32_MAX;
    for (;;) {
        const or_bvh_node *node = &s->nodes[cur];
        if (st) st->node_tests++;
        if (aabb_hit(node->bmin, node->bmax, r, tMin, tMax)) {
            const uint32_t cnt = node->primitiveCountAxis >> 16;
            if (cnt > 0) {
                const float tLeaf = tMax;
                for (uint32_t i = 0; i < cnt; ++i) {
                    if (st) st->prim_tests++;
                    if (hittable_hit(&s->prims[node->offset + i], r, tMin, tMax, rec)) {
                        tMax = rec->t;
                        elem = node->offset + i;
                    }
                }
                if (st && tMax > tLeaf) st->rises++;
                if (sp == 0) break;
                cur = stack[--sp];
            } else {
                int isNeg = dirIsNeg[(node->primitiveCountAxis >> 8) & 0xFF];
                if (sp >= 32) return -1; /* the reference overflows here (UB); reported, never silent */
                stack[sp++] = isNeg ? (cur + 1) : node->offset;
                if (st && sp > st->max_stack) st->max_stack = sp;
                cur = isNeg ? node->offset : (cur + 1);
            }
        } else {
            if (sp == 0) break;
            cur = stack[--sp];
        }
    }
    return elem != UINT32_MAX;
}

/* CUDA 2-D linear fetch, normalised coords, wrap (x) / clamp (y) (SURVEY.md Appendix C;
 * sampler settings Pathtracer.cpp:276-283) */
static v3 tex2d_bilinear(const or_texture *t, float u, float v, float *alpha_out)
{
    const float W = (float)t->width, Hh = (float)t->height;
    float uw = u - floorf(u);                 /* wrap */
    float x = uw * W - 0.5f;
    float y = v * Hh - 0.5f;
    float fx = floorf(x), fy = floorf(y);
    float a = x - fx, b = y - fy;
    a = floorf(a * 256.0f + 0.5f) * (1.0f / 256.0f);   /* 8 fractional bits */
    b = floorf(b * 256.0f + 0.5f) * (1.0f / 256.0f);
    int32_t w = (int32_t)t->width, h = (int32_t)t->height;
    int32_t i0 = (fx > -1.0e9f && fx < 1.0e9f) ? (int32_t)fx : 0;
    int32_t j0 = (fy > -1.0e9f && fy < 1.0e9f) ? (int32_t)fy : (fy > 0.0f ? h : -1);
    int32_t i1 = i0 + 1, j1 = j0 + 1;
    i0 = ((i0 % w) + w) % w;
    i1 = ((i1 % w) + w) % w;
    j0 = j0 < 0 ? 0 : (j0 > h - 1 ? h - 1 : j0);
    j1 = j1 < 0 ? 0 : (j1 > h - 1 ? h - 1 : j1);
    const float *T00 = t->texels + 4 * ((size_t)j0 * t->width + (size_t)i0);
    const float *T10 = t->texels + 4 * ((size_t)j0 * t->width + (size_t)i1);
    const float *T01 = t->texels + 4 * ((size_t)j1 * t->width + (size_t)i0);
    const float *T11 = t->texels + 4 * ((size_t)j1 * t->width + (size_t)i1);
    const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    float c[4];
    for (int k = 0; k < 4; ++k) c[k] = w00 * T00[k] + w10 * T10[k] + w01 * T01[k] + w11 * T11[k];
    if (alpha_out) *alpha_out = c[3];
    return V(c[0], c[1], c[2]);
}

OR_EXPORT void or_tex2d(const or_texture *t, float u, float v, float *rgba)
{
    float a;
    v3 c = tex2d_bilinear(t, u, v, &a);
    rgba[0] = c.x; rgba[1] = c.y; rgba[2] = c.z; rgba[3] = a;
}

/* ------------------------------------------------------------------------------------------ */
/* Shading (MonteCarlo.h, brdf.h, Material.inl)                                                */
/* ------------------------------------------------------------------------------------------ */
static inline v3 tangent_to_world(v3 N, v3 v) /* MonteCarlo.h:5-12 */
{
    v3 up = fabsf(N.z) < 0.999f ? V(0.0f, 0.0f, 1.0f) : V(1.0f, 0.0f, 0.0f);
    v3 tangent = v3_normalize(v3_cross(up, N));
    v3 bitangent = v3_cross(N, tangent);
    return v3_normalize(v3_add(v3_add(v3_scale(v.x, tangent), v3_scale(v.y, bitangent)), v3_scale(v.z, N)));
}

static inline v3 world_to_tangent(v3 N, v3 v) /* MonteCarlo.h:15-22 */
{
    v3 up = fabsf(N.z) < 0.999f ? V(0.0f, 0.0f, 1.0f) : V(1.0f, 0.0f, 0.0f);
    v3 tangent = v3_normalize(v3_cross(up, N));
    v3 bitangent = v3_cross(N, tangent);
    return v3_normalize(v3_add(v3_add(v3_scale(v.x, V(tangent.x, bitangent.x, N.x)),
                                      v3_scale(v.y, V(tangent.y, bitangent.y, N.y))),
                               v3_scale(v.z, V(tangent.z, bitangent.z, N.z))));
}

static inline v3 cosine_sample_hemisphere(float u0, float u1) /* MonteCarlo.h:24-30 */
{
    const float phi = 2.0f * PI_F * u0;
    const float cosTheta = sqrtf(u1);
    const float sinTheta = sqrtf(1.0f - u1);
    return V(pm_cosf(phi) * sinTheta, pm_sinf(phi) * sinTheta, cosTheta);
}

static inline float cosine_sample_hemisphere_pdf(v3 L) { return L.z / PI_F; } /* MonteCarlo.h:32-35 */

static inline float pow5(float v) { float v2 = v * v; return v2 * v2 * v; }     /* brdf.h:4-8 */

static inline float d_ggx(float NdotH, float a2)                                /* brdf.h:11-15 */
{
    float d = (NdotH * a2 - NdotH) * NdotH + 1.0f;
    return a2 / (PI_F * d * d);
}

static inline float v_smith_ggx_correlated(float NdotV, float NdotL, float a2)  /* brdf.h:18-24 */
{
    float lv = NdotL * sqrtf((-NdotV * a2 + NdotV) * NdotV + a2);
    float ll = NdotV * sqrtf((-NdotL * a2 + NdotL) * NdotL + a2);
    return 0.5f / (lv + ll + 1e-5f);
}

static inline v3 f_schlick(v3 F0, float VdotH)                                 /* brdf.h:27-32 */
{
    float p = pow5(1.0f - VdotH);
    return v3_adds(v3_scale(1.0f - p, F0), p);
}

static inline v3 specular_ggx(v3 F0, float NdotV, float NdotL, float NdotH, float VdotH, float a2) /* brdf.h:56-62 */
{
    float D = d_ggx(NdotH, a2);
    float Vis = v_smith_ggx_correlated(NdotV, NdotL, a2);
    v3 F = f_schlick(F0, VdotH);
    return v3_scale(D * Vis, F);
}

static inline v3 diffuse_lambert(v3 base) { return v3_scale(1.0f / PI_F, base); } /* brdf.h:51-54 */

/* MonteCarlo.h:73-101 */
static inline v3 importance_sample_ggx_vndf(v3 Vv, float u0, float u1, float a)
{
    v3 Vh = v3_normalize(V(a * Vv.x, a * Vv.y, Vv.z));
    float lensq = Vh.x * Vh.x + Vh.y * Vh.y;
    v3 T1 = lensq > 0.0f ? v3_scale(1.0f / sqrtf(lensq), V(-Vh.y, Vh.x, 0.0f)) : V(1.0f, 0.0f, 0.0f);
    v3 T2 = v3_cross(Vh, T1);
    float r = sqrtf(u0);
    float phi = 2.0f * PI_F * u1;
    float t1 = r * pm_cosf(phi);
    float t2 = r * pm_sinf(phi);
    float s = 0.5f * (1.0f + Vh.z);
    t2 = (1.0f - s) * sqrtf(1.0f - t1 * t1) + s * t2;
    v3 Nh = v3_add(v3_add(v3_scale(t1, T1), v3_scale(t2, T2)), v3_scale(sqrtf(clampf01(1.0f - t1 * t1 - t2 * t2)), Vh));
    return v3_normalize(V(a * Nh.x, a * Nh.y, clampf01(Nh.z)));
}

/* MonteCarlo.h:104-114 */
static inline float importance_sample_ggx_vndf_pdf(v3 H, v3 Vv, float a)
{
    float a2 = a * a;
    float NdotH = H.z;
    float VdotH = clampf01(v3_dot(Vv, H));
    float G1 = (2.0f * Vv.z) / (Vv.z + sqrtf(a2 + (1.0f - a2) * (Vv.z * Vv.z)));
    float Dv = (G1 * VdotH * d_ggx(NdotH, a2)) / Vv.z;
    return Dv / (4.0f * VdotH);
}

/* Material::sample (Material.inl:20-60) + lobes (:67-144).  Returns attenuation; *killed set
 * when the reflected direction is below the horizon (scattered ray then unused). */
static v3 material_sample(const or_scene *s, const ray_t *rin, const hit_rec *rec, xorwow_t *rng, ray_t *scattered,
                          float *pdf)
{
    const or_material *m = rec->mat;
    const v3 Vv = world_to_tangent(rec->normal, v3_neg(rin->d));
    v3 base = m->baseColor;
    if (m->textureIndex != 0) {
        v3 tap = tex2d_bilinear(&s->textures[m->textureIndex - 1], rec->u, rec->v, NULL);
        base = V(pm_powf(tap.x, 2.2f), pm_powf(tap.y, 2.2f), pm_powf(tap.z, 2.2f));
    }
    v3 dir = Vs(0.0f);
    v3 att = Vs(0.0f);
    float rnd0 = xorwow_uniform(rng);
    float rnd1 = xorwow_uniform(rng);
    const float a = m->roughness * m->roughness;
    const float a2 = a * a;
    switch (m->materialType) {
    case LAMBERT:
        dir = cosine_sample_hemisphere(rnd0, rnd1);
        *pdf = cosine_sample_hemisphere_pdf(dir);
        att = diffuse_lambert(base);
        break;
    case GGX: {
        dir = v3_reflect(v3_neg(Vv), importance_sample_ggx_vndf(Vv, rnd0, rnd1, a));
        if (dir.z < 0.0f) { *pdf = 1.0f; return Vs(0.0f); }
        const float NdotV = fabsf(Vv.z) + 1e-5f;
        const v3 H = v3_normalize(v3_add(Vv, dir));
        const float VdotH = clampf01(v3_dot(Vv, H));
        const float NdotH = clampf01(H.z);
        const float NdotL = clampf01(dir.z);
        *pdf = importance_sample_ggx_vndf_pdf(H, Vv, a);
        const v3 F0 = v3_lerp(Vs(0.04f), base, m->metalness);
        att = specular_ggx(F0, NdotV, NdotL, NdotH, VdotH, a2);
        break;
    }
    case LAMBERT_GGX: {
        if (rnd0 < 0.5f) {
            rnd0 = 2.0f * rnd0;
            dir = cosine_sample_hemisphere(rnd0, rnd1);
        } else {
            rnd0 = 2.0f * (rnd0 - 0.5f);
            dir = v3_reflect(v3_neg(Vv), importance_sample_ggx_vndf(Vv, rnd0, rnd1, a));
        }
        if (dir.z < 0.0f) { *pdf = 1.0f; return Vs(0.0f); }
        const float NdotV = fabsf(Vv.z) + 1e-5f;
        const v3 H = v3_normalize(v3_add(Vv, dir));
        const float VdotH = clampf01(v3_dot(Vv, H));
        const float NdotH = clampf01(H.z);
        const float NdotL = clampf01(dir.z);
        const float cosinePdf = cosine_sample_hemisphere_pdf(dir);
        const float ggxPdf = importance_sample_ggx_vndf_pdf(H, Vv, a);
        *pdf = (ggxPdf + cosinePdf) * 0.5f;
        const v3 F0 = v3_lerp(Vs(0.04f), base, m->metalness);
        const v3 kS = specular_ggx(F0, NdotV, NdotL, NdotH, VdotH, a2);
        const v3 kD = diffuse_lambert(base);
        att = v3_add(v3_scale(1.0f - m->metalness, kD), kS);
        break;
    }
    default:
        break;
    }
    scattered->o = rec->p;
    scattered->d = v3_normalize(tangent_to_world(rec->normal, dir));
    return att;
}

/* getColor (trace.cu:101-156) */
static v3 get_color(const or_scene *s, ray_t ray, xorwow_t *rng, or_stats *st, int *err)
{
    v3 T = Vs(1.0f);
    v3 L = Vs(0.0f);
    for (int it = 0; it < 5; ++it) {
        hit_rec rec;
        memset(&rec, 0, sizeof(rec));
        if (st) st->segments++;
        int found = hit_bvh(s, &ray, 0.001f, FLT_MAX, &rec, st);
        if (found < 0) { *err = 1; found = 0; }
        if (!found) {
            v3 c = Vs(0.0f);
            if (s->skyboxHandle != 0) {
                float theta = pm_acosf(ray.d.y);
                float phi = pm_atan2f(ray.d.z, ray.d.x);
                float v = theta / PI_F;
                float u = phi / TWO_PI_F;
                c = tex2d_bilinear(&s->textures[s->skyboxHandle - 1], u, v, NULL);
                if (st) st->sky_lookups++;
            }
            L = v3_add(L, v3_mul(T, c));
            break;
        }
        if (st) st->hits++;
        L = v3_add(L, v3_mul(T, rec.mat->emissive));
        ray_t scattered;
        float pdf = 0.0f;
        v3 att = material_sample(s, &ray, &rec, rng, &scattered, &pdf);
        if (v3_eq(att, Vs(0.0f)) || pdf == 0.0f) break;
        v3 w = v3_divs(v3_scale(fabsf(v3_dot(scattered.d, rec.normal)), att), pdf);
        T = v3_mul(T, w);
        ray = scattered;
    }
    return L;
}

/* ------------------------------------------------------------------------------------------ */
/* Kernels: initRandState (initRandState.cu:4-17), traceKernel (trace.cu:158-199), tonemap     */
/* (tonemap.cu:4-27).  Pixels are addressed by global (x, y); a "view" selects the row bands     */
/* b = band_offset + k * band_stride of band_rows rows each (band_rows = 1: rows                   */
/* y = offset + k * stride) so multi-GPU tiles can be reproduced.  Written out independently of   */
/* the kernel's global_row (pt_kernels.hip): the band of local row k is k / band_rows.            */
/* ------------------------------------------------------------------------------------------ */
static uint32_t view_rows(uint32_t height, uint32_t band_rows, uint32_t offset, uint32_t stride)
{
    uint32_t rows = 0;
    for (uint32_t b = offset; (uint64_t)b * band_rows < height; b += stride) {
        uint32_t end = (b + 1) * band_rows < height ? (b + 1) * band_rows : height;
        rows += end - b * band_rows;
    }
    return rows;
}

static uint32_t view_row(uint32_t k, uint32_t band_rows, uint32_t offset, uint32_t stride)
{
    uint32_t band = offset + (k / band_rows) * stride;
    return band * band_rows + k % band_rows;
}

OR_EXPORT uint32_t or_view_rows(uint32_t height, uint32_t band_rows, uint32_t offset, uint32_t stride)
{
    return view_rows(height, band_rows, offset, stride);
}

OR_EXPORT void or_init_rand_state(uint32_t width, uint32_t height, uint32_t band_rows, uint32_t row_offset,
                                  uint32_t row_stride, xorwow_t *states)
{
    uint32_t rows = view_rows(height, band_rows, row_offset, row_stride);
    for (uint32_t k = 0; k < rows; ++k) {
        uint32_t y = view_row(k, band_rows, row_offset, row_stride);
        for (uint32_t x = 0; x < width; ++x) {
            uint32_t idx = x + y * width;
            or_xorwow_init((uint64_t)(uint32_t)(1984u + idx), &states[(size_t)k * width + x]);
        }
    }
}

typedef struct {
    const or_scene *scene;
    const or_camera *cam;
    float *accum;
    xorwow_t *rng;
    uint32_t width, height, band_rows, row_offset, row_stride, rows, spp, chunks, ignoreFirst;
    uint32_t nthreads, tid, collect;
    uint32_t *next_row;   /* shared cursor: rows are handed out dynamically (any order gives the same bits) */
    or_stats stats;
    int err;
} render_job;

static void render_rows(render_job *j)
{
    const or_camera *cam = j->cam;
    for (;;) {
        uint32_t k = __atomic_fetch_add(j->next_row, 1u, __ATOMIC_RELAXED);
        if (k >= j->rows) break;
        uint32_t y = view_row(k, j->band_rows, j->row_offset, j->row_stride);
        for (uint32_t x = 0; x < j->width; ++x) {
            size_t li = (size_t)k * j->width + x;
            xorwow_t st = j->rng[li];
            float *acc = j->accum + 4 * li;
            for (uint32_t c = 0; c < j->chunks; ++c) {
                v3 color = Vs(0.0f);
                for (uint32_t i = 0; i < j->spp; ++i) {
                    j->stats.samples++;
                    float u = ((float)(int32_t)x + xorwow_uniform(&st)) / (float)j->width;
                    float v = ((float)(int32_t)y + xorwow_uniform(&st)) / (float)j->height;
                    ray_t r;
                    r.o = cam->origin; /* Camera.inl:25-28 */
                    r.d = v3_normalize(v3_add(v3_add(cam->lowerLeftCorner, v3_scale(u, cam->horizontal)),
                                              v3_scale(v, cam->vertical)));
                    color = v3_add(color, get_color(j->scene, r, &st, j->collect ? &j->stats : NULL, &j->err));
                }
                int ignore = (c == 0) ? (int)j->ignoreFirst : 0;
                if (!ignore) color = v3_add(color, V(acc[0], acc[1], acc[2]));
                acc[0] = color.x; acc[1] = color.y; acc[2] = color.z; acc[3] = 1.0f;
            }
            j->rng[li] = st;
        }
    }
}

static void *render_thread(void *p) { render_rows((render_job *)p); return NULL; }

/* Equivalent to `chunks` successive reference render(camera, spp, ignoreHistory_c) calls with
 * ignoreHistory_0 = ignore_first and ignoreHistory_c>0 = false (main.cpp:275-279).  Returns 0 on
 * success, -1 if a traversal stack would overflow (undefined behaviour in the reference). */
OR_EXPORT int or_render(const or_hittable *prims, uint32_t primCount, const or_bvh_node *nodes, uint32_t nodeCount,
                        const or_camera *cam, uint32_t skyboxHandle, const or_texture *textures, uint32_t textureCount,
                        uint32_t width, uint32_t height, uint32_t band_rows, uint32_t row_offset, uint32_t row_stride,
                        float *accum,
                        xorwow_t *rng, uint32_t spp, uint32_t chunks, int ignore_first, int nthreads, uint64_t *stats_out)
{
    or_scene s = { prims, primCount, nodes, nodeCount, skyboxHandle, textures, textureCount };
    uint32_t rows = view_rows(height, band_rows, row_offset, row_stride);
    if (nodeCount < 1 || primCount < 1 || spp == 0) return 0; /* Pathtracer.cpp:174: no launch */
    if (nthreads < 1) nthreads = 1;
    uint32_t next_row = 0;
    render_job *jobs = (render_job *)calloc((size_t)nthreads, sizeof(render_job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        render_job *j = &jobs[t];
        j->scene = &s; j->cam = cam; j->accum = accum; j->rng = rng;
        j->width = width; j->height = height; j->band_rows = band_rows; j->row_offset = row_offset; j->row_stride = row_stride; j->rows = rows;
        j->spp = spp; j->chunks = chunks; j->ignoreFirst = (uint32_t)(ignore_first != 0);
        j->nthreads = (uint32_t)nthreads; j->tid = (uint32_t)t; j->collect = stats_out != NULL;
        j->next_row = &next_row;
        if (nthreads > 1) pthread_create(&th[t], NULL, render_thread, j);
        else render_rows(j);
    }
    int err = 0;
    uint64_t agg[8] = { 0 };
    for (int t = 0; t < nthreads; ++t) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        err |= jobs[t].err;
        agg[0] += jobs[t].stats.node_tests; agg[1] += jobs[t].stats.prim_tests; agg[2] += jobs[t].stats.hits;
        agg[3] += jobs[t].stats.sky_lookups; agg[4] += jobs[t].stats.segments; agg[5] += jobs[t].stats.samples;
        if (jobs[t].stats.max_stack > agg[6]) agg[6] = jobs[t].stats.max_stack;
        agg[7] += jobs[t].stats.rises;
    }
    if (stats_out) memcpy(stats_out, agg, sizeof(agg));
    free(jobs);
    free(th);
    return err ? -1 : 0;
}

/* Test infrastructure for the speculative sample groups: the raw draw stream of one
 * pixel, and its per-sample log from any starting state -- the colour getColor returns
 * (trace.cu:190-193) and the draw pairs the sample consumed (1 for the jitter + 1 per hit,
 * Material.inl:40-41).  Same operations as render_rows. */
OR_EXPORT void or_xorwow_skip(xorwow_t *s, uint64_t draws)
{
    while (draws--) (void)xorwow_next(s);
}

OR_EXPORT int or_sample_log(const or_hittable *prims, uint32_t primCount, const or_bvh_node *nodes, uint32_t nodeCount,
                            const or_camera *cam, uint32_t skyboxHandle, const or_texture *textures, uint32_t textureCount,
                            uint32_t width, uint32_t height, uint32_t x, uint32_t y, xorwow_t *state, uint32_t n,
                            float *colors, uint8_t *pairs)
{
    or_scene s = { prims, primCount, nodes, nodeCount, skyboxHandle, textures, textureCount };
    int err = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t d0 = state->d;
        float u = ((float)(int32_t)x + xorwow_uniform(state)) / (float)width;
        float v = ((float)(int32_t)y + xorwow_uniform(state)) / (float)height;
        ray_t r;
        r.o = cam->origin;
        r.d = v3_normalize(v3_add(v3_add(cam->lowerLeftCorner, v3_scale(u, cam->horizontal)), v3_scale(v, cam->vertical)));
        v3 c = get_color(&s, r, state, NULL, &err);
        colors[3 * i] = c.x; colors[3 * i + 1] = c.y; colors[3 * i + 2] = c.z;
        pairs[i] = (uint8_t)(((state->d - d0) * 0x385e5f0du /* 1/362437 mod 2^32 */) / 2u);
    }
    return err ? -1 : 0;
}

/* tonemap.cu:4-27 (frames = the divisor passed by the caller, Pathtracer.cpp:328) */
OR_EXPORT void or_tonemap(const float *accum, size_t npix, uint32_t frames, uint8_t *out)
{
    for (size_t i = 0; i < npix; ++i) {
        v3 c = v3_divs(V(accum[4 * i], accum[4 * i + 1], accum[4 * i + 2]), (float)frames);
        c = v3_divv(c, v3_adds(c, 1.0f));
        float ch[3] = { pm_powf(c.x, 1.0f / 2.2f), pm_powf(c.y, 1.0f / 2.2f), pm_powf(c.z, 1.0f / 2.2f) };
        for (int k = 0; k < 3; ++k) {
            float f = ch[k] * 255.0f;
            int32_t q = (f != f) ? 0 : f2i_x86(f);
            out[4 * i + k] = (uint8_t)(q & 0xFF);
        }
        out[4 * i + 3] = 255;
    }
}

/* getHDRImageData (Pathtracer.cpp:299-315) */
OR_EXPORT void or_hdr_normalize(const float *accum, size_t npix, uint32_t frames, float *out)
{
    float inv = 1.0f / fmaxf((float)frames, 1.0f);
    for (size_t i = 0; i < 4 * npix; ++i) out[i] = accum[i] * inv;
}

OR_EXPORT uint32_t or_sizeof(int which)
{
    switch (which) {
    case 0: return (uint32_t)sizeof(or_material);
    case 1: return (uint32_t)sizeof(or_hittable);
    case 2: return (uint32_t)sizeof(or_cpu_hittable);
    case 3: return (uint32_t)sizeof(or_bvh_node);
    case 4: return (uint32_t)sizeof(or_camera);
    case 5: return (uint32_t)sizeof(xorwow_t);
    case 6: return (uint32_t)sizeof(or_texture);
    default: return 0;
    }
}
