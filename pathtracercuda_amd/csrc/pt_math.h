// pt_math.h -- device float math for the gfx950 path-tracing megakernel.
//
// Semantics follow the reference's __host__ __device__ headers operation for operation
// (PathtracerCUDA/src/pathtracer/vec3.inl, MonteCarlo.h, brdf.h): every division, the order of
// every sum, and the reciprocal-multiply forms (vec3 / s == (1/s) * v, vec3.inl:116-119) are kept,
// because one ulp anywhere can flip a hit/miss and decorrelate a pixel's RNG stream.  Compiled with
// -ffp-contract=off; hipcc's default IEEE division and sqrt are used (correctly rounded), and rcp_rn / sqrt_rn
// below for 1/x and sqrt(x) (also correctly rounded, proven exhaustively).
//
// The transcendentals are this project's own single-precision routines (Cephes-style reduction +
// minimax polynomials, no FMA): CUDA libdevice is not available on AMD and ocml's results differ
// in the last ulp, so the path fixes one definition of sinf/cosf/acosf/atan2f/powf (DESIGN.md
// "Float determinism").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PT_DEV __device__ __forceinline__

namespace pt {

constexpr float kPi = 3.14159265358979323846f;   // vec3.h:5
constexpr float kTwoPi = 2.0f * kPi;             // folded exactly as `2.0f * PI`
constexpr float kInvPi = 1.0f / kPi;             // brdf.h:53 `1.0f / PI`
constexpr float kFltMax = 3.402823466e+38f;

// Correctly rounded 1/x and sqrt(x) in fewer VALU instructions than hipcc's general expansions.
// tools/fp_exhaustive.hip checks every one of the 2^32 inputs on gfx950: v_rcp_f32 followed by one
// fma Newton step equals the correctly rounded reciprocal for 2^-125 <= |x| <= 2^125, and
// v_rsq_f32 followed by one Newton correction of x * rsq(x) with the exact fma residual
// (5 VALU; the v_sqrt_f32 + +-1 ulp residual test it replaces took 9) equals the correctly rounded
// square root for 2^-96 <= x <= FLT_MAX (profiles/r01_fp_exhaustive.json: 0 mismatches).  Other inputs
// (zero, denormals, huge values, inf, NaN) take the general path.  Being correctly rounded, both
// give exactly IEEE 1/x and sqrt(x) -- the oracle's and the reference's values.
PT_DEV float rcp_rn(float x)
{
    const float ax = __builtin_fabsf(x);
    if (ax >= 0x1p-125f && ax <= 0x1p125f) {
        const float y = __builtin_amdgcn_rcpf(x);
        const float e = __builtin_fmaf(-x, y, 1.0f);
        return __builtin_fmaf(e, y, y);
    }
    return 1.0f / x;
}

PT_DEV float sqrt_rn(float x)
{
    // one unsigned compare: 2^-96 <= x <= FLT_MAX (negatives, inf and NaN fall outside)
    if (__float_as_uint(x) - 0x0f800000u <= 0x7f7fffffu - 0x0f800000u) {
        const float y = __builtin_amdgcn_rsqf(x);          // ~1/sqrt(x)
        const float s0 = x * y, h = 0.5f * y;
        const float r = __builtin_fmaf(-s0, s0, x);        // exact residual x - s0^2
        return __builtin_fmaf(r, h, s0);
    }
    return sqrtf(x);
}

// A root and its reciprocal behind ONE range guard (each divergent guard costs the CU's scalar unit
// an exec-mask save, flip and restore): when the operand is in sqrt's fast range both fast
// sequences apply, otherwise both general paths run -- the same values either way.  (Round 5 also
// merged pairs of roots in shading this way, +0.62 %; round 6 replaced them by sqrt_dom where the
// operand's range is known, and the merge of the three ray reciprocals and of the cube test's three
// measured -1.1 % and is not used.)
PT_DEV bool sqrt_fast_ok(float x) { return __float_as_uint(x) - 0x0f800000u <= 0x7f7fffffu - 0x0f800000u; }
PT_DEV float rcp_fast(float x)
{
    const float y = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, y, 1.0f), y, y);
}
PT_DEV float sqrt_fast(float x)
{
    const float y = __builtin_amdgcn_rsqf(x);
    const float s0 = x * y, h = 0.5f * y;
    return __builtin_fmaf(__builtin_fmaf(-s0, s0, x), h, s0);
}
// sqrt_rn for operands known to be +0, NaN or inside the fast range [2^-96, FLT_MAX] -- no range
// guard, so no divergent region (exec-mask work on the CU's one scalar unit) and no out-of-line
// general path.  +0 -> +0 and a quiet NaN -> the same NaN, as sqrtf returns them (its special-class
// select passes the input through; operands computed by arithmetic are never signalling NaNs).
// Callers state why the precondition holds: e.g. curand_uniform values lie in [2^-33, 1], and
// differences of such values are 0 or at least 2^-48.  tools/fp_exhaustive.hip checks the domain.
PT_DEV float sqrt_dom(float x)
{
    const float y = __builtin_amdgcn_rsqf(x);
    const float s0 = x * y, h = 0.5f * y;
    const float s = __builtin_fmaf(__builtin_fmaf(-s0, s0, x), h, s0);
    return x > 0.0f ? s : x;
}

// 1 / sqrt_rn(x): a root in sqrt's fast range lies in [2^-48, 2^64], inside rcp's fast range
PT_DEV float rcp_sqrt_rn(float x)
{
    if (sqrt_fast_ok(x)) return rcp_fast(sqrt_fast(x));
    return rcp_rn(sqrtf(x));
}

// The same values with the guard as a wave-uniform branch: the fast sequence runs for every
// active lane, and only when some lane is outside the guard range does the wave evaluate the
// general expression (for all its lanes) and select it there.  A divergent if/else costs the
// scalar unit -- one per CU, shared by all its waves -- an exec-mask save, flip and restore per
// call; this form costs one compare-to-mask and one scalar branch.
PT_DEV float rcp_rn_u(float x)
{
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y, 1.0f);
    float r = __builtin_fmaf(e, y, y);
    const float ax = __builtin_fabsf(x);
    const bool ok = ax >= 0x1p-125f && ax <= 0x1p125f;
    if (__ballot(!ok) != 0ull) {
        const float g = 1.0f / x;
        r = ok ? r : g;
    }
    return r;
}

PT_DEV float sqrt_rn_u(float x)
{
    const float y = __builtin_amdgcn_rsqf(x);
    const float s0 = x * y, h = 0.5f * y;
    float s = __builtin_fmaf(__builtin_fmaf(-s0, s0, x), h, s0);
    const bool ok = __float_as_uint(x) - 0x0f800000u <= 0x7f7fffffu - 0x0f800000u;
    if (__ballot(!ok) != 0ull) {
        const float g = sqrtf(x);
        s = ok ? s : g;
    }
    return s;
}

// x / c for the constants c = PI, 2 PI: q = x * RN(1/c) corrected once with the exact residual
// fma(-c, q, x) (Markstein), behind the guard 2^-100 <= |x| <= 2^100 (other inputs, incl. 0,
// inf and NaN, divide).  Checked against the correctly rounded quotient for all 2^32 inputs by
// tools/fp_exhaustive.hip.
template <int K>
PT_DEV float div_const(float x)
{
    constexpr float c = K == 1 ? 3.14159265358979323846f : 2.0f * 3.14159265358979323846f;
    constexpr float y = 1.0f / c;                    // RN(1/c), folded at compile time
    const float ax = __builtin_fabsf(x);
    if (ax >= 0x1p-100f && ax <= 0x1p100f) {
        const float q = x * y;
        const float r = __builtin_fmaf(-c, q, x);
        return __builtin_fmaf(r, y, q);
    }
    return x / c;
}
PT_DEV float div_pi(float x) { return div_const<1>(x); }
PT_DEV float div_two_pi(float x) { return div_const<2>(x); }

struct f3 { float x, y, z; };

PT_DEV f3 mk(float x, float y, float z) { return f3{x, y, z}; }
PT_DEV f3 splat(float s) { return f3{s, s, s}; }
PT_DEV f3 neg(f3 a) { return f3{-a.x, -a.y, -a.z}; }
PT_DEV f3 add(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
PT_DEV f3 adds(f3 a, float s) { return f3{a.x + s, a.y + s, a.z + s}; }
PT_DEV f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
PT_DEV f3 mul(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
PT_DEV f3 scale(float t, f3 v) { return f3{t * v.x, t * v.y, t * v.z}; }
PT_DEV f3 divs(f3 v, float t) { return scale(rcp_rn(t), v); }
PT_DEV float dot(f3 u, f3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
PT_DEV f3 cross(f3 u, f3 v) { return f3{u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x}; }
PT_DEV float length(f3 v) { return sqrt_rn(v.x * v.x + v.y * v.y + v.z * v.z); }
// normalize = (1 / sqrt_rn(|v|^2)) * v with one range guard instead of two: when |v|^2 lies in
// sqrt_rn's fast range [2^-96, FLT_MAX], the root lies in [2^-48, 2^64], inside rcp_rn's fast range,
// so both fast sequences apply; otherwise both general paths run.  Same values as
// divs(v, length(v)); one divergent region (exec-mask work on the scalar unit) fewer per call.
PT_DEV f3 normalize(f3 v)
{
    const float l2 = v.x * v.x + v.y * v.y + v.z * v.z;
    float inv;
#if defined(PT_NORMALIZE_U) && PT_NORMALIZE_U
    {   // A/B: the guard as a wave-uniform branch (see rcp_rn_u)
        const float y = __builtin_amdgcn_rsqf(l2);
        const float s0 = l2 * y, h = 0.5f * y;
        const float l = __builtin_fmaf(__builtin_fmaf(-s0, s0, l2), h, s0);
        const float r = __builtin_amdgcn_rcpf(l);
        inv = __builtin_fmaf(__builtin_fmaf(-l, r, 1.0f), r, r);
        const bool ok = __float_as_uint(l2) - 0x0f800000u <= 0x7f7fffffu - 0x0f800000u;
        if (__ballot(!ok) != 0ull) {
            const float g = rcp_rn(sqrtf(l2));
            inv = ok ? inv : g;
        }
        return scale(inv, v);
    }
#endif
    if (__float_as_uint(l2) - 0x0f800000u <= 0x7f7fffffu - 0x0f800000u) {
        const float y = __builtin_amdgcn_rsqf(l2);
        const float s0 = l2 * y, h = 0.5f * y;
        const float l = __builtin_fmaf(__builtin_fmaf(-s0, s0, l2), h, s0);
        const float r = __builtin_amdgcn_rcpf(l);
        inv = __builtin_fmaf(__builtin_fmaf(-l, r, 1.0f), r, r);
    } else {
        inv = rcp_rn(sqrtf(l2));
    }
    return scale(inv, v);
}
// normalize for vectors whose |v|^2 is NaN or inside [2^-96, FLT_MAX] (unit-length up to rounding:
// a point on the unit sphere, a unit vector in an orthonormal frame, the cross product of the
// up vector with a unit normal at least 0.001 away from it) -- no range guard.  A NaN |v|^2 gives
// the same NaN as the general path: 1 / sqrtf(NaN) passes the NaN through (sqrtf's special-class
// select, then the division's fixup of a NaN denominator).
PT_DEV f3 normalize_dom(f3 v)
{
    const float l2 = v.x * v.x + v.y * v.y + v.z * v.z;
    const float y = __builtin_amdgcn_rsqf(l2);
    const float s0 = l2 * y, h = 0.5f * y;
    const float l = __builtin_fmaf(__builtin_fmaf(-s0, s0, l2), h, s0);
    const float r = __builtin_amdgcn_rcpf(l);
    const float inv = __builtin_fmaf(__builtin_fmaf(-l, r, 1.0f), r, r);
    return scale(l2 == l2 ? inv : l2, v);
}
PT_DEV f3 reflect(f3 v, f3 n) { return sub(v, scale(2.0f * dot(v, n), n)); }
PT_DEV f3 lerp(f3 x, f3 y, float a) { return add(scale(1.0f - a, x), scale(a, y)); }
PT_DEV float clamp01(float x) { x = x < 0.0f ? 0.0f : x; x = x > 1.0f ? 1.0f : x; return x; }
PT_DEV bool is_zero(f3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }

// ---------------------------------------------------------------------------------------------
// transcendentals (same algorithm, constants and evaluation order as the oracle restatement)
// ---------------------------------------------------------------------------------------------
constexpr float kFopi = 1.27323954473516f;
constexpr float kDp1 = 0.78515625f;
constexpr float kDp2 = 2.4187564849853515625e-4f;
constexpr float kDp3 = 3.77489497744594108e-8f;
constexpr float kPio2 = 1.5707963267948966192f;
constexpr float kPio4 = 0.7853981633974483096f;

PT_DEV float sin_poly(float z, float zz)
{
    return ((-1.9515295891E-4f * zz + 8.3321608736E-3f) * zz - 1.6666654611E-1f) * zz * z + z;
}
PT_DEV float cos_poly(float zz)
{
    float y = ((2.443315711809948E-5f * zz - 1.388731625493765E-3f) * zz + 4.166664568298827E-2f) * zz * zz;
    y = y - 0.5f * zz;
    return y + 1.0f;
}

// sin and cos of one argument x in [0, 65536] (both call sites pass 2*pi*u, u in (0,1]).
PT_DEV void sincos_pos(float x, float& s, float& c)
{
    int32_t j = (int32_t)(x * kFopi);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    bool sneg = false, cneg = false;
    if (j > 3) { sneg = true; cneg = true; j -= 4; }
    if (j > 1) cneg = !cneg;
    const float z = ((x - y * kDp1) - y * kDp2) - y * kDp3;
    const float zz = z * z;
    const float ps = sin_poly(z, zz);
    const float pc = cos_poly(zz);
    const bool swap = (j == 1 || j == 2);
    float rs = swap ? pc : ps;
    float rc = swap ? ps : pc;
    s = sneg ? -rs : rs;
    c = cneg ? -rc : rc;
}

PT_DEV float asin_core(float a)
{
    float x, z;
    bool flag;
    if (a > 0.5f) { z = 0.5f * (1.0f - a); x = sqrt_rn(z); flag = true; }
    else { x = a; z = x * x; flag = false; }
    float r;
    if (a < 1.0e-4f) r = a;
    else r = ((((4.2163199048E-2f * z + 2.4181311049E-2f) * z + 4.5470025998E-2f) * z + 7.4953002686E-2f) * z
              + 1.6666752422E-1f) * z * x + x;
    if (flag) { r = r + r; r = kPio2 - r; }
    return r;
}

PT_DEV float acos_(float x)
{
    if (!(x >= -1.0f && x <= 1.0f)) return (x != x) ? x : __uint_as_float(0x7fc00000u);
    if (x < -0.5f) return kPi - 2.0f * asin_core(sqrt_rn(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * asin_core(sqrt_rn(0.5f * (1.0f - x)));
    float r = asin_core(fabsf(x));
    return x < 0.0f ? kPio2 + r : kPio2 - r;
}

PT_DEV float atan_pos(float x)
{
    float y;
    if (x > 2.414213562373095f) { y = kPio2; x = -rcp_rn(x); }
    else if (x > 0.4142135623730950f) { y = kPio4; x = (x - 1.0f) / (x + 1.0f); }
    else y = 0.0f;
    const float z = x * x;
    return y + ((((8.05374449538e-2f * z - 1.38776856032E-1f) * z + 1.99777106478E-1f) * z - 3.33329491539E-1f) * z * x + x);
}

PT_DEV float atan2_(float y, float x)
{
    if (x != x || y != y) return x + y;
    if (y == 0.0f) {
        if (__float_as_uint(x) >> 31) return (__float_as_uint(y) >> 31) ? -kPi : kPi;
        return y;
    }
    if (x == 0.0f) return y < 0.0f ? -kPio2 : kPio2;
    const float ay = fabsf(y), ax = fabsf(x);
    if (__builtin_isinf(ax)) {
        float r;
        if (__builtin_isinf(ay)) r = (x > 0.0f) ? kPio4 : 3.0f * kPio4;
        else r = (x > 0.0f) ? 0.0f : kPi;
        return y < 0.0f ? -r : r;
    }
    float r = atan_pos(ay / ax);
    if (x < 0.0f) r = kPi - r;
    return y < 0.0f ? -r : r;
}

// Select forms of acos_ and atan2_ for the kernel (sky lookup, sphere/cylinder uv): every lane
// evaluates the operations of its own range -- the same operations in the same order as acos_ /
// atan2_, so the same bits -- but the ranges are chosen by selects instead of divergent branches
// (one sqrt with a per-lane operand, one polynomial), and the rare special inputs (NaN, zeros,
// infinities, |x| > 1) overwrite the result afterwards in reverse order of precedence.
PT_DEV float asin_core_le_half(float a)                  // asin_core for 0 <= a <= 0.5 (or NaN)
{
    const float z = a * a;
    const float p = ((((4.2163199048E-2f * z + 2.4181311049E-2f) * z + 4.5470025998E-2f) * z + 7.4953002686E-2f) * z
                     + 1.6666752422E-1f) * z * a + a;
    return a < 1.0e-4f ? a : p;
}

PT_DEV float acos_sel(float x)
{
    const bool lo = x < -0.5f, hi = x > 0.5f;
    // sqrt_dom: for |x| <= 1 the operand is +0 or >= 2^-26 (a multiple of ulp(x) / 2); |x| > 1 and NaN
    // give a negative or NaN operand whose root is never used (overwritten below)
    const float s = sqrt_dom(0.5f * (lo ? (1.0f + x) : (1.0f - x)));
    const float r = asin_core_le_half((lo || hi) ? s : fabsf(x));
    float res = lo ? kPi - 2.0f * r : (hi ? 2.0f * r : (x < 0.0f ? kPio2 + r : kPio2 - r));
    if (!(x >= -1.0f && x <= 1.0f)) res = (x != x) ? x : __uint_as_float(0x7fc00000u);
    return res;
}

PT_DEV float atan_pos_sel(float x)
{
    const bool big = x > 2.414213562373095f;
    const bool mid = !big && x > 0.4142135623730950f;
    // one division for both reduced ranges: -1 / x (= -rcp_rn(x): round-to-nearest is sign-symmetric)
    // or (x - 1) / (x + 1); tools/fp_exhaustive.hip checks the result against atan_pos for all inputs
    const float q = (big ? -1.0f : x - 1.0f) / (big ? x : x + 1.0f);
    const float y = big ? kPio2 : (mid ? kPio4 : 0.0f);
    const float t = (big || mid) ? q : x;
    const float z = t * t;
    return y + ((((8.05374449538e-2f * z - 1.38776856032E-1f) * z + 1.99777106478E-1f) * z - 3.33329491539E-1f) * z * t + t);
}

PT_DEV float atan2_sel(float y, float x)
{
    const float ay = fabsf(y), ax = fabsf(x);
    float r = atan_pos_sel(ay / ax);
    r = x < 0.0f ? kPi - r : r;
    r = y < 0.0f ? -r : r;
    if (__builtin_isinf(ax)) {
        const float q = __builtin_isinf(ay) ? ((x > 0.0f) ? kPio4 : 3.0f * kPio4) : ((x > 0.0f) ? 0.0f : kPi);
        r = y < 0.0f ? -q : q;
    }
    if (x == 0.0f) r = y < 0.0f ? -kPio2 : kPio2;
    if (y == 0.0f) r = (__float_as_uint(x) >> 31) ? ((__float_as_uint(y) >> 31) ? -kPi : kPi) : y;
    if (x != x || y != y) r = x + y;
    return r;
}

PT_DEV float log_(float x)
{
    uint32_t b = __float_as_uint(x);
    int32_t e = 0;
    if ((b >> 23) == 0) { x = x * 8388608.0f; b = __float_as_uint(x); e = -23; }
    e += (int32_t)((b >> 23) & 0xffu) - 126;
    x = __uint_as_float((b & 0x807fffffu) | 0x3f000000u);
    if (x < 0.707106781186547524f) { e -= 1; x = x + x - 1.0f; }
    else x = x - 1.0f;
    float z = x * x;
    float y = ((((((((7.0376836292E-2f * x - 1.1514610310E-1f) * x + 1.1676998740E-1f) * x - 1.2420140846E-1f) * x
                   + 1.4249322787E-1f) * x - 1.6668057665E-1f) * x + 2.0000714765E-1f) * x - 2.4999993993E-1f) * x
              + 3.3333331174E-1f) * x * z;
    const float fe = (float)e;
    y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    z = x + y;
    z = z + 0.693359375f * fe;
    return z;
}

PT_DEV float exp_(float x)
{
    if (x > 88.7228391f) return __uint_as_float(0x7f800000u);
    if (x < -103.972084f) return 0.0f;
    float z = floorf(1.44269504088896341f * x + 0.5f);
    x = x - z * 0.693359375f;
    x = x - z * -2.12194440e-4f;
    const int32_t n = (int32_t)z;
    z = x * x;
    float r = (((((1.9875691500E-4f * x + 1.3981999507E-3f) * x + 8.3334519073E-3f) * x + 4.1665795894E-2f) * x
                + 1.6666665459E-1f) * x + 5.0000001201E-1f) * z + x + 1.0f;
    const int32_t n1 = n / 2, n2 = n - n1;
    r = r * __uint_as_float((uint32_t)(n1 + 127) << 23);
    r = r * __uint_as_float((uint32_t)(n2 + 127) << 23);
    return r;
}

PT_DEV float pow_(float x, float y)
{
    if (x != x || y != y) return x + y;
    if (y == 0.0f || x == 1.0f) return 1.0f;
    if (x == 0.0f) return y > 0.0f ? 0.0f : __uint_as_float(0x7f800000u);
    if (x < 0.0f) return __uint_as_float(0x7fc00000u);
    if (__builtin_isinf(x)) return y > 0.0f ? x : 0.0f;
    return exp_(y * log_(x));
}

// float -> int32 with x86 cvttss2si semantics (used where the reference truncates to uchar)
PT_DEV int32_t f2i_x86(float f)
{
    if (!(f > -2147483904.0f && f < 2147483648.0f)) return INT32_MIN;
    return (int32_t)f;
}

// ---------------------------------------------------------------------------------------------
// cuRAND XORWOW: d + v[5] kept in registers for a whole launch
// ---------------------------------------------------------------------------------------------
struct Xorwow { uint32_t d, v0, v1, v2, v3, v4; };

PT_DEV Xorwow xorwow_init(uint64_t seed)
{
    const uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    const uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    const uint32_t t0 = 1099087573u * s0;
    const uint32_t t1 = 2591861531u * s1;
    Xorwow s;
    s.d = 6615241u + t1 + t0;
    s.v0 = 123456789u + t0;
    s.v1 = 362436069u ^ t0;
    s.v2 = 521288629u + t1;
    s.v3 = 88675123u ^ t1;
    s.v4 = 5783321u + t0;
    return s;
}

PT_DEV uint32_t xorwow_next(Xorwow& s)
{
    const uint32_t t = s.v0 ^ (s.v0 >> 2);
    s.v0 = s.v1;
    s.v1 = s.v2;
    s.v2 = s.v3;
    s.v3 = s.v4;
    s.v4 = (s.v4 ^ (s.v4 << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return s.v4 + s.d;
}

PT_DEV float uniform(Xorwow& s)   // curand_uniform: (0, 1]
{
    return (float)xorwow_next(s) * 2.3283064e-10f + (2.3283064e-10f / 2.0f);
}

// Advance by `draws` outputs (the values are not needed).  Used for the start states of speculative
// sample groups; the draw count between two states of one stream is recovered from the Weyl word d,
// which advances by 362437 per draw: draws = (d1 - d0) * kInvWeyl (mod 2^32).
constexpr uint32_t kInvWeyl = 0x385e5f0du;     // 362437^-1 mod 2^32

PT_DEV void xorwow_skip(Xorwow& s, uint32_t draws)
{
    for (uint32_t i = 0; i < draws; ++i) {
        const uint32_t t = s.v0 ^ (s.v0 >> 2);
        s.v0 = s.v1;
        s.v1 = s.v2;
        s.v2 = s.v3;
        s.v3 = s.v4;
        s.v4 = (s.v4 ^ (s.v4 << 4)) ^ (t ^ (t << 1));
    }
    s.d += 362437u * draws;
}

} // namespace pt
