// Exhaustive proof (all 2^32 float inputs, on the GPU) that the kernel's short reciprocal and
// square root (pt::rcp_rn, pt::sqrt_rn in pathtracercuda_amd/csrc/pt_math.h) return exactly the
// correctly rounded 1.0f / x and sqrtf(x) of hipcc's full-precision expansions, plus diagnostics
// showing why the fast sequences need their input-range guards.  NaN results compare as "both
// NaN".  Built by `make` into pathtracercuda_amd/lib/fp_exhaustive; tests/test_gpu_parity.py runs
// it; profiles/r01_fp_exhaustive.json holds a recorded output.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../pathtracercuda_amd/csrc/pt_math.h"

#define NSEQ 16
__device__ unsigned long long g_bad[NSEQ];
__device__ uint32_t g_first[NSEQ][8];

__device__ __forceinline__ bool same(float a, float b)
{
    return (a != a && b != b) || __float_as_uint(a) == __float_as_uint(b);
}

__device__ __forceinline__ void check_one(int k, bool ok, uint32_t x)
{
    if (ok) return;
    const unsigned long long n = atomicAdd(&g_bad[k], 1ull);
    if (n < 8) g_first[k][n] = x;
}

__global__ void check(uint32_t base)
{
    const uint32_t xb = base + blockIdx.x * blockDim.x + threadIdx.x;
    const float x = __uint_as_float(xb);
    const float ref_rcp = 1.0f / x;
    const float ref_sqrt = sqrtf(x);
    // the shipped functions, every input
    check_one(0, same(pt::rcp_rn(x), ref_rcp), xb);
    check_one(1, same(pt::sqrt_rn(x), ref_sqrt), xb);
    // diagnostics: the unguarded fast sequences over all inputs
    const float y = __builtin_amdgcn_rcpf(x);
    check_one(2, same(y, ref_rcp), xb);
    const float r1 = __builtin_fmaf(__builtin_fmaf(-x, y, 1.0f), y, y);
    check_one(3, same(r1, ref_rcp), xb);
    const float s = __builtin_amdgcn_sqrtf(x);
    check_one(4, same(s, ref_sqrt), xb);
    const float ry = __builtin_amdgcn_rsqf(x);
    const float s0 = x * ry;
    const float sc = __builtin_fmaf(__builtin_fmaf(-s0, s0, x), 0.5f * ry, s0);
    check_one(5, same(sc, ref_sqrt), xb);
    // x / pi and x / (2 pi) (the sky's theta / PI, phi / (2 PI), the cosine pdf z / PI)
    check_one(6, same(pt::div_pi(x), x / pt::kPi), xb);
    check_one(7, same(pt::div_two_pi(x), x / pt::kTwoPi), xb);
    // the wave-uniform-guard forms (pt_math.h *_u) used by the select-form primitive test
    check_one(8, same(pt::rcp_rn_u(x), ref_rcp), xb);
    check_one(9, same(pt::sqrt_rn_u(x), ref_sqrt), xb);
    // select forms of acos / atan (kernel sky lookup and uv) against the branchy forms the oracle
    // restates: bit for bit, NaN payloads included; atan2 with every x in each argument position,
    // paired with a hashed other argument (all bit patterns occur, specials included)
    check_one(10, __float_as_uint(pt::acos_sel(x)) == __float_as_uint(pt::acos_(x)), xb);
    check_one(11, __float_as_uint(pt::atan_pos_sel(x)) == __float_as_uint(pt::atan_pos(x)), xb);
    const float h = __uint_as_float((xb * 2654435761u) ^ 0x9e3779b9u);
    check_one(12, __float_as_uint(pt::atan2_sel(x, h)) == __float_as_uint(pt::atan2_(x, h)), xb);
    check_one(13, __float_as_uint(pt::atan2_sel(h, x)) == __float_as_uint(pt::atan2_(h, x)), xb);
    // sqrt_dom (guard-free root for operands that are +0, NaN or in [2^-96, FLT_MAX]): bit for bit,
    // NaN payloads included, against sqrtf on that domain.  The operands are results of arithmetic,
    // so their NaNs are quiet (signalling ones, which sqrtf would quiet, never reach it).
    const bool qnan = x != x && (xb & 0x00400000u) != 0u;
    const bool dom = xb == 0u || qnan || (xb - 0x0f800000u <= 0x7f7fffffu - 0x0f800000u);
    check_one(14, !dom || __float_as_uint(pt::sqrt_dom(x)) == __float_as_uint(ref_sqrt), xb);
    // normalize_dom's NaN rule: 1 / sqrtf(NaN) through the general path is that same (quiet) NaN
    check_one(15, !qnan || __float_as_uint(pt::rcp_rn(sqrtf(x))) == xb, xb);
}

int main()
{
    unsigned long long zero[NSEQ] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_bad), zero, sizeof(zero)) != hipSuccess) return 2;
    const uint32_t threads = 256, blocks = 1u << 16;       // 2^24 inputs per launch
    for (uint64_t base = 0; base < (1ull << 32); base += (uint64_t)threads * blocks)
        check<<<blocks, threads>>>((uint32_t)base);
    if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"kernel failed\"}\n"); return 1; }
    unsigned long long bad[NSEQ];
    uint32_t first[NSEQ][8];
    if (hipMemcpyFromSymbol(bad, HIP_SYMBOL(g_bad), sizeof(bad)) != hipSuccess) return 2;
    if (hipMemcpyFromSymbol(first, HIP_SYMBOL(g_first), sizeof(first)) != hipSuccess) return 2;
    const char* names[NSEQ] = {"rcp_rn", "sqrt_rn", "diag_rcp_raw_all_inputs", "diag_rcp_newton_unguarded",
                               "diag_sqrt_raw_all_inputs", "diag_sqrt_rsq_newton_unguarded", "div_pi", "div_two_pi",
                               "rcp_rn_u", "sqrt_rn_u", "acos_sel", "atan_pos_sel", "atan2_sel_y", "atan2_sel_x",
                               "sqrt_dom", "nan_through_rcp_sqrt"};
    printf("{\n  \"inputs\": 4294967296,\n");
    for (int k = 0; k < NSEQ; ++k) {
        printf("  \"%s\": {\"mismatches\": %llu, \"first\": [", names[k], bad[k]);
        for (int i = 0; i < 8 && (unsigned long long)i < bad[k]; ++i) printf("%s\"0x%08x\"", i ? ", " : "", first[k][i]);
        printf("]}%s\n", k + 1 < NSEQ ? "," : "");
    }
    printf("}\n");
    return 0;
}
