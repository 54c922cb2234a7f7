// Where the hardware places the waves of a persistent trace-kernel grid: every wave records its
// hardware ids (s_getreg HW_ID and XCC_ID) and start time, for the resident grids of the five- and
// six-wave builds (dynamic LDS sized like theirs so the occupancy matches).  Build here, run on the box:
//   hipcc --offload-arch=gfx950 -O2 -o tools/hwid_probe tools/hwid_probe.hip
//   tools/hwid_probe > gpurun_out/hwid.txt   (one line per wave: wpb block wave xcc se sh cu simd t)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

__global__ void probe(uint32_t* out, int wpb)
{
    extern __shared__ uint32_t pad[];
    const uint32_t wave = threadIdx.x >> 6;
    const uint64_t t = __builtin_amdgcn_s_memtime();
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
    const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);
    if ((threadIdx.x & 63u) == 0) {
        uint32_t* o = out + ((size_t)blockIdx.x * wpb + wave) * 4;
        o[0] = hw;
        o[1] = xcc;
        o[2] = (uint32_t)t;
        o[3] = (uint32_t)(t >> 32);
        pad[wave] = hw;                       // keep the LDS allocation
    }
    // stay resident a while, so every wave of the grid is placed before any leaves
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < 2000000ull) __builtin_amdgcn_s_sleep(10);
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&probe), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    struct Cfg { int wpb; size_t lds; } cfgs[] = {{4, 31616}, {8, 53120}};
    for (const Cfg& c : cfgs) {
        int perCu = 0;
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, reinterpret_cast<const void*>(&probe), c.wpb * 64, c.lds);
        const int grid = cus * perCu;
        const size_t n = (size_t)grid * c.wpb * 4;
        uint32_t* d = nullptr;
        hipMalloc(&d, n * 4);
        hipMemset(d, 0, n * 4);
        probe<<<grid, c.wpb * 64, c.lds>>>(d, c.wpb);
        if (hipDeviceSynchronize() != hipSuccess) { fprintf(stderr, "launch failed\n"); return 1; }
        std::vector<uint32_t> h(n);
        hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
        for (int b = 0; b < grid; ++b)
            for (int w = 0; w < c.wpb; ++w) {
                const uint32_t* o = &h[((size_t)b * c.wpb + w) * 4];
                const uint32_t hw = o[0];
                printf("%d %d %d %u %u %u %u %u %llu\n", c.wpb, b, w, o[1] & 0xf, (hw >> 13) & 7, (hw >> 12) & 1,
                       (hw >> 8) & 0xf, (hw >> 4) & 3, (unsigned long long)o[2] | ((unsigned long long)o[3] << 32));
            }
        hipFree(d);
        fprintf(stderr, "wpb %d: %d per CU, grid %d\n", c.wpb, perCu, grid);
    }
    return 0;
}
