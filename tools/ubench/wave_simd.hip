// Which SIMD each wave of a 12-wave (768-thread) workgroup lands on (HW_REG_HW_ID
// bits 5:4 on gfx9-family), for the fused sweeps' role layout (sm_sweep.hpp:
// wave 0 left halo, 1..9 own, 10 right halo, 11 poller).  Prints the wave -> SIMD
// map of the first few workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(768) k(unsigned* out)
{
    if ((threadIdx.x & 63) == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // hwreg(HW_REG_HW_ID, 0, 32)
        out[blockIdx.x * 12 + threadIdx.x / 64] = hw;
    }
}

int main()
{
    unsigned* d;
    const int nb = 256;
    (void)hipMalloc(&d, nb * 12 * 4);
    hipLaunchKernelGGL(k, dim3(nb), dim3(768), 0, 0, d);
    unsigned h[nb * 12];
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    int hist[12][4] = {};
    for (int b = 0; b < nb; b++)
        for (int w = 0; w < 12; w++) hist[w][(h[b * 12 + w] >> 4) & 3]++;
    for (int b = 0; b < 4; b++) {
        printf("wg %d:", b);
        for (int w = 0; w < 12; w++) printf(" w%d:simd%u", w, (h[b * 12 + w] >> 4) & 3);
        printf("  (cu %u se %u)\n", (h[b * 12] >> 8) & 15, (h[b * 12] >> 13) & 7);
    }
    printf("wave -> SIMD histogram over %d workgroups:\n", nb);
    for (int w = 0; w < 12; w++) printf("  wave %2d: %d %d %d %d\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
    return 0;
}
