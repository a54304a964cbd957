// Exhaustive check of smk::subpix_step (sm_common.hpp) against the integer division it replaces,
// over every (Sm - minS, Sq - minS) pair in [0, 65535]^2 and three minS offsets (the step only
// depends on the differences; the offsets exercise the int arithmetic).  Prints the mismatch count.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../stereo_match_amd/csrc/sm_common.hpp"
__global__ void k_check(unsigned long long* bad, int minS)
{
    const int a = blockIdx.x * 256 + threadIdx.x;  // Sm - minS
    unsigned long long nb = 0;
    for (int b = blockIdx.y; b < 65536; b += gridDim.y) {
        const int Sm = minS + a, Sq = minS + b;
        const int den = max(Sm + Sq - 2 * minS, 1);
        const int ref = ((Sm - Sq) * 16 + den) / (den * 2);
        nb += smk::subpix_step(Sm, Sq, minS) != ref;
    }
    if (nb) atomicAdd(bad, nb);
}
int main()
{
    unsigned long long* d;
    if (hipMalloc(&d, 8) != hipSuccess) return 1;
    int rc = 0;
    for (int minS : {0, 1234, -32768}) {
        hipMemset(d, 0, 8);
        hipLaunchKernelGGL(k_check, dim3(256, 1024), dim3(256), 0, 0, d, minS);
        unsigned long long h = 0;
        hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
        printf("minS %6d: %llu mismatches over 65536^2 pairs\n", minS, h);
        rc |= h != 0;
    }
    hipFree(d);
    return rc;
}
