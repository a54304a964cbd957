// Exhaustive check: is y1 = fma(fma(-t, y0, 1), y0, y0), y0 = v_rcp_f32(t), equal to the
// correctly rounded 1.0f / t for every float mantissa (t in [1, 2)) and a few exponents?
// hipcc --offload-arch=gfx950 -O3 tools/ubench/rcp_exact.hip -o /tmp/rcp_exact
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned* bad, unsigned* first, int e)
{
#pragma clang fp contract(off)
    const unsigned m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    const float t = __uint_as_float(((unsigned)(127 + e) << 23) | m);
    const float ref = 1.0f / t;
    const float y0 = __builtin_amdgcn_rcpf(t);
    const float r = __builtin_fmaf(-t, y0, 1.0f);
    const float y1 = __builtin_fmaf(r, y0, y0);
    if (__float_as_uint(y1) != __float_as_uint(ref)) {
        atomicAdd(bad, 1u);
        atomicMin(first, m);
    }
}

int main()
{
    unsigned *bad, *first;
    hipMalloc(&bad, 4);
    hipMalloc(&first, 4);
    int exps[24];
    for (int i = 0; i < 24; i++) exps[i] = i;
    unsigned total = 0;
    for (int e : exps) {
        unsigned z = 0, f = 0xFFFFFFFFu, hb = 0, hf = 0;
        hipMemcpy(bad, &z, 4, hipMemcpyHostToDevice);
        hipMemcpy(first, &f, 4, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k, dim3((1u << 23) / 256), dim3(256), 0, 0, bad, first, e);
        hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
        hipMemcpy(&hf, first, 4, hipMemcpyDeviceToHost);
        printf("exponent 2^%d: %u mismatches (first mantissa 0x%06x)\n", e, hb, hf);
        total += hb;
    }
    printf("total mismatches %u\n", total);
    return 0;
}
