// VALU issue rate and dependent latency on gfx950, by waves per SIMD and by
// independent chains per wave: the numbers that decide whether a kernel is
// issue-bound (SIMD capacity) or latency-bound (dependent chains, too few
// waves).  One workgroup of 64*WPS*4 threads per CU (WPS waves per SIMD),
// CH independent chains per lane, ITERS steps per chain.
// Output: cycles per wave-instruction per SIMD (issue view) and cycles per
// dependent step of one chain (latency view), at 2.4 GHz.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define ITERS 65536

template <int OP, int CH>
__global__ void k(uint32_t* out, uint32_t seed)
{
    uint32_t a[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) a[i] = seed * (threadIdx.x + i + 1);
    const uint32_t s = seed | 1;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < CH; i++) {
            uint32_t v = a[i], t;
            if constexpr (OP == 0) asm volatile("v_pk_add_u16 %0, %1, %2" : "=v"(t) : "v"(v), "s"(s));
            else if constexpr (OP == 1) asm volatile("v_pk_min_u16 %0, %1, %2" : "=v"(t) : "v"(v), "s"(s));
            else if constexpr (OP == 2) asm volatile("v_add_u32 %0, %1, %2" : "=v"(t) : "s"(s), "v"(v));
            else if constexpr (OP == 3)
                asm volatile("s_nop 1\n\tv_min_u32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1"
                             : "=v"(t) : "v"(v));
            else if constexpr (OP == 4) asm volatile("v_alignbit_b32 %0, %1, %2, 16" : "=v"(t) : "v"(v), "s"(s));
            else if constexpr (OP == 6) asm volatile("v_pk_min_f16 %0, %1, %2" : "=v"(t) : "v"(v), "s"(s));
            else if constexpr (OP == 7) asm volatile("v_pk_add_f16 %0, %1, %2" : "=v"(t) : "v"(v), "s"(s));
            else if constexpr (OP == 8) asm volatile("v_pk_minimum3_f16 %0, %1, %2, %1" : "=v"(t) : "v"(v), "s"(s));
            else t = __builtin_amdgcn_perm(v, s, 0x05040100u);
            a[i] = t;
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < CH; i++) r ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int OP, int CH>
float run(uint32_t* d, int wps)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    // one CU = 4*wps waves: one workgroup per CU up to 4 waves per SIMD, two above
    const int per_cu = wps > 4 ? 2 : 1, threads = 256 * wps / per_cu;
    hipLaunchKernelGGL((k<OP, CH>), dim3(256 * per_cu), dim3(threads), 0, 0, d, 3u);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k<OP, CH>), dim3(256 * per_cu), dim3(threads), 0, 0, d, 5u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return ms;
}

template <int OP, int CH>
void row(const char* name, uint32_t* d)
{
    for (int wps : {1, 2, 3, 4, 8}) {
        const float ms = run<OP, CH>(d, wps);
        const double cyc = ms * 1e-3 * 2.4e9;
        const double per_simd = (double)wps * ITERS * CH;  // wave-instructions per SIMD (1 CU = 1 WG)
        printf("%-22s chains %d  waves/SIMD %d  %7.3f ms  %6.2f cyc/instr/SIMD  %6.2f cyc/dependent step\n", name, CH,
               wps, ms, cyc / per_simd, cyc / ITERS);
    }
}

int main()
{
    uint32_t* d;
    (void)hipMalloc(&d, 512 * 1024 * 4);
    row<0, 1>("v_pk_add_u16", d);
    row<0, 8>("v_pk_add_u16", d);
    row<1, 1>("v_pk_min_u16", d);
    row<1, 8>("v_pk_min_u16", d);
    row<2, 1>("v_add_u32", d);
    row<2, 8>("v_add_u32", d);
    row<3, 1>("s_nop1+v_min_u32_dpp", d);
    row<3, 8>("s_nop1+v_min_u32_dpp", d);
    row<4, 8>("v_alignbit_b32", d);
    row<5, 8>("v_perm_b32", d);
    row<6, 1>("v_pk_min_f16", d);
    row<6, 8>("v_pk_min_f16", d);
    row<7, 8>("v_pk_add_f16", d);
    row<8, 1>("v_pk_minimum3_f16", d);
    row<8, 8>("v_pk_minimum3_f16", d);
    (void)hipFree(d);
    return 0;
}
