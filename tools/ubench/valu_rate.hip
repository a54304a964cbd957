// Throughput of individual VALU ops on gfx950: 8 independent chains per lane,
// full occupancy.  Reports ns per wave-instruction per SIMD and relative rate.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 4096
template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed)
{
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = seed * (threadIdx.x + i + 1);
    const uint32_t s = seed | 1;
    for (int it = 0; it < ITERS; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            uint32_t v = a[i];
            if constexpr (OP == 0) v = v + s;
            else if constexpr (OP == 1) v = __builtin_amdgcn_ubfe(v, 0, 31) + __popc(v);  // bcnt path
            else if constexpr (OP == 2) v = __builtin_amdgcn_perm(v, s, 0x05040100u);
            else if constexpr (OP == 3) { uint32_t t; asm volatile("v_min3_u32 %0, %1, %2, %3" : "=v"(t) : "v"(v), "s"(s), "v"(a[(i + 1) & 7])); v = t; }
            else if constexpr (OP == 4) v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));
            else if constexpr (OP == 5) { uint32_t t; asm volatile("v_bcnt_u32_b32 %0, %1, %2" : "=v"(t) : "v"(v), "v"(a[(i+3)&7])); v = t; }
            else if constexpr (OP == 6) { uint32_t t; asm volatile("v_xor_b32 %0, %1, %2" : "=v"(t) : "v"(v), "v"(a[(i+3)&7])); v = t; }
            else if constexpr (OP == 7) { uint32_t t; asm volatile("v_add_u32 %0, %1, %2" : "=v"(t) : "v"(v), "v"(a[(i+3)&7])); v = t; }
            else if constexpr (OP == 8) { uint32_t t; asm volatile("v_pk_add_u16 %0, %1, %2" : "=v"(t) : "v"(v), "v"(a[(i+3)&7])); v = t; }
            else if constexpr (OP == 9) { uint32_t t; asm volatile("v_pk_min_u16 %0, %1, %2" : "=v"(t) : "v"(v), "v"(a[(i+3)&7])); v = t; }
            else if constexpr (OP == 10) { uint32_t t; asm volatile("v_min_u32 %0, %1, %2" : "=v"(t) : "v"(v), "v"(a[(i+3)&7])); v = t; }
            else if constexpr (OP == 11) { uint32_t t; asm volatile("v_alignbit_b32 %0, %1, %2, 16" : "=v"(t) : "v"(v), "v"(a[(i+3)&7])); v = t; }
            else if constexpr (OP == 12) { uint32_t t; asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(t) : "v"(v), "v"(a[(i+3)&7]), "v"(a[(i+5)&7])); v = t; }
            else if constexpr (OP == 13) { uint32_t t; asm volatile("v_min_u16 %0, %1, %2" : "=v"(t) : "v"(v), "v"(a[(i+3)&7])); v = t; }
            else if constexpr (OP == 14) { uint32_t t; asm volatile("v_pk_sub_u16 %0, %1, %2" : "=v"(t) : "v"(v), "v"(a[(i+3)&7])); v = t; }
            else if constexpr (OP == 15) { uint32_t t; asm volatile("v_sub_u32 %0, %1, %2" : "=v"(t) : "v"(v), "v"(a[(i+3)&7])); v = t; }
            a[i] = v;
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) r ^= a[i];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int OP>
float run(uint32_t* d, int blocks)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 3u);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 5u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main()
{
    const int blocks = 256 * 8;  // 8 WGs of 4 waves per CU -> 8 waves/SIMD
    uint32_t* d;
    (void)hipMalloc(&d, blocks * 256 * 4);
    const char* names[] = {"v_add (compiler)", "ubfe+bcnt (compiler)", "v_perm", "v_min3 (asm)", "v_min_dpp fused",
                           "v_bcnt (asm)", "v_xor (asm)", "v_add (asm)", "v_pk_add_u16", "v_pk_min_u16", "v_min_u32",
                           "v_alignbit_b32", "v_add3_u32", "v_min_u16", "v_pk_sub_u16", "v_sub_u32"};
    float t[16] = {run<0>(d, blocks),  run<1>(d, blocks),  run<2>(d, blocks),  run<3>(d, blocks),
                   run<4>(d, blocks),  run<5>(d, blocks),  run<6>(d, blocks),  run<7>(d, blocks),
                   run<8>(d, blocks),  run<9>(d, blocks),  run<10>(d, blocks), run<11>(d, blocks),
                   run<12>(d, blocks), run<13>(d, blocks), run<14>(d, blocks), run<15>(d, blocks)};
    const double waves = blocks * 4.0, instr = (double)ITERS * 8;  // per wave (approx, 1 op per chain step)
    for (int i = 0; i < 16; i++) {
        const double per_simd = waves * instr / 1024.0;  // wave-instrs per SIMD
        printf("%-24s %8.3f ms  %6.2f cycles/wave-instr/SIMD @2.4GHz\n", names[i], t[i], t[i] * 1e-3 * 2.4e9 / per_simd);
    }
    return 0;
}
