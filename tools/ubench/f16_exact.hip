// Census path values as f16 bit patterns: for integers n < 2048 the u16 pattern n is the
// f16 value n * 2^-24 (denormal below 1024, exponent 1 above), so packed f16 add / sub / min
// / minimum3 on those patterns are integer arithmetic exactly (while results stay < 2048)
// provided f16 denormals are not flushed.  Checks every (a, b) pair (and a third operand for
// minimum3) against the integer result on the device; prints mismatch counts.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(unsigned* bad)
{
    const unsigned a = blockIdx.x, b = threadIdx.x + blockIdx.y * 1024;  // a, b < 2048
    const unsigned pa = a | (b << 16), pb = b | (a << 16), pc = ((a + b) & 2047) | (((a * 7 + b) & 2047) << 16);
    unsigned add, sub, mn, mn3, mx;
    asm volatile("v_pk_add_f16 %0, %1, %2" : "=v"(add) : "v"(pa), "v"(pb));
    asm volatile("v_pk_add_f16 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(sub) : "v"(pa), "v"(pb));
    asm volatile("v_pk_min_f16 %0, %1, %2" : "=v"(mn) : "v"(pa), "v"(pb));
    asm volatile("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(mn3) : "v"(pa), "v"(pb), "v"(pc));
    asm volatile("v_pk_max_f16 %0, %1, %2" : "=v"(mx) : "v"(pa), "v"(pb));
    const unsigned c0 = pc & 0xFFFF, c1 = pc >> 16;
    unsigned e = 0;
    if (a + b < 2048 && (add & 0xFFFF) != a + b) e |= 1;
    if (a >= b && (sub & 0xFFFF) != a - b) e |= 2;
    if ((mn & 0xFFFF) != (a < b ? a : b) || (mn >> 16) != (a < b ? a : b)) e |= 4;
    const unsigned m0 = min(min(a, b), c0), m1 = min(min(a, b), c1);
    if ((mn3 & 0xFFFF) != m0 || (mn3 >> 16) != m1) e |= 8;
    if ((mx & 0xFFFF) != (a > b ? a : b)) e |= 16;
    for (int i = 0; i < 5; i++)
        if (e & (1u << i)) atomicAdd(&bad[i], 1u);
}

int main()
{
    unsigned* d;
    (void)hipMalloc(&d, 5 * 4);
    (void)hipMemset(d, 0, 5 * 4);
    hipLaunchKernelGGL(k, dim3(2048, 2), dim3(1024), 0, 0, d);
    unsigned h[5];
    (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("f16-pattern integer arithmetic over a, b < 2048: mismatches add %u sub %u min %u minimum3 %u max %u\n",
           h[0], h[1], h[2], h[3], h[4]);
    return 0;
}
