// HBM store bandwidth on one MI355X: 16-byte-per-lane streaming stores (plain and
// nontemporal) over a 512 MB buffer, grid sizes from 1 to 16 workgroups per CU.
// Decides whether a store-heavy kernel (the census cost volume) is VALU- or store-bound.
#include <hip/hip_runtime.h>
#include <stdio.h>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
template <bool NT>
__global__ void __launch_bounds__(256) k_write(uint4* p, size_t n, uint32_t v)
{
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        if (NT) __builtin_nontemporal_store(v4u{v, v + 1, v + 2, (uint32_t)i}, reinterpret_cast<v4u*>(p + i));
        else p[i] = make_uint4(v, v + 1, v + 2, (uint32_t)i);
    }
}
int main()
{
    const size_t bytes = 512ull << 20, n = bytes / 16;
    uint4* p;
    CK(hipMalloc(&p, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int nt = 0; nt < 2; nt++)
        for (int wpc : {2, 4, 8, 16}) {
            const int grid = 256 * wpc;
            for (int r = 0; r < 3; r++) {
                if (nt) hipLaunchKernelGGL(k_write<true>, dim3(grid), dim3(256), 0, 0, p, n, 1u);
                else hipLaunchKernelGGL(k_write<false>, dim3(grid), dim3(256), 0, 0, p, n, 1u);
            }
            CK(hipEventRecord(a));
            const int reps = 20;
            for (int r = 0; r < reps; r++) {
                if (nt) hipLaunchKernelGGL(k_write<true>, dim3(grid), dim3(256), 0, 0, p, n, (uint32_t)r);
                else hipLaunchKernelGGL(k_write<false>, dim3(grid), dim3(256), 0, 0, p, n, (uint32_t)r);
            }
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            printf("write %s  WG/CU %2d  %.1f us per 512 MB  %.2f TB/s\n", nt ? "nt   " : "plain", wpc, ms * 1e3 / reps,
                   bytes * reps / (ms * 1e-3) / 1e12);
        }
    CK(hipFree(p));
    return 0;
}
