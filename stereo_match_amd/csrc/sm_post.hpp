// sm_post.hpp — 3x3 median (cv::medianBlur ksize 3, replicate border) and fill.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smk {

// -------------------------------------------------------------- median ---
__device__ __forceinline__ void cswap(int& a, int& b)
{
    const int t = min(a, b);
    b = max(a, b);
    a = t;
}

// blockIdx.z = pair; dst pairs are dst_pair elements apart
__global__ void __launch_bounds__(256) k_median3(const int16_t* __restrict__ src, int16_t* __restrict__ dst, int H, int W,
                                                 size_t dst_pair)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    src += (size_t)blockIdx.z * H * W;
    dst += (size_t)blockIdx.z * dst_pair;
    int p[9];
    int k = 0;
#pragma unroll
    for (int dy = -1; dy <= 1; dy++)
#pragma unroll
        for (int dx = -1; dx <= 1; dx++)
            p[k++] = src[(size_t)min(max(y + dy, 0), H - 1) * W + min(max(x + dx, 0), W - 1)];
    // median-of-9 sorting network (Paeth / Devillard)
    cswap(p[1], p[2]); cswap(p[4], p[5]); cswap(p[7], p[8]);
    cswap(p[0], p[1]); cswap(p[3], p[4]); cswap(p[6], p[7]);
    cswap(p[1], p[2]); cswap(p[4], p[5]); cswap(p[7], p[8]);
    cswap(p[0], p[3]); cswap(p[5], p[8]); cswap(p[4], p[7]);
    cswap(p[3], p[6]); cswap(p[1], p[4]); cswap(p[2], p[5]);
    cswap(p[4], p[7]); cswap(p[4], p[2]); cswap(p[6], p[4]);
    cswap(p[4], p[2]);
    dst[(size_t)y * W + x] = (int16_t)p[4];
}

__global__ void __launch_bounds__(256) k_fill16(int16_t* dst, size_t n, int16_t v)
{
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) dst[i] = v;
}

}  // namespace smk
