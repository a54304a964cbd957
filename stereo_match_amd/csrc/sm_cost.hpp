// sm_cost.hpp — matching-cost kernels: census 9x7 (north-star mode) and the
// OpenCV StereoSGBM cost (Sobel-x clip + raw channel Birchfield-Tomasi, box
// sum with OpenCV's clamped borders and frozen bottom rows).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_common.hpp"

namespace smk {

// -------------------------------------------------------------- census ---
// 9x7 census, clamped borders, bit k = I[n_k] < I[c] (row-major, centre
// skipped).  Tile 32x8 pixels + halo staged in LDS.  blockIdx.z = 2*pair + image.
struct CensusArgs {
    const uint8_t* img[2];  // pair 0 left / right
    uint64_t* out[2];       // census left / right [pair][H][W]
    size_t in_pair;         // bytes between consecutive pairs' images
    int H, W, stride;
};

constexpr int CT_W = 32, CT_H = 8;

__global__ void __launch_bounds__(256) k_census9x7(CensusArgs a)
{
    __shared__ uint8_t tile[CT_H + 6][CT_W + 8];
    const int which = blockIdx.z & 1, pair = blockIdx.z >> 1;
    const uint8_t* img = a.img[which] + (size_t)pair * a.in_pair;
    const int x0 = blockIdx.x * CT_W, y0 = blockIdx.y * CT_H;
    for (int i = threadIdx.x; i < (CT_H + 6) * (CT_W + 8); i += 256) {
        int ty = i / (CT_W + 8), tx = i % (CT_W + 8);
        int y = min(max(y0 + ty - 3, 0), a.H - 1), x = min(max(x0 + tx - 4, 0), a.W - 1);
        tile[ty][tx] = img[(size_t)y * a.stride + x];
    }
    __syncthreads();
    const int tx = threadIdx.x % CT_W, ty = threadIdx.x / CT_W;
    const int x = x0 + tx, y = y0 + ty;
    if (x >= a.W || y >= a.H) return;
    const int c = tile[ty + 3][tx + 4];
    uint64_t v = 0;
    int k = 0;
#pragma unroll
    for (int dy = 0; dy < 7; dy++)
#pragma unroll
        for (int dx = 0; dx < 9; dx++) {
            if (dy == 3 && dx == 4) continue;
            v |= (uint64_t)(tile[ty + dy][tx + dx] < c) << k;
            k++;
        }
    a.out[which][(size_t)pair * a.H * a.W + (size_t)y * a.W + x] = v;
}

// Hamming cost volume C[y][x1][d] = popcount(cl[y][X] ^ cr[y][X-minD-d]),
// X = x1 + minX1.  One thread per (y, x1, 8 disparities).
struct CensusCostArgs {
    const uint64_t* cl;
    const uint64_t* cr;
    uint8_t* C;
    int H, W, width1, D, minD, minX1;
};

__global__ void __launch_bounds__(256) k_census_cost(CensusCostArgs a)
{
    const int chunks = a.D / 8;
    const size_t n = (size_t)a.H * a.width1 * chunks;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        int ch = (int)(i % chunks);
        size_t pix = i / chunks;
        int x1 = (int)(pix % a.width1), y = (int)(pix / a.width1);
        int X = x1 + a.minX1;
        uint64_t l = a.cl[(size_t)y * a.W + X];
        const uint64_t* r = a.cr + (size_t)y * a.W + X - a.minD - ch * 8;
        uint2 w;
        uint8_t* b = reinterpret_cast<uint8_t*>(&w);
#pragma unroll
        for (int j = 0; j < 8; j++) b[j] = (uint8_t)__popcll(l ^ r[-j]);
        *reinterpret_cast<uint2*>(a.C + pix * a.D + ch * 8) = w;
    }
}

// ---------------------------------------------------------- SGBM cost ---
// Planes[img][ch][k][H][W] (u8): ch 0 = clipped Sobel-x, ch 1 = raw (both
// forced to ftzero at x = 0 and x = W-1); k 0 = value, 1 = BT min, 2 = BT max.
struct PrefilterArgs {
    const uint8_t* img[2];
    uint8_t* planes;
    int H, W, stride, ftzero;
};

__device__ __forceinline__ int sobel_clip(const uint8_t* img, int stride, int H, int W, int y, int x, int ftzero)
{
    if (x <= 0 || x >= W - 1) return ftzero;
    const uint8_t* r = img + (size_t)y * stride;
    const uint8_t* rn = img + (size_t)max(y - 1, 0) * stride;
    const uint8_t* rs = img + (size_t)min(y + 1, H - 1) * stride;
    int v = (r[x + 1] - r[x - 1]) * 2 + rn[x + 1] - rn[x - 1] + rs[x + 1] - rs[x - 1];
    return min(max(v, -ftzero), ftzero) + ftzero;
}

__device__ __forceinline__ int raw_px(const uint8_t* img, int stride, int W, int y, int x, int ftzero)
{
    if (x <= 0 || x >= W - 1) return ftzero;
    return img[(size_t)y * stride + x];
}

__global__ void __launch_bounds__(256) k_sgbm_prefilter(PrefilterArgs a)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, im = blockIdx.z;
    if (x >= a.W) return;
    const uint8_t* img = a.img[im];
    const size_t plane = (size_t)a.H * a.W;
    for (int ch = 0; ch < 2; ch++) {
        int v, vl, vr;
        if (ch == 0) {
            v = sobel_clip(img, a.stride, a.H, a.W, y, x, a.ftzero);
            vl = x > 0 ? (v + sobel_clip(img, a.stride, a.H, a.W, y, x - 1, a.ftzero)) / 2 : v;
            vr = x < a.W - 1 ? (v + sobel_clip(img, a.stride, a.H, a.W, y, x + 1, a.ftzero)) / 2 : v;
        } else {
            v = raw_px(img, a.stride, a.W, y, x, a.ftzero);
            vl = x > 0 ? (v + raw_px(img, a.stride, a.W, y, x - 1, a.ftzero)) / 2 : v;
            vr = x < a.W - 1 ? (v + raw_px(img, a.stride, a.W, y, x + 1, a.ftzero)) / 2 : v;
        }
        uint8_t* base = a.planes + ((size_t)(im * 2 + ch) * 3) * plane + (size_t)y * a.W + x;
        base[0] = (uint8_t)v;
        base[plane] = (uint8_t)min(min(vl, vr), v);
        base[2 * plane] = (uint8_t)max(max(vl, vr), v);
    }
}

__device__ __forceinline__ int bt_pix(const uint8_t* planes, size_t plane, int W, int y, int X, int xr)
{
    int acc = 0;
#pragma unroll
    for (int ch = 0; ch < 2; ch++) {
        const uint8_t* L = planes + ((size_t)(0 * 2 + ch) * 3) * plane + (size_t)y * W;
        const uint8_t* R = planes + ((size_t)(1 * 2 + ch) * 3) * plane + (size_t)y * W;
        int u = L[X], u0 = L[plane + X], u1 = L[2 * plane + X];
        int v = R[xr], v0 = R[plane + xr], v1 = R[2 * plane + xr];
        int c0 = max(max(0, u - v1), v0 - u);
        int c1 = max(max(0, v - u1), u0 - v);
        acc += min(c0, c1) >> (ch == 0 ? 0 : 2);
    }
    return acc;
}

// hsum[y][x1][d] = sum_{j=-SW2..SW2} pix(y, clamp(x1+j, 0, width1-1), d)
struct HsumArgs {
    const uint8_t* planes;
    uint16_t* hsum;
    int H, W, width1, D, minD, minX1, SW2;
};

__global__ void __launch_bounds__(256) k_sgbm_hsum(HsumArgs a)
{
    const size_t plane = (size_t)a.H * a.W;
    const size_t n = (size_t)a.H * a.width1 * a.D;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        int d = (int)(i % a.D);
        size_t pix = i / a.D;
        int x1 = (int)(pix % a.width1), y = (int)(pix / a.width1);
        int acc = 0;
        for (int j = -a.SW2; j <= a.SW2; j++) {
            int X = min(max(x1 + j, 0), a.width1 - 1) + a.minX1;
            acc += bt_pix(a.planes, plane, a.W, y, X, X - a.minD - d);
        }
        a.hsum[i] = (uint16_t)acc;
    }
}

// C_true[y] = wrap16(sum_{k=yc-SH2..yc+SH2} hsum[clamp(k)]), yc = clamp(y, 0, H-1-SH2);
// MODE_HH leaves rows y >= 1, y > H-1-SH2 at the P2 seed (C_true = 0).
struct VsumArgs {
    const uint16_t* hsum;
    uint16_t* C;
    int H, width1, D, SH2, hh;
};

__global__ void __launch_bounds__(256) k_sgbm_vsum(VsumArgs a)
{
    const size_t row = (size_t)a.width1 * a.D;
    const size_t n = (size_t)a.H * row;
    const int last = a.H - 1 - a.SH2;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        int y = (int)(i / row);
        size_t r = i % row;
        if (a.hh && y >= 1 && y > last) {
            a.C[i] = 0;
            continue;
        }
        int yc = max(0, min(y, last));
        int acc = 0;
        for (int k = yc - a.SH2; k <= yc + a.SH2; k++) acc += a.hsum[(size_t)min(max(k, 0), a.H - 1) * row + r];
        a.C[i] = (uint16_t)(int16_t)acc;
    }
}

}  // namespace smk
