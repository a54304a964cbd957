// sm_kernels.hpp — CDNA4 (gfx950) kernels of the stereo disparity hot path.
//
// Pipeline per pair:
//   cost   : census9x7 -> Hamming cost volume   (north-star mode)
//            or Sobel/BT prefilter -> hsum -> vsum box cost (OpenCV parity mode)
//   paths  : ONE launch aggregates every SGM direction; a "line" (row, column
//            or wrapped diagonal) is owned by one 16-lane DPP row, each lane
//            holding D/16 consecutive disparities; min over d is a 4-step DPP
//            butterfly, d±1 neighbours cross lanes with row_shr/row_shl.
//   wta    : one workgroup per image row: sum of the path volumes, first
//            argmin, uniqueness, integer sub-pixel, right-view disp2 in LDS
//            (atomicMin on a (minS, -x) key), disp12MaxDiff check.
//   median : 3x3 median, replicate border.
//
// Semantics: OpenCV StereoSGBM (restated in oracle/sgm_np.py; references in
// DESIGN.md).  All volumes are [y][x1][d] with d fastest, x1 in the OpenCV
// domain [minX1, maxX1).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smk {

constexpr int kMaxDirs = 8;
constexpr int kLineLanes = 16;  // one DPP row per line
constexpr uint32_t kBig = 0x7FFF;  // OpenCV MAX_COST used at d = -1 / d = D

// ----------------------------------------------------------------- DPP ---
enum : int {
    DPP_QP_XOR1 = 0xB1,          // quad_perm [1,0,3,2]
    DPP_QP_XOR2 = 0x4E,          // quad_perm [2,3,0,1]
    DPP_ROW_SHL1 = 0x101,        // lane i <- lane i+1 (within 16-lane row)
    DPP_ROW_SHR1 = 0x111,        // lane i <- lane i-1
    DPP_ROW_MIRROR = 0x140,      // lane i <- lane 15-i
    DPP_ROW_HALF_MIRROR = 0x141  // lane i <- lane 7-i (per 8-lane half)
};

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t src)
{
    // bound_ctrl = false: lanes whose source is outside the row keep `old`.
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)src, CTRL, 0xF, 0xF, false);
}

__device__ __forceinline__ uint32_t row16_min(uint32_t v)
{
    v = min(v, dpp<DPP_QP_XOR1>(v, v));
    v = min(v, dpp<DPP_QP_XOR2>(v, v));
    v = min(v, dpp<DPP_ROW_HALF_MIRROR>(v, v));
    v = min(v, dpp<DPP_ROW_MIRROR>(v, v));
    return v;
}

__device__ __forceinline__ uint32_t row16_or(uint32_t v)
{
    v |= dpp<DPP_QP_XOR1>(v, v);
    v |= dpp<DPP_QP_XOR2>(v, v);
    v |= dpp<DPP_ROW_HALF_MIRROR>(v, v);
    v |= dpp<DPP_ROW_MIRROR>(v, v);
    return v;
}

// ------------------------------------------------------ vector load/store
template <typename T, int N>
struct Vec {
    T v[N];
};

template <int N, typename T>
__device__ __forceinline__ void load_n(const T* __restrict__ p, uint32_t (&out)[N])
{
    constexpr int BYTES = N * (int)sizeof(T);
    if constexpr (BYTES % 16 == 0) {
#pragma unroll
        for (int c = 0; c < BYTES / 16; c++) {
            uint4 w = reinterpret_cast<const uint4*>(p)[c];
            const T* t = reinterpret_cast<const T*>(&w);
#pragma unroll
            for (int i = 0; i < 16 / (int)sizeof(T); i++) out[c * (16 / sizeof(T)) + i] = t[i];
        }
    } else if constexpr (BYTES % 8 == 0) {
#pragma unroll
        for (int c = 0; c < BYTES / 8; c++) {
            uint2 w = reinterpret_cast<const uint2*>(p)[c];
            const T* t = reinterpret_cast<const T*>(&w);
#pragma unroll
            for (int i = 0; i < 8 / (int)sizeof(T); i++) out[c * (8 / sizeof(T)) + i] = t[i];
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; i++) out[i] = p[i];
    }
}

template <int N, typename T>
__device__ __forceinline__ void store_n(T* __restrict__ p, const uint32_t (&in)[N])
{
    constexpr int BYTES = N * (int)sizeof(T);
    if constexpr (BYTES % 16 == 0) {
#pragma unroll
        for (int c = 0; c < BYTES / 16; c++) {
            uint4 w;
            T* t = reinterpret_cast<T*>(&w);
#pragma unroll
            for (int i = 0; i < 16 / (int)sizeof(T); i++) t[i] = (T)in[c * (16 / sizeof(T)) + i];
            reinterpret_cast<uint4*>(p)[c] = w;
        }
    } else if constexpr (BYTES % 8 == 0) {
#pragma unroll
        for (int c = 0; c < BYTES / 8; c++) {
            uint2 w;
            T* t = reinterpret_cast<T*>(&w);
#pragma unroll
            for (int i = 0; i < 8 / (int)sizeof(T); i++) t[i] = (T)in[c * (8 / sizeof(T)) + i];
            reinterpret_cast<uint2*>(p)[c] = w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < N; i++) p[i] = (T)in[i];
    }
}

// -------------------------------------------------------------- census ---
// 9x7 census, clamped borders, bit k = I[n_k] < I[c] (row-major, centre
// skipped).  Tile 32x8 pixels + halo staged in LDS.  blockIdx.z = image.
struct CensusArgs {
    const uint8_t* img[2];
    uint64_t* out[2];
    int H, W, stride;
};

constexpr int CT_W = 32, CT_H = 8;

__global__ void __launch_bounds__(256) k_census9x7(CensusArgs a)
{
    __shared__ uint8_t tile[CT_H + 6][CT_W + 8];
    const uint8_t* img = a.img[blockIdx.z];
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
    a.out[blockIdx.z][(size_t)y * a.W + x] = v;
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

// ----------------------------------------------------- path aggregation ---
struct PathArgs {
    const void* cost;  // [H][width1][D] CT
    void* L;           // [ndirs][H][width1][D] LT
    size_t vol;        // H*width1*D
    int H, width1, D, P1, P2, ndirs;
    int dx[kMaxDirs], dy[kMaxDirs];
    int blk_start[kMaxDirs + 1];
};

// L(p,d) = C(p,d) + min(Lp[d], min(Lp[d-1], Lp[d+1]) + P1, minLp + P2) - minLp
// (== OpenCV's Cbuf(+P2) form).  Line starts: Lp = 0, minLp = 0.
template <int DPL, typename CT, typename LT>
__global__ void __launch_bounds__(256) k_sgm_paths(PathArgs a)
{
    const int b = blockIdx.x;
    int k = 0;
#pragma unroll
    for (int i = 1; i < kMaxDirs; i++)
        if (i < a.ndirs && b >= a.blk_start[i]) k = i;
    const int dx = a.dx[k], dy = a.dy[k];
    const int g = threadIdx.x & (kLineLanes - 1);
    const int line = (b - a.blk_start[k]) * (256 / kLineLanes) + (int)(threadIdx.x / kLineLanes);
    const int H = a.H, W1 = a.width1, D = a.D;
    const int nlines = dy == 0 ? H : W1;
    if (line >= nlines) return;  // uniform per 16-lane row
    const int nsteps = dy == 0 ? W1 : H;
    const CT* __restrict__ cost = (const CT*)a.cost + g * DPL;
    LT* __restrict__ Lout = (LT*)a.L + (size_t)k * a.vol + g * DPL;
    const uint32_t P1 = (uint32_t)a.P1, P2 = (uint32_t)a.P2;

    uint32_t Lp[DPL];
#pragma unroll
    for (int i = 0; i < DPL; i++) Lp[i] = 0;
    uint32_t minLp = 0;

    int x, y;
    if (dy == 0) {
        y = line;
        x = dx > 0 ? 0 : W1 - 1;
    } else {
        y = dy > 0 ? 0 : H - 1;
        x = line;
    }
    for (int s = 0; s < nsteps; s++) {
        if (s > 0) {
            if (dy == 0) {
                x += dx;
            } else {
                y += dy;
                x += dx;
                if (x >= W1) x = 0;
                if (x < 0) x = W1 - 1;
                const bool wrapped = (dx > 0 && x == 0) || (dx < 0 && x == W1 - 1);
                if (wrapped) {
#pragma unroll
                    for (int i = 0; i < DPL; i++) Lp[i] = 0;
                    minLp = 0;
                }
            }
        }
        const size_t off = ((size_t)y * W1 + x) * D;
        uint32_t C[DPL];
        load_n<DPL>(cost + off, C);
        const uint32_t lm = dpp<DPP_ROW_SHR1>(kBig, Lp[DPL - 1]);
        const uint32_t lq = dpp<DPP_ROW_SHL1>(kBig, Lp[0]);
        const uint32_t delta = minLp + P2;
        uint32_t Ln[DPL];
        uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            const uint32_t a1 = i == 0 ? lm : Lp[i - 1];
            const uint32_t a2 = i == DPL - 1 ? lq : Lp[i + 1];
            uint32_t v = min(min(a1, a2) + P1, Lp[i]);
            v = min(v, delta);
            Ln[i] = C[i] + v - minLp;
            mn = min(mn, Ln[i]);
        }
        store_n<DPL>(Lout + off, Ln);
#pragma unroll
        for (int i = 0; i < DPL; i++) Lp[i] = Ln[i];
        minLp = row16_min(mn);
    }
}

// ----------------------------------------------------------------- WTA ---
struct WtaArgs {
    const void* L;
    size_t vol;
    int ndirs;
    int H, W, width1, D, minD, minX1, uniq, disp12;
    int16_t* disp;  // [H][W] pre-median
};

template <int DPL, typename LT>
__global__ void __launch_bounds__(256) k_wta(WtaArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int W = a.W, D = a.D, minD = a.minD, minX1 = a.minX1;
    const int maxX1 = minX1 + a.width1;
    const int INVALID = (minD - 1) * 16;
    uint32_t* key2 = smem;
    int* drow = reinterpret_cast<int*>(smem + W);
    const int y = blockIdx.x;
    for (int i = threadIdx.x; i < W; i += 256) {
        key2[i] = 0xFFFFFFFFu;
        drow[i] = INVALID;
    }
    __syncthreads();
    const int g = threadIdx.x & (kLineLanes - 1);
    const int grp = threadIdx.x / kLineLanes;
    const LT* __restrict__ Lb = (const LT*)a.L + g * DPL;
    const int u = a.uniq;
    for (int x = grp; x < a.width1; x += 256 / kLineLanes) {
        const size_t off = ((size_t)y * a.width1 + x) * D;
        uint32_t S[DPL];
#pragma unroll
        for (int i = 0; i < DPL; i++) S[i] = 0;
        for (int k = 0; k < a.ndirs; k++) {
            uint32_t t[DPL];
            load_n<DPL>(Lb + (size_t)k * a.vol + off, t);
#pragma unroll
            for (int i = 0; i < DPL; i++) S[i] += t[i];
        }
        uint32_t key = 0xFFFFFFFFu;
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            S[i] = min(S[i], 32767u);
            key = min(key, (S[i] << 16) | (uint32_t)(g * DPL + i));
        }
        key = row16_min(key);
        const int minS = (int)(key >> 16), best = (int)(key & 0xFFFF);
        uint32_t bad = 0, nb = 0;
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            const int d = g * DPL + i;
            const int dd = best - d;
            bad |= ((int)S[i] * (100 - u) < minS * 100 && (dd > 1 || dd < -1)) ? 1u : 0u;
            nb |= d == best - 1 ? S[i] : 0u;
            nb |= d == best + 1 ? (S[i] << 16) : 0u;
        }
        bad = row16_or(bad);
        nb = row16_or(nb);
        if (g == 0 && !bad && minS < 32767) {
            const int X = x + minX1;
            const int x2 = X - best - minD;
            atomicMin(&key2[x2], ((uint32_t)minS << 16) | (uint32_t)(0xFFFF - X));
            int d16;
            if (best > 0 && best < D - 1) {
                const int Sm = (int)(nb & 0xFFFF), Sq = (int)(nb >> 16);
                const int den = max(Sm + Sq - 2 * minS, 1);
                d16 = best * 16 + ((Sm - Sq) * 16 + den) / (den * 2);  // C truncation
            } else {
                d16 = best * 16;
            }
            drow[X] = d16 + minD * 16;
        }
    }
    __syncthreads();
    int16_t* out = a.disp + (size_t)y * W;
    for (int X = threadIdx.x; X < W; X += 256) {
        int d1 = drow[X];
        if (X >= minX1 && X < maxX1 && d1 != INVALID) {
            const int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
            const int _x = X - _d, x_ = X - d_;
            bool rej1 = false, rej2 = false;
            if (_x >= 0 && _x < W) {
                const uint32_t kk = key2[_x];
                const int d2 = kk == 0xFFFFFFFFu ? INVALID : (int)(0xFFFF - (kk & 0xFFFF)) - _x;
                rej1 = d2 >= minD && abs(d2 - _d) > a.disp12;
            }
            if (x_ >= 0 && x_ < W) {
                const uint32_t kk = key2[x_];
                const int d2 = kk == 0xFFFFFFFFu ? INVALID : (int)(0xFFFF - (kk & 0xFFFF)) - x_;
                rej2 = d2 >= minD && abs(d2 - d_) > a.disp12;
            }
            if (rej1 && rej2) d1 = INVALID;
        }
        out[X] = (int16_t)d1;
    }
}

// -------------------------------------------------------------- median ---
__device__ __forceinline__ void cswap(int& a, int& b)
{
    const int t = min(a, b);
    b = max(a, b);
    a = t;
}

__global__ void __launch_bounds__(256) k_median3(const int16_t* __restrict__ src, int16_t* __restrict__ dst, int H, int W)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
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
