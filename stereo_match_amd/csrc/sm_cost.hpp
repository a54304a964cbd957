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

constexpr int CT_W = 64, CT_H = 16, CT_PY = 4;  // tile; pixels per thread (vertical)
constexpr int CT_LW = CT_W + 12;                 // LDS row: 4 left halo + 64 + 4 right halo, dword padded

// Bits are assembled MSB-first with acc = 2*acc + (I[n] < I[c]) so each
// comparison is one compare + one add-with-carry; the 62 neighbours of a
// pixel are read as 3 aligned dwords per window row (bytes extracted by the
// compiler), and a thread computes CT_PY vertically adjacent pixels so the
// 7-row windows share their LDS reads.
__global__ void __launch_bounds__(256) k_census9x7(CensusArgs a)
{
    __shared__ uint32_t tile[CT_H + 6][CT_LW / 4];
    const int which = blockIdx.z & 1, pair = blockIdx.z >> 1;
    const uint8_t* img = a.img[which] + (size_t)pair * a.in_pair;
    const int x0 = blockIdx.x * CT_W, y0 = blockIdx.y * CT_H;
    uint8_t* tb = reinterpret_cast<uint8_t*>(&tile[0][0]);
    for (int i = threadIdx.x; i < (CT_H + 6) * CT_LW; i += 256) {
        const int ty = i / CT_LW, tx = i % CT_LW;
        const int y = min(max(y0 + ty - 3, 0), a.H - 1), x = min(max(x0 + tx - 4, 0), a.W - 1);
        tb[ty * CT_LW + tx] = img[(size_t)y * a.stride + x];
    }
    __syncthreads();
    const int tx = threadIdx.x % CT_W, ty0 = (threadIdx.x / CT_W) * CT_PY;
    const int x = x0 + tx;
    // window columns tx .. tx+8 in tile coordinates (tile col = image col - x0 + 4)
    const int wd = tx >> 2, sh = (tx & 3) * 8;
    uint32_t rows[CT_PY + 6][3];  // 12 bytes covering the 9 window columns, per tile row
#pragma unroll
    for (int r = 0; r < CT_PY + 6; r++) {
        const uint32_t w0 = tile[ty0 + r][wd], w1 = tile[ty0 + r][wd + 1], w2 = tile[ty0 + r][wd + 2];
        rows[r][0] = __builtin_amdgcn_alignbyte(w1, w0, sh >> 3);
        rows[r][1] = __builtin_amdgcn_alignbyte(w2, w1, sh >> 3);
        rows[r][2] = w2 >> sh;
    }
    auto px = [&](int r, int dx) -> uint32_t { return (rows[r][dx >> 2] >> ((dx & 3) * 8)) & 0xFF; };
#pragma unroll
    for (int p = 0; p < CT_PY; p++) {
        const int y = y0 + ty0 + p;
        const uint32_t c = px(p + 3, 4);
        uint32_t lo = 0, hi = 0;
        // bit k <-> neighbour k in row-major order with the centre skipped
#pragma unroll
        for (int k = 61; k >= 32; k--) {
            const int n = k < 31 ? k : k + 1;
            unsigned co;
            hi = __builtin_addc(hi, hi, px(p + n / 9, n % 9) < c ? 1u : 0u, &co);
        }
#pragma unroll
        for (int k = 31; k >= 0; k--) {
            const int n = k < 31 ? k : k + 1;
            unsigned co;
            lo = __builtin_addc(lo, lo, px(p + n / 9, n % 9) < c ? 1u : 0u, &co);
        }
        if (x < a.W && y < a.H)
            a.out[which][(size_t)pair * a.H * a.W + (size_t)y * a.W + x] = ((uint64_t)hi << 32) | lo;
    }
}

// Census Hamming cost volume for the path kernels' vertical family:
// C[pair][y][x1][d] = popcount(cl[y][X] ^ cr[y][X-minD-d]) (u8), X = x1 + minX1.
// One workgroup per (64 columns, row, pair): the 64 left codes and the
// 64+D-1 right codes they need staged in LDS; a thread writes 16 disparities
// (one 16-byte store) of one column, consecutive threads consecutive columns.
struct Cost8Args {
    const uint64_t* cl;
    const uint64_t* cr;
    size_t census_pair;
    uint8_t* C;
    size_t C_pair;
    int H, W, width1, D, minD, minX1;
};

constexpr int C8_TX = 64;

__global__ void __launch_bounds__(256) k_census_cost8(Cost8Args a)
{
    __shared__ uint64_t lc[C8_TX];
    __shared__ uint64_t rc[C8_TX + 256];
    __shared__ uint4 tile[C8_TX * 17];  // [x][D/16 + 1] 16-byte chunks (padded pitch)
    const int x0 = blockIdx.x * C8_TX, y = blockIdx.y, pair = blockIdx.z;
    const int nx = min(C8_TX, a.width1 - x0), D = a.D;
    const uint64_t* cl = a.cl + pair * a.census_pair + (size_t)y * a.W;
    const uint64_t* cr = a.cr + pair * a.census_pair + (size_t)y * a.W;
    const int X0 = x0 + a.minX1;
    const int rlo = X0 - a.minD - (D - 1);  // right column of rc[0]
    for (int i = threadIdx.x; i < nx; i += 256) lc[i] = cl[X0 + i];
    for (int i = threadIdx.x; i < nx + D - 1; i += 256) rc[i] = cr[rlo + i];
    __syncthreads();
    const int chunks = D / 16, pitch = chunks + 1;
    for (int i = threadIdx.x; i < nx * chunks; i += 256) {
        // consecutive lanes take consecutive columns: conflict-free LDS reads
        const int ch = i / nx, x = i - ch * nx;
        const uint64_t l = lc[x];
        // disparity d = 16*ch + j reads right column X - minD - d = rc[x + D - 1 - d]
        const uint64_t* r = rc + x + D - 1 - 16 * ch;
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            w[q] = (uint32_t)__popcll(l ^ r[-4 * q]) | ((uint32_t)__popcll(l ^ r[-4 * q - 1]) << 8) |
                   ((uint32_t)__popcll(l ^ r[-4 * q - 2]) << 16) | ((uint32_t)__popcll(l ^ r[-4 * q - 3]) << 24);
        }
        tile[x * pitch + ch] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    __syncthreads();
    // the tile's nx*D bytes are contiguous in C: coalesced 16-byte stores
    uint4* out = reinterpret_cast<uint4*>(a.C + pair * a.C_pair + ((size_t)y * a.width1 + x0) * D);
    for (int i = threadIdx.x; i < nx * chunks; i += 256) {
        const int x = i / chunks, ch = i - x * chunks;
        out[i] = tile[x * pitch + ch];
    }
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
    size_t in_pair;  // bytes between pairs' images
    uint8_t* planes;  // packed uint2 per pixel, [pair][view][H][W]
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

// Packed per-pixel planes for the BT cost: one uint2 per pixel per view,
// bytes [g, g_min, g_max, raw, raw_min, raw_max, 0, 0] (g = clipped Sobel-x,
// min/max over the half-pixel neighbours as calcPixelCostBT); blockIdx.z =
// 2*pair + view.
__global__ void __launch_bounds__(256) k_sgbm_prefilter(PrefilterArgs a)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, im = blockIdx.z & 1, pair = blockIdx.z >> 1;
    if (x >= a.W) return;
    const uint8_t* img = a.img[im] + (size_t)pair * a.in_pair;
    uint32_t b[6];
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
        b[3 * ch] = (uint32_t)v;
        b[3 * ch + 1] = (uint32_t)min(min(vl, vr), v);
        b[3 * ch + 2] = (uint32_t)max(max(vl, vr), v);
    }
    uint2 w;
    w.x = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
    w.y = b[4] | (b[5] << 8);
    reinterpret_cast<uint2*>(a.planes)[((size_t)(pair * 2 + im) * a.H + y) * a.W + x] = w;
}

// C_true[y][x1][d] for the rows OpenCV's incremental box filter actually
// updates (y < Yc = max(1, H - SH2)):
//   sum_{k=y-SH2..y+SH2} sum_{j=-SW2..SW2} pix(clamp(k,0,H-1), clamp(x1+j,0,width1-1), d)
// Tile of SC_TY rows x SC_TX columns x 8 disparities per workgroup: BT pixel
// costs of the halo tile -> LDS, horizontal then vertical sums in LDS.
constexpr int SC_TX = 64, SC_TY = 8, SC_MAXR = 5, SC_DC = 8;  // blockSize <= 11; disparities per chunk

struct SgbmCostArgs {
    const uint2* planes;  // packed, [pair][view][H][W]
    uint16_t* C;          // [pair][H][width1][D]
    size_t C_pair;
    int H, W, width1, D, minD, minX1, SW2, SH2, Yc;
};

__device__ __forceinline__ int bt_cost2(uint2 L, uint2 R)
{
    // bytes: [g, g_min, g_max, raw, raw_min, raw_max, -, -] of left (u) / right (v)
    int acc = 0;
#pragma unroll
    for (int ch = 0; ch < 2; ch++) {
        const uint32_t lw = ch == 0 ? L.x : (L.x >> 24) | (L.y << 8);
        const uint32_t rw = ch == 0 ? R.x : (R.x >> 24) | (R.y << 8);
        const int u = lw & 0xFF, u0 = (lw >> 8) & 0xFF, u1 = (lw >> 16) & 0xFF;
        const int v = rw & 0xFF, v0 = (rw >> 8) & 0xFF, v1 = (rw >> 16) & 0xFF;
        const int c0 = max(max(0, u - v1), v0 - u);
        const int c1 = max(max(0, v - u1), u0 - v);
        acc += min(c0, c1) >> (ch == 0 ? 0 : 2);
    }
    return acc;
}

// One workgroup per SC_TY x SC_TX output tile and ALL disparities (chunks of
// SC_DC): the left halo tile is staged once, the right planes once per chunk;
// BT pixel costs -> LDS bytes, then horizontal and vertical box sums with
// two disparities per 32-bit lane (SWAR; sums < 2^16 by the int16-exact
// domain check, and the int16 wrap is the low 16 bits).
__global__ void __launch_bounds__(256) k_sgbm_cost(SgbmCostArgs a)
{
    constexpr int HR = SC_TY + 2 * SC_MAXR, HC = SC_TX + 2 * SC_MAXR;
    __shared__ __attribute__((aligned(16))) uint2 lpl[HR][HC];
    __shared__ __attribute__((aligned(16))) uint2 rpl[HR][HC + SC_DC];
    __shared__ __attribute__((aligned(16))) uint2 pix[HR][HC];           // SC_DC byte costs
    __shared__ __attribute__((aligned(16))) uint4 hs[HR][SC_TX];         // SC_DC u16 sums
    const int x0 = blockIdx.x * SC_TX, y0 = blockIdx.y * SC_TY, pair = blockIdx.z;
    const int SW2 = a.SW2, SH2 = a.SH2, W1 = a.width1, W = a.W, D = a.D;
    const int rows_h = SC_TY + 2 * SH2, cols_h = SC_TX + 2 * SW2;
    const uint2* Lp = a.planes + (size_t)(pair * 2) * a.H * W;
    const uint2* Rp = Lp + (size_t)a.H * W;
    const int xlo = max(x0 - SW2, 0), xhi = min(x0 + SC_TX + SW2 - 1, W1 - 1);  // clamped x1 range
    const int rcols = xhi - xlo + SC_DC;
    uint16_t* Cb = a.C + pair * a.C_pair;
    for (int i = threadIdx.x; i < rows_h * cols_h; i += 256) {
        const int r = i / cols_h, c = i - r * cols_h;
        const int y = min(max(y0 - SH2 + r, 0), a.H - 1);
        lpl[r][c] = Lp[(size_t)y * W + min(max(x0 - SW2 + c, 0), W1 - 1) + a.minX1];
    }
    for (int d0 = 0; d0 < D; d0 += SC_DC) {
        const int rbase = xlo + a.minX1 - a.minD - d0 - (SC_DC - 1);  // right column of rpl[.][0]
        __syncthreads();  // previous chunk done with rpl / hs
        for (int i = threadIdx.x; i < rows_h * rcols; i += 256) {
            const int r = i / rcols, c = i - r * rcols;
            const int y = min(max(y0 - SH2 + r, 0), a.H - 1);
            rpl[r][c] = Rp[(size_t)y * W + rbase + c];
        }
        __syncthreads();
        for (int i = threadIdx.x; i < rows_h * cols_h; i += 256) {
            const int r = i / cols_h, c = i - r * cols_h;
            const int x1 = min(max(x0 - SW2 + c, 0), W1 - 1);
            const int ri = x1 - xlo + SC_DC - 1;  // right column index for disparity d0
            const uint2 L = lpl[r][c];
            uint32_t b[SC_DC];
#pragma unroll
            for (int j = 0; j < SC_DC; j++) b[j] = (uint32_t)bt_cost2(L, rpl[r][ri - j]);
            pix[r][c] = make_uint2(b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24),
                                   b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24));
        }
        __syncthreads();
        for (int i = threadIdx.x; i < rows_h * SC_TX; i += 256) {
            const int r = i / SC_TX, c = i - r * SC_TX;
            uint32_t e0 = 0, o0 = 0, e1 = 0, o1 = 0;  // u16 lanes: (d0,d2) (d1,d3) (d4,d6) (d5,d7)
            for (int j = 0; j <= 2 * SW2; j++) {
                const uint2 w = pix[r][c + j];
                e0 += w.x & 0x00FF00FFu;
                o0 += (w.x >> 8) & 0x00FF00FFu;
                e1 += w.y & 0x00FF00FFu;
                o1 += (w.y >> 8) & 0x00FF00FFu;
            }
            hs[r][c] = make_uint4(e0, o0, e1, o1);
        }
        __syncthreads();
        for (int i = threadIdx.x; i < SC_TY * SC_TX; i += 256) {
            const int r = i / SC_TX, c = i - r * SC_TX;
            const int y = y0 + r, x1 = x0 + c;
            if (y >= a.Yc || x1 >= W1) continue;
            uint32_t e0 = 0, o0 = 0, e1 = 0, o1 = 0;
            for (int k = 0; k <= 2 * SH2; k++) {
                const uint4 w = hs[r + k][c];
                e0 += w.x;
                o0 += w.y;
                e1 += w.z;
                o1 += w.w;
            }
            // interleave back to d order: (d0,d1) (d2,d3) (d4,d5) (d6,d7)
            uint4 o;
            o.x = (e0 & 0xFFFF) | (o0 << 16);
            o.y = (e0 >> 16) | (o0 & 0xFFFF0000u);
            o.z = (e1 & 0xFFFF) | (o1 << 16);
            o.w = (e1 >> 16) | (o1 & 0xFFFF0000u);
            *reinterpret_cast<uint4*>(Cb + ((size_t)y * W1 + x1) * D + d0) = o;
        }
    }
}

// Rows y >= Yc: MODE_SGBM reuses one C row, so they stay equal to row Yc-1;
// MODE_HH keeps one C row per y that is never updated (P2 seed only: C_true = 0).
__global__ void __launch_bounds__(256) k_sgbm_cost_tail(uint16_t* C, int H, int Yc, size_t row_elems, int hh)
{
    const size_t n = (size_t)(H - Yc) * row_elems / 8;
    const uint4* src = reinterpret_cast<const uint4*>(C + (size_t)(Yc - 1) * row_elems);
    uint4* dst = reinterpret_cast<uint4*>(C + (size_t)Yc * row_elems);
    const size_t per_row = row_elems / 8;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        dst[i] = hh ? make_uint4(0, 0, 0, 0) : src[i % per_row];
}

// ---------------------------------------------------------------------------
// External float32 cost volume (mc-cnn; the reference memmaps
// it at mapTo3D_mc_cnn.py:71) -> quantised u16 C[H][width1][D].
// d-major [D][H][W] in, d-minor out: an LDS-tiled transpose, HBM-bound
// (4 B read + 2 B written per cell).  q = rint((c + offset) * scale) in
// float32 clamped to [0, VOL_CMAX], NaN -> VOL_CMAX (oracle:
// sgm_np.quantize_volume).  (c + offset) * scale cannot be contracted into an
// FMA, so the two IEEE roundings match the oracle's.
constexpr int VOL_CMAX = 4095;


struct VolArgs {
    const float* vol;
    size_t vol_pair;  // elements between pairs
    uint16_t* C;
    size_t C_pair;  // elements between pairs
    int H, W, width1, D, minX1;
    float offset, scale;
};

__device__ inline uint32_t quant_cost(float c, float off, float sc)
{
    if (c != c) return VOL_CMAX;
    const float v = __builtin_rintf((c + off) * sc);
    if (!(v > 0.f)) return 0;
    if (v > (float)VOL_CMAX) return VOL_CMAX;
    return (uint32_t)v;
}

// TX columns per tile (64 or 128): each lane reads TX/64 consecutive floats
// of a plane row (64 lanes cover the tile's TX columns, TX*4 contiguous bytes).
template <int TX>
__global__ void __launch_bounds__(256) k_cost_volume_f32(VolArgs a)
{
    constexpr int PL = TX / 64;         // floats per lane per plane row
    extern __shared__ uint32_t tile[];  // [TX][D/2 + 1] packed u16 pairs (d even | d odd << 16)
    const int half = a.D >> 1, rowdw = half + 1;
    const int x0 = blockIdx.x * TX, y = blockIdx.y, pair = blockIdx.z;
    const int nx = min(TX, a.width1 - x0);
    const size_t plane = (size_t)a.H * a.W;
    const float* v = a.vol + pair * a.vol_pair + (size_t)y * a.W + a.minX1 + x0;
    for (int i = threadIdx.x; i < 64 * half; i += 256) {
        const int xl = (i & 63) * PL, dp = i >> 6;
        const float* p0 = v + (size_t)(2 * dp) * plane + xl;
        const float* p1 = p0 + plane;
        float c0[PL], c1[PL];
        if (xl + PL <= nx) {
            if constexpr (PL == 2) {
                typedef float f2v __attribute__((ext_vector_type(2)));
                const f2v a0 = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(p0));
                const f2v a1 = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(p1));
                c0[0] = a0[0]; c0[1] = a0[1]; c1[0] = a1[0]; c1[1] = a1[1];
            } else {
#pragma unroll
                for (int k = 0; k < PL; k++) {
                    c0[k] = __builtin_nontemporal_load(p0 + k);
                    c1[k] = __builtin_nontemporal_load(p1 + k);
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < PL; k++) {
                c0[k] = xl + k < nx ? p0[k] : 0.f;
                c1[k] = xl + k < nx ? p1[k] : 0.f;
            }
        }
#pragma unroll
        for (int k = 0; k < PL; k++)
            tile[(xl + k) * rowdw + dp] = quant_cost(c0[k], a.offset, a.scale) | (quant_cost(c1[k], a.offset, a.scale) << 16);
    }
    __syncthreads();
    uint32_t* out = reinterpret_cast<uint32_t*>(a.C + pair * a.C_pair + ((size_t)y * a.width1 + x0) * a.D);
    const int total = nx * half;
    for (int i = threadIdx.x; i < total; i += 256) {
        const int xl = i / half, j = i - xl * half;
        out[i] = tile[xl * rowdw + j];
    }
}

}  // namespace smk
