// sm_cost.hpp — matching-cost kernels: census 9x7 (north-star mode) and the
// OpenCV StereoSGBM cost (Sobel-x clip + raw channel Birchfield-Tomasi, box
// sum with OpenCV's clamped borders and frozen bottom rows).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

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
    uint32_t* zero_word;    // non-null: cleared by the first thread (the launch group's sweep flag)
};

// the launch group's first kernel clears its sweep give-up flag (instead of a memset node)
__device__ __forceinline__ void clear_group_flag(uint32_t* w)
{
    if (w && threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0) *w = 0u;
}

constexpr int CT_W = 64, CT_H = 16, CT_PY = 4;  // tile; pixels per thread (vertical)
constexpr int CT_LW = CT_W + 12;                 // LDS row: 4 left halo + 64 + 4 right halo, dword padded

// Bits are assembled MSB-first: I[n] - I[c] (bytes, so bit 31 of the 32-bit
// difference is I[n] < I[c]) shifted in by v_alignbit, acc = (acc << 1) | (diff >> 31):
// two VALU ops per bit, the byte select folded into the subtract (SDWA), no
// compare mask (a compare + select + shift + or, with hazard NOPs on the lane
// mask, was ~4 per bit); the 62 neighbours of a
// pixel are read as 3 aligned dwords per window row (bytes extracted by the
// compiler), and a thread computes CT_PY vertically adjacent pixels so the
// 7-row windows share their LDS reads.
__global__ void __launch_bounds__(256) k_census9x7(CensusArgs a)
{
    clear_group_flag(a.zero_word);
    __shared__ uint32_t tile[CT_H + 6][CT_LW / 4];
    const int which = blockIdx.z & 1, pair = blockIdx.z >> 1;
    const uint8_t* img = a.img[which] + (size_t)pair * a.in_pair;
    const int x0 = blockIdx.x * CT_W, y0 = blockIdx.y * CT_H;
    uint8_t* tb = reinterpret_cast<uint8_t*>(&tile[0][0]);
    // every byte load in flight before the first LDS write (a load -> wait -> write loop
    // serialises ~7 memory round trips per workgroup)
    constexpr int NT = (CT_H + 6) * CT_LW, NST = (NT + 255) / 256;
    uint32_t st[NST];
#pragma unroll
    for (int k = 0; k < NST; k++) {
        const int i = threadIdx.x + 256 * k;
        const int ty = i / CT_LW, tx = i % CT_LW;
        const int y = min(max(y0 + ty - 3, 0), a.H - 1), x = min(max(x0 + tx - 4, 0), a.W - 1);
        if (i < NT) st[k] = img[(size_t)y * a.stride + x];
    }
#pragma unroll
    for (int k = 0; k < NST; k++) {
        const int i = threadIdx.x + 256 * k;
        if (i < NT) tb[i] = (uint8_t)st[k];
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
            hi = __builtin_amdgcn_alignbit(hi, px(p + n / 9, n % 9) - c, 31);
        }
#pragma unroll
        for (int k = 31; k >= 0; k--) {
            const int n = k < 31 ? k : k + 1;
            lo = __builtin_amdgcn_alignbit(lo, px(p + n / 9, n % 9) - c, 31);
        }
        if (x < a.W && y < a.H)
            a.out[which][(size_t)pair * a.H * a.W + (size_t)y * a.W + x] = ((uint64_t)hi << 32) | lo;
    }
}

// Census Hamming cost volume for the path kernels (u8):
// C[pair][y][x1][d] = popcount(cl[y][X] ^ cr[y][X-minD-d]), X = x1 + minX1.
// One workgroup per (64 columns, C8_RY rows, pair); per row the 64 left codes
// and the 64+D-1 right codes they need are staged in LDS.  Thread (x, c0)
// computes 16-disparity chunks c0, c0+4, ... of column x (no index division),
// then the tile's nx*D contiguous bytes leave as coalesced 16-byte stores.
struct Cost8Args {
    const uint64_t* cl;
    const uint64_t* cr;
    size_t census_pair;
    uint8_t* C;
    size_t C_pair;
    int H, W, width1, D, minD, minX1;
    int nt;  // 1: nontemporal stores (the launch group's volume exceeds the Infinity Cache)
};

#ifndef CENSUS_COST_RY
#define CENSUS_COST_RY 4  // image rows per k_census_cost8 workgroup
#endif
constexpr int C8_TX = 64, C8_RY = CENSUS_COST_RY;

// (a << 8) | b in one VALU op (hipcc re-associates the shift-or chain into separate shifts)
__device__ __forceinline__ uint32_t lshl8_or(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_lshl_or_b32 %0, %1, 8, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__global__ void __launch_bounds__(256) k_census_cost8(Cost8Args a)
{
    __shared__ uint64_t lc[C8_TX];
    __shared__ uint64_t rc[C8_TX + 256];
    __shared__ uint4 tile[C8_TX * 17];  // [x][D/16 + 1] 16-byte chunks (padded pitch)
    const int x0 = blockIdx.x * C8_TX, pair = blockIdx.z, tid = threadIdx.x;
    const int nx = min(C8_TX, a.width1 - x0), D = a.D;
    const int X0 = x0 + a.minX1;
    const int rlo = X0 - a.minD - (D - 1);  // right column of rc[0]
    const int chunks = D / 16, pitch = chunks + 1;
    // i / chunks for i < 64 * 16 as a multiply-shift (exact: the error stays below 1/64)
    const uint32_t M = (65536u + (uint32_t)chunks - 1) / (uint32_t)chunks;
    const int xl = tid & 63, c0 = tid >> 6;
    const int nr = nx + D - 1;  // <= 319: two right codes per thread
    // the next row's codes are fetched into registers while this row computes
    uint64_t pl = 0, pr0 = 0, pr1 = 0;
    auto fetch = [&](int y) {
        const uint64_t* cl = a.cl + pair * a.census_pair + (size_t)y * a.W;
        const uint64_t* cr = a.cr + pair * a.census_pair + (size_t)y * a.W;
        if (tid < nx) pl = cl[X0 + tid];
        if (tid < nr) pr0 = cr[rlo + tid];
        if (tid + 256 < nr) pr1 = cr[rlo + 256 + tid];
    };
    if (blockIdx.y * C8_RY < a.H) fetch(blockIdx.y * C8_RY);
    for (int r = 0; r < C8_RY; r++) {
        const int y = blockIdx.y * C8_RY + r;
        if (y >= a.H) break;  // workgroup-uniform
        if (tid < nx) lc[tid] = pl;
        if (tid < nr) rc[tid] = pr0;
        if (tid + 256 < nr) rc[256 + tid] = pr1;
        if (r + 1 < C8_RY && y + 1 < a.H) fetch(y + 1);
        __syncthreads();  // also: the previous row's stores have read the tile
        if (xl < nx) {
            const uint64_t l = lc[xl];
            for (int ch = c0; ch < chunks; ch += 4) {
                // disparity d = 16*ch + j reads right column X - minD - d = rc[x + D - 1 - d]
                const uint64_t* rr = rc + xl + D - 1 - 16 * ch;
                uint32_t w[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    // packed as a shift-or chain (one v_lshl_or_b32 per byte; the or-tree of
                    // separate shifts took two VALU ops per byte)
                    uint32_t v = (uint32_t)__popcll(l ^ rr[-4 * q - 3]);
                    v = lshl8_or(v, (uint32_t)__popcll(l ^ rr[-4 * q - 2]));
                    v = lshl8_or(v, (uint32_t)__popcll(l ^ rr[-4 * q - 1]));
                    w[q] = lshl8_or(v, (uint32_t)__popcll(l ^ rr[-4 * q]));
                }
                tile[xl * pitch + ch] = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
        __syncthreads();
        uint4* out = reinterpret_cast<uint4*>(a.C + pair * a.C_pair + ((size_t)y * a.width1 + x0) * D);
        for (int i = tid; i < nx * chunks; i += 256) {
            const int x = (int)(((uint32_t)i * M) >> 16), ch = i - x * chunks;
            if (a.nt) {  // workgroup-uniform
                typedef unsigned v4u __attribute__((ext_vector_type(4)));
                const uint4 t = tile[x * pitch + ch];
                __builtin_nontemporal_store(v4u{t.x, t.y, t.z, t.w}, reinterpret_cast<v4u*>(out + i));
            } else {
                out[i] = tile[x * pitch + ch];
            }
        }
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
    uint8_t* planes;  // packed uint2 per pixel, [pair][view][channel][H][W]
    int H, W, stride, ftzero;
    int cn;  // channels per pixel (1 gray, 3 BGR interleaved; 0 = 1); stride in bytes
    uint32_t* zero_word;  // see CensusArgs
};

// Packed per-pixel planes for the BT cost: one uint2 per pixel per view,
// bytes [g, g_min, g_max, raw, raw_min, raw_max, 0, 0] (g = clipped Sobel-x,
// min/max over the half-pixel neighbours as calcPixelCostBT); blockIdx.z =
// (2*pair + view)*cn + channel (colour: one plane per channel, as OpenCV's
// calcPixelCostBT keeps a derivative and a raw row per channel).
#ifndef PREFILTER_ROWS
#define PREFILTER_ROWS 8  // image rows per k_sgbm_prefilter workgroup
#endif
constexpr int PF_ROWS = PREFILTER_ROWS;

// One workgroup per (256 columns, PF_ROWS rows, view): the PF_ROWS + 2 image rows
// (+2 halo columns each side) and the clipped Sobel of columns x0-1 .. x0+256 of each
// output row in LDS (a row of workgroups per image row re-read every input row 3x and
// left the launch dominated by its 2*H*pairs tiny workgroups).
__global__ void __launch_bounds__(256) k_sgbm_prefilter(PrefilterArgs a)
{
    clear_group_flag(a.zero_word);
    __shared__ uint8_t rows[PF_ROWS + 2][260];
    __shared__ int gs[PF_ROWS][258];
    const int cn = a.cn > 0 ? a.cn : 1;
    const int ch = blockIdx.z % cn, view = blockIdx.z / cn;
    const int x0 = blockIdx.x * 256, y0 = blockIdx.y * PF_ROWS, im = view & 1, pair = view >> 1;
    const int W = a.W, H = a.H, ft = a.ftzero, tid = threadIdx.x;
    const uint8_t* img = a.img[im] + (size_t)pair * a.in_pair + ch;
    // every byte load in flight before the first LDS write (a load -> wait -> write loop
    // serialises a memory round trip per staged row)
    uint32_t st0[PF_ROWS + 2], st1[PF_ROWS + 2];
    const size_t cx0 = (size_t)min(max(x0 - 2 + tid, 0), W - 1) * cn;
    const size_t cx1 = (size_t)min(max(x0 + 254 + tid, 0), W - 1) * cn;  // columns 256..259 (tid < 4)
#pragma unroll
    for (int r = 0; r < PF_ROWS + 2; r++) {
        const uint8_t* row = img + (size_t)min(max(y0 - 1 + r, 0), H - 1) * a.stride;
        st0[r] = row[cx0];
        if (tid < 4) st1[r] = row[cx1];
    }
#pragma unroll
    for (int r = 0; r < PF_ROWS + 2; r++) {
        rows[r][tid] = (uint8_t)st0[r];
        if (tid < 4) rows[r][256 + tid] = (uint8_t)st1[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < PF_ROWS; r++) {
        for (int i = tid; i < 258; i += 256) {  // column xx = x0 - 1 + i sits at rows[.][i + 1]
            const int xx = x0 - 1 + i, c = i + 1;
            int v = ft;
            if (xx > 0 && xx < W - 1) {
                v = (rows[r + 1][c + 1] - rows[r + 1][c - 1]) * 2 + rows[r][c + 1] - rows[r][c - 1] + rows[r + 2][c + 1] -
                    rows[r + 2][c - 1];
                v = min(max(v, -ft), ft) + ft;
            }
            gs[r][i] = v;
        }
    }
    __syncthreads();
    const int x = x0 + tid;
    if (x >= W) return;
#pragma unroll
    for (int r = 0; r < PF_ROWS; r++) {
        const int y = y0 + r;
        if (y >= H) break;
        auto raw = [&](int xx) { return (xx <= 0 || xx >= W - 1) ? ft : (int)rows[r + 1][xx - x0 + 2]; };
        uint32_t b[6];
        {
            const int v = gs[r][tid + 1];
            const int vl = x > 0 ? (v + gs[r][tid]) / 2 : v;
            const int vr = x < W - 1 ? (v + gs[r][tid + 2]) / 2 : v;
            b[0] = (uint32_t)v;
            b[1] = (uint32_t)min(min(vl, vr), v);
            b[2] = (uint32_t)max(max(vl, vr), v);
        }
        {
            const int v = raw(x);
            const int vl = x > 0 ? (v + raw(x - 1)) / 2 : v;
            const int vr = x < W - 1 ? (v + raw(x + 1)) / 2 : v;
            b[3] = (uint32_t)v;
            b[4] = (uint32_t)min(min(vl, vr), v);
            b[5] = (uint32_t)max(max(vl, vr), v);
        }
        uint2 w;
        w.x = b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24);
        w.y = b[4] | (b[5] << 8);
        reinterpret_cast<uint2*>(a.planes)[((size_t)blockIdx.z * H + y) * W + x] = w;
    }
}

// C_true[y][x1][d] for the rows OpenCV's incremental box filter actually
// updates (y < Yc = max(1, H - SH2)):
//   sum_{k=y-SH2..y+SH2} sum_{j=-SW2..SW2} pix(clamp(k,0,H-1), clamp(x1+j,0,width1-1), d)
// Tile of SC_TY rows x SC_TX columns x 8 disparities per workgroup: BT pixel
// costs of the halo tile -> LDS, horizontal then vertical sums in LDS.
// tile height: 8 measured fastest on MI355X (12: +13 %, 16: +12 % per pair at KITTI D=128)
#ifndef SGBM_COST_TY
#define SGBM_COST_TY 8
#endif
constexpr int SC_TY = SGBM_COST_TY, SC_DC = 8;  // output rows per tile; disparities per chunk

struct SgbmCostArgs {
    const uint2* planes;  // packed, [pair][view][H][W]
    uint16_t* C;          // [pair][H][width1][D]
    size_t C_pair;
    int H, W, width1, D, minD, minX1, SW2, SH2, Yc;
};

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t w) { return __builtin_bit_cast(u16x2, w); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ u16x2 subsat(u16x2 a, u16x2 b) { return __builtin_elementwise_sub_sat(a, b); }

// (r, c) walk over a rows x cols item grid with a 256-thread stride, no division per item
struct Walk {
    int r, c, rs, cs, cols;
    __device__ Walk(int tid, int cols_) : cols(cols_)
    {
        r = tid / cols;
        c = tid - r * cols;
        rs = 256 / cols;
        cs = 256 - rs * cols;
    }
    __device__ void next()
    {
        r += rs;
        c += cs;
        if (c >= cols) {
            c -= cols;
            r++;
        }
    }
};

// One workgroup per SC_TY x TX output tile and ALL disparities (chunks of
// SC_DC).  The BT costs run two disparities per 32-bit lane: the right
// view's six byte quantities (g, g_min, g_max, raw, raw_min, raw_max) are
// staged per chunk as u16 pairs of adjacent columns, so one LDS word feeds
// the (d, d+1) pair and the BT min/max/saturating-subtract work is packed
// 16-bit math.  Box sums: horizontal then vertical, SWAR u16 lanes (sums
// < 2^16 by the int16-exact domain check; the int16 wrap is the low 16 bits).
template <int TX, int MAXR>
__global__ void __launch_bounds__(256) k_sgbm_cost(SgbmCostArgs a)
{
    constexpr int HR = SC_TY + 2 * MAXR, HC = TX + 2 * MAXR, RC = HC + SC_DC;
    __shared__ __attribute__((aligned(16))) uint2 lpl[HR][HC];
    // the pair planes and the horizontal sums are never live together: one buffer
    constexpr int QW = 6 * HR * RC, HW = 4 * HR * TX;
    __shared__ __attribute__((aligned(16))) uint32_t qh[QW > HW ? QW : HW];
    __shared__ __attribute__((aligned(16))) uint4 pix[HR][HC];  // SC_DC costs as u16 pairs
    auto Qa = reinterpret_cast<uint4(*)[RC]>(qh);                // g, g_min, g_max, raw
    auto Qb = reinterpret_cast<uint2(*)[RC]>(qh + 4 * HR * RC);  // raw_min, raw_max
    auto hs = reinterpret_cast<uint4(*)[TX]>(qh);
    constexpr int NQ = (HR * (HC + SC_DC - 1) + 255) / 256;  // pair items per thread (max)
    const int x0 = blockIdx.x * TX, y0 = blockIdx.y * SC_TY, pair = blockIdx.z;
    const int SW2 = a.SW2, SH2 = a.SH2, W1 = a.width1, W = a.W, D = a.D;
    const int rows_h = SC_TY + 2 * SH2, cols_h = TX + 2 * SW2;
    const uint2* Lp = a.planes + (size_t)(pair * 2) * a.H * W;
    const uint2* Rp = Lp + (size_t)a.H * W;
    const int xlo = max(x0 - SW2, 0), xhi = min(x0 + TX + SW2 - 1, W1 - 1);  // clamped x1 range
    const int rpairs = xhi - xlo + SC_DC - 1;  // column pairs (k, k+1) needed per chunk
    uint16_t* Cb = a.C + pair * a.C_pair;
    const int tid = threadIdx.x;
    for (Walk w(tid, cols_h); w.r < rows_h; w.next()) {
        const int y = min(max(y0 - SH2 + w.r, 0), a.H - 1);
        lpl[w.r][w.c] = Lp[(size_t)y * W + min(max(x0 - SW2 + w.c, 0), W1 - 1) + a.minX1];
    }
    // right-view columns of the next chunk are loaded into registers while
    // the current chunk computes (L2 latency off the barrier-separated phases)
    uint2 pc0[NQ], pc1[NQ];
    auto load_right = [&](int d0) {
        const int rbase = xlo + a.minX1 - a.minD - d0 - (SC_DC - 1);  // right column of pair index 0
        Walk w(tid, rpairs);
#pragma unroll
        for (int i = 0; i < NQ; i++, w.next()) {
            if (w.r < rows_h && d0 < D) {
                const uint2* row = Rp + (size_t)min(max(y0 - SH2 + w.r, 0), a.H - 1) * W + rbase;
                pc0[i] = row[w.c];
                pc1[i] = row[w.c + 1];
            }
        }
    };
    load_right(0);
    for (int d0 = 0; d0 < D; d0 += SC_DC) {
        __syncthreads();  // previous chunk done with Q / hs
        {
            Walk w(tid, rpairs);
#pragma unroll
            for (int i = 0; i < NQ; i++, w.next()) {
                if (w.r < rows_h) {
                    const uint2 c0 = pc0[i], c1 = pc1[i];
                    // u16 pair (col k+1 | col k << 16) of each byte quantity
                    Qa[w.r][w.c] = make_uint4(__builtin_amdgcn_perm(c1.x, c0.x, 0x0c000c04u),
                                              __builtin_amdgcn_perm(c1.x, c0.x, 0x0c010c05u),
                                              __builtin_amdgcn_perm(c1.x, c0.x, 0x0c020c06u),
                                              __builtin_amdgcn_perm(c1.x, c0.x, 0x0c030c07u));
                    Qb[w.r][w.c] = make_uint2(__builtin_amdgcn_perm(c1.y, c0.y, 0x0c000c04u),
                                              __builtin_amdgcn_perm(c1.y, c0.y, 0x0c010c05u));
                }
            }
        }
        load_right(d0 + SC_DC);
        __syncthreads();
        for (Walk w(tid, cols_h); w.r < rows_h; w.next()) {
            const int x1 = min(max(x0 - SW2 + w.c, 0), W1 - 1);
            const int ri = x1 - xlo + SC_DC - 1;  // right column index (pair grid) of disparity d0
            const uint2 L = lpl[w.r][w.c];
            // left quantities broadcast to both lanes
            const u16x2 U0 = as_u16x2(__builtin_amdgcn_perm(0, L.x, 0x0c000c00u));
            const u16x2 U1 = as_u16x2(__builtin_amdgcn_perm(0, L.x, 0x0c010c01u));
            const u16x2 U2 = as_u16x2(__builtin_amdgcn_perm(0, L.x, 0x0c020c02u));
            const u16x2 U3 = as_u16x2(__builtin_amdgcn_perm(0, L.x, 0x0c030c03u));
            const u16x2 U4 = as_u16x2(__builtin_amdgcn_perm(0, L.y, 0x0c000c00u));
            const u16x2 U5 = as_u16x2(__builtin_amdgcn_perm(0, L.y, 0x0c010c01u));
            uint32_t P[SC_DC / 2];
#pragma unroll
            for (int j = 0; j < SC_DC; j += 2) {
                const int k = ri - j - 1;  // lanes: (d0+j, d0+j+1)
                const uint4 qa = Qa[w.r][k];
                const uint2 qb = Qb[w.r][k];
                const u16x2 V0 = as_u16x2(qa.x), V1 = as_u16x2(qa.y), V2 = as_u16x2(qa.z);
                const u16x2 V3 = as_u16x2(qa.w), V4 = as_u16x2(qb.x), V5 = as_u16x2(qb.y);
                // c0 = max(0, u - v1, v0 - u); c1 = max(0, v - u1, u0 - v); per channel min(c0, c1)
                const u16x2 g = __builtin_elementwise_min(__builtin_elementwise_max(subsat(U0, V2), subsat(V1, U0)),
                                                          __builtin_elementwise_max(subsat(V0, U2), subsat(U1, V0)));
                const u16x2 r = __builtin_elementwise_min(__builtin_elementwise_max(subsat(U3, V5), subsat(V4, U3)),
                                                          __builtin_elementwise_max(subsat(V3, U5), subsat(U4, V3)));
                P[j / 2] = as_u32(g + (r >> (u16x2)2));
            }
            pix[w.r][w.c] = make_uint4(P[0], P[1], P[2], P[3]);  // (d0 | d1 << 16), (d2 | d3 << 16), ...
        }
        __syncthreads();
        for (Walk w(tid, TX); w.r < rows_h; w.next()) {
            uint4 h = pix[w.r][w.c];
            for (int j = 1; j <= 2 * SW2; j++) {
                const uint4 v = pix[w.r][w.c + j];
                h.x += v.x;
                h.y += v.y;
                h.z += v.z;
                h.w += v.w;
            }
            hs[w.r][w.c] = h;
        }
        __syncthreads();
        for (Walk w(tid, TX); w.r < SC_TY; w.next()) {
            const int y = y0 + w.r, x1 = x0 + w.c;
            if (y >= a.Yc || x1 >= W1) continue;
            uint4 o = hs[w.r][w.c];
            for (int k = 1; k <= 2 * SH2; k++) {
                const uint4 v = hs[w.r + k][w.c];
                o.x += v.x;
                o.y += v.y;
                o.z += v.z;
                o.w += v.w;
            }
            *reinterpret_cast<uint4*>(Cb + ((size_t)y * W1 + x1) * D + d0) = o;
        }
    }
}

// Streaming form of the same box sum: one workgroup per (strip of TX
// columns, band of rows, pair), ALL disparities, walking its band row by row.
// Thread (p, cg) owns the disparity pair (2p, 2p+1) of CPT adjacent columns;
// per input row it computes the BT costs of its share of the strip + 2S halo
// columns once (u16 pairs in LDS), a running horizontal sum along its columns
// (2 LDS reads per output), and a running vertical sum with the last 2S+1
// rows' horizontal sums in a register ring — no recomputation of vertical
// halo rows, and a wave stores whole 256-byte d-rows (NP = D/2 lanes per
// column).  Sums are u16 pairs in u32 lanes: every subtracted term was added
// before, so no borrow crosses lanes.  Bands start 2S rows early (warm-up).
struct SgbmCost2Args {
    const uint2* planes;  // packed, [pair][view][H][W]
    uint16_t* C;          // [pair][H][width1][D]
    size_t C_pair;
    int H, W, width1, D, minD, minX1, Yc, band;
    int nt;  // 1: nontemporal stores (the launch group's volume exceeds the Infinity Cache)
};

template <int S, int CPT, int NLR>
__global__ void __launch_bounds__(256) k_sgbm_cost2(SgbmCost2Args a)
{
    constexpr int R = 2 * S + 1;
    extern __shared__ __attribute__((aligned(16))) uint32_t dsm[];
    const int D = a.D, NP = D >> 1, CG = blockDim.x / NP, TX = CG * CPT, NHC = TX + 2 * S;
    const int W = a.W, W1 = a.width1;
    const int tid = threadIdx.x, p = tid % NP, cg = tid / NP;
    const int x0 = blockIdx.x * TX, pair = blockIdx.z;
    const int xlo = max(x0 - S, 0), xhi = min(x0 + TX + S - 1, W1 - 1);
    const int rpairs = xhi - xlo + D - 1;   // right column pairs (k, k+1)
    const int rph = (rpairs + 1) >> 1;      // per parity
    const int rb = xlo + a.minX1 - a.minD - (D - 1);  // right column of pair index 0
    // LDS: left quantities broadcast form [NHC] (uint4 + uint2), right pairs split by
    // parity [2][rph] (uint4 + uint2), BT costs [NP][PP] (u16 pairs, column fastest,
    // odd pitch PP: lanes p hit distinct banks; a thread's columns are contiguous)
    uint4* Ua = reinterpret_cast<uint4*>(dsm);
    uint2* Ub = reinterpret_cast<uint2*>(Ua + NHC);
    uint4* Qa = reinterpret_cast<uint4*>(Ub + ((NHC + 1) & ~1));
    uint2* Qb = reinterpret_cast<uint2*>(Qa + 2 * rph);
    const int PP = (CG * ((NHC + CG - 1) / CG)) | 1;  // odd, >= every thread's run end
    // two row buffers: BT of row r+1 may start while slower threads still sum row r
    uint32_t* const pix2 = reinterpret_cast<uint32_t*>(Qb + 2 * rph) + p * PP;
    const uint2* Lp = a.planes + (size_t)(pair * 2) * a.H * W;
    const uint2* Rp = Lp + (size_t)a.H * W;
    const rsrc_t rc = make_rsrc(a.C + pair * a.C_pair, (uint64_t)a.H * W1 * D * 2);

    const int yb0 = blockIdx.y * a.band, yb1 = min(yb0 + a.band, a.Yc);
    const int r0 = yb0 - S, nsteps = yb1 + S - r0;  // input rows r0 .. yb1-1+S

    // register prefetch of one input row's planes: left halo columns, right column pairs
    constexpr int NL = NLR, NR = NLR;  // host: NHC, rpairs <= NLR * blockDim
    uint2 pl[NL], pr0[NR], pr1[NR];
    auto load_row = [&](int r) {
        const int y = min(max(r, 0), a.H - 1);
        const uint2* lrow = Lp + (size_t)y * W + a.minX1;
        const uint2* rrow = Rp + (size_t)y * W + rb;
#pragma unroll
        for (int i = 0; i < NL; i++) {
            const int c = tid + i * (int)blockDim.x;
            if (c < NHC) pl[i] = lrow[min(max(x0 - S + c, 0), W1 - 1)];
        }
#pragma unroll
        for (int i = 0; i < NR; i++) {
            const int k = tid + i * (int)blockDim.x;
            if (k < rpairs) {
                pr0[i] = rrow[k];
                pr1[i] = rrow[k + 1];
            }
        }
    };
    auto stage_row = [&]() {
#pragma unroll
        for (int i = 0; i < NL; i++) {
            const int c = tid + i * (int)blockDim.x;
            if (c < NHC) {
                const uint2 L = pl[i];
                Ua[c] = make_uint4(__builtin_amdgcn_perm(0, L.x, 0x0c000c00u), __builtin_amdgcn_perm(0, L.x, 0x0c010c01u),
                                   __builtin_amdgcn_perm(0, L.x, 0x0c020c02u), __builtin_amdgcn_perm(0, L.x, 0x0c030c03u));
                Ub[c] = make_uint2(__builtin_amdgcn_perm(0, L.y, 0x0c000c00u), __builtin_amdgcn_perm(0, L.y, 0x0c010c01u));
            }
        }
#pragma unroll
        for (int i = 0; i < NR; i++) {
            const int k = tid + i * (int)blockDim.x;
            if (k < rpairs) {
                const uint2 c0 = pr0[i], c1 = pr1[i];
                const int q = (k & 1) * rph + (k >> 1);
                // u16 pair (col k+1 | col k << 16): lanes (d, d+1) of one column
                Qa[q] = make_uint4(__builtin_amdgcn_perm(c1.x, c0.x, 0x0c000c04u), __builtin_amdgcn_perm(c1.x, c0.x, 0x0c010c05u),
                                   __builtin_amdgcn_perm(c1.x, c0.x, 0x0c020c06u), __builtin_amdgcn_perm(c1.x, c0.x, 0x0c030c07u));
                Qb[q] = make_uint2(__builtin_amdgcn_perm(c1.y, c0.y, 0x0c000c04u), __builtin_amdgcn_perm(c1.y, c0.y, 0x0c010c05u));
            }
        }
    };

    uint32_t ring[R][CPT], vs[CPT];
#pragma unroll
    for (int q = 0; q < R; q++)
#pragma unroll
        for (int i = 0; i < CPT; i++) ring[q][i] = 0;
#pragma unroll
    for (int i = 0; i < CPT; i++) vs[i] = 0;
    const int hx0 = cg * CPT;  // first own column, halo index minus S
    // valid halo columns (inside [0, W1)): [hlo, hhi]; strips at the image edges clamp
    const int hlo = max(0, S - x0), hhi = min(NHC - 1, W1 - 1 - x0 + S);
    const bool edge = hlo > 0 || hhi < NHC - 1;
    // BT work split: thread cg computes halo columns [hb0, hb1) of its pair p
    const int per = (NHC + CG - 1) / CG;
    // (every thread computes its whole run: halo columns outside [hlo, hhi] hold clamped-edge
    // garbage that the edge path of the horizontal sum never reads)
    const int hb0 = cg * per;
    // right pair index of column hb0 (and hb0 + 1) -> parity-split LDS slots
    const int kk0 = (x0 - S + hb0) - xlo + D - 2 - 2 * p;
    const int q0 = (kk0 & 1) * rph + (kk0 >> 1), q1 = ((kk0 + 1) & 1) * rph + ((kk0 + 1) >> 1);

    load_row(r0);
    for (int s0 = 0; s0 < nsteps; s0 += R) {
#pragma unroll
        for (int q = 0; q < R; q++) {
            const int st = s0 + q;
            if (st < nsteps) {  // workgroup-uniform
                // Ua/Qa were last read by the previous row's BT, which every thread
                // finished before the previous row's second barrier: no barrier here
                uint32_t* const pix = pix2 + (st & 1) * (NP * PP);
                stage_row();
                if (st + 1 < nsteps) load_row(r0 + st + 1);
                __syncthreads();
                // BT costs of this thread's contiguous run of valid halo columns, pair p
                {
                    int hc = hb0;
                    const uint4* ua = Ua + hc;
                    const uint2* ub = Ub + hc;
                    const uint4* qa0 = Qa + q0;
                    const uint2* qb0 = Qb + q0;
                    const uint4* qa1 = Qa + q1;
                    const uint2* qb1 = Qb + q1;
                    auto bt = [&](uint4 uA, uint2 uB, uint4 qa, uint2 qb) -> uint32_t {
                        const u16x2 U0 = as_u16x2(uA.x), U1 = as_u16x2(uA.y), U2 = as_u16x2(uA.z);
                        const u16x2 U3 = as_u16x2(uA.w), U4 = as_u16x2(uB.x), U5 = as_u16x2(uB.y);
                        const u16x2 V0 = as_u16x2(qa.x), V1 = as_u16x2(qa.y), V2 = as_u16x2(qa.z);
                        const u16x2 V3 = as_u16x2(qa.w), V4 = as_u16x2(qb.x), V5 = as_u16x2(qb.y);
                        const u16x2 g = __builtin_elementwise_min(__builtin_elementwise_max(subsat(U0, V2), subsat(V1, U0)),
                                                                  __builtin_elementwise_max(subsat(V0, U2), subsat(U1, V0)));
                        const u16x2 rr = __builtin_elementwise_min(__builtin_elementwise_max(subsat(U3, V5), subsat(V4, U3)),
                                                                   __builtin_elementwise_max(subsat(V3, U5), subsat(U4, V3)));
                        return as_u32(g + (rr >> (u16x2)2));
                    };
                    // consecutive columns alternate the parity of their right pair index;
                    // unrolled to the longest run (immediate LDS offsets from six bases: the
                    // rolled loop spent 17 address / counter ops per 32 BT ops)
                    // a run of N = per columns, N known at compile time for per = CPT + 1 or
                    // CPT + 2: groups of KG columns issue all their loads, then the BT ops, then
                    // the stores (the compiler cannot move a load above a pix store: one LDS array)
                    auto bt_run = [&](auto nc) {
                        constexpr int N = decltype(nc)::value, KG = 2;
#pragma unroll
                        for (int j0 = 0; j0 < N; j0 += KG) {
                            uint4 A[KG], Q[KG];
                            uint2 B[KG], R[KG];
#pragma unroll
                            for (int k = 0; k < KG; k++) {
                                const int j = j0 + k;
                                if (j < N) {
                                    A[k] = ua[j];
                                    B[k] = ub[j];
                                    Q[k] = (j & 1) ? qa1[j >> 1] : qa0[j >> 1];
                                    R[k] = (j & 1) ? qb1[j >> 1] : qb0[j >> 1];
                                }
                            }
#pragma unroll
                            for (int k = 0; k < KG; k++)
                                if (j0 + k < N) pix[hc + j0 + k] = bt(A[k], B[k], Q[k], R[k]);
                        }
                    };
                    if (per == CPT + 1) {
                        bt_run(std::integral_constant<int, CPT + 1>{});
                    } else if (per == CPT + 2) {
                        bt_run(std::integral_constant<int, CPT + 2>{});
                    } else {
                        for (int j = 0; j < per; j++)
                            pix[hc + j] = (j & 1) ? bt(ua[j], ub[j], qa1[j >> 1], qb1[j >> 1])
                                                  : bt(ua[j], ub[j], qa0[j >> 1], qb0[j >> 1]);
                    }
                }
                __syncthreads();
                // running horizontal sum along the thread's CPT columns (halo columns past
                // the image edge repeat the edge column), then the vertical ring
                uint32_t v[CPT + 2 * S];
                if (edge) {
#pragma unroll
                    for (int j = 0; j < CPT + 2 * S; j++) v[j] = pix[min(max(hx0 + j, hlo), hhi)];
                } else {
#pragma unroll
                    for (int j = 0; j < CPT + 2 * S; j++) v[j] = pix[hx0 + j];
                }
                uint32_t h = 0;
#pragma unroll
                for (int j = 0; j < 2 * S + 1; j++) h += v[j];
                const int y = r0 + st - S;  // output row of this step (valid when st >= 2S)
                const uint32_t ob = (((uint32_t)max(y, 0) * W1 + x0 + hx0) * D + 2 * p) * 2;
                const int nval = st >= 2 * S ? W1 - (x0 + hx0) : 0;
#pragma unroll
                for (int i = 0; i < CPT; i++) {
                    if (i) h += v[i + 2 * S] - v[i - 1];
                    vs[i] += h;
                    ring[q][i] = h;
                    // column step as the scalar offset: one voffset for all CPT stores
                    if (i < nval) {
                        if (a.nt) __builtin_amdgcn_raw_buffer_store_b32(vs[i], rc, ob, i * 2 * D, 2);
                        else __builtin_amdgcn_raw_buffer_store_b32(vs[i], rc, ob, i * 2 * D, 0);
                    }
                    vs[i] -= ring[(q + 1) % R][i];  // row r - 2S leaves the window
                }
            }
        }
    }
}

// Rows y >= Yc: MODE_SGBM reuses one C row, so they stay equal to row Yc-1;
// MODE_HH keeps one C row per y that is never updated (P2 seed only: C_true = 0).
__global__ void __launch_bounds__(256) k_sgbm_cost_tail(uint16_t* C, size_t C_pair, int H, int Yc, size_t row_elems, int hh)
{
    C += blockIdx.y * C_pair;  // one launch for the group's pairs
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

// Cost of the pad planes Dv..D-1 of a volume whose plane count Dv is not a multiple of 16
// (the kernels run D = the next multiple).  With C_pad >= VOL_CMAX + P2 no real disparity's
// path value ever takes a pad value as its minimum:
//  * every path keeps min over the real d of L <= VOL_CMAX (at the predecessor's argmin d0,
//    min(Lp[d0], ...) - minLp = 0, so L[d0] = C[d0]; the first step has Lp = 0);
//  * every pad value L >= C_pad (min(...) - minLp >= 0), so minLp over all D planes is the
//    minimum over the real ones, and at d = Dv-1 the term Lp[Dv] + P1 > minLp + P2 never
//    undercuts the min(...) of the unpadded recurrence (its edge Lp[Dv] = MAX).
// Pad values stay <= C_pad + P2 <= 28671 (normalize: P2 <= 12288), so no u16 path arithmetic
// wraps on them; the WTA kernels give the pad planes S = 0xFFFF (never the minimum, never
// "far") and take the sub-pixel step only for 0 < best < Dv - 1.
__host__ __device__ constexpr int vol_pad_cost(int P2) { return VOL_CMAX + P2; }

struct VolArgs {
    const float* vol;
    size_t vol_pair;  // elements between pairs
    uint16_t* C;
    size_t C_pair;  // elements between pairs
    int H, W, width1, D, minX1;
    int Dv;    // planes of the input volume (<= D); planes Dv..D-1 of C get cpad
    int cpad;  // vol_pad_cost(P2)
    int nt;  // 1: nontemporal stores (the launch group's volume exceeds the Infinity Cache)
    float offset, scale;
    const float* win;  // automatic window: [pair][2] = offset, scale (k_vol_window), else null
    // cells whose quantised value was clamped into [0, VOL_CMAX] / that were NaN (device counters)
    unsigned long long *clamped, *nans;
    uint32_t* zero_word;  // see CensusArgs
};

// ---- automatic quantisation window (sm_aggregate_cost_f32* with scale == 0): per pair, the
// finite minimum and maximum over the cells that get quantised (planes < Dv, every row, the
// matcher's columns [minX1, minX1 + width1)), then offset = -min, scale = VOL_CMAX / (max - min)
// in float32 (IEEE division; the oracle computes the same two roundings), so the whole range
// maps onto [0, VOL_CMAX] and no finite cost is clamped.
struct VolWinArgs {
    const float* vol;
    size_t vol_pair;  // elements between pairs
    int Dv, H, W, minX1, width1;
    uint32_t* keys;  // [pair][2]: order-preserving u32 keys of the minimum and the maximum
    float* win;      // [pair][2]: offset, scale
};

// unsigned order of the key = order of the float (no NaN enters)
__device__ inline uint32_t fkey(float f)
{
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ inline float fkey_inv(uint32_t k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k); }

__global__ void k_vol_keys_init(uint32_t* keys, int npairs)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < npairs) {
        keys[2 * i] = 0xFFFFFFFFu;
        keys[2 * i + 1] = 0u;
    }
}

// grid (blocks, pairs), 256 threads: block b reduces the domain rows (plane, y) = b, b + gridDim.x, ...
__global__ void __launch_bounds__(256) k_vol_minmax(VolWinArgs a)
{
    __shared__ uint32_t smin[4], smax[4];
    const float* v = a.vol + (size_t)blockIdx.y * a.vol_pair + a.minX1;
    uint32_t kmin = 0xFFFFFFFFu, kmax = 0u;
    const int lines = a.Dv * a.H;
    for (int l = blockIdx.x; l < lines; l += gridDim.x) {
        const float* row = v + (size_t)l * a.W;  // plane l / H, row l % H: planes are H*W apart
        for (int x = threadIdx.x; x < a.width1; x += 256) {
            const float f = __builtin_nontemporal_load(row + x);
            if (__builtin_isfinite(f)) {
                const uint32_t k = fkey(f);
                kmin = min(kmin, k);
                kmax = max(kmax, k);
            }
        }
    }
    kmin = group_min_u32_wave(kmin);
    kmax = group_max_u32_wave(kmax);
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        smin[wave] = kmin;
        smax[wave] = kmax;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; w++) {
            kmin = min(kmin, smin[w]);
            kmax = max(kmax, smax[w]);
        }
        if (kmin <= kmax) {
            atomicMin(&a.keys[2 * blockIdx.y], kmin);
            atomicMax(&a.keys[2 * blockIdx.y + 1], kmax);
        }
    }
}

__global__ void k_vol_window(VolWinArgs a, int npairs)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npairs) return;
    const uint32_t k0 = a.keys[2 * i], k1 = a.keys[2 * i + 1];
    float off = 0.f, sc = 1.f;  // no finite cost at all
    if (k0 <= k1) {
        const float mn = fkey_inv(k0), mx = fkey_inv(k1);
        off = -mn;
        const float d = mx - mn;
        sc = (d > 0.f && __builtin_isfinite(d)) ? (float)VOL_CMAX / d : 1.f;
    }
    a.win[2 * i] = off;
    a.win[2 * i + 1] = sc;
}

__device__ inline uint32_t quant_cost(float c, float off, float sc)
{
    if (c != c) return VOL_CMAX;
    const float v = __builtin_rintf((c + off) * sc);
    if (!(v > 0.f)) return 0;
    if (v > (float)VOL_CMAX) return VOL_CMAX;
    return (uint32_t)v;
}

// quant_cost, counting NaN cells and cells clamped into [0, VOL_CMAX]
__device__ inline uint32_t quant_cost_n(float c, float off, float sc, uint32_t& nclamp, uint32_t& nnan)
{
    if (c != c) {
        nnan++;
        return VOL_CMAX;
    }
    const float v = __builtin_rintf((c + off) * sc);
    nclamp += (v < 0.f || v > (float)VOL_CMAX || v != v) ? 1u : 0u;
    if (!(v > 0.f)) return 0;
    if (v > (float)VOL_CMAX) return VOL_CMAX;
    return (uint32_t)v;
}

// TX columns per tile (64 or 128): each lane reads TX/64 consecutive floats
// of a plane row (64 lanes cover the tile's TX columns, TX*4 contiguous bytes).
template <int TX>
__global__ void __launch_bounds__(256) k_cost_volume_f32(VolArgs a)
{
    clear_group_flag(a.zero_word);
    constexpr int PL = TX / 64;         // floats per lane per plane row
    extern __shared__ uint32_t tile[];  // [TX][D/2 + 1] packed u16 pairs (d even | d odd << 16)
    const int half = a.D >> 1, rowdw = half + 1;
    const int x0 = blockIdx.x * TX, y = blockIdx.y, pair = blockIdx.z;
    const float qoff = a.win ? a.win[2 * pair] : a.offset, qsc = a.win ? a.win[2 * pair + 1] : a.scale;
    uint32_t nclamp = 0, nnan = 0;
    const int nx = min(TX, a.width1 - x0);
    const size_t plane = (size_t)a.H * a.W;
    const float* v = a.vol + pair * a.vol_pair + (size_t)y * a.W + a.minX1 + x0;
    for (int i = threadIdx.x; i < 64 * half; i += 256) {
        const int xl = (i & 63) * PL, dp = i >> 6;
        // planes 2dp, 2dp + 1 inside the input volume (wave-uniform); the pad planes are
        // never read and get the pad cost (vol_pad_cost)
        const bool in0 = 2 * dp < a.Dv, in1 = 2 * dp + 1 < a.Dv;
        const float* p0 = v + (size_t)(2 * dp) * plane + xl;
        const float* p1 = p0 + plane;
        float c0[PL], c1[PL];
#pragma unroll
        for (int k = 0; k < PL; k++) c0[k] = c1[k] = 0.f;
        if (xl + PL <= nx) {
            if constexpr (PL == 2) {
                typedef float f2v __attribute__((ext_vector_type(2)));
                if (in0) {
                    const f2v a0 = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(p0));
                    c0[0] = a0[0]; c0[1] = a0[1];
                }
                if (in1) {
                    const f2v a1 = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(p1));
                    c1[0] = a1[0]; c1[1] = a1[1];
                }
            } else {
#pragma unroll
                for (int k = 0; k < PL; k++) {
                    if (in0) c0[k] = __builtin_nontemporal_load(p0 + k);
                    if (in1) c1[k] = __builtin_nontemporal_load(p1 + k);
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < PL; k++) {
                c0[k] = in0 && xl + k < nx ? p0[k] : 0.f;
                c1[k] = in1 && xl + k < nx ? p1[k] : 0.f;
            }
        }
#pragma unroll
        for (int k = 0; k < PL; k++) {
            const bool x_in = xl + k < nx;  // (columns past the domain are loaded as 0, not counted)
            uint32_t q0 = (uint32_t)a.cpad, q1 = (uint32_t)a.cpad;
            if (in0) q0 = x_in ? quant_cost_n(c0[k], qoff, qsc, nclamp, nnan) : quant_cost(c0[k], qoff, qsc);
            if (in1) q1 = x_in ? quant_cost_n(c1[k], qoff, qsc, nclamp, nnan) : quant_cost(c1[k], qoff, qsc);
            tile[(xl + k) * rowdw + dp] = q0 | (q1 << 16);
        }
    }
    if (a.clamped) {  // one atomic per wave that saw any
        nclamp = group_sum_u32_wave(nclamp);
        nnan = group_sum_u32_wave(nnan);
        if ((threadIdx.x & 63) == 0) {
            if (nclamp) atomicAdd(a.clamped, (unsigned long long)nclamp);
            if (nnan) atomicAdd(a.nans, (unsigned long long)nnan);
        }
    }
    __syncthreads();
    uint32_t* out = reinterpret_cast<uint32_t*>(a.C + pair * a.C_pair + ((size_t)y * a.width1 + x0) * a.D);
    const int total = nx * half;
    for (int i = threadIdx.x; i < total; i += 256) {
        const int xl = i / half, j = i - xl * half;
        if (a.nt) __builtin_nontemporal_store(tile[xl * rowdw + j], out + i);
        else out[i] = tile[xl * rowdw + j];
    }
}

}  // namespace smk
