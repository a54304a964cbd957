// sm_wide.hpp — OpenCV-SGBM outside the int16-exact range, on gfx950.
//
// The fast kernels (sm_cost.hpp, sm_paths.hpp, sm_sweep.hpp) assume no sum can
// reach 2^15, where saturating and plain arithmetic agree.  The reference's
// direct-matcher scripts leave that range: disparity_test.py:165-177
// (blockSize 23, preFilterCap 1, P2 887) and try_try.py:69-77 (BGR input,
// blockSize 16).  OpenCV's x86 build then decides the result through its
// CV_SIMD128 int16 arithmetic (restated in oracle/sgm_ref.c, header):
//   * C row 0: scalar loop with int16 casts   C = wrap16(C + hsum[k] * scale)
//   * C rows y >= 1 (while y + SH2 < H), saturating SIMD updates
//       x1 == 0:  C = sat16(sat16(Cprev + hsum[y+SH2]) - hsum[y-SH2-1])
//       x1 >= 1:  C = sat16(sat16(Cprev - hsum[y-SH2-1]) + hsum[y+SH2])
//     later rows frozen (MODE_SGBM) or left at the P2 seed (MODE_HH);
//   * every L step  L = sat16(sat16(min(Lp[d], sat16(Lp[d+-1] + P1), delta) - delta) + C)
//     with delta = wrap16(min_d Lp + P2) and Lp[-1] = Lp[D] = 32767;
//   * S = sat16 sums in OpenCV's order (E+SE, S+SW; then W (MODE_SGBM) or
//     W+NE, N+NW (MODE_HH)); WTA with signed S.
// So this path keeps OpenCV's int16 cost volume C (P2 seed included) and
// int16 path volumes, and computes them with sequential scans in the same
// order: rows in k_wide_vscan, path lines in k_wide_paths.  It serves only
// configurations the fast path cannot reproduce; it trades speed for
// exactness (simple line-per-16-lanes mapping, no fused sweeps).
#pragma once
#include "sm_common.hpp"

namespace smk {

__device__ __forceinline__ int sat16(int v) { return ::min(::max(v, -32768), 32767); }
__device__ __forceinline__ int wrap16(int v) { return (int)(int16_t)(uint16_t)(uint32_t)v; }

struct WideArgs {
    const uint2* planes;  // k_sgbm_prefilter planes [pair][view][cn][H][W]
    int16_t* hsum;        // [pair][H][width1][D] horizontal box sums
    int16_t* C;           // [pair][H][width1][D] OpenCV's C rows (P2 seed included)
    size_t vol;           // cells per pair
    int H, W, width1, D, minD, minX1, cn, SW2, SH2, P2, hh;  // hh: MODE_HH (fullDP) row rules
};

// BT cost of one channel plane pair: bytes [g, g_min, g_max, raw, raw_min, raw_max]
__device__ __forceinline__ int bt_pair(uint2 l, uint2 r)
{
    const int u = l.x & 255, u0 = (l.x >> 8) & 255, u1 = (l.x >> 16) & 255;
    const int v = r.x & 255, v0 = (r.x >> 8) & 255, v1 = (r.x >> 16) & 255;
    const int g = ::min(::max(::max(0, u - v1), v0 - u), ::max(::max(0, v - u1), u0 - v));
    const int U = l.x >> 24, U0 = l.y & 255, U1 = (l.y >> 8) & 255;
    const int V = r.x >> 24, V0 = r.y & 255, V1 = (r.y >> 8) & 255;
    const int w = ::min(::max(::max(0, U - V1), V0 - U), ::max(::max(0, V - U1), U0 - V));
    return g + (w >> 2);
}

// Horizontal box sums of one row strip: pixel costs of TX columns + 2*SW2 halo
// (clamped to [0, width1)) into LDS, then the (2*SW2+1)-wide window per
// (x1, d): OpenCV's running sums exactly while no window sum can pass 32767 (the host
// checks (2*SW2+1) * cn * (2*ftzero + 63); else k_wide_hsum_scan).  blockIdx = (strip, y, pair).
template <int TX>
__global__ void __launch_bounds__(256) k_wide_hsum(WideArgs a)
{
    extern __shared__ int16_t pix[];  // [TX + 2*SW2][D]
    const int x0 = blockIdx.x * TX, y = blockIdx.y, pair = blockIdx.z;
    const int D = a.D, W = a.W, W1 = a.width1, SW2 = a.SW2, cn = a.cn;
    const int ca = max(x0 - SW2, 0), cb = min(x0 + TX + SW2, W1);  // staged columns [ca, cb)
    const uint2* Lp = a.planes + (size_t)(pair * 2) * cn * a.H * W + (size_t)y * W;
    const uint2* Rp = Lp + (size_t)cn * a.H * W;
    const size_t plane = (size_t)a.H * W;
    for (int i = threadIdx.x; i < (cb - ca) * D; i += 256) {
        const int c = i / D, d = i - c * D;
        const int X = ca + c + a.minX1, Xr = X - a.minD - d;
        int s = 0;
        for (int ch = 0; ch < cn; ch++) s += bt_pair(Lp[ch * plane + X], Rp[ch * plane + Xr]);
        pix[c * D + d] = (int16_t)s;
    }
    __syncthreads();
    int16_t* out = a.hsum + (size_t)pair * a.vol + (size_t)y * W1 * D;
    const int xe = min(x0 + TX, W1);
    for (int i = threadIdx.x; i < (xe - x0) * D; i += 256) {
        const int c = i / D, d = i - c * D;
        const int x1 = x0 + c;
        int s = 0;
        for (int j = -SW2; j <= SW2; j++) s += pix[(min(max(x1 + j, 0), W1 - 1) - ca) * D + d];
        out[(size_t)x1 * D + d] = (int16_t)s;
    }
}

// k_wide_hsum where a window sum can pass 32767 ((2*SW2+1) * cn * (2*ftzero + 63) above
// it): OpenCV's own running scan along x, one thread per (row, d).  The rows it reads
// while the C rows are initialised (k <= SH2, y == 0) wrap like its scalar loop; the rows
// entering during the scan (k > SH2) saturate like its int16 SIMD update
//   hv = sat16(sat16(hv - pix[max(x - SW2 - 1, 0)]) + pix[min(x + SW2, width1 - 1)]).
// blockIdx = (row, pair).
__global__ void __launch_bounds__(256) k_wide_hsum_scan(WideArgs a)
{
    const int y = blockIdx.x, pair = blockIdx.y;
    const int D = a.D, W = a.W, W1 = a.width1, SW2 = a.SW2, cn = a.cn;
    const uint2* Lp = a.planes + (size_t)(pair * 2) * cn * a.H * W + (size_t)y * W;
    const uint2* Rp = Lp + (size_t)cn * a.H * W;
    const size_t plane = (size_t)a.H * W;
    const bool sat = y > a.SH2;
    int16_t* out = a.hsum + (size_t)pair * a.vol + (size_t)y * W1 * D;
    for (int d = threadIdx.x; d < D; d += 256) {
        auto pix = [&](int x1) {
            const int X = x1 + a.minX1, Xr = X - a.minD - d;
            int s = 0;
            for (int ch = 0; ch < cn; ch++) s += bt_pair(Lp[ch * plane + X], Rp[ch * plane + Xr]);
            return s;
        };
        int hv = pix(0) * (SW2 + 1);
        for (int x = 1; x <= SW2; x++) hv += pix(min(x, W1 - 1));
        hv = wrap16(hv);
        out[d] = (int16_t)hv;
        for (int x = 1; x < W1; x++) {
            const int add = pix(min(x + SW2, W1 - 1)), sub = pix(max(x - SW2 - 1, 0));
            hv = sat ? sat16(sat16(hv - sub) + add) : wrap16(hv + add - sub);
            out[(size_t)x * D + d] = (int16_t)hv;
        }
    }
}

// OpenCV's incremental vertical box update, one thread per (x1, d), rows in order.
__global__ void __launch_bounds__(256) k_wide_vscan(WideArgs a)
{
    const int D = a.D, W1 = a.width1, H = a.H, SH2 = a.SH2;
    const int pair = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= W1 * D) return;
    const bool x0col = i < D;
    const size_t row = (size_t)W1 * D;
    const int16_t* hs = a.hsum + (size_t)pair * a.vol + i;
    int16_t* C = a.C + (size_t)pair * a.vol + i;
    int c = a.P2;
    for (int k = 0; k <= SH2; k++)  // row 0: scalar loop, int16 casts
        c = wrap16(c + (int)hs[(size_t)min(k, H - 1) * row] * (k == 0 ? SH2 + 1 : 1));
    C[0] = (int16_t)c;
    for (int y = 1; y < H; y++) {
        if (y + SH2 < H) {
            const int add = hs[(size_t)(y + SH2) * row], sub = hs[(size_t)max(y - SH2 - 1, 0) * row];
            c = x0col ? sat16(sat16(c + add) - sub) : sat16(sat16(c - sub) + add);
        } else if (a.hh) {
            c = a.P2;  // MODE_HH: rows past the last update keep the P2 seed
        }              // MODE_SGBM: the C row buffer keeps its last update
        C[(size_t)y * row] = (int16_t)c;
    }
}

struct WidePathArgs {
    const int16_t* C;  // [pair][H][width1][D]
    size_t vol;        // cells per pair
    uint8_t* L;        // int16 path volumes [pair][slot][H][width1][D]
    size_t slot_bytes, L_pair_bytes;
    int H, width1, D, P1, P2, ndirs;
    int blk_start[9];  // first workgroup of each direction (slot order), blk_start[ndirs] = total
};

// One path line per 16-lane group (DPL = D/16 disparities per lane), 16 lines
// per workgroup; directions in slot order E, W, SE, S, SW, NE, N, NW.  A line
// enters the domain with Lp = 0, min Lp = 0 (OpenCV's zeroed border slots).
template <int DPL>
__global__ void __launch_bounds__(256) k_wide_paths(WidePathArgs a)
{
    const int pair = blockIdx.y;
    int k = 0;
    while (k + 1 < a.ndirs && (int)blockIdx.x >= a.blk_start[k + 1]) k++;
    const int l = ((int)blockIdx.x - a.blk_start[k]) * 16 + (int)(threadIdx.x >> 4);
    const int g = threadIdx.x & 15;
    const int dxs[8] = {1, -1, 1, 0, -1, 1, 0, -1}, dys[8] = {0, 0, 1, 1, 1, -1, -1, -1};
    const int dx = dxs[k], dy = dys[k], H = a.H, W1 = a.width1, D = a.D;
    int y, x, s0, s1;
    if (dy == 0) {  // a row
        if (l >= H) return;
        y = l;
        x = dx > 0 ? 0 : W1 - 1;
        s0 = 0;
        s1 = W1;
    } else {  // column / diagonal starting on the first row of the sweep, unwrapped
        const int nl = dx == 0 ? W1 : W1 + H - 1;
        if (l >= nl) return;
        const int xs = dx > 0 ? l - (H - 1) : l;
        y = dy > 0 ? 0 : H - 1;
        x = xs;
        s0 = dx > 0 ? max(0, -xs) : dx < 0 ? max(0, xs - (W1 - 1)) : 0;
        s1 = dx > 0 ? min(H, W1 - xs) : dx < 0 ? min(H, xs + 1) : H;
    }
    const int16_t* Cb = a.C + (size_t)pair * a.vol + g * DPL;
    int16_t* Lb = reinterpret_cast<int16_t*>(a.L + (size_t)pair * a.L_pair_bytes + (size_t)k * a.slot_bytes) + g * DPL;
    const int P1 = a.P1, P2 = a.P2;
    int Lp[DPL];
#pragma unroll
    for (int i = 0; i < DPL; i++) Lp[i] = 0;
    int delta = wrap16(0 + P2);
    for (int s = s0; s < s1; s++) {
        const int yy = y + s * dy, xx = x + s * dx;
        const size_t off = ((size_t)yy * W1 + xx) * D;
        // neighbours d-1 / d+1 across the line's lanes (biased to u32 for the DPP moves)
        const int lm = (int)Line<16>::prev(0xFFFFu, (uint32_t)(Lp[DPL - 1] + 32768)) - 32768;
        const int lq = (int)Line<16>::next(0xFFFFu, (uint32_t)(Lp[0] + 32768)) - 32768;
        uint32_t mn = 0xFFFFFFFFu;
        int Ln[DPL];
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            const int a1 = i == 0 ? lm : Lp[i - 1];
            const int a2 = i == DPL - 1 ? lq : Lp[i + 1];
            int v = ::min(Lp[i], ::min(sat16(a1 + P1), sat16(a2 + P1)));
            v = ::min(v, delta);
            Ln[i] = sat16(sat16(v - delta) + (int)Cb[off + i]);
            mn = ::min(mn, (uint32_t)(Ln[i] + 32768));
        }
        const int minL = (int)Line<16>::min(mn) - 32768;
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            Lb[off + i] = (int16_t)Ln[i];
            Lp[i] = Ln[i];
        }
        delta = wrap16(minL + P2);
    }
}

struct WideWtaArgs {
    const uint8_t* L;  // int16 path volumes, slots E, W, SE, S, SW[, NE, N, NW]
    size_t slot_bytes, L_pair_bytes;
    int H, W, width1, D, minD, minX1, uniq, disp12, ndirs;
    int16_t* disp;  // [pair][H][W] pre-median
    int16_t* wta;   // [pair][H][W] integer WTA index (best, -1 rejected / outside the domain), or null
};

// S in OpenCV's saturating order, WTA (MODE_SGBM: SIMD lane tie-break), the
// uniqueness test, sub-pixel step, disp2 and the disp12MaxDiff check; one
// workgroup of NT threads per (row, pair), a 16-lane group per pixel.
template <int DPL, int NT>
__global__ void __launch_bounds__(NT) k_wide_wta(WideWtaArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int W = a.W, D = a.D, minD = a.minD, minX1 = a.minX1, maxX1 = minX1 + a.width1;
    const int INVALID = (minD - 1) * 16;
    const int y = blockIdx.x, pair = blockIdx.y;
    uint32_t* key2 = smem;
    int* drow = reinterpret_cast<int*>(smem + W);
    int16_t* brow = reinterpret_cast<int16_t*>(smem + 2 * W);  // integer WTA index (only with a.wta)
    for (int i = threadIdx.x; i < W; i += NT) {
        key2[i] = 0xFFFFFFFFu;
        drow[i] = INVALID;
        if (a.wta) brow[i] = -1;
    }
    __syncthreads();
    const int g = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const bool lane8 = a.ndirs == 5;
    const int16_t* Lb = reinterpret_cast<const int16_t*>(a.L + (size_t)pair * a.L_pair_bytes) + g * DPL;
    const size_t slot = a.slot_bytes / 2;
    const int u = a.uniq;
    for (int x = grp; x < a.width1; x += NT / 16) {
        const size_t off = ((size_t)y * a.width1 + x) * D;
        int S[DPL];
        uint32_t key = 0xFFFFFFFFu;
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            auto Lk = [&](int k) { return (int)Lb[(size_t)k * slot + off + i]; };
            int s = sat16(sat16(0 + sat16(Lk(0) + Lk(2))) + sat16(Lk(3) + Lk(4)));  // E+SE, S+SW
            if (a.ndirs == 5)
                s = sat16(Lk(1) + s);  // backward W pass: L0 + Sp
            else
                s = sat16(sat16(s + sat16(Lk(1) + Lk(5))) + sat16(Lk(6) + Lk(7)));  // W+NE, N+NW
            S[i] = s;
            key = ::min(key, ((uint32_t)(s + 32768) << 16) | wta_rank(g * DPL + i, lane8));
        }
        key = row16_min(key);
        const int minS = (int)(key >> 16) - 32768, best = wta_unrank(key & 0xFFFF, lane8);
        uint32_t bad = 0, nb = 0;
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            const int d = g * DPL + i, dd = best - d;
            bad |= (S[i] * (100 - u) < minS * 100 && (dd > 1 || dd < -1)) ? 1u : 0u;
            nb |= d == best - 1 ? (uint32_t)(S[i] + 32768) : 0u;
            nb |= d == best + 1 ? ((uint32_t)(S[i] + 32768) << 16) : 0u;
        }
        bad = row16_or(bad);
        nb = row16_or(nb);
        // minS == 32767: every S saturated, OpenCV's bestDisp stays -1 (invalid)
        if (g == 0 && !bad && minS < 32767) {
            const int X = x + minX1;
            atomicMin(&key2[X - best - minD], ((uint32_t)(minS + 32768) << 16) | (uint32_t)(0xFFFF - X));
            int d16 = best * 16;
            if (best > 0 && best < D - 1) {
                const int Sm = (int)(nb & 0xFFFF) - 32768, Sq = (int)(nb >> 16) - 32768;
                d16 += subpix_step(Sm, Sq, minS);  // C truncation
            }
            drow[X] = d16 + minD * 16;
            if (a.wta) brow[X] = (int16_t)best;
        }
    }
    __syncthreads();
    int16_t* out = a.disp + (size_t)pair * a.H * W + (size_t)y * W;
    for (int X = threadIdx.x; X < W; X += NT) {
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
        if (a.wta) a.wta[(size_t)pair * a.H * W + (size_t)y * W + X] = brow[X];
    }
}

}  // namespace smk
