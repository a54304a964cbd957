// sm_bm.hpp — cv::StereoBM on the GPU (the reference's
// method="BM" branch, stereo_vision/stereo_vision.py:164-166).  Semantics:
// oracle/bm_np.py (X-Sobel prefilter, clamped SAD windows, texture and
// uniqueness tests, V-shaped integer sub-pixel fit, validateDisparity,
// speckles).
//
//   k_bm_prefilter  X-Sobel prefilter of both views (row pairs as OpenCV).
//   k_bm_fill       FILTERED everywhere (the region below is overwritten).
//   k_bm_sad        one workgroup per (strip of SWs output columns, band of
//                   rows, pair): column sums of |L - R| over the window height
//                   kept in LDS (vsum[column][d]) and slid down the band (add
//                   the entering row, subtract the leaving one), a horizontal
//                   sliding sum per disparity gives SAD[x][d], then WTA +
//                   texture + uniqueness + sub-pixel per pixel with
//                   256/SWs lanes per pixel.  Integer arithmetic: bit-exact.
//   k_bm_validate   validateDisparity (disp12MaxDiff >= 0), one block per row.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smk {

struct BmPrefilterArgs {
    const uint8_t* img[2];
    size_t in_pair;
    int stride;
    uint8_t* out[2];  // [pair][H][W]
    int H, W, cap;
};

__global__ void __launch_bounds__(256) k_bm_prefilter(BmPrefilterArgs a)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    const int which = blockIdx.z & 1, pair = blockIdx.z >> 1;
    if (x >= a.W) return;
    const uint8_t* src = a.img[which] + (size_t)pair * a.in_pair;
    uint8_t* dst = a.out[which] + (size_t)pair * a.H * a.W;
    int v = a.cap;
    const bool last_odd = (a.H & 1) && y == a.H - 1;
    if (x > 0 && x < a.W - 1 && a.W >= 3 && !last_odd) {
        const int yu = y > 0 ? y - 1 : min(1, a.H - 1);
        const int yd = y < a.H - 1 ? y + 1 : max(a.H - 2, 0);
        auto dx = [&](int r) { const uint8_t* p = src + (size_t)r * a.stride; return (int)p[x + 1] - (int)p[x - 1]; };
        const int d = dx(yu) + 2 * dx(y) + dx(yd);
        v = min(max(d, -a.cap), a.cap) + a.cap;
    }
    dst[(size_t)y * a.W + x] = (uint8_t)v;
}

__global__ void __launch_bounds__(256) k_bm_fill(int16_t* disp, size_t n, int16_t v)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t pair = blockIdx.y;
    if (i < n) disp[pair * n + i] = v;
}

struct BmArgs {
    const uint8_t* Lp;
    const uint8_t* Rp;  // prefiltered [pair][H][W]
    int16_t* disp;      // [pair][H][W]
    int* cost;          // [pair][H][W] minimum SAD (validateDisparity)
    int H, W, ndisp, mind0, lofs, rofs, SW2, cap, tex_thresh, uniq;
    int xs, xe, y0, y1;  // computed region: relative columns [xs, xe), rows [y0, y1)
    int SWs, band;       // strip width, rows per band
    int FILTERED;
};

__global__ void __launch_bounds__(256) k_bm_sad(BmArgs a)
{
    extern __shared__ int bsm[];
    const int ndisp = a.ndisp, SW2 = a.SW2, W = a.W;
    const int xa = a.xs + blockIdx.x * a.SWs, ya = a.y0 + blockIdx.y * a.band, pair = blockIdx.z;
    if (xa >= a.xe || ya >= a.y1) return;  // block-uniform
    const int nx = min(a.SWs, a.xe - xa), yb = min(ya + a.band, a.y1);
    const int NC = nx + 2 * SW2;
    int* vsum = bsm;                      // [NC][ndisp]
    int* sad = vsum + NC * ndisp;         // [SWs][ndisp]
    int* vtex = sad + a.SWs * ndisp;      // [NC]
    int* tsum = vtex + NC;                // [SWs]
    const uint8_t* Lp = a.Lp + (size_t)pair * a.H * W;
    const uint8_t* Rp = a.Rp + (size_t)pair * a.H * W;
    const int tid = threadIdx.x;
    auto lcol = [&](int c) { return min(max(xa - SW2 + c + a.lofs, 0), W - 1); };
    auto rcol = [&](int c) { return min(max(xa - SW2 + c + a.rofs, 0), W - ndisp); };
    const int total = NC * ndisp;
    // window sums of the band's first row
    for (int i = tid; i < total; i += 256) {
        const int c = i / ndisp, d = i - c * ndisp;
        const int lc = lcol(c), rc = rcol(c) + d;
        int s = 0;
        for (int r = ya - SW2; r <= ya + SW2; r++) s += abs((int)Lp[(size_t)r * W + lc] - (int)Rp[(size_t)r * W + rc]);
        vsum[i] = s;
    }
    for (int c = tid; c < NC; c += 256) {
        const int lc = lcol(c);
        int s = 0;
        for (int r = ya - SW2; r <= ya + SW2; r++) s += abs((int)Lp[(size_t)r * W + lc] - a.cap);
        vtex[c] = s;
    }
    const int ng = max(1, 256 / ndisp);           // thread groups sharing a disparity's sliding sum
    const int xper = (nx + ng - 1) / ng;
    const int TP = 256 / a.SWs;                   // lanes per pixel in the WTA
    // the entering / leaving rows of both views, staged in LDS per step
    uint8_t* lrow = reinterpret_cast<uint8_t*>(tsum + a.SWs);  // [2][NC]
    uint8_t* rrow = lrow + 2 * NC;                              // [2][RN]
    const int rb0 = rcol(0), RN = rcol(NC - 1) + ndisp - rb0;
    for (int y = ya; y < yb; y++) {
        if (y > ya) {
            const size_t ra = (size_t)(y + SW2) * W, rs = (size_t)(y - SW2 - 1) * W;
            for (int i = tid; i < 2 * NC; i += 256) {
                const int c = i % NC;
                lrow[i] = Lp[(i < NC ? ra : rs) + lcol(c)];
            }
            for (int i = tid; i < 2 * RN; i += 256) {
                const int k = i % RN;
                rrow[i] = Rp[(i < RN ? ra : rs) + rb0 + k];
            }
            __syncthreads();
            // (c, d) of item i = tid + 256k, advanced without a division per item
            int c = tid / ndisp, d = tid - (tid / ndisp) * ndisp;
            const int cstep = 256 / ndisp, dstep = 256 - cstep * ndisp;
            for (int i = tid; i < total; i += 256) {
                const int rk = rcol(c) - rb0 + d;
                vsum[i] += abs((int)lrow[c] - (int)rrow[rk]) - abs((int)lrow[NC + c] - (int)rrow[RN + rk]);
                c += cstep;
                d += dstep;
                if (d >= ndisp) {
                    d -= ndisp;
                    c++;
                }
            }
            for (int c = tid; c < NC; c += 256) vtex[c] += abs((int)lrow[c] - a.cap) - abs((int)lrow[NC + c] - a.cap);
        }
        __syncthreads();
        // horizontal sliding sums: SAD[x][d] = sum_{c = x .. x+2*SW2} vsum[c][d]
        if (tid < ng * ndisp) {
            const int d = tid % ndisp, g = tid / ndisp;
            const int xb0 = g * xper, xb1 = min(nx, xb0 + xper);
            if (xb0 < xb1) {
                int s = 0;
                for (int c = xb0; c <= xb0 + 2 * SW2; c++) s += vsum[c * ndisp + d];
                sad[xb0 * ndisp + d] = s;
                for (int x = xb0 + 1; x < xb1; x++) {
                    s += vsum[(x + 2 * SW2) * ndisp + d] - vsum[(x - 1) * ndisp + d];
                    sad[x * ndisp + d] = s;
                }
            }
        }
        for (int x = tid; x < nx; x += 256) {
            int s = 0;
            for (int c = x; c <= x + 2 * SW2; c++) s += vtex[c];
            tsum[x] = s;
        }
        __syncthreads();
        // WTA: TP consecutive lanes per pixel
        {
            const int x = tid / TP, q = tid % TP;
            const int* sx = sad + x * ndisp;
            unsigned key = 0xFFFFFFFFu;
            if (x < nx)
                for (int d = q; d < ndisp; d += TP) key = min(key, ((unsigned)sx[d] << 9) | (unsigned)d);
            for (int o = TP / 2; o > 0; o >>= 1) key = min(key, (unsigned)__shfl_xor((int)key, o));
            const int mind = (int)(key & 511), minsad = (int)(key >> 9);
            bool bad = false;
            if (x < nx && a.uniq > 0) {
                const int thresh = minsad + (minsad * a.uniq / 100);
                for (int d = q; d < ndisp; d += TP) bad |= (d < mind - 1 || d > mind + 1) && sx[d] <= thresh;
            }
            for (int o = TP / 2; o > 0; o >>= 1) bad |= __shfl_xor((int)bad, o) != 0;
            if (x < nx && q == 0) {
                const int X = xa + x + a.lofs;
                const size_t o = (size_t)pair * a.H * W + (size_t)y * W + X;
                int v = a.FILTERED;
                int c = 0;
                if (tsum[x] >= a.tex_thresh && !bad) {
                    const int p = mind + 1 < ndisp ? sx[mind + 1] : sx[ndisp - 2];
                    const int n = mind - 1 >= 0 ? sx[mind - 1] : sx[1];
                    const int den = p + n - 2 * minsad + abs(p - n);
                    v = ((ndisp - mind - 1 + a.mind0) * 256 + (den != 0 ? (p - n) * 256 / den : 0) + 15) >> 4;
                    c = minsad;
                }
                a.disp[o] = (int16_t)v;
                a.cost[o] = c;
            }
        }
        __syncthreads();
    }
}

struct BmValidateArgs {
    int16_t* disp;
    const int* cost;
    int H, W, minD, ndisp, maxdiff16;
};

// cv::validateDisparity, one block per (row, pair).  disp2 via LDS atomicMin
// on (cost, x) keys — OpenCV keeps the first x (ascending) with the strictly
// smallest cost — then the decisions of the whole row, then the writes (the
// reads of pass 2 must see pass-1 values, as OpenCV's separate disp2buf).
__global__ void __launch_bounds__(256) k_bm_validate(BmValidateArgs a)
{
    extern __shared__ unsigned long long vsm[];
    unsigned long long* key2 = vsm;                                   // [W]
    int* d2v = reinterpret_cast<int*>(vsm + a.W);                     // [W]
    uint8_t* kill = reinterpret_cast<uint8_t*>(d2v + a.W);            // [W]
    const int y = blockIdx.x, pair = blockIdx.y, W = a.W;
    int16_t* row = a.disp + ((size_t)pair * a.H + y) * W;
    const int* crow = a.cost + ((size_t)pair * a.H + y) * W;
    const int INV = (a.minD - 1) * 16;
    const int maxD = a.minD + a.ndisp;
    const int minX1 = max(maxD, 0), maxX1 = W + min(a.minD, 0);
    for (int x = threadIdx.x; x < W; x += 256) {
        key2[x] = ~0ull;
        kill[x] = 0;
    }
    __syncthreads();
    for (int x = minX1 + (int)threadIdx.x; x < maxX1; x += 256) {
        const int d = row[x];
        if (d == INV) continue;
        const int x2 = x - ((d + 8) >> 4);
        if (x2 < 0 || x2 >= W) continue;
        atomicMin(&key2[x2], ((unsigned long long)(unsigned)crow[x] << 32) | (unsigned)x);
    }
    __syncthreads();
    for (int x = threadIdx.x; x < W; x += 256) {
        const unsigned long long k = key2[x];
        d2v[x] = k == ~0ull ? INV : (int)row[(int)(k & 0xFFFFFFFFu)];
    }
    __syncthreads();
    for (int x = minX1 + (int)threadIdx.x; x < maxX1; x += 256) {
        const int d = row[x];
        if (d == INV) continue;
        const int xa = x - (d >> 4), xb = x - ((d + 15) >> 4);
        const bool ra = xa >= 0 && xa < W && d2v[xa] > INV && abs(d2v[xa] - d) > a.maxdiff16;
        const bool rb = xb >= 0 && xb < W && d2v[xb] > INV && abs(d2v[xb] - d) > a.maxdiff16;
        kill[x] = ra && rb;
    }
    __syncthreads();
    for (int x = minX1 + (int)threadIdx.x; x < maxX1; x += 256)
        if (kill[x]) row[x] = (int16_t)INV;
}

}  // namespace smk
