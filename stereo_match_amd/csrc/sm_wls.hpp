// sm_wls.hpp — WLS disparity post-filter (ximgproc DisparityWLSFilter +
// FastGlobalSmootherFilter) for gfx950.  SURVEY §8 f1; reference call:
// stereo_vision/stereo_vision.py:172-182.  Semantics: oracle/wls_np.py.
//
// Per launch group of G pairs:
//   k_wls_conf  one workgroup per (ROI row, pair): depth-discontinuity
//               confidence of the right row into LDS, then the left ROI row:
//               its own confidence, the discontinuity-aware LR check, x255,
//               and the two FGS right-hand sides num = conf*disp, den = conf.
//   k_fgs_rows  one lane per (ROI row, pair): Thomas solve along x for both
//               right-hand sides (they share the elimination factors).
//   k_fgs_cols  one lane per (ROI column, pair): the same along y
//               (coalesced: neighbouring lanes = neighbouring columns).
//   k_wls_final num/den (0 where den == 0), round-half-even, saturate int16,
//               fill 16*(min_disp-1) outside the ROI.
// Everything is float32 in the oracle's operation order with FP contraction
// off, so results are bit-identical to oracle/wls_np.py.  The sequential
// solves are latency-bound (one dependent divide per element); their
// parallelism is rows x pairs, which is why they run on whole launch groups.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smk {

struct WlsConfArgs {
    const int16_t* dl;  // [pair][H][W]
    const int16_t* dr;
    size_t disp_pair;  // elements between pairs
    float* num;        // [pair][h][w]
    float* den;
    size_t roi_pair;  // elements between pairs (h*w)
    int H, W;
    int x0, y0, w, h;  // left ROI
    int rx0;           // right ROI x (same y0, w, h)
    int radius, lrc_thresh;
    float roll_off;
    int use_confidence;
};

__device__ inline int reflect101(int i, int n)
{
    if (n == 1) return 0;
    if (i < 0) i = -i;
    if (i >= n) i = 2 * n - 2 - i;
    return i;
}

// max(1 - roll_off * (E[d^2] - E[d]^2), 0) over the (2r+1)^2 window at (y, x)
__device__ inline float discontinuity_conf(const int16_t* __restrict__ d, int H, int W, int y, int x, int r,
                                           double scale, float roll_off)
{
#pragma clang fp contract(off)
    int s = 0;
    long long s2 = 0;
    for (int dy = -r; dy <= r; dy++) {
        const int16_t* row = d + (size_t)reflect101(y + dy, H) * W;
        for (int dx = -r; dx <= r; dx++) {
            const int v = row[reflect101(x + dx, W)];
            s += v;
            s2 += (long long)v * v;
        }
    }
    const float m = (float)((double)s * scale);
    const float m2 = (float)((double)s2 * scale);
    const float var = m2 - m * m;
    const float c = 1.0f - roll_off * var;
    return c > 0.0f ? c : 0.0f;
}

__global__ void __launch_bounds__(256) k_wls_conf(WlsConfArgs a)
{
#pragma clang fp contract(off)
    extern __shared__ float confr[];  // right-view confidence of this row, [W]
    const int yr = blockIdx.x, pair = blockIdx.y;
    const int y = a.y0 + yr;
    const int16_t* dl = a.dl + pair * a.disp_pair;
    const int16_t* dr = a.dr + pair * a.disp_pair;
    float* num = a.num + pair * a.roi_pair + (size_t)yr * a.w;
    float* den = a.den + pair * a.roi_pair + (size_t)yr * a.w;
    const int16_t* dlrow = dl + (size_t)y * a.W;
    if (!a.use_confidence) {
        for (int j = threadIdx.x; j < a.w; j += 256) num[j] = (float)dlrow[a.x0 + j];
        return;
    }
    const double scale = 1.0 / (double)((2 * a.radius + 1) * (2 * a.radius + 1));
    for (int j = threadIdx.x; j < a.w; j += 256)
        confr[j] = discontinuity_conf(dr, a.H, a.W, y, a.rx0 + j, a.radius, scale, a.roll_off);
    __syncthreads();
    const int16_t* drrow = dr + (size_t)y * a.W;
    for (int j = threadIdx.x; j < a.w; j += 256) {
        const int X = a.x0 + j;
        float c = discontinuity_conf(dl, a.H, a.W, y, X, a.radius, scale, a.roll_off);
        const int d = dlrow[X];
        const int ri = X - (d >> 4);
        if (ri >= a.rx0 && ri < a.rx0 + a.w) {
            const int sum = d + drrow[ri];
            c = (sum < a.lrc_thresh && -sum < a.lrc_thresh) ? fminf(c, confr[ri - a.rx0]) : 0.0f;
        }
        c = c * 255.0f;
        num[j] = c * (float)d;
        den[j] = c;
    }
}

struct FgsArgs {
    float* u[2];  // right-hand sides, [pair][h][w], solved in place
    float* inter;  // elimination factors, [pair][h][w]
    size_t roi_pair;
    const uint8_t* guide;  // [pair] gray left view; ROI origin already applied
    size_t guide_pair;
    int guide_stride;
    int w, h;
    float lam;
    float tab[256];  // -exp(-k / sigma), k = |delta guide|
};

// Thomas solve of (I + lam*L_w) u = f along one line of n samples.
// P(i) = element offset of sample i, G(i) = guide offset of sample i.
template <int NRHS>
__device__ inline void fgs_line(const FgsArgs& a, const float* tab, float* __restrict__ u0, float* __restrict__ u1,
                                float* __restrict__ inter, const uint8_t* __restrict__ g, size_t step, size_t gstep,
                                int n)
{
#pragma clang fp contract(off)
    const float lam = a.lam;
    auto C = [&](int i) -> float {
        if (i >= n - 1) return 0.0f;
        const int d = (int)g[(size_t)(i + 1) * gstep] - (int)g[(size_t)i * gstep];
        return tab[d < 0 ? -d : d];
    };
    float cp = C(0);
    float denom = 1.0f - lam * cp;
    float ip = (lam * cp) / denom;
    inter[0] = ip;
    float p0 = u0[0] / denom, p1 = 0.f;
    u0[0] = p0;
    if (NRHS == 2) {
        p1 = u1[0] / denom;
        u1[0] = p1;
    }
    for (int i = 1; i < n; i++) {
        const float cj = C(i);
        const float t = 1.0f - lam * (cp + cj);
        const float lcp = lam * cp;
        denom = t - lcp * ip;
        ip = (lam * cj) / denom;
        inter[(size_t)i * step] = ip;
        p0 = (u0[(size_t)i * step] - lcp * p0) / denom;
        u0[(size_t)i * step] = p0;
        if (NRHS == 2) {
            p1 = (u1[(size_t)i * step] - lcp * p1) / denom;
            u1[(size_t)i * step] = p1;
        }
        cp = cj;
    }
    for (int i = n - 2; i >= 0; i--) {
        const float f = inter[(size_t)i * step];
        p0 = u0[(size_t)i * step] - f * p0;
        u0[(size_t)i * step] = p0;
        if (NRHS == 2) {
            p1 = u1[(size_t)i * step] - f * p1;
            u1[(size_t)i * step] = p1;
        }
    }
}

// ROWS: one lane per ROI row (solve along x); else one lane per ROI column.
template <int NRHS, bool ROWS>
__global__ void __launch_bounds__(64) k_fgs(FgsArgs a)
{
    __shared__ float tab[256];
    for (int i = threadIdx.x; i < 256; i += 64) tab[i] = a.tab[i];
    __syncthreads();
    const int line = blockIdx.x * 64 + threadIdx.x, pair = blockIdx.y;
    if (line >= (ROWS ? a.h : a.w)) return;
    const size_t base = pair * a.roi_pair + (ROWS ? (size_t)line * a.w : (size_t)line);
    const uint8_t* g = a.guide + pair * a.guide_pair + (ROWS ? (size_t)line * a.guide_stride : (size_t)line);
    const size_t step = ROWS ? 1 : (size_t)a.w;
    const size_t gstep = ROWS ? 1 : (size_t)a.guide_stride;
    fgs_line<NRHS>(a, tab, a.u[0] + base, NRHS == 2 ? a.u[1] + base : nullptr, a.inter + base, g, step, gstep,
                   ROWS ? a.w : a.h);
}

struct WlsFinalArgs {
    const float* num;
    const float* den;
    size_t roi_pair;
    int16_t* out;  // [pair][H][W]
    size_t out_pair;
    int H, W, x0, y0, w, h;
    int fill;  // 16*(min_disp-1)
    int use_confidence;
};

__global__ void __launch_bounds__(256) k_wls_final(WlsFinalArgs a)
{
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, pair = blockIdx.z;
    if (x >= a.W) return;
    int v = a.fill;
    const int j = x - a.x0, i = y - a.y0;
    if (j >= 0 && j < a.w && i >= 0 && i < a.h) {
        const size_t o = pair * a.roi_pair + (size_t)i * a.w + j;
        float q = a.num[o];
        if (a.use_confidence) {
            const float dd = a.den[o];
            q = dd != 0.0f ? q / dd : 0.0f;
        }
        float r = __builtin_rintf(q);
        r = r < -32768.0f ? -32768.0f : (r > 32767.0f ? 32767.0f : r);
        v = (q != q) ? 0 : (int)r;
    }
    a.out[pair * a.out_pair + (size_t)y * a.W + x] = (int16_t)v;
}

}  // namespace smk
