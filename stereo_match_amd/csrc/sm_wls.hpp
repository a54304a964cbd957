// sm_wls.hpp — WLS disparity post-filter (ximgproc DisparityWLSFilter +
// FastGlobalSmootherFilter) for gfx950.  SURVEY §8 f1; reference call:
// stereo_vision/stereo_vision.py:172-182.  Semantics: oracle/wls_np.py.
//
// Per launch group of G pairs (ROI arrays padded to hp x wp, multiples of 64,
// so every 64x64 tile access below is in bounds and 16-byte aligned):
//   k_wls_conf  one workgroup per (padded ROI row, pair): depth-discontinuity
//               confidence of the right row into LDS, then the left ROI row:
//               its own confidence, the discontinuity-aware LR check, x255,
//               the two FGS right-hand sides num = conf*disp, den = conf, and
//               the smoother's edge weights Ch (to x+1) and Cv (to y+1) from
//               the guide.  Padding is written as zeros.
//   k_fgs<ROWS> 64 lines per one-wave workgroup, one line per lane: Thomas
//               solve along the line for both right-hand sides (they share
//               the elimination factors).  ROWS: lines = ROI rows; else
//               lines = ROI columns.
//   k_wls_final num/den (0 where den == 0), round-half-even, saturate int16,
//               fill 16*(min_disp-1) outside the ROI.
// Everything is float32 in the oracle's operation order with FP contraction
// off, so results are bit-identical to oracle/wls_np.py.  The solves are
// latency-bound (a dependent reciprocal per element); their parallelism is
// lines x pairs, which is why they run on whole launch groups and why the
// tile traffic is prefetched a chunk ahead.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sm_common.hpp"

namespace smk {

constexpr int FT = 64, FP = 65;  // tile edge, LDS pitch (conflict-free both ways)

struct WlsConfArgs {
    const int16_t* dl;  // [pair][H][W]
    const int16_t* dr;
    size_t disp_pair;  // elements between pairs
    const uint8_t* guide;
    size_t guide_pair;  // bytes between pairs
    int guide_stride;
    float* num;  // [pair][hp][wp]
    float* den;
    float* Ch;
    float* Cv;
    size_t roi_pair;  // hp*wp
    int H, W;
    int x0, y0, w, h, wp;  // left ROI, padded pitch
    int rx0;               // right ROI x (same y0, w, h)
    int radius, lrc_thresh;
    float roll_off;
    int use_confidence;
    int weights;     // 1: also write Ch / Cv (0: k_wls_weights wrote them)
    int separable;   // 1: box sums through LDS column sums (wls_conf_lds bytes of dynamic LDS)
    float tab[256];  // -exp(-k / sigma), k = |delta guide|
};

// The smoother's edge weights from the guide alone (the part of k_wls_conf that does not
// need the disparity maps, so compute_disparity can run it, and the pivots, beside the
// matchers).  One workgroup per padded ROI row and pair.
__global__ void __launch_bounds__(256) k_wls_weights(WlsConfArgs a)
{
#pragma clang fp contract(off)
    __shared__ float tab[256];
    tab[threadIdx.x] = a.tab[threadIdx.x];
    __syncthreads();
    const int yr = blockIdx.x, pair = blockIdx.y;
    const size_t ro = pair * a.roi_pair + (size_t)yr * a.wp;
    float* Ch = a.Ch + ro;
    float* Cv = a.Cv + ro;
    const uint8_t* g = a.guide + pair * a.guide_pair + (size_t)(a.y0 + yr) * a.guide_stride + a.x0;
    for (int j = threadIdx.x; j < a.wp; j += 256) {
        float ch = 0.f, cv = 0.f;
        if (yr < a.h && j < a.w) {
            const int g0 = g[j];
            if (j < a.w - 1) {
                const int d = (int)g[j + 1] - g0;
                ch = tab[d < 0 ? -d : d];
            }
            if (yr < a.h - 1) {
                const int d = (int)g[j + a.guide_stride] - g0;
                cv = tab[d < 0 ? -d : d];
            }
        }
        Ch[j] = ch;
        Cv[j] = cv;
    }
}

// cv::borderInterpolate(BORDER_REFLECT_101): reflect until inside (a window
// wider than the image reflects more than once)
__device__ inline int reflect101(int i, int n)
{
    if (n == 1) return 0;
    while ((unsigned)i >= (unsigned)n) i = i < 0 ? -i : 2 * n - 2 - i;
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

// discontinuity_conf for n consecutive columns xs.. of row y, separably: the column
// sums of the window's 2r+1 rows (reflect-101) for the n + 2r columns the windows
// touch, then 2r+1-wide horizontal sums of those (integer sums: the same values as
// discontinuity_conf's loop in any order).  Writes out[0..n) (LDS); cs / cs2 hold
// n + 2r column sums.  All threads of the workgroup take part (barriers inside).
__device__ inline void conf_row(const int16_t* __restrict__ d, int H, int W, int y, int xs, int n, int r, double scale,
                                float roll_off, float* out, int* cs, long long* cs2)
{
#pragma clang fp contract(off)
    const int m = n + 2 * r;
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const int x = reflect101(xs - r + i, W);
        int s = 0;
        long long s2 = 0;
        for (int dy = -r; dy <= r; dy++) {
            const int v = d[(size_t)reflect101(y + dy, H) * W + x];
            s += v;
            s2 += (long long)v * v;
        }
        cs[i] = s;
        cs2[i] = s2;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
        int s = 0;
        long long s2 = 0;
        for (int k = 0; k <= 2 * r; k++) {
            s += cs[j + k];
            s2 += cs2[j + k];
        }
        const float mm = (float)((double)s * scale);
        const float m2 = (float)((double)s2 * scale);
        const float var = m2 - mm * mm;
        const float c = 1.0f - roll_off * var;
        out[j] = c > 0.0f ? c : 0.0f;
    }
    __syncthreads();
}

// dynamic LDS: tab[256], confr[w], confl[w], column sums cs[w + 2r] (int), cs2 (int64)
__host__ __device__ inline size_t wls_conf_lds(int w, int r)
{
    return ((size_t)(256 + 2 * w) * 4 + 7) / 8 * 8 + (size_t)(w + 2 * r) * 12 + 16;
}

__global__ void __launch_bounds__(256) k_wls_conf(WlsConfArgs a)
{
#pragma clang fp contract(off)
    extern __shared__ uint32_t smem[];  // tab[256], right / left confidence of this row [w], column sums
    float* tab = reinterpret_cast<float*>(smem);
    float* confr = tab + 256;
    float* confl = confr + a.w;
    long long* cs2 = reinterpret_cast<long long*>(smem + ((256 + 2 * a.w) + 1) / 2 * 2);
    int* cs = reinterpret_cast<int*>(cs2 + (a.w + 2 * a.radius));
    for (int i = threadIdx.x; i < 256; i += 256) tab[i] = a.tab[i];
    const int yr = blockIdx.x, pair = blockIdx.y;
    const size_t ro = pair * a.roi_pair + (size_t)yr * a.wp;
    float* num = a.num + ro;
    float* den = a.den + ro;
    float* Ch = a.Ch + ro;
    float* Cv = a.Cv + ro;
    if (yr >= a.h) {  // padding row
        for (int j = threadIdx.x; j < a.wp; j += 256) {
            num[j] = den[j] = 0.f;
            if (a.weights) Ch[j] = Cv[j] = 0.f;
        }
        return;
    }
    const int y = a.y0 + yr;
    const int16_t* dl = a.dl + pair * a.disp_pair;
    const int16_t* dr = a.dr + pair * a.disp_pair;
    const uint8_t* g = a.guide + pair * a.guide_pair + (size_t)y * a.guide_stride + a.x0;
    const int16_t* dlrow = dl + (size_t)y * a.W;
    __syncthreads();
    if (a.weights) {  // smoother weights (skipped when k_wls_weights computed them ahead)
        for (int j = threadIdx.x; j < a.wp; j += 256) {
            float ch = 0.f, cv = 0.f;
            if (j < a.w) {
                const int g0 = g[j];
                if (j < a.w - 1) {
                    const int d = (int)g[j + 1] - g0;
                    ch = tab[d < 0 ? -d : d];
                }
                if (yr < a.h - 1) {
                    const int d = (int)g[j + a.guide_stride] - g0;
                    cv = tab[d < 0 ? -d : d];
                }
            }
            Ch[j] = ch;
            Cv[j] = cv;
        }
    }
    if (!a.use_confidence) {
        for (int j = threadIdx.x; j < a.wp; j += 256) num[j] = j < a.w ? (float)dlrow[a.x0 + j] : 0.f;
        return;
    }
    const double scale = 1.0 / (double)((2 * a.radius + 1) * (2 * a.radius + 1));
    if (a.separable) {
        conf_row(dr, a.H, a.W, y, a.rx0, a.w, a.radius, scale, a.roll_off, confr, cs, cs2);
        conf_row(dl, a.H, a.W, y, a.x0, a.w, a.radius, scale, a.roll_off, confl, cs, cs2);
    } else {  // rows too wide for the column sums in LDS: per pixel (tab + confr only)
        for (int j = threadIdx.x; j < a.w; j += 256)
            confr[j] = discontinuity_conf(dr, a.H, a.W, y, a.rx0 + j, a.radius, scale, a.roll_off);
        __syncthreads();
    }
    const int16_t* drrow = dr + (size_t)y * a.W;
    for (int j = threadIdx.x; j < a.wp; j += 256) {
        if (j >= a.w) {
            num[j] = den[j] = 0.f;
            continue;
        }
        const int X = a.x0 + j;
        float c = a.separable ? confl[j] : discontinuity_conf(dl, a.H, a.W, y, X, a.radius, scale, a.roll_off);
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
    float* u[2];  // right-hand sides, [pair][hp][wp], solved in place
    float* inter;  // elimination factors, [pair][hp][wp]
    const float* C;  // edge weights along the solve direction (Ch or Cv)
    size_t roi_pair;
    int w, h, wp;
    float lam;
    int dbg;  // timing ablations (sm_api.hip DBG_FGS_*): 1 skip the sweeps, 2 skip global loads/stores
};

// Thomas solve of (I + lam*L_w) u = f along lines, 64 lines per workgroup
// (one wave, one line per lane):
//   forward   r = 1/(1 - lam(C[j-1]+C[j]) - lam C[j-1] c'[j-1]),
//             c'[j] = lam C[j] r,  d'[j] = (f[j] - lam C[j-1] d'[j-1]) r
//   backward  x[j] = d'[j] - c'[j] x[j+1]
// The recurrence is serial along a line, so lines are staged through LDS in
// 64x64 tiles.  Tile traffic uses float4 accesses on the padded arrays
// (ROWS: 16 lanes cover one line's 64 positions; columns: 16 lanes cover 64
// lines of one position), and the next chunk's tiles are loaded into
// registers while the current chunk is swept, so the per-chunk memory latency
// hides behind the dependent reciprocal chain.  Zero-initialised carries
// reproduce the oracle's first-element formulas exactly (x - 0*0 == x).
// 1/t for the Thomas pivots t in [1, 2^24): v_rcp_f32 plus one FMA Newton step is the
// correctly rounded reciprocal there (tools/ubench/rcp_exact.hip checks every float of
// [1, 2^24) against IEEE 1.0f / t: 0 mismatches), 3 dependent operations instead of the
// 10 of the IEEE division sequence.  The pivots of (I + lam L_w) are >= 1 (diagonally
// dominant, weights in [-1, 0]) and <= 1 + 2 lam; the host enables this only when
// 1 + 2 lam < 2^24 for every iteration (sm_api.hip run_wls).
template <bool FAST>
__device__ __forceinline__ float pivot_rcp(float t)
{
#pragma clang fp contract(off)
    if constexpr (FAST) {
        const float y = __builtin_amdgcn_rcpf(t);
        return __builtin_fmaf(__builtin_fmaf(-t, y, 1.0f), y, y);
    } else {
        return 1.0f / t;
    }
}

template <bool ROWS>
struct TileMap {
    // load k (0..15) of lane -> local (line, pos) of the float4's first element;
    // the float4 runs along pos (ROWS) or along line (columns)
    __device__ static void at(int k, int lane, int& ll, int& pl)
    {
        if (ROWS) {
            ll = 4 * k + (lane >> 4);
            pl = (lane & 15) * 4;
        } else {
            pl = 4 * k + (lane >> 4);
            ll = (lane & 15) * 4;
        }
    }
    __device__ static int tix(int ll, int pl) { return ROWS ? ll * FP + pl : pl * FP + ll; }
    __device__ static int tix_e(int ll, int pl, int e) { return ROWS ? tix(ll, pl + e) : tix(ll + e, pl); }
    __device__ static size_t eoff(int line, int pos, int wp)
    {
        return ROWS ? (size_t)line * wp + pos : (size_t)pos * wp + line;
    }
};

// Tile I/O through raw buffer ops: the per-lane byte offset of load k = 0 is
// in a VGPR; load k adds k*16*wp bytes (4 lines for ROWS, 4 positions for
// columns — the same stride) as a scalar offset, so the 16 accesses of a
// tile cost no extra address registers.
template <bool ROWS>
__device__ inline uint32_t tile_voff(int l0, int j0, int wp, int lane)
{
    int ll, pl;
    TileMap<ROWS>::at(0, lane, ll, pl);
    return (uint32_t)(TileMap<ROWS>::eoff(l0 + ll, j0 + pl, wp) * 4);
}

template <bool ROWS>
__device__ inline void tile_load(float4 (&r)[16], rsrc_t rs, uint32_t voff, int wp)
{
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, k * 16 * wp, 0);
        r[k] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
    }
}

template <bool ROWS>
__device__ inline void tile_to_lds(const float4 (&r)[16], float* T, int lane)
{
#pragma unroll
    for (int k = 0; k < 16; k++) {
        int ll, pl;
        TileMap<ROWS>::at(k, lane, ll, pl);
        T[TileMap<ROWS>::tix_e(ll, pl, 0)] = r[k].x;
        T[TileMap<ROWS>::tix_e(ll, pl, 1)] = r[k].y;
        T[TileMap<ROWS>::tix_e(ll, pl, 2)] = r[k].z;
        T[TileMap<ROWS>::tix_e(ll, pl, 3)] = r[k].w;
    }
}

template <bool ROWS>
__device__ inline void tile_store(rsrc_t rs, uint32_t voff, const float* T, int wp, int lane)
{
#pragma unroll
    for (int k = 0; k < 16; k++) {
        int ll, pl;
        TileMap<ROWS>::at(k, lane, ll, pl);
        u32x4 v;
        v[0] = __float_as_uint(T[TileMap<ROWS>::tix_e(ll, pl, 0)]);
        v[1] = __float_as_uint(T[TileMap<ROWS>::tix_e(ll, pl, 1)]);
        v[2] = __float_as_uint(T[TileMap<ROWS>::tix_e(ll, pl, 2)]);
        v[3] = __float_as_uint(T[TileMap<ROWS>::tix_e(ll, pl, 3)]);
        // the offset goes into the VGPR, soffset stays the literal 0: the compiler's hazard
        // recognizer treats a >64-bit MUBUF store with an SGPR soffset as free of the
        // store-data hazard and lets the next VALU overwrite the data VGPRs at once, which on
        // gfx950 under load stored those new values (addresses) instead of the tile
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff + (uint32_t)(k * 16 * wp), 0, 0);
    }
}

// The same tile I/O split over the waves of a workgroup: wave w moves the tile's loads
// k0 .. k0+NK-1 (k0 = NK*w, wave-uniform).
template <bool ROWS, int NK>
__device__ inline void tile_load_part(float4 (&r)[NK], rsrc_t rs, uint32_t voff, int wp, int k0)
{
#pragma unroll
    for (int k = 0; k < NK; k++) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, (k0 + k) * 16 * wp, 0);
        r[k] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
    }
}

template <bool ROWS, int NK>
__device__ inline void tile_to_lds_part(const float4 (&r)[NK], float* T, int lane, int k0)
{
#pragma unroll
    for (int k = 0; k < NK; k++) {
        int ll, pl;
        TileMap<ROWS>::at(k0 + k, lane, ll, pl);
        T[TileMap<ROWS>::tix_e(ll, pl, 0)] = r[k].x;
        T[TileMap<ROWS>::tix_e(ll, pl, 1)] = r[k].y;
        T[TileMap<ROWS>::tix_e(ll, pl, 2)] = r[k].z;
        T[TileMap<ROWS>::tix_e(ll, pl, 3)] = r[k].w;
    }
}

template <bool ROWS, int NK>
__device__ inline void tile_store_part(rsrc_t rs, uint32_t voff, const float* T, int wp, int lane, int k0)
{
#pragma unroll
    for (int k = 0; k < NK; k++) {
        int ll, pl;
        TileMap<ROWS>::at(k0 + k, lane, ll, pl);
        u32x4 v;
        v[0] = __float_as_uint(T[TileMap<ROWS>::tix_e(ll, pl, 0)]);
        v[1] = __float_as_uint(T[TileMap<ROWS>::tix_e(ll, pl, 1)]);
        v[2] = __float_as_uint(T[TileMap<ROWS>::tix_e(ll, pl, 2)]);
        v[3] = __float_as_uint(T[TileMap<ROWS>::tix_e(ll, pl, 3)]);
        // offset in the VGPR (see tile_store)
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff + (uint32_t)((k0 + k) * 16 * wp), 0, 0);
    }
}

template <int NRHS, bool ROWS, bool FAST = false>
__global__ void __launch_bounds__(64) k_fgs(FgsArgs a)
{
#pragma clang fp contract(off)
    __shared__ float Ct[FT * FP], U0[FT * FP], U1[NRHS == 2 ? FT * FP : 1], IT[FT * FP];
    const int lane = threadIdx.x, pair = blockIdx.y;
    const int n = ROWS ? a.w : a.h;
    const int l0 = blockIdx.x * FT, wp = a.wp;
    const uint64_t bytes = a.roi_pair * 4;
    const rsrc_t u0 = make_rsrc(a.u[0] + pair * a.roi_pair, bytes);
    const rsrc_t u1 = make_rsrc(a.u[NRHS == 2 ? 1 : 0] + pair * a.roi_pair, bytes);
    const rsrc_t inter = make_rsrc(a.inter + pair * a.roi_pair, bytes);
    const rsrc_t C = make_rsrc(a.C + pair * a.roi_pair, bytes);
    // byte offset of chunk c's first access: ROWS advance 64 positions (256 B),
    // columns advance 64 rows
    const uint32_t voff0 = tile_voff<ROWS>(l0, 0, wp, lane);
    const uint32_t cstep = ROWS ? FT * 4 : (uint32_t)FT * wp * 4;
    const bool mem = !(a.dbg & 2), sweep = !(a.dbg & 1);
    const float lam = a.lam;
    const int nchunks = (n + FT - 1) / FT;
    float4 rc[16], r0[16], r1[16];
    if (mem) {
        tile_load<ROWS>(rc, C, voff0, wp);
        tile_load<ROWS>(r0, u0, voff0, wp);
        if (NRHS == 2) tile_load<ROWS>(r1, u1, voff0, wp);
        tile_to_lds<ROWS>(rc, Ct, lane);
        tile_to_lds<ROWS>(r0, U0, lane);
        if (NRHS == 2) tile_to_lds<ROWS>(r1, U1, lane);
    }
    float ip = 0.f, p0 = 0.f, p1 = 0.f, cp = 0.f;
    for (int c = 0; c < nchunks; c++) {
        const int j0 = c * FT;
        const bool next = c + 1 < nchunks;
        __syncthreads();
        if (mem && next) {  // prefetch chunk c+1 (consumed after the sweep)
            const uint32_t vn = voff0 + (c + 1) * cstep;
            tile_load<ROWS>(rc, C, vn, wp);
            tile_load<ROWS>(r0, u0, vn, wp);
            if (NRHS == 2) tile_load<ROWS>(r1, u1, vn, wp);
        }
        const int m = sweep ? min(FT, n - j0) : 0;
        for (int jj = 0; jj < m; jj++) {
            const int t = TileMap<ROWS>::tix(lane, jj);
            const float cj = Ct[t];
            const float tt = 1.0f - lam * (cp + cj);
            const float lcp = lam * cp;
            const float r = pivot_rcp<FAST>(tt - lcp * ip);
            ip = (lam * cj) * r;
            IT[t] = ip;
            p0 = (U0[t] - lcp * p0) * r;
            U0[t] = p0;
            if (NRHS == 2) {
                p1 = (U1[t] - lcp * p1) * r;
                U1[t] = p1;
            }
            cp = cj;
        }
        __syncthreads();
        if (mem) {
            const uint32_t vc = voff0 + c * cstep;
            tile_store<ROWS>(u0, vc, U0, wp, lane);
            if (NRHS == 2) tile_store<ROWS>(u1, vc, U1, wp, lane);
            tile_store<ROWS>(inter, vc, IT, wp, lane);
            if (next) {
                __syncthreads();
                tile_to_lds<ROWS>(rc, Ct, lane);
                tile_to_lds<ROWS>(r0, U0, lane);
                if (NRHS == 2) tile_to_lds<ROWS>(r1, U1, lane);
            }
        }
    }
    // backward substitution; the last chunk's d' and c' are still in LDS
    for (int c = nchunks - 1; c >= 0; c--) {
        const int j0 = c * FT;
        const bool prev = c > 0;
        __syncthreads();
        if (mem && prev) {
            const uint32_t vp = voff0 + (c - 1) * cstep;
            tile_load<ROWS>(rc, inter, vp, wp);
            tile_load<ROWS>(r0, u0, vp, wp);
            if (NRHS == 2) tile_load<ROWS>(r1, u1, vp, wp);
        }
        const int m = sweep ? min(FT, n - j0) : 0;
        for (int jj = m - 1; jj >= 0; jj--) {
            const int t = TileMap<ROWS>::tix(lane, jj);
            if (c == nchunks - 1 && jj == m - 1) {  // x[n-1] = d'[n-1]
                p0 = U0[t];
                if (NRHS == 2) p1 = U1[t];
                continue;
            }
            const float f = IT[t];
            p0 = U0[t] - f * p0;
            U0[t] = p0;
            if (NRHS == 2) {
                p1 = U1[t] - f * p1;
                U1[t] = p1;
            }
        }
        __syncthreads();
        if (mem) {
            const uint32_t vc = voff0 + c * cstep;
            tile_store<ROWS>(u0, vc, U0, wp, lane);
            if (NRHS == 2) tile_store<ROWS>(u1, vc, U1, wp, lane);
            if (prev) {
                __syncthreads();
                tile_to_lds<ROWS>(rc, IT, lane);
                tile_to_lds<ROWS>(r0, U0, lane);
                if (NRHS == 2) tile_to_lds<ROWS>(r1, U1, lane);
            }
        }
    }
}

// ---- the Thomas pivots on their own (round 3).  The elimination factors of
// (I + lam L_w) depend only on the weights C and lam, not on the right-hand sides:
//   r[j] = 1/(1 - lam(C[j-1]+C[j]) - lam C[j-1] c'[j-1]),  c'[j] = (lam C[j]) r[j]
// k_fgs_pivots runs that chain (6 dependent operations per element) for every
// iteration's lam at once and stores r and c'; k_fgs_solve then carries only the
// right-hand sides (forward (f - lam C[j-1] d') r: 3 dependent operations; backward
// d' - c' x: 2).  Same float32 operations in the same order as k_fgs / oracle/wls_np.py.
struct FgsPivotArgs {
    const float* C;     // Ch (ROWS) or Cv, [pair][hp][wp]
    float* R;           // [it][pair][hp][wp] pivot reciprocals
    float* IT;          // [it][pair][hp][wp] elimination factors c'
    size_t roi_pair, var_stride;  // elements per pair, per iteration (= npairs * roi_pair)
    int w, h, wp;
    float lam[8];       // lam of each iteration (lam0 * att^it, float32 as the host iterates)
};

template <bool ROWS, bool FAST>
__global__ void __launch_bounds__(64) k_fgs_pivots(FgsPivotArgs a)
{
#pragma clang fp contract(off)
    __shared__ float Ct[FT * FP], RT[FT * FP], IT[FT * FP];
    const int lane = threadIdx.x, it = blockIdx.y, pair = blockIdx.z;
    const int n = ROWS ? a.w : a.h;
    const int l0 = blockIdx.x * FT, wp = a.wp;
    const uint64_t bytes = a.roi_pair * 4;
    const rsrc_t C = make_rsrc(a.C + pair * a.roi_pair, bytes);
    const size_t vo = (size_t)it * a.var_stride + pair * a.roi_pair;
    const rsrc_t R = make_rsrc(a.R + vo, bytes);
    const rsrc_t I = make_rsrc(a.IT + vo, bytes);
    const uint32_t voff0 = tile_voff<ROWS>(l0, 0, wp, lane);
    const uint32_t cstep = ROWS ? FT * 4 : (uint32_t)FT * wp * 4;
    const float lam = a.lam[it];
    const int nchunks = (n + FT - 1) / FT;
    float4 rc[16];
    tile_load<ROWS>(rc, C, voff0, wp);
    tile_to_lds<ROWS>(rc, Ct, lane);
    float ip = 0.f, cp = 0.f;
    for (int c = 0; c < nchunks; c++) {
        const int j0 = c * FT;
        const bool next = c + 1 < nchunks;
        __syncthreads();
        if (next) tile_load<ROWS>(rc, C, voff0 + (c + 1) * cstep, wp);
        const int m = min(FT, n - j0);
#pragma unroll 4
        for (int jj = 0; jj < m; jj++) {
            const int t = TileMap<ROWS>::tix(lane, jj);
            const float cj = Ct[t];
            const float tt = 1.0f - lam * (cp + cj);
            const float lcp = lam * cp;
            const float r = pivot_rcp<FAST>(tt - lcp * ip);
            ip = (lam * cj) * r;
            RT[t] = r;
            IT[t] = ip;
            cp = cj;
        }
        __syncthreads();
        const uint32_t vc = voff0 + c * cstep;
        tile_store<ROWS>(R, vc, RT, wp, lane);
        tile_store<ROWS>(I, vc, IT, wp, lane);
        if (next) {
            __syncthreads();
            tile_to_lds<ROWS>(rc, Ct, lane);
        }
    }
}

struct FgsSolveArgs {
    float* u[2];        // right-hand sides, [pair][hp][wp], solved in place
    const float* C;     // edge weights along the solve direction (Ch or Cv)
    const float* R;     // this iteration's pivot reciprocals [pair][hp][wp]
    const float* IT;    // this iteration's elimination factors
    size_t roi_pair;
    int w, h, wp;
    float lam;
};

// One full 64-step chunk of a line's forward (d' = (f - lam c'[j-1] d'[j-1]) r) or backward
// (x = d' - c' x[j+1]) sweep, the same float32 operations in the same order as the generic
// loops below.  The chunk runs in register sub-blocks of FGS_SB steps whose LDS operands are
// read before the previous sub-block's results are written back: the compiler cannot prove
// that U0[t'] (next step) and U0[t] (this step) differ, so the plain loop waited for each
// read after the preceding write (an LDS round trip per step on the dependent chain:
// ~180 cycles per step on the KITTI row pass).
#ifndef FGS_SB
#define FGS_SB 16
#endif
#ifndef FGS_NOCOMPUTE
#define FGS_NOCOMPUTE 0
#endif
// materialise a loaded value at this point of the program (the read cannot sink below it)
__device__ __forceinline__ void fgs_pin(float& x) { asm volatile("" : "+v"(x)); }
template <int NRHS, bool ROWS, class M = TileMap<ROWS>>
__device__ __forceinline__ void fgs_fwd_chunk(const float* RT, float* U0, float* U1, const float* Ct, int lane,
                                              float lam, float& p0, float& p1, float& cp)
{
#pragma clang fp contract(off)
    constexpr int SB = FGS_SB, NSB = FT / SB;
    float r[2][SB], u0[2][SB], u1[2][NRHS == 2 ? SB : 1], cc[2][SB];
#pragma unroll
    for (int k = 0; k < SB; k++) {
        const int t = M::tix(lane, k);
        r[0][k] = RT[t];
        u0[0][k] = U0[t];
        if (NRHS == 2) u1[0][k] = U1[t];
        cc[0][k] = Ct[t];
    }
#pragma unroll
    for (int k = 0; k < SB; k++) {
        fgs_pin(r[0][k]);
        fgs_pin(u0[0][k]);
        if (NRHS == 2) fgs_pin(u1[0][k]);
        fgs_pin(cc[0][k]);
    }
#pragma unroll
    for (int b = 0; b < NSB; b++) {
        const int cur = b & 1, nxt = cur ^ 1;
        if (b + 1 < NSB) {
#pragma unroll
            for (int k = 0; k < SB; k++) {
                const int t = M::tix(lane, (b + 1) * SB + k);
                r[nxt][k] = RT[t];
                u0[nxt][k] = U0[t];
                if (NRHS == 2) u1[nxt][k] = U1[t];
                cc[nxt][k] = Ct[t];
            }
        }
#pragma unroll
        for (int k = 0; k < SB; k++) {
            const float lcp = lam * cp;
            p0 = (u0[cur][k] - lcp * p0) * r[cur][k];
            u0[cur][k] = p0;
            if (NRHS == 2) {
                p1 = (u1[cur][k] - lcp * p1) * r[cur][k];
                u1[cur][k] = p1;
            }
            cp = cc[cur][k];
        }
        if (b + 1 < NSB) {  // the next sub-block's reads complete here, not inside the chain
#pragma unroll
            for (int k = 0; k < SB; k++) {
                fgs_pin(r[nxt][k]);
                fgs_pin(u0[nxt][k]);
                if (NRHS == 2) fgs_pin(u1[nxt][k]);
                fgs_pin(cc[nxt][k]);
            }
        }
#pragma unroll
        for (int k = 0; k < SB; k++) {
            const int t = M::tix(lane, b * SB + k);
            U0[t] = u0[cur][k];
            if (NRHS == 2) U1[t] = u1[cur][k];
        }
    }
}

// backward over a full chunk, positions 63 .. 0 (RT holds c')
template <int NRHS, bool ROWS, class M = TileMap<ROWS>>
__device__ __forceinline__ void fgs_bwd_chunk(const float* RT, float* U0, float* U1, int lane, float& p0, float& p1)
{
#pragma clang fp contract(off)
    constexpr int SB = FGS_SB, NSB = FT / SB;
    float f[2][SB], u0[2][SB], u1[2][NRHS == 2 ? SB : 1];
#pragma unroll
    for (int k = 0; k < SB; k++) {
        const int t = M::tix(lane, FT - 1 - k);
        f[0][k] = RT[t];
        u0[0][k] = U0[t];
        if (NRHS == 2) u1[0][k] = U1[t];
    }
#pragma unroll
    for (int k = 0; k < SB; k++) {
        fgs_pin(f[0][k]);
        fgs_pin(u0[0][k]);
        if (NRHS == 2) fgs_pin(u1[0][k]);
    }
#pragma unroll
    for (int b = 0; b < NSB; b++) {
        const int cur = b & 1, nxt = cur ^ 1;
        if (b + 1 < NSB) {
#pragma unroll
            for (int k = 0; k < SB; k++) {
                const int t = M::tix(lane, FT - 1 - (b + 1) * SB - k);
                f[nxt][k] = RT[t];
                u0[nxt][k] = U0[t];
                if (NRHS == 2) u1[nxt][k] = U1[t];
            }
        }
#pragma unroll
        for (int k = 0; k < SB; k++) {
            p0 = u0[cur][k] - f[cur][k] * p0;
            u0[cur][k] = p0;
            if (NRHS == 2) {
                p1 = u1[cur][k] - f[cur][k] * p1;
                u1[cur][k] = p1;
            }
        }
        if (b + 1 < NSB) {
#pragma unroll
            for (int k = 0; k < SB; k++) {
                fgs_pin(f[nxt][k]);
                fgs_pin(u0[nxt][k]);
                if (NRHS == 2) fgs_pin(u1[nxt][k]);
            }
        }
#pragma unroll
        for (int k = 0; k < SB; k++) {
            const int t = M::tix(lane, FT - 1 - b * SB - k);
            U0[t] = u0[cur][k];
            if (NRHS == 2) U1[t] = u1[cur][k];
        }
    }
}

// the right-hand-side sweeps of one pass given the pivots: 64 lines per workgroup of
// FGS_WAVES waves.  Each wave moves 1/FGS_WAVES of every 64 x 64 tile between HBM and LDS
// and runs the chains of 64/FGS_WAVES lines (its 64 lanes compute them FGS_WAVES times over
// and store equal values).  With one wave per 64 lines a chunk's tile traffic (4 arrays in,
// 2 out, 96 KB) was bound by what one wave keeps in flight: the KITTI row pass took 147 us,
// of which the tile traffic alone (timing ablation FGS_NOCOMPUTE) was ~60.
#ifndef FGS_WAVES
#define FGS_WAVES 4
#endif
#ifndef FGS_SPLIT
#define FGS_SPLIT 1
#endif
template <int NRHS, bool ROWS>
__global__ void __launch_bounds__(64 * FGS_WAVES) k_fgs_solve(FgsSolveArgs a)
{
#pragma clang fp contract(off)
    constexpr int NK = 16 / FGS_WAVES;  // tile loads per wave and array
    __shared__ float Ct[FT * FP], RT[FT * FP], U0[FT * FP], U1[NRHS == 2 ? FT * FP : 1];
    const int lane = threadIdx.x & 63, pair = blockIdx.y;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int k0 = wave * NK;
    const int cl = wave * (64 / FGS_WAVES) + (lane % (64 / FGS_WAVES));  // the line this lane's chain runs
    const int n = ROWS ? a.w : a.h;
    const int l0 = blockIdx.x * FT, wp = a.wp;
    const uint64_t bytes = a.roi_pair * 4;
    const rsrc_t u0 = make_rsrc(a.u[0] + pair * a.roi_pair, bytes);
    const rsrc_t u1 = make_rsrc(a.u[NRHS == 2 ? 1 : 0] + pair * a.roi_pair, bytes);
    const rsrc_t C = make_rsrc(a.C + pair * a.roi_pair, bytes);
    const rsrc_t R = make_rsrc(a.R + pair * a.roi_pair, bytes);
    const rsrc_t I = make_rsrc(a.IT + pair * a.roi_pair, bytes);
    const uint32_t voff0 = tile_voff<ROWS>(l0, 0, wp, lane);
    const uint32_t cstep = ROWS ? FT * 4 : (uint32_t)FT * wp * 4;
    const float lam = a.lam;
    const int nchunks = (n + FT - 1) / FT;
    float4 rc[NK], rr[NK], r0[NK], r1[NK];
    tile_load_part<ROWS, NK>(rc, C, voff0, wp, k0);
    tile_load_part<ROWS, NK>(rr, R, voff0, wp, k0);
    tile_load_part<ROWS, NK>(r0, u0, voff0, wp, k0);
    if (NRHS == 2) tile_load_part<ROWS, NK>(r1, u1, voff0, wp, k0);
    tile_to_lds_part<ROWS, NK>(rc, Ct, lane, k0);
    tile_to_lds_part<ROWS, NK>(rr, RT, lane, k0);
    tile_to_lds_part<ROWS, NK>(r0, U0, lane, k0);
    if (NRHS == 2) tile_to_lds_part<ROWS, NK>(r1, U1, lane, k0);
    // FGS_SPLIT: the two right-hand sides run on different lanes (lanes with bit 4 set take
    // u[1]), so every chain is scalar single-issue arithmetic instead of packed pairs
    constexpr bool SPLIT = NRHS == 2 && FGS_SPLIT;
    static_assert(!SPLIT || 64 / FGS_WAVES <= 16, "split chains need lanes 16..31 to repeat lanes 0..15's lines");
    constexpr int NC = SPLIT ? 1 : NRHS;  // chains per lane
    float* const UA = SPLIT && (lane & 16) ? U1 : U0;
    float* const UB = U1;
    float p0 = 0.f, p1 = 0.f, cp = 0.f;
    for (int c = 0; c < nchunks; c++) {
        const int j0 = c * FT;
        const bool next = c + 1 < nchunks;
        __syncthreads();
        if (next) {  // prefetch chunk c+1 (consumed after the sweep)
            const uint32_t vn = voff0 + (c + 1) * cstep;
            tile_load_part<ROWS, NK>(rc, C, vn, wp, k0);
            tile_load_part<ROWS, NK>(rr, R, vn, wp, k0);
            tile_load_part<ROWS, NK>(r0, u0, vn, wp, k0);
            if (NRHS == 2) tile_load_part<ROWS, NK>(r1, u1, vn, wp, k0);
        }
        const int m = min(FT, n - j0);
        if (FGS_NOCOMPUTE) {  // timing ablation (results wrong): the tile traffic alone
        } else if (m == FT) {
            fgs_fwd_chunk<NC, ROWS>(RT, UA, UB, Ct, cl, lam, p0, p1, cp);
        } else {
#pragma unroll 8
            for (int jj = 0; jj < m; jj++) {
                const int t = TileMap<ROWS>::tix(cl, jj);
                const float r = RT[t];
                const float lcp = lam * cp;
                p0 = (UA[t] - lcp * p0) * r;
                UA[t] = p0;
                if (NC == 2) {
                    p1 = (UB[t] - lcp * p1) * r;
                    UB[t] = p1;
                }
                cp = Ct[t];
            }
        }
        __syncthreads();
        const uint32_t vc = voff0 + c * cstep;
        tile_store_part<ROWS, NK>(u0, vc, U0, wp, lane, k0);
        if (NRHS == 2) tile_store_part<ROWS, NK>(u1, vc, U1, wp, lane, k0);
        if (next) {
            __syncthreads();
            tile_to_lds_part<ROWS, NK>(rc, Ct, lane, k0);
            tile_to_lds_part<ROWS, NK>(rr, RT, lane, k0);
            tile_to_lds_part<ROWS, NK>(r0, U0, lane, k0);
            if (NRHS == 2) tile_to_lds_part<ROWS, NK>(r1, U1, lane, k0);
        }
    }
    // backward substitution; the last chunk's d' is still in LDS (RT takes c')
    {
        __syncthreads();
        tile_load_part<ROWS, NK>(rr, I, voff0 + (nchunks - 1) * cstep, wp, k0);
        tile_to_lds_part<ROWS, NK>(rr, RT, lane, k0);
    }
    for (int c = nchunks - 1; c >= 0; c--) {
        const int j0 = c * FT;
        const bool prev = c > 0;
        __syncthreads();
        if (prev) {
            const uint32_t vp = voff0 + (c - 1) * cstep;
            tile_load_part<ROWS, NK>(rr, I, vp, wp, k0);
            tile_load_part<ROWS, NK>(r0, u0, vp, wp, k0);
            if (NRHS == 2) tile_load_part<ROWS, NK>(r1, u1, vp, wp, k0);
        }
        const int m = min(FT, n - j0);
        int jj = m - 1;
        if (c == nchunks - 1) {  // x[n-1] = d'[n-1]
            const int t = TileMap<ROWS>::tix(cl, jj);
            p0 = UA[t];
            if (NC == 2) p1 = UB[t];
            jj--;
        }
        if (FGS_NOCOMPUTE) {
        } else if (jj == FT - 1) {
            fgs_bwd_chunk<NC, ROWS>(RT, UA, UB, cl, p0, p1);
        } else {
#pragma unroll 8
            for (; jj >= 0; jj--) {
                const int t = TileMap<ROWS>::tix(cl, jj);
                const float f = RT[t];
                p0 = UA[t] - f * p0;
                UA[t] = p0;
                if (NC == 2) {
                    p1 = UB[t] - f * p1;
                    UB[t] = p1;
                }
            }
        }
        __syncthreads();
        const uint32_t vc = voff0 + c * cstep;
        tile_store_part<ROWS, NK>(u0, vc, U0, wp, lane, k0);
        if (NRHS == 2) tile_store_part<ROWS, NK>(u1, vc, U1, wp, lane, k0);
        if (prev) {
            __syncthreads();
            tile_to_lds_part<ROWS, NK>(rr, RT, lane, k0);
            tile_to_lds_part<ROWS, NK>(r0, U0, lane, k0);
            if (NRHS == 2) tile_to_lds_part<ROWS, NK>(r1, U1, lane, k0);
        }
    }
}

// ---- narrow tiles (round 4): 16 lines x 64 positions, one wave per workgroup.  The 64-line
// workgroups above put a pass's whole tile traffic through 6 CUs on the KITTI row pass (375
// lines): each 64-step chunk moved 96 KB through one CU's LDS between its chain steps, ~3 us
// per chunk.  With 16 lines per workgroup the same pass spreads over 4x the CUs, a chunk moves
// 24 KB, and the lane -> chain mapping (and so every chain's float32 operations and their
// order) is unchanged: lane l runs line l % 16 (lanes with bit 4 set: the second right-hand
// side), lanes 32..63 repeat lanes 0..31.
constexpr int FL = 16;       // lines per narrow tile
constexpr int FPC = FL + 1;  // LDS pitch of a column tile's position rows
template <bool ROWS>
struct TileMap16 {
    // load k (0..3) of lane -> local (line, pos) of the float4's first element; the float4
    // runs along pos (ROWS: 4 lines of 64 positions per load) or along line (columns: 16
    // positions of 16 lines per load)
    __device__ static void at(int k, int lane, int& ll, int& pl)
    {
        if (ROWS) {
            ll = 4 * k + (lane >> 4);
            pl = (lane & 15) * 4;
        } else {
            pl = 16 * k + (lane >> 2);
            ll = (lane & 3) * 4;
        }
    }
    __device__ static int tix(int ll, int pl) { return ROWS ? ll * FP + pl : pl * FPC + ll; }
    __device__ static int tix_e(int ll, int pl, int e) { return ROWS ? tix(ll, pl + e) : tix(ll + e, pl); }
    static constexpr int KSTEP = ROWS ? 16 : 64;  // byte step of load k per element of pitch wp
    static constexpr int TS = ROWS ? FL * FP : FT * FPC;
};

template <bool ROWS>
__device__ inline void tile16_load(float4 (&r)[4], rsrc_t rs, uint32_t voff, int wp)
{
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, k * TileMap16<ROWS>::KSTEP * wp, 0);
        r[k] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
    }
}

template <bool ROWS>
__device__ inline void tile16_to_lds(const float4 (&r)[4], float* T, int lane)
{
    using M = TileMap16<ROWS>;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int ll, pl;
        M::at(k, lane, ll, pl);
        T[M::tix_e(ll, pl, 0)] = r[k].x;
        T[M::tix_e(ll, pl, 1)] = r[k].y;
        T[M::tix_e(ll, pl, 2)] = r[k].z;
        T[M::tix_e(ll, pl, 3)] = r[k].w;
    }
}

template <bool ROWS>
__device__ inline void tile16_store(rsrc_t rs, uint32_t voff, const float* T, int wp, int lane)
{
    using M = TileMap16<ROWS>;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        int ll, pl;
        M::at(k, lane, ll, pl);
        u32x4 v;
        v[0] = __float_as_uint(T[M::tix_e(ll, pl, 0)]);
        v[1] = __float_as_uint(T[M::tix_e(ll, pl, 1)]);
        v[2] = __float_as_uint(T[M::tix_e(ll, pl, 2)]);
        v[3] = __float_as_uint(T[M::tix_e(ll, pl, 3)]);
        // offset in the VGPR, soffset the literal 0 (see tile_store: gfx950 store-data hazard)
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff + (uint32_t)(k * M::KSTEP * wp), 0, 0);
    }
}

template <int NRHS, bool ROWS>
__global__ void __launch_bounds__(64) k_fgs_solve16(FgsSolveArgs a)
{
#pragma clang fp contract(off)
    using M = TileMap16<ROWS>;
    __shared__ float Ct[M::TS], RT[M::TS], U0[M::TS], U1[NRHS == 2 ? M::TS : 1];
    const int lane = threadIdx.x, pair = blockIdx.y;
    const int cl = lane % FL;  // the line this lane's chain runs
    const int n = ROWS ? a.w : a.h;
    const int l0 = blockIdx.x * FL, wp = a.wp;
    const uint64_t bytes = a.roi_pair * 4;
    const rsrc_t u0 = make_rsrc(a.u[0] + pair * a.roi_pair, bytes);
    const rsrc_t u1 = make_rsrc(a.u[NRHS == 2 ? 1 : 0] + pair * a.roi_pair, bytes);
    const rsrc_t C = make_rsrc(a.C + pair * a.roi_pair, bytes);
    const rsrc_t R = make_rsrc(a.R + pair * a.roi_pair, bytes);
    const rsrc_t I = make_rsrc(a.IT + pair * a.roi_pair, bytes);
    int ll0, pl0;
    M::at(0, lane, ll0, pl0);
    const uint32_t voff0 = (uint32_t)(TileMap<ROWS>::eoff(l0 + ll0, pl0, wp) * 4);
    const uint32_t cstep = ROWS ? FT * 4 : (uint32_t)FT * wp * 4;
    const float lam = a.lam;
    const int nchunks = (n + FT - 1) / FT;
    float4 rc[4], rr[4], r0[4], r1[4];
    tile16_load<ROWS>(rc, C, voff0, wp);
    tile16_load<ROWS>(rr, R, voff0, wp);
    tile16_load<ROWS>(r0, u0, voff0, wp);
    if (NRHS == 2) tile16_load<ROWS>(r1, u1, voff0, wp);
    tile16_to_lds<ROWS>(rc, Ct, lane);
    tile16_to_lds<ROWS>(rr, RT, lane);
    tile16_to_lds<ROWS>(r0, U0, lane);
    if (NRHS == 2) tile16_to_lds<ROWS>(r1, U1, lane);
    constexpr bool SPLIT = NRHS == 2;  // lanes with bit 4 set take u[1] (scalar chains, as FGS_SPLIT)
    constexpr int NC = SPLIT ? 1 : NRHS;
    float* const UA = SPLIT && (lane & 16) ? U1 : U0;
    float* const UB = U1;
    float p0 = 0.f, p1 = 0.f, cp = 0.f;
    for (int c = 0; c < nchunks; c++) {
        const int j0 = c * FT;
        const bool next = c + 1 < nchunks;
        __syncthreads();
        if (next) {  // prefetch chunk c+1 (consumed after the sweep)
            const uint32_t vn = voff0 + (c + 1) * cstep;
            tile16_load<ROWS>(rc, C, vn, wp);
            tile16_load<ROWS>(rr, R, vn, wp);
            tile16_load<ROWS>(r0, u0, vn, wp);
            if (NRHS == 2) tile16_load<ROWS>(r1, u1, vn, wp);
        }
        const int m = min(FT, n - j0);
        if (m == FT) {
            fgs_fwd_chunk<NC, ROWS, M>(RT, UA, UB, Ct, cl, lam, p0, p1, cp);
        } else {
#pragma unroll 8
            for (int jj = 0; jj < m; jj++) {
                const int t = M::tix(cl, jj);
                const float r = RT[t];
                const float lcp = lam * cp;
                p0 = (UA[t] - lcp * p0) * r;
                UA[t] = p0;
                if (NC == 2) {
                    p1 = (UB[t] - lcp * p1) * r;
                    UB[t] = p1;
                }
                cp = Ct[t];
            }
        }
        __syncthreads();
        const uint32_t vc = voff0 + c * cstep;
        tile16_store<ROWS>(u0, vc, U0, wp, lane);
        if (NRHS == 2) tile16_store<ROWS>(u1, vc, U1, wp, lane);
        if (next) {
            __syncthreads();
            tile16_to_lds<ROWS>(rc, Ct, lane);
            tile16_to_lds<ROWS>(rr, RT, lane);
            tile16_to_lds<ROWS>(r0, U0, lane);
            if (NRHS == 2) tile16_to_lds<ROWS>(r1, U1, lane);
        }
    }
    // backward substitution; the last chunk's d' is still in LDS (RT takes c')
    {
        __syncthreads();
        tile16_load<ROWS>(rr, I, voff0 + (nchunks - 1) * cstep, wp);
        tile16_to_lds<ROWS>(rr, RT, lane);
    }
    for (int c = nchunks - 1; c >= 0; c--) {
        const int j0 = c * FT;
        const bool prev = c > 0;
        __syncthreads();
        if (prev) {
            const uint32_t vp = voff0 + (c - 1) * cstep;
            tile16_load<ROWS>(rr, I, vp, wp);
            tile16_load<ROWS>(r0, u0, vp, wp);
            if (NRHS == 2) tile16_load<ROWS>(r1, u1, vp, wp);
        }
        const int m = min(FT, n - j0);
        int jj = m - 1;
        if (c == nchunks - 1) {  // x[n-1] = d'[n-1]
            const int t = M::tix(cl, jj);
            p0 = UA[t];
            if (NC == 2) p1 = UB[t];
            jj--;
        }
        if (jj == FT - 1) {
            fgs_bwd_chunk<NC, ROWS, M>(RT, UA, UB, cl, p0, p1);
        } else {
#pragma unroll 8
            for (; jj >= 0; jj--) {
                const int t = M::tix(cl, jj);
                const float f = RT[t];
                p0 = UA[t] - f * p0;
                UA[t] = p0;
                if (NC == 2) {
                    p1 = UB[t] - f * p1;
                    UB[t] = p1;
                }
            }
        }
        __syncthreads();
        const uint32_t vc = voff0 + c * cstep;
        tile16_store<ROWS>(u0, vc, U0, wp, lane);
        if (NRHS == 2) tile16_store<ROWS>(u1, vc, U1, wp, lane);
        if (prev) {
            __syncthreads();
            tile16_to_lds<ROWS>(rr, RT, lane);
            tile16_to_lds<ROWS>(r0, U0, lane);
            if (NRHS == 2) tile16_to_lds<ROWS>(r1, U1, lane);
        }
    }
}

struct WlsFinalArgs {
    const float* num;
    const float* den;
    size_t roi_pair;
    int16_t* out;  // [pair][H][W]
    size_t out_pair;
    int H, W, x0, y0, w, h, wp;
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
        const size_t o = pair * a.roi_pair + (size_t)i * a.wp + j;
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
