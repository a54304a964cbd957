// sm_paths.hpp — SGM path aggregation on gfx950 (one launch, every direction,
// several pairs per launch via blockIdx.y).
//
// Recurrence (OpenCV computeDisparitySGBM with its P2-seeded Cbuf, i.e. the
// textbook Hirschmüller form; restated in oracle/sgm_np.py:_step):
//   L(p,d) = C(p,d) + min(Lp[d], min(Lp[d-1], Lp[d+1]) + P1, minLp + P2) - minLp
// with Lp = 0, minLp = 0 where a path enters the [minX1,maxX1) x [0,H) domain.
//
// Work decomposition:
//  * horizontal family (E, W): one line = one image row.  With D % 64 == 0 a
//    line is the whole wave (D/64 disparities per lane, min over d reduced to
//    an SGPR) — the horizontal chains are the longest serial dependency of the
//    pipeline, so they get the widest lines.  Census costs come from a register
//    sliding window shifted one disparity per step with wave_shr/wave_shl DPP;
//    the per-step left census and the one new right census value are staged
//    LANES steps at a time through wave-private LDS.
//  * vertical family (S, N and the four diagonals): 4 lines of 16 lanes per
//    wave (D/16 disparities per lane).  Diagonals are NOT wrapped: line b
//    visits x1 = b + dx*s, so a wave's 4 lines always sit on one image row at
//    4 consecutive columns; one staged window of D+3 right-census values in
//    wave-private LDS serves all of them.
//  * census cost = popcount(cl ^ cr) computed on the fly (no cost volume in
//    HBM); OpenCV-parity mode reads its int16 box-cost volume instead.
//  * outputs: one LT volume per direction [slot][H][width1][D] (d fastest).
#pragma once
#include "sm_common.hpp"

namespace smk {

struct PathsArgs {
    const uint64_t* cl;  // census left  [pair][H][W]
    const uint64_t* cr;  // census right [pair][H][W]
    size_t census_pair;  // elements per pair
    const uint16_t* cost;  // SGBM cost volume [pair][H][width1][D]
    size_t cost_pair;      // elements per pair
    uint8_t* L;            // path volumes [pair][slot][H][width1][D] (LT)
    size_t slot_bytes, L_pair_bytes;
    int H, W, width1, D, minD, minX1, P1, P2;
    int hblocks;  // workgroups per horizontal direction (slots 0 = E, 1 = W)
    int nv;       // vertical-family directions in this launch
    int v_dx[6], v_dy[6], v_slot[6], v_blk_start[7], v_line_lo[6], v_nlines[6];
};

template <int LANES, int DPL>
__device__ __forceinline__ uint32_t sgm_step(const uint32_t (&Lp)[DPL], uint32_t minLp, const uint32_t (&C)[DPL],
                                              uint32_t P1, uint32_t P2, uint32_t (&Ln)[DPL])
{
    const uint32_t lm = Line<LANES>::prev(kBig, Lp[DPL - 1]);
    const uint32_t lq = Line<LANES>::next(kBig, Lp[0]);
    const uint32_t delta = minLp + P2;
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
    return Line<LANES>::min(mn);
}

// raw (packed) cost words of DPL uint16 disparities, loaded ahead of use
template <int DPL>
struct RawCost {
    static constexpr int WORDS = (DPL * 2 + 3) / 4;
    uint32_t w[WORDS];
    __device__ __forceinline__ void load(const uint16_t* p)
    {
        if constexpr (DPL % 8 == 0) {
#pragma unroll
            for (int c = 0; c < DPL / 8; c++) {
                uint4 v = reinterpret_cast<const uint4*>(p)[c];
                w[4 * c] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
            }
        } else if constexpr (DPL % 4 == 0) {
#pragma unroll
            for (int c = 0; c < DPL / 4; c++) {
                uint2 v = reinterpret_cast<const uint2*>(p)[c];
                w[2 * c] = v.x; w[2 * c + 1] = v.y;
            }
        } else if constexpr (DPL % 2 == 0) {
#pragma unroll
            for (int c = 0; c < DPL / 2; c++) w[c] = reinterpret_cast<const uint32_t*>(p)[c];
        } else {
#pragma unroll
            for (int c = 0; c < WORDS; c++) {
                uint32_t lo = p[2 * c];
                uint32_t hi = 2 * c + 1 < DPL ? p[2 * c + 1] : 0u;
                w[c] = lo | (hi << 16);
            }
        }
    }
    __device__ __forceinline__ void unpack(uint32_t (&C)[DPL]) const
    {
#pragma unroll
        for (int i = 0; i < DPL; i++) C[i] = (w[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
    }
};

// ------------------------------------------------------- horizontal family
template <int LANES, int DPL, bool CENSUS, typename LT>
__device__ __forceinline__ void horz_family(const PathsArgs& a, int pair, int hb, uint64_t* stage)
{
    constexpr int LPW = 64 / LANES;
    const int dir = hb >= a.hblocks ? 1 : 0;  // 0: E (x increasing), 1: W (x decreasing)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane % LANES, kl = lane / LANES;
    const int wline = ((hb - dir * a.hblocks) * 4 + wave) * LPW;
    const int H = a.H, W = a.W, W1 = a.width1, D = a.D, minD = a.minD, minX1 = a.minX1;
    if (wline >= H) return;  // wave-uniform
    const bool line_ok = wline + kl < H;
    const int y = min(wline + kl, H - 1);
    const uint32_t P1 = (uint32_t)a.P1, P2 = (uint32_t)a.P2;
    LT* __restrict__ Lrow = (LT*)(a.L + (size_t)pair * a.L_pair_bytes + (size_t)dir * a.slot_bytes) +
                            (size_t)y * W1 * D + g * DPL;
    auto Xof = [&](int s) { return dir == 0 ? minX1 + s : minX1 + W1 - 1 - s; };

    uint32_t Lp[DPL];
#pragma unroll
    for (int i = 0; i < DPL; i++) Lp[i] = 0;
    uint32_t minLp = 0;

    if constexpr (CENSUS) {
        const uint64_t* __restrict__ clrow = a.cl + (size_t)pair * a.census_pair + (size_t)y * W;
        const uint64_t* __restrict__ crrow = a.cr + (size_t)pair * a.census_pair + (size_t)y * W;
        const int fr_off = dir == 0 ? -minD : -minD - (D - 1);
        uint64_t* st_cl = stage + kl * LANES;  // [LPW][LANES] left census per step
        uint64_t* st_fr = stage + 64 + kl * LANES;  // [LPW][LANES] entering right census per step
        uint64_t ccl, cfr;
        auto load_chunk = [&](int c) {
            const int X = Xof(min(c * LANES + g, W1 - 1));
            ccl = clrow[X];
            cfr = crrow[X + fr_off];
        };
        uint64_t wnd[DPL];
        {
            const int X = Xof(0);
#pragma unroll
            for (int i = 0; i < DPL; i++) wnd[i] = crrow[X - minD - (g * DPL + i)];
        }
        load_chunk(0);
        st_cl[g] = ccl;
        st_fr[g] = cfr;
        const int nchunks = (W1 + LANES - 1) / LANES;
        if (nchunks > 1) load_chunk(1);
        for (int s = 0; s < W1; s++) {
            const int sl = s % LANES;
            if (sl == 0 && s > 0) {
                st_cl[g] = ccl;
                st_fr[g] = cfr;
                const int c = s / LANES + 1;
                if (c < nchunks) load_chunk(c);
            }
            __builtin_amdgcn_wave_barrier();
            const uint64_t clv = st_cl[sl];
            const uint64_t frv = st_fr[sl];
            if (s > 0) {
                if (dir == 0) {
                    const uint64_t in = Line<LANES>::prev(frv, wnd[DPL - 1]);
#pragma unroll
                    for (int i = DPL - 1; i > 0; i--) wnd[i] = wnd[i - 1];
                    wnd[0] = in;
                } else {
                    const uint64_t in = Line<LANES>::next(frv, wnd[0]);
#pragma unroll
                    for (int i = 0; i < DPL - 1; i++) wnd[i] = wnd[i + 1];
                    wnd[DPL - 1] = in;
                }
            }
            uint32_t C[DPL], Ln[DPL];
#pragma unroll
            for (int i = 0; i < DPL; i++) C[i] = (uint32_t)__popcll(clv ^ wnd[i]);
            const uint32_t mn = sgm_step<LANES, DPL>(Lp, minLp, C, P1, P2, Ln);
            if (line_ok) store_n<DPL>(Lrow + (size_t)(Xof(s) - minX1) * D, Ln);
#pragma unroll
            for (int i = 0; i < DPL; i++) Lp[i] = Ln[i];
            minLp = mn;
        }
    } else {
        const uint16_t* __restrict__ crow = a.cost + (size_t)pair * a.cost_pair + (size_t)y * W1 * D + g * DPL;
        RawCost<DPL> nxt;
        nxt.load(crow + (size_t)(Xof(0) - minX1) * D);
        for (int s = 0; s < W1; s++) {
            uint32_t C[DPL], Ln[DPL];
            nxt.unpack(C);
            if (s + 1 < W1) nxt.load(crow + (size_t)(Xof(s + 1) - minX1) * D);
            const uint32_t mn = sgm_step<LANES, DPL>(Lp, minLp, C, P1, P2, Ln);
            if (line_ok) store_n<DPL>(Lrow + (size_t)(Xof(s) - minX1) * D, Ln);
#pragma unroll
            for (int i = 0; i < DPL; i++) Lp[i] = Ln[i];
            minLp = mn;
        }
    }
}

// --------------------------------------------------------- vertical family
template <int DPL, bool CENSUS, typename LT>
__device__ __forceinline__ void vert_family(const PathsArgs& a, int pair, int vb, uint64_t* win)
{
    constexpr int NW = (16 * DPL + 3 + 63) / 64;  // window entries per lane
    int k = 0;
#pragma unroll
    for (int i = 1; i < 6; i++)
        if (i < a.nv && vb >= a.v_blk_start[i]) k = i;
    const int dx = a.v_dx[k], dy = a.v_dy[k];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane & 15, kl = lane >> 4;
    const int wline = ((vb - a.v_blk_start[k]) * 4 + wave) * 4;
    if (wline >= a.v_nlines[k]) return;  // wave-uniform
    const bool line_ok = wline + kl < a.v_nlines[k];
    const int b0 = a.v_line_lo[k] + wline;  // x1 of line 0 at step 0 (unwrapped)
    const int H = a.H, W = a.W, W1 = a.width1, D = a.D, minD = a.minD, minX1 = a.minX1;
    const uint32_t P1 = (uint32_t)a.P1, P2 = (uint32_t)a.P2;
    int s_lo, s_hi;
    if (dx == 0) {
        s_lo = 0;
        s_hi = H;
    } else if (dx > 0) {
        s_lo = max(0, -(b0 + 3));
        s_hi = min(H, W1 - b0);
    } else {
        s_lo = max(0, b0 - W1 + 1);
        s_hi = min(H, b0 + 4);
    }
    LT* __restrict__ Lv = (LT*)(a.L + (size_t)pair * a.L_pair_bytes + (size_t)a.v_slot[k] * a.slot_bytes) + g * DPL;

    uint32_t Lp[DPL];
#pragma unroll
    for (int i = 0; i < DPL; i++) Lp[i] = 0;
    uint32_t minLp = 0;

    if constexpr (CENSUS) {
        const uint64_t* __restrict__ clp = a.cl + (size_t)pair * a.census_pair;
        const uint64_t* __restrict__ crp = a.cr + (size_t)pair * a.census_pair;
        uint64_t pw[NW];
        uint64_t pcl;
        auto fetch = [&](int s) {
            const int y = dy > 0 ? s : H - 1 - s;
            const int X0 = minX1 + b0 + dx * s;
            const uint64_t* row = crp + (size_t)y * W;
            const int base = X0 - minD - D + 1;
#pragma unroll
            for (int j = 0; j < NW; j++) pw[j] = row[min(max(base + lane + 64 * j, 0), W - 1)];
            pcl = clp[(size_t)y * W + min(max(X0 + kl, 0), W - 1)];
        };
        fetch(s_lo);
        for (int s = s_lo; s < s_hi; s++) {
#pragma unroll
            for (int j = 0; j < NW; j++)
                if (j < NW - 1 || lane + 64 * j < D + 3) win[lane + 64 * j] = pw[j];
            const uint64_t clv = pcl;
            __builtin_amdgcn_wave_barrier();
            if (s + 1 < s_hi) fetch(s + 1);
            uint32_t C[DPL], Ln[DPL];
            const int e0 = kl + D - 1 - g * DPL;
#pragma unroll
            for (int i = 0; i < DPL; i++) C[i] = (uint32_t)__popcll(clv ^ win[e0 - i]);
            const uint32_t mn = sgm_step<16, DPL>(Lp, minLp, C, P1, P2, Ln);
            const int x1 = b0 + kl + dx * s;
            if (line_ok && x1 >= 0 && x1 < W1) {
                const int y = dy > 0 ? s : H - 1 - s;
                store_n<DPL>(Lv + ((size_t)y * W1 + x1) * D, Ln);
#pragma unroll
                for (int i = 0; i < DPL; i++) Lp[i] = Ln[i];
                minLp = mn;
            }
        }
    } else {
        const uint16_t* __restrict__ cp = a.cost + (size_t)pair * a.cost_pair + g * DPL;
        RawCost<DPL> nxt;
        auto fetch = [&](int s) {
            const int y = dy > 0 ? s : H - 1 - s;
            const int x1 = min(max(b0 + kl + dx * s, 0), W1 - 1);
            nxt.load(cp + ((size_t)y * W1 + x1) * D);
        };
        fetch(s_lo);
        for (int s = s_lo; s < s_hi; s++) {
            uint32_t C[DPL], Ln[DPL];
            nxt.unpack(C);
            if (s + 1 < s_hi) fetch(s + 1);
            const uint32_t mn = sgm_step<16, DPL>(Lp, minLp, C, P1, P2, Ln);
            const int x1 = b0 + kl + dx * s;
            if (line_ok && x1 >= 0 && x1 < W1) {
                const int y = dy > 0 ? s : H - 1 - s;
                store_n<DPL>(Lv + ((size_t)y * W1 + x1) * D, Ln);
#pragma unroll
                for (int i = 0; i < DPL; i++) Lp[i] = Ln[i];
                minLp = mn;
            }
        }
    }
}

// LDS per wave: vertical window (D+3 u64) or horizontal staging (2 x 64 u64)
template <int DPLV>
constexpr int lds_per_wave()
{
    return (16 * DPLV + 3) > 128 ? (16 * DPLV + 3 + 1) & ~1 : 128;
}

template <int DPLV, int LANESH, int DPLH, bool CENSUS, typename LT>
__global__ void __launch_bounds__(256) k_sgm_paths(PathsArgs a)
{
    constexpr int PW = lds_per_wave<DPLV>();
    __shared__ __attribute__((aligned(16))) uint64_t lds[4 * PW];
    uint64_t* mine = lds + (threadIdx.x >> 6) * PW;
    const int pair = blockIdx.y;
    const int b = blockIdx.x;
    if (b < 2 * a.hblocks)
        horz_family<LANESH, DPLH, CENSUS, LT>(a, pair, b, mine);
    else
        vert_family<DPLV, CENSUS, LT>(a, pair, b - 2 * a.hblocks, mine);
}

// --------------------------------------------------------------------- WTA
// One workgroup of NT threads per (row, pair); a 16-lane group per pixel.
struct WtaArgs {
    const uint8_t* L;
    size_t slot_bytes, L_pair_bytes;
    int nslots;
    int H, W, width1, D, minD, minX1, uniq, disp12;
    int16_t* disp;  // [pair][H][W] pre-median
};

template <int DPL, typename LT, int NT>
__global__ void __launch_bounds__(NT) k_wta(WtaArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int W = a.W, D = a.D, minD = a.minD, minX1 = a.minX1;
    const int maxX1 = minX1 + a.width1;
    const int INVALID = (minD - 1) * 16;
    uint32_t* key2 = smem;
    int* drow = reinterpret_cast<int*>(smem + W);
    const int y = blockIdx.x, pair = blockIdx.y;
    for (int i = threadIdx.x; i < W; i += NT) {
        key2[i] = 0xFFFFFFFFu;
        drow[i] = INVALID;
    }
    __syncthreads();
    const int g = threadIdx.x & 15;
    const int grp = threadIdx.x >> 4;
    const LT* __restrict__ Lb = (const LT*)(a.L + (size_t)pair * a.L_pair_bytes) + g * DPL;
    const size_t slot = a.slot_bytes / sizeof(LT);
    const int u = a.uniq;
    for (int x = grp; x < a.width1; x += NT / 16) {
        const size_t off = ((size_t)y * a.width1 + x) * D;
        uint32_t S[DPL];
#pragma unroll
        for (int i = 0; i < DPL; i++) S[i] = 0;
        for (int k = 0; k < a.nslots; k++) {
            uint32_t t[DPL];
            load_n<DPL>(Lb + (size_t)k * slot + off, t);
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
    }
}

}  // namespace smk
