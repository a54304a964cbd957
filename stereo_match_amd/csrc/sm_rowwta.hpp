// sm_rowwta.hpp — fused horizontal paths + WTA, one wave per image row.
//
// OpenCV's MODE_SGBM runs the backward horizontal path inside the WTA loop
// (computeDisparitySGBM's `npasses == 1` branch); this kernel does the same on
// the GPU, which removes the W path volume from HBM entirely and takes both
// long (width1-step) serial chains out of the path-aggregation launch:
//   sweep 1 (x1 ascending):  E path, census cost from a register sliding
//                            window, L_E stored to its volume slot;
//   sweep 2 (x1 descending): W path, S = L_W + sum of the other slots
//                            (E + vertical family, prefetched one step ahead),
//                            then per pixel: first argmin, uniqueness test,
//                            C-truncating sub-pixel, disp2 key in LDS
//                            (atomicMin on (minS << 16) | (0xFFFF - x)),
//                            sub-pixel disparity in LDS;
//   final pass:              disp12MaxDiff check, raw row to HBM.
// A line is the whole wave (D/64 disparities per lane); every per-pixel
// reduction ends wave-uniform, so the per-pixel bookkeeping is scalar.
#pragma once
#include "sm_paths.hpp"

namespace smk {

struct RowArgs {
    const uint64_t* cl;  // census [pair][H][W] (census mode)
    const uint64_t* cr;
    size_t census_pair;
    const uint16_t* cost;  // SGBM cost volume [pair][H][width1][D] (parity mode)
    size_t cost_pair;
    uint8_t* L;  // path volumes [pair][slot][H][width1][D]; slot 0 = E, 1 = W (unused), 2.. = vertical
    size_t slot_bytes, L_pair_bytes;
    int H, W, width1, D, minD, minX1, P1, P2, uniq, disp12;
    int store_w;    // debug/parity: also store the W path volume (slot 1)
    int16_t* disp;  // [pair][H][W] pre-median
};

// One horizontal sweep of a 64-lane line over row y.  WTA == false: E path,
// stores its values.  WTA == true: W path fused with the winner-take-all.
template <bool WTA, int DPL, int NDIR, bool CENSUS, typename LT>
__device__ __forceinline__ void row_sweep(const RowArgs& a, int pair, int y, uint64_t* stage, uint32_t* key2,
                                          int16_t* drow)
{
    constexpr int DIR = WTA ? 1 : 0;
    constexpr int SGN = DIR == 0 ? 1 : -1;
    constexpr int NOTHER = NDIR - 1;  // slots summed into S besides W
    const int lane = threadIdx.x & 63;
    const int H = a.H, W = a.W, W1 = a.width1, D = a.D, minD = a.minD, minX1 = a.minX1;
    const uint32_t P1 = (uint32_t)a.P1, P2 = (uint32_t)a.P2;
    const uint64_t vol_bytes = (uint64_t)H * W1 * D * sizeof(LT);
    uint8_t* Lpair = a.L + (size_t)pair * a.L_pair_bytes;
    const int step_bytes = SGN * D * (int)sizeof(LT);
    const int off0 = (y * W1 + (DIR == 0 ? 0 : W1 - 1)) * D * (int)sizeof(LT) + lane * DPL * (int)sizeof(LT);

    // slot 0 (E) on the first sweep; slot 1 (W) only when asked for (parity debugging)
    rsrc_t rout = make_rsrc(Lpair + (WTA ? a.slot_bytes : 0), (WTA && !a.store_w) ? 0 : vol_bytes);
    rsrc_t rs[NOTHER > 0 ? NOTHER : 1];
    if constexpr (WTA) {
        rs[0] = make_rsrc(Lpair, vol_bytes);  // E
#pragma unroll
        for (int k = 1; k < NOTHER; k++) rs[k] = make_rsrc(Lpair + (size_t)(k + 1) * a.slot_bytes, vol_bytes);
    }
    using Raw = RawBytes<DPL * (int)sizeof(LT)>;
    Raw nx[NOTHER > 0 ? NOTHER : 1];
    auto fetch_other = [&](uint32_t off) {
        if constexpr (WTA) {
#pragma unroll
            for (int k = 0; k < NOTHER; k++) nx[k].load(rs[k], off);
        }
    };
    const int u = a.uniq;

    uint32_t Lp[DPL];
#pragma unroll
    for (int i = 0; i < DPL; i++) Lp[i] = 0;
    uint32_t minLp = 0;

    // per step: produce C[] for x1(s), then the common tail
    auto tail = [&](int s, int off, const uint32_t (&C)[DPL], const Raw (&oth)[NOTHER > 0 ? NOTHER : 1]) {
        uint32_t Ln[DPL];
        const uint32_t mn = sgm_step<64, DPL>(Lp, minLp, C, P1, P2, Ln);
        bstore_n<LT, DPL>(rout, s < W1 ? (uint32_t)off : kOOB, Ln);
        if constexpr (WTA) {
            uint32_t S[DPL];
            uint32_t kmin = 0xFFFFFFFFu;
#pragma unroll
            for (int i = 0; i < DPL; i++) {
                uint32_t acc = Ln[i];
#pragma unroll
                for (int k = 0; k < NOTHER; k++) acc += oth[k].template get<LT>(i);
                S[i] = min(acc, 32767u);
                kmin = min(kmin, (S[i] << 16) | wta_rank(lane * DPL + i, NDIR == 5));
            }
            kmin = Line<64>::min(kmin);
            const int minS = (int)(kmin >> 16), best = wta_unrank(kmin & 0xFFFF, NDIR == 5);
            bool badl = false;
#pragma unroll
            for (int i = 0; i < DPL; i++) {
                const int dd = best - (lane * DPL + i);
                badl |= ((int)S[i] * (100 - u) < minS * 100) && (dd > 1 || dd < -1);
            }
            const bool bad = __builtin_amdgcn_ballot_w64(badl) != 0;
            if (s < W1 && !bad && minS < 32767) {
                const int X = minX1 + W1 - 1 - s;
                int d16 = best * 16;
                if (best > 0 && best < D - 1) {
                    const int dm = best - 1, dq = best + 1;
                    uint32_t vm = 0, vq = 0;
#pragma unroll
                    for (int i = 0; i < DPL; i++) {
                        vm = (i == dm % DPL) ? S[i] : vm;
                        vq = (i == dq % DPL) ? S[i] : vq;
                    }
                    const int Sm = (int)__builtin_amdgcn_readlane(vm, dm / DPL);
                    const int Sq = (int)__builtin_amdgcn_readlane(vq, dq / DPL);
                    const int den = max(Sm + Sq - 2 * minS, 1);
                    d16 += ((Sm - Sq) * 16 + den) / (den * 2);  // C truncation
                }
                if (lane == 0) {
                    atomicMin(&key2[X - best - minD], ((uint32_t)minS << 16) | (uint32_t)(0xFFFF - X));
                    drow[X] = (int16_t)(d16 + minD * 16);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < DPL; i++) Lp[i] = Ln[i];
        minLp = mn;
    };

    const int nchunks = (W1 + 63) / 64;
    if constexpr (CENSUS) {
        const rsrc_t rcl = make_rsrc(a.cl + (size_t)pair * a.census_pair, (uint64_t)H * W * 8);
        const rsrc_t rcr = make_rsrc(a.cr + (size_t)pair * a.census_pair, (uint64_t)H * W * 8);
        const int fr_off = DIR == 0 ? -minD : -minD - (D - 1);
        uint64_t* st_cl = stage;
        uint64_t* st_fr = stage + 64;
        const int X0 = DIR == 0 ? minX1 : minX1 + W1 - 1;
        auto chunk_off = [&](int c) { return (uint32_t)((y * W + X0 + SGN * min(c * 64 + lane, W1 - 1)) * 8); };
        uint64_t wnd[DPL];
#pragma unroll
        for (int i = 0; i < DPL; i++)
            wnd[i] = bload_u64(rcr, (uint32_t)((y * W + X0 - SGN - minD - (lane * DPL + i)) * 8));
        uint64_t ccl = bload_u64(rcl, chunk_off(0));
        uint64_t cfr = bload_u64(rcr, chunk_off(0) + fr_off * 8);
        int off = off0;
        Raw cur[NOTHER > 0 ? NOTHER : 1];
        fetch_other((uint32_t)off);
        for (int c = 0; c < nchunks; c++) {
            st_cl[lane] = ccl;
            st_fr[lane] = cfr;
            const uint32_t nxt = chunk_off(min(c + 1, nchunks - 1));
            ccl = bload_u64(rcl, nxt);
            cfr = bload_u64(rcr, nxt + fr_off * 8);
            __builtin_amdgcn_wave_barrier();
            for (int t = 0; t < 64; t++) {
                const int s = c * 64 + t;
                const uint64_t clv = st_cl[t];
                const uint64_t frv = st_fr[t];
                if constexpr (DIR == 0) {
                    const uint64_t in = Line<64>::prev(frv, wnd[DPL - 1]);
#pragma unroll
                    for (int i = DPL - 1; i > 0; i--) wnd[i] = wnd[i - 1];
                    wnd[0] = in;
                } else {
                    const uint64_t in = Line<64>::next(frv, wnd[0]);
#pragma unroll
                    for (int i = 0; i < DPL - 1; i++) wnd[i] = wnd[i + 1];
                    wnd[DPL - 1] = in;
                }
                uint32_t C[DPL];
#pragma unroll
                for (int i = 0; i < DPL; i++) C[i] = (uint32_t)__popcll(clv ^ wnd[i]);
                if constexpr (WTA) {
#pragma unroll
                    for (int k = 0; k < NOTHER; k++) cur[k] = nx[k];
                    fetch_other(s + 1 < W1 ? (uint32_t)(off + step_bytes) : kOOB);
                }
                tail(s, off, C, cur);
                off += step_bytes;
            }
            __builtin_amdgcn_wave_barrier();
        }
    } else {
        const rsrc_t rc = make_rsrc(a.cost + (size_t)pair * a.cost_pair, (uint64_t)H * W1 * D * 2);
        const int coff0 = off0 / (int)sizeof(LT) * 2, cstep = step_bytes / (int)sizeof(LT) * 2;
        RawU16<DPL> nc;
        nc.load(rc, (uint32_t)coff0);
        int off = off0, coff = coff0;
        Raw cur[NOTHER > 0 ? NOTHER : 1];
        fetch_other((uint32_t)off);
        for (int s = 0; s < W1; s++) {
            uint32_t C[DPL];
            nc.unpack(C);
            coff += cstep;
            nc.load(rc, s + 1 < W1 ? (uint32_t)coff : kOOB);
            if constexpr (WTA) {
#pragma unroll
                for (int k = 0; k < NOTHER; k++) cur[k] = nx[k];
                fetch_other(s + 1 < W1 ? (uint32_t)(off + step_bytes) : kOOB);
            }
            tail(s, off, C, cur);
            off += step_bytes;
        }
    }
}

template <int DPL, int NDIR, bool CENSUS, typename LT>
__global__ void __launch_bounds__(64) k_row_wta(RowArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t sm64[];
    const int W = a.W, minD = a.minD, minX1 = a.minX1, maxX1 = a.minX1 + a.width1;
    const int INVALID = (minD - 1) * 16;
    uint64_t* stage = sm64;
    uint32_t* key2 = reinterpret_cast<uint32_t*>(sm64 + 128);
    int16_t* drow = reinterpret_cast<int16_t*>(key2 + W);
    const int y = blockIdx.x, pair = blockIdx.y, lane = threadIdx.x;
    for (int i = lane; i < W; i += 64) {
        key2[i] = 0xFFFFFFFFu;
        drow[i] = (int16_t)INVALID;
    }
    __builtin_amdgcn_wave_barrier();
    row_sweep<false, DPL, NDIR, CENSUS, LT>(a, pair, y, stage, key2, drow);
    __builtin_amdgcn_wave_barrier();
    row_sweep<true, DPL, NDIR, CENSUS, LT>(a, pair, y, stage, key2, drow);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    int16_t* out = a.disp + (size_t)pair * a.H * W + (size_t)y * W;
    for (int X = lane; X < W; X += 64) {
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
