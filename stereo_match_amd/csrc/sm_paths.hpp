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
#include "sm_pk.hpp"

namespace smk {

// the WTA's path-volume loads non-temporal (read once: census8 KITTI WTA 76.5 -> 69.1 us
// per pair); -DWTA_NT_LOADS=0 builds plain loads
#ifndef WTA_NT_LOADS
#define WTA_NT_LOADS 1
#endif

// cache policy of the path-volume stores: nt (2), so the volumes streaming out do not
// evict the launch group's cost volume from the Infinity Cache while the other directions
// re-read it (census8 KITTI: WTA 80 -> 74 us per pair; with Infinity-Cache-sized groups
// paths 156 -> 145, sm_api.hip group_size); -DPATHS_STORE_AUX=0 builds the default policy
#ifndef PATHS_STORE_AUX
#define PATHS_STORE_AUX 2
#endif

struct PathsArgs {
    const uint64_t* cl;  // census left  [pair][H][W]
    const uint64_t* cr;  // census right [pair][H][W]
    size_t census_pair;  // elements per pair
    const uint16_t* cost;  // SGBM cost volume [pair][H][width1][D]
    size_t cost_pair;      // elements per pair
    const uint8_t* cost8;  // census mode: precomputed u8 Hamming cost volume for the vertical family, or null
    uint8_t* L;            // path volumes [pair][slot][H][width1][D] (LT)
    size_t slot_bytes, L_pair_bytes;
    int H, W, width1, D, minD, minX1, P1, P2;
    int hblocks;  // workgroups per horizontal direction (slots 0 = E, 1 = W)
    int dbg;      // timing ablations only: 1 skip horizontal, 2 skip vertical, 4 drop stores
    int nv;       // vertical-family directions in this launch
    int v_dx[6], v_dy[6], v_slot[6], v_blk_start[7], v_line_lo[6], v_nlines[6];
    // fused-sweep fallback (sm_api.hip run_group): when set, the launch is a small
    // grid that does nothing unless *guard != 0 (a sweep strip gave up waiting for
    // its neighbours), and then walks all nblocks x npairs blocks grid-stride
    const uint32_t* guard;
    int nblocks, npairs;
};

// fallback launches read the sweep's group flag (written by another kernel)
__device__ __forceinline__ bool guard_clear(const uint32_t* g)
{
    return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
}

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

// ------------------------------------------------------- horizontal family
// Steps run in chunks of LANES; each chunk's left-census values and entering
// right-census values (one per step and line) are loaded one chunk ahead and
// staged in wave-private LDS.  Steps past the row end still execute (their
// stores land out of range and are dropped) so the inner loop has no
// conditional memory operation.
template <int DIR, int LANES, int DPL, bool CENSUS, typename LT>
__device__ __forceinline__ void horz_impl(const PathsArgs& a, int pair, int hb, uint64_t* stage)
{
    constexpr int LPW = 64 / LANES;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane % LANES, kl = lane / LANES;
    const int wline = ((hb - DIR * a.hblocks) * 4 + wave) * LPW;
    const int H = a.H, W = a.W, W1 = a.width1, D = a.D, minD = a.minD, minX1 = a.minX1;
    if (wline >= H) return;  // wave-uniform
    const bool line_ok = wline + kl < H;
    const int y = min(wline + kl, H - 1);
    const uint32_t P1 = (uint32_t)a.P1, P2 = (uint32_t)a.P2;
    const rsrc_t rout = make_rsrc(a.L + (size_t)pair * a.L_pair_bytes + (size_t)DIR * a.slot_bytes,
                                  (a.dbg & 4) ? 0 : (uint64_t)H * W1 * D * sizeof(LT));
    // byte offset of this lane's slice at step s: row y, x1 = DIR ? W1-1-s : s
    constexpr int SGN = DIR == 0 ? 1 : -1;
    const int step_bytes = SGN * D * (int)sizeof(LT);
    const int off0 = (y * W1 + (DIR == 0 ? 0 : W1 - 1)) * D * (int)sizeof(LT) + g * DPL * (int)sizeof(LT);
    const int nchunks = (W1 + LANES - 1) / LANES;

    uint32_t Lp[DPL];
#pragma unroll
    for (int i = 0; i < DPL; i++) Lp[i] = 0;
    uint32_t minLp = 0;

    if constexpr (CENSUS) {
        if (a.cost8 && !(a.dbg & 2048)) {  // costs from the precomputed u8 volume (same [H][W1][D] layout as L)
            // ring of PF loads in flight: step s uses ring[s % PF], then refills it with step s + PF
#ifndef HPF8
#define HPF8 8
#endif
            constexpr int PF = HPF8;
            const rsrc_t rc = make_rsrc(a.cost8 + (size_t)pair * a.cost_pair, (uint64_t)H * W1 * D);
            RawBytes<DPL> ring[PF];
#pragma unroll
            for (int k = 0; k < PF; k++) {
                ring[k].load(rc, k < W1 ? (uint32_t)(off0 + k * step_bytes) : kOOB);
                // issue order = slot order: the loop-head wait is the max over entry
                // paths, and slot 0 issued last would make it vmcnt(0) every round
                asm volatile("" ::: "memory");
            }
            int off = off0;
            for (int s0 = 0; s0 < W1; s0 += PF) {
#pragma unroll
                for (int k = 0; k < PF; k++) {
                    const int s = s0 + k;
                    uint32_t C[DPL], Ln[DPL];
                    // the slot is read only after the previous step (no hoisted unpacks,
                    // whose waits would cover the younger slots too)
#pragma unroll
                    for (int j = 0; j < RawBytes<DPL>::WORDS; j++) asm volatile("" : "+v"(ring[k].w[j]) : "v"(minLp));
#pragma unroll
                    for (int i = 0; i < DPL; i++) C[i] = ring[k].template get<uint8_t>(i);
                    // materialise the slot's values before its refill is issued: otherwise
                    // hipcc keeps both, rotates the ring with moves at the back-edge and
                    // those wait (vmcnt) for the loads just issued (no prefetch left)
#pragma unroll
                    for (int i = 0; i < DPL; i++) asm volatile("" : "+v"(C[i])::"memory");
                    ring[k].load(rc, s + PF < W1 ? (uint32_t)(off + PF * step_bytes) : kOOB);
                    const uint32_t mn = sgm_step<LANES, DPL>(Lp, minLp, C, P1, P2, Ln);
                    bstore_n<LT, DPL, PATHS_STORE_AUX>(rout, (line_ok && s < W1) ? (uint32_t)off : kOOB, Ln);
                    off += step_bytes;
#pragma unroll
                    for (int i = 0; i < DPL; i++) Lp[i] = Ln[i];
                    minLp = mn;
                }
            }
            return;
        }
        const rsrc_t rcl = make_rsrc(a.cl + (size_t)pair * a.census_pair, (uint64_t)H * W * 8);
        const rsrc_t rcr = make_rsrc(a.cr + (size_t)pair * a.census_pair, (uint64_t)H * W * 8);
        const int fr_off = DIR == 0 ? -minD : -minD - (D - 1);
        uint64_t* st_cl = stage + kl * LANES;       // [LPW][LANES] left census per step
        uint64_t* st_fr = stage + 64 + kl * LANES;  // [LPW][LANES] entering right census per step
        const int X0 = DIR == 0 ? minX1 : minX1 + W1 - 1;
        auto chunk_off = [&](int c) { return (uint32_t)((y * W + X0 + SGN * min(c * LANES + g, W1 - 1)) * 8); };
        // window for "step -1"; step 0's shift brings in its entering value
        // (the one element that would sit outside the image is shifted out)
        uint64_t wnd[DPL];
#pragma unroll
        for (int i = 0; i < DPL; i++)
            wnd[i] = bload_u64(rcr, (uint32_t)((y * W + X0 - SGN - minD - (g * DPL + i)) * 8));
        uint64_t ccl = bload_u64(rcl, chunk_off(0));
        uint64_t cfr = bload_u64(rcr, chunk_off(0) + fr_off * 8);
        int off = off0;
        for (int c = 0; c < nchunks; c++) {
            st_cl[g] = ccl;
            st_fr[g] = cfr;
            const uint32_t nxt = chunk_off(min(c + 1, nchunks - 1));
            ccl = bload_u64(rcl, nxt);
            cfr = bload_u64(rcr, nxt + fr_off * 8);
            __builtin_amdgcn_wave_barrier();
            const int lim = W1 - c * LANES;  // steps of this chunk inside the row
            for (int t = 0; t < LANES; t++) {
                const uint64_t clv = st_cl[t];
                const uint64_t frv = st_fr[t];
                if constexpr (DIR == 0) {
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
                uint32_t C[DPL], Ln[DPL];
#pragma unroll
                for (int i = 0; i < DPL; i++) C[i] = (uint32_t)__popcll(clv ^ wnd[i]);
                const uint32_t mn = sgm_step<LANES, DPL>(Lp, minLp, C, P1, P2, Ln);
                bstore_n<LT, DPL, PATHS_STORE_AUX>(rout, (line_ok && t < lim) ? (uint32_t)off : kOOB, Ln);
                off += step_bytes;
#pragma unroll
                for (int i = 0; i < DPL; i++) Lp[i] = Ln[i];
                minLp = mn;
            }
            __builtin_amdgcn_wave_barrier();
        }
    } else {
        // u16 cost volume; ring of PF loads in flight (the serial chain of one
        // line is short of independent work, so the loads are issued PF steps ahead)
#ifndef HPF16
#define HPF16 8  // sgbm5 sweeps, 8 KITTI pairs: E/W lines 86.8 -> 77.4 us per pair (4 -> 8)
#endif
        constexpr int PF = HPF16;
        const rsrc_t rc = make_rsrc(a.cost + (size_t)pair * a.cost_pair, (uint64_t)H * W1 * D * 2);
        const int coff0 = off0 / (int)sizeof(LT) * 2, cstep = step_bytes / (int)sizeof(LT) * 2;
        RawU16<DPL> ring[PF];
#pragma unroll
        for (int k = 0; k < PF; k++) {
            ring[k].load(rc, k < W1 ? (uint32_t)(coff0 + k * cstep) : kOOB);
            asm volatile("" ::: "memory");  // issue order = slot order (see the u8 ring)
        }
        int off = off0, coff = coff0;
        for (int s0 = 0; s0 < W1; s0 += PF) {
#pragma unroll
            for (int k = 0; k < PF; k++) {
                const int s = s0 + k;
                uint32_t C[DPL], Ln[DPL];
#pragma unroll
                for (int j = 0; j < RawU16<DPL>::WORDS; j++) asm volatile("" : "+v"(ring[k].w[j]) : "v"(minLp));
                ring[k].unpack(C);
#pragma unroll
                for (int i = 0; i < DPL; i++) asm volatile("" : "+v"(C[i])::"memory");  // see the u8 ring
                ring[k].load(rc, s + PF < W1 ? (uint32_t)(coff + PF * cstep) : kOOB);
                coff += cstep;
                const uint32_t mn = sgm_step<LANES, DPL>(Lp, minLp, C, P1, P2, Ln);
                bstore_n<LT, DPL, PATHS_STORE_AUX>(rout, (line_ok && s < W1) ? (uint32_t)off : kOOB, Ln);
                off += step_bytes;
#pragma unroll
                for (int i = 0; i < DPL; i++) Lp[i] = Ln[i];
                minLp = mn;
            }
        }
    }
}

template <int LANES, int DPL, bool CENSUS, typename LT>
__device__ __forceinline__ void horz_family(const PathsArgs& a, int pair, int hb, uint64_t* stage)
{
    if (hb < a.hblocks)
        horz_impl<0, LANES, DPL, CENSUS, LT>(a, pair, hb, stage);
    else
        horz_impl<1, LANES, DPL, CENSUS, LT>(a, pair, hb, stage);
}

// --------------------------------------------------------- vertical family
// A wave owns LPW = 64/VL lines b0 + 8*kl (lines of VL lanes, VL = 16 or 8):
// all on one image row per step, 8 columns apart.  The right-census window
// (D + 8*(LPW-1) values) is staged per step
// in wave-private LDS in class-major order, phys(e) = (e & 7)*S + (e >> 3)
// with S = 2 (mod 16): the coalesced window writes hit 16 distinct bank
// pairs per 16 lanes, and every per-element read is 16 consecutive slots per
// line with the 4 lines mostly reading the SAME slots (broadcast), so both
// are conflict-free and each read is a ds_read_b64 with an immediate offset.
template <int D, int LPW>
struct VWin {
    static constexpr int ENTRIES = D + 8 * (LPW - 1);
    static constexpr int S0 = (ENTRIES + 7) / 8;
    static constexpr int S = S0 + ((2 - S0 % 16) + 16) % 16;  // smallest S >= S0 with S % 16 == 2
    static constexpr int WORDS = 8 * S;                       // u64 per wave
    static constexpr int NW = (ENTRIES + 63) / 64;            // window values loaded per lane
    static __device__ __forceinline__ int phys(int e) { return (e & 7) * S + (e >> 3); }
};

template <int VL, int DPL, bool CENSUS, typename LT>
__device__ __forceinline__ void vert_family(const PathsArgs& a, int pair, int vb, uint64_t* win)
{
    constexpr int LPW = 64 / VL;
    using VW = VWin<VL * DPL, LPW>;
    int k = 0;
#pragma unroll
    for (int i = 1; i < 6; i++)
        if (i < a.nv && vb >= a.v_blk_start[i]) k = i;
    const int dx = a.v_dx[k], dy = a.v_dy[k];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane % VL, kl = lane / VL;
    // line numbering: 8 waves cover 8*LPW lines; wave w of the group owns lines w + 8*kl
    const int wv = (vb - a.v_blk_start[k]) * 4 + wave;
    const int wline = (wv >> 3) * (8 * LPW) + (wv & 7);  // relative line index of kl = 0
    if (wline >= a.v_nlines[k]) return;          // wave-uniform
    const bool line_ok = wline + 8 * kl < a.v_nlines[k];
    const int b0 = a.v_line_lo[k] + wline;  // x1 of line 0 at step 0 (unwrapped)
    const int H = a.H, W = a.W, W1 = a.width1, D = a.D, minD = a.minD, minX1 = a.minX1;
    const uint32_t P1 = (uint32_t)a.P1, P2 = (uint32_t)a.P2;
    int s_lo, s_hi;  // steps where at least one of the wave's lines is inside [0, W1)
    if (dx == 0) {
        s_lo = 0;
        s_hi = H;
    } else if (dx > 0) {
        s_lo = max(0, -(b0 + 8 * (LPW - 1)));
        s_hi = min(H, W1 - b0);
    } else {
        s_lo = max(0, b0 - W1 + 1);
        s_hi = min(H, b0 + 8 * (LPW - 1) + 1);
    }
    const int ysgn = dy > 0 ? 1 : -1;
    const int y_lo = dy > 0 ? s_lo : H - 1 - s_lo;
    const rsrc_t rout = make_rsrc(a.L + (size_t)pair * a.L_pair_bytes + (size_t)a.v_slot[k] * a.slot_bytes,
                                  (a.dbg & 4) ? 0 : (uint64_t)H * W1 * D * sizeof(LT));
    // this lane's output slice at step s: (y_lo + ysgn*(s-s_lo), x1 = b0 + 8kl + dx*s)
    int x1 = b0 + 8 * kl + dx * s_lo;
    int off = (y_lo * W1 + x1) * D * (int)sizeof(LT) + g * DPL * (int)sizeof(LT);
    const int step_bytes = (ysgn * W1 + dx) * D * (int)sizeof(LT);
    // a line enters the domain one step after x1 == enter_x; its state must be 0 then
    const int enter_x = dx > 0 ? -1 : W1;

    uint32_t Lp[DPL];
#pragma unroll
    for (int i = 0; i < DPL; i++) Lp[i] = 0;
    uint32_t minLp = 0;

    auto reset_entering = [&]() {
        if (dx != 0) {
            const bool ent = x1 == enter_x;
            if (__builtin_amdgcn_ballot_w64(ent)) {  // wave-uniform, at most 4 times per wave
#pragma unroll
                for (int i = 0; i < DPL; i++) Lp[i] = ent ? 0u : Lp[i];
                minLp = ent ? 0u : minLp;
            }
        }
    };

    if constexpr (CENSUS) {
        if (a.cost8) {  // costs read from the precomputed u8 volume [pair][H][W1][D] (same layout as L)
            const rsrc_t rc = make_rsrc(a.cost8 + (size_t)pair * a.cost_pair, (uint64_t)H * W1 * D);
            int coff = off;
            RawBytes<DPL> nxt;
            nxt.load(rc, (uint32_t)coff);
            for (int s = s_lo; s < s_hi; s++) {
                uint32_t C[DPL], Ln[DPL];
#pragma unroll
                for (int i = 0; i < DPL; i++) C[i] = nxt.template get<uint8_t>(i);
                coff += step_bytes;
                nxt.load(rc, (uint32_t)coff);  // out-of-range offsets read 0 (inactive lines only)
                const uint32_t mn = sgm_step<VL, DPL>(Lp, minLp, C, P1, P2, Ln);
                const bool active = line_ok && x1 >= 0 && x1 < W1;
                bstore_n<LT, DPL, PATHS_STORE_AUX>(rout, active ? (uint32_t)off : kOOB, Ln);
#pragma unroll
                for (int i = 0; i < DPL; i++) Lp[i] = Ln[i];
                minLp = mn;
                reset_entering();
                off += step_bytes;
                x1 += dx;
            }
            return;
        }
        const rsrc_t rcl = make_rsrc(a.cl + (size_t)pair * a.census_pair, (uint64_t)H * W * 8);
        const rsrc_t rcr = make_rsrc(a.cr + (size_t)pair * a.census_pair, (uint64_t)H * W * 8);
        // window entry e at step s = right census (y, X0 - minD - D + 1 + e), X0 = minX1 + b0 + dx*s;
        // entries outside the image are read only by inactive lines (range check returns 0).
        int woff = (y_lo * W + (minX1 + b0 + dx * s_lo) - minD - D + 1 + lane) * 8;
        int coff = (y_lo * W + (minX1 + b0 + dx * s_lo) + 8 * kl) * 8;
        const int wstep = (ysgn * W + dx) * 8;
        int wdst[VW::NW];
#pragma unroll
        for (int j = 0; j < VW::NW; j++) wdst[j] = VW::phys(lane + 64 * j);
        // line kl, element i reads e = D-1 + 8kl - g*DPL - i
        const int ebase = D - 1 + 8 * kl - g * DPL;
        uint64_t pw[VW::NW];
        uint64_t pcl;
        auto fetch = [&]() {
#pragma unroll
            for (int j = 0; j < VW::NW; j++) pw[j] = bload_u64(rcr, (uint32_t)(woff + 512 * j));
            pcl = bload_u64(rcl, (uint32_t)coff);
        };
        fetch();
        for (int s = s_lo; s < s_hi; s++) {
#pragma unroll
            for (int j = 0; j < VW::NW; j++)
                if (j < VW::NW - 1 || lane + 64 * j < VW::ENTRIES) win[wdst[j]] = pw[j];
            const uint64_t clv = pcl;
            __builtin_amdgcn_wave_barrier();
            woff += wstep;
            coff += wstep;
            fetch();  // next step (one redundant fetch after the last step)
            uint32_t C[DPL], Ln[DPL];
            if constexpr (DPL % 8 == 0) {
                // ebase = 7 (mod 8): phys(ebase - i) = (7 - i%8)*S + ebase/8 - i/8 -> immediate offsets
                const uint64_t* wl = win + (ebase >> 3);
#pragma unroll
                for (int i = 0; i < DPL; i++)
                    C[i] = (uint32_t)__popcll(clv ^ wl[(7 - (i & 7)) * VW::S - (i >> 3)]);
            } else {
#pragma unroll
                for (int i = 0; i < DPL; i++) C[i] = (uint32_t)__popcll(clv ^ win[VW::phys(ebase - i)]);
            }
            const uint32_t mn = sgm_step<VL, DPL>(Lp, minLp, C, P1, P2, Ln);
            const bool active = line_ok && x1 >= 0 && x1 < W1;
            bstore_n<LT, DPL, PATHS_STORE_AUX>(rout, active ? (uint32_t)off : kOOB, Ln);
#pragma unroll
            for (int i = 0; i < DPL; i++) Lp[i] = Ln[i];
            minLp = mn;
            reset_entering();
            off += step_bytes;
            x1 += dx;
            __builtin_amdgcn_wave_barrier();
        }
    } else {
        // u16 cost volume: a ring of VPF16 loads in flight, as the horizontal lines keep (one
        // load ahead made every step wait for a memory round trip; loads and the previous steps'
        // stores retire in order).  sgbm5 per-direction, 8 KITTI pairs: paths 202.9 -> 190.2 us
        // per pair at 4 (8: 194.3).  The last round runs up to VPF16 - 1 steps past s_hi with
        // nothing loaded or stored (their state is never used).
#ifndef VPF16
#define VPF16 4
#endif
        constexpr int PF = VPF16;
        const rsrc_t rc = make_rsrc(a.cost + (size_t)pair * a.cost_pair, (uint64_t)H * W1 * D * 2);
        int coff = off / (int)sizeof(LT) * 2;
        const int cstep = step_bytes / (int)sizeof(LT) * 2;
        const int nsteps = s_hi - s_lo;
        RawU16<DPL> ring[PF];
#pragma unroll
        for (int k = 0; k < PF; k++) {
            // out-of-range offsets read 0 (inactive lines only)
            ring[k].load(rc, k < nsteps ? (uint32_t)(coff + k * cstep) : kOOB);
            asm volatile("" ::: "memory");  // issue order = slot order (see the horizontal ring)
        }
        for (int s0 = 0; s0 < nsteps; s0 += PF) {
#pragma unroll
            for (int k = 0; k < PF; k++) {
                const int s = s0 + k;
                uint32_t C[DPL], Ln[DPL];
#pragma unroll
                for (int j = 0; j < RawU16<DPL>::WORDS; j++) asm volatile("" : "+v"(ring[k].w[j]) : "v"(minLp));
                ring[k].unpack(C);
#pragma unroll
                for (int i = 0; i < DPL; i++) asm volatile("" : "+v"(C[i])::"memory");
                ring[k].load(rc, s + PF < nsteps ? (uint32_t)(coff + PF * cstep) : kOOB);
                coff += cstep;
                const uint32_t mn = sgm_step<VL, DPL>(Lp, minLp, C, P1, P2, Ln);
                const bool active = line_ok && s < nsteps && x1 >= 0 && x1 < W1;
                bstore_n<LT, DPL, PATHS_STORE_AUX>(rout, active ? (uint32_t)off : kOOB, Ln);
#pragma unroll
                for (int i = 0; i < DPL; i++) Lp[i] = Ln[i];
                minLp = mn;
                reset_entering();
                off += step_bytes;
                x1 += dx;
            }
        }
    }
}

// LDS per wave: vertical window (class-major, VWin::WORDS u64) or horizontal staging (2 x 64 u64)
template <int D, int LPW>
constexpr int lds_per_wave()
{
    return VWin<D, LPW>::WORDS > 128 ? VWin<D, LPW>::WORDS : 128;
}

// VL: lanes per vertical-family line (16 or 8); DPLV = D / VL.  FB: the sweep
// engine's guarded fallback instance (see PathsArgs::guard); a separate
// instance so the normal one carries none of its code (registers).
template <int VL, int DPLV, int LANESH, int DPLH, bool CENSUS, typename LT, bool FB = false>
__global__ void __launch_bounds__(256) k_sgm_paths(PathsArgs a)
{
    constexpr int PW = lds_per_wave<VL * DPLV, 64 / VL>();
    __shared__ __attribute__((aligned(16))) uint64_t lds[4 * PW];
    uint64_t* mine = lds + (threadIdx.x >> 6) * PW;
    auto block = [&](int pair, int b) {
        if (b < 2 * a.hblocks) {
            if (!(a.dbg & 1)) horz_family<LANESH, DPLH, CENSUS, LT>(a, pair, b, mine);
        } else {
            if (!(a.dbg & 2)) vert_family<VL, DPLV, CENSUS, LT>(a, pair, b - 2 * a.hblocks, mine);
        }
    };
    if constexpr (FB) {  // wave-private LDS only: no barrier between blocks
        if (guard_clear(a.guard)) return;
        for (int v = blockIdx.x; v < a.nblocks * a.npairs; v += gridDim.x) block(v / a.nblocks, v % a.nblocks);
    } else {
        block(blockIdx.y, blockIdx.x);
    }
}

// --------------------------------------------------------------------- WTA
// One workgroup of NT threads per (row, pair); a 16-lane group per pixel.
struct WtaArgs {
    const uint8_t* L;
    size_t slot_bytes, L_pair_bytes;
    int nslots;
    int H, W, width1, D, minD, minX1, uniq, disp12;
    int Dv;         // real disparities (< D only for a padded cost volume: planes >= Dv are ignored)
    int16_t* disp;  // [pair][H][W] pre-median
    int16_t* wta;   // [pair][H][W] integer WTA index (best, -1 rejected / outside the domain), or null
    const uint16_t* part;  // hybrid engine: u16 S + SE + SW sums [pair][H][width1][D], or null
    size_t part_pair;      // elements
    int lane8;             // 5 paths: OpenCV's SIMD tie-break among equal minima (wta_rank)
    // sweep fallback (see PathsArgs::guard): grid-stride over H x npairs rows; the
    // launch's first workgroup counts the fallback in *fallbacks
    const uint32_t* guard;
    uint32_t* fallbacks;
    int npairs;
    // (not the fallback) the group's give-up flag: set, the row kernel writes nothing (the guarded
    // fallback, running beside it on another stream, writes the maps); null: always run
    const uint32_t* skip;
};

// The row's columns from u16 sums (the MODE 3 lines' patched partial with every path, or the
// per-direction engine's u16 volumes + partial), packed: two disparities per VOP3P instruction for the clamp, the WTA key
// and the uniqueness window (the fused sweep's form, sm_sweep.hpp), S[best -+ 1] from a row of
// S in LDS.  Same decisions as wta_row's scalar loop (sgbm5 KITTI: 26 VALU lane-ops per cell
// there, the kernel at full VALU issue).
// the packed loop's row of S per 16-lane group (one LDS array for both PAD instances)
template <int DPL, int NT>
__device__ __forceinline__ uint16_t* wta_packed_srow(int grp)
{
    __shared__ __attribute__((aligned(16))) uint16_t srow[NT / 16][16 * DPL];
    return &srow[grp][0];
}

template <int DPL, typename LT, int NT, bool PART_ONLY, bool PAD>
__device__ __forceinline__ void wta_packed_cols(const WtaArgs& a, const int y, const int pair, uint32_t* key2, int* drow,
                                              int16_t* brow)
{
    constexpr int NP = DPL / 2;
    const int D = a.D, minD = a.minD, minX1 = a.minX1, Dv = a.Dv;
    const int g = threadIdx.x & 15, grp = threadIdx.x >> 4;
    constexpr bool pad = PAD;  // Dv < D (a padded cost volume); a template parameter: no selects per word
    const int ku = 100 - a.uniq;
    uint32_t rk[DPL], padm[NP], dpk[NP];
#pragma unroll
    for (int i = 0; i < DPL; i++) rk[i] = wta_rank(g * DPL + i, a.lane8);
#pragma unroll
    for (int j = 0; j < NP; j++) {
        const int d0 = g * DPL + 2 * j;
        padm[j] = (d0 >= Dv ? 0x0000FFFFu : 0u) | (d0 + 1 >= Dv ? 0xFFFF0000u : 0u);
        dpk[j] = (uint32_t)(d0 + 1) * 0x10001u + 0x10000u;  // d + 1 per half
    }
    // S = the u16 partial (MODE 3 lines: every path) and / or the u16 per-direction volumes
    // (k < nslots), summed saturating: min(sum, 65535) clamped at 32767 below = min(sum, 32767)
    const size_t rowo = (size_t)y * a.width1 * D + g * DPL;
    const uint16_t* P = a.part ? a.part + (size_t)pair * a.part_pair + rowo : nullptr;
    const uint16_t* Lb = sizeof(LT) == 2 ? (const uint16_t*)(a.L + (size_t)pair * a.L_pair_bytes) + rowo : nullptr;
    const size_t slot = a.slot_bytes / 2;
    const int nslots = sizeof(LT) == 2 && !PART_ONLY ? a.nslots : 0;
    constexpr int MS = PART_ONLY ? 1 : 4;  // slots in flight (the partial-only kernel keeps none)
    uint16_t* sr = wta_packed_srow<DPL, NT>(grp);
    auto ldw = [&](const uint16_t* src, uint32_t (&w)[NP]) {
        if constexpr (NP % 4 == 0) {
#pragma unroll
            for (int k = 0; k < NP / 4; k++) {
                const uint4 q = reinterpret_cast<const uint4*>(src)[k];
                w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w;
            }
        } else if constexpr (NP % 2 == 0) {
#pragma unroll
            for (int k = 0; k < NP / 2; k++) {
                const uint2 q = reinterpret_cast<const uint2*>(src)[k];
                w[2 * k] = q.x; w[2 * k + 1] = q.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < NP; k++) w[k] = reinterpret_cast<const uint32_t*>(src)[k];
        }
    };
    uint32_t tq[NP];  // partial-only: the next column's words, loaded one column ahead
    if (PART_ONLY && grp < a.width1) ldw(P + (size_t)grp * D, tq);
    for (int x = grp; x < a.width1; x += NT / 16) {
        uint32_t Sp[NP], t[MS][NP], tp[NP];
        if constexpr (PART_ONLY) {
#pragma unroll
            for (int j = 0; j < NP; j++) tp[j] = tq[j];
            if (x + NT / 16 < a.width1) ldw(P + (size_t)(x + NT / 16) * D, tq);
        } else if (P) {
            ldw(P + (size_t)x * D, tp);
        }
#pragma unroll
        for (int j = 0; j < NP; j++) Sp[j] = 0u;
        for (int k0 = 0; k0 < nslots; k0 += MS) {  // MS slots' loads in flight before their adds
#pragma unroll
            for (int k = 0; k < MS; k++)
                if (k0 + k < nslots) ldw(Lb + (size_t)(k0 + k) * slot + (size_t)x * D, t[k]);
#pragma unroll
            for (int k = 0; k < MS; k++)
                if (k0 + k < nslots) {
#pragma unroll
                    for (int j = 0; j < NP; j++) Sp[j] = pk_adds(Sp[j], t[k][j]);
                }
        }
        if (P) {
#pragma unroll
            for (int j = 0; j < NP; j++) Sp[j] = pk_adds(Sp[j], tp[j]);
        }
        uint32_t key = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < NP; j++) {
            Sp[j] = pk_min(Sp[j], 0x7FFF7FFFu);  // min(S, 32767)
            if (pad) Sp[j] |= padm[j];           // pad planes of a cost volume: never the minimum
            key = ::min(key, ::min((Sp[j] << 16) | rk[2 * j], (Sp[j] & 0xFFFF0000u) | rk[2 * j + 1]));
        }
        // (u32 stores, u16 loads of the same LDS row: the compiler barriers keep type-based
        // alias analysis from moving the loads across the stores, here and in the next column)
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < NP; j++) reinterpret_cast<uint32_t*>(sr + g * DPL)[j] = Sp[j];
        asm volatile("" ::: "memory");
        key = row16_min(key);
        const uint32_t minS = key >> 16;
        const int best = wta_unrank(key & 0xFFFF, a.lane8);
        // uniqueness: m2 = min S outside best-1..best+1 (window entries pushed to >= 0xFFFD)
        const uint32_t bm1p = (uint32_t)best * 0x10001u;
        uint32_t m2p = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < NP; j++) {
            uint32_t t = pk_sub(dpk[j], bm1p);  // d + 1 - best: 0, 1, 2 inside the window
            t = pkw(__builtin_elementwise_sub_sat(pkv(0x00030003u), pkv(t)));
            m2p = pk_min(m2p, pk_window_push(t, Sp[j]));
        }
        const uint32_t m2 = row16_min(::min(m2p & 0xFFFFu, m2p >> 16));
        const bool bad = (int)m2 * ku < (int)minS * 100 && (!pad || m2 <= 32767u);
        if (g == 0 && !bad && minS < 32767u) {
            const int X = x + minX1;
            const int x2 = X - best - minD;
            atomicMin(&key2[x2], (minS << 16) | (uint32_t)(0xFFFF - X));
            int d16;
            if (best > 0 && best < Dv - 1) {
                const int Sm = sr[best - 1], Sq = sr[best + 1];
                d16 = best * 16 + subpix_step(Sm, Sq, (int)minS);  // C truncation
            } else {
                d16 = best * 16;
            }
            drow[X] = d16 + minD * 16;
            if (a.wta) brow[X] = (int16_t)best;
        }
    }
}

template <int DPL, typename LT, int NT, bool PART_ONLY = false>
__device__ __forceinline__ void wta_row(const WtaArgs& a, const int y, const int pair, uint32_t* smem)
{
    const int W = a.W, D = a.D, minD = a.minD, minX1 = a.minX1;
    const int maxX1 = minX1 + a.width1;
    const int INVALID = (minD - 1) * 16;
    uint32_t* key2 = smem;
    int* drow = reinterpret_cast<int*>(smem + W);
    int16_t* brow = reinterpret_cast<int16_t*>(smem + 2 * W);  // integer WTA index (only with a.wta)
    for (int i = threadIdx.x; i < W; i += NT) {
        key2[i] = 0xFFFFFFFFu;
        drow[i] = INVALID;
        if (a.wta) brow[i] = -1;
    }
    __syncthreads();
    const int g = threadIdx.x & 15;
    const int grp = threadIdx.x >> 4;
    const LT* __restrict__ Lb = (const LT*)(a.L + (size_t)pair * a.L_pair_bytes) + g * DPL;
    const size_t slot = a.slot_bytes / sizeof(LT);
    const int u = a.uniq;
    if constexpr (DPL % 2 == 0) {
        // the in-sweep lines' patched partial (PART_ONLY), or u16 direction volumes (+ partial)
        if constexpr (PART_ONLY) {
            if (a.Dv < a.D)
                wta_packed_cols<DPL, LT, NT, true, true>(a, y, pair, key2, drow, brow);
            else
                wta_packed_cols<DPL, LT, NT, true, false>(a, y, pair, key2, drow, brow);
            goto tail;
        } else if (sizeof(LT) == 2 && DPL <= 12) {  // (block-uniform; DPL 14, 16: the scalar loop's registers)
            if (a.Dv < a.D)
                wta_packed_cols<DPL, LT, NT, false, true>(a, y, pair, key2, drow, brow);
            else
                wta_packed_cols<DPL, LT, NT, false, false>(a, y, pair, key2, drow, brow);
            goto tail;
        }
    }
    for (int x = grp; x < a.width1; x += NT / 16) {
        const size_t off = ((size_t)y * a.width1 + x) * D;
        uint32_t S[DPL];
        if constexpr (sizeof(LT) == 1 && DPL % 4 == 0) {
            // SWAR: bytes split into even/odd 16-bit lanes, summed with plain
            // 32-bit adds (8 slots x 255 < 65536, no carry between lanes);
            // all slots' loads are issued before the first add
            constexpr int NW = DPL / 4;
            uint32_t w[8][NW];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (k < a.nslots) {
                    const uint32_t* src = reinterpret_cast<const uint32_t*>(Lb + (size_t)k * slot + off);
#pragma unroll
                    for (int j = 0; j < NW; j++) {
#if WTA_NT_LOADS
                        w[k][j] = __builtin_nontemporal_load(src + j);
#else
                        w[k][j] = src[j];
#endif
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < NW; j++) w[k][j] = 0;
                }
            }
            uint32_t ev[NW], od[NW];
#pragma unroll
            for (int j = 0; j < NW; j++) ev[j] = od[j] = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) {
#pragma unroll
                for (int j = 0; j < NW; j++) {
                    ev[j] += w[k][j] & 0x00FF00FFu;
                    od[j] += (w[k][j] >> 8) & 0x00FF00FFu;
                }
            }
#pragma unroll
            for (int j = 0; j < NW; j++) {
                S[4 * j + 0] = ev[j] & 0xFFFF;
                S[4 * j + 1] = od[j] & 0xFFFF;
                S[4 * j + 2] = ev[j] >> 16;
                S[4 * j + 3] = od[j] >> 16;
            }
        } else {
#pragma unroll
            for (int i = 0; i < DPL; i++) S[i] = 0;
            for (int k = 0; k < a.nslots; k++) {
                uint32_t t[DPL];
                load_n<DPL>(Lb + (size_t)k * slot + off, t);
#pragma unroll
                for (int i = 0; i < DPL; i++) S[i] += t[i];
            }
        }
        if (a.part) {  // wave-uniform
            uint32_t t[DPL];
            load_n<DPL>(a.part + (size_t)pair * a.part_pair + off + g * DPL, t);
#pragma unroll
            for (int i = 0; i < DPL; i++) S[i] += t[i];
        }
        uint32_t key = 0xFFFFFFFFu;
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            S[i] = min(S[i], 32767u);
            if (g * DPL + i >= a.Dv) S[i] = 0xFFFFu;  // pad planes of a cost volume: never the minimum
            key = min(key, (S[i] << 16) | wta_rank(g * DPL + i, a.lane8));
        }
        key = row16_min(key);
        const int minS = (int)(key >> 16), best = wta_unrank(key & 0xFFFF, a.lane8);
        uint32_t bad = 0, nb = 0;
#pragma unroll
        for (int i = 0; i < DPL; i++) {
            const int d = g * DPL + i;
            const int dd = best - d;
            bad |= ((int)S[i] * (100 - u) < minS * 100 && (dd > 1 || dd < -1) && d < a.Dv) ? 1u : 0u;
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
            if (best > 0 && best < a.Dv - 1) {
                const int Sm = (int)(nb & 0xFFFF), Sq = (int)(nb >> 16);
                d16 = best * 16 + subpix_step(Sm, Sq, minS);  // C truncation
            } else {
                d16 = best * 16;
            }
            drow[X] = d16 + minD * 16;
            if (a.wta) brow[X] = (int16_t)best;
        }
    }
tail:
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

// PART_ONLY: a.nslots == 0 and a.part set (the MODE 3 lines' 5-path partial), its own
// instance so the row loop keeps the registers of two workgroups per CU
template <int DPL, typename LT, int NT, bool FB = false, bool PART_ONLY = false>
__global__ void __launch_bounds__(NT) k_wta(WtaArgs a)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    if constexpr (FB) {  // sweep fallback: grid-stride over the rows of every pair
        if (guard_clear(a.guard)) return;
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(a.fallbacks, 1u);
        for (int v = blockIdx.x; v < a.H * a.npairs; v += gridDim.x) {
            wta_row<DPL, LT, NT, PART_ONLY>(a, v % a.H, v / a.H, smem);
            __syncthreads();  // the next row reuses the shared row buffers
        }
    } else {
        if (a.skip && __hip_atomic_load(a.skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
        wta_row<DPL, LT, NT, PART_ONLY>(a, blockIdx.x, blockIdx.y, smem);
    }
}

}  // namespace smk
