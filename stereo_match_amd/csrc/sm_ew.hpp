// sm_ew.hpp — horizontal (E, W) path volumes for the fused-sweep engine.
//
// The two horizontal directions are the longest serial chains of SGM: one
// image row, width1 steps, each step's recurrence needing the previous step's
// minimum over all D disparities.  The per-direction engine's row lines
// (sm_paths.hpp) run them in u32 registers with 16 lanes per line, and at a
// handful of waves per SIMD the chain latency (about 20 dependent VALU/DPP
// operations per step) is what the kernel waits on.  Here a line has VL lanes
// holding D/VL disparities each as D/(2 VL) u16 pairs (sm_pk.hpp): every step
// is NP independent packed recurrences (8 VOP3P per two disparities) followed
// by one in-lane min tree and log2(VL) DPP steps, so one wave per SIMD keeps
// the VALU issuing; the cost row is streamed through a PF-deep ring of
// whole-slice loads.
//
// Output layout and values are exactly those of the per-direction engine's
// horizontal family: slot 0 = E (x ascending), slot 1 = W, [H][width1][D] of LT.
#pragma once
#include "sm_pk.hpp"
#include "sm_sweep_host.hpp"

namespace smk {

#ifndef SWEEP_STREAM_AUX
#define SWEEP_STREAM_AUX 2  // cache policy of the E/W stores: nt (sm_sweep.hpp)
#endif
#ifndef EW_H16
#define EW_H16 1  // census: f16 form of the packed recurrence
#endif
#ifndef EW_STEPN
#define EW_STEPN 1  // the step's words stage by stage (no wait states between dependent VOP3P ops)
#endif

// grid (2 * a.nrb, pairs), 64 * a.wpb threads: workgroup b < nrb runs E lines, the rest W;
// each wave owns LPW = 64 / VL consecutive rows.
template <int VL, int NP, typename CT, typename LT, int PF>
__global__ void __launch_bounds__(256) k_ew(EwArgs a)
{
    constexpr int LPW = 64 / VL, DPL = 2 * NP, D = VL * DPL;
    constexpr int CB = DPL * (int)sizeof(CT);  // cost bytes per lane and step
    // issue priority against the down sweep's waves sharing the SIMDs (SM_TUNE_EW_PRIO; the
    // sweep's hand-off chain runs at 3, its other work at 2)
    switch (a.prio) {
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    case 3: __builtin_amdgcn_s_setprio(3); break;
    default: break;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane % VL, kl = lane / VL;
    const int dir = (int)blockIdx.x >= a.nrb ? 1 : 0;
    const int H = a.H, W1 = a.W1;
    const int y0 = (((int)blockIdx.x - dir * a.nrb) * a.wpb + wave) * LPW;
    if (y0 >= H) return;  // wave-uniform
    const bool line_ok = y0 + kl < H;
    const int y = min(y0 + kl, H - 1);
    const size_t pair = blockIdx.y;
    const uint64_t cells = (uint64_t)H * W1 * D;
    const rsrc_t rc = make_rsrc(a.cost + pair * a.cost_pair, cells * sizeof(CT));
    const rsrc_t ro = make_rsrc(a.out + pair * a.out_pair + (size_t)dir * a.out_slot, cells * sizeof(LT));
    // element index of this lane's slice, stepped along the row modulo 2^32 (a per-pair
    // volume stays below 2^32 bytes: the host's kMaxRecords guard)
    const uint32_t estep = dir ? (uint32_t)(-D) : (uint32_t)D;
    uint32_t e = ((uint32_t)y * (uint32_t)W1 + (uint32_t)(dir ? W1 - 1 : 0)) * (uint32_t)D + (uint32_t)(g * DPL);
    const uint32_t P1p = (uint32_t)a.P1 * 0x10001u, P2p = (uint32_t)a.P2 * 0x10001u;
    // census (u8 costs): the f16 form of the recurrence (sm_pk.hpp sweep_step2)
    constexpr bool H16 = sizeof(CT) == 1 && EW_H16;
    constexpr uint32_t EDGE = H16 ? 0x7BFF7BFFu : (kBig | (kBig << 16));
    const uint32_t eL = g == 0 ? EDGE : 0u, eR = g == VL - 1 ? EDGE : 0u;

    RawBytes<CB> ring[PF];
#pragma unroll
    for (int k = 0; k < PF; k++) {
        ring[k].load(rc, k < W1 ? (e + (uint32_t)k * estep) * (uint32_t)sizeof(CT) : kOOB);
        asm volatile("" ::: "memory");  // issue order = slot order (sm_paths.hpp horizontal ring)
    }
    uint32_t Lp[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) Lp[k] = 0;
    uint32_t minLp = 0;
    for (int s0 = 0; s0 < W1; s0 += PF) {
#pragma unroll
        for (int k = 0; k < PF; k++) {
            const int s = s0 + k;
            // the slot is read only after the previous step (no hoisted unpacks whose
            // waits would cover the younger slots), and its values are materialised
            // before the refill is issued (no ring rotation by moves at the back-edge)
#pragma unroll
            for (int j = 0; j < RawBytes<CB>::WORDS; j++) asm volatile("" : "+v"(ring[k].w[j]) : "v"(minLp));
            uint32_t C[NP];
            unpack_ct_pk<CT, DPL>(ring[k], C);
#pragma unroll
            for (int i = 0; i < NP; i++) asm volatile("" : "+v"(C[i])::"memory");
            ring[k].load(rc, s + PF < W1 ? (e + (uint32_t)PF * estep) * (uint32_t)sizeof(CT) : kOOB);
            uint32_t Ln[NP], mn;
            if constexpr (EW_STEPN) {  // stage-wise over the words (sm_pk.hpp sweep_step2n)
                uint32_t Lp1[1][NP], m1[1] = {minLp}, C1[1][NP], Ln1[1][NP], mn1[1];
#pragma unroll
                for (int i = 0; i < NP; i++) {
                    Lp1[0][i] = Lp[i];
                    C1[0][i] = C[i];
                }
                sweep_step2n<VL, NP, H16, 1>(Lp1, m1, C1, P1p, P2p, eL, eR, Ln1, mn1);
#pragma unroll
                for (int i = 0; i < NP; i++) Ln[i] = Ln1[0][i];
                mn = mn1[0];
            } else {
                mn = sweep_step2<VL, NP, H16>(Lp, minLp, C, P1p, P2p, eL, eR, Ln);  // minLp replicated
            }
            store_pk<LT, NP, SWEEP_STREAM_AUX>(ro, (line_ok && s < W1) ? e * (uint32_t)sizeof(LT) : kOOB, Ln);
            e += estep;
#pragma unroll
            for (int i = 0; i < NP; i++) Lp[i] = Ln[i];
            minLp = mn;
        }
    }
}

// columns of a repaired segment whose cost and partial slices load together (one memory round
// trip per RC columns on the walks' serial chain; the pass runs ~3 waves per SIMD, so the
// registers are there)
// timing ablation (results wrong where a walk never met): no phase-B carries
#ifndef EW_PATCH_NO_CARRY
#define EW_PATCH_NO_CARRY 0
#endif
#ifndef EW_PATCH_B64
#define EW_PATCH_B64 1  // phase B's carried walks on 64-lane lines where D % 128 == 0
#endif
// (0: by cost type — census 8, u16 16: census8 E/W patch 6.9 -> 6.4 us per pair at 8, 9.5 at 32;
// sgbm5 17.6 at 16, 20.0 at 8, 21.5 at 32)
#ifndef EW_PATCH_RC
#define EW_PATCH_RC 0
#endif
// ---------------------------------------------------------------------------
// Patch pass after a MODE 3 sweep (sm_sweep.hpp line waves).  Strip k's E line
// started from the zero state `ewarm` columns before the strip, so its values are exact from
// the column where its state met the true one.  Stored per (row, strip, direction): s_k, the
// state entering the strip, and e_k, the state at its far end.  Along a row's path order a
// strip is exact iff the state truly entering it equals the one its values came from; the
// first strip of each path enters from outside the domain (exact).
//   check: strip k is flagged where s_k != e_{k-1};
//   phase A (the wave's LPW lines in parallel, one flagged strip each): recompute strip k
//     from e_{k-1} beside its speculative trajectory from s_k and add (true - speculative)
//     to the partial column by column until the two trajectories are equal (every later
//     value is then equal).  Exact when strip k-1 is exact at its far end, i.e. unless
//     strip k-1's own walk never met;
//   phase B (rare; one line, in path order): after a strip whose walk never met (its end
//     state c_k, kept in its s_k slot), the next strips' values came from e_{k-1} while the
//     true state is the carried one: the same walk with (applied, true) = (e_{k-1}, carried)
//     until a strip's trajectories meet.
// E then W (the two directions touch the same partial cells), four rows per workgroup.
// u16 costs: the MODE 3 partial saturates at 0xFFFF; a cell below that holds the exact sum
// (every term >= 0), one at 0xFFFF stays there (the true five-path sum is then still
// >= 65535 - 2 * 16383 > 32767, so the WTA's 32767 clamp sees the same value).
// ATOM (the host's choice where 5 x path_max < 65536, so no partial cell saturates): the
// corrections are u32 atomic adds of (true - applied) per u16 pair as one signed addend, exact
// in any order while every half stays a valid sum (band patch argument), so the partial is never
// read and E and W of a row run in two waves side by side (twice the waves, no E -> W order).
template <int VL, int NP, typename CT, bool ATOM = false>
__global__ void __launch_bounds__(256) k_ew_patch(EwPatchArgs a)
{
    constexpr int LPW = 64 / VL, DPL = 2 * NP, D = VL * DPL;
    constexpr int CB = DPL * (int)sizeof(CT);
    constexpr bool H16 = sizeof(CT) == 1 && EW_H16;
    constexpr bool SAT = sizeof(CT) == 2;
    constexpr uint32_t EDGE = H16 ? 0x7BFF7BFFu : (kBig | (kBig << 16));
    // check phase: line kl of the wave checks the strips i = 1 + kl + LPW * u (u < KU) of a
    // chunk of LPW * KU path positions, all loads of a chunk in flight together
    constexpr int KU = 8;
    constexpr int CHUNK = LPW * KU;
    constexpr int RC = EW_PATCH_RC ? EW_PATCH_RC : sizeof(CT) == 1 ? 8 : 16;  // columns of a repaired segment loaded together
    if (a.guard && __hip_atomic_load(a.guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane % VL, kl = lane / VL;
    const int yw = (int)blockIdx.x * 4 + wave;  // one wave per image row (ATOM: per row and direction)
    const int y = ATOM ? yw >> 1 : yw;           // (wave-uniform)
    const int dir0 = ATOM ? (yw & 1) : 0, dir1 = ATOM ? dir0 + 1 : 2;
    const size_t pair = blockIdx.y;
    const int H = a.H, W1 = a.W1, nwg = a.nwg, CW = a.cw;
    if (y >= H) return;
    const uint64_t cells = (uint64_t)H * W1 * D;
    const rsrc_t rc = make_rsrc(a.cost + pair * a.cost_pair, cells * sizeof(CT));
    const rsrc_t rp = make_rsrc((const uint8_t*)a.part + pair * a.part_pair, cells * 2);
    uint32_t* const pw = reinterpret_cast<uint32_t*>((uint8_t*)a.part + pair * a.part_pair);  // (ATOM)
    // (second - first) per u16 half as one signed 32-bit addend, added atomically where nonzero
    auto atom_add = [&](uint32_t word, uint32_t first, uint32_t second) {
        const int lo = (int)(second & 0xFFFFu) - (int)(first & 0xFFFFu);
        const int hi = (int)(second >> 16) - (int)(first >> 16);
        const uint32_t add = (uint32_t)(hi * 65536 + lo);
        if (add) __hip_atomic_fetch_add(pw + word, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    const rsrc_t rs = make_rsrc(a.st + pair * a.st_pair, a.st_pair);
    const uint32_t P1p = (uint32_t)a.P1 * 0x10001u, P2p = (uint32_t)a.P2 * 0x10001u;
    const uint32_t eL = g == 0 ? EDGE : 0u, eR = g == VL - 1 ? EDGE : 0u;
    auto soff = [&](int k, int dir, int which) -> uint32_t {
        return (((((uint32_t)y * (uint32_t)nwg + (uint32_t)k) * 2u + (uint32_t)dir) * 2u + (uint32_t)which) *
                    (uint32_t)D + (uint32_t)(g * DPL)) * (uint32_t)sizeof(CT);
    };
    auto cell = [&](int c) -> uint32_t { return ((uint32_t)y * (uint32_t)W1 + (uint32_t)c) * (uint32_t)D + (uint32_t)(g * DPL); };
    auto line_all = [&](bool ok) -> bool { return group_min<VL>(ok ? 1u : 0u) != 0u; };
    auto same_state = [&](const uint32_t (&x)[NP], const uint32_t (&z)[NP]) -> bool {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < NP; i++) ok &= x[i] == z[i];
        return line_all(ok);
    };
    // the recurrence's replicated minimum (m | m << 16) of a stored state
    auto state_min = [&](const uint32_t (&x)[NP]) -> uint32_t {
        uint32_t m = x[0];
#pragma unroll
        for (int i = 1; i < NP; i++) m = pk_min(m, x[i]);
        m = ::min(m & 0xFFFFu, m >> 16);
        return group_min<VL>(m) * 0x10001u;
    };
    auto load_state = [&](uint32_t off, uint32_t (&v)[NP]) {
        RawBytes<CB> b;
        b.load(rs, off);
        unpack_ct_pk<CT, DPL>(b, v);
    };
    // the values of strip k (direction dir) came from the trajectory entering at A (the state
    // at aoff); the true one enters at T (the state at toff, or the caller's registers for
    // toff == kOOB): add (true - applied) to the partial until the two meet.  Returns 1 met,
    // 0 never met (T then holds the true trajectory's state at the strip's far end), 2 with
    // `check` where A == T (nothing to do).  Line-divergent.
    auto walk = [&](int k, int dir, uint32_t aoff, uint32_t toff, uint32_t (&T)[NP], bool check) -> int {
        const int x0 = k * CW, ncol = ::min(CW, W1 - x0);  // W: every repaired strip is full
        // columns in chunks of RC: the chunk's costs and partial slices load together (the
        // first chunk's beside the state loads: one memory round trip for both)
        RawBytes<CB> cc[RC];
        RawBytes<DPL * 2> pb[RC];
        auto issue1 = [&](int u, int o) {  // slot u <- column o of the walk
            const int c = dir ? x0 + CW - 1 - o : x0 + o;
            cc[u].load(rc, o < ncol ? cell(c) * (uint32_t)sizeof(CT) : kOOB);
            if constexpr (!ATOM) pb[u].load(rp, o < ncol ? cell(c) * 2u : kOOB);
        };
        auto issue = [&](int o0) {
#pragma unroll
            for (int u = 0; u < RC; u++) issue1(u, o0 + u);
        };
        issue(0);
        uint32_t A[NP];
        load_state(aoff, A);
        if (toff != kOOB) load_state(toff, T);
        if (check && same_state(A, T)) return 2;
        uint32_t Lq[2][NP], mq[2];
#pragma unroll
        for (int q = 0; q < NP; q++) {
            Lq[0][q] = A[q];
            Lq[1][q] = T[q];
        }
        mq[0] = state_min(Lq[0]);
        mq[1] = state_min(Lq[1]);
        bool met = false;
        for (int o0 = 0; o0 < ncol && !met; o0 += RC) {
            if (o0 > 0) issue(o0);
#pragma unroll
            for (int u = 0; u < RC; u++) {  // (no break: the loop must unroll)
                const int o = o0 + u;
                if (o >= ncol || met) continue;
                const int c = dir ? x0 + CW - 1 - o : x0 + o;
                uint32_t C2[2][NP], Ln[2][NP], mn[2], pv_[NP];
                unpack_ct_pk<CT, DPL>(cc[u], C2[0]);
#pragma unroll
                for (int q = 0; q < NP; q++) pv_[q] = ATOM ? 0u : pb[u].w[q];
#pragma unroll
                for (int q = 0; q < NP; q++) C2[1][q] = C2[0][q];
                sweep_step2n<VL, NP, H16, 2>(Lq, mq, C2, P1p, P2p, eL, eR, Ln, mn);
                if (same_state(Ln[0], Ln[1])) {
                    met = true;
                    continue;
                }
                if constexpr (ATOM) {
#pragma unroll
                    for (int q = 0; q < NP; q++) atom_add(cell(c) / 2u + (uint32_t)q, Ln[0][q], Ln[1][q]);
                }
                uint32_t P[NP];
#pragma unroll
                for (int q = 0; q < NP && !ATOM; q++) {
                    if constexpr (SAT) {
                        // a half pv < 0xFFFF is the exact sum, pv >= sv: (pv - sv) + tv saturating;
                        // pv == 0xFFFF stays (sat: 0xFFFF exactly there, from pv + 1 wrapping to 0)
                        const uint32_t pv = pv_[q];
                        const uint32_t x = pk_adds(pk_sub(pv, Ln[0][q]), Ln[1][q]);
                        const uint32_t sat = pk_sub(pk_min(pk_add(pv, 0x00010001u), 0x00010001u), 0x00010001u);
                        P[q] = pkw(__builtin_elementwise_max(pkv(x), pkv(sat)));
                    } else {  // census: every sum < 2^11, the u16 wrap is exact
                        P[q] = pk_add(pk_sub(pv_[q], Ln[0][q]), Ln[1][q]);
                    }
                }
                if constexpr (!ATOM) bstore_n<uint32_t, NP>(rp, cell(c) * 2u, P);
#pragma unroll
                for (int q = 0; q < NP; q++) {
                    Lq[0][q] = Ln[0][q];
                    Lq[1][q] = Ln[1][q];
                }
                mq[0] = mn[0];
                mq[1] = mn[1];
            }
        }
        if (!met) {  // the true far-end state, in the min-0 form of the stored boundary states
#pragma unroll
            for (int q = 0; q < NP; q++) T[q] = pk_sub(Lq[1][q], mq[1]);
        }
        return met ? 1 : 0;
    };
    // phase B on the whole wave: 64-lane lines (D % 128 == 0), DPLW disparities per lane, so a
    // carried walk's serial step is a quarter of a 16-lane line's per-lane work
    constexpr int DPLW = D % 128 == 0 ? D / 64 : 2, NPW = DPLW / 2;
    constexpr int CBW = DPLW * (int)sizeof(CT);
    auto soff64 = [&](int k, int dir, int which) -> uint32_t {
        return (((((uint32_t)y * (uint32_t)nwg + (uint32_t)k) * 2u + (uint32_t)dir) * 2u + (uint32_t)which) *
                    (uint32_t)D + (uint32_t)(lane * DPLW)) * (uint32_t)sizeof(CT);
    };
    auto cell64 = [&](int c) -> uint32_t {
        return ((uint32_t)y * (uint32_t)W1 + (uint32_t)c) * (uint32_t)D + (uint32_t)(lane * DPLW);
    };
    auto load_state64 = [&](uint32_t off, uint32_t (&v)[NPW]) {
        RawBytes<CBW> b;
        b.load(rs, off);
        unpack_ct_pk<CT, DPLW>(b, v);
    };
    auto same_state64 = [&](const uint32_t (&x)[NPW], const uint32_t (&z)[NPW]) -> bool {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < NPW; i++) ok &= x[i] == z[i];
        return __all(ok);
    };
    auto state_min64 = [&](const uint32_t (&x)[NPW]) -> uint32_t {
        uint32_t m = x[0];
#pragma unroll
        for (int i = 1; i < NPW; i++) m = pk_min(m, x[i]);
        m = ::min(m & 0xFFFFu, m >> 16);
        return Line<64>::min(m) * 0x10001u;
    };
    auto walk64 = [&](int k, int dir, uint32_t aoff, uint32_t toff, uint32_t (&T)[NPW], bool check) -> int {
        const int x0 = k * CW, ncol = ::min(CW, W1 - x0);  // W: every repaired strip is full
        // columns in chunks of RC: the chunk's costs and partial slices load together (the
        // first chunk's beside the state loads: one memory round trip for both)
        RawBytes<CBW> cc[RC];
        RawBytes<DPLW * 2> pb[RC];
        auto issue1 = [&](int u, int o) {  // slot u <- column o of the walk
            const int c = dir ? x0 + CW - 1 - o : x0 + o;
            cc[u].load(rc, o < ncol ? cell64(c) * (uint32_t)sizeof(CT) : kOOB);
            if constexpr (!ATOM) pb[u].load(rp, o < ncol ? cell64(c) * 2u : kOOB);
        };
        auto issue = [&](int o0) {
#pragma unroll
            for (int u = 0; u < RC; u++) issue1(u, o0 + u);
        };
        issue(0);
        uint32_t A[NPW];
        load_state64(aoff, A);
        if (toff != kOOB) load_state64(toff, T);
        if (check && same_state64(A, T)) return 2;
        uint32_t Lq[2][NPW], mq[2];
#pragma unroll
        for (int q = 0; q < NPW; q++) {
            Lq[0][q] = A[q];
            Lq[1][q] = T[q];
        }
        mq[0] = state_min64(Lq[0]);
        mq[1] = state_min64(Lq[1]);
        bool met = false;
        for (int o0 = 0; o0 < ncol && !met; o0 += RC) {
            if (o0 > 0) issue(o0);
#pragma unroll
            for (int u = 0; u < RC; u++) {  // (no break: the loop must unroll)
                const int o = o0 + u;
                if (o >= ncol || met) continue;
                const int c = dir ? x0 + CW - 1 - o : x0 + o;
                uint32_t C2[2][NPW], Ln[2][NPW], mn[2], pv_[NPW];
                unpack_ct_pk<CT, DPLW>(cc[u], C2[0]);
#pragma unroll
                for (int q = 0; q < NPW; q++) pv_[q] = ATOM ? 0u : pb[u].w[q];
#pragma unroll
                for (int q = 0; q < NPW; q++) C2[1][q] = C2[0][q];
                sweep_step2n<64, NPW, H16, 2>(Lq, mq, C2, P1p, P2p, 0u, 0u, Ln, mn);
                if (same_state64(Ln[0], Ln[1])) {
                    met = true;
                    continue;
                }
                if constexpr (ATOM) {
#pragma unroll
                    for (int q = 0; q < NPW; q++) atom_add(cell64(c) / 2u + (uint32_t)q, Ln[0][q], Ln[1][q]);
                }
                uint32_t P[NPW];
#pragma unroll
                for (int q = 0; q < NPW && !ATOM; q++) {
                    if constexpr (SAT) {
                        // a half pv < 0xFFFF is the exact sum, pv >= sv: (pv - sv) + tv saturating;
                        // pv == 0xFFFF stays (sat: 0xFFFF exactly there, from pv + 1 wrapping to 0)
                        const uint32_t pv = pv_[q];
                        const uint32_t x = pk_adds(pk_sub(pv, Ln[0][q]), Ln[1][q]);
                        const uint32_t sat = pk_sub(pk_min(pk_add(pv, 0x00010001u), 0x00010001u), 0x00010001u);
                        P[q] = pkw(__builtin_elementwise_max(pkv(x), pkv(sat)));
                    } else {  // census: every sum < 2^11, the u16 wrap is exact
                        P[q] = pk_add(pk_sub(pv_[q], Ln[0][q]), Ln[1][q]);
                    }
                }
                if constexpr (!ATOM) bstore_n<uint32_t, NPW>(rp, cell64(c) * 2u, P);
#pragma unroll
                for (int q = 0; q < NPW; q++) {
                    Lq[0][q] = Ln[0][q];
                    Lq[1][q] = Ln[1][q];
                }
                mq[0] = mn[0];
                mq[1] = mn[1];
            }
        }
        if (!met) {  // (min-0 form, as above)
#pragma unroll
            for (int q = 0; q < NPW; q++) T[q] = pk_sub(Lq[1][q], mq[1]);
        }
        return met ? 1 : 0;
    };
    // OR over the wave's lines (their first lanes) of a per-line 64-bit mask
    auto lines_or = [&](uint64_t v) -> uint64_t {
        uint64_t m = 0;
#pragma unroll
        for (int l = 0; l < LPW; l++) {
            const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l * VL);
            const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l * VL);
            m |= ((uint64_t)hi << 32) | lo;
        }
        return m;
    };
    // the other lanes' partial / state stores land before this wave's later loads of the same
    // cells (one wave: workgroup scope, i.e. vmcnt(0); agent scope would write back the L2)
    auto order_partial = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    // phase A's open strips (walk never met), one bit per path position i >= 1
    __shared__ uint64_t openm[4][kPatchMaxChunks];
    uint32_t nfix = 0, nopen = 0;  // walks (per line), open strips (wave-uniform)
    for (int dir = dir0; dir < dir1; dir++) {  // 0 = E (strips in x order), 1 = W (reverse)
        auto strip_of = [&](int i) { return dir ? nwg - 1 - i : i; };  // path position -> strip
        int first_open = nwg;  // wave-uniform
        for (int i0 = 1, ch = 0; i0 < nwg; i0 += CHUNK, ch++) {
            // ---- check: does the state entering strip i equal the end state stored by strip i - 1?
            RawBytes<CB> sb[KU], eb[KU];
#pragma unroll
            for (int u = 0; u < KU; u++) {
                const int i = i0 + kl + LPW * u;
                sb[u].load(rs, i < nwg ? soff(strip_of(i), dir, 0) : kOOB);
                eb[u].load(rs, i < nwg ? soff(strip_of(i - 1), dir, 1) : kOOB);
            }
            uint64_t bad = 0;  // bit i - i0: strip i's speculative start differs
#pragma unroll
            for (int u = 0; u < KU; u++) {
                bool ok = true;
#pragma unroll
                for (int q = 0; q < RawBytes<CB>::WORDS; q++) ok &= sb[u].w[q] == eb[u].w[q];
                ok = line_all(ok);
                if (!ok && i0 + kl + LPW * u < nwg) bad |= 1ull << (kl + LPW * u);
            }
            const uint64_t m = lines_or(bad);  // wave-uniform
            uint64_t open = 0;
            // ---- phase A: the flagged strips in rounds of LPW, line kl takes the round's kl-th
            uint64_t rest = m;
            while (rest) {
                int mine = -1;
#pragma unroll
                for (int l = 0; l < LPW; l++) {
                    if (rest && l == kl) mine = __builtin_ctzll(rest);
                    if (rest) rest &= rest - 1;
                }
                if (mine >= 0) {
                    const int i = i0 + mine, k = strip_of(i);
                    uint32_t T[NP];
                    nfix++;
                    if (walk(k, dir, soff(k, dir, 0), soff(strip_of(i - 1), dir, 1), T, false) == 0) {
                        // c_k, the true trajectory's far-end state, replaces s_k (read only above)
                        store_pk<CT, NP>(rs, soff(k, dir, 0), T);
                        open |= 1ull << mine;
                    }
                }
            }
            open = lines_or(open);
            nopen += (uint32_t)__builtin_popcountll(open);
            if (lane == 0) openm[wave][ch] = open;
            if (open && first_open == nwg) first_open = i0 + __builtin_ctzll(open);
        }
        if (first_open < nwg && !EW_PATCH_NO_CARRY && D % 128 == 0 && EW_PATCH_B64) {
            // ---- phase B on 64-lane lines (the same walk, the whole wave)
            order_partial();  // the other lanes' partial and c_k stores
            bool carry = false;
            uint32_t T[NPW];
#pragma unroll
            for (int q = 0; q < NPW; q++) T[q] = 0;
            for (int i = first_open; i < nwg; i++) {
                const int k = strip_of(i);
                if (carry) {
                    const int r = walk64(k, dir, soff64(strip_of(i - 1), dir, 1), kOOB, T, true);
                    nfix += r != 2 && kl == 0;
                    if (r != 0) carry = false;
                }
                const bool open_i = ((openm[wave][(i - 1) / CHUNK] >> ((i - 1) % CHUNK)) & 1ull) != 0;
                if (!carry && open_i) {
                    load_state64(soff64(k, dir, 0), T);
                    carry = true;
                }
            }
        } else if (first_open < nwg && !EW_PATCH_NO_CARRY) {
            // ---- phase B (line 0, path order from the first open strip): `carry` = the true
            // state entering strip i is T while strip i's values came from e_{i-1}
            order_partial();  // the other lanes' partial and c_k stores
            if (kl == 0) {
                bool carry = false;
                uint32_t T[NP];
#pragma unroll
                for (int q = 0; q < NP; q++) T[q] = 0;
                for (int i = first_open; i < nwg; i++) {
                    const int k = strip_of(i);
                    if (carry) {  // applied: e_{i-1}; the walk's first chunk loads beside it
                        const int r = walk(k, dir, soff(strip_of(i - 1), dir, 1), kOOB, T, true);
                        nfix += r != 2;
                        if (r != 0) carry = false;
                    }
                    // an open strip's values (from e_{i-1}, or corrected to the true trajectory
                    // where that met them) end at c_k: the next strip needs c_k, not e_k
                    const bool open_i = ((openm[wave][(i - 1) / CHUNK] >> ((i - 1) % CHUNK)) & 1ull) != 0;
                    if (!carry && open_i) {
                        load_state(soff(k, dir, 0), T);
                        carry = true;
                    }
                }
            }
        }
        if (!ATOM && dir == 0) order_partial();  // W touches the cells E wrote
    }
    if (a.fixes) {
        nfix = group_sum_u32_wave(g == 0 ? nfix : 0u);  // every line's walks
        if (lane == 0 && nfix) atomicAdd(a.fixes, (unsigned long long)nfix);
        if (lane == 0 && nopen) atomicAdd(a.fixes + 1, (unsigned long long)nopen);  // (the next counter)
    }
}

// ---- row-band patch (BandPatchArgs): grid (nbx, nband - 1, pairs), 256 threads.
// Line kl of wave w takes chain id = (blockIdx.x * 4 + w) * LPW + kl of boundary bi = blockIdx.y
// + 1: direction dir = id / W1 (0 S, 1 SE = +x, 2 SW = -x) entering band bi at column x = id % W1
// of the row above it, i.e. steps r = 0, 1, ... at column x + dx (r + 1) of row bi * band_h + r.
// Where the speculative entering state (band bi's warmup) differs from the band above's stored end
// state, the two trajectories are stepped side by side and (second - first) is added to the
// partial until they meet — across later band boundaries too, with no hand-off between walks:
// past a boundary the first trajectory continues as well, and there it is exactly the values that
// boundary's own walk (or none) left, so the contributions of all walks telescope to
// (true - speculative) in every band (u32 atomics on u16 pairs: exact whatever their order while
// no half leaves 0..65535, which the host guarantees).
template <int VL, int NP, typename CT>
__global__ void __launch_bounds__(256) k_band_patch(BandPatchArgs a)
{
    constexpr int LPW = 64 / VL, DPL = 2 * NP, D = VL * DPL, CB = DPL * (int)sizeof(CT);
    constexpr bool H16 = sizeof(CT) == 1 && EW_H16;
    constexpr uint32_t EDGE = H16 ? 0x7BFF7BFFu : (kBig | (kBig << 16));
    constexpr int RC = 8;  // chain steps whose costs load together
    if (a.guard && __hip_atomic_load(a.guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane % VL, kl = lane / VL;
    const int bi = (int)blockIdx.y + 1;
    const size_t pair = blockIdx.z;
    const int H = a.H, W1 = a.W1;
    const int y0 = bi * a.band_h;
    const int id = ((int)blockIdx.x * 4 + wave) * LPW + kl;
    const bool on = id < 3 * W1 && y0 < H;
    const int dir = on ? id / W1 : 0, x = on ? id % W1 : 0;
    const int dx = dir == 0 ? 0 : dir == 1 ? 1 : -1;
    // steps inside the image and the domain
    const int nr = !on ? 0 : dx == 0 ? H - y0 : dx > 0 ? min(H - y0, W1 - 1 - x) : min(H - y0, x);
    const uint64_t cells = (uint64_t)H * W1 * D;
    const rsrc_t rc = make_rsrc(a.cost + pair * a.cost_pair, cells * sizeof(CT));
    const rsrc_t rv = make_rsrc(a.vst + pair * a.vst_pair, a.vst_pair);
    uint32_t* part = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a.part) + pair * a.part_pair);
    const uint32_t P1p = (uint32_t)a.P1 * 0x10001u, P2p = (uint32_t)a.P2 * 0x10001u;
    const uint32_t eL = g == 0 ? EDGE : 0u, eR = g == VL - 1 ? EDGE : 0u;
    auto voff = [&](int band, int which, int col) -> uint32_t {
        return (((((uint32_t)band * 2u + (uint32_t)which) * 3u + (uint32_t)dir) * (uint32_t)W1 + (uint32_t)col) *
                    (uint32_t)D + (uint32_t)(g * DPL)) * (uint32_t)sizeof(CT);
    };
    auto cost_off = [&](int r) -> uint32_t {
        return r < nr ? (((uint32_t)(y0 + r) * (uint32_t)W1 + (uint32_t)(x + dx * (r + 1))) * (uint32_t)D +
                         (uint32_t)(g * DPL)) * (uint32_t)sizeof(CT)
                      : kOOB;
    };
    auto line_all = [&](bool ok) -> bool { return group_min<VL>(ok ? 1u : 0u) != 0u; };
    auto state_min = [&](const uint32_t (&v)[NP]) -> uint32_t {
        uint32_t m = v[0];
#pragma unroll
        for (int i = 1; i < NP; i++) m = pk_min(m, v[i]);
        m = ::min(m & 0xFFFFu, m >> 16);
        return group_min<VL>(m) * 0x10001u;
    };
    RawBytes<CB> sb, tb, cc[RC];
    sb.load(rv, on ? voff(bi, 0, x) : kOOB);      // speculative: band bi's warmup
    tb.load(rv, on ? voff(bi - 1, 1, x) : kOOB);  // the band above's end
#pragma unroll
    for (int u = 0; u < RC; u++) cc[u].load(rc, cost_off(u));
    uint32_t Lq[2][NP], mq[2];
    unpack_ct_pk<CT, DPL>(sb, Lq[0]);
    unpack_ct_pk<CT, DPL>(tb, Lq[1]);
    bool same = true;
#pragma unroll
    for (int i = 0; i < NP; i++) same &= Lq[0][i] == Lq[1][i];
    same = line_all(same);
    uint32_t nfix = 0, nlong = 0;
    if (on && !same && nr > 0) {
        nfix++;
        mq[0] = state_min(Lq[0]);
        mq[1] = state_min(Lq[1]);
        const int rb = min(H, y0 + a.band_h) - y0;  // steps inside band bi
        bool met = false;
        int r0 = 0;
        for (; r0 < nr && !met; r0 += RC) {
            if (r0 > 0) {
#pragma unroll
                for (int u = 0; u < RC; u++) cc[u].load(rc, cost_off(r0 + u));
            }
#pragma unroll
            for (int u = 0; u < RC; u++) {  // (no break: the loop must unroll)
                const int r = r0 + u;
                if (r >= nr || met) continue;
                uint32_t C2[2][NP], Ln[2][NP], mn[2];
                unpack_ct_pk<CT, DPL>(cc[u], C2[0]);
#pragma unroll
                for (int q = 0; q < NP; q++) C2[1][q] = C2[0][q];
                sweep_step2n<VL, NP, H16, 2>(Lq, mq, C2, P1p, P2p, eL, eR, Ln, mn);
                bool eq = true;
#pragma unroll
                for (int q = 0; q < NP; q++) eq &= Ln[0][q] == Ln[1][q];
                if (line_all(eq)) {
                    met = true;
                    continue;
                }
                nlong |= r >= rb ? 1u : 0u;  // (a walk that crossed the next boundary)
                // (second - first) per u16 half as one signed 32-bit addend
                const size_t w0 = (((size_t)(y0 + r) * (size_t)W1 + (size_t)(x + dx * (r + 1))) * D + g * DPL) / 2;
#pragma unroll
                for (int q = 0; q < NP; q++) {
                    const int lo = (int)(Ln[1][q] & 0xFFFFu) - (int)(Ln[0][q] & 0xFFFFu);
                    const int hi = (int)(Ln[1][q] >> 16) - (int)(Ln[0][q] >> 16);
                    const uint32_t add = (uint32_t)(hi * 65536 + lo);
                    if (add) __hip_atomic_fetch_add(part + w0 + q, add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
#pragma unroll
                for (int q = 0; q < NP; q++) {
                    Lq[0][q] = Ln[0][q];
                    Lq[1][q] = Ln[1][q];
                }
                mq[0] = mn[0];
                mq[1] = mn[1];
            }
        }
    }
    if (a.fixes) {
        nfix = group_sum_u32_wave(g == 0 ? nfix : 0u);
        nlong = group_sum_u32_wave(g == 0 ? nlong : 0u);
        if (lane == 0 && nfix) atomicAdd(a.fixes, (unsigned long long)nfix);
        if (lane == 0 && nlong) atomicAdd(a.fixes + 1, (unsigned long long)nlong);
    }
}

}  // namespace smk
