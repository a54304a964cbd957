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

// ---------------------------------------------------------------------------
// Patch pass after a MODE 3 sweep (sm_sweep.hpp line waves).  Strip k's E line
// started from the zero state `ewarm` columns before the strip, so its values are exact from
// the column where its state met the true one.  Walking one row's strips in path order, the
// trusted state entering strip k is strip k-1's stored end state as long as every earlier
// strip was exact (or was repaired up to the meeting point); where the stored entering state
// of strip k differs from it, the segment is recomputed from the trusted state beside the
// speculative one (from k's stored entering state) and the partial gets (true - speculative)
// column by column until the two trajectories are equal, after which every later value is
// equal.  A segment that never meets hands its true end state to the next strip.  One line of
// VL lanes per image row walks E, then W, so no two lines touch one partial cell.
// u16 costs: the MODE 3 partial saturates at 0xFFFF; a cell below that holds the exact sum
// (every term >= 0), one at 0xFFFF stays there (the true five-path sum is then still
// >= 65535 - 2 * 16383 > 32767, so the WTA's 32767 clamp sees the same value).
template <int VL, int NP, typename CT>
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
    constexpr int RC = 8;  // columns of a repaired segment loaded together
    if (a.guard && __hip_atomic_load(a.guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane % VL, kl = lane / VL;
    const int y = (int)blockIdx.x * 4 + wave;  // one wave per image row (wave-uniform)
    const size_t pair = blockIdx.y;
    const int H = a.H, W1 = a.W1, nwg = a.nwg, CW = a.cw;
    if (y >= H) return;
    const uint64_t cells = (uint64_t)H * W1 * D;
    const rsrc_t rc = make_rsrc(a.cost + pair * a.cost_pair, cells * sizeof(CT));
    const rsrc_t rp = make_rsrc((const uint8_t*)a.part + pair * a.part_pair, cells * 2);
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
    uint32_t nfix = 0;
    for (int dir = 0; dir < 2; dir++) {  // 0 = E (strips in x order), 1 = W (reverse)
        auto strip_of = [&](int i) { return dir ? nwg - 1 - i : i; };  // path position -> strip
        for (int i0 = 1; i0 < nwg; i0 += CHUNK) {
            // ---- check: does the state entering strip i equal the end state stored by strip i - 1?
            RawBytes<CB> sb[KU], eb[KU];
#pragma unroll
            for (int u = 0; u < KU; u++) {
                const int i = i0 + kl + LPW * u;
                sb[u].load(rs, i < nwg ? soff(strip_of(i), dir, 0) : kOOB);
                eb[u].load(rs, i < nwg ? soff(strip_of(i - 1), dir, 1) : kOOB);
            }
            uint64_t bad = 0;  // bit i - i0: strip i's speculative start differs (wave-uniform below)
#pragma unroll
            for (int u = 0; u < KU; u++) {
                bool ok = true;
#pragma unroll
                for (int q = 0; q < RawBytes<CB>::WORDS; q++) ok &= sb[u].w[q] == eb[u].w[q];
                ok = line_all(ok);
                if (!ok && i0 + kl + LPW * u < nwg) bad |= 1ull << (kl + LPW * u);
            }
            // OR over the wave's lines (their first lanes)
            uint64_t m = 0;
#pragma unroll
            for (int l = 0; l < LPW; l++) {
                const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)bad, l * VL);
                const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(bad >> 32), l * VL);
                m |= ((uint64_t)hi << 32) | lo;
            }
            if (m == 0) continue;  // every strip of the chunk started from the true state
            // ---- repair walk (line 0) from the chunk's first failing strip to the path's end:
            // the trusted state entering strip i is strip i - 1's stored end state while every
            // earlier strip was exact (same), else the true state the walk carries
            if (kl == 0) {
                bool same = true;
                uint32_t T[NP];
#pragma unroll
                for (int q = 0; q < NP; q++) T[q] = 0;
                for (int i = i0 + __builtin_ctzll(m); i < nwg; i++) {
                    const bool flagged = i - i0 < CHUNK ? ((m >> (i - i0)) & 1ull) != 0 : true;
                    if (same && !flagged) continue;  // checked above against the trusted end state
                    const int k = strip_of(i);
                    RawBytes<CB> s1, e1;
                    s1.load(rs, soff(k, dir, 0));
                    e1.load(rs, soff(strip_of(i - 1), dir, 1));
                    uint32_t S[NP], E[NP];
                    unpack_ct_pk<CT, DPL>(s1, S);
                    unpack_ct_pk<CT, DPL>(e1, E);
                    if (same) {
#pragma unroll
                        for (int q = 0; q < NP; q++) T[q] = E[q];
                    }
                    if (same_state(S, T)) {  // the speculative segment started from the true state
                        same = true;
                        continue;
                    }
                    // recompute strip k from T beside its speculative trajectory
                    uint32_t Lq[2][NP], mq[2];
#pragma unroll
                    for (int q = 0; q < NP; q++) {
                        Lq[0][q] = S[q];
                        Lq[1][q] = T[q];
                    }
                    mq[0] = state_min(Lq[0]);
                    mq[1] = state_min(Lq[1]);
                    const int x0 = k * CW, ncol = ::min(CW, W1 - x0);  // W: every repaired strip is full
                    bool met = false;
                    // columns in chunks of RC: the chunk's costs and partial slices load together
                    for (int o0 = 0; o0 < ncol && !met; o0 += RC) {
                        RawBytes<CB> cc[RC];
                        RawBytes<DPL * 2> pb[RC];
#pragma unroll
                        for (int u = 0; u < RC; u++) {
                            const int o = o0 + u;
                            const int c = dir ? x0 + CW - 1 - o : x0 + o;
                            cc[u].load(rc, o < ncol ? cell(c) * (uint32_t)sizeof(CT) : kOOB);
                            pb[u].load(rp, o < ncol ? cell(c) * 2u : kOOB);
                        }
#pragma unroll
                        for (int u = 0; u < RC; u++) {  // (no break: the loop must unroll)
                            const int o = o0 + u;
                            if (o >= ncol || met) continue;
                            const int c = dir ? x0 + CW - 1 - o : x0 + o;
                            uint32_t C2[2][NP], Ln[2][NP], mn[2];
                            unpack_ct_pk<CT, DPL>(cc[u], C2[0]);
#pragma unroll
                            for (int q = 0; q < NP; q++) C2[1][q] = C2[0][q];
                            sweep_step2n<VL, NP, H16, 2>(Lq, mq, C2, P1p, P2p, eL, eR, Ln, mn);
                            if (same_state(Ln[0], Ln[1])) {
                                met = true;
                                continue;
                            }
                            uint32_t P[NP];
#pragma unroll
                            for (int q = 0; q < NP; q++) {
                                if constexpr (SAT) {
                                    uint32_t h[2];
#pragma unroll
                                    for (int e = 0; e < 2; e++) {
                                        const uint32_t pv = (pb[u].w[q] >> (16 * e)) & 0xFFFFu;
                                        const uint32_t sv = (Ln[0][q] >> (16 * e)) & 0xFFFFu;
                                        const uint32_t tv = (Ln[1][q] >> (16 * e)) & 0xFFFFu;
                                        h[e] = pv == 0xFFFFu ? pv : ::min(pv - sv + tv, 0xFFFFu);
                                    }
                                    P[q] = h[0] | (h[1] << 16);
                                } else {  // census: every sum < 2^11, the u16 wrap is exact
                                    P[q] = pk_add(pk_sub(pb[u].w[q], Ln[0][q]), Ln[1][q]);
                                }
                            }
                            bstore_n<uint32_t, NP>(rp, cell(c) * 2u, P);
#pragma unroll
                            for (int q = 0; q < NP; q++) {
                                Lq[0][q] = Ln[0][q];
                                Lq[1][q] = Ln[1][q];
                            }
                            mq[0] = mn[0];
                            mq[1] = mn[1];
                        }
                    }
                    nfix++;
                    same = met;
                    if (!met) {  // the true end state of strip k enters strip k + 1
#pragma unroll
                        for (int q = 0; q < NP; q++) T[q] = Lq[1][q];
                    }
                }
            }
            break;  // the walk covered the rest of this direction
        }
    }
    if (a.fixes && lane == 0 && nfix) atomicAdd(a.fixes, nfix);
}

}  // namespace smk
