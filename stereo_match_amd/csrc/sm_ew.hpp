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

// NP packed u16 pairs -> LT bytes at byte offset off (u8: truncating pack; u16: as is)
template <typename LT, int NP, int AUX = 0>
__device__ __forceinline__ void store_pk(rsrc_t r, uint32_t off, const uint32_t (&w)[NP])
{
    if constexpr (sizeof(LT) == 2) {
        bstore_n<uint32_t, NP, AUX>(r, off, w);
    } else {
        constexpr int NW = NP / 2;
        if constexpr (NW > 0) {
            uint32_t b[NW];
#pragma unroll
            for (int j = 0; j < NW; j++) b[j] = __builtin_amdgcn_perm(w[2 * j + 1], w[2 * j], 0x06040200u);
            bstore_n<uint32_t, NW, AUX>(r, off, b);
        }
        if constexpr (NP % 2)
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)((w[NP - 1] & 0xFFu) | ((w[NP - 1] >> 8) & 0xFF00u)), r,
                                                  off + 4 * NW, 0, AUX);
    }
}

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

}  // namespace smk
