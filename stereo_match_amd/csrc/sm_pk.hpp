// sm_pk.hpp — lane-group reductions and the packed u16-pair SGM recurrence
// shared by the fused sweeps (sm_sweep.hpp) and the horizontal-line kernel
// (sm_ew.hpp).
#pragma once
#include "sm_common.hpp"

namespace smk {

template <int VL>
__device__ __forceinline__ uint32_t line_or(uint32_t v)
{
    v |= perm_dpp<DPP_QP_XOR1>(v);
    v |= perm_dpp<DPP_QP_XOR2>(v);
    v |= perm_dpp<DPP_ROW_HALF_MIRROR>(v);
    if constexpr (VL >= 16) v |= perm_dpp<DPP_ROW_MIRROR>(v);
    if constexpr (VL == 32) v = row_pair_combine(v, [](uint32_t a, uint32_t b) { return a | b; });
    return v;
}

// minimum over aligned groups of N lanes (N = 1, 2, 4, 8, 16 or 32: a 32-lane group spans two
// DPP rows, combined by v_permlane16_swap)
template <int N>
__device__ __forceinline__ uint32_t group_min(uint32_t v)
{
    static_assert(N == 1 || N == 2 || N == 4 || N == 8 || N == 16 || N == 32, "lane group of 1-32 lanes");
    if constexpr (N >= 2) v = ::min(v, perm_dpp<DPP_QP_XOR1>(v));
    if constexpr (N >= 4) v = ::min(v, perm_dpp<DPP_QP_XOR2>(v));
    if constexpr (N >= 8) v = ::min(v, perm_dpp<DPP_ROW_HALF_MIRROR>(v));
    if constexpr (N >= 16) v = ::min(v, perm_dpp<DPP_ROW_MIRROR>(v));
    if constexpr (N >= 32) v = row_pair_combine(v, [](uint32_t a, uint32_t b) { return ::min(a, b); });
    return v;
}

template <int N>
__device__ __forceinline__ uint32_t group_sum(uint32_t v)
{
    static_assert(N == 1 || N == 2 || N == 4 || N == 8 || N == 16 || N == 32, "lane group of 1-32 lanes");
    if constexpr (N >= 2) v += perm_dpp<DPP_QP_XOR1>(v);
    if constexpr (N >= 4) v += perm_dpp<DPP_QP_XOR2>(v);
    if constexpr (N >= 8) v += perm_dpp<DPP_ROW_HALF_MIRROR>(v);
    if constexpr (N >= 16) v += perm_dpp<DPP_ROW_MIRROR>(v);
    if constexpr (N >= 32) v = row_pair_combine(v, [](uint32_t a, uint32_t b) { return a + b; });
    return v;
}

template <int N>
__device__ __forceinline__ uint32_t group_max(uint32_t v)
{
    static_assert(N == 1 || N == 2 || N == 4 || N == 8 || N == 16 || N == 32, "lane group of 1-32 lanes");
    if constexpr (N >= 2) v = ::max(v, perm_dpp<DPP_QP_XOR1>(v));
    if constexpr (N >= 4) v = ::max(v, perm_dpp<DPP_QP_XOR2>(v));
    if constexpr (N >= 8) v = ::max(v, perm_dpp<DPP_ROW_HALF_MIRROR>(v));
    if constexpr (N >= 16) v = ::max(v, perm_dpp<DPP_ROW_MIRROR>(v));
    if constexpr (N >= 32) v = row_pair_combine(v, [](uint32_t a, uint32_t b) { return ::max(a, b); });
    return v;
}

// same recurrence as sm_paths.hpp:sgm_step, with VL-lane lines
template <int VL, int DPL>
__device__ __forceinline__ uint32_t sweep_step(const uint32_t (&Lp)[DPL], uint32_t minLp, const uint32_t (&C)[DPL],
                                               uint32_t P1, uint32_t P2, uint32_t (&Ln)[DPL])
{
    const uint32_t lm = Line<VL>::prev(kBig, Lp[DPL - 1]);
    const uint32_t lq = Line<VL>::next(kBig, Lp[0]);
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
    return group_min<VL>(mn);
}

// ---- packed form (even DPL): a lane's L vector as NP = DPL/2 u16 pairs
// (d even in the low half), two disparities per VOP3P instruction.  Every
// intermediate fits 16 bits: L <= max cost + P2 <= 16383 (host domain checks),
// the edge value is OpenCV's MAX_COST 0x7FFF, partial sums of three paths stay
// below 2^16 and the WTA sums saturate before the 32767 clamp.
typedef unsigned short pk16 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pk16 pkv(uint32_t w) { return __builtin_bit_cast(pk16, w); }
__device__ __forceinline__ uint32_t pkw(pk16 v) { return __builtin_bit_cast(uint32_t, v); }
__device__ __forceinline__ uint32_t pk_min(uint32_t a, uint32_t b) { return pkw(__builtin_elementwise_min(pkv(a), pkv(b))); }
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) { return pkw(pkv(a) + pkv(b)); }
__device__ __forceinline__ uint32_t pk_sub(uint32_t a, uint32_t b) { return pkw(pkv(a) - pkv(b)); }
__device__ __forceinline__ uint32_t pk_adds(uint32_t a, uint32_t b)
{
    return pkw(__builtin_elementwise_add_sat(pkv(a), pkv(b)));
}

// min(s + u * 0xFFFF, 0xFFFF) per u16 half (v_pk_mad_u16 with clamp; with the product
// truncated to 16 bits it is still >= 0xFFFD for u in 1..3): the uniqueness test's window
// entries (u = 3 - t > 0) pushed above every sum, the others (u = 0) unchanged, in one
// instruction instead of the negate + saturating add the compiler emits for it
__device__ __forceinline__ uint32_t pk_window_push(uint32_t u, uint32_t s)
{
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, -1, %2 clamp" : "=v"(r) : "v"(u), "v"(s));
    return r;
}

template <int VL, int NP>
__device__ __forceinline__ uint32_t sweep_step_pk(const uint32_t (&Lp)[NP], uint32_t minLp, const uint32_t (&C)[NP],
                                                  uint32_t P1p, uint32_t P2, uint32_t (&Ln)[NP])
{
    constexpr uint32_t EDGE = kBig | (kBig << 16);
    const uint32_t lm = Line<VL>::prev(EDGE, Lp[NP - 1]);  // its high half is d - 1 of element 0
    const uint32_t lq = Line<VL>::next(EDGE, Lp[0]);       // its low half is d + 1 of the last element
    const uint32_t mm = minLp * 0x10001u, dl = (minLp + P2) * 0x10001u;
    uint32_t mn = 0xFFFFFFFFu;
    uint32_t a1 = __builtin_amdgcn_alignbit(Lp[0], lm, 16);  // (d-1, d) neighbours of pair 0
#pragma unroll
    for (int k = 0; k < NP; k++) {
        const uint32_t a2 = __builtin_amdgcn_alignbit(k + 1 < NP ? Lp[k + 1] : lq, Lp[k], 16);  // (d+1, d+2)
        uint32_t v = pk_min(pk_add(pk_min(a1, a2), P1p), Lp[k]);
        v = pk_min(v, dl);
        Ln[k] = pk_add(C[k], pk_sub(v, mm));
        mn = pk_min(mn, Ln[k]);
        a1 = a2;
    }
    return group_min<VL>(::min(mn & 0xFFFFu, mn >> 16));
}

// ---- census form: every census path value, partial and S sum is an integer below 2048
// (L <= 62 + P2 <= 255, S <= 8 x 255), and for n < 2048 the u16 pattern n IS the f16 value
// n * 2^-24 (a denormal below 1024, exponent 1 above; kernels keep f16 denormals,
// .amdhsa_float_denorm_mode_16_64 3), so packed f16 add / sub / min are exact integer ops
// on the unchanged u16 patterns (tools/ubench/f16_exact.hip checks every operand pair) and
// gfx950's packed three-way minimum merges two steps of the recurrence.
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h16x2 hv(uint32_t w) { return __builtin_bit_cast(h16x2, w); }
__device__ __forceinline__ uint32_t hw(h16x2 v) { return __builtin_bit_cast(uint32_t, v); }
// IEEE-2019 minimum (no NaNs here): lowers to v_pk_minimum3_f16 without the operand
// canonicalisation minNum needs, and adjacent minima fuse into one three-way instruction
__device__ __forceinline__ uint32_t h2min(uint32_t a, uint32_t b) { return hw(__builtin_elementwise_minimum(hv(a), hv(b))); }
__device__ __forceinline__ uint32_t h2min3(uint32_t a, uint32_t b, uint32_t c)
{
    return hw(__builtin_elementwise_minimum(__builtin_elementwise_minimum(hv(a), hv(b)), hv(c)));
}
__device__ __forceinline__ uint32_t h2add(uint32_t a, uint32_t b) { return hw(hv(a) + hv(b)); }
__device__ __forceinline__ uint32_t h2sub(uint32_t a, uint32_t b) { return hw(hv(a) - hv(b)); }

// sweep_step_pk on census values in the f16 form: per packed word alignbit, min, add P1,
// minimum3 (Lp, minLp + P2), sub minLp, add C, and half a minimum3 for the row minimum
template <int VL, int NP>
__device__ __forceinline__ uint32_t sweep_step_h16(const uint32_t (&Lp)[NP], uint32_t minLp, const uint32_t (&C)[NP],
                                                   uint32_t P1p, uint32_t P2, uint32_t (&Ln)[NP])
{
    constexpr uint32_t EDGE = 0x7BFF7BFFu;  // largest finite f16 (OpenCV's MAX_COST edge: above every L)
    const uint32_t lm = Line<VL>::prev(EDGE, Lp[NP - 1]);
    const uint32_t lq = Line<VL>::next(EDGE, Lp[0]);
    const uint32_t mm = minLp * 0x10001u, dl = (minLp + P2) * 0x10001u;
    uint32_t a1 = __builtin_amdgcn_alignbit(Lp[0], lm, 16);
#pragma unroll
    for (int k = 0; k < NP; k++) {
        const uint32_t a2 = __builtin_amdgcn_alignbit(k + 1 < NP ? Lp[k + 1] : lq, Lp[k], 16);
        const uint32_t v = h2min3(h2add(h2min(a1, a2), P1p), Lp[k], dl);
        Ln[k] = h2add(h2sub(v, mm), C[k]);
        a1 = a2;
    }
    uint32_t mn;
    if constexpr (NP == 1) {
        mn = Ln[0];
    } else {
        mn = h2min(Ln[0], Ln[1]);
#pragma unroll
        for (int k = 2; k < NP; k += 2) mn = k + 1 < NP ? h2min3(mn, Ln[k], Ln[k + 1]) : h2min(mn, Ln[k]);
    }
    return group_min<VL>(::min(mn & 0xFFFFu, mn >> 16));
}

// The fused sweeps' form of the step (u16 or, for census, the f16 form):
//  * the row minimum travels replicated in both halves (m | m << 16): a lane's own
//    minimum is min(w, swap(w)) and the cross-lane steps are plain u32 minima (on
//    replicated words the u32 order is the order of m), so minLp + P2 is one packed add
//    and minLp needs no repacking;
//  * 16-lane lines take the d - 1 / d + 1 neighbours across lanes with zero-filling DPP
//    moves OR'ed with the per-lane edge constants eL / eR (EDGE on the line's first /
//    last lane, 0 elsewhere), which the compiler fuses into one v_or_b32_dpp each.
template <int VL, int NP, bool H16, bool DS = false>
__device__ __forceinline__ uint32_t sweep_step2(const uint32_t (&Lp)[NP], uint32_t mmp, const uint32_t (&C)[NP],
                                                uint32_t P1p, uint32_t P2p, uint32_t eL, uint32_t eR,
                                                uint32_t (&Ln)[NP])
{
    static_assert(!DS || H16, "deferred subtraction (sweep_step2n): census f16 form only");
    constexpr uint32_t EDGE = H16 ? 0x7BFF7BFFu : (kBig | (kBig << 16));
    uint32_t lm, lq;
    if constexpr (VL == 16) {
        lm = perm_dpp<DPP_ROW_SHR1>(Lp[NP - 1]) | eL;
        lq = perm_dpp<DPP_ROW_SHL1>(Lp[0]) | eR;
    } else if constexpr (VL == 8 || VL == 4) {  // lines inside a DPP row: the edge lanes select EDGE
        // the moves run in every lane BEFORE the select (inside a lane-divergent arm the
        // edge lanes would be inactive sources and read as 0)
        const uint32_t pm = perm_dpp<DPP_ROW_SHR1>(Lp[NP - 1]), pq = perm_dpp<DPP_ROW_SHL1>(Lp[0]);
        lm = eL ? EDGE : pm;
        lq = eR ? EDGE : pq;
    } else if constexpr (VL == 32) {  // lines across two DPP rows: whole-wave shifts, edge select
        const uint32_t pm = perm_dpp<DPP_WAVE_SHR1>(Lp[NP - 1]), pq = perm_dpp<DPP_WAVE_SHL1>(Lp[0]);
        lm = eL ? EDGE : pm;
        lq = eR ? EDGE : pq;
    } else {
        lm = Line<VL>::prev(EDGE, Lp[NP - 1]);
        lq = Line<VL>::next(EDGE, Lp[0]);
    }
    const uint32_t dl = H16 ? h2add(mmp, P2p) : pk_add(mmp, P2p);
    uint32_t a1 = __builtin_amdgcn_alignbit(Lp[0], lm, 16);
#pragma unroll
    for (int k = 0; k < NP; k++) {
        const uint32_t a2 = __builtin_amdgcn_alignbit(k + 1 < NP ? Lp[k + 1] : lq, Lp[k], 16);
        if constexpr (H16) {
            const uint32_t v = h2min3(h2add(h2min(a1, a2), P1p), Lp[k], dl);
            Ln[k] = DS ? h2add(v, C[k]) : h2add(h2sub(v, mmp), C[k]);
        } else {
            uint32_t v = pk_min(pk_add(pk_min(a1, a2), P1p), Lp[k]);
            v = pk_min(v, dl);
            Ln[k] = pk_add(C[k], pk_sub(v, mmp));
        }
        a1 = a2;
    }
    uint32_t mn = Ln[0];
    if constexpr (H16) {
#pragma unroll
        for (int k = 1; k < NP; k += 2) mn = k + 1 < NP ? h2min3(mn, Ln[k], Ln[k + 1]) : h2min(mn, Ln[k]);
        mn = h2min(mn, __builtin_amdgcn_alignbit(mn, mn, 16));
    } else {
#pragma unroll
        for (int k = 1; k < NP; k++) mn = pk_min(mn, Ln[k]);
        mn = pk_min(mn, __builtin_amdgcn_alignbit(mn, mn, 16));
    }
    return group_min<VL>(mn);  // replicated halves: u32 minima are exact
}

// ND independent recurrences of sweep_step2 (e.g. the A and B diagonals of one column, or a
// halo wave's two column sets), issued word by word across the directions: the packed
// (VOP3P) operations of one recurrence form a dependent chain, and on gfx950 a VOP3P that
// reads the VGPR the previous VALU wrote needs a wait state (s_nop 0) — with ND chains
// interleaved the dependent operations are never adjacent.  The DPP minimum steps are
// interleaved the same way (a DPP read of a VGPR the previous VALU wrote needs two wait
// states).  Same operations, same order per recurrence: results identical to sweep_step2.
template <int N, int ND>
__device__ __forceinline__ void group_min_n(uint32_t (&v)[ND])
{
    static_assert(N == 1 || N == 2 || N == 4 || N == 8 || N == 16 || N == 32 || N == 64, "lane group of 1-64 lanes");
    if constexpr (N >= 2) {
#pragma unroll
        for (int n = 0; n < ND; n++) v[n] = ::min(v[n], perm_dpp<DPP_QP_XOR1>(v[n]));
    }
    if constexpr (N >= 4) {
#pragma unroll
        for (int n = 0; n < ND; n++) v[n] = ::min(v[n], perm_dpp<DPP_QP_XOR2>(v[n]));
    }
    if constexpr (N >= 8) {
#pragma unroll
        for (int n = 0; n < ND; n++) v[n] = ::min(v[n], perm_dpp<DPP_ROW_HALF_MIRROR>(v[n]));
    }
    if constexpr (N >= 16) {
#pragma unroll
        for (int n = 0; n < ND; n++) v[n] = ::min(v[n], perm_dpp<DPP_ROW_MIRROR>(v[n]));
    }
    if constexpr (N >= 32) {
#pragma unroll
        for (int n = 0; n < ND; n++) v[n] = row_pair_combine(v[n], [](uint32_t a, uint32_t b) { return ::min(a, b); });
    }
    if constexpr (N >= 64) {  // the two wave halves: v_permlane32_swap
#pragma unroll
        for (int n = 0; n < ND; n++) {
            const auto r = __builtin_amdgcn_permlane32_swap(v[n], v[n], false, false);
            v[n] = ::min((uint32_t)r[0], (uint32_t)r[1]);
        }
    }
}

// DS (deferred subtraction, census f16 form only): the step leaves out "- minLp", so the new
// state is R = L + minLp (every later step is shift-invariant: min3(R, R_d+-1 + P1, minR + P2)
// moves with a constant shift of its input, so the true value of any state's successor is
// R_next - minR of that state).  The caller subtracts the input minima once per sum of paths
// instead of once per word and path, and renormalises the state (R - minR) often enough that
// every value stays below the f16 form's 2^11 (sm_sweep.hpp SWEEP_DS).
template <int VL, int NP, bool H16, int ND, bool DS = false>
__device__ __forceinline__ void sweep_step2n(const uint32_t (&Lp)[ND][NP], const uint32_t (&mmp)[ND],
                                             const uint32_t (&C)[ND][NP], uint32_t P1p, uint32_t P2p, uint32_t eL,
                                             uint32_t eR, uint32_t (&Ln)[ND][NP], uint32_t (&mn)[ND])
{
    static_assert(!DS || H16, "deferred subtraction: census f16 form only");
    constexpr uint32_t EDGE = H16 ? 0x7BFF7BFFu : (kBig | (kBig << 16));
    uint32_t lm[ND], lq[ND], dl[ND], a1[ND];
#pragma unroll
    for (int n = 0; n < ND; n++) {
        if constexpr (VL == 16) {
            lm[n] = perm_dpp<DPP_ROW_SHR1>(Lp[n][NP - 1]) | eL;
            lq[n] = perm_dpp<DPP_ROW_SHL1>(Lp[n][0]) | eR;
        } else if constexpr (VL == 8 || VL == 4) {
            const uint32_t pm = perm_dpp<DPP_ROW_SHR1>(Lp[n][NP - 1]), pq = perm_dpp<DPP_ROW_SHL1>(Lp[n][0]);
            lm[n] = eL ? EDGE : pm;
            lq[n] = eR ? EDGE : pq;
        } else if constexpr (VL == 32) {  // lines across two DPP rows: whole-wave shifts, edge select
            const uint32_t pm = perm_dpp<DPP_WAVE_SHR1>(Lp[n][NP - 1]), pq = perm_dpp<DPP_WAVE_SHL1>(Lp[n][0]);
            lm[n] = eL ? EDGE : pm;
            lq[n] = eR ? EDGE : pq;
        } else {
            lm[n] = Line<VL>::prev(EDGE, Lp[n][NP - 1]);
            lq[n] = Line<VL>::next(EDGE, Lp[n][0]);
        }
    }
#pragma unroll
    for (int n = 0; n < ND; n++) {
        dl[n] = H16 ? h2add(mmp[n], P2p) : pk_add(mmp[n], P2p);
        a1[n] = __builtin_amdgcn_alignbit(Lp[n][0], lm[n], 16);
    }
    // the words of one recurrence are independent too (a word's d-1 / d+1 neighbours come
    // from the previous step's L), so every stage runs over all ND x NP words before the next
    uint32_t v[ND][NP];
#pragma unroll
    for (int k = 0; k < NP; k++) {
#pragma unroll
        for (int n = 0; n < ND; n++)
            v[n][k] = __builtin_amdgcn_alignbit(k + 1 < NP ? Lp[n][k + 1] : lq[n], Lp[n][k], 16);
    }
    // v[n][k] now holds the (d+1, d+2) neighbours of word k; (d-1, d) = a1 for k = 0, else
    // v[n][k-1]
#pragma unroll
    for (int k = NP - 1; k >= 0; k--) {
#pragma unroll
        for (int n = 0; n < ND; n++) {
            const uint32_t lo = k == 0 ? a1[n] : v[n][k - 1];
            v[n][k] = H16 ? h2min(lo, v[n][k]) : pk_min(lo, v[n][k]);
        }
    }
    if constexpr (H16) {
#pragma unroll
        for (int k = 0; k < NP; k++)
#pragma unroll
            for (int n = 0; n < ND; n++) v[n][k] = h2add(v[n][k], P1p);
#pragma unroll
        for (int k = 0; k < NP; k++)
#pragma unroll
            for (int n = 0; n < ND; n++) v[n][k] = h2min3(v[n][k], Lp[n][k], dl[n]);
        if constexpr (!DS) {
#pragma unroll
            for (int k = 0; k < NP; k++)
#pragma unroll
                for (int n = 0; n < ND; n++) v[n][k] = h2sub(v[n][k], mmp[n]);
        }
#pragma unroll
        for (int k = 0; k < NP; k++)
#pragma unroll
            for (int n = 0; n < ND; n++) Ln[n][k] = h2add(v[n][k], C[n][k]);
    } else {
#pragma unroll
        for (int k = 0; k < NP; k++)
#pragma unroll
            for (int n = 0; n < ND; n++) v[n][k] = pk_add(v[n][k], P1p);
#pragma unroll
        for (int k = 0; k < NP; k++)
#pragma unroll
            for (int n = 0; n < ND; n++) v[n][k] = pk_min(v[n][k], Lp[n][k]);
#pragma unroll
        for (int k = 0; k < NP; k++)
#pragma unroll
            for (int n = 0; n < ND; n++) v[n][k] = pk_min(v[n][k], dl[n]);
#pragma unroll
        for (int k = 0; k < NP; k++)
#pragma unroll
            for (int n = 0; n < ND; n++) v[n][k] = pk_sub(v[n][k], mmp[n]);
#pragma unroll
        for (int k = 0; k < NP; k++)
#pragma unroll
            for (int n = 0; n < ND; n++) Ln[n][k] = pk_add(C[n][k], v[n][k]);
    }
#pragma unroll
    for (int n = 0; n < ND; n++) mn[n] = Ln[n][0];
    if constexpr (H16) {
#pragma unroll
        for (int k = 1; k < NP; k += 2) {
#pragma unroll
            for (int n = 0; n < ND; n++) mn[n] = k + 1 < NP ? h2min3(mn[n], Ln[n][k], Ln[n][k + 1]) : h2min(mn[n], Ln[n][k]);
        }
#pragma unroll
        for (int n = 0; n < ND; n++) mn[n] = h2min(mn[n], __builtin_amdgcn_alignbit(mn[n], mn[n], 16));
    } else {
#pragma unroll
        for (int k = 1; k < NP; k++) {
#pragma unroll
            for (int n = 0; n < ND; n++) mn[n] = pk_min(mn[n], Ln[n][k]);
        }
#pragma unroll
        for (int n = 0; n < ND; n++) mn[n] = pk_min(mn[n], __builtin_amdgcn_alignbit(mn[n], mn[n], 16));
    }
    group_min_n<VL, ND>(mn);  // replicated halves: u32 minima are exact
}

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

// raw cost / E / W bytes of one lane -> NP packed pairs (u16 already pairs; u8 widened)
template <typename CT, int DPL>
__device__ __forceinline__ void unpack_ct_pk(const RawBytes<DPL * (int)sizeof(CT)>& r, uint32_t (&C)[DPL / 2])
{
#pragma unroll
    for (int k = 0; k < DPL / 2; k++) {
        if constexpr (sizeof(CT) == 2) C[k] = r.w[k];
        else C[k] = __builtin_amdgcn_perm(0u, r.w[k >> 1], (k & 1) ? 0x0c030c02u : 0x0c010c00u);
    }
}

}  // namespace smk
