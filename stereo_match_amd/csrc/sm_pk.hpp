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
    if constexpr (VL == 16) v |= perm_dpp<DPP_ROW_MIRROR>(v);
    return v;
}

// minimum over aligned groups of N lanes (N = 4, 8 or 16)
template <int N>
__device__ __forceinline__ uint32_t group_min(uint32_t v)
{
    v = ::min(v, perm_dpp<DPP_QP_XOR1>(v));
    v = ::min(v, perm_dpp<DPP_QP_XOR2>(v));
    if constexpr (N >= 8) v = ::min(v, perm_dpp<DPP_ROW_HALF_MIRROR>(v));
    if constexpr (N >= 16) v = ::min(v, perm_dpp<DPP_ROW_MIRROR>(v));
    return v;
}

template <int N>
__device__ __forceinline__ uint32_t group_sum(uint32_t v)
{
    v += perm_dpp<DPP_QP_XOR1>(v);
    v += perm_dpp<DPP_QP_XOR2>(v);
    if constexpr (N >= 8) v += perm_dpp<DPP_ROW_HALF_MIRROR>(v);
    if constexpr (N >= 16) v += perm_dpp<DPP_ROW_MIRROR>(v);
    return v;
}

template <int N>
__device__ __forceinline__ uint32_t group_max(uint32_t v)
{
    v = ::max(v, perm_dpp<DPP_QP_XOR1>(v));
    v = ::max(v, perm_dpp<DPP_QP_XOR2>(v));
    if constexpr (N >= 8) v = ::max(v, perm_dpp<DPP_ROW_HALF_MIRROR>(v));
    if constexpr (N >= 16) v = ::max(v, perm_dpp<DPP_ROW_MIRROR>(v));
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
