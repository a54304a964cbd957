// sm_sweep.hpp — fused two-sweep SGM engine on gfx950.
//
// The per-direction engine (sm_paths.hpp) writes one path volume per direction
// and a WTA kernel re-reads all of them: 25 B of HBM traffic per cell at
// 8 paths.  Here the three directions that advance one image row per step in
// the same vertical sense share one sweep:
//   down sweep: S (0,+1), SE (+1,+1), SW (-1,+1)
//   up sweep:   N (0,-1), NE (+1,-1), NW (-1,-1)
// and their per-cell sum never leaves the chip except as one u16 partial
// (8 paths) — or not at all: the last sweep adds the horizontal (E, W) volumes
// and the other sweep's partial and runs the WTA / uniqueness / sub-pixel /
// disp2 step in place.  Traffic per cell (census, 8 paths): cost 1 B written,
// 4 B read (E, W, down, up), E/W 2 B written + 2 B read, partial 2 + 2 B = 13 B.
//
// Decomposition: a workgroup owns a strip of CW adjacent columns of one pair
// for all rows (4 waves, 64/VL columns per wave, VL lanes per column, DPL =
// D/VL disparities per lane).  The vertical direction is private to a lane
// group.  The diagonals read the previous row's L vector of the neighbouring
// column: inside the strip through a double-buffered LDS row (one barrier per
// row); across strips through tagged 8-byte granules written `sc1` by the
// edge column and polled `sc1` by the neighbouring workgroup (MI355X guide
// §6 Guideline 16, form R2: the data is the flag, no fence).  All workgroups
// of a pair must be co-resident: the host sizes the grid from the occupancy
// query, and every poll is bounded (timeout -> error word, never a hang).
//
// Recurrence and domain exactly as sm_paths.hpp / oracle/sgm_np.py: a path
// enters [minX1, maxX1) x [0, H) with Lp = 0 and minLp = 0 (the LDS halo
// columns of the outermost strips stay zero, inactive columns hold zero).
#pragma once
#include "sm_common.hpp"
#include "sm_sweep_host.hpp"

namespace smk {

typedef __attribute__((address_space(1))) unsigned long long gu64;

constexpr int SW_WAVES = 4;
constexpr uint32_t SW_SPIN_LIMIT = 1u << 19;
constexpr int SW_PF = 3;  // rows of inputs in flight per lane

template <int VL, int DPL>
struct SweepGeo {
    static constexpr int LPW = 64 / VL;            // columns per wave
    static constexpr int CW = SW_WAVES * LPW;      // columns per workgroup
    static constexpr int COLS = CW + 2;            // + one halo column each side
    static constexpr int D = VL * DPL;
    static constexpr int NG = (DPL + 1) / 2;       // granules per lane (two u16 per granule)
    static constexpr int NGR = VL * NG;            // granules per (strip, direction, row)
    static constexpr int LDS_BYTES = 2 * 2 * COLS * D * 2 + 2 * 2 * COLS * 4;
};

template <int VL>
__device__ __forceinline__ uint32_t line_or(uint32_t v)
{
    v |= perm_dpp<DPP_QP_XOR1>(v);
    v |= perm_dpp<DPP_QP_XOR2>(v);
    v |= perm_dpp<DPP_ROW_HALF_MIRROR>(v);
    if constexpr (VL == 16) v |= perm_dpp<DPP_ROW_MIRROR>(v);
    return v;
}

template <int VL>
__device__ __forceinline__ uint32_t line_min(uint32_t v)
{
    v = ::min(v, perm_dpp<DPP_QP_XOR1>(v));
    v = ::min(v, perm_dpp<DPP_QP_XOR2>(v));
    v = ::min(v, perm_dpp<DPP_ROW_HALF_MIRROR>(v));
    if constexpr (VL == 16) v = ::min(v, perm_dpp<DPP_ROW_MIRROR>(v));
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
    return line_min<VL>(mn);
}

// DPL u16 values of one lane in LDS (little-endian pairs), widest aligned chunks
template <int DPL>
__device__ __forceinline__ void lds_put(uint16_t* p, const uint32_t (&v)[DPL])
{
    if constexpr (DPL % 2 == 0) {
        uint32_t w[DPL / 2];
#pragma unroll
        for (int k = 0; k < DPL / 2; k++) w[k] = __builtin_amdgcn_perm(v[2 * k + 1], v[2 * k], 0x05040100u);
        if constexpr (DPL % 8 == 0) {
#pragma unroll
            for (int k = 0; k < DPL / 8; k++)
                reinterpret_cast<uint4*>(p)[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
        } else if constexpr (DPL % 4 == 0) {
#pragma unroll
            for (int k = 0; k < DPL / 4; k++) reinterpret_cast<uint2*>(p)[k] = make_uint2(w[2 * k], w[2 * k + 1]);
        } else {
#pragma unroll
            for (int k = 0; k < DPL / 2; k++) reinterpret_cast<uint32_t*>(p)[k] = w[k];
        }
    } else {
#pragma unroll
        for (int i = 0; i < DPL; i++) p[i] = (uint16_t)v[i];
    }
}

template <int DPL>
__device__ __forceinline__ void lds_get(const uint16_t* p, uint32_t (&v)[DPL])
{
    if constexpr (DPL % 8 == 0) {
#pragma unroll
        for (int k = 0; k < DPL / 8; k++) {
            const uint4 q = reinterpret_cast<const uint4*>(p)[k];
            const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int j = 0; j < 4; j++) {
                v[8 * k + 2 * j] = w[j] & 0xFFFFu;
                v[8 * k + 2 * j + 1] = w[j] >> 16;
            }
        }
    } else if constexpr (DPL % 4 == 0) {
#pragma unroll
        for (int k = 0; k < DPL / 4; k++) {
            const uint2 q = reinterpret_cast<const uint2*>(p)[k];
            v[4 * k] = q.x & 0xFFFFu;
            v[4 * k + 1] = q.x >> 16;
            v[4 * k + 2] = q.y & 0xFFFFu;
            v[4 * k + 3] = q.y >> 16;
        }
    } else if constexpr (DPL % 2 == 0) {
#pragma unroll
        for (int k = 0; k < DPL / 2; k++) {
            const uint32_t q = reinterpret_cast<const uint32_t*>(p)[k];
            v[2 * k] = q & 0xFFFFu;
            v[2 * k + 1] = q >> 16;
        }
    } else {
#pragma unroll
        for (int i = 0; i < DPL; i++) v[i] = p[i];
    }
}

template <typename CT, int DPL>
__device__ __forceinline__ void unpack_ct(const RawBytes<DPL * (int)sizeof(CT)>& r, uint32_t (&C)[DPL])
{
#pragma unroll
    for (int i = 0; i < DPL; i++) C[i] = r.template get<CT>(i);
}

// Workgroup barrier that orders LDS only.  __syncthreads() is a workgroup
// release of global memory too: each wave then waits (vmcnt) for its own
// just-issued global stores to be acknowledged before every row's barrier.
// Nothing global is exchanged inside a workgroup here (the strip hand-off has
// its own protocol), so only the LDS writes have to land first.
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Poll NG granules of one lane until every tag equals `tag` (lanes with !need
// do not load).  Wave-uniform exit; gives up after SW_SPIN_LIMIT passes.
template <int NG>
__device__ __forceinline__ void poll_granules(const gu64* src, bool need, uint32_t tag, uint32_t (&v)[NG], bool& dead,
                                              uint32_t* err)
{
    for (uint32_t spins = 0;; spins++) {
        bool ok = true;
        if (need) {
#pragma unroll
            for (int k = 0; k < NG; k++) {
                const unsigned long long x = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                v[k] = (uint32_t)x;
                ok &= (uint32_t)(x >> 32) == tag;
            }
        }
        if (__all(ok) || dead) return;
        if (spins >= SW_SPIN_LIMIT) {
            if ((threadIdx.x & 63) == 0) atomicOr(err, 1u);
            dead = true;
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

template <int VL, int DPL, typename CT, int MODE>
__global__ void __launch_bounds__(256) k_sweep(SweepArgs a)
{
    using G = SweepGeo<VL, DPL>;
    constexpr bool UP = MODE == 2;
    constexpr bool WTA = MODE != 0;
    constexpr int LPW = G::LPW, CW = G::CW, COLS = G::COLS, D = G::D, NG = G::NG, NGR = G::NGR;
    constexpr int CB = DPL * (int)sizeof(CT);  // cost / E / W bytes per lane and cell
    __shared__ __attribute__((aligned(16))) uint16_t lv[2][2][COLS][D];  // [buf][A=+dx, B=-dx][col+1][d]
    __shared__ uint32_t lmin[2][2][COLS];

    for (int i = threadIdx.x; i < 2 * 2 * COLS * D / 2; i += 256) reinterpret_cast<uint32_t*>(&lv[0][0][0][0])[i] = 0;
    for (int i = threadIdx.x; i < 2 * 2 * COLS; i += 256) (&lmin[0][0][0])[i] = 0;
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int kl = lane / VL, g = lane % VL;
    const int c = wave * LPW + kl;  // column inside the strip
    const int wg = blockIdx.x, pair = blockIdx.y;
    const int H = a.H, W1 = a.W1;
    const int x1 = wg * CW + c;
    const bool active = x1 < W1;
    const bool wave_ragged = wg * CW + wave * LPW + LPW > W1;  // wave-uniform
    const uint32_t P1 = (uint32_t)a.P1, P2 = (uint32_t)a.P2;

    const uint64_t cells = (uint64_t)H * W1 * D;
    const rsrc_t rc = make_rsrc(a.cost + (size_t)pair * a.cost_pair, cells * sizeof(CT));
    rsrc_t re = make_rsrc(nullptr, 0), rw = re, rp = re;
    if constexpr (WTA) {
        re = make_rsrc(a.ew + (size_t)pair * a.ew_pair, cells * sizeof(CT));
        rw = make_rsrc(a.ew + (size_t)pair * a.ew_pair + a.ew_slot, cells * sizeof(CT));
    }
    if constexpr (MODE != 1) rp = make_rsrc((const uint8_t*)a.part + (size_t)pair * a.part_pair, cells * 2);
    // element offset of this lane's slice in row y
    auto cell = [&](int y) -> uint32_t {
        return active ? ((uint32_t)y * (uint32_t)W1 + (uint32_t)x1) * (uint32_t)D + (uint32_t)(g * DPL) : 0xFFFFFFFFu;
    };
    auto boff = [&](uint32_t e, int bytes) -> uint32_t { return e == 0xFFFFFFFFu ? kOOB : e * (uint32_t)bytes; };

    gu64* hop = (gu64*)(a.hop + (size_t)pair * a.hop_pair);
    auto slot = [&](int strip, int dir, int s) -> size_t {
        return ((size_t)(strip * 2 + dir) * H + s) * NGR + (size_t)g * NG;
    };
    // the edge waves exchange with the neighbouring strips
    const bool has_left = wg > 0, has_right = wg + 1 < a.nwg;
    const bool cons_a = wave == 0 && has_left;                  // left halo of A (= SE / NE)
    const bool cons_b = wave == SW_WAVES - 1 && has_right;      // right halo of B (= SW / NW)
    const uint32_t tag0 = a.epoch << 16;
    // publishing: buffer stores (sc1) at an out-of-range offset for every other lane
    const rsrc_t rhop = make_rsrc(a.hop + (size_t)pair * a.hop_pair, (uint64_t)a.hop_pair * 8);
    const bool pub_a = wave == SW_WAVES - 1 && has_right && kl == LPW - 1;  // last column -> right strip
    const bool pub_b = wave == 0 && has_left && kl == 0;                   // first column -> left strip
    const bool edge_wave = (wave == 0 && has_left) || (wave == SW_WAVES - 1 && has_right);  // wave-uniform
    bool dead = (a.dbg & 1) != 0;

    uint32_t LV[DPL];
#pragma unroll
    for (int i = 0; i < DPL; i++) LV[i] = 0;
    uint32_t mV = 0;

    // per-step inputs through a ring of SW_PF rows in flight (the step is
    // short next to HBM latency under load; one row ahead left every step
    // waiting for its loads)
    constexpr int PF = SW_PF;
    RawBytes<CB> rc_[PF], re_[PF], rw_[PF];
    RawBytes<DPL * 2> rp_[PF];
    auto issue = [&](int k, int s) {  // loads of step s into ring slot k (rows past the end read 0)
        const uint32_t en = s < H ? cell(UP ? H - 1 - s : s) : 0xFFFFFFFFu;
        rc_[k].load(rc, boff(en, sizeof(CT)));
        if constexpr (WTA) {
            re_[k].load(re, boff(en, sizeof(CT)));
            rw_[k].load(rw, boff(en, sizeof(CT)));
        }
        if constexpr (MODE == 2) rp_[k].load(rp, boff(en, 2));
    };
#pragma unroll
    for (int k = 0; k < PF; k++) issue(k, k);

    for (int s0 = 0; s0 < H; s0 += PF) {
#pragma unroll
        for (int k = 0; k < PF; k++) {
            // whole ring rounds (no early exit: a break here makes the compiler
            // rotate the ring registers with moves that wait for the newest load);
            // steps s >= H run masked: out-of-range offsets, no hand-off, no WTA output
            const int s = s0 + k;
            const bool live = s < H;
            const int y = UP ? H - 1 - s : s;
            const int rb = (s + 1) & 1, wb = s & 1;
            const uint32_t e = live ? cell(y) : 0xFFFFFFFFu;
            uint32_t C[DPL];
            unpack_ct<CT, DPL>(rc_[k], C);
            uint32_t Ein[DPL], Win[DPL], Pin[DPL];
            if constexpr (WTA) {
                unpack_ct<CT, DPL>(re_[k], Ein);
                unpack_ct<CT, DPL>(rw_[k], Win);
            }
            if constexpr (MODE == 2) unpack_ct<uint16_t, DPL>(rp_[k], Pin);

            // diagonal predecessors: column c-1 (A) and c+1 (B) of the previous row
            uint32_t LA[DPL], LB[DPL];
            lds_get<DPL>(&lv[rb][0][c][g * DPL], LA);
            lds_get<DPL>(&lv[rb][1][c + 2][g * DPL], LB);
            uint32_t mA = lmin[rb][0][c], mB = lmin[rb][1][c + 2];
#ifndef SWEEP_NOPOLL
            if (s > 0 && live && !(a.dbg & 2)) {
                if (cons_a) {  // wave 0, column 0 <- last column of strip wg-1
                    uint32_t v[NG];
                    poll_granules<NG>(hop + slot(wg - 1, 0, s - 1), kl == 0, tag0 | (uint32_t)s, v, dead, a.err);
                    uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
                    for (int i = 0; i < DPL; i++) {
                        const uint32_t t = (v[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
                        LA[i] = kl == 0 ? t : LA[i];
                        mn = min(mn, t);
                    }
                    mn = line_min<VL>(mn);
                    mA = kl == 0 ? mn : mA;
                }
                if (cons_b) {  // last wave, last column <- column 0 of strip wg+1
                    uint32_t v[NG];
                    poll_granules<NG>(hop + slot(wg + 1, 1, s - 1), kl == LPW - 1, tag0 | (uint32_t)s, v, dead,
                                      a.err);
                    uint32_t mn = 0xFFFFFFFFu;
#pragma unroll
                    for (int i = 0; i < DPL; i++) {
                        const uint32_t t = (v[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
                        LB[i] = kl == LPW - 1 ? t : LB[i];
                        mn = min(mn, t);
                    }
                    mn = line_min<VL>(mn);
                    mB = kl == LPW - 1 ? mn : mB;
                }
            }
#endif

            // refill the ring only now: the polls above wait (vmcnt) for every older
            // load of the wave, so loads issued before them would be waited for too
            issue(k, s + PF);

            uint32_t nA[DPL], nB[DPL];
            uint32_t mnA = sweep_step<VL, DPL>(LA, mA, C, P1, P2, nA);
            uint32_t mnB = sweep_step<VL, DPL>(LB, mB, C, P1, P2, nB);
            if (wave_ragged) {  // columns past W1 stay at the entering state
#pragma unroll
                for (int i = 0; i < DPL; i++) {
                    nA[i] = active ? nA[i] : 0u;
                    nB[i] = active ? nB[i] : 0u;
                }
                mnA = active ? mnA : 0u;
                mnB = active ? mnB : 0u;
            }
            // hand the strip-edge columns to the neighbouring strips (sc1 stores by the
            // edge waves only: every store holds a vmcnt slot of the storing wave)
            if (edge_wave && live) {
                const uint32_t tag = tag0 | (uint32_t)(s + 1);
                const uint32_t oa = pub_a ? (uint32_t)(slot(wg, 0, s) * 8) : kOOB;
                const uint32_t ob = pub_b ? (uint32_t)(slot(wg, 1, s) * 8) : kOOB;
#pragma unroll
                for (int q = 0; q < NG; q++) {
                    const uint32_t va = nA[2 * q] | (2 * q + 1 < DPL ? nA[2 * q + 1] << 16 : 0u);
                    const uint32_t vb = nB[2 * q] | (2 * q + 1 < DPL ? nB[2 * q + 1] << 16 : 0u);
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{va, tag}, rhop, oa + 8 * q, 0, 16);
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{vb, tag}, rhop, ob + 8 * q, 0, 16);
                }
            }
            lds_put<DPL>(&lv[wb][0][c + 1][g * DPL], nA);
            lds_put<DPL>(&lv[wb][1][c + 1][g * DPL], nB);
            if (g == 0) {
                lmin[wb][0][c + 1] = mnA;
                lmin[wb][1][c + 1] = mnB;
            }

            uint32_t nV[DPL];
            const uint32_t mnV = sweep_step<VL, DPL>(LV, mV, C, P1, P2, nV);
#pragma unroll
            for (int i = 0; i < DPL; i++) LV[i] = nV[i];
            mV = mnV;

            if constexpr (MODE == 0) {
                uint32_t sum[DPL];
#pragma unroll
                for (int i = 0; i < DPL; i++) sum[i] = nV[i] + nA[i] + nB[i];
                bstore_n<uint16_t, DPL>(rp, boff(e, 2), sum);
            } else {
                uint32_t S[DPL];
                uint32_t key = 0xFFFFFFFFu;
#pragma unroll
                for (int i = 0; i < DPL; i++) {
                    uint32_t t = nV[i] + nA[i] + nB[i] + Ein[i] + Win[i];
                    if constexpr (MODE == 2) t += Pin[i];
                    S[i] = min(t, 32767u);
                    key = min(key, (S[i] << 16) | (uint32_t)(g * DPL + i));
                }
                key = line_min<VL>(key);
                const int minS = (int)(key >> 16), best = (int)(key & 0xFFFF);
                const int u = a.uniq;
                uint32_t bad = 0, nb = 0;
#pragma unroll
                for (int i = 0; i < DPL; i++) {
                    const int d = g * DPL + i;
                    const int dd = best - d;
                    bad |= ((int)S[i] * (100 - u) < minS * 100 && (dd > 1 || dd < -1)) ? 1u : 0u;
                    nb |= d == best - 1 ? S[i] : 0u;
                    nb |= d == best + 1 ? (S[i] << 16) : 0u;
                }
                bad = line_or<VL>(bad);
                nb = line_or<VL>(nb);
                if (g == 0 && active && live) {
                    const int X = x1 + a.minX1;
                    int d1 = (a.minD - 1) * 16;
                    if (!bad && minS < 32767) {
                        const int x2 = X - best - a.minD;
                        atomicMin(a.key2 + ((size_t)pair * H + y) * a.W + x2,
                                  ((uint32_t)minS << 16) | (uint32_t)(0xFFFF - X));
                        int d16;
                        if (best > 0 && best < D - 1) {
                            const int Sm = (int)(nb & 0xFFFF), Sq = (int)(nb >> 16);
                            const int den = max(Sm + Sq - 2 * minS, 1);
                            d16 = best * 16 + ((Sm - Sq) * 16 + den) / (den * 2);  // C truncation
                        } else {
                            d16 = best * 16;
                        }
                        d1 = d16 + a.minD * 16;
                    }
                    a.disp[((size_t)pair * H + y) * a.W + X] = (int16_t)d1;
                }
            }
            lds_barrier();
        }
    }
}

#if !defined(SWEEP_MODE) || SWEEP_MODE == 0  // one unit owns the non-template kernel
// LR consistency (disp12MaxDiff) against the disp2 keys of the whole row:
// same test as k_wta's tail (sm_paths.hpp); columns outside [minX1, maxX1)
// are INVALID.  blockIdx = (x tile, y, pair).
__global__ void __launch_bounds__(256) k_lr_check(const int16_t* __restrict__ pre, const uint32_t* __restrict__ key2,
                                                  int16_t* __restrict__ out, int H, int W, int minD, int minX1, int maxX1,
                                                  int disp12)
{
    const int X = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (X >= W) return;
    const size_t row = ((size_t)blockIdx.z * H + y) * W;
    const int INVALID = (minD - 1) * 16;
    int d1 = INVALID;
    if (X >= minX1 && X < maxX1) {
        d1 = pre[row + X];
        if (d1 != INVALID) {
            const int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
            const int _x = X - _d, x_ = X - d_;
            bool rej1 = false, rej2 = false;
            if (_x >= 0 && _x < W) {
                const uint32_t kk = key2[row + _x];
                const int d2 = kk == 0xFFFFFFFFu ? INVALID : (int)(0xFFFF - (kk & 0xFFFF)) - _x;
                rej1 = d2 >= minD && abs(d2 - _d) > disp12;
            }
            if (x_ >= 0 && x_ < W) {
                const uint32_t kk = key2[row + x_];
                const int d2 = kk == 0xFFFFFFFFu ? INVALID : (int)(0xFFFF - (kk & 0xFFFF)) - x_;
                rej2 = d2 >= minD && abs(d2 - d_) > disp12;
            }
            if (rej1 && rej2) d1 = INVALID;
        }
    }
    out[row + X] = (int16_t)d1;
}
#endif

}  // namespace smk
