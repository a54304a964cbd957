// sm_sweep2.hpp — fused sweeps with a column-per-lane layout (gfx950): a
// measured ablation of k_sweep (sm_sweep.hpp), selected by debug flags 128 /
// 1 << 27 (sm_api.hip sweep_variant), bit-exact, slower at the headline's
// 8 pairs per launch.
//
// Same algorithm, inputs, outputs and strip hand-off protocol as k_sweep;
// what changes is where a cell lives.  k_sweep gives a column VL = 16 adjacent
// lanes (8 disparities each), so every direction's minimum over d is a 4-step
// DPP reduction per column and every diagonal predecessor crosses lanes
// through an LDS row with a workgroup barrier.  Here a wave holds CPW = 16 or
// 8 adjacent columns: lane = column c + CPW * part, and a lane keeps its
// column's disparities [part*DQ, (part+1)*DQ) as NP = DQ/2 u16 pairs.
//   * diagonal predecessors (x -+ 1, previous row) are one DPP row_shr:1 /
//     row_shl:1 per word (CPW = 8: plus a select at the half-row edge); the
//     wave's edge lane takes the neighbouring wave's edge column (LDS,
//     double-buffered by row parity) as the DPP `old` operand;
//   * the minimum over d is an in-lane tree plus row_ror:8 (CPW = 8) and two
//     cross-row swaps (v_permlane16_swap, v_permlane32_swap);
//   * the d -+ 1 neighbours across a part boundary come from the neighbouring
//     part's lane through ds_bpermute (two words per direction).
// The wave issues about 25 % fewer VALU instructions than k_sweep (PMC), but a
// 16-column wave leaves one wave per SIMD at 8 KITTI pairs and its VALU ~43 %
// busy; with 8 columns the down sweep wins at 16 pairs per launch only.
//
// Strips: a workgroup holds NW compute waves = CPW*NW columns, the first and
// last HB = 4 of which are halos; at every HB-row block boundary the halo
// lanes' A (+dx) / B (-dx) state is replaced by the neighbouring strips' own
// state of the block's last row (tagged granules, polled by a dedicated wave:
// the k_sweep protocol, MI355X guide §6 G16 form R2).  Inside a block a halo
// column goes stale one column per row from the outer edge, which never
// reaches an own column within HB rows.
#pragma once
#include <type_traits>

#include "sm_pk.hpp"
#include "sm_sweep.hpp"

namespace smk {

template <int NW, int CPW, int NP>
struct Sweep2Geo {
    static constexpr int PARTS = 64 / CPW;        // lanes per column (disparity parts)
    static constexpr int HB = 4;                  // rows per block = halo columns per side
    static constexpr int NCOL = CPW * NW;         // columns held by the compute waves
    static constexpr int CW = NCOL - 2 * HB;      // own columns per strip
    static constexpr int DQ = 2 * NP;             // disparities per lane
    static constexpr int D = PARTS * DQ;
    static constexpr int THREADS = (NW + 1) * 64; // + the poller wave
    static constexpr int NPUB = HB * PARTS;       // publishing lanes per (strip, direction)
    static constexpr int NGR = NPUB * (NP + 1);   // granules per (strip, direction, block)
};

constexpr int DPP_ROW_ROR8 = 0x128;  // lane i <- lane (i + 8) mod 16 within the row

// minimum / sum over the lanes of a column (lanes c + CPW * part): row_ror:8 pairs the
// two parts of a DPP row (CPW = 8), the swaps the rows
template <int CPW>
__device__ __forceinline__ uint32_t quarter_min(uint32_t v)
{
    if constexpr (CPW == 8) v = ::min(v, perm_dpp<DPP_ROW_ROR8>(v));
    const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = ::min(a[0], a[1]);
    const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return ::min(b[0], b[1]);
}
template <int CPW>
__device__ __forceinline__ uint32_t quarter_sum(uint32_t v)
{
    if constexpr (CPW == 8) v += perm_dpp<DPP_ROW_ROR8>(v);
    const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = a[0] + a[1];
    const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return b[0] + b[1];
}

// one packed recurrence step for the quarter layout: P = predecessor vector,
// pm = its full-column minimum; returns the new column minimum
template <int CPW, int NP>
__device__ __forceinline__ uint32_t step_q(const uint32_t (&P)[NP], uint32_t pm, const uint32_t (&C)[NP], uint32_t P1p,
                                           uint32_t P2, int q, uint32_t (&Ln)[NP])
{
    constexpr uint32_t EDGE = kBig | (kBig << 16);
    constexpr int PARTS = 64 / CPW;
    const int lane = threadIdx.x & 63;
    uint32_t lm = (uint32_t)__builtin_amdgcn_ds_bpermute(((lane - CPW) & 63) * 4, (int)P[NP - 1]);
    uint32_t lq = (uint32_t)__builtin_amdgcn_ds_bpermute(((lane + CPW) & 63) * 4, (int)P[0]);
    lm = q == 0 ? EDGE : lm;          // its high half is d - 1 of element 0
    lq = q == PARTS - 1 ? EDGE : lq;  // its low half is d + 1 of the last element
    const uint32_t mm = pm * 0x10001u, dl = (pm + P2) * 0x10001u;
    uint32_t a1 = __builtin_amdgcn_alignbit(P[0], lm, 16);
#pragma unroll
    for (int k = 0; k < NP; k++) {
        const uint32_t a2 = __builtin_amdgcn_alignbit(k + 1 < NP ? P[k + 1] : lq, P[k], 16);
        uint32_t v = pk_min(pk_add(pk_min(a1, a2), P1p), P[k]);
        v = pk_min(v, dl);
        Ln[k] = pk_add(C[k], pk_sub(v, mm));
        a1 = a2;
    }
    uint32_t t[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) t[k] = Ln[k];
#pragma unroll
    for (int w = 1; w < NP; w *= 2)
#pragma unroll
        for (int k = 0; k + w < NP; k += 2 * w) t[k] = pk_min(t[k], t[k + w]);
    return quarter_min<CPW>(::min(t[0] & 0xFFFFu, t[0] >> 16));
}

template <int NWORDS>
__device__ __forceinline__ void lds_get_w(const uint32_t* p, uint32_t (&v)[NWORDS])
{
    static_assert(NWORDS % 4 == 0, "b128 chunks");
#pragma unroll
    for (int k = 0; k < NWORDS / 4; k++) {
        const uint4 x = reinterpret_cast<const uint4*>(p)[k];
        v[4 * k] = x.x; v[4 * k + 1] = x.y; v[4 * k + 2] = x.z; v[4 * k + 3] = x.w;
    }
}
template <int NWORDS>
__device__ __forceinline__ void lds_put_w(uint32_t* p, const uint32_t (&v)[NWORDS])
{
#pragma unroll
    for (int k = 0; k < NWORDS / 4; k++)
        reinterpret_cast<uint4*>(p)[k] = make_uint4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
}

template <int NW, int CPW, int NP, typename CT, int MODE, int PF>
__global__ void __launch_bounds__((Sweep2Geo<NW, CPW, NP>::THREADS)) k_sweep2(SweepArgs a)
{
    using G = Sweep2Geo<NW, CPW, NP>;
    constexpr int PARTS = G::PARTS, NPUB = G::NPUB;
    constexpr bool UP = MODE == 2;
    constexpr bool WTA = MODE != 0;
    constexpr int HB = G::HB, NCOL = G::NCOL, CW = G::CW, DQ = G::DQ, D = G::D, NGR = G::NGR;
    constexpr int CB = DQ * (int)sizeof(CT);  // cost / E / W bytes per lane and row
    static_assert(NP % 4 == 0, "LDS edge rows move in b128 chunks");
    // edge columns between the waves: [buf][A, B][slot][quarter][word]; A slot w+1 =
    // wave w's column 15, slot 0 = zero; B slot w+1 = wave w's column 0, slot NW+1 = zero
    __shared__ __attribute__((aligned(16))) uint32_t edge[2][2][NW + 2][PARTS][NP];
    __shared__ uint32_t emin[2][2][NW + 2];
    // halo snapshot from the neighbouring strips: [A, B][halo column][quarter][word]
    __shared__ __attribute__((aligned(16))) uint32_t stage[2][HB][PARTS][NP];
    __shared__ uint32_t smin[2][HB];
    // WTA sweeps: the row's aggregated costs S per own column (sub-pixel neighbours)
    __shared__ __attribute__((aligned(16))) uint16_t srow[WTA ? NW : 1][WTA ? CPW : 1][WTA ? D : 2];

    for (int i = threadIdx.x; i < 2 * 2 * (NW + 2) * PARTS * NP; i += G::THREADS) (&edge[0][0][0][0][0])[i] = 0;
    for (int i = threadIdx.x; i < 2 * 2 * (NW + 2); i += G::THREADS) (&emin[0][0][0])[i] = 0;
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wg = blockIdx.x, pair = blockIdx.y;
    const int H = a.H, W1 = a.W1;
    const int nblk = (H + HB - 1) / HB;
    const bool has_left = wg > 0, has_right = wg + 1 < a.nwg;
    const uint32_t tag0 = a.epoch << 16;
    unsigned long long* hopp = a.hop + (size_t)pair * a.hop_pair;
    auto gbase = [&](int strip, int dir, int b) -> size_t { return ((size_t)(strip * 2 + dir) * nblk + b) * NGR; };

    if (wave == NW) {
        // ---- poller: one lane per publishing lane of a neighbour (NPUB <= 32 per direction)
        const int dir = lane >> 5, p = lane & 31;  // p < NPUB: publisher lane (column p % HB, part p / HB)
        const bool need = p < NPUB && (dir == 0 ? has_left : has_right);
        const int src_strip = need ? (dir == 0 ? wg - 1 : wg + 1) : wg;
        bool dead = (a.dbg & 1) != 0;
        for (int b = 0; b < nblk; b++) {
#pragma unroll 1
            for (int j = 0; j < HB; j++) lds_barrier();
            if (b + 1 < nblk) {
                if ((has_left || has_right) && !(a.dbg & 2)) {  // wave-uniform
                    uint32_t v[NP + 1];
                    const gu64* src = (const gu64*)(hopp + gbase(src_strip, dir, b) + (size_t)(p % NPUB) * (NP + 1));
                    poll_granules<NP + 1>(src, need, tag0 | (uint32_t)(b + 1), v, dead, a.err);
                    if (need) {
                        const int col = p % HB, qq = p / HB;
                        uint32_t w[NP];
#pragma unroll
                        for (int t = 0; t < NP; t++) w[t] = v[t];
                        lds_put_w<NP>(&stage[dir][col][qq][0], w);
                        if (qq == 0) smin[dir][col] = v[NP];
                    }
                }
                lds_barrier();
            }
        }
        return;
    }

    // ---- compute waves
    const int c = lane % CPW, q = lane / CPW;
    const int j = wave * CPW + c;             // strip-local column
    const int x1 = wg * CW - HB + j;
    const bool active = x1 >= 0 && x1 < W1;
    const bool own = j >= HB && j < NCOL - HB;
    const int wx0 = wg * CW - HB + wave * CPW;
    const bool wave_ragged = wx0 < 0 || wx0 + CPW > W1;  // wave-uniform
    const uint32_t P1p = (uint32_t)a.P1 * 0x10001u, P2 = (uint32_t)a.P2;
    // publishing lanes at block ends: A from the last wave's last HB own columns,
    // B from the first wave's first HB own columns (index p = column + 4 * quarter)
    const bool pubA = wave == NW - 1 && c >= CPW - 2 * HB && c < CPW - HB && has_right;
    const bool pubB = wave == 0 && c >= HB && c < 2 * HB && has_left;
    const int pidx = (pubA ? c - (CPW - 2 * HB) : c - HB) + HB * q;
    const bool haloA = wave == 0 && c < HB && has_left;               // left halo: A refreshed per block
    const bool haloB = wave == NW - 1 && c >= CPW - HB && has_right;  // right halo: B refreshed

    const uint64_t cells = (uint64_t)H * W1 * D;
    const rsrc_t rc = make_rsrc(a.cost + (size_t)pair * a.cost_pair, cells * sizeof(CT));
    rsrc_t re = make_rsrc(nullptr, 0), rw = re, rp = re, rrec = re, rnb = re;
    if constexpr (WTA) {
        re = make_rsrc(a.ew + (size_t)pair * a.ew_pair, cells * sizeof(CT));
        rw = make_rsrc(a.ew + (size_t)pair * a.ew_pair + a.ew_slot, cells * sizeof(CT));
        rrec = make_rsrc(a.rec + (size_t)pair * H * a.W, (uint64_t)H * a.W * 4);
        rnb = make_rsrc(a.nb + (size_t)pair * H * a.W, (uint64_t)H * a.W * 4);
    }
    const int ku = 100 - a.uniq;
    if constexpr (MODE != 1) rp = make_rsrc((const uint8_t*)a.part + (size_t)pair * a.part_pair, cells * 2);
    const rsrc_t rhop = make_rsrc(hopp, (uint64_t)a.hop_pair * 8);
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    auto cell = [&](int y) -> uint32_t {
        return active ? ((uint32_t)y * (uint32_t)W1 + (uint32_t)x1) * (uint32_t)D + (uint32_t)(q * DQ) : NONE;
    };
    auto boff = [&](uint32_t e, int bytes) -> uint32_t { return e == NONE ? kOOB : e * (uint32_t)bytes; };

    uint32_t LA[NP], LB[NP], LV[NP];
#pragma unroll
    for (int i = 0; i < NP; i++) LA[i] = LB[i] = LV[i] = 0;
    uint32_t mA = 0, mB = 0, mV = 0;

    RawBytes<CB> rc_[PF], re_[PF], rw_[PF];
    RawBytes<DQ * 2> rp_[PF];
    auto issue = [&](int k, int s) {  // loads of step s into ring slot k (rows past the end read 0)
        const uint32_t en = s < H ? cell(UP ? H - 1 - s : s) : NONE;
        const uint32_t eo = own ? en : NONE;
        rc_[k].load(rc, boff(en, sizeof(CT)));
        if constexpr (WTA) {
            re_[k].load(re, boff(eo, sizeof(CT)));
            rw_[k].load(rw, boff(eo, sizeof(CT)));
        }
        if constexpr (MODE == 2) rp_[k].load(rp, boff(eo, 2));
    };
#pragma unroll
    for (int k = 0; k < PF; k++) issue(k, k);

    for (int b = 0; b < nblk; b++) {
#pragma unroll
        for (int jr = 0; jr < HB; jr++) {
            const int k = jr % PF;
            const int s = b * HB + jr;
            const bool live = s < H;
            const int y = UP ? H - 1 - s : s;
            const int rb = (s + 1) & 1, wb = s & 1;
            uint32_t C[NP], Ein[NP], Win[NP], Pin[NP];
            unpack_ct_pk<CT, DQ>(rc_[k], C);
            if constexpr (WTA) {
                unpack_ct_pk<CT, DQ>(re_[k], Ein);
                unpack_ct_pk<CT, DQ>(rw_[k], Win);
            }
            if constexpr (MODE == 2) unpack_ct_pk<uint16_t, DQ>(rp_[k], Pin);
#pragma unroll
            for (int i = 0; i < NP; i++) {  // materialise before the refill (sm_sweep.hpp)
                asm volatile("" : "+v"(C[i])::"memory");
                if constexpr (WTA) asm volatile("" : "+v"(Ein[i]), "+v"(Win[i])::"memory");
                if constexpr (MODE == 2) asm volatile("" : "+v"(Pin[i])::"memory");
            }
            issue(k, s + PF);

            // diagonal predecessors: column c-1 (A) / c+1 (B) of the previous row
            uint32_t eA[NP], eB[NP], PA[NP], PB[NP];
            lds_get_w<NP>(&edge[rb][0][wave][q][0], eA);
            lds_get_w<NP>(&edge[rb][1][wave + 2][q][0], eB);
            const uint32_t emA = emin[rb][0][wave], emB = emin[rb][1][wave + 2];
            // (CPW = 8: a DPP row holds two parts, so the shift is fixed up at c = 0 / CPW-1)
            const bool firstc = CPW == 8 && c == 0, lastc = CPW == 8 && c == CPW - 1;
#pragma unroll
            for (int i = 0; i < NP; i++) {
                PA[i] = dpp<DPP_ROW_SHR1>(eA[i], LA[i]);
                PB[i] = dpp<DPP_ROW_SHL1>(eB[i], LB[i]);
                if constexpr (CPW == 8) {
                    PA[i] = firstc ? eA[i] : PA[i];
                    PB[i] = lastc ? eB[i] : PB[i];
                }
            }
            uint32_t pmA = dpp<DPP_ROW_SHR1>(emA, mA), pmB = dpp<DPP_ROW_SHL1>(emB, mB);
            if constexpr (CPW == 8) {
                pmA = firstc ? emA : pmA;
                pmB = lastc ? emB : pmB;
            }
            uint32_t nA[NP], nB[NP], nV[NP];
            uint32_t mnA = step_q<CPW, NP>(PA, pmA, C, P1p, P2, q, nA);
            uint32_t mnB = step_q<CPW, NP>(PB, pmB, C, P1p, P2, q, nB);
            const uint32_t mnV = step_q<CPW, NP>(LV, mV, C, P1p, P2, q, nV);
            if (wave_ragged) {  // columns outside [0, W1) stay at the entering state
#pragma unroll
                for (int i = 0; i < NP; i++) {
                    nA[i] = active ? nA[i] : 0u;
                    nB[i] = active ? nB[i] : 0u;
                    nV[i] = active ? nV[i] : 0u;
                }
                mnA = active ? mnA : 0u;
                mnB = active ? mnB : 0u;
            }
            // edge columns for the neighbouring waves (next row reads buffer wb)
            if (c == CPW - 1) {
                lds_put_w<NP>(&edge[wb][0][wave + 1][q][0], nA);
                if (q == 0) emin[wb][0][wave + 1] = mnA;
            }
            if (c == 0) {
                lds_put_w<NP>(&edge[wb][1][wave + 1][q][0], nB);
                if (q == 0) emin[wb][1][wave + 1] = mnB;
            }
            // snapshot of the block's last row for the neighbouring strips' halos
            if (jr == HB - 1 && b + 1 < nblk && (wave == 0 || wave == NW - 1)) {  // wave-uniform
                const bool pub = pubA || pubB;
                const uint32_t tag = tag0 | (uint32_t)(b + 1);
                const uint32_t o = pub ? (uint32_t)((gbase(wg, pubA ? 0 : 1, b) + (size_t)pidx * (NP + 1)) * 8) : kOOB;
#pragma unroll
                for (int t = 0; t < NP; t++)
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{pubA ? nA[t] : nB[t], tag}, rhop, o + 8 * t, 0, 16);
                __builtin_amdgcn_raw_buffer_store_b64(u32x2{pubA ? mnA : mnB, tag}, rhop, o + 8 * NP, 0, 16);
            }

            const uint32_t e = live && own ? cell(y) : NONE;
            if constexpr (MODE == 0) {
                uint32_t out[NP];
#pragma unroll
                for (int i = 0; i < NP; i++) out[i] = pk_add(pk_add(nV[i], nA[i]), nB[i]);
                bstore_n<uint32_t, NP>(rp, boff(e, 2), out);
            } else {
                uint32_t Sp[NP];
                uint32_t key = 0xFFFFFFFFu;
#pragma unroll
                for (int i = 0; i < NP; i++) {
                    uint32_t t = pk_adds(pk_adds(pk_adds(pk_adds(nV[i], nA[i]), nB[i]), Ein[i]), Win[i]);
                    if constexpr (MODE == 2) t = pk_adds(t, Pin[i]);
                    t = pk_min(t, 0x7FFF7FFFu);  // min(sum, 32767)
                    Sp[i] = t;
                    const int d0 = q * DQ + 2 * i;
                    key = min(key, min((t << 16) | wta_rank(d0, MODE == 1), (t & 0xFFFF0000u) | wta_rank(d0 + 1, MODE == 1)));
                }
                lds_put_w<NP>(reinterpret_cast<uint32_t*>(&srow[wave][c][q * DQ]), Sp);
                key = quarter_min<CPW>(key);
                const uint32_t minS = key >> 16;
                const int best = wta_unrank(key & 0xFFFF, MODE == 1);  // MODE 1 = 5 paths
                const int bm = max(best - 1, 0), bq = min(best + 1, D - 1);
                const uint32_t Sm = srow[wave][c][bm];
                const uint32_t Sq = srow[wave][c][bq];
                bool ok;
                if (ku > 0) {
                    // uniqueness: S*ku < 100*minS  <=>  S < T = ceil(100*minS / ku); the pixel
                    // passes iff only best-1, best, best+1 are below T (sm_sweep.hpp)
                    const uint32_t lim = minS * 100u;
                    uint32_t T = 0xFFFFu;
                    if (lim <= 0xFFFFu * (uint32_t)ku) {
                        T = (uint32_t)((float)lim * a.inv_ku);
                        T += __umul24(T, (uint32_t)ku) < lim ? 1u : 0u;
                        T -= (T > 0 && __umul24(T - 1, (uint32_t)ku) >= lim) ? 1u : 0u;
                    }
                    const uint32_t Tp = T * 0x10001u;
                    uint32_t cp = 0;
#pragma unroll
                    for (int i = 0; i < NP; i++)
                        cp = pk_add(cp, pk_min(pkw(__builtin_elementwise_sub_sat(pkv(Tp), pkv(Sp[i]))), 0x10001u));
                    const uint32_t cnt = quarter_sum<CPW>((cp & 0xFFFFu) + (cp >> 16));
                    const uint32_t win = (minS < T ? 1u : 0u) + (best > 0 && Sm < T ? 1u : 0u) +
                                         (best < D - 1 && Sq < T ? 1u : 0u);
                    ok = cnt == win;
                } else {
                    uint32_t far = 0;
                    const int gb = q * DQ - best + 1;
#pragma unroll
                    for (int i = 0; i < NP; i++) {
                        const uint32_t lo = Sp[i] & 0xFFFFu, hi = Sp[i] >> 16;
                        far = max(far, (int)lo * ku < (int)minS * 100 ? (uint32_t)(gb + 2 * i) : 0u);
                        far = max(far, (int)hi * ku < (int)minS * 100 ? (uint32_t)(gb + 2 * i + 1) : 0u);
                    }
                    far = quarter_min<CPW>(~far);  // max over the parts
                    ok = ~far <= 2u;
                }
                ok = ok && minS < 32767u;
                const uint32_t recw = ok ? ((minS << 16) | (uint32_t)best) : 0xFFFFFFFFu;
                const uint32_t nbw = Sm | (Sq << 16);
                const bool wpx = q == 0 && own && active && live;
                const uint32_t px = (uint32_t)y * (uint32_t)a.W + (uint32_t)(x1 + a.minX1);
                __builtin_amdgcn_raw_buffer_store_b32(recw, rrec, wpx ? px * 4 : kOOB, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b32(nbw, rnb, wpx ? px * 4 : kOOB, 0, 0);
            }
#pragma unroll
            for (int i = 0; i < NP; i++) {
                LA[i] = nA[i];
                LB[i] = nB[i];
                LV[i] = nV[i];
            }
            mA = mnA;
            mB = mnB;
            mV = mnV;
            lds_barrier();
        }
        if (b + 1 < nblk) {
            lds_barrier();  // the poller has written the halo snapshot
            if (haloA) {
                lds_get_w<NP>(&stage[0][c][q][0], LA);
                mA = smin[0][c];
            }
            if (haloB) {
                lds_get_w<NP>(&stage[1][c - (CPW - HB)][q][0], LB);
                mB = smin[1][c - (CPW - HB)];
            }
        }
    }
}

}  // namespace smk
