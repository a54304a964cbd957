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
// and the other sweep's partial and runs the WTA / uniqueness / sub-pixel
// step in place (disp2 + the LR check follow in k_lr_rows).  Traffic per cell
// (census, 8 paths): cost 1 B written, 4 B read (E, W, down, up), E/W 2 B
// written + 2 B read, partial 2 + 2 B = 13 B.
//
// Decomposition.  A workgroup owns a strip of CW adjacent columns of one pair
// for all rows.  Its compute waves hold NCW*LPW columns (LPW = 64/VL columns
// per wave, VL lanes per column, DPL = D/VL disparities per lane): wave 0 is
// a LEFT HALO (the neighbour strip's last LPW columns, direction A = +dx only),
// waves 1..NCW-2 are the strip's own columns, wave NCW-1 is a RIGHT HALO (the
// next strip's first LPW columns, direction B = -dx only).  The vertical path
// is private to a lane group; the diagonals read the previous row's L vector
// of the neighbouring column through a double-buffered LDS row (one LDS-only
// barrier per row).
//
// Trapezoid exchange.  Rows run in blocks of HB = LPW.  At a block boundary
// the halo columns' A / B state is replaced by the neighbouring strips' own
// state of the block's last row; inside the block a halo column's value goes
// stale one column per row from the outer edge in, which never reaches an own
// column within HB rows.  So strips hand each other one LPW-column snapshot
// per HB rows (tagged 8-byte granules written `sc1`, polled `sc1`: MI355X guide
// §6 Guideline 16 form R2) instead of one column per row.  A dedicated POLLER
// wave does the polling and writes the snapshot into the halo columns' LDS
// slots between two barriers: it issues no other memory operation, so its
// vmcnt waits never drain the compute waves' load rings.  All workgroups of a
// pair must be co-resident (the host sizes the grid from the occupancy query);
// every poll is bounded (timeout -> error word, never a hang).
//
// Recurrence and domain exactly as sm_paths.hpp / oracle/sgm_np.py: a path
// enters [minX1, maxX1) x [0, H) with Lp = 0 and minLp = 0 (columns outside
// the domain hold the zero state).
#pragma once
#include "sm_common.hpp"
#include "sm_sweep_host.hpp"
#include "sm_pk.hpp"

#include <type_traits>

namespace smk {

typedef __attribute__((address_space(1))) unsigned long long gu64;

constexpr uint32_t SW_SPIN_LIMIT = 1u << 19;

// SWEEP_STATS builds (tools/build_variant.sh): shader-clock cycles each wave spends in
// the row / block synchronisation, summed per mode into SweepArgs::stats[8 * MODE + k]
// (MODE 3's line waves, words 40..44: 40 own waves in wait_lines, 41 line waves in wait_cons,
// 42 line waves in barriers, 43 line waves' lifetime, 44 line waves):
// 0 poller in polls, 1 poller in barriers, 2 compute waves in wait_row, 3 compute waves
// in block barriers, 4 compute waves' lifetime, 5 compute waves, 6 poller lifetime
#if SWEEP_STATS
#define SW_T0(v) const uint64_t v = __builtin_readcyclecounter()
#define SW_ACC(acc, v) acc += __builtin_readcyclecounter() - v
#else
#define SW_T0(v) (void)0
#define SW_ACC(acc, v) (void)0
#endif

// cache policy of the sweeps' read-once streams (E/W and partial loads, partial and E/W
// stores): nt (2) keeps them from evicting the cost volume the other passes re-read (census8
// sweeps 259.5 -> 256.1, sgbm5 259.8 -> 257.9, sgbm8 328.7 -> 323.9 us per pair); 0 = default
#ifndef SWEEP_STREAM_AUX
#define SWEEP_STREAM_AUX 2
#endif

// cache policy of the WTA sweep's cost loads (the cost volume's last reader): 0 = default
#ifndef SWEEP_COST_AUX
#define SWEEP_COST_AUX 0
#endif

// row synchronisation inside a block of HB rows: 1 = each wave waits for its two neighbours'
// published rows (LDS counters; modes 0 and 2), 0 = a workgroup barrier per row
#ifndef SWEEP_ROW_SYNC
#define SWEEP_ROW_SYNC 1
#endif
#ifndef SWEEP_ROW_SLEEP
#define SWEEP_ROW_SLEEP 1  // s_sleep between polls of the neighbours' row counters
#endif

// build-time switch back to the u32 recurrence for every DPL (comparison builds)
#ifndef SWEEP_U32
#define SWEEP_U32 0
#endif
// census (u8 costs): the packed recurrence in the f16 form (sm_pk.hpp sweep_step_h16)
#ifndef SWEEP_H16
#define SWEEP_H16 1
#endif
// census (f16 form): deferred subtraction of the previous row's minimum (sm_pk.hpp
// sweep_step2n DS): the path states run unnormalised, each sum of paths subtracts the input
// minima once, and every state is renormalised (R - min R) at least every SWEEP_DS_RN rows /
// line steps, which keeps every value below 2^11: after k steps R <= 62 k + 62 + P2 and the
// step's largest intermediate adds P1 (P2 <= 193, P1 < P2: k <= 25)
#ifndef SWEEP_DS
#define SWEEP_DS 1
#endif
#ifndef SWEEP_DS_LINES
#define SWEEP_DS_LINES 1  // the MODE 3 line waves too (their ring offsets beside the ring)
#endif
#ifndef SWEEP_DS_LANE0
#define SWEEP_DS_LANE0 0
#endif
#define SWEEP_DS_RN 16
static_assert(62 * SWEEP_DS_RN + 62 + 193 + 192 < 2048, "DS renormalisation interval too long for the f16 form");
// packed row loops: the recurrences that wait on the LDS row (A and B of an own wave, the
// column sets of a halo wave) issued interleaved (sm_pk.hpp sweep_step2n: no wait states
// between dependent VOP3P operations)
#ifndef SWEEP_STEPN
#define SWEEP_STEPN 1
#endif
#ifndef SWEEP_LDS_FIRST
#define SWEEP_LDS_FIRST 1  // a scheduling barrier after the row's LDS reads (see the row loop)
#endif

// NCW: compute waves per workgroup (left halo, NCW-2 own, right halo).  Every strip
// recomputes 2 halo waves' columns, so wider strips cost fewer instructions per own
// column; they also hold more waves per workgroup (fewer blocks per CU) and give fewer
// strips per pair.  Measured (KITTI D = 128, 8 pairs, profiles/r02/ablations/sweep_ncw_*):
// census8 sweeps 244 -> 217 us per pair at NCW 7 -> 11, sgbm5 247 -> 235, sgbm8 321 -> 287
// at NCW 13 (u16 costs); 9, 12, 14 and 15 are slower (the strip count against 256 CUs).
constexpr int kNarrowNcw = 7;
// latency instances (a launch of one or two pairs, or a pair on half the CUs: DESIGN.md §4.3):
// 3 own waves and single-set halos, so a KITTI pair's strips spread over ~90 CUs at D = 160
#ifndef SWEEP_LAT_NCW
#define SWEEP_LAT_NCW 5
#endif
constexpr int kLatNcw = SWEEP_LAT_NCW;
constexpr bool lat_built(int D) { return D % 32 == 0 && D >= 64 && D <= 224; }  // D = 256 spills
// HM: column sets per halo wave in the packed row loops.  A halo of HM*LPW columns stays
// exact for HM*LPW rows after a snapshot, so the strips hand off once per HM*LPW rows; the
// hand-off latency (us under the sweeps' streaming traffic, SWEEP_STATS) is paid half as
// often at HM = 2, for halo waves that step two column sets of their one direction.
#ifndef SWEEP_HM
#define SWEEP_HM 2
#endif
template <int VL, int DPL, int NCW_ = kNarrowNcw>
struct SweepGeo {
    static constexpr int LPW = 64 / VL;             // columns per wave (per column set)
    // column sets per halo wave (1 where fewer than 2 * SWEEP_HM own waves would publish the two
    // sides' snapshots: the latency instances' 2-3 own waves)
    static constexpr int HM = (DPL % 2 == 0 && !SWEEP_U32 && NCW_ >= 2 + 2 * SWEEP_HM) ? SWEEP_HM : 1;
    static constexpr int NCW = NCW_;                // compute waves: left halo, NCW-2 own, right halo
    static constexpr int THREADS = (NCW + 1) * 64;  // + the poller wave
    static constexpr int HW = HM * LPW;             // halo columns per side
    static constexpr int HB = HW;                   // rows per block = halo width
    static constexpr int NCOL = (NCW - 2) * LPW + 2 * HW;  // columns held by the compute waves
    static constexpr int COLS = NCOL + 2;           // + one never-written zero column each side
    static constexpr int CW = (NCW - 2) * LPW;      // own columns per workgroup
    static constexpr int D = VL * DPL;
    static constexpr int NG = (DPL + 1) / 2;        // granules per lane (two u16 per granule)
    // snapshot record of one (strip, direction, block): the HW boundary columns' states,
    // granule r = (q * HW + column) * VL + lane slice (q: the slice's q-th u16 pair), so
    // that each producer store instruction and each poller load instruction covers 64
    // consecutive granules, then one granule per column with its minimum
    static constexpr int NDAT = NG * HW * VL;
    static constexpr int SNG = NDAT + HW;           // granules per record
    // rows of inputs in flight per lane (a divisor of HB: the ring slot is the row's index in
    // its block); 2 where the wide strips' register budget needs it (12 waves, <= 168 VGPRs)
    // (32-lane lines: 2, so the 16-wave D = 256 instance stays within 128 VGPRs)
    static constexpr int PF = ((DPL >= 10 && NCW_ >= 11) || VL == 32) ? 2 : 4;
    static_assert(NCW - 2 >= 2 * HM, "the snapshot's own waves of the two sides are distinct");
    static_assert(HB % PF == 0, "the input ring is indexed by the row within a block");
};

// wide strips where every mode's instance keeps its registers at the wide block size
// (12 waves: <= 168 VGPRs, 14 waves: <= 128): NCW 11 for u8 costs, 13 for u16 costs where
// it fits (D = 128 needs up to 140 VGPRs in the per-role row loops of round 3: 11), else
// 11; 0 = not built (the host also checks for scratch and
// occupancy before it picks a wide instance, sm_sweep.hip)
constexpr int wide_ncw(int D, int ct_bytes)
{
    // D = 256 (u8): 32-lane lines (8 disparities per lane, as KITTI's 16-lane D = 128 lines)
    // in 16-wave workgroups of 13 own waves x 2 columns.  The 16-lane D = 256 instance needs
    // 183 / 219 VGPRs (modes 0 / 2): two waves per SIMD, one 8-wave strip per CU, and at
    // Middlebury width (2624 columns, 132 narrow strips) one pair per launch; this one fits
    // 4 waves per SIMD and 101 strips, i.e. two pairs per launch
    if (ct_bytes == 1 && D == 256) return 15;
    if (ct_bytes == 1) return (D <= 96 || D == 128 || D == 160 || D == 192) ? 11 : 0;
    if (D == 16 || D == 32 || D == 96) return 13;
    return (D == 48 || D == 80 || D == 128 || D == 160) ? 11 : 0;
}

// ---- MODE 3: the horizontal paths inside the down sweep.  NLW extra
// waves per workgroup run each row's E and W lines over the strip's own columns, starting
// `ewarm` columns outside the strip from the zero state (a speculation: exact once the line's
// state has met the true one), and leave E + W per own column in an LDS ring of LR rows that
// the own waves add into the partial.  A line wave's batch t covers RPW rows (an E and a W
// line each); the waves take part in the compute waves' two barriers per block of HB rows,
// running at most LEAD rows ahead of the block those waves are in.  Deadlock-free for
// LR >= LEAD + RPW: before a line wave's barrier pair b it has produced every row below
// (b + 1) * HB + LEAD, for which it needed rows up to (b + 1) * HB + LEAD + RPW - 1 - LR <=
// (b + 1) * HB - 2 consumed, all of which the compute waves consume before that barrier.
#ifndef SWEEP_NLW
#define SWEEP_NLW 4  // line waves per workgroup (3: the down sweep 13 us per pair slower, 5: 4 us)
#endif
// MODE 3 without the poller wave: each halo wave polls its neighbour strip's snapshot itself at
// the block end and writes it into its own LDS slots before it publishes the block's last row,
// so the snapshot is ordered by the row counters the neighbouring own wave already waits for
// (census8 down sweep 75.3 -> 74.6 us per pair; a fifth line wave in the freed slot: 78.9)
#ifndef SWEEP_HALO_POLL
#define SWEEP_HALO_POLL 1
#endif
#ifndef SWEEP_LINE_PRIO
#define SWEEP_LINE_PRIO 2  // issue priority of the line waves (compute waves: 3 on the hand-off chain, else 1;
                           // with the counter hand-off and the halo waves polling: 1 -> 2 census8 down
                           // sweep 76.0 -> 70.5 us per pair, sgbm5 89 -> 83, 3 level with 2, 0 level
                           // with 1; with block barriers 2 had cost 9 us)
#endif
// cost loads in flight per line lane (at most; the largest divisor of CW / 2 below this, so
// that the line's phases fall on ring-chunk boundaries): the lines run ahead of the compute
// waves, so their loads are the first touch of each cost row (HBM latency, not a cache hit)
#ifndef SWEEP_LPF8
#define SWEEP_LPF8 12  // u8 costs: 2 VGPRs per slot
#endif
#ifndef SWEEP_LPF16
#define SWEEP_LPF16 12  // u16 costs: 4 VGPRs per slot
#endif
constexpr int largest_divisor_upto(int n, int cap)
{
    for (int p = cap < n ? cap : n; p > 1; p--)
        if (n % p == 0) return p;
    return 1;
}
// rows the lines run ahead of the block the compute waves are in, in blocks of HB rows (a
// whole block: the lines work on block b + 1 while the compute waves run block b)
#ifndef SWEEP_LEAD_BLOCKS
#define SWEEP_LEAD_BLOCKS 1
#endif
// MODE 3 without workgroup barriers: the block hand-off (the poller's halo write) is ordered by
// LDS counters (the halo waves' row counters -> the poller, the poller's block counter -> the
// compute waves), so the line waves never stand in an s_barrier: they fill the cycles the
// compute waves spend waiting for the neighbouring strips with E / W work, throttled only by
// the ring (any LR >= RPW is deadlock-free: the earliest unproduced batch needs only rows the
// own waves can consume without it)
#ifndef SWEEP_LINE_NOBAR
#define SWEEP_LINE_NOBAR 1
#endif
// the same counter hand-off in the sweeps without line waves (bit MODE; row-synchronised modes
// only): the strip's waves away from the halos may start a block while the halo waves wait.
// With the halo waves polling (SWEEP_HALO_POLL, no poller wave) the MODE 4 up + WTA sweep ran
// 60.6 -> 57.2 us per pair (census8), Middlebury's MODE 2 2078 -> 1951 (modes 0 / 2 with E/W
// volumes: D = 256, mc-cnn); with the poller wave it had measured level.  MODE 1 (5 paths
// without lines) keeps its row barriers (SWEEP_ROWSYNC_M1)
#ifndef SWEEP_NOBAR_MODES
#define SWEEP_NOBAR_MODES 21
#endif
constexpr int kMaxLds = 163840;  // gfx950: LDS one workgroup may declare
// neighbour-counter row sync: KITTI 8 pairs, down sweep census8 96.4 -> 92.0 us per pair,
// sgbm8 124.0 -> 120.8, census8 WTA sweep level (96.6 / 96.0); the 5-path WTA sweep is
// slower with it (95.3 -> 97.9) and keeps the row barriers
#ifndef SWEEP_ROWSYNC_M1
#define SWEEP_ROWSYNC_M1 0
#endif
// the counter hand-off (no block barriers) and, with it, the halo waves' own polling: MODE 3
// (its line waves), the other row-synchronised modes in SWEEP_NOBAR_MODES
template <int DPL, int MODE>
constexpr bool sweep_nobar()
{
    return SWEEP_ROW_SYNC && (MODE != 1 || SWEEP_ROWSYNC_M1) && DPL % 2 == 0 && !SWEEP_U32 &&
           (MODE == 3 ? SWEEP_LINE_NOBAR != 0 : ((SWEEP_NOBAR_MODES >> MODE) & 1) != 0);
}
template <int DPL, int MODE>
constexpr bool sweep_halo_poll() { return sweep_nobar<DPL, MODE>() && SWEEP_HALO_POLL; }
template <int VL, int DPL, int NCW_, int MODE, int CTB = 1>
struct LineGeo {
    using G = SweepGeo<VL, DPL, NCW_>;
    static constexpr bool ON = MODE == 3;
    // census lines with deferred subtraction (SWEEP_DS): each ring cell's E and W offsets (the
    // lines' input minima at that column) beside the ring, 8 bytes per own column and row
    static constexpr bool DSO = CTB == 1 && SWEEP_DS && SWEEP_DS_LINES && SWEEP_H16 && VL != 8;  // (8-lane lines: spills)
    static constexpr bool HPOLL = sweep_halo_poll<DPL, MODE>();
    static constexpr int POLLER = HPOLL ? 0 : 1;  // poller waves
    // at most 16 waves per workgroup (1024 threads): compute waves + poller + lines
    static constexpr int NLW = !ON ? 0 : (SWEEP_NLW < 16 - POLLER - NCW_ ? SWEEP_NLW : 16 - POLLER - NCW_);
    static constexpr int RPW = G::LPW / 2;  // rows per line wave and batch
    // LDS besides the ring: lv, lmin, the counters, a margin
    static constexpr int BASE = 8 * G::COLS * G::D + 16 * G::COLS + 4 * NCW_ + 4 * 16 + 512 + 4 * G::D;  // (+ ring padding)
    static constexpr int ROWB = G::CW * G::D * 2 + (DSO ? G::CW * 8 : 0);  // ring row: u16 E + W sums of the own columns (+ offsets)
    static constexpr int FIT = (kMaxLds - BASE) / ROWB;
    static constexpr int LEAD0 = SWEEP_LEAD_BLOCKS * G::HB;
    static constexpr int LEAD = LEAD0 + RPW <= FIT ? LEAD0 : (FIT > RPW ? (FIT - RPW) / RPW * RPW : 0);
    static constexpr int LR = SWEEP_LINE_NOBAR ? FIT : LEAD + 2 * RPW <= FIT ? LEAD + 2 * RPW : LEAD + RPW;
    static constexpr bool BUILT = ON && NLW >= 3 && DPL % 2 == 0 && !SWEEP_U32 &&
                                  (SWEEP_LINE_NOBAR ? RPW <= FIT : LEAD + RPW <= FIT) &&
                                  G::CW % 2 == 0 && G::HB % RPW == 0 && RPW >= 1;
    // ring chunk of the line loop, per cost type (a divisor of CW / 2)
    // (8-lane lines: 9, the D = 64 u8 / D = 48 u16 wide instances spilled at 12)
    template <typename CT>
    static constexpr int lpf()
    {
        return largest_divisor_upto(G::CW / 2, VL == 8 ? 9 : sizeof(CT) == 1 ? SWEEP_LPF8 : SWEEP_LPF16);
    }
};
template <int VL, int DPL, int NCW_, int MODE>
constexpr int sweep_threads()
{
    using LG = LineGeo<VL, DPL, NCW_, MODE>;
    return SweepGeo<VL, DPL, NCW_>::THREADS + 64 * (LG::NLW - (LG::HPOLL ? 1 : 0));  // (HPOLL: no poller)
}

// NP packed words of one lane <-> LDS (widest aligned chunks)
template <int NP>
__device__ __forceinline__ void lds_get_pk(const uint16_t* p, uint32_t (&v)[NP])
{
    if constexpr (NP % 4 == 0) {
#pragma unroll
        for (int k = 0; k < NP / 4; k++) {
            const uint4 q = reinterpret_cast<const uint4*>(p)[k];
            v[4 * k] = q.x; v[4 * k + 1] = q.y; v[4 * k + 2] = q.z; v[4 * k + 3] = q.w;
        }
    } else if constexpr (NP % 2 == 0) {
#pragma unroll
        for (int k = 0; k < NP / 2; k++) {
            const uint2 q = reinterpret_cast<const uint2*>(p)[k];
            v[2 * k] = q.x; v[2 * k + 1] = q.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < NP; k++) v[k] = reinterpret_cast<const uint32_t*>(p)[k];
    }
}

template <int NP>
__device__ __forceinline__ void lds_put_pk(uint16_t* p, const uint32_t (&v)[NP])
{
    if constexpr (NP % 4 == 0) {
#pragma unroll
        for (int k = 0; k < NP / 4; k++)
            reinterpret_cast<uint4*>(p)[k] = make_uint4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    } else if constexpr (NP % 2 == 0) {
#pragma unroll
        for (int k = 0; k < NP / 2; k++) reinterpret_cast<uint2*>(p)[k] = make_uint2(v[2 * k], v[2 * k + 1]);
    } else {
#pragma unroll
        for (int k = 0; k < NP; k++) reinterpret_cast<uint32_t*>(p)[k] = v[k];
    }
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
// release of global memory too: each wave would then wait (vmcnt) for its own
// just-issued global stores before every row's barrier.  Nothing global is
// exchanged inside a workgroup here, so only the LDS writes have to land first.
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// the strip's boundary waves publish their snapshot before the block-end barrier (1; 0:
// after it), and with 2 the poller also polls the neighbours' before that barrier
#ifndef SWEEP_EARLY_XCHG
#define SWEEP_EARLY_XCHG 1
#endif

// Poll N granules per lane (granule k at src[k], polled where need[k]) until every tag
// equals `tag`.  Wave-uniform exit; gives up after SW_SPIN_LIMIT passes.
template <int N>
__device__ __forceinline__ void poll_set(const gu64* const (&src)[N], const bool (&need)[N], uint32_t tag,
                                         uint32_t (&v)[N], bool& dead, uint32_t* err)
{
    for (uint32_t spins = 0;; spins++) {
        // every load unconditional (src[k] always points into the hop buffer), so the N
        // loads of a pass are in flight together: a load inside a lane-divergent branch
        // gets its own wait before the branch closes, one memory round trip per granule
        unsigned long long x[N];
#pragma unroll
        for (int k = 0; k < N; k++) x[k] = __hip_atomic_load(src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = true;
#pragma unroll
        for (int k = 0; k < N; k++) {
            v[k] = (uint32_t)x[k];
            ok &= !need[k] || (uint32_t)(x[k] >> 32) == tag;
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

// Poll N consecutive granules of one lane (the k_sweep2 ablation's layout).
template <int N>
__device__ __forceinline__ void poll_granules(const gu64* src, bool need, uint32_t tag, uint32_t (&v)[N], bool& dead,
                                              uint32_t* err)
{
    const gu64* p[N];
    bool nd[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
        p[k] = src + k;
        nd[k] = need;
    }
    poll_set<N>(p, nd, tag, v, dead, err);
}

template <int VL, int DPL, typename CT, int MODE, int NCW_ = kNarrowNcw>
__global__ void __launch_bounds__((sweep_threads<VL, DPL, NCW_, MODE>())) k_sweep(SweepArgs a)
{
    using G = SweepGeo<VL, DPL, NCW_>;
    using LG = LineGeo<VL, DPL, NCW_, MODE, (int)sizeof(CT)>;
    constexpr bool UP = MODE == 2 || MODE == 4;
    constexpr bool WTA = MODE == 1 || MODE == 2 || MODE == 4;
    constexpr bool EWIN = MODE == 1 || MODE == 2;   // E / W path volumes read (k_ew)
    constexpr bool PARTR = MODE == 2 || MODE == 4;  // the down sweep's partial read
    constexpr bool LINES = MODE == 3;               // E / W lines in the kernel (line waves)
    constexpr bool HPOLL = LG::HPOLL;               // the halo waves poll their neighbours (no poller wave)
    static_assert(!LINES || LG::BUILT, "MODE 3 instance not built for this geometry");
    static_assert(MODE < 3 || (DPL % 2 == 0 && !SWEEP_U32), "MODES 3 / 4 run the packed row loops only");
    constexpr int NTH = sweep_threads<VL, DPL, NCW_, MODE>();
    // the down sweep shares its SIMDs with the E/W kernel (8 paths): its waves take issue
    // priority, the E/W waves fill the cycles it leaves (SWEEP_PRIO 0 = default priority)
#ifndef SWEEP_PRIO
#define SWEEP_PRIO 2
#endif
    // SWEEP_DYNPRIO (packed row loops): the row hand-off chain (wait for the neighbours' row,
    // diagonal steps, LDS writes, publish) runs at issue priority PRIO_HI, an own wave's work
    // that no other wave waits for (V-independent partial sums / WTA) at PRIO_LO, so the SIMD
    // issues the chain first and fills the gaps with the rest (halo waves: chain only)
#ifndef SWEEP_DYNPRIO
#define SWEEP_DYNPRIO 1
#endif
    constexpr int PRIO_HI = 3, PRIO_LO = MODE == 0 ? 2 : 1;  // mode 0 stays above the E/W kernel
    if constexpr (MODE == 0 && SWEEP_PRIO > 0) __builtin_amdgcn_s_setprio(SWEEP_PRIO);
    constexpr bool ROWSYNC = SWEEP_ROW_SYNC && (MODE != 1 || SWEEP_ROWSYNC_M1);
    // block hand-off by LDS counters instead of the two workgroup barriers per block
    constexpr bool NOBAR = sweep_nobar<DPL, MODE>();  // (the packed row loops)
    static_assert(!LINES || ROWSYNC, "the line waves mirror the row-synchronised barrier pattern");
    constexpr int LPW = G::LPW, NCW = G::NCW, HB = G::HB, NCOL = G::NCOL, COLS = G::COLS, CW = G::CW, D = G::D;
    constexpr int NG = G::NG, SNG = G::SNG, PF = G::PF, HM = G::HM, HW = G::HW;
    constexpr int CB = DPL * (int)sizeof(CT);  // cost / E / W bytes per lane and cell
    __shared__ __attribute__((aligned(16))) uint16_t lv[2][2][COLS][D];  // [buf][A=+dx, B=-dx][col+1][d]
    __shared__ uint32_t lmin[2][2][COLS];
    // WTA sweeps: each own column's aggregated costs S of the current row
    // (wave-local; the line's first lane reads S[best-1], S[best+1] back)
    __shared__ __attribute__((aligned(16))) uint16_t srow[WTA ? NCW - 2 : 1][WTA ? LPW : 1][WTA ? D : 2];
    // rows whose LDS state each compute wave has published (inside a block of HB rows the
    // waves synchronise with their two neighbours only; SWEEP_ROW_SYNC)
    __shared__ uint32_t rowcnt[NCW];
    // MODE 3: E + W of the own columns for LR rows; batches each line wave has completed;
    // rows each own wave has consumed from the ring
    // (one D-slice of padding on each side: a line's last step prefetches the column past the
    // strip, which is never used; the padding keeps that read inside the declared array)
    constexpr int RING_D = LINES ? D : 2;
    __shared__ __attribute__((aligned(16))) uint16_t ring_pad[(LINES ? LG::LR : 1) * (LINES ? CW : 1) * RING_D + 2 * RING_D];
    auto& ring = *reinterpret_cast<uint16_t(*)[LINES ? LG::LR : 1][LINES ? CW : 1][RING_D]>(ring_pad + RING_D);
    // DS census lines: [ring row][own column][E, W] input minima (the offsets of the ring's sums)
    __shared__ __attribute__((aligned(8))) uint32_t roff[LINES && LG::DSO ? LG::LR : 1][LINES && LG::DSO ? CW : 1][2];
    __shared__ uint32_t linecnt[LINES ? LG::NLW : 1], conscnt[NCW];
    __shared__ uint32_t pollcnt;  // NOBAR: blocks whose halo snapshot the poller has written

    // the workgroup's (pair, band, strip) item: blockIdx (x = band * nwg + strip, y = pair), or
    // the XCD-aware 1-D placement (SweepArgs::xcd_per)
    int bx = blockIdx.x, by = blockIdx.y;
    if (a.xcd_per > 0) {
        const int item = (int)(blockIdx.x & 7u) * a.xcd_per + (int)(blockIdx.x >> 3);
        if (item >= a.xcd_total) return;  // padding workgroup: no strip, nothing to wait for
        const int per_pair = a.nwg * (a.nband > 1 ? a.nband : 1);
        by = item / per_pair;
        bx = item - by * per_pair;
    }
    // row band of this workgroup (MODE 3 with a.nband > 1: bx = band * nwg + strip)
    const int nband = LINES && a.nband > 1 ? a.nband : 1;
    const int band = nband > 1 ? bx / a.nwg : 0;
    const int wg = bx - band * a.nwg, pair = by;
    const int H = a.H, W1 = a.W1;
    // rows: own [y0b, y1b), computed from ys (vertical warmup rows above the band: the zero state,
    // or the test's wrong state, enters at ys); step s is row ys + s (down sweeps), s < nrow
    const int y0b = nband > 1 ? band * a.band_h : 0;
    const int y1b = nband > 1 ? min(H, y0b + a.band_h) : H;
    const int ys = band > 0 ? max(0, y0b - a.vwarm) : 0;
    const int nrow = y1b - ys, wrows = y0b - ys;  // steps, warmup steps (wave-uniform)
    const int nblk = (nrow + HB - 1) / HB;
    const int nblk_rec = nband > 1 ? a.hop_nblk : nblk;  // record stride of the hop buffer
    const bool vguess = a.vguess && band > 0;  // tests: a wrong entering state
    // the wrong state of a column slot inside the domain: (d % 5) + 3 (slot & 1), minimum 3 (slot & 1)
    auto in_domain_slot = [&](int q) { const int x = wg * CW + (q - 1) - HW; return x >= 0 && x < W1; };

    for (int i = threadIdx.x; i < 2 * 2 * COLS * D / 2; i += NTH) {
        uint32_t v = 0;
        if (vguess) {
            const int q = (i / (D / 2)) % COLS, d0 = 2 * (i % (D / 2));
            if (in_domain_slot(q)) v = (uint32_t)(d0 % 5 + 3 * (q & 1)) | ((uint32_t)((d0 + 1) % 5 + 3 * (q & 1)) << 16);
        }
        reinterpret_cast<uint32_t*>(&lv[0][0][0][0])[i] = v;
    }
    for (int i = threadIdx.x; i < 2 * 2 * COLS; i += NTH) {
        const int q = i % COLS;
        (&lmin[0][0][0])[i] = vguess && in_domain_slot(q) ? (uint32_t)(3 * (q & 1)) * 0x10001u : 0u;
    }
    for (int i = threadIdx.x; i < NCW; i += NTH) rowcnt[i] = conscnt[i] = 0;
    if (threadIdx.x == 0) pollcnt = 0;

    if constexpr (LINES)
        for (int i = threadIdx.x; i < LG::NLW; i += NTH) linecnt[i] = 0;
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool has_left = wg > 0, has_right = wg + 1 < a.nwg;
    const uint32_t tag0 = a.epoch << 16;
    unsigned long long* hopp = a.hop + (size_t)pair * a.hop_pair;
    auto gbase = [&](int strip, int dir, int b) -> size_t {
        return ((size_t)((band * a.nwg + strip) * 2 + dir) * nblk_rec + b) * SNG;
    };

    if (!HPOLL && wave == NCW) {
        // ---- poller: halo snapshots of the neighbouring strips, once per block.  Granule
        // k*64 + lane of the two records (A from the left strip, then B from the right)
        constexpr int NDAT = G::NDAT;
        constexpr int GPL = (2 * SNG + 63) / 64;  // granules per poller lane
        int gdir[GPL], grec[GPL];
        bool gneed[GPL];
#pragma unroll
        for (int k = 0; k < GPL; k++) {
            const int r2 = k * 64 + lane;
            gdir[k] = r2 >= SNG ? 1 : 0;
            grec[k] = r2 - gdir[k] * SNG;
            gneed[k] = r2 < 2 * SNG && (gdir[k] == 0 ? has_left : has_right);
        }
        bool dead = (a.dbg & 1) != 0;
        [[maybe_unused]] uint64_t st_poll = 0, st_bar = 0;
        SW_T0(st_life);
        const bool xchg = (has_left || has_right) && !(a.dbg & 2);  // wave-uniform
        for (int b = 0; b < nblk; b++) {
            // the neighbours' snapshot of block b (published before their block-end barrier),
            // fetched before ours (SWEEP_EARLY_XCHG == 2) or after it
            uint32_t v[GPL];
            auto poll = [&]() {
                if (b + 1 < nblk && xchg) {
                    const gu64* src[GPL];
#pragma unroll
                    for (int k = 0; k < GPL; k++)
                        src[k] = (const gu64*)(hopp + gbase(gneed[k] ? wg + (gdir[k] ? 1 : -1) : wg, gdir[k], b) + grec[k]);
                    SW_T0(tp);
                    poll_set<GPL>(src, gneed, tag0 | (uint32_t)(b + 1), v, dead, a.err);
                    SW_ACC(st_poll, tp);
#if SWEEP_STATS
                    if (a.stats && (lane == 0 || lane == 32)) {  // observed time of (source strip, dir, block)
                        const int dir = lane == 0 ? 0 : 1;
                        if (dir == 0 ? has_left : has_right)
                            a.stats[1024 + 3 * 65536 + (size_t)MODE * 65536 +
                                    ((size_t)(pair * a.nwg + wg + (dir ? 1 : -1)) * 2 + dir) * nblk + b] =
                                __builtin_amdgcn_s_memrealtime();
                    }
#endif
                }
            };
            if (NOBAR) {
                // the neighbours' snapshot, then the halo waves' last row of the block in LDS (the
                // halo slots the poller overwrites; their readers wait for pollcnt)
                poll();
                SW_T0(tb);
                const uint32_t need = (uint32_t)((b + 1) * HB);
                for (uint32_t spins = 0; !(a.dbg & 4); spins++) {
                    const uint32_t n0 = __builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(&rowcnt[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                    const uint32_t n1 = __builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(&rowcnt[NCW - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                    if (min(n0, n1) >= need) {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                        break;
                    }
                    if (spins >= SW_SPIN_LIMIT) {
                        if (lane == 0) atomicOr(a.err, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                SW_ACC(st_bar, tb);
            } else if (ROWSYNC) {
                if (SWEEP_EARLY_XCHG == 2) poll();
                SW_T0(tb);
                if (!(a.dbg & 4)) lds_barrier();  // the compute waves' end-of-block barrier
                SW_ACC(st_bar, tb);
            } else {
#pragma unroll 1
                for (int j = 0; j < HB; j++) {
                    if (SWEEP_EARLY_XCHG == 2 && j == HB - 1) poll();  // after the rows the snapshot needs
                    if (!(a.dbg & 4)) lds_barrier();  // 4: timing only, no row barriers
                }
            }
            if (SWEEP_EARLY_XCHG != 2 && !NOBAR) poll();
            if (b + 1 < nblk) {
                if (xchg) {
                    const int wb = (b * HB + HB - 1) & 1;
#pragma unroll
                    for (int k = 0; k < GPL; k++) {
                        if (!gneed[k]) continue;
                        const int r = grec[k], dir = gdir[k];
                        if (r < NDAT) {
                            const int q = r / (HW * VL), pcol = (r / VL) % HW, gg = r % VL;
                            const int col = (dir == 0 ? pcol : NCOL - HW + pcol) + 1;  // LDS column slot
                            const int d = gg * DPL + 2 * q;
                            if (2 * q + 1 < DPL) *reinterpret_cast<uint32_t*>(&lv[wb][dir][col][d]) = v[k];
                            else lv[wb][dir][col][d] = (uint16_t)v[k];
                        } else {
                            const int pcol = r - NDAT;
                            lmin[wb][dir][(dir == 0 ? pcol : NCOL - HW + pcol) + 1] = v[k];
                        }
                    }
                }
                if (NOBAR) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                    __hip_atomic_store(&pollcnt, (uint32_t)(b + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                } else {
                    SW_T0(tb2);
                    lds_barrier();
                    SW_ACC(st_bar, tb2);
                }
            }
        }
#if SWEEP_STATS
        if (a.stats && lane == 0) {
            atomicAdd(a.stats + 8 * MODE + 0, (unsigned long long)st_poll);
            atomicAdd(a.stats + 8 * MODE + 1, (unsigned long long)st_bar);
            atomicAdd(a.stats + 8 * MODE + 6, (unsigned long long)(__builtin_readcyclecounter() - st_life));
            const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;  // HW_REG_XCC_ID
            const uint32_t lin = blockIdx.x + blockIdx.y * gridDim.x;
            atomicAdd(a.stats + 8 * MODE + 7, (unsigned long long)(xcc == lin % 8 ? 1 : 0) | (1ull << 32));
            if (MODE == 0 && lin < 2048) reinterpret_cast<uint8_t*>(a.stats + 128)[lin] = (uint8_t)(xcc | 0x80);
        }
#endif
        return;
    }

    if constexpr (LINES) {
        if (wave >= NCW + LG::POLLER) {
            // ---- line waves (MODE 3): line kl of the wave (VL lanes, DPL disparities per lane)
            // runs direction kl & 1 (0 = E, x ascending; 1 = W) of row y0 + (kl >> 1), over the
            // strip's own columns plus `ewarm` columns before them in its direction, from the
            // zero state.  Own column o gets E + W in ring[y % LR][o]; the state entering the
            // strip and the state at its far end go to the boundary-state buffer (k_ew_patch
            // checks them against the neighbours' and repairs the partial where they differ).
            constexpr int NLW = LG::NLW, RPW = LG::RPW, LR = LG::LR, LEAD = LG::LEAD;
            constexpr int NP = DPL / 2;
            constexpr int CB = DPL * (int)sizeof(CT);
            constexpr bool H16 = sizeof(CT) == 1 && SWEEP_H16;
            constexpr bool DSL = LG::DSO;  // deferred subtraction (census): renormalised at every chunk end
            constexpr uint32_t EDGE2 = H16 ? 0x7BFF7BFFu : (kBig | (kBig << 16));
            constexpr int LPF = LG::template lpf<CT>();  // cost loads in flight per lane (a divisor of CW / 2)
            static_assert(!DSL || LPF <= SWEEP_DS_RN, "DS lines renormalise once per chunk");
            const int li = wave - NCW - LG::POLLER;
            const int kl = lane / VL, g = lane % VL;
            const int dir = kl & 1, r = kl >> 1;
            const int H = a.H, W1 = a.W1, x0 = wg * CW;
            const uint32_t P1p = (uint32_t)a.P1 * 0x10001u, P2p = (uint32_t)a.P2 * 0x10001u;
            const uint32_t eL = g == 0 ? EDGE2 : 0u, eR = g == VL - 1 ? EDGE2 : 0u;
            const uint64_t cells = (uint64_t)H * W1 * D;
            const rsrc_t rc = make_rsrc(a.cost + (size_t)pair * a.cost_pair, cells * sizeof(CT));
            const rsrc_t rs = make_rsrc(a.st + (size_t)pair * a.st_pair, a.st_pair);
            __builtin_amdgcn_s_setprio(SWEEP_LINE_PRIO);
            int bn = 0;  // barrier pairs passed (the compute waves' two per block of HB rows)
            [[maybe_unused]] uint64_t lst_cons = 0, lst_bar = 0;
            SW_T0(lst_life);
            auto barriers_to = [&](int y0) {
                if constexpr (NOBAR) return;
                while (bn < nblk && (bn + 1) * HB + LEAD <= y0) {
                    SW_T0(tb);
                    if (!(a.dbg & 4)) lds_barrier();
                    if (bn + 1 < nblk) lds_barrier();
                    SW_ACC(lst_bar, tb);
                    bn++;
                }
            };
            // every own wave has consumed the rows below `need` from the ring
            auto wait_cons_spin = [&](int need) {
                for (uint32_t spins = 0;; spins++) {
                    uint32_t m = 0xFFFFFFFFu;
#pragma unroll
                    for (int w2 = 1; w2 <= NCW - 2; w2++)
                        m = min(m, __hip_atomic_load(&conscnt[w2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                    m = __builtin_amdgcn_readfirstlane(m);
                    if (m >= (uint32_t)need) {
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                        return;
                    }
                    if (spins >= SW_SPIN_LIMIT) {  // never expected: report; the guarded fallback recomputes
                        if (lane == 0) atomicOr(a.err, 1u);
                        return;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            };
            auto wait_cons = [&](int need) {
                if (need <= 0) return;
                SW_T0(tc);
                wait_cons_spin(need);
                SW_ACC(lst_cons, tc);
            };
            // Steps run in chunks of LPF (the cost-load ring): the warmup (rounded up to whole
            // chunks, w >= a.ewarm: a longer warmup only makes the guess better), then the CW / 2
            // own columns this line reaches first (plain ring writes), then the CW / 2 columns
            // the other direction's line wrote first (ring += this line's values).  No memory
            // operation of a step is conditional (a conditional store makes the compiler drain
            // the load ring, vmcnt(0), at every step); the boundary states are stored between
            // chunks.
            const int wch = (max(a.ewarm, 1) + LPF - 1) / LPF;  // warmup chunks
            const int w = wch * LPF, nsteps = w + CW;
            const int c0 = dir ? x0 + CW - 1 + w : x0 - w, cs = dir ? -1 : 1;  // column of step j: c0 + cs * j
            // loads are valid for steps j with (unsigned)(j - jlo) < jspan (columns in [0, W1))
            const int jlo = dir ? max(c0 - (W1 - 1), 0) : max(-c0, 0);
            const int jhi = min(nsteps, dir ? c0 + 1 : W1 - c0);
            const int cstep = cs * D * (int)sizeof(CT);  // byte step of the cost offset
            const int rstep = cs * D;                     // u16 step of the ring pointer (own column o)
            // batch t: the band's own rows u0 .. u0 + RPW - 1 (row y0b + u), ring row u % LR
            for (int t = 0;; t++) {
                const int u0 = (t * NLW + li) * RPW;
                if (u0 >= y1b - y0b) break;
                barriers_to(u0);
                wait_cons(u0 + RPW - LR);
                const int y = y0b + u0 + r;
                const bool yl = y < y1b;
                const uint32_t jspan = yl && jhi > jlo ? (uint32_t)(jhi - jlo) : 0u;
                // byte offset of step 0's cost slice (wraps for columns left of 0; never used there)
                const uint32_t coff = (((uint32_t)y * (uint32_t)W1 + (uint32_t)c0) * (uint32_t)D + (uint32_t)(g * DPL)) *
                                      (uint32_t)sizeof(CT);
                // ring row of y (a row >= H reuses a slot whose row every own wave has consumed
                // and no later row needs); own column o = h (E) or CW - 1 - h (W) at step w + h
                uint16_t* rp = &ring[(u0 + r) % LR][dir ? CW - 1 : 0][g * DPL];
                // (DS) this line's offset slot of own column o: rop + (j - w) * ostep
                uint32_t* rop = &roff[DSL ? (u0 + r) % LR : 0][DSL && dir ? CW - 1 : 0][DSL ? dir : 0];
                const int ostep = cs * 2;
                // boundary states of (y, strip, dir): [0] entering the strip, [1] at its far end
                const uint32_t so = yl ? ((((uint32_t)y * (uint32_t)a.nwg + (uint32_t)wg) * 2u + (uint32_t)dir) * 2u *
                                              (uint32_t)D + (uint32_t)(g * DPL)) * (uint32_t)sizeof(CT)
                                       : kOOB;
                auto coff_at = [&](int j) -> uint32_t {
                    return (uint32_t)(j - jlo) < jspan ? coff + (uint32_t)(j * cstep) : kOOB;
                };
                RawBytes<CB> cr[LPF];
#pragma unroll
                for (int k = 0; k < LPF; k++) {
                    cr[k].load(rc, coff_at(k));
                    asm volatile("" ::: "memory");  // issue order = slot order
                }
                uint32_t Lp[NP], mm = 0, old[NP];
#pragma unroll
                for (int i = 0; i < NP; i++) Lp[i] = old[i] = 0;
                // test mode: a deliberately wrong start state.  Only where the segment starts inside
                // the domain: one that enters it from outside starts from the entry state (the zero
                // state over zero costs), which makes the first strip of each path exact
                if (a.ewguess && jlo == 0) {
#pragma unroll
                    for (int i = 0; i < NP; i++) {
                        const uint32_t d0 = (uint32_t)(g * DPL + 2 * i);
                        Lp[i] = ((d0 * 7u + (uint32_t)y) % 61u) | ((((d0 + 1u) * 7u + (uint32_t)y) % 61u) << 16);
                    }
                    uint32_t m = Lp[0];
#pragma unroll
                    for (int i = 1; i < NP; i++) m = pk_min(m, Lp[i]);
                    m = min(m & 0xFFFFu, m >> 16);
                    mm = group_min<VL>(m) * 0x10001u;
                }
                // one chunk of LPF steps; RING: 0 none (warmup), 1 plain writes, 2 ring += values
                auto chunk = [&](int j0, auto ring_c) {
                    constexpr int RING = decltype(ring_c)::value;
#pragma unroll
                    for (int k = 0; k < LPF; k++) {
                        const int j = j0 + k;
                        // the slot is read after the previous step and unpacked before its
                        // refill is issued (sm_ew.hpp k_ew)
#pragma unroll
                        for (int q = 0; q < RawBytes<CB>::WORDS; q++) asm volatile("" : "+v"(cr[k].w[q]) : "v"(mm));
                        uint32_t C[1][NP];
                        unpack_ct_pk<CT, DPL>(cr[k], C[0]);
#pragma unroll
                        for (int i = 0; i < NP; i++) asm volatile("" : "+v"(C[0][i])::"memory");
                        cr[k].load(rc, coff_at(j + LPF));
                        uint32_t Lq[1][NP], mq[1] = {mm}, Ln[1][NP], mn[1];
#pragma unroll
                        for (int i = 0; i < NP; i++) Lq[0][i] = Lp[i];
                        sweep_step2n<VL, NP, H16, 1, DSL>(Lq, mq, C, P1p, P2p, eL, eR, Ln, mn);
#pragma unroll
                        for (int i = 0; i < NP; i++) Lp[i] = Ln[0][i];
                        if constexpr (DSL && RING != 0) {  // the column's value is Lp - (input minimum)
#if SWEEP_DS_LANE0
                            if (g == 0) rop[(j - w) * ostep] = mq[0];
#else
                            rop[(j - w) * ostep] = mq[0];  // every lane of the line: the same word, no exec mask
#endif
                        }
                        mm = mn[0];
                        if constexpr (RING != 0) {
                            uint16_t* p = rp + (j - w) * rstep;
                            if constexpr (RING == 2) {
                                uint32_t v[NP];
#pragma unroll
                                for (int i = 0; i < NP; i++) v[i] = pk_add(old[i], Lp[i]);
                                lds_put_pk<NP>(p, v);
                                // the next column (the other line wrote it; past the strip's last
                                // column: the ring's padding, never used)
                                lds_get_pk<NP>(p + rstep, old);
                            } else {
                                lds_put_pk<NP>(p, Lp);
                            }
                        }
                        if constexpr (DSL) {
                            if (k == LPF - 1) {  // chunk end (after the ring write): renormalise
#pragma unroll
                                for (int i = 0; i < NP; i++) Lp[i] = pk_sub(Lp[i], mm);
                                mm = 0;
                            }
                        }
                    }
                };
                const int half = CW / 2 / LPF;  // chunks per half strip
                // boundary states in the min-0 form (state - its minimum: every later output is
                // invariant to a constant shift of the state, so k_ew_patch compares and
                // recomputes on this form; DS lines are renormalised at every chunk end already)
                auto min0 = [&](uint32_t (&v)[NP]) {
#pragma unroll
                    for (int i = 0; i < NP; i++) v[i] = DSL ? Lp[i] : pk_sub(Lp[i], mm);
                };
                uint32_t sv[NP];
                for (int c = 0; c < wch; c++) chunk(c * LPF, std::integral_constant<int, 0>{});
                min0(sv);
                store_pk<CT, NP>(rs, so, sv);  // the state entering the strip
                for (int c = 0; c < half; c++) chunk(w + c * LPF, std::integral_constant<int, 1>{});
                // the first far-half column: the other line wrote it in the last step of the loop above
                lds_get_pk<NP>(rp + (CW / 2) * rstep, old);
                for (int c = 0; c < half; c++) chunk(w + (half + c) * LPF, std::integral_constant<int, 2>{});
                min0(sv);
                store_pk<CT, NP>(rs, yl ? so + (uint32_t)(D * sizeof(CT)) : kOOB, sv);  // the far end
                // the batch's ring rows are complete (LDS only: the state stores need no ordering)
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                __hip_atomic_store(&linecnt[li], (uint32_t)(t + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            barriers_to(0x7FFFFFFF);
#if SWEEP_STATS
            if (a.stats && lane == 0) {
                atomicAdd(a.stats + 41, (unsigned long long)lst_cons);
                atomicAdd(a.stats + 42, (unsigned long long)lst_bar);
                atomicAdd(a.stats + 43, (unsigned long long)(__builtin_readcyclecounter() - lst_life));
                atomicAdd(a.stats + 44, 1ull);
            }
#endif
            return;
        }
    }

    // ---- compute waves
    const int kl = lane / VL, g = lane % VL;
    // column slot among the compute waves (halo waves: of their first column set)
    const int c = wave == 0 ? kl : wave == NCW - 1 ? NCOL - HW + kl : HW + (wave - 1) * LPW + kl;
    const int x1 = wg * CW + c - HW;
    const bool active = x1 >= 0 && x1 < W1;
    const bool halo_l = wave == 0, halo_r = wave == NCW - 1, own = !halo_l && !halo_r;  // wave-uniform
    const int wx0 = wg * CW + wave * LPW - LPW;
    const bool wave_ragged = wx0 < 0 || wx0 + LPW > W1;  // wave-uniform: some column outside [0, W1)
    const uint32_t P1 = (uint32_t)a.P1, P2 = (uint32_t)a.P2;
    // row hand-off inside a block: a wave's step s reads its neighbours' row s-1 state
    // from one LDS buffer and writes its own row s into the other, which the neighbours
    // read at their step s-1; so step s may start once both neighbours have published
    // row s-1 (that also orders their reads of the buffer this step overwrites).  The
    // block's last row ends with a workgroup barrier (the poller's halo snapshot).
    const int wl = wave > 0 ? wave - 1 : wave, wr = wave < NCW - 1 ? wave + 1 : wave;
    bool sync_dead = (a.dbg & 4) != 0;
    auto publish_row = [&](int s) {
        __hip_atomic_store(&rowcnt[wave], (uint32_t)(s + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    [[maybe_unused]] uint64_t st_wait = 0, st_bbar = 0;
    SW_T0(st_clife);
    auto wait_row_spin = [&](int s) {
        for (uint32_t spins = 0;; spins++) {
            // both counters in flight at once (relaxed), one acquire for the pair
            const uint32_t nl = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&rowcnt[wl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            const uint32_t nr = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&rowcnt[wr], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (min(nl, nr) >= (uint32_t)s) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                return;
            }
            if (spins >= SW_SPIN_LIMIT) {  // never expected: report, let the guarded fallback recompute
                if (lane == 0) atomicOr(a.err, 1u);
                sync_dead = true;
                return;
            }
            if (SWEEP_ROW_SLEEP) __builtin_amdgcn_s_sleep(SWEEP_ROW_SLEEP);
        }
    };
    auto wait_row = [&](int s) {
        if (sync_dead) return;
        SW_T0(tw);
        wait_row_spin(s);
        SW_ACC(st_wait, tw);
    };
    // MODE 3: row s of the ring is complete (its line wave has finished the batch holding it)
    [[maybe_unused]] uint64_t st_wl = 0;
    auto wait_lines_spin = [&](int s) {
        if constexpr (LINES) {
            const int li = (s / LG::RPW) % LG::NLW;
            const uint32_t need = (uint32_t)(s / (LG::RPW * LG::NLW) + 1);
            for (uint32_t spins = 0;; spins++) {
                const uint32_t nd = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(&linecnt[li], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                if (nd >= need) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                    return;
                }
                if (spins >= SW_SPIN_LIMIT) {  // never expected: report, the guarded fallback recomputes
                    if (lane == 0) atomicOr(a.err, 1u);
                    return;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        } else {
            (void)s;
        }
    };
    auto wait_lines = [&](int s) {
        SW_T0(twl);
        wait_lines_spin(s);
        SW_ACC(st_wl, twl);
    };
    // NOBAR: the poller has written block b's halo snapshot into LDS
    auto wait_poll = [&](int b) {
        if constexpr (NOBAR) {
            for (uint32_t spins = 0; !sync_dead; spins++) {
                const uint32_t n = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(&pollcnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                if (n >= (uint32_t)b) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
                    return;
                }
                if (spins >= SW_SPIN_LIMIT) {
                    if (lane == 0) atomicOr(a.err, 1u);
                    sync_dead = true;
                    return;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        } else {
            (void)b;
        }
    };
    auto end_row = [&](int j, int s) {
        if (!ROWSYNC || j == HB - 1) {
            if (!(a.dbg & 4)) lds_barrier();
        } else {
            publish_row(s);
        }
    };

    const uint64_t cells = (uint64_t)H * W1 * D;
    const rsrc_t rc = make_rsrc(a.cost + (size_t)pair * a.cost_pair, cells * sizeof(CT));
    rsrc_t re = make_rsrc(nullptr, 0), rw = re, rp = re, rrec = re, rnb = re;
    if constexpr (EWIN) {
        re = make_rsrc(a.ew + (size_t)pair * a.ew_pair, cells * sizeof(CT));
        rw = make_rsrc(a.ew + (size_t)pair * a.ew_pair + a.ew_slot, cells * sizeof(CT));
    }
    if constexpr (WTA) {
        rrec = make_rsrc(a.rec + (size_t)pair * H * a.W, (uint64_t)H * a.W * 4);
        rnb = make_rsrc(a.nb + (size_t)pair * H * a.W, (uint64_t)H * a.W * 4);
    }
    const int ku = 100 - a.uniq;  // uniqueness: S*(100-u) < 100*minS
    if constexpr (MODE != 1) rp = make_rsrc((const uint8_t*)a.part + (size_t)pair * a.part_pair, cells * 2);
    const rsrc_t rhop = make_rsrc(hopp, (uint64_t)a.hop_pair * 8);
    constexpr uint32_t NONE = 0xFFFFFFFFu;
    // element offset of this lane's slice in row y (cost: every compute wave;
    // E/W/partial inputs and outputs: own columns only)
    auto cell = [&](int y) -> uint32_t {
        return active ? ((uint32_t)y * (uint32_t)W1 + (uint32_t)x1) * (uint32_t)D + (uint32_t)(g * DPL) : NONE;
    };
    auto boff = [&](uint32_t e, int bytes) -> uint32_t { return e == NONE ? kOOB : e * (uint32_t)bytes; };

    uint32_t LV[DPL];
#pragma unroll
    for (int i = 0; i < DPL; i++) LV[i] = 0;
    uint32_t mV = 0;

    // per-step inputs through a ring of PF rows in flight; every memory
    // operation of the step loop is issued by every compute wave (masked ones
    // at out-of-range offsets), so the compiler's counted vmcnt waits hold for
    // all of them and no wave waits for a load it issued this step
    RawBytes<CB> rc_[PF], re_[PF], rw_[PF];
    RawBytes<DPL * 2> rp_[PF];
    auto issue = [&](int k, int s) {  // loads of step s into ring slot k (rows past the end read 0)
        const uint32_t en = s < H ? cell(UP ? H - 1 - s : s) : NONE;
        const uint32_t eo = own ? en : NONE;
        rc_[k].template load<WTA ? SWEEP_COST_AUX : 0>(rc, boff(en, sizeof(CT)));
        if constexpr (EWIN) {
            re_[k].template load<SWEEP_STREAM_AUX>(re, boff(eo, sizeof(CT)));
            rw_[k].template load<SWEEP_STREAM_AUX>(rw, boff(eo, sizeof(CT)));
        }
        if constexpr (PARTR) rp_[k].template load<SWEEP_STREAM_AUX>(rp, boff(eo, 2));
    };
    if constexpr (DPL % 2 == 0 && !SWEEP_U32) {
        // ---- packed u16-pair form (same steps as the u32 loop below), one straight-line
        // row loop per wave role so the three directions of an own wave interleave:
        //   wait for the neighbours' row s-1 -> LDS reads of the diagonal predecessors ->
        //   V (no LDS input) while they land -> A, B -> LDS writes -> publish row s ->
        //   the partial sum (down sweep) or S + WTA + uniqueness (WTA sweeps), which no
        //   other wave waits for.
        // Columns outside [0, W1) need no masking: their costs load as 0 (out-of-range
        // buffer offsets), so a direction entering from outside the domain stays at the
        // entering state (L = 0 + min(0, P1, P2) - 0 = 0), and the garbage a direction
        // leaving the domain produces only flows further outward (A: rightward, B:
        // leftward), never into a domain column or a published halo snapshot.
        constexpr int NP = DPL / 2;
        const uint32_t P1p = P1 * 0x10001u, P2p = P2 * 0x10001u;
        // line-edge constants of sweep_step2 (16-lane lines): EDGE on the first / last lane
        constexpr uint32_t EDGE2 = (sizeof(CT) == 1 && SWEEP_H16) ? 0x7BFF7BFFu : (kBig | (kBig << 16));
        const uint32_t eL = g == 0 ? EDGE2 : 0u, eR = g == VL - 1 ? EDGE2 : 0u;
        // census sums stay below 2^11 (8 paths x (62 + P2 <= 193)): plain packed adds; u16
        // costs saturate in OpenCV's order (normalize's domain keeps L <= 16383)
        constexpr bool SAT = sizeof(CT) == 2;
        constexpr bool H16 = !SAT && SWEEP_H16;  // census: f16 form of the recurrence and the sums
        constexpr bool DS = H16 && SWEEP_DS;     // deferred subtraction (SWEEP_DS)
        static_assert(!DS || SWEEP_STEPN, "deferred subtraction runs the stage-wise steps");
        auto run = [&](auto role_c) {
            constexpr int ROLE = decltype(role_c)::value;  // 0 left halo (A), 1 own (A, B, V), 2 right halo (B)
            constexpr bool HAS_A = ROLE != 2, HAS_B = ROLE != 0, OWN = ROLE == 1;
            constexpr int NS = OWN ? 1 : HM;  // column sets of this wave (halo waves: HM)
            // this lane's column of set h: slot c + h*LPW, x1 + h*LPW
            auto cell_h = [&](int h, int y) -> uint32_t {
                const int xh = x1 + h * LPW;
                return xh >= 0 && xh < W1 ? ((uint32_t)y * (uint32_t)W1 + (uint32_t)xh) * (uint32_t)D + (uint32_t)(g * DPL)
                                          : NONE;
            };
            RawBytes<CB> rcs[PF][NS];
            auto issue_r = [&](int k, int s) {
                const int yy = UP ? H - 1 - s : ys + s;
#pragma unroll
                for (int h = 0; h < NS; h++)
                    rcs[k][h].template load<WTA ? SWEEP_COST_AUX : 0>(rc, boff(s < nrow ? cell_h(h, yy) : NONE, sizeof(CT)));
                if constexpr (OWN && EWIN) {
                    const uint32_t en = s < nrow ? cell(yy) : NONE;
                    re_[k].template load<SWEEP_STREAM_AUX>(re, boff(en, sizeof(CT)));
                    rw_[k].template load<SWEEP_STREAM_AUX>(rw, boff(en, sizeof(CT)));
                }
                if constexpr (OWN && PARTR) rp_[k].template load<SWEEP_STREAM_AUX>(rp, boff(s < nrow ? cell(yy) : NONE, 2));
            };
#pragma unroll
            for (int k = 0; k < PF; k++) issue_r(k, k);
            uint32_t LVp[NP];
#pragma unroll
            for (int i = 0; i < NP; i++) LVp[i] = 0;
            uint32_t mVl = 0;
            if (vguess && OWN && active) {  // (tests) the wrong entering state of the LDS rows, slot c + 1
                const uint32_t o = (uint32_t)(3 * ((c + 1) & 1));
#pragma unroll
                for (int i = 0; i < NP; i++) {
                    const int d0 = g * DPL + 2 * i;
                    LVp[i] = ((uint32_t)(d0 % 5) + o) | (((uint32_t)((d0 + 1) % 5) + o) << 16);
                }
                mVl = o * 0x10001u;
            }
            // MODE 3 with row bands: the own columns' S / SE / SW states (min-0 form) at the row
            // above the band (which 0, speculative) and at the band's last row (which 1)
            auto vstore = [&](int which, const uint32_t (&sV)[NP], uint32_t mV_, const uint32_t (&sA)[NP], uint32_t mA_,
                              const uint32_t (&sB)[NP], uint32_t mB_) {
                if constexpr (LINES && OWN) {
                    const rsrc_t rv = make_rsrc(a.vst + (size_t)pair * a.vst_pair, a.vst_pair);
                    auto off = [&](int dir) -> uint32_t {
                        return active ? (((((uint32_t)band * 2u + (uint32_t)which) * 3u + (uint32_t)dir) * (uint32_t)W1 +
                                          (uint32_t)x1) * (uint32_t)D + (uint32_t)(g * DPL)) * (uint32_t)sizeof(CT)
                                      : kOOB;
                    };
                    uint32_t v[NP];
#pragma unroll
                    for (int i = 0; i < NP; i++) v[i] = pk_sub(sV[i], mV_);
                    store_pk<CT, NP>(rv, off(0), v);
#pragma unroll
                    for (int i = 0; i < NP; i++) v[i] = pk_sub(sA[i], mA_);
                    store_pk<CT, NP>(rv, off(1), v);
#pragma unroll
                    for (int i = 0; i < NP; i++) v[i] = pk_sub(sB[i], mB_);
                    store_pk<CT, NP>(rv, off(2), v);
                }
            };
            // d + 1 of each packed half of this lane (uniqueness window test)
            uint32_t dpk[NP];
#pragma unroll
            for (int i = 0; i < NP; i++) dpk[i] = (uint32_t)(g * DPL + 2 * i + 1) * 0x10001u + 0x10000u;
            if constexpr (SWEEP_DYNPRIO && !OWN) __builtin_amdgcn_s_setprio(PRIO_HI);
            for (int b = 0; b < nblk; b++) {
#pragma unroll
                for (int j = 0; j < HB; j++) {
                    const int k = j % PF;
                    const int s = b * HB + j;
                    if constexpr (SWEEP_DYNPRIO && OWN) __builtin_amdgcn_s_setprio(PRIO_HI);
                    const bool live = s < nrow;
                    const int y = UP ? H - 1 - s : ys + s;
                    const int rb = (s + 1) & 1, wb = s & 1;
                    const uint32_t e = live ? cell(y) : NONE;
                    uint32_t C[NS][NP], Ein[NP], Win[NP], Pin[NP];
#pragma unroll
                    for (int h = 0; h < NS; h++) unpack_ct_pk<CT, DPL>(rcs[k][h], C[h]);
                    if constexpr (OWN && EWIN) {
                        unpack_ct_pk<CT, DPL>(re_[k], Ein);
                        unpack_ct_pk<CT, DPL>(rw_[k], Win);
                    }
                    if constexpr (OWN && PARTR) unpack_ct_pk<uint16_t, DPL>(rp_[k], Pin);
#pragma unroll
                    for (int i = 0; i < NP; i++) {  // before the refill (see the u32 loop)
#pragma unroll
                        for (int h = 0; h < NS; h++) asm volatile("" : "+v"(C[h][i])::"memory");
                        if constexpr (OWN && EWIN) asm volatile("" : "+v"(Ein[i]), "+v"(Win[i])::"memory");
                        if constexpr (OWN && PARTR) asm volatile("" : "+v"(Pin[i])::"memory");
                    }
                    issue_r(k, s + PF);
                    if (ROWSYNC && (j > 0 || NOBAR)) wait_row(s);
                    // diagonal predecessors: column c-1 (A) and c+1 (B) of the previous row
                    uint32_t LA[NS][NP], LB[NS][NP], mA[NS], mB[NS];
#pragma unroll
                    for (int h = 0; h < NS; h++) {
                        const int ch = c + h * LPW;
                        if constexpr (HAS_A) {
                            lds_get_pk<NP>(&lv[rb][0][ch][g * DPL], LA[h]);
                            mA[h] = lmin[rb][0][ch];
                        }
                        if constexpr (HAS_B) {
                            lds_get_pk<NP>(&lv[rb][1][ch + 2][g * DPL], LB[h]);
                            mB[h] = lmin[rb][1][ch + 2];
                        }
                    }
                    // 5-path sweep (row barriers): the LDS reads leave before the V step (which
                    // does not need them), so their latency overlaps V instead of adding to the
                    // row chain (the scheduler otherwise issued V first).  Measured on one box:
                    // sgbm5 4991 -> 5041-5068 pairs/s; the counter-synchronised sweeps (modes 0
                    // and 2) were slower with it (census8 6193 -> 6081-6088), so they keep the
                    // compiler's order
                    if constexpr (SWEEP_LDS_FIRST && MODE == 1) __builtin_amdgcn_sched_barrier(0);
                    uint32_t nV[NP], nA[NS][NP], nB[NS][NP], mnV = 0, mnA[NS], mnB[NS];
                    auto step = [&](const uint32_t(&Lp)[NP], uint32_t m, const uint32_t(&Ch)[NP], uint32_t(&Ln)[NP]) {
                        return sweep_step2<VL, NP, H16, DS>(Lp, m, Ch, P1p, P2p, eL, eR, Ln);
                    };
                    if constexpr (OWN) {
                        if constexpr (SWEEP_STEPN) {  // stage-wise over the words (sweep_step2n)
                            uint32_t Lp1[1][NP], m1[1] = {mVl}, C1[1][NP], Ln1[1][NP], mn1[1];
#pragma unroll
                            for (int i = 0; i < NP; i++) {
                                Lp1[0][i] = LVp[i];
                                C1[0][i] = C[0][i];
                            }
                            sweep_step2n<VL, NP, H16, 1, DS>(Lp1, m1, C1, P1p, P2p, eL, eR, Ln1, mn1);
#pragma unroll
                            for (int i = 0; i < NP; i++) nV[i] = Ln1[0][i];
                            mnV = mn1[0];
                        } else {
                            mnV = step(LVp, mVl, C[0], nV);
                        }
                    }
                    if constexpr (SWEEP_STEPN && OWN && NS == 1) {
                        // A and B of the column, interleaved (sm_pk.hpp sweep_step2n)
                        uint32_t Lp2[2][NP], m2[2], C2[2][NP], Ln2[2][NP], mn2[2];
#pragma unroll
                        for (int i = 0; i < NP; i++) {
                            Lp2[0][i] = LA[0][i];
                            Lp2[1][i] = LB[0][i];
                            C2[0][i] = C2[1][i] = C[0][i];
                        }
                        m2[0] = mA[0];
                        m2[1] = mB[0];
                        sweep_step2n<VL, NP, H16, 2, DS>(Lp2, m2, C2, P1p, P2p, eL, eR, Ln2, mn2);
#pragma unroll
                        for (int i = 0; i < NP; i++) {
                            nA[0][i] = Ln2[0][i];
                            nB[0][i] = Ln2[1][i];
                        }
                        mnA[0] = mn2[0];
                        mnB[0] = mn2[1];
                    } else if constexpr (SWEEP_STEPN && !OWN && NS > 1) {
                        // a halo wave's column sets of its one direction, interleaved
                        uint32_t Lpn[NS][NP], mn_in[NS], Lnn[NS][NP], mnn[NS];
#pragma unroll
                        for (int h = 0; h < NS; h++) {
                            if constexpr (HAS_A) {
#pragma unroll
                                for (int i = 0; i < NP; i++) Lpn[h][i] = LA[h][i];
                                mn_in[h] = mA[h];
                            } else {
#pragma unroll
                                for (int i = 0; i < NP; i++) Lpn[h][i] = LB[h][i];
                                mn_in[h] = mB[h];
                            }
                        }
                        sweep_step2n<VL, NP, H16, NS, DS>(Lpn, mn_in, C, P1p, P2p, eL, eR, Lnn, mnn);
#pragma unroll
                        for (int h = 0; h < NS; h++) {
#pragma unroll
                            for (int i = 0; i < NP; i++) {
                                if constexpr (HAS_A) nA[h][i] = Lnn[h][i];
                                else nB[h][i] = Lnn[h][i];
                            }
                            if constexpr (HAS_A) mnA[h] = mnn[h];
                            else mnB[h] = mnn[h];
                        }
                    } else {
#pragma unroll
                        for (int h = 0; h < NS; h++) {
                            if constexpr (HAS_A) mnA[h] = step(LA[h], mA[h], C[h], nA[h]);
                            if constexpr (HAS_B) mnB[h] = step(LB[h], mB[h], C[h], nB[h]);
                        }
                    }
                    // DS: the own wave's outputs are n - (input minimum) per path, summed first and
                    // corrected once (offs); the state passed on (LDS row, snapshot, next row) is
                    // renormalised at the block's last row and every SWEEP_DS_RN rows, the outputs'
                    // offsets then shrink by the removed minima (u16 arithmetic mod 2^16: the
                    // corrected sums are exact)
                    [[maybe_unused]] uint32_t offs = 0;
                    if constexpr (DS) {
                        if constexpr (OWN) offs = pk_add(pk_add(mVl, mA[0]), mB[0]);
                        if (j == HB - 1 || j % SWEEP_DS_RN == SWEEP_DS_RN - 1) {
                            if constexpr (OWN) {
                                offs = pk_sub(offs, pk_add(pk_add(mnV, mnA[0]), mnB[0]));
#pragma unroll
                                for (int i = 0; i < NP; i++) nV[i] = pk_sub(nV[i], mnV);
                                mnV = 0;
                            }
#pragma unroll
                            for (int h = 0; h < NS; h++) {
#pragma unroll
                                for (int i = 0; i < NP; i++) {
                                    if constexpr (HAS_A) nA[h][i] = pk_sub(nA[h][i], mnA[h]);
                                    if constexpr (HAS_B) nB[h][i] = pk_sub(nB[h][i], mnB[h]);
                                }
                                if constexpr (HAS_A) mnA[h] = 0;
                                if constexpr (HAS_B) mnB[h] = 0;
                            }
                        }
                    }
                    if constexpr (LINES && OWN) {  // row bands: the vertical paths' boundary states
                        if (nband > 1 && (s == wrows - 1 || (s == nrow - 1 && band + 1 < nband)))
                            vstore(s == wrows - 1 ? 0 : 1, nV, mnV, nA[0], mnA[0], nB[0], mnB[0]);
                    }
                    // snapshot of the block's last row for the neighbouring strips' halos: the
                    // strip's HM boundary own waves on each side (before the block-end barrier
                    // with SWEEP_EARLY_XCHG, so no wave of the strip waits for the others first)
                    auto snapshot = [&]() {
                        if (j == HB - 1 && b + 1 < nblk) {
                            const bool pa = wave >= NCW - 1 - HM && has_right, pb = wave <= HM && has_left;
                            if (pa || pb) {
                                const uint32_t tag = tag0 | (uint32_t)(b + 1);
                                const int pcol = (pa ? wave - (NCW - 1 - HM) : wave - 1) * LPW + kl;
                                const size_t rec = gbase(wg, pa ? 0 : 1, b);
#pragma unroll
                                for (int q = 0; q < NG; q++)  // 64 consecutive granules per store
                                    __builtin_amdgcn_raw_buffer_store_b64(
                                        u32x2{pa ? nA[0][q] : nB[0][q], tag}, rhop,
                                        (uint32_t)((rec + (size_t)(q * HW + pcol) * VL + g) * 8), 0, 16);
                                if (g == 0)  // the column's minimum (replicated halves, as lmin holds it)
                                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{pa ? mnA[0] : mnB[0], tag}, rhop,
                                                                          (uint32_t)((rec + G::NDAT + pcol) * 8), 0, 16);
#if SWEEP_STATS
                                if (a.stats && lane == 0 && (wave == NCW - 2 || wave == 1))  // publish time
                                    a.stats[1024 + (size_t)MODE * 65536 +
                                            ((size_t)(pair * a.nwg + wg) * 2 + (pa ? 0 : 1)) * nblk + b] =
                                        __builtin_amdgcn_s_memrealtime();
#endif
                            }
                        }
                    };
                    if constexpr (OWN && SWEEP_EARLY_XCHG) snapshot();
#pragma unroll
                    for (int h = 0; h < NS; h++) {
                        const int ch = c + h * LPW;
                        if constexpr (HAS_A) {
                            lds_put_pk<NP>(&lv[wb][0][ch + 1][g * DPL], nA[h]);
                            if (g == 0) lmin[wb][0][ch + 1] = mnA[h];
                        }
                        if constexpr (HAS_B) {
                            lds_put_pk<NP>(&lv[wb][1][ch + 1][g * DPL], nB[h]);
                            if (g == 0) lmin[wb][1][ch + 1] = mnB[h];
                        }
                    }
                    if constexpr (HPOLL && !OWN) {
                        // the block's last row: the neighbour strip's state of it replaces this
                        // halo wave's (stale) columns before the row is published
                        if (j == HB - 1 && b + 1 < nblk) {
                            constexpr int dirh = HAS_A ? 0 : 1;  // left halo: A from the left strip
                            if ((dirh == 0 ? has_left : has_right) && !(a.dbg & 2)) {
                                constexpr int GH = (SNG + 63) / 64, NDAT = G::NDAT;
                                const gu64* src[GH];
                                bool need[GH];
                                uint32_t v[GH];
#pragma unroll
                                for (int k = 0; k < GH; k++) {
                                    const int r = k * 64 + lane;
                                    need[k] = r < SNG;
                                    src[k] = (const gu64*)(hopp + gbase(wg + (dirh ? 1 : -1), dirh, b) + (need[k] ? r : 0));
                                }
                                SW_T0(tp);
                                poll_set<GH>(src, need, tag0 | (uint32_t)(b + 1), v, sync_dead, a.err);
                                SW_ACC(st_bbar, tp);
#pragma unroll
                                for (int k = 0; k < GH; k++) {
                                    if (!need[k]) continue;
                                    const int r = k * 64 + lane;
                                    if (r < NDAT) {
                                        const int q = r / (HW * VL), pcol = (r / VL) % HW, gg = r % VL;
                                        const int col = (dirh == 0 ? pcol : NCOL - HW + pcol) + 1;  // LDS column slot
                                        const int d = gg * DPL + 2 * q;
                                        if (2 * q + 1 < DPL) *reinterpret_cast<uint32_t*>(&lv[wb][dirh][col][d]) = v[k];
                                        else lv[wb][dirh][col][d] = (uint16_t)v[k];
                                    } else {
                                        const int pcol = r - NDAT;
                                        lmin[wb][dirh][(dirh == 0 ? pcol : NCOL - HW + pcol) + 1] = v[k];
                                    }
                                }
                            }
                        }
                    }
                    // the row is published (neighbour counters) or, at a block end and
                    // without row sync, closed by a barrier; the poller writes the halo
                    // snapshot after the block-end barrier, while the waves run their WTA
                    if (!ROWSYNC || (j == HB - 1 && !NOBAR)) {
                        SW_T0(tb);
                        if (!(a.dbg & 4)) lds_barrier();
                        SW_ACC(st_bbar, tb);
                    } else {
                        publish_row(s);
                    }
                    if constexpr (SWEEP_DYNPRIO && OWN) __builtin_amdgcn_s_setprio(PRIO_LO);
                    if constexpr (OWN) {
#pragma unroll
                        for (int i = 0; i < NP; i++) LVp[i] = nV[i];
                        mVl = mnV;
                        if constexpr (!SWEEP_EARLY_XCHG) snapshot();
                        // every per-word loop below runs stage by stage over the NP words (the
                        // words are independent: no wait state between dependent VOP3P ops)
                        if constexpr (MODE == 0) {
                            uint32_t out[NP];
#pragma unroll
                            for (int i = 0; i < NP; i++) out[i] = pk_add(nV[i], nA[0][i]);
#pragma unroll
                            for (int i = 0; i < NP; i++) out[i] = pk_add(out[i], nB[0][i]);
                            if constexpr (DS) {
#pragma unroll
                                for (int i = 0; i < NP; i++) out[i] = pk_sub(out[i], offs);
                            }
                            bstore_n<uint32_t, NP, SWEEP_STREAM_AUX>(rp, boff(e, 2), out);
                        } else if constexpr (MODE == 3) {
                          const int u = s - wrows;  // the band's own row index (< 0: a vertical warmup row)
                          if (u >= 0) {
                            // + E + W of this row from the line waves' ring (u16 costs: saturating,
                            // the WTA clamps at 32767 anyway; three paths alone stay below 2^16)
                            uint32_t out[NP], ewl[NP];
#pragma unroll
                            for (int i = 0; i < NP; i++) out[i] = pk_add(nV[i], nA[0][i]);
#pragma unroll
                            for (int i = 0; i < NP; i++) out[i] = pk_add(out[i], nB[0][i]);
                            if (live) wait_lines(u);
                            lds_get_pk<NP>(&ring[u % LG::LR][(wave - 1) * LPW + kl][g * DPL], ewl);
                            if constexpr (DS && LG::DSO) {  // + the E and W lines' offsets of this column
                                const uint2 ro = *reinterpret_cast<const uint2*>(&roff[u % LG::LR][(wave - 1) * LPW + kl][0]);
                                offs = pk_add(offs, pk_add(ro.x, ro.y));
                            }
#pragma unroll
                            for (int i = 0; i < NP; i++) out[i] = SAT ? pk_adds(out[i], ewl[i]) : pk_add(out[i], ewl[i]);
                            if constexpr (DS) {
#pragma unroll
                                for (int i = 0; i < NP; i++) out[i] = pk_sub(out[i], offs);
                            }
                            bstore_n<uint32_t, NP, SWEEP_STREAM_AUX>(rp, boff(e, 2), out);
                            // the ring row is read (the fence waits for the LDS read): the lines may reuse it
                            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                            __hip_atomic_store(&conscnt[wave], (uint32_t)(u + 1), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                          }
                        } else {
                            uint32_t Sp[NP], ew[NP];
                            // a padded cost volume (u16 costs only): its pad planes d >= Dv take
                            // S = 0xFFFF, above every real S <= 32767 (never the minimum, never
                            // below the uniqueness threshold)
                            const bool pad = SAT && a.Dv < D;  // wave-uniform
                            if constexpr (SAT) {
                                if constexpr (EWIN) {
#pragma unroll
                                    for (int i = 0; i < NP; i++) ew[i] = pk_adds(Ein[i], Win[i]);
                                    if constexpr (PARTR) {
#pragma unroll
                                        for (int i = 0; i < NP; i++) ew[i] = pk_adds(ew[i], Pin[i]);
                                    }
                                } else {  // MODE 4: the partial holds E and W already
#pragma unroll
                                    for (int i = 0; i < NP; i++) ew[i] = Pin[i];
                                }
#pragma unroll
                                for (int i = 0; i < NP; i++) Sp[i] = pk_adds(nV[i], nA[0][i]);
#pragma unroll
                                for (int i = 0; i < NP; i++) ew[i] = pk_adds(nB[0][i], ew[i]);
#pragma unroll
                                for (int i = 0; i < NP; i++) Sp[i] = pk_adds(Sp[i], ew[i]);
#pragma unroll
                                for (int i = 0; i < NP; i++) Sp[i] = pk_min(Sp[i], 0x7FFF7FFFu);  // min(sum, 32767)
                                if (pad) {
#pragma unroll
                                    for (int i = 0; i < NP; i++) {
                                        const int d0 = g * DPL + 2 * i;
                                        Sp[i] |= (d0 >= a.Dv ? 0x0000FFFFu : 0u) | (d0 + 1 >= a.Dv ? 0xFFFF0000u : 0u);
                                    }
                                }
                            } else {
                                if constexpr (EWIN) {
#pragma unroll
                                    for (int i = 0; i < NP; i++) ew[i] = pk_add(Ein[i], Win[i]);
                                    if constexpr (PARTR) {
#pragma unroll
                                        for (int i = 0; i < NP; i++) ew[i] = pk_add(ew[i], Pin[i]);
                                    }
                                } else {
#pragma unroll
                                    for (int i = 0; i < NP; i++) ew[i] = Pin[i];
                                }
#pragma unroll
                                for (int i = 0; i < NP; i++) Sp[i] = pk_add(nV[i], nA[0][i]);
#pragma unroll
                                for (int i = 0; i < NP; i++) ew[i] = pk_add(nB[0][i], ew[i]);
#pragma unroll
                                for (int i = 0; i < NP; i++) Sp[i] = pk_add(Sp[i], ew[i]);
                                if constexpr (DS) {
#pragma unroll
                                    for (int i = 0; i < NP; i++) Sp[i] = pk_sub(Sp[i], offs);
                                }
                            }
                            uint32_t key = 0xFFFFFFFFu;
#pragma unroll
                            for (int i = 0; i < NP; i++)
                                key = min(key, min((Sp[i] << 16) | wta_rank(g * DPL + 2 * i, MODE == 1),
                                                   (Sp[i] & 0xFFFF0000u) | wta_rank(g * DPL + 2 * i + 1, MODE == 1)));
                            asm volatile("" ::: "memory");  // u32 / u128 stores, u16 loads of srow: no reordering
                            lds_put_pk<NP>(&srow[(wave - 1) % (NCW - 2)][kl][g * DPL], Sp);
                            asm volatile("" ::: "memory");
                            key = group_min<VL>(key);
                            const uint32_t minS = key >> 16;
                            const int best = wta_unrank(key & 0xFFFF, MODE == 1);  // MODE 1 = 5 paths
                            const int bm = max(best - 1, 0), bq = min(best + 1, D - 1);
                            const uint32_t Sm = srow[(wave - 1) % (NCW - 2)][kl][bm];
                            const uint32_t Sq = srow[(wave - 1) % (NCW - 2)][kl][bq];
                            // uniqueness: the pixel is rejected iff some d with |d - best| > 1 has
                            // S[d]*(100-u) < 100*minS, i.e. iff m2 * ku < 100 * minS for m2 = the
                            // minimum of S outside best-1..best+1.  The window's entries are pushed
                            // to >= 0xFFFD (above every S <= 32767) before the minimum: t = d -
                            // (best-1) in {0, 1, 2} exactly inside it, 3 - t (saturating) > 0 there,
                            // times 0xFFFF = -(3 - t) mod 2^16.
                            const uint32_t bm1p = (uint32_t)best * 0x10001u;  // t = (d + 1) - best = d - (best - 1)
                            uint32_t tw[NP];
#pragma unroll
                            for (int i = 0; i < NP; i++) tw[i] = pk_sub(dpk[i], bm1p);
#pragma unroll
                            for (int i = 0; i < NP; i++) tw[i] = pkw(__builtin_elementwise_sub_sat(pkv(0x00030003u), pkv(tw[i])));
#pragma unroll
                            for (int i = 0; i < NP; i++) tw[i] = pk_window_push(tw[i], Sp[i]);
                            uint32_t m2p = tw[0];
#pragma unroll
                            for (int i = 1; i < NP; i++) m2p = pk_min(m2p, tw[i]);
                            const uint32_t m2 = group_min<VL>(min(m2p & 0xFFFFu, m2p >> 16));
                            // (m2 = 0xFFFF: no real far entry, only pad planes of a volume with Dv <= 3)
                            const bool ok = !(__mul24((int)m2, ku) < __mul24((int)minS, 100) && (!pad || m2 <= 32767u)) &&
                                            minS < 32767u;
                            const uint32_t recw = ok ? ((minS << 16) | (uint32_t)best) : 0xFFFFFFFFu;
                            const uint32_t nbw = Sm | (Sq << 16);
                            const bool wpx = g == 0 && active && live;
                            const uint32_t px = (uint32_t)y * (uint32_t)a.W + (uint32_t)(x1 + a.minX1);
                            __builtin_amdgcn_raw_buffer_store_b32(recw, rrec, wpx ? px * 4 : kOOB, 0, 0);
                            __builtin_amdgcn_raw_buffer_store_b32(nbw, rnb, wpx ? px * 4 : kOOB, 0, 0);
                        }
                    }
                }
                if (b + 1 < nblk && !HPOLL) {
                    SW_T0(tb);
                    if constexpr (NOBAR) wait_poll(b + 1);
                    else lds_barrier();  // the poller has written the halo snapshot
                    SW_ACC(st_bbar, tb);
                }
            }
#if SWEEP_STATS
            if (a.stats && lane == 0) {
                atomicAdd(a.stats + 8 * MODE + 2, (unsigned long long)st_wait);
                atomicAdd(a.stats + 8 * MODE + 3, (unsigned long long)st_bbar);
                atomicAdd(a.stats + 8 * MODE + 4, (unsigned long long)(__builtin_readcyclecounter() - st_clife));
                atomicAdd(a.stats + 8 * MODE + 5, 1ull);
                if (LINES) atomicAdd(a.stats + 40, (unsigned long long)st_wl);
            }
#endif
        };
        if (halo_l) run(std::integral_constant<int, 0>{});
        else if (halo_r) run(std::integral_constant<int, 2>{});
        else run(std::integral_constant<int, 1>{});
        return;
    }

#pragma unroll
    for (int k = 0; k < PF; k++) issue(k, k);
    for (int b = 0; b < nblk; b++) {
#pragma unroll
        for (int j = 0; j < HB; j++) {
            const int k = j % PF;
            const int s = b * HB + j;
            const bool live = s < H;
            const int y = UP ? H - 1 - s : s;
            const int rb = (s + 1) & 1, wb = s & 1;
            const uint32_t e = live ? cell(y) : NONE;
            uint32_t C[DPL];
            unpack_ct<CT, DPL>(rc_[k], C);
            uint32_t Ein[DPL], Win[DPL], Pin[DPL];
#pragma unroll
            for (int i = 0; i < DPL; i++) Ein[i] = Win[i] = Pin[i] = 0;
            if constexpr (EWIN) {
                unpack_ct<CT, DPL>(re_[k], Ein);
                unpack_ct<CT, DPL>(rw_[k], Win);
            }
            if constexpr (PARTR) unpack_ct<uint16_t, DPL>(rp_[k], Pin);
            // materialise the unpacked values before the slot is refilled: if the
            // unpack sinks below the refill, old and new slot values overlap and the
            // ring gets rotated by moves at the back-edge, which wait for the newest loads
#pragma unroll
            for (int i = 0; i < DPL; i++) {
                asm volatile("" : "+v"(C[i])::"memory");
                if constexpr (EWIN) asm volatile("" : "+v"(Ein[i]), "+v"(Win[i])::"memory");
                if constexpr (PARTR) asm volatile("" : "+v"(Pin[i])::"memory");
            }
            issue(k, s + PF);

            if (ROWSYNC && j > 0) wait_row(s);
            // diagonal predecessors: column c-1 (A) and c+1 (B) of the previous row
            uint32_t nA[DPL], nB[DPL];  // a halo wave leaves its other direction unset (never read)
            uint32_t mnA = 0, mnB = 0;
            if (!halo_r) {
                uint32_t LA[DPL];
                lds_get<DPL>(&lv[rb][0][c][g * DPL], LA);
                mnA = sweep_step<VL, DPL>(LA, lmin[rb][0][c], C, P1, P2, nA);
                if (wave_ragged) {  // columns outside [0, W1) stay at the entering state
#pragma unroll
                    for (int i = 0; i < DPL; i++) nA[i] = active ? nA[i] : 0u;
                    mnA = active ? mnA : 0u;
                }
                lds_put<DPL>(&lv[wb][0][c + 1][g * DPL], nA);
                if (g == 0) lmin[wb][0][c + 1] = mnA;
            }
            if (!halo_l) {
                uint32_t LB[DPL];
                lds_get<DPL>(&lv[rb][1][c + 2][g * DPL], LB);
                mnB = sweep_step<VL, DPL>(LB, lmin[rb][1][c + 2], C, P1, P2, nB);
                if (wave_ragged) {
#pragma unroll
                    for (int i = 0; i < DPL; i++) nB[i] = active ? nB[i] : 0u;
                    mnB = active ? mnB : 0u;
                }
                lds_put<DPL>(&lv[wb][1][c + 1][g * DPL], nB);
                if (g == 0) lmin[wb][1][c + 1] = mnB;
            }
            // snapshot of the block's last row for the neighbouring strips' halos
            if (j == HB - 1 && b + 1 < nblk) {
                const bool pa = wave == NCW - 2 && has_right, pb = wave == 1 && has_left;  // wave-uniform
                if (pa || pb) {
                    const uint32_t tag = tag0 | (uint32_t)(b + 1);
                    const size_t rec = gbase(wg, pa ? 0 : 1, b);  // HM = 1 here: column kl of the record
#pragma unroll
                    for (int q = 0; q < NG; q++) {
                        const uint32_t lo = pa ? nA[2 * q] : nB[2 * q];
                        const uint32_t hi = 2 * q + 1 < DPL ? (pa ? nA[2 * q + 1] : nB[2 * q + 1]) : 0u;
                        __builtin_amdgcn_raw_buffer_store_b64(u32x2{lo | (hi << 16), tag}, rhop,
                                                              (uint32_t)((rec + (size_t)(q * HW + kl) * VL + g) * 8), 0, 16);
                    }
                    if (g == 0)
                        __builtin_amdgcn_raw_buffer_store_b64(u32x2{pa ? mnA : mnB, tag}, rhop,
                                                              (uint32_t)((rec + G::NDAT + kl) * 8), 0, 16);
                }
            }

            uint32_t out[DPL];  // MODE 0: partial sum of the three directions
#pragma unroll
            for (int i = 0; i < DPL; i++) out[i] = 0;
            uint32_t recw = 0, nbw = 0;
            bool wpx = false;
            if (own) {
                uint32_t nV[DPL];
                const uint32_t mnV = sweep_step<VL, DPL>(LV, mV, C, P1, P2, nV);
#pragma unroll
                for (int i = 0; i < DPL; i++) LV[i] = nV[i];
                mV = mnV;
                if constexpr (MODE == 0) {
#pragma unroll
                    for (int i = 0; i < DPL; i++) out[i] = nV[i] + nA[i] + nB[i];
                } else {
                    uint32_t S[DPL];
                    uint32_t key = 0xFFFFFFFFu;
                    const bool pad = sizeof(CT) == 2 && a.Dv < D;  // padded cost volume (wave-uniform)
#pragma unroll
                    for (int i = 0; i < DPL; i++) {
                        uint32_t t = nV[i] + nA[i] + nB[i] + Ein[i] + Win[i];
                        if constexpr (PARTR) t += Pin[i];
                        if constexpr (sizeof(CT) == 2) t = min(t, 32767u);  // census sums stay below 2^11
                        if (pad && g * DPL + i >= a.Dv) t = 0xFFFFu;  // pad plane: never the minimum
                        S[i] = t;
                        key = min(key, (t << 16) | wta_rank(g * DPL + i, MODE == 1));
                    }
                    asm volatile("" ::: "memory");  // u32 / u128 stores, u16 loads of srow: no reordering
                    lds_put<DPL>(&srow[(wave - 1) % (NCW - 2)][kl][g * DPL], S);
                    asm volatile("" ::: "memory");
                    key = group_min<VL>(key);
                    const uint32_t minS = key >> 16;
                    const int best = wta_unrank(key & 0xFFFF, MODE == 1);  // MODE 1 = 5 paths
                    // far entries (|d - best| > 1) below the uniqueness threshold
                    uint32_t far = 0;
                    const int gb = g * DPL - best + 1;  // d - best + 1 of element 0
                    if (ku > 0) {  // S, minS < 2^15, ku <= 100: 24-bit multiplies are exact (full rate)
                        const uint32_t lim = __umul24(minS, 100u);
#pragma unroll
                        // (S <= 32767: not a pad plane; real sums never exceed it)
                        for (int i = 0; i < DPL; i++)
                            far = max(far, __umul24(S[i], (uint32_t)ku) < lim && (sizeof(CT) == 1 || S[i] <= 32767u)
                                               ? (uint32_t)(gb + i) : 0u);
                    } else {  // uniquenessRatio >= 100: the product form (rare)
#pragma unroll
                        for (int i = 0; i < DPL; i++)
                            far = max(far, (int)S[i] * ku < (int)minS * 100 && (sizeof(CT) == 1 || S[i] <= 32767u)
                                               ? (uint32_t)(gb + i) : 0u);
                    }
                    far = group_max<VL>(far);
                    const bool ok = far <= 2u && minS < 32767u;
                    const int bm = max(best - 1, 0), bq = min(best + 1, D - 1);
                    const uint32_t Sm = srow[(wave - 1) % (NCW - 2)][kl][bm];
                    const uint32_t Sq = srow[(wave - 1) % (NCW - 2)][kl][bq];
                    // disp2 candidate / sub-pixel inputs for k_lr_rows (~0: rejected)
                    recw = ok ? ((minS << 16) | (uint32_t)best) : 0xFFFFFFFFu;
                    nbw = Sm | (Sq << 16);
                    wpx = g == 0 && active && live;
                }
            }
            if constexpr (MODE == 0) {
                bstore_n<uint16_t, DPL, SWEEP_STREAM_AUX>(rp, own ? boff(e, 2) : kOOB, out);
            } else {
                const uint32_t px = (uint32_t)y * (uint32_t)a.W + (uint32_t)(x1 + a.minX1);
                __builtin_amdgcn_raw_buffer_store_b32(recw, rrec, wpx ? px * 4 : kOOB, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b32(nbw, rnb, wpx ? px * 4 : kOOB, 0, 0);
            }
            end_row(j, s);
        }
        if (b + 1 < nblk) lds_barrier();  // the poller has written the halo snapshot
    }
}

#if !defined(SWEEP_MODE) || (SWEEP_MODE == 0 && !SWEEP_WIDE)  // one unit owns the non-template kernel
// Winner's sub-pixel value, disp2 (right-view argmin, cv::StereoSGBM's
// disp2/disp2cost) and the disp12MaxDiff check from the WTA sweep's per-pixel
// records: the tail of k_wta (sm_paths.hpp) over one row per workgroup.
// rec = minS << 16 | best (~0: rejected by the uniqueness test or saturated),
// nb = S[best-1] | S[best+1] << 16.  Columns outside [minX1, maxX1) are
// INVALID.  blockIdx = (y, pair); dynamic LDS = 4*W bytes (disp2 keys) + 2*W
// (the row's sub-pixel disparities).
// wta (may be null): the integer WTA index per pixel (best, or -1 where rejected or outside
// [minX1, maxX1)), before the sub-pixel step, the LR check and the median.
__global__ void __launch_bounds__(256) k_lr_rows(const uint32_t* __restrict__ rec, const uint32_t* __restrict__ nbs,
                                                 int16_t* __restrict__ out, int16_t* __restrict__ wta, int H, int W,
                                                 int D, int minD, int minX1, int maxX1, int disp12,
                                                 const uint32_t* guard)
{
    // a strip of the group gave up: the guarded per-direction fallback (running beside this
    // kernel on another stream) writes the maps instead
    if (guard && __hip_atomic_load(guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
    extern __shared__ uint32_t key2[];
    int16_t* drow = reinterpret_cast<int16_t*>(key2 + W);
    const int y = blockIdx.x;
    const size_t row = ((size_t)blockIdx.y * H + y) * W;
    const int INVALID = (minD - 1) * 16;
    for (int X = threadIdx.x; X < W; X += 256) {
        key2[X] = 0xFFFFFFFFu;
        drow[X] = (int16_t)INVALID;
        if (wta && (X < minX1 || X >= maxX1)) wta[row + X] = -1;
    }
    __syncthreads();
    for (int X = minX1 + (int)threadIdx.x; X < maxX1; X += 256) {
        const uint32_t r = rec[row + X];
        if (wta) wta[row + X] = r != 0xFFFFFFFFu ? (int16_t)(r & 0xFFFF) : (int16_t)-1;
        if (r != 0xFFFFFFFFu) {
            const int best = (int)(r & 0xFFFF), minS = (int)(r >> 16);
            atomicMin(&key2[X - best - minD], (r & 0xFFFF0000u) | (uint32_t)(0xFFFF - X));
            int d16 = best * 16;
            if (best > 0 && best < D - 1) {
                const uint32_t nb = nbs[row + X];
                const int Sm = (int)(nb & 0xFFFF), Sq = (int)(nb >> 16);
                d16 += subpix_step(Sm, Sq, minS);  // C truncation
            }
            drow[X] = (int16_t)(d16 + minD * 16);
        }
    }
    __syncthreads();
    for (int X = threadIdx.x; X < W; X += 256) {
        int d1 = drow[X];
        if (X >= minX1 && X < maxX1 && d1 != INVALID) {
            const int _d = d1 >> 4, d_ = (d1 + 15) >> 4;
            const int _x = X - _d, x_ = X - d_;
            bool rej1 = false, rej2 = false;
            if (_x >= 0 && _x < W) {
                const uint32_t kk = key2[_x];
                const int d2 = kk == 0xFFFFFFFFu ? INVALID : (int)(0xFFFF - (kk & 0xFFFF)) - _x;
                rej1 = d2 >= minD && abs(d2 - _d) > disp12;
            }
            if (x_ >= 0 && x_ < W) {
                const uint32_t kk = key2[x_];
                const int d2 = kk == 0xFFFFFFFFu ? INVALID : (int)(0xFFFF - (kk & 0xFFFF)) - x_;
                rej2 = d2 >= minD && abs(d2 - d_) > disp12;
            }
            if (rej1 && rej2) d1 = INVALID;
        }
        out[row + X] = (int16_t)d1;
    }
}
#endif

}  // namespace smk
