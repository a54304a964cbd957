// sm_sweep_host.hpp — host interface of the fused-sweep kernels (sm_sweep.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace smk {

// MODE: 0 = down sweep writing the u16 partial (8 paths, first pass)
//       1 = down sweep + E/W + WTA (MODE_SGBM: 5 paths)
//       2 = up sweep + E/W + down partial + WTA (8 paths, second pass)
//       3 = down sweep + in-kernel E/W lines (speculative strip segments)
//           writing the u16 partial S + SE + SW + E + W and the segments' boundary states
//       4 = up sweep + partial + WTA (8 paths, second pass after MODE 3: no E/W volumes)
#ifndef SWEEP_STATS
#define SWEEP_STATS 0  // sm_sweep.hpp: wait-cycle counters (variant builds)
#endif

struct SweepArgs {
    const uint8_t* cost;  // [pair][H][W1][D] of CT
    size_t cost_pair;     // bytes
    const uint8_t* ew;    // E volume; W at ew + ew_slot (same layout, CT)
    size_t ew_pair, ew_slot;
    uint16_t* part;  // [pair][H][W1][D] u16 partial (written by MODE 0, read by MODE 2)
    size_t part_pair;  // bytes
    unsigned long long* hop;  // halo snapshot granules [pair][nwg][2][nblk][NGR]
    size_t hop_pair;          // granules per pair
    uint32_t* rec;   // [pair][H][W] WTA winners (minS << 16 | best, ~0 rejected), domain columns only
    uint32_t* nb;    // [pair][H][W] S[best-1] | S[best+1] << 16 (sub-pixel inputs)
    uint32_t* err;   // bit 0: a halo poll timed out
    int H, W, W1, D, minD, minX1, P1, P2, uniq;
    int Dv;        // real disparities (< D only for a padded cost volume: the WTA ignores d >= Dv)
    float inv_ku;  // 1 / (100 - uniq) (uniqueness threshold estimate; exact fix-up on the device)
    int nwg;
    uint32_t epoch;  // 1..65535, distinct from the previous launches on the same hop buffer
    int dbg;         // timing ablations only: 1 no waiting in the halo polls, 2 no polls, 4 no row barriers
    unsigned long long* stats;  // SWEEP_STATS builds only: per-mode wait-cycle counters (else null)
    // MODE 3: each strip's E and W line segments start `ewarm` (>= 1) columns outside the strip
    // from the zero state; their state entering the strip and at its far end go to
    // st[pair][y][strip][dir][2][D] (CT elements) for the patch pass (k_ew_patch)
    uint8_t* st;
    size_t st_pair;  // bytes
    int ewarm;
    int ewguess;  // 0: the zero state; 1 (tests): a deliberately wrong start state, every segment repaired
    // MODE 3 row bands (one or two pairs per call: DESIGN.md §4.5): workgroup blockIdx.x =
    // band * nwg + strip; band b owns rows [b * band_h, (b + 1) * band_h) and starts vwarm rows
    // above them from the zero state (a speculation: k_band_patch repairs the vertical paths
    // where it did not meet the true state).  The own columns' S / SE / SW states at the row
    // above the band (speculative) and at its last row go to
    // vst[pair][band][0 / 1][3][W1][D] (CT, min-0 form).  nband <= 1: one band of all rows.
    int nband, band_h, vwarm;
    int vguess;    // tests: bands > 0 start from a deliberately wrong state inside the domain
    int hop_nblk;  // halo blocks per strip record in the hop buffer (>= every band's block count)
    uint8_t* vst;
    size_t vst_pair;  // bytes
    // XCD-aware placement (xcd_per > 0): a 1-D grid of 8 * xcd_per workgroups; workgroup i runs
    // item (i % 8) * xcd_per + i / 8 of the (pair, band, strip) list (items >= xcd_total exit at
    // once), so each XCD holds a run of adjacent strips that share cost rows in its L2
    int xcd_per, xcd_total;
};


struct SweepInfo {
    int cw;             // own columns per workgroup (strip width)
    int hb;             // rows per halo block
    int ngr;            // halo granules per (strip, direction, block)
    int threads;        // threads per workgroup
    int blocks_per_cu;  // occupancy API answer for that block size
    int impl;           // kernel: 0 k_sweep narrow strips, 1 wide strips, 2 latency strips, 3 / 6 k_sweep2
    int dpl;            // disparities per lane (the per-wave work of a row scales with it)
    int ncw;            // compute waves (the threads also count the poller and MODE 3's line waves)
};

template <typename CT, int MODE, class F>
hipError_t with_d(int D, F& f);

// per mode (one translation unit each); hipErrorInvalidValue when (D, ct_bytes) is not built.
// variant 0: k_sweep, wide strips where built and usable (no scratch, >= 1 block per CU),
// narrow (7 compute waves) elsewhere; 1: narrow strips; 3 / 6: k_sweep2 (sm_sweep2.hpp) with
// that many compute waves per workgroup where built (u8 costs, D = 128), k_sweep elsewhere.
// sweep_info reports the kernel it picked in SweepInfo::impl; sweep_launch takes that impl.
hipError_t sweep_info_m0(int D, int ct_bytes, int variant, int device, SweepInfo* out);
hipError_t sweep_info_m1(int D, int ct_bytes, int variant, int device, SweepInfo* out);
hipError_t sweep_info_m2(int D, int ct_bytes, int variant, int device, SweepInfo* out);
hipError_t sweep_info_m3(int D, int ct_bytes, int variant, int device, SweepInfo* out);
hipError_t sweep_info_m4(int D, int ct_bytes, int variant, int device, SweepInfo* out);
hipError_t sweep_info_wide_m0(int D, int ct_bytes, int device, SweepInfo* out);
hipError_t sweep_info_wide_m1(int D, int ct_bytes, int device, SweepInfo* out);
hipError_t sweep_info_wide_m2(int D, int ct_bytes, int device, SweepInfo* out);
hipError_t sweep_info_wide_m3(int D, int ct_bytes, int device, SweepInfo* out);
hipError_t sweep_info_wide_m4(int D, int ct_bytes, int device, SweepInfo* out);
hipError_t sweep_info_lat_m0(int D, int ct_bytes, int device, SweepInfo* out);
hipError_t sweep_info_lat_m1(int D, int ct_bytes, int device, SweepInfo* out);
hipError_t sweep_info_lat_m2(int D, int ct_bytes, int device, SweepInfo* out);
hipError_t sweep_info_lat_m3(int D, int ct_bytes, int device, SweepInfo* out);
hipError_t sweep_info_lat_m4(int D, int ct_bytes, int device, SweepInfo* out);
hipError_t sweep_launch_lat_m0(int D, int ct_bytes, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_lat_m1(int D, int ct_bytes, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_lat_m2(int D, int ct_bytes, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_lat_m3(int D, int ct_bytes, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_lat_m4(int D, int ct_bytes, const SweepArgs& a, int npairs, hipStream_t stream);
// grid (a.nwg, npairs), SweepInfo::threads threads
hipError_t sweep_launch_m0(int D, int ct_bytes, int variant, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_m1(int D, int ct_bytes, int variant, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_m2(int D, int ct_bytes, int variant, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_m3(int D, int ct_bytes, int variant, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_m4(int D, int ct_bytes, int variant, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_wide_m0(int D, int ct_bytes, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_wide_m1(int D, int ct_bytes, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_wide_m2(int D, int ct_bytes, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_wide_m3(int D, int ct_bytes, const SweepArgs& a, int npairs, hipStream_t stream);
hipError_t sweep_launch_wide_m4(int D, int ct_bytes, const SweepArgs& a, int npairs, hipStream_t stream);

inline hipError_t sweep_info(int D, int ct_bytes, int mode, int variant, int device, SweepInfo* out)
{
    typedef hipError_t (*InfoW)(int, int, int, SweepInfo*);
    typedef hipError_t (*InfoV)(int, int, int, int, SweepInfo*);
    static const InfoW lat[5] = {sweep_info_lat_m0, sweep_info_lat_m1, sweep_info_lat_m2, sweep_info_lat_m3,
                                 sweep_info_lat_m4};
    static const InfoW wide[5] = {sweep_info_wide_m0, sweep_info_wide_m1, sweep_info_wide_m2, sweep_info_wide_m3,
                                  sweep_info_wide_m4};
    static const InfoV narrow[5] = {sweep_info_m0, sweep_info_m1, sweep_info_m2, sweep_info_m3, sweep_info_m4};
    if (mode < 0 || mode > 4) return hipErrorInvalidValue;
    if (variant == 2) return lat[mode](D, ct_bytes, device, out);  // latency instances (kLatNcw compute waves)
    if (variant == 0) {
        const hipError_t e = wide[mode](D, ct_bytes, device, out);
        if (e == hipSuccess) return e;
    }
    return narrow[mode](D, ct_bytes, variant == 1 ? 0 : variant, device, out);
}
inline hipError_t sweep_launch(int D, int ct_bytes, int mode, int impl, const SweepArgs& a, int npairs,
                               hipStream_t stream)
{
    typedef hipError_t (*LaunchW)(int, int, const SweepArgs&, int, hipStream_t);
    typedef hipError_t (*LaunchV)(int, int, int, const SweepArgs&, int, hipStream_t);
    static const LaunchW lat[5] = {sweep_launch_lat_m0, sweep_launch_lat_m1, sweep_launch_lat_m2, sweep_launch_lat_m3,
                                   sweep_launch_lat_m4};
    static const LaunchW wide[5] = {sweep_launch_wide_m0, sweep_launch_wide_m1, sweep_launch_wide_m2,
                                    sweep_launch_wide_m3, sweep_launch_wide_m4};
    static const LaunchV narrow[5] = {sweep_launch_m0, sweep_launch_m1, sweep_launch_m2, sweep_launch_m3,
                                      sweep_launch_m4};
    if (mode < 0 || mode > 4) return hipErrorInvalidValue;
    if (impl == 2) return lat[mode](D, ct_bytes, a, npairs, stream);
    if (impl == 1) return wide[mode](D, ct_bytes, a, npairs, stream);
    return narrow[mode](D, ct_bytes, impl, a, npairs, stream);
}
// sub-pixel + disp2 + disp12MaxDiff check from the WTA sweep's records, one row per workgroup;
// wta (may be null): the integer WTA index [pair][H][W] (-1: rejected / outside the domain);
// guard (may be null): the group's give-up flag, the kernel writes nothing when it is set
hipError_t lr_rows_launch(const uint32_t* rec, const uint32_t* nb, int16_t* out, int16_t* wta, int G, int H, int W,
                          int D, int minD, int minX1, int maxX1, int disp12, const uint32_t* guard, hipStream_t stream);

// horizontal (E, W) path volumes, packed recurrence (sm_ew.hpp / sm_ew.hip)
struct EwArgs {
    const uint8_t* cost;  // [pair][H][W1][D] of CT
    size_t cost_pair;     // bytes
    uint8_t* out;         // E volume [pair][H][W1][D] of LT; W at out + out_slot
    size_t out_pair, out_slot;
    int H, W1, P1, P2;
    int nrb;  // workgroups per direction (filled by ew_launch)
    int wpb;  // waves per workgroup, 1..4 (0: 4)
    int prio;  // wave issue priority 0..3
};
// lanes per line: vl = 4, 8 or 16 (0 = the default for D); hipErrorInvalidValue when
// (D, ct_bytes, vl) is not built.  LT = CT (u8 census costs -> u8 volumes, u16 -> u16).
hipError_t ew_launch(int D, int ct_bytes, int vl, EwArgs a, int npairs, hipStream_t stream);

// Patch pass after a MODE 3 sweep (sm_ew.hpp k_ew_patch): per image row, every strip's
// speculative E / W segment is checked against the trusted state its neighbour hands over;
// where they differ the segment is recomputed from the trusted state and the partial
// corrected until the two trajectories meet
struct EwPatchArgs {
    const uint8_t* cost;  // [pair][H][W1][D] of CT
    size_t cost_pair;     // bytes
    uint16_t* part;       // [pair][H][W1][D] u16 partial written by MODE 3
    size_t part_pair;     // bytes
    uint8_t* st;          // MODE 3 boundary states [pair][H][nwg][2][2][D] of CT; phase A overwrites the
                          // s_k slot of a strip whose walk never met with its true far-end state c_k
    size_t st_pair;       // bytes
    int H, W1, nwg, cw, P1, P2;
    const uint32_t* guard;  // the group's give-up flag: nothing to patch when set (the fallback recomputes)
    unsigned long long* fixes;  // [0] strip segments recomputed, [1] of them never met within the strip (u64 atomics)
    int atom;  // 1: no partial cell can saturate (5 x path_max < 65536): atomic corrections, E and W side by side
};
// Vertical patch after a banded MODE 3 sweep (sm_ew.hpp k_band_patch): each
// column's S / SE / SW state entering a band (speculative, from the band's warmup rows) is checked
// against the band above's stored end state; where they differ both trajectories are stepped down
// the chain and (second - first) added to the partial until they meet, across later boundaries
// too (the contributions telescope to true - speculative; no hand-off between walks).
struct BandPatchArgs {
    const uint8_t* cost;  // [pair][H][W1][D] of CT
    size_t cost_pair;     // bytes
    uint16_t* part;       // [pair][H][W1][D] u16 partial (u32 atomics on u16 pairs: exact while no
                          // cell saturates, which the host guarantees)
    size_t part_pair;     // bytes
    const uint8_t* vst;   // [pair][band][2][3][W1][D] of CT (SweepArgs::vst), min-0 form
    size_t vst_pair;      // bytes
    int H, W1, nband, band_h, P1, P2;
    int nbx;              // workgroups per boundary (blockIdx.x)
    const uint32_t* guard;  // the group's give-up flag: nothing to patch when set
    unsigned long long* fixes;  // [0] chains repaired, [1] of them still apart past the next boundary (u64 atomics)
};
hipError_t band_patch_launch(int D, int ct_bytes, const BandPatchArgs& a, int npairs, hipStream_t stream);

// chunks of LPW * 8 path positions per row and direction the patch pass handles (its open-strip
// masks in LDS): strips of a pair it accepts (16-lane lines where D % 32 == 0, else 8-lane)
constexpr int kPatchMaxChunks = 8;
constexpr int patch_max_strips(int D) { return 1 + kPatchMaxChunks * (D % 32 == 0 ? 4 : 8) * 8; }
hipError_t ew_patch_launch(int D, int ct_bytes, const EwPatchArgs& a, int npairs, hipStream_t stream);

}  // namespace smk
