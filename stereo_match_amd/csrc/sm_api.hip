// sm_api.hip — C-ABI (include/stereo_match_amd.h) around the gfx950 kernels.
//
// Host side of the drop-in boundary for stereo_vision/stereo_vision.py:153-179
// (cv2.StereoSGBM_create(...).compute).  Parameter normalisation mirrors
// OpenCV computeDisparitySGBM (see oracle/sgm_np.py:normalize_params).
//
// Pipeline per launch group of G pairs:
//   cost (census | SGBM BT+box) -> path aggregation -> WTA + disp2/LR -> median
// all on the caller's stream (A).  Optional overlap (debug flag 64): WTA and
// median of group g run on an internal stream B while group g+1 aggregates
// paths on A, double-buffered over two buffer sets; A waits for B at the end
// of every call, so callers only ever synchronise with their own stream.
// Measured on MI355X the overlap is a net loss for the
// headline config — the two kernels slow each other more than they overlap —
// so it stays opt-in.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/stereo_match_amd.h"
#include "sm_cost.hpp"
#include "sm_paths.hpp"
#include "sm_post.hpp"
#include "sm_wls.hpp"
#include "sm_speckle.hpp"
#include "sm_reproject.hpp"
#include "sm_bm.hpp"
#include "sm_wide.hpp"
#include "sm_sweep_host.hpp"

// SM_ABLATIONS=1 (make ablation -> libstereo_match_amd_ablate.so) also builds the measured
// ablations that the product library leaves out: the row-WTA kernel (sm_rowwta.hpp), the
// hybrid engine, k_sweep2 (sm_sweep.hip) and the timing switches whose results are wrong
#ifndef SM_ABLATIONS
#define SM_ABLATIONS 0
#endif
#if SM_ABLATIONS
#include "sm_rowwta.hpp"
#define SM_VERSION "stereo_match_amd 0.3.0 (gfx950, ablation build)"
#else
#define SM_VERSION "stereo_match_amd 0.3.0 (gfx950)"
#endif

namespace {

thread_local std::string g_thread_error;

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
};

struct Norm {
    // D: disparities the kernels run (a multiple of 16); Dv: the caller's numDisparities.
    // They differ only for an external cost volume whose plane count is not a multiple of
    // 16 (mc-cnn: 228, mapTo3D_mc_cnn.py:71): its planes Dv..D-1 carry the pad cost
    // VOL_CMAX + P2 (k_cost_volume_f32), which no path value of a real disparity ever takes
    // as its minimum (vol_pad_cost), and the WTA kernels ignore them.
    int minD, D, Dv, maxD, bs, P1, P2, ftzero, uniq, disp12, speckle_ws, speckle_range, cost, mode;
    int minX1, maxX1, width1, ndirs, dpl;
    int cn;    // input channels (1 gray, 3 BGR)
    bool wide;  // SGBM cost outside the int16-exact range (or BGR): sm_wide.hpp path
};

struct TimedEvent {
    int stage, pairs;
    hipEvent_t a, b;
};

// per-group device buffers (double-buffered across launch groups)
struct BufSet {
    DevBuf census[2], cost, L, raw;
    DevBuf part, key2, pre;  // sweep engine: u16 partial sums, WTA winner records, sub-pixel inputs
    DevBuf st;               // in-sweep E/W lines (MODE 3): the strip segments' boundary states
    DevBuf vst;              // MODE 3 row bands: the vertical paths' boundary states
    hipEvent_t paths_done = nullptr, wta_done = nullptr;
    bool pending = false;  // wta_done recorded and not yet waited for by stream A
};

// the E/W patch pass with atomic corrections where no partial cell can saturate (k_ew_patch ATOM)
#ifndef EW_PATCH_ATOM
#define EW_PATCH_ATOM 1
#endif

// debug flags (sm_set_debug_flags); 1 skip horizontal, 2 skip vertical and 4 drop stores are read in-kernel
constexpr int DBG_VL16 = 8, DBG_STORE_W = 16, DBG_ROW = 32, DBG_OVERLAP = 64, DBG_H64 = 512, DBG_NO_C8 = 1024;
// 256: the sweep engine's E/W volumes from the per-direction engine's row lines instead of
// the packed k_ew (ew_lanes); 128 and 1 << 27: the fused sweeps on k_sweep2 (see sweep_variant)
constexpr int DBG_OLD_EW = 256, DBG_SWEEP_V2 = 128, DBG_SWEEP2_NW = 1 << 27;
// WLS smoother timing ablations (results wrong): 1 << 28 skips the FGS sweeps, 1 << 29 its
// global loads/stores
constexpr int DBG_FGS_NO_SWEEP = 1 << 28, DBG_FGS_NO_MEM = 1 << 29;
// 1 << 30 (valid results): no Infinity-Cache-sized launch groups (group_size)
constexpr int DBG_NO_MALL_GROUPS = 1 << 30;
// 1 << 19 (valid results): the fused sweeps on narrow strips (7 compute waves) everywhere;
// 1 << 21: on wide strips wherever built and they fit, whatever sweep_model prefers
constexpr int DBG_NARROW_SWEEPS = 1 << 19, DBG_WIDE_SWEEPS = 1 << 21;
// 4096: per-direction engine (one path volume per direction + k_wta) instead of the fused sweeps
constexpr int DBG_LEGACY = 4096, DBG_SWEEP1 = 8192, DBG_SWEEP8 = 16384, DBG_HYBRID = 32768;
constexpr int DBG_COST_TILE = 1 << 22;
// 1 << 20 (valid results): compute_disparity runs its right matcher beside the left one on
// the twin context's stream instead of before it on the caller's stream
constexpr int DBG_CONCURRENT_LR = 1 << 20;
// 1 << 23 (valid results): raise every fused-sweep group's give-up flag, so the
// guarded per-direction fallback recomputes the group (tests the recovery path)
constexpr int DBG_FORCE_FALLBACK = 1 << 23;
// words of ctx->sweep_err: per-buffer-set group flags (set by a sweep strip that gave
// up waiting; cleared by the host before each group), the sticky error of the
// (unguarded) hybrid engine, and the count of fallback recomputations
constexpr int ERR_GROUP0 = 0, ERR_STICKY = 32, ERR_FALLBACKS = 48;
// (u64 words at 52, 54) the external cost-volume cells clamped by the quantisation window / NaN
// cells, and (u64 words at 56, 58) the E/W strip segments the patch pass recomputed and those
// whose walk never met within the strip (64-bit: a service repairs hundreds of segments per pair)
constexpr int ERR_VOL_CLAMPED = 52, ERR_VOL_NAN = 54, ERR_EW_REPAIRS = 56, ERR_EW_OPEN = 58;
// (u64 words at 60, 62) the row bands' vertical chains the band patch repaired / carried on
constexpr int ERR_BAND_REPAIRS = 60, ERR_BAND_OPEN = 62;
// timing ablation: no guarded fallback launches after the sweeps
constexpr int DBG_NO_FALLBACK = (int)0x80000000u;
// flags only the ablation build (SM_ABLATIONS) accepts: timing switches whose results are
// wrong (1, 2, 4 in the path kernels; 1 << 24..26 in the sweeps; 1 << 28, 1 << 29 in the WLS
// smoother; 1 << 31), the row-WTA kernel (16, 32), k_sweep2 (128, 1 << 27), the hybrid engine
constexpr int kAblationFlags = 1 | 2 | 4 | DBG_STORE_W | DBG_ROW | DBG_SWEEP_V2 | DBG_SWEEP2_NW | DBG_HYBRID |
                               (7 << 24) | DBG_FGS_NO_SWEEP | DBG_FGS_NO_MEM | DBG_NO_FALLBACK;

}  // namespace

struct sm_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;  // stream A
    hipStream_t side = nullptr;    // stream B
    DevBuf img[2], planes, out, dbg, volbuf, sp_parent, sp_count, rp_in, rp_out, rp_min, bm_pre[2], bm_cost;
    DevBuf wls_num, wls_den, wls_inter, wls_w, wls_disp[2], wls_out;  // WLS scratch
    DevBuf wls_R, wls_IT;         // WLS: Thomas pivots / elimination factors of every pass
    hipStream_t wls_stream = nullptr;  // compute_disparity: WLS weights + pivots beside the matchers
    hipStream_t lr_stream = nullptr;   // compute_disparity: the left matcher, staggered behind the right one
    hipEvent_t ev_stagger = nullptr;
    // (set by the caller for one call) recorded on the stream right after a MODE 3 down sweep;
    // sweep_done_hit tells the caller it was
    hipEvent_t sweep_done_ev = nullptr;
    bool sweep_done_hit = false;
    int tune_lr_stagger = 0;  // SM_TUNE_LR_STAGGER: 0 automatic (on), -1 off
    hipEvent_t ev_wls_fork = nullptr, ev_wls_ready = nullptr;
    DevBuf hop, sweep_err;  // sweep engine: strip-boundary granules, device error word
    DevBuf volwin;          // external cost volumes, automatic window: [pair] min/max keys + offset/scale

    void* pin = nullptr;    // page-locked host staging of the host-pointer entry points (HostStage)
    size_t pin_n = 0;
    // compute_disparity: the right matcher runs on a twin context (own streams and
    // buffers); created on first use, destroyed with this one
    sm_ctx* twin = nullptr;
    hipEvent_t ev_lr_fork = nullptr, ev_lr_join = nullptr;
    std::vector<uint32_t> cu_mask;  // sm_set_cu_mask words (applied to the twin too)
    uint32_t hop_epoch = 0;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;  // sweep engine: E/W kernel on the side stream
    hipEvent_t ev_fb_fork = nullptr, ev_fb_join = nullptr;  // sweep engine: fallback beside the LR pass
    hipEvent_t ev_ew_done = nullptr;  // banded lines: the E/W patch on the side stream (before the WTA)
    const uint32_t* fb_guard = nullptr;  // set while enqueuing a group's guarded per-direction fallback
    hipStream_t wta_override = nullptr;  // stream of the WTA launch when it is not stream_b()
    const uint32_t* wta_skip = nullptr;  // the WTA row kernel exits when this flag is set (WtaArgs::skip)
    int16_t* wta_dst = nullptr;  // integer WTA index of the current launch group (sm_compute_wta_*), or null
    BufSet set[2];
    int next_set = 0;
    // geometry of the last computation (for sm_debug_fetch): its last pair
    int lastH = 0, lastW = 0, last_width1 = 0, lastD = 0, last_ndirs = 0, last_cost = 0, last_minD = 0;
    int last_minX1 = 0, last_index = 0, last_set = 0;
    size_t last_L_pair = 0;
    uint32_t timing = 0;  // stages timed (bit = SM_STAGE_*), sm_set_timing
    int dbg_flags = 0;
    // sm_set_tuning knobs (0 = automatic)
    int tune_ew_lanes = 0, tune_sweep_ncw = 0, tune_ew_waves = 0, tune_ew_prio = 0;
    int tune_ew_warmup = 0, tune_sweep_lines = 0;  // in-sweep E/W lines: warmup columns, -1 off / 1 on
    int tune_ew_guess = 0;                         // 1: the lines start from a wrong state (tests)
    int tune_bands = 0, tune_band_warmup = 0, tune_band_guess = 0;  // MODE 3 row bands (SM_TUNE_BANDS ...)
    int tune_cost_wgs = 0;  // k_sgbm_cost2 workgroups a launch aims for (SM_TUNE_COST_WGS; 0: SGBM_COST2_WGS)
    int tune_sweep_xcd = 0;  // SM_TUNE_SWEEP_XCD: 1 the XCD-aware strip placement, -1 / 0 off
    long long line_groups = 0;  // launch groups run with the in-sweep E/W lines (SM_COUNTER_LINE_GROUPS)
    long long band_groups = 0;  // of them, with row bands (SM_COUNTER_BAND_GROUPS)
    long long line_strips = 0;  // strips x pairs of those groups (SM_COUNTER_LINE_STRIPS)
    std::vector<TimedEvent> pending;
    std::vector<hipEvent_t> free_events;
    double stage_ms[SM_NUM_STAGES] = {0};
    long long stage_launches[SM_NUM_STAGES] = {0};
    long long stage_pairs[SM_NUM_STAGES] = {0};
    std::string err;
};

namespace {

int fail(sm_ctx* ctx, int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    g_thread_error = buf;
    return code;
}

#define HIP_TRY(ctx, expr)                                                                           \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return fail((ctx), SM_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_),   \
                        __FILE__, __LINE__);                                                          \
    } while (0)

// (re)allocate; callers make sure no queued work still uses the old buffer
int ensure(sm_ctx* ctx, DevBuf& b, size_t bytes)
{
    if (b.n >= bytes && b.p) return SM_OK;
    if (b.p) {
        HIP_TRY(ctx, hipDeviceSynchronize());
        (void)hipFree(b.p);
        b.p = nullptr;
        b.n = 0;
    }
    size_t want = std::max<size_t>(bytes, 256);
    HIP_TRY(ctx, hipMalloc(&b.p, want));
    b.n = want;
    return SM_OK;
}

int normalize(sm_ctx* ctx, const sm_params* p, int H, int W, Norm& n, int cn = 1)
{
    if (!p) return fail(ctx, SM_E_ARG, "params is NULL");
    if (H <= 0 || W <= 0) return fail(ctx, SM_E_ARG, "empty image (%dx%d)", W, H);
    if (W > 32767) return fail(ctx, SM_E_UNSUPPORTED, "width %d > 32767", W);
    n.minD = p->min_disparity;
    n.D = n.Dv = p->num_disparities;
    if (p->cost_kind == SM_COST_VOLUME) {
        // an external volume has the planes it was made with (OpenCV's %16 assert belongs
        // to StereoSGBM's own cost); the kernels run the next multiple of 16
        if (n.Dv <= 0) return fail(ctx, SM_E_ARG, "cost volume needs at least one disparity plane (got %d)", n.Dv);
        n.D = (n.Dv + 15) & ~15;
    } else if (n.D <= 0 || n.D % 16 != 0) {
        return fail(ctx, SM_E_ARG, "numDisparities must be a positive multiple of 16 (got %d)", n.D);
    }
    if (n.D > 256) return fail(ctx, SM_E_UNSUPPORTED, "numDisparities %d > 256 not built", n.Dv);
    n.maxD = n.minD + n.Dv;
    n.bs = p->block_size > 0 ? p->block_size : 5;
    n.ftzero = std::max(p->pre_filter_cap, 15) | 1;
    n.uniq = p->uniqueness_ratio >= 0 ? p->uniqueness_ratio : 10;
    n.disp12 = p->disp12_max_diff > 0 ? p->disp12_max_diff : 1;
    n.P1 = p->P1 > 0 ? p->P1 : 2;
    n.P2 = std::max(p->P2 > 0 ? p->P2 : 5, n.P1 + 1);
    n.speckle_ws = p->speckle_window_size;
    n.speckle_range = p->speckle_range;
    n.cost = p->cost_kind;
    n.mode = p->mode;
    if (n.cost != SM_COST_SGBM && n.cost != SM_COST_CENSUS && n.cost != SM_COST_VOLUME)
        return fail(ctx, SM_E_ARG, "cost_kind %d unknown", n.cost);
    if (n.mode != SM_MODE_SGBM && n.mode != SM_MODE_HH)
        return fail(ctx, SM_E_UNSUPPORTED, "mode %d not supported (5 = MODE_SGBM, 8 = MODE_HH)", n.mode);
    if (cn != 1 && cn != 3) return fail(ctx, SM_E_ARG, "images must have 1 or 3 channels (got %d)", cn);
    if (cn != 1 && n.cost != SM_COST_SGBM) return fail(ctx, SM_E_UNSUPPORTED, "colour input needs the SGBM cost");
    n.cn = cn;
    n.wide = false;
    if (n.cost == SM_COST_SGBM) {
        // the fast kernels need every sum below 2^15 (no int16 saturation or wrap);
        // outside that, and for BGR input, the sm_wide.hpp path restates OpenCV's
        // x86 int16 arithmetic.  Window side 2*(bs/2)+1, as OpenCV's SW2 = bs/2.
        const int side = 2 * (n.bs / 2) + 1;
        const int maxpix = 2 * n.ftzero + (255 >> 2);
        n.wide = cn != 1 || n.bs / 2 > 5 || (long long)side * side * maxpix + n.P2 > 16383;
        if (n.ftzero > 127) return fail(ctx, SM_E_UNSUPPORTED, "preFilterCap %d > 126 not built", p->pre_filter_cap);
        if (n.bs / 2 > 27) return fail(ctx, SM_E_UNSUPPORTED, "blockSize %d > 55 not built", n.bs);
        if (n.P1 > 32767 || n.P2 > 32767) return fail(ctx, SM_E_UNSUPPORTED, "P1/P2 above 32767 not built");
    } else if (n.cost == SM_COST_CENSUS) {
        if (62 + n.P2 > 255) return fail(ctx, SM_E_UNSUPPORTED, "census mode needs P2 <= 193 (8-bit path values)");
    } else {
        if (smk::VOL_CMAX + n.P2 > 16383)
            return fail(ctx, SM_E_UNSUPPORTED, "cost-volume mode needs P2 <= %d", 16383 - smk::VOL_CMAX);
    }
    if (!n.wide && (n.P1 > 16383 || n.P2 > 16383)) return fail(ctx, SM_E_UNSUPPORTED, "P1/P2 too large");
    n.minX1 = std::max(n.maxD, 0);
    n.maxX1 = W + std::min(n.minD, 0);
    n.width1 = n.maxX1 - n.minX1;
    n.ndirs = n.mode;
    n.dpl = n.D / 16;
    return SM_OK;
}

hipEvent_t get_event(sm_ctx* ctx)
{
    if (!ctx->free_events.empty()) {
        hipEvent_t e = ctx->free_events.back();
        ctx->free_events.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

struct StageTimer {
    sm_ctx* ctx;
    hipStream_t s;
    int stage, pairs;
    hipEvent_t a = nullptr;
    StageTimer(sm_ctx* c, hipStream_t st, int stg, int np) : ctx(c), s(st), stage(stg), pairs(np)
    {
        if (ctx->timing & (1u << stage)) {
            a = get_event(ctx);
            (void)hipEventRecord(a, s);
        }
    }
    ~StageTimer()
    {
        if (a) {
            hipEvent_t b = get_event(ctx);
            (void)hipEventRecord(b, s);
            ctx->pending.push_back({stage, pairs, a, b});
        }
    }
};

void harvest_timing(sm_ctx* ctx)
{
    for (auto& t : ctx->pending) {
        (void)hipEventSynchronize(t.b);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, t.a, t.b);
        ctx->stage_ms[t.stage] += ms;
        ctx->stage_launches[t.stage] += 1;
        ctx->stage_pairs[t.stage] += t.pairs;
        ctx->free_events.push_back(t.a);
        ctx->free_events.push_back(t.b);
    }
    ctx->pending.clear();
}

// Page-locked staging for the host-pointer entry points: inputs are packed row
// by row into pinned memory and cross PCIe as one DMA each (a pageable
// hipMemcpy2D moves one row per transfer: ~3 ms for a KITTI image); outputs
// land in pinned memory and are copied out once the stream has synchronised.
// The whole call's bytes are reserved up front, so the buffer never moves
// while a DMA of this call is queued (host entry points are synchronous, so
// nothing of a previous call is in flight either).
struct HostStage {
    struct Out {
        void* dst;
        size_t off, bytes;
    };
    sm_ctx* ctx;
    size_t used = 0;
    std::vector<Out> outs;
    explicit HostStage(sm_ctx* c) : ctx(c) {}
    int reserve(size_t bytes)
    {
        if (ctx->pin_n >= bytes && ctx->pin) return SM_OK;
        if (ctx->pin) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            (void)hipHostFree(ctx->pin);
            ctx->pin = nullptr;
            ctx->pin_n = 0;
        }
        HIP_TRY(ctx, hipHostMalloc(&ctx->pin, bytes, hipHostMallocDefault));
        ctx->pin_n = bytes;
        return SM_OK;
    }
    uint8_t* take(size_t bytes)
    {
        uint8_t* p = (uint8_t*)ctx->pin + used;
        used += (bytes + 255) & ~size_t(255);
        return p;
    }
    // rows x row_bytes from host (pitch src_pitch) -> contiguous device buffer
    int in(void* dev, const void* src, size_t rows, size_t row_bytes, size_t src_pitch)
    {
        uint8_t* p = take(rows * row_bytes);
        if (src_pitch == row_bytes)
            std::memcpy(p, src, rows * row_bytes);
        else
            for (size_t r = 0; r < rows; r++) std::memcpy(p + r * row_bytes, (const uint8_t*)src + r * src_pitch, row_bytes);
        StageTimer t(ctx, ctx->stream, SM_STAGE_H2D, 1);
        HIP_TRY(ctx, hipMemcpyAsync(dev, p, rows * row_bytes, hipMemcpyHostToDevice, ctx->stream));
        return SM_OK;
    }
    int out(void* dst, const void* dev, size_t bytes)
    {
        uint8_t* p = take(bytes);
        outs.push_back({dst, (size_t)(p - (uint8_t*)ctx->pin), bytes});
        StageTimer t(ctx, ctx->stream, SM_STAGE_D2H, 1);
        HIP_TRY(ctx, hipMemcpyAsync(p, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
        return SM_OK;
    }
    int finish()
    {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        for (const Out& o : outs) std::memcpy(o.dst, (const uint8_t*)ctx->pin + o.off, o.bytes);
        return SM_OK;
    }
};
// staged bytes of n buffers of `bytes` each (256-byte slots)
inline size_t stage_bytes(size_t bytes, int n = 1) { return (size_t)n * ((bytes + 255) & ~size_t(255)); }

int grid_for(size_t n)
{
    size_t g = (n + 255) / 256;
    return (int)std::min<size_t>(std::max<size_t>(g, 1), 8192);
}

size_t elem_bytes(const Norm& n) { return n.cost == SM_COST_CENSUS ? 1 : 2; }  // path values: u8 census, else u16

// Output slots: 0 E, 1 W (horizontal family), 2 SE, 3 S, 4 SW (MODE_SGBM adds
// these three), 5 NE, 6 N, 7 NW (MODE_HH / 8-path adds these three).
const int kVdx[6] = {1, 0, -1, 1, 0, -1};
enum { DIRS_ALL = 0, DIRS_EW = 1, DIRS_EW_UP = 2 };
const int kVdy[6] = {1, 1, 1, -1, -1, -1};

// dynamic LDS a row kernel (k_wta, k_wide_wta, k_lr_rows: one image row's disp2 keys and
// sub-pixel values) may request: HIP's default per-workgroup limit
constexpr size_t kRowLds = 65536;
// bytes of path volumes per buffer set (MI355X: 288 GB of HBM).  Middlebury (2880 x 1988,
// D = 256) needs 13.4 GB per pair on the sweep engine (the guarded fallback's 8 direction
// volumes + the partial): 32 GB lets two pairs share a launch group, which the D = 256 wide
// sweeps run in one launch
constexpr size_t kSetBudget = size_t(32) << 30;
constexpr int kMaxGroup = 16;
// smallest launch group the fused sweeps run by default: their time per launch is nearly
// flat until the strips fill the CUs, so few pairs run on the per-direction engine (KITTI
// D = 128 per pair, sweeps vs per-direction: census8 6 pairs 285 vs 259 us, 8 pairs 217 vs
// 249; sgbm5 3 pairs 440 vs 395, 4 pairs 348 vs 368; sgbm8 3 pairs 540 vs 537)
bool sweep_fit_variant(sm_ctx* ctx, const Norm& n, int mode, int variant, struct SweepFit& f);
int sweep_min_pairs(sm_ctx* ctx, const Norm& n);
// u8 cost volumes of a per-direction launch group kept below this (MI355X Infinity Cache:
// 256 MiB), at no fewer than kMallMinPairs pairs per group
constexpr size_t kMallBudget = size_t(224) << 20;
constexpr int kMallMinPairs = 3;

struct Src {  // where a launch group's pairs come from (device pointers)
    const uint8_t* L = nullptr;  // census / SGBM: images, pair i at L + i*pair_stride
    const uint8_t* R = nullptr;
    size_t pair_stride = 0;
    const float* vol = nullptr;  // external cost: vol + i*vol_pair, [D][H][W] float32
    size_t vol_pair = 0;
    float offset = 0.f, scale = 1.f;
    Src advance(int i) const
    {
        Src s = *this;
        if (L) s.L += (size_t)i * pair_stride;
        if (R) s.R += (size_t)i * pair_stride;
        if (vol) s.vol += (size_t)i * vol_pair;
        return s;
    }
};

int hybrid_slots(const Norm& n);  // per-direction volumes kept by the hybrid engine

struct Geo {  // per-group geometry shared by the launches
    int H, W, stride, G;
    size_t vol, slot_bytes, L_pair, census_pair, cost_pair;
    bool sweep;   // fused-sweep engine (sm_sweep.hpp) instead of per-direction volumes
    bool lines;   // ... with the E/W lines inside the down sweep (MODE 3 + patch pass) instead of k_ew volumes
    bool hybrid;  // 8 paths: down sweep (u16 partial) beside a per-direction launch of E, W, NE, N, NW
};

bool row_mode(const sm_ctx* ctx, const Norm& n)
{
    return SM_ABLATIONS && (ctx->dbg_flags & DBG_ROW) && n.D % 64 == 0 && n.D == n.Dv;
}
bool overlap(const sm_ctx* ctx) { return (ctx->dbg_flags & DBG_OVERLAP) != 0; }
// census mode: the path kernels read a precomputed u8 Hamming cost volume
// (k_census_cost8) instead of computing popcounts per direction; ablation
// flag 1024 restores census-on-the-fly (flag 2048: only in the horizontal family)
bool use_cost8(const sm_ctx* ctx, const Norm& n)
{
    return n.cost == SM_COST_CENSUS && !(ctx->dbg_flags & DBG_NO_C8) && n.D <= 256;
}
hipStream_t stream_b(const sm_ctx* ctx)
{
    return ctx->wta_override ? ctx->wta_override : overlap(ctx) ? ctx->side : ctx->stream;
}

// ---- stream A: path aggregation -------------------------------------------
template <int DPLV, bool CENSUS, int VL, bool H16 = false>
int launch_paths_t(sm_ctx* ctx, const Norm& n, const Geo& g, BufSet& bs, int dirset)
{
    using LT = typename std::conditional<CENSUS, uint8_t, uint16_t>::type;
    constexpr int D = 16 * DPLV;
    constexpr bool WIDE = D % 64 == 0 && !H16;
    constexpr int LANESH = WIDE ? 64 : 16;
    constexpr int DPLH = D / LANESH;
    smk::PathsArgs pa{};
    pa.cl = (const uint64_t*)bs.census[0].p;
    pa.cr = (const uint64_t*)bs.census[1].p;
    pa.census_pair = g.census_pair;
    pa.cost = (const uint16_t*)bs.cost.p;
    pa.cost_pair = g.cost_pair;
    pa.cost8 = nullptr;
    if (use_cost8(ctx, n)) {
        pa.cost8 = (const uint8_t*)bs.cost.p;
        pa.cost_pair = g.vol;
    }
    pa.L = (uint8_t*)bs.L.p;
    pa.slot_bytes = g.slot_bytes;
    pa.L_pair_bytes = g.L_pair;
    pa.H = g.H;
    pa.W = g.W;
    pa.width1 = n.width1;
    pa.D = n.D;
    pa.minD = n.minD;
    pa.minX1 = n.minX1;
    pa.P1 = n.P1;
    pa.P2 = n.P2;
    pa.dbg = ctx->dbg_flags;
    const int lines_per_wg = 4 * (64 / LANESH);
    pa.hblocks = row_mode(ctx, n) ? 0 : (g.H + lines_per_wg - 1) / lines_per_wg;
    // DIRS_ALL: every direction; DIRS_EW: E and W only (sweep engine); DIRS_EW_UP:
    // E, W and the up family NE, N, NW (hybrid engine, slots 2..4)
    pa.nv = dirset == DIRS_ALL ? n.ndirs - 2 : dirset == DIRS_EW ? 0 : 3;
    const int k0 = dirset == DIRS_EW_UP ? 3 : 0;
    int blocks = 0;
    constexpr int LPWV = 64 / VL;
    for (int k = 0; k < pa.nv; k++) {
        const int dx = kVdx[k0 + k];
        pa.v_dx[k] = dx;
        pa.v_dy[k] = kVdy[k0 + k];
        pa.v_slot[k] = 2 + k;
        pa.v_line_lo[k] = dx > 0 ? -(g.H - 1) : 0;
        pa.v_nlines[k] = dx == 0 ? n.width1 : n.width1 + g.H - 1;
        pa.v_blk_start[k] = blocks;
        // waves come in groups of 8 covering 8*LPW lines (lines w + 8*kl)
        blocks += ((pa.v_nlines[k] + 8 * LPWV - 1) / (8 * LPWV)) * 2;
    }
    for (int k = pa.nv; k <= 6; k++) pa.v_blk_start[k] = blocks;
    dim3 grid(2 * pa.hblocks + blocks, g.G);
    if (ctx->fb_guard) {  // guarded fallback: a small grid that walks every block if the sweep gave up
        pa.guard = ctx->fb_guard;
        pa.nblocks = (int)grid.x;
        pa.npairs = g.G;
        grid = dim3(std::min<unsigned>(grid.x * g.G, 128u), 1);
    }
    StageTimer t(ctx, ctx->stream,
                 ctx->fb_guard ? SM_STAGE_FALLBACK : dirset == DIRS_EW ? SM_STAGE_HORIZONTAL : SM_STAGE_PATHS, g.G);
    if (ctx->fb_guard)
        hipLaunchKernelGGL((smk::k_sgm_paths<VL, DPLV * 16 / VL, LANESH, DPLH, CENSUS, LT, true>), grid, dim3(256), 0,
                           ctx->stream, pa);
    else
        hipLaunchKernelGGL((smk::k_sgm_paths<VL, DPLV * 16 / VL, LANESH, DPLH, CENSUS, LT>), grid, dim3(256), 0,
                           ctx->stream, pa);
    HIP_TRY(ctx, hipGetLastError());
    return SM_OK;
}

// ---- stream B: WTA (or the fused horizontal + WTA row kernel) ----------------
#ifndef WTA_NT
#define WTA_NT 1024  // threads per k_wta workgroup (one image row each)
#endif
template <int DPLV, bool CENSUS>
int launch_wta_t(sm_ctx* ctx, const Norm& n, const Geo& g, BufSet& bs)
{
    using LT = typename std::conditional<CENSUS, uint8_t, uint16_t>::type;
    StageTimer t(ctx, stream_b(ctx), ctx->fb_guard ? SM_STAGE_FALLBACK : SM_STAGE_WTA, g.G);
#if SM_ABLATIONS
    constexpr int D = 16 * DPLV;
    if constexpr (D % 64 == 0) {
        if (row_mode(ctx, n) && !ctx->fb_guard) {
            if (ctx->wta_dst) return fail(ctx, SM_E_UNSUPPORTED, "the row-WTA ablation has no WTA-index output");
            smk::RowArgs ra{};
            ra.cl = (const uint64_t*)bs.census[0].p;
            ra.cr = (const uint64_t*)bs.census[1].p;
            ra.census_pair = g.census_pair;
            ra.cost = (const uint16_t*)bs.cost.p;
            ra.cost_pair = g.cost_pair;
            ra.L = (uint8_t*)bs.L.p;
            ra.slot_bytes = g.slot_bytes;
            ra.L_pair_bytes = g.L_pair;
            ra.H = g.H;
            ra.W = g.W;
            ra.width1 = n.width1;
            ra.D = n.D;
            ra.minD = n.minD;
            ra.minX1 = n.minX1;
            ra.P1 = n.P1;
            ra.P2 = n.P2;
            ra.uniq = n.uniq;
            ra.disp12 = n.disp12;
            ra.store_w = (ctx->dbg_flags & DBG_STORE_W) ? 1 : 0;
            ra.disp = (int16_t*)bs.raw.p;
            const size_t smem = (1024 + (size_t)g.W * 6 + 15) & ~size_t(15);
            if (n.ndirs == 8)
                hipLaunchKernelGGL((smk::k_row_wta<D / 64, 8, CENSUS, LT>), dim3(g.H, g.G), dim3(64), smem, stream_b(ctx), ra);
            else
                hipLaunchKernelGGL((smk::k_row_wta<D / 64, 5, CENSUS, LT>), dim3(g.H, g.G), dim3(64), smem, stream_b(ctx), ra);
            HIP_TRY(ctx, hipGetLastError());
            return SM_OK;
        }
    }
#endif
    smk::WtaArgs wa{};
    wa.L = (const uint8_t*)bs.L.p;
    wa.slot_bytes = g.slot_bytes;
    wa.L_pair_bytes = g.L_pair;
    // in-sweep E/W lines (5 paths): S = the patched partial alone; the guarded fallback reads
    // every direction's volume
    const bool part_only = g.lines && !ctx->fb_guard;
    wa.nslots = part_only ? 0 : g.hybrid ? hybrid_slots(n) : n.ndirs;
    wa.part = (g.hybrid || part_only) ? (const uint16_t*)bs.part.p : nullptr;  // hybrid: S + SE + SW partial
    wa.part_pair = g.vol;
    wa.H = g.H;
    wa.W = g.W;
    wa.width1 = n.width1;
    wa.D = n.D;
    wa.Dv = n.Dv;
    wa.minD = n.minD;
    wa.minX1 = n.minX1;
    wa.uniq = n.uniq;
    wa.disp12 = n.disp12;
    wa.disp = (int16_t*)bs.raw.p;
    wa.wta = ctx->wta_dst;
    wa.lane8 = n.ndirs == 5;
    wa.skip = ctx->fb_guard ? nullptr : ctx->wta_skip;
    dim3 grid(g.H, g.G);
    const size_t smem = (size_t)g.W * (ctx->wta_dst ? 10 : 8) + 16;
    if (smem > kRowLds)
        return fail(ctx, SM_E_UNSUPPORTED, "width %d: the WTA row kernel's %zu B of LDS exceed %zu%s", g.W, smem,
                    kRowLds, ctx->wta_dst ? " (with the WTA index output)" : "");
    if (ctx->fb_guard) {
        wa.guard = ctx->fb_guard;
        wa.fallbacks = (uint32_t*)ctx->sweep_err.p + ERR_FALLBACKS;
        wa.npairs = g.G;
        grid = dim3(std::min(g.H * g.G, 64), 1);
    }
    if (ctx->fb_guard)
        hipLaunchKernelGGL((smk::k_wta<DPLV, LT, 1024, true>), grid, dim3(1024), smem, stream_b(ctx), wa);
    else if (wa.nslots == 0 && wa.part)
        hipLaunchKernelGGL((smk::k_wta<DPLV, LT, WTA_NT, false, DPLV % 2 == 0>), grid, dim3(WTA_NT), smem, stream_b(ctx),
                           wa);
    else
        hipLaunchKernelGGL((smk::k_wta<DPLV, LT, WTA_NT>), grid, dim3(WTA_NT), smem, stream_b(ctx), wa);
    HIP_TRY(ctx, hipGetLastError());
    return SM_OK;
}

template <int DPLV, bool CENSUS>
int launch_paths_dpl(sm_ctx* ctx, const Norm& n, const Geo& g, BufSet& bs, int dirset)
{
    // horizontal lines: 16 lanes (4 rows per wave); 64-lane lines (one row per
    // wave, the round-1 layout for D % 64 == 0) with the ablation flag
    if constexpr ((16 * DPLV) % 64 == 0) {
        if (ctx->dbg_flags & DBG_H64) {
            if (DPLV == 8 && !(ctx->dbg_flags & DBG_VL16))
                return launch_paths_t<DPLV, CENSUS, 8>(ctx, n, g, bs, dirset);
            return launch_paths_t<DPLV, CENSUS, 16>(ctx, n, g, bs, dirset);
        }
    }
    // 8-lane vertical lines at D = 128 (16-lane with the ablation flag)
    if constexpr (DPLV == 8) {
        if (!(ctx->dbg_flags & DBG_VL16)) return launch_paths_t<DPLV, CENSUS, 8, true>(ctx, n, g, bs, dirset);
    }
    return launch_paths_t<DPLV, CENSUS, 16, true>(ctx, n, g, bs, dirset);
}

enum { DISPATCH_PATHS = 0, DISPATCH_WTA = 1, DISPATCH_HORIZONTAL = 2, DISPATCH_HYBRID = 3 };

int dispatch(sm_ctx* ctx, const Norm& n, const Geo& g, BufSet& bs, int what)
{
    const bool census = n.cost == SM_COST_CENSUS;
    const int h = what == DISPATCH_HORIZONTAL ? DIRS_EW : what == DISPATCH_HYBRID ? DIRS_EW_UP : DIRS_ALL;
    switch (n.dpl) {
#define CASE(k)                                                                                               \
    case k:                                                                                                   \
        if (what == DISPATCH_WTA)                                                                             \
            return census ? launch_wta_t<k, true>(ctx, n, g, bs) : launch_wta_t<k, false>(ctx, n, g, bs);     \
        return census ? launch_paths_dpl<k, true>(ctx, n, g, bs, h) : launch_paths_dpl<k, false>(ctx, n, g, bs, h);
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
        CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
    default: return fail(ctx, SM_E_UNSUPPORTED, "numDisparities %d not built", n.D);
    }
}

// ---- fused-sweep engine (sm_sweep.hpp) -----------------------------------------
int ensure_event(sm_ctx* ctx, hipEvent_t& e);
bool use_sweep(const sm_ctx* ctx, const Norm& n, int H);

// Hybrid engine: the down sweep (S + SE + SW -> one u16 partial, latency-bound) runs
// on the side stream beside ONE per-direction launch of the other directions (8
// paths: E, W, NE, N, NW; 5 paths: E, W); k_wta then sums those volumes + the
// partial (8 paths: 21 instead of 25 B/cell)
int hybrid_slots(const Norm& n) { return n.ndirs == 8 ? 5 : 2; }

bool use_hybrid(const sm_ctx* ctx, const Norm& n, int H)
{
    if (!SM_ABLATIONS || (n.ndirs != 8 && n.ndirs != 5) || !(ctx->dbg_flags & DBG_HYBRID) ||
        (ctx->dbg_flags & (DBG_LEGACY | DBG_SWEEP8)))
        return false;
    sm_ctx tmp = *ctx;
    tmp.dbg_flags = (ctx->dbg_flags & ~DBG_HYBRID) | DBG_SWEEP8;  // same preconditions as the sweeps
    return use_sweep(&tmp, n, H);
}

// preconditions of the fused sweeps (run_pairs also requires sweep_min_pairs pairs per
// launch group unless flag 16384 forces them)
bool use_sweep(const sm_ctx* ctx, const Norm& n, int H)
{
    if (ctx->dbg_flags & (DBG_LEGACY | DBG_ROW)) return false;
    // every configuration whose preconditions hold: with wide strips (sm_sweep.hpp SweepGeo)
    // census 8 paths run 217 vs 249 us per KITTI pair against the per-direction engine, u16
    // costs at 8 paths (OpenCV MODE_HH, mc-cnn volumes) 1.5-1.7x faster
    if (n.cost == SM_COST_CENSUS && !use_cost8(ctx, n)) return false;  // the sweeps read the u8 cost volume
    // packed u16 recurrence (sm_sweep.hpp): every L must stay <= 16383 (SGBM costs: normalize's domain check)
    const int cmax = n.cost == SM_COST_CENSUS ? 64 : n.cost == SM_COST_VOLUME ? smk::VOL_CMAX : 0;
    if (cmax + n.P2 > 16383) return false;
    if (H > 65535 || n.width1 <= 0) return false;                      // row index lives in 16 tag bits
    const size_t W = (size_t)(n.maxX1 - std::min(n.minD, 0));
    if (W * 6 + 16 > kRowLds) return false;                              // k_lr_rows keeps a row in LDS
    return (uint64_t)H * n.width1 * n.D * 2 <= smk::kMaxRecords;
}

struct SweepJob {
    const uint8_t* cost;
    size_t cost_pair;
    const uint8_t* ew;
    size_t ew_pair, ew_slot;
    uint16_t* part;
    size_t part_pair;
    uint32_t* key2;
    uint32_t* pre;  // sub-pixel inputs (SweepArgs::nb)
    uint32_t* err;  // word a strip sets when it gives up waiting for a neighbour
    int G;
    uint8_t* st = nullptr;  // MODE 3: boundary states of the E/W strip segments
    size_t st_pair = 0;     // bytes
    int ewarm = 0;          // MODE 3: warmup columns of the E/W segments
    int ewguess = 0;        // MODE 3: 1 = a deliberately wrong start state (tests)
    // MODE 3 row bands (nband > 1: the wide instance)
    int nband = 1, band_h = 0, vwarm = 0, vguess = 0;
    uint8_t* vst = nullptr;
    size_t vst_pair = 0;
};

// CUs the stream may run on: its CU mask (sm_set_cu_mask), the whole device when unmasked
int stream_cus(hipStream_t st, int ncu)
{
    uint32_t mask[32] = {0};
    const uint32_t words = (uint32_t)std::min(32, (ncu + 31) / 32);
    if (hipExtStreamGetCUMask(st, words, mask) != hipSuccess) return ncu;
    int c = 0;
    for (uint32_t i = 0; i < words; i++) c += __builtin_popcount(mask[i]);
    return c > 0 ? std::min(c, ncu) : ncu;
}

int ensure_sweep_err(sm_ctx* ctx)
{
    if (ctx->sweep_err.p) return SM_OK;
    int rc = ensure(ctx, ctx->sweep_err, SWEEP_STATS ? (size_t(8) << 20) : 256);
    if (rc != SM_OK) return rc;
    HIP_TRY(ctx, hipMemsetAsync(ctx->sweep_err.p, 0, SWEEP_STATS ? (size_t(8) << 20) : 256, ctx->stream));
    return SM_OK;
}

// which fused-sweep kernel: k_sweep with wide strips where built (0, sm_sweep_host.hpp),
// flag 1 << 19 the narrow strips (1); ablation flags select k_sweep2 (column-per-lane layout,
// sm_sweep2.hpp; u8 costs at D = 128, k_sweep elsewhere): 128 -> 6 compute waves of 8
// columns, 1 << 27 -> 3 waves of 16 columns (slower at 8 pairs)
int sweep_variant(const sm_ctx* ctx)
{
    if (SM_ABLATIONS && (ctx->dbg_flags & DBG_SWEEP_V2)) return 6;
    if (SM_ABLATIONS && (ctx->dbg_flags & DBG_SWEEP2_NW)) return 3;
    return (ctx->dbg_flags & DBG_NARROW_SWEEPS) ? 1 : 0;
}

// strips per pair (nwg) and co-resident workgroups the context's stream can hold (cap) for one
// sweep mode and kernel variant; false when (D, cost type) is not built or the strips of a
// pair cannot all be co-resident
struct SweepFit {
    smk::SweepInfo si{};
    int nwg = 0, cap = 0, ncu = 0;
};
bool sweep_fit_variant(sm_ctx* ctx, const Norm& n, int mode, int variant, SweepFit& f)
{
    if (smk::sweep_info(n.D, (int)elem_bytes(n), mode, variant, ctx->device, &f.si) != hipSuccess) return false;
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess) return false;
    f.ncu = stream_cus(ctx->stream, std::max(ncu, 1));  // a CU-masked stream only reaches its CUs
    // the API's answer can be one block per CU high at >= 82 SGPRs (MI355X guide);
    // for 512-thread blocks SGPRs allow >= 3 per CU, so a margin is kept only above 2
    const int per_cu = f.si.blocks_per_cu >= 3 ? f.si.blocks_per_cu - 1 : std::max(f.si.blocks_per_cu, 1);
    f.cap = per_cu * f.ncu;
    f.nwg = (n.width1 + f.si.cw - 1) / f.si.cw;
    return f.nwg <= f.cap;
}

// census: enough pairs for the wide strips to occupy ~200 of the 256 CUs (KITTI: 31 strips
// per pair -> 7; Middlebury's 2624 columns: 101 strips of the D = 256 instance -> 2), at most
// 7; other costs: 3 (measured, see above)
int sweep_min_pairs(sm_ctx* ctx, const Norm& n)
{
    if (n.cost != SM_COST_CENSUS) return 3;
    SweepFit f;
    if (!sweep_fit_variant(ctx, n, 2, 0, f) || f.nwg <= 0) return 7;
    return std::max(2, std::min(7, (200 + f.nwg - 1) / f.nwg));
}

// modelled time of G pairs on one variant: the sweeps are bound by the instruction issue of
// the CU that holds the most strips, so (launches) x (strips per CU) x (compute waves per
// strip).  Wide strips recompute fewer halo columns per own column, narrow strips spread a
// few pairs over more CUs (KITTI D = 128 WTA sweep, 8 pairs: wide 95 vs narrow 108 us per
// pair; 3 pairs: 31 wide strips per pair leave 163 of 256 CUs idle)
double sweep_model(const SweepFit& f, int G)
{
    const int per_launch = std::max(1, std::min(G, f.cap / std::max(f.nwg, 1)));
    const int launches = (G + per_launch - 1) / per_launch;
    const int per_cu = (per_launch * f.nwg + f.ncu - 1) / std::max(f.ncu, 1);
    // a wave's work per row scales with its disparities per lane (the D = 256 wide instance
    // runs 32-lane lines: half the per-wave work of the 16-lane narrow one)
    return (double)launches * per_cu * (f.si.threads / 64 - 1) * std::max(f.si.dpl, 1);
}

// the kernel variant for one pass over G pairs (G = 0: any that fits, wide strips first).
// Candidates: wide strips (where built), narrow strips (kNarrowNcw compute waves) and the
// latency strips (kLatNcw: more, narrower strips for launches of one or two pairs); the
// smallest modelled issue time wins.  SM_TUNE_SWEEP_NCW forces the instance with that many
// compute waves.
bool sweep_capacity(sm_ctx* ctx, const Norm& n, int mode, int G, SweepFit& f)
{
    if (ctx->tune_sweep_ncw && sweep_variant(ctx) <= 1) {
        for (int v : {0, 1, 2}) {
            SweepFit t;
            if (sweep_fit_variant(ctx, n, mode, v, t) && t.si.ncw == ctx->tune_sweep_ncw) {
                f = t;
                return true;
            }
        }
        return false;
    }
    const int variant = sweep_variant(ctx);
    if (!sweep_fit_variant(ctx, n, mode, variant, f)) {
        // wide strips that do not fit: the narrow ones may
        if (!(variant == 0 && f.si.impl == 1 && sweep_fit_variant(ctx, n, mode, 1, f))) return false;
    } else if (variant == 0 && f.si.impl == 1 && G > 0 && !(ctx->dbg_flags & DBG_WIDE_SWEEPS)) {
        SweepFit nf;
        if (sweep_fit_variant(ctx, n, mode, 1, nf) && sweep_model(nf, G) < sweep_model(f, G)) f = nf;
    }
    if (variant == 0 && G > 0 && !(ctx->dbg_flags & DBG_WIDE_SWEEPS)) {
        SweepFit lf;
        if (sweep_fit_variant(ctx, n, mode, 2, lf) && sweep_model(lf, G) < sweep_model(f, G)) f = lf;
    }
    return true;
}

// every sweep pass of the configuration can make all strips of a pair co-resident (wide
// images on few CUs cannot: those run on the per-direction engine)
bool sweeps_fit(sm_ctx* ctx, const Norm& n, bool hybrid, bool lines = false)
{
    // passes: hybrid = the down sweep; 8 paths = down + up/WTA; 5 paths = down/WTA; with the
    // in-sweep E/W lines: the down sweep with lines (+ the up/WTA sweep over its partial)
    const int m8[2] = {0, 2}, m5[1] = {1}, mh[1] = {0}, l8[2] = {3, 4}, l5[1] = {3};
    const int* modes = hybrid ? mh : lines ? (n.ndirs == 8 ? l8 : l5) : n.ndirs == 8 ? m8 : m5;
    const int count = !hybrid && n.ndirs == 8 ? 2 : 1;
    for (int k = 0; k < count; k++) {
        SweepFit f;
        if (!sweep_capacity(ctx, n, modes[k], 0, f)) return false;
        if (lines && modes[k] == 3 && f.nwg > smk::patch_max_strips(n.D)) return false;  // the patch pass's masks
        // lines in narrow strips (no wide MODE 3 instance: D = 256 u8) pay the warmup on 20
        // columns and lost to the E/W volumes (Middlebury D = 256, 4 pairs: 167 vs 225 pairs/s)
        if (lines && modes[k] == 3 && f.si.ncw < 11) return false;
    }
    return true;
}

// one sweep pass (MODE 0/1/2, sm_sweep.hpp) over the job's G pairs, in launches
// whose workgroups are all co-resident (strips of a pair wait on each other)
int sweep_pass(sm_ctx* ctx, const Norm& n, const Geo& g, const SweepJob& j, int mode)
{
    SweepFit f;
    const bool banded = j.nband > 1;
    if (banded ? !(sweep_fit_variant(ctx, n, mode, 0, f) && f.si.impl == 1) : !sweep_capacity(ctx, n, mode, j.G, f)) {
        if (f.nwg > f.cap)
            return fail(ctx, SM_E_UNSUPPORTED, "sweep: %d strips exceed %d resident workgroups", f.nwg, f.cap);
        return fail(ctx, SM_E_UNSUPPORTED, "sweep: numDisparities %d not built", n.D);
    }
    const smk::SweepInfo& si = f.si;
    const int nwg = f.nwg, cap = f.cap;
    const int nb = banded ? j.nband : 1;
    // halo blocks per strip record: every band's rows (own + warmup) fit
    const int nblk = banded ? (j.band_h + j.vwarm + si.hb - 1) / si.hb : (g.H + si.hb - 1) / si.hb;
    // ablation / test flag 8192: one pair per sweep launch (exercises the chunked launches)
    const int per_launch = (ctx->dbg_flags & DBG_SWEEP1) ? 1 : std::max(1, std::min(j.G, cap / (nwg * nb)));
    const size_t hop_pair = (size_t)nwg * nb * 2 * nblk * si.ngr;
    const size_t hop_bytes = hop_pair * 8 * per_launch;
    if (hop_pair * 8 > smk::kMaxRecords) return fail(ctx, SM_E_UNSUPPORTED, "sweep: boundary buffer too large");
    int rc;
    if (ctx->hop.n < hop_bytes || !ctx->hop.p) {
        if ((rc = ensure(ctx, ctx->hop, hop_bytes)) != SM_OK) return rc;
        HIP_TRY(ctx, hipMemsetAsync(ctx->hop.p, 0, ctx->hop.n, ctx->stream));
        ctx->hop_epoch = 0;
    }
    if ((rc = ensure_sweep_err(ctx)) != SM_OK) return rc;
    for (int p0 = 0; p0 < j.G; p0 += per_launch) {
        const int np = std::min(per_launch, j.G - p0);
        if (++ctx->hop_epoch > 0xFFFFu) {  // tags repeat: clear the granules once per 65535 launches
            HIP_TRY(ctx, hipMemsetAsync(ctx->hop.p, 0, ctx->hop.n, ctx->stream));
            ctx->hop_epoch = 1;
        }
        smk::SweepArgs a{};
        a.cost = j.cost + (size_t)p0 * j.cost_pair;
        a.cost_pair = j.cost_pair;
        a.ew = j.ew ? j.ew + (size_t)p0 * j.ew_pair : nullptr;
        a.ew_pair = j.ew_pair;
        a.ew_slot = j.ew_slot;
        a.part = j.part ? (uint16_t*)((uint8_t*)j.part + (size_t)p0 * j.part_pair) : nullptr;
        a.part_pair = j.part_pair;
        a.hop = (unsigned long long*)ctx->hop.p;
        a.hop_pair = hop_pair;
        a.st = j.st ? j.st + (size_t)p0 * j.st_pair : nullptr;
        a.st_pair = j.st_pair;
        a.ewarm = j.ewarm;
        a.ewguess = j.ewguess;
        a.nband = nb;
        a.band_h = j.band_h;
        a.vwarm = j.vwarm;
        a.vguess = j.vguess;
        a.hop_nblk = nblk;
        a.vst = j.vst ? j.vst + (size_t)p0 * j.vst_pair : nullptr;
        a.vst_pair = j.vst_pair;
        if (ctx->tune_sweep_xcd > 0) {  // XCD-aware placement (SweepArgs::xcd_per)
            a.xcd_total = np * nwg * nb;
            a.xcd_per = (a.xcd_total + 7) / 8;
        }
        a.rec = j.key2 ? j.key2 + (size_t)p0 * g.H * g.W : nullptr;
        a.nb = j.pre ? j.pre + (size_t)p0 * g.H * g.W : nullptr;
        a.err = j.err;
        a.H = g.H;
        a.W = g.W;
        a.W1 = n.width1;
        a.D = n.D;
        a.Dv = n.Dv;
        a.minD = n.minD;
        a.minX1 = n.minX1;
        a.P1 = n.P1;
        a.P2 = n.P2;
        a.uniq = n.uniq;
        a.inv_ku = n.uniq < 100 ? 1.0f / (float)(100 - n.uniq) : 0.f;
        a.nwg = nwg;
        a.epoch = ctx->hop_epoch;
#if SWEEP_STATS
        a.stats = (unsigned long long*)((char*)ctx->sweep_err.p + 1024);
#endif
        a.dbg = (ctx->dbg_flags >> 24) & 7;  // timing ablations (results wrong): 1 no polls
        HIP_TRY(ctx, smk::sweep_launch(n.D, (int)elem_bytes(n), mode, si.impl, a, np, ctx->stream));
    }
    return SM_OK;
}

// launches of a scope go to another stream (restored on every exit path)
struct StreamSwap {
    sm_ctx* c;
    hipStream_t old;
    StreamSwap(sm_ctx* c_, hipStream_t s) : c(c_), old(c_->stream) { c->stream = s; }
    ~StreamSwap() { c->stream = old; }
};

// lanes per line of the sweep engine's E/W kernel (-1: the per-direction engine's row lines,
// also forced by flag 256).  u8 costs (8 KITTI pairs, beside the down sweep): the packed
// 8-lane lines, 114 vs 122 us per pair for the row lines (4 and 16 lanes no faster)
int ew_lanes(const sm_ctx* ctx, const Norm& n)
{
    if (ctx->tune_ew_lanes) return ctx->tune_ew_lanes;
    if (ctx->dbg_flags & DBG_OLD_EW) return -1;  // flag 256: the row lines
    // round 4 (tools/lr_probe.py, bench.py --tune): more lanes per line.  u16 costs beat the
    // row lines at every pair count measured: KITTI D = 128, 32 lanes, 1 / 2 / 8 pairs 168 ->
    // 120 / 262 -> 205 / 708 -> 655 us per launch; D = 160, 16 lanes, 1 / 2 / 4 pairs 208 ->
    // 204 / 422 -> 408 / 534 -> 520.  u8 costs beside the census down sweep (8 KITTI pairs, one
    // box): 8 lanes 5978, 16 lanes 6126, 32 lanes 6163 pairs/s: the lines themselves take a
    // little longer (74 vs 67 us per pair) but stretch the down sweep less (72 vs 78)
    if (n.D % 64 == 0) return 32;
    if (n.D % 32 == 0) return 16;
    return elem_bytes(n) == 1 ? 0 : -1;
}

// E and W path volumes of the sweep engine (slots 0, 1 of bs.L): the packed
// horizontal-line kernel (sm_ew.hpp), or the per-direction engine's row lines
int launch_ew(sm_ctx* ctx, const Norm& n, const Geo& g, BufSet& bs)
{
    const size_t et = elem_bytes(n);
    const int vl = ew_lanes(ctx, n);
    if (vl < 0) return dispatch(ctx, n, g, bs, DISPATCH_HORIZONTAL);
    smk::EwArgs a{};
    a.cost = (const uint8_t*)bs.cost.p;
    a.cost_pair = g.vol * et;
    a.out = (uint8_t*)bs.L.p;
    a.out_pair = g.L_pair;
    a.out_slot = g.slot_bytes;
    a.H = g.H;
    a.W1 = n.width1;
    a.P1 = n.P1;
    a.P2 = n.P2;
    a.wpb = ctx->tune_ew_waves;
    a.prio = ctx->tune_ew_prio;
    StageTimer t(ctx, ctx->stream, SM_STAGE_HORIZONTAL, g.G);
    const hipError_t e = smk::ew_launch(n.D, (int)et, vl, a, g.G, ctx->stream);
    if (e == hipErrorInvalidValue) return fail(ctx, SM_E_UNSUPPORTED, "E/W lines: numDisparities %d not built", n.D);
    HIP_TRY(ctx, e);
    return SM_OK;
}

// E/W volumes -> [down sweep partial] -> WTA sweep -> LR check into bs.raw.  With
// wta_stream != ctx->stream (5 paths, two-stream overlap) the WTA sweep and the
// LR pass run there, beside the next launch group's cost + E/W on ctx->stream.
int run_sweep(sm_ctx* ctx, const Norm& n, const Geo& g, BufSet& bs, hipStream_t wta_stream, uint32_t* err)
{
    const int G = g.G;
    int rc;
    const size_t et = elem_bytes(n);
    SweepJob j{};
    j.cost = (const uint8_t*)bs.cost.p;
    j.cost_pair = g.vol * et;
    j.ew = (const uint8_t*)bs.L.p;
    j.ew_pair = g.L_pair;
    j.ew_slot = g.slot_bytes;
    j.G = G;
    if ((rc = ensure(ctx, bs.key2, (size_t)G * g.H * g.W * 4)) != SM_OK) return rc;
    if ((rc = ensure(ctx, bs.pre, (size_t)G * g.H * g.W * 4)) != SM_OK) return rc;
    j.key2 = (uint32_t*)bs.key2.p;
    j.pre = (uint32_t*)bs.pre.p;
    j.err = err;
    {
        StageTimer t(ctx, ctx->stream, SM_STAGE_PATHS, G);
        if (n.ndirs == 8) {
            // 8 paths: the E/W kernel (latency-bound serial rows) runs on the side
            // stream beside the down sweep (latency-bound serial columns); the
            // WTA sweep needs both.  The sweep is enqueued first, so that its strips
            // (which wait on each other) are dispatched before the E/W workgroups
            // fill the CUs; E/W waits for the cost volume only.
            if ((rc = ensure_event(ctx, ctx->ev_fork)) != SM_OK) return rc;
            if ((rc = ensure_event(ctx, ctx->ev_join)) != SM_OK) return rc;
            HIP_TRY(ctx, hipEventRecord(ctx->ev_fork, ctx->stream));
            if ((rc = ensure(ctx, bs.part, (size_t)G * g.vol * 2)) != SM_OK) return rc;
            j.part = (uint16_t*)bs.part.p;
            j.part_pair = g.vol * 2;
            {
                StageTimer ts(ctx, ctx->stream, SM_STAGE_SWEEP, G);
                if ((rc = sweep_pass(ctx, n, g, j, 0)) != SM_OK) return rc;
            }
            HIP_TRY(ctx, hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
            const hipStream_t main = ctx->stream;
            ctx->stream = ctx->side;
            rc = launch_ew(ctx, n, g, bs);
            ctx->stream = main;
            if (rc != SM_OK) return rc;
            HIP_TRY(ctx, hipEventRecord(ctx->ev_join, ctx->side));
            HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
        } else if ((rc = launch_ew(ctx, n, g, bs)) != SM_OK) {
            return rc;
        }
    }
    if (wta_stream != ctx->stream) {
        HIP_TRY(ctx, hipEventRecord(bs.paths_done, ctx->stream));
        HIP_TRY(ctx, hipStreamWaitEvent(wta_stream, bs.paths_done, 0));
    }
    StreamSwap sw(ctx, wta_stream);
    StageTimer t(ctx, ctx->stream, SM_STAGE_WTA, G);
    StageTimer ts(ctx, ctx->stream, SM_STAGE_SWEEP_WTA, G);
    return sweep_pass(ctx, n, g, j, n.ndirs == 8 ? 2 : 1);
}

// after the WTA sweep (on stream ws): the LR pass into bs.raw and, unless flag 1 << 31, the
// guarded per-direction fallback of the group.  The fallback (two launches that exit at once
// while the group flag is clear) runs on a second stream beside the LR pass, which writes
// nothing when the flag is set, so neither waits for the other's launch latency; ws joins
// the second stream before the median reads bs.raw.
int sweep_finish(sm_ctx* ctx, const Norm& n, const Geo& g, BufSet& bs, hipStream_t ws, uint32_t* gflag)
{
    const bool fb = !(ctx->dbg_flags & DBG_NO_FALLBACK);
    int rc;
    if (fb && ws != ctx->stream) {
        // the WTA sweep runs on the second stream beside the next group (flag 64): a fallback
        // on ctx->stream would make that group wait for this group's WTA sweep, so it follows
        // the LR pass on ws instead (in order; the LR pass writes nothing when the flag is set)
        if (ctx->dbg_flags & DBG_FORCE_FALLBACK) HIP_TRY(ctx, hipMemsetAsync(gflag, 1, 1, ws));
        HIP_TRY(ctx, smk::lr_rows_launch((const uint32_t*)bs.key2.p, (const uint32_t*)bs.pre.p, (int16_t*)bs.raw.p,
                                         ctx->wta_dst, g.G, g.H, g.W, n.Dv, n.minD, n.minX1, n.maxX1, n.disp12,
                                         gflag, ws));
        StreamSwap sw(ctx, ws);
        ctx->wta_override = ws;
        ctx->fb_guard = gflag;
        rc = dispatch(ctx, n, g, bs, DISPATCH_PATHS);
        if (rc == SM_OK) rc = dispatch(ctx, n, g, bs, DISPATCH_WTA);
        ctx->fb_guard = nullptr;
        ctx->wta_override = nullptr;
        return rc;
    }
    hipStream_t fs = ctx->side;  // the stream the fallback runs on (ws == ctx->stream here)
    if (fb) {
        if (ctx->dbg_flags & DBG_FORCE_FALLBACK) HIP_TRY(ctx, hipMemsetAsync(gflag, 1, 1, ws));
        if ((rc = ensure_event(ctx, ctx->ev_fb_fork)) != SM_OK) return rc;
        if ((rc = ensure_event(ctx, ctx->ev_fb_join)) != SM_OK) return rc;
        HIP_TRY(ctx, hipEventRecord(ctx->ev_fb_fork, ws));
        HIP_TRY(ctx, hipStreamWaitEvent(fs, ctx->ev_fb_fork, 0));
        StreamSwap sw(ctx, fs);
        ctx->wta_override = fs;
        ctx->fb_guard = gflag;
        rc = dispatch(ctx, n, g, bs, DISPATCH_PATHS);
        if (rc == SM_OK) rc = dispatch(ctx, n, g, bs, DISPATCH_WTA);
        ctx->fb_guard = nullptr;
        ctx->wta_override = nullptr;
        if (rc != SM_OK) return rc;
        HIP_TRY(ctx, hipEventRecord(ctx->ev_fb_join, fs));
    }
    HIP_TRY(ctx, smk::lr_rows_launch((const uint32_t*)bs.key2.p, (const uint32_t*)bs.pre.p, (int16_t*)bs.raw.p,
                                     ctx->wta_dst, g.G, g.H, g.W, n.Dv, n.minD, n.minX1, n.maxX1, n.disp12,
                                     fb ? gflag : nullptr, ws));
    if (fb) HIP_TRY(ctx, hipStreamWaitEvent(ws, ctx->ev_fb_join, 0));
    return SM_OK;
}

// ---- in-sweep E/W lines: MODE 3 down sweep with line waves -> patch pass ->
// (8 paths) MODE 4 up/WTA sweep + LR pass, (5 paths) k_wta over the partial.  No E/W volumes:
// census 8 paths 7 instead of 13 B per cell, u16 5 paths 6 instead of 16.
// By default wherever the MODE 3 instance (and MODE 4 at 8 paths) fits; SM_TUNE_SWEEP_LINES -1,
// any SM_TUNE_EW_LANES value or flag 256 keep the E/W volumes (k_ew / row lines).
bool use_lines(sm_ctx* ctx, const Norm& n)
{
    if (ctx->tune_sweep_lines < 0 || ctx->tune_ew_lanes || (ctx->dbg_flags & DBG_OLD_EW)) return false;
    return sweeps_fit(ctx, n, false, true);
}

// warmup columns of the E/W strip segments: the speculative state meets the true one within
// 16 columns on ~98 % of KITTI census segments, 24 on ~97 % of u16 (settings.ini) ones
// (measured on the synthetic pairs with the numpy oracle); SM_TUNE_EW_WARMUP overrides
int ew_warmup(const sm_ctx* ctx, const Norm& n)
{
    if (ctx->tune_ew_warmup > 0) return ctx->tune_ew_warmup;
    // 16 columns for both cost types (sgbm5, 8 pairs: 6520-6535 pairs/s at 16 against 6444-6469
    // at 24, the patch pass's extra 4.5 us per pair below the sweep's 6 us saved)
    (void)n;
    return 16;
}

// largest value one path can take (normalize's domains): a 5-path sum of the banded engine must
// stay below 2^16, where the band patch's atomic corrections are exact (no saturation)
long long path_max(const Norm& n)
{
    if (n.cost == SM_COST_CENSUS) return 62 + n.P2;
    if (n.cost == SM_COST_VOLUME) return smk::VOL_CMAX + n.P2;
    const long long side = 2 * (n.bs / 2) + 1;
    return side * side * (2 * n.ftzero + (255 >> 2)) + n.P2;
}

// row bands per pair of a 5-path lines launch group of G pairs (1: none): so many that the
// strips of every band of the group are co-resident on the device's CUs (KITTI D = 160, one pair:
// 31 wide strips -> 8 bands of 47 rows), each band at least 24 rows.  SM_TUNE_BANDS forces a count.
int line_bands(const sm_ctx* ctx, const Norm& n, int H, int G)
{
    if (n.ndirs != 5 || ctx->tune_bands == 1 || 5 * path_max(n) > 65535) return 1;
    SweepFit f;
    if (!sweep_fit_variant(const_cast<sm_ctx*>(ctx), n, 3, 0, f) || f.si.impl != 1 || f.nwg <= 0) return 1;
    int nb = ctx->tune_bands >= 2 ? ctx->tune_bands : std::min(f.cap / std::max(1, G * f.nwg), H / 24);
    nb = std::min(nb, H);
    if (nb < 2) return 1;
    const int bh = (H + nb - 1) / nb;
    return (H + bh - 1) / bh;  // no empty band
}

// rows each band's vertical paths run before its own rows (speculation warmup; SM_TUNE_BAND_WARMUP)
int band_warmup(const sm_ctx* ctx, const Norm& n)
{
    if (ctx->tune_band_warmup > 0) return ctx->tune_band_warmup;
    return elem_bytes(n) == 1 ? 16 : 24;
}

int run_lines(sm_ctx* ctx, const Norm& n, const Geo& g, BufSet& bs, hipStream_t ws, uint32_t* gflag)
{
    const int G = g.G;
    const size_t et = elem_bytes(n);
    int rc;
    SweepJob j{};
    j.cost = (const uint8_t*)bs.cost.p;
    j.cost_pair = g.vol * et;
    j.G = G;
    j.err = gflag;
    if ((rc = ensure(ctx, bs.part, (size_t)G * g.vol * 2)) != SM_OK) return rc;
    j.part = (uint16_t*)bs.part.p;
    j.part_pair = g.vol * 2;
    SweepFit f;
    j.nband = line_bands(ctx, n, g.H, G);
    if (j.nband > 1 ? !sweep_fit_variant(ctx, n, 3, 0, f) : !sweep_capacity(ctx, n, 3, G, f))
        return fail(ctx, SM_E_UNSUPPORTED, "sweep lines: no instance fits");
    j.st_pair = ((size_t)g.H * f.nwg * 4 * n.D * et + 255) & ~size_t(255);
    if ((rc = ensure(ctx, bs.st, j.st_pair * G)) != SM_OK) return rc;
    j.st = (uint8_t*)bs.st.p;
    j.ewarm = ew_warmup(ctx, n);
    j.ewguess = ctx->tune_ew_guess;
    // one or two pairs (row bands): the patch passes' longest walks are the call's critical
    // path, so the u16 segments warm up longer (settings.ini D = 160, one pair: 24 -> 54 columns,
    // E/W repairs 551 -> 26 per matcher, device time per call 1114 -> 1058 us)
    if (j.nband > 1 && ctx->tune_ew_warmup <= 0 && et == 2) j.ewarm = 54;
    if (j.nband > 1) {
        j.band_h = (g.H + j.nband - 1) / j.nband;
        j.vwarm = band_warmup(ctx, n);
        j.vguess = ctx->tune_band_guess;
        j.vst_pair = ((size_t)j.nband * 6 * n.width1 * n.D * et + 255) & ~size_t(255);
        if ((rc = ensure(ctx, bs.vst, j.vst_pair * G)) != SM_OK) return rc;
        j.vst = (uint8_t*)bs.vst.p;
        ctx->band_groups++;
    }
    ctx->line_groups++;
    ctx->line_strips += (long long)f.nwg * G;
    const bool fb_side = n.ndirs == 5 && ws == ctx->stream && !(ctx->dbg_flags & DBG_NO_FALLBACK);
    {
        StageTimer t(ctx, ctx->stream, SM_STAGE_PATHS, G);
        {
            StageTimer ts(ctx, ctx->stream, SM_STAGE_SWEEP, G);
            if ((rc = sweep_pass(ctx, n, g, j, 3)) != SM_OK) return rc;
        }
        if (ctx->sweep_done_ev) {  // compute_disparity's stagger: the other matcher may start now
            HIP_TRY(ctx, hipEventRecord(ctx->sweep_done_ev, ctx->stream));
            ctx->sweep_done_hit = true;
        }
        smk::EwPatchArgs pa{};
        pa.cost = j.cost;
        pa.cost_pair = j.cost_pair;
        pa.part = j.part;
        pa.part_pair = j.part_pair * 1;
        pa.st = j.st;
        pa.st_pair = j.st_pair;
        pa.H = g.H;
        pa.W1 = n.width1;
        pa.nwg = f.nwg;
        pa.cw = f.si.cw;
        pa.P1 = n.P1;
        pa.P2 = n.P2;
        pa.guard = gflag;
        pa.fixes = reinterpret_cast<unsigned long long*>((uint32_t*)ctx->sweep_err.p + ERR_EW_REPAIRS);
        // u16 costs where no partial cell can saturate: atomic corrections, E and W side by side
        // (sm_ew.hpp ATOM; sgbm5 8 pairs: patch 17.6 -> 15.2 us per pair; census8: 6.9 -> 7.5)
        pa.atom = EW_PATCH_ATOM && et == 2 && 5 * path_max(n) < 65536 ? 1 : 0;
        auto ew_patch = [&](hipStream_t st) -> int {
            const hipError_t e = smk::ew_patch_launch(n.D, (int)et, pa, G, st);
            if (e == hipErrorInvalidValue) return fail(ctx, SM_E_UNSUPPORTED, "E/W patch: numDisparities %d not built", n.D);
            HIP_TRY(ctx, e);
            return SM_OK;
        };
        // with row bands and atomic corrections the E/W patch runs on the side stream beside the
        // band patch (both only add to the partial), ahead of the guarded fallback there
        const bool ew_side = fb_side && pa.atom && j.nband > 1;
        if (fb_side) {
            // 5 paths: the group flag is final after the sweep, so the guarded per-direction
            // fallback (two launches that exit at once unless a strip gave up) runs on the side
            // stream beside the patch passes and the WTA row kernel, which writes nothing when
            // the flag is set: the fallback's launch latency leaves the critical path
            if (ctx->dbg_flags & DBG_FORCE_FALLBACK) HIP_TRY(ctx, hipMemsetAsync(gflag, 1, 1, ctx->stream));
            if ((rc = ensure_event(ctx, ctx->ev_fb_fork)) != SM_OK) return rc;
            if ((rc = ensure_event(ctx, ctx->ev_fb_join)) != SM_OK) return rc;
            HIP_TRY(ctx, hipEventRecord(ctx->ev_fb_fork, ctx->stream));
            HIP_TRY(ctx, hipStreamWaitEvent(ctx->side, ctx->ev_fb_fork, 0));
            if (ew_side) {
                if ((rc = ensure_event(ctx, ctx->ev_ew_done)) != SM_OK) return rc;
                {
                    StageTimer th(ctx, ctx->side, SM_STAGE_HORIZONTAL, G);
                    if ((rc = ew_patch(ctx->side)) != SM_OK) return rc;
                }
                HIP_TRY(ctx, hipEventRecord(ctx->ev_ew_done, ctx->side));
            }
            StreamSwap sw(ctx, ctx->side);
            ctx->wta_override = ctx->side;
            ctx->fb_guard = gflag;
            rc = dispatch(ctx, n, g, bs, DISPATCH_PATHS);
            if (rc == SM_OK) rc = dispatch(ctx, n, g, bs, DISPATCH_WTA);
            ctx->fb_guard = nullptr;
            ctx->wta_override = nullptr;
            if (rc != SM_OK) return rc;
            HIP_TRY(ctx, hipEventRecord(ctx->ev_fb_join, ctx->side));
        }
        if (!ew_side) {
            StageTimer th(ctx, ctx->stream, SM_STAGE_HORIZONTAL, G);
            if ((rc = ew_patch(ctx->stream)) != SM_OK) return rc;
        }
        if (j.nband > 1) {  // then the vertical chains at the band boundaries (after: both touch the partial)
            smk::BandPatchArgs ba{};
            ba.cost = j.cost;
            ba.cost_pair = j.cost_pair;
            ba.part = j.part;
            ba.part_pair = j.part_pair;
            ba.vst = j.vst;
            ba.vst_pair = j.vst_pair;

            ba.H = g.H;
            ba.W1 = n.width1;
            ba.nband = j.nband;
            ba.band_h = j.band_h;
            ba.P1 = n.P1;
            ba.P2 = n.P2;
            ba.guard = gflag;
            ba.fixes = reinterpret_cast<unsigned long long*>((uint32_t*)ctx->sweep_err.p + ERR_BAND_REPAIRS);
            const hipError_t eb = smk::band_patch_launch(n.D, (int)et, ba, G, ctx->stream);
            if (eb == hipErrorInvalidValue) return fail(ctx, SM_E_UNSUPPORTED, "band patch: numDisparities %d not built", n.D);
            HIP_TRY(ctx, eb);
            // the WTA reads the partial both patches correct (the fallback's join comes after it)
            if (ew_side) HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_ew_done, 0));
        }
    }
    if (ws != ctx->stream) {
        HIP_TRY(ctx, hipEventRecord(bs.paths_done, ctx->stream));
        HIP_TRY(ctx, hipStreamWaitEvent(ws, bs.paths_done, 0));
    }
    if (n.ndirs == 8) {
        if ((rc = ensure(ctx, bs.key2, (size_t)G * g.H * g.W * 4)) != SM_OK) return rc;
        if ((rc = ensure(ctx, bs.pre, (size_t)G * g.H * g.W * 4)) != SM_OK) return rc;
        j.key2 = (uint32_t*)bs.key2.p;
        j.pre = (uint32_t*)bs.pre.p;
        {
            StreamSwap sw(ctx, ws);
            StageTimer t(ctx, ctx->stream, SM_STAGE_WTA, G);
            StageTimer ts(ctx, ctx->stream, SM_STAGE_SWEEP_WTA, G);
            if ((rc = sweep_pass(ctx, n, g, j, 4)) != SM_OK) return rc;
        }
        return sweep_finish(ctx, n, g, bs, ws, gflag);
    }
    // 5 paths: the WTA row kernel over the patched partial (k_wta: uniqueness, sub-pixel, LR)
    // into bs.raw, then the guarded per-direction fallback of the group (it exits at once
    // unless a strip gave up, and then overwrites bs.raw)
    StreamSwap sw(ctx, ws);
    ctx->wta_override = ws;
    {
        StageTimer ts(ctx, ws, SM_STAGE_SWEEP_WTA, G);
        ctx->wta_skip = fb_side ? gflag : nullptr;
        rc = dispatch(ctx, n, g, bs, DISPATCH_WTA);
        ctx->wta_skip = nullptr;
    }
    if (fb_side) {
        if (rc == SM_OK) HIP_TRY(ctx, hipStreamWaitEvent(ws, ctx->ev_fb_join, 0));
    } else if (rc == SM_OK && !(ctx->dbg_flags & DBG_NO_FALLBACK)) {
        if (ctx->dbg_flags & DBG_FORCE_FALLBACK) HIP_TRY(ctx, hipMemsetAsync(gflag, 1, 1, ws));
        ctx->fb_guard = gflag;
        rc = dispatch(ctx, n, g, bs, DISPATCH_PATHS);
        if (rc == SM_OK) rc = dispatch(ctx, n, g, bs, DISPATCH_WTA);
        ctx->fb_guard = nullptr;
    }
    ctx->wta_override = nullptr;
    return rc;
}

// hybrid 8-path aggregation (see use_hybrid); leaves per-direction slots 0..4 and bs.part for k_wta
int run_hybrid(sm_ctx* ctx, const Norm& n, const Geo& g, BufSet& bs)
{
    const int G = g.G;
    int rc;
    SweepJob j{};
    j.cost = (const uint8_t*)bs.cost.p;
    j.cost_pair = g.vol * elem_bytes(n);
    j.G = G;
    if ((rc = ensure_sweep_err(ctx)) != SM_OK) return rc;
    j.err = (uint32_t*)ctx->sweep_err.p + ERR_STICKY;  // no fallback here: a give-up is an error
    if ((rc = ensure(ctx, bs.part, (size_t)G * g.vol * 2)) != SM_OK) return rc;
    j.part = (uint16_t*)bs.part.p;
    j.part_pair = g.vol * 2;
    if ((rc = ensure_event(ctx, ctx->ev_fork)) != SM_OK) return rc;
    if ((rc = ensure_event(ctx, ctx->ev_join)) != SM_OK) return rc;
    StageTimer t(ctx, ctx->stream, SM_STAGE_PATHS, G);
    // the sweep first (its strips must become co-resident), then the per-direction launch
    HIP_TRY(ctx, hipEventRecord(ctx->ev_fork, ctx->stream));
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->side, ctx->ev_fork, 0));
    const hipStream_t main = ctx->stream;
    ctx->stream = ctx->side;
    {
        StageTimer ts(ctx, ctx->stream, SM_STAGE_SWEEP, G);
        rc = sweep_pass(ctx, n, g, j, 0);
    }
    ctx->stream = main;
    if (rc != SM_OK) return rc;
    HIP_TRY(ctx, hipEventRecord(ctx->ev_join, ctx->side));
    if ((rc = dispatch(ctx, n, g, bs, n.ndirs == 8 ? DISPATCH_HYBRID : DISPATCH_HORIZONTAL)) != SM_OK) return rc;
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
    return SM_OK;
}

// sticky device-side error of the unguarded (hybrid) sweep use; clears it.  The
// default sweep engine recovers on the device instead (run_group's fallback).
int check_sweep_errors(sm_ctx* ctx)
{
    if (ctx->twin) {
        int rc = check_sweep_errors(ctx->twin);
        if (rc != SM_OK) return fail(ctx, rc, "%s", ctx->twin->err.c_str());
    }
    if (!ctx->sweep_err.p) return SM_OK;
    uint32_t e = 0;
    uint32_t* w = (uint32_t*)ctx->sweep_err.p + ERR_STICKY;
    HIP_TRY(ctx, hipMemcpy(&e, w, 4, hipMemcpyDeviceToHost));
    if (e) {
        HIP_TRY(ctx, hipMemset(w, 0, 4));
        return fail(ctx, SM_E_HIP, "sweep: strip-boundary hand-off timed out (workgroups not co-resident?)");
    }
    return SM_OK;
}

// Cost volumes leave with nontemporal stores when the launch group's volume cannot stay in
// the 256 MB Infinity Cache anyway (census8, 8 KITTI pairs: 227.3 -> 219.9 us per pair, the
// sweeps after the cost faster too); a group that fits (one pair per call, the per-direction
// engine's cache-sized groups) keeps default stores, so its readers hit the cache
// (single-pair compute_disparity 1.98 vs 2.33 ms with nt).  DESIGN.md §4.1 "Cost stage".
int cost_nt(const Geo& g, size_t elem_bytes)
{
    return (size_t)g.G * g.vol * elem_bytes > ((size_t)224 << 20) ? 1 : 0;
}

// SGBM cost volume, streaming form (sm_cost.hpp k_sgbm_cost2): one workgroup per
// (TX-column strip, band of rows, pair)
#ifndef SGBM_COST2_WGS
#define SGBM_COST2_WGS 2048  // workgroups a launch aims for (bands = this / (strips x pairs))
#endif
template <int S, int CPT>
int launch_cost2_s(sm_ctx* ctx, const Norm& n, const Geo& g, const smk::SgbmCostArgs& sc)
{
    const int NP = n.D / 2, CG = std::max(1, 256 / NP), bd = NP * CG, TX = CG * CPT, NHC = TX + 2 * S;
    const int rpairs = TX + 2 * S + n.D - 1;
    if (NP > 256 || NHC > 4 * bd || rpairs > 4 * bd)
        return fail(ctx, SM_E_UNSUPPORTED, "sgbm cost: numDisparities %d not built", n.D);
    const bool one = NHC <= bd && rpairs <= bd;  // one prefetch slot per thread (fewer VGPRs)
    const int rph = (rpairs + 1) / 2;
    const size_t lds = (size_t)NHC * 16 + (size_t)((NHC + 1) & ~1) * 8 + (size_t)2 * rph * 24 + (size_t)2 * ((CG * ((NHC + CG - 1) / CG)) | 1) * NP * 4;
    smk::SgbmCost2Args c2{};
    c2.planes = sc.planes;
    c2.C = sc.C;
    c2.C_pair = sc.C_pair;
    c2.H = sc.H;
    c2.W = sc.W;
    c2.width1 = sc.width1;
    c2.D = sc.D;
    c2.minD = sc.minD;
    c2.minX1 = sc.minX1;
    c2.Yc = sc.Yc;
    c2.nt = cost_nt(g, 2);
    const int strips = (n.width1 + TX - 1) / TX;
    // enough workgroups to fill the chip; bands at least 8 rows (warm-up 2S rows each)
    const int wgs = ctx->tune_cost_wgs > 0 ? ctx->tune_cost_wgs : SGBM_COST2_WGS;
    const int want = std::max(1, wgs / std::max(1, strips * g.G));
    c2.band = std::max({(sc.Yc + want - 1) / want, 8, 4 * S});
    const int bands = (sc.Yc + c2.band - 1) / c2.band;
    if (one)
        hipLaunchKernelGGL((smk::k_sgbm_cost2<S, CPT, 1>), dim3(strips, bands, g.G), dim3(bd), lds, ctx->stream, c2);
    else
        hipLaunchKernelGGL((smk::k_sgbm_cost2<S, CPT, 4>), dim3(strips, bands, g.G), dim3(bd), lds, ctx->stream, c2);
    HIP_TRY(ctx, hipGetLastError());
    return SM_OK;
}

int launch_sgbm_cost2(sm_ctx* ctx, const Norm& n, const Geo& g, const smk::SgbmCostArgs& sc)
{
    if (ctx->dbg_flags & DBG_COST_TILE) return SM_OK;
    // 8 columns per thread: 16 measured slower (fewer waves: the register ring is 2S+1 x CPT)
    switch (n.bs / 2) {
    case 0: return launch_cost2_s<0, 8>(ctx, n, g, sc);
    case 1: return launch_cost2_s<1, 8>(ctx, n, g, sc);
    case 2: return launch_cost2_s<2, 8>(ctx, n, g, sc);
    case 3: return launch_cost2_s<3, 8>(ctx, n, g, sc);
    case 4: return launch_cost2_s<4, 8>(ctx, n, g, sc);
    case 5: return launch_cost2_s<5, 8>(ctx, n, g, sc);
    default: return fail(ctx, SM_E_UNSUPPORTED, "blockSize %d not built", n.bs);
    }
}

int group_size(const sm_ctx* ctx, const Norm& n, int H, int npairs, bool sweep, bool hybrid)
{
    const size_t cells = (size_t)H * std::max(n.width1, 1) * n.D;
    // sweep engine: a slot per direction (E and W, and every other direction's volume the
    // guarded fallback writes: run_pairs' L_pair) + the u16 partial at 8 paths; hybrid: 5
    // volumes + the partial; else one volume per direction
    const size_t per = sweep    ? cells * (n.ndirs * elem_bytes(n) + (n.ndirs == 8 ? 2 : 0))
                       : hybrid ? cells * (hybrid_slots(n) * elem_bytes(n) + 2)
                                : cells * elem_bytes(n) * n.ndirs;
    size_t g = std::max<size_t>(1, kSetBudget / std::max<size_t>(per, 1));
    // at least two groups per call when possible, so WTA(g) overlaps paths(g+1)
    const size_t half = overlap(ctx) ? std::max(1, (npairs + 1) / 2) : kMaxGroup;
    const int cap = (ctx->dbg_flags >> 16) & 7;  // ablation: launch-group size cap (0 = none)
    if (cap) return (int)std::min<size_t>({g, (size_t)cap, half});
    g = std::min<size_t>({g, (size_t)kMaxGroup, half});
    // per-direction engine, u8 costs: a group whose cost volumes fit the Infinity Cache keeps
    // them there while the 8 directions re-read them (the path volumes are stored nt, so
    // they do not evict them): KITTI census8, 8 pairs, 262 -> 249 us per pair in groups of
    // 4.  Only where that leaves >= kMallMinPairs pairs per group and at
    // most two groups per call (16 pairs: one group of 16 250 us, four of 4 256 us: the
    // horizontal chains need the pairs for parallelism); the groups are balanced.
    if (!sweep && !hybrid && elem_bytes(n) == 1 && !(ctx->dbg_flags & DBG_NO_MALL_GROUPS)) {
        const size_t fit = kMallBudget / std::max<size_t>(cells, 1);
        const size_t ngroups = fit ? ((size_t)npairs + fit - 1) / fit : 0;
        if (fit >= (size_t)kMallMinPairs && fit < g && ngroups <= 2)
            g = std::max<size_t>(1, ((size_t)npairs + ngroups - 1) / ngroups);
    }
    return (int)g;
}

int ensure_event(sm_ctx* ctx, hipEvent_t& e)
{
    if (!e) HIP_TRY(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return SM_OK;
}

// cv::filterSpeckles over G int16 maps (sm_speckle.hpp), enqueued on stream st.
int run_speckles(sm_ctx* ctx, hipStream_t st, int16_t* img, int G, int H, int W, int newval, int maxsize,
                 int maxdiff)
{
    StageTimer t(ctx, st, SM_STAGE_SPECKLE, G);
    const size_t npx = (size_t)H * W;
    int rc;
    if ((rc = ensure(ctx, ctx->sp_parent, G * npx * 4)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->sp_count, G * npx * 4)) != SM_OK) return rc;
    smk::SpeckleArgs sa{};
    sa.img = img;
    sa.parent = (int*)ctx->sp_parent.p;
    sa.count = (int*)ctx->sp_count.p;
    sa.H = H;
    sa.W = W;
    sa.newval = newval;
    sa.maxsize = maxsize;
    sa.maxdiff = maxdiff;
    const dim3 grid((unsigned)((npx + 255) / 256), G);
    hipLaunchKernelGGL(smk::k_speckle_init, grid, dim3(256), 0, st, sa);
    hipLaunchKernelGGL(smk::k_speckle_union, grid, dim3(256), 0, st, sa);
    hipLaunchKernelGGL(smk::k_speckle_count, grid, dim3(256), 0, st, sa);
    hipLaunchKernelGGL(smk::k_speckle_apply, grid, dim3(256), 0, st, sa);
    HIP_TRY(ctx, hipGetLastError());
    return SM_OK;
}

// median + speckle filter of a launch group's pre-median maps (bs.raw -> d_out) on
// stream sb, and the bookkeeping sm_debug_fetch reads
int finish_group(sm_ctx* ctx, const Geo& g, const Norm& n, BufSet& bs, int s, int16_t* d_out, hipStream_t sb)
{
    const int H = g.H, W = g.W, G = g.G;
    int rc;
    {
        StageTimer t(ctx, sb, SM_STAGE_MEDIAN, G);
        hipLaunchKernelGGL(smk::k_median3, dim3((W + 255) / 256, H, G), dim3(256), 0, sb,
                           (const int16_t*)bs.raw.p, d_out, H, W, (size_t)H * W);
        HIP_TRY(ctx, hipGetLastError());
    }
    if (n.speckle_ws > 0) {  // filterSpeckles(disp, INVALID, speckleWindowSize, 16*speckleRange)
        if ((rc = run_speckles(ctx, sb, d_out, G, H, W, (n.minD - 1) * 16, n.speckle_ws, 16 * n.speckle_range)) !=
            SM_OK)
            return rc;
    }
    if (sb != ctx->stream) {
        HIP_TRY(ctx, hipEventRecord(bs.wta_done, sb));
        bs.pending = true;
    }
    ctx->last_width1 = n.width1;
    ctx->last_index = G - 1;
    ctx->last_L_pair = g.L_pair;
    ctx->last_set = s;
    return SM_OK;
}

// OpenCV-SGBM outside the int16-exact range or on BGR input (sm_wide.hpp): planes
// per channel -> horizontal box sums -> OpenCV's row-by-row int16 C -> int16 path
// lines -> saturating S + WTA + LR check, all on the caller's stream, into bs.raw
template <int DPL>
int wide_paths_wta(sm_ctx* ctx, const Geo& g, const Norm& n, BufSet& bs)
{
    smk::WidePathArgs pa{};
    pa.C = (const int16_t*)bs.cost.p;
    pa.vol = g.vol;
    pa.L = (uint8_t*)bs.L.p;
    pa.slot_bytes = g.slot_bytes;
    pa.L_pair_bytes = g.L_pair;
    pa.H = g.H;
    pa.width1 = n.width1;
    pa.D = n.D;
    pa.P1 = n.P1;
    pa.P2 = n.P2;
    pa.ndirs = n.ndirs;
    const int dys[8] = {0, 0, 1, 1, 1, -1, -1, -1}, dxs[8] = {1, -1, 1, 0, -1, 1, 0, -1};
    int blocks = 0;
    for (int k = 0; k < n.ndirs; k++) {
        pa.blk_start[k] = blocks;
        const int nl = dys[k] == 0 ? g.H : dxs[k] == 0 ? n.width1 : n.width1 + g.H - 1;
        blocks += (nl + 15) / 16;
    }
    for (int k = n.ndirs; k <= 8; k++) pa.blk_start[k] = blocks;
    {
        StageTimer t(ctx, ctx->stream, SM_STAGE_PATHS, g.G);
        hipLaunchKernelGGL((smk::k_wide_paths<DPL>), dim3(blocks, g.G), dim3(256), 0, ctx->stream, pa);
        HIP_TRY(ctx, hipGetLastError());
    }
    smk::WideWtaArgs wa{};
    wa.L = (const uint8_t*)bs.L.p;
    wa.slot_bytes = g.slot_bytes;
    wa.L_pair_bytes = g.L_pair;
    wa.H = g.H;
    wa.W = g.W;
    wa.width1 = n.width1;
    wa.D = n.D;
    wa.minD = n.minD;
    wa.minX1 = n.minX1;
    wa.uniq = n.uniq;
    wa.disp12 = n.disp12;
    wa.ndirs = n.ndirs;
    wa.disp = (int16_t*)bs.raw.p;
    wa.wta = ctx->wta_dst;
    const size_t smem = (size_t)g.W * (wa.wta ? 10 : 8) + 16;
    if (smem > kRowLds)
        return fail(ctx, SM_E_UNSUPPORTED, "width %d: the WTA row kernel's %zu B of LDS exceed %zu%s", g.W, smem,
                    kRowLds, wa.wta ? " (with the WTA index output)" : "");
    StageTimer t(ctx, ctx->stream, SM_STAGE_WTA, g.G);
    hipLaunchKernelGGL((smk::k_wide_wta<DPL, 1024>), dim3(g.H, g.G), dim3(1024), smem, ctx->stream, wa);
    HIP_TRY(ctx, hipGetLastError());
    return SM_OK;
}

int run_wide(sm_ctx* ctx, const Src& src, const Geo& g, const Norm& n, BufSet& bs)
{
    const int H = g.H, W = g.W, G = g.G;
    int rc;
    {
        StageTimer t(ctx, ctx->stream, SM_STAGE_COST, G);
        if ((rc = ensure(ctx, ctx->planes, (size_t)G * 2 * n.cn * H * W * 8)) != SM_OK) return rc;
        if ((rc = ensure(ctx, bs.cost, (size_t)G * g.vol * 2)) != SM_OK) return rc;
        if ((rc = ensure(ctx, bs.part, (size_t)G * g.vol * 2)) != SM_OK) return rc;  // horizontal sums
        smk::PrefilterArgs pf{};
        pf.img[0] = src.L;
        pf.img[1] = src.R;
        pf.in_pair = src.pair_stride;
        pf.planes = (uint8_t*)ctx->planes.p;
        pf.H = H;
        pf.W = W;
        pf.stride = g.stride;
        pf.ftzero = n.ftzero;
        pf.cn = n.cn;
        hipLaunchKernelGGL(smk::k_sgbm_prefilter, dim3((W + 255) / 256, (H + smk::PF_ROWS - 1) / smk::PF_ROWS, 2 * G * n.cn), dim3(256), 0, ctx->stream,
                           pf);
        HIP_TRY(ctx, hipGetLastError());
        smk::WideArgs wa{};
        wa.planes = (const uint2*)ctx->planes.p;
        wa.hsum = (int16_t*)bs.part.p;
        wa.C = (int16_t*)bs.cost.p;
        wa.vol = g.vol;
        wa.H = H;
        wa.W = W;
        wa.width1 = n.width1;
        wa.D = n.D;
        wa.minD = n.minD;
        wa.minX1 = n.minX1;
        wa.cn = n.cn;
        wa.SW2 = n.bs / 2;
        wa.SH2 = n.bs / 2;
        wa.P2 = n.P2;
        wa.hh = n.mode == SM_MODE_HH;
        constexpr int TX = 64;
        // a window sum past 32767 makes OpenCV's saturating running sums differ from the window sums
        if ((long long)(2 * wa.SW2 + 1) * n.cn * (2 * n.ftzero + 63) > 32767)
            hipLaunchKernelGGL(smk::k_wide_hsum_scan, dim3(H, G), dim3(256), 0, ctx->stream, wa);
        else
            hipLaunchKernelGGL((smk::k_wide_hsum<TX>), dim3((n.width1 + TX - 1) / TX, H, G), dim3(256),
                               (size_t)(TX + 2 * wa.SW2) * n.D * 2, ctx->stream, wa);
        HIP_TRY(ctx, hipGetLastError());
        hipLaunchKernelGGL(smk::k_wide_vscan, dim3((unsigned)((g.vol / H + 255) / 256), G), dim3(256), 0,
                           ctx->stream, wa);
        HIP_TRY(ctx, hipGetLastError());
    }
    switch (n.dpl) {
#define CASE(k) \
    case k: return wide_paths_wta<k>(ctx, g, n, bs);
        CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) CASE(8)
        CASE(9) CASE(10) CASE(11) CASE(12) CASE(13) CASE(14) CASE(15) CASE(16)
#undef CASE
    default: return fail(ctx, SM_E_UNSUPPORTED, "numDisparities %d not built", n.D);
    }
}

// G pairs (device pointers; pair i at dL + i*pair_stride).
int run_group(sm_ctx* ctx, const Src& src, const Geo& g, const Norm& n, int16_t* d_out)
{
    const uint8_t *dL = src.L, *dR = src.R;
    const size_t pair_stride = src.pair_stride;
    const int H = g.H, W = g.W, G = g.G;
    const int s = overlap(ctx) ? ctx->next_set : 0;  // one buffer set unless overlapping
    ctx->next_set = s ^ 1;
    BufSet& bs = ctx->set[s];
    int rc;
    if ((rc = ensure_event(ctx, bs.paths_done)) != SM_OK) return rc;
    if ((rc = ensure_event(ctx, bs.wta_done)) != SM_OK) return rc;
    // buffer set s is free once stream B finished its previous group
    if (bs.pending) HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, bs.wta_done, 0));
    if (n.width1 <= 0) {
        const int INVALID = (n.minD - 1) * 16;
        for (int i = 0; i < G; i++) {
            hipLaunchKernelGGL(smk::k_fill16, dim3(grid_for((size_t)H * W)), dim3(256), 0, ctx->stream,
                               d_out + (size_t)i * H * W, (size_t)H * W, (int16_t)INVALID);
            HIP_TRY(ctx, hipGetLastError());
            if (ctx->wta_dst) {
                hipLaunchKernelGGL(smk::k_fill16, dim3(grid_for((size_t)H * W)), dim3(256), 0, ctx->stream,
                                   ctx->wta_dst + (size_t)i * H * W, (size_t)H * W, (int16_t)-1);
                HIP_TRY(ctx, hipGetLastError());
            }
        }
        bs.pending = false;
        ctx->last_width1 = 0;
        return SM_OK;
    }
    if ((rc = ensure(ctx, bs.L, g.L_pair * G)) != SM_OK) return rc;
    if ((rc = ensure(ctx, bs.raw, (size_t)G * H * W * 2)) != SM_OK) return rc;
    // the sweeps' give-up flag of this buffer set, cleared by the group's first kernel
    uint32_t* gflag = nullptr;
    if (g.sweep) {
        if ((rc = ensure_sweep_err(ctx)) != SM_OK) return rc;
        gflag = (uint32_t*)ctx->sweep_err.p + ERR_GROUP0 + s;
    }
    if (n.wide) {
        if ((rc = run_wide(ctx, src, g, n, bs)) != SM_OK) return rc;
        return finish_group(ctx, g, n, bs, s, d_out, ctx->stream);
    }
    {
        StageTimer t(ctx, ctx->stream, SM_STAGE_COST, G);
        if (n.cost == SM_COST_CENSUS) {
            for (int i = 0; i < 2; i++)
                if ((rc = ensure(ctx, bs.census[i], (size_t)G * g.census_pair * 8)) != SM_OK) return rc;
            smk::CensusArgs ca{};
            ca.img[0] = dL;
            ca.img[1] = dR;
            ca.out[0] = (uint64_t*)bs.census[0].p;
            ca.out[1] = (uint64_t*)bs.census[1].p;
            ca.in_pair = pair_stride;
            ca.H = H;
            ca.W = W;
            ca.stride = g.stride;
            ca.zero_word = gflag;
            hipLaunchKernelGGL(smk::k_census9x7,
                               dim3((W + smk::CT_W - 1) / smk::CT_W, (H + smk::CT_H - 1) / smk::CT_H, 2 * G),
                               dim3(256), 0, ctx->stream, ca);
            HIP_TRY(ctx, hipGetLastError());
            if (use_cost8(ctx, n)) {
                if ((rc = ensure(ctx, bs.cost, (size_t)G * g.vol)) != SM_OK) return rc;
                smk::Cost8Args c8{};
                c8.cl = ca.out[0];
                c8.cr = ca.out[1];
                c8.census_pair = g.census_pair;
                c8.C = (uint8_t*)bs.cost.p;
                c8.C_pair = g.vol;
                c8.H = H;
                c8.W = W;
                c8.width1 = n.width1;
                c8.D = n.D;
                c8.minD = n.minD;
                c8.minX1 = n.minX1;
                c8.nt = cost_nt(g, 1);
                hipLaunchKernelGGL(smk::k_census_cost8,
                                   dim3((n.width1 + smk::C8_TX - 1) / smk::C8_TX, (H + smk::C8_RY - 1) / smk::C8_RY, G),
                                   dim3(256),
                                   0, ctx->stream, c8);
                HIP_TRY(ctx, hipGetLastError());
            }
        } else if (n.cost == SM_COST_VOLUME) {
            if ((rc = ensure(ctx, bs.cost, (size_t)G * g.vol * 2)) != SM_OK) return rc;
            if ((rc = ensure_sweep_err(ctx)) != SM_OK) return rc;  // (holds the clamp / NaN counters)
            const float* win = nullptr;
            if (src.scale == 0.f || std::isnan(src.scale)) {  // scale 0 or NaN: the window from the volume's own range
                if ((rc = ensure(ctx, ctx->volwin, (size_t)G * 16)) != SM_OK) return rc;
                smk::VolWinArgs wa{};
                wa.vol = src.vol;
                wa.vol_pair = src.vol_pair;
                wa.Dv = n.Dv;
                wa.H = H;
                wa.W = W;
                wa.minX1 = n.minX1;
                wa.width1 = n.width1;
                wa.keys = (uint32_t*)ctx->volwin.p;
                wa.win = (float*)ctx->volwin.p + 2 * G;
                hipLaunchKernelGGL(smk::k_vol_keys_init, dim3((G + 255) / 256), dim3(256), 0, ctx->stream, wa.keys, G);
                const int lines = n.Dv * H;
                hipLaunchKernelGGL(smk::k_vol_minmax, dim3(std::min(lines, std::max(1, 2048 / G)), G), dim3(256), 0,
                                   ctx->stream, wa);
                hipLaunchKernelGGL(smk::k_vol_window, dim3((G + 255) / 256), dim3(256), 0, ctx->stream, wa, G);
                HIP_TRY(ctx, hipGetLastError());
                win = wa.win;
            }
            smk::VolArgs va{};
            va.win = win;
            va.clamped = (unsigned long long*)((uint32_t*)ctx->sweep_err.p + ERR_VOL_CLAMPED);
            va.nans = (unsigned long long*)((uint32_t*)ctx->sweep_err.p + ERR_VOL_NAN);
            va.vol = src.vol;
            va.vol_pair = src.vol_pair;
            va.C = (uint16_t*)bs.cost.p;
            va.C_pair = g.vol;
            va.H = H;
            va.W = W;
            va.width1 = n.width1;
            va.D = n.D;
            va.Dv = n.Dv;
            va.cpad = smk::vol_pad_cost(n.P2);
            va.minX1 = n.minX1;
            va.offset = src.offset;
            va.scale = src.scale;
            va.nt = cost_nt(g, 2);
            va.zero_word = gflag;
            // 64-column tiles measured faster than 128 (117 vs 130 us/pair at D=192)
            hipLaunchKernelGGL(smk::k_cost_volume_f32<64>, dim3((n.width1 + 63) / 64, H, G), dim3(256),
                               (size_t)64 * (n.D / 2 + 1) * 4, ctx->stream, va);
            HIP_TRY(ctx, hipGetLastError());
        } else {
            if ((rc = ensure(ctx, ctx->planes, (size_t)G * 2 * H * W * 8)) != SM_OK) return rc;
            if ((rc = ensure(ctx, bs.cost, (size_t)G * g.vol * 2)) != SM_OK) return rc;
            smk::PrefilterArgs pf{};
            pf.img[0] = dL;
            pf.img[1] = dR;
            pf.in_pair = pair_stride;
            pf.planes = (uint8_t*)ctx->planes.p;
            pf.H = H;
            pf.W = W;
            pf.stride = g.stride;
            pf.ftzero = n.ftzero;
            pf.cn = 1;
            pf.zero_word = gflag;
            hipLaunchKernelGGL(smk::k_sgbm_prefilter, dim3((W + 255) / 256, (H + smk::PF_ROWS - 1) / smk::PF_ROWS, 2 * G), dim3(256), 0, ctx->stream, pf);
            HIP_TRY(ctx, hipGetLastError());
            smk::SgbmCostArgs sc{};
            sc.planes = (const uint2*)ctx->planes.p;
            sc.C = (uint16_t*)bs.cost.p;
            sc.C_pair = g.vol;
            sc.H = H;
            sc.W = W;
            sc.width1 = n.width1;
            sc.D = n.D;
            sc.minD = n.minD;
            sc.minX1 = n.minX1;
            sc.SW2 = n.bs / 2;
            sc.SH2 = n.bs / 2;
            sc.Yc = std::max(1, H - n.bs / 2);
            // streaming box sums (k_sgbm_cost2); flag 1<<22 restores the tiled kernel
            if ((rc = launch_sgbm_cost2(ctx, n, g, sc)) != SM_OK) return rc;
            // 64-column tiles up to blockSize 7; 32-column tiles keep blockSize 9..11 within 64 KB of LDS
            if (!(ctx->dbg_flags & DBG_COST_TILE)) {
            } else if (n.bs <= 7)
                hipLaunchKernelGGL((smk::k_sgbm_cost<64, 3>),
                                   dim3((n.width1 + 63) / 64, (sc.Yc + smk::SC_TY - 1) / smk::SC_TY, G), dim3(256), 0,
                                   ctx->stream, sc);
            else
                hipLaunchKernelGGL((smk::k_sgbm_cost<32, 5>),
                                   dim3((n.width1 + 31) / 32, (sc.Yc + smk::SC_TY - 1) / smk::SC_TY, G), dim3(256), 0,
                                   ctx->stream, sc);
            HIP_TRY(ctx, hipGetLastError());
            if (sc.Yc < H) {
                const size_t row = (size_t)n.width1 * n.D;
                hipLaunchKernelGGL(smk::k_sgbm_cost_tail,
                                   dim3(std::max(1, grid_for((size_t)(H - sc.Yc) * row / 8) / G), G), dim3(256), 0,
                                   ctx->stream, sc.C, g.vol, H, sc.Yc, row, (int)(n.mode == SM_MODE_HH));
                HIP_TRY(ctx, hipGetLastError());
            }
        }
    }
    if (g.sweep) {
        // 5 paths: the WTA sweep of this group overlaps the next group's cost + E/W
        // (the 8-path sweeps keep the second stream for their E/W fork)
        const hipStream_t ws = n.ndirs == 5 ? stream_b(ctx) : ctx->stream;
        if (g.lines) {
            if ((rc = run_lines(ctx, n, g, bs, ws, gflag)) != SM_OK) return rc;
        } else if ((rc = run_sweep(ctx, n, g, bs, ws, gflag)) != SM_OK) {
            return rc;
        }
        // Strips of a sweep wait on their neighbours, so all of a launch's strips must be
        // resident together; the grid is sized for that (sweep_pass), but work on other
        // streams or processes can take the slots.  A strip that gives up raises the
        // group flag, and the guarded per-direction launch pair (a small grid that exits
        // at once while the flag is clear) then recomputes the whole group into bs.raw
        // (run_lines enqueues its own).
        if (!g.lines && (rc = sweep_finish(ctx, n, g, bs, ws, gflag)) != SM_OK) return rc;
    } else if (g.hybrid) {
        if ((rc = run_hybrid(ctx, n, g, bs)) != SM_OK) return rc;
    } else if ((rc = dispatch(ctx, n, g, bs, DISPATCH_PATHS)) != SM_OK) {
        return rc;
    }
    const hipStream_t sb = stream_b(ctx);
    if (sb != ctx->stream) {
        HIP_TRY(ctx, hipEventRecord(bs.paths_done, ctx->stream));
        HIP_TRY(ctx, hipStreamWaitEvent(sb, bs.paths_done, 0));
    }
    if (!g.sweep && (rc = dispatch(ctx, n, g, bs, DISPATCH_WTA)) != SM_OK) return rc;
    return finish_group(ctx, g, n, bs, s, d_out, sb);
}

// d_wta (may be null): the integer WTA index of every pair, [npairs][H][W] int16
int run_pairs(sm_ctx* ctx, const Src& src, int npairs, int H, int W, int stride, const Norm& n, int16_t* d_out,
              int16_t* d_wta = nullptr)
{
    ctx->lastH = H;
    ctx->lastW = W;
    ctx->lastD = n.D;
    ctx->last_ndirs = n.ndirs;
    ctx->last_cost = n.cost;
    ctx->last_minD = n.minD;
    ctx->last_minX1 = n.minX1;
    Geo g{};
    g.H = H;
    g.W = W;
    g.stride = stride;
    g.vol = (size_t)H * std::max(n.width1, 0) * n.D;
    g.slot_bytes = (g.vol * elem_bytes(n) + 255) & ~size_t(255);
    g.hybrid = !n.wide && use_hybrid(ctx, n, H) && sweeps_fit(ctx, n, true);
    const bool sweep_ok = !n.wide && !g.hybrid && use_sweep(ctx, n, H);
    g.lines = sweep_ok && use_lines(ctx, n);
    g.sweep = g.lines || (sweep_ok && sweeps_fit(ctx, n, false));
    if (ctx->tune_sweep_ncw && !n.wide && !g.hybrid && !g.sweep && use_sweep(ctx, n, H))
        return fail(ctx, SM_E_UNSUPPORTED, "no fused-sweep instance with %d compute waves fits (D %d)",
                    ctx->tune_sweep_ncw, n.D);
    // sweep engine: E and W volumes in slots 0/1 plus room for every direction's volume
    // (written only by the guarded fallback); hybrid: E, W (+ NE, N, NW at 8 paths)
    g.L_pair = g.slot_bytes * (g.hybrid ? hybrid_slots(n) : n.ndirs);
    g.census_pair = (size_t)H * W;
    g.cost_pair = n.cost == SM_COST_CENSUS ? 0 : g.vol;
    int G = group_size(ctx, n, H, npairs, g.sweep, g.hybrid);
    // the sweeps' parallelism is (strips x pairs): below sweep_min_pairs pairs per launch
    // group the per-direction engine is faster; flag 16384 forces them, and so
    // does SM_TUNE_SWEEP_NCW (a forced instance is measured, never silently replaced)
    // (5 paths with the in-sweep lines: the row bands fill the CUs instead)
    if (g.sweep && std::min(G, npairs) < sweep_min_pairs(ctx, n) && !(ctx->dbg_flags & DBG_SWEEP8) &&
        !ctx->tune_sweep_ncw && !(g.lines && line_bands(ctx, n, H, std::min(G, npairs)) > 1)) {
        g.sweep = g.lines = false;
        G = group_size(ctx, n, H, npairs, false, false);
    }
    // sm_debug_fetch(1): the sweep engine's E/W volumes (none with the in-sweep lines)
    ctx->last_ndirs = g.lines ? 0 : g.sweep ? 2 : g.hybrid ? hybrid_slots(n) : n.ndirs;
    int rc = SM_OK;
    {
        StageTimer total(ctx, ctx->stream, SM_STAGE_TOTAL, npairs);
        for (int i = 0; i < npairs && rc == SM_OK; i += G) {
            g.G = std::min(G, npairs - i);
            ctx->wta_dst = d_wta ? d_wta + (size_t)i * H * W : nullptr;
            rc = run_group(ctx, src.advance(i), g, n, d_out + (size_t)i * H * W);
        }
        ctx->wta_dst = nullptr;
        // join stream B back into the caller's stream
        for (auto& bs : ctx->set)
            if (bs.pending) {
                HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, bs.wta_done, 0));
                bs.pending = false;
            }
    }
    return rc;
}


// ---- WLS post-filter (sm_wls.hpp) ---------------------------------------------
struct WlsNorm {
    int x0, y0, w, h, rx0;
    int radius, lrc, use_conf, fill, num_iter;
    float lam, att, roll_off;
    float tab[256];
};

#ifndef WLS_IEEE_DIV
#define WLS_IEEE_DIV 0  // 1: the smoother's pivots always through IEEE division
#endif
constexpr int kWlsMaxPivotIters = 8;  // FgsPivotArgs::lam

// one smoother pass (sm_wls.hpp k_fgs) along rows or columns; FAST: pivot reciprocals by
// rcp + one FMA step (exact for pivots in [1, 2^24)).  A register-resident row variant (each
// lane's 16-32 elements in VGPRs, no LDS tiles) was bit-exact but slower (960 vs 885 us per
// single-pair WLS): the serial chain, not the LDS traffic, bounds the pass.
template <int NR, bool FAST>
void launch_fgs_t(bool rows, dim3 grid, hipStream_t st, const smk::FgsArgs& fa)
{
    if (rows) hipLaunchKernelGGL((smk::k_fgs<NR, true, FAST>), grid, dim3(64), 0, st, fa);
    else hipLaunchKernelGGL((smk::k_fgs<NR, false, FAST>), grid, dim3(64), 0, st, fa);
}

void launch_fgs(int nrhs, bool fast, bool rows, dim3 grid, hipStream_t st, const smk::FgsArgs& fa)
{
    if (nrhs == 2) fast ? launch_fgs_t<2, true>(rows, grid, st, fa) : launch_fgs_t<2, false>(rows, grid, st, fa);
    else fast ? launch_fgs_t<1, true>(rows, grid, st, fa) : launch_fgs_t<1, false>(rows, grid, st, fa);
}

int normalize_wls(sm_ctx* ctx, const sm_wls_params* p, int H, int W, WlsNorm& n)
{
    if (!p) return fail(ctx, SM_E_ARG, "wls params is NULL");
    if (H <= 0 || W <= 0) return fail(ctx, SM_E_ARG, "empty disparity map (%dx%d)", W, H);
    if (!(p->lambda >= 0) || !(p->sigma_color > 0)) return fail(ctx, SM_E_ARG, "lambda must be >= 0, sigma > 0");
    if (p->num_iter < 1) return fail(ctx, SM_E_ARG, "num_iter must be >= 1");
    if (p->depth_discontinuity_radius < 0 || p->depth_discontinuity_radius > 64)
        return fail(ctx, SM_E_ARG, "depth_discontinuity_radius %d outside [0, 64]", p->depth_discontinuity_radius);
    if (p->left_offset < 0 || p->right_offset < 0 || p->top_offset < 0 || p->bottom_offset < 0)
        return fail(ctx, SM_E_ARG, "negative ROI offset");
    n.x0 = p->left_offset;
    n.y0 = p->top_offset;
    n.w = W - p->left_offset - p->right_offset;
    n.h = H - p->top_offset - p->bottom_offset;
    n.rx0 = W - (n.x0 + n.w);  // right_view_valid_disp_ROI
    n.radius = p->depth_discontinuity_radius;
    n.lrc = p->lrc_thresh;
    n.use_conf = p->use_confidence != 0;
    n.fill = 16 * (p->min_disp - 1);
    n.num_iter = p->num_iter;
    n.lam = (float)p->lambda;
    n.att = p->lambda_attenuation;
    n.roll_off = p->roll_off;
    const double sg = (double)(float)p->sigma_color;
    for (int k = 0; k < 256; k++) n.tab[k] = (float)(-std::exp(-std::sqrt((double)k * k) / sg));
    return SM_OK;
}

// WLS scratch geometry: padded ROI (FT-multiple pitch) and the pairs per chunk
struct WlsGeo {
    bool roi;
    int wp, hp;
    size_t roi_elems;
    int G;  // pairs per chunk
};

WlsGeo wls_geo(const WlsNorm& n, int npairs)
{
    WlsGeo w{};
    w.roi = n.w > 0 && n.h > 0;
    w.wp = w.roi ? (n.w + smk::FT - 1) / smk::FT * smk::FT : 0;
    w.hp = w.roi ? (n.h + smk::FT - 1) / smk::FT * smk::FT : 0;
    w.roi_elems = (size_t)w.wp * w.hp;
    // scratch per pair: num, den, Ch, Cv, old-path inter, + rows/cols pivots and factors
    // of every iteration (4 * num_iter): floats of the ROI
    const size_t per = w.roi_elems * 4 * (5 + 4 * (size_t)std::min(n.num_iter, kWlsMaxPivotIters));
    w.G = (int)std::max<size_t>(1, std::min<size_t>(npairs, (size_t(6) << 30) / std::max<size_t>(per, 1)));
    return w;
}

// every pivot's reciprocal in [1, 2^24) -> the FMA-corrected reciprocal (exact there)
bool wls_fast(const WlsNorm& n)
{
    bool fast = !WLS_IEEE_DIV;
    float lam = n.lam;
    for (int it = 0; it < n.num_iter; it++, lam = lam * n.att)
        fast = fast && std::isfinite(lam) && 1.0 + 2.0 * (double)lam < 16777216.0;
    return fast;
}

int ensure_wls(sm_ctx* ctx, const WlsGeo& wg, const WlsNorm& n)
{
    if (!wg.roi) return SM_OK;
    const size_t e = (size_t)wg.G * wg.roi_elems * 4;
    int rc;
    if ((rc = ensure(ctx, ctx->wls_num, e)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->wls_den, e)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->wls_w, 2 * e)) != SM_OK) return rc;
    if (n.num_iter <= kWlsMaxPivotIters) {
        if ((rc = ensure(ctx, ctx->wls_R, 2 * (size_t)n.num_iter * e)) != SM_OK) return rc;
        if ((rc = ensure(ctx, ctx->wls_IT, 2 * (size_t)n.num_iter * e)) != SM_OK) return rc;
    } else if ((rc = ensure(ctx, ctx->wls_inter, e)) != SM_OK) {
        return rc;
    }
    return SM_OK;
}

// The part of the WLS filter that depends on the guide alone: the smoother's edge
// weights and (num_iter <= kWlsMaxPivotIters) the Thomas pivots of every pass
// (sm_wls.hpp k_fgs_pivots), for the g pairs of one chunk, on stream st.
int wls_prepare(sm_ctx* ctx, const uint8_t* guide, size_t guide_pair, int guide_stride, int g, const WlsNorm& n,
                const WlsGeo& wg, hipStream_t st)
{
    if (!wg.roi) return SM_OK;
    smk::WlsConfArgs ca{};
    ca.guide = guide;
    ca.guide_pair = guide_pair;
    ca.guide_stride = guide_stride;
    ca.Ch = (float*)ctx->wls_w.p;
    ca.Cv = (float*)ctx->wls_w.p + (size_t)wg.G * wg.roi_elems;
    ca.roi_pair = wg.roi_elems;
    ca.x0 = n.x0;
    ca.y0 = n.y0;
    ca.w = n.w;
    ca.h = n.h;
    ca.wp = wg.wp;
    std::memcpy(ca.tab, n.tab, sizeof ca.tab);
    hipLaunchKernelGGL(smk::k_wls_weights, dim3(wg.hp, g), dim3(256), 0, st, ca);
    HIP_TRY(ctx, hipGetLastError());
    if (n.num_iter > kWlsMaxPivotIters) return SM_OK;
    const bool fast = wls_fast(n);
    const size_t var = (size_t)g * wg.roi_elems, dirv = (size_t)n.num_iter * var;
    for (int dir = 0; dir < 2; dir++) {  // 0: rows (Ch), 1: columns (Cv)
        smk::FgsPivotArgs pa{};
        pa.C = dir == 0 ? ca.Ch : ca.Cv;
        pa.R = (float*)ctx->wls_R.p + dir * dirv;
        pa.IT = (float*)ctx->wls_IT.p + dir * dirv;
        pa.roi_pair = wg.roi_elems;
        pa.var_stride = var;
        pa.w = n.w;
        pa.h = n.h;
        pa.wp = wg.wp;
        float lam = n.lam;
        for (int it = 0; it < n.num_iter; it++, lam = lam * n.att) pa.lam[it] = lam;
        const dim3 grid((dir == 0 ? wg.hp : wg.wp) / smk::FT, n.num_iter, g);
        if (dir == 0 && fast) hipLaunchKernelGGL((smk::k_fgs_pivots<true, true>), grid, dim3(64), 0, st, pa);
        else if (dir == 0) hipLaunchKernelGGL((smk::k_fgs_pivots<true, false>), grid, dim3(64), 0, st, pa);
        else if (fast) hipLaunchKernelGGL((smk::k_fgs_pivots<false, true>), grid, dim3(64), 0, st, pa);
        else hipLaunchKernelGGL((smk::k_fgs_pivots<false, false>), grid, dim3(64), 0, st, pa);
        HIP_TRY(ctx, hipGetLastError());
    }
    return SM_OK;
}

// lines per smoother workgroup: 16 (k_fgs_solve16, one wave: a pass spreads over 4x the CUs
// of the 64-line tiles) or 64 (k_fgs_solve, FGS_WAVES waves); same chains, same results
#ifndef FGS_LINES
#define FGS_LINES 16
#endif
template <int NRHS>
void launch_fgs_solve(bool rows, int nlines, int g, hipStream_t st, const smk::FgsSolveArgs& fa)
{
    if (FGS_LINES == 16) {
        const dim3 grid(nlines / smk::FL, g);
        if (rows) hipLaunchKernelGGL((smk::k_fgs_solve16<NRHS, true>), grid, dim3(64), 0, st, fa);
        else hipLaunchKernelGGL((smk::k_fgs_solve16<NRHS, false>), grid, dim3(64), 0, st, fa);
        return;
    }
    const dim3 grid(nlines / smk::FT, g);
    if (rows) hipLaunchKernelGGL((smk::k_fgs_solve<NRHS, true>), grid, dim3(64 * FGS_WAVES), 0, st, fa);
    else hipLaunchKernelGGL((smk::k_fgs_solve<NRHS, false>), grid, dim3(64 * FGS_WAVES), 0, st, fa);
}

// npairs maps; pair i: displ/dispr at +i*disp_pair elements, guide at +i*guide_pair bytes.
// prepared: wls_prepare already ran for these pairs (one chunk holds them all).
int run_wls(sm_ctx* ctx, const int16_t* dl, const int16_t* dr, size_t disp_pair, const uint8_t* guide,
            size_t guide_pair, int guide_stride, int npairs, int H, int W, const WlsNorm& n, int16_t* d_out,
            bool prepared = false)
{
    if (npairs <= 0) return SM_OK;
    const WlsGeo wg = wls_geo(n, npairs);
    const int G = wg.G;
    const bool roi = wg.roi;
    const int wp = wg.wp, hp = wg.hp;
    const size_t roi_elems = wg.roi_elems;
    int rc;
    if ((rc = ensure_wls(ctx, wg, n)) != SM_OK) return rc;
    if (prepared && G < npairs) return fail(ctx, SM_E_ARG, "internal: prepared WLS batch exceeds one chunk");
    StageTimer t(ctx, ctx->stream, SM_STAGE_WLS, npairs);
    const bool pivots = n.num_iter <= kWlsMaxPivotIters;
    // the smoother's timing ablations live in k_fgs (num_iter > kWlsMaxPivotIters); the pivot
    // path's k_fgs_solve has no such switches, so an ablation run must not silently measure it
    if (pivots && (ctx->dbg_flags & (DBG_FGS_NO_SWEEP | DBG_FGS_NO_MEM)))
        return fail(ctx, SM_E_UNSUPPORTED, "WLS timing ablations need num_iter > %d (the k_fgs path)",
                    kWlsMaxPivotIters);
    for (int p0 = 0; p0 < npairs; p0 += G) {
        const int g = std::min(G, npairs - p0);
        if (roi) {
            if (!prepared &&
                (rc = wls_prepare(ctx, guide + (size_t)p0 * guide_pair, guide_pair, guide_stride, g, n, wg,
                                  ctx->stream)) != SM_OK)
                return rc;
            smk::WlsConfArgs ca{};
            ca.dl = dl + (size_t)p0 * disp_pair;
            ca.dr = dr ? dr + (size_t)p0 * disp_pair : nullptr;
            ca.disp_pair = disp_pair;
            ca.guide = guide + (size_t)p0 * guide_pair;
            ca.guide_pair = guide_pair;
            ca.guide_stride = guide_stride;
            ca.num = (float*)ctx->wls_num.p;
            ca.den = (float*)ctx->wls_den.p;
            ca.Ch = (float*)ctx->wls_w.p;
            ca.Cv = (float*)ctx->wls_w.p + (size_t)G * roi_elems;
            ca.roi_pair = roi_elems;
            ca.H = H;
            ca.W = W;
            ca.x0 = n.x0;
            ca.y0 = n.y0;
            ca.w = n.w;
            ca.h = n.h;
            ca.wp = wp;
            ca.rx0 = n.rx0;
            ca.radius = n.radius;
            ca.lrc_thresh = n.lrc;
            ca.roll_off = n.roll_off;
            ca.use_confidence = n.use_conf;
            ca.weights = 0;  // wls_prepare wrote Ch / Cv
            std::memcpy(ca.tab, n.tab, sizeof ca.tab);
            ca.separable = smk::wls_conf_lds(n.w, n.radius) <= 65536 ? 1 : 0;
            hipLaunchKernelGGL(smk::k_wls_conf, dim3(hp, g), dim3(256),
                               ca.separable ? smk::wls_conf_lds(n.w, n.radius) : (size_t)(256 + n.w) * 4, ctx->stream, ca);
            HIP_TRY(ctx, hipGetLastError());
            const int nrhs = n.use_conf ? 2 : 1;
            float lam = n.lam;
            if (pivots) {
                // the right-hand-side sweeps over the precomputed pivots (sm_wls.hpp)
                const size_t var = (size_t)g * roi_elems, dirv = (size_t)n.num_iter * var;
                smk::FgsSolveArgs fa{};
                fa.u[0] = ca.num;
                fa.u[1] = ca.den;
                fa.roi_pair = roi_elems;
                fa.w = n.w;
                fa.h = n.h;
                fa.wp = wp;
                for (int it = 0; it < n.num_iter; it++, lam = lam * n.att) {
                    fa.lam = lam;
                    for (int dir = 0; dir < 2; dir++) {
                        fa.C = dir == 0 ? ca.Ch : ca.Cv;
                        fa.R = (const float*)ctx->wls_R.p + dir * dirv + it * var;
                        fa.IT = (const float*)ctx->wls_IT.p + dir * dirv + it * var;
                        const int nlines = dir == 0 ? hp : wp;  // multiples of FT (and of FL)
                        if (nrhs == 2) launch_fgs_solve<2>(dir == 0, nlines, g, ctx->stream, fa);
                        else launch_fgs_solve<1>(dir == 0, nlines, g, ctx->stream, fa);
                        HIP_TRY(ctx, hipGetLastError());
                    }
                }
            } else {  // more iterations than the pivot buffers hold: pivots inside each pass
                smk::FgsArgs fa{};
                fa.u[0] = ca.num;
                fa.u[1] = ca.den;
                fa.inter = (float*)ctx->wls_inter.p;
                fa.roi_pair = roi_elems;
                fa.w = n.w;
                fa.h = n.h;
                fa.wp = wp;
                fa.dbg = ((ctx->dbg_flags & DBG_FGS_NO_SWEEP) ? 1 : 0) | ((ctx->dbg_flags & DBG_FGS_NO_MEM) ? 2 : 0);
                const bool fast = wls_fast(n);
                for (int it = 0; it < n.num_iter; it++, lam = lam * n.att) {
                    fa.lam = lam;
                    fa.C = ca.Ch;
                    launch_fgs(nrhs, fast, true, dim3(hp / smk::FT, g), ctx->stream, fa);
                    fa.C = ca.Cv;
                    launch_fgs(nrhs, fast, false, dim3(wp / smk::FT, g), ctx->stream, fa);
                    HIP_TRY(ctx, hipGetLastError());
                }
            }
        }
        smk::WlsFinalArgs wa{};
        wa.num = (const float*)ctx->wls_num.p;
        wa.den = (const float*)ctx->wls_den.p;
        wa.roi_pair = roi_elems;
        wa.out = d_out + (size_t)p0 * H * W;
        wa.out_pair = (size_t)H * W;
        wa.H = H;
        wa.W = W;
        wa.x0 = n.x0;
        wa.y0 = n.y0;
        wa.w = roi ? n.w : 0;
        wa.h = roi ? n.h : 0;
        wa.wp = wp;
        wa.fill = n.fill;
        wa.use_confidence = n.use_conf;
        hipLaunchKernelGGL(smk::k_wls_final, dim3((W + 255) / 256, H, g), dim3(256), 0, ctx->stream, wa);
        HIP_TRY(ctx, hipGetLastError());
    }
    return SM_OK;
}


// ---- StereoBM (sm_bm.hpp) --------------------------------------------------------
struct BmNorm {
    int minD, ndisp, SW2, cap, tex, uniq, sws, srange, d12;
    int lofs, rofs, width1;
    int vx, vy, vw, vh;  // valid disparity ROI
};

int normalize_bm(sm_ctx* ctx, const sm_bm_params* p, int H, int W, BmNorm& n)
{
    if (!p) return fail(ctx, SM_E_ARG, "params is NULL");
    if (H <= 0 || W <= 0) return fail(ctx, SM_E_ARG, "empty image (%dx%d)", W, H);
    if (p->pre_filter_type != 0 && p->pre_filter_type != 1) return fail(ctx, SM_E_ARG, "preFilterType must be 0 or 1");
    if (p->pre_filter_size < 5 || p->pre_filter_size > 255 || p->pre_filter_size % 2 == 0)
        return fail(ctx, SM_E_ARG, "preFilterSize must be odd and in [5, 255]");
    if (p->pre_filter_cap < 1 || p->pre_filter_cap > 63) return fail(ctx, SM_E_ARG, "preFilterCap must be in [1, 63]");
    const int bs = p->block_size;
    if (bs < 5 || bs > 255 || bs % 2 == 0 || bs >= std::min(H, W))
        return fail(ctx, SM_E_ARG, "blockSize must be odd, in [5, 255] and < min(width, height)");
    if (p->num_disparities <= 0 || p->num_disparities % 16 != 0)
        return fail(ctx, SM_E_ARG, "numDisparities must be a positive multiple of 16");
    if (p->num_disparities > 256) return fail(ctx, SM_E_UNSUPPORTED, "numDisparities %d > 256 not built", p->num_disparities);
    if (p->texture_threshold < 0 || p->uniqueness_ratio < 0)
        return fail(ctx, SM_E_ARG, "textureThreshold / uniquenessRatio must be >= 0");
    if (p->pre_filter_type == 0)
        return fail(ctx, SM_E_UNSUPPORTED, "PREFILTER_NORMALIZED_RESPONSE is not implemented on the GPU path");
    n.minD = p->min_disparity;
    n.ndisp = p->num_disparities;
    n.SW2 = bs / 2;
    n.cap = p->pre_filter_cap;
    n.tex = p->texture_threshold;
    n.uniq = p->uniqueness_ratio;
    n.sws = p->speckle_window_size;
    n.srange = p->speckle_range;
    n.d12 = p->disp12_max_diff;
    n.lofs = std::max(n.ndisp - 1 + n.minD, 0);
    n.rofs = -std::min(n.ndisp - 1 + n.minD, 0);
    n.width1 = W - n.rofs - n.ndisp + 1;
    const int maxD = n.minD + n.ndisp - 1;
    const int xmin = std::max(0, maxD) + n.SW2, xmax = W - n.SW2, ymin = n.SW2, ymax = H - n.SW2;
    if (xmax - xmin > 0 && ymax - ymin > 0) {
        n.vx = xmin;
        n.vy = ymin;
        n.vw = xmax - xmin;
        n.vh = ymax - ymin;
    } else {
        n.vx = n.vy = n.vw = n.vh = 0;
    }
    if (n.d12 >= 0 && (long long)n.d12 * 16 > 0x7FFFFFFF) n.d12 = 0x7FFFFFFF / 16;
    return SM_OK;
}

int run_bm(sm_ctx* ctx, const uint8_t* dL, const uint8_t* dR, size_t pair_stride, int npairs, int H, int W,
           int stride, const BmNorm& n, int16_t* d_out)
{
    if (npairs <= 0) return SM_OK;
    const size_t npx = (size_t)H * W;
    const int FILTERED = (n.minD - 1) * 16;
    const int xs = std::max(0, n.vx - n.lofs), xe = std::min(n.width1, n.vx + n.vw - n.lofs);
    const bool region = !(n.lofs >= W || n.rofs >= W || n.width1 < 1 || n.vw == 0 || xe <= xs);
    // strip width: largest of 64/32/16/8 whose LDS fits in 64 KB
    int sws = 0;
    size_t lds = 0;
    for (int c : {64, 32, 16, 8}) {
        const int NC = c + 2 * n.SW2;
        const size_t b = ((size_t)NC * n.ndisp + (size_t)c * n.ndisp + NC + c) * 4 + 2 * (2 * (size_t)NC + n.ndisp) + 16;
        if (b <= 65536) {
            sws = c;
            lds = b;
            break;
        }
    }
    if (region && !sws) return fail(ctx, SM_E_UNSUPPORTED, "blockSize/numDisparities too large for the GPU BM kernel");
    const int G = std::min(npairs, kMaxGroup);
    int rc;
    for (int i = 0; i < 2; i++)
        if ((rc = ensure(ctx, ctx->bm_pre[i], (size_t)G * npx)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->bm_cost, (size_t)G * npx * 4)) != SM_OK) return rc;
    StageTimer tt(ctx, ctx->stream, SM_STAGE_TOTAL, npairs);
    for (int p0 = 0; p0 < npairs; p0 += G) {
        const int g = std::min(G, npairs - p0);
        int16_t* out = d_out + (size_t)p0 * npx;
        hipLaunchKernelGGL(smk::k_bm_fill, dim3((unsigned)((npx + 255) / 256), g), dim3(256), 0, ctx->stream, out, npx,
                           (int16_t)FILTERED);
        if (region) {
            {
                StageTimer t(ctx, ctx->stream, SM_STAGE_COST, g);
                smk::BmPrefilterArgs pa{};
                pa.img[0] = dL + (size_t)p0 * pair_stride;
                pa.img[1] = dR + (size_t)p0 * pair_stride;
                pa.in_pair = pair_stride;
                pa.stride = stride;
                pa.out[0] = (uint8_t*)ctx->bm_pre[0].p;
                pa.out[1] = (uint8_t*)ctx->bm_pre[1].p;
                pa.H = H;
                pa.W = W;
                pa.cap = n.cap;
                hipLaunchKernelGGL(smk::k_bm_prefilter, dim3((W + 255) / 256, H, 2 * g), dim3(256), 0, ctx->stream, pa);
            }
            StageTimer t(ctx, ctx->stream, SM_STAGE_WTA, g);
            smk::BmArgs ba{};
            ba.Lp = (const uint8_t*)ctx->bm_pre[0].p;
            ba.Rp = (const uint8_t*)ctx->bm_pre[1].p;
            ba.disp = out;
            ba.cost = (int*)ctx->bm_cost.p;
            ba.H = H;
            ba.W = W;
            ba.ndisp = n.ndisp;
            ba.mind0 = n.minD;
            ba.lofs = n.lofs;
            ba.rofs = n.rofs;
            ba.SW2 = n.SW2;
            ba.cap = n.cap;
            ba.tex_thresh = n.tex;
            ba.uniq = n.uniq;
            ba.xs = xs;
            ba.xe = xe;
            ba.y0 = n.vy;
            ba.y1 = n.vy + n.vh;
            ba.SWs = sws;
            ba.band = 64;
            ba.FILTERED = FILTERED;
            const dim3 grid((unsigned)((xe - xs + sws - 1) / sws), (unsigned)((n.vh + ba.band - 1) / ba.band), g);
            hipLaunchKernelGGL(smk::k_bm_sad, grid, dim3(256), lds, ctx->stream, ba);
            HIP_TRY(ctx, hipGetLastError());
            if (n.d12 >= 0) {
                smk::BmValidateArgs va{};
                va.disp = out;
                va.cost = (const int*)ctx->bm_cost.p;
                va.H = H;
                va.W = W;
                va.minD = n.minD;
                va.ndisp = n.ndisp;
                va.maxdiff16 = n.d12 * 16;
                hipLaunchKernelGGL(smk::k_bm_validate, dim3(H, g), dim3(256), (size_t)W * 13, ctx->stream, va);
                HIP_TRY(ctx, hipGetLastError());
            }
        }
        if (n.sws > 0 && n.srange >= 0)
            if ((rc = run_speckles(ctx, ctx->stream, out, g, H, W, FILTERED, n.sws, n.srange)) != SM_OK) return rc;
    }
    return SM_OK;
}

// the third stream of compute_disparity (WLS guide-only work), on the context's CU mask
int ensure_lr_stream(sm_ctx* ctx)
{
    int rc;
    if ((rc = ensure_event(ctx, ctx->ev_stagger)) != SM_OK) return rc;
    if (ctx->lr_stream) return SM_OK;
    if (!ctx->cu_mask.empty())
        HIP_TRY(ctx, hipExtStreamCreateWithCUMask(&ctx->lr_stream, (uint32_t)ctx->cu_mask.size(), ctx->cu_mask.data()));
    else
        HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->lr_stream, hipStreamNonBlocking));
    return SM_OK;
}

int ensure_wls_stream(sm_ctx* ctx)
{
    int rc;
    if ((rc = ensure_event(ctx, ctx->ev_wls_fork)) != SM_OK) return rc;
    if ((rc = ensure_event(ctx, ctx->ev_wls_ready)) != SM_OK) return rc;
    if (ctx->wls_stream) return SM_OK;
    if (!ctx->cu_mask.empty())
        HIP_TRY(ctx, hipExtStreamCreateWithCUMask(&ctx->wls_stream, (uint32_t)ctx->cu_mask.size(), ctx->cu_mask.data()));
    else
        HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->wls_stream, hipStreamNonBlocking));
    return SM_OK;
}

}  // namespace

extern "C" {

const char* sm_version(void) { return SM_VERSION; }

int sm_abi_version(void) { return SM_ABI_VERSION; }

int sm_create(int device, sm_ctx** out)
{
    if (!out) return fail(nullptr, SM_E_ARG, "out is NULL");
    *out = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) return fail(nullptr, SM_E_HIP, "no HIP device available (%s)", hipGetErrorString(e));
    if (device < 0 || device >= ndev) return fail(nullptr, SM_E_ARG, "device %d out of range [0,%d)", device, ndev);
    sm_ctx* ctx = new sm_ctx();
    ctx->device = device;
    e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete ctx;
        return fail(nullptr, SM_E_HIP, "context creation failed: %s", hipGetErrorString(e));
    }
    ctx->stream = ctx->own_stream;
    *out = ctx;
    return SM_OK;
}

void sm_destroy(sm_ctx* ctx)
{
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipDeviceSynchronize();
    DevBuf* bufs[] = {&ctx->img[0],  &ctx->img[1],  &ctx->planes,    &ctx->out,         &ctx->dbg,
                      &ctx->volbuf,  &ctx->wls_num, &ctx->wls_den,   &ctx->wls_inter,   &ctx->wls_disp[0], &ctx->wls_w,
                      &ctx->wls_disp[1], &ctx->wls_out, &ctx->sp_parent, &ctx->sp_count,
                      &ctx->rp_in,   &ctx->rp_out,  &ctx->rp_min,    &ctx->bm_pre[0],   &ctx->bm_pre[1],
                      &ctx->bm_cost, &ctx->hop,     &ctx->sweep_err, &ctx->wls_R,      &ctx->wls_IT,
                      &ctx->volwin};
    for (DevBuf* b : bufs)
        if (b->p) (void)hipFree(b->p);
    for (auto& bs : ctx->set) {
        DevBuf* sb[] = {&bs.census[0], &bs.census[1], &bs.cost, &bs.L,  &bs.raw,
                        &bs.part,      &bs.key2,      &bs.pre,  &bs.st, &bs.vst};
        for (DevBuf* b : sb)
            if (b->p) (void)hipFree(b->p);
        if (bs.paths_done) (void)hipEventDestroy(bs.paths_done);
        if (bs.wta_done) (void)hipEventDestroy(bs.wta_done);
    }
    for (auto& t : ctx->pending) {
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    for (auto e : ctx->free_events) (void)hipEventDestroy(e);
    if (ctx->pin) (void)hipHostFree(ctx->pin);
    if (ctx->ev_lr_fork) (void)hipEventDestroy(ctx->ev_lr_fork);
    if (ctx->ev_lr_join) (void)hipEventDestroy(ctx->ev_lr_join);
    sm_destroy(ctx->twin);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_wls_fork) (void)hipEventDestroy(ctx->ev_wls_fork);
    if (ctx->ev_wls_ready) (void)hipEventDestroy(ctx->ev_wls_ready);
    if (ctx->wls_stream) (void)hipStreamDestroy(ctx->wls_stream);
    if (ctx->lr_stream) (void)hipStreamDestroy(ctx->lr_stream);
    if (ctx->ev_stagger) (void)hipEventDestroy(ctx->ev_stagger);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    if (ctx->ev_fb_fork) (void)hipEventDestroy(ctx->ev_fb_fork);
    if (ctx->ev_ew_done) (void)hipEventDestroy(ctx->ev_ew_done);
    if (ctx->ev_fb_join) (void)hipEventDestroy(ctx->ev_fb_join);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
}

// The twin context (compute_disparity's right matcher) keeps its own stream on purpose:
// it forks from and joins back into this ctx->stream by events, whichever stream that is.
int sm_set_stream(sm_ctx* ctx, void* hip_stream)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    ctx->stream = (hipStream_t)hip_stream;  // NULL = the device's default (null) stream
    return SM_OK;
}

int sm_reset_stream(sm_ctx* ctx)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    ctx->stream = ctx->own_stream;
    return SM_OK;
}

int sm_right_matcher_params(const sm_params* left, sm_params* right)
{
    if (!left || !right) return fail(nullptr, SM_E_ARG, "NULL params");
    *right = *left;
    right->min_disparity = -(left->min_disparity + left->num_disparities) + 1;
    right->uniqueness_ratio = 0;
    right->disp12_max_diff = 1000000;
    right->speckle_window_size = 0;
    return SM_OK;
}

int sm_compute_device(sm_ctx* ctx, const uint8_t* dL, const uint8_t* dR, int H, int W, int stride,
                      const sm_params* p, int16_t* d_out)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (!dL || !dR || !d_out) return fail(ctx, SM_E_ARG, "NULL image/output pointer");
    if (stride < W) return fail(ctx, SM_E_ARG, "stride %d < width %d", stride, W);
    Norm n;
    int rc = normalize(ctx, p, H, W, n);
    if (rc != SM_OK) return rc;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    Src src;
    src.L = dL;
    src.R = dR;
    return run_pairs(ctx, src, 1, H, W, stride, n, d_out);
}

int sm_compute_wta_batch_device(sm_ctx* ctx, const uint8_t* dL, const uint8_t* dR, int npairs, size_t pair_stride,
                                int H, int W, int stride, const sm_params* p, int16_t* d_out, int16_t* d_wta)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (npairs < 0) return fail(ctx, SM_E_ARG, "npairs < 0");
    if (!dL || !dR || !d_out) return fail(ctx, SM_E_ARG, "NULL image/output pointer");
    Norm n;
    int rc = normalize(ctx, p, H, W, n);
    if (rc != SM_OK) return rc;
    if (stride < W) return fail(ctx, SM_E_ARG, "stride %d < width %d", stride, W);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    Src src;
    src.L = dL;
    src.R = dR;
    src.pair_stride = pair_stride;
    return run_pairs(ctx, src, npairs, H, W, stride, n, d_out, d_wta);
}

int sm_compute_batch_device_cn(sm_ctx* ctx, const uint8_t* dL, const uint8_t* dR, int npairs, size_t pair_stride,
                               int H, int W, int stride, int channels, const sm_params* p, int16_t* d_out)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (npairs < 0) return fail(ctx, SM_E_ARG, "npairs < 0");
    if (!dL || !dR || !d_out) return fail(ctx, SM_E_ARG, "NULL image/output pointer");
    Norm n;
    int rc = normalize(ctx, p, H, W, n, channels);
    if (rc != SM_OK) return rc;
    if (stride < W * channels) return fail(ctx, SM_E_ARG, "stride %d < width %d x %d channels", stride, W, channels);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    Src src;
    src.L = dL;
    src.R = dR;
    src.pair_stride = pair_stride;
    return run_pairs(ctx, src, npairs, H, W, stride, n, d_out);
}

int sm_compute_batch_device(sm_ctx* ctx, const uint8_t* dL, const uint8_t* dR, int npairs, size_t pair_stride,
                            int H, int W, int stride, const sm_params* p, int16_t* d_out)
{
    return sm_compute_batch_device_cn(ctx, dL, dR, npairs, pair_stride, H, W, stride, 1, p, d_out);
}

namespace {
// host-pointer matcher call: pinned staging in, one pair, maps (+ the WTA index) out
int compute_host(sm_ctx* ctx, const uint8_t* L, const uint8_t* R, int H, int W, int stride, int channels,
                 const sm_params* p, int16_t* disp_out, int16_t* wta_out)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (!L || !R || !disp_out) return fail(ctx, SM_E_ARG, "NULL image/output pointer");
    Norm n;
    int rc = normalize(ctx, p, H, W, n, channels);
    if (rc != SM_OK) return rc;
    const size_t row = (size_t)W * channels;
    if ((size_t)stride < row) return fail(ctx, SM_E_ARG, "stride %d < width %d x %d channels", stride, W, channels);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t img = (size_t)H * row, maps = (size_t)H * W * 2;
    for (int i = 0; i < 2; i++)
        if ((rc = ensure(ctx, ctx->img[i], img)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->out, maps * (wta_out ? 2 : 1))) != SM_OK) return rc;
    HostStage hs(ctx);
    if ((rc = hs.reserve(stage_bytes(img, 2) + stage_bytes(maps, 2))) != SM_OK) return rc;
    if ((rc = hs.in(ctx->img[0].p, L, H, row, stride)) != SM_OK) return rc;
    if ((rc = hs.in(ctx->img[1].p, R, H, row, stride)) != SM_OK) return rc;
    Src src;
    src.L = (const uint8_t*)ctx->img[0].p;
    src.R = (const uint8_t*)ctx->img[1].p;
    int16_t* d_wta = wta_out ? (int16_t*)ctx->out.p + (size_t)H * W : nullptr;
    rc = run_pairs(ctx, src, 1, H, W, (int)row, n, (int16_t*)ctx->out.p, d_wta);
    if (rc != SM_OK) return rc;
    if ((rc = hs.out(disp_out, ctx->out.p, maps)) != SM_OK) return rc;
    if (wta_out && (rc = hs.out(wta_out, d_wta, maps)) != SM_OK) return rc;
    if ((rc = hs.finish()) != SM_OK) return rc;
    return check_sweep_errors(ctx);
}
}  // namespace

int sm_compute_cn(sm_ctx* ctx, const uint8_t* L, const uint8_t* R, int H, int W, int stride, int channels,
                  const sm_params* p, int16_t* disp_out)
{
    return compute_host(ctx, L, R, H, W, stride, channels, p, disp_out, nullptr);
}

int sm_compute(sm_ctx* ctx, const uint8_t* L, const uint8_t* R, int H, int W, int stride, const sm_params* p,
               int16_t* disp_out, int16_t* wta_out)
{
    return compute_host(ctx, L, R, H, W, stride, 1, p, disp_out, wta_out);
}

int sm_aggregate_cost_f32_device(sm_ctx* ctx, const float* d_cost, int npairs, size_t pair_stride_elems, int D,
                                 int H, int W, const sm_params* p, float offset, float scale, int16_t* d_out)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (npairs < 0) return fail(ctx, SM_E_ARG, "npairs < 0");
    if (!d_cost || !d_out || !p) return fail(ctx, SM_E_ARG, "NULL cost/output/params pointer");
    if (D != p->num_disparities)
        return fail(ctx, SM_E_ARG, "cost volume has %d planes but numDisparities = %d", D, p->num_disparities);
    if (npairs > 1 && pair_stride_elems < (size_t)D * H * W) return fail(ctx, SM_E_ARG, "pair stride too small");
    sm_params q = *p;
    q.cost_kind = SM_COST_VOLUME;
    Norm n;
    int rc = normalize(ctx, &q, H, W, n);
    if (rc != SM_OK) return rc;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    Src src;
    src.vol = d_cost;
    src.vol_pair = pair_stride_elems;
    src.offset = offset;
    src.scale = scale;
    return run_pairs(ctx, src, npairs, H, W, W, n, d_out);
}

int sm_aggregate_cost_f32(sm_ctx* ctx, const float* cost, int D, int H, int W, const sm_params* p, float offset,
                          float scale, int16_t* disp_out)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (!cost || !disp_out) return fail(ctx, SM_E_ARG, "NULL cost/output pointer");
    if (H <= 0 || W <= 0 || D <= 0) return fail(ctx, SM_E_ARG, "empty volume (%dx%dx%d)", D, H, W);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t img = (size_t)H * W;
    int rc;
    if ((rc = ensure(ctx, ctx->volbuf, img * D * 4)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->out, img * 2)) != SM_OK) return rc;
    {
        StageTimer t_(ctx, ctx->stream, SM_STAGE_H2D, 1);
        HIP_TRY(ctx, hipMemcpyAsync(ctx->volbuf.p, cost, img * D * 4, hipMemcpyHostToDevice, ctx->stream));
    }
    rc = sm_aggregate_cost_f32_device(ctx, (const float*)ctx->volbuf.p, 1, img * D, D, H, W, p, offset, scale,
                                      (int16_t*)ctx->out.p);
    if (rc != SM_OK) return rc;
    {
        StageTimer t_(ctx, ctx->stream, SM_STAGE_D2H, 1);
        HIP_TRY(ctx, hipMemcpyAsync(disp_out, ctx->out.p, img * 2, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return check_sweep_errors(ctx);
}

int sm_wls_default_params(const sm_params* left, sm_wls_params* out)
{
    if (!left || !out) return fail(nullptr, SM_E_ARG, "NULL params");
    const int minD = left->min_disparity, D = left->num_disparities, ws = left->block_size;
    out->lambda = 8000.0;
    out->sigma_color = 1.0;
    out->lrc_thresh = 24;
    out->depth_discontinuity_radius = (int)std::ceil(0.5 * ws);
    out->use_confidence = 1;
    out->min_disp = minD;
    out->left_offset = std::max(0, minD + D);
    out->right_offset = std::max(0, -minD);
    out->top_offset = 0;
    out->bottom_offset = 0;
    out->num_iter = 3;
    out->lambda_attenuation = 0.25f;
    out->roll_off = 0.001f;
    return SM_OK;
}

int sm_wls_filter_batch_device(sm_ctx* ctx, const int16_t* d_displ, const int16_t* d_dispr, const uint8_t* d_guide,
                               int npairs, size_t guide_pair_stride, int guide_stride, int H, int W,
                               const sm_wls_params* p, int16_t* d_out)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (npairs < 0) return fail(ctx, SM_E_ARG, "npairs < 0");
    if (!d_displ || !d_guide || !d_out) return fail(ctx, SM_E_ARG, "NULL disparity/guide/output pointer");
    if (guide_stride < W) return fail(ctx, SM_E_ARG, "guide stride %d < width %d", guide_stride, W);
    WlsNorm n;
    int rc = normalize_wls(ctx, p, H, W, n);
    if (rc != SM_OK) return rc;
    if (n.use_conf && !d_dispr) return fail(ctx, SM_E_ARG, "use_confidence needs the right disparity map");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return run_wls(ctx, d_displ, d_dispr, (size_t)H * W, d_guide, guide_pair_stride, guide_stride, npairs, H, W, n,
                   d_out);
}

int sm_wls_filter(sm_ctx* ctx, const int16_t* displ, const int16_t* dispr, const uint8_t* guide, int guide_stride,
                  int H, int W, const sm_wls_params* p, int16_t* out)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (!displ || !guide || !out) return fail(ctx, SM_E_ARG, "NULL disparity/guide/output pointer");
    if (guide_stride < W) return fail(ctx, SM_E_ARG, "guide stride %d < width %d", guide_stride, W);
    WlsNorm n;
    int rc = normalize_wls(ctx, p, H, W, n);
    if (rc != SM_OK) return rc;
    if (n.use_conf && !dispr) return fail(ctx, SM_E_ARG, "use_confidence needs the right disparity map");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t img = (size_t)H * W;
    if ((rc = ensure(ctx, ctx->wls_disp[0], img * 2)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->wls_disp[1], img * 2)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->img[0], img)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->wls_out, img * 2)) != SM_OK) return rc;
    HostStage hs(ctx);
    if ((rc = hs.reserve(stage_bytes(img * 2, 3) + stage_bytes(img))) != SM_OK) return rc;
    if ((rc = hs.in(ctx->wls_disp[0].p, displ, 1, img * 2, img * 2)) != SM_OK) return rc;
    if (dispr && (rc = hs.in(ctx->wls_disp[1].p, dispr, 1, img * 2, img * 2)) != SM_OK) return rc;
    if ((rc = hs.in(ctx->img[0].p, guide, H, W, guide_stride)) != SM_OK) return rc;
    rc = run_wls(ctx, (const int16_t*)ctx->wls_disp[0].p, dispr ? (const int16_t*)ctx->wls_disp[1].p : nullptr, img,
                 (const uint8_t*)ctx->img[0].p, img, W, 1, H, W, n, (int16_t*)ctx->wls_out.p);
    if (rc != SM_OK) return rc;
    if ((rc = hs.out(out, ctx->wls_out.p, img * 2)) != SM_OK) return rc;
    if ((rc = hs.finish()) != SM_OK) return rc;
    return check_sweep_errors(ctx);
}

// compute_disparity (stereo_vision/stereo_vision.py:132-184) in one call, on
// device pointers: left matcher with the createDisparityWLSFilter mutation
// (uniqueness 0, disp12MaxDiff 1e6, speckle 0), right matcher on the swapped
// pair, WLS filter guided by the left view.
int sm_compute_disparity_batch_device(sm_ctx* ctx, const uint8_t* dL, const uint8_t* dR, int npairs,
                                      size_t pair_stride, int H, int W, int stride, const sm_params* left,
                                      const sm_wls_params* wls, int16_t* d_displ, int16_t* d_dispr,
                                      int16_t* d_filtered)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (npairs < 0) return fail(ctx, SM_E_ARG, "npairs < 0");
    if (npairs == 0) return SM_OK;  // before wls_geo / wls_prepare size any launch from it
    if (!left || !wls) return fail(ctx, SM_E_ARG, "NULL params");
    if (!d_displ || !d_dispr || !d_filtered) return fail(ctx, SM_E_ARG, "NULL output pointer");
    sm_params lm = *left, rm;
    sm_right_matcher_params(left, &rm);  // createRightMatcher (:171) sees the unmutated matcher
    lm.uniqueness_ratio = 0;             // createDisparityWLSFilter (:172) mutates the left one
    lm.disp12_max_diff = 1000000;
    lm.speckle_window_size = 0;
    // the two matchers are independent: the right one runs on the twin context (its own
    // buffers), on the caller's stream before the left one (flag 1 << 20: beside it)
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    int rc;
    if (!ctx->twin) {
        if ((rc = sm_create(ctx->device, &ctx->twin)) != SM_OK) return fail(ctx, rc, "%s", g_thread_error.c_str());
        ctx->twin->timing = ctx->timing;
        ctx->twin->dbg_flags = ctx->dbg_flags;
        ctx->twin->tune_ew_lanes = ctx->tune_ew_lanes;
        ctx->twin->tune_sweep_ncw = ctx->tune_sweep_ncw;
        ctx->twin->tune_ew_waves = ctx->tune_ew_waves;
        ctx->twin->tune_ew_prio = ctx->tune_ew_prio;
        ctx->twin->tune_ew_warmup = ctx->tune_ew_warmup;
        ctx->twin->tune_sweep_lines = ctx->tune_sweep_lines;
        ctx->twin->tune_ew_guess = ctx->tune_ew_guess;
        ctx->twin->tune_bands = ctx->tune_bands;
        ctx->twin->tune_band_warmup = ctx->tune_band_warmup;
        ctx->twin->tune_band_guess = ctx->tune_band_guess;
        ctx->twin->tune_cost_wgs = ctx->tune_cost_wgs;
        ctx->twin->tune_sweep_xcd = ctx->tune_sweep_xcd;
        if (!ctx->cu_mask.empty() &&
            (rc = sm_set_cu_mask(ctx->twin, ctx->cu_mask.data(), (int)ctx->cu_mask.size())) != SM_OK)
            return fail(ctx, rc, "%s", ctx->twin->err.c_str());
    }
    if ((rc = ensure_event(ctx, ctx->ev_lr_fork)) != SM_OK) return rc;
    if ((rc = ensure_event(ctx, ctx->ev_lr_join)) != SM_OK) return rc;
    if (stride < W) return fail(ctx, SM_E_ARG, "stride %d < width %d", stride, W);
    WlsNorm wn;
    if ((rc = normalize_wls(ctx, wls, H, W, wn)) != SM_OK) return rc;
    sm_ctx* tw = ctx->twin;
    StageTimer call(ctx, ctx->stream, SM_STAGE_CALL, npairs);
    // the WLS filter's guide-only work (edge weights, the Thomas pivots of every pass) runs
    // on a third stream beside the two matchers when the batch fits one WLS chunk
    const WlsGeo wg = wls_geo(wn, npairs);
    const bool prep = wg.roi && wg.G >= npairs;
    if (prep) {
        if ((rc = ensure_wls(ctx, wg, wn)) != SM_OK) return rc;
        if ((rc = ensure_wls_stream(ctx)) != SM_OK) return rc;
        HIP_TRY(ctx, hipEventRecord(ctx->ev_wls_fork, ctx->stream));
        HIP_TRY(ctx, hipStreamWaitEvent(ctx->wls_stream, ctx->ev_wls_fork, 0));
        if ((rc = wls_prepare(ctx, dL, pair_stride, stride, npairs, wn, wg, ctx->wls_stream)) != SM_OK) return rc;
        HIP_TRY(ctx, hipEventRecord(ctx->ev_wls_ready, ctx->wls_stream));
    }
    HIP_TRY(ctx, hipEventRecord(ctx->ev_lr_fork, ctx->stream));
    // one matcher after the other: side by side they only shared the HBM bandwidth (KITTI
    // D = 160, one pair: matchers 1.32 ms concurrent, 1.22 ms in sequence; per matcher the
    // per-direction path kernel took 665 vs 332 us)
    const bool serial = (ctx->dbg_flags & DBG_CONCURRENT_LR) == 0;
    // staggered: the left matcher starts on a second stream as soon as the right
    // one's MODE 3 sweep is done, so its cost volume and sweep overlap the right one's
    // latency-bound patch passes and WTA (with no MODE 3 sweep: after the whole right matcher)
    const bool stagger = serial && ctx->tune_lr_stagger >= 0;
    if (stagger && (rc = ensure_lr_stream(ctx)) != SM_OK) return rc;
    {
        // serial: the twin enqueues on the caller's stream for this call only (restored on
        // every exit path, so the twin never keeps a stream it does not own)
        StreamSwap sw(tw, serial ? ctx->stream : tw->stream);
        HIP_TRY(ctx, hipStreamWaitEvent(tw->stream, ctx->ev_lr_fork, 0));
        tw->sweep_done_ev = stagger ? ctx->ev_stagger : nullptr;
        tw->sweep_done_hit = false;
        rc = sm_compute_batch_device(tw, dR, dL, npairs, pair_stride, H, W, stride, &rm, d_dispr);
        tw->sweep_done_ev = nullptr;
    }
    if (rc != SM_OK) return fail(ctx, rc, "right matcher: %s", tw->err.c_str());
    if (stagger) {
        if (!tw->sweep_done_hit) HIP_TRY(ctx, hipEventRecord(ctx->ev_stagger, ctx->stream));
        HIP_TRY(ctx, hipEventRecord(ctx->ev_lr_join, ctx->stream));  // the right matcher's end
        HIP_TRY(ctx, hipStreamWaitEvent(ctx->lr_stream, ctx->ev_stagger, 0));
        {
            StreamSwap sw(ctx, ctx->lr_stream);
            rc = sm_compute_batch_device(ctx, dL, dR, npairs, pair_stride, H, W, stride, &lm, d_displ);
        }
        // the caller's stream has the right matcher; it joins the left one (every path)
        HIP_TRY(ctx, hipEventRecord(ctx->ev_stagger, ctx->lr_stream));
        HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_stagger, 0));
    } else {
        HIP_TRY(ctx, hipEventRecord(ctx->ev_lr_join, serial ? ctx->stream : tw->stream));
        rc = sm_compute_batch_device(ctx, dL, dR, npairs, pair_stride, H, W, stride, &lm, d_displ);
    }
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_lr_join, 0));  // joined on every path
    if (prep) HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_wls_ready, 0));
    if (rc != SM_OK) return rc;
    return run_wls(ctx, d_displ, d_dispr, (size_t)H * W, dL, pair_stride, stride, npairs, H, W, wn, d_filtered, prep);
}

int sm_compute_disparity(sm_ctx* ctx, const uint8_t* L, const uint8_t* R, int H, int W, int stride,
                         const sm_params* left, const sm_wls_params* wls, int16_t* displ, int16_t* filtered)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (!L || !R || !displ || !filtered) return fail(ctx, SM_E_ARG, "NULL image/output pointer");
    if (stride < W || H <= 0 || W <= 0) return fail(ctx, SM_E_ARG, "bad geometry %dx%d stride %d", W, H, stride);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t img = (size_t)H * W;
    int rc;
    for (int i = 0; i < 2; i++)
        if ((rc = ensure(ctx, ctx->img[i], img)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->wls_disp[0], img * 2)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->wls_disp[1], img * 2)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->wls_out, img * 2)) != SM_OK) return rc;
    HostStage hs(ctx);
    if ((rc = hs.reserve(stage_bytes(img, 2) + stage_bytes(img * 2, 2))) != SM_OK) return rc;
    if ((rc = hs.in(ctx->img[0].p, L, H, W, stride)) != SM_OK) return rc;
    if ((rc = hs.in(ctx->img[1].p, R, H, W, stride)) != SM_OK) return rc;
    rc = sm_compute_disparity_batch_device(ctx, (const uint8_t*)ctx->img[0].p, (const uint8_t*)ctx->img[1].p, 1, img,
                                           H, W, W, left, wls, (int16_t*)ctx->wls_disp[0].p,
                                           (int16_t*)ctx->wls_disp[1].p, (int16_t*)ctx->wls_out.p);
    if (rc != SM_OK) return rc;
    if ((rc = hs.out(displ, ctx->wls_disp[0].p, img * 2)) != SM_OK) return rc;
    if ((rc = hs.out(filtered, ctx->wls_out.p, img * 2)) != SM_OK) return rc;
    if ((rc = hs.finish()) != SM_OK) return rc;
    return check_sweep_errors(ctx);
}

int sm_filter_speckles_device(sm_ctx* ctx, int16_t* d_img, int nimg, int H, int W, int new_val,
                              int max_speckle_size, int max_diff)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (!d_img || nimg < 0 || H <= 0 || W <= 0) return fail(ctx, SM_E_ARG, "bad image arguments");
    if ((long long)H * W >= (1LL << 31)) return fail(ctx, SM_E_UNSUPPORTED, "image too large");
    if (max_speckle_size <= 0 || nimg == 0) return SM_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return run_speckles(ctx, ctx->stream, d_img, nimg, H, W, new_val, max_speckle_size, max_diff);
}

int sm_filter_speckles(sm_ctx* ctx, int16_t* img, int H, int W, int new_val, int max_speckle_size, int max_diff)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (!img || H <= 0 || W <= 0) return fail(ctx, SM_E_ARG, "bad image arguments");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t bytes = (size_t)H * W * 2;
    int rc;
    if ((rc = ensure(ctx, ctx->out, bytes)) != SM_OK) return rc;
    {
        StageTimer t_(ctx, ctx->stream, SM_STAGE_H2D, 1);
        HIP_TRY(ctx, hipMemcpyAsync(ctx->out.p, img, bytes, hipMemcpyHostToDevice, ctx->stream));
    }
    if ((rc = sm_filter_speckles_device(ctx, (int16_t*)ctx->out.p, 1, H, W, new_val, max_speckle_size, max_diff)) !=
        SM_OK)
        return rc;
    {
        StageTimer t_(ctx, ctx->stream, SM_STAGE_D2H, 1);
        HIP_TRY(ctx, hipMemcpyAsync(img, ctx->out.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return check_sweep_errors(ctx);
}

int sm_reproject_image_to_3d_device(sm_ctx* ctx, const void* d_disp, int disp_type, int nimg, int H, int W,
                                    const double* Q, int handle_missing, float* d_xyz)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (!d_disp || !d_xyz || !Q || nimg < 0 || H <= 0 || W <= 0) return fail(ctx, SM_E_ARG, "bad arguments");
    if (disp_type != SM_DISP_S16 && disp_type != SM_DISP_F32)
        return fail(ctx, SM_E_UNSUPPORTED, "disparity type %d not supported (int16 or float32)", disp_type);
    if (nimg == 0) return SM_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    smk::ReprojArgs ra{};
    ra.disp = d_disp;
    ra.xyz = d_xyz;
    std::memcpy(ra.Q, Q, sizeof ra.Q);
    ra.H = H;
    ra.W = W;
    ra.handle_missing = handle_missing != 0;
    const size_t npx = (size_t)H * W;
    if (ra.handle_missing) {
        int rc;
        if ((rc = ensure(ctx, ctx->rp_min, (size_t)nimg * 8)) != SM_OK) return rc;
        int* keys = (int*)ctx->rp_min.p;
        HIP_TRY(ctx, hipMemsetD32Async((hipDeviceptr_t)keys, 0x7FFFFFFF, nimg, ctx->stream));
        const dim3 g((unsigned)std::min<size_t>((npx + 255) / 256, 1024), nimg);
        if (disp_type == SM_DISP_S16)
            hipLaunchKernelGGL(smk::k_disp_min<int16_t>, g, dim3(256), 0, ctx->stream, (const int16_t*)d_disp, keys, npx);
        else
            hipLaunchKernelGGL(smk::k_disp_min<float>, g, dim3(256), 0, ctx->stream, (const float*)d_disp, keys, npx);
        hipLaunchKernelGGL(smk::k_keys_to_float, dim3((nimg + 63) / 64), dim3(64), 0, ctx->stream, keys,
                           (float*)(keys + nimg), nimg);
        ra.min_disp = (const float*)(keys + nimg);
    }
    const dim3 grid((W + 255) / 256, H, nimg);
    if (disp_type == SM_DISP_S16)
        hipLaunchKernelGGL(smk::k_reproject<int16_t>, grid, dim3(256), 0, ctx->stream, ra);
    else
        hipLaunchKernelGGL(smk::k_reproject<float>, grid, dim3(256), 0, ctx->stream, ra);
    HIP_TRY(ctx, hipGetLastError());
    return SM_OK;
}

int sm_reproject_image_to_3d(sm_ctx* ctx, const void* disp, int disp_type, int H, int W, const double* Q,
                             int handle_missing, float* xyz)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (!disp || !xyz || !Q || H <= 0 || W <= 0) return fail(ctx, SM_E_ARG, "bad arguments");
    if (disp_type != SM_DISP_S16 && disp_type != SM_DISP_F32)
        return fail(ctx, SM_E_UNSUPPORTED, "disparity type %d not supported (int16 or float32)", disp_type);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t npx = (size_t)H * W, ib = npx * (disp_type == SM_DISP_S16 ? 2 : 4);
    int rc;
    if ((rc = ensure(ctx, ctx->rp_in, ib)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->rp_out, npx * 12)) != SM_OK) return rc;
    {
        StageTimer t_(ctx, ctx->stream, SM_STAGE_H2D, 1);
        HIP_TRY(ctx, hipMemcpyAsync(ctx->rp_in.p, disp, ib, hipMemcpyHostToDevice, ctx->stream));
    }
    if ((rc = sm_reproject_image_to_3d_device(ctx, ctx->rp_in.p, disp_type, 1, H, W, Q, handle_missing,
                                              (float*)ctx->rp_out.p)) != SM_OK)
        return rc;
    {
        StageTimer t_(ctx, ctx->stream, SM_STAGE_D2H, 1);
        HIP_TRY(ctx, hipMemcpyAsync(xyz, ctx->rp_out.p, npx * 12, hipMemcpyDeviceToHost, ctx->stream));
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return check_sweep_errors(ctx);
}

int sm_bm_default_params(int num_disparities, int block_size, sm_bm_params* out)
{
    if (!out) return fail(nullptr, SM_E_ARG, "out is NULL");
    out->min_disparity = 0;
    out->num_disparities = num_disparities;
    out->block_size = block_size;
    out->pre_filter_type = 1;
    out->pre_filter_size = 9;
    out->pre_filter_cap = 31;
    out->texture_threshold = 10;
    out->uniqueness_ratio = 15;
    out->speckle_window_size = 0;
    out->speckle_range = 0;
    out->disp12_max_diff = -1;
    return SM_OK;
}

int sm_bm_right_matcher_params(const sm_bm_params* left, sm_bm_params* right)
{
    if (!left || !right) return fail(nullptr, SM_E_ARG, "NULL params");
    sm_bm_default_params(left->num_disparities, left->block_size, right);
    right->min_disparity = -(left->min_disparity + left->num_disparities) + 1;
    right->texture_threshold = 0;
    right->uniqueness_ratio = 0;
    right->disp12_max_diff = 1000000;
    right->speckle_window_size = 0;
    return SM_OK;
}

int sm_bm_compute_batch_device(sm_ctx* ctx, const uint8_t* dL, const uint8_t* dR, int npairs, size_t pair_stride,
                               int H, int W, int stride, const sm_bm_params* p, int16_t* d_out)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (npairs < 0) return fail(ctx, SM_E_ARG, "npairs < 0");
    if (!dL || !dR || !d_out) return fail(ctx, SM_E_ARG, "NULL image/output pointer");
    if (stride < W) return fail(ctx, SM_E_ARG, "stride %d < width %d", stride, W);
    BmNorm n;
    int rc = normalize_bm(ctx, p, H, W, n);
    if (rc != SM_OK) return rc;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return run_bm(ctx, dL, dR, pair_stride, npairs, H, W, stride, n, d_out);
}

int sm_bm_compute(sm_ctx* ctx, const uint8_t* L, const uint8_t* R, int H, int W, int stride, const sm_bm_params* p,
                  int16_t* disp_out)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (!L || !R || !disp_out) return fail(ctx, SM_E_ARG, "NULL image/output pointer");
    if (stride < W) return fail(ctx, SM_E_ARG, "stride %d < width %d", stride, W);
    BmNorm n;
    int rc = normalize_bm(ctx, p, H, W, n);
    if (rc != SM_OK) return rc;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    const size_t img = (size_t)H * W;
    for (int i = 0; i < 2; i++)
        if ((rc = ensure(ctx, ctx->img[i], img)) != SM_OK) return rc;
    if ((rc = ensure(ctx, ctx->out, img * 2)) != SM_OK) return rc;
    HostStage hs(ctx);
    if ((rc = hs.reserve(stage_bytes(img, 2) + stage_bytes(img * 2))) != SM_OK) return rc;
    if ((rc = hs.in(ctx->img[0].p, L, H, W, stride)) != SM_OK) return rc;
    if ((rc = hs.in(ctx->img[1].p, R, H, W, stride)) != SM_OK) return rc;
    rc = run_bm(ctx, (const uint8_t*)ctx->img[0].p, (const uint8_t*)ctx->img[1].p, img, 1, H, W, W, n,
                (int16_t*)ctx->out.p);
    if (rc != SM_OK) return rc;
    if ((rc = hs.out(disp_out, ctx->out.p, img * 2)) != SM_OK) return rc;
    return hs.finish();
}

// Multi-device batch from one process: ctxs[k] (one per device,
// possibly the same device twice) takes the contiguous shard of pairs
// [k*npairs/ngpu, (k+1)*npairs/ngpu); one host thread per context copies its
// pairs in, runs sm_compute_batch_device on the context's stream and copies
// the maps out.  Synchronous.  (The driver-facing scaling path is one process
// per GPU over RCCL, bench.py; this entry point is for single-process callers.)
int sm_compute_batch(sm_ctx** ctxs, int ngpu, const uint8_t* const* left, const uint8_t* const* right, int npairs,
                     int H, int W, const sm_params* p, int16_t* out)
{
    if (!ctxs || ngpu <= 0) return fail(nullptr, SM_E_ARG, "need at least one context");
    if (npairs < 0 || !left || !right || !out || !p) return fail(nullptr, SM_E_ARG, "bad batch arguments");
    for (int k = 0; k < ngpu; k++)
        if (!ctxs[k]) return fail(nullptr, SM_E_ARG, "ctxs[%d] is NULL", k);
    if (npairs == 0) return SM_OK;
    std::vector<int> rcs(ngpu, SM_OK);
    auto work = [&](int k) {
        sm_ctx* ctx = ctxs[k];
        const int a = (int)((long long)npairs * k / ngpu), b = (int)((long long)npairs * (k + 1) / ngpu);
        const int n = b - a;
        if (n <= 0) return;
        auto run = [&]() -> int {
            HIP_TRY(ctx, hipSetDevice(ctx->device));
            Norm nm;
            int rc = normalize(ctx, p, H, W, nm);
            if (rc != SM_OK) return rc;
            const size_t img = (size_t)H * W;
            for (int i = 0; i < 2; i++)
                if ((rc = ensure(ctx, ctx->img[i], img * n)) != SM_OK) return rc;
            if ((rc = ensure(ctx, ctx->out, img * 2 * n)) != SM_OK) return rc;
            HostStage hs(ctx);
            if ((rc = hs.reserve(stage_bytes(img, 2 * n) + stage_bytes(img * 2 * n))) != SM_OK) return rc;
            for (int i = 0; i < n; i++) {
                if (!left[a + i] || !right[a + i]) return fail(ctx, SM_E_ARG, "pair %d has a NULL image", a + i);
                if ((rc = hs.in((uint8_t*)ctx->img[0].p + img * i, left[a + i], 1, img, img)) != SM_OK) return rc;
                if ((rc = hs.in((uint8_t*)ctx->img[1].p + img * i, right[a + i], 1, img, img)) != SM_OK) return rc;
            }
            Src src;
            src.L = (const uint8_t*)ctx->img[0].p;
            src.R = (const uint8_t*)ctx->img[1].p;
            src.pair_stride = img;
            if ((rc = run_pairs(ctx, src, n, H, W, W, nm, (int16_t*)ctx->out.p)) != SM_OK) return rc;
            if ((rc = hs.out(out + img * a, ctx->out.p, img * 2 * n)) != SM_OK) return rc;
            if ((rc = hs.finish()) != SM_OK) return rc;
            HIP_TRY(ctx, hipStreamSynchronize(ctx->side));
            return check_sweep_errors(ctx);
        };
        rcs[k] = run();
    };
    std::vector<std::thread> th;
    for (int k = 1; k < ngpu; k++) th.emplace_back(work, k);
    work(0);
    for (auto& t : th) t.join();
    for (int k = 0; k < ngpu; k++)
        if (rcs[k] != SM_OK) {
            g_thread_error = ctxs[k]->err;
            return rcs[k];
        }
    return SM_OK;
}

int sm_synchronize(sm_ctx* ctx)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (ctx->twin) {
        int rc = sm_synchronize(ctx->twin);
        if (rc != SM_OK) return fail(ctx, rc, "%s", ctx->twin->err.c_str());
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->side));
    return check_sweep_errors(ctx);
}

int sm_get_counters(sm_ctx* ctx, long long* sweep_fallbacks)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    uint32_t n = 0;
    if (ctx->sweep_err.p) {
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->side));
        HIP_TRY(ctx, hipMemcpy(&n, (uint32_t*)ctx->sweep_err.p + ERR_FALLBACKS, 4, hipMemcpyDeviceToHost));
    }
    long long t = 0;
    if (ctx->twin) sm_get_counters(ctx->twin, &t);
    if (sweep_fallbacks) *sweep_fallbacks = n + t;
    return SM_OK;
}

int sm_get_counter(sm_ctx* ctx, int which, long long* value)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (!value) return fail(ctx, SM_E_ARG, "value is NULL");
    if (which < SM_COUNTER_SWEEP_FALLBACKS || which > SM_COUNTER_LINE_STRIPS)
        return fail(ctx, SM_E_ARG, "unknown counter %d", which);
    long long v = 0;
    if (which == SM_COUNTER_LINE_GROUPS || which == SM_COUNTER_BAND_GROUPS || which == SM_COUNTER_LINE_STRIPS) {
        v = which == SM_COUNTER_LINE_GROUPS ? ctx->line_groups
            : which == SM_COUNTER_BAND_GROUPS ? ctx->band_groups : ctx->line_strips;
    } else if (ctx->sweep_err.p) {
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->side));
        if (which != SM_COUNTER_SWEEP_FALLBACKS) {  // u64 words
            unsigned long long u = 0;
            const int word = which == SM_COUNTER_VOLUME_CLAMPED ? ERR_VOL_CLAMPED
                             : which == SM_COUNTER_VOLUME_NAN   ? ERR_VOL_NAN
                             : which == SM_COUNTER_EW_OPEN      ? ERR_EW_OPEN
                             : which == SM_COUNTER_BAND_REPAIRS ? ERR_BAND_REPAIRS
                             : which == SM_COUNTER_BAND_OPEN    ? ERR_BAND_OPEN
                                                                : ERR_EW_REPAIRS;
            HIP_TRY(ctx, hipMemcpy(&u, (uint32_t*)ctx->sweep_err.p + word, 8, hipMemcpyDeviceToHost));
            v = (long long)u;
        } else {
            uint32_t u = 0;
            HIP_TRY(ctx, hipMemcpy(&u, (uint32_t*)ctx->sweep_err.p + ERR_FALLBACKS, 4, hipMemcpyDeviceToHost));
            v = u;
        }
    }
    long long t = 0;
    if (ctx->twin) {
        int rc = sm_get_counter(ctx->twin, which, &t);
        if (rc != SM_OK) return rc;
    }
    *value = v + t;
    return SM_OK;
}

int sm_set_cu_mask(sm_ctx* ctx, const uint32_t* mask, int nwords)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (nwords < 0 || (nwords > 0 && !mask)) return fail(ctx, SM_E_ARG, "bad CU mask");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    // the streams about to be replaced drain first (this context's only: other contexts'
    // and the caller's unrelated work keep running; the twin drains its own below)
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->own_stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->side));
    if (ctx->wls_stream) HIP_TRY(ctx, hipStreamSynchronize(ctx->wls_stream));
    if (ctx->lr_stream) HIP_TRY(ctx, hipStreamSynchronize(ctx->lr_stream));
    hipStream_t a = nullptr, b = nullptr;
    if (nwords > 0) {
        HIP_TRY(ctx, hipExtStreamCreateWithCUMask(&a, (uint32_t)nwords, mask));
        hipError_t e = hipExtStreamCreateWithCUMask(&b, (uint32_t)nwords, mask);
        if (e != hipSuccess) {
            (void)hipStreamDestroy(a);
            return fail(ctx, SM_E_HIP, "hipExtStreamCreateWithCUMask: %s", hipGetErrorString(e));
        }
    } else {
        HIP_TRY(ctx, hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        hipError_t e = hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
        if (e != hipSuccess) {
            (void)hipStreamDestroy(a);
            return fail(ctx, SM_E_HIP, "hipStreamCreateWithFlags: %s", hipGetErrorString(e));
        }
    }
    (void)hipStreamDestroy(ctx->own_stream);
    (void)hipStreamDestroy(ctx->side);
    if (ctx->wls_stream) {  // recreated on the new mask when next needed
        (void)hipStreamDestroy(ctx->wls_stream);
        ctx->wls_stream = nullptr;
    }
    if (ctx->lr_stream) {
        (void)hipStreamDestroy(ctx->lr_stream);
        ctx->lr_stream = nullptr;
    }
    ctx->own_stream = a;
    ctx->side = b;
    ctx->stream = a;
    ctx->cu_mask.assign(mask, mask + nwords);
    if (ctx->twin) {
        int rc = sm_set_cu_mask(ctx->twin, mask, nwords);
        if (rc != SM_OK) return fail(ctx, rc, "%s", ctx->twin->err.c_str());
    }
    return SM_OK;
}

int sm_set_timing(sm_ctx* ctx, int enable)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (ctx->twin) sm_set_timing(ctx->twin, enable);
    // 1: every stage; SM_TIMING_ONLY | stage bits: those stages only (each timed stage
    // records two events per launch, which delay the stream by about a microsecond each)
    ctx->timing = enable == 0 ? 0u
                : (enable & SM_TIMING_ONLY) ? (uint32_t)enable & ((1u << SM_NUM_STAGES) - 1)
                                            : (1u << SM_NUM_STAGES) - 1;
    return SM_OK;
}

int sm_set_debug_flags(sm_ctx* ctx, int flags)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (!SM_ABLATIONS && (flags & kAblationFlags))
        return fail(ctx, SM_E_UNSUPPORTED, "debug flags 0x%x need the ablation build (make -C stereo_match_amd/csrc "
                    "ablation; STEREO_MATCH_AMD_LIB=.../libstereo_match_amd_ablate.so)",
                    (unsigned)(flags & kAblationFlags));
    if (ctx->twin) sm_set_debug_flags(ctx->twin, flags);
    ctx->dbg_flags = flags;
    return SM_OK;
}

int sm_set_tuning(sm_ctx* ctx, int key, int value)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    switch (key) {
    case SM_TUNE_EW_LANES:
        if (value != 0 && value != -1 && value != 8 && value != 16 && value != 32 && value != 64)
            return fail(ctx, SM_E_ARG, "E/W lanes %d: 0, -1, 8, 16, 32 or 64", value);
        ctx->tune_ew_lanes = value;
        break;
    case SM_TUNE_EW_WAVES:
        if (value < 0 || value > 4) return fail(ctx, SM_E_ARG, "E/W waves per workgroup %d: 0..4", value);
        ctx->tune_ew_waves = value;
        break;
    case SM_TUNE_EW_PRIO:
        if (value < 0 || value > 3) return fail(ctx, SM_E_ARG, "E/W issue priority %d: 0..3", value);
        ctx->tune_ew_prio = value;
        break;
    case SM_TUNE_SWEEP_NCW:
        if (value < 0) return fail(ctx, SM_E_ARG, "sweep compute waves %d < 0", value);
        ctx->tune_sweep_ncw = value;
        break;
    case SM_TUNE_EW_WARMUP:
        if (value < 0 || value > 4096) return fail(ctx, SM_E_ARG, "E/W segment warmup %d: 0..4096", value);
        ctx->tune_ew_warmup = value;
        break;
    case SM_TUNE_EW_GUESS:
        if (value < 0 || value > 1) return fail(ctx, SM_E_ARG, "E/W guess %d: 0 or 1", value);
        ctx->tune_ew_guess = value;
        break;
    case SM_TUNE_SWEEP_LINES:
        if (value < -1 || value > 1) return fail(ctx, SM_E_ARG, "sweep lines %d: -1, 0 or 1", value);
        ctx->tune_sweep_lines = value;
        break;
    case SM_TUNE_BANDS:
        if (value < 0 || value > 65535) return fail(ctx, SM_E_ARG, "row bands %d: 0..65535", value);
        ctx->tune_bands = value;
        break;
    case SM_TUNE_BAND_WARMUP:
        if (value < 0 || value > 4096) return fail(ctx, SM_E_ARG, "band warmup %d: 0..4096", value);
        ctx->tune_band_warmup = value;
        break;
    case SM_TUNE_BAND_GUESS:
        if (value < 0 || value > 1) return fail(ctx, SM_E_ARG, "band guess %d: 0 or 1", value);
        ctx->tune_band_guess = value;
        break;
    case SM_TUNE_COST_WGS:
        if (value < 0 || value > 65536) return fail(ctx, SM_E_ARG, "cost workgroups %d: 0..65536", value);
        ctx->tune_cost_wgs = value;
        break;
    case SM_TUNE_SWEEP_XCD:
        if (value < -1 || value > 1) return fail(ctx, SM_E_ARG, "sweep XCD placement %d: -1, 0 or 1", value);
        ctx->tune_sweep_xcd = value;
        break;
    case SM_TUNE_LR_STAGGER:
        if (value < -1 || value > 1) return fail(ctx, SM_E_ARG, "matcher stagger %d: -1, 0 or 1", value);
        ctx->tune_lr_stagger = value;
        break;
    default: return fail(ctx, SM_E_ARG, "unknown tuning key %d", key);
    }
    if (ctx->twin) sm_set_tuning(ctx->twin, key, value);
    return SM_OK;
}

int sm_reset_timing(sm_ctx* ctx)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (ctx->twin) sm_reset_timing(ctx->twin);
    harvest_timing(ctx);
    for (int i = 0; i < SM_NUM_STAGES; i++) {
        ctx->stage_ms[i] = 0;
        ctx->stage_launches[i] = 0;
        ctx->stage_pairs[i] = 0;
    }
    return SM_OK;
}

int sm_get_timing(sm_ctx* ctx, int stage, double* total_ms, long long* launches, long long* pairs)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    if (stage < 0 || stage >= SM_NUM_STAGES) return fail(ctx, SM_E_ARG, "stage %d out of range", stage);
    harvest_timing(ctx);
    double ms = ctx->stage_ms[stage];
    long long nl = ctx->stage_launches[stage], np = ctx->stage_pairs[stage];
    if (ctx->twin) {  // the right matcher of compute_disparity (sm_compute_disparity_batch_device)
        double tms = 0;
        long long tl = 0, tp = 0;
        sm_get_timing(ctx->twin, stage, &tms, &tl, &tp);
        ms += tms;
        nl += tl;
        np += tp;
    }
    if (total_ms) *total_ms = ms;
    if (launches) *launches = nl;
    if (pairs) *pairs = np;
    return SM_OK;
}

long long sm_debug_fetch(sm_ctx* ctx, int what, void* host, size_t bytes)
{
    if (!ctx) return fail(nullptr, SM_E_ARG, "ctx is NULL");
    const size_t et = ctx->last_cost == SM_COST_CENSUS ? 1 : 2;
    const size_t vol = (size_t)ctx->lastH * ctx->last_width1 * ctx->lastD;
    const size_t slot_bytes = (vol * et + 255) & ~size_t(255);
    const size_t img = (size_t)ctx->lastH * ctx->lastW;
    const int li = ctx->last_index;
    BufSet& bs = ctx->set[ctx->last_set];
    size_t need;
    switch (what) {
    case 0: need = vol * et; break;
    case 1: need = vol * et * ctx->last_ndirs; break;
    case 2: need = img * 2; break;
    case 3: need = img * 16; break;
#if SWEEP_STATS
    case 20: need = 48 * 8; break;  // sm_sweep.hpp SWEEP_STATS counters (read and cleared)
    case 21: need = 2048; break;    // the down sweep's workgroups' XCC ids (| 0x80), by linear id
    case 22: need = 6 * 65536 * 8; break;  // snapshot publish / observe times (s_memrealtime)
#endif
    default: return fail(ctx, SM_E_ARG, "debug item %d unknown", what);
    }
#if SWEEP_STATS
    if (what == 22 && host) {
        HIP_TRY(ctx, hipDeviceSynchronize());
        if (!ctx->sweep_err.p) return 0;
        HIP_TRY(ctx, hipMemcpy(host, (char*)ctx->sweep_err.p + 1024 + 1024 * 8, need, hipMemcpyDeviceToHost));
        return (long long)need;
    }
    if (what == 21 && host) {
        HIP_TRY(ctx, hipDeviceSynchronize());
        if (!ctx->sweep_err.p) return 0;
        HIP_TRY(ctx, hipMemcpy(host, (char*)ctx->sweep_err.p + 1024 + 1024, need, hipMemcpyDeviceToHost));
        return (long long)need;
    }
    if (what == 20 && host) {
        HIP_TRY(ctx, hipDeviceSynchronize());
        if (!ctx->sweep_err.p) return 0;
        HIP_TRY(ctx, hipMemcpy(host, (char*)ctx->sweep_err.p + 1024, need, hipMemcpyDeviceToHost));
        HIP_TRY(ctx, hipMemset((char*)ctx->sweep_err.p + 1024, 0, need));
        return (long long)need;
    }
#endif
    if (!host) return (long long)need;
    if (bytes < need) return fail(ctx, SM_E_ARG, "host buffer too small (%zu < %zu)", bytes, need);
    if (need == 0) return 0;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->side));
    if (what == 0 && ctx->last_cost == SM_COST_CENSUS) {
        int rc = ensure(ctx, ctx->dbg, need);
        if (rc != SM_OK) return rc;
        smk::CensusCostArgs cc{};
        cc.cl = (const uint64_t*)bs.census[0].p + (size_t)li * img;
        cc.cr = (const uint64_t*)bs.census[1].p + (size_t)li * img;
        cc.C = (uint8_t*)ctx->dbg.p;
        cc.H = ctx->lastH;
        cc.W = ctx->lastW;
        cc.width1 = ctx->last_width1;
        cc.D = ctx->lastD;
        cc.minD = ctx->last_minD;
        cc.minX1 = ctx->last_minX1;
        hipLaunchKernelGGL(smk::k_census_cost, dim3(grid_for(vol / 8)), dim3(256), 0, ctx->stream, cc);
        HIP_TRY(ctx, hipGetLastError());
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        HIP_TRY(ctx, hipMemcpy(host, ctx->dbg.p, need, hipMemcpyDeviceToHost));
        return (long long)need;
    }
    switch (what) {
    case 0: HIP_TRY(ctx, hipMemcpy(host, (uint8_t*)bs.cost.p + (size_t)li * vol * et, need, hipMemcpyDeviceToHost)); break;
    case 1:
        for (int k = 0; k < ctx->last_ndirs; k++)
            HIP_TRY(ctx, hipMemcpy((uint8_t*)host + k * vol * et,
                                   (uint8_t*)bs.L.p + (size_t)li * ctx->last_L_pair + k * slot_bytes, vol * et,
                                   hipMemcpyDeviceToHost));
        break;
    case 2: HIP_TRY(ctx, hipMemcpy(host, (int16_t*)bs.raw.p + (size_t)li * img, need, hipMemcpyDeviceToHost)); break;
    case 3:
        HIP_TRY(ctx, hipMemcpy(host, (uint64_t*)bs.census[0].p + (size_t)li * img, img * 8, hipMemcpyDeviceToHost));
        HIP_TRY(ctx, hipMemcpy((uint8_t*)host + img * 8, (uint64_t*)bs.census[1].p + (size_t)li * img, img * 8,
                               hipMemcpyDeviceToHost));
        break;
    }
    return (long long)need;
}

const char* sm_last_error(sm_ctx* ctx)
{
    if (ctx) return ctx->err.c_str();
    return g_thread_error.c_str();
}

}  // extern "C"
