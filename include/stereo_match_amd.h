/*
 * stereo_match_amd.h — C-ABI of the MI355X stereo disparity engine.
 *
 * Drop-in boundary for the reference hot path
 *   stereo_vision/stereo_vision.py:132  compute_disparity(gray_l, gray_r, disparity_settings, method="SGBM")
 * whose arithmetic the reference reaches through
 *   stereo_vision/stereo_vision.py:153  cv2.StereoSGBM_create(minDisparity=..., ..., preFilterCap=...)
 *   stereo_vision/stereo_vision.py:178  left_matcher.compute(gray_l, gray_r)   -> int16 disparity x16
 *   stereo_vision/stereo_vision.py:179  right_matcher.compute(gray_r, gray_l)  (createRightMatcher, :171)
 * Python binds this header with ctypes (stereo_match_amd/_lib.py); see
 * INTEGRATION.md for the binding a maintainer adds on the reference side.
 *
 * Conventions: plain pointers + sizes, no torch types.  Every function
 * returns 0 on success or a negative SM_E* code; sm_last_error() gives the
 * text.  One context per device, not shared by concurrent threads.
 * Host-pointer entry points are synchronous on return; *_device entry
 * points are asynchronous on the context's stream (sm_set_stream).
 */
#ifndef STEREO_MATCH_AMD_H
#define STEREO_MATCH_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version.  3: sm_compute takes the nullable wta_out (9 arguments; SURVEY §8b's
 * signature).  The shared object carries it in its soname (libstereo_match_amd.so.3), so a
 * binary linked against an older ABI fails to load instead of passing a stray pointer as
 * wta_out; dlopen/ctypes callers compare sm_abi_version() with the value they were written
 * against (stereo_match_amd/_lib.py does). */
#define SM_ABI_VERSION 3

#define SM_OK 0
#define SM_E_ARG (-1)         /* bad argument: mirrors OpenCV's CV_Assert failures */
#define SM_E_HIP (-2)         /* HIP runtime / launch error */
#define SM_E_UNSUPPORTED (-4) /* valid for OpenCV but not implemented / outside exact range */

#define SM_COST_SGBM 0   /* OpenCV StereoSGBM cost: BT(Sobel-x clip) + BT(raw)>>2, blockSize^2 box */
#define SM_COST_CENSUS 1 /* north-star cost: 9x7 census + Hamming (no reference counterpart) */
#define SM_COST_VOLUME 2 /* external float32 cost volume (mc-cnn), set by sm_aggregate_cost_f32* */

#define SM_MODE_SGBM 5 /* cv2.STEREO_SGBM_MODE_SGBM: 5 paths (reference default) */
#define SM_MODE_HH 8   /* cv2.STEREO_SGBM_MODE_HH: 8 paths */

/* Field meaning follows cv2.StereoSGBM_create kwargs (reference:
 * stereo_vision/stereo_vision.py:153-163); unnormalised values are accepted
 * and normalised exactly as OpenCV does (P1<=0 -> 2, ...). */
typedef struct sm_params {
    int min_disparity;
    int num_disparities; /* > 0, multiple of 16 (OpenCV asserts this); cost volumes: any 1..256 */
    int block_size;      /* SADWindowSize; <= 0 -> 5 */
    int P1, P2;
    int disp12_max_diff;
    int uniqueness_ratio;
    int pre_filter_cap;
    int speckle_window_size; /* > 0: cv::filterSpeckles after the median (maxSpeckleSize) */
    int speckle_range;
    int cost_kind; /* SM_COST_* */
    int mode;      /* SM_MODE_SGBM | SM_MODE_HH */
} sm_params;

typedef struct sm_ctx sm_ctx;

/* Create a context bound to HIP device `device` (its own non-blocking stream). */
int sm_create(int device, sm_ctx** out);
void sm_destroy(sm_ctx* ctx);

/* Enqueue on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL means the device's default (null) stream. */
int sm_set_stream(sm_ctx* ctx, void* hip_stream);
/* Go back to the context's own non-blocking stream. */
int sm_reset_stream(sm_ctx* ctx);

/* StereoSGBM::compute(left, right) on host buffers (uint8, row stride in
 * bytes >= W).  disp_out: int16[H*W], disparity x16, invalid = (minD-1)*16.
 * Replaces stereo_vision/stereo_vision.py:178 (and :179 with the right
 * matcher's params, see sm_right_matcher_params).
 * wta_out (nullable): int16[H*W] raw integer WTA index, i.e. OpenCV's
 * bestDisp in [0, numDisparities) for pixels in [minX1, maxX1) that pass the
 * uniqueness test (and whose aggregated cost is not saturated), -1 elsewhere;
 * taken before the sub-pixel step, the disp12MaxDiff check and the median. */
int sm_compute(sm_ctx* ctx, const uint8_t* left, const uint8_t* right, int H, int W, int stride,
               const sm_params* p, int16_t* disp_out, int16_t* wta_out);

/* Same on device pointers already resident in HBM; enqueued on the context
 * stream, returns before completion. */
int sm_compute_device(sm_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right, int H, int W,
                      int stride, const sm_params* p, int16_t* d_disp_out);

/* Batch of npairs same-size pairs on device pointers: pair i reads
 * d_left + i*pair_stride_bytes (same for right) and writes
 * d_disp_out + i*H*W.  Asynchronous on the context stream.  Pairs are
 * processed in launch groups (several pairs per kernel launch) so that one
 * pair's serial horizontal paths overlap other pairs' work. */
int sm_compute_batch_device(sm_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right, int npairs,
                            size_t pair_stride_bytes, int H, int W, int stride, const sm_params* p,
                            int16_t* d_disp_out);

/* sm_compute_batch_device plus the integer WTA index of every pair (as sm_compute's
 * wta_out) at d_wta_out + i*H*W (int16; may be NULL).  Gray images. */
int sm_compute_wta_batch_device(sm_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right, int npairs,
                                size_t pair_stride_bytes, int H, int W, int stride, const sm_params* p,
                                int16_t* d_disp_out, int16_t* d_wta_out);

/* The same two entry points for cn-channel images (OpenCV's StereoSGBM takes
 * gray or BGR; the reference's try_try.py:56-57,81 passes cv2.imread BGR
 * images): channels = 1 or 3 interleaved bytes per pixel, stride in bytes
 * (>= W*channels), pair_stride in bytes.  BGR input and configurations whose
 * sums can reach 2^15 (blockSize > 11, large preFilterCap / P2: e.g.
 * disparity_test.py:165-177) run OpenCV's x86 int16 arithmetic exactly
 * (sm_wide.hpp); the rest take the fast kernels.  blockSize <= 55,
 * preFilterCap <= 126. */
int sm_compute_cn(sm_ctx* ctx, const uint8_t* left, const uint8_t* right, int H, int W, int stride, int channels,
                  const sm_params* p, int16_t* disp_out);
int sm_compute_batch_device_cn(sm_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right, int npairs,
                               size_t pair_stride, int H, int W, int stride, int channels, const sm_params* p,
                               int16_t* d_out);

/* SGM over an external matching-cost volume (mc-cnn; the reference memmaps
 * one as float32 (1, D, H, W) at mapTo3D_mc_cnn.py:71 and feeds its
 * disparities to the WLS filter, :81-100).  cost: float32 [D][H][W], d-major,
 * plane d = cost of left x against right x - (min_disparity + d); D must equal
 * p->num_disparities, any value in 1..256 (OpenCV's multiple-of-16 rule is
 * StereoSGBM's own; mc-cnn's -disp_max 228 volume has 228 planes: the kernels
 * run the next multiple of 16 with pad planes that never win).
 * Costs are quantised q = rint((c + offset) * scale)
 * (float32), clamped to [0, 4095], NaN -> 4095 (counted: SM_COUNTER_VOLUME_CLAMPED /
 * SM_COUNTER_VOLUME_NAN).  scale == 0 (or NaN) derives the window per pair on the device
 * from the volume itself: offset = -min, scale = 4095 / (max - min) (float32, IEEE division)
 * over the finite costs of the quantised cells (planes < D, columns [minX1, maxX1)), so no
 * finite cost is clamped; offset is then ignored (no finite cost: 0 and 1).  P1 / P2 are in
 * the quantised units.  The result is then aggregated with the
 * path recurrence / WTA / uniqueness / sub-pixel / LR / median of
 * sm_compute (p->mode paths; block_size and pre_filter_cap unused;
 * P2 <= 12288).  Output as sm_compute.  Host version is synchronous. */
int sm_aggregate_cost_f32(sm_ctx* ctx, const float* cost, int D, int H, int W, const sm_params* p, float offset,
                          float scale, int16_t* disp_out);
/* Batch on device pointers: pair i's volume at d_cost + i*pair_stride_elems
 * (elements, >= D*H*W), output d_disp_out + i*H*W.  Asynchronous. */
int sm_aggregate_cost_f32_device(sm_ctx* ctx, const float* d_cost, int npairs, size_t pair_stride_elems, int D,
                                 int H, int W, const sm_params* p, float offset, float scale, int16_t* d_disp_out);

/* ---- WLS post-filter: cv2.ximgproc.createDisparityWLSFilter(left_matcher)
 * + setLambda/setSigmaColor + filter(displ, gray_l, None, dispr)
 * (reference: stereo_vision/stereo_vision.py:172-175,182).  Fields mirror
 * DisparityWLSFilter's setters / the filter's construction parameters. */
typedef struct sm_wls_params {
    double lambda;                  /* setLambda (default 8000; settings.ini lmbda 80000) */
    double sigma_color;             /* setSigmaColor (default 1.0; settings.ini sigma 1.2) */
    int lrc_thresh;                 /* setLRCthresh (24, in 1/16 px) */
    int depth_discontinuity_radius; /* setDepthDiscontinuityRadius (ceil(0.5*blockSize) for SGBM) */
    int use_confidence;             /* 1: LR-confidence WLS (needs dispr); 0: plain FGS (Generic(false)) */
    int min_disp;                   /* fill outside the ROI: 16*(min_disp-1) */
    int left_offset, right_offset, top_offset, bottom_offset; /* valid ROI of the left map */
    int num_iter;                   /* fast global smoother iterations (3) */
    float lambda_attenuation;       /* per-iteration lambda factor (0.25) */
    float roll_off;                 /* depth-discontinuity roll-off (0.001) */
} sm_wls_params;

/* The filter createDisparityWLSFilter(matcher with params `left`) builds. */
int sm_wls_default_params(const sm_params* left, sm_wls_params* out);

/* DisparityWLSFilter::filter on host buffers: displ/dispr int16[H*W] x16
 * (dispr may be NULL when !use_confidence), guide = left gray view uint8
 * (row stride guide_stride).  out int16[H*W].  Synchronous. */
int sm_wls_filter(sm_ctx* ctx, const int16_t* displ, const int16_t* dispr, const uint8_t* guide, int guide_stride,
                  int H, int W, const sm_wls_params* p, int16_t* out);
/* Batch on device pointers (maps at +i*H*W, guides at +i*guide_pair_stride). */
int sm_wls_filter_batch_device(sm_ctx* ctx, const int16_t* d_displ, const int16_t* d_dispr, const uint8_t* d_guide,
                               int npairs, size_t guide_pair_stride, int guide_stride, int H, int W,
                               const sm_wls_params* p, int16_t* d_out);

/* compute_disparity (stereo_vision/stereo_vision.py:132-184) in one call:
 * `left` = the matcher as created from the settings (:153-163); the
 * createDisparityWLSFilter mutation (uniqueness 0, disp12MaxDiff 1e6,
 * speckle 0) is applied to it, the right matcher is derived as
 * createRightMatcher does and runs on the swapped pair, and `wls` (see
 * sm_wls_default_params, then lambda/sigma from the settings) filters.
 * Outputs displ and filtered int16[H*W] x16.  Synchronous. */
int sm_compute_disparity(sm_ctx* ctx, const uint8_t* left_img, const uint8_t* right_img, int H, int W, int stride,
                         const sm_params* left, const sm_wls_params* wls, int16_t* displ, int16_t* filtered);
/* Same over a device batch (pair i at +i*pair_stride bytes; maps at +i*H*W;
 * d_dispr receives the right matcher's maps). Asynchronous. */
int sm_compute_disparity_batch_device(sm_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right, int npairs,
                                      size_t pair_stride, int H, int W, int stride, const sm_params* left,
                                      const sm_wls_params* wls, int16_t* d_displ, int16_t* d_dispr,
                                      int16_t* d_filtered);

/* cv::filterSpeckles(img, newVal, maxSpeckleSize, maxDiff) in place on an
 * int16 map (what StereoSGBM::compute applies when speckleWindowSize > 0,
 * with newVal = 16*(minD-1), maxDiff = 16*speckleRange).  Host version is
 * synchronous; the device version filters nimg maps at d_img + i*H*W. */
int sm_filter_speckles(sm_ctx* ctx, int16_t* img, int H, int W, int new_val, int max_speckle_size, int max_diff);
int sm_filter_speckles_device(sm_ctx* ctx, int16_t* d_img, int nimg, int H, int W, int new_val,
                              int max_speckle_size, int max_diff);

/* cv::reprojectImageTo3D(disparity, Q, handleMissingValues, CV_32F): the
 * reference reprojects the filtered int16 map (disparity_calculation.py:302;
 * mapTo3D_mc_cnn.py:124 with float32) — xyz out float32 [H][W][3].
 * Q: 4x4 row-major float64.  Host version synchronous; the device version
 * handles nimg maps (disp + i*H*W, xyz + i*H*W*3). */
#define SM_DISP_S16 0
#define SM_DISP_F32 1
int sm_reproject_image_to_3d(sm_ctx* ctx, const void* disp, int disp_type, int H, int W, const double* Q,
                             int handle_missing, float* xyz);
int sm_reproject_image_to_3d_device(sm_ctx* ctx, const void* d_disp, int disp_type, int nimg, int H, int W,
                                    const double* Q, int handle_missing, float* d_xyz);

/* ---- StereoBM (the reference's method="BM" branch,
 * stereo_vision/stereo_vision.py:164-166: cv2.StereoBM_create(numDisparities,
 * blockSize)).  Fields follow cv::StereoBM's setters. */
typedef struct sm_bm_params {
    int min_disparity;
    int num_disparities;   /* > 0, multiple of 16 */
    int block_size;        /* SADWindowSize: odd, 5..255, < min(H, W) */
    int pre_filter_type;   /* 1 = PREFILTER_XSOBEL (default); 0 = NORMALIZED_RESPONSE (SM_E_UNSUPPORTED) */
    int pre_filter_size;   /* odd 5..255 (used by NORMALIZED_RESPONSE only) */
    int pre_filter_cap;    /* 1..63 (31) */
    int texture_threshold; /* 10 */
    int uniqueness_ratio;  /* 15 */
    int speckle_window_size;
    int speckle_range;     /* in disparity x16 units, as cv::StereoBM */
    int disp12_max_diff;   /* < 0: no left-right check (default -1) */
} sm_bm_params;

/* cv2.StereoBM_create(numDisparities, blockSize) defaults. */
int sm_bm_default_params(int num_disparities, int block_size, sm_bm_params* out);
/* ximgproc::createRightMatcher(StereoBM). */
int sm_bm_right_matcher_params(const sm_bm_params* left, sm_bm_params* right_out);
/* StereoBM::compute on host buffers (synchronous) / a device batch (asynchronous;
 * pair i at +i*pair_stride_bytes, output at +i*H*W).  int16 disparity x16,
 * invalid = 16*(minDisparity-1). */
int sm_bm_compute(sm_ctx* ctx, const uint8_t* left, const uint8_t* right, int H, int W, int stride,
                  const sm_bm_params* p, int16_t* disp_out);
int sm_bm_compute_batch_device(sm_ctx* ctx, const uint8_t* d_left, const uint8_t* d_right, int npairs,
                               size_t pair_stride_bytes, int H, int W, int stride, const sm_bm_params* p,
                               int16_t* d_disp_out);

/* Multi-device batch from ONE process (SURVEY §8b sm_compute_batch): ctxs[k]
 * (one per device) computes the contiguous shard [k*npairs/ngpu,
 * (k+1)*npairs/ngpu) of the host pairs left[i]/right[i] (uint8 H x W,
 * C-contiguous) into out + i*H*W (host).  One host thread per context;
 * synchronous.  The scaling path the benchmark uses is one process per GPU
 * (torch.distributed / RCCL); this is the single-process convenience. */
int sm_compute_batch(sm_ctx** ctxs, int ngpu, const uint8_t* const* left, const uint8_t* const* right, int npairs,
                     int H, int W, const sm_params* p, int16_t* out);

/* ximgproc::createRightMatcher(StereoSGBM) parameter derivation
 * (reference call: stereo_vision/stereo_vision.py:171). */
int sm_right_matcher_params(const sm_params* left, sm_params* right_out);

/* Wait for all work enqueued on the context stream.  The fused-sweep engine's
 * strips wait on their neighbours; when one gives up (its neighbours could not
 * be resident, e.g. other work held the CUs), the launch group is recomputed on
 * the device by the per-direction engine, so results stay exact and the call
 * succeeds (counted by sm_get_counters).  Only the opt-in hybrid engine reports
 * such a give-up as SM_E_HIP here (and synchronous entry points check it). */
int sm_synchronize(sm_ctx* ctx);

/* Counters since sm_create: launch groups the fused sweeps handed to the
 * guarded per-direction fallback.  Synchronises the context stream. */
int sm_get_counters(sm_ctx* ctx, long long* sweep_fallbacks);

/* One counter since sm_create (synchronises the context's streams):
 *   SM_COUNTER_SWEEP_FALLBACKS  launch groups the guarded per-direction fallback recomputed;
 *   SM_COUNTER_EW_REPAIRS       E/W strip segments of the in-sweep lines whose speculative
 *                               start state differed from the true one and that the patch
 *                               pass recomputed (results stay exact; a measure of the
 *                               speculation);
 *   SM_COUNTER_VOLUME_CLAMPED   external cost-volume cells (sm_aggregate_cost_f32*) whose
 *                               quantised value fell outside [0, 4095] and was clamped;
 *   SM_COUNTER_VOLUME_NAN       external cost-volume cells that were NaN (cost 4095);
 *   SM_COUNTER_LINE_GROUPS      launch groups whose horizontal paths ran inside the down
 *                               sweep (host-side count of the engine's choice);
 *   SM_COUNTER_EW_OPEN          of the EW_REPAIRS segments, those whose recomputed values had
 *                               not met the speculative ones by the strip's far end (the true
 *                               state was carried into the next strip);
 *   SM_COUNTER_BAND_REPAIRS     vertical (S / SE / SW) chains of the row-band engine (5 paths,
 *                               one or two pairs per launch group) whose speculative state
 *                               entering a band differed from the true one and that the band
 *                               patch recomputed;
 *   SM_COUNTER_BAND_OPEN        of those, chains whose repair walk had not met the speculative
 *                               trajectory by the band's last row (it continued into the next
 *                               band);
 *   SM_COUNTER_BAND_GROUPS      launch groups that ran with row bands (host-side count);
 *   SM_COUNTER_LINE_STRIPS      sweep strips x pairs of the LINE_GROUPS launch groups (host-side:
 *                               divided by the pairs, the strips per pair, whose boundary states
 *                               the patch pass reads). */
#define SM_COUNTER_SWEEP_FALLBACKS 0
#define SM_COUNTER_EW_REPAIRS 1
#define SM_COUNTER_VOLUME_CLAMPED 2
#define SM_COUNTER_VOLUME_NAN 3
#define SM_COUNTER_LINE_GROUPS 4
#define SM_COUNTER_EW_OPEN 5
#define SM_COUNTER_BAND_REPAIRS 6
#define SM_COUNTER_BAND_OPEN 7
#define SM_COUNTER_BAND_GROUPS 8
#define SM_COUNTER_LINE_STRIPS 9
int sm_get_counter(sm_ctx* ctx, int which, long long* value);

/* Restrict the context's own streams (the default stream and its internal
 * second stream) to a CU subset: mask = nwords 32-bit words, bit i = CU i
 * (hipExtStreamCreateWithCUMask); nwords = 0 restores unmasked streams.  The
 * fused sweeps size their co-resident launches from the CUs the stream can
 * reach.  Waits for queued work; resets sm_set_stream to the own stream. */
int sm_set_cu_mask(sm_ctx* ctx, const uint32_t* mask, int nwords);

/* Per-stage device timing with hipEvents on the context stream.
 * stage: 0 cost, 1 path aggregation, 2 WTA+LR, 3 median, 4 whole matcher
 * call, 5 WLS filter (confidence + smoother + final), 6 speckle filter.
 * total_ms: summed duration; launches: timed launches; pairs: pairs they covered. */
#define SM_STAGE_COST 0
#define SM_STAGE_PATHS 1
#define SM_STAGE_WTA 2
#define SM_STAGE_MEDIAN 3
#define SM_STAGE_TOTAL 4
#define SM_STAGE_WLS 5
#define SM_STAGE_SPECKLE 6
/* fused-sweep engine kernels (inside stages 1 and 2): E/W volumes, the
 * first (down) sweep writing the partial sums, the sweep fused with the WTA */
#define SM_STAGE_HORIZONTAL 7
#define SM_STAGE_SWEEP 8
#define SM_STAGE_SWEEP_WTA 9
/* host-pointer entry points: host->device copies of the images, device->host
 * copies of the maps (kept out of every other stage) */
#define SM_STAGE_H2D 10
#define SM_STAGE_D2H 11
/* guarded per-direction recomputation after the fused sweeps (near zero unless a
 * sweep strip gave up waiting for its neighbours; see sm_get_counters) */
#define SM_STAGE_FALLBACK 12
/* one whole compute_disparity call (sm_compute_disparity[_batch_device]): fork of the
 * right matcher, both matchers, join, WLS, on the caller's stream; the two matchers
 * run concurrently, so this (not the sum of their stages) is the call's device time */
#define SM_STAGE_CALL 13
#define SM_NUM_STAGES 14
/* enable: 0 off, 1 every stage, SM_TIMING_ONLY | (1 << stage) | ... only those
 * stages.  Every timed stage records two hipEvents per launch on its stream,
 * which delays the stream (KITTI census8, 8 pairs per call: every stage timed
 * costs about 12 us per pair of wall time), so a throughput measurement times
 * only the stages it reports. */
#define SM_TIMING_ONLY 0x40000000
int sm_set_timing(sm_ctx* ctx, int enable);
int sm_get_timing(sm_ctx* ctx, int stage, double* total_ms, long long* launches, long long* pairs);
int sm_reset_timing(sm_ctx* ctx);

/* Debug / parity: copy an intermediate of the LAST pair computed to host.
 * what: 0 cost volume C[H][width1][D] (uint8 census / uint16 SGBM, volume),
 *       1 path volumes L[P][H][width1][D] (uint8 census / uint16 SGBM),
 *         direction order E, W, SE, S, SW, NE, N, NW,
 *       2 pre-median disparity int16[H][W],
 *       3 census images uint64[2][H][W] (census mode).
 * Returns the byte size when host == NULL. */
long long sm_debug_fetch(sm_ctx* ctx, int what, void* host, size_t bytes);

/* Engine selection for measurements and parity debugging; every flag below gives
 * the same disparities as 0 (normal operation):
 *   4096     per-direction engine (one path volume per direction + WTA kernel), so
 *            sm_debug_fetch(1) returns every direction;
 *   16384    the fused sweeps wherever their preconditions hold (by default launch
 *            groups below 7 census / 3 other pairs run per-direction);
 *   8192     one pair per fused-sweep launch;  1 << 19 narrow sweep strips only;
 *   1 << 21  wide sweep strips wherever built;  256 the sweeps' E/W volumes from the
 *            per-direction engine's row lines;
 *   1 << 23  flag every sweep group as given up (the guarded fallback recomputes it);
 *   64       WTA + median on a second stream, overlapped with the next launch group;
 *   8, 512   16-lane vertical / 64-lane horizontal lines in the per-direction engine;
 *   1024, 2048  census Hamming costs on the fly (all / horizontal directions);
 *   1 << 22  tiled SGBM cost kernel;  bits 16-18 launch-group size cap;
 *   1 << 30  no Infinity-Cache-sized launch groups for the per-direction engine;
 *   1 << 20  sm_compute_disparity*: the right matcher beside the left one on the twin
 *            context's stream (default: before it, on the caller's stream).
 * The measured ablations (row-WTA kernel 16/32, k_sweep2 128 / 1 << 27, hybrid engine
 * 32768) and the timing switches whose results are wrong (1, 2, 4, 1 << 24..26,
 * 1 << 28, 1 << 29, 1 << 31) exist only in the ablation build (make ablation ->
 * libstereo_match_amd_ablate.so); this library returns SM_E_UNSUPPORTED for them. */
int sm_set_debug_flags(sm_ctx* ctx, int flags);

/* Launch-shape knobs for measurements (every value gives the same disparities):
 *   SM_TUNE_EW_LANES   lanes per line of the fused-sweep engine's E/W kernel:
 *                      0 automatic (32 where D % 64 == 0, 16 where D % 32 == 0), 8 / 16 /
 *                      32 / 64 the packed line kernel with that many lanes (where built
 *                      for D), -1 the per-direction engine's 16-lane row lines;
 *   SM_TUNE_SWEEP_NCW  compute waves per fused-sweep strip: 0 automatic (modelled per
 *                      launch), else 5 (latency strips), 7 (narrow) or the wide
 *                      instance's count where built; unbuilt counts fail the call.
 *   SM_TUNE_EW_WAVES   waves per workgroup of the packed E/W lines: 0 automatic, 1..4.
 *   SM_TUNE_EW_PRIO    issue priority (s_setprio 0..3) of the packed E/W lines' waves.
 *   SM_TUNE_EW_WARMUP  columns each in-sweep E/W strip segment runs before its strip
 *                      (0 automatic: 16; 54 for u16 costs in row bands; 1..4096; rounded up
 *                      to the line loop's load chunk).  Any value is exact (the patch pass
 *                      repairs segments that started wrong); large values cost line work.
 *   SM_TUNE_EW_GUESS   0 the segments start from the zero state; 1 (tests) from a
 *                      deliberately wrong state, so that nearly every segment is repaired.
 *   SM_TUNE_SWEEP_LINES the fused-sweep engine's horizontal paths: 0 automatic (inside the
 *                      down sweep wherever that instance is built), 1 the same, -1 the E/W
 *                      volume kernel (k_ew) before / beside the sweeps.
 *   SM_TUNE_BANDS      row bands of the 5-path lines engine: 0 automatic (enough bands to
 *                      occupy the CUs at one or two pairs per launch group), 1 none, 2..H that
 *                      many (speculative vertical paths patched at the band boundaries,
 *                      exact for any value).
 *   SM_TUNE_BAND_WARMUP rows each band's vertical paths run above it (0 automatic: 16 census,
 *                      24 u16 costs; 1..4096).  Any value is exact.
 *   SM_TUNE_BAND_GUESS 0 the bands start from the zero state; 1 (tests) from a deliberately
 *                      wrong state inside the domain, so that nearly every chain is repaired.
 *   SM_TUNE_COST_WGS   workgroups the SGBM cost kernel aims for per launch (0 automatic:
 *                      2048; its row bands are sized from it).
 *   SM_TUNE_SWEEP_XCD  fused sweeps: 1 place each XCD's workgroups on a run of adjacent strips
 *                      (their cost rows shared in its L2), 0 / -1 the plain grid order.
 *   SM_TUNE_LR_STAGGER sm_compute_disparity*: 0 automatic / 1 the left matcher starts on a
 *                      second stream once the right one's down sweep is done (overlapping its
 *                      patch passes and WTA); -1 the matchers strictly one after the other.
 * Returns SM_E_ARG for an unknown key or value. */
#define SM_TUNE_EW_LANES 1
#define SM_TUNE_SWEEP_NCW 2
#define SM_TUNE_EW_WAVES 3
#define SM_TUNE_EW_PRIO 4
#define SM_TUNE_EW_WARMUP 5
#define SM_TUNE_SWEEP_LINES 6
#define SM_TUNE_EW_GUESS 7
#define SM_TUNE_BANDS 8
#define SM_TUNE_BAND_WARMUP 9
#define SM_TUNE_BAND_GUESS 10
#define SM_TUNE_COST_WGS 11
#define SM_TUNE_LR_STAGGER 12
#define SM_TUNE_SWEEP_XCD 13
int sm_set_tuning(sm_ctx* ctx, int key, int value);

/* Last error text of ctx (or of the calling thread when ctx == NULL). */
const char* sm_last_error(sm_ctx* ctx);

/* Library version string. */
const char* sm_version(void);
/* SM_ABI_VERSION the library was built with. */
int sm_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* STEREO_MATCH_AMD_H */
