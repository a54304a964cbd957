/*
 * sgm_ref.c — CPU restatement of the stereo_match hot path.
 * TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py, never by the product path.
 *
 * PARITY STATUS: parity unpinned (OpenCV, which holds the reference's
 * arithmetic, is absent from this image and the reference ships no vectors —
 * see oracle/sgm_np.py header and DESIGN.md §3).
 *
 * This file deliberately follows the LOOP STRUCTURE of upstream OpenCV
 * computeDisparitySGBM (modules/calib3d/src/stereosgbm.cpp, the routine the
 * reference reaches through cv2.StereoSGBM_create(...).compute at
 * stereo_vision/stereo_vision.py:153,178): per-row calcPixelCostBT, a
 * ring of blockSize horizontal sums with an incremental vertical update
 * (Cbuf seeded with P2), one top-down pass computing r0..r3 into two
 * cyclic Lr/minLr row buffers, the backward horizontal r4 fused with WTA
 * (MODE_SGBM), or a second bottom-up pass (MODE_HH / 8 paths), followed by
 * disp2 + the disp12MaxDiff check, then medianBlur(3).  oracle/sgm_np.py
 * restates the same maths direction-by-direction in closed form; the two
 * must agree bit for bit (tests/test_oracle_kats.py).
 *
 * The census cost (north-star mode, no reference counterpart) feeds the same
 * row engine: C(x,y,d) = popcount(census_l ^ census_r) (+P2 seed).
 *
 * Arithmetic follows OpenCV's x86 build, where hasSIMD128() is true and the
 * CV_SIMD128 branches run (SSE2; OpenCV 3.x universal intrinsics, whose int16
 * + and - saturate): the incremental box-sum update of C for y > 0, every
 * L_r step and the S sums saturate to int16 (sat16), the delta = minLr + P2
 * broadcast is a (short) cast (wrap16), and MODE_SGBM's winner is chosen
 * per 8 x int16 lane (see the WTA below).  Row y == 0 of C and the x == 0
 * horizontal sums run the scalar loops (int16 casts: wrap16).  Inside the
 * int16-exact range the GPU's fast kernels cover (no sum can reach 2^15),
 * saturating and plain arithmetic agree; outside it (large blockSize,
 * preFilterCap, P2, colour input) these rules decide.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

typedef int16_t CostType;
#define MAX_COST 32767
#define DISP_SHIFT 4
#define DISP_SCALE 16

typedef struct {
    int min_disparity, num_disparities, block_size, P1, P2;
    int disp12_max_diff, uniqueness_ratio, pre_filter_cap;
    int speckle_window_size, speckle_range;
    int cost_kind; /* 0 = SGBM (BT + box), 1 = census 9x7 */
    int npaths;    /* 5 = MODE_SGBM, 8 = MODE_HH */
} sgm_ref_params;

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int sat16(int v) { return v > 32767 ? 32767 : (v < -32768 ? -32768 : v); }
static inline int wrap16(int v) { return (int)(int16_t)(uint16_t)(unsigned)v; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int iabs(int a) { return a < 0 ? -a : a; }

/* ---------------------------------------------------------------- census */
void sgm_ref_census9x7(const uint8_t* img, int H, int W, int stride, uint64_t* out)
{
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            int c = img[y * stride + x];
            uint64_t v = 0;
            int k = 0;
            for (int dy = -3; dy <= 3; dy++)
                for (int dx = -4; dx <= 4; dx++) {
                    if (!dy && !dx) continue;
                    int yy = imin(imax(y + dy, 0), H - 1), xx = imin(imax(x + dx, 0), W - 1);
                    if (img[yy * stride + xx] < c) v |= (uint64_t)1 << k;
                    k++;
                }
            out[(size_t)y * W + x] = v;
        }
}

/* ------------------------------------------------------ calcPixelCostBT */
/* cost[x1*D + d] for x1 in [0,width1): BT(left x1+minX1, right x1+minX1-minD-d)
 * summed over 2*cn channels: the clipped x-derivative of each colour channel
 * (shift 0), then each raw channel (shift 2).  Rows hold cn interleaved bytes
 * per pixel (cn = 1 gray, 3 BGR), stride in bytes. */
static void calc_pixel_cost_bt(const uint8_t* img1, const uint8_t* img2, int stride, int cn,
                               int H, int W, int y, int minD, int maxD,
                               CostType* cost, uint8_t* tmp, const uint8_t* tab)
{
    int minX1 = imax(maxD, 0), maxX1 = W + imin(minD, 0);
    int D = maxD - minD, width1 = maxX1 - minX1;
    const uint8_t* row1 = img1 + (size_t)y * stride;
    const uint8_t* row2 = img2 + (size_t)y * stride;
    int n = y > 0 ? -stride : 0, s = y < H - 1 ? stride : 0;
    /* prow1[c][x] (left), prow2[c][W-1-x] (right, reversed like OpenCV) */
    uint8_t* prow1 = tmp;
    uint8_t* prow2 = tmp + 2 * cn * W;
    uint8_t* buf0 = tmp + 4 * cn * W; /* v0 */
    uint8_t* buf1 = buf0 + W;         /* v1 */
    for (int c = 0; c < 2 * cn; c++) {
        prow1[W * c] = prow1[W * c + W - 1] = prow2[W * c] = prow2[W * c + W - 1] = tab[0];
    }
    for (int x = 1; x < W - 1; x++)
        for (int ch = 0; ch < cn; ch++) {
            int a = (x + 1) * cn + ch, b = (x - 1) * cn + ch;
            prow1[x + W * ch] = tab[(row1[a] - row1[b]) * 2 + row1[a + n] - row1[b + n] + row1[a + s] - row1[b + s]];
            prow2[W - 1 - x + W * ch] =
                tab[(row2[a] - row2[b]) * 2 + row2[a + n] - row2[b + n] + row2[a + s] - row2[b + s]];
            prow1[x + W * (cn + ch)] = row1[x * cn + ch];
            prow2[W - 1 - x + W * (cn + ch)] = row2[x * cn + ch];
        }
    memset(cost, 0, sizeof(CostType) * (size_t)width1 * D);
    for (int c = 0; c < 2 * cn; c++) {
        const uint8_t* p1 = prow1 + W * c;
        const uint8_t* p2 = prow2 + W * c;
        int diff_scale = c < cn ? 0 : 2;
        for (int x = 0; x < W; x++) {
            int v = p2[x];
            int vl = x > 0 ? (v + p2[x - 1]) / 2 : v;
            int vr = x < W - 1 ? (v + p2[x + 1]) / 2 : v;
            int v0 = imin(imin(vl, vr), v), v1 = imax(imax(vl, vr), v);
            buf0[x] = (uint8_t)v0;
            buf1[x] = (uint8_t)v1;
        }
        for (int x = minX1; x < maxX1; x++) {
            int u = p1[x];
            int ul = x > 0 ? (u + p1[x - 1]) / 2 : u;
            int ur = x < W - 1 ? (u + p1[x + 1]) / 2 : u;
            int u0 = imin(imin(ul, ur), u), u1 = imax(imax(ul, ur), u);
            CostType* cx = cost + (size_t)(x - minX1) * D - minD;
            for (int d = minD; d < maxD; d++) {
                int r = W - x - 1 + d; /* reversed index of right column x-d */
                int v = p2[r], v0 = buf0[r], v1 = buf1[r];
                int c0 = imax(imax(0, u - v1), v0 - u);
                int c1 = imax(imax(0, v - u1), u0 - v);
                cx[d] = (CostType)(cx[d] + (imin(c0, c1) >> diff_scale));
            }
        }
    }
}

/* ------------------------------------------------------------ median 3x3 */
static inline void sort2(int* a, int* b) { if (*a > *b) { int t = *a; *a = *b; *b = t; } }

void sgm_ref_median3(const int16_t* src, int H, int W, int16_t* dst)
{
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            int v[9], k = 0;
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    int yy = imin(imax(y + dy, 0), H - 1), xx = imin(imax(x + dx, 0), W - 1);
                    v[k++] = src[(size_t)yy * W + xx];
                }
            for (int i = 0; i < 9; i++)
                for (int j = 0; j < 8 - i; j++) sort2(&v[j], &v[j + 1]);
            dst[(size_t)y * W + x] = (int16_t)v[4];
        }
}

/* ------------------------------------------------------- speckle filter */
void sgm_ref_filter_speckles(int16_t* img, int H, int W, int newVal, int maxSpeckleSize, int maxDiff)
{
    int npix = H * W;
    int* labels = (int*)calloc((size_t)npix, sizeof(int));
    int* wbuf = (int*)malloc(sizeof(int) * 2 * (size_t)npix + 8);
    uint8_t* rtype = (uint8_t*)calloc((size_t)npix + 1, 1);
    int curlabel = 0;
    for (int i = 0; i < H; i++) {
        int16_t* ds = img + (size_t)i * W;
        int* ls = labels + (size_t)i * W;
        for (int j = 0; j < W; j++) {
            if (ds[j] == newVal) continue;
            if (ls[j]) {
                if (rtype[ls[j]]) ds[j] = (int16_t)newVal;
                continue;
            }
            int top = 0, px = j, py = i, count = 0;
            ls[j] = ++curlabel;
            for (;;) {
                count++;
                int16_t* dpp = img + (size_t)py * W + px;
                int dp = *dpp;
                int* lpp = labels + (size_t)py * W + px;
#define PUSH(cond, off, loff, nx, ny)                                                      \
    if ((cond) && !lpp[loff] && dpp[off] != newVal && iabs(dp - dpp[off]) <= maxDiff) { \
        lpp[loff] = curlabel; wbuf[2 * top] = (nx); wbuf[2 * top + 1] = (ny); top++;     \
    }
                PUSH(py < H - 1, W, W, px, py + 1)
                PUSH(py > 0, -W, -W, px, py - 1)
                PUSH(px < W - 1, 1, 1, px + 1, py)
                PUSH(px > 0, -1, -1, px - 1, py)
#undef PUSH
                if (!top) break;
                top--;
                px = wbuf[2 * top];
                py = wbuf[2 * top + 1];
            }
            if (count <= maxSpeckleSize) { rtype[ls[j]] = 1; ds[j] = (int16_t)newVal; }
            else rtype[ls[j]] = 0;
        }
    }
    free(labels); free(wbuf); free(rtype);
}

/* -------------------------------------------------- computeDisparitySGBM */
#define NR2 4

/* External f32 cost (mc-cnn volume, own definition — see sgm_np.quantize_volume):
 * q = rint((c + offset) * scale) in float32, clamped to [0, 4095], NaN -> 4095. */
#define VOLUME_CMAX 4095
static inline int quant_cost(float c, float offset, float scale)
{
    if (c != c) return VOLUME_CMAX;
    float t = (c + offset) * scale;
    float v = rintf(t);
    if (!(v > 0.f)) return 0;
    if (v > (float)VOLUME_CMAX) return VOLUME_CMAX;
    return (int)v;
}

/* one L_r step of the SIMD loop: L = min(Lp[d], Lp[d-1]+P1, Lp[d+1]+P1, delta);
 * L = (L - delta) + C, every + and - saturating to int16 (Lp[-1] = Lp[D] = MAX_COST) */
static inline int l_step(const CostType* Lp, int d, int P1, int delta, int Cpd)
{
    int v = imin((int)Lp[d], imin(sat16(Lp[d - 1] + P1), sat16(Lp[d + 1] + P1)));
    v = imin(v, delta);
    return sat16(sat16(v - delta) + Cpd);
}

static int compute_core(const uint8_t* img1, const uint8_t* img2, int H, int W, int stride, int cn,
                        const float* vol, float vol_offset, float vol_scale, const sgm_ref_params* prm,
                        int16_t* disp1, int apply_median, int16_t* dumpC, int16_t* wta)
{
    if ((!vol && (!img1 || !img2 || (cn != 1 && cn != 3) || stride < W * cn)) || !disp1 || !prm || H <= 0 ||
        W <= 0)
        return -1;
    int minD = prm->min_disparity, D = prm->num_disparities, maxD = minD + D;
    /* OpenCV's StereoSGBM asserts D % 16 == 0; an external cost volume (mc-cnn: D = 228,
     * mapTo3D_mc_cnn.py:71) has as many planes as it was made with, so D is free there */
    if (D <= 0 || (D % 16 && !vol)) return -1;
    int bs = prm->block_size > 0 ? prm->block_size : 5;
    int ftzero = imax(prm->pre_filter_cap, 15) | 1;
    int uniq = prm->uniqueness_ratio >= 0 ? prm->uniqueness_ratio : 10;
    int disp12 = prm->disp12_max_diff > 0 ? prm->disp12_max_diff : 1;
    int P1 = prm->P1 > 0 ? prm->P1 : 2;
    int P2 = imax(prm->P2 > 0 ? prm->P2 : 5, P1 + 1);
    int census = prm->cost_kind == 1;
    if (vol && P2 > 16383 - VOLUME_CMAX) return -1;
    int minX1 = imax(maxD, 0), maxX1 = W + imin(minD, 0), width1 = maxX1 - minX1;
    int INVALID = (minD - 1) * DISP_SCALE;
    int SW2 = bs / 2, SH2 = bs / 2;
    int fullDP = prm->npaths == 8, npasses = fullDP ? 2 : 1;
    enum { TAB_OFS = 256 * 4, TAB_SIZE = 256 + TAB_OFS * 2 };
    uint8_t clipTab[TAB_SIZE];
    for (int k = 0; k < TAB_SIZE; k++)
        clipTab[k] = (uint8_t)(imin(imax(k - TAB_OFS, -ftzero), ftzero) + ftzero);

    int16_t* out = apply_median ? (int16_t*)malloc(sizeof(int16_t) * (size_t)H * W) : disp1;
    for (size_t i = 0; i < (size_t)H * W; i++) out[i] = (int16_t)INVALID;
    if (wta)
        for (size_t i = 0; i < (size_t)H * W; i++) wta[i] = -1;
    if (minX1 >= maxX1) goto done;

    {
        size_t costBufSize = (size_t)width1 * D;
        size_t CSBufSize = costBufSize * (fullDP ? H : 1);
        int hsumBufNRows = SH2 * 2 + 2;
        int D2 = D + 2, NRD2 = NR2 * D2;
        CostType* Cbuf = (CostType*)malloc(sizeof(CostType) * CSBufSize);
        CostType* Sbuf = (CostType*)malloc(sizeof(CostType) * CSBufSize);
        CostType* hsumBuf = (CostType*)malloc(sizeof(CostType) * costBufSize * hsumBufNRows);
        CostType* pixDiff = (CostType*)malloc(sizeof(CostType) * costBufSize);
        size_t LrSize = (size_t)(width1 + 2) * NRD2, minLrSize = (size_t)(width1 + 2) * NR2;
        CostType* LrMem[2];
        CostType* minLrMem[2];
        for (int k = 0; k < 2; k++) {
            LrMem[k] = (CostType*)malloc(sizeof(CostType) * LrSize);
            minLrMem[k] = (CostType*)malloc(sizeof(CostType) * minLrSize);
        }
        CostType* disp2cost = (CostType*)malloc(sizeof(CostType) * (size_t)W);
        int16_t* disp2 = (int16_t*)malloc(sizeof(int16_t) * (size_t)W);
        uint8_t* tmp = (uint8_t*)malloc((size_t)W * (4 * cn + 2));
        uint64_t *cl = NULL, *cr = NULL;
        if (census) {
            if (cn != 1) return -1;
            cl = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)H * W);
            cr = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)H * W);
            sgm_ref_census9x7(img1, H, W, stride, cl);
            sgm_ref_census9x7(img2, H, W, stride, cr);
        }
        /* "add P2 to every C(x,y). it saves a few operations in the inner loops" */
        for (size_t k = 0; k < CSBufSize; k++) Cbuf[k] = (CostType)P2;

/* Lr slot of column x in [-1,width1], direction r, disparity d in [-1,D] */
#define LR(buf, x, r) ((buf) + ((size_t)((x) + 1) * NR2 + (r)) * D2 + 1)
#define MINLR(buf, x) ((buf) + (size_t)((x) + 1) * NR2)

        for (int pass = 1; pass <= npasses; pass++) {
            int y1, y2, dy, x1, x2, dx;
            if (pass == 1) { y1 = 0; y2 = H; dy = 1; x1 = 0; x2 = width1; dx = 1; }
            else { y1 = H - 1; y2 = -1; dy = -1; x1 = width1 - 1; x2 = -1; dx = -1; }
            CostType* Lr[2] = {LrMem[0], LrMem[1]};
            CostType* minLr[2] = {minLrMem[0], minLrMem[1]};
            for (int k = 0; k < 2; k++) {
                memset(Lr[k], 0, sizeof(CostType) * LrSize);
                memset(minLr[k], 0, sizeof(CostType) * minLrSize);
            }
            for (int y = y1; y != y2; y += dy) {
                CostType* C = Cbuf + (fullDP ? (size_t)y * costBufSize : 0);
                CostType* S = Sbuf + (fullDP ? (size_t)y * costBufSize : 0);
                if (pass == 1) {
                    if (vol) {
                        for (int x = 0; x < width1; x++)
                            for (int d = 0; d < D; d++)
                                C[(size_t)x * D + d] = (CostType)(
                                    P2 + quant_cost(vol[((size_t)d * H + y) * W + x + minX1], vol_offset, vol_scale));
                    } else if (census) {
                        const uint64_t* l = cl + (size_t)y * W;
                        const uint64_t* r = cr + (size_t)y * W;
                        for (int x = 0; x < width1; x++)
                            for (int d = 0; d < D; d++) {
                                int X = x + minX1;
                                C[(size_t)x * D + d] =
                                    (CostType)(P2 + __builtin_popcountll(l[X] ^ r[X - minD - d]));
                            }
                    } else {
                        int dy1 = y == 0 ? 0 : y + SH2, dy2 = y == 0 ? SH2 : dy1;
                        for (int k = dy1; k <= dy2; k++) {
                            CostType* hsumAdd = hsumBuf + (size_t)(imin(k, H - 1) % hsumBufNRows) * costBufSize;
                            if (k < H) {
                                calc_pixel_cost_bt(img1, img2, stride, cn, H, W, k, minD, maxD, pixDiff, tmp,
                                                   clipTab + TAB_OFS);
                                for (int d = 0; d < D; d++) {
                                    int acc = pixDiff[d] * (SW2 + 1);
                                    for (int x = 1; x <= SW2; x++) acc += pixDiff[(size_t)imin(x, width1 - 1) * D + d];
                                    hsumAdd[d] = (CostType)acc;
                                }
                                if (y > 0) {
                                    const CostType* hsumSub =
                                        hsumBuf + (size_t)(imax(y - SH2 - 1, 0) % hsumBufNRows) * costBufSize;
                                    const CostType* Cprev = !fullDP || y == 0 ? C : C - costBufSize;
                                    /* SIMD: v_load(Cprev) + v_load(hsumAdd) - v_load(hsumSub) */
                                    for (int d = 0; d < D; d++)
                                        C[d] = (CostType)sat16(sat16(Cprev[d] + hsumAdd[d]) - hsumSub[d]);
                                    for (size_t x = D; x < costBufSize; x += D) {
                                        const CostType* pixAdd = pixDiff + imin((int)x + SW2 * D, (width1 - 1) * D);
                                        const CostType* pixSub = pixDiff + imax((int)x - (SW2 + 1) * D, 0);
                                        for (int d = 0; d < D; d++) {
                                            /* hv = hv - psub + padd; Cx = Cx - hsumSub + hv (all saturating) */
                                            int hv = hsumAdd[x + d] =
                                                (CostType)sat16(sat16(hsumAdd[x - D + d] - pixSub[d]) + pixAdd[d]);
                                            C[x + d] = (CostType)sat16(sat16(Cprev[x + d] - hsumSub[x + d]) + hv);
                                        }
                                    }
                                } else {
                                    for (size_t x = D; x < costBufSize; x += D) {
                                        const CostType* pixAdd = pixDiff + imin((int)x + SW2 * D, (width1 - 1) * D);
                                        const CostType* pixSub = pixDiff + imax((int)x - (SW2 + 1) * D, 0);
                                        for (int d = 0; d < D; d++)
                                            hsumAdd[x + d] = (CostType)(hsumAdd[x - D + d] + pixAdd[d] - pixSub[d]);
                                    }
                                }
                            }
                            if (y == 0) {
                                int scale = k == 0 ? SH2 + 1 : 1;
                                for (size_t x = 0; x < costBufSize; x++)
                                    C[x] = (CostType)(C[x] + hsumAdd[x] * scale);
                            }
                        }
                    }
                    memset(S, 0, sizeof(CostType) * costBufSize);
                    if (dumpC) /* OpenCV's C row as stored (P2 seed included) */
                        memcpy(dumpC + (size_t)y * costBufSize, C, sizeof(CostType) * costBufSize);
                }

                /* clear the left and right borders of the current Lr row */
                memset(LR(Lr[0], -1, 0) - 1, 0, sizeof(CostType) * NRD2);
                memset(LR(Lr[0], width1, 0) - 1, 0, sizeof(CostType) * NRD2);
                memset(MINLR(minLr[0], -1), 0, sizeof(CostType) * NR2);
                memset(MINLR(minLr[0], width1), 0, sizeof(CostType) * NR2);

                /* r0 = (-dx,0), r1 = (-1,-dy), r2 = (0,-dy), r3 = (1,-dy); the
                 * SIMD broadcast of delta = minLr + P2 is a (short) cast */
                for (int x = x1; x != x2; x += dx) {
                    int delta0 = wrap16(MINLR(minLr[0], x - dx)[0] + P2);
                    int delta1 = wrap16(MINLR(minLr[1], x - 1)[1] + P2);
                    int delta2 = wrap16(MINLR(minLr[1], x)[2] + P2);
                    int delta3 = wrap16(MINLR(minLr[1], x + 1)[3] + P2);
                    CostType* Lr_p0 = LR(Lr[0], x - dx, 0);
                    CostType* Lr_p1 = LR(Lr[1], x - 1, 1);
                    CostType* Lr_p2 = LR(Lr[1], x, 2);
                    CostType* Lr_p3 = LR(Lr[1], x + 1, 3);
                    Lr_p0[-1] = Lr_p0[D] = Lr_p1[-1] = Lr_p1[D] = Lr_p2[-1] = Lr_p2[D] = Lr_p3[-1] =
                        Lr_p3[D] = MAX_COST;
                    const CostType* Cp = C + (size_t)x * D;
                    CostType* Sp = S + (size_t)x * D;
                    int minL0 = MAX_COST, minL1 = MAX_COST, minL2 = MAX_COST, minL3 = MAX_COST;
                    for (int d = 0; d < D; d++) {
                        int Cpd = Cp[d], L0, L1, L2, L3;
                        L0 = l_step(Lr_p0, d, P1, delta0, Cpd);
                        L1 = l_step(Lr_p1, d, P1, delta1, Cpd);
                        L2 = l_step(Lr_p2, d, P1, delta2, Cpd);
                        L3 = l_step(Lr_p3, d, P1, delta3, Cpd);
                        LR(Lr[0], x, 0)[d] = (CostType)L0; minL0 = imin(minL0, L0);
                        LR(Lr[0], x, 1)[d] = (CostType)L1; minL1 = imin(minL1, L1);
                        LR(Lr[0], x, 2)[d] = (CostType)L2; minL2 = imin(minL2, L2);
                        LR(Lr[0], x, 3)[d] = (CostType)L3; minL3 = imin(minL3, L3);
                        /* L0 = L0 + L1; L2 = L2 + L3; Sval = Sval + L0; Sval = Sval + L2 */
                        Sp[d] = (CostType)sat16(sat16(Sp[d] + sat16(L0 + L1)) + sat16(L2 + L3));
                    }
                    CostType* mL = MINLR(minLr[0], x);
                    mL[0] = (CostType)minL0; mL[1] = (CostType)minL1;
                    mL[2] = (CostType)minL2; mL[3] = (CostType)minL3;
                }

                if (pass == npasses) {
                    int16_t* drow = out + (size_t)y * W;
                    for (int x = 0; x < W; x++) {
                        drow[x] = disp2[x] = (int16_t)INVALID;
                        disp2cost[x] = MAX_COST;
                    }
                    for (int x = width1 - 1; x >= 0; x--) {
                        CostType* Sp = S + (size_t)x * D;
                        int minS = MAX_COST, bestDisp = -1, d;
                        if (npasses == 1) {
                            /* CV_SIMD128 branch (x86): lane i keeps the first minimum among
                             * d = i, i+8, ...; the lowest lane holding the overall minimum wins */
                            int laneMin[8], laneBest[8];
                            for (int i = 0; i < 8; i++) { laneMin[i] = MAX_COST; laneBest[i] = -1; }
                            int minL0 = MAX_COST;
                            int delta0 = wrap16(MINLR(minLr[0], x + 1)[0] + P2);
                            CostType* Lr_p0 = LR(Lr[0], x + 1, 0);
                            Lr_p0[-1] = Lr_p0[D] = MAX_COST;
                            CostType* Lr_p = LR(Lr[0], x, 0);
                            const CostType* Cp = C + (size_t)x * D;
                            for (d = 0; d < D; d++) {
                                int L0 = l_step(Lr_p0, d, P1, delta0, Cp[d]);
                                Lr_p[d] = (CostType)L0;
                                minL0 = imin(minL0, L0);
                                int Sval = Sp[d] = (CostType)sat16(L0 + Sp[d]);
                                if (laneMin[d & 7] > Sval) { laneMin[d & 7] = Sval; laneBest[d & 7] = d; }
                            }
                            MINLR(minLr[0], x)[0] = (CostType)minL0;
                            for (int i = 0; i < 8; i++) minS = imin(minS, laneMin[i]);
                            for (int i = 0; i < 8; i++)
                                if (laneMin[i] == minS) { bestDisp = laneBest[i]; break; }
                        } else {
                            for (d = 0; d < D; d++) {
                                int Sval = Sp[d];
                                if (Sval < minS) { minS = Sval; bestDisp = d; }
                            }
                        }
                        for (d = 0; d < D; d++)
                            if (Sp[d] * (100 - uniq) < minS * 100 && iabs(bestDisp - d) > 1) break;
                        if (d < D) continue;
                        d = bestDisp;
                        if (d < 0) continue; /* all S saturated: OpenCV leaves the pixel invalid */
                        if (wta) wta[(size_t)y * W + x + minX1] = (int16_t)d; /* the integer WTA index */
                        int _x2 = x + minX1 - d - minD;
                        if (disp2cost[_x2] > minS) {
                            disp2cost[_x2] = (CostType)minS;
                            disp2[_x2] = (int16_t)(d + minD);
                        }
                        if (0 < d && d < D - 1) {
                            int denom2 = imax(Sp[d - 1] + Sp[d + 1] - 2 * Sp[d], 1);
                            d = d * DISP_SCALE + ((Sp[d - 1] - Sp[d + 1]) * DISP_SCALE + denom2) / (denom2 * 2);
                        } else
                            d *= DISP_SCALE;
                        drow[x + minX1] = (int16_t)(d + minD * DISP_SCALE);
                    }
                    for (int x = minX1; x < maxX1; x++) {
                        int d1 = drow[x];
                        if (d1 == INVALID) continue;
                        int _d = d1 >> DISP_SHIFT;
                        int d_ = (d1 + DISP_SCALE - 1) >> DISP_SHIFT;
                        int _x = x - _d, x_ = x - d_;
                        if (0 <= _x && _x < W && disp2[_x] >= minD && iabs(disp2[_x] - _d) > disp12 &&
                            0 <= x_ && x_ < W && disp2[x_] >= minD && iabs(disp2[x_] - d_) > disp12)
                            drow[x] = (int16_t)INVALID;
                    }
                }
                /* shift the cyclic buffers */
                CostType* t = Lr[0]; Lr[0] = Lr[1]; Lr[1] = t;
                t = minLr[0]; minLr[0] = minLr[1]; minLr[1] = t;
            }
        }
#undef LR
#undef MINLR
        free(Cbuf); free(Sbuf); free(hsumBuf); free(pixDiff);
        for (int k = 0; k < 2; k++) { free(LrMem[k]); free(minLrMem[k]); }
        free(disp2cost); free(disp2); free(tmp); free(cl); free(cr);
    }
done:
    if (apply_median) {
        sgm_ref_median3(out, H, W, disp1);
        free(out);
    }
    if (prm->speckle_window_size > 0)
        sgm_ref_filter_speckles(disp1, H, W, INVALID, prm->speckle_window_size,
                                DISP_SCALE * prm->speckle_range);
    return 0;
}

int sgm_ref_compute(const uint8_t* img1, const uint8_t* img2, int H, int W, int stride,
                    const sgm_ref_params* prm, int16_t* disp1, int apply_median)
{
    return compute_core(img1, img2, H, W, stride, 1, NULL, 0.f, 1.f, prm, disp1, apply_median, NULL, NULL);
}

/* as sgm_ref_compute, plus the integer WTA index wta[H][W] (bestDisp in [0, D) of pixels
 * that pass the uniqueness test and are not saturated, -1 elsewhere; before the sub-pixel
 * step, the disp12MaxDiff check and the median) */
int sgm_ref_compute_wta(const uint8_t* img1, const uint8_t* img2, int H, int W, int stride,
                        const sgm_ref_params* prm, int16_t* disp1, int16_t* wta, int apply_median)
{
    return compute_core(img1, img2, H, W, stride, 1, NULL, 0.f, 1.f, prm, disp1, apply_median, NULL, wta);
}

/* cn-channel input (1 gray, 3 BGR interleaved), stride in bytes */
int sgm_ref_compute_cn(const uint8_t* img1, const uint8_t* img2, int H, int W, int stride, int cn,
                       const sgm_ref_params* prm, int16_t* disp1, int apply_median)
{
    return compute_core(img1, img2, H, W, stride, cn, NULL, 0.f, 1.f, prm, disp1, apply_median, NULL, NULL);
}

/* the cost volume C[H][width1][D] as OpenCV holds it for each row (int16, P2 seed included) */
int sgm_ref_cost_volume_cn(const uint8_t* img1, const uint8_t* img2, int H, int W, int stride, int cn,
                           const sgm_ref_params* prm, int16_t* C, int16_t* disp1)
{
    return compute_core(img1, img2, H, W, stride, cn, NULL, 0.f, 1.f, prm, disp1, 0, C, NULL);
}

/* SGM over an external d-major float32 cost volume vol[D][H][W] (mc-cnn). */
int sgm_ref_compute_volume(const float* vol, int H, int W, const sgm_ref_params* prm, float offset, float scale,
                           int16_t* disp1, int apply_median)
{
    if (!vol) return -1;
    return compute_core(NULL, NULL, H, W, W, 1, vol, offset, scale, prm, disp1, apply_median, NULL, NULL);
}
