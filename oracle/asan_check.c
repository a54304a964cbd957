/* asan_check.c: runs the C restatement (sgm_ref.c) under AddressSanitizer and
 * UndefinedBehaviorSanitizer over a sweep of small shapes, including the edge
 * cases the parity tests use: images narrower than the disparity range, one-row
 * images, negative minDisparity, blockSize up to 23, BGR input, both cost kinds,
 * 5 and 8 paths, speckle filtering and the f32 volume entry.
 * TEST INFRASTRUCTURE ONLY (built by `make -C oracle asan`, run by
 * tests/test_oracle_asan.py); nothing in stereo_match_amd/ links it. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int min_disparity, num_disparities, block_size, P1, P2;
    int disp12_max_diff, uniqueness_ratio, pre_filter_cap;
    int speckle_window_size, speckle_range;
    int cost_kind;
    int npaths;
} sgm_ref_params;

int sgm_ref_compute_cn(const uint8_t* img1, const uint8_t* img2, int H, int W, int stride, int cn,
                       const sgm_ref_params* prm, int16_t* disp1, int apply_median);
int sgm_ref_compute_volume(const float* vol, int H, int W, const sgm_ref_params* prm, float offset, float scale,
                           int16_t* disp1, int apply_median);
void sgm_ref_filter_speckles(int16_t* img, int H, int W, int newVal, int maxSpeckleSize, int maxDiff);

static uint32_t rng = 12345u;
static uint32_t next(void)
{
    rng ^= rng << 13;
    rng ^= rng >> 17;
    rng ^= rng << 5;
    return rng;
}

int main(void)
{
    static const int shapes[][2] = {{1, 40}, {7, 9}, {16, 48}, {23, 70}, {33, 101}};
    static const int disps[] = {16, 32, 64};
    static const int mins[] = {0, -5, 3};
    static const int blocks[] = {1, 3, 5, 11, 23};
    int runs = 0;
    for (size_t s = 0; s < sizeof(shapes) / sizeof(shapes[0]); s++) {
        const int H = shapes[s][0], W = shapes[s][1];
        for (int cn = 1; cn <= 3; cn += 2) {
            const int stride = W * cn + 3; /* padded rows */
            uint8_t* a = malloc((size_t)H * stride);
            uint8_t* b = malloc((size_t)H * stride);
            int16_t* d = malloc((size_t)H * W * sizeof(int16_t));
            for (int i = 0; i < H * stride; i++) {
                a[i] = (uint8_t)next();
                b[i] = (uint8_t)next();
            }
            for (size_t k = 0; k < sizeof(disps) / sizeof(disps[0]); k++)
                for (size_t m = 0; m < sizeof(mins) / sizeof(mins[0]); m++)
                    for (size_t q = 0; q < sizeof(blocks) / sizeof(blocks[0]); q++)
                        for (int kind = 0; kind < 2; kind++)
                            for (int np = 5; np <= 8; np += 3) {
                                if (kind == 1 && cn != 1) continue; /* census is gray only */
                                const int bs = blocks[q];
                                sgm_ref_params p = {mins[m], disps[k], bs, 8 * bs * bs, 32 * bs * bs,
                                                    (int)(next() % 3), (int)(next() % 16), 1 + (int)(next() % 63),
                                                    (int)(next() % 2) * 20, 2, kind, np};
                                if (p.P2 <= p.P1) p.P2 = p.P1 + 1;
                                if (sgm_ref_compute_cn(a, b, H, W, stride, cn, &p, d, 1) < 0) {
                                    fprintf(stderr, "compute failed H=%d W=%d cn=%d\n", H, W, cn);
                                    return 1;
                                }
                                if (p.speckle_window_size) sgm_ref_filter_speckles(d, H, W, -16, 20, 32);
                                runs++;
                            }
            free(a);
            free(b);
            free(d);
        }
        /* f32 d-major volume entry (mc-cnn) */
        const int D = 16;
        float* vol = malloc((size_t)D * H * W * sizeof(float));
        int16_t* d = malloc((size_t)H * W * sizeof(int16_t));
        for (int i = 0; i < D * H * W; i++) vol[i] = (float)(next() % 1000) / 100.f;
        sgm_ref_params p = {0, D, 1, 10, 120, 1, 5, 0, 0, 0, 0, 8};
        if (sgm_ref_compute_volume(vol, H, W, &p, 0.f, 16.f, d, 1) < 0) {
            fprintf(stderr, "volume failed H=%d W=%d\n", H, W);
            return 1;
        }
        runs++;
        free(vol);
        free(d);
    }
    printf("asan_check ok: %d runs\n", runs);
    return 0;
}
