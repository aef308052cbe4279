/*
 * oracle_sanitize.c -- host sanitizer run of the C oracle (SURVEY.md §5:
 * "-fsanitize=address build of the CPU restatement").  TEST INFRASTRUCTURE.
 *
 * Built by tests/native/Makefile (target `sanitize`) with
 * -fsanitize=address,undefined -fno-sanitize-recover=all and run by
 * tests/test_oracle_sanitize.py.  Every buffer is malloc'ed to its exact
 * size, so an out-of-bounds read or write of any oracle function -- the
 * sampler's corner reads at the row edges, the backward's scatter, the
 * pooling's floor widths -- aborts the run.  Inputs: odd widths, 1-5
 * levels, radius 1..4, and the coordinates the reference's own tests and
 * the GPU parity tests use (integer, negative, beyond the row, +-inf, NaN,
 * +-1e30, -0, subnormal).  A few known answers are checked on the way
 * (model.py:294 pooling, :267-281 sampling at integer positions, the
 * backward's corner weights summing to the output gradient).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/corr_oracle.c"

static unsigned rng = 12345u;
static float frand(void) {
    rng = rng * 1664525u + 1013904223u;
    return (float)((rng >> 8) & 0xFFFF) / 65536.0f - 0.5f;
}

static float *alloc(long n) {
    float *p = (float *)malloc((size_t)n * sizeof(float));
    if (!p) { fprintf(stderr, "malloc\n"); exit(2); }
    for (long i = 0; i < n; ++i) p[i] = frand();
    return p;
}

static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); ++fails; } } while (0)

static float special_x(int k, int w, int W) {
    const float sub = 1e-40f;
    switch (k % 12) {
        case 0: return (float)w;                        /* integer, in range */
        case 1: return (float)w - 0.37f * (float)(k % 7);
        case 2: return -3.5f;                           /* left of the row */
        case 3: return (float)W + 2.25f;                /* right of the row */
        case 4: return INFINITY;
        case 5: return -INFINITY;
        case 6: return NAN;
        case 7: return 1e30f;
        case 8: return -1e30f;
        case 9: return -0.0f;
        case 10: return sub;
        default: return (float)(W - 1);                 /* last element */
    }
}

static void run_case(int B, int D, int H, int W1, int W2, int levels, int radius) {
    const long P = (long)B * H * W1;
    float *f1 = alloc((long)B * D * H * W1), *f2 = alloc((long)B * D * H * W2);
    float **pyr = (float **)malloc(sizeof(float *) * levels);
    int *widths = (int *)malloc(sizeof(int) * levels);
    widths[0] = W2;
    pyr[0] = (float *)malloc(sizeof(float) * P * W2);
    oracle_corr_volume(f1, f2, B, D, H, W1, W2, pyr[0]);
    for (int l = 1; l < levels; ++l) {
        widths[l] = widths[l - 1] / 2;
        pyr[l] = (float *)malloc(sizeof(float) * P * widths[l] + 1);
        oracle_corr_pool(pyr[l - 1], P, widths[l - 1], pyr[l]);
        for (int j = 0; j < widths[l]; ++j) {                  /* model.py:294 */
            const float a = pyr[l - 1][2 * j], b = pyr[l - 1][2 * j + 1];
            CHECK(pyr[l][j] == (a + b) / 2.0f, "pool l=%d j=%d", l, j);
        }
    }
    const int T = 2 * radius + 1, C = levels * T;
    float *coords = (float *)malloc(sizeof(float) * 2 * B * H * W1);
    for (int b = 0; b < B; ++b)
        for (int h = 0; h < H; ++h)
            for (int w = 0; w < W1; ++w) {
                const long o = (long)b * 2 * H * W1 + (long)h * W1 + w;
                coords[o] = special_x((int)((b * 7 + h * 3 + w) % 97), w % W2, W2);
                coords[o + (long)H * W1] = 0.0f;
            }
    float *out = (float *)malloc(sizeof(float) * B * C * H * W1);
    oracle_corr_lookup((const float *const *)pyr, widths, levels, radius, coords, 2L * H * W1, B, H, W1, out);
    /* integer in-range x at level 0, tap 0: the element itself, up to the
     * normalise / unnormalise round trip (model.py:271, :275), which can move
     * x' by a few ulp (then w1 ~ 1e-6 of the neighbour difference) */
    for (int b = 0; b < B; ++b)
        for (int h = 0; h < H; ++h)
            for (int w = 0; w < W1; ++w) {
                const long o = (long)b * 2 * H * W1 + (long)h * W1 + w;
                const float x = coords[o];
                if (x == floorf(x) && x >= 0.0f && x <= (float)(W2 - 1) && W2 > 1) {
                    const long p = ((long)b * H + h) * W1 + w;
                    const float got = out[(((long)b * C + radius) * H + h) * W1 + w];
                    const float want = pyr[0][p * W2 + (long)x];
                    CHECK(fabsf(got - want) <= 1e-4f * (1.0f + fabsf(want)), "lookup integer x b=%d h=%d w=%d: %g vs %g",
                          b, h, w, got, want);
                }
            }
    float *gout = alloc((long)B * C * H * W1);
    float **gpyr = (float **)malloc(sizeof(float *) * levels);
    for (int l = 0; l < levels; ++l) gpyr[l] = (float *)calloc((size_t)P * widths[l], sizeof(float));
    oracle_corr_lookup_backward(gpyr, widths, levels, radius, coords, 2L * H * W1, B, H, W1, gout);
    /* a pixel whose x is an in-range integer (level 0, W2 > 2r + 2 away from
     * the edges): every tap's weight lands on its two corners, so the row sums
     * to the sum of the level-0 output gradients of that pixel */
    for (int w = radius + 1; w + radius + 1 < W1 && w + radius + 1 < W2; ++w) {
        const long o = (long)w;                                  /* b = 0, h = 0 */
        if (coords[o] != (float)w) continue;
        double s = 0.0, g = 0.0;
        for (int j = 0; j < W2; ++j) s += gpyr[0][(long)w * W2 + j];
        for (int t = 0; t < T; ++t) g += gout[(long)t * H * W1 + w];
        CHECK(fabs(s - g) <= 1e-5 * (1.0 + fabs(g)), "backward mass w=%d: %g vs %g", w, s, g);
    }
    float *scratch = (float *)malloc(sizeof(float) * P * W2);
    float *d1 = (float *)malloc(sizeof(float) * B * D * H * W1), *d2 = (float *)malloc(sizeof(float) * B * D * H * W2);
    for (int l = 0; l < levels; ++l)
        for (long k = 0; k < P * widths[l]; ++k)
            if (!isfinite(gpyr[l][k])) gpyr[l][k] = 0.0f;       /* NaN coords made NaN gradients */
    oracle_corr_build_backward(f1, f2, B, D, H, W1, W2, (const float *const *)gpyr, levels, scratch, d1, d2);
    for (long k = 0; k < (long)B * D * H * W1; ++k) CHECK(isfinite(d1[k]), "df1 not finite at %ld", k);
    for (long k = 0; k < (long)B * D * H * W2; ++k) CHECK(isfinite(d2[k]), "df2 not finite at %ld", k);
    free(f1); free(f2); free(coords); free(out); free(gout); free(scratch); free(d1); free(d2);
    for (int l = 0; l < levels; ++l) { free(pyr[l]); free(gpyr[l]); }
    free(pyr); free(gpyr); free(widths);
}

int main(void) {
    /* B, D, H, W1, W2, levels, radius: odd widths, 1-5 levels, r 1..4 */
    static const int cases[][7] = {
        {1, 8, 2, 16, 37, 4, 4}, {2, 5, 3, 13, 45, 3, 3}, {1, 3, 1, 40, 60, 5, 2},
        {1, 4, 2, 11, 16, 1, 1}, {2, 6, 2, 24, 31, 2, 4}, {1, 9, 1, 33, 240, 4, 4},
    };
    for (size_t c = 0; c < sizeof(cases) / sizeof(cases[0]); ++c) {
        const int *k = cases[c];
        run_case(k[0], k[1], k[2], k[3], k[4], k[5], k[6]);
    }
    if (fails) { fprintf(stderr, "%d check(s) failed\n", fails); return 1; }
    printf("oracle sanitize run ok: %zu cases\n", sizeof(cases) / sizeof(cases[0]));
    return 0;
}
