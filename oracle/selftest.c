/*
 * selftest.c -- host-only sanitizer run of the CPU oracle (SURVEY.md §5 "Race detection /
 * sanitizers": the build runs its C restatement under ASan/UBSan in this container).
 * Exercises every entry point of fedagg_oracle.c on ragged sizes, all dtypes, and checks
 * known answers for the conversions and the arithmetic.  Built with
 *   gcc -fsanitize=address,undefined -fno-sanitize-recover=all  (oracle/Makefile: selftest)
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void flame_oracle_reduce(int dtype, void *acc, int64_t numel, const void *const *clients,
                         const float *rates32, const double *rates64, int n, int init_first);
void flame_oracle_scale_add(int dtype, void *base, const void *agg, int64_t numel, int64_t goal, void *delta);
void flame_oracle_fedopt_adapt(int variant, const float *avg, const float *cur, float *m, float *v,
                               float *cur_out, int64_t numel, float b1, float omb1, float b2,
                               float omb2, float eta, float tau);
void flame_oracle_synth_f32(uint64_t seed, uint64_t stream, int64_t start, int64_t n, float scale, float *out);
void flame_oracle_f32_to_bf16(const float *x, uint16_t *y, int64_t n);
void flame_oracle_f32_to_f16(const float *x, uint16_t *y, int64_t n);

static int fails = 0;
#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); fails++; } } while (0)

int main(void) {
    /* conversions: known answers */
    float xs[] = {1.0f, 1.00390625f /* bf16 tie -> even */, 65504.0f, 65520.0f, 5.96046448e-08f, -0.0f, 3.0e-8f};
    uint16_t b[7], h[7];
    flame_oracle_f32_to_bf16(xs, b, 7);
    flame_oracle_f32_to_f16(xs, h, 7);
    CHECK(b[0] == 0x3F80 && b[1] == 0x3F80);
    CHECK(h[0] == 0x3C00 && h[2] == 0x7BFF && h[3] == 0x7C00 && h[4] == 0x0001 && h[5] == 0x8000);
    /* reduce: all dtypes, ragged sizes, heap buffers exactly sized (ASan catches overruns) */
    const int n = 5;
    float r32[5] = {0.1f, 0.2f, 0.3f, 0.25f, 0.15f};
    double r64[5] = {0.1, 0.2, 0.3, 0.25, 0.15};
    int64_t sizes[] = {0, 1, 7, 1023, 4099};
    size_t isz[] = {4, 2, 2, 8, 8, 4};
    for (int dt = 0; dt < 6; ++dt) {
        for (int si = 0; si < 5; ++si) {
            int64_t P = sizes[si];
            void *acc = calloc((size_t)(P ? P : 1), isz[dt]);
            const void *cl[5];
            void *own[5];
            for (int i = 0; i < n; ++i) {
                own[i] = malloc((size_t)(P ? P : 1) * isz[dt]);
                memset(own[i], 0x3C, (size_t)(P ? P : 1) * isz[dt]);
                cl[i] = own[i];
            }
            flame_oracle_reduce(dt, acc, P, cl, r32, r64, n, 0);
            flame_oracle_reduce(dt, acc, P, cl, r32, r64, n, 1);
            if (dt == 1 || dt == 2 || dt == 0 || dt == 3) {
                void *d = malloc((size_t)(P ? P : 1) * isz[dt]);
                flame_oracle_scale_add(dt, acc, cl[0], P, 3, d);
                free(d);
            }
            for (int i = 0; i < n; ++i) free(own[i]);
            free(acc);
        }
    }
    /* fp32 arithmetic known answer: 0 + 2*0.5 + 4*0.25 = 2 */
    float a0 = 0.f, c1 = 2.f, c2 = 4.f, rr[2] = {0.5f, 0.25f};
    const void *cc[2] = {&c1, &c2};
    flame_oracle_reduce(0, &a0, 1, cc, rr, NULL, 2, 0);
    CHECK(a0 == 2.0f);
    /* fedopt: finite outputs for every variant */
    float avg[3] = {1, 2, 3}, cur[3] = {0.5f, 2.5f, 3}, m[3] = {0}, v[3] = {0}, co[3];
    for (int var = 0; var < 3; ++var) {
        flame_oracle_fedopt_adapt(var, avg, cur, m, v, co, 3, 0.9f, 0.1f, 0.99f, 0.01f, 0.01f, 0.001f);
        for (int j = 0; j < 3; ++j) CHECK(isfinite(co[j]) && isfinite(m[j]) && v[j] >= 0.f);
    }
    /* synth: deterministic, mean ~0 */
    float *s = malloc(100000 * sizeof(float));
    flame_oracle_synth_f32(1, 2, 0, 100000, 1.0f / 37837.2f, s);  /* std ~ 1 */
    double mean = 0;
    for (int i = 0; i < 100000; ++i) mean += s[i];
    CHECK(fabs(mean / 100000) < 0.02);
    free(s);
    if (fails) return 1;
    puts("oracle selftest OK");
    return 0;
}
