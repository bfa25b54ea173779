/*
 * c_abi_fedavg.c -- the drop-in boundary used from plain C (no Python, no torch):
 * FedAvg of N client updates through flame_agg_reduce (include/flame_amd.h), checked
 * bitwise against the reference arithmetic (fedavg.py:84-104: tmp = v*rate; agg += tmp,
 * fp32, one rounding per op, clients in order).
 *
 *   gcc -O2 -ffp-contract=off -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I include examples/c_abi_fedavg.c
 *       -L flame_amd -lflame_amd -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/flame_amd -o build/c_abi_fedavg
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "flame_amd.h"

#define HIPCHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 2; } } while (0)

int main(void) {
    const int n = 19;
    const int64_t P = 100003;                 /* ragged: tail handled by the kernel */
    const int counts[19] = {5, 17, 3, 99, 1, 42, 7, 8, 13, 21, 34, 55, 89, 2, 4, 6, 10, 12, 14};
    int total = 0;
    for (int i = 0; i < n; ++i) total += counts[i];

    float *h_base = malloc(P * sizeof(float)), *h_exp = malloc(P * sizeof(float));
    float **h_cl = malloc(n * sizeof(float *));
    float rates[19];
    uint32_t s = 12345u;
    for (int64_t e = 0; e < P; ++e) { s = s * 1664525u + 1013904223u; h_base[e] = (float)(s >> 8) / 16777216.0f - 0.5f; }
    for (int i = 0; i < n; ++i) {
        h_cl[i] = malloc(P * sizeof(float));
        for (int64_t e = 0; e < P; ++e) { s = s * 1664525u + 1013904223u; h_cl[i][e] = ((float)(s >> 8) / 16777216.0f - 0.5f) * 0.01f; }
        rates[i] = (float)((double)counts[i] / (double)total);   /* python float -> fp32 */
    }
    /* reference arithmetic on the host */
    memcpy(h_exp, h_base, P * sizeof(float));
    for (int i = 0; i < n; ++i)
        for (int64_t e = 0; e < P; ++e) { volatile float t = h_cl[i][e] * rates[i]; h_exp[e] = h_exp[e] + t; }

    /* device buffers */
    float *d_base, *d_rates;
    void **h_ptrs = malloc(n * sizeof(void *)), **d_ptrs;
    HIPCHK(hipMalloc((void **)&d_base, P * sizeof(float)));
    HIPCHK(hipMemcpy(d_base, h_base, P * sizeof(float), hipMemcpyHostToDevice));
    for (int i = 0; i < n; ++i) {
        HIPCHK(hipMalloc(&h_ptrs[i], P * sizeof(float)));
        HIPCHK(hipMemcpy(h_ptrs[i], h_cl[i], P * sizeof(float), hipMemcpyHostToDevice));
    }
    HIPCHK(hipMalloc((void **)&d_ptrs, n * sizeof(void *)));
    HIPCHK(hipMemcpy(d_ptrs, h_ptrs, n * sizeof(void *), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc((void **)&d_rates, n * sizeof(float)));
    HIPCHK(hipMemcpy(d_rates, rates, n * sizeof(float), hipMemcpyHostToDevice));

    /* one segment: the aggregate is updated in place (out == in), as FedAvg mutates base */
    flame_segment seg;
    memset(&seg, 0, sizeof(seg));
    seg.out = d_base;
    seg.in = d_base;
    seg.numel = P;
    const int64_t chunk = flame_chunk_elems(FLAME_F32);
    const int64_t n_chunks = (P + chunk - 1) / chunk;
    flame_segment *d_seg;
    HIPCHK(hipMalloc((void **)&d_seg, sizeof(seg)));
    HIPCHK(hipMemcpy(d_seg, &seg, sizeof(seg), hipMemcpyHostToDevice));

    int rc = flame_agg_reduce(FLAME_F32, 0, d_seg, 1, n_chunks, (const void *const *)d_ptrs, n, d_rates, NULL, NULL);
    if (rc != FLAME_OK) { fprintf(stderr, "flame_agg_reduce: %d %s\n", rc, flame_last_error()); return 1; }
    /* argument errors come back as status codes, never aborts */
    if (flame_agg_reduce(FLAME_F32, 0, NULL, 0, 1, NULL, 0, NULL, NULL, NULL) != FLAME_EINVAL) return 1;
    HIPCHK(hipDeviceSynchronize());

    float *h_out = malloc(P * sizeof(float));
    HIPCHK(hipMemcpy(h_out, d_base, P * sizeof(float), hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t e = 0; e < P; ++e) bad += memcmp(&h_out[e], &h_exp[e], 4) != 0;
    printf("c_abi_fedavg: %lld / %lld elements differ (abi %d)\n", (long long)bad, (long long)P, flame_abi_version());
    return bad ? 1 : 0;
}
