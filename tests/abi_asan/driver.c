/* Host sanitizer run of the product library's C-ABI argument validation.
 *
 * Built against a copy of libflame_amd.so whose HOST code is compiled with
 * -fsanitize=address,undefined (device code untouched; tests/abi_asan/Makefile).  Every
 * call below carries malformed arguments -- NULL tables, out-of-range counts, unknown
 * flags, metadata blocks too large / misaligned / with tables outside them, random
 * offsets -- and must be refused on the host with an error code and a message, before
 * any HIP call, without a sanitizer report.  No GPU is needed. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "flame_amd.h"

static int failures = 0;
#define EXPECT(cond, what)                                                                   \
    do {                                                                                     \
        if (!(cond)) {                                                                       \
            fprintf(stderr, "FAIL %s:%d %s (last error: %s)\n", __FILE__, __LINE__, what,     \
                    flame_last_error());                                                     \
            ++failures;                                                                      \
        }                                                                                    \
    } while (0)
#define EXPECT_ERR(call, code, substr)                                                       \
    do {                                                                                     \
        int rc_ = (call);                                                                    \
        EXPECT(rc_ == (code), #call);                                                        \
        if ((substr)[0]) EXPECT(strstr(flame_last_error(), (substr)) != NULL, #call " msg");  \
    } while (0)

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; }

int main(void) {
    EXPECT(flame_abi_version() == 1, "abi version");
    EXPECT(flame_chunk_elems(99) == 0 && flame_chunk_elems(-1) == 0, "chunk_elems invalid dtype");
    EXPECT(flame_scale_add_chunk_elems(FLAME_I64) == 0, "scale_add chunk of an int dtype");
    const int64_t cap = flame_agg_argmeta_max_bytes();
    EXPECT(cap == 3584, "argmeta cap");

    void *fake = (void *)(uintptr_t)4096;     /* never dereferenced: checks run first */
    EXPECT_ERR(flame_agg_reduce(0, 0, NULL, 0, 1, NULL, 0, NULL, NULL, NULL), FLAME_EINVAL, "segment");
    EXPECT_ERR(flame_agg_reduce(0, 8, fake, 1, 1, NULL, 0, NULL, NULL, NULL), FLAME_EINVAL, "unknown flags");
    EXPECT_ERR(flame_agg_reduce(77, 0, fake, 1, 1, fake, 1, fake, NULL, NULL), FLAME_ENOTSUP, "");
    EXPECT_ERR(flame_fedbuff_scale_add(0, fake, 1, 1, 0, NULL), FLAME_EINVAL, "goal");
    EXPECT_ERR(flame_synth_fill(0, NULL, 5, 0, 0, 0, 1.f, NULL), FLAME_EINVAL, "");
    EXPECT_ERR(flame_fedopt_reduce_adapt(0, 0, 0, NULL, 0, 1, NULL, 0, NULL, 0, 0, 0, 0, 0, 0, NULL),
               FLAME_EINVAL, "");
    EXPECT_ERR(flame_fedopt_reduce_adapt(4, 0, 0, NULL, 0, 1, NULL, 0, NULL, 0, 0, 0, 0, 0, 0, NULL),
               FLAME_EINVAL, "");
    {   /* eager FedOPT chain: table, step_end, variant, flags and dtype checks before any HIP call */
        const float r = 0.5f;
        const uint8_t e = 1;
        EXPECT_ERR(flame_fedopt_chain(0, 0, 0, NULL, 0, 1, NULL, 1, &r, &e, 0, 0, 0, 0, 0, 0, NULL),
                   FLAME_EINVAL, "");
        EXPECT_ERR(flame_fedopt_chain(0, 0, 0, fake, 1, 1, fake, 1, &r, NULL, 0, 0, 0, 0, 0, 0, NULL),
                   FLAME_EINVAL, "step_end");
        EXPECT_ERR(flame_fedopt_chain(0, 0, 0, fake, 1, 1, fake, 0, &r, &e, 0, 0, 0, 0, 0, 0, NULL),
                   FLAME_EINVAL, "client");
        EXPECT_ERR(flame_fedopt_chain(0, 7, 0, fake, 1, 1, fake, 1, &r, &e, 0, 0, 0, 0, 0, 0, NULL),
                   FLAME_ENOTSUP, "variant");
        EXPECT_ERR(flame_fedopt_chain(0, 0, 2, fake, 1, 1, fake, 1, &r, &e, 0, 0, 0, 0, 0, 0, NULL),
                   FLAME_EINVAL, "unknown flags");
        EXPECT_ERR(flame_fedopt_chain(FLAME_F64, 0, 0, fake, 1, 1, fake, 1, &r, &e, 0, 0, 0, 0, 0, 0, NULL),
                   FLAME_ENOTSUP, "dtype");
    }
    EXPECT_ERR(flame_host_register(NULL, 0), FLAME_EINVAL, "");
    EXPECT_ERR(flame_host_unregister(NULL), FLAME_EINVAL, "");
    EXPECT_ERR(flame_host_device_pointer(NULL, NULL), FLAME_EINVAL, "");
    EXPECT_ERR(flame_feddyn_round(0, NULL, 0, 1, NULL, NULL, 0, 0, .5, .5, NULL), FLAME_EINVAL, "");
    EXPECT(flame_hier_resident_per_cu(FLAME_BF16, 0, 0) == -FLAME_EINVAL, "resident_per_cu n_mids 0");
    EXPECT(strstr(flame_last_error(), "n_mids") != NULL, "resident_per_cu msg");
    EXPECT(flame_hier_resident_per_cu(FLAME_I64, 0, 64) == -FLAME_ENOTSUP, "resident_per_cu int dtype");
    EXPECT_ERR(flame_feddyn_round(0, fake, 1, 1, fake, NULL, 2, 0, .5, .5, NULL), FLAME_EINVAL, "step flag");
    EXPECT_ERR(flame_feddyn_round(0, fake, 1, 1, fake, fake, 2, 3, .5, .5, NULL), FLAME_EINVAL, "n_phase1");
    EXPECT_ERR(flame_hier_fedbuff(0, 0, fake, 1, 1, 0, 1, fake, NULL, fake, fake, fake, fake, 0.f, NULL),
               FLAME_EINVAL, "middle");
    EXPECT_ERR(flame_hier_fedbuff(0, FLAME_HIER_SYNC, fake, 1, 1, 1, 1, fake, NULL, fake, fake, fake, fake, 0.f,
                                  NULL), FLAME_EINVAL, "SYNC");
    {   /* slab inserts: table checks run before any HIP call */
        flame_tile_copy tc[3] = {{fake, fake, 0, 0}, {fake, (char *)fake + 8, 100, 4096}, {NULL, fake, 5, 4096}};
        EXPECT_ERR(flame_slab_write(NULL, 1, NULL), FLAME_EINVAL, "NULL table");
        EXPECT_ERR(flame_slab_write(tc, -1, NULL), FLAME_EINVAL, "");
        EXPECT(flame_slab_write(tc, 1, NULL) == FLAME_OK, "slab_write: empty entries launch nothing");
        EXPECT_ERR(flame_slab_write(tc, 2, NULL), FLAME_EINVAL, "aligned");
        EXPECT_ERR(flame_slab_write_2d(tc + 2, 1, NULL), FLAME_EINVAL, "NULL pointer");
        tc[1].dst = fake;
        tc[1].nbytes = 3 * FLAME_TILE_BYTES;
        tc[1].dst_tile_stride = 100;
        EXPECT_ERR(flame_slab_write_2d(tc, 2, NULL), FLAME_EINVAL, "dst_tile_stride");
        tc[1].nbytes = -1;
        EXPECT_ERR(flame_slab_write(tc, 2, NULL), FLAME_EINVAL, "nbytes");
    }

    uint64_t blk[64];
    memset(blk, 0, sizeof blk);
    EXPECT_ERR(flame_agg_reduce_argmeta(0, 0, NULL, 80, 1, 1, 0, 80, -1, -1, NULL), FLAME_EINVAL, "");
    EXPECT_ERR(flame_agg_reduce_argmeta(0, 0, blk, cap + 8, 1, 1, 0, 80, -1, -1, NULL), FLAME_EINVAL, "");
    EXPECT_ERR(flame_agg_reduce_argmeta(0, 0, blk, 512, 1, 1, 100, 80, 96, -1, NULL), FLAME_EINVAL, "outside");
    EXPECT_ERR(flame_agg_reduce_argmeta(0, 0, blk, 512, 1, 1, 4, 80, -1, -1, NULL), FLAME_EINVAL, "rate");
    EXPECT_ERR(flame_agg_reduce_argmeta(0, 8, blk, 512, 1, 1, 4, 80, 112, -1, NULL), FLAME_EINVAL, "");
    EXPECT_ERR(flame_agg_reduce_argmeta(0, 0, blk, 513, 1, 1, 4, 80, 112, -1, NULL), FLAME_EINVAL, "");
    EXPECT_ERR(flame_hier_fedbuff_argmeta(0, 0, blk, 512, 1, 1, 1, 2, 64, -1, 504, 88, 96, 104, 0.f, NULL),
               FLAME_EINVAL, "outside");
    EXPECT_ERR(flame_hier_fedbuff_argmeta(0, 0, blk, 4096, 1, 1, 1, 2, 64, -1, 504, 88, 96, 104, 0.f, NULL),
               FLAME_EINVAL, "");
    EXPECT_ERR(flame_hier_fedbuff_argmeta(0, 16, blk, 512, 1, 1, 1, 2, 64, -1, 504, 88, 96, 104, 0.f, NULL),
               FLAME_EINVAL, "unknown flags");
    EXPECT_ERR(flame_fedopt_reduce_adapt_argmeta(0, 0, 0, blk, 512, 1, 1, 2, 504, 96, .9f, .1f, .99f, .01f, .01f,
                                                 .001f, NULL), FLAME_EINVAL, "outside");
    EXPECT_ERR(flame_fedopt_reduce_adapt_argmeta(0, 0, 0, blk, 4096, 1, 1, 2, 80, 96, .9f, .1f, .99f, .01f, .01f,
                                                 .001f, NULL), FLAME_EINVAL, "");
    EXPECT_ERR(flame_fedopt_reduce_adapt_argmeta(0, 0, 4, blk, 512, 1, 1, 2, 504, 96, .9f, .1f, .99f, .01f, .01f,
                                                 .001f, NULL), FLAME_EINVAL, "unknown flags");

    /* randomized: a table offset or count that puts a table outside the block must be refused
       (each draw is constructed to be invalid, so nothing is launched) */
    for (int it = 0; it < 20000; ++it) {
        const int64_t bytes = 8 * (int64_t)(1 + next() % 64);
        const int32_t segs = (int32_t)(1 + next() % 4), clients = (int32_t)(1 + next() % 40);
        const int64_t off_cl = (int64_t)(next() % 1024) - 64;
        const int64_t need = off_cl + (int64_t)segs * clients * 8;
        int64_t off_r = bytes + 8 * (int64_t)(next() % 16);        /* always past the end */
        if (need <= bytes && off_cl >= 0 && (next() & 1)) off_r = -8 * (int64_t)(1 + next() % 4);
        const int rc = flame_agg_reduce_argmeta(0, 0, blk, bytes, segs, 1, clients, off_cl, off_r, -1, NULL);
        EXPECT(rc == FLAME_EINVAL, "random argmeta refused");
        const int rh = flame_hier_fedbuff_argmeta(1, 0, blk, bytes, segs, 1, 1 + (int32_t)(next() % 8), clients,
                                                  off_cl, -1, bytes + 8 * (int64_t)(next() % 8), off_r, off_r, off_r,
                                                  0.f, NULL);
        EXPECT(rh == FLAME_EINVAL, "random hier argmeta refused");
        if (failures > 10) break;
    }
    if (failures) {
        fprintf(stderr, "%d failure(s)\n", failures);
        return 1;
    }
    printf("abi asan OK\n");
    return 0;
}
