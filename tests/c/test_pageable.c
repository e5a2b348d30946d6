/* Pageable (malloc'd) memory through the library, checked against the CPU oracle:
 *
 *  - the isa-l-shaped calls at sizes on both sides of the pinned-arena limit (small calls
 *    bounce through pinned memory with CPU copies, large ones through a device arena),
 *    in-place forms with repeated pointers, lengths that are odd multiples of 32 bytes
 *    (isa-l's granule) and bases off malloc's alignment;
 *  - draid_ec_host_encode / draid_ec_host_reconstruct on a malloc'd strided layout with
 *    gaps between strips and stripes (the gaps must come back untouched), stripe counts
 *    that end in a partial chunk, and a failure table that mixes none / one / two.
 *
 * Built plain and, for the GPU box, with the library's host code under AddressSanitizer
 * (make san-gpu).  Needs an MI355X. */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "draid_ec.h"
#include "isal_oracle.h"

#define CHECK(cond)                                                                        \
    do {                                                                                   \
        if (!(cond)) {                                                                     \
            fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond,            \
                    draid_ec_last_error());                                                \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

static void *xmalloc(size_t n)
{
    void *p = malloc(n ? n : 1);
    CHECK(p != NULL);
    return p;
}

/* k data vectors + P + Q of `len` bytes at `skew` bytes past malloc's alignment */
static void vector_calls(int k, int len, int skew, uint64_t seed)
{
    const int n = k + 2;
    uint8_t *raw[64], *got[64], *want[64];
    CHECK(n <= 64);
    for (int i = 0; i < n; ++i) {
        raw[i] = xmalloc((size_t)len + 64);
        got[i] = raw[i] + skew;
        want[i] = xmalloc((size_t)len);
        orc_fill_splitmix(want[i], (size_t)len, seed * 131 + (uint64_t)i);
        memcpy(got[i], want[i], (size_t)len);
    }
    /* P+Q */
    CHECK(draid_pq_gen(n, len, (void **)got) == 0);
    CHECK(orc_pq_gen(n, len, (void **)want) == 0);
    for (int i = 0; i < n; ++i)
        CHECK(memcmp(got[i], want[i], (size_t)len) == 0);
    CHECK(draid_pq_check(n, len, (void **)got) == 0);
    got[1][len / 2] ^= 0x40;
    CHECK(draid_pq_check(n, len, (void **)got) != 0);
    got[1][len / 2] ^= 0x40;
    /* XOR over k + 1, and its check */
    CHECK(draid_xor_gen(k + 1, len, (void **)got) == 0);
    CHECK(orc_xor_gen(k + 1, len, (void **)want) == 0);
    CHECK(memcmp(got[k], want[k], (size_t)len) == 0);
    CHECK(draid_xor_check(k + 1, len, (void **)got) == 0);
    got[k][len - 1] ^= 1;
    CHECK(draid_xor_check(k + 1, len, (void **)got) != 0);
    got[k][len - 1] ^= 1;
    /* constant multiply, out of place and in place (source == destination) */
    unsigned char tbl[32], otbl[32];
    draid_gf_vect_mul_init(0x8e, tbl);
    orc_gf_vect_mul_init(0x8e, otbl);
    CHECK(memcmp(tbl, otbl, 32) == 0);
    CHECK(draid_gf_vect_mul(len, tbl, got[0], got[k + 1]) == 0);
    CHECK(orc_gf_vect_mul(len, otbl, want[0], want[k + 1]) == 0);
    CHECK(memcmp(got[k + 1], want[k + 1], (size_t)len) == 0);
    CHECK(draid_gf_vect_mul(len, tbl, got[2], got[2]) == 0);
    CHECK(orc_gf_vect_mul(len, otbl, want[2], want[2]) == 0);
    CHECK(memcmp(got[2], want[2], (size_t)len) == 0);
    /* rebuild two lost data vectors from fresh parity */
    CHECK(draid_pq_gen(n, len, (void **)got) == 0);
    CHECK(orc_pq_gen(n, len, (void **)want) == 0);
    const int fail[2] = {0, k - 1};
    memset(got[0], 0xee, (size_t)len);
    memset(got[k - 1], 0xee, (size_t)len);
    CHECK(draid_recover(k, 2, len, (void **)got, 2, fail) == 0);
    for (int i = 0; i < n; ++i)
        CHECK(memcmp(got[i], want[i], (size_t)len) == 0);
    /* the bytes either side of every vector are as malloc left them or as we set them:
     * nothing to compare, but the sanitizer build sees any write outside [got, got+len) */
    for (int i = 0; i < n; ++i) {
        free(raw[i]);
        free(want[i]);
    }
    printf("ok vectors k=%d len=%d skew=%d\n", k, len, skew);
}

static void host_stripes(int k, int m, size_t strip_len, uint32_t nstripes, size_t strip_gap,
                         size_t stripe_gap, uint32_t chunk_stripes, uint32_t flags, uint64_t seed)
{
    const int n = k + m;
    const size_t strip_stride = strip_len + strip_gap;
    const size_t stripe_stride = strip_stride * (size_t)n + stripe_gap;
    const size_t bytes = stripe_stride * nstripes;
    uint8_t *got = xmalloc(bytes), *want = xmalloc(bytes);
    uint8_t *fail = xmalloc(2 * (size_t)nstripes);
    orc_fill_splitmix(want, bytes, seed);
    memcpy(got, want, bytes);
    draid_ec_host_stripes h = {(uint32_t)k, (uint32_t)m, strip_len, nstripes, flags, got,
                               strip_stride, stripe_stride};
    CHECK(draid_ec_host_encode(&h, chunk_stripes) == 0);
    CHECK(orc_encode_strided(k, m, strip_len, nstripes, want, strip_stride, stripe_stride) == 0);
    CHECK(memcmp(got, want, bytes) == 0);  /* parity equal, data and gaps untouched */
    for (uint32_t s = 0; s < nstripes; ++s) {
        const int how = (int)(s % 4);
        fail[2 * s] = how == 0 ? 0xFF : (uint8_t)(s % (uint32_t)n);
        fail[2 * s + 1] = (how == 3 && m == 2) ? (uint8_t)((s + 1 + s / 7) % (uint32_t)n) : 0xFF;
        if (fail[2 * s + 1] == fail[2 * s])
            fail[2 * s + 1] = 0xFF;
        for (int f = 0; f < 2; ++f)
            if (fail[2 * s + f] != 0xFF)
                memset(got + s * stripe_stride + fail[2 * s + f] * strip_stride, 0x5a, strip_len);
    }
    CHECK(draid_ec_host_reconstruct(&h, fail, chunk_stripes) == 0);
    CHECK(memcmp(got, want, bytes) == 0);
    /* a table the engine must refuse before touching anything */
    if (nstripes > 1) {
        fail[2] = (uint8_t)n;
        got[0] ^= 0xff;
        CHECK(draid_ec_host_reconstruct(&h, fail, chunk_stripes) == 1);
        got[0] ^= 0xff;
        CHECK(memcmp(got, want, bytes) == 0);
    }
    free(got);
    free(want);
    free(fail);
    printf("ok host stripes %d+%d x %zu B x %u (gaps %zu/%zu, chunk %u, flags %u)\n", k, m,
           strip_len, nstripes, strip_gap, stripe_gap, chunk_stripes, flags);
}

int main(void)
{
    /* pinned arena (a few KiB to 8 MiB per call) ... */
    vector_calls(4, 4096, 0, 1);
    vector_calls(8, 65536, 0, 2);
    vector_calls(3, 992, 16, 3);       /* 31 x 32 bytes, bases off malloc's alignment */
    vector_calls(10, 512 * 1024, 0, 4);
    /* ... and the device arena beyond it (12 x 1 MiB + padding > 8 MiB) */
    vector_calls(10, 1024 * 1024, 0, 5);
    vector_calls(6, 2 * 1024 * 1024 + 32, 8, 6);
    /* host stripes in pageable memory: bounced by the calling thread */
    host_stripes(8, 2, 65536, 100, 0, 0, 0, 0, 11);       /* 100 stripes: partial last chunk */
    host_stripes(4, 2, 4096, 37, 512, 1024, 0, 0, 12);    /* gaps between strips and stripes */
    host_stripes(4, 1, 16384, 64, 0, 4096, 16, 0, 13);    /* RAID5, explicit chunk */
    host_stripes(8, 2, 1024 * 1024, 5, 0, 0, 0, 0, 14);   /* a stripe larger than half a chunk */
    host_stripes(6, 2, 32768, 33, 0, 0, 8, DRAID_EC_HOST_STAGED, 15);  /* runtime-staged path */
    printf("PASS pageable\n");
    return 0;
}
