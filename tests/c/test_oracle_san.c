/* test_oracle_san.c -- the CPU oracle's encode / recover paths exercised under
 * AddressSanitizer + UndefinedBehaviorSanitizer (tests/c/Makefile `san`):
 * round trips encode -> erase -> recover for every failure set of small
 * stripes (k = 1..20, m = 1, 2, lengths that are not multiples of the word
 * size), the strided batch calls with 0xFF in either slot of the failure pair,
 * and the AVX-512 restatement against the scalar one where the CPU has it.
 * Host code only; no GPU.  Prints PASS and exits 0 when everything matches.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "isal_oracle.h"

static int g_fail;

#define EXPECT(c)                                                          \
    do {                                                                   \
        if (!(c)) {                                                        \
            fprintf(stderr, "%s:%d: EXPECT(%s)\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                      \
        }                                                                  \
    } while (0)

static uint64_t g_rng = 0x1234;
static uint8_t rnd8(void)
{
    g_rng = g_rng * 6364136223846793005ull + 1442695040888963407ull;
    return (uint8_t)(g_rng >> 56);
}

/* every single and dual failure set of one stripe through orc_recover */
static void roundtrip(int k, int m, int len)
{
    const int n = k + m;
    uint8_t *good = malloc((size_t)n * len), *work = malloc((size_t)n * len);
    void *v[257];
    for (int i = 0; i < k * len; i++)
        good[i] = rnd8();
    for (int j = 0; j < n; j++)
        v[j] = good + (size_t)j * len;
    /* any length (orc_pq_gen keeps isa-l's len % 32 == 0 contract) */
    EXPECT(orc_encode_strided(k, m, (size_t)len, 1, good, (size_t)len, (size_t)n * len) == 0);
    if (k > 1 && len % 32 == 0) {  /* the isa-l-shaped calls agree where they apply */
        uint8_t *alt = malloc((size_t)n * len);
        memcpy(alt, good, (size_t)k * len);
        for (int j = 0; j < n; j++)
            v[j] = alt + (size_t)j * len;
        EXPECT((m == 1 ? orc_xor_gen(n, len, v) : orc_pq_gen(n, len, v)) == 0);
        EXPECT(memcmp(alt, good, (size_t)n * len) == 0);
        free(alt);
    }
    for (int f0 = 0; f0 < n; f0++)
        for (int f1 = f0; f1 < n; f1++) {
            const int nf = f1 == f0 ? 1 : 2;
            if (nf > m)
                continue;
            const int fail[2] = {f1, f0};  /* descending order on purpose */
            memcpy(work, good, (size_t)n * len);
            for (int j = 0; j < n; j++)
                v[j] = work + (size_t)j * len;
            memset(v[f0], 0xA5, (size_t)len);
            memset(v[f1], 0x5A, (size_t)len);
            EXPECT(orc_recover(k, m, len, v, nf, nf == 1 ? fail + 1 : fail) == 0);
            EXPECT(memcmp(work, good, (size_t)n * len) == 0);
        }
    /* invalid sets are rejected without touching memory */
    const int dup[2] = {0, 0}, oob[1] = {n};
    for (int j = 0; j < n; j++)
        v[j] = good + (size_t)j * len;
    if (m == 2)
        EXPECT(orc_recover(k, m, len, v, 2, dup) == -1);
    EXPECT(orc_recover(k, m, len, v, 1, oob) == -1);
    free(good);
    free(work);
}

/* strided batch: encode, erase per the table, recover, compare; scalar and SIMD */
static void strided(int k, int m, size_t len, uint32_t B)
{
    const int n = k + m;
    const size_t ss = (size_t)n * len;
    uint8_t *a = calloc(B, ss), *b = malloc(B * ss), *good = malloc(B * ss);
    uint8_t *fail = malloc(2 * (size_t)B);
    for (uint32_t s = 0; s < B; s++)
        for (size_t i = 0; i < (size_t)k * len; i++)
            a[s * ss + i] = rnd8();
    EXPECT(orc_encode_strided(k, m, len, B, a, len, ss) == 0);
    memcpy(good, a, B * ss);
    if (orc_simd_available() == 1) {
        memcpy(b, a, B * ss);
        for (uint32_t s = 0; s < B; s++)
            memset(b + s * ss + (size_t)k * len, 0, (size_t)m * len);
        EXPECT(orc_simd_encode_strided(k, m, len, B, b, len, ss) == 0);
        EXPECT(memcmp(a, b, B * ss) == 0);
    }
    for (uint32_t s = 0; s < B; s++) {
        uint8_t f0 = (uint8_t)(s % n), f1 = 0xFF;
        if (m == 2 && s % 3 == 1 && s % 5 != 4)
            f1 = (uint8_t)((s + 1) % n);  /* dual */
        fail[2 * s] = (s % 5 == 4) ? 0xFF : f0;
        fail[2 * s + 1] = (s % 5 == 4) ? f0 : f1;
        memset(a + s * ss + f0 * len, 0x3C, len);
        if (f1 != 0xFF)
            memset(a + s * ss + f1 * len, 0xC3, len);
    }
    memcpy(b, a, B * ss);
    EXPECT(orc_recover_strided(k, m, len, B, a, len, ss, fail) == 0);
    EXPECT(memcmp(a, good, B * ss) == 0);
    if (orc_simd_available() == 1) {
        EXPECT(orc_simd_recover_strided(k, m, len, B, b, len, ss, fail) == 0);
        EXPECT(memcmp(b, good, B * ss) == 0);
    }
    free(a);
    free(b);
    free(good);
    free(fail);
}

int main(void)
{
    const int lens[] = {1, 7, 8, 33, 64, 100, 1024 + 5};
    for (int k = 1; k <= 20; k++)
        for (int m = 1; m <= 2; m++)
            for (unsigned i = 0; i < sizeof(lens) / sizeof(lens[0]); i++)
                roundtrip(k, m, lens[i]);
    strided(4, 1, 4096 + 7, 9);
    strided(8, 2, 1000, 12);
    strided(16, 2, 4096, 7);
    strided(1, 2, 64 + 1, 5);
    uint8_t t[32], src[96], dst[96];
    for (int i = 0; i < 96; i++)
        src[i] = (uint8_t)(i * 37 + 1);
    orc_gf_vect_mul_init(0x1D, t);
    EXPECT(orc_gf_vect_mul(96, t, src, dst) == 0);
    for (int i = 0; i < 96; i++)
        EXPECT(dst[i] == orc_gf_mul(0x1D, src[i]));
    for (int a = 1; a < 256; a++)
        EXPECT(orc_gf_mul((uint8_t)a, orc_gf_inv((uint8_t)a)) == 1);
    printf("%s (%d failures)\n", g_fail ? "FAIL" : "PASS", g_fail);
    return g_fail ? 1 : 0;
}
