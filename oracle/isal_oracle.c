/*
 * isal_oracle.c -- CPU ORACLE (test infrastructure only; see isal_oracle.h).
 *
 * Restates, without copying, the semantics of:
 *   - isa-l v2.30.0 raid_base.c  (xor_gen_base / pq_gen_base / *_check_base):
 *     external, not vendored (reference `isa-l/` submodule is empty);
 *     call sites raid5.c:197, raid5_simple.c:134,176, gf_vect_mul.c:45,101.
 *   - isa-l v2.30.0 ec_base.c    (gf_mul / gf_inv / gf_vect_mul_init /
 *     gf_vect_mul): call sites gf_vect_mul.c:60-66,108,267,310-326.
 *   - the reference's recovery compositions:
 *       RAID5 degraded read   module/bdev/raid/raid5.c:544-594
 *       D+P (data + P lost)    examples/bdev/gf_vect_mul/gf_vect_mul.c:242-281
 *       D+D (two data lost)    examples/bdev/gf_vect_mul/gf_vect_mul.c:283-347
 *   - RAID5 geometry           module/bdev/raid/raid5.c:165-186,1006-1007,1419-1426
 *
 * Field: GF(2^8) with reduction polynomial x^8+x^4+x^3+x^2+1 (0x11D) and
 * generator 2 -- isa-l's definition; the reference builds its coefficient
 * table by repeated gf_mul(c, 2) (gf_vect_mul.c:60-66) and uses 255 - x for
 * the inverse power (gf_vect_mul.c:267), i.e. multiplicative order 255.
 */
#define _GNU_SOURCE
#include "isal_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ GF */

static unsigned char g_exp[512];
static unsigned char g_log[256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void gf_build(void)
{
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
        g_exp[i] = (unsigned char)x;
        g_log[x] = (unsigned char)i;
        x <<= 1;
        if (x & 0x100)
            x ^= 0x11d;
    }
    for (int i = 255; i < 512; i++)
        g_exp[i] = g_exp[i - 255];
    g_log[0] = 0; /* undefined; never used for a == 0 */
}

static inline void gf_init(void) { pthread_once(&g_once, gf_build); }

/* ec_base.c gf_mul: 0 if either is 0, else exp[log a + log b mod 255]. */
unsigned char orc_gf_mul(unsigned char a, unsigned char b)
{
    gf_init();
    if (a == 0 || b == 0)
        return 0;
    return g_exp[g_log[a] + g_log[b]];
}

/* ec_base.c gf_inv: gf_inv(0) == 0, else exp[255 - log a]. */
unsigned char orc_gf_inv(unsigned char a)
{
    gf_init();
    if (a == 0)
        return 0;
    return g_exp[255 - g_log[a]];
}

unsigned char orc_gf_pow2(int e)
{
    gf_init();
    e %= 255;
    if (e < 0)
        e += 255;
    return g_exp[e];
}

void orc_gf_tables(unsigned char exp_out[256], unsigned char log_out[256])
{
    gf_init();
    memcpy(exp_out, g_exp, 256);
    memcpy(log_out, g_log, 256);
}

/* gf_vect_mul_init(c, tbl[32]): tbl[i] = c*i (i < 16), tbl[16+i] = c*(i<<4).
 * This is the nibble-table format isa-l's pshufb multiply consumes. */
void orc_gf_vect_mul_init(unsigned char c, unsigned char tbl[32])
{
    for (int i = 0; i < 16; i++) {
        tbl[i] = orc_gf_mul(c, (unsigned char)i);
        tbl[16 + i] = orc_gf_mul(c, (unsigned char)(i << 4));
    }
}

/* gf_vect_mul(len, tbl, src, dst): dst[i] = tbl[lo(src[i])] ^ tbl[16+hi(src[i])].
 * isa-l's SIMD dispatch requires len to be a multiple of 32 (raid.h /
 * gf_vect_mul.h contract); restated as: len < 0 or len % 32 -> fail (1). */
int orc_gf_vect_mul(int len, const unsigned char *tbl, const void *src, void *dest)
{
    if (len < 0 || (len & 31))
        return 1;
    const unsigned char *s = src;
    unsigned char *d = dest;
    for (int i = 0; i < len; i++)
        d[i] = tbl[s[i] & 15] ^ tbl[16 + (s[i] >> 4)];
    return 0;
}

/* ------------------------------------------------------------ raid.h */

/* xor_gen: array[vects-1] = XOR of array[0..vects-2], bytewise.
 * isa-l's xor_gen asm rejects fewer than two sources (vects < 3) and
 * accepts any length (tail handled bytewise). */
int orc_xor_gen(int vects, int len, void **array)
{
    if (vects < 3 || len < 0)
        return 1;
    unsigned char **v = (unsigned char **)array;
    unsigned char *dst = v[vects - 1];
    for (int i = 0; i < len; i++) {
        unsigned char p = v[0][i];
        for (int j = 1; j < vects - 1; j++)
            p ^= v[j][i];
        dst[i] = p;
    }
    return 0;
}

/* 8-lane SWAR multiply by 2 over GF(2^8)/0x11D, as pq_gen_base does it on a
 * machine word: shift every byte left and fold bit 7 back in as 0x1D. */
static inline uint64_t mul2_u64(uint64_t q)
{
    const uint64_t hi = q & 0x8080808080808080ull;
    const uint64_t mask = (hi << 1) - (hi >> 7); /* 0xFF in bytes with bit 7 */
    return ((q & 0x7f7f7f7f7f7f7f7full) << 1) ^ (mask & 0x1d1d1d1d1d1d1d1dull);
}

static inline unsigned char mul2_u8(unsigned char q)
{
    return (unsigned char)((q << 1) ^ ((q & 0x80) ? 0x1d : 0));
}

/* pq_gen: with k = vects-2 sources,
 *   P = array[k]   = XOR_j D_j
 *   Q = array[k+1] = XOR_j 2^j D_j   (Horner from j = k-1 down to 0).
 * isa-l's AVX2 dispatch requires >= 2 sources (vects >= 4) and len % 32 == 0;
 * anything else returns 1 without writing. */
int orc_pq_gen(int vects, int len, void **array)
{
    if (vects < 4 || len < 0 || (len & 31))
        return 1;
    const int k = vects - 2;
    unsigned char **v = (unsigned char **)array;
    const int words = len / 8;
    for (int w = 0; w < words; w++) {
        uint64_t p, q, s;
        memcpy(&s, v[k - 1] + 8 * (size_t)w, 8);
        p = q = s;
        for (int j = k - 2; j >= 0; j--) {
            memcpy(&s, v[j] + 8 * (size_t)w, 8);
            p ^= s;
            q = mul2_u64(q) ^ s;
        }
        memcpy(v[k] + 8 * (size_t)w, &p, 8);
        memcpy(v[k + 1] + 8 * (size_t)w, &q, 8);
    }
    return 0;
}

/* P+Q over any length (the batched API has no isa-l length contract):
 * 8-byte words, then a bytewise tail. */
static void pq_any(int k, size_t len, unsigned char **v)
{
    size_t w = 0;
    for (; w + 8 <= len; w += 8) {
        uint64_t p, q, s;
        memcpy(&s, v[k - 1] + w, 8);
        p = q = s;
        for (int j = k - 2; j >= 0; j--) {
            memcpy(&s, v[j] + w, 8);
            p ^= s;
            q = mul2_u64(q) ^ s;
        }
        memcpy(v[k] + w, &p, 8);
        memcpy(v[k + 1] + w, &q, 8);
    }
    for (; w < len; w++) {
        unsigned char p = v[k - 1][w], q = p;
        for (int j = k - 2; j >= 0; j--) {
            p ^= v[j][w];
            q = (unsigned char)(mul2_u8(q) ^ v[j][w]);
        }
        v[k][w] = p;
        v[k + 1][w] = q;
    }
}

/* xor_check: 0 iff XOR over all vects (including the parity) is zero. */
int orc_xor_check(int vects, int len, void **array)
{
    if (vects < 3 || len < 0)
        return 1;
    unsigned char **v = (unsigned char **)array;
    for (int i = 0; i < len; i++) {
        unsigned char p = 0;
        for (int j = 0; j < vects; j++)
            p ^= v[j][i];
        if (p)
            return 1;
    }
    return 0;
}

/* pq_check: 0 iff array[k], array[k+1] equal the P, Q pq_gen would write.
 * Recomputed bytewise (an independent path from orc_pq_gen's SWAR words). */
int orc_pq_check(int vects, int len, void **array)
{
    if (vects < 4 || len < 0 || (len & 31))
        return 1;
    const int k = vects - 2;
    unsigned char **v = (unsigned char **)array;
    for (int i = 0; i < len; i++) {
        unsigned char p = v[k - 1][i], q = p;
        for (int j = k - 2; j >= 0; j--) {
            p ^= v[j][i];
            q = (unsigned char)(mul2_u8(q) ^ v[j][i]);
        }
        if (v[k][i] != p || v[k + 1][i] != q)
            return 1;
    }
    return 0;
}

/* ------------------------------------------------------------ recovery */

/* dst[i] = c * src[i] through the 32-B nibble table (gf_vect_mul semantics). */
static inline unsigned char tbl_mul(const unsigned char *tbl, unsigned char x)
{
    return tbl[x & 15] ^ tbl[16 + (x >> 4)];
}

/*
 * Regenerate the strips listed in fail[] from the survivors.
 *   one data x (P alive)  : D_x = P ^ XOR_{i!=x} D_i               raid5.c:557-569
 *   data x + P            : D_x = 2^-x (Q ^ XOR_{i!=x} 2^i D_i)     gf_vect_mul.c:255-268
 *                           then P re-encoded
 *   data x + Q            : D_x from P, then Q re-encoded
 *   data x < y            : Pxy = P ^ XOR_{i!=x,y} D_i,
 *                           Qxy = Q ^ XOR_{i!=x,y} 2^i D_i,
 *                           A = 2^(y-x) / (2^(y-x) ^ 1), B = 2^-x / (2^(y-x) ^ 1),
 *                           D_x = A Pxy ^ B Qxy, D_y = Pxy ^ D_x    gf_vect_mul.c:296-330
 *   P and/or Q only       : re-encode
 * The syndromes run 8 bytes at a time (pq_gen_base word form); the constant
 * multiplies use gf_vect_mul_init nibble tables, one lookup pair per byte.
 */
int orc_recover(int k, int m, int len, void **array, int nfail, const int *fail)
{
    if (k < 1 || m < 1 || m > 2 || len < 0 || nfail < 0 || nfail > m)
        return -1;
    unsigned char **v = (unsigned char **)array;
    int lost[2] = { -1, -1 }, nd = 0, lostP = 0, lostQ = 0;
    for (int f = 0; f < nfail; f++) {
        int j = fail[f];
        if (j < 0 || j >= k + m)
            return -1;
        if (j < k) {
            if (nd == 1 && lost[0] == j)
                return -1;
            lost[nd++] = j;
        } else if (j == k) {
            if (lostP)
                return -1;
            lostP = 1;
        } else {
            if (lostQ)
                return -1;
            lostQ = 1;
        }
    }
    if (nd == 2 && lost[0] > lost[1]) {
        int t = lost[0]; lost[0] = lost[1]; lost[1] = t;
    }
    const int x = lost[0], y = lost[1];
    const int needq = (nd == 2) || (nd == 1 && lostP) || lostQ;
    unsigned char ta[32], tb[32];
    if (nd == 1 && !lostP) {
        orc_gf_vect_mul_init(orc_gf_pow2(x), ta);              /* Q rebuild: 2^x D_x */
    } else if (nd == 1) {
        orc_gf_vect_mul_init(orc_gf_pow2(255 - x), ta);        /* D_x = 2^-x (...)   */
    } else if (nd == 2) {
        unsigned char gyx = orc_gf_pow2(y - x);
        unsigned char den = orc_gf_inv((unsigned char)(gyx ^ 1));
        orc_gf_vect_mul_init(orc_gf_mul(gyx, den), ta);                 /* A */
        orc_gf_vect_mul_init(orc_gf_mul(orc_gf_pow2(255 - x), den), tb); /* B */
    }

    int i = 0;
    for (;;) {
        /* one 8-byte word, or the single-byte tail */
        const int w = (i + 8 <= len) ? 8 : (i < len ? 1 : 0);
        if (!w)
            break;
        uint64_t ps = 0, qs = 0, d = 0, pv = 0, qv = 0;
        for (int j = k - 1; j >= 0; j--) {
            d = 0;
            if (j != x && j != y)
                memcpy(&d, v[j] + i, (size_t)w);
            ps ^= d;
            if (needq)
                qs = mul2_u64(qs) ^ d;
        }
        if (!lostP)
            memcpy(&pv, v[k] + i, (size_t)w);
        if (m == 2 && !lostQ)
            memcpy(&qv, v[k + 1] + i, (size_t)w);
        unsigned char psb[8], qsb[8], pvb[8], qvb[8], o1[8], o2[8];
        memcpy(psb, &ps, 8); memcpy(qsb, &qs, 8);
        memcpy(pvb, &pv, 8); memcpy(qvb, &qv, 8);
        if (nd == 0) {
            if (lostP) memcpy(v[k] + i, psb, (size_t)w);
            if (lostQ) memcpy(v[k + 1] + i, qsb, (size_t)w);
        } else if (nd == 1) {
            for (int b = 0; b < w; b++) {
                if (!lostP) {
                    o1[b] = pvb[b] ^ psb[b];
                    o2[b] = qsb[b] ^ tbl_mul(ta, o1[b]);              /* Q if lost */
                } else {
                    o1[b] = tbl_mul(ta, (unsigned char)(qvb[b] ^ qsb[b]));
                    o2[b] = psb[b] ^ o1[b];                           /* P */
                }
            }
            memcpy(v[x] + i, o1, (size_t)w);
            if (lostP)
                memcpy(v[k] + i, o2, (size_t)w);
            else if (lostQ)
                memcpy(v[k + 1] + i, o2, (size_t)w);
        } else {
            for (int b = 0; b < w; b++) {
                unsigned char pxy = pvb[b] ^ psb[b];
                unsigned char qxy = qvb[b] ^ qsb[b];
                o1[b] = tbl_mul(ta, pxy) ^ tbl_mul(tb, qxy);
                o2[b] = pxy ^ o1[b];
            }
            memcpy(v[x] + i, o1, (size_t)w);
            memcpy(v[y] + i, o2, (size_t)w);
        }
        i += w;
    }
    return 0;
}

/* ------------------------------------------------------- strided batch */

static void strided_ptrs(int k, int m, uint8_t *base, size_t strip_stride,
                         size_t stripe_stride, uint32_t s, void **ptrs)
{
    for (int j = 0; j < k + m; j++)
        ptrs[j] = base + (size_t)s * stripe_stride + (size_t)j * strip_stride;
}

int orc_encode_strided(int k, int m, size_t len, uint32_t nstripes,
                       uint8_t *base, size_t strip_stride, size_t stripe_stride)
{
    void *ptrs[512];
    if (k + m > 512 || len > (size_t)0x7fffffff)
        return -1;
    for (uint32_t s = 0; s < nstripes; s++) {
        strided_ptrs(k, m, base, strip_stride, stripe_stride, s, ptrs);
        if (m == 1 && k == 1) {
            memcpy(ptrs[1], ptrs[0], len); /* P = D_0 (xor_gen needs vects >= 3) */
        } else if (m == 1) {
            int rc = orc_xor_gen(k + 1, (int)len, ptrs);
            if (rc)
                return rc;
        } else if (k == 1) {
            memcpy(ptrs[1], ptrs[0], len); /* P = Q = D_0 */
            memcpy(ptrs[2], ptrs[0], len);
        } else {
            pq_any(k, len, (unsigned char **)ptrs);
        }
    }
    return 0;
}

int orc_recover_strided(int k, int m, size_t len, uint32_t nstripes,
                        uint8_t *base, size_t strip_stride, size_t stripe_stride,
                        const uint8_t *fail)
{
    void *ptrs[512];
    if (k + m > 512 || len > (size_t)0x7fffffff)
        return -1;
    for (uint32_t s = 0; s < nstripes; s++) {
        int f[2], nf = 0;
        for (int t = 0; t < 2; t++)
            if (fail[2 * (size_t)s + t] != 0xFF)
                f[nf++] = fail[2 * (size_t)s + t];
        strided_ptrs(k, m, base, strip_stride, stripe_stride, s, ptrs);
        int rc = orc_recover(k, m, (int)len, ptrs, nf, f);
        if (rc)
            return rc;
    }
    return 0;
}

/* ------------------------------------------------------- CPU baseline */

struct bench_arg {
    int impl, k, m, with_rec;
    size_t len, strip_stride, stripe_stride;
    uint32_t s0, s1;
    uint8_t *base;
    const uint8_t *fail;
    int rc;
};

static void *bench_worker(void *p)
{
    struct bench_arg *a = p;
    uint32_t n = a->s1 - a->s0;
    uint8_t *b = a->base + (size_t)a->s0 * a->stripe_stride;
    if (a->impl == 1) {
        a->rc = orc_simd_encode_strided(a->k, a->m, a->len, n, b, a->strip_stride,
                                        a->stripe_stride);
        if (!a->rc && a->with_rec)
            a->rc = orc_simd_recover_strided(a->k, a->m, a->len, n, b, a->strip_stride,
                                             a->stripe_stride, a->fail + 2 * (size_t)a->s0);
        return NULL;
    }
    a->rc = orc_encode_strided(a->k, a->m, a->len, n, b, a->strip_stride, a->stripe_stride);
    if (!a->rc && a->with_rec)
        a->rc = orc_recover_strided(a->k, a->m, a->len, n, b, a->strip_stride,
                                    a->stripe_stride, a->fail + 2 * (size_t)a->s0);
    return NULL;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double orc_bench_encode_reconstruct(int k, int m, size_t len, uint32_t nstripes,
                                    uint8_t *base, size_t strip_stride,
                                    size_t stripe_stride, const uint8_t *fail,
                                    int with_reconstruct, int nthreads,
                                    double min_seconds, uint64_t *passes)
{
    return orc_bench_encode_reconstruct_impl(0, k, m, len, nstripes, base, strip_stride,
                                             stripe_stride, fail, with_reconstruct, nthreads,
                                             min_seconds, passes);
}

/* Persistent workers: every thread runs its stripe range once per pass, then
 * meets the others at a barrier, where thread 0 decides whether to stop (thread
 * creation per pass would dominate short passes). */
struct bench_team {
    struct bench_arg *args;
    pthread_barrier_t bar;
    double t0, min_seconds, el;
    uint64_t passes;
    volatile int stop;
};

struct bench_thread {
    struct bench_team *team;
    int id;
};

static void *bench_loop(void *p)
{
    struct bench_thread *bt = p;
    struct bench_team *tm = bt->team;
    for (;;) {
        bench_worker(&tm->args[bt->id]);
        pthread_barrier_wait(&tm->bar);
        if (bt->id == 0) {
            tm->passes++;
            tm->el = now_s() - tm->t0;
            tm->stop = tm->el >= tm->min_seconds;
        }
        pthread_barrier_wait(&tm->bar);
        if (tm->stop)
            break;
    }
    return NULL;
}

double orc_bench_encode_reconstruct_impl(int impl, int k, int m, size_t len, uint32_t nstripes,
                                         uint8_t *base, size_t strip_stride,
                                         size_t stripe_stride, const uint8_t *fail,
                                         int with_reconstruct, int nthreads,
                                         double min_seconds, uint64_t *passes)
{
    if (nthreads < 1)
        nthreads = 1;
    if ((uint32_t)nthreads > nstripes)
        nthreads = (int)nstripes;
    struct bench_arg *args = calloc((size_t)nthreads, sizeof(*args));
    struct bench_thread *bt = calloc((size_t)nthreads, sizeof(*bt));
    pthread_t *th = calloc((size_t)nthreads, sizeof(*th));
    struct bench_team tm;
    if (!args || !th || !bt || pthread_barrier_init(&tm.bar, NULL, (unsigned)nthreads)) {
        free(args);
        free(th);
        free(bt);
        return -1.0;
    }
    for (int t = 0; t < nthreads; t++) {
        args[t] = (struct bench_arg){ impl, k, m, with_reconstruct, len, strip_stride,
                                      stripe_stride,
                                      (uint32_t)((uint64_t)nstripes * t / nthreads),
                                      (uint32_t)((uint64_t)nstripes * (t + 1) / nthreads),
                                      base, fail, 0 };
        bt[t] = (struct bench_thread){ &tm, t };
    }
    tm.args = args;
    tm.min_seconds = min_seconds;
    tm.passes = 0;
    tm.stop = 0;
    tm.el = 0.0;
    tm.t0 = now_s();
    for (int t = 1; t < nthreads; t++)
        pthread_create(&th[t], NULL, bench_loop, &bt[t]);
    bench_loop(&bt[0]);
    for (int t = 1; t < nthreads; t++)
        pthread_join(th[t], NULL);
    pthread_barrier_destroy(&tm.bar);
    double el = tm.el;
    for (int t = 0; t < nthreads; t++)
        if (args[t].rc)
            el = -1.0;
    free(args);
    free(th);
    free(bt);
    if (passes)
        *passes = tm.passes;
    return el;
}

/* ------------------------------------------------------------ geometry */

/* raid5.c:1006-1007: parity chunk = data_chunks_num - stripe_index % n,
 * with data_chunks_num = n - base_bdevs_max_degraded (raid5.c:161-164). */
int orc_raid5_parity_chunk(int num_base_bdevs, int max_degraded, uint64_t stripe_index)
{
    return (num_base_bdevs - max_degraded) - (int)(stripe_index % (uint64_t)num_base_bdevs);
}

/* raid5.c:172-179: data index d lives on chunk d if d < p, else d + 1. */
int orc_raid5_data_chunk_to_disk(int parity_chunk, int data_idx)
{
    return data_idx < parity_chunk ? data_idx : data_idx + 1;
}

/* raid5.c:1419-1426 (raid5_start) as checked by raid5_ut.c:176-195. */
void orc_raid5_start_geometry(int num_base_bdevs, int max_degraded, uint64_t min_blockcnt,
                              uint32_t strip_size, uint64_t *stripe_blocks,
                              uint64_t *total_stripes, uint64_t *blockcnt,
                              uint64_t *optimal_io_boundary)
{
    *total_stripes = min_blockcnt / strip_size;
    *stripe_blocks = (uint64_t)strip_size * (uint64_t)(num_base_bdevs - max_degraded);
    *blockcnt = *stripe_blocks * *total_stripes;
    *optimal_io_boundary = *stripe_blocks;
}

/* ---------------------------------------------------------- generators */

/* glibc's rand() is random() on the default 128-byte TYPE_3 state; a private
 * random_r state of the same size yields the identical sequence without being
 * disturbed by other threads of the process (the HIP runtime, torch) that also
 * draw from the global rand() state. */
static struct random_data g_rd;
static char g_rstate[128];

void orc_srand(unsigned int seed)
{
    memset(&g_rd, 0, sizeof(g_rd));
    initstate_r(seed, g_rstate, sizeof(g_rstate), &g_rd);
}

/* gf_vect_mul.c:21-26: buf[i] = rand() truncated to a byte. */
void orc_rand_buffer(unsigned char *buf, long size)
{
    for (long i = 0; i < size; i++) {
        int32_t r;
        random_r(&g_rd, &r);
        buf[i] = (unsigned char)r;
    }
}

/* The same, straight from glibc's global rand() (only for cross-checking the
 * private-state generator in a quiet process). */
void orc_glibc_srand(unsigned int seed) { srand(seed); }
void orc_glibc_rand_buffer(unsigned char *buf, long size)
{
    for (long i = 0; i < size; i++)
        buf[i] = (unsigned char)rand();
}

uint64_t orc_splitmix64(uint64_t *state)
{
    uint64_t z = (*state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

void orc_fill_splitmix(uint8_t *buf, size_t len, uint64_t seed)
{
    uint64_t st = seed;
    size_t i = 0;
    for (; i + 8 <= len; i += 8) {
        uint64_t r = orc_splitmix64(&st);
        memcpy(buf + i, &r, 8);
    }
    if (i < len) {
        uint64_t r = orc_splitmix64(&st);
        memcpy(buf + i, &r, len - i);
    }
}

/* raid5_ut_ref.c:354-357: fill 0xFF, then the 8-byte block index at the
 * start of every block. */
void orc_fill_ut_ref_pattern(uint8_t *buf, uint64_t num_blocks, uint32_t blocklen)
{
    memset(buf, 0xff, (size_t)num_blocks * blocklen);
    for (uint64_t b = 0; b < num_blocks; b++)
        memcpy(buf + b * blocklen, &b, sizeof(b));
}
