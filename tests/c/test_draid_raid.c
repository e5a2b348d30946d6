/*
 * test_draid_raid.c -- C tests of the host RAID layer over libdraid_ec.so,
 * modelled on the reference's unit tests:
 *   - raid5_ut.c:61-105,176-195: geometry over n x blockcnt x blocklen x strip grid
 *   - raid5_ut_ref.c:284-397,489-512: full-stripe writes of the 0xFF + block-index
 *     pattern through fake base bdevs that memcpy each base write into a buffer,
 *     parity checked against the oracle; non-full-stripe writes must fail.
 *   - degraded reads with every single (RAID5/6) and double (RAID6) failure.
 * `--cpu-only` runs only the host logic (geometry, request and iovec mapping).
 */
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "draid_ec.h"
#include "draid_raid.h"
#include "isal_oracle.h"

static int g_fail;
#define CHECK(c)                                                                   \
    do {                                                                           \
        if (!(c)) {                                                                \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                              \
        }                                                                          \
    } while (0)
#define HIPOK(x)                                                                         \
    do {                                                                                 \
        int _rc = (x);                                                                   \
        if (_rc) {                                                                       \
            fprintf(stderr, "%s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #x, _rc,       \
                    draid_ec_last_error());                                              \
            exit(2);                                                                     \
        }                                                                                \
    } while (0)

/* raid5_ut.c:176-195, generalised to RAID6 */
static void test_geometry(void)
{
    const int levels[] = {5, 6};
    const int ns[] = {3, 4, 5, 6, 10};
    const uint64_t blockcnts[] = {1, 1024, 1024 * 1024};
    const uint32_t bls[] = {512, 4096};
    const uint32_t skbs[] = {1, 4, 128};
    for (unsigned a = 0; a < 2; a++)
        for (unsigned b = 0; b < 5; b++)
            for (unsigned c = 0; c < 3; c++)
                for (unsigned d = 0; d < 2; d++)
                    for (unsigned e = 0; e < 3; e++) {
                        const int lvl = levels[a], n = ns[b], m = lvl == 6 ? 2 : 1;
                        const uint32_t strip = skbs[e] * 1024 / bls[d];
                        if (strip == 0 || strip > blockcnts[c])
                            continue;
                        struct draid_raid r;
                        int rc = draid_raid_start(&r, lvl, n, bls[d], strip, blockcnts[c]);
                        if (n < m + 2) {
                            CHECK(rc == -EINVAL);
                            continue;
                        }
                        CHECK(rc == 0);
                        CHECK(r.stripe_blocks == (uint64_t)strip * (n - m));
                        CHECK(r.total_stripes == blockcnts[c] / strip);
                        CHECK(r.blockcnt == (blockcnts[c] - blockcnts[c] % strip) * (n - m));
                        CHECK(r.optimal_io_boundary == r.stripe_blocks);
                        if (lvl == 5) { /* agrees with the oracle's restatement of raid5.c */
                            uint64_t sb, ts, bc, oib;
                            orc_raid5_start_geometry(n, 1, blockcnts[c], strip, &sb, &ts, &bc,
                                                     &oib);
                            CHECK(sb == r.stripe_blocks && ts == r.total_stripes &&
                                  bc == r.blockcnt && oib == r.optimal_io_boundary);
                        }
                    }
    struct draid_raid r;
    CHECK(draid_raid_start(&r, 5, 4, 512, 3, 1024) == -EINVAL); /* strip not a power of 2 */
    CHECK(draid_raid_start(&r, 0, 4, 512, 8, 1024) == -EINVAL);
}

/* Parity placement and the ut_ref request list (raid5_ut_ref.c:436-452). */
static void test_mapping(void)
{
    for (int lvl = 5; lvl <= 6; lvl++)
        for (int n = lvl == 5 ? 3 : 4; n <= 10; n++) {
            struct draid_raid r;
            const uint32_t strip = 8;
            CHECK(draid_raid_start(&r, lvl, n, 512, strip, 64 * strip) == 0);
            const int m = r.max_degraded, k = n - m;
            for (uint64_t s = 0; s < (uint64_t)2 * n; s++) {
                int p, q;
                draid_raid_parity_chunks(&r, s, &p, &q);
                if (lvl == 5) {
                    CHECK(p == orc_raid5_parity_chunk(n, 1, s));
                    for (int d = 0; d < k; d++)
                        CHECK(draid_raid_data_disk(&r, s, d) == orc_raid5_data_chunk_to_disk(p, d));
                } else {
                    CHECK(q == (p + 1) % n);
                }
                int seen[DRAID_RAID_MAX_BASE] = {0};
                for (int d = 0; d < k; d++) {
                    const int disk = draid_raid_data_disk(&r, s, d);
                    CHECK(disk >= 0 && disk != p && disk != q && !seen[disk]);
                    seen[disk] = 1;
                    CHECK(draid_raid_disk_data_index(&r, s, disk) == d);
                }
                CHECK(draid_raid_disk_data_index(&r, s, p) == -1);
            }
            const uint64_t sb = r.stripe_blocks;
            const uint64_t reqs[][2] = {{0, 1}, {0, strip}, {0, strip + 1}, {0, sb},
                                        {1, 1}, {1, strip}, {1, strip + 1}, {strip, 1},
                                        {strip, strip}, {strip - 1, 1}, {strip - 1, strip},
                                        {strip - 1, 2}};
            for (unsigned i = 0; i < sizeof(reqs) / sizeof(reqs[0]); i++) {
                for (uint64_t s = 0; s < (uint64_t)n; s++) {
                    struct draid_stripe_req q;
                    const uint64_t off = s * sb + reqs[i][0], len = reqs[i][1];
                    if (reqs[i][0] + len > sb) {
                        CHECK(draid_raid_map_request(&r, off, len, &q) == -EINVAL);
                        continue;
                    }
                    CHECK(draid_raid_map_request(&r, off, len, &q) == 0);
                    uint64_t total = 0;
                    for (int disk = 0; disk < n; disk++) {
                        total += q.chunk[disk].req_blocks;
                        CHECK(q.chunk[disk].req_offset + q.chunk[disk].req_blocks <= strip);
                    }
                    CHECK(total == len);
                    CHECK(q.chunk[q.p_disk].req_blocks == 0);
                    CHECK(q.full_stripe == (reqs[i][0] == 0 && len == sb));
                    /* the first touched chunk starts at the request offset */
                    const int fd = draid_raid_data_disk(&r, s, q.first_data);
                    CHECK(q.chunk[fd].req_offset == reqs[i][0] % strip);
                }
            }
        }
    /* raid5_chunk_map_iov over an uneven parent list */
    uint8_t buf[100];
    struct iovec par[3] = {{buf, 10}, {buf + 10, 0}, {buf + 10, 90}}, out[4];
    /* a zero-length iovec inside the range is kept, as raid5.c:384-391 counts it */
    CHECK(draid_raid_map_iov(out, 4, par, 3, 5, 20) == 3);
    CHECK(out[0].iov_base == buf + 5 && out[0].iov_len == 5);
    CHECK(out[1].iov_len == 0);
    CHECK(out[2].iov_base == buf + 10 && out[2].iov_len == 15);
    CHECK(draid_raid_map_iov(out, 4, par, 3, 10, 90) == 1);
    CHECK(draid_raid_map_iov(out, 4, par, 3, 95, 10) == -EINVAL);
    CHECK(draid_raid_map_iov(out, 1, par, 3, 0, 20) == -ENOSPC);
    CHECK(draid_raid_map_iov(out, 4, par, 3, 0, 10) == 1);
}

/* raid5_simple stripe assembly (raid5_simple.c:347-423): k strip-sized children in
 * any order -> one parent list in data order; non-strip, repeated and foreign
 * children rejected. */
static void test_stripe_asm(void)
{
    struct draid_raid r;
    CHECK(draid_raid_start(&r, 6, 6, 512, 8, 64 * 8) == 0); /* k = 4, 4 KiB strips */
    const int k = 4;
    const size_t sb = 8 * 512;
    static uint8_t buf[4 * 4096];
    struct draid_stripe_asm a;
    draid_raid_asm_init(&a);
    const uint64_t s = 5, base = s * r.stripe_blocks;
    const int order[4] = {2, 0, 3, 1};
    for (int t = 0; t < k; t++) {
        const int d = order[t];
        struct iovec ch[2] = {{buf + d * sb, 1000}, {buf + d * sb + 1000, sb - 1000}};
        if (t == 1) {
            CHECK(draid_raid_asm_add(&r, &a, base + 8 * 2, 8, ch, 2) == -EINVAL); /* repeat */
            CHECK(draid_raid_asm_add(&r, &a, base + r.stripe_blocks + 8, 8, ch, 2) == -EINVAL);
            CHECK(draid_raid_asm_add(&r, &a, base + 8 * d + 1, 7, ch, 2) == -EINVAL); /* partial */
        }
        CHECK(draid_raid_asm_add(&r, &a, base + 8 * (uint64_t)d, 8, ch, 2) == (t == k - 1));
    }
    struct iovec out[16];
    const int n = draid_raid_asm_iov(&r, &a, out, 16);
    CHECK(n == 2 * k);
    size_t off = 0;
    for (int i = 0; i < n; i++) { /* data order: one contiguous parent image */
        CHECK(out[i].iov_base == buf + off);
        off += out[i].iov_len;
    }
    CHECK(off == k * sb);
    CHECK(draid_raid_asm_iov(&r, &a, out, 3) == -ENOSPC);
    /* the assembler is free again: a new stripe starts */
    struct iovec one = {buf, sb};
    CHECK(draid_raid_asm_add(&r, &a, (s + 1) * r.stripe_blocks, 8, &one, 1) == 0);
}

/* Disk failures -> per-stripe failure pairs and the rotated pointer table. */
static void test_fail_table(void)
{
    for (int lvl = 5; lvl <= 6; lvl++) {
        struct draid_raid r;
        const int n = lvl == 5 ? 5 : 10;
        CHECK(draid_raid_start(&r, lvl, n, 4096, 16, 16 * 64) == 0);
        const int m = r.max_degraded, k = n - m;
        uint8_t f[2 * 40];
        r.degraded_mask = 0;
        CHECK(draid_raid_fail_table(&r, 3, 40, f) == 0);
        for (int i = 0; i < 80; i++)
            CHECK(f[i] == DRAID_EC_FAIL_NONE);
        const int d0 = 1, d1 = n - 2;
        r.degraded_mask = (1u << d0) | (m == 2 ? 1u << d1 : 0);
        CHECK(draid_raid_fail_table(&r, 3, 40, f) == 0);
        for (int i = 0; i < 40; i++) {
            int p, q;
            draid_raid_parity_chunks(&r, 3 + (uint64_t)i, &p, &q);
            const int want0 = d0 == p ? k : d0 == q ? k + 1 : draid_raid_disk_data_index(&r, 3 + (uint64_t)i, d0);
            CHECK(f[2 * i] == want0);
            if (m == 2) {
                const int want1 = d1 == p ? k : d1 == q ? k + 1 : draid_raid_disk_data_index(&r, 3 + (uint64_t)i, d1);
                CHECK(f[2 * i + 1] == want1);
            } else {
                CHECK(f[2 * i + 1] == DRAID_EC_FAIL_NONE);
            }
        }
        r.degraded_mask = (1u << (m + 1)) - 1;
        CHECK(draid_raid_fail_table(&r, 0, 4, f) == -EIO);
        /* pointer table: strip j of stripe s on its rotated disk at (s - first) strips */
        static uint8_t disks[10][4];
        void *base[10];
        for (int d = 0; d < n; d++)
            base[d] = disks[d];
        void *tab[10 * 6];
        CHECK(draid_raid_strip_table(&r, 7, 6, base, 5, tab) == 0);
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < n; j++) {
                int p, q;
                draid_raid_parity_chunks(&r, 7 + (uint64_t)i, &p, &q);
                const int disk = j < k ? draid_raid_data_disk(&r, 7 + (uint64_t)i, j) : (j == k ? p : q);
                CHECK(tab[i * n + j] == (uint8_t *)base[disk] + (uint64_t)(2 + i) * 16 * 4096);
            }
        CHECK(draid_raid_strip_table(&r, 4, 1, base, 5, tab) == -EINVAL);
    }
}

/* Stripe cache and request queue (raid5.c:1047-1131, 485-521). */
static void test_stripe_slot_bytes(void)
{
    /* plain n * strip unless that is a multiple of 512 KiB */
    CHECK(draid_stripe_slot_bytes(10, 65536) == 10u * 65536);
    CHECK(draid_stripe_slot_bytes(5, 65536) == 5u * 65536);
    CHECK(draid_stripe_slot_bytes(18, 262144) == 18u * 262144);
    CHECK(draid_stripe_slot_bytes(8, 65536) == 8u * 65536 + 16384);
    CHECK(draid_stripe_slot_bytes(16, 65536) == 16u * 65536 + 16384);
    CHECK(draid_stripe_slot_bytes(4, 131072) == 4u * 131072 + 16384);
    CHECK(draid_stripe_slot_bytes(6, 4096) == 6u * 4096);
    CHECK(draid_stripe_slot_bytes(128, 4096) == 128u * 4096 + 16384);
    CHECK(draid_stripe_slot_bytes(4, 262144) == 4u * 262144);   /* P and Q a half each */
    printf("ok stripe slot stride\n");
}

static void test_stripe_cache(void)
{
    draid_stripe_cache *c;
    CHECK(draid_stripe_cache_create(&c, 0) == -EINVAL);
    CHECK(draid_stripe_cache_create(&c, 16) == 0);
    struct draid_stripe *a = draid_stripe_get(c, 7), *b = draid_stripe_get(c, 7);
    CHECK(a && a == b && a->index == 7 && a->slot < 16); /* one entry per stripe, two refs */
    CHECK(draid_stripe_cache_active(c) == 1);
    /* request queue: first runs at once, the others wait in arrival order */
    struct draid_stripe_waiter w[3];
    CHECK(draid_stripe_enqueue(c, a, &w[0]) == 1);
    CHECK(draid_stripe_enqueue(c, a, &w[1]) == 0);
    CHECK(draid_stripe_enqueue(c, a, &w[2]) == 0);
    CHECK(draid_stripe_complete(c, a, &w[0]) == &w[1]);
    CHECK(draid_stripe_complete(c, a, &w[2]) == NULL); /* a non-head leaves quietly */
    CHECK(draid_stripe_complete(c, a, &w[1]) == NULL);
    CHECK(draid_stripe_enqueue(c, a, &w[0]) == 1);
    CHECK(draid_stripe_complete(c, a, &w[0]) == NULL);
    draid_stripe_put(c, a);
    draid_stripe_put(c, b);
    /* fill every slot with referenced stripes: the next miss has nothing to reclaim */
    struct draid_stripe *held[16];
    int slots_seen[16] = {0};
    for (int i = 0; i < 16; i++) {
        held[i] = draid_stripe_get(c, 100 + (uint64_t)i);
        CHECK(held[i] != NULL);
        if (held[i])
            slots_seen[held[i]->slot]++;
    }
    for (int i = 0; i < 16; i++)
        CHECK(slots_seen[i] == 1);
    CHECK(draid_stripe_get(c, 999) == NULL);
    /* release the four least recently used: a miss reclaims from the LRU end */
    for (int i = 0; i < 4; i++)
        draid_stripe_put(c, held[i]);
    struct draid_stripe *n1 = draid_stripe_get(c, 999);
    CHECK(n1 != NULL && n1->index == 999);
    CHECK(draid_stripe_cache_active(c) <= 16);
    for (int i = 4; i < 16; i++) /* still-referenced entries were never reclaimed */
        CHECK(draid_stripe_get(c, 100 + (uint64_t)i) == held[i]);
    draid_stripe_cache_destroy(c);
}

/* Many threads issuing requests on a few hot stripes: per stripe at most one
 * request runs at a time, none is lost, and every entry is released. */
enum { ST_THREADS = 8, ST_REQS = 20000, ST_STRIPES = 12, ST_SLOTS = 8 };
struct st_req {
    struct draid_stripe_waiter w;
    struct draid_stripe *s;
    int done;
};
static draid_stripe_cache *g_sc;
static int g_running[ST_STRIPES];
static long g_completed;
static int g_violations;

static void st_run(struct st_req *r) /* the "stripe request" body */
{
    const uint64_t idx = r->s->index;
    if (__atomic_add_fetch(&g_running[idx], 1, __ATOMIC_SEQ_CST) != 1)
        __atomic_add_fetch(&g_violations, 1, __ATOMIC_SEQ_CST);
    for (volatile int spin = 0; spin < 200; spin++) /* hold the stripe a little while */
        ;
    __atomic_sub_fetch(&g_running[idx], 1, __ATOMIC_SEQ_CST);
}

static void *st_thread(void *arg)
{
    uint64_t rng = 0x1234 + (uint64_t)(uintptr_t)arg;
    static __thread struct st_req reqs[64];
    for (int i = 0; i < ST_REQS; i++) {
        struct st_req *r = &reqs[i % 64];
        /* its previous request may still wait in a stripe queue: the thread walking
         * that queue runs it (nothing blocks), then the slot is free again */
        while (i >= 64 && !__atomic_load_n(&r->done, __ATOMIC_ACQUIRE))
            ;
        r->done = 0;
        const uint64_t idx = orc_splitmix64(&rng) % ST_STRIPES;
        struct draid_stripe *s;
        while (!(s = draid_stripe_get(g_sc, idx))) /* every entry referenced: retry */
            ;
        r->s = s;
        r->w.arg = r;
        if (draid_stripe_enqueue(g_sc, s, &r->w) != 1)
            continue; /* queued behind a running request; its runner will run this one */
        /* run the head, then every request it hands on to (this thread's or others') */
        for (struct draid_stripe_waiter *w = &r->w; w;) {
            struct st_req *x = w->arg;
            st_run(x);
            struct draid_stripe_waiter *next = draid_stripe_complete(g_sc, x->s, w);
            draid_stripe_put(g_sc, x->s);
            __atomic_add_fetch(&g_completed, 1, __ATOMIC_SEQ_CST);
            __atomic_store_n(&x->done, 1, __ATOMIC_RELEASE);
            w = next;
        }
    }
    for (int i = 0; i < 64; i++) /* drain before the thread-local requests go away */
        while (!__atomic_load_n(&reqs[i].done, __ATOMIC_ACQUIRE))
            ;
    return NULL;
}

static void test_stripe_cache_threads(void)
{
    CHECK(draid_stripe_cache_create(&g_sc, ST_SLOTS) == 0);
    pthread_t t[ST_THREADS];
    for (int i = 0; i < ST_THREADS; i++)
        pthread_create(&t[i], NULL, st_thread, (void *)(uintptr_t)i);
    for (int i = 0; i < ST_THREADS; i++)
        pthread_join(t[i], NULL);
    CHECK(g_completed == (long)ST_THREADS * ST_REQS);
    CHECK(g_violations == 0);
    /* every reference released: all stripes reclaimable, so fresh ones fit */
    for (uint64_t i = 0; i < 3 * ST_SLOTS; i++) {
        struct draid_stripe *s = draid_stripe_get(g_sc, 1000 + i);
        CHECK(s != NULL);
        draid_stripe_put(g_sc, s);
    }
    draid_stripe_cache_destroy(g_sc);
}

/* ---------------------------------------------------------------- GPU tests */

static void d2d(void *dst, const void *src, size_t n, void *st)
{
    HIPOK(draid_ec_memcpy_async(dst, src, n, 2, st));
}

static int cmp_host(const uint8_t *a, const uint8_t *b, size_t n) { return memcmp(a, b, n) == 0; }

static void run_array(int lvl, int n, uint32_t blocklen, uint32_t strip_kb)
{
    struct draid_raid r;
    const uint32_t strip = strip_kb * 1024 / blocklen;
    const uint64_t nstripes = (uint64_t)n + 1;
    CHECK(draid_raid_start(&r, lvl, n, blocklen, strip, strip * nstripes) == 0);
    const int m = r.max_degraded, k = n - m;
    const size_t sb = (size_t)strip * blocklen, disk_bytes = sb * r.total_stripes;
    const size_t ub = (size_t)r.stripe_blocks * blocklen;

    draid_ec_ctx *ctx;
    HIPOK(draid_ec_ctx_create(&ctx));
    void *st = draid_ec_ctx_stream(ctx);
    uint8_t *disk[DRAID_RAID_MAX_BASE], *user, *pbuf[2], *chunk[DRAID_RAID_MAX_BASE], *junk;
    for (int d = 0; d < n; d++) {
        HIPOK(draid_ec_device_alloc((void **)&disk[d], disk_bytes));
        HIPOK(draid_ec_device_alloc((void **)&chunk[d], sb));
    }
    HIPOK(draid_ec_device_alloc((void **)&user, ub * r.total_stripes));
    HIPOK(draid_ec_device_alloc((void **)&pbuf[0], sb));
    HIPOK(draid_ec_device_alloc((void **)&pbuf[1], sb));
    HIPOK(draid_ec_device_alloc((void **)&junk, sb));

    /* user data: the raid5_ut_ref pattern, one new payload per stripe */
    uint8_t *hu = malloc(ub * r.total_stripes), *hj = malloc(sb);
    for (uint64_t s = 0; s < r.total_stripes; s++) {
        orc_fill_ut_ref_pattern(hu + s * ub, r.stripe_blocks, blocklen);
        hu[s * ub + 9] = (uint8_t)s;
    }
    memset(hj, 0xA5, sb);
    HIPOK(draid_ec_memcpy_async(user, hu, ub * r.total_stripes, 0, st));
    HIPOK(draid_ec_memcpy_async(junk, hj, sb, 0, st));

    for (uint64_t s = 0; s < r.total_stripes; s++) {
        struct draid_stripe_req q;
        CHECK(draid_raid_map_request(&r, s * r.stripe_blocks, r.stripe_blocks, &q) == 0);
        CHECK(q.full_stripe);
        /* the parent I/O arrives as three uneven iovecs */
        uint8_t *u = user + s * ub;
        const size_t a = ub / 3 + 7, b = ub / 5 + 1;
        struct iovec iov[3] = {{u, a}, {u + a, b}, {u + a + b, ub - a - b}};
        struct draid_base_io w[DRAID_RAID_MAX_BASE];
        int nw = 0;
        void *pq[2] = {pbuf[0], pbuf[1]};
        if (s & 1) { /* raid5_simple shape: k strip-sized children, last data chunk first */
            static struct draid_stripe_asm sa;
            draid_raid_asm_init(&sa);
            for (int d = k - 1; d >= 0; d--) {
                struct iovec ch[2] = {{u + d * sb, sb / 2}, {u + d * sb + sb / 2, sb - sb / 2}};
                CHECK(draid_raid_asm_add(&r, &sa, s * r.stripe_blocks + (uint64_t)d * strip, strip,
                                         ch, 2) == (d == 0));
            }
            struct iovec full[2 * DRAID_RAID_MAX_BASE];
            const int nf = draid_raid_asm_iov(&r, &sa, full, 2 * DRAID_RAID_MAX_BASE);
            CHECK(nf == 2 * k);
            CHECK(draid_raid_stripe_write(&r, ctx, &q, full, nf, pq, w, &nw) == 0);
        } else {
            CHECK(draid_raid_stripe_write(&r, ctx, &q, iov, 3, pq, w, &nw) == 0);
        }
        CHECK(nw == n);
        HIPOK(draid_ec_ctx_flush(ctx));
        /* fake base bdevs: memcpy every base write (raid5_ut_ref.c:284-323) */
        for (int i = 0; i < nw; i++) {
            size_t off = (size_t)w[i].offset_blocks * blocklen;
            for (int v = 0; v < w[i].iovcnt; v++) {
                d2d(disk[w[i].disk] + off, w[i].iov[v].iov_base, w[i].iov[v].iov_len, st);
                off += w[i].iov[v].iov_len;
            }
            CHECK(off == (size_t)(w[i].offset_blocks + w[i].num_blocks) * blocklen);
        }
        HIPOK(draid_ec_ctx_synchronize(ctx));
        /* non-full-stripe writes are rejected (raid5_ut_ref.c:489-512) */
        struct draid_stripe_req pr;
        CHECK(draid_raid_map_request(&r, s * r.stripe_blocks + 1, strip, &pr) == 0);
        CHECK(draid_raid_stripe_write(&r, ctx, &pr, iov, 3, pq, w, &nw) == -EINVAL);
    }

    /* partial-stripe writes: the RMW / RCW vote, prereads, parity update, writes */
    uint8_t *pre[DRAID_RAID_MAX_BASE], *nub;
    for (int d = 0; d < n; d++)
        HIPOK(draid_ec_device_alloc((void **)&pre[d], sb));
    HIPOK(draid_ec_device_alloc((void **)&nub, ub));
    uint8_t *hn = malloc(ub);
    uint64_t rng = 0x9e3779b97f4a7c15ull ^ (uint64_t)(n * 131 + lvl);
    int modes[3] = {0, 0, 0};
    for (int t = 0; t < 24; t++) {
        const uint64_t s = orc_splitmix64(&rng) % r.total_stripes;
        const uint64_t off = orc_splitmix64(&rng) % r.stripe_blocks;
        uint64_t len = 1 + orc_splitmix64(&rng) % (r.stripe_blocks - off);
        if (t % 4 == 0) /* some single-chunk requests */
            len = 1 + (orc_splitmix64(&rng) % (strip - off % strip));
        if (off == 0 && len == r.stripe_blocks)
            continue;
        orc_fill_splitmix(hn, len * blocklen, orc_splitmix64(&rng));
        HIPOK(draid_ec_memcpy_async(nub, hn, len * blocklen, 0, st));
        struct draid_stripe_req q;
        CHECK(draid_raid_map_request(&r, s * r.stripe_blocks + off, len, &q) == 0);
        CHECK(!q.full_stripe);
        struct draid_write_plan plan;
        struct draid_base_io io[2 * DRAID_RAID_MAX_BASE];
        int nio = 0;
        CHECK(draid_raid_plan_write(&r, &q, &plan, (void *const *)pre, io, &nio) == 0);
        modes[plan.mode]++;
        for (int i = 0; i < nio; i++) /* fake base prereads */
            d2d(io[i].iov[0].iov_base, disk[io[i].disk] + io[i].offset_blocks * blocklen,
                io[i].num_blocks * blocklen, st);
        const size_t half = (len * blocklen) / 2;
        struct iovec uiov[2] = {{nub, half}, {nub + half, len * blocklen - half}};
        CHECK(draid_raid_stripe_write_partial(&r, ctx, &q, &plan, uiov, 2, (void *const *)pre, io,
                                              &nio) == 0);
        HIPOK(draid_ec_ctx_flush(ctx));
        for (int i = 0; i < nio; i++) { /* fake base writes (stream-ordered after the kernel) */
            size_t o = (size_t)io[i].offset_blocks * blocklen;
            for (int v = 0; v < io[i].iovcnt; v++) {
                d2d(disk[io[i].disk] + o, io[i].iov[v].iov_base, io[i].iov[v].iov_len, st);
                o += io[i].iov[v].iov_len;
            }
        }
        HIPOK(draid_ec_ctx_synchronize(ctx));
        memcpy(hu + s * ub + off * blocklen, hn, len * blocklen);
    }
    if (k >= 3)
        CHECK(modes[DRAID_WRITE_RMW] > 0 && modes[DRAID_WRITE_RCW] > 0);
    for (int d = 0; d < n; d++)
        draid_ec_device_free(pre[d]);
    draid_ec_device_free(nub);
    free(hn);

    /* every stripe on the fake disks: data in place, parity == oracle */
    uint8_t *hd[DRAID_RAID_MAX_BASE];
    for (int d = 0; d < n; d++) {
        hd[d] = malloc(disk_bytes);
        HIPOK(draid_ec_memcpy_async(hd[d], disk[d], disk_bytes, 1, st));
    }
    HIPOK(draid_ec_ctx_synchronize(ctx));
    uint8_t *ref = malloc(sb * 2);
    for (uint64_t s = 0; s < r.total_stripes; s++) {
        int p, qd;
        draid_raid_parity_chunks(&r, s, &p, &qd);
        void *vec[DRAID_RAID_MAX_BASE + 2];
        for (int d = 0; d < k; d++) {
            const int disk_i = draid_raid_data_disk(&r, s, d);
            CHECK(cmp_host(hd[disk_i] + s * sb, hu + s * ub + d * sb, sb));
            vec[d] = hu + s * ub + d * sb;
        }
        vec[k] = ref;
        vec[k + 1] = ref + sb;
        CHECK((m == 1 ? orc_xor_gen(k + 1, (int)sb, vec) : orc_pq_gen(k + 2, (int)sb, vec)) == 0);
        CHECK(cmp_host(hd[p] + s * sb, ref, sb));
        if (m == 2)
            CHECK(cmp_host(hd[qd] + s * sb, ref + sb, sb));
    }

    /* degraded reads: every single failure, and every double failure for RAID6 */
    uint8_t *hc = malloc(sb);
    for (int f0 = 0; f0 < n; f0++)
        for (int f1 = (m == 2 ? f0 : n); f1 <= n; f1++) {
            if (f1 == f0 && f1 != n)
                continue;
            r.degraded_mask = (1u << f0) | (f1 < n ? (1u << f1) : 0);
            const uint64_t s = (uint64_t)(f0 + f1) % r.total_stripes;
            struct draid_base_io rd[DRAID_RAID_MAX_BASE];
            int nr = 0;
            for (int d = 0; d < n; d++)
                d2d(chunk[d], junk, sb, st); /* degraded chunks start as garbage */
            /* odd f0: the two-phase form (plan, base reads, then the rebuild) */
            const int two = f0 & 1;
            CHECK(draid_raid_stripe_degraded_read(&r, two ? NULL : ctx, s, (void *const *)chunk, rd,
                                                  &nr) == 0);
            CHECK(nr == n - (f1 < n ? 2 : 1));
            for (int i = 0; i < nr; i++) /* fake base reads */
                d2d(rd[i].iov[0].iov_base, disk[rd[i].disk] + rd[i].offset_blocks * blocklen, sb,
                    st);
            if (two)
                CHECK(draid_raid_stripe_degraded_rebuild(&r, ctx, s, (void *const *)chunk) == 0);
            HIPOK(draid_ec_ctx_flush(ctx));
            HIPOK(draid_ec_ctx_synchronize(ctx));
            for (int d = 0; d < n; d++) {
                HIPOK(draid_ec_memcpy_async(hc, chunk[d], sb, 1, st));
                HIPOK(draid_ec_ctx_synchronize(ctx));
                CHECK(cmp_host(hc, hd[d] + s * sb, sb));
            }
        }
    /* more failures than the level tolerates */
    r.degraded_mask = (1u << (m + 1)) - 1;
    struct draid_base_io rd[DRAID_RAID_MAX_BASE];
    int nr;
    CHECK(draid_raid_stripe_degraded_read(&r, ctx, 0, (void *const *)chunk, rd, &nr) == -EIO);

    /* ranged reads (raid5_stripe_read): the reference's read request grid
     * (raid5_ut_ref.c:439-463) on the first min(n, stripes) stripes plus random
     * requests, each healthy, with one and (RAID6) two degraded disks, and with
     * one more than the level tolerates; the bytes must arrive in the parent
     * iovecs exactly as the writes above left them. */
    uint8_t *ubuf, *ujunk, *hr = malloc(ub);
    HIPOK(draid_ec_device_alloc((void **)&ubuf, ub));
    HIPOK(draid_ec_device_alloc((void **)&ujunk, ub));
    memset(hr, 0x5A, ub);
    HIPOK(draid_ec_memcpy_async(ujunk, hr, ub, 0, st));
    static struct draid_base_io rio[3 * DRAID_RAID_MAX_BASE];
    const uint64_t grid[][2] = {{0, 1},          {0, strip},          {0, strip + 1},
                                {0, r.stripe_blocks}, {1, 1},          {1, strip},
                                {1, strip + 1},  {strip, 1},          {strip, strip},
                                {strip, strip + 1}, {strip - 1, 1},   {strip - 1, strip},
                                {strip - 1, strip + 1}, {strip - 1, 2}};
    const int ngrid = (int)(sizeof(grid) / sizeof(grid[0]));
    const uint64_t ns = r.total_stripes < (uint64_t)n ? r.total_stripes : (uint64_t)n;
    int rebuilt = 0, refused = 0, nreq = 0;
    for (int t = 0; t < ngrid * (int)ns + 64; t++) {
        uint64_t s, off, len;
        if (t < ngrid * (int)ns) {
            s = (uint64_t)(t % (int)ns);
            off = grid[t / (int)ns][0];
            len = grid[t / (int)ns][1];
            if (off + len > r.stripe_blocks)
                continue;
        } else {
            s = orc_splitmix64(&rng) % r.total_stripes;
            off = orc_splitmix64(&rng) % r.stripe_blocks;
            len = 1 + orc_splitmix64(&rng) % (r.stripe_blocks - off);
        }
        struct draid_stripe_req q;
        CHECK(draid_raid_map_request(&r, s * r.stripe_blocks + off, len, &q) == 0);
        const size_t nb = len * blocklen, h = nb / 3;
        struct iovec uiov[3] = {{ubuf, h}, {ubuf + h, 0}, {ubuf + h, nb - h}};
        for (int nd = 0; nd <= m + 1; nd++) {
            uint32_t mask = 0;
            while (__builtin_popcount(mask) < nd)
                mask |= 1u << (orc_splitmix64(&rng) % (uint64_t)n);
            if (nd == 1) /* always a rebuild */
                mask = 1u << draid_raid_data_disk(&r, s, q.first_data);
            r.degraded_mask = mask;
            int lost_req = 0;
            for (int disk = 0; disk < n; disk++)
                if ((mask >> disk & 1u) && disk != q.p_disk && disk != q.q_disk &&
                    q.chunk[disk].req_blocks)
                    lost_req = 1;
            for (int d = 0; d < n; d++)
                d2d(chunk[d], junk, sb, st);
            d2d(ubuf, ujunk, nb, st);
            int nio = -1;
            const int two = t & 1; /* odd t: plan the reads, rebuild after they are in */
            const int rc = draid_raid_stripe_read(&r, two ? NULL : ctx, &q, uiov, 3,
                                                  (void *const *)chunk, rio, &nio);
            nreq++;
            if (lost_req && nd > m) {
                CHECK(rc == -EIO);
                refused++;
                continue;
            }
            CHECK(rc == 0);
            if (rc)
                continue;
            rebuilt += lost_req;
            CHECK(nio <= 3 * n);
            for (int i = 0; i < nio; i++) { /* fake base reads */
                CHECK(!(mask & (1u << rio[i].disk)));
                size_t o = (size_t)rio[i].offset_blocks * blocklen;
                for (int v = 0; v < rio[i].iovcnt; v++) {
                    if (rio[i].iov[v].iov_len)
                        d2d(rio[i].iov[v].iov_base, disk[rio[i].disk] + o, rio[i].iov[v].iov_len,
                            st);
                    o += rio[i].iov[v].iov_len;
                }
                CHECK(o == (size_t)(rio[i].offset_blocks + rio[i].num_blocks) * blocklen);
            }
            if (two)
                CHECK(draid_raid_stripe_read_rebuild(&r, ctx, &q, uiov, 3, (void *const *)chunk) ==
                      0);
            HIPOK(draid_ec_ctx_flush(ctx));
            HIPOK(draid_ec_ctx_synchronize(ctx));
            HIPOK(draid_ec_memcpy_async(hr, ubuf, nb, 1, st));
            HIPOK(draid_ec_ctx_synchronize(ctx));
            CHECK(cmp_host(hr, hu + s * ub + off * blocklen, nb));
        }
    }
    CHECK(rebuilt > 0 && refused > 0);
    r.degraded_mask = 0;
    draid_ec_device_free(ubuf);
    draid_ec_device_free(ujunk);
    free(hr);

    for (int d = 0; d < n; d++) {
        draid_ec_device_free(disk[d]);
        draid_ec_device_free(chunk[d]);
        free(hd[d]);
    }
    draid_ec_device_free(user);
    draid_ec_device_free(pbuf[0]);
    draid_ec_device_free(pbuf[1]);
    draid_ec_device_free(junk);
    free(hu);
    free(hj);
    free(ref);
    free(hc);
    draid_ec_ctx_destroy(ctx);
    printf("  raid%d n=%d blocklen=%u strip=%uKiB (partial writes rmw=%d rcw=%d; ranged reads %d, "
           "%d rebuilt, %d refused): %s\n",
           lvl, n, blocklen, strip_kb, modes[DRAID_WRITE_RMW], modes[DRAID_WRITE_RCW], nreq,
           rebuilt, refused, g_fail ? "FAIL" : "ok");
}

/* Rebuild of failed disks held in device memory: encode every stripe of an
 * array through the rotated pointer table, erase one (or two) disks, rebuild them
 * with one batched reconstruct driven by the per-stripe failure table. */
static void run_rebuild(int lvl, int n, uint32_t strip_kb, uint64_t nstripes)
{
    struct draid_raid r;
    const uint32_t strip = strip_kb * 1024 / 4096;
    CHECK(draid_raid_start(&r, lvl, n, 4096, strip, strip * nstripes) == 0);
    const int m = r.max_degraded, k = n - m;
    const size_t sb = (size_t)strip * 4096, db = sb * nstripes;
    void *st;
    HIPOK(draid_ec_stream_create(&st));
    uint8_t *disk[DRAID_RAID_MAX_BASE], *hd[DRAID_RAID_MAX_BASE];
    uint8_t *zero = calloc(1, db), *tmp = malloc(db);
    for (int d = 0; d < n; d++) {
        HIPOK(draid_ec_device_alloc((void **)&disk[d], db));
        hd[d] = malloc(db);
        orc_fill_splitmix(hd[d], db, 0x5eed + (uint64_t)d); /* data, and garbage parity */
        HIPOK(draid_ec_memcpy_async(disk[d], hd[d], db, 0, st));
    }
    void **tab = malloc(sizeof(void *) * n * nstripes), **dtab;
    uint8_t *fail = malloc(2 * nstripes), *dfail;
    HIPOK(draid_ec_device_alloc((void **)&dtab, sizeof(void *) * n * nstripes));
    HIPOK(draid_ec_device_alloc((void **)&dfail, 2 * nstripes));
    CHECK(draid_raid_strip_table(&r, 0, (uint32_t)nstripes, (void *const *)disk, 0, tab) == 0);
    HIPOK(draid_ec_memcpy_async(dtab, tab, sizeof(void *) * n * nstripes, 0, st));
    draid_ec_stripe_batch b = {(uint32_t)k, (uint32_t)m, sb, (uint32_t)nstripes, 0, dtab};
    HIPOK(draid_ec_encode(&b, st));
    for (int d = 0; d < n; d++)
        HIPOK(draid_ec_memcpy_async(hd[d], disk[d], db, 1, st));
    HIPOK(draid_ec_stream_synchronize(st));
    /* parity on the disks == oracle, for a sample of stripes */
    uint8_t *ref = malloc(2 * sb);
    for (uint64_t s = 0; s < nstripes; s += 1 + nstripes / 7) {
        int p, q;
        draid_raid_parity_chunks(&r, s, &p, &q);
        void *vec[DRAID_RAID_MAX_BASE];
        for (int j = 0; j < k; j++)
            vec[j] = hd[draid_raid_data_disk(&r, s, j)] + s * sb;
        vec[k] = ref;
        vec[k + 1] = ref + sb;
        CHECK((m == 1 ? orc_xor_gen(k + 1, (int)sb, vec) : orc_pq_gen(k + 2, (int)sb, vec)) == 0);
        CHECK(cmp_host(hd[p] + s * sb, ref, sb));
        if (m == 2)
            CHECK(cmp_host(hd[q] + s * sb, ref + sb, sb));
    }
    /* fail every disk alone, and (RAID6) a few pairs: erase, rebuild, compare */
    int sets = 0;
    for (int f0 = 0; f0 < n; f0++)
        for (int f1 = (m == 2 ? f0 + 1 : n); f1 <= n; f1 += (m == 2 ? 3 : 1)) {
            r.degraded_mask = (1u << f0) | (f1 < n ? 1u << f1 : 0);
            CHECK(draid_raid_fail_table(&r, 0, (uint32_t)nstripes, fail) == 0);
            HIPOK(draid_ec_memcpy_async(dfail, fail, 2 * nstripes, 0, st));
            HIPOK(draid_ec_memcpy_async(disk[f0], zero, db, 0, st));
            if (f1 < n)
                HIPOK(draid_ec_memcpy_async(disk[f1], zero, db, 0, st));
            HIPOK(draid_ec_reconstruct(&b, dfail, st));
            for (int t = 0; t < 2; t++) {
                const int f = t ? f1 : f0;
                if (f >= n)
                    continue;
                HIPOK(draid_ec_memcpy_async(tmp, disk[f], db, 1, st));
                HIPOK(draid_ec_stream_synchronize(st));
                CHECK(cmp_host(tmp, hd[f], db));
            }
            sets++;
        }
    r.degraded_mask = 0;
    printf("  rebuild raid%d n=%d strip=%uKiB stripes=%llu: %d failure sets %s\n", lvl, n, strip_kb,
           (unsigned long long)nstripes, sets, g_fail ? "FAIL" : "ok");
    for (int d = 0; d < n; d++) {
        draid_ec_device_free(disk[d]);
        free(hd[d]);
    }
    draid_ec_device_free(dtab);
    draid_ec_device_free(dfail);
    draid_ec_stream_destroy(st);
    free(tab);
    free(fail);
    free(zero);
    free(tmp);
    free(ref);
}

int main(int argc, char **argv)
{
    const int cpu_only = argc > 1 && strcmp(argv[1], "--cpu-only") == 0;
    setvbuf(stdout, NULL, _IOLBF, 0); /* results survive a runtime teardown failure */
    test_geometry();
    test_mapping();
    test_stripe_asm();
    test_fail_table();
    test_stripe_slot_bytes();
    test_stripe_cache();
    test_stripe_cache_threads();
    printf("host logic: %s\n", g_fail ? "FAIL" : "ok");
    if (!cpu_only) {
        const int cfg[][4] = {{5, 3, 512, 4},  {5, 4, 4096, 4},  {5, 5, 512, 64}, {5, 5, 4096, 64},
                              {6, 4, 512, 4},  {6, 6, 4096, 64}, {6, 10, 4096, 64}, {6, 18, 4096, 4}};
        for (unsigned i = 0; i < sizeof(cfg) / sizeof(cfg[0]); i++)
            run_array(cfg[i][0], cfg[i][1], (uint32_t)cfg[i][2], (uint32_t)cfg[i][3]);
        run_rebuild(5, 5, 64, 40);
        run_rebuild(6, 10, 64, 30);
        run_rebuild(6, 18, 16, 37);
    }
    printf("%s (%d failures)\n", g_fail ? "FAIL" : "PASS", g_fail);
    return g_fail ? 1 : 0;
}
