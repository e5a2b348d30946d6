/*
 * bdevperf_gpu.c -- BASELINE config 1 with the GPU engine: RAID5 4+1
 * full-stripe writes of 256 KiB (64 KiB strips) over 5 RAM disks, queue depth 32,
 * driven the way an SPDK raid module on libdraid_ec would run them.
 *
 * The reference workload is bdevperf -w write -o 262144 -q 32 over a raid5 bdev
 * of 5 malloc bdevs; bdevperf itself needs SPDK + DPDK + isa-l and
 * is not buildable here, and oracle/bdevperf_raid5.c is its CPU counterpart (parity
 * by the isa-l xor_gen restatement on the reactor core).  Here the same requests
 * take the raid module's path through the host layer on one "reactor" thread:
 *   - user buffers and parity buffers are host memory registered once
 *     (draid_ec_host_register, as spdk_dma_malloc hugepages would be) and handed
 *     to the engine through their device addresses (draid_ec_host_device_pointer);
 *   - each 256 KiB write is mapped (draid_raid_map_request, raid5_handle_stripe)
 *     and queued (draid_raid_stripe_write: the iovec slicing of raid5_chunk_map_iov
 *     and the parity encode on a draid_ec_ctx); the I/Os of a group share one
 *     flush, i.e. one kernel that reads the data over PCIe in place and writes P;
 *   - a poller loop checks draid_ec_ctx_query (never blocks) and, for a finished
 *     group, issues the base writes = the malloc bdev's memcpy of every strip into
 *     its RAM disk (bdev_malloc.c:173-200), completes the I/Os and resubmits them.
 * Several groups (contexts) are in flight so the GPU encodes one while the core
 * copies another.  MiB/s = user bytes written / elapsed (bdevperf.c:244-249).
 *
 *   bdevperf_gpu [seconds=10] [qd=32] [groups=2]
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "draid_ec.h"
#include "draid_raid.h"

#define NDISK 5
#define BLOCKLEN 4096u
#define STRIP_BYTES (64u * 1024u)
#define MAX_GROUPS 16

struct io {
    uint64_t stripe;
    struct draid_base_io w[DRAID_RAID_MAX_BASE];
    int nw;
};

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

#define OK(x)                                                                               \
    do {                                                                                    \
        int _rc = (x);                                                                      \
        if (_rc) {                                                                          \
            fprintf(stderr, "%s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #x, _rc,          \
                    draid_ec_last_error());                                                 \
            exit(2);                                                                        \
        }                                                                                   \
    } while (0)

static struct draid_raid g_r;
static uint8_t *g_disk[NDISK];
static uint8_t *g_user_h, *g_user_d, *g_par_h, *g_par_d;
static size_t g_io_bytes, g_user_len, g_par_len;
static uint64_t g_next_stripe;

static void *to_host(void *dev)
{
    uint8_t *p = dev;
    if (p >= g_user_d && p < g_user_d + g_user_len)
        return g_user_h + (p - g_user_d);
    return g_par_h + (p - g_par_d);
}

/* Queue the group's writes on its context and launch them. */
static void submit(draid_ec_ctx *ctx, struct io *ios, int first, int count)
{
    for (int i = first; i < first + count; i++) {
        struct io *io = &ios[i];
        io->stripe = g_next_stripe++ % g_r.total_stripes;
        g_user_h[(size_t)i * g_io_bytes + (io->stripe * 64) % g_io_bytes] ^= 1; /* new payload */
        struct draid_stripe_req req;
        OK(draid_raid_map_request(&g_r, io->stripe * g_r.stripe_blocks, g_r.stripe_blocks, &req));
        struct iovec iov = {g_user_d + (size_t)i * g_io_bytes, g_io_bytes};
        void *pq[2] = {g_par_d + (size_t)i * STRIP_BYTES, NULL};
        OK(draid_raid_stripe_write(&g_r, ctx, &req, &iov, 1, pq, io->w, &io->nw));
    }
    OK(draid_ec_ctx_flush(ctx));
}

/* Base writes of a finished group: the malloc bdev's memcpy per strip. */
static void complete(struct io *ios, int first, int count)
{
    for (int i = first; i < first + count; i++)
        for (int j = 0; j < ios[i].nw; j++) {
            const struct draid_base_io *w = &ios[i].w[j];
            uint8_t *dst = g_disk[w->disk] + w->offset_blocks * BLOCKLEN;
            for (int v = 0; v < w->iovcnt; v++) {
                memcpy(dst, to_host(w->iov[v].iov_base), w->iov[v].iov_len);
                dst += w->iov[v].iov_len;
            }
        }
}

int main(int argc, char **argv)
{
    const double seconds = argc > 1 ? atof(argv[1]) : 10.0;
    const int qd = argc > 2 ? atoi(argv[2]) : 32;
    int groups = argc > 3 ? atoi(argv[3]) : 2;
    const size_t disk_bytes = (size_t)1 << 30;
    if (qd < 1 || groups < 1 || groups > MAX_GROUPS || qd % groups)
        return fprintf(stderr, "qd must be a multiple of groups (<= %d)\n", MAX_GROUPS), 1;
    const int per = qd / groups;

    OK(draid_raid_start(&g_r, 5, NDISK, BLOCKLEN, STRIP_BYTES / BLOCKLEN, disk_bytes / BLOCKLEN));
    g_io_bytes = (size_t)g_r.stripe_blocks * BLOCKLEN; /* 256 KiB */
    for (int d = 0; d < NDISK; d++) {
        g_disk[d] = aligned_alloc(4096, disk_bytes);
        if (!g_disk[d])
            return 1;
        memset(g_disk[d], 0, disk_bytes);
    }
    g_user_len = (size_t)qd * g_io_bytes;
    g_par_len = (size_t)qd * STRIP_BYTES;
    g_user_h = aligned_alloc(1 << 21, g_user_len);
    g_par_h = aligned_alloc(1 << 21, g_par_len);
    if (!g_user_h || !g_par_h)
        return 1;
    uint64_t x = 0x1234;
    for (size_t b = 0; b < g_user_len; b += 8) { /* xorshift payload */
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        memcpy(g_user_h + b, &x, 8);
    }
    memset(g_par_h, 0, g_par_len);
    /* hosts whose GPU runtime refuses to register existing memory: the same buffers
     * from the runtime's own pinned allocator instead (what a module does there) */
    int registered = 1;
    if (draid_ec_host_register(g_user_h, g_user_len) != 0) {
        uint8_t *u = NULL, *p = NULL;
        registered = 0;
        OK(draid_ec_host_alloc((void **)&u, g_user_len));
        OK(draid_ec_host_alloc((void **)&p, g_par_len));
        memcpy(u, g_user_h, g_user_len);
        memset(p, 0, g_par_len);
        free(g_user_h);
        free(g_par_h);
        g_user_h = u;
        g_par_h = p;
    } else {
        OK(draid_ec_host_register(g_par_h, g_par_len));
    }
    OK(draid_ec_host_device_pointer(g_user_h, (void **)&g_user_d));
    OK(draid_ec_host_device_pointer(g_par_h, (void **)&g_par_d));

    struct io *ios = calloc((size_t)qd, sizeof(*ios));
    draid_ec_ctx *ctx[MAX_GROUPS];
    int inflight[MAX_GROUPS];
    for (int g = 0; g < groups; g++)
        OK(draid_ec_ctx_create(&ctx[g]));
    /* the contexts look the addresses up themselves (a cached range lookup per iovec):
     * they then know that these launches read host memory and size them for the link */
    for (int g = 0; g < groups; g++)
        OK(draid_ec_ctx_set_host_pointers(ctx[g], 1));

    /* warm-up: one pass of every group */
    for (int g = 0; g < groups; g++) {
        submit(ctx[g], ios, g * per, per);
        OK(draid_ec_ctx_synchronize(ctx[g]));
        complete(ios, g * per, per);
    }
    uint64_t done = 0, polls = 0;
    const double t0 = now_s();
    for (int g = 0; g < groups; g++) {
        submit(ctx[g], ios, g * per, per);
        inflight[g] = 1;
    }
    double el = 0;
    int stop = 0;
    for (;;) {
        int busy = 0;
        for (int g = 0; g < groups; g++) {
            if (!inflight[g])
                continue;
            busy = 1;
            const int q = draid_ec_ctx_query(ctx[g]); /* the SPDK poller's check */
            polls++;
            if (q < 0)
                OK(q);
            if (q)
                continue;
            complete(ios, g * per, per);
            done += (uint64_t)per;
            inflight[g] = 0;
            if (!stop) {
                submit(ctx[g], ios, g * per, per);
                inflight[g] = 1;
            }
        }
        el = now_s() - t0;
        if (el >= seconds)
            stop = 1;
        if (stop && !busy)
            break;
    }

    /* every stripe written since the start: P == XOR of the data strips on disk */
    int ok = 1;
    const uint64_t check = g_next_stripe < g_r.total_stripes ? g_next_stripe : g_r.total_stripes;
    for (uint64_t s = 0; s < check && ok; s += 1 + check / 257)
        for (size_t b = 0; b < STRIP_BYTES && ok; b += 61) {
            uint8_t acc = 0;
            for (int d = 0; d < NDISK; d++)
                acc ^= g_disk[d][s * STRIP_BYTES + b];
            ok = acc == 0;
        }
    printf("{\"harness\": \"bdevperf_gpu\", \"config\": \"RAID5 4+1 full-stripe write, 64 KiB strip, "
           "5 RAM disks, parity on the GPU\", \"io_size\": %zu, \"qd\": %d, \"groups\": %d, "
           "\"seconds\": %.3f, \"ios\": %llu, \"mib_s\": %.1f, \"iops\": %.1f, \"polls\": %llu, "
           "\"parity_verified\": %s, \"device_address_equals_host\": %s, \"buffers\": \"%s\"}\n",
           g_io_bytes, qd, groups, el, (unsigned long long)done,
           (double)done * (double)g_io_bytes / el / (1024.0 * 1024.0), (double)done / el,
           (unsigned long long)polls, ok ? "true" : "false",
           g_user_d == g_user_h ? "true" : "false",
           registered ? "registered (hipHostRegister)" : "pinned allocator (hipHostMalloc)");
    for (int g = 0; g < groups; g++)
        draid_ec_ctx_destroy(ctx[g]);
    if (registered) {
        draid_ec_host_unregister(g_user_h);
        draid_ec_host_unregister(g_par_h);
    } else {
        draid_ec_host_free(g_user_h);
        draid_ec_host_free(g_par_h);
    }
    return ok ? 0 : 1;
}
