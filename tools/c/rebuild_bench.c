/*
 * rebuild_bench.c -- rebuilding failed disks of a RAID6 array held in HBM.
 *
 * The reference has no rebuild or resync; its degraded read
 * (raid5_complete_reconstructed_stripe_request, raid5.c:544-594) rebuilds one
 * request's range.  On the GPU a whole failed disk is one batched reconstruct:
 * draid_raid_strip_table gives every stripe's rotated pointers,
 * draid_raid_fail_table the failed disk's role (data index, P or Q) in each
 * stripe, and draid_ec_reconstruct rebuilds every stripe in one launch.
 *
 *   rebuild_bench [k=8] [strip_kib=64] [disk_gib=4] [reps=5]
 * Prints one JSON line per failure count (1 and 2 disks): failed-disk bytes
 * rebuilt per second and the algorithmic HBM traffic rate.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "draid_ec.h"
#include "draid_raid.h"

#define OK(x)                                                                               \
    do {                                                                                    \
        int _rc = (x);                                                                      \
        if (_rc) {                                                                          \
            fprintf(stderr, "%s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #x, _rc,          \
                    draid_ec_last_error());                                                 \
            exit(2);                                                                        \
        }                                                                                   \
    } while (0)

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char **argv)
{
    const int k = argc > 1 ? atoi(argv[1]) : 8;
    const uint32_t strip_kib = argc > 2 ? (uint32_t)atoi(argv[2]) : 64;
    const double disk_gib = argc > 3 ? atof(argv[3]) : 4.0;
    const int reps = argc > 4 ? atoi(argv[4]) : 5;
    const int n = k + 2;
    const size_t sb = (size_t)strip_kib * 1024;
    const uint64_t nstripes = (uint64_t)(disk_gib * (1ull << 30)) / sb;
    const size_t db = sb * nstripes;
    struct draid_raid r;
    OK(draid_raid_start(&r, 6, n, 4096, (uint32_t)(sb / 4096), (uint64_t)(db / 4096)));

    void *st;
    OK(draid_ec_stream_create(&st));
    uint8_t *disk[DRAID_RAID_MAX_BASE];
    const size_t fill = (size_t)64 << 20;
    uint8_t *h = malloc(fill);
    uint64_t x = 0x9e3779b97f4a7c15ull;
    for (size_t i = 0; i < fill; i += 8) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        memcpy(h + i, &x, 8);
    }
    for (int d = 0; d < n; d++) {
        OK(draid_ec_device_alloc((void **)&disk[d], db));
        for (size_t o = 0; o < db; o += fill)
            OK(draid_ec_memcpy_async(disk[d] + o, h, db - o < fill ? db - o : fill, 0, st));
    }
    void **tab = malloc(sizeof(void *) * n * nstripes), **dtab;
    uint8_t *fail = malloc(2 * nstripes), *dfail;
    OK(draid_ec_device_alloc((void **)&dtab, sizeof(void *) * n * nstripes));
    OK(draid_ec_device_alloc((void **)&dfail, 2 * nstripes));
    OK(draid_raid_strip_table(&r, 0, (uint32_t)nstripes, (void *const *)disk, 0, tab));
    OK(draid_ec_memcpy_async(dtab, tab, sizeof(void *) * n * nstripes, 0, st));
    draid_ec_stripe_batch b = {(uint32_t)k, 2, sb, (uint32_t)nstripes, 0, dtab};
    OK(draid_ec_encode(&b, st)); /* consistent parity everywhere */
    OK(draid_ec_stream_synchronize(st));

    const size_t sample = 16u << 20;
    uint8_t *before = malloc(sample), *after = malloc(sample);
    for (int nf = 1; nf <= 2; nf++) {
        const int f0 = 3 % n, f1 = (3 + n / 2) % n;
        r.degraded_mask = (1u << f0) | (nf == 2 ? 1u << f1 : 0);
        OK(draid_raid_fail_table(&r, 0, (uint32_t)nstripes, fail));
        OK(draid_ec_memcpy_async(dfail, fail, 2 * nstripes, 0, st));
        OK(draid_ec_memcpy_async(before, disk[f0] + db / 2, sample, 1, st));
        OK(draid_ec_stream_synchronize(st));
        double best = 1e30;
        for (int rep = 0; rep < reps + 1; rep++) { /* first pass warms up */
            OK(draid_ec_memcpy_async(disk[f0] + db / 2, h, sample, 0, st)); /* erase a sample */
            OK(draid_ec_stream_synchronize(st));
            const double t0 = now_s();
            OK(draid_ec_reconstruct(&b, dfail, st));
            OK(draid_ec_stream_synchronize(st));
            const double el = now_s() - t0;
            if (rep && el < best)
                best = el;
        }
        OK(draid_ec_memcpy_async(after, disk[f0] + db / 2, sample, 1, st));
        OK(draid_ec_stream_synchronize(st));
        const int ok = memcmp(before, after, sample) == 0;
        const double rebuilt = (double)nf * (double)db;
        const double traffic = (double)(k + nf) * (double)db; /* k survivors read, nf written */
        printf("{\"tool\": \"rebuild_bench\", \"raid\": \"RAID6 %d+2\", \"strip_bytes\": %zu, "
               "\"disk_bytes\": %zu, \"stripes\": %llu, \"failed_disks\": %d, \"seconds\": %.6f, "
               "\"rebuilt_gb_s\": %.1f, \"hbm_traffic_gb_s\": %.1f, \"sample_verified\": %s}\n",
               k, sb, db, (unsigned long long)nstripes, nf, best, rebuilt / best / 1e9,
               traffic / best / 1e9, ok ? "true" : "false");
        if (!ok)
            return 1;
    }
    for (int d = 0; d < n; d++)
        draid_ec_device_free(disk[d]);
    draid_ec_device_free(dtab);
    draid_ec_device_free(dfail);
    draid_ec_stream_destroy(st);
    return 0;
}
