/*
 * bdevperf_raid5.c -- CPU counterpart of BASELINE config 1 (test/baseline
 * infrastructure, not product code).
 *
 * Config 1 is "RAID5 4+1 full-stripe write, 64KiB strip, bdevperf over malloc
 * bdevs on CPU (isa-l reference path, no GPU)": bdevperf -w write -o 262144 -q 32
 * -t 10 over a raid5 bdev of 5 malloc bdevs.  bdevperf needs
 * SPDK + DPDK + isa-l, none of which can be built here, so this harness performs
 * the same per-request data movement on one core:
 *   - stripe index advances sequentially (bdevperf -w write is sequential);
 *   - qd task buffers of one I/O each, used round-robin (bdevperf allocates one
 *     buffer per outstanding task, -q 32);
 *   - parity disk p = (n-1) - s mod n, data index d on disk d<p ? d : d+1
 *     (raid5.c:1006-1007, 172-179);
 *   - each data strip is copied into its RAM disk (malloc bdev memcpy,
 *     bdev_malloc.c:173-200), parity = xor_gen(k+1, S, ...) over the k user
 *     strips (raid5_simple.c:176) written into the parity disk;
 *   - MiB/s = user bytes written / elapsed (bdevperf.c:244-249).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "isal_oracle.h"

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* Returns MiB/s of user data; *ios_out = completed 256 KiB writes.  disk_bytes
 * is the size of each RAM disk; io_size = k * strip (full-stripe writes); qd task
 * buffers. */
double orc_bdevperf_raid5_fsw(int n, size_t strip, size_t disk_bytes, int qd, double seconds,
                              uint64_t *ios_out, uint8_t *verify_ok)
{
    const int k = n - 1;
    const size_t io = (size_t)k * strip;
    const uint64_t stripes = disk_bytes / strip;
    uint8_t **disk = calloc((size_t)n, sizeof(*disk));
    if (qd < 1)
        qd = 1;
    uint8_t *tasks = aligned_alloc(4096, io * (size_t)qd);
    void **vec = calloc((size_t)n, sizeof(*vec));
    if (!disk || !tasks || !vec || stripes == 0)
        return -1.0;
    for (int d = 0; d < n; d++) {
        disk[d] = aligned_alloc(4096, disk_bytes);
        if (!disk[d])
            return -1.0;
        memset(disk[d], 0, disk_bytes);
    }
    orc_fill_splitmix(tasks, io * (size_t)qd, 0x1234);

    /* isa-l picks its AVX-512 xor_gen on this class of CPU: so does the harness */
    int (*xor_gen)(int, int, void **) = orc_simd_available() ? orc_simd_xor_gen : orc_xor_gen;
    uint64_t ios = 0, s = 0;
    double t0 = now_s(), el;
    do {
        for (int batch = 0; batch < 32; batch++) { /* -q 32 worth per clock check */
            const uint64_t si = s % stripes;
            uint8_t *user = tasks + (size_t)(s % (uint64_t)qd) * io;
            const int p = (n - 1) - (int)(s % (uint64_t)n);
            for (int d = 0; d < k; d++) {
                uint8_t *dst = disk[d < p ? d : d + 1] + si * strip;
                memcpy(dst, user + (size_t)d * strip, strip);
                vec[d] = dst;
            }
            vec[k] = disk[p] + si * strip;
            xor_gen(n, (int)strip, vec);
            user[(s * 64) % io] ^= 1; /* new payload each request */
            s++;
            ios++;
        }
        el = now_s() - t0;
    } while (el < seconds);

    /* spot-check the last stripe: parity == XOR of its data strips */
    if (verify_ok) {
        const uint64_t last = (s - 1) % stripes;
        const int p = (n - 1) - (int)((s - 1) % (uint64_t)n);
        uint8_t ok = 1;
        for (size_t b = 0; b < strip && ok; b += 97) {
            uint8_t x = 0;
            for (int d = 0; d < n; d++)
                x ^= disk[d][last * strip + b];
            ok = (x == 0);
        }
        (void)p;
        *verify_ok = ok;
    }
    for (int d = 0; d < n; d++)
        free(disk[d]);
    free(disk);
    free(tasks);
    free(vec);
    if (ios_out)
        *ios_out = ios;
    return (double)ios * (double)io / el / (1024.0 * 1024.0);
}
