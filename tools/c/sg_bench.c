/* sg_bench.c -- throughput of the scatter-gather context path (include/draid_ec.h
 * §2b) the way an SPDK module drives it: per stripe, iovec lists into
 * draid_ec_ctx_encode_sg / _reconstruct_sg / _update_sg, one flush per batch.
 * Reports host walk time per stripe, flush time, and GPU time of the batch
 * (HIP events on the context's stream), for RAID6 8+2 x 64 KiB x 4096 stripes
 * in device memory.  Usage: sg_bench [iov_bytes] [stripes] [reps] [shuffle] [autoflush]
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/uio.h>
#include <time.h>

#include "../../include/draid_ec.h"

#define K 8
#define M 2
#define N (K + M)
#define S (64u * 1024u)

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

#define CHECK(x)                                                                  \
    do {                                                                          \
        int rc_ = (x);                                                            \
        if (rc_ != 0) {                                                           \
            fprintf(stderr, "%s:%d %s = %d (%s)\n", __FILE__, __LINE__, #x, rc_, \
                    draid_ec_last_error());                                       \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

int main(int argc, char **argv)
{
    const size_t iov_bytes = argc > 1 ? strtoul(argv[1], 0, 0) : S;
    const uint32_t B = argc > 2 ? strtoul(argv[2], 0, 0) : 4096;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    const int shuffle = argc > 4 ? atoi(argv[4]) : 0; /* enqueue stripes in a random order */
    const uint64_t autoflush = argc > 5 ? strtoull(argv[5], 0, 0) : 0; /* ctx autoflush segments */
    const size_t niov = (S + iov_bytes - 1) / iov_bytes;
    uint8_t *buf = NULL;
    CHECK(draid_ec_device_alloc((void **)&buf, (size_t)B * N * S));
    {
        const size_t chunk = 64u << 20;
        uint8_t *h = malloc(chunk);
        for (size_t i = 0; i < chunk; ++i)
            h[i] = (uint8_t)(i * 2654435761u >> 13);
        for (size_t o = 0; o < (size_t)B * N * S; o += chunk) {
            size_t n = (size_t)B * N * S - o < chunk ? (size_t)B * N * S - o : chunk;
            CHECK(draid_ec_memcpy_async(buf + o, h, n, 0, NULL));
        }
        CHECK(draid_ec_stream_synchronize(NULL));
        free(h);
    }
    /* iovec lists: every strip split into niov pieces, stored in reverse order
     * inside the strip's region so that no two consecutive iovecs are adjacent
     * in memory (a truly scattered list; contiguous pieces would be merged) */
    struct iovec *iov = malloc(sizeof(struct iovec) * (size_t)B * N * niov);
    for (uint32_t s = 0; s < B; ++s)
        for (uint32_t j = 0; j < N; ++j)
            for (size_t v = 0; v < niov; ++v) {
                struct iovec *e = &iov[((size_t)s * N + j) * niov + v];
                const size_t len = (v + 1) * iov_bytes <= S ? iov_bytes : S - v * iov_bytes;
                e->iov_base = buf + ((size_t)s * N + j) * S + (S - v * iov_bytes - len);
                e->iov_len = len;
            }
    draid_ec_ctx *ctx;
    CHECK(draid_ec_ctx_create(&ctx));
    CHECK(draid_ec_ctx_set_autoflush(ctx, autoflush));
    hipStream_t st = (hipStream_t)draid_ec_ctx_stream(ctx);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    uint32_t *order = malloc(sizeof(uint32_t) * B);
    for (uint32_t s = 0; s < B; ++s)
        order[s] = s;
    if (shuffle) {
        uint64_t x = 0x9e3779b97f4a7c15ull;
        for (uint32_t s = B - 1; s > 0; --s) {
            x ^= x << 13, x ^= x >> 7, x ^= x << 17;
            const uint32_t r = (uint32_t)(x % (s + 1)), t = order[s];
            order[s] = order[r];
            order[r] = t;
        }
    }
    int cnt[N];
    for (int j = 0; j < N; ++j)
        cnt[j] = (int)niov;
    const char *names[3] = {"encode_sg", "reconstruct_sg", "update_sg"};
    for (int op = 0; op < 3; ++op) {
        double walk = 0, flush = 0, wall = 0;
        float gpu = 0;
        for (int r = -16; r < reps; ++r) { /* warm-ups fill all 16 descriptor slots */
            CHECK(draid_ec_ctx_synchronize(ctx));
            double t0 = now();
            /* With autoflush the queueing calls launch kernels themselves, so the
             * GPU window must open before the walk (it then spans host time too
             * and says nothing about the kernels' bandwidth: reported as null). */
            if (autoflush)
                hipEventRecord(e0, st);
            for (uint32_t q = 0; q < B; ++q) {
                const uint32_t s = order[q];
                const struct iovec *lists[N];
                for (int j = 0; j < N; ++j)
                    lists[j] = &iov[((size_t)s * N + j) * niov];
                if (op == 0) {
                    CHECK(draid_ec_ctx_encode_sg(ctx, K, M, lists, cnt, NULL, S));
                } else if (op == 1) {
                    int fail[2] = {(int)(s % K), (int)((s + 3) % K)};
                    CHECK(draid_ec_ctx_reconstruct_sg(ctx, K, M, lists, cnt, NULL, S, 2, fail));
                } else {
                    /* RMW of one whole data chunk: old = strip d, new = strip (d+1)%K */
                    const int d = (int)(s % K);
                    const struct iovec *ol[1] = {lists[d]}, *nl[1] = {lists[(d + 1) % K]};
                    const struct iovec *pl[2] = {lists[K], lists[K + 1]};
                    int oc[1] = {cnt[d]}, nc[1] = {cnt[d]}, pc[2] = {cnt[K], cnt[K + 1]};
                    CHECK(draid_ec_ctx_update_sg(ctx, K, M, 1, &d, ol, oc, nl, nc, pl, pc, S));
                }
            }
            double t1 = now();
            if (!autoflush)
                hipEventRecord(e0, st);
            CHECK(draid_ec_ctx_flush(ctx));
            double t2 = now();
            hipEventRecord(e1, st);
            CHECK(draid_ec_ctx_synchronize(ctx));
            double t3 = now();
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (r >= 0) {
                walk += t1 - t0;
                flush += t2 - t1;
                wall += t3 - t0;
                gpu += ms;
            }
        }
        /* algorithmic bytes per stripe: encode (k+m)S, dual reconstruct (k+2)S,
         * RMW of one chunk: old + new + P + Q read, P + Q written = 6S */
        const double per = op == 0 ? (double)N * S : op == 1 ? (double)(K + 2) * S : 6.0 * S;
        const double user = op == 2 ? (double)S : (double)K * S;
        char hbm[32] = "null";
        if (!autoflush)
            snprintf(hbm, sizeof(hbm), "%.1f", per * B / (gpu / reps * 1e-3) / 1e9);
        printf("{\"op\": \"%s\", \"iov_bytes\": %zu, \"stripes\": %u, \"shuffled\": %d, \"autoflush\": %llu, \"walk_us_per_stripe\": %.3f, "
               "\"flush_ms\": %.3f, \"gpu_ms\": %.3f, \"gpu_window\": \"%s\", \"gpu_hbm_gb_s\": %s, "
               "\"wall_ms\": %.3f, \"wall_user_gib_s\": %.1f}\n",
               names[op], iov_bytes, B, shuffle, (unsigned long long)autoflush, walk / reps / B * 1e6, flush / reps * 1e3, gpu / reps,
               autoflush ? "first queueing call to last kernel (includes the host walk)"
                         : "flush to last kernel",
               hbm, wall / reps * 1e3, user * B / (wall / reps) / (1024.0 * 1024 * 1024));
        fflush(stdout);
    }
    draid_ec_ctx_destroy(ctx);
    draid_ec_device_free(buf);
    free(iov);
    free(order);
    return 0;
}
