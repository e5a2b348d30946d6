// transient_probe.hip -- per-launch durations of the first encode / reconstruct
// launches of a process, next to a shader-clock probe.
//
// Question: the first reconstruct launches of a process run up to 25% slower
// than the steady state while the encode does not.  The probe times, per step,
//   [clock probe] [draid_ec_encode] [draid_ec_reconstruct]
// with HIP events on the launch stream, from a cold start, after an idle gap,
// and after a VALU-only burn, so the slow launches can be lined up with the
// shader clock (a fixed dependent VALU chain takes cycles / f_shader seconds).
//
// usage: transient_probe [k m strip_kib stripes steps]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <vector>

#include "../../include/draid_ec.h"

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                \
        }                                                                           \
    } while (0)

// One wave, a dependent chain of `iters` integer multiply-adds: its duration is
// iters * latency / f_shader.  out[0] = chain value, out[1] = s_memtime delta,
// out[2] = constant-rate (100 MHz) timer delta.
__global__ void k_clock_probe(uint64_t* out, uint32_t iters, uint32_t seed)
{
    const uint64_t c0 = clock64(), w0 = wall_clock64();
    uint32_t x = seed + threadIdx.x;
    for (uint32_t i = 0; i < iters; ++i)
        x = x * 1664525u + 1013904223u;
    const uint64_t c1 = clock64(), w1 = wall_clock64();
    if (threadIdx.x == 0) {
        out[0] = x;
        out[1] = c1 - c0;
        out[2] = w1 - w0;
    }
}

// Every CU busy with VALU work only (no memory traffic) for about `iters` chain steps.
__global__ void k_valu_burn(uint32_t* out, uint32_t iters)
{
    uint32_t x = blockIdx.x * 256u + threadIdx.x;
    for (uint32_t i = 0; i < iters; ++i)
        x = x * 1664525u + 1013904223u;
    if (x == 0xdeadbeefu)
        out[0] = x;
}

__global__ void k_fill(uint32_t* p, size_t nwords, uint32_t seed)
{
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t step = (size_t)gridDim.x * blockDim.x;
    for (; i < nwords; i += step) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 15;
        x *= 2246822519u;
        x ^= x >> 13;
        p[i] = x;
    }
}

struct Step {
    float probe_ms, enc_ms, rec_ms;
    uint64_t cyc, wall;
};

int main(int argc, char** argv)
{
    const uint32_t k = argc > 1 ? atoi(argv[1]) : 8, m = argc > 2 ? atoi(argv[2]) : 2;
    const uint64_t S = (argc > 3 ? atoi(argv[3]) : 64) * 1024ull;
    const uint32_t B = argc > 4 ? atoi(argv[4]) : 4096;
    const int steps = argc > 5 ? atoi(argv[5]) : 30;
    const uint32_t n = k + m;

    uint8_t* buf;
    CK(hipMalloc(&buf, (size_t)B * n * S));
    void** table;
    CK(hipMalloc(&table, sizeof(void*) * B * n));
    uint8_t* fail;
    CK(hipMalloc(&fail, 2 * B));
    uint64_t* probe_out;
    CK(hipMalloc(&probe_out, 3 * sizeof(uint64_t) * 4096));
    std::vector<void*> ht((size_t)B * n);
    std::vector<uint8_t> hf(2 * B);
    uint64_t r = 0x1234;
    for (uint32_t s = 0; s < B; ++s) {
        for (uint32_t j = 0; j < n; ++j)
            ht[(size_t)s * n + j] = buf + ((size_t)s * n + j) * S;
        r = r * 6364136223846793005ull + 1442695040888963407ull;
        const uint32_t x = (r >> 33) % k;
        r = r * 6364136223846793005ull + 1442695040888963407ull;
        const uint32_t y = (x + 1 + (r >> 33) % (k - 1)) % k;
        hf[2 * s] = (uint8_t)x;
        hf[2 * s + 1] = (uint8_t)y;
    }
    CK(hipMemcpy(table, ht.data(), sizeof(void*) * B * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(fail, hf.data(), 2 * B, hipMemcpyHostToDevice));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    k_fill<<<4096, 256, 0, st>>>((uint32_t*)buf, (size_t)B * n * S / 4, 7u);
    CK(hipStreamSynchronize(st));

    draid_ec_stripe_batch batch{k, m, S, B, 0, table};
    const int kMax = 256;
    std::vector<hipEvent_t> ev(4 * kMax);
    for (auto& e : ev)
        CK(hipEventCreate(&e));

    auto phase = [&](const char* name, int nsteps, bool do_enc, bool do_rec) {
        std::vector<Step> out(nsteps);
        for (int i = 0; i < nsteps; ++i) {
            CK(hipEventRecord(ev[4 * i], st));
            k_clock_probe<<<1, 64, 0, st>>>(probe_out + 3 * i, 4000, i);
            CK(hipEventRecord(ev[4 * i + 1], st));
            if (do_enc && draid_ec_encode(&batch, st)) {
                fprintf(stderr, "encode: %s\n", draid_ec_last_error());
                exit(2);
            }
            CK(hipEventRecord(ev[4 * i + 2], st));
            if (do_rec && draid_ec_reconstruct(&batch, fail, st)) {
                fprintf(stderr, "reconstruct: %s\n", draid_ec_last_error());
                exit(2);
            }
            CK(hipEventRecord(ev[4 * i + 3], st));
        }
        CK(hipStreamSynchronize(st));
        std::vector<uint64_t> po(3 * nsteps);
        CK(hipMemcpy(po.data(), probe_out, sizeof(uint64_t) * 3 * nsteps, hipMemcpyDeviceToHost));
        printf("{\"phase\": \"%s\", \"k\": %u, \"m\": %u, \"strip\": %llu, \"stripes\": %u, \"steps\": [",
               name, k, m, (unsigned long long)S, B);
        for (int i = 0; i < nsteps; ++i) {
            Step s;
            CK(hipEventElapsedTime(&s.probe_ms, ev[4 * i], ev[4 * i + 1]));
            CK(hipEventElapsedTime(&s.enc_ms, ev[4 * i + 1], ev[4 * i + 2]));
            CK(hipEventElapsedTime(&s.rec_ms, ev[4 * i + 2], ev[4 * i + 3]));
            printf("%s[%.4f, %.4f, %.4f, %llu, %llu]", i ? ", " : "", s.probe_ms, s.enc_ms, s.rec_ms,
                   (unsigned long long)po[3 * i + 1], (unsigned long long)po[3 * i + 2]);
        }
        printf("], \"columns\": [\"probe_ms\", \"encode_ms\", \"reconstruct_ms\", \"probe_s_memtime\", "
               "\"probe_wall_100mhz\"]}\n");
        fflush(stdout);
    };

    phase("cold_start", steps, true, true);
    sleep(2);
    phase("after_2s_idle", steps, true, true);
    phase("back_to_back_reconstruct_only", steps, false, true);
    sleep(2);
    phase("after_2s_idle_reconstruct_only", steps, false, true);
    sleep(2);
    phase("after_2s_idle_encode_only", steps, true, false);
    sleep(2);
    // ~10 ms of VALU-only load on every CU, then the steps at once
    uint32_t* sink = (uint32_t*)probe_out;
    k_valu_burn<<<256 * 4, 256, 0, st>>>(sink + 3 * 2 * 4000, 300000);
    phase("after_idle_then_valu_burn", steps, true, true);
    sleep(2);
    // memory-only load (the fill kernel a few times), then the steps
    for (int i = 0; i < 8; ++i)
        k_fill<<<4096, 256, 0, st>>>((uint32_t*)buf, (size_t)B * k * S / 4 / 4, 7u);
    phase("after_idle_then_fill", steps, true, true);
    return 0;
}
