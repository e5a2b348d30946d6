// event_gap_probe.hip -- what do event records between kernels of one stream cost the GPU?
// N kernels of a fixed length back to back on one stream, with 0, 1 or 2 hipEventRecord calls
// behind each; GPU time of the whole train from a first to a last timing event.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                \
        }                                                                           \
    } while (0)

__global__ void k_spin(uint32_t* out, uint32_t iters)
{
    uint32_t x = blockIdx.x * 256u + threadIdx.x;
    for (uint32_t i = 0; i < iters; ++i)
        x = x * 1664525u + 1013904223u;
    if (x == 0xdeadbeefu)
        out[0] = x;
}

int main(int argc, char** argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 200;
    const uint32_t iters = argc > 2 ? atoi(argv[2]) : 20000;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint32_t* d;
    CK(hipMalloc(&d, 4096));
    hipEvent_t t0, t1, ev[2][64];
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    for (int j = 0; j < 2; ++j)
        for (int i = 0; i < 64; ++i)
            CK(hipEventCreateWithFlags(&ev[j][i], hipEventDisableTiming));
    for (int events = 0; events <= 2; ++events) {
        float best = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(t0, st));
            for (int i = 0; i < n; ++i) {
                hipLaunchKernelGGL(k_spin, dim3(1024), dim3(256), 0, st, d, iters);
                for (int j = 0; j < events; ++j)
                    CK(hipEventRecord(ev[j][i % 64], st));
            }
            CK(hipEventRecord(t1, st));
            CK(hipStreamSynchronize(st));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, t0, t1));
            if (ms < best)
                best = ms;
        }
        printf("{\"kernels\": %d, \"events_behind_each\": %d, \"us_per_kernel\": %.2f}\n", n, events,
               best * 1e3f / n);
    }
    return 0;
}
