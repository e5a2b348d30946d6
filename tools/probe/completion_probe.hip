// completion_probe.hip -- how soon does the host see that a small kernel has finished?
//
// A poller (an SPDK reactor) cannot block, so it polls.  Three ways to learn that a
// launch is done, each timed from just before the launch call to the moment the host
// knows, median over many launches of a kernel that does almost nothing:
//   sync    hipStreamSynchronize (blocking; the reference point)
//   event   hipEventRecord behind the kernel, then spinning on hipEventQuery
//   flag    a one-lane kernel behind it stores a sequence number into pinned host
//           memory with a system-scope release; the host spins on that word
// usage: completion_probe [launches]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                \
        }                                                                           \
    } while (0)

__global__ void k_work(uint32_t* p)
{
    if (threadIdx.x == 0 && blockIdx.x == 0)
        p[0] += 1;
}

__global__ void k_flag(volatile uint64_t* flag, uint64_t seq)
{
    __atomic_store_n(const_cast<uint64_t*>(flag), seq, __ATOMIC_RELEASE);  // system scope
}

static double now_us()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static double median(std::vector<double>& v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 2000;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint32_t* d;
    CK(hipMalloc(&d, 4096));
    CK(hipMemset(d, 0, 4096));
    uint64_t* flag_h;
    CK(hipHostMalloc(&flag_h, 64, hipHostMallocDefault));
    uint64_t* flag_d;
    CK(hipHostGetDevicePointer((void**)&flag_d, flag_h, 0));
    *flag_h = 0;
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    std::vector<double> t_sync, t_event, t_flag, t_flag_launch;
    uint64_t seq = 0;
    for (int i = -50; i < n; ++i) {
        double t0 = now_us();
        hipLaunchKernelGGL(k_work, dim3(64), dim3(64), 0, st, d);
        CK(hipStreamSynchronize(st));
        double t1 = now_us();
        if (i >= 0)
            t_sync.push_back(t1 - t0);

        t0 = now_us();
        hipLaunchKernelGGL(k_work, dim3(64), dim3(64), 0, st, d);
        CK(hipEventRecord(ev, st));
        while (hipEventQuery(ev) == hipErrorNotReady)
            ;
        t1 = now_us();
        if (i >= 0)
            t_event.push_back(t1 - t0);

        ++seq;
        t0 = now_us();
        hipLaunchKernelGGL(k_work, dim3(64), dim3(64), 0, st, d);
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(1), 0, st, flag_d, seq);
        const double tl = now_us();
        while (__atomic_load_n(flag_h, __ATOMIC_ACQUIRE) < seq)
            ;
        t1 = now_us();
        if (i >= 0) {
            t_flag.push_back(t1 - t0);
            t_flag_launch.push_back(tl - t0);
        }
        CK(hipStreamSynchronize(st));
    }
    printf("{\"launches\": %d, \"sync_us\": %.1f, \"event_query_us\": %.1f, \"flag_us\": %.1f, "
           "\"flag_launch_calls_us\": %.1f}\n",
           n, median(t_sync), median(t_event), median(t_flag), median(t_flag_launch));
    return 0;
}
