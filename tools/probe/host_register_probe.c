/* Which kinds of host memory does hipHostRegister accept on this box?
 * One line per kind: shared / private anonymous mmap, posix_memalign, sizes. */
#define _GNU_SOURCE
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/resource.h>

static void try_reg(const char *name, void *p, size_t n, int touch, unsigned flags)
{
    if (touch)
        memset(p, 1, n);
    hipError_t e = hipHostRegister(p, n, flags);
    printf("%-32s n=%-9zu touch=%d flags=%u addr=%p -> %d %s\n", name, n, touch, flags, p, (int)e,
           hipGetErrorString(e));
    fflush(stdout);
    if (e == hipSuccess)
        (void)hipHostUnregister(p);
    else
        (void)hipGetLastError();
}

int main(void)
{
    struct rlimit rl;
    getrlimit(RLIMIT_MEMLOCK, &rl);
    printf("RLIMIT_MEMLOCK cur=%llu max=%llu\n", (unsigned long long)rl.rlim_cur,
           (unsigned long long)rl.rlim_max);
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    printf("devices=%d (%s)\n", n, hipGetErrorString(e));
    void *d;
    e = hipMalloc(&d, 4096);
    printf("hipMalloc -> %s\n", hipGetErrorString(e));
    const size_t sizes[] = {69632, 4u << 20};
    const unsigned flagsv[] = {hipHostRegisterMapped, hipHostRegisterDefault, hipHostRegisterPortable};
    for (int t = 0; t < 2; ++t)
        for (int s = 0; s < 2; ++s)
            for (int f = 0; f < 3; ++f) {
                size_t N = sizes[s];
                void *a = mmap(NULL, N, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
                try_reg("mmap shared anonymous", a, N, t, flagsv[f]);
                a = mmap(NULL, N, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
                try_reg("mmap private anonymous", a, N, t, flagsv[f]);
                void *p = NULL;
                if (posix_memalign(&p, 4096, N) == 0)
                    try_reg("posix_memalign", p, N, t, flagsv[f]);
            }
    return 0;
}
