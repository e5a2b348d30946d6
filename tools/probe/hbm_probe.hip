// hbm_probe.hip -- measurement-only kernels (not part of the product library):
// streaming read / write / copy at 16 B per lane with non-temporal hints, to
// measure the HBM bandwidth this MI355X actually sustains for each mix.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ src, uint64_t n,
                                              u32x4* __restrict__ sink)
{
    u32x4 acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * 4;
    for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) {
        u32x4 a = __builtin_nontemporal_load(src + i);
        u32x4 b = i + 256 < n ? __builtin_nontemporal_load(src + i + 256) : 0;
        u32x4 c = i + 512 < n ? __builtin_nontemporal_load(src + i + 512) : 0;
        u32x4 d = i + 768 < n ? __builtin_nontemporal_load(src + i + 768) : 0;
        acc ^= a ^ b ^ c ^ d;
    }
    if ((acc.x | acc.y | acc.z | acc.w) == 0x12345678u)  // practically never: keeps the loads live
        sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ dst, uint64_t n)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store((u32x4)(uint32_t)i, dst + i);
}

__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ src,
                                              u32x4* __restrict__ dst, uint64_t n)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

extern "C" {
int probe_read(const void* src, uint64_t bytes, void* sink, int grid, void* stream)
{
    hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)src, bytes / 16, (u32x4*)sink);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int probe_write(void* dst, uint64_t bytes, int grid, void* stream)
{
    hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, (hipStream_t)stream, (u32x4*)dst,
                       bytes / 16);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
int probe_copy(const void* src, void* dst, uint64_t bytes, int grid, void* stream)
{
    hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const u32x4*)src, (u32x4*)dst, bytes / 16);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
}

// Stripe-pattern probe: the encode kernel's memory pattern without its math.
// Block b -> stripe s = b / cps, chunk c = b % cps (4 KiB of every strip); each
// lane loads K 16-B vectors at stride S, XORs them, and stores the result to
// the M strips after the data (M = 0: pure read, result stored only if it is an
// impossible value).
template <int KT>
__global__ __launch_bounds__(64) void k_stripe_pattern(uint8_t* base, uint64_t S,
                                                        uint64_t stripe_stride, int K, int M,
                                                        uint32_t cps, u32x4* sink)
{
    const uint32_t s = blockIdx.x / cps, c = blockIdx.x % cps;
    uint8_t* st = base + s * stripe_stride + (uint64_t)c * 1024 + threadIdx.x * 16;
    u32x4 acc = 0;
    if constexpr (KT > 0) {
        u32x4 v[KT];
#pragma unroll
        for (int j = 0; j < KT; ++j)
            v[j] = __builtin_nontemporal_load((const u32x4*)(st + j * S));
#pragma unroll
        for (int j = 0; j < KT; ++j)
            acc ^= v[j];
        K = KT;
    } else {
        for (int j = 0; j < K; ++j)
            acc ^= __builtin_nontemporal_load((const u32x4*)(st + j * S));
    }
    if (M == 0) {
        if ((acc.x & acc.y & acc.z & acc.w) == 0xfffffffeu)
            sink[blockIdx.x & 1023] = acc;
        return;
    }
    for (int j = 0; j < M; ++j)
        __builtin_nontemporal_store(acc, (u32x4*)(st + (K + j) * S));
}

extern "C" int probe_stripe_pattern(void* base, uint64_t len, uint64_t S, uint64_t stripe_stride,
                                    int K, int M, uint32_t nstripes, void* sink, void* stream)
{
    // S = strip stride (len + pad); one wave per 1 KiB chunk of len, as the engine
    const uint32_t cps = (uint32_t)(len / 1024);
    auto kern = K == 8 ? k_stripe_pattern<8> : K == 16 ? k_stripe_pattern<16> : k_stripe_pattern<0>;
    hipLaunchKernelGGL(kern, dim3(cps * nstripes), dim3(64), 0, (hipStream_t)stream,
                       (uint8_t*)base, S, stripe_stride, K, M, cps, (u32x4*)sink);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Write-only, one item per workgroup (the engine's shape): workgroup b writes
// NTHR*VPL*16 contiguous bytes, VPL vectors per lane NTHR apart.
template <int NTHR, int VPL, bool NT>
__global__ __launch_bounds__(NTHR) void k_write_items(u32x4* dst)
{
    u32x4* p = dst + (uint64_t)blockIdx.x * NTHR * VPL + threadIdx.x;
    const u32x4 v = (u32x4)(blockIdx.x ^ threadIdx.x);
#pragma unroll
    for (int u = 0; u < VPL; ++u) {
        if constexpr (NT)
            __builtin_nontemporal_store(v, p + u * NTHR);
        else
            p[u * NTHR] = v;
    }
}

extern "C" int probe_write_items(void* dst, uint64_t bytes, int nthr, int vpl, int nt, void* stream)
{
    const uint64_t per = (uint64_t)nthr * vpl * 16;
    const dim3 g((unsigned)(bytes / per));
    hipStream_t s = (hipStream_t)stream;
#define W(N, V)                                                                      \
    if (nthr == N && vpl == V) {                                                     \
        if (nt)                                                                      \
            hipLaunchKernelGGL((k_write_items<N, V, true>), g, dim3(N), 0, s, (u32x4*)dst);  \
        else                                                                         \
            hipLaunchKernelGGL((k_write_items<N, V, false>), g, dim3(N), 0, s, (u32x4*)dst); \
        return hipGetLastError() == hipSuccess ? 0 : -1;                             \
    }
    W(64, 1) W(64, 4) W(256, 1) W(256, 4) W(1024, 1)
#undef W
    return -2;
}
