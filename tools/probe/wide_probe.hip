// wide_probe.hip -- does a wide stripe (k >= 14) encode faster when the strips of
// one item are divided among several waves of a workgroup?
//
// Every variant computes the same P+Q over the same strided stripes (strip j of
// stripe s at base + s*pitch + j*strip).  SPLIT = 1 is the production shape: one
// 64-lane wave loads 1 KiB of every strip.  SPLIT = 2 / 4: a workgroup of SPLIT
// waves, each loading k/SPLIT strips, partial P and Q (the latter scaled by
// 2^(first strip of the wave)) combined through LDS; wave 0 stores P, the last
// wave stores Q.  U = 2: an item is 2 KiB of every strip (two 16-byte vectors per
// lane and strip), so a workgroup's barrier and LDS exchange serve twice the
// bytes and half as many workgroups are dispatched.  Prints microseconds per launch and algorithmic GB/s, and checks
// every variant's parity against SPLIT = 1.
//
//   wide_probe K STRIP_KIB STRIPES [launches]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                   \
        }                                                                              \
    } while (0)

__device__ __forceinline__ uint32_t mul2(uint32_t q)
{
    const uint32_t top = (q >> 7) & 0x01010101u;
    const uint32_t red = __builtin_amdgcn_perm(0u, 0x00001d00u, top);
    return ((q << 1) & 0xfefefefeu) ^ red;
}
__device__ __forceinline__ u32x4 mul2(u32x4 q)
{
    u32x4 r;
    r.x = mul2(q.x);
    r.y = mul2(q.y);
    r.z = mul2(q.z);
    r.w = mul2(q.w);
    return r;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t* p, uint32_t bytes = 0x7fffffffu)
{
    // a load beyond `bytes` returns zeros without touching memory
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p), 0, static_cast<int>(bytes),
                                             0x00020000);
}

template <int K, int SPLIT, int WAVES, int U>
__global__ __launch_bounds__(64 * SPLIT)
    __attribute__((amdgpu_waves_per_eu(WAVES ? WAVES : 1, WAVES ? WAVES : 8))) void k_enc(
        uint8_t* base, uint32_t strip, uint64_t pitch, uint32_t cps, uint32_t nstripes, int xcd)
{
    constexpr int KW = (K + SPLIT - 1) / SPLIT;  // a ragged last wave reads zeros past strip K-1
    __shared__ u32x4 sp[SPLIT > 1 ? SPLIT : 1][U][64];
    __shared__ u32x4 sq[SPLIT > 1 ? SPLIT : 1][U][64];
    uint32_t b = blockIdx.x;
    if (xcd) {
        const uint32_t total = cps * nstripes, q = total >> 3, r = total & 7u;
        const uint32_t x = b & 7u, i = b >> 3;
        b = x * q + min(x, r) + i;
    }
    const uint32_t s = b / cps, c = b - s * cps;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint8_t* st = base + static_cast<uint64_t>(s) * pitch;
    // cps counts 1 KiB chunks; an item is U of them, 1 KiB apart
    int off[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        off[u] = static_cast<int>(((c * U + u) * 64u + lane) << 4);
    u32x4 p[U], q[U], d[KW][U];
#pragma unroll
    for (int j = KW - 1; j >= 0; --j) {
        const uint32_t jj = w * KW + j;
        const uint8_t* src = st + static_cast<uint64_t>(jj < K ? jj : 0) * strip;
#pragma unroll
        for (int u = 0; u < U; ++u)
            d[j][u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(src, jj < K ? strip : 0u), off[u],
                                                            0, 2);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        p[u] = 0;
        q[u] = 0;
#pragma unroll
        for (int j = KW - 1; j >= 0; --j) {
            p[u] ^= d[j][u];
            q[u] = mul2(q[u]) ^ d[j][u];
        }
    }
    uint8_t* dp = const_cast<uint8_t*>(st) + static_cast<uint64_t>(K) * strip;
    uint8_t* dq = dp + strip;
    if constexpr (SPLIT == 1) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            __builtin_amdgcn_raw_buffer_store_b128(p[u], rsrc(dp), off[u], 0, 18);
            __builtin_amdgcn_raw_buffer_store_b128(q[u], rsrc(dq), off[u], 0, 18);
        }
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            for (uint32_t i = 0; i < w * KW; ++i)
                q[u] = mul2(q[u]);
            sp[w][u][lane] = p[u];
            sq[w][u][lane] = q[u];
        }
        __syncthreads();
        // the U * 2 output vectors of the item are finished by as many waves as
        // there are: wave t takes output t, t + SPLIT, ...
#pragma unroll
        for (int o = 0; o < 2 * U; ++o) {
            if (static_cast<uint32_t>(o % SPLIT) != w)
                continue;
            const int u = o >> 1;
            const bool isq = o & 1;
            u32x4 a = isq ? sq[0][u][lane] : sp[0][u][lane];
#pragma unroll
            for (int t = 1; t < SPLIT; ++t)
                a ^= isq ? sq[t][u][lane] : sp[t][u][lane];
            __builtin_amdgcn_raw_buffer_store_b128(a, rsrc(isq ? dq : dp), off[u], 0, 18);
        }
    }
}

__global__ void k_fill(uint32_t* p, uint64_t n)
{
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
        uint64_t x = i * 0x9e3779b97f4a7c15ull;
        x ^= x >> 29;
        p[i] = static_cast<uint32_t>(x * 0xbf58476d1ce4e5b9ull >> 17);
    }
}

struct Run {
    const char* name;
    void (*fn)(uint8_t*, uint32_t, uint64_t, uint32_t, uint32_t, int);
    int split, u;
};

template <int K>
static void study(uint32_t strip, uint32_t nstripes, int launches)
{
    const uint64_t pitch = static_cast<uint64_t>(K + 2) * strip;
    const uint64_t bytes = pitch * nstripes;
    uint8_t* buf = nullptr;
    CK(hipMalloc(&buf, bytes));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, reinterpret_cast<uint32_t*>(buf), bytes / 4);
    CK(hipDeviceSynchronize());
    const uint32_t cps = strip / 1024;
#define V(S, W, U) { "split" #S " w" #W " u" #U, k_enc<K, S, W, U>, S, U }
#define VS(S) V(S, 0, 1), V(S, 5, 1), V(S, 6, 1), V(S, 7, 1), V(S, 8, 1)
#define VU(S) V(S, 0, 2), V(S, 3, 2), V(S, 4, 2), V(S, 5, 2), V(S, 6, 2), V(S, 8, 2)
    const Run runs[] = { V(1, 0, 1), V(1, 4, 1), V(1, 6, 1), VS(2), VS(4), VS(8), V(1, 0, 2), V(1, 3, 2),
                         VU(2), VU(4), VU(8) };
#undef VU
#undef VS
#undef V
    std::vector<uint8_t> want(2 * static_cast<size_t>(strip)), got(2 * static_cast<size_t>(strip));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double algo = static_cast<double>(bytes);
    for (int xcd = 0; xcd < 1; ++xcd) {
        for (const Run& r : runs) {
            const dim3 grid(cps / r.u * nstripes), block(64 * r.split);
            const uint32_t cps_items = cps / r.u;
            // parity of the last stripe: clear, compute, compare with split1
            CK(hipMemset(buf + pitch * (nstripes - 1) + static_cast<uint64_t>(K) * strip, 0, 2ull * strip));
            for (int i = 0; i < 5; ++i)
                hipLaunchKernelGGL(r.fn, grid, block, 0, 0, buf, strip, pitch, cps_items, nstripes, xcd);
            CK(hipGetLastError());
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < launches; ++i)
                hipLaunchKernelGGL(r.fn, grid, block, 0, 0, buf, strip, pitch, cps_items, nstripes, xcd);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            CK(hipMemcpy(got.data(), buf + pitch * (nstripes - 1) + static_cast<uint64_t>(K) * strip,
                         got.size(), hipMemcpyDeviceToHost));
            bool same = true;
            if (&r == &runs[0] && xcd == 0)
                want = got;
            else
                same = memcmp(want.data(), got.data(), got.size()) == 0;
            const double us = ms * 1000.0 / launches;
            printf("{\"k\": %d, \"strip_kib\": %u, \"stripes\": %u, \"variant\": \"%s\", \"xcd_map\": %d, "
                   "\"us\": %.1f, \"gb_s\": %.1f, \"same\": %s}\n",
                   K, strip / 1024, nstripes, r.name, xcd, us, algo / us / 1e3, same ? "true" : "false");
            fflush(stdout);
            if (!same)
                exit(1);
        }
    }
    CK(hipFree(buf));
}

int main(int argc, char** argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: %s K STRIP_KIB STRIPES [launches]\n", argv[0]);
        return 2;
    }
    const int k = atoi(argv[1]);
    const uint32_t strip = static_cast<uint32_t>(atoi(argv[2])) * 1024u;
    const uint32_t nstripes = static_cast<uint32_t>(atoi(argv[3]));
    const int launches = argc > 4 ? atoi(argv[4]) : 30;
    if (strip == 0 || nstripes == 0 || strip % 1024 != 0) {
        fprintf(stderr, "bad shape\n");
        return 2;
    }
    switch (k) {
    case 4:
        study<4>(strip, nstripes, launches);
        break;
    case 8:
        study<8>(strip, nstripes, launches);
        break;
    case 10:
        study<10>(strip, nstripes, launches);
        break;
    case 12:
        study<12>(strip, nstripes, launches);
        break;
    case 16:
        study<16>(strip, nstripes, launches);
        break;
    default:
        fprintf(stderr, "k must be 4, 8, 10, 12 or 16\n");
        return 2;
    }
    return 0;
}
