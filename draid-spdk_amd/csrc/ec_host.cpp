// ec_host.cpp -- host-resident stripes (SPDK bdev buffers in pinned host memory).
//
// The reference computes parity in place in host buffers: spdk_dma_malloc'd
// stripe buffers and user iovecs (raid5.c:1326-1359, 743-777).  For host
// stripes the GPU path is: copy the k data strips in (hipMemcpy2DAsync, one per
// strip index per chunk of stripes), encode in HBM, copy P (and Q) back out.
// Chunks rotate over kStreams streams, each with its own device staging area,
// so copy-in of one chunk, the kernel of another and copy-out of a third run
// concurrently (separate SDMA engines for H2D and D2H).  Stream order alone
// protects each staging area: its next chunk's copy-in is queued behind its
// previous chunk's copy-out.  The calls are synchronous.
//
// (That is the path DRAID_EC_HOST_STAGED selects, and the one host memory takes that the
// runtime knows but that is not one mapping.  Pageable memory does not use the runtime's
// copies at all: run_bounce below.)
//
// When the stripes are pinned or registered host memory (what SPDK's hugepage
// buffers become after draid_ec_host_register) the staging is skipped: one
// launch over the strided layout reads the strips it needs in place over PCIe
// and writes the results straight back.  Measured on MI355X (8+2 x 64 KiB x
// 4096, profiles/r01/host_path.json): encode 52 GiB/s and reconstruct 52 GiB/s
// of user data -- PCIe-read bound (55.8 GB/s) -- against 50 and 35 GiB/s
// staged, because a reconstruct reads only the k surviving strips.
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/draid_ec.h"
#include "ec_launch.hpp"

namespace {

constexpr int kStreams = 3;

struct Stage {
    hipStream_t stream = nullptr;
    uint8_t* dev = nullptr;       // [chunk][k+m][S]
    size_t dev_bytes = 0;
    void** table = nullptr;       // device pointer table for the staged chunk
    uint8_t* fail = nullptr;      // device [chunk][2]
    size_t table_entries = 0;
    uint32_t k = 0, m = 0, chunk = 0;
    uint64_t S = 0;
};

// One of two pinned buffers the pageable path bounces chunks of stripes through.
struct Bounce {
    hipStream_t stream = nullptr;
    uint8_t* host = nullptr;  // pinned: [rows][k+m][S], then the chunk's failure pairs
    uint8_t* dev = nullptr;   // the same memory as the GPU addresses it
    size_t bytes = 0;
    bool busy = false;        // a kernel over it has been launched and not waited for
    uint32_t c0 = 0, rows = 0;
};

struct HostEngine {
    int device = -1;
    Stage st[kStreams];
    Bounce bn[2];
    uint8_t* zfail = nullptr;  // device copy of the fail table (zero-copy path)
    size_t zfail_bytes = 0;
    ~HostEngine() { reset(); }
    void reset()
    {
        if (zfail)
            (void)hipFree(zfail);
        zfail = nullptr;
        zfail_bytes = 0;
        for (Bounce& b : bn) {
            if (b.stream) {
                (void)hipStreamSynchronize(b.stream);
                (void)hipStreamDestroy(b.stream);
            }
            if (b.host)
                (void)hipHostFree(b.host);
            b = Bounce();
        }
        for (Stage& s : st) {
            if (s.stream)
                (void)hipStreamSynchronize(s.stream);
            if (s.dev)
                (void)hipFree(s.dev);
            if (s.table)
                (void)hipFree(s.table);
            if (s.fail)
                (void)hipFree(s.fail);
            if (s.stream)
                (void)hipStreamDestroy(s.stream);
            s = Stage();
        }
    }
};

thread_local HostEngine t_eng;

int prepare(Stage& s, uint32_t k, uint32_t m, uint64_t S, uint32_t chunk)
{
    hipError_t e;
    if (!s.stream && (e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess)
        return draid::fail_hip(e, "hipStreamCreate(host engine)");
    if (s.k == k && s.m == m && s.S == S && s.chunk == chunk)
        return 0;
    (void)hipStreamSynchronize(s.stream);
    const size_t bytes = static_cast<size_t>(chunk) * (k + m) * S;
    if (s.dev_bytes < bytes) {
        if (s.dev)
            (void)hipFree(s.dev);
        s.dev = nullptr;
        s.dev_bytes = 0;
        if ((e = hipMalloc(&s.dev, bytes)) != hipSuccess)
            return draid::fail_hip(e, "hipMalloc(host staging)");
        s.dev_bytes = bytes;
    }
    const size_t entries = static_cast<size_t>(chunk) * (k + m);
    if (s.table_entries < entries) {
        if (s.table)
            (void)hipFree(s.table);
        if (s.fail)
            (void)hipFree(s.fail);
        s.table = nullptr;
        s.fail = nullptr;
        s.table_entries = 0;
        if ((e = hipMalloc(&s.table, entries * sizeof(void*))) != hipSuccess)
            return draid::fail_hip(e, "hipMalloc(host staging table)");
        if ((e = hipMalloc(&s.fail, static_cast<size_t>(chunk) * 2)) != hipSuccess)
            return draid::fail_hip(e, "hipMalloc(host staging fail)");
        s.table_entries = entries;
    }
    std::vector<void*> t(entries);
    for (size_t i = 0; i < entries; ++i)
        t[i] = s.dev + i * S;  // stripe-major: stripe c strip j at (c*(k+m)+j)*S
    if ((e = hipMemcpy(s.table, t.data(), entries * sizeof(void*), hipMemcpyHostToDevice)) !=
        hipSuccess)
        return draid::fail_hip(e, "hipMemcpy(host staging table)");
    s.k = k;
    s.m = m;
    s.S = S;
    s.chunk = chunk;
    return 0;
}

int check_host(const draid_ec_host_stripes* h)
{
    if (!h || !h->base)
        return draid::fail_arg("host stripes descriptor / base is NULL");
    if (h->k < 1 || h->k > 255 || h->m < 1 || h->m > 2 || (h->flags & ~DRAID_EC_HOST_STAGED))
        return draid::fail_arg("host stripes need 1 <= k <= 255, m in {1,2}, flags in {0, "
                               "DRAID_EC_HOST_STAGED}");
    if (h->strip_stride < h->strip_len)
        return draid::fail_arg("strip_stride < strip_len");
    if (!draid::launch_fits(h->strip_len, h->nstripes))
        return draid::fail_arg("stripes too large for one launch (strip_len <= 0x7fff0000, "
                               "ceil(strip_len / 1 KiB) * nstripes < 2^31)");
    return 0;
}

HostEngine& engine()
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (t_eng.device != dev) {
        t_eng.reset();
        t_eng.device = dev;
    }
    return t_eng;
}

// Device address of a host range mapped into the GPU as one piece (hipHostMalloc
// or hipHostRegister), or nullptr for pageable memory.
uint8_t* mapped_range(const void* p, uint64_t span)
{
    auto dev_addr = [](const void* q) -> uint8_t* {
        hipPointerAttribute_t a{};
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
        if (a.type != hipMemoryTypeHost || !a.devicePointer)
            return nullptr;
        // devicePointer pairs with hostPointer (which may be the allocation base)
        const uint8_t* hp = a.hostPointer ? static_cast<const uint8_t*>(a.hostPointer)
                                          : static_cast<const uint8_t*>(q);
        return static_cast<uint8_t*>(a.devicePointer) + (static_cast<const uint8_t*>(q) - hp);
    };
    uint8_t* d0 = dev_addr(p);
    if (!d0)
        return nullptr;
    uint8_t* d1 = dev_addr(static_cast<const uint8_t*>(p) + (span - 1));
    return d1 == d0 + (span - 1) ? d0 : nullptr;
}

uint64_t host_span(const draid_ec_host_stripes* h)
{
    return static_cast<uint64_t>(h->nstripes - 1) * h->stripe_stride +
           static_cast<uint64_t>(h->k + h->m - 1) * h->strip_stride + h->strip_len;
}

// In-place path over mapped host stripes: one launch, then wait.
template <class Launch>
int run_mapped(Launch&& launch)
{
    HostEngine& eng = engine();
    Stage& s = eng.st[0];
    hipError_t e;
    if (!s.stream && (e = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) != hipSuccess)
        return draid::fail_hip(e, "hipStreamCreate(host engine)");
    {
        // every strip crosses PCIe: the launch runs faster with few items resident
        draid::HostLaunch host(true);
        e = launch(eng, s.stream);
    }
    if (e != hipSuccess)
        return draid::fail_hip(e, "launch (mapped host stripes)");
    if ((e = hipStreamSynchronize(s.stream)) != hipSuccess)
        return draid::fail_hip(e, "hipStreamSynchronize(mapped host stripes)");
    return 0;
}

// Shared driver: per chunk, copy in `in_lo..in_hi` strip indices, run `launch`,
// copy out per `copy_out`.
template <class Launch, class CopyOut>
int run_chunks(const draid_ec_host_stripes* h, uint32_t chunk, uint32_t in_lo, uint32_t in_hi,
               Launch&& launch, CopyOut&& copy_out)
{
    const uint32_t k = h->k, m = h->m, n = k + m;
    const uint64_t S = h->strip_len;
    if (chunk == 0)
        chunk = 64;
    chunk = std::min(chunk, std::max<uint32_t>(1, h->nstripes));
    (void)engine();
    for (Stage& s : t_eng.st) {
        int rc = prepare(s, k, m, S, chunk);
        if (rc)
            return rc;
    }
    uint8_t* base = static_cast<uint8_t*>(h->base);
    hipError_t e = hipSuccess;
    for (uint32_t c0 = 0, ci = 0; c0 < h->nstripes; c0 += chunk, ++ci) {
        Stage& s = t_eng.st[ci % kStreams];
        const uint32_t rows = std::min(chunk, h->nstripes - c0);
        uint8_t* hb = base + static_cast<uint64_t>(c0) * h->stripe_stride;
        for (uint32_t j = in_lo; j < in_hi; ++j) {
            e = hipMemcpy2DAsync(s.dev + j * S, n * S, hb + j * h->strip_stride, h->stripe_stride,
                                 S, rows, hipMemcpyHostToDevice, s.stream);
            if (e != hipSuccess)
                return draid::fail_hip(e, "hipMemcpy2DAsync(H2D strips)");
        }
        if ((e = launch(s, c0, rows)) != hipSuccess)
            return draid::fail_hip(e, "launch (host path)");
        if ((e = copy_out(s, c0, rows, hb)) != hipSuccess)
            return draid::fail_hip(e, "copy-out (host path)");
    }
    for (Stage& s : t_eng.st)
        if ((e = hipStreamSynchronize(s.stream)) != hipSuccess)
            return draid::fail_hip(e, "hipStreamSynchronize(host path)");
    return 0;
}

// Pageable stripes.  The runtime's copies of pageable memory are slow -- strided ones
// (hipMemcpy2DAsync, a row per strip) run at 4 GiB/s of user data on the shapes below,
// where the same calls on pinned memory reach 35-50 -- so this path does not use them:
// the CPU copies a chunk of stripes into a pinned buffer (only the strips the kernel
// reads), the kernel works on the buffer in place over PCIe like the mapped path, and
// the CPU copies the strips it wrote back out.  Two buffers: the GPU works on one chunk
// while the CPU moves the next one in and the previous one out.  fail == nullptr: encode.
int run_bounce(const draid_ec_host_stripes* h, const uint8_t* fail)
{
    const uint32_t k = h->k, m = h->m, n = k + m;
    const uint64_t S = h->strip_len;
    const uint64_t stripe_bytes = n * S;
    // chunks of about 16 MiB: small enough for the copies of one to hide behind the
    // kernel of another
    const uint32_t chunk = static_cast<uint32_t>(
        std::min<uint64_t>(h->nstripes, std::max<uint64_t>(1, (16u << 20) / stripe_bytes)));
    const size_t need = static_cast<size_t>(chunk) * stripe_bytes + 2 * static_cast<size_t>(chunk);
    HostEngine& eng = engine();
    hipError_t e;
    for (Bounce& b : eng.bn) {
        if (!b.stream &&
            (e = hipStreamCreateWithFlags(&b.stream, hipStreamNonBlocking)) != hipSuccess)
            return draid::fail_hip(e, "hipStreamCreate(host engine)");
        if (b.bytes < need) {
            if (b.host)
                (void)hipHostFree(b.host);
            b.host = b.dev = nullptr;
            b.bytes = 0;
            if ((e = hipHostMalloc(reinterpret_cast<void**>(&b.host), need,
                                   hipHostMallocDefault)) != hipSuccess)
                return draid::fail_hip(e, "hipHostMalloc(bounce buffer for pageable stripes)");
            if ((e = hipHostGetDevicePointer(reinterpret_cast<void**>(&b.dev), b.host, 0)) !=
                hipSuccess)
                return draid::fail_hip(e, "hipHostGetDevicePointer(bounce buffer)");
            b.bytes = need;
        }
        b.busy = false;
    }
    uint8_t* base = static_cast<uint8_t*>(h->base);
    // the strips of stripe s the kernel writes: parity (encode) or the lost ones
    auto written = [&](uint32_t s, uint32_t j) {
        if (!fail)
            return j >= k;
        return fail[2 * static_cast<size_t>(s)] == j || fail[2 * static_cast<size_t>(s) + 1] == j;
    };
    auto finish = [&](Bounce& b) -> int {
        if (!b.busy)
            return 0;
        b.busy = false;
        if ((e = hipStreamSynchronize(b.stream)) != hipSuccess)
            return draid::fail_hip(e, "hipStreamSynchronize(pageable stripes)");
        for (uint32_t r = 0; r < b.rows; ++r)
            for (uint32_t j = 0; j < n; ++j)
                if (written(b.c0 + r, j))
                    memcpy(base + static_cast<uint64_t>(b.c0 + r) * h->stripe_stride +
                               j * h->strip_stride,
                           b.host + (static_cast<uint64_t>(r) * n + j) * S, S);
        return 0;
    };
    int rc = 0;
    for (uint32_t c0 = 0, ci = 0; c0 < h->nstripes && rc == 0; c0 += chunk, ++ci) {
        Bounce& b = eng.bn[ci & 1];
        if ((rc = finish(b)) != 0)
            break;
        b.c0 = c0;
        b.rows = std::min(chunk, h->nstripes - c0);
        for (uint32_t r = 0; r < b.rows; ++r) {
            const size_t s = static_cast<size_t>(c0) + r;
            if (fail && fail[2 * s] == DRAID_EC_FAIL_NONE && fail[2 * s + 1] == DRAID_EC_FAIL_NONE)
                continue;  // nothing lost: the kernel skips the stripe, so nothing is read
            // The kernel reads every surviving data strip, P whenever it survives, and Q
            // only for a plan that needs the Q syndrome -- two data strips lost, or one and
            // P (kern_reconstruct.hpp: useQ = needq && !lostQ).  A Q it has no use for
            // stays where it is.
            bool needQ = true;
            if (fail) {
                const uint32_t f0 = fail[2 * s], f1 = fail[2 * s + 1];
                const uint32_t nd = (f0 < k ? 1u : 0u) + (f1 < k && f1 != f0 ? 1u : 0u);
                needQ = nd == 2 || (nd == 1 && (f0 == k || f1 == k));
            }
            for (uint32_t j = 0; j < n; ++j)
                if (!written(c0 + r, j) && (j <= k || needQ))
                    memcpy(b.host + (static_cast<uint64_t>(r) * n + j) * S,
                           base + static_cast<uint64_t>(c0 + r) * h->stripe_stride +
                               j * h->strip_stride,
                           S);
        }
        draid::HostLaunch host(true);
        if (fail) {
            uint8_t* f = b.host + static_cast<size_t>(chunk) * stripe_bytes;
            memcpy(f, fail + 2 * static_cast<size_t>(c0), 2 * static_cast<size_t>(b.rows));
            e = draid::launch_reconstruct_strided(k, m, S, b.rows, b.dev, S, stripe_bytes,
                                                  b.dev + static_cast<size_t>(chunk) * stripe_bytes,
                                                  nullptr, b.stream);
        } else {
            e = draid::launch_encode_strided(k, m, S, b.rows, b.dev, S, stripe_bytes, b.stream);
        }
        if (e != hipSuccess) {
            rc = draid::fail_hip(e, "launch (pageable stripes)");
            break;
        }
        b.busy = true;
    }
    for (Bounce& b : eng.bn) {
        const int r2 = finish(b);  // also after a failure: nothing may still run on the buffers
        if (rc == 0)
            rc = r2;
    }
    return rc;
}

// Pageable memory: the GPU runtime does not know the range at all.
bool is_pageable(const draid_ec_host_stripes* h)
{
    const void* d = nullptr;
    return draid::translate(h->base, 1, &d) == 1;
}

}  // namespace

extern "C" {

int draid_ec_host_encode(const draid_ec_host_stripes* h, uint32_t chunk_stripes)
{
    int rc = check_host(h);
    if (rc || h->nstripes == 0 || h->strip_len == 0)
        return rc;
    const uint32_t k = h->k, m = h->m, n = k + m;
    const uint64_t S = h->strip_len;
    if (!(h->flags & DRAID_EC_HOST_STAGED)) {
        if (uint8_t* d = mapped_range(h->base, host_span(h)))
            return run_mapped([&](HostEngine&, hipStream_t st) {
                return draid::launch_encode_strided(k, m, S, h->nstripes, d, h->strip_stride,
                                                    h->stripe_stride, st);
            });
        if (is_pageable(h))
            return run_bounce(h, nullptr);
    }
    return run_chunks(
        h, chunk_stripes, 0, k,
        [&](Stage& s, uint32_t, uint32_t rows) {
            return draid::launch_encode(k, m, S, rows,
                                        reinterpret_cast<const uint8_t* const*>(s.table), nullptr,
                                        s.stream);
        },
        [&](Stage& s, uint32_t, uint32_t rows, uint8_t* hb) {
            for (uint32_t j = k; j < n; ++j) {
                hipError_t e =
                    hipMemcpy2DAsync(hb + j * h->strip_stride, h->stripe_stride, s.dev + j * S,
                                     n * S, S, rows, hipMemcpyDeviceToHost, s.stream);
                if (e != hipSuccess)
                    return e;
            }
            return hipSuccess;
        });
}

int draid_ec_host_reconstruct(const draid_ec_host_stripes* h, const uint8_t* fail,
                              uint32_t chunk_stripes)
{
    int rc = check_host(h);
    if (rc || h->nstripes == 0 || h->strip_len == 0)
        return rc;
    if (!fail)
        return draid::fail_arg("host reconstruct: fail table is NULL");
    if (h->k + h->m > 255)  // failure indices are bytes, 0xFF = none
        return draid::fail_arg("host reconstruct needs k + m <= 255");
    const uint32_t k = h->k, m = h->m, n = k + m;
    const uint64_t S = h->strip_len;
    // The table is host memory here, so stripes that cannot be rebuilt are found
    // before anything runs (raid5_simple fails the stripe on an arithmetic error,
    // raid5_simple.c:177-180,321-325; a storage engine must not report success
    // for strips it left as they were).
    for (uint32_t s = 0; s < h->nstripes; ++s) {
        const uint8_t* f = fail + 2 * static_cast<size_t>(s);
        const bool oob = (f[0] != DRAID_EC_FAIL_NONE && f[0] >= n) ||
                         (f[1] != DRAID_EC_FAIL_NONE && f[1] >= n);
        const uint32_t nf = (f[0] < n ? 1u : 0u) + ((f[1] < n && f[1] != f[0]) ? 1u : 0u);
        if (oob || nf > m)
            return draid::fail_arg("host reconstruct: a stripe lists more failures than m or an "
                                   "index outside the stripe (nothing was rebuilt)");
    }
    if (!(h->flags & DRAID_EC_HOST_STAGED))
        if (uint8_t* d = mapped_range(h->base, host_span(h)))
            return run_mapped([&](HostEngine& eng, hipStream_t st) {
                const size_t fb = 2 * static_cast<size_t>(h->nstripes);
                hipError_t e;
                if (eng.zfail_bytes < fb) {
                    if (eng.zfail)
                        (void)hipFree(eng.zfail);
                    eng.zfail = nullptr;
                    eng.zfail_bytes = 0;
                    if ((e = hipMalloc(&eng.zfail, fb)) != hipSuccess)
                        return e;
                    eng.zfail_bytes = fb;
                }
                if ((e = hipMemcpyAsync(eng.zfail, fail, fb, hipMemcpyHostToDevice, st)) !=
                    hipSuccess)
                    return e;
                return draid::launch_reconstruct_strided(k, m, S, h->nstripes, d,
                                                         h->strip_stride, h->stripe_stride,
                                                         eng.zfail, nullptr, st);
            });
    if (!(h->flags & DRAID_EC_HOST_STAGED) && is_pageable(h))
        return run_bounce(h, fail);
    return run_chunks(
        h, chunk_stripes, 0, n,
        [&](Stage& s, uint32_t c0, uint32_t rows) {
            hipError_t e = hipMemcpyAsync(s.fail, fail + 2 * static_cast<size_t>(c0), 2 * rows,
                                          hipMemcpyHostToDevice, s.stream);
            if (e != hipSuccess)
                return e;
            return draid::launch_reconstruct(k, m, S, rows,
                                             reinterpret_cast<const uint8_t* const*>(s.table),
                                             nullptr, s.fail, 0xff, 0xff, nullptr, s.stream);
        },
        [&](Stage& s, uint32_t c0, uint32_t rows, uint8_t* hb) {
            for (uint32_t r = 0; r < rows; ++r) {
                // the strips the kernel regenerated (same decoding as decode_failures)
                const uint8_t* f = fail + 2 * static_cast<size_t>(c0 + r);
                const bool v0 = f[0] < n;
                const bool v1 = f[1] < n && !(v0 && f[1] == f[0]);
                if ((v0 ? 1u : 0u) + (v1 ? 1u : 0u) > m)
                    continue;  // unrecoverable: the kernel left it untouched
                for (int t = 0; t < 2; ++t) {
                    const uint32_t j = f[t];
                    if (!(t == 0 ? v0 : v1))
                        continue;
                    hipError_t e = hipMemcpyAsync(hb + r * h->stripe_stride + j * h->strip_stride,
                                                  s.dev + (static_cast<uint64_t>(r) * n + j) * S,
                                                  S, hipMemcpyDeviceToHost, s.stream);
                    if (e != hipSuccess)
                        return e;
                }
            }
            return hipSuccess;
        });
}

}  // extern "C"
