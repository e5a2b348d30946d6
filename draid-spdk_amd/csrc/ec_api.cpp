// ec_api.cpp -- extern "C" boundary of libdraid_ec.so (declared in
// include/draid_ec.h).  Argument checking follows isa-l v2.30's raid.h /
// gf_vect_mul.h contracts (the functions the reference binds at
// module/bdev/raid/raid5.c:189-201, raid5_simple.c:131-135 and
// examples/bdev/gf_vect_mul/gf_vect_mul.c:40-49,101,108); the arithmetic runs in
// the HIP kernels of ec_kernels.hip.  There is no CPU fallback: when no GPU is
// usable every compute entry point fails with a negative code.
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/draid_ec.h"
#include "ec_gf.hpp"
#include "ec_launch.hpp"
#include "per_device.hpp"

using draid::ArgPtrTable;
using draid::kMaxArgPtrs;

namespace {
thread_local char t_err[256] = "";
}  // namespace

namespace draid {
int fail_hip(hipError_t e, const char* what)
{
    // The runtime keeps a failed call's code as the thread's "last error" until
    // somebody reads it: clear it, or the next HIP user in the process (torch
    // checks after every launch) reports this library's error as its own.
    (void)hipGetLastError();
    snprintf(t_err, sizeof(t_err), "%s: %s (%d)", what, hipGetErrorString(e), static_cast<int>(e));
    return -static_cast<int>(e == hipSuccess ? 1 : e);
}

int fail_arg(const char* what)
{
    snprintf(t_err, sizeof(t_err), "invalid argument: %s", what);
    return 1;
}
}  // namespace draid

using draid::fail_arg;
using draid::fail_hip;

namespace {

hipStream_t sync_stream() { return hipStreamPerThread; }

// Per-thread, per-GPU scratch: a device pointer table for calls with more
// vectors than fit in kernel arguments, a 4-byte flag for the *_check calls, and
// a device staging arena for vectors in pageable host memory.  Table and arena
// are memory of the GPU that was current when they were allocated, so a thread
// that moves to another GPU (draid_ec_set_device) gets that GPU's own set.
// The flag is pinned HOST memory (flag_dev: its address on this GPU): the host
// clears it with a store and reads the verdict with a load, the kernel touches it
// only when it finds a mismatch -- no memset and no copy back per call.
struct Scratch {
    void* table = nullptr;
    size_t table_bytes = 0;
    uint32_t* flag = nullptr;
    uint32_t* flag_dev = nullptr;
    uint8_t* arena = nullptr;
    size_t arena_bytes = 0;
    // Pageable vectors of an ordinary call (a stripe of 64 KiB strips) do not go through the
    // device arena but through this pinned HOST one: the CPU copies them in, the kernel
    // reads and writes them there over PCIe, the CPU copies the results out -- two or three
    // runtime copies of pageable memory per call cost more than the call (bounce_dev: the
    // arena's address on this GPU).
    uint8_t* bounce = nullptr;
    uint8_t* bounce_dev = nullptr;
    size_t bounce_bytes = 0;
    ~Scratch()
    {
        if (table)
            (void)hipFree(table);
        if (flag)
            (void)hipHostFree(flag);
        if (arena)
            (void)hipFree(arena);
        if (bounce)
            (void)hipHostFree(bounce);
    }
};
// Calls that stage more than this go through the device arena (the copies then run at the
// runtime's pageable rate either way, and pinned memory is not for hoarding).
constexpr size_t kBounceMax = 8u << 20;
size_t bounce_max()
{
    static const size_t v = [] {
        const char* e = getenv("DRAID_EC_BOUNCE_MAX");  // bytes; A/B runs
        return e ? static_cast<size_t>(strtoull(e, nullptr, 0)) : kBounceMax;
    }();
    return v;
}
thread_local draid::PerDevice<Scratch> t_scratch_of;

// The calling thread's scratch on its current GPU; null (with the error
// recorded) when there is no usable current device.
Scratch* scratch()
{
    int dev = -1;
    const hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) {
        (void)fail_hip(e, "hipGetDevice");
        return nullptr;
    }
    Scratch* s = t_scratch_of.at(dev);
    if (!s)
        (void)fail_arg("the current GPU's ordinal is beyond what the library keeps state for");
    return s;
}

// The vectors of one synchronous call as a kernel may address them.
//
// isa-l works on whatever host memory it is given (raid5.c:188-201 passes
// spdk_dma_malloc'd chunk buffers and user iovecs).  Here each vector is
// resolved first (ec_xlate.cpp): device memory and pinned / registered host
// memory are used in place, at their device addresses.  A vector in pageable
// memory is never handed to a kernel -- that would be a GPU memory fault, which
// ends the process instead of returning an error -- but staged: copied into a
// per-thread device arena before the launch if the call reads it, and copied
// back afterwards if the call writes it.  Equal host pointers share one staging
// buffer, so in-place forms ({from, to, to}) keep their meaning.
enum : uint8_t { kIn = 1, kOut = 2 };

struct Vectors {
    std::vector<void*> dev;  // what the kernel gets, per vector
    struct Staged {
        void* host;
        size_t offset;
        uint8_t use;
    };
    std::vector<Staged> staged;
    size_t len = 0;
    uint8_t* arena = nullptr;  // the staging arena the offsets refer to (this call's GPU)
    uint8_t* bounce = nullptr; // ... or the pinned host arena, as the CPU sees it

    int resolve(void* const* host, const uint8_t* use, int n, size_t bytes)
    {
        dev.assign(static_cast<size_t>(n), nullptr);
        staged.clear();
        len = bytes;
        size_t need = 0;
        std::vector<int> slot(static_cast<size_t>(n), -1);
        for (int i = 0; i < n; ++i) {
            const void* d = nullptr;
            const int how = draid::translate(host[i], bytes, &d);
            if (how == 0) {
                dev[i] = const_cast<void*>(d);
                continue;
            }
            if (!host[i])
                return fail_arg("a vector pointer is NULL");
            if (how == 2)
                return fail_arg("a vector is device memory of a GPU other than the current one");
            for (size_t s = 0; s < staged.size(); ++s)
                if (staged[s].host == host[i])
                    slot[i] = static_cast<int>(s);
            if (slot[i] < 0) {
                slot[i] = static_cast<int>(staged.size());
                staged.push_back({host[i], need, 0});
                need += (bytes + 255) & ~size_t(255);
            }
            staged[slot[i]].use |= use[i];
        }
        arena = nullptr;
        bounce = nullptr;
        if (staged.empty())
            return 0;
        Scratch* sc = scratch();
        if (!sc)
            return -1;
        if (need <= bounce_max()) {
            if (sc->bounce_bytes < need) {
                if (sc->bounce)
                    (void)hipHostFree(sc->bounce);
                sc->bounce = sc->bounce_dev = nullptr;
                sc->bounce_bytes = 0;
                const size_t cap = std::max<size_t>(need, 1u << 20);
                hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&sc->bounce), cap,
                                             hipHostMallocDefault);
                if (e == hipSuccess)
                    e = hipHostGetDevicePointer(reinterpret_cast<void**>(&sc->bounce_dev),
                                                sc->bounce, 0);
                if (e != hipSuccess) {
                    if (sc->bounce)
                        (void)hipHostFree(sc->bounce);
                    sc->bounce = nullptr;
                    return fail_hip(e, "hipHostMalloc(staging for pageable vectors)");
                }
                sc->bounce_bytes = cap;
            }
            bounce = sc->bounce;
            for (int i = 0; i < n; ++i)
                if (slot[i] >= 0)
                    dev[i] = sc->bounce_dev + staged[slot[i]].offset;
            for (const Staged& s : staged)
                if (s.use & kIn)
                    memcpy(bounce + s.offset, s.host, bytes);
            return 0;
        }
        if (sc->arena_bytes < need) {
            if (sc->arena)
                (void)hipFree(sc->arena);
            sc->arena = nullptr;
            sc->arena_bytes = 0;
            const hipError_t e = hipMalloc(&sc->arena, need);
            if (e != hipSuccess)
                return fail_hip(e, "hipMalloc(staging for pageable vectors)");
            sc->arena_bytes = need;
        }
        arena = sc->arena;
        for (int i = 0; i < n; ++i)
            if (slot[i] >= 0)
                dev[i] = arena + staged[slot[i]].offset;
        for (const Staged& s : staged) {
            if (!(s.use & kIn))
                continue;
            const hipError_t e = hipMemcpyAsync(arena + s.offset, s.host, bytes,
                                                hipMemcpyHostToDevice, sync_stream());
            if (e != hipSuccess)
                return fail_hip(e, "hipMemcpyAsync(stage pageable vector in)");
        }
        return 0;
    }

    // Queues the copies back to pageable destinations (before the final wait).
    hipError_t write_back() const
    {
        if (bounce)
            return hipSuccess;  // copied out by the CPU after the wait (copy_out)
        for (const Staged& s : staged) {
            if (!(s.use & kOut))
                continue;
            const hipError_t e = hipMemcpyAsync(s.host, arena + s.offset, len,
                                                hipMemcpyDeviceToHost, sync_stream());
            if (e != hipSuccess)
                return e;
        }
        return hipSuccess;
    }

    // After the wait: results from the pinned arena to their pageable destinations.
    void copy_out() const
    {
        if (!bounce)
            return;
        for (const Staged& s : staged)
            if (s.use & kOut)
                memcpy(s.host, bounce + s.offset, len);
    }
};
thread_local Vectors t_vec;

// Resolves the n vectors of a stripe call whose last `nout` are written.
int resolve_stripe(void** array, int n, int nout, size_t len)
{
    uint8_t use[kMaxArgPtrs];
    std::vector<uint8_t> big;
    uint8_t* u = use;
    if (n > kMaxArgPtrs) {
        big.resize(static_cast<size_t>(n));
        u = big.data();
    }
    for (int i = 0; i < n; ++i)
        u[i] = i < n - nout ? kIn : kOut;
    return t_vec.resolve(array, u, n, len);
}

// Makes the pointers of one stripe available to a kernel: in kernel arguments
// when they fit, else in the per-thread device table.
int stage_pointers(void* const* array, int n, ArgPtrTable* args, const uint8_t* const** table)
{
    *table = nullptr;
    if (n <= kMaxArgPtrs) {
        memset(args, 0, sizeof(*args));
        for (int i = 0; i < n; ++i)
            args->p[i] = static_cast<const uint8_t*>(array[i]);
        return 0;
    }
    const size_t bytes = sizeof(void*) * static_cast<size_t>(n);
    Scratch* sc = scratch();
    if (!sc)
        return -1;
    if (sc->table_bytes < bytes) {
        if (sc->table)
            (void)hipFree(sc->table);
        sc->table = nullptr;
        sc->table_bytes = 0;
        hipError_t e = hipMalloc(&sc->table, bytes);
        if (e != hipSuccess)
            return fail_hip(e, "hipMalloc(pointer table)");
        sc->table_bytes = bytes;
    }
    hipError_t e = hipMemcpyAsync(sc->table, array, bytes, hipMemcpyHostToDevice, sync_stream());
    if (e != hipSuccess)
        return fail_hip(e, "hipMemcpyAsync(pointer table)");
    *table = static_cast<const uint8_t* const*>(sc->table);
    return 0;
}

int finish_sync(hipError_t e, const char* what)
{
    if (e != hipSuccess)
        return fail_hip(e, what);
    e = t_vec.write_back();
    if (e != hipSuccess)
        return fail_hip(e, "hipMemcpyAsync(write staged vector back)");
    e = hipStreamSynchronize(sync_stream());
    if (e != hipSuccess)
        return fail_hip(e, "hipStreamSynchronize");
    t_vec.copy_out();
    return 0;
}

int encode_one(uint32_t k, uint32_t m, int len, void** array)
{
    int rc = resolve_stripe(array, static_cast<int>(k + m), static_cast<int>(m),
                            static_cast<size_t>(len));
    if (rc)
        return rc;
    ArgPtrTable args;
    const uint8_t* const* table;
    rc = stage_pointers(t_vec.dev.data(), static_cast<int>(k + m), &args, &table);
    if (rc)
        return rc;
    return finish_sync(draid::launch_encode(k, m, static_cast<uint64_t>(len), 1, table,
                                            table ? nullptr : &args, sync_stream()),
                       "launch_encode");
}

int check_one(uint32_t k, uint32_t m, int len, void** array)
{
    Scratch* sc = scratch();
    if (!sc)
        return -1;
    if (!sc->flag) {
        hipError_t e = hipHostMalloc(&sc->flag, 64, hipHostMallocDefault);
        if (e == hipSuccess)
            e = hipHostGetDevicePointer(reinterpret_cast<void**>(&sc->flag_dev), sc->flag, 0);
        if (e != hipSuccess) {
            if (sc->flag)
                (void)hipHostFree(sc->flag);
            sc->flag = nullptr;
            return fail_hip(e, "hipHostMalloc(flag)");
        }
    }
    int rc = resolve_stripe(array, static_cast<int>(k + m), 0, static_cast<size_t>(len));
    if (rc)
        return rc;
    ArgPtrTable args;
    const uint8_t* const* table;
    rc = stage_pointers(t_vec.dev.data(), static_cast<int>(k + m), &args, &table);
    if (rc)
        return rc;
    // (the previous call on this thread has been waited for: nothing else writes the flag)
    __atomic_store_n(sc->flag, 0u, __ATOMIC_RELEASE);
    rc = finish_sync(draid::launch_check(k, m, static_cast<uint64_t>(len), table,
                                         table ? nullptr : &args, sc->flag_dev, sync_stream()),
                     "launch_check");
    if (rc)
        return rc;
    return __atomic_load_n(sc->flag, __ATOMIC_ACQUIRE) ? 1 : 0;
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------- isa-l shaped

int draid_xor_gen(int vects, int len, void** array)
{
    if (vects < 3 || len < 0 || !array)
        return fail_arg("xor_gen needs vects >= 3, len >= 0");
    if (len == 0)
        return 0;
    return encode_one(static_cast<uint32_t>(vects - 1), 1, len, array);
}

int draid_pq_gen(int vects, int len, void** array)
{
    if (vects < 4 || len < 0 || (len & 31) || !array)
        return fail_arg("pq_gen needs vects >= 4, len % 32 == 0");
    if (len == 0)
        return 0;
    return encode_one(static_cast<uint32_t>(vects - 2), 2, len, array);
}

int draid_xor_check(int vects, int len, void** array)
{
    if (vects < 3 || len < 0 || !array)
        return fail_arg("xor_check needs vects >= 3, len >= 0");
    if (len == 0)
        return 0;
    return check_one(static_cast<uint32_t>(vects - 1), 1, len, array);
}

int draid_pq_check(int vects, int len, void** array)
{
    if (vects < 4 || len < 0 || (len & 31) || !array)
        return fail_arg("pq_check needs vects >= 4, len % 32 == 0");
    if (len == 0)
        return 0;
    return check_one(static_cast<uint32_t>(vects - 2), 2, len, array);
}

unsigned char draid_gf_mul(unsigned char a, unsigned char b) { return draid::gf_mul_host(a, b); }

unsigned char draid_gf_inv(unsigned char a) { return draid::gf_inv_host(a); }

void draid_gf_vect_mul_init(unsigned char c, unsigned char* tbl)
{
    for (int i = 0; i < 16; ++i) {
        tbl[i] = draid::gf_mul_host(c, static_cast<uint8_t>(i));
        tbl[16 + i] = draid::gf_mul_host(c, static_cast<uint8_t>(i << 4));
    }
}

int draid_gf_vect_mul(int len, unsigned char* tbl, void* src, void* dest)
{
    if (len < 0 || (len & 31) || !tbl)
        return fail_arg("gf_vect_mul needs len % 32 == 0");
    if (len == 0)
        return 0;
    void* v[2] = {src, dest};
    const uint8_t use[2] = {kIn, kOut};
    if (const int rc = t_vec.resolve(v, use, 2, static_cast<size_t>(len)))
        return rc;
    return finish_sync(draid::launch_gf_vect_mul(static_cast<uint64_t>(len), tbl,
                                                 static_cast<const uint8_t*>(t_vec.dev[0]),
                                                 static_cast<uint8_t*>(t_vec.dev[1]), sync_stream()),
                       "launch_gf_vect_mul");
}

int draid_recover(int k, int m, int len, void** array, int nfail, const int* fail)
{
    // failed strip indices travel as bytes with 0xFF = none, so every index
    // 0 .. k+m-1 must stay below 0xFF
    if (k < 1 || k + m > 255 || m < 1 || m > 2 || len < 0 || nfail < 0 || nfail > m || !array ||
        (nfail && !fail))
        return fail_arg("recover needs k >= 1, k + m <= 255, m in {1,2}, nfail <= m");
    uint8_t f[2] = {DRAID_EC_FAIL_NONE, DRAID_EC_FAIL_NONE};
    for (int i = 0; i < nfail; ++i) {
        if (fail[i] < 0 || fail[i] >= k + m)
            return fail_arg("recover: failed index out of range");
        if (i == 1 && fail[1] == fail[0])
            return fail_arg("recover: duplicate failed index");
        f[i] = static_cast<uint8_t>(fail[i]);
    }
    if (nfail == 0 || len == 0)
        return 0;
    std::vector<uint8_t> use(static_cast<size_t>(k + m), kIn);
    for (int i = 0; i < nfail; ++i)
        use[fail[i]] = kOut;
    int rc = t_vec.resolve(array, use.data(), k + m, static_cast<size_t>(len));
    if (rc)
        return rc;
    ArgPtrTable args;
    const uint8_t* const* table;
    rc = stage_pointers(t_vec.dev.data(), k + m, &args, &table);
    if (rc)
        return rc;
    return finish_sync(draid::launch_reconstruct(static_cast<uint32_t>(k), static_cast<uint32_t>(m),
                                                 static_cast<uint64_t>(len), 1, table,
                                                 table ? nullptr : &args, nullptr, f[0], f[1],
                                                 nullptr, sync_stream()),
                       "launch_reconstruct");
}

// ---------------------------------------------------------------- batched

static int check_batch(const draid_ec_stripe_batch* b)
{
    if (!b)
        return fail_arg("batch is NULL");
    if (b->k < 1 || b->k > 255 || b->m < 1 || b->m > 2 || b->flags != 0)
        return fail_arg("batch needs 1 <= k <= 255, m in {1,2}, flags == 0");
    if (b->nstripes && (!b->strips || b->strip_len == 0))
        return b->strip_len == 0 ? 0 : fail_arg("batch strips table is NULL");
    if (!draid::launch_fits(b->strip_len, b->nstripes))
        return fail_arg("batch too large for one launch (strip_len <= 0x7fff0000, "
                        "ceil(strip_len / 1 KiB) * nstripes < 2^31)");
    return 0;
}

int draid_ec_encode(const draid_ec_stripe_batch* b, void* stream)
{
    int rc = check_batch(b);
    if (rc || !b->nstripes || !b->strip_len)
        return rc;
    hipError_t e = draid::launch_encode(b->k, b->m, b->strip_len, b->nstripes,
                                        reinterpret_cast<const uint8_t* const*>(b->strips), nullptr,
                                        static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail_hip(e, "launch_encode");
}

int draid_ec_reconstruct(const draid_ec_stripe_batch* b, const uint8_t* fail, void* stream)
{
    return draid_ec_reconstruct_status(b, fail, nullptr, stream);
}

int draid_ec_reconstruct_status(const draid_ec_stripe_batch* b, const uint8_t* fail,
                                uint32_t* unrecoverable, void* stream)
{
    int rc = check_batch(b);
    if (rc || !b->nstripes || !b->strip_len)
        return rc;
    if (b->k + b->m > 255)  // failure indices are bytes, 0xFF = none
        return fail_arg("reconstruct needs k + m <= 255");
    if (!fail)
        return fail_arg("reconstruct: fail table is NULL");
    hipError_t e = draid::launch_reconstruct(
        b->k, b->m, b->strip_len, b->nstripes, reinterpret_cast<const uint8_t* const*>(b->strips),
        nullptr, fail, DRAID_EC_FAIL_NONE, DRAID_EC_FAIL_NONE, unrecoverable,
        static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail_hip(e, "launch_reconstruct");
}

static int check_strided(const draid_ec_strided_stripes* d)
{
    if (!d)
        return fail_arg("strided stripes descriptor is NULL");
    if (d->k < 1 || d->k > 255 || d->m < 1 || d->m > 2 || d->flags != 0)
        return fail_arg("strided stripes need 1 <= k <= 255, m in {1,2}, flags == 0");
    if (d->nstripes && d->strip_len && !d->base)
        return fail_arg("strided stripes base is NULL");
    if (!draid::launch_fits(d->strip_len, d->nstripes))
        return fail_arg("stripes too large for one launch (strip_len <= 0x7fff0000, "
                        "ceil(strip_len / 1 KiB) * nstripes < 2^31)");
    return 0;
}

int draid_ec_encode_strided(const draid_ec_strided_stripes* d, void* stream)
{
    int rc = check_strided(d);
    if (rc || !d->nstripes || !d->strip_len)
        return rc;
    hipError_t e = draid::launch_encode_strided(d->k, d->m, d->strip_len, d->nstripes,
                                                static_cast<const uint8_t*>(d->base),
                                                d->strip_stride, d->stripe_stride,
                                                static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail_hip(e, "launch_encode_strided");
}

int draid_ec_reconstruct_strided(const draid_ec_strided_stripes* d, const uint8_t* fail,
                                 void* stream)
{
    return draid_ec_reconstruct_strided_status(d, fail, nullptr, stream);
}

int draid_ec_reconstruct_strided_status(const draid_ec_strided_stripes* d, const uint8_t* fail,
                                        uint32_t* unrecoverable, void* stream)
{
    int rc = check_strided(d);
    if (rc || !d->nstripes || !d->strip_len)
        return rc;
    if (d->k + d->m > 255)  // failure indices are bytes, 0xFF = none
        return fail_arg("reconstruct needs k + m <= 255");
    if (!fail)
        return fail_arg("reconstruct: fail table is NULL");
    hipError_t e = draid::launch_reconstruct_strided(
        d->k, d->m, d->strip_len, d->nstripes, static_cast<const uint8_t*>(d->base),
        d->strip_stride, d->stripe_stride, fail, unrecoverable, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail_hip(e, "launch_reconstruct_strided");
}

// ---------------------------------------------------------------- runtime

int draid_ec_abi_version(void) { return DRAID_EC_ABI_VERSION; }

const char* draid_ec_last_error(void) { return t_err; }

int draid_ec_set_device(int device)
{
    hipError_t e = hipSetDevice(device);
    return e == hipSuccess ? 0 : fail_hip(e, "hipSetDevice");
}

int draid_ec_device_current(int* device)
{
    if (!device)
        return fail_arg("device_current: device is NULL");
    hipError_t e = hipGetDevice(device);
    return e == hipSuccess ? 0 : fail_hip(e, "hipGetDevice");
}

int draid_ec_device_count(int* count)
{
    if (!count)
        return fail_arg("device_count: count is NULL");
    hipError_t e = hipGetDeviceCount(count);
    return e == hipSuccess ? 0 : fail_hip(e, "hipGetDeviceCount");
}

int draid_ec_stream_create(void** stream)
{
    if (!stream)
        return fail_arg("stream_create: stream is NULL");
    hipStream_t s = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e != hipSuccess)
        return fail_hip(e, "hipStreamCreateWithFlags");
    *stream = s;
    return 0;
}

int draid_ec_stream_destroy(void* stream)
{
    hipError_t e = hipStreamDestroy(static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail_hip(e, "hipStreamDestroy");
}

int draid_ec_stream_query(void* stream)
{
    hipError_t e = hipStreamQuery(static_cast<hipStream_t>(stream));
    if (e == hipSuccess)
        return 0;
    if (e == hipErrorNotReady)
        return 1;
    return fail_hip(e, "hipStreamQuery");
}

int draid_ec_stream_synchronize(void* stream)
{
    hipError_t e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail_hip(e, "hipStreamSynchronize");
}

int draid_ec_device_alloc(void** ptr, size_t bytes)
{
    if (!ptr)
        return fail_arg("device_alloc: ptr is NULL");
    hipError_t e = hipMalloc(ptr, bytes);
    return e == hipSuccess ? 0 : fail_hip(e, "hipMalloc");
}

int draid_ec_device_free(void* ptr)
{
    draid::translate_invalidate();  // cached ranges may name this memory
    hipError_t e = hipFree(ptr);
    return e == hipSuccess ? 0 : fail_hip(e, "hipFree");
}

int draid_ec_host_alloc(void** ptr, size_t bytes)
{
    if (!ptr)
        return fail_arg("host_alloc: ptr is NULL");
    *ptr = nullptr;
    hipError_t e = hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocMapped | hipHostMallocPortable);
    return e == hipSuccess ? 0 : fail_hip(e, "hipHostMalloc");
}

int draid_ec_host_free(void* ptr)
{
    draid::translate_invalidate();  // cached ranges may name this memory
    hipError_t e = hipHostFree(ptr);
    return e == hipSuccess ? 0 : fail_hip(e, "hipHostFree");
}

int draid_ec_host_register(void* ptr, size_t bytes)
{
    hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable);
    return e == hipSuccess ? 0 : fail_hip(e, "hipHostRegister");
}

int draid_ec_host_unregister(void* ptr)
{
    draid::translate_invalidate();  // cached ranges may name this memory
    hipError_t e = hipHostUnregister(ptr);
    return e == hipSuccess ? 0 : fail_hip(e, "hipHostUnregister");
}

int draid_ec_host_device_pointer(const void* ptr, void** dev_ptr)
{
    if (!dev_ptr)
        return fail_arg("host_device_pointer: dev_ptr is NULL");
    *dev_ptr = nullptr;
    hipPointerAttribute_t a{};
    if (!ptr || hipPointerGetAttributes(&a, ptr) != hipSuccess) {
        (void)hipGetLastError();
        return fail_arg("host_device_pointer: not a registered or pinned host address");
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer)
        return fail_arg("host_device_pointer: not a registered or pinned host address");
    // devicePointer pairs with hostPointer (the start of the mapping)
    const uint8_t* hp = a.hostPointer ? static_cast<const uint8_t*>(a.hostPointer)
                                      : static_cast<const uint8_t*>(ptr);
    *dev_ptr = static_cast<uint8_t*>(a.devicePointer) + (static_cast<const uint8_t*>(ptr) - hp);
    return 0;
}

int draid_ec_memcpy_async(void* dst, const void* src, size_t bytes, int kind, void* stream)
{
    hipMemcpyKind k;
    switch (kind) {
    case 0: k = hipMemcpyHostToDevice; break;
    case 1: k = hipMemcpyDeviceToHost; break;
    case 2: k = hipMemcpyDeviceToDevice; break;
    default: return fail_arg("memcpy kind must be 0, 1 or 2");
    }
    hipError_t e = hipMemcpyAsync(dst, src, bytes, k, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? 0 : fail_hip(e, "hipMemcpyAsync");
}

// Test/bench hook (not in the public header): pick a kernel variant for A/B
// comparisons inside one process.  0 = default (non-temporal), 1 = plain loads.
void draid_ec_set_variant(int v) { draid::set_variant(v); }

}  // extern "C"
