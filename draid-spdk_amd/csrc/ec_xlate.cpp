// ec_xlate.cpp -- which addresses may a kernel touch, and under which name?
//
// The reference hands isa-l plain host pointers: spdk_dma_malloc'd chunk
// buffers and the iovecs of user I/O (raid5_xor_buf, module/bdev/raid/raid5.c:
// 188-201; raid5_xor_stripe, raid5_simple.c:141-203).  A GPU can only follow a
// host pointer that the HIP runtime has mapped (hipHostMalloc, hipHostRegister),
// possibly at a different device address, and a kernel launched on anything
// else takes a memory fault that ends the whole process.  So every entry point
// that receives pointers from the caller's side of the boundary resolves them
// here first:
//   device memory                  -> itself
//   pinned / registered host memory -> its device address
//   anything else                   -> "not accessible" (the caller stages or
//                                      rejects it; it is never handed to a kernel)
//
// Device memory belongs to one GPU: a range resolved there is good for kernels
// on that GPU only (no peer access is set up by this library), so every range
// remembers its device and a lookup says which GPU the kernel will run on.
//
// hipPointerGetAttributes costs microseconds, so each thread keeps the ranges it
// has resolved (the whole allocation or registration around the pointer) and a
// hit costs a few compares.  Ranges go stale when memory is freed or
// unregistered: the library's own free / unregister calls and
// draid_ec_pointer_cache_flush() start a new epoch that empties every thread's
// cache.
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <atomic>

#include "../../include/draid_ec.h"
#include "ec_launch.hpp"
#include "per_device.hpp"

namespace {

struct Range {
    uintptr_t lo = 0, hi = 0;  // host-side name of the range: [lo, hi)
    intptr_t delta = 0;        // device address = host address + delta
    int device = draid::kAnyDevice;  // the GPU whose memory it is; host memory: any
    bool host = false;               // pinned / registered host memory: every access crosses PCIe
};

constexpr int kWays = 32;

struct Cache {
    uint64_t epoch = 0;
    int n = 0;
    Range r[kWays];  // most recently used first
};

std::atomic<uint64_t> g_epoch{1};
thread_local Cache t_cache;

// Resolves p through the runtime.  0 = range filled in, 1 = not GPU accessible.
int query(const void* p, size_t len, Range* out)
{
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // unknown pointers are reported as an error by some runtimes
        return 1;
    }
    const uintptr_t q = reinterpret_cast<uintptr_t>(p);
    uintptr_t dev = 0;
    if (a.type == hipMemoryTypeDevice) {
        dev = q;
        out->device = a.device;
    } else if (a.type == hipMemoryTypeManaged || a.type == hipMemoryTypeUnified) {
        dev = q;  // migrates to whichever GPU touches it
    } else if (a.type == hipMemoryTypeHost && a.devicePointer) {
        // devicePointer names the same byte as hostPointer, which is p itself or
        // the start of its mapping depending on the runtime version
        const uintptr_t hp = a.hostPointer ? reinterpret_cast<uintptr_t>(a.hostPointer) : q;
        dev = reinterpret_cast<uintptr_t>(a.devicePointer) + (q - hp);
        out->host = true;
    } else {
        return 1;  // pageable host memory, arrays, mappings without a device address
    }
    out->delta = static_cast<intptr_t>(dev - q);
    // the allocation / registration around it, so neighbours hit the cache
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(dev)) == hipSuccess &&
        base && size) {
        const uintptr_t b = reinterpret_cast<uintptr_t>(base);
        if (b <= dev && dev + (len ? len : 1) <= b + size) {
            out->lo = b - static_cast<uintptr_t>(out->delta);
            out->hi = out->lo + size;
            return 0;
        }
    } else {
        (void)hipGetLastError();
    }
    // range unknown: vouch for the queried bytes only if their last byte resolves
    // to the same mapping
    out->lo = q;
    out->hi = q + (len ? len : 1);
    if (len > 1) {
        hipPointerAttribute_t b{};
        const void* last = static_cast<const uint8_t*>(p) + (len - 1);
        if (hipPointerGetAttributes(&b, last) != hipSuccess) {
            (void)hipGetLastError();
            return 1;
        }
        uintptr_t dl = 0;
        const uintptr_t ql = reinterpret_cast<uintptr_t>(last);
        if (b.type == hipMemoryTypeHost && b.devicePointer) {
            const uintptr_t hp = b.hostPointer ? reinterpret_cast<uintptr_t>(b.hostPointer) : ql;
            dl = reinterpret_cast<uintptr_t>(b.devicePointer) + (ql - hp);
        } else if (b.type == hipMemoryTypeDevice || b.type == hipMemoryTypeManaged ||
                   b.type == hipMemoryTypeUnified) {
            dl = ql;
        } else {
            return 1;
        }
        if (dl != dev + (len - 1))
            return 1;
    }
    return 0;
}

}  // namespace

namespace draid {

// The GPU a kernel launched now would run on.
static int current_device()
{
    int d = kAnyDevice;
    if (hipGetDevice(&d) != hipSuccess) {
        (void)hipGetLastError();
        return kAnyDevice;
    }
    return d;
}

static bool usable(const Range& r, int on_device)
{
    if (r.device == kAnyDevice || on_device == kAnyDevice)
        return true;
    return range_usable_on(r.device, on_device == kCurrentDevice ? current_device() : on_device);
}

int translate(const void* p, size_t len, const void** dev, int on_device, bool* host_memory)
{
    *dev = nullptr;
    if (host_memory)
        *host_memory = false;
    if (!p)
        return 1;
    Cache& c = t_cache;
    const uint64_t now = g_epoch.load(std::memory_order_acquire);
    if (c.epoch != now) {
        c.epoch = now;
        c.n = 0;
    }
    const uintptr_t q = reinterpret_cast<uintptr_t>(p);
    const uintptr_t end = q + (len ? len : 1);
    for (int i = 0; i < c.n; ++i) {
        if (q >= c.r[i].lo && end <= c.r[i].hi) {
            const Range hit = c.r[i];
            for (int j = i; j > 0; --j)  // move to front
                c.r[j] = c.r[j - 1];
            c.r[0] = hit;
            if (!usable(hit, on_device))
                return 2;  // another GPU's memory
            *dev = reinterpret_cast<const void*>(q + static_cast<uintptr_t>(hit.delta));
            if (host_memory)
                *host_memory = hit.host;
            return 0;
        }
    }
    Range r;
    if (query(p, len, &r))
        return 1;
    if (c.n < kWays)
        ++c.n;
    for (int j = c.n - 1; j > 0; --j)
        c.r[j] = c.r[j - 1];
    c.r[0] = r;
    if (!usable(r, on_device))
        return 2;
    *dev = reinterpret_cast<const void*>(q + static_cast<uintptr_t>(r.delta));
    if (host_memory)
        *host_memory = r.host;
    return 0;
}

void translate_invalidate() { g_epoch.fetch_add(1, std::memory_order_acq_rel); }

}  // namespace draid

extern "C" {

int draid_ec_device_pointer(const void* ptr, size_t len, void** dev_ptr)
{
    if (!dev_ptr)
        return draid::fail_arg("device_pointer: dev_ptr is NULL");
    const void* d = nullptr;
    if (draid::translate(ptr, len, &d)) {
        *dev_ptr = nullptr;
        return draid::fail_arg("device_pointer: the range is not memory of the current GPU and "
                               "not pinned or registered host memory");
    }
    *dev_ptr = const_cast<void*>(d);
    return 0;
}

void draid_ec_pointer_cache_flush(void) { draid::translate_invalidate(); }

}  // extern "C"
