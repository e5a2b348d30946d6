// ec_mgpu.cpp -- one process, several GPUs.
//
// Stripes are independent (only requests to the SAME stripe serialise,
// module/bdev/raid/raid5.c:1047-1054), so a node's GPUs share the work by stripe
// index with no data exchanged between them: stripe s lives on, and is encoded
// or rebuilt by, device s mod G -- or the devices take contiguous ranges.  The
// benchmark harness does this with one process per GPU; an SPDK target is ONE
// process, so the same split must be drivable from one thread.  A
// draid_ec_mgpu holds a stream per device; each call walks the devices,
// makes each current in turn and enqueues that device's shard on its stream
// (launches are asynchronous, a few microseconds each), so all GPUs run
// concurrently.  No collective, no peer access, no xGMI traffic.
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <new>
#include <vector>

#include "../../include/draid_ec.h"
#include "ec_launch.hpp"

struct draid_ec_mgpu {
    std::vector<int> device;
    std::vector<hipStream_t> stream;
};

namespace {

struct Current {
    int prev = -1;
    Current() { (void)hipGetDevice(&prev); }
    ~Current()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

int mg_arg(const char* what) { return draid::fail_arg(what); }

// Runs f(slot) with slot's device current, for every slot; stops at the first error.
template <class F>
int each_device(draid_ec_mgpu* mg, F&& f)
{
    Current keep;
    for (size_t d = 0; d < mg->device.size(); ++d) {
        hipError_t e = hipSetDevice(mg->device[d]);
        if (e != hipSuccess)
            return draid::fail_hip(e, "hipSetDevice");
        if (const int rc = f(static_cast<int>(d)))
            return rc;
    }
    return 0;
}

}  // namespace

extern "C" {

int draid_ec_shard_of(uint64_t stripe, uint64_t nstripes, int ndevices, int policy)
{
    if (ndevices < 1 || stripe >= nstripes)
        return -1;
    if (policy == DRAID_EC_SHARD_MOD)
        return static_cast<int>(stripe % static_cast<uint64_t>(ndevices));
    // contiguous ranges [nstripes*d/G, nstripes*(d+1)/G): the device whose range holds it
    const uint64_t g = static_cast<uint64_t>(ndevices);
    uint64_t d = static_cast<uint64_t>((static_cast<unsigned __int128>(stripe) * g) / nstripes);
    while (d + 1 < g && static_cast<uint64_t>((static_cast<unsigned __int128>(nstripes) * (d + 1)) / g) <= stripe)
        ++d;
    while (d > 0 && static_cast<uint64_t>((static_cast<unsigned __int128>(nstripes) * d) / g) > stripe)
        --d;
    return static_cast<int>(d);
}

int draid_ec_shard_range(uint64_t nstripes, int ndevices, int device, uint64_t* lo, uint64_t* hi)
{
    if (ndevices < 1 || device < 0 || device >= ndevices || !lo || !hi)
        return mg_arg("shard_range needs 0 <= device < ndevices and result pointers");
    const unsigned __int128 n = nstripes;
    *lo = static_cast<uint64_t>(n * static_cast<uint64_t>(device) / static_cast<uint64_t>(ndevices));
    *hi = static_cast<uint64_t>(n * (static_cast<uint64_t>(device) + 1) / static_cast<uint64_t>(ndevices));
    return 0;
}

uint64_t draid_ec_shard_count(uint64_t nstripes, int ndevices, int device, int policy)
{
    if (ndevices < 1 || device < 0 || device >= ndevices)
        return 0;
    if (policy == DRAID_EC_SHARD_MOD) {
        const uint64_t g = static_cast<uint64_t>(ndevices), d = static_cast<uint64_t>(device);
        return nstripes / g + (d < nstripes % g ? 1 : 0);
    }
    uint64_t lo, hi;
    (void)draid_ec_shard_range(nstripes, ndevices, device, &lo, &hi);
    return hi - lo;
}

int draid_ec_mgpu_create(draid_ec_mgpu** out, int ndevices, const int* devices)
{
    if (!out)
        return mg_arg("mgpu out pointer is NULL");
    *out = nullptr;
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess)
        return draid::fail_hip(e, "hipGetDeviceCount");
    if (ndevices <= 0)
        ndevices = count;  // every visible GPU
    if (ndevices < 1 || ndevices > 64)
        return mg_arg("mgpu needs 1..64 device slots");
    draid_ec_mgpu* mg = new (std::nothrow) draid_ec_mgpu();
    if (!mg)
        return mg_arg("out of host memory");
    Current keep;
    for (int d = 0; d < ndevices; ++d) {
        const int dev = devices ? devices[d] : d;
        if (dev < 0 || dev >= count) {
            draid_ec_mgpu_destroy(mg);
            return mg_arg("mgpu: device index out of range");
        }
        hipStream_t s = nullptr;
        if ((e = hipSetDevice(dev)) != hipSuccess ||
            (e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess) {
            draid_ec_mgpu_destroy(mg);
            return draid::fail_hip(e, "mgpu stream creation");
        }
        mg->device.push_back(dev);
        mg->stream.push_back(s);
    }
    *out = mg;
    return 0;
}

int draid_ec_mgpu_destroy(draid_ec_mgpu* mg)
{
    if (!mg)
        return 0;
    Current keep;
    for (size_t d = 0; d < mg->stream.size(); ++d) {
        (void)hipSetDevice(mg->device[d]);
        (void)hipStreamSynchronize(mg->stream[d]);
        (void)hipStreamDestroy(mg->stream[d]);
    }
    delete mg;
    return 0;
}

int draid_ec_mgpu_devices(const draid_ec_mgpu* mg) { return mg ? static_cast<int>(mg->device.size()) : 0; }

int draid_ec_mgpu_device(const draid_ec_mgpu* mg, int slot)
{
    return mg && slot >= 0 && slot < static_cast<int>(mg->device.size()) ? mg->device[slot] : -1;
}

void* draid_ec_mgpu_stream(draid_ec_mgpu* mg, int slot)
{
    return mg && slot >= 0 && slot < static_cast<int>(mg->stream.size()) ? mg->stream[slot] : nullptr;
}

int draid_ec_mgpu_encode(draid_ec_mgpu* mg, const draid_ec_stripe_batch* batches)
{
    if (!mg || !batches)
        return mg_arg("mgpu_encode needs an mgpu and one batch per device slot");
    return each_device(mg, [&](int d) {
        return batches[d].nstripes ? draid_ec_encode(&batches[d], mg->stream[d]) : 0;
    });
}

int draid_ec_mgpu_reconstruct(draid_ec_mgpu* mg, const draid_ec_stripe_batch* batches,
                              const uint8_t* const* fail, uint32_t* const* unrecoverable)
{
    if (!mg || !batches || !fail)
        return mg_arg("mgpu_reconstruct needs an mgpu, one batch and one fail table per slot");
    return each_device(mg, [&](int d) {
        if (!batches[d].nstripes)
            return 0;
        return draid_ec_reconstruct_status(&batches[d], fail[d],
                                           unrecoverable ? unrecoverable[d] : nullptr,
                                           mg->stream[d]);
    });
}

int draid_ec_mgpu_encode_strided(draid_ec_mgpu* mg, const draid_ec_strided_stripes* shards)
{
    if (!mg || !shards)
        return mg_arg("mgpu_encode_strided needs an mgpu and one descriptor per device slot");
    return each_device(mg, [&](int d) {
        return shards[d].nstripes ? draid_ec_encode_strided(&shards[d], mg->stream[d]) : 0;
    });
}

int draid_ec_mgpu_reconstruct_strided(draid_ec_mgpu* mg, const draid_ec_strided_stripes* shards,
                                      const uint8_t* const* fail, uint32_t* const* unrecoverable)
{
    if (!mg || !shards || !fail)
        return mg_arg("mgpu_reconstruct_strided needs an mgpu, descriptors and fail tables");
    return each_device(mg, [&](int d) {
        if (!shards[d].nstripes)
            return 0;
        return draid_ec_reconstruct_strided_status(&shards[d], fail[d],
                                                   unrecoverable ? unrecoverable[d] : nullptr,
                                                   mg->stream[d]);
    });
}

int draid_ec_mgpu_query(draid_ec_mgpu* mg)
{
    if (!mg)
        return mg_arg("mgpu is NULL");
    int running = 0;
    for (hipStream_t s : mg->stream) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipErrorNotReady) {
            (void)hipGetLastError();
            running = 1;
        } else if (e != hipSuccess) {
            return draid::fail_hip(e, "hipStreamQuery");
        }
    }
    return running;
}

int draid_ec_mgpu_synchronize(draid_ec_mgpu* mg)
{
    if (!mg)
        return mg_arg("mgpu is NULL");
    return each_device(mg, [&](int d) {
        const hipError_t e = hipStreamSynchronize(mg->stream[d]);
        return e == hipSuccess ? 0 : draid::fail_hip(e, "hipStreamSynchronize");
    });
}

}  // extern "C"
