// ec_static.hip -- draid_pq_check_static(): the P+Q check for callers that
// cannot allocate (code under HIP graph capture, tight scrub loops, harnesses
// that forbid hipMalloc).
//
// draid_pq_check() (ec_api.cpp) keeps two pieces of device scratch per thread,
// allocated with hipMalloc on first use: a 4-byte mismatch flag the check kernel
// ORs into, and a pointer table for stripes with more vectors than fit in kernel
// arguments.  This variant keeps both in a file-scope __device__ array instead
// -- every GPU the library runs on holds its own 4 KiB copy until the process
// ends -- fills the table with small kernels whose arguments carry the pointers,
// clears the flag with a kernel (not hipMemsetAsync, so the sequence can be
// captured into a graph), and writes the verdict to a caller-provided
// device-accessible word instead of copying it back: no hipMalloc, hipFree,
// hipMemcpy or synchronisation anywhere on the path.
//
// Like every pointer-taking entry point it resolves the vectors and the result
// word before any kernel sees them (ec_xlate.cpp: a cached lookup per pointer,
// no allocation): device memory of the current GPU and pinned / registered host
// memory are used at their device addresses; anything else -- pageable memory,
// which draid_pq_check() would stage through an arena this variant must not
// allocate -- is an error return with nothing launched, never a GPU fault.
//
// The array is shared by every call on a GPU: calls that overlap on one GPU
// (different streams or threads) race on it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "../../include/draid_ec.h"
#include "ec_launch.hpp"

namespace {

constexpr int kStaticMaxVects = DRAID_PQ_CHECK_STATIC_MAX_VECTS;
constexpr size_t kFlagBytes = 256;  // flag word, padded so the table starts on its own line
constexpr size_t kScratchBytes = 4096;
static_assert(kFlagBytes + sizeof(void*) * kStaticMaxVects <= kScratchBytes, "scratch too small");

// In host code this name is only a handle for hipGetSymbolAddress: the device
// address (one per GPU) comes from scratch_of() below and is what kernels,
// and anything else that touches the memory, are given.
static __device__ __align__(256) unsigned char scratch[kScratchBytes];

constexpr int kMaxDevices = 64;
std::mutex g_lock;
unsigned char* g_scratch_ptr[kMaxDevices];  // device address of `scratch` on each GPU

// Device address of the current device's copy of the array, resolved once per
// device with that device current.
int scratch_of(unsigned char** out)
{
    int dev = -1;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess)
        return draid::fail_hip(e, "hipGetDevice");
    if (dev < 0 || dev >= kMaxDevices)
        return draid::fail_arg("pq_check_static: device index above 63");
    std::lock_guard<std::mutex> hold(g_lock);
    if (!g_scratch_ptr[dev]) {
        void* p = nullptr;
        e = hipGetSymbolAddress(&p, HIP_SYMBOL(scratch));
        if (e != hipSuccess || !p)
            return draid::fail_hip(e, "hipGetSymbolAddress(scratch)");
        g_scratch_ptr[dev] = static_cast<unsigned char*>(p);
    }
    *out = g_scratch_ptr[dev];
    return 0;
}

constexpr int kChunkPtrs = 32;
struct PtrChunk {
    const uint8_t* p[kChunkPtrs];
};

// table[off .. off+n) = chunk; the first launch of a call also clears the flag.
__global__ void k_static_stage(const uint8_t** table, uint32_t* flag, PtrChunk chunk, int off,
                               int n, int clear)
{
    const int t = threadIdx.x;
    if (t < n)
        table[off + t] = chunk.p[t];
    if (clear && t == 0)
        *flag = 0;
}

__global__ void k_static_finish(const uint32_t* flag, uint32_t* result)
{
    *result = *flag ? 1u : 0u;
}

}  // namespace

extern "C" int draid_pq_check_static(int vects, int len, void** array, uint32_t* result,
                                     void* stream)
{
    if (vects < 4 || len < 0 || (len & 31) || !array || !result)
        return draid::fail_arg("pq_check_static needs vects >= 4, len % 32 == 0, a result word");
    if (vects > kStaticMaxVects)
        return draid::fail_arg("pq_check_static: more than DRAID_PQ_CHECK_STATIC_MAX_VECTS (257) "
                               "vectors do not fit the static pointer table");
    if (!draid::launch_fits(static_cast<uint64_t>(len), 1))
        return draid::fail_arg("pq_check_static: len above 0x7fff0000");
    // every address first: nothing is launched unless the GPU can reach all of them
    const uint8_t* vec[kStaticMaxVects];
    for (int i = 0; i < vects; ++i) {
        const void* d = nullptr;
        if (len > 0 && draid::translate(array[i], static_cast<size_t>(len), &d))
            return draid::fail_arg("pq_check_static: a vector is neither memory of the current GPU "
                                   "nor pinned / registered host memory (pageable vectors need "
                                   "draid_pq_check, which may allocate a staging arena)");
        vec[i] = static_cast<const uint8_t*>(d);
    }
    const void* res = nullptr;
    if (draid::translate(result, sizeof(uint32_t), &res))
        return draid::fail_arg("pq_check_static: the result word is neither memory of the current "
                               "GPU nor pinned / registered host memory");
    unsigned char* scr = nullptr;
    if (const int rc = scratch_of(&scr))
        return rc;
    uint32_t* flag = reinterpret_cast<uint32_t*>(scr);
    const uint8_t** table = reinterpret_cast<const uint8_t**>(scr + kFlagBytes);
    hipStream_t st = static_cast<hipStream_t>(stream);
    for (int off = 0; off < vects; off += kChunkPtrs) {
        PtrChunk c{};
        const int n = vects - off < kChunkPtrs ? vects - off : kChunkPtrs;
        for (int i = 0; i < n; ++i)
            c.p[i] = vec[off + i];
        hipLaunchKernelGGL(k_static_stage, dim3(1), dim3(64), 0, st, table, flag, c, off, n,
                           off == 0);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess)
            return draid::fail_hip(e, "launch(k_static_stage)");
    }
    hipError_t e = hipSuccess;
    if (len > 0)
        e = draid::launch_check(static_cast<uint32_t>(vects - 2), 2, static_cast<uint64_t>(len),
                                table, nullptr, flag, st);
    if (e != hipSuccess)
        return draid::fail_hip(e, "launch_check");
    hipLaunchKernelGGL(k_static_finish, dim3(1), dim3(1), 0, st, flag,
                       static_cast<uint32_t*>(const_cast<void*>(res)));
    e = hipGetLastError();
    return e == hipSuccess ? 0 : draid::fail_hip(e, "launch(k_static_finish)");
}
