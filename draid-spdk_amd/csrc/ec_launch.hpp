// ec_launch.hpp -- internal launcher interface between the C ABI (ec_api.cpp)
// and the HIP kernels (ec_kernels.hip).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace draid {

// Pointers for the synchronous isa-l-shaped calls travel in the kernel
// arguments (one stripe); above this many vectors they go through a device table.
constexpr int kMaxArgPtrs = 34;

// Launch limits (argument errors, checked before any launch): in-kernel strip
// offsets are 32-bit, and one launch covers at most 2^31 - 1 work items of
// kItemBytes of every strip of a stripe.
constexpr uint64_t kMaxStripLen = 0x7fff0000ull;
constexpr uint64_t kItemBytes = 1024;
inline bool launch_fits(uint64_t strip_len, uint64_t nstripes)
{
    return strip_len <= kMaxStripLen &&
           (strip_len + kItemBytes - 1) / kItemBytes * nstripes <= 0x7fffffffull;
}

struct ArgPtrTable {
    const uint8_t* p[kMaxArgPtrs];
};

// Encode: m = 1 (XOR parity) or 2 (P+Q).
//   table != nullptr : device table [nstripes][k+m]
//   table == nullptr : *args holds the k+m pointers of one stripe (nstripes == 1)
hipError_t launch_encode(uint32_t k, uint32_t m, uint64_t len, uint32_t nstripes,
                         const uint8_t* const* table, const ArgPtrTable* args,
                         hipStream_t stream);

// Strided layout: strip j of stripe s at base + s*stripe_stride + j*strip_stride.
hipError_t launch_encode_strided(uint32_t k, uint32_t m, uint64_t len, uint32_t nstripes,
                                 const uint8_t* base, uint64_t strip_stride,
                                 uint64_t stripe_stride, hipStream_t stream);
hipError_t launch_reconstruct_strided(uint32_t k, uint32_t m, uint64_t len, uint32_t nstripes,
                                      const uint8_t* base, uint64_t strip_stride,
                                      uint64_t stripe_stride, const uint8_t* fail_dev,
                                      uint32_t* bad_dev, hipStream_t stream);

// Reconstruct.  fail_dev: device [nstripes][2] (0xFF = none); when null,
// (f0, f1) apply to every stripe.  bad_dev (may be null): device-accessible
// counter incremented once per stripe that cannot be rebuilt (more failures
// than m, or an index outside the stripe).
hipError_t launch_reconstruct(uint32_t k, uint32_t m, uint64_t len, uint32_t nstripes,
                              const uint8_t* const* table, const ArgPtrTable* args,
                              const uint8_t* fail_dev, uint8_t f0, uint8_t f1, uint32_t* bad_dev,
                              hipStream_t stream);

// Check: sets *flag_dev to non-zero if any stored parity differs.
hipError_t launch_check(uint32_t k, uint32_t m, uint64_t len,
                        const uint8_t* const* table, const ArgPtrTable* args,
                        uint32_t* flag_dev, hipStream_t stream);

// dest = c * src (c given by its isa-l 32-byte nibble table).
hipError_t launch_gf_vect_mul(uint64_t len, const uint8_t tbl[32], const uint8_t* src,
                              uint8_t* dst, hipStream_t stream);

// Segment work lists (scatter-gather, ec_ctx.cpp).  op: 0 encode, 1 reconstruct,
// 2 read-modify-write update.
// A work item is {segment, chunk}; chunk covers work_chunk_bytes(op, k) bytes.
uint32_t work_chunk_bytes(int op, uint32_t k);
// work == nullptr: every segment is `ulen` bytes and item b is chunk
// b % cps of segment b / cps (cps = ceil(ulen / work_chunk_bytes)); seg_len
// is then unused.
// row_bytes == 0: `table` holds one row of 64-bit strip pointers per segment.
// row_bytes != 0: compact rows, row_bytes apart -- an 8-byte base pointer, then
// the int32 offset of every strip from it (then anything).
hipError_t launch_encode_work(uint32_t k, uint32_t m, const uint8_t* const* table,
                              uint32_t row_bytes, const uint32_t* seg_len, const void* work,
                              uint32_t ulen, uint32_t nwork, hipStream_t stream);
// Reconstruct rows of pointers are `tstride` pointers wide (k + m strips, then
// anything); segment s's failure pair is fail[fstride * s], fail[fstride * s + 1].
hipError_t launch_reconstruct_work(uint32_t k, uint32_t m, const uint8_t* const* table,
                                   uint32_t tstride, uint32_t row_bytes, const uint32_t* seg_len,
                                   const uint8_t* fail, uint32_t fstride, const void* work,
                                   uint32_t ulen, uint32_t nwork, hipStream_t stream);

// Read-modify-write parity update over a segment work list (op 2): table rows
// [O_0, N_0, ..., O_{nd-1}, N_{nd-1}, P, (Q)], exps rows sorted descending.
hipError_t launch_update_work(uint32_t m, uint32_t nd, const uint8_t* const* table,
                              const uint8_t* exps, const uint32_t* seg_len, const void* work,
                              uint32_t ulen, uint32_t nwork, hipStream_t stream);

// Error reporting shared by every C entry point (ec_api.cpp): records the
// message for draid_ec_last_error(); fail_hip returns -hipError, fail_arg 1.
int fail_hip(hipError_t e, const char* what);
int fail_arg(const char* what);

// Pointer resolution (ec_xlate.cpp): the address a kernel may use for the
// caller's [p, p + len) -- device memory as is, pinned / registered host memory
// at its device address.  Returns 0; 1 when the range is not GPU accessible
// (pageable host memory: stage it or reject it); 2 when it is device memory of a
// GPU other than `on_device` (reject it).  Neither may ever reach a kernel.  on_device is the ordinal of the GPU
// the kernel will run on; kCurrentDevice = the calling thread's current one.
// Results are cached per thread; translate_invalidate() empties every thread's
// cache.
constexpr int kCurrentDevice = -2;
// *host_memory (may be null): the range is pinned / registered HOST memory.
int translate(const void* p, size_t len, const void** dev, int on_device = kCurrentDevice,
              bool* host_memory = nullptr);
void translate_invalidate();

// While one is alive (and `on`), the launches of the calling thread are launches on
// strips in HOST memory: the segment work lists (launch_*_work) and the strided batches
// (launch_*_strided) run their looping form, one workgroup per CU (ec_kernels.hip).
class HostLaunch {
public:
    explicit HostLaunch(bool on);
    ~HostLaunch();
    HostLaunch(const HostLaunch&) = delete;
    HostLaunch& operator=(const HostLaunch&) = delete;

private:
    bool prev_;
};

// Variant selector for A/B experiments inside one process (0 = default).
void set_variant(int v);
int get_variant();

}  // namespace draid
