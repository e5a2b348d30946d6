// ec_ctx.cpp -- per-channel context for scatter-gather stripes.
//
// The reference walks the iovec lists of a stripe's chunks and calls isa-l once
// per contiguous run:
//   raid5_xor_iovs     module/bdev/raid/raid5.c:221-283   (dest/src lists from byte offsets)
//   raid5_xor_stripe   module/bdev/raid/raid5_simple.c:141-203 (k data lists + parity)
//   raid5_chunk_map_iov raid5.c:358-426 (slicing a parent bdev_io's iovecs)
// Here the same walk runs on the host but, instead of calling the arithmetic per
// run, it appends each run to a gather-descriptor list (k+m device-accessible
// pointers + a length).  draid_ec_ctx_flush() uploads every queued descriptor
// with one DMA from a pinned ring slot and launches one kernel per (op, k, m)
// group over all of them.  A context is single-threaded, like an SPDK
// io_channel: one per reactor thread.
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/uio.h>

#include <algorithm>
#include <vector>

#include "../../include/draid_ec.h"
#include "ec_launch.hpp"

namespace {

constexpr int kSlots = 4;
constexpr uint64_t kMaxSegment = 1ull << 30;

struct Group {
    int op;  // 0 encode, 1 reconstruct, 2 read-modify-write update
    uint32_t k, m;                  // op 2: k = 2 * touched chunks (old/new list pairs)
    std::vector<const void*> ptrs;  // [nseg][k+m]
    std::vector<uint32_t> len;      // [nseg]
    std::vector<uint8_t> fail;      // [nseg][2] failure pair (op 1) / [nseg][k/2] exponents (op 2)
};

struct Slot {
    void* host = nullptr;  // pinned
    void* dev = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
    bool used = false;
};

int ctx_fail(hipError_t e, const char* what) { return draid::fail_hip(e, what); }
int ctx_arg(const char* what) { return draid::fail_arg(what); }

size_t align8(size_t x) { return (x + 7) & ~size_t(7); }

}  // namespace

struct draid_ec_ctx {
    hipStream_t stream = nullptr;
    int device = 0;
    std::vector<Group> groups;
    Slot slots[kSlots];
    int next = 0;
    uint64_t queued_segments = 0;
};

namespace {

Group& group_for(draid_ec_ctx* c, int op, uint32_t k, uint32_t m)
{
    for (Group& g : c->groups)
        if (g.op == op && g.k == k && g.m == m)
            return g;
    c->groups.push_back(Group{op, k, m, {}, {}, {}});
    return c->groups.back();
}

// Iterator over one strip's iovec list (raid5_simple.c iov_iter).
struct IovIter {
    const struct iovec* v;
    int cnt;
    int idx;
    size_t off;
};

// Positions the iterator `offset` bytes into the list (raid5.c:235-255).
bool iter_seek(IovIter& it, size_t offset)
{
    it.idx = 0;
    it.off = 0;
    while (it.idx < it.cnt && offset >= it.v[it.idx].iov_len) {
        offset -= it.v[it.idx].iov_len;
        ++it.idx;
    }
    if (it.idx >= it.cnt)
        return false;
    it.off = offset;
    return true;
}

// The walk of raid5_xor_stripe: runs of n = min over strips of the bytes left
// in each strip's current iovec; one descriptor per run.
int walk(draid_ec_ctx* c, int op, uint32_t k, uint32_t m, const struct iovec* const* iovs,
         const int* iovcnt, const size_t* offset, size_t len, const uint8_t* meta,
         uint32_t nmeta)
{
    const uint32_t n = k + m;
    if (n > 512)
        return ctx_arg("k + m > 512");
    IovIter it[512];
    for (uint32_t j = 0; j < n; ++j) {
        if (!iovs || !iovs[j] || !iovcnt || iovcnt[j] < 0)
            return ctx_arg("iovec list missing");
        it[j] = IovIter{iovs[j], iovcnt[j], 0, 0};
        if (len && !iter_seek(it[j], offset ? offset[j] : 0))
            return ctx_arg("iovec list shorter than offset");
    }
    Group& g = group_for(c, op, k, m);
    const size_t n_ptrs = g.ptrs.size(), n_len = g.len.size(), n_fail = g.fail.size();
    const uint64_t n_q = c->queued_segments;
    auto rollback = [&](const char* what) {  // a rejected stripe queues nothing
        g.ptrs.resize(n_ptrs);
        g.len.resize(n_len);
        g.fail.resize(n_fail);
        c->queued_segments = n_q;
        return ctx_arg(what);
    };
    size_t remaining = len;
    while (remaining > 0) {
        size_t run = std::min<size_t>(remaining, kMaxSegment);
        for (uint32_t j = 0; j < n; ++j) {
            while (it[j].idx < it[j].cnt && it[j].off == it[j].v[it[j].idx].iov_len) {
                ++it[j].idx;  // skip exhausted / zero-length entries
                it[j].off = 0;
            }
            if (it[j].idx >= it[j].cnt)
                return rollback("iovec list shorter than len");
            run = std::min<size_t>(run, it[j].v[it[j].idx].iov_len - it[j].off);
        }
        for (uint32_t j = 0; j < n; ++j) {
            g.ptrs.push_back(static_cast<const uint8_t*>(it[j].v[it[j].idx].iov_base) + it[j].off);
            it[j].off += run;
        }
        g.len.push_back(static_cast<uint32_t>(run));
        g.fail.insert(g.fail.end(), meta, meta + nmeta);
        ++c->queued_segments;
        remaining -= run;
    }
    return 0;
}

int flush_group(draid_ec_ctx* c, Group& g)
{
    const size_t nseg = g.len.size();
    if (nseg == 0)
        return 0;
    const uint32_t cb = draid::work_chunk_bytes(g.op, g.k);
    // Uniform segments (every run the same length: whole strips, fixed-size
    // iovecs) need no work list -- the kernel derives (segment, chunk) itself.
    const bool uniform = std::all_of(g.len.begin(), g.len.end(),
                                     [&](uint32_t l) { return l == g.len[0]; });
    std::vector<uint32_t> work;  // pairs {seg, chunk}
    uint64_t nwork64;
    if (uniform) {
        nwork64 = static_cast<uint64_t>(nseg) * std::max<uint32_t>(1, (g.len[0] + cb - 1) / cb);
    } else {
        for (size_t s = 0; s < nseg; ++s) {
            const uint32_t cps = std::max<uint32_t>(1, (g.len[s] + cb - 1) / cb);
            for (uint32_t ch = 0; ch < cps; ++ch) {
                work.push_back(static_cast<uint32_t>(s));
                work.push_back(ch);
            }
        }
        nwork64 = work.size() / 2;
    }
    if (nwork64 > 0x7fffffffull)
        return ctx_arg("flush: too many work items queued (flush more often)");
    const uint32_t nwork = static_cast<uint32_t>(nwork64);
    const size_t o_ptr = 0;
    const size_t o_len = align8(o_ptr + g.ptrs.size() * sizeof(void*));
    const size_t o_fail = align8(o_len + (uniform ? 0 : nseg * sizeof(uint32_t)));
    const size_t o_work = align8(o_fail + g.fail.size());
    const size_t bytes = o_work + work.size() * sizeof(uint32_t);

    Slot& sl = c->slots[c->next];
    c->next = (c->next + 1) % kSlots;
    hipError_t e;
    if (sl.used) {  // back-pressure: the slot's previous upload+launch must be done
        e = hipEventSynchronize(sl.done);
        if (e != hipSuccess)
            return ctx_fail(e, "hipEventSynchronize(slot)");
    }
    if (sl.cap < bytes) {
        if (sl.host)
            (void)hipHostFree(sl.host);
        if (sl.dev)
            (void)hipFree(sl.dev);
        sl.host = sl.dev = nullptr;
        sl.cap = 0;
        const size_t cap = std::max<size_t>(bytes * 2, 64 * 1024);
        if ((e = hipHostMalloc(&sl.host, cap, hipHostMallocDefault)) != hipSuccess)
            return ctx_fail(e, "hipHostMalloc(descriptor ring)");
        if ((e = hipMalloc(&sl.dev, cap)) != hipSuccess)
            return ctx_fail(e, "hipMalloc(descriptor ring)");
        sl.cap = cap;
    }
    uint8_t* h = static_cast<uint8_t*>(sl.host);
    memcpy(h + o_ptr, g.ptrs.data(), g.ptrs.size() * sizeof(void*));
    if (!uniform)
        memcpy(h + o_len, g.len.data(), nseg * sizeof(uint32_t));
    if (!g.fail.empty())
        memcpy(h + o_fail, g.fail.data(), g.fail.size());
    if (!work.empty())
        memcpy(h + o_work, work.data(), work.size() * sizeof(uint32_t));
    if ((e = hipMemcpyAsync(sl.dev, sl.host, bytes, hipMemcpyHostToDevice, c->stream)) !=
        hipSuccess)
        return ctx_fail(e, "hipMemcpyAsync(descriptors)");
    const uint8_t* d = static_cast<const uint8_t*>(sl.dev);
    const auto* tab = reinterpret_cast<const uint8_t* const*>(d + o_ptr);
    const auto* lens = reinterpret_cast<const uint32_t*>(d + o_len);
    const void* wl = uniform ? nullptr : d + o_work;
    const uint32_t ulen = g.len[0];
    if (g.op == 0)
        e = draid::launch_encode_work(g.k, g.m, tab, lens, wl, ulen, nwork, c->stream);
    else if (g.op == 1)
        e = draid::launch_reconstruct_work(g.k, g.m, tab, lens, d + o_fail, wl, ulen, nwork,
                                           c->stream);
    else
        e = draid::launch_update_work(g.m, g.k / 2, tab, d + o_fail, lens, wl, ulen, nwork,
                                      c->stream);
    if (e != hipSuccess)
        return ctx_fail(e, "launch (segment work list)");
    if ((e = hipEventRecord(sl.done, c->stream)) != hipSuccess)
        return ctx_fail(e, "hipEventRecord(slot)");
    sl.used = true;
    g.ptrs.clear();
    g.len.clear();
    g.fail.clear();
    return 0;
}

}  // namespace

extern "C" {

int draid_ec_ctx_create(draid_ec_ctx** out)
{
    if (!out)
        return ctx_arg("ctx out pointer is NULL");
    draid_ec_ctx* c = new (std::nothrow) draid_ec_ctx();
    if (!c)
        return ctx_arg("out of host memory");
    hipError_t e = hipGetDevice(&c->device);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    for (int i = 0; e == hipSuccess && i < kSlots; ++i)
        e = hipEventCreateWithFlags(&c->slots[i].done, hipEventDisableTiming);
    if (e != hipSuccess) {
        int rc = ctx_fail(e, "draid_ec_ctx_create");
        draid_ec_ctx_destroy(c);
        return rc;
    }
    *out = c;
    return 0;
}

int draid_ec_ctx_destroy(draid_ec_ctx* c)
{
    if (!c)
        return 0;
    if (c->stream)
        (void)hipStreamSynchronize(c->stream);
    for (Slot& s : c->slots) {
        if (s.host)
            (void)hipHostFree(s.host);
        if (s.dev)
            (void)hipFree(s.dev);
        if (s.done)
            (void)hipEventDestroy(s.done);
    }
    if (c->stream)
        (void)hipStreamDestroy(c->stream);
    delete c;
    return 0;
}

void* draid_ec_ctx_stream(draid_ec_ctx* c) { return c ? c->stream : nullptr; }

int draid_ec_ctx_encode_sg(draid_ec_ctx* c, uint32_t k, uint32_t m,
                           const struct iovec* const* iovs, const int* iovcnt,
                           const size_t* offset, size_t len)
{
    if (!c || k < 1 || k > 255 || m < 1 || m > 2)
        return ctx_arg("encode_sg needs a ctx, 1 <= k <= 255, m in {1,2}");
    return walk(c, 0, k, m, iovs, iovcnt, offset, len, nullptr, 0);
}

int draid_ec_ctx_reconstruct_sg(draid_ec_ctx* c, uint32_t k, uint32_t m,
                                const struct iovec* const* iovs, const int* iovcnt,
                                const size_t* offset, size_t len, int nfail, const int* fail)
{
    if (!c || k < 1 || k > 255 || m < 1 || m > 2 || nfail < 0 || nfail > (int)m ||
        (nfail && !fail))
        return ctx_arg("reconstruct_sg needs a ctx, 1 <= k <= 255, m in {1,2}, nfail <= m");
    uint8_t f[2] = {DRAID_EC_FAIL_NONE, DRAID_EC_FAIL_NONE};
    for (int i = 0; i < nfail; ++i) {
        if (fail[i] < 0 || fail[i] >= (int)(k + m) || (i == 1 && fail[1] == fail[0]))
            return ctx_arg("reconstruct_sg: bad failed index");
        f[i] = static_cast<uint8_t>(fail[i]);
    }
    if (nfail == 0)
        return 0;
    return walk(c, 1, k, m, iovs, iovcnt, offset, len, f, 2);
}

int draid_ec_ctx_update_sg(draid_ec_ctx* c, uint32_t k, uint32_t m, uint32_t nd,
                           const int* data_idx, const struct iovec* const* old_iovs,
                           const int* old_cnt, const struct iovec* const* new_iovs,
                           const int* new_cnt, const struct iovec* const* par_iovs,
                           const int* par_cnt, size_t len)
{
    if (!c || k < 1 || k > 255 || m < 1 || m > 2 || nd < 1 || nd > k || !data_idx || !old_iovs ||
        !old_cnt || !new_iovs || !new_cnt || !par_iovs || !par_cnt)
        return ctx_arg("update_sg needs a ctx, 1 <= nd <= k <= 255, m in {1,2}, all lists");
    // Sort the touched chunks by data index, descending (Horner with gaps).
    uint32_t order[256];
    for (uint32_t i = 0; i < nd; ++i) {
        if (data_idx[i] < 0 || data_idx[i] >= static_cast<int>(k))
            return ctx_arg("update_sg: data index out of range");
        order[i] = i;
    }
    std::sort(order, order + nd, [&](uint32_t a, uint32_t b) { return data_idx[a] > data_idx[b]; });
    const struct iovec* lists[2 * 255 + 2];
    int cnts[2 * 255 + 2];
    uint8_t exps[255];
    for (uint32_t t = 0; t < nd; ++t) {
        const uint32_t i = order[t];
        if (t && data_idx[order[t - 1]] == data_idx[i])
            return ctx_arg("update_sg: duplicate data index");
        lists[2 * t] = old_iovs[i];
        cnts[2 * t] = old_cnt[i];
        lists[2 * t + 1] = new_iovs[i];
        cnts[2 * t + 1] = new_cnt[i];
        exps[t] = static_cast<uint8_t>(data_idx[i]);
    }
    for (uint32_t j = 0; j < m; ++j) {
        lists[2 * nd + j] = par_iovs[j];
        cnts[2 * nd + j] = par_cnt[j];
    }
    return walk(c, 2, 2 * nd, m, lists, cnts, nullptr, len, exps, nd);
}

int draid_ec_ctx_flush(draid_ec_ctx* c)
{
    if (!c)
        return ctx_arg("ctx is NULL");
    for (Group& g : c->groups) {
        int rc = flush_group(c, g);
        if (rc)
            return rc;
    }
    c->queued_segments = 0;
    return 0;
}

int draid_ec_ctx_query(draid_ec_ctx* c)
{
    if (!c)
        return ctx_arg("ctx is NULL");
    hipError_t e = hipStreamQuery(c->stream);
    if (e == hipSuccess)
        return 0;
    if (e == hipErrorNotReady)
        return 1;
    return ctx_fail(e, "hipStreamQuery");
}

int draid_ec_ctx_synchronize(draid_ec_ctx* c)
{
    if (!c)
        return ctx_arg("ctx is NULL");
    hipError_t e = hipStreamSynchronize(c->stream);
    return e == hipSuccess ? 0 : ctx_fail(e, "hipStreamSynchronize");
}

uint64_t draid_ec_ctx_queued(draid_ec_ctx* c) { return c ? c->queued_segments : 0; }

}  // extern "C"
