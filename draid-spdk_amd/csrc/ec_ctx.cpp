// ec_ctx.cpp -- per-channel context for scatter-gather stripes.
//
// The reference walks the iovec lists of a stripe's chunks and calls isa-l once
// per contiguous run:
//   raid5_xor_iovs     module/bdev/raid/raid5.c:221-283   (dest/src lists from byte offsets)
//   raid5_xor_stripe   module/bdev/raid/raid5_simple.c:141-203 (k data lists + parity)
//   raid5_chunk_map_iov raid5.c:358-426 (slicing a parent bdev_io's iovecs)
// Here the same walk runs on the host but, instead of calling the arithmetic per
// run, it appends each run to a gather-descriptor list (k+m device-accessible
// pointers, written straight into pinned memory, + a length).
// draid_ec_ctx_flush() DMAs the queued descriptors of each (op, k, m) group in
// pieces of about 1 MiB on a copy stream and launches one kernel per piece on
// the compute stream, so uploads overlap kernels; pieces of small segments are
// uploaded already while the batch is still being queued (stage_ahead).  A context is
// single-threaded, like an SPDK io_channel: one per reactor thread.
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/uio.h>

#include <algorithm>
#include <deque>
#include <vector>

#include "../../include/draid_ec.h"
#include "ec_launch.hpp"

namespace {

constexpr int kSlots = 16;
// Pieces a context may hold uploaded but not yet launched (below): the other
// slots stay free for the pieces a flush packs itself.
constexpr int kMaxStaged = 12;
// A small launch reads its descriptors where the host wrote them, in pinned memory,
// instead of waiting for their upload (stage_piece).  Small: work items (1 KiB chunks
// of a stripe) + 16 x segments within this limit -- about 400 stripes of 64 KiB
// strips, 100 of them cut into 4 KiB runs, 120 of 256 KiB strips.
constexpr size_t kInplaceLimit = 32768;
constexpr size_t kPieceBytes = 1u << 20;       // descriptors per launch (≈ 1 MiB)
constexpr size_t kMinPieceSegments = 4096;
constexpr uint64_t kMaxSegment = 1ull << 30;
constexpr uint64_t kWideFlushes = 64;  // see draid_ec_ctx::wide_until

// Growable array in pinned host memory.  The walk writes a group's strip
// pointers here and the flush DMAs them to the device straight from it, so the
// pointers -- (k+m) * 8 bytes of every run, nearly all of a piece's
// descriptor bytes -- are written once, not walked into pageable memory and
// then packed into a ring slot.  Growth never initialises the new elements.
class PinnedPtrs {
public:
    PinnedPtrs() = default;
    PinnedPtrs(const PinnedPtrs&) = delete;
    PinnedPtrs& operator=(const PinnedPtrs&) = delete;
    ~PinnedPtrs() { if (p_) (void)hipHostFree(p_); }
    void swap(PinnedPtrs& o) { std::swap(p_, o.p_); std::swap(n_, o.n_); std::swap(cap_, o.cap_); }
    size_t size() const { return n_; }
    const void** data() { return p_; }
    const void* operator[](size_t i) const { return p_[i]; }
    void clear() { n_ = 0; }
    void shrink(size_t n) { n_ = std::min(n_, n); }
    bool full(size_t add) const { return n_ + add > cap_; }  // grow(add) would move the array
    // Appends `add` uninitialised elements; null when pinned memory runs out.
    const void** grow(size_t add)
    {
        if (n_ + add > cap_) {
            size_t cap = std::max<size_t>(cap_ ? cap_ * 2 : (1u << 20) / sizeof(void*), n_ + add);
            void* q = nullptr;
            if (hipHostMalloc(&q, cap * sizeof(void*), hipHostMallocDefault) != hipSuccess)
                return nullptr;
            if (n_)
                memcpy(q, p_, n_ * sizeof(void*));
            if (p_)
                (void)hipHostFree(p_);  // never in flight: see Group::ready() and walk()
            p_ = static_cast<const void**>(q);
            cap_ = cap;
        }
        const void** out = p_ + n_;
        n_ += add;
        return out;
    }

private:
    const void** p_ = nullptr;
    size_t n_ = 0, cap_ = 0;
};

// Slots (8 bytes each) of one segment's row.  A row of pointers: k + m of them,
// plus one for a reconstruct's failure pair.  A compact row: the base pointer, then
// the int32 offset of every strip from it, then (reconstruct) the failure pair in
// an int32 slot of its own -- 48 instead of 80 bytes for an 8+2 encode segment.
constexpr uint32_t row_slots(int op, uint32_t n, bool compact)
{
    return compact ? (8u + 4u * n + (op == 1 ? 4u : 0u) + 7u) / 8u : n + (op == 1 ? 1u : 0u);
}

// A piece of a group whose descriptors are in a ring slot and on their way to
// the device (or there already); only its launch is left.
struct Staged {
    int slot = -1;
    size_t s0 = 0, s1 = 0;          // the group's segments [s0, s1)
    bool uniform = false;           // every segment the same length: no work list
    bool inplace = false;           // the kernel reads the descriptors from the slot's pinned
                                    // host memory: nothing was uploaded
    bool host_data = false;         // most of the segments have strips in host memory: PCIe
                                    // bound, better with few items resident (HostLaunch)
    uint32_t nwork = 0, ulen = 0;   // work items; the uniform length
    size_t o_len = 0, o_fail = 0, o_work = 0;  // offsets into the slot
};

struct Group {
    Group(int op_, uint32_t k_, uint32_t m_, uint32_t level_, bool compact_)
        : op(op_), level(level_), k(k_), m(m_), compact(compact_),
          w(row_slots(op_, k_ + m_, compact_))
    {
    }
    Group(const Group&) = delete;
    Group& operator=(const Group&) = delete;
    ~Group()
    {
        for (hipEvent_t e : uploaded)
            if (e)
                (void)hipEventDestroy(e);
    }
    int op;  // 0 encode, 1 reconstruct, 2 read-modify-write update
    uint32_t level;  // fences in front of its segments within their requests (draid_ec_ctx_fence)
    uint64_t first_seq = 0;         // queue position of the batch's first segment in this group
    uint32_t k, m;                  // op 2: k = 2 * touched chunks (old/new list pairs)
    bool compact;                   // rows of base + int32 offsets instead of pointers
    uint32_t w;                     // 8-byte slots per segment (row_slots)
    PinnedPtrs ptrs;                // [nseg][w]; op 1: the slot behind the strips holds the
                                    // failure pair in its first two bytes (uploaded with the row)
    std::vector<uint32_t> len;      // [nseg]
    std::vector<uint8_t> host;      // [nseg] 1: a strip of the segment is pinned / registered HOST
                                    // memory (known only to a context that resolves host pointers)
    std::vector<uint8_t> fail;      // op 2: [nseg][k/2] exponents
    // Double-buffered pointer storage: a flush whose pieces DMA straight from
    // `ptrs` records uploaded[0] behind those copies and swaps in `spare`, so the
    // next batch is walked while the copies run; a buffer is written again only
    // once its copies are done.
    PinnedPtrs spare;
    hipEvent_t uploaded[2] = {nullptr, nullptr};  // [0] for ptrs, [1] for spare
    bool pending[2] = {false, false};
    bool direct = false;  // copies of this batch DMA'd from ptrs
    // Pieces uploaded from inside the queueing calls, ahead of the flush (see
    // stage_ahead): always the batch's leading segments [0, staged_upto), in order.
    std::vector<Staged> staged;
    size_t staged_upto = 0;
    uint64_t tail_bytes = 0;  // sum of len over the segments from staged_upto on

    int ready()  // before writing into ptrs
    {
        if (!pending[0])
            return 0;
        pending[0] = false;
        const hipError_t e = hipEventSynchronize(uploaded[0]);
        return e == hipSuccess ? 0 : draid::fail_hip(e, "hipEventSynchronize(descriptors)");
    }
};

struct Slot {
    void* host = nullptr;  // pinned
    void* host_dev = nullptr;  // the device's address of `host`
    void* dev = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;      // an event of this slot's own
    hipEvent_t wait = nullptr;      // recorded behind the slot's latest kernel: `done`, or
                                    // the event one flush shares (record_launched)
    hipEvent_t uploaded = nullptr;  // the piece's descriptors are on the device
    bool used = false;
    bool unrecorded = false;        // launched, no event recorded behind it yet
    bool staged = false;            // holds a piece that has not launched yet: not to be reused
};

int ctx_fail(hipError_t e, const char* what) { return draid::fail_hip(e, what); }
int ctx_arg(const char* what) { return draid::fail_arg(what); }

size_t align8(size_t x) { return (x + 7) & ~size_t(7); }

}  // namespace

struct draid_ec_ctx {
    hipStream_t stream = nullptr;   // kernels
    hipStream_t copy = nullptr;     // descriptor uploads
    int device = 0;
    std::deque<Group> groups;  // deque: groups never move (pinned storage, events)
    Slot slots[kSlots];
    int next = 0;
    std::vector<int> unrecorded;  // slots launched since the last event record (record_launched)
    int staged_slots = 0;    // slots holding uploaded pieces that wait for their launch
    bool stage_ahead = true; // DRAID_EC_CTX_STAGE_AHEAD=0 turns the early uploads off (A/B, tests)
    size_t inplace_limit = kInplaceLimit;  // DRAID_EC_CTX_INPLACE_LIMIT (A/B, tests; 0: never)
    uint64_t queued_segments = 0;
    int address_order = 1;  // DRAID_EC_CTX_ADDRESS_ORDER: 0 off, 1 auto, 2 any out-of-order group
                            // (diagnostics and tests)
    std::vector<uint32_t> perm, bucket;
    uint64_t autoflush = 0;  // launch a group once it holds this many segments (0 = off)
    uint64_t seq = 0;        // segments queued so far (orders the groups of a flush)
    bool host_pointers = false;  // iov_base values are the caller's host addresses: resolve them
    bool compact_rows = true;    // DRAID_EC_CTX_ROWS=64 turns compact rows off (A/B, tests)
    // A run whose strips lie more than 2 GiB apart goes into a group of its own, which is a
    // launch of its own: a caller whose buffers are spread like that (a request pool far from
    // the user buffers) would pay two launches per flush for as long as some runs fit and
    // some do not.  So after such a run every row is a row of pointers until kWideFlushes
    // flushes have passed without one.
    uint64_t flushes = 0, wide_until = 0;
    int fail_after = 0;      // test hook: the n-th piece from now fails before it launches
    // Flush tickets: an event recorded behind each ticketed flush, so a poller can
    // complete the requests of one flush while later ones are still running.
    static constexpr uint64_t kTickets = 64;
    hipEvent_t ticket_ev[kTickets] = {};
    uint64_t ticket_next = 1, ticket_done = 0;
    // draid_ec_ctx_mark / rollback: segments per group when the mark was set, and
    // how many launches had happened (a launch since then makes it stale).
    std::vector<size_t> mark_nseg;
    uint64_t mark_seq = 0, mark_launches = 0, launches = 0;
    bool marked = false;
    uint32_t level = 0;  // segments queued now go to groups of this level
};

namespace {
// Work on a context's streams is issued with its device current.
struct DeviceGuard {
    int prev = -1;
    bool switched = false;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev)
            switched = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard()
    {
        if (switched)
            (void)hipSetDevice(prev);
    }
};

void recount(draid_ec_ctx* c)
{
    uint64_t n = 0;
    for (const Group& g : c->groups)
        n += g.len.size();
    c->queued_segments = n;
}
}  // namespace

namespace {

// Address order.  A batch whose stripes sit at scattered addresses (stripe-cache
// slots or user buffers taken out of order) runs 7-11% slower than the same
// stripes visited in address order (measured: locality at tens-of-MiB
// scale), so a group whose segments jump back in memory is launched sorted by
// the address of their first strip -- a stable counting sort into at most 4096
// buckets (>= 1 MiB each) over the group's address range, O(segments).
// Segments of one group have no mutual order to keep: they run in one kernel or
// in pieces of it.  Left as queued: groups that never step back more than
// kOrderSlack (locally reversed runs are as local as sorted ones), and groups of
// small segments, whose kernel time per segment is below the cost of packing
// them one by one.
constexpr uintptr_t kOrderSlack = 16u << 20;
constexpr uint64_t kOrderMinSegmentBytes = 128u << 10;  // len * (k + m), on average

// Returns the order (segment i -> g's segment perm[i]), or null: keep as queued.
const uint32_t* address_order(draid_ec_ctx* c, const Group& g)
{
    const size_t nseg = g.len.size(), n = g.k + g.m;
    const bool force = c->address_order == 2;
    if (!c->address_order || nseg < 2)
        return nullptr;
    uint64_t bytes = 0;
    for (uint32_t l : g.len)
        bytes += l;
    if (!force && bytes * n < kOrderMinSegmentBytes * nseg)
        return nullptr;
    auto key = [&](size_t s) { return reinterpret_cast<uintptr_t>(g.ptrs[s * g.w]); };
    uintptr_t lo = key(0), hi = lo;
    bool local = true;
    for (size_t s = 1; s < nseg; ++s) {
        const uintptr_t v = key(s);
        local &= v + (force ? 0 : kOrderSlack) >= (force ? key(s - 1) : hi);
        lo = std::min(lo, v);
        hi = std::max(hi, v);
    }
    if (local)
        return nullptr;
    int shift = force ? 0 : 20;
    while (((hi - lo) >> shift) >= 4096)
        ++shift;
    const size_t nb = ((hi - lo) >> shift) + 1;
    c->bucket.assign(nb + 1, 0);
    for (size_t s = 0; s < nseg; ++s)
        ++c->bucket[((key(s) - lo) >> shift) + 1];
    for (size_t b = 1; b <= nb; ++b)
        c->bucket[b] += c->bucket[b - 1];
    c->perm.resize(nseg);
    for (size_t s = 0; s < nseg; ++s)
        c->perm[c->bucket[(key(s) - lo) >> shift]++] = static_cast<uint32_t>(s);
    return c->perm.data();
}

Group& group_for(draid_ec_ctx* c, int op, uint32_t k, uint32_t m, bool compact)
{
    for (Group& g : c->groups)
        if (g.op == op && g.k == k && g.m == m && g.level == c->level && g.compact == compact)
            return g;
    c->groups.emplace_back(op, k, m, c->level, compact);
    return c->groups.back();
}

// Iterator over one strip's iovec list (raid5_simple.c iov_iter).  It carries
// the current position and the bytes left in the current iovec, so the walk
// reads the iovec array only when an iovec ends.
struct IovIter {
    const struct iovec* v;
    int cnt;
    int idx;
    const uint8_t* p;  // current byte (the caller's address)
    size_t left;       // bytes left in v[idx] from p
    intptr_t delta;    // device address = p + delta (0 unless the ctx resolves host pointers)
    bool xl;           // resolve each iovec (draid_ec_ctx_set_host_pointers)
    bool bad;          // an iovec was not GPU accessible
    bool host;         // the iovec the iterator stands in is pinned / registered host memory
    int device;        // the context's GPU: where the kernels will run

    // Device-address offset of one iovec, or false when the GPU cannot reach it.
    static bool resolve(const struct iovec& e, intptr_t* d, int device, bool* host_memory)
    {
        *d = 0;
        *host_memory = false;
        if (e.iov_len == 0)
            return true;
        const void* dev = nullptr;
        if (draid::translate(e.iov_base, e.iov_len, &dev, device, host_memory))
            return false;
        *d = static_cast<const uint8_t*>(dev) - static_cast<const uint8_t*>(e.iov_base);
        return true;
    }

    void enter(int i)
    {
        idx = i;
        p = static_cast<const uint8_t*>(v[i].iov_base);
        left = v[i].iov_len;
        if (xl) {
            bool h = false;
            if (!resolve(v[i], &delta, device, &h))
                bad = true;
            host = h;  // of the iovec the iterator stands in
        }
    }
};

// Positions the iterator `offset` bytes into the list (raid5.c:235-255).
bool iter_seek(IovIter& it, size_t offset)
{
    int i = 0;
    while (i < it.cnt && offset >= it.v[i].iov_len) {
        offset -= it.v[i].iov_len;
        ++i;
    }
    if (i >= it.cnt)
        return false;
    it.enter(i);
    it.p += offset;
    it.left -= offset;
    return true;
}

int flush_group(draid_ec_ctx* c, Group& g);
size_t piece_segments(const Group& g);
int stage_ahead(draid_ec_ctx* c, Group& g);

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
        it[j] = IovIter{iovs[j], iovcnt[j], 0, nullptr, 0, 0, c->host_pointers, false, false,
                        c->device};
        if (len && !iter_seek(it[j], offset ? offset[j] : 0))
            return ctx_arg("iovec list shorter than offset");
        if (it[j].bad)
            return ctx_arg("an iovec is neither memory of the context's GPU nor pinned / "
                           "registered host memory");
    }
    // A run whose strips all lie within +-2 GiB of its first strip -- every run of
    // an ordinary stripe -- is queued as a compact row; one that does not is queued
    // as a row of pointers, in a group of its own ((op, k, m) groups carry no order
    // among their segments, so splitting them by row format changes nothing).
    struct Touched {
        Group* g = nullptr;
        size_t n_ptrs = 0, n_len = 0, n_fail = 0;
        uint64_t tail_bytes = 0;
    } touched[2];
    int ready_rc = 0;
    auto use = [&](bool compact) -> Group* {
        Touched& t = touched[compact ? 1 : 0];
        if (!t.g) {
            Group& g = group_for(c, op, k, m, compact);
            if ((ready_rc = g.ready()) != 0)
                return nullptr;
            t.g = &g;
            t.n_ptrs = g.ptrs.size();
            t.n_len = g.len.size();
            t.n_fail = g.fail.size();
            t.tail_bytes = g.tail_bytes;
        }
        return t.g;
    };
    const uint64_t n_q = c->queued_segments, n_seq = c->seq;
    auto rollback = [&](const char* what) {  // a rejected stripe queues nothing
        for (Touched& t : touched)
            if (t.g) {
                t.g->ptrs.shrink(t.n_ptrs);
                t.g->len.resize(t.n_len);
                t.g->host.resize(t.n_len);
                t.g->fail.resize(t.n_fail);
                t.g->tail_bytes = t.tail_bytes;
            }
        c->queued_segments = n_q;
        c->seq = n_seq;
        return ctx_arg(what);
    };
    bool may_compact = c->compact_rows && op != 2 && c->flushes >= c->wide_until;
    const uint8_t* ptr[512];
    uintptr_t fpair = 0;
    if (op == 1)
        memcpy(&fpair, meta, 2);
    size_t remaining = len;
    while (remaining > 0) {
        size_t run = std::min<size_t>(remaining, kMaxSegment);
        for (uint32_t j = 0; j < n; ++j) {
            IovIter& t = it[j];
            if (t.left >= run)
                continue;  // this strip does not shorten the run
            while (t.left == 0) {  // skip exhausted / zero-length entries
                if (t.idx + 1 >= t.cnt)
                    return rollback("iovec list shorter than len");
                t.enter(t.idx + 1);
            }
            if (t.left >= run)
                continue;  // the next iovec covers the run: no merge scan
            // Bytes available contiguously from here: the rest of this iovec plus
            // any following iovecs that continue it in memory (a split buffer
            // needs no extra descriptors; the arithmetic is per byte, so merging
            // adjacent runs cannot change the result).
            size_t avail = t.left;
            const uint8_t* end = t.p + t.left;
            for (int x = t.idx + 1; x < t.cnt && avail < run; ++x) {
                if (t.v[x].iov_len == 0)
                    continue;
                if (t.v[x].iov_base != end)
                    break;
                if (t.xl) {  // adjacent for the host: also adjacent for the device?
                    intptr_t d;
                    bool h;
                    if (!IovIter::resolve(t.v[x], &d, t.device, &h) || d != t.delta)
                        break;
                }
                avail += t.v[x].iov_len;
                end += t.v[x].iov_len;
            }
            run = std::min<size_t>(run, avail);
        }
        // One pass writes the run's row and moves every strip's iterator on.  The row
        // is written as a compact one where those are allowed, and redone as a row of
        // pointers in the rare run that turns out not to fit.
        Group* gp = use(may_compact);
        if (!gp) {
            const int rc = ready_rc;
            (void)rollback("descriptor storage not ready");
            return rc;
        }
        // (growing moves the rows: no early upload may still be reading them)
        if (gp->direct && gp->ptrs.full(gp->w))
            (void)hipStreamSynchronize(c->copy);
        const void** out = gp->ptrs.grow(gp->w);
        if (!out)
            return rollback("out of pinned host memory for descriptors");
        const uint8_t* const p0 = it[0].p + it[0].delta;
        int32_t* const off = reinterpret_cast<int32_t*>(out + 1);
        bool fits = true, bad = false, seg_host = false;
        for (uint32_t j = 0; j < n; ++j) {
            IovIter& t = it[j];
            const uint8_t* const pj = t.p + t.delta;
            ptr[j] = pj;
            seg_host |= t.host;
            if (may_compact) {
                const intptr_t d = pj - p0;
                off[j] = static_cast<int32_t>(d);
                fits &= d == static_cast<int32_t>(d);
            } else {
                out[j] = pj;
            }
            if (run <= t.left) {
                t.p += run;
                t.left -= run;
            } else {
                size_t r = run;  // crossed merged iovecs
                while (r > t.left) {
                    r -= t.left;
                    t.enter(t.idx + 1);
                }
                t.p += r;
                t.left -= r;
            }
            bad |= t.bad;
        }
        if (bad)
            return rollback("an iovec is neither memory of the context's GPU nor pinned / "
                            "registered host memory");
        if (may_compact && fits) {
            out[0] = p0;
            if (op == 1)
                off[n] = static_cast<int32_t>(fpair);  // the failure pair rides behind the strips
        } else {
            if (may_compact) {  // strips more than 2 GiB apart: a row of pointers after all
                c->wide_until = c->flushes + kWideFlushes;
                gp->ptrs.shrink(gp->ptrs.size() - gp->w);
                if (!(gp = use(false))) {
                    const int rc = ready_rc;
                    (void)rollback("descriptor storage not ready");
                    return rc;
                }
                if (gp->direct && gp->ptrs.full(gp->w))
                    (void)hipStreamSynchronize(c->copy);
                if (!(out = gp->ptrs.grow(gp->w)))
                    return rollback("out of pinned host memory for descriptors");
                for (uint32_t j = 0; j < n; ++j)
                    out[j] = ptr[j];
                may_compact = false;  // the rest of this stripe's runs too
            }
            if (op == 1)
                out[n] = reinterpret_cast<const void*>(fpair);
        }
        Group& g = *gp;
        if (g.len.empty())
            g.first_seq = c->seq;
        ++c->seq;
        g.len.push_back(static_cast<uint32_t>(run));
        g.host.push_back(seg_host ? 1 : 0);
        g.tail_bytes += run;
        if (op != 1 && nmeta)
            g.fail.insert(g.fail.end(), meta, meta + nmeta);
        ++c->queued_segments;
        remaining -= run;
    }
    // (a group behind a fence waits for the flush: its predecessors must launch first)
    for (Touched& t : touched) {
        if (t.g && c->autoflush && t.g->level == 0 && t.g->len.size() >= c->autoflush) {
            DeviceGuard on(c->device);
            const int rc = flush_group(c, *t.g);
            recount(c);
            if (rc)
                return rc;
        } else if (t.g && c->stage_ahead && t.g->len.size() - t.g->staged_upto >= piece_segments(*t.g)) {
            DeviceGuard on(c->device);
            const int rc = stage_ahead(c, *t.g);
            if (rc)
                return rc;
        }
    }
    return 0;
}

constexpr int kSlotBusy = 0x7fff;  // stage_piece(ahead): not an error, nothing staged

// Segments of a group per launch: about kPieceBytes of descriptors.
size_t piece_segments(const Group& g)
{
    const size_t per_seg = g.w * sizeof(void*) + sizeof(uint32_t) + 2 * sizeof(uint32_t);
    return std::max<size_t>(kMinPieceSegments, kPieceBytes / per_seg);
}

// Forgets the staged pieces that reach beyond segment `keep` (their slots are
// free again; copies still in flight into them are harmless, the copy stream
// runs the next upload into the same slot behind them).
void drop_staged(draid_ec_ctx* c, Group& g, size_t keep)
{
    while (!g.staged.empty() && g.staged.back().s1 > keep) {
        c->slots[g.staged.back().slot].staged = false;
        --c->staged_slots;
        g.staged.pop_back();
    }
    g.staged_upto = g.staged.empty() ? 0 : g.staged.back().s1;
    uint64_t tail = 0;
    for (size_t s = g.staged_upto; s < g.len.size(); ++s)
        tail += g.len[s];
    g.tail_bytes = tail;
}

// One event for all the pieces launched since the last one: a record between two
// kernels costs the stream 3-4 us, so a flush records once behind its last piece, not
// behind each, and a ticketed flush lets the ticket's event serve (`shared`, which the
// caller has just recorded).  The slots wait on that event before they are used again.
int record_launched(draid_ec_ctx* c, hipEvent_t shared)
{
    if (c->unrecorded.empty())
        return 0;
    hipEvent_t ev = shared;
    if (!ev) {
        ev = c->slots[c->unrecorded.back()].done;
        const hipError_t e = hipEventRecord(ev, c->stream);
        if (e != hipSuccess)
            return ctx_fail(e, "hipEventRecord(slots)");
    }
    for (int si : c->unrecorded) {
        c->slots[si].wait = ev;
        c->slots[si].unrecorded = false;
    }
    c->unrecorded.clear();
    return 0;
}

// First half of a launch over segments [s0, s1) of a group: pack their
// descriptors into the next pinned ring slot and DMA them on the copy stream.
// `perm` (may be null): segment i of the group is g's segment perm[i].
// `ahead`: called from a queueing call -- never waits for a slot still in use
// (returns kSlotBusy and stages nothing).
int stage_piece(draid_ec_ctx* c, Group& g, const uint32_t* perm, size_t s0, size_t s1, bool ahead,
                Staged* out)
{
    const size_t nseg = s1 - s0;
    const size_t nmeta = g.fail.size() / g.len.size();  // bytes of meta per segment
    const uint32_t cb = draid::work_chunk_bytes(g.op, g.k);
    std::vector<uint32_t> plen;
    if (perm) {
        plen.resize(nseg);
        for (size_t i = 0; i < nseg; ++i)
            plen[i] = g.len[perm[s0 + i]];
    }
    const uint32_t* lenp = perm ? plen.data() : g.len.data() + s0;
    // Uniform segments (every run the same length: whole strips, fixed-size
    // iovecs) need no work list -- the kernel derives (segment, chunk) itself.
    const bool uniform =
        std::all_of(lenp, lenp + nseg, [&](uint32_t l) { return l == lenp[0]; });
    std::vector<uint32_t> work;  // pairs {seg, chunk}
    uint64_t nwork64;
    if (uniform) {
        nwork64 = static_cast<uint64_t>(nseg) * std::max<uint32_t>(1, (lenp[0] + cb - 1) / cb);
    } else {
        for (size_t s = 0; s < nseg; ++s) {
            const uint32_t cps = std::max<uint32_t>(1, (lenp[s] + cb - 1) / cb);
            for (uint32_t ch = 0; ch < cps; ++ch) {
                work.push_back(static_cast<uint32_t>(s));
                work.push_back(ch);
            }
        }
        nwork64 = work.size() / 2;
    }
    if (nwork64 > 0x7fffffffull)
        return ctx_arg("flush: too many work items queued (flush more often)");
    const size_t o_ptr = 0;
    const uint32_t w = g.w;
    const size_t o_len = align8(o_ptr + nseg * w * sizeof(void*));
    const size_t o_fail = align8(o_len + (uniform ? 0 : nseg * sizeof(uint32_t)));
    const size_t o_work = align8(o_fail + nseg * nmeta);
    const size_t bytes = o_work + work.size() * sizeof(uint32_t);

    // the next slot that holds no piece waiting for its launch (at least
    // kSlots - kMaxStaged of them never do)
    int si = c->next;
    while (c->slots[si].staged)
        si = (si + 1) % kSlots;
    Slot& sl = c->slots[si];
    hipError_t e;
    if (sl.used) {  // back-pressure: the slot's previous upload+launch must be done
        if (sl.unrecorded) {  // launched in this very batch: its event is still to come
            const int rc = record_launched(c, nullptr);
            if (rc)
                return rc;
        }
        if (ahead) {
            if ((e = hipEventQuery(sl.wait)) == hipErrorNotReady) {
                (void)hipGetLastError();
                return kSlotBusy;
            }
        } else {
            e = hipEventSynchronize(sl.wait);
        }
        if (e != hipSuccess)
            return ctx_fail(e, "hipEventSynchronize(slot)");
    }
    c->next = (si + 1) % kSlots;
    if (sl.cap < bytes) {
        if (sl.host)
            (void)hipHostFree(sl.host);
        if (sl.dev)
            (void)hipFree(sl.dev);
        sl.host = sl.host_dev = sl.dev = nullptr;
        sl.cap = 0;
        const size_t cap = std::max<size_t>(bytes * 2, 64 * 1024);
        if ((e = hipHostMalloc(&sl.host, cap, hipHostMallocDefault)) != hipSuccess)
            return ctx_fail(e, "hipHostMalloc(descriptor ring)");
        if ((e = hipHostGetDevicePointer(&sl.host_dev, sl.host, 0)) != hipSuccess)
            return ctx_fail(e, "hipHostGetDevicePointer(descriptor ring)");
        if ((e = hipMalloc(&sl.dev, cap)) != hipSuccess)
            return ctx_fail(e, "hipMalloc(descriptor ring)");
        sl.cap = cap;
    }
    uint8_t* h = static_cast<uint8_t*>(sl.host);
    // A small launch (a poller's batch of a few dozen requests) reads its
    // descriptors in place: uploading a few KiB costs the host 20 us of runtime calls
    // (copy, event, cross-stream wait) and the GPU as long again before the kernel may
    // start, while the kernel's reads of pinned memory add a PCIe round trip per item,
    // which a launch this small does not notice.  Large launches do (4096 stripes of
    // 4 KiB runs: 1.39 vs 1.00 ms), so they upload.  Wall time of one flush of B
    // 8+2 stripes at 64 KiB runs (64 items each), in place vs uploaded: B = 2..32
    // 21-25 vs 41-46 us, 64: 31 vs 46, 128: 42 vs 53, 256: 59-65 vs 74-75, 1024: encode
    // 198 vs 177; at 4 KiB runs (4 items each) 64 stripes = 1024 segments 65 vs 72,
    // 256 stripes = 4096 segments 195 vs 176.  That fits about 8 ns per segment (its
    // row's first trip over the link) plus 0.5 ns per item (the row again, from the
    // cache) against the upload's 20 us, which is the limit above with some margin.
    const bool inplace = !ahead && nwork64 + 16 * static_cast<uint64_t>(nseg) <= c->inplace_limit;
    if (inplace && !perm)
        memcpy(h + o_ptr, g.ptrs.data() + s0 * w, nseg * w * sizeof(void*));
    if (perm) {
        auto* hp = reinterpret_cast<const void**>(h + o_ptr);
        for (size_t i = 0; i < nseg; ++i)
            memcpy(hp + i * w, g.ptrs.data() + (size_t)perm[s0 + i] * w, w * sizeof(void*));
        for (size_t i = 0; nmeta && i < nseg; ++i)
            memcpy(h + o_fail + i * nmeta, g.fail.data() + (size_t)perm[s0 + i] * nmeta, nmeta);
    } else if (nmeta) {
        memcpy(h + o_fail, g.fail.data() + s0 * nmeta, nseg * nmeta);
    }
    if (!uniform)
        memcpy(h + o_len, lenp, nseg * sizeof(uint32_t));
    if (!work.empty())
        memcpy(h + o_work, work.data(), work.size() * sizeof(uint32_t));
    // DMA the piece's descriptors: a piece in queue order takes its rows straight
    // from the group's pinned storage and only the rest (lengths, update exponents,
    // work list; none for uniform encode segments) from the slot; a piece in address
    // order was packed into the slot row by row above and goes up in one copy.
    if (inplace)
        e = hipSuccess;
    else if (perm)
        e = hipMemcpyAsync(sl.dev, sl.host, bytes, hipMemcpyHostToDevice, c->copy);
    else {
        e = hipMemcpyAsync(static_cast<uint8_t*>(sl.dev) + o_ptr, g.ptrs.data() + s0 * w,
                           nseg * w * sizeof(void*), hipMemcpyHostToDevice, c->copy);
        if (e == hipSuccess && bytes > o_len)
            e = hipMemcpyAsync(static_cast<uint8_t*>(sl.dev) + o_len, h + o_len, bytes - o_len,
                               hipMemcpyHostToDevice, c->copy);
        g.direct = true;
    }
    if (e != hipSuccess)
        return ctx_fail(e, "hipMemcpyAsync(descriptors)");
    if (!inplace && (e = hipEventRecord(sl.uploaded, c->copy)) != hipSuccess)
        return ctx_fail(e, "descriptor upload event");
    size_t host_segs = 0;
    for (size_t i = 0; i < nseg; ++i)
        host_segs += g.host[perm ? perm[s0 + i] : s0 + i];
    out->host_data = 2 * host_segs > nseg;
    out->inplace = inplace;
    out->slot = si;
    out->s0 = s0;
    out->s1 = s1;
    out->uniform = uniform;
    out->nwork = static_cast<uint32_t>(nwork64);
    out->ulen = lenp[0];
    out->o_len = o_len;
    out->o_fail = o_fail;
    out->o_work = o_work;
    return 0;
}

// Second half: the piece's kernel on the compute stream, behind its upload.
// Copies therefore overlap the kernels of earlier pieces and flushes.
int launch_piece(draid_ec_ctx* c, Group& g, const Staged& st)
{
    Slot& sl = c->slots[st.slot];
    const uint32_t n = g.k + g.m, w = g.w;
    hipError_t e;
    if (!st.inplace && (e = hipStreamWaitEvent(c->stream, sl.uploaded, 0)) != hipSuccess)
        return ctx_fail(e, "descriptor upload event");
    const uint8_t* d = static_cast<const uint8_t*>(st.inplace ? sl.host_dev : sl.dev);
    // strips in host memory: a PCIe-bound launch runs faster with few items resident
    draid::HostLaunch host(st.host_data);
    const auto* tab = reinterpret_cast<const uint8_t* const*>(d);
    const auto* lens = reinterpret_cast<const uint32_t*>(d + st.o_len);
    const void* wl = st.uniform ? nullptr : d + st.o_work;
    const uint32_t row_bytes = g.compact ? static_cast<uint32_t>(w * sizeof(void*)) : 0u;
    // the failure pair's place in a row: behind the k + m pointers, or offsets
    const size_t o_pair = g.compact ? 8 + 4 * static_cast<size_t>(n) : n * sizeof(void*);
    if (g.op == 0)
        e = draid::launch_encode_work(g.k, g.m, tab, row_bytes, lens, wl, st.ulen, st.nwork,
                                      c->stream);
    else if (g.op == 1)
        e = draid::launch_reconstruct_work(g.k, g.m, tab, w, row_bytes, lens, d + o_pair,
                                           static_cast<uint32_t>(w * sizeof(void*)), wl, st.ulen,
                                           st.nwork, c->stream);
    else
        e = draid::launch_update_work(g.m, g.k / 2, tab, d + st.o_fail, lens, wl, st.ulen,
                                      st.nwork, c->stream);
    if (e != hipSuccess)
        return ctx_fail(e, "launch (segment work list)");
    sl.used = true;
    if (!sl.unrecorded) {
        sl.unrecorded = true;
        c->unrecorded.push_back(st.slot);
    }
    return 0;
}

// Descriptors ahead of the flush.  A batch of small runs carries a lot of
// descriptor bytes per strip byte (4 KiB iovecs: 3 MiB per 4096 stripes), and a
// flush that starts uploading them only when it is called leaves the GPU waiting
// for the first piece.  So once a group holds a whole piece of segments that no
// flush will reorder (small ones), the queueing call that completes the piece
// uploads it there and then; the flush finds it on the device and only launches.
// A piece is final when it is uploaded: segments are only ever appended, and a
// rollback that cuts into a staged piece drops it (drop_staged).
int stage_ahead(draid_ec_ctx* c, Group& g)
{
    const size_t piece = piece_segments(g);
    const uint32_t n = g.k + g.m;
    while (g.len.size() - g.staged_upto >= piece && c->staged_slots < kMaxStaged) {
        const size_t tail = g.len.size() - g.staged_upto;
        if (g.tail_bytes * n >= kOrderMinSegmentBytes * tail)
            break;  // large segments: few descriptors, and the flush may sort them
        Staged st;
        const int rc = stage_piece(c, g, nullptr, g.staged_upto, g.staged_upto + piece, true, &st);
        if (rc == kSlotBusy)
            break;  // the next free slot is still in flight: the flush will do it
        if (rc)
            return rc;
        uint64_t bytes = 0;
        for (size_t s = st.s0; s < st.s1; ++s)
            bytes += g.len[s];
        g.tail_bytes -= bytes;
        c->slots[st.slot].staged = true;
        ++c->staged_slots;
        g.staged.push_back(st);
        g.staged_upto = st.s1;
    }
    return 0;
}

// Launches a group in pieces of about kPieceBytes of descriptors, so the upload
// of piece i+1 overlaps the kernel of piece i.
// A group of one segment whose pointers fit in the kernel arguments (the
// low-queue-depth case: one stripe per poll) launches the single-stripe kernel
// directly -- no descriptor upload, no ring slot, no cross-stream event.
int flush_single(draid_ec_ctx* c, Group& g)
{
    draid::ArgPtrTable args;
    memset(&args, 0, sizeof(args));
    const uint32_t n = g.k + g.m;
    const uint8_t* row = reinterpret_cast<const uint8_t*>(g.ptrs.data());
    for (uint32_t j = 0; j < n; ++j) {
        if (g.compact) {
            int32_t off;
            memcpy(&off, row + 8 + 4 * j, sizeof(off));
            args.p[j] = static_cast<const uint8_t*>(g.ptrs[0]) + off;
        } else {
            args.p[j] = static_cast<const uint8_t*>(g.ptrs[j]);
        }
    }
    hipError_t e;
    if (g.op == 0)
        e = draid::launch_encode(g.k, g.m, g.len[0], 1, nullptr, &args, c->stream);
    else {
        uint8_t f[4];
        memcpy(f, row + (g.compact ? 8 + 4 * n : n * sizeof(void*)), sizeof(f));  // the pair's slot
        e = draid::launch_reconstruct(g.k, g.m, g.len[0], 1, nullptr, &args, nullptr, f[0], f[1],
                                      nullptr, c->stream);
    }
    g.ptrs.clear();
    g.len.clear();
    g.host.clear();
    g.fail.clear();
    g.tail_bytes = 0;
    return e == hipSuccess ? 0 : ctx_fail(e, "launch (single segment)");
}

int flush_group(draid_ec_ctx* c, Group& g)
{
    const size_t nseg = g.len.size();
    if (nseg == 0)
        return 0;
    ++c->launches;
    if (nseg == 1 && g.op != 2 && g.k + g.m <= static_cast<uint32_t>(draid::kMaxArgPtrs))
        return flush_single(c, g);
    const size_t piece = piece_segments(g);
    // (a batch with pieces on the device already keeps its queue order)
    const uint32_t* perm = g.staged.empty() ? address_order(c, g) : nullptr;
    int rc = 0;
    size_t launched = 0;
    auto injected = [&]() {  // test hook: this piece fails before it launches
        return c->fail_after > 0 && --c->fail_after == 0
                   ? ctx_fail(hipErrorOutOfMemory, "flush piece (injected failure)")
                   : 0;
    };
    for (const Staged& st : g.staged) {
        if ((rc = injected()) != 0 || (rc = launch_piece(c, g, st)) != 0)
            break;
        launched = st.s1;
    }
    for (size_t s0 = g.staged_upto; rc == 0 && s0 < nseg; s0 += piece) {
        Staged st;
        if ((rc = injected()) != 0 ||
            (rc = stage_piece(c, g, perm, s0, std::min(nseg, s0 + piece), false, &st)) != 0 ||
            (rc = launch_piece(c, g, st)) != 0)
            break;
        launched = st.s1;
    }
    drop_staged(c, g, 0);  // launched, or (on failure) queued again below
    if (rc && launched < nseg) {
        // A piece failed (descriptor memory, the work-item limit, a launch error):
        // the pieces before it are running, this one and the rest are not.  Keep
        // exactly those segments queued, in their queue order, so the caller can
        // flush again or fail precisely the requests that did not run.
        (void)hipStreamSynchronize(c->copy);  // nothing may still read g.ptrs
        g.pending[0] = g.pending[1] = false;
        g.direct = false;
        std::vector<uint32_t> rest;
        rest.reserve(nseg - launched);
        for (size_t i = launched; i < nseg; ++i)
            rest.push_back(perm ? perm[i] : static_cast<uint32_t>(i));
        std::sort(rest.begin(), rest.end());
        const size_t nmeta = g.fail.size() / nseg;
        const void** rows = g.ptrs.data();
        uint64_t tail = 0;
        for (size_t i = 0; i < rest.size(); ++i) {  // rest[i] >= i: forward moves are safe
            memmove(rows + i * g.w, rows + static_cast<size_t>(rest[i]) * g.w,
                    g.w * sizeof(void*));
            g.len[i] = g.len[rest[i]];
            g.host[i] = g.host[rest[i]];
            tail += g.len[i];
            if (nmeta)
                memmove(g.fail.data() + i * nmeta, g.fail.data() + rest[i] * nmeta, nmeta);
        }
        g.ptrs.shrink(rest.size() * g.w);
        g.len.resize(rest.size());
        g.host.resize(rest.size());
        g.fail.resize(rest.size() * nmeta);
        g.tail_bytes = tail;
        return rc;
    }
    if (g.direct) {  // copies from g.ptrs in flight: walk the next batch into the spare
        hipError_t e = hipSuccess;
        if (!g.uploaded[0])
            e = hipEventCreateWithFlags(&g.uploaded[0], hipEventDisableTiming);
        if (e == hipSuccess)
            e = hipEventRecord(g.uploaded[0], c->copy);
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(c->copy);
            if (rc == 0)
                rc = ctx_fail(e, "descriptor storage event");
        } else {
            g.pending[0] = true;
        }
        g.ptrs.swap(g.spare);
        std::swap(g.uploaded[0], g.uploaded[1]);
        std::swap(g.pending[0], g.pending[1]);
        g.direct = false;
    }
    g.ptrs.clear();
    g.len.clear();
    g.host.clear();
    g.fail.clear();
    g.tail_bytes = 0;
    return rc;
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
    const char* rows = getenv("DRAID_EC_CTX_ROWS");
    if (rows && strcmp(rows, "64") == 0)
        c->compact_rows = false;
    const char* order = getenv("DRAID_EC_CTX_ADDRESS_ORDER");
    if (order && (order[0] == '0' || order[0] == '2'))
        c->address_order = order[0] - '0';
    const char* ahead = getenv("DRAID_EC_CTX_STAGE_AHEAD");
    // (a context told to sort every group cannot upload pieces in queue order)
    if ((ahead && ahead[0] == '0') || c->address_order == 2)
        c->stage_ahead = false;
    if (const char* inplace = getenv("DRAID_EC_CTX_INPLACE_LIMIT"))
        c->inplace_limit = strtoul(inplace, nullptr, 0);
    hipError_t e = hipGetDevice(&c->device);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking);
    for (int i = 0; e == hipSuccess && i < kSlots; ++i) {
        e = hipEventCreateWithFlags(&c->slots[i].done, hipEventDisableTiming);
        if (e == hipSuccess)
            e = hipEventCreateWithFlags(&c->slots[i].uploaded, hipEventDisableTiming);
    }
    for (uint64_t i = 0; e == hipSuccess && i < draid_ec_ctx::kTickets; ++i)
        e = hipEventCreateWithFlags(&c->ticket_ev[i], hipEventDisableTiming);
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
    DeviceGuard on(c->device);
    if (c->stream)
        (void)hipStreamSynchronize(c->stream);
    for (hipEvent_t ev : c->ticket_ev)
        if (ev)
            (void)hipEventDestroy(ev);
    if (c->copy)
        (void)hipStreamSynchronize(c->copy);
    for (Slot& s : c->slots) {
        if (s.host)
            (void)hipHostFree(s.host);
        if (s.dev)
            (void)hipFree(s.dev);
        if (s.done)
            (void)hipEventDestroy(s.done);
        if (s.uploaded)
            (void)hipEventDestroy(s.uploaded);
    }
    if (c->stream)
        (void)hipStreamDestroy(c->stream);
    if (c->copy)
        (void)hipStreamDestroy(c->copy);
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
    if (!c || k < 1 || k + m > 255 || m < 1 || m > 2 || nfail < 0 || nfail > (int)m ||
        (nfail && !fail))
        return ctx_arg("reconstruct_sg needs a ctx, k >= 1, k + m <= 255, m in {1,2}, nfail <= m");
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

// record: one event behind everything this flush launched (false: the caller records
// one of its own and hands it to record_launched).
static int flush_all(draid_ec_ctx* c, bool record)
{
    DeviceGuard on(c->device);
    // Groups launch level by level (draid_ec_ctx_fence), and within a level in
    // the order their first segment of this batch was queued (a group object
    // outlives its batches, so creation order says nothing).
    Group* order[64];
    std::vector<Group*> many;
    size_t n = 0;
    for (Group& g : c->groups)
        if (!g.len.empty()) {
            if (n < 64)
                order[n] = &g;
            else {
                if (many.empty())
                    many.assign(order, order + 64);
                many.push_back(&g);
            }
            ++n;
        }
    Group** gp = many.empty() ? order : many.data();
    std::sort(gp, gp + n, [](const Group* a, const Group* b) {
        return a->level != b->level ? a->level < b->level : a->first_seq < b->first_seq;
    });
    int rc = 0;
    for (size_t i = 0; i < n && rc == 0; ++i)
        rc = flush_group(c, *gp[i]);
    recount(c);  // on failure: exactly the segments that did not launch
    c->level = 0;
    ++c->flushes;
    if (record || rc) {
        const int rr = record_launched(c, nullptr);
        if (rc == 0)
            rc = rr;
    }
    return rc;
}

int draid_ec_ctx_flush(draid_ec_ctx* c)
{
    if (!c)
        return ctx_arg("ctx is NULL");
    return flush_all(c, true);
}

int draid_ec_ctx_flush_ticket(draid_ec_ctx* c, uint64_t* ticket)
{
    if (!c || !ticket)
        return ctx_arg("flush_ticket needs a ctx and a ticket pointer");
    *ticket = 0;
    const int rc = flush_all(c, false);
    if (rc)
        return rc;
    DeviceGuard on(c->device);
    const uint64_t t = c->ticket_next;
    hipError_t e;
    if (t - c->ticket_done > draid_ec_ctx::kTickets) {  // the event slot is still in use
        const uint64_t old = t - draid_ec_ctx::kTickets;
        if ((e = hipEventSynchronize(c->ticket_ev[old % draid_ec_ctx::kTickets])) != hipSuccess) {
            (void)record_launched(c, nullptr);
            return ctx_fail(e, "hipEventSynchronize(ticket)");
        }
        c->ticket_done = old;
    }
    hipEvent_t tev = c->ticket_ev[t % draid_ec_ctx::kTickets];
    if ((e = hipEventRecord(tev, c->stream)) != hipSuccess) {
        (void)record_launched(c, nullptr);
        return ctx_fail(e, "hipEventRecord(ticket)");
    }
    // the ticket's event also tells when this flush's ring slots are free again (a slot
    // is used again 16 launches later at the earliest, the event 64 tickets later: were
    // it recorded again by then, the slot would wait for a later flush, never a shorter time)
    (void)record_launched(c, tev);
    c->ticket_next = t + 1;
    *ticket = t;
    return 0;
}

int draid_ec_ctx_ticket_query(draid_ec_ctx* c, uint64_t ticket)
{
    if (!c || ticket == 0 || ticket >= c->ticket_next)
        return ctx_arg("ticket_query: not a ticket of this context");
    if (ticket <= c->ticket_done)
        return 0;
    const hipError_t e = hipEventQuery(c->ticket_ev[ticket % draid_ec_ctx::kTickets]);
    if (e == hipSuccess) {
        c->ticket_done = ticket;  // stream order: every earlier flush is done too
        return 0;
    }
    if (e == hipErrorNotReady) {
        (void)hipGetLastError();
        return 1;
    }
    return ctx_fail(e, "hipEventQuery(ticket)");
}

int draid_ec_ctx_set_host_pointers(draid_ec_ctx* c, int on)
{
    if (!c)
        return ctx_arg("ctx is NULL");
    c->host_pointers = on != 0;
    return 0;
}

// Test hook (not in the public header): the n-th piece launched from now on
// fails before it does anything, as a descriptor allocation failure would.
void draid_ec_ctx_test_fail_after(draid_ec_ctx* c, int n)
{
    if (c)
        c->fail_after = n;
}

// Test hook (not in the public header): pieces uploaded ahead of the flush that
// wait for their launch.
int draid_ec_ctx_test_staged(draid_ec_ctx* c) { return c ? c->staged_slots : 0; }

int draid_ec_ctx_query(draid_ec_ctx* c)
{
    if (!c)
        return ctx_arg("ctx is NULL");
    hipError_t e = hipStreamQuery(c->stream);
    if (e == hipSuccess)
        return 0;
    if (e == hipErrorNotReady) {
        (void)hipGetLastError();
        return 1;
    }
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

int draid_ec_ctx_discard_queued(draid_ec_ctx* c)
{
    if (!c)
        return ctx_arg("ctx is NULL");
    for (Group& g : c->groups) {
        g.len.clear();
        g.host.clear();
        drop_staged(c, g, 0);
        // the storage may still feed an earlier flush's copies, or this batch's early ones
        if (g.ready() || g.direct)
            (void)hipStreamSynchronize(c->copy);
        g.direct = false;
        g.ptrs.clear();
        g.fail.clear();
    }
    c->queued_segments = 0;
    return 0;
}

int draid_ec_ctx_mark(draid_ec_ctx* c)
{
    if (!c)
        return ctx_arg("ctx is NULL");
    c->mark_nseg.resize(c->groups.size());
    size_t i = 0;
    for (const Group& g : c->groups)
        c->mark_nseg[i++] = g.len.size();
    c->mark_seq = c->seq;
    c->mark_launches = c->launches;
    c->marked = true;
    c->level = 0;  // a request starts in front of every fence
    return 0;
}

int draid_ec_ctx_fence(draid_ec_ctx* c)
{
    if (!c)
        return ctx_arg("ctx is NULL");
    ++c->level;
    return 0;
}

int draid_ec_ctx_rollback(draid_ec_ctx* c)
{
    if (!c)
        return ctx_arg("ctx is NULL");
    if (!c->marked)
        return ctx_arg("rollback without a mark");
    c->marked = false;
    if (c->launches != c->mark_launches)
        return ctx_arg("rollback: segments queued since the mark have been launched");
    size_t i = 0;
    for (Group& g : c->groups) {  // groups are only ever appended: index i is stable
        const size_t keep = i < c->mark_nseg.size() ? c->mark_nseg[i] : 0;
        ++i;
        const size_t have = g.len.size();
        if (have <= keep)
            continue;
        const size_t nmeta = g.fail.size() / have;
        g.ptrs.shrink(keep * g.w);
        g.len.resize(keep);
        g.host.resize(keep);
        g.fail.resize(keep * nmeta);
        drop_staged(c, g, keep);  // a piece uploaded early that held any of them
    }
    c->seq = c->mark_seq;
    c->level = 0;
    recount(c);
    return 0;
}

int draid_ec_ctx_set_autoflush(draid_ec_ctx* c, uint64_t segments)
{
    if (!c)
        return ctx_arg("ctx is NULL");
    c->autoflush = segments;
    return 0;
}

}  // extern "C"
