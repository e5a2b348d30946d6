/*
 * draid_ec.h -- C ABI of the MI355X erasure-coding engine (libdraid_ec.so).
 *
 * Drop-in boundary for the parity hot path of kyleshu/draid-spdk's RAID
 * bdev modules (module/bdev/raid/).  Two nested surfaces, the two the reference
 * itself has:
 *
 *  1. The isa-l v2.30 arithmetic ABI the raid modules call (raid.h /
 *     gf_vect_mul.h), re-implemented as HIP kernels on gfx950.  Same argument
 *     meaning, same array order, same 0 / non-zero return convention, and --
 *     like isa-l, which the reference hands spdk_dma_malloc'd chunk buffers and
 *     user iovecs (raid5.c:188-201) -- any kind of pointer: device memory is
 *     used in place; pinned or registered host memory is read and written in
 *     place through its device address (looked up per call, cached per thread);
 *     pageable host memory is copied through a per-thread staging buffer
 *     (pinned host memory for calls that stage up to 8 MiB, device memory
 *     beyond).  No pointer the GPU cannot reach is ever handed to a kernel.
 *     Calls are synchronous, like isa-l's: they run on the calling thread's
 *     per-thread stream and return once the result is in memory.
 *
 *  2. A batched, asynchronous stripe API for the GPU path proper: many
 *     independent stripes per launch through a device-resident pointer table,
 *     enqueued on a caller-owned stream so an SPDK reactor never blocks (the
 *     raid module keeps one stream per io_channel and completes requests from
 *     a poller on draid_ec_stream_query()).
 *
 * No torch or HIP types appear in these signatures: streams are `void *`
 * (a hipStream_t underneath), memory is plain pointers and sizes.
 *
 * Return convention: 0 = success; 1 = the arguments are rejected with
 * isa-l's semantics (nothing written); negative = HIP runtime failure
 * (draid_ec_last_error() has the message).
 */
#ifndef DRAID_EC_H
#define DRAID_EC_H

#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DRAID_EC_ABI_VERSION 1
#define DRAID_EC_FAIL_NONE 0xFFu /* unused slot of a per-stripe failure pair */

/* ------------------------------------------------------------------------
 * 1. isa-l-shaped synchronous entry points
 * ---------------------------------------------------------------------- */

/* XOR parity: array[vects-1] = XOR of array[0 .. vects-2], len bytes each.
 * Replaces isa-l xor_gen() (isa-l/include/raid.h, v2.30) as called by
 *   raid5_xor_buf        module/bdev/raid/raid5.c:188-201   (vects = 3, in place)
 *   raid5_xor_gen        module/bdev/raid/raid5_simple.c:131-135,176 (vects = k+1)
 *   xor_buf              examples/bdev/gf_vect_mul/gf_vect_mul.c:40-49
 * vects < 3 or len < 0 -> 1.  The destination may alias a source. */
int draid_xor_gen(int vects, int len, void **array);

/* P+Q parity: k = vects-2 sources; array[k] = P = XOR_j D_j,
 * array[k+1] = Q = XOR_j 2^j D_j over GF(2^8)/0x11D.
 * Replaces isa-l pq_gen() as called at gf_vect_mul.c:101,152,199,253,294.
 * vects < 4, len < 0 or len % 32 != 0 -> 1 (isa-l's SIMD contract). */
int draid_pq_gen(int vects, int len, void **array);

/* 0 iff XOR over all vects pointers is zero (isa-l xor_check()). */
int draid_xor_check(int vects, int len, void **array);

/* 0 iff array[k], array[k+1] hold the P, Q of array[0..k-1]
 * (isa-l pq_check(); used at gf_vect_mul.c:178-179). */
int draid_pq_check(int vects, int len, void **array);

/* draid_pq_check() for callers that cannot allocate.  No counterpart in the
 * reference: it exists for callers that may not call hipMalloc -- code under HIP
 * graph capture, tight scrub loops, harnesses that forbid allocation.
 * draid_pq_check() keeps its mismatch flag and (above 34 vectors) its pointer
 * table in device memory it allocates on first use; this variant keeps both in
 * a 4 KiB static device array inside the library (one copy per GPU, held until
 * the process ends) and allocates, frees and copies nothing.
 * Same arguments and argument errors as draid_pq_check(), except:
 *   array  every vector must be memory the GPU can use in place -- device memory
 *          of the current GPU, or pinned / registered host memory (host or device
 *          address) -- because a pageable vector would need the staging arena
 *          draid_pq_check() allocates: such a vector returns 1 and nothing is
 *          launched (it is never handed to a kernel);
 *   vects  at most DRAID_PQ_CHECK_STATIC_MAX_VECTS (the static table), else 1;
 *   result word of the same kinds of memory; receives 0 if P and Q match, 1 if not;
 *   stream the work is enqueued here and the call returns without waiting:
 *          *result is valid once the stream has finished.
 * Every call on a GPU shares that GPU's array: calls that overlap in time on
 * one GPU (other streams or threads) race and may report the wrong verdict.
 * Under stream capture: a thread's first call on a GPU looks the array's address
 * up (hipGetSymbolAddress) and its first call with a given buffer asks the
 * runtime what that memory is; make one call outside the captured region first,
 * after which a call with the same buffers only launches kernels. */
#define DRAID_PQ_CHECK_STATIC_MAX_VECTS 257 /* k = 255 data strips + P + Q */
int draid_pq_check_static(int vects, int len, void **array, uint32_t *result, void *stream);

/* GF(2^8) scalar helpers (host-side; isa-l erasure_code.h gf_mul / gf_inv,
 * gf_vect_mul.h gf_vect_mul_init -- gf_vect_mul.c:60-66,313-322). */
unsigned char draid_gf_mul(unsigned char a, unsigned char b);
unsigned char draid_gf_inv(unsigned char a);
void draid_gf_vect_mul_init(unsigned char c, unsigned char *tbl /* [32] */);

/* dest = c * src over len bytes, with tbl from draid_gf_vect_mul_init(c).
 * Replaces isa-l gf_vect_mul() (gf_vect_mul.c:108,158,221,256,267,310-326).
 * len < 0 or len % 32 != 0 -> 1. src and dest may alias. */
int draid_gf_vect_mul(int len, unsigned char *tbl, void *src, void *dest);

/* Composite recovery of one stripe (the compositions of
 * raid5.c:544-594 and gf_vect_mul.c:242-347 as one kernel):
 * array = k data pointers, then P (array[k]) and, for m == 2, Q (array[k+1]).
 * The nfail (<= m) strips listed in fail[] are regenerated in place.
 * k + m <= 255 (every reconstruct call: strip indices are bytes, 0xFF = none).
 * Invalid or unrecoverable failure sets -> 1. */
int draid_recover(int k, int m, int len, void **array, int nfail, const int *fail);

/* ------------------------------------------------------------------------
 * 2. Batched asynchronous stripe API
 * ---------------------------------------------------------------------- */

typedef struct draid_ec_stripe_batch {
    uint32_t k;            /* data strips per stripe, 1 .. 255 (reconstruct:
                            * k + m <= 255)                                    */
    uint32_t m;            /* parity strips: 1 = RAID5 (P), 2 = RAID6 (P, Q)  */
    uint64_t strip_len;    /* bytes per strip (same for every stripe)         */
    uint32_t nstripes;     /* stripes in this batch                           */
    uint32_t flags;        /* reserved, must be 0                             */
    /* DEVICE-resident table of nstripes * (k + m) device pointers, stripe-major:
     * strips[s*(k+m) + j] is data strip j (isa-l array order) for j < k,
     * P for j == k, Q for j == k+1.  16-byte aligned strips run the vector
     * path; any alignment is correct. */
    void *const *strips;
} draid_ec_stripe_batch;

/* Full-stripe encode of every stripe in the batch (P for m == 1, P and Q for
 * m == 2).  Enqueued on `stream`; returns without waiting.  One call covers
 * strip_len <= 0x7fff0000 and ceil(strip_len / 1 KiB) * nstripes < 2^31 (else 1,
 * as for every batched / strided / host call). */
int draid_ec_encode(const draid_ec_stripe_batch *batch, void *stream);

/* Degraded-read / rebuild reconstruct.  `fail` is a DEVICE array of
 * nstripes * 2 bytes: the (up to two) failed strip indices of each stripe
 * (0..k-1 data, k = P, k+1 = Q; DRAID_EC_FAIL_NONE = unused).  The listed
 * strips are regenerated into their table pointers.  A stripe with more
 * failures than m, or with an entry in [k+m, 0xFF), is left untouched -- also its
 * other, valid entry: a pair with a wild index is not trusted at all. */
int draid_ec_reconstruct(const draid_ec_stripe_batch *batch, const uint8_t *fail,
                         void *stream);

/* draid_ec_reconstruct that also reports what it could not rebuild (the
 * reference fails a stripe whose arithmetic fails, raid5_simple.c:177-180,
 * 321-325): *unrecoverable, a device-accessible uint32_t (device memory, or the
 * device address of pinned host memory), is incremented once for every stripe
 * whose pair lists more failures than m or an index in [k+m, 0xFF).  Those
 * stripes are left untouched.  The counter is only added to: clear it before
 * the call (or accumulate over several); read it once `stream` has finished. */
int draid_ec_reconstruct_status(const draid_ec_stripe_batch *batch, const uint8_t *fail,
                                uint32_t *unrecoverable, void *stream);

/* Regular layout, no pointer table: strip j of stripe s at
 * base + s*stripe_stride + j*strip_stride (a stripe cache allocated as one
 * array, raid5.c:1331-1353 with the n chunk buffers of a stripe adjacent). */
typedef struct draid_ec_strided_stripes {
    uint32_t k, m;           /* as draid_ec_stripe_batch                          */
    uint64_t strip_len;      /* bytes per strip                                   */
    uint32_t nstripes;
    uint32_t flags;          /* 0, or DRAID_EC_HOST_STAGED for the 2c host calls  */
    void *base;
    uint64_t strip_stride;   /* >= strip_len                                      */
    uint64_t stripe_stride;
} draid_ec_strided_stripes;

/* As draid_ec_encode / draid_ec_reconstruct over a strided layout.  `base` is
 * device memory, or pinned / registered host memory (read in place over PCIe).
 * `fail` is a DEVICE array as above. */
int draid_ec_encode_strided(const draid_ec_strided_stripes *s, void *stream);
int draid_ec_reconstruct_strided(const draid_ec_strided_stripes *s, const uint8_t *fail,
                                 void *stream);
int draid_ec_reconstruct_strided_status(const draid_ec_strided_stripes *s, const uint8_t *fail,
                                        uint32_t *unrecoverable, void *stream);

/* ------------------------------------------------------------------------
 * 2b. Scatter-gather stripes through a per-channel context
 *
 * The reference walks each chunk's iovec list and calls isa-l once per
 * contiguous run (raid5_xor_iovs, raid5.c:221-283; raid5_xor_stripe,
 * raid5_simple.c:141-203).  A context runs the same walk on the host but queues
 * each run as a gather descriptor; draid_ec_ctx_flush() uploads the queued
 * descriptors in ~1 MiB pieces (copy stream) and launches one kernel per piece
 * of each (op, k, m) group, so uploads overlap earlier kernels.
 * A context owns a stream and is used by one thread (one per SPDK io_channel).
 * ---------------------------------------------------------------------- */

typedef struct draid_ec_ctx draid_ec_ctx;

int draid_ec_ctx_create(draid_ec_ctx **ctx);       /* on the current device */
int draid_ec_ctx_destroy(draid_ec_ctx *ctx);
void *draid_ec_ctx_stream(draid_ec_ctx *ctx);

/* Queue one stripe's encode.  Strip j (k data, then P, then Q) is `len` bytes
 * starting `offset[j]` bytes into iovs[j][0 .. iovcnt[j]) (offset may be NULL).
 * Every iov_base is a device-usable address (device memory, or the device
 * address of pinned / registered host memory) -- unless the context resolves
 * host pointers itself, see draid_ec_ctx_set_host_pointers.
 * The queueing calls (encode_sg, reconstruct_sg, update_sg) normally only write
 * descriptors into pinned memory.  They can wait -- for the descriptor upload of
 * the flush before last, when a group is queued into again while those copies
 * still run -- and they allocate pinned memory when a group outgrows its
 * descriptor storage (it doubles, from 1 MiB).  A call that completes a ~1 MiB
 * piece of descriptors of small segments (under 128 KiB of strips each) also
 * starts that piece's upload, so a flush of many small runs finds most of its
 * descriptors on the device (at most 12 pieces wait like that; the call never
 * waits for a ring slot; DRAID_EC_CTX_STAGE_AHEAD=0 turns it off). */
int draid_ec_ctx_encode_sg(draid_ec_ctx *ctx, uint32_t k, uint32_t m,
                           const struct iovec *const *iovs, const int *iovcnt,
                           const size_t *offset, size_t len);

/* Queue one stripe's reconstruct of the nfail (<= m) strips listed in fail[]. */
int draid_ec_ctx_reconstruct_sg(draid_ec_ctx *ctx, uint32_t k, uint32_t m,
                                const struct iovec *const *iovs, const int *iovcnt,
                                const size_t *offset, size_t len, int nfail, const int *fail);

/* Queue a read-modify-write parity update (raid5_stripe_write_preread_complete_rmw,
 * raid5.c:705-741, extended to Q): nd touched data chunks with distinct data
 * indices data_idx[i] < k, each with iovec lists of its old and new contents;
 * par_iovs[0] is P and (m == 2) par_iovs[1] is Q, updated in place:
 *   P ^= XOR_i (old_i ^ new_i),  Q ^= XOR_i 2^{data_idx[i]} (old_i ^ new_i).
 * Every list covers `len` bytes from its start. */
int draid_ec_ctx_update_sg(draid_ec_ctx *ctx, uint32_t k, uint32_t m, uint32_t nd,
                           const int *data_idx, const struct iovec *const *old_iovs,
                           const int *old_cnt, const struct iovec *const *new_iovs,
                           const int *new_cnt, const struct iovec *const *par_iovs,
                           const int *par_cnt, size_t len);

/* Launch everything queued.  Non-blocking, except that each ~1 MiB piece of
 * descriptors takes one of 16 ring slots and waits for that slot's previous
 * kernel when all 16 are in flight (and allocates the slot's buffers on first
 * use or growth).  A small launch (about 400 stripes of 64 KiB strips, 100 cut
 * into 4 KiB runs, 120 of 256 KiB strips) uploads nothing: its kernel reads the
 * descriptors from the slot's pinned host memory, which takes 20 us off the
 * flush and as much off the time to completion (larger launches upload; the
 * limit can be set with DRAID_EC_CTX_INPLACE_LIMIT, 0 = always upload).  The
 * context's stream is non-blocking: it does not wait for work on other
 * streams, so every queued buffer must hold its data when flush is called.
 * Order: segments queued with the same (op, k, m) form a group and carry no
 * order among themselves (the flush may run them in address order).  Groups
 * run one after the other on one stream, in the order in which their FIRST
 * segment of this batch was queued -- which says nothing about two segments of
 * different groups once several requests share a batch (request A's encode
 * opens the encode group, request B then queues a rebuild and an encode that
 * reads the rebuilt strips: B's encode would run with A's, ahead of B's
 * rebuild).  Work that reads what earlier work of the same request writes
 * therefore puts a draid_ec_ctx_fence() between the two; any dependency on
 * work of an EARLIER flush is already ordered by the stream.
 * On failure (a piece's descriptor memory, the work-item limit, a launch
 * error) the pieces launched so far keep running, every segment that did not
 * launch stays queued -- draid_ec_ctx_queued() counts exactly those -- and the
 * error is returned: flush again, or fail the requests still queued.
 * draid_ec_ctx_query: 0 idle, 1 running, < 0 error. */
int draid_ec_ctx_flush(draid_ec_ctx *ctx);
/* draid_ec_ctx_flush, then a ticket for everything launched so far:
 * draid_ec_ctx_ticket_query(ticket) is 0 once all of it has finished, 1 while it
 * runs -- whatever was flushed later may still be running.  This is what a
 * poller completes requests on (draid_ec_ctx_query only turns 0 when the whole
 * stream is idle, which a busy channel never is).  At most 64 tickets may be
 * outstanding; the 65th flush_ticket waits for the oldest. */
int draid_ec_ctx_flush_ticket(draid_ec_ctx *ctx, uint64_t *ticket);
int draid_ec_ctx_ticket_query(draid_ec_ctx *ctx, uint64_t ticket);
/* on != 0: every iov_base handed to this context is the CALLER'S address -- a
 * host pointer of pinned / registered memory (an SPDK buffer) or a device
 * pointer -- and is resolved to its device address while the descriptors are
 * written (draid_ec_device_pointer's cached lookup, one per iovec).  A stripe
 * with an iovec the GPU cannot reach is rejected with 1 and queues nothing.
 * The context then also knows which segments lie in host memory, and runs
 * batches of those in kernels that loop over the work items with one workgroup
 * per CU (a PCIe-bound launch of a few dozen stripes is 11-13% faster that way
 * than with a workgroup per item, a large one 3%).  Off by default. */
int draid_ec_ctx_set_host_pointers(draid_ec_ctx *ctx, int on);
int draid_ec_ctx_query(draid_ec_ctx *ctx);
int draid_ec_ctx_synchronize(draid_ec_ctx *ctx);
uint64_t draid_ec_ctx_queued(draid_ec_ctx *ctx);   /* segments queued since last flush */
/* Drops every queued segment (after a failed flush whose requests the caller
 * fails instead of retrying).  Work already launched is not affected. */
int draid_ec_ctx_discard_queued(draid_ec_ctx *ctx);
/* All-or-nothing queueing of a request that takes several queueing calls (a
 * degraded write: rebuild, then re-encode; an RMW over several ranges).
 * draid_ec_ctx_mark remembers what is queued now; draid_ec_ctx_rollback drops
 * every segment queued since, in every group, and leaves the earlier ones as
 * they were -- so a request whose n-th call fails (an unreachable iovec) leaves
 * nothing behind that a later flush would run on buffers it no longer owns.
 * One mark at a time; rollback returns 1 without a mark, or when something was
 * launched since the mark (a flush, or autoflush: those segments are running). */
int draid_ec_ctx_mark(draid_ec_ctx *ctx);
int draid_ec_ctx_rollback(draid_ec_ctx *ctx);
/* Segments queued from now on (until the next draid_ec_ctx_mark, rollback or
 * flush) run after every segment queued in this batch before their request's
 * fence: a request that rebuilds lost strips into its buffers and then encodes
 * over them calls mark, queues the rebuild, calls fence, queues the encode.
 * Requests stay batched: all work in front of a fence shares launches per
 * (op, k, m) as before, all work behind one fence likewise; the flush runs the
 * first kind, then the second (then work behind a second fence, ...).
 * Autoflush never launches work behind a fence early. */
int draid_ec_ctx_fence(draid_ec_ctx *ctx);

/* Launch an (op, k, m) group as soon as it holds `segments` queued segments,
 * from inside the queueing call (0 = only at draid_ec_ctx_flush, the default).
 * For callers whose buffers hold their data when a stripe is queued (an SPDK
 * module queues a stripe once its data or prereads are in): the GPU then runs
 * while the host walks the rest of the batch.  A queueing call that launches
 * returns the launch's error, if any.  Such a launch carries only its own
 * group: it may run before segments queued earlier in other groups, so work
 * on the same buffers in different groups needs a flush in between (as it
 * does anyway when a later group must run first). */
int draid_ec_ctx_set_autoflush(draid_ec_ctx *ctx, uint64_t segments);

/* ------------------------------------------------------------------------
 * 2c. Host-resident stripes (PCIe-inclusive path)
 *
 * SPDK's stripe buffers are host hugepages.  When the whole range is pinned or
 * registered (draid_ec_host_register) the kernel reads the strips it needs in
 * place over PCIe and writes P/Q (or the rebuilt strips) straight back: one
 * launch, no staging -- a reconstruct moves only the surviving strips.  With
 * flags = DRAID_EC_HOST_STAGED (or host memory the runtime knows that is not one
 * mapping) the calls copy the input strips in (hipMemcpy2DAsync per strip
 * index over a chunk of stripes), run the kernel in HBM and copy the results
 * back, pipelined over three streams; chunk_stripes = stripes per pipeline
 * stage (0 = 64).  Pageable memory is bounced through two pinned buffers by the
 * calling thread itself (the runtime's strided copies of pageable memory run at
 * a quarter of that): only the strips the kernel reads go in, only the strips
 * it wrote come out.  Synchronous.
 * ---------------------------------------------------------------------- */

#define DRAID_EC_HOST_STAGED 1u

typedef draid_ec_strided_stripes draid_ec_host_stripes;   /* base is HOST memory */

/* Data strips in, P (and Q) out. */
int draid_ec_host_encode(const draid_ec_host_stripes *h, uint32_t chunk_stripes);

/* All k+m strips in, the failed strips (HOST fail[nstripes][2], as
 * draid_ec_reconstruct) out.  The table is checked before anything runs: a
 * stripe with more failures than m, or an index in [k+m, 0xFF), -> 1 and nothing
 * is rebuilt. */
int draid_ec_host_reconstruct(const draid_ec_host_stripes *h, const uint8_t *fail,
                              uint32_t chunk_stripes);

/* ------------------------------------------------------------------------
 * 2d. Several GPUs from one process
 *
 * Stripes are independent (the reference only serialises requests to the same
 * stripe, raid5.c:1047-1054), so the GPUs of a node share them by index with no
 * data exchanged between devices.  The benchmark spreads them with one process
 * per GPU; an SPDK target is one process, so a draid_ec_mgpu drives the same
 * split from one thread: a stream per device slot, each call enqueues every
 * slot's shard on its own device and returns without waiting, all devices run
 * concurrently.  Device slot d's shard (pointer table, strips, fail table,
 * counter) lives in device d's memory.
 * ---------------------------------------------------------------------- */

#define DRAID_EC_SHARD_RANGE 0 /* device d owns stripes [n*d/G, n*(d+1)/G)           */
#define DRAID_EC_SHARD_MOD 1   /* device d owns stripes s with s mod G == d (a bdev's
                                * stripes, in arrival order)                          */

/* Which device slot owns stripe `stripe` of `nstripes` over `ndevices`; -1 when
 * out of range.  Pure arithmetic (usable without a GPU). */
int draid_ec_shard_of(uint64_t stripe, uint64_t nstripes, int ndevices, int policy);
/* The contiguous range of slot `device`, and how many stripes a slot owns. */
int draid_ec_shard_range(uint64_t nstripes, int ndevices, int device, uint64_t *lo, uint64_t *hi);
uint64_t draid_ec_shard_count(uint64_t nstripes, int ndevices, int device, int policy);

typedef struct draid_ec_mgpu draid_ec_mgpu;

/* ndevices <= 0: one slot per visible GPU.  devices (may be NULL: 0, 1, ...)
 * lists the GPU of each slot; a GPU may appear more than once. */
int draid_ec_mgpu_create(draid_ec_mgpu **mg, int ndevices, const int *devices);
int draid_ec_mgpu_destroy(draid_ec_mgpu *mg);
int draid_ec_mgpu_devices(const draid_ec_mgpu *mg);
int draid_ec_mgpu_device(const draid_ec_mgpu *mg, int slot);   /* the slot's GPU */
void *draid_ec_mgpu_stream(draid_ec_mgpu *mg, int slot);

/* One batch / descriptor per slot (nstripes == 0: nothing for that device);
 * fail[d] and unrecoverable[d] as in draid_ec_reconstruct_status, in slot d's
 * memory (unrecoverable may be NULL altogether). */
int draid_ec_mgpu_encode(draid_ec_mgpu *mg, const draid_ec_stripe_batch *batches);
int draid_ec_mgpu_reconstruct(draid_ec_mgpu *mg, const draid_ec_stripe_batch *batches,
                              const uint8_t *const *fail, uint32_t *const *unrecoverable);
int draid_ec_mgpu_encode_strided(draid_ec_mgpu *mg, const draid_ec_strided_stripes *shards);
int draid_ec_mgpu_reconstruct_strided(draid_ec_mgpu *mg, const draid_ec_strided_stripes *shards,
                                      const uint8_t *const *fail,
                                      uint32_t *const *unrecoverable);
/* 0 = every device idle, 1 = some still running, < 0 = error. */
int draid_ec_mgpu_query(draid_ec_mgpu *mg);
int draid_ec_mgpu_synchronize(draid_ec_mgpu *mg);

/* ------------------------------------------------------------------------
 * 3. Runtime helpers (device, streams, memory)
 * ---------------------------------------------------------------------- */

int draid_ec_abi_version(void);
const char *draid_ec_last_error(void);
int draid_ec_set_device(int device);
int draid_ec_device_current(int *device);
int draid_ec_device_count(int *count);

int draid_ec_stream_create(void **stream);
int draid_ec_stream_destroy(void *stream);
/* 0 = all enqueued work done, 1 = still running, < 0 = error.  Non-blocking:
 * the SPDK poller of a raid io_channel calls this. */
int draid_ec_stream_query(void *stream);
int draid_ec_stream_synchronize(void *stream);

int draid_ec_device_alloc(void **ptr, size_t bytes);
int draid_ec_device_free(void *ptr);
/* Host memory the GPU can reach, from the runtime's own pinned allocator (mapped
 * and portable: every GPU of the process sees it at the same address).  For an
 * environment's DMA allocator (spdk_dma_malloc) to sit on when the driver
 * refuses to register memory it did not allocate; 4 KiB aligned. */
int draid_ec_host_alloc(void **ptr, size_t bytes);
int draid_ec_host_free(void *ptr);
/* Pin + map an existing host range (e.g. spdk_dma_malloc hugepages,
 * raid5.c:1340-1342) so kernels and DMA can reach it. */
int draid_ec_host_register(void *ptr, size_t bytes);
int draid_ec_host_unregister(void *ptr);
/* The device address of a host byte inside a registered or pinned range: the
 * pointer to hand to the section 1 / 2 / 2b calls (a registration may map host
 * memory at a different device address, hipHostGetDevicePointer).  The section
 * 2c calls take host addresses and translate themselves.  Returns 0, or 1 with
 * *dev_ptr = NULL when ptr is not in a mapped host range. */
int draid_ec_host_device_pointer(const void *ptr, void **dev_ptr);
/* The address a kernel may use for the caller's [ptr, ptr + len): device memory
 * -> itself, pinned / registered host memory -> its device address.  Returns 0,
 * or 1 with *dev_ptr = NULL when the range is neither (pageable host memory).
 * This is the lookup every pointer-taking entry point of sections 1 and 2b
 * does; results are cached per thread by allocation, so a hit costs a few
 * compares.  The cache is emptied by draid_ec_device_free, draid_ec_host_unregister
 * and draid_ec_pointer_cache_flush -- call the last one after freeing or
 * unregistering memory behind the library's back if its addresses may be reused. */
int draid_ec_device_pointer(const void *ptr, size_t len, void **dev_ptr);
void draid_ec_pointer_cache_flush(void);
/* kind: 0 host->device, 1 device->host, 2 device->device. */
int draid_ec_memcpy_async(void *dst, const void *src, size_t bytes, int kind, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* DRAID_EC_H */
