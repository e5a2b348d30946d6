/*
 * draid_raid.h -- host-side RAID5/RAID6 stripe layer over the draid_ec C ABI.
 *
 * The SPDK-independent part of a raid level module (module/bdev/raid/raid5.c,
 * raid5_simple.c): array geometry, parity placement, mapping a stripe request
 * onto chunks, slicing the parent I/O's iovecs per chunk, and the full-stripe
 * write / degraded read drivers that hand the parity arithmetic to the GPU
 * through a draid_ec_ctx.  A real SPDK module (draid-spdk_amd/spdk/raid_gpu.c) wraps these
 * calls with spdk_bdev_io / io_channel / poller glue; everything here is plain C
 * on host memory that the GPU can reach (registered or device memory).
 */
#ifndef DRAID_RAID_H
#define DRAID_RAID_H

#include <stdbool.h>
#include <stdint.h>
#include <sys/uio.h>

#include "draid_ec.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DRAID_RAID_MAX_BASE 32
#define DRAID_RAID_MAX_IOV 64

/* struct raid_bdev / raid5_info fields the data path needs (bdev_raid.h:96-160,
 * raid5.c:113-135). */
struct draid_raid {
    uint8_t level;            /* 5 or 6 */
    uint8_t num_base_bdevs;   /* n */
    uint8_t max_degraded;     /* parity strips per stripe: 1 (RAID5), 2 (RAID6) */
    uint32_t blocklen;        /* bytes per block */
    uint32_t strip_size;      /* blocks per strip (power of two) */
    uint32_t strip_size_shift;
    uint64_t stripe_blocks;   /* data blocks per stripe */
    uint64_t total_stripes;
    uint64_t blockcnt;        /* exported capacity in blocks */
    uint64_t optimal_io_boundary;
    uint32_t degraded_mask;   /* bit d set: base bdev d is degraded (bdev_raid.h:91-92) */
};

/* raid5_start geometry (raid5.c:1399-1426), generalised to m parity strips.
 * Returns 0 or -EINVAL (n too small for the level, strip not a power of two). */
int draid_raid_start(struct draid_raid *r, int level, int num_base_bdevs, uint32_t blocklen,
                     uint32_t strip_size_blocks, uint64_t min_base_blockcnt);

/* Parity placement.  RAID5: p = (n-1) - s mod n (raid5.c:1006-1007).  RAID6
 * (undefined by the reference): p as RAID5, q = (p+1) mod n.
 * Data indices fill the remaining disks in ascending order. */
void draid_raid_parity_chunks(const struct draid_raid *r, uint64_t stripe, int *p, int *q);
int draid_raid_data_disk(const struct draid_raid *r, uint64_t stripe, int data_idx);
int draid_raid_disk_data_index(const struct draid_raid *r, uint64_t stripe, int disk); /* -1 for P/Q */

/* Per-chunk request of a stripe request (struct chunk, raid5.c:52-88). */
struct draid_chunk_req {
    uint64_t req_offset;      /* blocks from the chunk start */
    uint64_t req_blocks;
};

/* raid5_handle_stripe (raid5.c:962-1055): maps [stripe_offset, +blocks) of one
 * stripe onto its chunks.  chunk[] is indexed by base bdev. */
struct draid_stripe_req {
    uint64_t stripe_index;
    int p_disk, q_disk;       /* q_disk = -1 for RAID5 */
    int first_data, last_data;/* data indices touched */
    bool full_stripe;
    struct draid_chunk_req chunk[DRAID_RAID_MAX_BASE];
};

int draid_raid_map_request(const struct draid_raid *r, uint64_t offset_blocks,
                           uint64_t num_blocks, struct draid_stripe_req *out);

/* raid5_chunk_map_iov (raid5.c:358-426): the iovecs covering [offset, offset+len)
 * of a parent iovec list.  Returns the iovec count, or -EINVAL / -ENOSPC. */
int draid_raid_map_iov(struct iovec *out, int out_max, const struct iovec *iov, int iovcnt,
                       uint64_t offset, uint64_t len);

/* One base-bdev I/O the module must issue (spdk_bdev_{read,write}v_blocks,
 * raid5.c:617-662): base LBA = stripe * strip_size + offset (raid5.c:648). */
struct draid_base_io {
    int disk;
    uint64_t offset_blocks;
    uint64_t num_blocks;
    int iovcnt;
    struct iovec iov[DRAID_RAID_MAX_IOV];
};

/* Full-stripe write (raid5_stripe_write_preread_complete / raid5_xor_stripe):
 * slices the parent iovecs into the k data chunks, queues the parity encode into
 * parity_buf[0] (P) and parity_buf[1] (Q, RAID6) on ctx, and fills writes[0..n)
 * with every base write to issue once the ctx has completed (after
 * draid_ec_ctx_flush + query/synchronize).  Non-full-stripe requests are
 * rejected with -EINVAL, as raid5_simple does (raid5_simple.c:381-395). */
int draid_raid_stripe_write(const struct draid_raid *r, draid_ec_ctx *ctx,
                            const struct draid_stripe_req *req, const struct iovec *iov,
                            int iovcnt, void *const parity_buf[2],
                            struct draid_base_io *writes, int *nwrites);

/* Partial-stripe writes, two phases as in raid5_stripe_write (raid5.c:779-867).
 * The vote: with the parity range = the touched chunk's range (one chunk) or the
 * whole strip (several), every data chunk with fewer requested blocks than the
 * parity range votes for read-modify-write, every touched chunk against. */
enum draid_write_mode { DRAID_WRITE_RMW = 1, DRAID_WRITE_RCW = 2 };

struct draid_write_plan {
    int mode;
    uint64_t p_offset, p_blocks;                         /* parity range within the strip */
    struct draid_chunk_req preread[DRAID_RAID_MAX_BASE]; /* per disk; blocks == 0: none */
};

/* Phase 1: vote and list the prereads.  preread_buf[disk] are strip-sized
 * buffers; a preread of [off, off+blocks) lands at the same offset in them.
 * For P and Q they also receive the new parity range.  Full-stripe requests
 * need no plan (draid_raid_stripe_write). */
int draid_raid_plan_write(const struct draid_raid *r, const struct draid_stripe_req *req,
                          struct draid_write_plan *plan, void *const *preread_buf,
                          struct draid_base_io *reads, int *nreads);

/* Phase 2, once the prereads are in (raid5_stripe_write_preread_complete[_rmw],
 * raid5.c:705-777): queue the parity work on ctx -- RMW: P ^= old ^ new (and
 * Q ^= 2^i (old ^ new)) per touched chunk range; RCW: P (and Q) re-encoded over
 * the parity range from preread and new data -- into preread_buf[p] (and [q]),
 * and fill writes[] with the new data ranges and the parity range. */
int draid_raid_stripe_write_partial(const struct draid_raid *r, draid_ec_ctx *ctx,
                                    const struct draid_stripe_req *req,
                                    const struct draid_write_plan *plan, const struct iovec *iov,
                                    int iovcnt, void *const *preread_buf,
                                    struct draid_base_io *writes, int *nwrites);

/* Degraded read of a whole stripe (raid5_stripe_read + the reconstruct of
 * raid5_complete_reconstructed_stripe_request, raid5.c:544-594,869-946,
 * generalised to two failures): `chunk_buf[disk]` are the stripe's per-disk
 * buffers (strip bytes each) that the caller fills with the surviving base
 * reads listed in reads[]; the reconstruct of the degraded chunks into
 * chunk_buf is queued on ctx; afterwards the caller copies data chunks out (or
 * passes chunk_buf of data disks = the user's buffers).  -EIO if more disks are
 * degraded than the level tolerates. */
int draid_raid_stripe_degraded_read(const struct draid_raid *r, draid_ec_ctx *ctx,
                                    uint64_t stripe, void *const *chunk_buf,
                                    struct draid_base_io *reads, int *nreads);
/* Two-phase form for base reads that complete asynchronously (a real module):
 * draid_raid_stripe_degraded_read with ctx = NULL lists the reads only; once they
 * are in, draid_raid_stripe_degraded_rebuild queues the reconstruct on ctx.  (With
 * a ctx the one call does both: right when the reads are ordered before the
 * flush, e.g. copies on the ctx's stream.)  Work queued afterwards that reads the
 * rebuilt strips -- the re-encode of a degraded partial write -- goes behind a
 * draid_ec_ctx_fence(ctx): several requests may share the batch, and without
 * the fence that encode would launch with the encodes queued before this
 * rebuild. */
int draid_raid_stripe_degraded_rebuild(const struct draid_raid *r, draid_ec_ctx *ctx,
                                       uint64_t stripe, void *const *chunk_buf);

/* Ranged read of one stripe request (raid5_stripe_read, raid5.c:869-946, and
 * raid5_complete_reconstructed_stripe_request, raid5.c:544-594, generalised to
 * RAID6).  Healthy: one base read per requested data chunk straight into the
 * parent iovecs.  With requested data chunks on degraded disks, R = the union of
 * their requested ranges is rebuilt, as the reference rebuilds d_chunk's range:
 * every other needed strip is read over R (Q only when two strips are lost) and
 * the reconstruct of R is queued on ctx.  Unlike the reference, which prereads
 * the union of a requested chunk's range and R into a stripe buffer and then
 * memcpys the requested part back (raid5.c:910-917,572-590), the parts of R a
 * request covers are read into the parent iovecs, the rest into chunk_buf, and
 * the kernel gathers R from both: no copy pass.  Lost requested ranges are
 * rebuilt straight into the parent iovecs.  chunk_buf[disk] are strip-sized
 * scratch buffers; reads[] must hold 3 * n entries.  With a ctx the
 * reconstruct is queued at once (the reads must then reach memory before the
 * flush runs); see the two-phase form below.  -EIO if a rebuild is needed and more
 * disks are degraded than the level tolerates. */
int draid_raid_stripe_read(const struct draid_raid *r, draid_ec_ctx *ctx,
                           const struct draid_stripe_req *req, const struct iovec *iov,
                           int iovcnt, void *const *chunk_buf, struct draid_base_io *reads,
                           int *nreads);
/* Two-phase form (as for the whole-stripe read): draid_raid_stripe_read with
 * ctx = NULL plans the reads; after they complete, draid_raid_stripe_read_rebuild
 * with the same arguments queues the reconstruct of the lost requested range. */
int draid_raid_stripe_read_rebuild(const struct draid_raid *r, draid_ec_ctx *ctx,
                                   const struct draid_stripe_req *req, const struct iovec *iov,
                                   int iovcnt, void *const *chunk_buf);

/* Disk-level failures to stripe-level kernel input, for batched degraded reads
 * and for rebuilding a failed disk (the rotation of raid5.c:1006-1007 gives a
 * disk a different role -- data index, P or Q -- in every stripe).
 *
 * draid_raid_fail_table: fail[2*i], fail[2*i+1] = the isa-l indices (data
 * 0..k-1, P = k, Q = k+1) of stripe first+i's strips on the disks in
 * r->degraded_mask, DRAID_EC_FAIL_NONE-padded -- the `fail` array of
 * draid_ec_reconstruct.  -EIO if more disks are degraded than the level
 * tolerates.
 *
 * draid_raid_strip_table: the pointer table of draid_ec_stripe_batch for stripes
 * [first, first+count) when base disk d's blocks start at disk_base[d] (disks in
 * HBM, or staging regions mirroring them): strip j of stripe s (isa-l order) at
 * disk_base[disk(s, j)] + (s - disk_first) * strip bytes, where disk_first is the
 * stripe at each disk_base.  Host memory; copy it to the device for the call. */
int draid_raid_fail_table(const struct draid_raid *r, uint64_t first, uint32_t count,
                          uint8_t *fail);
int draid_raid_strip_table(const struct draid_raid *r, uint64_t first, uint32_t count,
                           void *const *disk_base, uint64_t disk_first, void **table);

/* Stripe assembly of raid5_simple (raid5_submit_write_request,
 * raid5_simple.c:347-423): with the bdev layer splitting writes at strip
 * boundaries, a full-stripe write arrives as k strip-sized child I/Os on a
 * channel; they are gathered per channel (r5ch->current_stripe_request) and the
 * stripe is encoded once the k-th has arrived.  Children may arrive in any order;
 * one stripe is assembled at a time. */
struct draid_stripe_asm {
    uint64_t stripe_index;
    int active;                          /* a stripe is being assembled */
    int received;                        /* data chunks present */
    uint32_t have;                       /* bit d: data chunk d present */
    int iovcnt[DRAID_RAID_MAX_BASE];
    struct iovec iov[DRAID_RAID_MAX_BASE][DRAID_RAID_MAX_IOV];
};

void draid_raid_asm_init(struct draid_stripe_asm *a);
/* Adds one child write [offset_blocks, +num_blocks).  Returns 1 when the stripe's
 * k data chunks are all present (fetch the stripe's parent iovecs with
 * draid_raid_asm_iov, then draid_raid_stripe_write; the assembler is free
 * again), 0 while chunks are missing, -EINVAL for a child that is not exactly
 * one strip (raid5_simple rejects non-full-stripe writes, raid5_simple.c:381-395),
 * repeats a chunk or belongs to another stripe than the one being assembled. */
int draid_raid_asm_add(const struct draid_raid *r, struct draid_stripe_asm *a,
                       uint64_t offset_blocks, uint64_t num_blocks, const struct iovec *iov,
                       int iovcnt);
/* The assembled stripe's iovecs in data order (one parent list for the whole
 * stripe), into out[0 .. out_max); returns the count or -ENOSPC. */
int draid_raid_asm_iov(const struct draid_raid *r, const struct draid_stripe_asm *a,
                       struct iovec *out, int out_max);

/* ------------------------------------------------------------------------
 * Stripe cache and per-stripe request queue (raid5_get_stripe /
 * raid5_reclaim_stripes, raid5.c:1057-1131; the stripe's request list,
 * raid5.c:1047-1054,485-521).  A fixed pool of nslots entries (RAID_MAX_STRIPES,
 * bdev_raid.h:39, in the reference); entry i owns slot i of a stripe region the
 * caller allocates -- n strips of strip bytes per slot, stripe-major, in HBM or
 * registered host memory -- so a batch of cached stripes is one
 * draid_ec_strided_stripes descriptor.  Thread-safe.
 * ---------------------------------------------------------------------- */

typedef struct draid_stripe_cache draid_stripe_cache;

struct draid_stripe {              /* the public part of a cache entry */
    uint64_t index;                /* stripe index */
    uint32_t slot;                 /* its buffers: slot * draid_stripe_slot_bytes() into the region */
};

/* Bytes from one slot of the stripe region to the next (the stripe stride of the
 * draid_ec_strided_stripes descriptor): n strips, plus 16 KiB when that is a
 * multiple of 512 KiB and the strips are 128 KiB or smaller.  With such a stride
 * the parity strips of every stripe have the same address bit 18, and a batch
 * whose writes all fall into one 256 KiB half of a 512 KiB period runs 14-19%
 * slower on the MI355X (6+2 x 64 KiB strips: 471 us per 5120 stripes against 394
 * with the pad); the pad shifts them from slot to slot. */
uint64_t draid_stripe_slot_bytes(uint32_t n, uint64_t strip_bytes);

struct draid_stripe_waiter {       /* one request on a stripe (embedded by the caller) */
    struct draid_stripe_waiter *next;
    void *arg;
};

int draid_stripe_cache_create(draid_stripe_cache **cache, uint32_t nslots);
void draid_stripe_cache_destroy(draid_stripe_cache *cache);
/* Looks the stripe up or claims an entry for it (reclaiming unreferenced
 * least-recently-used entries when none is free) and takes a reference.  NULL
 * when every entry is referenced: queue the request and retry after a put
 * (raid5.c:1310-1318). */
struct draid_stripe *draid_stripe_get(draid_stripe_cache *cache, uint64_t index);
void draid_stripe_put(draid_stripe_cache *cache, struct draid_stripe *stripe);
/* Appends a request to the stripe's queue: 1 = it is the only one, submit it
 * now; 0 = it waits for the requests ahead of it. */
int draid_stripe_enqueue(draid_stripe_cache *cache, struct draid_stripe *stripe,
                         struct draid_stripe_waiter *w);
/* Removes a finished request; returns the next request to submit, or NULL. */
struct draid_stripe_waiter *draid_stripe_complete(draid_stripe_cache *cache,
                                                  struct draid_stripe *stripe,
                                                  struct draid_stripe_waiter *w);
uint32_t draid_stripe_cache_active(draid_stripe_cache *cache); /* entries mapped to stripes */

#ifdef __cplusplus
}
#endif
#endif /* DRAID_RAID_H */
