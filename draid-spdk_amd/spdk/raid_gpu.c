/*
 * raid_gpu.c -- RAID6 (and RAID5) level module for SPDK's raid bdev whose parity
 * arithmetic runs on an MI355X through libdraid_ec.so.
 *
 * It plugs into the reference's raid framework exactly as its own level modules
 * do: a `struct raid_bdev_module` registered with RAID_MODULE_REGISTER
 * (module/bdev/raid/bdev_raid.h:286-348), called through
 * raid_bdev_submit_request (bdev_raid.c:495-529) and completing parent I/O with
 * raid_bdev_io_complete (bdev_raid.c:325-331).  The reference has no RAID6
 * module: raid6.c is a clone of raid5.c that computes no Q and registers as
 * RAID5 (raid6.c:189,220,1361-1372).  What each part follows:
 *
 *   start / geometry         raid5_start, raid5.c:1399-1489 (draid_raid_start)
 *   request mapping          raid5_submit_rw_request / raid5_handle_stripe,
 *                            raid5.c:1292-1324,962-1055 (draid_raid_map_request)
 *   one request per stripe   the stripe's request queue, raid5.c:1047-1054,485-521
 *                            (draid_stripe_cache)
 *   full-stripe write        raid5_stripe_write_preread_complete, raid5.c:743-777,
 *                            and raid5_xor_stripe, raid5_simple.c:141-203
 *   partial write            raid5_stripe_write (the RMW / RCW vote) and the two
 *                            preread-complete handlers, raid5.c:705-867
 *   read / degraded read     raid5_stripe_read, raid5.c:869-946, and
 *                            raid5_complete_reconstructed_stripe_request, :544-594
 *   base bdev I/O, -ENOMEM   raid5_submit_chunk_request, raid5.c:617-689
 *   per-channel resources    raid5_io_channel_resource_init, raid5.c:1491-1541
 *
 * Where the reference calls isa-l synchronously on the reactor, this module
 * puts a request whose data and prereads are in on its channel's ready list and
 * returns; the channel's poller walks ready requests onto a per-channel
 * draid_ec_ctx, launches them together (at most two launches in flight per GPU,
 * each at most half of the channel's requests: see rg_poll) and finishes the
 * requests of each launch when its ticket completes.  A reactor never waits for
 * the GPU.
 *
 * Degraded operation (bdev_raid.h:91-92,163; the reference only has the flags
 * and a commented-out setter, bdev_raid.c:1157-1170): requests read the
 * per-disk `degraded` flags at submit time.  Up to base_bdevs_max_degraded
 * disks may be degraded: reads rebuild the lost requested ranges, writes keep
 * parity consistent and skip the lost disks.  A base bdev I/O error marks the
 * disk degraded (raid_gpu_set_degraded) and the request is redone against the
 * new state instead of failing, as long as the array can still tolerate it.
 *
 * Buffers: every buffer a kernel touches -- the parent I/O's iovecs and this
 * module's strip buffers from spdk_dma_malloc -- must be memory the GPU can reach
 * (SPDK's DMA memory registered once with draid_ec_host_register, or allocated
 * through draid_ec_host_alloc).  The contexts resolve the host addresses
 * themselves; an I/O whose buffer is not reachable fails with an error log, it
 * is never handed to a kernel.
 */
#include "bdev_raid.h"

#include "spdk/env.h"
#include "spdk/likely.h"
#include "spdk/log.h"
#include "spdk/string.h"
#include "spdk/thread.h"
#include "spdk/util.h"

#include "draid_ec.h"
#include "draid_raid.h"
#include "raid_gpu.h"

/* Stripe requests in flight per channel (raid5_simple.c:14 keeps 128 with one
 * parity buffer each, raid5.c:1508 512 without buffers; here each owns n strip
 * buffers): 128, fewer where that many would pin more than RG_POOL_BYTES per
 * channel, never fewer than 32.  A launch carries up to half of them, and over
 * PCIe every launch costs about 40 us whatever its size, so larger is faster. */
#define RG_REQUESTS_DEFAULT 128
#define RG_REQUESTS_MIN 32
#define RG_REQUESTS_MAX 512
#define RG_POOL_BYTES (256ull << 20)
#define RG_MAX_GPUS 8
/* Launches a channel keeps in flight per GPU.  While that many run, what the
 * reactor queues waits for the next poll instead of being launched in ever
 * smaller pieces: one batch computes while the next one grows, the GPU never
 * idles for lack of a queued launch, and a flush never has to wait for one of
 * the context's descriptor ring slots. */
#ifndef RG_MAX_INFLIGHT
#define RG_MAX_INFLIGHT 2
#endif
/* A launch takes at most 1 / RG_TAKE_DIV of the channel's busy requests. */
#ifndef RG_TAKE_DIV
#define RG_TAKE_DIV 2
#endif
#define RG_CACHE_STRIPES RAID_MAX_STRIPES

enum rg_kind { RG_WRITE_FULL, RG_WRITE_PARTIAL, RG_WRITE_DEGRADED, RG_READ };

enum rg_phase {
	RG_PHASE_PREREAD,	/* base reads before the parity work */
	RG_PHASE_GPU,		/* parity work queued or running */
	RG_PHASE_WRITE,		/* base writes after the parity work */
	RG_PHASE_READ,		/* plain base reads of a healthy read */
};

struct rg_info {
	struct raid_bdev *raid_bdev;
	struct draid_raid geom;
	draid_stripe_cache *stripes;	/* per-stripe request queue, shared by the channels */
	int ngpus;			/* slots: contexts per channel, stripe s on slot s mod ngpus */
	int ndevices;			/* GPUs the slots are dealt over */
	int nrequests;			/* stripe requests (with n strip buffers each) per channel */
	int refs;			/* the raid bdev (until stop) + every open channel */
	bool stopped;			/* stop has run: new requests fail, running ones finish */
	struct raid_gpu_stats stats;
};

/* The framework stops a level module as soon as the array leaves the online
 * state -- on a hot-remove that is while channels are open and requests in
 * flight (raid_bdev_deconfigure, bdev_raid.c:1267-1289) -- so what the requests
 * use lives until the last channel is gone. */
static void
rg_info_put(struct rg_info *info)
{
	if (__atomic_sub_fetch(&info->refs, 1, __ATOMIC_ACQ_REL) == 0) {
		draid_stripe_cache_destroy(info->stripes);
		free(info);
	}
}

#define RG_COUNT(info, field) __atomic_fetch_add(&(info)->stats.field, 1, __ATOMIC_RELAXED)

/* Section timing for the module bench (raid_gpu.h, struct raid_gpu_prof). */
#ifdef DRAID_RAID_GPU_PROFILE
static struct raid_gpu_prof g_prof;

static inline uint64_t
rg_now_ns(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}
#define RG_TIC(t) const uint64_t t = rg_now_ns()
#define RG_TOC(t, section)                                                                  \
	do {                                                                               \
		__atomic_fetch_add(&g_prof.section.ns, rg_now_ns() - (t), __ATOMIC_RELAXED); \
		__atomic_fetch_add(&g_prof.section.calls, 1, __ATOMIC_RELAXED);            \
	} while (0)
#else
#define RG_TIC(t) do {} while (0)
#define RG_TOC(t, section) do {} while (0)
#endif

void
raid_gpu_get_prof(struct raid_gpu_prof *prof, bool reset)
{
#ifdef DRAID_RAID_GPU_PROFILE
	*prof = g_prof;
	if (reset) {
		memset(&g_prof, 0, sizeof(g_prof));
	}
#else
	(void)reset;
	memset(prof, 0, sizeof(*prof));
#endif
}

static const char *
rg_level_name(const struct raid_bdev *raid_bdev)
{
	/* the framework's name table has no "raid6" entry (bdev_raid.c:880-889) */
	return raid_bdev->level == RAID5 ? "raid5" : "raid6";
}

void
raid_gpu_get_stats(const struct raid_bdev *raid_bdev, struct raid_gpu_stats *stats)
{
	const struct rg_info *info = raid_bdev->module_private;

	if (info) {
		*stats = info->stats;
	} else {
		memset(stats, 0, sizeof(*stats));
	}
}

struct rg_channel;

struct rg_request {
	struct rg_channel *ch;
	struct raid_bdev_io *raid_io;
	struct spdk_thread *thread;
	enum rg_kind kind;
	enum rg_phase phase;
	struct draid_raid geom;		/* the array's geometry + the degraded mask it runs under */
	struct draid_stripe_req sreq;
	struct draid_write_plan plan;
	struct draid_stripe *stripe;
	struct draid_stripe_waiter waiter;
	int gpu;			/* which of the channel's contexts: stripe mod ngpus */
	uint64_t ticket;
	int attempts;
	uint32_t io_failed;		/* disks whose I/O failed in this phase */
	int remaining;			/* base I/Os of this phase still to complete */
	int nio, next_io;
	bool io_write;
	bool submitting;
	struct draid_base_io *ios;	/* 3 * n entries */
	void **chunk_buf;		/* n strip buffers */
	struct spdk_bdev_io_wait_entry waitq;
	TAILQ_ENTRY(rg_request) link;
};

struct rg_channel {
	struct rg_info *info;
	draid_ec_ctx *ctx[RG_MAX_GPUS];
	uint64_t last_ticket[RG_MAX_GPUS];	/* of the latest flush */
	uint64_t done_ticket[RG_MAX_GPUS];	/* highest ticket seen finished */
	struct spdk_poller *poller;
	struct rg_request *requests;
	uint8_t *pool;			/* nrequests * n strip buffers */
	struct rg_request **batch;	/* the poller's launch under construction */
	bool pool_registered;		/* this channel registered the pool with the GPU runtime */
	TAILQ_HEAD(, rg_request) free_reqs;
	int busy_reqs;			/* stripe requests not on free_reqs */
	TAILQ_HEAD(, rg_request) ready;	/* data and prereads in: parity work to be launched */
	TAILQ_HEAD(, rg_request) running;	/* launched: waiting for the ticket */
	TAILQ_HEAD(, spdk_bdev_io_wait_entry) waiting;	/* parent I/O waiting for a request */
};

static void rg_start_request(struct rg_request *req);
static void rg_submit_ios(struct rg_request *req);
static void rg_submit_rw_request(struct raid_bdev_io *raid_io);

static inline struct raid_bdev_io_channel *
rg_raid_ch(struct rg_channel *ch)
{
	return (struct raid_bdev_io_channel *)((uint8_t *)ch - sizeof(struct raid_bdev_io_channel));
}

static uint32_t
rg_degraded_mask(const struct raid_bdev *raid_bdev)
{
	uint32_t mask = 0;
	uint8_t i;

	/* the flags are written on whichever thread sees a disk fail */
	for (i = 0; i < raid_bdev->num_base_bdevs; i++) {
		if (__atomic_load_n(&raid_bdev->base_bdev_info[i].degraded, __ATOMIC_ACQUIRE)) {
			mask |= 1u << i;
		}
	}
	return mask;
}

/* The reference's fault-injection hook (bdev_raid.c:1157-1170, commented out
 * there) as a function: marks a base bdev degraded or healthy again. */
static pthread_mutex_t g_degraded_lock = PTHREAD_MUTEX_INITIALIZER;

int
raid_gpu_set_degraded(struct raid_bdev *raid_bdev, uint8_t slot, bool degraded)
{
	uint32_t mask;
	int rc = 0;

	if (slot >= raid_bdev->num_base_bdevs) {
		return -EINVAL;
	}
	/* two channels' threads may see two different disks fail at the same time:
	 * the "one more than the level tolerates" test and the update are one step */
	pthread_mutex_lock(&g_degraded_lock);
	mask = rg_degraded_mask(raid_bdev);
	if (degraded && !(mask & (1u << slot)) &&
	    __builtin_popcount(mask) >= raid_bdev->module->base_bdevs_max_degraded) {
		rc = -EBUSY;
	} else {
		mask = degraded ? mask | (1u << slot) : mask & ~(1u << slot);
		__atomic_store_n(&raid_bdev->base_bdev_info[slot].degraded, degraded, __ATOMIC_RELEASE);
		__atomic_store_n(&raid_bdev->degraded, mask != 0, __ATOMIC_RELEASE);
	}
	pthread_mutex_unlock(&g_degraded_lock);
	return rc;
}

/* What a hot-remove handler calls for an online array of this module instead of
 * taking the whole array offline (raid_bdev_remove_base_bdev -> raid_bdev_deconfigure,
 * bdev_raid.c:1333-1365): the removed base bdev becomes a degraded disk.  New
 * requests plan around it from the next submit on; requests that already have
 * I/O on it see that I/O fail or succeed and are redone if it failed.  The base
 * bdev's descriptor and channels stay open until the array is deleted (the
 * framework releases them in raid_bdev_destruct, bdev_raid.c:285-323, for every
 * base bdev whose removal is scheduled), so the removed bdev's own unregister
 * completes only then. */
int
raid_gpu_base_bdev_removed(struct raid_bdev *raid_bdev, struct raid_base_bdev_info *base_info)
{
	const long slot = base_info - raid_bdev->base_bdev_info;
	int rc;

	if (raid_bdev->module == NULL || raid_bdev->module->submit_rw_request != rg_submit_rw_request) {
		return -ENOTSUP;	/* another level module's array */
	}
	if (raid_bdev->state != RAID_BDEV_STATE_ONLINE || raid_bdev->destruct_called ||
	    raid_bdev->module_private == NULL) {
		return -ENODEV;		/* not serving I/O: let the framework clean up */
	}
	if (slot < 0 || slot >= raid_bdev->num_base_bdevs) {
		return -EINVAL;
	}
	rc = raid_gpu_set_degraded(raid_bdev, (uint8_t)slot, true);
	if (rc != 0) {
		SPDK_ERRLOG("base bdev %ld of %s removed: more failures than %s tolerates\n", slot,
			    raid_bdev->bdev.name, rg_level_name(raid_bdev));
		return rc;
	}
	SPDK_NOTICELOG("base bdev %ld of %s removed: the array stays online, degraded\n", slot,
		       raid_bdev->bdev.name);
	return 0;
}

/* ------------------------------------------------------------ completion */

static void _rg_start_request(void *ctx)
{
	rg_start_request(ctx);
}

static void rg_submit(struct raid_bdev_io *raid_io, bool waited);

static void _rg_resubmit(void *ctx)
{
	rg_submit(ctx, true);
}

/* raid5_complete_stripe_request (raid5.c:485-521): complete the parent I/O, hand
 * the stripe to its next queued request, give the request back. */
static void
rg_complete(struct rg_request *req, enum spdk_bdev_io_status status)
{
	struct rg_channel *ch = req->ch;
	struct rg_info *info = ch->info;
	struct raid_bdev_io *raid_io = req->raid_io;
	struct spdk_bdev_io_wait_entry *wqe;

	if (req->stripe) {
		RG_TIC(t_sq);
		struct draid_stripe_waiter *next = draid_stripe_complete(info->stripes, req->stripe,
						   &req->waiter);
		draid_stripe_put(info->stripes, req->stripe);
		RG_TOC(t_sq, stripe_queue);
		req->stripe = NULL;
		if (next) {
			struct rg_request *nreq = next->arg;
			/* the next request may live on another channel's thread (raid5.c:501-505) */
			if (nreq->thread == spdk_get_thread()) {
				rg_start_request(nreq);
			} else {
				RG_COUNT(info, handoffs);
				spdk_thread_send_msg(nreq->thread, _rg_start_request, nreq);
			}
		}
	}
	req->raid_io = NULL;
	TAILQ_INSERT_HEAD(&ch->free_reqs, req, link);
	ch->busy_reqs--;
	/* The freed request goes to the parent I/O that has waited longest, before the
	 * completion below lets the caller submit a new one (a bdevperf-style caller
	 * resubmits from its completion callback and would take the request every
	 * time, leaving the waiting I/O where it is for as long as the load lasts). */
	while (!TAILQ_EMPTY(&ch->free_reqs) && (wqe = TAILQ_FIRST(&ch->waiting)) != NULL) {
		TAILQ_REMOVE(&ch->waiting, wqe, link);
		wqe->cb_fn(wqe->cb_arg);
		if (TAILQ_FIRST(&ch->waiting) == wqe) {
			break;	/* back at the head: it waits for a stripe, not for a request */
		}
	}
	{
		RG_TIC(t_c);
		raid_bdev_io_complete(raid_io, status);
		RG_TOC(t_c, complete);
	}
}

/* ------------------------------------------------------------ base bdev I/O */

static void rg_phase_done(struct rg_request *req);

static void
rg_io_finished(struct rg_request *req)
{
	assert(req->remaining > 0);
	if (--req->remaining == 0 && !req->submitting) {
		rg_phase_done(req);
	}
}

static void
rg_chunk_io_done(struct spdk_bdev_io *bdev_io, bool success, void *cb_arg)
{
	struct rg_request *req = cb_arg;
	int disk = -1;
	uint8_t i;

	/* which disk: the completed I/O's bdev (raid5.c:596-615 gets it from the chunk) */
	if (bdev_io) {
		for (i = 0; i < req->geom.num_base_bdevs; i++) {
			if (req->ch->info->raid_bdev->base_bdev_info[i].bdev == bdev_io->bdev) {
				disk = i;
				break;
			}
		}
		spdk_bdev_free_io(bdev_io);
	}
	if (!success && disk >= 0) {
		req->io_failed |= 1u << disk;
	}
	rg_io_finished(req);
}

static void _rg_submit_ios(void *ctx)
{
	rg_submit_ios(ctx);
}

/* raid5_submit_chunk_request (raid5.c:617-689): one spdk_bdev_{read,write}v_blocks
 * per listed base I/O; -ENOMEM parks the request on the base bdev's io_wait queue
 * and continues from the same I/O. */
static void
rg_submit_ios(struct rg_request *req)
{
	struct rg_channel *ch = req->ch;
	struct raid_bdev *raid_bdev = ch->info->raid_bdev;
	struct raid_bdev_io_channel *raid_ch = rg_raid_ch(ch);

	RG_TIC(t_io);
	req->submitting = true;
	while (req->next_io < req->nio) {
		struct draid_base_io *io = &req->ios[req->next_io];
		struct raid_base_bdev_info *base_info = &raid_bdev->base_bdev_info[io->disk];
		struct spdk_io_channel *base_ch = raid_ch->base_channel[io->disk];
		int rc;

		if (req->geom.degraded_mask & (1u << io->disk)) {
			/* a write to a lost disk: parity carries it (reads never list one) */
			req->next_io++;
			req->remaining--;
			continue;
		}
		if (req->io_write) {
			rc = spdk_bdev_writev_blocks(base_info->desc, base_ch, io->iov, io->iovcnt,
						     io->offset_blocks, io->num_blocks,
						     rg_chunk_io_done, req);
		} else {
			rc = spdk_bdev_readv_blocks(base_info->desc, base_ch, io->iov, io->iovcnt,
						    io->offset_blocks, io->num_blocks,
						    rg_chunk_io_done, req);
		}
		if (spdk_unlikely(rc == -ENOMEM)) {
			req->waitq.bdev = base_info->bdev;
			req->waitq.cb_fn = _rg_submit_ios;
			req->waitq.cb_arg = req;
			spdk_bdev_queue_io_wait(base_info->bdev, base_ch, &req->waitq);
			req->submitting = false;
			RG_TOC(t_io, base_submit);
			return;
		}
		req->next_io++;
		if (spdk_unlikely(rc != 0)) {
			SPDK_ERRLOG("base bdev %d: submit failed: %s\n", io->disk, spdk_strerror(-rc));
			req->io_failed |= 1u << io->disk;
			req->remaining--;
		}
	}
	req->submitting = false;
	RG_TOC(t_io, base_submit);
	if (req->remaining == 0) {
		rg_phase_done(req);
	}
}

static void
rg_issue(struct rg_request *req, int nio, bool write, enum rg_phase phase)
{
	req->phase = phase;
	req->nio = nio;
	req->next_io = 0;
	req->remaining = nio;
	req->io_write = write;
	req->io_failed = 0;
	if (nio == 0) {
		rg_phase_done(req);
		return;
	}
	rg_submit_ios(req);
}

/* ------------------------------------------------------------ parity work */

/* Everything the request's parity work reads is in memory: the poller walks it
 * onto the context and launches it with whatever else became ready. */
static void
rg_gpu_ready(struct rg_request *req)
{
	req->phase = RG_PHASE_GPU;
	TAILQ_INSERT_TAIL(&req->ch->ready, req, link);
}

/* The parity work of a request finished on the GPU. */
static void
rg_gpu_done(struct rg_request *req)
{
	if (req->kind == RG_READ) {
		rg_complete(req, SPDK_BDEV_IO_STATUS_SUCCESS);
		return;
	}
	/* ios[] already lists the base writes (filled when the work was queued) */
	rg_issue(req, req->nio, true, RG_PHASE_WRITE);
}

static int
rg_queue_error(struct rg_request *req, int rc, const char *what)
{
	SPDK_ERRLOG("stripe %" PRIu64 ": %s failed (%d): %s\n", req->sreq.stripe_index, what, rc,
		    draid_ec_last_error());
	return rc;
}

/* A request's parity work is queued whole or not at all: it may take several
 * queueing calls (rebuild then re-encode; one update per touched range), and a
 * later call can fail (a parent iovec the GPU cannot reach) after earlier ones
 * queued segments on this request's strip buffers and the parent's iovecs.  The
 * request is then failed and its buffers reused, so those segments must not
 * run. */
static int
rg_queue_failed(struct rg_request *req, draid_ec_ctx *ctx, int rc, const char *what)
{
	rg_queue_error(req, rc, what);
	if (draid_ec_ctx_rollback(ctx) != 0) {
		/* cannot happen without autoflush; never leave a dangling segment */
		SPDK_ERRLOG("stripe %" PRIu64 ": rollback failed: %s\n", req->sreq.stripe_index,
			    draid_ec_last_error());
	}
	return rc;
}

/* Queues the parity work of a write whose prereads (if any) are in, and lists
 * its base writes in ios[]. */
static int
rg_queue_write(struct rg_request *req)
{
	struct spdk_bdev_io *bdev_io = spdk_bdev_io_from_ctx(req->raid_io);
	draid_ec_ctx *ctx = req->ch->ctx[req->gpu];
	int nw = 0, rc;
	RG_TIC(t_w);

	draid_ec_ctx_mark(ctx);
	if (req->kind == RG_WRITE_FULL) {
		void *parity[2] = { req->chunk_buf[req->sreq.p_disk],
				    req->sreq.q_disk >= 0 ? req->chunk_buf[req->sreq.q_disk] : NULL
				  };

		rc = draid_raid_stripe_write(&req->geom, ctx, &req->sreq, bdev_io->u.bdev.iovs,
					     bdev_io->u.bdev.iovcnt, parity, req->ios, &nw);
		if (rc) {
			return rg_queue_failed(req, ctx, rc, "draid_raid_stripe_write");
		}
	} else {
		if (req->kind == RG_WRITE_DEGRADED) {
			/* every surviving strip is in chunk_buf: rebuild the lost ones there,
			 * then re-encode the whole strip range over old + new data (the
			 * reconstruct-write of raid5.c:743-777 with nothing left to read) */
			rc = draid_raid_stripe_degraded_rebuild(&req->geom, ctx, req->sreq.stripe_index,
								req->chunk_buf);
			if (rc) {
				return rg_queue_failed(req, ctx, rc, "draid_raid_stripe_degraded_rebuild");
			}
			/* the encode below reads the rebuilt strips: it must not share a launch
			 * with encodes other requests queued ahead of this rebuild */
			draid_ec_ctx_fence(ctx);
			memset(&req->plan, 0, sizeof(req->plan));
			req->plan.mode = DRAID_WRITE_RCW;
			req->plan.p_offset = 0;
			req->plan.p_blocks = req->geom.strip_size;
		}
		rc = draid_raid_stripe_write_partial(&req->geom, ctx, &req->sreq, &req->plan,
						     bdev_io->u.bdev.iovs, bdev_io->u.bdev.iovcnt,
						     req->chunk_buf, req->ios, &nw);
		if (rc) {
			return rg_queue_failed(req, ctx, rc, "draid_raid_stripe_write_partial");
		}
	}
	req->nio = nw;
	RG_TOC(t_w, walk);
	return 0;
}

/* The rebuild of a degraded read's lost requested range, straight into the
 * parent's iovecs. */
static int
rg_queue_read_rebuild(struct rg_request *req)
{
	struct spdk_bdev_io *bdev_io = spdk_bdev_io_from_ctx(req->raid_io);
	draid_ec_ctx *ctx = req->ch->ctx[req->gpu];
	int rc;
	RG_TIC(t_w);

	draid_ec_ctx_mark(ctx);
	rc = draid_raid_stripe_read_rebuild(&req->geom, ctx, &req->sreq, bdev_io->u.bdev.iovs,
					    bdev_io->u.bdev.iovcnt, req->chunk_buf);
	RG_TOC(t_w, walk);
	if (rc) {
		return rg_queue_failed(req, ctx, rc, "draid_raid_stripe_read_rebuild");
	}
	return 0;
}

/* ------------------------------------------------------------ phases */

static bool
rg_absorb_failures(struct rg_request *req)
{
	struct raid_bdev *raid_bdev = req->ch->info->raid_bdev;
	uint32_t failed = req->io_failed;
	uint8_t i;

	for (i = 0; failed && i < raid_bdev->num_base_bdevs; i++) {
		if (!(failed & (1u << i))) {
			continue;
		}
		if (raid_gpu_set_degraded(raid_bdev, i, true) != 0) {
			SPDK_ERRLOG("base bdev %u failed: more failures than %s tolerates\n", i,
				    rg_level_name(raid_bdev));
			return false;
		}
		SPDK_NOTICELOG("base bdev %u failed: raid bdev %s is degraded\n", i,
			       raid_bdev->bdev.name);
	}
	return true;
}

static void
rg_phase_done(struct rg_request *req)
{
	if (spdk_unlikely(req->io_failed)) {
		/* a base bdev failed under this request: mark it degraded and, when the
		 * level still tolerates that, redo the request against the new state */
		const bool tolerable = rg_absorb_failures(req);

		if (req->phase == RG_PHASE_WRITE) {
			/* parity was computed over all the new data: a lost disk's write
			 * is covered by it */
			rg_complete(req, tolerable ? SPDK_BDEV_IO_STATUS_SUCCESS :
				    SPDK_BDEV_IO_STATUS_FAILED);
			return;
		}
		if (!tolerable || ++req->attempts > req->geom.max_degraded + 1) {
			rg_complete(req, SPDK_BDEV_IO_STATUS_FAILED);
			return;
		}
		RG_COUNT(req->ch->info, redone);
		rg_start_request(req);
		return;
	}

	switch (req->phase) {
	case RG_PHASE_PREREAD:
		/* the surviving ranges (read) or the prereads (write) are in */
		rg_gpu_ready(req);
		break;
	case RG_PHASE_READ:
	case RG_PHASE_WRITE:
		rg_complete(req, SPDK_BDEV_IO_STATUS_SUCCESS);
		break;
	default:
		assert(false);
		rg_complete(req, SPDK_BDEV_IO_STATUS_FAILED);
		break;
	}
}

/* The request owns its stripe: plan it against the current degraded state
 * (raid5_submit_stripe_request, raid5.c:948-960). */
static void
rg_start_request(struct rg_request *req)
{
	struct rg_info *info = req->ch->info;
	struct spdk_bdev_io *bdev_io = spdk_bdev_io_from_ctx(req->raid_io);
	const int n = req->geom.num_base_bdevs;
	int nio = 0, rc, ndeg;
	bool write = bdev_io->type == SPDK_BDEV_IO_TYPE_WRITE;

	req->geom.degraded_mask = rg_degraded_mask(info->raid_bdev);
	ndeg = __builtin_popcount(req->geom.degraded_mask);
	if (ndeg > req->geom.max_degraded) {
		SPDK_ERRLOG("stripe %" PRIu64 ": %d base bdevs degraded, %s tolerates %u\n",
			    req->sreq.stripe_index, ndeg, rg_level_name(info->raid_bdev),
			    req->geom.max_degraded);
		rg_complete(req, SPDK_BDEV_IO_STATUS_FAILED);
		return;
	}

	if (!write) {
		uint32_t lost_requested = 0;
		int disk;

		req->kind = RG_READ;
		for (disk = 0; disk < n; disk++) {
			if ((req->geom.degraded_mask & (1u << disk)) && disk != req->sreq.p_disk &&
			    disk != req->sreq.q_disk && req->sreq.chunk[disk].req_blocks) {
				lost_requested |= 1u << disk;
			}
		}
		{
			RG_TIC(t_p);
			rc = draid_raid_stripe_read(&req->geom, NULL, &req->sreq, bdev_io->u.bdev.iovs,
						    bdev_io->u.bdev.iovcnt, req->chunk_buf, req->ios,
						    &nio);
			RG_TOC(t_p, plan);
		}
		if (rc) {
			rg_queue_error(req, rc, "draid_raid_stripe_read");
			rg_complete(req, SPDK_BDEV_IO_STATUS_FAILED);
			return;
		}
		/* healthy chunks: plain reads into the parent iovecs (raid5.c:933-945);
		 * a lost requested chunk: the other strips' ranges first, then the rebuild */
		if (lost_requested) {
			RG_COUNT(info, degraded_reads);
		} else {
			RG_COUNT(info, reads);
		}
		rg_issue(req, nio, false, lost_requested ? RG_PHASE_PREREAD : RG_PHASE_READ);
		return;
	}

	if (ndeg == 0 && req->sreq.full_stripe) {
		req->kind = RG_WRITE_FULL;
		RG_COUNT(info, full_stripe_writes);
		rg_gpu_ready(req);
		return;
	}
	if (ndeg == 0) {
		req->kind = RG_WRITE_PARTIAL;
		{
			RG_TIC(t_p);
			rc = draid_raid_plan_write(&req->geom, &req->sreq, &req->plan, req->chunk_buf,
						   req->ios, &nio);
			RG_TOC(t_p, plan);
		}
		if (rc) {
			rg_queue_error(req, rc, "draid_raid_plan_write");
			rg_complete(req, SPDK_BDEV_IO_STATUS_FAILED);
			return;
		}
		if (req->plan.mode == DRAID_WRITE_RMW) {
			RG_COUNT(info, rmw_writes);
		} else {
			RG_COUNT(info, rcw_writes);
		}
		rg_issue(req, nio, false, RG_PHASE_PREREAD);
		return;
	}
	if (req->sreq.full_stripe) {
		/* every data strip is new: encode, then skip the writes to lost disks */
		req->kind = RG_WRITE_FULL;
		RG_COUNT(info, full_stripe_writes);
		rg_gpu_ready(req);
		return;
	}
	/* partial write to a degraded array: read every surviving strip, rebuild the
	 * lost ones, re-encode over old + new data */
	req->kind = RG_WRITE_DEGRADED;
	RG_COUNT(info, degraded_writes);
	rc = draid_raid_stripe_degraded_read(&req->geom, NULL, req->sreq.stripe_index, req->chunk_buf,
					     req->ios, &nio);
	if (rc) {
		rg_queue_error(req, rc, "draid_raid_stripe_degraded_read");
		rg_complete(req, SPDK_BDEV_IO_STATUS_FAILED);
		return;
	}
	rg_issue(req, nio, false, RG_PHASE_PREREAD);
}

/* ------------------------------------------------------------ submit */

/* raid5_submit_rw_request (raid5.c:1292-1324): the bdev layer has split the
 * parent I/O at stripe boundaries (optimal_io_boundary, set in rg_start). */
static void
rg_submit_rw_request(struct raid_bdev_io *raid_io)
{
	rg_submit(raid_io, false);
}

/* waited: the parent I/O comes from the head of the channel's waiting list. */
static void
rg_submit(struct raid_bdev_io *raid_io, bool waited)
{
	struct spdk_bdev_io *bdev_io = spdk_bdev_io_from_ctx(raid_io);
	struct rg_channel *ch = raid_bdev_io_channel_get_resource(raid_io->raid_ch);
	struct rg_info *info = ch->info;	/* module_private is gone once the module stopped */
	struct rg_request *req;
	int rc;

	if (spdk_unlikely(info->stopped)) {
		/* the array went offline (a base bdev was removed, or it is being
		 * deleted) with this channel still open */
		raid_bdev_io_complete(raid_io, SPDK_BDEV_IO_STATUS_FAILED);
		return;
	}
	req = TAILQ_FIRST(&ch->free_reqs);
	if (spdk_unlikely(req == NULL || (!waited && !TAILQ_EMPTY(&ch->waiting)))) {
		/* all stripe requests in flight: retry when one completes
		 * (raid5_simple.c:364-370).  Parent I/O of one channel gets its requests in
		 * the order it was submitted: a new one queues behind those that wait. */
		struct spdk_bdev_io_wait_entry *wqe = &raid_io->waitq_entry;

		wqe->cb_fn = _rg_resubmit;
		wqe->cb_arg = raid_io;
		if (waited) {
			TAILQ_INSERT_HEAD(&ch->waiting, wqe, link);	/* it keeps its place */
		} else {
			TAILQ_INSERT_TAIL(&ch->waiting, wqe, link);
		}
		return;
	}

	{
		RG_TIC(t_m);
		req->geom = info->geom;
		rc = draid_raid_map_request(&req->geom, bdev_io->u.bdev.offset_blocks,
					    bdev_io->u.bdev.num_blocks, &req->sreq);
		RG_TOC(t_m, map);
	}
	if (spdk_unlikely(rc != 0)) {
		SPDK_ERRLOG("request [%" PRIu64 ", +%" PRIu64 ") does not map onto one stripe\n",
			    bdev_io->u.bdev.offset_blocks, bdev_io->u.bdev.num_blocks);
		raid_bdev_io_complete(raid_io, SPDK_BDEV_IO_STATUS_FAILED);
		return;
	}
	{
		RG_TIC(t_sq);
		req->stripe = draid_stripe_get(info->stripes, req->sreq.stripe_index);
		RG_TOC(t_sq, stripe_queue);
	}
	if (spdk_unlikely(req->stripe == NULL)) {
		/* every cached stripe is referenced (raid5.c:1310-1318): retry later */
		struct spdk_bdev_io_wait_entry *wqe = &raid_io->waitq_entry;

		wqe->cb_fn = _rg_resubmit;
		wqe->cb_arg = raid_io;
		if (waited) {
			TAILQ_INSERT_HEAD(&ch->waiting, wqe, link);
		} else {
			TAILQ_INSERT_TAIL(&ch->waiting, wqe, link);
		}
		return;
	}
	TAILQ_REMOVE(&ch->free_reqs, req, link);
	ch->busy_reqs++;
	req->raid_io = raid_io;
	req->thread = spdk_get_thread();
	req->gpu = (int)(req->sreq.stripe_index % (uint64_t)info->ngpus);
	req->attempts = 0;
	req->io_failed = 0;
	req->waiter.arg = req;
	/* requests on one stripe run one at a time, in arrival order
	 * (raid5.c:1047-1054) */
	{
		RG_TIC(t_sq);
		rc = draid_stripe_enqueue(info->stripes, req->stripe, &req->waiter);
		RG_TOC(t_sq, stripe_queue);
	}
	if (rc == 1) {
		rg_start_request(req);
	}
}

/* ------------------------------------------------------------ poller */

/* A flush failed: `batch` holds the requests walked onto the context for it. */
static void
rg_fail_batch(struct rg_channel *ch, int gpu, struct rg_request **batch, int n)
{
	int i;

	/* launched pieces may still write the requests' buffers: wait them out */
	draid_ec_ctx_synchronize(ch->ctx[gpu]);
	draid_ec_ctx_discard_queued(ch->ctx[gpu]);
	for (i = 0; i < n; i++) {
		rg_complete(batch[i], SPDK_BDEV_IO_STATUS_FAILED);
	}
}

/* Finishes the requests whose launch has completed, then launches the parity
 * work of requests that became ready -- one launch per GPU and poll.
 *
 * How much goes into a launch decides how well the GPU and the reactor overlap.
 * Everything that is ready in one launch -- the obvious choice -- locks a busy
 * channel into step: all its requests compute together, then do their base I/O
 * together, then are resubmitted together, and the GPU idles through the
 * reactor's part and the reactor through the GPU's.  So a launch takes at most
 * half of the channel's requests in flight (one when there is only one), and
 * no more than RG_MAX_INFLIGHT launches run per GPU: two groups of requests
 * form that alternate between the GPU and the reactor, and whatever becomes
 * ready while both launches run joins the next one. */
static int
rg_poll(void *arg)
{
	struct rg_channel *ch = arg;
	struct rg_info *info = ch->info;
	struct rg_request *req, *tmp;
	struct rg_request **batch = ch->batch;
	uint64_t running_from[RG_MAX_GPUS] = { 0 };	/* lowest ticket found still running */
	int g, busy = 0;

	/* tickets of one context finish in order and `running` is in launch order, so
	 * one query per context and poll tells "still running" for all that follow */
	TAILQ_FOREACH_SAFE(req, &ch->running, link, tmp) {
		int rc;

		g = req->gpu;
		if (running_from[g] && req->ticket >= running_from[g]) {
			continue;
		}
		if (req->ticket <= ch->done_ticket[g]) {
			rc = 0;
		} else {
			RG_TIC(t_q);
			rc = draid_ec_ctx_ticket_query(ch->ctx[g], req->ticket);
			RG_TOC(t_q, poll);
		}
		if (rc == 1) {
			running_from[g] = req->ticket;	/* another GPU's requests may be done */
			continue;
		}
		busy = 1;
		TAILQ_REMOVE(&ch->running, req, link);
		/* over, one way or the other: it no longer counts as in flight */
		ch->done_ticket[g] = spdk_max(ch->done_ticket[g], req->ticket);
		if (spdk_unlikely(rc != 0)) {
			SPDK_ERRLOG("parity work failed (%d): %s\n", rc, draid_ec_last_error());
			rg_complete(req, SPDK_BDEV_IO_STATUS_FAILED);
			continue;
		}
		rg_gpu_done(req);
	}
	if (TAILQ_EMPTY(&ch->ready)) {
		return busy ? SPDK_POLLER_BUSY : SPDK_POLLER_IDLE;
	}
	for (g = 0; g < info->ngpus; g++) {
		const int take = spdk_max(1, (ch->busy_reqs + RG_TAKE_DIV - 1) / RG_TAKE_DIV);
		uint64_t ticket;
		int rc, n = 0, i;

		if (ch->last_ticket[g] - ch->done_ticket[g] >= RG_MAX_INFLIGHT) {
			busy = 1;
			continue;	/* what is ready waits, and grows, until a launch finishes */
		}
		TAILQ_FOREACH_SAFE(req, &ch->ready, link, tmp) {
			if (req->gpu != g) {
				continue;
			}
			if (n == take) {
				break;
			}
			TAILQ_REMOVE(&ch->ready, req, link);
			rc = req->kind == RG_READ ? rg_queue_read_rebuild(req) : rg_queue_write(req);
			if (spdk_unlikely(rc != 0)) {
				/* nothing of it is queued (rg_queue_failed) */
				rg_complete(req, SPDK_BDEV_IO_STATUS_FAILED);
				continue;
			}
			batch[n++] = req;
		}
		if (n == 0) {
			continue;
		}
		busy = 1;
		{
			RG_TIC(t_f);
			rc = draid_ec_ctx_flush_ticket(ch->ctx[g], &ticket);
			RG_TOC(t_f, flush);
		}
		if (spdk_unlikely(rc != 0)) {
			SPDK_ERRLOG("parity flush failed (%d): %s\n", rc, draid_ec_last_error());
			rg_fail_batch(ch, g, batch, n);
			continue;
		}
		RG_COUNT(info, flushes);
		ch->last_ticket[g] = ticket;
		for (i = 0; i < n; i++) {
			RG_COUNT(info, gpu_requests);
			batch[i]->ticket = ticket;
			TAILQ_INSERT_TAIL(&ch->running, batch[i], link);
		}
	}
	return busy ? SPDK_POLLER_BUSY : SPDK_POLLER_IDLE;
}

/* ------------------------------------------------------------ channel, start, stop */

static void
rg_io_channel_resource_deinit(void *resource)
{
	struct rg_channel *ch = resource;
	int g;

	assert(TAILQ_EMPTY(&ch->ready) && TAILQ_EMPTY(&ch->running) && TAILQ_EMPTY(&ch->waiting));
	spdk_poller_unregister(&ch->poller);
	for (g = 0; g < RG_MAX_GPUS; g++) {
		if (ch->ctx[g]) {
			draid_ec_ctx_destroy(ch->ctx[g]);
			ch->ctx[g] = NULL;
		}
	}
	if (ch->requests) {
		int i;

		for (i = 0; i < ch->info->nrequests; i++) {
			free(ch->requests[i].ios);
			free(ch->requests[i].chunk_buf);
		}
		free(ch->requests);
		ch->requests = NULL;
	}
	free(ch->batch);
	ch->batch = NULL;
	if (ch->pool) {
		if (ch->pool_registered) {
			/* drops the pinning and the library's cached translation of the range,
			 * so a later allocation at these addresses is looked up afresh */
			draid_ec_host_unregister(ch->pool);
			ch->pool_registered = false;
		}
		spdk_dma_free(ch->pool);
		ch->pool = NULL;
	}
	if (ch->info) {
		rg_info_put(ch->info);
		ch->info = NULL;
	}
}

/* raid5_io_channel_resource_init (raid5.c:1491-1541): the channel's request
 * pool and strip buffers, plus one context per GPU and the completion poller. */
static int
rg_io_channel_resource_init(struct raid_bdev *raid_bdev, void *resource)
{
	struct rg_channel *ch = resource;
	struct rg_info *info = raid_bdev->module_private;
	const int n = raid_bdev->num_base_bdevs;
	const size_t strip_bytes = (size_t)raid_bdev->strip_size * raid_bdev->bdev.blocklen;
	struct raid_base_bdev_info *base_info;
	size_t alignment = 4096;
	int i, j, g, dev = 0;

	memset(ch, 0, sizeof(*ch));
	ch->info = info;
	__atomic_add_fetch(&info->refs, 1, __ATOMIC_RELAXED);
	TAILQ_INIT(&ch->free_reqs);
	TAILQ_INIT(&ch->ready);
	TAILQ_INIT(&ch->running);
	TAILQ_INIT(&ch->waiting);

	RAID_FOR_EACH_BASE_BDEV(raid_bdev, base_info) {
		alignment = spdk_max(alignment, spdk_bdev_get_buf_align(base_info->bdev));
	}
	ch->pool = spdk_dma_malloc((size_t)info->nrequests * n * strip_bytes, alignment, NULL);
	ch->requests = calloc((size_t)info->nrequests, sizeof(*ch->requests));
	ch->batch = calloc((size_t)info->nrequests, sizeof(*ch->batch));
	if (!ch->pool || !ch->requests || !ch->batch) {
		goto err;
	}
	{
		/* the strip buffers must be GPU reachable: DMA memory the environment
		 * registered (or allocated through draid_ec_host_alloc) already is */
		void *dev_ptr;

		if (draid_ec_device_pointer(ch->pool, (size_t)info->nrequests * n * strip_bytes,
					    &dev_ptr) != 0) {
			if (draid_ec_host_register(ch->pool,
						   (size_t)info->nrequests * n * strip_bytes) != 0) {
				SPDK_ERRLOG("strip buffers are not GPU reachable and cannot be "
					    "registered: %s\n", draid_ec_last_error());
				goto err;
			}
			ch->pool_registered = true;
		}
	}
	for (i = 0; i < info->nrequests; i++) {
		struct rg_request *req = &ch->requests[i];

		req->ch = ch;
		req->ios = calloc((size_t)3 * n, sizeof(*req->ios));
		req->chunk_buf = calloc(n, sizeof(*req->chunk_buf));
		if (!req->ios || !req->chunk_buf) {
			goto err;
		}
		for (j = 0; j < n; j++) {
			req->chunk_buf[j] = ch->pool + ((size_t)i * n + j) * strip_bytes;
		}
		TAILQ_INSERT_TAIL(&ch->free_reqs, req, link);
	}
	/* one context per GPU; stripe s runs on context s mod ngpus */
	draid_ec_device_current(&dev);
	for (g = 0; g < info->ngpus; g++) {
		int rc = draid_ec_set_device(g % info->ndevices);

		if (rc == 0) {
			rc = draid_ec_ctx_create(&ch->ctx[g]);
		}
		if (rc == 0) {
			rc = draid_ec_ctx_set_host_pointers(ch->ctx[g], 1);
		}
		if (rc != 0) {
			SPDK_ERRLOG("GPU %d: context creation failed (%d): %s\n", g, rc,
				    draid_ec_last_error());
			draid_ec_set_device(dev);
			goto err;
		}
	}
	draid_ec_set_device(dev);
	ch->poller = SPDK_POLLER_REGISTER(rg_poll, ch, 0);
	if (!ch->poller) {
		goto err;
	}
	return 0;
err:
	SPDK_ERRLOG("Failed to allocate raid gpu io channel\n");
	rg_io_channel_resource_deinit(ch);
	return -ENOMEM;
}

/* raid5_start (raid5.c:1399-1489) */
static int
rg_start(struct raid_bdev *raid_bdev)
{
	uint64_t min_blockcnt = UINT64_MAX;
	struct raid_base_bdev_info *base_info;
	struct rg_info *info;
	const char *env = getenv("DRAID_RAID_GPUS"), *env_req = getenv("DRAID_RAID_REQUESTS");
	int level = raid_bdev->level == RAID5 ? 5 : 6;
	int rc, count = 0;

	info = calloc(1, sizeof(*info));
	if (!info) {
		SPDK_ERRLOG("Failed to allocate raid gpu info\n");
		return -ENOMEM;
	}
	info->raid_bdev = raid_bdev;
	info->refs = 1;
	/* requests a channel works on at once (raid5_simple.c:14 keeps 128); more of
	 * them make larger launches when the queue is deep, at n strip buffers each */
	{
		const uint64_t stripe_bytes = (uint64_t)raid_bdev->num_base_bdevs * raid_bdev->strip_size *
					      raid_bdev->bdev.blocklen;
		const uint64_t fit = stripe_bytes ? RG_POOL_BYTES / stripe_bytes : RG_REQUESTS_DEFAULT;

		info->nrequests = (int)spdk_min(RG_REQUESTS_DEFAULT, spdk_max(RG_REQUESTS_MIN, fit));
	}
	if (env_req && atoi(env_req) > 0) {
		info->nrequests = spdk_min(spdk_max(atoi(env_req), 2), RG_REQUESTS_MAX);
	}
	RAID_FOR_EACH_BASE_BDEV(raid_bdev, base_info) {
		min_blockcnt = spdk_min(min_blockcnt, base_info->bdev->blockcnt);
	}
	rc = draid_raid_start(&info->geom, level, raid_bdev->num_base_bdevs, raid_bdev->bdev.blocklen,
			      raid_bdev->strip_size, min_blockcnt);
	if (rc == 0) {
		rc = draid_stripe_cache_create(&info->stripes, RG_CACHE_STRIPES);
	}
	if (rc != 0) {
		SPDK_ERRLOG("raid%d over %u base bdevs: invalid geometry\n", level,
			    raid_bdev->num_base_bdevs);
		free(info);
		return rc;
	}
	/* stripes spread over G slots by index (stripe mod G), one slot per GPU of the
	 * node unless DRAID_RAID_GPUS sets G */
	if (draid_ec_device_count(&count) != 0 || count < 1) {
		SPDK_ERRLOG("no GPU: %s\n", draid_ec_last_error());
		draid_stripe_cache_destroy(info->stripes);
		free(info);
		return -ENODEV;
	}
	info->ndevices = spdk_min(count, RG_MAX_GPUS);
	info->ngpus = info->ndevices;
	if (env && atoi(env) > 0) {
		/* fewer slots than GPUs leaves GPUs unused; more puts several slots on one
		 * GPU (slot g on GPU g mod count), which is how the routing is exercised
		 * on a one-GPU machine */
		info->ngpus = spdk_min(atoi(env), RG_MAX_GPUS);
	}

	raid_bdev->bdev.blockcnt = info->geom.blockcnt;
	/* one stripe per request: the bdev layer splits at stripe boundaries
	 * (raid5.c:1427-1428) */
	raid_bdev->bdev.optimal_io_boundary = info->geom.stripe_blocks;
	raid_bdev->bdev.split_on_optimal_io_boundary = true;
	raid_bdev->bdev.write_unit_size = info->geom.stripe_blocks;
	raid_bdev->module_private = info;
	return 0;
}

static void
rg_stop(struct raid_bdev *raid_bdev)
{
	struct rg_info *info = raid_bdev->module_private;

	if (info) {
		raid_bdev->module_private = NULL;
		__atomic_store_n(&info->stopped, true, __ATOMIC_RELEASE);
		rg_info_put(info);	/* freed with the last channel */
	}
}

static struct raid_bdev_module g_raid6_gpu_module = {
	.level = RAID6,
	.base_bdevs_min = 4,
	.base_bdevs_max_degraded = 2,
	.io_channel_resource_size = sizeof(struct rg_channel),
	.start = rg_start,
	.stop = rg_stop,
	.submit_rw_request = rg_submit_rw_request,
	.io_channel_resource_init = rg_io_channel_resource_init,
	.io_channel_resource_deinit = rg_io_channel_resource_deinit,
};
RAID_MODULE_REGISTER(&g_raid6_gpu_module)

#ifdef DRAID_SPDK_WITH_RAID5
/* The same engine as the RAID5 level (XOR parity only).  Off by default: the
 * reference's raid5.c registers RAID5 when CONFIG_RAID5=y and the framework
 * allows one module per level (bdev_raid.c:83-92). */
static struct raid_bdev_module g_raid5_gpu_module = {
	.level = RAID5,
	.base_bdevs_min = 3,
	.base_bdevs_max_degraded = 1,
	.io_channel_resource_size = sizeof(struct rg_channel),
	.start = rg_start,
	.stop = rg_stop,
	.submit_rw_request = rg_submit_rw_request,
	.io_channel_resource_init = rg_io_channel_resource_init,
	.io_channel_resource_deinit = rg_io_channel_resource_deinit,
};
RAID_MODULE_REGISTER(&g_raid5_gpu_module)
#endif

SPDK_LOG_REGISTER_COMPONENT(bdev_raid_gpu)
