/*
 * raid_gpu.h -- what the GPU raid level module (raid_gpu.c) exports besides its
 * `struct raid_bdev_module` registration.
 */
#ifndef DRAID_SPDK_RAID_GPU_H
#define DRAID_SPDK_RAID_GPU_H

#include "bdev_raid.h"

/* Marks base bdev `slot` of a raid bdev degraded (or healthy again) and keeps
 * raid_bdev->degraded in step: the setter the reference only has as commented-out
 * test code (module/bdev/raid/bdev_raid.c:1157-1170).  A hot-remove handler that
 * keeps the array online calls it instead of raid_bdev_deconfigure
 * (bdev_raid.c:1333-1365); tests use it to inject disk failures.  Requests
 * already planned finish under the state they started with.
 * Returns 0, -EINVAL for a bad slot, -EBUSY when one more degraded disk would
 * exceed the level's base_bdevs_max_degraded. */
int raid_gpu_set_degraded(struct raid_bdev *raid_bdev, uint8_t slot, bool degraded);

/* For the framework's hot-remove path: turns the removal of `base_info`'s bdev
 * into a degraded disk of an online array of this module, where the reference
 * takes the array offline (raid_bdev_remove_base_bdev, bdev_raid.c:1333-1365).
 * The patch is one statement in front of that function's raid_bdev_deconfigure
 * call:
 *	if (raid_gpu_base_bdev_removed(raid_bdev, base_info) == 0) { return; }
 * Returns 0 when the array stays online (the caller returns); -EBUSY when the
 * level cannot tolerate one more lost disk, -ENOTSUP for another module's array,
 * -ENODEV when the array is not online -- the caller then goes on to
 * raid_bdev_deconfigure as before. */
int raid_gpu_base_bdev_removed(struct raid_bdev *raid_bdev, struct raid_base_bdev_info *base_info);

/* What the module has done on a raid bdev since it started (diagnostics and
 * tests; summed over the channels). */
struct raid_gpu_stats {
	uint64_t full_stripe_writes;	/* parity encoded from new data alone */
	uint64_t rmw_writes;		/* partial writes by read-modify-write */
	uint64_t rcw_writes;		/* partial writes by reconstruct-write */
	uint64_t degraded_writes;	/* partial writes that first rebuilt lost strips */
	uint64_t reads;			/* reads served by plain base reads */
	uint64_t degraded_reads;	/* reads that rebuilt a lost requested range */
	uint64_t redone;		/* requests redone after a base bdev failed under them */
	uint64_t handoffs;		/* a stripe handed to a request of another thread
					 * (spdk_thread_send_msg, as raid5.c:501-505) */
	uint64_t flushes;		/* launches: one per poller iteration with queued work */
	uint64_t gpu_requests;		/* requests whose parity work those launches carried */
};
void raid_gpu_get_stats(const struct raid_bdev *raid_bdev, struct raid_gpu_stats *stats);

/* Where a reactor's time goes inside the module, summed over every array and
 * channel of the process: nanoseconds and calls per section.  Only a build with
 * -DDRAID_RAID_GPU_PROFILE measures (two clock reads around each section); any
 * other build reports zeros. */
struct raid_gpu_prof_section {
	uint64_t ns, calls;
};
struct raid_gpu_prof {
	struct raid_gpu_prof_section map;	/* request -> stripe, chunk ranges (draid_raid_map_request) */
	struct raid_gpu_prof_section stripe_queue;	/* stripe cache get / enqueue / complete / put */
	struct raid_gpu_prof_section plan;	/* preread / read planning (host layer, no context calls) */
	struct raid_gpu_prof_section walk;	/* iovec walk + descriptors queued on the context */
	struct raid_gpu_prof_section base_submit;	/* spdk_bdev_{read,write}v_blocks calls */
	struct raid_gpu_prof_section flush;	/* draid_ec_ctx_flush_ticket: upload + launch */
	struct raid_gpu_prof_section poll;	/* ticket queries of the running requests */
	struct raid_gpu_prof_section complete;	/* raid_bdev_io_complete and what it calls */
};
void raid_gpu_get_prof(struct raid_gpu_prof *prof, bool reset);

#endif /* DRAID_SPDK_RAID_GPU_H */
