/*
 * test_raid_module.c -- the GPU raid level module under the reference's own raid
 * framework.
 *
 * Linked from: the reference's bdev_raid.c (compiled where it lies), the module
 * draid-spdk_amd/spdk/raid_gpu.c, the SPDK runtime stand-in spdk_stub.c,
 * libdraid_ec.so and -- as the checker only -- the CPU oracle.
 *
 * A raid bdev is created through the framework's own entry points
 * (raid_bdev_config_add / raid_bdev_create / raid_bdev_add_base_devices,
 * bdev_raid.c:785-878,1042-1111,1520-1542), over RAM base bdevs.  Every I/O goes
 * in through the registered bdev's fn_table->submit_request, i.e.
 * raid_bdev_submit_request (bdev_raid.c:495-529), after the bdev-layer split at
 * optimal_io_boundary; completions come from the module's poller.
 *
 * After every step the whole array is checked against a byte model of the
 * volume: each data strip on its disk equals the model, and each stripe's P and
 * Q equal the oracle's pq_gen / xor_gen over the model's data.  Degraded cases
 * flip base_info->degraded the way the reference's commented-out hook does
 * (bdev_raid.c:1157-1170), kill the RAM disk so that any I/O sent to it fails,
 * and check read data and the surviving disks; the lost disks' contents must be
 * recoverable from the survivors (oracle recover) and equal the model.
 */
#include "raid_test_common.h"

/* ---- scenarios */

/* the request grid of raid5_ut_ref.c:439-454 (reads) and :495-501 (partial writes) */
static int
request_grid(const struct array *a, uint64_t out[][2])
{
	const uint64_t st = a->strip_blocks, sb = a->stripe_blocks;
	const uint64_t g[][2] = {
		{ 0, 1 }, { 0, st }, { 0, st + 1 }, { 0, sb }, { 1, 1 }, { 1, st }, { 1, st + 1 },
		{ st, 1 }, { st, st }, { st, st + 1 }, { st - 1, 1 }, { st - 1, st }, { st - 1, st + 1 },
		{ st - 1, 2 }, { 0, sb - 1 }, { 1, sb - 1 }, { sb - st, st }, { sb - 1, 1 },
		{ st * 2, sb - st * 2 },
	};
	int i, n = 0;

	for (i = 0; i < (int)SPDK_COUNTOF(g); i++) {
		if (g[i][1] == 0 || g[i][0] + g[i][1] > sb) {
			continue;
		}
		out[n][0] = g[i][0];
		out[n][1] = g[i][1];
		n++;
	}
	return n;
}

static void
run_healthy(struct array *a)
{
	uint64_t grid[32][2];
	const int ng = request_grid(a, grid);
	uint64_t s;
	int i;

	snprintf(g_case, sizeof(g_case), "raid%d n=%d strip=%uKiB: full-stripe writes", a->level, a->n,
		 (unsigned)(a->strip_bytes / 1024));
	/* one stripe, several stripes in one I/O (the bdev layer splits), scattered iovecs */
	do_write(a, 0, a->stripe_blocks, 1, true);
	check_array(a, 0);
	do_write(a, a->stripe_blocks, a->stripe_blocks * 3, 5, true);
	check_array(a, 0);
	do_write(a, 0, a->stripes * a->stripe_blocks, 7, true);
	check_array(a, 0);

	snprintf(g_case, sizeof(g_case), "raid%d n=%d: reads", a->level, a->n);
	for (s = 0; s < spdk_min(a->stripes, (uint64_t)a->n + 1); s++) {
		for (i = 0; i < ng; i++) {
			do_read(a, s * a->stripe_blocks + grid[i][0], grid[i][1], 1 + i % 3, true);
		}
	}
	do_read(a, a->strip_blocks / 2, a->stripe_blocks * 2 + 1, 3, true);	/* across stripes */

	snprintf(g_case, sizeof(g_case), "raid%d n=%d: partial writes (RMW and RCW)", a->level, a->n);
	for (s = 0; s < spdk_min(a->stripes, (uint64_t)a->n + 1); s++) {
		for (i = 0; i < ng; i++) {
			do_write(a, s * a->stripe_blocks + grid[i][0], grid[i][1], 1 + i % 4, true);
		}
		check_array(a, 0);
	}
	do_write(a, a->stripe_blocks - 1, a->stripe_blocks + 2, 2, true);	/* tail + full + head */
	check_array(a, 0);
}

static void
run_degraded(struct array *a)
{
	uint64_t grid[32][2];
	const int ng = request_grid(a, grid);
	struct stub_bdev_stats st;
	int d0, d1, i, cases = 0;
	uint64_t s;

	for (d0 = 0; d0 < a->n; d0++) {
		for (d1 = (a->m == 2 ? d0 : a->n - 1); d1 < a->n; d1++) {
			uint32_t lost = 1u << d0;

			if (a->m == 2 && d1 != d0) {
				lost |= 1u << d1;
			} else if (a->m == 2 && d1 == d0 && d0 % 3) {
				continue;	/* single failures of a RAID6: every third disk */
			}
			if (a->n > 6 && (cases % 3) && __builtin_popcount(lost) == 2) {
				cases++;
				continue;	/* wide arrays: a third of the pairs */
			}
			cases++;
			snprintf(g_case, sizeof(g_case), "raid%d n=%d lost=0x%x: degraded reads", a->level,
				 a->n, lost);
			set_lost(a, lost);
			for (i = 0; i < a->n; i++) {
				stub_ram_bdev_stats(a->base[i], NULL, true);
			}
			for (s = 0; s < spdk_min(a->stripes, (uint64_t)a->n); s++) {
				for (i = 0; i < ng; i++) {
					do_read(a, s * a->stripe_blocks + grid[i][0], grid[i][1], 1 + i % 3,
						true);
				}
			}
			/* the lost disks were never touched */
			for (i = 0; i < a->n; i++) {
				stub_ram_bdev_stats(a->base[i], &st, false);
				if (lost & (1u << i)) {
					CHECK(st.reads == 0 && st.writes == 0 && st.failed == 0);
				}
			}
			snprintf(g_case, sizeof(g_case), "raid%d n=%d lost=0x%x: degraded writes", a->level,
				 a->n, lost);
			s = (uint64_t)cases % a->stripes;
			do_write(a, s * a->stripe_blocks, a->stripe_blocks, 2, true);	/* full stripe */
			for (i = 0; i < ng; i += 3) {
				const uint64_t t = (s + 1 + (uint64_t)i) % a->stripes;

				do_write(a, t * a->stripe_blocks + grid[i][0], grid[i][1], 1 + i % 2, true);
			}
			for (i = 0; i < a->n; i++) {
				stub_ram_bdev_stats(a->base[i], &st, false);
				if (lost & (1u << i)) {
					CHECK(st.reads == 0 && st.writes == 0 && st.failed == 0);
				}
			}
			check_array(a, lost);
			/* bring the disks back in sync with the model for the next case: a
			 * healthy full rewrite of everything (no rebuild in the reference) */
			set_lost(a, 0);
			do_write(a, 0, a->stripes * a->stripe_blocks, 3, true);
			check_array(a, 0);
		}
	}
	/* one failure more than the level tolerates */
	snprintf(g_case, sizeof(g_case), "raid%d n=%d: too many failures", a->level, a->n);
	set_lost(a, a->m == 2 ? 0x3 : 0x1);
	CHECK(raid_gpu_set_degraded(a->raid, (uint8_t)(a->n - 1), true) == -EBUSY);
	set_lost(a, 0);
}

static void
run_faults(struct array *a)
{
	const int errors_before = stub_error_count();
	uint64_t off;
	int i;

	/* -ENOMEM from base bdevs: parked on the io_wait queue and retried
	 * (raid5.c:664-676) */
	snprintf(g_case, sizeof(g_case), "raid%d n=%d: -ENOMEM retries", a->level, a->n);
	for (i = 0; i < a->n; i++) {
		stub_inject_enomem(a->base[i], 2);
	}
	do_write(a, 0, a->stripe_blocks, 1, true);
	do_write(a, a->stripe_blocks + 1, a->strip_blocks, 1, true);
	do_read(a, 0, a->stripe_blocks * 2, 2, true);
	check_array(a, 0);
	for (i = 0; i < a->n; i++) {
		struct stub_bdev_stats st;

		stub_ram_bdev_stats(a->base[i], &st, false);
		stub_inject_enomem(a->base[i], 0);
	}

	/* a disk dies under a read: the module marks it degraded and redoes the
	 * request as a degraded read */
	snprintf(g_case, sizeof(g_case), "raid%d n=%d: disk dies under a read", a->level, a->n);
	{
		const int victim = data_disk(a, 2 % a->stripes, 0);

		stub_set_dead(a->base[victim], true);
		CHECK(!a->raid->degraded);
		do_read(a, (2 % a->stripes) * a->stripe_blocks, a->stripe_blocks, 1, true);
		CHECK(a->raid->degraded && a->raid->base_bdev_info[victim].degraded);
		/* and under a partial write: a second disk (RAID6) or failure (RAID5) */
		if (a->m == 2) {
			const int victim2 = (victim + 2) % a->n;

			stub_set_dead(a->base[victim2], true);
			off = (3 % a->stripes) * a->stripe_blocks + 1;
			do_write(a, off, a->strip_blocks + 1, 2, true);
			CHECK(a->raid->base_bdev_info[victim2].degraded);
			check_array(a, (1u << victim) | (1u << victim2));
			/* a third: the request fails, with an error, and nothing hangs */
			{
				uint8_t *buf = dma(a->stripe_blocks * a->blocklen);
				int third = 0;

				while (third == victim || third == victim2) {
					third++;
				}
				stub_set_dead(a->base[third], true);
				CHECK(!volume_io(a, SPDK_BDEV_IO_TYPE_READ, 0, a->stripe_blocks, buf, 1));
				CHECK(!a->raid->base_bdev_info[third].degraded);
				stub_set_dead(a->base[third], false);
				spdk_dma_free(buf);
			}
			CHECK(stub_error_count() > errors_before);
		} else {
			check_array(a, 1u << victim);
		}
		set_lost(a, 0);
		do_write(a, 0, a->stripes * a->stripe_blocks, 2, true);
		check_array(a, 0);
	}

	/* A request's parity work is queued whole or not at all.  A degraded partial
	 * write queues the rebuild of the lost strips first and its re-encode second;
	 * with a parent buffer the GPU cannot reach the second call fails.  The rebuild
	 * must not stay queued: the request is failed, and the next request -- which
	 * gets the same stripe request and strip buffers -- would have them rewritten
	 * under it by the next launch.  Next here: a healthy RMW of the chunk whose
	 * strip buffer that rebuild would have written. */
	snprintf(g_case, sizeof(g_case), "raid%d n=%d: failed request leaves nothing queued", a->level,
		 a->n);
	{
		const uint64_t s1 = 1 % a->stripes, s2 = 4 % a->stripes;
		const int victim = data_disk(a, s1, 0);
		const int before = stub_error_count();
		uint8_t *buf;
		int d2 = 0;

		set_lost(a, 1u << victim);
		stub_set_plain_dma(true);
		buf = dma((a->strip_blocks + 1) * a->blocklen);
		stub_set_plain_dma(false);
		CHECK(!volume_io(a, SPDK_BDEV_IO_TYPE_WRITE, s1 * a->stripe_blocks + 1, a->strip_blocks + 1,
				 buf, 1));
		CHECK(stub_error_count() > before);
		spdk_dma_free(buf);
		set_lost(a, 0);
		while (d2 < a->k && data_disk(a, s2, d2) != victim) {
			d2++;
		}
		if (d2 < a->k) {
			do_write(a, s2 * a->stripe_blocks + (uint64_t)d2 * a->strip_blocks,
				 spdk_max(1u, a->strip_blocks / 2), 1, true);
		}
		do_write(a, s1 * a->stripe_blocks + 1, a->strip_blocks + 1, 2, true);
		check_array(a, 0);
	}

	/* a buffer the GPU cannot reach: the I/O fails, the process lives */
	snprintf(g_case, sizeof(g_case), "raid%d n=%d: pageable I/O buffer", a->level, a->n);
	{
		uint8_t *buf;
		const int before = stub_error_count();

		stub_set_plain_dma(true);
		buf = dma(a->stripe_blocks * a->blocklen);
		stub_set_plain_dma(false);
		CHECK(!volume_io(a, SPDK_BDEV_IO_TYPE_WRITE, 0, a->stripe_blocks, buf, 1));
		CHECK(stub_error_count() > before);
		spdk_dma_free(buf);
		check_array(a, 0);
	}
}

/* Many I/Os in flight: more than the channel's requests, several on one stripe. */
struct flight {
	struct io_wait w;
	struct iovec iov;
	uint8_t *buf;
	uint64_t off, blocks;
	bool write;
};

static void
run_queue_depth(struct array *a)
{
	enum { N = 160 };
	struct flight *f = calloc(N, sizeof(*f));
	int i, all = 0;

	snprintf(g_case, sizeof(g_case), "raid%d n=%d: %d I/Os in flight", a->level, a->n, N);
	CHECK(f != NULL);
	for (i = 0; i < N; i++) {
		const uint64_t s = (uint64_t)(i * 7) % a->stripes;

		/* writes only, disjoint within a stripe per round so any order gives the
		 * same bytes: chunk (i / stripes) % k of stripe s, plus full stripes */
		f[i].write = true;
		if (i % 5 == 0) {
			f[i].off = s * a->stripe_blocks;
			f[i].blocks = a->stripe_blocks;
		} else {
			const uint64_t c = (uint64_t)(i / 5) % (uint64_t)a->k;

			f[i].off = s * a->stripe_blocks + c * a->strip_blocks + (i % 2 && a->strip_blocks > 1);
			f[i].blocks = spdk_max(1u, a->strip_blocks / 2);
		}
		f[i].buf = dma(f[i].blocks * a->blocklen);
		fill(f[i].buf, f[i].blocks * a->blocklen, &a->seed);
		f[i].iov.iov_base = f[i].buf;
		f[i].iov.iov_len = f[i].blocks * a->blocklen;
	}
	/* submitted in order: requests on one stripe must also take effect in order */
	for (i = 0; i < N; i++) {
		CHECK(stub_bdev_submit(a->bdev, a->ch, SPDK_BDEV_IO_TYPE_WRITE, &f[i].iov, 1, f[i].off,
				       f[i].blocks, io_done, &f[i].w) == 0);
		memcpy(a->model + f[i].off * a->blocklen, f[i].buf, f[i].blocks * a->blocklen);
	}
	for (i = 0; i < 2000000 && !all; i++) {
		int j;

		stub_poll();
		all = 1;
		for (j = 0; j < N; j++) {
			all &= f[j].w.done;
		}
	}
	CHECK(all);
	for (i = 0; i < N; i++) {
		CHECK(f[i].w.success);
		spdk_dma_free(f[i].buf);
	}
	free(f);
	check_array(a, 0);
	do_read(a, 0, a->stripes * a->stripe_blocks, 4, true);
}

static void
run_array(int level, int n, uint32_t strip_kb, uint32_t blocklen, uint64_t stripes, bool thorough)
{
	struct array a;

	array_create(&a, level, n, strip_kb, blocklen, stripes);
	run_healthy(&a);
	run_queue_depth(&a);
	if (thorough) {
		run_degraded(&a);
	}
	run_faults(&a);
	{
		struct raid_gpu_stats st;

		/* every path of the module ran on this array */
		raid_gpu_get_stats(a.raid, &st);
		CHECK(st.full_stripe_writes > 0 && st.rmw_writes + st.rcw_writes > 0 && st.reads > 0);
		CHECK(n < 6 || (st.rmw_writes > 0 && st.rcw_writes > 0));
		CHECK(st.degraded_reads > 0 && st.degraded_writes > 0 && st.redone > 0);
		CHECK(st.flushes > 0 && st.gpu_requests > st.flushes);	/* launches carry batches */
		printf("   full %" PRIu64 " rmw %" PRIu64 " rcw %" PRIu64 " degraded-write %" PRIu64
		       " read %" PRIu64 " degraded-read %" PRIu64 " redone %" PRIu64 " | %" PRIu64
		       " requests in %" PRIu64 " launches\n", st.full_stripe_writes, st.rmw_writes,
		       st.rcw_writes, st.degraded_writes, st.reads, st.degraded_reads, st.redone,
		       st.gpu_requests, st.flushes);
	}
	snprintf(g_case, sizeof(g_case), "raid%d n=%d: teardown", level, n);
	array_destroy(&a);
	printf("ok raid%d n=%d strip=%uKiB blocklen=%u stripes=%" PRIu64 "\n", level, n, strip_kb, blocklen,
	       stripes);
	fflush(stdout);
}

int
main(int argc, char **argv)
{
	int count = 0;

	if (argc > 1 && strcmp(argv[1], "-v") == 0) {
		stub_set_log_level(2);
	}
	if (draid_ec_device_count(&count) != 0 || count < 1) {
		fprintf(stderr, "no GPU: %s\n", draid_ec_last_error());
		return 2;
	}
	/* the metric's shape: RAID6 8+2, 64 KiB strips, 4096-byte blocks */
	run_array(6, 10, 64, 4096, 12, true);
	/* the smallest RAID6, tiny strips, 512-byte blocks; a wide one */
	run_array(6, 4, 4, 512, 9, true);
	run_array(6, 6, 16, 4096, 7, true);
	run_array(6, 18, 8, 512, 5, false);
#ifdef DRAID_SPDK_WITH_RAID5
	/* config 1's shape (RAID5 4+1, 64 KiB strips) and raid5_ut's smallest */
	run_array(5, 5, 64, 4096, 8, true);
	run_array(5, 3, 4, 512, 6, true);
#endif
	printf("raid module under the reference framework: %d array checks passed, %d errors logged "
	       "(the expected ones)\n", g_checks, stub_error_count());
	return 0;
}
