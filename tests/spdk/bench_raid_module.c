/*
 * bench_raid_module.c -- bdevperf-shaped load on the GPU raid level module under
 * the reference's raid framework (bdev_raid.c) and the SPDK runtime stand-in.
 *
 * The workload of the reference's own benchmark for its raid modules
 * (test/bdev/bdevperf/bdevperf.c: `-w write -o <stripe> -q <depth> -t <s>` over
 * malloc bdevs): QD full-stripe writes kept outstanding against RAM base bdevs on
 * one "reactor" thread, completions resubmitting, MiB/s and IOPS at the end
 * (bdevperf.c:244-249).  Also 1-strip writes (the read-modify-write path) and
 * degraded full-stripe reads.  The RAM disks copy every strip on completion like
 * the malloc bdev (module/bdev/malloc/bdev_malloc.c:173-200), so this measures
 * the whole request path of one core -- mapping, the stripe queue, the parity
 * launch, base I/O and the copies -- not the kernels.
 *
 * With "null" as the sixth argument the base bdevs complete every I/O without
 * moving data (what module/bdev/null does): what is left is the module itself
 * and, for writes and degraded reads, the GPU reading the request buffers over
 * PCIe.  A build of the module with -DDRAID_RAID_GPU_PROFILE (the _prof binary)
 * adds where a reactor's time goes per request: request mapping, the stripe
 * queue, planning, the iovec walk, base I/O submission, the flush (descriptor
 * upload + launch), ticket polling, parent completion; the rest of the reactor's
 * time per request is the runtime stand-in and the bench's own resubmission.
 *
 *   bench_raid_module [level n strip_kib qd seconds [null]]   default: 6 10 64 32 2
 */
#include "spdk/stdinc.h"

#include "bdev_raid.h"
#include "spdk/bdev_module.h"
#include "spdk/env.h"
#include "spdk/thread.h"
#include "spdk/util.h"

#include "draid_ec.h"
#include "raid_gpu.h"
#include "spdk_stub.h"

#define CHECK(cond)                                                                   \
	do {                                                                          \
		if (!(cond)) {                                                        \
			fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
			exit(1);                                                      \
		}                                                                     \
	} while (0)

static bool g_null;

struct job;
struct task {
	struct job *job;
	struct iovec iov;
	uint8_t *buf;
	uint64_t done;	/* this task's completed I/Os: a task that waits forever shows here */
};

struct job {
	struct spdk_bdev *bdev;
	struct spdk_io_channel *ch;
	enum spdk_bdev_io_type type;
	uint64_t io_blocks, stride_blocks, span_blocks, next, done, failed;
	int outstanding;
	bool draining;
};

static double
now_s(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void task_submit(struct task *t);

static void
task_done(struct spdk_bdev_io *bdev_io, bool success, void *cb_arg)
{
	struct task *t = cb_arg;
	struct job *j = t->job;

	spdk_bdev_free_io(bdev_io);
	j->outstanding--;
	j->done++;
	if (!j->draining) {
		t->done++;
	}
	if (!success) {
		j->failed++;
	}
	if (!j->draining) {
		task_submit(t);
	}
}

static void
task_submit(struct task *t)
{
	struct job *j = t->job;
	uint64_t off = j->next;

	j->next += j->stride_blocks;
	if (j->next + j->io_blocks > j->span_blocks) {
		j->next = 0;
	}
	j->outstanding++;
	CHECK(stub_bdev_submit(j->bdev, j->ch, j->type, &t->iov, 1, off, j->io_blocks, task_done,
			       t) == 0);
}

static void
run_job(const char *name, struct raid_bdev *raid, struct spdk_io_channel *ch,
	enum spdk_bdev_io_type type, uint64_t io_blocks, uint64_t stride_blocks, int qd, double seconds)
{
	struct spdk_bdev *bdev = &raid->bdev;
	struct raid_gpu_stats s0, s1;
	struct raid_gpu_prof pr;
	struct job j = { .bdev = bdev, .ch = ch, .type = type, .io_blocks = io_blocks };
	struct task *tasks = calloc((size_t)qd, sizeof(*tasks));
	double t0, t1;
	int i;

	CHECK(tasks != NULL);
	j.stride_blocks = stride_blocks ? stride_blocks : io_blocks;
	j.span_blocks = bdev->blockcnt - bdev->blockcnt % io_blocks;
	for (i = 0; i < qd; i++) {
		tasks[i].job = &j;
		tasks[i].buf = spdk_dma_malloc(io_blocks * bdev->blocklen, 4096, NULL);
		CHECK(tasks[i].buf != NULL);
		memset(tasks[i].buf, 0x5a + i, io_blocks * bdev->blocklen);
		tasks[i].iov.iov_base = tasks[i].buf;
		tasks[i].iov.iov_len = io_blocks * bdev->blocklen;
	}
	raid_gpu_get_stats(raid, &s0);
	raid_gpu_get_prof(&pr, true);
	t0 = now_s();
	for (i = 0; i < qd; i++) {
		task_submit(&tasks[i]);
	}
	while (now_s() - t0 < seconds) {
		stub_poll();
	}
	j.draining = true;
	while (j.outstanding > 0) {
		stub_poll();
	}
	t1 = now_s();
	raid_gpu_get_stats(raid, &s1);
	raid_gpu_get_prof(&pr, false);
	printf("{\"job\": \"%s\", \"base_bdevs\": \"%s\", \"level\": %d, \"n\": %u, \"strip_kib\": %u, "
	       "\"io_kib\": %llu, \"qd\": %d, "
	       "\"seconds\": %.2f, \"ios\": %llu, \"failed\": %llu, \"iops\": %.0f, \"mib_s\": %.0f, "
	       "\"launches\": %llu, \"requests_per_launch\": %.1f",
	       name, g_null ? "null" : "ram", raid->level == RAID5 ? 5 : 6, raid->num_base_bdevs,
	       raid->strip_size * bdev->blocklen / 1024,
	       (unsigned long long)(io_blocks * bdev->blocklen / 1024), qd, t1 - t0,
	       (unsigned long long)j.done, (unsigned long long)j.failed, (double)j.done / (t1 - t0),
	       (double)j.done * (double)(io_blocks * bdev->blocklen) / (t1 - t0) / 1048576.0,
	       (unsigned long long)(s1.flushes - s0.flushes),
	       s1.flushes > s0.flushes ? (double)(s1.gpu_requests - s0.gpu_requests) /
	       (double)(s1.flushes - s0.flushes) : 0.0);
	{
		uint64_t lo = UINT64_MAX, hi = 0;

		for (i = 0; i < qd; i++) {
			lo = spdk_min(lo, tasks[i].done);
			hi = spdk_max(hi, tasks[i].done);
		}
		/* before the drain: how evenly the outstanding I/Os were served */
		printf(", \"task_ios_min\": %llu, \"task_ios_max\": %llu", (unsigned long long)lo,
		       (unsigned long long)hi);
	}
	printf(", \"reactor_us_per_request\": %.3f", (t1 - t0) * 1e6 / (double)j.done);
	if (pr.map.calls) {
		/* module sections, microseconds of reactor time per completed request */
		const double per = 1e-3 / (double)j.done;
		const double sum = (double)(pr.map.ns + pr.stripe_queue.ns + pr.plan.ns + pr.walk.ns +
					    pr.base_submit.ns + pr.flush.ns + pr.poll.ns + pr.complete.ns);

		printf(", \"module_us_per_request\": {\"map\": %.3f, \"stripe_queue\": %.3f, \"plan\": %.3f, "
		       "\"walk\": %.3f, \"base_submit\": %.3f, \"flush\": %.3f, \"poll\": %.3f, "
		       "\"complete_and_resubmit\": %.3f, \"sum\": %.3f}, \"ticket_queries_per_request\": %.1f",
		       (double)pr.map.ns * per, (double)pr.stripe_queue.ns * per, (double)pr.plan.ns * per,
		       (double)pr.walk.ns * per, (double)pr.base_submit.ns * per, (double)pr.flush.ns * per,
		       (double)pr.poll.ns * per, (double)pr.complete.ns * per, sum * per,
		       (double)pr.poll.calls / (double)j.done);
	}
	printf("}\n");
	fflush(stdout);
	CHECK(j.failed == 0);
	for (i = 0; i < qd; i++) {
		spdk_dma_free(tasks[i].buf);
	}
	free(tasks);
}

static void
removed_cb(void *ctx, int rc)
{
	*(int *)ctx = rc == 0 ? 1 : -1;
}

int
main(int argc, char **argv)
{
	const int level = argc > 1 ? atoi(argv[1]) : 6;
	const int n = argc > 2 ? atoi(argv[2]) : 10;
	const uint32_t strip_kib = argc > 3 ? (uint32_t)atoi(argv[3]) : 64;
	const int qd = argc > 4 ? atoi(argv[4]) : 32;
	const double seconds = argc > 5 ? atof(argv[5]) : 2.0;
	const bool null_io = argc > 6 && strcmp(argv[6], "null") == 0;
	const uint32_t blocklen = 4096;
	const uint32_t strip_blocks = strip_kib * 1024 / blocklen;
	const uint64_t stripes = 256;
	struct spdk_bdev *base[32];
	struct raid_bdev_config *cfg;
	struct raid_bdev *raid;
	struct spdk_io_channel *ch;
	char bname[32];
	int i, done = 0, count = 0;
	int k;

	if (draid_ec_device_count(&count) != 0 || count < 1) {
		fprintf(stderr, "no GPU: %s\n", draid_ec_last_error());
		return 2;
	}
	g_null = null_io;
	CHECK(n >= 3 && n <= 32 && strip_blocks > 0 && qd > 0 && (level == 5 || level == 6));
	k = n - (level == 5 ? 1 : 2);
	CHECK(raid_bdev_config_add("bench", strip_kib, (uint8_t)n, level == 5 ? RAID5 : RAID6, &cfg) == 0);
	for (i = 0; i < n; i++) {
		snprintf(bname, sizeof(bname), "bench_base%d", i);
		base[i] = stub_ram_bdev_create(bname, stripes * strip_blocks, blocklen);
		CHECK(base[i] != NULL);
		stub_set_null_io(base[i], null_io);
		CHECK(raid_bdev_config_add_base_bdev(cfg, bname, (uint8_t)i) == 0);
	}
	CHECK(raid_bdev_create(cfg) == 0);
	CHECK(raid_bdev_add_base_devices(cfg) == 0);
	raid = cfg->raid_bdev;
	CHECK(raid && raid->state == RAID_BDEV_STATE_ONLINE);
	ch = spdk_get_io_channel(raid);
	CHECK(ch != NULL);

	run_job("full_stripe_write", raid, ch, SPDK_BDEV_IO_TYPE_WRITE, (uint64_t)strip_blocks * k, 0, qd,
		seconds);
	/* one strip per stripe, so the queue depth is not spent waiting on one stripe's turn */
	run_job("strip_write_rmw", raid, ch, SPDK_BDEV_IO_TYPE_WRITE, strip_blocks,
		(uint64_t)strip_blocks * k, qd, seconds);
	run_job("full_stripe_read", raid, ch, SPDK_BDEV_IO_TYPE_READ, (uint64_t)strip_blocks * k, 0, qd,
		seconds);
	CHECK(raid_gpu_set_degraded(raid, 1, true) == 0);
	stub_set_dead(base[1], true);
	run_job("full_stripe_read_1_degraded", raid, ch, SPDK_BDEV_IO_TYPE_READ,
		(uint64_t)strip_blocks * k, 0, qd, seconds);
	if (level == 6) {
		CHECK(raid_gpu_set_degraded(raid, 4, true) == 0);
		stub_set_dead(base[4], true);
		run_job("full_stripe_read_2_degraded", raid, ch, SPDK_BDEV_IO_TYPE_READ,
			(uint64_t)strip_blocks * k, 0, qd, seconds);
	}

	spdk_put_io_channel(ch);
	raid_bdev_remove_base_devices(cfg, removed_cb, &done);
	CHECK(done == 1);
	raid_bdev_config_cleanup(cfg);
	for (i = 0; i < n; i++) {
		stub_ram_bdev_destroy(base[i]);
	}
	return 0;
}
