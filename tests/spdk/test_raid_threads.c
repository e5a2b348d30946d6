/*
 * test_raid_threads.c -- the GPU raid level module on several SPDK threads, and
 * through the removal of a base bdev.
 *
 * The reference serialises the requests of one stripe and hands the stripe's
 * next request to the thread of the channel it came in on (raid5.c:1047-1054,
 * 496-505); its unit tests simulate several SPDK threads in one process
 * (test/common/lib/ut_multithread.c:78,200).  Here, under the reference's own
 * bdev_raid.c and the runtime stand-in:
 *
 *  1. interleaved: four SPDK threads, one channel each on a RAID6 8+2 x 64 KiB
 *     array, stepped round-robin from one OS thread in changing order.  Every
 *     round queues full-stripe writes, RMW and RCW partial writes, reads and
 *     degraded reads from all threads onto the same few stripes.  Requests of
 *     one stripe must take effect in arrival order whichever thread they came
 *     from, so the byte model applies writes in submission order and every read
 *     must return the model as it stood when the read was submitted.  Rounds run
 *     healthy, with one and two lost disks, and with a disk that dies while the
 *     round is in flight.  At least one cross-thread hand-off must be seen.
 *  2. channel exhaustion: more requests per channel than it has stripe requests.
 *  3. OS threads: the same array with each SPDK thread driven by its own
 *     pthread -- real interleaving of the stripe cache, the per-channel contexts
 *     and the message rings.  Writers own disjoint chunks of the shared stripes,
 *     so the outcome does not depend on the order.
 *  4. hot-remove (bdev_raid.c:1333-1390): a base bdev is removed with I/O in
 *     flight.  With the reference's framework as it is the array goes offline:
 *     requests in flight finish, later ones fail, nothing stays allocated.  With
 *     the one-statement redirect to raid_gpu_base_bdev_removed compiled into the
 *     framework (-DDRAID_TEST_HOT_REMOVE_REDIRECT, the second binary of the
 *     Makefile) the array stays online, degraded, until one disk more than the
 *     level tolerates is removed.
 *
 * After every step the RAM disks are compared with the CPU oracle's P and Q over
 * the model, strip by strip.
 */
#include "raid_test_common.h"

#include <pthread.h>

#define NT 4

static uint64_t
rnd(uint64_t *s)
{
	uint64_t z = (*s += 0x9E3779B97F4A7C15ull);

	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

struct op {
	struct io_wait w;
	struct iovec iov[3];
	int iovcnt;
	uint8_t *buf, *expect;	/* reads: the model's bytes when the read was submitted */
	uint64_t off, blocks;
	bool write;
	int thread;
};

/* I/O buffers come out of one pinned arena per run. */
struct arena {
	uint8_t *base;
	size_t size, used;
};

static uint8_t *
arena_get(struct arena *ar, size_t bytes)
{
	uint8_t *p;

	bytes = (bytes + 4095) & ~(size_t)4095;
	CHECK(ar->used + bytes <= ar->size);
	p = ar->base + ar->used;
	ar->used += bytes;
	return p;
}

static void
op_prepare(struct array *a, struct arena *ar, struct op *o, uint64_t *rng)
{
	const uint64_t bytes = o->blocks * a->blocklen;
	const int pieces = 1 + (int)(rnd(rng) % 3);
	uint64_t pos = 0;
	int i;

	memset(&o->w, 0, sizeof(o->w));
	o->buf = arena_get(ar, bytes);
	o->expect = NULL;
	o->iovcnt = 0;
	for (i = 0; i < pieces && pos < bytes; i++) {
		uint64_t n = (i == pieces - 1) ? bytes - pos : (bytes / pieces) & ~(uint64_t)(a->blocklen - 1);

		if (n == 0) {
			n = bytes - pos;
		}
		o->iov[o->iovcnt].iov_base = o->buf + pos;
		o->iov[o->iovcnt].iov_len = n;
		pos += n;
		o->iovcnt++;
	}
	if (o->write) {
		orc_fill_splitmix(o->buf, bytes, rnd(rng));
	} else {
		memset(o->buf, 0xA5, bytes);
	}
}

/* Submits on the op's thread; the model moves at submit time. */
static void
op_submit(struct array *a, struct spdk_io_channel **tch, struct op *o)
{
	const uint64_t bytes = o->blocks * a->blocklen;

	stub_set_thread(o->thread);
	if (o->write) {
		memcpy(a->model + o->off * a->blocklen, o->buf, bytes);
	} else {
		o->expect = malloc(bytes);
		CHECK(o->expect != NULL);
		memcpy(o->expect, a->model + o->off * a->blocklen, bytes);
	}
	CHECK(stub_bdev_submit(a->bdev, tch[o->thread],
			       o->write ? SPDK_BDEV_IO_TYPE_WRITE : SPDK_BDEV_IO_TYPE_READ, o->iov,
			       o->iovcnt, o->off, o->blocks, io_done, &o->w) == 0);
}

static void
op_verify(struct array *a, struct op *o, bool expect_ok)
{
	CHECK(o->w.done);
	CHECK(o->w.success == expect_ok);
	if (!o->write && o->w.success &&
	    memcmp(o->buf, o->expect, o->blocks * a->blocklen) != 0) {
		uint64_t b, first = UINT64_MAX, nbad = 0, now = 0;

		for (b = 0; b < o->blocks; b++) {
			const uint8_t *got = o->buf + b * a->blocklen;

			if (memcmp(got, o->expect + b * a->blocklen, a->blocklen) != 0) {
				first = spdk_min(first, b);
				nbad++;
				/* is it what the volume holds by now (a later write overtook the read)? */
				now += memcmp(got, a->model + (o->off + b) * a->blocklen, a->blocklen) == 0;
			}
		}
		fprintf(stderr, "thread %d read [%" PRIu64 ", +%" PRIu64 ") differs from the model: %" PRIu64
			" blocks, first at +%" PRIu64 " (stripe %" PRIu64 ", data chunk %" PRIu64 " on disk %d); %"
			PRIu64 " of them hold what was written later\n", o->thread, o->off, o->blocks, nbad,
			first, (o->off + first) / a->stripe_blocks,
			(o->off + first) % a->stripe_blocks / a->strip_blocks,
			data_disk(a, (o->off + first) / a->stripe_blocks,
				  (int)((o->off + first) % a->stripe_blocks / a->strip_blocks)), now);
		CHECK(!"read data differs");
	}
	free(o->expect);
	o->expect = NULL;
}

/* A request on one of the first `hot` stripes. */
static void
op_random(struct array *a, struct op *o, int hot, uint64_t *rng)
{
	const uint64_t s = rnd(rng) % (uint64_t)hot, st = a->strip_blocks, sb = a->stripe_blocks;
	const unsigned kind = (unsigned)(rnd(rng) % 100);
	uint64_t in, n;

	if (kind < 10) {		/* full stripe */
		o->write = true;
		in = 0;
		n = sb;
	} else if (kind < 45) {		/* inside one strip, or over a strip boundary: RMW */
		o->write = true;
		in = rnd(rng) % (sb - 1);
		n = 1 + rnd(rng) % st;
	} else if (kind < 60) {		/* most of a stripe: RCW */
		o->write = true;
		in = rnd(rng) % st;
		n = st * (uint64_t)(a->k / 2 + 1) + rnd(rng) % st;
	} else {
		o->write = false;
		in = rnd(rng) % sb;
		n = 1 + rnd(rng) % (kind < 70 ? sb + st : 2 * st);	/* some cross into the next stripe */
	}
	o->off = s * sb + in;
	if (kind < 60 && in + n > sb) {
		n = sb - in;		/* writes stay inside their stripe */
	}
	if (o->off + n > a->stripes * sb) {
		n = a->stripes * sb - o->off;
	}
	o->blocks = n;
}

/* Steps every thread, in an order and with a weight that change from iteration
 * to iteration, until every op is done. */
static void
poll_all(struct op *ops, int nops, struct array *a, int kill_disk, int kill_at)
{
	struct timespec t0, t;
	int it, i, all = 0;

	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (it = 0; !all; it++) {
		if (kill_disk >= 0 && it == kill_at) {
			stub_set_dead(a->base[kill_disk], true);
		}
		for (i = 0; i < NT; i++) {
			const int t_id = (i * 3 + it) % NT;	/* 3 and NT are coprime */
			int times = 1 + ((it + t_id) % 3 == 0);

			while (times--) {
				stub_poll_thread(t_id);
			}
		}
		all = 1;
		for (i = 0; i < nops; i++) {
			all &= ops[i].w.done;
		}
		clock_gettime(CLOCK_MONOTONIC, &t);
		CHECK((t.tv_sec - t0.tv_sec) < 60);
	}
}

static uint64_t
cross_thread_msgs(bool reset)
{
	struct stub_thread_stats st;
	uint64_t n = 0;
	int t;

	for (t = 0; t < NT; t++) {
		stub_thread_stats(t, &st, reset);
		n += st.msgs_from_other_threads;
	}
	return n;
}

static void
get_channels(struct array *a, struct spdk_io_channel **tch)
{
	int t;

	tch[0] = a->ch;		/* array_create took thread 0's */
	for (t = 1; t < NT; t++) {
		stub_set_thread(t);
		tch[t] = spdk_get_io_channel(a->raid);
		CHECK(tch[t] != NULL && tch[t] != tch[0]);
	}
	stub_set_thread(0);
}

static void
put_channels(struct spdk_io_channel **tch)
{
	int t, i;

	for (i = 0; i < 4; i++) {
		stub_poll_threads();
	}
	for (t = 1; t < NT; t++) {
		stub_set_thread(t);
		spdk_put_io_channel(tch[t]);
	}
	stub_set_thread(0);
}

/* ------------------------------------------------------------ 1. interleaved */

static void
run_interleaved(void)
{
	enum { NOPS = 28 * NT, HOT = 5 };
	struct array a;
	struct spdk_io_channel *tch[NT];
	struct arena ar;
	struct op *ops = calloc(NOPS, sizeof(*ops));
	struct raid_gpu_stats st;
	uint64_t rng = 0x7EA1;
	int round, i;
	/* per round: disks lost from the start; a disk that dies in flight (-1: none) */
	const struct { uint32_t lost; int kill; } plan[] = {
		{ 0, -1 }, { 0, -1 }, { 1u << 2, -1 }, { 0, 6 }, { (1u << 0) | (1u << 9), -1 },
		{ 1u << 5, 8 }, { 0, -1 },
	};

	stub_set_thread(0);
	array_create(&a, 6, 10, 64, 4096, 16);
	get_channels(&a, tch);
	ar.size = (size_t)NOPS * (a.stripe_blocks + 2 * a.strip_blocks) * a.blocklen;
	ar.base = dma(ar.size);
	CHECK(ops != NULL);
	cross_thread_msgs(true);

	snprintf(g_case, sizeof(g_case), "interleaved: fill");
	do_write(&a, 0, a.stripes * a.stripe_blocks, 3, true);
	check_array(&a, 0);

	for (round = 0; round < (int)SPDK_COUNTOF(plan); round++) {
		uint32_t lost = plan[round].lost;

		snprintf(g_case, sizeof(g_case), "interleaved round %d: lost 0x%x, disk %d dies in flight",
			 round, lost, plan[round].kill);
		stub_set_thread(0);
		set_lost(&a, lost);
		ar.used = 0;
		for (i = 0; i < NOPS; i++) {
			ops[i].thread = (int)(rnd(&rng) % NT);
			op_random(&a, &ops[i], HOT, &rng);
			op_prepare(&a, &ar, &ops[i], &rng);
		}
		for (i = 0; i < NOPS; i++) {
			op_submit(&a, tch, &ops[i]);
			if (i % 9 == 8) {
				stub_poll_thread(i % NT);	/* some progress while submitting */
			}
		}
		poll_all(ops, NOPS, &a, plan[round].kill, 2);
		for (i = 0; i < NOPS; i++) {
			op_verify(&a, &ops[i], true);
		}
		stub_set_thread(0);
		if (plan[round].kill >= 0) {
			/* the module found the dead disk by itself */
			CHECK(a.raid->base_bdev_info[plan[round].kill].degraded);
			lost |= 1u << plan[round].kill;
		}
		check_array(&a, lost);
		if (lost) {
			/* no rebuild in the reference: a healthy rewrite resyncs the disks */
			set_lost(&a, 0);
			do_write(&a, 0, a.stripes * a.stripe_blocks, 3, true);
			check_array(&a, 0);
		}
	}

	/* A disk that dies with a read on it in flight, for certain (in the rounds above it
	 * depends on how far the requests have come when the disk goes): base I/O completes
	 * at the next poll of its thread, so a read submitted now, and a disk that dies
	 * before that poll, fails in flight; the module marks the disk degraded, redoes the
	 * request as a degraded read and completes it with the right bytes. */
	snprintf(g_case, sizeof(g_case), "a read in flight when its disk dies");
	{
		struct op o;
		uint64_t before;
		const int victim = data_disk(&a, 2, 1);

		memset(&o, 0, sizeof(o));
		ar.used = 0;
		o.thread = 1;
		o.write = false;
		o.off = 2 * a.stripe_blocks;
		o.blocks = a.stripe_blocks;
		op_prepare(&a, &ar, &o, &rng);
		raid_gpu_get_stats(a.raid, &st);
		before = st.redone;
		op_submit(&a, tch, &o);
		stub_set_dead(a.base[victim], true);
		poll_all(&o, 1, &a, -1, 0);
		op_verify(&a, &o, true);
		stub_set_thread(0);
		CHECK(a.raid->base_bdev_info[victim].degraded);
		raid_gpu_get_stats(a.raid, &st);
		CHECK(st.redone > before);
		check_array(&a, 1u << victim);
		set_lost(&a, 0);
		do_write(&a, 0, a.stripes * a.stripe_blocks, 3, true);
		check_array(&a, 0);
	}

	raid_gpu_get_stats(a.raid, &st);
	printf("   interleaved: full %" PRIu64 " rmw %" PRIu64 " rcw %" PRIu64 " degraded-write %" PRIu64
	       " read %" PRIu64 " degraded-read %" PRIu64 " redone %" PRIu64 " | hand-offs %" PRIu64
	       ", cross-thread messages %" PRIu64 "\n", st.full_stripe_writes, st.rmw_writes,
	       st.rcw_writes, st.degraded_writes, st.reads, st.degraded_reads, st.redone, st.handoffs,
	       cross_thread_msgs(false));
	/* the stripe of a finished request went to a request of another thread */
	CHECK(st.handoffs > 0);
	CHECK(cross_thread_msgs(false) >= st.handoffs);
	CHECK(st.full_stripe_writes > 0 && st.rmw_writes > 0 && st.rcw_writes > 0 && st.reads > 0);
	CHECK(st.degraded_reads > 0 && st.degraded_writes > 0 && st.redone > 0);

	/* ---- 2. more requests per channel than it has stripe requests: order is then
	 * only kept per stripe queue, so every thread writes chunks of its own */
	snprintf(g_case, sizeof(g_case), "channel exhaustion on %d threads", NT);
	{
		enum { PER = 100 };
		struct op *big = calloc((size_t)PER * NT, sizeof(*big));
		int t, n = 0;

		CHECK(big != NULL);
		ar.used = 0;
		for (t = 0; t < NT; t++) {
			for (i = 0; i < PER; i++) {
				struct op *o = &big[n++];
				const uint64_t s = rnd(&rng) % a.stripes;
				const uint64_t c = (uint64_t)t + NT * (rnd(&rng) % (uint64_t)(a.k / NT));

				o->thread = t;
				o->write = i % 3 != 2;
				o->blocks = 1 + rnd(&rng) % a.strip_blocks;
				o->off = s * a.stripe_blocks + c * a.strip_blocks +
					 rnd(&rng) % (a.strip_blocks - o->blocks + 1);
				op_prepare(&a, &ar, o, &rng);
			}
		}
		/* thread by thread, so each channel runs out of stripe requests */
		for (i = 0; i < n; i++) {
			op_submit(&a, tch, &big[i]);
		}
		poll_all(big, n, &a, -1, 0);
		for (i = 0; i < n; i++) {
			op_verify(&a, &big[i], true);
		}
		free(big);
		stub_set_thread(0);
		check_array(&a, 0);
	}

	put_channels(tch);
	spdk_dma_free(ar.base);
	free(ops);
	snprintf(g_case, sizeof(g_case), "interleaved: teardown");
	array_destroy(&a);
	printf("ok interleaved: %d SPDK threads on one RAID6 8+2 x 64 KiB array\n", NT);
	fflush(stdout);
}

/* ------------------------------------------------------------ 3. OS threads */

struct worker {
	struct array *a;
	int id;
	uint64_t rng;
	double seconds;
	pthread_barrier_t *barrier;
	uint64_t ops_done, reads_checked;
	struct arena ar;
};

/* Thread w owns data chunks w, w + NT, ... of the shared stripes and the whole of
 * stripe `shared + w`. */
static void *
worker_main(void *arg)
{
	enum { BATCH = 24 };
	struct worker *w = arg;
	struct array *a = w->a;
	const uint64_t shared = a->stripes - NT, st = a->strip_blocks, sb = a->stripe_blocks;
	struct spdk_io_channel *tch[NT] = { NULL };
	struct op ops[BATCH];
	struct timespec t0, t;
	int i;

	stub_set_thread(w->id);
	tch[w->id] = spdk_get_io_channel(a->raid);
	CHECK(tch[w->id] != NULL);
	pthread_barrier_wait(w->barrier);
	clock_gettime(CLOCK_MONOTONIC, &t0);
	do {
		w->ar.used = 0;
		for (i = 0; i < BATCH; i++) {
			struct op *o = &ops[i];
			const unsigned kind = (unsigned)(rnd(&w->rng) % 100);

			o->thread = w->id;
			if (kind < 70) {
				/* one of this thread's chunks of a stripe every thread writes */
				const uint64_t s = rnd(&w->rng) % shared;
				const uint64_t c = (uint64_t)w->id + NT * (rnd(&w->rng) % (uint64_t)(a->k / NT));

				o->write = kind < 45;
				o->blocks = 1 + rnd(&w->rng) % st;
				o->off = s * sb + c * st + rnd(&w->rng) % (st - o->blocks + 1);
			} else {
				/* this thread's own stripe: full-stripe and RCW writes, wide reads */
				const uint64_t s = shared + (uint64_t)w->id;

				o->write = kind < 90;
				if (kind < 78) {
					o->off = s * sb;
					o->blocks = sb;
				} else {
					o->off = s * sb + rnd(&w->rng) % st;
					o->blocks = st * (uint64_t)(a->k / 2 + 1);
				}
			}
			op_prepare(a, &w->ar, o, &w->rng);
		}
		for (i = 0; i < BATCH; i++) {
			op_submit(a, tch, &ops[i]);
		}
		for (i = 0; i < BATCH; i++) {
			CHECK(stub_poll_self_until(&ops[i].w.done, 60.0));
		}
		for (i = 0; i < BATCH; i++) {
			w->reads_checked += !ops[i].write;
			op_verify(a, &ops[i], true);
		}
		w->ops_done += BATCH;
		clock_gettime(CLOCK_MONOTONIC, &t);
	} while ((t.tv_sec - t0.tv_sec) + (t.tv_nsec - t0.tv_nsec) * 1e-9 < w->seconds);
	for (i = 0; i < 4; i++) {
		stub_poll();
	}
	spdk_put_io_channel(tch[w->id]);
	return NULL;
}

static void
run_os_threads(uint32_t lost, int kill_disk, double seconds)
{
	struct array a;
	struct worker w[NT];
	pthread_t th[NT];
	pthread_barrier_t barrier;
	struct raid_gpu_stats st;
	uint64_t total = 0;
	int t;

	stub_set_thread(0);
	array_create(&a, 6, 10, 64, 4096, 12 + NT);
	snprintf(g_case, sizeof(g_case), "OS threads: lost 0x%x, disk %d dies in flight", lost, kill_disk);
	do_write(&a, 0, a.stripes * a.stripe_blocks, 3, true);
	check_array(&a, 0);
	set_lost(&a, lost);
	/* thread 0's channel from array_create is not used by a worker: worker 0 takes
	 * a second reference on its own OS thread */
	cross_thread_msgs(true);
	pthread_barrier_init(&barrier, NULL, NT + 1);
	for (t = 0; t < NT; t++) {
		memset(&w[t], 0, sizeof(w[t]));
		w[t].a = &a;
		w[t].id = t;
		w[t].rng = 0xC0FFEE + (uint64_t)t * 7919 + lost;
		w[t].seconds = seconds;
		w[t].barrier = &barrier;
		w[t].ar.size = (size_t)24 * (a.stripe_blocks + a.strip_blocks) * a.blocklen;
		w[t].ar.base = dma(w[t].ar.size);
		CHECK(pthread_create(&th[t], NULL, worker_main, &w[t]) == 0);
	}
	pthread_barrier_wait(&barrier);
	if (kill_disk >= 0) {
		usleep((useconds_t)(seconds * 0.3e6));
		stub_set_dead(a.base[kill_disk], true);
	}
	for (t = 0; t < NT; t++) {
		CHECK(pthread_join(th[t], NULL) == 0);
		total += w[t].ops_done;
		spdk_dma_free(w[t].ar.base);
	}
	pthread_barrier_destroy(&barrier);
	stub_set_thread(0);
	if (kill_disk >= 0) {
		CHECK(a.raid->base_bdev_info[kill_disk].degraded);
		lost |= 1u << kill_disk;
	}
	check_array(&a, lost);
	raid_gpu_get_stats(a.raid, &st);
	printf("   OS threads (lost 0x%x): %" PRIu64 " requests, hand-offs %" PRIu64
	       ", cross-thread messages %" PRIu64 ", redone %" PRIu64 ", %" PRIu64 " requests in %" PRIu64
	       " launches\n", lost, total, st.handoffs, cross_thread_msgs(false), st.redone,
	       st.gpu_requests, st.flushes);
	CHECK(total >= (uint64_t)24 * NT);
	CHECK(cross_thread_msgs(false) >= st.handoffs);
	set_lost(&a, 0);
	do_write(&a, 0, a.stripes * a.stripe_blocks, 3, true);
	check_array(&a, 0);
	snprintf(g_case, sizeof(g_case), "OS threads: teardown");
	array_destroy(&a);
	printf("ok OS threads: %d pthreads, one SPDK thread each, lost 0x%x\n", NT, lost);
	fflush(stdout);
}

/* ------------------------------------------------------------ 4. hot-remove */

struct user_events {
	int removed;
};

static void
user_event_cb(enum spdk_bdev_event_type type, struct spdk_bdev *bdev, void *ctx)
{
	struct user_events *ev = ctx;

	(void)bdev;
	if (type == SPDK_BDEV_EVENT_REMOVE) {
		ev->removed++;
	}
}

static bool
live_equal(const struct stub_live *x, const struct stub_live *y)
{
	return x->ios == y->ios && x->descs == y->descs && x->channels == y->channels &&
	       x->pollers == y->pollers && x->msgs == y->msgs && x->dma == y->dma &&
	       x->io_devices == y->io_devices;
}

/* Disjoint requests in flight on two threads: every data chunk is written or
 * read by at most one of them, so the outcome has one answer. */
static int
flight_prepare(struct array *a, struct arena *ar, struct op *ops, int max, uint64_t *rng)
{
	uint64_t s;
	int c, n = 0;

	ar->used = 0;
	for (s = 0; s < a->stripes && n < max; s++) {
		for (c = 0; c < a->k && n < max; c += 2) {
			struct op *o = &ops[n];

			o->thread = n % 2;
			o->write = n % 3 != 2;
			o->blocks = 1 + rnd(rng) % a->strip_blocks;
			o->off = s * a->stripe_blocks + (uint64_t)c * a->strip_blocks;
			if (n % 7 == 0) {
				o->blocks = 2 * a->strip_blocks;	/* two chunks */
			}
			op_prepare(a, ar, o, rng);
			n++;
		}
	}
	return n;
}

static void
run_hot_remove(void)
{
	enum { MAXOPS = 48 };
	struct array a;
	struct spdk_io_channel *tch[NT];
	struct spdk_bdev_desc *desc = NULL;
	struct user_events ev = { 0 };
	struct stub_live before, after;
	struct arena ar;
	struct op ops[MAXOPS];
	struct raid_bdev_config *cfg;
	char name[32];
	uint64_t rng = 0xD15C;
	uint32_t lost = 0;	/* disks whose contents no longer count */
	int removed = 0;	/* base bdevs hot-removed */
	uint8_t *buf;
	int i, n, done = 0;

	stub_set_thread(0);
	stub_poll_threads();	/* pollers unregistered earlier are freed by their thread's next poll */
	stub_live(&before);
	array_create(&a, 6, 10, 64, 4096, 8);
	cfg = a.cfg;
	snprintf(name, sizeof(name), "%s", a.bdev->name);
	/* a user of the raid bdev: an open descriptor, as bdevperf or a target holds */
	CHECK(spdk_bdev_open_ext(name, true, user_event_cb, &ev, &desc) == 0);
	get_channels(&a, tch);
	ar.size = (size_t)MAXOPS * 2 * a.strip_bytes;
	ar.base = dma(ar.size);
	buf = dma(a.stripes * a.stripe_blocks * a.blocklen);
	do_write(&a, 0, a.stripes * a.stripe_blocks, 3, true);
	check_array(&a, 0);

#ifdef DRAID_TEST_HOT_REMOVE_REDIRECT
	/* ---- with the redirect: removals the level tolerates leave the array online */
	{
		const int victims[2] = { 3, 7 };
		int v;

		for (v = 0; v < 2; v++) {
			snprintf(g_case, sizeof(g_case), "hot-remove of base %d with I/O in flight: stays online",
				 victims[v]);
			n = flight_prepare(&a, &ar, ops, MAXOPS, &rng);
			for (i = 0; i < n; i++) {
				op_submit(&a, tch, &ops[i]);
			}
			stub_poll_thread(0);
			stub_poll_thread(1);
			/* the device is gone and its users are told so */
			stub_set_dead(a.base[victims[v]], true);
			stub_hot_remove(a.base[victims[v]]);
			poll_all(ops, n, &a, -1, 0);
			for (i = 0; i < n; i++) {
				op_verify(&a, &ops[i], true);
			}
			stub_set_thread(0);
			lost |= 1u << victims[v];
			removed++;
			CHECK(a.raid->state == RAID_BDEV_STATE_ONLINE && ev.removed == 0);
			CHECK(a.raid->base_bdev_info[victims[v]].degraded && a.raid->degraded);
			CHECK(a.raid->base_bdev_info[victims[v]].remove_scheduled);
			check_array(&a, lost);
			/* and it serves I/O: everything reads back, writes keep parity */
			do_read(&a, 0, a.stripes * a.stripe_blocks, 4, true);
			do_write(&a, a.strip_blocks / 2, a.stripe_blocks * 2, 2, true);
			do_write(&a, 3 * a.stripe_blocks, a.stripe_blocks, 1, true);
			check_array(&a, lost);
		}
	}
	/* one more than RAID6 tolerates: the handler declines and the reference's path runs */
	snprintf(g_case, sizeof(g_case), "hot-remove of a third base bdev: offline");
	n = stub_error_count();
	stub_hot_remove(a.base[1]);	/* its bytes stay valid: nothing writes them any more */
	for (i = 0; i < 8; i++) {
		stub_poll_threads();
	}
	CHECK(stub_error_count() > n);
	removed++;
#else
	/* ---- the reference as it is: the array goes offline under the I/O */
	snprintf(g_case, sizeof(g_case), "hot-remove of base 3 with I/O in flight: offline");
	n = flight_prepare(&a, &ar, ops, MAXOPS, &rng);
	for (i = 0; i < n; i++) {
		op_submit(&a, tch, &ops[i]);
	}
	stub_poll_thread(0);
	stub_poll_thread(1);
	stub_set_dead(a.base[3], true);
	stub_hot_remove(a.base[3]);
	poll_all(ops, n, &a, -1, 0);
	/* requests that were in flight ran to the end (the lost disk's share is
	 * carried by parity): each completed once, none is torn */
	for (i = 0; i < n; i++) {
		op_verify(&a, &ops[i], true);
	}
	lost = 1u << 3;
	removed = 1;
	check_array(&a, lost);
#endif
	/* offline: the module was stopped, the user was told, new I/O fails at once */
	stub_set_thread(0);
	CHECK(a.raid->state == RAID_BDEV_STATE_OFFLINE);
	CHECK(a.raid->module_private == NULL);
	CHECK(ev.removed == 1);
	{
		struct raid_gpu_stats st;

		raid_gpu_get_stats(a.raid, &st);	/* safe on a stopped array: zeros */
		CHECK(st.reads == 0 && st.flushes == 0);
	}
	snprintf(g_case, sizeof(g_case), "I/O to the offline array fails cleanly");
	for (n = 0; n < 2; n++) {
		struct io_wait w = { 0, true };
		struct iovec iov = { buf, a.stripe_blocks * a.blocklen };

		stub_set_thread(n);
		CHECK(stub_bdev_submit(a.bdev, tch[n], n ? SPDK_BDEV_IO_TYPE_WRITE : SPDK_BDEV_IO_TYPE_READ,
				       &iov, 1, (uint64_t)n * a.stripe_blocks, a.stripe_blocks, io_done,
				       &w) == 0);
		CHECK(stub_poll_until(&w.done, 10.0));
		CHECK(!w.success);
	}
	stub_set_thread(0);
	check_array(&a, lost);		/* the failed write touched nothing */

	/* the user reacts to the remove event: channels back, descriptor closed; the
	 * framework then destructs the raid bdev and lets go of the removed base bdevs
	 * (raid_bdev_destruct, bdev_raid.c:285-323) */
	snprintf(g_case, sizeof(g_case), "teardown after hot-remove");
	put_channels(tch);
	spdk_put_io_channel(a.ch);
	spdk_bdev_close(desc);
	for (i = 0; i < 4; i++) {
		stub_poll_threads();
	}
	CHECK(cfg->raid_bdev != NULL && cfg->raid_bdev->destruct_called);
	CHECK(cfg->raid_bdev->num_base_bdevs_discovered == a.n - removed);
	raid_bdev_remove_base_devices(cfg, removed_cb, &done);
	for (i = 0; i < 4; i++) {
		stub_poll_threads();
	}
	CHECK(done == 1 && cfg->raid_bdev == NULL);	/* freed with its last base bdev */
	raid_bdev_config_cleanup(cfg);
	for (i = 0; i < a.n; i++) {
		stub_ram_bdev_destroy(a.base[i]);
	}
	spdk_dma_free(ar.base);
	spdk_dma_free(buf);
	free(a.model);
	stub_poll_threads();
	stub_live(&after);
	if (!live_equal(&before, &after)) {
		fprintf(stderr, "still allocated: ios %" PRId64 " descs %" PRId64 " channels %" PRId64
			" pollers %" PRId64 " msgs %" PRId64 " dma %" PRId64 " io_devices %" PRId64 "\n",
			after.ios - before.ios, after.descs - before.descs, after.channels - before.channels,
			after.pollers - before.pollers, after.msgs - before.msgs, after.dma - before.dma,
			after.io_devices - before.io_devices);
		CHECK(!"the runtime still holds something after the array is gone");
	}
#ifdef DRAID_TEST_HOT_REMOVE_REDIRECT
	printf("ok hot-remove with the redirect: online through two removals, offline at the third\n");
#else
	printf("ok hot-remove, reference behaviour: array offline, in-flight I/O finished, later I/O "
	       "failed, nothing left allocated\n");
#endif
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
	CHECK(stub_allocate_threads(NT) == 0);
	run_interleaved();
#ifndef DRAID_TEST_HOT_REMOVE_REDIRECT
	run_os_threads(0, -1, 0.6);
	run_os_threads(1u << 4, 7, 0.8);
#else
	(void)run_os_threads;
#endif
	run_hot_remove();
	printf("raid module on %d SPDK threads: %d array checks passed, %d errors logged (the expected "
	       "ones)\n", NT, g_checks, stub_error_count());
	return 0;
}
