/*
 * raid_test_common.h -- what the raid module harnesses share: an array of RAM
 * base bdevs created through the reference framework's own entry points
 * (raid_bdev_config_add / raid_bdev_create / raid_bdev_add_base_devices,
 * bdev_raid.c:785-878,1042-1111,1520-1542), a byte model of the volume, volume
 * I/O helpers, and the checker that compares every strip on the RAM disks with
 * the CPU oracle's parity over the model.  Included once per test program.
 */
#ifndef DRAID_TEST_RAID_COMMON_H
#define DRAID_TEST_RAID_COMMON_H

#include "spdk/stdinc.h"

#include "bdev_raid.h"
#include "spdk/bdev_module.h"
#include "spdk/env.h"
#include "spdk/thread.h"
#include "spdk/util.h"

#include "draid_ec.h"
#include "raid_gpu.h"
#include "spdk_stub.h"
#include "../../oracle/isal_oracle.h"

#define CHECK(cond)                                                                          \
	do {                                                                                 \
		if (!(cond)) {                                                               \
			fprintf(stderr, "FAIL %s:%d: %s  [%s]\n", __FILE__, __LINE__, #cond, g_case); \
			fflush(stderr);                                                      \
			exit(1);                                                             \
		}                                                                            \
	} while (0)

static char g_case[256] = "";
static int g_checks;

struct array {
	int level, n, m, k;
	uint32_t blocklen, strip_blocks;
	uint64_t base_blocks, stripes, stripe_blocks, strip_bytes;
	struct spdk_bdev *base[32];
	struct raid_bdev_config *cfg;
	struct raid_bdev *raid;
	struct spdk_bdev *bdev;
	struct spdk_io_channel *ch;
	uint8_t *model;		/* the volume's expected bytes */
	uint64_t seed;
};

/* ---- layout, restated independently of the module (raid5.c:1006-1007,172-179;
 * RAID6: Q on the disk after P) */
static int parity_disk(const struct array *a, uint64_t s) { return (a->n - 1) - (int)(s % (uint64_t)a->n); }
static int q_disk(const struct array *a, uint64_t s) { return a->m == 2 ? (parity_disk(a, s) + 1) % a->n : -1; }
__attribute__((unused)) static int
data_disk(const struct array *a, uint64_t s, int d)
{
	const int p = parity_disk(a, s), q = q_disk(a, s);
	int disk, idx = 0;

	for (disk = 0; disk < a->n; disk++) {
		if (disk == p || disk == q) {
			continue;
		}
		if (idx++ == d) {
			return disk;
		}
	}
	return -1;
}

__attribute__((unused)) static uint8_t *
disk_strip(const struct array *a, int disk, uint64_t s)
{
	return stub_ram_bdev_data(a->base[disk]) + s * a->strip_bytes;
}

/* ---- I/O helpers */

struct io_wait {
	volatile int done;
	bool success;
};

__attribute__((unused)) static void
io_done(struct spdk_bdev_io *bdev_io, bool success, void *cb_arg)
{
	struct io_wait *w = cb_arg;

	w->success = success;
	w->done = 1;
	spdk_bdev_free_io(bdev_io);
}

__attribute__((unused)) static void
fill(uint8_t *buf, size_t len, uint64_t *seed)
{
	orc_fill_splitmix(buf, len, (*seed)++);
}

/* Volume I/O of [off, off+blocks) through up to `pieces` iovecs; waits. */
__attribute__((unused)) static bool
volume_io(struct array *a, enum spdk_bdev_io_type type, uint64_t off, uint64_t blocks, uint8_t *buf,
	  int pieces)
{
	struct iovec iov[8];
	struct io_wait w = { 0, false };
	const uint64_t bytes = blocks * a->blocklen;
	int i, cnt = 0;
	uint64_t pos = 0;

	if (pieces > 8) {
		pieces = 8;
	}
	for (i = 0; i < pieces && pos < bytes; i++) {
		uint64_t n = (i == pieces - 1) ? bytes - pos : (bytes / pieces) & ~(uint64_t)(a->blocklen - 1);

		if (n == 0) {
			n = bytes - pos;
		}
		iov[cnt].iov_base = buf + pos;
		iov[cnt].iov_len = n;
		pos += n;
		cnt++;
	}
	CHECK(stub_bdev_submit(a->bdev, a->ch, type, iov, cnt, off, blocks, io_done, &w) == 0);
	CHECK(stub_poll_until(&w.done, 30.0));
	return w.success;
}

__attribute__((unused)) static uint8_t *
dma(size_t bytes)
{
	uint8_t *p = spdk_dma_zmalloc(bytes, 4096, NULL);

	CHECK(p != NULL);
	return p;
}

/* ---- the checker */

/* Every surviving disk against the model; lost disks (mask) must be what the
 * oracle recovers from the survivors. */
__attribute__((unused)) static void
check_array(struct array *a, uint32_t lost)
{
	const size_t sb = a->strip_bytes;
	uint8_t *want[34], *scratch = malloc((size_t)(a->k + 2) * sb);
	uint64_t s;
	int j;

	CHECK(scratch != NULL);
	for (s = 0; s < a->stripes; s++) {
		void *vec[34];
		int fail[2], nfail = 0;

		for (j = 0; j < a->k; j++) {
			want[j] = a->model + (s * a->k + j) * sb;
			vec[j] = want[j];
		}
		want[a->k] = scratch + (size_t)a->k * sb;
		want[a->k + 1] = scratch + (size_t)(a->k + 1) * sb;
		vec[a->k] = want[a->k];
		vec[a->k + 1] = want[a->k + 1];
		if (a->m == 2) {
			CHECK(orc_pq_gen(a->k + 2, (int)sb, vec) == 0);
		} else {
			CHECK(orc_xor_gen(a->k + 1, (int)sb, vec) == 0);
		}
		for (j = 0; j < a->k + a->m; j++) {
			const int disk = j < a->k ? data_disk(a, s, j) : j == a->k ? parity_disk(a, s) : q_disk(a, s);

			if (lost & (1u << disk)) {
				fail[nfail++] = j;
				continue;
			}
			if (memcmp(disk_strip(a, disk, s), want[j], sb) != 0) {
				fprintf(stderr, "stripe %" PRIu64 " strip %d (%s) on disk %d differs\n", s, j,
					j < a->k ? "data" : j == a->k ? "P" : "Q", disk);
				CHECK(!"array content differs from the oracle");
			}
		}
		if (nfail) {
			/* rebuild the lost strips from the DISKS' surviving bytes with the oracle */
			uint8_t *tmp = malloc((size_t)(a->k + a->m) * sb);
			void *dv[34];

			CHECK(tmp != NULL && nfail <= a->m);
			for (j = 0; j < a->k + a->m; j++) {
				const int disk = j < a->k ? data_disk(a, s, j) : j == a->k ? parity_disk(a, s) :
						 q_disk(a, s);

				dv[j] = tmp + (size_t)j * sb;
				if (!(lost & (1u << disk))) {
					memcpy(dv[j], disk_strip(a, disk, s), sb);
				} else {
					memset(dv[j], 0xEE, sb);
				}
			}
			CHECK(orc_recover(a->k, a->m, (int)sb, dv, nfail, fail) == 0);
			for (j = 0; j < nfail; j++) {
				CHECK(memcmp(dv[fail[j]], want[fail[j]], sb) == 0);
			}
			free(tmp);
		}
	}
	free(scratch);
	g_checks++;
}

__attribute__((unused)) static void
do_write(struct array *a, uint64_t off, uint64_t blocks, int pieces, bool expect_ok)
{
	uint8_t *buf = dma(blocks * a->blocklen);
	bool ok;

	fill(buf, blocks * a->blocklen, &a->seed);
	ok = volume_io(a, SPDK_BDEV_IO_TYPE_WRITE, off, blocks, buf, pieces);
	CHECK(ok == expect_ok);
	if (ok) {
		memcpy(a->model + off * a->blocklen, buf, blocks * a->blocklen);
	}
	spdk_dma_free(buf);
}

__attribute__((unused)) static void
do_read(struct array *a, uint64_t off, uint64_t blocks, int pieces, bool expect_ok)
{
	uint8_t *buf = dma(blocks * a->blocklen);
	bool ok;

	memset(buf, 0xA5, blocks * a->blocklen);
	ok = volume_io(a, SPDK_BDEV_IO_TYPE_READ, off, blocks, buf, pieces);
	CHECK(ok == expect_ok);
	if (ok && memcmp(buf, a->model + off * a->blocklen, blocks * a->blocklen) != 0) {
		fprintf(stderr, "read [%" PRIu64 ", +%" PRIu64 ") differs from the model\n", off, blocks);
		CHECK(!"read data differs");
	}
	spdk_dma_free(buf);
}

/* ---- array lifecycle through the reference's framework */

static int g_arrays;

__attribute__((unused)) static void
array_create(struct array *a, int level, int n, uint32_t strip_kb, uint32_t blocklen, uint64_t stripes)
{
	char name[32], base[32];
	int i;

	memset(a, 0, sizeof(*a));
	a->level = level;
	a->n = n;
	a->m = level == 6 ? 2 : 1;
	a->k = n - a->m;
	a->blocklen = blocklen;
	a->strip_blocks = strip_kb * 1024 / blocklen;
	a->strip_bytes = (uint64_t)strip_kb * 1024;
	a->stripes = stripes;
	a->base_blocks = stripes * a->strip_blocks + (a->strip_blocks > 1 ? a->strip_blocks / 2 : 0);
	a->stripe_blocks = (uint64_t)a->k * a->strip_blocks;
	a->seed = 0x1234 + (uint64_t)g_arrays * 1000;
	snprintf(name, sizeof(name), "raid%d_%d", level, g_arrays);
	CHECK(raid_bdev_config_add(name, strip_kb, (uint8_t)n, level == 6 ? RAID6 : RAID5, &a->cfg) == 0);
	for (i = 0; i < n; i++) {
		snprintf(base, sizeof(base), "base%d_%d", g_arrays, i);
		a->base[i] = stub_ram_bdev_create(base, a->base_blocks, blocklen);
		CHECK(a->base[i] != NULL);
		CHECK(raid_bdev_config_add_base_bdev(a->cfg, base, (uint8_t)i) == 0);
	}
	CHECK(raid_bdev_create(a->cfg) == 0);
	CHECK(raid_bdev_add_base_devices(a->cfg) == 0);
	a->raid = a->cfg->raid_bdev;
	CHECK(a->raid != NULL && a->raid->state == RAID_BDEV_STATE_ONLINE);
	a->bdev = stub_bdev_by_name(name);
	CHECK(a->bdev == &a->raid->bdev);
	/* raid5_ut.c:176-195's geometry expectations, for m parity strips */
	CHECK(a->bdev->blockcnt == a->stripes * a->stripe_blocks);
	CHECK(a->bdev->optimal_io_boundary == a->stripe_blocks);
	CHECK(a->raid->module->base_bdevs_max_degraded == a->m);
	a->ch = spdk_get_io_channel(a->raid);
	CHECK(a->ch != NULL);
	a->model = calloc(a->stripes * a->stripe_blocks, blocklen);
	CHECK(a->model != NULL);
	g_arrays++;
}

__attribute__((unused)) static void
removed_cb(void *ctx, int rc)
{
	*(int *)ctx = rc == 0 ? 1 : -1;
}

__attribute__((unused)) static void
array_destroy(struct array *a)
{
	int done = 0, i;

	for (i = 0; i < 4; i++) {
		stub_poll();	/* let the channel's poller see its lists empty */
	}
	spdk_put_io_channel(a->ch);
	raid_bdev_remove_base_devices(a->cfg, removed_cb, &done);
	CHECK(done == 1);
	raid_bdev_config_cleanup(a->cfg);
	for (i = 0; i < a->n; i++) {
		stub_ram_bdev_destroy(a->base[i]);
	}
	stub_poll();
	free(a->model);
}

__attribute__((unused)) static void
set_lost(struct array *a, uint32_t mask)
{
	int i;

	for (i = 0; i < a->n; i++) {
		const bool lost = (mask >> i) & 1;

		if (!lost) {
			CHECK(raid_gpu_set_degraded(a->raid, (uint8_t)i, false) == 0);
		}
		stub_set_dead(a->base[i], lost);
	}
	for (i = 0; i < a->n; i++) {
		if ((mask >> i) & 1) {
			CHECK(raid_gpu_set_degraded(a->raid, (uint8_t)i, true) == 0);
		}
	}
	CHECK(a->raid->degraded == (mask != 0));
}

#endif /* DRAID_TEST_RAID_COMMON_H */
