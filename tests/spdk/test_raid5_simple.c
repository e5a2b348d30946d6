/*
 * test_raid5_simple.c -- the reference's own RAID5 module calling the engine at its
 * own xor_gen call site.
 *
 * module/bdev/raid/raid5_simple.c is compiled UNMODIFIED from /root/reference,
 * with include/isa-l/include/raid.h in place of isa-l's header and
 * libdraid_isal.so in place of libisal, so raid5_xor_stripe
 * (raid5_simple.c:141-203) -> raid5_xor_gen -> xor_gen (raid5_simple.c:131-135,176)
 * runs on the MI355X.  It is driven through the reference's framework
 * (bdev_raid.c) over the SPDK runtime stand-in, with the flow of the reference's
 * parity known-answer test, test/unit/lib/bdev/raid/raid5.c/raid5_ut_ref.c:
 *   - data pattern: 0xFF fill with the 8-byte block index at the start of every
 *     block (:354-357);
 *   - a full-stripe write arrives as k strip-sized children of one parent I/O
 *     (the bdev layer splits at optimal_io_boundary = strip, :378-390);
 *   - expected parity: the bytewise XOR of the k data strips (:324-330,362-369),
 *     compared with memcmp (:393-397); data must land unchanged (:394);
 *   - reads over the request grid return the written data (:434-465);
 *   - non-full-stripe writes FAIL (:489-512).
 * Grid: n in {3,4,5}, blocklen in {512,4096}, strip in {1,4,128} KiB (:75-78).
 */
#include "spdk/stdinc.h"

#include "bdev_raid.h"
#include "spdk/bdev_module.h"
#include "spdk/env.h"
#include "spdk/thread.h"
#include "spdk/util.h"

#include "spdk_stub.h"

#define CHECK(cond)                                                                      \
	do {                                                                             \
		if (!(cond)) {                                                           \
			fprintf(stderr, "FAIL %s:%d: %s  [%s]\n", __FILE__, __LINE__, #cond, g_case); \
			exit(1);                                                         \
		}                                                                        \
	} while (0)

static char g_case[160];

struct io_wait {
	volatile int done;
	bool success;
};

static void
io_done(struct spdk_bdev_io *bdev_io, bool success, void *cb_arg)
{
	struct io_wait *w = cb_arg;

	w->success = success;
	w->done = 1;
	spdk_bdev_free_io(bdev_io);
}

static bool
volume_io(struct spdk_bdev *bdev, struct spdk_io_channel *ch, enum spdk_bdev_io_type type,
	  uint64_t off, uint64_t blocks, void *buf)
{
	struct iovec iov = { buf, blocks * bdev->blocklen };
	struct io_wait w = { 0, false };

	CHECK(stub_bdev_submit(bdev, ch, type, &iov, 1, off, blocks, io_done, &w) == 0);
	CHECK(stub_poll_until(&w.done, 30.0));
	return w.success;
}

static void
removed_cb(void *ctx, int rc)
{
	*(int *)ctx = rc == 0 ? 1 : -1;
}

static int g_arrays, g_parity_checks;

static void
run(int n, uint32_t blocklen, uint32_t strip_kb, uint64_t base_blocks)
{
	const uint32_t strip = strip_kb * 1024 / blocklen;
	const int k = n - 1;
	struct spdk_bdev *base[8], *bdev;
	struct raid_bdev_config *cfg;
	struct raid_bdev *raid;
	struct spdk_io_channel *ch;
	char name[32], bname[32];
	uint64_t stripe_blocks, total_stripes, s, block;
	size_t strip_bytes, stripe_bytes;
	uint8_t *src, *dst, *ref;
	int i, done = 0;

	if (strip == 0 || strip > base_blocks) {
		return;		/* raid5_ut_ref.c:101-105 drops these combinations */
	}
	snprintf(g_case, sizeof(g_case), "n=%d blocklen=%u strip=%uKiB", n, blocklen, strip_kb);
	snprintf(name, sizeof(name), "r5s_%d", g_arrays);
	CHECK(raid_bdev_config_add(name, strip_kb, (uint8_t)n, RAID5, &cfg) == 0);
	for (i = 0; i < n; i++) {
		snprintf(bname, sizeof(bname), "r5s_base%d_%d", g_arrays, i);
		base[i] = stub_ram_bdev_create(bname, base_blocks, blocklen);
		CHECK(base[i] != NULL);
		CHECK(raid_bdev_config_add_base_bdev(cfg, bname, (uint8_t)i) == 0);
	}
	g_arrays++;
	CHECK(raid_bdev_create(cfg) == 0);
	CHECK(raid_bdev_add_base_devices(cfg) == 0);
	raid = cfg->raid_bdev;
	CHECK(raid && raid->state == RAID_BDEV_STATE_ONLINE);
	bdev = &raid->bdev;
	stripe_blocks = (uint64_t)strip * k;
	total_stripes = base_blocks / strip;
	/* raid5_ut_ref.c:176-183 */
	CHECK(bdev->blockcnt == stripe_blocks * total_stripes);
	CHECK(bdev->optimal_io_boundary == strip);
	ch = spdk_get_io_channel(raid);
	CHECK(ch != NULL);

	strip_bytes = (size_t)strip * blocklen;
	stripe_bytes = strip_bytes * k;
	src = spdk_dma_malloc(stripe_bytes, 4096, NULL);
	dst = spdk_dma_malloc(stripe_bytes, 4096, NULL);
	ref = malloc(strip_bytes);
	CHECK(src && dst && ref);

	for (s = 0; s < spdk_min((uint64_t)n, total_stripes); s++) {
		const int pdisk = k - (int)(s % (uint64_t)n);	/* raid5_simple.c:125-129 */
		size_t b;
		int d, disk;

		/* raid5_ut_ref.c:354-357 */
		memset(src, 0xff, stripe_bytes);
		for (block = 0; block < stripe_blocks; block++) {
			*(uint64_t *)(src + block * blocklen) = block + s * 1000003u;
		}
		CHECK(volume_io(bdev, ch, SPDK_BDEV_IO_TYPE_WRITE, s * stripe_blocks, stripe_blocks, src));
		/* the known answer: XOR of the data strips (raid5_ut_ref.c:324-330,362-369) */
		memset(ref, 0, strip_bytes);
		for (d = 0; d < k; d++) {
			for (b = 0; b < strip_bytes; b++) {
				ref[b] ^= src[(size_t)d * strip_bytes + b];
			}
		}
		CHECK(memcmp(stub_ram_bdev_data(base[pdisk]) + s * strip_bytes, ref, strip_bytes) == 0);
		g_parity_checks++;
		for (d = 0, disk = 0; d < k; d++, disk++) {
			if (disk == pdisk) {
				disk++;
			}
			CHECK(memcmp(stub_ram_bdev_data(base[disk]) + s * strip_bytes,
				     src + (size_t)d * strip_bytes, strip_bytes) == 0);
		}
		/* reads (each child is at most a strip, raid5_simple.c:488): whole stripe and
		 * the grid's unaligned pieces */
		memset(dst, 0, stripe_bytes);
		CHECK(volume_io(bdev, ch, SPDK_BDEV_IO_TYPE_READ, s * stripe_blocks, stripe_blocks, dst));
		CHECK(memcmp(dst, src, stripe_bytes) == 0);
		if (strip > 1) {
			memset(dst, 0, stripe_bytes);
			CHECK(volume_io(bdev, ch, SPDK_BDEV_IO_TYPE_READ, s * stripe_blocks + strip - 1, 2,
					dst));
			CHECK(memcmp(dst, src + (size_t)(strip - 1) * blocklen, 2 * (size_t)blocklen) == 0);
		}
	}
	/* a non-full-stripe write fails (raid5_ut_ref.c:489-512).  Last, and only one:
	 * the reference module keeps the failed request as its "current stripe"
	 * (raid5_simple.c:371-395), so the channel is not usable for writes afterwards. */
	CHECK(!volume_io(bdev, ch, SPDK_BDEV_IO_TYPE_WRITE, 0, strip, src));

	spdk_dma_free(src);
	spdk_dma_free(dst);
	free(ref);
	spdk_put_io_channel(ch);
	raid_bdev_remove_base_devices(cfg, removed_cb, &done);
	CHECK(done == 1);
	raid_bdev_config_cleanup(cfg);
	for (i = 0; i < n; i++) {
		stub_ram_bdev_destroy(base[i]);
	}
	printf("ok raid5_simple %s\n", g_case);
	fflush(stdout);
}

int
main(void)
{
	const int ns[] = { 3, 4, 5 };
	const uint64_t blockcnts[] = { 1, 1024, 4096 };
	const uint32_t blocklens[] = { 512, 4096 };
	const uint32_t strips[] = { 1, 4, 128 };
	size_t a, b, c, d;

	for (a = 0; a < SPDK_COUNTOF(ns); a++) {
		for (b = 0; b < SPDK_COUNTOF(blockcnts); b++) {
			for (c = 0; c < SPDK_COUNTOF(blocklens); c++) {
				for (d = 0; d < SPDK_COUNTOF(strips); d++) {
					run(ns[a], blocklens[c], strips[d], blockcnts[b]);
				}
			}
		}
	}
	printf("raid5_simple.c on the engine: %d arrays, %d stripe parities equal the known answer\n",
	       g_arrays, g_parity_checks);
	return g_parity_checks > 0 ? 0 : 1;
}
