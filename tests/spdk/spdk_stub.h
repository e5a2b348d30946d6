/*
 * spdk_stub.h -- test-side controls of the SPDK runtime stand-in (spdk_stub.c)
 * that the raid module harnesses link instead of libspdk.
 */
#ifndef DRAID_TEST_SPDK_STUB_H
#define DRAID_TEST_SPDK_STUB_H

#include "spdk/bdev_module.h"

/* A RAM-backed base bdev ("malloc bdev"), registered under `name`. */
struct spdk_bdev *stub_ram_bdev_create(const char *name, uint64_t blockcnt, uint32_t blocklen);
void stub_ram_bdev_destroy(struct spdk_bdev *bdev);
uint8_t *stub_ram_bdev_data(struct spdk_bdev *bdev);

/* Fault injection: the next `count` I/Os completing on the bdev fail (no data is
 * transferred); the next `count` submissions return -ENOMEM. */
void stub_inject_io_error(struct spdk_bdev *bdev, int count);
void stub_inject_enomem(struct spdk_bdev *bdev, int count);
/* Every I/O of the bdev fails from now on (a dead disk) / works again. */
void stub_set_dead(struct spdk_bdev *bdev, bool dead);
/* Sends SPDK_BDEV_EVENT_REMOVE to every open descriptor of the bdev, each as a
 * message on the thread that opened it (delivered by that thread's next poll). */
void stub_hot_remove(struct spdk_bdev *bdev);
/* Reads and writes of the bdev complete without moving data, as on
 * module/bdev/null: what is left to measure is the code above the base bdevs. */
void stub_set_null_io(struct spdk_bdev *bdev, bool null_io);

struct stub_bdev_stats {
	uint64_t reads, writes, read_blocks, write_blocks, enomem, failed;
};
void stub_ram_bdev_stats(struct spdk_bdev *bdev, struct stub_bdev_stats *out, bool reset);

/* Submits one I/O to a registered (raid) bdev the way the bdev layer does:
 * allocates the spdk_bdev_io with the module's context behind it, splits at
 * optimal_io_boundary when the bdev asks for it, and calls
 * fn_table->submit_request for the I/O or each child.  cb runs when the whole
 * I/O has completed.  Returns 0 or -errno. */
int stub_bdev_submit(struct spdk_bdev *bdev, struct spdk_io_channel *ch, enum spdk_bdev_io_type type,
		     struct iovec *iov, int iovcnt, uint64_t offset_blocks, uint64_t num_blocks,
		     spdk_bdev_io_completion_cb cb, void *cb_arg);

struct spdk_bdev *stub_bdev_by_name(const char *name);

/* SPDK threads, in the manner of test/common/lib/ut_multithread.c
 * (allocate_threads / set_thread / poll_thread / poll_threads).  One thread
 * (id 0) exists from the start.  stub_set_thread() makes a thread current for
 * the calling OS thread: spdk_get_thread() returns it, channels, pollers and
 * descriptors created from then on belong to it.  One OS thread can step all
 * of them (deterministic interleaving), or each can be driven by an OS thread of
 * its own that calls stub_set_thread(id) once and then stub_poll(). */
#define STUB_MAX_THREADS 16
int stub_allocate_threads(int num_threads);
int stub_num_threads(void);
void stub_set_thread(int id);
int stub_thread_id(const struct spdk_thread *thread);

struct stub_thread_stats {
	uint64_t msgs;				/* messages sent to the thread */
	uint64_t msgs_from_other_threads;	/* ... by a thread other than itself */
};
void stub_thread_stats(int id, struct stub_thread_stats *out, bool reset);

/* One reactor iteration of the current thread: messages, io_wait retries, base
 * bdev completions, pollers.  Returns the number of things that ran. */
int stub_poll(void);
/* One iteration of thread `id` / of every thread in turn, from one OS thread. */
int stub_poll_thread(int id);
int stub_poll_threads(void);
/* Polls every thread in turn until `*done` is non-zero; false on time-out (seconds). */
bool stub_poll_until(volatile int *done, double seconds);
/* The same, polling only the current thread (for a thread run by its own OS thread). */
bool stub_poll_self_until(volatile int *done, double seconds);

/* What the runtime still holds: spdk_bdev_io's not yet freed, open descriptors,
 * io_channels, pollers, undelivered messages, DMA blocks, io_devices. */
struct stub_live {
	int64_t ios, descs, channels, pollers, msgs, dma, io_devices;
};
void stub_live(struct stub_live *out);

/* 0 errors only (default), 1 + warnings, 2 + notices, 3 everything. */
void stub_set_log_level(int level);
/* Errors logged so far (SPDK_ERRLOG calls). */
int stub_error_count(void);

/* DMA memory comes from the GPU runtime's pinned allocator by default (reachable
 * by kernels without registration); plain == true switches spdk_dma_malloc to
 * posix_memalign (pageable), to test how callers react to unreachable buffers. */
void stub_set_plain_dma(bool plain);

#endif /* DRAID_TEST_SPDK_STUB_H */
