/*
 * spdk_stub.c -- a stand-in for the parts of the SPDK runtime that
 * module/bdev/raid uses, so that the reference's raid framework (bdev_raid.c,
 * compiled from /root/reference where it lies) and a raid level module can be
 * linked and driven in a test process without libspdk / DPDK.
 *
 * It plays the role that DEFINE_STUB / MOCK_SET, test/common/lib/test_env.c and
 * ut_multithread.c play for the reference's own unit tests
 * (test/unit/lib/bdev/raid/bdev_raid.c/bdev_raid_ut.c:39-42,104-139), but does
 * real work where the I/O path needs it:
 *   - SPDK threads (test/common/lib/ut_multithread.c:78,200 allocate_threads /
 *     set_thread / poll_threads): up to STUB_MAX_THREADS of them, each with its own
 *     message ring, pollers, io_wait queue, base-bdev completions and io_channels;
 *     spdk_get_thread() is the current one.  They can be stepped round-robin from
 *     one OS thread (the ut_multithread way, deterministic interleaving) or each
 *     be run by an OS thread of its own (the message ring is the only structure
 *     another thread writes, and it is locked);
 *   - bdev registry, open/close/claim, remove events and the deferred destruct of
 *     spdk_bdev_unregister (lib/bdev/bdev.c:5850-5947: open descriptors are told
 *     SPDK_BDEV_EVENT_REMOVE on their own thread, the bdev is destructed when the
 *     last one closes), io_device + one io_channel per (device, thread);
 *   - RAM base bdevs whose reads and writes complete asynchronously, on the
 *     submitting thread, with -ENOMEM and I/O error injection; a no-copy mode
 *     (what module/bdev/null does) for measuring the layers above;
 *   - the bdev layer's submit path for the raid bdev: spdk_bdev_io allocation
 *     with the module's driver context, splitting at optimal_io_boundary with
 *     spdk_bdev_io_get_split_parent(), parent completion;
 *   - pollers, io_wait queues, mempools, DMA memory;
 *   - counts of what is still allocated (I/Os, descriptors, channels, pollers,
 *     messages, DMA blocks), for leak checks.
 * DMA memory (spdk_dma_malloc) comes from the GPU runtime's pinned allocator
 * (draid_ec_host_alloc): in a deployment SPDK's hugepage memory is registered with
 * the GPU once; the pool this runs on refuses hipHostRegister, and allocating
 * from the runtime gives the same result -- host buffers kernels can reach.
 *
 * Test infrastructure only.  Nothing here is part of the product.
 */
#include "spdk/stdinc.h"

#include "spdk/bdev_module.h"
#include "spdk/env.h"
#include "spdk/json.h"
#include "spdk/log.h"
#include "spdk/string.h"
#include "spdk/thread.h"
#include "spdk/util.h"

#include "draid_ec.h"
#include "spdk_stub.h"

/* ------------------------------------------------------------ logging */

static int g_log_level = 0;
static int g_error_count;

void stub_set_log_level(int level) { g_log_level = level; }
int stub_error_count(void) { return __atomic_load_n(&g_error_count, __ATOMIC_RELAXED); }

void
spdk_log(enum spdk_log_level level, const char *file, const int line, const char *func,
	 const char *format, ...)
{
	va_list ap;

	if (level == SPDK_LOG_ERROR) {
		__atomic_fetch_add(&g_error_count, 1, __ATOMIC_RELAXED);
	}
	if ((int)level > g_log_level) {
		return;
	}
	fprintf(stderr, "[spdk %s] %s:%d %s: ", level == SPDK_LOG_ERROR ? "ERROR" :
		level == SPDK_LOG_WARN ? "WARN" : "note", file ? file : "", line, func ? func : "");
	va_start(ap, format);
	vfprintf(stderr, format, ap);
	va_end(ap);
}

void spdk_log_register_flag(const char *name, struct spdk_log_flag *flag) { (void)name; (void)flag; }

const char *spdk_strerror(int errnum) { return strerror(errnum); }

uint32_t
spdk_u32log2(uint32_t x)
{
	return x == 0 ? 0 : 31u - (uint32_t)__builtin_clz(x);
}

/* ------------------------------------------------------------ json (unused output) */

int spdk_json_write_null(struct spdk_json_write_ctx *w) { (void)w; return 0; }
int spdk_json_write_string(struct spdk_json_write_ctx *w, const char *v) { (void)w; (void)v; return 0; }
int spdk_json_write_array_begin(struct spdk_json_write_ctx *w) { (void)w; return 0; }
int spdk_json_write_array_end(struct spdk_json_write_ctx *w) { (void)w; return 0; }
int spdk_json_write_object_begin(struct spdk_json_write_ctx *w) { (void)w; return 0; }
int spdk_json_write_object_end(struct spdk_json_write_ctx *w) { (void)w; return 0; }
int spdk_json_write_name(struct spdk_json_write_ctx *w, const char *n) { (void)w; (void)n; return 0; }
int spdk_json_write_named_uint32(struct spdk_json_write_ctx *w, const char *n, uint32_t v)
{ (void)w; (void)n; (void)v; return 0; }
int spdk_json_write_named_string(struct spdk_json_write_ctx *w, const char *n, const char *v)
{ (void)w; (void)n; (void)v; return 0; }
int spdk_json_write_named_array_begin(struct spdk_json_write_ctx *w, const char *n)
{ (void)w; (void)n; return 0; }
int spdk_json_write_named_object_begin(struct spdk_json_write_ctx *w, const char *n)
{ (void)w; (void)n; return 0; }

/* ------------------------------------------------------------ what is still allocated */

static struct stub_live g_live;

#define LIVE_ADD(field, d) __atomic_fetch_add(&g_live.field, (d), __ATOMIC_RELAXED)

void
stub_live(struct stub_live *out)
{
	out->ios = __atomic_load_n(&g_live.ios, __ATOMIC_RELAXED);
	out->descs = __atomic_load_n(&g_live.descs, __ATOMIC_RELAXED);
	out->channels = __atomic_load_n(&g_live.channels, __ATOMIC_RELAXED);
	out->pollers = __atomic_load_n(&g_live.pollers, __ATOMIC_RELAXED);
	out->msgs = __atomic_load_n(&g_live.msgs, __ATOMIC_RELAXED);
	out->dma = __atomic_load_n(&g_live.dma, __ATOMIC_RELAXED);
	out->io_devices = __atomic_load_n(&g_live.io_devices, __ATOMIC_RELAXED);
}

/* ------------------------------------------------------------ DMA memory, mempools */

static bool g_plain_dma;

void stub_set_plain_dma(bool plain) { g_plain_dma = plain; }

/* An allocation remembers which allocator made it (header in front of the
 * aligned block). */
struct dma_hdr {
	void *raw;
	uint64_t pinned;
};

void *
spdk_dma_malloc(size_t size, size_t align, uint64_t *phys_addr)
{
	const size_t a = align < 64 ? 64 : align;
	void *raw = NULL;
	uint8_t *p;
	struct dma_hdr *h;

	if (phys_addr) {
		*phys_addr = 0;
	}
	if (g_plain_dma) {
		raw = malloc(size + a + sizeof(*h));
	} else if (draid_ec_host_alloc(&raw, size + a + sizeof(*h)) != 0) {
		fprintf(stderr, "stub: draid_ec_host_alloc(%zu): %s\n", size, draid_ec_last_error());
		return NULL;
	}
	if (!raw) {
		return NULL;
	}
	p = (uint8_t *)(((uintptr_t)raw + sizeof(*h) + a - 1) & ~(uintptr_t)(a - 1));
	h = (struct dma_hdr *)p - 1;
	h->raw = raw;
	h->pinned = !g_plain_dma;
	LIVE_ADD(dma, 1);
	return p;
}

void *
spdk_dma_zmalloc(size_t size, size_t align, uint64_t *phys_addr)
{
	void *p = spdk_dma_malloc(size, align, phys_addr);

	if (p) {
		memset(p, 0, size);
	}
	return p;
}

void
spdk_dma_free(void *buf)
{
	struct dma_hdr *h;

	if (!buf) {
		return;
	}
	h = (struct dma_hdr *)buf - 1;
	LIVE_ADD(dma, -1);
	if (h->pinned) {
		draid_ec_host_free(h->raw);
	} else {
		free(h->raw);
	}
}

struct spdk_mempool {
	size_t count, ele_size, nfree;
	uint8_t *mem;
	void **free_list;
};

struct spdk_mempool *
spdk_mempool_create_ctor(const char *name, size_t count, size_t ele_size, size_t cache_size,
			 int socket_id, spdk_mempool_obj_cb_t *obj_init, void *obj_init_arg)
{
	struct spdk_mempool *mp = calloc(1, sizeof(*mp));
	size_t i;

	(void)name;
	(void)cache_size;
	(void)socket_id;
	if (!mp) {
		return NULL;
	}
	ele_size = (ele_size + 63) & ~(size_t)63;
	mp->count = count;
	mp->ele_size = ele_size;
	mp->mem = calloc(count, ele_size);
	mp->free_list = calloc(count, sizeof(void *));
	if (!mp->mem || !mp->free_list) {
		free(mp->mem);
		free(mp->free_list);
		free(mp);
		return NULL;
	}
	for (i = 0; i < count; i++) {
		void *obj = mp->mem + i * ele_size;

		if (obj_init) {
			obj_init(mp, obj_init_arg, obj, (unsigned)i);
		}
		mp->free_list[count - 1 - i] = obj;	/* get() hands out object 0 first */
	}
	mp->nfree = count;
	return mp;
}

struct spdk_mempool *
spdk_mempool_create(const char *name, size_t count, size_t ele_size, size_t cache_size, int socket_id)
{
	return spdk_mempool_create_ctor(name, count, ele_size, cache_size, socket_id, NULL, NULL);
}

void *
spdk_mempool_get(struct spdk_mempool *mp)
{
	return mp->nfree ? mp->free_list[--mp->nfree] : NULL;
}

void
spdk_mempool_put(struct spdk_mempool *mp, void *ele)
{
	assert(mp->nfree < mp->count);
	mp->free_list[mp->nfree++] = ele;
}

void
spdk_mempool_free(struct spdk_mempool *mp)
{
	if (mp) {
		free(mp->mem);
		free(mp->free_list);
		free(mp);
	}
}

/* ------------------------------------------------------------ threads, messages, pollers */

struct stub_msg {
	spdk_msg_fn fn;
	void *ctx;
	TAILQ_ENTRY(stub_msg) link;
};

struct spdk_poller {
	spdk_poller_fn fn;
	void *arg;
	bool dead;
	struct spdk_thread *thread;
	TAILQ_ENTRY(spdk_poller) link;
};

/* One SPDK thread (lib/thread/thread.c:972 spdk_thread_poll drains the same
 * things in the same order: messages, then pollers).  Only `msgs` is touched by
 * other threads. */
struct spdk_thread {
	int id;
	pthread_mutex_t lock;
	TAILQ_HEAD(, stub_msg) msgs;
	TAILQ_HEAD(, spdk_poller) pollers;
	TAILQ_HEAD(, spdk_bdev_io) completions;		/* base bdev I/O submitted here */
	TAILQ_HEAD(, spdk_bdev_io_wait_entry) io_wait;
	struct stub_thread_stats stats;
};

static struct spdk_thread g_threads[STUB_MAX_THREADS];
static int g_nthreads = 1;
static __thread struct spdk_thread *t_thread;

__attribute__((constructor)) static void
stub_threads_init(void)
{
	int i;

	for (i = 0; i < STUB_MAX_THREADS; i++) {
		struct spdk_thread *t = &g_threads[i];

		t->id = i;
		pthread_mutex_init(&t->lock, NULL);
		TAILQ_INIT(&t->msgs);
		TAILQ_INIT(&t->pollers);
		TAILQ_INIT(&t->completions);
		TAILQ_INIT(&t->io_wait);
	}
}

struct spdk_thread *spdk_get_thread(void) { return t_thread ? t_thread : &g_threads[0]; }

int
stub_allocate_threads(int num_threads)
{
	if (num_threads < 1 || num_threads > STUB_MAX_THREADS) {
		return -EINVAL;
	}
	g_nthreads = num_threads;
	return 0;
}

int stub_num_threads(void) { return g_nthreads; }

void
stub_set_thread(int id)
{
	assert(id >= 0 && id < g_nthreads);
	t_thread = &g_threads[id];
}

int stub_thread_id(const struct spdk_thread *thread) { return thread->id; }

void
stub_thread_stats(int id, struct stub_thread_stats *out, bool reset)
{
	struct spdk_thread *t = &g_threads[id];

	pthread_mutex_lock(&t->lock);
	if (out) {
		*out = t->stats;
	}
	if (reset) {
		memset(&t->stats, 0, sizeof(t->stats));
	}
	pthread_mutex_unlock(&t->lock);
}

int
spdk_thread_send_msg(const struct spdk_thread *thread, spdk_msg_fn fn, void *ctx)
{
	struct spdk_thread *t = (struct spdk_thread *)thread;
	struct stub_msg *m = calloc(1, sizeof(*m));

	if (!m) {
		return -ENOMEM;
	}
	m->fn = fn;
	m->ctx = ctx;
	LIVE_ADD(msgs, 1);
	pthread_mutex_lock(&t->lock);
	TAILQ_INSERT_TAIL(&t->msgs, m, link);
	t->stats.msgs++;
	if (t != spdk_get_thread()) {
		t->stats.msgs_from_other_threads++;
	}
	pthread_mutex_unlock(&t->lock);
	return 0;
}

struct spdk_poller *
spdk_poller_register_named(spdk_poller_fn fn, void *arg, uint64_t period_microseconds,
			   const char *name)
{
	struct spdk_poller *p = calloc(1, sizeof(*p));

	(void)period_microseconds;
	(void)name;
	if (!p) {
		return NULL;
	}
	p->fn = fn;
	p->arg = arg;
	p->thread = spdk_get_thread();
	TAILQ_INSERT_TAIL(&p->thread->pollers, p, link);
	LIVE_ADD(pollers, 1);
	return p;
}

struct spdk_poller *
spdk_poller_register(spdk_poller_fn fn, void *arg, uint64_t period_microseconds)
{
	return spdk_poller_register_named(fn, arg, period_microseconds, NULL);
}

void
spdk_poller_unregister(struct spdk_poller **ppoller)
{
	if (ppoller && *ppoller) {
		/* only its own thread may touch a poller (lib/thread/thread.c:1607-1628) */
		if ((*ppoller)->thread != spdk_get_thread()) {
			fprintf(stderr, "stub: poller of thread %d unregistered from thread %d\n",
				(*ppoller)->thread->id, spdk_get_thread()->id);
			abort();
		}
		(*ppoller)->dead = true;	/* freed by that thread's poll, which may be iterating */
		*ppoller = NULL;
	}
}

/* ------------------------------------------------------------ io devices and channels */

struct io_device {
	void *io_device;
	spdk_io_channel_create_cb create_cb;
	spdk_io_channel_destroy_cb destroy_cb;
	spdk_io_device_unregister_cb unregister_cb;
	uint32_t ctx_size;
	struct spdk_io_channel *ch[STUB_MAX_THREADS];	/* one per thread */
	int nch;
	bool unregistered;
	TAILQ_ENTRY(io_device) link;
};
static TAILQ_HEAD(, io_device) g_io_devices = TAILQ_HEAD_INITIALIZER(g_io_devices);
static pthread_mutex_t g_io_devices_lock = PTHREAD_MUTEX_INITIALIZER;

struct spdk_io_channel {
	struct io_device *dev;
	struct spdk_thread *thread;
	int ref;
};
SPDK_STATIC_ASSERT(sizeof(struct spdk_io_channel) <= SPDK_IO_CHANNEL_STRUCT_SIZE,
		   "io channel header too large");

static struct io_device *
io_device_find(void *io_device)
{
	struct io_device *d;

	pthread_mutex_lock(&g_io_devices_lock);
	TAILQ_FOREACH(d, &g_io_devices, link) {
		if (d->io_device == io_device && !d->unregistered) {
			break;
		}
	}
	pthread_mutex_unlock(&g_io_devices_lock);
	return d;
}

void
spdk_io_device_register(void *io_device, spdk_io_channel_create_cb create_cb,
			spdk_io_channel_destroy_cb destroy_cb, uint32_t ctx_size, const char *name)
{
	struct io_device *d = calloc(1, sizeof(*d));

	(void)name;
	assert(d != NULL);
	d->io_device = io_device;
	d->create_cb = create_cb;
	d->destroy_cb = destroy_cb;
	d->ctx_size = ctx_size;
	pthread_mutex_lock(&g_io_devices_lock);
	TAILQ_INSERT_TAIL(&g_io_devices, d, link);
	pthread_mutex_unlock(&g_io_devices_lock);
	LIVE_ADD(io_devices, 1);
}

/* The device goes away once it is unregistered and its last channel is released
 * (lib/thread/thread.c:2029-2095); its unregister callback runs then. */
static void
io_device_release(struct io_device *d)
{
	bool gone;

	pthread_mutex_lock(&g_io_devices_lock);
	gone = d->unregistered && d->nch == 0;
	if (gone) {
		TAILQ_REMOVE(&g_io_devices, d, link);
	}
	pthread_mutex_unlock(&g_io_devices_lock);
	if (gone) {
		if (d->unregister_cb) {
			d->unregister_cb(d->io_device);
		}
		free(d);
		LIVE_ADD(io_devices, -1);
	}
}

void
spdk_io_device_unregister(void *io_device, spdk_io_device_unregister_cb unregister_cb)
{
	struct io_device *d = io_device_find(io_device);

	if (!d) {
		return;
	}
	d->unregister_cb = unregister_cb;
	d->unregistered = true;
	io_device_release(d);
}

struct spdk_io_channel *
spdk_get_io_channel(void *io_device)
{
	struct io_device *d = io_device_find(io_device);
	struct spdk_thread *t = spdk_get_thread();
	struct spdk_io_channel *ch;

	if (!d) {
		return NULL;
	}
	if (d->ch[t->id]) {
		d->ch[t->id]->ref++;
		return d->ch[t->id];
	}
	ch = calloc(1, SPDK_IO_CHANNEL_STRUCT_SIZE + d->ctx_size);
	if (!ch) {
		return NULL;
	}
	ch->dev = d;
	ch->thread = t;
	ch->ref = 1;
	if (d->create_cb(io_device, spdk_io_channel_get_ctx(ch)) != 0) {
		free(ch);
		return NULL;
	}
	d->ch[t->id] = ch;
	__atomic_fetch_add(&d->nch, 1, __ATOMIC_RELAXED);
	LIVE_ADD(channels, 1);
	return ch;
}

void
spdk_put_io_channel(struct spdk_io_channel *ch)
{
	struct io_device *d = ch->dev;

	/* a channel belongs to the thread that got it (lib/thread/thread.c:2250-2267) */
	if (ch->thread != spdk_get_thread()) {
		fprintf(stderr, "stub: channel of thread %d released from thread %d\n", ch->thread->id,
			spdk_get_thread()->id);
		abort();
	}
	assert(ch->ref > 0);
	if (--ch->ref > 0) {
		return;
	}
	d->destroy_cb(d->io_device, spdk_io_channel_get_ctx(ch));
	d->ch[ch->thread->id] = NULL;
	pthread_mutex_lock(&g_io_devices_lock);
	d->nch--;
	pthread_mutex_unlock(&g_io_devices_lock);
	free(ch);
	LIVE_ADD(channels, -1);
	io_device_release(d);
}

struct spdk_io_channel *
spdk_io_channel_from_ctx(void *ctx)
{
	return (struct spdk_io_channel *)((uint8_t *)ctx - SPDK_IO_CHANNEL_STRUCT_SIZE);
}

struct spdk_thread *spdk_io_channel_get_thread(struct spdk_io_channel *ch) { return ch->thread; }

/* ------------------------------------------------------------ bdev registry */

struct spdk_bdev_desc {
	struct spdk_bdev *bdev;
	spdk_bdev_event_cb_t event_cb;
	void *event_ctx;
	struct spdk_thread *thread;	/* the opener's: remove events are delivered there */
	int refs;			/* remove notifications in flight */
	bool closed;
	TAILQ_ENTRY(spdk_bdev_desc) link;
};

static TAILQ_HEAD(, spdk_bdev) g_bdevs = TAILQ_HEAD_INITIALIZER(g_bdevs);
static TAILQ_HEAD(, spdk_bdev_module) g_modules = TAILQ_HEAD_INITIALIZER(g_modules);

void
spdk_bdev_module_list_add(struct spdk_bdev_module *bdev_module)
{
	TAILQ_INSERT_TAIL(&g_modules, bdev_module, internal.tailq);
}

void spdk_bdev_module_examine_done(struct spdk_bdev_module *module) { (void)module; }

struct spdk_bdev *
stub_bdev_by_name(const char *name)
{
	struct spdk_bdev *b;

	TAILQ_FOREACH(b, &g_bdevs, internal.link) {
		if (strcmp(b->name, name) == 0) {
			return b;
		}
	}
	return NULL;
}

struct spdk_bdev *spdk_bdev_get_by_name(const char *name) { return stub_bdev_by_name(name); }

int
spdk_bdev_register(struct spdk_bdev *bdev)
{
	if (!bdev->name || stub_bdev_by_name(bdev->name)) {
		return -EEXIST;
	}
	TAILQ_INIT(&bdev->internal.open_descs);
	bdev->internal.claim_module = NULL;
	bdev->internal.status = SPDK_BDEV_STATUS_READY;
	bdev->internal.unregister_cb = NULL;
	TAILQ_INSERT_TAIL(&g_bdevs, bdev, internal.link);
	return 0;
}

/* bdev_fini (lib/bdev/bdev.c:5826-5847): destruct, then the unregister callback. */
static void
bdev_fini(struct spdk_bdev *bdev)
{
	spdk_bdev_unregister_cb cb = bdev->internal.unregister_cb;
	void *ctx = bdev->internal.unregister_ctx;
	int rc = 0;

	if (bdev->fn_table && bdev->fn_table->destruct) {
		rc = bdev->fn_table->destruct(bdev->ctxt);	/* may free the bdev */
	}
	if (cb) {
		cb(ctx, rc);
	}
}

static void
remove_notify(void *arg)
{
	struct spdk_bdev_desc *desc = arg;

	desc->refs--;
	if (!desc->closed) {
		desc->event_cb(SPDK_BDEV_EVENT_REMOVE, desc->bdev, desc->event_ctx);
	} else if (desc->refs == 0) {
		free(desc);
		LIVE_ADD(descs, -1);
	}
}

static int
notify_open_descs(struct spdk_bdev *bdev)
{
	struct spdk_bdev_desc *desc;
	int n = 0;

	TAILQ_FOREACH(desc, &bdev->internal.open_descs, link) {
		if (desc->event_cb) {
			desc->refs++;
			spdk_thread_send_msg(desc->thread, remove_notify, desc);
		}
		n++;
	}
	return n;
}

/* spdk_bdev_unregister (lib/bdev/bdev.c:5850-5947): every open descriptor gets
 * SPDK_BDEV_EVENT_REMOVE as a message on its own thread; the bdev is destructed
 * when the last of them closes (at once if none is open). */
void
spdk_bdev_unregister(struct spdk_bdev *bdev, spdk_bdev_unregister_cb cb_fn, void *cb_arg)
{
	if (bdev->internal.status == SPDK_BDEV_STATUS_REMOVING) {
		if (cb_fn) {
			cb_fn(cb_arg, -EBUSY);
		}
		return;
	}
	bdev->internal.status = SPDK_BDEV_STATUS_REMOVING;
	bdev->internal.unregister_cb = cb_fn;
	bdev->internal.unregister_ctx = cb_arg;
	TAILQ_REMOVE(&g_bdevs, bdev, internal.link);	/* no new opens by name */
	if (notify_open_descs(bdev) == 0) {
		bdev_fini(bdev);
	}
}

int
spdk_bdev_open_ext(const char *bdev_name, bool write, spdk_bdev_event_cb_t event_cb, void *event_ctx,
		   struct spdk_bdev_desc **_desc)
{
	struct spdk_bdev *bdev = stub_bdev_by_name(bdev_name);
	struct spdk_bdev_desc *desc;

	(void)write;
	if (!bdev) {
		return -ENODEV;
	}
	desc = calloc(1, sizeof(*desc));
	if (!desc) {
		return -ENOMEM;
	}
	desc->bdev = bdev;
	desc->event_cb = event_cb;
	desc->event_ctx = event_ctx;
	desc->thread = spdk_get_thread();
	TAILQ_INSERT_TAIL(&bdev->internal.open_descs, desc, link);
	LIVE_ADD(descs, 1);
	*_desc = desc;
	return 0;
}

void
spdk_bdev_close(struct spdk_bdev_desc *desc)
{
	struct spdk_bdev *bdev = desc->bdev;

	/* lib/bdev/bdev.c:6092: a descriptor is closed on the thread that opened it */
	if (desc->thread != spdk_get_thread()) {
		fprintf(stderr, "stub: descriptor of thread %d closed from thread %d\n", desc->thread->id,
			spdk_get_thread()->id);
		abort();
	}
	TAILQ_REMOVE(&bdev->internal.open_descs, desc, link);
	desc->closed = true;
	if (desc->refs == 0) {
		free(desc);
		LIVE_ADD(descs, -1);
	}
	if (bdev->internal.status == SPDK_BDEV_STATUS_REMOVING &&
	    TAILQ_EMPTY(&bdev->internal.open_descs)) {
		bdev_fini(bdev);
	}
}

struct spdk_bdev *spdk_bdev_desc_get_bdev(struct spdk_bdev_desc *desc) { return desc->bdev; }

int
spdk_bdev_module_claim_bdev(struct spdk_bdev *bdev, struct spdk_bdev_desc *desc,
			    struct spdk_bdev_module *module)
{
	(void)desc;
	if (bdev->internal.claim_module) {
		return -EPERM;
	}
	bdev->internal.claim_module = module;
	return 0;
}

void spdk_bdev_module_release_bdev(struct spdk_bdev *bdev) { bdev->internal.claim_module = NULL; }

size_t spdk_bdev_get_buf_align(const struct spdk_bdev *bdev) { return (size_t)1 << bdev->required_alignment; }

/* A base bdev is pulled out from under its users: what spdk_bdev_unregister of
 * that bdev does to them (the event only; the RAM disk itself stays until
 * stub_ram_bdev_destroy, I/O to it fails once the test marks it dead). */
void
stub_hot_remove(struct spdk_bdev *bdev)
{
	notify_open_descs(bdev);
}

/* ------------------------------------------------------------ RAM base bdevs */

struct ram_bdev {
	struct spdk_bdev bdev;
	uint8_t *data;
	int fail_next, enomem_next;	/* atomics: any thread submits and completes */
	bool dead;
	bool null_io;			/* complete without moving data (module/bdev/null) */
	struct stub_bdev_stats stats;
};

#define RAM_STAT(r, field, d) __atomic_fetch_add(&(r)->stats.field, (d), __ATOMIC_RELAXED)

/* Takes one from a countdown of injected faults; false when none is left. */
static bool
take_one(int *counter)
{
	int v = __atomic_load_n(counter, __ATOMIC_RELAXED);

	while (v > 0) {
		if (__atomic_compare_exchange_n(counter, &v, v - 1, false, __ATOMIC_RELAXED,
						__ATOMIC_RELAXED)) {
			return true;
		}
	}
	return false;
}

static struct spdk_bdev_module g_ram_module = { .name = "stub_ram" };

static int ram_channel_create(void *io_device, void *ctx_buf) { (void)io_device; (void)ctx_buf; return 0; }
static void ram_channel_destroy(void *io_device, void *ctx_buf) { (void)io_device; (void)ctx_buf; }

static bool
ram_io_type_supported(void *ctx, enum spdk_bdev_io_type io_type)
{
	(void)ctx;
	return io_type == SPDK_BDEV_IO_TYPE_READ || io_type == SPDK_BDEV_IO_TYPE_WRITE ||
	       io_type == SPDK_BDEV_IO_TYPE_RESET || io_type == SPDK_BDEV_IO_TYPE_FLUSH ||
	       io_type == SPDK_BDEV_IO_TYPE_UNMAP;
}

static struct spdk_io_channel *ram_get_io_channel(void *ctx) { return spdk_get_io_channel(ctx); }

static const struct spdk_bdev_fn_table g_ram_fn_table = {
	.io_type_supported = ram_io_type_supported,
	.get_io_channel = ram_get_io_channel,
};

static struct ram_bdev *
ram_of(struct spdk_bdev *bdev)
{
	assert(bdev->module == &g_ram_module);
	return SPDK_CONTAINEROF(bdev, struct ram_bdev, bdev);
}

struct spdk_bdev *
stub_ram_bdev_create(const char *name, uint64_t blockcnt, uint32_t blocklen)
{
	struct ram_bdev *r = calloc(1, sizeof(*r));

	if (!r) {
		return NULL;
	}
	r->data = calloc(blockcnt, blocklen);
	r->bdev.name = strdup(name);
	r->bdev.product_name = "stub ram disk";
	r->bdev.blocklen = blocklen;
	r->bdev.blockcnt = blockcnt;
	r->bdev.ctxt = r;
	r->bdev.module = &g_ram_module;
	r->bdev.fn_table = &g_ram_fn_table;
	if (!r->data || !r->bdev.name || spdk_bdev_register(&r->bdev) != 0) {
		free(r->data);
		free(r->bdev.name);
		free(r);
		return NULL;
	}
	spdk_io_device_register(r, ram_channel_create, ram_channel_destroy, 0, name);
	return &r->bdev;
}

void
stub_ram_bdev_destroy(struct spdk_bdev *bdev)
{
	struct ram_bdev *r = ram_of(bdev);

	TAILQ_REMOVE(&g_bdevs, bdev, internal.link);
	spdk_io_device_unregister(r, NULL);
	free(r->data);
	free(r->bdev.name);
	free(r);
}

uint8_t *stub_ram_bdev_data(struct spdk_bdev *bdev) { return ram_of(bdev)->data; }
void stub_inject_io_error(struct spdk_bdev *bdev, int count)
{ __atomic_store_n(&ram_of(bdev)->fail_next, count, __ATOMIC_RELAXED); }
void stub_inject_enomem(struct spdk_bdev *bdev, int count)
{ __atomic_store_n(&ram_of(bdev)->enomem_next, count, __ATOMIC_RELAXED); }
void stub_set_dead(struct spdk_bdev *bdev, bool dead)
{ __atomic_store_n(&ram_of(bdev)->dead, dead, __ATOMIC_RELAXED); }
void stub_set_null_io(struct spdk_bdev *bdev, bool null_io) { ram_of(bdev)->null_io = null_io; }

void
stub_ram_bdev_stats(struct spdk_bdev *bdev, struct stub_bdev_stats *out, bool reset)
{
	struct ram_bdev *r = ram_of(bdev);

	if (out) {
		*out = r->stats;
	}
	if (reset) {
		memset(&r->stats, 0, sizeof(r->stats));
	}
}

struct spdk_io_channel *
spdk_bdev_get_io_channel(struct spdk_bdev_desc *desc)
{
	return desc->bdev->fn_table->get_io_channel(desc->bdev->ctxt);
}

bool
spdk_bdev_io_type_supported(struct spdk_bdev *bdev, enum spdk_bdev_io_type io_type)
{
	return bdev->fn_table->io_type_supported(bdev->ctxt, io_type);
}

/* ------------------------------------------------------------ base bdev I/O */

void
spdk_bdev_free_io(struct spdk_bdev_io *bdev_io)
{
	free(bdev_io);
	LIVE_ADD(ios, -1);
}

/* I/O goes through the submitting thread's own channel (include/spdk/bdev.h: "ch
 * must be a channel of the calling thread"). */
static void
check_channel_thread(const struct spdk_io_channel *ch, const char *what)
{
	if (ch && ch->thread != spdk_get_thread()) {
		fprintf(stderr, "stub: %s on thread %d through a channel of thread %d\n", what,
			spdk_get_thread()->id, ch->thread->id);
		abort();
	}
}

static int
ram_submit(struct spdk_bdev_desc *desc, struct spdk_io_channel *ch, enum spdk_bdev_io_type type,
	   struct iovec *iov, int iovcnt, uint64_t offset_blocks, uint64_t num_blocks,
	   spdk_bdev_io_completion_cb cb, void *cb_arg)
{
	struct ram_bdev *r = ram_of(desc->bdev);
	struct spdk_bdev_io *io;

	check_channel_thread(ch, "base bdev I/O");
	if (take_one(&r->enomem_next)) {
		RAM_STAT(r, enomem, 1);
		return -ENOMEM;
	}
	if (type != SPDK_BDEV_IO_TYPE_RESET && offset_blocks + num_blocks > r->bdev.blockcnt) {
		return -EINVAL;
	}
	io = calloc(1, sizeof(*io));
	if (!io) {
		return -ENOMEM;
	}
	io->bdev = &r->bdev;
	io->type = type;
	io->u.bdev.iovs = iov;
	io->u.bdev.iovcnt = iovcnt;
	io->u.bdev.offset_blocks = offset_blocks;
	io->u.bdev.num_blocks = num_blocks;
	io->internal.cb = cb;
	io->internal.caller_ctx = cb_arg;
	io->internal.desc = desc;
	LIVE_ADD(ios, 1);
	TAILQ_INSERT_TAIL(&spdk_get_thread()->completions, io, internal.link);
	return 0;
}

int
spdk_bdev_readv_blocks(struct spdk_bdev_desc *desc, struct spdk_io_channel *ch, struct iovec *iov,
		       int iovcnt, uint64_t offset_blocks, uint64_t num_blocks,
		       spdk_bdev_io_completion_cb cb, void *cb_arg)
{
	return ram_submit(desc, ch, SPDK_BDEV_IO_TYPE_READ, iov, iovcnt, offset_blocks, num_blocks, cb,
			  cb_arg);
}

int
spdk_bdev_writev_blocks(struct spdk_bdev_desc *desc, struct spdk_io_channel *ch, struct iovec *iov,
			int iovcnt, uint64_t offset_blocks, uint64_t num_blocks,
			spdk_bdev_io_completion_cb cb, void *cb_arg)
{
	return ram_submit(desc, ch, SPDK_BDEV_IO_TYPE_WRITE, iov, iovcnt, offset_blocks, num_blocks, cb,
			  cb_arg);
}

int
spdk_bdev_reset(struct spdk_bdev_desc *desc, struct spdk_io_channel *ch, spdk_bdev_io_completion_cb cb,
		void *cb_arg)
{
	return ram_submit(desc, ch, SPDK_BDEV_IO_TYPE_RESET, NULL, 0, 0, 0, cb, cb_arg);
}

int
spdk_bdev_queue_io_wait(struct spdk_bdev *bdev, struct spdk_io_channel *ch,
			struct spdk_bdev_io_wait_entry *entry)
{
	(void)bdev;
	check_channel_thread(ch, "io_wait");
	TAILQ_INSERT_TAIL(&spdk_get_thread()->io_wait, entry, link);
	return 0;
}

/* The data moves when the I/O completes, so a caller that reuses a buffer too
 * early, or reads one before completion, shows. */
static void
ram_complete(struct spdk_bdev_io *io)
{
	struct ram_bdev *r = ram_of(io->bdev);
	bool ok = true;
	int i;

	if (__atomic_load_n(&r->dead, __ATOMIC_RELAXED)) {
		ok = false;
	} else if (io->type != SPDK_BDEV_IO_TYPE_RESET && take_one(&r->fail_next)) {
		ok = false;
	}
	if (ok && (io->type == SPDK_BDEV_IO_TYPE_READ || io->type == SPDK_BDEV_IO_TYPE_WRITE)) {
		uint8_t *p = r->data + io->u.bdev.offset_blocks * r->bdev.blocklen;
		uint64_t left = io->u.bdev.num_blocks * r->bdev.blocklen;

		for (i = 0; i < io->u.bdev.iovcnt && left && !r->null_io; i++) {
			const uint64_t n = spdk_min(left, (uint64_t)io->u.bdev.iovs[i].iov_len);

			if (io->type == SPDK_BDEV_IO_TYPE_READ) {
				memcpy(io->u.bdev.iovs[i].iov_base, p, n);
			} else {
				memcpy(p, io->u.bdev.iovs[i].iov_base, n);
			}
			p += n;
			left -= n;
		}
		if (left && !r->null_io) {
			ok = false;	/* iovecs shorter than the block range */
		}
		if (io->type == SPDK_BDEV_IO_TYPE_READ) {
			RAM_STAT(r, reads, 1);
			RAM_STAT(r, read_blocks, io->u.bdev.num_blocks);
		} else {
			RAM_STAT(r, writes, 1);
			RAM_STAT(r, write_blocks, io->u.bdev.num_blocks);
		}
	}
	if (!ok) {
		RAM_STAT(r, failed, 1);
	}
	io->internal.cb(io, ok, io->internal.caller_ctx);
}

/* ------------------------------------------------------------ the bdev layer above a raid bdev */

static int
module_ctx_size(struct spdk_bdev *bdev)
{
	return bdev->module && bdev->module->get_ctx_size ? bdev->module->get_ctx_size() : 0;
}

static void
user_complete(struct spdk_bdev_io *io, bool success)
{
	io->internal.cb(io, success, io->internal.caller_ctx);
}

/* Completion of a child of a split I/O (lib/bdev/bdev.c bdev_io_split_done). */
static void
stub_split_done(struct spdk_bdev_io *child, bool success, void *cb_arg)
{
	struct spdk_bdev_io *parent = cb_arg;

	spdk_bdev_free_io(child);
	if (!success) {
		parent->internal.status = SPDK_BDEV_IO_STATUS_FAILED;
	}
	assert(parent->u.bdev.split_outstanding > 0);
	if (--parent->u.bdev.split_outstanding == 0 && parent->u.bdev.split_remaining_num_blocks == 0) {
		user_complete(parent, parent->internal.status == SPDK_BDEV_IO_STATUS_SUCCESS);
	}
}

struct spdk_bdev_io *
spdk_bdev_io_get_split_parent(struct spdk_bdev_io *bdev_io)
{
	return bdev_io->internal.cb == stub_split_done ? bdev_io->internal.caller_ctx : NULL;
}

void
spdk_bdev_io_complete(struct spdk_bdev_io *bdev_io, enum spdk_bdev_io_status status)
{
	bdev_io->internal.status = (int8_t)status;
	bdev_io->internal.cb(bdev_io, status == SPDK_BDEV_IO_STATUS_SUCCESS, bdev_io->internal.caller_ctx);
}

void
spdk_bdev_io_get_buf(struct spdk_bdev_io *bdev_io, spdk_bdev_io_get_buf_cb cb, uint64_t len)
{
	(void)len;
	/* reads always arrive with buffers here */
	cb((struct spdk_io_channel *)bdev_io->internal.ch, bdev_io,
	   bdev_io->u.bdev.iovs && bdev_io->u.bdev.iovs[0].iov_base);
}

static struct spdk_bdev_io *
alloc_io(struct spdk_bdev *bdev, struct spdk_io_channel *ch, enum spdk_bdev_io_type type,
	 uint64_t offset_blocks, uint64_t num_blocks)
{
	struct spdk_bdev_io *io = calloc(1, sizeof(*io) + (size_t)module_ctx_size(bdev));

	if (io) {
		LIVE_ADD(ios, 1);
		io->bdev = bdev;
		io->type = type;
		io->u.bdev.offset_blocks = offset_blocks;
		io->u.bdev.num_blocks = num_blocks;
		io->internal.ch = (struct spdk_bdev_channel *)ch;
		io->internal.status = SPDK_BDEV_IO_STATUS_SUCCESS;
	}
	return io;
}

int
stub_bdev_submit(struct spdk_bdev *bdev, struct spdk_io_channel *ch, enum spdk_bdev_io_type type,
		 struct iovec *iov, int iovcnt, uint64_t offset_blocks, uint64_t num_blocks,
		 spdk_bdev_io_completion_cb cb, void *cb_arg)
{
	struct spdk_bdev_io *parent;
	const uint64_t boundary = bdev->optimal_io_boundary;
	uint64_t off = offset_blocks, left = num_blocks, consumed = 0;

	check_channel_thread(ch, "raid bdev I/O");
	if (offset_blocks + num_blocks > bdev->blockcnt || num_blocks == 0) {
		return -EINVAL;
	}
	parent = alloc_io(bdev, ch, type, offset_blocks, num_blocks);
	if (!parent) {
		return -ENOMEM;
	}
	parent->u.bdev.iovs = iov;
	parent->u.bdev.iovcnt = iovcnt;
	parent->internal.cb = cb;
	parent->internal.caller_ctx = cb_arg;
	if (!bdev->split_on_optimal_io_boundary || boundary == 0 ||
	    offset_blocks / boundary == (offset_blocks + num_blocks - 1) / boundary) {
		bdev->fn_table->submit_request(ch, parent);
		return 0;
	}
	/* bdev_io_should_split / _bdev_rw_split (lib/bdev/bdev.c:2596-2622,2223):
	 * children end at each boundary; their iovecs are slices of the parent's */
	parent->u.bdev.split_remaining_num_blocks = num_blocks;
	parent->u.bdev.split_outstanding = 1;	/* held while children are being submitted */
	while (left > 0) {
		const uint64_t n = spdk_min(left, boundary - off % boundary);
		struct spdk_bdev_io *child = alloc_io(bdev, ch, type, off, n);
		uint64_t skip = consumed * bdev->blocklen, want = n * bdev->blocklen;
		int i, c = 0;

		assert(child != NULL);
		for (i = 0; i < iovcnt && want; i++) {
			if (skip >= iov[i].iov_len) {
				skip -= iov[i].iov_len;
				continue;
			}
			assert(c < BDEV_IO_NUM_CHILD_IOV);
			child->child_iov[c].iov_base = (uint8_t *)iov[i].iov_base + skip;
			child->child_iov[c].iov_len = spdk_min(want, (uint64_t)iov[i].iov_len - skip);
			want -= child->child_iov[c].iov_len;
			skip = 0;
			c++;
		}
		assert(want == 0);
		child->u.bdev.iovs = child->child_iov;
		child->u.bdev.iovcnt = c;
		child->internal.cb = stub_split_done;
		child->internal.caller_ctx = parent;
		parent->u.bdev.split_outstanding++;
		parent->u.bdev.split_remaining_num_blocks -= n;
		off += n;
		left -= n;
		consumed += n;
		bdev->fn_table->submit_request(ch, child);
	}
	if (--parent->u.bdev.split_outstanding == 0) {
		user_complete(parent, parent->internal.status == SPDK_BDEV_IO_STATUS_SUCCESS);
	}
	return 0;
}

/* ------------------------------------------------------------ the reactor */

/* One iteration of the current thread: messages, io_wait retries, base bdev
 * completions, pollers (spdk_thread_poll, lib/thread/thread.c:910-1010). */
int
stub_poll(void)
{
	struct spdk_thread *t = spdk_get_thread();
	int ran = 0;
	struct stub_msg *m;
	struct spdk_bdev_io *io;
	struct spdk_poller *p, *ptmp;
	TAILQ_HEAD(, stub_msg) msgs = TAILQ_HEAD_INITIALIZER(msgs);
	TAILQ_HEAD(, spdk_bdev_io_wait_entry) waits = TAILQ_HEAD_INITIALIZER(waits);
	TAILQ_HEAD(, spdk_bdev_io) done = TAILQ_HEAD_INITIALIZER(done);
	struct spdk_bdev_io_wait_entry *w;

	/* messages sent while these run wait for the next iteration */
	pthread_mutex_lock(&t->lock);
	TAILQ_SWAP(&msgs, &t->msgs, stub_msg, link);
	pthread_mutex_unlock(&t->lock);
	while ((m = TAILQ_FIRST(&msgs)) != NULL) {
		TAILQ_REMOVE(&msgs, m, link);
		m->fn(m->ctx);
		free(m);
		LIVE_ADD(msgs, -1);
		ran++;
	}
	TAILQ_SWAP(&waits, &t->io_wait, spdk_bdev_io_wait_entry, link);
	while ((w = TAILQ_FIRST(&waits)) != NULL) {
		TAILQ_REMOVE(&waits, w, link);
		w->cb_fn(w->cb_arg);
		ran++;
	}
	TAILQ_SWAP(&done, &t->completions, spdk_bdev_io, internal.link);
	while ((io = TAILQ_FIRST(&done)) != NULL) {
		TAILQ_REMOVE(&done, io, internal.link);
		ram_complete(io);
		ran++;
	}
	TAILQ_FOREACH_SAFE(p, &t->pollers, link, ptmp) {
		if (!p->dead && p->fn(p->arg) > 0) {
			ran++;
		}
	}
	TAILQ_FOREACH_SAFE(p, &t->pollers, link, ptmp) {
		if (p->dead) {
			TAILQ_REMOVE(&t->pollers, p, link);
			free(p);
			LIVE_ADD(pollers, -1);
		}
	}
	return ran;
}

int
stub_poll_thread(int id)
{
	struct spdk_thread *saved = t_thread;
	int ran;

	stub_set_thread(id);
	ran = stub_poll();
	t_thread = saved;
	return ran;
}

int
stub_poll_threads(void)
{
	int i, ran = 0;

	for (i = 0; i < g_nthreads; i++) {
		ran += stub_poll_thread(i);
	}
	return ran;
}

static bool
poll_until(volatile int *done, double seconds, bool all_threads)
{
	struct timespec t0, t;

	clock_gettime(CLOCK_MONOTONIC, &t0);
	while (!*done) {
		if (all_threads) {
			stub_poll_threads();
		} else {
			stub_poll();
		}
		clock_gettime(CLOCK_MONOTONIC, &t);
		if ((t.tv_sec - t0.tv_sec) + (t.tv_nsec - t0.tv_nsec) * 1e-9 > seconds) {
			return false;
		}
	}
	return true;
}

bool stub_poll_until(volatile int *done, double seconds) { return poll_until(done, seconds, true); }
bool stub_poll_self_until(volatile int *done, double seconds) { return poll_until(done, seconds, false); }
