/*
 * draid_stripe_cache.c -- the raid module's stripe cache and per-stripe request
 * queue (see draid_raid.h), restating raid5.c without SPDK / DPDK types:
 *   raid5_get_stripe       raid5.c:1088-1131  lookup or claim an entry, move it to
 *                                             the MRU end, take a reference
 *   raid5_reclaim_stripes  raid5.c:1057-1086  free unreferenced entries from the
 *                                             LRU end when no entry is free
 *   request queue          raid5.c:1047-1054  requests on one stripe run one at a
 *                          raid5.c:485-521    time, in arrival order
 * The reference keys an rte_hash by stripe index; here a chained table over a fixed
 * pool of entries.  Each entry owns slot i of a caller-allocated stripe region
 * (n strips of strip bytes per slot, stripe-major), so the whole cache can live in
 * HBM or registered host memory and be handed to the strided calls of draid_ec.h.
 * One cache-wide lock (the reference's active_stripes_lock; its per-stripe
 * requests_lock is folded into it: every critical section is a few pointer moves).
 */
#include "../../include/draid_raid.h"

#include <errno.h>
#include <pthread.h>
#include <stddef.h>
#include <stdlib.h>

struct entry {
    struct draid_stripe pub;
    uint32_t refs;
    int active;                       /* in the hash and on the LRU list */
    struct entry *lru_prev, *lru_next; /* active list: head = most recently used */
    struct entry *hash_next;
    struct entry *free_next;
    struct draid_stripe_waiter *qhead, *qtail;
};

struct draid_stripe_cache {
    pthread_mutex_t lock;
    uint32_t nslots, nbuckets, nactive;
    struct entry *entries;
    struct entry **buckets;
    struct entry *lru_head, *lru_tail, *free_list;
};

static struct entry *ent(struct draid_stripe *s)
{
    return (struct entry *)((char *)s - offsetof(struct entry, pub));
}

static uint32_t bucket_of(const struct draid_stripe_cache *c, uint64_t index)
{
    uint64_t z = index + 0x9e3779b97f4a7c15ull; /* splitmix64 finaliser */
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return (uint32_t)((z ^ (z >> 31)) & (c->nbuckets - 1));
}

static void lru_unlink(struct draid_stripe_cache *c, struct entry *e)
{
    if (e->lru_prev)
        e->lru_prev->lru_next = e->lru_next;
    else
        c->lru_head = e->lru_next;
    if (e->lru_next)
        e->lru_next->lru_prev = e->lru_prev;
    else
        c->lru_tail = e->lru_prev;
    e->lru_prev = e->lru_next = NULL;
}

static void lru_push_head(struct draid_stripe_cache *c, struct entry *e)
{
    e->lru_prev = NULL;
    e->lru_next = c->lru_head;
    if (c->lru_head)
        c->lru_head->lru_prev = e;
    else
        c->lru_tail = e;
    c->lru_head = e;
}

static void hash_remove(struct draid_stripe_cache *c, struct entry *e)
{
    struct entry **pp = &c->buckets[bucket_of(c, e->pub.index)];
    while (*pp && *pp != e)
        pp = &(*pp)->hash_next;
    if (*pp)
        *pp = e->hash_next;
    e->hash_next = NULL;
}

uint64_t draid_stripe_slot_bytes(uint32_t n, uint64_t strip_bytes)
{
    const uint64_t b = (uint64_t)n * strip_bytes;

    /* strips of 256 KiB and more put P and Q into different halves by themselves */
    return (strip_bytes <= (128u << 10) && (b % (512u << 10)) == 0) ? b + (16u << 10) : b;
}

int draid_stripe_cache_create(draid_stripe_cache **out, uint32_t nslots)
{
    if (!out || nslots == 0)
        return -EINVAL;
    struct draid_stripe_cache *c = calloc(1, sizeof(*c));
    if (!c)
        return -ENOMEM;
    c->nslots = nslots;
    c->nbuckets = 1;
    while (c->nbuckets < 2 * nslots)
        c->nbuckets <<= 1;
    c->entries = calloc(nslots, sizeof(*c->entries));
    c->buckets = calloc(c->nbuckets, sizeof(*c->buckets));
    if (!c->entries || !c->buckets || pthread_mutex_init(&c->lock, NULL)) {
        free(c->entries);
        free(c->buckets);
        free(c);
        return -ENOMEM;
    }
    for (uint32_t i = nslots; i-- > 0;) { /* free list in slot order */
        c->entries[i].pub.slot = i;
        c->entries[i].free_next = c->free_list;
        c->free_list = &c->entries[i];
    }
    *out = c;
    return 0;
}

void draid_stripe_cache_destroy(draid_stripe_cache *c)
{
    if (!c)
        return;
    pthread_mutex_destroy(&c->lock);
    free(c->entries);
    free(c->buckets);
    free(c);
}

/* raid5_reclaim_stripes: unreferenced entries from the LRU end to the free list,
 * up to nslots/8 of them (raid5.c:1063-1064,1080-1082).  Caller holds the lock. */
static int reclaim(struct draid_stripe_cache *c)
{
    const int to_reclaim = (int)(c->nslots / 8) - (int)c->nslots + (int)c->nactive;
    int reclaimed = 0;
    for (struct entry *e = c->lru_tail, *prev; e; e = prev) {
        prev = e->lru_prev;
        if (e->refs > 0)
            continue;
        lru_unlink(c, e);
        hash_remove(c, e);
        e->active = 0;
        c->nactive--;
        e->free_next = c->free_list;
        c->free_list = e;
        if (++reclaimed > to_reclaim)
            break;
    }
    return reclaimed;
}

struct draid_stripe *draid_stripe_get(draid_stripe_cache *c, uint64_t index)
{
    if (!c)
        return NULL;
    pthread_mutex_lock(&c->lock);
    struct entry *e = c->buckets[bucket_of(c, index)];
    while (e && e->pub.index != index)
        e = e->hash_next;
    if (e) {
        lru_unlink(c, e);
    } else {
        if (!c->free_list && reclaim(c) == 0) {
            pthread_mutex_unlock(&c->lock); /* every entry referenced: retry later */
            return NULL;
        }
        e = c->free_list;
        c->free_list = e->free_next;
        e->free_next = NULL;
        e->pub.index = index;
        e->qhead = e->qtail = NULL;
        const uint32_t b = bucket_of(c, index);
        e->hash_next = c->buckets[b];
        c->buckets[b] = e;
        e->active = 1;
        c->nactive++;
    }
    lru_push_head(c, e);
    e->refs++;
    pthread_mutex_unlock(&c->lock);
    return &e->pub;
}

void draid_stripe_put(draid_stripe_cache *c, struct draid_stripe *s)
{
    if (!c || !s)
        return;
    pthread_mutex_lock(&c->lock);
    struct entry *e = ent(s);
    if (e->refs)
        e->refs--;
    pthread_mutex_unlock(&c->lock);
}

int draid_stripe_enqueue(draid_stripe_cache *c, struct draid_stripe *s,
                         struct draid_stripe_waiter *w)
{
    if (!c || !s || !w)
        return -EINVAL;
    pthread_mutex_lock(&c->lock);
    struct entry *e = ent(s);
    const int head = e->qhead == NULL; /* raid5.c:1048: submit now if the queue was empty */
    w->next = NULL;
    if (e->qtail)
        e->qtail->next = w;
    else
        e->qhead = w;
    e->qtail = w;
    pthread_mutex_unlock(&c->lock);
    return head;
}

struct draid_stripe_waiter *draid_stripe_complete(draid_stripe_cache *c, struct draid_stripe *s,
                                                  struct draid_stripe_waiter *w)
{
    if (!c || !s || !w)
        return NULL;
    pthread_mutex_lock(&c->lock);
    struct entry *e = ent(s);
    struct draid_stripe_waiter *next = NULL;
    if (e->qhead == w) { /* raid5.c:497-500: drop the finished head, hand on to the next */
        e->qhead = w->next;
        if (!e->qhead)
            e->qtail = NULL;
        next = e->qhead;
    } else { /* not the head (an aborted request): unlink it, nothing to start */
        struct draid_stripe_waiter *p = e->qhead;
        while (p && p->next != w)
            p = p->next;
        if (p) {
            p->next = w->next;
            if (e->qtail == w)
                e->qtail = p;
        }
    }
    w->next = NULL;
    pthread_mutex_unlock(&c->lock);
    return next;
}

uint32_t draid_stripe_cache_active(draid_stripe_cache *c)
{
    if (!c)
        return 0;
    pthread_mutex_lock(&c->lock);
    const uint32_t n = c->nactive;
    pthread_mutex_unlock(&c->lock);
    return n;
}
