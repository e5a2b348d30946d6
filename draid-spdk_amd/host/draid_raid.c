/*
 * draid_raid.c -- host-side RAID5/RAID6 stripe layer (see draid_raid.h).
 *
 * Restates the data-path logic of the reference's raid5 module
 * (module/bdev/raid/raid5.c) without SPDK types, and drives the parity
 * arithmetic through the draid_ec context (GPU) instead of isa-l.
 */
#include "../../include/draid_raid.h"

#include <errno.h>
#include <string.h>

static int is_pow2(uint32_t x) { return x && !(x & (x - 1)); }

static uint32_t log2u(uint32_t x)
{
    uint32_t s = 0;
    while ((1u << s) < x)
        s++;
    return s;
}

int draid_raid_start(struct draid_raid *r, int level, int n, uint32_t blocklen,
                     uint32_t strip_size, uint64_t min_base_blockcnt)
{
    const int m = level == 6 ? 2 : (level == 5 ? 1 : 0);
    if (!r || !m || n < m + 2 || n > DRAID_RAID_MAX_BASE || blocklen == 0 || !is_pow2(strip_size))
        return -EINVAL;
    memset(r, 0, sizeof(*r));
    r->level = (uint8_t)level;
    r->num_base_bdevs = (uint8_t)n;
    r->max_degraded = (uint8_t)m;
    r->blocklen = blocklen;
    r->strip_size = strip_size;
    r->strip_size_shift = log2u(strip_size);
    /* raid5.c:1419-1426 */
    r->total_stripes = min_base_blockcnt / strip_size;
    r->stripe_blocks = (uint64_t)strip_size * (uint64_t)(n - m);
    r->blockcnt = r->stripe_blocks * r->total_stripes;
    r->optimal_io_boundary = r->stripe_blocks;
    return 0;
}

void draid_raid_parity_chunks(const struct draid_raid *r, uint64_t stripe, int *p, int *q)
{
    const int n = r->num_base_bdevs;
    /* raid5.c:1006-1007: data_chunks_num - stripe % n == (n-1) - stripe % n for RAID5 */
    const int pd = (n - 1) - (int)(stripe % (uint64_t)n);
    *p = pd;
    *q = r->max_degraded == 2 ? (pd + 1) % n : -1;
}

int draid_raid_data_disk(const struct draid_raid *r, uint64_t stripe, int data_idx)
{
    int p, q;
    draid_raid_parity_chunks(r, stripe, &p, &q);
    for (int disk = 0, d = 0; disk < r->num_base_bdevs; disk++) {
        if (disk == p || disk == q)
            continue;
        if (d++ == data_idx)
            return disk;
    }
    return -1;
}

int draid_raid_disk_data_index(const struct draid_raid *r, uint64_t stripe, int disk)
{
    int p, q;
    draid_raid_parity_chunks(r, stripe, &p, &q);
    if (disk == p || disk == q)
        return -1;
    int d = 0;
    for (int i = 0; i < disk; i++)
        if (i != p && i != q)
            d++;
    return d;
}

/* raid5_handle_stripe, raid5.c:994-1041 */
int draid_raid_map_request(const struct draid_raid *r, uint64_t offset_blocks,
                           uint64_t num_blocks, struct draid_stripe_req *out)
{
    if (!r || !out || num_blocks == 0)
        return -EINVAL;
    const uint64_t stripe = offset_blocks / r->stripe_blocks;
    const uint64_t from = offset_blocks - stripe * r->stripe_blocks;
    const uint64_t to = from + num_blocks;
    if (to > r->stripe_blocks || stripe >= r->total_stripes)
        return -EINVAL; /* the bdev layer splits on optimal_io_boundary */
    memset(out, 0, sizeof(*out));
    out->stripe_index = stripe;
    draid_raid_parity_chunks(r, stripe, &out->p_disk, &out->q_disk);
    out->first_data = (int)(from >> r->strip_size_shift);
    out->last_data = (int)((to - 1) >> r->strip_size_shift);
    out->full_stripe = from == 0 && to == r->stripe_blocks;
    for (int d = out->first_data; d <= out->last_data; d++) {
        const int disk = draid_raid_data_disk(r, stripe, d);
        const uint64_t cfrom = (uint64_t)d << r->strip_size_shift;
        const uint64_t cto = cfrom + r->strip_size;
        uint64_t off = from > cfrom ? from - cfrom : 0;
        uint64_t blocks = (to < cto ? to - cfrom : r->strip_size) - off;
        out->chunk[disk].req_offset = off;
        out->chunk[disk].req_blocks = blocks;
    }
    return 0;
}

/* raid5_chunk_map_iov, raid5.c:358-426 */
int draid_raid_map_iov(struct iovec *out, int out_max, const struct iovec *iov, int iovcnt,
                       uint64_t offset, uint64_t len)
{
    int i = 0, n = 0;
    uint64_t off = 0;
    while (i < iovcnt && off + iov[i].iov_len <= offset) {
        off += iov[i].iov_len;
        i++;
    }
    if (i >= iovcnt && len)
        return -EINVAL;
    while (len > 0) {
        if (i >= iovcnt)
            return -EINVAL;
        if (n >= out_max)
            return -ENOSPC;
        const uint64_t skip = offset - off;
        uint64_t take = iov[i].iov_len - skip;
        if (take > len)
            take = len;
        out[n].iov_base = (uint8_t *)iov[i].iov_base + skip;
        out[n].iov_len = take;
        n++;
        len -= take;
        offset += take;
        off += iov[i].iov_len;
        i++;
    }
    return n;
}

int draid_raid_stripe_write(const struct draid_raid *r, draid_ec_ctx *ctx,
                            const struct draid_stripe_req *req, const struct iovec *iov,
                            int iovcnt, void *const parity_buf[2],
                            struct draid_base_io *writes, int *nwrites)
{
    if (!r || !ctx || !req || !writes || !nwrites || !parity_buf)
        return -EINVAL;
    if (!req->full_stripe)
        return -EINVAL; /* raid5_simple.c:381-395: only full-stripe writes */
    const int n = r->num_base_bdevs, m = r->max_degraded, k = n - m;
    const uint64_t sb = (uint64_t)r->strip_size * r->blocklen;
    const struct iovec *lists[DRAID_RAID_MAX_BASE];
    int cnts[DRAID_RAID_MAX_BASE];
    struct iovec pq[2];

    for (int d = 0; d < k; d++) {
        const int disk = draid_raid_data_disk(r, req->stripe_index, d);
        struct draid_base_io *w = &writes[disk];
        int c = draid_raid_map_iov(w->iov, DRAID_RAID_MAX_IOV, iov, iovcnt, (uint64_t)d * sb, sb);
        if (c < 0)
            return c;
        w->iovcnt = c;
        lists[d] = w->iov;
        cnts[d] = c;
    }
    for (int j = 0; j < m; j++) {
        pq[j].iov_base = parity_buf[j];
        pq[j].iov_len = sb;
        lists[k + j] = &pq[j];
        cnts[k + j] = 1;
        const int disk = j == 0 ? req->p_disk : req->q_disk;
        writes[disk].iovcnt = 1;
        writes[disk].iov[0] = pq[j];
    }
    for (int disk = 0; disk < n; disk++) {
        writes[disk].disk = disk;
        writes[disk].offset_blocks = req->stripe_index << r->strip_size_shift; /* raid5.c:648 */
        writes[disk].num_blocks = r->strip_size;
    }
    int rc = draid_ec_ctx_encode_sg(ctx, (uint32_t)k, (uint32_t)m, lists, cnts, NULL, sb);
    if (rc)
        return rc > 0 ? -EINVAL : rc;
    *nwrites = n;
    return 0;
}

int draid_raid_stripe_degraded_read(const struct draid_raid *r, draid_ec_ctx *ctx,
                                    uint64_t stripe, void *const *chunk_buf,
                                    struct draid_base_io *reads, int *nreads)
{
    if (!r || !ctx || !chunk_buf || !reads || !nreads)
        return -EINVAL;
    const int n = r->num_base_bdevs, m = r->max_degraded, k = n - m;
    const uint64_t sb = (uint64_t)r->strip_size * r->blocklen;
    int p, q, fail[2], nfail = 0, nr = 0;
    draid_raid_parity_chunks(r, stripe, &p, &q);
    for (int disk = 0; disk < n; disk++) {
        if (r->degraded_mask & (1u << disk)) {
            if (nfail == m)
                return -EIO;
            const int d = draid_raid_disk_data_index(r, stripe, disk);
            fail[nfail++] = d >= 0 ? d : (disk == p ? k : k + 1);
            continue;
        }
        struct draid_base_io *rd = &reads[nr++];
        rd->disk = disk;
        rd->offset_blocks = stripe << r->strip_size_shift;
        rd->num_blocks = r->strip_size;
        rd->iovcnt = 1;
        rd->iov[0].iov_base = chunk_buf[disk];
        rd->iov[0].iov_len = sb;
    }
    *nreads = nr;
    if (nfail == 0)
        return 0;
    struct iovec v[DRAID_RAID_MAX_BASE];
    const struct iovec *lists[DRAID_RAID_MAX_BASE];
    int cnts[DRAID_RAID_MAX_BASE];
    for (int j = 0; j < n; j++) { /* isa-l order: data 0..k-1, P, Q */
        const int disk = j < k ? draid_raid_data_disk(r, stripe, j) : (j == k ? p : q);
        v[j].iov_base = chunk_buf[disk];
        v[j].iov_len = sb;
        lists[j] = &v[j];
        cnts[j] = 1;
    }
    int rc = draid_ec_ctx_reconstruct_sg(ctx, (uint32_t)k, (uint32_t)m, lists, cnts, NULL, sb,
                                         nfail, fail);
    return rc > 0 ? -EINVAL : rc;
}
