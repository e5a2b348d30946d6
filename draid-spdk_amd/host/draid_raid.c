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

/* Whole-stripe degraded read: reads (when `reads` is given) and the reconstruct
 * (when `ctx` is given) of stripe `stripe`. */
static int degraded_read(const struct draid_raid *r, draid_ec_ctx *ctx, uint64_t stripe,
                         void *const *chunk_buf, struct draid_base_io *reads, int *nreads)
{
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
        if (!reads)
            continue;
        struct draid_base_io *rd = &reads[nr++];
        rd->disk = disk;
        rd->offset_blocks = stripe << r->strip_size_shift;
        rd->num_blocks = r->strip_size;
        rd->iovcnt = 1;
        rd->iov[0].iov_base = chunk_buf[disk];
        rd->iov[0].iov_len = sb;
    }
    if (nreads)
        *nreads = nr;
    if (nfail == 0 || !ctx)
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

int draid_raid_stripe_degraded_read(const struct draid_raid *r, draid_ec_ctx *ctx,
                                    uint64_t stripe, void *const *chunk_buf,
                                    struct draid_base_io *reads, int *nreads)
{
    if (!r || !chunk_buf || !reads || !nreads)
        return -EINVAL;
    return degraded_read(r, ctx, stripe, chunk_buf, reads, nreads);
}

int draid_raid_stripe_degraded_rebuild(const struct draid_raid *r, draid_ec_ctx *ctx,
                                       uint64_t stripe, void *const *chunk_buf)
{
    if (!r || !ctx || !chunk_buf)
        return -EINVAL;
    return degraded_read(r, ctx, stripe, chunk_buf, NULL, NULL);
}

/* ------------------------------------------------------------ partial writes */

static void add_io(struct draid_base_io *io, int disk, uint64_t stripe_lba, uint64_t off,
                   uint64_t blocks, void *buf, uint32_t blocklen)
{
    io->disk = disk;
    io->offset_blocks = stripe_lba + off;
    io->num_blocks = blocks;
    io->iovcnt = 1;
    io->iov[0].iov_base = (uint8_t *)buf + off * blocklen;
    io->iov[0].iov_len = blocks * blocklen;
}

/* raid5_stripe_write, raid5.c:779-867 */
int draid_raid_plan_write(const struct draid_raid *r, const struct draid_stripe_req *req,
                          struct draid_write_plan *plan, void *const *preread_buf,
                          struct draid_base_io *reads, int *nreads)
{
    if (!r || !req || !plan || !preread_buf || !reads || !nreads || req->full_stripe)
        return -EINVAL;
    const int n = r->num_base_bdevs;
    const uint64_t strip = r->strip_size, lba = req->stripe_index << r->strip_size_shift;
    memset(plan, 0, sizeof(*plan));
    if (req->first_data == req->last_data) {
        const int fd = draid_raid_data_disk(r, req->stripe_index, req->first_data);
        plan->p_offset = req->chunk[fd].req_offset;
        plan->p_blocks = req->chunk[fd].req_blocks;
    } else {
        plan->p_offset = 0;
        plan->p_blocks = strip;
    }
    int balance = 0;
    for (int disk = 0; disk < n; disk++) {
        if (disk == req->p_disk || disk == req->q_disk)
            continue;
        if (req->chunk[disk].req_blocks < plan->p_blocks)
            balance++;
        if (req->chunk[disk].req_blocks > 0)
            balance--;
    }
    plan->mode = balance > 0 ? DRAID_WRITE_RMW : DRAID_WRITE_RCW;
    int nr = 0;
    for (int disk = 0; disk < n; disk++) {
        const bool parity = disk == req->p_disk || disk == req->q_disk;
        const struct draid_chunk_req *c = &req->chunk[disk];
        struct draid_chunk_req *pr = &plan->preread[disk];
        if (plan->mode == DRAID_WRITE_RMW) {
            /* old data of the touched ranges and the old parity range */
            pr->req_offset = parity ? plan->p_offset : c->req_offset;
            pr->req_blocks = parity ? plan->p_blocks : c->req_blocks;
        } else if (parity) {
            pr->req_blocks = 0; /* reconstruct-write: parity is recomputed */
        } else if (req->first_data == req->last_data) {
            if (!c->req_blocks) { /* non-request chunks: the parity range */
                pr->req_offset = plan->p_offset;
                pr->req_blocks = plan->p_blocks;
            }
        } else if (c->req_offset) { /* complete the chunk in front of the request */
            pr->req_offset = 0;
            pr->req_blocks = c->req_offset;
        } else { /* behind the request (the whole chunk if untouched) */
            pr->req_offset = c->req_blocks;
            pr->req_blocks = strip - c->req_blocks;
        }
        if (pr->req_blocks)
            add_io(&reads[nr++], disk, lba, pr->req_offset, pr->req_blocks, preread_buf[disk],
                   r->blocklen);
    }
    *nreads = nr;
    return 0;
}

/* User-iovec slice holding data chunk d's strip blocks [a, b). */
static int user_slice(const struct draid_raid *r, const struct draid_stripe_req *req, int d,
                      uint64_t a, uint64_t b, const struct iovec *iov, int iovcnt,
                      struct iovec *out, int out_max)
{
    const uint64_t from = (uint64_t)req->first_data * r->strip_size +
                          req->chunk[draid_raid_data_disk(r, req->stripe_index,
                                                          req->first_data)].req_offset;
    const uint64_t soff = (uint64_t)d * r->strip_size + a; /* stripe offset of block a */
    return draid_raid_map_iov(out, out_max, iov, iovcnt, (soff - from) * r->blocklen,
                              (b - a) * r->blocklen);
}

int draid_raid_stripe_write_partial(const struct draid_raid *r, draid_ec_ctx *ctx,
                                    const struct draid_stripe_req *req,
                                    const struct draid_write_plan *plan, const struct iovec *iov,
                                    int iovcnt, void *const *preread_buf,
                                    struct draid_base_io *writes, int *nwrites)
{
    if (!r || !ctx || !req || !plan || !iov || !preread_buf || !writes || !nwrites)
        return -EINVAL;
    const int n = r->num_base_bdevs, m = r->max_degraded, k = n - m;
    const uint32_t bl = r->blocklen;
    const uint64_t lba = req->stripe_index << r->strip_size_shift;
    const uint64_t p0 = plan->p_offset, p1 = plan->p_offset + plan->p_blocks;
    int pdisk[2] = {req->p_disk, req->q_disk};
    struct iovec pv[2];
    const struct iovec *plist[2] = {&pv[0], &pv[1]};
    int pcnt[2] = {1, 1};
    int rc = 0;

    if (plan->mode == DRAID_WRITE_RMW) {
        /* elementary strip ranges between every touched chunk's boundaries */
        uint64_t cut[2 * DRAID_RAID_MAX_BASE + 2];
        int nc = 0;
        for (int d = req->first_data; d <= req->last_data; d++) {
            const struct draid_chunk_req *c =
                &req->chunk[draid_raid_data_disk(r, req->stripe_index, d)];
            cut[nc++] = c->req_offset;
            cut[nc++] = c->req_offset + c->req_blocks;
        }
        for (int i = 1; i < nc; i++) /* insertion sort: nc <= 2k */
            for (int j = i; j > 0 && cut[j - 1] > cut[j]; j--) {
                uint64_t t = cut[j];
                cut[j] = cut[j - 1];
                cut[j - 1] = t;
            }
        static __thread struct iovec ov[DRAID_RAID_MAX_BASE], nv[DRAID_RAID_MAX_BASE]
                                                                 [DRAID_RAID_MAX_IOV];
        for (int i = 0; i + 1 < nc; i++) {
            const uint64_t a = cut[i], b = cut[i + 1];
            if (a == b)
                continue;
            int idx[DRAID_RAID_MAX_BASE], nd = 0, ncnt[DRAID_RAID_MAX_BASE], ocnt[DRAID_RAID_MAX_BASE];
            const struct iovec *ol[DRAID_RAID_MAX_BASE], *nl[DRAID_RAID_MAX_BASE];
            for (int d = req->first_data; d <= req->last_data; d++) {
                const int disk = draid_raid_data_disk(r, req->stripe_index, d);
                const struct draid_chunk_req *c = &req->chunk[disk];
                if (c->req_offset > a || c->req_offset + c->req_blocks < b)
                    continue;
                ov[nd].iov_base = (uint8_t *)preread_buf[disk] + a * bl;
                ov[nd].iov_len = (b - a) * bl;
                ol[nd] = &ov[nd];
                ocnt[nd] = 1;
                int cnt = user_slice(r, req, d, a, b, iov, iovcnt, nv[nd], DRAID_RAID_MAX_IOV);
                if (cnt < 0)
                    return cnt;
                nl[nd] = nv[nd];
                ncnt[nd] = cnt;
                idx[nd++] = d;
            }
            if (!nd)
                continue;
            for (int j = 0; j < m; j++) {
                pv[j].iov_base = (uint8_t *)preread_buf[pdisk[j]] + a * bl;
                pv[j].iov_len = (b - a) * bl;
            }
            rc = draid_ec_ctx_update_sg(ctx, (uint32_t)k, (uint32_t)m, (uint32_t)nd, idx, ol, ocnt,
                                        nl, ncnt, plist, pcnt, (b - a) * bl);
            if (rc)
                return rc > 0 ? -EINVAL : rc;
        }
    } else {
        /* reconstruct-write: every data chunk over [p0, p1) from preread + new data */
        static __thread struct iovec dv[DRAID_RAID_MAX_BASE][DRAID_RAID_MAX_IOV + 2];
        const struct iovec *dl[DRAID_RAID_MAX_BASE + 2];
        int dcnt[DRAID_RAID_MAX_BASE + 2];
        for (int d = 0; d < k; d++) {
            const int disk = draid_raid_data_disk(r, req->stripe_index, d);
            const struct draid_chunk_req *c = &req->chunk[disk];
            int cnt = 0;
            const uint64_t u0 = c->req_blocks ? c->req_offset : p1;
            const uint64_t u1 = c->req_blocks ? c->req_offset + c->req_blocks : p1;
            if (p0 < u0) { /* preread in front */
                dv[d][cnt].iov_base = (uint8_t *)preread_buf[disk] + p0 * bl;
                dv[d][cnt++].iov_len = (u0 - p0) * bl;
            }
            if (u1 > u0) {
                int c2 = user_slice(r, req, d, u0, u1, iov, iovcnt, &dv[d][cnt],
                                    DRAID_RAID_MAX_IOV);
                if (c2 < 0)
                    return c2;
                cnt += c2;
            }
            if (u1 < p1) { /* preread behind */
                dv[d][cnt].iov_base = (uint8_t *)preread_buf[disk] + u1 * bl;
                dv[d][cnt++].iov_len = (p1 - u1) * bl;
            }
            dl[d] = dv[d];
            dcnt[d] = cnt;
        }
        for (int j = 0; j < m; j++) {
            pv[j].iov_base = (uint8_t *)preread_buf[pdisk[j]] + p0 * bl;
            pv[j].iov_len = (p1 - p0) * bl;
            dl[k + j] = &pv[j];
            dcnt[k + j] = 1;
        }
        rc = draid_ec_ctx_encode_sg(ctx, (uint32_t)k, (uint32_t)m, dl, dcnt, NULL, (p1 - p0) * bl);
        if (rc)
            return rc > 0 ? -EINVAL : rc;
    }

    /* base writes: the new data ranges, then the parity range */
    int nw = 0;
    for (int d = req->first_data; d <= req->last_data; d++) {
        const int disk = draid_raid_data_disk(r, req->stripe_index, d);
        const struct draid_chunk_req *c = &req->chunk[disk];
        if (!c->req_blocks)
            continue;
        struct draid_base_io *w = &writes[nw++];
        w->disk = disk;
        w->offset_blocks = lba + c->req_offset;
        w->num_blocks = c->req_blocks;
        int cnt = user_slice(r, req, d, c->req_offset, c->req_offset + c->req_blocks, iov, iovcnt,
                             w->iov, DRAID_RAID_MAX_IOV);
        if (cnt < 0)
            return cnt;
        w->iovcnt = cnt;
    }
    for (int j = 0; j < m; j++)
        add_io(&writes[nw++], pdisk[j], lba, p0, p1 - p0, preread_buf[pdisk[j]], bl);
    *nwrites = nw;
    return 0;
}

/* ------------------------------------------------------------ ranged reads */

/* One base read of data chunk d's requested blocks into the parent iovecs
 * (CHUNK_READ, raid5.c:929-930,935-943). */
static int read_request(const struct draid_raid *r, const struct draid_stripe_req *req, int d,
                        const struct iovec *iov, int iovcnt, struct draid_base_io *io)
{
    const int disk = draid_raid_data_disk(r, req->stripe_index, d);
    const struct draid_chunk_req *c = &req->chunk[disk];
    io->disk = disk;
    io->offset_blocks = (req->stripe_index << r->strip_size_shift) + c->req_offset;
    io->num_blocks = c->req_blocks;
    const int cnt = user_slice(r, req, d, c->req_offset, c->req_offset + c->req_blocks, iov,
                               iovcnt, io->iov, DRAID_RAID_MAX_IOV);
    if (cnt < 0)
        return cnt;
    io->iovcnt = cnt;
    return 0;
}

/* The part of strip range [a, b) that data chunk d's request covers, clamped:
 * [*u0, *u1), or empty (*u0 == *u1 == b) for parity, unrequested chunks and
 * disjoint requests. */
static void covered(const struct draid_chunk_req *c, int d, uint64_t a, uint64_t b, uint64_t *u0,
                    uint64_t *u1)
{
    uint64_t x = c->req_offset, y = c->req_offset + c->req_blocks;
    if (d < 0 || !c->req_blocks || y <= a || x >= b)
        x = y = b;
    *u0 = x < a ? a : x;
    *u1 = y > b ? b : y;
}

/* Strip j's iovecs over [a, b): the covered part from the parent iovecs, the
 * rest at the same offset in buf. */
static int range_list(const struct draid_raid *r, const struct draid_stripe_req *req, int disk,
                      int d, uint64_t a, uint64_t b, const struct iovec *iov, int iovcnt,
                      void *buf, struct iovec *out, int out_max)
{
    const uint32_t bl = r->blocklen;
    uint64_t u0, u1;
    covered(&req->chunk[disk], d, a, b, &u0, &u1);
    int n = 0;
    if (a < u0) {
        out[n].iov_base = (uint8_t *)buf + a * bl;
        out[n++].iov_len = (u0 - a) * bl;
    }
    if (u0 < u1) {
        const int c2 = user_slice(r, req, d, u0, u1, iov, iovcnt, out + n, out_max - n - 1);
        if (c2 < 0)
            return c2;
        n += c2;
    }
    if (u1 < b) {
        out[n].iov_base = (uint8_t *)buf + u1 * bl;
        out[n++].iov_len = (b - u1) * bl;
    }
    return n;
}

/* Ranged read: the base reads (when `reads` is given) and the reconstruct of the
 * lost requested range (when `ctx` is given). */
static int ranged_read(const struct draid_raid *r, draid_ec_ctx *ctx,
                       const struct draid_stripe_req *req, const struct iovec *iov, int iovcnt,
                       void *const *chunk_buf, struct draid_base_io *reads, int *nreads)
{
    const int n = r->num_base_bdevs, m = r->max_degraded, k = n - m;
    const uint64_t s = req->stripe_index, lba = s << r->strip_size_shift;
    const int pdisk = req->p_disk, qdisk = req->q_disk;
    /* R = [lo, hi): the requested ranges of degraded data chunks (raid5.c:882-891
     * picks the one d_chunk; RAID6 may have two) */
    uint64_t lo = r->strip_size, hi = 0;
    int ndeg = 0;
    for (int disk = 0; disk < n; disk++) {
        if (!(r->degraded_mask & (1u << disk)))
            continue;
        ndeg++;
        const struct draid_chunk_req *c = &req->chunk[disk];
        if (disk == pdisk || disk == qdisk || !c->req_blocks)
            continue;
        if (c->req_offset < lo)
            lo = c->req_offset;
        if (c->req_offset + c->req_blocks > hi)
            hi = c->req_offset + c->req_blocks;
    }
    int nr = 0, rc;
    if (hi <= lo) { /* nothing to rebuild: plain reads (raid5.c:933-945) */
        for (int d = req->first_data; reads && d <= req->last_data; d++) {
            if (!req->chunk[draid_raid_data_disk(r, s, d)].req_blocks)
                continue;
            if ((rc = read_request(r, req, d, iov, iovcnt, &reads[nr++])) < 0)
                return rc;
        }
        if (nreads)
            *nreads = nr;
        return 0;
    }
    if (ndeg > m)
        return -EIO;
    /* lost strips in isa-l order; a read never regenerates Q, so a lost Q is
     * left out and Q is read only when two strips are lost */
    int fail[2], nfail = 0;
    for (int disk = 0; disk < n; disk++)
        if ((r->degraded_mask & (1u << disk)) && disk != qdisk)
            fail[nfail++] = disk == pdisk ? k : draid_raid_disk_data_index(r, s, disk);
    const int needq = nfail == 2;
    static __thread struct iovec lv[DRAID_RAID_MAX_BASE][DRAID_RAID_MAX_IOV + 2];
    const struct iovec *lists[DRAID_RAID_MAX_BASE];
    int cnts[DRAID_RAID_MAX_BASE];
    for (int j = 0; j < n; j++) {
        const int disk = j < k ? draid_raid_data_disk(r, s, j) : (j == k ? pdisk : qdisk);
        const int d = j < k ? j : -1;
        const struct draid_chunk_req *c = &req->chunk[disk];
        /* sources and rebuilt outputs over R: requested parts in the parent
         * iovecs, the rest in chunk_buf (a lost Q, or Q when unneeded, is never
         * touched by the kernel) */
        const int cnt = range_list(r, req, disk, d, lo, hi, iov, iovcnt, chunk_buf[disk], lv[j],
                                   DRAID_RAID_MAX_IOV + 2);
        if (cnt < 0)
            return cnt;
        lists[j] = lv[j];
        cnts[j] = cnt;
        if (!reads || (r->degraded_mask & (1u << disk)) || (disk == qdisk && !needq))
            continue;
        if (d >= 0 && c->req_blocks && (rc = read_request(r, req, d, iov, iovcnt, &reads[nr++])) < 0)
            return rc;
        /* the parts of R its request does not cover (CHUNK_PREREAD, raid5.c:896-917) */
        uint64_t u0, u1;
        covered(c, d, lo, hi, &u0, &u1);
        if (lo < u0)
            add_io(&reads[nr++], disk, lba, lo, u0 - lo, chunk_buf[disk], r->blocklen);
        if (u1 < hi)
            add_io(&reads[nr++], disk, lba, u1, hi - u1, chunk_buf[disk], r->blocklen);
    }
    if (nreads)
        *nreads = nr;
    if (!ctx)
        return 0;
    rc = draid_ec_ctx_reconstruct_sg(ctx, (uint32_t)k, (uint32_t)m, lists, cnts, NULL,
                                     (hi - lo) * r->blocklen, nfail, fail);
    return rc > 0 ? -EINVAL : rc;
}

int draid_raid_stripe_read(const struct draid_raid *r, draid_ec_ctx *ctx,
                           const struct draid_stripe_req *req, const struct iovec *iov,
                           int iovcnt, void *const *chunk_buf, struct draid_base_io *reads,
                           int *nreads)
{
    if (!r || !req || !iov || !chunk_buf || !reads || !nreads)
        return -EINVAL;
    return ranged_read(r, ctx, req, iov, iovcnt, chunk_buf, reads, nreads);
}

int draid_raid_stripe_read_rebuild(const struct draid_raid *r, draid_ec_ctx *ctx,
                                   const struct draid_stripe_req *req, const struct iovec *iov,
                                   int iovcnt, void *const *chunk_buf)
{
    if (!r || !ctx || !req || !iov || !chunk_buf)
        return -EINVAL;
    return ranged_read(r, ctx, req, iov, iovcnt, chunk_buf, NULL, NULL);
}

/* ------------------------------------------------------------ stripe assembly */

void draid_raid_asm_init(struct draid_stripe_asm *a)
{
    if (a) {
        a->active = 0;
        a->received = 0;
        a->have = 0;
    }
}

/* raid5_submit_write_request, raid5_simple.c:347-423 */
int draid_raid_asm_add(const struct draid_raid *r, struct draid_stripe_asm *a,
                       uint64_t offset_blocks, uint64_t num_blocks, const struct iovec *iov,
                       int iovcnt)
{
    if (!r || !a || !iov || iovcnt < 1 || iovcnt > DRAID_RAID_MAX_IOV)
        return -EINVAL;
    const uint64_t stripe = offset_blocks / r->stripe_blocks;
    const uint64_t off = offset_blocks - stripe * r->stripe_blocks;
    if (num_blocks != r->strip_size || (off & (r->strip_size - 1)) || stripe >= r->total_stripes)
        return -EINVAL; /* only whole strips of a full-stripe write */
    const int d = (int)(off >> r->strip_size_shift);
    uint64_t bytes = 0;
    for (int i = 0; i < iovcnt; i++)
        bytes += iov[i].iov_len;
    if (bytes != (uint64_t)r->strip_size * r->blocklen)
        return -EINVAL;
    if (!a->active) { /* the first child of a stripe (raid5_simple.c:356-374) */
        a->active = 1;
        a->stripe_index = stripe;
        a->received = 0;
        a->have = 0;
    } else if (a->stripe_index != stripe || (a->have & (1u << d))) {
        return -EINVAL;
    }
    memcpy(a->iov[d], iov, (size_t)iovcnt * sizeof(*iov));
    a->iovcnt[d] = iovcnt;
    a->have |= 1u << d;
    if (++a->received < r->num_base_bdevs - r->max_degraded)
        return 0;
    a->active = 0; /* all k data chunks: encode (raid5_simple.c:416-420) */
    return 1;
}

int draid_raid_asm_iov(const struct draid_raid *r, const struct draid_stripe_asm *a,
                       struct iovec *out, int out_max)
{
    if (!r || !a || !out)
        return -EINVAL;
    const int k = r->num_base_bdevs - r->max_degraded;
    int n = 0;
    for (int d = 0; d < k; d++) {
        if (!(a->have & (1u << d)))
            return -EINVAL;
        if (n + a->iovcnt[d] > out_max)
            return -ENOSPC;
        memcpy(out + n, a->iov[d], (size_t)a->iovcnt[d] * sizeof(*out));
        n += a->iovcnt[d];
    }
    return n;
}

/* ------------------------------------------------------------ disk-level tables */

int draid_raid_fail_table(const struct draid_raid *r, uint64_t first, uint32_t count,
                          uint8_t *fail)
{
    if (!r || !fail)
        return -EINVAL;
    const int n = r->num_base_bdevs, m = r->max_degraded, k = n - m;
    int deg[2], nd = 0;
    for (int disk = 0; disk < n; disk++)
        if (r->degraded_mask & (1u << disk)) {
            if (nd == m)
                return -EIO;
            deg[nd++] = disk;
        }
    for (uint32_t i = 0; i < count; i++) {
        const uint64_t s = first + i;
        int p, q;
        draid_raid_parity_chunks(r, s, &p, &q);
        for (int t = 0; t < 2; t++) {
            uint8_t v = DRAID_EC_FAIL_NONE;
            if (t < nd) {
                const int d = draid_raid_disk_data_index(r, s, deg[t]);
                v = (uint8_t)(d >= 0 ? d : (deg[t] == p ? k : k + 1));
            }
            fail[2 * (size_t)i + t] = v;
        }
    }
    return 0;
}

int draid_raid_strip_table(const struct draid_raid *r, uint64_t first, uint32_t count,
                           void *const *disk_base, uint64_t disk_first, void **table)
{
    if (!r || !disk_base || !table || first < disk_first)
        return -EINVAL;
    const int n = r->num_base_bdevs, m = r->max_degraded, k = n - m;
    const uint64_t sb = (uint64_t)r->strip_size * r->blocklen;
    for (uint32_t i = 0; i < count; i++) {
        const uint64_t s = first + i;
        int p, q;
        draid_raid_parity_chunks(r, s, &p, &q);
        for (int j = 0; j < n; j++) {
            const int disk = j < k ? draid_raid_data_disk(r, s, j) : (j == k ? p : q);
            table[(size_t)i * n + j] = (uint8_t *)disk_base[disk] + (s - disk_first) * sb;
        }
    }
    return 0;
}
