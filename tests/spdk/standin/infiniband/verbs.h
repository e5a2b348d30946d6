/* Stand-in for <infiniband/verbs.h> (libibverbs, a system package this image
 * lacks).  The reference's include/spdk/env.h:45 includes it for one prototype,
 * spdk_rdma_create_mem_map_external(struct ibv_pd *pd) (env.h:1427), which nothing
 * in module/bdev/raid uses.  Declaring the struct tag is all that takes.
 * Used ONLY by the tests/spdk harness builds; it is not part of the product and
 * not of the oracle. */
#ifndef DRAID_TEST_STANDIN_VERBS_H
#define DRAID_TEST_STANDIN_VERBS_H
struct ibv_pd;
#endif
