/*
 * isal_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * This is a plain-C restatement of the parity arithmetic the reference
 * (kyleshu/draid-spdk, an SPDK v22.01-pre fork) reaches through isa-l v2.30.0
 * (`isa-l/` submodule, EMPTY in the reference tree), plus
 * the reference's own RAID5 geometry.  It is the checker for the HIP engine:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  The product path (draid-spdk_amd/) never links or calls it.
 *
 * Parity status: isa-l is not vendored and cannot be built here.  XOR parity is
 * pinned by the reference's known-answer test
 * (test/unit/lib/bdev/raid/raid5.c/raid5_ut_ref.c:324-330,350-397); P+Q and the
 * recovery formulas are pinned by the self-checks of
 * examples/bdev/gf_vect_mul/gf_vect_mul.c:95-347 reproduced bit for bit with
 * glibc srand(0x1234)/rand() inputs, and by isa-l's published field definition
 * (polynomial 0x11D, generator 2).  Exact Q bytes have no golden bytes in the
 * reference: they are pinned by that definition plus the example's algebraic
 * checks (Q == XOR_i gf_vect_mul(2^i, D_i)), not by reference output.
 */
#ifndef DRAID_ISAL_ORACLE_H
#define DRAID_ISAL_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- GF(2^8), poly 0x11D, generator 2 (isa-l ec_base.c gf_mul/gf_inv) ---- */
unsigned char orc_gf_mul(unsigned char a, unsigned char b);
unsigned char orc_gf_inv(unsigned char a);
unsigned char orc_gf_pow2(int e);                /* 2^e, e taken mod 255 */
void orc_gf_tables(unsigned char exp_out[256], unsigned char log_out[256]);
void orc_gf_vect_mul_init(unsigned char c, unsigned char tbl[32]);
int  orc_gf_vect_mul(int len, const unsigned char *tbl, const void *src, void *dest);

/* ---- isa-l raid.h semantics (raid_base.c restated) ---- */
int orc_xor_gen(int vects, int len, void **array);
int orc_pq_gen(int vects, int len, void **array);
int orc_xor_check(int vects, int len, void **array);
int orc_pq_check(int vects, int len, void **array);

/* ---- recovery (gf_vect_mul.c:242-347 and raid5.c:544-594 restated) ----
 * array = k data pointers, then P (array[k]) and, for m == 2, Q (array[k+1]).
 * fail[0..nfail-1] are strip indices in [0, k+m) whose contents are
 * regenerated in place from the survivors.  Returns 0, or -1 on an
 * unrecoverable / invalid failure set. */
int orc_recover(int k, int m, int len, void **array, int nfail, const int *fail);

/* ---- batched helpers over a strided stripe layout (tests/bench) ----
 * Stripe s, strip j lives at base + s*stripe_stride + j*strip_stride.      */
int orc_encode_strided(int k, int m, size_t len, uint32_t nstripes,
                       uint8_t *base, size_t strip_stride, size_t stripe_stride);
int orc_recover_strided(int k, int m, size_t len, uint32_t nstripes,
                        uint8_t *base, size_t strip_stride, size_t stripe_stride,
                        const uint8_t *fail /* [nstripes][2], 0xFF = none */);

/* CPU baseline timing: repeats encode (+ dual-data reconstruct when
 * with_reconstruct) over the strided batch for at least min_seconds using
 * nthreads pthreads (stripes partitioned by contiguous ranges).  Returns the
 * elapsed seconds and writes the number of full passes done to *passes. */
/* AVX-512 (+GFNI affine) restatement of isa-l's x86 kernels (isal_simd.c):
 * the CPU baseline.  Same results and failure semantics as the strided calls
 * above, except that unrecoverable / empty failure sets are skipped (as the
 * GPU kernels do).  -1 when the CPU lacks AVX-512BW or GFNI. */
int orc_simd_available(void);
int orc_simd_xor_gen(int vects, int len, void **array);
int orc_simd_encode_strided(int k, int m, size_t len, uint32_t nstripes, uint8_t *base,
                            size_t strip_stride, size_t stripe_stride);
int orc_simd_recover_strided(int k, int m, size_t len, uint32_t nstripes, uint8_t *base,
                             size_t strip_stride, size_t stripe_stride, const uint8_t *fail);
/* impl 0: scalar restatement, 1: AVX-512 restatement */
double orc_bench_encode_reconstruct_impl(int impl, int k, int m, size_t len, uint32_t nstripes,
                                         uint8_t *base, size_t strip_stride,
                                         size_t stripe_stride, const uint8_t *fail,
                                         int with_reconstruct, int nthreads,
                                         double min_seconds, uint64_t *passes);
double orc_bench_encode_reconstruct(int k, int m, size_t len, uint32_t nstripes,
                                    uint8_t *base, size_t strip_stride,
                                    size_t stripe_stride, const uint8_t *fail,
                                    int with_reconstruct, int nthreads,
                                    double min_seconds, uint64_t *passes);

/* ---- BASELINE config 1 CPU harness (bdevperf_raid5.c) ---- */
double orc_bdevperf_raid5_fsw(int n, size_t strip, size_t disk_bytes, int qd, double seconds,
                              uint64_t *ios_out, uint8_t *verify_ok);

/* ---- reference RAID5 geometry (module/bdev/raid/raid5.c) ---- */
int  orc_raid5_parity_chunk(int num_base_bdevs, int max_degraded, uint64_t stripe_index);
int  orc_raid5_data_chunk_to_disk(int parity_chunk, int data_idx);
void orc_raid5_start_geometry(int num_base_bdevs, int max_degraded, uint64_t min_blockcnt,
                              uint32_t strip_size, uint64_t *stripe_blocks,
                              uint64_t *total_stripes, uint64_t *blockcnt,
                              uint64_t *optimal_io_boundary);

/* ---- input generators ---- */
void orc_srand(unsigned int seed);                         /* glibc srand, private state */
void orc_rand_buffer(unsigned char *buf, long size);      /* gf_vect_mul.c:21-26 */
void orc_glibc_srand(unsigned int seed);                   /* global glibc srand */
void orc_glibc_rand_buffer(unsigned char *buf, long size); /* global glibc rand */
uint64_t orc_splitmix64(uint64_t *state);
void orc_fill_splitmix(uint8_t *buf, size_t len, uint64_t seed);
void orc_fill_ut_ref_pattern(uint8_t *buf, uint64_t num_blocks, uint32_t blocklen);

#ifdef __cplusplus
}
#endif
#endif
