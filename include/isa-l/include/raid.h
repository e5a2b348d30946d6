/*
 * isa-l/include/raid.h -- drop-in for the header of that name in isa-l v2.30.
 *
 * The reference includes "isa-l/include/raid.h" and calls xor_gen / pq_gen
 * (module/bdev/raid/raid5.c:189,197; raid5_simple.c:11,134,176;
 * examples/bdev/gf_vect_mul/gf_vect_mul.c:1,45,101,168-169,178).  With this
 * directory on the include path ahead of isa-l's, and libdraid_isal.so linked
 * instead of libisal, those call sites run on the MI355X engine unmodified:
 * each function forwards to its draid_* namesake in libdraid_ec.so
 * (include/draid_ec.h), same arguments, same 0 / non-zero return.
 * Any host or device pointer is accepted (pageable memory is staged).
 */
#ifndef DRAID_ISAL_COMPAT_RAID_H
#define DRAID_ISAL_COMPAT_RAID_H

#ifdef __cplusplus
extern "C" {
#endif

/* array[vects-1] = XOR of array[0 .. vects-2]; vects >= 3. */
int xor_gen(int vects, int len, void **array);
/* 0 iff the XOR of all vects vectors is zero. */
int xor_check(int vects, int len, void **array);
/* array[vects-2] = P, array[vects-1] = Q over GF(2^8)/0x11D; vects >= 4, len % 32 == 0. */
int pq_gen(int vects, int len, void **array);
/* 0 iff the stored P and Q match the sources. */
int pq_check(int vects, int len, void **array);

/* isa-l's portable-C entry points: same semantics as the ones above. */
int xor_gen_base(int vects, int len, void **array);
int xor_check_base(int vects, int len, void **array);
int pq_gen_base(int vects, int len, void **array);
int pq_check_base(int vects, int len, void **array);

#ifdef __cplusplus
}
#endif
#endif /* DRAID_ISAL_COMPAT_RAID_H */
