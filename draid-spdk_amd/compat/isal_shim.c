/*
 * isal_shim.c -- libdraid_isal.so: isa-l's own symbol names over the MI355X
 * engine, so the reference's call sites link against it in place of libisal
 * (headers: include/isa-l/include/).  One forwarding function per symbol the
 * reference binds: raid5.c:197, raid5_simple.c:134,
 * examples/bdev/gf_vect_mul/gf_vect_mul.c:45,63,65,101,108,168,178,267.
 */
#include "../../include/draid_ec.h"
#include "../../include/isa-l/include/erasure_code.h"
#include "../../include/isa-l/include/gf_vect_mul.h"
#include "../../include/isa-l/include/raid.h"

int xor_gen(int vects, int len, void **array) { return draid_xor_gen(vects, len, array); }
int xor_check(int vects, int len, void **array) { return draid_xor_check(vects, len, array); }
int pq_gen(int vects, int len, void **array) { return draid_pq_gen(vects, len, array); }
int pq_check(int vects, int len, void **array) { return draid_pq_check(vects, len, array); }

int xor_gen_base(int vects, int len, void **array) { return draid_xor_gen(vects, len, array); }
int xor_check_base(int vects, int len, void **array) { return draid_xor_check(vects, len, array); }
int pq_gen_base(int vects, int len, void **array) { return draid_pq_gen(vects, len, array); }
int pq_check_base(int vects, int len, void **array) { return draid_pq_check(vects, len, array); }

void gf_vect_mul_init(unsigned char c, unsigned char *gftbl) { draid_gf_vect_mul_init(c, gftbl); }

int gf_vect_mul(int len, unsigned char *gftbl, void *src, void *dest)
{
    return draid_gf_vect_mul(len, gftbl, src, dest);
}

int gf_vect_mul_base(int len, unsigned char *a, unsigned char *src, unsigned char *dest)
{
    return draid_gf_vect_mul(len, a, src, dest);
}

unsigned char gf_mul(unsigned char a, unsigned char b) { return draid_gf_mul(a, b); }
unsigned char gf_inv(unsigned char a) { return draid_gf_inv(a); }
