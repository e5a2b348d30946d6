/*
 * isa-l/include/gf_vect_mul.h -- drop-in for the isa-l v2.30 header of that name
 * (used by examples/bdev/gf_vect_mul/gf_vect_mul.c:2,65,108,158,...).  Forwards
 * to draid_gf_vect_mul_init / draid_gf_vect_mul (include/draid_ec.h).
 */
#ifndef DRAID_ISAL_COMPAT_GF_VECT_MUL_H
#define DRAID_ISAL_COMPAT_GF_VECT_MUL_H

#ifdef __cplusplus
extern "C" {
#endif

/* The 32-byte table of constant c: c * (0..15) then c * (0..15 << 4). */
void gf_vect_mul_init(unsigned char c, unsigned char *gftbl);
/* dest = c * src over len bytes (len % 32 == 0), c given by its table. */
int gf_vect_mul(int len, unsigned char *gftbl, void *src, void *dest);
int gf_vect_mul_base(int len, unsigned char *a, unsigned char *src, unsigned char *dest);

#ifdef __cplusplus
}
#endif
#endif /* DRAID_ISAL_COMPAT_GF_VECT_MUL_H */
