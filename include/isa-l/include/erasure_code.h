/*
 * isa-l/include/erasure_code.h -- the part of the isa-l v2.30 header of that name
 * that the reference uses: the scalar GF(2^8) helpers
 * (examples/bdev/gf_vect_mul/gf_vect_mul.c:3,63,313-322).  isa-l's Reed-Solomon
 * matrix and ec_encode_data entry points are not on the reference's path and
 * are not provided.
 */
#ifndef DRAID_ISAL_COMPAT_ERASURE_CODE_H
#define DRAID_ISAL_COMPAT_ERASURE_CODE_H

#ifdef __cplusplus
extern "C" {
#endif

unsigned char gf_mul(unsigned char a, unsigned char b);
unsigned char gf_inv(unsigned char a);

#ifdef __cplusplus
}
#endif
#endif /* DRAID_ISAL_COMPAT_ERASURE_CODE_H */
