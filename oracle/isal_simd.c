/*
 * isal_simd.c -- AVX-512 restatement of the isa-l v2.30 parity kernels, for the
 * CPU baseline only (bench.py cpu_baseline, kind "port").  TEST INFRASTRUCTURE:
 * never linked into libdraid_ec.so.
 *
 * isa-l's own x86 paths (raid/pq_gen_avx512.asm, erasure_code/gf_vect_mul_avx512
 * and the GFNI variants of later releases) are not in /root/reference (empty
 * submodule); this file restates their published algorithms:
 *   pq_gen : 64-byte vectors, Q by Horner with mul2(q) = (q + q) ^ (0x1D where the
 *            byte's top bit was set)  -- the vpaddb / vpcmpb / vpblendmb sequence
 *   c * x  : a constant GF(2^8)/0x11D multiply is GF(2)-linear, applied as one
 *            8x8 bit-matrix affine transform per byte (gf2p8affineqb); GFNI's own
 *            gf2p8mulb uses the AES polynomial 0x11B and cannot be used directly.
 * Recovery follows the same cases as orc_recover (isal_oracle.c, itself citing
 * raid5.c:557-569 and gf_vect_mul.c:255-330).  Byte-exact against the scalar
 * oracle (tests/test_oracle.py::test_simd_matches_scalar).
 */
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

#include "isal_oracle.h"

#define SIMD_TARGET __attribute__((target("avx512f,avx512bw,gfni")))

int orc_simd_available(void)
{
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
           __builtin_cpu_supports("gfni");
}

/* Bit matrix of x -> c*x for gf2p8affineqb: output bit i = parity(row_i & x),
 * row_i stored in byte 7-i; bit j of row_i = bit i of c * 2^j. */
static uint64_t affine_of(unsigned char c)
{
    uint64_t a = 0;
    for (int i = 0; i < 8; i++) {
        unsigned row = 0;
        for (int j = 0; j < 8; j++)
            if ((orc_gf_mul(c, (unsigned char)(1u << j)) >> i) & 1u)
                row |= 1u << j;
        a |= (uint64_t)row << (8 * (7 - i));
    }
    return a;
}

SIMD_TARGET static inline __m512i mul2(__m512i q)
{
    const __mmask64 hi = _mm512_movepi8_mask(q);
    return _mm512_xor_si512(_mm512_add_epi8(q, q),
                            _mm512_maskz_mov_epi8(hi, _mm512_set1_epi8(0x1d)));
}

SIMD_TARGET static inline __m512i mulc(__m512i x, __m512i a)
{
    return _mm512_gf2p8affine_epi64_epi8(x, a, 0);
}

SIMD_TARGET static inline __m512i ld(const unsigned char *p) { return _mm512_loadu_si512(p); }
SIMD_TARGET static inline void st(unsigned char *p, __m512i v) { _mm512_storeu_si512(p, v); }

/* P (+Q) of one stripe: v[0..k) data, v[k] P, v[k+1] Q; len % 64 handled by
 * the scalar oracle. */
SIMD_TARGET static int encode_one(int k, int m, size_t len, unsigned char **v)
{
    const size_t body = len & ~(size_t)63;
    for (size_t i = 0; i < body; i += 64) {
        __m512i p = ld(v[k - 1] + i), q = p;
        for (int j = k - 2; j >= 0; j--) {
            const __m512i d = ld(v[j] + i);
            p = _mm512_xor_si512(p, d);
            if (m == 2)
                q = _mm512_xor_si512(mul2(q), d);
        }
        st(v[k] + i, p);
        if (m == 2)
            st(v[k + 1] + i, q);
    }
    for (size_t i = body; i < len; i++) {  /* bytewise tail */
        unsigned char p = v[k - 1][i], q = p;
        for (int j = k - 2; j >= 0; j--) {
            p ^= v[j][i];
            q = (unsigned char)(((q << 1) ^ ((q & 0x80) ? 0x1d : 0)) ^ v[j][i]);
        }
        v[k][i] = p;
        if (m == 2)
            v[k + 1][i] = q;
    }
    return 0;
}

SIMD_TARGET static int recover_one(int k, int m, size_t len, unsigned char **v, int nfail,
                                   const int *fail)
{
    int lost[2] = { -1, -1 }, nd = 0, lostP = 0, lostQ = 0;
    for (int f = 0; f < nfail; f++) {
        const int j = fail[f];
        if (j < 0 || j >= k + m)
            return -1;
        if (j < k) {
            if (nd == 1 && lost[0] == j)
                return -1;
            lost[nd++] = j;
        } else if (j == k) {
            lostP = 1;
        } else {
            lostQ = 1;
        }
    }
    if (nd == 2 && lost[0] > lost[1]) {
        const int t = lost[0];
        lost[0] = lost[1];
        lost[1] = t;
    }
    const int x = lost[0], y = lost[1];
    const int needq = (nd == 2) || (nd == 1 && lostP) || lostQ;
    uint64_t a1 = 0, a2 = 0;
    if (nd == 1 && !lostP) {
        a1 = affine_of(orc_gf_pow2(x));
    } else if (nd == 1) {
        a1 = affine_of(orc_gf_pow2(255 - x));
    } else if (nd == 2) {
        const unsigned char gyx = orc_gf_pow2(y - x);
        const unsigned char den = orc_gf_inv((unsigned char)(gyx ^ 1));
        a1 = affine_of(orc_gf_mul(gyx, den));
        a2 = affine_of(orc_gf_mul(orc_gf_pow2(255 - x), den));
    }
    const __m512i A1 = _mm512_set1_epi64((long long)a1), A2 = _mm512_set1_epi64((long long)a2);
    const size_t body = len & ~(size_t)63;
    for (size_t i = 0; i < body; i += 64) {
        __m512i ps = _mm512_setzero_si512(), qs = ps;
        for (int j = k - 1; j >= 0; j--) {
            const __m512i d = (j != x && j != y) ? ld(v[j] + i) : _mm512_setzero_si512();
            ps = _mm512_xor_si512(ps, d);
            if (needq)
                qs = _mm512_xor_si512(mul2(qs), d);
        }
        if (nd == 0) {
            if (lostP)
                st(v[k] + i, ps);
            if (lostQ)
                st(v[k + 1] + i, qs);
        } else if (nd == 1) {
            if (!lostP) {
                const __m512i dx = _mm512_xor_si512(ld(v[k] + i), ps);
                st(v[x] + i, dx);
                if (lostQ)
                    st(v[k + 1] + i, _mm512_xor_si512(qs, mulc(dx, A1)));
            } else {
                const __m512i dx = mulc(_mm512_xor_si512(ld(v[k + 1] + i), qs), A1);
                st(v[x] + i, dx);
                st(v[k] + i, _mm512_xor_si512(ps, dx));
            }
        } else {
            const __m512i pxy = _mm512_xor_si512(ld(v[k] + i), ps);
            const __m512i qxy = _mm512_xor_si512(ld(v[k + 1] + i), qs);
            const __m512i dx = _mm512_xor_si512(mulc(pxy, A1), mulc(qxy, A2));
            st(v[x] + i, dx);
            st(v[y] + i, _mm512_xor_si512(pxy, dx));
        }
    }
    if (body < len) {
        void *t[2 + 255];
        for (int j = 0; j < k + m; j++)
            t[j] = v[j] + body;
        return orc_recover(k, m, (int)(len - body), t, nfail, fail);
    }
    return 0;
}

/* xor_gen(vects, len, array) (isa-l raid.h semantics, xor_gen_avx512): the last
 * pointer receives the XOR of the others; any length (bytewise tail). */
SIMD_TARGET int orc_simd_xor_gen(int vects, int len, void **array)
{
    if (vects < 3 || len < 0)
        return 1;
    unsigned char **v = (unsigned char **)array;
    const int k = vects - 1;
    const size_t body = (size_t)len & ~(size_t)63;
    for (size_t i = 0; i < body; i += 64) {
        __m512i p = ld(v[0] + i);
        for (int j = 1; j < k; j++)
            p = _mm512_xor_si512(p, ld(v[j] + i));
        st(v[k] + i, p);
    }
    for (size_t i = body; i < (size_t)len; i++) {
        unsigned char p = v[0][i];
        for (int j = 1; j < k; j++)
            p ^= v[j][i];
        v[k][i] = p;
    }
    return 0;
}

int orc_simd_encode_strided(int k, int m, size_t len, uint32_t nstripes, uint8_t *base,
                            size_t strip_stride, size_t stripe_stride)
{
    if (k < 1 || k > 255 || m < 1 || m > 2 || !orc_simd_available())
        return -1;
    unsigned char *v[2 + 255];
    for (uint32_t s = 0; s < nstripes; s++) {
        for (int j = 0; j < k + m; j++)
            v[j] = base + (size_t)s * stripe_stride + (size_t)j * strip_stride;
        if (encode_one(k, m, len, v))
            return -1;
    }
    return 0;
}

int orc_simd_recover_strided(int k, int m, size_t len, uint32_t nstripes, uint8_t *base,
                             size_t strip_stride, size_t stripe_stride, const uint8_t *fail)
{
    if (k < 1 || k > 255 || m < 1 || m > 2 || !orc_simd_available())
        return -1;
    unsigned char *v[2 + 255];
    for (uint32_t s = 0; s < nstripes; s++) {
        int f[2], nf = 0;
        for (int t = 0; t < 2; t++) {
            const int j = fail[2 * (size_t)s + t];
            if (j < k + m && !(t == 1 && nf == 1 && f[0] == j))
                f[nf++] = j;
        }
        if (nf == 0 || nf > m)
            continue;  /* nothing to do / unrecoverable: left untouched */
        for (int j = 0; j < k + m; j++)
            v[j] = base + (size_t)s * stripe_stride + (size_t)j * strip_stride;
        if (recover_one(k, m, len, v, nf, f))
            return -1;
    }
    return 0;
}
