// ec_gf.hpp -- GF(2^8) arithmetic for the MI355X erasure-coding engine.
//
// Field: GF(2^8) / x^8+x^4+x^3+x^2+1 (0x11D), generator 2 -- the field isa-l
// v2.30 uses for pq_gen / gf_mul (reference call sites:
// examples/bdev/gf_vect_mul/gf_vect_mul.c:60-66,101,267).
//
// Everything here is byte-parallel integer work on 32-bit VALU lanes: no MFMA.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace draid {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// exp[0..511] (exp[i] = 2^(i mod 255)) and log[0..255] (log[0] unused).
struct GfTables {
    uint8_t exp[512];
    uint8_t log[256];
};

constexpr GfTables make_gf_tables()
{
    GfTables t{};
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
        t.exp[i] = static_cast<uint8_t>(x);
        t.log[x] = static_cast<uint8_t>(i);
        x <<= 1;
        if (x & 0x100u)
            x ^= 0x11Du;
    }
    for (int i = 255; i < 512; ++i)
        t.exp[i] = t.exp[i - 255];
    return t;
}

inline constexpr GfTables kGfHost = make_gf_tables();

// ---- host-side scalar helpers (isa-l ec_base.c gf_mul / gf_inv semantics) ----
inline uint8_t gf_mul_host(uint8_t a, uint8_t b)
{
    if (!a || !b)
        return 0;
    return kGfHost.exp[kGfHost.log[a] + kGfHost.log[b]];
}
inline uint8_t gf_inv_host(uint8_t a) { return a ? kGfHost.exp[255 - kGfHost.log[a]] : 0; }

// ---- device: multiply every byte by 2 (isa-l pq_gen_base word form) ----
// Per byte: (q << 1) ^ (bit 7 set ? 0x1d : 0).  The reduction byte is looked up
// with one v_perm_b32 whose selector is the byte's top bit (entry 0 = 0x00,
// entry 1 = 0x1d): 6 VALU ops per dword (shift, and, perm, shift, and, xor)
// against 8 for the shift-and-subtract mask form.  The reconstruct of a narrow
// stripe is VALU-sensitive: when the shader clock dips under a fresh memory load
// (2.4 -> 1.6 GHz for the first ~10 ms after an idle gap, tools/probe/
// transient_probe.hip) a kernel near the VALU limit slows down with it.
__device__ __forceinline__ uint32_t gf_mul2(uint32_t q)
{
    const uint32_t top = (q >> 7) & 0x01010101u;
    const uint32_t red = __builtin_amdgcn_perm(0u, 0x00001d00u, top);
    return ((q << 1) & 0xfefefefeu) ^ red;
}
__device__ __forceinline__ u32x4 gf_mul2(u32x4 q)
{
    u32x4 r;
    r.x = gf_mul2(q.x);
    r.y = gf_mul2(q.y);
    r.z = gf_mul2(q.z);
    r.w = gf_mul2(q.w);
    return r;
}

// ---- device: multiply by a constant c through isa-l's 32-byte nibble table ----
// lo[w] byte b = c * (4w + b)         (tbl[0..15]  of gf_vect_mul_init)
// hi[w] byte b = c * ((4w + b) << 4)  (tbl[16..31] of gf_vect_mul_init)
// isa-l looks the nibbles up with pshufb; on CDNA4 two v_perm_b32 (8-entry byte
// selects from a register pair) plus a bit-3 blend do the same in registers.
struct NibTable {
    uint32_t lo[4];
    uint32_t hi[4];
};

__host__ __device__ __forceinline__ uint32_t mul2_byte(uint32_t c)
{
    return ((c << 1) ^ ((c & 0x80u) ? 0x1du : 0u)) & 0xffu;
}

// Closed form: with p_b = c * 2^b, word w of the low table holds entries
// 4w..4w+3 = base_w ^ {0, p0, p1, p0^p1}, base_w = (w&1 ? p2 : 0) ^ (w&2 ? p3 : 0);
// the high table is the same over p4..p7.  ~30 scalar ops for both halves (the
// constant is wave-uniform, so this runs on the SALU).
__host__ __device__ __forceinline__ void nib_words(uint32_t p0, uint32_t p1, uint32_t p2,
                                                       uint32_t p3, uint32_t w[4])
{
    const uint32_t t = (p0 << 8) | (p1 << 16) | ((p0 ^ p1) << 24);
    w[0] = t;
    w[1] = t ^ (p2 * 0x01010101u);
    w[2] = t ^ (p3 * 0x01010101u);
    w[3] = t ^ ((p2 ^ p3) * 0x01010101u);

}

__host__ __device__ inline NibTable make_nib_table(uint32_t c)
{
    uint32_t p[8];  // c * 2^i
    p[0] = c & 0xffu;
#pragma unroll
    for (int i = 1; i < 8; ++i)
        p[i] = mul2_byte(p[i - 1]);
    NibTable t;
    nib_words(p[0], p[1], p[2], p[3], t.lo);
    nib_words(p[4], p[5], p[6], p[7], t.hi);
    return t;
}

// 16-entry byte table lookup of the nibble held in every byte of n.
__device__ __forceinline__ uint32_t lut16(const uint32_t t[4], uint32_t n)
{
    const uint32_t sel = n & 0x07070707u;
    const uint32_t a = __builtin_amdgcn_perm(t[1], t[0], sel);  // entries 0..7
    const uint32_t b = __builtin_amdgcn_perm(t[3], t[2], sel);  // entries 8..15
    const uint32_t b3 = n & 0x08080808u;
    const uint32_t m = (b3 << 5) - (b3 >> 3);                   // 0xFF where n >= 8
    return (a & ~m) | (b & m);
}

__device__ __forceinline__ uint32_t gf_mulc(const NibTable& t, uint32_t x)
{
    return lut16(t.lo, x & 0x0f0f0f0fu) ^ lut16(t.hi, (x >> 4) & 0x0f0f0f0fu);
}
__device__ __forceinline__ u32x4 gf_mulc(const NibTable& t, u32x4 x)
{
    u32x4 r;
    r.x = gf_mulc(t, x.x);
    r.y = gf_mulc(t, x.y);
    r.z = gf_mulc(t, x.z);
    r.w = gf_mulc(t, x.w);
    return r;
}

// ---- device: multiply by a wave-uniform constant through 3-bit tables ----
// c * x is linear over GF(2), so x splits into bits 0-2, 3-5 and 6-7 and
//   c * x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6],
// with T0[r] = c*r, T1[r] = c*(r << 3), T2[r] = c*(r << 6).  An 8-entry byte
// table is one register pair, so each term is a single v_perm_b32 with the
// 3-bit field as selector: 9 VALU ops per dword (two shifts, three ands, three
// perms, one three-way xor) against 22 for the two 16-entry nibble lookups.
// The 20 table bytes are built on the SALU from the constant (closed form).
struct MulTable {
    uint32_t t0[2];  // bytes c*0 .. c*7
    uint32_t t1[2];  // bytes c*(0<<3) .. c*(7<<3)
    uint32_t t2;     // bytes c*(0<<6) .. c*(3<<6)
};

// Entries r = 0..7 over the three basis products (pa, pb, pc) = c * 2^{b, b+1, b+2}.
__host__ __device__ __forceinline__ void tri_words(uint32_t pa, uint32_t pb, uint32_t pc,
                                                   uint32_t w[2])
{
    w[0] = (pa << 8) | (pb << 16) | ((pa ^ pb) << 24);
    w[1] = w[0] ^ (pc * 0x01010101u);
}

__host__ __device__ inline MulTable make_mul_table(uint32_t c)
{
    uint32_t p[8];  // c * 2^i
    p[0] = c & 0xffu;
#pragma unroll
    for (int i = 1; i < 8; ++i)
        p[i] = mul2_byte(p[i - 1]);
    MulTable t;
    tri_words(p[0], p[1], p[2], t.t0);
    tri_words(p[3], p[4], p[5], t.t1);
    t.t2 = (p[6] << 8) | (p[7] << 16) | ((p[6] ^ p[7]) << 24);
    return t;
}

__device__ __forceinline__ uint32_t gf_mulc(const MulTable& t, uint32_t x)
{
    const uint32_t s0 = x & 0x07070707u;
    const uint32_t s1 = (x >> 3) & 0x07070707u;
    const uint32_t s2 = (x >> 6) & 0x03030303u;
    return __builtin_amdgcn_perm(t.t0[1], t.t0[0], s0) ^
           __builtin_amdgcn_perm(t.t1[1], t.t1[0], s1) ^ __builtin_amdgcn_perm(0u, t.t2, s2);
}
__device__ __forceinline__ u32x4 gf_mulc(const MulTable& t, u32x4 x)
{
    u32x4 r;
    r.x = gf_mulc(t, x.x);
    r.y = gf_mulc(t, x.y);
    r.z = gf_mulc(t, x.z);
    r.w = gf_mulc(t, x.w);
    return r;
}

}  // namespace draid
