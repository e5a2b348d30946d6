// kern_mem.hpp -- strip pointer providers, 16-byte and byte memory accesses with their cache policies, strip loops.
// Part of the kernel translation unit (ec_kernels.hip includes these in order); not
// a public interface.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ec_gf.hpp"
#include "ec_launch.hpp"

namespace draid {

// ------------------------------------------------------------ pointers

// AS4: read the table through the constant address space.  The table is input
// only, and a constant-space read at a wave-uniform index is always a scalar load
// (an ordinary global read becomes a per-lane load as soon as any store, atomic,
// LDS write or barrier precedes it, and its pointer then lives in VGPRs).  The
// split kernels and every reconstruct need that; the one-wave encode (k = 2, the
// runtime-k fallback, the check kernels) ran 2% faster on ordinary reads (4+1 x
// 64 KiB 203.2 vs 207.4 us), which the compiler already turns into scalar loads
// there.
#ifndef DRAID_KEEP_POINTERS
#define DRAID_KEEP_POINTERS 1
#endif
template <bool AS4>
struct TablePtrsT {
    const uint8_t* const* tab;
    uint32_t stride;
    __device__ __forceinline__ const uint8_t* get(uint32_t s, int j) const
    {
        if constexpr (AS4) {
            typedef const uint8_t* const __attribute__((address_space(4)))* ctab;
            const uint8_t* p = ((ctab)(uintptr_t)tab)[(size_t)s * stride + j];
#if DRAID_KEEP_POINTERS
            // Opaque to the register allocator: a constant-space load is trivially
            // rematerialisable, and under SGPR pressure the compiler re-read the whole
            // pointer row (s_load_dwordx16 + wait) in front of EVERY strip load of
            // the one-wave reconstruct, serialising the loads behind scalar round trips.
            asm("" : "+s"(p));
#endif
            return p;
        } else {
            return tab[(size_t)s * stride + j];
        }
    }
};
#if defined(DRAID_TABLE_PLAIN)
using TablePtrs = TablePtrsT<false>;
#else
using TablePtrs = TablePtrsT<true>;
#endif
using TablePlain = TablePtrsT<false>;

// Regular layout: strip j of stripe s at base + s*stripe_stride + j*strip_stride
// (a stripe cache laid out as one array, or pinned host stripes read in place).
struct StridedPtrs {
    const uint8_t* base;
    uint64_t strip_stride, stripe_stride;
    __device__ __forceinline__ const uint8_t* get(uint32_t s, int j) const
    {
        return base + s * stripe_stride + static_cast<uint64_t>(j) * strip_stride;
    }
};

// Compact rows of the scatter-gather lists (ec_ctx.cpp): segment s is
//   [8-byte base pointer][int32 offset of strip 0, 1, ... from it][anything]
// row_bytes apart -- a little over half the bytes of a row of 64-bit pointers,
// which is what a batch of short runs spends its PCIe upload on.  Read through the
// constant address space like the pointer table: scalar loads, the strip base in
// SGPRs.
struct RowOffs {
    const uint8_t* rows;
    uint32_t row_bytes;
    __device__ __forceinline__ const uint8_t* get(uint32_t s, int j) const
    {
        typedef const uint8_t* const __attribute__((address_space(4)))* cbase;
        typedef const int32_t __attribute__((address_space(4)))* coff;
        const uintptr_t row = reinterpret_cast<uintptr_t>(rows) + static_cast<size_t>(s) * row_bytes;
        const uint8_t* p = ((cbase)row)[0] + ((coff)(row + 8))[j];
#if DRAID_KEEP_POINTERS
        asm("" : "+s"(p));
#endif
        return p;
    }
};

struct ArgPtrs {
    ArgPtrTable t;
    __device__ __forceinline__ const uint8_t* get(uint32_t, int j) const { return t.p[j]; }
};

// ------------------------------------------------------------ memory words

// Strip pointers come from a table of generic pointers; casting to the global
// address space lets the compiler emit global_load/store with the uniform strip
// base in SGPRs and a 32-bit per-lane offset (saddr + voffset form) instead of
// flat instructions with 64-bit per-lane addresses.
typedef const u32x4 __attribute__((address_space(1)))* gcv4;
typedef u32x4 __attribute__((address_space(1)))* gv4;
typedef const uint8_t __attribute__((address_space(1)))* gcb;
typedef uint8_t __attribute__((address_space(1)))* gb;

// W = u32x4: one 16-byte vector, index in vectors.  W = uint32_t: one byte
// held in the low 8 bits, index in bytes (tails and unaligned strips).
// Indices are 32-bit: strips are < 4 GiB (checked on the host).
//
// POL (cache policy of the 16-byte accesses): bit 0 non-temporal loads, bit 1
// non-temporal stores (global instructions).  Bits 8..15 / 16..23 select
// buffer instructions instead, with explicit gfx950 cache-policy bits
// (aux = sc0 1 | nt 2 | sc1 16): load aux + 1 / store aux + 1 (0 = global form).
// The production policies (EncCfg / RecCfg below) are two of these.
constexpr int pol_aux(int load_aux, int store_aux)
{
    return 3 | ((load_aux + 1) << 8) | ((store_aux + 1) << 16);
}

// 1: the shared-item reconstruct loads a strip it skips (lost, or not needed)
// through a descriptor with no records instead of branching around the load
// (Mem<u32x4>::ld_if): 16+2 x 256 KiB dual 380 vs 389 us.  The one-wave
// reconstruct keeps its uniform branches -- there the same change is neutral to
// 1% slower (8+2 x 128 KiB single 377.6 vs 374.1, 4+1 207.6 vs 204.0).  0 for A/B.
#ifndef DRAID_DEAD_LOADS
#define DRAID_DEAD_LOADS 1
#endif

template <class W>
struct Mem;

template <>
struct Mem<u32x4> {
    static __device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const uint8_t* p)
    {
        // p is wave-uniform (a strip base), so the descriptor lives in SGPRs
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p), 0, 0x7fffffff,
                                                 0x00020000);
    }
    template <int POL>
    static __device__ __forceinline__ u32x4 ld(const uint8_t* p, uint32_t i)
    {
        constexpr int aux = (POL >> 8) & 0xff;
        if constexpr (aux != 0)
            return __builtin_amdgcn_raw_buffer_load_b128(rsrc(p), static_cast<int>(i << 4), 0,
                                                         aux - 1);
        gcv4 q = (gcv4)(p + (i << 4));
        if constexpr ((POL & 1) != 0)
            return __builtin_nontemporal_load(q);
        else
            return *q;
    }
    // Loads vector i when `live` (wave-uniform), zeros otherwise.  Through a buffer
    // descriptor a dead load is one with no records -- it returns zeros without
    // touching memory -- so a skipped strip costs neither a branch nor the moves
    // that zero its registers.
    template <int POL>
    static __device__ __forceinline__ u32x4 ld_if(const uint8_t* p, uint32_t i, bool live)
    {
        constexpr int aux = (POL >> 8) & 0xff;
        if constexpr (aux != 0 && DRAID_DEAD_LOADS) {
            const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint8_t*>(p), 0, live ? 0x7fffffff : 0, 0x00020000);
            return __builtin_amdgcn_raw_buffer_load_b128(r, static_cast<int>(i << 4), 0, aux - 1);
        } else {
            return live ? ld<POL>(p, i) : u32x4(0);
        }
    }
    template <int POL>
    static __device__ __forceinline__ void st(const uint8_t* p, uint32_t i, u32x4 v)
    {
        constexpr int aux = (POL >> 16) & 0xff;
        if constexpr (aux != 0) {
            __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(p), static_cast<int>(i << 4), 0,
                                                   aux - 1);
            return;
        }
        gv4 q = (gv4)(const_cast<uint8_t*>(p) + (i << 4));
        if constexpr ((POL & 2) != 0)
            __builtin_nontemporal_store(v, q);
        else
            *q = v;
    }
    static __device__ __forceinline__ bool any(u32x4 v) { return (v.x | v.y | v.z | v.w) != 0; }
};

template <>
struct Mem<uint32_t> {
    template <int POL>
    static __device__ __forceinline__ uint32_t ld(const uint8_t* p, uint32_t i)
    {
        return *((gcb)p + i);
    }
    template <int POL>
    static __device__ __forceinline__ uint32_t ld_if(const uint8_t* p, uint32_t i, bool live)
    {
        return live ? ld<POL>(p, i) : 0u;
    }
    template <int POL>
    static __device__ __forceinline__ void st(const uint8_t* p, uint32_t i, uint32_t v)
    {
        *((gb)const_cast<uint8_t*>(p) + i) = static_cast<uint8_t>(v);
    }
    static __device__ __forceinline__ bool any(uint32_t v) { return (v & 0xffu) != 0; }
};

// ND (1 or 2) consecutive dwords at a byte offset, with the store policy of POL.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <int POL, int ND>
__device__ __forceinline__ void st_words(const uint8_t* p, uint32_t byte_off,
                                         const uint32_t (&v)[ND])
{
    static_assert(ND == 1 || ND == 2, "a dword or a pair");
    constexpr int aux = (POL >> 16) & 0xff;
    if constexpr (aux != 0) {
        if constexpr (ND == 1)
            __builtin_amdgcn_raw_buffer_store_b32(v[0], Mem<u32x4>::rsrc(p),
                                                  static_cast<int>(byte_off), 0, aux - 1);
        else
            __builtin_amdgcn_raw_buffer_store_b64(u32x2{v[0], v[1]}, Mem<u32x4>::rsrc(p),
                                                  static_cast<int>(byte_off), 0, aux - 1);
    } else {
        typedef uint32_t __attribute__((address_space(1)))* gw;
        gw q = (gw)(const_cast<uint8_t*>(p) + byte_off);
#pragma unroll
        for (int n = 0; n < ND; ++n) {
            if constexpr ((POL & 2) != 0)
                __builtin_nontemporal_store(v[n], q + n);
            else
                q[n] = v[n];
        }
    }
}

// Calls f(j) for j = k-1 down to 0; fully unrolled when k is a template constant.
template <int KT, class F>
__device__ __forceinline__ void for_sources_desc(int k, F&& f)
{
    if constexpr (KT > 0) {
#pragma unroll
        for (int j = KT - 1; j >= 0; --j)
            f(j);
    } else {
        for (int j = k - 1; j >= 0; --j)
            f(j);
    }
}

// Run-time stripe width (k without an unrolled instance): the strips in blocks of
// kRtBlock, from the top down, every load of a block issued before the block's
// arithmetic -- a plain loop over j would wait for each strip before asking for
// the next.  The top block may reach past strip k-1: those slots load nothing
// (ld_if with live == false, through the pointer of strip k-1, never one past the
// row) and hand zeros to acc, which a Horner chain that is still zero ignores.
// live(j): wave-uniform, false for a strip that must not be read.
constexpr int kRtBlock = 8;
template <int U, int POL, class W, class Ptrs, class Live, class Acc>
__device__ __forceinline__ void for_blocks_desc(const Ptrs& pp, uint32_t s, int k,
                                                const bool (&ok)[U], uint32_t i0,
                                                uint32_t stride, Live&& live, Acc&& acc)
{
    using MW = Mem<W>;
    for (int jb = ((k + kRtBlock - 1) / kRtBlock) * kRtBlock; jb > 0; jb -= kRtBlock) {
        W d[kRtBlock][U];
#pragma unroll
        for (int t = kRtBlock - 1; t >= 0; --t) {
            const int j = jb - kRtBlock + t;
            const bool on = j < k && live(j);
            const uint8_t* src = pp.get(s, j < k ? j : k - 1);
#pragma unroll
            for (int u = 0; u < U; ++u)
                d[t][u] = ok[u] ? MW::template ld_if<POL>(src, i0 + u * stride, on) : W(0);
        }
#pragma unroll
        for (int t = kRtBlock - 1; t >= 0; --t)
            acc(d[t]);
    }
}

}  // namespace draid
