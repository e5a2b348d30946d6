// kern_encode.hpp -- the encode: one wave per item (k_encode) and items shared by several waves (k_encode_split).
// Part of the kernel translation unit (ec_kernels.hip includes these in order); not
// a public interface.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ec_gf.hpp"
#include "ec_launch.hpp"
#include "kern_mem.hpp"
#include "kern_cfg.hpp"

namespace draid {

// ------------------------------------------------------------ encode core

// Computes P (and Q for M == 2) over the U elements i0 + u*stride (< n) and
// either stores them (CHECK == false) or compares them with the stored parity.
// BOUNDED == false: the caller guarantees every element is in range (full
// chunks), so no load or store is predicated.
template <int KT, int M, int U, int POL, bool CHECK, bool BOUNDED, class W, class Ptrs>
__device__ __forceinline__ bool encode_elems(const Ptrs& pp, uint32_t s, int k, uint32_t i0,
                                             uint32_t stride, uint32_t n)
{
    using MW = Mem<W>;
    W p[U], q[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        ok[u] = !BOUNDED || i0 + u * stride < n;
        p[u] = W(0);
        q[u] = W(0);
    }
    if constexpr (KT > 0) {
        for_sources_desc<KT>(k, [&](int j) {
            const uint8_t* src = pp.get(s, j);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const W d = ok[u] ? MW::template ld<POL>(src, i0 + u * stride) : W(0);
                p[u] ^= d;
                if constexpr (M == 2)
                    q[u] = gf_mul2(q[u]) ^ d;
            }
        });
    } else {
        for_blocks_desc<U, POL, W>(
            pp, s, k, ok, i0, stride, [](int) { return true; },
            [&](const W(&d)[U]) __attribute__((always_inline)) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    p[u] ^= d[u];
                    if constexpr (M == 2)
                        q[u] = gf_mul2(q[u]) ^ d[u];
                }
            });
    }
    const uint8_t* dp = pp.get(s, k);
    const uint8_t* dq = (M == 2) ? pp.get(s, k + 1) : nullptr;
    bool bad = false;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (!ok[u])
            continue;
        const uint32_t i = i0 + u * stride;
        if constexpr (CHECK) {
            bad |= MW::any(MW::template ld<0>(dp, i) ^ p[u]);
            if constexpr (M == 2)
                bad |= MW::any(MW::template ld<0>(dq, i) ^ q[u]);
        } else {
            MW::template st<POL>(dp, i, p[u]);
            if constexpr (M == 2)
                MW::template st<POL>(dq, i, q[u]);
        }
    }
    return bad;
}

template <int KT, int M, class Ptrs>
__device__ __forceinline__ bool stripe_aligned(const Ptrs& pp, uint32_t s, int k)
{
    uintptr_t acc = 0;
    if constexpr (KT > 0) {
#pragma unroll
        for (int j = 0; j < KT + M; ++j)
            acc |= reinterpret_cast<uintptr_t>(pp.get(s, j));
    } else {
        for (int j = 0; j < k + M; ++j)
            acc |= reinterpret_cast<uintptr_t>(pp.get(s, j));
    }
    return (acc & 15u) == 0;
}

// One work item = chunk c (NTHR*U vectors) of every strip of stripe s.
template <int KT, int M, bool CHECK, class C, class Ptrs>
__device__ __forceinline__ bool encode_item(const Ptrs& pp, uint32_t s, uint32_t c, int k,
                                            uint32_t len, uint32_t cps)
{
    constexpr int NTHR = C::NTHR, U = C::U, POL = C::POL;
    constexpr uint32_t EPB = static_cast<uint32_t>(NTHR) * U;  // vectors per item
    const uint32_t nvec = len >> 4;
    bool bad = false;
    if (stripe_aligned<KT, M>(pp, s, k)) {
        const uint32_t i0 = c * EPB + threadIdx.x;
        if ((c + 1) * EPB <= nvec)
            bad = encode_elems<KT, M, U, POL, CHECK, false, u32x4>(pp, s, k, i0, NTHR, nvec);
        else
            bad = encode_elems<KT, M, U, POL, CHECK, true, u32x4>(pp, s, k, i0, NTHR, nvec);
        const uint32_t tail = len & 15u;
        if (tail && c == cps - 1 && threadIdx.x < tail)
            bad |= encode_elems<0, M, 1, 0, CHECK, true, uint32_t>(
                pp, s, k, nvec * 16 + threadIdx.x, NTHR, len);
    } else {
        const uint32_t b1 = min(len, (c + 1) * EPB * 16);
        for (uint32_t b = c * EPB * 16 + threadIdx.x; b < b1; b += NTHR)
            bad |= encode_elems<0, M, 1, 0, CHECK, true, uint32_t>(pp, s, k, b, NTHR, b1);
    }
    return bad;
}

template <int KT, int M, bool CHECK, class C, class Ptrs>
__global__ __launch_bounds__(C::NTHR) DRAID_WAVES_PER_EU(C) void k_encode(Ptrs pp, uint32_t k_rt, uint32_t len,
                                                    uint32_t cps, uint32_t nstripes,
                                                    uint32_t* flag)
{
    const int k = KT > 0 ? KT : static_cast<int>(k_rt);
    const uint32_t total = cps * nstripes;
    bool bad = false;
    for (uint32_t b = blockIdx.x; b < total; b += (C::MAP == 2 ? gridDim.x : total)) {
        uint32_t s, c;
        item_coords<C>(b, cps, nstripes, s, c);
        bad |= encode_item<KT, M, CHECK, C>(pp, s, c, k, len, cps);
    }
    if constexpr (CHECK) {
        if (bad)
            atomicOr(flag, 1u);
    }
}

template <int SPLIT>
struct SplitLds {
    u32x4 p[SPLIT][64];
    u32x4 q[SPLIT][64];
};

// 2^e in GF(2^8); e is a compile-time constant wherever this is used, so the
// multiplication table built from it folds into immediates.
__host__ __device__ constexpr uint32_t gf_exp2_const(int e)
{
    uint32_t c = 1;
    for (int i = 0; i < e; ++i)
        c = ((c << 1) ^ ((c & 0x80u) ? 0x1du : 0u)) & 0xffu;
    return c;
}

template <int SPLIT>
__device__ __forceinline__ u32x4 split_sum(const u32x4 (&part)[SPLIT][64], uint32_t lane)
{
    u32x4 a = part[0][lane];
#pragma unroll
    for (int t = 1; t < SPLIT; ++t)
        a ^= part[t][lane];
    return a;
}

// Vector i of every strip: wave 0 ends up storing (or checking) P, the last wave Q.
template <int KT, int M, int SPLIT, int POL, bool CHECK, bool BOUNDED, class Ptrs>
__device__ __forceinline__ bool encode_split_vec(const Ptrs& pp, uint32_t s, uint32_t w,
                                                 uint32_t lane, uint32_t i, uint32_t nvec,
                                                 SplitLds<SPLIT>& lds)
{
    using MW = Mem<u32x4>;
    constexpr int KW = (KT + SPLIT - 1) / SPLIT;
    const bool ok = !BOUNDED || i < nvec;
    // Every pointer is fetched before the barrier: a table read after it can no
    // longer be a scalar load (LDS writes and the barrier count as clobbers).
    const uint8_t* dp = pp.get(s, KT);
    const uint8_t* dq = (M == 2) ? pp.get(s, KT + 1) : dp;
    const PartPQ part = wave_case<0, SPLIT>(w, [=, &pp](auto wc) __attribute__((always_inline)) {
        constexpr int J0 = decltype(wc)::value * KW;
        u32x4 p = 0, q = 0;
#pragma unroll
        for (int j = KW - 1; j >= 0; --j) {
            u32x4 d = 0;
            if (J0 + j < KT && ok)
                d = MW::template ld<POL>(pp.get(s, J0 + j), i);
            p ^= d;
            if constexpr (M == 2)
                q = gf_mul2(q) ^ d;
        }
        if constexpr (M == 2 && J0 != 0)
            q = gf_mulc(make_mul_table(gf_exp2_const(J0)), q);
        return PartPQ{p, q};
    });
    lds.p[w][lane] = part.p;
    if constexpr (M == 2)
        lds.q[w][lane] = part.q;
    __syncthreads();
    bool bad = false;
    if (w == 0) {
        const u32x4 a = split_sum<SPLIT>(lds.p, lane);
        if (ok) {
            if constexpr (CHECK)
                bad = MW::any(MW::template ld<0>(dp, i) ^ a);
            else
                MW::template st<POL>(dp, i, a);
        }
    }
    if constexpr (M == 2) {
        if (w == SPLIT - 1) {
            const u32x4 a = split_sum<SPLIT>(lds.q, lane);
            if (ok) {
                if constexpr (CHECK)
                    bad = MW::any(MW::template ld<0>(dq, i) ^ a);
                else
                    MW::template st<POL>(dq, i, a);
            }
        }
    }
    return bad;
}

// The 16-byte vectors go through the split path; a byte tail (len % 16) and
// strips that are not 16-byte aligned take the one-wave byte path on wave 0.
template <int KT, int M, bool CHECK, class C, class Ptrs>
__device__ __forceinline__ bool encode_item_split(const Ptrs& pp, uint32_t s, uint32_t c,
                                                  uint32_t len, uint32_t cps,
                                                  SplitLds<C::SPLIT>& lds)
{
    constexpr int SPLIT = C::SPLIT, POL = C::POL;
    constexpr uint32_t L = 64;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t nvec = len >> 4;
    bool bad = false;
    if (stripe_aligned<KT, M>(pp, s, KT)) {
        const uint32_t i = c * L + lane;
        if ((c + 1) * L <= nvec)
            bad = encode_split_vec<KT, M, SPLIT, POL, CHECK, false>(pp, s, w, lane, i, nvec, lds);
        else
            bad = encode_split_vec<KT, M, SPLIT, POL, CHECK, true>(pp, s, w, lane, i, nvec, lds);
        const uint32_t tail = len & 15u;
        if (w == 0 && tail && c == cps - 1 && lane < tail)
            bad |= encode_elems<0, M, 1, 0, CHECK, true, uint32_t>(pp, s, KT, nvec * 16 + lane, L,
                                                                    len);
    } else if (w == 0) {
        const uint32_t b1 = min(len, (c + 1) * L * 16);
        for (uint32_t b = c * L * 16 + lane; b < b1; b += L)
            bad |= encode_elems<0, M, 1, 0, CHECK, true, uint32_t>(pp, s, KT, b, L, b1);
    }
    return bad;
}

template <int KT, int M, bool CHECK, class C, class Ptrs>
__global__ __launch_bounds__(C::NTHR) DRAID_WAVES_PER_EU(C) void k_encode_split(
    Ptrs pp, uint32_t len, uint32_t cps, uint32_t nstripes, uint32_t* flag, ItemGrid ig)
{
    static_assert(KT > 0 && C::SPLIT > 1 && C::MAP == 0, "one split item per workgroup, stripe order");
    __shared__ SplitLds<C::SPLIT> lds;
    uint32_t c, s;
    ig.coords(c, s);
    if (s >= nstripes)
        return;  // uniform: the ragged last z-slice
    const bool bad = encode_item_split<KT, M, CHECK, C>(pp, s, c, len, cps, lds);
    if constexpr (CHECK) {
        if (bad)
            atomicOr(flag, 1u);
    }
}

}  // namespace draid
