// kern_worklist.hpp -- scatter-gather work-list kernels, the read-modify-write update, gf_vect_mul.
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
#include "kern_encode.hpp"
#include "kern_reconstruct.hpp"

namespace draid {

// ------------------------------------------------------------ segment work lists

// Scatter-gather form (ec_ctx.cpp): a batch of variable-length segments, each
// one contiguous run across the k+m strips of a stripe (what raid5_xor_stripe,
// raid5_simple.c:141-203, hands to one xor_gen call).  The host expands the
// segments into work items (segment, chunk) so one launch covers them all.
struct WorkItem {
    uint32_t seg;
    uint32_t chunk;
};

// Where work item b comes from: an explicit (segment, chunk) list, or -- when
// every queued segment has the same length (full-strip runs, fixed-size iovecs)
// -- arithmetic, so the item costs no descriptor load at all.
struct WorkSrc {
    const WorkItem* list;      // nullptr: uniform segments
    const uint32_t* seg_len;   // list mode
    uint32_t ulen, ucps;       // uniform mode: segment length, items per segment
    __device__ __forceinline__ void get(uint32_t b, uint32_t cb, uint32_t& seg, uint32_t& chunk,
                                        uint32_t& len, uint32_t& cps) const
    {
        if (list) {
            const WorkItem w = list[b];
            seg = w.seg;
            chunk = w.chunk;
            len = seg_len[seg];
            cps = (len + cb - 1) / cb;
        } else {
            seg = b / ucps;
            chunk = b - seg * ucps;
            len = ulen;
            cps = ucps;
        }
    }
};

// Pointer-table reads of the one-wave work-list encode: ordinary reads for a
// compiled width (the compiler makes them scalar loads, measured 2% faster than
// constant-space reads there), constant-space reads for a run-time width, whose
// strip index is a loop variable.
template <int KT>
using WorkEncPtrs = std::conditional_t<(KT > 0), TablePlain, TablePtrs>;

template <int KT, int M, bool CHECK, class C, class P = WorkEncPtrs<KT>>
__global__ __launch_bounds__(C::NTHR) DRAID_WAVES_PER_EU(C) void k_encode_work(
    P pp, uint32_t k_rt, WorkSrc ws, uint32_t nwork)
{
    constexpr uint32_t CB = static_cast<uint32_t>(C::NTHR) * C::U * 16;
    const int k = KT > 0 ? KT : static_cast<int>(k_rt);
    for (uint32_t b = blockIdx.x; b < nwork; b += gridDim.x) {
        uint32_t seg, chunk, len, cps;
        ws.get(b, CB, seg, chunk, len, cps);
        encode_item<KT, M, CHECK, C>(pp, seg, chunk, k, len, cps);
    }
}

// The shared-item encode over a segment list: one workgroup per work item.
template <int KT, int M, class C, class P = TablePtrs>
__global__ __launch_bounds__(C::NTHR) DRAID_WAVES_PER_EU(C) void k_encode_work_split(
    P pp, WorkSrc ws, uint32_t nwork)
{
    static_assert(KT > 0 && C::SPLIT > 1, "shared items need a compile-time width");
    constexpr uint32_t CB = static_cast<uint32_t>(C::ITEM) * C::U * 16;
    __shared__ SplitLds<C::SPLIT> lds;
    uint32_t seg, chunk, len, cps;
    ws.get(blockIdx.x, CB, seg, chunk, len, cps);
    encode_item_split<KT, M, false, C>(pp, seg, chunk, len, cps, lds);
}

template <int KT, int M, class C, class P = TablePtrs>
__global__ __launch_bounds__(C::NTHR) DRAID_WAVES_PER_EU(C) void k_reconstruct_work(P pp, uint32_t k_rt,
                                                              WorkSrc ws, const uint8_t* fail,
                                                              uint32_t fstride, uint32_t nwork)
{
    __shared__ LdsGf lds;
    const uint8_t* l_exp = reinterpret_cast<const uint8_t*>(lds.w);
    const uint8_t* l_log = l_exp + 512;
    constexpr uint32_t CB = static_cast<uint32_t>(C::NTHR) * C::U * 16;
    const int k = KT > 0 ? KT : static_cast<int>(k_rt);
    TabStage<C::NTHR> tabs;
    if constexpr (M == 2)
        tabs.load();
    for (uint32_t b = blockIdx.x; b < nwork; b += gridDim.x) {
        uint32_t seg, chunk, len, cps;
        ws.get(b, CB, seg, chunk, len, cps);
        const uint8_t* f = fail + static_cast<size_t>(fstride) * seg;
        RecPlan pl = decode_failures<M>(k, f[0], f[1]);
        if (pl.skip)
            continue;
        if constexpr (M == 1) {
            reconstruct_item<KT, M, C>(pp, seg, chunk, k, len, cps, pl, [](RecPlan&) {});
        } else {
            reconstruct_item<KT, M, C>(pp, seg, chunk, k, len, cps, pl, [&](RecPlan& p) {
                tabs.store(lds);
                plan_constants(p, l_exp, l_log);
            });
        }
    }
}

// The column reconstruct over a segment list: one workgroup per work item.  The
// failure pair rides at a row stride beside the segment's pointers.
template <int KT, int M, class C, class P = TablePtrs>
__global__ __launch_bounds__(C::NTHR) DRAID_WAVES_PER_EU(C) void k_reconstruct_work_cols(
    P pp, WorkSrc ws, const uint8_t* fail, uint32_t fstride, uint32_t nwork)
{
    static_assert(KT > 0 && C::SPLIT > 1, "shared items need a compile-time width");
    constexpr uint32_t CB = static_cast<uint32_t>(C::ITEM) * C::U * 16;
    __shared__ ColLds<KT> lds;
    uint32_t seg, chunk, len, cps;
    ws.get(blockIdx.x, CB, seg, chunk, len, cps);
    const bool aligned = stripe_aligned<KT, M>(pp, seg, KT);  // pointer row and pair read together
    const uint32_t f = load_fail_pair_at(fail + static_cast<size_t>(fstride) * seg);
    RecPlan pl = decode_failures_mask<KT, M>(f & 0xffu, f >> 8);
    if (!pl.skip)  // uniform across the workgroup
        reconstruct_item_cols<KT, M, C>(pp, seg, chunk, len, cps, pl, aligned, lds);
}

// ------------------------------------------------------------ read-modify-write

// Small-write parity update (raid5_stripe_write_preread_complete_rmw,
// raid5.c:705-741, extended to Q): for the nd data chunks a segment touches,
// with old contents O_i and new contents N_i at data index e_i,
//   P' = P ^ XOR_i (O_i ^ N_i),   Q' = Q ^ XOR_i 2^{e_i} (O_i ^ N_i).
// Each 2^{e_i} is a constant multiplication through the ready-made table of that
// power (c_plan.mul, a scalar read): 9 VALU operations per dword whatever the
// exponent, against up to k-1 doublings of 6.
// Segment table row: [O_0, N_0, O_1, N_1, ..., P, (Q)]; exps row: e_0, e_1, ...
// The row and the exponents are read through the constant address space, so the
// strip bases stay in SGPRs (a base in VGPRs costs a readfirstlane loop around
// every buffer access).  NDT = 1, 2: nd at compile time, every load of the item
// issued before the first use; NDT = 0: run-time nd.

// Byte idx of a device byte array that the kernel never writes: a scalar load of
// the aligned word around it.
__device__ __forceinline__ uint32_t load_const_byte(const uint8_t* a, size_t idx)
{
    const uintptr_t p = reinterpret_cast<uintptr_t>(a) + idx;
    typedef const uint32_t __attribute__((address_space(4)))* ccw;
    const uint32_t w = ((ccw)(p & ~static_cast<uintptr_t>(3)))[0];
    return (w >> ((static_cast<uint32_t>(p) & 3u) * 8u)) & 0xffu;
}

template <int M, int NDT, class C>
__device__ __forceinline__ void update_item(const uint8_t* const* tab, uint32_t nd_rt,
                                            const uint8_t* exps, const WorkSrc& ws, uint32_t b)
{
    constexpr uint32_t EPB = static_cast<uint32_t>(C::NTHR) * C::U;
    static_assert(C::U == 1, "one vector per lane");
    const uint32_t nd = NDT > 0 ? NDT : nd_rt;
    uint32_t seg, chunk, len, cps;
    ws.get(b, EPB * 16, seg, chunk, len, cps);
    const TablePtrs row{tab, 2 * nd + M};
    const uint8_t* pP = row.get(seg, static_cast<int>(2 * nd));
    const uint8_t* pQ = M == 2 ? row.get(seg, static_cast<int>(2 * nd + 1)) : pP;
    uintptr_t acc = reinterpret_cast<uintptr_t>(pP) | reinterpret_cast<uintptr_t>(pQ);
    if constexpr (NDT > 0) {
#pragma unroll
        for (int t = 0; t < 2 * NDT; ++t)
            acc |= reinterpret_cast<uintptr_t>(row.get(seg, t));
    } else {
        for (uint32_t t = 0; t < 2 * nd; ++t)
            acc |= reinterpret_cast<uintptr_t>(row.get(seg, static_cast<int>(t)));
    }
    const size_t e0 = static_cast<size_t>(seg) * nd;
    auto body = [&](auto tag, uint32_t i) __attribute__((always_inline)) {
        using W = decltype(tag);
        using MW = Mem<W>;
        W dp = W(0), dq = W(0);
        if constexpr (NDT > 0) {
            W o[NDT], n[NDT];
#pragma unroll
            for (int t = 0; t < NDT; ++t) {
                o[t] = MW::template ld<C::POL>(row.get(seg, 2 * t), i);
                n[t] = MW::template ld<C::POL>(row.get(seg, 2 * t + 1), i);
            }
            const W p0 = MW::template ld<C::POL>(pP, i);
            const W q0 = M == 2 ? MW::template ld<C::POL>(pQ, i) : W(0);
#pragma unroll
            for (int t = 0; t < NDT; ++t) {
                const W delta = o[t] ^ n[t];
                dp ^= delta;
                if constexpr (M == 2)
                    dq ^= gf_mulc(mul_table_exp2(load_const_byte(exps, e0 + t)), delta);
            }
            MW::template st<C::POL>(pP, i, p0 ^ dp);
            if constexpr (M == 2)
                MW::template st<C::POL>(pQ, i, q0 ^ dq);
        } else {
            const W p0 = MW::template ld<C::POL>(pP, i);
            const W q0 = M == 2 ? MW::template ld<C::POL>(pQ, i) : W(0);
            for (uint32_t t = 0; t < nd; ++t) {
                const W delta = MW::template ld<C::POL>(row.get(seg, static_cast<int>(2 * t)), i) ^
                                MW::template ld<C::POL>(row.get(seg, static_cast<int>(2 * t + 1)), i);
                dp ^= delta;
                if constexpr (M == 2)
                    dq ^= gf_mulc(mul_table_exp2(load_const_byte(exps, e0 + t)), delta);
            }
            MW::template st<C::POL>(pP, i, p0 ^ dp);
            if constexpr (M == 2)
                MW::template st<C::POL>(pQ, i, q0 ^ dq);
        }
    };
    if ((acc & 15u) == 0) {
        const uint32_t nvec = len >> 4;
        const uint32_t i = chunk * EPB + threadIdx.x;
        if (i < nvec)
            body(u32x4{}, i);
        const uint32_t tail = len & 15u;
        if (tail && chunk == cps - 1 && threadIdx.x < tail)
            body(uint32_t{}, nvec * 16 + threadIdx.x);
    } else {
        const uint32_t b1 = min(len, (chunk + 1) * EPB * 16);
        for (uint32_t i = chunk * EPB * 16 + threadIdx.x; i < b1; i += C::NTHR)
            body(uint32_t{}, i);
    }
}

// LOOP == false: one work item per workgroup.  LOOP == true: a grid-stride loop, for
// launches with fewer workgroups than items (strips in host memory, ec_kernels.hip).
template <int M, int NDT, class C, bool LOOP = false>
__global__ __launch_bounds__(C::NTHR) DRAID_WAVES_PER_EU(C) void k_update_work(
    const uint8_t* const* tab, uint32_t nd_rt, const uint8_t* exps, WorkSrc ws, uint32_t nwork)
{
    if constexpr (LOOP) {
        for (uint32_t b = blockIdx.x; b < nwork; b += gridDim.x)
            update_item<M, NDT, C>(tab, nd_rt, exps, ws, b);
    } else {
        if (blockIdx.x < nwork)
            update_item<M, NDT, C>(tab, nd_rt, exps, ws, blockIdx.x);
    }
}

// ------------------------------------------------------------ gf_vect_mul

// dst = c * src through the caller's table (gf_vect_mul.c:108 call shape).  T is the
// table form: the caller's two 16-entry nibble tables as they are (NibTable, 22
// VALU operations per dword), or -- when the host found the table to be a linear
// map, as every table from gf_vect_mul_init is -- the same map as three 3-bit
// tables (MulTable, 9 operations).  One workgroup per NTHR * U vectors, no
// grid-stride loop; POL as in the encode.  Measured through the synchronous call
// on 1 GiB / 256 MiB (GB/s of read + write, tools/gpu_gfv_ab.sh, profiles/r02/
// gf_vect_mul_ab.jsonl): one wave x one vector 6.51 / 5.89, 256 lanes x 1 6.41 /
// 5.73, 256 x 2 5.97 / 5.51, 256 x 4 5.82 / 5.25, 64 x 4 6.14 / 5.47; global nt
// instead of buffer accesses 6.32, plain 6.04.  The grid-stride kernel with the
// nibble tables and plain accesses that this replaces: 4.48 / 4.80.
#ifndef DRAID_GFV_NTHR
#define DRAID_GFV_NTHR 64
#endif
#ifndef DRAID_GFV_U
#define DRAID_GFV_U 1
#endif
#ifndef DRAID_GFV_POL
#define DRAID_GFV_POL pol_aux(2, 18)
#endif
template <class T, int NTHR, int U, int POL>
__global__ __launch_bounds__(NTHR) void k_gf_vect_mul(const uint8_t* src, uint8_t* dst,
                                                      uint32_t len, T t)
{
    constexpr uint32_t VPB = static_cast<uint32_t>(NTHR) * U;  // vectors per workgroup
    const uint32_t tid = threadIdx.x;
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) == 0) {
        const uint32_t nvec = len >> 4;
        const uint32_t i0 = blockIdx.x * VPB + tid;
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = i0 + u * NTHR < nvec ? Mem<u32x4>::ld<POL>(src, i0 + u * NTHR) : u32x4(0);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + u * NTHR < nvec)
                Mem<u32x4>::st<POL>(dst, i0 + u * NTHR, gf_mulc(t, v[u]));
        const uint32_t tail = len & 15u;  // the last workgroup also owns the ragged bytes
        if (tail && blockIdx.x == gridDim.x - 1 && tid < tail)
            Mem<uint32_t>::st<0>(dst, nvec * 16 + tid,
                                 gf_mulc(t, Mem<uint32_t>::ld<0>(src, nvec * 16 + tid)));
    } else {
        const uint32_t b1 = min(len, (blockIdx.x + 1) * VPB * 16u);
        for (uint32_t b = blockIdx.x * VPB * 16u + tid; b < b1; b += NTHR)
            Mem<uint32_t>::st<0>(dst, b, gf_mulc(t, Mem<uint32_t>::ld<0>(src, b)));
    }
}

}  // namespace draid
