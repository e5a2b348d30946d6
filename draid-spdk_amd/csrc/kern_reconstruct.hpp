// kern_reconstruct.hpp -- the reconstruct: failure decode and plan, one wave per item (k_reconstruct), loads by strip / arithmetic by column (k_reconstruct_cols).
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

namespace draid {

// exp/log tables of the field, staged into LDS by the one-wave reconstruct
__constant__ GfTables c_gf = make_gf_tables();

// ------------------------------------------------------------ reconstruct

// Per-stripe recovery plan; every value is uniform across the workgroup.
struct RecPlan {
    int x, y;          // lost data strips (x < y), -1 = none
    int nd;            // number of lost data strips
    bool lostP, lostQ; // parity strips to regenerate
    bool needq;        // the Q syndrome over the survivors is needed
    bool skip;         // unrecoverable / nothing to do
    bool bad;          // more failures than M parities, or an index outside the stripe
    uint64_t lost;     // bit j set: strip j is lost (decode_failures_mask only)
    MulTable t1, t2;   // constant multipliers (see plan_constants)
};

// The stripe's two failure bytes, fail[2s] | fail[2s+1] << 8, through aligned word
// reads at a wave-uniform address -- scalar loads.  A byte load would be a vector
// memory instruction, and an item whose first instruction waits a full memory
// round trip before the plan is known, and only then issues its strip loads,
// takes half as long again.
__device__ __forceinline__ uint32_t load_fail_pair_at(const uint8_t* pair)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(pair);
    // constant address space: the table is input only, never written by the kernel
    typedef const uint32_t __attribute__((address_space(4)))* ccw;
    const ccw w = (ccw)(a & ~static_cast<uintptr_t>(3));
    const uint32_t at = static_cast<uint32_t>(a) & 3u;
    uint32_t v = w[0] >> (at * 8u);
    if (at == 3u)  // the pair straddles two words (a table at an odd address)
        v |= w[1] << 8;
    return v & 0xffffu;
}
__device__ __forceinline__ uint32_t load_fail_pair(const uint8_t* fail, uint32_t s)
{
    return load_fail_pair_at(fail + 2 * static_cast<size_t>(s));
}

// Decodes the (wave-uniform) failure pair: which strips are lost, which
// syndromes are needed.  No table lookups -- runs before any load is issued, on
// the scalar unit, so it is written without branches: every wave of every item
// runs it ahead of its first strip load.
template <int M>
__device__ __forceinline__ RecPlan decode_failures(int k, uint32_t f0, uint32_t f1)
{
    RecPlan pl;
    constexpr int kNone = 0x7fffffff;  // 0xff: no failure in this slot
    const int ra = static_cast<int>(__builtin_amdgcn_readfirstlane(f0));
    const int rb = static_cast<int>(__builtin_amdgcn_readfirstlane(f1));
    const int a = ra == 0xff ? kNone : ra, b = rb == 0xff ? kNone : rb;
    const bool da = a < k, db = b < k && b != a;  // lost data strips
    pl.nd = (da ? 1 : 0) + (db ? 1 : 0);
    const int lo = da ? a : (db ? b : -1);
    const int hi = (da && db) ? b : -1;
    pl.x = (hi >= 0 && hi < lo) ? hi : lo;
    pl.y = (hi >= 0 && hi < lo) ? lo : hi;
    pl.lostP = a == k || b == k;
    pl.lostQ = a == k + 1 || b == k + 1;
    const bool oob = (a != kNone && a >= k + M) || (b != kNone && b >= k + M);
    if (M == 1)
        pl.lostQ = false;  // index k + 1 is outside a RAID5 stripe (counted by oob)
    const int nf = pl.nd + (pl.lostP ? 1 : 0) + (pl.lostQ ? 1 : 0);
    pl.skip = (nf == 0) || (nf > M) || oob;  // a counted stripe is left untouched
    pl.bad = oob || nf > M;
    pl.needq = (M == 2) && (pl.nd == 2 || (pl.nd == 1 && pl.lostP) || pl.lostQ);
    return pl;
}

// The same decode for a stripe of at most 64 strips known at compile time, over a
// bit mask of the lost strips (one word up to 32 strips, two beyond): a third of
// the scalar instructions, and "is strip j lost" becomes a one-instruction bit
// test per load.  Every wave of a split item runs this ahead of its strip loads,
// so its length is item latency.
template <int K, int M>
__device__ __forceinline__ RecPlan decode_failures_mask(uint32_t f0, uint32_t f1)
{
    static_assert(K + M <= 64, "two mask words");
    constexpr uint32_t N = K + M;
    RecPlan pl;
    const uint32_t a = __builtin_amdgcn_readfirstlane(f0), b = __builtin_amdgcn_readfirstlane(f1);
    const bool oob = (a >= N && a != 0xffu) || (b >= N && b != 0xffu);
    int nf;
    if constexpr (N <= 32) {
        constexpr uint32_t DATA = (K >= 32) ? 0xffffffffu : ((1u << K) - 1u);
        const uint32_t L = (a < N ? 1u << a : 0u) | (b < N ? 1u << b : 0u);
        const uint32_t D = L & DATA;
        pl.lost = L;
        pl.nd = __builtin_popcount(D);
        pl.x = __builtin_ffs(static_cast<int>(D)) - 1;              // lowest lost data strip, or -1
        pl.y = pl.nd == 2 ? 31 - __builtin_clz(D) : -1;
        pl.lostP = (L >> K) & 1u;
        pl.lostQ = M == 2 && ((L >> (K + 1)) & 1u);
        nf = __builtin_popcount(L);
    } else {
        constexpr uint64_t DATA = (1ull << K) - 1ull;
        const uint64_t L = (a < N ? 1ull << a : 0ull) | (b < N ? 1ull << b : 0ull);
        const uint64_t D = L & DATA;
        pl.lost = L;
        pl.nd = __builtin_popcountll(D);
        pl.x = __builtin_ffsll(static_cast<long long>(D)) - 1;
        pl.y = pl.nd == 2 ? 63 - __builtin_clzll(D) : -1;
        pl.lostP = (L >> K) & 1u;
        pl.lostQ = M == 2 && ((L >> (K + 1)) & 1u);
        nf = __builtin_popcountll(L);
    }
    pl.skip = (nf == 0) || (nf > M) || oob;  // a counted stripe is left untouched
    pl.bad = oob || nf > M;
    pl.needq = (M == 2) && (pl.nd == 2 || (pl.nd == 1 && pl.lostP) || pl.lostQ);
    return pl;
}

// GF constants of the plan from exp/log tables (gf_vect_mul.c:255-268 for
// 2^-x, :296-326 for the D+D constants A and B).
__device__ __forceinline__ void plan_constants(RecPlan& pl, const uint8_t* t_exp,
                                               const uint8_t* t_log)
{
    uint32_t c1 = 0, c2 = 0;
    if (pl.nd == 1 && !pl.lostP && pl.lostQ) {
        c1 = t_exp[pl.x];                                   // Q = Qs ^ 2^x D_x
    } else if (pl.nd == 1 && pl.lostP) {
        c1 = t_exp[255 - pl.x];                             // D_x = 2^-x (Q ^ Qs)
    } else if (pl.nd == 2) {
        const uint32_t gyx = t_exp[pl.y - pl.x];
        const uint32_t den = t_exp[255 - t_log[gyx ^ 1u]];  // 1 / (2^(y-x) ^ 1)
        c1 = t_exp[t_log[gyx] + t_log[den]];                // A = 2^(y-x) / (...)
        c2 = t_exp[(255 - pl.x) + t_log[den]];              // B = 2^-x / (...)
    }
    // Wave-uniform (one stripe per workgroup): the table build runs on the SALU.
    c1 = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(c1));
    c2 = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(c2));
    pl.t1 = make_mul_table(c1);
    pl.t2 = make_mul_table(c2);
}

// Loads and syndrome accumulation for U elements, then `constants(pl)` (which
// may stage tables and hit a workgroup barrier -- every lane calls it exactly
// once, after its loads are in flight), then the outputs.
// QS == false: the plan needs no Q syndrome (one data strip rebuilt from P, or P
// alone regenerated), so the Horner doublings -- most of the kernel's VALU work --
// are not compiled into this instance at all.
template <int KT, int M, int U, int POL, bool BOUNDED, bool NOMUL, bool QS, class W, class Ptrs,
          class F>
__device__ __forceinline__ void recover_elems(const Ptrs& pp, uint32_t s, int k, RecPlan& pl,
                                              uint32_t i0, uint32_t stride, uint32_t n,
                                              F&& constants)
{
    using MW = Mem<W>;
    const uint8_t* pP = pp.get(s, k);
    const uint8_t* pQ = (M == 2) ? pp.get(s, k + 1) : pP;
    // Lost (or unneeded) strips are skipped with wave-uniform branches: their
    // pointers stay scalar, no load depends on another, and every surviving
    // load of the lane is in flight before the first XOR.  (Re-pointing a lost
    // strip at an address already loaded lets the compiler forward that value,
    // which makes every later load wait for it.)
    const bool useP = !pl.lostP;
    const bool useQ = pl.needq && !pl.lostQ;
    W ps[U], qs[U], pv[U], qv[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        ok[u] = !BOUNDED || i0 + u * stride < n;
        ps[u] = W(0);
        qs[u] = W(0);
        pv[u] = (useP && ok[u]) ? MW::template ld<POL>(pP, i0 + u * stride) : W(0);
        qv[u] = (useQ && ok[u]) ? MW::template ld<POL>(pQ, i0 + u * stride) : W(0);
    }
    auto fold = [&](const W(&d)[U]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ps[u] ^= d[u];
            if constexpr (M == 2 && QS)
                qs[u] = gf_mul2(qs[u]) ^ d[u];
        }
    };
    if constexpr (KT > 0) {
        for_sources_desc<KT>(k, [&](int j) {
            const bool live = (j != pl.x) && (j != pl.y);
            W d[U];
            const uint8_t* src = pp.get(s, j);
#pragma unroll
            for (int u = 0; u < U; ++u)
                d[u] = (live && ok[u]) ? MW::template ld<POL>(src, i0 + u * stride) : W(0);
            fold(d);
        });
    } else {
        const int x = pl.x, y = pl.y;
        for_blocks_desc<U, POL, W>(
            pp, s, k, ok, i0, stride, [=](int j) { return j != x && j != y; }, fold);
    }
    constants(pl);
    const uint8_t* pX = pl.x >= 0 ? pp.get(s, pl.x) : nullptr;
    const uint8_t* pY = pl.y >= 0 ? pp.get(s, pl.y) : nullptr;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (!ok[u])
            continue;
        const uint32_t i = i0 + u * stride;
        if constexpr (M == 1) {
            // RAID5: the one lost strip (data or P) is the XOR of the survivors
            MW::template st<POL>(pl.nd == 0 ? pP : pX, i, pv[u] ^ ps[u]);
        } else if (pl.nd == 0) {
            if (pl.lostP)
                MW::template st<POL>(pP, i, ps[u]);
            if (M == 2 && pl.lostQ)
                MW::template st<POL>(pQ, i, qs[u]);
        } else if (pl.nd == 1) {
            if (!pl.lostP) {
                const W dx = pv[u] ^ ps[u];
                MW::template st<POL>(pX, i, dx);
                if (M == 2 && pl.lostQ)
                    MW::template st<POL>(pQ, i, qs[u] ^ gf_mulc(pl.t1, dx));
            } else {
                const W dx = gf_mulc(pl.t1, qv[u] ^ qs[u]);
                MW::template st<POL>(pX, i, dx);
                MW::template st<POL>(pP, i, ps[u] ^ dx);
            }
        } else {
            const W pxy = pv[u] ^ ps[u];
            const W qxy = qv[u] ^ qs[u];
            // NOMUL: diagnostic builds only (tools/sweep.py) -- wrong results.
            const W dx = NOMUL ? (pxy ^ qxy) : (gf_mulc(pl.t1, pxy) ^ gf_mulc(pl.t2, qxy));
            MW::template st<POL>(pX, i, dx);
            MW::template st<POL>(pY, i, pxy ^ dx);
        }
    }
}

// Tables for the plan's constants, read with wave-uniform indices through scalar
// loads (their own counter: they complete while the strip loads are in flight,
// with no LDS staging and no barrier).
//   lden[d]  log of 1 / (2^d ^ 1), 0 < d < 255 -- the one inverse of the D+D
//            constants (gf_vect_mul.c:296-326), as a word image of a byte table
//   mul[i]   the MulTable of the constant 2^i (5 words used of 8), i < 255
// Every constant of a plan is a power of two (2^x, 2^-x, A = 2^(d + lden[d]),
// B = 2^(255 - x + lden[d])), so its table is one 32-byte read by exponent
// instead of ~55 scalar operations building it.
struct PlanTables {
    uint32_t lden[64];
    uint32_t mul[255][8];
};

constexpr PlanTables make_plan_tables()
{
    const GfTables g = make_gf_tables();
    PlanTables t{};
    for (int d = 1; d < 255; ++d) {
        const uint32_t l = (255u - g.log[g.exp[d] ^ 1u]) % 255u;
        t.lden[d >> 2] |= l << ((d & 3) * 8);
    }
    for (int i = 0; i < 255; ++i) {
        uint32_t p[8] = {};
        for (int b = 0; b < 8; ++b)
            p[b] = g.exp[i + b];  // 2^i * 2^b
        // same layout as make_mul_table / tri_words
        t.mul[i][0] = (p[0] << 8) | (p[1] << 16) | ((p[0] ^ p[1]) << 24);
        t.mul[i][1] = t.mul[i][0] ^ (p[2] * 0x01010101u);
        t.mul[i][2] = (p[3] << 8) | (p[4] << 16) | ((p[3] ^ p[4]) << 24);
        t.mul[i][3] = t.mul[i][2] ^ (p[5] * 0x01010101u);
        t.mul[i][4] = (p[6] << 8) | (p[7] << 16) | ((p[6] ^ p[7]) << 24);
    }
    return t;
}

__constant__ PlanTables c_plan = make_plan_tables();

__device__ __forceinline__ uint32_t word_byte(const uint32_t* t, uint32_t idx)
{
    return (t[idx >> 2] >> ((idx & 3u) << 3)) & 0xffu;
}

// MulTable of 2^e, e < 510.
__device__ __forceinline__ MulTable mul_table_exp2(uint32_t e)
{
    e = e >= 255u ? e - 255u : e;
    const uint32_t* w = c_plan.mul[e];
    MulTable t;
    t.t0[0] = w[0];
    t.t0[1] = w[1];
    t.t1[0] = w[2];
    t.t1[1] = w[3];
    t.t2 = w[4];
    return t;
}

// The plan's two multiplication tables from scalar reads of c_plan; the same
// constants as plan_constants.
struct PlanMul {
    MulTable t1, t2;
};
__device__ __forceinline__ PlanMul plan_constants_scalar(int nd, int x, int y, bool lostP,
                                                         bool lostQ)
{
    PlanMul m{};
    if (nd == 1 && !lostP && lostQ) {
        m.t1 = mul_table_exp2(x);                          // Q = Qs ^ 2^x D_x
    } else if (nd == 1 && lostP) {
        m.t1 = mul_table_exp2(255u - x);                   // D_x = 2^-x (Q ^ Qs)
    } else if (nd == 2) {
        const uint32_t d = static_cast<uint32_t>(y - x);
        const uint32_t l = word_byte(c_plan.lden, d);
        m.t1 = mul_table_exp2(d + l);                      // A = 2^(y-x) / (2^(y-x) ^ 1)
        m.t2 = mul_table_exp2(255u - x + l);               // B = 2^-x / (2^(y-x) ^ 1)
    }
    return m;
}

// LDS image of the exp/log tables (768 B).
struct LdsGf {
    uint32_t w[(512 + 256) / 4];
};

template <int NTHR>
__device__ __forceinline__ void stage_gf_tables(LdsGf& lds)
{
    const uint32_t* g = reinterpret_cast<const uint32_t*>(&c_gf);
    for (int t = threadIdx.x; t < (512 + 256) / 4; t += NTHR)
        lds.w[t] = g[t];
    __syncthreads();
}

// The GF tables staged through registers: each lane loads its words FIRST, before
// any strip load (vmcnt retires in issue order, so the LDS write then waits only
// for them, not for the strip loads issued after), and writes them to LDS once
// its strip loads are in flight -- staging and barrier overlap the loads.
template <int NTHR>
struct TabStage {
    static constexpr int kWords = (512 + 256) / 4;
    static constexpr int kPerLane = (kWords + NTHR - 1) / NTHR;
    uint32_t w[kPerLane];
    __device__ __forceinline__ void load()
    {
#pragma unroll
        for (int i = 0; i < kPerLane; ++i) {
            const int t = threadIdx.x + i * NTHR;
            w[i] = t < kWords ? reinterpret_cast<const uint32_t*>(&c_gf)[t] : 0u;
        }
    }
    __device__ __forceinline__ void put(LdsGf& lds) const
    {
#pragma unroll
        for (int i = 0; i < kPerLane; ++i) {
            const int t = threadIdx.x + i * NTHR;
            if (t < kWords)
                lds.w[t] = w[i];
        }
    }
    __device__ __forceinline__ void store(LdsGf& lds) const
    {
        put(lds);
        __syncthreads();
    }
};

template <int KT, int M, class C, class Ptrs, class F>
__device__ __forceinline__ void reconstruct_item(const Ptrs& pp, uint32_t s, uint32_t c, int k,
                                                 uint32_t len, uint32_t cps, RecPlan& pl,
                                                 F&& constants)
{
    constexpr int NTHR = C::NTHR, U = C::U, POL = C::POL;
    constexpr uint32_t EPB = static_cast<uint32_t>(NTHR) * U;
    const uint32_t nvec = len >> 4;
    auto none = [](RecPlan&) {};
    if (stripe_aligned<KT, M>(pp, s, k)) {
        const uint32_t i0 = c * EPB + threadIdx.x;
        if ((c + 1) * EPB <= nvec) {
            if (M == 2 && !pl.needq)  // wave-uniform
                recover_elems<KT, M, U, POL, false, C::PLAN == 3, false, u32x4>(
                    pp, s, k, pl, i0, NTHR, nvec, constants);
            else
                recover_elems<KT, M, U, POL, false, C::PLAN == 3, true, u32x4>(
                    pp, s, k, pl, i0, NTHR, nvec, constants);
        } else {
            // Partial last chunk (rare): one vector at a time keeps this path's
            // registers below the main path's, so it does not cap occupancy.
            constants(pl);
#pragma unroll 1
            for (int u = 0; u < U; ++u)
                recover_elems<KT, M, 1, POL, true, false, true, u32x4>(pp, s, k, pl, i0 + u * NTHR, NTHR, nvec,
                                                          none);
        }
        const uint32_t tail = len & 15u;
        if (tail && c == cps - 1 && threadIdx.x < tail)
            recover_elems<0, M, 1, 0, true, false, true, uint32_t>(pp, s, k, pl, nvec * 16 + threadIdx.x,
                                                      NTHR, len, none);
    } else {
        constants(pl);
        const uint32_t b1 = min(len, (c + 1) * EPB * 16);
        for (uint32_t b = c * EPB * 16 + threadIdx.x; b < b1; b += NTHR)
            recover_elems<0, M, 1, 0, true, false, true, uint32_t>(pp, s, k, pl, b, NTHR, b1, none);
    }
}

template <int KT, int M, class C, class Ptrs>
__global__ __launch_bounds__(C::NTHR) DRAID_WAVES_PER_EU(C) void k_reconstruct(Ptrs pp, uint32_t k_rt, uint32_t len,
                                                         uint32_t cps, uint32_t nstripes,
                                                         const uint8_t* fail, uint32_t f01,
                                                         uint32_t* bad)
{
    __shared__ LdsGf lds;
    const uint8_t* l_exp = reinterpret_cast<const uint8_t*>(lds.w);
    const uint8_t* l_log = l_exp + 512;
    const int k = KT > 0 ? KT : static_cast<int>(k_rt);
    const uint32_t total = cps * nstripes;
    if constexpr (C::MAP == 2)
        stage_gf_tables<C::NTHR>(lds);  // once per persistent workgroup
    TabStage<C::NTHR> tabs;
    if constexpr (M == 2 && C::MAP != 2 && C::PLAN == 0)
        tabs.load();
    for (uint32_t b = blockIdx.x; b < total; b += (C::MAP == 2 ? gridDim.x : total)) {
        uint32_t s, c;
        item_coords<C>(b, cps, nstripes, s, c);
        uint32_t f0 = f01 & 0xffu, f1 = (f01 >> 8) & 0xffu;
        if (fail) {
            // The pair is read with byte (vector) loads for the P+Q widths 8..12 and
            // through scalar word loads otherwise: measured, not derived -- same-box
            // A/B of whole library builds (tools/gpu_lib_ab_shapes.sh, profiles/r02/
            // split/fail_read_ab.jsonl), microseconds per launch, vector vs scalar:
            // 8+2 x 64 KiB dual 409.8 vs 417.6, 10+2 497 vs 506, 12+2 301 vs 305; but
            // 5+2 305 vs 288, 4+1 213 vs 203, 3+1 353 vs 328, 8+2 x 128 KiB single 385 vs
            // 380, 14+2 347 vs 343.
            if constexpr (M == 2 && KT >= 8 && KT <= 12) {
                f0 = fail[2 * (size_t)s];
                f1 = fail[2 * (size_t)s + 1];
            } else {
                const uint32_t f = load_fail_pair(fail, s);
                f0 = f & 0xffu;
                f1 = f >> 8;
            }
        }
        RecPlan pl = decode_failures<M>(k, f0, f1);
        // A stripe that cannot be rebuilt is left untouched and counted once (by
        // the workgroup of its first chunk) when the caller asked for the count.
        // Skipped stripes are the only ones counted before any load: a store or
        // atomic ahead of the pointer-table reads would keep them from being
        // scalar loads.
        const bool count_bad = bad && pl.bad && c == 0 && threadIdx.x == 0;
        if (pl.skip) {
            if (count_bad)
                atomicAdd(bad, 1u);
            continue;  // uniform across the workgroup
        }
        if constexpr (M == 1) {
            // RAID5 rebuilds by XOR alone: no constants, no tables, no barrier
            reconstruct_item<KT, M, C>(pp, s, c, k, len, cps, pl, [](RecPlan&) {});
        } else if constexpr (C::PLAN == 2 || C::PLAN == 3) {
            // DIAGNOSTIC ONLY (tools/sweep.py): constants left zero, no LDS, no
            // barrier -- wrong results, measures what the plan step costs.
            reconstruct_item<KT, M, C>(pp, s, c, k, len, cps, pl, [&](RecPlan& p) {
                p.t1 = make_mul_table(0);
                p.t2 = make_mul_table(0);
            });
        } else if constexpr (C::PLAN == 4) {
            // constants from scalar reads of c_plan: no LDS, no barrier
            reconstruct_item<KT, M, C>(pp, s, c, k, len, cps, pl, [&](RecPlan& p) {
                const PlanMul mul = plan_constants_scalar(p.nd, p.x, p.y, p.lostP, p.lostQ);
                p.t1 = mul.t1;
                p.t2 = mul.t2;
            });
        } else if constexpr (C::PLAN == 1) {
            reconstruct_item<KT, M, C>(pp, s, c, k, len, cps, pl, [&](RecPlan& p) {
                plan_constants(p, c_gf.exp, c_gf.log);
            });
        } else if constexpr (C::MAP == 2) {
            reconstruct_item<KT, M, C>(pp, s, c, k, len, cps, pl, [&](RecPlan& p) {
                plan_constants(p, l_exp, l_log);
            });
        } else {
            // Stage the tables while this lane's strip loads are in flight.
            reconstruct_item<KT, M, C>(pp, s, c, k, len, cps, pl, [&](RecPlan& p) {
                tabs.store(lds);
                plan_constants(p, l_exp, l_log);
            });
        }
        if (count_bad)
            atomicAdd(bad, 1u);
    }
}

// The rebuilt strips' ND dwords per lane from the two syndromes of their columns
// (pt: P ^ survivors, qt: Q ^ Horner sum of the survivors): the output stage both
// shared reconstructs end in.
template <int M, int POL, int ND>
__device__ __forceinline__ void store_rebuilt(const RecPlan& pl, const uint8_t* pP,
                                              const uint8_t* pQ, const uint8_t* pX,
                                              const uint8_t* pY, uint32_t ob,
                                              const uint32_t (&pt)[ND], const uint32_t (&qt)[ND])
{
    uint32_t o1[ND], o2[ND];
    if constexpr (M == 1) {
        st_words<POL, ND>(pl.nd == 0 ? pP : pX, ob, pt);  // RAID5: XOR of the survivors
    } else if (pl.nd == 0) {
        if (pl.lostP)
            st_words<POL, ND>(pP, ob, pt);
        if (M == 2 && pl.lostQ)
            st_words<POL, ND>(pQ, ob, qt);
    } else if (pl.nd == 1) {
        if (!pl.lostP) {
            st_words<POL, ND>(pX, ob, pt);
            if (M == 2 && pl.lostQ) {
#pragma unroll
                for (int n = 0; n < ND; ++n)
                    o2[n] = qt[n] ^ gf_mulc(pl.t1, pt[n]);
                st_words<POL, ND>(pQ, ob, o2);
            }
        } else {
#pragma unroll
            for (int n = 0; n < ND; ++n) {
                o1[n] = gf_mulc(pl.t1, qt[n]);
                o2[n] = pt[n] ^ o1[n];
            }
            st_words<POL, ND>(pX, ob, o1);
            st_words<POL, ND>(pP, ob, o2);
        }
    } else {
#pragma unroll
        for (int n = 0; n < ND; ++n) {
            o1[n] = gf_mulc(pl.t1, pt[n]) ^ gf_mulc(pl.t2, qt[n]);
            o2[n] = pt[n] ^ o1[n];
        }
        st_words<POL, ND>(pX, ob, o1);
        st_words<POL, ND>(pY, ob, o2);
    }
}

// ---- shared reconstruct: loads dealt by strip, arithmetic dealt by column
//
// Dealing the reconstruct's ARITHMETIC by strip as the encode does (a Horner chain
// per wave over its strips on whole 16-byte vectors, the Q part scaled by a
// constant to line up, parts XORed through LDS) was built and measured: the
// scaling costs 36 VALU per wave, which a VALU-heavy dual-failure rebuild cannot
// afford (8+2: 580 VALU per item against 435 for one wave), and it lost to the
// one-wave kernel below k = 16 (profiles/r02/split/).  Here only the LOADS are
// dealt by strip: each wave loads its strips as 16-byte vectors and parks them in
// LDS untouched (one row per strip; a strip that is lost or not needed arrives as
// zeros through a descriptor with no records).  The surviving P rides on the last
// wave and the surviving Q on the wave with the fewest data strips.  The plan's
// constants come from scalar table reads placed between the issue of the strip
// loads and the barrier.  After the one barrier every wave owns its share of the
// item's 256 dword columns and runs the one Horner chain down all k strips of its
// columns: the same arithmetic as the one-wave kernel, no scaling, spread evenly
// over the waves whatever the failure pattern.
template <int KT>
struct ColLds {
    u32x4 row[KT + 2][64];  // rows 0..KT-1 data strips, KT the surviving P, KT+1 the surviving Q
};

template <int KT, int M, int SPLIT, int POL, bool BOUNDED, bool QS, class Ptrs>
__device__ __forceinline__ void recover_cols_vec(const Ptrs& pp, uint32_t s, RecPlan& pl,
                                                 uint32_t w, uint32_t lane, uint32_t i,
                                                 uint32_t nvec, ColLds<KT>& lds)
{
    using MW = Mem<u32x4>;
    static_assert(SPLIT == 2 || SPLIT == 4, "every wave finishes 16 / SPLIT bytes per lane");
    constexpr int KW = (KT + SPLIT - 1) / SPLIT;
    constexpr int REM = SPLIT * KW - KT;
    constexpr uint32_t WP = SPLIT - 1, WQ = REM >= 2 ? SPLIT - 1 : SPLIT - 2;
    const bool ok = !BOUNDED || i < nvec;
    const uint8_t* pP = pp.get(s, KT);
    const uint8_t* pQ = (M == 2) ? pp.get(s, KT + 1) : pP;
    const uint8_t* pX = pl.x >= 0 ? pp.get(s, pl.x) : nullptr;
    const uint8_t* pY = pl.y >= 0 ? pp.get(s, pl.y) : nullptr;
    // (one word where the stripe fits one: the bit tests stay 32-bit scalar ops)
    const std::conditional_t<(KT + M <= 32), uint32_t, uint64_t> lost =
        static_cast<std::conditional_t<(KT + M <= 32), uint32_t, uint64_t>>(pl.lost);
    const bool haveP = !pl.lostP, haveQ = M == 2 && QS && pl.needq && !pl.lostQ;
    // phase 1: this wave's strips -> LDS rows (zeros for the ones it skips)
    wave_case<0, SPLIT>(w, [=, &pp, &lds](auto wc) __attribute__((always_inline)) {
        constexpr uint32_t W = decltype(wc)::value;
        constexpr int J0 = static_cast<int>(W) * KW;
        u32x4 d[KW], pv = 0, qv = 0;
#pragma unroll
        for (int j = KW - 1; j >= 0; --j) {
            d[j] = 0;
            if (J0 + j < KT)
                d[j] = ok ? MW::template ld_if<POL>(pp.get(s, J0 + j), i, !((lost >> (J0 + j)) & 1u))
                          : u32x4(0);
        }
        if constexpr (W == WP)
            pv = ok ? MW::template ld_if<POL>(pP, i, haveP) : u32x4(0);
        if constexpr (W == WQ)
            qv = ok ? MW::template ld_if<POL>(pQ, i, haveQ) : u32x4(0);
#pragma unroll
        for (int j = KW - 1; j >= 0; --j)
            if (J0 + j < KT)
                lds.row[J0 + j][lane] = d[j];
        if constexpr (W == WP)
            lds.row[KT][lane] = pv;
        if constexpr (W == WQ)
            lds.row[KT + 1][lane] = qv;
        return PartPQ{};
    });
    if constexpr (M == 2) {
        const PlanMul mul = plan_constants_scalar(pl.nd, pl.x, pl.y, pl.lostP, pl.lostQ);
        pl.t1 = mul.t1;
        pl.t2 = mul.t2;
    }
    __syncthreads();
    // phase 2: this wave's columns, all strips
    constexpr int ND = 4 / SPLIT;
    const uint32_t t = (w * 64u + lane) * ND;
    const uint32_t ob = ((i - lane) << 4) + t * 4u;
    const bool okw = !BOUNDED || ob < (nvec << 4);
    const uint32_t* L = reinterpret_cast<const uint32_t*>(lds.row);
    uint32_t pt[ND], qt[ND];
#pragma unroll
    for (int n = 0; n < ND; ++n) {
        pt[n] = 0;
        qt[n] = 0;
    }
#pragma unroll
    for (int j = KT - 1; j >= 0; --j) {
#pragma unroll
        for (int n = 0; n < ND; ++n) {
            const uint32_t d = L[j * 256 + t + n];
            pt[n] ^= d;
            if constexpr (M == 2 && QS)
                qt[n] = gf_mul2(qt[n]) ^ d;
        }
    }
#pragma unroll
    for (int n = 0; n < ND; ++n) {
        pt[n] ^= L[KT * 256 + t + n];
        if constexpr (M == 2 && QS)
            qt[n] ^= L[(KT + 1) * 256 + t + n];
    }
    if (!okw)
        return;
    store_rebuilt<M, POL, ND>(pl, pP, pQ, pX, pY, ob, pt, qt);
}

// Chunk c of stripe (or segment) s with its failure pair decoded: the 16-byte vectors
// through the column path, a byte tail and unaligned strips on wave 0's byte path.
template <int KT, int M, class C, class Ptrs>
__device__ __forceinline__ void reconstruct_item_cols(const Ptrs& pp, uint32_t s, uint32_t c,
                                                      uint32_t len, uint32_t cps, RecPlan& pl,
                                                      bool aligned, ColLds<KT>& lds)
{
    constexpr int SPLIT = C::SPLIT, POL = C::POL;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t nvec = len >> 4;
    auto none = [](RecPlan&) {};
    if (aligned) {
        const uint32_t i = c * 64u + lane;
        if ((c + 1) * 64u <= nvec) {
            if (M == 2 && !pl.needq)
                recover_cols_vec<KT, M, SPLIT, POL, false, false>(pp, s, pl, w, lane, i, nvec, lds);
            else
                recover_cols_vec<KT, M, SPLIT, POL, false, true>(pp, s, pl, w, lane, i, nvec, lds);
        } else {
            recover_cols_vec<KT, M, SPLIT, POL, true, true>(pp, s, pl, w, lane, i, nvec, lds);
        }
        const uint32_t tail = len & 15u;
        if (w == 0 && tail && c == cps - 1 && lane < tail)
            recover_elems<0, M, 1, 0, true, false, true, uint32_t>(pp, s, KT, pl,
                                                                   nvec * 16 + lane, 64, len, none);
    } else if (w == 0) {
        const PlanMul mul = plan_constants_scalar(pl.nd, pl.x, pl.y, pl.lostP, pl.lostQ);
        pl.t1 = mul.t1;
        pl.t2 = mul.t2;
        const uint32_t b1 = min(len, (c + 1) * 1024u);
        for (uint32_t b = c * 1024u + lane; b < b1; b += 64)
            recover_elems<0, M, 1, 0, true, false, true, uint32_t>(pp, s, KT, pl, b, 64, b1, none);
    }
}

template <int KT, int M, class C, class Ptrs>
__global__ __launch_bounds__(C::NTHR) DRAID_WAVES_PER_EU(C) void k_reconstruct_cols(
    Ptrs pp, uint32_t len, uint32_t cps, uint32_t nstripes, const uint8_t* fail, uint32_t f01,
    uint32_t* bad, ItemGrid ig)
{
    static_assert(KT > 0 && C::SPLIT > 1 && C::MAP == 0, "one shared item per workgroup, stripe order");
    __shared__ ColLds<KT> lds;
    uint32_t c, s;
    ig.coords(c, s);
    if (s >= nstripes)
        return;
    // The pointer row and the failure pair are independent scalar reads: both are
    // issued before either is used, so an item pays one memory round trip for
    // them, not two, before its strip loads can go out.
    const bool aligned = stripe_aligned<KT, M>(pp, s, KT);
    uint32_t f0 = f01 & 0xffu, f1 = (f01 >> 8) & 0xffu;
    if (fail) {
        const uint32_t f = load_fail_pair(fail, s);
        f0 = f & 0xffu;
        f1 = f >> 8;
    }
    RecPlan pl = decode_failures_mask<KT, M>(f0, f1);
    const bool count_bad = bad && pl.bad && c == 0 && threadIdx.x == 0;
    if (!pl.skip)
        reconstruct_item_cols<KT, M, C>(pp, s, c, len, cps, pl, aligned, lds);
    if (count_bad)
        atomicAdd(bad, 1u);
}

// ---- shared reconstruct of wide stripes: loads AND arithmetic dealt by strip
//
// The column division parks every strip of the item in LDS, (k + 2) KiB per item:
// from k = 21 up that is what limits how many items a CU holds (32+2: four), and
// each wave still loads k / 2 or k / 4 strips for the same single barrier.  Wide
// stripes therefore divide the arithmetic by strip too, as the encode does: wave w
// accumulates P and the Horner form of Q over the survivors among its strips
// (a lost strip arrives as zeros), scales its Q part by the constant 2^(first
// strip of the wave) -- 9 VALU per dword once per wave, which at six to eight
// strips per wave costs little, where at two to four it was what sank this
// division below k = 16 -- and the surviving P and Q ride on the last and the
// first wave (whose scale is 1).  The parts meet in 2 * SPLIT KiB of LDS, and after
// the barrier every wave finishes 16 / SPLIT bytes per lane of the rebuilt strips
// from the XOR of the parts: the syndromes themselves.
template <int KT, int M, int SPLIT, int POL, bool BOUNDED, bool QS, class Ptrs>
__device__ __forceinline__ void recover_split_vec(const Ptrs& pp, uint32_t s, RecPlan& pl,
                                                  uint32_t w, uint32_t lane, uint32_t i,
                                                  uint32_t nvec, SplitLds<SPLIT>& lds)
{
    using MW = Mem<u32x4>;
    static_assert(SPLIT == 2 || SPLIT == 4, "every wave finishes 16 / SPLIT bytes per lane");
    constexpr int KW = (KT + SPLIT - 1) / SPLIT;
    const bool ok = !BOUNDED || i < nvec;
    const uint8_t* pP = pp.get(s, KT);
    const uint8_t* pQ = (M == 2) ? pp.get(s, KT + 1) : pP;
    const uint8_t* pX = pl.x >= 0 ? pp.get(s, pl.x) : nullptr;
    const uint8_t* pY = pl.y >= 0 ? pp.get(s, pl.y) : nullptr;
    const std::conditional_t<(KT + M <= 32), uint32_t, uint64_t> lost =
        static_cast<std::conditional_t<(KT + M <= 32), uint32_t, uint64_t>>(pl.lost);
    const bool haveP = !pl.lostP, haveQ = M == 2 && QS && pl.needq && !pl.lostQ;
    const PartPQ part = wave_case<0, SPLIT>(w, [=, &pp](auto wc) __attribute__((always_inline)) {
        constexpr int W = decltype(wc)::value;
        constexpr int J0 = W * KW;
        u32x4 d[KW], pv = 0, qv = 0;
#pragma unroll
        for (int j = KW - 1; j >= 0; --j) {
            d[j] = 0;
            if (J0 + j < KT)
                d[j] = ok ? MW::template ld_if<POL>(pp.get(s, J0 + j), i, !((lost >> (J0 + j)) & 1u))
                          : u32x4(0);
        }
        if constexpr (W == SPLIT - 1)
            pv = ok ? MW::template ld_if<POL>(pP, i, haveP) : u32x4(0);
        if constexpr (W == 0)
            qv = ok ? MW::template ld_if<POL>(pQ, i, haveQ) : u32x4(0);
        u32x4 p = 0, q = 0;
#pragma unroll
        for (int j = KW - 1; j >= 0; --j) {
            if (J0 + j < KT) {
                p ^= d[j];
                if constexpr (M == 2 && QS)
                    q = gf_mul2(q) ^ d[j];
            }
        }
        if constexpr (M == 2 && QS && J0 != 0)
            q = gf_mulc(make_mul_table(gf_exp2_const(J0)), q);
        return PartPQ{p ^ pv, q ^ qv};
    });
    lds.p[w][lane] = part.p;
    if constexpr (M == 2 && QS)
        lds.q[w][lane] = part.q;
    if constexpr (M == 2) {
        const PlanMul mul = plan_constants_scalar(pl.nd, pl.x, pl.y, pl.lostP, pl.lostQ);
        pl.t1 = mul.t1;
        pl.t2 = mul.t2;
    }
    __syncthreads();
    constexpr int ND = 4 / SPLIT;
    const uint32_t t = (w * 64u + lane) * ND;
    const uint32_t ob = ((i - lane) << 4) + t * 4u;
    const bool okw = !BOUNDED || ob < (nvec << 4);
    const uint32_t* LP = reinterpret_cast<const uint32_t*>(lds.p);
    const uint32_t* LQ = reinterpret_cast<const uint32_t*>(lds.q);
    uint32_t pt[ND], qt[ND];
#pragma unroll
    for (int n = 0; n < ND; ++n) {
        pt[n] = 0;
        qt[n] = 0;
#pragma unroll
        for (int r = 0; r < SPLIT; ++r) {
            pt[n] ^= LP[r * 256 + t + n];
            if constexpr (M == 2 && QS)
                qt[n] ^= LQ[r * 256 + t + n];
        }
    }
    if (!okw)
        return;
    store_rebuilt<M, POL, ND>(pl, pP, pQ, pX, pY, ob, pt, qt);
}

template <int KT, int M, class C, class Ptrs>
__device__ __forceinline__ void reconstruct_item_split(const Ptrs& pp, uint32_t s, uint32_t c,
                                                       uint32_t len, uint32_t cps, RecPlan& pl,
                                                       bool aligned, SplitLds<C::SPLIT>& lds)
{
    constexpr int SPLIT = C::SPLIT, POL = C::POL;
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t nvec = len >> 4;
    auto none = [](RecPlan&) {};
    if (aligned) {
        const uint32_t i = c * 64u + lane;
        if ((c + 1) * 64u <= nvec) {
            if (M == 2 && !pl.needq)
                recover_split_vec<KT, M, SPLIT, POL, false, false>(pp, s, pl, w, lane, i, nvec, lds);
            else
                recover_split_vec<KT, M, SPLIT, POL, false, true>(pp, s, pl, w, lane, i, nvec, lds);
        } else {
            recover_split_vec<KT, M, SPLIT, POL, true, true>(pp, s, pl, w, lane, i, nvec, lds);
        }
        const uint32_t tail = len & 15u;
        if (w == 0 && tail && c == cps - 1 && lane < tail)
            recover_elems<0, M, 1, 0, true, false, true, uint32_t>(pp, s, KT, pl,
                                                                   nvec * 16 + lane, 64, len, none);
    } else if (w == 0) {
        const PlanMul mul = plan_constants_scalar(pl.nd, pl.x, pl.y, pl.lostP, pl.lostQ);
        pl.t1 = mul.t1;
        pl.t2 = mul.t2;
        const uint32_t b1 = min(len, (c + 1) * 1024u);
        for (uint32_t b = c * 1024u + lane; b < b1; b += 64)
            recover_elems<0, M, 1, 0, true, false, true, uint32_t>(pp, s, KT, pl, b, 64, b1, none);
    }
}

template <int KT, int M, class C, class Ptrs>
__global__ __launch_bounds__(C::NTHR) DRAID_WAVES_PER_EU(C) void k_reconstruct_split(
    Ptrs pp, uint32_t len, uint32_t cps, uint32_t nstripes, const uint8_t* fail, uint32_t f01,
    uint32_t* bad, ItemGrid ig)
{
    static_assert(KT > 0 && C::SPLIT > 1 && C::MAP == 0, "one shared item per workgroup, stripe order");
    __shared__ SplitLds<C::SPLIT> lds;
    uint32_t c, s;
    ig.coords(c, s);
    if (s >= nstripes)
        return;
    const bool aligned = stripe_aligned<KT, M>(pp, s, KT);
    uint32_t f0 = f01 & 0xffu, f1 = (f01 >> 8) & 0xffu;
    if (fail) {
        const uint32_t f = load_fail_pair(fail, s);
        f0 = f & 0xffu;
        f1 = f >> 8;
    }
    RecPlan pl = decode_failures_mask<KT, M>(f0, f1);
    const bool count_bad = bad && pl.bad && c == 0 && threadIdx.x == 0;
    if (!pl.skip)
        reconstruct_item_split<KT, M, C>(pp, s, c, len, cps, pl, aligned, lds);
    if (count_bad)
        atomicAdd(bad, 1u);
}

}  // namespace draid
