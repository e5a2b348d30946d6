// kern_cfg.hpp -- launch configuration (Cfg), item coordinates, and what the shared-item kernels have in common.
// Part of the kernel translation unit (ec_kernels.hip includes these in order); not
// a public interface.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ec_gf.hpp"
#include "ec_launch.hpp"
#include "kern_mem.hpp"

namespace draid {

// Launch configuration knobs (A/B-tested with tools/sweep.py):
//   NTHR  lanes per workgroup           U    16-B vectors per lane per strip
//   POL   bit0 nt loads, bit1 nt stores
//   MAP   0: block b -> (stripe b / cps, chunk b % cps)
//         1: chunk-major (chunk b / nstripes, stripe b % nstripes)
//         2: persistent grid-stride over stripe-major items
//   PLAN  (one-wave reconstruct) 0: exp/log tables staged in LDS, 1: scalar reads of
//         the __constant__ tables (no LDS, no barrier)
//   WAVES waves per SIMD the kernel is built for (0: the compiler's choice).
//         The compiler pads the register allocation so exactly this many waves
//         fit: fewer resident waves keep fewer DRAM pages open at once, which
//         is worth more to these streaming kernels than the extra latency
//         hiding (8+2 x 64 KiB dual reconstruct: 0.411 ms at 5 waves, 0.420 at
//         the 7 its 70 VGPRs would allow, 0.417 at 4).
//   SPLIT waves that share one item: the workgroup has SPLIT * 64 lanes, the item
//         is still 64 lanes wide (1 KiB of every strip at U = 1), and wave w loads
//         only strips [w*KW, (w+1)*KW), KW = ceil(k / SPLIT); the encode's partial
//         sums (k_encode_split) or the reconstruct's raw strips (k_reconstruct_cols)
//         meet in LDS.  NTHR_ counts the lanes of the whole workgroup.
template <int NTHR_, int U_, int POL_, int MAP_, int PLAN_ = 0, int WAVES_ = 0, int SPLIT_ = 1>
struct Cfg {
    static constexpr int NTHR = NTHR_, U = U_, POL = POL_, MAP = MAP_, PLAN = PLAN_,
                         WAVES = WAVES_, SPLIT = SPLIT_, ITEM = NTHR_ / SPLIT_;
    static_assert(SPLIT_ == 1 || (NTHR_ == 64 * SPLIT_ && U_ == 1), "a split item is one wave wide");
};
#define DRAID_WAVES_PER_EU(C) \
    __attribute__((amdgpu_waves_per_eu((C::WAVES) ? (C::WAVES) : 1, (C::WAVES) ? (C::WAVES) : 8)))

template <class C>
__device__ __forceinline__ void item_coords(uint32_t b, uint32_t cps, uint32_t nstripes,
                                            uint32_t& s, uint32_t& c)
{
    if constexpr (C::MAP == 1) {
        c = b / nstripes;
        s = b - c * nstripes;
    } else if constexpr (C::MAP == 3) {
        // XCD-aware: the dispatcher deals workgroup b to XCD b % 8; give each XCD a
        // contiguous run of items (whole stripes) instead of every 8th chunk.
        const uint32_t total = cps * nstripes, q = total >> 3, r = total & 7u;
        const uint32_t x = b & 7u, i = b >> 3;
        const uint32_t bb = x * q + min(x, r) + i;
        s = bb / cps;
        c = bb - s * cps;
    } else if constexpr (C::MAP >= 4 && C::MAP <= 7) {
        // Groups of G stripes swept together (lab study): consecutive workgroups
        // take G different stripes; MAP 4/6 also skew each stripe's chunk by
        // s_local * cps / G ("diagonal"), MAP 5/7 keep the same chunk (group
        // chunk-major).  A ragged last group falls back to stripe order.
        constexpr uint32_t G = (C::MAP == 4 || C::MAP == 5) ? 16u : 4u;
        constexpr bool diag = (C::MAP == 4 || C::MAP == 6);
        const uint32_t per_group = G * cps, g = b / per_group;
        if ((g + 1) * G <= nstripes) {
            const uint32_t i = b - g * per_group, sl = i % G, cc = i / G;
            s = g * G + sl;
            c = diag ? (cc + sl * (cps / G)) % cps : cc;
        } else {
            s = b / cps;
            c = b - s * cps;
        }
    } else {
        s = b / cps;
        c = b - s * cps;
    }
}

// ------------------------------------------------------------ split items
//
// The same item (1 KiB of every strip of one stripe) shared by SPLIT waves of one
// workgroup.  A wave that loads all k strips of an item keeps k KiB in flight and
// holds its slot until the last of them has arrived; the CU then either has few
// waves (idle slots while workgroups turn over) or far more bytes in flight than
// the memory system needs, and DRAM efficiency falls as k grows (16+2: 6.0 TB/s).
// With the strips of the item dealt over 3-4 waves every wave has 2-4 loads, a CU
// holds 6 items instead of 16-24, and the same shapes stream 5-7% faster
// (tools/probe/wide_probe.hip: 8+2 x 64 KiB 6.96 vs 6.64 TB/s, 16+2 x 256 KiB
// 6.42 vs 6.00).  Wave w accumulates P and the Horner form of Q over its strips
// [w*KW, (w+1)*KW), scales its Q part by 2^(w*KW), and the parts are XORed
// through LDS after one barrier.

// Split kernels take a 2-D/3-D grid -- x the chunk, y (and z beyond 65535) the
// stripe -- so an item's coordinates cost no division.  A grid whose x extent is
// tiny dispatches slowly (8+2 x 4 KiB strips, x = 4: 531 us per launch against 444
// for the same items on a 1-D grid), so when a strip has fewer than 64 chunks and
// their number is a power of two, 2^fold neighbouring stripes share one x row:
// x = chunk | stripe_low << cshift.  Otherwise fold = 0 and cshift = 31 (x < 2^31,
// so the same two shifts and the mask leave chunk = x, stripe_low = 0).
constexpr uint32_t kGridY = 65535;
struct ItemGrid {
    uint32_t cshift, fold;
    __device__ __forceinline__ void coords(uint32_t& c, uint32_t& s) const
    {
        c = blockIdx.x & ((1u << cshift) - 1u);
        s = ((blockIdx.z * kGridY + blockIdx.y) << fold) + (blockIdx.x >> cshift);
    }
};

// Partial sums of one wave.
struct PartPQ {
    u32x4 p, q;
};

// Returns part(std::integral_constant<int, W>) for the wave's own index W = w
// (wave-uniform, scalar branches).  Each wave gets code specialised for its
// strips: strip indices are constants, so a pointer table row is fetched with
// scalar loads of fixed offsets (a run-time strip index turns them into per-lane
// loads plus a readfirstlane loop around every strip access).  The parts come
// back by value -- sums captured by reference end up in scratch memory.
template <int W, int SPLIT, class F>
__device__ __forceinline__ auto wave_case(uint32_t w, const F& part)
{
    if constexpr (W + 1 == SPLIT) {
        return part(std::integral_constant<int, W>{});
    } else {
        if (w == W)
            return part(std::integral_constant<int, W>{});
        return wave_case<W + 1, SPLIT>(w, part);
    }
}

}  // namespace draid
