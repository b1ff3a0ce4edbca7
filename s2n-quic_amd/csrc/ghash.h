// ghash.h — GHASH on LDS tables (gfx950): the 8-bit byte tables of the quad kernel (one key per workgroup segment) and
// the per-wave 4-bit tables of the many-key kernels.  Shared by aes_gcm.hip and tools/ubench/aes_core.hip.
#pragma once

#include "device_common.h"

namespace qpp {
namespace dev {

// ---------------------------------------------------------------- GHASH: Y <- Y * H via 16 byte tables in LDS
// X * H = xor_j T_j[x_j] (GF(2)-linear in X), T_j[x] = (x at byte j) * H.  The running value is kept as
// Z = Y ^ C_next so that the xor with the next block folds into the last xor3 of the table reduction.
//
// Conflict-free layout: T_j[x] lives at x * 256 + j * 16, so a 256-byte row holds the 16 tables' entries for
// one byte value and table j always sits in bank quad j.  A ds_read_b128 serves 16 lanes per LDS cycle; if
// those lanes all read the SAME table j with random x they pile onto one bank quad (with the old j * 4096 +
// x * 16 layout they spread randomly: ~3x cycles, 27 % of all LDS cycles were bank conflicts).  So every lane
// walks the 16 byte positions in its own order: lane r = lane % 16 = 4 q + b reads, at step (k, i), byte
// j(k, i) = 4 ((k + q) & 3) + ((i + b) & 3).  Within each 16-lane group of ds_read_b128 ({0-3,12-15,20-27},
// {4-11,16-19,28-31}, and the same + 32) the lanes have distinct r, hence distinct j: one LDS cycle per group.
// The word part of that order is a rotation of Z's words by q (W[k] = Z.w[(k + q) & 3], two v_cndmask levels),
// the byte part a per-lane v_perm selector; the address (x << 8 | j << 4) is that one v_perm.
#ifndef QPP_GHASH_DEPTH
#define QPP_GHASH_DEPTH 9  // LDS reads in flight per GHASH product (PIPE)
#endif
template <bool PIPE>
struct GhashT {
    uint32_t lc[4];   // byte i of lc[k] = 16 * j(k, i)
    uint32_t sel[4];  // v_perm selector of step i: byte0 <- lc[k].b_i, byte1 <- W[k].b_((i+b)&3), bytes 2,3 <- 0
    bool q1, q2;      // word rotation by q = q1 + 2 q2

    __device__ __forceinline__ static GhashT make() {
        GhashT g;
        const uint32_t r = threadIdx.x & 15u, q = r >> 2, b = r & 3u;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            uint32_t v = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) v |= ((4u * ((k + q) & 3u) + ((i + b) & 3u)) << 4) << (8 * i);
            g.lc[k] = v;
        }
#pragma unroll
        for (int i = 0; i < 4; i++) g.sel[i] = 0x0c0c0000u | ((4u + ((i + b) & 3u)) << 8) | (uint32_t)i;
        g.q1 = q & 1u;
        g.q2 = (q >> 1) & 1u;
        return g;
    }
    // W = Z with its words rotated by q
    __device__ __forceinline__ uint4 rot(uint4 z) const {
        const uint4 a = q1 ? make_uint4(z.y, z.z, z.w, z.x) : z;
        return q2 ? make_uint4(a.z, a.w, a.x, a.y) : a;
    }
    template <int K, int I>
    __device__ __forceinline__ uint4 look(const uint4 &w) const {
        const uint32_t wk = K == 0 ? w.x : K == 1 ? w.y : K == 2 ? w.z : w.w;
        return lds_ld128(kLdsGhash + __builtin_amdgcn_perm(wk, lc[K], sel[I]));
    }
    // (Z * H) ^ c in natural word order, from W = rot(Z).
    // PIPE: 9 reads in flight, the xor tree consuming them 3 at a time and each consumed triple's registers taking the
    // next reads (left alone, the scheduler issued 3, waited for them, and so on: six LDS round trips per product).
    // AES-128 seal 1.389 -> 1.362 ms; all 16 reads in flight spilled VGPRs (1.459 ms).  The AES-256 kernels use it
    // too since the interior-group I/O freed registers (no VGPR spills; AES-256 1 key seal 1.737 -> 1.721 ms).
    __device__ __forceinline__ uint4 prod(const uint4 &w, uint4 c) const {
        if constexpr (!PIPE) {
            const uint4 a = xor3(look<0, 0>(w), look<0, 1>(w), look<0, 2>(w));
            const uint4 b = xor3(look<0, 3>(w), look<1, 0>(w), look<1, 1>(w));
            const uint4 d = xor3(look<1, 2>(w), look<1, 3>(w), look<2, 0>(w));
            const uint4 e = xor3(look<2, 1>(w), look<2, 2>(w), look<2, 3>(w));
            const uint4 f = xor3(look<3, 0>(w), look<3, 1>(w), look<3, 2>(w));
            const uint4 g = xor3(a, b, d);
            const uint4 h = xor3(e, f, look<3, 3>(w));
            return xor3(g, h, c);
        }
        if constexpr (QPP_GHASH_DEPTH != 9) return prod_d<QPP_GHASH_DEPTH>(w, c);
        uint4 l[16];
        auto issue = [&](auto ic) {
            constexpr int i = decltype(ic)::value;
            l[i] = look<i / 4, i % 4>(w);
        };
        static_for<9>(issue);
        __builtin_amdgcn_sched_barrier(0);
        const uint4 a = xor3(l[0], l[1], l[2]);
        issue(std::integral_constant<int, 9>{});
        issue(std::integral_constant<int, 10>{});
        issue(std::integral_constant<int, 11>{});
        __builtin_amdgcn_sched_barrier(0);
        const uint4 b = xor3(l[3], l[4], l[5]);
        issue(std::integral_constant<int, 12>{});
        issue(std::integral_constant<int, 13>{});
        issue(std::integral_constant<int, 14>{});
        __builtin_amdgcn_sched_barrier(0);
        const uint4 d = xor3(l[6], l[7], l[8]);
        issue(std::integral_constant<int, 15>{});
        __builtin_amdgcn_sched_barrier(0);
        const uint4 g = xor3(a, b, d);
        const uint4 e = xor3(l[9], l[10], l[11]);
        const uint4 f = xor3(l[12], l[13], l[14]);
        const uint4 h = xor3(e, f, l[15]);
        return xor3(g, h, c);
    }
    // D reads in flight (D a multiple of 3): each consumed triple's registers take the next 3 reads
    template <int D>
    __device__ __forceinline__ uint4 prod_d(const uint4 &w, uint4 c) const {
        uint4 l[16], x[5];
        auto issue = [&](auto ic) {
            constexpr int i = decltype(ic)::value;
            if constexpr (i < 16) l[i] = look<i / 4, i % 4>(w);
        };
        static_for<D>(issue);
        static_for<5>([&](auto tc) {
            constexpr int t = decltype(tc)::value;
            __builtin_amdgcn_sched_barrier(0);
            x[t] = xor3(l[3 * t], l[3 * t + 1], l[3 * t + 2]);
            issue(std::integral_constant<int, 3 * t + D>{});
            issue(std::integral_constant<int, 3 * t + D + 1>{});
            issue(std::integral_constant<int, 3 * t + D + 2>{});
        });
        __builtin_amdgcn_sched_barrier(0);
        return xor3(xor3(x[0], x[1], x[2]), xor3(x[3], x[4], l[15]), c);
    }
    // one chain step: W' = rot(Z * H ^ c)
    __device__ __forceinline__ uint4 mulx(const uint4 &w, uint4 c) const { return rot(prod(w, c)); }
};
using Ghash = GhashT<false>;

// Build both table sets for one key.  All threads take part; ends with a barrier.
__device__ inline void build_tables(const DevKey *__restrict__ key) {
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    // V powers -> LDS
    for (uint32_t i = tid; i < 128; i += nthr) {
        const uint32_t *v = key->V[i];
        lds_st128(kLdsV + 16 * i, make_uint4(v[0], v[1], v[2], v[3]));
    }
    build_aes_tables(kLdsAes);
    __syncthreads();
    // GHASH tables: entry e = 16 x + j (consecutive threads fill one row); T_j[x] = xor of V[8j+i] over the set
    // bits (bit 7-i) of x
    for (uint32_t e = tid; e < 4096; e += nthr) {
        const uint32_t j = e & 15, x = e >> 4;
        uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; i++)
            if ((x >> (7 - i)) & 1) acc = acc ^ lds_ld128(kLdsV + 16 * (8 * j + i));
        lds_st128(kLdsGhash + 256 * x + 16 * j, acc);
    }
    __syncthreads();
}

// ---------------------------------------------------------------- GHASH with per-wave 4-bit tables (many keys)
// X * H = xor_b (Thi_b[x_b >> 4] ^ Tlo_b[x_b & 15]): 32 reads of 16 B per product instead of 16, but the tables of
// one key are 8 KiB, so each of the 8 waves of a workgroup holds its own key's tables in [0, 64 KiB): wave w at
// w * 8 KiB, high-nibble table at +0, low-nibble table at +4 KiB, entry (b, n) at n * 256 + b * 16.  That is the
// byte layout of Ghash with a 16-entry "x", so the same lane rotation keeps every ds_read_b128 conflict-free and
// the address is still ONE v_perm: the nibbles are split into bytes whose upper nibble carries (wave, half), i.e.
// address bits 12-15.
// BASE: LDS offset of the table region; a region at or above 64 KiB costs one address add per lookup (the v_perm
// address covers 16 bits).  make(w): tables w * 8 KiB into the region (wave w, or a per-lane power in quad.hip).
template <uint32_t BASE = kLdsGhash>
struct Ghash4T {
    Ghash g;            // lane rotation, per-lane selectors (byte positions)
    uint32_t hi_or, lo_or;  // 0x10101010 * (2 wave + half): the upper nibble of every split byte
    __device__ __forceinline__ static Ghash4T make(uint32_t wave) {
        Ghash4T h;
        h.g = Ghash::make();
        h.hi_or = 0x01010101u * ((2u * wave + 0u) << 4);
        h.lo_or = 0x01010101u * ((2u * wave + 1u) << 4);
        return h;
    }
    __device__ __forceinline__ uint4 rot(uint4 z) const { return g.rot(z); }
    template <int K, int I>
    __device__ __forceinline__ uint4 look(uint32_t wk) const {
        return lds_ld128(BASE + __builtin_amdgcn_perm(wk, g.lc[K], g.sel[I]));
    }
    // 32 reads, ~9 in flight: the running xor takes two per step and the next two are issued behind it (4096 keys x
    // 2 Mi packets: seal 3.64 -> 3.50 ms over the word-by-word form the scheduler serialised)
    __device__ __forceinline__ uint4 prod(const uint4 &w, uint4 c) const { return prod_impl<true>(w, c); }
    // W * H alone (no zero operand kept live: the quad kernels' final products, where a zero uint4 held across the
    // packet loop was spilled)
    __device__ __forceinline__ uint4 prod(const uint4 &w) const { return prod_impl<false>(w, w); }
    template <bool C>
    __device__ __forceinline__ uint4 prod_impl(const uint4 &w, uint4 c) const {
        const uint32_t wk[4] = {w.x, w.y, w.z, w.w};
        uint32_t hs[4], ls[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            hs[k] = __builtin_amdgcn_bitop3_b32(wk[k] >> 4, 0x0f0f0f0fu, hi_or, 0xea);  // (a & b) | c
            ls[k] = __builtin_amdgcn_bitop3_b32(wk[k], 0x0f0f0f0fu, lo_or, 0xea);
        }
        uint4 r[32];
        auto issue = [&](auto ic) {
            constexpr int i = decltype(ic)::value, k = i / 8, j = i % 8;
            r[i] = look<k, j % 4>(j < 4 ? hs[k] : ls[k]);
        };
        static_for<9>(issue);
        __builtin_amdgcn_sched_barrier(0);
        uint4 acc = c;
        static_for<16>([&](auto tc) {
            constexpr int t = decltype(tc)::value;
            if constexpr (!C && t == 0) acc = r[0] ^ r[1];
            else acc = xor3(acc, r[2 * t], r[2 * t + 1]);
            if constexpr (2 * t + 9 < 32) issue(std::integral_constant<int, 2 * t + 9>{});
            if constexpr (2 * t + 10 < 32) issue(std::integral_constant<int, 2 * t + 10>{});
            __builtin_amdgcn_sched_barrier(0);
        });
        return acc;
    }
    __device__ __forceinline__ uint4 mulx(const uint4 &w, uint4 c) const { return rot(prod(w, c)); }
};
using Ghash4 = Ghash4T<>;

// The calling wave's Ghash4 tables for `key` (from its V[m] = H * x^m): lane l fills byte b = l >> 2, half
// h = (l >> 1) & 1, nibbles n = 8 (l & 1) .. + 7; T[n] = xor of V[8 b + 4 h + i] over the set bits (bit 3 - i) of n.
// Ends with a wave-level LDS sync (the caller must have synced before overwriting a previous key's tables).
__device__ __forceinline__ void build_gh4(const DevKey *__restrict__ key, uint32_t wave, uint32_t lane) {
    const uint32_t b = lane >> 2, h = (lane >> 1) & 1u, n0 = 8u * (lane & 1u);
    uint4 v[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t *p = key->V[8 * b + 4 * h + i];
        v[i] = make_uint4(p[0], p[1], p[2], p[3]);
    }
    const uint32_t base = kLdsGhash + wave * 8192u + h * 4096u + b * 16u;
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
        const uint32_t n = n0 + k;
        uint4 e = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; i++)
            if ((n >> (3 - i)) & 1u) e = e ^ v[i];
        lds_st128(base + n * 256u, e);
    }
    wave_lds_sync();
}

}  // namespace dev
}  // namespace qpp
