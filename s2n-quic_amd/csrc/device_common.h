// device_common.h — device-side building blocks shared by the packet-protection kernels (gfx950).
#pragma once

#include <utility>

#include "qpp_internal.h"

namespace qpp {
namespace dev {

constexpr uint32_t kLdsGhash = 0;
constexpr uint32_t kLdsAes = 65536;
constexpr uint32_t kLdsV = 131072;      // GHASH key powers, only while the tables are built
constexpr uint32_t kLdsStage = 131072;  // per-wave payload staging (aes_gcm.hip Stage), after the build
constexpr uint32_t kLdsMax = 163840;    // 160 KiB per workgroup

// LDS is addressed by plain 32-bit offsets into the workgroup's allocation.  Every kernel that uses these
// helpers declares exactly one LDS array (which therefore starts at offset 0) and touches LDS only through
// them, so there is no base-symbol add per access (with `lds + off` hipcc emitted a `v_add_u32 v, 0, v` per
// table lookup: a quarter of the AES round's VALU work).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) u32x4 lds_u128;
__device__ __forceinline__ uint32_t lds_ld32(uint32_t a) { return *(const lds_u32 *)(size_t)a; }
__device__ __forceinline__ uint4 lds_ld128(uint32_t a) {
    const u32x4 v = *(const lds_u128 *)(size_t)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void lds_st32(uint32_t a, uint32_t v) { *(lds_u32 *)(size_t)a = v; }
// ds_add_rtn_u32: the old value (workgroup scope)
__device__ __forceinline__ uint32_t lds_add32(uint32_t a, uint32_t v) {
    return __hip_atomic_fetch_add((lds_u32 *)(size_t)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) u32x2 lds_u64;
__device__ __forceinline__ uint2 lds_ld64(uint32_t a) {
    const u32x2 v = *(const lds_u64 *)(size_t)a;
    return make_uint2(v.x, v.y);
}
__device__ __forceinline__ void lds_st64(uint32_t a, uint2 v) {
    u32x2 t;
    t.x = v.x; t.y = v.y;
    *(lds_u64 *)(size_t)a = t;
}
__device__ __forceinline__ void lds_st128(uint32_t a, uint4 v) {
    u32x4 t;
    t.x = v.x; t.y = v.y; t.z = v.z; t.w = v.w;
    *(lds_u128 *)(size_t)a = t;
}

static __device__ const uint8_t d_sbox[256] = {
#define S(i) kSBox.v[i]
#define S8(i) S(i), S(i + 1), S(i + 2), S(i + 3), S(i + 4), S(i + 5), S(i + 6), S(i + 7)
#define S64(i) S8(i), S8(i + 8), S8(i + 16), S8(i + 24), S8(i + 32), S8(i + 40), S8(i + 48), S8(i + 56)
    S64(0), S64(64), S64(128), S64(192)
#undef S64
#undef S8
#undef S
};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t rotl16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t xtime4(uint32_t s) {  // xtime on one byte held in the low 8 bits
    return ((s << 1) ^ ((s & 0x80) ? 0x1b : 0)) & 0xff;
}

__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);  // unaligned-capable global_load_dwordx4
    return v;
}
__device__ __forceinline__ void st16(uint8_t *p, uint4 v) { __builtin_memcpy(p, &v, 16); }
// streaming (nt) store of the cooperative payload chunks: the sealed / opened bytes are not read again by the kernel.
// Seal 1.39 -> 1.34 ms at 1 Mi x 1200 B (nt LOADS were 1.86 ms: the next group's chunk reuses the fetched lines).
// The address may be unaligned (global_store_dwordx4 takes any byte address on gfx950).
__device__ __forceinline__ void st16_nt(uint8_t *p, uint4 v) {
    u32x4 t;
    t.x = v.x; t.y = v.y; t.z = v.z; t.w = v.w;
    __builtin_nontemporal_store(t, (u32x4 *)p);
}
__device__ __forceinline__ uint4 operator^(uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); }

// keep bytes [0, r) of a 16-byte block (1 <= r <= 16)
__device__ __forceinline__ uint4 keep_bytes(uint4 v, uint32_t r) {
    auto m = [r](uint32_t k) -> uint32_t {
        int b = (int)r - 4 * (int)k;
        return b >= 4 ? 0xffffffffu : b <= 0 ? 0u : ((1u << (8 * b)) - 1u);
    };
    return make_uint4(v.x & m(0), v.y & m(1), v.z & m(2), v.w & m(3));
}

__device__ __forceinline__ void st_bytes(uint8_t *p, uint4 v, uint32_t r) {
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t i = 0; i < 16; i++)
        if (i < r) p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // gfx950 v_bitop3_b32: one op for a ^ b ^ c
}
__device__ __forceinline__ uint4 xor3(uint4 a, uint4 b, uint4 c) {
    return make_uint4(xor3(a.x, b.x, c.x), xor3(a.y, b.y, c.y), xor3(a.z, b.z, c.z), xor3(a.w, b.w, c.w));
}

// ---------------------------------------------------------------- AES with bank-replicated LDS T-tables
// Column c of a round: T0[s_c.b0] ^ T1[s_c+1.b1] ^ T2[s_c+2.b2] ^ T3[s_c+3.b3] ^ rk, with T2 = rotl16(T0) and
// T3 = rotl16(T1), so only T0/T1 are stored (64 KiB replicated); per column: 4 lookups + 4 VALU.
struct AesLds {
    uint32_t laneword;  // byte0 = 4 * (lane % 32), byte2 = table base >> 16
    __device__ __forceinline__ uint32_t rot(uint32_t x) const { return x; }  // (AesQ4's lane convention: none here)

    // address of T0[byte K of w] (T1 is at +128): ONE v_perm_b32
    template <int K>
    __device__ __forceinline__ uint32_t addr(uint32_t w) const {
        // byte0 <- laneword.b0, byte1 <- w.bK, byte2 <- laneword.b2, byte3 <- 0
        return __builtin_amdgcn_perm(w, laneword, (0x0cu << 24) | (2u << 16) | ((4u + K) << 8) | 0u);
    }
    template <int K>
    __device__ __forceinline__ uint32_t t0(uint32_t w) const { return lds_ld32(addr<K>(w)); }
    template <int K>
    __device__ __forceinline__ uint32_t t1(uint32_t w) const { return lds_ld32(addr<K>(w) + 128); }

    __device__ __forceinline__ uint32_t col(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) const {
        return xor3(t0<0>(a), t1<1>(b), k) ^ rotl16(t0<2>(c) ^ t1<3>(d));
    }
    __device__ __forceinline__ uint32_t last(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) const {
        // S[x] = byte1 of T0[x] = byte2/byte3 of T1[x]; lo|hi are disjoint so one xor3 finishes the column
        uint32_t lo = __builtin_amdgcn_perm(t1<1>(b), t0<0>(a), 0x0c0c0601u);
        uint32_t hi = __builtin_amdgcn_perm(t1<3>(d), t0<2>(c), 0x07020c0cu);
        return xor3(lo, hi, k);
    }
    __device__ __forceinline__ void round(uint32_t (&s)[4], const uint32_t *__restrict__ rk) const {
        uint32_t u0 = col(s[0], s[1], s[2], s[3], rk[0]);
        uint32_t u1 = col(s[1], s[2], s[3], s[0], rk[1]);
        uint32_t u2 = col(s[2], s[3], s[0], s[1], rk[2]);
        uint32_t u3 = col(s[3], s[0], s[1], s[2], rk[3]);
        s[0] = u0; s[1] = u1; s[2] = u2; s[3] = u3;
    }
    __device__ __forceinline__ uint4 final(const uint32_t (&s)[4], const uint32_t *__restrict__ rk) const {
        return make_uint4(last(s[0], s[1], s[2], s[3], rk[0]), last(s[1], s[2], s[3], s[0], rk[1]),
                          last(s[2], s[3], s[0], s[1], rk[2]), last(s[3], s[0], s[1], s[2], rk[3]));
    }

    // One block over the 4 lanes of a quad (every lane of every quad active, the same block in a quad): lane s holds
    // column s of the state and takes columns s + 1, s + 2, s + 3 from its neighbours by DPP quad_perm each round, so
    // it does one column's 4 lookups instead of the block's 16; round keys from LDS at o (word s of each round).
    // Returns column s of E(in) (in: column s of the plaintext block).
    template <int NR>
    __device__ __forceinline__ uint32_t encrypt_quad(uint32_t in, uint32_t o, uint32_t s) const {
        auto nb = [](uint32_t v, auto ctrl) {
            return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, decltype(ctrl)::value, 0xf, 0xf, false);
        };
        using R1 = std::integral_constant<int, 0x39>;  // lane s reads s + 1
        using R2 = std::integral_constant<int, 0x4e>;  // s + 2
        using R3 = std::integral_constant<int, 0x93>;  // s + 3
        uint32_t x = in ^ lds_ld32(o + 4u * s);
#pragma unroll
        for (int r = 1; r < NR; r++) {
            const uint32_t b = nb(x, R1{}), c = nb(x, R2{}), d = nb(x, R3{});
            x = col(x, b, c, d, lds_ld32(o + 16u * (uint32_t)r + 4u * s));
        }
        const uint32_t b = nb(x, R1{}), c = nb(x, R2{}), d = nb(x, R3{});
        return last(x, b, c, d, lds_ld32(o + 16u * (uint32_t)NR + 4u * s));
    }
    // Full AES of one block with the round keys in LDS at byte offset o (read where used: no 44 / 60 registers held)
    template <int NR>
    __device__ __forceinline__ uint4 encrypt_lrk(uint4 in, uint32_t o) const {
        auto k4 = [&](int r, uint32_t (&k)[4]) {
            const uint4 v = lds_ld128(o + 16u * (uint32_t)r);
            k[0] = v.x; k[1] = v.y; k[2] = v.z; k[3] = v.w;
        };
        uint32_t k[4];
        k4(0, k);
        uint32_t s[4] = {in.x ^ k[0], in.y ^ k[1], in.z ^ k[2], in.w ^ k[3]};
#pragma unroll
        for (int r = 1; r < NR; r++) {
            k4(r, k);
            round(s, k);
        }
        k4(NR, k);
        return final(s, k);
    }
    // Full AES of one block (no caching): HP mask, key setup, page-crossing groups.
    template <int NR>
    __device__ __forceinline__ uint4 encrypt(uint4 in, const uint32_t *__restrict__ rk) const {
        uint32_t s[4] = {in.x ^ rk[0], in.y ^ rk[1], in.z ^ rk[2], in.w ^ rk[3]};
#pragma unroll
        for (int r = 1; r < NR; r++) round(s, rk + 4 * r);
        return final(s, rk + 4 * NR);
    }
};

// Counter-mode round caching.  For CTR blocks nonce || be32(c) only the last byte of the block changes while
// c stays inside one 256-block page, so after round 1 only column 0 varies (one lookup) and round 2 needs
// four lookups (one per output column).  `Page` holds the per-packet, per-page constants.
struct CtrPage {
    uint32_t k0, k1, k2, k3;  // round-1 output (k0 without the varying T3 term)
    uint32_t l0, l1, l2, l3;  // round-2 output without the varying terms
    uint32_t x3;              // rk[3] byte 3 (xored with the counter's low byte)
    uint32_t page;            // c >> 8 these constants belong to

    __device__ __forceinline__ void build(const AesLds &a, const uint32_t *__restrict__ rk, uint32_t n0, uint32_t n1,
                                          uint32_t n2, uint32_t pg) {
        const uint32_t s0 = n0 ^ rk[0], s1 = n1 ^ rk[1], s2 = n2 ^ rk[2], s3 = bswap32(pg << 8) ^ rk[3];
        k0 = xor3(a.t0<0>(s0), a.t1<1>(s1), rk[4]) ^ rotl16(a.t0<2>(s2));
        k1 = a.col(s1, s2, s3, s0, rk[5]);
        k2 = a.col(s2, s3, s0, s1, rk[6]);
        k3 = a.col(s3, s0, s1, s2, rk[7]);
        l0 = xor3(a.t1<1>(k1), rk[8], rotl16(a.t0<2>(k2) ^ a.t1<3>(k3)));
        l1 = xor3(a.t0<0>(k1), a.t1<1>(k2), rk[9]) ^ rotl16(a.t0<2>(k3));
        l2 = xor3(a.t0<0>(k2), a.t1<1>(k3), rk[10]) ^ rotl16(a.t1<3>(k1));
        l3 = xor3(a.t0<0>(k3), rk[11], rotl16(a.t0<2>(k1) ^ a.t1<3>(k2)));
        x3 = rk[3] >> 24;
        page = pg;
    }
    // state after rounds 1 and 2 for counter c (same page)
    __device__ __forceinline__ void two_rounds(const AesLds &a, uint32_t c, uint32_t (&v)[4]) const {
        const uint32_t x = (c & 0xffu) ^ x3;
        const uint32_t u0 = k0 ^ rotl16(a.t1<0>(x));  // T3[x]
        v[0] = l0 ^ a.t0<0>(u0);
        v[1] = l1 ^ rotl16(a.t1<3>(u0));              // T3[u0.b3]
        v[2] = l2 ^ rotl16(a.t0<2>(u0));              // T2[u0.b2]
        v[3] = l3 ^ a.t1<1>(u0);                      // T1[u0.b1]
    }
};

// NB counter blocks c, c+1, ... (all inside page.page) -> NB keystream blocks, lookups of all NB blocks
// interleaved round by round for ILP.
template <int NR, int NB>
__device__ __forceinline__ void ctr_keystream(const AesLds &a, const CtrPage &pg, const uint32_t *__restrict__ rk,
                                              uint32_t c, uint4 (&ks)[NB]) {
    uint32_t s[NB][4];
#pragma unroll
    for (int j = 0; j < NB; j++) pg.two_rounds(a, c + j, s[j]);
#pragma unroll
    for (int r = 3; r < NR; r++)
#pragma unroll
        for (int j = 0; j < NB; j++) a.round(s[j], rk + 4 * r);
#pragma unroll
    for (int j = 0; j < NB; j++) ks[j] = a.final(s[j], rk + 4 * NR);
}

// The same keystream, software-pipelined by hand.  Left to itself the scheduler issues 2-8 T-table reads and then
// waits for them (lgkmcnt 0..4 every few instructions): each wave has little LDS work in flight and the SIMD idles
// whenever both of its waves wait.  Here the rounds 3..NR of the NB blocks are cut into "units" (round r, block j,
// column c: 4 lookups + the column's combine), ordered column-major over the blocks, and the lookups of unit t + D
// are issued before unit t is combined (D = NB - 1: unit t + NB is the first that needs the round unit t finishes).
// So 4 (NB - 1) = 12 reads stay in flight (lgkmcnt(12) before each combine; the counter holds 15), and
// sched_barrier(0) pins that order against the scheduler's clustering.
template <typename F, int... Is>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
// f(integral_constant<int, i>) for i = 0 .. N-1 with every index a compile-time constant: a #pragma unroll loop of
// 192 steps (AES-256) is not unrolled by the compiler, and its state arrays then live in scratch memory
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// STRIDE: the NB blocks are counters c0, c0 + STRIDE, ... (the quad layout's lane takes every 4th counter block)
template <int NR, int NB, int STRIDE = 1>
__device__ __forceinline__ void ctr_keystream_pipe(const AesLds &a, const CtrPage &pg, const uint32_t *__restrict__ rk,
                                                   uint32_t c0, uint4 (&ks)[NB]) {
    static_assert(NB >= 1 && NB <= 4, "pipeline depth NB - 1 lookups groups of 4 within the 15-read counter");
    constexpr int D = NB - 1;
    constexpr int U = (NR - 2) * 4 * NB;  // units of rounds 3..NR
    // round states by parity; the final round writes into the parity buffer of round NR - 2, dead by then
    uint32_t st[2][NB][4];
    uint32_t ld[D + 1][4];  // lookups of the units in flight (ring)
#pragma unroll
    for (int j = 0; j < NB; j++) pg.two_rounds(a, c0 + STRIDE * j, st[0][j]);  // round-2 state (round 2 is even)
    auto issue = [&](auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int r = 3 + u / (4 * NB), c = (u / NB) & 3, j = u % NB;
        const uint32_t *s = st[(r - 1) & 1][j];
        uint32_t *l = ld[u % (D + 1)];
        l[0] = a.t0<0>(s[c]);
        l[1] = a.t1<1>(s[(c + 1) & 3]);
        l[2] = a.t0<2>(s[(c + 2) & 3]);
        l[3] = a.t1<3>(s[(c + 3) & 3]);
    };
    auto combine = [&](auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int r = 3 + u / (4 * NB), c = (u / NB) & 3, j = u % NB;
        const uint32_t *l = ld[u % (D + 1)];
        const uint32_t k = rk[4 * r + c];
        if constexpr (r < NR) {
            st[r & 1][j][c] = xor3(l[0], l[1], k) ^ rotl16(l[2] ^ l[3]);
        } else {  // final round: S-box bytes only (AesLds::last)
            const uint32_t lo = __builtin_amdgcn_perm(l[1], l[0], 0x0c0c0601u);
            const uint32_t hi = __builtin_amdgcn_perm(l[3], l[2], 0x07020c0cu);
            st[NR & 1][j][c] = xor3(lo, hi, k);
        }
    };
    static_for<D>([&](auto uc) { issue(uc); });
    static_for<U>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        if constexpr (u + D < U) issue(std::integral_constant<int, u + D>{});
        __builtin_amdgcn_sched_barrier(0);
        combine(uc);
        __builtin_amdgcn_sched_barrier(0);
    });
#pragma unroll
    for (int j = 0; j < NB; j++) ks[j] = make_uint4(st[NR & 1][j][0], st[NR & 1][j][1], st[NR & 1][j][2], st[NR & 1][j][3]);
}

// The same pipeline with the units in block-major order (round r, block j, column c) and each block's state updated
// in place: a block's 4 new columns wait in `nw` until its 4th unit has issued its lookups (D <= 3 units ahead), so
// the state is NB x 4 words instead of the parity pair's 2 x NB x 4 -- 12 VGPRs fewer at NB = 4, what lets the quad
// kernel (quad.hip) run more waves per SIMD without spilling.  Same lookups, same combines, same results.
template <int NR, int NB, int STRIDE = 1>
__device__ __forceinline__ void ctr_keystream_inplace(const AesLds &a, const CtrPage &pg, const uint32_t *__restrict__ rk,
                                                      uint32_t c0, uint4 (&ks)[NB]) {
    static_assert(NB >= 1 && NB <= 4, "pipeline depth NB - 1 lookups groups of 4 within the 15-read counter");
    constexpr int D = NB - 1;
    constexpr int U = (NR - 2) * 4 * NB;  // units of rounds 3..NR
    uint32_t st[NB][4];
    uint32_t nw[4];
    uint32_t ld[D + 1][4];  // lookups of the units in flight (ring)
#pragma unroll
    for (int j = 0; j < NB; j++) pg.two_rounds(a, c0 + STRIDE * j, st[j]);
    auto issue = [&](auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int j = (u / 4) % NB, c = u % 4;
        const uint32_t *s = st[j];
        uint32_t *l = ld[u % (D + 1)];
        l[0] = a.t0<0>(s[c]);
        l[1] = a.t1<1>(s[(c + 1) & 3]);
        l[2] = a.t0<2>(s[(c + 2) & 3]);
        l[3] = a.t1<3>(s[(c + 3) & 3]);
    };
    auto combine = [&](auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int r = 3 + u / (4 * NB), j = (u / 4) % NB, c = u % 4;
        const uint32_t *l = ld[u % (D + 1)];
        const uint32_t k = rk[4 * r + c];
        if constexpr (r < NR) {
            nw[c] = xor3(l[0], l[1], k) ^ rotl16(l[2] ^ l[3]);
        } else {  // final round: S-box bytes only (AesLds::last)
            const uint32_t lo = __builtin_amdgcn_perm(l[1], l[0], 0x0c0c0601u);
            const uint32_t hi = __builtin_amdgcn_perm(l[3], l[2], 0x07020c0cu);
            nw[c] = xor3(lo, hi, k);
        }
        if constexpr (c == 3) {  // the block's 4 units have all issued (D <= 3): its new state replaces the old
#pragma unroll
            for (int i = 0; i < 4; i++) st[j][i] = nw[i];
        }
    };
    static_for<D>([&](auto uc) { issue(uc); });
    static_for<U>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        if constexpr (u + D < U) issue(std::integral_constant<int, u + D>{});
        __builtin_amdgcn_sched_barrier(0);
        combine(uc);
        __builtin_amdgcn_sched_barrier(0);
    });
#pragma unroll
    for (int j = 0; j < NB; j++) ks[j] = make_uint4(st[j][0], st[j][1], st[j][2], st[j][3]);
}

// AES T0/T1 bank-replicated tables for the AesLds view: row x = 256 B, dword slot 0..31 = T0[x], 32..63 =
// T1[x] = rotl8 T0[x].  Thread t owns S-box value x = t % 256 (one S-box load) and writes its row's slots in an
// order rotated by x, so a wave's 64 stores of one step go to 32 distinct banks per 32-lane group.  Needs
// blockDim.x % 256 == 0 (every launch: 256..1024 threads).  No barrier inside.
// base: LDS offset of the 64 KiB table region (a multiple of 64 KiB).
__device__ __forceinline__ void build_aes_tables(uint32_t base) {
    const uint32_t x = threadIdx.x & 255u;
    const uint32_t s = d_sbox[x], s2 = xtime4(s);
    const uint32_t t0 = s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
    const uint32_t t1 = __builtin_amdgcn_alignbit(t0, t0, 24);
    for (uint32_t d = threadIdx.x; d < 16384; d += blockDim.x) {
        const uint32_t slot = ((d >> 8) + x) & 63u;
        lds_st32(base + 256u * x + 4u * slot, slot < 32 ? t0 : t1);
    }
}

__device__ __forceinline__ AesLds make_aes(uint32_t base) {
    return AesLds{((threadIdx.x & 31u) << 2) | base};
}

// ---------------------------------------------------------------- AES on four T-tables, quarter-split (quad kernel)
// All four tables T_m = rotl(T0, 8 m) are stored, so a column is T0[a] ^ T1[b] ^ T2[c] ^ T3[d] ^ k in two v_bitop3
// (AesLds needs four VALU: the rotl16 that makes T2/T3 from T0/T1 and its xor) -- 6 VALU per column instead of 8.
// They fit in the same 32 KiB of rows a 2-table layout with 32 copies needs by keeping 8 copies of each and
// splitting every 32-lane LDS group into quarters q = (lane >> 3) & 3 that read DIFFERENT tables in the same
// instruction: row x (256 B, lower 128 B used) holds dword 8 m + i = copy i of T_m[x], lane l reads copy l % 8,
// so in lookup slot K (the column's term K: byte K of word c + K through T_K) quarter q reads table (K + q) % 4 and
// the 32 lanes hit 32 distinct banks.  For that, quarter q holds every state word rotated left by 8 q bits: byte
// (K + q) % 4 of its register is the natural byte K, and T_{K+q}[x] = rotl(T_K[x], 8 q), so the slot sums are the
// natural column rotated by 8 q -- the lane's convention again -- provided the round key is rotated too (one
// v_alignbit per round-key word, shared by the blocks a lane runs together).  The last round picks the S-box bytes
// by per-lane v_perm selectors straight into natural order, so keystream and round-10 key are natural.
// LDS: tables at [65536, 131072); the address is ONE v_perm (byte1 = state byte, byte0 = 4 + 32 m + 4 (lane % 8))
// plus the instruction's offset 65532 (a 16-bit field: 65536 itself does not fit).  The upper 128 B of every row
// are free.  (tools/q4_model.py checks this convention against FIPS-197 in Python.)
struct AesQ4 {
    static constexpr uint32_t kOff = 65532;  // region base 65536 minus the 4 in every byte0
    uint32_t lw;        // byte m = 4 + 32 m + 4 (lane % 8): copy of T_m this lane reads
    uint32_t sel[4];    // slot K: byte0 <- lw.b(T_K), byte1 <- w.b(T_K), bytes 2, 3 <- 0; T_K = (K + q) % 4
    uint32_t selx;      // the counter byte (low byte of its word) through T_(3+q)%4 (CtrPageQ4::two_rounds)
    uint32_t sh;        // rotl by 8 q = alignbit(x, x, sh)
    uint32_t flo, fhi;  // last round: natural S-box bytes 0, 1 (from slots 0, 1) and 2, 3 (slots 2, 3)

    __device__ __forceinline__ static AesQ4 make() {
        AesQ4 a;
        const uint32_t l = threadIdx.x & 7u, q = (threadIdx.x >> 3) & 3u;
        a.lw = 0;
#pragma unroll
        for (uint32_t m = 0; m < 4; m++) a.lw |= (4u + 32u * m + 4u * l) << (8 * m);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            const uint32_t t = (k + q) & 3u;
            a.sel[k] = 0x0c0c0000u | ((4u + t) << 8) | t;
        }
        a.selx = 0x0c0c0400u | ((3u + q) & 3u);
        a.sh = (32u - 8u * q) & 31u;
        // slot K's table entry has the S-box value at bytes (1 + K + q) % 4 and (2 + K + q) % 4
        a.flo = 0x0c0c0000u | ((4u + ((2u + q) & 3u)) << 8) | ((1u + q) & 3u);
        a.fhi = ((4u + q) << 24) | (((3u + q) & 3u) << 16) | 0x0c0cu;
        return a;
    }
    __device__ __forceinline__ uint32_t rot(uint32_t x) const { return __builtin_amdgcn_alignbit(x, x, sh); }
    template <int K>
    __device__ __forceinline__ uint32_t look(uint32_t w) const {
        return lds_ld32(__builtin_amdgcn_perm(w, lw, sel[K]) + kOff);
    }
    __device__ __forceinline__ uint32_t lookx(uint32_t w) const {
        return lds_ld32(__builtin_amdgcn_perm(w, lw, selx) + kOff);
    }
    // column from the 4 slot lookups (kr: the round key word rotated by rot())
    __device__ __forceinline__ static uint32_t comb(uint32_t l0, uint32_t l1, uint32_t l2, uint32_t l3, uint32_t kr) {
        return xor3(xor3(l0, l1, l2), l3, kr);
    }
    // last round from the 4 slot lookups: natural order, natural key word
    __device__ __forceinline__ uint32_t fin(uint32_t l0, uint32_t l1, uint32_t l2, uint32_t l3, uint32_t k) const {
        return xor3(__builtin_amdgcn_perm(l1, l0, flo), __builtin_amdgcn_perm(l3, l2, fhi), k);
    }
    __device__ __forceinline__ uint32_t col(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t kr) const {
        return comb(look<0>(a), look<1>(b), look<2>(c), look<3>(d), kr);
    }
    __device__ __forceinline__ uint32_t last(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) const {
        return fin(look<0>(a), look<1>(b), look<2>(c), look<3>(d), k);
    }
    // Full AES of one natural block (no caching): page-crossing groups, header protection, key setup
    template <int NR>
    __device__ __forceinline__ uint4 encrypt(uint4 in, const uint32_t *__restrict__ rk) const {
        uint32_t s[4] = {rot(in.x ^ rk[0]), rot(in.y ^ rk[1]), rot(in.z ^ rk[2]), rot(in.w ^ rk[3])};
#pragma unroll
        for (int r = 1; r < NR; r++) {
            uint32_t kr[4];
#pragma unroll
            for (int c = 0; c < 4; c++) kr[c] = rot(rk[4 * r + c]);
            const uint32_t u0 = col(s[0], s[1], s[2], s[3], kr[0]), u1 = col(s[1], s[2], s[3], s[0], kr[1]);
            const uint32_t u2 = col(s[2], s[3], s[0], s[1], kr[2]), u3 = col(s[3], s[0], s[1], s[2], kr[3]);
            s[0] = u0; s[1] = u1; s[2] = u2; s[3] = u3;
        }
        const uint32_t *k = rk + 4 * NR;
        return make_uint4(last(s[0], s[1], s[2], s[3], k[0]), last(s[1], s[2], s[3], s[0], k[1]),
                          last(s[2], s[3], s[0], s[1], k[2]), last(s[3], s[0], s[1], s[2], k[3]));
    }
};

// The AesQ4 tables at `base` (65536): thread t owns x = t % 256 (one S-box load) and writes its row's 32 used dwords in
// an order rotated by x (a wave's stores of one step hit distinct banks).  Needs blockDim.x % 256 == 0.  No barrier.
__device__ __forceinline__ void build_aes_tables_q4(uint32_t base) {
    const uint32_t x = threadIdx.x & 255u;
    const uint32_t s = d_sbox[x], s2 = xtime4(s);
    const uint32_t t0 = s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
    for (uint32_t d = threadIdx.x; d < 8192; d += blockDim.x) {
        const uint32_t slot = ((d >> 8) + x) & 31u, m = slot >> 3;
        lds_st32(base + 256u * x + 4u * slot, __builtin_amdgcn_alignbit(t0, t0, (32u - 8u * m) & 31u));
    }
}

// Round keys read through the constant address space (scalar loads into SGPRs; the key records are not written while
// a kernel reads them).  The host pass of this code sees a plain pointer (it never runs there).
#ifdef __HIP_DEVICE_COMPILE__
typedef const __attribute__((address_space(4))) uint4 *RkPtr;
#else
typedef const uint4 *RkPtr;
#endif

// CtrPage in the AesQ4 convention (every constant rotated by 8 q; the counter byte x3 natural)
struct CtrPageQ4 {
    uint32_t k0, k1, k2, k3;  // round-1 output (k0 without the varying slot-3 term)
    uint32_t l0, l1, l2, l3;  // round-2 output without the varying terms
    uint32_t x3;              // rk[3] byte 3 (xored with the counter's low byte)
    uint32_t page;            // c >> 8 these constants belong to

    // from round keys in memory (rounds 0..2 only; RK: a pointer type, e.g. into the constant address space)
    template <typename RK>
    __device__ __forceinline__ void build(const AesQ4 &a, RK rkp, uint32_t n0, uint32_t n1, uint32_t n2, uint32_t pg) {
        const uint4 r0 = rkp[0], r1 = rkp[1], r2 = rkp[2];
        const uint32_t rk[12] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w};
        build(a, rk, n0, n1, n2, pg);
    }
    __device__ __forceinline__ void build(const AesQ4 &a, const uint32_t *__restrict__ rk, uint32_t n0, uint32_t n1,
                                          uint32_t n2, uint32_t pg) {
        const uint32_t s0 = a.rot(n0 ^ rk[0]), s1 = a.rot(n1 ^ rk[1]), s2 = a.rot(n2 ^ rk[2]),
                       s3 = a.rot(bswap32(pg << 8) ^ rk[3]);
        // round 1; the counter's low byte is natural byte 3 of word 3: slot 3 of column 0
        k0 = xor3(a.look<0>(s0), a.look<1>(s1), a.look<2>(s2)) ^ a.rot(rk[4]);
        k1 = a.col(s1, s2, s3, s0, a.rot(rk[5]));
        k2 = a.col(s2, s3, s0, s1, a.rot(rk[6]));
        k3 = a.col(s3, s0, s1, s2, a.rot(rk[7]));
        // round 2 without column 0's terms (slot 0 of col 0, slot 3 of col 1, slot 2 of col 2, slot 1 of col 3)
        l0 = xor3(a.look<1>(k1), a.look<2>(k2), a.look<3>(k3)) ^ a.rot(rk[8]);
        l1 = xor3(a.look<0>(k1), a.look<1>(k2), a.look<2>(k3)) ^ a.rot(rk[9]);
        l2 = xor3(a.look<0>(k2), a.look<1>(k3), a.look<3>(k1)) ^ a.rot(rk[10]);
        l3 = xor3(a.look<0>(k3), a.look<2>(k1), a.look<3>(k2)) ^ a.rot(rk[11]);
        x3 = rk[3] >> 24;
        page = pg;
    }
    // state after rounds 1 and 2 for counter c (same page), AesQ4 convention
    __device__ __forceinline__ void two_rounds(const AesQ4 &a, uint32_t c, uint32_t (&v)[4]) const {
        const uint32_t u0 = k0 ^ a.lookx(c ^ x3);  // natural T3[x] rotated: T_(3+q)[x]
        v[0] = l0 ^ a.look<0>(u0);
        v[1] = l1 ^ a.look<3>(u0);
        v[2] = l2 ^ a.look<2>(u0);
        v[3] = l3 ^ a.look<1>(u0);
    }
};

// ctr_keystream_inplace on AesQ4 (same unit order and pipeline; the round's 4 key words rotated once per round for
// all NB blocks).  Reads rk[12 ..] only (rounds 3..NR: rounds 1 and 2 are the page's).
#ifndef QPP_Q4_DEPTH
#define QPP_Q4_DEPTH 3  // units (4 lookups each) issued ahead of the one combined (<= NB - 1)
#endif
template <int NR, int NB, int STRIDE = 1>
__device__ __forceinline__ void ctr_keystream_q4(const AesQ4 &a, const CtrPageQ4 &pg, const uint32_t *__restrict__ rk,
                                                 uint32_t c0, uint4 (&ks)[NB]) {
    static_assert(NB >= 1 && NB <= 4, "pipeline depth NB - 1 lookups groups of 4 within the 15-read counter");
    constexpr int D = NB - 1 < QPP_Q4_DEPTH ? NB - 1 : QPP_Q4_DEPTH;
    constexpr int U = (NR - 2) * 4 * NB;  // units of rounds 3..NR
    uint32_t st[NB][4];
    uint32_t nw[4];
    uint32_t kr[4];
    uint32_t ld[D + 1][4];
#pragma unroll
    for (int j = 0; j < NB; j++) pg.two_rounds(a, c0 + STRIDE * j, st[j]);
    auto issue = [&](auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int j = (u / 4) % NB, c = u % 4;
        const uint32_t *s = st[j];
        uint32_t *l = ld[u % (D + 1)];
        l[0] = a.look<0>(s[c]);
        l[1] = a.look<1>(s[(c + 1) & 3]);
        l[2] = a.look<2>(s[(c + 2) & 3]);
        l[3] = a.look<3>(s[(c + 3) & 3]);
    };
    auto combine = [&](auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int r = 3 + u / (4 * NB), j = (u / 4) % NB, c = u % 4;
        const uint32_t *l = ld[u % (D + 1)];
        if constexpr (u % (4 * NB) == 0) {  // the round's first unit: its key words (rotated but in the last round)
#pragma unroll
            for (int i = 0; i < 4; i++) kr[i] = r < NR ? a.rot(rk[4 * r + i]) : rk[4 * r + i];
        }
        if constexpr (r < NR) {
            nw[c] = AesQ4::comb(l[0], l[1], l[2], l[3], kr[c]);
        } else {
            nw[c] = a.fin(l[0], l[1], l[2], l[3], kr[c]);
        }
        if constexpr (c == 3) {
#pragma unroll
            for (int i = 0; i < 4; i++) st[j][i] = nw[i];
        }
    };
    static_for<D>([&](auto uc) { issue(uc); });
    static_for<U>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        if constexpr (u + D < U) issue(std::integral_constant<int, u + D>{});
        __builtin_amdgcn_sched_barrier(0);
        combine(uc);
        __builtin_amdgcn_sched_barrier(0);
    });
#pragma unroll
    for (int j = 0; j < NB; j++) ks[j] = make_uint4(st[j][0], st[j][1], st[j][2], st[j][3]);
}

// ---------------------------------------------------------------- packet view, header protection (both AES kernels)
struct PacketView {
    uint8_t *base;       // packet start (AAD)
    uint32_t aad_len, len, pn_len;
    uint32_t n0, n1, n2; // nonce words
};

__device__ __forceinline__ PacketView load_packet(const qpp_pkt &d, const DevKey *__restrict__ key, uint8_t *arena) {
    PacketView p;
    p.base = arena + d.off;
    p.aad_len = d.aad_len;
    p.len = d.pt_len;
    p.pn_len = d.pn_len;
    // Iv::nonce: iv XOR (0u32 || pn_be64)  (src/iv.rs:27-39)
    p.n0 = key->iv[0];
    p.n1 = key->iv[1] ^ bswap32((uint32_t)(d.pn >> 32));
    p.n2 = key->iv[2] ^ bswap32((uint32_t)d.pn);
    return p;
}

// apply_header_protection (header_crypto.rs:80-95) as two independent loads issued before the mask is known and
// up to 5 independent byte stores: no dependent byte-load loop after the mask.  The dword at base + hdr_len may
// run past the PN into the payload (callers checked payload >= 4 - pn_len); only bytes [0, pn_len) are stored.
struct HdrBytes {
    uint32_t b0, pnw;
};
__device__ __forceinline__ HdrBytes hdr_load(const uint8_t *base, uint32_t hdr_len) {
    HdrBytes h;
    h.b0 = base[0];
    __builtin_memcpy(&h.pnw, base + hdr_len, 4);
    return h;
}

__device__ __forceinline__ void hdr_apply(uint8_t *base, uint32_t hdr_len, uint32_t pn_len, HdrBytes h, uint32_t m0,
                                          uint32_t m1) {
    const uint32_t nb0 = h.b0 ^ (m0 & ((h.b0 & 0x80) ? 0x0fu : 0x1fu));
    base[0] = (uint8_t)nb0;
    // hdr_len == 0 (a header of PN bytes only): PN byte 0 is byte 0 after its first-byte masking, as in the
    // reference's in-place order
    const uint32_t pnw = hdr_len ? h.pnw : (h.pnw & 0xffffff00u) | (nb0 & 0xffu);
    const uint32_t x = pnw ^ ((m0 >> 8) | (m1 << 24));
    base[hdr_len] = (uint8_t)x;
    if (pn_len > 1) base[hdr_len + 1] = (uint8_t)(x >> 8);
    if (pn_len > 2) base[hdr_len + 2] = (uint8_t)(x >> 16);
    if (pn_len > 3) base[hdr_len + 3] = (uint8_t)(x >> 24);
}

// Header protection mask from the 16-byte sample (first 5 bytes of AES_hp(sample)).  The HP round keys are read
// once per packet into VGPRs: hoisted into SGPRs for the whole kernel they pushed the packet round keys out of
// SGPRs (measured: 36 SGPR spills and per-iteration round-key reloads, a slower seal).  Split in two so that a
// caller can issue the key and header loads early and let their latency pass under other work.
template <int HNR>
struct HpPrefetch {
    uint32_t rk[4 * (HNR + 1)];
    HdrBytes h;
    __device__ __forceinline__ void load(const uint32_t *hp_rk_g, const uint8_t *base, uint32_t hdr_len,
                                         uint32_t flags) {
        // launder the pointer through a VGPR: the loads below cannot be hoisted or kept in SGPRs
        uint64_t a = (uint64_t)hp_rk_g;
        asm volatile("" : "+v"(a));
        const uint4 *src = (const uint4 *)a;
#pragma unroll
        for (int i = 0; i < HNR + 1; i++) {
            const uint4 v = src[i];
            rk[4 * i] = v.x; rk[4 * i + 1] = v.y; rk[4 * i + 2] = v.z; rk[4 * i + 3] = v.w;
        }
        h = (flags & QPP_HP_APPLY) ? hdr_load(base, hdr_len) : HdrBytes{0, 0};
    }
    // round keys in LDS (finish_lds reads them there when needed): only the header bytes are prefetched
    __device__ __forceinline__ void load_hdr(const uint8_t *base, uint32_t hdr_len, uint32_t flags) {
        h = (flags & QPP_HP_APPLY) ? hdr_load(base, hdr_len) : HdrBytes{0, 0};
    }
    __device__ __forceinline__ void finish_lds(const AesLds &aes, uint32_t lds_rk, uint4 sample, uint8_t *base,
                                               uint32_t hdr_len, uint32_t pn_len, uint8_t *mask_out, uint32_t flags) {
#pragma unroll
        for (int i = 0; i < 4 * (HNR + 1); i++) rk[i] = lds_ld32(lds_rk + 4 * i);
        finish(aes, sample, base, hdr_len, pn_len, mask_out, flags);
    }
    __device__ __forceinline__ void finish(const AesLds &aes, uint4 sample, uint8_t *base, uint32_t hdr_len,
                                           uint32_t pn_len, uint8_t *mask_out, uint32_t flags) const {
        apply(aes.encrypt<HNR>(sample, rk), base, hdr_len, pn_len, mask_out, flags);
    }
    // m = AES_hp(sample), computed by the caller
    __device__ __forceinline__ void apply(uint4 m, uint8_t *base, uint32_t hdr_len, uint32_t pn_len, uint8_t *mask_out,
                                          uint32_t flags) const {
        if (flags & QPP_HP_MASK_OUT) {
            mask_out[0] = (uint8_t)m.x; mask_out[1] = (uint8_t)(m.x >> 8); mask_out[2] = (uint8_t)(m.x >> 16);
            mask_out[3] = (uint8_t)(m.x >> 24); mask_out[4] = (uint8_t)m.y;
        }
        if (flags & QPP_HP_APPLY) hdr_apply(base, hdr_len, pn_len, h, m.x, m.y);  // header_crypto.rs:80-95
    }
};

template <int HNR>
__device__ __forceinline__ void hp_finish(const AesLds &aes, const uint32_t *hp_rk_g, uint4 sample,
                                          uint8_t *base, uint32_t hdr_len, uint32_t pn_len, uint8_t *mask_out,
                                          uint32_t flags) {
    HpPrefetch<HNR> hp;
    hp.load(hp_rk_g, base, hdr_len, flags);
    hp.finish(aes, sample, base, hdr_len, pn_len, mask_out, flags);
}

// ---------------------------------------------------------------- ChaCha20 block (RFC 8439 §2.3) and the ChaCha HP mask
__device__ __forceinline__ uint32_t rotl(uint32_t v, int c) { return __builtin_amdgcn_alignbit(v, v, 32 - c); }

#define QR(a, b, c, d)                \
    a += b; d ^= a; d = rotl(d, 16);  \
    c += d; b ^= c; b = rotl(b, 12);  \
    a += b; d ^= a; d = rotl(d, 8);   \
    c += d; b ^= c; b = rotl(b, 7);

// RFC 8439 §2.3 block function: out[16] = keystream words
__device__ __forceinline__ void chacha_block(const uint32_t k[8], uint32_t ctr, uint32_t n0, uint32_t n1, uint32_t n2,
                                             uint32_t out[16]) {
    uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, k[0], k[1], k[2], k[3],
                      k[4], k[5], k[6], k[7], ctr, n0, n1, n2};
#pragma unroll
    for (int i = 0; i < 10; i++) {
        QR(x[0], x[4], x[8], x[12]);
        QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]);
        QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]);
        QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]);
        QR(x[3], x[4], x[9], x[14]);
    }
    const uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, k[0], k[1], k[2], k[3],
                             k[4], k[5], k[6], k[7], ctr, n0, n1, n2};
#pragma unroll
    for (int i = 0; i < 16; i++) out[i] = x[i] + in[i];
}

__device__ __forceinline__ uint32_t chacha_hp_word(const uint32_t hk[8], uint4 sample, uint32_t *w1) {
    uint32_t ks[16];
    chacha_block(hk, sample.x, sample.y, sample.z, sample.w, ks);
    *w1 = ks[1];
    return ks[0];
}

// ---------------------------------------------------------------- receive-side header unprotection of one packet
//  for unprotect_kernel and the fused receive kernel (aes_gcm.hip aes_gcm_rx_kernel):
//   sample at header_len + 4 (payload.rs:151-169) -> mask (header_key.rs:52-56) -> remove_header_protection in place
//   (header_crypto.rs:98-123: first byte, pn_len = (b0 & 3) + 1, PN bytes) -> expand the PN against the space's
//   largest acknowledged PN (packet/number/mod.rs:191-238) -> the packet key by the key-phase bit 0x04
//   (key_phase.rs:12,46; KeySet::decrypt_packet, keyset.rs:113-143; long headers: key_idx[0]) -> the qpp_pkt the
//   open consumes.  A packet too short for the sample is DECODE_ERROR and marked QPP_PKT_SKIP; key slots outside the
//   table are INTERNAL_ERROR (never read).  `aes` views T-tables already in LDS.
// AES_HP = false (the fused ChaCha receive, no T-tables in LDS): a header key that is not a ChaCha20 key is refused
// (INTERNAL_ERROR) -- the host launches that kernel only when no AES record is live.  A header-key slot that holds no
// key at all (freed) is refused by both forms, before any header byte is written.
// chosen (optional): the first 16 bytes (suite, nr, hp_nr, live) of the record of the key the packet was sent to,
// loaded with the rest (the fused receive checks it is a live packet key without another round trip).
// AES: the T-table view (AesLds, or AesQ4 in the quad kernels).
template <bool AES_HP = true, typename AES = AesLds>
__device__ __forceinline__ qpp_pkt rx_unprotect_one(const AES &aes, const DevKey *__restrict__ keys, uint32_t key_cap,
                                                    const qpp_rx_pkt &r, uint8_t *__restrict__ arena, int8_t *status,
                                                    uint32_t i, uint4 *chosen = nullptr) {
    qpp_pkt d{};
    d.off = r.off;
    d.key_idx = r.key_idx[0];
    d.aad_len = r.header_len;
    uint8_t *base = arena + r.off;
    const uint32_t hdr = r.header_len;
    if ((uint32_t)r.len < hdr + 4 + 16) {
        d.flags = QPP_PKT_SKIP;
        status[i] = QPP_DECODE_ERROR;
        return d;
    }
    if (r.key_idx[0] >= key_cap || r.key_idx[1] >= key_cap) {  // slots outside the key table: refused, never read
        d.flags = QPP_PKT_SKIP;
        d.key_idx = 0;
        status[i] = QPP_INTERNAL_ERROR;
        return d;
    }
    const DevKey *__restrict__ hk = keys + r.key_idx[0];
    // The three packet loads (byte 0, the 4 bytes that may hold the PN -- len >= hdr + 20 was checked above -- and
    // the sample) are issued together with the key record's, before its check: one memory round trip for both
    // instead of two in a row (a refused packet's bytes are read but never written)
    const uint4 smp = ld16(base + hdr + 4);
    uint32_t pnw;
    __builtin_memcpy(&pnw, base + hdr, 4);
    uint8_t b0 = base[0];
    const uint4 hw = *(const uint4 *)hk;  // suite, nr, hp_nr, live
    uint4 hw1 = make_uint4(0, 0, 0, 0);
    if (chosen) hw1 = *(const uint4 *)(keys + r.key_idx[1]);
    // the header key's round keys (AES: up to 15 x 4 words; ChaCha20: the first 8), issued now as well
    uint32_t hrk[60];
#pragma unroll
    for (int q = 0; q < (AES_HP ? 15 : 2); q++) {
        const uint4 v = ((const uint4 *)hk->hp_rk)[q];
        hrk[4 * q] = v.x; hrk[4 * q + 1] = v.y; hrk[4 * q + 2] = v.z; hrk[4 * q + 3] = v.w;
    }
    if (hw.w == 0 || (!AES_HP && hw.x != QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256)) {
        d.flags = QPP_PKT_SKIP;
        status[i] = QPP_INTERNAL_ERROR;
        return d;
    }
    uint32_t m0, m1;
    if (hw.x == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256) {
        m0 = chacha_hp_word(hrk, smp, &m1);
    } else if constexpr (AES_HP) {
        const uint4 m = hw.z == 10 ? aes.template encrypt<10>(smp, hrk) : aes.template encrypt<14>(smp, hrk);
        m0 = m.x;
        m1 = m.y;
    } else {
        m0 = m1 = 0;  // unreachable: refused above
    }
    const bool is_long = (b0 & 0x80) != 0;
    b0 ^= (uint8_t)m0 & (is_long ? 0x0f : 0x1f);
    base[0] = b0;
    const uint32_t pn_len = (b0 & 3u) + 1u;
    const uint32_t mm = (m0 >> 8) | (m1 << 24);  // mask bytes 1..4, byte j of the PN at bits 8j
    if (hdr == 0) pnw = (pnw & 0xffffff00u) | b0;  // PN byte 0 is byte 0, already unmasked above
    // unmask PN bytes [0, pn_len); bytes past pn_len are written back unchanged (this lane owns the packet)
    pnw ^= pn_len == 4u ? mm : (mm & ((1u << (8u * pn_len)) - 1u));
    __builtin_memcpy(base + hdr, &pnw, 4);
    const uint64_t trunc = bswap32(pnw) >> (8u * (4u - pn_len));  // PN bytes big-endian
    d.pn = decode_packet_number(r.largest_pn & kPnMask, trunc, 8 * pn_len);
    const bool phase1 = !is_long && (b0 & 0x04);
    d.key_idx = phase1 ? r.key_idx[1] : r.key_idx[0];
    if (chosen) *chosen = phase1 ? hw1 : hw;
    d.aad_len = (uint16_t)(hdr + pn_len);
    d.pt_len = (uint16_t)(r.len - hdr - pn_len - 16);
    d.pn_len = (uint8_t)pn_len;
    return d;
}

// ---------------------------------------------------------------- per-wave payload staging
// Coalesced payload I/O through a per-wave LDS staging area.  A lane-per-packet load touches 64 scattered lines
// per wave instruction (packets are ~1.2 KB apart) and thrashes L1 (measured: with the payload I/O confined to an
// L1-resident window the seal ran 1.9 -> 1.5 ms at NB = 4, and 3.1 -> 1.2 ms at NB = 2 / 1024 threads).  So each
// group's NB x 16 B per packet is moved cooperatively: in wave instruction i, the NB lanes of a lane-group of NB
// load the NB chunks of ONE packet (p = PPI i + lane / NB, 64 B contiguous at NB = 4), write them to LDS at slot
// 64 i + lane, and every lane then reads its own packet's NB blocks back.  Outputs go the other way.  The chunk a
// lane moves is rotated by rho(p) so that the owner's accesses (slot(p, k) = 64 (p / PPI) + NB (p % PPI) +
// ((k + rho(p)) % NB)) hit distinct bank quads per lane group (conflict-free).
template <int NB>
struct Stage {
    static constexpr uint32_t PPI = 64 / NB, ROT = 16 / NB;
    uint32_t base;  // this wave's 64 * NB * 16 byte region
    uint32_t lane;
    // rotation of packet p's chunks: NB = 4: (p/2 + p/16) % 4 keeps both the owner's ds_read_b128 (16-lane groups, 64
    // banks) and its ds_write_b128 (8-lane groups, 32 banks) conflict-free (p/4 left the writes 2-way;
    // tests/test_kernel_layouts.py checks both); other NB: p / ROT (reads only)
    static __device__ __forceinline__ uint32_t rho(uint32_t p) {
        return NB == 4 ? ((p >> 1) + (p >> 4)) & 3u : p / ROT;
    }
    __device__ __forceinline__ uint32_t own(uint32_t k) const {  // LDS address of my packet's chunk k
        return base + 16u * (64u * (lane / PPI) + NB * (lane % PPI) + ((k + rho(lane)) % NB));
    }
    __device__ __forceinline__ uint32_t coop(int i) const { return base + 16u * (64u * i + lane); }
    __device__ __forceinline__ uint32_t coop_src(int i) const { return PPI * i + lane / NB; }  // packet lane
    __device__ __forceinline__ uint32_t coop_chunk(int i) const {
        const uint32_t p = coop_src(i);
        return ((lane % NB) + NB - rho(p) % NB) % NB;
    }
};

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
    return v;
}
__device__ __forceinline__ void wave_lds_sync() {
    // the wave's own LDS traffic is in order; this keeps the compiler from moving LDS accesses across the exchange
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace dev
}  // namespace qpp
