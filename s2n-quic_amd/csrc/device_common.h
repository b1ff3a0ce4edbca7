// device_common.h — device-side building blocks shared by the packet-protection kernels (gfx950).
#pragma once

#include "qpp_internal.h"

namespace qpp {
namespace dev {

constexpr uint32_t kLdsGhash = 0;
constexpr uint32_t kLdsAes = 65536;
constexpr uint32_t kLdsV = 131072;
constexpr uint32_t kLdsBytes = kLdsV + 128 * 16;

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

// ---------------------------------------------------------------- AES with bank-replicated LDS T-tables
struct AesLds {
    const uint8_t *lds;
    uint32_t laneword;  // byte0 = 4 * (lane % 32), byte2 = 0x01 (64 KiB table base)

    // T0[byte k of w] / T1[byte k of w]
    template <int K>
    __device__ __forceinline__ uint32_t addr(uint32_t w) const {
        // v_perm_b32: byte0 <- laneword.b0, byte1 <- w.bK, byte2 <- laneword.b2, byte3 <- 0
        return __builtin_amdgcn_perm(w, laneword, (0x0cu << 24) | (2u << 16) | ((4u + K) << 8) | 0u);
    }
    template <int K>
    __device__ __forceinline__ uint32_t t0(uint32_t w) const { return *(const uint32_t *)(lds + addr<K>(w)); }
    template <int K>
    __device__ __forceinline__ uint32_t t1(uint32_t w) const { return *(const uint32_t *)(lds + addr<K>(w) + 128); }

    __device__ __forceinline__ uint32_t col(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) const {
        return t0<0>(a) ^ t1<1>(b) ^ rotl16(t0<2>(c) ^ t1<3>(d)) ^ k;
    }
    __device__ __forceinline__ uint32_t last(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) const {
        // S[x] = byte1 of T0[x]; = byte2 and byte3 of T1[x]
        uint32_t lo = __builtin_amdgcn_perm(t1<1>(b), t0<0>(a), 0x0c0c0601u);
        uint32_t hi = __builtin_amdgcn_perm(t1<3>(d), t0<2>(c), 0x07020c0cu);
        return (lo | hi) ^ k;
    }

    template <int NR>
    __device__ __forceinline__ uint4 encrypt(uint4 in, const uint32_t *__restrict__ rk) const {
        uint32_t s0 = in.x ^ rk[0], s1 = in.y ^ rk[1], s2 = in.z ^ rk[2], s3 = in.w ^ rk[3];
#pragma unroll
        for (int r = 1; r < NR; r++) {
            uint32_t u0 = col(s0, s1, s2, s3, rk[4 * r + 0]);
            uint32_t u1 = col(s1, s2, s3, s0, rk[4 * r + 1]);
            uint32_t u2 = col(s2, s3, s0, s1, rk[4 * r + 2]);
            uint32_t u3 = col(s3, s0, s1, s2, rk[4 * r + 3]);
            s0 = u0; s1 = u1; s2 = u2; s3 = u3;
        }
        return make_uint4(last(s0, s1, s2, s3, rk[4 * NR + 0]), last(s1, s2, s3, s0, rk[4 * NR + 1]),
                          last(s2, s3, s0, s1, rk[4 * NR + 2]), last(s3, s0, s1, s2, rk[4 * NR + 3]));
    }
};


// AES T0/T1 bank-replicated tables for the AesLds view: dword d -> row x = d >> 6, slot = d & 63
// (slots 32..63 hold T1 = rotl8 T0).  No barrier inside.
__device__ __forceinline__ void build_aes_tables(uint8_t *lds) {
    for (uint32_t d = threadIdx.x; d < 16384; d += blockDim.x) {
        uint32_t x = d >> 6, slot = d & 63;
        uint32_t s = d_sbox[x], s2 = xtime4(s);
        uint32_t t0 = s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
        *(uint32_t *)(lds + kLdsAes + 4 * d) = slot < 32 ? t0 : __builtin_amdgcn_alignbit(t0, t0, 24);
    }
}

__device__ __forceinline__ AesLds make_aes(const uint8_t *lds) {
    return AesLds{lds, ((threadIdx.x & 31u) << 2) | (1u << 16)};
}

}  // namespace dev
}  // namespace qpp
