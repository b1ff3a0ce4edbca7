// aes_core.hip — microbenchmarks that decide the AES-GCM formulation (VERDICT r2 "Next round" #1, SURVEY §7:
// "the T-table vs byte-sliced (v_bitop3) AES choice is decided by microbenchmark").  No memory I/O in the timed
// kernels: every lane folds its keystream / GHASH value into a register accumulator, one word per lane is stored.
//
//   issue <op>     wave64 issue cost of single VALU ops (8 independent chains per lane), cycles from s_memtime
//   ttab2          CTR keystream, product T-table core (T0/T1 bank-replicated, T2/T3 = rotl16; CtrPage + pipe)
//   ttab4          the same with all four tables in LDS (T2/T3 stored: 2 VALU per column fewer, 64 KiB more LDS)
//   bitslice       CTR keystream, bitsliced AES-128 (Boyar-Peralta S-box circuit; 32 blocks per lane, v_bitop3 by
//                  the compiler), no LDS at all
//   ghash8         GHASH product chain alone, 8-bit tables (product lane kernel)
//   aesgh          ttab2 + ghash8 interleaved per 4-block group as process_packet runs them (the compute floor of the
//                  product kernel without payload I/O)
// Every AES variant is checked against OpenSSL AES-128-ECB of the same counter blocks.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 aes_core.hip -o /tmp/aes_core -lcrypto
#include <hip/hip_runtime.h>
#include <openssl/evp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../s2n-quic_amd/csrc/device_common.h"
#include "../../s2n-quic_amd/csrc/ghash.h"

using namespace qpp;
using namespace qpp::dev;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

struct Clock {
    uint64_t t0, t1, r0, r1;  // s_memtime / s_memrealtime at the start and end of workgroup 0's thread 0
};

// per-workgroup census (start/end s_memrealtime, HW_ID, XCC_ID), when g_census is set
struct WgRec {
    uint64_t r0, r1;
    uint32_t hwid, xcc;
};
__device__ WgRec *g_census;
__device__ __forceinline__ void census(bool end) {
    if (threadIdx.x == 0 && g_census) {
        WgRec *w = g_census + blockIdx.x;
        if (!end) {
            w->r0 = __builtin_amdgcn_s_memrealtime();
            w->hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            w->xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);
        } else {
            w->r1 = __builtin_amdgcn_s_memrealtime();
        }
    }
}
__device__ __forceinline__ void clk_start(Clock *c) {
    census(false);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        c->t0 = __builtin_amdgcn_s_memtime();
        c->r0 = __builtin_amdgcn_s_memrealtime();
    }
}
__device__ __forceinline__ void clk_end(Clock *c) {
    census(true);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        c->t1 = __builtin_amdgcn_s_memtime();
        c->r1 = __builtin_amdgcn_s_memrealtime();
    }
}

// ---------------------------------------------------------------- VALU issue cost
template <int OP>
__global__ __launch_bounds__(256) void issue_k(uint32_t *out, int iters, uint32_t seed, Clock *clk) {
    uint32_t u[8];
    float f[8];
    for (int i = 0; i < 8; i++) {
        u[i] = seed * (i + 3) + threadIdx.x;
        f[i] = (float)u[i];
    }
    const uint32_t c = seed | 0x10101u;
    __syncthreads();
    clk_start(clk);
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (OP == 0) u[i] = u[i] ^ (c + i);
            if (OP == 1) u[i] = __builtin_amdgcn_bitop3_b32(u[i], c, c + i, 0x96);
            if (OP == 2) u[i] = __builtin_amdgcn_perm(u[i], c + i, 0x05040100u);
            if (OP == 3) u[i] = u[i] + (c + i);
            if (OP == 4) f[i] = __builtin_fmaf(f[i], 1.0000001f, 0.5f);
            if (OP == 5) u[i] = __builtin_amdgcn_alignbit(u[i], u[i], 7);
            if (OP == 6) u[i] = (u[i] & (c + i)) ^ c;  // candidate for one v_bitop3
        }
    }
    clk_end(clk);
    uint32_t s = 0;
    for (int i = 0; i < 8; i++) s += u[i] + (uint32_t)f[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// ---------------------------------------------------------------- T-table CTR core
// T2/T3 region for ttab4: [0, 64 KiB) rows x = T2[x] x 32 | T3[x] x 32 (T0/T1 at kLdsAes as in the product)
__device__ __forceinline__ void build_aes_tables23(uint32_t base) {
    const uint32_t x = threadIdx.x & 255u;
    const uint32_t s = d_sbox[x], s2 = xtime4(s);
    const uint32_t t0 = s2 | (s << 8) | (s << 16) | ((s2 ^ s) << 24);
    const uint32_t t1 = __builtin_amdgcn_alignbit(t0, t0, 24);
    const uint32_t t2 = rotl16(t0), t3 = rotl16(t1);
    for (uint32_t d = threadIdx.x; d < 16384; d += blockDim.x) {
        const uint32_t slot = ((d >> 8) + x) & 63u;
        lds_st32(base + 256u * x + 4u * slot, slot < 32 ? t2 : t3);
    }
}
template <int K>
__device__ __forceinline__ uint32_t addr23(const AesLds &a, uint32_t w) {  // T2 row in [0, 64 KiB): byte2 = 0
    return __builtin_amdgcn_perm(w, a.laneword, (0x0cu << 24) | (0x0cu << 16) | ((4u + K) << 8) | 0u);
}

template <int NR, int NB, bool FOUR>
__device__ __forceinline__ void keystream_pipe(const AesLds &a, const CtrPage &pg, const uint32_t *__restrict__ rk,
                                               uint32_t c0, uint4 (&ks)[NB]) {
    constexpr int D = NB - 1;
    constexpr int U = (NR - 2) * 4 * NB;
    uint32_t st[2][NB][4];
    uint32_t ld[D + 1][4];
#pragma unroll
    for (int j = 0; j < NB; j++) pg.two_rounds(a, c0 + j, st[0][j]);
    auto issue = [&](auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int r = 3 + u / (4 * NB), c = (u / NB) & 3, j = u % NB;
        const uint32_t *s = st[(r - 1) & 1][j];
        uint32_t *l = ld[u % (D + 1)];
        l[0] = a.t0<0>(s[c]);
        l[1] = a.t1<1>(s[(c + 1) & 3]);
        if constexpr (FOUR && r < NR) {
            l[2] = lds_ld32(addr23<2>(a, s[(c + 2) & 3]));
            l[3] = lds_ld32(addr23<3>(a, s[(c + 3) & 3]) + 128);
        } else {
            l[2] = a.t0<2>(s[(c + 2) & 3]);
            l[3] = a.t1<3>(s[(c + 3) & 3]);
        }
    };
    auto combine = [&](auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int r = 3 + u / (4 * NB), c = (u / NB) & 3, j = u % NB;
        const uint32_t *l = ld[u % (D + 1)];
        const uint32_t k = rk[4 * r + c];
        if constexpr (r < NR) {
            if constexpr (FOUR) st[r & 1][j][c] = xor3(xor3(l[0], l[1], k), l[2], l[3]);
            else st[r & 1][j][c] = xor3(l[0], l[1], k) ^ rotl16(l[2] ^ l[3]);
        } else {
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

// each lane: P "packets" (nonce = f(lane, p)) x G groups of 4 counter blocks starting at counter 1
template <bool FOUR, bool GH, int WG>
__global__ __launch_bounds__(WG) void ttab_k(const uint32_t *__restrict__ rk_g, const DevKey *__restrict__ key, int P,
                                              int G, uint4 *out, uint4 *chk, Clock *clk) {
    constexpr int NB = 4, NR = 10;
    if (FOUR) build_aes_tables23(0);
    if (GH) {
        build_tables(key);  // GHASH tables at [0, 64 KiB) + AES T0/T1 at 64 KiB (+ barrier)
    } else {
        build_aes_tables(kLdsAes);
        __syncthreads();
    }
    uint32_t rk[44];
#pragma unroll
    for (int r = 0; r < 44; r++) rk[r] = __builtin_amdgcn_readfirstlane(rk_g[r]);
    const AesLds aes = make_aes(kLdsAes);
    const GhashT<true> gh = GhashT<true>::make();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint4 acc = make_uint4(0, 0, 0, 0), z = make_uint4(0, 0, 0, 0);
    __syncthreads();
    clk_start(clk);
    for (int p = 0; p < P; p++) {
        const uint32_t n0 = tid * 0x9e3779b9u, n1 = (uint32_t)p * 0x85ebca6bu + tid, n2 = 0x01234567u ^ tid;
        CtrPage pg;
        pg.build(aes, rk, n0, n1, n2, 0);
        for (int g = 0; g < G; g++) {
            uint4 ks[NB];
            keystream_pipe<NR, NB, FOUR>(aes, pg, rk, (uint32_t)(NB * g + 1), ks);
            if (chk && tid == 0 && p == 0 && g == 0)
                for (int j = 0; j < NB; j++) chk[j] = ks[j];
            if constexpr (GH) {
#pragma unroll
                for (int j = 0; j < NB; j++) z = gh.mulx(z, ks[j]);
            } else {
#pragma unroll
                for (int j = 0; j < NB; j++) acc = acc ^ ks[j];
            }
        }
    }
    clk_end(clk);
    out[tid] = acc ^ z;
}

// GHASH chain alone: B products per lane
__global__ __launch_bounds__(512) void ghash_k(const DevKey *__restrict__ key, int B, uint4 *out, Clock *clk) {
    build_tables(key);
    const GhashT<true> gh = GhashT<true>::make();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint4 z = make_uint4(tid, tid * 3, tid * 5, tid * 7);
    uint4 c = make_uint4(tid ^ 1, tid ^ 2, tid ^ 3, tid ^ 4);
    clk_start(clk);
    for (int b = 0; b < B; b += 4) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            z = gh.mulx(z, c);
            c.x += 0x9e3779b9u;
        }
    }
    clk_end(clk);
    out[tid] = z;
}

// ---------------------------------------------------------------- bitsliced AES-128 CTR
#define BP_SBOX(T, U0, U1, U2, U3, U4, U5, U6, U7, S0, S1, S2, S3, S4, S5, S6, S7)                                      \
    do {                                                                                                                \
        T T1 = U0 ^ U3, T2 = U0 ^ U5, T3 = U0 ^ U6, T4 = U3 ^ U5, T5 = U4 ^ U6, T6 = T1 ^ T5, T7 = U1 ^ U2;             \
        T T8 = U7 ^ T6, T9 = U7 ^ T7, T10 = T6 ^ T7, T11 = U1 ^ U5, T12 = U2 ^ U5, T13 = T3 ^ T4, T14 = T6 ^ T11;      \
        T T15 = T5 ^ T11, T16 = T5 ^ T12, T17 = T9 ^ T16, T18 = U3 ^ U7, T19 = T7 ^ T18, T20 = T1 ^ T19;               \
        T T21 = U6 ^ U7, T22 = T7 ^ T21, T23 = T2 ^ T22, T24 = T2 ^ T10, T25 = T20 ^ T17, T26 = T3 ^ T16;              \
        T T27 = T1 ^ T12;                                                                                               \
        T M1 = T13 & T6, M2 = T23 & T8, M3 = T14 ^ M1, M4 = T19 & U7, M5 = M4 ^ M1, M6 = T3 & T16, M7 = T22 & T9;      \
        T M8 = T26 ^ M6, M9 = T20 & T17, M10 = M9 ^ M6, M11 = T1 & T15, M12 = T4 & T27, M13 = M12 ^ M11;              \
        T M14 = T2 & T10, M15 = M14 ^ M11, M16 = M3 ^ M2, M17 = M5 ^ T24, M18 = M8 ^ M7, M19 = M10 ^ M15;              \
        T M20 = M16 ^ M13, M21 = M17 ^ M15, M22 = M18 ^ M13, M23 = M19 ^ T25, M24 = M22 ^ M23, M25 = M22 & M20;        \
        T M26 = M21 ^ M25, M27 = M20 ^ M21, M28 = M23 ^ M25, M29 = M28 & M27, M30 = M26 & M24, M31 = M20 & M23;       \
        T M32 = M27 & M31, M33 = M27 ^ M25, M34 = M21 & M22, M35 = M24 & M34, M36 = M24 ^ M25, M37 = M21 ^ M29;       \
        T M38 = M32 ^ M33, M39 = M23 ^ M30, M40 = M35 ^ M36, M41 = M38 ^ M40, M42 = M37 ^ M39, M43 = M37 ^ M38;       \
        T M44 = M39 ^ M40, M45 = M42 ^ M41, M46 = M44 & T6, M47 = M40 & T8, M48 = M39 & U7, M49 = M43 & T16;          \
        T M50 = M38 & T9, M51 = M37 & T17, M52 = M42 & T15, M53 = M45 & T27, M54 = M41 & T10, M55 = M44 & T13;        \
        T M56 = M40 & T23, M57 = M39 & T19, M58 = M43 & T3, M59 = M38 & T22, M60 = M37 & T20, M61 = M42 & T1;         \
        T M62 = M45 & T4, M63 = M41 & T2;                                                                              \
        T L0 = M61 ^ M62, L1 = M50 ^ M56, L2 = M46 ^ M48, L3 = M47 ^ M55, L4 = M54 ^ M58, L5 = M49 ^ M61;             \
        T L6 = M62 ^ L5, L7 = M46 ^ L3, L8 = M51 ^ M59, L9 = M52 ^ M53, L10 = M53 ^ L4, L11 = M60 ^ L2;               \
        T L12 = M48 ^ M51, L13 = M50 ^ L0, L14 = M52 ^ M61, L15 = M55 ^ L1, L16 = M56 ^ L0, L17 = M57 ^ L1;           \
        T L18 = M58 ^ L8, L19 = M63 ^ L4, L20 = L0 ^ L1, L21 = L1 ^ L7, L22 = L3 ^ L12, L23 = L18 ^ L2;               \
        T L24 = L15 ^ L9, L25 = L6 ^ L10, L26 = L7 ^ L9, L27 = L8 ^ L10, L28 = L11 ^ L14, L29 = L11 ^ L17;            \
        S0 = L6 ^ L24;                                                                                                  \
        S1 = ~(L16 ^ L26);                                                                                              \
        S2 = ~(L19 ^ L28);                                                                                              \
        S3 = L6 ^ L21;                                                                                                  \
        S4 = L20 ^ L22;                                                                                                 \
        S5 = L25 ^ L29;                                                                                                 \
        S6 = ~(L13 ^ L27);                                                                                              \
        S7 = ~(L6 ^ L23);                                                                                               \
    } while (0)

// state word 8 p + b = bit b (LSB 0) of byte p of the 32 blocks of this lane (bit k of the word = block k).
// SubBytes in place (the circuit reads every input before it writes an output); ShiftRows is folded into the reads of
// MixColumns (and of the final AddRoundKey), so the loop-carried state stays in natural byte order.
__device__ __forceinline__ void bs_sub(uint32_t (&s)[128]) {
    static_for<16>([&](auto pc) {
        constexpr int p = decltype(pc)::value;
        uint32_t *u = s + 8 * p;
        BP_SBOX(uint32_t, u[7], u[6], u[5], u[4], u[3], u[2], u[1], u[0], u[7], u[6], u[5], u[4], u[3], u[2], u[1], u[0]);
        __builtin_amdgcn_sched_barrier(0);  // one S-box at a time (interleaving all 16 spilled)
    });
}
// byte index, before ShiftRows, of byte (row r, column c) after it
__device__ __host__ constexpr int sr(int c, int r) { return 4 * ((c + r) & 3) + r; }
// round-key masks (0 or ~0 per state bit) of round r: 128 words at LDS offset 512 r, read as uniform broadcasts
__device__ __forceinline__ void bs_mix_ark(uint32_t (&s)[128], uint32_t r) {
    uint32_t t[128];
#pragma unroll
    for (int c = 0; c < 4; c++) {
#pragma unroll
        for (int rr = 0; rr < 4; rr++) {
            const uint32_t *a0 = s + 8 * sr(c, rr), *a1 = s + 8 * sr(c, (rr + 1) & 3);
            const uint32_t *a2 = s + 8 * sr(c, (rr + 2) & 3), *a3 = s + 8 * sr(c, (rr + 3) & 3);
            uint32_t x[8];
#pragma unroll
            for (int b = 0; b < 8; b++) x[b] = a0[b] ^ a1[b];
            const uint32_t xt[8] = {x[7], x[0] ^ x[7], x[1], x[2] ^ x[7], x[3] ^ x[7], x[4], x[5], x[6]};
            const uint4 k0 = lds_ld128(512u * r + 32u * (4 * c + rr)), k1 = lds_ld128(512u * r + 32u * (4 * c + rr) + 16);
            const uint32_t k[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
            uint32_t *o = t + 8 * (4 * c + rr);
#pragma unroll
            for (int b = 0; b < 8; b++) o[b] = xor3(xt[b], a1[b], a2[b]) ^ a3[b] ^ k[b];
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int i = 0; i < 128; i++) s[i] = t[i];
}

__global__ __launch_bounds__(256) void bitslice_k(const uint32_t *__restrict__ rk_g, int P, uint32_t *out,
                                                  uint32_t *chk, Clock *clk) {
    for (uint32_t i = threadIdx.x; i < 11 * 128; i += blockDim.x) {
        const uint32_t r = i >> 7, w = i & 127u, p = w >> 3, b = w & 7u;
        lds_st32(4u * i, 0u - ((rk_g[4 * r + (p >> 2)] >> (8 * (p & 3) + b)) & 1u));
    }
    __syncthreads();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    clk_start(clk);
    for (int p = 0; p < P; p++) {
        // 32 counter blocks: bytes 0..11 nonce, bytes 12..15 be32(32 p + k), k = block = bit k of every word
        const uint32_t nw[3] = {tid * 0x9e3779b9u, (uint32_t)p * 0x85ebca6bu + tid, 0x01234567u ^ tid};
        const uint32_t cbase = 32u * (uint32_t)p;
        uint32_t s[128];
#pragma unroll
        for (int q = 0; q < 16; q++) {
#pragma unroll
            for (int b = 0; b < 8; b++) {
                uint32_t w;
                if (q < 12) {
                    w = 0u - ((nw[q >> 2] >> (8 * (q & 3) + b)) & 1u);
                } else {
                    const int sh = 8 * (15 - q) + b;  // bit of the big-endian counter
                    const uint32_t pat[5] = {0xaaaaaaaau, 0xccccccccu, 0xf0f0f0f0u, 0xff00ff00u, 0xffff0000u};
                    w = sh < 5 ? pat[sh] : 0u - ((cbase >> sh) & 1u);
                }
                s[8 * q + b] = w ^ lds_ld32(4u * (8 * q + b));
            }
        }
#pragma unroll 1
        for (uint32_t r = 1; r < 10; r++) {
            bs_sub(s);
            bs_mix_ark(s, r);
        }
        bs_sub(s);
        uint32_t f[128];
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
            for (int rr = 0; rr < 4; rr++)
#pragma unroll
                for (int b = 0; b < 8; b++) f[8 * (4 * c + rr) + b] = s[8 * sr(c, rr) + b] ^ lds_ld32(4u * (1280 + 8 * (4 * c + rr) + b));
        if (chk && tid == 0 && p == 0)
            for (int i = 0; i < 128; i++) chk[i] = f[i];
#pragma unroll
        for (int i = 0; i < 128; i++) acc ^= f[i] + (uint32_t)i;
    }
    clk_end(clk);
    out[tid] = acc;
}

// ---------------------------------------------------------------- host
static void aes_ecb(const uint8_t key[16], const uint8_t *in, uint8_t *outb, int n) {
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    int l = 0;
    EVP_EncryptInit_ex(c, EVP_aes_128_ecb(), nullptr, key, nullptr);
    EVP_CIPHER_CTX_set_padding(c, 0);
    EVP_EncryptUpdate(c, outb, &l, in, 16 * n);
    EVP_CIPHER_CTX_free(c);
}
static void expand(const uint8_t key[16], uint32_t rk[44]) {
    static const uint8_t rcon[10] = {1, 2, 4, 8, 16, 32, 64, 128, 27, 54};
    uint8_t w[176];
    memcpy(w, key, 16);
    for (int i = 16, r = 0; i < 176; i += 4) {
        uint8_t t[4] = {w[i - 4], w[i - 3], w[i - 2], w[i - 1]};
        if (i % 16 == 0) {
            uint8_t u = t[0];
            t[0] = kSBox.v[t[1]] ^ rcon[r++];
            t[1] = kSBox.v[t[2]];
            t[2] = kSBox.v[t[3]];
            t[3] = kSBox.v[u];
        }
        for (int j = 0; j < 4; j++) w[i + j] = w[i - 16 + j] ^ t[j];
    }
    for (int i = 0; i < 44; i++) rk[i] = w[4 * i] | (w[4 * i + 1] << 8) | (w[4 * i + 2] << 16) | ((uint32_t)w[4 * i + 3] << 24);
}
static void put_be32(uint8_t *p, uint32_t v) {
    p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = v;
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "all";
    const bool all = !strcmp(mode, "all");
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    uint8_t key[16];
    for (int i = 0; i < 16; i++) key[i] = (uint8_t)(0x2b + 17 * i);
    uint32_t rk[44];
    expand(key, rk);
    uint32_t *d_rk, *d_u32;
    uint4 *d_out, *d_chk;
    Clock *d_clk;
    DevKey *d_key;
    CK(hipMalloc(&d_rk, sizeof(rk)));
    CK(hipMemcpy(d_rk, rk, sizeof(rk), hipMemcpyHostToDevice));
    CK(hipMalloc(&d_out, (size_t)cus * 1024 * 16));
    CK(hipMalloc(&d_u32, (size_t)cus * 1024 * 4 * 8));
    CK(hipMalloc(&d_chk, 128 * 4));
    CK(hipMalloc(&d_clk, sizeof(Clock)));
    // a DevKey with some V[m] (GHASH timing does not depend on the values)
    std::vector<DevKey> hk(1);
    memset(hk.data(), 0, sizeof(DevKey));
    for (int m = 0; m < 128; m++)
        for (int w = 0; w < 4; w++) hk[0].V[m][w] = 0x9e3779b9u * (uint32_t)(4 * m + w + 1);
    CK(hipMalloc(&d_key, sizeof(DevKey)));
    CK(hipMemcpy(d_key, hk.data(), sizeof(DevKey), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto clock_of = [&](double *cyc, double *ghz) {
        Clock c;
        CK(hipMemcpy(&c, d_clk, sizeof c, hipMemcpyDeviceToHost));
        *cyc = (double)(c.t1 - c.t0);
        *ghz = (double)(c.t1 - c.t0) / ((double)(c.r1 - c.r0) * 10.0);  // s_memrealtime: 100 MHz
    };
    auto timed = [&](auto launch) {
        float best = 1e30f;
        for (int rep = 0; rep < 4; rep++) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipGetLastError());
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep && ms < best) best = ms;
        }
        return best;
    };

    if (all || !strcmp(mode, "issue")) {
        const char *names[] = {"v_xor_b32", "v_bitop3_b32", "v_perm_b32", "v_add_u32", "v_fma_f32", "v_alignbit_b32",
                               "(a&b)^c"};
        for (int bpc : {2, 8}) {  // 256-thread blocks per CU: 2 or 8 waves per SIMD
            for (int op = 0; op < 7; op++) {
                const int iters = 16384, blocks = cus * bpc;
                float ms = timed([&] {
                    switch (op) {
                        case 0: hipLaunchKernelGGL(issue_k<0>, dim3(blocks), dim3(256), 0, 0, d_u32, iters, 3u, d_clk); break;
                        case 1: hipLaunchKernelGGL(issue_k<1>, dim3(blocks), dim3(256), 0, 0, d_u32, iters, 3u, d_clk); break;
                        case 2: hipLaunchKernelGGL(issue_k<2>, dim3(blocks), dim3(256), 0, 0, d_u32, iters, 3u, d_clk); break;
                        case 3: hipLaunchKernelGGL(issue_k<3>, dim3(blocks), dim3(256), 0, 0, d_u32, iters, 3u, d_clk); break;
                        case 4: hipLaunchKernelGGL(issue_k<4>, dim3(blocks), dim3(256), 0, 0, d_u32, iters, 3u, d_clk); break;
                        case 5: hipLaunchKernelGGL(issue_k<5>, dim3(blocks), dim3(256), 0, 0, d_u32, iters, 3u, d_clk); break;
                        default: hipLaunchKernelGGL(issue_k<6>, dim3(blocks), dim3(256), 0, 0, d_u32, iters, 3u, d_clk); break;
                    }
                });
                double cyc, ghz;
                clock_of(&cyc, &ghz);
                // per SIMD: bpc waves, each iters x 8 instructions (+ loop overhead)
                const double per_instr = cyc / ((double)iters * 8 * bpc);
                const double wi_per_ns = (double)blocks * 4 * iters * 8 / (ms * 1e6);
                printf("issue waves/SIMD %d %-16s %.3f ms  %.2f cycles/wave-instr/SIMD (s_memtime, %.2f GHz)  %.1f wave-instr/ns\n",
                       bpc, names[op], ms, per_instr, ghz, wi_per_ns);
            }
        }
    }

    auto check_ttab = [&](const char *name) {
        uint4 ks[4];
        CK(hipMemcpy(ks, d_chk, sizeof ks, hipMemcpyDeviceToHost));
        const uint32_t tid = 0;
        uint32_t nw[3] = {tid * 0x9e3779b9u, 0u * 0x85ebca6bu + tid, 0x01234567u ^ tid};
        uint8_t in[64], want[64];
        for (int j = 0; j < 4; j++) {
            memcpy(in + 16 * j, nw, 12);
            put_be32(in + 16 * j + 12, 1 + j);
        }
        aes_ecb(key, in, want, 4);
        const bool ok = !memcmp(ks, want, 64);
        printf("%s check vs OpenSSL: %s\n", name, ok ? "ok" : "MISMATCH");
        return ok;
    };
    const int P = 16, G = 19;  // 16 x 76 blocks per lane
    const double blocks_tt = (double)cus * 512 * P * G * 4;
    auto report = [&](const char *name, float ms, double blocks, int waves_per_cu) {
        double cyc, ghz;
        clock_of(&cyc, &ghz);
        const double wave_blocks_per_cu = blocks / 64 / cus;
        printf("%-10s %.3f ms  %.1f G blocks/s  %.1f cycles per wave-block per CU (wg0: %.0f cycles, %.2f GHz, %d waves/CU)\n",
               name, ms, blocks / (ms * 1e6), cyc / wave_blocks_per_cu, cyc, ghz, waves_per_cu);
    };
    WgRec *d_cen = nullptr;
    if (!strcmp(mode, "census")) {
        CK(hipMalloc(&d_cen, sizeof(WgRec) * 4096));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_census), &d_cen, sizeof(d_cen)));
    }
    auto census_report = [&](const char *name, int nwg) {
        if (!d_cen) return;
        std::vector<WgRec> w(nwg);
        CK(hipMemcpy(w.data(), d_cen, sizeof(WgRec) * nwg, hipMemcpyDeviceToHost));
        uint64_t t0 = ~0ull, t1 = 0;
        for (auto &x : w) { t0 = x.r0 < t0 ? x.r0 : t0; t1 = x.r1 > t1 ? x.r1 : t1; }
        std::vector<int> cnt(1 << 16, 0);
        int distinct = 0, maxc = 0, late = 0;
        double dur_min = 1e30, dur_max = 0;
        for (auto &x : w) {
            const uint32_t cu = ((x.xcc & 15u) << 12) | ((x.hwid >> 8) & 0xfffu);  // xcc | se | sh | cu
            if (!cnt[cu]++) distinct++;
            maxc = cnt[cu] > maxc ? cnt[cu] : maxc;
            const double d = (double)(x.r1 - x.r0) / 100.0;  // us
            dur_min = d < dur_min ? d : dur_min;
            dur_max = d > dur_max ? d : dur_max;
            if ((x.r0 - t0) / 100.0 > 0.25 * (t1 - t0) / 100.0) late++;
        }
        printf("census %-10s %d WGs on %d distinct CUs (max %d per CU), span %.1f us, WG duration %.1f-%.1f us, %d started late (>25%% of span)\n",
               name, nwg, distinct, maxc, (t1 - t0) / 100.0, dur_min, dur_max, late);
    };
    auto run_tt = [&](const char *name, auto kern, int wg) {
        const double blocks = (double)cus * wg * P * G * 4;
        float ms = timed([&] {
            hipLaunchKernelGGL(kern, dim3(cus), dim3(wg), kLdsMax, 0, d_rk, d_key, P, G, d_out, d_chk, d_clk);
        });
        report(name, ms, blocks, wg / 64);
        check_ttab(name);
        census_report(name, cus);
    };
    if (!strcmp(mode, "census")) {
        run_tt("ttab2/512", ttab_k<false, false, 512>, 512);
        run_tt("ttab2/1024", ttab_k<false, false, 1024>, 1024);
        printf("device: %d CUs, %s\n", cus, prop.gcnArchName);
    }
    if (all || !strcmp(mode, "ttab2")) {
        run_tt("ttab2/512", ttab_k<false, false, 512>, 512);
        run_tt("ttab2/1024", ttab_k<false, false, 1024>, 1024);
    }
    if (all || !strcmp(mode, "ttab4")) {
        run_tt("ttab4/512", ttab_k<true, false, 512>, 512);
        run_tt("ttab4/1024", ttab_k<true, false, 1024>, 1024);
    }
    if (all || !strcmp(mode, "aesgh")) {
        run_tt("aesgh/512", ttab_k<false, true, 512>, 512);
        run_tt("aesgh/1024", ttab_k<false, true, 1024>, 1024);
    }
    if (all || !strcmp(mode, "ghash8")) {
        const int B = P * G * 4;
        float ms = timed([&] { hipLaunchKernelGGL(ghash_k, dim3(cus), dim3(512), kLdsMax, 0, d_key, B, d_out, d_clk); });
        report("ghash8", ms, (double)cus * 512 * B, 8);
    }
    if (all || !strcmp(mode, "bitslice")) {
        const int PB = 4;  // 4 x 32 blocks per lane
        for (int bpc : {1, 2}) {  // 256-thread blocks per CU (VGPR-limited anyway)
            const int blocks = cus * bpc * 4;  // oversubscribe: the hardware keeps what fits
            float ms = timed([&] {
                hipLaunchKernelGGL(bitslice_k, dim3(blocks), dim3(256), 6144, 0, d_rk, PB, (uint32_t *)d_out,
                                   (uint32_t *)d_chk, d_clk);
            });
            report("bitslice", ms, (double)blocks * 256 * PB * 32, 0);
        }
        uint32_t w[128];
        CK(hipMemcpy(w, d_chk, sizeof w, hipMemcpyDeviceToHost));
        const uint32_t nw[3] = {0u, 0u, 0x01234567u};
        uint8_t in[512], want[512];
        for (int k = 0; k < 32; k++) {
            memcpy(in + 16 * k, nw, 12);
            put_be32(in + 16 * k + 12, (uint32_t)k);
        }
        aes_ecb(key, in, want, 32);
        int bad = 0;
        for (int k = 0; k < 32; k++)
            for (int q = 0; q < 16; q++) {
                uint8_t v = 0;
                for (int b = 0; b < 8; b++) v |= ((w[8 * q + b] >> k) & 1u) << b;
                bad += v != want[16 * k + q];
            }
        printf("bitslice check vs OpenSSL: %s (%d bad bytes)\n", bad ? "MISMATCH" : "ok", bad);
    }
    return 0;
}
