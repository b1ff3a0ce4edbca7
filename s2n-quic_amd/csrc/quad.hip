// quad.hip — AES-128/256-GCM seal/open + AES header protection, "quad" layout: FOUR lanes per packet (gfx950).
//
// Replaces the aws-lc-rs calls behind quic/s2n-quic-crypto:
//   seal  <LessSafeKey as Aead>::encrypt -> seal_in_place_scatter   src/aead/default.rs:44-62
//   open  <LessSafeKey as Aead>::decrypt -> open_in_place           src/aead/default.rs:65-93
//   HP    HeaderKey::header_protection_mask -> new_mask             src/header_key.rs:52-56
// with the nonce of Iv::nonce (src/iv.rs:27-39).
//
// Why four lanes per packet (tools/ubench/aes_core.hip): the AES + GHASH core runs more blocks per second
// the more waves a SIMD holds, and the round-2 lane-per-packet kernel (deleted in round 3) was held at 2 by its per-wave
// payload staging (32 KiB of LDS next to 128 KiB of tables) and its ~220 VGPRs.  Here the 4 lanes of a quad move a
// packet's bytes themselves -- lane s takes counter slots t = 4 k + s, so each wave instruction loads 64 contiguous
// bytes of each of 16 packets and one 4-block group of a lane covers 256 contiguous bytes of its packet -- with no
// staging at all; a workgroup is 768 threads (12 waves, 3 per SIMD, <= 168 VGPRs: QPP_QUAD_WG).
//
// GHASH over four lanes: the sequence X_1..X_n (AAD blocks, ciphertext blocks, length block) is dealt to the lanes
// by virtual slot (AAD block i at t = i + 1 - a, ciphertext block j at t = j + 1, length block at t = m + 1; lane
// t mod 4), every lane runs a Horner chain with H^4 (8-bit tables), and at the end lane s multiplies its chain by
// H^e_s, e_s = (m + 2) - (its last slot) in 1..4 (4-bit tables, one per power, chosen per lane), and the quad
// XOR-reduces: Y = xor_s A_s H^e_s = xor_i X_i H^(n + 1 - i).  Tag = Y ^ E_K(J0) (slot 0 = J0 lives in lane 0).
//
// LDS (160 KiB, one workgroup per CU):
//   [0, 64K)     8-bit GHASH tables of H^4 (GhashT layout)
//   [64K, 128K)  AES tables (AesQ4: T0..T3, 8 copies each, in the lower 128 B of 256 rows; AesLds: T0/T1 x 32)
//   [128K, 160K) 4-bit GHASH tables of H^1..H^4 (Ghash4 layout, power e at 128K + 8K (e - 1))
// While a key's tables are built, [64K, 72K) holds V_e[m] = H^e x^m (e = 1..4), before the AES tables overwrite it.
#include <stdlib.h>

#include "device_common.h"
#include "ghash.h"

namespace qpp {
namespace {
using namespace dev;

constexpr uint32_t kQLdsPow = 131072;  // 4-bit tables of H^1..H^4
constexpr uint32_t kQLdsVe = 65536;    // V_e during the build
#ifndef QPP_QUAD_WG
#define QPP_QUAD_WG 768  // AES-128: 3 waves per SIMD (<= 168 VGPRs); 1024 (4 waves, <= 128) spills, 9 % slower (r03w4)
#endif
#ifndef QPP_QUAD_WG256
#define QPP_QUAD_WG256 768  // AES-256 (60 round-key words, 14 rounds of pipeline state)
#endif
// AES on four quarter-split T-tables (AesQ4, device_common.h; the two-table AesLds + rotl16 form measured 2 % slower
// in the quad kernel, round 4, profiles/r04a)
using QAes = AesQ4;
using QPage = CtrPageQ4;
__device__ __forceinline__ QAes make_qaes() { return AesQ4::make(); }
__device__ __forceinline__ void build_qaes() { build_aes_tables_q4(kLdsAes); }
template <int NR, int NB, int STRIDE>
__device__ __forceinline__ void qkeystream(const QAes &a, const QPage &pg, RkPtr rkp, uint32_t c0,
                                           uint4 (&ks)[NB]) {
    // rounds 3..NR only: 32 / 48 words at the group's start (the page build reads rounds 0..2 itself, when it runs)
    uint32_t rk[4 * (NR + 1)];
#pragma unroll
    for (int r = 3; r <= NR; r++) {
        const uint4 v = rkp[r];
        rk[4 * r] = v.x; rk[4 * r + 1] = v.y; rk[4 * r + 2] = v.z; rk[4 * r + 3] = v.w;
    }
    ctr_keystream_q4<NR, NB, STRIDE>(a, pg, rk, c0, ks);
}
__device__ __forceinline__ uint4 ld_payload(const uint8_t *p) { return ld16(p); }
#ifndef QPP_QUAD_NT
#define QPP_QUAD_NT 1  // payload stores streaming (nt); 0: plain stores (write-traffic A/B)
#endif
__device__ __forceinline__ void st_payload(uint8_t *p, uint4 v) {
    if (QPP_QUAD_NT) st16_nt(p, v);  // streaming: the sealed / opened bytes are not read again
    else st16(p, v);
}
template <int NR>  // (NR = 0: a launch over both sizes)
constexpr int kQuadWG = NR == 14 ? QPP_QUAD_WG256 : QPP_QUAD_WG;
// Counter blocks per lane in one group (a group = 4 QNB slots of the packet per quad).  4: 16 slots = 256 bytes of a
// packet per group; fewer blocks per group hold fewer registers (the 1024-thread build, 4 waves per SIMD).
#ifndef QPP_QUAD_NB
#define QPP_QUAD_NB 4
#endif
#ifndef QPP_QUAD_TRACE
// A wave's priority is raised (s_setprio) from its group's payload loads to the group's end (the XOR, the stores and
// the GHASH steps) and dropped for the next group's keystream: the arbiter then favours the wave that holds a group's
// memory round trip over the waves in their keystream, so loads and stores go out earlier and the LDS array is fed from
// both.  Round 6, same box, alternating rounds: seal 1.1630 -> 1.1450 ms (4 rounds), then 1.1387 -> 1.1123 ms
// (3 rounds; levels 1 and 3: 1.1210 / 1.1232), 300 B 1.5652 -> 1.5458 ms, receive neutral (profiles/r06/prio).
// QPP_QUAD_PRIO 0 turns it off; QPP_QUAD_PRIO_DROP 1 drops it right after the stores instead (same time).
#ifndef QPP_QUAD_PRIO
#define QPP_QUAD_PRIO 2
#endif
#ifndef QPP_QUAD_PRIO_DROP
#define QPP_QUAD_PRIO_DROP 0
#endif
#define QPP_QUAD_TRACE 0  // 1: workgroups 0 and grid/2 print their table-build and total cycles (s_memtime); 2: all
#endif
#ifndef QPP_QUAD_EK0C
#define QPP_QUAD_EK0C 1  // E_K(J0) kept as one column per lane from group 0's keystream (0: seal keeps the block in every
                         // lane, open recomputes it on the quad at the end)
#endif
#ifndef QPP_QUAD_TAGEARLY
#define QPP_QUAD_TAGEARLY 1  // open: the received tag loaded before the last group (0: after the final product)
#endif
#ifndef QPP_QUAD_ABL
#define QPP_QUAD_ABL 0  // ablation bits for timing A/Bs only (wrong bytes): 1 no interior payload loads, 2 no interior
                        // stores, 4 no header protection, 8 no final H^e product (the quad sums the chains as they are); DESIGN §5
                        // round 6 has what each cost
#endif
constexpr int kQNB = QPP_QUAD_NB, kQSG = 4 * kQNB;
static_assert(kQNB >= 2 && kQNB <= 4, "group size");


// X * H through the 8-bit tables of H at [0, 64K) (T_j[x] at 256 x + 16 j): the setup's products
__device__ __forceinline__ uint4 mul_h8(uint4 x) {
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 16; j++) acc = acc ^ lds_ld128(256u * ((w[j >> 2] >> (8 * (j & 3))) & 0xffu) + 16u * j);
    return acc;
}
// 8-bit tables T_j[x] = (x at byte j) * P at [0, 64K) from V_P[m] = P x^m at LDS offset v
__device__ __forceinline__ void build8(uint32_t v) {
    for (uint32_t e = threadIdx.x; e < 4096; e += blockDim.x) {
        const uint32_t j = e & 15, x = e >> 4;
        uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; i++)
            if ((x >> (7 - i)) & 1) acc = acc ^ lds_ld128(v + 16 * (8 * j + i));
        lds_st128(256 * x + 16 * j, acc);
    }
}

// The tables of one key segment from the key's pow slot (slot < pow.cap; burst.hip pow_setup_kernel fills it at install):
// the 4-bit tables of H^2, H^4 (T_1, T_2) and H^3 are copied (burst layout, entry (pos = 2 b + h, n) at 256 pos + 16 n,
// transposed to this kernel's 4096 h + 256 n + 16 b), H's are built from V[m], and the 8-bit tables of H^4 are two
// lookups each in H^4's 4-bit tables (T_j[x] = high nibble (x >> 4) at byte j ^ low nibble (x & 15) at byte j, times
// H^4).  The AES tables are not touched.  Round 6: the derivation in LDS below (V_e by three
// dependent products, two 8-bit builds with up to 8 reads per entry, the AES tables rebuilt over its scratch) took a
// tenth of a 4096-key batch's seal (QPP_QUAD_TRACE: 35 k of 349 k s_memtime ticks per segment).  Ends with a barrier.
__device__ void quad_tables_pow(const DevKey *__restrict__ key, const uint4 *__restrict__ src) {
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    for (uint32_t idx = tid; idx < 4 * 512; idx += nthr) {
        const uint32_t t = idx >> 9, ent = idx & 511u, pos = ent >> 4, n = ent & 15u, b = pos >> 1, h = pos & 1u;
        uint4 v;
        uint32_t e;  // power
        if (t == 0) {  // H: xor of V[8 b + 4 h + i] over the set bits (bit 3 - i) of n
            e = 1;
            const uint4 *V = (const uint4 *)key->V;
            v = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint4 x = V[8 * b + 4 * h + i];
                const uint32_t m = 0u - ((n >> (3 - i)) & 1u);
                v = v ^ make_uint4(x.x & m, x.y & m, x.z & m, x.w & m);
            }
        } else {  // t = 1: T_1 = H^2, 2: T_2 = H^4, 3: H^3
            e = t == 1 ? 2u : t == 2 ? 4u : 3u;
            v = src[(t == 3 ? kPowH3 / 16 : (t - 1) * 512u) + ent];
        }
        lds_st128(kQLdsPow + 8192 * (e - 1) + 4096 * h + 256 * n + 16 * b, v);
    }
    __syncthreads();
    constexpr uint32_t h4 = kQLdsPow + 3 * 8192;
    for (uint32_t ent = tid; ent < 4096; ent += nthr) {
        const uint32_t j = ent & 15u, x = ent >> 4;
        lds_st128(256 * x + 16 * j, lds_ld128(h4 + 256 * (x >> 4) + 16 * j) ^ lds_ld128(h4 + 4096 + 256 * (x & 15u) + 16 * j));
    }
    __syncthreads();
}

// All tables of one key (every thread takes part; ends with a barrier).  The caller synced before (the previous
// key's tables are no longer read).  (Keys without a pow slot: the derivation in LDS, AES tables rebuilt after it.)
__device__ void quad_tables(const DevKey *__restrict__ key) {
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    for (uint32_t i = tid; i < 128; i += nthr) {
        const uint32_t *v = key->V[i];
        lds_st128(kQLdsVe + 16 * i, make_uint4(v[0], v[1], v[2], v[3]));
    }
    __syncthreads();
    build8(kQLdsVe);  // tables of H
    __syncthreads();
    for (uint32_t e = 1; e < 4; e++) {  // V_{e+1}[m] = H * V_e[m]
        if (tid < 128) lds_st128(kQLdsVe + 2048 * e + 16 * tid, mul_h8(lds_ld128(kQLdsVe + 2048 * (e - 1) + 16 * tid)));
        __syncthreads();
    }
    // 4-bit tables of H^e: entry (half h, byte b, nibble n) at 128K + 8K (e - 1) + 4K h + 256 n + 16 b =
    // xor of V_e[8 b + 4 h + i] over the set bits (bit 3 - i) of n
    for (uint32_t idx = tid; idx < 4 * 2 * 16 * 16; idx += nthr) {
        const uint32_t e = idx >> 9, h = (idx >> 8) & 1u, b = (idx >> 4) & 15u, n = idx & 15u;
        uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; i++)
            if ((n >> (3 - i)) & 1u) acc = acc ^ lds_ld128(kQLdsVe + 2048 * e + 16 * (8 * b + 4 * h + i));
        lds_st128(kQLdsPow + 8192 * e + 4096 * h + 256 * n + 16 * b, acc);
    }
    __syncthreads();  // the tables of H are dead
    build8(kQLdsVe + 3 * 2048);  // tables of H^4 (the Horner step)
    __syncthreads();  // V_e are dead
    build_qaes();
    __syncthreads();
}

// quad_perm DPP (row-local, 4-lane groups): lane l reads lane 4 (l / 4) + sel[l % 4]
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint4 qperm(uint4 v) {
    return make_uint4(qperm<CTRL>(v.x), qperm<CTRL>(v.y), qperm<CTRL>(v.z), qperm<CTRL>(v.w));
}
constexpr int kQuadSwap1 = 0xb1;   // [1, 0, 3, 2]
constexpr int kQuadSwap2 = 0x4e;   // [2, 3, 0, 1]
constexpr int kQuadBcast0 = 0x00;  // [0, 0, 0, 0]
constexpr int kQuadBcast1 = 0x55;  // [1, 1, 1, 1]
constexpr int kQuadBcast2 = 0xaa;  // [2, 2, 2, 2]

// AES of one block over the 4 lanes of a quad, column s of the state in lane s: per round each lane takes bytes 1, 2, 3
// of its right-hand neighbours' columns through DPP (3 moves) and does its column's 4 lookups, so a once-per-packet
// block (the header-protection mask; E_K(J0) when opening) costs the wave a quarter of what one lane doing the whole
// block costs.  rk_g: a key schedule in the key record (lane s reads word s of each round).  Returns column s of E(in).
constexpr int kQuadRot1 = 0x39;  // [1, 2, 3, 0]
constexpr int kQuadRot3 = 0x93;  // [3, 0, 1, 2]
// QPP_QUAD_HPS: rk_g is uniform (the segment's key record): each round's four words by one scalar load where the
// round uses them, the lane's column selected in VGPRs -- instead of NR + 1 vector loads per packet, which queue
// behind the packet's payload loads and stores (0: the vector loads)
#ifndef QPP_QUAD_HPS
#define QPP_QUAD_HPS 1
#endif
template <int NR>
__device__ __forceinline__ uint32_t aes_quad(const QAes &a, const uint32_t *__restrict__ rk_g, uint32_t col, uint32_t s) {
    uint32_t rk[NR + 1];
    RkPtr hp{};
    if (QPP_QUAD_HPS) {
        uint64_t p = (uint64_t)rk_g;
        asm volatile("" : "+s"(p));  // (uniform; not hoisted)
        hp = (RkPtr)p;
    } else {
#pragma unroll
        for (int r = 0; r <= NR; r++) rk[r] = rk_g[4 * r + s];
    }
    auto rkey = [&](int r) {
        if (!QPP_QUAD_HPS) return rk[r];
        const uint4 v = hp[r];
        return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
    };
    uint32_t x = a.rot(col ^ rkey(0));  // (the lane's convention: AesQ4 rotates every word by 8 q)
#pragma unroll
    for (int r = 1; r <= NR; r++) {
        const uint32_t b = qperm<kQuadRot1>(x), c = qperm<kQuadSwap2>(x), d = qperm<kQuadRot3>(x);
        if (r < NR) {
            x = a.col(x, b, c, d, a.rot(rkey(r)));
        } else {
            x = a.last(x, b, c, d, rkey(r));
        }
    }
    return x;
}

// The descriptor again at the packet's tail (through a laundered pointer, so that the compiler reloads it instead of
// keeping its fields in VGPRs across the group loop: the loop needs only the payload offset, length and nonce)
// (the base is uniform and the index a lane's own packet: no 64-bit pointer is kept live across the loop)
__device__ __forceinline__ qpp_pkt reload_desc(const qpp_pkt *descs, uint32_t i) {
    uint32_t v = i;
    asm volatile("" : "+v"(v));
    return descs[v];
}

// One packet per quad; s = lane % 4.  has = false: the quad has no packet (its lanes only keep the wave's loop shape).
// Addresses are 32-bit offsets into the arena (SGPR base + VGPR offset).
template <int NR, bool SEAL, bool HEAD>
__device__ __forceinline__ void quad_packet(const QAes &aes, const GhashT<true> &gh, const DevKey *__restrict__ key,
                                            bool has, const qpp_pkt &d,
                                            const qpp_pkt *__restrict__ descs, uint32_t pkt_index,
                                            uint8_t *__restrict__ arena, uint8_t *masks, int8_t *status,
                                            uint32_t flags, uint32_t s) {
    // loop state
    const uint32_t aad_len = d.aad_len, len = has ? d.pt_len : 0u, pay = d.off + aad_len;
    const uint32_t pn_len = SEAL ? (uint32_t)d.pn_len : 0u;  // (seal: header protection)
    // Iv::nonce (iv.rs:27-39); the key's iv by scalar loads (a uniform pointer through the constant address space:
    // as a vector load it waited behind every memory operation of the previous packet, once per packet)
    // (not in the AES-256 seal: there the scalar iv and the AAD load moved behind the page build below measured 2.6 %
    // slower, 6 alternating rounds; everywhere else 0.6-2.5 % faster, round 6)
    constexpr bool kLatePro = !SEAL || NR == 10;
    uint32_t iv0, iv1, iv2;
    if constexpr (kLatePro) {
        uint64_t iva = (uint64_t)key->iv;
        asm volatile("" : "+s"(iva));
        const __attribute__((address_space(4))) uint32_t *ivp = (const __attribute__((address_space(4))) uint32_t *)iva;
        iv0 = ivp[0]; iv1 = ivp[1]; iv2 = ivp[2];
    } else {
        iv0 = key->iv[0]; iv1 = key->iv[1]; iv2 = key->iv[2];
    }
    const uint32_t n0 = iv0, n1 = iv1 ^ bswap32((uint32_t)(d.pn >> 32)), n2 = iv2 ^ bswap32((uint32_t)d.pn);
    const int nfull = (int)(len >> 4), rem = (int)(len & 15), m = nfull + (rem ? 1 : 0);
    const int a = has ? (int)((aad_len + 15) >> 4) : 0;
    auto at = [&](uint32_t off) { return arena + off; };

    // Round keys: scalar loads where they are used (the key record stays in the scalar cache), through a pointer
    // laundered per group so that no load is hoisted out of the group loop (held for the whole loop, 44 / 60 words
    // exhausted the SGPRs and went to VGPRs); a group's keystream loads rounds 3..NR, the page build rounds 0..2
    auto round_keys = [&]() {
        uint64_t a = (uint64_t)key->rk;
        asm volatile("" : "+s"(a));  // reloaded here, not hoisted into SGPRs for the whole loop
        // Through the constant address space: a uniform load from a global pointer is a scalar load only when the
        // compiler can prove no store of the kernel clobbers it, which the laundering hides -- the round keys were
        // FLAT loads into 32-44 VGPRs (uniform values in vector registers, the register budget of the waves)
        return (RkPtr)a;
    };
    QPage pg;
    // AAD blocks of this lane: virtual slots t = 1 - a .. 0, t = s (mod 4).  A lane's first AAD block starts its chain
    // (w = rot(x): no product of zero); a lane with no AAD block starts at w = 0 and its first data step multiplies zero
    // (one product more for those lanes, in exchange for no started-flag control flow in the group loop).  With the
    // usual 1..2 AAD blocks no lane has a second one and the product loop is skipped by the whole wave.
    // (a zero made here, per packet: a zero uint4 kept from the kernel's start was spilled in the receive kernel)
    uint32_t z0;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z0));
    uint4 w = make_uint4(z0, z0, z0, z0);
    {
        auto aad_block = [&](int t) {
            const uint32_t i = (uint32_t)(t + a - 1);
            uint4 x = ld16(at(d.off + 16 * i));
            const uint32_t r = aad_len - 16 * i;
            return r < 16 ? keep_bytes(x, r) : x;
        };
        int t = (1 - a) + (((int)s - (1 - a)) & 3);
        // the lane's first AAD block is loaded here and taken into the chain after the page build below, whose LDS
        // work covers the load's round trip
        // (loaded by every lane, a lane without an AAD block reading the packet's first bytes: a conditional load
        // joins into a copy that waits for it; masked below, after the page build: a use here waits)
        const bool has_aad = t <= 0;
        const uint32_t i0 = (uint32_t)(t + a - 1), r0 = aad_len - 16 * i0;
        if constexpr (!kLatePro) {
            if (has_aad) {
                w = gh.rot(aad_block(t));
                t += 4;
            }
        }
        const uint4 x0 = kLatePro ? ld16(at(d.off + (has_aad ? 16 * i0 : 0u))) : make_uint4(z0, z0, z0, z0);
        pg.build(aes, round_keys(), n0, n1, n2, 0);
        if (kLatePro && has_aad) {
            w = gh.rot(r0 < 16 ? keep_bytes(x0, r0) : x0);
            t += 4;
        }
        for (; t <= 0; t += 4) w = gh.mulx(w, aad_block(t));
    }

    const int ngroups = has ? (m + kQSG) / kQSG : 0;  // counter slots 0 (J0) .. m
    const int G = (int)wave_max((uint32_t)ngroups);
    const int min_full = (int)__builtin_amdgcn_readfirstlane(wave_min(has ? (uint32_t)nfull : 0u));
    auto interior = [&](int g) { return g >= 1 && kQSG * g + kQSG - 1 <= min_full; };  // every slot a whole payload block
    // group 0 when slots 1..15 are whole payload blocks in every packet of the wave: the interior path, with slot 0
    // (J0: keystream only, neither stored nor hashed) masked per lane
    // (HEAD: the AES-128-only kernels; in the AES-256 and both-sizes instances the extra path cost 10-14 VGPRs of
    // spills and 3 % of AES-256's seal time.  The AES-128 open spills 4 VGPRs with it -- one reload per packet, none in
    // the group loop -- and still runs 0.6 % faster than without it, 6 alternating rounds: round 6)
    const bool head_ok = HEAD && kQSG - 1 <= min_full;  // uniform
    // counter blocks per lane the last group needs (uniform): the longest packet's slots past 16 (G - 1)
    const int tail_slots = (int)wave_max(has ? (uint32_t)max(0, m + 1 - kQSG * (G - 1)) : 0u);
    // length block: be64(aad bits) || be64(payload bits)
    auto lenblk = [&]() { return make_uint4(0, bswap32(aad_len * 8), 0, bswap32(len * 8)); };
    bool len_done = !has;

    constexpr int HNR = NR == 10 ? 10 : 14;
    const bool want_hp = SEAL && (flags & (QPP_HP_MASK_OUT | QPP_HP_APPLY)) != 0;
    uint4 ek0 = make_uint4(0, 0, 0, 0);  // seal: E_K(J0) (slot 0: lane 0, group 0)
    uint32_t ek0c = 0;                    // (QPP_QUAD_EK0C) column s of E_K(J0) in lane s

    bool hp_done = false;                // seal: header protection applied after group 0 (quad-uniform)
    // Header protection as soon as the sample exists: the sample (ciphertext bytes [4 - pn_len, 20 - pn_len),
    // payload.rs:151-169) lies in ciphertext blocks 0 and 1 -- slots 1 and 2, group 0, lanes 1 and 2 -- when the payload
    // has at least 20 - pn_len bytes.  The header bytes are then written while the packet's first 64-byte segment still
    // holds group 0's ciphertext in L2 (one memory write for both, not two), and nothing is read back.
    // The header bytes the mask applies to (the first byte and the PN's 4-byte window) are loaded with group 0's payload
    // (one memory round trip for both), the descriptor fields are the packet's own (no reload)
    const bool hp_at0 = want_hp && has && pn_len >= 1 && pn_len <= 4 && len + pn_len >= 20;  // quad-uniform
    HdrBytes hb{0u, 0u};
    auto hp_early = [&](const uint4 &ct) {
        if (!hp_at0) return;
        const uint4 b0 = qperm<kQuadBcast1>(ct), b1 = qperm<kQuadBcast2>(ct);  // ciphertext blocks 0 and 1
        const uint32_t lo = s == 0 ? b0.x : s == 1 ? b0.y : s == 2 ? b0.z : b0.w;
        const uint32_t hi = s == 0 ? b0.y : s == 1 ? b0.z : s == 2 ? b0.w : b1.x;
        const uint32_t col = __builtin_amdgcn_alignbyte(hi, lo, 4 - pn_len);  // sample column s
        const uint32_t m0 = aes_quad<HNR>(aes, key->hp_rk, col, s);
        const uint32_t m1 = qperm<kQuadBcast1>(m0);  // column 1 (mask byte 4 is its byte 0)
        if (s == 0) {
            if (flags & QPP_HP_MASK_OUT) {
                uint8_t *mo = masks + 5 * (size_t)pkt_index;
                mo[0] = (uint8_t)m0; mo[1] = (uint8_t)(m0 >> 8); mo[2] = (uint8_t)(m0 >> 16);
                mo[3] = (uint8_t)(m0 >> 24); mo[4] = (uint8_t)m1;
            }
            const uint32_t hdr_len = aad_len - pn_len;
            if (flags & QPP_HP_APPLY) hdr_apply(at(pay - aad_len), hdr_len, pn_len, hb, m0, m1);
        }
        hp_done = true;
    };

    // one group: slots t = kQSG g + 4 k + s, k < NBG; slot t holds counter t + 1 and ciphertext block t - 1
    auto group = [&](auto nbc, int g) __attribute__((always_inline)) {
        constexpr int NBG = decltype(nbc)::value;
        const bool head = NBG == kQNB && g == 0 && head_ok;  // uniform
        const bool inner = NBG == kQNB && interior(g);  // uniform
        const RkPtr rkp = round_keys();
        const int t0 = kQSG * g + (int)s;
        uint4 ks[NBG];
        uint4 in[NBG];
        const uint32_t c0 = (uint32_t)t0 + 1u;
        // The nonce words are laundered where the loop uses them (a new page; the straddling group): left alone, the
        // compiler hoisted the page build's first-round lookups addresses out of the loop as loop invariants and
        // spilled them (16 scratch accesses per group in the open kernel).
        uint32_t m0 = n0, m1 = n1, m2 = n2;
        if (((kQSG * g + 1) >> 8) == ((kQSG * g + kQSG) >> 8)) {  // uniform: no lane's counters straddle a 256-block page
            if ((c0 >> 8) != pg.page) {
                asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2));
                pg.build(aes, rkp, m0, m1, m2, c0 >> 8);
            }
            qkeystream<NR, NBG, 4>(aes, pg, rkp, c0, ks);
        } else {
            asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2));
            uint32_t rk[4 * (NR + 1)];
#pragma unroll
            for (int r = 0; r <= NR; r++) {
                const uint4 v = rkp[r];
                rk[4 * r] = v.x; rk[4 * r + 1] = v.y; rk[4 * r + 2] = v.z; rk[4 * r + 3] = v.w;
            }
            static_for<NBG>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                ks[k] = aes.encrypt<NR>(make_uint4(m0, m1, m2, bswap32(c0 + 4 * k)), rk);
            });
        }
        // payload after the keystream (loading the next interior group's payload while this group hashes measured 8 %
        // slower: 1.248 vs 1.152 ms seal, 8 VGPRs spilled, profiles/r04h_ab; loading this group's before the keystream
        // 4 % slower at 3 waves/SIMD (14 VGPRs spilled) and 7.5 % slower at 2 waves/SIMD (256 VGPRs, no spill); an L2
        // touch of the next group's lines 3.7 % slower: round 6, profiles/r06/head)
        if (QPP_QUAD_PRIO) __builtin_amdgcn_s_setprio(QPP_QUAD_PRIO);
        if (SEAL && g == 0 && hp_at0 && (flags & QPP_HP_APPLY) && s == 0) hb = hdr_load(at(pay - aad_len), aad_len - pn_len);
        if (head) {
            // slot 0 (lane 0, k = 0) reads the payload's first block instead of the bytes before it (never used)
            const uint32_t b = pay + 16 * (uint32_t)(t0 - 1);
#pragma unroll
            for (int k = 0; k < NBG; k++) in[k] = ld_payload(at(k == 0 && s == 0 ? pay : b + 64 * k));
        } else if (inner) {
            const uint32_t b = pay + 16 * (uint32_t)(t0 - 1);
#pragma unroll
            for (int k = 0; k < NBG; k++) {
                if (QPP_QUAD_ABL & 1) in[k] = make_uint4(b + k, b ^ k, b, k);
                else in[k] = ld_payload(at(b + 64 * k));
            }
        } else {
#pragma unroll
            for (int k = 0; k < NBG; k++) {
                const int j = t0 + 4 * k - 1;
                in[k] = ld_payload(at(pay + (j >= 0 && 16 * j <= (int)len ? 16 * (uint32_t)j : 0u)));
            }
        }
        uint4 out[NBG];
#pragma unroll
        for (int k = 0; k < NBG; k++) out[k] = in[k] ^ ks[k];
        if constexpr (SEAL) {
            // (QPP_QUAD_EK0C=0: E_K(J0), slot 0 of lane 0, kept whole in every lane until the tag is known)
            if (g == 0 && !QPP_QUAD_EK0C) ek0 = ks[0];
        }
        if (QPP_QUAD_EK0C && g == 0) {
            // slot 0 of group 0 is counter block 1 = J0 in lane 0: its column s to lane s (quad broadcasts of lane 0)
            const uint32_t c0w = qperm<kQuadBcast0>(ks[0].x), c1w = qperm<kQuadBcast0>(ks[0].y),
                           c2w = qperm<kQuadBcast0>(ks[0].z), c3w = qperm<kQuadBcast0>(ks[0].w);
            ek0c = s == 0 ? c0w : s == 1 ? c1w : s == 2 ? c2w : c3w;
        }
        if (head) {
            const uint32_t b = pay + 16 * (uint32_t)(t0 - 1);
#pragma unroll
            for (int k = 0; k < NBG; k++)
                if (k != 0 || s != 0) st_payload(at(b + 64 * k), out[k]);
#pragma unroll
            for (int k = 0; k < NBG; k++) {
                const uint4 wn = gh.mulx(w, SEAL ? out[k] : in[k]);
                if (k != 0) {
                    w = wn;
                } else {  // slot 0 is not hashed (per component: a select of the whole vector went through scratch)
                    w.x = s != 0 ? wn.x : w.x;
                    w.y = s != 0 ? wn.y : w.y;
                    w.z = s != 0 ? wn.z : w.z;
                    w.w = s != 0 ? wn.w : w.w;
                }
            }
        } else if (inner) {
            const uint32_t b = pay + 16 * (uint32_t)(t0 - 1);
            // (Every chunk in its own group.  Deferring the last 64 bytes of an interior group to the next group's
            // first store, and holding the packet's first 64 ciphertext bytes and its header bytes to its end next to
            // the tag, were both measured to write MORE, not less, and to run slower: round 5, profiles/r05/r05i --
            // seal WRITE_SIZE 1.473 / 1.491 vs 1.457 MB per launch, seal 1.161 / 1.173 vs 1.152 ms.)
#pragma unroll
            for (int k = 0; k < NBG; k++)
                if (!(QPP_QUAD_ABL & 2)) st_payload(at(b + 64 * k), out[k]);
            if (QPP_QUAD_PRIO && QPP_QUAD_PRIO_DROP == 1) __builtin_amdgcn_s_setprio(0);
#pragma unroll
            for (int k = 0; k < NBG; k++) w = gh.mulx(w, SEAL ? out[k] : in[k]);
        } else {
            // (rem laundered here: left alone, the compiler hoisted keep_bytes' four masks out of the group loop and
            // held them -- and spilled others -- for the whole packet)
            uint32_t rl = (uint32_t)rem;
            asm volatile("" : "+v"(rl));
#pragma unroll
            for (int k = 0; k < NBG; k++) {
                const int t = t0 + 4 * k, j = t - 1;
                const bool full = t >= 1 && j < nfull, part = rem && j == nfull, lenslot = has && t == m + 1;
                if (full) st_payload(at(pay + 16 * (uint32_t)j), out[k]);
                if (part) st_bytes(at(pay + 16 * (uint32_t)j), keep_bytes(out[k], rl), rl);
                // the length block rides in the slot after the payload when the group reaches it
                const uint4 x = lenslot ? lenblk() : part ? keep_bytes(SEAL ? out[k] : in[k], rl)
                                                        : (SEAL ? out[k] : in[k]);
                if (full || part || lenslot) w = gh.mulx(w, x);
                len_done = len_done || lenslot;
            }
        }
        if (SEAL && g == 0 && !(QPP_QUAD_ABL & 4)) hp_early(out[0]);
        if (QPP_QUAD_PRIO) __builtin_amdgcn_s_setprio(0);
    };
    for (int g = 0; g + 1 < G; g++) group(std::integral_constant<int, kQNB>{}, g);
    // open: the received tag's column s, loaded before the last group so that its round trip passes under that
    // group's work (it was loaded after the final product, its latency exposed once per packet)
    uint32_t want = 0;
    if (!SEAL && QPP_QUAD_TAGEARLY) __builtin_memcpy(&want, at(pay + len + 4 * s), 4);
    if (G > 0) {  // the last group with as few counter blocks per lane as its longest packet needs
        // (small packets: a 300-B packet's second group needs 1 block per lane, not 3)
        if (tail_slots <= 4) group(std::integral_constant<int, 1>{}, G - 1);
        else if (kQNB == 2 || tail_slots <= 8) group(std::integral_constant<int, 2>{}, G - 1);
        else if (kQNB == 3 || tail_slots <= 12) group(std::integral_constant<int, kQNB < 3 ? kQNB : 3>{}, G - 1);
        else group(std::integral_constant<int, kQNB>{}, G - 1);
    }
    if (!len_done && (((m + 1) & 3) == (int)s)) w = gh.mulx(w, lenblk());
    // this lane's chain times H^e, e = (m + 2) - its last slot; then the quad's sum
    const int t_last = (m + 1) - (((m + 1) - (int)s) & 3);
    const uint32_t e = (uint32_t)(m + 2 - t_last);  // 1..4 (a lane with no block has w = 0 and any e)
    Ghash4T<kQLdsPow> fin;
    for (int k = 0; k < 4; k++) {  // the same lane rotation as the Horner chain
        fin.g.lc[k] = gh.lc[k];
        fin.g.sel[k] = gh.sel[k];
    }
    fin.g.q1 = gh.q1;
    fin.g.q2 = gh.q2;
    fin.hi_or = 0x01010101u * ((2u * (e - 1u)) << 4);
    fin.lo_or = 0x01010101u * ((2u * (e - 1u) + 1u) << 4);
    uint4 y = (QPP_QUAD_ABL & 8) ? w : fin.prod(w);
    y = y ^ qperm<kQuadSwap1>(y);
    y = y ^ qperm<kQuadSwap2>(y);

    if constexpr (SEAL) {
        if (QPP_QUAD_EK0C) {  // tag = GHASH ^ E_K(J0), column s by lane s
            const uint32_t t = (s == 0 ? y.x : s == 1 ? y.y : s == 2 ? y.z : y.w) ^ ek0c;
            if (has) __builtin_memcpy(at(pay + len + 4 * s), &t, 4);
        } else if (has && s == 0) {
            st16(at(pay + len), y ^ ek0);
        }
        const bool hp = !(QPP_QUAD_ABL & 4) && want_hp && has && pn_len >= 1 && pn_len <= 4 && len >= 4 - pn_len;
        if (hp && !hp_done) {  // short payloads: the sample runs into the tag
            // header-protection sample = ciphertext||tag bytes [4 - pn_len, 20 - pn_len) (payload.rs:151-169), column s
            // read back (the quad's lanes stored the blocks and lane 0 the tag: a wavefront fence orders them first;
            // read back rather than kept in registers across the loop); the mask AES on the quad (aes_quad)
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            uint32_t col;
            __builtin_memcpy(&col, at(pay + 4 - pn_len + 4 * s), 4);
            const uint32_t m0 = aes_quad<HNR>(aes, key->hp_rk, col, s);
            const uint32_t m1 = qperm<kQuadBcast1>(m0);  // column 1 (mask byte 4 is its byte 0)
            if (s == 0) {
                if (flags & QPP_HP_MASK_OUT) {
                    uint8_t *mo = masks + 5 * (size_t)pkt_index;
                    mo[0] = (uint8_t)m0; mo[1] = (uint8_t)(m0 >> 8); mo[2] = (uint8_t)(m0 >> 16);
                    mo[3] = (uint8_t)(m0 >> 24); mo[4] = (uint8_t)m1;
                }
                const uint32_t hdr_len = aad_len - pn_len;
                if (flags & QPP_HP_APPLY) hdr_apply(at(pay - aad_len), hdr_len, pn_len, hdr_load(at(pay - aad_len), hdr_len), m0, m1);
            }
        }
        if (!has || s != 0) return;
        if (status) status[pkt_index] = want_hp && !hp ? QPP_DECODE_ERROR : QPP_OK;
    } else {
        // E_K(J0) column s in lane s (from group 0's keystream; QPP_QUAD_EK0C=0: recomputed on the quad here, J0 = nonce ||
        // be32(1)), compared column by column with the received tag, the verdict OR-ed over the quad: all 16 bytes
        // compared, no early exit
        uint32_t ek0 = ek0c;
        if (!QPP_QUAD_EK0C) {
            const qpp_pkt dt = reload_desc(descs, pkt_index);
            const uint32_t j0 = s == 0 ? key->iv[0]
                              : s == 1 ? key->iv[1] ^ bswap32((uint32_t)(dt.pn >> 32))
                              : s == 2 ? key->iv[2] ^ bswap32((uint32_t)dt.pn)
                                       : bswap32(1u);
            uint32_t sl = s;
            asm volatile("" : "+v"(sl));  // (left alone, the compiler kept &key->rk[s] in a VGPR pair across the packet
                                          // loop of each key segment and spilled it: 4 VGPRs of scratch per open)
            ek0 = aes_quad<NR>(aes, key->rk, j0, sl);
        }
        if (!QPP_QUAD_TAGEARLY) __builtin_memcpy(&want, at(pay + len + 4 * s), 4);
        const uint32_t ys = s == 0 ? y.x : s == 1 ? y.y : s == 2 ? y.z : y.w;
        uint32_t diff = ys ^ ek0 ^ want;
        diff |= qperm<kQuadSwap1>(diff);
        diff |= qperm<kQuadSwap2>(diff);
        if (!has || s != 0) return;
        const bool ok = diff == 0;
        if (!ok) {
            // never release unauthenticated plaintext (the quad's other lanes stored it: order these stores after theirs)
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            for (int b = 0; b < nfull; b++) st16(at(pay + 16 * b), make_uint4(0, 0, 0, 0));
            if (rem) st_bytes(at(pay + 16 * nfull), make_uint4(0, 0, 0, 0), (uint32_t)rem);
        }
        status[pkt_index] = ok ? QPP_OK : QPP_DECRYPT_ERROR;
    }
}

// One workgroup per CU (grid = CUs) over an equal slice of the key-sorted packets (plan meta,
// same single-key mode), 256 packets per pass.
template <bool SEAL, int NR, int WG = kQuadWG<NR>, bool HEAD = false>
__device__ __forceinline__ void quad_slices(const DevKey *__restrict__ keys, const qpp_pkt *__restrict__ descs,
                                            const uint32_t *__restrict__ perm, const WorkItem *__restrict__ work,
                                            const uint32_t *__restrict__ meta, uint8_t *__restrict__ arena,
                                            uint8_t *masks, int8_t *status, uint32_t flags, uint32_t single,
                                            uint32_t n_single, const PowTables pow, uint32_t fix_lo = 0,
                                            uint32_t fix_hi = 0) {
    // fix_hi != 0 (with a single key): this workgroup alone takes descs [fix_lo, fix_hi) (the fused receive's local
    // slices), not its share of the grid's split
    const bool one = single != 0xffffffffu;  // uniform
    uint32_t i_lo = 0, i_hi = 1, p0 = 0, n = n_single;
    if (!one) {
        const uint32_t items = meta[0], i10 = meta[1], n10 = meta[2], n14 = meta[3];
        i_lo = NR == 10 ? 0 : i10;
        i_hi = NR == 10 ? i10 : items;
        p0 = NR == 10 ? 0 : n10;
        n = NR == 10 ? n10 : n14;
    }
    const uint32_t P = ((n + gridDim.x - 1) / gridDim.x + 15u) & ~15u;  // whole waves (16 packets) per slice
    uint32_t lo = fix_hi ? fix_lo : p0 + min(n, blockIdx.x * P);
    const uint32_t hi = fix_hi ? fix_hi : p0 + min(n, (blockIdx.x + 1) * P);
    if (lo >= hi) return;  // uniform
    uint32_t i = i_lo, j = i_hi;  // the item holding lo: largest i with work[i].begin <= lo
    while (!one && j - i > 1) {
        const uint32_t mid = (i + j) >> 1;
        if (work[mid].begin <= lo) i = mid; else j = mid;
    }
    const QAes aes = make_qaes();
    const GhashT<true> gh = GhashT<true>::make();
    const uint32_t s = threadIdx.x & 3u, q = threadIdx.x >> 2;
    build_qaes();  // once: the segments' table builds from a pow slot leave them alone (the first barrier below orders it)
#if QPP_QUAD_TRACE
    uint64_t t_beg = __builtin_amdgcn_s_memtime(), t_tab = 0, r_beg = __builtin_amdgcn_s_memrealtime();
    uint32_t n_seg = 0;
#endif
    for (; lo < hi; i++) {  // key segments of the slice
        WorkItem w = one ? WorkItem{single, 0u, n, (uint32_t)NR} : work[i];
        // (uniform; the fused receive kernel's work items are written by the same launch, so not scalar-loaded)
        w.key = __builtin_amdgcn_readfirstlane(w.key);
        w.begin = __builtin_amdgcn_readfirstlane(w.begin);
        w.count = __builtin_amdgcn_readfirstlane(w.count);
        const uint32_t end = min(hi, w.begin + w.count);
        const DevKey *__restrict__ key = keys + w.key;
        __syncthreads();  // every wave is done with the previous segment's tables
#if QPP_QUAD_TRACE
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
        if (w.key < pow.cap) quad_tables_pow(key, (const uint4 *)(pow.base + (size_t)w.key * kPowBytes));
        else quad_tables(key);
#if QPP_QUAD_TRACE
        t_tab += __builtin_amdgcn_s_memtime() - t0;
        n_seg++;
#endif
        for (uint32_t t0 = lo; t0 < end; t0 += WG / 4) {
            const uint32_t t = t0 + q;
            const bool real = t < end;
            const uint32_t pi = one ? (real ? t : lo) : perm[real ? t : lo];
            const qpp_pkt d = descs[pi];  // (any valid descriptor for quads without a packet)
            bool has = real && !(d.flags & QPP_PKT_SKIP);
            if (one && has && d.key_idx != single) {  // not the live key: refused, untouched
                if (status && s == 0) status[pi] = QPP_INTERNAL_ERROR;
                has = false;
            }
            quad_packet<NR, SEAL, HEAD>(aes, gh, key, has, d, descs, pi, arena, masks, status, flags, s);
        }
        lo = end;
    }
#if QPP_QUAD_TRACE
    __syncthreads();
    if (threadIdx.x == 0 && (QPP_QUAD_TRACE == 2 || blockIdx.x == 0 || blockIdx.x == gridDim.x / 2))
        printf("quad wg %u seal %d nr %d: %u segments, tables %llu of %llu cycles, real %llu-%llu\n", blockIdx.x,
               (int)SEAL, NR, n_seg, (unsigned long long)t_tab, (unsigned long long)(__builtin_amdgcn_s_memtime() - t_beg),
               (unsigned long long)r_beg, (unsigned long long)__builtin_amdgcn_s_memrealtime());
#endif
}

// NR = 10 / 14: one AES size; NR = 0: a planned batch holding both sizes in ONE launch -- each workgroup opens its
// slice of the AES-128 packets, then its slice of the AES-256 packets (round count per key segment, tables per key),
// as the fused receive's open phase does, instead of two serial full-chip launches
template <bool SEAL, int NR>
__global__ __launch_bounds__(kQuadWG<NR>) void aes_gcm_quad_kernel(const DevKey *__restrict__ keys,
                                                              const qpp_pkt *__restrict__ descs,
                                                              const uint32_t *__restrict__ perm,
                                                              const WorkItem *__restrict__ work,
                                                              const uint32_t *__restrict__ meta,
                                                              uint8_t *__restrict__ arena, uint8_t *masks,
                                                              int8_t *status, uint32_t flags, uint32_t single,
                                                              uint32_t n_single, const PowTables pow) {
    constexpr int WG = kQuadWG<NR>;
    if constexpr (NR != 14) quad_slices<SEAL, 10, WG, NR == 10>(keys, descs, perm, work, meta, arena, masks, status, flags, single, n_single, pow);
    if constexpr (NR != 10) quad_slices<SEAL, 14, WG>(keys, descs, perm, work, meta, arena, masks, status, flags, single, n_single, pow);
}

// ---------------------------------------------------------------- fused receive path, any key mix, ONE launch
// crypto::unprotect + crypto::decrypt for a GRO batch (quic/s2n-quic-core/src/crypto/packet_protection.rs; the key by
// the key-phase bit, crypto/application/keyset.rs:113-143; the suite per key, cipher_suite/negotiated.rs:15-125),
// whatever the connections' keys and suites, as one cooperative launch in four phases separated by grid barriers:
//   A. each workgroup unprotects its slice of rx[] (one lane per packet: rx_unprotect_one -- HP mask of any suite,
//      first byte and PN unmasked in place, PN expanded, key chosen), writes descs_out[], and counts its packets per
//      chosen key in LDS (the GHASH table area is free until phase D);
//   B. the last workgroup past A turns the global counts into each key's first perm index -- AES-128 keys first, then
//      AES-256, then ChaCha20 -- and one work item per AES key;
//   C. each workgroup reserves a block per key it saw (one atomic per key) and scatters its packets into perm[];
//   D. the quad open over the key-sorted AES-128 packets, then the AES-256 ones, exactly as aes_gcm_quad_kernel runs a
//      planned batch (both round counts in one launch: the segment's NR is a template instance, the tables per key).
// A local slice (all its packets bound for the open under one AES key) skips B-C: its workgroup opens it in place right
// after A, counted in no plan, then takes its share of D.  A batch of one key is all local slices: no workgroup waits
// for another (round 6: the barriers and phases B-C were 60-130 us of a 1.35 ms 1 Mi-packet receive).
// The ChaCha20-Poly1305 packets (perm[scratch[3], + scratch[2])) are opened by chacha_kernel in selection mode, launched
// right behind on the same stream (no host round trip).  It replaces unprotect_kernel + the three plan launches + the
// open launches (tests/test_gpu_rx_fused.py: bit-exact against that path and the oracle).  A barrier that does not
// complete within a second (a workgroup that never became resident) makes every workgroup leave: its packets bound for
// the open phase report INTERNAL_ERROR, payload untouched, and the context's timeout counter is raised.
#ifndef QPP_RX_TRACE
#define QPP_RX_TRACE 0  // 1: workgroups 0, grid/2 and the last print their phase times (s_memrealtime); 2: all
#endif
constexpr uint32_t kRxCtl = kQLdsPow;     // LDS: barrier verdict; [kRxCtl + 64, +320 B) phase B scan sums
constexpr uint32_t kRxCls = kRxCtl + 1024;  // LDS: phase B's class byte per key (<= kRxHistMax)
typedef __attribute__((address_space(3))) uint8_t lds_u8;
constexpr uint32_t kRxHistMax = 16384;    // LDS bins [0, 64 KiB): keys per workgroup in phases A-C
constexpr uint64_t kRxBarrierTicks = 100000000ull;  // 1 s of s_memrealtime (100 MHz)
constexpr int8_t kRxOpen = 0x7f;  // status of a packet bound for the open phase (never a final status)

// scratch (device, words): [0] workgroups past phase A, [1] failed, [2] ChaCha packets, [3] their first perm index,
// [4] phase B done, [5] workgroups past phase C | counts[key_cap] @16 | cursor[key_cap] | meta[4] | work[]  (the first
// 16 + 2 key_cap words are zeroed before each launch)
constexpr uint32_t kRxLocal = kRxCtl + 8;  // LDS: the slice's one key (0xffffffff: none) and its class, after phase A

// a workgroup's arrival at a counter (every thread calls; its global writes so far are released with it): the count
// before it, acquired (the last arrival at [0] sees every other workgroup's phase-A counts)
__device__ uint32_t rx_arrive(uint32_t *ctr) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const uint32_t old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        lds_st32(kRxCtl, old);
    }
    __syncthreads();
    return lds_ld32(kRxCtl);
}

// wait until *ctr >= target (every thread calls); false: a barrier of this launch timed out (1 s) -- leave
__device__ bool rx_wait(uint32_t *scratch, uint32_t *ctr, uint32_t target) {
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t ok = 1;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (__hip_atomic_load(&scratch[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                __builtin_amdgcn_s_memrealtime() - t0 > kRxBarrierTicks) {
                __hip_atomic_store(&scratch[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        lds_st32(kRxCtl, ok);
    }
    __syncthreads();
    return lds_ld32(kRxCtl) != 0;
}

// the open class of a live packet key: 0 AES-128, 1 AES-256, 2 ChaCha20-Poly1305 (3: not opened here)
__device__ __forceinline__ uint32_t rx_class(uint4 kw, bool chacha) {
    if (kw.w != 1) return 3u;
    if (kw.x == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256) return chacha ? 2u : 3u;
    return kw.y == 10 ? 0u : kw.y == 14 ? 1u : 3u;
}

// AES: 10 or 14 when the live AES packet keys are all of one size (that instance alone: no registers spent on the
// other), 0 for both sizes in one launch (the launch's workgroup size: kQuadWG<10>, or kQuadWG<14> for 14 alone)
template <int AES>
constexpr int kRxWG = AES == 14 ? kQuadWG<14> : kQuadWG<10>;
template <int AES>
__global__ __launch_bounds__(kRxWG<AES>) void aes_gcm_quad_rx_kernel(const DevKey *__restrict__ keys,
                                                                 uint32_t key_cap, const qpp_rx_pkt *__restrict__ rx,
                                                                 uint32_t n, uint8_t *arena, qpp_pkt *descs_out,
                                                                 int8_t *status, uint32_t *scratch, uint32_t *perm,
                                                                 uint32_t *timeouts, uint32_t chacha, const PowTables pow) {
    uint32_t *counts = scratch + 16, *cursor = counts + key_cap, *meta = cursor + key_cap;
    WorkItem *work = (WorkItem *)(meta + 4);  // 16-byte aligned: key_cap is even
#if QPP_RX_TRACE
    uint64_t ts[8] = {};
    ts[0] = __builtin_amdgcn_s_memrealtime();
#define RX_TS(i) ts[i] = __builtin_amdgcn_s_memrealtime()
#else
#define RX_TS(i) (void)0
#endif
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    const uint32_t bins = min(key_cap, kRxHistMax);  // (the launch requires key_cap <= kRxHistMax)
    build_qaes();
    for (uint32_t i = tid; i < bins; i += nt) lds_st32(4 * i, 0);
    if (tid == 0) lds_st32(kRxLocal, 0xffffffffu);
    __syncthreads();
    const QAes aes = make_qaes();
    RX_TS(1);
    // A: unprotect the slice, count per chosen key
    const uint32_t P = (n + gridDim.x - 1) / gridDim.x;
    const uint32_t lo = min(n, blockIdx.x * P), hi = min(n, lo + P);
    // A packet goes to the open phase when its chosen key is a live packet key (an AES one, or a ChaCha20 one when the
    // launch opens those too); the others get INTERNAL_ERROR (descs_out as unprotect_kernel writes it: the multi-launch
    // path's plan refuses them likewise) -- except a ChaCha20 packet of an AES-only batch, which the multi-launch path
    // leaves alone as well.  The verdict is kept in status (kRxOpen) for phase C, which must scatter exactly the packets
    // phase A counted (a record retired meanwhile must not change it); phase D (or the ChaCha launch) overwrites it.
    // (the next packet's rx descriptor is loaded while this one is unprotected: one round trip off each packet)
    qpp_rx_pkt r_next = lo + tid < hi ? rx[lo + tid] : qpp_rx_pkt{};
    for (uint32_t t = lo + tid; t < hi; t += nt) {
        const qpp_rx_pkt r = r_next;
        if (t + nt < hi) r_next = rx[t + nt];
        uint4 kw;  // the chosen key's suite, nr, hp_nr, live (loaded with the header key's record)
        const qpp_pkt d = rx_unprotect_one(aes, keys, key_cap, r, arena, status, t, &kw);
        if (!(d.flags & QPP_PKT_SKIP)) {
            const uint32_t cls = rx_class(kw, chacha != 0);
            if (cls < 3) {
                status[t] = kRxOpen;
                lds_add32(4 * d.key_idx, 1u);
            } else if (!(kw.w == 1 && kw.x == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256)) {
                status[t] = QPP_INTERNAL_ERROR;
            }
        }
        descs_out[t] = d;
    }
    // a barrier that timed out: this workgroup's packets that were to be opened report INTERNAL_ERROR, untouched (their
    // headers stay unprotected, as the multi-launch path leaves a packet its open refuses), and the context's timeout
    // counter says so (qpp_ctx_rx_timeouts)
    auto bail = [&]() {
        if (tid == 0) __hip_atomic_fetch_add(timeouts, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (uint32_t t = lo + tid; t < hi; t += nt)
            if (status[t] == kRxOpen) status[t] = QPP_INTERNAL_ERROR;
    };
    __syncthreads();
    // A local slice: every packet of the slice goes to the open phase under ONE AES key this instance opens (a GRO batch
    // of one connection, or of many connections' packets already grouped) -- the workgroup opens it itself, right
    // after phase A and in rx order, outside the global plan (no counts, no scatter, no wait for the other slices).
    // The other slices go through phases B-D as before; the local ones take their share of phase D afterwards.
    for (uint32_t k = tid; k < bins; k += nt) {
        const uint32_t c = lds_ld32(4 * k);
        if (c && c == hi - lo) {  // (one bin at most)
            const uint32_t cls = rx_class(*(const uint4 *)(keys + k), chacha != 0);
            if ((cls == 0 && AES != 14) || (cls == 1 && AES != 10)) {
                lds_st32(kRxLocal, k);
                lds_st32(kRxLocal + 4, cls);
            }
        }
    }
    __syncthreads();
    const uint32_t local = lds_ld32(kRxLocal), lcls = local != 0xffffffffu ? lds_ld32(kRxLocal + 4) : 2u;  // uniform
    if (local == 0xffffffffu) {
        for (uint32_t k = tid; k < bins; k += nt) {
            const uint32_t c = lds_ld32(4 * k);
            if (c) __hip_atomic_fetch_add(&counts[k], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    RX_TS(2);
    // B: the last workgroup past phase A -- each key's first perm index (cursor; AES-128 keys, then AES-256, then
    // ChaCha20) and one work item per AES key with packets (AES-128 items first: the planned-batch layout quad_slices
    // reads from meta); then it raises [4]
    const bool last = rx_arrive(&scratch[0]) == gridDim.x - 1;  // uniform
    RX_TS(3);
    if (last) {
        const uint32_t chunk = (key_cap + nt - 1) / nt, k0 = min(key_cap, tid * chunk), k1 = min(key_cap, k0 + chunk);
        auto cls_of = [&](uint32_t k) { return rx_class(*(const uint4 *)(keys + k), chacha != 0); };
        // per thread: packets of each class (0..2) and AES keys with packets of each AES class (3, 4)
        uint32_t v[5] = {0, 0, 0, 0, 0};
        for (uint32_t k = k0; k < k1; k++) {
            const uint32_t c = counts[k];
            if (!c) continue;
            // (< 3: phase A counted only packets of open classes; a record that changed since -- never while the
            // batch is in flight, by the key-retirement rules -- is opened as AES-128 with whatever it holds, so it
            // fails its tags instead of indexing past the three classes; the class is kept for the second loop)
            uint32_t cls = cls_of(k);
            if (cls >= 3) cls = 0;
            *(lds_u8 *)(size_t)(kRxCls + k) = (uint8_t)cls;
            v[cls] += c;
            if (cls < 2) v[3 + cls] += 1;
        }
        // exclusive scans of the five per-thread counts in thread order: inclusive scan inside each wave (shuffles),
        // the waves' totals through LDS (a thread-0 loop over 768 entries took ~40 us)
        const uint32_t lane = tid & 63u, wv = tid >> 6, nwv = (nt + 63u) >> 6;
        uint32_t is[5];
#pragma unroll
        for (int j = 0; j < 5; j++) is[j] = v[j];
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
#pragma unroll
            for (int j = 0; j < 5; j++) {
                const uint32_t p = (uint32_t)__shfl_up((int)is[j], o, 64);
                if (lane >= o) is[j] += p;
            }
        }
        if (lane == 63) {
#pragma unroll
            for (int j = 0; j < 5; j++) lds_st32(kRxCtl + 64 + 4 * (16 * j + wv), is[j]);
        }
        __syncthreads();
        uint32_t ex[5], tot[5];
#pragma unroll
        for (int j = 0; j < 5; j++) {
            ex[j] = is[j] - v[j];
            tot[j] = 0;
        }
        for (uint32_t w = 0; w < nwv; w++) {
#pragma unroll
            for (int j = 0; j < 5; j++) {
                const uint32_t ws = lds_ld32(kRxCtl + 64 + 4 * (16 * j + w));
                if (w < wv) ex[j] += ws;
                tot[j] += ws;
            }
        }
        uint32_t off[3] = {ex[0], tot[0] + ex[1], tot[0] + tot[1] + ex[2]};
        uint32_t item[2] = {ex[3], tot[3] + ex[4]};
        if (tid == 0) {
            meta[0] = tot[3] + tot[4];     // work items
            meta[1] = tot[3];              // AES-128 items
            meta[2] = tot[0];              // AES-128 packets
            meta[3] = tot[1];              // AES-256 packets
            scratch[2] = tot[2];           // ChaCha20 packets ...
            scratch[3] = tot[0] + tot[1];  // ... from this perm index on
        }
        for (uint32_t k = k0; k < k1; k++) {
            const uint32_t c = counts[k];
            if (!c) continue;
            const uint32_t cls = *(const lds_u8 *)(size_t)(kRxCls + k);  // (the first loop's verdict, same thread)
            cursor[k] = off[cls];
            if (cls < 2) work[item[cls]++] = WorkItem{k, off[cls], c, cls ? 14u : 10u};
            off[cls] += c;
        }
        rx_arrive(&scratch[4]);
    }
    if (local == 0xffffffffu) {
        if (!rx_wait(scratch, &scratch[4], 1)) return bail();
        RX_TS(4);
        // C: one block of perm per key this workgroup saw, then its packets into it
        for (uint32_t k = tid; k < bins; k += nt) {
            const uint32_t c = lds_ld32(4 * k);
            if (c) lds_st32(4 * k, __hip_atomic_fetch_add(&cursor[k], c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        }
        __syncthreads();
        for (uint32_t t = lo + tid; t < hi; t += nt)
            if (status[t] == kRxOpen) perm[lds_add32(4 * descs_out[t].key_idx, 1u)] = t;
        RX_TS(5);
    }
    rx_arrive(&scratch[5]);  // (a local slice scatters nothing)
    // D: pass 0 (local slices): the workgroup's own slice under its key; pass 1: the key-sorted global plan (tables per
    // key segment, as a planned batch), the AES-128 packets, then the AES-256 ones, once every slice is scattered
    constexpr int WG = kRxWG<AES>;
    if (local != 0xffffffffu) {  // (trace: "C" is the local open)
        RX_TS(4);
        if constexpr (AES != 14)
            if (lcls == 0) quad_slices<false, 10, WG>(keys, descs_out, perm, work, meta, arena, nullptr, status, 0u, local, hi, pow, lo, hi);
        if constexpr (AES != 10)
            if (lcls == 1) quad_slices<false, 14, WG>(keys, descs_out, perm, work, meta, arena, nullptr, status, 0u, local, hi, pow, lo, hi);
        RX_TS(5);
    }
    if (!rx_wait(scratch, &scratch[5], gridDim.x)) return bail();
    RX_TS(6);
    if constexpr (AES != 14) quad_slices<false, 10, WG>(keys, descs_out, perm, work, meta, arena, nullptr, status, 0u, ~0u, 0u, pow);
    if constexpr (AES != 10) quad_slices<false, 14, WG>(keys, descs_out, perm, work, meta, arena, nullptr, status, 0u, ~0u, 0u, pow);
#if QPP_RX_TRACE
    RX_TS(7);
    if (threadIdx.x == 0 && (QPP_RX_TRACE == 2 || blockIdx.x == 0 || blockIdx.x == gridDim.x - 1 || blockIdx.x == gridDim.x / 2))
        printf("rx wg %u: tables %.2f A %.2f bar1 %.2f B %.2f C %.2f bar3 %.2f D %.2f us start %llu end %llu last %d\n",
               blockIdx.x, (ts[1] - ts[0]) / 100.0, (ts[2] - ts[1]) / 100.0, (ts[3] - ts[2]) / 100.0,
               (ts[4] - ts[3]) / 100.0, (ts[5] - ts[4]) / 100.0, (ts[6] - ts[5]) / 100.0, (ts[7] - ts[6]) / 100.0,
               (unsigned long long)ts[0], (unsigned long long)ts[7], (int)last);
#endif
}

template <bool SEAL, int NR>
void launch_quad(dim3 grid, hipStream_t s, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb,
                 uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags, uint32_t single, uint32_t n_single,
                 const PowTables &pow) {
    hipLaunchKernelGGL((aes_gcm_quad_kernel<SEAL, NR>), grid, dim3(kQuadWG<NR>), kLdsMax, s, keys, descs, pb.perm, pb.work,
                       pb.n_work, arena, masks, status, flags, single, n_single, pow);
}
}  // namespace

uint32_t quad_rx_max_keys() { return kRxHistMax; }

hipError_t launch_aes_gcm_quad_rx(uint32_t aes, uint32_t grid, hipStream_t s, const DevKey *keys, uint32_t key_cap,
                                  const qpp_rx_pkt *rx, uint32_t n, uint8_t *arena, qpp_pkt *descs_out, int8_t *status,
                                  uint32_t *scratch, uint32_t *perm, uint32_t *timeouts, bool chacha,
                                  const PowTables &pow) {
    if (key_cap > kRxHistMax || (key_cap & 1u)) return hipErrorInvalidValue;
    uint32_t ch = chacha ? 1u : 0u;
    PowTables pw = pow;
    void *args[] = {&keys, &key_cap, &rx, &n, &arena, &descs_out, &status, &scratch, &perm, &timeouts, &ch, &pw};
    // cooperative: the grid barriers need every workgroup resident (one per CU: grid <= the CUs it may use)
    const void *f = aes == 10   ? reinterpret_cast<const void *>(&aes_gcm_quad_rx_kernel<10>)
                    : aes == 14 ? reinterpret_cast<const void *>(&aes_gcm_quad_rx_kernel<14>)
                                : reinterpret_cast<const void *>(&aes_gcm_quad_rx_kernel<0>);
    const dim3 block(aes == 14 ? kRxWG<14> : kRxWG<10>);
    // A plain launch: the grid is at most the CUs the context's resident servers leave and a workgroup takes a whole
    // CU's LDS, so on a device this context owns every workgroup is resident at once -- the guarantee the grid
    // barriers need (and hipLaunchCooperativeKernel gives no more than that against another context's kernels; the
    // barriers' timeout covers that case).  QPP_RX_COOP=1: the cooperative launch API instead (under rocprofv3 a
    // process that had made cooperative launches crashed in exit(), after the profiler's finalization: round 3 and
    // round 4, profiles/r04b).
    static const bool coop = [] {
        const char *e = getenv("QPP_RX_COOP");
        return e && e[0] == '1';
    }();
    if (coop) return hipLaunchCooperativeKernel(f, dim3(grid), block, args, kLdsMax, s);
    return hipLaunchKernel(f, dim3(grid), block, args, kLdsMax, s);
}

// The quad-layout kernels behind launch_aes_gcm / launch_aes_gcm_single (aes_gcm.hip chooses).  single = 0xffffffff:
// planned batch (pb), else the one live AES key's slot (descs[0, n_single) in order, other slots refused).
hipError_t launch_aes_gcm_quad(bool seal, uint32_t nr, dim3 grid, hipStream_t s, const DevKey *keys,
                               const qpp_pkt *descs, const PlanBuffers &pb, uint8_t *arena, uint8_t *masks,
                               int8_t *status, uint32_t flags, uint32_t single, uint32_t n_single,
                               const PowTables &pow) {
    if (nr == 10) {
        if (seal) launch_quad<true, 10>(grid, s, keys, descs, pb, arena, masks, status, flags, single, n_single, pow);
        else launch_quad<false, 10>(grid, s, keys, descs, pb, arena, masks, status, flags, single, n_single, pow);
    } else if (nr == 14) {
        if (seal) launch_quad<true, 14>(grid, s, keys, descs, pb, arena, masks, status, flags, single, n_single, pow);
        else launch_quad<false, 14>(grid, s, keys, descs, pb, arena, masks, status, flags, single, n_single, pow);
    } else {  // both sizes (a planned batch)
        if (seal) launch_quad<true, 0>(grid, s, keys, descs, pb, arena, masks, status, flags, single, n_single, pow);
        else launch_quad<false, 0>(grid, s, keys, descs, pb, arena, masks, status, flags, single, n_single, pow);
    }
    return hipGetLastError();
}

}  // namespace qpp
