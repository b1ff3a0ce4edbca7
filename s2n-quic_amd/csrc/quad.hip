// quad.hip — AES-128/256-GCM seal/open + AES header protection, "quad" layout: FOUR lanes per packet (gfx950).
//
// Replaces the aws-lc-rs calls behind quic/s2n-quic-crypto (as aes_gcm.hip's lane kernel does):
//   seal  <LessSafeKey as Aead>::encrypt -> seal_in_place_scatter   src/aead/default.rs:44-62
//   open  <LessSafeKey as Aead>::decrypt -> open_in_place           src/aead/default.rs:65-93
//   HP    HeaderKey::header_protection_mask -> new_mask             src/header_key.rs:52-56
// with the nonce of Iv::nonce (src/iv.rs:27-39).
//
// Why four lanes per packet (tools/ubench/aes_core.hip): the AES + GHASH core runs 16 % more blocks per
// second at 4 waves per SIMD than at 2, and the lane-per-packet kernel cannot get there: its per-wave payload staging
// (32 KiB of LDS next to 128 KiB of tables) and its ~220 VGPRs hold it at 2.  Here the 4 lanes of a quad move a
// packet's bytes themselves -- lane s takes counter slots t = 4 k + s, so each wave instruction loads 64 contiguous
// bytes of each of 16 packets and one 4-block group of a lane covers 256 contiguous bytes of its packet -- with no
// staging at all, and a workgroup is 1024 threads (16 waves, <= 128 VGPRs).
//
// GHASH over four lanes: the sequence X_1..X_n (AAD blocks, ciphertext blocks, length block) is dealt to the lanes
// by virtual slot (AAD block i at t = i + 1 - a, ciphertext block j at t = j + 1, length block at t = m + 1; lane
// t mod 4), every lane runs a Horner chain with H^4 (8-bit tables), and at the end lane s multiplies its chain by
// H^e_s, e_s = (m + 2) - (its last slot) in 1..4 (4-bit tables, one per power, chosen per lane), and the quad
// XOR-reduces: Y = xor_s A_s H^e_s = xor_i X_i H^(n + 1 - i).  Tag = Y ^ E_K(J0) (slot 0 = J0 lives in lane 0).
//
// LDS (160 KiB, one workgroup per CU):
//   [0, 64K)     8-bit GHASH tables of H^4 (GhashT layout)
//   [64K, 128K)  AES T0/T1 (AesLds)
//   [128K, 160K) 4-bit GHASH tables of H^1..H^4 (Ghash4 layout, power e at 128K + 8K (e - 1))
// While a key's tables are built, [64K, 72K) holds V_e[m] = H^e x^m (e = 1..4), before the AES tables overwrite it.
#include "device_common.h"
#include "ghash.h"

namespace qpp {
namespace {
using namespace dev;

constexpr uint32_t kQLdsPow = 131072;  // 4-bit tables of H^1..H^4
constexpr uint32_t kQLdsVe = 65536;    // V_e during the build
#ifndef QPP_QUAD_WG
#define QPP_QUAD_WG 768  // 3 waves per SIMD (<= 168 VGPRs: no spills); 1024 (4 waves, <= 128) spilled: 8 % slower (profiles/r03g_wg)
#endif
constexpr int kQuadWG = QPP_QUAD_WG;
constexpr uint32_t kQuadPkts = kQuadWG / 4;  // packets per workgroup pass

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

// All tables of one key (every thread takes part; ends with a barrier).  The caller synced before (the previous
// key's tables are no longer read).
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
    build_aes_tables(kLdsAes);
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
constexpr int kQuadBcast1 = 0x55;  // [1, 1, 1, 1]
constexpr int kQuadBcast2 = 0xaa;  // [2, 2, 2, 2]

// AES of one block over the 4 lanes of a quad, column s of the state in lane s: per round each lane takes bytes 1, 2, 3
// of its right-hand neighbours' columns through DPP (3 moves) and does its column's 4 lookups, so a once-per-packet
// block (the header-protection mask; E_K(J0) when opening) costs the wave a quarter of what one lane doing the whole
// block costs.  rk_g: a key schedule in the key record (lane s reads word s of each round).  Returns column s of E(in).
constexpr int kQuadRot1 = 0x39;  // [1, 2, 3, 0]
constexpr int kQuadRot3 = 0x93;  // [3, 0, 1, 2]
template <int NR>
__device__ __forceinline__ uint32_t aes_quad(const AesLds &a, const uint32_t *__restrict__ rk_g, uint32_t col, uint32_t s) {
    uint32_t rk[NR + 1];
#pragma unroll
    for (int r = 0; r <= NR; r++) rk[r] = rk_g[4 * r + s];
    uint32_t x = col ^ rk[0];
#pragma unroll
    for (int r = 1; r <= NR; r++) {
        const uint32_t b = qperm<kQuadRot1>(x), c = qperm<kQuadSwap2>(x), d = qperm<kQuadRot3>(x);
        if (r < NR) {
            x = a.col(x, b, c, d, rk[r]);
        } else {
            x = a.last(x, b, c, d, rk[r]);
        }
    }
    return x;
}

// The descriptor again at the packet's tail (through a laundered pointer, so that the compiler reloads it instead of
// keeping its fields in VGPRs across the group loop: the loop needs only the payload offset, length and nonce)
__device__ __forceinline__ qpp_pkt reload_desc(const qpp_pkt *p) {
    uint64_t a = (uint64_t)p;
    asm volatile("" : "+v"(a));
    return *(const qpp_pkt *)a;
}

// One packet per quad; s = lane % 4.  has = false: the quad has no packet (its lanes only keep the wave's loop shape).
// Addresses are 32-bit offsets into the arena (SGPR base + VGPR offset).
template <int NR, bool SEAL>
__device__ __forceinline__ void quad_packet(const AesLds &aes, const GhashT<true> &gh, const DevKey *__restrict__ key,
                                            bool has, const qpp_pkt &d,
                                            const qpp_pkt *__restrict__ dptr, uint32_t pkt_index,
                                            uint8_t *__restrict__ arena, uint8_t *masks, int8_t *status,
                                            uint32_t flags, uint32_t s) {
    // loop state
    const uint32_t aad_len = d.aad_len, len = has ? d.pt_len : 0u, pay = d.off + aad_len;
    const uint32_t n0 = key->iv[0], n1 = key->iv[1] ^ bswap32((uint32_t)(d.pn >> 32)),  // Iv::nonce (iv.rs:27-39)
                   n2 = key->iv[2] ^ bswap32((uint32_t)d.pn);
    const int nfull = (int)(len >> 4), rem = (int)(len & 15), m = nfull + (rem ? 1 : 0);
    const int a = has ? (int)((aad_len + 15) >> 4) : 0;
    auto at = [&](uint32_t off) { return arena + off; };

    // AAD blocks of this lane: virtual slots t = 1 - a .. 0, t = s (mod 4).  The chain starts at w = 0: its first step
    // multiplies zero (one product more per lane that has no AAD block, in exchange for no started-flag control flow)
    uint4 w = make_uint4(0, 0, 0, 0);
    for (int t = (1 - a) + (((int)s - (1 - a)) & 3); t <= 0; t += 4) {
        const uint32_t i = (uint32_t)(t + a - 1);
        uint4 x = ld16(at(d.off + 16 * i));
        const uint32_t r = aad_len - 16 * i;
        if (r < 16) x = keep_bytes(x, r);
        w = gh.mulx(w, x);
    }

    // Round keys: scalar loads where they are used (the key record stays in the scalar cache) instead of 44 / 60 SGPRs
    // held for the whole kernel, which pushed other uniform values into VGPR lanes (a v_readlane per use in the loop)
    auto round_keys = [&](uint32_t (&k)[4 * (NR + 1)]) {
        uint64_t a = (uint64_t)key->rk;
        asm volatile("" : "+s"(a));  // reloaded here, not hoisted into SGPRs for the whole loop
        const uint4 *p = (const uint4 *)a;
#pragma unroll
        for (int r = 0; r <= NR; r++) {
            const uint4 v = p[r];
            k[4 * r] = v.x; k[4 * r + 1] = v.y; k[4 * r + 2] = v.z; k[4 * r + 3] = v.w;
        }
    };
    CtrPage pg;
    {
        uint32_t rk[4 * (NR + 1)];
        round_keys(rk);
        pg.build(aes, rk, n0, n1, n2, 0);
    }
    const int ngroups = has ? (m + 1 + 15) >> 4 : 0;  // counter slots 0 (J0) .. m
    const int G = (int)wave_max((uint32_t)ngroups);
    const int min_full = (int)__builtin_amdgcn_readfirstlane(wave_min(has ? (uint32_t)nfull : 0u));
    auto interior = [&](int g) { return g >= 1 && 16 * g + 15 <= min_full; };  // every slot a whole payload block
    // counter blocks per lane the last group needs (uniform): the longest packet's slots past 16 (G - 1)
    const int tail_slots = (int)wave_max(has ? (uint32_t)max(0, m + 1 - 16 * (G - 1)) : 0u);
    // length block: be64(aad bits) || be64(payload bits)
    auto lenblk = [&]() { return make_uint4(0, bswap32(aad_len * 8), 0, bswap32(len * 8)); };
    bool len_done = !has;

    // one group: slots t = 16 g + 4 k + s, k < NBG; slot t holds counter t + 1 and ciphertext block t - 1
    auto group = [&](auto nbc, int g) {
        constexpr int NBG = decltype(nbc)::value;
        const bool inner = NBG == 4 && interior(g);  // uniform
        uint32_t rk[4 * (NR + 1)];
        round_keys(rk);
        const int t0 = 16 * g + (int)s;
        uint4 ks[NBG];
        const uint32_t c0 = (uint32_t)t0 + 1u;
        // The nonce words are laundered where the loop uses them (a new page; the straddling group): left alone, the
        // compiler hoisted the page build's first-round lookups addresses out of the loop as loop invariants and
        // spilled them (16 scratch accesses per group in the open kernel).
        uint32_t m0 = n0, m1 = n1, m2 = n2;
        if ((g & 15) != 15) {  // uniform: no lane's counters straddle a 256-block page
            if ((c0 >> 8) != pg.page) {
                asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2));
                pg.build(aes, rk, m0, m1, m2, c0 >> 8);
            }
            ctr_keystream_pipe<NR, NBG, 4>(aes, pg, rk, c0, ks);
        } else {
            asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2));
            static_for<NBG>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                ks[k] = aes.encrypt<NR>(make_uint4(m0, m1, m2, bswap32(c0 + 4 * k)), rk);
            });
        }
        // payload loads after the keystream: held across the AES pipeline they cost 16 VGPRs at its peak (spills at
        // 128); the other 3 waves of the SIMD cover their latency
        uint4 in[NBG];
        if (inner) {
            const uint32_t b = pay + 16 * (uint32_t)(t0 - 1);
#pragma unroll
            for (int k = 0; k < NBG; k++) in[k] = ld16(at(b + 64 * k));
        } else {
#pragma unroll
            for (int k = 0; k < NBG; k++) {
                const int j = t0 + 4 * k - 1;
                in[k] = ld16(at(pay + (j >= 0 && 16 * j <= (int)len ? 16 * (uint32_t)j : 0u)));
            }
        }
        uint4 out[NBG];
#pragma unroll
        for (int k = 0; k < NBG; k++) out[k] = in[k] ^ ks[k];
        if constexpr (SEAL) {
            // E_K(J0) (slot 0, lane 0) waits in the tag's place until the tag is known (4 VGPRs fewer across the loop;
            // opening needs the received tag there and recomputes E_K(J0) on the quad at the end instead)
            if (g == 0 && has && s == 0) st16(at(pay + len), ks[0]);
        }
        if (inner) {
            const uint32_t b = pay + 16 * (uint32_t)(t0 - 1);
#pragma unroll
            for (int k = 0; k < NBG; k++) st16_nt(at(b + 64 * k), out[k]);
#pragma unroll
            for (int k = 0; k < NBG; k++) w = gh.mulx(w, SEAL ? out[k] : in[k]);
        } else {
#pragma unroll
            for (int k = 0; k < NBG; k++) {
                const int t = t0 + 4 * k, j = t - 1;
                const bool full = t >= 1 && j < nfull, part = rem && j == nfull, lenslot = has && t == m + 1;
                if (full) st16_nt(at(pay + 16 * (uint32_t)j), out[k]);
                if (part) st_bytes(at(pay + 16 * (uint32_t)j), keep_bytes(out[k], (uint32_t)rem), (uint32_t)rem);
                // the length block rides in the slot after the payload when the group reaches it
                const uint4 x = lenslot ? lenblk() : part ? keep_bytes(SEAL ? out[k] : in[k], (uint32_t)rem)
                                                        : (SEAL ? out[k] : in[k]);
                if (full || part || lenslot) w = gh.mulx(w, x);
                len_done = len_done || lenslot;
            }
        }
    };
    for (int g = 0; g + 1 < G; g++) group(std::integral_constant<int, 4>{}, g);
    if (G > 0) {  // the last group with as few counter blocks per lane as its longest packet needs
        if (tail_slots <= 12) group(std::integral_constant<int, 3>{}, G - 1);
        else group(std::integral_constant<int, 4>{}, G - 1);
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
    uint4 y = fin.prod(w, make_uint4(0, 0, 0, 0));
    y = y ^ qperm<kQuadSwap1>(y);
    y = y ^ qperm<kQuadSwap2>(y);

    if constexpr (SEAL) {
        if (has && s == 0) st16(at(pay + len), y ^ ld16(at(pay + len)));  // tag = GHASH ^ E_K(J0) (stashed at group 0)
        constexpr int HNR = NR == 10 ? 10 : 14;
        const bool want_hp = (flags & (QPP_HP_MASK_OUT | QPP_HP_APPLY)) != 0;
        const qpp_pkt dt = reload_desc(dptr);
        const uint32_t pn_len = dt.pn_len;
        const bool hp = want_hp && has && pn_len >= 1 && pn_len <= 4 && len >= 4 - pn_len;  // quad-uniform
        if (hp) {
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
                if (flags & QPP_HP_APPLY) hdr_apply(at(dt.off), hdr_len, pn_len, hdr_load(at(dt.off), hdr_len), m0, m1);
            }
        }
        if (!has || s != 0) return;
        if (status) status[pkt_index] = want_hp && !hp ? QPP_DECODE_ERROR : QPP_OK;
    } else {
        // E_K(J0) on the quad (column s in lane s; J0 = nonce || be32(1)), compared column by column with the received
        // tag, the verdict OR-ed over the quad: all 16 bytes compared, no early exit
        const qpp_pkt dt = reload_desc(dptr);
        const uint32_t j0 = s == 0 ? key->iv[0]
                          : s == 1 ? key->iv[1] ^ bswap32((uint32_t)(dt.pn >> 32))
                          : s == 2 ? key->iv[2] ^ bswap32((uint32_t)dt.pn)
                                   : bswap32(1u);
        const uint32_t ek0 = aes_quad<NR>(aes, key->rk, j0, s);
        uint32_t want;
        __builtin_memcpy(&want, at(pay + len + 4 * s), 4);
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

// One workgroup per CU (grid = CUs) over an equal slice of the key-sorted packets, as aes_gcm_kernel (same plan meta,
// same single-key mode), 256 packets per pass.
template <bool SEAL, int NR>
__global__ __launch_bounds__(kQuadWG) void aes_gcm_quad_kernel(const DevKey *__restrict__ keys,
                                                              const qpp_pkt *__restrict__ descs,
                                                              const uint32_t *__restrict__ perm,
                                                              const WorkItem *__restrict__ work,
                                                              const uint32_t *__restrict__ meta,
                                                              uint8_t *__restrict__ arena, uint8_t *masks,
                                                              int8_t *status, uint32_t flags, uint32_t single,
                                                              uint32_t n_single) {
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
    uint32_t lo = p0 + min(n, blockIdx.x * P);
    const uint32_t hi = p0 + min(n, (blockIdx.x + 1) * P);
    if (lo >= hi) return;  // uniform
    uint32_t i = i_lo, j = i_hi;  // the item holding lo: largest i with work[i].begin <= lo
    while (!one && j - i > 1) {
        const uint32_t mid = (i + j) >> 1;
        if (work[mid].begin <= lo) i = mid; else j = mid;
    }
    const AesLds aes = make_aes(kLdsAes);
    const GhashT<true> gh = GhashT<true>::make();
    const uint32_t s = threadIdx.x & 3u, q = threadIdx.x >> 2;
    for (; lo < hi; i++) {  // key segments of the slice
        const WorkItem w = one ? WorkItem{single, 0u, n, (uint32_t)NR} : work[i];
        const uint32_t end = min(hi, w.begin + w.count);
        const DevKey *__restrict__ key = keys + w.key;
        __syncthreads();  // every wave is done with the previous segment's tables
        quad_tables(key);
        for (uint32_t t0 = lo; t0 < end; t0 += kQuadPkts) {
            const uint32_t t = t0 + q;
            const bool real = t < end;
            const uint32_t pi = one ? (real ? t : lo) : perm[real ? t : lo];
            const qpp_pkt d = descs[pi];  // (any valid descriptor for quads without a packet)
            bool has = real && !(d.flags & QPP_PKT_SKIP);
            if (one && has && d.key_idx != single) {  // not the live key: refused, untouched
                if (status && s == 0) status[pi] = QPP_INTERNAL_ERROR;
                has = false;
            }
            quad_packet<NR, SEAL>(aes, gh, key, has, d, descs + pi, pi, arena, masks, status, flags, s);
        }
        lo = end;
    }
}

template <bool SEAL, int NR>
void launch_quad(dim3 grid, hipStream_t s, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb,
                 uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags, uint32_t single, uint32_t n_single) {
    hipLaunchKernelGGL((aes_gcm_quad_kernel<SEAL, NR>), grid, dim3(kQuadWG), kLdsMax, s, keys, descs, pb.perm, pb.work,
                       pb.n_work, arena, masks, status, flags, single, n_single);
}
}  // namespace

// The quad-layout kernels behind launch_aes_gcm / launch_aes_gcm_single (aes_gcm.hip chooses).  single = 0xffffffff:
// planned batch (pb), else the one live AES key's slot (descs[0, n_single) in order, other slots refused).
hipError_t launch_aes_gcm_quad(bool seal, uint32_t nr, dim3 grid, hipStream_t s, const DevKey *keys,
                               const qpp_pkt *descs, const PlanBuffers &pb, uint8_t *arena, uint8_t *masks,
                               int8_t *status, uint32_t flags, uint32_t single, uint32_t n_single) {
    if (nr == 10) {
        if (seal) launch_quad<true, 10>(grid, s, keys, descs, pb, arena, masks, status, flags, single, n_single);
        else launch_quad<false, 10>(grid, s, keys, descs, pb, arena, masks, status, flags, single, n_single);
    } else {
        if (seal) launch_quad<true, 14>(grid, s, keys, descs, pb, arena, masks, status, flags, single, n_single);
        else launch_quad<false, 14>(grid, s, keys, descs, pb, arena, masks, status, flags, single, n_single);
    }
    return hipGetLastError();
}

}  // namespace qpp
