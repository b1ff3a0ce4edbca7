// burst.hip — small-batch AES-128/256-GCM seal/open (+ AES header protection) for gfx950: one WAVE per packet.
//
// Same operations and outputs as aes_gcm.hip (seal_in_place_scatter / open_in_place, src/aead/default.rs:44-93;
// HeaderKey::header_protection_mask, src/header_key.rs:52-56), for the batches the transport actually flushes:
// a GSO burst is at most 64 packets (quic/s2n-quic-platform/src/features/gso.rs:86).  The lane-per-packet kernel
// needs ~10^5 packets to fill the chip and takes one lane's serial time per packet (~135 us for 1200 B: 77 blocks
// x 10 dependent LDS rounds); here the 64 lanes of a wave split one packet's blocks, so a burst costs a few AES
// round chains instead.
//
// GHASH in parallel.  The packet's blocks X_0 .. X_{m-1} (AAD, ciphertext, length block) are front-padded with
// zeros to 64 K blocks (leading zeros do not change a Horner sum), lane l takes blocks l, l + 64, ...:
//   Y = sum_j X'_j H^(64K - j) = H * sum_l acc_l H^(63 - l),   acc_l = Horner over the lane's blocks with H^64,
// and the lane sum is a 6-level tree whose level t multiplies the left half by H^(2^t).  All multiplications are
// by one of 7 fixed powers P_t = H^(2^t), t = 0..6, each through a 4-bit table per nibble position
// (T_t[pos][nib] = (nib at nibble pos) * P_t, 32 x 16 x 16 B = 8 KiB): 32 ds_read_b128 per product, and every
// lane of a step reads the same 256-byte row, so the 16 nibble values sit in 16 distinct bank quads (no conflicts).
// T_0 comes from the key record's V[m] = H x^m; T_{t+1}[e] = T_t[e] * P_t through T_t.
//
// LDS (dynamic, offsets): [0, 64 KiB) AES T0/T1 bank-replicated (as aes_gcm.hip); [64, 120 KiB) T_0 .. T_6.
#include "chacha_wave.h"

namespace qpp {
namespace {
using namespace dev;

constexpr uint32_t kBurstAes = 0;
constexpr uint32_t kBurstGh = 65536;
constexpr uint32_t kBurstTab = 8192;
constexpr uint32_t kBurstHpRk = kBurstGh + 7 * kBurstTab;  // the work item key's HP round keys (240 B)
constexpr uint32_t kBurstLds = kBurstHpRk + 256;          // 120 KiB + 256 B: one workgroup per CU
#ifndef QPP_BURST_WAVES
#define QPP_BURST_WAVES 8  // measured: 4 waves 34 / 80 / 137 us seal at 64 / 4096 / 8192 packets, 8 waves 30 / 56 / 93, 12 waves 29 / 62 / 91
#endif
constexpr int kBurstWaves = QPP_BURST_WAVES;              // packets in flight per CU (one workgroup per CU)
constexpr int kBurstWG = 64 * kBurstWaves;
static_assert(kBurstLds <= kLdsMax, "LDS budget");

__device__ __forceinline__ uint32_t tab(int t) { return kBurstGh + (uint32_t)t * kBurstTab; }

// Z * P_t through T_t: nibble pos 2k = high nibble of byte k, 2k + 1 = its low nibble (GCM bit order: the byte's
// 0x80 bit is the lowest power of x).
// At most D byte positions (2 D reads) in flight: left to itself the compiler issued all 32 reads first -- 128 VGPRs
// for one product, which pushed the persistent server kernel (this code plus its polling state) into scratch memory,
// and on the pinned ring every scratch reload after the first payload stores waited for their PCIe round trip.
// 8 positions in flight still keep the LDS pipe busy (16 b128 reads issue in 64 cycles, about its latency).
__device__ __forceinline__ uint4 gmul(uint32_t base, uint4 z) {
#ifndef QPP_GMUL_DEPTH
#define QPP_GMUL_DEPTH 8  // (12, and either without the schedule barriers: the same server latency, profiles/r04s)
#endif
    constexpr int D = QPP_GMUL_DEPTH;
    const uint32_t w[4] = {z.x, z.y, z.z, z.w};
    uint4 hi[D], lo[D], acc[4];
    auto issue = [&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const uint32_t byte = w[k >> 2] >> (8 * (k & 3));
        hi[k % D] = lds_ld128(base + 512u * k + (byte & 0xf0u));
        lo[k % D] = lds_ld128(base + 512u * k + 256u + ((byte & 0x0fu) << 4));
    };
    static_for<D>([&](auto kc) { issue(kc); });
    static_for<16>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
#if !defined(QPP_GMUL_FREE)
        __builtin_amdgcn_sched_barrier(0);
#endif
        acc[k & 3] = k < 4 ? hi[k % D] ^ lo[k % D] : xor3(acc[k & 3], hi[k % D], lo[k % D]);
        if constexpr (k + D < 16) issue(std::integral_constant<int, k + D>{});
    });
    return xor3(acc[0], acc[1], acc[2] ^ acc[3]);
}

// T_0 of one key from its V[m] (nibble bit j <-> GCM bit index 4 pos + 3 - j).  No barrier inside.
__device__ __forceinline__ void burst_t0(const DevKey *__restrict__ key) {
    const uint4 *V = (const uint4 *)key->V;
    for (uint32_t e = threadIdx.x; e < 512; e += blockDim.x) {
        const uint32_t pos = e >> 4, nib = e & 15u;
        uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; j++)
            if ((nib >> j) & 1u) acc = acc ^ V[4 * pos + 3 - j];
        lds_st128(tab(0) + 16u * e, acc);
    }
}

// T_1 .. T_6 from T_0 in LDS: T_{t+1}[e] = T_t[e] * P_t through T_t (6 dependent levels).  Ends with a barrier.
__device__ __forceinline__ void burst_powers() {
    __syncthreads();
    for (int t = 0; t < 6; t++) {
        for (uint32_t e = threadIdx.x; e < 512; e += blockDim.x)
            lds_st128(tab(t + 1) + 16u * e, gmul(tab(t), lds_ld128(tab(t) + 16u * e)));
        __syncthreads();
    }
}

// T_0 .. T_6 for one key (the AES tables are built by the caller, before the work item is even read).  T_1 .. T_6
// come from the key's precomputed slot when it has one (pow.cap > slot: filled by pow_setup_kernel at install), else
// they are built here.  Ends with a barrier.
__device__ void burst_tables(const DevKey *__restrict__ key, uint32_t slot, const PowTables pow) {
    burst_t0(key);
    if (slot < pow.cap) {
        const uint4 *src = (const uint4 *)(pow.base + (size_t)slot * kPowBytes);
        for (uint32_t i = threadIdx.x; i < kPowTables * 8192u / 16; i += blockDim.x) lds_st128(tab(1) + 16u * i, src[i]);
        __syncthreads();
    } else {
        burst_powers();
    }
}

// One workgroup per listed slot: T_1 .. T_6 of an AES packet key into its pow slot, then the table of H^3 = T_1's
// entries times H (through T_0) -- the quad kernels' 4-bit tables of H^2, H^3, H^4 (quad.hip quad_tables).
constexpr uint32_t kPowSetupLds = kBurstGh + 8u * kBurstTab;  // T_0 .. T_6 and H^3's table: 128 KiB
__global__ __launch_bounds__(512) void pow_setup_kernel(const DevKey *__restrict__ keys,
                                                        const uint32_t *__restrict__ slots, const PowTables pow) {
    const uint32_t slot = slots[blockIdx.x];
    if (slot >= pow.cap) return;  // uniform
    const DevKey *__restrict__ key = keys + slot;
    if (key->live != 1 || key->suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256) return;
    burst_t0(key);
    burst_powers();
    for (uint32_t e = threadIdx.x; e < 512; e += blockDim.x)
        lds_st128(tab(7) + 16u * e, gmul(tab(0), lds_ld128(tab(1) + 16u * e)));
    __syncthreads();
    static_assert(kPowBytes == 7u * 8192u, "pow slot = T_1 .. T_6 + H^3");
    uint4 *dst = (uint4 *)(pow.base + (size_t)slot * kPowBytes);
    for (uint32_t i = threadIdx.x; i < kPowBytes / 16; i += blockDim.x) dst[i] = lds_ld128(tab(1) + 16u * i);
}

__device__ __forceinline__ uint4 shfl4_down(uint4 v, unsigned d) {
    return make_uint4((uint32_t)__shfl_down((int)v.x, d, 64), (uint32_t)__shfl_down((int)v.y, d, 64),
                      (uint32_t)__shfl_down((int)v.z, d, 64), (uint32_t)__shfl_down((int)v.w, d, 64));
}
// The persistent txq server's per-workgroup copy of its cached key's iv | rk | hp_rk (LDS, after the tables and
// the control words): no device-memory round trip per packet for them; its record header (suite, nr, hp_nr, live) at
// kTxsKeyHdr.
constexpr uint32_t kTxsCtl = kBurstLds;         // LDS: the polled slot (288 B) and the exit flag, for every wave
constexpr uint32_t kTxsStopFlag = kTxsCtl + 16 * kTxsPollLanes;
constexpr uint32_t kTxsKey = kTxsCtl + 320;
constexpr uint32_t kTxsKeyHdr = kTxsKey + 496;  // (iv | rk | hp_rk: 124 words)
constexpr uint32_t kTxsTrace = kTxsKey + 512;  // QPP_TXS_TRACE: wave 0's stamps inside its packet (8 words)
// header-protection mask items (kTxsMaskNr): their key's record header (suite, nr, hp_nr, live) and HP round keys,
// apart from the packet key above so that a mask between two seals of one key costs that key nothing
constexpr uint32_t kTxsMaskKey = kTxsTrace + 32;
// two-wave per-packet items (txs_two_wave): wave 1's 64 GHASH accumulators, then wave 0's tag verdict
constexpr uint32_t kTxsXchg = kTxsMaskKey + 256;
constexpr uint32_t kTxsLds = kTxsXchg + 1024 + 16;
static_assert(kTxsStopFlag + 4 <= kTxsKey && kTxsLds <= kLdsMax && kBurstWaves == (int)kTxsWaves, "server LDS");
#ifndef QPP_TXS_TRACE
#define QPP_TXS_TRACE 0  // 1: workgroup 0 stamps its phases into the mailbox (tools/diag/server_trace.py)
#endif
// wave 0, lane 0 of a server workgroup: s_memrealtime (low word) after all of this lane's loads have landed
#define TXS_STAMP(j)                                                                          \
    do {                                                                                      \
        if (QPP_TXS_TRACE && LDSKEY && threadIdx.x == 0) {                                    \
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                      \
            lds_st32(kTxsTrace + 4 * (j), (uint32_t)__builtin_amdgcn_s_memrealtime());        \
        }                                                                                     \
    } while (0)

// One packet on one wave (all 64 lanes; d is wave-uniform).  LDSKEY: the key's iv and header-protection round keys
// come from the server's LDS copy (kTxsKey) instead of the key record.
template <int NR, bool SEAL, bool LDSKEY = false>
__device__ __forceinline__ void burst_packet(const AesLds &aes, const DevKey *__restrict__ key,
                                             const uint32_t *__restrict__ rk, const qpp_pkt &d, uint32_t pi,
                                             uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags) {
    const uint32_t lane = threadIdx.x & 63u;
    PacketView p;
    if constexpr (LDSKEY) {
        p.base = arena + d.off;
        p.aad_len = d.aad_len;
        p.len = d.pt_len;
        p.pn_len = d.pn_len;
        p.n0 = lds_ld32(kTxsKey);  // Iv::nonce (src/iv.rs:27-39)
        p.n1 = lds_ld32(kTxsKey + 4) ^ bswap32((uint32_t)(d.pn >> 32));
        p.n2 = lds_ld32(kTxsKey + 8) ^ bswap32((uint32_t)d.pn);
    } else {
        p = load_packet(d, key, arena);
    }
    uint8_t *pay = p.base + p.aad_len;
    const uint32_t a = (p.aad_len + 15u) >> 4, c = (p.len + 15u) >> 4, m = a + c + 1;
    const uint32_t K = (m + 63u) >> 6, pad = 64u * K - m;
    // Each lane reads at most one 16-byte block per pass (a payload block or an AAD block).  The reads of a pair of
    // passes are issued before the previous pair's AES, so a packet pays one memory round trip, not one per pass
    // (over PCIe, from the pinned ring of a txq flush, a round trip is ~1.5-2.5 us).
    auto block = [&](uint32_t k) {
        const int i = (int)(lane + 64u * k) - (int)pad;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (i >= (int)a && i < (int)(a + c)) v = ld16(pay + 16u * (uint32_t)(i - (int)a));
        else if (i >= 0 && i < (int)a) v = ld16(p.base + 16u * (uint32_t)i);
        return v;
    };
    TXS_STAMP(0);
    uint4 nx0 = block(0), nx1 = K > 1 ? block(1) : make_uint4(0, 0, 0, 0);
    // header-protection round keys and header bytes: issued now, used after the passes (one memory round trip off
    // the end of the chain)
    constexpr int HNR = NR == 10 ? 10 : 14;
    const bool hp_on = SEAL && (flags & (QPP_HP_MASK_OUT | QPP_HP_APPLY)) != 0;
    HpPrefetch<HNR> hpk;
    constexpr uint32_t hp_lds = LDSKEY ? kTxsKey + 16 + 240 : kBurstHpRk;  // the HP round keys in LDS
    if (hp_on && lane == 0 && p.pn_len >= 1 && p.pn_len <= 4) hpk.load_hdr(p.base, p.aad_len - p.pn_len, flags);
    // open: the received tag, read now with the payload (read after the plaintext stores, it waited for their
    // round trip: stores and loads share one counter)
    uint4 want = make_uint4(0, 0, 0, 0);
    if (!SEAL && lane == 0) want = ld16(pay + p.len);
    uint4 acc = make_uint4(0, 0, 0, 0), ct0 = acc, ct1 = acc;  // ct0/ct1: ciphertext blocks 0/1 where owned
    uint4 ek = acc;  // E_K(J0), computed in pass 0 by the idle lane pad - 1 inside the data lanes' AES stream
    // counter block of this lane in pass k (data block b uses counter b + 2; J0 = counter 1 for everything else)
    auto ctr = [&](uint32_t k) {
        const int i = (int)(lane + 64u * k) - (int)pad;
        const bool data = i >= (int)a && i < (int)(a + c);
        return make_uint4(p.n0, p.n1, p.n2, bswap32(data ? (uint32_t)(i - (int)a) + 2u : 1u));
    };
    // pass k's payload block, the stores and the Horner step (acc * H^64 ^ x)
    auto pass = [&](uint32_t k, const uint4 &raw, const uint4 &ks) {
        const int i = (int)(lane + 64u * k) - (int)pad;  // block index in the GHASH sequence
        const bool data = i >= (int)a && i < (int)(a + c);
        const uint32_t b = (uint32_t)i - a;
        if (k == 0 && i == -1) ek = ks;
        uint4 x = make_uint4(0, 0, 0, 0);
        if (i >= 0 && i < (int)a) {
            const uint32_t off = 16u * (uint32_t)i;
            x = raw;
            if (p.aad_len - off < 16u) x = keep_bytes(x, p.aad_len - off);
        } else if (data) {
            const uint32_t r = p.len - 16u * b;
            uint4 in = raw, out = raw ^ ks;
            if (r >= 16u) {
                st16(pay + 16u * b, out);
            } else {
                out = keep_bytes(out, r);
                in = keep_bytes(in, r);
                st_bytes(pay + 16u * b, out, r);
            }
            x = SEAL ? out : in;
            if (b == 0) ct0 = x;
            if (b == 1) ct1 = x;
        } else if (i == (int)m - 1) {
            x = make_uint4(0, bswap32(p.aad_len * 8u), 0, bswap32(p.len * 8u));  // be64 bit lengths
        }
        acc = k ? gmul(tab(6), acc) ^ x : x;
    };
    // LDSKEY: the round keys from the server's LDS copy, one broadcast read per round (held in SGPRs for the whole
    // packet, 44 / 60 words, they crowded the server kernel's registers into scratch memory, and every reload after
    // the first ring stores waited for those stores' PCIe round trip)
    auto rkey = [&](int r, uint32_t (&k)[4]) {
        if constexpr (LDSKEY) {
            uint32_t o = kTxsKey + 16u + 16u * (uint32_t)r;
            asm volatile("" : "+v"(o));  // read where used, not hoisted out of the pass loop into 44-60 VGPRs
            const uint4 v = lds_ld128(o);
            k[0] = v.x; k[1] = v.y; k[2] = v.z; k[3] = v.w;
        } else {
            k[0] = rk[4 * r]; k[1] = rk[4 * r + 1]; k[2] = rk[4 * r + 2]; k[3] = rk[4 * r + 3];
        }
    };
    // Passes in pairs: the two passes' AES chains are independent, so they run interleaved (one chain of dependent
    // LDS rounds for both instead of one each); a pass past the packet (K odd) computes a discarded block.
    for (uint32_t k = 0; k < K; k += 2) {
        const uint4 r0 = nx0, r1 = nx1;
        if (k + 2 < K) nx0 = block(k + 2);
        if (k + 3 < K) nx1 = block(k + 3);
        if (k == 0) TXS_STAMP(1);
        const uint4 c0 = ctr(k), c1 = ctr(k + 1);
        // (round r + 1's key words read while round r runs: read right before its round, an LDS key read added its
        // latency to every round of the chain)
        uint32_t kk[4], kn[4];
        rkey(0, kk);
        rkey(1, kn);
        uint32_t s0[4] = {c0.x ^ kk[0], c0.y ^ kk[1], c0.z ^ kk[2], c0.w ^ kk[3]};
        if (k + 1 < K) {  // (uniform) a pair: two chains interleaved
            uint32_t s1[4] = {c1.x ^ kk[0], c1.y ^ kk[1], c1.z ^ kk[2], c1.w ^ kk[3]};
#pragma unroll
            for (int r = 1; r < NR; r++) {
#pragma unroll
                for (int i = 0; i < 4; i++) kk[i] = kn[i];
                rkey(r + 1, kn);
                aes.round(s0, kk);
                aes.round(s1, kk);
            }
            const uint4 ks0 = aes.final(s0, kn), ks1 = aes.final(s1, kn);
            pass(k, r0, ks0);
            pass(k + 1, r1, ks1);
        } else {  // the last pass of an odd count alone (the pair computed a discarded second chain)
#pragma unroll
            for (int r = 1; r < NR; r++) {
#pragma unroll
                for (int i = 0; i < 4; i++) kk[i] = kn[i];
                rkey(r + 1, kn);
                aes.round(s0, kk);
            }
            pass(k, r0, aes.final(s0, kn));
        }
    }
    TXS_STAMP(2);
    // Header protection (seal): the sample (ciphertext || tag)[4 - pn_len, 20 - pn_len) (payload.rs:151-169) lies in
    // ciphertext blocks 0 and 1 unless the payload is short (then it runs into the tag: after the tag, below).  Every
    // lane computes the mask of the same sample, in the same basic block as the lane tree, so that the two dependent
    // chains (AES rounds, tree levels) overlap instead of adding up.
    const uint32_t s_off = 4u - p.pn_len;
    const bool hp_ok = hp_on && p.pn_len >= 1 && p.pn_len <= 4 && p.len >= s_off;  // (uniform)
    const bool hp_early = hp_ok && p.len >= s_off + 16u;
    uint4 hmask = make_uint4(0, 0, 0, 0);
    if constexpr (SEAL) {
        const uint32_t o0 = (pad + a) & 63u;
        const uint4 c0 = shfl4(ct0, (int)o0), c1 = shfl4(ct1, (int)((o0 + 1u) & 63u));
        const uint32_t sh = s_off & 3u;  // (pn_len outside 1..4: any shift, the mask is not used)
        const uint4 smp = make_uint4(__builtin_amdgcn_alignbyte(c0.y, c0.x, sh), __builtin_amdgcn_alignbyte(c0.z, c0.y, sh),
                                     __builtin_amdgcn_alignbyte(c0.w, c0.z, sh), __builtin_amdgcn_alignbyte(c1.x, c0.w, sh));
        const uint4 smp0 = s_off == 0u ? c0 : smp;  // pn_len 4: the sample is block 0
        // (split over each quad: a quarter of the block's lookups per lane, next to the lane tree's table reads)
        const uint32_t q = lane & 3u;
        const uint32_t col = aes.encrypt_quad<HNR>(q == 0 ? smp0.x : q == 1 ? smp0.y : q == 2 ? smp0.z : smp0.w, hp_lds, q);
        hmask = make_uint4((uint32_t)__builtin_amdgcn_mov_dpp((int)col, 0x00, 0xf, 0xf, false),
                           (uint32_t)__builtin_amdgcn_mov_dpp((int)col, 0x55, 0xf, 0xf, false), 0u, 0u);
    }
    // lane tree: level t combines lanes l and l + 2^t (l a multiple of 2^(t+1)) as v_l * H^(2^t) ^ v_(l+2^t)
#pragma unroll
    for (int t = 0; t < 6; t++) acc = gmul(tab(t), acc) ^ shfl4_down(acc, 1u << t);
    TXS_STAMP(3);
    uint4 ek0;
    if (pad) {
        ek0 = shfl4(ek, (int)pad - 1);
    } else {  // (pad == 0: no idle lane in pass 0)
        const uint4 j0 = make_uint4(p.n0, p.n1, p.n2, bswap32(1u));
        if constexpr (LDSKEY) ek0 = aes.encrypt_lrk<NR>(j0, kTxsKey + 16u);
        else ek0 = aes.encrypt<NR>(j0, rk);
    }
    const uint4 tag = shfl4(gmul(tab(0), acc), 0) ^ ek0;  // Y = Q * H, from lane 0

    if (SEAL) {
        if (lane == 0) st16(pay + p.len, tag);
        int8_t st = QPP_OK;
        if (hp_on) {
            if (!hp_ok) {
                st = QPP_DECODE_ERROR;
            } else if (hp_early) {
                if (lane == 0) hpk.apply(hmask, p.base, p.aad_len - p.pn_len, p.pn_len, masks + 5 * (size_t)pi, flags);
            } else {  // short payload: the sample runs into the tag
                const uint32_t o0 = (pad + a) & 63u;
                const uint4 c0 = shfl4(ct0, (int)o0), c1 = shfl4(ct1, (int)((o0 + 1u) & 63u));
                uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
                for (uint32_t q = 0; q < 16; q++) {
                    const uint32_t pos = s_off + q;
                    const uint32_t v = pos < p.len ? (pos < 16u ? byte_of(c0, pos) : byte_of(c1, pos - 16u))
                                                   : byte_of(tag, pos - p.len);
                    w[q >> 2] |= v << (8 * (q & 3));
                }
                const uint4 smp = make_uint4(w[0], w[1], w[2], w[3]);
                if (lane == 0)
                    hpk.apply(aes.encrypt_lrk<HNR>(smp, hp_lds), p.base, p.aad_len - p.pn_len, p.pn_len,
                              masks + 5 * (size_t)pi, flags);
            }
        }
        TXS_STAMP(4);
        if (status && lane == 0) status[pi] = st;
    } else {
        const uint4 diff = tag ^ shfl4(want, 0);
        const bool ok = (diff.x | diff.y | diff.z | diff.w) == 0;  // all 16 bytes compared, no early exit
        if (!ok) {
            // never release unauthenticated plaintext: each lane zeroes the blocks it wrote (same-lane order)
            for (uint32_t k = 0; k < K; k++) {
                const int i = (int)(lane + 64u * k) - (int)pad;
                if (i >= (int)a && i < (int)(a + c)) {
                    const uint32_t b = (uint32_t)i - a, r = p.len - 16u * b;
                    if (r >= 16u) st16(pay + 16u * b, make_uint4(0, 0, 0, 0));
                    else st_bytes(pay + 16u * b, make_uint4(0, 0, 0, 0), r);
                }
            }
        }
        if (lane == 0) status[pi] = ok ? QPP_OK : QPP_DECRYPT_ERROR;
    }
}

template <bool SEAL, int NR>
__global__ __launch_bounds__(kBurstWG) void aes_gcm_burst_kernel(const DevKey *__restrict__ keys,
                                                                  const qpp_pkt *__restrict__ descs,
                                                                  const uint32_t *__restrict__ perm,
                                                                  const WorkItem *__restrict__ work,
                                                                  const uint32_t *__restrict__ n_work,
                                                                  uint8_t *__restrict__ arena, uint8_t *masks,
                                                                  int8_t *status, uint32_t flags, const PowTables pow) {
    // A burst's latency is a chain of memory round trips (pinned host memory for a zero-copy txq flush), so the
    // independent ones overlap: the AES tables (S-box) are built while the work count is read, and each wave's first
    // descriptor is fetched while the key's GHASH tables load.
    const uint32_t nw = *n_work;
    build_aes_tables(kBurstAes);
    if (blockIdx.x >= nw) return;  // uniform: grid is sized for the worst case
    const WorkItem w = work[blockIdx.x];
    if (w.nr != NR) return;
    const DevKey *__restrict__ key = keys + w.key;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t pi0 = 0;
    qpp_pkt d0{};
    if (wave < w.count) {
        pi0 = perm[w.begin + wave];
        d0 = descs[pi0];
    }
    if (threadIdx.x < 60) lds_st32(kBurstHpRk + 4 * threadIdx.x, key->hp_rk[threadIdx.x]);  // (burst_tables' barrier)
    burst_tables(key, w.key, pow);
    const AesLds aes = make_aes(kBurstAes);
    uint32_t rk[4 * (NR + 1)];
#pragma unroll
    for (int i = 0; i < 4 * (NR + 1); i++) rk[i] = __builtin_amdgcn_readfirstlane(key->rk[i]);
    for (uint32_t q = wave; q < w.count; q += kBurstWG / 64) {
        const uint32_t pi = q == wave ? pi0 : perm[w.begin + q];
        const qpp_pkt d = q == wave ? d0 : descs[pi];
        if (d.flags & QPP_PKT_SKIP) continue;
        burst_packet<NR, SEAL>(aes, key, rk, d, pi, arena, masks, status, flags);
    }
}

// ---------------------------------------------------------------- persistent transmit-queue server
// qpp_txq_create_persistent: the seal of a GSO burst without a kernel launch per flush.  The transport's queue.flush()
// (endpoint/mod.rs:158 -> socket/io/tx.rs:204-268) posts a flush by writing into pinned host memory; the workgroups
// below are already resident, with the AES tables built and the last key's GHASH tables and key words in LDS, and
// write completion words back into the same memory when the burst is sealed.
//
// Protocol (one flush in flight; the host posts the next only after every workgroup's `done`):
// * workgroup b polls its own TxsSlot: one wave-wide read (19 lanes x 16 B) returns the flush seq, the key epoch,
//   the workgroup's first work item and that item's descriptors, each tagged with the seq -- a read that raced the
//   host's writes shows a stale tag and is simply repeated.  So the flush, its plan and its descriptors cost one PCIe
//   round trip, and polls overlap (two in flight) so a new flush is seen within a fraction of one;
// * item i (one key, <= 8 packets, host-built) goes to workgroup i % grid, packet q of it to wave q; items beyond the
//   first of a workgroup (flushes of > grid items) are read from the items / sdesc arrays;
// * a workgroup keeps the GHASH tables and key words of the key it used last until a flush carries a new key epoch
//   (the host bumps it whenever key records were installed since its previous post: a slot can have been reused);
// * every flush starts with a system-scope acquire: the ring is pinned host memory the GPU caches like any other, and
//   the transport rewrites the same offsets flush after flush;
// * completion: every storing wave drains its stores, the workgroup releases at system scope and writes its slot's
//   done = seq; the host waits for all of them;
// * a workgroup leaves on the stop word, or after idle_ticks without a flush -- the host never posts to a server
//   that may be leaving on its own: after a quarter of that idle time without a post it stops the server and starts
//   a new one first (api.cpp srv_submit), so a flush is seen by every workgroup or by none (the idle exit is for a
//   host that went away).

// A transmit flush's packet is sealed and header-protected; a per-packet request (kTxsPktNoHp: Key::encrypt,
// kTxsPktOpen: Key::decrypt) is sealed without header protection or opened, its status into the slot (status[wave]).
template <int NR>
__device__ __forceinline__ void txs_item(const AesLds &aes, const DevKey *key, const qpp_pkt &d,
                                         uint32_t wave, uint32_t count, uint8_t *ring, int8_t *status) {
    const uint32_t *rk = nullptr;  // (the round keys come from LDS: burst_packet<.., LDSKEY = true>)
    if (wave < count && !(d.flags & QPP_PKT_SKIP)) {
        if (d.flags & kTxsPktOpen)
            burst_packet<NR, false, true>(aes, key, rk, d, wave, ring, nullptr, status, 0);
        else if (d.flags & kTxsPktNoHp)
            burst_packet<NR, true, true>(aes, key, rk, d, wave, ring, nullptr, status, 0);
        else
            burst_packet<NR, true, true>(aes, key, rk, d, 0, ring, nullptr, nullptr, QPP_HP_APPLY);
    }
}

// A ChaCha20-Poly1305 work item (cipher_suite.rs:270-284): one wave per packet (chacha_wave_packet, the burst kernel's
// code), the key and HP key from the LDS copy, the header protected in place
__device__ __forceinline__ void txs_item_chacha(const qpp_pkt &d, uint32_t wave, uint32_t count, uint8_t *ring,
                                                int8_t *status, uint32_t lane) {
    uint32_t k[8], hk[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        k[i] = __builtin_amdgcn_readfirstlane(lds_ld32(kTxsKey + 16 + 4 * i));
        hk[i] = __builtin_amdgcn_readfirstlane(lds_ld32(kTxsKey + 256 + 4 * i));
    }
    // Iv::nonce (src/iv.rs:27-39)
    const uint32_t n0 = lds_ld32(kTxsKey), n1 = lds_ld32(kTxsKey + 4) ^ bswap32((uint32_t)(d.pn >> 32)),
                   n2 = lds_ld32(kTxsKey + 8) ^ bswap32((uint32_t)d.pn);
    if (wave < count && !(d.flags & QPP_PKT_SKIP)) {
        if (d.flags & kTxsPktOpen)
            chacha_wave_packet<false>(k, n0, n1, n2, hk, d, ring, nullptr, status + wave, 0, lane);
        else if (d.flags & kTxsPktNoHp)
            chacha_wave_packet<true>(k, n0, n1, n2, hk, d, ring, nullptr, status + wave, 0, lane);
        else
            chacha_wave_packet<true>(k, n0, n1, n2, hk, d, ring, nullptr, nullptr, QPP_HP_APPLY, lane);
    }
}

// A header-protection mask item (HeaderKey::*_header_protection_mask, header_key.rs:52-56): the 16-byte sample at
// ring offset d.off, the 5 mask bytes written at d.off + 16, by lane 0 of wave 0 (every lane computes the block)
__device__ __forceinline__ void txs_mask_item(const AesLds &aes, const qpp_pkt &d, uint32_t wave, uint32_t count,
                                              uint8_t *ring, uint32_t lane) {
    if (!(wave < count)) return;
    const uint4 smp = ld16(ring + d.off);
    const uint32_t suite = lds_ld32(kTxsMaskKey), hp_nr = lds_ld32(kTxsMaskKey + 8);
    uint32_t m0 = 0, m1 = 0;
    if (suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256) {
        uint32_t hk[8];
#pragma unroll
        for (int i = 0; i < 8; i++) hk[i] = lds_ld32(kTxsMaskKey + 16 + 4 * i);
        m0 = chacha_hp_quad(hk, smp, lane & 3u, &m1);
    } else {
        const uint32_t q = lane & 3u, in = q == 0 ? smp.x : q == 1 ? smp.y : q == 2 ? smp.z : smp.w;
        const uint32_t col = hp_nr == 14 ? aes.encrypt_quad<14>(in, kTxsMaskKey + 16, q)
                                         : aes.encrypt_quad<10>(in, kTxsMaskKey + 16, q);
        m0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)col, 0x00, 0xf, 0xf, false);
        m1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)col, 0x55, 0xf, 0xf, false);
    }
    if (lane == 0) {
        uint8_t *o = ring + d.off + 16;
        o[0] = (uint8_t)m0; o[1] = (uint8_t)(m0 >> 8); o[2] = (uint8_t)(m0 >> 16); o[3] = (uint8_t)(m0 >> 24);
        o[4] = (uint8_t)m1;
    }
}

// A per-packet item (seal without HP, or open) of a packet of one or two 64-block passes, one wave per pass: wave w
// runs pass w (one AES chain each instead of a pair interleaved on one wave -- for one pass burst_packet computes a
// discarded second chain -- the chain is issue-bound on a single wave); with two passes wave 1 hands its lanes' GHASH
// accumulators over LDS and wave 0 combines them (acc0 * H^64 + acc1, the Horner step of the pair); wave 0 runs the
// lane tree and the tag.  Opening: wave 0's verdict goes back over LDS and each wave zeroes the plaintext it
// wrote (a wave's own stores stay ordered).  Every wave of the workgroup calls it (one or two barriers).
template <int NR, bool SEAL>
__device__ __forceinline__ void txs_two_wave(const AesLds &aes, const qpp_pkt &d, uint32_t wave, uint8_t *ring,
                                             int8_t *status) {
    const uint32_t lane = threadIdx.x & 63u;
    uint8_t *base = ring + d.off;
    const uint32_t aad_len = d.aad_len, len = d.pt_len;
    uint8_t *pay = base + aad_len;
    const uint32_t a = (aad_len + 15u) >> 4, c = (len + 15u) >> 4, m = a + c + 1, K = m > 64u ? 2u : 1u,
                   pad = 64u * K - m;
    const uint32_t n0 = lds_ld32(kTxsKey), n1 = lds_ld32(kTxsKey + 4) ^ bswap32((uint32_t)(d.pn >> 32)),
                   n2 = lds_ld32(kTxsKey + 8) ^ bswap32((uint32_t)d.pn);  // Iv::nonce (src/iv.rs:27-39)
    const uint32_t k = wave;  // this wave's pass (waves >= 2: none)
    const int i = (int)(lane + 64u * k) - (int)pad;
    const bool data = i >= (int)a && i < (int)(a + c), aadb = i >= 0 && i < (int)a;
    const uint32_t b = (uint32_t)i - a;
    uint4 acc = make_uint4(0, 0, 0, 0), ek = acc, want = acc;
    if (wave < K) {
        uint4 raw = make_uint4(0, 0, 0, 0);
        if (data) raw = ld16(pay + 16u * b);
        else if (aadb) raw = ld16(base + 16u * (uint32_t)i);
        if (!SEAL && wave == 0 && lane == 0) want = ld16(pay + len);
        // AES of the lane's counter block (data block b: counter b + 2; every other lane J0 = counter 1)
        uint32_t kk[4], kn[4];
        auto rkey = [&](int r, uint32_t (&o)[4]) {
            uint32_t off = kTxsKey + 16u + 16u * (uint32_t)r;
            asm volatile("" : "+v"(off));
            const uint4 v = lds_ld128(off);
            o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
        };
        rkey(0, kk);
        rkey(1, kn);
        const uint32_t ctr = bswap32(data ? b + 2u : 1u);
        uint32_t st[4] = {n0 ^ kk[0], n1 ^ kk[1], n2 ^ kk[2], ctr ^ kk[3]};
#pragma unroll
        for (int r = 1; r < NR; r++) {
#pragma unroll
            for (int q = 0; q < 4; q++) kk[q] = kn[q];
            rkey(r + 1, kn);
            aes.round(st, kk);
        }
        const uint4 ks = aes.final(st, kn);
        if (wave == 0 && i == -1) ek = ks;  // E_K(J0) from the idle lane pad - 1 of pass 0
        uint4 x = make_uint4(0, 0, 0, 0);
        if (aadb) {
            const uint32_t off = 16u * (uint32_t)i;
            x = aad_len - off < 16u ? keep_bytes(raw, aad_len - off) : raw;
        } else if (data) {
            const uint32_t r = len - 16u * b;
            uint4 in = raw, out = raw ^ ks;
            if (r >= 16u) {
                st16(pay + 16u * b, out);
            } else {
                out = keep_bytes(out, r);
                in = keep_bytes(in, r);
                st_bytes(pay + 16u * b, out, r);
            }
            x = SEAL ? out : in;
        } else if (i == (int)m - 1) {
            x = make_uint4(0, bswap32(aad_len * 8u), 0, bswap32(len * 8u));  // be64 bit lengths
        }
        acc = x;
        if (wave == 1) lds_st128(kTxsXchg + 16u * lane, acc);
    }
    __syncthreads();
    bool ok = true;
    if (wave == 0) {
        if (K == 2) acc = gmul(tab(6), acc) ^ lds_ld128(kTxsXchg + 16u * lane);  // the pair's Horner step
#pragma unroll
        for (int t = 0; t < 6; t++) acc = gmul(tab(t), acc) ^ shfl4_down(acc, 1u << t);
        const uint4 ek0 = pad ? shfl4(ek, (int)pad - 1)
                              : aes.encrypt_lrk<NR>(make_uint4(n0, n1, n2, bswap32(1u)), kTxsKey + 16u);
        const uint4 tag = shfl4(gmul(tab(0), acc), 0) ^ ek0;
        if constexpr (SEAL) {
            if (lane == 0) {
                st16(pay + len, tag);
                status[0] = QPP_OK;
            }
        } else {
            const uint4 diff = tag ^ shfl4(want, 0);
            ok = (diff.x | diff.y | diff.z | diff.w) == 0;  // all 16 bytes compared
            if (lane == 0) {
                lds_st32(kTxsXchg + 1024u, ok ? 1u : 0u);
                status[0] = ok ? QPP_OK : QPP_DECRYPT_ERROR;
            }
        }
    }
    if constexpr (!SEAL) {
        __syncthreads();
        ok = lds_ld32(kTxsXchg + 1024u) != 0;
        if (!ok && wave < K && data) {  // never release unauthenticated plaintext: each wave zeroes its own blocks
            const uint32_t r = len - 16u * b;
            if (r >= 16u) st16(pay + 16u * b, make_uint4(0, 0, 0, 0));
            else st_bytes(pay + 16u * b, make_uint4(0, 0, 0, 0), r);
        }
    }
}

// one 16-byte chunk of the slot (lane < kTxsPollLanes), in ONE load past every cache (sc0 sc1: the host writes it;
// a chunk is read whole, so its tag vouches for its other words)
// lane kTxsPollLanes reads the device's eviction word in the same load (api.cpp release: every resident server of the
// device leaves at its next poll without a complete flush, so that a free past the parked bound need not wait for it)
__device__ __forceinline__ uint4 txs_poll(const TxsSlot *slot, const uint32_t *evict, uint32_t lane) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    uint4 v = make_uint4(0, 0, 0, 0);
    const u32x4 *src = lane < kTxsPollLanes ? (const u32x4 *)slot + lane : (const u32x4 *)evict;
    if (lane <= kTxsPollLanes) {
        const u32x4 c = *(const volatile u32x4 *)src;
        v = make_uint4(c.x, c.y, c.z, c.w);
    }
    return v;
}

__global__ __launch_bounds__(kBurstWG) void txq_server_kernel(const DevKey *keys, const PowTables pow, TxsMail *mail,
                                                              TxsSlot *slots, const WorkItem *items,
                                                              const qpp_pkt *sdesc, uint8_t *ring, uint32_t ring_bytes,
                                                              uint32_t seq0, uint32_t idle_ticks,
                                                              const uint32_t *evict) {
    build_aes_tables(kBurstAes);
    __syncthreads();
    const AesLds aes = make_aes(kBurstAes);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    TxsSlot *slot = slots + blockIdx.x;
    uint32_t seen = seq0, cached = 0xffffffffu, mcached = 0xffffffffu, epoch = 0xffffffffu;
    {
        // A server relaunched behind a posted flush (seq0 = posted - 1: the previous one left on its idle timeout
        // before every workgroup had seen it) must not seal it again in the workgroups that did: the ring is sealed in
        // place.  This workgroup's `done` equal to its slot's seq means it already has.  (Kernel start: no cache holds
        // these host-written words yet.)
        const uint32_t posted = *(const volatile uint32_t *)&slot->seq;
        const uint32_t done = *(const volatile uint32_t *)&slot->done;
        if (posted != seq0 && done == posted) seen = posted;
    }
    uint64_t t_seen = 0;  // thread 0: when this workgroup saw the flush (s_memrealtime)
    for (;;) {
        if (wave == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t stop = 0;
            uint4 cur = txs_poll(slot, evict, lane);
            for (;;) {
                __builtin_amdgcn_s_sleep(4);
                const uint4 nxt = txs_poll(slot, evict, lane);  // in flight while `cur` is examined
                const uint32_t seq = __shfl((int)cur.x, 0, 64), word = __shfl((int)cur.y, 0, 64);
                if (seq != seen) {
                    if ((word & kTxsItemsMask) == kTxsStop) {
                        stop = 1;
                        break;
                    }
                    // every chunk of this flush must carry its seq (last word): the item (chunk 1) and the
                    // descriptors 0 .. count - 1 (descriptor q in chunks 2 + 2q, 3 + 2q)
                    const uint32_t item_cnt = __shfl((int)cur.y, 1, 64);
                    bool ok = true;
                    if (lane == 1) ok = cur.w == seq;
                    if (lane >= 2 && lane < kTxsPollLanes && (lane - 2) / 2 < item_cnt) ok = cur.w == seq;
                    if (__all(ok)) break;
                }
                // idle timeout, or evicted (between flushes only: a complete flush above is served first)
                if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks || __shfl((int)cur.x, kTxsPollLanes, 64)) {
                    stop = 1;
                    break;
                }
                cur = nxt;
            }
            if (lane < kTxsPollLanes) lds_st128(kTxsCtl + 16 * lane, cur);
            if (lane == 0) {
                lds_st32(kTxsStopFlag, stop);
                // (telemetry stamp kept in a register and stored with t_done: a store here would be waited for by
                // the acquire below and by this wave's first payload loads -- a PCIe write round trip)
                t_seen = __builtin_amdgcn_s_memrealtime();
                // Every flush: the CU's vector cache (and L2's non-coherent lines) dropped, so that this flush's ring
                // bytes are read from the host, not the lines the previous flush left for the same offsets (the ring
                // is reused flush after flush; without it, every flush after the first of one server launch sealed
                // stale plaintext: tools/diag/server_mismatch.py), and key records installed since are visible.
                // (Reading the ring past the caches instead -- volatile loads, then system-scope buffer loads --
                // measured slower, and the buffer-load build faulted the GPU on a many-key flush: round 4, r04k.)
                if (!stop) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            }
        }
        __syncthreads();
        const uint32_t stop = lds_ld32(kTxsStopFlag);
        if (stop) break;  // uniform
        const uint4 hdr = lds_ld128(kTxsCtl);
        const uint4 it0 = lds_ld128(kTxsCtl + 16);
        const WorkItem w0{it0.x, 0u, it0.y, it0.z};  // (begin unused: its descriptors came with the slot)
        const uint4 da = lds_ld128(kTxsCtl + 32 + 32 * wave), db = lds_ld128(kTxsCtl + 48 + 32 * wave);
        qpp_pkt d0;
        d0.pn = (uint64_t)da.x | (uint64_t)da.y << 32;
        d0.key_idx = da.z;
        d0.off = db.x;
        d0.aad_len = (uint16_t)db.y;
        d0.pt_len = (uint16_t)(db.y >> 16);
        d0.pn_len = (uint8_t)db.z;
        d0.flags = (uint8_t)(db.z >> 8);
        d0.reserved = 0;
        seen = hdr.x;
        const uint32_t n_items = hdr.y & kTxsItemsMask, ep = hdr.y >> 24;
        // Items beyond the slot's and the key records change between flushes: read with VECTOR loads through
        // laundered pointers (wave-uniform addresses were otherwise scalar loads, whose cache no fence covers)
        const WorkItem *items_v = items;
        const qpp_pkt *sdesc_v = sdesc;
        const DevKey *keys_v = keys;
        asm volatile("" : "+v"(items_v), "+v"(sdesc_v), "+v"(keys_v));
        if (ep != epoch) {
            epoch = ep;
            cached = mcached = 0xffffffffu;
        }
        uint64_t tr[4] = {0, 0, 0, 0}, clk0 = 0;
        if (QPP_TXS_TRACE && threadIdx.x == 0) {
            tr[0] = __builtin_amdgcn_s_memrealtime();
            clk0 = __builtin_amdgcn_s_memtime();  // shader clock: its rate over the flush = the clock the flush ran at
            tr[1] = tr[0];
        }
        // a descriptor whose bytes do not lie inside the ring is refused, never dereferenced (the host validates every
        // push: this counter stays 0 -- VERDICT r4 #3(a) asked for the check on every ring offset the server reads)
        auto in_ring = [&](const qpp_pkt &x) {
            return (uint64_t)x.off + x.aad_len + x.pt_len + 16u <= (uint64_t)ring_bytes;
        };
        for (uint32_t it = blockIdx.x; it < n_items; it += gridDim.x) {
            const bool first = it == blockIdx.x;
            const WorkItem w = first ? w0 : items_v[it];
            qpp_pkt d = first ? d0 : sdesc_v[it * kBurstWaves + wave];
            if (wave < w.count && !(d.flags & QPP_PKT_SKIP) && !in_ring(d)) {
                d.flags |= QPP_PKT_SKIP;
                if (lane == 0) __hip_atomic_fetch_add(&mail->oob, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            const DevKey *key = keys_v + w.key;
            if (w.count == 0) continue;  // (a per-packet request posts one packet to one workgroup, none to the others)
            if (w.nr == kTxsMaskNr) {  // uniform: a mask item -- its key's header and HP round keys, cached apart
                if (w.key != mcached) {
                    __syncthreads();
                    const uint32_t *kw = (const uint32_t *)key;
                    if (threadIdx.x < 4) lds_st32(kTxsMaskKey + 4 * threadIdx.x, kw[threadIdx.x]);
                    else if (threadIdx.x < 64) lds_st32(kTxsMaskKey + 16 + 4 * (threadIdx.x - 4), kw[64 + threadIdx.x]);
                    __syncthreads();
                    mcached = w.key;
                }
                if (lds_ld32(kTxsMaskKey + 12) != 0) txs_mask_item(aes, d, wave, w.count, ring, lane);  // (live 1 or 2)
                continue;
            }
            if (w.key != cached) {  // uniform
                __syncthreads();  // every wave is done with the previous key's tables
                // iv | rk | hp_rk: 124 consecutive words of the record (DevKey: iv at word 4), then its header
                const uint32_t *kw = (const uint32_t *)key;
                if (threadIdx.x < 124) lds_st32(kTxsKey + 4 * threadIdx.x, kw[4 + threadIdx.x]);
                else if (threadIdx.x < 128) lds_st32(kTxsKeyHdr + 4 * (threadIdx.x - 124), kw[threadIdx.x - 124]);
                if (w.nr == 10 || w.nr == 14) burst_tables(key, w.key, pow);  // (ends with a barrier)
                else __syncthreads();  // (ChaCha20: no GHASH tables)
                cached = w.key;
            }
            // the record as installed (a key freed since the flush was planned: its packets are left alone, as the
            // launched path's kernels refuse them)
            const uint32_t k_suite = lds_ld32(kTxsKeyHdr), k_nr = lds_ld32(kTxsKeyHdr + 4),
                           k_live = lds_ld32(kTxsKeyHdr + 12);
            if (first && w.count == 1 && k_live == 1 && k_nr == w.nr && (w.nr == 10 || w.nr == 14)) {
                // a per-packet seal / open of a packet of one or two 64-block passes: a wave per pass (txs_two_wave).  Every
                // wave decides from wave 0's descriptor (the slot copy in LDS), so all take the same branch.
                const uint4 da = lds_ld128(kTxsCtl + 32), db = lds_ld128(kTxsCtl + 48);
                qpp_pkt dd;
                dd.pn = (uint64_t)da.x | (uint64_t)da.y << 32;
                dd.key_idx = da.z;
                dd.off = db.x;
                dd.aad_len = (uint16_t)db.y;
                dd.pt_len = (uint16_t)(db.y >> 16);
                dd.pn_len = (uint8_t)db.z;
                dd.flags = (uint8_t)(db.z >> 8);
                dd.reserved = 0;
                const uint32_t mm = ((dd.aad_len + 15u) >> 4) + ((dd.pt_len + 15u) >> 4) + 1u;
                if ((dd.flags & (kTxsPktNoHp | kTxsPktOpen)) && !(dd.flags & QPP_PKT_SKIP) && mm <= 128u && in_ring(dd)) {
                    const bool open = (dd.flags & kTxsPktOpen) != 0;
                    if (w.nr == 10) {
                        if (open) txs_two_wave<10, false>(aes, dd, wave, ring, slot->status);
                        else txs_two_wave<10, true>(aes, dd, wave, ring, slot->status);
                    } else {
                        if (open) txs_two_wave<14, false>(aes, dd, wave, ring, slot->status);
                        else txs_two_wave<14, true>(aes, dd, wave, ring, slot->status);
                    }
                    continue;
                }
            }
            if (k_live == 1 && k_nr == w.nr) {
                if (w.nr == 10) txs_item<10>(aes, key, d, wave, w.count, ring, slot->status);
                else if (w.nr == 14) txs_item<14>(aes, key, d, wave, w.count, ring, slot->status);
                else if (k_suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256)
                    txs_item_chacha(d, wave, w.count, ring, slot->status, lane);
            }
        }
        // completion: this workgroup's ring stores reach the host before its done word
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (QPP_TXS_TRACE && threadIdx.x == 0) tr[2] = __builtin_amdgcn_s_memrealtime();
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            if (blockIdx.x == 0) {
                if (QPP_TXS_TRACE) {
                    tr[3] = __builtin_amdgcn_s_memrealtime();
                    const uint64_t clk1 = __builtin_amdgcn_s_memtime();
                    for (int j = 0; j < 4; j++)
                        __hip_atomic_store(&mail->pad0[j], tr[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(&mail->pad0[4], clk1 - clk0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    for (int j = 0; j < 5; j++)
                        __hip_atomic_store(&mail->pad1[j], lds_ld32(kTxsTrace + 4 * j), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
                }
                __hip_atomic_store(&mail->t_done, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(&mail->t_seen, t_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            __hip_atomic_store(&slot->done, seen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();  // (the next poll's LDS copy does not overwrite this flush's before every wave read it)
    }
}

template <bool SEAL, int NR>
void launch_burst(dim3 grid, hipStream_t s, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb,
                  uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags, const PowTables &pow) {
    hipLaunchKernelGGL((aes_gcm_burst_kernel<SEAL, NR>), grid, dim3(kBurstWG), kBurstLds, s, keys, descs, pb.perm,
                       pb.work, pb.n_work, arena, masks, status, flags, pow);
}
}  // namespace

uint32_t burst_packets_per_item(uint32_t n, uint32_t n_cu) {
    // enough items to spread the batch over every CU; an item fills the workgroup's waves (or, for tiny batches,
    // 4 of them, so more CUs take part); at most 8 packets per wave
    const uint32_t w = (uint32_t)kBurstWaves;
    uint32_t per = n_cu ? (n + n_cu - 1) / n_cu : 8u * w;
    per = per <= w ? ((per + 3u) & ~3u) : (per + w - 1) / w * w;
    return per < 4u ? 4u : per > 8u * w ? 8u * w : per;
}

hipError_t launch_aes_gcm_burst(bool seal, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb,
                                uint32_t n, uint32_t key_cap, uint32_t per, uint8_t *arena, uint8_t *masks,
                                int8_t *status, uint32_t flags, uint32_t suites, const PowTables &pow,
                                hipStream_t s) {
    if (!n) return hipSuccess;
    const dim3 grid(plan_max_work(n, key_cap, per));
    if (suites & (1u << QPP_SUITE_TLS_AES_128_GCM_SHA256)) {
        if (seal) launch_burst<true, 10>(grid, s, keys, descs, pb, arena, masks, status, flags, pow);
        else launch_burst<false, 10>(grid, s, keys, descs, pb, arena, masks, status, flags, pow);
    }
    if (suites & (1u << QPP_SUITE_TLS_AES_256_GCM_SHA384)) {
        if (seal) launch_burst<true, 14>(grid, s, keys, descs, pb, arena, masks, status, flags, pow);
        else launch_burst<false, 14>(grid, s, keys, descs, pb, arena, masks, status, flags, pow);
    }
    return hipGetLastError();
}

hipError_t launch_txq_server(const DevKey *keys, const PowTables &pow, TxsMail *mail, TxsSlot *slots,
                             const WorkItem *items, const qpp_pkt *sdesc, uint8_t *ring, uint32_t ring_bytes,
                             uint32_t seq0, uint32_t idle_ticks, uint32_t wgs, const uint32_t *evict, hipStream_t s) {
    hipLaunchKernelGGL(txq_server_kernel, dim3(wgs), dim3(kBurstWG), kTxsLds, s, keys, pow, mail, slots, items,
                       sdesc, ring, ring_bytes, seq0, idle_ticks, evict);
    return hipGetLastError();
}

hipError_t launch_pow_setup(const DevKey *keys, const uint32_t *slots, uint32_t count, const PowTables &pow,
                            hipStream_t s) {
    if (!count || !pow.cap) return hipSuccess;
    hipLaunchKernelGGL(pow_setup_kernel, dim3(count), dim3(512), kPowSetupLds, s, keys, slots, pow);
    return hipGetLastError();
}

}  // namespace qpp
