// chacha.hip — ChaCha20-Poly1305 seal/open + the standalone header-protection mask kernel (gfx950).
//
// Replaces, for TLS_CHACHA20_POLY1305_SHA256 (quic/s2n-quic-crypto/src/cipher_suite.rs:270-284,
// cipher_suite/ring.rs:121), aws-lc-rs's RFC 8439 AEAD behind <LessSafeKey as Aead>::{encrypt,decrypt}
// (src/aead/default.rs:44-93) and quic::CHACHA20 HeaderProtectionKey::new_mask (src/header_key.rs:52-56):
//   mask = ChaCha20(hp, counter = LE32(sample[0..4]), nonce = sample[4..16]) over 5 zero bytes.
//
// Mapping: one lane per packet, pure VALU (ARX + 26-bit-limb Poly1305); LDS only stages the payload for coalesced
// I/O, so keys are per lane and a mixed-key batch needs no grouping.  Each iteration produces one 64-byte keystream
// block, seals 4 x 16 bytes and absorbs them into Poly1305.
#include "device_common.h"

namespace qpp {
namespace {
using namespace dev;

// Poly1305 (RFC 8439 §2.5) in 5 x 26-bit limbs; every block of the AEAD MAC stream is a full 16-byte
// block (AAD and ciphertext are zero-padded), so the 2^128 bit is always set.
struct Poly1305 {
    uint32_t r0, r1, r2, r3, r4, s1, s2, s3, s4;
    uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0, h4 = 0;

    __device__ __forceinline__ void init(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
        r0 = k0 & 0x3ffffff;
        r1 = ((k0 >> 26) | (k1 << 6)) & 0x3ffff03;
        r2 = ((k1 >> 20) | (k2 << 12)) & 0x3ffc0ff;
        r3 = ((k2 >> 14) | (k3 << 18)) & 0x3f03fff;
        r4 = (k3 >> 8) & 0x00fffff;
        s1 = r1 * 5; s2 = r2 * 5; s3 = r3 * 5; s4 = r4 * 5;
    }
    __device__ __forceinline__ void block(uint4 m) {
        h0 += m.x & 0x3ffffff;
        h1 += ((m.x >> 26) | (m.y << 6)) & 0x3ffffff;
        h2 += ((m.y >> 20) | (m.z << 12)) & 0x3ffffff;
        h3 += ((m.z >> 14) | (m.w << 18)) & 0x3ffffff;
        h4 += (m.w >> 8) | (1u << 24);
        uint64_t d0 = (uint64_t)h0 * r0 + (uint64_t)h1 * s4 + (uint64_t)h2 * s3 + (uint64_t)h3 * s2 + (uint64_t)h4 * s1;
        uint64_t d1 = (uint64_t)h0 * r1 + (uint64_t)h1 * r0 + (uint64_t)h2 * s4 + (uint64_t)h3 * s3 + (uint64_t)h4 * s2;
        uint64_t d2 = (uint64_t)h0 * r2 + (uint64_t)h1 * r1 + (uint64_t)h2 * r0 + (uint64_t)h3 * s4 + (uint64_t)h4 * s3;
        uint64_t d3 = (uint64_t)h0 * r3 + (uint64_t)h1 * r2 + (uint64_t)h2 * r1 + (uint64_t)h3 * r0 + (uint64_t)h4 * s4;
        uint64_t d4 = (uint64_t)h0 * r4 + (uint64_t)h1 * r3 + (uint64_t)h2 * r2 + (uint64_t)h3 * r1 + (uint64_t)h4 * r0;
        uint32_t c;
        c = (uint32_t)(d0 >> 26); h0 = (uint32_t)d0 & 0x3ffffff;
        d1 += c; c = (uint32_t)(d1 >> 26); h1 = (uint32_t)d1 & 0x3ffffff;
        d2 += c; c = (uint32_t)(d2 >> 26); h2 = (uint32_t)d2 & 0x3ffffff;
        d3 += c; c = (uint32_t)(d3 >> 26); h3 = (uint32_t)d3 & 0x3ffffff;
        d4 += c; c = (uint32_t)(d4 >> 26); h4 = (uint32_t)d4 & 0x3ffffff;
        h0 += c * 5; c = h0 >> 26; h0 &= 0x3ffffff;
        h1 += c;
    }
    // tag = (h mod p + s) mod 2^128
    __device__ __forceinline__ uint4 finish(uint32_t s0w, uint32_t s1w, uint32_t s2w, uint32_t s3w) {
        uint32_t c;
        c = h1 >> 26; h1 &= 0x3ffffff; h2 += c;
        c = h2 >> 26; h2 &= 0x3ffffff; h3 += c;
        c = h3 >> 26; h3 &= 0x3ffffff; h4 += c;
        c = h4 >> 26; h4 &= 0x3ffffff; h0 += c * 5;
        c = h0 >> 26; h0 &= 0x3ffffff; h1 += c;
        // g = h + 5 - 2^130
        uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= 0x3ffffff;
        uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffff;
        uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffff;
        uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffff;
        uint32_t g4 = h4 + c - (1u << 26);
        uint32_t sel = (g4 >> 31) - 1;  // all ones if h >= p
        h0 = (h0 & ~sel) | (g0 & sel); h1 = (h1 & ~sel) | (g1 & sel); h2 = (h2 & ~sel) | (g2 & sel);
        h3 = (h3 & ~sel) | (g3 & sel); h4 = (h4 & ~sel) | (g4 & sel);
        uint32_t w0 = h0 | (h1 << 26), w1 = (h1 >> 6) | (h2 << 20), w2 = (h2 >> 12) | (h3 << 14), w3 = (h3 >> 18) | (h4 << 8);
        uint64_t f = (uint64_t)w0 + s0w; w0 = (uint32_t)f;
        f = (uint64_t)w1 + s1w + (f >> 32); w1 = (uint32_t)f;
        f = (uint64_t)w2 + s2w + (f >> 32); w2 = (uint32_t)f;
        f = (uint64_t)w3 + s3w + (f >> 32); w3 = (uint32_t)f;
        return make_uint4(w0, w1, w2, w3);
    }
};

__device__ __forceinline__ void apply_mask(uint8_t *base, uint32_t hdr_len, uint32_t pn_len, uint32_t m0, uint32_t m1,
                                           uint8_t *mask_out, uint32_t flags) {
    if (flags & QPP_HP_MASK_OUT) {
        mask_out[0] = (uint8_t)m0; mask_out[1] = (uint8_t)(m0 >> 8); mask_out[2] = (uint8_t)(m0 >> 16);
        mask_out[3] = (uint8_t)(m0 >> 24); mask_out[4] = (uint8_t)m1;
    }
    if (flags & QPP_HP_APPLY) hdr_apply(base, hdr_len, pn_len, hdr_load(base, hdr_len), m0, m1);  // header_crypto.rs:80-95
}

// One lane per packet, software-pipelined over 64-byte chunks: the keystream of chunk c+1 is computed in the same
// basic block as the Poly1305 steps of chunk c (independent chains).  The payload moves through a per-wave LDS stage
// that holds a PAIR of chunks (128 B per packet): every other chunk, 8 wave instructions load the next pair as 8
// packets x 128 contiguous bytes each (into registers, a pair ahead), and 8 more store the finished pair the same
// way; the owner lane reads its 16-B blocks from the stage and writes its output blocks back in place.  The kernel is
// bound by this payload I/O (1 Mi x 1200 B seal: 1.10 ms with 64-B chunks both ways, 0.71 ms with the loads and
// stores cut out, 1.09 ms with the ChaCha20 or the Poly1305 work cut out instead; 0.96 ms with 128-B stores), and
// 128-B chunks both ways are what the copy ubench showed cheapest (tools/ubench/copy_pattern.hip: in-place copy
// 1.09 ms with 64-B chunks, 0.86-0.92 with 128-B stores, 0.75-0.79 with 128-B loads and stores).
// Stage slot of packet p's block j of the pair: 64 (p / 8) + 8 (p % 8) + ((j + p + (p >> 4)) % 8).  A lane-linear
// access (slot 64 i + l) is packet 8 i + l / 8, so 8 lanes cover one packet's 128 contiguous bytes; the owner's
// ds_write_b128 (8-lane groups) and ds_read_b128 (16-lane groups) hit distinct bank quads.
// Per-wave LDS: pair stage 8 KiB | (payload offset, length) of the wave's 64 packets.
constexpr uint32_t kChachaStage = 64u * 16u * 8u;
constexpr uint32_t kChachaWaveLds = kChachaStage + 64u * 8u;
__device__ __forceinline__ uint32_t chacha_rho(uint32_t p) { return (p + (p >> 4)) & 7u; }

// RX (open only): the fused receive path for a context with no live AES record -- each lane first unprotects its
// packet of rx[] (rx_unprotect_one: HP removal, PN expansion, key phase; ChaCha20 header keys only), writes the
// qpp_pkt to descs_out and opens it with the key the phase picked.  Same outputs as unprotect_kernel + this kernel.
// Selection mode (sel != nullptr, open only): the packets are descs[sel[sel_meta[1] + i]], i < min(n, sel_meta[0]) --
// the ChaCha20 packets the fused receive kernel (quad.hip) sorted behind its AES packets, their count on the device.
template <bool SEAL, bool RX = false>
__global__ __launch_bounds__(256, 3) void chacha_kernel(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                    const qpp_pkt *__restrict__ descs, uint32_t n,
                                                    uint8_t *__restrict__ arena, uint8_t *masks, int8_t *status,
                                                    uint32_t flags, const qpp_rx_pkt *__restrict__ rx = nullptr,
                                                    qpp_pkt *__restrict__ descs_out = nullptr,
                                                    const uint32_t *__restrict__ sel = nullptr,
                                                    const uint32_t *__restrict__ sel_meta = nullptr) {
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t pi = slot;  // the packet (descriptor, status and mask index)
    if (sel) {
        const uint32_t cnt = min(n, sel_meta[0]);
        if (blockIdx.x * blockDim.x >= cnt) return;  // (workgroup-uniform: the grid is sized for n)
        n = cnt;
        pi = slot < cnt ? sel[sel_meta[1] + slot] : 0u;
    }
    const bool valid = slot < n;
    qpp_pkt d;
    if constexpr (RX) {
        static_assert(!SEAL, "the receive path opens");
        if (valid) {
            d = rx_unprotect_one<false>(AesLds{0}, keys, key_cap, rx[pi], arena, status, pi);
            descs_out[pi] = d;
        } else {
            d = qpp_pkt{};
            d.flags = QPP_PKT_SKIP;  // helper lane
        }
    } else {
        d = valid ? descs[pi] : sel ? descs[sel[sel_meta[1]]] : descs[n - 1];  // (any valid descriptor for helper lanes)
    }
    const bool bad_slot = d.key_idx >= key_cap;    // never dereferenced: the packet is refused
    const DevKey *__restrict__ key = keys + (bad_slot ? 0u : d.key_idx);
    // a slot outside the table, a freed slot or a header-key-only slot holds no packet key: refused (no AES kernel
    // takes such a packet either: the plan gives it no work item with a round count)
    const bool refused = bad_slot || key->live != 1;
    if (refused && valid && status && !(d.flags & QPP_PKT_SKIP)) status[pi] = QPP_INTERNAL_ERROR;
    const bool has = valid && !refused && key->suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256 &&
                     !(d.flags & QPP_PKT_SKIP);
    if (!__any(has)) return;  // wave-uniform: AES packets go to the AES kernels
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t stage = (threadIdx.x >> 6) * kChachaWaveLds, tab = stage + kChachaStage;
    uint32_t k[8];
#pragma unroll
    for (int i = 0; i < 8; i++) k[i] = key->rk[i];
    // Iv::nonce (src/iv.rs:27-39)
    const uint32_t n0 = key->iv[0], n1 = key->iv[1] ^ bswap32((uint32_t)(d.pn >> 32)), n2 = key->iv[2] ^ bswap32((uint32_t)d.pn);
    uint8_t *base = arena + d.off;
    const uint32_t aad_len = d.aad_len, len = has ? d.pt_len : 0;
    uint8_t *pay = base + aad_len;

    uint32_t ks[16];
    chacha_block(k, 0, n0, n1, n2, ks);  // one-time Poly1305 key
    Poly1305 mac;
    mac.init(ks[0], ks[1], ks[2], ks[3]);
    const uint32_t sw0 = ks[4], sw1 = ks[5], sw2 = ks[6], sw3 = ks[7];
    if (has)
        for (uint32_t off = 0; off < aad_len; off += 16) {
            uint4 a = ld16(base + off);
            if (aad_len - off < 16) a = keep_bytes(a, aad_len - off);
            mac.block(a);
        }
    const uint32_t nch = (len + 63) / 64;  // chunks, the partial tail included
    const uint32_t C = wave_max(nch);
    lds_st64(tab + 8u * lane, make_uint2((uint32_t)(pay - arena), len));
    wave_lds_sync();
    // lane-linear role in pair instruction i: packet 8 i + lane / 8, block j of the pair
    // (lj(i) + rho(p)) % 8 = lane % 8, rho(p) = (lane / 8 + i / 2) % 8
    auto lj = [&](int i) { return ((lane & 7u) - (lane / 8u + (uint32_t)(i >> 1))) & 7u; };
    auto own_slot = [&](uint32_t j) {
        return stage + 16u * (64u * (lane / 8u) + 8u * (lane % 8u) + ((j + chacha_rho(lane)) & 7u));
    };
    // Interior pairs (wave-uniform test): all 8 blocks of pair m are whole payload blocks of every packet of the wave,
    // so the pair moves without clamps or predicated stores (as the AES kernels' interior groups)
    const uint32_t min_full = __builtin_amdgcn_readfirstlane(wave_min(has ? (len >> 4) : 0u));
    auto inner_pair = [&](uint32_t m) { return 8u * m + 8u <= min_full; };
    // pair m = blocks 8 m .. 8 m + 7, clamped inside payload||tag (unused when out of range)
    auto pair_load = [&](uint32_t m, uint4 (&r)[8]) {
        if (inner_pair(m)) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const uint32_t ox = lds_ld32(tab + 8u * (8u * i + lane / 8u));
                r[i] = ld16(arena + ox + 16u * (8u * m + lj(i)));
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint2 ol = lds_ld64(tab + 8u * (8u * i + lane / 8u));
            const uint32_t o = 16u * (8u * m + lj(i));
            r[i] = ld16(arena + ol.x + (o < ol.y ? o : 0u));
        }
    };
    auto pair_store = [&](uint32_t m) {  // the full blocks of pair m of the wave's 64 packets
        if (inner_pair(m)) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const uint4 v = lds_ld128(stage + 16u * (64u * i + lane));
                const uint32_t ox = lds_ld32(tab + 8u * (8u * i + lane / 8u));
                st16_nt(arena + ox + 16u * (8u * m + lj(i)), v);
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint4 v = lds_ld128(stage + 16u * (64u * i + lane));
            const uint2 ol = lds_ld64(tab + 8u * (8u * i + lane / 8u));
            const uint32_t o = 16u * (8u * m + lj(i));
            if (o + 16 <= ol.y) st16_nt(arena + ol.x + o, v);
        }
    };
    uint4 rin[8], cb[4];
    pair_load(0, rin);
    chacha_block(k, 1, n0, n1, n2, ks);
    for (uint32_t c = 0; c < C; c++) {
        if (!(c & 1u)) {  // pair top: the pair's inputs into the stage, the next pair's loads issued
#pragma unroll
            for (int i = 0; i < 8; i++) lds_st128(stage + 16u * (64u * i + lane), rin[i]);
            pair_load((c >> 1) + 1, rin);
            wave_lds_sync();
        }
        uint4 in[4];
#pragma unroll
        for (int q = 0; q < 4; q++) in[q] = lds_ld128(own_slot(4u * (c & 1u) + q));
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t o = 64 * c + 16 * q;
            uint4 out = in[q] ^ make_uint4(ks[4 * q], ks[4 * q + 1], ks[4 * q + 2], ks[4 * q + 3]);
            lds_st128(own_slot(4u * (c & 1u) + q), out);  // full blocks leave through the pair store
            cb[q] = SEAL ? out : in[q];
            if (!inner_pair(c >> 1) && o < len && len - o < 16) {  // the partial last block: this lane stores its bytes
                const uint32_t r = len - o;
                out = keep_bytes(out, r);
                st_bytes(pay + o, out, r);
                cb[q] = SEAL ? out : keep_bytes(in[q], r);
            }
        }
        if ((c & 1u) || c + 1 == C) {
            wave_lds_sync();
            pair_store(c >> 1);
            wave_lds_sync();  // the next pair's inputs overwrite the stage
        }
        chacha_block(k, c + 2, n0, n1, n2, ks);  // next chunk ...
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (inner_pair(c >> 1) || 64 * c + 16 * q < len) mac.block(cb[q]);  // ... beside this chunk's MAC
    }
    if (!has) return;
    mac.block(make_uint4(aad_len, 0, len, 0));  // le64(aad_len) || le64(ct_len)
    const uint4 tag = mac.finish(sw0, sw1, sw2, sw3);

    if (SEAL) {
        st16(pay + len, tag);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // other lanes stored this packet's ciphertext
        int8_t st8 = QPP_OK;
        if (flags & (QPP_HP_MASK_OUT | QPP_HP_APPLY)) {
            const uint32_t s = 4 - d.pn_len;
            if (d.pn_len < 1 || d.pn_len > 4 || len < s) {
                st8 = QPP_DECODE_ERROR;
            } else {
                const uint4 smp = ld16(pay + s);
                uint32_t hk[8];
#pragma unroll
                for (int i = 0; i < 8; i++) hk[i] = key->hp_rk[i];
                uint32_t m1, m0 = chacha_hp_word(hk, smp, &m1);
                apply_mask(base, aad_len - d.pn_len, d.pn_len, m0, m1, masks + 5 * (size_t)pi, flags);
            }
        }
        if (status) status[pi] = st8;
    } else {
        const uint4 diff = tag ^ ld16(pay + len);
        const bool ok = (diff.x | diff.y | diff.z | diff.w) == 0;
        if (!ok) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            for (uint32_t o = 0; o < len; o += 16) {
                if (len - o >= 16) st16(pay + o, make_uint4(0, 0, 0, 0));
                else st_bytes(pay + o, make_uint4(0, 0, 0, 0), len - o);
            }
        }
        status[pi] = ok ? QPP_OK : QPP_DECRYPT_ERROR;
    }
}

// ---------------------------------------------------------------- small batches: one WAVE per packet
// The burst form of chacha_kernel (the AES twin is burst.hip): the 64 lanes of a wave split one packet.  Lane l
// takes the MAC-stream blocks j = l, l + 64, ... of the zero-front-padded stream (AAD, ciphertext, lengths), so
//   tag_pre = sum_j X'_j r^(64K - j) = r * sum_l acc_l r^(63 - l),   acc_l = Horner over the lane's blocks in r^64,
// and the lanes are summed by a 6-level tree (level t multiplies the left half by r^(2^t)).  The powers r^(2^t)
// are six squarings of the packet's own r (every lane computes them; no tables).  A ciphertext block's keystream is
// the 16-byte quarter of its ChaCha20 block (counter 1 + b/4) that the lane computes itself.

struct P130 {  // element mod 2^130 - 5, 5 x 26-bit limbs (partially reduced, as Poly1305::block leaves them)
    uint32_t l0, l1, l2, l3, l4;
};
__device__ __forceinline__ P130 p_block(uint4 m, uint32_t hibit) {
    return P130{m.x & 0x3ffffff, ((m.x >> 26) | (m.y << 6)) & 0x3ffffff, ((m.y >> 20) | (m.z << 12)) & 0x3ffffff,
                ((m.z >> 14) | (m.w << 18)) & 0x3ffffff, (m.w >> 8) | hibit};
}
__device__ __forceinline__ P130 p_add(P130 a, P130 b) {
    return P130{a.l0 + b.l0, a.l1 + b.l1, a.l2 + b.l2, a.l3 + b.l3, a.l4 + b.l4};
}
// a * b mod p for general operands: limbs of a < 2^29 (a tree level adds up to 7 reduced values), limbs of b
// < 2^26 + 2^11 (a reduced power of r; unlike the clamped r itself its top limb bits are not cleared), so the
// column sums reach 2^60 and every carry is kept in 64 bits (a 32-bit carry, as Poly1305::block may use with the
// clamped r, truncates here: found by the ragged-batch parity test).
__device__ __forceinline__ P130 p_mul(P130 a, P130 b) {
    const uint32_t s1 = b.l1 * 5, s2 = b.l2 * 5, s3 = b.l3 * 5, s4 = b.l4 * 5;
    uint64_t d0 = (uint64_t)a.l0 * b.l0 + (uint64_t)a.l1 * s4 + (uint64_t)a.l2 * s3 + (uint64_t)a.l3 * s2 + (uint64_t)a.l4 * s1;
    uint64_t d1 = (uint64_t)a.l0 * b.l1 + (uint64_t)a.l1 * b.l0 + (uint64_t)a.l2 * s4 + (uint64_t)a.l3 * s3 + (uint64_t)a.l4 * s2;
    uint64_t d2 = (uint64_t)a.l0 * b.l2 + (uint64_t)a.l1 * b.l1 + (uint64_t)a.l2 * b.l0 + (uint64_t)a.l3 * s4 + (uint64_t)a.l4 * s3;
    uint64_t d3 = (uint64_t)a.l0 * b.l3 + (uint64_t)a.l1 * b.l2 + (uint64_t)a.l2 * b.l1 + (uint64_t)a.l3 * b.l0 + (uint64_t)a.l4 * s4;
    uint64_t d4 = (uint64_t)a.l0 * b.l4 + (uint64_t)a.l1 * b.l3 + (uint64_t)a.l2 * b.l2 + (uint64_t)a.l3 * b.l1 + (uint64_t)a.l4 * b.l0;
    P130 h;
    uint64_t c;
    c = d0 >> 26; h.l0 = (uint32_t)d0 & 0x3ffffff;
    d1 += c; c = d1 >> 26; h.l1 = (uint32_t)d1 & 0x3ffffff;
    d2 += c; c = d2 >> 26; h.l2 = (uint32_t)d2 & 0x3ffffff;
    d3 += c; c = d3 >> 26; h.l3 = (uint32_t)d3 & 0x3ffffff;
    d4 += c; c = d4 >> 26; h.l4 = (uint32_t)d4 & 0x3ffffff;
    const uint64_t t = (uint64_t)h.l0 + c * 5;  // c < 2^35
    h.l0 = (uint32_t)t & 0x3ffffff;
    h.l1 += (uint32_t)(t >> 26);
    return h;
}
__device__ __forceinline__ P130 p_shfl_down(P130 v, unsigned d) {
    return P130{(uint32_t)__shfl_down((int)v.l0, d, 64), (uint32_t)__shfl_down((int)v.l1, d, 64),
                (uint32_t)__shfl_down((int)v.l2, d, 64), (uint32_t)__shfl_down((int)v.l3, d, 64),
                (uint32_t)__shfl_down((int)v.l4, d, 64)};
}
__device__ __forceinline__ uint4 shfl4(uint4 v, int src) {
    return make_uint4((uint32_t)__shfl((int)v.x, src, 64), (uint32_t)__shfl((int)v.y, src, 64),
                      (uint32_t)__shfl((int)v.z, src, 64), (uint32_t)__shfl((int)v.w, src, 64));
}
__device__ __forceinline__ uint32_t byte_of(uint4 v, uint32_t i) {  // byte i (< 16) of v
    const uint32_t w = i < 4 ? v.x : i < 8 ? v.y : i < 12 ? v.z : v.w;
    return (w >> (8 * (i & 3))) & 0xffu;
}

template <bool SEAL>
__global__ __launch_bounds__(256) void chacha_burst_kernel(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                          const qpp_pkt *__restrict__ descs, uint32_t n,
                                                          uint8_t *__restrict__ arena, uint8_t *masks, int8_t *status,
                                                          uint32_t flags) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t pi = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (pi >= n) return;
    const qpp_pkt d = descs[pi];
    if (d.key_idx >= key_cap) {  // wave-uniform: a slot outside the table is refused, never dereferenced
        if (status && lane == 0 && !(d.flags & QPP_PKT_SKIP)) status[pi] = QPP_INTERNAL_ERROR;
        return;
    }
    const DevKey *__restrict__ key = keys + d.key_idx;
    if (key->live != 1) {  // freed or header-key-only slot: refused
        if (status && lane == 0 && !(d.flags & QPP_PKT_SKIP)) status[pi] = QPP_INTERNAL_ERROR;
        return;
    }
    if (key->suite != QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256 || (d.flags & QPP_PKT_SKIP)) return;  // wave-uniform
    uint32_t k[8];
#pragma unroll
    for (int i = 0; i < 8; i++) k[i] = key->rk[i];
    const uint32_t n0 = key->iv[0], n1 = key->iv[1] ^ bswap32((uint32_t)(d.pn >> 32)), n2 = key->iv[2] ^ bswap32((uint32_t)d.pn);
    uint8_t *base = arena + d.off;
    const uint32_t aad_len = d.aad_len, len = d.pt_len;
    uint8_t *pay = base + aad_len;

    const uint32_t a = (aad_len + 15u) >> 4, c = (len + 15u) >> 4, m = a + c + 1;
    const uint32_t K = (m + 63u) >> 6, pad = 64u * K - m;
    P130 acc{0, 0, 0, 0, 0};
    uint4 ct0 = make_uint4(0, 0, 0, 0), ct1 = ct0;  // ciphertext blocks 0/1 where this lane owns them (HP sample)
    uint4 pk0 = ct0, pk1 = ct0;                       // the one-time Poly1305 key (r, s), in lane pad - 1
    P130 rp[7];                                       // r^(2^t), from pass 1 on (pass 0 needs no power of r)
    for (uint32_t kk = 0; kk < K; kk++) {
        const int i = (int)(lane + 64u * kk) - (int)pad;
        const bool data = i >= (int)a && i < (int)(a + c);
        const bool key0 = kk == 0 && i == -1;  // ChaCha block 0 (the Poly1305 key) rides in an idle lane of pass 0
        const uint32_t b = (uint32_t)i - a;
        uint4 in = make_uint4(0, 0, 0, 0);
        uint32_t ks[16];
        if (data || key0) {
            if (data) in = ld16(pay + 16u * b);
            chacha_block(k, data ? 1u + (b >> 2) : 0u, n0, n1, n2, ks);
        }
        if (key0) {
            pk0 = make_uint4(ks[0], ks[1], ks[2], ks[3]);
            pk1 = make_uint4(ks[4], ks[5], ks[6], ks[7]);
        }
        uint4 x = make_uint4(0, 0, 0, 0);
        uint32_t hib = 1u << 24;  // the 2^128 bit of every (padded, full) MAC block
        if (i < 0) {
            hib = 0;  // front padding: a zero term
        } else if (i < (int)a) {
            const uint32_t off = 16u * (uint32_t)i;
            x = ld16(base + off);
            if (aad_len - off < 16u) x = keep_bytes(x, aad_len - off);
        } else if (data) {
            const uint32_t r = len - 16u * b, q = b & 3u;
            const uint4 kq = make_uint4(q == 0 ? ks[0] : q == 1 ? ks[4] : q == 2 ? ks[8] : ks[12],
                                        q == 0 ? ks[1] : q == 1 ? ks[5] : q == 2 ? ks[9] : ks[13],
                                        q == 0 ? ks[2] : q == 1 ? ks[6] : q == 2 ? ks[10] : ks[14],
                                        q == 0 ? ks[3] : q == 1 ? ks[7] : q == 2 ? ks[11] : ks[15]);
            uint4 out = in ^ kq;
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
        } else {
            x = make_uint4(aad_len, 0, len, 0);  // le64(aad_len) || le64(ct_len)
        }
        const P130 xb = p_block(x, hib);
        if (kk == 0) {
            acc = xb;
            // Poly1305 key to every lane (pad == 0: no idle lane in pass 0, so every lane computes block 0)
            if (pad) {
                pk0 = shfl4(pk0, (int)pad - 1);
                pk1 = shfl4(pk1, (int)pad - 1);
            } else {
                chacha_block(k, 0, n0, n1, n2, ks);
                pk0 = make_uint4(ks[0], ks[1], ks[2], ks[3]);
                pk1 = make_uint4(ks[4], ks[5], ks[6], ks[7]);
            }
            Poly1305 key_r;
            key_r.init(pk0.x, pk0.y, pk0.z, pk0.w);
            rp[0] = P130{key_r.r0, key_r.r1, key_r.r2, key_r.r3, key_r.r4};
#pragma unroll
            for (int t = 1; t < 7; t++) rp[t] = p_mul(rp[t - 1], rp[t - 1]);
        } else {
            acc = p_add(p_mul(acc, rp[6]), xb);
        }
    }
    const uint32_t sw0 = pk1.x, sw1 = pk1.y, sw2 = pk1.z, sw3 = pk1.w;
#pragma unroll
    for (int t = 0; t < 6; t++) acc = p_add(p_mul(acc, rp[t]), p_shfl_down(acc, 1u << t));
    const P130 y = p_mul(acc, rp[0]);
    Poly1305 fin;
    fin.h0 = y.l0; fin.h1 = y.l1; fin.h2 = y.l2; fin.h3 = y.l3; fin.h4 = y.l4;
    const uint4 tag = shfl4(fin.finish(sw0, sw1, sw2, sw3), 0);  // lane 0 holds the sum

    if (SEAL) {
        if (lane == 0) st16(pay + len, tag);
        int8_t st8 = QPP_OK;
        if (flags & (QPP_HP_MASK_OUT | QPP_HP_APPLY)) {
            const uint32_t s = 4u - d.pn_len;
            if (d.pn_len < 1 || d.pn_len > 4 || len < s) {
                st8 = QPP_DECODE_ERROR;
            } else {
                const uint32_t o0 = (pad + a) & 63u;
                const uint4 c0 = shfl4(ct0, (int)o0), c1 = shfl4(ct1, (int)((o0 + 1u) & 63u));
                uint4 smp;
                if (len >= s + 16u) {  // sample = (ciphertext || tag)[s, s + 16) from ciphertext blocks 0 and 1
                    smp = make_uint4(__builtin_amdgcn_alignbyte(c0.y, c0.x, s), __builtin_amdgcn_alignbyte(c0.z, c0.y, s),
                                     __builtin_amdgcn_alignbyte(c0.w, c0.z, s), __builtin_amdgcn_alignbyte(c1.x, c0.w, s));
                } else {
                    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
                    for (uint32_t q = 0; q < 16; q++) {
                        const uint32_t pos = s + q;
                        const uint32_t v = pos < len ? (pos < 16u ? byte_of(c0, pos) : byte_of(c1, pos - 16u))
                                                     : byte_of(tag, pos - len);
                        w[q >> 2] |= v << (8 * (q & 3));
                    }
                    smp = make_uint4(w[0], w[1], w[2], w[3]);
                }
                uint32_t hk[8];
#pragma unroll
                for (int i = 0; i < 8; i++) hk[i] = key->hp_rk[i];
                uint32_t m1, m0 = chacha_hp_word(hk, smp, &m1);
                if (lane == 0) apply_mask(base, aad_len - d.pn_len, d.pn_len, m0, m1, masks + 5 * (size_t)pi, flags);
            }
        }
        if (status && lane == 0) status[pi] = st8;
    } else {
        const uint4 diff = tag ^ ld16(pay + len);
        const bool ok = (diff.x | diff.y | diff.z | diff.w) == 0;
        if (!ok) {  // each lane zeroes the plaintext blocks it wrote (same-lane order)
            for (uint32_t kk = 0; kk < K; kk++) {
                const int i = (int)(lane + 64u * kk) - (int)pad;
                if (i >= (int)a && i < (int)(a + c)) {
                    const uint32_t b = (uint32_t)i - a, r = len - 16u * b;
                    if (r >= 16u) st16(pay + 16u * b, make_uint4(0, 0, 0, 0));
                    else st_bytes(pay + 16u * b, make_uint4(0, 0, 0, 0), r);
                }
            }
        }
        if (lane == 0) status[pi] = ok ? QPP_OK : QPP_DECRYPT_ERROR;
    }
}

// Header-protection masks for any suite, one lane per packet; AES keys use the LDS T-tables with the
// lane's own round keys.  Sample at off + aad_len - pn_len + 4.
__global__ __launch_bounds__(1024) void hp_mask_kernel(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                      const qpp_pkt *__restrict__ descs, uint32_t n,
                                                      const uint8_t *__restrict__ arena, uint8_t *masks) {
    // 64 KiB of dynamic LDS (the launch reserves it), addressed by offset through lds_ld32/lds_st32
    build_aes_tables(0);
    __syncthreads();
    const uint32_t pi = blockIdx.x * blockDim.x + threadIdx.x;
    if (pi >= n) return;
    const qpp_pkt d = descs[pi];
    uint8_t *o = masks + 5 * (size_t)pi;
    if (d.key_idx >= key_cap) {  // no key: an all-zero mask (the caller's descriptor is wrong)
        o[0] = o[1] = o[2] = o[3] = o[4] = 0;
        return;
    }
    const DevKey *__restrict__ key = keys + d.key_idx;
    const uint4 smp = ld16(arena + d.off + d.aad_len - d.pn_len + 4);
    uint32_t m0, m1;
    if (key->suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256) {
        uint32_t hk[8];
#pragma unroll
        for (int i = 0; i < 8; i++) hk[i] = key->hp_rk[i];
        m0 = chacha_hp_word(hk, smp, &m1);
    } else {
        const AesLds aes = make_aes(0);
        uint4 m = key->hp_nr == 10 ? aes.encrypt<10>(smp, key->hp_rk) : aes.encrypt<14>(smp, key->hp_rk);
        m0 = m.x; m1 = m.y;
    }
    o[0] = (uint8_t)m0; o[1] = (uint8_t)(m0 >> 8); o[2] = (uint8_t)(m0 >> 16); o[3] = (uint8_t)(m0 >> 24); o[4] = (uint8_t)m1;
}

// Receive-side header unprotection for a GRO batch, one lane per packet:
//   sample at header_len + 4 (payload.rs:151-169) -> mask (header_key.rs:52-56) -> remove_header_protection in place
//   (header_crypto.rs:98-123: first byte, pn_len = (b0 & 3) + 1, PN bytes) -> expand the PN against the space's
//   largest acknowledged PN (packet/number/mod.rs:191-238) -> the packet key by the key-phase bit 0x04
//   (key_phase.rs:12,46; KeySet::decrypt_packet, keyset.rs:113-143; long headers: key_idx[0]) -> the qpp_pkt the
//   open kernels consume.  A packet too short for the sample is DECODE_ERROR and marked QPP_PKT_SKIP; a packet whose
//   chosen key is not a live packet key is INTERNAL_ERROR here already (no open kernel takes it, whatever the batch's
//   QPP_ONLY_* flags; the fused receive kernel decides the same in its phase A).
__global__ __launch_bounds__(1024) void unprotect_kernel(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                        const qpp_rx_pkt *__restrict__ rx, uint32_t n,
                                                        uint8_t *__restrict__ arena, qpp_pkt *descs_out,
                                                        int8_t *status) {
    // 64 KiB of dynamic LDS: the AES T-tables for the AES header keys
    build_aes_tables(0);
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint4 kw;
    const qpp_pkt d = rx_unprotect_one(make_aes(0), keys, key_cap, rx[i], arena, status, i, &kw);
    if (!(d.flags & QPP_PKT_SKIP) && kw.w != 1) status[i] = QPP_INTERNAL_ERROR;
    descs_out[i] = d;
}

}  // namespace

hipError_t launch_unprotect(const DevKey *keys, uint32_t key_cap, const qpp_rx_pkt *rx, uint32_t n, uint8_t *arena,
                            qpp_pkt *descs_out, int8_t *status, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(unprotect_kernel, dim3((n + 1023) / 1024), dim3(1024), 65536, s, keys, key_cap, rx, n, arena,
                       descs_out, status);
    return hipGetLastError();
}

hipError_t launch_chacha(bool seal, const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n,
                         uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags, bool burst, hipStream_t s) {
    if (!n) return hipSuccess;
    if (burst) {  // one wave per packet, 4 per workgroup
        if (seal)
            hipLaunchKernelGGL(chacha_burst_kernel<true>, dim3((n + 3) / 4), dim3(256), 0, s, keys, key_cap, descs, n, arena,
                               masks, status, flags);
        else
            hipLaunchKernelGGL(chacha_burst_kernel<false>, dim3((n + 3) / 4), dim3(256), 0, s, keys, key_cap, descs, n, arena,
                               masks, status, flags);
        return hipGetLastError();
    }
    const dim3 grid((n + 255) / 256), block(256);
    const uint32_t lds = 4u * kChachaWaveLds;  // 4 waves, 34 KiB
    if (seal)
        hipLaunchKernelGGL(chacha_kernel<true>, grid, block, lds, s, keys, key_cap, descs, n, arena, masks, status, flags,
                           nullptr, nullptr);
    else
        hipLaunchKernelGGL(chacha_kernel<false>, grid, block, lds, s, keys, key_cap, descs, n, arena, masks, status, flags,
                           nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_chacha_sel(const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n_max,
                             uint8_t *arena, int8_t *status, const uint32_t *sel, const uint32_t *sel_meta, hipStream_t s) {
    if (!n_max) return hipSuccess;
    const dim3 grid((n_max + 255) / 256), block(256);
    const uint32_t lds = 4u * kChachaWaveLds;
    hipLaunchKernelGGL((chacha_kernel<false, false>), grid, block, lds, s, keys, key_cap, descs, n_max, arena, nullptr,
                       status, 0u, nullptr, nullptr, sel, sel_meta);
    return hipGetLastError();
}

hipError_t launch_chacha_rx(const DevKey *keys, uint32_t key_cap, const qpp_rx_pkt *rx, uint32_t n, uint8_t *arena,
                            qpp_pkt *descs_out, int8_t *status, hipStream_t s) {
    if (!n) return hipSuccess;
    const dim3 grid((n + 255) / 256), block(256);
    const uint32_t lds = 4u * kChachaWaveLds;
    hipLaunchKernelGGL((chacha_kernel<false, true>), grid, block, lds, s, keys, key_cap, nullptr, n, arena, nullptr,
                       status, 0u, rx, descs_out);
    return hipGetLastError();
}

hipError_t launch_hp_mask(const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n,
                          const uint8_t *arena, uint8_t *masks, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hp_mask_kernel, dim3((n + 1023) / 1024), dim3(1024), 65536, s, keys, key_cap, descs, n,
                       arena, masks);
    return hipGetLastError();
}

}  // namespace qpp
