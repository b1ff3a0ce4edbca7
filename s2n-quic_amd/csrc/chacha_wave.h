// chacha_wave.h — ChaCha20-Poly1305 building blocks shared by chacha.hip (lane and wave kernels) and burst.hip (the
// persistent transmit-queue server): Poly1305 in 26-bit limbs, the header-protection mask application, and the
// one-WAVE-per-packet seal/open (RFC 8439 AEAD, quic/s2n-quic-crypto/src/cipher_suite.rs:270-284).
#pragma once

#include "device_common.h"

namespace qpp {
namespace dev {

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

// hb: the header bytes hdr_load read (read before any store of the packet by the wave-per-packet code)
__device__ __forceinline__ void apply_mask(uint8_t *base, uint32_t hdr_len, uint32_t pn_len, uint32_t m0, uint32_t m1,
                                           uint8_t *mask_out, uint32_t flags, HdrBytes hb) {
    if (flags & QPP_HP_MASK_OUT) {
        mask_out[0] = (uint8_t)m0; mask_out[1] = (uint8_t)(m0 >> 8); mask_out[2] = (uint8_t)(m0 >> 16);
        mask_out[3] = (uint8_t)(m0 >> 24); mask_out[4] = (uint8_t)m1;
    }
    if (flags & QPP_HP_APPLY) hdr_apply(base, hdr_len, pn_len, hb, m0, m1);  // header_crypto.rs:80-95
}
__device__ __forceinline__ void apply_mask(uint8_t *base, uint32_t hdr_len, uint32_t pn_len, uint32_t m0, uint32_t m1,
                                           uint8_t *mask_out, uint32_t flags) {
    apply_mask(base, hdr_len, pn_len, m0, m1, mask_out, flags,
               (flags & QPP_HP_APPLY) ? hdr_load(base, hdr_len) : HdrBytes{0, 0});
}

// ---------------------------------------------------------------- one WAVE per packet
// The 64 lanes of a wave split one packet.  Lane l takes the MAC-stream blocks j = l, l + 64, ... of the
// zero-front-padded stream (AAD, ciphertext, lengths), so
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

// quad_perm DPP: lane l reads lane 4 (l / 4) + sel[l % 4]
template <int CTRL>
__device__ __forceinline__ uint32_t cq_perm(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
// The ChaCha20 block of the header-protection key (header_key.rs:52-56: counter = sample[0..4], nonce =
// sample[4..16]; RFC 9001 §5.4.4) split over the 4 lanes of a quad: lane s holds column s (words s, 4 + s, 8 + s,
// 12 + s), a column round is one quarter-round per lane, and a diagonal round one quarter-round on (a_s, b_s+1,
// c_s+2, d_s+3) with those words moved in and back out by DPP -- a quarter of a whole block's VALU per lane (the
// block is on the latency chain of every sealed packet of the wave-per-packet code).  Every lane of every quad must
// be active.  Returns mask word 0 (bytes 0..3) and *w1 = word 1 (byte 4), in every lane.
__device__ __forceinline__ uint32_t chacha_hp_quad(const uint32_t hk[8], uint4 smp, uint32_t s, uint32_t *w1) {
    constexpr uint32_t k0 = 0x61707865u, k1 = 0x3320646eu, k2 = 0x79622d32u, k3 = 0x6b206574u;
    const uint32_t a0 = s == 0 ? k0 : s == 1 ? k1 : s == 2 ? k2 : k3;
    const uint32_t b0 = s == 0 ? hk[0] : s == 1 ? hk[1] : s == 2 ? hk[2] : hk[3];
    const uint32_t c0 = s == 0 ? hk[4] : s == 1 ? hk[5] : s == 2 ? hk[6] : hk[7];
    const uint32_t d0 = s == 0 ? smp.x : s == 1 ? smp.y : s == 2 ? smp.z : smp.w;
    uint32_t a = a0, b = b0, c = c0, d = d0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        QR(a, b, c, d);  // column round
        b = cq_perm<0x39>(b); c = cq_perm<0x4e>(c); d = cq_perm<0x93>(d);  // (a_s, b_s+1, c_s+2, d_s+3)
        QR(a, b, c, d);  // diagonal round
        b = cq_perm<0x93>(b); c = cq_perm<0x4e>(c); d = cq_perm<0x39>(d);  // back to their columns
    }
    const uint32_t w = a + a0;  // keystream word s
    *w1 = cq_perm<0x55>(w);
    return cq_perm<0x00>(w);
}

// ChaCha20 block cb (equal within a quad) over the 4 lanes of the quad, as chacha_hp_quad: lane s computes column s
// and returns ROW s after a 4 x 4 transpose through DPP -- keystream words 4 s .. 4 s + 3, the 16 bytes of the block's
// quarter s.  Every lane of every quad must be active.
__device__ __forceinline__ uint4 chacha_row_quad(const uint32_t (&k)[8], uint32_t cb, uint32_t n0, uint32_t n1,
                                                 uint32_t n2, uint32_t s) {
    constexpr uint32_t k0 = 0x61707865u, k1 = 0x3320646eu, k2 = 0x79622d32u, k3 = 0x6b206574u;
    const uint32_t a0 = s == 0 ? k0 : s == 1 ? k1 : s == 2 ? k2 : k3;
    const uint32_t b0 = s == 0 ? k[0] : s == 1 ? k[1] : s == 2 ? k[2] : k[3];
    const uint32_t c0 = s == 0 ? k[4] : s == 1 ? k[5] : s == 2 ? k[6] : k[7];
    const uint32_t d0 = s == 0 ? cb : s == 1 ? n0 : s == 2 ? n1 : n2;
    uint32_t a = a0, b = b0, c = c0, d = d0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
        QR(a, b, c, d);
        b = cq_perm<0x39>(b); c = cq_perm<0x4e>(c); d = cq_perm<0x93>(d);
        QR(a, b, c, d);
        b = cq_perm<0x93>(b); c = cq_perm<0x4e>(c); d = cq_perm<0x39>(d);
    }
    const uint32_t w[4] = {a + a0, b + b0, c + c0, d + d0};  // column s, rows 0..3
    // lane s wants row s: word 4 s + t = row s of column t, i.e. register w[s] of lane t.  For a rotation rho, lane t
    // offers w[(t - rho) & 3] and lane s reads lane (s + rho) & 3: it receives word 4 s + ((s + rho) & 3).
    auto pick = [&](uint32_t j) { return j == 0 ? w[0] : j == 1 ? w[1] : j == 2 ? w[2] : w[3]; };
    const uint32_t r0 = pick(s);
    const uint32_t r1 = cq_perm<0x39>(pick((s - 1u) & 3u));
    const uint32_t r2 = cq_perm<0x4e>(pick((s - 2u) & 3u));
    const uint32_t r3 = cq_perm<0x93>(pick((s - 3u) & 3u));
    // component t came with rho = (t - s) & 3
    auto comp = [&](uint32_t t) {
        const uint32_t rho = (t - s) & 3u;
        return rho == 0 ? r0 : rho == 1 ? r1 : rho == 2 ? r2 : r3;
    };
    return make_uint4(comp(0), comp(1), comp(2), comp(3));
}

// One packet, one wave (every lane calls it with the same d).  k: the ChaCha20 key, n0..n2: the packet's nonce words
// (Iv::nonce, iv.rs:27-39), hk: the header-protection key (read only when sealing with an HP flag).  Seal: ciphertext
// and tag in place, HP mask out / applied per flags, *status_out = OK / DECODE_ERROR (no room for the sample).  Open:
// plaintext in place (zeroed on a bad tag, all 16 tag bytes compared), *status_out = OK / DECRYPT_ERROR.  status_out
// and mask_out are written by lane 0 only (status_out may be null when sealing).
// Each lane's block of pass kk + 1 is loaded before pass kk's ChaCha20 block and Poly1305 step: a packet pays one
// memory round trip, not one per pass (the transmit-queue server reads the ring over PCIe).  Nothing is read after
// the first store (stores and loads share one counter: a read after them waits for their PCIe round trip).
template <bool SEAL>
__device__ __forceinline__ void chacha_wave_packet(const uint32_t (&k)[8], uint32_t n0, uint32_t n1, uint32_t n2,
                                                   const uint32_t *hk, const qpp_pkt &d, uint8_t *arena,
                                                   uint8_t *mask_out, int8_t *status_out, uint32_t flags,
                                                   uint32_t lane) {
    uint8_t *base = arena + d.off;
    const uint32_t aad_len = d.aad_len, len = d.pt_len;
    uint8_t *pay = base + aad_len;
    const uint32_t a = (aad_len + 15u) >> 4, c = (len + 15u) >> 4, m = a + c + 1;
    const uint32_t K = (m + 63u) >> 6, pad = 64u * K - m;
    // the lane's input block of pass kk: AAD block (front) or payload block (data), else nothing to read
    auto load = [&](uint32_t kk) {
        const int i = (int)(lane + 64u * kk) - (int)pad;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (i >= 0 && i < (int)a) v = ld16(base + 16u * (uint32_t)i);
        else if (i >= (int)a && i < (int)(a + c)) v = ld16(pay + 16u * ((uint32_t)i - a));
        return v;
    };
    P130 acc{0, 0, 0, 0, 0};
    uint4 ct0 = make_uint4(0, 0, 0, 0), ct1 = ct0;  // ciphertext blocks 0/1 where this lane owns them (HP sample)
    uint4 pk0 = ct0, pk1 = ct0;                       // the one-time Poly1305 key (r, s), in lane pad - 1
    P130 rp[7];                                       // r^(2^t), from pass 1 on (pass 0 needs no power of r)
    uint4 nxt = load(0);
    // Keystream by quads: quad j of pass kk computes ChaCha block 1 + (base_b + 4 j) / 4 split over its four lanes
    // (chacha_row_quad: a quarter of a block's VALU per lane, where every lane computing its own data block's whole
    // ChaCha block did 4x the work -- the 4 lanes of a block computed it 4 times), so lane L holds the keystream of
    // data block base_b + L; the data block of lane l is base_b + l - delta (delta aligns the MAC layout's data blocks
    // to quads), read from lane l - delta, or for l < delta from lane 64 + l - delta of the previous pass.
    const uint32_t delta = (pad + a) & 3u;
    uint4 prev_row = make_uint4(0, 0, 0, 0);
    // the header bytes the HP mask is applied to (seal) / the received tag (open), read with the first blocks
    const bool hdr_want = SEAL && (flags & QPP_HP_APPLY) && d.pn_len >= 1 && d.pn_len <= 4;
    HdrBytes hb{0, 0};
    if (hdr_want && lane == 0) hb = hdr_load(base, aad_len - d.pn_len);
    uint4 want = make_uint4(0, 0, 0, 0);
    if (!SEAL && lane == 0) want = ld16(pay + len);
    for (uint32_t kk = 0; kk < K; kk++) {
        const int i = (int)(lane + 64u * kk) - (int)pad;
        const bool data = i >= (int)a && i < (int)(a + c);
        const uint32_t b = (uint32_t)i - a;
        uint4 in = nxt;
        if (kk + 1 < K) nxt = load(kk + 1);
        const int base_b = 64 * (int)kk - (int)pad - (int)a + (int)delta;  // a multiple of 4
        const int cbq = 1 + (base_b >> 2) + (int)(lane >> 2);
        const uint4 row = chacha_row_quad(k, cbq > 0 ? (uint32_t)cbq : 0u, n0, n1, n2, lane & 3u);
        uint4 kq = row;
        if (delta) {  // (uniform)
            const int src = (int)((lane - delta) & 63u);
            const uint4 cur = shfl4(row, src), prv = shfl4(prev_row, src);
            kq = lane >= delta ? cur : prv;
        }
        prev_row = row;
        if (kk == 0) {  // the Poly1305 key: ChaCha block 0, rows 0 and 1, from the quad that computed it
            const int j0 = -(base_b >> 2) - 1;  // (uniform)
            if (j0 >= 0 && j0 < 16) {
                pk0 = shfl4(row, 4 * j0);
                pk1 = shfl4(row, 4 * j0 + 1);
            } else {
                const uint4 r0 = chacha_row_quad(k, 0u, n0, n1, n2, lane & 3u);
                pk0 = shfl4(r0, 0);
                pk1 = shfl4(r0, 1);
            }
        }
        uint4 x = make_uint4(0, 0, 0, 0);
        uint32_t hib = 1u << 24;  // the 2^128 bit of every (padded, full) MAC block
        if (i < 0) {
            hib = 0;  // front padding: a zero term
        } else if (i < (int)a) {
            const uint32_t off = 16u * (uint32_t)i;
            x = aad_len - off < 16u ? keep_bytes(in, aad_len - off) : in;
        } else if (data) {
            const uint32_t r = len - 16u * b;
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
                uint32_t hkr[8];
#pragma unroll
                for (int i = 0; i < 8; i++) hkr[i] = hk[i];
                uint32_t m1, m0 = chacha_hp_quad(hkr, smp, lane & 3u, &m1);
                if (lane == 0) apply_mask(base, aad_len - d.pn_len, d.pn_len, m0, m1, mask_out, flags, hb);
            }
        }
        if (status_out && lane == 0) *status_out = st8;
    } else {
        const uint4 diff = tag ^ shfl4(want, 0);
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
        if (lane == 0) *status_out = ok ? QPP_OK : QPP_DECRYPT_ERROR;
    }
}

}  // namespace dev
}  // namespace qpp
