/*
 * qpp_oracle.c — plain-C restatement of the QUIC packet-protection path.
 * TEST INFRASTRUCTURE ONLY (see qpp_oracle.h): the checker, never the product.
 *
 * Written for clarity, not speed: byte-oriented AES (FIPS-197), bit-serial GHASH
 * (SP 800-38D Algorithm 1), RFC 8439 ChaCha20 / Poly1305, FIPS 180-4 SHA-2.
 */
#include "qpp_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ AES */

static uint8_t orc_sbox[256];
static int orc_sbox_ready;

static uint8_t gf_mul8(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return p;
}

/* S-box built from its definition (multiplicative inverse + affine map, FIPS-197 §5.1.1)
 * so the oracle does not share a transcribed table with the product. */
static void orc_build_sbox(void) {
    if (orc_sbox_ready) return;
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        if (x) {
            for (int y = 1; y < 256; y++)
                if (gf_mul8((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        }
        uint8_t s = inv, r = inv;
        for (int k = 0; k < 4; k++) {
            r = (uint8_t)((r << 1) | (r >> 7));
            s ^= r;
        }
        orc_sbox[x] = (uint8_t)(s ^ 0x63);
    }
    orc_sbox_ready = 1;
}

int orc_aes_expand(const uint8_t *key, size_t key_len, uint8_t rk[240]) {
    orc_build_sbox();
    int nk = (int)(key_len / 4), rounds = nk + 6;
    int total = 4 * (rounds + 1);
    memcpy(rk, key, key_len);
    uint8_t rcon = 1;
    for (int i = nk; i < total; i++) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % nk == 0) {
            uint8_t t0 = t[0];
            t[0] = (uint8_t)(orc_sbox[t[1]] ^ rcon);
            t[1] = orc_sbox[t[2]];
            t[2] = orc_sbox[t[3]];
            t[3] = orc_sbox[t0];
            rcon = gf_mul8(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            for (int k = 0; k < 4; k++) t[k] = orc_sbox[t[k]];
        }
        for (int k = 0; k < 4; k++) rk[4 * i + k] = (uint8_t)(rk[4 * (i - nk) + k] ^ t[k]);
    }
    return rounds;
}

void orc_aes_encrypt_block(const uint8_t rk[240], int rounds, const uint8_t in[16], uint8_t out[16]) {
    orc_build_sbox();
    uint8_t s[16];
    for (int i = 0; i < 16; i++) s[i] = (uint8_t)(in[i] ^ rk[i]);
    for (int r = 1; r <= rounds; r++) {
        uint8_t t[16];
        /* SubBytes + ShiftRows: state byte (row i, col c) at s[4c+i] */
        for (int c = 0; c < 4; c++)
            for (int i = 0; i < 4; i++) t[4 * c + i] = orc_sbox[s[4 * ((c + i) & 3) + i]];
        if (r != rounds) {
            for (int c = 0; c < 4; c++) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                s[4 * c + 0] = (uint8_t)(gf_mul8(a0, 2) ^ gf_mul8(a1, 3) ^ a2 ^ a3);
                s[4 * c + 1] = (uint8_t)(a0 ^ gf_mul8(a1, 2) ^ gf_mul8(a2, 3) ^ a3);
                s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ gf_mul8(a2, 2) ^ gf_mul8(a3, 3));
                s[4 * c + 3] = (uint8_t)(gf_mul8(a0, 3) ^ a1 ^ a2 ^ gf_mul8(a3, 2));
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; i++) s[i] ^= rk[16 * r + i];
    }
    memcpy(out, s, 16);
}

/* ------------------------------------------------------------------ GCM */

/* SP 800-38D §6.3 Algorithm 1, bit by bit (bit 0 = MSB of byte 0). */
void orc_ghash_mul(uint8_t x[16], const uint8_t h[16]) {
    uint8_t z[16] = {0}, v[16];
    memcpy(v, h, 16);
    for (int i = 0; i < 128; i++) {
        if ((x[i >> 3] >> (7 - (i & 7))) & 1)
            for (int k = 0; k < 16; k++) z[k] ^= v[k];
        int lsb = v[15] & 1;
        for (int k = 15; k > 0; k--) v[k] = (uint8_t)((v[k] >> 1) | (v[k - 1] << 7));
        v[0] >>= 1;
        if (lsb) v[0] ^= 0xe1;
    }
    memcpy(x, z, 16);
}

static void ghash_update(uint8_t y[16], const uint8_t h[16], const uint8_t *data, size_t len) {
    while (len) {
        size_t n = len < 16 ? len : 16;
        for (size_t k = 0; k < n; k++) y[k] ^= data[k];
        orc_ghash_mul(y, h);
        data += n;
        len -= n;
    }
}

static void put_be64(uint8_t *p, uint64_t v) {
    for (int i = 7; i >= 0; i--) { p[i] = (uint8_t)v; v >>= 8; }
}

/* encrypt=1: seal buf in place, tag -> tag_out; encrypt=0: decrypt, computed tag -> tag_out */
static void aes_gcm_core(const uint8_t *key, size_t key_len, const uint8_t nonce[12],
                         const uint8_t *aad, size_t aad_len, uint8_t *buf, size_t len,
                         int encrypt, uint8_t tag_out[16]) {
    uint8_t rk[240], h[16] = {0}, j0[16], ek0[16], y[16] = {0};
    int rounds = orc_aes_expand(key, key_len, rk);
    orc_aes_encrypt_block(rk, rounds, h, h);
    memcpy(j0, nonce, 12);
    j0[12] = 0; j0[13] = 0; j0[14] = 0; j0[15] = 1;
    orc_aes_encrypt_block(rk, rounds, j0, ek0);
    ghash_update(y, h, aad, aad_len);
    uint32_t ctr = 1;
    for (size_t off = 0; off < len; off += 16) {
        uint8_t cb[16], ks[16];
        ctr++;
        memcpy(cb, nonce, 12);
        cb[12] = (uint8_t)(ctr >> 24); cb[13] = (uint8_t)(ctr >> 16);
        cb[14] = (uint8_t)(ctr >> 8);  cb[15] = (uint8_t)ctr;
        orc_aes_encrypt_block(rk, rounds, cb, ks);
        size_t n = len - off < 16 ? len - off : 16;
        if (!encrypt) ghash_update(y, h, buf + off, n);
        for (size_t k = 0; k < n; k++) buf[off + k] ^= ks[k];
        if (encrypt) ghash_update(y, h, buf + off, n);
    }
    uint8_t lens[16];
    put_be64(lens, (uint64_t)aad_len * 8);
    put_be64(lens + 8, (uint64_t)len * 8);
    ghash_update(y, h, lens, 16);
    for (int k = 0; k < 16; k++) tag_out[k] = (uint8_t)(y[k] ^ ek0[k]);
}

/* ------------------------------------------------------- ChaCha20-Poly1305 */

static uint32_t rotl32(uint32_t v, int c) { return (v << c) | (v >> (32 - c)); }
static uint32_t le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

#define QR(a, b, c, d)                                   \
    a += b; d ^= a; d = rotl32(d, 16);                   \
    c += d; b ^= c; b = rotl32(b, 12);                   \
    a += b; d ^= a; d = rotl32(d, 8);                    \
    c += d; b ^= c; b = rotl32(b, 7);

void orc_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], uint8_t out[64]) {
    uint32_t in[16], x[16];
    in[0] = 0x61707865; in[1] = 0x3320646e; in[2] = 0x79622d32; in[3] = 0x6b206574;
    for (int i = 0; i < 8; i++) in[4 + i] = le32(key + 4 * i);
    in[12] = counter;
    for (int i = 0; i < 3; i++) in[13 + i] = le32(nonce + 4 * i);
    memcpy(x, in, sizeof x);
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
    for (int i = 0; i < 16; i++) {
        uint32_t v = x[i] + in[i];
        out[4 * i] = (uint8_t)v; out[4 * i + 1] = (uint8_t)(v >> 8);
        out[4 * i + 2] = (uint8_t)(v >> 16); out[4 * i + 3] = (uint8_t)(v >> 24);
    }
}

/* RFC 8439 §2.5, with exact 130-bit arithmetic in three 64-bit words (__int128 products). */
void orc_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len, uint8_t tag[16]) {
    typedef unsigned __int128 u128;
    uint64_t r0 = ((uint64_t)le32(key) | ((uint64_t)le32(key + 4) << 32)) & 0x0ffffffc0fffffffULL;
    uint64_t r1 = ((uint64_t)le32(key + 8) | ((uint64_t)le32(key + 12) << 32)) & 0x0ffffffc0ffffffcULL;
    uint64_t h0 = 0, h1 = 0, h2 = 0; /* h = h0 + h1*2^64 + h2*2^128 */
    while (len) {
        uint8_t blk[17] = {0};
        size_t n = len < 16 ? len : 16;
        memcpy(blk, msg, n);
        blk[n] = 1;
        uint64_t m0 = (uint64_t)le32(blk) | ((uint64_t)le32(blk + 4) << 32);
        uint64_t m1 = (uint64_t)le32(blk + 8) | ((uint64_t)le32(blk + 12) << 32);
        uint64_t m2 = blk[16];
        u128 t = (u128)h0 + m0; h0 = (uint64_t)t;
        t = (u128)h1 + m1 + (uint64_t)(t >> 64); h1 = (uint64_t)t;
        h2 = h2 + m2 + (uint64_t)(t >> 64);
        /* h * r; r1 has low 2 bits clear and r < 2^124 so the products fit */
        u128 d0 = (u128)h0 * r0;
        u128 d1 = (u128)h0 * r1 + (u128)h1 * r0;
        u128 d2 = (u128)h1 * r1 + (u128)h2 * r0;
        u128 d3 = (u128)h2 * r1;
        /* columns: d0 + d1<<64 + d2<<128 + d3<<192 */
        uint64_t c0 = (uint64_t)d0;
        d1 += (uint64_t)(d0 >> 64);
        uint64_t c1 = (uint64_t)d1;
        d2 += (uint64_t)(d1 >> 64);
        uint64_t c2 = (uint64_t)d2;
        d3 += (uint64_t)(d2 >> 64);
        uint64_t c3 = (uint64_t)d3;
        /* value = c0 + c1 2^64 + c2 2^128 + c3 2^192; reduce mod 2^130-5:
         * low = bits [0,130), high = value >> 130; value ≡ low + 5*high */
        uint64_t l0 = c0, l1 = c1, l2 = c2 & 3;
        uint64_t hh0 = (c2 >> 2) | (c3 << 62), hh1 = c3 >> 2;
        /* 5*high = 4*high + high */
        u128 a = (u128)l0 + hh0 + (hh0 << 2);
        uint64_t carry_hi = hh0 >> 62;
        h0 = (uint64_t)a;
        u128 b = (u128)l1 + hh1 + (hh1 << 2) + carry_hi + (uint64_t)(a >> 64);
        h1 = (uint64_t)b;
        h2 = l2 + (hh1 >> 62) + (uint64_t)(b >> 64);
        msg += n;
        len -= n;
    }
    /* final reduction: compute h - p, select if non-negative */
    u128 t = (u128)h0 + 5;
    uint64_t g0 = (uint64_t)t;
    t = (u128)h1 + (uint64_t)(t >> 64);
    uint64_t g1 = (uint64_t)t;
    uint64_t g2 = h2 + (uint64_t)(t >> 64);
    if (g2 >> 2) { h0 = g0; h1 = g1; } /* h >= p */
    uint64_t s0 = (uint64_t)le32(key + 16) | ((uint64_t)le32(key + 20) << 32);
    uint64_t s1 = (uint64_t)le32(key + 24) | ((uint64_t)le32(key + 28) << 32);
    t = (u128)h0 + s0; h0 = (uint64_t)t;
    h1 = h1 + s1 + (uint64_t)(t >> 64);
    for (int i = 0; i < 8; i++) { tag[i] = (uint8_t)(h0 >> (8 * i)); tag[8 + i] = (uint8_t)(h1 >> (8 * i)); }
}

static void chacha_poly_core(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                             uint8_t *buf, size_t len, int encrypt, uint8_t tag_out[16]) {
    uint8_t blk[64];
    orc_chacha20_block(key, 0, nonce, blk);
    uint8_t otk[32];
    memcpy(otk, blk, 32);
    /* mac data = aad || pad16 || ct || pad16 || le64(aad_len) || le64(ct_len) */
    size_t pa = (16 - aad_len % 16) % 16, pc = (16 - len % 16) % 16;
    size_t mlen = aad_len + pa + len + pc + 16;
    uint8_t stackbuf[4096];
    uint8_t *mac = stackbuf;
    static uint8_t *heap;  /* oracle is single-threaded test code */
    static size_t heap_len;
    if (mlen > sizeof stackbuf) {
        if (heap_len < mlen) {
            heap = (uint8_t *)realloc(heap, mlen);
            heap_len = mlen;
        }
        mac = heap;
    }
    memset(mac, 0, mlen);
    if (aad_len) memcpy(mac, aad, aad_len);  /* (aad / buf may be NULL at length 0) */
    if (!encrypt && len) memcpy(mac + aad_len + pa, buf, len);
    for (size_t off = 0; off < len; off += 64) {
        orc_chacha20_block(key, (uint32_t)(1 + off / 64), nonce, blk);
        size_t n = len - off < 64 ? len - off : 64;
        for (size_t k = 0; k < n; k++) buf[off + k] ^= blk[k];
    }
    if (encrypt && len) memcpy(mac + aad_len + pa, buf, len);
    uint8_t *lens = mac + aad_len + pa + len + pc;
    for (int i = 0; i < 8; i++) {
        lens[i] = (uint8_t)((uint64_t)aad_len >> (8 * i));
        lens[8 + i] = (uint8_t)((uint64_t)len >> (8 * i));
    }
    orc_poly1305(otk, mac, mlen, tag_out);
}

/* ------------------------------------------------------------------ SHA-2 */

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static uint32_t rotr32(uint32_t v, int c) { return (v >> c) | (v << (32 - c)); }

static void sha256_block(uint32_t st[8], const uint8_t *p) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
        uint32_t t1 = h + (rotr32(e, 6) ^ rotr32(e, 11) ^ rotr32(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (rotr32(a, 2) ^ rotr32(a, 13) ^ rotr32(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

void orc_sha256(const uint8_t *msg, size_t len, uint8_t out[32]) {
    uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    size_t full = len / 64;
    for (size_t i = 0; i < full; i++) sha256_block(st, msg + 64 * i);
    uint8_t tail[128] = {0};
    size_t rem = len % 64;
    if (rem) memcpy(tail, msg + 64 * full, rem);
    tail[rem] = 0x80;
    size_t tl = rem < 56 ? 64 : 128;
    put_be64(tail + tl - 8, (uint64_t)len * 8);
    for (size_t i = 0; i < tl; i += 64) sha256_block(st, tail + i);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(st[i] >> 24); out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8); out[4 * i + 3] = (uint8_t)st[i];
    }
}

static const uint64_t K512[80] = {
    0x428a2f98d728ae22ULL, 0x7137449123ef65cdULL, 0xb5c0fbcfec4d3b2fULL, 0xe9b5dba58189dbbcULL, 0x3956c25bf348b538ULL,
    0x59f111f1b605d019ULL, 0x923f82a4af194f9bULL, 0xab1c5ed5da6d8118ULL, 0xd807aa98a3030242ULL, 0x12835b0145706fbeULL,
    0x243185be4ee4b28cULL, 0x550c7dc3d5ffb4e2ULL, 0x72be5d74f27b896fULL, 0x80deb1fe3b1696b1ULL, 0x9bdc06a725c71235ULL,
    0xc19bf174cf692694ULL, 0xe49b69c19ef14ad2ULL, 0xefbe4786384f25e3ULL, 0x0fc19dc68b8cd5b5ULL, 0x240ca1cc77ac9c65ULL,
    0x2de92c6f592b0275ULL, 0x4a7484aa6ea6e483ULL, 0x5cb0a9dcbd41fbd4ULL, 0x76f988da831153b5ULL, 0x983e5152ee66dfabULL,
    0xa831c66d2db43210ULL, 0xb00327c898fb213fULL, 0xbf597fc7beef0ee4ULL, 0xc6e00bf33da88fc2ULL, 0xd5a79147930aa725ULL,
    0x06ca6351e003826fULL, 0x142929670a0e6e70ULL, 0x27b70a8546d22ffcULL, 0x2e1b21385c26c926ULL, 0x4d2c6dfc5ac42aedULL,
    0x53380d139d95b3dfULL, 0x650a73548baf63deULL, 0x766a0abb3c77b2a8ULL, 0x81c2c92e47edaee6ULL, 0x92722c851482353bULL,
    0xa2bfe8a14cf10364ULL, 0xa81a664bbc423001ULL, 0xc24b8b70d0f89791ULL, 0xc76c51a30654be30ULL, 0xd192e819d6ef5218ULL,
    0xd69906245565a910ULL, 0xf40e35855771202aULL, 0x106aa07032bbd1b8ULL, 0x19a4c116b8d2d0c8ULL, 0x1e376c085141ab53ULL,
    0x2748774cdf8eeb99ULL, 0x34b0bcb5e19b48a8ULL, 0x391c0cb3c5c95a63ULL, 0x4ed8aa4ae3418acbULL, 0x5b9cca4f7763e373ULL,
    0x682e6ff3d6b2b8a3ULL, 0x748f82ee5defb2fcULL, 0x78a5636f43172f60ULL, 0x84c87814a1f0ab72ULL, 0x8cc702081a6439ecULL,
    0x90befffa23631e28ULL, 0xa4506cebde82bde9ULL, 0xbef9a3f7b2c67915ULL, 0xc67178f2e372532bULL, 0xca273eceea26619cULL,
    0xd186b8c721c0c207ULL, 0xeada7dd6cde0eb1eULL, 0xf57d4f7fee6ed178ULL, 0x06f067aa72176fbaULL, 0x0a637dc5a2c898a6ULL,
    0x113f9804bef90daeULL, 0x1b710b35131c471bULL, 0x28db77f523047d84ULL, 0x32caab7b40c72493ULL, 0x3c9ebe0a15c9bebcULL,
    0x431d67c49c100d4cULL, 0x4cc5d4becb3e42b6ULL, 0x597f299cfc657e2aULL, 0x5fcb6fab3ad6faecULL, 0x6c44198c4a475817ULL};

static uint64_t rotr64(uint64_t v, int c) { return (v >> c) | (v << (64 - c)); }

static void sha512_block(uint64_t st[8], const uint8_t *p) {
    uint64_t w[80];
    for (int i = 0; i < 16; i++) {
        uint64_t v = 0;
        for (int k = 0; k < 8; k++) v = (v << 8) | p[8 * i + k];
        w[i] = v;
    }
    for (int i = 16; i < 80; i++) {
        uint64_t s0 = rotr64(w[i - 15], 1) ^ rotr64(w[i - 15], 8) ^ (w[i - 15] >> 7);
        uint64_t s1 = rotr64(w[i - 2], 19) ^ rotr64(w[i - 2], 61) ^ (w[i - 2] >> 6);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 80; i++) {
        uint64_t t1 = h + (rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41)) + ((e & f) ^ (~e & g)) + K512[i] + w[i];
        uint64_t t2 = (rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39)) + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

void orc_sha384(const uint8_t *msg, size_t len, uint8_t out[48]) {
    uint64_t st[8] = {0xcbbb9d5dc1059ed8ULL, 0x629a292a367cd507ULL, 0x9159015a3070dd17ULL, 0x152fecd8f70e5939ULL,
                      0x67332667ffc00b31ULL, 0x8eb44a8768581511ULL, 0xdb0c2e0d64f98fa7ULL, 0x47b5481dbefa4fa4ULL};
    size_t full = len / 128;
    for (size_t i = 0; i < full; i++) sha512_block(st, msg + 128 * i);
    uint8_t tail[256] = {0};
    size_t rem = len % 128;
    if (rem) memcpy(tail, msg + 128 * full, rem);
    tail[rem] = 0x80;
    size_t tl = rem < 112 ? 128 : 256;
    put_be64(tail + tl - 8, (uint64_t)len * 8); /* high 64 bits of the 128-bit length stay 0 */
    for (size_t i = 0; i < tl; i += 128) sha512_block(st, tail + i);
    for (int i = 0; i < 6; i++)
        for (int k = 0; k < 8; k++) out[8 * i + k] = (uint8_t)(st[i] >> (56 - 8 * k));
}

static void hash_any(size_t hash_len, const uint8_t *m, size_t len, uint8_t *out) {
    if (hash_len == 32) orc_sha256(m, len, out); else orc_sha384(m, len, out);
}

void orc_hmac(size_t hash_len, const uint8_t *key, size_t key_len, const uint8_t *msg, size_t len, uint8_t *out) {
    size_t bs = hash_len == 32 ? 64 : 128;
    uint8_t k0[128] = {0}, ipad[128], opad[128], inner[48];
    if (key_len > bs) hash_any(hash_len, key, key_len, k0); else memcpy(k0, key, key_len);
    for (size_t i = 0; i < bs; i++) { ipad[i] = (uint8_t)(k0[i] ^ 0x36); opad[i] = (uint8_t)(k0[i] ^ 0x5c); }
    /* inner = H(ipad || msg) — assemble into one buffer (messages here are small) */
    uint8_t tmp[128 + 512];
    if (len > 512) return; /* not needed for this path */
    memcpy(tmp, ipad, bs);
    if (len) memcpy(tmp + bs, msg, len);
    hash_any(hash_len, tmp, bs + len, inner);
    memcpy(tmp, opad, bs); memcpy(tmp + bs, inner, hash_len);
    hash_any(hash_len, tmp, bs + hash_len, out);
}

void orc_hkdf_extract(size_t hash_len, const uint8_t *salt, size_t salt_len, const uint8_t *ikm, size_t ikm_len, uint8_t *prk) {
    orc_hmac(hash_len, salt, salt_len, ikm, ikm_len, prk);
}

void orc_hkdf_expand(size_t hash_len, const uint8_t *prk, const uint8_t *info, size_t info_len, uint8_t *out, size_t out_len) {
    uint8_t t[48], msg[48 + 256 + 1];
    size_t tlen = 0, done = 0;
    for (uint8_t i = 1; done < out_len; i++) {
        memcpy(msg, t, tlen);
        if (info_len) memcpy(msg + tlen, info, info_len);
        msg[tlen + info_len] = i;
        orc_hmac(hash_len, prk, hash_len, msg, tlen + info_len + 1, t);
        tlen = hash_len;
        size_t n = out_len - done < hash_len ? out_len - done : hash_len;
        memcpy(out + done, t, n);
        done += n;
    }
}

/* RFC 8446 §7.1 HkdfLabel = u16 length || u8 len("tls13 "+label) || "tls13 "+label || u8 0
 * (quic/s2n-quic-core/src/crypto/label.rs:57-68) */
void orc_hkdf_expand_label(size_t hash_len, const uint8_t *secret, const char *label, uint8_t *out, size_t out_len) {
    uint8_t info[2 + 1 + 255 + 1];
    size_t ll = strlen(label);
    info[0] = (uint8_t)(out_len >> 8);
    info[1] = (uint8_t)out_len;
    info[2] = (uint8_t)(6 + ll);
    memcpy(info + 3, "tls13 ", 6);
    memcpy(info + 9, label, ll);
    info[9 + ll] = 0;
    orc_hkdf_expand(hash_len, secret, info, 10 + ll, out, out_len);
}

/* ------------------------------------------------------------------ suites */

size_t orc_suite_key_len(int suite) { return suite == ORC_AES_128_GCM_SHA256 ? 16 : 32; }
size_t orc_suite_hash_len(int suite) { return suite == ORC_AES_256_GCM_SHA384 ? 48 : 32; }

/* quic/s2n-quic-crypto/src/iv.rs:27-39 */
void orc_nonce(const uint8_t iv[12], uint64_t pn, uint8_t nonce[12]) {
    memset(nonce, 0, 4);
    put_be64(nonce + 4, pn);
    for (int i = 0; i < 12; i++) nonce[i] ^= iv[i];
}

/* quic/s2n-quic-crypto/src/cipher_suite.rs:52-63,85-103 */
int orc_derive(int suite, const uint8_t *secret, uint8_t *key, uint8_t iv[12], uint8_t *hp) {
    size_t hl = orc_suite_hash_len(suite), kl = orc_suite_key_len(suite);
    orc_hkdf_expand_label(hl, secret, "quic key", key, kl);
    orc_hkdf_expand_label(hl, secret, "quic iv", iv, 12);
    orc_hkdf_expand_label(hl, secret, "quic hp", hp, kl);
    return 0;
}

/* quic/s2n-quic-crypto/src/cipher_suite.rs:68-83 */
int orc_update_secret(int suite, const uint8_t *secret, uint8_t *next_secret) {
    size_t hl = orc_suite_hash_len(suite);
    orc_hkdf_expand_label(hl, secret, "quic ku", next_secret, hl);
    return 0;
}

/* quic/s2n-quic-crypto/src/initial.rs:29-53, salt quic/s2n-quic-core/src/crypto/initial.rs:29 */
void orc_initial_secrets(const uint8_t *dcid, size_t dcid_len, uint8_t client[32], uint8_t server[32]) {
    static const uint8_t salt[20] = {0x38, 0x76, 0x2c, 0xf7, 0xf5, 0x59, 0x34, 0xb3, 0x4d, 0x17,
                                     0x9a, 0xe6, 0xa4, 0xc8, 0x0c, 0xad, 0xcc, 0xbb, 0x7f, 0x0a};
    uint8_t prk[32];
    orc_hkdf_extract(32, salt, 20, dcid, dcid_len, prk);
    orc_hkdf_expand_label(32, prk, "client in", client, 32);
    orc_hkdf_expand_label(32, prk, "server in", server, 32);
}

int orc_seal(int suite, const uint8_t *key, const uint8_t nonce[12],
             const uint8_t *aad, size_t aad_len, uint8_t *buf, size_t pt_len) {
    if (suite == ORC_CHACHA20_POLY1305_SHA256)
        chacha_poly_core(key, nonce, aad, aad_len, buf, pt_len, 1, buf + pt_len);
    else
        aes_gcm_core(key, orc_suite_key_len(suite), nonce, aad, aad_len, buf, pt_len, 1, buf + pt_len);
    return ORC_OK;
}

/* cipher_suite.rs:117-144: len < 16 -> DECRYPT_ERROR; aead/default.rs:65-93 */
int orc_open(int suite, const uint8_t *key, const uint8_t nonce[12],
             const uint8_t *aad, size_t aad_len, uint8_t *buf, size_t ct_tag_len) {
    if (ct_tag_len < 16) return ORC_DECRYPT_ERROR;
    size_t len = ct_tag_len - 16;
    uint8_t tag[16];
    if (suite == ORC_CHACHA20_POLY1305_SHA256)
        chacha_poly_core(key, nonce, aad, aad_len, buf, len, 0, tag);
    else
        aes_gcm_core(key, orc_suite_key_len(suite), nonce, aad, aad_len, buf, len, 0, tag);
    uint8_t diff = 0;
    for (int i = 0; i < 16; i++) diff |= (uint8_t)(tag[i] ^ buf[len + i]);
    if (diff) {
        if (len) memset(buf, 0, len); /* never release unauthenticated plaintext */
        return ORC_DECRYPT_ERROR;
    }
    return ORC_OK;
}

/* quic/s2n-quic-crypto/src/header_key.rs:52-56 -> aws-lc quic::HeaderProtectionKey::new_mask */
void orc_hp_mask(int suite, const uint8_t *hp_key, const uint8_t sample[16], uint8_t mask[5]) {
    if (suite == ORC_CHACHA20_POLY1305_SHA256) {
        uint8_t blk[64];
        orc_chacha20_block(hp_key, le32(sample), sample + 4, blk);
        memcpy(mask, blk, 5);
    } else {
        uint8_t rk[240], out[16];
        int rounds = orc_aes_expand(hp_key, orc_suite_key_len(suite), rk);
        orc_aes_encrypt_block(rk, rounds, sample, out);
        memcpy(mask, out, 5);
    }
}

/* header_crypto.rs:63-95 */
static void apply_mask(uint8_t *pkt, size_t pn_off, size_t pn_len, const uint8_t mask[5]) {
    pkt[0] ^= (uint8_t)(mask[0] & ((pkt[0] & 0x80) ? 0x0f : 0x1f));
    for (size_t i = 0; i < pn_len; i++) pkt[pn_off + i] ^= mask[1 + i];
}

/* packet/encoding.rs:274-278 -> crypto/mod.rs:181-247 */
int orc_protect_packet(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp,
                       uint64_t pn, uint8_t *pkt, size_t header_len, size_t pn_len, size_t payload_len) {
    uint8_t nonce[12], mask[5];
    orc_nonce(iv, pn, nonce);
    size_t aad_len = header_len + pn_len;
    orc_seal(suite, key, nonce, pkt, aad_len, pkt + aad_len, payload_len);
    /* sample at header_len + 4 (payload.rs:151-169) */
    if (header_len + 4 + 16 > aad_len + payload_len + 16) return ORC_DECODE_ERROR;
    orc_hp_mask(suite, hp, pkt + header_len + 4, mask);
    apply_mask(pkt, header_len, pn_len, mask);
    return ORC_OK;
}

/* crypto/mod.rs:195-204,251-264 and header_crypto.rs:98-123 */
int orc_unprotect_packet(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp,
                         uint64_t full_pn, uint8_t *pkt, size_t header_len, size_t pkt_len,
                         size_t *pn_len_out) {
    uint8_t nonce[12], mask[5];
    if (header_len + 4 + 16 > pkt_len) return ORC_DECODE_ERROR;
    orc_hp_mask(suite, hp, pkt + header_len + 4, mask);
    pkt[0] ^= (uint8_t)(mask[0] & ((pkt[0] & 0x80) ? 0x0f : 0x1f));
    size_t pn_len = (size_t)(pkt[0] & 3) + 1;
    for (size_t i = 0; i < pn_len; i++) pkt[header_len + i] ^= mask[1 + i];
    if (pn_len_out) *pn_len_out = pn_len;
    orc_nonce(iv, full_pn, nonce);
    size_t aad_len = header_len + pn_len;
    return orc_open(suite, key, nonce, pkt, aad_len, pkt + aad_len, pkt_len - aad_len);
}

void orc_seal_batch(const orc_key *keys, const orc_pkt *pkts, size_t n, uint8_t *arena,
                    uint8_t *masks, int flags) {
    for (size_t i = 0; i < n; i++) {
        const orc_pkt *p = &pkts[i];
        const orc_key *k = &keys[p->key_idx];
        uint8_t nonce[12], mask[5];
        uint8_t *base = arena + p->off;
        orc_nonce(k->iv, p->pn, nonce);
        orc_seal(k->suite, k->key, nonce, base, p->aad_len, base + p->aad_len, p->pt_len);
        if (flags & 3) {
            size_t hdr = (size_t)p->aad_len - p->pn_len;
            orc_hp_mask(k->suite, k->hp, base + hdr + 4, mask);
            if (flags & 1) memcpy(masks + 5 * i, mask, 5);
            if (flags & 2) apply_mask(base, hdr, p->pn_len, mask);
        }
    }
}

/* ---- FIPS mode: the sealing nonce order of aws-lc's TLS 1.3 AES-GCM AEAD (EVP_aead_aes_*_gcm_tls13 behind aws-lc-rs
 * 1.12 TlsRecordSealingKey, which s2n-quic-crypto's `fips` feature uses: aead/fips.rs:13-60, cipher_suite/ring.rs:13-31).
 * aws-lc is not vendored in the reference; this restates its published seal check on the nonce bytes themselves:
 * given = big-endian u64 of nonce[4..12]; the first seal sets mask = given; given ^= mask; refuse if
 * given == 2^64 - 1 or given < min_next; else min_next = given + 1.  Parity unpinned: the reference holds no vectors. */
int orc_fips_seal_ok(orc_fips_state *st, const uint8_t nonce[12]) {
    uint64_t given = 0;
    for (int i = 4; i < 12; i++) given = (given << 8) | nonce[i];
    if (!st->seen) {
        st->mask = given;
        st->seen = 1;
    }
    given ^= st->mask;
    if (given == UINT64_MAX || given < st->min_next) return 0;
    st->min_next = given + 1;
    return 1;
}

/* orc_seal_batch, one packet after the other, with the FIPS check for keys whose fips[key] is set: a refused packet
 * is left untouched with status 3 (INTERNAL_ERROR), the others get status 0. */
void orc_seal_batch_fips(const orc_key *keys, const uint8_t *fips, orc_fips_state *states, const orc_pkt *pkts,
                         size_t n, uint8_t *arena, uint8_t *masks, int flags, int8_t *status) {
    for (size_t i = 0; i < n; i++) {
        const orc_pkt *p = &pkts[i];
        uint8_t nonce[12];
        orc_nonce(keys[p->key_idx].iv, p->pn, nonce);
        if (fips[p->key_idx] && !orc_fips_seal_ok(&states[p->key_idx], nonce)) {
            status[i] = 3;
            continue;
        }
        status[i] = 0;
        orc_seal_batch(keys, p, 1, arena, masks ? masks + 5 * i : NULL, flags);
    }
}

void orc_open_batch(const orc_key *keys, const orc_pkt *pkts, size_t n, uint8_t *arena, int8_t *status) {
    for (size_t i = 0; i < n; i++) {
        const orc_pkt *p = &pkts[i];
        const orc_key *k = &keys[p->key_idx];
        uint8_t nonce[12];
        uint8_t *base = arena + p->off;
        orc_nonce(k->iv, p->pn, nonce);
        status[i] = (int8_t)orc_open(k->suite, k->key, nonce, base, p->aad_len, base + p->aad_len,
                                     (size_t)p->pt_len + 16);
    }
}

/* ---- packet numbers ---- */
uint64_t orc_decode_packet_number(uint64_t largest_pn, uint64_t truncated_pn, unsigned pn_nbits) {
    /* tests.rs:141-158, the `catch!` blocks: a checked sub/add that overflows makes its condition false */
    const uint64_t expected_pn = largest_pn + 1;
    const uint64_t pn_win = (uint64_t)1 << pn_nbits;
    const uint64_t pn_hwin = pn_win / 2;
    const uint64_t pn_mask = pn_win - 1;
    const uint64_t candidate_pn = (expected_pn & ~pn_mask) | truncated_pn;
    const uint64_t limit62 = (uint64_t)1 << 62, varint_max = limit62 - 1;
    uint64_t r = candidate_pn;
    if (expected_pn >= pn_hwin && candidate_pn <= expected_pn - pn_hwin && limit62 >= pn_win &&
        candidate_pn < limit62 - pn_win)
        r = candidate_pn + pn_win;
    else if (expected_pn <= UINT64_MAX - pn_hwin && candidate_pn > expected_pn + pn_hwin && candidate_pn >= pn_win)
        r = candidate_pn - pn_win;
    return r < varint_max ? r : varint_max;
}

int orc_truncate_packet_number(uint64_t pn, uint64_t largest_pn, uint64_t *truncated, size_t *pn_len) {
    if (pn < largest_pn) return ORC_DECODE_ERROR;
    const uint64_t d = pn - largest_pn;
    if (d > (UINT64_MAX >> 1)) return ORC_DECODE_ERROR;
    const uint64_t range = d * 2;
    size_t len;
    if (range <= 0xff) len = 1;
    else if (range <= 0xffff) len = 2;
    else if (range <= 0xffffff) len = 3;
    else if (range <= 0xffffffffull) len = 4;
    else return ORC_DECODE_ERROR;
    *pn_len = len;
    *truncated = pn & ((len == 4) ? 0xffffffffull : (((uint64_t)1 << (8 * len)) - 1));
    return ORC_OK;
}

void orc_unprotect_open_batch(const orc_key *keys, const orc_rx_pkt *rx, size_t n, uint8_t *arena, orc_pkt *out,
                              int8_t *status) {
    for (size_t i = 0; i < n; i++) {
        const orc_rx_pkt *r = &rx[i];
        uint8_t *pkt = arena + r->off;
        orc_pkt *d = &out[i];
        memset(d, 0, sizeof *d);
        d->off = r->off;
        d->key_idx = r->key_idx[0];
        d->aad_len = r->header_len;
        /* payload.rs:151-169: the sample must fit */
        if ((size_t)r->header_len + 4 + 16 > r->len) {
            d->flags = 1;
            status[i] = ORC_DECODE_ERROR;
            continue;
        }
        const orc_key *hk = &keys[r->key_idx[0]];
        uint8_t mask[5];
        orc_hp_mask(hk->suite, hk->hp, pkt + r->header_len + 4, mask);
        pkt[0] ^= (uint8_t)(mask[0] & ((pkt[0] & 0x80) ? 0x0f : 0x1f));
        const size_t pn_len = (size_t)(pkt[0] & 3) + 1;
        uint64_t trunc = 0;
        for (size_t j = 0; j < pn_len; j++) {
            pkt[r->header_len + j] ^= mask[1 + j];
            trunc = (trunc << 8) | pkt[r->header_len + j];
        }
        const uint64_t pn = orc_decode_packet_number(r->largest_pn & (((uint64_t)1 << 62) - 1), trunc, (unsigned)(8 * pn_len));
        const int phase = (pkt[0] & 0x80) ? 0 : ((pkt[0] >> 2) & 1); /* key_phase.rs:46-49 */
        const orc_key *k = &keys[r->key_idx[phase]];
        d->pn = pn;
        d->key_idx = r->key_idx[phase];
        d->aad_len = (uint16_t)(r->header_len + pn_len);
        d->pt_len = (uint16_t)(r->len - r->header_len - pn_len - 16);
        d->pn_len = (uint8_t)pn_len;
        uint8_t nonce[12];
        orc_nonce(k->iv, pn, nonce);
        status[i] = (int8_t)orc_open(k->suite, k->key, nonce, pkt, d->aad_len, pkt + d->aad_len, (size_t)d->pt_len + 16);
    }
}
