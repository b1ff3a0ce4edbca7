// keysched.hip — batched key installation on the GPU (key-update churn).
//
// Replaces, for a batch of n traffic secrets, the per-key CPU work of quic/s2n-quic-crypto:
//   TLS_*::new(secret)  key = HKDF-Expand-Label(secret, "quic key"), iv = ..."quic iv", hp = ..."quic hp"
//                       (src/cipher_suite.rs:52-63,85-103; src/iv.rs:14-24; src/header_key.rs:33-49)
//   TLS_*::update()     secret' = HKDF-Expand-Label(secret, "quic ku", Hash.len); the header key is NOT
//                       re-derived (src/cipher_suite.rs:68-83; RFC 9001 §6), `updates` times
// followed by the AES key expansion of the packet and header keys (FIPS-197 §5.2) and the device key record; the
// GHASH key powers follow in key_setup_kernel (aes_gcm.hip).  One lane per key: SHA-256 / SHA-384 compressions
// on VALU, HMAC with the one-block message an Expand-Label of <= 48 output bytes needs (RFC 5869 T(1)).
#include "device_common.h"

namespace qpp {
namespace {
using namespace dev;

__device__ const uint32_t d_k256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ const uint64_t d_k512[80] = {
    0x428a2f98d728ae22, 0x7137449123ef65cd, 0xb5c0fbcfec4d3b2f, 0xe9b5dba58189dbbc, 0x3956c25bf348b538,
    0x59f111f1b605d019, 0x923f82a4af194f9b, 0xab1c5ed5da6d8118, 0xd807aa98a3030242, 0x12835b0145706fbe,
    0x243185be4ee4b28c, 0x550c7dc3d5ffb4e2, 0x72be5d74f27b896f, 0x80deb1fe3b1696b1, 0x9bdc06a725c71235,
    0xc19bf174cf692694, 0xe49b69c19ef14ad2, 0xefbe4786384f25e3, 0x0fc19dc68b8cd5b5, 0x240ca1cc77ac9c65,
    0x2de92c6f592b0275, 0x4a7484aa6ea6e483, 0x5cb0a9dcbd41fbd4, 0x76f988da831153b5, 0x983e5152ee66dfab,
    0xa831c66d2db43210, 0xb00327c898fb213f, 0xbf597fc7beef0ee4, 0xc6e00bf33da88fc2, 0xd5a79147930aa725,
    0x06ca6351e003826f, 0x142929670a0e6e70, 0x27b70a8546d22ffc, 0x2e1b21385c26c926, 0x4d2c6dfc5ac42aed,
    0x53380d139d95b3df, 0x650a73548baf63de, 0x766a0abb3c77b2a8, 0x81c2c92e47edaee6, 0x92722c851482353b,
    0xa2bfe8a14cf10364, 0xa81a664bbc423001, 0xc24b8b70d0f89791, 0xc76c51a30654be30, 0xd192e819d6ef5218,
    0xd69906245565a910, 0xf40e35855771202a, 0x106aa07032bbd1b8, 0x19a4c116b8d2d0c8, 0x1e376c085141ab53,
    0x2748774cdf8eeb99, 0x34b0bcb5e19b48a8, 0x391c0cb3c5c95a63, 0x4ed8aa4ae3418acb, 0x5b9cca4f7763e373,
    0x682e6ff3d6b2b8a3, 0x748f82ee5defb2fc, 0x78a5636f43172f60, 0x84c87814a1f0ab72, 0x8cc702081a6439ec,
    0x90befffa23631e28, 0xa4506cebde82bde9, 0xbef9a3f7b2c67915, 0xc67178f2e372532b, 0xca273eceea26619c,
    0xd186b8c721c0c207, 0xeada7dd6cde0eb1e, 0xf57d4f7fee6ed178, 0x06f067aa72176fba, 0x0a637dc5a2c898a6,
    0x113f9804bef90dae, 0x1b710b35131c471b, 0x28db77f523047d84, 0x32caab7b40c72493, 0x3c9ebe0a15c9bebc,
    0x431d67c49c100d4c, 0x4cc5d4becb3e42b6, 0x597f299cfc657e2a, 0x5fcb6fab3ad6faec, 0x6c44198c4a475817};

template <typename W>
__device__ __forceinline__ W rotr(W v, int c) {
    return (v >> c) | (v << (8 * (int)sizeof(W) - c));
}

// FIPS 180-4 compression of one block (16 big-endian words of W) into st.
template <typename W>
__device__ void sha2_block(W st[8], const uint8_t *blk) {
    constexpr bool k32 = sizeof(W) == 4;
    constexpr int R = k32 ? 64 : 80;
    W w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        W v = 0;
#pragma unroll
        for (int b = 0; b < (int)sizeof(W); b++) v = (W)((v << 8) | blk[i * sizeof(W) + b]);
        w[i] = v;
    }
    W a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < R; i++) {
        W wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const W x = w[(i - 15) & 15], y = w[(i - 2) & 15];
            const W s0 = k32 ? (rotr<W>(x, 7) ^ rotr<W>(x, 18) ^ (x >> 3)) : (rotr<W>(x, 1) ^ rotr<W>(x, 8) ^ (x >> 7));
            const W s1 = k32 ? (rotr<W>(y, 17) ^ rotr<W>(y, 19) ^ (y >> 10)) : (rotr<W>(y, 19) ^ rotr<W>(y, 61) ^ (y >> 6));
            wi = w[(i - 16) & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
        }
        const W S1 = k32 ? (rotr<W>(e, 6) ^ rotr<W>(e, 11) ^ rotr<W>(e, 25)) : (rotr<W>(e, 14) ^ rotr<W>(e, 18) ^ rotr<W>(e, 41));
        const W S0 = k32 ? (rotr<W>(a, 2) ^ rotr<W>(a, 13) ^ rotr<W>(a, 22)) : (rotr<W>(a, 28) ^ rotr<W>(a, 34) ^ rotr<W>(a, 39));
        W K;
        if constexpr (k32) K = d_k256[i]; else K = d_k512[i];
        const W t1 = h + S1 + ((e & f) ^ (~e & g)) + K + wi;
        const W t2 = S0 + ((a & b) ^ (a & c) ^ (b & c));
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

template <typename W>
__device__ __forceinline__ void sha2_init(W st[8]) {
    if constexpr (sizeof(W) == 4) {
        const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
        for (int i = 0; i < 8; i++) st[i] = iv[i];
    } else {  // SHA-384
        const uint64_t iv[8] = {0xcbbb9d5dc1059ed8, 0x629a292a367cd507, 0x9159015a3070dd17, 0x152fecd8f70e5939,
                                0x67332667ffc00b31, 0x8eb44a8768581511, 0xdb0c2e0d64f98fa7, 0x47b5481dbefa4fa4};
        for (int i = 0; i < 8; i++) st[i] = iv[i];
    }
}

// Final block: msg (len < block - 2 * sizeof(W)) || 0x80 || 0 ... || big-endian bit length of (B + len) bytes.
template <typename W>
__device__ void sha2_last(W st[8], const uint8_t *msg, int len, uint8_t *digest, int digest_len) {
    constexpr int B = 16 * sizeof(W);
    uint8_t blk[B];
    for (int i = 0; i < B; i++) blk[i] = i < len ? msg[i] : 0;
    blk[len] = 0x80;
    const uint64_t bits = (uint64_t)(B + len) * 8;
    for (int i = 0; i < 8; i++) blk[B - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha2_block<W>(st, blk);
    for (int i = 0; i < digest_len; i++) digest[i] = (uint8_t)(st[i / sizeof(W)] >> (8 * (sizeof(W) - 1 - i % sizeof(W))));
}

// HKDF-Expand-Label(secret, label, "", out_len) = HMAC(secret, HkdfLabel || 0x01)[0..out_len]
// (quic/s2n-quic-core/src/crypto/label.rs:57-68; RFC 8446 §7.1; out_len <= Hash.len: one HKDF block).
template <typename W>
__device__ void expand_label(const uint8_t *secret, const char *label, int label_len, uint8_t *out, int out_len) {
    constexpr int B = 16 * sizeof(W), HL = sizeof(W) == 4 ? 32 : 48;
    uint8_t pad[B], info[32], inner[HL], t[HL];
    W st[8];
    for (int i = 0; i < B; i++) pad[i] = (i < HL ? secret[i] : 0) ^ 0x36;
    sha2_init<W>(st);
    sha2_block<W>(st, pad);
    int n = 0;
    info[n++] = (uint8_t)(out_len >> 8);
    info[n++] = (uint8_t)out_len;
    info[n++] = (uint8_t)(6 + label_len);
    const char tls13[6] = {'t', 'l', 's', '1', '3', ' '};
    for (int i = 0; i < 6; i++) info[n++] = (uint8_t)tls13[i];
    for (int i = 0; i < label_len; i++) info[n++] = (uint8_t)label[i];
    info[n++] = 0;  // empty context
    info[n++] = 1;  // HKDF-Expand counter T(1)
    sha2_last<W>(st, info, n, inner, HL);
    for (int i = 0; i < B; i++) pad[i] = (i < HL ? secret[i] : 0) ^ 0x5c;
    sha2_init<W>(st);
    sha2_block<W>(st, pad);
    sha2_last<W>(st, inner, HL, t, HL);
    for (int i = 0; i < out_len; i++) out[i] = t[i];
}

__device__ void label_expand(int hash_len, const uint8_t *secret, const char *label, int label_len, uint8_t *out,
                             int out_len) {
    if (hash_len == 32) expand_label<uint32_t>(secret, label, label_len, out, out_len);
    else expand_label<uint64_t>(secret, label, label_len, out, out_len);
}

// FIPS-197 §5.2 into little-endian column words (the layout of DevKey::rk, kdf.cpp aes_expand_key)
__device__ int aes_expand(const uint8_t *key, int key_len, uint32_t *rk) {
    const int nk = key_len / 4, rounds = nk + 6, total = 4 * (rounds + 1);
    auto sub = [](uint32_t w) {
        return (uint32_t)d_sbox[w & 0xff] | ((uint32_t)d_sbox[(w >> 8) & 0xff] << 8) |
               ((uint32_t)d_sbox[(w >> 16) & 0xff] << 16) | ((uint32_t)d_sbox[w >> 24] << 24);
    };
    for (int i = 0; i < nk; i++)
        rk[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) |
                ((uint32_t)key[4 * i + 3] << 24);
    uint32_t rcon = 1;
    for (int i = nk; i < total; i++) {
        uint32_t t = rk[i - 1];
        if (i % nk == 0) {
            t = sub((t >> 8) | (t << 24)) ^ rcon;
            rcon = xtime4(rcon);
        } else if (nk > 6 && i % nk == 4) {
            t = sub(t);
        }
        rk[i] = rk[i - nk] ^ t;
    }
    return rounds;
}

// material record per key (host handles are filled from it): secret' | key | iv | hp
constexpr int kMatSecret = 0, kMatKey = 48, kMatIv = 80, kMatHp = 96, kMatBytes = 128;

// hp_in == nullptr: the header key is derived from the given secret ("quic hp", TLS_*::new); otherwise it is taken
// from hp_in (kl bytes per key): the header key of the key being updated (OneRttKey::derive_next_key keeps it).
__global__ __launch_bounds__(64) void key_derive_kernel(DevKey *keys, const uint32_t *__restrict__ slots, uint32_t n,
                                                       int suite, const uint8_t *__restrict__ secrets,
                                                       const uint8_t *__restrict__ hp_in, uint32_t updates,
                                                       uint8_t *material, uint32_t fips) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int hl = suite == QPP_SUITE_TLS_AES_256_GCM_SHA384 ? 48 : 32;
    const int kl = suite == QPP_SUITE_TLS_AES_128_GCM_SHA256 ? 16 : 32;
    uint8_t s[48], t[48], key[32], iv[12], hp[32];
    for (int j = 0; j < hl; j++) s[j] = secrets[(size_t)i * hl + j];
    if (hp_in) {
        for (int j = 0; j < kl; j++) hp[j] = hp_in[(size_t)i * kl + j];
    } else {
        label_expand(hl, s, "quic hp", 7, hp, kl);  // header key of the first secret, kept by every update
    }
    for (uint32_t u = 0; u < updates; u++) {
        label_expand(hl, s, "quic ku", 7, t, hl);
        for (int j = 0; j < hl; j++) s[j] = t[j];
    }
    label_expand(hl, s, "quic key", 8, key, kl);
    label_expand(hl, s, "quic iv", 7, iv, 12);

    DevKey *k = keys + slots[i];
    k->suite = (uint32_t)suite;
    for (int w = 0; w < 3; w++)
        k->iv[w] = (uint32_t)iv[4 * w] | ((uint32_t)iv[4 * w + 1] << 8) | ((uint32_t)iv[4 * w + 2] << 16) |
                   ((uint32_t)iv[4 * w + 3] << 24);
    k->iv[3] = 0;
    if (suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256) {
        k->nr = 0;
        k->hp_nr = 0;
        for (int w = 0; w < 8; w++) {
            k->rk[w] = (uint32_t)key[4 * w] | ((uint32_t)key[4 * w + 1] << 8) | ((uint32_t)key[4 * w + 2] << 16) |
                       ((uint32_t)key[4 * w + 3] << 24);
            k->hp_rk[w] = (uint32_t)hp[4 * w] | ((uint32_t)hp[4 * w + 1] << 8) | ((uint32_t)hp[4 * w + 2] << 16) |
                          ((uint32_t)hp[4 * w + 3] << 24);
        }
    } else {
        k->nr = (uint32_t)aes_expand(key, kl, k->rk);
        k->hp_nr = (uint32_t)aes_expand(hp, kl, k->hp_rk);
    }
    k->live = 1;
    k->fips = fips && suite != QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256 ? 1u : 0u;  // no FIPS ChaCha (ring.rs:116-121)
    k->fips_seen = 0;
    k->fips_mask = 0;
    k->fips_min_next = 0;
    uint8_t *m = material + (size_t)i * kMatBytes;
    for (int j = 0; j < hl; j++) m[kMatSecret + j] = s[j];
    for (int j = 0; j < kl; j++) m[kMatKey + j] = key[j];
    for (int j = 0; j < 12; j++) m[kMatIv + j] = iv[j];
    for (int j = 0; j < kl; j++) m[kMatHp + j] = hp[j];
    for (int j = 0; j < 48; j++) s[j] = t[j] = 0;
}

}  // namespace

uint32_t key_material_bytes() { return kMatBytes; }

hipError_t launch_key_derive(DevKey *keys, const uint32_t *slots, uint32_t n, int suite, const uint8_t *secrets,
                             const uint8_t *hp_in, uint32_t updates, uint8_t *material, uint32_t fips,
                             const PowTables &pow, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(key_derive_kernel, dim3((n + 63) / 64), dim3(64), 0, s, keys, slots, n, suite, secrets, hp_in,
                       updates, material, fips);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_key_install(keys, slots, nullptr, n, pow, s);
}

}  // namespace qpp
