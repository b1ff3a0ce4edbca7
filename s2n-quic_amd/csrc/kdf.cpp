// kdf.cpp — host-side key schedule of the engine: SHA-256/384, HMAC, HKDF-Expand-Label (RFC 8446 §7.1)
// and the AES key expansion.  This is key installation, not the data path: the reference derives keys on
// the CPU too (quic/s2n-quic-crypto/src/cipher_suite.rs:52-104 via aws-lc-rs hkdf).  Every operation that
// encrypts data (including H = E_K(0)) runs on the GPU.
#include <string.h>

#include <array>
#include <vector>

#include "qpp_internal.h"

namespace qpp {
namespace {

template <typename W>
constexpr W rotr(W v, int c) {
    return (v >> c) | (v << (sizeof(W) * 8 - c));
}

// FIPS 180-4 round constants: fractional parts of cube roots of the first primes.
constexpr std::array<uint32_t, 64> k256 = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

constexpr std::array<uint64_t, 80> k512 = {
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

// Generic Merkle–Damgård SHA-2 over word type W (uint32_t: SHA-256, uint64_t: SHA-384/512).
template <typename W>
struct Sha2 {
    static constexpr size_t kWords = sizeof(W) == 4 ? 64 : 80;
    static constexpr size_t kBlock = 16 * sizeof(W);
    W st[8];
    uint8_t buf[kBlock];
    size_t fill = 0;
    uint64_t total = 0;

    explicit Sha2(const W (&iv)[8]) { memcpy(st, iv, sizeof st); }

    static W sig0(W x) { return sizeof(W) == 4 ? rotr<W>(x, 7) ^ rotr<W>(x, 18) ^ (x >> 3) : rotr<W>(x, 1) ^ rotr<W>(x, 8) ^ (x >> 7); }
    static W sig1(W x) { return sizeof(W) == 4 ? rotr<W>(x, 17) ^ rotr<W>(x, 19) ^ (x >> 10) : rotr<W>(x, 19) ^ rotr<W>(x, 61) ^ (x >> 6); }
    static W Sig0(W x) { return sizeof(W) == 4 ? rotr<W>(x, 2) ^ rotr<W>(x, 13) ^ rotr<W>(x, 22) : rotr<W>(x, 28) ^ rotr<W>(x, 34) ^ rotr<W>(x, 39); }
    static W Sig1(W x) { return sizeof(W) == 4 ? rotr<W>(x, 6) ^ rotr<W>(x, 11) ^ rotr<W>(x, 25) : rotr<W>(x, 14) ^ rotr<W>(x, 18) ^ rotr<W>(x, 41); }
    static W K(size_t i) {
        if constexpr (sizeof(W) == 4) return k256[i]; else return k512[i];
    }

    void compress(const uint8_t *p) {
        W w[kWords];
        for (size_t i = 0; i < 16; i++) {
            W v = 0;
            for (size_t b = 0; b < sizeof(W); b++) v = (W)((v << 8) | p[i * sizeof(W) + b]);
            w[i] = v;
        }
        for (size_t i = 16; i < kWords; i++) w[i] = w[i - 16] + sig0(w[i - 15]) + w[i - 7] + sig1(w[i - 2]);
        W a[8];
        memcpy(a, st, sizeof a);
        for (size_t i = 0; i < kWords; i++) {
            W t1 = a[7] + Sig1(a[4]) + ((a[4] & a[5]) ^ (~a[4] & a[6])) + K(i) + w[i];
            W t2 = Sig0(a[0]) + ((a[0] & a[1]) ^ (a[0] & a[2]) ^ (a[1] & a[2]));
            for (int k = 7; k > 0; k--) a[k] = a[k - 1];
            a[4] += t1;
            a[0] = t1 + t2;
        }
        for (int k = 0; k < 8; k++) st[k] += a[k];
    }

    void update(const uint8_t *p, size_t n) {
        total += n;
        while (n) {
            size_t take = kBlock - fill < n ? kBlock - fill : n;
            memcpy(buf + fill, p, take);
            fill += take; p += take; n -= take;
            if (fill == kBlock) { compress(buf); fill = 0; }
        }
    }

    void finish(uint8_t *out, size_t out_len) {
        uint64_t bits = total * 8;
        uint8_t pad = 0x80;
        update(&pad, 1);
        uint8_t zero = 0;
        size_t len_field = 2 * sizeof(W);  // 8 (SHA-256) or 16 (SHA-512 family)
        while (fill != kBlock - len_field) update(&zero, 1);
        uint8_t lenb[16] = {0};
        for (int i = 0; i < 8; i++) lenb[len_field - 1 - i] = (uint8_t)(bits >> (8 * i));
        update(lenb, len_field);
        for (size_t i = 0; i < out_len; i++) out[i] = (uint8_t)(st[i / sizeof(W)] >> (8 * (sizeof(W) - 1 - i % sizeof(W))));
    }
};

constexpr uint32_t kIv256[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
constexpr uint64_t kIv384[8] = {0xcbbb9d5dc1059ed8, 0x629a292a367cd507, 0x9159015a3070dd17, 0x152fecd8f70e5939,
                                0x67332667ffc00b31, 0x8eb44a8768581511, 0xdb0c2e0d64f98fa7, 0x47b5481dbefa4fa4};

// Streaming HMAC over SHA-256 (hash_len 32) or SHA-384 (hash_len 48).
class Hmac {
  public:
    Hmac(size_t hash_len, const uint8_t *key, size_t key_len) : hl_(hash_len), s256_(kIv256), s384_(kIv384) {
        size_t bs = block();
        uint8_t k0[128] = {0};
        if (key_len > bs) {
            Hmac::digest(hl_, key, key_len, k0);
        } else {
            memcpy(k0, key, key_len);
        }
        for (size_t i = 0; i < bs; i++) { opad_[i] = k0[i] ^ 0x5c; k0[i] ^= 0x36; }
        feed(k0, bs);
        secure_zero(k0, sizeof k0);
    }
    void feed(const uint8_t *p, size_t n) { if (hl_ == 32) s256_.update(p, n); else s384_.update(p, n); }
    void finish(uint8_t *out) {
        uint8_t inner[48];
        if (hl_ == 32) s256_.finish(inner, 32); else s384_.finish(inner, 48);
        Sha2<uint32_t> o256(kIv256);
        Sha2<uint64_t> o384(kIv384);
        if (hl_ == 32) { o256.update(opad_, 64); o256.update(inner, 32); o256.finish(out, 32); }
        else { o384.update(opad_, 128); o384.update(inner, 48); o384.finish(out, 48); }
        secure_zero(inner, sizeof inner);
        secure_zero(opad_, sizeof opad_);
    }
    static void digest(size_t hl, const uint8_t *p, size_t n, uint8_t *out) {
        if (hl == 32) { Sha2<uint32_t> h(kIv256); h.update(p, n); h.finish(out, 32); }
        else { Sha2<uint64_t> h(kIv384); h.update(p, n); h.finish(out, 48); }
    }

  private:
    size_t block() const { return hl_ == 32 ? 64 : 128; }
    size_t hl_;
    Sha2<uint32_t> s256_;
    Sha2<uint64_t> s384_;
    uint8_t opad_[128];
};

}  // namespace

void secure_zero(void *p, size_t n) {
    volatile uint8_t *v = (volatile uint8_t *)p;
    while (n--) *v++ = 0;
}

size_t suite_key_len(int suite) { return suite == QPP_SUITE_TLS_AES_128_GCM_SHA256 ? 16 : 32; }
size_t suite_hash_len(int suite) { return suite == QPP_SUITE_TLS_AES_256_GCM_SHA384 ? 48 : 32; }

void hkdf_extract(size_t hash_len, const uint8_t *salt, size_t salt_len, const uint8_t *ikm, size_t ikm_len,
                  uint8_t *prk) {
    Hmac h(hash_len, salt, salt_len);
    h.feed(ikm, ikm_len);
    h.finish(prk);
}

// HKDF-Expand(secret, HkdfLabel(len, "tls13 " + label, ""), len) — quic/s2n-quic-core/src/crypto/label.rs:57-68
void hkdf_expand_label(size_t hash_len, const uint8_t *secret, const char *label, uint8_t *out, size_t out_len) {
    std::vector<uint8_t> info;
    size_t ll = strlen(label);
    info.push_back((uint8_t)(out_len >> 8));
    info.push_back((uint8_t)out_len);
    info.push_back((uint8_t)(6 + ll));
    for (const char *p = "tls13 "; *p; ++p) info.push_back((uint8_t)*p);
    for (size_t i = 0; i < ll; i++) info.push_back((uint8_t)label[i]);
    info.push_back(0);
    uint8_t t[48];
    size_t done = 0;
    for (uint8_t counter = 1; done < out_len; counter++) {
        Hmac h(hash_len, secret, hash_len);
        if (counter > 1) h.feed(t, hash_len);
        h.feed(info.data(), info.size());
        h.feed(&counter, 1);
        h.finish(t);
        size_t take = out_len - done < hash_len ? out_len - done : hash_len;
        memcpy(out + done, t, take);
        done += take;
    }
    secure_zero(t, sizeof t);
}

// FIPS-197 §5.2 key expansion into little-endian column words (rk[i] = bytes 4i..4i+3 of the schedule).
int aes_expand_key(const uint8_t *key, size_t key_len, uint32_t rk[60]) {
    const int nk = (int)key_len / 4, rounds = nk + 6, total = 4 * (rounds + 1);
    auto sub = [](uint32_t w) {
        return (uint32_t)kSBox.v[w & 0xff] | ((uint32_t)kSBox.v[(w >> 8) & 0xff] << 8) |
               ((uint32_t)kSBox.v[(w >> 16) & 0xff] << 16) | ((uint32_t)kSBox.v[w >> 24] << 24);
    };
    for (int i = 0; i < nk; i++) memcpy(&rk[i], key + 4 * i, 4);
    uint8_t rcon = 1;
    for (int i = nk; i < total; i++) {
        uint32_t t = rk[i - 1];
        if (i % nk == 0) {
            t = sub((t >> 8) | (t << 24)) ^ rcon;  // RotWord on a little-endian image is a right rotate
            rcon = gf_mul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            t = sub(t);
        }
        rk[i] = rk[i - nk] ^ t;
    }
    return rounds;
}

}  // namespace qpp
