// host_check.cpp — ASan/UBSan run over the engine's host-side C/C++ (TEST INFRASTRUCTURE):
//   * kdf.cpp: SHA-2 / HMAC / HKDF-Expand-Label / AES key expansion of the engine's host key schedule,
//     cross-checked against the oracle (oracle/qpp_oracle.c) on RFC 9001 A.1 and on random secrets;
//   * qpp_internal.h decode_packet_number (host copy of the receive path's PN expansion) against the oracle;
//   * the oracle itself: seal -> open round trips over ragged lengths, all three suites.
// Built with -fsanitize=address,undefined by tests/sanitize/Makefile; any report aborts with a non-zero status.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "../../oracle/qpp_oracle.h"
#include "../../s2n-quic_amd/csrc/qpp_internal.h"

#define CHECK(c)                                                           \
    do {                                                                   \
        if (!(c)) {                                                        \
            fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c); \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

static void hex(const char *s, uint8_t *out) {
    for (size_t i = 0; s[2 * i]; i++) sscanf(s + 2 * i, "%2hhx", &out[i]);
}

int main() {
    std::mt19937_64 rng(0x5a17);
    auto fill = [&](uint8_t *p, size_t n) {
        for (size_t i = 0; i < n; i++) p[i] = (uint8_t)rng();
    };
    // RFC 9001 A.1: initial secrets from the DCID 8394c8f03e515708 (quic/s2n-quic-crypto/src/initial.rs tests)
    uint8_t dcid[8], salt[20], prk[32], client[32], oc[32], os_[32];
    hex("8394c8f03e515708", dcid);
    hex("38762cf7f55934b34d179ae6a4c80cadccbb7f0a", salt);
    qpp::hkdf_extract(32, salt, 20, dcid, 8, prk);
    qpp::hkdf_expand_label(32, prk, "client in", client, 32);
    orc_initial_secrets(dcid, 8, oc, os_);
    CHECK(memcmp(client, oc, 32) == 0);
    uint8_t want_key[16];
    hex("1f369613dd76d5467730efcbe3b1a22d", want_key);
    uint8_t key[32];
    qpp::hkdf_expand_label(32, client, "quic key", key, 16);
    CHECK(memcmp(key, want_key, 16) == 0);
    // random secrets, every suite: host key schedule == oracle; AES expansion == oracle's
    for (int it = 0; it < 300; it++) {
        const int suite = 1 + it % 3;
        const size_t hl = qpp::suite_hash_len(suite), kl = qpp::suite_key_len(suite);
        uint8_t secret[48], k1[32], iv1[12], hp1[32], k2[32], iv2[12], hp2[32], nxt1[48], nxt2[48];
        fill(secret, hl);
        qpp::hkdf_expand_label(hl, secret, "quic key", k1, kl);
        qpp::hkdf_expand_label(hl, secret, "quic iv", iv1, 12);
        qpp::hkdf_expand_label(hl, secret, "quic hp", hp1, kl);
        CHECK(orc_derive(suite, secret, k2, iv2, hp2) == 0);
        CHECK(!memcmp(k1, k2, kl) && !memcmp(iv1, iv2, 12) && !memcmp(hp1, hp2, kl));
        qpp::hkdf_expand_label(hl, secret, "quic ku", nxt1, hl);
        CHECK(orc_update_secret(suite, secret, nxt2) == 0);
        CHECK(!memcmp(nxt1, nxt2, hl));
        if (suite != 3) {
            uint32_t rk[60];
            uint8_t ork[240];
            const int nr = qpp::aes_expand_key(k1, kl, rk);
            CHECK(nr == orc_aes_expand(k1, kl, ork));
            CHECK(memcmp(rk, ork, 16 * (size_t)(nr + 1)) == 0);  // little-endian column words == byte order
        }
        qpp::secure_zero(secret, sizeof secret);
    }
    // receive-side PN expansion: host copy == oracle (RFC 9000 A.3), including edges near 2^62
    for (int it = 0; it < 200000; it++) {
        const unsigned bits = 8u * (1u + (unsigned)(rng() % 4));
        uint64_t largest = rng() & ((1ull << 62) - 1);
        if (it % 7 == 0) largest = (1ull << 62) - 1 - (rng() % 70000);
        if (it % 11 == 0) largest = rng() % 70000;
        const uint64_t trunc = rng() & ((1ull << bits) - 1);
        CHECK(qpp::decode_packet_number(largest, trunc, bits) == orc_decode_packet_number(largest, trunc, bits));
    }
    // oracle seal -> open round trips (ragged lengths incl. 0 and partial blocks), tamper -> reject
    for (int it = 0; it < 400; it++) {
        const int suite = 1 + it % 3;
        const size_t kl = orc_suite_key_len(suite), aad_len = rng() % 40, pt_len = it < 40 ? (size_t)it : rng() % 1500;
        std::vector<uint8_t> k(kl), aad(aad_len), buf(pt_len + 16), orig;
        uint8_t nonce[12];
        fill(k.data(), kl);
        fill(aad.data(), aad_len);
        fill(buf.data(), pt_len);
        fill(nonce, 12);
        orig.assign(buf.begin(), buf.begin() + (long)pt_len);
        CHECK(orc_seal(suite, k.data(), nonce, aad.data(), aad_len, buf.data(), pt_len) == 0);
        std::vector<uint8_t> bad = buf;
        bad[rng() % bad.size()] ^= 1;
        CHECK(orc_open(suite, k.data(), nonce, aad.data(), aad_len, bad.data(), bad.size()) != 0);
        CHECK(orc_open(suite, k.data(), nonce, aad.data(), aad_len, buf.data(), buf.size()) == 0);
        CHECK(pt_len == 0 || memcmp(buf.data(), orig.data(), pt_len) == 0);
    }
    printf("host_check ok\n");
    return 0;
}
