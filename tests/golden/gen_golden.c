/*
 * gen_golden.c — generates the golden fixtures (tests/golden, one .json per family).
 *
 * The reference's arithmetic lives in aws-lc-rs ^1.12 (quic/s2n-quic-crypto/Cargo.toml:19),
 * which is not vendored and cannot be built offline.  OpenSSL 3.0.2 libcrypto (present in
 * this image) implements the same standardized functions; it reproduces the RFC 9001
 * Appendix A vectors bit-exactly (tests/test_oracle_golden.py checks that too), so it is
 * used here as an independent stand-in to produce vectors for the cases the reference's own
 * tests do not pin (AES-256-GCM, ChaCha20-Poly1305 seal/open, odd lengths, key updates).
 *
 * Build + run: sh tests/golden/generate.sh   (needs /usr/include/openssl; not needed to run tests)
 *
 * Deterministic: xorshift64* seeded per file.
 */
#include <openssl/core_names.h>
#include <openssl/evp.h>
#include <openssl/kdf.h>
#include <openssl/params.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t rng_state;
static uint64_t rng(void) {
    uint64_t x = rng_state;
    x ^= x >> 12; x ^= x << 25; x ^= x >> 27;
    rng_state = x;
    return x * 0x2545F4914F6CDD1DULL;
}
static void rand_bytes(uint8_t *p, size_t n) { for (size_t i = 0; i < n; i++) p[i] = (uint8_t)(rng() >> 56); }

static void hex(FILE *f, const uint8_t *p, size_t n) {
    fputc('"', f);
    for (size_t i = 0; i < n; i++) fprintf(f, "%02x", p[i]);
    fputc('"', f);
}

static void die(const char *m) { fprintf(stderr, "gen_golden: %s\n", m); exit(1); }

static const EVP_CIPHER *aead_cipher(int suite) {
    return suite == 1 ? EVP_aes_128_gcm() : suite == 2 ? EVP_aes_256_gcm() : EVP_chacha20_poly1305();
}
static size_t key_len(int suite) { return suite == 1 ? 16 : 32; }

static void seal(int suite, const uint8_t *key, const uint8_t nonce[12], const uint8_t *aad, size_t aad_len,
                 const uint8_t *pt, size_t len, uint8_t *ct, uint8_t tag[16]) {
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    int outl;
    if (!EVP_EncryptInit_ex(c, aead_cipher(suite), NULL, NULL, NULL)) die("init");
    if (!EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL)) die("ivlen");
    if (!EVP_EncryptInit_ex(c, NULL, NULL, key, nonce)) die("key");
    if (aad_len && !EVP_EncryptUpdate(c, NULL, &outl, aad, (int)aad_len)) die("aad");
    if (len && !EVP_EncryptUpdate(c, ct, &outl, pt, (int)len)) die("pt");
    if (!EVP_EncryptFinal_ex(c, ct + len, &outl)) die("final");
    if (!EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_GET_TAG, 16, tag)) die("tag");
    EVP_CIPHER_CTX_free(c);
}

static void hp_mask(int suite, const uint8_t *hp, const uint8_t sample[16], uint8_t mask[5]) {
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    uint8_t out[32] = {0}, zero[16] = {0};
    int outl;
    if (suite == 3) {
        /* EVP_chacha20 IV = LE32 counter || 96-bit nonce == the 16-byte sample itself */
        if (!EVP_EncryptInit_ex(c, EVP_chacha20(), NULL, hp, sample)) die("chacha");
        if (!EVP_EncryptUpdate(c, out, &outl, zero, 5)) die("chacha upd");
    } else {
        if (!EVP_EncryptInit_ex(c, suite == 1 ? EVP_aes_128_ecb() : EVP_aes_256_ecb(), NULL, hp, NULL)) die("ecb");
        EVP_CIPHER_CTX_set_padding(c, 0);
        if (!EVP_EncryptUpdate(c, out, &outl, sample, 16)) die("ecb upd");
    }
    memcpy(mask, out, 5);
    EVP_CIPHER_CTX_free(c);
}

static void expand_label(const char *md, const uint8_t *secret, size_t slen, const char *label,
                         uint8_t *out, size_t out_len) {
    uint8_t info[64];
    size_t ll = strlen(label);
    info[0] = (uint8_t)(out_len >> 8); info[1] = (uint8_t)out_len; info[2] = (uint8_t)(6 + ll);
    memcpy(info + 3, "tls13 ", 6); memcpy(info + 9, label, ll); info[9 + ll] = 0;
    EVP_KDF *kdf = EVP_KDF_fetch(NULL, "HKDF", NULL);
    EVP_KDF_CTX *k = EVP_KDF_CTX_new(kdf);
    int mode = EVP_KDF_HKDF_MODE_EXPAND_ONLY;
    OSSL_PARAM p[5];
    p[0] = OSSL_PARAM_construct_utf8_string(OSSL_KDF_PARAM_DIGEST, (char *)md, 0);
    p[1] = OSSL_PARAM_construct_octet_string(OSSL_KDF_PARAM_KEY, (void *)secret, slen);
    p[2] = OSSL_PARAM_construct_octet_string(OSSL_KDF_PARAM_INFO, info, 10 + ll);
    p[3] = OSSL_PARAM_construct_int(OSSL_KDF_PARAM_MODE, &mode);
    p[4] = OSSL_PARAM_construct_end();
    if (EVP_KDF_derive(k, out, out_len, p) <= 0) die("hkdf");
    EVP_KDF_CTX_free(k);
    EVP_KDF_free(kdf);
}

static void nonce_of(const uint8_t iv[12], uint64_t pn, uint8_t nonce[12]) {
    memset(nonce, 0, 4);
    for (int i = 0; i < 8; i++) nonce[4 + i] = (uint8_t)(pn >> (56 - 8 * i));
    for (int i = 0; i < 12; i++) nonce[i] ^= iv[i];
}

static void gen_aead(int suite, const char *path) {
    static const size_t lens[] = {0, 1, 2, 15, 16, 17, 20, 31, 32, 33, 47, 48, 63, 64, 65, 100,
                                  127, 128, 129, 255, 256, 300, 1000, 1162, 1200, 1452, 8000};
    static const size_t aads[] = {0, 6, 21, 22, 13, 1, 16, 33};
    FILE *f = fopen(path, "w");
    if (!f) die("open");
    rng_state = 0x5eed0000ULL + (uint64_t)suite * 7919;
    fprintf(f, "{\"suite\": %d, \"generator\": \"OpenSSL %s EVP (tests/golden/gen_golden.c)\", \"cases\": [\n",
            suite, OPENSSL_VERSION_STR);
    size_t ncase = sizeof lens / sizeof lens[0] + 8;
    for (size_t ci = 0; ci < ncase; ci++) {
        size_t len = ci < sizeof lens / sizeof lens[0] ? lens[ci] : (size_t)(rng() % 1500);
        size_t aad_len = aads[ci % (sizeof aads / sizeof aads[0])];
        uint8_t key[32], iv[12], nonce[12], aad[64], tag[16];
        uint8_t *pt = malloc(len + 1), *ct = malloc(len + 16);
        rand_bytes(key, key_len(suite));
        rand_bytes(iv, 12);
        rand_bytes(aad, aad_len);
        rand_bytes(pt, len);
        uint64_t pn = (ci & 1) ? (rng() & ((1ULL << 62) - 1)) : (rng() & 0xffffffffULL);
        nonce_of(iv, pn, nonce);
        seal(suite, key, nonce, aad, aad_len, pt, len, ct, tag);
        fprintf(f, " {\"key\": "); hex(f, key, key_len(suite));
        fprintf(f, ", \"iv\": "); hex(f, iv, 12);
        fprintf(f, ", \"pn\": %llu", (unsigned long long)pn);
        fprintf(f, ", \"nonce\": "); hex(f, nonce, 12);
        fprintf(f, ", \"aad\": "); hex(f, aad, aad_len);
        fprintf(f, ", \"pt\": "); hex(f, pt, len);
        fprintf(f, ", \"ct\": "); hex(f, ct, len);
        fprintf(f, ", \"tag\": "); hex(f, tag, 16);
        fprintf(f, "}%s\n", ci + 1 < ncase ? "," : "");
        free(pt); free(ct);
    }
    fprintf(f, "]}\n");
    fclose(f);
}

static void gen_hp(const char *path) {
    FILE *f = fopen(path, "w");
    if (!f) die("open");
    rng_state = 0x5eed00ffULL;
    fprintf(f, "{\"generator\": \"OpenSSL %s EVP (tests/golden/gen_golden.c)\", \"cases\": [\n", OPENSSL_VERSION_STR);
    int first = 1;
    for (int suite = 1; suite <= 3; suite++)
        for (int i = 0; i < 24; i++) {
            uint8_t hp[32], sample[16], mask[5];
            rand_bytes(hp, key_len(suite));
            rand_bytes(sample, 16);
            if (i == 0) memset(sample, 0, 16);
            if (i == 1) memset(sample, 0xff, 16);
            hp_mask(suite, hp, sample, mask);
            fprintf(f, "%s {\"suite\": %d, \"hp\": ", first ? "" : ",\n", suite); hex(f, hp, key_len(suite));
            fprintf(f, ", \"sample\": "); hex(f, sample, 16);
            fprintf(f, ", \"mask\": "); hex(f, mask, 5);
            fputc('}', f);
            first = 0;
        }
    fprintf(f, "\n]}\n");
    fclose(f);
}

static void gen_kdf(const char *path) {
    FILE *f = fopen(path, "w");
    if (!f) die("open");
    rng_state = 0x5eed0abcULL;
    fprintf(f, "{\"generator\": \"OpenSSL %s HKDF (tests/golden/gen_golden.c)\", \"chains\": [\n", OPENSSL_VERSION_STR);
    int first = 1;
    for (int suite = 1; suite <= 3; suite++)
        for (int i = 0; i < 4; i++) {
            const char *md = suite == 2 ? "SHA384" : "SHA256";
            size_t hl = suite == 2 ? 48 : 32, kl = key_len(suite);
            uint8_t secret[48];
            rand_bytes(secret, hl);
            fprintf(f, "%s {\"suite\": %d, \"secret\": ", first ? "" : ",\n", suite); hex(f, secret, hl);
            fprintf(f, ", \"steps\": [");
            for (int step = 0; step < 4; step++) {
                uint8_t key[32], iv[12], hp[32], next[48];
                expand_label(md, secret, hl, "quic key", key, kl);
                expand_label(md, secret, hl, "quic iv", iv, 12);
                expand_label(md, secret, hl, "quic hp", hp, kl);
                fprintf(f, "%s{\"secret\": ", step ? ", " : ""); hex(f, secret, hl);
                fprintf(f, ", \"key\": "); hex(f, key, kl);
                fprintf(f, ", \"iv\": "); hex(f, iv, 12);
                fprintf(f, ", \"hp\": "); hex(f, hp, kl);
                fputc('}', f);
                expand_label(md, secret, hl, "quic ku", next, hl);
                memcpy(secret, next, hl);
            }
            fprintf(f, "]}");
            first = 0;
        }
    fprintf(f, "\n]}\n");
    fclose(f);
}

int main(int argc, char **argv) {
    const char *dir = argc > 1 ? argv[1] : "tests/golden";
    char p[512];
    snprintf(p, sizeof p, "%s/aead_aes128gcm.json", dir); gen_aead(1, p);
    snprintf(p, sizeof p, "%s/aead_aes256gcm.json", dir); gen_aead(2, p);
    snprintf(p, sizeof p, "%s/aead_chacha20poly1305.json", dir); gen_aead(3, p);
    snprintf(p, sizeof p, "%s/hp_masks.json", dir); gen_hp(p);
    snprintf(p, sizeof p, "%s/kdf_chains.json", dir); gen_kdf(p);
    return 0;
}
