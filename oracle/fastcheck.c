/*
 * fastcheck.c — full-size batch checker for the GPU parity tests.  TEST INFRASTRUCTURE ONLY: never linked into
 * libqpp.so; only tests/ load it (tests/_oracle.py fast_seal_batch).
 *
 * orc_seal_batch (qpp_oracle.c) restates the algorithm byte by byte and seals ~1 MB/s: at BASELINE's full sizes
 * (1 Mi x 1200 B) the GPU tests could only compare a 1500-packet sample with it.  This file computes the same
 * batch result — nonce iv ^ pn (quic/s2n-quic-crypto/src/iv.rs:27-39), AEAD seal in place with the tag after the
 * payload (aead/default.rs:44-62), HP mask AES-ECB / ChaCha20 of the sample at header_len + 4
 * (header_key.rs:52-56, payload.rs:151-169), optional mask application (header_crypto.rs:80-95) — through OpenSSL
 * 3 EVP (the CRYPTOGAMS AES-NI / PCLMUL / ChaCha assembly aws-lc also carries) on up to 16 threads, so every packet
 * of a full-size batch is checked.  It is itself checked against the restatement (tests/test_fastcheck.py), which
 * is the pinned oracle.  Same semantics as orc_seal_batch, packet for packet.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include <openssl/evp.h>

#include "qpp_oracle.h"

typedef struct {
    const orc_key *keys;
    const orc_pkt *pkts;
    size_t lo, hi;
    uint8_t *arena, *masks;
    int flags, ok;
} fc_job;

static const EVP_CIPHER *fc_aead(int suite) {
    return suite == 1 ? EVP_aes_128_gcm() : suite == 2 ? EVP_aes_256_gcm() : EVP_chacha20_poly1305();
}

/* RFC 9001 §5.4.3 / §5.4.4: first 5 bytes of AES-ECB(hp, sample), or of ChaCha20(hp, counter = sample[0..4] LE,
 * nonce = sample[4..16]) over zeros — OpenSSL's 16-byte ChaCha20 IV is exactly counter(LE) || nonce. */
static int fc_hp_mask(EVP_CIPHER_CTX *c, const orc_key *k, const uint8_t sample[16], uint8_t mask[5]) {
    uint8_t out[32];
    int len = 0;
    if (k->suite == 3) {
        static const uint8_t zeros[16] = {0};
        if (!EVP_EncryptInit_ex(c, EVP_chacha20(), NULL, k->hp, sample)) return 0;
        if (!EVP_EncryptUpdate(c, out, &len, zeros, 16)) return 0;
    } else {
        if (!EVP_EncryptInit_ex(c, k->suite == 1 ? EVP_aes_128_ecb() : EVP_aes_256_ecb(), NULL, k->hp, NULL)) return 0;
        EVP_CIPHER_CTX_set_padding(c, 0);
        if (!EVP_EncryptUpdate(c, out, &len, sample, 16)) return 0;
    }
    memcpy(mask, out, 5);
    return 1;
}

static void *fc_worker(void *arg) {
    fc_job *j = (fc_job *)arg;
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new(), *h = EVP_CIPHER_CTX_new();
    j->ok = c && h;
    int cur = -1;
    for (size_t i = j->lo; i < j->hi && j->ok; i++) {
        const orc_pkt *p = &j->pkts[i];
        const orc_key *k = &j->keys[p->key_idx];
        uint8_t nonce[12], mask[5];
        uint8_t *base = j->arena + p->off, *pay = base + p->aad_len;
        orc_nonce(k->iv, p->pn, nonce);
        int len = 0;
        if ((int)p->key_idx != cur) {  /* key change: full init (key schedule); otherwise only the nonce */
            j->ok = EVP_EncryptInit_ex(c, fc_aead(k->suite), NULL, NULL, NULL) &&
                    EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL) &&
                    EVP_EncryptInit_ex(c, NULL, NULL, k->key, nonce);
            cur = (int)p->key_idx;
        } else {
            j->ok = EVP_EncryptInit_ex(c, NULL, NULL, NULL, nonce);
        }
        if (!j->ok) break;
        if (p->aad_len) j->ok = EVP_EncryptUpdate(c, NULL, &len, base, p->aad_len);
        if (j->ok && p->pt_len) j->ok = EVP_EncryptUpdate(c, pay, &len, pay, p->pt_len);
        if (j->ok) j->ok = EVP_EncryptFinal_ex(c, pay + p->pt_len, &len) &&
                           EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_AEAD_GET_TAG, 16, pay + p->pt_len);
        if (!j->ok) break;
        if (j->flags & 3) {
            const size_t hdr = (size_t)p->aad_len - p->pn_len;
            j->ok = fc_hp_mask(h, k, base + hdr + 4, mask);
            if (!j->ok) break;
            if (j->flags & 1) memcpy(j->masks + 5 * i, mask, 5);
            if (j->flags & 2) {  /* in place, in the reference's order (byte 0 first: a PN at offset 0 sees it) */
                base[0] ^= (uint8_t)(mask[0] & ((base[0] & 0x80) ? 0x0f : 0x1f));
                for (size_t b = 0; b < p->pn_len; b++) base[hdr + b] ^= mask[1 + b];
            }
        }
    }
    EVP_CIPHER_CTX_free(c);
    EVP_CIPHER_CTX_free(h);
    return NULL;
}

/* orc_seal_batch on `threads` threads (1..16).  Returns 1 on success, 0 if OpenSSL refused a call. */
int fc_seal_batch(const orc_key *keys, const orc_pkt *pkts, size_t n, uint8_t *arena, uint8_t *masks, int flags,
                  int threads) {
    if (threads < 1) threads = 1;
    if (threads > 16) threads = 16;
    if ((size_t)threads > n) threads = n ? (int)n : 1;
    fc_job jobs[16];
    pthread_t tid[16];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (fc_job){keys, pkts, n * t / threads, n * (t + 1) / threads, arena, masks, flags, 1};
        if (pthread_create(&tid[t], NULL, fc_worker, &jobs[t])) {
            fc_worker(&jobs[t]);
            tid[t] = 0;
        }
    }
    int ok = 1;
    for (int t = 0; t < threads; t++) {
        if (tid[t]) pthread_join(tid[t], NULL);
        ok &= jobs[t].ok;
    }
    return ok;
}
