/*
 * cpu_baseline.c — the reference's CPU path timed beside the GPU (bench.py cpu_baseline leg).
 * TEST/MEASUREMENT INFRASTRUCTURE ONLY: never linked into libqpp.so.
 *
 * What is timed is the per-packet loop the reference runs (quic/s2n-quic-crypto/src/aead/default.rs:44-93,
 * src/iv.rs:27-39, src/header_key.rs:52-56): nonce = iv ^ pn, AEAD seal in place with a 16-byte tag,
 * HP mask from the 16-byte sample; then open of the same packet.  One EVP_CIPHER_CTX per key and thread,
 * IV set per packet — the shape of dc/s2n-quic-dc-benches/src/crypto/encrypt.rs:59-82.
 *
 * aws-lc-rs (the reference's crypto) cannot be built offline; OpenSSL 3 libcrypto runs the same
 * CRYPTOGAMS AES-NI/VAES + PCLMULQDQ GCM and ChaCha20-Poly1305 assembly and is bit-exact with it on
 * the RFC 9001 vectors.  Without libcrypto the harness falls back to the (slow) oracle restatement and
 * says so via cpubase_impl().
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "qpp_oracle.h"

#ifdef HAVE_OPENSSL
#include <openssl/crypto.h>
#include <openssl/evp.h>
#endif

typedef struct {
    int suite, packets, pt_len, aad_len, with_hp;
    double seconds;
    uint64_t bytes;  /* payload bytes processed (seal + open) */
    int ok;
    int cpu;         /* pin the worker to this CPU (-1: no pinning) */
} job_t;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void fill(uint8_t *p, size_t n, uint64_t seed) {
    for (size_t i = 0; i < n; i++) {
        seed = seed * 6364136223846793005ULL + 1442695040888963407ULL;
        p[i] = (uint8_t)(seed >> 56);
    }
}

#ifdef HAVE_OPENSSL
static const EVP_CIPHER *aead(int suite) {
    return suite == 1 ? EVP_aes_128_gcm() : suite == 2 ? EVP_aes_256_gcm() : EVP_chacha20_poly1305();
}
#endif

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    if (j->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(j->cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof set, &set);
    }
    const int stride = j->aad_len + j->pt_len + 16;
    uint8_t *arena = malloc((size_t)stride * j->packets);
    uint8_t key[32], iv[12], hp[32];
    fill(arena, (size_t)stride * j->packets, 0x5eed0001);
    fill(key, 32, 1); fill(iv, 12, 2); fill(hp, 32, 3);
    j->bytes = 0;
    j->ok = 1;
    double t0 = now_s();
    uint64_t pn = 0;
#ifdef HAVE_OPENSSL
    EVP_CIPHER_CTX *enc = EVP_CIPHER_CTX_new(), *dec = EVP_CIPHER_CTX_new(), *hpc = EVP_CIPHER_CTX_new();
    EVP_EncryptInit_ex(enc, aead(j->suite), NULL, NULL, NULL);
    EVP_CIPHER_CTX_ctrl(enc, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL);
    EVP_EncryptInit_ex(enc, NULL, NULL, key, NULL);
    EVP_DecryptInit_ex(dec, aead(j->suite), NULL, NULL, NULL);
    EVP_CIPHER_CTX_ctrl(dec, EVP_CTRL_AEAD_SET_IVLEN, 12, NULL);
    EVP_DecryptInit_ex(dec, NULL, NULL, key, NULL);
    if (j->suite == 3) EVP_EncryptInit_ex(hpc, EVP_chacha20(), NULL, hp, NULL);
    else { EVP_EncryptInit_ex(hpc, j->suite == 1 ? EVP_aes_128_ecb() : EVP_aes_256_ecb(), NULL, hp, NULL); EVP_CIPHER_CTX_set_padding(hpc, 0); }
#endif
    do {
        for (int i = 0; i < j->packets; i++, pn++) {
            uint8_t *p = arena + (size_t)stride * i, *pay = p + j->aad_len, nonce[12], mask[16];
            orc_nonce(iv, pn, nonce);
#ifdef HAVE_OPENSSL
            int outl;
            EVP_EncryptInit_ex(enc, NULL, NULL, NULL, nonce);
            EVP_EncryptUpdate(enc, NULL, &outl, p, j->aad_len);
            EVP_EncryptUpdate(enc, pay, &outl, pay, j->pt_len);
            EVP_EncryptFinal_ex(enc, pay + j->pt_len, &outl);
            EVP_CIPHER_CTX_ctrl(enc, EVP_CTRL_AEAD_GET_TAG, 16, pay + j->pt_len);
            if (j->with_hp) {
                if (j->suite == 3) {
                    uint8_t zero[5] = {0};
                    EVP_EncryptInit_ex(hpc, NULL, NULL, NULL, pay);  /* IV = LE32 ctr || nonce = sample */
                    EVP_EncryptUpdate(hpc, mask, &outl, zero, 5);
                } else {
                    EVP_EncryptUpdate(hpc, mask, &outl, pay, 16);
                }
                p[0] ^= mask[0] & 0x1f;
            }
            if (j->with_hp) p[0] ^= mask[0] & 0x1f;  /* receiver removes HP before opening */
            EVP_DecryptInit_ex(dec, NULL, NULL, NULL, nonce);
            EVP_DecryptUpdate(dec, NULL, &outl, p, j->aad_len);
            EVP_DecryptUpdate(dec, pay, &outl, pay, j->pt_len);
            EVP_CIPHER_CTX_ctrl(dec, EVP_CTRL_AEAD_SET_TAG, 16, pay + j->pt_len);
            if (EVP_DecryptFinal_ex(dec, pay + j->pt_len, &outl) <= 0) j->ok = 0;
#else
            if (orc_seal(j->suite, key, nonce, p, j->aad_len, pay, j->pt_len)) j->ok = 0;
            if (j->with_hp) orc_hp_mask(j->suite, hp, pay, mask);
            if (orc_open(j->suite, key, nonce, p, j->aad_len, pay, j->pt_len + 16)) j->ok = 0;
#endif
            j->bytes += 2ull * j->pt_len;
        }
    } while (now_s() - t0 < j->seconds);
    j->seconds = now_s() - t0;
#ifdef HAVE_OPENSSL
    EVP_CIPHER_CTX_free(enc); EVP_CIPHER_CTX_free(dec); EVP_CIPHER_CTX_free(hpc);
#endif
    free(arena);
    return NULL;
}

const char *cpubase_impl(void) {
#ifdef HAVE_OPENSSL
    return OpenSSL_version(OPENSSL_VERSION);
#else
    return "oracle restatement (no libcrypto)";
#endif
}

/* Runs `threads` workers, each looping over its own `packets` x pt_len batch for >= `seconds`; worker t is pinned to
 * cpus[t] when cpus is non-NULL (one worker per physical core: bench.py picks them).
 * Returns aggregate seal+open payload throughput in GiB/s (2^30 B/s); *ok = 1 if every open verified. */
double cpubase_run(int suite, int threads, int packets, int pt_len, int aad_len, int with_hp, double seconds, int *ok,
                   const int *cpus) {
    pthread_t *tid = calloc((size_t)threads, sizeof *tid);
    job_t *jobs = calloc((size_t)threads, sizeof *jobs);
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){suite, packets, pt_len, aad_len, with_hp, seconds, 0, 0, cpus ? cpus[t] : -1};
        pthread_create(&tid[t], NULL, worker, &jobs[t]);
    }
    double total = 0, tmax = 0;
    int all_ok = 1;
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        total += (double)jobs[t].bytes;
        if (jobs[t].seconds > tmax) tmax = jobs[t].seconds;
        all_ok &= jobs[t].ok;
    }
    free(tid);
    free(jobs);
    if (ok) *ok = all_ok;
    return total / tmax / (double)(1ull << 30);
}

/* The CPU's raw AEAD seal rate on one thread: one `msg_len`-byte message sealed over and over (no per-packet
 * nonce set-up, no HP, no open) -- the AES-NI/VAES + (V)PCLMULQDQ kernel alone, to separate it from the per-packet
 * EVP overhead that the packet loop above pays (GiB/s).  Runs on its own pinned thread. */
typedef struct {
    int suite, msg_len, cpu;
    double seconds, gibs;
} bulk_t;

static void *bulk_worker(void *arg) {
    bulk_t *b = (bulk_t *)arg;
    if (b->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(b->cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof set, &set);
    }
    uint8_t *buf = malloc((size_t)b->msg_len + 16), key[32], nonce[12] = {0};
    fill(buf, (size_t)b->msg_len, 9);
    fill(key, 32, 1);
    uint64_t bytes = 0;
    double t0 = now_s();
#ifdef HAVE_OPENSSL
    EVP_CIPHER_CTX *enc = EVP_CIPHER_CTX_new();
    EVP_EncryptInit_ex(enc, aead(b->suite), NULL, key, nonce);
    int outl;
    do {
        for (int r = 0; r < 64; r++) {
            EVP_EncryptInit_ex(enc, NULL, NULL, NULL, nonce);
            EVP_EncryptUpdate(enc, buf, &outl, buf, b->msg_len);
            EVP_EncryptFinal_ex(enc, buf + b->msg_len, &outl);
            bytes += (uint64_t)b->msg_len;
        }
    } while (now_s() - t0 < b->seconds);
    EVP_CIPHER_CTX_free(enc);
#endif
    b->gibs = (double)bytes / (now_s() - t0) / (double)(1ull << 30);
    free(buf);
    return NULL;
}

double cpubase_bulk_seal(int suite, int msg_len, double seconds, int cpu) {
    bulk_t b = {suite, msg_len, cpu, seconds, 0.0};
    pthread_t t;
    if (pthread_create(&t, NULL, bulk_worker, &b)) return 0.0;
    pthread_join(t, NULL);
    return b.gibs;
}
