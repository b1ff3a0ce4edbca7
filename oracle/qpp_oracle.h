/*
 * qpp_oracle.h — CPU restatement of the QUIC packet-protection hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the *checker* for the MI355X
 * engine (s2n-quic_amd/).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product library (libqpp.so)
 * never links, calls or falls back to anything in oracle/.
 *
 * What it restates (reference = aws/s2n-quic 0.88.0 at /root/reference):
 *   - nonce = iv XOR (0u32 || pn_be64)          quic/s2n-quic-crypto/src/iv.rs:27-39
 *   - AEAD seal/open (AES-128/256-GCM, ChaCha20-Poly1305), tag appended after
 *     the payload, open = split tag + verify      quic/s2n-quic-crypto/src/cipher_suite.rs:116-156,
 *                                                 quic/s2n-quic-crypto/src/aead/default.rs:44-93
 *   - header-protection mask (5 bytes)          quic/s2n-quic-crypto/src/header_key.rs:52-56
 *     AES: AES-ECB(hp, sample)[0..5]; ChaCha: ChaCha20(hp, ctr=LE32(sample[0..4]),
 *     nonce=sample[4..16]) over 5 zero bytes    specs/.../rfc9001.txt:1323-1360
 *   - apply/remove header protection            quic/s2n-quic-core/src/crypto/header_crypto.rs:80-123
 *   - HKDF-Expand-Label derivation of key/iv/hp and "quic ku" update
 *                                               quic/s2n-quic-crypto/src/cipher_suite.rs:52-104,
 *                                               quic/s2n-quic-core/src/crypto/label.rs:57-68
 *   - Initial secrets (salt + "client in"/"server in")
 *                                               quic/s2n-quic-crypto/src/initial.rs:29-68
 *
 * The arithmetic itself lives in aws-lc-rs ^1.12 (quic/s2n-quic-crypto/Cargo.toml:19),
 * which is not vendored (no Cargo.lock, no sources under /root/reference) and
 * cannot be built here (no Rust toolchain).  This file restates the published
 * algorithms (FIPS-197 AES, NIST SP 800-38D GCM, RFC 8439 ChaCha20-Poly1305,
 * FIPS 180-4 SHA-2, RFC 2104 HMAC, RFC 5869 HKDF, RFC 8446 §7.1 Expand-Label).
 * It is pinned by the RFC 9001 Appendix A vectors held in the reference's own
 * files and by OpenSSL-generated fixtures (tests/golden/).
 */
#ifndef QPP_ORACLE_H
#define QPP_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Suite ids match include/qpp.h (QPP_SUITE_*). */
enum {
    ORC_AES_128_GCM_SHA256 = 1,
    ORC_AES_256_GCM_SHA384 = 2,
    ORC_CHACHA20_POLY1305_SHA256 = 3,
};

/* Status codes match include/qpp.h / packet_protection::Error. */
enum { ORC_OK = 0, ORC_DECODE_ERROR = 1, ORC_DECRYPT_ERROR = 2, ORC_INTERNAL_ERROR = 3 };

/* ---- primitives ---- */
int  orc_aes_expand(const uint8_t *key, size_t key_len, uint8_t rk[240]); /* returns rounds */
void orc_aes_encrypt_block(const uint8_t rk[240], int rounds, const uint8_t in[16], uint8_t out[16]);
void orc_ghash_mul(uint8_t x[16], const uint8_t h[16]);               /* x = x * h in GF(2^128) */
void orc_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], uint8_t out[64]);
void orc_poly1305(const uint8_t key[32], const uint8_t *msg, size_t len, uint8_t tag[16]);

void orc_sha256(const uint8_t *msg, size_t len, uint8_t out[32]);
void orc_sha384(const uint8_t *msg, size_t len, uint8_t out[48]);
/* hash_len 32 -> SHA-256, 48 -> SHA-384 */
void orc_hmac(size_t hash_len, const uint8_t *key, size_t key_len, const uint8_t *msg, size_t len, uint8_t *out);
void orc_hkdf_extract(size_t hash_len, const uint8_t *salt, size_t salt_len, const uint8_t *ikm, size_t ikm_len, uint8_t *prk);
void orc_hkdf_expand(size_t hash_len, const uint8_t *prk, const uint8_t *info, size_t info_len, uint8_t *out, size_t out_len);
void orc_hkdf_expand_label(size_t hash_len, const uint8_t *secret, const char *label, uint8_t *out, size_t out_len);

/* ---- suite-level (quic/s2n-quic-crypto) ---- */
size_t orc_suite_key_len(int suite);   /* 16 or 32 */
size_t orc_suite_hash_len(int suite);  /* 32 or 48 */
void   orc_nonce(const uint8_t iv[12], uint64_t pn, uint8_t nonce[12]);
/* key/iv/hp from a traffic secret (TLS_*::new) */
int    orc_derive(int suite, const uint8_t *secret, uint8_t *key, uint8_t iv[12], uint8_t *hp);
/* secret' = HKDF-Expand-Label(secret, "quic ku", "", Hash.length) (TLS_*::update) */
int    orc_update_secret(int suite, const uint8_t *secret, uint8_t *next_secret);
/* Initial secrets from the client DCID (initial.rs) */
void   orc_initial_secrets(const uint8_t *dcid, size_t dcid_len, uint8_t client[32], uint8_t server[32]);

/* AEAD with the appended-tag layout of Key::encrypt / Key::decrypt.
 * seal: buf[0..pt_len) plaintext -> ciphertext, tag written to buf[pt_len..pt_len+16).
 * open: buf[0..ct_tag_len) = ct||tag; on success buf[0..ct_tag_len-16) = plaintext.
 *       returns ORC_DECRYPT_ERROR on short input or bad tag (buffer zeroed on bad tag). */
int orc_seal(int suite, const uint8_t *key, const uint8_t nonce[12],
             const uint8_t *aad, size_t aad_len, uint8_t *buf, size_t pt_len);
int orc_open(int suite, const uint8_t *key, const uint8_t nonce[12],
             const uint8_t *aad, size_t aad_len, uint8_t *buf, size_t ct_tag_len);
void orc_hp_mask(int suite, const uint8_t *hp_key, const uint8_t sample[16], uint8_t mask[5]);

/* ---- packet level (crypto::{encrypt,protect,unprotect,decrypt}) ----
 * pkt = header (header_len bytes, PN not included) || pn bytes (pn_len) || payload || tag.
 * protect: seal payload with aad = header||pn, then apply HP with the sample at header_len+4. */
int orc_protect_packet(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp,
                       uint64_t pn, uint8_t *pkt, size_t header_len, size_t pn_len, size_t payload_len);
/* unprotect: remove HP (pn_len decoded from byte 0), decrypt.  *pn_len_out and the truncated
 * packet number bytes are returned; full_pn must be supplied by the caller (PN expansion is
 * out of scope).  Returns ORC_OK / ORC_DECRYPT_ERROR / ORC_DECODE_ERROR. */
int orc_unprotect_packet(int suite, const uint8_t *key, const uint8_t iv[12], const uint8_t *hp,
                         uint64_t full_pn, uint8_t *pkt, size_t header_len, size_t pkt_len,
                         size_t *pn_len_out);

/* ---- batch form (mirrors qpp_seal_batch / qpp_open_batch semantics, host arrays) ----
 * Descriptor layout is identical to qpp_pkt in include/qpp.h. */
typedef struct orc_pkt {
    uint64_t pn;
    uint32_t key_idx;
    uint32_t off;
    uint16_t aad_len;
    uint16_t pt_len;
    uint8_t  pn_len;
    uint8_t  flags;
    uint16_t reserved;
} orc_pkt;

typedef struct orc_key {
    int     suite;
    uint8_t key[32];
    uint8_t iv[12];
    uint8_t hp[32];
} orc_key;

/* flags bit 0: write 5-byte mask to masks[5*i]; bit 1: apply mask to the header in place */
void orc_seal_batch(const orc_key *keys, const orc_pkt *pkts, size_t n, uint8_t *arena,
                    uint8_t *masks, int flags);
void orc_open_batch(const orc_key *keys, const orc_pkt *pkts, size_t n, uint8_t *arena, int8_t *status);
/* FIPS mode (aws-lc TLS 1.3 AEAD sealing nonce order, see qpp_oracle.c) */
typedef struct orc_fips_state {
    uint64_t mask, min_next;
    int seen, pad;
} orc_fips_state;
int orc_fips_seal_ok(orc_fips_state *st, const uint8_t nonce[12]);
void orc_seal_batch_fips(const orc_key *keys, const uint8_t *fips, orc_fips_state *states, const orc_pkt *pkts,
                         size_t n, uint8_t *arena, uint8_t *masks, int flags, int8_t *status);

/* ---- packet numbers (quic/s2n-quic-core/src/packet/number) ---- */
/* RFC 9000 A.3 DecodePacketNumber, as rfc_decoder in packet/number/tests.rs:108-159 states it, clamped to
 * VarInt::MAX (tests.rs:189-194; mod.rs:235). */
uint64_t orc_decode_packet_number(uint64_t largest_pn, uint64_t truncated_pn, unsigned pn_nbits);
/* PacketNumber::truncate (packet_number.rs:135-143, mod.rs:81-93, packet_number_len.rs:163-172).
 * Returns ORC_DECODE_ERROR when pn < largest or the range needs more than 4 bytes. */
int orc_truncate_packet_number(uint64_t pn, uint64_t largest_pn, uint64_t *truncated, size_t *pn_len);

/* ---- receive batch (mirrors qpp_unprotect_open_batch; qpp_rx_pkt layout) ---- */
typedef struct orc_rx_pkt {
    uint64_t largest_pn;
    uint32_t key_idx[2];
    uint32_t off;
    uint16_t header_len;
    uint16_t len;
} orc_rx_pkt;
/* per packet: crypto::unprotect (mod.rs:195-204) -> TruncatedPacketNumber::expand -> key by key phase
 * (keyset.rs:113-143) -> crypto::decrypt (mod.rs:251-264); out[i] / status[i] as the ABI documents */
void orc_unprotect_open_batch(const orc_key *keys, const orc_rx_pkt *rx, size_t n, uint8_t *arena, orc_pkt *out,
                              int8_t *status);

#ifdef __cplusplus
}
#endif
#endif
