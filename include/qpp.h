/*
 * qpp.h — C ABI of the MI355X QUIC packet-protection engine (libqpp.so).
 *
 * Drop-in boundary for quic/s2n-quic-crypto (aws/s2n-quic 0.88.0).  Each entry point names the
 * reference interface it replaces (paths relative to the reference repository root).
 *
 * Two faces, as SURVEY.md §8(b) describes:
 *   - per-packet functions mirroring the Key / HeaderKey / OneRttKey traits
 *     (quic/s2n-quic-core/src/crypto/{key.rs:8-35, header_crypto.rs:11-31, one_rtt.rs:11-14});
 *     each one is a batch of one run on the GPU (synchronous);
 *   - batch functions over device-resident packet arenas, which the kernels and bench use.
 *
 * Rules: no exceptions cross the ABI; plain pointers and sizes only; a qpp_ctx is used by one
 * host thread at a time and owns one GPU; a qpp_key may be used from one thread at a time
 * (the traits are Send, not Sync).  All memory passed in is owned by the caller.
 *
 * Asynchrony: batch calls are asynchronous on the stream they are given.  Freeing a key (or header key) is
 * stream-ordered: its device record is zeroized after every batch already enqueued on any stream of the context,
 * and its slot is reused only after that, so a key may be freed while batches that use it are still in flight.
 * Each stream gets its own plan scratch, so batches on different streams of one context may overlap.
 */
#ifndef QPP_H
#define QPP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QPP_ABI_VERSION 2

/* Cipher suites (quic/s2n-quic-crypto/src/cipher_suite.rs:250-301). */
typedef enum qpp_suite {
    QPP_SUITE_TLS_AES_128_GCM_SHA256 = 1,
    QPP_SUITE_TLS_AES_256_GCM_SHA384 = 2,
    QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256 = 3,
} qpp_suite;

/* Return codes (quic/s2n-quic-core/src/crypto/packet_protection.rs:24-40), plus two the ABI needs. */
typedef enum qpp_status {
    QPP_OK = 0,
    QPP_DECODE_ERROR = 1,   /* packet_protection::Error::DECODE_ERROR (e.g. sample out of range) */
    QPP_DECRYPT_ERROR = 2,  /* packet_protection::Error::DECRYPT_ERROR (bad tag / short input) */
    QPP_INTERNAL_ERROR = 3, /* packet_protection::Error::INTERNAL_ERROR (seal failure, bad capacity) */
    QPP_UNSUPPORTED = 4,    /* NegotiatedCipherSuite::new returned None (cipher_suite/negotiated.rs:52-68) */
    QPP_DEVICE_ERROR = 5,   /* no MI355X / HIP runtime failure: the engine fails loudly, never falls back */
    QPP_ROTATION_NOT_SUPPORTED = 6, /* dc open::Error::RotationNotSupported (dc/s2n-quic-dc/src/crypto.rs:59-66) */
} qpp_status;

typedef enum qpp_endpoint { QPP_ENDPOINT_CLIENT = 0, QPP_ENDPOINT_SERVER = 1 } qpp_endpoint;

typedef struct qpp_ctx qpp_ctx;
typedef struct qpp_key qpp_key;
typedef struct qpp_header_key qpp_header_key;

/* ------------------------------------------------------------------ context (one per GPU) */

/* Opens GPU `device` (HIP ordinal).  QPP_DEVICE_ERROR if there is no usable gfx950 device. */
int qpp_ctx_create(int device, qpp_ctx **out);
void qpp_ctx_destroy(qpp_ctx *ctx);
/* Default stream used by the per-packet functions and by batch calls given stream == NULL. */
void *qpp_ctx_stream(qpp_ctx *ctx);
/* Waits for every stream of THIS context (batch streams, key installs and retirements, the host pipeline, transmit
 * queues' flushes, every stream made by qpp_stream_create and every non-null stream given to qpp_memcpy_*,
 * qpp_memset_d, qpp_event_record or qpp_stream_wait_event -- until qpp_stream_destroy releases it; a caller's own
 * stream handed to the context must therefore be released through qpp_stream_destroy, or outlive the context) and
 * stops its resident servers; never the whole device: another context's resident server keeps
 * running (hipDeviceSynchronize would wait for its idle exit, or forever while it is fed).  The same holds for every
 * call of the library: no free or wait of one context waits for another context's servers (see qpp_dev_free). */
int qpp_ctx_synchronize(qpp_ctx *ctx);
/* AES-GCM batches of at most max_packets packets (default 16384, env QPP_BURST_MAX) run one wave per packet
 * (latency: a 64-packet GSO burst); larger ones by the throughput kernels (quad / wave-item; qpp_ctx_set_aes_kernel).  ChaCha20-Poly1305 batches switch
 * at max_packets / 4.  0 = never one wave per packet.  Outputs are identical either way. */
int qpp_ctx_set_burst_max(qpp_ctx *ctx, size_t max_packets);
/* Per-packet calls (qpp_seal, qpp_seal_scatter, qpp_open, qpp_dc_*) through the context's packet server (on by default;
 * env QPP_PACKET_SERVER=0 turns it off): a persistent kernel of 4 workgroups, started by the first such call, that
 * seals / opens one packet posted through pinned memory without a kernel launch, and leaves after
 * QPP_TXQ_SERVER_IDLE_MS (200) without a call.  Packets of more than 16 KiB (header + payload + tag) and FIPS seals
 * take the launched path.  Outputs are identical either way.  on = 0 stops and frees the server.
 * Resident servers are accounted per DEVICE, over every context of the process (packet servers and persistent
 * transmit queues alike): at most GPU_MAX_HW_QUEUES (default 4) are resident on a device at once -- the runtime maps
 * the streams of one priority level onto that many hardware queues, and a server launched onto a hardware queue
 * another server holds would wait for that server's idle exit -- so a call that finds every server slot taken is
 * launched instead (same results), and a transmit-queue flush takes the launched path.  A server's launch also waits
 * for the device's latest fused receive (qpp_unprotect_open_batch): its grid did not count the server's CUs. */
int qpp_ctx_set_packet_server(qpp_ctx *ctx, int on);
/* Per-packet calls the packet server has taken so far, and its kernel launches (it leaves when idle). */
int qpp_ctx_packet_server_info(const qpp_ctx *ctx, uint64_t *calls, uint64_t *starts);
/* AES-GCM batches larger than burst_max: the quad kernel (four lanes per packet, one workgroup per CU over a slice of
 * the key-sorted packets) serves batches with at least 128 packets per live AES key (1024 past 16384 live AES keys),
 * the wave-item kernel (one key per 64-packet wave) batches with fewer (many keys, few packets each).  This forces one of them
 * (env QPP_AES_KERNEL=quad|wave); outputs are identical.  QPP_AES_KERNEL_LANE is the round-1..3 name of the quad
 * selector (the lane-per-packet kernel it named was replaced by the quad kernel) and is kept for source compatibility. */
#define QPP_AES_KERNEL_AUTO 0
#define QPP_AES_KERNEL_QUAD 1
#define QPP_AES_KERNEL_LANE QPP_AES_KERNEL_QUAD
#define QPP_AES_KERNEL_WAVE 2
int qpp_ctx_set_aes_kernel(qpp_ctx *ctx, int kernel);
/* FIPS mode: the s2n-quic-crypto `fips` cargo feature (cipher_suite/ring.rs:13-31, aead/fips.rs:13-60).  AES packet
 * keys created while it is on (qpp_key_new*, _update*, _raw) seal like aws-lc's TLS 1.3 record AEAD
 * (TlsRecordSealingKey, aws-lc-rs 1.12): a key's first seal fixes mask = its pn, and every seal needs
 * given = pn ^ mask >= the previous accepted given + 1 (and given != 2^64 - 1); a refused packet is not sealed, its
 * bytes are left untouched and its status is QPP_INTERNAL_ERROR (qpp_seal returns it; a qpp_txq flush with refused
 * packets reports it to qpp_txq_wait / qpp_txq_poll).  A batch applies the rule in batch order, per key.
 * ChaCha20-Poly1305 keys have no FIPS form (ring.rs:116-121); opening is never gated.  Keys created before the call
 * keep their mode. */
int qpp_ctx_set_fips(qpp_ctx *ctx, int on);
int qpp_key_fips(const qpp_key *key);  /* 1: the key seals in FIPS mode */
int qpp_abi_version(void);
/* Key-table occupancy (diagnostics / tests): slots allocated, high-water slot index, slots retired but not yet
 * reusable (their zeroization is still behind in-flight batches). */
int qpp_ctx_key_slots(qpp_ctx *ctx, uint32_t *capacity, uint32_t *high_water, uint32_t *retired);

/* ------------------------------------------------------------------ keys */

/* TLS_*::new(secret) -> (Self, HeaderKey): key/iv/hp = HKDF-Expand-Label(secret, "quic key"/"quic iv"/"quic hp")
 * (quic/s2n-quic-crypto/src/cipher_suite.rs:52-63,85-103; header_key.rs:33-49; iv.rs:14-24).
 * secret_len must equal the suite's hash length (32 for SHA-256 suites, 48 for SHA-384). */
int qpp_key_new(qpp_ctx *ctx, int suite, const uint8_t *secret, size_t secret_len, qpp_key **out);
/* TLS_*::new(secret) -> Option<(Self, HeaderKey)> (cipher_suite.rs:85-103; negotiated.rs:95-134) as two
 * independently owned handles: the header key outlives every packet key derived from this one by updates
 * (KeySet::rotate_phase drops old keys, keyset.rs:94-96, while the space keeps its header key, space/application.rs:70). */
int qpp_key_new_pair(qpp_ctx *ctx, int suite, const uint8_t *secret, size_t secret_len, qpp_key **key,
                     qpp_header_key **header_key);
/* Raw key material (fixtures, Retry/other consumers).  A raw key has no secret: update fails. */
int qpp_key_new_raw(qpp_ctx *ctx, int suite, const uint8_t *key, size_t key_len, const uint8_t iv[12],
                    const uint8_t *hp, size_t hp_len, qpp_key **out);
/* TLS_*::update / OneRttKey::derive_next_key: secret' = Expand-Label(secret, "quic ku", Hash.len);
 * key/iv re-derived; the header-protection key is carried over unchanged (RFC 9001 §6)
 * (cipher_suite.rs:68-83, one_rtt.rs:11-14). */
int qpp_key_update(const qpp_key *key, qpp_key **out);
/* Batched OneRttKey::derive_next_key (one_rtt.rs:11-14, cipher_suite.rs:68-83): out[i] = update(keys[i]), all keys
 * of one context (any suites), derived on the GPU in one pass per suite; each header key is carried over.  The
 * KeySet rotation of many connections at once (keyset.rs:75-96). */
int qpp_key_update_batch(qpp_key *const *keys, size_t n, qpp_key **out);
/* Zeroizes host and device copies (cipher_suite.rs:106-114,189-193); stream-ordered (see Asynchrony above). */
void qpp_key_free(qpp_key *key);
/* qpp_key_free over n keys (the old keys of a KeySet rotation across many connections, keyset.rs:94-96); the device
 * records are zeroized by one pass per run of consecutive slots.  NULL entries are skipped. */
void qpp_key_free_batch(qpp_key *const *keys, size_t n);
/* Index of this key in its context's device key table: the value to put in qpp_pkt.key_idx. */
uint32_t qpp_key_slot(const qpp_key *key);
/* qpp_key_slot of n keys into slots[i] (UINT32_MAX for NULL): a transport re-stamping its connections' key slots
 * after a batch rotation reads them in one call. */
void qpp_key_slot_batch(const qpp_key *const *keys, size_t n, uint32_t *slots);
int qpp_key_suite(const qpp_key *key);
/* Key::tag_len (16), HeaderKey::{sealing,opening}_sample_len (16), Key::aead_{confidentiality,integrity}_limit
 * (cipher_suite.rs:158-175, 247-301). */
size_t qpp_tag_len(const qpp_key *key);
size_t qpp_sample_len(const qpp_key *key);
uint64_t qpp_confidentiality_limit(const qpp_key *key);
uint64_t qpp_integrity_limit(const qpp_key *key);
/* Test introspection: copies the derived key (16/32), iv (12) and hp (16/32) bytes. */
int qpp_key_material(const qpp_key *key, uint8_t *key_out, uint8_t iv_out[12], uint8_t *hp_out);

/* Batched key installation on the GPU (key-update churn): n traffic secrets (host memory,
 * n * hash_len bytes) each go through `updates` TLS_*::update steps ("quic ku", cipher_suite.rs:68-83), then
 * TLS_*::new's key / iv derivation; the header key is the one of the given secret (not updated, RFC 9001 §6).
 * HKDF, AES key expansion and the GHASH key powers all run in one device pass; out[0..n) receive the handles
 * (each equivalent to qpp_key_new(secret) followed by `updates` qpp_key_update calls). */
int qpp_key_new_batch(qpp_ctx *ctx, int suite, const uint8_t *secrets, size_t n, uint32_t updates, qpp_key **out);

/* InitialKey::new_{client,server}(dcid): AES-128-GCM keys from the Initial salt
 * (quic/s2n-quic-crypto/src/initial.rs:29-80).  Returns the endpoint's sealer and opener. */
int qpp_initial_keys(qpp_ctx *ctx, int endpoint, const uint8_t *dcid, size_t dcid_len,
                     qpp_key **sealer, qpp_key **opener);
/* The same, plus the InitialHeaderKey pair (initial.rs:54-66: HeaderKeyPair { sealer, opener }) as independently
 * owned header keys.  header_sealer and header_opener are both NULL or both non-NULL. */
int qpp_initial_keys_pair(qpp_ctx *ctx, int endpoint, const uint8_t *dcid, size_t dcid_len, qpp_key **sealer,
                          qpp_key **opener, qpp_header_key **header_sealer, qpp_header_key **header_opener);

/* ------------------------------------------------------------------ header keys (header_key.rs:7-63) */

/* HeaderKey::new(secret, "quic hp", alg) (header_key.rs:33-49).  Its own device slot: usable as key_idx of
 * qpp_hp_mask_batch descriptors (never of seal/open batches, which refuse it with QPP_INTERNAL_ERROR). */
int qpp_header_key_new(qpp_ctx *ctx, int suite, const uint8_t *secret, size_t secret_len, qpp_header_key **out);
/* From the raw header-protection key (16 / 32 bytes). */
int qpp_header_key_new_raw(qpp_ctx *ctx, int suite, const uint8_t *hp, size_t hp_len, qpp_header_key **out);
/* Zeroizes host and device copies; stream-ordered like qpp_key_free. */
void qpp_header_key_free(qpp_header_key *hk);
uint32_t qpp_header_key_slot(const qpp_header_key *hk);
int qpp_header_key_suite(const qpp_header_key *hk);
/* HeaderKey::{sealing,opening}_sample_len (16) */
size_t qpp_header_key_sample_len(const qpp_header_key *hk);
/* HeaderKey::{sealing,opening}_header_protection_mask(sample) -> [u8; 5] (header_key.rs:10-30,52-56). */
int qpp_header_key_mask(const qpp_header_key *hk, const uint8_t *sample, size_t sample_len, uint8_t mask[5]);

/* ------------------------------------------------------------------ per packet (trait mirror) */

/* Key::encrypt(pn, header, payload): payload[0..payload_len) plaintext is sealed in place and the
 * 16-byte tag is written at payload + payload_len; payload_cap must be >= payload_len + 16
 * (aead/default.rs:44-62; cipher_suite.rs:146-156).  QPP_INTERNAL_ERROR on bad capacity. */
int qpp_seal(qpp_key *key, uint64_t pn, const uint8_t *header, size_t header_len,
             uint8_t *payload, size_t payload_len, size_t payload_cap);
/* seal_in_place_scatter (aead/default.rs:44-62): in_out sealed in place; the ciphertext of extra_in is
 * written to extra_out_and_tag[0..extra_len) and the tag after it (extra_out_and_tag holds extra_len+16). */
int qpp_seal_scatter(qpp_key *key, uint64_t pn, const uint8_t *header, size_t header_len,
                     uint8_t *in_out, size_t in_len, const uint8_t *extra_in, size_t extra_len,
                     uint8_t *extra_out_and_tag);
/* Key::decrypt(pn, header, payload): payload = ciphertext || tag (payload_len bytes);
 * on success payload[0..payload_len-16) holds the plaintext.  QPP_DECRYPT_ERROR on a bad tag or
 * payload_len < 16 (cipher_suite.rs:117-144; aead/default.rs:65-93); on a bad tag the
 * plaintext region is zeroed so unauthenticated plaintext is never released. */
int qpp_open(const qpp_key *key, uint64_t pn, const uint8_t *header, size_t header_len,
             uint8_t *payload, size_t payload_len);
/* The mask of the header key a qpp_key was derived with (the key's own copy; a transport holding a separate
 * HeaderKey uses qpp_header_key_mask). */
int qpp_hp_mask(const qpp_key *key, const uint8_t *sample, size_t sample_len, uint8_t mask[5]);

/* ------------------------------------------------------------------ dc consumers
 * dc/s2n-quic-dc's packet keys use the same AEAD, nonce (u64 PN -> 0u32 || be64, XOR iv; dc/s2n-quic-dc/src/crypto.rs:
 * 178-185, crypto/awslc.rs:364-370) and AAD = header as the QUIC path, so they run on the same kernels.  dc packets
 * in a device arena are plain qpp_pkt records (pn_len = 0, no HP flags) for qpp_seal_batch / qpp_open_batch. */

/* seal::Application::new / open::Application::new(key, iv, algorithm) (crypto/awslc.rs:24-33,157-166): raw key and
 * iv, no header key (the dc protocol has no header protection).  Any of the three suites. */
int qpp_dc_key_new(qpp_ctx *ctx, int suite, const uint8_t *key, size_t key_len, const uint8_t iv[12], qpp_key **out);
/* seal::Application::encrypt(pn, header, extra_payload, payload_and_tag) (crypto/awslc.rs:53-83):
 * inline_len = len - 16 - extra_len plaintext bytes at payload_and_tag are sealed in place, the ciphertext of
 * extra_payload follows them and the 16-byte tag ends the buffer (seal_in_place_scatter).  len < 16 + extra_len
 * (the reference's `assume!`) is QPP_INTERNAL_ERROR. */
int qpp_dc_seal(const qpp_key *key, uint64_t pn, const uint8_t *header, size_t header_len,
                const uint8_t *extra_payload, size_t extra_len, uint8_t *payload_and_tag, size_t len);
/* open::Application::decrypt(key_phase, pn, header, payload_in, tag, payload_out) (crypto/awslc.rs:176-204):
 * open_separate_gather.  key_phase != 0 -> QPP_ROTATION_NOT_SUPPORTED; a tag that is not 16 bytes or does not
 * verify -> QPP_DECRYPT_ERROR (open::Error::InvalidTag), payload_out zeroed. */
int qpp_dc_open(const qpp_key *key, int key_phase, uint64_t pn, const uint8_t *header, size_t header_len,
                const uint8_t *payload_in, const uint8_t *tag, size_t tag_len, uint8_t *payload_out,
                size_t payload_len);
/* open::Application::decrypt_in_place(key_phase, pn, header, payload, tag) (crypto/awslc.rs:207-227):
 * open_in_place_separate_tag; errors as qpp_dc_open. */
int qpp_dc_open_in_place(const qpp_key *key, int key_phase, uint64_t pn, const uint8_t *header, size_t header_len,
                         uint8_t *payload, size_t payload_len, const uint8_t *tag, size_t tag_len);

/* ------------------------------------------------------------------ batches (device-resident) */

/* One packet of a batch.  The packet's bytes live in a device arena at `off`:
 *   [off, off+aad_len)                 AAD = header || packet-number bytes (the `header` of Key::encrypt)
 *   [off+aad_len, off+aad_len+pt_len)  payload (plaintext for seal, ciphertext for open)
 *   [.. +pt_len, .. +pt_len+16)        tag (written by seal, read by open)
 * The HP sample is at off + aad_len - pn_len + 4 (payload.rs:151-169: header_len + 4). */
typedef struct qpp_pkt {
    uint64_t pn;       /* full packet number (62-bit) -> Iv::nonce (iv.rs:27-39) */
    uint32_t key_idx;  /* qpp_key_slot() of the key to use */
    uint32_t off;      /* byte offset of the packet in the arena; the whole packet (header, payload, tag) must
                          lie in [arena, arena + 4 GiB): one batch addresses a 4 GiB window, larger sets of
                          packets go in several batches (keeps the descriptor at 24 B) */
    uint16_t aad_len;  /* header length including the packet-number bytes */
    uint16_t pt_len;   /* payload length, tag excluded */
    uint8_t pn_len;    /* 1..4 packet-number bytes (header protection) */
    uint8_t flags;     /* 0, or QPP_PKT_SKIP */
    uint16_t reserved;
} qpp_pkt;             /* 24 bytes */

#define QPP_PKT_SKIP 0x1u     /* qpp_pkt.flags: the kernels leave this packet (and its status) untouched */

/* Batch flags */
#define QPP_HP_MASK_OUT 0x1u   /* write the 5-byte HP mask of packet i to masks[5*i] */
#define QPP_HP_APPLY 0x2u      /* apply the mask to the header in place (header_crypto.rs:80-95) */
#define QPP_ONLY_AES 0x10u     /* hint: every key in the batch is an AES-GCM key */
#define QPP_ONLY_CHACHA 0x20u  /* hint: every key in the batch is ChaCha20-Poly1305 */
#define QPP_KEY_BY_CONN 0x40u  /* host batches: qpp_pkt.key_idx is a connection index into the table of
                                  qpp_ctx_set_conn_keys, resolved to the connection's current key on the device */

/* Seal n packets: all pointers are device pointers (descs, arena, masks, status); masks may be NULL
 * unless QPP_HP_MASK_OUT; status may be NULL (per-packet QPP_OK / QPP_DECODE_ERROR when the HP sample
 * does not fit).  stream = hipStream_t or NULL for the context's stream.  Asynchronous. */
int qpp_seal_batch(qpp_ctx *ctx, const qpp_pkt *descs, size_t n, uint8_t *arena, uint8_t *masks,
                   int8_t *status, uint32_t flags, void *stream);
/* Open n packets in place; status[i] = QPP_OK or QPP_DECRYPT_ERROR (payload zeroed on failure). */
int qpp_open_batch(qpp_ctx *ctx, const qpp_pkt *descs, size_t n, uint8_t *arena, int8_t *status,
                   uint32_t flags, void *stream);
/* Header-protection masks for n packets: sample at off + aad_len - pn_len + 4 (for receive, pass
 * aad_len = header_len and pn_len = 0).  masks[5*i]. */
int qpp_hp_mask_batch(qpp_ctx *ctx, const qpp_pkt *descs, size_t n, const uint8_t *arena, uint8_t *masks,
                      void *stream);

/* ------------------------------------------------------------------ host pipeline (packets in host memory)

 * The path starts and ends in host memory (the UDP socket buffer, platform socket/io/tx.rs:204-268, rx.rs).  A host
 * batch is cut into chunks of consecutive packets; each chunk's span of the arena is copied H2D, sealed and/or
 * opened on the GPU and copied back D2H, chunks overlapping on three streams over a fixed ring of device buffers
 * (so a batch may be far larger than the ring).  descs / arena / masks / status are HOST pointers, all four pinned
 * (qpp_host_alloc) for full PCIe rate and overlap: a pageable one makes every chunk's copies synchronous with the
 * host thread, which serialises the pipeline.  Descriptors must be in ascending, non-overlapping arena order and stay
 * untouched until the ticket completes.  ops: QPP_OP_SEAL, QPP_OP_OPEN, or both (seal then open on the device:
 * the round trip; QPP_HP_APPLY is refused there since the opener needs the unprotected header).  Returns when every
 * chunk is enqueued; *ticket completes when the last chunk is back in host memory. */
#define QPP_OP_SEAL 0x1u
#define QPP_OP_OPEN 0x2u
int qpp_host_batch_submit(qpp_ctx *ctx, const qpp_pkt *descs, size_t n, uint8_t *arena, uint8_t *masks,
                          int8_t *status, uint32_t flags, uint32_t ops, uint64_t *ticket);
/* *done = 1 once the ticket's batch is back in host memory (the ticket stays valid until waited on). */
int qpp_host_batch_query(qpp_ctx *ctx, uint64_t ticket, int *done);
/* Blocks until the ticket's batch is back in host memory, then releases the ticket. */
int qpp_host_batch_wait(qpp_ctx *ctx, uint64_t ticket);
/* Ring geometry: packets and bytes per chunk, chunk buffers.  Default: buffers for 262144 packets / 384 MiB, 4 of
 * them, and each batch cut into ~16 chunks of 64 Ki-256 Ki packets (at least 64 per live AES key); setting a geometry
 * fixes the chunk size.  Waits for the device. */
int qpp_ctx_set_host_pipe(qpp_ctx *ctx, size_t chunk_packets, size_t chunk_bytes, size_t slots);
/* The connection -> key slot table of QPP_KEY_BY_CONN host batches (the transport's KeySets,
 * crypto/application/keyset.rs: a key update replaces the key behind a connection's entry, not the packets queued
 * for it).  slots[c] = qpp_key_slot of connection c's current packet key.  Stream-ordered on the host pipeline:
 * batches submitted before the call resolve through the previous table, later ones through this one; the caller's
 * array may be reused on return. */
int qpp_ctx_set_conn_keys(qpp_ctx *ctx, const uint32_t *slots, size_t n);

/* ------------------------------------------------------------------ deferred transmit queue */

/* The transport seals one packet at a time, in place, into the GSO segment buffer and applies header protection
 * right after (packet/encoding.rs:274-278, crypto/mod.rs:182-247; platform socket/io/tx.rs:204-268).  A qpp_txq
 * defers both: the transport encodes header || PN || plaintext into the queue's ring (pinned host memory, the
 * segment buffer), qpp_txq_push records what Key::encrypt + HeaderKey::sealing_header_protection_mask would have
 * done, and qpp_txq_flush (at the end of a GSO burst / queue.flush(), endpoint/mod.rs:158) protects every pushed
 * packet in one device batch: the ring then holds the protected packets, tags included. */
typedef struct qpp_txq qpp_txq;
int qpp_txq_create(qpp_ctx *ctx, size_t ring_bytes, size_t max_packets, qpp_txq **out);
/* The same queue with up to in_flight (1..64) flushes outstanding (qpp_txq_flush_async): each flush has its own
 * descriptors and plan; flushes go out round-robin on up to 4 streams of the queue.  The ring bytes of a flushed
 * packet belong to the engine until its ticket completes (the transport encodes the next bursts elsewhere in the
 * ring).  qpp_txq_create(..) = in_flight 1. */
int qpp_txq_create_async(qpp_ctx *ctx, size_t ring_bytes, size_t max_packets, size_t in_flight, qpp_txq **out);
/* The same queue (one flush in flight) served by a PERSISTENT kernel: the transport's queue.flush() posts the
 * flush through a doorbell word in pinned host memory instead of launching kernels, and qpp_txq_wait spins on a
 * completion word the kernel writes back into the same page (no launch, no runtime call, no interrupt per flush).
 * The server keeps the AES tables and the last key's GHASH tables in LDS between flushes; it occupies a few CUs
 * (QPP_TXQ_SERVER_WGS, default 16; full-chip batch kernels of every context on the device size their grids around
 * them).  It counts against the device's GPU_MAX_HW_QUEUES server slots (qpp_ctx_set_packet_server): with none free,
 * flushes take the launched path until one is.  A flush
 * after a quarter of QPP_TXQ_SERVER_IDLE_MS (default 200) without one restarts it first (one launch); the kernel itself
 * leaves after the whole idle time (a host that went away).  Flushes with a
 * ChaCha20-Poly1305 packet, or while a FIPS key is live, take the launched path of qpp_txq_create (same results).
 * Replaces the per-flush launch behind quic/s2n-quic-platform/src/socket/io/tx.rs:204-268. */
int qpp_txq_create_persistent(qpp_ctx *ctx, size_t ring_bytes, size_t max_packets, qpp_txq **out);
/* Flushes sealed by the persistent server / by launched kernels, and server launches so far (any queue). */
int qpp_txq_info(const qpp_txq *q, uint64_t *server_flushes, uint64_t *launched_flushes, uint64_t *server_starts);
/* Persistent queue: microseconds from the server seeing the last posted flush's doorbell to its completion word. */
int qpp_txq_server_time(const qpp_txq *q, double *us);
/* Persistent queue: descriptors its server refused because their bytes were not inside the ring (never read or
 * written; qpp_txq_push validates every packet, so this stays 0 -- a device-side check of every ring offset). */
int qpp_txq_server_refused(const qpp_txq *q, uint64_t *count);
/* Device `device`: times a free past the parked-memory bound evicted the device's resident servers (every context's:
 * each leaves at its next poll without a complete flush, and its queue relaunches it at its next post), and one-shot
 * server launches that finished a posted flush whose server had left while every server slot of the device was taken
 * (on the owning context's normal-priority stream).  See qpp_dev_free. */
int qpp_dev_server_evictions(int device, uint64_t *evictions, uint64_t *oneshots);
/* Diagnostics: the server's clock (100 MHz) at the last flush's doorbell, workgroup 0's phase stamps and shader-clock
 * cycles over its work (a build with QPP_TXS_TRACE, else 0) and its completion word:
 * {seen, broadcast, item read, packets done, arrival, done, shader cycles broadcast -> arrival}, then the low words
 * of wave 0's stamps inside its packet {start, first block in, passes done, lane tree done, HP done}. */
int qpp_txq_server_stamps(const qpp_txq *q, uint64_t out[12]);
void qpp_txq_destroy(qpp_txq *q);
/* Host pointer to the ring (ring_bytes, pinned). */
uint8_t *qpp_txq_ring(qpp_txq *q);
/* The packet at ring[off]: header (header_len bytes, PN excluded) || PN (pn_len bytes) || payload_len bytes of
 * plaintext, with 16 bytes after it for the tag.  QPP_DECODE_ERROR when payload_len + pn_len < 4 (no room for
 * the HP sample, encoding.rs:178-188); QPP_INTERNAL_ERROR on a bad range, a full queue or a key of another
 * context. */
int qpp_txq_push(qpp_txq *q, const qpp_key *key, uint64_t pn, size_t off, size_t header_len, size_t pn_len,
                 size_t payload_len);
/* qpp_txq_push for a scatter::Buffer with an `extra` tail (common/s2n-codec/src/encoder/scatter.rs:6-68;
 * encoding.rs:245-270 re-wraps the inline bytes + extra before crypto::encrypt): the packet's inline plaintext
 * (inline_len bytes after header || PN) is already in the ring; the extra bytes are copied into the ring right after
 * it (what scatter::Buffer::flatten does, since the engine seals contiguous bytes), then the packet is pushed with
 * payload_len = inline_len + extra_len.  extra may be NULL when extra_len is 0.  Same errors as qpp_txq_push; nothing
 * is copied unless the push is accepted. */
int qpp_txq_push_scatter(qpp_txq *q, const qpp_key *key, uint64_t pn, size_t off, size_t header_len, size_t pn_len,
                         size_t inline_len, const uint8_t *extra, size_t extra_len);
/* n pushes at once from ready descriptors (key_idx = qpp_key_slot of a live key of this context, off into the ring,
 * aad_len = header_len + pn_len, flags 0): for bindings whose per-call cost dominates a GSO burst (Python), same
 * checks as qpp_txq_push; nothing is queued unless every descriptor passes. */
int qpp_txq_push_descs(qpp_txq *q, const qpp_pkt *descs, size_t n);
/* Seal + header-protect every pushed packet (one qpp_seal_batch with QPP_HP_APPLY), wait, empty the queue. */
int qpp_txq_flush(qpp_txq *q);
/* The same without waiting: *ticket names the flush (0 when nothing was pushed).  Returns once the flush is enqueued;
 * if all in_flight slots are busy, first waits for the oldest.  The queue is empty again for the next burst. */
int qpp_txq_flush_async(qpp_txq *q, uint64_t *ticket);
/* *done = 1 once the ticket's packets are protected in the ring (then the socket may send them). */
int qpp_txq_poll(qpp_txq *q, uint64_t ticket, int *done);
/* Blocks until the ticket's packets are protected in the ring. */
int qpp_txq_wait(qpp_txq *q, uint64_t ticket);
/* Coalescing: flush_async holds bursts back until `bursts` of them are in (or the next would not fit max_packets),
 * then sends them as one launch; polling or waiting on a held ticket sends it at once.  Default 1 (every flush_async
 * sends).  Fewer, larger launches: the host's per-launch cost is what bounds a stream of small GSO bursts. */
int qpp_txq_set_coalesce(qpp_txq *q, size_t bursts);
size_t qpp_txq_pending(const qpp_txq *q);

/* ------------------------------------------------------------------ receive path */

/* One received, still protected packet of a GRO batch. */
typedef struct qpp_rx_pkt {
    uint64_t largest_pn;  /* largest acknowledged PN of the packet-number space (PacketNumber::as_u64) */
    uint32_t key_idx[2];  /* KeySet crypto[0] / crypto[1] slots: the key-phase bit of a short header picks one
                             (crypto/application/keyset.rs:113-143); long headers use key_idx[0].  The header key
                             is key_idx[0]'s (header keys are not updated, RFC 9001 §6). */
    uint32_t off;         /* first byte of the packet in the arena */
    uint16_t header_len;  /* bytes before the packet-number field (tag byte || DCID for a short header) */
    uint16_t len;         /* bytes of the whole packet: header || PN || payload || tag */
} qpp_rx_pkt;             /* 24 bytes */

/* Receive side of crypto::{unprotect, decrypt} for n packets, on the device: sample at header_len + 4
 * (payload.rs:151-169) -> mask -> remove_header_protection in place (header_crypto.rs:98-123: pn_len from the
 * unmasked first byte) -> expand the packet number against largest_pn (packet/number/mod.rs:191-238) -> choose the
 * key by the key phase -> open in place.  descs_out[i] receives the resulting qpp_pkt (pn = expanded packet number,
 * key_idx = chosen slot, aad_len = header_len + pn_len, pt_len, pn_len; flags = QPP_PKT_SKIP when rejected);
 * status[i] = QPP_OK, QPP_DECODE_ERROR (no room for the sample, short.rs / payload.rs), QPP_DECRYPT_ERROR, or
 * QPP_INTERNAL_ERROR (a slot outside the table, a key_idx[0] slot holding no key -- nothing touched -- or a chosen
 * packet key that is not live: header unprotected, payload untouched).  QPP_ONLY_AES / QPP_ONLY_CHACHA: packets whose
 * (live) key is of the other family are unprotected but not opened, their status left as it was.
 * Launches: with any live AES packet key and a batch of the quad kernel's size (see qpp_ctx_set_aes_kernel),
 * ONE cooperative launch unprotects, groups by the chosen key and opens the AES packets of both sizes, and one more
 * launch on the same stream opens the ChaCha20 packets it sorted out (when ChaCha20 keys are live); with no AES record
 * live, one launch of the ChaCha20 kernel; otherwise unprotect + plan + open kernels.  Identical outputs on every path
 * (env QPP_RX_FUSED=0 forces the multi-launch one).  The fused launch needs all its workgroups resident at once (grid
 * barriers), which the engine arranges within the process: its grid is the CUs every context's resident servers leave
 * on the device, fused receives of a device run one after another (a second one, on any stream of any context, waits
 * for the first), and a server starts only after the latest fused receive.  If the workgroups are still not all
 * resident within a second (CUs held by another process's kernels), its AES packets report QPP_INTERNAL_ERROR with
 * the header unprotected and the payload untouched, and qpp_ctx_rx_timeouts counts it.
 * rx, descs_out, arena and status are device pointers.  Asynchronous. */
int qpp_unprotect_open_batch(qpp_ctx *ctx, const qpp_rx_pkt *rx, size_t n, uint8_t *arena, qpp_pkt *descs_out,
                             int8_t *status, uint32_t flags, void *stream);

/* PacketNumber::truncate (packet/number/packet_number.rs:135-143, mod.rs:81-93): the 1..4-byte encoding of pn
 * relative to the largest acknowledged PN.  QPP_DECODE_ERROR when pn < largest_acked or the distance needs > 4 bytes. */
int qpp_pn_truncate(uint64_t pn, uint64_t largest_acked, uint64_t *truncated, size_t *pn_len);
/* TruncatedPacketNumber::expand (packet/number/mod.rs:191-238, RFC 9000 A.3), clamped to 2^62 - 1. */
uint64_t qpp_pn_expand(uint64_t largest_acked, uint64_t truncated, size_t pn_len);

/* ------------------------------------------------------------------ device plumbing */

/* hipFree / hipHostFree wait for every stream of the device, a resident server's too (which leaves only on its idle
 * time, or never while it is fed).  So qpp_dev_free / qpp_host_free -- and every free inside the library -- free at
 * once only while no server of the device (of any context, this one's included) is resident; otherwise the buffer is
 * parked (up to 2 GiB per device, env QPP_PARKED_MAX_MB) and freed by the next free, qpp_ctx_synchronize or
 * qpp_ctx_destroy of any context that finds none resident.  Past the bound the free EVICTS the device's resident
 * servers (every context's: each leaves at its next poll that finds no complete flush, after the flush in hand) and
 * then frees: it waits microseconds for them, never for a server's idle exit; an evicted queue relaunches its server
 * at its next post (qpp_dev_server_evictions counts both).  Below the bound a free never stops a server.  Work already
 * enqueued that reads the buffer is unaffected.  No view of a freed buffer may be used afterwards. */
int qpp_dev_alloc(qpp_ctx *ctx, size_t bytes, void **out);
void qpp_dev_free(qpp_ctx *ctx, void *ptr);
int qpp_host_alloc(qpp_ctx *ctx, size_t bytes, void **out); /* pinned host memory */
void qpp_host_free(qpp_ctx *ctx, void *ptr);
int qpp_memcpy_h2d(qpp_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream);
int qpp_memcpy_d2h(qpp_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream);
int qpp_memcpy_d2d(qpp_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream);
int qpp_memset_d(qpp_ctx *ctx, void *dst, int value, size_t bytes, void *stream);
int qpp_stream_create(qpp_ctx *ctx, void **out);
void qpp_stream_destroy(qpp_ctx *ctx, void *stream);
int qpp_stream_synchronize(qpp_ctx *ctx, void *stream);
int qpp_event_create(qpp_ctx *ctx, void **out);
void qpp_event_destroy(qpp_ctx *ctx, void *event);
int qpp_event_record(qpp_ctx *ctx, void *event, void *stream);
int qpp_event_elapsed_ms(qpp_ctx *ctx, void *start, void *stop, float *ms);
/* Makes `stream` wait for `event` (copy/compute overlap across streams). */
int qpp_stream_wait_event(qpp_ctx *ctx, void *stream, void *event);
/* Last HIP error string of this context (for diagnostics). */
const char *qpp_ctx_last_error(qpp_ctx *ctx);
/* Workgroups of the fused receive launch (qpp_unprotect_open_batch) that left on a grid-barrier timeout since the
 * context was created: a cooperative launch whose workgroups could not all be resident within a second (a foreign
 * kernel holding CUs).  Their packets bound for the open phase reported QPP_INTERNAL_ERROR with the payload untouched
 * and the header already unprotected.  0 in normal operation.  Waits for the context's batch streams. */
int qpp_ctx_rx_timeouts(qpp_ctx *ctx, uint64_t *count);

#ifdef __cplusplus
}
#endif
#endif
