// qpp_internal.h — shared between the host runtime (api.cpp, kdf.cpp) and the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/qpp.h"

namespace qpp {

// ---------------------------------------------------------------- AES S-box, built at compile time
// From its definition (FIPS-197 §5.1.1): multiplicative inverse in GF(2^8) (x^254) + affine map.
constexpr uint8_t gf_mul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return p;
}
constexpr uint8_t gf_inv(uint8_t x) {
    // x^254 = x^-1 (and 0 -> 0)
    uint8_t r = 1, b = x;
    for (int e = 254; e; e >>= 1) {
        if (e & 1) r = gf_mul(r, b);
        b = gf_mul(b, b);
    }
    return x ? r : 0;
}
struct SBox {
    uint8_t v[256];
    constexpr SBox() : v() {
        for (int x = 0; x < 256; x++) {
            uint8_t i = gf_inv((uint8_t)x), s = i, r = i;
            for (int k = 0; k < 4; k++) {
                r = (uint8_t)((r << 1) | (r >> 7));
                s ^= r;
            }
            v[x] = (uint8_t)(s ^ 0x63);
        }
    }
};
constexpr SBox kSBox{};
static_assert(kSBox.v[0x00] == 0x63 && kSBox.v[0x53] == 0xed && kSBox.v[0xff] == 0x16, "sbox");

// ---------------------------------------------------------------- packet numbers
constexpr uint64_t kPnMask = (1ull << 62) - 1;  // PacketNumber::as_u64 drops the space bits
// RFC 9000 A.3 DecodePacketNumber as quic/s2n-quic-core/src/packet/number/mod.rs:191-238 states it (no data-dependent
// branches; the result is clamped to VarInt::MAX = 2^62 - 1 like VarInt::new(..).unwrap_or(MAX)).
__host__ __device__ inline uint64_t decode_packet_number(uint64_t largest, uint64_t truncated, uint32_t nbits) {
    const uint64_t expected = largest + 1, win = 1ull << nbits, hwin = win >> 1, mask = win - 1;
    uint64_t cand = (expected & ~mask) | truncated;
    const bool a = expected >= hwin && cand <= expected - hwin;
    const bool b = cand < (1ull << 62) - win;
    const bool c = cand > expected + hwin;
    const bool d = cand >= win;
    const bool ab = a && b, cd = !ab && c && d;
    cand += ab ? win : 0;
    cand -= cd ? win : 0;
    return cand > kPnMask ? kPnMask : cand;
}

// ---------------------------------------------------------------- device key record
// One per key slot, in HBM, replicated per GPU context.  Words are little-endian images of the
// byte strings (dword c of an AES state = column c, row 0 in the low byte).
struct alignas(16) DevKey {
    uint32_t suite;      // qpp_suite
    uint32_t nr;         // AES rounds of the packet key (10/14), 0 for ChaCha
    uint32_t hp_nr;      // AES rounds of the HP key
    uint32_t live;       // 1 while the slot holds a packet key (+ its header key), 2: a header key only, 0: free
    uint32_t iv[4];      // 12-byte iv, iv[3] = 0
    uint32_t rk[60];     // AES round keys (11/15 x 4 words) | ChaCha key in rk[0..8)
    uint32_t hp_rk[60];  // AES HP round keys                | ChaCha HP key in hp_rk[0..8)
    uint32_t H[4];       // GHASH key E_K(0^128)                  (filled on device by key setup)
    uint32_t V[128][4];  // V[m] = H * x^m in GCM bit order      (filled on device by key setup)
    // FIPS mode (fips.hip): the sealing nonce-order state of aws-lc's TLS 1.3 AEAD, kept and advanced on the device
    uint32_t fips;           // 1: seals are gated (an AES packet key created with qpp_ctx_set_fips on)
    uint32_t fips_seen;      // 1 once the key's first seal fixed fips_mask
    uint64_t fips_mask;      // pn of the key's first seal (given = pn ^ mask)
    uint64_t fips_min_next;  // the smallest given the next seal may use
    uint64_t fips_pad;
};
static_assert(sizeof(DevKey) == 2608, "DevKey layout");

// Grouping of an AES batch by key (GHASH tables are per key and live in LDS).
struct WorkItem {
    uint32_t key;    // key slot
    uint32_t begin;  // first index into perm[]
    uint32_t count;  // packets (<= the variant's packets per item)
    uint32_t nr;     // AES rounds for this key
};

constexpr int kMinPacketsPerItem = 4;
constexpr uint32_t kWavePacketsPerItem = 64;  // aes_gcm_wave_kernel: one wave, one key, <= 64 packets per work item
// batches with fewer packets per live AES key take the wave kernel: 128 while every live key can have a pow slot (the quad
// kernel's per-segment tables come from it), else 1024 (round 6 crossover, profiles/r06/manykey: 4096 keys x 64 / 128 /
// 256 / 512 packets per key, quad vs wave 386 / 645 / 781 / 876 vs 489 / 610 / 668 / 666 GiB/s)
constexpr uint32_t kWaveKernelPacketsPerKey = 128;
constexpr uint32_t kWaveKernelPacketsPerKeyNoPow = 1024;
constexpr uint32_t kQuadPerItem = 0x7fffffffu;  // aes_gcm_quad_kernel: one work item per key (workgroups take equal slices)
constexpr uint32_t kBurstMaxDefault = 16384;  // AES batches up to this many packets run one wave per packet
constexpr uint32_t kChachaBurstShift = 2;     // ChaCha20-Poly1305 batches up to burst_max >> 2 do (its lane kernel
                                              // fills the chip with fewer packets: crossover ~6 Ki vs ~20 Ki)
constexpr uint32_t kTxqZeroCopyMax = 1024;    // txq flushes up to this many packets run on the pinned ring in place
                                              // (coalesced bursts: 512-packet launches were 36 % faster in place)
constexpr int kMaxPlanKeys = 8192;      // keys binned in LDS by the plan kernels (larger tables: global bins)

// Per-key GHASH power tables of the burst kernel (burst.hip): T_t = 4-bit tables of H^(2^t), t = 1..6, 48 KiB per
// key slot below `cap`, computed when the key is installed (they used to be rebuilt by every workgroup of every
// burst launch: about half of a 64-packet flush).  Slots >= cap (huge key tables) still build them per launch.
// A slot: T_1 .. T_6, the 4-bit tables of H^(2^t) (burst kernels, servers), then the 4-bit table of H^3 (with T_1 =
// H^2 and T_2 = H^4: the quad kernels' per-key-segment tables come from the slot instead of being derived in LDS)
constexpr uint32_t kPowTables = 6;
constexpr uint32_t kPowH3 = kPowTables * 8192u;
constexpr uint32_t kPowBytes = kPowH3 + 8192u;
constexpr uint32_t kPowSlots = 16384;  // at most 896 MiB per context (allocated as the key table grows)
struct PowTables {
    uint8_t *base;  // [cap][kPowBytes]
    uint32_t cap;
};

// ---------------------------------------------------------------- launchers (aes_gcm.hip, chacha.hip, plan.hip)
struct PlanBuffers {
    uint32_t *counts;   // [key_cap] packets per key
    uint32_t *cursor;   // [key_cap] scatter cursors
    uint32_t *istart;   // [2][key_cap + 1] first work item per key and AES size (used when key_cap > kMaxPlanKeys)
    uint32_t *perm;     // [n_cap] packet indices grouped by key
    uint32_t *kq;       // [n_cap] each packet's planned key (0xffffffff: not a live AES key), plan_hist -> plan_scatter
    WorkItem *work;     // [n_cap / kMinPacketsPerItem + key_cap + 1]
    uint32_t *n_work;   // [8] plan meta: work items, AES-128 items, AES-128 packets, AES-256 packets, other packets
                        // (ChaCha20, refused) and their first perm index, and plan-internal [6] count and [7] cursor
                        // (zero between plans; plan.hip)
};

// aes_gcm.hip: records[i] (device, may be nullptr = already in place) -> keys[slots[i]], then H / V[m] for AES keys
hipError_t launch_key_install(DevKey *keys, const uint32_t *slots, const DevKey *records, uint32_t count,
                              const PowTables &pow, hipStream_t s);
// keysched.hip: n secrets -> updates x "quic ku" -> key/iv -> DevKey records keys[slots[i]] and per-key material
// (secret' | key | iv | hp, key_material_bytes() each); then key install.  The header key is derived from the given
// secret ("quic hp") when hp_in is nullptr, else taken from hp_in (suite key length per key: update batches).
// fips: the new keys seal in FIPS mode (AES suites only; see DevKey::fips)
hipError_t launch_key_derive(DevKey *keys, const uint32_t *slots, uint32_t n, int suite, const uint8_t *secrets,
                             const uint8_t *hp_in, uint32_t updates, uint8_t *material, uint32_t fips,
                             const PowTables &pow, hipStream_t s);
uint32_t key_material_bytes();
// the plan of an n-packet batch also lists the non-AES packets behind the AES ones (pb.perm[meta[5] ..], meta[4] of
// them) -- the three-launch plan does, plan_small does not
bool plan_lists_others(uint32_t n, uint32_t key_cap);
hipError_t launch_plan(const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n, PlanBuffers pb,
                       uint32_t per, hipStream_t s);
uint32_t plan_max_work(uint32_t n, uint32_t key_cap, uint32_t per);
// QPP_KEY_BY_CONN: descs[i].key_idx = map[descs[i].key_idx] (0xffffffff past map_n), in place on the device copy
hipError_t launch_conn_remap(qpp_pkt *descs, uint32_t n, const uint32_t *map, uint32_t map_n, hipStream_t s);
// burst.hip: one wave per packet for small batches (GSO bursts); work items of whole waves, <= 64 packets
uint32_t burst_packets_per_item(uint32_t n, uint32_t n_cu);
hipError_t launch_aes_gcm_burst(bool seal, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb,
                                uint32_t n, uint32_t key_cap, uint32_t per, uint8_t *arena, uint8_t *masks,
                                int8_t *status, uint32_t flags, uint32_t suites, const PowTables &pow, hipStream_t s);
// Persistent transmit-queue server (burst.hip txq_server_kernel; api.cpp qpp_txq_create_persistent).
// One TxsSlot per server workgroup in pinned, coherent host memory: the host writes the workgroup's first work item
// and its descriptors (each tagged with the flush's seq) and then seq; the workgroup polls its slot (one wave-wide
// read gets the flush, the item and the descriptors together) and writes `done` = seq when its packets are sealed.
constexpr uint32_t kTxsWaves = 8;  // server workgroup = 8 waves, one packet per wave per work item
constexpr uint32_t kTxsItemsMask = 0xffffffu;
constexpr uint32_t kTxsStop = 0xffffffu;
// Descriptor flags of the per-packet requests (qpp_seal / qpp_open through the context's packet server, api.cpp
// run_one_server): never set by the transport (qpp_txq_push_descs refuses any flag)
constexpr uint8_t kTxsPktNoHp = 0x40;  // seal without header protection (Key::encrypt), status written
constexpr uint8_t kTxsPktOpen = 0x80;  // open (Key::decrypt), status written
constexpr uint32_t kTxsMaskNr = 0xffu;  // WorkItem.nr of a header-protection mask item (qpp_hp_mask, qpp_header_key_mask)
// Every 16-byte chunk carries the flush's seq as its last word (the host stores it after the chunk's other words):
// the server reads each chunk with ONE 16-byte load, so a chunk whose tag matches is wholly this flush's.  (With the
// tag in only one chunk of a descriptor, a poll could combine a stale first half -- the previous flush's pn, key and
// offset -- with a fresh second half, and seal a packet with the previous flush's descriptor.)
struct alignas(16) TxsSlotDesc {
    uint64_t pn;
    uint32_t key_idx, tag0;
    uint32_t off;
    uint32_t lens;  // aad_len | pt_len << 16
    uint32_t misc;  // pn_len | flags << 8
    uint32_t tag1;
};
struct alignas(64) TxsSlot {
    uint32_t seq;   // flush seq, written last
    uint32_t word;  // key epoch << 24 | the flush's work items (kTxsStop: exit)
    uint32_t pad0[2];
    uint32_t it_key, it_count, it_nr, it_tag;  // this workgroup's first work item (count 0: none)
    TxsSlotDesc desc[kTxsWaves];
    alignas(64) uint32_t done;  // written by the server: the seq whose packets this workgroup has sealed
    int8_t status[kTxsWaves];   // per-packet requests (kTxsPktOpen / kTxsPktNoHp): wave q's packet status, before done
    uint32_t pad2[13];
};
static_assert(sizeof(TxsSlot) == 384 && offsetof(TxsSlot, desc) == 32 && offsetof(TxsSlot, done) == 320, "TxsSlot");
constexpr uint32_t kTxsPollLanes = 18;  // 16-byte chunks of [seq .. desc[7]] = 288 bytes
struct alignas(64) TxsMail {  // telemetry (s_memrealtime, 100 MHz)
    uint64_t t_seen, t_done;  // workgroup 0 saw the flush / finished it
    uint64_t pad0[6];         // QPP_TXS_TRACE: workgroup 0's phase stamps and shader cycles
    uint32_t pad1[16];        // QPP_TXS_TRACE: wave 0's stamps inside its packet
    uint32_t oob;             // descriptors the server refused because their bytes lie outside the ring (0: always)
    uint32_t pad2[15];
};
// ring_bytes: the ring's size -- a descriptor whose bytes [off, off + aad + payload + 16) do not lie inside is refused
// (never read or written) and counted in mail->oob.  evict: the device's eviction word (16 B, coherent pinned memory):
// non-zero makes every workgroup leave at its next poll that finds no complete flush.
hipError_t launch_txq_server(const DevKey *keys, const PowTables &pow, TxsMail *mail, TxsSlot *slots,
                             const WorkItem *items, const qpp_pkt *sdesc, uint8_t *ring, uint32_t ring_bytes,
                             uint32_t seq0, uint32_t idle_ticks, uint32_t wgs, const uint32_t *evict, hipStream_t s);
// the burst power tables of keys[slots[i]] (AES packet keys with slot < pow.cap), after their V[m] are in place
hipError_t launch_pow_setup(const DevKey *keys, const uint32_t *slots, uint32_t count, const PowTables &pow,
                            hipStream_t s);
// suites: bit (1 << suite) for every suite with a live key in the context (launches only what can occur)
// plan with per = kQuadPerItem; one workgroup per CU, each an equal slice of the key-sorted packets
hipError_t launch_aes_gcm(bool seal, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb, uint32_t n,
                          uint32_t n_cu, uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags,
                          uint32_t suites, const PowTables &pow, hipStream_t s);
// one live AES key (slot, nr): the quad kernel over descs[0, n) without a plan; packets of any other slot are refused
// (status INTERNAL_ERROR)
hipError_t launch_aes_gcm_single(bool seal, const DevKey *keys, const qpp_pkt *descs, uint32_t slot, uint32_t nr,
                                 uint32_t n, uint32_t n_cu, uint8_t *arena, uint8_t *masks, int8_t *status,
                                 uint32_t flags, const PowTables &pow, hipStream_t s);
// quad.hip: the quad-layout (4 lanes per packet, 768-thread workgroups) throughput kernel behind the two above
// quad.hip: fused unprotect -> PN expand -> key-phase choice -> open for any mix of live packet keys (AES-128 and
// AES-256 opened in the launch -- aes = 10 / 14 when only one size is live, 0 for both; ChaCha20 packets, when `chacha`, sorted to perm[scratch[3], + scratch[2]) for
// launch_chacha_sel behind it), one cooperative launch of `grid` workgroups (<= the CUs it may use; key_cap <=
// quad_rx_max_keys(), even).  scratch: 16 + 2 key_cap + 4 + 4 (key_cap + 1) words, the first 16 + 2 key_cap zeroed
// before the launch; perm: n words.  timeouts: a device word every workgroup that left on a barrier timeout increments
// (qpp_ctx_rx_timeouts).
uint32_t quad_rx_max_keys();
hipError_t launch_aes_gcm_quad_rx(uint32_t aes, uint32_t grid, hipStream_t s, const DevKey *keys, uint32_t key_cap,
                                  const qpp_rx_pkt *rx, uint32_t n, uint8_t *arena, qpp_pkt *descs_out, int8_t *status,
                                  uint32_t *scratch, uint32_t *perm, uint32_t *timeouts, bool chacha,
                                  const PowTables &pow);
// chacha.hip: open descs[sel[sel_meta[1] + i]] for i < min(n_max, sel_meta[0]) (count and base on the device)
hipError_t launch_chacha_sel(const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n_max,
                             uint8_t *arena, int8_t *status, const uint32_t *sel, const uint32_t *sel_meta, hipStream_t s);
// the same selection for seal or open of a planned batch (sel = the plan's perm, sel_meta = its meta + 4)
hipError_t launch_chacha_sel_batch(bool seal, const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n_max,
                                   uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags, const uint32_t *sel,
                                   const uint32_t *sel_meta, hipStream_t s);
hipError_t launch_aes_gcm_quad(bool seal, uint32_t nr, dim3 grid, hipStream_t s, const DevKey *keys,
                               const qpp_pkt *descs, const PlanBuffers &pb, uint8_t *arena, uint8_t *masks,
                               int8_t *status, uint32_t flags, uint32_t single, uint32_t n_single,
                               const PowTables &pow);
// many keys: work items of <= kWavePacketsPerItem packets (plan with per = kWavePacketsPerItem), one wave each
hipError_t launch_aes_gcm_wave(bool seal, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb, uint32_t n,
                               uint32_t key_cap, uint32_t n_cu, uint8_t *arena, uint8_t *masks, int8_t *status,
                               uint32_t flags, uint32_t suites, hipStream_t s);
// burst: one wave per packet (small batches) instead of one lane per packet
// key_cap: slots in the key table; a packet naming a slot >= key_cap is never dereferenced (status INTERNAL_ERROR)
hipError_t launch_chacha(bool seal, const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n,
                         uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags, bool burst, hipStream_t s);
// receive side: remove header protection, expand the PN, choose the key by key phase -> descs_out (chacha.hip)
// fused unprotect -> PN expand -> open for a context with no live AES record (chacha.hip)
hipError_t launch_chacha_rx(const DevKey *keys, uint32_t key_cap, const qpp_rx_pkt *rx, uint32_t n, uint8_t *arena,
                            qpp_pkt *descs_out, int8_t *status, hipStream_t s);
hipError_t launch_unprotect(const DevKey *keys, uint32_t key_cap, const qpp_rx_pkt *rx, uint32_t n, uint8_t *arena,
                            qpp_pkt *descs_out, int8_t *status, hipStream_t s);
hipError_t launch_hp_mask(const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n,
                          const uint8_t *arena, uint8_t *masks, hipStream_t s);
// FIPS mode (fips.hip): copies descs[0, n) to *descs_out (in scratch) with QPP_PKT_SKIP on every packet of a FIPS key
// whose nonce does not come strictly after its key's previous seal (batch order), status[j] = QPP_INTERNAL_ERROR for
// them (status may be nullptr) and *refused += their count (may be nullptr); advances the keys' nonce state.
size_t fips_scratch_bytes(uint32_t n);
hipError_t launch_fips_gate(DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n, void *scratch,
                            size_t scratch_bytes, qpp_pkt **descs_out, int8_t *status, uint32_t *refused,
                            hipStream_t s);

// ---------------------------------------------------------------- host key schedule (kdf.cpp)
size_t suite_key_len(int suite);
size_t suite_hash_len(int suite);
void hkdf_expand_label(size_t hash_len, const uint8_t *secret, const char *label, uint8_t *out, size_t out_len);
void hkdf_extract(size_t hash_len, const uint8_t *salt, size_t salt_len, const uint8_t *ikm, size_t ikm_len,
                  uint8_t *prk);
int aes_expand_key(const uint8_t *key, size_t key_len, uint32_t rk[60]);  // returns rounds
void secure_zero(void *p, size_t n);

}  // namespace qpp
