// chacha.hip — ChaCha20-Poly1305 seal/open + the standalone header-protection mask kernel (gfx950).
//
// Replaces, for TLS_CHACHA20_POLY1305_SHA256 (quic/s2n-quic-crypto/src/cipher_suite.rs:270-284,
// cipher_suite/ring.rs:121), aws-lc-rs's RFC 8439 AEAD behind <LessSafeKey as Aead>::{encrypt,decrypt}
// (src/aead/default.rs:44-93) and quic::CHACHA20 HeaderProtectionKey::new_mask (src/header_key.rs:52-56):
//   mask = ChaCha20(hp, counter = LE32(sample[0..4]), nonce = sample[4..16]) over 5 zero bytes.
//
// Mapping: one lane per packet, pure VALU (ARX + 26-bit-limb Poly1305); LDS only stages the payload for coalesced
// I/O, so keys are per lane and a mixed-key batch needs no grouping.  Each iteration produces one 64-byte keystream
// block, seals 4 x 16 bytes and absorbs them into Poly1305.
#include "chacha_wave.h"

namespace qpp {
namespace {
using namespace dev;

// One lane per packet, software-pipelined over 64-byte chunks: the keystream of chunk c+1 is computed in the same
// basic block as the Poly1305 steps of chunk c (independent chains).  The payload moves through a per-wave LDS stage
// that holds a PAIR of chunks (128 B per packet): every other chunk, 8 wave instructions load the next pair as 8
// packets x 128 contiguous bytes each (into registers, a pair ahead), and 8 more store the finished pair the same
// way; the owner lane reads its 16-B blocks from the stage and writes its output blocks back in place.  The kernel is
// bound by this payload I/O (1 Mi x 1200 B seal: 1.10 ms with 64-B chunks both ways, 0.71 ms with the loads and
// stores cut out, 1.09 ms with the ChaCha20 or the Poly1305 work cut out instead; 0.96 ms with 128-B stores), and
// 128-B chunks both ways are what the copy ubench showed cheapest (tools/ubench/copy_pattern.hip: in-place copy
// 1.09 ms with 64-B chunks, 0.86-0.92 with 128-B stores, 0.75-0.79 with 128-B loads and stores).
// Stage slot of packet p's block j of the pair: 64 (p / 8) + 8 (p % 8) + ((j + p + (p >> 4)) % 8).  A lane-linear
// access (slot 64 i + l) is packet 8 i + l / 8, so 8 lanes cover one packet's 128 contiguous bytes; the owner's
// ds_write_b128 (8-lane groups) and ds_read_b128 (16-lane groups) hit distinct bank quads.
// Per-wave LDS: pair stage 8 KiB | (payload offset, length) of the wave's 64 packets.
constexpr uint32_t kChachaStage = 64u * 16u * 8u;
constexpr uint32_t kChachaWaveLds = kChachaStage + 64u * 8u;
__device__ __forceinline__ uint32_t chacha_rho(uint32_t p) { return (p + (p >> 4)) & 7u; }

// RX (open only): the fused receive path for a context with no live AES record -- each lane first unprotects its
// packet of rx[] (rx_unprotect_one: HP removal, PN expansion, key phase; ChaCha20 header keys only), writes the
// qpp_pkt to descs_out and opens it with the key the phase picked.  Same outputs as unprotect_kernel + this kernel.
// Selection mode (sel != nullptr): the packets are descs[sel[sel_meta[1] + i]], i < min(n, sel_meta[0]) -- the ChaCha20
// packets the fused receive kernel (quad.hip) sorted behind its AES packets, or the non-AES packets a batch's plan
// listed behind its AES packets (plan.hip), their count on the device.
template <bool SEAL, bool RX = false>
__global__ __launch_bounds__(256, 3) void chacha_kernel(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                    const qpp_pkt *__restrict__ descs, uint32_t n,
                                                    uint8_t *__restrict__ arena, uint8_t *masks, int8_t *status,
                                                    uint32_t flags, const qpp_rx_pkt *__restrict__ rx = nullptr,
                                                    qpp_pkt *__restrict__ descs_out = nullptr,
                                                    const uint32_t *__restrict__ sel = nullptr,
                                                    const uint32_t *__restrict__ sel_meta = nullptr) {
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t pi = slot;  // the packet (descriptor, status and mask index)
    if (sel) {
        const uint32_t cnt = min(n, sel_meta[0]);
        if (blockIdx.x * blockDim.x >= cnt) return;  // (workgroup-uniform: the grid is sized for n)
        n = cnt;
        pi = slot < cnt ? sel[sel_meta[1] + slot] : 0u;
    }
    const bool valid = slot < n;
    qpp_pkt d;
    if constexpr (RX) {
        static_assert(!SEAL, "the receive path opens");
        if (valid) {
            d = rx_unprotect_one<false>(AesLds{0}, keys, key_cap, rx[pi], arena, status, pi);
            descs_out[pi] = d;
        } else {
            d = qpp_pkt{};
            d.flags = QPP_PKT_SKIP;  // helper lane
        }
    } else {
        d = valid ? descs[pi] : sel ? descs[sel[sel_meta[1]]] : descs[n - 1];  // (any valid descriptor for helper lanes)
    }
    const bool bad_slot = d.key_idx >= key_cap;    // never dereferenced: the packet is refused
    const DevKey *__restrict__ key = keys + (bad_slot ? 0u : d.key_idx);
    // a slot outside the table, a freed slot or a header-key-only slot holds no packet key: refused (no AES kernel
    // takes such a packet either: the plan gives it no work item with a round count)
    const bool refused = bad_slot || key->live != 1;
    if (refused && valid && status && !(d.flags & QPP_PKT_SKIP)) status[pi] = QPP_INTERNAL_ERROR;
    const bool has = valid && !refused && key->suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256 &&
                     !(d.flags & QPP_PKT_SKIP);
    if (!__any(has)) return;  // wave-uniform: AES packets go to the AES kernels
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t stage = (threadIdx.x >> 6) * kChachaWaveLds, tab = stage + kChachaStage;
    uint32_t k[8];
#pragma unroll
    for (int i = 0; i < 8; i++) k[i] = key->rk[i];
    // Iv::nonce (src/iv.rs:27-39)
    const uint32_t n0 = key->iv[0], n1 = key->iv[1] ^ bswap32((uint32_t)(d.pn >> 32)), n2 = key->iv[2] ^ bswap32((uint32_t)d.pn);
    uint8_t *base = arena + d.off;
    const uint32_t aad_len = d.aad_len, len = has ? d.pt_len : 0;
    uint8_t *pay = base + aad_len;

    uint32_t ks[16];
    chacha_block(k, 0, n0, n1, n2, ks);  // one-time Poly1305 key
    Poly1305 mac;
    mac.init(ks[0], ks[1], ks[2], ks[3]);
    const uint32_t sw0 = ks[4], sw1 = ks[5], sw2 = ks[6], sw3 = ks[7];
    if (has)
        for (uint32_t off = 0; off < aad_len; off += 16) {
            uint4 a = ld16(base + off);
            if (aad_len - off < 16) a = keep_bytes(a, aad_len - off);
            mac.block(a);
        }
    const uint32_t nch = (len + 63) / 64;  // chunks, the partial tail included
    const uint32_t C = wave_max(nch);
    lds_st64(tab + 8u * lane, make_uint2((uint32_t)(pay - arena), len));
    wave_lds_sync();
    // lane-linear role in pair instruction i: packet 8 i + lane / 8, block j of the pair
    // (lj(i) + rho(p)) % 8 = lane % 8, rho(p) = (lane / 8 + i / 2) % 8
    auto lj = [&](int i) { return ((lane & 7u) - (lane / 8u + (uint32_t)(i >> 1))) & 7u; };
    auto own_slot = [&](uint32_t j) {
        return stage + 16u * (64u * (lane / 8u) + 8u * (lane % 8u) + ((j + chacha_rho(lane)) & 7u));
    };
    // Interior pairs (wave-uniform test): all 8 blocks of pair m are whole payload blocks of every packet of the wave,
    // so the pair moves without clamps or predicated stores (as the AES kernels' interior groups)
    const uint32_t min_full = __builtin_amdgcn_readfirstlane(wave_min(has ? (len >> 4) : 0u));
    auto inner_pair = [&](uint32_t m) { return 8u * m + 8u <= min_full; };
    // pair m = blocks 8 m .. 8 m + 7, clamped inside payload||tag (unused when out of range)
    auto pair_load = [&](uint32_t m, uint4 (&r)[8]) {
        if (inner_pair(m)) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const uint32_t ox = lds_ld32(tab + 8u * (8u * i + lane / 8u));
                r[i] = ld16(arena + ox + 16u * (8u * m + lj(i)));
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint2 ol = lds_ld64(tab + 8u * (8u * i + lane / 8u));
            const uint32_t o = 16u * (8u * m + lj(i));
            r[i] = ld16(arena + ol.x + (o < ol.y ? o : 0u));
        }
    };
    auto pair_store = [&](uint32_t m) {  // the full blocks of pair m of the wave's 64 packets
        if (inner_pair(m)) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const uint4 v = lds_ld128(stage + 16u * (64u * i + lane));
                const uint32_t ox = lds_ld32(tab + 8u * (8u * i + lane / 8u));
                st16_nt(arena + ox + 16u * (8u * m + lj(i)), v);
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint4 v = lds_ld128(stage + 16u * (64u * i + lane));
            const uint2 ol = lds_ld64(tab + 8u * (8u * i + lane / 8u));
            const uint32_t o = 16u * (8u * m + lj(i));
            if (o + 16 <= ol.y) st16_nt(arena + ol.x + o, v);
        }
    };
    uint4 rin[8], cb[4];
    pair_load(0, rin);
    chacha_block(k, 1, n0, n1, n2, ks);
    for (uint32_t c = 0; c < C; c++) {
        if (!(c & 1u)) {  // pair top: the pair's inputs into the stage, the next pair's loads issued
#pragma unroll
            for (int i = 0; i < 8; i++) lds_st128(stage + 16u * (64u * i + lane), rin[i]);
            pair_load((c >> 1) + 1, rin);
            wave_lds_sync();
        }
        uint4 in[4];
#pragma unroll
        for (int q = 0; q < 4; q++) in[q] = lds_ld128(own_slot(4u * (c & 1u) + q));
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t o = 64 * c + 16 * q;
            uint4 out = in[q] ^ make_uint4(ks[4 * q], ks[4 * q + 1], ks[4 * q + 2], ks[4 * q + 3]);
            lds_st128(own_slot(4u * (c & 1u) + q), out);  // full blocks leave through the pair store
            cb[q] = SEAL ? out : in[q];
            if (!inner_pair(c >> 1) && o < len && len - o < 16) {  // the partial last block: this lane stores its bytes
                const uint32_t r = len - o;
                out = keep_bytes(out, r);
                st_bytes(pay + o, out, r);
                cb[q] = SEAL ? out : keep_bytes(in[q], r);
            }
        }
        if ((c & 1u) || c + 1 == C) {
            wave_lds_sync();
            pair_store(c >> 1);
            wave_lds_sync();  // the next pair's inputs overwrite the stage
        }
        chacha_block(k, c + 2, n0, n1, n2, ks);  // next chunk ...
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (inner_pair(c >> 1) || 64 * c + 16 * q < len) mac.block(cb[q]);  // ... beside this chunk's MAC
    }
    if (!has) return;
    mac.block(make_uint4(aad_len, 0, len, 0));  // le64(aad_len) || le64(ct_len)
    const uint4 tag = mac.finish(sw0, sw1, sw2, sw3);

    if (SEAL) {
        st16(pay + len, tag);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // other lanes stored this packet's ciphertext
        int8_t st8 = QPP_OK;
        if (flags & (QPP_HP_MASK_OUT | QPP_HP_APPLY)) {
            const uint32_t s = 4 - d.pn_len;
            if (d.pn_len < 1 || d.pn_len > 4 || len < s) {
                st8 = QPP_DECODE_ERROR;
            } else {
                const uint4 smp = ld16(pay + s);
                uint32_t hk[8];
#pragma unroll
                for (int i = 0; i < 8; i++) hk[i] = key->hp_rk[i];
                uint32_t m1, m0 = chacha_hp_word(hk, smp, &m1);
                apply_mask(base, aad_len - d.pn_len, d.pn_len, m0, m1, masks + 5 * (size_t)pi, flags);
            }
        }
        if (status) status[pi] = st8;
    } else {
        const uint4 diff = tag ^ ld16(pay + len);
        const bool ok = (diff.x | diff.y | diff.z | diff.w) == 0;
        if (!ok) {
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            for (uint32_t o = 0; o < len; o += 16) {
                if (len - o >= 16) st16(pay + o, make_uint4(0, 0, 0, 0));
                else st_bytes(pay + o, make_uint4(0, 0, 0, 0), len - o);
            }
        }
        status[pi] = ok ? QPP_OK : QPP_DECRYPT_ERROR;
    }
}

// ---------------------------------------------------------------- small batches: one WAVE per packet
// The burst form of chacha_kernel (the AES twin is burst.hip): the 64 lanes of a wave split one packet
// (chacha_wave_packet, chacha_wave.h; the transmit-queue server runs the same code).
template <bool SEAL>
__global__ __launch_bounds__(256) void chacha_burst_kernel(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                          const qpp_pkt *__restrict__ descs, uint32_t n,
                                                          uint8_t *__restrict__ arena, uint8_t *masks, int8_t *status,
                                                          uint32_t flags) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t pi = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
    if (pi >= n) return;
    const qpp_pkt d = descs[pi];
    if (d.key_idx >= key_cap) {  // wave-uniform: a slot outside the table is refused, never dereferenced
        if (status && lane == 0 && !(d.flags & QPP_PKT_SKIP)) status[pi] = QPP_INTERNAL_ERROR;
        return;
    }
    const DevKey *__restrict__ key = keys + d.key_idx;
    if (key->live != 1) {  // freed or header-key-only slot: refused
        if (status && lane == 0 && !(d.flags & QPP_PKT_SKIP)) status[pi] = QPP_INTERNAL_ERROR;
        return;
    }
    if (key->suite != QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256 || (d.flags & QPP_PKT_SKIP)) return;  // wave-uniform
    uint32_t k[8];
#pragma unroll
    for (int i = 0; i < 8; i++) k[i] = key->rk[i];
    // Iv::nonce (src/iv.rs:27-39)
    const uint32_t n0 = key->iv[0], n1 = key->iv[1] ^ bswap32((uint32_t)(d.pn >> 32)), n2 = key->iv[2] ^ bswap32((uint32_t)d.pn);
    chacha_wave_packet<SEAL>(k, n0, n1, n2, key->hp_rk, d, arena, masks ? masks + 5 * (size_t)pi : nullptr,
                             status ? status + pi : nullptr,
                             flags, lane);
}

// Header-protection masks for any suite, one lane per packet; AES keys use the LDS T-tables with the
// lane's own round keys.  Sample at off + aad_len - pn_len + 4.
__global__ __launch_bounds__(1024) void hp_mask_kernel(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                      const qpp_pkt *__restrict__ descs, uint32_t n,
                                                      const uint8_t *__restrict__ arena, uint8_t *masks) {
    // 64 KiB of dynamic LDS (the launch reserves it), addressed by offset through lds_ld32/lds_st32
    build_aes_tables(0);
    __syncthreads();
    const uint32_t pi = blockIdx.x * blockDim.x + threadIdx.x;
    if (pi >= n) return;
    const qpp_pkt d = descs[pi];
    uint8_t *o = masks + 5 * (size_t)pi;
    if (d.key_idx >= key_cap) {  // no key: an all-zero mask (the caller's descriptor is wrong)
        o[0] = o[1] = o[2] = o[3] = o[4] = 0;
        return;
    }
    const DevKey *__restrict__ key = keys + d.key_idx;
    const uint4 smp = ld16(arena + d.off + d.aad_len - d.pn_len + 4);
    uint32_t m0, m1;
    if (key->suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256) {
        uint32_t hk[8];
#pragma unroll
        for (int i = 0; i < 8; i++) hk[i] = key->hp_rk[i];
        m0 = chacha_hp_word(hk, smp, &m1);
    } else {
        const AesLds aes = make_aes(0);
        uint4 m = key->hp_nr == 10 ? aes.encrypt<10>(smp, key->hp_rk) : aes.encrypt<14>(smp, key->hp_rk);
        m0 = m.x; m1 = m.y;
    }
    o[0] = (uint8_t)m0; o[1] = (uint8_t)(m0 >> 8); o[2] = (uint8_t)(m0 >> 16); o[3] = (uint8_t)(m0 >> 24); o[4] = (uint8_t)m1;
}

// Receive-side header unprotection for a GRO batch, one lane per packet:
//   sample at header_len + 4 (payload.rs:151-169) -> mask (header_key.rs:52-56) -> remove_header_protection in place
//   (header_crypto.rs:98-123: first byte, pn_len = (b0 & 3) + 1, PN bytes) -> expand the PN against the space's
//   largest acknowledged PN (packet/number/mod.rs:191-238) -> the packet key by the key-phase bit 0x04
//   (key_phase.rs:12,46; KeySet::decrypt_packet, keyset.rs:113-143; long headers: key_idx[0]) -> the qpp_pkt the
//   open kernels consume.  A packet too short for the sample is DECODE_ERROR and marked QPP_PKT_SKIP; a packet whose
//   chosen key is not a live packet key is INTERNAL_ERROR here already (no open kernel takes it, whatever the batch's
//   QPP_ONLY_* flags; the fused receive kernel decides the same in its phase A).
__global__ __launch_bounds__(1024) void unprotect_kernel(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                        const qpp_rx_pkt *__restrict__ rx, uint32_t n,
                                                        uint8_t *__restrict__ arena, qpp_pkt *descs_out,
                                                        int8_t *status) {
    // 64 KiB of dynamic LDS: the AES T-tables for the AES header keys
    build_aes_tables(0);
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint4 kw;
    const qpp_pkt d = rx_unprotect_one(make_aes(0), keys, key_cap, rx[i], arena, status, i, &kw);
    if (!(d.flags & QPP_PKT_SKIP) && kw.w != 1) status[i] = QPP_INTERNAL_ERROR;
    descs_out[i] = d;
}

}  // namespace

hipError_t launch_unprotect(const DevKey *keys, uint32_t key_cap, const qpp_rx_pkt *rx, uint32_t n, uint8_t *arena,
                            qpp_pkt *descs_out, int8_t *status, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(unprotect_kernel, dim3((n + 1023) / 1024), dim3(1024), 65536, s, keys, key_cap, rx, n, arena,
                       descs_out, status);
    return hipGetLastError();
}

hipError_t launch_chacha(bool seal, const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n,
                         uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags, bool burst, hipStream_t s) {
    if (!n) return hipSuccess;
    if (burst) {  // one wave per packet, 4 per workgroup
        if (seal)
            hipLaunchKernelGGL(chacha_burst_kernel<true>, dim3((n + 3) / 4), dim3(256), 0, s, keys, key_cap, descs, n, arena,
                               masks, status, flags);
        else
            hipLaunchKernelGGL(chacha_burst_kernel<false>, dim3((n + 3) / 4), dim3(256), 0, s, keys, key_cap, descs, n, arena,
                               masks, status, flags);
        return hipGetLastError();
    }
    const dim3 grid((n + 255) / 256), block(256);
    const uint32_t lds = 4u * kChachaWaveLds;  // 4 waves, 34 KiB
    if (seal)
        hipLaunchKernelGGL(chacha_kernel<true>, grid, block, lds, s, keys, key_cap, descs, n, arena, masks, status, flags,
                           nullptr, nullptr);
    else
        hipLaunchKernelGGL(chacha_kernel<false>, grid, block, lds, s, keys, key_cap, descs, n, arena, masks, status, flags,
                           nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_chacha_sel(const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n_max,
                             uint8_t *arena, int8_t *status, const uint32_t *sel, const uint32_t *sel_meta, hipStream_t s) {
    if (!n_max) return hipSuccess;
    const dim3 grid((n_max + 255) / 256), block(256);
    const uint32_t lds = 4u * kChachaWaveLds;
    hipLaunchKernelGGL((chacha_kernel<false, false>), grid, block, lds, s, keys, key_cap, descs, n_max, arena, nullptr,
                       status, 0u, nullptr, nullptr, sel, sel_meta);
    return hipGetLastError();
}

hipError_t launch_chacha_sel_batch(bool seal, const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n_max,
                                   uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags, const uint32_t *sel,
                                   const uint32_t *sel_meta, hipStream_t s) {
    if (!n_max) return hipSuccess;
    const dim3 grid((n_max + 255) / 256), block(256);
    const uint32_t lds = 4u * kChachaWaveLds;
    if (seal)
        hipLaunchKernelGGL((chacha_kernel<true, false>), grid, block, lds, s, keys, key_cap, descs, n_max, arena, masks,
                           status, flags, nullptr, nullptr, sel, sel_meta);
    else
        hipLaunchKernelGGL((chacha_kernel<false, false>), grid, block, lds, s, keys, key_cap, descs, n_max, arena, nullptr,
                           status, 0u, nullptr, nullptr, sel, sel_meta);
    return hipGetLastError();
}

hipError_t launch_chacha_rx(const DevKey *keys, uint32_t key_cap, const qpp_rx_pkt *rx, uint32_t n, uint8_t *arena,
                            qpp_pkt *descs_out, int8_t *status, hipStream_t s) {
    if (!n) return hipSuccess;
    const dim3 grid((n + 255) / 256), block(256);
    const uint32_t lds = 4u * kChachaWaveLds;
    hipLaunchKernelGGL((chacha_kernel<false, true>), grid, block, lds, s, keys, key_cap, nullptr, n, arena, nullptr,
                       status, 0u, rx, descs_out);
    return hipGetLastError();
}

hipError_t launch_hp_mask(const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n,
                          const uint8_t *arena, uint8_t *masks, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(hp_mask_kernel, dim3((n + 1023) / 1024), dim3(1024), 65536, s, keys, key_cap, descs, n,
                       arena, masks);
    return hipGetLastError();
}

}  // namespace qpp
