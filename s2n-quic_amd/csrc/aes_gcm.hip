// aes_gcm.hip — AES-128/256-GCM seal/open + AES header protection for gfx950 (MI355X).
//
// Replaces the aws-lc-rs calls behind quic/s2n-quic-crypto:
//   seal  <LessSafeKey as Aead>::encrypt -> seal_in_place_scatter   src/aead/default.rs:44-62
//   open  <LessSafeKey as Aead>::decrypt -> open_in_place           src/aead/default.rs:65-93
//   HP    HeaderKey::header_protection_mask -> new_mask             src/header_key.rs:52-56
// with the nonce of Iv::nonce (src/iv.rs:27-39).
//
// This file holds the MANY-KEY throughput kernel (aes_gcm_wave_kernel), the key setup kernels and the AES launchers;
// the one-key-per-slice throughput kernel is quad.hip's (four lanes per packet), the small-batch kernel burst.hip's.
//
// aes_gcm_wave_kernel (DESIGN.md §3 "Many keys"): one LANE per packet, one key per 64-packet WAVE.  A packet's CTR
// keystream, its ciphertext and its GHASH chain stay in one lane's registers from the first block to the tag; the
// wave's payload moves through a per-wave LDS staging area (Stage, coalesced 64-B chunks).  LDS:
//   [0, 64 KiB)     per-wave 4-bit GHASH tables of the wave's key (Ghash4, 8 KiB per wave)
//   [64, 128 KiB)   AES T0/T1 replicated once per LDS bank: row x = 256 B = T0[x] x 32 banks | T1[x] x 32 banks,
//                   so a lane's lookup always hits bank (lane % 32): conflict-free, and its address
//                   (x << 8 | lane*4 | 64 KiB) is ONE v_perm_b32 from the state word.
//   [128, 160 KiB)  payload staging (Stage<NB>).
// AES rounds: T0[a] ^ T1[b] ^ rotl16(T0[c] ^ T1[d]) ^ rk (T2 = rotl16 T0, T3 = rotl16 T1).
#include <stdlib.h>
#include <string.h>

#include "device_common.h"
#include "ghash.h"

namespace qpp {
namespace {
using namespace dev;

// GHASH over the AAD (zero-padded to 16 bytes), as the pending (rotated) Z of the chain.
template <typename GH>
__device__ __forceinline__ uint4 ghash_aad_w(const GH &gh, const uint8_t *aad, uint32_t aad_len) {
    uint4 w = make_uint4(0, 0, 0, 0);
    for (uint32_t off = 0; off < aad_len; off += 16) {
        uint4 a = ld16(aad + off);
        uint32_t r = aad_len - off;
        if (r < 16) a = keep_bytes(a, r);
        w = off ? gh.mulx(w, a) : gh.rot(a);  // Y_0 = 0: the first Z is the block itself
    }
    return w;
}

// One packet per lane (has = false: the lane only helps with the wave's cooperative I/O).  Counter blocks are
// grouped [NB*g + 1, NB*g + NB + 1): counter 1 is J0 (E_K(J0) masks the tag), counter b + 2 is data block b, so a
// packet of n blocks takes ceil((n + 1) / NB) groups (75 blocks: 19 groups of 4, not 20 with a discarded counter 0).
// A group normally lies inside one 256-block page (CtrPage constants hold for all of it); the group that straddles a
// page boundary (packets of >= 253 blocks, once per 256) is wave-uniform and takes full AES rounds.
// The GHASH steps of group g-1 are issued in the same loop body as the keystream of group g, so the two independent
// dependency chains overlap.
template <int NR, int NB, bool SEAL, typename GH>
__device__ __forceinline__ void process_packet(const AesLds &aes, const GH &gh, const Stage<NB> &st,
                                               const DevKey *__restrict__ key, const uint32_t *__restrict__ rk,
                                               bool has, const qpp_pkt &d, uint32_t pkt_index, uint8_t *arena,
                                               uint8_t *masks, int8_t *status, uint32_t flags) {
    static_assert(NB >= 2 && (256 % NB) == 0, "NB must divide 256");
    PacketView p = load_packet(d, key, arena);
    if (!has) p.len = 0;
    uint8_t *pay = p.base + p.aad_len;
    CtrPage pg;
    pg.build(aes, rk, p.n0, p.n1, p.n2, 0);
    uint4 z = has ? ghash_aad_w(gh, p.base, p.aad_len) : make_uint4(0, 0, 0, 0);  // rotated running value

    const int nfull = (int)(p.len >> 4), rem = (int)(p.len & 15);
    const int nblk = nfull + (rem ? 1 : 0);
    const int ngroups = has ? (nblk + 1 + NB - 1) / NB : 0;
    const int G = (int)wave_max((uint32_t)ngroups);  // the wave runs the longest packet's groups

    // cooperative roles: payload offset and length of the packet whose chunk this lane moves in instruction i
    uint32_t co_off[NB], co_len[NB], co_k[NB];
    const uint32_t my_off = (uint32_t)(pay - arena);
#pragma unroll
    for (int i = 0; i < NB; i++) {
        co_off[i] = (uint32_t)__shfl((int)my_off, (int)st.coop_src(i), 64);
        co_len[i] = (uint32_t)__shfl((int)p.len, (int)st.coop_src(i), 64);
        co_k[i] = st.coop_chunk(i);
    }
    // Interior groups (wave-uniform test): every chunk the wave moves in group g is a whole payload block of its packet
    // (g >= 1 and NB g + NB - 2 < the wave's shortest payload in blocks), so loads and stores need no clamp and no
    // branch, and address from a uniform base (SGPRs) + a per-lane 32-bit offset fixed for the whole packet.  Edge
    // groups (the first, the last ones of the shortest packet) keep the clamped, predicated form.
    const uint32_t min_full = __builtin_amdgcn_readfirstlane(wave_min(has ? (p.len >> 4) : 0u));  // uniform: a scalar branch
    auto interior = [&](int g) { return g >= 1 && (uint32_t)(NB * g + NB - 1) <= min_full; };
    uint32_t co_vo[NB];  // chunk k of the role's packet at group g: arena + (16 NB g - 16) + co_vo
#pragma unroll
    for (int i = 0; i < NB; i++) co_vo[i] = co_off[i] + 16u * co_k[i];
    // chunk of block b = NB g - 1 + k, clamped inside payload||tag (its value is unused when out of range)
    auto co_load = [&](int g, uint4 (&v)[NB]) {
        if (interior(g)) {
            const uint8_t *gb = arena + (16u * NB * (uint32_t)g - 16u);
#pragma unroll
            for (int i = 0; i < NB; i++) v[i] = ld16(gb + co_vo[i]);
            return;
        }
#pragma unroll
        for (int i = 0; i < NB; i++) {
            const int b = NB * g - 1 + (int)co_k[i];
            const bool ok = b >= 0 && 16 * b <= (int)co_len[i];
            v[i] = ld16(arena + co_off[i] + (ok ? 16u * (uint32_t)b : 0u));
        }
    };

    uint4 ks[NB], cin[NB], ek0 = make_uint4(0, 0, 0, 0), smp = make_uint4(0, 0, 0, 0);
    // Cooperative stores of group g-1 are issued at the top of iteration g, AFTER this group's prefetched loads
    // have been consumed: vmcnt counts loads and stores together, so a store issued behind a prefetch would make
    // the next wait for that prefetch also wait for the store's write acknowledgement.
    auto co_store = [&](int g, const uint4 (&v)[NB]) {
        if (interior(g)) {
            uint8_t *gb = arena + (16u * NB * (uint32_t)g - 16u);
#pragma unroll
            for (int i = 0; i < NB; i++) st16_nt(gb + co_vo[i], v[i]);
            return;
        }
#pragma unroll
        for (int i = 0; i < NB; i++) {
            const int b = NB * g - 1 + (int)co_k[i];
            if (b >= 0 && b < (int)(co_len[i] >> 4)) st16_nt(arena + co_off[i] + 16u * (uint32_t)b, v[i]);
        }
    };
    co_load(0, cin);
    for (int g = 0; g < G; g++) {
        uint4 co_out[NB];
        if (g) {  // the previous group's outputs, still in the staging area
#pragma unroll
            for (int i = 0; i < NB; i++) co_out[i] = lds_ld128(st.coop(i));
            wave_lds_sync();
        }
        // this group's inputs: coalesced chunks -> LDS -> my packet's blocks
#pragma unroll
        for (int i = 0; i < NB; i++) lds_st128(st.coop(i), cin[i]);
        if (g) co_store(g - 1, co_out);
        wave_lds_sync();
        uint4 in[NB];
#pragma unroll
        for (int j = 0; j < NB; j++) in[j] = lds_ld128(st.own(j));
        co_load(g + 1, cin);  // prefetch the next group (latency hidden by this group's AES)

        const uint32_t c = (uint32_t)(NB * g + 1);  // counter of slot 0 (wave-uniform)
        if (((c + NB - 1) >> 8) == (c >> 8)) {
            if ((c >> 8) != pg.page) pg.build(aes, rk, p.n0, p.n1, p.n2, c >> 8);
            ctr_keystream_pipe<NR, NB>(aes, pg, rk, c, ks);  // +3-4 % over the scheduler's own order
        } else {  // straddles a page boundary: plain rounds (unrolled: a runtime index into ks[] would make the
                  // compiler move the array to LDS, on top of the 160 KiB the launch reserves)
            static_for<NB>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                ks[j] = aes.encrypt<NR>(make_uint4(p.n0, p.n1, p.n2, bswap32(c + j)), rk);
            });
        }
        if (g == 0) {
            ek0 = ks[0];
            // header-protection sample = ciphertext bytes [4 - pn_len, 20 - pn_len) (payload.rs:151-169), from
            // blocks 0 and 1 (slots 1 and 2 of group 0) while they are in registers; packets whose sample reaches
            // into the tag (payload < 20 - pn_len bytes) read it back from memory at the end instead
            if constexpr (SEAL && NB >= 3) {
                const uint4 o1 = in[1] ^ ks[1], o2 = in[2] ^ ks[2];
                const uint32_t sh = (4u - p.pn_len) & 3u;
                smp = make_uint4(__builtin_amdgcn_alignbyte(o1.y, o1.x, sh), __builtin_amdgcn_alignbyte(o1.z, o1.y, sh),
                                 __builtin_amdgcn_alignbyte(o1.w, o1.z, sh), __builtin_amdgcn_alignbyte(o2.x, o1.w, sh));
            }
        }
        const int b0 = NB * g - 1;  // data block of slot 0
        const bool inner = interior(g);  // uniform: every lane's NB blocks are whole payload blocks
        uint4 cg[NB];               // the group's ciphertext blocks, for GHASH
#pragma unroll
        for (int j = 0; j < NB; j++) {
            const int b = b0 + j;
            const uint4 out = in[j] ^ ks[j];
            lds_st128(st.own(j), out);  // full blocks leave through the cooperative store below
            cg[j] = SEAL ? out : in[j];  // (unused unless 0 <= b < nblk)
            if (!inner && b == nfull && rem) {
                const uint4 o = keep_bytes(out, rem);
                st_bytes(pay + 16 * b, o, rem);
                cg[j] = SEAL ? o : keep_bytes(in[j], rem);
            }
        }
        // GHASH of the group.  Inside the packets (every lane's NB blocks valid: all but the first and last groups of a
        // uniform batch) the steps run branch-free, so the word rotation is a select and no exec-mask bookkeeping
        // surrounds each step.  (Deferring them behind the next group's keystream kept 16 more VGPRs live for no
        // overlap: the keystream pipeline is fenced by scheduling barriers.)
        if (inner || __all(b0 >= 0 && b0 + NB <= nblk)) {
#pragma unroll
            for (int j = 0; j < NB; j++) z = gh.mulx(z, cg[j]);
        } else {
#pragma unroll
            for (int j = 0; j < NB; j++)
                if (b0 + j >= 0 && b0 + j < nblk) z = gh.mulx(z, cg[j]);
        }
        wave_lds_sync();
    }
    if (G) {
        uint4 co_out[NB];
#pragma unroll
        for (int i = 0; i < NB; i++) co_out[i] = lds_ld128(st.coop(i));
        co_store(G - 1, co_out);
        wave_lds_sync();  // the next packet pass reuses the staging area
    }
    // HP round keys and header bytes: loads issued here, used after the last GHASH steps
    constexpr int HNR = NR == 10 ? 10 : 14;
    const bool hp = SEAL && (flags & (QPP_HP_MASK_OUT | QPP_HP_APPLY)) && has && p.pn_len >= 1 && p.pn_len <= 4 &&
                    p.len >= 4 - p.pn_len;
    const uint32_t hdr_len = p.aad_len - p.pn_len;
    HpPrefetch<HNR> hpk;
    if (hp) hpk.load(key->hp_rk, p.base, hdr_len, flags);
    if (!has) return;
    // length block: be64(aad bits) || be64(payload bits); tag = Y * H ^ E_K(J0)
    z = gh.mulx(z, make_uint4(0, bswap32(p.aad_len * 8), 0, bswap32(p.len * 8)));
    const uint4 tag = gh.prod(z, ek0);

    if (SEAL) {
        st16(pay + p.len, tag);
        int8_t st = QPP_OK;
        if (flags & (QPP_HP_MASK_OUT | QPP_HP_APPLY)) {
            if (!hp) {
                st = QPP_DECODE_ERROR;
            } else {
                if (NB < 3 || p.len < 20 - p.pn_len) {
                    // the sample reaches into the tag: read ciphertext||tag back (blocks 0/1 were stored by OTHER
                    // lanes of this wave, the tail and the tag by this lane: a wavefront fence orders them first)
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    smp = ld16(pay + 4 - p.pn_len);
                }
                hpk.finish(aes, smp, p.base, hdr_len, p.pn_len, masks + 5 * (size_t)pkt_index, flags);
            }
        }
        if (status) status[pkt_index] = st;
    } else {
        const uint4 want = ld16(pay + p.len);
        const uint4 diff = tag ^ want;
        const bool ok = (diff.x | diff.y | diff.z | diff.w) == 0;  // all 16 bytes compared, no early exit
        if (!ok) {
            // never release unauthenticated plaintext (other lanes stored it: order these stores after theirs)
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            for (int b = 0; b < nfull; b++) st16(pay + 16 * b, make_uint4(0, 0, 0, 0));
            if (rem) st_bytes(pay + 16 * nfull, make_uint4(0, 0, 0, 0), rem);
        }
        status[pkt_index] = ok ? QPP_OK : QPP_DECRYPT_ERROR;
    }
}

// Many keys, few packets per key (key churn, a chunk of a host batch): work items of <= 64 packets of one key (a
// wave), each wave with its own key's Ghash4 tables and round keys, the AES T-tables shared by the workgroup.  A
// workgroup loops over items (grid-stride over waves), so every lane has a packet whenever its key has >= 64 packets
// in the batch (aes_gcm_quad_kernel wants ~1024 per workgroup: its tables are rebuilt per key segment).
template <bool SEAL, int NB, int NR>
__global__ __launch_bounds__(512) void aes_gcm_wave_kernel(const DevKey *__restrict__ keys,
                                                           const qpp_pkt *__restrict__ descs,
                                                           const uint32_t *__restrict__ perm,
                                                           const WorkItem *__restrict__ work,
                                                           const uint32_t *__restrict__ n_work,
                                                           uint8_t *__restrict__ arena, uint8_t *masks, int8_t *status,
                                                           uint32_t flags) {
    const uint32_t nw = *n_work;
    if (blockIdx.x * 8u >= nw) return;  // uniform
    build_aes_tables(kLdsAes);
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const AesLds aes = make_aes(kLdsAes);
    const Ghash4 gh = Ghash4::make(wave);
    Stage<NB> st;
    st.lane = lane;
    st.base = kLdsStage + wave * (64u * 16u * NB);
    for (uint32_t it = blockIdx.x * 8u + wave; it < nw; it += gridDim.x * 8u) {  // wave-uniform
        const WorkItem w = work[it];
        if (w.nr != NR) continue;  // the other AES size's launch serves it
        const DevKey *__restrict__ key = keys + w.key;
        build_gh4(key, wave, lane);
        uint32_t rk[4 * (NR + 1)];
#pragma unroll
        for (int i = 0; i < 4 * (NR + 1); i++) rk[i] = __builtin_amdgcn_readfirstlane(key->rk[i]);
        const bool real = lane < w.count;
        const uint32_t pi = real ? perm[w.begin + lane] : perm[w.begin];
        const qpp_pkt d = descs[pi];
        const bool has = real && !(d.flags & QPP_PKT_SKIP);
        process_packet<NR, NB, SEAL>(aes, gh, st, key, rk, has, d, pi, arena, masks, status, flags);
        wave_lds_sync();  // the next item rebuilds this wave's tables
    }
}

// ---------------------------------------------------------------- key setup: H = E_K(0), V[m] = H * x^m
__device__ void aes_bytewise(const uint32_t *rk, int nr, uint8_t s[16]) {
    auto rkb = [rk](int i) { return (uint8_t)(rk[i >> 2] >> (8 * (i & 3))); };
    for (int i = 0; i < 16; i++) s[i] ^= rkb(i);
    for (int r = 1; r <= nr; r++) {
        uint8_t t[16];
        for (int c = 0; c < 4; c++)
            for (int i = 0; i < 4; i++) t[4 * c + i] = d_sbox[s[4 * ((c + i) & 3) + i]];
        for (int c = 0; c < 4; c++) {
            uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
            if (r != nr) {
                uint8_t x = a0 ^ a1 ^ a2 ^ a3;
                s[4 * c + 0] = a0 ^ x ^ (uint8_t)xtime4(a0 ^ a1);
                s[4 * c + 1] = a1 ^ x ^ (uint8_t)xtime4(a1 ^ a2);
                s[4 * c + 2] = a2 ^ x ^ (uint8_t)xtime4(a2 ^ a3);
                s[4 * c + 3] = a3 ^ x ^ (uint8_t)xtime4(a3 ^ a0);
            } else {
                s[4 * c] = a0; s[4 * c + 1] = a1; s[4 * c + 2] = a2; s[4 * c + 3] = a3;
            }
        }
        for (int i = 0; i < 16; i++) s[i] ^= rkb(16 * r + i);
    }
}

// Key install: record i (when records != nullptr) is copied into slot slots[i], then H = E_K(0) and V[m] = H * x^m are
// derived for it.  A slot list (not a range) so that retired slots can be reused and a live slot next to a new one is
// never rewritten while in-flight batches read it.  Header-key-only records (live == 2) and ChaCha keys need no GHASH
// powers.
__global__ void key_install_kernel(DevKey *keys, const uint32_t *__restrict__ slots,
                                   const DevKey *__restrict__ records, uint32_t count) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    DevKey *k = keys + slots[i];
    if (records) {
        const uint4 *src = (const uint4 *)(records + i);
        uint4 *dst = (uint4 *)k;
        for (uint32_t w = 0; w < sizeof(DevKey) / 16; w++) dst[w] = src[w];
    }
    if (k->live != 1 || k->suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256) return;
    uint8_t v[16] = {0};
    aes_bytewise(k->rk, (int)k->nr, v);
    for (int m = 0; m < 128; m++) {
        for (int w = 0; w < 4; w++)
            k->V[m][w] = (uint32_t)v[4 * w] | ((uint32_t)v[4 * w + 1] << 8) | ((uint32_t)v[4 * w + 2] << 16) |
                         ((uint32_t)v[4 * w + 3] << 24);
        if (m == 0)
            for (int w = 0; w < 4; w++) k->H[w] = k->V[0][w];
        // v <- v * x : shift right by one bit in GCM order, reduce by 0xE1 || 0^120
        int lsb = v[15] & 1;
        for (int b = 15; b > 0; b--) v[b] = (uint8_t)((v[b] >> 1) | (v[b - 1] << 7));
        v[0] >>= 1;
        if (lsb) v[0] ^= 0xe1;
    }
}

}  // namespace

hipError_t launch_key_install(DevKey *keys, const uint32_t *slots, const DevKey *records, uint32_t count,
                              const PowTables &pow, hipStream_t s) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(key_install_kernel, dim3((count + 63) / 64), dim3(64), 0, s, keys, slots, records, count);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_pow_setup(keys, slots, count, pow, s);
}

hipError_t launch_aes_gcm_single(bool seal, const DevKey *keys, const qpp_pkt *descs, uint32_t slot, uint32_t nr,
                                 uint32_t n, uint32_t n_cu, uint8_t *arena, uint8_t *masks, int8_t *status,
                                 uint32_t flags, const PowTables &pow, hipStream_t s) {
    if (!n) return hipSuccess;
    const PlanBuffers none{};
    const uint32_t waves = (n + 15) / 16;  // quad layout: 16 packets per wave
    const dim3 grid(waves < n_cu ? waves : n_cu);
    return launch_aes_gcm_quad(seal, nr, grid, s, keys, descs, none, arena, masks, status, flags, slot, n, pow);
}

hipError_t launch_aes_gcm_wave(bool seal, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb, uint32_t n,
                               uint32_t key_cap, uint32_t n_cu, uint8_t *arena, uint8_t *masks, int8_t *status,
                               uint32_t flags, uint32_t suites, hipStream_t s) {
    if (!n) return hipSuccess;
    // one 160-KiB workgroup per CU: a grid of 2 rounds of the chip (the second round's workgroups start as the
    // first finish), each wave looping over the work items
    const uint32_t items = plan_max_work(n, key_cap, kWavePacketsPerItem);
    const uint32_t wgs = (items + 7) / 8;
    const dim3 grid(wgs < 2 * n_cu ? wgs : 2 * n_cu), block(512);
    const uint32_t lds = kLdsMax;
#define QPP_WAVE_LAUNCH(S, NR)                                                                                  \
    hipLaunchKernelGGL((aes_gcm_wave_kernel<S, 4, NR>), grid, block, lds, s, keys, descs, pb.perm, pb.work,      \
                       pb.n_work, arena, masks, status, flags)
    if (suites & (1u << QPP_SUITE_TLS_AES_128_GCM_SHA256)) {
        if (seal) QPP_WAVE_LAUNCH(true, 10);
        else QPP_WAVE_LAUNCH(false, 10);
    }
    if (suites & (1u << QPP_SUITE_TLS_AES_256_GCM_SHA384)) {
        if (seal) QPP_WAVE_LAUNCH(true, 14);
        else QPP_WAVE_LAUNCH(false, 14);
    }
#undef QPP_WAVE_LAUNCH
    return hipGetLastError();
}

hipError_t launch_aes_gcm(bool seal, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb, uint32_t n,
                          uint32_t n_cu, uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags,
                          uint32_t suites, const PowTables &pow, hipStream_t s) {
    if (!n) return hipSuccess;
    // one slice per CU (quad.hip); a batch smaller than a wave per CU takes fewer workgroups
    const uint32_t waves = (n + 15) / 16;
    const dim3 grid(waves < n_cu ? waves : n_cu);
    const bool a128 = suites & (1u << QPP_SUITE_TLS_AES_128_GCM_SHA256), a256 = suites & (1u << QPP_SUITE_TLS_AES_256_GCM_SHA384);
    // both sizes in ONE launch when both are live (each workgroup: its AES-128 slice, then its AES-256 slice), not
    // two serial full-chip launches
    if (a128 || a256)
        launch_aes_gcm_quad(seal, a128 && a256 ? 0u : a128 ? 10u : 14u, grid, s, keys, descs, pb, arena, masks, status,
                            flags, 0xffffffffu, 0, pow);
    return hipGetLastError();
}

}  // namespace qpp
