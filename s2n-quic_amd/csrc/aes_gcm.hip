// aes_gcm.hip — AES-128/256-GCM seal/open + AES header protection for gfx950 (MI355X).
//
// Replaces the aws-lc-rs calls behind quic/s2n-quic-crypto:
//   seal  <LessSafeKey as Aead>::encrypt -> seal_in_place_scatter   src/aead/default.rs:44-62
//   open  <LessSafeKey as Aead>::decrypt -> open_in_place           src/aead/default.rs:65-93
//   HP    HeaderKey::header_protection_mask -> new_mask             src/header_key.rs:52-56
// with the nonce of Iv::nonce (src/iv.rs:27-39).
//
// Mapping: one LANE per packet.  A packet's CTR keystream, its ciphertext and its
// GHASH chain stay in one lane's registers from the first block to the tag, so there is no
// cross-lane traffic at all.  A workgroup = 1024 packets that share one key (the plan kernels
// group a mixed-key batch), because both lookup tables live in LDS:
//   [0, 64 KiB)     GHASH tables T_j[x] = (x at byte j) * H, 16 positions x 256 entries x 16 B
//   [64, 128 KiB)   AES T0/T1 replicated once per LDS bank: row x = 256 B = T0[x] x 32 banks | T1[x] x 32 banks,
//                   so a lane's lookup always hits bank (lane % 32): conflict-free, and its address
//                   (x << 8 | lane*4 | 64 KiB) is ONE v_perm_b32 from the state word.
//   [128, 130 KiB)  V[m] = H * x^m staging for the GHASH table build.
// AES rounds: T0[a] ^ T1[b] ^ rotl16(T0[c] ^ T1[d]) ^ rk (T2 = rotl16 T0, T3 = rotl16 T1).
#include <stdlib.h>

#include "device_common.h"

namespace qpp {
namespace {
using namespace dev;

// ---------------------------------------------------------------- GHASH: Y <- Y * H via 16 byte tables in LDS
// X * H = xor_j T_j[x_j] (GF(2)-linear in X).  The running value is kept as Z = Y ^ C_next so that the
// xor with the next block folds into the last xor3 of the table reduction.
struct GhashLds {
    const uint8_t *lds;
    template <int J>
    __device__ __forceinline__ uint4 tj(uint32_t w) const {
        constexpr int kShift = 8 * (J & 3);
        uint32_t off = ((w >> kShift) & 0xffu) << 4;
        return *(const uint4 *)(lds + kLdsGhash + J * 4096 + off);
    }
    // returns z * H ^ c
    __device__ __forceinline__ uint4 mulx(uint4 z, uint4 c) const {
        uint4 a = xor3(tj<0>(z.x), tj<1>(z.x), tj<2>(z.x));
        uint4 b = xor3(tj<3>(z.x), tj<4>(z.y), tj<5>(z.y));
        uint4 d = xor3(tj<6>(z.y), tj<7>(z.y), tj<8>(z.z));
        uint4 e = xor3(tj<9>(z.z), tj<10>(z.z), tj<11>(z.z));
        uint4 f = xor3(tj<12>(z.w), tj<13>(z.w), tj<14>(z.w));
        uint4 g = xor3(a, b, d);
        uint4 h = xor3(e, f, tj<15>(z.w));
        return xor3(g, h, c);
    }
};

// ---------------------------------------------------------------- phased group: AES-CTR x NB + GHASH, LDS-batched
// hipcc left to itself keeps only 2-4 LDS reads in flight per wave (it trades latency for registers), so the
// group is written as explicit phases: every lookup of one AES round for all NB blocks, plus the 16 lookups of
// one GHASH step, is issued before a scheduling barrier, and the xors follow it.  One phase per AES round; the
// NB GHASH steps of the previous group ride in the first NB phases.
__device__ __forceinline__ void gh_load(const GhashLds &gh, uint4 z, uint4 (&m)[16]) {
    m[0] = gh.tj<0>(z.x);   m[1] = gh.tj<1>(z.x);   m[2] = gh.tj<2>(z.x);   m[3] = gh.tj<3>(z.x);
    m[4] = gh.tj<4>(z.y);   m[5] = gh.tj<5>(z.y);   m[6] = gh.tj<6>(z.y);   m[7] = gh.tj<7>(z.y);
    m[8] = gh.tj<8>(z.z);   m[9] = gh.tj<9>(z.z);   m[10] = gh.tj<10>(z.z); m[11] = gh.tj<11>(z.z);
    m[12] = gh.tj<12>(z.w); m[13] = gh.tj<13>(z.w); m[14] = gh.tj<14>(z.w); m[15] = gh.tj<15>(z.w);
}
__device__ __forceinline__ uint4 gh_reduce(const uint4 (&m)[16], uint4 c) {
    const uint4 a = xor3(m[0], m[1], m[2]), b = xor3(m[3], m[4], m[5]), d = xor3(m[6], m[7], m[8]);
    const uint4 e = xor3(m[9], m[10], m[11]), f = xor3(m[12], m[13], m[14]);
    return xor3(xor3(a, b, d), xor3(e, f, m[15]), c);
}
__device__ __forceinline__ void round_load(const AesLds &a, const uint32_t (&s)[4], uint32_t (&t)[16]) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
        t[4 * c + 0] = a.t0<0>(s[c]);
        t[4 * c + 1] = a.t1<1>(s[(c + 1) & 3]);
        t[4 * c + 2] = a.t0<2>(s[(c + 2) & 3]);
        t[4 * c + 3] = a.t1<3>(s[(c + 3) & 3]);
    }
}
__device__ __forceinline__ void round_mix(const uint32_t (&t)[16], const uint32_t *__restrict__ rk, uint32_t (&s)[4]) {
#pragma unroll
    for (int c = 0; c < 4; c++) s[c] = xor3(t[4 * c], t[4 * c + 1], rk[c]) ^ rotl16(t[4 * c + 2] ^ t[4 * c + 3]);
}
__device__ __forceinline__ uint4 round_final(const uint32_t (&t)[16], const uint32_t *__restrict__ rk) {
    uint32_t o[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const uint32_t lo = __builtin_amdgcn_perm(t[4 * c + 1], t[4 * c], 0x0c0c0601u);
        const uint32_t hi = __builtin_amdgcn_perm(t[4 * c + 3], t[4 * c + 2], 0x07020c0cu);
        o[c] = xor3(lo, hi, rk[c]);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}
#define QPP_PHASE_BARRIER() __builtin_amdgcn_sched_barrier(0)

// Keystream of NB counter blocks c..c+NB-1 into ks[]; if GH, also absorbs cb[0..NB-1] into the GHASH chain z.
template <int NR, int NB, bool CACHED, bool GH>
__device__ __forceinline__ void group_phased(const AesLds &a, const GhashLds &gh, const CtrPage &pg,
                                             const uint32_t *__restrict__ rk, uint32_t n0, uint32_t n1, uint32_t n2,
                                             uint32_t c, uint4 (&ks)[NB], uint4 &z, const uint4 (&cb)[NB]) {
    uint32_t s[NB][4];
    uint32_t t[NB][16];
    uint4 gm[16];
    int phase = 0;  // GHASH step done in this phase (compile-time after unrolling)
    if constexpr (CACHED) {
        // phase 1: the one varying lookup of round 1 (T3[x], x = counter byte ^ rk)
        uint32_t tv[NB];
#pragma unroll
        for (int j = 0; j < NB; j++) tv[j] = a.t1<0>(((c + j) & 0xffu) ^ pg.x3);
        if (GH) gh_load(gh, z, gm);
        QPP_PHASE_BARRIER();
        uint32_t u0[NB];
#pragma unroll
        for (int j = 0; j < NB; j++) u0[j] = pg.k0 ^ rotl16(tv[j]);
        if (GH) z = gh_reduce(gm, cb[0]);
        phase++;
        // phase 2: four lookups of round 2
#pragma unroll
        for (int j = 0; j < NB; j++) {
            t[j][0] = a.t0<0>(u0[j]);
            t[j][1] = a.t1<3>(u0[j]);
            t[j][2] = a.t0<2>(u0[j]);
            t[j][3] = a.t1<1>(u0[j]);
        }
        if (GH && NB > 1) gh_load(gh, z, gm);
        QPP_PHASE_BARRIER();
#pragma unroll
        for (int j = 0; j < NB; j++) {
            s[j][0] = pg.l0 ^ t[j][0];
            s[j][1] = pg.l1 ^ rotl16(t[j][1]);
            s[j][2] = pg.l2 ^ rotl16(t[j][2]);
            s[j][3] = pg.l3 ^ t[j][3];
        }
        if (GH && NB > 1) z = gh_reduce(gm, cb[NB > 1 ? 1 : 0]);
        phase++;
    } else {
#pragma unroll
        for (int j = 0; j < NB; j++) {
            s[j][0] = n0 ^ rk[0]; s[j][1] = n1 ^ rk[1]; s[j][2] = n2 ^ rk[2]; s[j][3] = bswap32(c + j) ^ rk[3];
        }
#pragma unroll
        for (int r = 1; r <= 2; r++) {
#pragma unroll
            for (int j = 0; j < NB; j++) round_load(a, s[j], t[j]);
            if (GH && phase < NB) gh_load(gh, z, gm);
            QPP_PHASE_BARRIER();
#pragma unroll
            for (int j = 0; j < NB; j++) round_mix(t[j], rk + 4 * r, s[j]);
            if (GH && phase < NB) z = gh_reduce(gm, cb[phase < NB ? phase : 0]);
            phase++;
        }
    }
#pragma unroll
    for (int r = 3; r < NR; r++) {
#pragma unroll
        for (int j = 0; j < NB; j++) round_load(a, s[j], t[j]);
        if (GH && phase < NB) gh_load(gh, z, gm);
        QPP_PHASE_BARRIER();
#pragma unroll
        for (int j = 0; j < NB; j++) round_mix(t[j], rk + 4 * r, s[j]);
        if (GH && phase < NB) z = gh_reduce(gm, cb[phase < NB ? phase : 0]);
        phase++;
    }
#pragma unroll
    for (int j = 0; j < NB; j++) round_load(a, s[j], t[j]);
    if (GH && phase < NB) gh_load(gh, z, gm);
    QPP_PHASE_BARRIER();
#pragma unroll
    for (int j = 0; j < NB; j++) ks[j] = round_final(t[j], rk + 4 * NR);
    if (GH && phase < NB) z = gh_reduce(gm, cb[phase < NB ? phase : 0]);
    phase++;
#pragma unroll
    for (int j = 0; j < NB; j++)
        if (GH && j >= phase) z = gh.mulx(z, cb[j]);  // NB > NR: leftover steps
}

// Build both table sets for one key.  All 1024 threads take part; ends with a barrier.
__device__ void build_tables(uint8_t *lds, const DevKey *__restrict__ key) {
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    // V powers -> LDS
    for (uint32_t i = tid; i < 128; i += nthr) {
        const uint32_t *v = key->V[i];
        *(uint4 *)(lds + kLdsV + 16 * i) = make_uint4(v[0], v[1], v[2], v[3]);
    }
    build_aes_tables(lds);
    __syncthreads();
    // GHASH tables: entry e = 256 j + x; T_j[x] = xor of V[8j+i] over set bits (bit 7-i) of x
    for (uint32_t e = tid; e < 4096; e += nthr) {
        uint32_t j = e >> 8, x = e & 255;
        uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; i++)
            if ((x >> (7 - i)) & 1) acc = acc ^ *(const uint4 *)(lds + kLdsV + 16 * (8 * j + i));
        *(uint4 *)(lds + kLdsGhash + 16 * e) = acc;
    }
    __syncthreads();
}

struct PacketView {
    uint8_t *base;       // packet start (AAD)
    uint32_t aad_len, len, pn_len;
    uint32_t n0, n1, n2; // nonce words
};

__device__ __forceinline__ PacketView load_packet(const qpp_pkt &d, const DevKey *__restrict__ key, uint8_t *arena) {
    PacketView p;
    p.base = arena + d.off;
    p.aad_len = d.aad_len;
    p.len = d.pt_len;
    p.pn_len = d.pn_len;
    // Iv::nonce: iv XOR (0u32 || pn_be64)  (src/iv.rs:27-39)
    p.n0 = key->iv[0];
    p.n1 = key->iv[1] ^ bswap32((uint32_t)(d.pn >> 32));
    p.n2 = key->iv[2] ^ bswap32((uint32_t)d.pn);
    return p;
}

// Header protection mask from the 16-byte sample (first 5 bytes of AES_hp(sample)).  The HP round keys are read
// here through a volatile pointer so the compiler cannot hoist them into SGPRs for the whole kernel: they are
// used once per packet, and hoisting them spills the packet round keys (measured: 36 SGPR spills, slower seal).
template <int HNR>
__device__ __forceinline__ void hp_finish(const AesLds &aes, const uint32_t *hp_rk_g, uint4 sample,
                                          uint8_t *base, uint32_t hdr_len, uint32_t pn_len, uint8_t *mask_out,
                                          uint32_t flags) {
    uint32_t hp_rk[4 * (HNR + 1)];
    const volatile uint4 *src = (const volatile uint4 *)hp_rk_g;
#pragma unroll
    for (int i = 0; i < HNR + 1; i++) {
        const uint4 v = make_uint4(src[i].x, src[i].y, src[i].z, src[i].w);
        hp_rk[4 * i] = v.x; hp_rk[4 * i + 1] = v.y; hp_rk[4 * i + 2] = v.z; hp_rk[4 * i + 3] = v.w;
    }
    uint4 m = aes.encrypt<HNR>(sample, hp_rk);
    if (flags & QPP_HP_MASK_OUT) {
        mask_out[0] = (uint8_t)m.x; mask_out[1] = (uint8_t)(m.x >> 8); mask_out[2] = (uint8_t)(m.x >> 16);
        mask_out[3] = (uint8_t)(m.x >> 24); mask_out[4] = (uint8_t)m.y;
    }
    if (flags & QPP_HP_APPLY) {
        // header_crypto.rs:80-95
        uint8_t b0 = base[0];
        base[0] = b0 ^ ((uint8_t)m.x & ((b0 & 0x80) ? 0x0f : 0x1f));
        uint32_t mm = (m.x >> 8) | (m.y << 24);
        for (uint32_t i = 0; i < pn_len; i++) base[hdr_len + i] ^= (uint8_t)(mm >> (8 * i));
    }
}

// GHASH over the AAD (zero-padded to 16 bytes), as the pending Z of the chain.
__device__ __forceinline__ uint4 ghash_aad_z(const GhashLds &gh, const uint8_t *aad, uint32_t aad_len) {
    uint4 z = make_uint4(0, 0, 0, 0);
    for (uint32_t off = 0; off < aad_len; off += 16) {
        uint4 a = ld16(aad + off);
        uint32_t r = aad_len - off;
        if (r < 16) a = keep_bytes(a, r);
        z = gh.mulx(z, a);
    }
    return z;
}

// One packet per lane.  Blocks are processed NB at a time: the keystream of group g+1 is computed in the same
// basic block as the GHASH chain of group g, so the two independent dependency chains overlap.
template <int NR, int NB, bool SEAL, bool PHASED>
__device__ __forceinline__ void process_packet(const AesLds &aes, const GhashLds &gh, const DevKey *__restrict__ key,
                                               const qpp_pkt &d, uint32_t pkt_index, uint8_t *arena, uint8_t *masks,
                                               int8_t *status, uint32_t flags) {
    const uint32_t *__restrict__ rk = key->rk;
    PacketView p = load_packet(d, key, arena);
    uint8_t *pay = p.base + p.aad_len;
    CtrPage pg;
    pg.build(aes, rk, p.n0, p.n1, p.n2, 0);
    // E_K(J0), J0 = nonce || 1 (page 0)
    uint4 ek0;
    {
        uint32_t s[4];
        pg.two_rounds(aes, 1, s);
#pragma unroll
        for (int r = 3; r < NR; r++) aes.round(s, rk + 4 * r);
        ek0 = aes.final(s, rk + 4 * NR);
    }
    // GHASH state Z = Y ^ (next block), so Y_next * H ^ C folds into one mulx.  Z starts at 0: a leading
    // zero block does not change GHASH, so every block (AAD included) is absorbed with the same step.
    uint4 z = ghash_aad_z(gh, p.base, p.aad_len);

    const uint32_t nfull = p.len >> 4, rem = p.len & 15;
    const uint32_t ngroups = nfull / NB;
    uint4 ks[NB], in[NB];
    const uint32_t ctr = 2;
    // group 0: loads stay inside payload||tag (a block start o is readable for 16 bytes iff o <= len)
#pragma unroll
    for (int j = 0; j < NB; j++) in[j] = ld16(16u * j <= p.len ? pay + 16 * j : pay);
    {
        uint4 none[NB];
        group_phased<NR, NB, true, false>(aes, gh, pg, rk, p.n0, p.n1, p.n2, ctr, ks, z, none);
    }
    // first two ciphertext blocks for the HP sample (used only when len >= 32, i.e. both are full blocks)
    uint4 c0 = SEAL ? in[0] ^ ks[0] : in[0];
    uint4 c1 = NB > 1 ? (SEAL ? in[NB > 1 ? 1 : 0] ^ ks[NB > 1 ? 1 : 0] : in[NB > 1 ? 1 : 0]) : c0;
    for (uint32_t g = 0; g < ngroups; g++) {
        uint4 cblk[NB];
#pragma unroll
        for (int j = 0; j < NB; j++) {
            const uint4 out = in[j] ^ ks[j];
            st16(pay + 16 * (NB * g + j), out);
            cblk[j] = SEAL ? out : in[j];
        }
        // next group's input blocks and keystream (also serve the tail after the last full group)
        const uint32_t nb = NB * (g + 1);
#pragma unroll
        for (int j = 0; j < NB; j++) {
            const uint32_t o = 16 * (nb + j);
            in[j] = ld16(o <= p.len ? pay + o : pay);
        }
        const uint32_t c = ctr + nb;
        if (PHASED) {
            // keystream of the next group with this group's GHASH steps interleaved phase by phase
            if (((c + NB - 1) >> 8) != (c >> 8)) {
                group_phased<NR, NB, false, true>(aes, gh, pg, rk, p.n0, p.n1, p.n2, c, ks, z, cblk);
            } else {
                if ((c >> 8) != pg.page) pg.build(aes, rk, p.n0, p.n1, p.n2, c >> 8);
                group_phased<NR, NB, true, true>(aes, gh, pg, rk, p.n0, p.n1, p.n2, c, ks, z, cblk);
            }
        } else {
            // keystream of the next group, then this group's GHASH chain; the compiler interleaves the two
            if (((c + NB - 1) >> 8) != (c >> 8)) {
                ctr_keystream_full<NR, NB>(aes, rk, p.n0, p.n1, p.n2, c, ks);
            } else {
                if ((c >> 8) != pg.page) pg.build(aes, rk, p.n0, p.n1, p.n2, c >> 8);
                ctr_keystream<NR, NB>(aes, pg, rk, c, ks);
            }
#pragma unroll
            for (int j = 0; j < NB; j++) z = gh.mulx(z, cblk[j]);
        }
    }
    // tail: up to NB-1 full blocks and one partial block; their keystream is already in ks[]
    const uint32_t done = NB * ngroups;
#pragma unroll
    for (int j = 0; j < NB; j++) {
        const uint32_t b = done + j;
        if (b < nfull) {
            const uint4 out = in[j] ^ ks[j];
            st16(pay + 16 * b, out);
            z = gh.mulx(z, SEAL ? out : in[j]);
        } else if (b == nfull && rem) {
            const uint4 out = keep_bytes(in[j] ^ ks[j], rem);
            st_bytes(pay + 16 * b, out, rem);
            z = gh.mulx(z, SEAL ? out : keep_bytes(in[j], rem));
        }
    }
    if (NB == 1 && p.len >= 32) c1 = ld16(pay + 16);  // NB == 1 has no second block in registers
    // length block: be64(aad bits) || be64(payload bits); then the final multiply
    z = gh.mulx(z, make_uint4(0, bswap32(p.aad_len * 8), 0, bswap32(p.len * 8)));
    const uint4 tag = gh.mulx(z, ek0);  // Y * H ^ E_K(J0)

    if (SEAL) {
        st16(pay + p.len, tag);
        int8_t st = QPP_OK;
        if (flags & (QPP_HP_MASK_OUT | QPP_HP_APPLY)) {
            // sample = ciphertext||tag bytes [4 - pn_len, 20 - pn_len)  (payload.rs:151-169)
            const uint32_t s = 4 - p.pn_len;
            if (p.pn_len < 1 || p.pn_len > 4 || p.len < s) {
                st = QPP_DECODE_ERROR;
            } else {
                uint4 smp;
                if (p.len >= 32) {
                    smp.x = __builtin_amdgcn_alignbyte(c0.y, c0.x, s);
                    smp.y = __builtin_amdgcn_alignbyte(c0.z, c0.y, s);
                    smp.z = __builtin_amdgcn_alignbyte(c0.w, c0.z, s);
                    smp.w = __builtin_amdgcn_alignbyte(c1.x, c0.w, s);
                } else {
                    smp = ld16(pay + s);  // short payload: sample reaches into the tag just stored
                }
                const uint32_t hdr_len = p.aad_len - p.pn_len;
                if (key->hp_nr == 10)
                    hp_finish<10>(aes, key->hp_rk, smp, p.base, hdr_len, p.pn_len, masks + 5 * (size_t)pkt_index, flags);
                else
                    hp_finish<14>(aes, key->hp_rk, smp, p.base, hdr_len, p.pn_len, masks + 5 * (size_t)pkt_index, flags);
            }
        }
        if (status) status[pkt_index] = st;
    } else {
        const uint4 want = ld16(pay + p.len);
        const uint4 diff = tag ^ want;
        const bool ok = (diff.x | diff.y | diff.z | diff.w) == 0;  // all 16 bytes compared, no early exit
        if (!ok) {
            // never release unauthenticated plaintext
            for (uint32_t b = 0; b < nfull; b++) st16(pay + 16 * b, make_uint4(0, 0, 0, 0));
            if (rem) st_bytes(pay + 16 * nfull, make_uint4(0, 0, 0, 0), rem);
        }
        status[pkt_index] = ok ? QPP_OK : QPP_DECRYPT_ERROR;
    }
}

template <bool SEAL, int NB, int WG, bool PHASED>
__global__ __launch_bounds__(WG) void aes_gcm_kernel(const DevKey *__restrict__ keys, const qpp_pkt *__restrict__ descs,
                                                    const uint32_t *__restrict__ perm, const WorkItem *__restrict__ work,
                                                    const uint32_t *__restrict__ n_work, uint8_t *__restrict__ arena,
                                                    uint8_t *masks, int8_t *status, uint32_t flags) {
#ifdef QPP_STATIC_LDS
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
#else
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];  // measured faster than static (seal), see DESIGN
#endif
    if (blockIdx.x >= *n_work) return;  // uniform: grid is sized for the worst case
    const WorkItem w = work[blockIdx.x];
    const DevKey *__restrict__ key = keys + w.key;
    build_tables(lds, key);
    const AesLds aes = make_aes(lds);
    const GhashLds gh{lds};
    for (uint32_t t = threadIdx.x; t < w.count; t += WG) {  // WG < 1024: several passes over the work item
        const uint32_t pi = perm[w.begin + t];
        const qpp_pkt d = descs[pi];
        if (w.nr == 10)
            process_packet<10, NB, SEAL, PHASED>(aes, gh, key, d, pi, arena, masks, status, flags);
        else
            process_packet<14, NB, SEAL, PHASED>(aes, gh, key, d, pi, arena, masks, status, flags);
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

__global__ void key_setup_kernel(DevKey *keys, uint32_t first, uint32_t count) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    DevKey *k = keys + first + i;
    if (!k->live || k->suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256) return;
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

hipError_t launch_key_setup(DevKey *keys, uint32_t first, uint32_t count, hipStream_t s) {
    if (!count) return hipSuccess;
    hipLaunchKernelGGL(key_setup_kernel, dim3((count + 63) / 64), dim3(64), 0, s, keys, first, count);
    return hipGetLastError();
}

namespace {
#ifdef QPP_STATIC_LDS
constexpr uint32_t kDynLds = 0;
#else
constexpr uint32_t kDynLds = kLdsBytes;
#endif
// (blocks per lane-iteration NB, workgroup size WG, packets per work item PER) variants; QPP_AES_VARIANT=<index>
// selects one (tuning knob).  One workgroup per CU (130 KiB LDS), so WG = waves per CU x 64.
struct Variant {
    int nb, wg, per;
    bool phased;
};
constexpr Variant kVariants[] = {{6, 512, 1024, false}, {4, 512, 1024, false}, {4, 512, 1024, true},
                                 {2, 512, 1024, true},  {2, 1024, 1024, false}, {8, 512, 1024, false},
                                 {4, 512, 512, false}};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

template <bool SEAL>
void launch_variant(int v, dim3 grid, hipStream_t s, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb,
                    uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags) {
#define QPP_AES_LAUNCH(NB, WG, PH)                                                                                 \
    hipLaunchKernelGGL((aes_gcm_kernel<SEAL, NB, WG, PH>), grid, dim3(WG), kDynLds, s, keys, descs, pb.perm,     \
                       pb.work, pb.n_work, arena, masks, status, flags)
    switch (v) {
        case 0: QPP_AES_LAUNCH(6, 512, false); break;
        case 1: QPP_AES_LAUNCH(4, 512, false); break;
        case 2: QPP_AES_LAUNCH(4, 512, true); break;
        case 3: QPP_AES_LAUNCH(2, 512, true); break;
        case 4: QPP_AES_LAUNCH(2, 1024, false); break;
        case 5: QPP_AES_LAUNCH(8, 512, false); break;
        default: QPP_AES_LAUNCH(4, 512, false); break;
    }
#undef QPP_AES_LAUNCH
}

int aes_variant() {
    static int v = [] {
        const char *e = getenv("QPP_AES_VARIANT");
        int x = e ? atoi(e) : kDefaultAesVariant;
        return (x >= 0 && x < kNumVariants) ? x : kDefaultAesVariant;
    }();
    return v;
}
}  // namespace

uint32_t aes_packets_per_item() { return (uint32_t)kVariants[aes_variant()].per; }

hipError_t launch_aes_gcm(bool seal, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb, uint32_t n,
                          uint32_t key_cap, uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags,
                          hipStream_t s) {
    if (!n) return hipSuccess;
    const dim3 grid(plan_max_work(n, key_cap, aes_packets_per_item()));
    if (seal)
        launch_variant<true>(aes_variant(), grid, s, keys, descs, pb, arena, masks, status, flags);
    else
        launch_variant<false>(aes_variant(), grid, s, keys, descs, pb, arena, masks, status, flags);
    return hipGetLastError();
}

}  // namespace qpp
