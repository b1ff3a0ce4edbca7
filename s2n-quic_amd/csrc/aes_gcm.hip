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
// here, once per packet, into VGPRs: hoisted into SGPRs for the whole kernel they pushed the packet round keys out
// of SGPRs (measured: 36 SGPR spills and per-iteration round-key reloads, a slower seal).
template <int HNR>
__device__ __forceinline__ void hp_finish(const AesLds &aes, const uint32_t *hp_rk_g, uint4 sample,
                                          uint8_t *base, uint32_t hdr_len, uint32_t pn_len, uint8_t *mask_out,
                                          uint32_t flags) {
    // launder the pointer through a VGPR: the loads below cannot be hoisted or kept in SGPRs
    uint64_t a = (uint64_t)hp_rk_g;
    asm volatile("" : "+v"(a));
    const uint4 *src = (const uint4 *)a;
    uint32_t hp_rk[4 * (HNR + 1)];
#pragma unroll
    for (int i = 0; i < HNR + 1; i++) {
        const uint4 v = src[i];
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

// One packet per lane.  Counter blocks are grouped [NB*g, NB*g + NB) with NB | 256, so a group never crosses a
// 256-block page (CtrPage constants hold for the whole group) and the packet runs through ONE loop body:
//   counter 0: unused (its keystream is discarded), counter 1: J0 -> E_K(J0) masks the tag,
//   counter b + 2: data block b.
// The GHASH steps of group g-1 are issued in the same basic block as the keystream of group g, so the two
// independent dependency chains overlap.
template <int NR, int NB, bool SEAL>
__device__ __forceinline__ void process_packet(const AesLds &aes, const GhashLds &gh, const DevKey *__restrict__ key,
                                               const qpp_pkt &d, uint32_t pkt_index, uint8_t *arena, uint8_t *masks,
                                               int8_t *status, uint32_t flags) {
    static_assert(NB >= 2 && (256 % NB) == 0, "NB must divide 256 (and hold counter 1)");
    const uint32_t *__restrict__ rk = key->rk;
    PacketView p = load_packet(d, key, arena);
    uint8_t *pay = p.base + p.aad_len;
    CtrPage pg;
    pg.build(aes, rk, p.n0, p.n1, p.n2, 0);
    uint4 z = ghash_aad_z(gh, p.base, p.aad_len);

    const int nfull = (int)(p.len >> 4), rem = (int)(p.len & 15);
    const int nblk = nfull + (rem ? 1 : 0);
    const int ngroups = (nblk + 2 + NB - 1) / NB;
    uint4 ks[NB], in[NB], cprev[NB], ek0 = make_uint4(0, 0, 0, 0);
    int bprev = -NB;  // first block index of the previous group (for its GHASH validity)
    // group 0 inputs: slots 0, 1 are counters 0 and 1 (no data)
#pragma unroll
    for (int j = 0; j < NB; j++) {
        const int b = j - 2;
        in[j] = ld16(b >= 0 && 16 * b <= (int)p.len ? pay + 16 * b : pay);
    }
    for (int g = 0; g < ngroups; g++) {
        const uint32_t c = (uint32_t)(NB * g);
        if ((c >> 8) != pg.page) pg.build(aes, rk, p.n0, p.n1, p.n2, c >> 8);
        ctr_keystream<NR, NB>(aes, pg, rk, c, ks);
        // GHASH of the previous group (independent of the keystream just issued)
#pragma unroll
        for (int j = 0; j < NB; j++)
            if (bprev + j >= 0 && bprev + j < nblk) z = gh.mulx(z, cprev[j]);
        if (g == 0) ek0 = ks[1];
        const int b0 = NB * g - 2;  // data block of slot 0
#pragma unroll
        for (int j = 0; j < NB; j++) {
            const int b = b0 + j;
            const uint4 out = in[j] ^ ks[j];
            if (b >= 0 && b < nfull) {
                st16(pay + 16 * b, out);
                cprev[j] = SEAL ? out : in[j];
            } else if (b == nfull && rem) {
                const uint4 o = keep_bytes(out, rem);
                st_bytes(pay + 16 * b, o, rem);
                cprev[j] = SEAL ? o : keep_bytes(in[j], rem);
            }
        }
        bprev = b0;
        // next group's input blocks (clamped inside payload||tag)
#pragma unroll
        for (int j = 0; j < NB; j++) {
            const int b = b0 + NB + j;
            in[j] = ld16(16 * b <= (int)p.len ? pay + 16 * b : pay);
        }
    }
#pragma unroll
    for (int j = 0; j < NB; j++)
        if (bprev + j >= 0 && bprev + j < nblk) z = gh.mulx(z, cprev[j]);
    // length block: be64(aad bits) || be64(payload bits); tag = Y * H ^ E_K(J0)
    z = gh.mulx(z, make_uint4(0, bswap32(p.aad_len * 8), 0, bswap32(p.len * 8)));
    const uint4 tag = gh.mulx(z, ek0);

    if (SEAL) {
        st16(pay + p.len, tag);
        int8_t st = QPP_OK;
        if (flags & (QPP_HP_MASK_OUT | QPP_HP_APPLY)) {
            // sample = ciphertext||tag bytes [4 - pn_len, 20 - pn_len)  (payload.rs:151-169), read back: the lane
            // wrote those bytes itself (same-lane store -> load ordering)
            const uint32_t s = 4 - p.pn_len;
            if (p.pn_len < 1 || p.pn_len > 4 || p.len < s) {
                st = QPP_DECODE_ERROR;
            } else {
                const uint4 smp = ld16(pay + s);
                const uint32_t hdr_len = p.aad_len - p.pn_len;
                hp_finish<NR == 10 ? 10 : 14>(aes, key->hp_rk, smp, p.base, hdr_len, p.pn_len,
                                              masks + 5 * (size_t)pkt_index, flags);
            }
        }
        if (status) status[pkt_index] = st;
    } else {
        const uint4 want = ld16(pay + p.len);
        const uint4 diff = tag ^ want;
        const bool ok = (diff.x | diff.y | diff.z | diff.w) == 0;  // all 16 bytes compared, no early exit
        if (!ok) {
            // never release unauthenticated plaintext
            for (int b = 0; b < nfull; b++) st16(pay + 16 * b, make_uint4(0, 0, 0, 0));
            if (rem) st_bytes(pay + 16 * nfull, make_uint4(0, 0, 0, 0), rem);
        }
        status[pkt_index] = ok ? QPP_OK : QPP_DECRYPT_ERROR;
    }
}

template <bool SEAL, int NB, int WG, int NR>
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
    if (w.nr != NR) return;  // AES-128 and AES-256 work items are served by separate launches (SGPR budget)
    const DevKey *__restrict__ key = keys + w.key;
    build_tables(lds, key);
    const AesLds aes = make_aes(lds);
    const GhashLds gh{lds};
    for (uint32_t t = threadIdx.x; t < w.count; t += WG) {  // WG < 1024: several passes over the work item
        const uint32_t pi = perm[w.begin + t];
        const qpp_pkt d = descs[pi];
        process_packet<NR, NB, SEAL>(aes, gh, key, d, pi, arena, masks, status, flags);
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
};
constexpr Variant kVariants[] = {{4, 512, 1024}, {8, 512, 1024}, {2, 1024, 1024}, {4, 512, 512}, {2, 512, 1024}};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);

template <bool SEAL, int NR>
void launch_variant(int v, dim3 grid, hipStream_t s, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb,
                    uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags) {
#define QPP_AES_LAUNCH(NB, WG)                                                                                    \
    hipLaunchKernelGGL((aes_gcm_kernel<SEAL, NB, WG, NR>), grid, dim3(WG), kDynLds, s, keys, descs, pb.perm,     \
                       pb.work, pb.n_work, arena, masks, status, flags)
    switch (v) {
        case 0: QPP_AES_LAUNCH(4, 512); break;
        case 1: QPP_AES_LAUNCH(8, 512); break;
        case 2: QPP_AES_LAUNCH(2, 1024); break;
        case 3: QPP_AES_LAUNCH(4, 512); break;
        default: QPP_AES_LAUNCH(2, 512); break;
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
                          uint32_t suites, hipStream_t s) {
    if (!n) return hipSuccess;
    const dim3 grid(plan_max_work(n, key_cap, aes_packets_per_item()));
    const int v = aes_variant();
    if (suites & (1u << QPP_SUITE_TLS_AES_128_GCM_SHA256)) {
        if (seal) launch_variant<true, 10>(v, grid, s, keys, descs, pb, arena, masks, status, flags);
        else launch_variant<false, 10>(v, grid, s, keys, descs, pb, arena, masks, status, flags);
    }
    if (suites & (1u << QPP_SUITE_TLS_AES_256_GCM_SHA384)) {
        if (seal) launch_variant<true, 14>(v, grid, s, keys, descs, pb, arena, masks, status, flags);
        else launch_variant<false, 14>(v, grid, s, keys, descs, pb, arena, masks, status, flags);
    }
    return hipGetLastError();
}

}  // namespace qpp
