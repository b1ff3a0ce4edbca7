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
#include "device_common.h"

namespace qpp {
namespace {
using namespace dev;

// ---------------------------------------------------------------- GHASH: Y <- Y * H via 16 byte tables in LDS
struct GhashLds {
    const uint8_t *lds;
    template <int J>
    __device__ __forceinline__ uint4 tj(uint32_t w) const {
        constexpr int kShift = 8 * (J & 3);
        uint32_t off = ((w >> kShift) & 0xffu) << 4;
        return *(const uint4 *)(lds + kLdsGhash + J * 4096 + off);
    }
    __device__ __forceinline__ uint4 mul(uint4 y) const {
        uint4 a = tj<0>(y.x) ^ tj<1>(y.x) ^ tj<2>(y.x) ^ tj<3>(y.x);
        uint4 b = tj<4>(y.y) ^ tj<5>(y.y) ^ tj<6>(y.y) ^ tj<7>(y.y);
        uint4 c = tj<8>(y.z) ^ tj<9>(y.z) ^ tj<10>(y.z) ^ tj<11>(y.z);
        uint4 d = tj<12>(y.w) ^ tj<13>(y.w) ^ tj<14>(y.w) ^ tj<15>(y.w);
        return (a ^ b) ^ (c ^ d);
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

// GHASH over the AAD (zero-padded to 16 bytes).  Reads past the AAD stay inside payload||tag.
__device__ __forceinline__ uint4 ghash_aad(const GhashLds &gh, const uint8_t *aad, uint32_t aad_len) {
    uint4 y = make_uint4(0, 0, 0, 0);
    for (uint32_t off = 0; off < aad_len; off += 16) {
        uint4 a = ld16(aad + off);
        uint32_t r = aad_len - off;
        if (r < 16) a = keep_bytes(a, r);
        y = gh.mul(y ^ a);
    }
    return y;
}

// Header protection mask from the 16-byte sample (first 5 bytes of AES_hp(sample)).
template <int HNR>
__device__ __forceinline__ void hp_finish(const AesLds &aes, const uint32_t *__restrict__ hp_rk, uint4 sample,
                                          uint8_t *base, uint32_t hdr_len, uint32_t pn_len, uint8_t *mask_out,
                                          uint32_t flags) {
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

template <int NR, bool SEAL>
__device__ __forceinline__ void process_packet(const AesLds &aes, const GhashLds &gh, const DevKey *__restrict__ key,
                                               const qpp_pkt &d, uint32_t pkt_index, uint8_t *arena, uint8_t *masks,
                                               int8_t *status, uint32_t flags) {
    const uint32_t *__restrict__ rk = key->rk;
    PacketView p = load_packet(d, key, arena);
    uint8_t *pay = p.base + p.aad_len;
    // J0 = nonce || 1 ; E_K(J0) masks the tag
    const uint4 ek0 = aes.encrypt<NR>(make_uint4(p.n0, p.n1, p.n2, 0x01000000u), rk);
    uint4 y = ghash_aad(gh, p.base, p.aad_len);

    const uint32_t nfull = p.len >> 4, rem = p.len & 15;
    uint4 c0 = make_uint4(0, 0, 0, 0), c1 = c0;  // first two ciphertext blocks (HP sample)
    uint4 nxt = ld16(pay);                         // in bounds: payload||tag is >= 16 bytes
    uint32_t ctr = 2;
    for (uint32_t b = 0; b < nfull; b++) {
        uint4 in = nxt;
        nxt = ld16(pay + 16 * (b + 1));  // block b+1 (or the partial/tag area): still inside payload||tag
        uint4 ks = aes.encrypt<NR>(make_uint4(p.n0, p.n1, p.n2, bswap32(ctr++)), rk);
        uint4 out = in ^ ks;
        st16(pay + 16 * b, out);
        uint4 c = SEAL ? out : in;
        if (b == 0) c0 = c;
        if (b == 1) c1 = c;
        y = gh.mul(y ^ c);
    }
    if (rem) {
        uint4 in = nxt;
        uint4 ks = aes.encrypt<NR>(make_uint4(p.n0, p.n1, p.n2, bswap32(ctr)), rk);
        uint4 out = keep_bytes(in ^ ks, rem);
        st_bytes(pay + 16 * nfull, out, rem);
        uint4 c = SEAL ? out : keep_bytes(in, rem);
        if (nfull == 0) c0 = c;
        if (nfull == 1) c1 = c;
        y = gh.mul(y ^ c);
    }
    // length block: be64(aad bits) || be64(payload bits)
    y = gh.mul(y ^ make_uint4(0, bswap32(p.aad_len * 8), 0, bswap32(p.len * 8)));
    const uint4 tag = y ^ ek0;

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

template <bool SEAL>
__global__ __launch_bounds__(kPacketsPerGroup) void aes_gcm_kernel(const DevKey *__restrict__ keys,
                                                                  const qpp_pkt *__restrict__ descs,
                                                                  const uint32_t *__restrict__ perm,
                                                                  const WorkItem *__restrict__ work,
                                                                  const uint32_t *__restrict__ n_work,
                                                                  uint8_t *__restrict__ arena, uint8_t *masks,
                                                                  int8_t *status, uint32_t flags) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    if (blockIdx.x >= *n_work) return;  // uniform: grid is sized for the worst case
    const WorkItem w = work[blockIdx.x];
    const DevKey *__restrict__ key = keys + w.key;
    build_tables(lds, key);
    if (threadIdx.x >= w.count) return;
    const uint32_t pi = perm[w.begin + threadIdx.x];
    const qpp_pkt d = descs[pi];
    AesLds aes = make_aes(lds);
    GhashLds gh{lds};
    if (w.nr == 10)
        process_packet<10, SEAL>(aes, gh, key, d, pi, arena, masks, status, flags);
    else
        process_packet<14, SEAL>(aes, gh, key, d, pi, arena, masks, status, flags);
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

hipError_t launch_aes_gcm(bool seal, const DevKey *keys, const qpp_pkt *descs, const PlanBuffers &pb, uint32_t n,
                          uint32_t key_cap, uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags,
                          hipStream_t s) {
    if (!n) return hipSuccess;
    const uint32_t grid = plan_max_work(n, key_cap);
    if (seal)
        hipLaunchKernelGGL(aes_gcm_kernel<true>, dim3(grid), dim3(kPacketsPerGroup), kLdsBytes, s, keys, descs, pb.perm,
                           pb.work, pb.n_work, arena, masks, status, flags);
    else
        hipLaunchKernelGGL(aes_gcm_kernel<false>, dim3(grid), dim3(kPacketsPerGroup), kLdsBytes, s, keys, descs,
                           pb.perm, pb.work, pb.n_work, arena, masks, status, flags);
    return hipGetLastError();
}

}  // namespace qpp
