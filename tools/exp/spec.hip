// spec.hip — AES-128/256-GCM seal/open of large batches with SPECIALIZED waves (gfx950, round 5).
//
// Replaces the same aws-lc-rs calls as quad.hip, behind quic/s2n-quic-crypto:
//   seal  <LessSafeKey as Aead>::encrypt -> seal_in_place_scatter   src/aead/default.rs:44-62
//   open  <LessSafeKey as Aead>::decrypt -> open_in_place           src/aead/default.rs:65-93
//   HP    HeaderKey::header_protection_mask -> new_mask             src/header_key.rs:52-56
// with the nonce of Iv::nonce (src/iv.rs:27-39); a batch over several keys and both AES sizes is the per-key dispatch of
// src/cipher_suite/negotiated.rs:15-30.
//
// Why: the quad kernel runs the AES-CTR keystream, GHASH, the payload I/O and the per-packet glue in
// every wave.  That needs 168 VGPRs, so a CU holds 3 waves per SIMD, and its two binding pipes -- the LDS array (AES
// T-table and GHASH table reads) and VALU issue -- are each about two-thirds busy with 41 % of wave cycles parked.
// Here one 1024-thread workgroup per CU (4 waves per SIMD, <= 128 VGPRs) splits the work by role:
//   waves 0..11 ("A"): the CTR keystream in the quad layout of quad.hip (four lanes per packet, lane s takes counter
//                      slots t = 4 k + s; slot t = counter t + 1, ciphertext block t - 1) and the payload I/O; when
//                      sealing also E_K(J0) (slot 0) and the early header-protection mask (the sample is ciphertext
//                      blocks 0-1), both handed to the G waves in LDS;
//   waves 12..15 ("G"): GHASH with ONE lane per packet (48 packets per wave): Horner with H (8-bit tables of H) over
//                      the AAD, ciphertext and length blocks, then the tag, header protection and the status.
// A pass is 192 packets (16 per A wave).  Pass k runs L_k "steps" (groups of 16 counter slots: the longest packet's
// count); the workgroup walks the steps of all its passes in phases separated by s_barrier (no memory fence):
//   seal: A does step p, G step p - 2.  G reads ciphertext A stored two phases earlier: in the phase between, A either
//         consumed a load of its own (a load's data waits for every older memory operation of the wave, its stores
//         included) or drained vmcnt, so those stores are complete before the barrier;
//   open: G does step p, A step p - 1.  G has loaded and hashed a group's ciphertext before A overwrites it with
//         plaintext; G's verdict of a packet reaches A at that packet's last group, and A zeroes a rejected payload.
// The AES work per block is the quad kernel's (same tables, same CTR page caching, same pipeline); what changes is the
// register budget of each wave (4 instead of 3 waves per SIMD) and that the per-packet glue (AAD, length block, the
// H^e products of the four-lane GHASH, tag) leaves the AES waves.
//
// LDS (160 KiB, one workgroup per CU):
//   [0, 64K)      8-bit GHASH tables of H (GhashT layout, T_j[x] at 256 x + 16 j)
//   [64K, 128K)   AES tables (AesQ4: T0..T3, 8 copies each, in the lower 128 B of 256 rows)
//   [128K, ...)   V[m] = H x^m (table build) | E_K(J0) and HP mask slots (A -> G) | verdicts (G -> A) | pass lengths
#include "device_common.h"
#include "ghash.h"

namespace qpp {
namespace {
using namespace dev;

constexpr int kSpecWG = 1024;
constexpr uint32_t kSA = 12;                 // A waves
constexpr uint32_t kSPass = 16u * kSA;       // packets per pass (16 per A wave)
constexpr uint32_t kSGL = kSPass / 4u;       // packets per G wave (its lanes 0..47)
// Hand-off slots are indexed by pass modulo 3: pass k's slots are written at its first step and read at most two phases
// after its last step, and pass k + 3 starts no earlier than that (every pass has L >= 1)
constexpr uint32_t kSBufs = 3;
constexpr uint32_t kSLdsV = 131072;                                // V[m] = H x^m while the tables are built (2 KiB)
constexpr uint32_t kSLdsEk = kSLdsV + 2048;                        // [3][192] x 16 B: E_K(J0) of a sealed packet
constexpr uint32_t kSLdsMask = kSLdsEk + kSBufs * kSPass * 16u;    // [3][192] x 8 B: its HP mask words m0, m1
constexpr uint32_t kSLdsVerd = kSLdsMask + kSBufs * kSPass * 8u;   // [3][192] x 4 B: an opened packet's tag verdict
constexpr uint32_t kSLdsPass = kSLdsVerd + kSBufs * kSPass * 4u;   // steps (groups) of each pass of the chunk
constexpr uint32_t kSMaxPass = (kLdsMax - kSLdsPass) / 4u;         // passes per chunk (3648: 700 Ki packets)
static_assert(kSLdsPass < kLdsMax && kSMaxPass >= 1024, "spec LDS layout");

using QAes = AesQ4;
using QPage = CtrPageQ4;

#ifndef QPP_SPEC_TRACE
#define QPP_SPEC_TRACE 0  // 1: workgroup 0's waves print their work / barrier-wait cycles per chunk (s_memtime)
#endif
#ifndef QPP_SPEC_GPF
#define QPP_SPEC_GPF 0  // G waves: the next 4 ciphertext blocks loaded while 4 are hashed (A/B)
#endif
#ifndef QPP_SPEC_ROLES
#define QPP_SPEC_ROLES 3  // diagnostic builds: 1 = the A waves only, 2 = the G waves only (wrong results; timing)
#endif
struct SpecClock {
#if QPP_SPEC_TRACE
    uint64_t t, work = 0, wait = 0;
    __device__ __forceinline__ void start() { t = __builtin_amdgcn_s_memtime(); }
    __device__ __forceinline__ void worked() { const uint64_t n = __builtin_amdgcn_s_memtime(); work += n - t; t = n; }
    __device__ __forceinline__ void waited() { const uint64_t n = __builtin_amdgcn_s_memtime(); wait += n - t; t = n; }
    __device__ __forceinline__ void report(const char *role, uint32_t nph) const {
        if (blockIdx.x == 0 && (threadIdx.x & 63u) == 0)
            printf("spec %s wave %u: phases %u work %lu wait %lu cycles\n", role, threadIdx.x >> 6, nph,
                   (unsigned long)work, (unsigned long)wait);
    }
#else
    __device__ __forceinline__ void start() {}
    __device__ __forceinline__ void worked() {}
    __device__ __forceinline__ void waited() {}
    __device__ __forceinline__ void report(const char *, uint32_t) const {}
#endif
};

// the barrier between phases: no memory fence (the A waves' stores are ordered by their own later loads, see above);
// the wave's LDS operations are complete (the hand-off slots)
#ifndef QPP_SPEC_NOBAR
#define QPP_SPEC_NOBAR 0  // diagnostic builds (with QPP_SPEC_ROLES 1 or 2): the role runs without the phase barriers
#endif
__device__ __forceinline__ void spec_barrier() {
    if (QPP_SPEC_NOBAR) return;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint32_t lds_max32(uint32_t a, uint32_t v) {
    return __hip_atomic_fetch_max((lds_u32 *)(size_t)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}
// groups of 16 counter slots (slot 0 = J0 .. slot m, m payload blocks) of a payload of pt_len bytes
__device__ __forceinline__ uint32_t spec_groups(uint32_t pt_len) { return (((pt_len + 15u) >> 4) + 16u) >> 4; }

template <int CTRL>
__device__ __forceinline__ uint32_t sqperm(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ uint4 sqperm(uint4 v) {
    return make_uint4(sqperm<CTRL>(v.x), sqperm<CTRL>(v.y), sqperm<CTRL>(v.z), sqperm<CTRL>(v.w));
}
constexpr int kSQBcast1 = 0x55, kSQBcast2 = 0xaa, kSQRot1 = 0x39, kSQSwap2 = 0x4e, kSQRot3 = 0x93;

// AES of one block over the 4 lanes of a quad (column s in lane s; quad.hip aes_quad): the early HP mask
template <int NR>
__device__ __forceinline__ uint32_t spec_aes_quad(const QAes &a, const uint32_t *__restrict__ rk_g, uint32_t col,
                                                  uint32_t s) {
    uint32_t rk[NR + 1];
#pragma unroll
    for (int r = 0; r <= NR; r++) rk[r] = rk_g[4 * r + s];
    uint32_t x = a.rot(col ^ rk[0]);
#pragma unroll
    for (int r = 1; r <= NR; r++) {
        const uint32_t b = sqperm<kSQRot1>(x), c = sqperm<kSQSwap2>(x), d = sqperm<kSQRot3>(x);
        x = r < NR ? a.col(x, b, c, d, a.rot(rk[r])) : a.last(x, b, c, d, rk[r]);
    }
    return x;
}

// The key's tables: 8-bit GHASH tables of H at [0, 64K) and the AES tables.  Every thread takes part; the caller synced
// before (the previous key's tables are no longer read); ends with a barrier.
__device__ void spec_tables(const DevKey *__restrict__ key) {
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    if (tid < 128) {
        const uint32_t *v = key->V[tid];
        lds_st128(kSLdsV + 16 * tid, make_uint4(v[0], v[1], v[2], v[3]));
    }
    __syncthreads();
    for (uint32_t e = tid; e < 4096; e += nthr) {  // T_j[x] = xor of V[8 j + i] over the set bits (bit 7 - i) of x
        const uint32_t j = e & 15, x = e >> 4;
        uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 8; i++)
            if ((x >> (7 - i)) & 1) acc = acc ^ lds_ld128(kSLdsV + 16 * (8 * j + i));
        lds_st128(kLdsGhash + 256 * x + 16 * j, acc);
    }
    build_aes_tables_q4(kLdsAes);
    __syncthreads();
}

// The descriptor again (laundered index: its fields are not held in VGPRs across the phase loop)
__device__ __forceinline__ qpp_pkt spec_desc(const qpp_pkt *descs, uint32_t i) {
    uint32_t v = i;
    asm volatile("" : "+v"(v));
    return descs[v];
}

// ---------------------------------------------------------------- A waves: keystream + payload I/O (quad layout)
template <bool SEAL, int NR>
__device__ __forceinline__ void spec_a(const DevKey *__restrict__ key, const qpp_pkt *__restrict__ descs,
                                       const uint32_t *__restrict__ perm, bool one, uint32_t single, uint32_t c_lo,
                                       uint32_t c_hi, uint32_t npass, uint32_t S, uint8_t *__restrict__ arena,
                                       int8_t *status, uint32_t flags) {
    const QAes aes = QAes::make();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, s = lane & 3u;
    const uint32_t ql = 16u * wave + (lane >> 2);  // the quad's packet within the pass
    auto at = [&](uint32_t off) { return arena + off; };
    // Round keys through the constant address space, reloaded per group (quad.hip: held for the whole loop they
    // exhausted the SGPRs)
    auto round_keys = [&]() {
        uint64_t a = (uint64_t)key->rk;
        asm volatile("" : "+s"(a));
        return (RkPtr)a;
    };
    const bool want_hp = SEAL && (flags & (QPP_HP_MASK_OUT | QPP_HP_APPLY)) != 0;
    // the pass's packet of this quad, and the wave's group bounds
    uint32_t pi = 0, pay = 0, len = 0, n0 = 0, n1 = 0, n2 = 0;
    int nfull = 0, rem = 0, ng = 0, Gw = 0, min_full = 0, tail_slots = 0;
    bool has = false;
    QPage pg;
    uint32_t k = 0, g = 0, L = npass ? lds_ld32(kSLdsPass) : 0u;
    const uint32_t nph = SEAL ? S + 2u : S + 1u;
    SpecClock clk;
    clk.start();

    auto interior = [&](int gg) { return gg >= 1 && 16 * gg + 15 <= min_full; };  // every slot a whole payload block
    // one group: slots t = 16 g + 4 j + s, j < NBG
    auto group = [&](auto nbc, int gi, uint32_t buf) __attribute__((always_inline)) {
        constexpr int NBG = decltype(nbc)::value;
        const bool inner = NBG == 4 && interior(gi);  // uniform
        const RkPtr rkp = round_keys();
        const int t0 = 16 * gi + (int)s;
        uint4 ks[NBG];
        const uint32_t c0 = (uint32_t)t0 + 1u;
        uint32_t m0 = n0, m1 = n1, m2 = n2;
        if ((gi & 15) != 15) {  // uniform: no lane's counters straddle a 256-block page
            if ((c0 >> 8) != pg.page) {
                asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2));
                pg.build(aes, rkp, m0, m1, m2, c0 >> 8);
            }
            uint32_t rk[4 * (NR + 1)];
#pragma unroll
            for (int r = 3; r <= NR; r++) {
                const uint4 v = rkp[r];
                rk[4 * r] = v.x; rk[4 * r + 1] = v.y; rk[4 * r + 2] = v.z; rk[4 * r + 3] = v.w;
            }
            ctr_keystream_q4<NR, NBG, 4>(aes, pg, rk, c0, ks);
        } else {
            asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2));
            uint32_t rk[4 * (NR + 1)];
#pragma unroll
            for (int r = 0; r <= NR; r++) {
                const uint4 v = rkp[r];
                rk[4 * r] = v.x; rk[4 * r + 1] = v.y; rk[4 * r + 2] = v.z; rk[4 * r + 3] = v.w;
            }
            static_for<NBG>([&](auto kc) {
                constexpr int j = decltype(kc)::value;
                ks[j] = aes.encrypt<NR>(make_uint4(m0, m1, m2, bswap32(c0 + 4 * j)), rk);
            });
        }
        uint4 in[NBG];
        if (inner) {
            const uint32_t b = pay + 16 * (uint32_t)(t0 - 1);
#pragma unroll
            for (int j = 0; j < NBG; j++) in[j] = ld16(at(b + 64 * j));
        } else {
#pragma unroll
            for (int j = 0; j < NBG; j++) {
                const int bj = t0 + 4 * j - 1;
                in[j] = ld16(at(pay + (bj >= 0 && 16 * bj <= (int)len ? 16 * (uint32_t)bj : 0u)));
            }
        }
        uint4 out[NBG];
#pragma unroll
        for (int j = 0; j < NBG; j++) out[j] = in[j] ^ ks[j];
        if (inner) {
            const uint32_t b = pay + 16 * (uint32_t)(t0 - 1);
#pragma unroll
            for (int j = 0; j < NBG; j++) st16(at(b + 64 * j), out[j]);
        } else {
            uint32_t rl = (uint32_t)rem;
            asm volatile("" : "+v"(rl));
#pragma unroll
            for (int j = 0; j < NBG; j++) {
                const int t = t0 + 4 * j, bj = t - 1;
                if (t >= 1 && bj < nfull) st16(at(pay + 16 * (uint32_t)bj), out[j]);
                if (rem && bj == nfull) st_bytes(at(pay + 16 * (uint32_t)bj), keep_bytes(out[j], rl), rl);
            }
        }
        if constexpr (SEAL) {
            if (gi == 0) {
                // E_K(J0) (slot 0: lane 0 of the quad, block 0) for the G wave's tag
                const uint32_t slot = buf * kSPass + ql;
                if (has && s == 0) lds_st128(kSLdsEk + 16 * slot, ks[0]);
                // the header-protection mask as soon as its sample exists: ciphertext bytes [4 - pn_len, 20 - pn_len)
                // (payload.rs:151-169) lie in ciphertext blocks 0 and 1 = slots 1, 2 of group 0 (lanes 1, 2) when the
                // payload has at least 20 - pn_len bytes; the mask goes to the G wave, which applies it after hashing
                // the header (the header is AAD)
                const uint32_t pn_len = spec_desc(descs, pi).pn_len;
                if (want_hp && has && pn_len >= 1 && pn_len <= 4 && len + pn_len >= 20) {  // quad-uniform
                    const uint4 b0 = sqperm<kSQBcast1>(out[0]), b1 = sqperm<kSQBcast2>(out[0]);
                    const uint32_t lo = s == 0 ? b0.x : s == 1 ? b0.y : s == 2 ? b0.z : b0.w;
                    const uint32_t hi = s == 0 ? b0.y : s == 1 ? b0.z : s == 2 ? b0.w : b1.x;
                    const uint32_t col = __builtin_amdgcn_alignbyte(hi, lo, 4 - pn_len);
                    const uint32_t hm0 = spec_aes_quad<NR>(aes, key->hp_rk, col, s);
                    const uint32_t hm1 = sqperm<kSQBcast1>(hm0);  // column 1 (mask byte 4 is its byte 0)
                    if (s == 0) lds_st64(kSLdsMask + 8 * slot, make_uint2(hm0, hm1));
                }
            }
        } else {
            // the packet's last group: the G wave's verdict (written one phase earlier); a rejected packet's plaintext
            // is never released (all of it zeroed; the quad's other lanes stored theirs: a wavefront fence first)
            if (has && gi == ng - 1) {  // quad-uniform
                const uint32_t ok = lds_ld32(kSLdsVerd + 4 * (buf * kSPass + ql));
                if (!ok && s == 0) {
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    for (int bj = 0; bj < nfull; bj++) st16(at(pay + 16 * (uint32_t)bj), make_uint4(0, 0, 0, 0));
                    if (rem) st_bytes(at(pay + 16 * (uint32_t)nfull), make_uint4(0, 0, 0, 0), (uint32_t)rem);
                }
            }
        }
    };

    for (uint32_t p = 0; p < nph; p++) {
        const bool act = SEAL ? p < S : p >= 1u;
        bool loaded = false;
        if (act) {
            const uint32_t buf = k % kSBufs;
            if (g == 0) {  // a new pass: this quad's packet
                const uint32_t t = c_lo + kSPass * k + ql;
                const bool real = t < c_hi;
                pi = one ? (real ? t : c_lo) : perm[real ? t : c_lo];
                const qpp_pkt d = descs[pi];
                has = real && !(d.flags & QPP_PKT_SKIP);
                if (one && has && d.key_idx != single) {  // not the live key: refused, untouched
                    if (status && s == 0) status[pi] = QPP_INTERNAL_ERROR;
                    has = false;
                }
                len = has ? d.pt_len : 0u;
                pay = d.off + d.aad_len;
                n0 = key->iv[0];
                n1 = key->iv[1] ^ bswap32((uint32_t)(d.pn >> 32));  // Iv::nonce (iv.rs:27-39)
                n2 = key->iv[2] ^ bswap32((uint32_t)d.pn);
                nfull = (int)(len >> 4);
                rem = (int)(len & 15);
                const int m = nfull + (rem ? 1 : 0);
                ng = has ? (m + 16) >> 4 : 0;
                Gw = (int)__builtin_amdgcn_readfirstlane(wave_max((uint32_t)ng));
                min_full = (int)__builtin_amdgcn_readfirstlane(wave_min(has ? (uint32_t)nfull : 0u));
                tail_slots = (int)__builtin_amdgcn_readfirstlane(
                    wave_max(has ? (uint32_t)max(0, m + 1 - 16 * (Gw - 1)) : 0u));
                uint64_t rka = (uint64_t)key->rk;
                asm volatile("" : "+s"(rka));
                pg.build(aes, (RkPtr)rka, n0, n1, n2, 0);
            }
            const int gi = (int)g;
            if (gi < Gw) {
                if (gi + 1 < Gw) group(std::integral_constant<int, 4>{}, gi, buf);
                else if (tail_slots <= 4) group(std::integral_constant<int, 1>{}, gi, buf);
                else if (tail_slots <= 8) group(std::integral_constant<int, 2>{}, gi, buf);
                else if (tail_slots <= 12) group(std::integral_constant<int, 3>{}, gi, buf);
                else group(std::integral_constant<int, 4>{}, gi, buf);
                loaded = true;
            }
            if (++g == L) {
                g = 0;
                ++k;
                L = k < npass ? lds_ld32(kSLdsPass + 4 * k) : 0u;
            }
        }
        if (!loaded) drain_vm();  // no load of this phase orders the previous phase's stores: drain them
        clk.worked();
        spec_barrier();
        clk.waited();
    }
    clk.report("A", nph);
}

// ---------------------------------------------------------------- G waves: GHASH (lane per packet), tag, HP, status
template <bool SEAL, int NR>
__device__ __forceinline__ void spec_g(const DevKey *__restrict__ key, const qpp_pkt *__restrict__ descs,
                                       const uint32_t *__restrict__ perm, bool one, uint32_t single, uint32_t c_lo,
                                       uint32_t c_hi, uint32_t npass, uint32_t S, uint8_t *__restrict__ arena,
                                       uint8_t *masks, int8_t *status, uint32_t flags) {
    const QAes aes = QAes::make();  // a lane's own AES block: open's E_K(J0), a short payload's HP mask
    const GhashT<true> gh = GhashT<true>::make();
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t gl = kSGL * (wave - kSA) + lane;  // the lane's packet within the pass
    const bool mine = lane < kSGL;
    auto at = [&](uint32_t off) { return arena + off; };
    const bool want_hp = SEAL && (flags & (QPP_HP_MASK_OUT | QPP_HP_APPLY)) != 0;
    uint32_t pi = 0, off = 0, aad_len = 0, len = 0;
    int m = 0, ng = 0;
    bool has = false;
    uint4 w = make_uint4(0, 0, 0, 0);  // Horner state, lane-rotated (GhashT: W = rot(Z))
    uint32_t k = 0, g = 0, L = npass ? lds_ld32(kSLdsPass) : 0u;
    const uint32_t nph = SEAL ? S + 2u : S + 1u;
    SpecClock clk;
    clk.start();
    for (uint32_t p = 0; p < nph; p++) {
        const bool act = SEAL ? p >= 2u : p < S;
        if (act) {
            const uint32_t buf = k % kSBufs, slot = buf * kSPass + gl;
            if (g == 0) {  // a new pass: this lane's packet, its AAD blocks
                const uint32_t t = c_lo + kSPass * k + gl;
                const bool real = mine && t < c_hi;
                pi = one ? (real ? t : c_lo) : perm[real ? t : c_lo];
                const qpp_pkt d = descs[pi];
                has = real && !(d.flags & QPP_PKT_SKIP) && (!one || d.key_idx == single);
                off = d.off;
                aad_len = d.aad_len;
                len = has ? d.pt_len : 0u;
                m = (int)((len + 15u) >> 4);
                ng = has ? (m + 16) >> 4 : 0;
                w = make_uint4(0, 0, 0, 0);
                if (has) {
                    const uint32_t a = (aad_len + 15u) >> 4;
                    for (uint32_t i = 0; i < a; i++) {
                        uint4 x = ld16(at(off + 16 * i));
                        const uint32_t r = aad_len - 16 * i;
                        w = gh.mulx(w, r < 16 ? keep_bytes(x, r) : x);  // (from w = 0: the first block is X_1)
                    }
                }
            }
            if (has && (int)g < ng) {
                const uint32_t pay = off + aad_len;
                const int gi = (int)g, jb = gi == 0 ? 0 : 16 * gi - 1, je = min(m, 16 * gi + 15);
                const uint32_t rl = len & 15u;
                // ciphertext blocks [jb, je) in batches of 4 (a next batch in flight while one is hashed spilled
                // VGPRs)
                auto ldb = [&](int j) { return ld16(at(pay + 16u * (uint32_t)(j < je ? j : jb))); };
#if QPP_SPEC_GPF
                uint4 c[4], nx[4];
#pragma unroll
                for (int i = 0; i < 4; i++) c[i] = ldb(jb + i);
                for (int j = jb; j < je; j += 4) {
#pragma unroll
                    for (int i = 0; i < 4; i++) nx[i] = ldb(j + 4 + i);
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int bj = j + i;
                        if (bj < je) w = gh.mulx(w, (rl && bj == m - 1) ? keep_bytes(c[i], rl) : c[i]);
                    }
#pragma unroll
                    for (int i = 0; i < 4; i++) c[i] = nx[i];
                }
#else
                for (int j = jb; j < je; j += 4) {
                    uint4 c[4];
#pragma unroll
                    for (int i = 0; i < 4; i++) c[i] = ldb(j + i);
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int bj = j + i;
                        if (bj < je) w = gh.mulx(w, (rl && bj == m - 1) ? keep_bytes(c[i], rl) : c[i]);
                    }
                }
#endif
                if (gi == ng - 1) {  // the packet's last group: length block, Y, tag
                    w = gh.mulx(w, make_uint4(0, bswap32(aad_len * 8), 0, bswap32(len * 8)));
                    const uint4 y = gh.prod(w, make_uint4(0, 0, 0, 0));  // Y = Z * H, natural order
                    const qpp_pkt dt = spec_desc(descs, pi);
                    if constexpr (SEAL) {
                        const uint4 tag = y ^ lds_ld128(kSLdsEk + 16 * slot);  // tag = GHASH ^ E_K(J0)
                        st16(at(pay + len), tag);
                        const uint32_t pn_len = dt.pn_len;
                        const bool hp = want_hp && pn_len >= 1 && pn_len <= 4 && len >= 4 - pn_len;
                        if (hp) {
                            uint32_t hm0, hm1;
                            if (len + pn_len >= 20) {  // the A wave's mask
                                const uint2 mm = lds_ld64(kSLdsMask + 8 * slot);
                                hm0 = mm.x;
                                hm1 = mm.y;
                            } else {  // short payload: the sample runs into the tag (stored above by this lane)
                                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                                uint4 smp;
                                __builtin_memcpy(&smp, at(pay + 4 - pn_len), 16);
                                const uint4 mm = aes.encrypt<NR>(smp, key->hp_rk);
                                hm0 = mm.x;
                                hm1 = mm.y;
                            }
                            if (flags & QPP_HP_MASK_OUT) {
                                uint8_t *mo = masks + 5 * (size_t)pi;
                                mo[0] = (uint8_t)hm0; mo[1] = (uint8_t)(hm0 >> 8); mo[2] = (uint8_t)(hm0 >> 16);
                                mo[3] = (uint8_t)(hm0 >> 24); mo[4] = (uint8_t)hm1;
                            }
                            const uint32_t hdr_len = aad_len - pn_len;
                            if (flags & QPP_HP_APPLY) hdr_apply(at(off), hdr_len, pn_len, hdr_load(at(off), hdr_len), hm0, hm1);
                        }
                        if (status) status[pi] = want_hp && !hp ? QPP_DECODE_ERROR : QPP_OK;
                    } else {
                        // E_K(J0) by this lane (J0 = nonce || be32(1)); all 16 tag bytes compared, no early exit
                        const uint4 j0 = make_uint4(key->iv[0], key->iv[1] ^ bswap32((uint32_t)(dt.pn >> 32)),
                                                    key->iv[2] ^ bswap32((uint32_t)dt.pn), bswap32(1u));
                        const uint4 ek0 = aes.encrypt<NR>(j0, key->rk);
                        const uint4 diff = y ^ ek0 ^ ld16(at(pay + len));
                        const bool ok = (diff.x | diff.y | diff.z | diff.w) == 0;
                        status[pi] = ok ? QPP_OK : QPP_DECRYPT_ERROR;
                        lds_st32(kSLdsVerd + 4 * slot, ok ? 1u : 0u);  // A zeroes a rejected payload
                    }
                }
            }
            if (++g == L) {
                g = 0;
                ++k;
                L = k < npass ? lds_ld32(kSLdsPass + 4 * k) : 0u;
            }
        }
        clk.worked();
        spec_barrier();
        clk.waited();
    }
    clk.report("G", nph);
}

// One workgroup per CU over an equal slice of the key-sorted packets (plan meta; or the single-key mode), key segment by
// key segment (tables per key), each segment in chunks of <= kSMaxPass passes.
template <bool SEAL, int NR>
__device__ __forceinline__ void spec_slices(const DevKey *__restrict__ keys, const qpp_pkt *__restrict__ descs,
                                            const uint32_t *__restrict__ perm, const WorkItem *__restrict__ work,
                                            const uint32_t *__restrict__ meta, uint8_t *__restrict__ arena,
                                            uint8_t *masks, int8_t *status, uint32_t flags, uint32_t single,
                                            uint32_t n_single) {
    const bool one = single != 0xffffffffu;  // uniform
    uint32_t i_lo = 0, i_hi = 1, p0 = 0, n = n_single;
    if (!one) {
        const uint32_t items = meta[0], i10 = meta[1], n10 = meta[2], n14 = meta[3];
        i_lo = NR == 10 ? 0 : i10;
        i_hi = NR == 10 ? i10 : items;
        p0 = NR == 10 ? 0 : n10;
        n = NR == 10 ? n10 : n14;
    }
    const uint32_t P = ((n + gridDim.x - 1) / gridDim.x + 15u) & ~15u;  // whole A waves (16 packets) per slice
    uint32_t lo = p0 + min(n, blockIdx.x * P);
    const uint32_t hi = p0 + min(n, (blockIdx.x + 1) * P);
    if (lo >= hi) return;  // uniform
    uint32_t i = i_lo, j = i_hi;  // the item holding lo: largest i with work[i].begin <= lo
    while (!one && j - i > 1) {
        const uint32_t mid = (i + j) >> 1;
        if (work[mid].begin <= lo) i = mid; else j = mid;
    }
    const uint32_t tid = threadIdx.x, nt = blockDim.x, wave = tid >> 6, lane = tid & 63u;
    for (; lo < hi; i++) {  // key segments of the slice
        WorkItem wi = one ? WorkItem{single, 0u, n, (uint32_t)NR} : work[i];
        wi.key = __builtin_amdgcn_readfirstlane(wi.key);
        wi.begin = __builtin_amdgcn_readfirstlane(wi.begin);
        wi.count = __builtin_amdgcn_readfirstlane(wi.count);
        const uint32_t end = min(hi, wi.begin + wi.count);
        const DevKey *__restrict__ key = keys + wi.key;
        __syncthreads();  // every wave is done with the previous segment's tables
        spec_tables(key);
        for (uint32_t c_lo = lo; c_lo < end; c_lo += kSMaxPass * kSPass) {
            const uint32_t c_hi = min(end, c_lo + kSMaxPass * kSPass);
            const uint32_t npass = (c_hi - c_lo + kSPass - 1) / kSPass;
            // each pass's steps: the groups of its longest packet (>= 1)
            for (uint32_t q = tid; q < npass; q += nt) lds_st32(kSLdsPass + 4 * q, 1u);
            __syncthreads();
            for (uint32_t t = c_lo + tid; t < c_hi; t += nt) {
                const uint32_t pi = one ? t : perm[t];
                const qpp_pkt d = descs[pi];
                if (!(d.flags & QPP_PKT_SKIP) && (!one || d.key_idx == single)) {
                    const uint32_t ngr = spec_groups(d.pt_len);
                    if (ngr > 1) lds_max32(kSLdsPass + 4 * ((t - c_lo) / kSPass), ngr);
                }
            }
            __syncthreads();
            uint32_t S = 0;
            for (uint32_t q = lane; q < npass; q += 64) S += lds_ld32(kSLdsPass + 4 * q);
            S = __builtin_amdgcn_readfirstlane(wave_sum(S));
            if (wave < kSA) {
                if (QPP_SPEC_ROLES & 1) spec_a<SEAL, NR>(key, descs, perm, one, single, c_lo, c_hi, npass, S, arena, status, flags);
                else for (uint32_t p = 0; p < (SEAL ? S + 2u : S + 1u); p++) spec_barrier();
            } else {
                if (QPP_SPEC_ROLES & 2) spec_g<SEAL, NR>(key, descs, perm, one, single, c_lo, c_hi, npass, S, arena, masks, status, flags);
                else for (uint32_t p = 0; p < (SEAL ? S + 2u : S + 1u); p++) spec_barrier();
            }
            __syncthreads();  // (both roles ran S + 2 / S + 1 barriers)
        }
        lo = end;
    }
}

// AES: 10 or 14 (one size), 0 both sizes in one launch (the AES-128 slice, then the AES-256 slice: a planned batch)
template <bool SEAL, int AES>
__global__ __launch_bounds__(kSpecWG) void aes_gcm_spec_kernel(const DevKey *__restrict__ keys,
                                                              const qpp_pkt *__restrict__ descs,
                                                              const uint32_t *__restrict__ perm,
                                                              const WorkItem *__restrict__ work,
                                                              const uint32_t *__restrict__ meta,
                                                              uint8_t *__restrict__ arena, uint8_t *masks,
                                                              int8_t *status, uint32_t flags, uint32_t single,
                                                              uint32_t n_single) {
    if constexpr (AES != 14) spec_slices<SEAL, 10>(keys, descs, perm, work, meta, arena, masks, status, flags, single, n_single);
    if constexpr (AES == 0) __syncthreads();
    if constexpr (AES != 10) spec_slices<SEAL, 14>(keys, descs, perm, work, meta, arena, masks, status, flags, single, n_single);
}
}  // namespace

// aes: 10, 14, or 0 (a planned batch with both sizes, one launch)
hipError_t launch_aes_gcm_spec(bool seal, uint32_t aes, dim3 grid, hipStream_t s, const DevKey *keys,
                               const qpp_pkt *descs, const PlanBuffers &pb, uint8_t *arena, uint8_t *masks,
                               int8_t *status, uint32_t flags, uint32_t single, uint32_t n_single) {
#define QPP_SPEC_LAUNCH(S, A)                                                                                       \
    hipLaunchKernelGGL((aes_gcm_spec_kernel<S, A>), grid, dim3(kSpecWG), kLdsMax, s, keys, descs, pb.perm, pb.work, \
                       pb.n_work, arena, masks, status, flags, single, n_single)
    if (aes == 10) {
        if (seal) QPP_SPEC_LAUNCH(true, 10);
        else QPP_SPEC_LAUNCH(false, 10);
    } else if (aes == 14) {
        if (seal) QPP_SPEC_LAUNCH(true, 14);
        else QPP_SPEC_LAUNCH(false, 14);
    } else {
        if (seal) QPP_SPEC_LAUNCH(true, 0);
        else QPP_SPEC_LAUNCH(false, 0);
    }
#undef QPP_SPEC_LAUNCH
    return hipGetLastError();
}

}  // namespace qpp
