// fips.hip — the sealing nonce-order gate of FIPS mode (gfx950).
//
// s2n-quic-crypto's `fips` cargo feature (cipher_suite/ring.rs:13-31) backs every AES packet key with
// aws_lc_rs::aead::TlsRecordSealingKey (aead/fips.rs:13-31, 38-60): aws-lc's TLS 1.3 AES-GCM AEAD
// (EVP_aead_aes_{128,256}_gcm_tls13, aws-lc-rs 1.12 / aws-lc crypto/fipsmodule/cipher/e_aes.c, not vendored in the
// reference) refuses a seal whose nonce does not come strictly after the previous one:
//   given = big-endian u64 of nonce[4..12];  on the key's first seal: mask = given  (its sequence number is taken as 0)
//   given ^= mask;  refuse if given == UINT64_MAX or given < min_next;  else min_next = given + 1
// and the encrypt call fails (s2n-quic maps it to INTERNAL_ERROR) without touching the buffer.  With the QUIC nonce
// iv ^ (0^32 || pn) (iv.rs:27-39) the iv cancels: given = pn ^ pn_first.  ChaCha20-Poly1305 keys have no FIPS form
// (ring.rs:116-121).  Opening is not gated (TlsRecordOpeningKey).
//
// A batch seals its packets "in batch order" (qpp.h): packet j of key k is refused iff given_j < min_next(k) at batch
// start, given_j == UINT64_MAX, or given_j <= max{given_l : l < j, key_l = k} (a refused packet never raises min_next:
// it is below it, so the sequential rule reduces to this prefix maximum).  On the device:
//   1. fips_prepare: descs -> descs_out (the copy the seal kernels read); sort key (slot << ib) | j per gated packet,
//      (sentinel << ib) | j for the rest
//   2. radix sort (rocPRIM): gated packets grouped by key, batch order within a key
//   3. fips_heads: a key's first gated packet fixes its mask if it has never sealed
//   4. fips_values: v = given + 1 (0 for given == UINT64_MAX) and the key of every sorted position
//   5. inclusive max-scan of v by key (rocPRIM)
//   6. fips_apply: refused packets get QPP_PKT_SKIP in descs_out and QPP_INTERNAL_ERROR in status
//   7. fips_tails: min_next = max(min_next, the key's largest v)
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan_by_key.hpp>

#include "qpp_internal.h"

namespace qpp {
namespace {

__device__ __forceinline__ bool gated(const DevKey *keys, uint32_t key_cap, const qpp_pkt &d) {
    return !(d.flags & QPP_PKT_SKIP) && d.key_idx < key_cap && keys[d.key_idx].live == 1 && keys[d.key_idx].fips;
}

__global__ void fips_prepare(const DevKey *__restrict__ keys, uint32_t key_cap, const qpp_pkt *__restrict__ descs,
                             uint32_t n, qpp_pkt *__restrict__ descs_out, uint64_t *__restrict__ sk, uint32_t ib,
                             uint64_t sentinel) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const qpp_pkt d = descs[j];
    descs_out[j] = d;
    sk[j] = ((gated(keys, key_cap, d) ? (uint64_t)d.key_idx : sentinel) << ib) | j;
}

__global__ void fips_heads(DevKey *__restrict__ keys, const qpp_pkt *__restrict__ descs,
                           const uint64_t *__restrict__ sorted, uint32_t n, uint32_t ib, uint64_t sentinel) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t k = sorted[p] >> ib;
    if (k == sentinel || (p && (sorted[p - 1] >> ib) == k)) return;
    DevKey &key = keys[k];
    if (!key.fips_seen) {  // the key's first seal ever: its sequence number is taken as 0
        key.fips_mask = descs[sorted[p] & ((1ull << ib) - 1)].pn;
        key.fips_seen = 1;
    }
}

__global__ void fips_values(const DevKey *__restrict__ keys, const qpp_pkt *__restrict__ descs,
                            const uint64_t *__restrict__ sorted, uint32_t n, uint32_t ib, uint64_t sentinel,
                            uint32_t *__restrict__ seg, uint64_t *__restrict__ v) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t k = sorted[p] >> ib;
    seg[p] = (uint32_t)k;  // the sentinel (key_cap) is no key slot: the ungated packets form one segment of their own
    if (k == sentinel) {
        v[p] = 0;
        return;
    }
    const uint64_t given = descs[sorted[p] & ((1ull << ib) - 1)].pn ^ keys[k].fips_mask;
    v[p] = given == ~0ull ? 0 : given + 1;
}

__global__ void fips_apply(const DevKey *__restrict__ keys, const uint64_t *__restrict__ sorted, uint32_t n,
                           uint32_t ib, uint64_t sentinel, const uint64_t *__restrict__ v,
                           const uint64_t *__restrict__ incl, qpp_pkt *__restrict__ descs_out, int8_t *status,
                           uint32_t *refused) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t k = sorted[p] >> ib;
    if (k == sentinel) return;
    const bool head = !p || (sorted[p - 1] >> ib) != k;
    const uint64_t prev = head ? 0 : incl[p - 1];  // largest given + 1 of the key's earlier packets (0: none)
    const uint64_t x = v[p];                       // given + 1, 0 when given == UINT64_MAX
    const bool ok = x != 0 && x - 1 >= keys[k].fips_min_next && x > prev;
    if (ok) return;
    const uint32_t j = (uint32_t)(sorted[p] & ((1ull << ib) - 1));
    descs_out[j].flags |= QPP_PKT_SKIP;  // the seal kernels leave it (and its status) untouched
    if (status) status[j] = QPP_INTERNAL_ERROR;
    if (refused) atomicAdd(refused, 1u);
}

__global__ void fips_tails(DevKey *__restrict__ keys, const uint64_t *__restrict__ sorted, uint32_t n, uint32_t ib,
                           uint64_t sentinel, const uint64_t *__restrict__ incl) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t k = sorted[p] >> ib;
    if (k == sentinel || (p + 1 < n && (sorted[p + 1] >> ib) == k)) return;
    DevKey &key = keys[k];
    if (incl[p] > key.fips_min_next) key.fips_min_next = incl[p];  // refused packets are never above it
}

uint32_t bits_for(uint64_t x) {  // bits to hold 0..x
    uint32_t b = 1;
    while (b < 64 && (x >> b)) b++;
    return b;
}

struct MaxOp {
    __host__ __device__ uint64_t operator()(uint64_t a, uint64_t b) const { return a > b ? a : b; }
};
struct SameKey {
    __host__ __device__ bool operator()(uint32_t a, uint32_t b) const { return a == b; }
};

}  // namespace

size_t fips_scratch_bytes(uint32_t n) {
    // sk | sorted | v | incl (8 B each) | seg (4 B) | descs_out (24 B), each rounded to 256 B, + rocPRIM temp
    const size_t a = ((size_t)n * 8 + 255) & ~(size_t)255, s = ((size_t)n * 4 + 255) & ~(size_t)255,
                 d = ((size_t)n * sizeof(qpp_pkt) + 255) & ~(size_t)255;
    size_t t1 = 0, t2 = 0;
    rocprim::radix_sort_keys(nullptr, t1, (uint64_t *)nullptr, (uint64_t *)nullptr, n, 0, 64);
    rocprim::inclusive_scan_by_key(nullptr, t2, (uint32_t *)nullptr, (uint64_t *)nullptr, (uint64_t *)nullptr, (size_t)n,
                                   MaxOp(), SameKey());
    return 4 * a + s + d + ((std::max(t1, t2) + 255) & ~(size_t)255) + 256;
}

hipError_t launch_fips_gate(DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n, void *scratch,
                            size_t scratch_bytes, qpp_pkt **descs_out, int8_t *status, uint32_t *refused,
                            hipStream_t s) {
    if (!n) return hipSuccess;
    if (key_cap >= 0xffffffffu) return hipErrorInvalidValue;
    uint8_t *b = (uint8_t *)scratch;
    const size_t a = ((size_t)n * 8 + 255) & ~(size_t)255, sg = ((size_t)n * 4 + 255) & ~(size_t)255,
                 d = ((size_t)n * sizeof(qpp_pkt) + 255) & ~(size_t)255;
    uint64_t *sk = (uint64_t *)b, *sorted = (uint64_t *)(b + a), *v = (uint64_t *)(b + 2 * a),
             *incl = (uint64_t *)(b + 3 * a);
    uint32_t *seg = (uint32_t *)(b + 4 * a);
    qpp_pkt *out = (qpp_pkt *)(b + 4 * a + sg);
    uint8_t *temp = b + 4 * a + sg + d;
    if (4 * a + sg + d > scratch_bytes) return hipErrorInvalidValue;
    size_t temp_bytes = scratch_bytes - (4 * a + sg + d);
    const uint32_t ib = bits_for(n - 1), kb = bits_for(key_cap);  // key_cap itself is the sentinel
    if (ib + kb > 64) return hipErrorInvalidValue;
    const uint64_t sentinel = key_cap;
    const dim3 grid((n + 255) / 256), block(256);
    hipLaunchKernelGGL(fips_prepare, grid, block, 0, s, keys, key_cap, descs, n, out, sk, ib, sentinel);
    hipError_t e = rocprim::radix_sort_keys(temp, temp_bytes, sk, sorted, n, 0, ib + kb, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fips_heads, grid, block, 0, s, keys, out, sorted, n, ib, sentinel);
    hipLaunchKernelGGL(fips_values, grid, block, 0, s, keys, out, sorted, n, ib, sentinel, seg, v);
    temp_bytes = scratch_bytes - (4 * a + sg + d);
    e = rocprim::inclusive_scan_by_key(temp, temp_bytes, seg, v, incl, (size_t)n, MaxOp(), SameKey(), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(fips_apply, grid, block, 0, s, keys, sorted, n, ib, sentinel, v, incl, out, status, refused);
    hipLaunchKernelGGL(fips_tails, grid, block, 0, s, keys, sorted, n, ib, sentinel, incl);
    *descs_out = out;
    return hipGetLastError();
}

}  // namespace qpp
