// plan.hip — groups the AES packets of a batch by key so that every AES-GCM workgroup serves ONE key
// (its GHASH tables are per key and live in LDS).  Three small launches, all device-side, so a batch
// whose descriptors are already in HBM never round-trips to the host:
//   1. plan_hist   : packets per key (LDS-privatised counts, one global add per touched key per block)
//   2. plan_scan   : one workgroup: key offsets, work list {key, begin, count<=per, rounds}, n_work
//   3. plan_scatter: perm[] = packet indices grouped by key (LDS ranks + one global reservation per key)
// ChaCha20-Poly1305 packets are skipped (their kernel needs no grouping).
// The reference has no batching at all (Key::encrypt is per packet); this is the
// batch former the MI355X design adds in front of the kernels.
#include "device_common.h"

namespace qpp {
namespace {

constexpr int kPlanBlock = 1024;
constexpr uint32_t kPlanPerThread = 4;  // packets per thread in plan_hist / plan_scatter (amortises the per-block bins)

__device__ __forceinline__ bool is_aes(const DevKey *keys, uint32_t k) {
    return keys[k].suite != QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256;
}

// key_cap <= kMaxPlanKeys: bins in LDS.  Larger key tables use global atomics directly.
__global__ __launch_bounds__(kPlanBlock) void plan_hist(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                       const qpp_pkt *__restrict__ descs, uint32_t n,
                                                       uint32_t *__restrict__ counts) {
    __shared__ uint32_t bins[kMaxPlanKeys];
    const bool local = key_cap <= (uint32_t)kMaxPlanKeys;
    if (local)
        for (uint32_t i = threadIdx.x; i < key_cap; i += blockDim.x) bins[i] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kPlanPerThread; j++) {
        const uint32_t pi = (blockIdx.x * kPlanPerThread + j) * blockDim.x + threadIdx.x;
        uint32_t k = ~0u;
        if (pi < n) {
            k = descs[pi].key_idx;
            if (k >= key_cap || !is_aes(keys, k)) k = ~0u;
        }
        // a run of same-key packets fills whole waves (one connection's burst; a single-key batch): one atomic per
        // wave instead of 64 serialised same-address LDS atomics
        const uint32_t k0 = __builtin_amdgcn_readfirstlane(k);
        if (__all(k == k0)) {
            if (k0 != ~0u && (threadIdx.x & 63u) == 0) {
                if (local) atomicAdd(&bins[k0], 64u);
                else atomicAdd(&counts[k0], 64u);
            }
        } else if (k != ~0u) {
            if (local) atomicAdd(&bins[k], 1u);
            else atomicAdd(&counts[k], 1u);
        }
    }
    __syncthreads();
    if (local)
        for (uint32_t i = threadIdx.x; i < key_cap; i += blockDim.x)
            if (bins[i]) atomicAdd(&counts[i], bins[i]);
}

// Single workgroup.  Exclusive scans over keys of (a) packet counts -> cursor (scatter base per key) and
// (b) work items per key -> istart; then every thread emits work items w = tid, tid+1024, ... by a binary
// search of istart (in LDS), so a single key with 16 Ki work items is not written by one lane.
__global__ __launch_bounds__(kPlanBlock) void plan_scan(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                       uint32_t *__restrict__ counts, uint32_t *__restrict__ cursor,
                                                       uint32_t *__restrict__ istart_g, WorkItem *__restrict__ work,
                                                       uint32_t *__restrict__ n_work, uint32_t per) {
    __shared__ uint32_t sc[kPlanBlock], si[kPlanBlock];
    __shared__ uint32_t istart_l[kMaxPlanKeys + 1];
    __shared__ uint32_t carry_c, carry_i;
    const bool local = key_cap <= (uint32_t)kMaxPlanKeys;
    uint32_t *istart = local ? istart_l : istart_g;
    if (threadIdx.x == 0) { carry_c = 0; carry_i = 0; }
    __syncthreads();
    for (uint32_t base = 0; base < key_cap; base += kPlanBlock) {
        const uint32_t k = base + threadIdx.x;
        const uint32_t c = k < key_cap ? counts[k] : 0;
        const uint32_t items = (c + per - 1) / per;
        sc[threadIdx.x] = c;
        si[threadIdx.x] = items;
        __syncthreads();
        for (uint32_t off = 1; off < kPlanBlock; off <<= 1) {  // Hillis-Steele inclusive scan
            uint32_t a = threadIdx.x >= off ? sc[threadIdx.x - off] : 0;
            uint32_t b = threadIdx.x >= off ? si[threadIdx.x - off] : 0;
            __syncthreads();
            sc[threadIdx.x] += a;
            si[threadIdx.x] += b;
            __syncthreads();
        }
        if (k < key_cap) {
            cursor[k] = carry_c + sc[threadIdx.x] - c;
            istart[k] = carry_i + si[threadIdx.x] - items;
        }
        __syncthreads();
        if (threadIdx.x == kPlanBlock - 1) { carry_c += sc[threadIdx.x]; carry_i += si[threadIdx.x]; }
        __syncthreads();
    }
    const uint32_t total = carry_i;
    if (threadIdx.x == 0) { istart[key_cap] = total; *n_work = total; }
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < total; w += kPlanBlock) {
        uint32_t lo = 0, hi = key_cap;  // largest k with istart[k] <= w (keys with no items share a start)
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (istart[mid] <= w) lo = mid; else hi = mid;
        }
        const uint32_t i = w - istart[lo];
        const uint32_t left = counts[lo] - i * per;
        // cursor[] still holds the key's first perm index: plan_scatter runs after this kernel
        work[w] = WorkItem{lo, cursor[lo] + i * per, left < per ? left : per, keys[lo].nr};
    }
    // counts[] is all-zero between plans (zeroed once at allocation, then here after its last read), so the next
    // plan_hist needs no memset launch
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < key_cap; k += kPlanBlock) counts[k] = 0;
}

__global__ __launch_bounds__(kPlanBlock) void plan_scatter(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                          const qpp_pkt *__restrict__ descs, uint32_t n,
                                                          uint32_t *__restrict__ cursor, uint32_t *__restrict__ perm) {
    __shared__ uint32_t bins[kMaxPlanKeys];
    const bool local = key_cap <= (uint32_t)kMaxPlanKeys;
    if (local)
        for (uint32_t i = threadIdx.x; i < key_cap; i += blockDim.x) bins[i] = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t ks[kPlanPerThread], rank[kPlanPerThread];
#pragma unroll
    for (uint32_t j = 0; j < kPlanPerThread; j++) {
        const uint32_t pi = (blockIdx.x * kPlanPerThread + j) * blockDim.x + threadIdx.x;
        uint32_t k = 0xffffffffu;
        rank[j] = 0;
        if (pi < n) {
            k = descs[pi].key_idx;
            if (k >= key_cap || !is_aes(keys, k)) k = 0xffffffffu;
        }
        const uint32_t k0 = __builtin_amdgcn_readfirstlane(k);
        if (__all(k == k0)) {  // whole wave on one key (see plan_hist): one reservation of 64 consecutive ranks
            if (k0 != 0xffffffffu) {
                uint32_t base = 0;
                if (lane == 0) base = local ? atomicAdd(&bins[k0], 64u) : atomicAdd(&cursor[k0], 64u);
                base = (uint32_t)__shfl((int)base, 0, 64) + lane;
                if (local) rank[j] = base;
                else perm[base] = pi;
            }
        } else if (k != 0xffffffffu) {
            if (local) rank[j] = atomicAdd(&bins[k], 1u);
            else perm[atomicAdd(&cursor[k], 1u)] = pi;
        }
        ks[j] = k;
    }
    __syncthreads();
    if (local) {
        // reserve one contiguous range per touched key; reuse bins[] for the range start
        for (uint32_t i = threadIdx.x; i < key_cap; i += blockDim.x)
            if (bins[i]) bins[i] = atomicAdd(&cursor[i], bins[i]);
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < kPlanPerThread; j++)
            if (ks[j] != 0xffffffffu) perm[bins[ks[j]] + rank[j]] = (blockIdx.x * kPlanPerThread + j) * blockDim.x + threadIdx.x;
    }
}

// Small batches (n <= kPlanSmallMax = 8 Ki, key_cap <= kMaxPlanKeys): the three stages above in ONE workgroup and one
// launch (a GSO burst pays ~4 us here instead of a memset + three launches, ~17 us).  Each thread keeps the keys
// of its <= 8 packets in registers; keys are scanned 8 per thread with a wave scan + a 16-entry workgroup scan.
// Dynamic LDS: cur[kMaxPlanKeys + 1] (counts, then scatter cursors), ist[kMaxPlanKeys + 1] (first work item),
// wave totals.
constexpr uint32_t kPlanSmallMax = 8 * kPlanBlock;  // (at 16 Ki the one workgroup took ~18 us more than the 3 launches)
constexpr uint32_t kPlanSmallLds = 4 * (2 * (kMaxPlanKeys + 1) + 64);

__global__ __launch_bounds__(kPlanBlock) void plan_small(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                        const qpp_pkt *__restrict__ descs, uint32_t n,
                                                        uint32_t *__restrict__ perm, WorkItem *__restrict__ work,
                                                        uint32_t *__restrict__ n_work, uint32_t per) {
    extern __shared__ uint32_t smem[];
    uint32_t *cur = smem, *ist = smem + kMaxPlanKeys + 1, *wt = ist + kMaxPlanKeys + 1;  // wt: [2][16]
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    for (uint32_t k = tid; k <= key_cap; k += kPlanBlock) cur[k] = 0;
    __syncthreads();
    uint32_t mine[kPlanSmallMax / kPlanBlock];  // key slot of packets tid + 1024 j (~0u: not an AES packet)
#pragma unroll
    for (uint32_t j = 0; j < kPlanSmallMax / kPlanBlock; j++) {
        const uint32_t pi = tid + kPlanBlock * j;
        uint32_t k = ~0u;
        if (pi < n) {
            k = descs[pi].key_idx;
            if (k >= key_cap || !is_aes(keys, k)) k = ~0u;
            else atomicAdd(&cur[k], 1u);
        }
        mine[j] = k;
    }
    __syncthreads();
    // exclusive scans over keys of counts (-> cursors) and work items (-> ist), kpt consecutive keys per thread
    const uint32_t kpt = (key_cap + kPlanBlock - 1) / kPlanBlock, k0 = tid * kpt;
    uint32_t lc = 0, li = 0;
    for (uint32_t j = 0; j < kpt; j++) {
        const uint32_t c = k0 + j < key_cap ? cur[k0 + j] : 0;
        lc += c;
        li += (c + per - 1) / per;
    }
    uint32_t sc = lc, si = li;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t a = (uint32_t)__shfl_up((int)sc, o, 64), b = (uint32_t)__shfl_up((int)si, o, 64);
        if (lane >= (uint32_t)o) { sc += a; si += b; }
    }
    if (lane == 63) { wt[wave] = sc; wt[16 + wave] = si; }
    __syncthreads();
    uint32_t bc = 0, bi = 0, tc = 0, ti = 0;
    for (uint32_t w = 0; w < kPlanBlock / 64; w++) {
        if (w < wave) { bc += wt[w]; bi += wt[16 + w]; }
        tc += wt[w];
        ti += wt[16 + w];
    }
    uint32_t pc = bc + sc - lc, pw = bi + si - li;  // exclusive prefixes at this thread's first key
    for (uint32_t j = 0; j < kpt; j++) {  // each thread rewrites only its own keys
        const uint32_t k = k0 + j;
        if (k >= key_cap) break;
        const uint32_t c = cur[k];
        cur[k] = pc;
        ist[k] = pw;
        pc += c;
        pw += (c + per - 1) / per;
    }
    if (tid == 0) { cur[key_cap] = tc; ist[key_cap] = ti; *n_work = ti; }
    __syncthreads();
    for (uint32_t w = tid; w < ti; w += kPlanBlock) {
        uint32_t lo = 0, hi = key_cap;  // largest k with ist[k] <= w (keys without items share a start)
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (ist[mid] <= w) lo = mid; else hi = mid;
        }
        const uint32_t i = w - ist[lo];
        const uint32_t left = cur[lo + 1] - cur[lo] - i * per;
        work[w] = WorkItem{lo, cur[lo] + i * per, left < per ? left : per, keys[lo].nr};
    }
    __syncthreads();  // the work items read the cursors' start values; the scatter advances them
#pragma unroll
    for (uint32_t j = 0; j < kPlanSmallMax / kPlanBlock; j++)
        if (mine[j] != ~0u) perm[atomicAdd(&cur[mine[j]], 1u)] = tid + kPlanBlock * j;
}

}  // namespace

uint32_t plan_max_work(uint32_t n, uint32_t key_cap, uint32_t per) {
    const uint32_t by_packets = (n + per - 1) / per;
    const uint32_t by_keys = key_cap < n ? key_cap : n;
    return by_packets + by_keys;
}

hipError_t launch_plan(const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n, PlanBuffers pb,
                       uint32_t per, hipStream_t s) {
    if (n <= kPlanSmallMax && key_cap <= (uint32_t)kMaxPlanKeys) {
        hipLaunchKernelGGL(plan_small, dim3(1), dim3(kPlanBlock), kPlanSmallLds, s, keys, key_cap, descs, n, pb.perm,
                           pb.work, pb.n_work, per);
        return hipGetLastError();
    }
    const dim3 grid((n + kPlanBlock * kPlanPerThread - 1) / (kPlanBlock * kPlanPerThread));
    hipLaunchKernelGGL(plan_hist, grid, dim3(kPlanBlock), 0, s, keys, key_cap, descs, n, pb.counts);
    hipLaunchKernelGGL(plan_scan, dim3(1), dim3(kPlanBlock), 0, s, keys, key_cap, pb.counts, pb.cursor, pb.istart, pb.work,
                       pb.n_work, per);
    hipLaunchKernelGGL(plan_scatter, grid, dim3(kPlanBlock), 0, s, keys, key_cap, descs, n, pb.cursor, pb.perm);
    return hipGetLastError();
}

}  // namespace qpp
