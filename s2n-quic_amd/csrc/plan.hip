// plan.hip — groups the AES packets of a batch by key so that every AES-GCM workgroup serves ONE key
// (its GHASH tables are per key and live in LDS).  Three small launches, all device-side, so a batch
// whose descriptors are already in HBM never round-trips to the host:
//   1. plan_hist   : packets per key (LDS-privatised counts, one global add per touched key per block)
//   2. plan_scan   : one workgroup: key offsets, work list {key, begin, count<=per, rounds}, n_work
//   3. plan_scatter: perm[] = packet indices grouped by key (LDS ranks + one global reservation per key)
// Every other packet (ChaCha20-Poly1305 keys, refused slots) goes, ungrouped, behind the AES packets in perm[] (round
// 5): the ChaCha20 kernel then visits only those (selection mode) instead of every packet of a mixed batch -- its lane
// per packet idled on the AES packets, so a third of ChaCha packets cost a whole ChaCha batch.
// The reference has no batching at all (Key::encrypt is per packet); this is the
// batch former the MI355X design adds in front of the kernels.
#include "device_common.h"

namespace qpp {
namespace {

constexpr int kPlanBlock = 1024;
constexpr uint32_t kPlanPerThread = 4;  // packets per thread in plan_hist / plan_scatter (amortises the per-block bins)

// a live AES packet key (freed slots, header-key-only slots and ChaCha keys are not planned; the ChaCha kernel, which
// visits every packet, reports the refused ones)
__device__ __forceinline__ bool is_aes(const DevKey *keys, uint32_t k) {
    const DevKey &d = keys[k];
    return d.live == 1 && d.suite != QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256 && (d.nr == 10 || d.nr == 14);
}

// key_cap <= kMaxPlanKeys: bins in LDS.  Larger key tables use global atomics directly.
__global__ __launch_bounds__(kPlanBlock) void plan_hist(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                       const qpp_pkt *__restrict__ descs, uint32_t n,
                                                       uint32_t *__restrict__ counts, uint32_t *__restrict__ kq,
                                                       uint32_t *__restrict__ meta) {
    __shared__ uint32_t bins[kMaxPlanKeys];
    __shared__ uint32_t others;
    const bool local = key_cap <= (uint32_t)kMaxPlanKeys;
    if (local)
        for (uint32_t i = threadIdx.x; i < key_cap; i += blockDim.x) bins[i] = 0;
    if (threadIdx.x == 0) others = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kPlanPerThread; j++) {
        const uint32_t pi = (blockIdx.x * kPlanPerThread + j) * blockDim.x + threadIdx.x;
        uint32_t k = ~0u;
        if (pi < n) {
            k = descs[pi].key_idx;
            if (k >= key_cap || !is_aes(keys, k)) k = ~0u;
            kq[pi] = k;  // (plan_scatter reads this instead of the descriptor and the key record again)
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
        // the other packets (not a live AES key): one count for all of them
        const uint64_t other = __ballot(pi < n && k == ~0u);
        if (other && (threadIdx.x & 63u) == 0) atomicAdd(&others, (uint32_t)__popcll(other));
    }
    __syncthreads();
    if (local)
        for (uint32_t i = threadIdx.x; i < key_cap; i += blockDim.x)
            if (bins[i]) atomicAdd(&counts[i], bins[i]);
    if (threadIdx.x == 0 && others) atomicAdd(&meta[6], others);
}

// Single workgroup.  Exclusive scans over keys of (a) packet counts -> cursor (scatter base per key) and
// (b) work items per key -> istart; then every thread emits work items w = tid, tid+1024, ... by a binary
// search of istart (in LDS), so a single key with 16 Ki work items is not written by one lane.
// Class-major: the AES-128 keys' packets and items come first, then the AES-256 keys' (two scans), so each AES size's
// launch sees one contiguous range of perm and of the work list.  meta = {items, AES-128 items, AES-128 packets,
// AES-256 packets, other packets, their first perm index, [6] the other packets' count (plan_hist; zeroed here after
// its read), [7] their scatter cursor (plan_scatter)}.
__global__ __launch_bounds__(kPlanBlock) void plan_scan(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                       uint32_t *__restrict__ counts, uint32_t *__restrict__ cursor,
                                                       uint32_t *__restrict__ istart_g, WorkItem *__restrict__ work,
                                                       uint32_t *__restrict__ meta, uint32_t per) {
    // Round 6: one pass over the keys, kpt consecutive keys per thread, the four sums (packets and items of each
    // class) scanned together -- wave scans by shuffles and one 16-entry scan of the wave totals -- instead of a
    // Hillis-Steele scan per 1024 keys and class (20 barriers each): 35 -> a few us for 4096 keys (plan_small's scan)
    __shared__ uint32_t istart_l[2 * (kMaxPlanKeys + 1)];
    __shared__ uint32_t wt[4][kPlanBlock / 64];
    const bool local = key_cap <= (uint32_t)kMaxPlanKeys;
    uint32_t *istart = local ? istart_l : istart_g;  // [2][key_cap + 1]: per class, non-decreasing in k
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t kpt = (key_cap + kPlanBlock - 1) / kPlanBlock, k0 = tid * kpt;
    auto cls_of = [&](uint32_t k) { return keys[k].nr == 14 ? 1u : 0u; };
    // this thread's counts and classes, loaded once (all loads issued together; up to kMaxPlanKeys keys)
    constexpr uint32_t kKpt = kMaxPlanKeys / kPlanBlock;
    uint32_t cc[kKpt], cl[kKpt];
#pragma unroll
    for (uint32_t j = 0; j < kKpt; j++) {
        const uint32_t k = k0 + j;
        cc[j] = j < kpt && k < key_cap ? counts[k] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < kKpt; j++) cl[j] = cc[j] ? cls_of(k0 + j) : 0u;
    uint32_t v[4] = {0, 0, 0, 0};  // packets of class 0, 1; items of class 0, 1 (this thread's keys)
    for (uint32_t j = 0; j < kpt; j++) {
        const uint32_t k = k0 + j;
        if (k >= key_cap) break;
        const uint32_t c = j < kKpt ? cc[j] : counts[k];
        if (!c) continue;
        const uint32_t cls = j < kKpt ? cl[j] : cls_of(k);
        v[cls] += c;
        v[2 + cls] += (c - 1) / per + 1;
    }
    uint32_t sc[4];  // inclusive wave scans
#pragma unroll
    for (int i = 0; i < 4; i++) sc[i] = v[i];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t a = (uint32_t)__shfl_up((int)sc[i], o, 64);
            if (lane >= (uint32_t)o) sc[i] += a;
        }
    }
    if (lane == 63) {
#pragma unroll
        for (int i = 0; i < 4; i++) wt[i][wave] = sc[i];
    }
    __syncthreads();
    uint32_t pre[4], tot[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        pre[i] = sc[i] - v[i];
        tot[i] = 0;
        for (uint32_t w = 0; w < kPlanBlock / 64; w++) {
            if (w < wave) pre[i] += wt[i][w];
            tot[i] += wt[i][w];
        }
    }
    // class-major: class 0's packets and items from 0, class 1's behind them
    uint32_t pc[2] = {pre[0], tot[0] + pre[1]}, pw[2] = {pre[2], tot[2] + pre[3]};
    uint32_t *ist0 = istart, *ist1 = istart + key_cap + 1;
    for (uint32_t j = 0; j < kpt; j++) {
        const uint32_t k = k0 + j;
        if (k >= key_cap) break;
        const uint32_t c = j < kKpt ? cc[j] : counts[k];
        ist0[k] = pw[0];
        ist1[k] = pw[1];
        if (!c) continue;
        const uint32_t cls = j < kKpt ? cl[j] : cls_of(k);
        cursor[k] = pc[cls];
        pc[cls] += c;
        pw[cls] += (c - 1) / per + 1;
    }
    const uint32_t total = tot[2] + tot[3], i10 = tot[2];
    if (tid == 0) {
        ist0[key_cap] = i10;
        ist1[key_cap] = total;
        meta[0] = total; meta[1] = i10; meta[2] = tot[0]; meta[3] = tot[1];
        meta[4] = meta[6]; meta[5] = tot[0] + tot[1]; meta[6] = 0; meta[7] = tot[0] + tot[1];
    }
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < total; w += kPlanBlock) {
        const uint32_t *ist = istart + (w >= i10 ? key_cap + 1 : 0);
        uint32_t lo = 0, hi = key_cap;  // largest k with ist[k] <= w (keys with no items share a start)
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (ist[mid] <= w) lo = mid; else hi = mid;
        }
        const uint32_t i = w - ist[lo];
        const uint32_t left = counts[lo] - i * per;
        // cursor[] still holds the key's first perm index: plan_scatter runs after this kernel
        work[w] = WorkItem{lo, cursor[lo] + i * per, left < per ? left : per, keys[lo].nr};
    }
    // counts[] is all-zero between plans (zeroed once at allocation, then here after its last read), so the next
    // plan_hist needs no memset launch
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < key_cap; k += kPlanBlock) counts[k] = 0;
}

__global__ __launch_bounds__(kPlanBlock) void plan_scatter(uint32_t key_cap, const uint32_t *__restrict__ kq, uint32_t n,
                                                          uint32_t *__restrict__ cursor, uint32_t *__restrict__ perm,
                                                          uint32_t *__restrict__ meta) {
    __shared__ uint32_t bins[kMaxPlanKeys];
    __shared__ uint32_t others;
    const bool local = key_cap <= (uint32_t)kMaxPlanKeys;
    if (local)
        for (uint32_t i = threadIdx.x; i < key_cap; i += blockDim.x) bins[i] = 0;
    if (threadIdx.x == 0) others = 0;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t ks[kPlanPerThread], rank[kPlanPerThread], orank[kPlanPerThread];
#pragma unroll
    for (uint32_t j = 0; j < kPlanPerThread; j++) {
        const uint32_t pi = (blockIdx.x * kPlanPerThread + j) * blockDim.x + threadIdx.x;
        const uint32_t k = pi < n ? kq[pi] : 0xffffffffu;
        rank[j] = 0;
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
        // the other packets: a rank in the block's run of them (wave ballot + one LDS add per wave)
        const bool oth = pi < n && k == 0xffffffffu;
        const uint64_t ob = __ballot(oth);
        uint32_t obase = 0;
        if (ob && lane == 0) obase = atomicAdd(&others, (uint32_t)__popcll(ob));
        obase = (uint32_t)__shfl((int)obase, 0, 64);
        orank[j] = oth ? obase + (uint32_t)__popcll(ob & ((1ull << lane) - 1ull)) : 0xffffffffu;
    }
    __syncthreads();
    // one reservation of the block's run of other packets behind the AES packets (meta[7]: plan_scan set it there)
    if (threadIdx.x == 0 && others) others = atomicAdd(&meta[7], others);
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kPlanPerThread; j++)
        if (orank[j] != 0xffffffffu) perm[others + orank[j]] = (blockIdx.x * kPlanPerThread + j) * blockDim.x + threadIdx.x;
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
// Dynamic LDS: counts / scatter cursors, start cursors, first work item per key and class, wave totals.
constexpr uint32_t kPlanSmallMax = 8 * kPlanBlock;  // (at 16 Ki the one workgroup took ~18 us more than the 3 launches)
constexpr uint32_t kPlanSmallLds = 4 * (4 * (kMaxPlanKeys + 1) + 64);

__global__ __launch_bounds__(kPlanBlock) void plan_small(const DevKey *__restrict__ keys, uint32_t key_cap,
                                                        const qpp_pkt *__restrict__ descs, uint32_t n,
                                                        uint32_t *__restrict__ perm, WorkItem *__restrict__ work,
                                                        uint32_t *__restrict__ n_work, uint32_t per) {
    extern __shared__ uint32_t smem[];
    // cur[kMaxPlanKeys + 1] (counts, then scatter cursors) | start cursors | ist2[2][kMaxPlanKeys + 1] | wt[2][16]
    uint32_t *cur = smem, *ist2 = smem + 2 * (kMaxPlanKeys + 1), *wt = ist2 + 2 * (kMaxPlanKeys + 1);
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
    // exclusive scans over keys of counts (-> cursors) and work items (-> ist), kpt consecutive keys per thread,
    // class-major (AES-128 keys first, then AES-256: see plan_scan); ist[cls][k] non-decreasing in k per class
    const uint32_t kpt = (key_cap + kPlanBlock - 1) / kPlanBlock, k0 = tid * kpt;
    uint32_t cnt[2], itm[2];  // class totals
    uint32_t *st0 = smem + kMaxPlanKeys + 1;  // start cursors (cur[] is reused for the counts until the scans end)
    for (uint32_t cls = 0; cls < 2; cls++) {
        uint32_t *ist = ist2 + cls * (kMaxPlanKeys + 1);
        const uint32_t cb = cls ? cnt[0] : 0, ib = cls ? itm[0] : 0;
        auto cnt_of = [&](uint32_t k) -> uint32_t {
            const uint32_t c = cur[k];
            return c && (keys[k].nr == 14) == (cls == 1) ? c : 0;
        };
        uint32_t lc = 0, li = 0;
        for (uint32_t j = 0; j < kpt; j++) {
            const uint32_t c = k0 + j < key_cap ? cnt_of(k0 + j) : 0;
            lc += c;
            li += c ? (c - 1) / per + 1 : 0;
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
        __syncthreads();  // wt[] is rewritten by the next class
        uint32_t pc = cb + bc + sc - lc, pw = ib + bi + si - li;  // exclusive prefixes at this thread's first key
        for (uint32_t j = 0; j < kpt; j++) {  // each thread writes only its own keys
            const uint32_t k = k0 + j;
            if (k >= key_cap) break;
            const uint32_t c = cnt_of(k);
            if (c) st0[k] = pc;
            ist[k] = pw;
            pc += c;
            pw += c ? (c - 1) / per + 1 : 0;
        }
        cnt[cls] = cb + tc;
        itm[cls] = ib + ti;
        if (tid == 0) ist[key_cap] = itm[cls];
    }
    __syncthreads();
    const uint32_t ti = itm[1], i10 = itm[0];
    if (tid == 0) { n_work[0] = ti; n_work[1] = i10; n_work[2] = cnt[0]; n_work[3] = cnt[1] - cnt[0]; }
    for (uint32_t w = tid; w < ti; w += kPlanBlock) {
        const uint32_t *ist = ist2 + (w >= i10 ? kMaxPlanKeys + 1 : 0);
        uint32_t lo = 0, hi = key_cap;  // largest k with ist[k] <= w (keys without items share a start)
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (ist[mid] <= w) lo = mid; else hi = mid;
        }
        const uint32_t i = w - ist[lo];
        const uint32_t left = cur[lo] - i * per;
        work[w] = WorkItem{lo, st0[lo] + i * per, left < per ? left : per, keys[lo].nr};
    }
    __syncthreads();  // the counts are read by the work items; from here cur[] holds the scatter cursors
    for (uint32_t k = tid; k < key_cap; k += kPlanBlock)
        if (cur[k]) cur[k] = st0[k];
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

bool plan_lists_others(uint32_t n, uint32_t key_cap) { return !(n <= kPlanSmallMax && key_cap <= (uint32_t)kMaxPlanKeys); }

hipError_t launch_plan(const DevKey *keys, uint32_t key_cap, const qpp_pkt *descs, uint32_t n, PlanBuffers pb,
                       uint32_t per, hipStream_t s) {
    if (!plan_lists_others(n, key_cap)) {
        hipLaunchKernelGGL(plan_small, dim3(1), dim3(kPlanBlock), kPlanSmallLds, s, keys, key_cap, descs, n, pb.perm,
                           pb.work, pb.n_work, per);
        return hipGetLastError();
    }
    const dim3 grid((n + kPlanBlock * kPlanPerThread - 1) / (kPlanBlock * kPlanPerThread));
    hipLaunchKernelGGL(plan_hist, grid, dim3(kPlanBlock), 0, s, keys, key_cap, descs, n, pb.counts, pb.kq, pb.n_work);
    hipLaunchKernelGGL(plan_scan, dim3(1), dim3(kPlanBlock), 0, s, keys, key_cap, pb.counts, pb.cursor, pb.istart, pb.work,
                       pb.n_work, per);
    hipLaunchKernelGGL(plan_scatter, grid, dim3(kPlanBlock), 0, s, key_cap, pb.kq, n, pb.cursor, pb.perm, pb.n_work);
    return hipGetLastError();
}

// Connection-indexed descriptors (QPP_KEY_BY_CONN): key_idx names a connection's entry in the device table `map`
// (the transport's KeySet, crypto/application/keyset.rs: a key update swaps the key behind the entry, the packets
// queued for the connection do not change); the slot it holds replaces key_idx in the batch's device copy.  An index
// past the table becomes 0xffffffff, a slot outside every key table (the packet is refused, INTERNAL_ERROR).
__global__ void conn_remap_kernel(qpp_pkt *descs, uint32_t n, const uint32_t *__restrict__ map, uint32_t map_n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = descs[i].key_idx;
    descs[i].key_idx = c < map_n ? map[c] : 0xffffffffu;
}

hipError_t launch_conn_remap(qpp_pkt *descs, uint32_t n, const uint32_t *map, uint32_t map_n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(conn_remap_kernel, dim3((n + 255) / 256), dim3(256), 0, s, descs, n, map, map_n);
    return hipGetLastError();
}

}  // namespace qpp
