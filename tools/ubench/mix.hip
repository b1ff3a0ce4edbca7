// mix.hip — how far can one CU co-issue LDS-array work and VALU work in the quad kernel's instruction mix?
// (VERDICT r5 "Next round" #1: settle the headline kernel's ceiling with one decisive microbenchmark.)
//
// No global memory in any timed loop: every lane folds what it computes into registers and stores one 16-byte word at
// the end.  One workgroup per CU (160 KiB of LDS each), 512 / 768 / 1024 threads = 2 / 3 / 4 waves per SIMD.
//
//   real    the quad kernel's group body itself (csrc/quad.hip): ctr_keystream_q4 over 4 counter blocks per lane
//           (CtrPageQ4 rounds 1-2 cached, AesQ4 lookups) + 4 GHASH Horner steps (GhashT<true>::mulx) per group --
//           the product's exact per-lane mix AND dependency shape, minus the payload loads and stores
//   aes     the keystream alone (no GHASH)
//   ghash   the 4 GHASH steps alone (the keystream replaced by a counter)
//   synth   the same counts per 4 blocks with NO data dependency from a load to a later address: 4 independent
//           "columns" per block whose addresses come from a counter, 133 ds_read_b32 + 16 ds_read_b128 per block and
//           the VALU the product spends per lookup -- the co-issue ceiling of this instruction mix on this hardware
//   lds     ds_read_b32 alone (conflict-free, per-lane bank copies), no VALU: the LDS array's own peak
//   valu    v_perm / v_bitop3 alone: VALU issue peak
//
// Cycles are s_memtime of workgroup 0 (shader clock); "per wave-block" = one 16-B block for every lane of one wave.
// Counters: run under `rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES
// SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- ./mix <mode>` (tools/ubench/run_mix.sh does every pass).
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/ubench/mix.hip -o tools/ubench/mix
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../s2n-quic_amd/csrc/device_common.h"
#include "../../s2n-quic_amd/csrc/ghash.h"

using namespace qpp;
using namespace qpp::dev;

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

struct Clock {
    uint64_t t0, t1, r0, r1;
};
__device__ __forceinline__ void clk_mark(Clock *c, bool end) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (!end) {
            c->t0 = __builtin_amdgcn_s_memtime();
            c->r0 = __builtin_amdgcn_s_memrealtime();
        } else {
            c->t1 = __builtin_amdgcn_s_memtime();
            c->r1 = __builtin_amdgcn_s_memrealtime();
        }
    }
}

// LDS filled with arbitrary words (timing does not depend on table values; every address the code forms stays in
// its region: AesQ4 lookups in [64 KiB, 128 KiB), GHASH lookups in [0, 64 KiB))
__device__ void fill_lds() {
    for (uint32_t i = threadIdx.x; i < kLdsMax / 4; i += blockDim.x) lds_st32(4 * i, i * 0x9e3779b9u ^ 0x5bd1e995u);
    __syncthreads();
}

// ---------------------------------------------------------------- real: the group body
template <int MODE, int WG>  // MODE 0 real, 1 aes, 2 ghash
__global__ __launch_bounds__(WG) void real_k(const DevKey *__restrict__ key, int G, uint4 *out, Clock *clk) {
    fill_lds();
    const AesQ4 aes = AesQ4::make();
    const GhashT<true> gh = GhashT<true>::make();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, s = threadIdx.x & 3u;
    const uint32_t n0 = tid * 0x9e3779b9u, n1 = tid ^ 0x85ebca6bu, n2 = 0x01234567u ^ tid;
    uint64_t a = (uint64_t)key->rk;
    asm volatile("" : "+s"(a));
    RkPtr rkp = (RkPtr)a;
    CtrPageQ4 pg;
    pg.build(aes, rkp, n0, n1, n2, 0);
    uint4 w = make_uint4(0, 0, 0, 0), acc = make_uint4(tid, 0, 0, 0);
    __syncthreads();
    clk_mark(clk, false);
    for (int g = 0; g < G; g++) {
        const uint32_t c0 = (uint32_t)(16 * g) + s + 1u;
        uint64_t ap = (uint64_t)key->rk;
        asm volatile("" : "+s"(ap));  // round keys reloaded per group, as the product does
        const RkPtr rk = (RkPtr)ap;
        uint4 ks[4];
        if constexpr (MODE != 2) {
            if ((c0 >> 8) != pg.page) {
                uint32_t m0 = n0, m1 = n1, m2 = n2;
                asm volatile("" : "+v"(m0), "+v"(m1), "+v"(m2));
                pg.build(aes, rk, m0, m1, m2, c0 >> 8);
            }
            uint32_t r[44];
#pragma unroll
            for (int i = 3; i <= 10; i++) {
                const uint4 v = rk[i];
                r[4 * i] = v.x; r[4 * i + 1] = v.y; r[4 * i + 2] = v.z; r[4 * i + 3] = v.w;
            }
            ctr_keystream_q4<10, 4, 4>(aes, pg, r, c0, ks);
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) ks[k] = make_uint4(c0 + 4 * k, n0, n1, n2);
        }
        if constexpr (MODE != 1) {
#pragma unroll
            for (int k = 0; k < 4; k++) w = gh.mulx(w, ks[k] ^ acc);  // (ciphertext = payload ^ keystream)
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) acc = acc ^ ks[k];
        }
    }
    clk_mark(clk, true);
    out[tid] = w ^ acc;
}

// ---------------------------------------------------------------- synth: same counts, no load -> address dependency
// Per block: AESU units of (4 x [v_perm address + ds_read_b32] + 2 v_bitop3 into an accumulator + VX extra VALU),
// then (GH) one GHASH-shaped product: 16 x [v_perm address + ds_read_b128] + 5 xor3 of uint4 + word selects.
// 4 blocks per group, their units interleaved (unit-major) with D units issued ahead, as ctr_keystream_q4 does.
template <int WG, int AESU, int VX, bool GH, int D>
__global__ __launch_bounds__(WG) void synth_k(int G, uint4 *out, Clock *clk) {
    fill_lds();
    const AesQ4 aes = AesQ4::make();
    const GhashT<true> gh = GhashT<true>::make();
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t ctr[4], acc[4];
#pragma unroll
    for (int b = 0; b < 4; b++) {
        ctr[b] = tid * (0x9e3779b9u + b);
        acc[b] = b;
    }
    uint4 gacc = make_uint4(tid, 1, 2, 3);
    const uint32_t kc = tid | 0x01000193u;
    __syncthreads();
    clk_mark(clk, false);
    for (int g = 0; g < G; g++) {
        constexpr int U = 4 * AESU;  // units of the group, block-interleaved: unit u -> block u % 4
        uint32_t ld[D + 1][4];
        auto issue = [&](auto uc) {
            constexpr int u = decltype(uc)::value, b = u % 4;
            uint32_t *l = ld[u % (D + 1)];
            asm volatile("" : "+v"(ctr[b]));  // (no precomputed address sequences)
            l[0] = aes.look<0>(ctr[b]);
            l[1] = aes.look<1>(ctr[b]);
            l[2] = aes.look<2>(ctr[b]);
            l[3] = aes.look<3>(ctr[b]);
            ctr[b] += 0x01030507u;  // next addresses from the counter (1 VALU)
        };
        auto combine = [&](auto uc) {
            constexpr int u = decltype(uc)::value, b = u % 4;
            const uint32_t *l = ld[u % (D + 1)];
            // (v_bitop3 builtins, not ^: LLVM reassociates a plain xor chain across the whole group and defers it)
            uint32_t x = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(l[0], l[1], l[2], 0x96), l[3], acc[b], 0x96);
#pragma unroll
            for (int v = 0; v < VX; v++) x = __builtin_amdgcn_bitop3_b32(x, kc, (uint32_t)v, 0x96);
            asm volatile("" : "+v"(x));  // materialized here (no reassociation across units)
            acc[b] = x;
        };
        static_for<D>([&](auto uc) { issue(uc); });
        static_for<U>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            if constexpr (u + D < U) issue(std::integral_constant<int, u + D>{});
            __builtin_amdgcn_sched_barrier(0);
            combine(uc);
            __builtin_amdgcn_sched_barrier(0);
        });
        if constexpr (GH) {
#pragma unroll
            for (int b = 0; b < 4; b++) {
                // GHASH-shaped: the product's 16 reads (addresses from the AES accumulators, not from its own result)
                const uint4 wv = make_uint4(acc[b], acc[(b + 1) & 3], ctr[b], ctr[(b + 2) & 3]);
                gacc = gh.mulx(wv, gacc);
            }
        }
    }
    clk_mark(clk, true);
    out[tid] = gacc ^ make_uint4(acc[0], acc[1], acc[2], acc[3]);
}

// ---------------------------------------------------------------- lds / valu alone
template <int WG>
__global__ __launch_bounds__(WG) void lds_k(int G, uint4 *out, Clock *clk) {
    fill_lds();
    const uint32_t base = 65536u + 4u * (threadIdx.x & 31u);  // lane's copy: bank lane % 32, rows by the offset field
    uint32_t a = base;
    uint32_t r[16];
#pragma unroll
    for (int i = 0; i < 16; i++) r[i] = 0;
    __syncthreads();
    clk_mark(clk, false);
    for (int g = 0; g < G; g++) {
        asm volatile("" : "+v"(a));
#pragma unroll
        for (int i = 0; i < 16; i++) {
            uint32_t v;
            asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(256 * (i * 13 % 64)));
            r[i] ^= v;  // 1 VALU per read: the minimum that keeps the loads (the LDS array stays the bound)
        }
    }
    clk_mark(clk, true);
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) x ^= r[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = make_uint4(x, 0, 0, 0);
}
template <int WG>
__global__ __launch_bounds__(WG) void valu_k(int G, uint4 *out, Clock *clk) {
    uint32_t u[8];
#pragma unroll
    for (int i = 0; i < 8; i++) u[i] = threadIdx.x * (i + 3);
    const uint32_t c = blockIdx.x | 0x10101u;
    clk_mark(clk, false);
    for (int g = 0; g < G; g++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            u[i] = __builtin_amdgcn_perm(u[i], c + i, 0x05040100u);
            u[i] = __builtin_amdgcn_bitop3_b32(u[i], c, c + i, 0x96);
        }
    }
    clk_mark(clk, true);
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= u[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = make_uint4(x, 0, 0, 0);
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "all";
    const bool all = !strcmp(mode, "all");
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    DevKey hk;
    memset(&hk, 0, sizeof hk);
    for (int i = 0; i < 60; i++) hk.rk[i] = 0x9e3779b9u * (uint32_t)(i + 1);
    DevKey *d_key;
    uint4 *d_out;
    Clock *d_clk;
    CK(hipMalloc(&d_key, sizeof hk));
    CK(hipMemcpy(d_key, &hk, sizeof hk, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_out, (size_t)cus * 1024 * 16));
    CK(hipMalloc(&d_clk, sizeof(Clock)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // Each line: mode, waves/SIMD, ms, G blocks/s, CU cycles per wave-block (wall time x the measured clock over the
    // wave-blocks one CU runs), and workgroup 0's own cycles per wave-block (s_memtime).
    auto run = [&](const char *name, int wg, double blocks_per_lane, auto launch) {
        float best = 1e30f;
        for (int rep = 0; rep < 4; rep++) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipGetLastError());
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep && ms < best) best = ms;
        }
        Clock c;
        CK(hipMemcpy(&c, d_clk, sizeof c, hipMemcpyDeviceToHost));
        const double cyc = (double)(c.t1 - c.t0), ghz = cyc / ((double)(c.r1 - c.r0) * 10.0);
        const double wave_blocks_per_cu = (double)wg / 64.0 * blocks_per_lane;
        const double blocks = (double)cus * wg * blocks_per_lane;
        printf("%-14s w/SIMD %d  %8.3f ms  %7.1f G blocks/s  %6.1f cyc/wave-block/CU (wall x %.2f GHz)  wg0 %6.1f\n", name,
               wg / 256, best, blocks / (best * 1e6), best * 1e6 * ghz / wave_blocks_per_cu, ghz, cyc / wave_blocks_per_cu);
    };
    const int G = 2048;  // groups of 4 blocks per lane
#define RUN_WG(NAME, KERN, WG, BPL, ...) \
    run(NAME, WG, BPL, [&] { hipLaunchKernelGGL(KERN, dim3(cus), dim3(WG), kLdsMax, 0, __VA_ARGS__); })
    if (all || !strcmp(mode, "real")) {
        RUN_WG("real", (real_k<0, 512>), 512, 4.0 * G, d_key, G, d_out, d_clk);
        RUN_WG("real", (real_k<0, 768>), 768, 4.0 * G, d_key, G, d_out, d_clk);
        RUN_WG("real", (real_k<0, 1024>), 1024, 4.0 * G, d_key, G, d_out, d_clk);
    }
    if (all || !strcmp(mode, "aes")) {
        RUN_WG("aes", (real_k<1, 768>), 768, 4.0 * G, d_key, G, d_out, d_clk);
        RUN_WG("aes", (real_k<1, 1024>), 1024, 4.0 * G, d_key, G, d_out, d_clk);
    }
    if (all || !strcmp(mode, "ghash")) {
        RUN_WG("ghash", (real_k<2, 768>), 768, 4.0 * G, d_key, G, d_out, d_clk);
        RUN_WG("ghash", (real_k<2, 1024>), 1024, 4.0 * G, d_key, G, d_out, d_clk);
    }
    if (all || !strcmp(mode, "synth")) {
        // 33 units x 4 lookups = 132 ds_read_b32 per block (the product: 133), 4 perm + 2 bitop3 + 1 add per unit
        // (+ VX more bitop3): VX = 0 is the real body's VALU count per 4 blocks within a few percent
        RUN_WG("synth/d3", (synth_k<512, 33, 0, true, 3>), 512, 4.0 * G, G, d_out, d_clk);
        RUN_WG("synth/d3", (synth_k<768, 33, 0, true, 3>), 768, 4.0 * G, G, d_out, d_clk);
        RUN_WG("synth/d3", (synth_k<1024, 33, 0, true, 3>), 1024, 4.0 * G, G, d_out, d_clk);
        RUN_WG("synth/d6", (synth_k<768, 33, 0, true, 6>), 768, 4.0 * G, G, d_out, d_clk);
        RUN_WG("synth/d6", (synth_k<1024, 33, 0, true, 6>), 1024, 4.0 * G, G, d_out, d_clk);
        RUN_WG("synth/nogh", (synth_k<768, 33, 0, false, 3>), 768, 4.0 * G, G, d_out, d_clk);
        RUN_WG("synth/vx2", (synth_k<768, 33, 2, true, 3>), 768, 4.0 * G, G, d_out, d_clk);
        RUN_WG("synth/vx2", (synth_k<1024, 33, 2, true, 3>), 1024, 4.0 * G, G, d_out, d_clk);
    }
    if (all || !strcmp(mode, "lds")) {
        // 16 reads per iteration; "blocks" here = reads / 16
        RUN_WG("lds", (lds_k<512>), 512, (double)G, G, d_out, d_clk);
        RUN_WG("lds", (lds_k<768>), 768, (double)G, G, d_out, d_clk);
        RUN_WG("lds", (lds_k<1024>), 1024, (double)G, G, d_out, d_clk);
    }
    if (all || !strcmp(mode, "valu")) {
        // 16 VALU per iteration; "blocks" = iterations
        RUN_WG("valu", (valu_k<768>), 768, (double)G * 8, G * 8, d_out, d_clk);
        RUN_WG("valu", (valu_k<1024>), 1024, (double)G * 8, G * 8, d_out, d_clk);
    }
    printf("device: %d CUs, %s\n", cus, prop.gcnArchName);
    return 0;
}
