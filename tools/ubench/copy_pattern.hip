// copy_pattern.hip — calibration of FETCH_SIZE / WRITE_SIZE (rocprofv3 --pmc) for the access pattern of the lane-per-
// packet AES-GCM kernel: every wave owns 64 packets; in each group iteration the 4 lanes of a lane-group move ONE
// packet's 64-byte chunk (16 B each), read then written back in place (what seal does to the payload).  Modes:
//   0 coop     : the kernel's pattern, packets at a 1248-B stride, payload at +21 (chunks straddle 64-B segments)
//   1 aligned  : the same pattern with every chunk 64-B aligned (1280-B stride, payload at +64, chunk = blocks 4g..4g+3)
//   2 stream   : in-place 16 B per lane over the same payload bytes, consecutive lanes consecutive (the guide's
//                calibrated case)
//   3 coop_nt  : mode 0 with streaming (nt) stores, as the kernels store their payload chunks since round 2
//   4 coop_read: mode 0's loads only (one dword per packet written), for the read-side calibration alone
//   5 coop128_read: loads only, 8 lanes per packet (128-B chunks, 8 packets per wave instruction)
//   6 coop256_read: loads only, 16 lanes per packet (256-B chunks, 4 packets per wave instruction)
//   7 / 8 / 9: nt stores only with 64- / 128- / 256-B chunks; 10 / 11: in-place copy (nt stores) with 128- / 256-B chunks
//   12: in-place copy, loads in 128-B chunks (8 lanes per packet, two 64-B groups), nt stores in 64-B chunks
//   13: in-place copy, loads in 64-B chunks, nt stores in 128-B chunks (two groups' outputs at a time)
// Algorithmic traffic is the same in all modes: 1200 B read + 1200 B written per packet.
// usage: copy_pattern <mode> [packets] [reps]   (prints mode, ms per launch, algorithmic GB)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kPay = 1200;

__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
    uint4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}
__device__ __forceinline__ void st16(uint8_t *p, uint4 v) { __builtin_memcpy(p, &v, 16); }
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_nt(uint8_t *p, uint4 v) {
    u32x4 t;
    t.x = v.x; t.y = v.y; t.z = v.z; t.w = v.w;
    __builtin_nontemporal_store(t, (u32x4 *)p);
}

template <int MODE>
__global__ __launch_bounds__(256) void copy_kernel(uint8_t *arena, uint32_t n, uint32_t stride, uint32_t pay_off) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (MODE == 2) {
        const size_t total = (size_t)n * stride / 16;
        for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
            const size_t pkt = i * 16 / stride, o = i * 16 % stride;
            if (o < pay_off || o + 16 > pay_off + kPay) continue;  // payload bytes only (the same bytes as above)
            uint8_t *p = arena + i * 16;
            st16(p, ld16(p) ^ make_uint4(0x01010101u, 0, 0, (uint32_t)pkt));
        }
        return;
    }
    const uint32_t first = wave * 64;
    if (first >= n) return;
    if (MODE == 13) {
        for (int h = 0; h < (kPay / 16 + 2 + 7) / 8; h++) {
            uint4 r[8];
#pragma unroll
            for (int gg = 0; gg < 2; gg++)
#pragma unroll
                for (int i = 0; i < 4; i++) {  // 64-B loads: lane-group of 4 -> packet 16 i + lane / 4
                    const uint32_t p = first + 16 * i + lane / 4;
                    const int b = 8 * h + 4 * gg - 2 + (int)(lane & 3);
                    r[4 * gg + i] = (p < n && b >= 0 && 16 * (b + 1) <= kPay)
                                        ? ld16(arena + (size_t)p * stride + pay_off + 16 * b) : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
            for (int i = 0; i < 8; i++) {  // 128-B stores: lane-group of 8 -> packet 8 i + lane / 8
                const uint32_t p = first + 8 * i + lane / 8;
                const int b = 8 * h - 2 + (int)(lane % 8);
                if (p >= n || b < 0 || 16 * (b + 1) > kPay) continue;
                st16_nt(arena + (size_t)p * stride + pay_off + 16 * b, r[i] ^ make_uint4(0x01010101u, 0, 0, p));
            }
        }
        return;
    }
    if (MODE == 12) {
        for (int h = 0; h < (kPay / 16 + 2 + 7) / 8; h++) {
            uint4 r[8];
#pragma unroll
            for (int i = 0; i < 8; i++) {  // 128-B loads: lane-group of 8 -> packet 8 i + lane / 8
                const uint32_t p = first + 8 * i + lane / 8;
                const int b = 8 * h - 2 + (int)(lane % 8);
                r[i] = (p < n && b >= 0 && 16 * (b + 1) <= kPay) ? ld16(arena + (size_t)p * stride + pay_off + 16 * b)
                                                                 : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int gg = 0; gg < 2; gg++)
#pragma unroll
                for (int i = 0; i < 4; i++) {  // 64-B stores: lane-group of 4 -> packet 16 i + lane / 4
                    const uint32_t p = first + 16 * i + lane / 4;
                    const int b = 8 * h + 4 * gg - 2 + (int)(lane & 3);
                    if (p >= n || b < 0 || 16 * (b + 1) > kPay) continue;
                    st16_nt(arena + (size_t)p * stride + pay_off + 16 * b, r[4 * gg + i] ^ make_uint4(0x01010101u, 0, 0, p));
                }
        }
        return;
    }
    if (MODE >= 5) {
        constexpr int L = (MODE == 5 || MODE == 8 || MODE == 10) ? 8 : MODE == 7 ? 4 : 16, PPI = 64 / L;
        constexpr bool LD = MODE == 5 || MODE == 6 || MODE >= 10, ST = MODE >= 7;
        uint32_t acc = 0;
        for (int g = 0; g < (kPay / 16 + 2 + L - 1) / L; g++) {
#pragma unroll
            for (int i = 0; i < L; i++) {
                const uint32_t p = first + PPI * i + lane / L;
                const int b = L * g - 2 + (int)(lane % L);
                if (p >= n || b < 0 || 16 * (b + 1) > kPay) continue;
                uint8_t *q = arena + (size_t)p * stride + pay_off + 16 * b;
                const uint4 v = LD ? ld16(q) : make_uint4(p, b, 0, 0);
                if (ST) st16_nt(q, v ^ make_uint4(0x01010101u, 0, 0, p));
                else acc += v.x ^ v.y ^ v.z ^ v.w;
            }
        }
        if (ST) return;
        if (lane < 16 && first + lane < n) *(uint32_t *)(arena + (size_t)(first + lane) * stride) = acc;
        return;
    }
    const int groups = (kPay / 16 + 2 + 3) / 4;
    uint32_t acc = 0;
    for (int g = 0; g < groups; g++) {
#pragma unroll
        for (int i = 0; i < 4; i++) {           // wave instruction i: lane-group q = lane / 4 moves packet 16 i + q
            const uint32_t p = first + 16 * i + lane / 4;
            const int b = MODE != 1 ? 4 * g - 2 + (int)(lane & 3) : 4 * g + (int)(lane & 3);
            if (p >= n || b < 0 || 16 * (b + 1) > kPay) continue;
            uint8_t *q = arena + (size_t)p * stride + pay_off + 16 * b;
            const uint4 v = ld16(q);
            if (MODE == 4) acc += v.x ^ v.y ^ v.z ^ v.w;
            else if (MODE == 3) st16_nt(q, v ^ make_uint4(0x01010101u, 0, 0, p));
            else st16(q, v ^ make_uint4(0x01010101u, 0, 0, p));
        }
    }
    if (MODE == 4 && lane < 16 && first + lane < n)  // keeps the loads; 4 B per 4 packets, noise in WRITE_SIZE
        *(uint32_t *)(arena + (size_t)(first + lane) * stride) = acc;
}

int main(int argc, char **argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : (1u << 20);
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const uint32_t stride = mode == 1 ? 1280 : 1248, pay_off = mode == 1 ? 64 : 21;
    uint8_t *arena = nullptr;
    if (hipMalloc(&arena, (size_t)n * stride) != hipSuccess) return 1;
    hipMemset(arena, 0x5a, (size_t)n * stride);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const dim3 block(256), grid(mode == 2 ? 4096 : (n / 64 + 3) / 4);
    float total = 0;
    for (int r = 0; r < reps + 1; r++) {
        hipEventRecord(e0, 0);
        if (mode == 0) hipLaunchKernelGGL(copy_kernel<0>, grid, block, 0, 0, arena, n, stride, pay_off);
        else if (mode == 1) hipLaunchKernelGGL(copy_kernel<1>, grid, block, 0, 0, arena, n, stride, pay_off);
        else if (mode == 3) hipLaunchKernelGGL(copy_kernel<3>, grid, block, 0, 0, arena, n, stride, pay_off);
        else if (mode == 4) hipLaunchKernelGGL(copy_kernel<4>, grid, block, 0, 0, arena, n, stride, pay_off);
        else if (mode == 5) hipLaunchKernelGGL(copy_kernel<5>, grid, block, 0, 0, arena, n, stride, pay_off);
        else if (mode == 6) hipLaunchKernelGGL(copy_kernel<6>, grid, block, 0, 0, arena, n, stride, pay_off);
        else if (mode == 7) hipLaunchKernelGGL(copy_kernel<7>, grid, block, 0, 0, arena, n, stride, pay_off);
        else if (mode == 8) hipLaunchKernelGGL(copy_kernel<8>, grid, block, 0, 0, arena, n, stride, pay_off);
        else if (mode == 9) hipLaunchKernelGGL(copy_kernel<9>, grid, block, 0, 0, arena, n, stride, pay_off);
        else if (mode == 10) hipLaunchKernelGGL(copy_kernel<10>, grid, block, 0, 0, arena, n, stride, pay_off);
        else if (mode == 11) hipLaunchKernelGGL(copy_kernel<11>, grid, block, 0, 0, arena, n, stride, pay_off);
        else if (mode == 12) hipLaunchKernelGGL(copy_kernel<12>, grid, block, 0, 0, arena, n, stride, pay_off);
        else if (mode == 13) hipLaunchKernelGGL(copy_kernel<13>, grid, block, 0, 0, arena, n, stride, pay_off);
        else hipLaunchKernelGGL(copy_kernel<2>, grid, block, 0, 0, arena, n, stride, pay_off);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (r) total += ms;
    }
    if (hipGetLastError() != hipSuccess) return 2;
    printf("{\"mode\": %d, \"packets\": %u, \"stride\": %u, \"ms\": %.4f, \"alg_read_gb\": %.4f, \"alg_write_gb\": %.4f}\n",
           mode, n, stride, total / reps, n * (double)kPay / 1e9, n * (double)kPay / 1e9);
    hipFree(arena);
    return 0;
}
