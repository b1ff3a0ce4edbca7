// Microbenchmark: wave64 issue cost of the single VALU instructions the kernels are made of (gfx950).
// 8 independent chains per lane, one instruction per chain step (checked in the ISA: hipcc --save-temps), 256-thread
// blocks, 8 blocks per CU.  Prints wave-instructions per ns chip-wide and cycles per wave-instruction per SIMD at
// the clock given on the command line (default 2.1 GHz, the clock this chip holds under load).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t *out, int iters, uint32_t seed) {
    uint32_t u[8];
    for (int i = 0; i < 8; i++) u[i] = seed * (i + 3) + threadIdx.x;
    const uint32_t c = seed | 0x10101u;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (OP == 0) u[i] = u[i] ^ (c + i);                                        // v_xor_b32
            if (OP == 1) u[i] = u[i] + (c + i);                                        // v_add_u32
            if (OP == 2) u[i] = __builtin_amdgcn_alignbit(u[i], u[i], 7);              // v_alignbit_b32 (rotate)
            if (OP == 3) u[i] = __builtin_amdgcn_bitop3_b32(u[i], c, c + i, 0x96);     // v_bitop3_b32 (xor3)
            if (OP == 4) u[i] = __builtin_amdgcn_perm(u[i], c + i, 0x05040100u);       // v_perm_b32
            if (OP == 5) u[i] = u[i] * (c + i);                                        // v_mul_lo_u32
        }
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; i++) s += u[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main(int argc, char **argv) {
    const double ghz = argc > 1 ? atof(argv[1]) : 2.1;
    uint32_t *out;
    hipMalloc(&out, 8 << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int bpc = argc > 2 ? atoi(argv[2]) : 8;  // 256-thread blocks per CU (2: 2 waves per SIMD)
    const int blocks = 256 * bpc, iters = 8192;
    const char *names[] = {"v_xor_b32", "v_add_u32", "v_alignbit_b32", "v_bitop3_b32", "v_perm_b32", "v_mul_lo_u32"};
    for (int op = 0; op < 6; op++) {
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(e0);
            switch (op) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u); break;
                case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u); break;
                case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u); break;
                default: hipLaunchKernelGGL(k<5>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u); break;
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double wi = (double)blocks * 4 * iters * 8;  // 4 waves per block, 8 instructions per iteration
            const double per_ns = wi / (ms * 1e6);
            if (rep == 2)
                printf("bpc %d %-16s %.3f ms  %.0f wave-instr/ns chip-wide  %.2f cycles/wave-instr/SIMD at %.2f GHz\n", bpc, names[op],
                       ms, per_ns, 1024.0 * ghz / per_ns, ghz);
        }
    }
    return 0;
}
