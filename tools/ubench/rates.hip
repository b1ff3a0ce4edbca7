// Microbenchmark: issue rate of v_mad_u64_u32 vs v_fma_f64 vs v_mul_lo_u32 vs v_add_u32 on gfx950 (8 independent
// chains per lane, 1024-thread blocks, 4 blocks per CU).  Prints ns per wave-instruction per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int OP>
__global__ __launch_bounds__(256) void k(uint64_t *out, int iters, uint32_t seed) {
    uint64_t a[8];
    double f[8];
    uint32_t u[8];
    for (int i = 0; i < 8; i++) { a[i] = seed + i + threadIdx.x; f[i] = (double)(seed + i); u[i] = seed * (i + 3) + threadIdx.x; }
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if (OP == 0) a[i] = (uint64_t)(uint32_t)a[i] * (uint32_t)(a[i] >> 7) + a[i];   // v_mad_u64_u32
            if (OP == 1) f[i] = __builtin_fma(f[i], 1.0000001, 0.5);                      // v_fma_f64
            if (OP == 2) u[i] = u[i] * (u[i] | 1u) + 7u;                                   // v_mul_lo_u32 (+add)
            if (OP == 3) u[i] = (u[i] + 0x9e3779b9u) ^ (u[i] >> 3);                        // add + xor (2 ops)
        }
    }
    uint64_t s = 0;
    for (int i = 0; i < 8; i++) s += a[i] + (uint64_t)f[i] + u[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
    uint64_t *out;
    hipMalloc(&out, 8 << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int blocks = 256 * 8, iters = 4096;
    const char *names[] = {"v_mad_u64_u32 (+add64)", "v_fma_f64", "v_mul_lo_u32 (+add)", "v_add_u32+v_xor"};
    for (int op = 0; op < 4; op++) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(e0);
            if (op == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u);
            if (op == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u);
            if (op == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u);
            if (op == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters, 3u);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double wave_instr = (double)blocks * 4 * iters * 8;  // 4 waves per block, 8 ops per iteration
            if (rep) printf("%-24s %.3f ms  -> %.2f wave-instr/ns chip-wide (%.3f per CU per ns)\n", names[op], ms,
                            wave_instr / (ms * 1e6), wave_instr / (ms * 1e6) / 256);
        }
    }
    return 0;
}
