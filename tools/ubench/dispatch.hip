// dispatch.hip — fixed cost of a launch by workgroup shape: every workgroup spins until s_memrealtime has advanced by
// T ticks (100 MHz), so event time - T/100 MHz is what the launch adds (LDS allocation, wave launch, drain).
#include <hip/hip_runtime.h>
#include <stdio.h>
template <int WG>
__global__ __launch_bounds__(WG) void spin(uint64_t ticks, uint64_t *out) {
    extern __shared__ uint32_t lds[];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t t = t0;
    while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) out[blockIdx.x] = t - t0 + lds[0] * 0;
}
int main() {
    uint64_t *out;
    hipMalloc(&out, 1 << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (uint64_t ticks : {1000ull, 100000ull}) {
        for (int wg : {256, 512, 1024}) {
            for (int lds : {0, 65536, 163840}) {
                float best = 1e9;
                for (int rep = 0; rep < 4; rep++) {
                    hipEventRecord(e0);
                    if (wg == 256) hipLaunchKernelGGL(spin<256>, dim3(256), dim3(wg), lds, 0, ticks, out);
                    if (wg == 512) hipLaunchKernelGGL(spin<512>, dim3(256), dim3(wg), lds, 0, ticks, out);
                    if (wg == 1024) hipLaunchKernelGGL(spin<1024>, dim3(256), dim3(wg), lds, 0, ticks, out);
                    hipEventRecord(e1);
                    hipEventSynchronize(e1);
                    float ms;
                    hipEventElapsedTime(&ms, e0, e1);
                    if (rep && ms < best) best = ms;
                }
                printf("spin %6llu ticks (%.3f ms at 100 MHz)  wg %4d  lds %6d: event %.3f ms  (+%.1f us)\n",
                       (unsigned long long)ticks, ticks / 1e5, wg, lds, best, (best - ticks / 1e5) * 1e3);
            }
        }
    }
    return 0;
}
