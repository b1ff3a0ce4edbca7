// free_sync.hip — which HIP free calls wait for a resident (persistent) kernel on ANOTHER stream?
//
// api.cpp stops a context's resident servers before every hipFree / hipHostFree (quiet_for_free), because those calls
// wait for every stream of the device.  With several contexts per process, one context's free would also wait for
// another context's server, which leaves only when idle.  This program measures each free form beside a bounded
// resident kernel (it spins on a host-mapped stop word and exits by itself after 2 s at the latest):
//   hipFree, hipHostFree, hipFreeAsync (memory from hipMallocAsync) + hipStreamSynchronize of its own stream,
//   hipMallocAsync, hipHostUnregister (of malloc'd memory hipHostRegister'ed), hipStreamDestroy / hipEventDestroy of
//   idle ones, hipHostMalloc, hipMalloc.
// A call that takes ~2 s waited for the resident kernel.
// Build: hipcc -O2 --offload-arch=gfx950 free_sync.hip -o free_sync
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

// one workgroup: thread 0 polls the stop word (system scope) until it is set or 2 s (s_memrealtime, 100 MHz) passed
__global__ void resident(const volatile unsigned *stop, unsigned *out) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned n = 0;
    while (__hip_atomic_load(stop, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;
        __builtin_amdgcn_s_sleep(32);
        n++;
    }
    out[0] = n;
}

static double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main() {
    hipStream_t srv, other;
    CK(hipStreamCreateWithFlags(&srv, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&other, hipStreamNonBlocking));
    unsigned *stop = nullptr, *out = nullptr;
    CK(hipHostMalloc((void **)&stop, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipMalloc((void **)&out, 64));
    const char *names[] = {"hipFree", "hipHostFree", "hipFreeAsync+streamsync", "hipMallocAsync+streamsync",
                           "hipHostUnregister", "hipStreamDestroy", "hipEventDestroy", "hipHostMalloc", "hipMalloc"};
    printf("{");
    for (int form = 0; form < 9; form++) {
        void *d = nullptr, *h = nullptr, *a = nullptr, *reg = aligned_alloc(4096, 1 << 20), *h2 = nullptr, *d2 = nullptr;
        CK(hipHostRegister(reg, 1 << 20, hipHostRegisterDefault));
        hipStream_t idle;
        hipEvent_t ev;
        CK(hipStreamCreateWithFlags(&idle, hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        CK(hipMalloc(&d, 1 << 20));
        CK(hipHostMalloc(&h, 1 << 20, hipHostMallocDefault));
        CK(hipMallocAsync(&a, 1 << 20, other));
        CK(hipStreamSynchronize(other));
        *stop = 0;
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        hipLaunchKernelGGL(resident, dim3(1), dim3(64), 0, srv, stop, out);
        CK(hipGetLastError());
        // let the kernel start
        const auto tw = std::chrono::steady_clock::now();
        while (ms_since(tw) < 50) {
        }
        const auto t = std::chrono::steady_clock::now();
        void *a2 = nullptr;
        if (form == 0) CK(hipFree(d));
        if (form == 1) CK(hipHostFree(h));
        if (form == 2) {
            CK(hipFreeAsync(a, other));
            CK(hipStreamSynchronize(other));
        }
        if (form == 3) {
            CK(hipMallocAsync(&a2, 1 << 21, other));
            CK(hipStreamSynchronize(other));
        }
        if (form == 4) CK(hipHostUnregister(reg));
        if (form == 5) CK(hipStreamDestroy(idle));
        if (form == 6) CK(hipEventDestroy(ev));
        if (form == 7) CK(hipHostMalloc(&h2, 1 << 20, hipHostMallocDefault));
        if (form == 8) CK(hipMalloc(&d2, 1 << 20));
        const double dt = ms_since(t);
        __atomic_store_n(stop, 1u, __ATOMIC_SEQ_CST);
        CK(hipStreamSynchronize(srv));
        printf("%s\"%s_ms\": %.2f", form ? ", " : "", names[form], dt);
        if (form != 0) CK(hipFree(d));
        if (form != 1) CK(hipHostFree(h));
        if (form != 2) CK(hipFreeAsync(a, other));
        if (a2) CK(hipFreeAsync(a2, other));
        CK(hipStreamSynchronize(other));
        if (form != 4) CK(hipHostUnregister(reg));
        free(reg);
        if (form != 5) CK(hipStreamDestroy(idle));
        if (form != 6) CK(hipEventDestroy(ev));
        if (h2) CK(hipHostFree(h2));
        if (d2) CK(hipFree(d2));
    }
    printf("}\n");
    CK(hipFree(out));
    CK(hipHostFree(stop));
    return 0;
}
