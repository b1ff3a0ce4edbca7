// bar_probe.hip — can the host write device memory directly (fine-grained device memory mapped through the PCIe BAR),
// and what does a host -> GPU doorbell cost through it versus through pinned host memory?
//
// The packet server's doorbell and payload sit in pinned host memory today: the server polls them across PCIe (a
// read round trip per poll) and then reads the payload across PCIe.  If the host can post its writes straight into
// device memory, the server polls and reads local memory instead.  Measured here, one resident workgroup answering
// `rounds` doorbells (it exits by itself after 2 s at the latest):
//   host:  pinned host memory (coherent, mapped) doorbell, reply in pinned host memory
//   dev:   fine-grained device memory doorbell (host writes through the BAR), reply in pinned host memory
// Prints {"dev_host_access": bool, "host_us": median round trip, "dev_us": ...}.
// Build: hipcc -O2 --offload-arch=gfx950 bar_probe.hip -o bar_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

// thread 0 waits for bell == i (system scope), answers reply = i, for i = 1..rounds; 2-s bound
__global__ void responder(const unsigned *bell, unsigned *reply, unsigned rounds) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned i = 1; i <= rounds; i++) {
        while (__hip_atomic_load(bell, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != i) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) return;
        }
        __hip_atomic_store(reply, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double run(unsigned *bell, const unsigned *dev_bell, unsigned *reply, unsigned rounds) {
    *reply = 0;
    __atomic_store_n(bell, 0u, __ATOMIC_SEQ_CST);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(responder, dim3(1), dim3(64), 0, s, dev_bell, reply, rounds);
    CK(hipGetLastError());
    std::vector<double> us;
    auto spin = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - spin).count() < 0.05) {
    }
    for (unsigned i = 1; i <= rounds; i++) {
        const auto t = std::chrono::steady_clock::now();
        __atomic_store_n(bell, i, __ATOMIC_SEQ_CST);
        while (__atomic_load_n((volatile unsigned *)reply, __ATOMIC_ACQUIRE) != i) {
            if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count() > 0.5) {
                fprintf(stderr, "no reply at round %u\n", i);
                CK(hipStreamSynchronize(s));
                return -1;
            }
        }
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t).count());
    }
    CK(hipStreamSynchronize(s));
    CK(hipStreamDestroy(s));
    std::sort(us.begin(), us.end());
    return us[us.size() / 2];
}

int main() {
    unsigned *hbell = nullptr, *reply = nullptr, *dbell = nullptr;
    CK(hipHostMalloc((void **)&hbell, 64, hipHostMallocCoherent | hipHostMallocMapped));
    CK(hipHostMalloc((void **)&reply, 64, hipHostMallocCoherent | hipHostMallocMapped));
    const double host_us = run(hbell, hbell, reply, 2000);
    hipError_t e = hipExtMallocWithFlags((void **)&dbell, 4096, hipDeviceMallocFinegrained);
    hipPointerAttribute_t attr{};
    bool host_access = false;
    if (e == hipSuccess && hipPointerGetAttributes(&attr, dbell) == hipSuccess)
        host_access = attr.hostPointer != nullptr;
    printf("{\"host_us\": %.2f, \"finegrained_alloc\": %s, \"attr_type\": %d, \"host_pointer\": %s", host_us,
           e == hipSuccess ? "true" : "false", (int)attr.type, host_access ? "true" : "false");
    fflush(stdout);
    if (host_access) {
        unsigned *hp = (unsigned *)attr.hostPointer;
        const double dev_us = run(hp, dbell, reply, 2000);
        printf(", \"dev_us\": %.2f", dev_us);
    }
    printf("}\n");
    return 0;
}
