// bar_probe.hip — can the host write device memory directly (fine-grained device memory mapped through the PCIe BAR),
// and what does a host -> GPU doorbell cost through it versus through pinned host memory?
//
// The packet server's doorbell and payload sit in pinned host memory today: the server polls them across PCIe (a
// read round trip per poll) and then reads the payload across PCIe.  If the host can post its writes straight into
// device memory, the server polls and reads local memory instead.  Measured here, one resident workgroup answering
// `rounds` doorbells (it exits by itself after 2 s at the latest):
//   host:  pinned host memory (coherent, mapped) doorbell, reply in pinned host memory
//   dev:   fine-grained device memory doorbell (host writes through the BAR), reply in pinned host memory
//   data:  the answer preceded by a 16-byte data store to pinned memory (the server's result + done order: data,
//          then a system-scope release store of the done word, which waits for the data store's acknowledgement)
//   one:   the answer and 12 bytes of data in ONE 16-byte store (an NVMe-style completion entry: no ordering wait)
//   order: 1216 bytes of data (64 lanes, plain 16-byte stores), s_waitcnt vmcnt(0), then a PLAIN store of the answer
//          (no release fence: no L2 write-back); the host checks every data byte as soon as it sees the answer --
//          whether the acknowledgement alone orders stores to coherent pinned memory (mismatches counted)
//   fenced: the same 1216 bytes, then the server's completion as it is (release fence + system-scope release store)
// Prints {"host_us": median round trip, "data_us": ..., "one_us": ..., "finegrained_alloc": ..., ...}.
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

// mode 1: a 16-byte data store, then the release store of the answer; mode 2: the answer inside one 16-byte store
__global__ void responder_data(const unsigned *bell, unsigned *reply, unsigned *data, unsigned rounds, int mode) {
    if (threadIdx.x != 0) return;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned i = 1; i <= rounds; i++) {
        while (__hip_atomic_load(bell, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != i) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) return;
        }
        if (mode == 1) {
            *(volatile u32x4 *)data = u32x4{i, i + 1, i + 2, i + 3};
            __hip_atomic_store(reply, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
            *(volatile u32x4 *)reply = u32x4{i, i + 1, i + 2, i + 3};
        }
    }
}

// 64 lanes store 19 x 16 B of pattern i, wait for their acknowledgements, lane 0 stores the answer plainly
__global__ void responder_order(const unsigned *bell, unsigned *reply, unsigned *data, unsigned rounds, int fence) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const unsigned lane = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned i = 1; i <= rounds; i++) {
        while (__hip_atomic_load(bell, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != i) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) return;
        }
        for (unsigned k = lane; k < 76; k += 64) {
            const unsigned v = i * 131u + k;
            *(volatile u32x4 *)(data + 4 * k) = u32x4{v, v ^ 1u, v ^ 2u, v ^ 3u};
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {
            if (fence) {  // the server's completion today: release fence, then a system-scope release store
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                __hip_atomic_store(reply, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
                *(volatile unsigned *)reply = i;
            }
        }
    }
}
static unsigned order_bad = 0;

static double run(unsigned *bell, const unsigned *dev_bell, unsigned *reply, unsigned rounds, int mode = 0,
                  unsigned *data = nullptr) {
    *reply = 0;
    __atomic_store_n(bell, 0u, __ATOMIC_SEQ_CST);
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    if (mode == 0) hipLaunchKernelGGL(responder, dim3(1), dim3(64), 0, s, dev_bell, reply, rounds);
    else if (mode == 3 || mode == 4)
        hipLaunchKernelGGL(responder_order, dim3(1), dim3(64), 0, s, dev_bell, reply, data, rounds, mode == 4 ? 1 : 0);
    else hipLaunchKernelGGL(responder_data, dim3(1), dim3(64), 0, s, dev_bell, reply, data, rounds, mode);
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
        if (mode == 3 || mode == 4)
            for (unsigned k = 0; k < 76; k++) {
                const unsigned v = i * 131u + k;
                const volatile unsigned *d = data + 4 * k;
                if (d[0] != v || d[1] != (v ^ 1u) || d[2] != (v ^ 2u) || d[3] != (v ^ 3u)) order_bad++;
            }
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
    unsigned *data = nullptr;
    CK(hipHostMalloc((void **)&data, 64, hipHostMallocCoherent | hipHostMallocMapped));
    const double data_us = run(hbell, hbell, reply, 2000, 1, data);
    const double one_us = run(hbell, hbell, reply, 2000, 2, data);
    unsigned *big = nullptr;
    CK(hipHostMalloc((void **)&big, 76 * 16, hipHostMallocCoherent | hipHostMallocMapped));
    const double order_us = run(hbell, hbell, reply, 200000, 3, big);
    const double fenced_us = run(hbell, hbell, reply, 20000, 4, big);
    hipError_t e = hipExtMallocWithFlags((void **)&dbell, 4096, hipDeviceMallocFinegrained);
    hipPointerAttribute_t attr{};
    bool host_access = false;
    if (e == hipSuccess && hipPointerGetAttributes(&attr, dbell) == hipSuccess)
        host_access = attr.hostPointer != nullptr;
    printf("{\"host_us\": %.2f, \"data_us\": %.2f, \"one_us\": %.2f, \"order_us\": %.2f, \"fenced_us\": %.2f, \"order_rounds\": 200000, \"order_mismatched_16B\": %u, \"finegrained_alloc\": %s, \"attr_type\": %d, \"host_pointer\": %s", host_us, data_us, one_us, order_us, fenced_us, order_bad,
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
