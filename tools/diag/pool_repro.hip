// pool_repro.hip — standalone check of the stream-ordered allocator in the pattern the round-5 fuzz failure came from
// (tests/test_gpu_fuzz.py corrupted batch buffers in page-sized runs with hipMallocAsync / hipFreeAsync,
// 8 of 44 seeds, and not with hipMalloc / hipFree: profiles/r05/r05v/fuzzab.txt).
//
// The library's allocator of that build (commit b8eef59, api.cpp dmalloc / dfree), reproduced without the library:
//   dmalloc: hipMallocAsync on an allocation stream, then hipStreamSynchronize of that stream;
//   dfree:   an event recorded on every stream of the context, the allocation stream waits for each, hipFreeAsync on it.
// What the fuzz did with such a buffer, also reproduced:
//   upload:  hipMemcpyAsync from PAGEABLE host memory (a numpy array) on the context stream, then synchronize it;
//   batch:   an in-place kernel on another stream (the fuzz's "side" stream) that rewrites every byte (x -> f(x));
//   check:   synchronize every stream, hipMemcpyAsync device -> pageable host, compare every byte with f(pattern).
// Buffers live for a random number of steps (several in flight, sizes 64 KiB .. 16 MiB as the fuzz's arenas), so the
// pool recycles blocks while other buffers' uploads and kernels are in flight.
//
// usage: pool_repro [mode] [steps] [seed]   mode: async (hipMallocAsync / hipFreeAsync, as b8eef59) | sync (hipMalloc
// / hipFree, the shipped build) | async_pinned (async allocator, pinned host staging instead of pageable) | async_keep
// (async allocator, the default pool's release threshold at UINT64_MAX: it never gives memory back at a synchronize).  Prints one
// line per corrupted buffer (first bad byte, run length, the allocation's step and size) and a summary; exit 1 when
// any byte is wrong.
//
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/diag/pool_repro.hip -o tools/diag/pool_repro
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                           \
        }                                                                                      \
    } while (0)

__device__ __host__ inline uint8_t fbyte(uint8_t x, uint32_t salt) { return (uint8_t)((x ^ salt) * 167u + 13u); }

// the "seal": every byte rewritten in place, 16 B per lane per step (as the batch kernels do)
__global__ void rewrite(uint8_t *p, size_t n, uint32_t salt) {
    const size_t stride = (size_t)gridDim.x * blockDim.x * 16;
    for (size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; i < n; i += stride) {
        const size_t m = n - i < 16 ? n - i : 16;
        for (size_t j = 0; j < m; j++) p[i + j] = fbyte(p[i + j], salt);
    }
}

struct Buf {
    uint8_t *d = nullptr;
    size_t n = 0;
    int born = 0, dies = 0;
    uint32_t salt = 0;
    std::vector<uint8_t> want;
};

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "async";
    const int steps = argc > 2 ? atoi(argv[2]) : 400;
    const uint32_t seed = argc > 3 ? (uint32_t)strtoul(argv[3], nullptr, 0) : 0xF025u;
    const bool async = strncmp(mode, "async", 5) == 0, pinned = strcmp(mode, "async_pinned") == 0;
    std::mt19937_64 rng(seed);
    hipStream_t ctx, side, astream;
    CK(hipStreamCreateWithFlags(&ctx, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&astream, hipStreamNonBlocking));
    const hipStream_t all[] = {ctx, side};
    std::vector<hipEvent_t> evs(2);
    for (auto &e : evs) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (strcmp(mode, "async_keep") == 0) {
        hipMemPool_t pool;
        CK(hipDeviceGetDefaultMemPool(&pool, 0));
        uint64_t thr = UINT64_MAX;
        CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
    }
    uint8_t *stage = nullptr;
    if (pinned) CK(hipHostMalloc(&stage, 16u << 20, hipHostMallocDefault));
    auto dmalloc = [&](size_t n) {
        uint8_t *p = nullptr;
        if (async) {
            CK(hipMallocAsync((void **)&p, n, astream));
            CK(hipStreamSynchronize(astream));
        } else {
            CK(hipMalloc((void **)&p, n));
        }
        return p;
    };
    auto dfree = [&](uint8_t *p) {
        if (async) {
            for (int i = 0; i < 2; i++) {
                CK(hipEventRecord(evs[i], all[i]));
                CK(hipStreamWaitEvent(astream, evs[i], 0));
            }
            CK(hipFreeAsync(p, astream));
        } else {
            CK(hipFree(p));
        }
    };
    std::vector<Buf> live;
    long bad_bufs = 0, bad_bytes = 0, checked = 0;
    std::vector<uint8_t> host, got;
    auto check = [&](Buf &b) {
        for (hipStream_t s : all) CK(hipStreamSynchronize(s));
        got.resize(b.n);
        CK(hipMemcpyAsync(got.data(), b.d, b.n, hipMemcpyDeviceToHost, ctx));
        CK(hipStreamSynchronize(ctx));
        checked++;
        size_t first = SIZE_MAX, last = 0, cnt = 0;
        for (size_t i = 0; i < b.n; i++)
            if (got[i] != b.want[i]) {
                if (first == SIZE_MAX) first = i;
                last = i;
                cnt++;
            }
        if (cnt) {
            bad_bufs++;
            bad_bytes += (long)cnt;
            printf("CORRUPT buffer born step %d size %zu: %zu bytes wrong in [%zu, %zu] (run %zu), dev %p, first bad VA %p"
                   " (offset %#zx in its 2 MiB page)\n", b.born, b.n, cnt, first, last, last - first + 1, (void *)b.d,
                   (void *)(b.d + first), (size_t)(uintptr_t)(b.d + first) & ((2u << 20) - 1));
        }
    };
    for (int step = 0; step < steps; step++) {
        // retire the buffers whose time has come: check, then free
        for (size_t i = 0; i < live.size();) {
            if (live[i].dies <= step) {
                check(live[i]);
                dfree(live[i].d);
                live.erase(live.begin() + (long)i);
            } else {
                i++;
            }
        }
        // a new batch buffer: size as the fuzz arenas (1 .. 20000 packets of up to ~1.4 KB)
        const size_t sizes[] = {64u << 10, 300u << 10, 3u << 20, 7u << 20, 14u << 20};
        Buf b;
        b.n = sizes[rng() % 5] + (rng() % 65536);
        b.born = step;
        b.dies = step + 1 + (int)(rng() % 6);
        b.salt = (uint32_t)rng();
        b.d = dmalloc(b.n);
        host.resize(b.n);
        for (size_t i = 0; i < b.n; i += 8) {
            const uint64_t v = rng();
            memcpy(&host[i], &v, std::min<size_t>(8, b.n - i));
        }
        // upload from pageable memory on the context stream, synchronized (DeviceBuffer.upload)
        if (pinned) {
            memcpy(stage, host.data(), b.n);
            CK(hipMemcpyAsync(b.d, stage, b.n, hipMemcpyHostToDevice, ctx));
        } else {
            CK(hipMemcpyAsync(b.d, host.data(), b.n, hipMemcpyHostToDevice, ctx));
        }
        CK(hipStreamSynchronize(ctx));
        // the in-place batch on the side stream or the context stream (half each)
        const hipStream_t s = (rng() & 1) ? side : ctx;
        hipLaunchKernelGGL(rewrite, dim3(1024), dim3(256), 0, s, b.d, b.n, b.salt);
        CK(hipGetLastError());
        b.want.resize(b.n);
        for (size_t i = 0; i < b.n; i++) b.want[i] = fbyte(host[i], b.salt);
        live.push_back(std::move(b));
    }
    for (Buf &b : live) {
        check(b);
        dfree(b.d);
    }
    for (hipStream_t s : {ctx, side, astream}) CK(hipStreamSynchronize(s));
    printf("mode %s seed %#x steps %d: %ld buffers checked, %ld corrupted, %ld bytes wrong\n", mode, seed, steps, checked,
           bad_bufs, bad_bytes);
    return bad_bufs ? 1 : 0;
}
