// bw_probe.hip -- what streaming HBM rate does this MI355X reach for read, write and copy?
// Calibrates the "measured ceiling" that DESIGN.md reports the encode fraction against
// (the guide quotes 6.29 TB/s for a float4 copy).  Variants: grid-stride vs per-block
// contiguous, unroll depth, block size, non-temporal loads / stores, hipMemcpyDtoD.
// Build: hipcc --offload-arch=gfx950 -O3 -o bench_tools/bw_probe bench_tools/bw_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
#define CK(x)                                                            \
    do {                                                                 \
        hipError_t e_ = (x);                                             \
        if (e_ != hipSuccess) {                                          \
            printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); \
            return 1;                                                    \
        }                                                                \
    } while (0)

// MODE bit0: nt loads, bit1: nt stores
template <int U, int B, int MODE>
__global__ __launch_bounds__(B) void k_copy_gs(const v4u *__restrict__ s, v4u *__restrict__ d, size_t n) {
    const size_t stride = size_t(gridDim.x) * B;
    size_t i = size_t(blockIdx.x) * B + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = (MODE & 1) ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (MODE & 2) __builtin_nontemporal_store(v[u], d + i + u * stride);
            else d[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride) d[i] = s[i];
}

// each block copies one contiguous range
template <int U, int B, int MODE>
__global__ __launch_bounds__(B) void k_copy_blk(const v4u *__restrict__ s, v4u *__restrict__ d, size_t n) {
    const size_t per = (n + gridDim.x - 1) / gridDim.x;
    const size_t lo = size_t(blockIdx.x) * per, hi = std::min(lo + per, n);
    size_t i = lo + threadIdx.x;
    for (; i + (U - 1) * B < hi; i += U * B) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = (MODE & 1) ? __builtin_nontemporal_load(s + i + u * B) : s[i + u * B];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (MODE & 2) __builtin_nontemporal_store(v[u], d + i + u * B);
            else d[i + u * B] = v[u];
        }
    }
    for (; i < hi; i += B) d[i] = s[i];
}

template <int U, int B, int MODE>
__global__ __launch_bounds__(B) void k_read_gs(const v4u *__restrict__ s, size_t n, uint32_t *sink) {
    const size_t stride = size_t(gridDim.x) * B;
    size_t i = size_t(blockIdx.x) * B + threadIdx.x;
    uint32_t acc = 0;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = (MODE & 1) ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u].x ^ v[u].w;
    }
    for (; i < n; i += stride) acc ^= s[i].y;
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

template <int U, int B, int MODE>
__global__ __launch_bounds__(B) void k_write_gs(v4u *__restrict__ d, size_t n) {
    const size_t stride = size_t(gridDim.x) * B;
    size_t i = size_t(blockIdx.x) * B + threadIdx.x;
    const v4u v = v4u{uint32_t(i), 1u, 2u, 3u};
    for (; i + (U - 1) * stride < n; i += U * stride) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (MODE & 2) __builtin_nontemporal_store(v, d + i + u * stride);
            else d[i + u * stride] = v;
        }
    }
    for (; i < n; i += stride) d[i] = v;
}

template <class F>
static float timeit(F &&launch, int reps = 14) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> t;
    for (int r = 0; r < reps; r++) {
        (void)hipEventRecord(e0);
        launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r >= 4) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    const size_t G = size_t(1) << 30;
    uint8_t *a, *b;
    uint32_t *sink;
    CK(hipMalloc(&a, 2 * G));
    CK(hipMalloc(&b, 2 * G));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, 2 * G));
    CK(hipMemset(b, 2, 2 * G));
    auto rep = [&](const char *name, double bytes, float ms) {
        printf("%-40s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    const size_t n = G / 16;
    for (int i = 0; i < 200; i++) k_copy_gs<4, 256, 0><<<4096, 256>>>((const v4u *)a, (v4u *)b, n);
    (void)hipDeviceSynchronize();
    char nm[96];
#define COPY(U, B, MODE, GRID)                                                                                   \
    snprintf(nm, sizeof nm, "copy gs U%d B%d mode%d grid%d", U, B, MODE, GRID);                             \
    rep(nm, 2.0 * G, timeit([&] { k_copy_gs<U, B, MODE><<<GRID, B>>>((const v4u *)a, (v4u *)b, n); }));
#define COPYB(U, B, MODE, GRID)                                                                                  \
    snprintf(nm, sizeof nm, "copy blk U%d B%d mode%d grid%d", U, B, MODE, GRID);                            \
    rep(nm, 2.0 * G, timeit([&] { k_copy_blk<U, B, MODE><<<GRID, B>>>((const v4u *)a, (v4u *)b, n); }));
    COPY(1, 256, 0, 16384)
    COPY(2, 256, 0, 4096)
    COPY(4, 256, 0, 2048)
    COPY(8, 256, 0, 1024)
    COPY(4, 512, 0, 1024)
    COPY(4, 1024, 0, 512)
    COPY(4, 256, 1, 2048)
    COPY(4, 256, 2, 2048)
    COPY(4, 256, 3, 2048)
    COPY(1, 256, 2, 16384)
    COPYB(4, 256, 0, 2048)
    COPYB(4, 512, 0, 1024)
    COPYB(8, 512, 0, 512)
    COPYB(4, 256, 2, 2048)
    rep("hipMemcpyDtoD 1 GiB", 2.0 * G, timeit([&] { (void)hipMemcpyAsync(b, a, G, hipMemcpyDeviceToDevice, 0); }));
    // 256 MiB copy (fits the Infinity Cache) for comparison
    rep("copy gs U4 256MiB (MALL-resident)", 0.5 * G,
        timeit([&] { k_copy_gs<4, 256, 0><<<2048, 256>>>((const v4u *)a, (v4u *)b, n / 4); }));
#define READ(U, B, MODE, GRID)                                                                                   \
    snprintf(nm, sizeof nm, "read gs 2GiB U%d B%d mode%d grid%d", U, B, MODE, GRID);                        \
    rep(nm, 2.0 * G, timeit([&] { k_read_gs<U, B, MODE><<<GRID, B>>>((const v4u *)a, 2 * n, sink); }));
    READ(4, 256, 0, 4096)
    READ(8, 256, 0, 4096)
    READ(8, 256, 0, 8192)
    READ(16, 256, 0, 2048)
    READ(8, 256, 1, 4096)
#define WRITE(U, B, MODE, GRID)                                                                                  \
    snprintf(nm, sizeof nm, "write gs 2GiB U%d B%d mode%d grid%d", U, B, MODE, GRID);                       \
    rep(nm, 2.0 * G, timeit([&] { k_write_gs<U, B, MODE><<<GRID, B>>>((v4u *)b, 2 * n); }));
    WRITE(4, 256, 0, 4096)
    WRITE(8, 256, 0, 2048)
    WRITE(4, 256, 2, 4096)
    rep("hipMemsetAsync 2 GiB", 2.0 * G, timeit([&] { (void)hipMemsetAsync(b, 3, 2 * G, 0); }));
    return 0;
}
