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

#include "../clay_amd/csrc/bitslice.hpp"  // dma16, lds_barrier, wait_vm_rt (LDS-DMA helpers)

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

// encode-like traffic mix: 5 reads per 2 writes (the (10,4) encode reads 10 chunks and writes 4)
template <int U, int B, int MODE>
__global__ __launch_bounds__(B) void k_mix_gs(const v4u *__restrict__ s, v4u *__restrict__ d, size_t n) {
    const size_t stride = size_t(gridDim.x) * B;
    size_t i = size_t(blockIdx.x) * B + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        v4u v[U][5];
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
            for (int k = 0; k < 5; k++) v[u][k] = s[i + u * stride + k * n];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const v4u w0 = v[u][0] ^ v[u][1] ^ v[u][2], w1 = v[u][3] ^ v[u][4] ^ v[u][0];
            if (MODE & 2) {
                __builtin_nontemporal_store(w0, d + i + u * stride);
                __builtin_nontemporal_store(w1, d + i + u * stride + n);
            } else {
                d[i + u * stride] = w0;
                d[i + u * stride + n] = w1;
            }
        }
    }
}

// LDS-DMA copy with role-split waves, one workgroup per CU (the encode's structure): 4 loader
// waves stream 16 KiB slots into an R-slot LDS ring with global_load_lds_dwordx4 and counted
// vmcnt waits; 8 writer waves read each landed slot (ds_read_b128) and store it.  Each XCD
// owns a contiguous region; its 32 workgroups take adjacent 16 KiB slots round robin.
template <int R, int MODE>
__global__ __launch_bounds__(768) void k_copy_dma(const uint8_t *__restrict__ s, uint8_t *__restrict__ d, size_t nbytes) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    using namespace clay::bs;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3, ns = gridDim.x >> 3;
    const size_t region = nbytes / 8, x0 = xcd * region;
    const uint32_t nslot_total = uint32_t(region / 16384);
    const uint32_t nsteps = nslot_total > slot ? (nslot_total - slot + ns - 1) / ns : 0;
    auto src_of = [&](uint32_t k) { return x0 + (size_t(slot) + size_t(k) * ns) * 16384; };
    if (wave < 4) {
        const uint32_t lds0 = lds_addr_of(smem);
        uint32_t issued = 0;
        auto issue = [&](uint32_t k) {
            const uint8_t *base = s + src_of(k);
#pragma unroll
            for (int j = 0; j < 4; j++)
                dma16(lds0 + (k % R) * 16384u + uint32_t(wave * 4 + j) * 1024u, base,
                      uint32_t(wave * 4 + j) * 1024u + uint32_t(lane) * 16u);
            issued++;
        };
        while (issued < nsteps && issued < uint32_t(R - 1)) issue(issued);
        for (uint32_t k = 0; k < nsteps; k++) {
            wait_vm_rt(int((issued - (k + 1)) * 4));
            lds_barrier();
            if (issued < nsteps && issued < k + uint32_t(R)) issue(issued);  // into slot (k-1) % R
        }
        return;
    }
    const int w = wave - 4;
    for (uint32_t k = 0; k < nsteps; k++) {
        lds_barrier();
        const uint8_t *sl = smem + (k % R) * 16384u;
        uint8_t *dst = d + src_of(k);
        const v4u a0 = *reinterpret_cast<const v4u *>(sl + w * 2048 + lane * 16);
        const v4u a1 = *reinterpret_cast<const v4u *>(sl + w * 2048 + 1024 + lane * 16);
        if (MODE & 2) {
            __builtin_nontemporal_store(a0, reinterpret_cast<v4u *>(dst + w * 2048 + lane * 16));
            __builtin_nontemporal_store(a1, reinterpret_cast<v4u *>(dst + w * 2048 + 1024 + lane * 16));
        } else {
            *reinterpret_cast<v4u *>(dst + w * 2048 + lane * 16) = a0;
            *reinterpret_cast<v4u *>(dst + w * 2048 + 1024 + lane * 16) = a1;
        }
    }
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
    // role-split LDS-DMA copy (loader + writer waves per CU, the encode's structure)
    int cus = 256;
    {
        hipDeviceProp_t pr;
        if (hipGetDeviceProperties(&pr, 0) == hipSuccess) cus = pr.multiProcessorCount;
    }
#define COPYDMA(R, MODE)                                                                                         \
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&k_copy_dma<R, MODE>),                              \
                           hipFuncAttributeMaxDynamicSharedMemorySize, R * 16384));                          \
    snprintf(nm, sizeof nm, "copy lds-dma R%d mode%d grid%d", R, MODE, cus);                                  \
    rep(nm, 2.0 * G, timeit([&] { k_copy_dma<R, MODE><<<cus, 768, R * 16384>>>(a, b, G); }));
    COPYDMA(4, 0)
    COPYDMA(8, 0)
    COPYDMA(9, 0)
    COPYDMA(8, 2)
    // the encode's traffic mix: 5 reads : 2 writes
    const size_t nm5 = G / 80;  // 5 * nm5 * 16 B = 1 GiB read, 2 * nm5 * 16 B written
#define MIX(U, B, MODE, GRID)                                                                                    \
    snprintf(nm, sizeof nm, "mix 5r:2w U%d B%d mode%d grid%d", U, B, MODE, GRID);                           \
    rep(nm, 7.0 * nm5 * 16, timeit([&] { k_mix_gs<U, B, MODE><<<GRID, B>>>((const v4u *)a, (v4u *)b, nm5); }));
    MIX(1, 256, 0, 8192)
    MIX(2, 256, 0, 4096)
    MIX(2, 256, 2, 4096)
    MIX(4, 256, 0, 2048)
    return 0;
}
