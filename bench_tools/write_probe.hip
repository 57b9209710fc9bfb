// write_probe.hip -- how fast can the encode's parity writes go?  The parity of a
// (10,4,13) 1 GiB stripe is 4 chunks x 256 rows (layers) of sc = 419,432 bytes.
//   A: tile order (the encode's): tile = W bytes of all 1,024 rows; each store
//      instruction writes (1024 / W) rows x W bytes; tiles dealt per XCD (v6 map)
//   B: row runs: each workgroup step writes R contiguous bytes of one row
//   C: contiguous (memset-like) over the 4 parity chunks
// Build: hipcc --offload-arch=gfx950 -O3 -o bench_tools/write_probe bench_tools/write_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int POL>
__device__ __forceinline__ void stp(void *p, v4u v);
// ASG 0: per-XCD regions (v6/stream map), 1: global round robin
template <int W, int NT, int POL = 0, int ASG = 0>
__global__ __launch_bounds__(512) void k_tile_order(uint8_t *par, uint32_t sc, uint64_t chunk) {
    const uint32_t ntiles = (sc + W - 1) / W, tpx = (ntiles + 7) / 8, nsl = gridDim.x / 8, b = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int RPI = 1024 / W;
    const int lr = lane / (W / 16), lof = (lane % (W / 16)) * 16;
    const uint32_t nt_loop = ASG == 0 ? tpx : ntiles;
    for (uint32_t t = ASG == 0 ? (b >> 3) : b; t < nt_loop && (ASG == 1 || (b & 7) * tpx + t < ntiles); t += ASG == 0 ? nsl : gridDim.x) {
        const uint32_t b0 = (ASG == 0 ? ((b & 7) * tpx + t) : t) * W;
        if (b0 + W > sc) continue;
        for (int i = 0; i < 1024 / RPI / 8; i++) {
            const int row = (wave * (1024 / RPI / 8) + i) * RPI + lr;
            uint8_t *p = par + uint64_t(row >> 8) * chunk + uint64_t(row & 255) * sc + b0 + lof;
            const v4u v = {uint32_t(row), b0, 1u, 2u};
            if (NT) __builtin_nontemporal_store(v, reinterpret_cast<v4u *>(p));
            else if (POL) stp<POL>(p, v);
            else *reinterpret_cast<v4u *>(p) = v;
        }
    }
}

// B: a workgroup step = 8 KiB of one row (8 waves x 1 KiB), steps dealt round robin
__global__ __launch_bounds__(512) void k_row_runs(uint8_t *par, uint32_t sc, uint64_t chunk) {
    const uint32_t runs_per_row = sc / 8192, nsteps = 1024 * runs_per_row;
    for (uint32_t s = blockIdx.x; s < nsteps; s += gridDim.x) {
        const uint32_t row = s / runs_per_row, run = s % runs_per_row;
        uint8_t *p = par + uint64_t(row >> 8) * chunk + uint64_t(row & 255) * sc + run * 8192 + threadIdx.x * 16;
        *reinterpret_cast<v4u *>(p) = v4u{row, run, 1u, 2u};
    }
}

// POL: 0 plain, 1 nt, 2 sc0, 3 sc1, 4 sc0 sc1, 5 sc0 nt, 6 sc1 nt, 7 sc0 sc1 nt
template <int POL>
__device__ __forceinline__ void stp(void *p, v4u v) {
    if (POL == 8) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
    if (POL == 0) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
    if (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    if (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
    if (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    if (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    if (POL == 5) asm volatile("global_store_dwordx4 %0, %1, off sc0 nt" ::"v"(p), "v"(v) : "memory");
    if (POL == 6) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    if (POL == 7) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}
template <int POL = 0, int U = 1>
__global__ __launch_bounds__(512) void k_contig(uint8_t *par, uint64_t bytes) {
    const uint64_t per = (bytes / 16 + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = uint64_t(blockIdx.x) * per, hi = std::min(lo + per, bytes / 16);
    uint64_t i = lo + threadIdx.x;
    for (; i + (U - 1) * 512 < hi; i += 512 * U)
#pragma unroll
        for (int u = 0; u < U; u++) stp<POL>(reinterpret_cast<v4u *>(par) + i + u * 512, v4u{uint32_t(i), 1u, 2u, 3u});
    for (; i < hi; i += 512) stp<POL>(reinterpret_cast<v4u *>(par) + i, v4u{uint32_t(i), 1u, 2u, 3u});
}
// lane writes 64 contiguous bytes (4 stores), wave covers 4 KiB
template <int POL = 0>
__global__ __launch_bounds__(512) void k_contig64(uint8_t *par, uint64_t bytes) {
    const uint64_t n64 = bytes / 64;
    const uint64_t per = (n64 + gridDim.x - 1) / gridDim.x;
    const uint64_t lo = uint64_t(blockIdx.x) * per, hi = std::min(lo + per, n64);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += 512)
#pragma unroll
        for (int u = 0; u < 4; u++) stp<POL>(par + i * 64 + u * 16, v4u{uint32_t(i), 1u, 2u, 3u});
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
    const uint32_t sc = 419432;
    const uint64_t chunk = uint64_t(sc) * 256;
    uint8_t *par;
    if (hipMalloc(&par, 4 * chunk) != hipSuccess) return 1;
    (void)hipMemset(par, 0, 4 * chunk);
    const double bytes = 4.0 * chunk;
    auto rep = [&](const char *name, float ms) {
        printf("%-36s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    for (int i = 0; i < 400; i++) k_contig<><<<2048, 512>>>(par, uint64_t(4 * chunk));
    (void)hipDeviceSynchronize();
    for (int rr = 0; rr < 2; rr++) {
        rep("A W256 asg0 plain", timeit([&] { k_tile_order<256, 0, 0, 0><<<256, 512>>>(par, sc, chunk); }));
        rep("A W256 asg1 plain", timeit([&] { k_tile_order<256, 0, 0, 1><<<256, 512>>>(par, sc, chunk); }));
        rep("A W256 asg0 sc0", timeit([&] { k_tile_order<256, 0, 2, 0><<<256, 512>>>(par, sc, chunk); }));
        rep("A W256 asg0 sc1", timeit([&] { k_tile_order<256, 0, 3, 0><<<256, 512>>>(par, sc, chunk); }));
        rep("A W256 asg0 sc0sc1", timeit([&] { k_tile_order<256, 0, 4, 0><<<256, 512>>>(par, sc, chunk); }));
        rep("A W256 asg0 sc0sc1nt", timeit([&] { k_tile_order<256, 0, 7, 0><<<256, 512>>>(par, sc, chunk); }));
        rep("A W256 asg0 sc1nt", timeit([&] { k_tile_order<256, 0, 6, 0><<<256, 512>>>(par, sc, chunk); }));
        rep("A W1024 asg0 plain", timeit([&] { k_tile_order<1024, 0, 0, 0><<<256, 512>>>(par, sc, chunk); }));
        rep("A W1024 asg1 plain", timeit([&] { k_tile_order<1024, 0, 0, 1><<<256, 512>>>(par, sc, chunk); }));
        rep("A W1024 asg0 sc1", timeit([&] { k_tile_order<1024, 0, 3, 0><<<256, 512>>>(par, sc, chunk); }));
        rep("hipMemsetAsync", timeit([&] { (void)hipMemsetAsync(par, 3, 4 * chunk, 0); }));
    }
    return 0;
}
