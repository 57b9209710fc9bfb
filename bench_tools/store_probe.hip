// store_probe.hip -- why does hipMemsetAsync write HBM at ~6.5 TB/s while our store kernels
// top out at 3.8-5.3 TB/s?  (VERDICT r03 "next round" item 1.)
//
// The runtime's fill kernel (__amd_rocclr_fillBufferAligned, OpenCL source embedded in
// libamdhip64) is a plain grid-stride loop of 16-byte stores of a CONSTANT pattern:
//     element = buf + (group * wg + lane) ; while (element < end) { *element = pat; element += next_chunk; }
// Its grid / workgroup come from the kernel trace of this program (rocprofv3 --kernel-trace).
// This probe separates the three things that differ between it and our store kernels:
//   data  : constant pattern vs per-lane distinct vs random bytes (bit toggles on the HBM bus)
//   shape : grid size, workgroup size, unroll depth, grid-stride vs per-block contiguous
//   order : the encode's parity order (256-B runs of 1,024 rows) vs contiguous
// Build: hipcc --offload-arch=gfx950 -O3 -o bench_tools/store_probe bench_tools/store_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

// DATA 0: constant 0x03 bytes (memset's value), 1: per-lane distinct, mostly constant words
// (the old probes), 2: random bytes (a per-lane xorshift state, advanced per store)
template <int DATA>
__device__ __forceinline__ v4u make_val(v4u &st, uint64_t i) {
    if (DATA == 0) return v4u{0x03030303u, 0x03030303u, 0x03030303u, 0x03030303u};
    if (DATA == 1) return v4u{uint32_t(i), 1u, 2u, 3u};
    // cheap per-store scramble: 4 xorshift32 lanes
    st ^= st << 13;
    st ^= st >> 17;
    st ^= st << 5;
    return st;
}

__device__ __forceinline__ v4u seed_of(uint64_t i) {
    uint32_t s = uint32_t(i) * 2654435761u + 0x9e3779b9u;
    return v4u{s | 1u, (s ^ 0x5bd1e995u) | 1u, (s * 7u) | 1u, (s + 0x27d4eb2fu) | 1u};
}

// clone of the runtime fill loop: one 16-B store per iteration, grid-stride
template <int DATA>
__global__ void k_fill_clone(v4u *__restrict__ d, size_t n) {
    size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    v4u st = seed_of(i);
    for (; i < n; i += stride) d[i] = make_val<DATA>(st, i);
}

// grid-stride with U stores per iteration
template <int DATA, int U>
__global__ void k_write_gs(v4u *__restrict__ d, size_t n) {
    const size_t stride = size_t(gridDim.x) * blockDim.x;
    size_t i = size_t(blockIdx.x) * blockDim.x + threadIdx.x;
    v4u st = seed_of(i);
    for (; i + (U - 1) * stride < n; i += U * stride) {
#pragma unroll
        for (int u = 0; u < U; u++) d[i + u * stride] = make_val<DATA>(st, i);
    }
    for (; i < n; i += stride) d[i] = make_val<DATA>(st, i);
}

// per-block contiguous range
template <int DATA, int U>
__global__ void k_write_blk(v4u *__restrict__ d, size_t n) {
    const size_t per = (n + gridDim.x - 1) / gridDim.x;
    const size_t lo = size_t(blockIdx.x) * per, hi = std::min(lo + per, n);
    const size_t B = blockDim.x;
    size_t i = lo + threadIdx.x;
    v4u st = seed_of(i);
    for (; i + (U - 1) * B < hi; i += U * B) {
#pragma unroll
        for (int u = 0; u < U; u++) d[i + u * B] = make_val<DATA>(st, i);
    }
    for (; i < hi; i += B) d[i] = make_val<DATA>(st, i);
}

// the encode's parity order: tile = 256 bytes of each of 1,024 rows (4 chunks x 256 layers of
// sc bytes); a wave-instruction writes 4 rows x 256 B; tiles dealt per XCD (contiguous byte
// region per XCD, 32 workgroups per XCD round robin), 512 threads per workgroup
template <int DATA>
__global__ __launch_bounds__(512) void k_parity_order(uint8_t *par, uint32_t sc, uint64_t chunk) {
    const uint32_t ntiles = sc / 256, tpx = (ntiles + 7) / 8, nsl = gridDim.x / 8, b = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int lr = lane >> 4, lof = (lane & 15) * 16;
    v4u st = seed_of(threadIdx.x + blockIdx.x * 512u);
    for (uint32_t t = b >> 3; t < tpx && (b & 7) * tpx + t < ntiles; t += nsl) {
        const uint32_t b0 = ((b & 7) * tpx + t) * 256;
        for (int i = 0; i < 32; i++) {
            const int row = (wave * 32 + i) * 4 + lr;
            uint8_t *p = par + uint64_t(row >> 8) * chunk + uint64_t(row & 255) * sc + b0 + lof;
            *reinterpret_cast<v4u *>(p) = make_val<DATA>(st, row);
        }
    }
}

// Variants of the parity pattern (random data): the same 1,024 rows x sc bytes, a tile = W bytes of
// every row, 512 threads per workgroup, grid 256 (one per CU).
//   ORDER 0: XCD-blocked (XCD x owns a contiguous byte region, its 32 workgroups round robin)
//   ORDER 1: chip round robin (tile t -> workgroup t % 256: the chip covers 256 adjacent tiles)
//   ORDER 2: one contiguous byte range per workgroup
//   ROWS: 0 = wave w writes rows 128w.. (the encode), 1 = step i of all 8 waves writes 32
//   consecutive rows, 2 = every wave writes 1 row at a time (W/1024 rows per instruction group)
template <int W, int ORDER, int ROWS>
__global__ __launch_bounds__(512) void k_parity_var(uint8_t *par, uint32_t sc, uint64_t chunk) {
    const uint32_t ntiles = sc / W, b = blockIdx.x, G = gridDim.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    constexpr int RPI = 1024 / W;                    // rows per wave instruction (W <= 1024)
    constexpr int NI = 1024 / 8 / RPI;               // instructions per wave per tile
    const int lr = lane / (64 / RPI), lof = (lane % (64 / RPI)) * 16;
    v4u st = seed_of(threadIdx.x + blockIdx.x * 512u);
    uint32_t t0, tstep, tn;
    if (ORDER == 0) {
        const uint32_t tpx = (ntiles + 7) / 8, nsl = G / 8;
        t0 = (b & 7) * tpx + (b >> 3);
        tstep = nsl;
        tn = (b & 7) * tpx + tpx < ntiles ? (b & 7) * tpx + tpx : ntiles;
    } else if (ORDER == 1) {
        t0 = b;
        tstep = G;
        tn = ntiles;
    } else {
        const uint32_t per = (ntiles + G - 1) / G;
        t0 = b * per;
        tstep = 1;
        tn = t0 + per < ntiles ? t0 + per : ntiles;
    }
    for (uint32_t t = t0; t < tn; t += tstep) {
        const uint32_t b0 = t * W;
        for (int i = 0; i < NI; i++) {
            int row;
            if (ROWS == 0) row = (wave * NI + i) * RPI + lr;
            else row = (i * 8 + wave) * RPI + lr;
            uint8_t *p = par + uint64_t(row >> 8) * chunk + uint64_t(row & 255) * sc + b0 + lof;
            *reinterpret_cast<v4u *>(p) = make_val<2>(st, row);
        }
    }
}

template <class F>
static float timeit(F &&launch, int reps = 16) {
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

int main(int argc, char **argv) {
    const char *only = argc > 1 ? argv[1] : "all";
    const size_t G = size_t(1) << 30;
    const size_t bytes = 2 * G, n = bytes / 16;
    uint8_t *b;
    if (hipMalloc(&b, bytes) != hipSuccess) return 1;
    (void)hipMemset(b, 0, bytes);
    auto rep = [&](const char *name, double nb, float ms) {
        printf("%-44s %8.4f ms  %7.1f GB/s\n", name, ms, nb / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    // warm the clock up
    for (int i = 0; i < 300; i++) k_write_gs<1, 1><<<4096, 256>>>((v4u *)b, n);
    (void)hipDeviceSynchronize();
    char nm[128];
    const bool all = !strcmp(only, "all");
    if (all || !strcmp(only, "memset")) {
        rep("hipMemsetAsync 2 GiB value 3", bytes, timeit([&] { (void)hipMemsetAsync(b, 3, bytes, 0); }));
        rep("hipMemsetD32Async 2 GiB", bytes, timeit([&] { (void)hipMemsetD32Async((hipDeviceptr_t)b, 0x12345678u, bytes / 4, 0); }));
        rep("hipMemsetAsync 430 MB value 3", 4.0 * 419432 * 256,
            timeit([&] { (void)hipMemsetAsync(b, 3, size_t(4) * 419432 * 256, 0); }));
    }
    if (all || !strcmp(only, "clone")) {
        // the runtime loop, swept over grid / workgroup, three data kinds
        for (int data = 0; data < 3; data++)
            for (int wg : {256, 1024})
                for (int grid : {256, 1024, 2048, 4096, 8192, 16384, 65536}) {
                    if (size_t(grid) * wg > n) continue;
                    snprintf(nm, sizeof nm, "clone D%d wg%d grid%d", data, wg, grid);
                    rep(nm, bytes, timeit([&] {
                            if (data == 0) k_fill_clone<0><<<grid, wg>>>((v4u *)b, n);
                            if (data == 1) k_fill_clone<1><<<grid, wg>>>((v4u *)b, n);
                            if (data == 2) k_fill_clone<2><<<grid, wg>>>((v4u *)b, n);
                        }));
                }
    }
    if (all || !strcmp(only, "gs")) {
#define GS(D, U, WG, GRID)                                                                          \
    snprintf(nm, sizeof nm, "gs D%d U%d wg%d grid%d", D, U, WG, GRID);                            \
    rep(nm, bytes, timeit([&] { k_write_gs<D, U><<<GRID, WG>>>((v4u *)b, n); }));
#define BLK(D, U, WG, GRID)                                                                         \
    snprintf(nm, sizeof nm, "blk D%d U%d wg%d grid%d", D, U, WG, GRID);                           \
    rep(nm, bytes, timeit([&] { k_write_blk<D, U><<<GRID, WG>>>((v4u *)b, n); }));
        GS(0, 4, 256, 4096)
        GS(1, 4, 256, 4096)
        GS(2, 4, 256, 4096)
        GS(0, 8, 256, 2048)
        GS(2, 8, 256, 2048)
        BLK(0, 4, 256, 2048)
        BLK(2, 4, 256, 2048)
        BLK(0, 4, 512, 1024)
        BLK(2, 4, 512, 1024)
        BLK(0, 1, 1024, 256)
        BLK(2, 1, 1024, 256)
    }
    if (all || !strcmp(only, "parity")) {
        const uint32_t sc = 419432;
        const uint64_t chunk = uint64_t(sc) * 256;
        const double pb = 4.0 * chunk;
        for (int data = 0; data < 3; data++) {
            snprintf(nm, sizeof nm, "parity order D%d grid256", data);
            rep(nm, pb, timeit([&] {
                    if (data == 0) k_parity_order<0><<<256, 512>>>(b, sc, chunk);
                    if (data == 1) k_parity_order<1><<<256, 512>>>(b, sc, chunk);
                    if (data == 2) k_parity_order<2><<<256, 512>>>(b, sc, chunk);
                }));
        }
    }
    if (all || !strcmp(only, "pvar")) {
        const uint32_t sc = 419432;
        const uint64_t chunk = uint64_t(sc) * 256;
        const double pb = 4.0 * chunk;
#define PV(W, O, R)                                                                                 \
    snprintf(nm, sizeof nm, "parity W%d order%d rows%d", W, O, R);                                \
    rep(nm, pb, timeit([&] { k_parity_var<W, O, R><<<256, 512>>>(b, sc, chunk); }));
        PV(256, 0, 0) PV(256, 0, 1) PV(256, 1, 0) PV(256, 1, 1) PV(256, 2, 0) PV(256, 2, 1)
        PV(512, 0, 0) PV(512, 0, 1) PV(512, 1, 0) PV(512, 1, 1) PV(512, 2, 0)
        PV(1024, 0, 0) PV(1024, 0, 1) PV(1024, 1, 0) PV(1024, 1, 1) PV(1024, 2, 0)
    }
    return 0;
}
