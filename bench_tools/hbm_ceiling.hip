// hbm_ceiling.hip -- what HBM rate can the (10,4,13) 1 GiB encode access pattern reach on
// this box, with no GF arithmetic at all?
//   stream-read   : read the 10 data chunks contiguously (dwordx4, U loads in flight/lane)
//   stream-copy   : read 10 chunks + write 4 chunks contiguously (the encode byte counts)
//   tile<W,U>     : the encode pattern: a tile = W bytes of every (node, layer) sub-chunk
//                   row (2,560 rows read, 1,024 rows written); tiles dealt per XCD in
//                   contiguous regions; each lane keeps U 16-byte loads in flight
// Build: hipcc --offload-arch=gfx950 -O3 -o bench_tools/hbm_ceiling bench_tools/hbm_ceiling.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__);            \
            return 1;                                                               \
        }                                                                           \
    } while (0)

struct Ptrs {
    const uint8_t *d[10];
    uint8_t *p[4];
};

template <int U>
__global__ __launch_bounds__(256) void k_stream_read(const uint4 *src, size_t n, uint32_t *sink) {
    uint32_t acc = 0;
    const size_t stride = size_t(gridDim.x) * 256;
    size_t i = size_t(blockIdx.x) * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = src[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u].x ^ v[u].w;
    }
    for (; i < n; i += stride) acc ^= src[i].y;
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

// each workgroup streams its own contiguous block (DRAM-page friendly)
template <int U>
__global__ __launch_bounds__(512) void k_block_read(const uint4 *src, size_t n, uint32_t *sink) {
    const size_t per = (n + gridDim.x - 1) / gridDim.x;
    const size_t lo = size_t(blockIdx.x) * per, hi = lo + per < n ? lo + per : n;
    uint32_t acc = 0;
    size_t i = lo + threadIdx.x;
    for (; i + (U - 1) * 512 < hi; i += U * 512) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = src[i + u * 512];
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u].x ^ v[u].w;
    }
    for (; i < hi; i += 512) acc ^= src[i].y;
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

// per iteration: 5 loads from the data stream, 2 stores to the parity stream (10:4)
template <int U>
__global__ __launch_bounds__(256) void k_stream_copy(const uint4 *src, uint4 *dst, size_t nunits) {
    const size_t stride = size_t(gridDim.x) * 256;
    for (size_t i = size_t(blockIdx.x) * 256 + threadIdx.x; i < nunits; i += stride) {
        uint4 v[5];
#pragma unroll
        for (int u = 0; u < 5; u++) v[u] = src[i * 5 + u];
        dst[i * 2] = make_uint4(v[0].x ^ v[1].x, v[2].y, v[3].z, v[4].w);
        dst[i * 2 + 1] = make_uint4(v[0].y, v[1].z ^ v[4].x, v[2].w, v[3].x);
    }
}

// Encode pattern from registers.  Workgroup of 512 lanes; a tile is W bytes of 2,560 read
// rows and 1,024 written rows; L = W / 16 lanes per row, 512 / L rows per wave-wide step.
// ST: 0 = no stores, 1 = contiguous 16-byte pieces per lane, 2 = v6/v7 gapped pair (lane
// owns 32 contiguous bytes, two dwordx4 stores 16 bytes apart), 3 = reads skipped
template <int W, int U, int ST = 1>
__global__ __launch_bounds__(512) void k_tile(Ptrs P, uint32_t sc, uint32_t region, uint32_t ns, uint32_t *sink) {
    constexpr int L = W / 16, RPS = 512 / L;
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    const uint32_t x0 = xcd * region, x1 = std::min(x0 + region, sc);
    const int r0 = threadIdx.x / L;
    const uint32_t off = (threadIdx.x % L) * 16;
    uint32_t acc = 0;
    for (uint32_t b0 = x0 + slot * W; b0 + W <= x1; b0 += ns * W) {
        // reads: rows r0, r0 + RPS, ... of 2,560, U in flight
        for (int r = r0; ST != 3 && r < 2560; r += U * RPS) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int row = r + u * RPS;
                const int rr = row < 2560 ? row : r0;
                v[u] = *reinterpret_cast<const uint4 *>(P.d[rr >> 8] + uint32_t(rr & 255) * sc + b0 + off);
            }
#pragma unroll
            for (int u = 0; u < U; u++) acc ^= v[u].x ^ v[u].w;
        }
        if (ST == 1 || ST == 3)
            for (int r = r0; r < 1024; r += RPS)
                *reinterpret_cast<uint4 *>(P.p[r >> 8] + uint32_t(r & 255) * sc + b0 + off) =
                    make_uint4(acc, r, b0, 0);
        if (ST >= 4) {  // contiguous, cache policy: 4 nt, 5 sc1, 6 sc0 sc1, 7 sc1 nt
            for (int r = r0; r < 1024; r += RPS) {
                uint8_t *p = P.p[r >> 8] + uint32_t(r & 255) * sc + b0 + off;
                typedef uint32_t u4 __attribute__((ext_vector_type(4)));
                const u4 v = {acc, uint32_t(r), b0, 0u};
                if (ST == 4) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
                if (ST == 5) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
                if (ST == 6) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
                if (ST == 7) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
            }
        }
        if (ST == 2) {  // W / 32 lanes per row, each 32 bytes as two stores
            constexpr int L2 = W / 32, RPS2 = 512 / L2;
            const int q0 = threadIdx.x / L2;
            const uint32_t o2 = (threadIdx.x % L2) * 32;
            for (int r = q0; r < 1024; r += RPS2) {
                uint8_t *p = P.p[r >> 8] + uint32_t(r & 255) * sc + b0 + o2;
                *reinterpret_cast<uint4 *>(p) = make_uint4(acc, r, b0, 0);
                *reinterpret_cast<uint4 *>(p + 16) = make_uint4(acc, r, b0, 1);
            }
        }
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

template <class F>
static float timeit(F &&launch) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> t;
    for (int r = 0; r < 10; r++) {
        hipEventRecord(e0);
        launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    const uint32_t sc = 419432;
    const size_t chunk = size_t(sc) * 256;
    uint8_t *data, *par;
    uint32_t *sink;
    CK(hipMalloc(&data, 10 * chunk));
    CK(hipMalloc(&par, 4 * chunk));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(data, 1, 10 * chunk));
    CK(hipMemset(par, 0, 4 * chunk));
    Ptrs P;
    for (int i = 0; i < 10; i++) P.d[i] = data + i * chunk;
    for (int i = 0; i < 4; i++) P.p[i] = par + i * chunk;
    const double rd = 10.0 * chunk, all = 14.0 * chunk;
    auto rep = [&](const char *name, double bytes, float ms) {
        printf("%-34s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    char nm[96];
    for (int g : {1024, 2048, 4096}) {
        snprintf(nm, sizeof nm, "stream-read U4 grid %d", g);
        rep(nm, rd, timeit([&] { k_stream_read<4><<<g, 256>>>((const uint4 *)data, rd / 16, sink); }));
        snprintf(nm, sizeof nm, "stream-read U8 grid %d", g);
        rep(nm, rd, timeit([&] { k_stream_read<8><<<g, 256>>>((const uint4 *)data, rd / 16, sink); }));
        snprintf(nm, sizeof nm, "stream-copy 10:4 grid %d", g);
        rep(nm, all, timeit([&] { k_stream_copy<1><<<g, 256>>>((const uint4 *)data, (uint4 *)par, 2 * chunk / 16); }));
    }
    for (int g : {256, 512, 1024}) {
        snprintf(nm, sizeof nm, "block-read U8 grid %d x512", g);
        rep(nm, rd, timeit([&] { k_block_read<8><<<g, 512>>>((const uint4 *)data, rd / 16, sink); }));
        snprintf(nm, sizeof nm, "block-read U16 grid %d x512", g);
        rep(nm, rd, timeit([&] { k_block_read<16><<<g, 512>>>((const uint4 *)data, rd / 16, sink); }));
    }
    const uint32_t region = ((sc + 7) / 8 + 31) / 32 * 32;
    auto tile = [&](auto wc, auto uc, uint32_t ns) {
        constexpr int W = decltype(wc)::value, U = decltype(uc)::value;
        snprintf(nm, sizeof nm, "tile W%d U%d wg/xcd %u", W, U, ns);
        rep(nm, all, timeit([&] { k_tile<W, U><<<8 * ns, 512>>>(P, sc, region, ns, sink); }));
    };
    auto tile_st = [&](auto wc, auto stc) {
        constexpr int W = decltype(wc)::value, ST = decltype(stc)::value;
        const char *sn[] = {"reads only", "contig stores", "gapped stores", "stores only", "nt stores", "sc1 stores",
                            "sc0sc1 stores", "sc1nt stores"};
        snprintf(nm, sizeof nm, "tile W%d U8 %s", W, sn[ST]);
        const double b = ST == 0 ? rd : ST == 3 ? 4.0 * chunk : all;
        rep(nm, b, timeit([&] { k_tile<W, 8, ST><<<8 * 32, 512>>>(P, sc, region, 32, sink); }));
    };
    tile_st(std::integral_constant<int, 256>{}, std::integral_constant<int, 0>{});
    tile_st(std::integral_constant<int, 256>{}, std::integral_constant<int, 1>{});
    tile_st(std::integral_constant<int, 256>{}, std::integral_constant<int, 2>{});
    tile_st(std::integral_constant<int, 256>{}, std::integral_constant<int, 3>{});
    tile_st(std::integral_constant<int, 256>{}, std::integral_constant<int, 4>{});
    tile_st(std::integral_constant<int, 256>{}, std::integral_constant<int, 5>{});
    tile_st(std::integral_constant<int, 256>{}, std::integral_constant<int, 6>{});
    tile_st(std::integral_constant<int, 256>{}, std::integral_constant<int, 7>{});
    tile_st(std::integral_constant<int, 1024>{}, std::integral_constant<int, 0>{});
    tile_st(std::integral_constant<int, 1024>{}, std::integral_constant<int, 3>{});
    using I = std::integral_constant<int, 0>;
    (void)sizeof(I);
    tile(std::integral_constant<int, 128>{}, std::integral_constant<int, 8>{}, 32);
    tile(std::integral_constant<int, 256>{}, std::integral_constant<int, 4>{}, 32);
    tile(std::integral_constant<int, 256>{}, std::integral_constant<int, 8>{}, 32);
    tile(std::integral_constant<int, 256>{}, std::integral_constant<int, 16>{}, 32);
    tile(std::integral_constant<int, 256>{}, std::integral_constant<int, 8>{}, 64);
    tile(std::integral_constant<int, 512>{}, std::integral_constant<int, 8>{}, 32);
    tile(std::integral_constant<int, 512>{}, std::integral_constant<int, 16>{}, 32);
    tile(std::integral_constant<int, 1024>{}, std::integral_constant<int, 8>{}, 32);
    tile(std::integral_constant<int, 2048>{}, std::integral_constant<int, 8>{}, 32);
    return 0;
}
