// page_probe.hip -- which 256-byte pieces of one sub-chunk row share an HBM page?
// A "tile" reads, from each of the 2,560 (node, layer) rows of the (10,4,13) 1 GiB stripe,
// P = 4 pieces of 256 bytes at b0 + j * S (j = 0..3).  S = 256 is a contiguous 1 KiB run;
// if pieces S apart land in one DRAM page the rate stays at the contiguous rate.
// Tiles are dealt so the whole row is covered once.  Reads only (mode 0) or reads +
// parity-sized stores of the same shape (mode 1).
// Build: hipcc --offload-arch=gfx950 -O3 -o bench_tools/page_probe bench_tools/page_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

struct Ptrs {
    const uint8_t *d[10];
    uint8_t *p[4];
};

// one wave = one row x 4 pieces x 256 B; 8 waves; U rows in flight per wave
template <int U, int MODE>
__global__ __launch_bounds__(512) void k_stride(Ptrs P, uint32_t sc, uint32_t S, uint32_t ntiles, uint32_t *sink) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t j = lane >> 4, o = (lane & 15) * 16;
    const uint32_t per_block = S / 256;
    uint32_t acc = 0;
    for (uint32_t tk = blockIdx.x; tk < ntiles * 8; tk += gridDim.x) {  // task = tile x 1/8 of the rows
        const uint32_t t = tk >> 3, rlo = (tk & 7) * 320, rhi = rlo + 320;
        const uint32_t b0 = (t / per_block) * 4 * S + (t % per_block) * 256 + j * S + o;
        for (int r = rlo + wave; r < int(rhi); r += 8 * U) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int row = r + 8 * u < int(rhi) ? r + 8 * u : r;
                v[u] = *reinterpret_cast<const uint4 *>(P.d[row >> 8] + uint32_t(row & 255) * sc + b0);
            }
#pragma unroll
            for (int u = 0; u < U; u++) acc ^= v[u].x ^ v[u].w;
        }
        if (MODE == 1)
            for (int r = (tk & 7) * 128 + wave; r < int((tk & 7) * 128 + 128); r += 8)
                *reinterpret_cast<uint4 *>(P.p[r >> 8] + uint32_t(r & 255) * sc + b0) = make_uint4(acc, r, b0, 0);
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

int main() {
    const uint32_t sc = 419432;
    const size_t chunk = size_t(sc) * 256;
    uint8_t *data, *par;
    uint32_t *sink;
    if (hipMalloc(&data, 10 * chunk) || hipMalloc(&par, 4 * chunk) || hipMalloc(&sink, 64)) return 1;
    (void)hipMemset(data, 1, 10 * chunk);
    Ptrs P;
    for (int i = 0; i < 10; i++) P.d[i] = data + i * chunk;
    for (int i = 0; i < 4; i++) P.p[i] = par + i * chunk;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int mode = 0; mode < 2; mode++)
        for (uint32_t S : {256u, 512u, 1024u, 4096u, 16384u, 32768u, 65536u, 98304u, 131072u}) {
            const uint32_t blocks = sc / (4 * S);  // whole blocks only
            const uint32_t ntiles = blocks * (S / 256);
            const double bytes = double(ntiles) * 1024.0 * (mode ? 3584.0 : 2560.0);
            std::vector<float> t;
            for (int r = 0; r < 8; r++) {
                (void)hipEventRecord(e0);
                if (mode == 0) k_stride<8, 0><<<1024, 512>>>(P, sc, S, ntiles, sink);
                else k_stride<8, 1><<<1024, 512>>>(P, sc, S, ntiles, sink);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (r >= 2) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            printf("%s S=%6u  tiles %6u  %.4f ms  %7.1f GB/s\n", mode ? "rd+wr" : "read ", S, ntiles, t[t.size() / 2],
                   bytes / (t[t.size() / 2] * 1e-3) / 1e9);
            fflush(stdout);
        }
    return 0;
}
