// membench.hip -- access-pattern ceiling for the Clay encode data layout (no GF math).
// Tile = W byte positions of every (node, layer) sub-chunk: read 10 nodes x 256 layers
// x W, write 4 x 256 x W (the (10,4,13) 1 GiB stripe: sc = 419,432).  Compared with a
// plain streaming copy of the same byte counts.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Ptrs { const uint8_t* d[10]; uint8_t* p[4]; };

// one workgroup per tile; lanes coalesced along positions; reads XOR-reduced into
// a register (kept live), writes derived values
template <int W>
__global__ __launch_bounds__(256) void k_tile(Ptrs P, uint64_t sc, uint32_t ntiles) {
    constexpr int LPS = W / 8;            // lanes per segment (8 B each)
    constexpr int SEG = 256 / LPS;        // segments per block-wide instruction
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t b0 = uint64_t(tile) * W;
        const int lane_seg = threadIdx.x / LPS, lp = threadIdx.x % LPS;
        const uint64_t pos = b0 + lp * 8;
        uint2 acc = make_uint2(0, 0);
        if (pos + 8 <= sc) {
            for (int s = lane_seg; s < 2560; s += SEG) {
                const int node = s / 256, z = s % 256;
                uint2 v = *reinterpret_cast<const uint2*>(P.d[node] + uint64_t(z) * sc + pos);
                acc.x ^= v.x + s; acc.y ^= v.y;
            }
            for (int s = lane_seg; s < 1024; s += SEG) {
                const int node = s / 256, z = s % 256;
                *reinterpret_cast<uint2*>(P.p[node] + uint64_t(z) * sc + pos) = make_uint2(acc.x ^ s, acc.y);
            }
        }
    }
}

__global__ void k_copy(const uint4* __restrict__ a, uint4* __restrict__ b, size_t nr, size_t nw) {
    size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x, st = size_t(gridDim.x) * blockDim.x;
    uint4 acc = make_uint4(0,0,0,0);
    for (size_t k = i; k < nr; k += st) { uint4 v = a[k]; acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w; }
    for (size_t k = i; k < nw; k += st) b[k] = make_uint4(acc.x ^ k, acc.y, acc.z, acc.w);
}

template <int W>
float run_tile(Ptrs P, uint64_t sc, int grid) {
    uint32_t nt = uint32_t((sc + W - 1) / W);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    std::vector<float> t;
    for (int r = 0; r < 8; r++) {
        hipEventRecord(e0);
        k_tile<W><<<grid, 256>>>(P, sc, nt);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    const uint64_t sc = 419432, chunk = sc * 256;
    uint8_t *data, *par;
    CK(hipMalloc(&data, 10 * chunk)); CK(hipMalloc(&par, 4 * chunk));
    CK(hipMemset(data, 1, 10 * chunk));
    Ptrs P; for (int i = 0; i < 10; i++) P.d[i] = data + i * chunk; for (int i = 0; i < 4; i++) P.p[i] = par + i * chunk;
    const double bytes = 14.0 * chunk;
    int grids[] = {256 * 4, 256 * 8, 256 * 16};
    for (int g : grids) {
        printf("grid %5d  W=64 %.1f  W=128 %.1f  W=256 %.1f  W=512 %.1f  W=2048 %.1f  GB/s\n", g,
               bytes / run_tile<64>(P, sc, g) / 1e6, bytes / run_tile<128>(P, sc, g) / 1e6,
               bytes / run_tile<256>(P, sc, g) / 1e6, bytes / run_tile<512>(P, sc, g) / 1e6,
               bytes / run_tile<2048>(P, sc, g) / 1e6);
    }
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    std::vector<float> t;
    for (int r = 0; r < 8; r++) {
        hipEventRecord(e0);
        k_copy<<<256 * 8, 256>>>((const uint4*)data, (uint4*)par, 10 * chunk / 16, 4 * chunk / 16);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1); if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    printf("streaming copy (read 10 chunks, write 4): %.1f GB/s (%.3f ms)\n", bytes / t[t.size()/2] / 1e6, t[t.size()/2]);
    return 0;
}
