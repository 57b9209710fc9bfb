// dmabench4.hip -- (from dmabench3) + tile->CU mapping variants + single-buffer batches.
// dmabench3.hip -- access-pattern ceiling for slot rings: slot = 4 nodes x L layers x W
// bytes (layers of one d3-group when L = 64), ring of R slots (R-1 in flight), barrier per
// slot; a tile = W bytes of every sub-chunk; parity-sized stores per tile (16 B per lane).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <algorithm>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)
struct Args { const uint8_t *data[10]; uint8_t *par[4]; uint32_t sc, ntiles, tpx, nslots; };
__device__ __forceinline__ void dma16(uint32_t lds, const uint8_t *sb, uint32_t voff) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds), "v"(voff), "s"(sb) : "memory");
}
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); __builtin_amdgcn_s_barrier(); }
template <int N> __device__ __forceinline__ void wvm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// slot s of a tile: section Y = s / G, group g = s % G (G = 256 / L); real nodes only
template <int W, int L, int BLOCK>
__device__ int issue(const Args &a, uint32_t lds, int tid, uint32_t b0, int s) {
    constexpr int G = 256 / L;
    constexpr int LPR = W / 16;                       // lanes per row
    constexpr int ROWS = 4 * L;                       // rows in a slot (node, layer)
    constexpr int PER = ROWS * LPR / BLOCK;           // 16-B pieces per thread
    const int Y = s / G, g = s % G;
    int n = 0;
    for (int i = 0; i < PER; i++) {
        const int piece = i * BLOCK + tid;
        const int row = piece / LPR, off = (piece % LPR) * 16;
        const int x = row / L, l = row % L;
        const int node = __builtin_amdgcn_readfirstlane(Y * 4 + x);  // uniform per wave
        // (instruction-uniform node: BLOCK*i..: row range spans one node when L*LPR >= BLOCK)
        uint32_t pos = b0 + off;
        if (pos + 16 > a.sc) pos = a.sc - 16;
        const int layer = g * L + l;   // layers of group g (contiguous here; layout is irrelevant to HBM)
        if (node < 10) { dma16(lds + uint32_t(i * BLOCK * 16), a.data[node], uint32_t(layer) * a.sc + pos); n++; }
    }
    return n;
}
template <int W, int L, int R, int BLOCK, bool GLOBAL>
__global__ __launch_bounds__(BLOCK) void k(Args a, uint32_t *sink) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    constexpr int SLOT = 4 * L * W, G = 256 / L, SPT = 3 * G;
    const int tid = threadIdx.x;
    const uint32_t base = uint32_t(size_t((__attribute__((address_space(3))) uint8_t *)sm));
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    uint32_t ntile = 0;
    if (GLOBAL) {
        for (uint32_t t = blockIdx.x; t < a.ntiles; t += gridDim.x) ntile++;
    } else {
        const uint32_t ntix = (a.tpx > slot) ? (a.tpx - slot + a.nslots - 1) / a.nslots : 0;
        for (uint32_t t = 0; t < ntix; t++) if (xcd * a.tpx + slot + t * a.nslots < a.ntiles) ntile++;
    }
    const uint32_t nsl = ntile * SPT;
    auto tile_of = [&](uint32_t s) {
        return GLOBAL ? blockIdx.x + (s / SPT) * gridDim.x : xcd * a.tpx + slot + (s / SPT) * a.nslots;
    };
    uint32_t acc = 0;
    constexpr int AH = R > 1 ? R - 1 : 1;
    for (uint32_t s = 0; s < nsl && s < AH; s++) issue<W, L, BLOCK>(a, base + (s % R) * SLOT, tid, tile_of(s) * W, s % SPT);
    for (uint32_t s = 0; s < nsl; s++) {
        wvm<0>();
        bar();
        if (R > 1 && s + AH < nsl) issue<W, L, BLOCK>(a, base + ((s + AH) % R) * SLOT, tid, tile_of(s + AH) * W, (s + AH) % SPT);
        for (int e = tid * 16; e < SLOT; e += BLOCK * 16) {
            const uint4 v = *reinterpret_cast<const uint4 *>(sm + (s % R) * SLOT + e);
            acc ^= v.x ^ v.w;
        }
        if (R == 1) {
            bar();
            if (s + 1 < nsl) issue<W, L, BLOCK>(a, base, tid, tile_of(s + 1) * W, (s + 1) % SPT);
        }
        if (s % SPT == SPT - 1) {
            const uint32_t b0 = tile_of(s) * W;
            if (b0 + W <= a.sc)
                for (int x = 0; x < 4; x++)
                    for (int e = tid * 16; e < 256 * W; e += BLOCK * 16) {
                        const int layer = e / W, o = e % W;
                        *reinterpret_cast<uint4 *>(a.par[x] + size_t(layer) * a.sc + b0 + o) = make_uint4(acc, x, e, 0);
                    }
        }
    }
    wvm<0>();
    if (acc == 0x12345678u) sink[0] = acc;
}
template <int W, int L, int R, int BLOCK, bool GLOBAL = false>
float run(Args a, uint32_t *sink, int cus) {
    const int lds = R * 4 * L * W;
    if (lds > 160 * 1024) return -1;
    hipFuncSetAttribute((const void *)&k<W, L, R, BLOCK, GLOBAL>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    a.ntiles = (a.sc + W - 1) / W; a.tpx = (a.ntiles + 7) / 8;
    a.nslots = std::min<uint32_t>(cus / 8, a.tpx);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    float best = 1e9;
    for (int it = 0; it < 8; it++) {
        hipEventRecord(e0);
        k<W, L, R, BLOCK, GLOBAL><<<a.nslots * 8, BLOCK, lds>>>(a, sink);
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        if (it >= 2 && ms < best) best = ms;
    }
    return best;
}
int main() {
    const uint32_t sc = 419432, alpha = 256;
    const size_t chunk = size_t(sc) * alpha;
    Args a{};
    for (int i = 0; i < 10; i++) { void *p; CK(hipMalloc(&p, chunk)); hipMemset(p, i, chunk); a.data[i] = (const uint8_t *)p; }
    for (int i = 0; i < 4; i++) { void *p; CK(hipMalloc(&p, chunk)); a.par[i] = (uint8_t *)p; }
    uint32_t *sink; CK(hipMalloc(&sink, 64));
    a.sc = sc;
    hipDeviceProp_t pr; hipGetDeviceProperties(&pr, 0);
    const int cu = pr.multiProcessorCount;
    auto rep = [&](const char *n, float ms) { printf("%-26s %.4f ms  %.0f GB/s\n", n, ms, 14.0 * chunk / (ms * 1e-3) / 1e9); };
    rep("W256 L64 R2 (v6:8)", run<256, 64, 2, 512>(a, sink, cu));
    rep("W256 L64 R2 global-map", run<256, 64, 2, 512, true>(a, sink, cu));
    rep("W128 L64 R5 (v6:4)", run<128, 64, 5, 256>(a, sink, cu));
    rep("W128 L64 R5 global-map", run<128, 64, 5, 256, true>(a, sink, cu));
    rep("W128 L256 R1", run<128, 256, 1, 512>(a, sink, cu));
    rep("W256 L128 R1", run<256, 128, 1, 512>(a, sink, cu));
    rep("W512 L64 R1", run<512, 64, 1, 512>(a, sink, cu));
    rep("W512 L64 R1 global-map", run<512, 64, 1, 512, true>(a, sink, cu));
    rep("W1024 L32 R1", run<1024, 32, 1, 512>(a, sink, cu));
    rep("W64 L256 R2", run<64, 256, 2, 512>(a, sink, cu));
    rep("W256 L64 R2 (v6:8)", run<256, 64, 2, 512>(a, sink, cu));
    return 0;
}
