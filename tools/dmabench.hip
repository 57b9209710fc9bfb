// dmabench.hip -- memory ceiling of the v4 encode access pattern, no GF math.
// Same tile / section / DMA address pattern as Bs4Kernel<10,4> (16-byte LDS-DMA into a
// wave-private ring of D stages, 8 KiB each), parity-sized dwordx4 stores per tile.
// Varies D (sections in flight per wave) and whether sections end in a block barrier.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)
struct Args { const uint8_t *data[10]; uint8_t *par[4]; uint32_t sc, ntiles, tpx, nslots; };
__device__ __forceinline__ void dma16(uint32_t lds, const uint8_t *sb, uint32_t voff) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, %3\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(lds), "v"(voff), "s"(sb) : "memory");
}
template <int N> __device__ __forceinline__ void wvm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); __builtin_amdgcn_s_barrier(); }
constexpr int WY[3] = {64, 16, 4};
__device__ __forceinline__ int zl(int line, int Y) { int w = WY[Y]; return (line / w) * w * 4 + line % w; }
__device__ void issue(const Args &a, uint32_t lds, int wave, int lane, uint32_t b0, int Y) {
    const int s = lane & 15, r = lane >> 4, pg = s & 1, d = r & 1;
    for (int i = 0; i < 8; i++) {
        const int node = Y * 4 + (i >> 1);
        if (node >= 10) continue;
        const int ll = (s >> 3) | ((((i & 1) << 1) | (r >> 1)) << 1);
        const int jc = (((s >> 1) & 3) - (i >> 1)) & 3;
        uint32_t pos = b0 + uint32_t(2 * pg + d) * 16u;
        if (pos + 16 > a.sc) pos = a.sc - 16;
        dma16(lds + i * 1024, a.data[node], uint32_t(zl(wave * 8 + ll, Y) + jc * WY[Y]) * a.sc + pos);
    }
}
template <int D, bool BAR>
__global__ __launch_bounds__(512) void k(Args a, uint32_t *sink) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t ring = uint32_t(size_t((__attribute__((address_space(3))) uint8_t *)sm)) + wave * D * 8192;
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    // flatten (tile, section) into a stream of sections for this workgroup
    const uint32_t ntix = (a.tpx > slot) ? (a.tpx - slot + a.nslots - 1) / a.nslots : 0;
    uint32_t nsec = 0;
    for (uint32_t t = 0; t < ntix; t++) if (xcd * a.tpx + slot + t * a.nslots < a.ntiles) nsec += 3;
    auto tile_of = [&](uint32_t s) { return xcd * a.tpx + slot + (s / 3) * a.nslots; };
    uint32_t acc = 0;
    for (uint32_t s = 0; s < nsec && s < D; s++) issue(a, ring + (s % D) * 8192, wave, lane, tile_of(s) * 64, s % 3);
    for (uint32_t s = 0; s < nsec; s++) {
        // wait for section s: allow the younger sections (up to D-1) in flight
        const uint32_t ahead = (nsec - 1 - s) < uint32_t(D - 1) ? (nsec - 1 - s) : uint32_t(D - 1);
        // each section is <= 8 DMA instr; stores in between are waited conservatively
        if (ahead >= 2) wvm<16>(); else if (ahead == 1) wvm<8>(); else wvm<0>();
        if (ahead >= 2 && D == 3) {} // (counts approximate for the 4-instr Y=2 section: conservative)
        const uint4 v = *reinterpret_cast<const uint4 *>(sm + (ring - uint32_t(size_t((__attribute__((address_space(3))) uint8_t *)sm))) + (s % D) * 8192 + lane * 16);
        acc ^= v.x ^ v.w;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (s + D < nsec) issue(a, ring + ((s + D) % D) * 8192, wave, lane, tile_of(s + D) * 64, (s + D) % 3);
        if (s % 3 == 2) {  // finish: parity stores 8 x 16 B per lane
            const uint32_t b0 = tile_of(s) * 64;
            const int pg = lane & 1, j = (lane >> 1) & 3, gl = lane >> 3;
            const uint32_t z0 = (wave * 8 + gl) * 4;
            if (b0 + 64 <= a.sc)
                for (int x = 0; x < 4; x++) {
                    uint8_t *p = a.par[x] + (z0 + j) * a.sc + b0 + 32 * pg;
                    *reinterpret_cast<uint4 *>(p) = make_uint4(acc, x, 0, 0);
                    *reinterpret_cast<uint4 *>(p + 16) = make_uint4(acc, x, 1, 0);
                }
        }
        if (BAR) bar();
    }
    wvm<0>();
    if (acc == 0x12345678u) sink[0] = acc;
}
template <int D, bool BAR>
float run(const Args &a0, uint32_t *sink, int cus, int per_cu) {
    Args a = a0;
    const int lds = 8 * D * 8192;
    hipFuncSetAttribute((const void *)&k<D, BAR>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    a.nslots = std::min<uint32_t>((cus / 8) * per_cu, a.tpx);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    float best = 1e9;
    for (int it = 0; it < 8; it++) {
        hipEventRecord(e0);
        k<D, BAR><<<a.nslots * 8, 512, lds>>>(a, sink);
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
    a.sc = sc; a.ntiles = (sc + 63) / 64; a.tpx = (a.ntiles + 7) / 8;
    hipDeviceProp_t pr; hipGetDeviceProperties(&pr, 0);
    const double bytes = 14.0 * chunk;
    auto rep = [&](const char *n, float ms) { printf("%-14s %.4f ms  %.0f GB/s\n", n, ms, bytes / (ms * 1e-3) / 1e9); };
    const int cu = pr.multiProcessorCount;
    rep("D1 bar 1/CU", run<1, true>(a, sink, cu, 1));
    rep("D1 free 1/CU", run<1, false>(a, sink, cu, 1));
    rep("D1 bar 2/CU", run<1, true>(a, sink, cu, 2));
    rep("D1 free 2/CU", run<1, false>(a, sink, cu, 2));
    rep("D2 bar 1/CU", run<2, true>(a, sink, cu, 1));
    rep("D2 free 1/CU", run<2, false>(a, sink, cu, 1));
    rep("D1 bar 1/CU", run<1, true>(a, sink, cu, 1));
    return 0;
}
