// dmabench2.hip -- does a wider contiguous run per sub-chunk row raise the ceiling of the
// encode access pattern?  Block = 8 waves; per section the block DMAs 4 nodes x 256 layers
// x W bytes (16-byte LDS-DMA, 1 KiB per instruction = (1024/W) rows x W bytes), single
// buffered (D=1) or double buffered (D=2), barrier per section; parity-sized stores.
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
template <int N> __device__ __forceinline__ void wvm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); __builtin_amdgcn_s_barrier(); }
// section s of tile: nodes 4s..4s+3 (real < 10), all 256 layers, W bytes at b0
template <int W>
__device__ void issue(const Args &a, uint32_t lds, int wave, int lane, uint32_t b0, int s) {
    constexpr int RPI = 1024 / W;                 // rows per instruction
    constexpr int IPN = 256 / RPI;                // instructions per node (all layers)
    constexpr int IPW = IPN / 8;                  // per wave per node
    const int r = lane / (W / 16), off = (lane % (W / 16)) * 16;
    for (int x = 0; x < 4; x++) {
        const int node = s * 4 + x;
        if (node >= 10) continue;
        for (int i = 0; i < IPW; i++) {
            const int ins = wave * IPW + i;
            const int layer = ins * RPI + r;
            uint32_t pos = b0 + off;
            if (pos + 16 > a.sc) pos = a.sc - 16;
            dma16(lds + uint32_t((x * IPN + ins) * 1024), a.data[node], uint32_t(layer) * a.sc + pos);
        }
    }
}
template <int W, int D, bool ST>
__global__ __launch_bounds__(512) void k(Args a, uint32_t *sink) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    constexpr int SEC = 4 * 256 * W;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t base = uint32_t(size_t((__attribute__((address_space(3))) uint8_t *)sm));
    const uint32_t xcd = blockIdx.x & 7u, slot = blockIdx.x >> 3;
    const uint32_t ntix = (a.tpx > slot) ? (a.tpx - slot + a.nslots - 1) / a.nslots : 0;
    uint32_t nsec = 0;
    for (uint32_t t = 0; t < ntix; t++) if (xcd * a.tpx + slot + t * a.nslots < a.ntiles) nsec += 3;
    auto tile_of = [&](uint32_t s) { return xcd * a.tpx + slot + (s / 3) * a.nslots; };
    uint32_t acc = 0;
    for (uint32_t s = 0; s < nsec && s < D; s++) issue<W>(a, base + (s % D) * SEC, wave, lane, tile_of(s) * W, s % 3);
    for (uint32_t s = 0; s < nsec; s++) {
        if (D == 2 && s + 1 < nsec) wvm<32>(); else wvm<0>();   // conservative
        bar();
        const uint4 v = *reinterpret_cast<const uint4 *>(sm + (s % D) * SEC + threadIdx.x * 16);
        acc ^= v.x ^ v.w;
        bar();
        if (s + D < nsec) issue<W>(a, base + ((s + D) % D) * SEC, wave, lane, tile_of(s + D) * W, (s + D) % 3);
        if (ST && s % 3 == 2) {
            const uint32_t b0 = tile_of(s) * W;
            if (b0 + W <= a.sc)
                for (int x = 0; x < 4; x++)
                    for (int e = threadIdx.x * 16; e < 256 * W; e += 512 * 16) {
                        const int layer = e / W, o = e % W;
                        *reinterpret_cast<uint4 *>(a.par[x] + size_t(layer) * a.sc + b0 + o) = make_uint4(acc, x, e, 0);
                    }
        }
    }
    wvm<0>();
    if (acc == 0x12345678u) sink[0] = acc;
}
template <int W, int D, bool ST>
float run(Args a, uint32_t *sink, int cus) {
    const int lds = D * 4 * 256 * W;
    if (lds > 160 * 1024) return -1;
    hipFuncSetAttribute((const void *)&k<W, D, ST>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    a.ntiles = (a.sc + W - 1) / W; a.tpx = (a.ntiles + 7) / 8;
    a.nslots = std::min<uint32_t>(cus / 8, a.tpx);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    float best = 1e9;
    for (int it = 0; it < 8; it++) {
        hipEventRecord(e0);
        k<W, D, ST><<<a.nslots * 8, 512, lds>>>(a, sink);
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
    auto rep = [&](const char *n, float ms, double bytes) { printf("%-22s %.4f ms  %.0f GB/s\n", n, ms, bytes / (ms * 1e-3) / 1e9); };
    const double rw = 14.0 * chunk, ro = 10.0 * chunk;
    rep("W64  D1 reads+stores", run<64, 1, true>(a, sink, cu), rw);
    rep("W64  D2 reads+stores", run<64, 2, true>(a, sink, cu), rw);
    rep("W128 D1 reads+stores", run<128, 1, true>(a, sink, cu), rw);
    rep("W64  D1 reads only", run<64, 1, false>(a, sink, cu), ro);
    rep("W64  D2 reads only", run<64, 2, false>(a, sink, cu), ro);
    rep("W128 D1 reads only", run<128, 1, false>(a, sink, cu), ro);
    rep("W32  D2 reads only", run<32, 2, false>(a, sink, cu), ro);
    rep("W32  D4 reads only", run<32, 4, false>(a, sink, cu), ro);
    rep("W64  D1 reads+stores", run<64, 1, true>(a, sink, cu), rw);
    return 0;
}
