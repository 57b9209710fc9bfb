// stamp_v6.hip -- where does a k_bs6_encode wave spend its cycles?  Builds the kernel with
// CLAY_STAMPS (per-phase s_memtime sums per wave), runs the BASELINE stripe shape and
// prints the mean cycles per step of each phase over all waves.
#define CLAY_STAMPS 1
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <type_traits>
#include <vector>
#include <algorithm>
#include "../clay_amd/csrc/gf256.hpp"
#include "../clay_amd/csrc/bitslice6.hpp"
using namespace clay::bs;
template <int PARTS, bool EARLY>
void run(const char *name, BsArgs a, int cus) {
    using Kn = Bs6Kernel<10, 4, PARTS, EARLY>;
    hipFuncSetAttribute((const void *)&k_bs6_encode<10, 4, PARTS, EARLY>, hipFuncAttributeMaxDynamicSharedMemorySize, Kn::LDS_BYTES);
    a.ntiles = uint32_t((a.sc + Kn::W - 1) / Kn::W);
    a.tiles_per_xcd = (a.ntiles + 7) / 8;
    a.nslots = std::min<uint32_t>(cus / 8, a.tiles_per_xcd);
    const int nb = a.nslots * 8;
    uint64_t *d; hipMalloc(&d, size_t(nb) * Kn::WAVES * 8 * 8);
    hipMemset(d, 0, size_t(nb) * Kn::WAVES * 64);
    hipMemcpyToSymbol(HIP_SYMBOL(g_clay_stamps), &d, sizeof(d));
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    float ms = 0;
    for (int it = 0; it < 3; it++) {
        hipEventRecord(e0);
        k_bs6_encode<10, 4, PARTS, EARLY><<<nb, Kn::BLOCK, Kn::LDS_BYTES>>>(a);
        hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
    }
    std::vector<uint64_t> h(size_t(nb) * Kn::WAVES * 8);
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double sum[6] = {}, steps = 0;
    for (size_t w = 0; w < h.size() / 8; w++) { for (int i = 0; i < 6; i++) sum[i] += h[w * 8 + i]; steps += h[w * 8 + 6]; }
    const char *nm[6] = {"wait(dma)", "barrier", "issue", "compute", "group-end", "drain"};
    printf("%s: %.4f ms, cycles per step per wave:", name, ms);
    double tot = 0;
    for (int i = 0; i < 6; i++) { printf("  %s %.0f", nm[i], sum[i] / steps); tot += sum[i] / steps; }
    printf("  | total %.0f\n", tot);
    hipFree(d);
}
int main() {
    const uint64_t sc = 419432, alpha = 256;
    const size_t chunk = sc * alpha;
    BsArgs a{};
    for (int i = 0; i < 10; i++) { void *p; hipMalloc(&p, chunk); hipMemset(p, i * 37 + 1, chunk); a.data[i] = (const uint8_t *)p; }
    for (int i = 0; i < 4; i++) { void *p; hipMalloc(&p, chunk); a.par[i] = (uint8_t *)p; }
    a.sc = sc;
    hipDeviceProp_t pr; hipGetDeviceProperties(&pr, 0);
    run<8, false>("v6 W256", a, pr.multiProcessorCount);
    run<8, true>("v6 W256 early", a, pr.multiProcessorCount);
    run<4, false>("v6 W128", a, pr.multiProcessorCount);
    return 0;
}
