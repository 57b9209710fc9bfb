// repair_probe.hip -- where does the streaming repair kernel's time go?  Times
// k_bs_repair_stream<9,3,Y0=0> on the BASELINE (9,3,11) repair (chunk 268,435,458, sc =
// 3,314,018, gathered helpers: 11 x 27 sub-chunks), or with a third argument "10" the (10,4,13)
// repair of node 0 (chunk 107,374,592, sc = 419,432, 13 helpers x 64 sub-chunks), with parts
// switched off (PROBE bits: 1 = no math, 2 = no DMA, 4 = no output stores; wrong bytes, this
// tool only).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bench_tools/repair_probe bench_tools/repair_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../clay_amd/csrc/repair_kernel.hpp"

using namespace clay::bs;

template <int PARTS, int LOADERS, int PROBE, int KD = 9, int M = 3>
static float run(RepStreamArgs sa, int reps) {
    using Kn = BsRepairStream<KD, M, 0, PARTS, LOADERS>;
    auto fn = &k_bs_repair_stream<KD, M, 0, PARTS, LOADERS, PROBE>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, Kn::LDS_BYTES);
    sa.region = uint32_t(((sa.r.sc + 7) / 8 + 31) / 32 * 32);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> t;
    for (int r = 0; r < reps; r++) {
        (void)hipEventRecord(e0);
        fn<<<dim3(sa.ns * 8), dim3(Kn::BLOCK), Kn::LDS_BYTES>>>(sa);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r >= 3) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

// the direct kernel k_bs_repair<10,4,0> (W = 128, global loads, one workgroup per tile)
static float run_direct10(RepArgs a, int reps) {
    using Kn = BsRepair<10, 4, 0>;
    a.b_start = 0;
    a.ntiles = uint32_t((a.sc + Kn::W - 1) / Kn::W);
    a.per_xcd = (a.ntiles + 7) / 8;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> t;
    for (int r = 0; r < reps; r++) {
        (void)hipEventRecord(e0);
        k_bs_repair<10, 4, 0><<<dim3(a.per_xcd * 8), dim3(Kn::BLOCK)>>>(a);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r >= 3) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

static int main10(uint64_t sc) {
    // (10,4,13): 16 internal nodes, 14 real (12, 13 shortened are virtual data nodes 10, 11 -> the
    // kernel's node index i < KD or i >= K = 12 is real); lost node 0, helpers 1..9, 12..15
    const uint64_t hbytes = 64 * sc, chunk = 256 * sc;
    uint8_t *h, *out;
    if (hipMalloc(&h, 16 * hbytes) != hipSuccess || hipMalloc(&out, chunk) != hipSuccess) return 1;
    {
        std::vector<uint8_t> v(16 * hbytes);
        uint64_t x = 0x9E3779B97F4A7C15ull;
        for (auto &b : v) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; b = uint8_t(x >> 24); }
        (void)hipMemcpy(h, v.data(), v.size(), hipMemcpyHostToDevice);
    }
    RepStreamArgs sa{};
    for (int i = 1; i < 16; i++) sa.r.h[i] = h + uint64_t(i) * hbytes;
    sa.r.out = out;
    sa.r.sc = sc;
    sa.r.x0 = 0;
    sa.r.full = 0;
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    sa.ns = uint32_t(cus / 8);
    const double bytes = double(13 * hbytes + chunk);
    auto rep = [&](const char *n, float ms) {
        printf("%-36s %8.4f ms  %7.1f GB/s (algorithmic)\n", n, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    for (int i = 0; i < 20; i++) run<8, 4, 0, 10, 4>(sa, 10);  // clocks up
    printf("(10,4,13) sc %llu\n", (unsigned long long)sc);
    for (int rr = 0; rr < 2; rr++) {
        rep("W256 L4 full", run<8, 4, 0, 10, 4>(sa, 15));
        rep("W256 L4 memory only (no math)", run<8, 4, 1, 10, 4>(sa, 15));
        rep("W256 L4 reads only", run<8, 4, 5, 10, 4>(sa, 15));
        rep("W256 L4 math + stores (no DMA)", run<8, 4, 2, 10, 4>(sa, 15));
        rep("W256 L4 no stores", run<8, 4, 4, 10, 4>(sa, 15));
        rep("W256 L2 full", run<8, 2, 0, 10, 4>(sa, 15));
        rep("W128 L4 full", run<4, 4, 0, 10, 4>(sa, 15));
        rep("W128 L4 memory only (no math)", run<4, 4, 1, 10, 4>(sa, 15));
        rep("W128 L4 reads only", run<4, 4, 5, 10, 4>(sa, 15));
        rep("W128 L4 math + stores (no DMA)", run<4, 4, 2, 10, 4>(sa, 15));
        rep("W128 L2 full", run<4, 2, 0, 10, 4>(sa, 15));
        rep("direct k_bs_repair (W128)", run_direct10(sa.r, 15));
    }
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 3 && atoi(argv[3]) == 10) return main10(argc > 1 && atoll(argv[1]) > 0 ? uint64_t(atoll(argv[1])) : 419432ull);
    const uint64_t sc = argc > 1 ? uint64_t(atoll(argv[1])) : 3314018ull;
    const uint64_t hbytes = 27 * sc, chunk = 81 * sc;
    uint8_t *h, *out;
    if (hipMalloc(&h, 12 * hbytes) != hipSuccess || hipMalloc(&out, chunk) != hipSuccess) return 1;
    {
        std::vector<uint8_t> v(12 * hbytes);
        uint64_t x = 0x9E3779B97F4A7C15ull;
        for (auto &b : v) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; b = uint8_t(x >> 24); }
        (void)hipMemcpy(h, v.data(), v.size(), hipMemcpyHostToDevice);
    }
    RepStreamArgs sa{};
    for (int i = 1; i < 12; i++) sa.r.h[i] = h + uint64_t(i) * hbytes;  // lost node 0 = (y0 0, x0 0)
    sa.r.out = out;
    sa.r.sc = sc;
    sa.r.x0 = 0;
    sa.r.full = 0;
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    sa.ns = uint32_t(cus / 8);
    const double bytes = double(11 * hbytes + chunk);
    auto rep = [&](const char *n, float ms) {
        printf("%-36s %8.4f ms  %7.1f GB/s (algorithmic)\n", n, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    for (int i = 0; i < 20; i++) run<16, 2, 0>(sa, 10);  // clocks up
    printf("sc %llu\n", (unsigned long long)sc);
    const bool sweep = argc > 2;
    for (int rr = 0; rr < 2; rr++) {
        rep("W512 L2 full", run<16, 2, 0>(sa, 15));
        rep("W512 L2 memory only (no math)", run<16, 2, 1>(sa, 15));
        if (sweep) {
            rep("W512 L1 full", run<16, 1, 0>(sa, 15));
            rep("W512 L7 full", run<16, 7, 0>(sa, 15));
            rep("W256 L1 full", run<8, 1, 0>(sa, 15));
            rep("W256 L7 full", run<8, 7, 0>(sa, 15));
            rep("W256 L7 memory only (no math)", run<8, 7, 1>(sa, 15));
            continue;
        }
        rep("W512 L2 reads only", run<16, 2, 5>(sa, 15));
        rep("W512 L2 math + stores (no DMA)", run<16, 2, 2>(sa, 15));
        rep("W512 L2 stores only", run<16, 2, 3>(sa, 15));
    }
    return 0;
}
