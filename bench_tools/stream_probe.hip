// stream_probe.hip -- where does the streaming encode kernel's time go?  Times
// k_stream_encode on the BASELINE (10,4,13) 1 GiB stripe with parts switched off
// (PROBE bits: 1 = no math, 2 = no DMA, 4 = no parity stores; the probes write wrong
// bytes and exist only in this tool, never in libclay_amd.so).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o bench_tools/stream_probe bench_tools/stream_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <vector>

#include "../clay_amd/csrc/stream_encode.hpp"

using namespace clay::bs;

template <int L, int PROBE>
static float run(BsArgs a, int reps) {
    using Kn = StreamEnc<10, L>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_stream_encode<10, L, PROBE>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, Kn::LDS_BYTES);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<float> t;
    for (int r = 0; r < reps; r++) {
        (void)hipEventRecord(e0);
        k_stream_encode<10, L, PROBE><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), Kn::LDS_BYTES>>>(a);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r >= 3) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

// steady state: n back-to-back launches between one pair of events (what bench.py and the
// profiler see); mean per launch
template <int L, int PROBE, int MAP = 0>
static float run_b2b(BsArgs a, int n, int warm = 50) {
    using Kn = StreamEnc<10, L>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_stream_encode<10, L, PROBE, MAP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, Kn::LDS_BYTES);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < warm; i++)
        k_stream_encode<10, L, PROBE, MAP><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), Kn::LDS_BYTES>>>(a);
    (void)hipEventRecord(e0);
    for (int i = 0; i < n; i++)
        k_stream_encode<10, L, PROBE, MAP><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), Kn::LDS_BYTES>>>(a);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
        printf("HIP error (probe %d): %s\n", PROBE, hipGetErrorString(err));
        exit(3);
    }
    return ms / float(n);
}

// Segment timing (PROBE 4096, stream_encode.hpp TimeAcc): per-workgroup s_memtime sums of the
// last of `n` back-to-back launches, then one single launch timed with events to convert cycles
// to time.  Prints per-tile averages over the workgroups and the start / end spread.
template <int TP, int MAP = 0>
static void timing_report(BsArgs a, int n) {
    using Kn = StreamEnc<10, 4>;
    const int grid = int(a.nslots) * 8;
    const size_t rec = size_t(grid) * 12 * 24;
    uint64_t *tb;
    (void)hipMalloc(&tb, rec * 8);
    (void)hipMemset(tb, 0, rec * 8);
    a.par[4] = reinterpret_cast<uint8_t *>(tb);
    const float ms_plain = run_b2b<4, 0, MAP>(a, n);
    const float ms_tm = run_b2b<4, TP, MAP>(a, n);
    std::vector<uint64_t> h(rec);
    (void)hipMemcpy(h.data(), tb, rec * 8, hipMemcpyDeviceToHost);
    printf("b2b ms: plain %.4f  timing-probe %.4f (s_memtime counts per XCD; cycles below are per tile)\n", ms_plain, ms_tm);
    printf("wave  role     total   bar/vm y0   y1    y2 | math/bar y0   y1    y2 | issue y0  y1    y2 | end g0  g1    g2    g3\n");
    for (int w = 0; w < 12; w++) {
        double v[3][3] = {}, ge[4] = {}, tot = 0;
        int cnt = 0;
        for (int b = 0; b < grid; b++) {
            const uint64_t *p = &h[(size_t(b) * 12 + w) * 24];
            const double nt = double(p[16]);
            if (nt == 0) continue;
            cnt++;
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) v[i][j] += double(p[i * 3 + j]) / nt;
            for (int g = 0; g < 4; g++) ge[g] += double(p[9 + g]) / nt;
            tot += double(p[15] - p[13]) / nt;
        }
        const double G = cnt ? cnt : 1;
        printf("%4d  %-7s %7.0f  %6.0f %6.0f %6.0f | %6.0f %6.0f %6.0f | %6.0f %6.0f %6.0f | %5.0f %5.0f %5.0f %5.0f\n", w,
               w < 8 ? "compute" : "loader", tot / G, v[0][0] / G, v[0][1] / G, v[0][2] / G, v[1][0] / G, v[1][1] / G,
               v[1][2] / G, v[2][0] / G, v[2][1] / G, v[2][2] / G, ge[0] / G, ge[1] / G, ge[2] / G, ge[3] / G);
    }
    fflush(stdout);
    (void)hipFree(tb);
    (void)Kn::BLOCK;
}

int main(int argc, char **argv) {
    // sc of the BASELINE stripe by default; another value (e.g. 419456 = 128-aligned rows)
    // isolates the cost of the 8-byte row alignment of the reference layout
    const uint32_t sc = argc > 1 ? uint32_t(atoi(argv[1])) : 419432;
    const bool quick = argc > 2;
    const size_t chunk = size_t(sc) * 256;
    uint8_t *data, *par;
    if (hipMalloc(&data, 10 * chunk) != hipSuccess || hipMalloc(&par, 4 * chunk) != hipSuccess) return 1;
    {  // random bytes: the XOR networks' switching power sets the clock (constant data runs faster)
        std::vector<uint8_t> h(10 * chunk);
        uint64_t x = 0x9E3779B97F4A7C15ull;
        for (auto &b : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; b = uint8_t(x >> 24); }
        (void)hipMemcpy(data, h.data(), h.size(), hipMemcpyHostToDevice);
    }
    BsArgs a{};
    for (int i = 0; i < 10; i++) a.data[i] = data + i * chunk;
    for (int x = 0; x < 4; x++) a.par[x] = par + x * chunk;
    a.sc = sc;
    // XCD region: sc / 8 rounded up to 32 bytes (the library's), or to argv[3] bytes (alignment A/B)
    const uint32_t ralign = argc > 3 ? uint32_t(atoi(argv[3])) : 32u;
    a.tiles_per_xcd = uint32_t(((sc + 7) / 8 + ralign - 1) / ralign * ralign);
    a.nslots = 32;
    const double bytes = 14.0 * chunk;
    auto rep = [&](const char *n, float ms) {
        printf("%-34s %8.4f ms  %7.1f GB/s (algorithmic)\n", n, ms, bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_stream_encode<10, 2, 0>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, StreamEnc<10, 2>::LDS_BYTES);
    for (int i = 0; i < 300; i++) k_stream_encode<10, 2, 0><<<dim3(a.nslots * 8), dim3(StreamEnc<10, 2>::BLOCK), StreamEnc<10, 2>::LDS_BYTES>>>(a);
    {
        const hipError_t e = hipDeviceSynchronize();
        const hipError_t e2 = hipGetLastError();
        if (e != hipSuccess || e2 != hipSuccess) {
            printf("HIP error after warm-up: %s / %s\n", hipGetErrorString(e), hipGetErrorString(e2));
            return 3;
        }
    }
    if (argc > 2 && argv[2][0] == 't') {  // segment timing of the full kernel
        printf("sc %u segment timing\n", sc);
        timing_report<4096>(a, 200);
        printf("---- deferred end of group (PROBE 8192)\n");
        timing_report<4096 | 8192>(a, 200);
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'd') {  // deferred end-of-group work (PROBE 8192) A/B
        printf("sc %u deferred end-of-group A/B, back-to-back\n", sc);
        for (int rr = 0; rr < 3; rr++) {
            rep("b2b full", run_b2b<4, 0>(a, 200));
            rep("b2b full, end of group after the next barrier", run_b2b<4, 8192>(a, 200));
            rep("b2b memory only", run_b2b<4, 1>(a, 200));
            rep("b2b memory only, deferred", run_b2b<4, 8193>(a, 200));
            rep("b2b full, no sched barrier between nodes", run_b2b<4, 16384>(a, 200));
            rep("b2b full, sched barrier every 2 nodes", run_b2b<4, 32768>(a, 200));
            rep("b2b full, deferred + every 2 nodes", run_b2b<4, 32768 | 8192>(a, 200));
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'p') {  // balanced issue priority (PROBE 131072) A/B
        printf("sc %u balanced priority A/B, back-to-back\n", sc);
        for (int rr = 0; rr < 3; rr++) {
            rep("b2b full", run_b2b<4, 0>(a, 200));
            rep("b2b full, balanced priority", run_b2b<4, 131072>(a, 200));
            rep("b2b math + stores (no DMA)", run_b2b<4, 2>(a, 200));
            rep("b2b math + stores (no DMA), balanced priority", run_b2b<4, 2 | 131072>(a, 200));
        }
        timing_report<4096 | 131072>(a, 200);
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'v') {  // steady-state variants: which parts add
        // live = SINK probes (stream_encode.hpp PROBE 262144): the end-of-group work runs and the
        // parity stores become XORs into a sink, so the math cannot be deleted (the
        // round-5 "no stores" variants 4 / 6 compiled to 4 / 3 v_bitop3 and timed nothing)
        printf("sc %u variants, back-to-back (200 launches after 50 untimed)\n", sc);
        for (int rr = 0; rr < 3; rr++) {
            rep("b2b full", run_b2b<4, 0>(a, 200));
            rep("b2b memory only (DMA + stores, no math)", run_b2b<4, 1>(a, 200));
            rep("b2b reads only", run_b2b<4, 5>(a, 200));
            rep("b2b stores only", run_b2b<4, 3>(a, 200));
            rep("b2b live reads + math (no stores)", run_b2b<4, 262144>(a, 200));
            rep("b2b live math only (no DMA, no stores)", run_b2b<4, 262146>(a, 200));
            rep("b2b math + stores (no DMA)", run_b2b<4, 2>(a, 200));
            rep("b2b math + stores, no DMA, no barriers", run_b2b<4, 2 | 65536>(a, 200));
            rep("b2b live math only, no barriers", run_b2b<4, 262146 | 65536>(a, 200));
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'n') {  // round-6 lane map (MAP 1: light section 2 on waves 4-7; MAP 2: on 0-3)
        printf("sc %u lane map A/B, back-to-back (200 launches after 50 untimed)\n", sc);
        if (argv[2][1] == 't') {  // segment timing of the maps
            timing_report<4096, 0>(a, 200);
            printf("---- map 3\n");
            timing_report<4096, 3>(a, 200);
            return 0;
        }
        // bytes of every map against map 0 (the library's, parity-tested against the oracle)
        const size_t pbytes = 4 * chunk;
        std::vector<uint8_t> ref(pbytes), got(pbytes);
        auto snap = [&](std::vector<uint8_t> &v) {
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(v.data(), par, pbytes, hipMemcpyDeviceToHost);
        };
        (void)hipMemset(par, 0, pbytes);
        run_b2b<4, 0, 0>(a, 1, 0);
        snap(ref);
        auto check = [&](const char *name) {
            snap(got);
            printf("  bytes %s == map 0: %s\n", name, ref == got ? "yes" : "NO");
            (void)hipMemset(par, 0, pbytes);
        };
        run_b2b<4, 0, 1>(a, 1, 0); check("map 1");
        run_b2b<4, 0, 3>(a, 1, 0); check("map 3");
        run_b2b<4, 0, 4>(a, 1, 0); check("map 4");
        run_b2b<4, 0, 5>(a, 1, 0); check("map 5");
        run_b2b<4, 0, 6>(a, 1, 0); check("map 6");
        run_b2b<4, 0, 7>(a, 1, 0); check("map 7");
        run_b2b<4, 0, 8>(a, 1, 0); check("map 8");
        run_b2b<4, 0, 9>(a, 1, 0); check("map 9");
        if (argv[2][1] == '8') {  // map 8 / 9 (red skip A/B), map 0, priorities
            for (int rr = 0; rr < 3; rr++) {
                rep("b2b full, map 0 (round 5)", run_b2b<4, 0, 0>(a, 200));
                rep("b2b full, map 8", run_b2b<4, 0, 8>(a, 200));
                rep("b2b full, map 9 (map 8 without red skip)", run_b2b<4, 0, 9>(a, 200));
                rep("b2b full, map 8, waves 4-7 prio 1", run_b2b<4, 16, 8>(a, 200));
                rep("b2b full, map 8, no sched barriers", run_b2b<4, 16384, 8>(a, 200));
                rep("b2b full, map 8, sched barrier / 2 nodes", run_b2b<4, 32768, 8>(a, 200));
                rep("b2b memory only, map 8", run_b2b<4, 1, 8>(a, 200));
                rep("b2b live math only, map 8", run_b2b<4, 262146, 8>(a, 200));
                rep("b2b live reads + math, map 8", run_b2b<4, 262144, 8>(a, 200));
                rep("b2b math + stores, map 8", run_b2b<4, 2, 8>(a, 200));
            }
            timing_report<4096, 8>(a, 200);
            return 0;
        }
        for (int rr = 0; rr < 3; rr++) {
            rep("b2b full, map 0 (round 5)", run_b2b<4, 0, 0>(a, 200));
            rep("b2b memory only, map 0", run_b2b<4, 1, 0>(a, 200));
            rep("b2b full, map 1 (k 2,3,4 pair 16)", run_b2b<4, 0, 1>(a, 200));
            rep("b2b memory only, map 1", run_b2b<4, 1, 1>(a, 200));
            rep("b2b full, map 3 (map 1, permlane pair 32)", run_b2b<4, 0, 3>(a, 200));
            rep("b2b full, map 4 (k 3,2,4 pair 32)", run_b2b<4, 0, 4>(a, 200));
            rep("b2b memory only, map 4", run_b2b<4, 1, 4>(a, 200));
            rep("b2b full, map 5 (k 4,3,2 pair 64)", run_b2b<4, 0, 5>(a, 200));
            rep("b2b memory only, map 5", run_b2b<4, 1, 5>(a, 200));
            rep("b2b full, map 6 (k 5,4,3 pair 128)", run_b2b<4, 0, 6>(a, 200));
            rep("b2b memory only, map 6", run_b2b<4, 1, 6>(a, 200));
            rep("b2b full, map 7 (k 2,5,4 pair 16)", run_b2b<4, 0, 7>(a, 200));
            rep("b2b memory only, map 7", run_b2b<4, 1, 7>(a, 200));
            rep("b2b full, map 8 (k 4,5,3 pair 64)", run_b2b<4, 0, 8>(a, 200));
            rep("b2b memory only, map 8", run_b2b<4, 1, 8>(a, 200));
            rep("b2b live math only, map 1", run_b2b<4, 262146, 1>(a, 200));
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'w') {  // the 'v' variants, 10 launches each (for one rocprofv3 --pmc pass)
        rep("full", run_b2b<4, 0>(a, 10, 2));
        rep("memory only", run_b2b<4, 1>(a, 10, 2));
        rep("reads only", run_b2b<4, 5>(a, 10, 2));
        rep("stores only", run_b2b<4, 3>(a, 10, 2));
        rep("live reads + math", run_b2b<4, 262144>(a, 10, 2));
        rep("live math only", run_b2b<4, 262146>(a, 10, 2));
        rep("math + stores", run_b2b<4, 2>(a, 10, 2));
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'f') {  // the no-barrier timing probe, bounds-checked
        unsigned int *flag;
        (void)hipMalloc(&flag, 4);
        (void)hipMemset(flag, 0, 4);
        a.par[5] = reinterpret_cast<uint8_t *>(flag);
        printf("sc %u no-barrier timing probe (PROBE 4096|65536|2) with bounds checks (524288)\n", sc);
        timing_report<4096 | 65536 | 2 | 524288>(a, 50);
        unsigned int h = 0;
        (void)hipMemcpy(&h, flag, 4, hipMemcpyDeviceToHost);
        printf("bounds flags 0x%x (bits 0-3 parity store of node X, 4-7 ragged store, 8 compute record, 9 loader record)\n", h);
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'a') {  // alignment A/B: run with sc and region alignment from argv
        printf("sc %u (row start mod 128 varies: %s), XCD region %u (alignment %u)\n", sc,
               sc % 128 ? "yes" : "no, rows 128-aligned", a.tiles_per_xcd, ralign);
        for (int rr = 0; rr < 2; rr++) {
            rep("b2b full", run_b2b<4, 0>(a, 200));
            rep("b2b memory only (DMA + stores)", run_b2b<4, 1>(a, 200));
            rep("b2b stores only", run_b2b<4, 3>(a, 200));
            rep("b2b reads only", run_b2b<4, 5>(a, 200));
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'l') {  // steady state: loader-wave count
        printf("sc %u back-to-back loader sweep\n", sc);
        for (int rr = 0; rr < 3; rr++) {
            rep("b2b L4 full", run_b2b<4, 0>(a, 200));
            rep("b2b L2 full", run_b2b<2, 0>(a, 200));
            rep("b2b L1 full", run_b2b<1, 0>(a, 200));
            rep("b2b L4 full, loaders prio 0", run_b2b<4, 8>(a, 200));
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'b') {  // steady state, back-to-back launches
        printf("sc %u back-to-back (200 launches after 50 untimed)\n", sc);
        for (int rr = 0; rr < 3; rr++) {
            rep("b2b L4 full (CSE)", run_b2b<4, 0>(a, 200));
            rep("b2b L4 full, no CSE", run_b2b<4, 1024>(a, 200));
            rep("b2b L4 memory only", run_b2b<4, 1>(a, 200));
            rep("b2b L4 math + stores (CSE)", run_b2b<4, 2>(a, 200));
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'm') {  // tile map A/B (PROBE bit 2048 = chip round robin)
        printf("sc %u tile map (XCD-blocked vs chip round robin), back-to-back\n", sc);
        for (int rr = 0; rr < 3; rr++) {
            rep("b2b full, XCD-blocked", run_b2b<4, 0>(a, 200));
            rep("b2b full, chip RR", run_b2b<4, 2048>(a, 200));
            rep("b2b memory only, XCD-blocked", run_b2b<4, 1>(a, 200));
            rep("b2b memory only, chip RR", run_b2b<4, 2049>(a, 200));
            rep("b2b stores only, XCD-blocked", run_b2b<4, 3>(a, 200));
            rep("b2b stores only, chip RR", run_b2b<4, 2051>(a, 200));
            rep("b2b reads only, XCD-blocked", run_b2b<4, 5>(a, 200));
            rep("b2b reads only, chip RR", run_b2b<4, 2053>(a, 200));
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'x') {  // CSE folds A/B (PROBE bit 1024 = without)
        printf("sc %u cse folds\n", sc);
        for (int rr = 0; rr < 3; rr++) {
            rep("L4 full, row-by-row folds", run<4, 1024>(a, 15));
            rep("L4 full (CSE folds)", run<4, 0>(a, 15));
            rep("L0 full, row-by-row folds", run<0, 1024>(a, 15));
            rep("L0 full (CSE folds)", run<0, 0>(a, 15));
            rep("L4 math + stores, row-by-row folds", run<4, 1026>(a, 15));
            rep("L4 math + stores (CSE folds)", run<4, 2>(a, 15));
        }
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'c') {  // cache-policy A/B (PROBE bits 64..512)
        printf("sc %u cache policies\n", sc);
        for (int rr = 0; rr < 2; rr++) {
            rep("L4 full", run<4, 0>(a, 15));
            rep("L4 full, nt loads", run<4, 64>(a, 15));
            rep("L4 full, nt stores", run<4, 256>(a, 15));
            rep("L4 full, nt loads + stores", run<4, 320>(a, 15));
            rep("L4 full, sc1 loads", run<4, 128>(a, 15));
            rep("L4 full, sc1 stores", run<4, 512>(a, 15));
            rep("L4 memory only", run<4, 1>(a, 15));
            rep("L4 memory only, nt loads", run<4, 65>(a, 15));
            rep("L4 memory only, nt stores", run<4, 257>(a, 15));
            rep("L4 memory only, nt both", run<4, 321>(a, 15));
            rep("L4 reads, nt", run<4, 69>(a, 15));
            rep("L4 stores only, nt", run<4, 259>(a, 15));
        }
        return 0;
    }
    if (quick) {
        printf("sc %u\n", sc);
        for (int rr = 0; rr < 2; rr++) {
            rep("L4 full", run<4, 0>(a, 15));
            rep("L4 no math (memory only)", run<4, 1>(a, 15));
            rep("L4 reads", run<4, 5>(a, 15));
            rep("L4 stores only", run<4, 3>(a, 15));
            rep("L4 memory only, rotated stores", run<4, 33>(a, 15));
            rep("L4 stores only, rotated", run<4, 35>(a, 15));
        }
        return 0;
    }
    for (int rr = 0; rr < 2; rr++) {
        rep("L0 full", run<0, 0>(a, 15));
        rep("L1 full", run<1, 0>(a, 15));
        rep("L2 full", run<2, 0>(a, 15));
        rep("L4 full loaders prio 0", run<4, 8>(a, 15));
        rep("L4 full waves 4-7 prio 1", run<4, 16>(a, 15));
        rep("L2 full waves 4-7 prio 1", run<2, 16>(a, 15));
        rep("L4 full", run<4, 0>(a, 15));
        rep("L0 no math (memory only)", run<0, 1>(a, 15));
        rep("L4 no math (memory only)", run<4, 1>(a, 15));
        rep("L0 reads", run<0, 5>(a, 15));
        rep("L4 reads", run<4, 5>(a, 15));
        rep("L4 no DMA (math + stores)", run<4, 2>(a, 15));
        rep("L4 stores only", run<4, 3>(a, 15));
    }
    return 0;
}
