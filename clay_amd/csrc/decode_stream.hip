// decode_stream.hip -- instantiations and launchers of the streaming decode kernels (the local
// decode, stream_local.hpp, and the fused decode v2, stream_fused2.hpp), in their own translation
// unit so they compile in parallel with engine.hip.  The host-side planning (erasure pattern -> DecArgs) is in engine.hip.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <mutex>
#include <set>
#include <utility>

#include "stream_decode.hpp"
#include "stream_local.hpp"
#include "stream_fused2.hpp"
#include "tuning.hpp"

namespace clay {

template <int KD, int G>
static hipError_t launch_local(const bs::DecArgs &a, hipStream_t stream, int dev) {
    using Kn = bs::StreamDec<KD, G>;
    static std::mutex mu;
    static std::set<int> done;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!done.count(dev)) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&bs::k_stream_local<KD, G>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, Kn::LDS_BYTES);
            if (e != hipSuccess) return e;
            done.insert(dev);
        }
    }
    bs::k_stream_local<KD, G><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), Kn::LDS_BYTES, stream>>>(a);
    return hipGetLastError();
}

// the local decode (stream_local.hpp): erasures in section g plus at most one other section
hipError_t launch_stream_local_kernel(int kd, int g, const bs::DecArgs &a, hipStream_t stream, int dev) {
    if (kd == 10) {
        switch (g) {
        case 0: return launch_local<10, 0>(a, stream, dev);
        case 1: return launch_local<10, 1>(a, stream, dev);
        case 2: return launch_local<10, 2>(a, stream, dev);
        case 3: return launch_local<10, 3>(a, stream, dev);
        default: break;
        }
    } else if (kd == 9) {
        switch (g) {
        case 0: return launch_local<9, 0>(a, stream, dev);
        case 1: return launch_local<9, 1>(a, stream, dev);
        case 2: return launch_local<9, 2>(a, stream, dev);
        case 3: return launch_local<9, 3>(a, stream, dev);
        default: break;
        }
    }
    return hipErrorInvalidValue;
}

template <int KD, int PROBE = 0, bool TWO = false>
static hipError_t launch_f2(const bs::DecArgs &a, hipStream_t stream, int dev) {
    static std::mutex mu;
    static std::set<int> done;
    const int lds = int(a.ring + a.ne) * bs::kDecBuf;  // ring + S/C region (ne rows)
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!done.count(dev)) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&bs::k_stream_fused2<KD, 3, PROBE, TWO>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) return e;
            done.insert(dev);
        }
    }
    bs::k_stream_fused2<KD, 3, PROBE, TWO><<<dim3(a.nslots * 8), dim3(bs::StreamDec<KD, 3>::BLOCK), lds, stream>>>(a);
    return hipGetLastError();
}

// the fused decode v2 (stream_fused2.hpp): erasures in distinct y-sections, or (two = true, round
// 6) two erasures in some section
hipError_t launch_stream_fused2_kernel(int kd, const bs::DecArgs &a, hipStream_t stream, int dev, bool two) {
#ifdef CLAY_DECODE_PROBES
    const int probe = tuning().decode_probe;
    // the TWO instantiation: 31 no rounds, 32 no stores, 34 no phase-A math, 35 memory only, 40 timing
    if (two && kd == 10) {
        switch (probe) {
        case 31: return launch_f2<10, 1, true>(a, stream, dev);
        case 32: return launch_f2<10, 2, true>(a, stream, dev);
        case 34: return launch_f2<10, 4, true>(a, stream, dev);
        case 35: return launch_f2<10, 13, true>(a, stream, dev);
        case 40: return launch_f2<10, 16, true>(a, stream, dev);
        default: break;
        }
    }
#endif
    if (two) {
        if (kd == 10) return launch_f2<10, 0, true>(a, stream, dev);
        if (kd == 9) return launch_f2<9, 0, true>(a, stream, dev);
        return hipErrorInvalidValue;
    }
#ifdef CLAY_DECODE_PROBES
    // 31 no rounds, 32 no stores, 34 no phase-A math, 35 memory only, 36 no rounds / presolve,
    // 37 no rounds / stores, 38 no rounds / phase-A math (presolve kept), 39 no presolve
    // 40: the full kernel with s_memtime segment timing (workgroup 0 prints its compute wave 0 and
    // loader wave 0 totals); 41 / 42: the rounds at priority 0 (without / with the timing); 43 / 44:
    // phase A without the per-section compile-time copies (without / with the timing)
    if (kd == 10 && probe >= 31 && probe <= 44) {
        switch (probe) {
        case 40: return launch_f2<10, 16>(a, stream, dev);
        case 41: return launch_f2<10, 64>(a, stream, dev);
        case 42: return launch_f2<10, 64 | 16>(a, stream, dev);
        case 43: return launch_f2<10, 128>(a, stream, dev);
        case 44: return launch_f2<10, 128 | 16>(a, stream, dev);
        case 31: return launch_f2<10, 1>(a, stream, dev);
        case 32: return launch_f2<10, 2>(a, stream, dev);
        case 34: return launch_f2<10, 4>(a, stream, dev);
        case 35: return launch_f2<10, 13>(a, stream, dev);
        case 36: return launch_f2<10, 9>(a, stream, dev);
        case 37: return launch_f2<10, 3>(a, stream, dev);
        case 38: return launch_f2<10, 5>(a, stream, dev);
        case 39: return launch_f2<10, 8>(a, stream, dev);
        default: break;
        }
    }
#endif
    if (kd == 10) return launch_f2<10>(a, stream, dev);
    if (kd == 9) return launch_f2<9>(a, stream, dev);
    return hipErrorInvalidValue;
}

}  // namespace clay
