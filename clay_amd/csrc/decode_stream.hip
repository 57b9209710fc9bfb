// decode_stream.hip -- instantiations and launcher of the streaming decode kernel
// (stream_decode.hpp), in their own translation unit so they compile in parallel with
// engine.hip.  The host-side planning (erasure pattern -> DecArgs) is in engine.hip.
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

template <int KD, int G, int PROBE = 0>
static hipError_t launch_one(const bs::DecArgs &a, hipStream_t stream, int dev) {
    using Kn = bs::StreamDec<KD, G>;
    static std::mutex mu;
    static std::set<int> done;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!done.count(dev)) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&bs::k_stream_decode<KD, G, PROBE>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, Kn::LDS_BYTES);
            if (e != hipSuccess) return e;
            done.insert(dev);
        }
    }
    bs::k_stream_decode<KD, G, PROBE><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), Kn::LDS_BYTES, stream>>>(a);
    return hipGetLastError();
}

template <int KD, int G, int SPROBE = 0, int SKIP = 0, int YPROBE = 0>
static hipError_t launch_split(const bs::DecArgs &a, hipStream_t stream, int dev) {
    using Kn = bs::StreamDec<KD, G>;
    static std::mutex mu;
    static std::set<int> done;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!done.count(dev)) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&bs::k_stream_syn<KD, G, YPROBE>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, Kn::LDS_BYTES);
            if (e == hipSuccess)
                e = hipFuncSetAttribute(reinterpret_cast<const void *>(&bs::k_stream_solve<KD, G, SPROBE>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, bs::kSolveLds);
            if (e != hipSuccess) return e;
            done.insert(dev);
        }
    }
    if (!(SKIP & 1)) {
        bs::k_stream_syn<KD, G, YPROBE><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), Kn::LDS_BYTES, stream>>>(a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (SKIP & 2) return hipSuccess;
    bs::DecArgs b = a;  // solve: 128-byte tiles, XCD regions of whole tiles, one workgroup per CU
    const uint32_t nst = uint32_t((a.sc + 127) / 128);
    b.region = (nst + 7) / 8 * 128;
    bs::k_stream_solve<KD, G, SPROBE><<<dim3(b.nslots * 8), dim3(1024), bs::kSolveLds, stream>>>(b);
    return hipGetLastError();
}

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

template <int KD, int PROBE = 0>
static hipError_t launch_f2(const bs::DecArgs &a, hipStream_t stream, int dev) {
    static std::mutex mu;
    static std::set<int> done;
    const int lds = int(a.ring + a.ne) * bs::kDecBuf;  // ring + S/C region (ne rows)
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!done.count(dev)) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&bs::k_stream_fused2<KD, 3, PROBE>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            if (e != hipSuccess) return e;
            done.insert(dev);
        }
    }
    bs::k_stream_fused2<KD, 3, PROBE><<<dim3(a.nslots * 8), dim3(bs::StreamDec<KD, 3>::BLOCK), lds, stream>>>(a);
    return hipGetLastError();
}

// the fused decode v2 (stream_fused2.hpp): one erasure per y-section
hipError_t launch_stream_fused2_kernel(int kd, const bs::DecArgs &a, hipStream_t stream, int dev) {
#ifdef CLAY_DECODE_PROBES
    const int probe = tuning().decode_probe;
    // 31 no rounds, 32 no stores, 34 no phase-A math, 35 memory only, 36 no rounds / presolve,
    // 37 no rounds / stores, 38 no rounds / phase-A math (presolve kept), 39 no presolve
    // 40: the full kernel with s_memtime segment timing (workgroup 0 prints its compute wave 0 and
    // loader wave 0 totals)
    if (kd == 10 && probe >= 31 && probe <= 40) {
        switch (probe) {
        case 40: return launch_f2<10, 16>(a, stream, dev);
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

// a.ws != nullptr: split decode (two launches), else the fused single-launch kernel
hipError_t launch_stream_decode_kernel(int kd, const bs::DecArgs &a, hipStream_t stream, int dev) {
#ifdef CLAY_DECODE_PROBES
    // CLAY_DECODE_PROBE: skip parts of the kernel (measurement only: the probe library
    // libclay_amd_probe.so, `make probe`; the product library has no probe instantiations)
    const int probe = tuning().decode_probe;
    if (kd == 10 && probe && a.ws) {
        switch (probe) {  // split decode: 11 solve no work, 12 solve no stores, 13 syn only, 14 solve only,
                          // 15 solve no S DMA
        case 11: return launch_split<10, 3, 1>(a, stream, dev);
        case 12: return launch_split<10, 3, 2>(a, stream, dev);
        case 13: return launch_split<10, 3, 0, 2>(a, stream, dev);
        case 14: return launch_split<10, 3, 0, 1>(a, stream, dev);
        case 15: return launch_split<10, 3, 4>(a, stream, dev);
        case 16: return launch_split<10, 3, 8, 1>(a, stream, dev);   // solve only, no presolve
        case 17: return launch_split<10, 3, 16, 1>(a, stream, dev);  // solve only, no rounds
        case 18: return launch_split<10, 3, 3, 1>(a, stream, dev);   // solve only: S DMA only
        case 19: return launch_split<10, 3, 5, 1>(a, stream, dev);   // solve only: output stores only
        case 20: return launch_split<10, 3, 1, 1>(a, stream, dev);   // solve only: DMA + stores
        case 21: return launch_split<10, 3, 0, 2, 2>(a, stream, dev);  // syn only, no phase-A math
        case 22: return launch_split<10, 3, 0, 2, 4>(a, stream, dev);  // syn only, no DMA
        case 23: return launch_split<10, 3, 32, 1>(a, stream, dev);    // solve only, nt output stores
        case 24: return launch_split<10, 3, 37, 1>(a, stream, dev);    // solve only, nt stores only
        default: break;
        }
    }
    if (kd == 10 && probe) {
        switch (probe) {
        case 1: return launch_one<10, 3, 1>(a, stream, dev);
        case 2: return launch_one<10, 3, 2>(a, stream, dev);
        case 3: return launch_one<10, 3, 3>(a, stream, dev);
        case 7: return launch_one<10, 3, 7>(a, stream, dev);
        default: break;
        }
    }
#endif
    if (a.ws) {
        if (kd == 10) return launch_split<10, 3>(a, stream, dev);
        if (kd == 9) return launch_split<9, 3>(a, stream, dev);
        return hipErrorInvalidValue;
    }
    if (kd == 10) return launch_one<10, 3>(a, stream, dev);
    if (kd == 9) return launch_one<9, 3>(a, stream, dev);
    return hipErrorInvalidValue;
}

}  // namespace clay
