// decode_stream.hip -- instantiations and launcher of the streaming decode kernel
// (stream_decode.hpp), in their own translation unit so they compile in parallel with
// engine.hip.  The host-side planning (erasure pattern -> DecArgs) is in engine.hip.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <mutex>
#include <set>
#include <utility>

#include "stream_decode.hpp"

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

hipError_t launch_stream_decode_kernel(int kd, const bs::DecArgs &a, hipStream_t stream, int dev) {
#ifdef CLAY_DECODE_PROBES
    // CLAY_DECODE_PROBE: skip parts of the kernel (measurement only: the probe library
    // libclay_amd_probe.so, `make probe`; the product library has no probe instantiations)
    static const int probe = [] {
        const char *e = getenv("CLAY_DECODE_PROBE");
        return e ? atoi(e) : 0;
    }();
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
    if (kd == 10) return launch_one<10, 3>(a, stream, dev);
    if (kd == 9) return launch_one<9, 3>(a, stream, dev);
    return hipErrorInvalidValue;
}

}  // namespace clay
