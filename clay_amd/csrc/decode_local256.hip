// decode_local256.hip -- instantiations and launcher of the local decode on 256-byte row runs
// (stream_local256.hpp), in its own translation unit so it compiles in parallel with the others;
// built twice: LOCAL256_ANY = 0 (8-byte rows) and 1 (any sub-chunk, decode_local256_any.hip).
// The host-side planning (erasure pattern -> DecArgs) is in engine.hip.
#include <hip/hip_runtime.h>

#include <mutex>
#include <set>

#include "stream_local256.hpp"

#ifndef LOCAL256_ANY
#define LOCAL256_ANY 0
#endif

namespace clay {

constexpr bool kAny = LOCAL256_ANY != 0;

template <int KD, int G, int NE>
static hipError_t launch_l256(const bs::DecArgs &a, hipStream_t stream, int dev) {
    using Kn = bs::Local256<KD, G, NE, kAny>;
    static std::mutex mu;
    static std::set<int> done;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!done.count(dev)) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&bs::k_stream_local256<KD, G, NE, kAny>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, Kn::LDS_BYTES);
            if (e != hipSuccess) return e;
            done.insert(dev);
        }
    }
    bs::k_stream_local256<KD, G, NE, kAny><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), Kn::LDS_BYTES, stream>>>(a);
    return hipGetLastError();
}

template <int KD, int NE>
static hipError_t launch_l256_g(int g, const bs::DecArgs &a, hipStream_t stream, int dev) {
    switch (g) {
    case 0: return launch_l256<KD, 0, NE>(a, stream, dev);
    case 1: return launch_l256<KD, 1, NE>(a, stream, dev);
    case 2: return launch_l256<KD, 2, NE>(a, stream, dev);
    case 3: return launch_l256<KD, 3, NE>(a, stream, dev);
    default: return hipErrorInvalidValue;
    }
}

// one erasure in section g plus at most one in another section, or two in g (ne = 1 or 2)
#if LOCAL256_ANY
hipError_t launch_stream_local256_any_kernel(int kd, int g, const bs::DecArgs &a, hipStream_t stream, int dev) {
#else
hipError_t launch_stream_local256_kernel(int kd, int g, const bs::DecArgs &a, hipStream_t stream, int dev) {
#endif
    if (kd == 10) return a.ne == 1 ? launch_l256_g<10, 1>(g, a, stream, dev) : launch_l256_g<10, 2>(g, a, stream, dev);
    if (kd == 9) return a.ne == 1 ? launch_l256_g<9, 1>(g, a, stream, dev) : launch_l256_g<9, 2>(g, a, stream, dev);
    return hipErrorInvalidValue;
}

}  // namespace clay
