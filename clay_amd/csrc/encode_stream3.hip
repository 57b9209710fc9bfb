// encode_stream3.hip -- instantiations and launcher of the (9,3) streaming encode
// (stream_encode3.hpp), in their own translation unit so they compile in parallel.
#include <hip/hip_runtime.h>

#include <mutex>
#include <set>

#include "stream_encode3.hpp"

namespace clay {

template <int L>
static hipError_t launch3(const bs::Enc3Args &a, hipStream_t stream, int dev) {
    using Kn = bs::StreamEnc3<9, 3, L>;
    static std::mutex mu;
    static std::set<int> done;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!done.count(dev)) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&bs::k_stream_encode3<9, 3, L>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, Kn::LDS_BYTES);
            if (e != hipSuccess) return e;
            done.insert(dev);
        }
    }
    bs::k_stream_encode3<9, 3, L><<<dim3(a.ns * 8), dim3(Kn::BLOCK), Kn::LDS_BYTES, stream>>>(a);
    return hipGetLastError();
}

// (9,3) streaming encode of one stripe: loaders = 2 or 7 loader waves
hipError_t launch_stream_encode3_kernel(int loaders, const bs::Enc3Args &a, hipStream_t stream, int dev) {
    if (loaders == 7) return launch3<7>(a, stream, dev);
    return launch3<2>(a, stream, dev);
}

}  // namespace clay
