// repair_stream.hip -- instantiations and launchers of the bit-sliced repair kernels
// (repair_kernel.hpp), in their own translation unit; the host-side checks are in engine.hip.
#include <hip/hip_runtime.h>

#include <mutex>
#include <set>
#include <utility>

#include "repair_kernel.hpp"

namespace clay {

template <int KD, int M, int Y0>
static hipError_t launch_one(bs::RepArgs a, hipStream_t stream) {
    using Kn = bs::BsRepair<KD, M, Y0>;
    a.ntiles = uint32_t((a.sc - a.b_start + Kn::W - 1) / Kn::W);
    a.per_xcd = (a.ntiles + 7) / 8;
    bs::k_bs_repair<KD, M, Y0><<<dim3(a.per_xcd * 8), dim3(Kn::BLOCK), 0, stream>>>(a);
    return hipGetLastError();
}

// streaming variant: one workgroup per CU; returns hipErrorNotSupported when the launch should
// fall back to the direct kernel
template <int KD, int M, int Y0, int PARTS, int LOADERS>
static hipError_t launch_stream(const bs::RepArgs &a, hipStream_t stream, int dev, int cus, bool force,
                                int *launches, bool *streamed) {
    using Kn = bs::BsRepairStream<KD, M, Y0, PARTS, LOADERS>;
    const uint64_t nfull = a.sc / uint64_t(Kn::W);
    const uint32_t ns = uint32_t(cus >= 8 ? cus / 8 : 1);
    if (!force && nfull < uint64_t(8) * ns) return hipErrorNotSupported;  // under one tile per CU
    if (a.sc < 16) return hipErrorNotSupported;  // a partial tile reads whole 16-byte pieces
    if (a.sc * uint64_t(Kn::B::ALPHA) >= (uint64_t(1) << 32)) return hipErrorNotSupported;  // 32-bit row offsets
    {
        static std::mutex mu;
        static std::set<int> done;
        std::lock_guard<std::mutex> lk(mu);
        if (!done.count(dev)) {
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&bs::k_bs_repair_stream<KD, M, Y0, PARTS, LOADERS>),
                                               hipFuncAttributeMaxDynamicSharedMemorySize, Kn::LDS_BYTES);
            if (e != hipSuccess) return e;
            done.insert(dev);
        }
    }
    bs::RepStreamArgs sa{};
    sa.r = a;
    sa.region = uint32_t(((a.sc + 7) / 8 + 31) / 32 * 32);
    sa.ns = ns;
    bs::k_bs_repair_stream<KD, M, Y0, PARTS, LOADERS><<<dim3(ns * 8), dim3(Kn::BLOCK), Kn::LDS_BYTES, stream>>>(sa);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    *launches += 1;
    *streamed = true;
    return hipSuccess;
}

template <int KD, int M, int PARTS, int LOADERS>
static hipError_t launch_km(int y0, const bs::RepArgs &a, hipStream_t stream, int dev, int cus, int stream_mode,
                            bool *streamed, int *launches) {
    *streamed = false;
    *launches = 1;
    if constexpr (PARTS > 0) {
        if (stream_mode > 0) {
            *launches = 0;
            hipError_t e = hipErrorNotSupported;
            const bool force = stream_mode == 2;
            switch (y0) {
            case 0: e = launch_stream<KD, M, 0, PARTS, LOADERS>(a, stream, dev, cus, force, launches, streamed); break;
            case 1: e = launch_stream<KD, M, 1, PARTS, LOADERS>(a, stream, dev, cus, force, launches, streamed); break;
            case 2: e = launch_stream<KD, M, 2, PARTS, LOADERS>(a, stream, dev, cus, force, launches, streamed); break;
            default:
                if constexpr (bs::Shape<KD, M>::T > 3) e = launch_stream<KD, M, 3, PARTS, LOADERS>(a, stream, dev, cus, force, launches, streamed);
                break;
            }
            if (e != hipErrorNotSupported) return e;
            if (stream_mode == 3) return hipErrorNotSupported;  // streaming kernel only
            *launches = 1;
        }
    }
    if (stream_mode == 3) return hipErrorNotSupported;
    switch (y0) {
    case 0: return launch_one<KD, M, 0>(a, stream);
    case 1: return launch_one<KD, M, 1>(a, stream);
    case 2: return launch_one<KD, M, 2>(a, stream);
    default:
        if constexpr (bs::Shape<KD, M>::T > 3) return launch_one<KD, M, 3>(a, stream);
        return hipErrorInvalidValue;
    }
}

// stream_mode: 0 = direct kernel, 1 = streaming kernel when the sub-chunk gives every CU a
// tile, 2 = streaming kernel whenever the code has one, 3 = the streaming kernel when the
// sub-chunk gives every CU a tile, else nothing.  Returns 1 = direct kernel launched, 2 =
// streaming kernel launched, 0 = no instantiation for (k, m) (or none launched in mode 3), < 0 =
// HIP error; *launches = kernel launches issued.
int launch_bs_repair_kernel(int k, int m, int y0, const bs::RepArgs &a, hipStream_t stream, int dev, int cus,
                            int stream_mode, int *launches) {
    hipError_t e;
    bool streamed = false;
    if (k == 9 && m == 3) e = launch_km<9, 3, 16, 7>(y0, a, stream, dev, cus, stream_mode, &streamed, launches);
    // (10,4): 128-byte tiles (12.8 per CU on the 1 GiB stripe's 419,432-byte sub-chunks; 256-byte
    // tiles: 6.4 per CU and a longer tail, 0.161 vs 0.139 ms, profiles/r04/repair/)
    else if (k == 10 && m == 4) e = launch_km<10, 4, 4, 4>(y0, a, stream, dev, cus, stream_mode, &streamed, launches);
    else if (k == 4 && m == 2) e = launch_km<4, 2, 0, 0>(y0, a, stream, dev, cus, stream_mode, &streamed, launches);
    else return 0;
    if (e == hipErrorNotSupported && stream_mode == 3) return 0;
    if (e != hipSuccess) return -int(e);
    return streamed ? 2 : 1;
}

}  // namespace clay
