// line_kernels.hip -- instantiations and launchers of the line-local bit-sliced kernels
// (bitslice_line.hpp) for (4,2,5): the encode and the single-erasure decode of every node.
#include "bitslice_line.hpp"

namespace clay {

namespace {
constexpr int kPg = 64;  // 32-position groups per tile: 2048 positions, 4 lines x 64 lanes
}

template <int E>
static hipError_t launch42(bool bt, const bs::Dec1Args &a, hipStream_t stream) {
    using Kn = bs::Dec1Kernel<4, 2, E, kPg>;
    if (bt) bs::k_bs_decode1<4, 2, E, kPg, true><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), 0, stream>>>(a);
    else bs::k_bs_decode1<4, 2, E, kPg><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), 0, stream>>>(a);
    return hipGetLastError();
}

hipError_t launch_bs_decode1_kernel(int k, int m, int e, bool bt, const bs::Dec1Args &a, hipStream_t stream) {
    if (k == 4 && m == 2) {
        switch (e) {
        case 0: return launch42<0>(bt, a, stream);
        case 1: return launch42<1>(bt, a, stream);
        case 2: return launch42<2>(bt, a, stream);
        case 3: return launch42<3>(bt, a, stream);
        case 4: return launch42<4>(bt, a, stream);
        case 5: return launch42<5>(bt, a, stream);
        default: break;
        }
    }
    return hipErrorInvalidValue;
}

hipError_t launch_bs_encode1_kernel(int k, int m, bool bt, const bs::Enc1Args &a, hipStream_t stream) {
    if (k == 4 && m == 2) {
        using Kn = bs::Enc1Kernel<4, 2, kPg>;
        if (bt) bs::k_bs_encode1<4, 2, kPg, true><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), 0, stream>>>(a);
        else bs::k_bs_encode1<4, 2, kPg><<<dim3(a.nslots * 8), dim3(Kn::BLOCK), 0, stream>>>(a);
        return hipGetLastError();
    }
    return hipErrorInvalidValue;
}

int bs_decode1_tile(int k, int m) { return (k == 4 && m == 2) ? bs::Dec1Kernel<4, 2, 0, kPg>::W : 0; }

}  // namespace clay
