// kernels.hpp -- device-side GF(2^8) helpers shared by the Clay kernels (gfx950).
//
// Byte layout: 4 GF(2^8) symbols packed in a uint32 (SWAR).  Multiplication by a
// run-time constant c uses three v_perm_b32 byte lookups on the bit fields
// [2:0], [5:3], [7:6] of each byte (gf256.hpp perm_table); multiplication by
// gamma = 2 (transforms.rs:20) is the xtime shift-and-reduce for poly 0x11D.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace clay {

struct GfTab {
    uint32_t w0, w1, w2, w3, w4;
};

__device__ __forceinline__ GfTab load_tab(const uint32_t *__restrict__ t) {
    GfTab r;
    r.w0 = t[0];
    r.w1 = t[1];
    r.w2 = t[2];
    r.w3 = t[3];
    r.w4 = t[4];
    return r;
}

struct GfIdx {
    uint32_t i0, i1, i2;
};
__device__ __forceinline__ GfIdx gf_idx(uint32_t x) {
    GfIdx r;
    r.i0 = x & 0x07070707u;
    r.i1 = (x >> 3) & 0x07070707u;
    r.i2 = (x >> 6) & 0x03030303u;
    return r;
}
__device__ __forceinline__ uint32_t gf_mul_idx(const GfIdx &i, const GfTab &t) {
    return __builtin_amdgcn_perm(t.w1, t.w0, i.i0) ^ __builtin_amdgcn_perm(t.w3, t.w2, i.i1) ^
           __builtin_amdgcn_perm(t.w4, t.w4, i.i2);
}
__device__ __forceinline__ uint32_t gf_mul(uint32_t x, const GfTab &t) { return gf_mul_idx(gf_idx(x), t); }

// multiply 4 packed symbols by gamma = 2
__device__ __forceinline__ uint32_t gf_xt(uint32_t x) {
    uint32_t h = (x >> 7) & 0x01010101u;
    return ((x << 1) & 0xfefefefeu) ^ (h * 0x1du);
}

template <int N>
struct Words {
    uint32_t w[N];
};

template <int BYTES>
__device__ __forceinline__ Words<(BYTES + 3) / 4> vload(const uint8_t *p) {
    Words<(BYTES + 3) / 4> r;
    if constexpr (BYTES == 16) {
        uint4 v = *reinterpret_cast<const uint4 *>(p);
        r.w[0] = v.x; r.w[1] = v.y; r.w[2] = v.z; r.w[3] = v.w;
    } else if constexpr (BYTES == 8) {
        uint2 v = *reinterpret_cast<const uint2 *>(p);
        r.w[0] = v.x; r.w[1] = v.y;
    } else if constexpr (BYTES == 4) {
        r.w[0] = *reinterpret_cast<const uint32_t *>(p);
    } else if constexpr (BYTES == 2) {
        r.w[0] = *reinterpret_cast<const uint16_t *>(p);
    } else {
        r.w[0] = *p;
    }
    return r;
}

template <int BYTES>
__device__ __forceinline__ void vstore(uint8_t *p, const Words<(BYTES + 3) / 4> &v) {
    if constexpr (BYTES == 16) {
        *reinterpret_cast<uint4 *>(p) = make_uint4(v.w[0], v.w[1], v.w[2], v.w[3]);
    } else if constexpr (BYTES == 8) {
        *reinterpret_cast<uint2 *>(p) = make_uint2(v.w[0], v.w[1]);
    } else if constexpr (BYTES == 4) {
        *reinterpret_cast<uint32_t *>(p) = v.w[0];
    } else if constexpr (BYTES == 2) {
        *reinterpret_cast<uint16_t *>(p) = uint16_t(v.w[0]);
    } else {
        *p = uint8_t(v.w[0]);
    }
}

}  // namespace clay
