// valu_rate.hip -- issue rate of the VALU instructions the bit-sliced kernels are made of
// (v_bitop3_b32, v_xor_b32, v_perm_b32, v_lshlrev_b32) on gfx950: one workgroup per CU of
// WAVES waves (WAVES / 4 per SIMD), each lane running 16 independent chains of ITER x OP.
// Prints SIMD cycles per wave-instruction (clock from s_memtime inside the kernel).
// Build: hipcc --offload-arch=gfx950 -O3 -o bench_tools/valu_rate bench_tools/valu_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

template <int OP>
__device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b, uint32_t c) {
    if constexpr (OP == 0) return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
    if constexpr (OP == 1) return a ^ b;
    if constexpr (OP == 2) return __builtin_amdgcn_perm(a, b, c);
    if constexpr (OP == 3) return (a << 3) ^ 0;  // v_lshlrev
    return a;
}

template <int OP, int ITER>
__global__ void k_rate(uint32_t *out, uint64_t *cyc, uint32_t seed) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = seed * (threadIdx.x + 1) + uint32_t(i) * 0x9E3779B9u;
    const uint32_t b = seed ^ 0x5bd1e995u, c = seed + 0x0c0d0e0fu;
    __syncthreads();
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; it++) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            v[i] = op<OP>(v[i], b, c);
            asm volatile("" : "+v"(v[i]));
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) x ^= v[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
static void run(const char *name, int waves) {
    constexpr int ITER = 4096;
    uint32_t *out;
    uint64_t *cyc;
    (void)hipMalloc(&out, 256 * 1024 * 4);
    (void)hipMalloc(&cyc, 256 * 8);
    for (int r = 0; r < 3; r++) k_rate<OP, ITER><<<256, 64 * waves>>>(out, cyc, 7u);
    (void)hipDeviceSynchronize();
    std::vector<uint64_t> h(256);
    (void)hipMemcpy(h.data(), cyc, 256 * 8, hipMemcpyDeviceToHost);
    double avg = 0;
    for (auto x : h) avg += double(x);
    avg /= 256.0;
    const double instr_per_simd = double(ITER) * 16.0 * waves / 4.0;  // wave-instructions per SIMD
    printf("%-12s waves/CU %2d (%d per SIMD): %.2f cycles per wave-instruction per SIMD\n", name, waves, waves / 4,
           avg / instr_per_simd);
    fflush(stdout);
    (void)hipFree(out);
    (void)hipFree(cyc);
}

int main() {
    for (int w : {4, 8, 12, 16}) {  // waves per CU
        run<0>("v_bitop3", w);
        run<1>("v_xor", w);
        run<2>("v_perm", w);
        run<3>("v_lshlrev", w);
    }
    return 0;
}
