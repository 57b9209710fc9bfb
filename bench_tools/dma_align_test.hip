// Does global_load_lds_dwordx4 deliver correct bytes from 8-byte (not 16) aligned sources?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
__global__ void k(const uint8_t* src, uint32_t* out, int misalign) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    const uint8_t* p = src + misalign + threadIdx.x * 16;
    unsigned keep;
    uint32_t la = uint32_t(size_t((__attribute__((address_space(3))) uint8_t*)sm));
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "s"(la), "v"(p) : "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += 64) out[i] = reinterpret_cast<uint32_t*>(sm)[i];
}
int main() {
    std::vector<uint8_t> h(4096); for (int i = 0; i < 4096; i++) h[i] = uint8_t(i * 7 + 3);
    uint8_t* d; uint32_t* o; hipMalloc(&d, 4096); hipMalloc(&o, 1024);
    hipMemcpy(d, h.data(), 4096, hipMemcpyHostToDevice);
    for (int mis : {0, 1, 2, 3, 4, 6, 8, 12}) {
        hipMemset(o, 0, 1024);
        k<<<1, 64, 1024>>>(d, o, mis);
        std::vector<uint8_t> r(1024); hipMemcpy(r.data(), o, 1024, hipMemcpyDeviceToHost);
        int bad = 0; for (int i = 0; i < 1024; i++) bad += r[i] != h[mis + i];
        printf("misalign %2d: %s (%d bad bytes)\n", mis, bad ? "WRONG" : "ok", bad);
    }
    return 0;
}
