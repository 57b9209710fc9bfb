// gf256.hpp -- host-side GF(2^8) and Reed-Solomon generator math for the planner.
//
// Field and code construction are those of the reference's RS dependency,
// reed-solomon-erasure 6.0.0 (Cargo.lock:496-508; call sites transforms.rs:15,
// decode.rs:9,176-180, repair.rs:207-211): polynomial 0x11D, generator 2,
// systematic matrix = vandermonde(total, data) * inverse(top data x data).
// Only matrices/coefficients are computed here; all byte work runs on the GPU.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace clay {

struct GF {
    uint8_t exp[512];
    uint8_t log[256];
    uint8_t mul_[256][256];

    static const GF &get() {
        static const GF g;
        return g;
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return mul_[a][b]; }
    uint8_t inv(uint8_t a) const { return a ? exp[255 - log[a]] : 0; }
    uint8_t div(uint8_t a, uint8_t b) const {  // b != 0
        if (!a) return 0;
        int l = int(log[a]) - int(log[b]);
        return exp[l < 0 ? l + 255 : l];
    }
    uint8_t pow(uint8_t a, size_t n) const {
        if (n == 0) return 1;
        if (a == 0) return 0;
        return exp[(size_t(log[a]) * n) % 255];
    }

  private:
    GF() {
        unsigned b = 1;
        for (int i = 0; i < 255; i++) {
            exp[i] = uint8_t(b);
            log[b] = uint8_t(i);
            b <<= 1;
            if (b & 0x100) b ^= 0x11D;
        }
        for (int i = 255; i < 512; i++) exp[i] = exp[i - 255];
        log[0] = 0;
        for (int a = 0; a < 256; a++)
            for (int c = 0; c < 256; c++)
                mul_[a][c] = (a && c) ? exp[log[a] + log[c]] : 0;
    }
};

// Clay pairwise-transform constants (transforms.rs:20, :307-308, decode.rs:569)
constexpr uint8_t kGamma = 2;
inline uint8_t gamma_det() { return 1 ^ GF::get().mul(kGamma, kGamma); }      // 1 + g^2 = 5
inline uint8_t gamma_det_inv() { return GF::get().inv(gamma_det()); }          // 0xA7
inline uint8_t gamma_inv() { return GF::get().inv(kGamma); }                   // 0x8E

// n x n inverse by Gauss-Jordan; false if singular.
inline bool gf_invert(const std::vector<uint8_t> &a, size_t n, std::vector<uint8_t> &inv) {
    const GF &g = GF::get();
    std::vector<uint8_t> m(a);
    inv.assign(n * n, 0);
    for (size_t i = 0; i < n; i++) inv[i * n + i] = 1;
    for (size_t c = 0; c < n; c++) {
        size_t piv = c;
        while (piv < n && m[piv * n + c] == 0) piv++;
        if (piv == n) return false;
        if (piv != c)
            for (size_t j = 0; j < n; j++) {
                std::swap(m[c * n + j], m[piv * n + j]);
                std::swap(inv[c * n + j], inv[piv * n + j]);
            }
        uint8_t s = g.inv(m[c * n + c]);
        for (size_t j = 0; j < n; j++) {
            m[c * n + j] = g.mul(m[c * n + j], s);
            inv[c * n + j] = g.mul(inv[c * n + j], s);
        }
        for (size_t r = 0; r < n; r++) {
            if (r == c || m[r * n + c] == 0) continue;
            uint8_t f = m[r * n + c];
            for (size_t j = 0; j < n; j++) {
                m[r * n + j] ^= g.mul(f, m[c * n + j]);
                inv[r * n + j] ^= g.mul(f, inv[c * n + j]);
            }
        }
    }
    return true;
}

// Systematic RS(data, parity) generator, (data+parity) x data, row-major.
// Error codes follow ReedSolomon::new: 1 TooFewDataShards, 2 TooFewParityShards, 3 TooManyShards.
inline int rs_generator(size_t data, size_t parity, std::vector<uint8_t> &out) {
    if (data == 0) return 1;
    if (parity == 0) return 2;
    if (data + parity > 256) return 3;
    const GF &g = GF::get();
    size_t total = data + parity;
    std::vector<uint8_t> v(total * data), top(data * data), ti;
    for (size_t r = 0; r < total; r++)
        for (size_t c = 0; c < data; c++) v[r * data + c] = g.pow(uint8_t(r), c);
    for (size_t i = 0; i < data * data; i++) top[i] = v[i];
    gf_invert(top, data, ti);
    out.assign(total * data, 0);
    for (size_t r = 0; r < total; r++)
        for (size_t c = 0; c < data; c++) {
            uint8_t acc = 0;
            for (size_t i = 0; i < data; i++) acc ^= g.mul(v[r * data + i], ti[i * data + c]);
            out[r * data + c] = acc;
        }
    return 0;
}

inline const char *rs_error_name(int e) {
    switch (e) {
    case 1: return "TooFewDataShards";
    case 2: return "TooFewParityShards";
    case 3: return "TooManyShards";
    case 4: return "TooFewShardsPresent";
    case 5: return "SingularMatrix";
    default: return "Unknown";
    }
}

// 32-byte v_perm_b32 lookup table for "multiply 4 packed bytes by c":
//   w[0],w[1]: c*i for i in 0..7   (low 3 bits)
//   w[2],w[3]: c*(i<<3) for i 0..7 (bits 3..5)
//   w[4]:      c*(i<<6) for i 0..3 (bits 6..7)
inline void perm_table(uint8_t c, uint32_t w[8]) {
    const GF &g = GF::get();
    uint8_t b[20];
    for (int i = 0; i < 8; i++) b[i] = g.mul(c, uint8_t(i));
    for (int i = 0; i < 8; i++) b[8 + i] = g.mul(c, uint8_t(i << 3));
    for (int i = 0; i < 4; i++) b[16 + i] = g.mul(c, uint8_t(i << 6));
    for (int k = 0; k < 5; k++)
        w[k] = uint32_t(b[4 * k]) | uint32_t(b[4 * k + 1]) << 8 | uint32_t(b[4 * k + 2]) << 16 |
               uint32_t(b[4 * k + 3]) << 24;
    w[5] = w[6] = w[7] = 0;
}

}  // namespace clay
