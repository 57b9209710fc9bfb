// code.hpp -- ClayCode parameters, error plumbing, host-side validation.
// Mirrors lib.rs:94-259 (new / checked_pow), decode.rs:36-126 (decode input
// validation, in the reference's precedence), repair.rs:22-126 (index lists,
// minimum_to_repair) and repair.rs:146-245 (repair validation).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/clay.h"

namespace clay {

struct Error {
    int kind = CLAY_OK;
    size_t a = 0, b = 0, c = 0;
    std::string msg;
    explicit operator bool() const { return kind != CLAY_OK; }
};

Error make_error(int kind, size_t a, size_t b, size_t c, const char *fmt, ...)
    __attribute__((format(printf, 5, 6)));
int report(const Error &e, clay_error_t *out);

bool checked_pow(size_t base, size_t exp, size_t *out);   // lib.rs:245-259
Error code_new(size_t k, size_t m, size_t d, clay_code_t *out);  // lib.rs:94-147
size_t encoded_chunk_size(const clay_code_t &c, size_t len);      // encode.rs:33-42

inline size_t internal_of(const clay_code_t &c, size_t ext) { return ext < c.k ? ext : ext + c.nu; }
inline bool is_shortened(const clay_code_t &c, size_t internal) {
    return internal >= c.k && internal < c.k + c.nu;
}
// z -> base-q digits, MSB first (coords.rs:30-40)
void plane_vector(const clay_code_t &c, size_t z, size_t *out);
// decode.rs:413-435
size_t companion_layer(const clay_code_t &c, size_t z, size_t x, size_t y, size_t z_y);

// decode.rs:36-126 validation.  On success fills erased (internal ids, sorted set)
// and the chunk size.
struct AvailView {
    const size_t *ids;
    const size_t *lens;
    size_t n;
};
Error validate_decode(const clay_code_t &c, const AvailView &av, const size_t *erasures,
                      size_t n_erasures, size_t *chunk_size, std::vector<uint8_t> &erased_int);

// repair.rs:22-49
Error repair_subchunk_indices(const clay_code_t &c, size_t lost_internal, std::vector<size_t> &out);
// repair.rs:61-126
Error minimum_to_repair(const clay_code_t &c, size_t lost, const size_t *avail, size_t n_avail,
                        std::vector<size_t> &helpers, std::vector<size_t> &subchunks);
// repair.rs:146-245 validation; fills helper presence (internal ids) and the index list.
Error validate_repair(const clay_code_t &c, size_t lost, const size_t *ids, const size_t *lens,
                      size_t n_helpers, size_t chunk_size, std::vector<uint8_t> &helper_int,
                      std::vector<long> &helper_slot_of_id, std::vector<size_t> &subchunks);

}  // namespace clay
