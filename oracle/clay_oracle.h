/*
 * clay_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the spool-labs/clay (clay-codes 0.1.2) reference algorithm,
 * used as the parity checker for the MI355X engine in clay_amd/ and as the timed
 * CPU baseline ("port") in bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library.  The product path
 * (libclay_amd.so) never links, loads or calls it.
 *
 * Error layout is byte-identical to clay_error_t in include/clay.h so tests can
 * compare error kinds / payloads / messages field by field.
 */
#ifndef CLAY_ORACLE_H
#define CLAY_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    size_t k, m, n, d, q, t, nu, sub_chunk_no, beta;
    size_t original_count, recovery_count;
} oc_code_t;

typedef struct {
    int kind;          /* 0 ok, 1..9 = ClayError variants (error.rs:5-24) */
    size_t a, b, c;    /* variant payload fields, in declaration order */
    char msg[256];     /* Display string (error.rs:26-54) */
} oc_error_t;

enum {
    OC_OK = 0,
    OC_INVALID_PARAMETERS = 1,
    OC_INSUFFICIENT_HELPERS = 2,
    OC_INVALID_CHUNK_SIZE = 3,
    OC_INSUFFICIENT_HELPER_DATA = 4,
    OC_INCONSISTENT_CHUNK_SIZES = 5,
    OC_TOO_MANY_ERASURES = 6,
    OC_RECONSTRUCTION_FAILED = 7,
    OC_MISSING_Y_SECTION_HELPER = 8,
    OC_OVERFLOW = 9,
};

/* ---- GF(2^8) / reed-solomon-erasure 6.0.0 known-answer access ---- */
uint8_t oc_gf_add(uint8_t a, uint8_t b);
uint8_t oc_gf_mul(uint8_t a, uint8_t b);
uint8_t oc_gf_div(uint8_t a, uint8_t b);  /* b != 0 */
uint8_t oc_gf_exp(uint8_t a, size_t n);
/* full systematic matrix (total x data), row-major, into out[total*data] */
int oc_rs_matrix(size_t data, size_t parity, uint8_t *out);
/* rs.encode on `data+parity` shards of `len` bytes (shards[data..] overwritten) */
int oc_rs_encode(size_t data, size_t parity, uint8_t *const *shards, size_t len);
/* rs.reconstruct: present[i]==0 marks a missing shard (buffer still provided) */
int oc_rs_reconstruct(size_t data, size_t parity, uint8_t *const *shards,
                      const uint8_t *present, size_t len);

/* ---- clay-codes helpers with in-tree KATs ---- */
void oc_get_plane_vector(size_t z, size_t t, size_t q, size_t *out);
size_t oc_get_companion_layer(const oc_code_t *p, size_t z, size_t x, size_t y, size_t z_y);
size_t oc_get_max_iscore(const oc_code_t *p, const size_t *erased, size_t n_erased);
int oc_checked_pow(size_t base, size_t exp, size_t *out); /* 1 ok, 0 overflow */
int oc_repair_subchunk_indices(const oc_code_t *p, size_t lost_internal, size_t *out,
                               size_t *n_out, oc_error_t *err);
void oc_prt(const uint8_t *c, const uint8_t *cs, uint8_t *u, uint8_t *us, size_t len);
void oc_pft(const uint8_t *u, const uint8_t *us, uint8_t *c, uint8_t *cs, size_t len);
/* transforms.rs:132-142 / 149-161 (partial transforms) */
void oc_c_from_u_and_cstar(const uint8_t *u, const uint8_t *cs, uint8_t *c, size_t len);
void oc_u_from_c_and_ustar(const uint8_t *c, const uint8_t *us, uint8_t *u, size_t len);

/* ---- ClayCode API (lib.rs:94-241) ---- */
int oc_new(size_t k, size_t m, size_t d, oc_code_t *out, oc_error_t *err);
int oc_new_default(size_t k, size_t m, oc_code_t *out, oc_error_t *err);
double oc_normalized_repair_bandwidth(const oc_code_t *p);
size_t oc_encoded_chunk_size(const oc_code_t *p, size_t data_len);
/* out: n chunks of chunk_size bytes, k data then m parity, contiguous */
int oc_encode(const oc_code_t *p, const uint8_t *data, size_t len, uint8_t *out,
              oc_error_t *err);
int oc_decode(const oc_code_t *p, const size_t *ids, const uint8_t *const *bufs,
              const size_t *lens, size_t n_avail, const size_t *erasures, size_t n_erasures,
              uint8_t *out, size_t out_cap, size_t *out_len, oc_error_t *err);
int oc_minimum_to_repair(const oc_code_t *p, size_t lost, const size_t *avail, size_t n_avail,
                         size_t *helpers_out, size_t *n_helpers, size_t *idx_out,
                         size_t *n_idx, oc_error_t *err);
int oc_repair(const oc_code_t *p, size_t lost, const size_t *ids, const uint8_t *const *bufs,
              const size_t *lens, size_t n_helpers, size_t chunk_size, uint8_t *out,
              oc_error_t *err);

/* 1 = AVX2 nibble-shuffle region multiply (as the dependency's simd_c), 0 = scalar table */
void oc_set_simd(int enable);
int oc_simd_available(void);

#ifdef __cplusplus
}
#endif
#endif
