/*
 * clay_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A plain-C restatement of the reference CPU path of spool-labs/clay
 * (crate clay-codes 0.1.2, /root/reference), following its control flow
 * statement by statement so that outputs are byte-identical for ANY input,
 * including non-codeword inputs to decode/repair.  Every function cites the
 * reference file:line it restates.
 *
 * The GF(2^8) / Reed-Solomon layer lives in the third-party crate
 * `reed-solomon-erasure` 6.0.0 (Cargo.lock:496-508, checksum 7263373d...),
 * which is NOT vendored in /root/reference.  Its published algorithm is
 * restated here (section "reed-solomon-erasure 6.0.0"):
 *   - galois_8: field poly x^8+x^4+x^3+x^2+1 (0x11D), generator 2;
 *     add = xor, mul = table, div/exp via log tables;
 *   - ReedSolomon::new(data, parity): errors if data==0 / parity==0 /
 *     data+parity > 256; matrix = vandermonde(total, data) * inv(top square);
 *   - encode: parity_i = sum_j M[data+i][j] * shard_j;
 *   - reconstruct: first `data` present shards (index order) -> invert that
 *     sub-matrix -> rebuild missing data; then missing parity from all data.
 *   - region multiply: `simd-accel` feature (Cargo.toml:15-16) = C SIMD nibble
 *     shuffle (simd_c/reedsolomon.c); restated below as AVX2 PSHUFB, selectable
 *     at run time, results identical to the scalar table path.
 *
 * PARITY PINNING (see DESIGN.md "Oracle"): the reference cannot be built here
 * (no cargo/rustc; dependency not vendored).  The reference holds no golden
 * byte vectors.  This restatement is pinned by (1) the reference's in-tree KATs
 * (transforms.rs:216-225, coords.rs:46-60, decode.rs:628-651, lib.rs:321-335,
 * repair.rs:442-461), (2) its property tests re-run against this oracle
 * (roundtrips, repair == chunk for every node, error variants/messages), and
 * (3) the dependency's published KATs (galois_8 mul/exp, RS(5,5) encode).
 * Parity bytes themselves are pinned only through (3).
 */
#include "clay_oracle.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

/* ======================================================================
 * reed-solomon-erasure 6.0.0 :: galois_8 (restated; not vendored)
 * ====================================================================== */
static uint8_t EXP_TABLE[512];
static uint8_t LOG_TABLE[256];
static uint8_t MUL_TABLE[256][256];
static int g_tables_ready = 0;
static int g_use_simd = 1;

static void gf_init(void) {
    if (g_tables_ready) return;
    /* generating polynomial 29 (0x11D without the x^8 term), generator 2 */
    unsigned b = 1;
    for (int i = 0; i < 255; i++) {
        EXP_TABLE[i] = (uint8_t)b;
        LOG_TABLE[b] = (uint8_t)i;
        b <<= 1;
        if (b & 0x100) b ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) EXP_TABLE[i] = EXP_TABLE[i - 255];
    LOG_TABLE[0] = 0;
    for (int a = 0; a < 256; a++)
        for (int c = 0; c < 256; c++)
            MUL_TABLE[a][c] = (a == 0 || c == 0) ? 0
                                                 : EXP_TABLE[LOG_TABLE[a] + LOG_TABLE[c]];
    g_tables_ready = 1;
}

uint8_t oc_gf_add(uint8_t a, uint8_t b) { return a ^ b; }
uint8_t oc_gf_mul(uint8_t a, uint8_t b) { gf_init(); return MUL_TABLE[a][b]; }
uint8_t oc_gf_div(uint8_t a, uint8_t b) {
    gf_init();
    if (a == 0) return 0;
    if (b == 0) { fprintf(stderr, "oracle: Divisor is 0\n"); abort(); }
    int lr = (int)LOG_TABLE[a] - (int)LOG_TABLE[b];
    if (lr < 0) lr += 255;
    return EXP_TABLE[lr];
}
uint8_t oc_gf_exp(uint8_t a, size_t n) {
    gf_init();
    if (n == 0) return 1;
    if (a == 0) return 0;
    size_t lr = (size_t)LOG_TABLE[a] * n;
    while (lr >= 255) lr -= 255;
    return EXP_TABLE[lr];
}

/* galois_8::mul_slice / mul_slice_add.  Scalar table, or AVX2 nibble shuffle
 * (the `simd-accel` C path): out = c*in (xor into out for _add). */
#if defined(__x86_64__)
__attribute__((target("avx2")))
static size_t simd_mul(uint8_t c, const uint8_t *in, uint8_t *out, size_t len, int add) {
    uint8_t lo[16], hi[16];
    for (int i = 0; i < 16; i++) { lo[i] = MUL_TABLE[c][i]; hi[i] = MUL_TABLE[c][i << 4]; }
    __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)lo));
    __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)hi));
    __m256i mask = _mm256_set1_epi8(0x0f);
    size_t done = 0;
    for (; done + 32 <= len; done += 32) {
        __m256i x = _mm256_loadu_si256((const __m256i *)(in + done));
        __m256i l = _mm256_and_si256(x, mask);
        __m256i h = _mm256_and_si256(_mm256_srli_epi64(x, 4), mask);
        __m256i r = _mm256_xor_si256(_mm256_shuffle_epi8(tlo, l), _mm256_shuffle_epi8(thi, h));
        if (add) r = _mm256_xor_si256(r, _mm256_loadu_si256((const __m256i *)(out + done)));
        _mm256_storeu_si256((__m256i *)(out + done), r);
    }
    return done;
}
#endif

static int g_simd_ok = -1;
int oc_simd_available(void) {
#if defined(__x86_64__)
    if (g_simd_ok < 0) { __builtin_cpu_init(); g_simd_ok = __builtin_cpu_supports("avx2") ? 1 : 0; }
    return g_simd_ok;
#else
    return 0;
#endif
}
void oc_set_simd(int enable) { g_use_simd = enable; }

static void mul_slice_impl(uint8_t c, const uint8_t *in, uint8_t *out, size_t len, int add) {
    size_t done = 0;
#if defined(__x86_64__)
    if (g_use_simd && oc_simd_available()) done = simd_mul(c, in, out, len, add);
#endif
    const uint8_t *t = MUL_TABLE[c];
    if (add) for (size_t i = done; i < len; i++) out[i] ^= t[in[i]];
    else     for (size_t i = done; i < len; i++) out[i] = t[in[i]];
}
static void mul_slice(uint8_t c, const uint8_t *in, uint8_t *out, size_t len) { mul_slice_impl(c, in, out, len, 0); }
static void mul_slice_add(uint8_t c, const uint8_t *in, uint8_t *out, size_t len) { mul_slice_impl(c, in, out, len, 1); }

/* ---------------- reed-solomon-erasure :: matrix ---------------- */
/* Gaussian elimination inverse (matrix.rs invert / gaussian_elim).  Returns 0 if singular. */
static int mat_invert(const uint8_t *a, size_t n, uint8_t *inv) {
    size_t w = 2 * n;
    uint8_t *m = (uint8_t *)calloc(n * w, 1);
    for (size_t r = 0; r < n; r++) {
        memcpy(m + r * w, a + r * n, n);
        m[r * w + n + r] = 1;
    }
    for (size_t r = 0; r < n; r++) {
        if (m[r * w + r] == 0) {
            size_t rb;
            for (rb = r + 1; rb < n; rb++)
                if (m[rb * w + r] != 0) break;
            if (rb == n) { free(m); return 0; }
            for (size_t c = 0; c < w; c++) { uint8_t t = m[r * w + c]; m[r * w + c] = m[rb * w + c]; m[rb * w + c] = t; }
        }
        if (m[r * w + r] != 1) {
            uint8_t s = oc_gf_div(1, m[r * w + r]);
            for (size_t c = 0; c < w; c++) m[r * w + c] = MUL_TABLE[m[r * w + c]][s];
        }
        for (size_t rb = r + 1; rb < n; rb++) {
            uint8_t s = m[rb * w + r];
            if (s) for (size_t c = 0; c < w; c++) m[rb * w + c] ^= MUL_TABLE[s][m[r * w + c]];
        }
    }
    for (size_t d = 0; d < n; d++)
        for (size_t ra = 0; ra < d; ra++) {
            uint8_t s = m[ra * w + d];
            if (s) for (size_t c = 0; c < w; c++) m[ra * w + c] ^= MUL_TABLE[s][m[d * w + c]];
        }
    for (size_t r = 0; r < n; r++) memcpy(inv + r * n, m + r * w + n, n);
    free(m);
    return 1;
}

typedef struct {
    size_t data, parity, total;
    uint8_t *matrix; /* total x data */
} rs_t;

static const char *RS_ERR_NAMES[] = {"", "TooFewDataShards", "TooFewParityShards", "TooManyShards",
                                     "TooFewShardsPresent", "SingularMatrix"};
enum { RSE_OK = 0, RSE_TOO_FEW_DATA = 1, RSE_TOO_FEW_PARITY = 2, RSE_TOO_MANY = 3,
       RSE_TOO_FEW_PRESENT = 4, RSE_SINGULAR = 5 };

/* ReedSolomon::new (reed-solomon-erasure core.rs; build_matrix) */
static int rs_new(rs_t *rs, size_t data, size_t parity) {
    gf_init();
    memset(rs, 0, sizeof(*rs));
    if (data == 0) return RSE_TOO_FEW_DATA;
    if (parity == 0) return RSE_TOO_FEW_PARITY;
    if (data + parity > 256) return RSE_TOO_MANY;
    size_t total = data + parity;
    uint8_t *v = (uint8_t *)malloc(total * data);
    for (size_t r = 0; r < total; r++)
        for (size_t c = 0; c < data; c++) v[r * data + c] = oc_gf_exp((uint8_t)r, c);
    uint8_t *top_inv = (uint8_t *)malloc(data * data);
    mat_invert(v, data, top_inv); /* vandermonde top is invertible */
    rs->matrix = (uint8_t *)calloc(total * data, 1);
    for (size_t r = 0; r < total; r++)
        for (size_t c = 0; c < data; c++) {
            uint8_t acc = 0;
            for (size_t i = 0; i < data; i++) acc ^= MUL_TABLE[v[r * data + i]][top_inv[i * data + c]];
            rs->matrix[r * data + c] = acc;
        }
    free(v);
    free(top_inv);
    rs->data = data; rs->parity = parity; rs->total = total;
    return RSE_OK;
}
static void rs_free(rs_t *rs) { free(rs->matrix); rs->matrix = NULL; }

/* code_some_slices: input-major loop, mul_slice for input 0 then mul_slice_add */
static void code_some_slices(const rs_t *rs, const uint8_t *const *rows, size_t nrows,
                             const uint8_t *const *inputs, uint8_t *const *outputs, size_t len) {
    for (size_t i = 0; i < rs->data; i++)
        for (size_t r = 0; r < nrows; r++) {
            if (i == 0) mul_slice(rows[r][i], inputs[i], outputs[r], len);
            else        mul_slice_add(rows[r][i], inputs[i], outputs[r], len);
        }
}

/* ReedSolomon::encode: parity from all data shards */
static void rs_encode(const rs_t *rs, uint8_t *const *shards, size_t len) {
    const uint8_t *rows[256];
    for (size_t p = 0; p < rs->parity; p++) rows[p] = rs->matrix + (rs->data + p) * rs->data;
    code_some_slices(rs, rows, rs->parity, (const uint8_t *const *)shards, shards + rs->data, len);
}

/* ReedSolomon::reconstruct (reconstruct_internal, data_only = false) */
static int rs_reconstruct(const rs_t *rs, uint8_t *const *shards, const uint8_t *present, size_t len) {
    size_t npresent = 0;
    for (size_t i = 0; i < rs->total; i++) npresent += present[i] ? 1 : 0;
    if (npresent == rs->total) return RSE_OK;
    if (npresent < rs->data) return RSE_TOO_FEW_PRESENT;
    size_t valid[256], nvalid = 0, invalid[256], ninvalid = 0;
    const uint8_t *sub[256];
    uint8_t *missing_data[256];
    for (size_t i = 0; i < rs->total; i++) {
        if (!present[i]) {
            if (i < rs->data) { missing_data[ninvalid] = shards[i]; invalid[ninvalid++] = i; }
        } else if (nvalid < rs->data) {
            sub[nvalid] = shards[i];
            valid[nvalid++] = i;
        }
    }
    size_t d = rs->data;
    uint8_t *subm = (uint8_t *)malloc(d * d), *dec = (uint8_t *)malloc(d * d);
    for (size_t r = 0; r < d; r++) memcpy(subm + r * d, rs->matrix + valid[r] * d, d);
    if (!mat_invert(subm, d, dec)) { free(subm); free(dec); return RSE_SINGULAR; }
    const uint8_t *rows[256];
    for (size_t r = 0; r < ninvalid; r++) rows[r] = dec + invalid[r] * d;
    if (ninvalid) code_some_slices(rs, rows, ninvalid, sub, missing_data, len);
    /* missing parity from the (now complete) data shards */
    uint8_t *missing_parity[256];
    size_t np = 0;
    for (size_t i = rs->data; i < rs->total; i++)
        if (!present[i]) { rows[np] = rs->matrix + i * d; missing_parity[np++] = shards[i]; }
    if (np) code_some_slices(rs, rows, np, (const uint8_t *const *)shards, missing_parity, len);
    free(subm);
    free(dec);
    return RSE_OK;
}

int oc_rs_matrix(size_t data, size_t parity, uint8_t *out) {
    rs_t rs;
    int e = rs_new(&rs, data, parity);
    if (e) return e;
    memcpy(out, rs.matrix, rs.total * rs.data);
    rs_free(&rs);
    return 0;
}
int oc_rs_encode(size_t data, size_t parity, uint8_t *const *shards, size_t len) {
    rs_t rs;
    int e = rs_new(&rs, data, parity);
    if (e) return e;
    rs_encode(&rs, shards, len);
    rs_free(&rs);
    return 0;
}
int oc_rs_reconstruct(size_t data, size_t parity, uint8_t *const *shards, const uint8_t *present, size_t len) {
    rs_t rs;
    int e = rs_new(&rs, data, parity);
    if (e) return e;
    e = rs_reconstruct(&rs, shards, present, len);
    rs_free(&rs);
    return e;
}

/* ======================================================================
 * clay-codes 0.1.2
 * ====================================================================== */
static int set_err(oc_error_t *err, int kind, size_t a, size_t b, size_t c, const char *fmt, ...) {
    if (err) {
        err->kind = kind; err->a = a; err->b = b; err->c = c;
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(err->msg, sizeof(err->msg), fmt, ap);
        va_end(ap);
    }
    return kind;
}
static void clear_err(oc_error_t *err) { if (err) memset(err, 0, sizeof(*err)); }

/* lib.rs:245-259 checked_pow */
int oc_checked_pow(size_t base, size_t exp, size_t *out) {
    size_t result = 1, b = base, e = exp;
    while (e > 0) {
        if (e & 1) { if (__builtin_mul_overflow(result, b, &result)) return 0; }
        e >>= 1;
        if (e > 0) { if (__builtin_mul_overflow(b, b, &b)) return 0; }
    }
    *out = result;
    return 1;
}

/* lib.rs:94-147 ClayCode::new */
int oc_new(size_t k, size_t m, size_t d, oc_code_t *out, oc_error_t *err) {
    clear_err(err);
    if (k < 1) return set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: k must be at least 1");
    if (m < 1) return set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: m must be at least 1");
    if (d < k + 1 || d > k + m - 1)
        return set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: d must be in range [%zu, %zu], got %zu",
                       k + 1, k + m - 1, d);
    size_t q = d - k + 1, n = k + m;
    size_t nu = (n % q == 0) ? 0 : q - (n % q);
    size_t t = (n + nu) / q;
    size_t alpha;
    if (!oc_checked_pow(q, t, &alpha))
        return set_err(err, OC_OVERFLOW, 0, 0, 0, "Arithmetic overflow: q^t = %zu^%zu overflows", q, t);
    size_t beta = alpha / q;
    size_t oc = k + nu, rc = m;
    if (oc > 32768 || rc > 32768)
        return set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: Total nodes exceeds reed-solomon limit of 32768");
    out->k = k; out->m = m; out->n = n; out->d = d; out->q = q; out->t = t; out->nu = nu;
    out->sub_chunk_no = alpha; out->beta = beta; out->original_count = oc; out->recovery_count = rc;
    return 0;
}
/* lib.rs:150-152 */
int oc_new_default(size_t k, size_t m, oc_code_t *out, oc_error_t *err) { return oc_new(k, m, k + m - 1, out, err); }
/* lib.rs:239-241 */
double oc_normalized_repair_bandwidth(const oc_code_t *p) {
    return (double)p->d / ((double)p->k * (double)(p->d - p->k + 1));
}

/* coords.rs:30-40 (MSB first) */
void oc_get_plane_vector(size_t z, size_t t, size_t q, size_t *out) {
    size_t rem = z;
    for (size_t i = 0; i < t; i++) { out[t - 1 - i] = rem % q; rem /= q; }
}

/* decode.rs:413-435 get_companion_layer */
size_t oc_get_companion_layer(const oc_code_t *p, size_t z, size_t x, size_t y, size_t z_y) {
    long long alpha = (long long)p->sub_chunk_no;
    long long mult = 1;
    for (size_t i = 0; i < p->t - 1 - y; i++) mult *= (long long)p->q;
    long long diff = (long long)x - (long long)z_y;
    long long v = ((long long)z + diff * mult) % alpha;
    if (v < 0) v += alpha;
    return (size_t)v;
}

/* decode.rs:548-561 get_max_iscore */
static size_t max_iscore_set(const oc_code_t *p, const uint8_t *erased) {
    uint8_t wv[4096] = {0};
    size_t is = 0, tn = p->q * p->t;
    for (size_t i = 0; i < tn; i++)
        if (erased[i]) { size_t y = i / p->q; if (!wv[y]) { wv[y] = 1; is++; } }
    return is;
}
size_t oc_get_max_iscore(const oc_code_t *p, const size_t *er, size_t n) {
    size_t tn = p->q * p->t;
    uint8_t *s = (uint8_t *)calloc(tn, 1);
    for (size_t i = 0; i < n; i++) if (er[i] < tn) s[er[i]] = 1;
    size_t r = max_iscore_set(p, s);
    free(s);
    return r;
}

/* ---------------- transforms.rs (gamma = 2) ---------------- */
#define GAMMA 2
/* transforms.rs:42-55 prt_compute_both */
void oc_prt(const uint8_t *c, const uint8_t *cs, uint8_t *u, uint8_t *us, size_t len) {
    gf_init();
    for (size_t i = 0; i < len; i++) {
        u[i] = c[i] ^ MUL_TABLE[GAMMA][cs[i]];
        us[i] = MUL_TABLE[GAMMA][c[i]] ^ cs[i];
    }
}
/* transforms.rs:65-89 prt_compute_both_oriented */
static void prt_oriented(const uint8_t *cxy, const uint8_t *csw, int xy_primary, uint8_t *uxy, uint8_t *usw, size_t len) {
    if (xy_primary) {
        for (size_t i = 0; i < len; i++) {
            uxy[i] = cxy[i] ^ MUL_TABLE[GAMMA][csw[i]];
            usw[i] = MUL_TABLE[GAMMA][cxy[i]] ^ csw[i];
        }
    } else {
        for (size_t i = 0; i < len; i++) {
            uxy[i] = MUL_TABLE[GAMMA][csw[i]] ^ cxy[i];
            usw[i] = csw[i] ^ MUL_TABLE[GAMMA][cxy[i]];
        }
    }
}
/* transforms.rs:108-125 pft_compute_both */
void oc_pft(const uint8_t *u, const uint8_t *us, uint8_t *c, uint8_t *cs, size_t len) {
    gf_init();
    uint8_t det = 1 ^ MUL_TABLE[GAMMA][GAMMA];
    uint8_t det_inv = oc_gf_div(1, det);
    for (size_t i = 0; i < len; i++) {
        c[i] = MUL_TABLE[u[i] ^ MUL_TABLE[GAMMA][us[i]]][det_inv];
        cs[i] = MUL_TABLE[MUL_TABLE[GAMMA][u[i]] ^ us[i]][det_inv];
    }
}
/* transforms.rs:132-142 compute_c_from_u_and_cstar */
static void c_from_u_and_cstar(const uint8_t *uxy, const uint8_t *cc, uint8_t *c, size_t len) {
    for (size_t i = 0; i < len; i++) c[i] = uxy[i] ^ MUL_TABLE[GAMMA][cc[i]];
}
/* transforms.rs:149-161 compute_u_from_c_and_ustar */
static void u_from_c_and_ustar(const uint8_t *cxy, const uint8_t *uc, uint8_t *u, size_t len) {
    uint8_t det = 1 ^ MUL_TABLE[GAMMA][GAMMA];
    for (size_t i = 0; i < len; i++) u[i] = MUL_TABLE[det][cxy[i]] ^ MUL_TABLE[GAMMA][uc[i]];
}
/* exported for the reference's test_partial_transform_roundtrips (transforms.rs:192-213) */
void oc_c_from_u_and_cstar(const uint8_t *u, const uint8_t *cs, uint8_t *c, size_t len) { c_from_u_and_cstar(u, cs, c, len); }
void oc_u_from_c_and_ustar(const uint8_t *c, const uint8_t *us, uint8_t *u, size_t len) { u_from_c_and_ustar(c, us, u, len); }
/* decode.rs:566-576 compute_cstar_from_c_and_u */
static void cstar_from_c_and_u(const uint8_t *ch, const uint8_t *uh, uint8_t *out, size_t len) {
    uint8_t gi = oc_gf_div(1, GAMMA);
    for (size_t i = 0; i < len; i++) out[i] = MUL_TABLE[uh[i] ^ ch[i]][gi];
}

/* ---------------- decode.rs ---------------- */
typedef struct {
    const oc_code_t *p;
    size_t tn, alpha, sc, chunk;
    uint8_t **chunks;   /* tn chunk buffers (C plane) */
    uint8_t *u_buf;     /* tn x chunk (U plane) */
    uint8_t *u_comp;    /* tn x alpha */
    rs_t rs;
} layered_t;

#define UB(L, node, z) ((L)->u_buf + (node) * (L)->chunk + (z) * (L)->sc)
#define CB(L, node, z) ((L)->chunks[node] + (z) * (L)->sc)

/* decode.rs:332-408 decode_uncoupled_layer */
static int decode_uncoupled_layer(const oc_code_t *p, const uint8_t *erased, size_t z, size_t sc,
                                  uint8_t *u_buf, size_t chunk, const rs_t *rs, oc_error_t *err) {
    size_t tn = p->q * p->t, off = z * sc, ps = p->original_count, ne = 0;
    int has_orig = 0, has_par = 0;
    for (size_t i = 0; i < tn; i++)
        if (erased[i]) { ne++; if (i < ps) has_orig = 1; else has_par = 1; }
    if (ne > p->m)
        return set_err(err, OC_TOO_MANY_ERASURES, p->m, ne, 0, "Too many erasures: max %zu supported, got %zu", p->m, ne);
    if (ne == 0) return 0;
    uint8_t *tmp = (uint8_t *)malloc(tn * sc); /* the per-layer shard copies (to_vec) */
    uint8_t *sh[256];
    for (size_t i = 0; i < tn; i++) sh[i] = tmp + i * sc;
    if (has_orig) {
        uint8_t present[256];
        for (size_t i = 0; i < tn; i++) {
            present[i] = !erased[i];
            if (present[i]) memcpy(sh[i], u_buf + i * chunk + off, sc);
            else memset(sh[i], 0, sc);
        }
        int e = rs_reconstruct(rs, sh, present, sc);
        if (e) { free(tmp); return set_err(err, OC_RECONSTRUCTION_FAILED, 0, 0, 0,
                                           "RS reconstruction failed: Layer %zu RS reconstruct failed: %s", z, RS_ERR_NAMES[e]); }
        for (size_t i = 0; i < tn; i++)
            if (erased[i]) memcpy(u_buf + i * chunk + off, sh[i], sc);
    } else if (has_par) {
        for (size_t i = 0; i < tn; i++) memcpy(sh[i], u_buf + i * chunk + off, sc);
        rs_encode(rs, sh, sc);
        for (size_t i = ps; i < tn; i++)
            if (erased[i]) memcpy(u_buf + i * chunk + off, sh[i], sc);
    }
    free(tmp);
    return 0;
}

/* decode.rs:438-468 get_uncoupled_from_coupled */
static void get_uncoupled_from_coupled(layered_t *L, size_t x, size_t y, size_t z, size_t z_y, size_t z_sw) {
    size_t q = L->p->q, sc = L->sc;
    size_t nxy = y * q + x, nsw = y * q + z_y;
    uint8_t *uxy = (uint8_t *)malloc(sc), *usw = (uint8_t *)malloc(sc);
    if (x < z_y) oc_prt(CB(L, nxy, z), CB(L, nsw, z_sw), uxy, usw, sc);
    else         oc_prt(CB(L, nsw, z_sw), CB(L, nxy, z), usw, uxy, sc);
    memcpy(UB(L, nxy, z), uxy, sc);
    memcpy(UB(L, nsw, z_sw), usw, sc);
    free(uxy); free(usw);
}

/* decode.rs:260-329 decode_layered_with_tracking */
static int decode_layered_with_tracking(layered_t *L, const uint8_t *erased, size_t z, oc_error_t *err) {
    const oc_code_t *p = L->p;
    size_t q = p->q, t = p->t, tn = L->tn, sc = L->sc, alpha = L->alpha;
    size_t zv[64];
    oc_get_plane_vector(z, t, q, zv);
    uint8_t needs[256];
    memcpy(needs, erased, tn);
    for (size_t x = 0; x < q; x++) {
        for (size_t y = 0; y < t; y++) {
            size_t nxy = q * y + x, z_y = zv[y], nsw = q * y + z_y;
            size_t z_sw = oc_get_companion_layer(p, z, x, y, z_y);
            if (erased[nxy]) continue;
            if (z_y == x) {
                memcpy(UB(L, nxy, z), CB(L, nxy, z), sc);
                L->u_comp[nxy * alpha + z] = 1;
            } else if (!erased[nsw]) {
                if (z_y < x) {
                    get_uncoupled_from_coupled(L, x, y, z, z_y, z_sw);
                    L->u_comp[nxy * alpha + z] = 1;
                    L->u_comp[nsw * alpha + z_sw] = 1;
                }
            } else {
                if (L->u_comp[nsw * alpha + z_sw]) {
                    uint8_t *u = (uint8_t *)malloc(sc);
                    u_from_c_and_ustar(CB(L, nxy, z), UB(L, nsw, z_sw), u, sc);
                    memcpy(UB(L, nxy, z), u, sc);
                    free(u);
                    L->u_comp[nxy * alpha + z] = 1;
                } else {
                    needs[nxy] = 1;
                }
            }
        }
    }
    int e = decode_uncoupled_layer(p, needs, z, sc, L->u_buf, L->chunk, &L->rs, err);
    if (e) return e;
    for (size_t i = 0; i < tn; i++) if (needs[i]) L->u_comp[i * alpha + z] = 1;
    return 0;
}

/* decode.rs:471-495 recover_type1_erasure */
static void recover_type1_erasure(layered_t *L, size_t x, size_t y, size_t z, size_t z_y, size_t z_sw) {
    size_t q = L->p->q, sc = L->sc, nxy = y * q + x, nsw = y * q + z_y;
    uint8_t *c = (uint8_t *)malloc(sc);
    c_from_u_and_cstar(UB(L, nxy, z), CB(L, nsw, z_sw), c, sc);
    memcpy(CB(L, nxy, z), c, sc);
    free(c);
}

/* decode.rs:498-528 get_coupled_from_uncoupled */
static void get_coupled_from_uncoupled(layered_t *L, size_t x, size_t y, size_t z, size_t z_y, size_t z_sw) {
    size_t q = L->p->q, sc = L->sc, nxy = y * q + x, nsw = y * q + z_y;
    uint8_t *cxy = (uint8_t *)malloc(sc), *csw = (uint8_t *)malloc(sc);
    if (x < z_y) oc_pft(UB(L, nxy, z), UB(L, nsw, z_sw), cxy, csw, sc);
    else         oc_pft(UB(L, nsw, z_sw), UB(L, nxy, z), csw, cxy, sc);
    memcpy(CB(L, nxy, z), cxy, sc);
    memcpy(CB(L, nsw, z_sw), csw, sc);
    free(cxy); free(csw);
}

/* decode.rs:167-257 decode_layered */
static int decode_layered(const oc_code_t *p, const uint8_t *erased, uint8_t **chunks, size_t chunk,
                          size_t sc, oc_error_t *err) {
    layered_t L;
    memset(&L, 0, sizeof(L));
    L.p = p; L.tn = p->q * p->t; L.alpha = p->sub_chunk_no; L.sc = sc; L.chunk = chunk; L.chunks = chunks;
    int e = rs_new(&L.rs, p->original_count, p->recovery_count);
    if (e) return set_err(err, OC_RECONSTRUCTION_FAILED, 0, 0, 0, "RS reconstruction failed: RS init failed: %s", RS_ERR_NAMES[e]);
    L.u_buf = (uint8_t *)calloc(L.tn * chunk, 1);
    L.u_comp = (uint8_t *)calloc(L.tn * L.alpha, 1);
    size_t *order = (size_t *)calloc(L.alpha, sizeof(size_t));
    size_t zv[64], q = p->q, t = p->t;
    /* decode.rs:531-545 set_planes_sequential_decoding_order */
    for (size_t z = 0; z < L.alpha; z++) {
        oc_get_plane_vector(z, t, q, zv);
        for (size_t i = 0; i < L.tn; i++)
            if (erased[i] && i % q == zv[i / q]) order[z]++;
    }
    size_t max_is = max_iscore_set(p, erased);
    int rc = 0;
    for (size_t is = 0; is <= max_is && !rc; is++) {
        for (size_t z = 0; z < L.alpha && !rc; z++)
            if (order[z] == is) rc = decode_layered_with_tracking(&L, erased, z, err);
        for (size_t z = 0; z < L.alpha && !rc; z++) {
            if (order[z] != is) continue;
            oc_get_plane_vector(z, t, q, zv);
            for (size_t nxy = 0; nxy < L.tn; nxy++) {
                if (!erased[nxy]) continue;
                size_t x = nxy % q, y = nxy / q, z_y = zv[y], nsw = y * q + z_y;
                size_t z_sw = oc_get_companion_layer(p, z, x, y, z_y);
                if (z_y != x) {
                    if (!erased[nsw]) recover_type1_erasure(&L, x, y, z, z_y, z_sw);
                    else if (z_y < x) get_coupled_from_uncoupled(&L, x, y, z, z_y, z_sw);
                } else {
                    memcpy(CB(&L, nxy, z), UB(&L, nxy, z), sc);
                }
            }
        }
    }
    free(order);
    free(L.u_buf);
    free(L.u_comp);
    rs_free(&L.rs);
    return rc;
}

/* encode.rs:33-42 */
size_t oc_encoded_chunk_size(const oc_code_t *p, size_t len) {
    size_t min_size = p->k * p->sub_chunk_no * 2;
    size_t padded = len == 0 ? min_size : ((len + min_size - 1) / min_size) * min_size;
    if (padded < min_size) padded = min_size;
    return padded / p->k;
}

/* encode.rs:30-80 encode */
int oc_encode(const oc_code_t *p, const uint8_t *data, size_t len, uint8_t *out, oc_error_t *err) {
    clear_err(err);
    gf_init();
    size_t chunk = oc_encoded_chunk_size(p, len);
    size_t padded = chunk * p->k;
    size_t sc = chunk / p->sub_chunk_no;
    size_t tn = p->q * p->t;
    uint8_t **chunks = (uint8_t **)malloc(tn * sizeof(uint8_t *));
    for (size_t i = 0; i < tn; i++) chunks[i] = (uint8_t *)calloc(chunk, 1);
    for (size_t i = 0; i < p->k; i++) {
        size_t lo = i * chunk;
        if (lo < len) memcpy(chunks[i], data + lo, (len - lo) < chunk ? (len - lo) : chunk);
    }
    (void)padded;
    uint8_t *er = (uint8_t *)calloc(tn, 1);
    for (size_t i = p->k + p->nu; i < tn; i++) er[i] = 1;
    int rc = decode_layered(p, er, chunks, chunk, sc, err);
    if (!rc) {
        for (size_t i = 0; i < p->k; i++) memcpy(out + i * chunk, chunks[i], chunk);
        for (size_t i = p->k + p->nu, j = p->k; i < tn; i++, j++) memcpy(out + j * chunk, chunks[i], chunk);
    }
    for (size_t i = 0; i < tn; i++) free(chunks[i]);
    free(chunks);
    free(er);
    return rc;
}

static int contains(const size_t *a, size_t n, size_t v) {
    for (size_t i = 0; i < n; i++) if (a[i] == v) return 1;
    return 0;
}

/* decode.rs:31-161 decode.  The HashMap is passed as parallel arrays; "first
 * chunk" (decode.rs:54-56) and the scan orders are the array order. */
int oc_decode(const oc_code_t *p, const size_t *ids, const uint8_t *const *bufs, const size_t *lens,
              size_t n_avail, const size_t *er, size_t n_er, uint8_t *out, size_t out_cap,
              size_t *out_len, oc_error_t *err) {
    clear_err(err);
    gf_init();
    if (out_len) *out_len = 0;
    if (n_avail == 0 && n_er == 0) return 0;
    if (n_avail == 0)
        return set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0,
                       "Invalid parameters: No available chunks provided but erasures are non-empty");
    if (n_er > p->m)
        return set_err(err, OC_TOO_MANY_ERASURES, p->m, n_er, 0, "Too many erasures: max %zu supported, got %zu", p->m, n_er);
    size_t chunk = lens[0];
    if (chunk == 0 || chunk % p->sub_chunk_no != 0)
        return set_err(err, OC_INVALID_CHUNK_SIZE, p->sub_chunk_no, chunk, 0,
                       "Invalid chunk size: expected divisible by %zu, got %zu", p->sub_chunk_no, chunk);
    for (size_t i = 1; i < n_avail; i++)
        if (lens[i] != chunk)
            return set_err(err, OC_INCONSISTENT_CHUNK_SIZES, chunk, ids[i], lens[i],
                           "Chunk %zu has size %zu but expected %zu (same as first chunk)", ids[i], lens[i], chunk);
    for (size_t i = 0; i < n_avail; i++)
        if (ids[i] >= p->n)
            return set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: Chunk index %zu out of range [0, %zu)", ids[i], p->n);
    for (size_t i = 0; i < n_er; i++)
        if (er[i] >= p->n)
            return set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: Erasure index %zu out of range [0, %zu)", er[i], p->n);
    for (size_t i = 0; i < n_er; i++)
        if (contains(ids, n_avail, er[i]))
            return set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0,
                           "Invalid parameters: Node %zu is both in available chunks and marked as erased", er[i]);
    size_t expected = p->n - n_er;
    if (n_avail != expected)
        return set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0,
                       "Invalid parameters: Expected %zu available chunks (n=%zu - erasures=%zu), but got %zu",
                       expected, p->n, n_er, n_avail);
    for (size_t node = 0; node < p->n; node++)
        if (!contains(er, n_er, node) && !contains(ids, n_avail, node))
            return set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0,
                           "Invalid parameters: Node %zu is neither erased nor provided in available chunks", node);
    size_t sc = chunk / p->sub_chunk_no, tn = p->q * p->t;
    uint8_t **chunks = (uint8_t **)malloc(tn * sizeof(uint8_t *));
    for (size_t i = 0; i < tn; i++) chunks[i] = (uint8_t *)calloc(chunk, 1);
    for (size_t i = 0; i < n_avail; i++) {
        size_t in = ids[i] < p->k ? ids[i] : ids[i] + p->nu;
        memcpy(chunks[in], bufs[i], chunk);
    }
    uint8_t *es = (uint8_t *)calloc(tn, 1);
    for (size_t i = 0; i < n_er; i++) es[er[i] < p->k ? er[i] : er[i] + p->nu] = 1;
    int rc = decode_layered(p, es, chunks, chunk, sc, err);
    if (!rc) {
        size_t need = p->k * chunk;
        if (out_cap < need) rc = set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: output buffer too small");
        else {
            for (size_t i = 0; i < p->k; i++) memcpy(out + i * chunk, chunks[i], chunk);
            if (out_len) *out_len = need;
        }
    }
    for (size_t i = 0; i < tn; i++) free(chunks[i]);
    free(chunks);
    free(es);
    return rc;
}

/* ---------------- repair.rs ---------------- */
/* repair.rs:22-49 get_repair_subchunk_indices */
int oc_repair_subchunk_indices(const oc_code_t *p, size_t lost_internal, size_t *out, size_t *n_out, oc_error_t *err) {
    size_t y_lost = lost_internal / p->q, x_lost = lost_internal % p->q;
    size_t seq, nseq;
    if (!oc_checked_pow(p->q, p->t - 1 - y_lost, &seq))
        return set_err(err, OC_OVERFLOW, 0, 0, 0, "Arithmetic overflow: q^(t-1-y) = %zu^%zu overflows", p->q, p->t - 1 - y_lost);
    if (!oc_checked_pow(p->q, y_lost, &nseq))
        return set_err(err, OC_OVERFLOW, 0, 0, 0, "Arithmetic overflow: q^y = %zu^%zu overflows", p->q, y_lost);
    size_t n = 0;
    for (size_t s = 0; s < nseq; s++) {
        size_t base = x_lost * seq + s * p->q * seq;
        for (size_t o = 0; o < seq; o++) out[n++] = base + o;
    }
    *n_out = n;
    return 0;
}

/* repair.rs:61-126 minimum_to_repair */
int oc_minimum_to_repair(const oc_code_t *p, size_t lost, const size_t *avail, size_t n_avail,
                         size_t *helpers_out, size_t *n_helpers, size_t *idx_out, size_t *n_idx,
                         oc_error_t *err) {
    clear_err(err);
    *n_helpers = 0;
    if (lost >= p->n)
        return set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: Invalid lost node index: %zu >= %zu", lost, p->n);
    size_t li = lost < p->k ? lost : lost + p->nu;
    int e = oc_repair_subchunk_indices(p, li, idx_out, n_idx, err);
    if (e) return e;
    size_t d = p->k + p->q - 1;
    size_t *res = (size_t *)malloc((p->q + n_avail + 1) * sizeof(size_t));
    size_t nr = 0, ys = li / p->q;
    for (size_t x = 0; x < p->q; x++) {
        size_t node = ys * p->q + x, ext;
        if (node == li) continue;
        if (node < p->k) ext = node;
        else if (node >= p->k + p->nu) ext = node - p->nu;
        else continue;
        if (contains(avail, n_avail, ext)) res[nr++] = ext;
    }
    for (size_t i = 0; i < n_avail; i++) {
        if (nr >= d) break;
        size_t node = avail[i];
        if (!contains(res, nr, node) && node != lost) res[nr++] = node;
    }
    if (nr < d) { free(res); return set_err(err, OC_INSUFFICIENT_HELPERS, d, nr, 0, "Insufficient helpers: need %zu, got %zu", d, nr); }
    for (size_t i = 0; i < d; i++) helpers_out[i] = res[i];
    *n_helpers = d;
    free(res);
    return 0;
}

/* repair.rs:140-421 repair */
int oc_repair(const oc_code_t *p, size_t lost, const size_t *ids, const uint8_t *const *bufs,
              const size_t *lens, size_t n_helpers, size_t chunk_size, uint8_t *out, oc_error_t *err) {
    clear_err(err);
    gf_init();
    size_t d = p->k + p->q - 1, q = p->q, t = p->t, alpha = p->sub_chunk_no;
    if (lost >= p->n)
        return set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: Invalid lost node index: %zu >= %zu", lost, p->n);
    if (n_helpers < d)
        return set_err(err, OC_INSUFFICIENT_HELPERS, d, n_helpers, 0, "Insufficient helpers: need %zu, got %zu", d, n_helpers);
    if (chunk_size == 0 || chunk_size % alpha != 0)
        return set_err(err, OC_INVALID_CHUNK_SIZE, alpha, chunk_size, 0, "Invalid chunk size: expected divisible by %zu, got %zu", alpha, chunk_size);
    size_t li = lost < p->k ? lost : lost + p->nu;
    size_t *ridx = (size_t *)malloc(alpha * sizeof(size_t)), nridx = 0;
    int rc = oc_repair_subchunk_indices(p, li, ridx, &nridx, err);
    if (rc) { free(ridx); return rc; }
    size_t sc = chunk_size / alpha, expected = nridx * sc, tn = q * t;
    size_t lost_y = li / q;
    for (size_t x = 0; x < q; x++) {
        size_t node = lost_y * q + x;
        if (node == li) continue;
        if (node >= p->k && node < p->k + p->nu) continue;
        size_t ext = node < p->k ? node : node - p->nu;
        if (!contains(ids, n_helpers, ext)) {
            free(ridx);
            return set_err(err, OC_MISSING_Y_SECTION_HELPER, lost, ext, 0,
                           "Missing required y-section helper %zu for repairing node %zu", ext, lost);
        }
    }
    rs_t rs;
    int re = rs_new(&rs, p->original_count, p->recovery_count);
    if (re) { free(ridx); return set_err(err, OC_RECONSTRUCTION_FAILED, 0, 0, 0, "RS reconstruction failed: RS init failed: %s", RS_ERR_NAMES[re]); }
    uint8_t *u_buf = (uint8_t *)calloc(tn * chunk_size, 1);
    uint8_t *u_comp = (uint8_t *)calloc(tn * alpha, 1);
    memset(out, 0, chunk_size);
    const uint8_t **hi = (const uint8_t **)calloc(tn, sizeof(uint8_t *)); /* helper_internal */
    for (size_t i = 0; i < n_helpers; i++) {
        size_t ext = ids[i];
        if (ext >= p->n) {
            rc = set_err(err, OC_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: Helper index %zu out of range [0, %zu)", ext, p->n);
            goto done;
        }
        size_t in = ext < p->k ? ext : ext + p->nu;
        if (lens[i] != expected) {
            rc = set_err(err, OC_INSUFFICIENT_HELPER_DATA, ext, expected, lens[i], "Helper %zu provided %zu bytes, expected %zu", ext, lens[i], expected);
            goto done;
        }
        hi[in] = bufs[i];
    }
    uint8_t *aloof = (uint8_t *)calloc(tn, 1);
    for (size_t i = 0; i < tn; i++)
        if (i != li && !hi[i] && (i < p->k || i >= p->k + p->nu)) aloof[i] = 1;
    uint8_t *zero = (uint8_t *)calloc(expected ? expected : 1, 1);
    for (size_t i = p->k; i < p->k + p->nu; i++) hi[i] = zero;
    long *plane_ind = (long *)malloc(alpha * sizeof(long));
    for (size_t z = 0; z < alpha; z++) plane_ind[z] = -1;
    for (size_t i = 0; i < nridx; i++) plane_ind[ridx[i]] = (long)i;
    /* BTreeMap<order, Vec<z>>: ascending order, then repair-index order */
    size_t *ord = (size_t *)malloc(nridx * sizeof(size_t)), max_ord = 0, zv[64];
    for (size_t i = 0; i < nridx; i++) {
        size_t z = ridx[i], o = 0;
        oc_get_plane_vector(z, t, q, zv);
        if (li % q == zv[li / q]) o++;
        for (size_t nd = 0; nd < tn; nd++) if (aloof[nd] && nd % q == zv[nd / q]) o++;
        ord[i] = o;
        if (o > max_ord) max_ord = o;
    }
    uint8_t *base = (uint8_t *)calloc(tn, 1);
    for (size_t x = 0; x < q; x++) base[lost_y * q + x] = 1;
    for (size_t i = 0; i < tn; i++) if (aloof[i]) base[i] = 1;
    uint8_t gamma_det = 1 ^ MUL_TABLE[GAMMA][GAMMA];
    (void)gamma_det;
    for (size_t o = 0; o <= max_ord && !rc; o++) {
        for (size_t pi = 0; pi < nridx && !rc; pi++) {
            if (ord[pi] != o) continue;
            size_t z = ridx[pi];
            oc_get_plane_vector(z, t, q, zv);
            uint8_t le[256];
            memcpy(le, base, tn);
            /* Phase 1 */
            for (size_t y = 0; y < t; y++)
                for (size_t x = 0; x < q; x++) {
                    size_t nxy = y * q + x;
                    if (base[nxy]) continue;
                    if (hi[nxy]) {
                        size_t z_y = zv[y], z_sw = oc_get_companion_layer(p, z, x, y, z_y), nsw = y * q + z_y;
                        if (z_y == x) {
                            memcpy(u_buf + nxy * chunk_size + z * sc, hi[nxy] + plane_ind[z] * sc, sc);
                            u_comp[nxy * alpha + z] = 1;
                        } else if (aloof[nsw]) {
                            if (u_comp[nsw * alpha + z_sw]) {
                                uint8_t *u = (uint8_t *)malloc(sc);
                                u_from_c_and_ustar(hi[nxy] + plane_ind[z] * sc, u_buf + nsw * chunk_size + z_sw * sc, u, sc);
                                memcpy(u_buf + nxy * chunk_size + z * sc, u, sc);
                                free(u);
                                u_comp[nxy * alpha + z] = 1;
                            } else {
                                le[nxy] = 1;
                            }
                        } else if (hi[nsw]) {
                            if (plane_ind[z_sw] >= 0) {
                                uint8_t *uxy = (uint8_t *)malloc(sc), *usw = (uint8_t *)malloc(sc);
                                prt_oriented(hi[nxy] + plane_ind[z] * sc, hi[nsw] + plane_ind[z_sw] * sc, x < z_y, uxy, usw, sc);
                                memcpy(u_buf + nxy * chunk_size + z * sc, uxy, sc);
                                memcpy(u_buf + nsw * chunk_size + z_sw * sc, usw, sc);
                                free(uxy); free(usw);
                                u_comp[nxy * alpha + z] = 1;
                                u_comp[nsw * alpha + z_sw] = 1;
                            }
                        } else {
                            le[nxy] = 1;
                        }
                    } else {
                        le[nxy] = 1;
                    }
                }
            /* Phase 2 */
            rc = decode_uncoupled_layer(p, le, z, sc, u_buf, chunk_size, &rs, err);
            if (rc) break;
            for (size_t i = 0; i < tn; i++) if (le[i]) u_comp[i * alpha + z] = 1;
            /* Phase 3 */
            for (size_t nd = 0; nd < tn; nd++) {
                if (!base[nd] || aloof[nd]) continue;
                size_t x = nd % q, y = nd / q, z_y = zv[y], nsw = y * q + z_y;
                size_t z_sw = oc_get_companion_layer(p, z, x, y, z_y);
                if (x == z_y) {
                    if (nd == li) memcpy(out + z * sc, u_buf + nd * chunk_size + z * sc, sc);
                } else if (nsw == li) {
                    if (hi[nd]) {
                        uint8_t *c = (uint8_t *)malloc(sc);
                        cstar_from_c_and_u(hi[nd] + plane_ind[z] * sc, u_buf + nd * chunk_size + z * sc, c, sc);
                        memcpy(out + z_sw * sc, c, sc);
                        free(c);
                    }
                }
            }
        }
    }
    free(base); free(ord); free(plane_ind); free(zero); free(aloof);
done:
    free(hi); free(u_comp); free(u_buf); free(ridx);
    rs_free(&rs);
    return rc;
}
