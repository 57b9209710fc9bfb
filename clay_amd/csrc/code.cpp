// code.cpp -- parameters and validation with the reference's error precedence.
#include "code.hpp"
#include "tuning.hpp"

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>

namespace clay {

Error make_error(int kind, size_t a, size_t b, size_t c, const char *fmt, ...) {
    Error e;
    e.kind = kind;
    e.a = a;
    e.b = b;
    e.c = c;
    char buf[256];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    e.msg = buf;
    return e;
}

int report(const Error &e, clay_error_t *out) {
    if (out) {
        out->kind = e.kind;
        out->a = e.a;
        out->b = e.b;
        out->c = e.c;
        std::snprintf(out->msg, sizeof(out->msg), "%s", e.msg.c_str());
    }
    return e.kind;
}

bool checked_pow(size_t base, size_t exp, size_t *out) {
    size_t result = 1, b = base, e = exp;
    while (e > 0) {
        if ((e & 1) && __builtin_mul_overflow(result, b, &result)) return false;
        e >>= 1;
        if (e > 0 && __builtin_mul_overflow(b, b, &b)) return false;
    }
    *out = result;
    return true;
}

Error code_new(size_t k, size_t m, size_t d, clay_code_t *out) {
    if (k < 1) return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: k must be at least 1");
    if (m < 1) return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: m must be at least 1");
    if (d < k + 1 || d > k + m - 1)
        return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0,
                          "Invalid parameters: d must be in range [%zu, %zu], got %zu", k + 1, k + m - 1, d);
    size_t q = d - k + 1, n = k + m;
    size_t nu = (n % q == 0) ? 0 : q - (n % q);
    size_t t = (n + nu) / q;
    size_t alpha;
    if (!checked_pow(q, t, &alpha))
        return make_error(CLAY_ERR_OVERFLOW, 0, 0, 0, "Arithmetic overflow: q^t = %zu^%zu overflows", q, t);
    if (k + nu > 32768 || m > 32768)
        return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0,
                          "Invalid parameters: Total nodes exceeds reed-solomon limit of 32768");
    out->k = k;
    out->m = m;
    out->n = n;
    out->d = d;
    out->q = q;
    out->t = t;
    out->nu = nu;
    out->sub_chunk_no = alpha;
    out->beta = alpha / q;
    out->original_count = k + nu;
    out->recovery_count = m;
    return Error{};
}

size_t encoded_chunk_size(const clay_code_t &c, size_t len) {
    size_t min_size = c.k * c.sub_chunk_no * 2;
    size_t padded = len == 0 ? min_size : ((len + min_size - 1) / min_size) * min_size;
    if (padded < min_size) padded = min_size;
    return padded / c.k;
}

void plane_vector(const clay_code_t &c, size_t z, size_t *out) {
    size_t rem = z;
    for (size_t i = 0; i < c.t; i++) {
        out[c.t - 1 - i] = rem % c.q;
        rem /= c.q;
    }
}

size_t companion_layer(const clay_code_t &c, size_t z, size_t x, size_t y, size_t z_y) {
    size_t w = 1;
    for (size_t i = 0; i + 1 + y < c.t; i++) w *= c.q;
    // z_sw = (z + (x - z_y) * q^(t-1-y)) mod alpha; digit y of z is z_y so this never wraps.
    return x >= z_y ? z + (x - z_y) * w : z - (z_y - x) * w;
}

static bool contains(const size_t *a, size_t n, size_t v) {
    for (size_t i = 0; i < n; i++)
        if (a[i] == v) return true;
    return false;
}

Error validate_decode(const clay_code_t &c, const AvailView &av, const size_t *er, size_t ner,
                      size_t *chunk_size, std::vector<uint8_t> &erased) {
    *chunk_size = 0;
    if (av.n == 0)
        return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0,
                          "Invalid parameters: No available chunks provided but erasures are non-empty");
    if (ner > c.m)
        return make_error(CLAY_ERR_TOO_MANY_ERASURES, c.m, ner, 0, "Too many erasures: max %zu supported, got %zu",
                          c.m, ner);
    size_t chunk = av.lens[0];
    if (chunk == 0 || chunk % c.sub_chunk_no != 0)
        return make_error(CLAY_ERR_INVALID_CHUNK_SIZE, c.sub_chunk_no, chunk, 0,
                          "Invalid chunk size: expected divisible by %zu, got %zu", c.sub_chunk_no, chunk);
    for (size_t i = 1; i < av.n; i++)
        if (av.lens[i] != chunk)
            return make_error(CLAY_ERR_INCONSISTENT_CHUNK_SIZES, chunk, av.ids[i], av.lens[i],
                              "Chunk %zu has size %zu but expected %zu (same as first chunk)", av.ids[i],
                              av.lens[i], chunk);
    for (size_t i = 0; i < av.n; i++)
        if (av.ids[i] >= c.n)
            return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0,
                              "Invalid parameters: Chunk index %zu out of range [0, %zu)", av.ids[i], c.n);
    for (size_t i = 0; i < ner; i++)
        if (er[i] >= c.n)
            return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0,
                              "Invalid parameters: Erasure index %zu out of range [0, %zu)", er[i], c.n);
    for (size_t i = 0; i < ner; i++)
        if (contains(av.ids, av.n, er[i]))
            return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0,
                              "Invalid parameters: Node %zu is both in available chunks and marked as erased",
                              er[i]);
    // HashMap keys are unique; parallel arrays could repeat an id.
    for (size_t i = 0; i < av.n; i++)
        for (size_t j = i + 1; j < av.n; j++)
            if (av.ids[i] == av.ids[j])
                return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0,
                                  "Invalid parameters: Chunk index %zu given twice", av.ids[i]);
    size_t expected = c.n - ner;
    if (av.n != expected)
        return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0,
                          "Invalid parameters: Expected %zu available chunks (n=%zu - erasures=%zu), but got %zu",
                          expected, c.n, ner, av.n);
    for (size_t node = 0; node < c.n; node++)
        if (!contains(er, ner, node) && !contains(av.ids, av.n, node))
            return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0,
                              "Invalid parameters: Node %zu is neither erased nor provided in available chunks",
                              node);
    // decode_layered builds ReedSolomon::new(original_count, recovery_count) before any
    // layer work, even with no data node erased (decode.rs:175-180): galois_8 allows at
    // most 256 shards
    if (c.original_count + c.recovery_count > 256)
        return make_error(CLAY_ERR_RECONSTRUCTION_FAILED, 0, 0, 0,
                          "RS reconstruction failed: RS init failed: TooManyShards");
    erased.assign(c.q * c.t, 0);
    for (size_t i = 0; i < ner; i++) erased[internal_of(c, er[i])] = 1;
    *chunk_size = chunk;
    return Error{};
}

Error repair_subchunk_indices(const clay_code_t &c, size_t li, std::vector<size_t> &out) {
    size_t y = li / c.q, x = li % c.q, seq, nseq;
    if (!checked_pow(c.q, c.t - 1 - y, &seq))
        return make_error(CLAY_ERR_OVERFLOW, 0, 0, 0, "Arithmetic overflow: q^(t-1-y) = %zu^%zu overflows", c.q,
                          c.t - 1 - y);
    if (!checked_pow(c.q, y, &nseq))
        return make_error(CLAY_ERR_OVERFLOW, 0, 0, 0, "Arithmetic overflow: q^y = %zu^%zu overflows", c.q, y);
    out.clear();
    out.reserve(c.sub_chunk_no / c.q);
    for (size_t s = 0; s < nseq; s++) {
        size_t base = x * seq + s * c.q * seq;
        for (size_t o = 0; o < seq; o++) out.push_back(base + o);
    }
    return Error{};
}

Error minimum_to_repair(const clay_code_t &c, size_t lost, const size_t *av, size_t nav,
                        std::vector<size_t> &helpers, std::vector<size_t> &sub) {
    helpers.clear();
    if (lost >= c.n)
        return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: Invalid lost node index: %zu >= %zu",
                          lost, c.n);
    size_t li = internal_of(c, lost);
    Error e = repair_subchunk_indices(c, li, sub);
    if (e) return e;
    size_t d = c.k + c.q - 1, ys = li / c.q;
    for (size_t x = 0; x < c.q; x++) {
        size_t node = ys * c.q + x, ext;
        if (node == li) continue;
        if (node < c.k) ext = node;
        else if (node >= c.k + c.nu) ext = node - c.nu;
        else continue;
        if (contains(av, nav, ext)) helpers.push_back(ext);
    }
    for (size_t i = 0; i < nav; i++) {
        if (helpers.size() >= d) break;
        size_t node = av[i];
        if (!contains(helpers.data(), helpers.size(), node) && node != lost) helpers.push_back(node);
    }
    if (helpers.size() < d)
        return make_error(CLAY_ERR_INSUFFICIENT_HELPERS, d, helpers.size(), 0, "Insufficient helpers: need %zu, got %zu",
                          d, helpers.size());
    helpers.resize(d);
    return Error{};
}

Error validate_repair(const clay_code_t &c, size_t lost, const size_t *ids, const size_t *lens, size_t nh,
                      size_t chunk_size, std::vector<uint8_t> &helper_int, std::vector<long> &slot_of_id,
                      std::vector<size_t> &sub) {
    size_t d = c.k + c.q - 1, alpha = c.sub_chunk_no;
    if (lost >= c.n)
        return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: Invalid lost node index: %zu >= %zu",
                          lost, c.n);
    if (nh < d)
        return make_error(CLAY_ERR_INSUFFICIENT_HELPERS, d, nh, 0, "Insufficient helpers: need %zu, got %zu", d, nh);
    if (chunk_size == 0 || chunk_size % alpha != 0)
        return make_error(CLAY_ERR_INVALID_CHUNK_SIZE, alpha, chunk_size, 0,
                          "Invalid chunk size: expected divisible by %zu, got %zu", alpha, chunk_size);
    size_t li = internal_of(c, lost);
    Error e = repair_subchunk_indices(c, li, sub);
    if (e) return e;
    size_t sc = chunk_size / alpha, expected = sub.size() * sc, ly = li / c.q;
    for (size_t x = 0; x < c.q; x++) {
        size_t node = ly * c.q + x;
        if (node == li || is_shortened(c, node)) continue;
        size_t ext = node < c.k ? node : node - c.nu;
        if (!contains(ids, nh, ext))
            return make_error(CLAY_ERR_MISSING_Y_SECTION_HELPER, lost, ext, 0,
                              "Missing required y-section helper %zu for repairing node %zu", ext, lost);
    }
    if (c.original_count + c.recovery_count > 256)
        return make_error(CLAY_ERR_RECONSTRUCTION_FAILED, 0, 0, 0,
                          "RS reconstruction failed: RS init failed: TooManyShards");
    for (size_t i = 0; i < nh; i++)
        for (size_t j = i + 1; j < nh; j++)
            if (ids[i] == ids[j])
                return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: Helper index %zu given twice",
                                  ids[i]);
    helper_int.assign(c.q * c.t, 0);
    slot_of_id.assign(c.q * c.t, -1);
    for (size_t i = 0; i < nh; i++) {
        if (ids[i] >= c.n)
            return make_error(CLAY_ERR_INVALID_PARAMETERS, 0, 0, 0, "Invalid parameters: Helper index %zu out of range [0, %zu)",
                              ids[i], c.n);
        if (lens && lens[i] != expected)
            return make_error(CLAY_ERR_INSUFFICIENT_HELPER_DATA, ids[i], expected, lens[i],
                              "Helper %zu provided %zu bytes, expected %zu", ids[i], lens[i], expected);
        size_t in = internal_of(c, ids[i]);
        helper_int[in] = 1;
        slot_of_id[in] = long(i);
    }
    return Error{};
}

// ---- tuning knobs: read once, at load time (tuning.hpp) ----
static Tuning read_tuning() {
    Tuning t;
    auto ival = [](const char *name, long long def) -> long long {
        const char *e = getenv(name);
        return e && *e ? atoll(e) : def;
    };
    t.plan_inline = ival("CLAY_PLAN_INLINE", 1) == 0 ? 0 : 1;
    t.plan_dup = int(ival("CLAY_PLAN_DUP", -1));
    t.plan_fold_cost = int(ival("CLAY_PLAN_FOLD_COST", -1));
    t.plan_defer_out = int(ival("CLAY_PLAN_DEFER_OUT", -1));
    t.plan_merge_slack = int(ival("CLAY_PLAN_MERGE_SLACK", -1));
    t.plan_debug = getenv("CLAY_PLAN_DEBUG") != nullptr;
    const long long w = ival("CLAY_TEXEC_WAVES", 0);
    t.texec_waves = w == 4 || w == 8 || w == 16 ? int(w) : 0;
    t.texec_lds = size_t(ival("CLAY_TEXEC_LDS_KB", 80)) * 1024;
    t.texec_big = ival("CLAY_TEXEC_BIG", 0) != 0;
    t.gexec_pipe = ival("CLAY_GEXEC_PIPE", 1) != 0;
    t.gexec_order = uint32_t(ival("CLAY_GEXEC_ORDER", 2));
    const long long tpw = ival("CLAY_GEXEC_TPW", 0);
    t.gexec_tpw = tpw >= 1 && tpw <= 64 ? int(tpw) : 0;
    t.gexec_small = uint64_t(ival("CLAY_GEXEC_SMALL", 2048));
    t.gexec_big = uint64_t(ival("CLAY_GEXEC_BIG", 32768));
    t.host_piece = size_t(ival("CLAY_HOST_PIECE_MB", 256)) << 20;
    t.host_streams = int(ival("CLAY_HOST_STREAMS", 2));
    t.decode_probe = int(ival("CLAY_DECODE_PROBE", 0));
    const long long ring = ival("CLAY_DECODE_RING", 10);
    t.decode_ring = uint32_t(ring >= 6 && ring <= 10 ? ring : 10);
    t.local_w64 = ival("CLAY_LOCAL_W64", 0) != 0;
    return t;
}
// namespace-scope: initialised when the library is loaded, before any ABI call
static const Tuning g_tuning = read_tuning();
const Tuning &tuning() { return g_tuning; }

}  // namespace clay
