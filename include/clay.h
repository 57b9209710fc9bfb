/*
 * clay.h -- C ABI of the MI355X-native Clay (Coupled-Layer MSR) erasure-code engine.
 *
 * Drop-in boundary for the `ClayCode` API of spool-labs/clay (crate clay-codes
 * 0.1.2).  Every entry point names the reference interface it replaces.  The
 * signatures use plain pointers and sizes only (no torch / HIP types): a Rust
 * `extern "C"` block, ctypes, JNI or cgo binds them directly.
 *
 * Conventions
 *   - Return value: 0 on success, otherwise the error kind (enum clay_error_kind);
 *     if `err` is non-NULL it receives kind, payload fields and the Display text
 *     of the reference's ClayError (error.rs:26-54).
 *   - All buffers are caller-allocated; size-query helpers replace Rust's owned
 *     Vec returns.  `HashMap<usize, Vec<u8>>` arguments become parallel arrays
 *     (ids[i], bufs[i], lens[i]); where the reference depends on HashMap
 *     iteration order (decode.rs:54-56, repair.rs:225) this ABI uses array order.
 *   - Thread safety: like the reference (ClayCode is immutable, lib.rs:58), all
 *     functions may be called concurrently, from any thread, on any stream.  There is
 *     no process-wide lock: plan caches and per-device buffer pools are locked only
 *     for bookkeeping, never across a launch or a wait on the caller's stream.
 *   - Device buffers the library needs (U workspaces of decode/repair/staged encode,
 *     staging buffers of the host API) come from a per-device pool; a buffer is reused
 *     once the event recorded after its last use has completed, so streams that come
 *     and go do not grow device memory.  Buffers and pointer tables first used inside
 *     a stream capture stay reserved for the captured graph.
 *   - Host-buffer functions (clay_encode / clay_decode / clay_repair) copy to the
 *     GPU, run the HIP kernels and copy back.  *_device functions take device
 *     pointers and a hipStream_t (passed as void*) and are asynchronous.
 *   - There is no CPU fallback: without a usable GPU, compute entry points fail
 *     with CLAY_ERR_DEVICE.
 */
#ifndef CLAY_H
#define CLAY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CLAY_ABI_VERSION 4

/* ClayCode public fields (lib.rs:59-82) + the two private RS counts (lib.rs:79-81). */
typedef struct clay_code {
    size_t k, m, n, d, q, t, nu, sub_chunk_no, beta;
    size_t original_count, recovery_count;
} clay_code_t;

/* ClayError (error.rs:5-24).  Payload fields a,b,c follow declaration order:
 *   InsufficientHelpers{needed, provided}           -> a, b
 *   InvalidChunkSize{expected, actual}              -> a, b
 *   InsufficientHelperData{helper, expected, actual}-> a, b, c
 *   InconsistentChunkSizes{first_size, mismatched_idx, mismatched_size} -> a, b, c
 *   TooManyErasures{max, actual}                    -> a, b
 *   MissingYSectionHelper{lost_node, missing_helper}-> a, b
 * String variants carry their text in msg only. */
enum clay_error_kind {
    CLAY_OK = 0,
    CLAY_ERR_INVALID_PARAMETERS = 1,
    CLAY_ERR_INSUFFICIENT_HELPERS = 2,
    CLAY_ERR_INVALID_CHUNK_SIZE = 3,
    CLAY_ERR_INSUFFICIENT_HELPER_DATA = 4,
    CLAY_ERR_INCONSISTENT_CHUNK_SIZES = 5,
    CLAY_ERR_TOO_MANY_ERASURES = 6,
    CLAY_ERR_RECONSTRUCTION_FAILED = 7,
    CLAY_ERR_MISSING_Y_SECTION_HELPER = 8,
    CLAY_ERR_OVERFLOW = 9,
    /* not in the reference: HIP runtime / device failure, unsupported device shape */
    CLAY_ERR_DEVICE = 100,
};

typedef struct clay_error {
    int kind;
    size_t a, b, c;
    char msg[256];
} clay_error_t;

/* ------------------------------------------------------------------ */
/* Parameters                                                          */
/* ------------------------------------------------------------------ */

/* ClayCode::new(k, m, d)            -- lib.rs:94-147 */
int clay_new(size_t k, size_t m, size_t d, clay_code_t *out, clay_error_t *err);
/* ClayCode::new_default(k, m)       -- lib.rs:150-152 (d = k + m - 1) */
int clay_new_default(size_t k, size_t m, clay_code_t *out, clay_error_t *err);
/* ClayCode::normalized_repair_bandwidth -- lib.rs:239-241 */
double clay_normalized_repair_bandwidth(const clay_code_t *code);
/* Chunk size ClayCode::encode produces for `data_len` bytes -- encode.rs:33-42 */
size_t clay_encoded_chunk_size(const clay_code_t *code, size_t data_len);

/* ------------------------------------------------------------------ */
/* Host-buffer API (mirrors the reference semantics)                   */
/* ------------------------------------------------------------------ */

/* ClayCode::encode(data) -> Vec<Vec<u8>>   -- lib.rs:176-178, encode.rs:30-80.
 * out_chunks: n host buffers of chunk_size bytes (chunk_size must equal
 * clay_encoded_chunk_size(code, len)); [0,k) receive the zero-padded data
 * chunks, [k,n) the parity chunks.  The reference panics on an internal error
 * (encode.rs:67-68); this ABI returns CLAY_ERR_RECONSTRUCTION_FAILED instead. */
int clay_encode(const clay_code_t *code, const uint8_t *data, size_t len,
                uint8_t *const *out_chunks, size_t chunk_size, clay_error_t *err);

/* ClayCode::decode(available, erasures) -> Vec<u8> -- lib.rs:188-194, decode.rs:31-161.
 * available: n_avail entries (ids, bufs, lens).  out receives k*chunk bytes
 * (the first k internal chunks, padding included, decode.rs:155-158);
 * *out_len = k*chunk (0 for the empty/empty case).  out_cap < k*chunk ->
 * CLAY_ERR_INVALID_PARAMETERS. */
int clay_decode(const clay_code_t *code, const size_t *ids, const uint8_t *const *bufs,
                const size_t *lens, size_t n_avail, const size_t *erasures, size_t n_erasures,
                uint8_t *out, size_t out_cap, size_t *out_len, clay_error_t *err);

/* ClayCode::minimum_to_repair(lost, available) -- lib.rs:207-213, repair.rs:61-126.
 * Every helper needs the same sub-chunk list (repair.rs:102,113), so the result
 * is helpers_out[0..*n_helpers) (capacity >= d) plus one index list
 * subchunks_out[0..*n_subchunks) (capacity >= beta). */
int clay_minimum_to_repair(const clay_code_t *code, size_t lost_node, const size_t *available,
                           size_t n_available, size_t *helpers_out, size_t *n_helpers,
                           size_t *subchunks_out, size_t *n_subchunks, clay_error_t *err);

/* ClayCode::repair(lost, helper_data, chunk_size) -- lib.rs:226-233, repair.rs:140-421.
 * helper i: ids[i], bufs[i] (lens[i] bytes = the beta sub-chunks concatenated in
 * minimum_to_repair order).  out receives chunk_size bytes. */
int clay_repair(const clay_code_t *code, size_t lost_node, const size_t *ids,
                const uint8_t *const *bufs, const size_t *lens, size_t n_helpers,
                size_t chunk_size, uint8_t *out, clay_error_t *err);

/* ------------------------------------------------------------------ */
/* Device-resident API (HBM in, HBM out; asynchronous on `stream`)      */
/* ------------------------------------------------------------------ */

/* Encode one stripe already resident in HBM.  data_chunks: k device pointers
 * (chunk_size bytes each, chunk_size % sub_chunk_no == 0), parity_chunks: m
 * device pointers.  Pointer arrays themselves are host memory.  Same bytes as
 * clay_encode's parity for the same (padded) data.  stream: hipStream_t or NULL. */
int clay_encode_device(const clay_code_t *code, const uint8_t *const *data_chunks,
                       uint8_t *const *parity_chunks, size_t chunk_size, int device,
                       void *stream, clay_error_t *err);

/* Batched encode: `n_stripes` independent stripes, stripe s uses
 * data_chunks[s*k .. s*k+k) and parity_chunks[s*m .. s*m+m). */
int clay_encode_device_batch(const clay_code_t *code, const uint8_t *const *data_chunks,
                             uint8_t *const *parity_chunks, size_t n_stripes, size_t chunk_size,
                             int device, void *stream, clay_error_t *err);

/* Host-streaming encode (host memory in, host memory out; blocking).  data_chunks:
 * k host pointers, parity_chunks: m host pointers (chunk_size bytes each; pin
 * them, e.g. hipHostMalloc / hipHostRegister, for overlap).  The stripe is cut
 * into pieces of piece_bytes (0 = auto, ~128 MiB of input per piece) of every
 * sub-chunk; each piece is copied in with one 2D copy per node, encoded on the
 * device and its parity copied out, round-robin over n_streams (0 = 2) streams
 * so H2D, encode and D2H of consecutive pieces overlap.  Same parity bytes as
 * clay_encode / clay_encode_device.  Replaces the host-side entry of
 * ClayCode::encode (lib.rs:165-167 -> encode.rs:30-80) for callers that hold
 * the data chunks in host memory. */
int clay_encode_host_pipelined(const clay_code_t *code, const uint8_t *const *data_chunks,
                               uint8_t *const *parity_chunks, size_t chunk_size, int device,
                               size_t piece_bytes, int n_streams, clay_error_t *err);

/* Batched encode of n_stripes stripes laid out at fixed strides in device memory
 * (the reference encodes one stripe per call, encode.rs:30-80):
 * data node i of stripe s at data + s*data_stripe_stride + i*data_node_stride, parity
 * node j at parity + s*parity_stripe_stride + j*parity_node_stride (bytes; e.g. a
 * contiguous [n_stripes][k][chunk] buffer has node stride chunk, stripe stride k*chunk).
 * Same results as clay_encode_device_batch with the equivalent pointer arrays, with O(1)
 * host work per call.  Asynchronous on `stream`. */
int clay_encode_device_strided(const clay_code_t *code, const uint8_t *data, int64_t data_node_stride,
                               int64_t data_stripe_stride, uint8_t *parity, int64_t parity_node_stride,
                               int64_t parity_stripe_stride, size_t n_stripes, size_t chunk_size, int device,
                               void *stream, clay_error_t *err);

/* Y-grouped chunk layout ("Option C" of the reference's
 * docs/clay-practical-implementation.md:416-582, in the crate's MSB-first digit order):
 * for y-section y, the chunk's alpha sub-chunks reordered as blocks x = 0..q-1 of beta
 * sub-chunks, block x = the layers z with digit_y(z) == x in ascending order
 * (= get_repair_subchunk_indices of node (y, x), repair.rs:22-49).  A helper stored this
 * way serves the repair of node (y, x) from ONE contiguous range, group + x*beta*sc, which
 * can be passed straight to clay_repair_device.  Device buffers of chunk_size bytes, not
 * in place; asynchronous on `stream`. */
int clay_chunk_to_ygroup(const clay_code_t *code, size_t y, const uint8_t *chunk, uint8_t *group,
                         size_t chunk_size, int device, void *stream, clay_error_t *err);
int clay_ygroup_to_chunk(const clay_code_t *code, size_t y, const uint8_t *group, uint8_t *chunk,
                         size_t chunk_size, int device, void *stream, clay_error_t *err);

/* Decode / rebuild on device.  chunks: n device pointers, NULL for every erased
 * node (validation as decode.rs:36-126 with available = the non-NULL entries).
 * out_chunks: n device pointers; for every erased DATA node out_chunks[i] must
 * be non-NULL and receives the rebuilt chunk; for an erased PARITY node a
 * non-NULL out_chunks[i] also receives the rebuilt parity chunk (the value the
 * reference computes internally, decode.rs:213-253); other entries are ignored. */
int clay_decode_device(const clay_code_t *code, const uint8_t *const *chunks,
                       const size_t *erasures, size_t n_erasures, uint8_t *const *out_chunks,
                       size_t chunk_size, int device, void *stream, clay_error_t *err);

/* clay_decode_device for callers whose chunks are ONE CODEWORD (the crate's own usage: chunks
 * that ClayCode::encode produced), chosen per call.  A decode of one erased node with every other
 * node present, in a q = m code with a streaming repair kernel ((9,3,11), (10,4,13), (4,2,5)),
 * rebuilds the node with the repair of repair.rs:140-421 from the whole chunks (last exec path
 * "bs-repair-stream", when the sub-chunk gives every CU a tile): it reads only the alpha / q layers
 * of the node's repair plane (repair.rs:61-126) instead of every layer ((10,4,13) 1 GiB {0}:
 * 0.137 ms vs 0.350 on the local decode).  On a codeword the bytes equal decode.rs:31-161's (the
 * codeword through the k data chunks is unique); on chunks that are NOT one codeword they differ,
 * which is why clay_decode_device never takes this route.  Every other pattern runs exactly as
 * clay_decode_device.  The choice is an argument of the call, not process state: concurrent
 * clay_decode_device calls are unaffected.  The repair route is taken under exec modes auto and
 * "stream" only (as clay_repair_device's kernel choice); under "grouped" / "tile" the call runs
 * as clay_decode_device.  No reference counterpart (decode.rs has one path). */
int clay_decode_device_codeword(const clay_code_t *code, const uint8_t *const *chunks,
                                const size_t *erasures, size_t n_erasures, uint8_t *const *out_chunks,
                                size_t chunk_size, int device, void *stream, clay_error_t *err);

/* Repair on device: helper buffers are device pointers (beta*sub-chunk bytes),
 * out is a device buffer of chunk_size bytes. */
int clay_repair_device(const clay_code_t *code, size_t lost_node, const size_t *helper_ids,
                       const uint8_t *const *helper_bufs, size_t n_helpers, size_t chunk_size,
                       uint8_t *out, int device, void *stream, clay_error_t *err);

/* Repair on device from WHOLE helper chunks (device pointers, chunk_size bytes
 * each): the kernels read the beta repair layers of repair.rs:22-49 in place, so
 * callers holding full chunks in HBM skip the gather/concat that
 * minimum_to_repair's index lists imply (repair.rs:61-126).
 * Same output bytes as clay_repair on the gathered sub-chunks. */
int clay_repair_device_full_chunks(const clay_code_t *code, size_t lost_node, const size_t *helper_ids,
                                   const uint8_t *const *helper_chunks, size_t n_helpers,
                                   size_t chunk_size, uint8_t *out, int device, void *stream,
                                   clay_error_t *err);

/* ------------------------------------------------------------------ */
/* Engine control / introspection                                      */
/* ------------------------------------------------------------------ */

/* Pre-allocate an idle pooled workspace for chunk_size (any stream may take it) and
 * build + upload the code's encode plan, so that a later call allocates nothing --
 * e.g. before stream capture.  The workspace is q x t x chunk_size bytes, the grouped
 * executor's U workspace for that chunk size, held per in-flight call (the streaming
 * kernels need none).  Decode/repair plans and the
 * streaming decode's pattern tables depend on the erasure pattern: run one call per
 * pattern before capturing it (a capture that needs an unprepared one fails with
 * CLAY_ERR_DEVICE rather than allocating). */
int clay_reserve_workspace(const clay_code_t *code, size_t chunk_size, int device,
                           clay_error_t *err);

/* Free the device's idle pooled buffers (waiting for their last users' events) and
 * its unpinned batch pointer tables.  Buffers in use or owned by captured graphs stay. */
int clay_release_workspace(int device, clay_error_t *err);

/* Reclaim what calls made inside stream captures left to their graphs: the pointer tables of
 * captured batch calls (a 4 MiB per-device arena; a captured batch of n stripes takes
 * n x 130 x 8 bytes, so about a dozen 300-stripe captures fill it, after which capturing
 * such calls fails with CLAY_ERR_DEVICE) and the pooled workspaces pinned to graphs.
 * The caller MUST first synchronise every stream that replays those graphs and destroy the
 * graphs: the released workspaces are handed to the next call at once, with no event to wait
 * on, so a replay still running would race that call.  It does not synchronise the device
 * itself (that would invalidate another thread's capture in global mode), so it is safe while
 * other threads capture unrelated work; it fails (nothing released) while one of this
 * library's calls runs inside a capture, or while a capture that took a workspace or a table
 * from this library is still open.  No reference counterpart. */
int clay_release_captured(int device, clay_error_t *err);

/* Bytes of device memory held by the device's buffer pool (tests / monitoring). */
size_t clay_workspace_bytes(int device);

/* Encode path selection (process-wide; tests and benchmarks).  Low byte = path:
 *   0 auto      -- the streaming kernel for q = 4, t = 4 codes with k = 9 / 10 (the
 *                  BASELINE (10,4,13)) and for (9,3,11) (k_stream_encode3: any sub-chunk
 *                  size >= 16 and any alignment); (4,2,5): the line-local bit-sliced kernel
 *                  (k_bs_encode1, "bitsliced-line-k4m2-w2048", any sub-chunk and alignment);
 *                  else the bit-sliced v1 kernel if the code has a
 *                  compiled instantiation; else the byte-sliced fused kernel when the
 *                  parity is one y-section; else the staged plan executor.  Batches of
 *                  >= 4 stripes of <= 4 MiB of data run as one staged launch per level.
 *                  The LDS-DMA kernel (stream) needs sub-chunks that are
 *                  multiples of 8 bytes and 8-byte aligned chunk pointers (else auto
 *                  falls through); the v1 kernel takes any sub-chunk size and alignment.
 *   1 staged    -- the plan executor (k_gexec), any code
 *   2 fused     -- byte-sliced fused kernel (q == m <= 4)
 *   3 bitsliced -- bit-sliced v1 (register loads); variant = lanes per column group
 *                  for (10,4,13): 0 (2), 1, 4; (4,2,5) runs v1 here, not the line kernel
 *   5 stream    -- the streaming kernel (stream_encode.hpp); variant = loader waves
 *                  for (10,4,13): 0 (= 4, the default), 1, 2, 4; (9,4,12) always runs
 *                  4 loader waves (its variant is accepted and ignored); (9,3,11): 7 loader
 *                  waves for variant 7, else 2 (stream_encode3.hpp)
 * (4, the v6 kernel of round 1, is retired.)  Bits 8..15 = variant.  Every accepted (path, variant) produces the reference's
 * parity bytes; any other value returns -1 and leaves the setting unchanged.
 * Returns the previous setting (path | variant << 8). */
int clay_set_encode_path(int mode);

/* Plan executor for decode, repair and the staged encode (process-wide tuning knob; no
 * reference counterpart -- the crate has one CPU path).  A mode only chooses kernels: every
 * mode returns the reference's bytes on any input.
 *   0 auto    -- the tile-fused executor (one launch, U workspace in LDS) for small plans
 *                (<= 32 op groups) whose U slots fit the LDS budget, else the grouped
 *                per-level executor; for q = 4, t = 4 codes ((10,4,13), (9,4,12)) with
 *                sc >= 512: decodes whose erasures lie in one y-section plus at most one
 *                erasure in one other section ({0}, {0,4}, {0,1}, {0,1,4}, {0,1,2,3}, ...) run
 *                a single-launch local decode: one erasure in its section plus at most one
 *                more, or two in one section ({0}, {12}, {0,4}, {0,1}), on 256-byte row runs
 *                (k_stream_local256, last path "stream-local256", any sub-chunk), the others
 *                on 64-byte tiles (k_stream_local, "stream-local", sc % 8 == 0) -- except
 *                three erasures as two in one section and one in another ({0,1,4}), which
 *                take the fused decode v2 first; 3 or 4 erasures with at most two per
 *                y-section (sc % 8 == 0; the BASELINE {0,4,8,12} and the (2,1,1) / (2,2)
 *                patterns included) the fused decode v2 (k_stream_fused2, "stream-fused2");
 *                (4,2,5) with one erasure and every other chunk present: the single-erasure
 *                bit-sliced decode (k_bs_decode1, "bs-decode1", any sub-chunk and alignment)
 *   1 grouped -- always the grouped executor (k_gexec, one launch per level)
 *   2 tile    -- the tile executor wherever its U slots fit, whatever the plan size
 *   (auto and stream: repair of (9,3,11), (10,4,13), (4,2,5) from all n - 1 other nodes runs
 *    the bit-sliced repair kernels: k_bs_repair_stream (LDS-DMA streaming, one workgroup per
 *    CU; auto when the sub-chunk gives every CU a tile, stream for any sub-chunk >= 16 bytes
 *    of (9,3,11) / (10,4,13); last path "bs-repair-stream"), else k_bs_repair ("bs-repair"))
 *   3 stream  -- every decode a streaming kernel takes on it: the local decode where it takes
 *                the pattern (the (2,1) patterns: the fused decode v2 first), else the fused
 *                decode v2 (2-4 erasures, at most two per section); everything else as auto
 *   5 stream-local -- every decode a local kernel takes on it ("stream-local256" /
 *                "stream-local"); else as auto
 *   6 stream-fused2 -- decodes of 2-4 erasures with at most two per y-section on the fused
 *                decode v2 (k_stream_fused2, "stream-fused2"; ring of 10 - e node buffers: a
 *                section's surviving real nodes fit it, two neighbouring sections that do not
 *                run as a split step; the loader waves' round items fit their registers);
 *                else as auto
 * (4 and 7 are retired: the single-launch decode of round 3 and the process-wide "codeword"
 * mode, now the per-call clay_decode_device_codeword.)
 * No CLAY_* environment variable is read on a call path; the measurement knobs (planner and
 * executor tuning, CLAY_LOCAL_W64 = the 64-byte local kernel for every local pattern) are read
 * once when the library is loaded.
 * Returns the previous mode, or -1 for an unknown mode (setting unchanged). */
int clay_set_exec_mode(int mode);
/* Plan executor the calling thread's last decode / repair / staged encode ran on:
 * "tile" (k_texec), "grouped" (k_gexec), "stream-local256" (k_stream_local256), "stream-local"
 * (k_stream_local), "stream-fused2"
 * (k_stream_fused2), "bs-decode1" (k_bs_decode1), "bs-repair-stream" (k_bs_repair_stream),
 * "bs-repair" (k_bs_repair) or "none". */
const char *clay_last_exec_path(void);

/* Name of the path the last encode on this thread used ("fused-q4w128p8", "staged", ...). */
const char *clay_last_encode_path(void);

/* Number of kernel launches the last device call on this thread issued. */
size_t clay_last_launch_count(void);

/* Introspection (tests / tooling): export the staged-engine plan -- the
 * reference's layered algorithm replayed into GF(2^8) region ops
 * "dst = XOR coef*src" -- for kind 0 = encode, 1 = decode (mask = erased
 * internal nodes, want = erased nodes whose C is wanted), 2 = repair (mask =
 * helper internal nodes, lost = external lost node).  Records are uint32:
 * ops_out[4*i..] = {dst_base, dst_slot, src_begin, nsrc}, srcs_out[4*j..] =
 * {base, slot, coef, 0}, stages_out = stage begin offsets (n_stages+1).  Base
 * index b: b < tn -> C[node b]; tn <= b < 2tn -> helper H[node b-tn]; 2tn -> U
 * workspace (slot = node*alpha + z); 2tn+1 -> repaired chunk.  counts[] =
 * {n_ops, n_srcs, n_stages+1}.  Capacities too small -> only counts filled. */
int clay_plan_export(const clay_code_t *code, int kind, const uint8_t *mask, const uint8_t *want,
                     size_t lost_node, uint32_t *ops_out, size_t ops_cap, uint32_t *srcs_out,
                     size_t srcs_cap, uint32_t *stages_out, size_t stages_cap, size_t counts[3],
                     clay_error_t *err);

/* ABI version (CLAY_ABI_VERSION) and build string. */
int clay_abi_version(void);
const char *clay_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* CLAY_H */
