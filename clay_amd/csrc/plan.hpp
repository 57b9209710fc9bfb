// plan.hpp -- symbolic replay of the reference's layered algorithms into a
// staged list of GF(2^8) region operations executed by the GPU.
//
// Every byte operation of the reference (PRT/PFT and partial transforms,
// transforms.rs:42-161; red copies, decode.rs:284-289/245-250; per-layer RS
// encode/reconstruct, decode.rs:332-408; repair phases, repair.rs:309-416) is a
// GF-linear combination of whole sub-chunks:   dst = XOR_j coef_j * src_j.
// The planner runs the reference control flow (iscore order, u_computed
// tracking, per-layer erasure sets, RS row selection) on region NAMES instead
// of bytes, so the emitted op DAG computes exactly the reference's linear map --
// byte-identical output for any input, codeword or not.  It then removes dead
// ops and groups the rest into dependency levels (one kernel launch per level).
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <unordered_map>
#include <vector>

#include "code.hpp"

namespace clay {

enum RegionKind : uint32_t { RK_C = 0, RK_H = 1, RK_U = 2, RK_OUT = 3 };

inline uint64_t rkey(uint32_t kind, uint32_t node, uint32_t slot) {
    return (uint64_t(kind) << 56) | (uint64_t(node) << 32) | uint64_t(slot);
}
inline uint32_t rkind(uint64_t k) { return uint32_t(k >> 56); }
inline uint32_t rnode(uint64_t k) { return uint32_t((k >> 32) & 0xFFFFFF); }
inline uint32_t rslot(uint64_t k) { return uint32_t(k); }

// Device-side records (kernel reads these).
struct DevSrc {
    uint32_t base;  // pointer-table index
    uint32_t slot;  // sub-chunk index within that buffer
    uint32_t coef;  // GF(2^8) coefficient (1..255)
    uint32_t pad;
};
struct DevOp {
    uint32_t base, slot;       // destination
    uint32_t src_begin, nsrc;  // into DevSrc array
};

// Multi-destination group (one launch block = one group x one tile): every op of
// a stage that reads exactly the same source set -- the m parity/reconstruct rows
// of one layer's RS call (decode.rs:369-398), the two halves of a PRT/PFT pair
// (transforms.rs:42-125) -- is merged, so each source tile is read from HBM once
// and feeds up to kMaxGroupDst accumulators.
constexpr uint32_t kMaxGroupDst = 8;
struct DevGroup {
    uint32_t src_begin, nsrc;  // into gsrcs (coef field unused)
    uint32_t dst_begin, ndst;  // into gdsts
    uint32_t coef_begin;       // gcoef[coef_begin + d*nsrc + s]
    uint32_t pad[3];
};

struct Plan {
    // pointer table layout: [0, tn) = C[node], [tn, 2tn) = H[node], 2tn = U workspace
    // (slot = node*alpha + z), 2tn+1 = OUT.
    uint32_t tn = 0, alpha = 0;
    std::vector<DevOp> ops;           // grouped by stage
    std::vector<DevSrc> srcs;
    std::vector<uint32_t> stage_begin;  // size = stages + 1
    // grouped form of the same stages (built by group_ops(); what the device runs)
    std::vector<DevGroup> groups;
    std::vector<DevSrc> gsrcs, gdsts;
    std::vector<uint32_t> gcoef;
    std::vector<uint32_t> gstage_begin;  // size = stages + 1, into groups
    std::vector<uint32_t> gstage_maxd;   // max ndst per stage
    bool uses_u = false;
    size_t total_src_terms = 0;
    // device copies (owned by the runtime, per device)
    void *d_ops = nullptr, *d_srcs = nullptr;
    // >0: group_ops also merges groups of a stage whose source-set union adds at most
    // merge_slack sources (CLAY_PLAN_MERGE_SLACK overrides)
    int merge_slack = 0;
    void group_ops();
    int device = -1;
};

class PlanBuilder {
  public:
    struct Term {
        uint64_t key;
        int32_t ver;  // producing op index, -1 = external input
        uint8_t coef;
    };
    struct Op {
        uint64_t dst;
        int32_t prev;  // previous version of dst (-1 none)
        std::vector<Term> src;
    };

    std::vector<Op> ops;
    std::unordered_map<uint64_t, int32_t> cur;  // region -> current version
    std::vector<uint8_t> zero_c, zero_h;          // per internal node: C / H input is known zero
    // >0: also fold ops over final versions with up to fold_cost sources when the
    // consumer-layer count says it saves HBM traffic (CLAY_PLAN_FOLD_COST).  Decode,
    // encode and repair plans use 24 (profiles/r02/plan_sweep): (10,4,13) 4-erasure
    // decode 0.91 -> 0.86 ms (6 -> 5 levels), (9,3,11) staged encode 1.35 -> 1.24 ms;
    // repair (9,3,11) with merge_slack 2 becomes ONE level of 27 groups (15 helper
    // reads + 2 companions, 3 outputs each): 0.43 -> 0.33 ms.
    int fold_cost = 0;
    // copied to Plan::merge_slack by finalize()
    int merge_slack = 0;
    // >0: <= 2-source ops also substitute a still-read producer of <= dup_cost final
    // sources (CLAY_PLAN_DUP overrides); pairs with merge_slack
    int dup_cost = 0;
    // move small final-output ops to the last level (CLAY_PLAN_DEFER_OUT overrides)
    bool defer_outputs = false;

    // dst = XOR coef*src; terms on zero regions / zero coefs are dropped.
    void emit(uint64_t dst, const std::vector<std::pair<uint64_t, uint8_t>> &terms);
    std::unique_ptr<Plan> finalize(const std::vector<uint64_t> &outputs, uint32_t tn, uint32_t alpha);

  private:
    bool is_zero(uint64_t key, int32_t ver) const;
    void inline_inputs(const std::vector<uint64_t> &outputs);
};

// Per-code RS cache (generator rows + reconstruct matrices by valid-row set).
struct RsCtx {
    size_t K = 0, M = 0, T = 0;
    std::vector<uint8_t> gen;  // T x K
    int init_err = 0;
    std::unordered_map<std::string, std::vector<uint8_t>> inv_cache;
    explicit RsCtx(const clay_code_t &c);
    const std::vector<uint8_t> *inverse_for(const std::vector<size_t> &valid);
};

// encode = decode_layered with the parity nodes erased (encode.rs:57-68).
Error plan_encode(const clay_code_t &c, RsCtx &rs, std::unique_ptr<Plan> &out);
// decode.rs:152 decode_layered over the erased set; outputs = C of the erased
// internal nodes whose want_out flag is set.
Error plan_decode(const clay_code_t &c, RsCtx &rs, const std::vector<uint8_t> &erased,
                  const std::vector<uint8_t> &want_out, std::unique_ptr<Plan> &out);
// repair.rs:140-421 with the given helper set (internal ids) and index list.
Error plan_repair(const clay_code_t &c, RsCtx &rs, size_t lost, const std::vector<uint8_t> &helper_int,
                  const std::vector<long> &slot_of_id, const std::vector<size_t> &subchunks,
                  std::unique_ptr<Plan> &out, bool full_chunks = false);

}  // namespace clay
