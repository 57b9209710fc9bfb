// plan.cpp -- symbolic replay of decode_layered / repair into GF region ops.
#include "plan.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>

#include "gf256.hpp"
#include "tuning.hpp"

namespace clay {

// ---------------------------------------------------------------------------
// PlanBuilder
// ---------------------------------------------------------------------------
bool PlanBuilder::is_zero(uint64_t key, int32_t ver) const {
    if (ver >= 0) return ops[ver].src.empty();
    switch (rkind(key)) {
    case RK_C: return rnode(key) < zero_c.size() && zero_c[rnode(key)];
    case RK_H: return rnode(key) < zero_h.size() && zero_h[rnode(key)];
    default: return true;  // U / OUT never written yet: zero-initialised (decode.rs:184, repair.rs:214,220)
    }
}

void PlanBuilder::emit(uint64_t dst, const std::vector<std::pair<uint64_t, uint8_t>> &terms) {
    std::vector<Term> src;
    src.reserve(terms.size());
    for (const auto &t : terms) {
        if (t.second == 0) continue;
        auto it = cur.find(t.first);
        int32_t ver = it == cur.end() ? -1 : it->second;
        if (is_zero(t.first, ver)) continue;
        bool merged = false;
        for (auto &s : src)
            if (s.key == t.first && s.ver == ver) {
                s.coef ^= t.second;
                merged = true;
                break;
            }
        if (!merged) src.push_back(Term{t.first, ver, t.second});
    }
    src.erase(std::remove_if(src.begin(), src.end(), [](const Term &s) { return s.coef == 0; }), src.end());
    auto it = cur.find(dst);
    int32_t prev = it == cur.end() ? -1 : it->second;
    if (prev >= 0) {  // identical rewrite (e.g. repair's PRT from both sides, repair.rs:345-365)
        const auto &p = ops[prev].src;
        if (p.size() == src.size()) {
            bool same = true;
            for (const auto &s : src) {
                bool found = false;
                for (const auto &r : p)
                    if (r.key == s.key && r.ver == s.ver && r.coef == s.coef) {
                        found = true;
                        break;
                    }
                if (!found) {
                    same = false;
                    break;
                }
            }
            if (same) return;
        }
    }
    ops.push_back(Op{dst, prev, std::move(src)});
    cur[dst] = int32_t(ops.size() - 1);
}

// Forward substitution of short ops over stable inputs.  An op that is not an
// output and whose <= 2 sources are input regions nothing ever rewrites (the red
// copies U = C, decode.rs:284-289, and PRT pairs U = C + g*C*, transforms.rs:42-55,
// over available chunks / helper payloads) is folded into every consumer:
// consumer term c*dst becomes c*coef_s*src_s, equal terms merge by XOR.  The
// linear map is unchanged; the U round trip through HBM disappears and the
// consumer group reads the inputs directly.  CLAY_PLAN_INLINE=0 disables.
void PlanBuilder::inline_inputs(const std::vector<uint64_t> &outputs) {
    if (!tuning().plan_inline) return;
    const size_t n = ops.size();
    std::unordered_map<uint64_t, int> written;
    for (const auto &o : ops) written[o.dst] = 1;
    std::vector<uint8_t> is_out(n, 0), inl(n, 0);
    for (uint64_t o : outputs) {
        auto it = cur.find(o);
        if (it != cur.end() && it->second >= 0) is_out[it->second] = 1;
    }
    // readers counted per consumer layer (dst slot): the RS rows of one layer form one
    // group on the device and read a shared source once
    std::vector<std::vector<uint32_t>> rl(n);
    for (const auto &o : ops)
        for (const auto &t : o.src)
            if (t.ver >= 0 && std::find(rl[t.ver].begin(), rl[t.ver].end(), rslot(o.dst)) == rl[t.ver].end())
                rl[t.ver].push_back(rslot(o.dst));
    const GF &gf = GF::get();
    const int dup_env = tuning().plan_dup;
    const size_t dup_max = size_t(dup_env >= 0 ? dup_env : dup_cost);
    // all sources of op p are final versions (nothing rewrites them afterwards)
    auto final_srcs = [&](size_t p) {
        for (const auto &t : ops[p].src) {
            auto it = cur.find(t.key);
            if (t.ver < 0 ? written.count(t.key) != 0 : (it == cur.end() || it->second != t.ver)) return false;
        }
        return true;
    };
    for (size_t i = 0; i < n; i++) {
        // duplication (dup_max > 0): a <= 2-source output op also substitutes a producer that other
        // ops still read, when the producer's <= dup_max sources are final -- the op moves
        // to the producer's level and group_ops' merge puts it into the producer's group
        // (one extra source), instead of a separate level re-reading the materialised value
        const bool small = dup_max > 0 && is_out[i] && ops[i].src.size() <= 2;
        auto subst = [&](const Term &t) {
            return t.ver >= 0 && (inl[t.ver] || (small && ops[t.ver].src.size() <= dup_max && final_srcs(t.ver)));
        };
        bool any = false;
        for (const auto &t : ops[i].src) any |= subst(t);
        if (any) {
            std::vector<Term> nt;
            for (const auto &t : ops[i].src) {
                if (subst(t)) {
                    for (const auto &u : ops[t.ver].src) nt.push_back(Term{u.key, u.ver, gf.mul(t.coef, u.coef)});
                } else {
                    nt.push_back(t);
                }
            }
            std::vector<Term> merged;
            for (const auto &t : nt) {
                bool hit = false;
                for (auto &m : merged)
                    if (m.key == t.key && m.ver == t.ver) {
                        m.coef ^= t.coef;
                        hit = true;
                        break;
                    }
                if (!hit) merged.push_back(t);
            }
            merged.erase(std::remove_if(merged.begin(), merged.end(), [](const Term &s) { return s.coef == 0; }),
                         merged.end());
            ops[i].src = std::move(merged);
        }
        if (is_out[i]) continue;
        const size_t ns = ops[i].src.size(), r = rl[i].size();
        const int cost_env = tuning().plan_fold_cost;
        const int cost_fold = cost_env >= 0 ? cost_env : fold_cost;
        // sources: never-written inputs (any reader count), or final versions of
        // computed regions when at most 2 ops read this one (folding then never
        // adds HBM reads: 2 + 1 + r round-trip bytes vs 2r direct).
        bool inputs = true, finals = true;
        for (const auto &t : ops[i].src) {
            inputs &= t.ver < 0 && !written.count(t.key);
            auto it = cur.find(t.key);
            finals &= t.ver < 0 ? !written.count(t.key) : (it != cur.end() && it->second == t.ver);
        }
        if (ns <= 2 && (inputs || (finals && r <= 2))) inl[i] = 1;
        // traffic model: r consumer layers each re-read ns sources, against ns reads +
        // 1 write + r reads of the materialised region
        else if (cost_fold && finals && r * ns <= ns + 1 + r && ns <= size_t(cost_fold)) inl[i] = 1;
    }
}

std::unique_ptr<Plan> PlanBuilder::finalize(const std::vector<uint64_t> &outputs, uint32_t tn, uint32_t alpha) {
    inline_inputs(outputs);
    const size_t n = ops.size();
    std::vector<uint8_t> live(n, 0);
    for (uint64_t o : outputs) {
        auto it = cur.find(o);
        if (it != cur.end() && it->second >= 0) live[it->second] = 1;
    }
    for (size_t i = n; i-- > 0;) {
        if (!live[i]) continue;
        for (const auto &s : ops[i].src)
            if (s.ver >= 0) live[s.ver] = 1;
    }
    // dependency levels: RAW on sources, WAW/WAR on the destination's older live version
    std::vector<int> level(n, 0), max_reader(n, 0);
    int max_level = 0;
    for (size_t i = 0; i < n; i++) {
        if (!live[i]) continue;
        int lv = 1;
        for (const auto &s : ops[i].src)
            if (s.ver >= 0) lv = std::max(lv, level[s.ver] + 1);
        for (int32_t p = ops[i].prev; p >= 0; p = ops[p].prev)
            if (live[p]) {
                lv = std::max(lv, std::max(level[p], max_reader[p]) + 1);
                break;
            }
        level[i] = lv;
        for (const auto &s : ops[i].src)
            if (s.ver >= 0) max_reader[s.ver] = std::max(max_reader[s.ver], lv);
        max_level = std::max(max_level, lv);
    }
    // Deferred outputs (defer_outputs / CLAY_PLAN_DEFER_OUT): small ops (<= 2 sources) that
    // write a final output nothing reads, over final source versions, move from their
    // earliest level to the last one -- the tail levels fill with independent work
    // instead of idling at level boundaries.
    const int defer_env = tuning().plan_defer_out;
    if ((defer_env >= 0 ? defer_env != 0 : defer_outputs) && max_level > 2) {
        std::vector<int> nread(n, 0);
        for (size_t i = 0; i < n; i++)
            if (live[i])
                for (const auto &sv : ops[i].src)
                    if (sv.ver >= 0) nread[sv.ver]++;
        auto final_ver = [&](uint64_t key, int32_t ver) {
            auto it = cur.find(key);
            return ver < 0 ? it == cur.end() : (it != cur.end() && it->second == ver);
        };
        for (size_t i = 0; i < n; i++) {
            if (!live[i] || nread[i] || rkind(ops[i].dst) == RK_U || ops[i].src.size() > 2) continue;
            if (!final_ver(ops[i].dst, int32_t(i))) continue;
            bool ok = true;
            for (const auto &sv : ops[i].src) ok &= final_ver(sv.key, sv.ver);
            if (ok) level[i] = max_level;
        }
    }
    auto plan = std::make_unique<Plan>();
    plan->tn = tn;
    plan->alpha = alpha;
    auto base_of = [&](uint64_t key, uint32_t *slot) -> uint32_t {
        uint32_t node = rnode(key);
        *slot = rslot(key);
        switch (rkind(key)) {
        case RK_C: return node;
        case RK_H: return tn + node;
        case RK_U:
            plan->uses_u = true;
            *slot = node * alpha + rslot(key);
            return 2 * tn;
        default: return 2 * tn + 1;
        }
    };
    plan->stage_begin.push_back(0);
    for (int lv = 1; lv <= max_level; lv++) {
        for (size_t i = 0; i < n; i++) {
            if (!live[i] || level[i] != lv) continue;
            DevOp d{};
            d.base = base_of(ops[i].dst, &d.slot);
            d.src_begin = uint32_t(plan->srcs.size());
            d.nsrc = uint32_t(ops[i].src.size());
            for (const auto &s : ops[i].src) {
                DevSrc ds{};
                ds.base = base_of(s.key, &ds.slot);
                ds.coef = s.coef;
                plan->srcs.push_back(ds);
            }
            plan->total_src_terms += d.nsrc;
            plan->ops.push_back(d);
        }
        plan->stage_begin.push_back(uint32_t(plan->ops.size()));
    }
    plan->merge_slack = merge_slack;
    plan->group_ops();
    return plan;
}

// Merge the ops of each stage that read the same (base, slot) source set.  Ops of
// one stage never read each other's destinations (levels above), so a group may
// read all of its sources before writing any destination.
void Plan::group_ops() {
    groups.clear(); gsrcs.clear(); gdsts.clear(); gcoef.clear(); gstage_begin.assign(1, 0); gstage_maxd.clear();
    struct G {
        std::vector<std::pair<uint32_t, uint32_t>> src;  // sorted (base, slot)
        std::vector<DevSrc> dst;
        std::vector<std::vector<uint32_t>> coef;          // per dst, aligned with src
    };
    for (size_t s = 0; s + 1 < stage_begin.size(); s++) {
        std::vector<G> gs;
        std::map<std::vector<std::pair<uint32_t, uint32_t>>, size_t> open;
        for (uint32_t i = stage_begin[s]; i < stage_begin[s + 1]; i++) {
            const DevOp &op = ops[i];
            std::vector<std::pair<std::pair<uint32_t, uint32_t>, uint32_t>> t;
            for (uint32_t j = 0; j < op.nsrc; j++) {
                const DevSrc &d = srcs[op.src_begin + j];
                t.push_back({{d.base, d.slot}, d.coef});
            }
            std::sort(t.begin(), t.end());
            bool dup = false;  // a repeated source term stays a single-op group (coefs not merged)
            for (size_t j = 1; j < t.size(); j++) dup |= t[j].first == t[j - 1].first;
            std::vector<std::pair<uint32_t, uint32_t>> key;
            for (auto &x : t) key.push_back(x.first);
            size_t gi;
            auto it = dup || key.empty() ? open.end() : open.find(key);
            if (it != open.end() && gs[it->second].dst.size() < kMaxGroupDst) {
                gi = it->second;
            } else {
                gi = gs.size();
                gs.push_back(G{key, {}, {}});
                if (!dup && !key.empty()) open[key] = gi;
            }
            DevSrc dd{};
            dd.base = op.base;
            dd.slot = op.slot;
            gs[gi].dst.push_back(dd);
            std::vector<uint32_t> cf;
            for (auto &x : t) cf.push_back(x.second);
            gs[gi].coef.push_back(cf);
        }
        // Near-identical source sets (merge_slack > 0): fold group b into group a when the
        // union adds at most merge_slack sources to the larger set, so e.g. repair's three
        // folded outputs of one layer (15 shared helper reads + one own companion each)
        // share one source pass; the merged coefficient rows hold 0 for absent sources.
        const int slack_env = tuning().plan_merge_slack;
        const size_t slack = size_t(slack_env >= 0 ? slack_env : merge_slack);
        if (slack > 0 && gs.size() > 1) {
            std::vector<uint8_t> gone(gs.size(), 0);
            // a group whose source list repeats a region (two versions of one slot) keeps
            // its own rows: re-aligning by region would fold the two coefficients together
            auto has_rep = [](const G &x) {
                for (size_t j = 1; j < x.src.size(); j++)
                    if (x.src[j] == x.src[j - 1]) return true;
                return false;
            };
            for (size_t a = 0; a < gs.size(); a++) {
                if (gone[a] || gs[a].src.empty() || has_rep(gs[a])) continue;
                for (size_t b = a + 1; b < gs.size(); b++) {
                    if (gone[b] || gs[b].src.empty() || gs[a].dst.size() + gs[b].dst.size() > kMaxGroupDst ||
                        has_rep(gs[b]))
                        continue;
                    std::vector<std::pair<uint32_t, uint32_t>> u;
                    std::set_union(gs[a].src.begin(), gs[a].src.end(), gs[b].src.begin(), gs[b].src.end(),
                                   std::back_inserter(u));
                    if (u.size() > std::max(gs[a].src.size(), gs[b].src.size()) + slack) continue;
                    // re-align both groups' coefficient rows to the union
                    G m{u, {}, {}};
                    for (G *x : {&gs[a], &gs[b]})
                        for (size_t d = 0; d < x->dst.size(); d++) {
                            std::vector<uint32_t> row(u.size(), 0);
                            for (size_t j = 0; j < x->src.size(); j++)
                                row[size_t(std::lower_bound(u.begin(), u.end(), x->src[j]) - u.begin())] = x->coef[d][j];
                            m.dst.push_back(x->dst[d]);
                            m.coef.push_back(row);
                        }
                    gs[a] = std::move(m);
                    gone[b] = 1;
                }
            }
            std::vector<G> kept;
            for (size_t a = 0; a < gs.size(); a++)
                if (!gone[a]) kept.push_back(std::move(gs[a]));
            gs = std::move(kept);
        }
        if (tuning().plan_debug) {
            size_t nsrc = 0, ndst = 0;
            std::map<size_t, size_t> hist;
            for (auto &g : gs) {
                nsrc += g.src.size();
                ndst += g.dst.size();
                hist[g.dst.size()]++;
            }
            fprintf(stderr, "stage %zu: groups %zu src reads %zu dst writes %zu | dst-count histogram:", s, gs.size(), nsrc,
                    ndst);
            for (auto &h : hist) fprintf(stderr, " %zu:%zu", h.first, h.second);
            fprintf(stderr, "\n");
        }
        uint32_t maxd = 1;
        for (auto &g : gs) {
            DevGroup dg{};
            dg.src_begin = uint32_t(gsrcs.size());
            dg.nsrc = uint32_t(g.src.size());
            dg.dst_begin = uint32_t(gdsts.size());
            dg.ndst = uint32_t(g.dst.size());
            dg.coef_begin = uint32_t(gcoef.size());
            for (auto &x : g.src) {
                DevSrc d{};
                d.base = x.first;
                d.slot = x.second;
                gsrcs.push_back(d);
            }
            for (auto &d : g.dst) gdsts.push_back(d);
            for (auto &cf : g.coef) gcoef.insert(gcoef.end(), cf.begin(), cf.end());
            maxd = std::max(maxd, dg.ndst);
            groups.push_back(dg);
        }
        gstage_begin.push_back(uint32_t(groups.size()));
        gstage_maxd.push_back(maxd);
    }
}

// ---------------------------------------------------------------------------
// RS context (reed-solomon-erasure ReedSolomon::new + reconstruct matrices)
// ---------------------------------------------------------------------------
RsCtx::RsCtx(const clay_code_t &c) {
    K = c.original_count;
    M = c.recovery_count;
    T = K + M;
    init_err = rs_generator(K, M, gen);
}

const std::vector<uint8_t> *RsCtx::inverse_for(const std::vector<size_t> &valid) {
    std::string key;
    key.reserve(valid.size() * 2);
    for (size_t v : valid) {
        key.push_back(char(v & 0xFF));
        key.push_back(char(v >> 8));
    }
    auto it = inv_cache.find(key);
    if (it != inv_cache.end()) return &it->second;
    std::vector<uint8_t> sub(K * K), inv;
    for (size_t r = 0; r < K; r++)
        for (size_t c = 0; c < K; c++) sub[r * K + c] = gen[valid[r] * K + c];
    if (!gf_invert(sub, K, inv)) return nullptr;
    return &(inv_cache[key] = std::move(inv));
}

// decode.rs:332-408 decode_uncoupled_layer, symbolically.  `uk(node)` names the
// U region of `node` at this layer.
template <class UK>
static Error uncoupled_layer(const clay_code_t &c, RsCtx &rs, PlanBuilder &b, const std::vector<uint8_t> &er,
                             size_t z, UK uk) {
    const size_t tn = c.q * c.t, K = c.original_count;
    size_t ne = 0;
    bool has_orig = false, has_par = false;
    for (size_t i = 0; i < tn; i++)
        if (er[i]) {
            ne++;
            (i < K ? has_orig : has_par) = true;
        }
    if (ne > c.m)
        return make_error(CLAY_ERR_TOO_MANY_ERASURES, c.m, ne, 0, "Too many erasures: max %zu supported, got %zu", c.m,
                          ne);
    if (ne == 0) return Error{};
    const GF &g = GF::get();
    std::vector<std::pair<uint64_t, uint8_t>> terms;
    if (has_orig) {
        // ReedSolomon::reconstruct: first K present shards in index order
        std::vector<size_t> valid;
        for (size_t i = 0; i < tn && valid.size() < K; i++)
            if (!er[i]) valid.push_back(i);
        if (valid.size() < K)
            return make_error(CLAY_ERR_RECONSTRUCTION_FAILED, 0, 0, 0,
                              "RS reconstruction failed: Layer %zu RS reconstruct failed: TooFewShardsPresent", z);
        const std::vector<uint8_t> *inv = rs.inverse_for(valid);
        if (!inv)
            return make_error(CLAY_ERR_RECONSTRUCTION_FAILED, 0, 0, 0,
                              "RS reconstruction failed: Layer %zu RS reconstruct failed: SingularMatrix", z);
        for (size_t i = 0; i < K; i++) {
            if (!er[i]) continue;
            terms.clear();
            for (size_t j = 0; j < K; j++) terms.push_back({uk(valid[j]), (*inv)[i * K + j]});
            b.emit(uk(i), terms);
        }
        // missing parity re-encoded from all (present + rebuilt) data shards,
        // composed onto the valid shards
        for (size_t p = K; p < tn; p++) {
            if (!er[p]) continue;
            std::vector<uint8_t> coef(K, 0);
            for (size_t col = 0; col < K; col++) {
                uint8_t gpc = rs.gen[p * K + col];
                if (!gpc) continue;
                if (!er[col]) {
                    size_t j = size_t(std::find(valid.begin(), valid.end(), col) - valid.begin());
                    coef[j] ^= gpc;
                } else {
                    for (size_t j = 0; j < K; j++) coef[j] ^= g.mul(gpc, (*inv)[col * K + j]);
                }
            }
            terms.clear();
            for (size_t j = 0; j < K; j++) terms.push_back({uk(valid[j]), coef[j]});
            b.emit(uk(p), terms);
        }
    } else if (has_par) {  // ReedSolomon::encode, copy back erased parities
        for (size_t p = K; p < tn; p++) {
            if (!er[p]) continue;
            terms.clear();
            for (size_t col = 0; col < K; col++) terms.push_back({uk(col), rs.gen[p * K + col]});
            b.emit(uk(p), terms);
        }
    }
    return Error{};
}

// decode.rs:167-257 decode_layered (+ :260-329 with_tracking, :438-528 helpers)
static Error replay_layered(const clay_code_t &c, RsCtx &rs, PlanBuilder &b, const std::vector<uint8_t> &er) {
    if (rs.init_err)
        return make_error(CLAY_ERR_RECONSTRUCTION_FAILED, 0, 0, 0, "RS reconstruction failed: RS init failed: %s",
                          rs_error_name(rs.init_err));
    const size_t q = c.q, t = c.t, tn = q * t, alpha = c.sub_chunk_no;
    const uint8_t g1 = 1, gm = kGamma, det = gamma_det(), dinv = gamma_det_inv();
    const uint8_t dinv_g = GF::get().mul(dinv, kGamma);
    auto C = [](size_t node, size_t z) { return rkey(RK_C, uint32_t(node), uint32_t(z)); };
    auto U = [](size_t node, size_t z) { return rkey(RK_U, uint32_t(node), uint32_t(z)); };
    std::vector<uint8_t> ucomp(tn * alpha, 0);
    std::vector<size_t> order(alpha, 0), zv(t);
    for (size_t z = 0; z < alpha; z++) {  // decode.rs:531-545
        plane_vector(c, z, zv.data());
        for (size_t i = 0; i < tn; i++)
            if (er[i] && i % q == zv[i / q]) order[z]++;
    }
    size_t max_is = 0;  // decode.rs:548-561
    {
        std::vector<uint8_t> seen(t, 0);
        for (size_t i = 0; i < tn; i++)
            if (er[i] && !seen[i / q]) {
                seen[i / q] = 1;
                max_is++;
            }
    }
    for (size_t is = 0; is <= max_is; is++) {
        for (size_t z = 0; z < alpha; z++) {
            if (order[z] != is) continue;
            plane_vector(c, z, zv.data());
            std::vector<uint8_t> needs(er);
            for (size_t x = 0; x < q; x++)
                for (size_t y = 0; y < t; y++) {
                    size_t nxy = q * y + x, z_y = zv[y], nsw = q * y + z_y;
                    size_t z_sw = companion_layer(c, z, x, y, z_y);
                    if (er[nxy]) continue;
                    if (z_y == x) {
                        b.emit(U(nxy, z), {{C(nxy, z), g1}});
                        ucomp[nxy * alpha + z] = 1;
                    } else if (!er[nsw]) {
                        if (z_y < x) {  // PRT, symmetric in orientation (transforms.rs:42-55)
                            b.emit(U(nxy, z), {{C(nxy, z), g1}, {C(nsw, z_sw), gm}});
                            b.emit(U(nsw, z_sw), {{C(nxy, z), gm}, {C(nsw, z_sw), g1}});
                            ucomp[nxy * alpha + z] = 1;
                            ucomp[nsw * alpha + z_sw] = 1;
                        }
                    } else if (ucomp[nsw * alpha + z_sw]) {  // U = det*C + g*U* (transforms.rs:149-161)
                        b.emit(U(nxy, z), {{C(nxy, z), det}, {U(nsw, z_sw), gm}});
                        ucomp[nxy * alpha + z] = 1;
                    } else {
                        needs[nxy] = 1;
                    }
                }
            Error e = uncoupled_layer(c, rs, b, needs, z, [&](size_t node) { return U(node, z); });
            if (e) return e;
            for (size_t i = 0; i < tn; i++)
                if (needs[i]) ucomp[i * alpha + z] = 1;
        }
        for (size_t z = 0; z < alpha; z++) {
            if (order[z] != is) continue;
            plane_vector(c, z, zv.data());
            for (size_t nxy = 0; nxy < tn; nxy++) {
                if (!er[nxy]) continue;
                size_t x = nxy % q, y = nxy / q, z_y = zv[y], nsw = y * q + z_y;
                size_t z_sw = companion_layer(c, z, x, y, z_y);
                if (z_y != x) {
                    if (!er[nsw]) {  // type 1: C = U + g*C* (transforms.rs:132-142)
                        b.emit(C(nxy, z), {{U(nxy, z), g1}, {C(nsw, z_sw), gm}});
                    } else if (z_y < x) {  // PFT (transforms.rs:108-125)
                        b.emit(C(nxy, z), {{U(nxy, z), dinv}, {U(nsw, z_sw), dinv_g}});
                        b.emit(C(nsw, z_sw), {{U(nxy, z), dinv_g}, {U(nsw, z_sw), dinv}});
                    }
                } else {
                    b.emit(C(nxy, z), {{U(nxy, z), g1}});
                }
            }
        }
    }
    return Error{};
}

static void init_zero_inputs(const clay_code_t &c, PlanBuilder &b) {
    const size_t tn = c.q * c.t;
    b.zero_c.assign(tn, 0);
    b.zero_h.assign(tn, 0);
    for (size_t i = c.k; i < c.k + c.nu; i++) b.zero_c[i] = b.zero_h[i] = 1;
}

Error plan_encode(const clay_code_t &c, RsCtx &rs, std::unique_ptr<Plan> &out) {
    const size_t tn = c.q * c.t;
    std::vector<uint8_t> er(tn, 0), want(tn, 0);
    for (size_t i = c.k + c.nu; i < tn; i++) er[i] = want[i] = 1;
    return plan_decode(c, rs, er, want, out);
}

Error plan_decode(const clay_code_t &c, RsCtx &rs, const std::vector<uint8_t> &er, const std::vector<uint8_t> &want,
                  std::unique_ptr<Plan> &out) {
    PlanBuilder b;
    b.fold_cost = 24;
    init_zero_inputs(c, b);
    Error e = replay_layered(c, rs, b, er);
    if (e) return e;
    std::vector<uint64_t> outs;
    for (size_t i = 0; i < er.size(); i++)
        if (er[i] && want[i])
            for (size_t z = 0; z < c.sub_chunk_no; z++) outs.push_back(rkey(RK_C, uint32_t(i), uint32_t(z)));
    out = b.finalize(outs, uint32_t(c.q * c.t), uint32_t(c.sub_chunk_no));
    return Error{};
}

// repair.rs:140-421
Error plan_repair(const clay_code_t &c, RsCtx &rs, size_t lost, const std::vector<uint8_t> &hin,
                  const std::vector<long> &slot_of_id, const std::vector<size_t> &ridx, std::unique_ptr<Plan> &out,
                  bool full_chunks) {
    (void)slot_of_id;
    if (rs.init_err)
        return make_error(CLAY_ERR_RECONSTRUCTION_FAILED, 0, 0, 0, "RS reconstruction failed: RS init failed: %s",
                          rs_error_name(rs.init_err));
    const size_t q = c.q, t = c.t, tn = q * t, alpha = c.sub_chunk_no;
    const size_t li = internal_of(c, lost), lost_y = li / q;
    const uint8_t g1 = 1, gm = kGamma, det = gamma_det(), ginv = gamma_inv();
    PlanBuilder b;
    b.fold_cost = 24;
    b.merge_slack = 2;
    init_zero_inputs(c, b);
    // helper_internal: real helpers + shortened nodes as zero helpers (repair.rs:258-261)
    std::vector<uint8_t> helper(tn, 0), aloof(tn, 0), base(tn, 0);
    for (size_t i = 0; i < tn; i++) helper[i] = hin[i] || is_shortened(c, i);
    for (size_t i = 0; i < tn; i++)  // repair.rs:248-255
        if (i != li && !hin[i] && !is_shortened(c, i)) aloof[i] = 1;
    std::vector<long> pind(alpha, -1);
    for (size_t i = 0; i < ridx.size(); i++) pind[ridx[i]] = long(i);
    // helper payload slot: position in the beta-sub-chunk list (repair.rs:225-240), or
    // layer z itself when the helpers are whole chunks (device-side gather)
    auto H = [&](size_t node, size_t z) {
        return rkey(RK_H, uint32_t(node), uint32_t(full_chunks ? long(z) : pind[z]));
    };
    auto U = [](size_t node, size_t z) { return rkey(RK_U, uint32_t(node), uint32_t(z)); };
    auto OUT = [](size_t z) { return rkey(RK_OUT, 0, uint32_t(z)); };
    std::vector<size_t> zv(t), ord(ridx.size());
    size_t max_ord = 0;
    for (size_t i = 0; i < ridx.size(); i++) {  // repair.rs:270-288
        plane_vector(c, ridx[i], zv.data());
        size_t o = (li % q == zv[li / q]) ? 1 : 0;
        for (size_t nd = 0; nd < tn; nd++)
            if (aloof[nd] && nd % q == zv[nd / q]) o++;
        ord[i] = o;
        max_ord = std::max(max_ord, o);
    }
    for (size_t x = 0; x < q; x++) base[lost_y * q + x] = 1;  // repair.rs:291-297
    for (size_t i = 0; i < tn; i++)
        if (aloof[i]) base[i] = 1;
    std::vector<uint8_t> ucomp(tn * alpha, 0);
    for (size_t o = 0; o <= max_ord; o++)
        for (size_t pi = 0; pi < ridx.size(); pi++) {
            if (ord[pi] != o) continue;
            size_t z = ridx[pi];
            plane_vector(c, z, zv.data());
            std::vector<uint8_t> le(base);
            for (size_t y = 0; y < t; y++)  // Phase 1
                for (size_t x = 0; x < q; x++) {
                    size_t nxy = y * q + x;
                    if (base[nxy]) continue;
                    if (!helper[nxy]) {
                        le[nxy] = 1;
                        continue;
                    }
                    size_t z_y = zv[y], z_sw = companion_layer(c, z, x, y, z_y), nsw = y * q + z_y;
                    if (z_y == x) {
                        b.emit(U(nxy, z), {{H(nxy, z), g1}});
                        ucomp[nxy * alpha + z] = 1;
                    } else if (aloof[nsw]) {
                        if (ucomp[nsw * alpha + z_sw]) {
                            b.emit(U(nxy, z), {{H(nxy, z), det}, {U(nsw, z_sw), gm}});
                            ucomp[nxy * alpha + z] = 1;
                        } else {
                            le[nxy] = 1;
                        }
                    } else if (helper[nsw]) {
                        if (pind[z_sw] >= 0) {  // prt_compute_both_oriented, symmetric
                            b.emit(U(nxy, z), {{H(nxy, z), g1}, {H(nsw, z_sw), gm}});
                            b.emit(U(nsw, z_sw), {{H(nxy, z), gm}, {H(nsw, z_sw), g1}});
                            ucomp[nxy * alpha + z] = 1;
                            ucomp[nsw * alpha + z_sw] = 1;
                        }
                    } else {
                        le[nxy] = 1;
                    }
                }
            Error e = uncoupled_layer(c, rs, b, le, z, [&](size_t node) { return U(node, z); });  // Phase 2
            if (e) return e;
            for (size_t i = 0; i < tn; i++)
                if (le[i]) ucomp[i * alpha + z] = 1;
            for (size_t nd = 0; nd < tn; nd++) {  // Phase 3
                if (!base[nd] || aloof[nd]) continue;
                size_t x = nd % q, y = nd / q, z_y = zv[y], nsw = y * q + z_y;
                size_t z_sw = companion_layer(c, z, x, y, z_y);
                if (x == z_y) {
                    if (nd == li) b.emit(OUT(z), {{U(nd, z), g1}});
                } else if (nsw == li && helper[nd]) {  // C* = (U + C)/g (decode.rs:566-576)
                    b.emit(OUT(z_sw), {{U(nd, z), ginv}, {H(nd, z), ginv}});
                }
            }
        }
    std::vector<uint64_t> outs;
    for (size_t z = 0; z < alpha; z++) outs.push_back(OUT(z));
    // Every OUT slot is written by the replay; an unwritten slot would stay zero (repair.rs:220).
    for (size_t z = 0; z < alpha; z++)
        if (!b.cur.count(OUT(z))) b.emit(OUT(z), {});
    out = b.finalize(outs, uint32_t(tn), uint32_t(alpha));
    return Error{};
}

}  // namespace clay
