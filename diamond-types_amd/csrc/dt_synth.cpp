// dt_synth.cpp -- deterministic synthetic concurrent documents (BASELINE.json configs[3]: "1M
// synthetic concurrent docs, 4-16 agents, ~5k ops each"), modelled on the reference's fuzzers
// (make_random_change, src/list_fuzzer_tools.rs:38-104; merge_fuzz, src/listmerge/fuzzer.rs:34-129).
// Two families: dtgpu_synth_merge_oplog, the SURVEY.md 8(d)4 generator (per-step pairwise
// merges, partially merged graphs; MergeGen below), the configs[3] workload; and the epoch
// generator (dtgpu_synth_oplog):
//
//   * seed = 0xD1A0_0000 + doc index, xoshiro256** (seeded through splitmix64);
//   * k ~ U{4..16} agents named "a0".."a15";
//   * the history is a sequence of epochs (20..200 edits): every agent edits its own branch
//     from the epoch's common version, the edits of different agents interleave in LV order
//     (so the agents' branches are concurrent), and the epoch ends with every branch merged;
//   * an edit inserts with p = 0.55 (0.45 once the branch holds >= 100 chars) 1-2 chars of
//     a-z at a uniform position -- a 2-char insert is typed backwards (two 1-char prepends)
//     with p = 0.5 -- or deletes a span of 1..10 chars, as backspaces (one char at a time,
//     right to left) with p = 0.5.
//
// Positions are computed from each agent's own branch; the merged length at an epoch end
// needs no CRDT (base chars deleted by anyone go, surviving own inserts stay), so the
// generator is independent of the engine it feeds.
#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/dtgpu.h"

namespace {

struct Rng {   // xoshiro256**
    uint64_t s[4];
    static uint64_t splitmix(uint64_t &x) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    explicit Rng(uint64_t seed) { for (auto &v : s) v = splitmix(seed); }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
    bool chance(double p) { return double(next() >> 11) * (1.0 / 9007199254740992.0) < p; }
};

// Op record: agent, kind (0 ins, 1 del), pos, len, text (<= 2 ASCII bytes), parents.
struct Op {
    uint32_t agent, kind;
    uint64_t pos, len;
    char text[2];
    std::vector<uint64_t> parents;
};

void generate(uint64_t doc, uint32_t target, uint32_t &n_agents, std::vector<Op> &ops) {
    Rng rng(0xD1A00000ull + doc);
    n_agents = 4 + uint32_t(rng.below(13));
    ops.clear();
    uint64_t base_len = 0, lv = 0;
    std::vector<uint64_t> frontier;   // the epoch's common version
    while (lv < target) {
        const uint32_t steps = 20 + uint32_t(rng.below(181));
        // per agent branch: char identities (>= 0: base char index, < 0: own insert)
        std::vector<std::vector<int64_t>> br(n_agents);
        std::vector<int64_t> head(n_agents, -1);   // last LV of the agent in this epoch
        std::vector<std::vector<uint8_t>> base_del(n_agents, std::vector<uint8_t>(base_len, 0));
        for (auto &b : br) { b.resize(base_len); for (uint64_t i = 0; i < base_len; i++) b[i] = int64_t(i); }
        int64_t own = -1;
        for (uint32_t st = 0; st < steps && lv < target; st++) {
            const uint32_t a = uint32_t(rng.below(n_agents));
            auto &b = br[a];
            auto parents = [&]() {
                return head[a] >= 0 ? std::vector<uint64_t>{uint64_t(head[a])} : frontier;
            };
            const uint64_t len = b.size();
            const bool ins = len == 0 || rng.chance(len < 100 ? 0.55 : 0.45);
            if (ins) {
                const uint32_t n = 1 + uint32_t(rng.below(2));
                const uint64_t pos = rng.below(len + 1);
                char t[2] = {char('a' + rng.below(26)), char('a' + rng.below(26))};
                if (n == 2 && rng.chance(0.5)) {   // typed backwards: two prepends at pos
                    for (uint32_t j = 0; j < 2; j++) {
                        Op o{a, 0, pos, 1, {t[j], 0}, parents()};
                        ops.push_back(o);
                        head[a] = int64_t(lv++);
                        b.insert(b.begin() + int64_t(pos), own--);
                    }
                } else {
                    Op o{a, 0, pos, n, {t[0], t[1]}, parents()};
                    ops.push_back(o);
                    lv += n;
                    head[a] = int64_t(lv - 1);
                    for (uint32_t j = 0; j < n; j++) b.insert(b.begin() + int64_t(pos + j), own--);
                }
            } else {
                const uint64_t pos = rng.below(len);
                const uint64_t span = 1 + rng.below(std::min<uint64_t>(10, len - pos));
                auto erase = [&](uint64_t p) {
                    if (b[p] >= 0) base_del[a][size_t(b[p])] = 1;
                    b.erase(b.begin() + int64_t(p));
                };
                if (span > 1 && rng.chance(0.5)) {   // backspaces, right to left
                    for (uint64_t j = 0; j < span; j++) {
                        Op o{a, 1, pos + span - 1 - j, 1, {0, 0}, parents()};
                        ops.push_back(o);
                        head[a] = int64_t(lv++);
                        erase(pos + span - 1 - j);
                    }
                } else {
                    Op o{a, 1, pos, span, {0, 0}, parents()};
                    ops.push_back(o);
                    lv += span;
                    head[a] = int64_t(lv - 1);
                    for (uint64_t j = 0; j < span; j++) erase(pos);
                }
            }
        }
        // merge every branch: base chars nobody deleted + every agent's surviving inserts
        uint64_t nl = 0;
        for (uint64_t i = 0; i < base_len; i++) {
            bool gone = false;
            for (uint32_t a = 0; a < n_agents && !gone; a++) gone = base_del[a][i];
            nl += !gone;
        }
        std::vector<uint64_t> nf;
        for (uint32_t a = 0; a < n_agents; a++) {
            for (int64_t id : br[a]) nl += id < 0;
            if (head[a] >= 0) nf.push_back(uint64_t(head[a]));
        }
        if (!nf.empty()) {
            std::sort(nf.begin(), nf.end());
            frontier = nf;
        }
        base_len = nl;
    }
}

// ---- SURVEY.md 8(d)4 generator: per-step pairwise merges ----------------------------------
//
//   * seed = 0xD1A0_0000 + doc index, xoshiro256**; k ~ U{4..16} agents "a0".."a15" (or a
//     given k: the wide variant with more concurrent chains than the device prep handles);
//   * until LVs >= target, every step: pick an agent uniformly; with p = 0.1 merge another
//     agent's frontier into it (Graph::find_dominators_2, tools.rs:545-578); then one edit of
//     make_random_change (src/list_fuzzer_tools.rs:38-104): insert with p = 0.55 (0.45 once the
//     branch holds >= 100 chars) 1-2 chars of a-z at a uniform position, a 2-char insert typed
//     backwards (two 1-char prepends) with p = 0.5; otherwise delete a span of
//     U{1..min(10, len - pos)} chars, as backspaces with p = 0.5.
//
// Positions come from the editing agent's branch text.  The generator keeps every item in one
// global document order (each insert integrated by the YjsMod rules of merge.rs:154-278
// against the editing agent's history -- the state an LV-order replay reaches), so a branch's
// text is the global order filtered by that branch's history: items it inserted and did not
// delete.  Workload generation only; the checkout of the result is the engine's job and the
// tests check it against the oracle.
struct MergeGen {
    Rng rng;
    uint32_t k;
    std::vector<std::string> names;
    std::vector<uint32_t> rank;                     // byte-wise name order
    std::vector<std::vector<uint64_t>> hist;        // per agent: LV bitset of its history
    std::vector<std::vector<uint64_t>> front;       // per agent: frontier (ascending)
    std::vector<uint64_t> seq;                      // per agent: next seq
    // per LV
    std::vector<uint32_t> lv_agent, lv_seq;
    std::vector<int64_t> ol, orr;                   // inserts: origins (-1 ROOT / END)
    std::vector<std::vector<uint32_t>> deleters;    // inserts: LVs that deleted the item
    std::vector<uint32_t> order;                    // global document order of inserted LVs
    std::vector<uint32_t> gidx;                     // per inserted LV: index in `order`
    uint64_t n_lv = 0;

    MergeGen(uint64_t doc, uint32_t agents) : rng(0xD1A00000ull + doc) {
        k = 4 + uint32_t(rng.below(13));
        if (agents) k = agents;
        for (uint32_t a = 0; a < k; a++) names.push_back("a" + std::to_string(a));
        std::vector<uint32_t> ids(k);
        for (uint32_t a = 0; a < k; a++) ids[a] = a;
        std::sort(ids.begin(), ids.end(), [&](uint32_t x, uint32_t y) { return names[x] < names[y]; });
        rank.assign(k, 0);
        for (uint32_t r = 0; r < k; r++) rank[ids[r]] = r;
        hist.assign(k, {});
        front.assign(k, {});
        seq.assign(k, 0);
    }
    bool in_hist(uint32_t a, uint64_t lv) const {
        const auto &h = hist[a];
        return (lv >> 6) < h.size() && ((h[lv >> 6] >> (lv & 63)) & 1ull);
    }
    void set_hist(uint32_t a, uint64_t lv) {
        auto &h = hist[a];
        if ((lv >> 6) >= h.size()) h.resize((lv >> 6) + 1, 0);
        h[lv >> 6] |= 1ull << (lv & 63);
    }
    bool visible(uint32_t a, uint32_t item) const {
        if (!in_hist(a, item)) return false;
        for (uint32_t d : deleters[item]) if (in_hist(a, d)) return false;
        return true;
    }
    std::vector<uint32_t> view(uint32_t a) const {
        std::vector<uint32_t> v;
        for (uint32_t x : order) if (visible(a, x)) v.push_back(x);
        return v;
    }
    uint64_t new_lv(uint32_t a) {
        const uint64_t lv = n_lv++;
        lv_agent.push_back(a);
        lv_seq.push_back(uint32_t(seq[a]++));
        ol.push_back(-1); orr.push_back(-1);
        deleters.emplace_back();
        gidx.push_back(0xFFFFFFFFu);
        return lv;
    }
    void advance(uint32_t a, uint64_t lv) {   // the agent's frontier moves to its new LV
        set_hist(a, lv);
        front[a].assign(1, lv);
    }
    int64_t pos_after(int64_t x) const { return x < 0 ? 0 : int64_t(gidx[size_t(x)]) + 1; }
    int64_t pos_right(int64_t x) const { return x < 0 ? int64_t(order.size()) : int64_t(gidx[size_t(x)]); }
    // insert one char: the item after visible index p - 1 of agent a's branch
    void insert_char(uint32_t a, const std::vector<uint32_t> &v, uint64_t p, uint64_t lv) {
        const int64_t left = p ? int64_t(v[p - 1]) : -1;
        const size_t cur = size_t(pos_after(left));
        size_t r = cur;
        while (r < order.size() && !in_hist(a, order[r])) r++;   // origin_right: first non-NIY
        const int64_t right = r < order.size() ? int64_t(order[r]) : -1;
        size_t at = cur;
        if (r > cur) {   // YjsMod integrate over the concurrent (NIY) items, merge.rs:154-278
            const int64_t my_l = pos_after(left) - 1, my_r = pos_right(right);
            bool scanning = false;
            size_t start = cur, c = cur;
            for (; c < order.size(); c++) {
                const uint32_t o = order[c];
                if (int64_t(o) == right) break;
                const int64_t l2 = pos_after(ol[o]) - 1;
                if (l2 < my_l) break;
                if (l2 == my_l) {
                    if (orr[o] == right) {
                        const uint32_t ra = rank[a], rb = rank[lv_agent[o]];
                        if (ra < rb || (ra == rb && lv_seq[lv] < lv_seq[o])) break;
                        scanning = false;
                    } else if (pos_right(orr[o]) < my_r) {
                        if (!scanning) { scanning = true; start = c; }
                    } else {
                        scanning = false;
                    }
                }
            }
            at = scanning ? start : c;
        }
        ol[lv] = left;
        orr[lv] = right;
        order.insert(order.begin() + int64_t(at), uint32_t(lv));
        for (size_t i = at; i < order.size(); i++) gidx[order[i]] = uint32_t(i);
    }
    void merge_into(uint32_t a, uint32_t b) {   // a's version := find_dominators_2(a, b)
        std::vector<uint64_t> f;
        for (uint64_t x : front[a])
            if (!(in_hist(b, x) && !std::binary_search(front[b].begin(), front[b].end(), x))) f.push_back(x);
        for (uint64_t y : front[b])
            if (!(in_hist(a, y) && !std::binary_search(front[a].begin(), front[a].end(), y))) f.push_back(y);
        std::sort(f.begin(), f.end());
        f.erase(std::unique(f.begin(), f.end()), f.end());
        auto &ha = hist[a];
        const auto &hb = hist[b];
        if (hb.size() > ha.size()) ha.resize(hb.size(), 0);
        for (size_t i = 0; i < hb.size(); i++) ha[i] |= hb[i];
        front[a] = f;
    }
    void run(uint32_t target, std::vector<Op> &ops) {
        ops.clear();
        while (n_lv < target) {
            const uint32_t a = uint32_t(rng.below(k));
            if (k > 1 && rng.chance(0.1)) {
                uint32_t b = uint32_t(rng.below(k - 1));
                if (b >= a) b++;
                merge_into(a, b);
            }
            const std::vector<uint32_t> v = view(a);
            const uint64_t len = v.size();
            if (len == 0 || rng.chance(len < 100 ? 0.55 : 0.45)) {
                const uint32_t n = 1 + uint32_t(rng.below(2));
                const uint64_t pos = rng.below(len + 1);
                const char t[2] = {char('a' + rng.below(26)), char('a' + rng.below(26))};
                if (n == 2 && rng.chance(0.5)) {   // typed backwards: two prepends at pos
                    for (uint32_t j = 0; j < 2; j++) {
                        ops.push_back(Op{a, 0, pos, 1, {t[j], 0}, front[a]});
                        const uint64_t lv = new_lv(a);
                        const std::vector<uint32_t> vv = j ? view(a) : v;
                        insert_char(a, vv, pos, lv);
                        advance(a, lv);
                    }
                } else {
                    ops.push_back(Op{a, 0, pos, n, {t[0], t[1]}, front[a]});
                    std::vector<uint32_t> vv = v;
                    for (uint32_t j = 0; j < n; j++) {
                        const uint64_t lv = new_lv(a);
                        insert_char(a, vv, pos + j, lv);
                        advance(a, lv);
                        vv.insert(vv.begin() + int64_t(pos + j), uint32_t(lv));
                    }
                }
            } else {
                const uint64_t pos = rng.below(len);
                const uint64_t span = 1 + rng.below(std::min<uint64_t>(10, len - pos));
                const bool back = span > 1 && rng.chance(0.5);
                if (back) {   // backspaces, right to left: one op per char
                    for (uint64_t j = 0; j < span; j++) {
                        ops.push_back(Op{a, 1, pos + span - 1 - j, 1, {0, 0}, front[a]});
                        const uint64_t lv = new_lv(a);
                        deleters[v[pos + span - 1 - j]].push_back(uint32_t(lv));
                        advance(a, lv);
                    }
                } else {
                    ops.push_back(Op{a, 1, pos, span, {0, 0}, front[a]});
                    for (uint64_t j = 0; j < span; j++) {
                        const uint64_t lv = new_lv(a);
                        deleters[v[pos + j]].push_back(uint32_t(lv));
                        advance(a, lv);
                    }
                }
            }
        }
    }
};

dtgpu_status build_oplog(uint32_t na, const std::vector<Op> &ops, dtgpu_oplog **out) {
    dtgpu_oplog *o = dtgpu_oplog_new();
    std::vector<int32_t> agents(na);
    for (uint32_t a = 0; a < na; a++) {
        const std::string name = "a" + std::to_string(a);
        agents[a] = dtgpu_oplog_get_or_create_agent_id(o, name.data(), name.size());
    }
    for (const Op &op : ops) {
        int64_t r;
        if (op.kind == 0)
            r = dtgpu_oplog_add_insert_at(o, agents[op.agent], op.parents.data(), op.parents.size(), op.pos, op.text,
                                          size_t(op.len));
        else
            r = dtgpu_oplog_add_delete_at(o, agents[op.agent], op.parents.data(), op.parents.size(), op.pos,
                                          op.pos + op.len);
        if (r < 0) {
            dtgpu_oplog_free(o);
            return DTGPU_ERR_ARG;
        }
    }
    *out = o;
    return DTGPU_OK;
}

}  // namespace

extern "C" {

size_t dtgpu_synth_ops(uint64_t doc, uint32_t target_ops, uint32_t *n_agents, uint32_t *out, size_t cap) {
    uint32_t na = 0;
    std::vector<Op> ops;
    generate(doc, target_ops, na, ops);
    if (n_agents) *n_agents = na;
    size_t w = 0;
    for (const Op &o : ops) {
        const size_t need = 7 + o.parents.size();
        if (out && w + need <= cap) {
            out[w] = o.agent; out[w + 1] = o.kind; out[w + 2] = uint32_t(o.pos); out[w + 3] = uint32_t(o.len);
            out[w + 4] = uint8_t(o.text[0]); out[w + 5] = uint8_t(o.text[1]); out[w + 6] = uint32_t(o.parents.size());
            for (size_t k = 0; k < o.parents.size(); k++) out[w + 7 + k] = uint32_t(o.parents[k]);
        }
        w += need;
    }
    return w;
}

dtgpu_status dtgpu_synth_oplog(uint64_t doc, uint32_t target_ops, dtgpu_oplog **out) {
    if (!out) return DTGPU_ERR_ARG;
    uint32_t na = 0;
    std::vector<Op> ops;
    generate(doc, target_ops, na, ops);
    return build_oplog(na, ops, out);
}

dtgpu_status dtgpu_synth_merge_oplog(uint64_t doc, uint32_t target_ops, uint32_t n_agents, dtgpu_oplog **out) {
    if (!out || n_agents > 4096) return DTGPU_ERR_ARG;
    MergeGen g(doc, n_agents);
    std::vector<Op> ops;
    g.run(target_ops, ops);
    return build_oplog(g.k, ops, out);
}

}  // extern "C"
