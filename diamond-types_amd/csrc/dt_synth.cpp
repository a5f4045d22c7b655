// dt_synth.cpp -- deterministic synthetic concurrent documents (BASELINE.json configs[3]: "1M
// synthetic concurrent docs, 4-16 agents, ~5k ops each"), modelled on the reference's fuzzers
// (make_random_change, src/list_fuzzer_tools.rs:38-104; merge_fuzz, src/listmerge/fuzzer.rs:34-129):
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

}  // extern "C"
