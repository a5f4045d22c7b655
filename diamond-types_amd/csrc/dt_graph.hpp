// dt_graph.hpp -- host/device layout of the batched causal-graph queries (dt_graph.hip).
#pragma once
#include <stdint.h>

namespace dtgpu {

constexpr uint32_t GQ_MAX_FRONTIER = 16;
enum : uint32_t { GQ_DIFF = 0, GQ_CONFLICT = 1, GQ_CONTAINS = 2, GQ_DOMINATORS = 3, GQ_DIFF_LEVEL = 4,
                  GQ_CONFLICT_LEVEL = 5 };
enum : uint32_t { GQ_OK = 0, GQ_OVERFLOW = 1, GQ_BAD_INPUT = 2 };

// Graph arena: per graph, n_ent + 1 quads (start, end, shadow, parents offset); the extra quad
// carries the parents end offset.  Parents are absolute offsets into one parents array.
struct GraphQuery {
    uint32_t kind, ent_off, n_ent, na, nb, out_off, out_cap;
    int32_t target;                      // CONTAINS (-1 = ROOT)
    uint64_t scr_off;                    // level kinds: per-query HBM scratch (LevelParams.qscr)
    uint32_t scr_tp, pad;                // CONFLICT_LEVEL: time-point pool capacity
    int32_t a[GQ_MAX_FRONTIER], b[GQ_MAX_FRONTIER];
};

struct GraphResult {
    uint32_t status, n0, n1, n_common;   // DIFF: spans only-a / only-b; CONFLICT: spans; CONTAINS: n0 = 0/1
    int32_t common[GQ_MAX_FRONTIER];     // CONFLICT: the common frontier; DOMINATORS: the result
};

struct GraphParams {
    const uint32_t *ents;
    const uint32_t *par;
    uint32_t *out;                       // DIFF: pairs, a then b (out_cap / 4 each); CONFLICT: triples
    const GraphQuery *queries;
    GraphResult *results;
    uint32_t n_queries;
};

int launch_graph_queries(const GraphParams &p, void *stream);

// Level-synchronous kernels (dt_level.hip).  Per-entry arrays are indexed like the entry quads
// (graph g's entry e at ent_off + e; every graph owns n_ent + 1 slots), per-slot arrays like
// the parents array.  All per-entry state is in HBM (no size cap): the levelling's counters
// (3 words per entry slot, at 3 * ent_off), each level query's marks (and, for conflict spans,
// bucket heads and a time-point pool) at its scr_off.
inline uint64_t conflict_level_words(uint64_t n_ent, uint64_t n_par) { return 4 * n_ent + 4 * (34 + n_ent + n_par); }
inline uint32_t conflict_level_tps(uint64_t n_ent, uint64_t n_par) { return uint32_t(34 + n_ent + n_par); }
struct LevelGraph { uint32_t ent_off, n_ent; };
// The query kernels keep the marks (2 words per entry) in LDS when every levelled graph of the
// launch has at most this many entries (48 KiB; sized to the largest graph, so small graphs keep
// many queries per CU); larger graphs keep them in HBM scratch.  (The conflict sweep's bucket
// heads and candidates in LDS as well measured slower: half the queries per CU.)
constexpr uint32_t kLevelLdsEntries = 6144;
struct LevelParams {
    const uint32_t *ents, *par;   // the GraphParams arena
    uint32_t *pent, *child;       // per parent slot: its parent's entry; children CSR (by parent entry)
    uint32_t *level, *order;      // per entry: its level; the entries in level order
    uint32_t *lvl_off;            // per graph: level L's entries are order[lvl_off[L], lvl_off[L + 1])
    uint32_t *meta;               // per graph at 2 * ent_off: number of levels, status
    uint32_t *gscr;               // per graph at 3 * ent_off: child counts / CSR offsets / pending
    uint32_t *qscr;               // per level query at its scr_off
    const LevelGraph *graphs;
    uint32_t n_graphs;
    uint32_t lds_ent;             // query kernels: the marks of graphs up to this many entries in LDS
};
int launch_levels(const LevelParams &p, void *stream);
int launch_level_diff(const LevelParams &p, const GraphParams &q, void *stream);
int launch_level_conflict(const LevelParams &p, const GraphParams &q, void *stream);

}  // namespace dtgpu
