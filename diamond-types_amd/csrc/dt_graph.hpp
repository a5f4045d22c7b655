// dt_graph.hpp -- host/device layout of the batched causal-graph queries (dt_graph.hip).
#pragma once
#include <stdint.h>

namespace dtgpu {

// Frontiers have no size cap (the reference's are SmallVecs): a query's versions live in a
// frontier arena, its common frontier / dominators in a common arena.  The heap walks run with
// their queues in LDS (first pass); a query whose queue outgrows LDS -- or whose time points carry
// more than GQ_LDS_MERGED merged versions -- is answered again in a second pass with its queues in
// HBM scratch sized from its graph (no capacity limit).
constexpr uint32_t GQ_LDS_MERGED = 16;
enum : uint32_t { GQ_DIFF = 0, GQ_CONFLICT = 1, GQ_CONTAINS = 2, GQ_DOMINATORS = 3, GQ_DIFF_LEVEL = 4,
                  GQ_CONFLICT_LEVEL = 5 };
// statuses (0..2 public; GQ_QUEUE_FULL is internal: the query moves to the HBM pass)
enum : uint32_t { GQ_OK = 0, GQ_OVERFLOW = 1, GQ_BAD_INPUT = 2, GQ_QUEUE_FULL = 3 };

// Graph arena: per graph, n_ent + 1 quads (start, end, shadow, parents offset); the extra quad
// carries the parents end offset.  Parents are absolute offsets into one parents array.
struct GraphQuery {
    uint32_t kind, ent_off, n_ent, na, nb, out_off, out_cap;
    int32_t target;                      // CONTAINS (-1 = ROOT)
    uint64_t scr_off;                    // level kinds: per-query HBM scratch (LevelParams.qscr)
    uint32_t scr_tp, pad;                // CONFLICT_LEVEL: time-point pool capacity
    uint32_t f_off;                      // a = front[f_off, +na), b = front[f_off + na, +nb)
    uint32_t c_off, c_cap;               // common[c_off, +c_cap)
    uint32_t max_par;                    // the most parents of any entry of the query's graph
    uint64_t h_off;                      // HBM pass: heap scratch (GraphParams.hscr words)
    uint32_t hk_cap, htp_cap;            // HBM pass: key heap / time-point heap capacities
};

struct GraphResult {
    uint32_t status, n0, n1, n_common;   // DIFF: spans only-a / only-b; CONFLICT: spans; CONTAINS: n0 = 0/1
};

struct GraphParams {
    const uint32_t *ents;
    const uint32_t *par;
    uint32_t *out;                       // DIFF: pairs, a then b (out_cap / 4 each); CONFLICT: triples
    const GraphQuery *queries;
    GraphResult *results;
    uint32_t n_queries;
    const int32_t *front;                // frontier arena
    int32_t *common;                     // CONFLICT: the common frontier; DOMINATORS: the result
    uint32_t *hscr;                      // HBM pass heap scratch
};

// Heap scratch of a query in the HBM pass (words): a key heap of one entry per parent slot of the
// graph and per version element, and a time-point heap whose points are (4 + widest version)
// words each (see dt_graph.hip).
__host__ __device__ inline uint32_t gq_key_cap(uint64_t n_par, uint32_t na, uint32_t nb) { return uint32_t(n_par + na + nb + 4); }
__host__ __device__ inline uint32_t gq_tp_cap(uint64_t n_ent, uint64_t n_par, uint32_t na, uint32_t nb) {
    return uint32_t(n_ent + n_par + na + nb + 8);
}
__host__ __device__ inline uint32_t gq_tp_words(uint32_t max_par, uint32_t na, uint32_t nb) {
    uint32_t w = max_par;
    if (na > w) w = na;
    if (nb > w) w = nb;
    return 4 + w;
}

// big = false: every heap-walk query, queues in LDS; big = true: only the queries the first launch
// left at GQ_QUEUE_FULL, queues in HBM scratch (GraphQuery.h_off / hk_cap / htp_cap)
int launch_graph_queries(const GraphParams &p, void *stream, bool big);

// Level-synchronous kernels (dt_level.hip).  Per-entry arrays are indexed like the entry quads
// (graph g's entry e at ent_off + e; every graph owns n_ent + 1 slots), per-slot arrays like
// the parents array.  All per-entry state is in HBM (no size cap): the levelling's counters
// (3 words per entry slot, at 3 * ent_off), each level query's marks (and, for conflict spans,
// bucket heads and a time-point pool) at its scr_off.
// Time points of a level conflict query: the two versions, one per visited entry (its parents) and
// one per version element or parent slot a merge point shatters into.
inline uint32_t conflict_level_tps(uint64_t n_ent, uint64_t n_par, uint32_t na, uint32_t nb) {
    return uint32_t(4 + n_ent + n_par + na + nb);
}
// marks (2 words per entry), bucket heads, candidates, the time-point pool (kLevelPointWords
// each) and an HBM bucket for entries that more than BUCKET_CAP points enter (one word per point)
constexpr uint32_t kLevelPointWords = 5;
inline uint64_t conflict_level_words(uint64_t n_ent, uint64_t n_par, uint32_t na, uint32_t nb) {
    return 4 * n_ent + (kLevelPointWords + 1ull) * conflict_level_tps(n_ent, n_par, na, nb);
}
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
    uint32_t lvl_lds;             // level_kernel: its counters and frontier queue in LDS for graphs up
                                  // to this many entries (0: in gscr / order in HBM)
    uint32_t sweep_pts;           // conflict sweep, first pass: LDS capacity in live time points
    uint32_t *prof;               // nullable (DTGPU_LVL_PROF): per conflict query 4 words -- cycles/16
                                  // in marks, candidate list, sweep; entries the sweep visited
};
// level_kernel keeps child counts, CSR offsets, pending counts and the level-order queue (4 words
// per entry) in LDS when every levelled graph has at most this many entries
constexpr uint32_t kLevelLdsLevelling = 9000;
inline size_t level_lds_bytes(uint32_t n) { return n ? 16 * (size_t(n) + 1) : 0; }
int launch_levels(const LevelParams &p, void *stream);
int launch_level_diff(const LevelParams &p, const GraphParams &q, void *stream);
// big = false: every level conflict query, time points in LDS; big = true: only the queries the
// first launch left at GQ_QUEUE_FULL, time points in HBM scratch
int launch_level_conflict(const LevelParams &p, const GraphParams &q, void *stream, bool big);

}  // namespace dtgpu
