// dt_prep.hpp -- host/device layout of the planner-input builder (dt_prep.hip): the decoded
// oplog arenas of dt_decode.hip in, the PlanInput arrays of dt_host.hpp (build_plan_input) out.
#pragma once
#include <stdint.h>

#include "dt_device.hpp"
#include "dt_host.hpp"

namespace dtgpu {

constexpr uint32_t PREP_MAX_CHAINS = 64;   // wider histories are prepared on the host
// PREP_BOUNDS: a debug-mode bounds assert failed (a table index outside the document's arena);
// PrepResult.pad then names the table (PREP_T_*)
enum : uint32_t { PREP_OK = 0, PREP_WIDE = 1, PREP_BAD = 2, PREP_SKIP = 3, PREP_BOUNDS = 4 };
enum : uint32_t { PREP_T_CHILD = 1, PREP_T_ROWS = 2, PREP_T_PAIRS = 3, PREP_T_DOFF = 4, PREP_T_DENSE = 5, PREP_T_ERECP = 6,
                  PREP_T_ENTRY = 7 };

struct PrepDesc {
    // decoder arenas (offsets in the decoder's units: quads / pairs / words / bytes)
    uint64_t d_op, d_arun, d_ent, d_poff, d_par, d_ver, d_agent, d_in;
    uint32_t n_ops, n_aruns, ne, n_par, n_ver, n_agents, n_lv, skip;
    // words per parent-vector row: PREP_MAX_CHAINS until the staging pass has counted the
    // document's chains, then that count rounded up to a multiple of four (a decomposition that
    // would open a chain past it reports PREP_WIDE); the planner reads rows with the same stride
    uint32_t row_stride, pad;
    // planner arenas (offsets in PlanDesc units)
    uint64_t o_par;     // par / pent / pch / pcnt slots
    uint64_t o_child;   // child slots
    uint64_t o_op;      // Cmd units
    uint64_t o_arun;    // quads
    uint64_t o_tip;     // pairs
    uint64_t o_erec;    // words (EREC_WORDS per entry)
    uint64_t o_doff;    // words (PREP_MAX_CHAINS + 1)
    uint64_t o_dense;   // words (n_lv)
    uint64_t o_rows;    // words (PREP_MAX_CHAINS per entry reserved): parent vectors of the decomposition
    uint64_t o_scr;     // words (even): owner (n_par, padded), {chain, seq0 - start} (2 ne), coff, eop (ne + 1 each)
};

struct PrepResult {
    uint32_t status, n_chains, n_ins, pad;
};

struct PrepParams {
    const uint8_t *in;
    const uint32_t *d_ops, *d_aruns, *d_ent, *d_poff, *d_par, *d_ver, *d_agents;
    uint32_t *par, *pent, *pch, *pcnt, *child, *aruns, *tip, *erec, *doff, *dense, *rows, *scr;
    Cmd *opc;
    const PrepDesc *docs;
    PrepResult *results;
    uint32_t n_docs, max_entries;   // n_docs: the grid (the list's length when doc_list is set)
    const uint32_t *doc_list;       // nullable: block i prepares docs[doc_list[i]]
    uint32_t check;                 // debug mode (DTGPU_DEBUG): the bounds-checked kernel
    // nullable: per document (by index) the stage of a three-launch pass -- prep_kernel's first
    // half (parents, children, first op runs) sets 1, chain_kernel sets 2 when it decomposed the
    // document into chains, the second half decomposes the rest itself; null: one launch
    uint32_t *chain_flag;
    uint32_t mode;                  // set by launch_prep: 0 whole kernel, 1 first half, 2 second half
    uint32_t chain_w;               // chain_kernel: the widest row stride of the batch (0: unknown)
    uint32_t short_rec;             // entry records: heads only (a pass whose walk reads the CSR and
                                    // whose planner reads heads: dt_host.hpp PlanInput::erec)
};
// chain_kernel: documents per wave, lanes (= chains) per document; per document a ring of the
// last 2 CHAIN_GROUP entries' rows (chain_w words each, 0: CHAIN_GROUP) and {entry, chain, sd}
constexpr uint32_t CHAIN_GROUP = 16, CHAIN_DOCS = 64 / CHAIN_GROUP;
constexpr uint32_t chain_ring_width(uint32_t w) { return w && w < CHAIN_GROUP ? w : CHAIN_GROUP; }
constexpr uint32_t chain_lds_words(uint32_t w) { return 2 * CHAIN_GROUP * (chain_ring_width(w) + 3); }

// owner (n_par, padded to even), {chain, seq0 - start} pairs (2 ne), coff, eop (ne + 1 each), then
// per entry {children | first child slot << 16, first child | last child << 16} (2 ne used of 4 ne,
// the walk kernel's): even,
// so every document's pair array is 8-byte aligned
inline uint64_t prep_scratch_words(uint32_t n_par, uint32_t ne) { return (uint64_t(n_par) + 1) / 2 * 2 + 8ull * ne + 2; }
inline uint64_t prep_kids_offset(uint32_t n_par, uint32_t ne) { return (uint64_t(n_par) + 1) / 2 * 2 + 4ull * ne + 2; }

int launch_prep(const PrepParams &p, void *stream);

// Cut planning inside the checkout pass (cut_kernel): for every cut document (SegGroup), from the
// decoded oplog, the cut ranges (dtgpu_api.cpp cut_ranges), the cuts nearest to equal cost
// shares (plan_segments) and each segment's LV range and placeholder bound, written into its
// DocDesc.  Staging only reserves each segment's arenas (SegCap: the placeholders and inserts
// its arenas hold) and poisons the descriptors' ranges, so a pass without this kernel fails.
// A segment's replay cost in LVs: the replay holds one item per LV, so an op run costs its
// length (inserted items, deleted items toggled) plus a fixed share per run (the position lookup
// and the block loads): the cuts share out w_op * runs + LVs, not the runs alone (rustcode's
// pastes of 50k characters put 4x the work in 1/16th of the runs).  cost(j) = w_op * j + the LV
// of op run j; the total is w_op * runs + the last run's end.
constexpr uint32_t SEG_W_OP = 48;   // default w_op (DTGPU_SEG_W)
struct SegPlan { uint32_t w_op, n_targets; uint64_t scr_off; };   // per group: the cost weight of an
                                                                  // op run, the target count, scratch (words)
// per seg_docs slot: the reserved placeholders and inserts, and the host plan's LV range, which
// the kernel writes instead of its own when it declines the document (its cuts differ from the
// reserved segments, or a bound exceeds what was reserved; DOC_CUT_HOST marks it)
struct SegCap { uint32_t u, ins, lo, hi; };
struct CutParams {
    const uint32_t *d_ops, *d_ent, *d_poff, *d_par;   // decoder arenas (as PrepParams)
    const PrepDesc *pdocs;                            // per document
    const SegGroup *groups;
    const uint32_t *seg_docs;
    const SegPlan *plans;
    const SegCap *caps;
    DocDesc *docs;
    const uint32_t *pent;   // prep's first half: each parent slot's entry (the kernel then runs after
                            // it); null: the kernel searches the entries itself
    uint32_t *scr;      // per group cut_scratch_words (SegPlan::scr_off)
    uint32_t n_groups, max_ne;   // max_ne: the LDS table's entries (the groups' largest document)
    // staging (sizing mode): groups hold one document each with count = the target count; the
    // kernel writes per group CUT_SIZED_WORDS words -- the segment count (0: not cut), then per
    // segment {first LV, end LV, placeholders, inserted chars} -- instead of descriptors
    uint32_t *sized;
};
constexpr uint32_t CUT_SIZED_WORDS = 1 + 4 * 64;
// suffix minima (ne + 1), cut ranges (2 ne), alignment
inline uint64_t cut_scratch_words(uint32_t ne) { return 3ull * ne + 4; }
int launch_cut(const CutParams &p, void *stream);
// The three-launch pass one stage at a time (1: first half, 2: chains, 3: second half), so a
// caller can start work that needs only the first half (the planner's walk) beside the rest.
// Requires p.chain_flag and !p.check.
int launch_prep_stage(const PrepParams &p, void *stream, int stage);
// An empty one-wave kernel that opens a checkout pass when DTGPU_PASS_MARK is set at staging:
// the PMC traffic tool (tools/traffic.py) sums the dispatches after the last marker, whatever
// mix of streams and pipelines the pass uses.
int launch_pass_mark(void *stream);

}  // namespace dtgpu
