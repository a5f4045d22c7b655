// dt_device.hpp -- host/device shared layout of a staged batch (see dt_replay.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>

#include "dt_host.hpp"

namespace dtgpu {

// The last launch's error (hipGetLastError, which also clears it), named on stderr with the
// launching file and line when set: a failed launch is never anonymous.
inline hipError_t launch_error(const char *file = __builtin_FILE(), int line = __builtin_LINE()) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) fprintf(stderr, "[dtgpu] launch error at %s:%d: %s\n", file, line, hipGetErrorString(e));
    return e;
}

// Per-document descriptor (device resident).  Offsets index the batch arenas.
struct DocDesc {
    uint64_t cmd_off;       // into cmds (Cmd units)
    uint64_t lv_off;        // into per-LV arenas (cbyte, st, blk, slot, aux, orr)
    uint64_t content_off;   // into content (bytes)
    uint64_t arun_off;      // into aruns (uint32 units)
    uint64_t blk_off;       // into items (blocks of 64 uint32)
    uint64_t out_off;       // into out (bytes)
    uint64_t gidx_off;      // into gidx (bytes), large-document tier only
    uint64_t tlist_off;     // into tlist (uint32 units)
    uint32_t ncmd, n_lv, n_aruns, max_blocks, out_cap, content_len;
    uint32_t ascii;         // every inserted char is one byte
    // Cut replay (a long document replayed as segments on several waves, see dt_replay.hip
    // "segments"): this replay applies the commands of the LV range [seg_lo, seg_hi) on top of
    // seg_u placeholder items standing for the text at seg_lo, and writes its visible items as a
    // source list (src_off, src_cap entries) instead of text.  Plain documents: seg_lo = seg_u =
    // 0, seg_hi = ~0, src_off = ~0.
    uint32_t seg_lo, seg_hi, seg_u, src_cap;
    uint64_t pc_off;        // into pos / ao: lv_off, or a segment's own region (n_lv + seg_u words)
    uint64_t src_off;       // into src (uint32 units), or ~0
    uint32_t flags;         // DOC_CRITICAL
};
constexpr uint32_t SEG_PHANTOM = 0x80000000u;   // source-list entry: placeholder item index
// The batch's critical path (dtgpu_api.cpp mark_critical): a replay several times longer than the
// batch's typical one, which the waves beside it would otherwise slow down by sharing the SIMD's
// issue; its waves take the top priority.
constexpr uint32_t DOC_CRITICAL = 1u;
// A linear history checked out on the fast-forward piece table (dt_ff.hip), not replayed.
constexpr uint32_t DOC_FF = 2u;
// A cut document whose segments' ranges came from the host plan because cut_kernel declined it
// (dt_prep.hip; tests assert the device plan is the one used).
constexpr uint32_t DOC_CUT_HOST = 4u;

struct DocResult {
    uint32_t status, out_len;
    uint64_t hash;
    uint32_t n_items, n_blocks;
    uint32_t fail_cmd, fail_site;   // diagnostics: command index and code site of the first error
    uint32_t n_sb, lds;             // superblocks at the end; 1 when the index was in LDS
    uint32_t dbg[22];               // DTGPU_DEBUG invariant-failure detail / cycle profile
};

// Packed per-item location word (dt_replay.hip): count | block | slot.
constexpr uint32_t LOC_CNT_SHIFT = 24;
constexpr uint32_t LOC_BLK_SHIFT = 6;
constexpr uint32_t LOC_BLK_MASK = 0x3FFFF;
constexpr uint32_t LOC_MAX_BLOCKS = LOC_BLK_MASK + 1;

struct BatchParams {
    const Cmd *cmds;
    const uint32_t *tlist;
    const uint32_t *cbyte;
    const uint8_t *content;
    const uint32_t *aruns;
    uint32_t *pos;   // per LV: block | count << 16 (dt_replay.hip pc[])
    unsigned long long *ao;
    uint32_t *items;
    unsigned long long *m2;   // per block: visible, live slot masks
    uint8_t *out;
    uint8_t *gidx;
    const DocDesc *docs;
    const uint32_t *doc_list;
    uint32_t n_list;
    uint32_t lds_blocks;    // block-index capacity held in LDS (LDS tiers)
    uint32_t lds_sb;        // superblock capacity held in LDS (LDS tiers)
    uint32_t *fb_list;      // LDS-tier documents handed to the HBM tier (capacity overflow)
    uint32_t *fb_count;
    uint32_t fb_slots;      // HBM tier: grid slots for handed-back documents (all LDS-tier docs)
    uint32_t debug;         // DTGPU_DEBUG: bit 0 invariant checks, bit 1 cycle profile
    DocResult *results;
    // transformed-ops mode only (launch_replay_xf): never-deleted masks per block, never-deleted
    // totals per top position (blk_off + 2 * doc), transformed position per LV
    unsigned long long *mup;
    uint32_t *tup;
    uint32_t *xf;
    uint32_t *src;   // cut replay: the segments' source lists (DocDesc::src_off)
    uint32_t lds_flat;   // LDS tiers: 1 = the flat 2-level index (IX_FLAT), 0 = the 3-level one
    uint32_t prio_from;  // LDS tiers: workgroups from this index on (dispatched after the first
                         // resident set) raise their wave priority (0: off)
    uint32_t n_cu;       // compute units of the batch's device (resident-set sizes)
    uint32_t prio_on;    // LDS tiers: late workgroups raise their priority (prio_from computed at launch)
    uint32_t tog_waves;  // 1: retreat / advance passes on one wave; else helper waves on the big tiers
    uint32_t tog_mw_lds; // LDS index bytes from which a tier gets helper waves
};

// Cut replay: after the replay, one workgroup per cut document resolves its segments' source
// lists in order (each placeholder to the previous segment's entry) and writes the text.
struct SegGroup { uint32_t first, count; };   // into seg_docs: the document's segments in LV order
struct CombineParams {
    const SegGroup *groups;
    const uint32_t *seg_docs;
    uint32_t n_groups;
    const DocDesc *docs;
    DocResult *results;
    uint32_t *src;
    const uint32_t *cbyte;
    const uint8_t *content;
    uint8_t *out;
    uint32_t n_cu;   // compute units of the batch's device
};
int launch_combine(const CombineParams &p, void *stream);

// Superblock capacity for an index of `mb` blocks: every superblock but the first holds >= 32
// blocks (they split 64 -> 32 + 32).
__host__ __device__ inline uint32_t sb_capacity(uint32_t mb) { return mb / 32 + 2; }
// Bytes of a block index for `mb` blocks (dt_replay.hip bind_index): per block the packed
// counts (u32) and the (superblock, index) position (u32; u16 when `narrow`, the LDS tier); per
// superblock visible / live totals, list length, top position (u32 each)
// and a 64-entry u16 block list.
__host__ __device__ inline uint64_t index_bytes_ms(uint64_t mb, uint64_t ms, bool narrow) {
    const uint64_t per_block = narrow ? 4 * mb + 4 * ((mb + 1) / 2) : 8 * mb;
    return ((per_block + 16 * ms + 128 * ms) + 15) & ~uint64_t(15);
}
__host__ __device__ inline uint64_t index_bytes(uint64_t mb, bool narrow = false) {
    return index_bytes_ms(mb, sb_capacity(uint32_t(mb)), narrow);
}
// LDS tiers size the superblock pool for the expected fill (superblocks hold 32..64 blocks,
// ~44 on the benchmark traces) rather than the worst case: LDS is what bounds how many
// documents share a CU, and a document that outgrows the pool is handed to the HBM tier like
// one that outgrows its blocks (split_sb, ErrCapacity site 21).
constexpr uint32_t LDS_SB_FILL = 40;
__host__ __device__ inline uint32_t lds_sb_capacity(uint32_t mb, uint32_t fill = LDS_SB_FILL) {
    const uint32_t opt = mb / fill + 3;
    return opt < sb_capacity(mb) ? opt : sb_capacity(mb);
}
// The flat LDS index (dt_replay.hip IX_FLAT): per block the packed counts (u32), its position
// and the block at each position (u16 each); per 64 positions the packed visible | live totals.
__host__ __device__ inline uint32_t flat_chunks(uint32_t mb) { return (mb + 63) / 64; }
__host__ __device__ inline uint64_t flat_index_bytes(uint64_t mb) {
    return ((4 * mb + 8 * ((mb + 1) / 2) + 4 * uint64_t(flat_chunks(uint32_t(mb)))) + 15) & ~uint64_t(15);
}
// The flat index serves the smallest LDS tier; a split costs O(blocks / 64) lane rounds, so it is
// kept to documents of at most this many blocks.
constexpr uint32_t FLAT_MAX_BLOCKS = 2048;
constexpr uint32_t MAX_DOC_BLOCKS = 65535;   // block ids are u16 in the superblock lists

// ---- device planner (dt_plan.hip) -------------------------------------------------------------
constexpr uint32_t PLAN_MAX_AGENTS = 512;
constexpr uint32_t PLAN_MAX_LDS_ENTRIES = 16384;   // u16 todo + u16 pending per entry in LDS
enum PlanStatus : uint32_t {
    PLAN_OK = 0, PLAN_NOT_CHAIN = 1, PLAN_TLIST_FULL = 2, PLAN_CMDS_FULL = 3, PLAN_TOO_MANY_AGENTS = 4,
    PLAN_ERR_INTERNAL = 5, PLAN_TODO_FULL = 6, PLAN_WIDE_MERGE = 7,
};
constexpr uint32_t PLAN_TODO_CAP = 512;   // ready-entry stack slots per wave (LDS, u16 each)
struct PlanDesc {       // per document; offsets index the concatenated PlanInput arrays
    uint64_t e_off;     // entries
    uint64_t par_off;   // par / pent
    uint64_t child_off, op_off, arun_off, tip_off;
    uint64_t base_off;  // vv rows scratch (n_entries * n_agents)
    uint64_t erec_off, doff_off, dense_off;
    uint64_t cmd_off, tlist_off;
    uint64_t prow_off;    // parent version vectors (per entry, row_stride words, chains < n_agents)
    uint32_t ne, n_agents, n_aruns, ntip, n_lv, ccap, tcap, skip;
    uint32_t row_stride, pad;
    uint64_t coff_off, poff_off;   // device staging: per entry children (prep scratch), parent offsets (decoder)
};
struct PlanResult {
    uint32_t status, ncmd, ntlist, n_tip;
    uint64_t n_retreat, n_advance;
    uint64_t prof[6];   // DTGPU_PLAN_PROF: cycles in record wait, parents, children+pick, emit, ops, init
};
struct PlanParams {
    const uint32_t *par, *pent, *pch, *pcnt, *child, *aruns, *tip, *erec, *doff, *dense;
    const Cmd *opc;
    uint32_t *base;
    const uint32_t *prow;   // per-entry parent version vectors (prep / build_plan_input), <= 64 chains
    uint32_t lds_entries;   // per-wave LDS capacity (entries) of the todo stack / pending counts
    uint32_t max_agents;    // largest agent count among device-planned documents
    uint32_t prof;          // cycle profile into PlanResult.prof
    uint32_t split;         // <= 64 chains: the two-phase planner (order, then lane-parallel steps)
    uint32_t *order;        // two-phase planner: walk orders, document d's at its entry offset
    uint32_t *walk;         // nullable: per document {status, steps} of walk_kernel (the orders
                            // four documents per wave); null: the planner walks itself
    const uint32_t *coff, *poff;   // walk_kernel's CSR mode: children offsets, parent offsets
    uint32_t todo_cap;             // walk_kernel: stack slots per document (0: PLAN_TODO_CAP) -- the
                                   // staging walk's deepest stack, so more walks share a CU's LDS
    Cmd *cmds;
    uint32_t *tlist;
    const PlanDesc *docs;
    PlanResult *results;
    uint32_t n_docs, count_only;   // n_docs: the grid (the list's length when doc_list is set)
    const uint32_t *doc_list;      // nullable: block i plans docs[doc_list[i]]
};
int launch_plan(const PlanParams &q, void *stream, bool walk = true);
// walk_kernel alone; csr: children and parent counts from prep's CSR (ready after prep's first
// half, so the walk can run beside the chain decomposition) instead of the entry records
int launch_walk(const PlanParams &q, void *stream, bool csr);

// One replay pass: the LDS tiers (index in LDS, sized per tier) and then the HBM-index tier,
// which also replays the LDS-tier documents that outgrew their LDS capacity.  A tier kernel
// lasts as long as its longest replay, so tiers queued on one stream add up: the biggest tiers
// (few, long documents) each run on a side stream of their own, forked from and joined back
// into `stream`, beside the smallest tier; every list indexes docs[].
constexpr int kMaxLdsTiers = 4;
constexpr int kSideStreams = kMaxLdsTiers - 1;
struct ReplayLaunch {
    const BatchParams *lds;   // n_lds LDS tiers, smallest index first
    int n_lds;
    const BatchParams *large;
    void *stream;                   // hipStream_t
    void *side[kSideStreams];       // hipStream_t: tier n_lds - 1 - k on side[k]
    void *ev_fork;                  // hipEvent_t
    void *ev_join[kSideStreams];    // hipEvent_t
    bool keep_fb = false;           // the fallback counter was reset by the caller (split passes)
    int join_side = -1;             // split pass: side[join_side] carries the big tier's own
                                    // prep / plan / replay; s joins it before the HBM tier always
};
int launch_replay(const ReplayLaunch &r);
// Transformed-ops replay of large's documents (HBM index tier): BaseMoved positions per LV.
int launch_replay_xf(const BatchParams &large, void *stream);

}  // namespace dtgpu
