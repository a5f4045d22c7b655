// dt_replay.hip -- per-document eg-walker replay + text materialisation on MI355X (gfx950).
//
// One wavefront (64 lanes) replays one document's command stream (built on the host from the
// spanning-tree walk, dt_host.cpp::build_plan).  This is the checkout-from-ROOT per-item
// formulation of the reference's M2Tracker (src/listmerge/merge.rs:89-581,
// advance_retreat.rs:58-153, yjsspan.rs:13-228).
//
// Document = a 3-level order-statistic tree of inserted chars (items):
//   block        64 item slots in document order; items[] (LV ids), and the visible / live
//                (non-NIY) bit masks mvis[] / mlive[]: HBM.
//   superblock   an ordered list of <= 64 block ids (sbl) with visible / live totals.
//   top          the ordered list of superblocks: top[p] = superblock id << 16 | visible
//                total, tlive[p] = live total, by top position p.
//   The block and superblock index (packed per-block counts: visible | live << 8 | items << 16;
//   block -> (superblock, index) opos; the superblock lists and totals) lives in LDS for
//   documents whose index fits the LDS budget and in HBM otherwise (same code).  A full block
//   splits 64 -> 32 + 32 and a full superblock 64 -> 32 + 32, so a split costs O(64) work.
//   pc[lv]       inserted LV: its block (low 16 bits) | its count << 16 (count 0 = NIY, 1 =
//                inserted, k >= 2 deleted k-1 times).  One word, so a retreat/advance lane and a
//                block rebuild read one array.  The block is written when the item is inserted
//                and when a split moves it to a new block -- never for the items an insert shifts
//                inside a block (content-tree notifies its marker index only when an entry
//                changes leaf, crates/content-tree/src/mutations.rs:76-110,196;
//                src/listmerge/markers.rs).  The slot, where needed (YjsMod's document-order
//                keys), is found in the row.
//   Block masks (visible / live) are a cache of the counts: a retreat/advance pass changes
//   counts only and marks the blocks whose masks it invalidated (DIRTY bit of the packed
//   count); the next command that loads such a block rebuilds its masks from pc[].
//   ao[lv]       Ins: origin_left | origin_right << 32; Del: the item it deleted.
//   Every per-document structure is touched by its own wave only, so no global atomics are
//   needed: on gfx950 every global atomic, whatever its scope, leaves L2 as a memory-side
//   request (profiles/r2_calib: 32 B of WRITE_SIZE per atomic even on an L2-resident line),
//   while plain stores are absorbed by the write-back L2.  Lanes of one pass that touch the
//   same item are merged in registers; the index counts live in LDS (LDS tier) or take one
//   atomic per distinct block (HBM tier).
//
// Commands: INS / DEL apply one op run; TOG applies one walk step's whole retreat + advance
// set in one lane-parallel pass.  Counters make that legal: a retreat subtracts one, an advance
// adds one, and an item's final count is its old count plus the sum of its deltas whatever the
// order, so the pass ends in the state the reference reaches by retreating in descending LV
// order and then advancing (advance_retreat.rs:58-153).  Visibility (count == 1) and liveness
// (count >= 1) follow from the old and new counts.  The retreat set is contained in the
// current version, so old count + the retreats never goes negative (checked).
//
// The plan ends with a TOG that advances to the tip, so the final visible set is the checkout:
// materialisation stream-compacts visible items in document order (list/merge.rs:63-95).
//
// Document order is the lexicographic order of (top position, index in superblock, slot):
// YjsMod compares those keys directly (merge.rs:154-278) instead of counting items.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <stdint.h>

#include "dt_device.hpp"

namespace dtgpu {
namespace dev {

typedef unsigned long long u64;

#define DEV __device__ __forceinline__

DEV uint32_t lane_id() { return __lane_id(); }
DEV void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); }
DEV uint32_t bcast(uint32_t v, uint32_t l) { return uint32_t(__builtin_amdgcn_readlane(int(v), int(l))); }
DEV u64 bcast64(u64 v, uint32_t l) {
    return (u64(bcast(uint32_t(v >> 32), l)) << 32) | u64(bcast(uint32_t(v), l));
}
DEV uint32_t first_lane(u64 m) { return uint32_t(__ffsll((long long)m) - 1); }
DEV uint32_t last_lane(u64 m) { return 63u - uint32_t(__clzll((long long)m)); }
// Wave-uniform values are pinned to scalar registers: control flow that depends on them is
// scalar (no exec-mask loops), which is both what the algorithm means and what keeps hipcc
// from treating the sequential replay as divergent.
DEV uint32_t U(uint32_t v) { return uint32_t(__builtin_amdgcn_readfirstlane(int(v))); }
DEV u64 U64(u64 v) {   // (readfirstlane returns int: keep both halves unsigned)
    return (u64(U(uint32_t(v >> 32))) << 32) | u64(U(uint32_t(v)));
}
DEV uint32_t shfl(uint32_t v, uint32_t src) {
    return uint32_t(__builtin_amdgcn_ds_bpermute(int(src << 2), int(v)));
}
DEV u64 lanes_below(uint32_t l) { return l >= 64 ? ~0ull : ((1ull << l) - 1ull); }
// Set bits of m below this lane (v_mbcnt: two VALU ops, no 64-bit shifts).
DEV uint32_t bits_below(u64 m) {
    return __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
}
// The replay's scalar issue is its bottleneck (one SALU per SIMD per 4 cycles; +48 SALU per
// command costs the full issue time, +48 VALU 40 % of it): per-lane flags are kept as 0/1
// integers in VGPRs.  A bool per lane is a lane mask in SGPRs, and each &&, || or ! on it is a
// 64-bit scalar op; the empty asm keeps the compiler from folding the integer back into one.
DEV uint32_t vflag(bool c) {
    uint32_t x = c ? 1u : 0u;
    asm volatile("" : "+v"(x));
    return x;
}
// __ballot with the mask straight from the compare (the HIP wrapper adds a select and a compare).
#define BALLOT(c) __ballot(c)

// Inclusive wave prefix sum over 64 lanes with DPP: Hillis-Steele inside each 16-lane row
// (row_shr 1/2/4/8), then row_bcast:15 and row_bcast:31 carry the row totals forward.
// Validated against a sequential prefix sum by tools/scan_probe.hip.
DEV uint32_t wave_scan(uint32_t x) {
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x142, 0xA, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x143, 0xC, 0xF, false));
    return x;
}
// The same over lanes 0..31 only (lanes 32..63 left partial): one DPP step fewer.
DEV uint32_t wave_scan32(uint32_t x) {
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x142, 0xA, 0xF, false));
    return x;
}
DEV uint32_t wave_sum(uint32_t v) { return uint32_t(__builtin_amdgcn_readlane(int(wave_scan(v)), 63)); }
DEV u64 wave_sum64(u64 v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
DEV u64 splitmix(u64 z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
DEV uint32_t utf8_len(uint8_t c) { return c < 0x80 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : 4; }

constexpr uint32_t BLK = 64;   // slots per block
constexpr uint32_t SBC = 64;   // block capacity of a superblock list
constexpr uint32_t ROOT_ID = 0xFFFFFFFFu;
constexpr uint32_t END_ID = 0xFFFFFFFEu;
constexpr uint32_t NONE = 0xFFFFFFFFu;
// packed per-block counts
constexpr uint32_t C_VIS = 1u, C_LIVE = 1u << 8, C_ITEMS = 1u << 16;
constexpr uint32_t C_UP = 1u << 24;   // transformed-ops mode: items never deleted (<= 64: 7 bits)
constexpr uint32_t C_DIRTY = 1u << 31;   // the block's masks are stale (a toggle changed counts)
DEV uint32_t c_vis(uint32_t c) { return c & 0xFFu; }
DEV uint32_t c_live(uint32_t c) { return (c >> 8) & 0xFFu; }
DEV uint32_t c_items(uint32_t c) { return (c >> 16) & 0xFFu; }
DEV uint32_t c_up(uint32_t c) { return (c >> 24) & 0x7Fu; }
// pc[] word: block | count << 16 (MAX_DOC_BLOCKS = 65535; a count past 65535 is ErrCheckout)
DEV uint32_t pc_blk(uint32_t w) { return w & 0xFFFFu; }
DEV uint32_t pc_cnt(uint32_t w) { return w >> 16; }
DEV uint32_t pc_of(uint32_t b, uint32_t k) { return b | (k << 16); }

// Per-document state (pc, masks) is only ever read and written by its own wave with plain
// accesses, which the CU keeps coherent for that wave: plain loads may hit L1.  The HBM-index
// words that the HBM tier updates with memory-side atomics are read L2-coherently (ld_sc).
template <typename T> DEV T ld(const T *p) { return *p; }
// Cold state (kernel arguments and document descriptor fields used only at the end of a document
// or on rare paths) is re-read where it is used: volatile, so the compiler neither keeps it in
// SGPRs across the command loop nor spills it there (the hot loop is SGPR-bound).
template <typename T> DEV T vld(const T *p) { return *reinterpret_cast<const volatile T *>(p); }
DEV const BatchParams &KP() {
    return *(const BatchParams *)(__builtin_amdgcn_kernarg_segment_ptr());
}
// A pointer re-read from the arguments is generic to the compiler: declare it global so its
// accesses are global_load / global_store (vmcnt only), not flat.
#define GLOBAL_AS __attribute__((address_space(1)))
template <typename T> DEV GLOBAL_AS T *gp(T *p) { return (GLOBAL_AS T *)p; }
template <typename T> DEV void st(T *p, T v) { *p = v; }
// L2-coherent accesses (a load must never meet a stale L1 line of a word an atomic changed).
template <typename T> DEV T ld_sc(const T *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
template <typename T> DEV void st_sc(T *p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
DEV uint32_t cv_add(uint32_t *p, uint32_t d) { return __hip_atomic_fetch_add(p, d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
template <typename T> DEV void at_xor(T *p, T v) { __hip_atomic_fetch_xor(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
template <typename T> DEV void at_add(T *p, T v) { __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
template <typename T> DEV void at_or(T *p, T v) { __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }

// Index accessors.  LDS tier: plain LDS (one wave owns the workgroup).  HBM tier: words that
// atomics touch are read L2-coherently.
template <int L> DEV uint32_t ix(const uint32_t *p) {
    if (L) return *p;
    return ld_sc(p);
}
template <int L> DEV uint32_t ix16(const uint16_t *p) { return *p; }

enum ProfSlot { P_INS = 0, P_DEL, P_TOG, P_MAT, P_YJS, P_SPLIT, P_FIND, P_BLOAD, P_ORR, P_RUN, P_R1, P_R2, P_R3, P_N_YJS, P_N_SPLIT,
                P_T1, P_T2, P_T3, P_N_DIRTY, P_N_LOAD, P_N };   // P_T*: retreat/advance pass split (entries + merge, counts, index)

struct Doc {
    // inputs
    const Cmd *cmds;
    uint32_t ncmd, n_lv;   // n_lv: item ids (the LVs, then a segment's placeholders)
    const uint32_t *tlist;
    const DocDesc *desc;   // cold fields (content, agent runs, output) are read from it when used
    // per-LV state (HBM)
    uint32_t *pc;    // inserted LV: block | count << 16 (plain loads / stores)
    u64 *ao;         // Ins: origin_left | origin_right << 32; Del: the item it deleted (low word)
    // blocks (HBM)
    uint32_t *items;
    u64 *m2;         // per block: visible mask, live mask (adjacent: one wave load / store)
    uint32_t max_blocks, max_sb;
    // index (LDS or HBM)
    uint32_t *cnt, *opos;                                // per block (opos: HBM tier)
    uint16_t *opos16;                                    // per block (opos: LDS tier)
    uint32_t *sbn, *sbpos;                               // per superblock
    uint32_t *top, *tlive;                               // by top position
    uint16_t *sbl;                                       // per superblock: SBC block ids
    // wave-uniform scalars
    uint32_t nb, nsb;
    uint32_t err;
    uint32_t debug;
    uint32_t site;
    uint32_t steps;               // watchdog: loop iterations left; every loop iteration is charged; a bound
                                  // violation ends the document with ErrCapacity
    uint64_t prof[P_N];
    uint32_t doc;
    // the block the last insert / delete left behind, in registers (items lane by lane, masks):
    // typing keeps hitting it, so the next command skips its load.  Memory always holds the
    // same state (every change is stored); a toggle touching the block drops it.
    uint32_t cb, cit;
    u64 cmv, cml;
    // transformed-ops mode (iter_xf_operations): per block the never-deleted mask, per top
    // position the never-deleted total, per LV the transformed position written out
    u64 *mup;
    uint32_t *tup;
    uint32_t *xf;
};

DEV void fail(Doc &D, uint32_t code, uint32_t site) {
    if (!D.err) { D.err = code; D.site = site; }
}
// Charge one loop iteration; returns false (and flags the document) past the budget.  Charged:
// the command loop and the loops that walk the index (YjsMod scan, next live block, agent
// search), whose termination rests on the index being consistent; every other loop retires at
// least one item, lane or block per round.
DEV bool charge(Doc &D) {
    if (D.steps == 0) { fail(D, ErrCapacity, 1); return false; }
    D.steps--;
    return true;
}
template <bool PROF> DEV uint64_t tick() { return PROF ? __builtin_amdgcn_s_memtime() : 0; }

// Index kinds (the template parameter L of the navigation code; nonzero = the index is in LDS):
//   IX_HBM   3-level index in HBM (big documents, LDS overflow, transformed-ops mode)
//   IX_LDS   3-level index in LDS (the big LDS tiers)
//   IX_FLAT  2-level index in LDS (the smallest tier: friendsforever-sized documents).  The
//            blocks in document order are one array ord[] (block id by position), opos16[b] is
//            block b's position, and ctot[c] (held in D.top) packs the visible | live << 16
//            totals of positions [64c, 64c + 64).  A split shifts ord[] right of the new block
//            (O(blocks / 64) lane rounds; ~550 splits per friendsforever document) and moves one
//            block's totals across each chunk boundary it passes.  8 bytes per block and 4 per 64
//            blocks instead of 6 per block + 144 per superblock: friendsforever's index takes
//            4.9 KB instead of 6.2 KB, so 32 documents share a CU's 160 KiB instead of 25.
constexpr int IX_HBM = 0, IX_LDS = 1, IX_FLAT = 2;
// Block -> (superblock << 6 | index in its list); flat index: block -> position.  The LDS tiers
// keep it in 16 bits (superblock ids below 1024; positions below 65536).
template <int L> DEV uint32_t opos_of(const Doc &D, uint32_t b) {
    if (L) return D.opos16[b];
    return ix<L>(D.opos + b);
}
template <int L> DEV void set_opos(Doc &D, uint32_t b, uint32_t v) {
    if (L) D.opos16[b] = uint16_t(v);
    else D.opos[b] = v;
}

// ---- navigation ------------------------------------------------------------------------------

template <int L> DEV uint32_t first_block(const Doc &D) {
    if (L == IX_FLAT) return U(D.sbl[0]);
    return U(ix16<L>(D.sbl + size_t(U(ix<L>(D.top)) >> 16) * SBC));
}
// Next block in document order, or NONE.
template <int L> DEV uint32_t next_block(const Doc &D, uint32_t b) {
    if (L == IX_FLAT) {
        const uint32_t p = U(D.opos16[b]) + 1;
        return p < D.nb ? U(D.sbl[p]) : NONE;
    }
    const uint32_t o = U(opos_of<L>(D, b));
    const uint32_t S = o >> 6, i = o & 63u;
    if (i + 1 < U(ix<L>(D.sbn + S))) return U(ix16<L>(D.sbl + size_t(S) * SBC + i + 1));
    const uint32_t p = U(ix<L>(D.sbpos + S)) + 1;
    if (p >= D.nsb) return NONE;
    return U(ix16<L>(D.sbl + size_t(U(ix<L>(D.top + p)) >> 16) * SBC));
}
// Document-order key of (block, slot).
template <int L> DEV uint32_t key_at(const Doc &D, uint32_t b, uint32_t s) {
    if (L == IX_FLAT) return (uint32_t(D.opos16[b]) << 6) | s;
    const uint32_t o = opos_of<L>(D, b);
    return (ix<L>(D.sbpos + (o >> 6)) << 12) | ((o & 63u) << 6) | s;
}
// Slot of `item` in block b, per lane (divergent lanes allowed): the first match in the row.
// Rows are never cleared above their count, so a stale copy of an item can sit there -- but
// only above the live part, and the live copy comes first.
DEV uint32_t find_slot(const Doc &D, uint32_t b, uint32_t item) {
    const uint4 *row = reinterpret_cast<const uint4 *>(D.items + size_t(b) * BLK);
    uint32_t s = BLK;
    for (uint32_t q = 0; q < BLK / 4 && s == BLK; q += 2) {
        uint4 v[2];
#pragma unroll
        for (uint32_t j = 0; j < 2; j++) v[j] = row[q + j];
#pragma unroll
        for (int j = 1; j >= 0; j--) {
            const uint32_t o = 4 * (q + uint32_t(j));
            if (v[j].w == item) s = o + 3;
            if (v[j].z == item) s = o + 2;
            if (v[j].y == item) s = o + 1;
            if (v[j].x == item) s = o;
        }
    }
    return s;
}
// Document-order key of an inserted item, per lane.
template <int L> DEV uint32_t key_of(const Doc &D, uint32_t item) {
    const uint32_t b = pc_blk(ld(D.pc + item));
    return key_at<L>(D, b, find_slot(D, b, item));
}
// Same for a wave-uniform item: one row load and a ballot.
template <int L> DEV uint32_t ukey_of(const Doc &D, uint32_t item) {
    const uint32_t b = U(pc_blk(ld(D.pc + item)));
    const u64 m = BALLOT(D.items[size_t(b) * BLK + lane_id()] == item);
    return U(key_at<L>(D, b, first_lane(m)));
}

// Block holding visible index p and the rank k of that item among the block's visible items
// (content-tree cursor_at_content_pos, root.rs:50-89): prefix scans over superblock totals,
// then over the chosen superblock's block counts.
struct Found {
    uint32_t b, k;     // block, rank of the item among the block's visible items
    uint32_t S, tp;    // its superblock and that superblock's top position
    uint32_t c;        // the block's packed counts (flat index), NONE: not gathered
};
template <int L>
DEV bool find_vis(Doc &D, uint32_t p, Found &f) {
    const uint32_t l = lane_id();
    uint32_t base = 0, S = NONE;
    if (L == IX_FLAT) {   // chunk totals, then the chunk's blocks
        const uint32_t nc = (D.nb + 63) >> 6;
        {   // at most 32 chunks (FLAT_MAX_BLOCKS): one scan over lanes 0..31
            const uint32_t w0 = D.top[min(l, nc - 1)];
            const uint32_t v = l < nc ? (w0 & 0xFFFFu) : 0u;
            const uint32_t inc = wave_scan32(v);
            const u64 m = BALLOT(inc > p) & 0xFFFFFFFFull;
            if (!m) return false;
            S = first_lane(m);
            base = bcast(inc - v, S);
        }
        f.S = f.tp = S;
        const uint32_t q = (S << 6) + l;
        const uint32_t b0 = D.sbl[min(q, D.nb - 1)];
        const uint32_t w = D.cnt[b0];
        const uint32_t b = q < D.nb ? b0 : 0;
        const uint32_t v = q < D.nb ? c_vis(w) : 0;
        const uint32_t inc = wave_scan(v);
        const u64 m = BALLOT(base + inc > p);
        if (!m) return false;
        const uint32_t fl = first_lane(m);
        f.b = U(bcast(b, fl));
        f.k = U(p - base - bcast(inc - v, fl));
        f.c = U(bcast(w, fl));
        return true;
    }
    for (uint32_t c = 0; c < D.nsb; c += 64) {
        const uint32_t i = c + l;
        const uint32_t w0 = ix<L>(D.top + min(i, D.nsb - 1));   // clamped, then masked: no exec branch
        const uint32_t w = i < D.nsb ? w0 : 0;
        const uint32_t v = w & 0xFFFFu;
        const uint32_t inc = wave_scan(v);
        const u64 m = BALLOT(base + inc > p);
        if (m) {
            const uint32_t fl = first_lane(m);
            S = U(bcast(w, fl) >> 16);
            f.tp = U(c + fl);
            base += bcast(inc - v, fl);
            break;
        }
        base += bcast(inc, 63);
    }
    if (S == NONE) return false;
    f.S = S;
    f.c = NONE;
    const uint32_t n = U(ix<L>(D.sbn + S));
    const uint32_t b0 = ix16<L>(D.sbl + size_t(S) * SBC + l);   // a list row holds SBC slots
    const uint32_t b = l < n ? b0 : 0;
    const uint32_t v0 = c_vis(ix<L>(D.cnt + b));
    const uint32_t v = l < n ? v0 : 0;
    const uint32_t inc = wave_scan(v);
    const u64 m = BALLOT(base + inc > p);
    if (!m) return false;
    const uint32_t fl = first_lane(m);
    f.b = U(bcast(b, fl));
    f.k = U(p - base - bcast(inc - v, fl));
    return true;
}

// Slot of the k-th set bit of a wave-uniform mask.
DEV uint32_t select_bit(u64 m, uint32_t k) {
    const uint32_t l = lane_id();
    const bool set = (m >> l) & 1ull;
    const uint32_t before = uint32_t(__popcll(m & lanes_below(l)));
    return first_lane(BALLOT(set && before == k));
}

// First block after b (document order) with a live item, or NONE (origin_right search,
// merge.rs:405-423).
template <int L>
DEV uint32_t next_live_block(Doc &D, uint32_t b) {
    const uint32_t l = lane_id();
    if (L == IX_FLAT) {
        const uint32_t p0 = U(D.opos16[b]) + 1, nc = (D.nb + 63) >> 6;
        uint32_t c = p0 >> 6;
        {   // rest of p0's chunk
            const uint32_t q = (c << 6) + l;
            const uint32_t b0 = D.sbl[min(q, D.nb - 1)];
            const bool in = q >= p0 && q < D.nb;
            const uint32_t bl = in ? b0 : 0;
            const uint32_t cl = c_live(D.cnt[bl]);
            const u64 m = BALLOT(in && cl != 0);
            if (m) return U(bcast(bl, first_lane(m)));
        }
        for (c = c + 1; c < nc; c += 64) {   // later chunks by their live totals
            if (!charge(D)) return NONE;
            const uint32_t i = c + l;
            const uint32_t t = D.top[min(i, nc - 1)] >> 16;
            const u64 m = BALLOT(i < nc && t != 0);
            if (m) {
                const uint32_t q = ((c + first_lane(m)) << 6) + l;
                const uint32_t b0 = D.sbl[min(q, D.nb - 1)];
                const uint32_t bl = q < D.nb ? b0 : 0;
                const uint32_t cl = c_live(D.cnt[bl]);
                const u64 m2 = BALLOT(q < D.nb && cl != 0);
                if (!m2) { fail(D, ErrCheckout, 19); return NONE; }
                return U(bcast(bl, first_lane(m2)));
            }
        }
        return NONE;
    }
    const uint32_t o = U(opos_of<L>(D, b));
    uint32_t S = o >> 6;
    {   // rest of b's superblock
        const uint32_t n = U(ix<L>(D.sbn + S)), i0 = (o & 63u) + 1;
        const uint32_t b0 = ix16<L>(D.sbl + size_t(S) * SBC + l);
        const uint32_t bl = l < n ? b0 : 0;
        const uint32_t cl = c_live(ix<L>(D.cnt + bl));
        const u64 m = BALLOT(l >= i0 && l < n && cl != 0);
        if (m) return U(bcast(bl, first_lane(m)));
    }
    for (uint32_t p = U(ix<L>(D.sbpos + S)) + 1; p < D.nsb; p += 64) {
        if (!charge(D)) return NONE;
        const uint32_t i = p + l;
        const uint32_t tl = ix<L>(D.tlive + min(i, D.nsb - 1));
        const u64 m = BALLOT(i < D.nsb && tl != 0);
        if (m) {
            S = U(ix<L>(D.top + p + first_lane(m)) >> 16);
            const uint32_t n = U(ix<L>(D.sbn + S));
            const uint32_t b0 = ix16<L>(D.sbl + size_t(S) * SBC + l);
            const uint32_t bl = l < n ? b0 : 0;
            const uint32_t cl = c_live(ix<L>(D.cnt + bl));
            const u64 m2 = BALLOT(l < n && cl != 0);
            if (!m2) { fail(D, ErrCheckout, 19); return NONE; }
            return U(bcast(bl, first_lane(m2)));
        }
    }
    return NONE;
}

// ---- block maintenance ---------------------------------------------------------------------

// Split the full superblock S (64 blocks): its upper half becomes a new superblock right after
// it in the top order.
template <int L, bool XF>
DEV void split_sb(Doc &D, uint32_t S) {
    const uint32_t l = lane_id();
    if (D.nsb >= D.max_sb) { fail(D, ErrCapacity, 21); return; }
    const uint32_t S2 = D.nsb;
    uint32_t vis = 0, live = 0, up = 0;
    {
        const uint32_t b = ix16<L>(D.sbl + size_t(S) * SBC + l);
        const uint32_t c = ix<L>(D.cnt + b);
        vis = c_vis(c);
        live = c_live(c);
        up = c_up(c);
        wave_fence();
        if (l >= SBC / 2) {
            D.sbl[size_t(S2) * SBC + (l - SBC / 2)] = uint16_t(b);
            set_opos<L>(D, b, (S2 << 6) | (l - SBC / 2));
        }
    }
    const uint32_t vh = wave_sum(l >= 32 ? vis : 0), lh = wave_sum(l >= 32 ? live : 0);
    const uint32_t vl = wave_sum(l < 32 ? vis : 0), ll = wave_sum(l < 32 ? live : 0);
    const uint32_t uh = XF ? wave_sum(l >= 32 ? up : 0) : 0, ul = XF ? wave_sum(l < 32 ? up : 0) : 0;
    const uint32_t p = U(ix<L>(D.sbpos + S)) + 1;
    // shift top[p .. nsb) / tlive right by one, highest chunk first
    for (int c = int(D.nsb) - 1; c >= int(p); c -= 64) {
        const int i = c - int(l);
        uint32_t w = 0, lv = 0, uv = 0;
        if (i >= int(p)) { w = ix<L>(D.top + i); lv = ix<L>(D.tlive + i); if (XF) uv = ix<L>(D.tup + i); }
        wave_fence();
        if (i >= int(p)) {
            D.top[i + 1] = w; D.tlive[i + 1] = lv; D.sbpos[w >> 16] = uint32_t(i + 1);
            if (XF) D.tup[i + 1] = uv;
        }
        wave_fence();
    }
    if (l == 0) {
        D.sbn[S] = SBC / 2;
        D.sbn[S2] = SBC / 2;
        D.top[p - 1] = (S << 16) | vl; D.tlive[p - 1] = ll;
        D.top[p] = (S2 << 16) | vh; D.tlive[p] = lh;
        D.sbpos[S2] = p;
        if (XF) { D.tup[p - 1] = ul; D.tup[p] = uh; }
    }
    wave_fence();
    D.nsb++;
}

// Split the full block b (items in `it` lane by lane, masks mv / ml) at slot c: items [c, 64)
// move to a new block b2 placed right after b in its superblock.
template <int L, bool XF>
DEV uint32_t split_block(Doc &D, uint32_t b, uint32_t c, uint32_t it, u64 mv, u64 ml) {
    const uint32_t l = lane_id();
    if (D.nb >= D.max_blocks) { fail(D, ErrCapacity, 12); return 0; }
    const uint32_t b2 = D.nb;
    u64 mu = 0, mu_lo = 0, mu_hi = 0;
    if (XF) {
        mu = U64(ld(D.mup + b));
        mu_lo = mu & lanes_below(c);
        mu_hi = c >= 64 ? 0ull : mu >> c;
    }
    if (l >= c) {   // the moved items change block (content-tree's notify on a leaf split)
        D.items[size_t(b2) * BLK + (l - c)] = it;
        st(D.pc + it, (ld(D.pc + it) & 0xFFFF0000u) | b2);
    }
    const u64 lo = lanes_below(c);
    const u64 mv_hi = c >= 64 ? 0ull : mv >> c, ml_hi = c >= 64 ? 0ull : ml >> c;
    if (l < 4) {   // both blocks' mask pairs in one store
        const u64 v = l == 0 ? (mv & lo) : l == 1 ? (ml & lo) : l == 2 ? mv_hi : ml_hi;
        st(D.m2 + 2 * size_t(l < 2 ? b : b2) + (l & 1), v);
    }
    if (L == IX_FLAT) {   // b2 goes to position pos + 1: shift ord[pos + 1, nb) right by one
        const uint32_t pos = U(D.opos16[b]);
        for (int hi = int(D.nb) - 1; hi > int(pos); hi -= 64) {   // highest chunk first
            const int q = hi - int(l);
            const bool mvl = q > int(pos);
            uint32_t v = 0;
            if (mvl) v = D.sbl[q];
            wave_fence();
            if (mvl) {
                D.sbl[q + 1] = uint16_t(v);
                D.opos16[v] = uint16_t(q + 1);
                if (((q + 1) & 63) == 0) {   // v crosses into the next chunk: move its totals
                    const uint32_t cv = D.cnt[v];
                    const uint32_t w = c_vis(cv) | (c_live(cv) << 16);
                    at_add(D.top + (uint32_t(q) >> 6), 0u - w);
                    at_add(D.top + (uint32_t(q + 1) >> 6), w);
                }
            }
            wave_fence();
        }
        if (l == 0) {
            const uint32_t v2 = uint32_t(__popcll(mv_hi)), l2 = uint32_t(__popcll(ml_hi));
            D.cnt[b2] = v2 * C_VIS + l2 * C_LIVE + (BLK - c) * C_ITEMS;
            D.cnt[b] = uint32_t(__popcll(mv & lo)) * C_VIS + uint32_t(__popcll(ml & lo)) * C_LIVE + c * C_ITEMS;
            D.sbl[pos + 1] = uint16_t(b2);
            D.opos16[b2] = uint16_t(pos + 1);
            if (((pos + 1) & 63) == 0) {   // b2's items leave b's chunk
                const uint32_t w = v2 | (l2 << 16);
                at_add(D.top + (pos >> 6), 0u - w);
                at_add(D.top + ((pos + 1) >> 6), w);
            }
        }
        wave_fence();
        D.nb++;
        return b2;
    }
    const uint32_t o = U(opos_of<L>(D, b));
    const uint32_t S = o >> 6, i = o & 63u, n = U(ix<L>(D.sbn + S));
    {   // shift S's list after i right by one
        uint32_t v = 0;
        const bool mv_lane = l > i && l < n;
        if (mv_lane) v = ix16<L>(D.sbl + size_t(S) * SBC + l);
        wave_fence();
        if (mv_lane) {
            D.sbl[size_t(S) * SBC + l + 1] = uint16_t(v);
            set_opos<L>(D, v, (S << 6) | (l + 1));
        }
    }
    if (l == 0) {
        D.cnt[b2] = uint32_t(__popcll(mv_hi)) * C_VIS + uint32_t(__popcll(ml_hi)) * C_LIVE + (BLK - c) * C_ITEMS +
                    uint32_t(__popcll(mu_hi)) * C_UP;
        D.cnt[b] = uint32_t(__popcll(mv & lo)) * C_VIS + uint32_t(__popcll(ml & lo)) * C_LIVE + c * C_ITEMS +
                   uint32_t(__popcll(mu_lo)) * C_UP;
        if (XF) { st(D.mup + b, mu_lo); st(D.mup + b2, mu_hi); }
        D.sbl[size_t(S) * SBC + i + 1] = uint16_t(b2);
        set_opos<L>(D, b2, (S << 6) | (i + 1));
        D.sbn[S] = n + 1;
    }
    wave_fence();
    D.nb++;
    if (n + 1 == SBC) split_sb<L, XF>(D, S);
    return b2;
}

// Cut point for splitting a full block that receives an insert at slot s.  The LDS tier cuts
// at the insert point clamped to [16, 48]: an edit inside a block leaves the text after the
// cursor in one block and the typing room in the other, so blocks end up ~43 items full on
// the benchmark traces instead of ~35 (tools/blocksim.py measured the policies).  Its
// capacity is sized for that fill; a document that still outgrows it is handed to the HBM
// tier, which always cuts at the midpoint so every block keeps >= 32 items and
// n_ins / 32 + 2 blocks suffice.
template <int L> DEV uint32_t cut_point(uint32_t s) { return L ? min(max(s, 16u), 48u) : BLK / 2; }

// Transformed-ops mode: the upstream position of slot s of block b -- the never-deleted items
// before it in document order (MarkerMetrics upstream_len, metrics.rs:18-66; the position
// integrate() / apply() report as BaseMoved, merge.rs:154-278, 457-556).
template <int L>
DEV uint32_t up_rank(Doc &D, uint32_t b, uint32_t s) {
    const uint32_t l = lane_id();
    const uint32_t o = U(opos_of<L>(D, b));
    const uint32_t S = o >> 6, i = o & 63u, tp = U(ix<L>(D.sbpos + S));
    uint32_t r = 0;
    for (uint32_t c = 0; c < tp; c += 64) r += wave_sum(c + l < tp ? ix<L>(D.tup + c + l) : 0u);
    const uint32_t bl = l < i ? ix16<L>(D.sbl + size_t(S) * SBC + l) : 0;
    r += wave_sum(l < i ? c_up(ix<L>(D.cnt + bl)) : 0u);
    r += uint32_t(__popcll(U64(ld(D.mup + b)) & lanes_below(s)));
    return U(r);
}

// Insert the run [lv, lv+k) before slot s of block b (all new items visible).  `it` holds the
// block's items lane by lane (lanes >= the block count are don't-care); mv / ml its masks.
template <int L, bool PROF, bool XF>
DEV void insert_run(Doc &D, uint32_t b, uint32_t s, uint32_t it, u64 mv, u64 ml, uint32_t lv, uint32_t k,
                    uint32_t ol, uint32_t orr, uint32_t tph, uint32_t c_in) {
    D.cb = NONE;
    const uint32_t l = lane_id();
    const uint32_t lv0 = lv, k0 = k;
    if (XF) {   // the run's items land at consecutive upstream positions
        const uint32_t r0 = up_rank<L>(D, b, s);
        for (uint32_t j = l; j < k0; j += 64) D.xf[lv0 + j] = r0 + j;
    }
    if (!XF && c_in != NONE && c_items(c_in) + k <= BLK) {
        // the common case as straight-line code: the run fits the block (no split, one round)
        const uint32_t shifted = shfl(it, l >= k ? l - k : l);
        it = l < s ? it : (l < s + k ? lv + (l - s) : shifted);
        D.items[size_t(b) * BLK + l] = it;
        if (l >= s && l < s + k) st(D.pc + it, pc_of(b, 1u));
        const u64 low = lanes_below(s);
        const u64 ins = lanes_below(k) << s;
        mv = k == 64 ? ins : ((mv & low) | ((mv & ~low) << k) | ins);
        ml = k == 64 ? ins : ((ml & low) | ((ml & ~low) << k) | ins);
        st(D.m2 + 2 * size_t(b) + (l & 1u), (l & 1u) ? ml : mv);
        if (tph == NONE) tph = L == IX_FLAT ? U(uint32_t(D.opos16[b]) >> 6) : U(ix<L>(D.sbpos + (opos_of<L>(D, b) >> 6)));
        if (l == 0) {
            D.cnt[b] = c_in + k * (C_VIS + C_LIVE + C_ITEMS);
            if (L == IX_FLAT) {
                at_add(D.top + tph, k | (k << 16));
            } else {
                at_add(D.top + tph, k);
                at_add(D.tlive + tph, k);
            }
        }
        if (l < k) D.ao[lv + l] = u64(l == 0 ? ol : lv + l - 1) | (u64(orr) << 32);
        wave_fence();
        D.cb = b; D.cit = it; D.cmv = mv; D.cml = ml;
        return;
    }
    while (k > 0) {   // each round inserts >= 1 item or splits (bounded by max_blocks)
        // b's packed counts: the caller's clean copy on the first round, reloaded after a split
        const uint32_t c = c_in != NONE ? c_in : U(ix<L>(D.cnt + b));
        c_in = NONE;
        const uint32_t bc = c_items(c);
        if (bc == BLK) {
            const uint64_t t0 = tick<PROF>();
            const uint32_t cut = cut_point<L>(s);
            const uint32_t b2 = split_block<L, XF>(D, b, cut, it, mv, ml);
            if (D.err) return;
            tph = NONE;   // a split may move superblocks in the top order
            if (s > cut || cut == BLK) {
                b = b2;
                s -= cut;
                it = shfl(it, (l + cut) & 63u);
                mv = cut >= 64 ? 0ull : mv >> cut;
                ml = cut >= 64 ? 0ull : ml >> cut;
            } else {
                mv &= lanes_below(cut);
                ml &= lanes_below(cut);
            }
            if (PROF) { D.prof[P_SPLIT] += tick<PROF>() - t0; D.prof[P_N_SPLIT]++; }
            continue;
        }
        uint64_t tr = tick<PROF>();
        const uint32_t m = min(k, BLK - bc);
        uint32_t *items = D.items + size_t(b) * BLK;
        // the block after the insert, lane = slot: the row from the insert point on is written
        // with one store; only the new items get a block in pos[] (shifted ones stay put)
        const uint32_t shifted = shfl(it, l >= m ? l - m : l);
        it = l < s ? it : (l < s + m ? lv + (l - s) : shifted);
        items[l] = it;   // the whole row: slots past the count are don't-care
        if (l >= s && l < s + m) st(D.pc + it, pc_of(b, 1u));
        if (PROF) { const uint64_t t = tick<PROF>(); D.prof[P_R1] += t - tr; tr = t; }
        const u64 low = lanes_below(s);
        const u64 ins = lanes_below(m) << s;
        mv = m == 64 ? ins : ((mv & low) | ((mv & ~low) << m) | ins);
        ml = m == 64 ? ins : ((ml & low) | ((ml & ~low) << m) | ins);
        st(D.m2 + 2 * size_t(b) + (l & 1u), (l & 1u) ? ml : mv);   // every lane: no exec branch
        if (XF) {
            u64 mu = U64(ld(D.mup + b));
            mu = m == 64 ? ins : ((mu & low) | ((mu & ~low) << m) | ins);
            if (l == 0) st(D.mup + b, mu);
        }
        if (tph == NONE) tph = L == IX_FLAT ? U(uint32_t(D.opos16[b]) >> 6) : U(ix<L>(D.sbpos + (opos_of<L>(D, b) >> 6)));
        if (l == 0) {   // the superblock's totals by atomic add: no dependent read
            D.cnt[b] = c + m * (C_VIS + C_LIVE + C_ITEMS + (XF ? C_UP : 0u));
            const uint32_t tp = tph;
            if (L == IX_FLAT) {
                at_add(D.top + tp, m | (m << 16));
            } else {
                at_add(D.top + tp, m);
                at_add(D.tlive + tp, m);
            }
            if (XF) at_add(D.tup + tp, m);
        }
        wave_fence();
        if (PROF) { const uint64_t t = tick<PROF>(); D.prof[P_R2] += t - tr; tr = t; }
        lv += m;
        k -= m;
        s += m;
    }
    D.cb = b; D.cit = it; D.cmv = mv; D.cml = ml;   // block state after the run
    const uint64_t t3 = tick<PROF>();
    for (uint32_t j0 = 0; j0 < k0; j0 += 64) {   // wave-uniform loop, masked store
        const uint32_t j = j0 + l, nit = lv0 + j;
        if (j < k0) D.ao[nit] = u64(j == 0 ? ol : nit - 1) | (u64(orr) << 32);
    }
    if (PROF) D.prof[P_R3] += tick<PROF>() - t3;
}

// YjsMod tie-break key of an LV: (agent name rank, seq) (merge.rs:199-218).  64-ary search
// over the agent runs; `lv` is wave-uniform.
DEV void agent_of(Doc &D, uint32_t lv, uint32_t &rank, uint32_t &seq) {
    const uint32_t l = lane_id();
    const GLOBAL_AS uint32_t *aruns = gp(vld(&KP().aruns)) + U(uint32_t(vld(&D.desc->arun_off)));
    uint32_t lo = 0, n = U(vld(&D.desc->n_aruns));   // last run with start <= lv lies in [lo, lo+n)
    while (n > 64) {
        if (!charge(D)) { rank = seq = 0; return; }
        const uint32_t stride = (n + 63) / 64;
        const uint32_t idx = lo + l * stride;
        const bool ok = l * stride < n && aruns[4 * idx] <= lv;
        const uint32_t k = uint32_t(__popcll(BALLOT(ok)));
        const uint32_t nlo = lo + (k ? k - 1 : 0) * stride;
        n = min(stride, lo + n - nlo);
        lo = nlo;
    }
    const bool ok = l < n && aruns[4 * (lo + l)] <= lv;
    const uint32_t k = uint32_t(__popcll(BALLOT(ok)));
    const uint32_t j = U(lo + (k ? k - 1 : 0));
    rank = U(aruns[4 * j + 1]);
    seq = U(aruns[4 * j + 2]) + (lv - U(aruns[4 * j]));
}

// YjsMod integrate (merge.rs:154-278) over the not-inserted-yet items between the cursor
// (b, s) and origin_right (rb, rs) (rb == NONE: END), one block of candidates at a time.
// Every candidate's keys come in lane-parallel; the sequential scan state machine is resolved
// with ballots: the first stopping lane ends the scan, and `scanning` is the state after the
// last event lane before it.  Returns the insertion point in (b, s).
template <int L>
DEV void yjs_scan(Doc &D, uint32_t &b, uint32_t &s, uint32_t rb, uint32_t rs, uint32_t my_l, uint32_t my_r,
                  uint32_t ol_new, uint32_t orr_new, uint32_t lv) {
    const uint32_t l = lane_id();
    uint32_t new_rank, new_seq;
    agent_of(D, lv, new_rank, new_seq);
    bool scanning = false;
    uint32_t st_b = 0, st_s = 0;
    uint32_t cb = b, cs = s;
    for (;;) {
        if (!charge(D)) return;
        const uint32_t cnt = c_items(U(ix<L>(D.cnt + cb)));
        if (cs >= cnt) {   // next block in document order
            const uint32_t nx = next_block<L>(D, cb);
            if (nx == NONE) break;   // end of document
            cb = nx;
            cs = 0;
            continue;
        }
        const uint32_t end = cb == rb ? rs : cnt;
        if (cs >= end) break;   // reached origin_right
        const bool inr = l >= cs && l < end;
        const uint32_t o = l < cnt ? D.items[size_t(cb) * BLK + l] : 0;
        uint32_t ol_o = ROOT_ID, orr_o = END_ID;
        if (inr) {
            const u64 x = D.ao[o];
            ol_o = uint32_t(x);
            orr_o = uint32_t(x >> 32);
        }
        // kl = key(origin_left) + 1 against my_l.  Without a key lookup when the candidate's
        // origin_left is mine (equal), ROOT (0), or the candidate just before it in the scanned
        // range (after the cursor, so after my origin_left: greater) -- concurrent typing
        // (merge.rs:199-243 compares cursor positions; the same order).
        const uint32_t prev = shfl(o, (l - 1) & 63u);
        const bool l_eq = ol_o == ol_new, l_root = ol_o == ROOT_ID;
        const bool l_gt = !l_eq && !l_root && l > cs && ol_o == prev;
        uint32_t kl = l_eq ? my_l : (l_root ? 0u : (l_gt ? my_l + 1u : 0u));
        if (BALLOT(inr && !l_eq && !l_root && !l_gt)) {
            if (inr && !l_eq && !l_root && !l_gt) kl = key_of<L>(D, ol_o) + 1u;
        }
        // kr = key(origin_right): only where the scan state machine reads it
        uint32_t kr = 0xFFFFFFFFu;
        const bool need_r = inr && kl == my_l && orr_o != orr_new && orr_o != END_ID;
        if (BALLOT(need_r)) {
            if (need_r) kr = key_of<L>(D, orr_o);
        }
        const bool tie = inr && kl == my_l && orr_o == orr_new;
        bool new_lt = false;
        for (u64 mt = BALLOT(tie); mt; mt &= mt - 1) {
            const uint32_t f = first_lane(mt);
            uint32_t r2, s2;
            agent_of(D, U(bcast(o, f)), r2, s2);
            const bool lt = new_rank < r2 || (new_rank == r2 && new_seq < s2);
            if (l == f) new_lt = lt;
        }
        const bool stop = inr && (kl < my_l || (tie && new_lt));
        const bool setv = inr && kl == my_l && orr_o != orr_new && kr < my_r;
        const bool clr = inr && kl == my_l && !stop && !setv;
        const u64 ms = BALLOT(stop);
        const uint32_t lim = ms ? first_lane(ms) : end;
        const u64 below = lanes_below(lim);
        const u64 mset = BALLOT(setv) & below, mclr = BALLOT(clr) & below;
        if (mset | mclr) {
            const int lc = mclr ? int(last_lane(mclr)) : -1;
            const int ls = mset ? int(last_lane(mset)) : -1;
            if (ls > lc) {
                const u64 after = lc >= 0 ? (mset & ~((2ull << lc) - 1ull)) : mset;
                if (lc >= 0 || !scanning) { scanning = true; st_b = cb; st_s = first_lane(after); }
            } else {
                scanning = false;
            }
        }
        cs = lim;
        if (ms) break;
    }
    if (scanning) { b = st_b; s = st_s; }
    else { b = cb; s = cs; }
    b = U(b);
    s = U(s);
}

// Items and masks of block b (packed count c) into registers: items lane by lane, masks
// wave-uniform.  A block whose masks a retreat/advance pass invalidated (DIRTY) gets them
// rebuilt from the items' counts and stored back clean.
template <int L, bool PROF = false>
DEV void load_block(Doc &D, uint32_t b, uint32_t c, uint32_t &it, u64 &mv, u64 &ml) {
    const uint32_t l = lane_id();
    const uint32_t bc = c_items(c);
    if (PROF) { D.prof[P_N_LOAD]++; if (c & C_DIRTY) D.prof[P_N_DIRTY]++; }
    const uint32_t it0 = D.items[size_t(b) * BLK + l];   // the row holds BLK slots
    it = l < bc ? it0 : 0;
    if (c & C_DIRTY) {
        const uint32_t k = pc_cnt(ld(D.pc + it));   // lanes past the count read item 0's word
        mv = BALLOT(l < bc && k == 1u);
        ml = BALLOT(l < bc && k != 0u);
        st(D.m2 + 2 * size_t(b) + (l & 1u), (l & 1u) ? ml : mv);
        if (l == 0) D.cnt[b] = c & ~C_DIRTY;
        wave_fence();
    } else {
        const u64 x = ld(D.m2 + 2 * size_t(b) + (l & 1u));
        mv = bcast64(x, 0);
        ml = bcast64(x, 1);
    }
}

// Apply an insert run at visible position pos (M2Tracker::apply Ins + integrate,
// merge.rs:154-278, 383-455).
template <int L, bool PROF, bool XF>
DEV void do_insert(Doc &D, uint32_t lv, uint32_t k, uint32_t pos) {
    uint64_t tp = tick<PROF>();
    uint32_t b, kk = 0, tph = 0;   // tph: top position of b's superblock (first block: 0)
    uint32_t fcnt = NONE;          // b's packed counts when the lookup gathered them
    if (pos == 0) {
        b = first_block<L>(D);
    } else {
        Found f;
        if (!find_vis<L>(D, pos - 1, f)) { fail(D, ErrCheckout, 13); return; }
        b = f.b;
        kk = f.k;
        tph = f.tp;
        fcnt = f.c;
    }
    if (PROF) { const uint64_t t = tick<PROF>(); D.prof[P_FIND] += t - tp; tp = t; }
    const uint32_t c0 = L == IX_FLAT && fcnt != NONE ? fcnt : U(ix<L>(D.cnt + b));
    const uint32_t bc = c_items(c0);
    uint32_t cb = c0 & ~C_DIRTY;   // b's packed counts once its masks are current
    uint32_t it;
    u64 mv, ml;
    if (b == D.cb) { it = D.cit; mv = D.cmv; ml = D.cml; }
    else load_block<L, PROF>(D, b, c0, it, mv, ml);
    uint32_t s = 0, ol = ROOT_ID;
    if (pos) {
        const uint32_t s0 = select_bit(mv, kk);
        if (s0 >= bc) { fail(D, ErrCheckout, 13); return; }
        ol = U(bcast(it, s0));
        s = s0 + 1;
    }
    if (PROF) { const uint64_t t = tick<PROF>(); D.prof[P_BLOAD] += t - tp; tp = t; }
    // origin_right: first live item at or after the cursor (possibly a deleted one)
    const u64 mlr = s >= 64 ? 0ull : (ml & (~0ull << s));
    uint32_t rb, rs, orr;
    bool direct;
    if (mlr) {
        rb = b;
        rs = first_lane(mlr);
        orr = U(bcast(it, rs));
        direct = rs == s;
    } else {
        rb = next_live_block<L>(D, b);
        if (D.err) return;
        if (rb != NONE) {
            uint32_t rit;
            u64 rmv, rml;
            load_block<L, PROF>(D, rb, U(ix<L>(D.cnt + rb)), rit, rmv, rml);
            rs = first_lane(rml);
            orr = U(bcast(rit, rs));
        } else {
            rs = 0;
            orr = END_ID;
        }
        // direct iff no item lies between the cursor and origin_right
        if (s < bc) direct = false;
        else {
            const uint32_t nx = next_block<L>(D, b);
            direct = nx == NONE || (rb == nx && rs == 0);
        }
    }
    if (PROF) { const uint64_t t = tick<PROF>(); D.prof[P_ORR] += t - tp; tp = t; }
    if (!direct) {
        const uint32_t my_l = ol == ROOT_ID ? 0u : ukey_of<L>(D, ol) + 1u;
        const uint32_t my_r = orr == END_ID ? 0xFFFFFFFFu : ukey_of<L>(D, orr);
        const uint32_t b0 = b;
        yjs_scan<L>(D, b, s, rb, rs, my_l, my_r, ol, orr, lv);
        if (D.err) return;
        if (b != b0) {
            cb = U(ix<L>(D.cnt + b));
            if (b == D.cb) { it = D.cit; mv = D.cmv; ml = D.cml; }
            else load_block<L, PROF>(D, b, cb, it, mv, ml);
            cb &= ~C_DIRTY;
            tph = NONE;
        }
        if (PROF) { const uint64_t t = tick<PROF>(); D.prof[P_YJS] += t - tp; tp = t; D.prof[P_N_YJS]++; }
    }
    const uint64_t sp0 = PROF ? D.prof[P_SPLIT] : 0;
    insert_run<L, PROF, XF>(D, b, s, it, mv, ml, lv, k, ol, orr, tph, cb);
    if (PROF) D.prof[P_RUN] += tick<PROF>() - tp - (D.prof[P_SPLIT] - sp0);
}

// Apply a delete run: n visible items from position pos (merge.rs:457-556).  LV lv+j targets
// the j-th item (fwd) or the (n-1-j)-th item (reversed / backspace runs, op_metrics.rs:184-202).
template <int L, bool PROF, bool XF>
DEV void do_delete(Doc &D, uint32_t lv, uint32_t n, uint32_t pos, bool fwd) {
    const uint32_t l = lane_id();
    uint32_t j0 = 0;
    uint32_t up_done = 0;   // XF: never-deleted items this run deleted in earlier (left) blocks
    while (j0 < n) {   // each round deletes >= 1 item or fails
        Found f;
        if (!find_vis<L>(D, pos, f)) { fail(D, ErrCheckout, 14); return; }
        const uint32_t b = f.b, kk = f.k, tpos = f.tp;
        const uint32_t c0 = L == IX_FLAT && f.c != NONE ? f.c : U(ix<L>(D.cnt + b));
        uint32_t it;
        u64 mv, ml;
        if (b == D.cb) { it = D.cit; mv = D.cmv; ml = D.cml; }
        else load_block<L, PROF>(D, b, c0, it, mv, ml);
        const uint32_t c = c0 & ~C_DIRTY;   // load_block left the block clean
        const uint32_t avail = c_vis(c) - kk;
        const uint32_t take = min(avail, n - j0);
        const uint32_t r = uint32_t(__popcll(mv & lanes_below(l)));
        const bool sel = ((mv >> l) & 1ull) && r >= kk && r < kk + take;
        const u64 selm = BALLOT(sel);
        if (uint32_t(__popcll(selm)) != take || take == 0) { fail(D, ErrCheckout, 15); return; }
        u64 mu = 0;
        uint32_t base = 0;
        if (XF) {
            mu = U64(ld(D.mup + b));
            base = up_rank<L>(D, b, 0);
        }
        if (sel) {
            const uint32_t j = j0 + (r - kk);
            const uint32_t dlv = fwd ? lv + j : lv + n - 1 - j;
            st(D.pc + it, pc_of(b, 2u));   // visible (count 1) -> deleted once
            *reinterpret_cast<uint32_t *>(D.ao + dlv) = it;
            if (XF) {
                // LV order applies a forward run left to right (the run's items to the left are
                // already gone) and a backspace run right to left (the ones to the left, in
                // this block and in earlier blocks, are still there)
                const u64 below = lanes_below(l);
                const uint32_t x = fwd ? base + uint32_t(__popcll(mu & ~selm & below))
                                       : base + uint32_t(__popcll(mu & below)) + up_done;
                D.xf[dlv] = ((mu >> l) & 1ull) ? x : NONE;   // NONE: DeleteAlreadyHappened
            }
        }
        const uint32_t gone = XF ? uint32_t(__popcll(mu & selm)) : 0u;   // never-deleted items deleted now
        up_done += gone;
        if (l == 0) {
            st(D.m2 + 2 * size_t(b), mv & ~selm);
            D.cnt[b] = c - take * C_VIS - gone * C_UP;
            at_add(D.top + tpos, 0u - take);
            if (XF) {
                st(D.mup + b, mu & ~selm);
                D.tup[tpos] = ix<L>(D.tup + tpos) - gone;
            }
        }
        wave_fence();
        D.cb = b; D.cit = it; D.cmv = mv & ~selm; D.cml = ml;
        j0 += take;
    }
}

// One walk step's retreat + advance set (advance_retreat.rs:58-153), lane-parallel.
// Entry: LV | is_del << 30 | advance << 31.
// `pre` is the first 64-entry chunk when the caller prefetched it (have_pre).
// Counts change with plain loads and stores (the wave owns the document): lanes that touch the
// same item -- only a deleted item can be touched twice (two deletes of it, or a delete and its
// own insert) -- are merged first.  Blocks whose visibility / liveness changed are marked
// DIRTY; their masks are rebuilt when a command next loads them.
template <int L, bool PROF>
DEV void toggle_pass(Doc &D, uint32_t off, uint32_t n, uint32_t pre, bool have_pre) {
    const uint32_t l = lane_id();
    uint64_t tq = tick<PROF>();
    // Software pipeline over the 64-entry chunks: the entry list and the delete targets are
    // read-only here, so chunk j + 1's entries and targets are fetched while chunk j's counts
    // are read and written; the counts themselves are read only after the previous chunk's
    // stores (same-address order within the wave), so a later chunk sees earlier updates.
    // (loads are issued by every lane at clamped addresses and masked after: no exec branches;
    // a lane with no delete target reads ao[0], one line for the whole wave)
    auto resolve = [&](uint32_t j, uint32_t e, uint32_t &item, bool &del, bool &bad) {
        const bool valid = j + l < n;
        const uint32_t lv = e & 0x3FFFFFFFu;
        bad = valid && lv >= D.n_lv;
        del = valid && !bad && ((e >> 30) & 1u);
        const uint32_t tgt = *reinterpret_cast<const uint32_t *>(D.ao + (del ? lv : 0u));
        item = valid ? (del ? tgt : lv) : 0u;
    };
    if (n == 0) return;
    const uint32_t last = off + n - 1;
    uint32_t e_cur = have_pre ? pre : D.tlist[min(off + l, last)];
    uint32_t e_nx = 0;
    if (n > 64) e_nx = D.tlist[min(off + 64 + l, last)];
    uint32_t it_cur;
    bool del_cur, bad_cur;
    resolve(0, e_cur, it_cur, del_cur, bad_cur);
    for (uint32_t j = 0; j < n; j += 64) {
        // (an invalid lane's item is 0 < n_lv; the deltas are arithmetic on the advance bit, so
        // no divergent block)
        bool bad = bad_cur || it_cur >= D.n_lv;
        bool act = j + l < n && !bad;
        const bool del = del_cur;
        const uint32_t item = it_cur;
        int32_t d = int32_t((e_cur >> 31) << 1) - 1;   // net delta (+1 advance, -1 retreat)
        int32_t dneg = int32_t(e_cur >> 31) - 1;       // sum of the retreats (applied first)
        // the next chunk's targets and the one after's entries, in flight behind this chunk
        if (j + 64 < n) {
            e_cur = e_nx;
            resolve(j + 64, e_cur, it_cur, del_cur, bad_cur);
            e_nx = D.tlist[min(off + j + 128 + l, last)];
        }
        if (BALLOT(bad)) { fail(D, ErrCheckout, 16); return; }
        if (PROF) { const uint64_t t = tick<PROF>(); D.prof[P_T1] += t - tq; tq = t; }
        // lanes whose item another lane also touches: every lane's item against every other
        // lane's (63 lane rotations, four independent chains); only those go through the merge
        // (a few delete lanes: the merge loop over them is cheaper than the rotations)
        const u64 dmask = BALLOT(act && del);
        bool dup = del;
        if (__popcll(dmask) > 4) {
            dup = false;
            // (a running min of xors: equality tests OR-ed as lane masks would each be a scalar op)
            const uint32_t x = act ? item : (0x80000000u | l);   // inactive lanes never match
            uint32_t r0 = x, r1 = shfl(x, (l + 16) & 63u), r2 = shfl(x, (l + 32) & 63u), r3 = shfl(x, (l + 48) & 63u);
            uint32_t mn = min(min(r1 ^ x, r2 ^ x), r3 ^ x);
#pragma unroll
            for (int k = 1; k < 16; k++) {
                r0 = uint32_t(__builtin_amdgcn_mov_dpp(int(r0), 0x13C, 0xF, 0xF, false));   // wave_ror:1
                r1 = uint32_t(__builtin_amdgcn_mov_dpp(int(r1), 0x13C, 0xF, 0xF, false));
                r2 = uint32_t(__builtin_amdgcn_mov_dpp(int(r2), 0x13C, 0xF, 0xF, false));
                r3 = uint32_t(__builtin_amdgcn_mov_dpp(int(r3), 0x13C, 0xF, 0xF, false));
                mn = min(mn, min(min(r0 ^ x, r1 ^ x), min(r2 ^ x, r3 ^ x)));
            }
            dup = mn == 0u;
        }
        for (u64 dm = BALLOT(act && dup); dm;) {   // each round retires >= 1 lane
            const uint32_t t = bcast(item, first_lane(dm));
            const u64 same = BALLOT(act && item == t);
            if (__popcll(same) > 1) {
                const bool mine = (same >> l) & 1ull;
                const int32_t sum = int32_t(wave_sum(mine ? uint32_t(d) : 0u));
                const int32_t neg = int32_t(wave_sum(mine ? uint32_t(dneg) : 0u));
                if (mine) {
                    if (l == first_lane(same)) { d = sum; dneg = neg; }
                    else act = false;
                }
            }
            dm &= ~same;
        }
        bool fv = false, fl = false;
        uint32_t b = 0;
        int32_t dv = 0, dl = 0;
        {   // every lane loads (inactive ones item 0's word); only the store is masked
            const uint32_t w = ld(D.pc + (act ? item : 0u));
            const uint32_t bw = pc_blk(w), oc = pc_cnt(w), nc = oc + uint32_t(d);
            // oc + dneg < 0, oc + d > 0xFFFF or a block past the count: one sign test
            const bool badc = act && int32_t((oc + uint32_t(dneg)) | (0xFFFFu - nc) | (D.nb - 1u - bw)) < 0;
            const bool ok = act && !badc;
            bad = bad || badc;
            if (ok) st(D.pc + item, pc_of(bw, nc));
            b = ok ? bw : 0u;
            fv = ok && ((oc == 1) != (nc == 1));
            fl = ok && ((oc != 0) != (nc != 0));
            dv = fv ? (nc == 1 ? 1 : -1) : 0;
            dl = fl ? (nc != 0 ? 1 : -1) : 0;
        }
        if (BALLOT(bad)) { fail(D, ErrCheckout, 16); return; }
        const bool flip = fv || fl;
        if (BALLOT(flip && b == D.cb)) D.cb = NONE;
        if (PROF) { const uint64_t t = tick<PROF>(); D.prof[P_T2] += t - tq; tq = t; }
        if (L == IX_FLAT) {   // flat LDS index: the chunk's packed totals in one atomic
            if (flip) {
                at_add(D.top + (uint32_t(D.opos16[b]) >> 6), uint32_t(dv) + (uint32_t(dl) << 16));
                at_add(D.cnt + b, uint32_t(dv) * C_VIS + uint32_t(dl) * C_LIVE);
                at_or(D.cnt + b, C_DIRTY);
            }
        } else if (L) {   // LDS index: per-lane LDS atomics
            if (flip) {
                const uint32_t tp = ix<L>(D.sbpos + (opos_of<L>(D, b) >> 6));
                if (fv) at_add(D.top + tp, uint32_t(dv));
                if (fl) at_add(D.tlive + tp, uint32_t(dl));
                at_add(D.cnt + b, uint32_t(dv) * C_VIS + uint32_t(dl) * C_LIVE);
                at_or(D.cnt + b, C_DIRTY);
            }
        } else {   // HBM index: one atomic per distinct block (a global atomic is a memory-side request)
            for (u64 pend = BALLOT(flip); pend;) {   // each round retires >= 1 lane
                const uint32_t f = first_lane(pend);
                const uint32_t bb = bcast(b, f);
                const u64 same = BALLOT(flip && b == bb);
                const bool mine = (same >> l) & 1ull;
                const uint32_t sv = wave_sum(mine ? uint32_t(dv) : 0u), sl = wave_sum(mine ? uint32_t(dl) : 0u);
                if (l == f) {
                    const uint32_t tp = ix<L>(D.sbpos + (opos_of<L>(D, bb) >> 6));
                    if (sv) at_add(D.top + tp, sv);
                    if (sl) at_add(D.tlive + tp, sl);
                    at_add(D.cnt + bb, sv * C_VIS + sl * C_LIVE);
                    at_or(D.cnt + bb, C_DIRTY);
                }
                pend &= ~same;
            }
        }
        if (PROF) { const uint64_t t = tick<PROF>(); D.prof[P_T3] += t - tq; tq = t; }
    }
    wave_fence();
}

// Multi-wave retreat / advance pass (the big LDS tiers' workgroups have TOG_WAVES waves; the
// first replays, the others wait at a barrier until a long pass is posted).  The counters make
// the pass order-free (see toggle_pass), so the waves take 64-entry chunks round robin and
// change each item's count with one returning atomic: its visibility / liveness transition is
// read off the old and new count of that atomic, and the transitions of an item touched twice
// telescope to its net change whatever the interleaving (a count may pass through "-1"
// transiently; the block and superblock counts are modular sums and end exact).
#ifndef DTGPU_TOG_WAVES
#define DTGPU_TOG_WAVES 4
#endif
#ifndef DTGPU_TOG_MW_MIN
#define DTGPU_TOG_MW_MIN 512
#endif
constexpr uint32_t TOG_WAVES = DTGPU_TOG_WAVES;
constexpr uint32_t TOG_MW_MIN = DTGPU_TOG_MW_MIN;   // entries: shorter passes stay on the replay wave
__shared__ uint32_t tog_job[4];        // {off, n, go (0: the document is done), error}
template <int L>
DEV void toggle_chunks(Doc &D, uint32_t off, uint32_t n, uint32_t w0) {
    const uint32_t l = lane_id();
    uint32_t err = 0;
    // the next chunk's entries and delete targets are fetched before this chunk's atomics
    auto fetch = [&](uint32_t j, uint32_t &e, uint32_t &tgt) {
        e = D.tlist[off + min(j + l, n - 1)];
        const uint32_t lv = e & 0x3FFFFFFFu;
        const bool del = j + l < n && ((e >> 30) & 1u) && lv < D.n_lv;
        tgt = *reinterpret_cast<const uint32_t *>(D.ao + (del ? lv : 0u));
    };
    uint32_t e = 0, tgt = 0;
    if (w0 * 64 < n) fetch(w0 * 64, e, tgt);
    for (uint32_t j = w0 * 64; j < n; j += TOG_WAVES * 64) {
        const bool valid = j + l < n;
        const uint32_t lv = e & 0x3FFFFFFFu;
        const bool del = valid && ((e >> 30) & 1u) && lv < D.n_lv;
        const uint32_t item = del ? tgt : lv;
        const bool act = valid && lv < D.n_lv && item < D.n_lv;
        if (valid && !act) err = 1;
        const uint32_t d = (e >> 31) ? 1u : 0xFFFFu;   // +1 / -1 in the 16-bit count field
        if (j + TOG_WAVES * 64 < n) fetch(j + TOG_WAVES * 64, e, tgt);
        uint32_t old = 0;
        if (act) old = __hip_atomic_fetch_add(D.pc + item, d << 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t oc = old >> 16, nc = (oc + d) & 0xFFFFu, b = old & 0xFFFFu;
        const bool fv = act && ((oc == 1) != (nc == 1)), fl = act && ((oc != 0) != (nc != 0));
        if (fv || fl) {
            const uint32_t dv = fv ? (nc == 1 ? 1u : 0xFFFFFFFFu) : 0u, dl = fl ? (nc != 0 ? 1u : 0xFFFFFFFFu) : 0u;
            if (L == IX_FLAT) {
                at_add(D.top + (uint32_t(D.opos16[b]) >> 6), dv + (dl << 16));
            } else {
                const uint32_t tp = ix<L>(D.sbpos + (opos_of<L>(D, b) >> 6));
                if (fv) at_add(D.top + tp, dv);
                if (fl) at_add(D.tlive + tp, dl);
            }
            at_add(D.cnt + b, dv * C_VIS + dl * C_LIVE);
            at_or(D.cnt + b, C_DIRTY);
        }
    }
    if (BALLOT(err)) at_or(&tog_job[3], 1u);
}
// The replay wave's side: post the pass, take its share, wait for the others.
template <int L>
DEV void toggle_mw(Doc &D, uint32_t off, uint32_t n) {
    if (lane_id() == 0) { tog_job[0] = off; tog_job[1] = n; tog_job[2] = 1; tog_job[3] = 0; }
    __syncthreads();
    toggle_chunks<L>(D, off, n, 0);
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // other waves' atomics: no stale L1 lines
    if (U(tog_job[3])) fail(D, ErrCheckout, 16);
    D.cb = NONE;
}
// The other waves: passes until the replay wave reports the document done.
template <int L>
DEV void toggle_helper(Doc &D, uint32_t w) {
    for (;;) {
        __syncthreads();
        if (!U(tog_job[2])) return;
        toggle_chunks<L>(D, U(tog_job[0]), U(tog_job[1]), w);
        __syncthreads();
    }
}

// Stream-compact the visible items (the tip's content) in document order into out[]
// (list/merge.rs:63-95).  G blocks per round keep that many dependent gathers in flight.
// Visibility comes from the counts (the final advance to the tip leaves masks stale): the
// count and the byte offset of every item are gathered together, so this adds no round trip.
template <int L>
DEV void materialise(Doc &D, GLOBAL_AS uint8_t *out, uint32_t cap, uint32_t &len_out, u64 &hash_out, uint32_t &items_out) {
    constexpr uint32_t G = 8;
    const uint32_t l = lane_id();
    const GLOBAL_AS uint32_t *cbyte = gp(vld(&KP().cbyte)) + vld(&D.desc->lv_off);
    const GLOBAL_AS uint8_t *content = gp(vld(&KP().content)) + vld(&D.desc->content_off);
    const bool ascii = U(vld(&D.desc->ascii)) != 0;
    uint32_t total = 0, items = 0;
    u64 h = 0;
    const uint32_t nlists = L == IX_FLAT ? 1u : D.nsb;   // the flat index is one list
    for (uint32_t p = 0; p < nlists; p++) {
        const uint16_t *list = D.sbl;
        uint32_t n = D.nb, ncap = D.nb;
        if (L != IX_FLAT) {
            const uint32_t S = U(ix<L>(D.top + p)) >> 16;
            n = U(ix<L>(D.sbn + S));
            list = D.sbl + size_t(S) * SBC;
            ncap = SBC;
        }
        for (uint32_t i = 0; i < n; i += G) {
            // lane g < G fetches block g's id and item count
            const bool gl = l < G && i + l < n;
            const uint32_t b0 = ix16<L>(list + min(i + (l & (G - 1)), ncap - 1));
            const uint32_t bl = gl ? b0 : 0;
            const uint32_t n0 = c_items(ix<L>(D.cnt + bl));
            const uint32_t nl = gl ? n0 : 0;
            items += wave_sum(nl);
            uint32_t it[G], cb[G], k[G];
            bool vis[G];
#pragma unroll
            for (uint32_t g = 0; g < G; g++) {
                const uint32_t b = bcast(bl, g);
                vis[g] = l < bcast(nl, g);
                const uint32_t i0 = D.items[size_t(b) * BLK + l];   // the row holds BLK slots
                it[g] = vis[g] ? i0 : 0;
            }
#pragma unroll
            for (uint32_t g = 0; g < G; g++) {
                const uint32_t w = ld(D.pc + it[g]), c = cbyte[it[g]];   // it = 0 past the count
                k[g] = vis[g] ? pc_cnt(w) : 0;
                cb[g] = vis[g] ? c : 0;
            }
#pragma unroll
            for (uint32_t g = 0; g < G; g++) vis[g] = vis[g] && k[g] == 1u;
            if (ascii) {
                uint8_t by[G];
#pragma unroll
                for (uint32_t g = 0; g < G; g++) by[g] = vis[g] ? content[cb[g]] : 0;
#pragma unroll
                for (uint32_t g = 0; g < G; g++) {
                    const uint32_t c = vis[g] ? 1u : 0u;
                    const uint32_t inc = wave_scan(c);
                    const uint32_t at = total + inc - c;
                    if (c) {
                        if (at < cap) out[at] = by[g];
                        h += splitmix((u64(at) << 8) | by[g]);
                    }
                    total += bcast(inc, 63);
                }
            } else {
#pragma unroll
                for (uint32_t g = 0; g < G; g++) {
                    const uint32_t c = vis[g] ? utf8_len(content[cb[g]]) : 0u;
                    const uint32_t inc = wave_scan(c);
                    const uint32_t at = total + inc - c;
                    for (uint32_t k = 0; k < c; k++) {
                        const uint8_t byte = content[cb[g] + k];
                        if (at + k < cap) out[at + k] = byte;
                        h += splitmix((u64(at + k) << 8) | byte);
                    }
                    total += bcast(inc, 63);
                }
            }
        }
    }
    len_out = total;
    hash_out = wave_sum64(h);
    items_out = items;
}

// ---- segments (cut replay) -------------------------------------------------------------------
// A long document whose causal graph has cut points -- LVs v such that every op below v is in
// the history of every op at or above v, so the text at v is a plain string that the later ops
// address only by position (the reference's fast-forward boundary, merge.rs:811-840, taken at
// any such v instead of only before the first concurrent entry) -- replays as segments on
// separate waves.  The segment [lo, hi) starts from seg_u placeholder items (ids n_lv + p)
// standing for the text at lo.  seg_u is an upper bound on that text's length (the host takes
// inserts - deletes + concurrent deletes below lo: only a concurrent delete can hit an item
// that is already deleted).  Placeholders past the true length are never addressed by a
// position (every later op addresses the true text), and an insert at the true end lands in
// front of them: its origin_right is the first placeholder instead of END, which sorts after
// every real item in YjsMod's keys as END does.  A placeholder is always live, so it is never
// a YjsMod candidate; only its document-order key and pc[] word are read.  launch_combine
// resolves the segments' source lists into the text.

// LV of the first apply command at or after i (NONE past the last one).
DEV uint32_t first_apply_lv(const Cmd *cmds, uint32_t ncmd, uint32_t i) {
    for (; i < ncmd; i++) {
        const Cmd c = cmds[i];
        if ((c.op & 15u) != CMD_TOG) return c.lv;
    }
    return NONE;
}
// First command of the segment that starts at LV v: the walk visits ancestors first, so every
// command of an entry below the cut precedes every command of an entry above it, and "the first
// apply command at or after i has lv >= v" is monotone in i (64-ary search).
DEV uint32_t seg_cmd(const Cmd *cmds, uint32_t ncmd, uint32_t v) {
    const uint32_t l = lane_id();
    uint32_t lo = 0, hi = ncmd;   // answer in [lo, hi]
    while (lo < hi) {
        const uint32_t step = max(1u, (hi - lo + 63) / 64), b = lo;
        const uint32_t i = b + l * step;
        const bool in = i < hi;
        const u64 m = BALLOT(in && first_apply_lv(cmds, ncmd, i) >= v);
        if (m) {
            const uint32_t f = first_lane(m);
            hi = b + f * step;
            lo = f ? b + (f - 1) * step + 1 : b;
        } else {
            lo = b + last_lane(BALLOT(in)) * step + 1;
        }
        lo = U(lo);
        hi = U(hi);
    }
    return lo;
}
// True when the last apply command before c runs past LV v (the cut is not a command boundary).
DEV bool seg_straddles(const Cmd *cmds, uint32_t c, uint32_t v) {
    if (v == NONE || c == 0) return false;
    bool bad = false;
    if (lane_id() == 0) {
        for (uint32_t j = c; j-- > 0;) {
            const Cmd x = cmds[j];
            if ((x.op & 15u) != CMD_TOG) { bad = x.lv + x.len > v; break; }
        }
    }
    return BALLOT(bad) != 0;
}
constexpr uint32_t PH_FILL = 48;   // placeholder items per block (the HBM tier keeps >= 32)
constexpr uint32_t PH_SB = 40;     // placeholder blocks per superblock
// The tracker a segment starts from: u visible placeholder items in document order.
template <int L>
DEV bool init_phantoms(Doc &D, uint32_t u) {
    const uint32_t l = lane_id();
    const uint32_t base = U(vld(&D.desc->n_lv));   // placeholder ids follow the LVs
    const uint32_t nbp = (u + PH_FILL - 1) / PH_FILL, nsb = (nbp + PH_SB - 1) / PH_SB;
    if (nbp + 1 > D.max_blocks || (L != IX_FLAT && nsb + 1 > D.max_sb)) { fail(D, ErrCapacity, 12); return false; }
    if (L == IX_FLAT) {   // block b at position b; chunk totals of 64 blocks
        for (uint32_t b = l; b < nbp; b += 64) {
            const uint32_t k = min(PH_FILL, u - b * PH_FILL);
            D.cnt[b] = k * (C_VIS + C_LIVE + C_ITEMS);
            D.opos16[b] = uint16_t(b);
            D.sbl[b] = uint16_t(b);
            st(D.m2 + 2 * size_t(b), lanes_below(k));
            st(D.m2 + 2 * size_t(b) + 1, lanes_below(k));
        }
        for (uint32_t c = l; c < D.max_sb; c += 64) {   // max_sb: the chunk capacity
            const uint32_t lo = min(u, c * 64 * PH_FILL), hi = min(u, (c + 1) * 64 * PH_FILL);
            D.top[c] = (hi - lo) | ((hi - lo) << 16);
        }
    } else {
    for (uint32_t b = l; b < nbp; b += 64) {
        const uint32_t k = min(PH_FILL, u - b * PH_FILL);
        const uint32_t S = b / PH_SB, i = b % PH_SB;
        D.cnt[b] = k * (C_VIS + C_LIVE + C_ITEMS);
        set_opos<L>(D, b, (S << 6) | i);
        D.sbl[size_t(S) * SBC + i] = uint16_t(b);
        st(D.m2 + 2 * size_t(b), lanes_below(k));
        st(D.m2 + 2 * size_t(b) + 1, lanes_below(k));
    }
    for (uint32_t S = l; S < nsb; S += 64) {
        const uint32_t nb = min(PH_SB, nbp - S * PH_SB);
        const uint32_t nv = min(nb * PH_FILL, u - S * PH_SB * PH_FILL);
        D.sbn[S] = nb;
        D.sbpos[S] = S;
        D.top[S] = (S << 16) | nv;
        D.tlive[S] = nv;
    }
    }
    for (uint32_t b = 0; b < nbp; b++) {   // rows: one wave store per block
        const uint32_t k = min(PH_FILL, u - b * PH_FILL);
        D.items[size_t(b) * BLK + l] = l < k ? base + b * PH_FILL + l : 0u;
    }
    for (uint32_t p = l; p < u; p += 64) st(D.pc + base + p, pc_of(p / PH_FILL, 1u));
    wave_fence();
    D.nb = nbp;
    D.nsb = nsb;
    return true;
}
// A segment's visible items in document order as a source list (an LV, or SEG_PHANTOM | the
// placeholder's index), gathered G blocks per round as materialise() does.
template <int L>
DEV void materialise_src(Doc &D, GLOBAL_AS uint32_t *src, uint32_t cap, uint32_t &len_out, uint32_t &items_out) {
    constexpr uint32_t G = 8;
    const uint32_t l = lane_id();
    const uint32_t n_lv = U(vld(&D.desc->n_lv));   // D.n_lv also counts the placeholders
    uint32_t total = 0, items = 0;
    const uint32_t nlists = L == IX_FLAT ? 1u : D.nsb;   // the flat index is one list
    for (uint32_t p = 0; p < nlists; p++) {
        const uint16_t *list = D.sbl;
        uint32_t n = D.nb, ncap = D.nb;
        if (L != IX_FLAT) {
            const uint32_t S = U(ix<L>(D.top + p)) >> 16;
            n = U(ix<L>(D.sbn + S));
            list = D.sbl + size_t(S) * SBC;
            ncap = SBC;
        }
        for (uint32_t i = 0; i < n; i += G) {
            const bool gl = l < G && i + l < n;
            const uint32_t b0 = ix16<L>(list + min(i + (l & (G - 1)), ncap - 1));
            const uint32_t bl = gl ? b0 : 0;
            const uint32_t n0 = c_items(ix<L>(D.cnt + bl));
            const uint32_t nl = gl ? n0 : 0;
            items += wave_sum(nl);
            uint32_t it[G];
            bool vis[G];
#pragma unroll
            for (uint32_t g = 0; g < G; g++) {
                const uint32_t b = bcast(bl, g);
                vis[g] = l < bcast(nl, g);
                const uint32_t i0 = D.items[size_t(b) * BLK + l];
                it[g] = vis[g] ? i0 : 0;
            }
#pragma unroll
            for (uint32_t g = 0; g < G; g++) vis[g] = vis[g] && pc_cnt(ld(D.pc + it[g])) == 1u;
#pragma unroll
            for (uint32_t g = 0; g < G; g++) {
                const uint32_t c = vis[g] ? 1u : 0u;
                const uint32_t inc = wave_scan(c);
                const uint32_t at = total + inc - c;
                if (c && at < cap) src[at] = it[g] < n_lv ? it[g] : (SEG_PHANTOM | (it[g] - n_lv));
                total += bcast(inc, 63);
            }
        }
    }
    len_out = total;
    items_out = items;
}

// Debug-mode consistency check of the whole structure (DTGPU_DEBUG=1): returns 0 or a code.
// Checks every block's counts against its masks (clean blocks) or against cv[] (DIRTY blocks),
// and that pos[] names each item's block.
template <int L, bool XF>
DEV uint32_t check_invariants(Doc &D, DocResult *res) {
    const uint32_t l = lane_id();
    const uint32_t n_ids = D.n_lv;   // LVs, then a segment's placeholders
    uint32_t blocks = 0;
    const uint32_t nlists = L == IX_FLAT ? (D.nb + 63) >> 6 : D.nsb;   // flat: chunks of 64 positions
    for (uint32_t p = 0; p < nlists; p++) {
        uint32_t S = p, n;
        if (L == IX_FLAT) {
            n = min(64u, D.nb - 64 * p);
        } else {
            S = U(ix<L>(D.top + p)) >> 16;
            if (U(ix<L>(D.sbpos + S)) != p) return 205;
            n = U(ix<L>(D.sbn + S));
            if (n == 0 || n >= SBC) return 206;
        }
        uint32_t tv = 0, tl = 0, tu = 0;
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t b = U(ix16<L>(D.sbl + size_t(S) * (L == IX_FLAT ? 64u : SBC) + i));
            if (U(opos_of<L>(D, b)) != (L == IX_FLAT ? 64 * p + i : ((S << 6) | i))) return 201;
            const uint32_t c = U(ix<L>(D.cnt + b));
            const uint32_t cnt = c_items(c);
            const bool dirty = (c & C_DIRTY) != 0;
            u64 mv = U64(ld(D.m2 + 2 * size_t(b))), ml = U64(ld(D.m2 + 2 * size_t(b) + 1));
            if (dirty) {   // stale masks: check the counts against cv[] instead
                const uint32_t i2 = l < cnt ? D.items[size_t(b) * BLK + l] : 0;
                const uint32_t k = l < cnt && i2 < n_ids ? pc_cnt(ld(D.pc + i2)) : 0u;
                mv = BALLOT(l < cnt && k == 1u);
                ml = BALLOT(l < cnt && k != 0u);
            }
            if (uint32_t(__popcll(mv)) != c_vis(c) || uint32_t(__popcll(ml)) != c_live(c)) return 207;
            if (XF && uint32_t(__popcll(U64(ld(D.mup + b)))) != c_up(c)) return 209;
            if (XF) tu += c_up(c);
            tv += c_vis(c);
            tl += c_live(c);
            bool bad = false;
            uint32_t w = 0, it = 0xFFFFFFFFu;
            if (l < cnt) {
                it = D.items[size_t(b) * BLK + l];
                if (it >= n_ids) bad = true;
                else {
                    w = pc_blk(ld(D.pc + it));
                    const uint32_t k = pc_cnt(ld(D.pc + it));
                    if (((mv >> l) & 1) != (k == 1 ? 1u : 0u)) bad = true;
                    if (((ml >> l) & 1) != (k != 0 ? 1u : 0u)) bad = true;
                    if (w != b || find_slot(D, b, it) != l) bad = true;
                }
            } else if (((mv | ml) >> l) & 1) bad = true;
            const u64 bm = BALLOT(bad);
            if (bm) {
                if (l == first_lane(bm)) {
                    res->dbg[0] = b; res->dbg[1] = l; res->dbg[2] = cnt; res->dbg[3] = it; res->dbg[4] = w;
                    res->dbg[5] = uint32_t(mv); res->dbg[6] = uint32_t(mv >> 32);
                    res->dbg[7] = uint32_t(ml); res->dbg[8] = uint32_t(ml >> 32);
                }
                return 202;
            }
            blocks++;
        }
        if (tv != (U(ix<L>(D.top + p)) & 0xFFFFu)) return 203;
        if (tl != (L == IX_FLAT ? U(ix<L>(D.top + p)) >> 16 : U(ix<L>(D.tlive + p)))) return 204;
        if (XF && tu != U(ix<L>(D.tup + p))) return 210;
    }
    if (blocks != D.nb) return 208;
    if (L == IX_FLAT) {   // chunks past the last position hold nothing
        for (uint32_t c = nlists + l; c < D.max_sb; c += 64)
            if (BALLOT(D.top[c] != 0)) return 211;
    }
    return 0;
}

template <int L, bool PROF, bool XF, bool MW>
DEV void run_doc(Doc &D) {
    const uint32_t l = lane_id();
    D.nb = 1;
    D.nsb = 1;
    D.err = 0;
    D.site = 0;
    // a segment (cut replay) applies its LV range's commands only
    const uint32_t seg_lo = U(vld(&D.desc->seg_lo)), seg_hi = U(vld(&D.desc->seg_hi));
    if (!XF && (seg_lo != 0 || seg_hi != NONE)) {
        const uint32_t c0 = seg_lo ? U(seg_cmd(D.cmds, D.ncmd, seg_lo)) : 0u;
        const uint32_t c1 = seg_hi != NONE ? U(seg_cmd(D.cmds, D.ncmd, seg_hi)) : D.ncmd;
        if (c1 < c0 || seg_straddles(D.cmds, c0, seg_lo) || seg_straddles(D.cmds, c1, seg_hi)) fail(D, ErrCheckout, 30);
        else { D.cmds += c0; D.ncmd = c1 - c0; }
    }
    D.steps = uint32_t(min<uint64_t>(64ull * (uint64_t(D.ncmd) + D.n_lv) + 4096, 0xFFFFFFF0ull));
    const uint32_t seg_u = XF ? 0u : U(vld(&D.desc->seg_u));
    if (seg_u) {
        if (!D.err) init_phantoms<L>(D, seg_u);
    } else {
        // fresh tracker: one empty block in one superblock (per-LV words are written when their
        // item is inserted)
        if (L == IX_FLAT) {   // every chunk total starts at zero (chunks fill as blocks split)
            for (uint32_t c = l; c < D.max_sb; c += 64) D.top[c] = 0;
            if (l == 0) { D.cnt[0] = 0; D.opos16[0] = 0; D.sbl[0] = 0; }
        } else if (l == 0) {
            D.cnt[0] = 0; set_opos<L>(D, 0, 0);
            D.sbl[0] = 0; D.sbn[0] = 1; D.sbpos[0] = 0; D.top[0] = 0; D.tlive[0] = 0;
            if (XF) { D.tup[0] = 0; st(D.mup, 0ull); }
        }
        if (l < 2) st(D.m2 + l, 0ull);
        wave_fence();
    }
    D.cb = NONE;
    D.cit = 0;
    D.cmv = D.cml = 0;
    if (PROF) for (int i = 0; i < P_N; i++) D.prof[i] = 0;
    const uint64_t t_start = tick<PROF>();
    // commands are fetched 64 at a time (one per lane) and broadcast with readlane; the first
    // tlist chunk of a TOG is fetched while the command before it runs (tlist is read-only)
    uint32_t pf = 0;
    bool pf_ok = false;
    uint32_t ci = 0;   // the command being applied (the failing one when the loop ends on an error)
    for (uint32_t base = 0; base < D.ncmd && !D.err; base += 64) {
        const uint32_t n_here = min(64u, D.ncmd - base);
        Cmd pre = {0, 0, 0, 0};
        pre = D.cmds[min(base + l, D.ncmd - 1)];   // lanes past n_here are never read
        // The chunk's commands checked lane-parallel: a malformed one (an unknown op, an apply
        // run outside the LVs) ends the replay at its index; the retreat / advance passes are a
        // mask, so each command's look-ahead is one bit test.  (The scalar unit is what a
        // batch's replay is bound by: per-command bookkeeping is kept off it.)
        const uint32_t op_l = pre.op & 15u;
        const bool apply_l = op_l == CMD_INS || op_l == CMD_DEL;
        const u64 bad_cmds = BALLOT(l < n_here && (op_l > CMD_TOG || (apply_l && (pre.len == 0 || pre.lv >= D.n_lv ||
                                                                               pre.len > D.n_lv - pre.lv))));
        const u64 tog_cmds = BALLOT(l < n_here && op_l == CMD_TOG);
        const uint32_t n_ok = bad_cmds ? first_lane(bad_cmds) : n_here;
        for (uint32_t j = 0; j < n_ok && !D.err; j++) {
            ci = base + j;
            const uint32_t op = U(bcast(pre.op, j)), a = U(bcast(pre.lv, j)), n = U(bcast(pre.len, j)),
                           pos = U(bcast(pre.pos, j));
            uint32_t nx_pf = 0;
            bool nx_ok = false;
            if ((tog_cmds >> j) & 2ull) {   // the next command is a pass: its first entries now
                const uint32_t o2 = U(bcast(pre.lv, j + 1)), n2 = U(bcast(pre.len, j + 1));
                if (n2) nx_pf = D.tlist[o2 + min(l, n2 - 1)];
                nx_ok = true;
            }
            const uint64_t t0 = tick<PROF>();
            if ((op & 15u) == CMD_INS) {
                do_insert<L, PROF, XF>(D, a, n, pos);
                if (PROF) D.prof[P_INS] += tick<PROF>() - t0;
            } else if ((op & 15u) == CMD_DEL) {
                do_delete<L, PROF, XF>(D, a, n, pos, (op & 16u) != 0);
                if (PROF) D.prof[P_DEL] += tick<PROF>() - t0;
            } else {
                if (MW && n >= TOG_MW_MIN) toggle_mw<L>(D, a, n);
                else toggle_pass<L, PROF>(D, a, n, pf, pf_ok);
                if (PROF) D.prof[P_TOG] += tick<PROF>() - t0;
            }
            if (PROF && (D.debug & 1u) && !D.err) {   // invariant checks: instrumented builds only
                const uint32_t code = check_invariants<L, XF>(D, vld(&KP().results) + D.doc);
                if (code) fail(D, ErrCheckout, code);
            }
            pf = nx_pf;
            pf_ok = nx_ok;
        }
        if (bad_cmds && !D.err) {
            ci = base + n_ok;
            fail(D, ErrCheckout, (U(bcast(pre.op, n_ok)) & 15u) > CMD_TOG ? 18u : 17u);
        }
    }
    // an LDS-tier document that outgrew its optimistic block capacity is queued for the HBM
    // tier, which replays it again from scratch
    if (L && D.err == ErrCapacity && (D.site == 12 || D.site == 21)) {
        uint32_t *fb_list = vld(&KP().fb_list);
        if (fb_list) {
            if (l == 0) gp(fb_list)[atomicAdd(vld(&KP().fb_count), 1u)] = D.doc;
            return;
        }
    }
    uint32_t len = 0, n_items = 0;
    u64 h = 0;
    const uint64_t t_mat = tick<PROF>();
    if (!D.err) {
        const uint64_t so = vld(&D.desc->src_off);
        if (!XF && so != ~0ull) {   // a segment: its source list, resolved by launch_combine
            const uint32_t cap = U(vld(&D.desc->src_cap));
            materialise_src<L>(D, gp(vld(&KP().src)) + so, cap, len, n_items);
            if (len > cap) { fail(D, ErrCapacity, 32); len = 0; }   // (cap bounds the items: unreachable)
        } else {
            GLOBAL_AS uint8_t *out = gp(vld(&KP().out)) + vld(&D.desc->out_off);
            materialise<L>(D, out, U(vld(&D.desc->out_cap)), len, h, n_items);
        }
    }
    GLOBAL_AS DocResult *res = gp(vld(&KP().results)) + D.doc;
    if (l == 0) {
        res->status = D.err;
        res->out_len = len;
        res->hash = h;
        res->n_items = n_items;
        res->n_blocks = D.nb;
        res->n_sb = D.nsb;
        res->lds = L ? 1u : 0u;
        res->fail_cmd = D.err ? ci : 0;
        res->fail_site = D.err ? D.site : 0;
        if (PROF && (D.debug & 2u)) {
            D.prof[P_MAT] = tick<PROF>() - t_mat;
            for (int i = 0; i < P_T1; i++) res->dbg[i] = uint32_t(D.prof[i] >> (i < P_N_YJS ? 4 : 0));
            res->dbg[15] = uint32_t((tick<PROF>() - t_start) >> 4);
            for (int i = P_T1; i < P_N_DIRTY; i++) res->dbg[16 + (i - P_T1)] = uint32_t(D.prof[i] >> 4);
            res->dbg[19] = uint32_t(D.prof[P_N_DIRTY]);
            res->dbg[20] = uint32_t(D.prof[P_N_LOAD]);
        }
    }
}

// Carve an index for `mb` blocks / `ms` superblocks out of `base` (LDS or HBM); layout must
// match index_bytes().
DEV void bind_index(Doc &D, uint8_t *base, uint32_t mb, uint32_t ms, bool narrow) {
    uint32_t *w = reinterpret_cast<uint32_t *>(base);
    D.cnt = w; w += mb;
    if (narrow) { D.opos16 = reinterpret_cast<uint16_t *>(w); D.opos = nullptr; w += (mb + 1) / 2; }
    else { D.opos = w; D.opos16 = nullptr; w += mb; }
    D.top = w; w += ms;
    D.tlive = w; w += ms;
    D.sbn = w; w += ms;
    D.sbpos = w; w += ms;
    D.sbl = reinterpret_cast<uint16_t *>(w);
}

// The flat index (IX_FLAT) for `mb` blocks; layout must match flat_index_bytes().
DEV void bind_index_flat(Doc &D, uint8_t *base, uint32_t mb) {
    uint32_t *w = reinterpret_cast<uint32_t *>(base);
    D.cnt = w; w += mb;
    D.opos16 = reinterpret_cast<uint16_t *>(w); w += (mb + 1) / 2;
    D.sbl = reinterpret_cast<uint16_t *>(w); w += (mb + 1) / 2;   // ord[]: block by position
    D.top = w;                                                     // ctot[]: per 64 positions
    D.opos = D.tlive = D.sbn = D.sbpos = nullptr;
}

// One 64-lane workgroup per document of the list (the hardware dispatcher is the work queue;
// LDS per workgroup bounds how many documents share a CU).
// MW: TOG_WAVES waves per workgroup, the others helping with long retreat / advance passes
// (the big LDS tiers: one or two documents per CU, so the extra waves cost no occupancy).
// WAVES: the occupancy the compiler budgets registers for (the flat tier's documents are small
// enough for 32 per CU, i.e. 8 waves per SIMD if the kernel takes <= 80 SGPRs and <= 64 VGPRs).
template <int LDS_INDEX, bool PROF, bool XF, bool MW = false, int WAVES = 1>
__global__ __launch_bounds__(MW ? 64 * TOG_WAVES : 64) __attribute__((amdgpu_waves_per_eu(WAVES))) void replay_kernel(BatchParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t di = U(blockIdx.x);
    // A workgroup dispatched into a slot an earlier document freed starts as the youngest wave
    // on its SIMD, and the arbiter serves older waves first: such a late document would run to
    // the end of the batch at the back of the queue.  It takes the higher priority instead, so
    // the batch's last documents finish beside the first round's slowest ones.
    if (P.prio_from && di >= P.prio_from) __builtin_amdgcn_s_setprio(3);
    uint32_t d;
    if (di < P.n_list) {
        d = U(P.doc_list[di]);
    } else {   // HBM tier: documents the LDS tier handed back
        if (LDS_INDEX || !P.fb_count) return;
        const uint32_t j = di - P.n_list;
        if (j >= U(__hip_atomic_load(P.fb_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) return;
        d = U(P.fb_list[j]);
    }
    const DocDesc dd = P.docs[d];
    if (dd.flags & DOC_CRITICAL) __builtin_amdgcn_s_setprio(3);
    Doc D;
    D.doc = d;
    D.desc = P.docs + d;
    D.debug = P.debug & 3u;
    D.cmds = P.cmds + dd.cmd_off;
    D.ncmd = U(dd.ncmd);
    // item ids: the LVs, then a segment's placeholders (cut replay)
    D.n_lv = U(dd.n_lv) + (XF ? 0u : U(dd.seg_u));
    D.tlist = P.tlist + dd.tlist_off;
    D.pc = P.pos + dd.pc_off;   // lv_off, or a segment's own region
    D.ao = P.ao + dd.pc_off;
    D.items = P.items + dd.blk_off * BLK;
    D.m2 = P.m2 + 2 * dd.blk_off;
    D.max_blocks = U(dd.max_blocks);
    D.max_sb = sb_capacity(D.max_blocks);
    static_assert(!(XF && LDS_INDEX), "transformed-ops mode replays on the HBM index");
    static_assert(!(MW && LDS_INDEX != IX_LDS), "helper waves serve the 3-level LDS tiers");
    if (LDS_INDEX == IX_FLAT) {
        if (D.max_blocks > P.lds_blocks) D.max_blocks = P.lds_blocks;
        D.max_sb = flat_chunks(P.lds_blocks);   // chunk capacity
        bind_index_flat(D, smem, P.lds_blocks);
    } else if (LDS_INDEX) {
        if (D.max_blocks > P.lds_blocks) D.max_blocks = P.lds_blocks;
        D.max_sb = P.lds_sb;
        bind_index(D, smem, P.lds_blocks, D.max_sb, true);
    } else {
        bind_index(D, P.gidx + dd.gidx_off, D.max_blocks, D.max_sb, false);
    }
    if (XF) {
        D.mup = P.mup + dd.blk_off;
        D.tup = P.tup + dd.blk_off + 2ull * d;   // sb_capacity(mb) <= mb + 2 slots per document
        D.xf = P.xf + dd.lv_off;
    }
    if (MW) {
        const uint32_t w = U(threadIdx.x / 64);
        if (w) { toggle_helper<LDS_INDEX>(D, w); return; }
    }
    run_doc<LDS_INDEX, PROF, XF, MW>(D);
    if (MW) {   // release the helper waves
        if (lane_id() == 0) tog_job[2] = 0;
        __syncthreads();
    }
}


// Cut replay: one workgroup per cut document resolves its segments' source lists in LV order --
// a placeholder of segment k is entry p of segment k-1's resolved list; segment k's entries
// from the first placeholder past that list's length on are the surplus placeholders (a
// suffix, checked) -- and writes the text with materialise()'s bytes and hash.  The document's
// own result slot (its first segment) gets the length and hash, or the first failing
// segment's status.
// COMBINE_THREADS: 1024 threads for a few cut documents (long texts: node_nodecc's 13 segments
// combine in ~0.9 ms), 256 for many (a batch's cut documents in one round of workgroups, not four)
template <uint32_t COMBINE_THREADS>
__global__ __launch_bounds__(COMBINE_THREADS) void combine_kernel(CombineParams P) {
    __shared__ uint32_t s_cut, s_bad, s_wsum[COMBINE_THREADS / 64];
    __shared__ u64 s_h[COMBINE_THREADS / 64];
    const SegGroup g = P.groups[blockIdx.x];
    const uint32_t t = threadIdx.x, w = t / 64, nw = COMBINE_THREADS / 64;
    const uint32_t d0 = P.seg_docs[g.first];
    DocResult *res0 = P.results + d0;
    uint32_t status = 0, site = 0, fcmd = 0;
    for (uint32_t k = 0; k < g.count && !status; k++) {
        const DocResult &r = P.results[P.seg_docs[g.first + k]];
        status = r.status; site = r.fail_site; fcmd = r.fail_cmd;
    }
    if (status) {
        __syncthreads();
        if (t == 0) { res0->status = status; res0->fail_site = site; res0->fail_cmd = fcmd; res0->out_len = 0; res0->hash = 0; }
        return;
    }
    const uint32_t *R = P.src + P.docs[d0].src_off;
    uint32_t nR = P.results[d0].out_len;
    if (t == 0) s_bad = 0;
    for (uint32_t k = 1; k < g.count; k++) {
        const uint32_t dk = P.seg_docs[g.first + k];
        uint32_t *S = P.src + P.docs[dk].src_off;
        const uint32_t nS = P.results[dk].out_len;
        if (t == 0) {   // "a surplus placeholder" is monotone along the list: binary search
            uint32_t lo = 0, hi = nS;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) / 2, e = S[mid];
                if ((e & SEG_PHANTOM) && (e & ~SEG_PHANTOM) >= nR) hi = mid;
                else lo = mid + 1;
            }
            s_cut = lo;
            // surplus placeholders are the last ones, in order: the suffix is exactly them
            if (lo < nS && S[nS - 1] != (SEG_PHANTOM | (S[lo] & ~SEG_PHANTOM) + (nS - 1 - lo))) s_bad = 1;
        }
        __syncthreads();
        const uint32_t cut = s_cut;
        for (uint32_t i = t; i < cut; i += COMBINE_THREADS) {
            const uint32_t e = S[i];
            if (e & SEG_PHANTOM) {
                if ((e & ~SEG_PHANTOM) < nR) S[i] = R[e & ~SEG_PHANTOM];
                else s_bad = 1;   // (the suffix search makes this unreachable)
            }
        }
        __syncthreads();
        R = S;
        nR = cut;
    }
    const DocDesc &dd = P.docs[d0];
    const uint32_t *cbyte = P.cbyte + dd.lv_off;
    const uint8_t *content = P.content + dd.content_off;
    uint8_t *out = P.out + dd.out_off;
    const uint32_t cap = dd.out_cap, n_lv = dd.n_lv, clen = dd.content_len;
    const bool ascii = dd.ascii != 0;
    u64 h = 0;
    uint32_t base = 0;
    for (uint32_t i0 = 0; i0 < nR; i0 += COMBINE_THREADS) {
        const uint32_t i = i0 + t;
        uint32_t cb = 0, len = 0;
        if (i < nR) {
            const uint32_t e = R[i];
            const uint32_t c = e < n_lv ? cbyte[e] : NONE;
            if (c < clen) { cb = c; len = ascii ? 1u : utf8_len(content[c]); }
            else s_bad = 1;
        }
        const uint32_t inc = wave_scan(len);
        if ((t & 63) == 63) s_wsum[w] = inc;
        __syncthreads();
        uint32_t before = 0, round = 0;
        for (uint32_t j = 0; j < nw; j++) { const uint32_t x = s_wsum[j]; if (j < w) before += x; round += x; }
        const uint32_t at = base + before + inc - len;
        for (uint32_t k = 0; k < len; k++) {
            const uint8_t by = content[cb + k];
            if (at + k < cap) out[at + k] = by;
            h += splitmix((u64(at + k) << 8) | by);
        }
        base += round;
        __syncthreads();   // s_wsum reused next round
    }
    h = wave_sum64(h);
    if ((t & 63) == 0) s_h[w] = h;
    __syncthreads();
    if (t == 0) {
        u64 H = 0;
        for (uint32_t j = 0; j < nw; j++) H += s_h[j];
        if (s_bad) { res0->status = ErrCheckout; res0->fail_site = 31; res0->out_len = 0; res0->hash = 0; }
        else { res0->out_len = base; res0->hash = H; }
    }
}

}  // namespace dev

static int launch_lds_tier(const BatchParams &q, hipStream_t s, bool prof) {
    if (!q.n_list) return OK;
    if (q.lds_flat) {   // the flat index: small documents, one wave each
        if (q.lds_blocks > FLAT_MAX_BLOCKS) return ErrArg;
        size_t lds = size_t(flat_index_bytes(q.lds_blocks));
        if (lds > 64 * 1024) return ErrArg;
        // resident documents per CU: 8 waves per SIMD (the kernel's register budget) or what the
        // LDS allows (allocated in 1280-byte granules; tools/occ_probe.hip measured both)
        BatchParams qp = q;
        qp.prio_from = 0;
        if (q.prio_on) {
            // (the batch's own device: late_documents sizes the same resident set from it)
            const size_t gran = (lds + 1279) / 1280 * 1280;
            const size_t per_cu = std::min<size_t>(32, 163840 / std::max<size_t>(gran, 1280));
            qp.prio_from = uint32_t(per_cu * size_t(std::max<uint32_t>(q.n_cu, 1)));
        }
        if (prof) hipLaunchKernelGGL((dev::replay_kernel<dev::IX_FLAT, true, false>), dim3(q.n_list), dim3(64), lds, s, qp);
        else hipLaunchKernelGGL((dev::replay_kernel<dev::IX_FLAT, false, false, false, 8>), dim3(q.n_list), dim3(64), lds, s, qp);
        return launch_error() == hipSuccess ? OK : ErrHip;
    }
    size_t lds = size_t(index_bytes_ms(q.lds_blocks, q.lds_sb, true));
    if (lds > 160 * 1024) return ErrArg;   // a tier cap above the CU's LDS
    // documents whose index takes >= 32 KiB of LDS (at most four per CU) replay with helper
    // waves for long retreat / advance passes (DTGPU_TOG_WAVES=1: one wave)
    constexpr size_t kStatic = sizeof(uint32_t) * 4;   // tog_job: the multi-wave kernel's static LDS
    const size_t mw_min = q.tog_mw_lds;   // the LDS bytes from which a tier gets helper waves
    const bool mw = lds >= mw_min && lds + kStatic <= 160 * 1024 && q.tog_waves != 1;
    // allow dynamic LDS up to the CU's 160 KiB: a per-function, per-device attribute, set on
    // every launch (cheap) so it holds on whatever device the batch runs
    const void *fn = mw ? (prof ? reinterpret_cast<const void *>(&dev::replay_kernel<dev::IX_LDS, true, false, true>)
                                : reinterpret_cast<const void *>(&dev::replay_kernel<dev::IX_LDS, false, false, true>))
                        : (prof ? reinterpret_cast<const void *>(&dev::replay_kernel<dev::IX_LDS, true, false>)
                                : reinterpret_cast<const void *>(&dev::replay_kernel<dev::IX_LDS, false, false>));
    if (lds + (mw ? kStatic : 0) > 64 * 1024 &&
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(160 * 1024 - (mw ? kStatic : 0))) != hipSuccess)
        return ErrHip;
    if (mw) {
        const dim3 blk(64 * dev::TOG_WAVES);
        if (prof) hipLaunchKernelGGL((dev::replay_kernel<dev::IX_LDS, true, false, true>), dim3(q.n_list), blk, lds, s, q);
        else hipLaunchKernelGGL((dev::replay_kernel<dev::IX_LDS, false, false, true>), dim3(q.n_list), blk, lds, s, q);
    } else if (prof) {
        hipLaunchKernelGGL((dev::replay_kernel<dev::IX_LDS, true, false>), dim3(q.n_list), dim3(64), lds, s, q);
    } else {
        hipLaunchKernelGGL((dev::replay_kernel<dev::IX_LDS, false, false>), dim3(q.n_list), dim3(64), lds, s, q);
    }
    return launch_error() == hipSuccess ? OK : ErrHip;
}

int launch_replay(const ReplayLaunch &r) {
    hipStream_t s = reinterpret_cast<hipStream_t>(r.stream);
    const BatchParams &large = *r.large;
    bool prof = (large.debug & 3u) != 0;   // invariant checks and cycle profiles: the instrumented kernels
    uint32_t n_lds = 0;
    const uint32_t *fb_count = nullptr;
    for (int t = 0; t < r.n_lds; t++) {
        prof |= (r.lds[t].debug & 3u) != 0;
        n_lds += r.lds[t].n_list;
        if (r.lds[t].fb_count) fb_count = r.lds[t].fb_count;
    }
    if (n_lds) {
        if (fb_count && !r.keep_fb && hipMemsetAsync(const_cast<uint32_t *>(fb_count), 0, sizeof(uint32_t), s) != hipSuccess)
            return ErrHip;
        // fork: the biggest tiers start first, each on its own side stream; the smallest tier
        // runs on the main stream
        int n_side = 0;
        while (n_side < kSideStreams && n_side < r.n_lds - 1 && r.side[n_side] && r.ev_join[n_side]) n_side++;
        const bool fork = n_side > 0 && r.ev_fork;
        if (fork) {
            if (hipEventRecord(reinterpret_cast<hipEvent_t>(r.ev_fork), s) != hipSuccess) return ErrHip;
            for (int k = 0; k < n_side; k++)
                if (hipStreamWaitEvent(reinterpret_cast<hipStream_t>(r.side[k]), reinterpret_cast<hipEvent_t>(r.ev_fork), 0) !=
                    hipSuccess)
                    return ErrHip;
        }
        for (int t = r.n_lds - 1; t >= 0; t--) {
            const int k = r.n_lds - 1 - t;
            const int e = launch_lds_tier(r.lds[t], (fork && k < n_side) ? reinterpret_cast<hipStream_t>(r.side[k]) : s, prof);
            if (e) return e;
        }
        if (fork) {
            for (int k = 0; k < n_side; k++)
                if (hipEventRecord(reinterpret_cast<hipEvent_t>(r.ev_join[k]), reinterpret_cast<hipStream_t>(r.side[k])) != hipSuccess ||
                    hipStreamWaitEvent(s, reinterpret_cast<hipEvent_t>(r.ev_join[k]), 0) != hipSuccess)
                    return ErrHip;
        }
    }
    // split pass: the big tier's side pipeline must be done before the HBM tier reads the
    // fallback queue and before anything synchronising on s sees the batch as finished -- also
    // when no other LDS tier forked above (then nothing else joined that stream)
    if (r.join_side >= 0) {
        if (r.join_side >= kSideStreams || !r.side[r.join_side] || !r.ev_join[r.join_side]) return ErrArg;
        if (hipEventRecord(reinterpret_cast<hipEvent_t>(r.ev_join[r.join_side]), reinterpret_cast<hipStream_t>(r.side[r.join_side])) !=
                hipSuccess ||
            hipStreamWaitEvent(s, reinterpret_cast<hipEvent_t>(r.ev_join[r.join_side]), 0) != hipSuccess)
            return ErrHip;
    }
    // HBM tier: its own list plus a slot per LDS-tier document that may be handed back
    const uint32_t grid = large.n_list + (large.fb_list ? large.fb_slots : 0);
    if (grid) {
        if (prof) hipLaunchKernelGGL((dev::replay_kernel<dev::IX_HBM, true, false>), dim3(grid), dim3(64), 0, s, large);
        else hipLaunchKernelGGL((dev::replay_kernel<dev::IX_HBM, false, false>), dim3(grid), dim3(64), 0, s, large);
        if (launch_error() != hipSuccess) return ErrHip;
    }
    return OK;
}

// Transformed-ops replay (iter_xf_operations): HBM-tier index, one workgroup per document of
// `large`, per-LV transformed positions into large.xf.
int launch_replay_xf(const BatchParams &large, void *stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (!large.n_list) return OK;
    if (!large.xf || !large.mup || !large.tup) return ErrArg;
    if (large.debug & 3u) hipLaunchKernelGGL((dev::replay_kernel<dev::IX_HBM, true, true>), dim3(large.n_list), dim3(64), 0, s, large);
    else hipLaunchKernelGGL((dev::replay_kernel<dev::IX_HBM, false, true>), dim3(large.n_list), dim3(64), 0, s, large);
    return launch_error() == hipSuccess ? OK : ErrHip;
}

int launch_combine(const CombineParams &p, void *stream) {
    if (!p.n_groups) return OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uint32_t n_cu = p.n_cu ? p.n_cu : 256u;   // the batch's device
    if (p.n_groups >= 2 * n_cu) hipLaunchKernelGGL(dev::combine_kernel<256>, dim3(p.n_groups), dim3(256), 0, s, p);
    else hipLaunchKernelGGL(dev::combine_kernel<1024>, dim3(p.n_groups), dim3(1024), 0, s, p);
    return launch_error() == hipSuccess ? OK : ErrHip;
}

}  // namespace dtgpu
