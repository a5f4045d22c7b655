// dt_span.hip -- per-document eg-walker replay over run-length spans + text materialisation on
// MI355X (gfx950).
//
// One wavefront (64 lanes) replays one document's command stream: INS / DEL op runs and TOG
// passes (one walk step's retreat + advance set), produced by dt_plan.hip on the device or
// dt_host.cpp::build_plan.  This is the checkout-from-ROOT formulation of the reference's
// M2Tracker (src/listmerge/merge.rs:89-581, advance_retreat.rs:58-153) over
// the representation the reference's tracker itself keeps: run-length YjsSpans
// (src/listmerge/yjsspan.rs:13-228) in document order.
//
//   span    a run of consecutive inserted LVs, adjacent in document order, with one state (0 not
//           inserted yet, 1 inserted, k >= 2 deleted k-1 times) and one ever_deleted flag.  Item
//           lv0 + i (i > 0) has origin_left lv0 + i - 1 and every item the span's origin_right
//           (yjsspan.rs:29-32).  8 bytes: lv0 | (len | ever_deleted << 20 | state << 21) << 32.
//           A span is cut wherever a later command touches part of it (YjsSpan::truncate).
//   block   <= 64 spans in document order: row b of rows[], one span per lane (one 512-B load).
//   index   blocks in superblocks (<= 64 block ids each), superblocks in a top-level order, with
//           per-block visible-item / span / live-span counts and per-superblock totals: the
//           content-tree's order statistics (crates/content-tree/src/root.rs:50-89) as a 3-level
//           blocked array.  In LDS for documents whose index fits their tier, in HBM otherwise
//           (same code; the wave owns its document, so both use plain loads and stores).
//   lk[lv]  inserted LV: its block (content-tree's marker index, src/listmerge/markers.rs) --
//           rewritten for the moved LVs when a block splits; delete LV: the item it deleted
//           (markers.rs DelTarget).
//   ao[lv]  inserted LV: origin_left | origin_right << 32 (YjsMod's inputs, merge.rs:154-278).
//
// INS: locate visible index pos-1 (index scans, or the cached last block), derive origin_left /
// origin_right from the row (merge.rs:383-423), run YjsMod only when NIY spans lie between them,
// place one span (cutting the span under the cursor when the insert lands inside it).
// DEL: locate, cut the covered visible range out of the row lane-parallel (<= 2 cuts per block),
// state 1 -> 2, record each deleted LV's target (reversed runs: op_metrics.rs:184-202).
// TOG: the entries' items (LV, or the target of a delete LV) and their blocks are gathered 64 at
// a time and grouped into runs of contiguous items in one block; each run adds +-1 to the state
// of the spans it covers (cutting at most two).  Counters make the order irrelevant: an item's
// final count is its old count plus its deltas, which equals the reference's retreat-then-advance
// (advance_retreat.rs:58-153).
// The plan ends with a TOG that advances to the tip; materialisation copies the visible spans'
// bytes (each span's text is one contiguous range of the insert content) in document order
// (list/merge.rs:63-95).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <stdint.h>

#include "dt_device.hpp"

namespace dtgpu {
namespace sdev {

typedef unsigned long long u64;

#define DEV __device__ __forceinline__

DEV uint32_t lane_id() { return __lane_id(); }
DEV void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); }
DEV uint32_t bcast(uint32_t v, uint32_t l) { return uint32_t(__builtin_amdgcn_readlane(int(v), int(l))); }
DEV uint32_t first_lane(u64 m) { return uint32_t(__ffsll((long long)m) - 1); }
DEV uint32_t last_lane(u64 m) { return 63u - uint32_t(__clzll((long long)m)); }
// Wave-uniform values pinned to scalar registers (scalar control flow, no exec-mask loops).
DEV uint32_t U(uint32_t v) { return uint32_t(__builtin_amdgcn_readfirstlane(int(v))); }
DEV uint32_t shfl(uint32_t v, uint32_t src) {
    return uint32_t(__builtin_amdgcn_ds_bpermute(int(src << 2), int(v)));
}
DEV u64 lanes_below(uint32_t l) { return l >= 64 ? ~0ull : ((1ull << l) - 1ull); }
// Inclusive wave prefix sum (DPP row_shr 1/2/4/8, row_bcast 15/31; as dt_replay.hip).
DEV uint32_t wave_scan(uint32_t x) {
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x142, 0xA, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x143, 0xC, 0xF, false));
    return x;
}
DEV uint32_t wave_sum(uint32_t v) { return U(bcast(wave_scan(v), 63)); }
DEV u64 wave_sum64(u64 v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}
// Number of lanes whose (non-decreasing across lanes) `inc` is <= x: for a lane-prefix-sum
// `inc`, the lane whose range [inc - c, inc) holds x.  Per lane (x may differ between lanes).
DEV uint32_t lane_search(uint32_t inc, uint32_t x) {
    uint32_t s = 0;
#pragma unroll
    for (uint32_t st = 32; st; st >>= 1)
        if (shfl(inc, s + st - 1) <= x) s += st;
    return s;
}
DEV u64 splitmix(u64 z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
DEV uint32_t utf8_len(uint8_t c) { return c < 0x80 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : 4; }

constexpr uint32_t NS = SPAN_NS;   // span slots per block
constexpr uint32_t SBC = 64;       // block capacity of a superblock list
constexpr uint32_t ROOT_ID = 0xFFFFFFFFu;
constexpr uint32_t END_ID = 0xFFFFFFFEu;
constexpr uint32_t NONE = 0xFFFFFFFFu;
// span word (high half of the 8-byte span): len | ever_deleted << 20 | state << 21
constexpr uint32_t LEN_MASK = (1u << 20) - 1;
constexpr uint32_t ED_BIT = 1u << 20;
constexpr uint32_t ST_SHIFT = 21;
constexpr uint32_t ST_MAX = (1u << 11) - 1;
DEV uint32_t s_len(uint32_t w) { return w & LEN_MASK; }
DEV uint32_t s_st(uint32_t w) { return w >> ST_SHIFT; }
DEV uint32_t s_vis(uint32_t w) { return s_st(w) == 1 ? s_len(w) : 0u; }
DEV uint32_t with_len(uint32_t w, uint32_t len) { return (w & ~LEN_MASK) | len; }
// block meta word: spans | live (non-NIY) spans << 8
constexpr uint32_t M_LIVE = 1u << 8;
DEV uint32_t m_n(uint32_t m) { return m & 0xFFu; }
DEV uint32_t m_live(uint32_t m) { return (m >> 8) & 0xFFu; }

enum ProfSlot { P_INS = 0, P_DEL, P_TOG, P_MAT, P_YJS, P_SPLIT, P_FIND, P_BLOAD, P_ORR, P_RUN, P_HIT, P_RUNS, P_RELINK,
                P_N_YJS, P_N_SPLIT, P_T1, P_T2, P_T3, P_N };

// Hot per-document state: scalars the command loop touches (the compiler keeps them in SGPRs).
struct Doc {
    const Cmd *cmds;
    uint32_t ncmd, n_lv;
    const uint32_t *tlist;
    uint32_t *lk;   // insert LV: its block; delete LV: the item it deleted
    u64 *ao;        // insert LV: origin_left | origin_right << 32
    u64 *rows;      // NS spans per block
    uint32_t *ix;   // index base (LDS tiers: the workgroup's dynamic LDS; HBM tier: gidx)
    uint32_t mb, ms;   // HBM tier: the index's block / superblock capacity (LDS tiers: MB, span_lds_sb(MB))
    uint32_t nb, nsb;
    uint32_t err, ci;
    uint32_t debug, slow, trace, dump_at, dump_n;
    uint32_t steps, step_limit;   // watchdog: a bound violation ends the document with ErrCapacity
    // the last insert / delete's block: its row in registers (lane = slot), span count, visible
    // items, top position of its superblock and the visible rank of its first item.  Typing keeps
    // hitting it, so the next command skips the index walk and the row load.  Memory holds the
    // same state (every change is stored).  cb == NONE: nothing cached.
    uint32_t cb, cn, ccnt, ctp, cbase;
    uint32_t crl, crw;
};
// Cold per-document state, in LDS (read on rare paths: YjsMod, splits, materialisation, errors).
struct Cold {
    const uint32_t *cbyte;
    const uint8_t *content;
    const uint32_t *aruns;
    uint32_t *fb_list, *fb_count;   // LDS tier: capacity-overflow queue for the HBM tier
    uint32_t n_aruns, ascii, doc, site, n_items, max_blocks, max_sb;
    uint64_t prof[P_N];
};
__shared__ Cold g_cold;

DEV void fail(Doc &D, uint32_t code, uint32_t site) {
    if (!D.err) { D.err = code; g_cold.site = site; }
}
DEV bool charge(Doc &D) {
    if (++D.steps > D.step_limit) { fail(D, ErrCapacity, 1); return false; }
    return true;
}
template <bool PROF> DEV uint64_t tick() { return PROF ? __builtin_amdgcn_s_memtime() : 0; }

// Index layout (bind order, span_index_bytes): u32 cnt[mb], meta[mb]; by top position tv, tl,
// ts, tn [ms]; by superblock sbn, sbpos [ms]; then opos[mb] and sbl[64 ms] (u16 in LDS, u32 in
// HBM).  LDS tiers have compile-time capacities, so every offset is an immediate.
template <uint32_t MB> DEV uint32_t mb_of(const Doc &D) { return MB ? MB : D.mb; }
template <uint32_t MB> DEV uint32_t ms_of(const Doc &D) { return MB ? span_lds_sb(MB) : D.ms; }
template <uint32_t MB> DEV uint32_t *CNT(const Doc &D) { return D.ix; }
template <uint32_t MB> DEV uint32_t *META(const Doc &D) { return D.ix + mb_of<MB>(D); }
template <uint32_t MB> DEV uint32_t *TV(const Doc &D) { return D.ix + 2 * mb_of<MB>(D); }
template <uint32_t MB> DEV uint32_t *TL(const Doc &D) { return TV<MB>(D) + ms_of<MB>(D); }
template <uint32_t MB> DEV uint32_t *TS(const Doc &D) { return TV<MB>(D) + 2 * ms_of<MB>(D); }
template <uint32_t MB> DEV uint32_t *TN(const Doc &D) { return TV<MB>(D) + 3 * ms_of<MB>(D); }
template <uint32_t MB> DEV uint32_t *SBN(const Doc &D) { return TV<MB>(D) + 4 * ms_of<MB>(D); }
template <uint32_t MB> DEV uint32_t *SBPOS(const Doc &D) { return TV<MB>(D) + 5 * ms_of<MB>(D); }
template <uint32_t MB> DEV uint32_t *EXT(const Doc &D) { return TV<MB>(D) + 6 * ms_of<MB>(D); }
template <uint32_t MB> DEV uint32_t opos_of(const Doc &D, uint32_t b) {
    if (MB) return reinterpret_cast<const uint16_t *>(EXT<MB>(D))[b];
    return EXT<MB>(D)[b];
}
template <uint32_t MB> DEV void set_opos(Doc &D, uint32_t b, uint32_t v) {
    if (MB) reinterpret_cast<uint16_t *>(EXT<MB>(D))[b] = uint16_t(v);
    else EXT<MB>(D)[b] = v;
}
template <uint32_t MB> DEV uint32_t sbl_at(const Doc &D, size_t i) {
    if (MB) return reinterpret_cast<const uint16_t *>(EXT<MB>(D))[mb_of<MB>(D) + i];
    return EXT<MB>(D)[mb_of<MB>(D) + i];
}
template <uint32_t MB> DEV void set_sbl(Doc &D, size_t i, uint32_t v) {
    if (MB) reinterpret_cast<uint16_t *>(EXT<MB>(D))[mb_of<MB>(D) + i] = uint16_t(v);
    else EXT<MB>(D)[mb_of<MB>(D) + i] = v;
}
// Index counter update from one lane.  LDS tiers: a returnless LDS atomic (fire and forget: no
// read-back round trip on the command's critical path).  HBM tier: plain read-modify-write (the
// wave owns the document; a global atomic would leave L2 as a memory-side request).
template <uint32_t MB> DEV void ix_add(uint32_t *p, uint32_t v) {
    if (MB) __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else *p += v;
}
template <uint32_t MB> DEV uint32_t top_of(const Doc &D, uint32_t b) { return U(SBPOS<MB>(D)[U(opos_of<MB>(D, b)) >> 6]); }

// ---- rows ------------------------------------------------------------------------------------

DEV void load_row(const Doc &D, uint32_t b, uint32_t n, uint32_t &rl, uint32_t &rw) {
    const u64 v = D.rows[size_t(b) * NS + lane_id()];
    rl = uint32_t(v);
    rw = lane_id() < n ? uint32_t(v >> 32) : 0u;
}
template <uint32_t MB> DEV void get_row(const Doc &D, uint32_t b, uint32_t &rl, uint32_t &rw, uint32_t &n) {
    if (b == D.cb) {
        rl = D.crl; rw = D.crw; n = D.cn;
        return;
    }
    const u64 v = D.rows[size_t(b) * NS + lane_id()];   // issued before the count it is masked by
    n = U(m_n(META<MB>(D)[b]));
    rl = uint32_t(v);
    rw = lane_id() < n ? uint32_t(v >> 32) : 0u;
}
DEV void store_row(Doc &D, uint32_t b, uint32_t rl, uint32_t rw, uint32_t from, uint32_t n) {
    const uint32_t l = lane_id();
    if (l >= from && l < n) D.rows[size_t(b) * NS + l] = u64(rl) | (u64(rw) << 32);
}
// Slot j of the k-th visible item of a row and its offset o in that span (j = 64: none).
DEV void row_find_vis(uint32_t rw, uint32_t k, uint32_t &j, uint32_t &o) {
    const uint32_t v = s_vis(rw);
    const uint32_t inc = wave_scan(v);
    const u64 m = __ballot(inc > k);
    j = m ? first_lane(m) : 64u;
    o = m ? U(k - bcast(inc - v, j)) : 0u;
}

// ---- navigation ------------------------------------------------------------------------------

template <uint32_t MB> DEV uint32_t first_block(const Doc &D) { return U(sbl_at<MB>(D, size_t(U(TS<MB>(D)[0])) * SBC)); }
// Next block in document order, or NONE.
template <uint32_t MB> DEV uint32_t next_block(const Doc &D, uint32_t b) {
    const uint32_t o = U(opos_of<MB>(D, b));
    const uint32_t S = o >> 6, i = o & 63u;
    if (i + 1 < U(SBN<MB>(D)[S])) return U(sbl_at<MB>(D, size_t(S) * SBC + i + 1));
    const uint32_t p = U(SBPOS<MB>(D)[S]) + 1;
    if (p >= D.nsb) return NONE;
    return U(sbl_at<MB>(D, size_t(U(TS<MB>(D)[p])) * SBC));
}
// The block holding visible index p, the top position of its superblock and the visible rank of
// its first item (content-tree cursor_at_content_pos, root.rs:50-89): prefix scans over the
// superblock totals, then over the chosen superblock's block counts.
template <uint32_t MB> DEV bool find_block(Doc &D, uint32_t p, uint32_t &b, uint32_t &tp, uint32_t &base_out) {
    const uint32_t l = lane_id();
    uint32_t base = 0;
    for (uint32_t c = 0; c < D.nsb; c += 64) {
        const uint32_t i = min(c + l, D.nsb - 1);   // clamped, then masked: no exec branch
        const uint32_t v0 = TV<MB>(D)[i], s0 = TS<MB>(D)[i], n0 = TN<MB>(D)[i];
        const uint32_t v = c + l < D.nsb ? v0 : 0;
        const uint32_t inc = wave_scan(v);
        const u64 m = __ballot(base + inc > p);
        if (m) {
            const uint32_t fl = first_lane(m);
            const uint32_t S = U(bcast(s0, fl)), n = U(bcast(n0, fl));
            tp = U(c + fl);
            base += U(bcast(inc - v, fl));
            const uint32_t bl0 = sbl_at<MB>(D, size_t(S) * SBC + l);   // a list row holds SBC slots
            const uint32_t bl = l < n ? bl0 : 0;
            const uint32_t w0 = CNT<MB>(D)[bl];
            const uint32_t w = l < n ? w0 : 0;
            const uint32_t inc2 = wave_scan(w);
            const u64 m2 = __ballot(base + inc2 > p);
            if (!m2) return false;
            const uint32_t f2 = first_lane(m2);
            b = U(bcast(bl, f2));
            base_out = U(base + bcast(inc2 - w, f2));
            return true;
        }
        base += U(bcast(inc, 63));
    }
    return false;
}
// First block after b (document order) with a live span, or NONE (origin_right search,
// merge.rs:405-423).
template <uint32_t MB> DEV uint32_t next_live_block(Doc &D, uint32_t b) {
    const uint32_t l = lane_id();
    const uint32_t o = U(opos_of<MB>(D, b));
    uint32_t S = o >> 6;
    {   // rest of b's superblock
        const uint32_t n = U(SBN<MB>(D)[S]), i0 = (o & 63u) + 1;
        const uint32_t b0 = sbl_at<MB>(D, size_t(S) * SBC + l);
        const uint32_t bl = l < n ? b0 : 0;
        const uint32_t lv = m_live(META<MB>(D)[bl]);
        const u64 m = __ballot(l >= i0 && l < n && lv != 0);
        if (m) return U(bcast(bl, first_lane(m)));
    }
    for (uint32_t p = U(SBPOS<MB>(D)[S]) + 1; p < D.nsb; p += 64) {
        if (!charge(D)) return NONE;
        const uint32_t i = min(p + l, D.nsb - 1);
        const uint32_t tl0 = TL<MB>(D)[i], ts0 = TS<MB>(D)[i], tn0 = TN<MB>(D)[i];
        const u64 m = __ballot(p + l < D.nsb && tl0 != 0);
        if (m) {
            const uint32_t f = first_lane(m);
            S = U(bcast(ts0, f));
            const uint32_t n = U(bcast(tn0, f));
            const uint32_t b0 = sbl_at<MB>(D, size_t(S) * SBC + l);
            const uint32_t bl = l < n ? b0 : 0;
            const uint32_t lv = m_live(META<MB>(D)[bl]);
            const u64 m2 = __ballot(l < n && lv != 0);
            if (!m2) { fail(D, ErrCheckout, 19); return NONE; }
            return U(bcast(bl, first_lane(m2)));
        }
    }
    return NONE;
}
// Document-order key of an inserted item: (top position, index in superblock, slot, offset).
template <uint32_t MB> DEV u64 key_of(Doc &D, uint32_t item) {
    const uint32_t l = lane_id();
    const uint32_t b = U(D.lk[item]);
    if (b >= D.nb) { fail(D, ErrCheckout, 24); return 0; }
    uint32_t rl, rw, n;
    get_row<MB>(D, b, rl, rw, n);
    const u64 m = __ballot(l < n && item >= rl && item - rl < s_len(rw));
    if (!m) { fail(D, ErrCheckout, 24); return 0; }
    const uint32_t j = first_lane(m);
    const uint32_t off = item - U(bcast(rl, j));
    const uint32_t o = U(opos_of<MB>(D, b));
    const uint32_t tp = U(SBPOS<MB>(D)[o >> 6]);
    return (u64(tp) << 32) | (u64(o & 63u) << 26) | (u64(j) << 20) | off;
}

// ---- block maintenance -----------------------------------------------------------------------

// Split the full superblock S (64 blocks): its upper half becomes a new superblock right after it
// in the top order.  The cached block's top position may move: the cache is dropped.
template <uint32_t MB> DEV void split_sb(Doc &D, uint32_t S) {
    const uint32_t l = lane_id();
    if (D.nsb >= g_cold.max_sb) { fail(D, ErrCapacity, 21); return; }
    const uint32_t S2 = D.nsb;
    const uint32_t b = sbl_at<MB>(D, size_t(S) * SBC + l);
    const uint32_t vis = CNT<MB>(D)[b], live = m_live(META<MB>(D)[b]);
    wave_fence();
    if (l >= SBC / 2) {
        set_sbl<MB>(D, size_t(S2) * SBC + (l - SBC / 2), b);
        set_opos<MB>(D, b, (S2 << 6) | (l - SBC / 2));
    }
    const uint32_t vh = wave_sum(l >= 32 ? vis : 0), lh = wave_sum(l >= 32 ? live : 0);
    const uint32_t vl = wave_sum(l < 32 ? vis : 0), ll = wave_sum(l < 32 ? live : 0);
    const uint32_t p = U(SBPOS<MB>(D)[S]) + 1;
    // shift the top arrays [p, nsb) right by one, highest chunk first
    for (int c = int(D.nsb) - 1; c >= int(p); c -= 64) {
        const int i = c - int(l);
        uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
        if (i >= int(p)) { a0 = TV<MB>(D)[i]; a1 = TL<MB>(D)[i]; a2 = TS<MB>(D)[i]; a3 = TN<MB>(D)[i]; }
        wave_fence();
        if (i >= int(p)) {
            TV<MB>(D)[i + 1] = a0; TL<MB>(D)[i + 1] = a1; TS<MB>(D)[i + 1] = a2; TN<MB>(D)[i + 1] = a3;
            SBPOS<MB>(D)[a2] = uint32_t(i + 1);
        }
        wave_fence();
    }
    if (l == 0) {
        SBN<MB>(D)[S] = SBC / 2;
        SBN<MB>(D)[S2] = SBC / 2;
        TV<MB>(D)[p - 1] = vl; TL<MB>(D)[p - 1] = ll; TN<MB>(D)[p - 1] = SBC / 2;
        TV<MB>(D)[p] = vh; TL<MB>(D)[p] = lh; TS<MB>(D)[p] = S2; TN<MB>(D)[p] = SBC / 2;
        SBPOS<MB>(D)[S2] = p;
    }
    wave_fence();
    D.nsb++;
    D.cb = NONE;
}

// lk[] of every LV of the spans with len_l > 0 (lane l: first LV rl, length len) := b.
template <bool PROF> DEV void relink(Doc &D, uint32_t rl, uint32_t len, uint32_t b) {
    const uint32_t l = lane_id();
    const uint32_t inc = wave_scan(len);
    const uint32_t total = U(bcast(inc, 63));
    if (PROF) g_cold.prof[P_RELINK] += total;
    for (uint32_t c = 0; c < total; c += 64) {
        const uint32_t u = c + l;
        const uint32_t s = lane_search(inc, u);
        const uint32_t src = shfl(rl, s) + (u - shfl(inc - len, s));
        if (u < total) D.lk[src] = b;
    }
}

// Split block b (row rl / rw, n spans): spans [n/2, n) move to a new block b2 placed right after
// b in its superblock (content-tree's leaf split; the moved LVs' markers are rewritten).  Returns
// false (document failed) when the block pool is exhausted.
template <uint32_t MB, bool PROF>
DEV bool split_block(Doc &D, uint32_t b, uint32_t rl, uint32_t rw, uint32_t n, uint32_t &b2, uint32_t &cut) {
    const uint32_t l = lane_id();
    const uint64_t t0 = tick<PROF>();
    if (D.nb >= g_cold.max_blocks) { fail(D, ErrCapacity, 12); return false; }
    b2 = D.nb;
    cut = n >> 1;
    const bool mv = l >= cut && l < n;
    if (mv) D.rows[size_t(b2) * NS + (l - cut)] = u64(rl) | (u64(rw) << 32);
    const uint32_t vis = s_vis(rw), live = (l < n && s_st(rw) != 0) ? 1u : 0u;
    const uint32_t vr = wave_sum(mv ? vis : 0), lr = wave_sum(mv ? live : 0);
    const uint32_t vl = wave_sum(l < cut ? vis : 0), ll = wave_sum(l < cut ? live : 0);
    relink<PROF>(D, rl, mv ? s_len(rw) : 0u, b2);
    const uint32_t o = U(opos_of<MB>(D, b));
    const uint32_t S = o >> 6, i = o & 63u, m = U(SBN<MB>(D)[S]);
    {   // shift S's list after i right by one
        uint32_t v = 0;
        const bool sh = l > i && l < m;
        if (sh) v = sbl_at<MB>(D, size_t(S) * SBC + l);
        wave_fence();
        if (sh) {
            set_sbl<MB>(D, size_t(S) * SBC + l + 1, v);
            set_opos<MB>(D, v, (S << 6) | (l + 1));
        }
    }
    if (l == 0) {
        CNT<MB>(D)[b] = vl;
        CNT<MB>(D)[b2] = vr;
        META<MB>(D)[b] = cut | (ll << 8);
        META<MB>(D)[b2] = (n - cut) | (lr << 8);
        set_sbl<MB>(D, size_t(S) * SBC + i + 1, b2);
        set_opos<MB>(D, b2, (S << 6) | (i + 1));
        SBN<MB>(D)[S] = m + 1;
        TN<MB>(D)[SBPOS<MB>(D)[S]] = m + 1;
    }
    wave_fence();
    D.nb++;
    if (D.cb == b) D.cb = NONE;
    if (m + 1 == SBC) split_sb<MB>(D, S);
    if (PROF) { g_cold.prof[P_SPLIT] += tick<PROF>() - t0; g_cold.prof[P_N_SPLIT]++; }
    return D.err == 0;
}

// New row from cutting every lane's span at x1 <= x2 into [0,x1) [x1,x2) [x2,len), empty pieces
// dropped: the middle piece takes word mw's state / flag, the outer ones keep the lane's word.
// Lanes past the row (len 0) produce nothing; the caller guarantees <= NS pieces.
DEV void expand_row(uint32_t &rl, uint32_t &rw, uint32_t x1, uint32_t x2, uint32_t mw) {
    const uint32_t l = lane_id();
    const uint32_t len = s_len(rw);
    const uint32_t c = (x1 > 0 ? 1u : 0u) + (x2 > x1 ? 1u : 0u) + (len > x2 ? 1u : 0u);
    const uint32_t inc = wave_scan(c);
    const uint32_t total = bcast(inc, 63);
    const uint32_t s = min(lane_search(inc, l), 63u);
    const uint32_t q = l - (shfl(inc, s) - shfl(c, s));
    const uint32_t sl = shfl(rl, s), sw = shfl(rw, s), s1 = shfl(x1, s), s2 = shfl(x2, s), sm = shfl(mw, s);
    const uint32_t e0 = s1 > 0 ? 1u : 0u, e1 = s2 > s1 ? 1u : 0u;
    const uint32_t pid = q < e0 ? 0u : (q < e0 + e1 ? 1u : 2u);
    const uint32_t a = pid == 0 ? 0u : (pid == 1 ? s1 : s2);
    const uint32_t e = pid == 0 ? s1 : (pid == 1 ? s2 : s_len(sw));
    const uint32_t w = pid == 1 ? sm : sw;
    const bool on = l < total;
    rl = on ? sl + a : 0u;
    rw = on ? with_len(w, e - a) : 0u;
}

// ---- commands --------------------------------------------------------------------------------

// YjsMod tie-break key of an LV: (agent name rank, seq) (merge.rs:199-218).  64-ary search over
// the agent runs; `lv` is wave-uniform.
DEV void agent_of(Doc &D, uint32_t lv, uint32_t &rank, uint32_t &seq) {
    const uint32_t l = lane_id();
    uint32_t lo = 0, n = g_cold.n_aruns;   // last run with start <= lv lies in [lo, lo+n)
    while (n > 64) {
        if (!charge(D)) { rank = seq = 0; return; }
        const uint32_t stride = (n + 63) / 64;
        const uint32_t idx = lo + l * stride;
        const bool ok = l * stride < n && g_cold.aruns[4 * idx] <= lv;
        const uint32_t k = uint32_t(__popcll(__ballot(ok)));
        const uint32_t nlo = lo + (k ? k - 1 : 0) * stride;
        n = min(stride, lo + n - nlo);
        lo = nlo;
    }
    const bool ok = l < n && g_cold.aruns[4 * (lo + l)] <= lv;
    const uint32_t k = uint32_t(__popcll(__ballot(ok)));
    const uint32_t j = U(lo + (k ? k - 1 : 0));
    rank = U(g_cold.aruns[4 * j + 1]);
    seq = U(g_cold.aruns[4 * j + 2]) + (lv - U(g_cold.aruns[4 * j]));
}

// YjsMod integrate (merge.rs:154-278): scan the not-inserted-yet spans from the cursor (b, s) up
// to origin_right's span (rb, rs) (rb == NONE: END), one span at a time like the reference (the
// inner items of a span always compare Greater, merge.rs:243-258).  Returns the insertion point.
template <uint32_t MB>
DEV void yjs_scan(Doc &D, uint32_t &b, uint32_t &s, uint32_t rb, uint32_t rs, uint32_t ol, uint32_t orr, uint32_t lv) {
    const u64 my_l = ol == ROOT_ID ? 0ull : key_of<MB>(D, ol) + 1ull;
    const u64 my_r = orr == END_ID ? ~0ull : key_of<MB>(D, orr);
    uint32_t nr, nq;
    agent_of(D, lv, nr, nq);
    bool scanning = false;
    uint32_t sb0 = 0, ss0 = 0;
    uint32_t cb = b, cs = s;
    uint32_t rl, rw, n;
    get_row<MB>(D, cb, rl, rw, n);
    while (!D.err) {
        if (!charge(D)) return;
        if (cs >= n) {
            const uint32_t nx = next_block<MB>(D, cb);
            if (nx == NONE) break;   // end of the document
            cb = nx;
            cs = 0;
            get_row<MB>(D, cb, rl, rw, n);
            continue;
        }
        if (cb == rb && cs == rs) break;   // reached origin_right
        const uint32_t o = U(bcast(rl, cs));
        if (s_st(U(bcast(rw, cs))) != 0) { fail(D, ErrCheckout, 25); return; }
        const u64 x = D.ao[o];
        const uint32_t ol_o = U(uint32_t(x)), orr_o = U(uint32_t(x >> 32));
        const u64 kl = ol_o == ROOT_ID ? 0ull : key_of<MB>(D, ol_o) + 1ull;
        if (kl < my_l) break;   // insert before o
        if (kl == my_l) {
            if (orr_o == orr) {   // concurrent: order by agent name, then seq
                uint32_t r2, q2;
                agent_of(D, o, r2, q2);
                if (nr < r2 || (nr == r2 && nq < q2)) break;
                scanning = false;
            } else {
                const u64 kr = orr_o == END_ID ? ~0ull : key_of<MB>(D, orr_o);
                if (kr < my_r) {
                    if (!scanning) { scanning = true; sb0 = cb; ss0 = cs; }
                } else {
                    scanning = false;
                }
            }
        }
        cs++;
    }
    if (scanning) { b = sb0; s = ss0; }
    else { b = cb; s = cs; }
}

// Apply an insert run at visible position pos (M2Tracker::apply Ins + integrate,
// merge.rs:154-278, 383-455).
template <uint32_t MB, bool PROF>
DEV void do_insert(Doc &D, uint32_t lv, uint32_t k, uint32_t pos) {
    const uint32_t l = lane_id();
    uint64_t tq = tick<PROF>();
    uint32_t b, tp = 0, base = 0;
    bool known = true;   // base / tp valid for the insertion block (the cache can take it)
    if (pos == 0) {
        b = first_block<MB>(D);
    } else {
        const uint32_t q = pos - 1;
        if (D.cb != NONE && q >= D.cbase && q - D.cbase < D.ccnt) {
            b = D.cb; tp = D.ctp; base = D.cbase;
            if (PROF) g_cold.prof[P_HIT]++;
        } else if (!find_block<MB>(D, q, b, tp, base)) {
            fail(D, ErrCheckout, 13);
            return;
        }
    }
    if (PROF) { const uint64_t t = tick<PROF>(); g_cold.prof[P_FIND] += t - tq; tq = t; }
    uint32_t rl, rw, n;
    get_row<MB>(D, b, rl, rw, n);
    uint32_t s = 0, j = 0, o = 0;
    uint32_t ol = ROOT_ID, orr = END_ID;
    bool mid = false;
    if (pos) {
        row_find_vis(rw, pos - 1 - base, j, o);
        if (j >= n) { fail(D, ErrCheckout, 13); return; }
        const uint32_t wj = U(bcast(rw, j));
        ol = U(bcast(rl, j)) + o;
        if (o + 1 < s_len(wj)) { mid = true; orr = ol + 1; }   // the next item is live: direct
        s = j + 1;
    }
    if (PROF) { const uint64_t t = tick<PROF>(); g_cold.prof[P_BLOAD] += t - tq; tq = t; }
    bool direct = mid;
    if (!mid) {
        // origin_right: first live span at or after the cursor (possibly a deleted one)
        uint32_t rb = NONE, rs = 0;
        const u64 m = __ballot(l >= s && l < n && s_st(rw) != 0);
        if (m) {
            rb = b;
            rs = first_lane(m);
            orr = U(bcast(rl, rs));
            direct = rs == s;
        } else {
            rb = next_live_block<MB>(D, b);
            if (D.err) return;
            if (rb != NONE) {
                uint32_t xl, xw, xn;
                get_row<MB>(D, rb, xl, xw, xn);
                const u64 m2 = __ballot(l < xn && s_st(xw) != 0);
                if (!m2) { fail(D, ErrCheckout, 19); return; }
                rs = first_lane(m2);
                orr = U(bcast(xl, rs));
            }
            // direct iff no span lies between the cursor and origin_right
            if (s >= n) {
                const uint32_t nx = next_block<MB>(D, b);
                direct = rb == NONE ? nx == NONE : (nx == rb && rs == 0);
            }
        }
        if (PROF) { const uint64_t t = tick<PROF>(); g_cold.prof[P_ORR] += t - tq; tq = t; }
        if (!direct) {
            const uint32_t b0 = b;
            yjs_scan<MB>(D, b, s, rb, rs, ol, orr, lv);
            if (D.err) return;
            if (b != b0) {
                get_row<MB>(D, b, rl, rw, n);
                known = false;
            }
            if (PROF) { const uint64_t t = tick<PROF>(); g_cold.prof[P_YJS] += t - tq; tq = t; g_cold.prof[P_N_YJS]++; }
        }
    }
    // place the run as spans of <= LEN_MASK items each, consecutively from slot s (a mid-span
    // insert first cuts span j after offset o)
    uint32_t left = k, at = lv;
    while (left > 0 && !D.err) {
        const uint32_t kk = min(left, LEN_MASK);
        const uint32_t grow = mid ? 2u : 1u;
        if (n + grow > NS) {
            uint32_t b2, cut;
            if (!split_block<MB, PROF>(D, b, rl, rw, n, b2, cut)) return;
            const uint32_t vleft = wave_sum(l < cut ? s_vis(rw) : 0u);
            if (s > cut) {   // the insertion point moved to the new block
                b = b2;
                s -= cut;
                if (mid) j -= cut;
                rl = shfl(rl, (l + cut) & 63u);
                const uint32_t w2 = shfl(rw, (l + cut) & 63u);
                rw = l + cut < n ? w2 : 0u;
                n -= cut;
                base += vleft;
            } else {
                rw = l < cut ? rw : 0u;
                n = cut;
            }
            tp = top_of<MB>(D, b);
            continue;
        }
        uint32_t nl, nw;
        const uint32_t from = mid ? j : s;
        if (mid) {   // slot j: [lv0, o+1); j+1: the run; j+2: the rest of span j; then the old j+1..
            const uint32_t src = l <= j + 2 ? j : l - 2;
            const uint32_t xl = shfl(rl, src), xw = shfl(rw, src);
            if (l < j) { nl = rl; nw = rw; }
            else if (l == j) { nl = rl; nw = with_len(rw, o + 1); }
            else if (l == j + 1) { nl = at; nw = kk | (1u << ST_SHIFT); }
            else if (l == j + 2) { nl = xl + o + 1; nw = with_len(xw, s_len(xw) - o - 1); }
            else { nl = xl; nw = xw; }
        } else {
            const uint32_t src = (l - 1) & 63u;
            const uint32_t xl = shfl(rl, src), xw = shfl(rw, src);
            nl = l < s ? rl : (l == s ? at : xl);
            nw = l < s ? rw : (l == s ? (kk | (1u << ST_SHIFT)) : (l > 0 ? xw : 0u));
        }
        store_row(D, b, nl, nw, from, n + grow);
        for (uint32_t c = 0; c < kk; c += 64) {
            const uint32_t i = c + l;
            if (i < kk) {
                D.lk[at + i] = b;
                D.ao[at + i] = u64(at + i == lv ? ol : at + i - 1) | (u64(orr) << 32);
            }
        }
        if (l == 0) {
            ix_add<MB>(&CNT<MB>(D)[b], kk);
            ix_add<MB>(&META<MB>(D)[b], grow * (1u + M_LIVE));
            if (known) { ix_add<MB>(&TV<MB>(D)[tp], kk); ix_add<MB>(&TL<MB>(D)[tp], grow); }
        }
        if (!known) {   // after a YjsMod scan moved the insertion point: its top position
            if (l == 0) {
                const uint32_t t2 = SBPOS<MB>(D)[opos_of<MB>(D, b) >> 6];
                ix_add<MB>(&TV<MB>(D)[t2], kk);
                ix_add<MB>(&TL<MB>(D)[t2], grow);
            }
        }
        wave_fence();
        rl = nl; rw = nw; n += grow;
        s = (mid ? j + 2 : s + 1);
        if (mid) { j = s - 1; mid = false; }
        at += kk;
        left -= kk;
    }
    if (D.err) return;
    if (known) {
        D.cb = b; D.cn = n; D.ccnt = wave_sum(s_vis(rw)); D.ctp = tp; D.cbase = base;
        D.crl = rl; D.crw = rw;
    } else {
        D.cb = NONE;
    }
    if (PROF) g_cold.prof[P_RUN] += tick<PROF>() - tq;
}

// Apply a delete run: n visible items from position pos (merge.rs:457-556).  LV lv+j targets
// the j-th item (fwd) or the (n-1-j)-th item (reversed / backspace runs, op_metrics.rs:184-202).
template <uint32_t MB, bool PROF>
DEV void do_delete(Doc &D, uint32_t lv, uint32_t n_del, uint32_t pos, bool fwd) {
    const uint32_t l = lane_id();
    uint32_t done = 0;
    while (done < n_del) {   // each round deletes >= 1 item, splits a block, or fails
        if (!charge(D)) return;
        uint32_t b, tp, base;
        if (D.cb != NONE && pos >= D.cbase && pos - D.cbase < D.ccnt) {
            b = D.cb; tp = D.ctp; base = D.cbase;
            if (PROF) g_cold.prof[P_HIT]++;
        } else if (!find_block<MB>(D, pos, b, tp, base)) {
            fail(D, ErrCheckout, 14);
            return;
        }
        uint32_t rl, rw, n;
        get_row<MB>(D, b, rl, rw, n);
        const uint32_t kk = pos - base;
        const uint32_t len = s_len(rw), v = s_vis(rw);
        const uint32_t inc = wave_scan(v), ex = inc - v;
        const uint32_t bvis = U(bcast(inc, 63));
        if (kk >= bvis) { fail(D, ErrCheckout, 15); return; }
        const uint32_t take = min(n_del - done, bvis - kk);
        const uint32_t lo = kk, hi = kk + take;   // the block's visible range [lo, hi) goes
        const bool cov = v > 0 && inc > lo && ex < hi;
        const uint32_t x1 = cov ? (lo > ex ? lo - ex : 0u) : len;
        const uint32_t x2 = cov ? (hi < inc ? hi - ex : len) : len;
        const uint32_t pieces = (x1 > 0 ? 1u : 0u) + (x2 > x1 ? 1u : 0u) + (len > x2 ? 1u : 0u);
        const uint32_t grow = wave_sum(pieces) - n;
        if (n + grow > NS) {
            uint32_t b2, cut;
            if (!split_block<MB, PROF>(D, b, rl, rw, n, b2, cut)) return;
            D.cb = NONE;
            continue;   // locate again
        }
        // targets: deleted ordinal u (document order) = visible index lo + u of this block
        const u64 cm = __ballot(cov);
        const uint32_t d0 = done;
        if ((cm & (cm - 1)) == 0) {   // one span: consecutive items
            const uint32_t f = first_lane(cm);
            const uint32_t t0 = U(bcast(rl, f)) + (lo - U(bcast(ex, f)));
            for (uint32_t c = 0; c < take; c += 64) {
                const uint32_t u = c + l;
                if (u < take) D.lk[fwd ? lv + d0 + u : lv + n_del - 1 - (d0 + u)] = t0 + u;
            }
        } else {
            for (uint32_t c = 0; c < take; c += 64) {
                const uint32_t u = c + l;
                const uint32_t q = lo + u;
                const uint32_t sj = min(lane_search(inc, q), 63u);
                const uint32_t item = shfl(rl, sj) + (q - shfl(ex, sj));
                if (u < take) D.lk[fwd ? lv + d0 + u : lv + n_del - 1 - (d0 + u)] = item;
            }
        }
        // visible (1) -> deleted once (2), ever_deleted
        const uint32_t mw = (rw & LEN_MASK) | (2u << ST_SHIFT) | ED_BIT;
        if (grow) expand_row(rl, rw, x1, x2, mw);
        else if (cov) rw = mw;
        const uint32_t from = first_lane(cm);
        store_row(D, b, rl, rw, from, n + grow);
        if (l == 0) {
            ix_add<MB>(&CNT<MB>(D)[b], 0u - (take));
            ix_add<MB>(&META<MB>(D)[b], grow * (1u + M_LIVE));   // every piece of a visible span is live
            ix_add<MB>(&TV<MB>(D)[tp], 0u - (take));
            ix_add<MB>(&TL<MB>(D)[tp], grow);
        }
        wave_fence();
        D.cb = b; D.cn = n + grow; D.ccnt = bvis - take; D.ctp = tp; D.cbase = base;
        D.crl = rl; D.crw = rw;
        done += take;
    }
}

// One toggle run: items [lo, hi] (all in block b) get state += d (kd bit 1: advance; bit 0: a
// delete's targets).  The spans covering them are cut to the run's bounds (<= 2 cuts).  ckey:
// document-order key of the cached block (its base moves with changes before it).
template <uint32_t MB, bool PROF>
DEV void apply_run(Doc &D, uint32_t b, uint32_t lo, uint32_t hi, uint32_t kd, uint32_t ckey, bool &relinked) {
    const uint32_t l = lane_id();
    const uint32_t d = (kd & 2u) ? 1u : 0xFFFFFFFFu;
    uint32_t rl, rw, n;
    get_row<MB>(D, b, rl, rw, n);
    uint32_t hb[2] = {b, 0};
    int halves = 1;
    for (int h = 0; h < halves; h++) {
        if (h == 1) {   // the upper half of a block split below
            b = hb[1];
            get_row<MB>(D, b, rl, rw, n);
        }
        const uint32_t len = s_len(rw), st = s_st(rw);
        const bool ov = len > 0 && rl <= hi && rl + len > lo;
        const uint32_t x1 = ov ? (lo > rl ? lo - rl : 0u) : len;
        const uint32_t x2 = ov ? (hi + 1 < rl + len ? hi + 1 - rl : len) : len;
        const uint32_t pieces = (x1 > 0 ? 1u : 0u) + (x2 > x1 ? 1u : 0u) + (len > x2 ? 1u : 0u);
        const uint32_t grow = wave_sum(pieces) - n;
        if (n + grow > NS) {
            if (halves == 2) { fail(D, ErrCheckout, 26); return; }
            uint32_t b2, cut;
            if (!split_block<MB, PROF>(D, b, rl, rw, n, b2, cut)) return;
            relinked = true;
            D.cb = NONE;
            hb[1] = b2;
            halves = 2;
            rw = l < cut ? rw : 0u;
            n = cut;
            h--;   // redo this half with the lower part
            continue;
        }
        const uint32_t nst = st + d;
        if (__ballot(ov && (st == 0 ? d != 1u : nst > ST_MAX))) { fail(D, ErrCheckout, 16); return; }
        const uint32_t mw = (rw & ~(0x7FFu << ST_SHIFT)) | (nst << ST_SHIFT) | ((kd == 3u) ? ED_BIT : 0u);
        const uint32_t w_in = x2 - x1;
        const int32_t dv1 = ov ? (int32_t(nst == 1) - int32_t(st == 1)) * int32_t(w_in) : 0;
        const uint32_t lin = (l < n && st != 0) ? 1u : 0u;
        const uint32_t lout = st != 0 ? ((x1 > 0 ? 1u : 0u) + (len > x2 ? 1u : 0u)) : 0u;
        const uint32_t lmid = (ov && nst != 0) || (!ov && x2 > x1 && st != 0) ? 1u : 0u;
        const uint32_t dv = wave_sum(uint32_t(dv1));
        const uint32_t dl = wave_sum(lout + lmid - lin);
        const u64 om = __ballot(ov);
        if (!om) continue;
        if (grow) expand_row(rl, rw, x1, x2, mw);
        else if (ov) rw = mw;
        store_row(D, b, rl, rw, first_lane(om), n + grow);
        const uint32_t o = U(opos_of<MB>(D, b));
        const uint32_t tp = U(SBPOS<MB>(D)[o >> 6]);
        if (l == 0) {
            ix_add<MB>(&CNT<MB>(D)[b], dv);
            ix_add<MB>(&META<MB>(D)[b], grow + (dl << 8));
            ix_add<MB>(&TV<MB>(D)[tp], dv);
            ix_add<MB>(&TL<MB>(D)[tp], dl);
        }
        wave_fence();
        if (b == D.cb) {
            D.crl = rl; D.crw = rw; D.cn = n + grow; D.ccnt += dv;
        } else if (D.cb != NONE && dv != 0 && ((tp << 6) | (o & 63u)) < ckey) {
            D.cbase += dv;
        }
    }
}

// One walk step's retreat + advance set (advance_retreat.rs:58-153).  Entry: LV | is_del << 30 |
// advance << 31.  `pre` is the first 64-entry chunk when the caller prefetched it (have_pre).
// Per 64 entries: gather the items (a delete LV's target) and their blocks, cut the lanes into
// runs of contiguous items of one kind in one block, then visit each distinct block once: its
// row is loaded and every run in it applied in one lane-parallel pass when each touched span is
// covered whole by one run (the common case: toggles retreat / advance whole earlier edits),
// else run by run with cuts (apply_run).
template <uint32_t MB, bool PROF>
DEV void toggle_pass(Doc &D, uint32_t off, uint32_t n, uint32_t pre, bool have_pre) {
    const uint32_t l = lane_id();
    if (n == 0) return;
    uint64_t tq = tick<PROF>();
    const uint32_t last = off + n - 1;
    uint32_t ckey = 0;
    if (D.cb != NONE) {
        const uint32_t o = U(opos_of<MB>(D, D.cb));
        ckey = (U(SBPOS<MB>(D)[o >> 6]) << 6) | (o & 63u);
    }
    uint32_t e = have_pre ? pre : D.tlist[min(off + l, last)];
    for (uint32_t c = 0; c < n; c += 64) {
        const bool valid = c + l < n;
        const uint32_t x = e & 0x3FFFFFFFu;
        const uint32_t kd = (e >> 30) & 3u;   // bit 0: a delete's target, bit 1: advance
        bool bad = valid && x >= D.n_lv;
        const uint32_t xs = valid && !bad ? x : 0u;
        const uint32_t t = D.lk[xs];   // block of an insert LV / target of a delete LV
        const bool isdel = (kd & 1u) != 0;
        bad = bad || (valid && isdel && t >= D.n_lv);
        const uint32_t item = valid && !bad ? (isdel ? t : xs) : 0u;
        uint32_t blk = t;
        if (isdel) blk = D.lk[item];
        if (c + 64 < n) e = D.tlist[min(off + c + 64 + l, last)];   // next chunk, in flight
        if (__ballot(bad || (valid && blk >= D.nb))) { fail(D, ErrCheckout, 16); return; }
        if (PROF) { const uint64_t t2 = tick<PROF>(); g_cold.prof[P_T1] += t2 - tq; tq = t2; }
        const u64 vm = __ballot(valid);
        // runs: consecutive lanes of one kind and block whose items step by +1 (or all by -1)
        auto heads_of = [&](uint32_t bk) -> u64 {
            const uint32_t pl = (l - 1) & 63u;
            const uint32_t pi = shfl(item, pl), pb = shfl(bk, pl), pk = shfl(kd, pl);
            const bool asc = item == pi + 1, desc = item + 1 == pi;
            const bool c0 = l > 0 && valid && bk == pb && kd == pk && (asc || desc);
            const uint32_t pc0 = shfl(c0 ? 1u : 0u, pl), pasc = shfl(asc ? 1u : 0u, pl);
            const bool cont = c0 && !(pc0 && ((pasc != 0) != asc));
            return __ballot(valid && !cont);
        };
        u64 heads = heads_of(blk);
        u64 pend = vm;
        uint32_t nB = NONE, nrl = 0, nrw = 0, nn = 0;   // the next distinct block's row, in flight
        u64 bound = heads | ~vm;   // run boundaries: run starts and lanes outside the runs
        auto tail_of = [&](uint32_t hl) -> uint32_t {
            const u64 after = bound & ~lanes_below(hl + 1);
            return after ? first_lane(after) - 1 : 63u;
        };
        while (pend) {
            if (!charge(D)) return;
            const uint32_t B = U(bcast(blk, first_lane(pend)));
            const u64 inB = __ballot(valid && blk == B) & pend;
            const u64 hb = heads & inB;
            // one pass over B's row: per span, the runs overlapping it
            uint32_t rl, rw, nsp;
            if (B == nB) {
                rl = nrl; rw = l < nn ? nrw : 0u; nsp = nn;
            } else {
                get_row<MB>(D, B, rl, rw, nsp);
            }
            nB = NONE;
            {   // issue the next distinct block's row load before working on this one
                const u64 rest = pend & ~inB;
                if (rest) {
                    const uint32_t B2 = U(bcast(blk, first_lane(rest)));
                    if (B2 != D.cb) {
                        const u64 v = D.rows[size_t(B2) * NS + l];
                        nrl = uint32_t(v);
                        nrw = uint32_t(v >> 32);
                        nn = U(m_n(META<MB>(D)[B2]));
                        nB = B2;
                    }
                }
            }
            const uint32_t len = s_len(rw), st = s_st(rw);
            uint32_t nov = 0, dd = 0, kk = 0;
            bool part = false;
            for (u64 h = hb; h; h &= h - 1) {
                const uint32_t hl = first_lane(h);
                const uint32_t tl_ = tail_of(hl);
                const uint32_t ih = U(bcast(item, hl)), it = U(bcast(item, tl_)), k2 = U(bcast(kd, hl));
                const uint32_t lo = min(ih, it), hi = max(ih, it);
                const bool ov = len > 0 && rl <= hi && rl + len > lo;
                const bool full = rl >= lo && rl + len <= hi + 1;
                nov += ov ? 1u : 0u;
                part = part || (ov && !full);
                if (ov) { dd = (k2 & 2u) ? 1u : 0xFFFFFFFFu; kk = k2; }
            }
            if (PROF) g_cold.prof[P_RUNS] += uint32_t(__popcll(hb));
            bool relinked = false;
            if (__ballot(part || nov > 1) || D.slow) {   // cuts needed: run by run
                for (u64 h = hb; h; h &= h - 1) {
                    const uint32_t hl = first_lane(h);
                    const uint32_t tl_ = tail_of(hl);
                    const uint32_t ih = U(bcast(item, hl)), it = U(bcast(item, tl_));
                    bool rel = false;
                    apply_run<MB, PROF>(D, B, min(ih, it), max(ih, it), U(bcast(kd, hl)), ckey, rel);
                    if (D.err) return;
                    if (rel) {   // B split: the rest of its runs may sit in either half
                        relinked = true;
                        if (h & (h - 1)) {
                            // finish B's remaining runs through apply_run, which locates by lk
                            for (u64 h2 = h & (h - 1); h2; h2 &= h2 - 1) {
                                const uint32_t hl2 = first_lane(h2);
                                const uint32_t tl2 = tail_of(hl2);
                                const uint32_t ia = U(bcast(item, hl2)), ib = U(bcast(item, tl2));
                                const uint32_t lo2 = min(ia, ib), hi2 = max(ia, ib), k3 = U(bcast(kd, hl2));
                                // a run may now straddle both halves: apply it piecewise by block
                                for (uint32_t x0 = lo2; x0 <= hi2 && !D.err;) {
                                    const uint32_t bx = U(D.lk[x0]);
                                    uint32_t x1 = x0;   // extend while the items stay in bx
                                    while (x1 < hi2 && U(D.lk[x1 + 1]) == bx) x1++;
                                    bool r2 = false;
                                    apply_run<MB, PROF>(D, bx, x0, x1, k3, ckey, r2);
                                    x0 = x1 + 1;
                                }
                                if (D.err) return;
                            }
                        }
                        break;
                    }
                }
            } else if (__ballot(nov != 0)) {   // every touched span covered whole by one run
                const uint32_t nst = st + dd;
                const bool ov = nov != 0;
                if (__ballot(ov && (st == 0 ? dd != 1u : nst > ST_MAX))) { fail(D, ErrCheckout, 16); return; }
                const uint32_t dv1 = ov ? uint32_t((int32_t(nst == 1) - int32_t(st == 1)) * int32_t(len)) : 0u;
                const uint32_t dl1 = ov ? uint32_t(int32_t(nst != 0) - int32_t(st != 0)) : 0u;
                const uint32_t dv = wave_sum(dv1), dl = wave_sum(dl1);
                const u64 om = __ballot(ov);
                if (ov) rw = (rw & ~(0x7FFu << ST_SHIFT)) | (nst << ST_SHIFT) | (kk == 3u ? ED_BIT : 0u);
                if (ov) D.rows[size_t(B) * NS + l] = u64(rl) | (u64(rw) << 32);
                const uint32_t o = U(opos_of<MB>(D, B));
                const uint32_t tp = U(SBPOS<MB>(D)[o >> 6]);
                if (l == 0) {
                    ix_add<MB>(&CNT<MB>(D)[B], dv);
                    ix_add<MB>(&META<MB>(D)[B], dl << 8);
                    ix_add<MB>(&TV<MB>(D)[tp], dv);
                    ix_add<MB>(&TL<MB>(D)[tp], dl);
                }
                wave_fence();
                if (B == D.cb) {
                    D.crw = rw; D.ccnt += dv;
                } else if (D.cb != NONE && dv != 0 && ((tp << 6) | (o & 63u)) < ckey) {
                    D.cbase += dv;
                }
                (void)om;
            }
            pend &= ~inB;
            if (relinked) {   // a block split moved LVs: the pending lanes' blocks are stale
                nB = NONE;
                blk = isdel ? D.lk[item] : D.lk[xs];
                heads = (heads_of(blk) | (pend & ~(pend << 1))) & pend;
                bound = heads | ~pend;
                if (D.cb == NONE) ckey = 0;
            }
        }
        if (PROF) { const uint64_t t2 = tick<PROF>(); g_cold.prof[P_T2] += t2 - tq; tq = t2; }
    }
}

// Copy the visible spans' text (one contiguous range of the insert content each) in document
// order into out[] (list/merge.rs:63-95), with the order-dependent hash the host checks.
template <uint32_t MB> DEV void materialise(Doc &D, uint8_t *out, uint32_t cap, uint32_t &len_out, u64 &hash_out) {
    const uint32_t l = lane_id();
    uint32_t total = 0, items = 0;
    u64 h = 0;
    for (uint32_t p = 0; p < D.nsb; p++) {
        const uint32_t S = U(TS<MB>(D)[p]), nbk = U(TN<MB>(D)[p]);
        for (uint32_t i = 0; i < nbk; i++) {
            const uint32_t b = U(sbl_at<MB>(D, size_t(S) * SBC + i));
            const uint32_t n = U(m_n(META<MB>(D)[b]));
            if (n == 0) continue;   // the empty first block of an empty document
            uint32_t rl, rw;
            load_row(D, b, n, rl, rw);
            items += wave_sum(s_len(rw));
            const uint32_t len = s_vis(rw);
            const uint32_t c0 = g_cold.cbyte[len ? rl : 0u];
            uint32_t nb = len;
            if (!g_cold.ascii && len) {
                const uint32_t cl = g_cold.cbyte[rl + len - 1];
                nb = cl - c0 + utf8_len(g_cold.content[cl]);
            }
            const uint32_t inc = wave_scan(nb);
            const uint32_t tb = U(bcast(inc, 63));
            for (uint32_t c = 0; c < tb; c += 64) {
                const uint32_t u = c + l;
                const uint32_t s = min(lane_search(inc, u), 63u);
                const uint32_t src = shfl(c0, s) + (u - (shfl(inc, s) - shfl(nb, s)));
                if (u < tb) {
                    const uint8_t by = g_cold.content[src];
                    const uint32_t at = total + u;
                    if (at < cap) out[at] = by;
                    h += splitmix((u64(at) << 8) | by);
                }
            }
            total += tb;
        }
    }
    len_out = total;
    hash_out = wave_sum64(h);
    g_cold.n_items = items;
}

// Debug-mode consistency check of the whole structure (DTGPU_DEBUG=1): 0 or a code.  Every block
// reached through the index: span count / live count / visible count against its row, spans
// non-empty with legal states, every item's lk[] naming the block, (superblock, index) positions,
// superblock totals, and the cached block's state.
template <uint32_t MB> DEV uint32_t check_invariants(Doc &D, DocResult *res) {
    const uint32_t l = lane_id();
    uint32_t blocks = 0, base = 0;
    for (uint32_t p = 0; p < D.nsb; p++) {
        const uint32_t S = U(TS<MB>(D)[p]);
        if (U(SBPOS<MB>(D)[S]) != p) return 205;
        const uint32_t nbk = U(TN<MB>(D)[p]);
        if (nbk != U(SBN<MB>(D)[S]) || nbk == 0 || nbk >= SBC) return 206;
        uint32_t tv = 0, tl = 0;
        for (uint32_t i = 0; i < nbk; i++) {
            const uint32_t b = U(sbl_at<MB>(D, size_t(S) * SBC + i));
            if (b >= D.nb) return 209;
            if (U(opos_of<MB>(D, b)) != ((S << 6) | i)) return 201;
            const uint32_t mt = U(META<MB>(D)[b]), n = m_n(mt);
            if (n > NS || (n == 0 && D.nb > 1)) return 210;
            uint32_t rl, rw;
            load_row(D, b, n, rl, rw);
            const uint32_t len = s_len(rw), st = s_st(rw);
            if (__ballot(l < n && (len == 0 || st > ST_MAX))) return 211;
            if (wave_sum(s_vis(rw)) != U(CNT<MB>(D)[b])) return 207;
            if (wave_sum(l < n && st != 0 ? 1u : 0u) != m_live(mt)) return 212;
            // every item of every span links back to b
            const uint32_t inc = wave_scan(len);
            const uint32_t total = U(bcast(inc, 63));
            bool bad = false;
            uint32_t bad_item = 0;
            for (uint32_t c = 0; c < total; c += 64) {
                const uint32_t u = c + l;
                const uint32_t s = min(lane_search(inc, u), 63u);
                const uint32_t item = shfl(rl, s) + (u - (shfl(inc, s) - shfl(len, s)));
                if (u < total && (item >= D.n_lv || D.lk[item] != b)) { bad = true; bad_item = item; }
            }
            const u64 bm = __ballot(bad);
            if (bm) {
                if (l == first_lane(bm)) { res->dbg[0] = b; res->dbg[1] = bad_item; res->dbg[2] = D.lk[bad_item]; }
                return 202;
            }
            if (b == D.cb) {
                if (D.cn != n || D.ccnt != U(CNT<MB>(D)[b]) || D.ctp != p || D.cbase != base) return 213;
                if (__ballot(l < n && (D.crl != rl || D.crw != rw))) return 214;
            }
            tv += U(CNT<MB>(D)[b]);
            tl += m_live(mt);
            base += U(CNT<MB>(D)[b]);
            blocks++;
        }
        if (tv != U(TV<MB>(D)[p])) return 203;
        if (tl != U(TL<MB>(D)[p])) return 204;
    }
    if (blocks != D.nb) return 208;
    return 0;
}

template <uint32_t MB, bool PROF>
DEV void run_doc(Doc &D, uint8_t *out, uint32_t cap, DocResult *res) {
    const uint32_t l = lane_id();
    // fresh tracker: one empty block in one superblock
    if (l == 0) {
        CNT<MB>(D)[0] = 0; META<MB>(D)[0] = 0; set_opos<MB>(D, 0, 0);
        set_sbl<MB>(D, 0, 0); SBN<MB>(D)[0] = 1; SBPOS<MB>(D)[0] = 0;
        TV<MB>(D)[0] = 0; TL<MB>(D)[0] = 0; TS<MB>(D)[0] = 0; TN<MB>(D)[0] = 1;
    }
    wave_fence();
    D.nb = 1;
    D.nsb = 1;
    D.err = 0;
    g_cold.n_items = 0;
    D.steps = 0;
    D.step_limit = uint32_t(min<uint64_t>(64ull * (uint64_t(D.ncmd) + D.n_lv) + 4096, 0xFFFFFFF0ull));
    g_cold.site = 0;
    D.ci = 0;
    D.cb = NONE;
    D.cn = D.ccnt = D.ctp = D.cbase = 0;
    D.crl = D.crw = 0;
    if (PROF) for (int i = 0; i < P_N; i++) g_cold.prof[i] = 0;
    const uint64_t t_start = tick<PROF>();
    // commands are fetched 64 at a time (one per lane) and broadcast; the first tlist chunk of a
    // TOG is fetched while the command before it runs (tlist is read-only)
    uint32_t pf = 0;
    bool pf_ok = false;
    for (uint32_t base = 0; base < D.ncmd && !D.err && !D.dump_n; base += 64) {
        const uint32_t n_here = min(64u, D.ncmd - base);
        const Cmd pre = D.cmds[min(base + l, D.ncmd - 1)];
        for (uint32_t j = 0; j < n_here && !D.err; j++) {
            D.ci = base + j;
            const uint32_t op = U(bcast(pre.op, j)), a = U(bcast(pre.lv, j)), n = U(bcast(pre.len, j)),
                           pos = U(bcast(pre.pos, j));
            if (!charge(D)) break;
            uint32_t nx_pf = 0;
            bool nx_ok = false;
            if (j + 1 < n_here && (U(bcast(pre.op, j + 1)) & 15u) == CMD_TOG) {
                const uint32_t o2 = U(bcast(pre.lv, j + 1)), n2 = U(bcast(pre.len, j + 1));
                if (n2) nx_pf = D.tlist[o2 + min(l, n2 - 1)];
                nx_ok = true;
            }
            const uint64_t t0 = tick<PROF>();
            switch (op & 15u) {
                case CMD_INS:
                    if (n == 0 || a >= D.n_lv || n > D.n_lv - a) { fail(D, ErrCheckout, 17); break; }
                    do_insert<MB, PROF>(D, a, n, pos);
                    if (PROF) g_cold.prof[P_INS] += tick<PROF>() - t0;
                    break;
                case CMD_DEL:
                    if (n == 0 || a >= D.n_lv || n > D.n_lv - a) { fail(D, ErrCheckout, 17); break; }
                    do_delete<MB, PROF>(D, a, n, pos, (op & 16u) != 0);
                    if (PROF) g_cold.prof[P_DEL] += tick<PROF>() - t0;
                    break;
                case CMD_TOG:
                    toggle_pass<MB, PROF>(D, a, n, pf, pf_ok);
                    if (PROF) g_cold.prof[P_TOG] += tick<PROF>() - t0;
                    break;
                default: fail(D, ErrCheckout, 18); break;
            }
            if (D.debug && !D.err) {
                const uint32_t code = check_invariants<MB>(D, res);
                if (code) fail(D, ErrCheckout, code);
            }
            if (D.dump_at && D.ci + 1 == D.dump_at && !D.err) {   // DTGPU_DEBUG bit 4: the span list
                uint32_t k = 0;                                   // in document order after one command
                for (uint32_t p = 0; p < D.nsb; p++) {
                    const uint32_t S = U(TS<MB>(D)[p]), nbk = U(TN<MB>(D)[p]);
                    for (uint32_t i = 0; i < nbk; i++) {
                        const uint32_t b = U(sbl_at<MB>(D, size_t(S) * SBC + i));
                        const uint32_t nn = U(m_n(META<MB>(D)[b]));
                        uint32_t rl, rw;
                        load_row(D, b, nn, rl, rw);
                        if (l < nn && 8ull * (k + l + 1) <= cap) {
                            reinterpret_cast<uint32_t *>(out)[2 * (k + l)] = rl;
                            reinterpret_cast<uint32_t *>(out)[2 * (k + l) + 1] = rw;
                        }
                        k += nn;
                    }
                }
                D.dump_n = k;
                break;
            }
            if (D.trace && !D.err) {   // DTGPU_DEBUG bit 3: visible total after every command into out[]
                uint32_t tot = 0;
                for (uint32_t q = 0; q < D.nsb; q += 64) tot += wave_sum(q + l < D.nsb ? TV<MB>(D)[q + l] : 0u);
                if (l == 0 && 4ull * (D.ci + 1) <= cap) reinterpret_cast<uint32_t *>(out)[D.ci] = tot;
            }
            pf = nx_pf;
            pf_ok = nx_ok;
        }
    }
    // an LDS-tier document that outgrew its optimistic capacity is queued for the HBM tier,
    // which replays it again from scratch
    if (MB && D.err == ErrCapacity && (g_cold.site == 12 || g_cold.site == 21) && g_cold.fb_list) {
        if (l == 0) g_cold.fb_list[atomicAdd(g_cold.fb_count, 1u)] = g_cold.doc;
        return;
    }
    uint32_t len = 0;
    u64 h = 0;
    const uint64_t t_mat = tick<PROF>();
    if (D.dump_at) len = min(8u * D.dump_n, cap & ~7u);
    else if (D.trace) len = min(4u * D.ncmd, cap & ~3u);
    else if (!D.err) materialise<MB>(D, out, cap, len, h);
    if (l == 0) {
        res->status = (D.trace || D.dump_at) ? 0u : D.err;   // a trace is read even when the replay failed
        res->out_len = len;
        res->hash = h;
        res->n_items = g_cold.n_items;
        res->n_blocks = D.nb;
        res->n_sb = D.nsb;
        res->lds = MB ? 1u : 0u;
        res->fail_cmd = D.err ? D.ci : 0;
        res->fail_site = D.err ? g_cold.site : 0;
        if (PROF) {
            g_cold.prof[P_MAT] = tick<PROF>() - t_mat;
            for (int i = 0; i < P_T1; i++) res->dbg[i] = uint32_t(g_cold.prof[i] >> (i < P_HIT ? 4 : 0));
            res->dbg[15] = uint32_t((tick<PROF>() - t_start) >> 4);
            for (int i = P_T1; i < P_N; i++) res->dbg[16 + (i - P_T1)] = uint32_t(g_cold.prof[i] >> 4);
        }
    }
}

// One 64-lane workgroup per document of the list (the hardware dispatcher is the work queue; LDS
// per workgroup bounds how many documents share a CU).  MB: the LDS tier's block capacity, or 0
// for the HBM-index tier.
template <uint32_t MB, bool PROF>
__global__ __launch_bounds__(64) void span_kernel(BatchParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t di = U(blockIdx.x);
    uint32_t d;
    if (di < P.n_list) {
        d = U(P.doc_list[di]);
    } else {   // HBM tier: documents the LDS tier handed back
        if (MB || !P.fb_count) return;
        const uint32_t j = di - P.n_list;
        if (j >= U(__hip_atomic_load(P.fb_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) return;
        d = U(P.fb_list[j]);
    }
    const DocDesc dd = P.docs[d];
    Doc D;
    if (lane_id() == 0) {
        g_cold.doc = d;
        g_cold.fb_list = MB ? P.fb_list : nullptr;
        g_cold.fb_count = P.fb_count;
        g_cold.cbyte = P.cbyte + dd.lv_off;
        g_cold.content = P.content + dd.content_off;
        g_cold.aruns = P.aruns + dd.arun_off;
        g_cold.n_aruns = dd.n_aruns;
        g_cold.ascii = dd.ascii;
        g_cold.max_blocks = MB ? min(dd.max_blocks, MB) : dd.max_blocks;
        g_cold.max_sb = MB ? span_lds_sb(MB) : span_sb_capacity(dd.max_blocks);
    }
    D.debug = P.debug & 1u;
    D.slow = (P.debug >> 2) & 1u;   // DTGPU_DEBUG bit 2: toggles run by run (no one-pass path)
    D.trace = (P.debug >> 3) & 1u;
    D.dump_at = (P.debug >> 4) & 1u ? (P.debug >> 8) : 0u;   // DTGPU_DEBUG = 16 + 256 * (command + 1)
    D.dump_n = 0;
    D.cmds = P.cmds + dd.cmd_off;
    D.ncmd = U(dd.ncmd);
    D.n_lv = U(dd.n_lv);
    D.tlist = P.tlist + dd.tlist_off;
    D.lk = P.pos + dd.lv_off;
    D.ao = P.ao + dd.lv_off;
    D.rows = P.rows + dd.blk_off * NS;
    if (MB) {
        D.ix = reinterpret_cast<uint32_t *>(smem);
        D.mb = MB;
        D.ms = span_lds_sb(MB);
    } else {
        D.ix = reinterpret_cast<uint32_t *>(P.gidx + dd.gidx_off);
        D.mb = U(dd.max_blocks);
        D.ms = span_sb_capacity(D.mb);
    }
    wave_fence();
    run_doc<MB, PROF>(D, P.out + dd.out_off, U(dd.out_cap), &P.results[d]);
}

}  // namespace sdev

template <uint32_t MB>
static int launch_tier(const BatchParams &q, hipStream_t s, bool prof) {
    constexpr size_t lds = size_t(span_index_bytes(MB, span_lds_sb(MB), true));
    static_assert(lds <= 160 * 1024 - 512, "tier index above the CU's LDS");
    // dynamic LDS above 64 KiB needs the per-function attribute (set on every launch: it holds
    // for whatever device the batch runs on)
    const void *fn = prof ? reinterpret_cast<const void *>(&sdev::span_kernel<MB, true>)
                          : reinterpret_cast<const void *>(&sdev::span_kernel<MB, false>);
    if (lds > 64 * 1024 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)) != hipSuccess)
        return ErrHip;
    if (prof) hipLaunchKernelGGL((sdev::span_kernel<MB, true>), dim3(q.n_list), dim3(64), lds, s, q);
    else hipLaunchKernelGGL((sdev::span_kernel<MB, false>), dim3(q.n_list), dim3(64), lds, s, q);
    return hipGetLastError() == hipSuccess ? OK : ErrHip;
}
static int launch_span_lds_tier(int t, const BatchParams &q, hipStream_t s, bool prof) {
    if (!q.n_list) return OK;
    if (q.lds_blocks != kSpanTierBlocks[t]) return ErrArg;
    switch (t) {
        case 0: return launch_tier<kSpanTierBlocks[0]>(q, s, prof);
        case 1: return launch_tier<kSpanTierBlocks[1]>(q, s, prof);
        case 2: return launch_tier<kSpanTierBlocks[2]>(q, s, prof);
        case 3: return launch_tier<kSpanTierBlocks[3]>(q, s, prof);
        default: return ErrArg;
    }
}

int launch_span_replay(const ReplayLaunch &r) {
    hipStream_t s = reinterpret_cast<hipStream_t>(r.stream);
    const BatchParams &large = *r.large;
    bool prof = large.debug & 2u;
    uint32_t n_lds = 0;
    const uint32_t *fb_count = nullptr;
    for (int t = 0; t < r.n_lds; t++) {
        prof |= (r.lds[t].debug & 2u) != 0;
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
            const int e = launch_span_lds_tier(t, r.lds[t], (fork && k < n_side) ? reinterpret_cast<hipStream_t>(r.side[k]) : s, prof);
            if (e) return e;
        }
        if (fork) {
            for (int k = 0; k < n_side; k++)
                if (hipEventRecord(reinterpret_cast<hipEvent_t>(r.ev_join[k]), reinterpret_cast<hipStream_t>(r.side[k])) != hipSuccess ||
                    hipStreamWaitEvent(s, reinterpret_cast<hipEvent_t>(r.ev_join[k]), 0) != hipSuccess)
                    return ErrHip;
        }
    }
    // HBM tier: its own list plus a slot per LDS-tier document that may be handed back
    const uint32_t grid = large.n_list + (large.fb_list ? large.fb_slots : 0);
    if (grid) {
        if (prof) hipLaunchKernelGGL((sdev::span_kernel<0, true>), dim3(grid), dim3(64), 0, s, large);
        else hipLaunchKernelGGL((sdev::span_kernel<0, false>), dim3(grid), dim3(64), 0, s, large);
        if (hipGetLastError() != hipSuccess) return ErrHip;
    }
    return OK;
}

}  // namespace dtgpu
