// dt_replay.hip -- per-document eg-walker replay + text materialisation on MI355X (gfx950).
//
// One wavefront (64 lanes) replays one document's command stream (built on the host from the
// spanning-tree walk, dt_host.cpp::build_plan).  This is the checkout-from-ROOT per-item
// formulation of the reference's M2Tracker (src/listmerge/merge.rs:89-581,
// advance_retreat.rs:58-153, yjsspan.rs:13-228):
//
//   items      one per inserted char, kept in document order in 64-slot blocks (HBM);
//   block idx  per block: visible mask, live (non-NIY) mask, item count, order position;
//              per 64 blocks (superblock): visible / item totals.  In LDS for documents
//              whose block count fits the LDS budget, in HBM otherwise (same code).
//   per-LV     state (0 NIY, 1 inserted, k>=2 deleted k-1 times; bit7 = ever_deleted),
//              block id, slot, origin_left or delete target, origin_right (HBM).
//
// Positional lookups are wave-parallel: a 64-lane prefix scan over superblock totals, a
// second over the 64 blocks of the chosen superblock, then a ballot select of the k-th set
// bit inside the block's visible mask.  Retreat/advance commands are lane-parallel over the
// LVs of one run (distinct items by construction), with LDS atomics on the masks.
// Materialisation walks blocks in order and stream-compacts never-deleted chars (prefix
// scan), writing UTF-8 bytes and an order-sensitive hash.
//
// Memory ordering: every cross-lane hand-off stays inside one wavefront; a wavefront-scope
// fence (compiler barrier) separates the phases (AMDGPU memory model: no cache maintenance is
// needed between lanes of one wavefront).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dt_device.hpp"

namespace dtgpu {
namespace dev {

typedef unsigned long long u64;

#define DEV __device__ __forceinline__

DEV uint32_t lane_id() { return __lane_id(); }
DEV void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); }
DEV uint32_t bcast(uint32_t v, uint32_t l) { return uint32_t(__builtin_amdgcn_readlane(int(v), int(l))); }
DEV uint32_t first_lane(u64 m) { return uint32_t(__ffsll((long long)m) - 1); }
// Wave-uniform values are pinned to scalar registers: control flow that depends on them is
// scalar (no exec-mask loops), which is both what the algorithm means and what keeps hipcc
// from treating the sequential replay as divergent.
DEV uint32_t U(uint32_t v) { return uint32_t(__builtin_amdgcn_readfirstlane(int(v))); }
DEV u64 U64(u64 v) {   // (readfirstlane returns int: keep both halves unsigned)
    return (u64(U(uint32_t(v >> 32))) << 32) | u64(U(uint32_t(v)));
}

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
constexpr uint32_t SB = 64;    // blocks per superblock
constexpr uint32_t ROOT_ID = 0xFFFFFFFFu;
constexpr uint32_t END_ID = 0xFFFFFFFEu;
constexpr uint8_t DEL_BIT = 0x80;

struct Doc {
    // inputs
    const Cmd *cmds;
    uint32_t ncmd, n_lv;
    const uint32_t *cbyte;
    const uint8_t *content;
    const uint32_t *aruns;
    uint32_t n_aruns;
    // per-LV state
    uint8_t *st;
    uint32_t *blk;
    uint8_t *slot;
    uint32_t *aux;
    uint32_t *orr;
    // blocks
    uint32_t *items;
    uint32_t max_blocks;
    // block index
    u64 *mvis, *mlive;
    uint32_t *ord, *opos, *svis, *scnt;
    uint8_t *bcnt;
    // wave-uniform scalars
    uint32_t nb;
    uint32_t err;
    uint32_t n_items;
    uint32_t debug;
    uint32_t site, ci;
    uint64_t steps, step_limit;   // watchdog: every loop iteration is charged; a bound
                                  // violation ends the document with ErrCapacity
};

// Charge one loop iteration; returns false (and flags the document) past the budget, so every
// loop in the replay provably terminates whatever the input.
DEV void fail(Doc &D, uint32_t code, uint32_t site) {
    if (!D.err) { D.err = code; D.site = site; }
}
DEV bool charge(Doc &D) {
    if (++D.steps > D.step_limit) { fail(D, ErrCapacity, 1); return false; }
    return true;
}

struct Cursor { uint32_t b, s; };

// ---- order-statistic queries -------------------------------------------------------------

// Item holding visible index p (content-tree cursor_at_content_pos, root.rs:50-89).
DEV bool find_vis(Doc &D, uint32_t p, Cursor &out) {
    const uint32_t l = lane_id();
    const uint32_t nsb = (D.nb + SB - 1) / SB;
    uint32_t base = 0, sb = 0;
    bool found = false;
    for (uint32_t c = 0; c < nsb; c += 64) {
        const uint32_t i = c + l;
        const uint32_t v = i < nsb ? D.svis[i] : 0;
        const uint32_t inc = wave_scan(v);
        const u64 m = __ballot(base + inc > p);
        if (m) {
            const uint32_t fl = first_lane(m);
            sb = c + fl;
            base += bcast(inc - v, fl);
            found = true;
            break;
        }
        base += bcast(inc, 63);
    }
    if (!found) return false;
    const uint32_t i = sb * SB + l;
    const uint32_t b = i < D.nb ? D.ord[i] : 0;
    const uint32_t v = i < D.nb ? uint32_t(__popcll(D.mvis[b])) : 0;
    const uint32_t inc = wave_scan(v);
    const u64 m = __ballot(base + inc > p);
    if (!m) return false;
    const uint32_t fl = first_lane(m);
    const uint32_t bb = bcast(b, fl);
    const uint32_t off = p - base - bcast(inc - v, fl);
    const u64 mv = U64(D.mvis[bb]);
    const bool set = (mv >> l) & 1ull;
    const uint32_t before = uint32_t(__popcll(mv & ((1ull << l) - 1ull)));
    const u64 m2 = __ballot(set && before == off);
    if (!m2) return false;
    out.b = bb;
    out.s = first_lane(m2);
    return true;
}

// Document index of an item (number of items before it in list order).
DEV uint64_t rank_of(Doc &D, uint32_t item) {
    const uint32_t l = lane_id();
    uint32_t b = U(D.blk[item]), s = U(D.slot[item]);
    if (b >= D.nb) { fail(D, ErrCheckout, 11); b = 0; s = 0; }
    const uint32_t p = U(D.opos[b]), sb = p / SB;
    uint32_t acc = 0;
    for (uint32_t c = 0; c < sb; c += 64) {
        const uint32_t i = c + l;
        acc += i < sb ? D.scnt[i] : 0;
    }
    {
        const uint32_t i = sb * SB + l;
        acc += i < p ? uint32_t(D.bcnt[D.ord[i]]) : 0;
    }
    return uint64_t(wave_sum(acc)) + s;
}

// Move a cursor at the end of a block to the start of the next block in order.
DEV void normalize(Doc &D, Cursor &c) {
    while (c.s >= U(D.bcnt[c.b])) {
        if (!charge(D)) return;
        const uint32_t p = U(D.opos[c.b]) + 1;
        if (p >= D.nb) return;   // end of document
        c.b = U(D.ord[p]);
        c.s = 0;
    }
}

// First item at/after c that is not NIY (origin_right search, merge.rs:405-423).
DEV bool next_live(Doc &D, Cursor c, Cursor &out) {
    const uint32_t l = lane_id();
    const u64 ml = c.s >= 64 ? 0ull : (U64(D.mlive[c.b]) & (~0ull << c.s));
    if (ml) { out.b = c.b; out.s = first_lane(ml); return true; }
    for (uint32_t p0 = U(D.opos[c.b]) + 1; p0 < D.nb; p0 += 64) {
        const uint32_t i = p0 + l;
        const uint32_t b = i < D.nb ? D.ord[i] : 0;
        const u64 m = __ballot(i < D.nb && D.mlive[b] != 0ull);
        if (m) {
            const uint32_t fl = first_lane(m);
            out.b = bcast(b, fl);
            out.s = first_lane(U64(D.mlive[out.b]));
            return true;
        }
    }
    return false;
}

// ---- block maintenance ---------------------------------------------------------------------

DEV void recompute_sb(Doc &D, uint32_t from_sb) {
    const uint32_t l = lane_id();
    const uint32_t nsb = (D.nb + SB - 1) / SB;
    for (uint32_t s = from_sb; s < nsb; s++) {
        const uint32_t i = s * SB + l;
        const uint32_t b = i < D.nb ? D.ord[i] : 0;
        const uint32_t v = i < D.nb ? uint32_t(__popcll(D.mvis[b])) : 0;
        const uint32_t c = i < D.nb ? uint32_t(D.bcnt[b]) : 0;
        const uint32_t tv = wave_sum(v), tc = wave_sum(c);
        if (l == 0) { D.svis[s] = tv; D.scnt[s] = tc; }
    }
    wave_fence();
}

// Split a full block: its upper half moves to a new block placed right after it in order.
DEV uint32_t split_block(Doc &D, uint32_t b) {
    const uint32_t l = lane_id();
    if (D.nb >= D.max_blocks) { fail(D, ErrCapacity, 12); return 0; }
    const uint32_t b2 = D.nb;
    uint32_t *src = D.items + size_t(b) * BLK;
    uint32_t *dst = D.items + size_t(b2) * BLK;
    if (l >= BLK / 2) {
        const uint32_t v = src[l];
        dst[l - BLK / 2] = v;
        D.blk[v] = b2;
        D.slot[v] = uint8_t(l - BLK / 2);
    }
    const uint32_t p = U(D.opos[b]) + 1;
    // shift ord[p .. nb) right by one, highest chunk first
    for (int c = int(D.nb) - 1; c >= int(p); c -= 64) {
        const int i = c - int(l);
        uint32_t v = 0;
        if (i >= int(p)) v = D.ord[i];
        wave_fence();
        if (i >= int(p)) { D.ord[i + 1] = v; D.opos[v] = uint32_t(i + 1); }
        wave_fence();
    }
    if (l == 0) {
        D.mvis[b2] = D.mvis[b] >> 32;
        D.mvis[b] &= 0xFFFFFFFFull;
        D.mlive[b2] = D.mlive[b] >> 32;
        D.mlive[b] &= 0xFFFFFFFFull;
        D.bcnt[b2] = BLK / 2;
        D.bcnt[b] = BLK / 2;
        D.ord[p] = b2;
        D.opos[b2] = p;
    }
    wave_fence();
    D.nb++;
    recompute_sb(D, (p - 1) / SB);
    return b2;
}

// Insert the run [lv, lv+k) at cursor c (all new items visible).
DEV void insert_run(Doc &D, Cursor c, uint32_t lv, uint32_t k, uint32_t ol, uint32_t orr) {
    const uint32_t l = lane_id();
    const uint32_t lv0 = lv, k0 = k;
    uint32_t b = c.b, s = c.s;
    while (k > 0) {
        if (!charge(D)) return;
        const uint32_t cnt = U(D.bcnt[b]);
        if (cnt == BLK) {
            const uint32_t b2 = split_block(D, b);
            if (D.err) return;
            if (s > BLK / 2) { b = b2; s -= BLK / 2; }
            continue;
        }
        const uint32_t m = min(k, BLK - cnt);
        uint32_t *items = D.items + size_t(b) * BLK;
        const uint32_t v = l < cnt ? items[l] : 0;
        wave_fence();
        if (l >= s && l < cnt) { items[l + m] = v; D.slot[v] = uint8_t(l + m); }
        if (l >= s && l < s + m) {
            const uint32_t it = lv + (l - s);
            items[l] = it;
            D.slot[it] = uint8_t(l);
            D.blk[it] = b;
        }
        if (l == 0) {
            const u64 low = s == 0 ? 0ull : (~0ull >> (64 - s));
            const u64 ins = (m == 64 ? ~0ull : ((1ull << m) - 1ull)) << s;
            const u64 mv = D.mvis[b], ml = D.mlive[b];
            const u64 hv = m == 64 ? 0ull : ((mv & ~low) << m);
            const u64 hl = m == 64 ? 0ull : ((ml & ~low) << m);
            D.mvis[b] = (mv & low) | hv | ins;
            D.mlive[b] = (ml & low) | hl | ins;
            D.bcnt[b] = uint8_t(cnt + m);
            const uint32_t sbi = D.opos[b] / SB;
            D.svis[sbi] += m;
            D.scnt[sbi] += m;
        }
        wave_fence();
        lv += m;
        k -= m;
        s += m;
    }
    // per-item metadata last: origin loads issued before the block work have landed by now
    for (uint32_t j = l; j < k0; j += 64) {
        const uint32_t it = lv0 + j;
        D.st[it] = 1;
        D.aux[it] = j == 0 ? ol : it - 1;
        D.orr[it] = orr;
    }
}

// YjsMod tie-break by agent name rank then seq (merge.rs:199-218).
DEV void agent_of(const Doc &D, uint32_t lv, uint32_t &rank, uint32_t &seq) {
    uint32_t lo = 0, hi = D.n_aruns;   // last run with start <= lv
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (U(D.aruns[3 * mid]) <= lv) lo = mid; else hi = mid;
    }
    rank = U(D.aruns[3 * lo + 1]);
    seq = U(D.aruns[3 * lo + 2]) + (lv - U(D.aruns[3 * lo]));
}

DEV uint64_t rank_left(Doc &D, uint32_t ol) { return ol == ROOT_ID ? 0 : rank_of(D, ol) + 1; }
DEV uint64_t rank_right(Doc &D, uint32_t orr) { return orr == END_ID ? ~0ull : rank_of(D, orr); }

// Apply an insert run at visible position pos (M2Tracker::apply Ins + integrate,
// merge.rs:154-278, 383-455).
DEV void do_insert(Doc &D, uint32_t lv, uint32_t k, uint32_t pos) {
    Cursor cur;
    uint32_t ol;
    if (pos == 0) {
        ol = ROOT_ID;
        cur.b = U(D.ord[0]);
        cur.s = 0;
    } else {
        Cursor c;
        if (!find_vis(D, pos - 1, c)) { fail(D, ErrCheckout, 13); return; }
        ol = D.items[size_t(c.b) * BLK + c.s];   // same value in every lane; consumed late
        cur.b = c.b;
        cur.s = c.s + 1;
    }
    normalize(D, cur);
    Cursor rc;
    const bool has_r = next_live(D, cur, rc);
    const uint32_t orr = has_r ? D.items[size_t(rc.b) * BLK + rc.s] : END_ID;
    const bool at_end = cur.s >= U(D.bcnt[cur.b]);
    const bool direct = has_r ? (rc.b == cur.b && rc.s == cur.s) : at_end;
    if (!direct) {
        // concurrent NIY items between cursor and origin_right: YjsMod scan
        ol = U(ol);
        const uint32_t orr_u = U(orr);
        const uint64_t my_l = rank_left(D, ol), my_r = rank_right(D, orr_u);
        uint32_t new_rank = 0, new_seq = 0;
        agent_of(D, lv, new_rank, new_seq);
        bool scanning = false;
        Cursor scan_start = cur, c = cur;
        for (;;) {
            if (!charge(D)) return;
            if (c.s >= U(D.bcnt[c.b])) break;   // reached the end of the document
            const uint32_t o = U(D.items[size_t(c.b) * BLK + c.s]);
            if (o == orr_u) break;
            const uint64_t ol_o = rank_left(D, U(D.aux[o]));
            if (ol_o < my_l) break;
            if (ol_o == my_l) {
                const uint32_t orr_o = U(D.orr[o]);
                if (orr_o == orr_u) {
                    uint32_t r2, s2;
                    agent_of(D, o, r2, s2);
                    const bool ins_here = new_rank < r2 || (new_rank == r2 && new_seq < s2);
                    if (ins_here) break;
                    scanning = false;
                } else {
                    if (rank_right(D, orr_o) < my_r) {
                        if (!scanning) { scanning = true; scan_start = c; }
                    } else scanning = false;
                }
            }
            c.s++;
            normalize(D, c);
        }
        cur = scanning ? scan_start : c;
    }
    insert_run(D, cur, lv, k, ol, orr);
    D.n_items += k;
}

// Apply a delete run: n visible items from position pos (merge.rs:457-556).  LV lv+j targets
// the j-th item (fwd) or the (n-1-j)-th item (reversed / backspace runs).
DEV void do_delete(Doc &D, uint32_t lv, uint32_t n, uint32_t pos, bool fwd) {
    const uint32_t l = lane_id();
    uint32_t j0 = 0;
    while (j0 < n) {
        if (!charge(D)) return;
        Cursor c;
        if (!find_vis(D, pos, c)) { fail(D, ErrCheckout, 14); return; }
        const u64 vm = U64(D.mvis[c.b]) & (~0ull << c.s);
        const uint32_t avail = uint32_t(__popcll(vm));
        const uint32_t take = min(avail, n - j0);
        const uint32_t r = uint32_t(__popcll(vm & ((1ull << l) - 1ull)));
        const bool sel = ((vm >> l) & 1ull) && r < take;
        const u64 selm = __ballot(sel);
        bool bad = false;
        if (sel) {
            const uint32_t item = D.items[size_t(c.b) * BLK + l];
            const uint32_t j = j0 + r;
            const uint32_t dlv = fwd ? lv + j : lv + n - 1 - j;
            const uint8_t old = D.st[item];
            if ((old & 0x7F) != 1) bad = true;
            D.st[item] = DEL_BIT | 2;
            D.aux[dlv] = item;
        }
        if (__ballot(bad)) { fail(D, ErrCheckout, 15); return; }
        if (l == 0) {
            D.mvis[c.b] &= ~selm;
            D.svis[D.opos[c.b] / SB] -= take;
        }
        wave_fence();
        j0 += take;
    }
}

// Retreat / advance one run of LVs (advance_retreat.rs:58-153).  Items in one run are
// distinct, so lanes proceed independently; mask and superblock updates are LDS atomics.
template <bool ADVANCE, bool IS_DEL>
DEV void toggle_run(Doc &D, uint32_t lv, uint32_t n) {
    const uint32_t l = lane_id();
    for (uint32_t j = 0; j < n; j += 64) {
        const uint32_t v = lv + j + l;
        bool bad = false;
        if (j + l < n) {
            const uint32_t item = IS_DEL ? D.aux[v] : v;
            if (item >= D.n_lv) {
                bad = true;
            } else {
                const uint8_t old = D.st[item];
                const uint32_t state = old & 0x7F;
                uint32_t b = D.blk[item], s = D.slot[item];
                if (b >= D.nb || s >= BLK || (!IS_DEL && !ADVANCE && state == 0)) { bad = true; b = 0; s = 0; }
                const u64 bit = 1ull << s;
                const uint32_t sbi = D.opos[b] / SB;
                if (bad) {
                } else if (!IS_DEL) {
                    if (ADVANCE) {
                        if (state != 0) bad = true;
                        D.st[item] = uint8_t(old | 1);
                        atomicOr(&D.mvis[b], bit);
                        atomicOr(&D.mlive[b], bit);
                        atomicAdd(&D.svis[sbi], 1u);
                    } else {
                        if (state != 1) bad = true;
                        D.st[item] = uint8_t(old & DEL_BIT);
                        atomicAnd(&D.mvis[b], ~bit);
                        atomicAnd(&D.mlive[b], ~bit);
                        atomicSub(&D.svis[sbi], 1u);
                    }
                } else {
                    if (ADVANCE) {
                        if (state == 0 || state >= 0x7F) bad = true;
                        D.st[item] = uint8_t(DEL_BIT | (state + 1));
                        if (state == 1) { atomicAnd(&D.mvis[b], ~bit); atomicSub(&D.svis[sbi], 1u); }
                    } else {
                        if (state < 2) bad = true;
                        D.st[item] = uint8_t((old & DEL_BIT) | (state - 1));
                        if (state == 2) { atomicOr(&D.mvis[b], bit); atomicAdd(&D.svis[sbi], 1u); }
                    }
                }
            }
        }
        if (__ballot(bad)) { fail(D, ErrCheckout, 16); return; }
        wave_fence();
    }
}

// Stream-compact never-deleted chars in document order into out[] (list/merge.rs:63-95).
DEV void materialise(Doc &D, uint8_t *out, uint32_t cap, uint32_t &len_out, u64 &hash_out) {
    const uint32_t l = lane_id();
    uint32_t total = 0;
    u64 h = 0;
    for (uint32_t i = 0; i < D.nb; i++) {
        const uint32_t b = U(D.ord[i]);
        const uint32_t cnt = U(D.bcnt[b]);
        uint32_t cb = 0, n = 0;
        if (l < cnt) {
            const uint32_t it = D.items[size_t(b) * BLK + l];
            if (!(D.st[it] & DEL_BIT)) {
                cb = D.cbyte[it];
                n = utf8_len(D.content[cb]);
            }
        }
        const uint32_t inc = wave_scan(n);
        const uint32_t at = total + inc - n;
        for (uint32_t k = 0; k < n; k++) {
            const uint8_t byte = D.content[cb + k];
            if (at + k < cap) out[at + k] = byte;
            h += splitmix((u64(at + k) << 8) | byte);
        }
        total += bcast(inc, 63);
    }
    len_out = total;
    hash_out = wave_sum64(h);
}

// Debug-mode consistency check of the whole structure (DTGPU_DEBUG): returns 0 or a code.
DEV uint32_t check_invariants(Doc &D, DocResult *res) {
    const uint32_t l = lane_id();
    uint32_t code = 0;
    for (uint32_t i = 0; i < D.nb; i++) {
        const uint32_t b = U(D.ord[i]);
        if (U(D.opos[b]) != i) return 201;
        const uint32_t cnt = U(D.bcnt[b]);
        const u64 mv = U64(D.mvis[b]), ml = U64(D.mlive[b]);
        bool bad = false;
        if (l < cnt) {
            const uint32_t it = D.items[size_t(b) * BLK + l];
            if (it >= D.n_lv) bad = true;
            else {
                const uint32_t st = D.st[it] & 0x7F;
                if (((mv >> l) & 1) != (st == 1 ? 1u : 0u)) bad = true;
                if (((ml >> l) & 1) != (st != 0 ? 1u : 0u)) bad = true;
                if (D.blk[it] != b || D.slot[it] != l) bad = true;
            }
        } else if (((mv | ml) >> l) & 1) bad = true;
        const u64 bm = __ballot(bad);
        if (bm) {
            const uint32_t fl = first_lane(bm);
            if (l == fl) {
                const uint32_t it = l < cnt ? D.items[size_t(b) * BLK + l] : 0xFFFFFFFFu;
                res->dbg[0] = b; res->dbg[1] = l; res->dbg[2] = cnt; res->dbg[3] = it;
                res->dbg[4] = it < D.n_lv ? D.st[it] : 999; res->dbg[5] = it < D.n_lv ? D.blk[it] : 999;
                res->dbg[6] = it < D.n_lv ? D.slot[it] : 999;
                res->dbg[7] = uint32_t(mv); res->dbg[8] = uint32_t(mv >> 32); res->dbg[9] = uint32_t(ml);
            }
            return 202;
        }
    }
    const uint32_t nsb = (D.nb + SB - 1) / SB;
    for (uint32_t s = 0; s < nsb; s++) {
        const uint32_t i = s * SB + l;
        const uint32_t b = i < D.nb ? D.ord[i] : 0;
        const uint32_t v = i < D.nb ? uint32_t(__popcll(D.mvis[b])) : 0;
        const uint32_t c = i < D.nb ? uint32_t(D.bcnt[b]) : 0;
        if (U(wave_sum(v)) != U(D.svis[s])) code = 203;
        if (U(wave_sum(c)) != U(D.scnt[s])) code = 204;
        if (code) return code;
    }
    return 0;
}

DEV void run_doc(Doc &D, uint8_t *out, uint32_t cap, DocResult *res) {
    const uint32_t l = lane_id();
    // fresh tracker: one empty block, every LV not-inserted-yet
    for (uint32_t i = l; i < D.n_lv; i += 64) D.st[i] = 0;
    if (l == 0) {
        D.ord[0] = 0; D.opos[0] = 0; D.bcnt[0] = 0; D.mvis[0] = 0; D.mlive[0] = 0;
        D.svis[0] = 0; D.scnt[0] = 0;
    }
    wave_fence();
    D.nb = 1;
    D.err = 0;
    D.n_items = 0;
    D.steps = 0;
    D.step_limit = 64ull * (uint64_t(D.ncmd) + D.n_lv) + 4096;
    D.site = 0;
    // commands are fetched 64 at a time (one per lane) and broadcast with readlane
    for (uint32_t base = 0; base < D.ncmd && !D.err; base += 64) {
        const uint32_t n_here = min(64u, D.ncmd - base);
        Cmd pre = {0, 0, 0, 0};
        if (l < n_here) pre = D.cmds[base + l];
        for (uint32_t j = 0; j < n_here && !D.err; j++) {
            const uint32_t ci = base + j;
            D.ci = ci;
            Cmd c;
            c.op = bcast(pre.op, j); c.lv = bcast(pre.lv, j); c.len = bcast(pre.len, j); c.pos = bcast(pre.pos, j);
            const uint32_t op = c.op & 15u;
            if (c.len == 0 || c.lv >= D.n_lv || c.len > D.n_lv - c.lv) { fail(D, ErrCheckout, 17); break; }
            if (!charge(D)) break;
            switch (op) {
                case CMD_INS: do_insert(D, c.lv, c.len, c.pos); break;
                case CMD_DEL: do_delete(D, c.lv, c.len, c.pos, (c.op & 16u) != 0); break;
                case CMD_ADV_INS: toggle_run<true, false>(D, c.lv, c.len); break;
                case CMD_ADV_DEL: toggle_run<true, true>(D, c.lv, c.len); break;
                case CMD_RET_INS: toggle_run<false, false>(D, c.lv, c.len); break;
                case CMD_RET_DEL: toggle_run<false, true>(D, c.lv, c.len); break;
                default: fail(D, ErrCheckout, 18); break;
            }
            if (D.debug && !D.err) {
                const uint32_t code = check_invariants(D, res);
                if (code) fail(D, ErrCheckout, code);
            }
        }
    }
    uint32_t len = 0;
    u64 h = 0;
    if (!D.err) materialise(D, out, cap, len, h);
    if (l == 0) {
        res->status = D.err;
        res->out_len = len;
        res->hash = h;
        res->n_items = D.n_items;
        res->n_blocks = D.nb;
        res->fail_cmd = D.err ? D.ci : 0;
        res->fail_site = D.err ? D.site : 0;
    }
}

// Carve a block index for capacity `mb` out of `base` (LDS or HBM).
DEV void bind_index(Doc &D, uint8_t *base, uint32_t mb) {
    const uint32_t nsb = (mb + 63) / 64;
    D.mvis = reinterpret_cast<u64 *>(base);
    D.mlive = D.mvis + mb;
    D.ord = reinterpret_cast<uint32_t *>(D.mlive + mb);
    D.opos = D.ord + mb;
    D.svis = D.opos + mb;
    D.scnt = D.svis + nsb;
    D.bcnt = reinterpret_cast<uint8_t *>(D.scnt + nsb);
}

// One 64-lane workgroup per document of the list (the hardware dispatcher is the work queue;
// LDS per workgroup bounds how many documents share a CU).
template <bool LDS_INDEX>
__global__ __launch_bounds__(64) void replay_kernel(BatchParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t di = U(blockIdx.x);
    if (di >= P.n_list) return;
    const uint32_t d = U(P.doc_list[di]);
    const DocDesc dd = P.docs[d];
    Doc D;
    D.debug = P.debug;
    D.cmds = P.cmds + dd.cmd_off;
    D.ncmd = U(dd.ncmd);
    D.n_lv = U(dd.n_lv);
    D.cbyte = P.cbyte + dd.lv_off;
    D.content = P.content + dd.content_off;
    D.aruns = P.aruns + dd.arun_off;
    D.n_aruns = U(dd.n_aruns);
    D.st = P.st + dd.lv_off;
    D.blk = P.blk + dd.lv_off;
    D.slot = P.slot + dd.lv_off;
    D.aux = P.aux + dd.lv_off;
    D.orr = P.orr + dd.lv_off;
    D.items = P.items + dd.blk_off * BLK;
    D.max_blocks = U(dd.max_blocks);
    if (LDS_INDEX) {
        bind_index(D, smem, P.lds_blocks);
        if (D.max_blocks > P.lds_blocks) D.max_blocks = P.lds_blocks;
    } else {
        bind_index(D, P.gidx + dd.gidx_off, D.max_blocks);
    }
    run_doc(D, P.out + dd.out_off, U(dd.out_cap), &P.results[d]);
}

}  // namespace dev

int launch_replay(const BatchParams &small, const BatchParams &large, void *stream, int n_cu) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (small.n_list) {
        const size_t lds = size_t(index_bytes(small.lds_blocks));
        hipLaunchKernelGGL(dev::replay_kernel<true>, dim3(small.n_list), dim3(64), lds, s, small);
        if (hipGetLastError() != hipSuccess) return ErrHip;
    }
    if (large.n_list) {
        hipLaunchKernelGGL(dev::replay_kernel<false>, dim3(large.n_list), dim3(64), 0, s, large);
        if (hipGetLastError() != hipSuccess) return ErrHip;
    }
    return OK;
}

}  // namespace dtgpu
