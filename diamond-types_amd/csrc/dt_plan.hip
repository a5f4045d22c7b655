// dt_plan.hip -- device walk planner: the decoded oplog of each document -> the replay command
// stream (INS / DEL / TOG commands + retreat/advance entries) consumed by dt_replay.hip.
//
// One wavefront plans one document, walking the causal graph in the reference's spanning-tree
// order (SpanningTreeWalker, src/listmerge/txn_trace.rs:114-333): a todo stack seeded with the
// root entries; merge entries (>= 2 parents) wait while a non-merge entry is ready
// (txn_trace.rs:249-266); an entry becomes ready when its last parent entry is consumed.
//
// Between two consumed entries the tracker moves from the previous entry's last LV to the next
// entry's parents: retreat (ancestors of the old frontier not in the new one) then advance
// (the converse) -- Graph::diff_rev (src/causalgraph/graph/tools.rs:176-292).  The planner gets
// those sets from version vectors over causal chains: the host partitions the graph entries
// into chains (each entry extends the chain whose tail is one of its parents, dt_host.cpp
// build_plan_input), so the ancestor set of a version is a prefix of every chain,
// { (chain, seq) : seq < vv[chain] }, and a diff is one seq range per chain, copied out of a
// dense per-chain seq -> LV table.  (Diamond-types' agents are not chains in general: a git
// import has one author committing on concurrent branches.)
//
// vv rows (one per entry: the version vector of the entry's parents) live in HBM scratch;
// lane l keeps chains l, l + 64, ... of the current vector (K chunks: K = 1 up to 64 chains,
// K = 8 up to 512).  The todo stack and the pending-parent counts live in LDS.  Per consumed
// entry the wave issues one record load (as soon as the entry is picked, overlapping the
// previous entry's emission), one batch of independent loads (its op runs and children) and,
// when the frontier moves sideways, one gather per 64 retreat/advance entries.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dt_device.hpp"

namespace dtgpu {
namespace pdev {

typedef unsigned long long u64;
#define DEV __device__ __forceinline__

DEV uint32_t lane_id() { return __lane_id(); }
DEV uint32_t U(uint32_t v) { return uint32_t(__builtin_amdgcn_readfirstlane(int(v))); }
DEV uint32_t bcast(uint32_t v, uint32_t l) { return uint32_t(__builtin_amdgcn_readlane(int(v), int(l))); }
DEV uint32_t first_lane(u64 m) { return uint32_t(__ffsll((long long)m) - 1); }
DEV void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); }
DEV uint32_t wave_scan(uint32_t x) {   // inclusive prefix sum (same DPP sequence as dt_replay.hip)
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x142, 0xA, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x143, 0xC, 0xF, false));
    return x;
}

struct P {
    // inputs (decoded oplog)
    const uint32_t *erec, *par, *pent, *pch, *pcnt, *child, *doff, *dense, *tip;
    const Cmd *opc;
    uint32_t ne, A, ntip, n_lv;
    // scratch: vv rows in HBM; todo stack and pending parent counts in LDS (u16)
    uint32_t *base;
    uint32_t *order;       // two-phase planner: the walk order (ne words)
    const uint32_t *prow;  // K = 1: each entry's parent version vector (row_stride words)
    uint32_t row_stride;
    uint16_t *todo;      // ready entries (PLAN_TODO_CAP slots)
    uint8_t *pending;    // per entry: unvisited parents | merge flag
    // outputs
    Cmd *cmds;
    uint32_t *tlist;
    const uint32_t *walk;  // walk_kernel's {status, steps} for this document, or null
    uint32_t ccap, tcap;
    uint32_t count_only;   // sizing pass: count commands and entries, write nothing
    // wave-uniform state
    uint32_t nc, nt, err;
    uint32_t steps, limit;
    uint32_t n_ret, n_adv;
    uint32_t prof;
};
// DTGPU_PLAN_PROF cycle counters: in LDS, so that the (usually off) profile holds no SGPRs
__shared__ uint64_t g_pc[7];   // six phases, then the last timestamp
DEV void tk(const P &p) {
    if (p.prof && lane_id() == 0) { for (int i = 0; i < 6; i++) g_pc[i] = 0; g_pc[6] = __builtin_amdgcn_s_memtime(); }
}
#define PT(slot) do { if (p.prof) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    if (lane_id() == 0) { g_pc[slot] += t_ - g_pc[6]; g_pc[6] = t_; } } } while (0)

DEV void fail(P &p, uint32_t code) {
    if (!p.err) p.err = code;
}
DEV bool charge(P &p) {
    if (++p.steps > p.limit) { fail(p, PLAN_ERR_INTERNAL); return false; }
    return true;
}

// Entry record (EREC_WORDS words) lane by lane; R(rw, k) reads word k.
enum {
    R_START = 0, R_END, R_POFF, R_NP, R_OP0, R_NOP, R_CHAIN, R_SEQ0, R_CH0, R_NCH, R_PAR0,
    R_PENT0, R_PCH0, R_PCNT0, R_PENT1, R_PCH1, R_PCNT1, R_LASTCH, R_FIRSTCH
};
DEV uint32_t load_rec(const P &p, uint32_t e) {
    const uint32_t l = lane_id();
    return l < EREC_WORDS ? p.erec[erec_word(p.ne, e, l)] : 0;
}
DEV uint32_t R(uint32_t rw, int k) { return U(bcast(rw, uint32_t(k))); }

template <int K> struct VV { uint32_t v[K]; };

template <int K> DEV void vv_zero(VV<K> &x) {
#pragma unroll
    for (int k = 0; k < K; k++) x.v[k] = 0;
}
template <int K> DEV void vv_max(VV<K> &x, const VV<K> &y) {
#pragma unroll
    for (int k = 0; k < K; k++) x.v[k] = max(x.v[k], y.v[k]);
}
template <int K> DEV bool vv_differ(const VV<K> &x, const VV<K> &y) {
    bool d = false;
#pragma unroll
    for (int k = 0; k < K; k++) d |= x.v[k] != y.v[k];
    return __ballot(d) != 0;
}
template <int K> DEV void load_row(const P &p, uint32_t e, VV<K> &row) {
    const uint32_t l = lane_id();
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t a = l + 64 * k;
        row.v[k] = a < p.A ? p.base[size_t(e) * p.A + a] : 0;
    }
}
template <int K> DEV void store_row(P &p, uint32_t e, const VV<K> &row) {
    const uint32_t l = lane_id();
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t a = l + 64 * k;
        if (a < p.A) p.base[size_t(e) * p.A + a] = row.v[k];
    }
}

// The frontier moves along entry e (chain c, first seq s0) up to LV `upto`: row[c] becomes
// s0 + the entry's LVs so far.  check: the chain must continue exactly where row[c] stands
// (the chain decomposition guarantees it; a mismatch means a corrupt plan input).
template <int K>
DEV void fold_entry(P &p, uint32_t start, uint32_t end, uint32_t upto, uint32_t c, uint32_t s0, VV<K> &row,
                    bool check) {
    const uint32_t l = lane_id();
    const uint32_t hi = min(end, upto + 1);
    if (c >= p.A || hi <= start) { fail(p, PLAN_ERR_INTERNAL); return; }
    bool bad = false;
#pragma unroll
    for (int k = 0; k < K; k++) {
        if (c == l + 64 * k) {
            if (check && row.v[k] != s0) bad = true;
            row.v[k] = check ? s0 + (hi - start) : max(row.v[k], s0 + (hi - start));
        }
    }
    if (__ballot(bad)) fail(p, PLAN_NOT_CHAIN);
}

// Version vector of the version {lv} (lv inside entry e): the entry's parent vector plus the
// entry's own LVs up to lv.
template <int K> DEV void vv_at(P &p, uint32_t lv, uint32_t e, VV<K> &row) {
    const uint32_t rw = load_rec(p, e);
    load_row(p, e, row);
    fold_entry<K>(p, R(rw, R_START), R(rw, R_END), lv, R(rw, R_CHAIN), R(rw, R_SEQ0), row, false);
}

// Emit the retreat (from has more) / advance (to has more) entries of a diff: per agent one
// seq range of its dense seq -> (LV | is_del) table.  The ranges of one 64-agent chunk are
// gathered together, 64 entries per load.
template <int K>
DEV void emit_diff(P &p, const VV<K> &from, const VV<K> &to, const VV<K> &dlo, const VV<K> &dhi, bool allow_retreat) {
    const uint32_t l = lane_id();
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t a = l + 64 * k;
        const bool act = a < p.A && from.v[k] != to.v[k];
        const u64 am = __ballot(act);
        if (!am) continue;
        if (__ballot(act && to.v[k] < from.v[k] && !allow_retreat)) { fail(p, PLAN_ERR_INTERNAL); return; }
        const bool adv = to.v[k] > from.v[k];
        const uint32_t s0 = adv ? from.v[k] : to.v[k];
        const uint32_t n = act ? (adv ? to.v[k] - from.v[k] : from.v[k] - to.v[k]) : 0;
        const uint32_t d0 = dlo.v[k], d1 = dhi.v[k];
        if (__ballot(act && d0 + s0 + n > d1)) { fail(p, PLAN_ERR_INTERNAL); return; }
        const uint32_t inc = wave_scan(n);
        const uint32_t total = bcast(inc, 63);
        const uint32_t n_adv = bcast(wave_scan(adv ? n : 0), 63);
        if (uint64_t(p.nt) + total > p.tcap) { fail(p, PLAN_TLIST_FULL); return; }
        if (!p.count_only) {
            const uint32_t src = d0 + s0, off = inc - n;   // per agent lane
            bool bad = false;
            for (uint32_t c = 0; c < total; c += 64) {
                const uint32_t u = c + l;
                uint32_t from_idx = 0, flag = 0;
                for (u64 m = am; m; m &= m - 1) {   // the agent whose output slice holds u
                    const uint32_t j = first_lane(m);
                    const uint32_t o = U(bcast(off, j)), nn = U(bcast(n, j));
                    const uint32_t sj = U(bcast(src, j)), fj = U(bcast(adv ? TL_ADV : 0u, j));
                    if (u >= o && u < o + nn) { from_idx = sj + (u - o); flag = fj; }
                }
                if (u < total) {
                    const uint32_t v = p.dense[from_idx];
                    if (v == 0xFFFFFFFFu) bad = true;
                    p.tlist[p.nt + u] = v | flag;
                }
            }
            if (__ballot(bad)) { fail(p, PLAN_ERR_INTERNAL); return; }
        }
        p.nt += total;
        p.n_adv += n_adv;
        p.n_ret += total - n_adv;
    }
}

// emit_diff for <= 64 chains split in two: emit_issue (as soon as both vectors are known)
// computes the per-chain ranges and issues the gather of the first 64 dense-table words;
// emit_store (after the children bookkeeping has hidden that latency) writes them and any
// further chunks.  Same output as emit_diff<1>.
struct Emit {
    bool any;
    u64 am;
    uint32_t off, n, src, fl;    // per chain lane: output offset, count, dense source, advance flag
    uint32_t total, n_adv;
    uint32_t dv, dfl;            // lane u < 64: dense word and flag of output u
};
DEV void emit_issue(P &p, const VV<1> &from, const VV<1> &to, const VV<1> &dlo, const VV<1> &dhi,
                    bool allow_retreat, Emit &E) {
    const uint32_t l = lane_id();
    const bool act = l < p.A && from.v[0] != to.v[0];
    E.am = __ballot(act);
    E.any = E.am != 0;
    E.total = E.n_adv = 0;
    E.dv = 0; E.dfl = 0;
    if (!E.any) return;
    if (__ballot(act && to.v[0] < from.v[0] && !allow_retreat)) { fail(p, PLAN_ERR_INTERNAL); E.any = false; return; }
    const bool adv = to.v[0] > from.v[0];
    const uint32_t s0 = adv ? from.v[0] : to.v[0];
    const uint32_t n = act ? (adv ? to.v[0] - from.v[0] : from.v[0] - to.v[0]) : 0;
    if (__ballot(act && dlo.v[0] + s0 + n > dhi.v[0])) { fail(p, PLAN_ERR_INTERNAL); E.any = false; return; }
    const uint32_t inc = wave_scan(n);
    E.total = bcast(inc, 63);
    E.n_adv = bcast(wave_scan(adv ? n : 0), 63);
    E.off = inc - n; E.n = n; E.src = dlo.v[0] + s0; E.fl = adv ? TL_ADV : 0u;
    if (p.count_only) return;
    uint32_t from_idx = 0, flag = 0;
    for (u64 m = E.am; m; m &= m - 1) {   // the chain whose output slice holds lane l (few chains move)
        const uint32_t j = first_lane(m);
        const uint32_t o = U(bcast(E.off, j)), nn = U(bcast(E.n, j));
        if (o >= 64) break;
        if (l >= o && l < o + nn) { from_idx = U(bcast(E.src, j)) + (l - o); flag = U(bcast(E.fl, j)); }
    }
    if (l < E.total) { E.dv = p.dense[from_idx]; E.dfl = flag; }
}
DEV void emit_store(P &p, const Emit &E) {
    const uint32_t l = lane_id();
    if (uint64_t(p.nt) + E.total > p.tcap) { fail(p, PLAN_TLIST_FULL); return; }
    if (!p.count_only) {
        bool bad = l < E.total && E.dv == 0xFFFFFFFFu;
        if (l < E.total) p.tlist[p.nt + l] = E.dv | E.dfl;
        // outputs past the first 64: each moving chain's slice is one contiguous copy out of its
        // dense table
        if (E.total > 64) {
            for (u64 m = E.am; m; m &= m - 1) {
                const uint32_t j = first_lane(m);
                const uint32_t o = U(bcast(E.off, j)), nn = U(bcast(E.n, j));
                const uint32_t src = U(bcast(E.src, j)), fl = U(bcast(E.fl, j));
                const uint32_t a = max(o, 64u), b = o + nn;
                for (uint32_t u0 = a; u0 < b; u0 += 64) {
                    const uint32_t u = u0 + l;
                    if (u < b) {
                        const uint32_t v = p.dense[src + (u - o)];
                        if (v == 0xFFFFFFFFu) bad = true;
                        p.tlist[p.nt + u] = v | fl;
                    }
                }
            }
        }
        if (__ballot(bad)) { fail(p, PLAN_ERR_INTERNAL); return; }
    }
    p.nt += E.total;
    p.n_adv += E.n_adv;
    p.n_ret += E.total - E.n_adv;
}

DEV void push_cmd(P &p, uint32_t op, uint32_t a, uint32_t n, uint32_t pos) {
    if (uint64_t(p.nc) >= p.ccap) { fail(p, PLAN_CMDS_FULL); return; }
    if (lane_id() == 0 && !p.count_only) p.cmds[p.nc] = Cmd{op, a, n, pos};
    p.nc++;
}

constexpr uint8_t MERGE_BIT = 0x80;   // pending byte: parent count (<= 127) | merge flag

// Next entry to consume: the todo top, unless it is a merge and a non-merge is ready
// (txn_trace.rs:249-266).  Pops it.
DEV uint32_t pick(P &p, uint32_t &top) {
    const uint32_t l = lane_id();
    uint32_t idx = U(p.todo[top - 1]);
    if (p.pending[idx] & MERGE_BIT) {
        int found = -1;
        for (int hi = int(top) - 1; hi >= 0 && found < 0; hi -= 64) {
            const int i = hi - int(l);
            const bool ok = i >= 0 && !(p.pending[p.todo[i]] & MERGE_BIT);
            const u64 m = __ballot(ok);
            if (m) found = hi - int(first_lane(m));
        }
        if (found >= 0) {
            idx = U(p.todo[found]);
            if (l == 0) p.todo[found] = p.todo[top - 1];
            wave_fence();
        }
    }
    top--;
    return idx;
}

template <int K>
DEV void plan_doc(P &p, PlanResult *res) {
    const uint32_t l = lane_id();
    VV<K> vf, vp, dlo, dhi;
    vv_zero(vf);
    // each chain's dense-table slice, kept in registers
#pragma unroll
    for (int k = 0; k < K; k++) {
        const uint32_t a = l + 64 * k;
        dlo.v[k] = a < p.A ? p.doff[a] : 0;
        dhi.v[k] = a < p.A ? p.doff[a + 1] : 0;
    }
    // pending parent counts (+ merge flag); the todo stack holds the roots, first root on top
    uint32_t top = 0;
    bool bad_np = false;
    for (uint32_t c = 0; c < p.ne; c += 64) {
        const uint32_t e = c + l;
        if (e < p.ne) {
            const uint32_t np = p.erec[size_t(e) * EREC_HEAD + R_NP];
            if (np > 0x7Fu) bad_np = true;
            p.pending[e] = uint8_t(min(np, 0x7Fu) | (np >= 2 ? MERGE_BIT : 0));
        }
    }
    for (int c = int((p.ne + 63) / 64) - 1; c >= 0; c--) {
        if (!charge(p)) break;
        const uint32_t e = uint32_t(c) * 64 + (63 - l);   // descending entry index across lanes
        const bool root = e < p.ne && p.erec[size_t(e) * EREC_HEAD + R_NP] == 0;
        const u64 m = __ballot(root);
        const uint32_t rank = uint32_t(__popcll(m & ((1ull << l) - 1ull)));
        if (top + uint32_t(__popcll(m)) > PLAN_TODO_CAP) { fail(p, PLAN_TODO_FULL); break; }
        if (root) p.todo[top + rank] = uint16_t(e);
        top += uint32_t(__popcll(m));
    }
    if (__ballot(bad_np)) fail(p, PLAN_WIDE_MERGE);
    wave_fence();
    tk(p);
    PT(5);
    uint32_t f = 0xFFFFFFFFu;   // current frontier: ROOT or one LV
    bool have = top > 0;
    uint32_t idx = have ? pick(p, top) : 0;
    uint32_t rw = have ? load_rec(p, idx) : 0;
    while (have && !p.err) {
        if (!charge(p)) break;
        // the entry's op runs, agent runs and children: independent loads, issued together
        const uint32_t np = R(rw, R_NP), op0 = R(rw, R_OP0), nop = R(rw, R_NOP), ch0 = R(rw, R_CH0),
                       nch = R(rw, R_NCH), chain = R(rw, R_CHAIN), seq0 = R(rw, R_SEQ0);
        PT(0);
        const uint32_t e_start = R(rw, R_START), e_end = R(rw, R_END);
        // speculation: the entry's last child is usually the next one consumed
        const uint32_t spec = R(rw, R_LASTCH);
        const uint32_t rw_spec = spec != 0xFFFFFFFFu ? load_rec(p, spec) : 0;
        // (four scalars, not a Cmd: a struct assigned under a branch goes through scratch)
        const uint32_t *opw = reinterpret_cast<const uint32_t *>(p.opc);
        uint32_t oc0 = 0, oc1 = 0, oc2 = 0, oc3 = 0;
        if (l < nop && !p.count_only) {
            const size_t w = 4 * size_t(op0 + l);
            oc0 = opw[w]; oc1 = opw[w + 1]; oc2 = opw[w + 2]; oc3 = opw[w + 3];
        }
        const uint32_t ch = l < nch ? p.child[ch0 + l] : 0;
        // version vector of the parents
        if (np == 1 && R(rw, R_PAR0) == f) {
            vp = vf;
        } else {
            // parents' vectors: each parent entry's row plus its chain's ops up to the parent;
            // up to 4 parents' rows in flight at once
            vv_zero(vp);
            const uint32_t po = R(rw, R_POFF);
            for (uint32_t j0 = 0; j0 < np; j0 += 4) {
                uint32_t pe[4], pc[4], pn[4];
                VV<K> t[4];
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    const uint32_t j = j0 + jj;
                    pe[jj] = pc[jj] = pn[jj] = 0;
                    if (j < np) {
                        if (j < 2) {
                            pe[jj] = R(rw, R_PENT0 + 3 * int(j));
                            pc[jj] = R(rw, R_PCH0 + 3 * int(j));
                            pn[jj] = R(rw, R_PCNT0 + 3 * int(j));
                        } else {
                            pe[jj] = U(p.pent[po + j]);
                            pc[jj] = U(p.pch[po + j]);
                            pn[jj] = U(p.pcnt[po + j]);
                        }
                        load_row(p, pe[jj], t[jj]);
                    }
                }
#pragma unroll
                for (int jj = 0; jj < 4; jj++) {
                    if (j0 + jj >= np) break;
                    vv_max(vp, t[jj]);
#pragma unroll
                    for (int k = 0; k < K; k++)
                        if (pc[jj] == l + 64 * uint32_t(k)) vp.v[k] = max(vp.v[k], pn[jj]);
                }
            }
        }
        store_row(p, idx, vp);
        PT(1);
        const VV<K> v_old = vf;
        // the frontier moves to the entry's last LV; its runs must continue the agents' chains
        vf = vp;
        fold_entry<K>(p, e_start, e_end, e_end - 1, chain, seq0, vf, true);
        if (p.err) break;
        // K = 1: the retreat / advance gather is issued now and stored after the children work
        Emit em;
        em.any = false;
        if constexpr (K == 1) {
            if (vv_differ(v_old, vp)) emit_issue(p, v_old, vp, dlo, dhi, true, em);
            if (p.err) break;
        }
        // children whose last parent this was become ready (pushed in child index order); the
        // next entry is picked and its record requested before this entry's output is written
        for (uint32_t c = 0; c < nch; c += 64) {
            const uint32_t chv = c == 0 ? ch : (c + l < nch ? p.child[ch0 + c + l] : 0);
            bool ready = false;
            if (c + l < nch) {
                const uint8_t pd = uint8_t(p.pending[chv] - 1);
                p.pending[chv] = pd;
                ready = (pd & 0x7F) == 0;
            }
            const u64 m = __ballot(ready);
            const uint32_t rank = uint32_t(__popcll(m & ((1ull << l) - 1ull)));
            if (top + uint32_t(__popcll(m)) > PLAN_TODO_CAP) { fail(p, PLAN_TODO_FULL); break; }
            if (ready) p.todo[top + rank] = uint16_t(chv);
            top += uint32_t(__popcll(m));
        }
        wave_fence();
        have = top > 0;
        if (have) {
            idx = pick(p, top);
            rw = idx == spec ? rw_spec : load_rec(p, idx);
        }
        PT(2);
        // retreat / advance to the parents, then apply the entry's op runs
        if constexpr (K == 1) {
            if (em.any) {
                const uint32_t t0 = p.nt;
                emit_store(p, em);
                if (p.err) break;
                if (p.nt > t0) push_cmd(p, CMD_TOG, t0, p.nt - t0, 0);
            }
        } else if (vv_differ(v_old, vp)) {
            const uint32_t t0 = p.nt;
            emit_diff<K>(p, v_old, vp, dlo, dhi, true);
            if (p.err) break;
            if (p.nt > t0) push_cmd(p, CMD_TOG, t0, p.nt - t0, 0);
        }
        PT(3);
        if (uint64_t(p.nc) + nop > p.ccap) { fail(p, PLAN_CMDS_FULL); break; }
        if (!p.count_only) {
            if (l < nop) {
                uint32_t *cw = reinterpret_cast<uint32_t *>(p.cmds) + 4 * size_t(p.nc + l);
                cw[0] = oc0; cw[1] = oc1; cw[2] = oc2; cw[3] = oc3;
            }
            for (uint32_t j = 64 + l; j < nop; j += 64) p.cmds[p.nc + j] = p.opc[op0 + j];
        }
        p.nc += nop;
        f = e_end - 1;
        PT(4);
    }
    // advance to the tip (cg.version): the replay then holds the checkout
    if (!p.err) {
        VV<K> vt;
        vv_zero(vt);
        for (uint32_t j = 0; j < p.ntip; j++) {
            VV<K> t;
            vv_at<K>(p, U(p.tip[2 * j]), U(p.tip[2 * j + 1]), t);
            vv_max(vt, t);
        }
        if (!p.err && vv_differ(vf, vt)) {
            const uint32_t t0 = p.nt;
            const uint32_t adv0 = p.n_adv;
            emit_diff<K>(p, vf, vt, dlo, dhi, false);
            if (!p.err && p.nt > t0) push_cmd(p, CMD_TOG, t0, p.nt - t0, 0);
            res->n_tip = uint32_t(p.n_adv - adv0);
            p.n_adv = adv0;
        }
    }
    if (l == 0) {
        for (int i = 0; i < 6; i++) res->prof[i] = p.prof ? g_pc[i] : 0;
        res->status = p.err;
        res->ncmd = p.nc;
        res->ntlist = p.nt;
        res->n_retreat = p.n_ret;
        res->n_advance = p.n_adv;
    }
}

// ---- <= 64 chains: the software-pipelined walk ------------------------------------------------
//
// Same walk, same output as plan_doc<1>, reordered so that one entry's memory round trips hide
// behind another's work:
//   * the ready stack lives in registers (Stk below): a push or pick is a few lane operations,
//     not a chain of dependent LDS reads;
//   * the next entry is picked right after the current entry's children are counted (a child
//     list of <= 2 comes from the record: its first and last child), and its record and its
//     parent version vector are requested before this entry's diff work;
//   * the parent version vector of every entry is precomputed (the prep kernel's chain
//     decomposition / build_plan_input compute it anyway), so a merge costs no parent-row
//     round trips;
//   * this entry's retreat / advance gather is issued, and written out (with its op-run
//     commands) one iteration later, behind the next entry's children / pick.
// The record sits in one VGPR (lane k: word k), fields broadcast on demand.  (Through the
// scalar cache it would share lgkmcnt with the walk's LDS traffic: every LDS read after the
// s_load would wait for it -- measured slower.)
struct Rec { uint32_t w, row; };   // the record and the entry's parent version vector (lane = chain)
DEV Rec srec(const P &p, uint32_t e) {
    const uint32_t l = lane_id();
    return Rec{load_rec(p, e), l < p.A ? p.prow[size_t(e) * p.row_stride + l] : 0u};
}
DEV uint32_t F(const Rec &r, int k) { return R(r.w, k); }

// The ready stack with its top 64 entries in registers: lane i holds position nl + i (the
// nl bottom entries sit in LDS todo[0, nl)), bit i of mm says whether lane i's entry is a merge.
// Pushes, pops and the merge-skipping pick (txn_trace.rs:249-266, same positions as pick()) are
// register operations; LDS is touched only when the stack outgrows 64 or drains into its
// bottom part.
struct Stk {
    uint32_t v;      // lane i: entry at position nl + i (i < n)
    u64 mm;          // merge flags of the register part
    uint32_t n, nl;  // entries in registers / in LDS
};
// Push the lanes of `ready` (child index order = lane order), entry in chv, merge flag in mg.
DEV bool stk_push(P &p, Stk &S, u64 ready, uint32_t chv, bool mg) {
    const uint32_t l = lane_id();
    const uint32_t cnt = uint32_t(__popcll(ready));
    if (!cnt) return true;
    if (S.nl + S.n + cnt > PLAN_TODO_CAP) { fail(p, PLAN_TODO_FULL); return false; }
    if (S.n + cnt > 64) {   // spill the register part to LDS (merge flags stay in pending[])
        if (l < S.n) p.todo[S.nl + l] = uint16_t(S.v);
        S.nl += S.n;
        S.n = 0;
        S.mm = 0;
        wave_fence();
    }
    // ready lanes in lane order onto positions n, n + 1, ... (usually one or two)
    const u64 mgm = __ballot(mg);
    uint32_t at = S.n;
    for (u64 r = ready; r; r &= r - 1, at++) {
        const uint32_t j = first_lane(r);
        const uint32_t e = bcast(chv, j);
        S.v = l == at ? e : S.v;
        if ((mgm >> j) & 1ull) S.mm |= 1ull << at;
    }
    S.n += cnt;
    return true;
}
// Pop the next entry (as pick()); has_any: S.n + S.nl > 0.
DEV uint32_t stk_pick(P &p, Stk &S) {
    const uint32_t l = lane_id();
    if (S.n == 0) {   // refill from LDS: its top 32 (or fewer) positions
        const uint32_t k = min(S.nl, 32u);
        const uint32_t base = S.nl - k;
        const uint32_t e = l < k ? uint32_t(p.todo[base + l]) : 0u;
        const bool mg = l < k && (p.pending[e] & MERGE_BIT);
        S.v = e;
        S.mm = __ballot(mg);
        S.n = k;
        S.nl = base;
    }
    const uint32_t t = S.n - 1;
    uint32_t idx = bcast(S.v, t);
    if ((S.mm >> t) & 1ull) {
        const u64 nm = ~S.mm & ((1ull << t) - 1ull);
        if (nm) {   // the highest non-merge below the top takes its place
            const uint32_t pos = 63u - uint32_t(__clzll((long long)nm));
            const uint32_t x = bcast(S.v, pos);
            S.v = l == pos ? idx : S.v;
            S.mm |= 1ull << pos;
            idx = x;
        } else if (S.nl) {   // scan the LDS part, top down
            int found = -1;
            for (int hi = int(S.nl) - 1; hi >= 0 && found < 0; hi -= 64) {
                const int i = hi - int(l);
                const bool ok = i >= 0 && !(p.pending[p.todo[i]] & MERGE_BIT);
                const u64 m = __ballot(ok);
                if (m) found = hi - int(first_lane(m));
            }
            if (found >= 0) {
                const uint32_t x = U(p.todo[found]);
                if (l == 0) p.todo[found] = uint16_t(idx);
                wave_fence();
                idx = x;
            }
        }
    }
    S.mm &= ~(1ull << t);
    S.n--;
    return U(idx);
}

DEV void plan_doc1(P &p, PlanResult *res) {
    const uint32_t l = lane_id();
    const uint32_t dlo = l < p.A ? p.doff[l] : 0, dhi = l < p.A ? p.doff[l + 1] : 0;
    VV<1> dl, dh;
    dl.v[0] = dlo; dh.v[0] = dhi;
    uint32_t top = 0;
    bool bad_np = false;
    for (uint32_t c = 0; c < p.ne; c += 64) {
        const uint32_t e = c + l;
        if (e < p.ne) {
            const uint32_t np = p.erec[size_t(e) * EREC_HEAD + R_NP];
            if (np > 0x7Fu) bad_np = true;
            p.pending[e] = uint8_t(min(np, 0x7Fu) | (np >= 2 ? MERGE_BIT : 0));
        }
    }
    for (int c = int((p.ne + 63) / 64) - 1; c >= 0; c--) {
        if (!charge(p)) break;
        const uint32_t e = uint32_t(c) * 64 + (63 - l);
        const bool root = e < p.ne && p.erec[size_t(e) * EREC_HEAD + R_NP] == 0;
        const u64 m = __ballot(root);
        const uint32_t rank = uint32_t(__popcll(m & ((1ull << l) - 1ull)));
        if (top + uint32_t(__popcll(m)) > PLAN_TODO_CAP) { fail(p, PLAN_TODO_FULL); break; }
        if (root) p.todo[top + rank] = uint16_t(e);
        top += uint32_t(__popcll(m));
    }
    if (__ballot(bad_np)) fail(p, PLAN_WIDE_MERGE);
    wave_fence();
    Stk S;
    S.v = 0; S.mm = 0; S.n = 0; S.nl = top;
    tk(p);
    PT(5);
    VV<1> vf;
    vf.v[0] = 0;
    // the previous entry's deferred output: its diff (gather in flight) and its op runs
    Emit pe_em;
    pe_em.any = false;
    uint32_t pe_nop = 0, pe_op0 = 0;
    uint4 pe_oc = make_uint4(0, 0, 0, 0);
    bool pe_have = false;
    const uint4 *opw4 = reinterpret_cast<const uint4 *>(p.opc);
    auto flush = [&]() {   // the previous entry's TOG, tlist slice and op-run commands
        if (!pe_have) return;
        if (pe_em.any) {
            const uint32_t t0 = p.nt;
            emit_store(p, pe_em);
            if (p.err) return;
            if (p.nt > t0) push_cmd(p, CMD_TOG, t0, p.nt - t0, 0);
        }
        if (uint64_t(p.nc) + pe_nop > p.ccap) { fail(p, PLAN_CMDS_FULL); return; }
        if (!p.count_only) {
            uint4 *cw = reinterpret_cast<uint4 *>(p.cmds) + p.nc;
            if (l < pe_nop) cw[l] = pe_oc;
            for (uint32_t j = 64 + l; j < pe_nop; j += 64) cw[j] = opw4[pe_op0 + j];
        }
        p.nc += pe_nop;
        pe_have = false;
    };
    bool have = S.nl > 0;
    uint32_t idx = have ? stk_pick(p, S) : 0;
    Rec rc;
    if (have) rc = srec(p, idx);
    while (have && !p.err) {
        if (!charge(p)) break;
        const uint32_t nch = F(rc, R_NCH), ch0 = F(rc, R_CH0), lastch = F(rc, R_LASTCH), firstch = F(rc, R_FIRSTCH);
        PT(0);
        // children whose last parent this is become ready (pushed in child index order); the
        // next entry is picked and its record requested before this entry's own work
        uint32_t ch = l == 0 ? firstch : lastch;
        if (nch > 2) ch = l < nch ? p.child[ch0 + l] : 0;
        for (uint32_t c = 0; c < nch; c += 64) {
            const uint32_t chv = c == 0 ? ch : (c + l < nch ? p.child[ch0 + c + l] : 0);
            bool ready = false, mg = false;
            if (c + l < nch) {
                const uint8_t pd = uint8_t(p.pending[chv] - 1);
                p.pending[chv] = pd;
                ready = (pd & 0x7F) == 0;
                mg = (pd & MERGE_BIT) != 0;
            }
            if (!stk_push(p, S, __ballot(ready), chv, mg)) break;
        }
        if (p.err) break;
        have = S.n + S.nl > 0;
        uint32_t nidx = 0;
        Rec nrc;
        if (have) {
            nidx = stk_pick(p, S);
            nrc = srec(p, nidx);
        }
        PT(2);
        // this entry's op runs (written out with its diff one iteration later)
        const uint32_t op0 = F(rc, R_OP0), nop = F(rc, R_NOP);
        uint4 oc = make_uint4(0, 0, 0, 0);
        if (l < nop && !p.count_only) oc = opw4[op0 + l];
        // the previous entry's output (its gather has been in flight since the end of its
        // iteration)
        flush();
        if (p.err) break;
        PT(4);
        const uint32_t e_start = F(rc, R_START), e_end = F(rc, R_END), po = F(rc, R_POFF), np = F(rc, R_NP);
        const uint32_t chain = F(rc, R_CHAIN), seq0 = F(rc, R_SEQ0), par0 = F(rc, R_PAR0);
        // version vector of the parents: the entry's precomputed row
        VV<1> vp;
        vp.v[0] = rc.row;
        (void)po; (void)np; (void)par0;
        PT(1);
        const VV<1> v_old = vf;
        vf = vp;
        fold_entry<1>(p, e_start, e_end, e_end - 1, chain, seq0, vf, true);
        if (p.err) break;
        pe_em.any = false;
        if (vv_differ(v_old, vp)) emit_issue(p, v_old, vp, dl, dh, true, pe_em);
        if (p.err) break;
        pe_have = true;
        pe_nop = nop; pe_op0 = op0;
        pe_oc = oc;
        idx = nidx;
        rc = nrc;
        PT(3);
    }
    if (!p.err) flush();
    // advance to the tip (cg.version): the replay then holds the checkout
    if (!p.err) {
        VV<1> vt;
        vv_zero(vt);
        for (uint32_t j = 0; j < p.ntip; j++) {
            const uint32_t tlv = U(p.tip[2 * j]), te = U(p.tip[2 * j + 1]);
            const Rec tr = srec(p, te);
            VV<1> t;
            t.v[0] = tr.row;
            fold_entry<1>(p, F(tr, R_START), F(tr, R_END), tlv, F(tr, R_CHAIN), F(tr, R_SEQ0), t, false);
            vv_max(vt, t);
        }
        if (!p.err && vv_differ(vf, vt)) {
            const uint32_t t0 = p.nt;
            const uint32_t adv0 = p.n_adv;
            emit_diff<1>(p, vf, vt, dl, dh, false);
            if (!p.err && p.nt > t0) push_cmd(p, CMD_TOG, t0, p.nt - t0, 0);
            res->n_tip = uint32_t(p.n_adv - adv0);
            p.n_adv = adv0;
        }
    }
    if (l == 0) {
        for (int i = 0; i < 6; i++) res->prof[i] = p.prof ? g_pc[i] : 0;
        res->status = p.err;
        res->ncmd = p.nc;
        res->ntlist = p.nt;
        res->n_retreat = p.n_ret;
        res->n_advance = p.n_adv;
    }
}

// ---- <= 64 chains, two phases -----------------------------------------------------------------
//
// The walk order depends only on the graph (children, merge flags), and what a walk step emits
// depends only on the step's entry and the one before it: the frontier before step i is the
// previous entry's parent vector with that entry's own LVs folded in (fold_entry), the frontier it
// moves to is entry i's parent vector.  So:
//   phase A (sequential, wave-uniform): the spanning-tree order alone -- pick, children
//     bookkeeping, one record load per step -- written to the document's scratch (p.base);
//   phase B (lane-parallel, lane = walk step): each step's retreat / advance ranges and op runs
//     sized, offsets by prefix sums, then every step's TOG command, tlist slice and op-run
//     commands written by its own lane.
// Same output as plan_doc1 (tested against the host walk).
constexpr uint32_t kSplitLaneTl = 24, kSplitLaneOps = 8;   // per-lane step writes up to these sizes
constexpr uint32_t kSplitRegChains = 4;   // up to this many moving chains per step: output-parallel chunk writes
constexpr uint32_t kSplitSegChunk = 4096;
constexpr uint32_t kSplitCopyDepth = 8;   // big steps: 8 x 64 dense-table loads per round trip   // ... for chunks writing up to this many entries / commands
DEV void plan_doc_split(P &p, PlanResult *res) {
    const uint32_t l = lane_id();
    uint32_t top = 0;
    bool bad_np = false;
    for (uint32_t c = 0; c < p.ne && !p.walk; c += 64) {
        const uint32_t e = c + l;
        if (e < p.ne) {
            const uint32_t np = p.erec[size_t(e) * EREC_HEAD + R_NP];
            if (np > 0x7Fu) bad_np = true;
            p.pending[e] = uint8_t(min(np, 0x7Fu) | (np >= 2 ? MERGE_BIT : 0));
        }
    }
    for (int c = p.walk ? -1 : int((p.ne + 63) / 64) - 1; c >= 0; c--) {
        if (!charge(p)) break;
        const uint32_t e = uint32_t(c) * 64 + (63 - l);
        const bool root = e < p.ne && p.erec[size_t(e) * EREC_HEAD + R_NP] == 0;
        const u64 m = __ballot(root);
        const uint32_t rank = uint32_t(__popcll(m & ((1ull << l) - 1ull)));
        if (top + uint32_t(__popcll(m)) > PLAN_TODO_CAP) { fail(p, PLAN_TODO_FULL); break; }
        if (root) p.todo[top + rank] = uint16_t(e);
        top += uint32_t(__popcll(m));
    }
    if (__ballot(bad_np)) fail(p, PLAN_WIDE_MERGE);
    wave_fence();
    tk(p);
    PT(5);
    // ---- phase A: the order (walk_kernel's, when it ran) ----
    uint32_t *order = p.order;   // ne words
    Stk S;
    S.v = 0; S.mm = 0; S.n = 0; S.nl = top;
    bool have = S.nl > 0 && !p.err && !p.walk;
    uint32_t idx = have ? stk_pick(p, S) : 0;
    uint32_t rw = have ? load_rec(p, idx) : 0;
    uint32_t ns = 0;
    uint32_t ordv = 0;   // lane j: order[64 * (ns / 64) + j] until its 64 are stored together
    if (p.walk) {
        const uint32_t wst = U(p.walk[0]) & 0xFFFFu;   // (high 16 bits: the walk's stack depth)
        ns = U(p.walk[1]);
        if (wst) fail(p, wst);
    }
    while (have && !p.err) {
        if (!charge(p)) break;
        if (ns >= p.ne) { fail(p, PLAN_ERR_INTERNAL); break; }
        ordv = l == (ns & 63u) ? idx : ordv;
        if ((ns & 63u) == 63u) order[ns - 63 + l] = ordv;
        ns++;
        const uint32_t nch = R(rw, R_NCH), ch0 = R(rw, R_CH0), lastch = R(rw, R_LASTCH), firstch = R(rw, R_FIRSTCH);
        uint32_t ch = l == 0 ? firstch : lastch;
        if (nch > 2) ch = l < nch ? p.child[ch0 + l] : 0;
        for (uint32_t c = 0; c < nch; c += 64) {
            const uint32_t chv = c == 0 ? ch : (c + l < nch ? p.child[ch0 + c + l] : 0);
            bool ready = false, mg = false;
            if (c + l < nch) {
                const uint8_t pd = uint8_t(p.pending[chv] - 1);
                p.pending[chv] = pd;
                ready = (pd & 0x7F) == 0;
                mg = (pd & MERGE_BIT) != 0;
            }
            if (!stk_push(p, S, __ballot(ready), chv, mg)) break;
        }
        if (p.err) break;
        have = S.n + S.nl > 0;
        if (have) {
            idx = stk_pick(p, S);
            rw = load_rec(p, idx);
        }
    }
    if (!p.walk && (ns & 63u) && l < (ns & 63u)) order[(ns & ~63u) + l] = ordv;
    PT(0);
    // every lane reads the order phase A wrote
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // each chain's dense-table slice, in LDS (the todo stack's space: phase A is done)
    uint32_t *sdoff = reinterpret_cast<uint32_t *>(p.todo);
    if (l <= p.A) sdoff[l] = p.doff[l];
    wave_fence();
    // ---- phase B: per step, lane = step ----
    const uint32_t A = p.A;
    const uint32_t rs = p.row_stride;
    uint32_t err_step = 0xFFFFFFFFu, err_code = 0;
    uint32_t last_e = 0;
    for (uint32_t c0 = 0; c0 < ns && !p.err; c0 += 64) {
        const uint32_t i = c0 + l;
        const bool valid = i < ns;
        const uint32_t e = valid ? order[i] : 0;
        const bool hp = valid && i > 0;
        const uint32_t ep = hp ? order[i - 1] : 0;
        const uint4 *r4 = reinterpret_cast<const uint4 *>(p.erec);   // the heads (32 bytes each)
        const uint4 a0 = r4[size_t(e) * (EREC_HEAD / 4)], a1 = r4[size_t(e) * (EREC_HEAD / 4) + 1];
        uint4 b0 = make_uint4(0, 0, 0, 0), b1 = make_uint4(0, 0, 0, 0);
        if (hp) { b0 = r4[size_t(ep) * (EREC_HEAD / 4)]; b1 = r4[size_t(ep) * (EREC_HEAD / 4) + 1]; }
        const uint32_t e_start = a0.x, e_end = a0.y, op0 = a1.x, nop = a1.y, chain = a1.z, seq0 = a1.w;
        const uint32_t p_start = b0.x, p_end = b0.y, p_chain = b1.z, p_seq0 = b1.w;
        uint32_t code = 0;
        if (valid && (chain >= A || e_end <= e_start)) code = PLAN_ERR_INTERNAL;
        if (valid && p.prow[size_t(e) * rs + min(chain, rs - 1)] != seq0 && !code) code = PLAN_NOT_CHAIN;
        // the frontier before the step (the previous entry folded) against the step's parents
        uint32_t total = 0, nadv = 0;
        // the step's first kSplitRegChains moving chains (ascending): range length, dense source,
        // advance bit; more moving chains than that send the chunk to the per-step writes
        uint32_t sn[kSplitRegChains], ss[kSplitRegChains], sadv = 0, nmov = 0;
#pragma unroll
        for (uint32_t a = 0; a < kSplitRegChains; a++) sn[a] = ss[a] = 0;
        auto chain_diff = [&](uint32_t a, uint32_t to, uint32_t from) {
            if (hp && a == p_chain) from = p_seq0 + (p_end - p_start);
            const bool adv = to > from;
            const uint32_t n = adv ? to - from : from - to;
            const uint32_t s0 = adv ? from : to;
            if (n && sdoff[a] + s0 + n > sdoff[a + 1] && !code) code = PLAN_ERR_INTERNAL;
            total += n;
            nadv += adv ? n : 0;
            if (n) {
#pragma unroll
                for (uint32_t q = 0; q < kSplitRegChains; q++)
                    if (nmov == q) { sn[q] = n; ss[q] = sdoff[a] + s0; }
                if (adv && nmov < kSplitRegChains) sadv |= 1u << nmov;
                nmov++;
            }
        };
        if ((rs & 3u) == 0) {   // rows 16-byte aligned (device staging): four chains per load
            const uint4 *r4e = reinterpret_cast<const uint4 *>(p.prow + size_t(e) * rs);
            const uint4 *r4p = reinterpret_cast<const uint4 *>(p.prow + size_t(ep) * rs);
            for (uint32_t a = 0; a < A; a += 4) {
                const uint4 t4 = valid ? r4e[a / 4] : make_uint4(0, 0, 0, 0);
                const uint4 f4 = hp ? r4p[a / 4] : make_uint4(0, 0, 0, 0);
                chain_diff(a, t4.x, f4.x);
                if (a + 1 < A) chain_diff(a + 1, t4.y, f4.y);
                if (a + 2 < A) chain_diff(a + 2, t4.z, f4.z);
                if (a + 3 < A) chain_diff(a + 3, t4.w, f4.w);
            }
        } else {
            for (uint32_t a = 0; a < A; a++)
                chain_diff(a, valid ? p.prow[size_t(e) * rs + a] : 0u, hp ? p.prow[size_t(ep) * rs + a] : 0u);
        }
        if (!valid) total = nadv = 0;
        const uint32_t ncmd = valid ? (total ? 1u : 0u) + nop : 0u;
        // offsets: prefix sums over the chunk's steps
        const uint32_t ic = wave_scan(ncmd), it = wave_scan(total);
        const uint32_t co = p.nc + ic - ncmd, to0 = p.nt + it - total;
        const uint32_t sum_c = bcast(ic, 63), sum_t = bcast(it, 63);
        const uint32_t sum_adv = bcast(wave_scan(nadv), 63);
        PT(1);
        if (code) { err_step = i; err_code = code; }
        const u64 em = __ballot(code != 0);
        if (em) {   // the first failing step ends the walk, as plan_doc1 stops there
            fail(p, bcast(code, first_lane(em)));
            break;
        }
        if (uint64_t(p.nc) + sum_c > p.ccap) { fail(p, PLAN_CMDS_FULL); break; }
        if (uint64_t(p.nt) + sum_t > p.tcap) { fail(p, PLAN_TLIST_FULL); break; }
        // small steps: each lane writes its own step; a step with a long diff or many op runs
        // is written by the whole wave afterwards (a lane copying node_nodecc's thousands of
        // entries alone would serialise the chunk)
        // A <= 4: output-parallel chunk writes, unless the chunk's output is long (node_nodecc's
        // steps retreat / advance thousands of entries each): then step by step, each step's
        // ranges copied contiguously by the whole wave
        const bool seg_chunk = sum_t > kSplitSegChunk || sum_c > kSplitSegChunk;
        const bool outpar = !__ballot(valid && nmov > kSplitRegChains) && !seg_chunk;
        const bool big = valid && (!outpar ? (seg_chunk || total > kSplitLaneTl || nop > kSplitLaneOps) : false);
        if (!p.count_only && outpar) {
            // output-parallel: output u of the chunk belongs to the first step whose inclusive
            // prefix exceeds it (a binary search over the lanes), inside it to the chain range
            // that covers it; 4 x 64 outputs per round, their loads in flight together
            const uint32_t T0 = p.nt, C0 = p.nc;
            bool bad = false;
            for (uint32_t r = 0; r < sum_t; r += 256) {
                uint32_t val[4], fl[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t u = r + 64 * uint32_t(q) + l;
                    uint32_t j = 0;
#pragma unroll
                    for (uint32_t st = 32; st; st >>= 1)
                        if (u >= uint32_t(__shfl(int(it), int(j + st - 1)))) j += st;
                    j = min(j, 63u);
                    const uint32_t w = u - (uint32_t(__shfl(int(it), int(j))) - uint32_t(__shfl(int(total), int(j))));
                    const uint32_t av = uint32_t(__shfl(int(sadv), int(j)));
                    uint32_t before = 0, src = 0, f = 0;
                    bool found = false;
#pragma unroll
                    for (uint32_t a = 0; a < kSplitRegChains; a++) {
                        const uint32_t na = uint32_t(__shfl(int(sn[a]), int(j)));
                        const uint32_t sa = uint32_t(__shfl(int(ss[a]), int(j)));
                        if (!found && w < before + na) { src = sa + (w - before); f = (av >> a) & 1u ? TL_ADV : 0u; found = true; }
                        before += na;
                    }
                    val[q] = u < sum_t ? p.dense[src] : 0u;
                    fl[q] = f;
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t u = r + 64 * uint32_t(q) + l;
                    if (u < sum_t) {
                        bad |= val[q] == 0xFFFFFFFFu;
                        p.tlist[T0 + u] = val[q] | fl[q];
                    }
                }
            }
            for (uint32_t r = 0; r < sum_c; r += 256) {   // 4 x 64 commands per round
                Cmd cv[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t u = r + 64 * uint32_t(q) + l;
                    uint32_t j = 0;
#pragma unroll
                    for (uint32_t st = 32; st; st >>= 1)
                        if (u >= uint32_t(__shfl(int(ic), int(j + st - 1)))) j += st;
                    j = min(j, 63u);
                    const uint32_t k = u - (uint32_t(__shfl(int(ic), int(j))) - uint32_t(__shfl(int(ncmd), int(j))));
                    const uint32_t tj = uint32_t(__shfl(int(total), int(j))), t0j = uint32_t(__shfl(int(to0), int(j)));
                    const uint32_t o0j = uint32_t(__shfl(int(op0), int(j)));
                    cv[q] = Cmd{CMD_TOG, t0j, tj, 0};
                    if (u < sum_c && !(tj && k == 0)) cv[q] = p.opc[o0j + k - (tj ? 1u : 0u)];
                }
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t u = r + 64 * uint32_t(q) + l;
                    if (u < sum_c) p.cmds[C0 + u] = cv[q];
                }
            }
            if (bad) { err_step = i; err_code = PLAN_ERR_INTERNAL; }
        }
        if (!p.count_only && valid && !big && !outpar) {
            uint32_t cw = co;
            bool bad = false;
            if (total) {
                p.cmds[cw++] = Cmd{CMD_TOG, to0, total, 0};
                uint32_t u = to0;
                for (uint32_t a = 0; a < A; a++) {
                    const uint32_t to = p.prow[size_t(e) * rs + a];
                    uint32_t from = hp ? p.prow[size_t(ep) * rs + a] : 0;
                    if (hp && a == p_chain) from = p_seq0 + (p_end - p_start);
                    if (to == from) continue;
                    const bool adv = to > from;
                    const uint32_t n = adv ? to - from : from - to;
                    const uint32_t src = sdoff[a] + (adv ? from : to), fl = adv ? TL_ADV : 0u;
                    uint32_t k = 0;
                    for (; k + 4 <= n; k += 4) {   // four loads in flight per round
                        uint32_t v[4];
#pragma unroll
                        for (int q = 0; q < 4; q++) v[q] = p.dense[src + k + q];
#pragma unroll
                        for (int q = 0; q < 4; q++) { bad |= v[q] == 0xFFFFFFFFu; p.tlist[u + q] = v[q] | fl; }
                        u += 4;
                    }
                    for (; k < n; k++) {
                        const uint32_t v = p.dense[src + k];
                        bad |= v == 0xFFFFFFFFu;
                        p.tlist[u++] = v | fl;
                    }
                }
            }
            for (uint32_t j = 0; j < nop; j++) p.cmds[cw + j] = p.opc[op0 + j];
            if (bad) { err_step = i; err_code = PLAN_ERR_INTERNAL; }
        }
        PT(2);
        if (!p.count_only) {
            for (u64 bm = __ballot(big); bm; bm &= bm - 1) {   // the big steps, one at a time
                const uint32_t j = first_lane(bm);
                const uint32_t be = U(bcast(e, j)), bep = U(bcast(ep, j)), bhp = U(bcast(hp ? 1u : 0u, j));
                const uint32_t bpc = U(bcast(p_chain, j)), bpv = U(bcast(p_seq0 + (p_end - p_start), j));
                const uint32_t bto = U(bcast(to0, j)), bco = U(bcast(co, j)), btot = U(bcast(total, j));
                const uint32_t bop0 = U(bcast(op0, j)), bnop = U(bcast(nop, j));
                uint32_t cw = bco;
                if (btot) {
                    if (l == 0) p.cmds[cw] = Cmd{CMD_TOG, bto, btot, 0};
                    cw++;
                    // lane = chain: its range, its offset in the step's slice, then 64 outputs per round
                    const uint32_t to = l < A ? p.prow[size_t(be) * rs + l] : 0u;
                    uint32_t from = bhp && l < A ? p.prow[size_t(bep) * rs + l] : 0u;
                    if (bhp && l == bpc) from = bpv;
                    const bool adv = to > from;
                    const uint32_t n = adv ? to - from : from - to;
                    const uint32_t src = (l < A ? sdoff[l] : 0u) + (adv ? from : to), fl = adv ? TL_ADV : 0u;
                    const uint32_t off = wave_scan(n) - n;
                    bool bad = false;
                    for (u64 am = __ballot(n != 0); am; am &= am - 1) {
                        const uint32_t a = first_lane(am);
                        const uint32_t o = U(bcast(off, a)), nn = U(bcast(n, a)), sa = U(bcast(src, a)), fa = U(bcast(fl, a));
                        for (uint32_t u0 = 0; u0 < nn; u0 += 64 * kSplitCopyDepth) {   // loads in flight together
                            uint32_t v[kSplitCopyDepth];
#pragma unroll
                            for (int q = 0; q < int(kSplitCopyDepth); q++) {
                                const uint32_t u = u0 + 64 * uint32_t(q) + l;
                                v[q] = u < nn ? p.dense[sa + u] : 0u;
                            }
#pragma unroll
                            for (int q = 0; q < int(kSplitCopyDepth); q++) {
                                const uint32_t u = u0 + 64 * uint32_t(q) + l;
                                if (u < nn) {
                                    bad |= v[q] == 0xFFFFFFFFu;
                                    p.tlist[bto + o + u] = v[q] | fa;
                                }
                            }
                        }
                    }
                    if (__ballot(bad)) err_code = PLAN_ERR_INTERNAL;
                }
                for (uint32_t k = l; k < bnop; k += 64) p.cmds[cw + k] = p.opc[bop0 + k];
            }
        }
        PT(4);
        if (__ballot(err_code != 0)) { fail(p, PLAN_ERR_INTERNAL); break; }
        p.nc += sum_c;
        p.nt += sum_t;
        p.n_adv += sum_adv;
        p.n_ret += sum_t - sum_adv;
        last_e = U(bcast(e, min(63u, ns - 1 - c0)));
    }
    (void)err_step;
    PT(3);
    // advance to the tip (cg.version): from the last step's entry folded
    if (!p.err) {
        VV<1> vf;
        vf.v[0] = 0;
        if (ns) {
            const uint32_t rl = load_rec(p, last_e);
            vf.v[0] = l < A ? p.prow[size_t(last_e) * rs + l] : 0u;
            fold_entry<1>(p, R(rl, R_START), R(rl, R_END), R(rl, R_END) - 1, R(rl, R_CHAIN), R(rl, R_SEQ0), vf, false);
        }
        VV<1> dl, dh;
        dl.v[0] = l < A ? sdoff[l] : 0u;
        dh.v[0] = l < A ? sdoff[l + 1] : 0u;
        VV<1> vt;
        vv_zero(vt);
        for (uint32_t j = 0; j < p.ntip && !p.err; j++) {
            const uint32_t tlv = U(p.tip[2 * j]), te = U(p.tip[2 * j + 1]);
            const Rec tr = srec(p, te);
            VV<1> t;
            t.v[0] = tr.row;
            fold_entry<1>(p, F(tr, R_START), F(tr, R_END), tlv, F(tr, R_CHAIN), F(tr, R_SEQ0), t, false);
            vv_max(vt, t);
        }
        if (!p.err && vv_differ(vf, vt)) {
            const uint32_t t0 = p.nt;
            const uint32_t adv0 = p.n_adv;
            emit_diff<1>(p, vf, vt, dl, dh, false);
            if (!p.err && p.nt > t0) push_cmd(p, CMD_TOG, t0, p.nt - t0, 0);
            res->n_tip = uint32_t(p.n_adv - adv0);
            p.n_adv = adv0;
        }
    }
    if (l == 0) {
        for (int i = 0; i < 6; i++) res->prof[i] = p.prof ? g_pc[i] : 0;
        res->status = p.err;
        res->ncmd = p.nc;
        res->ntlist = p.nt;
        res->n_retreat = p.n_ret;
        res->n_advance = p.n_adv;
    }
}

// K = agent chunks per lane.  Documents with <= 64 agents run in the K = 1 instantiation, the
// others (<= PLAN_MAX_AGENTS) in the wide one; each kernel skips the other's documents.
template <int K, bool SPLIT = false>
DEV void plan_entry(const PlanParams &Q) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lds16[];
    if (blockIdx.x >= Q.n_docs) return;
    const uint32_t d = U(Q.doc_list ? Q.doc_list[blockIdx.x] : blockIdx.x);
    const PlanDesc pd = Q.docs[d];
    PlanResult *res = Q.results + d;
    if (pd.skip) return;   // planned on the host
    const uint32_t A = U(pd.n_agents);
    if (K == 1 ? A > 64 : A <= 64) return;
    P p;
    p.erec = Q.erec + pd.erec_off;
    p.par = Q.par + pd.par_off;
    p.pent = Q.pent + pd.par_off;
    p.pch = Q.pch + pd.par_off;
    p.pcnt = Q.pcnt + pd.par_off;
    p.child = Q.child + pd.child_off;
    p.opc = Q.opc + pd.op_off;
    p.doff = Q.doff + pd.doff_off;
    p.dense = Q.dense + pd.dense_off;
    p.tip = Q.tip + pd.tip_off * 2;
    p.ne = U(pd.ne);
    p.A = A;
    p.ntip = U(pd.ntip);
    p.n_lv = U(pd.n_lv);
    p.todo = lds16;
    p.pending = reinterpret_cast<uint8_t *>(lds16 + PLAN_TODO_CAP);
    p.base = Q.base + pd.base_off;
    p.prow = Q.prow + pd.prow_off;
    p.order = Q.order + pd.erec_off / EREC_WORDS;
    p.walk = SPLIT && Q.walk ? Q.walk + 2 * size_t(d) : nullptr;
    p.row_stride = pd.row_stride;
    p.cmds = Q.cmds + pd.cmd_off;
    p.tlist = Q.tlist + pd.tlist_off;
    p.count_only = Q.count_only;
    p.ccap = Q.count_only ? 0xFFFFFFFFu : U(pd.ccap);
    p.tcap = Q.count_only ? 0xFFFFFFFFu : U(pd.tcap);
    p.nc = p.nt = p.err = 0;
    p.steps = 0;
    p.limit = uint32_t(min<uint64_t>(1024ull * (uint64_t(p.ne) + 16) + 4ull * pd.n_lv + (1u << 20), 0xFFFFFFF0ull));
    p.n_ret = p.n_adv = 0;
    p.prof = Q.prof;
    res->n_tip = 0;
    if (p.ne > Q.lds_entries) {
        if (lane_id() == 0) res->status = PLAN_ERR_INTERNAL;
        return;
    }
#ifndef DTGPU_PLAN_OLD
    if constexpr (K == 1) {
        if constexpr (SPLIT) plan_doc_split(p, res);
        else plan_doc1(p, res);
    } else {
        plan_doc<K>(p, res);
    }
#else
    plan_doc<K>(p, res);
#endif
}

#ifndef DTGPU_PLAN_WAVES
#define DTGPU_PLAN_WAVES 6   // occupancy target of the <= 64-chain planner (tuning knob)
#endif
template <bool SPLIT>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DTGPU_PLAN_WAVES))) void plan_kernel_1(PlanParams Q) {
    plan_entry<1, SPLIT>(Q);
}
__global__ __launch_bounds__(64) void plan_kernel_wide(PlanParams Q) { plan_entry<PLAN_MAX_AGENTS / 64>(Q); }


// ---- walk_kernel: the spanning-tree orders of CHAIN_WALK_DOCS documents per wave ----------------
// plan_doc_split's phase A for <= 64-chain documents, each on a 16-lane group: the same stack
// (a flat LDS stack here: push at the top, pick = the top unless it is a merge and a non-merge is
// below, which then swaps places with it), the same pending counts, one record load per step.
// A walk is a sequential chain of dependent steps whose work is a few lane operations, so one
// document per wave left most issue slots to waiting; four share each instruction here.  The plan
// kernel then runs phase B from the stored order (PlanParams.walk: status, steps).
constexpr uint32_t WG = 16, WALK_DOCS = 64 / WG;
DEV uint32_t wsh(uint32_t v, uint32_t src) { return uint32_t(__shfl(int(v), int(src))); }
// s_waitcnt vmcnt(0) alone, inside the branch that loads: where the paths meet the compiler then
// sees nothing pending and places no wait of its own -- a wait there would also wait for the
// order store of the step before (vmcnt counts stores), a full memory round trip per 16 steps
DEV void walk_wait_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }
template <bool CSR>
__global__ __launch_bounds__(64) void walk_kernel(PlanParams Q) {
    extern __shared__ __attribute__((aligned(16))) uint16_t wl16[];
    const uint32_t l = lane_id(), g = l / WG, c = l % WG, base = g * WG;
    const uint32_t cap = Q.todo_cap ? Q.todo_cap : PLAN_TODO_CAP;   // stack slots (even)
    const uint32_t stride = cap + (Q.lds_entries + 1) / 2;   // u16 per group: stack, pending bytes
    uint16_t *todo = wl16 + g * stride;
    uint8_t *pend = reinterpret_cast<uint8_t *>(todo + cap);
    const uint32_t li = blockIdx.x * WALK_DOCS + g;
    bool on = li < Q.n_docs;
    const uint32_t d = on ? (Q.doc_list ? Q.doc_list[li] : li) : 0u;
    const PlanDesc pd = Q.docs[d];
    on = on && !pd.skip && pd.n_agents <= 64 && pd.ne <= Q.lds_entries;
    const uint32_t ne = on ? pd.ne : 0u;
    const uint32_t *erec = Q.erec + pd.erec_off;
    const uint32_t *child = Q.child + pd.child_off;
    const uint32_t *coff = CSR ? Q.coff + pd.coff_off : nullptr, *poff = CSR ? Q.poff + pd.poff_off : nullptr;
    uint32_t *order = Q.order + pd.erec_off / EREC_WORDS;
    uint32_t err = 0, top = 0, hw = 0;   // hw: the stack's high-water mark
    const uint32_t limit = uint32_t(min<uint64_t>(1024ull * (uint64_t(ne) + 16) + 4ull * pd.n_lv + (1u << 20), 0xFFFFFFF0ull));
    uint32_t steps = 0;
    const uint32_t below = (1u << c) - 1u;
    bool bad_np = false;
    for (uint32_t e = c; e < ne; e += WG) {
        const uint32_t np = CSR ? poff[e + 1] - poff[e] : erec[size_t(e) * EREC_HEAD + R_NP];
        if (np > 0x7Fu) bad_np = true;
        pend[e] = uint8_t(min(np, 0x7Fu) | (np >= 2 ? MERGE_BIT : 0));
    }
    if ((uint32_t(__ballot(bad_np) >> base) & 0xFFFFu) && on) err = PLAN_WIDE_MERGE;
    // roots, highest index first, so the lowest root ends on the top
    for (int cb = int((ne + WG - 1) / WG) - 1; cb >= 0 && !err; cb--) {
        const uint32_t e = uint32_t(cb) * WG + (WG - 1 - c);
        const bool root = e < ne && (CSR ? poff[e + 1] == poff[e] : erec[size_t(e) * EREC_HEAD + R_NP] == 0);
        const uint32_t m = uint32_t(__ballot(root) >> base) & 0xFFFFu;
        if (top + uint32_t(__popc(m)) > cap) { err = PLAN_TODO_FULL; break; }
        if (root) todo[top + uint32_t(__popc(m & below))] = uint16_t(e);
        top += uint32_t(__popc(m));
        hw = max(hw, top);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    uint32_t ns = 0, ordv = 0;
    uint32_t wb = 0xFFFFFFFFu;   // CSR: the 64 entries whose records the group holds
    uint2 wk[4] = {};
    bool act = on && !err && top > 0;
    while (__ballot(act)) {
        if (act) {
            if (++steps > limit) { err = PLAN_ERR_INTERNAL; act = false; }
        }
        if (act) {
            // pick: the top, unless it is a merge and a non-merge lies below (it takes its place)
            const uint32_t t = top - 1;
            uint32_t idx = todo[t];
            if (pend[idx] & MERGE_BIT) {
                int found = -1;
                for (int hi = int(t) - 1; hi >= 0 && found < 0; hi -= int(WG)) {
                    const int i = hi - int(c);
                    const bool okk = i >= 0 && !(pend[todo[i]] & MERGE_BIT);
                    const uint32_t m = uint32_t(__ballot(okk) >> base) & 0xFFFFu;
                    if (m) found = hi - (__ffs(int(m)) - 1);
                }
                if (found >= 0) {
                    const uint32_t x = todo[found];
                    __builtin_amdgcn_wave_barrier();
                    if (c == 0) todo[found] = uint16_t(idx);
                    idx = x;
                }
            }
            top = t;
            ordv = c == (ns & (WG - 1)) ? idx : ordv;
            if ((ns & (WG - 1)) == WG - 1) order[ns - (WG - 1) + c] = ordv;
            ns++;
            // the entry's children (first / last from the record; a longer list from the CSR)
            uint32_t nch, ch0, firstch = 0, lastch = 0;
            if (CSR) {   // prep's first half: {children | first slot << 16, first | last child << 16}
                // the records of 64 consecutive entries stay in the group's lanes (lane c, word j:
                // entry wb + 16 j + c): a walk mostly steps to a nearby later entry, so few steps
                // load (friendsforever: 5 % of steps miss a 64-entry window, 19 % a 16-entry one,
                // and four documents share each wave's stall)
                if ((idx & ~63u) != wb) {
                    wb = idx & ~63u;
                    const uint2 *k2 = reinterpret_cast<const uint2 *>(coff);
#pragma unroll
                    for (uint32_t j = 0; j < 4; j++) wk[j] = k2[min(wb + WG * j + c, ne - 1)];
                    walk_wait_vm();
                }
                const uint32_t o = idx - wb, j = o / WG;   // group-uniform: each lane picks the word
                const uint2 v = j == 0 ? wk[0] : j == 1 ? wk[1] : j == 2 ? wk[2] : wk[3];
                const uint32_t src = base + (o & (WG - 1));
                const uint32_t w0 = wsh(v.x, src), w1 = wsh(v.y, src);
                nch = w0 & 0xFFFFu; ch0 = w0 >> 16; firstch = w1 & 0xFFFFu; lastch = w1 >> 16;
            } else {
                const uint32_t wsel = c == 0 ? R_NCH : c == 1 ? R_CH0 : c == 2 ? R_FIRSTCH : R_LASTCH;
                const uint32_t rv = erec[erec_word(ne, idx, wsel)];
                nch = wsh(rv, base); ch0 = wsh(rv, base + 1); firstch = wsh(rv, base + 2); lastch = wsh(rv, base + 3);
            }
            for (uint32_t cc = 0; cc < nch; cc += WG) {
                const bool has = cc + c < nch;
                uint32_t chv = nch <= 2 ? (c == 0 ? firstch : lastch) : 0u;
                if (has && nch > 2) {
                    chv = child[ch0 + cc + c];
                    walk_wait_vm();
                }
                bool ready = false;
                if (has) {
                    const uint8_t pdv = uint8_t(pend[chv] - 1);
                    pend[chv] = pdv;
                    ready = (pdv & 0x7F) == 0;
                }
                const uint32_t m = uint32_t(__ballot(ready) >> base) & 0xFFFFu;
                if (top + uint32_t(__popc(m)) > cap) { err = PLAN_TODO_FULL; break; }
                if (ready) todo[top + uint32_t(__popc(m & below))] = uint16_t(chv);
                top += uint32_t(__popc(m));
                hw = max(hw, top);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            act = !err && top > 0;
        }
    }
    if (on && (ns & (WG - 1)) && c < (ns & (WG - 1))) order[(ns & ~(WG - 1)) + c] = ordv;
    if (on && c == 0) {
        Q.walk[2 * size_t(d)] = err | (hw << 16);   // status | stack high-water mark << 16
        Q.walk[2 * size_t(d) + 1] = ns;
    }
}

}  // namespace pdev

int launch_walk(const PlanParams &q, void *stream, bool csr) {
    if (!q.n_docs || !q.split || !q.walk) return OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const size_t cap = q.todo_cap ? q.todo_cap : PLAN_TODO_CAP;
    if (cap > PLAN_TODO_CAP || (cap & 1u)) return ErrArg;
    const size_t wlds = size_t(pdev::WALK_DOCS) * 2 * (cap + (q.lds_entries + 1) / 2);
    const dim3 grid((q.n_docs + pdev::WALK_DOCS - 1) / pdev::WALK_DOCS);
    if (wlds > 160 * 1024) return ErrArg;
    if (wlds > 64 * 1024) {   // past the default dynamic-LDS limit (documents near PLAN_MAX_LDS_ENTRIES)
        const void *fn = csr ? reinterpret_cast<const void *>(&pdev::walk_kernel<true>) : reinterpret_cast<const void *>(&pdev::walk_kernel<false>);
        if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(160 * 1024)) != hipSuccess) return ErrHip;
    }
    if (csr) hipLaunchKernelGGL(pdev::walk_kernel<true>, grid, dim3(64), wlds, s, q);
    else hipLaunchKernelGGL(pdev::walk_kernel<false>, grid, dim3(64), wlds, s, q);
    return launch_error() == hipSuccess ? OK : ErrHip;
}

int launch_plan(const PlanParams &q, void *stream, bool walk) {
    if (!q.n_docs) return OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const size_t lds = 2 * size_t(PLAN_TODO_CAP) + ((size_t(q.lds_entries) + 15) & ~size_t(15));   // todo + pending
    if (walk && q.split && q.walk && launch_walk(q, stream, false)) return ErrHip;
    if (q.split) hipLaunchKernelGGL(pdev::plan_kernel_1<true>, dim3(q.n_docs), dim3(64), lds, s, q);
    else hipLaunchKernelGGL(pdev::plan_kernel_1<false>, dim3(q.n_docs), dim3(64), lds, s, q);
    if (launch_error() != hipSuccess) return ErrHip;
    if (q.max_agents > 64) {
        hipLaunchKernelGGL(pdev::plan_kernel_wide, dim3(q.n_docs), dim3(64), lds, s, q);
        if (launch_error() != hipSuccess) return ErrHip;
    }
    return OK;
}

}  // namespace dtgpu
