// dt_graph.hip -- batched causal-graph queries on MI355X.
//
// One 64-lane wavefront answers one query against one graph held in HBM (entries as
// (start, end, shadow, parents offset) quads plus a parents array, the layout of
// graph/mod.rs:25-53).  The three queries walk the graph from the newest versions down with a
// max-priority queue, as the reference does, because the conflict-span fixtures pin the walk
// order (spans come out newest-first, merged when contiguous):
//   DIFF      Graph::diff_rev / diff_slow_internal        src/causalgraph/graph/tools.rs:176-292
//   CONFLICT  Graph::find_conflicting(_slow)              tools.rs:296-484 (TimePoint heap)
//   CONTAINS  Graph::frontier_contains_version            tools.rs:88-146 (shadow shortcut)
//   DOMINATORS Graph::find_dominators_2                   tools.rs:545-647 (tagged-LV heap)
// The queues live in LDS (per wave); the walk is wave-uniform scalar code and the batch gives
// the parallelism: every query of the batch runs concurrently, one per wavefront.  A query whose
// queue outgrows LDS, or whose time points carry more than GQ_LDS_MERGED merged versions,
// reports GQ_QUEUE_FULL and is answered again by a second launch (BIG) with its queues in HBM
// scratch sized from its graph: frontiers and queues have no capacity limit, as in the reference
// (BinaryHeap / SmallVec).  (The
// checkout path itself diffs versions with per-chain version vectors in dt_plan.hip; these
// kernels serve merge(from != ROOT) callers and the graph fixtures.)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dt_graph.hpp"
#include "dt_device.hpp"

namespace dtgpu {
namespace gdev {

constexpr int KEY_CAP = 256;     // diff / contains queue in LDS (entries)
constexpr int TP_CAP = 64;       // find_conflicting queue in LDS (time points)
constexpr int TP_WORDS = 4 + GQ_LDS_MERGED;
enum : uint32_t { F_A = 0, F_B = 1, F_S = 2 };

struct Ent { int32_t start, end, shadow; uint32_t poff; };

struct G {
    const Ent *e;          // n + 1 quads (the last one carries the parents end offset)
    const uint32_t *par;
    uint32_t n;
    __device__ __forceinline__ uint32_t find(int32_t lv) const {   // entry holding lv, or n
        uint32_t lo = 0, hi = n;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (lv >= e[mid].end) lo = mid + 1; else hi = mid;
        }
        return lo < n && lv >= e[lo].start ? lo : n;
    }
};

// ---- max-heap of (lv << 2 | flag) keys in LDS (BinaryHeap<(LV, DiffFlag)>) ------------------
struct KHeap {
    uint32_t *v;
    uint32_t n, cap;
    __device__ __forceinline__ bool push(uint32_t k) {
        if (n >= cap) return false;
        uint32_t i = n++;
        while (i > 0) {
            const uint32_t p = (i - 1) >> 1;
            const uint32_t vp = v[p];
            if (vp >= k) break;
            v[i] = vp;
            i = p;
        }
        v[i] = k;
        return true;
    }
    __device__ __forceinline__ uint32_t top() const { return v[0]; }
    __device__ __forceinline__ uint32_t pop() {
        const uint32_t t = v[0];
        const uint32_t x = v[--n];
        uint32_t i = 0;
        for (;;) {
            const uint32_t l = 2 * i + 1, r = l + 1;
            uint32_t m = i, vm = x;
            if (l < n && v[l] > vm) { m = l; vm = v[l]; }
            if (r < n && v[r] > vm) { m = r; vm = v[r]; }
            if (m == i) break;
            v[i] = vm;
            i = m;
        }
        if (n) v[i] = x;
        return t;
    }
};
__device__ __forceinline__ int32_t k_lv(uint32_t k) { return int32_t(k >> 2); }
__device__ __forceinline__ uint32_t k_fl(uint32_t k) { return k & 3u; }
__device__ __forceinline__ uint32_t mkkey(int32_t lv, uint32_t f) { return (uint32_t(lv) << 2) | f; }

// Span lists written newest-first, merging a span that ends where the previous one starts
// (push_reversed_rle / the harness's push_rev_rle).
struct Spans {
    uint32_t *out;
    uint32_t cap, n, words;   // words per span: 2 (diff) or 3 (with flag)
    int32_t ls, le;
    uint32_t lf;
    bool have, overflow;
    __device__ __forceinline__ void init(uint32_t *o, uint32_t c, uint32_t w) {
        out = o; cap = c; n = 0; words = w; have = false; overflow = false; ls = le = 0; lf = 0;
    }
    __device__ __forceinline__ void flush() {
        if (!have) return;
        if (n >= cap) { overflow = true; have = false; return; }
        if (__lane_id() == 0) {
            out[words * n] = uint32_t(ls);
            out[words * n + 1] = uint32_t(le);
            if (words == 3) out[words * n + 2] = lf;
        }
        n++;
        have = false;
    }
    __device__ __forceinline__ void push(int32_t s, int32_t e, uint32_t f) {
        if (have && lf == f && ls == e) { ls = s; return; }
        flush();
        have = true; ls = s; le = e; lf = f;
    }
};

// The common frontier / dominators of a query, written to its slot of the common arena.
struct Common {
    int32_t *out;
    uint32_t cap, n;
    bool overflow;
    __device__ __forceinline__ void push(int32_t v) {
        if (n >= cap) { overflow = true; return; }
        if (__lane_id() == 0) out[n] = v;
        n++;
    }
};

// ---- diff_rev (tools.rs:176-292) --------------------------------------------------------------
__device__ __forceinline__ uint32_t q_diff(const G &g, const GraphQuery &q, const int32_t *a, const int32_t *b, KHeap h,
                                           Spans &sa, Spans &sb) {
    bool same = q.na == q.nb;
    for (uint32_t i = 0; same && i < q.na; i++) same = a[i] == b[i];
    if (same) return GQ_OK;
    if (q.na == 1 && q.nb == 1) {   // is_direct_descendant_coarse
        const int32_t x = a[0], y = b[0];
        const uint32_t ex = g.find(x), ey = g.find(y);
        if (ex == g.n || ey == g.n) return GQ_BAD_INPUT;
        if (x > y && y >= g.e[ex].start) { sa.push(y + 1, x + 1, 0); return GQ_OK; }
        if (y > x && x >= g.e[ey].start) { sb.push(x + 1, y + 1, 0); return GQ_OK; }
    }
    for (uint32_t i = 0; i < q.na; i++) if (!h.push(mkkey(a[i], F_A))) return GQ_QUEUE_FULL;
    for (uint32_t i = 0; i < q.nb; i++) if (!h.push(mkkey(b[i], F_B))) return GQ_QUEUE_FULL;
    int32_t shared = 0;
    while (h.n) {
        const uint32_t it = h.pop();
        int32_t ord = k_lv(it);
        uint32_t flag = k_fl(it);
        if (flag == F_S) shared--;
        while (h.n && k_lv(h.top()) == ord) {
            const uint32_t pk = h.top();
            if (k_fl(pk) != flag) flag = F_S;
            if (k_fl(pk) == F_S) shared--;
            h.pop();
        }
        const uint32_t ei = g.find(ord);
        if (ei == g.n) return GQ_BAD_INPUT;
        const Ent e = g.e[ei];
        while (h.n && k_lv(h.top()) >= e.start) {
            const uint32_t pk = h.top();
            if (k_fl(pk) != flag) {
                if (flag == F_A) sa.push(k_lv(pk) + 1, ord + 1, 0);
                else if (flag == F_B) sb.push(k_lv(pk) + 1, ord + 1, 0);
                ord = k_lv(pk);
                flag = F_S;
            }
            if (k_fl(pk) == F_S) shared--;
            h.pop();
        }
        if (flag == F_A) sa.push(e.start, ord + 1, 0);
        else if (flag == F_B) sb.push(e.start, ord + 1, 0);
        const uint32_t p1 = g.e[ei + 1].poff;
        for (uint32_t k = e.poff; k < p1; k++) {
            if (!h.push(mkkey(int32_t(g.par[k]), flag))) return GQ_QUEUE_FULL;
            if (flag == F_S) shared++;
        }
        if (int32_t(h.n) == shared) break;
    }
    return GQ_OK;
}

// ---- frontier_contains_version (tools.rs:88-146) ----------------------------------------------
__device__ __forceinline__ uint32_t contains_version(const G &g, const int32_t *a, uint32_t na, int32_t t, KHeap h,
                                                     uint32_t &found) {
    found = 0;
    if (t < 0) { found = 1; return GQ_OK; }   // ROOT is in every version
    for (uint32_t i = 0; i < na; i++) if (a[i] == t) { found = 1; return GQ_OK; }
    if (!na) return GQ_OK;
    for (uint32_t i = 0; i < na; i++) {
        if (a[i] > t) {
            const uint32_t ei = g.find(a[i]);
            if (ei == g.n) return GQ_BAD_INPUT;
            if (t >= g.e[ei].shadow) { found = 1; return GQ_OK; }
        }
    }
    for (uint32_t i = 0; i < na; i++) if (a[i] > t && !h.push(mkkey(a[i], 0))) return GQ_QUEUE_FULL;
    while (h.n) {
        const int32_t ord = k_lv(h.pop());
        const uint32_t ei = g.find(ord);
        if (ei == g.n) return GQ_BAD_INPUT;
        const Ent e = g.e[ei];
        if (t >= e.shadow) { found = 1; return GQ_OK; }
        while (h.n && k_lv(h.top()) >= e.start) h.pop();
        const uint32_t p1 = g.e[ei + 1].poff;
        for (uint32_t k = e.poff; k < p1; k++) {
            const int32_t p = int32_t(g.par[k]);
            if (p == t) { found = 1; return GQ_OK; }
            if (p > t && !h.push(mkkey(p, 0))) return GQ_QUEUE_FULL;
        }
    }
    return GQ_OK;
}
__device__ __forceinline__ uint32_t q_contains(const G &g, const GraphQuery &q, const int32_t *a, KHeap h, uint32_t &found) {
    return contains_version(g, a, q.na, q.target, h, found);
}

// ---- find_dominators_2 (tools.rs:545-578) over find_dominators_full_internal (:588-647) ----------
// The union's members in no other member's history, ascending.  a and b are sorted frontiers
// (dominator sets, as the reference assumes).  The heap holds LV << 1, low bit 0 for an input
// and 1 for a parent reached by the walk, so a walked LV pops before an input equal to it; the
// walk stops once every input has popped or an entry's shadow covers the smallest input.
__device__ __forceinline__ uint32_t q_dominators(const G &g, const GraphQuery &q, const int32_t *a, const int32_t *b, KHeap h,
                                                 Common &out) {
    if (!q.na || !q.nb) {
        const int32_t *s = q.na ? a : b;
        const uint32_t n = q.na ? q.na : q.nb;
        for (uint32_t i = 0; i < n; i++) out.push(s[i]);
        return GQ_OK;
    }
    for (uint32_t i = 0; i < q.na; i++) if (g.find(a[i]) == g.n) return GQ_BAD_INPUT;
    for (uint32_t i = 0; i < q.nb; i++) if (g.find(b[i]) == g.n) return GQ_BAD_INPUT;
    if (q.na == 1 && q.nb == 1) {   // version_cmp (tools.rs:67-85)
        const int32_t x = a[0], y = b[0];
        if (x == y) { out.push(y); return GQ_OK; }
        const int32_t hi = x > y ? x : y, lo = x > y ? y : x;
        uint32_t f = 0;
        const uint32_t st = contains_version(g, &hi, 1, lo, h, f);
        if (st != GQ_OK) return st;
        if (!f) out.push(lo);
        out.push(hi);
        return GQ_OK;
    }
    const int32_t first_v = a[0] < b[0] ? a[0] : b[0];
    for (uint32_t i = 0; i < q.na; i++) if (!h.push(uint32_t(a[i]) << 1)) return GQ_QUEUE_FULL;
    for (uint32_t i = 0; i < q.nb; i++) if (!h.push(uint32_t(b[i]) << 1)) return GQ_QUEUE_FULL;
    uint32_t remaining = q.na + q.nb;
    int32_t last = -1;
    while (h.n) {
        const uint32_t ve = h.pop();
        const int32_t v = int32_t(ve >> 1);
        if (!(ve & 1u)) {   // an input: a dominator (nothing walked covers it); descending
            out.push(v);
            last = v;
            remaining--;
        }
        const uint32_t ei = g.find(v);
        if (ei == g.n) return GQ_BAD_INPUT;
        const Ent e = g.e[ei];
        if (e.shadow <= first_v) break;   // every input left lies in this entry's shadow
        while (h.n && int32_t(h.top() >> 1) >= e.start) {   // inside this entry: covered
            const uint32_t ve2 = h.pop();
            if (!(ve2 & 1u)) {
                if (last != int32_t(ve2 >> 1)) last = int32_t(ve2 >> 1);   // dominated (visit(v, false))
                remaining--;
            }
        }
        if (!remaining) break;
        const uint32_t p1 = g.e[ei + 1].poff;
        for (uint32_t k = e.poff; k < p1; k++)
            if (!h.push((g.par[k] << 1) | 1u)) return GQ_QUEUE_FULL;
    }
    if (out.overflow) return GQ_OVERFLOW;
    // ascending: reverse the slot in place (lane 0 wrote it)
    if (__lane_id() == 0) {
        for (uint32_t i = 0, n = out.n; i < n / 2; i++) {
            const int32_t x = out.out[i], y = out.out[n - 1 - i];
            out.out[i] = y;
            out.out[n - 1 - i] = x;
        }
    }
    return GQ_OK;
}

// ---- find_conflicting (tools.rs:296-484) ------------------------------------------------------
// TimePoint = (last, merged_with), compared by last + 1 (ROOT first), then fewer merged_with is
// greater, then the flag (the Ord of (TimePoint, DiffFlag)).  Layout per time point, w words:
// [last, nm, flag, pad, merged_with...]; w = TP_WORDS in LDS, 4 + the widest version in HBM.
struct TPHeap {
    uint32_t *v;
    uint32_t n, cap, w;
    __device__ __forceinline__ uint32_t *at(uint32_t i) const { return v + size_t(i) * w; }
    __device__ __forceinline__ static int cmp(const uint32_t *x, const uint32_t *y) {
        const uint32_t lx = x[0] + 1u, ly = y[0] + 1u;   // ROOT (-1) -> 0
        if (lx != ly) return lx < ly ? -1 : 1;
        if (x[1] != y[1]) return x[1] > y[1] ? -1 : 1;
        if (x[2] != y[2]) return x[2] < y[2] ? -1 : 1;
        return 0;
    }
    __device__ __forceinline__ static void copy(uint32_t *d, const uint32_t *s) {
        const uint32_t k = 4 + s[1];   // only the words in use
        for (uint32_t q = 0; q < k; q++) d[q] = s[q];
    }
    __device__ __forceinline__ void swap(uint32_t *x, uint32_t *y) const {
        const uint32_t k = 4 + (x[1] > y[1] ? x[1] : y[1]);
        for (uint32_t q = 0; q < k; q++) { const uint32_t t = x[q]; x[q] = y[q]; y[q] = t; }
    }
    __device__ __forceinline__ bool push(const uint32_t *tp) {
        if (n >= cap || 4 + tp[1] > w) return false;
        uint32_t i = n++;
        copy(at(i), tp);
        while (i > 0) {
            const uint32_t p = (i - 1) >> 1;
            if (cmp(at(i), at(p)) <= 0) break;
            swap(at(i), at(p));
            i = p;
        }
        return true;
    }
    __device__ __forceinline__ void pop(uint32_t *out) {
        copy(out, at(0));
        n--;
        if (n) copy(at(0), at(n));
        uint32_t i = 0;
        for (;;) {
            const uint32_t l = 2 * i + 1, r = l + 1;
            uint32_t m = i;
            if (l < n && cmp(at(l), at(m)) > 0) m = l;
            if (r < n && cmp(at(r), at(m)) > 0) m = r;
            if (m == i) break;
            swap(at(i), at(m));
            i = m;
        }
    }
    __device__ __forceinline__ static bool eq_time(const uint32_t *x, const uint32_t *y) {
        if (x[0] != y[0] || x[1] != y[1]) return false;
        for (uint32_t k = 0; k < x[1]; k++) if (x[4 + k] != y[4 + k]) return false;
        return true;
    }
};
// TimePoint from a sorted frontier (last = newest, merged_with = the rest)
__device__ __forceinline__ void tp_make(uint32_t *t, const int32_t *f, uint32_t n, uint32_t flag) {
    t[0] = n ? uint32_t(f[n - 1]) : 0xFFFFFFFFu;
    t[1] = n > 1 ? n - 1 : 0;
    t[2] = flag;
    t[3] = 0;
    for (uint32_t k = 0; k + 1 < n; k++) t[4 + k] = uint32_t(f[k]);
}
__device__ __forceinline__ void tp_one(uint32_t *t, uint32_t lv, uint32_t flag) {
    t[0] = lv; t[1] = 0; t[2] = flag; t[3] = 0;
}

// scratch: three time points of h.w words (the popped point, a temporary, a consumed point)
__device__ __forceinline__ uint32_t q_conflict(const G &g, const GraphQuery &q, const int32_t *a, const int32_t *b,
                                               TPHeap h, uint32_t *scratch, Spans &sp, Common &common) {
    bool same = q.na == q.nb;
    for (uint32_t i = 0; same && i < q.na; i++) same = a[i] == b[i];
    if (same) {
        for (uint32_t i = 0; i < q.na; i++) common.push(a[i]);
        return GQ_OK;
    }
    if (q.na == 1 && q.nb == 1) {
        const int32_t x = a[0], y = b[0];
        const uint32_t ex = g.find(x), ey = g.find(y);
        if (ex == g.n || ey == g.n) return GQ_BAD_INPUT;
        if (x > y && y >= g.e[ex].start) { sp.push(y + 1, x + 1, F_A); common.push(y); return GQ_OK; }
        if (y > x && x >= g.e[ey].start) { sp.push(x + 1, y + 1, F_B); common.push(x); return GQ_OK; }
    }
    if (q.na > h.w - 3 || q.nb > h.w - 3) return GQ_QUEUE_FULL;   // a version wider than a time point
    uint32_t *tm = scratch, *tmp = scratch + h.w, *pk = scratch + 2 * h.w;
    tp_make(tmp, a, q.na, F_A);
    if (!h.push(tmp)) return GQ_QUEUE_FULL;
    tp_make(tmp, b, q.nb, F_B);
    if (!h.push(tmp)) return GQ_QUEUE_FULL;
    for (;;) {
        h.pop(tm);
        uint32_t flag = tm[2];
        const int32_t t = int32_t(tm[0]);
        if (t < 0) return GQ_OK;   // ROOT: nothing in common
        while (h.n && TPHeap::eq_time(h.at(0), tm)) {
            if (h.at(0)[2] != flag) flag = F_S;
            h.pop(tmp);
        }
        if (!h.n) {
            for (uint32_t k = 0; k < tm[1]; k++) common.push(int32_t(tm[4 + k]));
            common.push(t);
            return GQ_OK;
        }
        for (uint32_t k = 0; k < tm[1]; k++) {   // shatter a merge point
            tp_one(tmp, tm[4 + k], flag);
            if (!h.push(tmp)) return GQ_QUEUE_FULL;
        }
        const uint32_t ei = g.find(t);
        if (ei == g.n) return GQ_BAD_INPUT;
        const Ent e = g.e[ei];
        int32_t rs = e.start, re = t + 1;
        for (;;) {
            if (!h.n) {
                common.push(re - 1);
                return GQ_OK;
            }
            const int32_t pl = int32_t(h.at(0)[0]);
            if (pl >= 0 && pl >= e.start) {   // the next point lies inside this entry: consume it
                h.pop(pk);
                const uint32_t next_flag = pk[2];
                if (int32_t(pk[0]) + 1 < re) {
                    const int32_t cut = rs + (int32_t(pk[0]) + 1 - e.start);   // range.truncate
                    sp.push(cut, re, flag);
                    re = cut;
                }
                for (uint32_t k = 0; k < pk[1]; k++) {
                    tp_one(tmp, pk[4 + k], next_flag);
                    if (!h.push(tmp)) return GQ_QUEUE_FULL;
                }
                if (next_flag != flag) flag = F_S;
            } else {   // emit the rest of the entry and continue from its parents
                sp.push(rs, re, flag);
                const uint32_t p0 = e.poff, p1 = g.e[ei + 1].poff;
                const uint32_t np = p1 - p0;
                if (np + 3 > h.w) return GQ_QUEUE_FULL;   // wider than a time point here
                tmp[0] = np ? g.par[p1 - 1] : 0xFFFFFFFFu;
                tmp[1] = np > 1 ? np - 1 : 0;
                tmp[2] = flag;
                tmp[3] = 0;
                for (uint32_t k = 0; k + 1 < np; k++) tmp[4 + k] = g.par[p0 + k];
                if (!h.push(tmp)) return GQ_QUEUE_FULL;
                break;
            }
        }
    }
}

// BIG = false: queues in LDS; BIG = true: the second pass, only over the queries the first one
// reported GQ_QUEUE_FULL for, queues in HBM scratch (hscr + h_off: key heap, time-point heap,
// three scratch time points).
template <bool BIG>
__global__ __launch_bounds__(64) void graph_query_kernel(GraphParams P) {
    __shared__ uint32_t heap[BIG ? 1 : KEY_CAP];
    __shared__ uint32_t tpv[BIG ? 1 : TP_CAP * TP_WORDS];
    __shared__ uint32_t scratch[BIG ? 1 : 3 * TP_WORDS];
    const uint32_t qi = blockIdx.x;
    if (qi >= P.n_queries) return;
    const GraphQuery q = P.queries[qi];
    if (q.kind == GQ_DIFF_LEVEL || q.kind == GQ_CONFLICT_LEVEL) return;   // dt_level.hip answers these
    if (BIG && P.results[qi].status != GQ_QUEUE_FULL) return;
    G g{reinterpret_cast<const Ent *>(P.ents) + q.ent_off, P.par, q.n_ent};
    GraphResult r{};
    uint32_t *out = P.out + size_t(q.out_off);
    const int32_t *a = P.front + q.f_off, *b = a + q.na;
    Common common{P.common + q.c_off, q.c_cap, 0, false};
    uint32_t *hk = BIG ? P.hscr + q.h_off : heap;
    const uint32_t tw = BIG ? gq_tp_words(q.max_par, q.na, q.nb) : uint32_t(TP_WORDS);
    uint32_t *ht = BIG ? hk + q.hk_cap : tpv;
    uint32_t *hs = BIG ? ht + size_t(q.htp_cap) * tw : scratch;
    KHeap kh{hk, 0, BIG ? q.hk_cap : uint32_t(KEY_CAP)};
    TPHeap th{ht, 0, BIG ? q.htp_cap : uint32_t(TP_CAP), tw};
    uint32_t st = GQ_OK;
    if (q.kind == GQ_DIFF) {
        Spans sa, sb;
        sa.init(out, q.out_cap / 4, 2);
        sb.init(out + 2 * (q.out_cap / 4), q.out_cap / 4, 2);
        st = q_diff(g, q, a, b, kh, sa, sb);
        sa.flush();
        sb.flush();
        if (st == GQ_OK && (sa.overflow || sb.overflow)) st = GQ_OVERFLOW;
        r.n0 = sa.n;
        r.n1 = sb.n;
    } else if (q.kind == GQ_CONFLICT) {
        Spans sp;
        sp.init(out, q.out_cap / 3, 3);
        st = q_conflict(g, q, a, b, th, hs, sp, common);
        sp.flush();
        if (st == GQ_OK && (sp.overflow || common.overflow)) st = GQ_OVERFLOW;
        r.n0 = sp.n;
        r.n_common = common.n;
    } else if (q.kind == GQ_CONTAINS) {
        uint32_t f = 0;
        st = q_contains(g, q, a, kh, f);
        r.n0 = f;
    } else if (q.kind == GQ_DOMINATORS) {
        st = q_dominators(g, q, a, b, kh, common);
        r.n_common = common.n;
    } else {
        st = GQ_BAD_INPUT;
    }
    if (BIG && st == GQ_QUEUE_FULL) st = GQ_OVERFLOW;   // cannot happen: the scratch is sized from the graph
    r.status = st;
    if (__lane_id() == 0) P.results[qi] = r;
}

}  // namespace gdev

int launch_graph_queries(const GraphParams &p, void *stream, bool big) {
    if (!p.n_queries) return 0;
    if (big) hipLaunchKernelGGL(gdev::graph_query_kernel<true>, dim3(p.n_queries), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), p);
    else hipLaunchKernelGGL(gdev::graph_query_kernel<false>, dim3(p.n_queries), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), p);
    return launch_error() == hipSuccess ? 0 : 66;
}

}  // namespace dtgpu
