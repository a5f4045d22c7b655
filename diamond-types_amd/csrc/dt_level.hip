// dt_level.hip -- level-synchronous causal-graph kernels (north_star "Causal graph": conflict-span
// detection, diff and topological levelling as level-synchronous propagation over CSR parent
// arrays in HBM).  Every per-entry array can live in HBM, so graphs of any size are levelled
// (the query kernels' marks sit in LDS for graphs up to kLevelLdsEntries entries).
//
// level_kernel (one 256-thread workgroup per graph) levels the graph's entries: level(e) =
// 1 + max level of its parent entries (roots 0), so every child sits on a higher level than
// its parents.  Built in place from the entry quads and parent LVs of dt_graph.hip's arena:
//   1. parent slot -> parent entry (one binary search per slot, all slots in parallel) and a
//      children CSR (counting sort of the slots by parent entry, atomics on the graph's
//      counter words);
//   2. Kahn's algorithm one level per round: the round's frontier releases the children whose
//      last pending parent it held; the rounds' frontiers, concatenated, are the entries in
//      level order (order[], level offsets lvl_off[]).
// Marks (both query kernels): mA[e] / mB[e] = the highest LV of entry e in the history of a / b
// (a history holds a prefix of every entry it touches).  Seeded with the two versions, they are
// pushed level by level from the highest level down: a level's entries push their marks to
// their parents' entries with atomicMax, all in parallel, and a barrier separates the levels.
//
// level_diff_kernel answers Graph::diff (tools.rs:158-292) from the marks: only-a of entry e is
// (mB[e], mA[e]], the spans newest first, merged when contiguous -- the same lists as the heap
// walk (dt_graph.hip q_diff).
//
// level_conflict_kernel answers Graph::find_conflicting (tools.rs:296-484).  The marks decide
// each span's flag: an LV x of entry e is in the history of a iff x <= mA[e] (of b iff x <=
// mB[e]), so a span is OnlyA, OnlyB or Shared by membership.  What the marks do not give is
// where the reference's walk cuts its spans and where it stops (the single common point): the
// walk pops time points (a version, or an entry's parents) highest first, consumes every point
// inside the entry it enters (a span boundary at each), then pushes the entry's parents, and
// stops when one point is left.  Because a point is always pushed below the entry that creates
// it, the walk is a sweep over the entries in descending order with each entry's pending points
// in a bucket: no heap.  The workgroup lists the entries the marks touch, highest first (a
// prefix-sum compaction), and one thread runs the sweep over that list, sorting each entry's
// points in an LDS buffer; the list, the bucket heads and the point pool are HBM scratch of the
// query.  The marks of both query kernels sit in LDS for graphs up to kLevelLdsEntries entries
// (their per-level atomicMax traffic), in HBM scratch beyond.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dt_graph.hpp"

namespace dtgpu {
namespace ldev {

struct Ent { int32_t start, end, shadow; uint32_t poff; };

__device__ __forceinline__ uint32_t find(const Ent *e, uint32_t n, int32_t lv) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (lv >= e[mid].end) lo = mid + 1; else hi = mid;
    }
    return lo < n && lv >= e[lo].start ? lo : n;
}

constexpr uint32_t NT = 256;

__global__ __launch_bounds__(256) void level_kernel(LevelParams P) {
    __shared__ uint32_t s_sum[NT];
    __shared__ uint32_t s_tail, s_bad;
    const uint32_t g = blockIdx.x, t = threadIdx.x;
    if (g >= P.n_graphs) return;
    const LevelGraph G = P.graphs[g];
    const uint32_t n = G.n_ent, base = G.ent_off;
    uint32_t *meta = P.meta + 2 * size_t(base);   // [0] = levels, [1] = status
    uint32_t *cur = P.gscr + 3 * size_t(base);    // child counts, then fill cursors (n + 1)
    uint32_t *cofs = cur + (n + 1);               // children CSR offsets (n + 1)
    uint32_t *pend = cofs + (n + 1);              // parents not yet levelled (n)
    const Ent *E = reinterpret_cast<const Ent *>(P.ents) + base;
    const uint32_t plo = E[0].poff, phi = E[n].poff;
    if (t == 0) { s_bad = 0; s_tail = 0; }
    for (uint32_t e = t; e < n; e += NT) {
        cur[e] = 0;
        pend[e] = E[e + 1].poff - E[e].poff;
    }
    __syncthreads();
    for (uint32_t k = plo + t; k < phi; k += NT) {
        const uint32_t pe = find(E, n, int32_t(P.par[k]));
        if (pe == n) { s_bad = 1; continue; }
        P.pent[k] = pe;
        atomicAdd(&cur[pe], 1u);
    }
    __syncthreads();
    if (s_bad) {
        if (t == 0) { meta[0] = 0; meta[1] = GQ_BAD_INPUT; }
        return;
    }
    // exclusive scan of the child counts: per-thread chunks, then the 256 chunk totals
    const uint32_t per = (n + NT - 1) / NT, c0 = min(n, t * per), c1 = min(n, c0 + per);
    uint32_t sum = 0;
    for (uint32_t e = c0; e < c1; e++) sum += cur[e];
    s_sum[t] = sum;
    __syncthreads();
    if (t == 0) {
        uint32_t run = 0;
        for (uint32_t i = 0; i < NT; i++) { const uint32_t x = s_sum[i]; s_sum[i] = run; run += x; }
        cofs[n] = run;
    }
    __syncthreads();
    {
        uint32_t run = s_sum[t];
        for (uint32_t e = c0; e < c1; e++) {
            const uint32_t c = cur[e];
            cofs[e] = run;
            cur[e] = run;
            run += c;
        }
    }
    __syncthreads();
    for (uint32_t e = t; e < n; e += NT)
        for (uint32_t k = E[e].poff; k < E[e + 1].poff; k++) P.child[plo + atomicAdd(&cur[P.pent[k]], 1u)] = e;
    for (uint32_t e = t; e < n; e += NT)
        if (pend[e] == 0) P.order[base + atomicAdd(&s_tail, 1u)] = e;   // roots: level 0
    __syncthreads();
    // one level per round; a round's frontier is order[head, tail)
    uint32_t head = 0, tail = s_tail, L = 0;
    while (head < tail) {
        if (t == 0) P.lvl_off[base + L] = head;
        for (uint32_t i = head + t; i < tail; i += NT) {
            const uint32_t e = P.order[base + i];
            P.level[base + e] = L;
            for (uint32_t j = cofs[e]; j < cofs[e + 1]; j++) {
                const uint32_t c = P.child[plo + j];
                if (atomicSub(&pend[c], 1u) == 1u) P.order[base + atomicAdd(&s_tail, 1u)] = c;
            }
        }
        __syncthreads();
        head = tail;
        tail = s_tail;
        L++;
        __syncthreads();   // every thread has read s_tail before the next round adds to it
    }
    if (t == 0) {
        P.lvl_off[base + L] = head;
        meta[0] = L;
        meta[1] = head == n ? GQ_OK : GQ_BAD_INPUT;   // a cycle leaves entries unlevelled
    }
}

// The marks of a query (see the header), level by level.  Every thread returns the same status.
__device__ uint32_t push_marks(const LevelParams &P, const GraphQuery &q, const int32_t *qa, const Ent *E, int32_t *mA,
                               int32_t *mB, uint32_t *s_top, uint32_t *s_st) {
    const uint32_t t = threadIdx.x, n = q.n_ent, base = q.ent_off;
    for (uint32_t e = t; e < n; e += NT) { mA[e] = -1; mB[e] = -1; }
    __syncthreads();
    if (t == 0) {   // seed the marks with the two versions
        uint32_t top = 0, st = GQ_OK;
        for (uint32_t i = 0; i < q.na + q.nb && st == GQ_OK; i++) {
            const int32_t v = qa[i];   // a then b: one run in the frontier arena
            const uint32_t e = find(E, n, v);
            if (e == n) { st = GQ_BAD_INPUT; break; }
            int32_t *m = i < q.na ? mA : mB;
            m[e] = max(m[e], v);
            top = max(top, P.level[base + e]);
        }
        *s_top = top;
        *s_st = st;
    }
    __syncthreads();
    if (*s_st != GQ_OK) return *s_st;
    // highest level first: a level's marks are final once every higher level has pushed
    for (int32_t L = int32_t(*s_top); L >= 0; L--) {
        const uint32_t i0 = P.lvl_off[base + L], i1 = P.lvl_off[base + L + 1];
        for (uint32_t i = i0 + t; i < i1; i += NT) {
            const uint32_t e = P.order[base + i];
            const int32_t xa = mA[e], xb = mB[e];
            if (xa < 0 && xb < 0) continue;
            for (uint32_t k = E[e].poff; k < E[e + 1].poff; k++) {
                const uint32_t pe = P.pent[k];
                const int32_t p = int32_t(P.par[k]);
                if (xa >= 0) atomicMax(&mA[pe], p);
                if (xb >= 0) atomicMax(&mB[pe], p);
            }
        }
        __syncthreads();
    }
    return GQ_OK;
}

// Spans newest first, contiguous ones merged (push_reversed_rle); 2 words per span (diff) or 3
// (with the flag, conflict), as dt_graph.hip writes them.
struct RevSpans {
    uint32_t *out;
    uint32_t cap, n, words;
    int32_t ls, le;
    uint32_t lf;
    bool have, overflow;
    __device__ void push(int32_t s, int32_t e, uint32_t f = 0) {
        if (have && ls == e && lf == f) { ls = s; return; }
        flush();
        have = true; ls = s; le = e; lf = f;
    }
    __device__ void flush() {
        if (!have) return;
        if (n >= cap) { overflow = true; have = false; return; }
        out[words * n] = uint32_t(ls);
        out[words * n + 1] = uint32_t(le);
        if (words == 3) out[words * n + 2] = lf;
        n++;
        have = false;
    }
};

__global__ __launch_bounds__(256) void level_diff_kernel(LevelParams P, GraphParams Q) {
    __shared__ uint32_t s_top, s_st;
    const uint32_t qi = blockIdx.x, t = threadIdx.x;
    if (qi >= Q.n_queries) return;
    const GraphQuery &q = Q.queries[qi];
    if (q.kind != GQ_DIFF_LEVEL) return;
    const uint32_t n = q.n_ent, base = q.ent_off;
    const uint32_t *meta = P.meta + 2 * size_t(base);
    GraphResult *res = Q.results + qi;
    if (meta[1] != GQ_OK) {
        if (t == 0) { res->status = meta[1]; res->n0 = res->n1 = res->n_common = 0; }
        return;
    }
    const Ent *E = reinterpret_cast<const Ent *>(P.ents) + base;
    extern __shared__ int32_t lmarks[];   // P.lds_ent > 0: the marks live in LDS
    int32_t *mA = P.lds_ent ? lmarks : reinterpret_cast<int32_t *>(P.qscr + q.scr_off), *mB = mA + n;
    const uint32_t st = push_marks(P, q, Q.front + q.f_off, E, mA, mB, &s_top, &s_st);
    if (st != GQ_OK) {
        if (t == 0) { res->status = st; res->n0 = res->n1 = res->n_common = 0; }
        return;
    }
    if (t == 0) {
        uint32_t *out = Q.out + size_t(q.out_off);
        RevSpans sa{out, q.out_cap / 4, 0, 2, 0, 0, 0, false, false};
        RevSpans sb{out + 2 * (q.out_cap / 4), q.out_cap / 4, 0, 2, 0, 0, 0, false, false};
        for (int32_t e = int32_t(n) - 1; e >= 0; e--) {
            const int32_t xa = mA[e], xb = mB[e], s = E[e].start;
            if (xa > xb) sa.push(xb >= s ? xb + 1 : s, xa + 1);
            else if (xb > xa) sb.push(xa >= s ? xa + 1 : s, xb + 1);
        }
        sa.flush();
        sb.flush();
        res->status = (sa.overflow || sb.overflow) ? GQ_OVERFLOW : GQ_OK;
        res->n0 = sa.n;
        res->n1 = sb.n;
        res->n_common = 0;
    }
}

// ---- find_conflicting: marks + a bucketed sweep ------------------------------------------------
enum : uint32_t { F_A = 0, F_B = 1, F_S = 2 };
enum : uint32_t { TP_ONE = 0, TP_PARENTS = 1, TP_QA = 2, TP_QB = 3 };
constexpr int32_t ROOT_LV = -1;
constexpr uint32_t PW = kLevelPointWords;
constexpr uint32_t BUCKET_CAP = 64;   // time points that enter one entry sorted in LDS (more: in HBM)

// A time point (the reference's TimePoint + DiffFlag) in the query's pool: PW words
// {next in its bucket, flag | kind << 2, frontier size, reference, last element}: a single LV
// (TP_ONE: ref = the LV), an entry's parents (TP_PARENTS: ref = the entry), or one of the two
// versions.
struct Sweep {
    const Ent *E;
    const uint32_t *par, *pent;   // parent LVs and their entries (per parent slot)
    const int32_t *qa, *qb;   // the two versions (frontier arena)
    int32_t *head;
    uint32_t *pool;
    uint32_t n, cap, used, npend;
    bool overflow;

    __device__ int32_t elem(uint32_t tp, uint32_t k) const {
        const uint32_t *w = pool + PW * size_t(tp);
        switch (w[1] >> 2) {
            case TP_ONE: return int32_t(w[3]);
            case TP_PARENTS: return int32_t(par[E[w[3]].poff + k]);
            case TP_QA: return qa[k];
            default: return qb[k];
        }
    }
    __device__ uint32_t size(uint32_t tp) const { return pool[PW * size_t(tp) + 2]; }
    __device__ uint32_t flag(uint32_t tp) const { return pool[PW * size_t(tp) + 1] & 3u; }
    __device__ int32_t last(uint32_t tp) const { return int32_t(pool[PW * size_t(tp) + 4]); }
    __device__ bool same(uint32_t x, uint32_t y) const {   // TimePoint equality: the whole frontier
        const uint32_t s = size(x);
        if (s != size(y)) return false;
        for (uint32_t k = 0; k < s; k++) if (elem(x, k) != elem(y, k)) return false;
        return true;
    }
    // heap order of (TimePoint, DiffFlag) (tools.rs:309-318): higher last first, fewer merged
    // members first, then the higher flag
    __device__ bool before(uint32_t x, uint32_t y) const {
        const int32_t lx = last(x), ly = last(y);
        if (lx != ly) return lx > ly;
        if (size(x) != size(y)) return size(x) < size(y);
        return flag(x) > flag(y);
    }
    // `e`: the entry holding the point's last element when the caller knows it (the levelling's
    // parent-slot entries), n when it must be searched (the versions)
    __device__ void push(uint32_t kind, uint32_t ref, uint32_t sz, uint32_t f, int32_t l, uint32_t e) {
        if (used >= cap) { overflow = true; return; }
        const uint32_t tp = used++;
        uint32_t *w = pool + PW * size_t(tp);
        w[1] = f | (kind << 2);
        w[2] = sz;
        w[3] = ref;
        w[4] = uint32_t(l);
        npend++;
        if (l == ROOT_LV) { w[0] = 0xFFFFFFFFu; return; }   // ROOT: popped only when nothing else is left
        if (e == n) e = find(E, n, l);
        if (e == n) { overflow = true; return; }
        w[0] = uint32_t(head[e]);
        head[e] = int32_t(tp);
    }
    // element k of point tp as a TP_ONE point (a shattered frontier)
    __device__ void push_elem(uint32_t tp, uint32_t k, uint32_t f) {
        const uint32_t *w = pool + PW * size_t(tp);
        const int32_t x = elem(tp, k);
        push(TP_ONE, uint32_t(x), 1, f, x, (w[1] >> 2) == TP_PARENTS ? pent[E[w[3]].poff + k] : n);
    }
};

__global__ __launch_bounds__(256) void level_conflict_kernel(LevelParams P, GraphParams Q) {
    __shared__ uint32_t s_top, s_st, s_ncand;
    __shared__ uint32_t s_sum[NT];
    __shared__ uint32_t bkl[BUCKET_CAP];
    const uint32_t qi = blockIdx.x, t = threadIdx.x;
    if (qi >= Q.n_queries) return;
    const GraphQuery &q = Q.queries[qi];
    if (q.kind != GQ_CONFLICT_LEVEL) return;
    const uint32_t n = q.n_ent, base = q.ent_off;
    const uint32_t *meta = P.meta + 2 * size_t(base);
    GraphResult *res = Q.results + qi;
    const Ent *E = reinterpret_cast<const Ent *>(P.ents) + base;
    uint32_t *out = Q.out + size_t(q.out_off);
    if (meta[1] != GQ_OK) {
        if (t == 0) { res->status = meta[1]; res->n0 = res->n_common = 0; }
        return;
    }
    const int32_t *qa = Q.front + q.f_off, *qb = qa + q.na;
    int32_t *common = Q.common + q.c_off;   // written by thread 0 only
    // the reference's short circuits (tools.rs:445-480), decided by thread 0 for the group
    if (t == 0) {
        uint32_t st = 0xFFFFFFFFu;   // 0xFFFFFFFF: no short circuit
        bool same = q.na == q.nb;
        for (uint32_t i = 0; same && i < q.na; i++) same = qa[i] == qb[i];
        RevSpans sp{out, q.out_cap / 3, 0, 3, 0, 0, 0, false, false};
        uint32_t nc = 0;
        if (same) {
            st = q.na <= q.c_cap ? GQ_OK : GQ_OVERFLOW;
            for (uint32_t i = 0; i < q.na && i < q.c_cap; i++) common[nc++] = qa[i];
        } else if (q.na == 1 && q.nb == 1 && q.c_cap) {
            const int32_t x = qa[0], y = qb[0];
            const uint32_t ex = find(E, n, x), ey = find(E, n, y);
            if (ex == n || ey == n) st = GQ_BAD_INPUT;
            else if (x > y && y >= E[ex].start) { sp.push(y + 1, x + 1, F_A); common[nc++] = y; st = GQ_OK; }
            else if (y > x && x >= E[ey].start) { sp.push(x + 1, y + 1, F_B); common[nc++] = x; st = GQ_OK; }
        }
        if (st != 0xFFFFFFFFu) {
            sp.flush();
            res->status = st;
            res->n0 = sp.n;
            res->n_common = nc;
        }
        s_st = st;
    }
    __syncthreads();
    if (s_st != 0xFFFFFFFFu) return;
    __syncthreads();   // every thread read s_st before push_marks reuses it
    int32_t *hbm = reinterpret_cast<int32_t *>(P.qscr + q.scr_off);
    extern __shared__ int32_t lmarks[];   // P.lds_ent > 0: the marks live in LDS
    int32_t *mA = P.lds_ent ? lmarks : hbm, *mB = mA + n, *head = hbm + 2 * n;
    uint32_t *cand = reinterpret_cast<uint32_t *>(head + n);
    uint32_t *pool = cand + n;
    for (uint32_t e = t; e < n; e += NT) head[e] = -1;
    const uint32_t mst = push_marks(P, q, qa, E, mA, mB, &s_top, &s_st);
    if (mst != GQ_OK) {
        if (t == 0) { res->status = mst; res->n0 = res->n_common = 0; }
        return;
    }
    // the entries the marks touch, highest first (a workgroup prefix sum over per-thread chunks):
    // the only ones the sweep can visit
    {
        const uint32_t per = (n + NT - 1) / NT, c0 = min(n, t * per), c1 = min(n, c0 + per);
        uint32_t cnt = 0;
        for (uint32_t i = c0; i < c1; i++) {
            const uint32_t e = n - 1 - i;
            cnt += (mA[e] >= E[e].start || mB[e] >= E[e].start) ? 1u : 0u;
        }
        s_sum[t] = cnt;
        __syncthreads();
        if (t == 0) {
            uint32_t run = 0;
            for (uint32_t i = 0; i < NT; i++) { const uint32_t x = s_sum[i]; s_sum[i] = run; run += x; }
            s_ncand = run;
        }
        __syncthreads();
        uint32_t at = s_sum[t];
        for (uint32_t i = c0; i < c1; i++) {
            const uint32_t e = n - 1 - i;
            if (mA[e] >= E[e].start || mB[e] >= E[e].start) cand[at++] = e;
        }
        __syncthreads();
    }
    if (t != 0) return;
    // ---- the sweep (one thread) ----
    Sweep S{E, P.par, P.pent, qa, qb, head, pool, n, q.scr_tp, 0, 0, false};
    uint32_t *hbk = pool + PW * size_t(q.scr_tp);   // an entry's bucket past BUCKET_CAP points
    RevSpans sp{out, q.out_cap / 3, 0, 3, 0, 0, 0, false, false};
    // a span's flag is its membership: x in H(a) iff x <= mA[e], in H(b) iff x <= mB[e]
    auto mflag = [&](uint32_t e, int32_t x) -> uint32_t {
        const bool ia = x <= mA[e], ib = x <= mB[e];
        return ia && ib ? F_S : (ia ? F_A : F_B);
    };
    S.push(TP_QA, 0, q.na, F_A, q.na ? qa[q.na - 1] : ROOT_LV, n);
    S.push(TP_QB, 0, q.nb, F_B, q.nb ? qb[q.nb - 1] : ROOT_LV, n);
    uint32_t st = GQ_OK, nc = 0;
    const uint32_t ncand = s_ncand;
    uint32_t ci = 0;
    int32_t e = -1;
    for (;;) {
        // the next entry holding a pending point: only entries the marks touch can
        e = -1;
        while (ci < ncand) {
            const uint32_t x = cand[ci++];
            if (head[x] >= 0) { e = int32_t(x); break; }
        }
        if (S.overflow) { st = GQ_OVERFLOW; break; }
        if (e < 0) break;   // only ROOT points left: nothing in common
        // the bucket in heap order (insertion sort; buckets are small -- in LDS up to BUCKET_CAP
        // points, in the query's HBM scratch beyond)
        uint32_t m = 0;
        for (int32_t x = head[e]; x >= 0; x = int32_t(pool[PW * size_t(x)])) m++;
        uint32_t *bk = m <= BUCKET_CAP ? bkl : hbk;
        m = 0;
        for (int32_t x = head[e]; x >= 0; x = int32_t(pool[PW * size_t(x)])) {
            uint32_t j = m++;
            while (j > 0 && S.before(uint32_t(x), bk[j - 1])) { bk[j] = bk[j - 1]; j--; }
            bk[j] = uint32_t(x);
        }
        head[e] = -1;
        // pop the top point and its duplicates
        const uint32_t T = bk[0];
        uint32_t flag = S.flag(T);
        S.npend--;
        uint32_t i = 1;
        while (i < m && S.same(bk[i], T)) {
            if (S.flag(bk[i]) != flag) flag = F_S;
            S.npend--;
            i++;
        }
        if (S.npend == 0) {   // collapsed to one point: the common version
            const uint32_t sz = S.size(T);
            if (sz > q.c_cap) { st = GQ_OVERFLOW; break; }
            for (uint32_t k = 0; k < sz; k++) common[nc++] = S.elem(T, k);
            break;
        }
        for (uint32_t k = 0; k + 1 < S.size(T); k++) S.push_elem(T, k, flag);   // shatter
        const int32_t es = E[e].start;
        int32_t re = S.last(T) + 1;
        bool stopped = false;
        for (; i < m; i++) {   // the other points inside this entry, highest first
            const uint32_t u = bk[i];
            const int32_t ul = S.last(u);
            S.npend--;
            if (ul + 1 < re) {
                sp.push(ul + 1, re, mflag(uint32_t(e), re - 1));
                re = ul + 1;
            }
            for (uint32_t k = 0; k + 1 < S.size(u); k++) S.push_elem(u, k, S.flag(u));
            if (S.flag(u) != flag) flag = F_S;
            if (S.npend == 0) {   // nothing left but this point: it is the common version
                if (!q.c_cap) { st = GQ_OVERFLOW; stopped = true; break; }
                common[nc++] = re - 1;
                stopped = true;
                break;
            }
        }
        if (stopped) break;
        sp.push(es, re, mflag(uint32_t(e), re - 1));
        const uint32_t p0 = E[e].poff, np = E[e + 1].poff - p0;
        if (np) S.push(TP_PARENTS, uint32_t(e), np, flag, int32_t(P.par[p0 + np - 1]), P.pent[p0 + np - 1]);
        else S.push(TP_PARENTS, uint32_t(e), 0, flag, ROOT_LV, n);
    }
    if (st == GQ_OK && S.overflow) st = GQ_OVERFLOW;
    sp.flush();
    if (st == GQ_OK && sp.overflow) st = GQ_OVERFLOW;
    res->status = st;
    res->n0 = sp.n;
    res->n_common = nc;
}

}  // namespace ldev

int launch_levels(const LevelParams &p, void *stream) {
    if (!p.n_graphs) return 0;
    hipLaunchKernelGGL(ldev::level_kernel, dim3(p.n_graphs), dim3(ldev::NT), 0, reinterpret_cast<hipStream_t>(stream), p);
    return hipGetLastError() == hipSuccess ? 0 : 66;
}

int launch_level_diff(const LevelParams &p, const GraphParams &q, void *stream) {
    if (!q.n_queries) return 0;
    hipLaunchKernelGGL(ldev::level_diff_kernel, dim3(q.n_queries), dim3(ldev::NT), 2 * size_t(p.lds_ent) * 4,
                       reinterpret_cast<hipStream_t>(stream), p, q);
    return hipGetLastError() == hipSuccess ? 0 : 66;
}

int launch_level_conflict(const LevelParams &p, const GraphParams &q, void *stream) {
    if (!q.n_queries) return 0;
    hipLaunchKernelGGL(ldev::level_conflict_kernel, dim3(q.n_queries), dim3(ldev::NT), 2 * size_t(p.lds_ent) * 4,
                       reinterpret_cast<hipStream_t>(stream), p, q);
    return hipGetLastError() == hipSuccess ? 0 : 66;
}

}  // namespace dtgpu
