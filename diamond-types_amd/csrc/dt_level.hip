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
#include "dt_device.hpp"

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

// LDS: every graph of the launch has at most P.lvl_lds entries (a template parameter, so every
// access is an LDS or a global instruction, never a flat one)
template <bool LDS>
__global__ __launch_bounds__(256) void level_kernel(LevelParams P) {
    __shared__ uint32_t s_sum[NT];
    __shared__ uint32_t s_tail, s_bad;
    const uint32_t g = blockIdx.x, t = threadIdx.x;
    if (g >= P.n_graphs) return;
    const LevelGraph G = P.graphs[g];
    const uint32_t n = G.n_ent, base = G.ent_off;
    uint32_t *meta = P.meta + 2 * size_t(base);   // [0] = levels, [1] = status
    // LDS (graphs up to P.lvl_lds entries): the round loop's dependent chain -- frontier entry,
    // its children offsets, each child's pending count -- stays out of HBM and its memory-side
    // atomics; the queue is copied to order[] at the end
    extern __shared__ uint32_t lsh[];
    uint32_t *cur = LDS ? lsh : P.gscr + 3 * size_t(base);   // child counts, then fill cursors (n + 1)
    uint32_t *cofs = cur + (n + 1);                          // children CSR offsets (n + 1)
    uint32_t *pend = cofs + (n + 1);                         // parents not yet levelled (n)
    uint32_t *ord = LDS ? pend + n : P.order + base;         // entries in level order (n)
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
        if (pend[e] == 0) ord[atomicAdd(&s_tail, 1u)] = e;   // roots: level 0
    __syncthreads();
    // one level per round; a round's frontier is ord[head, tail)
    uint32_t head = 0, tail = s_tail, L = 0;
    while (head < tail) {
        if (t == 0) P.lvl_off[base + L] = head;
        for (uint32_t i = head + t; i < tail; i += NT) {
            const uint32_t e = ord[i];
            P.level[base + e] = L;
            for (uint32_t j = cofs[e]; j < cofs[e + 1]; j++) {
                const uint32_t c = P.child[plo + j];
                if (atomicSub(&pend[c], 1u) == 1u) ord[atomicAdd(&s_tail, 1u)] = c;
            }
        }
        __syncthreads();
        head = tail;
        tail = s_tail;
        L++;
        __syncthreads();   // every thread has read s_tail before the next round adds to it
    }
    if (LDS)
        for (uint32_t i = t; i < head; i += NT) P.order[base + i] = ord[i];
    if (t == 0) {
        P.lvl_off[base + L] = head;
        meta[0] = L;
        meta[1] = head == n ? GQ_OK : GQ_BAD_INPUT;   // a cycle leaves entries unlevelled
    }
}

// The marks of a query (see the header), level by level.  Every thread returns the same status.
__device__ __forceinline__ uint32_t push_marks(const LevelParams &P, const GraphQuery &q, const int32_t *qa, const Ent *E, int32_t *mA,
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

template <bool LM>   // the marks in LDS (every levelled graph has at most P.lds_ent entries)
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
    extern __shared__ int32_t lmarks[];
    int32_t *mA = LM ? lmarks : reinterpret_cast<int32_t *>(P.qscr + q.scr_off), *mB = mA + n;
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
// versions.  LP: the pool is LDS (capacity P.sweep_pts; consumed points are recycled, so only
// the live ones count), else the query's HBM scratch.
template <bool LP>
struct Sweep {
    const Ent *E;
    const uint32_t *par, *pent;   // parent LVs and their entries (per parent slot)
    const int32_t *qa, *qb;   // the two versions (frontier arena)
    int32_t *head;            // per entry: its bucket (LDS or HBM)
    uint32_t *lpool, *pool;
    uint32_t n, cap, used, npend;
    bool overflow;
    uint32_t freed = 0xFFFFFFFFu;   // consumed points, linked through word 0: reused first, so the
                                    // live points (a few per frontier element) stay in the LDS part

    __device__ uint32_t *pt(uint32_t tp) const { return LP ? lpool + PW * tp : pool + PW * size_t(tp); }
    __device__ int32_t elem(uint32_t tp, uint32_t k) const {
        const uint32_t *w = pt(tp);
        switch (w[1] >> 2) {
            case TP_ONE: return int32_t(w[3]);
            case TP_PARENTS: return int32_t(par[E[w[3]].poff + k]);
            case TP_QA: return qa[k];
            default: return qb[k];
        }
    }
    __device__ uint32_t size(uint32_t tp) const { return pt(tp)[2]; }
    __device__ uint32_t flag(uint32_t tp) const { return pt(tp)[1] & 3u; }
    __device__ int32_t last(uint32_t tp) const { return int32_t(pt(tp)[4]); }
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
        uint32_t tp;
        if (freed != 0xFFFFFFFFu) { tp = freed; freed = pt(tp)[0]; }
        else if (used >= cap) { overflow = true; return; }
        else tp = used++;
        uint32_t *w = pt(tp);
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
    __device__ void release(uint32_t tp) { pt(tp)[0] = freed; freed = tp; }
    // element k of point tp as a TP_ONE point (a shattered frontier)
    __device__ void push_elem(uint32_t tp, uint32_t k, uint32_t f) {
        const uint32_t *w = pt(tp);
        const int32_t x = elem(tp, k);
        push(TP_ONE, uint32_t(x), 1, f, x, (w[1] >> 2) == TP_PARENTS ? pent[E[w[3]].poff + k] : n);
    }
};

__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t l) { return uint32_t(__builtin_amdgcn_readlane(int(v), int(l))); }

// LM: marks and bucket heads in LDS.  LP (first pass): the time points and sorted buckets in LDS;
// a query that outgrows them ends at GQ_QUEUE_FULL and is answered again by the !LP launch, which
// handles only those queries, with its points in the query's HBM scratch.
template <bool LM, bool LP>
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
    if (!LP && res->status != GQ_QUEUE_FULL) return;   // the second pass: only the queries the first left
    const Ent *E = reinterpret_cast<const Ent *>(P.ents) + base;
    uint32_t *out = Q.out + size_t(q.out_off);
    if (meta[1] != GQ_OK) {
        if (t == 0) { res->status = meta[1]; res->n0 = res->n_common = 0; }
        return;
    }
    const int32_t *qa = Q.front + q.f_off, *qb = qa + q.na;
    int32_t *common = Q.common + q.c_off;   // written by wave 0 only
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
    // LDS: the marks and bucket heads (LM), then the time points (LP)
    extern __shared__ int32_t lmarks[];
    const uint32_t le = P.lds_ent;
    int32_t *mA = LM ? lmarks : hbm, *mB = mA + n;
    int32_t *head = LM ? lmarks + 2 * le : hbm + 2 * n;
    uint32_t *lpool = reinterpret_cast<uint32_t *>(LM ? lmarks + 3 * le : lmarks);
    uint32_t *cand = reinterpret_cast<uint32_t *>(hbm + 3 * n);
    uint32_t *pool = cand + n;
    for (uint32_t e = t; e < n; e += NT) head[e] = -1;
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    const uint32_t mst = push_marks(P, q, qa, E, mA, mB, &s_top, &s_st);
    const uint64_t c1 = __builtin_amdgcn_s_memtime();
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
    if (t >= 64) return;
    const uint64_t c2 = __builtin_amdgcn_s_memtime();
    uint32_t visited = 0;
    // ---- the sweep: wave 0, every lane running the same sequential walk (so its state stays
    // wave-uniform), the lanes fetching the next 64 candidates' entries and parents at once ----
    const uint32_t lane = t;
    Sweep<LP> S{E, P.par, P.pent, qa, qb, head, lpool, pool, n, LP ? P.sweep_pts : q.scr_tp, 0, 0, false};
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
    // lane j of the batch: candidate cand[bbase - bhave + j], its start, parent count and last parent
    uint32_t b_e = 0, b_np = 0, b_lpe = n;
    int32_t b_s = 0, b_lp = ROOT_LV;
    uint32_t bbase = 0, bhave = 0, bj = 0;
    for (;;) {
        // the next entry holding a pending point: only entries the marks touch can
        int32_t e = -1;
        uint32_t jj = 0;
        for (;;) {
            if (bj >= bhave) {
                if (bbase >= ncand) break;
                bhave = min(64u, ncand - bbase);
                const uint32_t x = lane < bhave ? cand[bbase + lane] : 0u;
                const uint32_t p0 = E[x].poff, p1 = E[x + 1].poff;
                b_e = x;
                b_s = E[x].start;
                b_np = p1 - p0;
                b_lp = ROOT_LV;
                b_lpe = n;
                if (p1 > p0) { b_lp = int32_t(P.par[p1 - 1]); b_lpe = P.pent[p1 - 1]; }
                bbase += bhave;
                bj = 0;
            }
            const int32_t hv = lane >= bj && lane < bhave ? head[b_e] : -1;
            const uint64_t m = __ballot(hv >= 0);
            if (m) {
                jj = uint32_t(__ffsll((long long)m) - 1);
                e = int32_t(rdlane(b_e, jj));
                bj = jj + 1;
                break;
            }
            bj = bhave;
        }
        if (S.overflow) { st = LP ? GQ_QUEUE_FULL : GQ_OVERFLOW; break; }
        if (e < 0) break;   // only ROOT points left: nothing in common
        visited++;
        // the bucket in heap order (insertion sort; buckets are small -- in LDS up to BUCKET_CAP
        // points, in the query's HBM scratch beyond)
        uint32_t m = 0;
        for (int32_t x = head[e]; x >= 0; x = int32_t(S.pt(uint32_t(x))[0])) m++;
        if (LP && m > BUCKET_CAP) { st = GQ_QUEUE_FULL; break; }
        uint32_t *bk = LP || m <= BUCKET_CAP ? bkl : hbk;
        m = 0;
        for (int32_t x = head[e]; x >= 0; x = int32_t(S.pt(uint32_t(x))[0])) {
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
        const int32_t es = int32_t(rdlane(uint32_t(b_s), jj));
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
        for (uint32_t k = 0; k < m; k++) S.release(bk[k]);   // every point of the bucket is consumed
        S.push(TP_PARENTS, uint32_t(e), rdlane(b_np, jj), flag, int32_t(rdlane(uint32_t(b_lp), jj)), rdlane(b_lpe, jj));
    }
    if (st == GQ_OK && S.overflow) st = LP ? GQ_QUEUE_FULL : GQ_OVERFLOW;
    sp.flush();
    if (st == GQ_OK && sp.overflow) st = GQ_OVERFLOW;
    if (lane == 0) {
        res->status = st;
        res->n0 = sp.n;
        res->n_common = nc;
        if (P.prof) {
            const uint64_t c3 = __builtin_amdgcn_s_memtime();
            uint32_t *w = P.prof + 4 * size_t(qi);
            w[0] = uint32_t((c1 - c0) >> 4);
            w[1] = uint32_t((c2 - c1) >> 4);
            w[2] = uint32_t((c3 - c2) >> 4);
            w[3] = visited;
        }
    }
}

}  // namespace ldev

int launch_levels(const LevelParams &p, void *stream) {
    if (!p.n_graphs) return 0;
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (p.lvl_lds) hipLaunchKernelGGL(ldev::level_kernel<true>, dim3(p.n_graphs), dim3(ldev::NT), level_lds_bytes(p.lvl_lds), st, p);
    else hipLaunchKernelGGL(ldev::level_kernel<false>, dim3(p.n_graphs), dim3(ldev::NT), 0, st, p);
    return launch_error() == hipSuccess ? 0 : 66;
}

int launch_level_diff(const LevelParams &p, const GraphParams &q, void *stream) {
    if (!q.n_queries) return 0;
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (p.lds_ent) hipLaunchKernelGGL(ldev::level_diff_kernel<true>, dim3(q.n_queries), dim3(ldev::NT), 8 * size_t(p.lds_ent), st, p, q);
    else hipLaunchKernelGGL(ldev::level_diff_kernel<false>, dim3(q.n_queries), dim3(ldev::NT), 0, st, p, q);
    return launch_error() == hipSuccess ? 0 : 66;
}

int launch_level_conflict(const LevelParams &p, const GraphParams &q, void *stream, bool big) {
    if (!q.n_queries) return 0;
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const size_t lm = 12 * size_t(p.lds_ent), lp = big ? 0 : 4 * size_t(p.sweep_pts) * kLevelPointWords;
    if (p.lds_ent) {
        if (big) hipLaunchKernelGGL((ldev::level_conflict_kernel<true, false>), dim3(q.n_queries), dim3(ldev::NT), lm + lp, st, p, q);
        else hipLaunchKernelGGL((ldev::level_conflict_kernel<true, true>), dim3(q.n_queries), dim3(ldev::NT), lm + lp, st, p, q);
    } else {
        if (big) hipLaunchKernelGGL((ldev::level_conflict_kernel<false, false>), dim3(q.n_queries), dim3(ldev::NT), lp, st, p, q);
        else hipLaunchKernelGGL((ldev::level_conflict_kernel<false, true>), dim3(q.n_queries), dim3(ldev::NT), lp, st, p, q);
    }
    return launch_error() == hipSuccess ? 0 : 66;
}

}  // namespace dtgpu
