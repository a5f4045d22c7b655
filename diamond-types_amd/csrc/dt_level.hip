// dt_level.hip -- level-synchronous causal-graph kernels (north_star "Causal graph": diff and
// topological levelling as level-synchronous propagation over CSR parent arrays in HBM).
//
// level_kernel (one 256-thread workgroup per graph) levels the graph's entries: level(e) =
// 1 + max level of its parent entries (roots 0), so every child sits on a higher level than
// its parents.  Built in place from the entry quads and parent LVs of dt_graph.hip's arena:
//   1. parent slot -> parent entry (one binary search per slot, all slots in parallel) and a
//      children CSR (counting sort of the slots by parent entry, LDS atomics);
//   2. Kahn's algorithm one level per round: the round's frontier releases the children whose
//      last pending parent it held; the rounds' frontiers, concatenated, are the entries in
//      level order (order[], level offsets lvl_off[]).
// level_diff_kernel (one workgroup per query) answers Graph::diff (tools.rs:158-292) by
// propagating two marks down the levels: mA[e] / mB[e] = the highest LV of entry e in the
// history of a / b (the history holds a prefix of every entry it touches); a level's entries
// push their marks to their parents' entries with LDS atomicMax, all in parallel, and a barrier
// separates the levels.  only-a of entry e is (mB[e], mA[e]], and the spans come out newest
// first, merged when contiguous -- the same lists as the heap walk (dt_graph.hip q_diff).
//
// The heap walk stops as soon as the two walks meet; the level sweep visits every level from
// the inputs' highest down to the roots.  tools/level_bench.py times both on the same queries.
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
    __shared__ uint32_t s_cur[LVL_MAX_ENTRIES + 1];    // child counts, then fill cursors
    __shared__ uint32_t s_cofs[LVL_MAX_ENTRIES + 1];   // children CSR offsets
    __shared__ uint32_t s_pend[LVL_MAX_ENTRIES];       // parents not yet levelled
    __shared__ uint32_t s_sum[NT];
    __shared__ uint32_t s_tail, s_bad;
    const uint32_t g = blockIdx.x, t = threadIdx.x;
    if (g >= P.n_graphs) return;
    const LevelGraph G = P.graphs[g];
    const uint32_t n = G.n_ent, base = G.ent_off;
    uint32_t *meta = P.meta + 2 * size_t(base);   // [0] = levels, [1] = status
    if (n > LVL_MAX_ENTRIES) {
        if (t == 0) { meta[0] = 0; meta[1] = GQ_OVERFLOW; }
        return;
    }
    const Ent *E = reinterpret_cast<const Ent *>(P.ents) + base;
    const uint32_t plo = E[0].poff, phi = E[n].poff;
    if (t == 0) { s_bad = 0; s_tail = 0; }
    for (uint32_t e = t; e < n; e += NT) {
        s_cur[e] = 0;
        s_pend[e] = E[e + 1].poff - E[e].poff;
    }
    __syncthreads();
    for (uint32_t k = plo + t; k < phi; k += NT) {
        const uint32_t pe = find(E, n, int32_t(P.par[k]));
        if (pe == n) { s_bad = 1; continue; }
        P.pent[k] = pe;
        atomicAdd(&s_cur[pe], 1u);
    }
    __syncthreads();
    if (s_bad) {
        if (t == 0) { meta[0] = 0; meta[1] = GQ_BAD_INPUT; }
        return;
    }
    // exclusive scan of the child counts: per-thread chunks, then the 256 chunk totals
    const uint32_t per = (n + NT - 1) / NT, c0 = min(n, t * per), c1 = min(n, c0 + per);
    uint32_t sum = 0;
    for (uint32_t e = c0; e < c1; e++) sum += s_cur[e];
    s_sum[t] = sum;
    __syncthreads();
    if (t == 0) {
        uint32_t run = 0;
        for (uint32_t i = 0; i < NT; i++) { const uint32_t x = s_sum[i]; s_sum[i] = run; run += x; }
        s_cofs[n] = run;
    }
    __syncthreads();
    {
        uint32_t run = s_sum[t];
        for (uint32_t e = c0; e < c1; e++) {
            const uint32_t c = s_cur[e];
            s_cofs[e] = run;
            s_cur[e] = run;
            run += c;
        }
    }
    __syncthreads();
    for (uint32_t e = t; e < n; e += NT)
        for (uint32_t k = E[e].poff; k < E[e + 1].poff; k++) P.child[plo + atomicAdd(&s_cur[P.pent[k]], 1u)] = e;
    for (uint32_t e = t; e < n; e += NT)
        if (s_pend[e] == 0) P.order[base + atomicAdd(&s_tail, 1u)] = e;   // roots: level 0
    __syncthreads();
    // one level per round; a round's frontier is order[head, tail)
    uint32_t head = 0, tail = s_tail, L = 0;
    while (head < tail) {
        if (t == 0) P.lvl_off[base + L] = head;
        for (uint32_t i = head + t; i < tail; i += NT) {
            const uint32_t e = P.order[base + i];
            P.level[base + e] = L;
            for (uint32_t j = s_cofs[e]; j < s_cofs[e + 1]; j++) {
                const uint32_t c = P.child[plo + j];
                if (atomicSub(&s_pend[c], 1u) == 1u) P.order[base + atomicAdd(&s_tail, 1u)] = c;
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

// Spans newest first, contiguous ones merged (push_reversed_rle), as dt_graph.hip writes them.
struct RevSpans {
    uint32_t *out;
    uint32_t cap, n;
    int32_t ls, le;
    bool have, overflow;
    __device__ void push(int32_t s, int32_t e) {
        if (have && ls == e) { ls = s; return; }
        flush();
        have = true; ls = s; le = e;
    }
    __device__ void flush() {
        if (!have) return;
        if (n >= cap) { overflow = true; have = false; return; }
        out[2 * n] = uint32_t(ls);
        out[2 * n + 1] = uint32_t(le);
        n++;
        have = false;
    }
};

__global__ __launch_bounds__(256) void level_diff_kernel(LevelParams P, GraphParams Q) {
    __shared__ int32_t mA[LVL_MAX_ENTRIES], mB[LVL_MAX_ENTRIES];
    __shared__ uint32_t s_top, s_st;
    const uint32_t qi = blockIdx.x, t = threadIdx.x;
    if (qi >= Q.n_queries) return;
    const GraphQuery &q = Q.queries[qi];
    if (q.kind != GQ_DIFF_LEVEL) return;
    const uint32_t n = q.n_ent, base = q.ent_off;
    const uint32_t *meta = P.meta + 2 * size_t(base);
    GraphResult *res = Q.results + qi;
    if (meta[1] != GQ_OK || q.na > GQ_MAX_FRONTIER || q.nb > GQ_MAX_FRONTIER) {
        if (t == 0) { res->status = meta[1] != GQ_OK ? meta[1] : GQ_BAD_INPUT; res->n0 = res->n1 = res->n_common = 0; }
        return;
    }
    const Ent *E = reinterpret_cast<const Ent *>(P.ents) + base;
    for (uint32_t e = t; e < n; e += NT) { mA[e] = -1; mB[e] = -1; }
    __syncthreads();
    if (t == 0) {   // seed the marks with the two versions
        uint32_t top = 0, st = GQ_OK;
        for (uint32_t i = 0; i < q.na + q.nb && st == GQ_OK; i++) {
            const int32_t v = i < q.na ? q.a[i] : q.b[i - q.na];
            const uint32_t e = find(E, n, v);
            if (e == n) { st = GQ_BAD_INPUT; break; }
            int32_t *m = i < q.na ? mA : mB;
            m[e] = max(m[e], v);
            top = max(top, P.level[base + e]);
        }
        s_top = top;
        s_st = st;
    }
    __syncthreads();
    if (s_st != GQ_OK) {
        if (t == 0) { res->status = s_st; res->n0 = res->n1 = res->n_common = 0; }
        return;
    }
    // highest level first: a level's marks are final once every higher level has pushed
    for (int32_t L = int32_t(s_top); L >= 0; L--) {
        const uint32_t i0 = P.lvl_off[base + L], i1 = P.lvl_off[base + L + 1];
        for (uint32_t i = i0 + t; i < i1; i += NT) {
            const uint32_t e = P.order[base + i];
            const int32_t xa = mA[e], xb = mB[e];
            if (xa < 0 && xb < 0) continue;
            for (uint32_t k = E[e].poff; k < E[e + 1].poff; k++) {
                const uint32_t pe = P.pent[k];
                const int32_t p = int32_t(Q.par[k]);
                if (xa >= 0) atomicMax(&mA[pe], p);
                if (xb >= 0) atomicMax(&mB[pe], p);
            }
        }
        __syncthreads();
    }
    if (t == 0) {
        uint32_t *out = Q.out + size_t(q.out_off);
        RevSpans sa{out, q.out_cap / 4, 0, 0, 0, false, false};
        RevSpans sb{out + 2 * (q.out_cap / 4), q.out_cap / 4, 0, 0, 0, false, false};
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

}  // namespace ldev

int launch_levels(const LevelParams &p, void *stream) {
    if (!p.n_graphs) return 0;
    hipLaunchKernelGGL(ldev::level_kernel, dim3(p.n_graphs), dim3(ldev::NT), 0, reinterpret_cast<hipStream_t>(stream), p);
    return hipGetLastError() == hipSuccess ? 0 : 66;
}

int launch_level_diff(const LevelParams &p, const GraphParams &q, void *stream) {
    if (!q.n_queries) return 0;
    hipLaunchKernelGGL(ldev::level_diff_kernel, dim3(q.n_queries), dim3(ldev::NT), 0, reinterpret_cast<hipStream_t>(stream), p, q);
    return hipGetLastError() == hipSuccess ? 0 : 66;
}

}  // namespace dtgpu
