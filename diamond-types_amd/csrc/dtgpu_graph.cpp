// dtgpu_graph.cpp -- C ABI of the batched causal-graph queries (include/dtgpu.h,
// dtgpu_graph_queries).  Graphs arrive as the reference's GraphEntrySimple lists and are built
// with Graph::push (entry merging and shadows as graph/mod.rs:85-128 computes them), then every
// query of the batch runs on the device, one wavefront each (dt_graph.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/dtgpu.h"
#include "dt_devbuf.hpp"
#include "dt_graph.hpp"
#include "dt_host.hpp"

using namespace dtgpu;

// experiment switches for the level-synchronous conflict sweep (unset: the defaults)
static uint32_t env_u32(const char *name, uint32_t dflt) {
    const char *v = std::getenv(name);
    return v && *v ? uint32_t(std::strtoul(v, nullptr, 10)) : dflt;
}

extern "C" dtgpu_status dtgpu_graph_queries(const int64_t *hist, const size_t *hist_off, size_t n_graphs,
                                            const dtgpu_graph_query *queries, size_t nq, int64_t *spans,
                                            size_t span_cap, int64_t *common, size_t common_cap,
                                            dtgpu_graph_answer *answers, float *ms) {
    if ((n_graphs && (!hist || !hist_off)) || (nq && (!queries || !answers)) || (nq && span_cap && !spans) ||
        (nq && common_cap && !common))
        return DTGPU_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return DTGPU_ERR_NO_DEVICE;
    // graphs -> entry quads + parents
    std::vector<uint32_t> ents, par;
    std::vector<uint32_t> goff(n_graphs), gn(n_graphs), gmaxp(n_graphs, 0);
    for (size_t g = 0; g < n_graphs; g++) {
        Graph G;
        for (size_t i = hist_off[g]; i < hist_off[g + 1];) {
            if (i + 3 > hist_off[g + 1]) return DTGPU_ERR_ARG;
            const int64_t s = hist[i], e = hist[i + 1], np = hist[i + 2];
            if (s < 0 || e <= s || e >= (int64_t(1) << 30) || np < 0 || i + 3 + size_t(np) > hist_off[g + 1])
                return DTGPU_ERR_ARG;
            std::vector<uint64_t> p(static_cast<size_t>(np));
            for (int64_t k = 0; k < np; k++) {
                if (hist[i + 3 + k] < 0 || hist[i + 3 + k] >= s) return DTGPU_ERR_ARG;
                p[size_t(k)] = uint64_t(hist[i + 3 + k]);
            }
            G.push(p, uint64_t(s), uint64_t(e));
            i += 3 + size_t(np);
        }
        goff[g] = uint32_t(ents.size() / 4);
        gn[g] = uint32_t(G.entries.size());
        for (const GraphEntry &e : G.entries) {
            gmaxp[g] = std::max(gmaxp[g], uint32_t(e.parents.size()));
            ents.push_back(uint32_t(e.start));
            ents.push_back(uint32_t(e.end));
            ents.push_back(uint32_t(e.shadow));
            ents.push_back(uint32_t(par.size()));
            for (uint64_t p : e.parents) par.push_back(uint32_t(p));
        }
        ents.insert(ents.end(), {0u, 0u, 0u, uint32_t(par.size())});
    }
    std::vector<GraphQuery> q(nq);
    std::vector<int32_t> front;   // every query's versions, a then b
    // every query's output spans in one u32-indexed arena: out_off = i * out_cap must not wrap
    if (span_cap > (size_t(1) << 28)) return DTGPU_ERR_ARG;
    const uint32_t out_cap = uint32_t(4 * std::max<size_t>(span_cap, 1));
    if (uint64_t(nq) * out_cap > (uint64_t(1) << 31)) return DTGPU_ERR_ARG;
    const uint32_t c_cap = uint32_t(std::min<size_t>(common_cap, 1u << 24));
    // every query's common-frontier slots in one u32-indexed arena (as the frontier arena's 2^28 check)
    if (uint64_t(nq) * c_cap > (uint64_t(1) << 28)) return DTGPU_ERR_ARG;
    auto npar_of = [&](uint32_t ent_off, uint32_t n_ent) -> uint64_t {
        return ents[4 * (size_t(ent_off) + n_ent) + 3] - ents[4 * size_t(ent_off) + 3];
    };
    for (size_t i = 0; i < nq; i++) {
        const dtgpu_graph_query &s = queries[i];
        GraphQuery &d = q[i];
        std::memset(&d, 0, sizeof d);
        const size_t nb = s.kind == GQ_CONTAINS ? 0 : s.nb;
        if (s.graph >= n_graphs || s.kind > GQ_CONFLICT_LEVEL || (s.na && !s.a) || (nb && !s.b) ||
            s.na + nb > (size_t(1) << 28))
            return DTGPU_ERR_ARG;
        d.kind = s.kind;
        d.ent_off = goff[s.graph];
        d.n_ent = gn[s.graph];
        d.na = uint32_t(s.na);
        d.nb = uint32_t(nb);
        d.f_off = uint32_t(front.size());
        for (size_t k = 0; k < s.na; k++) front.push_back(int32_t(std::max<int64_t>(std::min<int64_t>(s.a[k], INT32_MAX), -1)));
        for (size_t k = 0; k < nb; k++) front.push_back(int32_t(std::max<int64_t>(std::min<int64_t>(s.b[k], INT32_MAX), -1)));
        d.target = int32_t(std::max<int64_t>(s.target, -1));
        d.out_off = uint32_t(i) * out_cap;
        d.out_cap = out_cap;
        d.c_off = uint32_t(i) * c_cap;
        d.c_cap = c_cap;
        d.max_par = gmaxp[s.graph];
        const uint64_t npar = npar_of(d.ent_off, d.n_ent);
        d.hk_cap = gq_key_cap(npar, d.na, d.nb);
        d.htp_cap = gq_tp_cap(d.n_ent, npar, d.na, d.nb);
    }
    // HBM scratch of the level-synchronous queries: marks (diff), marks + buckets + time points
    // (conflict spans), sized by the query's graph
    uint64_t qscr_words = 0;
    for (size_t i = 0; i < nq; i++) {
        GraphQuery &d = q[i];
        if (d.kind != GQ_DIFF_LEVEL && d.kind != GQ_CONFLICT_LEVEL) continue;
        const uint64_t npar = npar_of(d.ent_off, d.n_ent);
        d.scr_off = qscr_words;
        if (d.kind == GQ_DIFF_LEVEL) qscr_words += 2ull * d.n_ent;
        else {
            d.scr_tp = conflict_level_tps(d.n_ent, npar, d.na, d.nb);
            qscr_words += conflict_level_words(d.n_ent, npar, d.na, d.nb);
        }
    }
    // graphs that level-synchronous diffs run on
    std::vector<LevelGraph> lg;
    {
        std::vector<uint8_t> want(n_graphs, 0);
        for (size_t i = 0; i < nq; i++)
            if (queries[i].kind == GQ_DIFF_LEVEL || queries[i].kind == GQ_CONFLICT_LEVEL) want[queries[i].graph] = 1;
        for (size_t g = 0; g < n_graphs; g++) if (want[g]) lg.push_back(LevelGraph{goff[g], gn[g]});
    }
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    DevBuf<uint32_t> d_ents, d_par, d_out, d_hscr;
    DevBuf<int32_t> d_front, d_common;
    DevBuf<GraphQuery> d_q;
    DevBuf<GraphResult> d_r;
    DevBuf<uint32_t> d_pent, d_child, d_level, d_order, d_loff, d_meta, d_gscr, d_qscr, d_prof;
    DevBuf<LevelGraph> d_lg;
    dtgpu_status rc = DTGPU_OK;
    std::vector<GraphResult> res(nq);
    std::vector<uint32_t> out(size_t(nq) * out_cap);
    std::vector<int32_t> com(size_t(nq) * c_cap);
    do {
#define CK(x) do { if ((x) != hipSuccess) { rc = DTGPU_ERR_HIP; goto done; } } while (0)
        CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(d_ents.upload(ents, st));
        CK(d_par.upload(par, st));
        CK(d_q.upload(q, st));
        CK(d_r.alloc(nq));
        CK(d_out.alloc(out.size()));
        CK(d_front.upload(front, st));
        CK(d_common.alloc(std::max<size_t>(com.size(), 1)));
        {
            GraphParams P{d_ents.p, d_par.p, d_out.p, d_q.p, d_r.p, uint32_t(nq), d_front.p, d_common.p, nullptr};
            LevelParams LP{};
            if (!lg.empty()) {
                const size_t nquad = ents.size() / 4;
                CK(d_pent.alloc(par.size()));
                CK(d_child.alloc(par.size()));
                CK(d_level.alloc(nquad));
                CK(d_order.alloc(nquad));
                CK(d_loff.alloc(nquad));
                CK(d_meta.alloc(2 * nquad));
                CK(d_gscr.alloc(3 * nquad));
                CK(d_qscr.alloc(std::max<uint64_t>(qscr_words, 1)));
                CK(d_lg.upload(lg, st));
                uint32_t max_ent = 0;
                for (const LevelGraph &g : lg) max_ent = std::max(max_ent, g.n_ent);
                LP = LevelParams{d_ents.p, d_par.p, d_pent.p, d_child.p, d_level.p, d_order.p, d_loff.p, d_meta.p,
                                 d_gscr.p, d_qscr.p, d_lg.p, uint32_t(lg.size()),
                                 max_ent <= kLevelLdsEntries ? max_ent : 0u,
                                 max_ent <= kLevelLdsLevelling ? max_ent : 0u,
                                 std::max<uint32_t>(8, env_u32("DTGPU_LVL_PTS_LDS", 64)), nullptr};
                if (env_u32("DTGPU_LVL_PROF", 0)) {
                    CK(d_prof.alloc(4 * nq));
                    CK(hipMemsetAsync(d_prof.p, 0, 4 * nq * 4, st));
                    LP.prof = d_prof.p;
                }
            }
            CK(hipEventRecord(e0, st));
            if (launch_graph_queries(P, st, false)) { rc = DTGPU_ERR_HIP; goto done; }
            // the heap walks whose queues outgrew LDS, again with their queues in HBM scratch
            bool any_heap = false;
            for (size_t i = 0; i < nq; i++) any_heap |= q[i].kind != GQ_DIFF_LEVEL && q[i].kind != GQ_CONFLICT_LEVEL;
            if (any_heap) {
                std::vector<GraphResult> r1(nq);
                CK(hipMemcpyAsync(r1.data(), d_r.p, nq * sizeof(GraphResult), hipMemcpyDeviceToHost, st));
                CK(hipStreamSynchronize(st));
                uint64_t hw = 0;
                for (size_t i = 0; i < nq; i++) {
                    if (r1[i].status != GQ_QUEUE_FULL) continue;
                    GraphQuery &d = q[i];
                    d.h_off = hw;
                    hw += d.hk_cap + uint64_t(d.htp_cap + 3) * gq_tp_words(d.max_par, d.na, d.nb);
                }
                if (hw) {
                    CK(d_hscr.alloc(hw));
                    // the heap offsets into the same query buffer (P and the level kernels hold it)
                    CK(hipMemcpyAsync(d_q.p, q.data(), nq * sizeof(GraphQuery), hipMemcpyHostToDevice, st));
                    P.hscr = d_hscr.p;
                    if (launch_graph_queries(P, st, true)) { rc = DTGPU_ERR_HIP; goto done; }
                }
            }
            if (!lg.empty() && (launch_levels(LP, st) || launch_level_diff(LP, P, st) || launch_level_conflict(LP, P, st, false))) {
                rc = DTGPU_ERR_HIP;
                goto done;
            }
            // the level conflict queries whose live time points or buckets outgrew LDS, again with
            // their points in HBM scratch
            bool any_lc = false;
            for (size_t i = 0; i < nq; i++) any_lc |= q[i].kind == GQ_CONFLICT_LEVEL;
            if (any_lc) {
                std::vector<GraphResult> r1(nq);
                CK(hipMemcpyAsync(r1.data(), d_r.p, nq * sizeof(GraphResult), hipMemcpyDeviceToHost, st));
                CK(hipStreamSynchronize(st));
                bool full = false;
                for (size_t i = 0; i < nq; i++) full |= q[i].kind == GQ_CONFLICT_LEVEL && r1[i].status == GQ_QUEUE_FULL;
                if (full && launch_level_conflict(LP, P, st, true)) { rc = DTGPU_ERR_HIP; goto done; }
            }
            CK(hipEventRecord(e1, st));
        }
        if (nq) {
            CK(hipMemcpyAsync(res.data(), d_r.p, nq * sizeof(GraphResult), hipMemcpyDeviceToHost, st));
            CK(hipMemcpyAsync(out.data(), d_out.p, out.size() * 4, hipMemcpyDeviceToHost, st));
            if (!com.empty()) CK(hipMemcpyAsync(com.data(), d_common.p, com.size() * 4, hipMemcpyDeviceToHost, st));
        }
        CK(hipStreamSynchronize(st));
        if (d_prof.p) {   // DTGPU_LVL_PROF: per-phase summary of the conflict sweeps (stderr)
            std::vector<uint32_t> pr(4 * nq);
            CK(hipMemcpy(pr.data(), d_prof.p, pr.size() * 4, hipMemcpyDeviceToHost));
            double sum[4] = {0, 0, 0, 0};
            uint32_t mx[4] = {0, 0, 0, 0}, nk = 0, worst = 0;
            for (size_t i = 0; i < nq; i++) {
                if (q[i].kind != GQ_CONFLICT_LEVEL) continue;
                nk++;
                for (int k = 0; k < 4; k++) { sum[k] += pr[4 * i + k]; mx[k] = std::max(mx[k], pr[4 * i + k]); }
                if (pr[4 * i] + pr[4 * i + 1] + pr[4 * i + 2] > pr[4 * worst] + pr[4 * worst + 1] + pr[4 * worst + 2]) worst = uint32_t(i);
            }
            if (nk)
                fprintf(stderr, "lvlprof queries=%u mean kcyc marks=%.1f cand=%.1f sweep=%.1f visited=%.1f | max %.1f %.1f %.1f %u"
                        " | worst marks=%.1f cand=%.1f sweep=%.1f visited=%u\n", nk, sum[0] / nk * 0.016, sum[1] / nk * 0.016,
                        sum[2] / nk * 0.016, sum[3] / nk, mx[0] * 0.016, mx[1] * 0.016, mx[2] * 0.016, mx[3],
                        pr[4 * worst] * 0.016, pr[4 * worst + 1] * 0.016, pr[4 * worst + 2] * 0.016, pr[4 * worst + 3]);
        }
        if (ms) {
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            *ms = t;
        }
#undef CK
    } while (false);
    for (size_t i = 0; i < nq && rc == DTGPU_OK; i++) {
        const GraphResult &r = res[i];
        dtgpu_graph_answer &a = answers[i];
        std::memset(&a, 0, sizeof a);
        a.status = r.status == GQ_QUEUE_FULL ? uint32_t(GQ_OVERFLOW) : r.status;
        const uint32_t *o = out.data() + size_t(i) * out_cap;
        int64_t *sp = spans ? spans + i * span_cap * 3 : nullptr;
        if (q[i].kind == GQ_DIFF || q[i].kind == GQ_DIFF_LEVEL) {
            if (r.n0 + r.n1 > span_cap) { a.status = GQ_OVERFLOW; continue; }
            for (uint32_t k = 0; k < r.n0; k++) { sp[3 * k] = int32_t(o[2 * k]); sp[3 * k + 1] = int32_t(o[2 * k + 1]); sp[3 * k + 2] = 0; }
            const uint32_t *ob = o + 2 * (out_cap / 4);
            for (uint32_t k = 0; k < r.n1; k++) {
                int64_t *t = sp + 3 * (r.n0 + k);
                t[0] = int32_t(ob[2 * k]); t[1] = int32_t(ob[2 * k + 1]); t[2] = 1;
            }
            a.n_a = r.n0;
            a.n_b = r.n1;
        } else if (q[i].kind == GQ_CONFLICT || q[i].kind == GQ_CONFLICT_LEVEL) {
            if (r.n0 > span_cap) { a.status = GQ_OVERFLOW; continue; }
            for (uint32_t k = 0; k < 3 * r.n0; k++) sp[k] = int32_t(o[k]);
            a.n_a = r.n0;
            a.n_common = r.n_common;
            for (uint32_t k = 0; k < r.n_common && k < c_cap; k++) common[i * common_cap + k] = com[size_t(i) * c_cap + k];
        } else if (q[i].kind == GQ_DOMINATORS) {
            a.n_common = r.n_common;
            for (uint32_t k = 0; k < r.n_common && k < c_cap; k++) common[i * common_cap + k] = com[size_t(i) * c_cap + k];
        } else {
            a.n_a = r.n0;
        }
    }
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
    return rc;
}
