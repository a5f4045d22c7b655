// dtgpu_api.cpp -- C ABI of libdtgpu (include/dtgpu.h): oplog handles, batch staging in HBM,
// device checkout.  There is no CPU checkout path: without a HIP device every checkout call
// returns DTGPU_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <queue>
#include <set>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/dtgpu.h"
#include "dt_decoded.hpp"
#include "dt_devbuf.hpp"
#include "dt_device.hpp"
#include "dt_host.hpp"
#include "dt_prep.hpp"
#include "dt_encoder.hpp"
#include "dt_ff.hpp"

using namespace dtgpu;

struct dtgpu_oplog {
    HostOpLog o;
    std::vector<uint64_t> last_added;   // the frontier the last decode_and_add reported
};

namespace {

// Checkouts replay on the per-item tracker (dt_replay.hip); its LDS tiers go by index bytes: a
// document whose expected index fits a tier replays with its index in LDS, friendsforever-sized
// documents many per CU, a node_nodecc-sized one alone on a CU.  Bigger documents and LDS
// overflows replay on the HBM-index tier.
constexpr int kLdsTiers = kMaxLdsTiers;
constexpr uint64_t kItemTierCap[kLdsTiers] = {12 * 1024, 32 * 1024, 64 * 1024, 160 * 1024};
int item_tier(uint32_t est) {
    const uint64_t bytes = index_bytes_ms(est, lds_sb_capacity(est), true);
    for (int t = 0; t < kLdsTiers; t++) if (bytes <= kItemTierCap[t]) return t;
    return -1;
}
// How a batch checks out: the defaults, then dtgpu_batch_opts (the API's knobs), then the DTGPU_*
// environment overrides (experiments, A/B runs, tests), read once when the batch is created.
struct Settings {
    bool ff = true;            // linear histories on the fast-forward path (dt_ff.hip)
    bool seg = true;           // cut replay (long documents as LV segments on several waves)
    uint64_t seg_ops = 500;    // op runs per segment (raised to the batch's fair share per wave slot)
    uint32_t seg_max = 32;     // segments per document: measured against 16-64 on the six cut traces
    uint32_t seg_w = SEG_W_OP; // the cut planner's cost weight of an op run
    bool seg_fair = true;      // the fair-share floor on seg_ops
    bool seg_late = true;      // late documents of the smallest tier cut once
    // expected inserted chars per block when sizing a document's LDS index: blocks end up ~43
    // items full on the benchmark traces (cut_point, dt_replay.hip), sized at 40 (tests force the
    // LDS overflow -> HBM tier hand-back with a large value)
    uint64_t lds_fill = 40;
    bool flat = true;          // the smallest LDS tier on the flat 2-level index (IX_FLAT)
    bool plan_split = true;    // the <= 64-chain planner in two phases (walk order, then lane-parallel steps)
    // the walk four documents per wave (walk_kernel) before the plan kernel (also for a single
    // document: its walk then runs beside prep's second half, 12.9 -> 12.0 ms)
    bool plan_walk = true;
    bool prep_chains = true;   // prep as three launches, the chain decomposition four documents per wave
    bool walk_overlap = true;  // the walk on its own stream beside prep's second half
    bool host_plan = false;    // walk plans built on the host
    bool split = true;         // split pass for skewed batches
    bool critical = true;      // critical replays first, at top wave priority
    bool fallback = true;      // LDS-tier documents that outgrow their index replay on the HBM tier
    bool prio = true;          // late workgroups of the flat tier raise their wave priority
    uint32_t tog_waves = 0;    // 1: retreat / advance passes on one wave (else DTGPU_TOG_WAVES helpers)
    uint32_t tog_mw_lds = 32 * 1024;   // LDS index bytes from which a tier gets helper waves
    uint32_t debug = 0;        // bit 0 invariant checks, bit 1 cycle profile (the instrumented kernels)
    bool prep_check = false;   // the bounds-checked prep kernel
    bool pass_mark = false;    // every pass opens with pass_mark_kernel (tools/traffic.py)
    bool plan_prof = false, enc_prof = false;
    uint32_t enc_lds_text = 0;
};
Settings settings_for(const dtgpu_batch_opts *o) {
    Settings c;
    if (o) {
        c.ff = !(o->flags & DTGPU_OPT_NO_FAST_FORWARD);
        c.seg = !(o->flags & DTGPU_OPT_NO_SEGMENTS);
        c.host_plan = (o->flags & DTGPU_OPT_HOST_PLAN) != 0;
        c.split = !(o->flags & DTGPU_OPT_NO_SPLIT);
        c.critical = !(o->flags & DTGPU_OPT_NO_CRITICAL);
        c.debug = (o->flags & DTGPU_OPT_DEBUG) ? 1u : 0u;
        c.pass_mark = (o->flags & DTGPU_OPT_PASS_MARK) != 0;
        if (o->seg_ops) c.seg_ops = o->seg_ops;
        if (o->seg_max) c.seg_max = o->seg_max;
        if (o->lds_fill) c.lds_fill = o->lds_fill;
    }
    auto on = [](const char *name, bool &v) { if (const char *e = getenv(name)) v = *e != '0'; };
    auto set = [](const char *name) { return getenv(name) != nullptr; };
    auto num = [](const char *name, uint64_t lo, uint64_t hi, uint64_t &v) {
        if (const char *e = getenv(name)) v = std::min<uint64_t>(std::max<uint64_t>(lo, strtoull(e, nullptr, 10)), hi);
    };
    on("DTGPU_FF", c.ff);
    on("DTGPU_SEG", c.seg);
    num("DTGPU_SEG_OPS", 1, UINT64_MAX, c.seg_ops);
    uint64_t x = c.seg_max; num("DTGPU_SEG_MAX", 1, 64, x); c.seg_max = uint32_t(std::min<uint64_t>(x, 64));
    x = c.seg_w; num("DTGPU_SEG_W", 0, 1u << 20, x); c.seg_w = uint32_t(x);
    on("DTGPU_SEG_FAIR", c.seg_fair);
    on("DTGPU_SEG_LATE", c.seg_late);
    num("DTGPU_LDS_FILL", 1, UINT64_MAX, c.lds_fill);
    on("DTGPU_FLAT", c.flat);
    on("DTGPU_PLAN_SPLIT", c.plan_split);
    on("DTGPU_PLAN_WALK", c.plan_walk);
    on("DTGPU_PREP_CHAINS", c.prep_chains);
    on("DTGPU_CRITICAL", c.critical);
    on("DTGPU_PRIO", c.prio);
    if (set("DTGPU_HOST_PLAN")) c.host_plan = true;
    if (set("DTGPU_NO_SPLIT")) c.split = false;
    if (set("DTGPU_NO_FALLBACK")) c.fallback = false;
    if (set("DTGPU_NO_WALK_OVERLAP")) c.walk_overlap = false;
    if (const char *e = getenv("DTGPU_DEBUG")) c.debug = uint32_t(atoi(e) ? atoi(e) : 1);
    c.prep_check = c.debug != 0 || set("DTGPU_PREP_CHECK");
    if (set("DTGPU_PASS_MARK")) c.pass_mark = true;
    c.plan_prof = set("DTGPU_PLAN_PROF");
    c.enc_prof = set("DTGPU_ENC_PROF");
    x = c.tog_waves; num("DTGPU_TOG_WAVES", 0, 64, x); c.tog_waves = uint32_t(x);
    x = c.tog_mw_lds; num("DTGPU_TOG_MW_LDS", 0, UINT64_MAX, x); c.tog_mw_lds = uint32_t(std::min<uint64_t>(x, UINT32_MAX));
    x = 0; num("DTGPU_ENC_LDS_TEXT", 0, 24064, x); c.enc_lds_text = uint32_t(x);
    return c;
}
// Per-document replay layout: block capacity, HBM index bytes, LDS tier.
struct Layout { uint32_t max_blocks; uint64_t gidx; int tier; uint32_t tier_blocks; };
Layout replay_layout(uint64_t n_ins, uint64_t lds_fill, bool hbm_only) {
    Layout L{};
    L.max_blocks = uint32_t(n_ins / 32 + 2);
    L.gidx = index_bytes(L.max_blocks);
    const uint32_t est = uint32_t(std::min<uint64_t>(L.max_blocks, n_ins / lds_fill + 8));
    L.tier = hbm_only ? -1 : item_tier(est);
    L.tier_blocks = est;
    return L;
}

// ---- cut replay (dt_replay.hip "segments") ------------------------------------------------------
// A long document replays as segments on several waves, cut at LVs v where the prefix [0, v)
// is one version ({v-1}) and every later entry has it in its history: the reference fast-forwards
// exactly there (merge.rs:811-840) because the text at v is then a plain string.  Cuts go at op
// run starts (every command boundary is one), spread so that the segments hold about equal op
// runs.  A segment's placeholders bound the text at its start: inserts - deletes + the deletes
// that are concurrent with some other op (a delete can hit an already deleted item only then).
struct SegCut { uint32_t lo, hi, u; uint64_t ins; };   // LV range, placeholders, inserted chars in range
struct SegInput {
    uint64_t n_lv = 0;
    std::vector<std::pair<uint64_t, uint64_t>> ent;   // entries [start, end) in LV order
    std::vector<uint32_t> poff;                       // parents CSR (ent.size() + 1)
    std::vector<uint64_t> par;
    std::vector<std::array<uint64_t, 3>> ops;         // op runs (lv, len, kind: 0 ins, 1 del) in LV order
};
struct SegSettings { bool on; uint64_t ops_per_seg; uint32_t max_seg, w_op; };
SegSettings seg_settings(const Settings &c) {
    return SegSettings{c.seg, c.seg_ops, std::min<uint32_t>(c.seg_max, 64), c.seg_w};   // (<= 64: the device cut planning's lane per segment)
}
// Cut ranges [a, b] (every v in them is a cut), in LV order: at entry k ([s, t), parents P)
// the prefix's frontier minus P must be empty (then [0, v) is the version {v-1} for s < v <= t),
// and every later entry's parents must be >= v-1 (so each has v-1 in its history).
std::vector<std::pair<uint64_t, uint64_t>> cut_ranges(const SegInput &in) {
    const size_t ne = in.ent.size();
    std::vector<int64_t> sufmin(ne + 1, INT64_MAX);
    for (size_t k = ne; k-- > 0;) {
        int64_t mp = -1;   // ROOT
        if (in.poff[k + 1] > in.poff[k]) {
            mp = INT64_MAX;
            for (uint32_t j = in.poff[k]; j < in.poff[k + 1]; j++) mp = std::min<int64_t>(mp, int64_t(in.par[j]));
        }
        sufmin[k] = std::min(sufmin[k + 1], mp);
    }
    std::vector<std::pair<uint64_t, uint64_t>> cuts;
    std::set<uint64_t> F;   // frontier of the prefix
    for (size_t k = 0; k < ne; k++) {
        const uint64_t s = in.ent[k].first, t = in.ent[k].second;
        for (uint32_t j = in.poff[k]; j < in.poff[k + 1]; j++) F.erase(in.par[j]);
        if (F.empty()) {
            const int64_t lim = sufmin[k + 1] == INT64_MAX ? int64_t(t) : std::min<int64_t>(int64_t(t), sufmin[k + 1] + 1);
            if (lim >= int64_t(s) + 1) cuts.push_back({s + 1, uint64_t(lim)});
        }
        F.insert(t - 1);
    }
    return cuts;
}
std::vector<SegCut> plan_segments(const SegInput &in, const SegSettings &cfg) {
    std::vector<SegCut> out;
    const size_t ne = in.ent.size(), nop = in.ops.size();
    const uint32_t S = uint32_t(std::min<uint64_t>(cfg.max_seg, nop / cfg.ops_per_seg));
    if (S < 2 || ne == 0 || in.n_lv >= 0x7FFFFFFFull) return out;
    const std::vector<std::pair<uint64_t, uint64_t>> cuts = cut_ranges(in);
    if (cuts.empty()) return out;
    auto in_cut = [&](uint64_t v) {
        auto it = std::upper_bound(cuts.begin(), cuts.end(), std::make_pair(v, UINT64_MAX));
        return it != cuts.begin() && v <= std::prev(it)->second;
    };
    auto linear = [&](uint64_t lv, uint64_t len) {   // every op in [lv, lv+len) is concurrent with nothing
        auto it = std::upper_bound(cuts.begin(), cuts.end(), std::make_pair(lv, UINT64_MAX));
        return it != cuts.begin() && lv + len <= std::prev(it)->second;
    };
    // op-run starts that are cuts, nearest to the op runs where the cost reaches each equal share
    // (SegPlan::w_op, dt_prep.hpp); later cuts a quarter share of the cost past the previous one
    auto cost = [&](size_t j) { return uint64_t(cfg.w_op) * j + in.ops[j][0]; };
    const uint64_t total = uint64_t(cfg.w_op) * nop + in.ops[nop - 1][0] + in.ops[nop - 1][1], q4c = total / (4ull * S);
    std::vector<size_t> pick;
    for (uint32_t k = 1; k < S; k++) {
        const uint64_t tc = uint64_t(k) * total / S;
        size_t lo = 0, hi = nop;   // the first op run whose cost reaches tc
        while (lo < hi) {
            const size_t mid = (lo + hi) / 2;
            if (cost(mid) < tc) lo = mid + 1; else hi = mid;
        }
        const size_t target = lo;
        size_t best = SIZE_MAX;
        for (size_t d = 0; d < nop && best == SIZE_MAX; d++) {
            for (size_t j : {target - std::min(target, d), target + d}) {
                if (j > 0 && j < nop && in_cut(in.ops[j][0])) { best = j; break; }
            }
            if (d > nop / (2 * S)) break;   // no cut near this target
        }
        if (best != SIZE_MAX && (pick.empty() || cost(best) > cost(pick.back()) + q4c)) pick.push_back(best);
    }
    while (!pick.empty() && total - cost(pick.back()) < q4c) pick.pop_back();
    if (pick.empty()) return out;
    // prefix counts at the picked op runs
    int64_t ins = 0, del = 0, dconc = 0;
    size_t pi = 0;
    std::vector<std::array<int64_t, 3>> at(pick.size());
    uint64_t seg_ins = 0;
    std::vector<uint64_t> seg_ins_v;
    for (size_t j = 0; j <= nop; j++) {
        if (pi < pick.size() && j == pick[pi]) { at[pi++] = {ins, del, dconc}; seg_ins_v.push_back(seg_ins); seg_ins = 0; }
        if (j == nop) break;
        const auto &o = in.ops[j];
        if (o[2] == 0) { ins += int64_t(o[1]); seg_ins += o[1]; }
        else { del += int64_t(o[1]); if (!linear(o[0], o[1])) dconc += int64_t(o[1]); }
    }
    seg_ins_v.push_back(seg_ins);
    for (size_t k = 0; k <= pick.size(); k++) {
        SegCut c{};
        c.lo = k ? uint32_t(in.ops[pick[k - 1]][0]) : 0u;
        c.hi = k < pick.size() ? uint32_t(in.ops[pick[k]][0]) : 0xFFFFFFFFu;
        c.u = k ? uint32_t(std::max<int64_t>(0, std::min(at[k - 1][0], at[k - 1][0] - at[k - 1][1] + at[k - 1][2]))) : 0u;
        c.ins = seg_ins_v[k];
        out.push_back(c);
    }
    return out;
}

}  // namespace

struct dtgpu_batch {
    int device = 0;
    int n_cu = 256;
    Settings cfg;   // opts + DTGPU_* overrides, fixed at creation
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev_mid = nullptr, ev1 = nullptr;
    size_t n = 0;
    std::vector<uint32_t> host_status;   // decode / plan status per doc
    std::vector<uint64_t> n_lv;
    std::vector<DocDesc> docs;
    std::vector<uint32_t> tier_list[kLdsTiers], large_list;   // LDS tiers (index bytes), HBM tier
    std::vector<uint8_t> host_planned;   // 0: device-planned; else why the host planned it
    uint32_t tier_blocks[kLdsTiers] = {};
    uint32_t debug = 0;
    hipStream_t side[kSideStreams] = {};   // big LDS tiers run beside the small ones, one stream each
    hipEvent_t ev_fork = nullptr, ev_join[kSideStreams] = {};
    // device-staged split pass: the biggest LDS tier's documents run prep -> plan -> replay on
    // that tier's side stream, beside the other documents' prep and plan (d_split: the big
    // tier's documents, then the rest)
    bool split = false;
    int split_tier = -1;
    uint32_t n_big = 0, n_rest = 0;
    DevBuf<uint32_t> d_split;
    uint64_t alg_in_bytes = 0, total_lv = 0;
    float last_plan_ms = 0, last_replay_ms = 0;

    // device planner inputs (the decoded oplogs) and scratch
    DevBuf<uint32_t> p_par, p_pent, p_pch, p_pcnt, p_child, p_tip, p_erec, p_doff, p_dense;
    DevBuf<Cmd> p_opc;
    DevBuf<uint32_t> p_base;
    DevBuf<uint32_t> p_order;
    DevBuf<uint32_t> p_walk;    // walk_kernel: per document {status, steps}
    DevBuf<uint32_t> pr_chain;   // prep's three-launch pass: per document its stage (dt_prep.hpp)   // two-phase planner: each document's walk order (by entry arena offset)
    DevBuf<PlanDesc> p_docs;
    DevBuf<PlanResult> p_results;
    PlanParams plan{};
    uint32_t n_gpu_planned = 0;

    DevBuf<Cmd> d_cmds;
    DevBuf<uint32_t> d_tlist, d_cbyte, d_aruns, d_pos, d_items, d_lists, d_counter;
    DevBuf<unsigned long long> d_ao, d_m2, d_mup;
    DevBuf<uint32_t> d_tup, d_xf;   // transformed-ops batches only
    bool xf_mode = false;
    DevBuf<uint8_t> d_content, d_out, d_gidx;
    DevBuf<uint32_t> d_fb;   // [0] = count, then the handed-back documents
    DevBuf<DocDesc> d_docs;
    DevBuf<DocResult> d_results;
    BatchParams tier[kLdsTiers]{}, large{};
    // cut replay: segment documents (docs[n..]: a long document's later LV ranges, replayed
    // beside its first one) and the combine step that joins their source lists into its text
    std::vector<uint64_t> seg_cost;
    std::vector<uint64_t> first_cost;   // per document: its first segment's LVs when cut (else 0)
    std::vector<uint64_t> n_runs;       // per document: its op runs (mark_critical)
    std::vector<SegGroup> seg_groups;
    std::vector<uint32_t> seg_docs;
    DevBuf<SegGroup> d_groups;
    DevBuf<uint32_t> d_segdocs, d_src;
    CombineParams comb{};
    // device-staged batches: the cut planning runs in every pass (cut_kernel, dt_prep.hpp); staging
    // only reserves each segment's arenas and uploads its descriptor with a poisoned LV range
    std::vector<SegPlan> seg_plans;
    std::vector<SegCap> seg_caps;
    DevBuf<SegPlan> d_plans;
    DevBuf<SegCap> d_caps;
    DevBuf<uint32_t> d_cutscr;
    CutParams cut{};
    hipEvent_t ev_cut = nullptr;
    hipEvent_t ev_splan = nullptr;   // split pass: the big tier's plans are done (segments may
                                     // replay in another tier, on the main stream)

    // device-staged batches (dtgpu_batch_create_device): the decoded oplogs stay in the
    // decoder's arenas (content and per-LV offsets are read there by the replay) and the
    // planner inputs are built by the prep kernel
    std::unique_ptr<dtgpu_decoded> dec;
    DevBuf<uint32_t> pr_rows, pr_scr;
    DevBuf<PrepDesc> pr_docs;
    DevBuf<PrepResult> pr_res;
    PrepParams prep{};
    hipEvent_t ev_dec = nullptr, ev_prep = nullptr;
    // the planner's walk beside prep's second half: a side stream (idle until the replay), since
    // a process gets GPU_MAX_HW_QUEUES = 4 hardware queues and a fifth stream would share one --
    // serialising two replay tiers that should run side by side
    hipStream_t wstream = nullptr;
    hipEvent_t ev_w0 = nullptr, ev_w1 = nullptr;
    hipStream_t ws_side = nullptr;                    // split pass: the side pipeline's walk
    hipEvent_t ev_sw0 = nullptr, ev_sw1 = nullptr;
    float last_decode_ms = 0, last_prep_ms = 0;

    // linear histories (dt_ff.hip): a document whose history is one graph entry checks out on the
    // fast-forward piece table instead of prep -> plan -> replay (staging still prepares and plans
    // it, for the batched encoder); the pass's prep / plan lists hold the other documents
    std::vector<uint8_t> ff_doc;          // per document: 1 = fast-forward path
    uint32_t n_ff = 0, n_track = 0;       // documents on each path
    DevBuf<uint32_t> d_track;             // the tracker's documents (prep / plan doc_list)
    DevBuf<uint32_t> f_ops;               // host-staged batches: op runs as the decoder's quads
    DevBuf<FFDoc> f_docs;
    DevBuf<FFSeg> f_segs;
    DevBuf<FFPair> f_pairs;
    DevBuf<FFChunk> f_chunks;
    DevBuf<int32_t> f_delta;
    DevBuf<uint32_t> f_bad, f_pa, f_pb, f_ca, f_cb, f_boff;
    FFParams ff{};
    bool pass_mark = false;   // DTGPU_PASS_MARK at staging: every pass opens with pass_mark_kernel

    // batched encoder (dtgpu_batch_encode): per-document descriptors, scratch, output
    std::vector<EncDesc> e_desc;
    std::vector<EncResult> e_res;
    DevBuf<EncDesc> e_docs;
    DevBuf<EncResult> e_dres;
    DevBuf<uint32_t> e_w;
    DevBuf<uint8_t> e_b, e_out;
    EncParams enc{};

    ~dtgpu_batch() {
        if (ev_splan) (void)hipEventDestroy(ev_splan);
        if (ev_cut) (void)hipEventDestroy(ev_cut);
        if (ev_sw0) (void)hipEventDestroy(ev_sw0);
        if (ev_sw1) (void)hipEventDestroy(ev_sw1);
        if (ws_side) (void)hipStreamDestroy(ws_side);
        if (ev_w0) (void)hipEventDestroy(ev_w0);
        if (ev_w1) (void)hipEventDestroy(ev_w1);
        if (ev_dec) (void)hipEventDestroy(ev_dec);
        if (ev_prep) (void)hipEventDestroy(ev_prep);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev_mid) (void)hipEventDestroy(ev_mid);
        if (ev1) (void)hipEventDestroy(ev1);
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        for (int k = 0; k < kSideStreams; k++) {
            if (ev_join[k]) (void)hipEventDestroy(ev_join[k]);
            if (side[k]) (void)hipStreamDestroy(side[k]);
        }
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace {

struct Prepared {
    Status status = OK;
    HostOpLog log;
    PlanInput pi;
    Plan plan;             // host plan: only for documents the device planner declines
    bool host_plan = false;
    std::vector<uint64_t> xf_from, xf_merge;   // transformed-ops batches: the merge to report
    size_t xf_first = 0;                       // first reported command of the plan
};

void prepare_from_oplog(const HostOpLog &src, Prepared &p) {
    p.log = src;
    p.log.finish();
    p.status = build_plan(p.log, p.plan);
}
// Decoded oplog -> device planner input (the walk itself runs on the GPU).
void prepare_input(Prepared &p) {
    if (p.status == OK) p.status = build_plan_input(p.log, p.pi);
}

int threads_for(const dtgpu_batch_opts *opts, size_t n) {
    int t = opts && opts->host_threads > 0 ? opts->host_threads : int(std::thread::hardware_concurrency());
    if (t < 1) t = 1;
    if (size_t(t) > n) t = int(std::max<size_t>(n, 1));
    return t;
}

template <typename F>
void parallel_for(size_t n, int threads, F f) {
    std::atomic<size_t> next{0};
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++)
        pool.emplace_back([&] { for (size_t i; (i = next.fetch_add(1)) < n;) f(i); });
    for (auto &th : pool) th.join();
}

template <typename T>
void append(std::vector<T> &dst, const std::vector<T> &src) { dst.insert(dst.end(), src.begin(), src.end()); }

size_t n_lds_docs(const dtgpu_batch &B) {
    size_t k = 0;
    for (int t = 0; t < kLdsTiers; t++) k += B.tier_list[t].size();
    return k;
}
// Launch order of the documents: the LDS tiers, then the HBM tier; inside a list the documents
// go by descending LVs (a cut document's first segment by its own), so the hardware dispatcher
// starts the longest replays first (LPT inside the GPU: the short ones fill in behind them), the
// critical ones (DOC_CRITICAL) before all.
std::vector<uint32_t> tier_lists(dtgpu_batch &B) {
    std::vector<uint32_t> all;
    auto by_cost = [&](std::vector<uint32_t> &v) {
        auto cost = [&](uint32_t d) -> uint64_t {
            if (B.docs[d].flags & DOC_CRITICAL) return UINT64_MAX;   // the critical path first
            if (d >= B.n) return B.seg_cost[d - B.n];
            return d < B.first_cost.size() && B.first_cost[d] ? B.first_cost[d] : B.n_lv[d];
        };
        std::stable_sort(v.begin(), v.end(), [&](uint32_t a, uint32_t b) { return cost(a) > cost(b); });
        append(all, v);
    };
    for (int t = 0; t < kLdsTiers; t++) by_cost(B.tier_list[t]);
    by_cost(B.large_list);
    return all;
}
dtgpu_status set_tier_params(dtgpu_batch &B, const BatchParams &base) {
    const bool fb = n_lds_docs(B) && B.cfg.fallback;
    size_t off = 0;
    for (int t = 0; t < kLdsTiers; t++) {
        BatchParams &q = B.tier[t];
        q = base;
        q.doc_list = B.d_lists.p + off;
        q.n_list = uint32_t(B.tier_list[t].size());
        q.lds_blocks = B.tier_blocks[t];
        q.lds_sb = lds_sb_capacity(q.lds_blocks);
        q.lds_flat = t == 0 && B.cfg.flat && q.lds_blocks <= FLAT_MAX_BLOCKS ? 1u : 0u;
        q.prio_on = B.cfg.prio ? 1u : 0u;
        q.tog_waves = B.cfg.tog_waves;
        q.tog_mw_lds = B.cfg.tog_mw_lds;
        off += B.tier_list[t].size();
        if (fb) { q.fb_count = B.d_fb.p; q.fb_list = B.d_fb.p + 1; }
    }
    B.large = base;
    B.large.doc_list = B.d_lists.p + off;
    B.large.n_list = uint32_t(B.large_list.size());
    if (fb) {
        B.large.fb_count = B.d_fb.p;
        B.large.fb_list = B.d_fb.p + 1;
        B.large.fb_slots = uint32_t(off);   // every LDS-tier document may be handed back
    }
    for (int t = 0; t < kLdsTiers; t++) B.tier[t].n_cu = uint32_t(B.n_cu);
    B.large.n_cu = uint32_t(B.n_cu);
    B.debug = base.debug;
    if (!B.ev_fork && DTGPU_HIP_FAILED(hipEventCreateWithFlags(&B.ev_fork, hipEventDisableTiming))) return DTGPU_ERR_HIP;
    if (!B.ev_splan && DTGPU_HIP_FAILED(hipEventCreateWithFlags(&B.ev_splan, hipEventDisableTiming))) return DTGPU_ERR_HIP;
    for (int k = 0; k < kSideStreams; k++) {
        if (!B.side[k] && DTGPU_HIP_FAILED(hipStreamCreateWithFlags(&B.side[k], hipStreamNonBlocking))) return DTGPU_ERR_HIP;
        if (!B.ev_join[k] && DTGPU_HIP_FAILED(hipEventCreateWithFlags(&B.ev_join[k], hipEventDisableTiming))) return DTGPU_ERR_HIP;
    }
    return DTGPU_OK;
}
int replay_all(dtgpu_batch *B, hipStream_t s, int skip_tier = -1) {
    ReplayLaunch r{};
    BatchParams tiers[kLdsTiers];
    for (int t = 0; t < kLdsTiers; t++) {
        tiers[t] = B->tier[t];
        if (t == skip_tier) tiers[t].n_list = 0;   // replayed by the split pipeline
    }
    r.lds = tiers;
    r.keep_fb = skip_tier >= 0;
    r.join_side = skip_tier >= 0 ? kLdsTiers - 1 - skip_tier : -1;   // launch_split_side's stream
    r.n_lds = kLdsTiers;
    r.large = &B->large;
    r.stream = s;
    for (int k = 0; k < kSideStreams; k++) { r.side[k] = B->side[k]; r.ev_join[k] = B->ev_join[k]; }
    r.ev_fork = B->ev_fork;
    // split pass: a segment of a big-tier document may sit in a tier replayed from s
    if (skip_tier >= 0 && !B->seg_groups.empty() && hipStreamWaitEvent(s, B->ev_splan, 0) != hipSuccess) return ErrHip;
    const int e = launch_replay(r);
    return e ? e : launch_combine(B->comb, s);   // cut documents: their segments' texts joined
}

// Cut replay inputs from a host oplog (one long document).
void seg_input_from_log(const HostOpLog &o, SegInput &si) {
    si.n_lv = o.n_lv;
    si.poff.push_back(0);
    for (const GraphEntry &g : o.graph.entries) {
        si.ent.push_back({g.start, g.end});
        for (uint64_t p : g.parents) si.par.push_back(p);
        si.poff.push_back(uint32_t(si.par.size()));
    }
    for (const OpRun &r : o.ops) si.ops.push_back({r.lv, r.len, uint64_t(r.kind)});
}
// Add document i's later segments (cuts[1..]) as documents of its replay tier (or the HBM
// tier) and make document i the first segment.  pc_total / blk_total / gidx_total / src_total
// are the arenas' running sizes.
bool add_segments(dtgpu_batch &B, uint32_t i, const std::vector<SegCut> &cuts, int tier, uint32_t,
                  uint64_t lds_fill, uint64_t &pc_total, uint64_t &blk_total, uint64_t &gidx_total, uint64_t &src_total) {
    std::vector<uint32_t> mb(cuts.size(), 0);
    for (size_t k = 1; k < cuts.size(); k++) {
        // placeholders 48 per block, then the inserts -- and at least what the HBM tier's
        // midpoint splits guarantee (every block keeps >= 32 items, so (u + ins) / 32 + 2
        // blocks hold any placement of the inserts among the placeholders)
        const uint64_t m = std::max<uint64_t>((uint64_t(cuts[k].u) + 47) / 48 + cuts[k].ins / 32 + 3,
                                              (uint64_t(cuts[k].u) + cuts[k].ins) / 32 + 3);
        if (m > std::min<uint64_t>(LOC_MAX_BLOCKS, MAX_DOC_BLOCKS)) return false;
        mb[k] = uint32_t(m);
    }
    const SegGroup g{uint32_t(B.seg_docs.size()), uint32_t(cuts.size())};
    {
        DocDesc &d0 = B.docs[i];
        d0.seg_hi = cuts[0].hi;
        d0.src_off = src_total;
        d0.src_cap = uint32_t(cuts[0].ins);
        src_total += cuts[0].ins;
    }
    B.seg_docs.push_back(i);
    if (B.first_cost.size() < B.n) B.first_cost.resize(B.n, 0);
    B.first_cost[i] = std::max<uint64_t>(1, cuts[0].hi);
    const uint64_t n_lv = B.docs[i].n_lv;
    for (size_t k = 1; k < cuts.size(); k++) {
        DocDesc e = B.docs[i];
        e.seg_lo = cuts[k].lo;
        e.seg_hi = cuts[k].hi;
        e.seg_u = cuts[k].u;
        e.pc_off = pc_total;
        pc_total += n_lv + cuts[k].u;
        e.max_blocks = mb[k];
        e.blk_off = blk_total;
        blk_total += mb[k];
        e.gidx_off = gidx_total;
        gidx_total += index_bytes(mb[k]);
        e.src_off = src_total;
        e.src_cap = uint32_t(cuts[k].u + cuts[k].ins);
        src_total += e.src_cap;
        const uint32_t idx = uint32_t(B.docs.size());
        B.docs.push_back(e);
        B.seg_cost.push_back(cuts[k].hi == 0xFFFFFFFFu ? n_lv - cuts[k].lo : cuts[k].hi - cuts[k].lo);
        B.seg_docs.push_back(idx);
        // its own replay tier, sized for its placeholders and inserts, never above its
        // document's: a split pass replays the biggest tier beside the other documents' plans,
        // so a segment may sit there only when its document is planned there too (the main
        // stream waits for the big tier's plans before replaying any tier: see replay_all); a
        // document on the HBM tier keeps its segments there
        const Layout lay = replay_layout(cuts[k].u + cuts[k].ins, lds_fill, false);
        if (tier >= 0 && lay.tier >= 0 && lay.tier <= tier) {
            const uint32_t est = std::max<uint32_t>(lay.tier_blocks, uint32_t((uint64_t(cuts[k].u) + 47) / 48 + 8));
            B.tier_list[lay.tier].push_back(idx);
            B.tier_blocks[lay.tier] = std::max(B.tier_blocks[lay.tier], std::min(est, mb[k]));
        } else {
            B.large_list.push_back(idx);
        }
    }
    B.seg_groups.push_back(g);
    return true;
}
// Which documents of a batch replay as segments, and how long a segment is: a document is cut
// when it holds at least two segments' worth of op runs, where a segment is DTGPU_SEG_OPS op
// runs or the batch's fair share per wave slot (all op runs over 8 waves per CU), whichever is
// more -- a batch of many equal documents already fills the GPU and is left alone.
template <typename NOps>
std::vector<uint32_t> seg_candidates(size_t n, SegSettings &sc, int n_cu, bool fair, NOps n_ops) {
    std::vector<uint32_t> c;
    if (!sc.on) return c;
    uint64_t total = 0;
    for (size_t i = 0; i < n; i++) total += n_ops(i);
    if (fair) sc.ops_per_seg = std::max<uint64_t>(sc.ops_per_seg, total / (uint64_t(std::max(n_cu, 1)) * 8));
    for (size_t i = 0; i < n; i++)
        if (n_ops(i) >= 2 * sc.ops_per_seg) c.push_back(uint32_t(i));
    return c;
}
// The documents the smallest LDS tier dispatches after its first resident round (its list runs
// longest first, so these are its shortest): they start when the first round's documents begin
// to finish and would run to the end of the batch at low occupancy; each is cut once where its
// history allows, so its two halves finish earlier beside each other.  (Device-staged batches:
// the pass itself plans the cut, cut_kernel.)
template <typename NOps>
std::vector<uint8_t> late_documents(const dtgpu_batch &B, const SegSettings &sc, NOps n_ops) {
    std::vector<uint8_t> late(B.n, 0);
    if (!sc.on || !B.cfg.seg_late || B.tier_list[0].empty() || !B.cfg.flat || B.tier_blocks[0] > FLAT_MAX_BLOCKS) return late;
    const size_t lds = size_t(flat_index_bytes(B.tier_blocks[0]));
    const size_t gran = (lds + 1279) / 1280 * 1280;
    const size_t resident = std::min<size_t>(32, 163840 / std::max<size_t>(gran, 1280)) * size_t(std::max(B.n_cu, 1));
    std::vector<uint32_t> order(B.tier_list[0].begin(), B.tier_list[0].end());
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return B.n_lv[a] > B.n_lv[b]; });
    // (a batch of many rounds: its last round's worth, the documents that end the batch)
    const size_t from = std::max(resident, order.size() > resident ? order.size() - resident : size_t(0));
    for (size_t k = from; k < order.size(); k++)
        if (order[k] < B.n && n_ops(order[k]) >= 128) late[order[k]] = 1;
    return late;
}
// The batch's critical replays (DOC_CRITICAL): a batch whose longest replay unit -- a document
// replayed whole, by the cut planner's cost (SEG_W_OP per op run + LVs); a segment, by its
// document's cost over its segment count -- is at
// least 3x the median gives the units within half of it the top wave priority, as long as they are
// at most an eighth of the units (mixed batches: git-makefile's 50 uncut documents among 1,500
// segments and documents; a batch of equal documents marks none).  DTGPU_CRITICAL=0: off.
void mark_critical(dtgpu_batch &B) {
    for (DocDesc &d : B.docs) d.flags &= ~DOC_CRITICAL;
    if (!B.cfg.critical || B.docs.size() < 2) return;
    std::vector<uint32_t> per(B.docs.size(), 1);   // segments of each unit's document
    for (const SegGroup &g : B.seg_groups)
        for (uint32_t k = 0; k < g.count; k++) per[B.seg_docs[g.first + k]] = g.count;
    std::vector<uint32_t> owner(B.docs.size());   // a segment document's document
    for (size_t d = 0; d < B.docs.size(); d++) owner[d] = uint32_t(d);
    for (const SegGroup &g : B.seg_groups)
        for (uint32_t k = 1; k < g.count; k++) owner[B.seg_docs[g.first + k]] = B.seg_docs[g.first];
    std::vector<double> cost;   // replay units (fast-forwarded documents do not replay)
    std::vector<uint32_t> unit;
    for (size_t i = 0; i < B.docs.size(); i++) {
        if (B.docs[i].flags & DOC_FF) continue;
        const size_t o = owner[i];
        const double runs = o < B.n_runs.size() ? double(B.n_runs[o]) : 0.0;
        cost.push_back((double(SEG_W_OP) * runs + double(B.docs[i].n_lv)) / per[i]);
        unit.push_back(uint32_t(i));
    }
    if (cost.size() < 2) return;
    std::vector<double> srt = cost;
    std::nth_element(srt.begin(), srt.begin() + srt.size() / 2, srt.end());
    const double med = srt[srt.size() / 2], mx = *std::max_element(cost.begin(), cost.end());
    if (mx < 3.0 * med) return;
    size_t n = 0;
    for (double c : cost) n += c >= mx / 2;
    if (8 * n > cost.size()) return;
    for (size_t k = 0; k < cost.size(); k++)
        if (cost[k] >= mx / 2) B.docs[unit[k]].flags |= DOC_CRITICAL;
}
// The batch's combine step and source-list arena (after every add_segments).
hipError_t finish_segments(dtgpu_batch &B, uint64_t src_total, const uint32_t *cbyte, const uint8_t *content, hipStream_t s) {
    hipError_t e = hipSuccess;
    if ((e = B.d_src.alloc(std::max<uint64_t>(src_total, 1))) != hipSuccess) return e;
    if (!B.seg_groups.empty()) {
        if ((e = B.d_groups.upload(B.seg_groups, s)) != hipSuccess || (e = B.d_segdocs.upload(B.seg_docs, s)) != hipSuccess) return e;
    }
    CombineParams &c = B.comb;
    c.groups = B.d_groups.p;
    c.seg_docs = B.d_segdocs.p;
    c.n_groups = uint32_t(B.seg_groups.size());
    c.docs = B.d_docs.p;
    c.results = B.d_results.p;
    c.src = B.d_src.p;
    c.cbyte = cbyte;
    c.content = content;
    c.out = B.d_out.p;
    c.n_cu = uint32_t(B.n_cu);
    return hipSuccess;
}

// ---- linear histories (dt_ff.hip) ---------------------------------------------------------------
// A document checks out on the fast-forward path when its whole history is one graph entry: the
// reference's merge then fast-forwards through every op (merge.rs:811-840; Graph::push extends
// the last entry whenever a span continues it, so one entry <=> a linear history).
struct FFIn { uint64_t op_off; uint32_t n_ops; uint32_t doc; };   // op runs: quads into `ops`
// The fast-forward layout of the batch's linear documents: segments of FF_RUNS op runs, the
// composition pairs of every level, the copy chunks.  out_off / out_cap / lv_off / content_off /
// ascii come from B.docs (the documents' normal layout); the tracker documents become the
// pass's prep / plan list.
hipError_t stage_ff(dtgpu_batch &B, const std::vector<FFIn> &in, const uint32_t *ops, const uint32_t *cbyte,
                    const uint8_t *content, hipStream_t s) {
    hipError_t e = hipSuccess;
    B.pass_mark = B.cfg.pass_mark;   // (profiling runs: tools/traffic.py)
    std::vector<uint32_t> track;
    for (size_t i = 0; i < B.n; i++)
        if (!B.ff_doc[i]) track.push_back(uint32_t(i));
    B.n_track = uint32_t(track.size());
    B.n_ff = uint32_t(in.size());
    if ((e = B.d_track.upload(track, s)) != hipSuccess) return e;
    B.prep.doc_list = B.d_track.p;
    B.prep.n_docs = B.n_track;
    B.plan.doc_list = B.d_track.p;
    B.plan.n_docs = B.n_track;
    if (in.empty()) return hipSuccess;
    std::vector<FFDoc> docs;
    std::vector<FFSeg> segs;
    std::vector<std::vector<FFPair>> lv;
    std::vector<FFChunk> chunks;
    for (const FFIn &f : in) {
        const DocDesc &d = B.docs[f.doc];
        FFDoc q{};
        q.op_off = f.op_off;
        q.lv_off = d.lv_off;
        q.content_off = d.content_off;
        q.out_off = d.out_off;
        q.n_ops = f.n_ops;
        q.first_seg = uint32_t(segs.size());
        q.n_seg = (f.n_ops + FF_RUNS - 1) / FF_RUNS;
        q.piece_off = uint64_t(FF_PIECES) * q.first_seg;
        q.out_cap = d.out_cap;
        q.result = f.doc;
        q.ascii = d.ascii;
        while ((1u << q.levels) < q.n_seg) q.levels++;
        const uint32_t di = uint32_t(docs.size());
        for (uint32_t k = 0; k < q.n_seg; k++)
            segs.push_back(FFSeg{di, k * FF_RUNS, std::min<uint32_t>(FF_RUNS, f.n_ops - k * FF_RUNS), 0});
        if (lv.size() < q.levels) lv.resize(q.levels);
        for (uint32_t k = 0; k < q.levels; k++) {
            const uint32_t g = 1u << k;
            for (uint32_t a = 0; a < q.n_seg; a += 2 * g) lv[k].push_back(FFPair{di, a, a + g < q.n_seg ? a + g : FF_NONE, 0});
        }
        for (uint64_t c = 0; c < d.out_cap; c += FF_CHUNK) chunks.push_back(FFChunk{di, uint32_t(c)});
        docs.push_back(q);
    }
    if (lv.size() > 32) return hipErrorInvalidValue;
    FFParams &p = B.ff;
    p = FFParams{};
    std::vector<FFPair> pairs;
    for (size_t k = 0; k < lv.size(); k++) {
        p.level_off[k] = uint32_t(pairs.size());
        append(pairs, lv[k]);
    }
    p.level_off[lv.size()] = uint32_t(pairs.size());
    const size_t slots = size_t(FF_PIECES) * segs.size();
    if ((e = B.f_docs.upload(docs, s)) != hipSuccess || (e = B.f_segs.upload(segs, s)) != hipSuccess ||
        (e = B.f_pairs.upload(pairs, s)) != hipSuccess || (e = B.f_chunks.upload(chunks, s)) != hipSuccess ||
        (e = B.f_delta.alloc(segs.size())) != hipSuccess || (e = B.f_bad.alloc(docs.size())) != hipSuccess ||
        (e = B.f_pa.alloc(4 * slots)) != hipSuccess || (e = B.f_pb.alloc(4 * slots)) != hipSuccess ||
        (e = B.f_ca.alloc(segs.size())) != hipSuccess || (e = B.f_cb.alloc(segs.size())) != hipSuccess ||
        (e = B.f_boff.alloc(slots)) != hipSuccess)
        return e;
    p.ops = ops;
    p.cbyte = cbyte;
    p.content = content;
    p.out = B.d_out.p;
    p.results = B.d_results.p;
    p.docs = B.f_docs.p;
    p.segs = B.f_segs.p;
    p.pairs = B.f_pairs.p;
    p.chunks = B.f_chunks.p;
    p.n_docs = uint32_t(docs.size());
    p.n_segs = uint32_t(segs.size());
    p.n_chunks = uint32_t(chunks.size());
    p.n_levels = uint32_t(lv.size());
    p.delta = B.f_delta.p;
    p.bad = B.f_bad.p;
    p.pa = B.f_pa.p; p.pb = B.f_pb.p;
    p.ca = B.f_ca.p; p.cb = B.f_cb.p;
    p.boff = B.f_boff.p;
    return hipSuccess;
}

// xf: a transformed-ops batch (iter_xf_operations): host plans in TransformedOpsIter order
// (build_xf_plan), every document on the HBM-index tier, never-deleted masks / totals and the
// per-LV transformed-position arena allocated.
dtgpu_status stage(std::vector<Prepared> &prep, const dtgpu_batch_opts *opts, dtgpu_batch **out, bool xf = false) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return DTGPU_ERR_NO_DEVICE;
    auto B = std::make_unique<dtgpu_batch>();
    B->cfg = settings_for(opts);
    B->device = opts ? opts->device : 0;
#define CK(x) do { if (DTGPU_HIP_FAILED(x)) return DTGPU_ERR_HIP; } while (0)
    CK(hipSetDevice(B->device));
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, B->device) == hipSuccess && prop.multiProcessorCount > 0)
        B->n_cu = prop.multiProcessorCount;
    CK(hipStreamCreateWithFlags(&B->stream, hipStreamNonBlocking));
    CK(hipEventCreate(&B->ev0)); CK(hipEventCreate(&B->ev_mid)); CK(hipEventCreate(&B->ev1)); CK(hipEventCreate(&B->ev_prep));
    hipStream_t s = B->stream;
    const size_t n = prep.size();
    const int threads = threads_for(opts, n);
    B->n = n;
    B->host_status.resize(n);
    B->n_lv.resize(n);
    B->n_runs.assign(n, 0);
    B->docs.resize(n);
    B->host_planned.assign(n, 0);
    B->ff_doc.assign(n, 0);
    const bool force_host = xf || B->cfg.host_plan;

    // ---- 1. device planner inputs; a sizing pass of the planner gives exact stream sizes ----
    std::vector<PlanDesc> pdesc(n);
    {
        std::vector<uint32_t> par, pent, pch, pcnt, child, tip, aruns, erec, doff, dense, base_rows;
        std::vector<Cmd> opc;
        uint64_t base_total = 0, n_entries = 0;
        uint32_t lds_entries = 0, max_agents = 0;
        for (size_t i = 0; i < n; i++) {
            Prepared &p = prep[i];
            PlanDesc &q = pdesc[i];
            std::memset(&q, 0, sizeof q);
            q.skip = 1;
            if (p.status != OK) continue;
            const PlanInput &pi = p.pi;
            const uint64_t ne = pi.est.size() / 2;
            const bool host = force_host || !pi.device_ok || pi.n_chains > PLAN_MAX_AGENTS ||
                              ne > PLAN_MAX_LDS_ENTRIES || ne * std::max<uint32_t>(pi.n_chains, 1) > (64ull << 20);
            if (host) p.host_plan = true;
            q.skip = host ? 1 : 0;
            q.e_off = n_entries;
            q.par_off = par.size();
            q.child_off = child.size();
            q.op_off = opc.size();
            q.arun_off = aruns.size() / 4;
            q.tip_off = tip.size() / 2;
            q.erec_off = erec.size();
            q.doff_off = doff.size();
            q.dense_off = dense.size();
            q.base_off = base_total;
            q.prow_off = base_total;   // host-staged: the base rows arrive filled (build_plan_input)
            q.row_stride = pi.n_chains;
            q.ne = uint32_t(ne);
            q.n_agents = pi.n_chains;
            q.n_aruns = uint32_t(pi.aruns.size() / 4);
            q.ntip = uint32_t(pi.tip.size() / 2);
            q.n_lv = uint32_t(p.log.n_lv);
            append(aruns, pi.aruns);   // also the replay's tie-break runs
            if (host) continue;
            append(par, pi.par); append(pent, pi.pent); append(pch, pi.pch); append(pcnt, pi.pcnt);
            append(child, pi.child); append(opc, pi.opc);
            append(tip, pi.tip); append(erec, pi.erec); append(doff, pi.doff); append(dense, pi.dense);
            if (pi.prow.size() == ne * pi.n_chains) append(base_rows, pi.prow);
            else base_rows.resize(base_rows.size() + ne * pi.n_chains, 0);
            base_total += ne * pi.n_chains;
            n_entries += ne;
            lds_entries = std::max<uint32_t>(lds_entries, uint32_t(ne));
            max_agents = std::max<uint32_t>(max_agents, pi.n_chains);
        }
        CK(B->p_par.upload(par, s)); CK(B->p_pent.upload(pent, s)); CK(B->p_child.upload(child, s));
        CK(B->p_pch.upload(pch, s)); CK(B->p_pcnt.upload(pcnt, s));
        CK(B->p_opc.upload(opc, s)); CK(B->d_aruns.upload(aruns, s)); CK(B->p_tip.upload(tip, s));
        CK(B->p_erec.upload(erec, s)); CK(B->p_doff.upload(doff, s)); CK(B->p_dense.upload(dense, s));
        CK(B->p_base.upload(base_rows, s));
        CK(B->p_order.alloc(std::max<size_t>(erec.size() / EREC_WORDS, 1)));
        CK(B->p_walk.alloc(2 * std::max<size_t>(n, 1)));
        CK(B->p_docs.upload(pdesc, s));
        CK(B->p_results.alloc(n));
        CK(hipMemsetAsync(B->p_results.p, 0, std::max<size_t>(n, 1) * sizeof(PlanResult), s));
        PlanParams &q = B->plan;
        q.par = B->p_par.p; q.pent = B->p_pent.p; q.pch = B->p_pch.p; q.pcnt = B->p_pcnt.p;
        q.child = B->p_child.p; q.opc = B->p_opc.p;
        q.aruns = B->d_aruns.p; q.tip = B->p_tip.p; q.erec = B->p_erec.p; q.doff = B->p_doff.p;
        q.dense = B->p_dense.p; q.base = B->p_base.p; q.prow = B->p_base.p; q.order = B->p_order.p;
        q.walk = B->cfg.plan_walk ? B->p_walk.p : nullptr;
        q.split = B->cfg.plan_split ? 1u : 0u;
        q.lds_entries = (lds_entries + 7) & ~7u;
        q.max_agents = max_agents;
        q.prof = B->cfg.plan_prof ? 1u : 0u;
        q.docs = B->p_docs.p; q.results = B->p_results.p; q.n_docs = uint32_t(n);
        q.count_only = 1;
        if (launch_plan(q, s) != OK) { DTGPU_HIP_FAILED(hipErrorLaunchFailure); return DTGPU_ERR_HIP; }
        q.count_only = 0;
    }
    std::vector<PlanResult> pres(n);
    CK(hipMemcpyAsync(pres.data(), B->p_results.p, std::max<size_t>(n, 1) * sizeof(PlanResult), hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    // documents the device planner declined are planned on the host
    std::vector<uint8_t> reason(n, 0);
    for (size_t i = 0; i < n; i++) {
        if (prep[i].status != OK) continue;
        if (pdesc[i].skip) reason[i] = force_host ? 1 : 2;
        else if (pres[i].status != PLAN_OK) { prep[i].host_plan = true; reason[i] = uint8_t(16 + pres[i].status); }
    }
    parallel_for(n, threads, [&](size_t i) {
        Prepared &p = prep[i];
        if (p.status == OK && p.host_plan)
            p.status = xf ? build_xf_plan_from(p.log, p.xf_from, p.xf_merge, p.plan, p.xf_first) : build_plan(p.log, p.plan);
    });

    // ---- 2. per-document layout ---------------------------------------------------------------
    std::vector<Cmd> hcmds;     // host plans, at their documents' offsets
    std::vector<uint32_t> htlist, cbyte;
    std::vector<uint8_t> content;
    uint64_t cmd_total = 0, tlist_total = 0;
    uint64_t lv_total = 0, blk_total = 0, out_total = 0, gidx_total = 0;
    // expected inserted chars per block in the LDS tier (per tracker); DTGPU_LDS_FILL overrides it
    // for experiments (a document that outgrows its LDS index replays on the HBM tier)
    const uint64_t lds_fill = B->cfg.lds_fill;
    std::vector<int> seg_tier(n, -2);          // replay tier per document (-2: not replayed)
    std::vector<uint32_t> seg_est(n, 0);
    for (size_t i = 0; i < n; i++) {
        Prepared &p = prep[i];
        B->host_status[i] = p.status;
        B->n_lv[i] = p.log.n_lv;
        B->n_runs[i] = p.log.ops.size();
        B->total_lv += p.log.n_lv;
        DocDesc &d = B->docs[i];
        std::memset(&d, 0, sizeof d);
        d.seg_hi = 0xFFFFFFFFu;   // not a segment (cut replay)
        d.src_off = ~0ull;
        const uint64_t aq = p.pi.aruns.size() / 4;
        d.arun_off = pdesc[i].arun_off * 4;
        if (p.status != OK) { pdesc[i].skip = 1; continue; }
        uint64_t n_ins = 0;
        for (const OpRun &r : p.log.ops) if (r.kind == 0) n_ins += r.len;
        if (n_ins / 32 + 2 > std::min<uint64_t>(LOC_MAX_BLOCKS, MAX_DOC_BLOCKS)) { B->host_status[i] = ErrCapacity; pdesc[i].skip = 1; continue; }
        d.cmd_off = cmd_total;
        d.tlist_off = tlist_total;
        if (p.host_plan) {
            B->host_planned[i] = reason[i] ? reason[i] : 2;
            pdesc[i].skip = 1;
            d.ncmd = uint32_t(p.plan.cmds.size());
            hcmds.resize(cmd_total);
            htlist.resize(tlist_total);
            append(hcmds, p.plan.cmds);
            append(htlist, p.plan.tlist);
            cmd_total += p.plan.cmds.size();
            tlist_total += p.plan.tlist.size();
        } else {
            d.ncmd = pres[i].ncmd;
            pdesc[i].cmd_off = cmd_total;
            pdesc[i].tlist_off = tlist_total;
            pdesc[i].ccap = pres[i].ncmd;
            pdesc[i].tcap = pres[i].ntlist;
            cmd_total += pres[i].ncmd;
            tlist_total += pres[i].ntlist;
            B->n_gpu_planned++;
        }
        d.ascii = p.log.ins_content.size() == n_ins ? 1u : 0u;
        d.lv_off = lv_total;
        d.pc_off = lv_total;
        d.n_lv = uint32_t(p.log.n_lv);
        d.content_off = content.size();
        d.content_len = uint32_t(p.log.ins_content.size());
        d.n_aruns = uint32_t(aq);
        if (!xf && B->cfg.ff && p.log.graph.entries.size() == 1 && !p.log.ops.empty() && p.log.content_complete) {
            // a linear history: the fast-forward path (dt_ff.hip), out arena only
            B->ff_doc[i] = 1;
            d.flags |= DOC_FF;
            out_total = (out_total + 15) & ~15ull;
            d.out_off = out_total;
            d.out_cap = uint32_t(p.log.ins_content.size());
            out_total += (uint64_t(d.out_cap) + 15) & ~15ull;
            cbyte.insert(cbyte.end(), p.log.ins_cbyte.begin(), p.log.ins_cbyte.end());
            content.insert(content.end(), p.log.ins_content.begin(), p.log.ins_content.end());
            lv_total += p.log.n_lv;
            uint64_t parents = 0;
            for (const GraphEntry &g : p.log.graph.entries) parents += g.parents.size();
            B->alg_in_bytes += 16ull * p.log.ops.size() + 8ull * p.log.graph.entries.size() + 4ull * parents +
                               12ull * p.log.agent_runs.size() + d.content_len;
            continue;
        }
        const Layout lay = replay_layout(n_ins, lds_fill, xf);
        d.max_blocks = lay.max_blocks;
        d.blk_off = blk_total;
        d.out_off = out_total;
        d.out_cap = uint32_t(p.log.ins_content.size());
        cbyte.insert(cbyte.end(), p.log.ins_cbyte.begin(), p.log.ins_cbyte.end());
        content.insert(content.end(), p.log.ins_content.begin(), p.log.ins_content.end());
        lv_total += p.log.n_lv;
        blk_total += d.max_blocks;
        out_total += d.out_cap;
        // compulsory input bytes of the decoded oplog (SURVEY.md §8d merge-only formula):
        // 16 per op run + (8 + 4 per parent) per graph entry + 12 per agent run + inserted
        // bytes; the text written is added from the results (dtgpu_batch_algorithmic_bytes)
        uint64_t parents = 0;
        for (const GraphEntry &g : p.log.graph.entries) parents += g.parents.size();
        B->alg_in_bytes += 16ull * p.log.ops.size() + 8ull * p.log.graph.entries.size() + 4ull * parents +
                           12ull * p.log.agent_runs.size() + d.content_len;
        // every document gets an HBM index (the LDS tier hands back documents that outgrow
        // their optimistic LDS capacity); the LDS tier is sized from the expected block fill
        d.gidx_off = gidx_total;
        gidx_total += lay.gidx;
        const int t = lay.tier;
        seg_tier[i] = t;
        seg_est[i] = lay.tier_blocks;
        if (t >= 0) {
            B->tier_list[t].push_back(uint32_t(i));
            B->tier_blocks[t] = std::max(B->tier_blocks[t], lay.tier_blocks);
        } else {
            B->large_list.push_back(uint32_t(i));
        }
    }
    // host-planned documents' agent runs are not in the planner arrays: append them
    {
        std::vector<uint32_t> extra;
        uint64_t base_q = B->d_aruns.n / 4;
        for (size_t i = 0; i < n; i++) {
            if (!B->host_planned[i]) continue;
            B->docs[i].arun_off = (base_q + extra.size() / 4) * 4;
            append(extra, prep[i].pi.aruns.empty() ? prep[i].plan.agent_runs : prep[i].pi.aruns);
        }
        if (!extra.empty()) {
            std::vector<uint32_t> all(B->d_aruns.n);
            if (B->d_aruns.n)
                CK(hipMemcpyAsync(all.data(), B->d_aruns.p, all.size() * 4, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            append(all, extra);
            DevBuf<uint32_t> fresh;
            CK(fresh.upload(all, s));
            std::swap(B->d_aruns.p, fresh.p);
            std::swap(B->d_aruns.n, fresh.n);
            B->plan.aruns = B->d_aruns.p;
        }
    }
    // cut replay: long documents' later LV ranges as documents of their own
    uint64_t pc_total = lv_total, src_total = 0;
    if (!xf) {
        SegSettings sc = seg_settings(B->cfg);
        for (uint32_t i : seg_candidates(n, sc, B->n_cu, B->cfg.seg_fair, [&](size_t k) { return seg_tier[k] != -2 ? prep[k].log.ops.size() : 0; })) {
            SegInput si;
            seg_input_from_log(prep[i].log, si);
            const std::vector<SegCut> cuts = plan_segments(si, sc);
            if (cuts.size() >= 2)
                add_segments(*B, i, cuts, seg_tier[i], seg_est[i], lds_fill, pc_total, blk_total, gidx_total, src_total);
        }
    }
    hcmds.resize(cmd_total);
    htlist.resize(tlist_total);
    CK(B->d_cmds.upload(hcmds, s));
    CK(B->d_tlist.upload(htlist, s));
    CK(B->p_docs.upload(pdesc, s));
    B->plan.docs = B->p_docs.p;
    B->plan.cmds = B->d_cmds.p;
    B->plan.tlist = B->d_tlist.p;
    CK(B->d_cbyte.upload(cbyte, s));
    CK(B->d_content.upload(content, s));
    mark_critical(*B);
    CK(B->d_docs.upload(B->docs, s));
    CK(B->d_lists.upload(tier_lists(*B), s));
    CK(B->d_pos.alloc(pc_total));
    CK(B->d_ao.alloc(pc_total));
    CK(B->d_items.alloc(blk_total * 64));
    CK(B->d_m2.alloc(2 * blk_total));
    CK(B->d_out.alloc(out_total));
    CK(B->d_gidx.alloc(gidx_total));
    CK(B->d_fb.alloc(n_lds_docs(*B) + 1));
    CK(B->d_counter.alloc(2));
    CK(B->d_results.alloc(B->docs.size()));
    CK(hipMemsetAsync(B->d_results.p, 0, std::max<size_t>(B->docs.size(), 1) * sizeof(DocResult), s));
    CK(finish_segments(*B, src_total, B->d_cbyte.p, B->d_content.p, s));
    {   // linear documents: their op runs as the decoder's quads (lv, len, pos, kind | fwd << 1)
        std::vector<FFIn> ffin;
        std::vector<uint32_t> quads;
        for (size_t i = 0; i < n; i++) {
            if (!B->ff_doc[i]) continue;
            ffin.push_back(FFIn{quads.size() / 4, uint32_t(prep[i].log.ops.size()), uint32_t(i)});
            for (const OpRun &r : prep[i].log.ops)
                quads.insert(quads.end(), {uint32_t(r.lv), uint32_t(r.len), uint32_t(r.pos), uint32_t(r.kind) | (uint32_t(r.fwd) << 1)});
        }
        CK(B->f_ops.upload(quads, s));
        CK(stage_ff(*B, ffin, B->f_ops.p, B->d_cbyte.p, B->d_content.p, s));
    }
    if (xf) {
        CK(B->d_mup.alloc(blk_total));
        CK(B->d_tup.alloc(blk_total + 2 * n));
        CK(B->d_xf.alloc(lv_total));
    }
    CK(hipStreamSynchronize(s));
#undef CK
    BatchParams base{};
    B->xf_mode = xf;
    base.mup = B->d_mup.p;
    base.tup = B->d_tup.p;
    base.xf = B->d_xf.p;
    base.debug = B->cfg.debug;
    base.cmds = B->d_cmds.p;
    base.tlist = B->d_tlist.p;
    base.cbyte = B->d_cbyte.p;
    base.content = B->d_content.p;
    base.aruns = B->d_aruns.p;
    base.pos = B->d_pos.p;
    base.ao = B->d_ao.p;
    base.items = B->d_items.p;
    base.m2 = B->d_m2.p;
    base.out = B->d_out.p;
    base.gidx = B->d_gidx.p;
    base.docs = B->d_docs.p;
    base.results = B->d_results.p;
    base.src = B->d_src.p;
    if (set_tier_params(*B, base) != DTGPU_OK) { DTGPU_HIP_FAILED(hipErrorUnknown); return DTGPU_ERR_HIP; }
    *out = B.release();
    return DTGPU_OK;
}

// Device-staged batch: `.dt` bytes -> device decode -> device prep -> planner sizing pass ->
// replay layout.  The host only reads back per-document counts to size the arenas.  Documents
// the device path hands back (decoder or prep limits) get status DTGPU_DECODE_DEFER.
// `dec` is a decoded handle (dtgpu_decode_create: decoded here; dtgpu_decode_add: already merged).
dtgpu_status stage_device(dtgpu_decoded *dec, const dtgpu_batch_opts *opts, dtgpu_batch **out) {
    auto B = std::make_unique<dtgpu_batch>();
    B->cfg = settings_for(opts);
    B->device = dec->device;
    B->dec.reset(dec);
    dtgpu_decoded &Dd = *B->dec;
    const size_t n = Dd.n;
    if (hipSetDevice(B->device) != hipSuccess) return DTGPU_ERR_HIP;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, B->device) == hipSuccess && prop.multiProcessorCount > 0)
        B->n_cu = prop.multiProcessorCount;
    B->stream = Dd.stream;   // one stream for decode, prep, plan and replay
    Dd.stream = nullptr;     // owned by the batch from here on
#define CK(x) do { if (DTGPU_HIP_FAILED(x)) return DTGPU_ERR_HIP; } while (0)
    CK(hipEventCreate(&B->ev0)); CK(hipEventCreate(&B->ev_mid)); CK(hipEventCreate(&B->ev1));
    CK(hipEventCreate(&B->ev_dec)); CK(hipEventCreate(&B->ev_prep));
    CK(hipEventCreateWithFlags(&B->ev_w0, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&B->ev_w1, hipEventDisableTiming));
    hipStream_t s = B->stream;
    if (!Dd.merged) {
        if (launch_decode(Dd.P, s)) return DTGPU_ERR_HIP;
        CK(hipMemcpyAsync(Dd.res.data(), Dd.d_res.p, n * sizeof(DecodeResult), hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    }
    stage_prof("stage: decode pass");
    B->n = n;
    B->host_status.assign(n, OK);
    B->n_lv.assign(n, 0);
    B->n_runs.assign(n, 0);
    B->docs.assign(n, DocDesc{});
    B->host_planned.assign(n, 0);
    B->ff_doc.assign(n, 0);
    const bool ff_on = B->cfg.ff;

    // ---- prep layout ----------------------------------------------------------------------------
    std::vector<PrepDesc> pd(n);
    uint64_t o_par = 0, o_op = 0, o_arun = 0, o_tip = 0, o_erec = 0, o_doff = 0, o_dense = 0, o_rows = 0, o_scr = 0;
    uint32_t max_e = 1;
    for (size_t i = 0; i < n; i++) {
        const DecodeResult &r = Dd.res[i];
        const DecodeDesc &d = Dd.desc[i];
        PrepDesc &q = pd[i];
        std::memset(&q, 0, sizeof q);
        q.skip = 1;
        uint32_t st = r.status;
        if (st == OK && !r.content_complete) st = ErrCheckout;   // content.unwrap() in apply_to
        if (st == OK && (r.n_lv >= MAX_PLAN_LV || r.n_entries > PLAN_MAX_LDS_ENTRIES)) st = DECODE_DEFER;
        B->host_status[i] = st;
        B->n_lv[i] = r.n_lv;
        B->n_runs[i] = r.n_ops;
        if (st != OK) continue;
        if (ff_on && r.n_entries == 1 && r.n_ops > 0) B->ff_doc[i] = 1;   // linear history (dt_ff.hip)
        q.skip = 0;
        q.d_op = d.op_off; q.d_arun = d.arun_off; q.d_ent = d.ent_off; q.d_poff = d.poff_off; q.d_par = d.par_off;
        q.d_ver = d.ver_off; q.d_agent = d.agent_off; q.d_in = d.in_off;
        q.n_ops = r.n_ops; q.n_aruns = r.n_aruns; q.ne = r.n_entries; q.n_par = r.n_parents; q.n_ver = r.n_version;
        q.n_agents = r.n_agents; q.n_lv = uint32_t(r.n_lv);
        q.o_par = o_par; o_par += r.n_parents;
        q.o_child = q.o_par;
        q.o_op = o_op; o_op += r.n_ops;
        q.o_arun = o_arun; o_arun += r.n_aruns;
        q.o_tip = o_tip; o_tip += r.n_version;
        q.o_erec = o_erec; o_erec += uint64_t(EREC_WORDS) * r.n_entries;
        q.o_doff = o_doff; o_doff += PREP_MAX_CHAINS + 1;
        q.o_dense = o_dense; o_dense += r.n_lv;
        q.o_rows = o_rows; o_rows += uint64_t(PREP_MAX_CHAINS) * r.n_entries;
        q.row_stride = PREP_MAX_CHAINS;
        q.o_scr = o_scr; o_scr += prep_scratch_words(r.n_parents, r.n_entries);
        max_e = std::max<uint32_t>(max_e, r.n_entries);
    }
    CK(B->p_par.alloc(o_par)); CK(B->p_pent.alloc(o_par)); CK(B->p_pch.alloc(o_par)); CK(B->p_pcnt.alloc(o_par));
    CK(B->p_child.alloc(o_par)); CK(B->p_opc.alloc(o_op)); CK(B->d_aruns.alloc(4 * o_arun));
    CK(B->p_tip.alloc(2 * o_tip)); CK(B->p_erec.alloc(o_erec)); CK(B->p_doff.alloc(o_doff));
    CK(B->p_dense.alloc(o_dense)); CK(B->pr_rows.alloc(o_rows)); CK(B->pr_scr.alloc(o_scr));
    // prep stores each entry's parent vector at the chains that exist by then; the words past
    // them stay zero from here on (every pass writes the same words)
    CK(hipMemsetAsync(B->pr_rows.p, 0, std::max<uint64_t>(o_rows, 1) * sizeof(uint32_t), s));
    CK(B->pr_docs.upload(pd, s)); CK(B->pr_res.alloc(n));
    PrepParams &pp = B->prep;
    pp.in = Dd.in.p;
    pp.d_ops = Dd.ops.p; pp.d_aruns = Dd.aruns.p; pp.d_ent = Dd.ent.p; pp.d_poff = Dd.poff.p; pp.d_par = Dd.par.p;
    pp.d_ver = Dd.ver.p; pp.d_agents = Dd.agents.p;
    pp.par = B->p_par.p; pp.pent = B->p_pent.p; pp.pch = B->p_pch.p; pp.pcnt = B->p_pcnt.p; pp.child = B->p_child.p;
    pp.aruns = B->d_aruns.p; pp.tip = B->p_tip.p; pp.erec = B->p_erec.p; pp.doff = B->p_doff.p; pp.dense = B->p_dense.p;
    pp.rows = B->pr_rows.p; pp.scr = B->pr_scr.p; pp.opc = B->p_opc.p;
    if (B->cfg.prep_chains) {
        CK(B->pr_chain.alloc(std::max<size_t>(n, 1)));
        pp.chain_flag = B->pr_chain.p;
    }
    pp.docs = B->pr_docs.p; pp.results = B->pr_res.p; pp.n_docs = uint32_t(n); pp.max_entries = max_e;
    // debug mode (DTGPU_DEBUG, or DTGPU_PREP_CHECK alone): the bounds-checked prep kernel
    pp.check = B->cfg.prep_check ? 1u : 0u;
    if (launch_prep(pp, s)) return DTGPU_ERR_HIP;
    std::vector<PrepResult> prr(n);
    CK(hipMemcpyAsync(prr.data(), B->pr_res.p, n * sizeof(PrepResult), hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    stage_prof("stage: prep layout + pass");

    // ---- planner sizing pass ----------------------------------------------------------------------
    std::vector<PlanDesc> pdesc(n);
    uint64_t base_total = 0;
    uint32_t lds_entries = 0, max_agents = 0;
    for (size_t i = 0; i < n; i++) {
        PlanDesc &q = pdesc[i];
        std::memset(&q, 0, sizeof q);
        q.skip = 1;
        if (B->host_status[i] != OK) continue;
        if (prr[i].status != PREP_OK) { B->host_status[i] = prr[i].status == PREP_WIDE ? DECODE_DEFER : ErrCheckout; continue; }
        const PrepDesc &r = pd[i];
        q.skip = 0;
        q.par_off = r.o_par; q.child_off = r.o_child; q.op_off = r.o_op; q.arun_off = r.o_arun; q.tip_off = r.o_tip;
        q.erec_off = r.o_erec; q.doff_off = r.o_doff; q.dense_off = r.o_dense;
        q.base_off = base_total;
        q.prow_off = r.o_rows;   // device-staged: the prep kernel's parent vectors
        q.coff_off = r.o_scr + prep_kids_offset(r.n_par, r.ne);   // walk kernel: children per entry
        q.poff_off = r.d_poff;
        q.row_stride = PREP_MAX_CHAINS;
        q.ne = r.ne; q.n_agents = prr[i].n_chains; q.n_aruns = r.n_aruns; q.ntip = r.n_ver; q.n_lv = r.n_lv;
        base_total += uint64_t(r.ne) * std::max<uint32_t>(prr[i].n_chains, 1);
        lds_entries = std::max<uint32_t>(lds_entries, r.ne);
        max_agents = std::max<uint32_t>(max_agents, prr[i].n_chains);
    }
    CK(B->p_base.alloc(base_total));
    CK(B->p_order.alloc(std::max<uint64_t>(o_erec / EREC_WORDS, 1)));
    CK(B->p_walk.alloc(2 * std::max<size_t>(n, 1)));
    CK(B->p_docs.upload(pdesc, s));
    CK(B->p_results.alloc(n));
    CK(hipMemsetAsync(B->p_results.p, 0, std::max<size_t>(n, 1) * sizeof(PlanResult), s));
    PlanParams &q = B->plan;
    q.par = B->p_par.p; q.pent = B->p_pent.p; q.pch = B->p_pch.p; q.pcnt = B->p_pcnt.p; q.child = B->p_child.p;
    q.opc = B->p_opc.p; q.aruns = B->d_aruns.p; q.tip = B->p_tip.p; q.erec = B->p_erec.p; q.doff = B->p_doff.p;
    q.dense = B->p_dense.p; q.base = B->p_base.p; q.prow = B->pr_rows.p; q.order = B->p_order.p;
    q.walk = B->cfg.plan_walk ? B->p_walk.p : nullptr;
    q.coff = B->pr_scr.p;
    q.poff = Dd.poff.p;
    q.split = B->cfg.plan_split ? 1u : 0u;
    q.lds_entries = (lds_entries + 7) & ~7u;
    q.max_agents = max_agents;
    q.prof = B->cfg.plan_prof ? 1u : 0u;
    q.docs = B->p_docs.p; q.results = B->p_results.p; q.n_docs = uint32_t(n);
    q.count_only = 1;
    q.todo_cap = 0;
    if (launch_plan(q, s) != OK) { DTGPU_HIP_FAILED(hipErrorLaunchFailure); return DTGPU_ERR_HIP; }
    q.count_only = 0;
    std::vector<PlanResult> pres(n);
    CK(hipMemcpyAsync(pres.data(), B->p_results.p, std::max<size_t>(n, 1) * sizeof(PlanResult), hipMemcpyDeviceToHost, s));
    std::vector<uint32_t> wres;
    if (q.walk) {
        wres.resize(2 * n);
        CK(hipMemcpyAsync(wres.data(), q.walk, 2 * n * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    }
    CK(hipStreamSynchronize(s));
    // the walks of every later pass are the same walks: their stacks get the deepest one seen
    // here (plus slack), not PLAN_TODO_CAP -- the walk kernel's LDS then leaves room for the
    // chain decomposition's waves beside it.  (A deeper walk would fail its document visibly,
    // PLAN_TODO_FULL; the walk is deterministic, so none does.)
    if (q.walk && q.split) {
        uint32_t deep = 0;
        for (size_t i = 0; i < n; i++)
            if (!pdesc[i].skip && pres[i].status == PLAN_OK) deep = std::max(deep, wres[2 * i] >> 16);
        q.todo_cap = std::min<uint32_t>(PLAN_TODO_CAP, (deep + 16 + 1) & ~1u);
    }

    stage_prof("stage: planner sizing pass");
    // ---- replay layout ---------------------------------------------------------------------------
    uint64_t cmd_total = 0, tlist_total = 0, blk_total = 0, out_total = 0, gidx_total = 0;
    const uint64_t lds_fill = B->cfg.lds_fill;
    std::vector<int> seg_tier(n, -2);          // replay tier per document (-2: not replayed)
    std::vector<uint32_t> seg_est(n, 0);
    for (size_t i = 0; i < n; i++) {
        DocDesc &d = B->docs[i];
        std::memset(&d, 0, sizeof d);
        d.seg_hi = 0xFFFFFFFFu;   // not a segment (cut replay)
        d.src_off = ~0ull;
        if (B->host_status[i] != OK) { pdesc[i].skip = 1; continue; }
        if (pres[i].status != PLAN_OK) { B->host_status[i] = DECODE_DEFER; pdesc[i].skip = 1; continue; }
        const DecodeResult &r = Dd.res[i];
        const DecodeDesc &dd = Dd.desc[i];
        const uint64_t n_ins = prr[i].n_ins;
        d.cmd_off = cmd_total; d.tlist_off = tlist_total;
        d.ncmd = pres[i].ncmd;
        pdesc[i].cmd_off = cmd_total; pdesc[i].tlist_off = tlist_total;
        pdesc[i].ccap = pres[i].ncmd; pdesc[i].tcap = pres[i].ntlist;
        cmd_total += pres[i].ncmd;
        tlist_total += pres[i].ntlist;
        B->n_gpu_planned++;
        d.ascii = r.n_content == n_ins ? 1u : 0u;
        d.lv_off = dd.lv_off;                 // per-LV arenas share the decoder's LV numbering
        d.pc_off = dd.lv_off;
        d.n_lv = uint32_t(r.n_lv);
        d.content_off = dd.content_off;       // inserted text read in place
        d.content_len = r.n_content;
        d.arun_off = pd[i].o_arun * 4;
        d.n_aruns = r.n_aruns;
        if (B->ff_doc[i]) {   // the fast-forward path: out arena only (dt_ff.hip)
            d.flags |= DOC_FF;
            out_total = (out_total + 15) & ~15ull;
            d.out_off = out_total;
            d.out_cap = r.n_content;
            out_total += (uint64_t(d.out_cap) + 15) & ~15ull;
            B->total_lv += r.n_lv;
            B->alg_in_bytes += 16ull * r.n_ops + 8ull * r.n_entries + 4ull * r.n_parents + 12ull * r.n_aruns + r.n_content;
            continue;
        }
        if (n_ins / 32 + 2 > std::min<uint64_t>(LOC_MAX_BLOCKS, MAX_DOC_BLOCKS)) { B->host_status[i] = ErrCapacity; pdesc[i].skip = 1; continue; }
        const Layout lay = replay_layout(n_ins, lds_fill, false);
        d.max_blocks = lay.max_blocks;
        d.blk_off = blk_total;
        d.out_off = out_total;
        d.out_cap = r.n_content;
        blk_total += d.max_blocks;
        out_total += d.out_cap;
        B->total_lv += r.n_lv;
        B->alg_in_bytes += 16ull * r.n_ops + 8ull * r.n_entries + 4ull * r.n_parents + 12ull * r.n_aruns + r.n_content;
        d.gidx_off = gidx_total;
        gidx_total += lay.gidx;
        const int t = lay.tier;
        seg_tier[i] = t;
        seg_est[i] = lay.tier_blocks;
        if (t >= 0) {
            B->tier_list[t].push_back(uint32_t(i));
            B->tier_blocks[t] = std::max(B->tier_blocks[t], lay.tier_blocks);
        } else {
            B->large_list.push_back(uint32_t(i));
        }
    }
    const uint64_t lv_total = Dd.cbyte.n;
    // cut replay: long documents' later LV ranges as documents of their own
    uint64_t pc_total = lv_total, src_total = 0;
    {
        SegSettings sc = seg_settings(B->cfg);
        const std::vector<uint32_t> cand = seg_candidates(n, sc, B->n_cu, B->cfg.seg_fair, [&](size_t k) { return seg_tier[k] != -2 ? Dd.res[k].n_ops : 0u; });
        std::vector<uint8_t> late = late_documents(*B, sc, [&](size_t k) { return Dd.res[k].n_ops; });
        for (uint32_t i : cand) late[i] = 0;
        std::vector<uint32_t> all = cand;
        for (size_t i = 0; i < n; i++) if (late[i]) all.push_back(uint32_t(i));
        std::sort(all.begin(), all.end());
        // the cut planning itself (cut_kernel in sizing mode), one launch over every candidate
        // and one copy back: the same deterministic kernel every pass then runs against the
        // arenas reserved here (a host plan would need each document's decoded arrays back)
        std::vector<SegGroup> sg;
        std::vector<SegPlan> sp;
        std::vector<uint32_t> sdocs;
        uint64_t sscr = 0;
        uint32_t smax_ne = 0;
        for (uint32_t i : all) {
            const DecodeResult &r = Dd.res[i];
            SegSettings c = sc;
            if (late[i]) { c.max_seg = 2; c.ops_per_seg = std::max<uint64_t>(1, r.n_ops / 2); }
            const uint32_t T = uint32_t(std::min<uint64_t>(c.max_seg, r.n_ops / c.ops_per_seg));
            if (T < 2 || r.n_entries == 0 || r.n_lv >= 0x7FFFFFFFull || r.n_entries > PLAN_MAX_LDS_ENTRIES) continue;
            sg.push_back(SegGroup{uint32_t(sdocs.size()), T});
            sdocs.push_back(i);
            sp.push_back(SegPlan{c.w_op, T, sscr});
            sscr += (cut_scratch_words(r.n_entries) + 1) & ~1ull;
            smax_ne = std::max<uint32_t>(smax_ne, r.n_entries);
        }
        std::vector<uint32_t> sized(sg.size() * CUT_SIZED_WORDS);
        if (!sg.empty()) {
            DevBuf<SegGroup> dg;
            DevBuf<SegPlan> dp;
            DevBuf<uint32_t> dd, dscr, dout;
            CK(dg.upload(sg, s)); CK(dp.upload(sp, s)); CK(dd.upload(sdocs, s));
            CK(dscr.alloc(std::max<uint64_t>(sscr, 1))); CK(dout.alloc(sized.size()));
            CutParams c{};
            c.d_ops = Dd.ops.p; c.d_ent = Dd.ent.p; c.d_poff = Dd.poff.p; c.d_par = Dd.par.p;
            c.pdocs = B->pr_docs.p;
            c.groups = dg.p; c.seg_docs = dd.p; c.plans = dp.p;
            c.scr = dscr.p;
            c.n_groups = uint32_t(sg.size());
            c.max_ne = smax_ne;
            c.sized = dout.p;
            if (launch_cut(c, s)) return DTGPU_ERR_HIP;
            CK(hipMemcpyAsync(sized.data(), dout.p, sized.size() * 4, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
        }
        uint64_t scr = 0;
        for (size_t g = 0; g < sg.size(); g++) {
            const uint32_t i = sdocs[g];
            const uint32_t *z = sized.data() + g * CUT_SIZED_WORDS;
            std::vector<SegCut> cuts(std::min<uint32_t>(z[0], 64));
            for (size_t k = 0; k < cuts.size(); k++) cuts[k] = SegCut{z[1 + 4 * k], z[2 + 4 * k], z[3 + 4 * k], z[4 + 4 * k]};
            if (cuts.size() < 2 ||
                !add_segments(*B, i, cuts, seg_tier[i], seg_est[i], lds_fill, pc_total, blk_total, gidx_total, src_total))
                continue;
            B->seg_plans.push_back(SegPlan{sp[g].w_op, sp[g].n_targets, scr});
            for (const SegCut &k : cuts) B->seg_caps.push_back(SegCap{k.u, uint32_t(k.ins), k.lo, k.hi});
            scr += (cut_scratch_words(Dd.res[i].n_entries) + 1) & ~1ull;
            B->cut.max_ne = std::max<uint32_t>(B->cut.max_ne, Dd.res[i].n_entries);
        }
        CK(B->d_cutscr.alloc(std::max<uint64_t>(scr, 1)));
    }
    stage_prof("stage: layout + cut plans");
    // every later pass: parent-vector rows as wide as the document's chains (staging counted
    // them), four-word aligned for the planner's 16-byte row loads -- a 64-word row per entry
    // spread two live words over a cache line of their own (prep's stores, the planner's loads)
    uint32_t widest = 0;
    for (size_t i = 0; i < n; i++) {
        if (pd[i].skip || prr[i].status != PREP_OK) continue;
        const uint32_t rs = std::min<uint32_t>((std::max<uint32_t>(prr[i].n_chains, 1) + 3) & ~3u, PREP_MAX_CHAINS);
        pd[i].row_stride = rs;
        pdesc[i].row_stride = rs;
        widest = std::max(widest, rs);
    }
    B->prep.chain_w = widest;   // the chain decomposition's LDS ring rows, as wide as needed
    CK(B->pr_docs.upload(pd, s));
    B->prep.docs = B->pr_docs.p;
    CK(B->d_cmds.alloc(cmd_total));
    CK(B->d_tlist.alloc(tlist_total));
    CK(B->p_docs.upload(pdesc, s));
    B->plan.docs = B->p_docs.p;
    B->plan.cmds = B->d_cmds.p;
    B->plan.tlist = B->d_tlist.p;
    {   // every segment's LV range is the pass's cut planning's to write (poisoned here: a replay
        // without it fails, ErrCheckout site 30)
        mark_critical(*B);
        std::vector<DocDesc> up = B->docs;
        for (uint32_t d : B->seg_docs) { up[d].seg_lo = 0xFFFFFFFFu; up[d].seg_hi = 0; }
        CK(B->d_docs.upload(up, s));
    }
    CK(B->d_lists.upload(tier_lists(*B), s));
    CK(B->d_pos.alloc(pc_total));
    CK(B->d_ao.alloc(pc_total));
    CK(B->d_items.alloc(blk_total * 64));
    CK(B->d_m2.alloc(2 * blk_total));
    CK(B->d_out.alloc(out_total));
    CK(B->d_gidx.alloc(gidx_total));
    CK(B->d_fb.alloc(n_lds_docs(*B) + 1));
    CK(B->d_counter.alloc(2));
    CK(B->d_results.alloc(B->docs.size()));
    CK(hipMemsetAsync(B->d_results.p, 0, std::max<size_t>(B->docs.size(), 1) * sizeof(DocResult), s));
    CK(finish_segments(*B, src_total, Dd.cbyte.p, Dd.content.p, s));
    {   // linear documents: the fast-forward layout over the decoder's op runs, in place
        std::vector<FFIn> ffin;
        for (size_t i = 0; i < n; i++)
            if (B->ff_doc[i] && B->host_status[i] == OK) ffin.push_back(FFIn{Dd.desc[i].op_off, Dd.res[i].n_ops, uint32_t(i)});
            else B->ff_doc[i] = 0;
        CK(stage_ff(*B, ffin, Dd.ops.p, Dd.cbyte.p, Dd.content.p, s));
    }
    if (!B->seg_groups.empty()) {
        CK(B->d_plans.upload(B->seg_plans, s));
        CK(B->d_caps.upload(B->seg_caps, s));
        CutParams &c = B->cut;
        c.d_ops = Dd.ops.p; c.d_ent = Dd.ent.p; c.d_poff = Dd.poff.p; c.d_par = Dd.par.p;
        c.pdocs = B->pr_docs.p;
        c.groups = B->d_groups.p;
        c.seg_docs = B->d_segdocs.p;
        c.plans = B->d_plans.p;
        c.caps = B->d_caps.p;
        c.docs = B->d_docs.p;
        c.scr = B->d_cutscr.p;
        c.pent = B->p_pent.p;
        c.n_groups = uint32_t(B->seg_groups.size());
        if (!B->ev_cut) CK(hipEventCreateWithFlags(&B->ev_cut, hipEventDisableTiming));
    }
    CK(hipStreamSynchronize(s));
    stage_prof("stage: arenas + uploads");
#undef CK
    BatchParams base{};
    base.debug = B->cfg.debug;
    base.cmds = B->d_cmds.p;
    base.tlist = B->d_tlist.p;
    base.cbyte = Dd.cbyte.p;
    base.content = Dd.content.p;
    base.aruns = B->d_aruns.p;
    base.pos = B->d_pos.p;
    base.ao = B->d_ao.p;
    base.items = B->d_items.p;
    base.m2 = B->d_m2.p;
    base.out = B->d_out.p;
    base.gidx = B->d_gidx.p;
    base.docs = B->d_docs.p;
    base.results = B->d_results.p;
    base.src = B->d_src.p;
    if (set_tier_params(*B, base) != DTGPU_OK) { DTGPU_HIP_FAILED(hipErrorUnknown); return DTGPU_ERR_HIP; }
    B->wstream = B->side[kSideStreams - 1];   // the smallest side tier's stream (see wstream)
    // split pass: when an LDS tier rides a side stream and other documents exist, its
    // documents' prep and plan do not wait for everyone else's (a skewed batch's longest replays
    // start as soon as their own plans are done).  The tier: the critical documents' (DOC_CRITICAL,
    // the batch's longest replays), else the biggest non-empty one.  Its segment documents'
    // documents are planned there too (the main pipeline's replay waits for those plans).
    if (B->cfg.split) {
        int tb = -1;
        for (int t = kLdsTiers - 1; t >= 1 && tb < 0; t--)
            for (uint32_t d : B->tier_list[t])
                if (B->docs[d].flags & DOC_CRITICAL) { tb = t; break; }
        for (int t = kLdsTiers - 1; t >= 1 && tb < 0; t--)
            if (!B->tier_list[t].empty()) tb = t;
        if (tb >= 1) {
            std::vector<uint32_t> owner(B->docs.size());   // a segment document's document
            for (size_t d = 0; d < B->docs.size(); d++) owner[d] = uint32_t(d);
            for (const SegGroup &g : B->seg_groups)
                for (uint32_t k = 1; k < g.count; k++) owner[B->seg_docs[g.first + k]] = B->seg_docs[g.first];
            std::vector<uint8_t> big(n, 0);
            std::vector<uint32_t> lst;   // in the tier's order
            for (uint32_t d : B->tier_list[tb])
                if (owner[d] < n && !big[owner[d]]) { big[owner[d]] = 1; lst.push_back(owner[d]); }
            const size_t nb = lst.size();
            for (size_t i = 0; i < n; i++)
                if (!big[i] && !B->ff_doc[i]) lst.push_back(uint32_t(i));
            if (lst.size() > nb) {
                if (DTGPU_HIP_FAILED(B->d_split.upload(lst, s)) || DTGPU_HIP_FAILED(hipStreamSynchronize(s))) return DTGPU_ERR_HIP;
                B->split = true;
                B->split_tier = tb;
                if (!B->ws_side && DTGPU_HIP_FAILED(hipStreamCreateWithFlags(&B->ws_side, hipStreamNonBlocking))) return DTGPU_ERR_HIP;
                if (!B->ev_sw0 && DTGPU_HIP_FAILED(hipEventCreateWithFlags(&B->ev_sw0, hipEventDisableTiming))) return DTGPU_ERR_HIP;
                if (!B->ev_sw1 && DTGPU_HIP_FAILED(hipEventCreateWithFlags(&B->ev_sw1, hipEventDisableTiming))) return DTGPU_ERR_HIP;
                B->n_big = uint32_t(nb);
                B->n_rest = uint32_t(lst.size() - nb);
            }
        }
    }
    stage_prof("stage: split setup");
    *out = B.release();
    return DTGPU_OK;
}

// A split pass plans its cuts beside the side pipeline's prep, before the main pipeline's: the cut
// kernel then finds each parent's entry itself.
CutParams cut_before_prep(const dtgpu_batch *B) {
    CutParams c = B->cut;
    c.pent = nullptr;
    return c;
}
// The split pass's side pipeline (see stage_device): after a fork from s, the big tier's
// prep, plan and replay on its side stream.  The fallback counter is reset first, on s, since
// both pipelines' LDS tiers append to it; the main pipeline's replay_all(skip_tier) joins the
// side stream (launch_replay's fork / join of that tier's stream) before the HBM tier.
int launch_split_side(dtgpu_batch *B, hipStream_t s) {
    const int tb = B->split_tier;
    hipStream_t sb = B->side[kLdsTiers - 1 - tb];
    const BatchParams &q = B->tier[tb];
    if (q.fb_count && hipMemsetAsync(const_cast<uint32_t *>(q.fb_count), 0, sizeof(uint32_t), s) != hipSuccess) return ErrHip;
    if (hipEventRecord(B->ev_fork, s) != hipSuccess || hipStreamWaitEvent(sb, B->ev_fork, 0) != hipSuccess) return ErrHip;
    PrepParams pp = B->prep;
    pp.doc_list = B->d_split.p;
    pp.n_docs = B->n_big;
    PlanParams qq = B->plan;
    qq.doc_list = B->d_split.p;
    qq.n_docs = B->n_big;
    // as prep_and_plan: the walk (CSR mode, after prep's first half) on a stream of its own,
    // beside the chain decomposition and prep's second half
    const bool overlap = B->n_gpu_planned && B->prep.chain_flag && !B->prep.check && B->plan.walk && B->plan.coff &&
                         B->ws_side && B->cfg.walk_overlap;
    if (overlap) {
        pp.short_rec = B->plan.split ? 1u : 0u;
        if (launch_prep_stage(pp, sb, 1)) return ErrHip;
        if (hipEventRecord(B->ev_sw0, sb) != hipSuccess || hipStreamWaitEvent(B->ws_side, B->ev_sw0, 0) != hipSuccess) return ErrHip;
        if (launch_walk(qq, B->ws_side, true) != OK || hipEventRecord(B->ev_sw1, B->ws_side) != hipSuccess) return ErrHip;
        if (launch_prep_stage(pp, sb, 2) || launch_prep_stage(pp, sb, 3)) return ErrHip;
        if (hipStreamWaitEvent(sb, B->ev_sw1, 0) != hipSuccess || launch_plan(qq, sb, false) != OK) return ErrHip;
    } else {
        if (launch_prep(pp, sb)) return ErrHip;
        if (B->n_gpu_planned && launch_plan(qq, sb) != OK) return ErrHip;
    }
    if (hipEventRecord(B->ev_splan, sb) != hipSuccess) return ErrHip;
    // the cut planning on s, beside the side pipeline's prep and plan (the main pipeline's prep
    // follows it there); the side replay waits for it
    if (B->cut.n_groups && (launch_cut(cut_before_prep(B), s) || hipEventRecord(B->ev_cut, s) != hipSuccess ||
                            hipStreamWaitEvent(sb, B->ev_cut, 0) != hipSuccess))
        return ErrHip;
    BatchParams tiers[kLdsTiers];
    for (int t = 0; t < kLdsTiers; t++) {
        tiers[t] = B->tier[t];
        if (t != tb) tiers[t].n_list = 0;
    }
    BatchParams large = B->large;
    large.n_list = 0;
    large.fb_slots = 0;
    ReplayLaunch r{};
    r.lds = tiers;
    r.n_lds = kLdsTiers;
    r.large = &large;
    r.stream = sb;
    r.keep_fb = true;
    return launch_replay(r);
}
// The main pipeline's prep and plan of a split pass (the documents outside the big tier).
int launch_split_prep(dtgpu_batch *B, hipStream_t s) {
    PrepParams pp = B->prep;
    pp.doc_list = B->d_split.p + B->n_big;
    pp.n_docs = B->n_rest;
    return launch_prep(pp, s) ? ErrHip : OK;
}
int launch_split_plan(dtgpu_batch *B, hipStream_t s) {
    if (!B->n_gpu_planned) return OK;
    PlanParams qq = B->plan;
    qq.doc_list = B->d_split.p + B->n_big;
    qq.n_docs = B->n_rest;
    return launch_plan(qq, s);
}

// One checkout pass on stream s: prep (device-staged batches), plan (device), replay.
// Prep then plan for a device-staged batch.  With the three-launch prep and the walk kernel, the
// walk (CSR mode: it needs only prep's first half) runs on B->wstream beside the chain
// decomposition and prep's second half, and the plan kernel waits for it.  `mid` (nullable) is
// recorded between the two on s.
int prep_and_plan(dtgpu_batch *B, hipStream_t s, hipEvent_t mid) {
    const bool prep = B->dec != nullptr;
    const bool overlap = prep && B->n_gpu_planned && B->prep.chain_flag && !B->prep.check && B->plan.walk &&
                         B->plan.coff && B->wstream && B->cfg.walk_overlap;
    if (!overlap) {
        if (prep && launch_prep(B->prep, s)) return ErrHip;
        if (launch_cut(B->cut, s)) return ErrHip;   // (after prep: it reads the parents' entries)
        if (mid && hipEventRecord(mid, s) != hipSuccess) return ErrHip;
        return B->n_gpu_planned ? launch_plan(B->plan, s) : OK;
    }
    // the walk reads prep's CSR and, split, the planner only the entry records' heads
    PrepParams pp = B->prep;
    pp.short_rec = B->plan.split ? 1u : 0u;
    if (launch_prep_stage(pp, s, 1)) return ErrHip;
    if (hipEventRecord(B->ev_w0, s) != hipSuccess || hipStreamWaitEvent(B->wstream, B->ev_w0, 0) != hipSuccess) return ErrHip;
    if (launch_walk(B->plan, B->wstream, true) != OK) return ErrHip;
    if (hipEventRecord(B->ev_w1, B->wstream) != hipSuccess) return ErrHip;
    // the cut planning after the walk (it reads prep's parent entries), beside prep's second half
    // and the planner (only the replay needs it)
    if (B->cut.n_groups && (launch_cut(B->cut, B->wstream) || hipEventRecord(B->ev_cut, B->wstream) != hipSuccess))
        return ErrHip;
    if (launch_prep_stage(pp, s, 2) || launch_prep_stage(pp, s, 3)) return ErrHip;
    if (mid && hipEventRecord(mid, s) != hipSuccess) return ErrHip;
    if (hipStreamWaitEvent(s, B->ev_w1, 0) != hipSuccess) return ErrHip;
    if (launch_plan(B->plan, s, false) != OK) return ErrHip;
    if (B->cut.n_groups && hipStreamWaitEvent(s, B->ev_cut, 0) != hipSuccess) return ErrHip;
    return OK;
}

// The linear documents' checkout (dt_ff.hip) on s: first in a pass, or, in a split pass, right
// after the side pipeline's fork (beside it, before the main pipeline's prep).
int launch_ff_pass(dtgpu_batch *B, hipStream_t s) { return B->n_ff ? launch_ff(B->ff, s) : OK; }
// The tracker part of a pass (prep -> plan -> replay), unless every document fast-forwards.
bool tracker_pass(const dtgpu_batch *B) { return B->n_track != 0 || B->ff_doc.empty(); }

int launch_all(dtgpu_batch *B, hipStream_t s) {
    if (B->pass_mark && launch_pass_mark(s)) return ErrHip;
    if (B->xf_mode) return launch_replay_xf(B->large, s);
    if (B->split) {
        int e = launch_split_side(B, s);   // (it plans the cuts too)
        if (!e) e = launch_ff_pass(B, s);
        if (!e) e = launch_split_prep(B, s);
        if (!e) e = launch_split_plan(B, s);
        return e ? e : replay_all(B, s, B->split_tier);
    }
    int e = launch_ff_pass(B, s);
    if (e || !tracker_pass(B)) return e;
    e = prep_and_plan(B, s, nullptr);   // device-staged: walker inputs first
    return e ? e : replay_all(B, s);
}

}  // namespace

extern "C" {

// ---- oplog ----------------------------------------------------------------------------------
dtgpu_status dtgpu_oplog_load(const uint8_t *bytes, size_t len, int ignore_crc, dtgpu_oplog **out) {
    if (!out || (!bytes && len)) return DTGPU_ERR_ARG;
    auto h = std::make_unique<dtgpu_oplog>();
    Status s = decode_dt(bytes, len, ignore_crc != 0, h->o);
    if (s != OK) { *out = nullptr; return dtgpu_status(s); }
    *out = h.release();
    return DTGPU_OK;
}
dtgpu_oplog *dtgpu_oplog_new(void) { return new dtgpu_oplog(); }
void dtgpu_oplog_free(dtgpu_oplog *o) { delete o; }
dtgpu_status dtgpu_oplog_decode_and_add(dtgpu_oplog *h, const uint8_t *bytes, size_t len, int ignore_crc,
                                        uint64_t *frontier, size_t cap, size_t *n_frontier) {
    if (!h || (!bytes && len) || (!frontier && cap)) return DTGPU_ERR_ARG;
    std::vector<uint64_t> f;
    const Status s = decode_and_add(bytes, len, ignore_crc != 0, h->o, f);
    if (s != OK) return dtgpu_status(s);
    for (size_t i = 0; i < f.size() && i < cap; i++) frontier[i] = f[i];
    if (n_frontier) *n_frontier = f.size();
    h->last_added = std::move(f);
    return DTGPU_OK;
}
size_t dtgpu_oplog_last_added_frontier(const dtgpu_oplog *h, uint64_t *out, size_t cap) {
    if (!h) return 0;
    for (size_t i = 0; i < h->last_added.size() && i < cap; i++) out[i] = h->last_added[i];
    return h->last_added.size();
}
int64_t dtgpu_oplog_doc_id(const dtgpu_oplog *h, char *out, size_t cap) {
    if (!h || !h->o.has_doc_id) return -1;
    if (out) std::memcpy(out, h->o.doc_id.data(), std::min(cap, h->o.doc_id.size()));
    return int64_t(h->o.doc_id.size());
}
dtgpu_status dtgpu_oplog_set_doc_id(dtgpu_oplog *h, const char *id, size_t len) {
    if (!h) return DTGPU_ERR_ARG;
    if (!id) { h->o.doc_id.clear(); h->o.has_doc_id = false; return DTGPU_OK; }
    if (!utf8_valid(reinterpret_cast<const uint8_t *>(id), len)) return DTGPU_ERR_ARG;
    h->o.doc_id.assign(id, len);
    h->o.has_doc_id = true;
    return DTGPU_OK;
}
int32_t dtgpu_oplog_get_or_create_agent_id(dtgpu_oplog *o, const char *name, size_t len) {
    if (!o || (!name && len)) return -1;
    return o->o.agent_id(name, len);
}
static bool parents_ok(const HostOpLog &o, const uint64_t *parents, size_t np) {
    for (size_t i = 0; i < np; i++) if (parents[i] >= o.n_lv) return false;
    return true;
}
int64_t dtgpu_oplog_add_insert_at(dtgpu_oplog *h, int32_t agent, const uint64_t *parents, size_t np,
                                  uint64_t pos, const char *utf8, size_t nbytes) {
    if (!h || agent < 0 || size_t(agent) >= h->o.agent_names.size() || !parents_ok(h->o, parents, np)) return -1;
    const uint8_t *s = reinterpret_cast<const uint8_t *>(utf8);
    if (nbytes && !utf8_valid(s, nbytes)) return -1;
    uint64_t nchars = 0;
    for (size_t i = 0; i < nbytes; i += utf8_len(s[i])) nchars++;
    const uint64_t start = h->o.n_lv;
    if (!nchars) return int64_t(start) - 1;
    h->o.push_ins(pos, s, nbytes, nchars, true);
    h->o.add_span(uint32_t(agent), std::vector<uint64_t>(parents, parents + np), start, start + nchars);
    return int64_t(start + nchars - 1);
}
int64_t dtgpu_oplog_add_delete_at(dtgpu_oplog *h, int32_t agent, const uint64_t *parents, size_t np,
                                  uint64_t del_start, uint64_t del_end) {
    if (!h || agent < 0 || size_t(agent) >= h->o.agent_names.size() || !parents_ok(h->o, parents, np)) return -1;
    const uint64_t start = h->o.n_lv;
    if (del_end <= del_start) return int64_t(start) - 1;
    h->o.push_del(del_start, del_end - del_start, true);
    h->o.add_span(uint32_t(agent), std::vector<uint64_t>(parents, parents + np), start, start + (del_end - del_start));
    return int64_t(h->o.n_lv - 1);
}
int64_t dtgpu_oplog_add_insert(dtgpu_oplog *h, int32_t agent, uint64_t pos, const char *utf8, size_t nbytes) {
    if (!h) return -1;
    std::vector<uint64_t> v = h->o.version;
    return dtgpu_oplog_add_insert_at(h, agent, v.data(), v.size(), pos, utf8, nbytes);
}
int64_t dtgpu_oplog_add_delete_without_content(dtgpu_oplog *h, int32_t agent, uint64_t s, uint64_t e) {
    if (!h) return -1;
    std::vector<uint64_t> v = h->o.version;
    return dtgpu_oplog_add_delete_at(h, agent, v.data(), v.size(), s, e);
}
size_t dtgpu_oplog_len(const dtgpu_oplog *h) { return h ? size_t(h->o.n_lv) : 0; }
size_t dtgpu_oplog_cut_ranges(const dtgpu_oplog *h, uint64_t *out, size_t cap) {
    if (!h) return 0;
    SegInput si;
    seg_input_from_log(h->o, si);
    const auto cuts = cut_ranges(si);
    for (size_t k = 0; k < cuts.size() && k < cap && out; k++) { out[2 * k] = cuts[k].first; out[2 * k + 1] = cuts[k].second; }
    return cuts.size();
}
size_t dtgpu_oplog_local_frontier(const dtgpu_oplog *h, uint64_t *out, size_t cap) {
    if (!h) return 0;
    for (size_t i = 0; i < h->o.version.size() && i < cap; i++) out[i] = h->o.version[i];
    return h->o.version.size();
}

// Graph::find_dominators_2 (src/causalgraph/graph/tools.rs:545-578): the frontier of the union
// of two versions -- the members not in the history of another member, ascending.
int64_t dtgpu_oplog_dominators(const dtgpu_oplog *h, const uint64_t *a, size_t na, const uint64_t *b, size_t nb,
                               uint64_t *out, size_t cap) {
    if (!h || (na && !a) || (nb && !b)) return -1;
    std::vector<uint64_t> u(a, a + na);
    u.insert(u.end(), b, b + nb);
    for (uint64_t v : u) if (v >= h->o.n_lv) return -1;
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    std::vector<uint64_t> dom;
    std::vector<std::pair<uint64_t, uint64_t>> only_a, only_b;
    for (uint64_t v : u) {
        bool dominated = false;
        for (uint64_t w : u) {
            if (w <= v) continue;   // a version is only in the history of later LVs
            h->o.graph.diff_rev({v}, {w}, only_a, only_b);
            if (only_a.empty()) { dominated = true; break; }
        }
        if (!dominated) dom.push_back(v);
    }
    for (size_t i = 0; i < dom.size() && i < cap; i++) out[i] = dom[i];
    return int64_t(dom.size());
}

dtgpu_status dtgpu_oplog_plan_stats(const dtgpu_oplog *h, uint64_t out[4]) {
    if (!h || !out) return DTGPU_ERR_ARG;
    Prepared p;
    prepare_from_oplog(h->o, p);
    if (p.status != OK) return dtgpu_status(p.status);
    out[0] = p.plan.n_steps;
    out[1] = p.plan.n_retreat;
    out[2] = p.plan.n_advance;
    out[3] = p.plan.cmds.size();
    return DTGPU_OK;
}

size_t dtgpu_oplog_plan_commands(const dtgpu_oplog *h, uint32_t *cmds, size_t cap) {
    if (!h) return 0;
    Prepared p;
    prepare_from_oplog(h->o, p);
    if (p.status != OK) return 0;
    for (size_t i = 0; i < p.plan.cmds.size() && i < cap; i++) {
        cmds[4 * i] = p.plan.cmds[i].op;
        cmds[4 * i + 1] = p.plan.cmds[i].lv;
        cmds[4 * i + 2] = p.plan.cmds[i].len;
        cmds[4 * i + 3] = p.plan.cmds[i].pos;
    }
    return p.plan.cmds.size();
}

dtgpu_status dtgpu_oplog_encode(const dtgpu_oplog *h, const uint64_t *from, size_t n_from, uint32_t flags, uint8_t *out,
                                size_t cap, size_t *out_len) {
    if (!h || (n_from && !from)) return DTGPU_ERR_ARG;
    if (flags & ~uint32_t(DTGPU_ENCODE_FULL)) return DTGPU_ERR_ARG;   // see dtgpu.h
    std::vector<uint64_t> f(n_from + 1);
    const int64_t nf = dtgpu_oplog_dominators(h, from, n_from, nullptr, 0, f.data(), f.size());
    if (nf < 0) return DTGPU_ERR_ARG;
    f.resize(size_t(nf));
    std::vector<uint8_t> start, bytes;
    const bool with_start = (flags & DTGPU_ENCODE_STORE_START_BRANCH_CONTENT) && !f.empty();
    if (with_start) {   // ListBranch::new_at_local_version(self, from) (encode_oplog.rs:612-615), on the GPU
        size_t n = 0;   // the text is at most every inserted byte
        start.resize(h->o.ins_content.size() + 1);
        const dtgpu_status cs = dtgpu_checkout(h, f.data(), f.size(), start.data(), start.size(), &n);
        if (cs != DTGPU_OK) return cs;
        start.resize(n);
    }
    const Status st = encode_dt(h->o, f, (flags & DTGPU_ENCODE_STORE_INSERTED_CONTENT) != 0,
                                (flags & DTGPU_ENCODE_COMPRESS_CONTENT) != 0, with_start ? &start : nullptr, bytes);
    if (st != OK) return dtgpu_status(st);
    if (out_len) *out_len = bytes.size();
    if (!out) return DTGPU_OK;
    if (cap < bytes.size()) return DTGPU_ERR_ARG;
    std::memcpy(out, bytes.data(), bytes.size());
    return DTGPU_OK;
}

dtgpu_status dtgpu_lz4_compress(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len) {
    if (!in && n) return DTGPU_ERR_ARG;
    std::vector<uint8_t> c;
    lz4_block_compress(in, n, c);
    if (out_len) *out_len = c.size();
    if (!out) return DTGPU_OK;
    if (cap < c.size()) return DTGPU_ERR_ARG;
    std::memcpy(out, c.data(), c.size());
    return DTGPU_OK;
}

size_t dtgpu_oplog_xf_order(const dtgpu_oplog *h, const uint64_t *from, size_t n_from, const uint64_t *merge,
                            size_t n_merge, uint32_t *out, size_t cap) {
    if (!h || (n_from && !from) || (n_merge && !merge)) return 0;
    HostOpLog log = h->o;
    log.finish();
    std::vector<uint64_t> f(n_from + 1), m(n_merge + 1);
    const int64_t nf = dtgpu_oplog_dominators(h, from, n_from, nullptr, 0, f.data(), f.size());
    const int64_t nm = dtgpu_oplog_dominators(h, merge, n_merge, nullptr, 0, m.data(), m.size());
    if (nf < 0 || nm < 0) return 0;
    f.resize(size_t(nf));
    m.resize(size_t(nm));
    Plan plan;
    size_t first = 0;
    if (build_xf_plan_from(log, f, m, plan, first) != OK) return 0;
    size_t k = 0;
    for (size_t i = first; i < plan.cmds.size(); i++) {
        const Cmd &c = plan.cmds[i];
        if ((c.op & 15u) == CMD_TOG) continue;
        for (uint32_t j = 0; j < c.len; j++, k++) if (k < cap) out[k] = c.lv + j;
    }
    return k;
}

size_t dtgpu_oplog_plan_tlist(const dtgpu_oplog *h, uint32_t *out, size_t cap) {
    if (!h) return 0;
    Prepared p;
    prepare_from_oplog(h->o, p);
    if (p.status != OK) return 0;
    if (out) std::memcpy(out, p.plan.tlist.data(), std::min(cap, p.plan.tlist.size()) * sizeof(uint32_t));
    return p.plan.tlist.size();
}

size_t dtgpu_oplog_ins_content(const dtgpu_oplog *h, uint8_t *out, size_t cap) {
    if (!h) return 0;
    const auto &c = h->o.ins_content;
    if (out) std::memcpy(out, c.data(), std::min(cap, c.size()));
    return c.size();
}
size_t dtgpu_oplog_char_offsets(const dtgpu_oplog *h, uint32_t *out, size_t cap) {
    if (!h) return 0;
    const auto &c = h->o.ins_cbyte;
    if (out) std::memcpy(out, c.data(), std::min(cap, c.size()) * sizeof(uint32_t));
    return c.size();
}
size_t dtgpu_oplog_agent_runs(const dtgpu_oplog *h, uint32_t *out, size_t cap) {
    if (!h) return 0;
    Prepared p;
    prepare_from_oplog(h->o, p);
    const auto &a = p.plan.agent_runs;
    if (out) std::memcpy(out, a.data(), std::min(cap, a.size()) * sizeof(uint32_t));
    return a.size();
}

size_t dtgpu_oplog_export(const dtgpu_oplog *h, int what, void *out, size_t cap) {
    if (!h) return 0;
    const HostOpLog &o = h->o;
    std::vector<uint32_t> w;
    std::vector<uint8_t> b;
    bool bytes = false;
    switch (what) {
        case DTGPU_EXPORT_OPS: {   // split at graph entries, as the decoders produce them
            HostOpLog f;
            f.ops = o.ops;
            f.graph = o.graph;
            f.finish();
            for (const OpRun &r : f.ops) {
                w.push_back(uint32_t(r.lv)); w.push_back(uint32_t(r.len)); w.push_back(uint32_t(r.pos));
                w.push_back(uint32_t(r.kind) | (uint32_t(r.fwd) << 1));
            }
            break;
        }
        case DTGPU_EXPORT_AGENT_RUNS:
            for (const AgentRun &r : o.agent_runs) {
                w.push_back(uint32_t(r.lv)); w.push_back(uint32_t(r.len)); w.push_back(r.agent); w.push_back(uint32_t(r.seq));
            }
            break;
        case DTGPU_EXPORT_ENTRIES:
            for (const GraphEntry &e : o.graph.entries) { w.push_back(uint32_t(e.start)); w.push_back(uint32_t(e.end)); }
            break;
        case DTGPU_EXPORT_PARENT_OFFSETS: {
            uint32_t k = 0;
            for (const GraphEntry &e : o.graph.entries) { w.push_back(k); k += uint32_t(e.parents.size()); }
            w.push_back(k);
            break;
        }
        case DTGPU_EXPORT_PARENTS:
            for (const GraphEntry &e : o.graph.entries) for (uint64_t p : e.parents) w.push_back(uint32_t(p));
            break;
        case DTGPU_EXPORT_CONTENT: b = o.ins_content; bytes = true; break;
        case DTGPU_EXPORT_CHAR_OFFSETS: w = o.ins_cbyte; break;
        case DTGPU_EXPORT_VERSION: for (uint64_t v : o.version) w.push_back(uint32_t(v)); break;
        case DTGPU_EXPORT_AGENT_NAMES:
            for (const std::string &nm : o.agent_names) { b.push_back(uint8_t(nm.size())); b.insert(b.end(), nm.begin(), nm.end()); }
            bytes = true;
            break;
        case DTGPU_EXPORT_DOC_ID:
            b.push_back(o.has_doc_id ? 1 : 0);
            if (o.has_doc_id) b.insert(b.end(), o.doc_id.begin(), o.doc_id.end());
            bytes = true;
            break;
        default: return 0;
    }
    const size_t per = what == DTGPU_EXPORT_OPS || what == DTGPU_EXPORT_AGENT_RUNS ? 4 : what == DTGPU_EXPORT_ENTRIES ? 2 : 1;
    if (bytes) {
        if (out) std::memcpy(out, b.data(), std::min(cap, b.size()));
        return b.size();
    }
    const size_t count = w.size() / per;
    if (out) std::memcpy(out, w.data(), std::min(cap, count) * per * 4);
    return count;
}

// ---- batch ----------------------------------------------------------------------------------
dtgpu_status dtgpu_batch_create(const uint8_t *const *docs, const size_t *lens, size_t n,
                                const dtgpu_batch_opts *opts, dtgpu_batch **out) {
    if (!out || (n && (!docs || !lens))) return DTGPU_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return DTGPU_ERR_NO_DEVICE;
    std::vector<Prepared> prep(n);
    const bool ignore_crc = opts && opts->ignore_crc;
    parallel_for(n, threads_for(opts, n), [&](size_t i) {
        Prepared &p = prep[i];
        p.status = decode_dt(docs[i], lens[i], ignore_crc, p.log);
        prepare_input(p);
    });
    return stage(prep, opts, out);
}
dtgpu_status dtgpu_batch_create_from_oplogs(const dtgpu_oplog *const *oplogs, size_t n,
                                            const dtgpu_batch_opts *opts, dtgpu_batch **out) {
    if (!out || (n && !oplogs)) return DTGPU_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return DTGPU_ERR_NO_DEVICE;
    std::vector<Prepared> prep(n);
    parallel_for(n, threads_for(opts, n), [&](size_t i) {
        prep[i].log = oplogs[i]->o;
        prep[i].log.finish();
        prepare_input(prep[i]);
    });
    return stage(prep, opts, out);
}
dtgpu_status dtgpu_batch_create_xf(const dtgpu_oplog *const *oplogs, size_t n, const dtgpu_batch_opts *opts,
                                   dtgpu_batch **out) {
    if (!out || (n && !oplogs)) return DTGPU_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return DTGPU_ERR_NO_DEVICE;
    std::vector<Prepared> prep(n);
    parallel_for(n, threads_for(opts, n), [&](size_t i) {
        prep[i].log = oplogs[i]->o;
        prep[i].log.finish();
        prep[i].xf_merge = prep[i].log.version;
        prepare_input(prep[i]);
    });
    return stage(prep, opts, out, true);
}
dtgpu_status dtgpu_batch_xf_positions(dtgpu_batch *B, size_t i, uint32_t *out, size_t cap, size_t *n_out) {
    if (!B || i >= B->n || !B->xf_mode) return DTGPU_ERR_ARG;
    if (B->host_status[i] != OK) return dtgpu_status(B->host_status[i]);
    const size_t n = size_t(B->n_lv[i]);
    if (n_out) *n_out = n;
    if (!out) return DTGPU_OK;
    if (cap < n) return DTGPU_ERR_ARG;
    DocResult r;
    if (hipMemcpyAsync(&r, B->d_results.p + i, sizeof r, hipMemcpyDeviceToHost, B->stream) != hipSuccess ||
        (n && hipMemcpyAsync(out, B->d_xf.p + B->docs[i].lv_off, n * 4, hipMemcpyDeviceToHost, B->stream) != hipSuccess) ||
        hipStreamSynchronize(B->stream) != hipSuccess)
        return DTGPU_ERR_HIP;
    return r.status == OK ? DTGPU_OK : dtgpu_status(r.status);
}
dtgpu_status dtgpu_batch_create_device(const uint8_t *const *docs, const size_t *lens, size_t n,
                                       const dtgpu_batch_opts *opts, dtgpu_batch **out) {
    if (!out || (n && (!docs || !lens))) return DTGPU_ERR_ARG;
    dtgpu_decoded *dh = nullptr;
    const dtgpu_status st = dtgpu_decode_create(docs, lens, n, opts, &dh);
    if (st != DTGPU_OK) return st;
    return stage_device(dh, opts, out);
}

dtgpu_status dtgpu_batch_create_decoded(dtgpu_decoded *dec, dtgpu_batch **out) {
    if (!dec || !out) return DTGPU_ERR_ARG;
    if (!dec->stream && hipStreamCreateWithFlags(&dec->stream, hipStreamNonBlocking) != hipSuccess) {
        dtgpu_decode_free(dec);   // consumed on failure too (dtgpu.h)
        return DTGPU_ERR_HIP;
    }
    return stage_device(dec, nullptr, out);
}
dtgpu_status dtgpu_batch_run_e2e_timed(dtgpu_batch *B, float ms[4]) {
    if (!B || !B->dec || B->dec->merged) return DTGPU_ERR_ARG;
    if (hipSetDevice(B->device) != hipSuccess) return DTGPU_ERR_HIP;
    hipStream_t s = B->stream;
    // decode + prep + plan + replay from the `.dt` bytes in HBM
    if (hipEventRecord(B->ev_dec, s) != hipSuccess) return DTGPU_ERR_HIP;
    if (launch_decode(B->dec->P, s)) return DTGPU_ERR_HIP;
    if (hipEventRecord(B->ev_prep, s) != hipSuccess) return DTGPU_ERR_HIP;
    if (launch_ff_pass(B, s)) return DTGPU_ERR_HIP;   // linear documents (dt_ff.hip)
    if (tracker_pass(B) ? prep_and_plan(B, s, B->ev0) != OK : hipEventRecord(B->ev0, s) != hipSuccess) return DTGPU_ERR_HIP;
    if (hipEventRecord(B->ev_mid, s) != hipSuccess) return DTGPU_ERR_HIP;
    int st = tracker_pass(B) ? replay_all(B, s) : OK;
    if (st) return dtgpu_status(st);
    if (hipEventRecord(B->ev1, s) != hipSuccess) return DTGPU_ERR_HIP;
    if (hipEventSynchronize(B->ev1) != hipSuccess) return DTGPU_ERR_HIP;
    float td = 0, tp = 0, tl = 0, tr = 0;
    if (hipEventElapsedTime(&td, B->ev_dec, B->ev_prep) != hipSuccess || hipEventElapsedTime(&tp, B->ev_prep, B->ev0) != hipSuccess ||
        hipEventElapsedTime(&tl, B->ev0, B->ev_mid) != hipSuccess || hipEventElapsedTime(&tr, B->ev_mid, B->ev1) != hipSuccess)
        return DTGPU_ERR_HIP;
    B->last_decode_ms = td; B->last_prep_ms = tp; B->last_plan_ms = tl; B->last_replay_ms = tr;
    if (ms) { ms[0] = td; ms[1] = tp; ms[2] = tl; ms[3] = tr; }
    return DTGPU_OK;
}
dtgpu_status dtgpu_batch_encode(dtgpu_batch *B, uint32_t flags, float *kernel_ms) {
    if (!B || !B->dec || B->xf_mode) return DTGPU_ERR_ARG;
    if (flags & ~uint32_t(DTGPU_ENCODE_FULL)) return DTGPU_ERR_ARG;
    if (hipSetDevice(B->device) != hipSuccess) return DTGPU_ERR_HIP;
    hipStream_t s = B->stream;
#define CK(x) do { if (DTGPU_HIP_FAILED(x)) return DTGPU_ERR_HIP; } while (0)
    if (B->e_desc.empty() && B->n) {   // layout once per batch
        const dtgpu_decoded &Dd = *B->dec;
        B->e_desc.assign(B->n, EncDesc{});
        uint64_t w = 0, b = 0, o = 0;
        uint32_t max_agents = 1, max_text = 0;
        for (size_t i = 0; i < B->n; i++) {
            EncDesc &e = B->e_desc[i];
            e.skip = 1;
            if (B->host_status[i] != OK) continue;
            const DecodeResult &r = Dd.res[i];
            const DecodeDesc &d = Dd.desc[i];
            const DocDesc &dd = B->docs[i];
            e.skip = 0;
            e.in_off = d.in_off; e.arun_off = d.arun_off; e.ent_off = d.ent_off; e.poff_off = d.poff_off;
            e.par_off = d.par_off; e.content_off = d.content_off; e.lv_off = d.lv_off; e.agent_off = d.agent_off;
            e.cmd_off = dd.cmd_off;
            e.ncmd = dd.ncmd; e.n_aruns = r.n_aruns; e.ne = r.n_entries; e.n_agents = r.n_agents;
            e.n_lv = uint32_t(r.n_lv); e.n_content = r.n_content;
            e.doc_id_off = r.doc_id_off; e.doc_id_len = r.doc_id_len;
            e.w_off = w; w += enc_words(e.ne, e.ncmd, e.n_aruns, e.n_agents);
            e.b_off = b; b += (r.n_content + lz4_bound(r.n_content) + 15) / 16 * 16;   // 16-B aligned text
            // output bound: header + names + doc id + every stream at its widest varints
            const uint64_t cap = 128 + 11ull * r.n_agents + 64 + (r.doc_id_len != 0xFFFFFFFFu ? r.doc_id_len : 0) +
                                 30ull * (uint64_t(r.n_aruns) + r.n_entries) + 20ull * e.ncmd + 10ull * r.n_entries +
                                 10ull * r.n_parents + lz4_bound(r.n_content) + d.in_len;   // names are in the input
            e.out_off = o; e.out_cap = uint32_t(std::min<uint64_t>(cap, 0xFFFFFFF0ull)); o += (e.out_cap + 15) / 16 * 16;   // 16-B aligned (CRC reads)
            max_agents = std::max(max_agents, r.n_agents);
            max_text = std::max(max_text, r.n_content);
        }
        CK(B->e_docs.upload(B->e_desc, s));
        CK(B->e_dres.alloc(B->n));
        CK(B->e_w.alloc(std::max<uint64_t>(w, 1)));
        CK(B->e_b.alloc(std::max<uint64_t>(b, 1)));
        CK(B->e_out.alloc(std::max<uint64_t>(o, 1)));
        EncParams &q = B->enc;
        q.in = Dd.in.p; q.content = Dd.content.p;
        q.aruns = Dd.aruns.p; q.ent = Dd.ent.p; q.poff = Dd.poff.p; q.par = Dd.par.p; q.cbyte = Dd.cbyte.p;
        q.agents = Dd.agents.p;
        q.cmds = B->d_cmds.p;
        q.w = B->e_w.p; q.b = B->e_b.p; q.out = B->e_out.p;
        q.docs = B->e_docs.p; q.results = B->e_dres.p;
        q.n_docs = uint32_t(B->n);
        q.max_agents = max_agents;
        // kernel 2 stages a document's text in LDS for the LZ4 pass when it fits: 16 KiB of hash
        // table + 512 B of output ring + <= 23.5 KiB of text keeps 4 waves per CU
        // measured (10k friendsforever): 60 ms with the text in LDS (4 waves per CU), 44 ms with
        // it read from HBM at 9 waves per CU -- occupancy wins in a batch, so staging is opt-in
        q.lds_text = 0;
        (void)max_text;
        q.lds_text = B->cfg.enc_lds_text;
        q.prof = B->cfg.enc_prof ? 1u : 0u;
        for (int k = 0; k < 32; k++) q.x2n[k] = Dd.P.x2n[k];
    }
    // the walk order: the planner's commands (prep + plan, as a checkout pass runs them), for
    // every document (a checkout pass skips the fast-forwarded ones: their lists cover the rest)
    {
        PrepParams pp = B->prep;
        PlanParams qq = B->plan;
        pp.doc_list = nullptr; pp.n_docs = uint32_t(B->n);
        qq.doc_list = nullptr; qq.n_docs = uint32_t(B->n);
        if (launch_prep(pp, s)) return DTGPU_ERR_HIP;
        if (B->n_gpu_planned && launch_plan(qq, s) != OK) return DTGPU_ERR_HIP;
    }
    B->enc.flags = flags;
    CK(hipMemsetAsync(B->e_dres.p, 0, std::max<size_t>(B->n, 1) * sizeof(EncResult), s));
    CK(hipEventRecord(B->ev0, s));
    if (launch_encode(B->enc, s)) return DTGPU_ERR_HIP;
    CK(hipEventRecord(B->ev1, s));
    B->e_res.resize(B->n);
    CK(hipMemcpyAsync(B->e_res.data(), B->e_dres.p, B->n * sizeof(EncResult), hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, B->ev0, B->ev1));
#undef CK
    if (kernel_ms) *kernel_ms = ms;
    return DTGPU_OK;
}

dtgpu_status dtgpu_batch_encoded(const dtgpu_batch *B, size_t i, uint8_t *out, size_t cap, size_t *out_len,
                                 uint64_t prof[14]) {
    if (!B || i >= B->n || B->e_res.size() != B->n) return DTGPU_ERR_ARG;
    if (B->host_status[i] != OK) return dtgpu_status(B->host_status[i]);
    const EncResult &r = B->e_res[i];
    if (r.status != OK) return dtgpu_status(r.status);
    if (prof) {
        for (int k = 0; k < 6; k++) prof[k] = r.prof[k];
        for (int k = 0; k < 3; k++) prof[6 + k] = r.lzcyc[k];
        for (int k = 0; k < 3; k++) prof[9 + k] = r.lzst[k];
        prof[12] = r.prof[6];
        prof[13] = r.prof[7];
    }
    if (out_len) *out_len = r.len;
    if (!out) return DTGPU_OK;
    if (cap < r.len) return DTGPU_ERR_ARG;
    if (hipSetDevice(B->device) != hipSuccess) return DTGPU_ERR_HIP;
    if (hipMemcpy(out, B->e_out.p + B->e_desc[i].out_off, r.len, hipMemcpyDeviceToHost) != hipSuccess) return DTGPU_ERR_HIP;
    return DTGPU_OK;
}

uint64_t dtgpu_batch_encoded_bytes(const dtgpu_batch *B, int which) {
    if (!B || B->e_res.size() != B->n) return 0;
    uint64_t t = 0;
    for (size_t i = 0; i < B->n; i++) {
        if (B->host_status[i] != OK || B->e_res[i].status != OK) continue;
        const DecodeResult &r = B->dec->res[i];
        if (which == 0) t += B->e_res[i].len;
        else t += 16ull * r.n_ops + 8ull * r.n_entries + 4ull * r.n_parents + 16ull * r.n_aruns + r.n_content;
    }
    return t;
}

dtgpu_status dtgpu_batch_run(dtgpu_batch *B, void *stream) {
    if (!B) return DTGPU_ERR_ARG;
    if (hipSetDevice(B->device) != hipSuccess) return DTGPU_ERR_HIP;
    void *s = stream ? stream : reinterpret_cast<void *>(B->stream);
    if (B->debug)
        fprintf(stderr, "[dtgpu] launch lds tiers %u/%u/%u/%u (blocks %u/%u/%u/%u) hbm %u\n", B->tier[0].n_list,
                B->tier[1].n_list, B->tier[2].n_list, B->tier[3].n_list, B->tier[0].lds_blocks, B->tier[1].lds_blocks,
                B->tier[2].lds_blocks, B->tier[3].lds_blocks, B->large.n_list);
    if (B->debug) {
        size_t nc = 0;
        for (const DocDesc &d : B->docs) nc += (d.flags & DOC_CRITICAL) != 0;
        fprintf(stderr, "[dtgpu] critical %zu of %zu replays; split tier %d (%u + %u documents)\n", nc, B->docs.size(),
                B->split ? B->split_tier : -1, B->n_big, B->n_rest);
    }
    dtgpu_status st = dtgpu_status(launch_all(B, reinterpret_cast<hipStream_t>(s)));
    if (B->debug) {
        fprintf(stderr, "[dtgpu] launched status %d\n", int(st));
        hipError_t e = hipStreamSynchronize(reinterpret_cast<hipStream_t>(s));
        fprintf(stderr, "[dtgpu] synced %d\n", int(e));
    }
    return st;
}
dtgpu_status dtgpu_batch_run_timed(dtgpu_batch *B, float *ms) {
    if (!B) return DTGPU_ERR_ARG;
    if (hipSetDevice(B->device) != hipSuccess) return DTGPU_ERR_HIP;
    // one checkout pass of the whole batch on its stream: for device-staged batches the walker
    // inputs (prep_kernel: parent entries, children CSR, chain decomposition -- what
    // SpanningTreeWalker::new builds inside checkout_tip, txn_trace.rs:114-188), then the walk
    // planner, then replay + materialisation
    hipStream_t s = B->stream;
    const bool prep = B->dec && !B->xf_mode;
    const bool split = prep && B->split;   // split pass: prep / plan times are the main pipeline's
    if (B->pass_mark && launch_pass_mark(s)) return DTGPU_ERR_HIP;
    if (hipEventRecord(B->ev_prep, s) != hipSuccess) return DTGPU_ERR_HIP;
    if (split && launch_split_side(B, s)) return DTGPU_ERR_HIP;   // (it plans the cuts too)
    // linear documents (dt_ff.hip): a batch of only those reports their pass as its replay time
    if (!B->xf_mode && !tracker_pass(B)) {
        if (hipEventRecord(B->ev0, s) != hipSuccess || hipEventRecord(B->ev_mid, s) != hipSuccess) return DTGPU_ERR_HIP;
    }
    if (!B->xf_mode && launch_ff_pass(B, s)) return DTGPU_ERR_HIP;
    if (!B->xf_mode && !tracker_pass(B)) {
    } else if (split) {
        if (launch_split_prep(B, s) != OK || hipEventRecord(B->ev0, s) != hipSuccess || launch_split_plan(B, s) != OK)
            return DTGPU_ERR_HIP;
    } else if (B->xf_mode) {
        if (hipEventRecord(B->ev0, s) != hipSuccess) return DTGPU_ERR_HIP;
        if (B->n_gpu_planned && launch_plan(B->plan, s) != OK) return DTGPU_ERR_HIP;
    } else if (prep_and_plan(B, s, B->ev0) != OK) {
        return DTGPU_ERR_HIP;
    }
    if (tracker_pass(B) && hipEventRecord(B->ev_mid, s) != hipSuccess) return DTGPU_ERR_HIP;
    int st = B->xf_mode ? launch_replay_xf(B->large, s) : tracker_pass(B) ? replay_all(B, s, split ? B->split_tier : -1) : OK;
    if (st) return dtgpu_status(st);
    if (hipEventRecord(B->ev1, s) != hipSuccess) return DTGPU_ERR_HIP;
    if (hipEventSynchronize(B->ev1) != hipSuccess) return DTGPU_ERR_HIP;
    float t = 0, tp = 0, tq = 0;
    if (hipEventElapsedTime(&t, B->ev_prep, B->ev1) != hipSuccess) return DTGPU_ERR_HIP;
    if (hipEventElapsedTime(&tq, B->ev_prep, B->ev0) != hipSuccess) return DTGPU_ERR_HIP;
    if (hipEventElapsedTime(&tp, B->ev0, B->ev_mid) != hipSuccess) return DTGPU_ERR_HIP;
    B->last_prep_ms = prep ? tq : 0.0f;
    B->last_plan_ms = tp;
    B->last_replay_ms = t - tp - tq;
    if (ms) *ms = t;
    return DTGPU_OK;
}
dtgpu_status dtgpu_batch_sync(dtgpu_batch *B) {
    if (!B) return DTGPU_ERR_ARG;
    return hipStreamSynchronize(B->stream) == hipSuccess ? DTGPU_OK : DTGPU_ERR_HIP;
}
size_t dtgpu_batch_size(const dtgpu_batch *B) { return B ? B->n : 0; }
dtgpu_status dtgpu_batch_last_times(const dtgpu_batch *B, float out[3]) {
    if (!B || !out) return DTGPU_ERR_ARG;
    out[0] = B->last_plan_ms;
    out[1] = B->last_replay_ms;
    out[2] = B->last_prep_ms;
    return DTGPU_OK;
}
size_t dtgpu_batch_segments(dtgpu_batch *B, size_t doc, uint32_t *out, size_t cap) {
    if (!B || doc >= B->n) return 0;
    for (const SegGroup &g : B->seg_groups) {
        if (B->seg_docs[g.first] != doc) continue;
        if (hipSetDevice(B->device) != hipSuccess) return 0;
        for (uint32_t k = 0; k < g.count && k < cap; k++) {
            const uint32_t d = B->seg_docs[g.first + k];
            DocDesc e{};   // the device descriptor: the pass's cut planning wrote the range
            DocResult r{};
            if (hipMemcpyAsync(&r, B->d_results.p + d, sizeof r, hipMemcpyDeviceToHost, B->stream) != hipSuccess ||
                hipMemcpyAsync(&e, B->d_docs.p + d, sizeof e, hipMemcpyDeviceToHost, B->stream) != hipSuccess ||
                hipStreamSynchronize(B->stream) != hipSuccess)
                return 0;
            uint32_t *w = out + 12 * size_t(k);
            const size_t slot = size_t(g.first) + k;
            const bool dev_cut = slot < B->seg_caps.size();   // device-staged: the pass plans the cuts
            w[8] = dev_cut && (e.flags & DOC_CUT_HOST) ? 1u : 0u;
            w[9] = dev_cut ? B->seg_caps[slot].lo : e.seg_lo;
            w[10] = dev_cut ? B->seg_caps[slot].hi : e.seg_hi;
            w[11] = dev_cut ? B->seg_caps[slot].u : e.seg_u;
            w[0] = e.seg_lo; w[1] = e.seg_hi; w[2] = e.seg_u;
            // the first segment's result slot is the document's: the combine step rewrote it
            w[3] = k ? r.status : 0u; w[4] = k ? r.out_len : 0u; w[5] = r.dbg[15];
            w[6] = r.lds; w[7] = r.n_blocks;
        }
        return g.count;
    }
    return 0;
}
size_t dtgpu_batch_host_planned(const dtgpu_batch *B, uint8_t *flags, size_t cap) {
    if (!B) return 0;
    if (flags) for (size_t i = 0; i < B->n && i < cap; i++) flags[i] = B->host_planned[i];
    size_t k = 0;
    for (uint8_t f : B->host_planned) k += f != 0;
    return k;
}
size_t dtgpu_batch_fast_forwarded(const dtgpu_batch *B, uint8_t *flags, size_t cap) {
    if (!B) return 0;
    if (flags) for (size_t i = 0; i < B->n && i < cap; i++) flags[i] = i < B->ff_doc.size() ? B->ff_doc[i] : 0;
    return B->n_ff;
}
dtgpu_status dtgpu_batch_plan(dtgpu_batch *B, size_t i, uint32_t *cmds, size_t cmd_cap, uint32_t *tlist,
                              size_t tlist_cap, size_t *n_cmds, size_t *n_tlist) {
    if (!B || i >= B->n) return DTGPU_ERR_ARG;
    if (B->host_status[i] != OK) return dtgpu_status(B->host_status[i]);
    if (i < B->ff_doc.size() && B->ff_doc[i]) {   // fast-forwarded: a checkout pass plans no walk for it
        if (n_cmds) *n_cmds = 0;
        if (n_tlist) *n_tlist = 0;
        return DTGPU_OK;
    }
    const DocDesc &d = B->docs[i];
    std::vector<Cmd> c(d.ncmd);
    if (d.ncmd && hipMemcpyAsync(c.data(), B->d_cmds.p + d.cmd_off, d.ncmd * sizeof(Cmd), hipMemcpyDeviceToHost, B->stream) != hipSuccess)
        return DTGPU_ERR_HIP;
    if (hipStreamSynchronize(B->stream) != hipSuccess) return DTGPU_ERR_HIP;
    size_t nt = 0;
    for (const Cmd &x : c) if ((x.op & 15u) == CMD_TOG) nt = std::max<size_t>(nt, size_t(x.lv) + x.len);
    if (n_cmds) *n_cmds = c.size();
    if (n_tlist) *n_tlist = nt;
    if (cmds) {
        if (cmd_cap < c.size()) return DTGPU_ERR_ARG;
        std::memcpy(cmds, c.data(), c.size() * sizeof(Cmd));
    }
    if (tlist && nt) {
        if (tlist_cap < nt) return DTGPU_ERR_ARG;
        if (hipMemcpyAsync(tlist, B->d_tlist.p + d.tlist_off, nt * 4, hipMemcpyDeviceToHost, B->stream) != hipSuccess ||
            hipStreamSynchronize(B->stream) != hipSuccess)
            return DTGPU_ERR_HIP;
    }
    return DTGPU_OK;
}
uint64_t dtgpu_batch_algorithmic_bytes(dtgpu_batch *B) {
    if (!B) return 0;
    std::vector<dtgpu_doc_result> r(B->n);
    if (B->n && dtgpu_batch_results(B, r.data()) != DTGPU_OK) return 0;
    uint64_t out = 0;
    for (const auto &x : r) out += x.text_len;
    return B->alg_in_bytes + out;
}
dtgpu_status dtgpu_batch_plan_profile(dtgpu_batch *B, size_t i, uint64_t out[8]) {
    if (!B || i >= B->n || !out) return DTGPU_ERR_ARG;
    PlanResult r;
    if (hipMemcpyAsync(&r, B->p_results.p + i, sizeof r, hipMemcpyDeviceToHost, B->stream) != hipSuccess ||
        hipStreamSynchronize(B->stream) != hipSuccess)
        return DTGPU_ERR_HIP;
    for (int k = 0; k < 6; k++) out[k] = r.prof[k];
    out[6] = r.ncmd;
    out[7] = r.ntlist;
    return DTGPU_OK;
}
dtgpu_status dtgpu_batch_doc_stats(dtgpu_batch *B, size_t i, uint32_t out[29]) {
    if (!B || i >= B->docs.size() || !out) return DTGPU_ERR_ARG;   // (past n: the segment documents)
    DocResult r;
    if (hipMemcpyAsync(&r, B->d_results.p + i, sizeof r, hipMemcpyDeviceToHost, B->stream) != hipSuccess ||
        hipStreamSynchronize(B->stream) != hipSuccess)
        return DTGPU_ERR_HIP;
    out[0] = r.n_items; out[1] = r.n_blocks; out[2] = r.fail_cmd; out[3] = r.fail_site;
    out[4] = B->docs[i].ncmd; out[5] = B->docs[i].max_blocks;
    for (int k = 0; k < 16; k++) out[6 + k] = r.dbg[k];
    out[22] = r.n_sb;
    out[23] = r.lds;
    for (int k = 0; k < 3; k++) out[24 + k] = r.dbg[16 + k];
    out[27] = r.dbg[19];   // block loads that rebuilt stale masks
    out[28] = r.dbg[20];   // block loads (not from the registers' cached block)
    return DTGPU_OK;
}
uint64_t dtgpu_batch_total_lv(const dtgpu_batch *B) { return B ? B->total_lv : 0; }

dtgpu_status dtgpu_batch_results(dtgpu_batch *B, dtgpu_doc_result *res) {
    if (!B || (!res && B->n)) return DTGPU_ERR_ARG;
    std::vector<DocResult> dr(B->n);
    if (B->n && hipMemcpyAsync(dr.data(), B->d_results.p, B->n * sizeof(DocResult), hipMemcpyDeviceToHost, B->stream) != hipSuccess)
        return DTGPU_ERR_HIP;
    if (hipStreamSynchronize(B->stream) != hipSuccess) return DTGPU_ERR_HIP;
    for (size_t i = 0; i < B->n; i++) {
        res[i].status = B->host_status[i] != OK ? B->host_status[i] : dr[i].status;
        res[i].reserved = 0;
        res[i].text_len = res[i].status == OK ? dr[i].out_len : 0;
        res[i].text_hash = res[i].status == OK ? dr[i].hash : 0;
        res[i].n_lv = B->n_lv[i];
    }
    return DTGPU_OK;
}
dtgpu_status dtgpu_batch_text(dtgpu_batch *B, size_t i, uint8_t *out, size_t cap, size_t *out_len) {
    if (!B || i >= B->n) return DTGPU_ERR_ARG;
    if (B->host_status[i] != OK) return dtgpu_status(B->host_status[i]);
    DocResult r;
    if (hipMemcpyAsync(&r, B->d_results.p + i, sizeof r, hipMemcpyDeviceToHost, B->stream) != hipSuccess ||
        hipStreamSynchronize(B->stream) != hipSuccess)
        return DTGPU_ERR_HIP;
    if (r.status != OK) {
        if (B->debug)
            fprintf(stderr, "[dtgpu] doc %zu status %u fail_cmd %u fail_site %u items %u blocks %u dbg %u %u %u %u %u %u %u %x %x %x\n", i, r.status,
                    r.fail_cmd, r.fail_site, r.n_items, r.n_blocks, r.dbg[0], r.dbg[1], r.dbg[2], r.dbg[3], r.dbg[4],
                    r.dbg[5], r.dbg[6], r.dbg[7], r.dbg[8], r.dbg[9]);
        return dtgpu_status(r.status);
    }
    if (out_len) *out_len = r.out_len;
    if (!out) return DTGPU_OK;
    if (cap < r.out_len) return DTGPU_ERR_ARG;
    if (r.out_len && (hipMemcpyAsync(out, B->d_out.p + B->docs[i].out_off, r.out_len, hipMemcpyDeviceToHost, B->stream) != hipSuccess ||
                      hipStreamSynchronize(B->stream) != hipSuccess))
        return DTGPU_ERR_HIP;
    return DTGPU_OK;
}
void dtgpu_batch_free(dtgpu_batch *B) { delete B; }

dtgpu_status dtgpu_batch_checkout(const uint8_t *const *docs, const size_t *lens, size_t n,
                                  const dtgpu_batch_opts *opts, dtgpu_doc_result *results) {
    dtgpu_batch *B = nullptr;
    dtgpu_status s = dtgpu_batch_create(docs, lens, n, opts, &B);
    if (s) return s;
    s = dtgpu_batch_run(B, nullptr);
    if (!s) s = dtgpu_batch_results(B, results);
    dtgpu_batch_free(B);
    return s;
}

// ListOpLog::checkout(&[LV]) (src/list/oplog.rs:32-36) is a merge from ROOT over the history of
// `version`.  That history is closed under parents, so it is an oplog of its own: its LVs are
// compacted in order (agents, seqs and op positions unchanged -- every op's position is relative
// to its parents' version, which lies inside the history) and its tip checkout is the checkout
// at `version`.  The sub-oplog is built here and checked out by the same device path.
static Status history_oplog(const HostOpLog &o, const std::vector<uint64_t> &version, HostOpLog &s) {
    for (uint64_t v : version) if (v >= o.n_lv) return ErrCheckout;
    std::vector<std::pair<uint64_t, uint64_t>> hist, none;
    o.graph.diff_rev(version, {}, hist, none);   // Hist(version), newest first
    std::reverse(hist.begin(), hist.end());
    std::vector<uint64_t> base(hist.size());      // new LV of each range's start
    uint64_t nn = 0;
    for (size_t i = 0; i < hist.size(); i++) { base[i] = nn; nn += hist[i].second - hist[i].first; }
    auto map = [&](uint64_t lv) -> uint64_t {      // old LV (inside the history) -> new LV
        size_t i = size_t(std::upper_bound(hist.begin(), hist.end(), lv,
                                           [](uint64_t v, const std::pair<uint64_t, uint64_t> &r) { return v < r.second; }) -
                          hist.begin());
        return base[i] + (lv - hist[i].first);
    };
    s = HostOpLog();
    s.agent_names = o.agent_names;
    s.agent_seqs.assign(o.agent_names.size(), {});
    size_t oi = 0, ai = 0, ei = 0;
    for (const auto &r : hist) {
        // agent assignment
        while (ai < o.agent_runs.size() && o.agent_runs[ai].lv + o.agent_runs[ai].len <= r.first) ai++;
        for (size_t k = ai; k < o.agent_runs.size() && o.agent_runs[k].lv < r.second; k++) {
            const AgentRun &a = o.agent_runs[k];
            const uint64_t x = std::max(a.lv, r.first), y = std::min(a.lv + a.len, r.second);
            if (x < y) s.assign(a.agent, a.seq + (x - a.lv), map(x), y - x);
        }
        // op runs, clipped (rev delete runs delete right to left: op_metrics.rs:184-202)
        while (oi < o.ops.size() && o.ops[oi].lv + o.ops[oi].len <= r.first) oi++;
        for (size_t k = oi; k < o.ops.size() && o.ops[k].lv < r.second; k++) {
            const OpRun &op = o.ops[k];
            const uint64_t x = std::max(op.lv, r.first), y = std::min(op.lv + op.len, r.second);
            if (x >= y) continue;
            if (op.kind == 0) {
                for (uint64_t u = x; u < y;) {   // pieces of uniform ContentIsKnown
                    const bool known = o.ins_cbyte[u] != ~0u;
                    uint64_t w = u + 1;
                    while (w < y && (o.ins_cbyte[w] != ~0u) == known) w++;
                    size_t b0 = 0, b1 = 0;
                    if (known) {
                        b0 = o.ins_cbyte[u];
                        b1 = o.ins_cbyte[w - 1] + utf8_len(o.ins_content[o.ins_cbyte[w - 1]]);
                    }
                    s.push_ins(op.pos + (u - op.lv), known ? o.ins_content.data() + b0 : nullptr, b1 - b0, w - u, known);
                    u = w;
                }
            } else if (op.fwd) {
                s.push_del(op.pos, y - x, true);
            } else {
                s.push_del(op.pos + (op.lv + op.len - y), y - x, false);
            }
        }
        // graph entries, clipped: a piece that starts inside an entry continues its previous LV
        while (ei < o.graph.entries.size() && o.graph.entries[ei].end <= r.first) ei++;
        for (size_t k = ei; k < o.graph.entries.size() && o.graph.entries[k].start < r.second; k++) {
            const GraphEntry &e = o.graph.entries[k];
            const uint64_t x = std::max(e.start, r.first), y = std::min(e.end, r.second);
            if (x >= y) continue;
            std::vector<uint64_t> par;
            if (x == e.start) for (uint64_t p : e.parents) par.push_back(map(p));
            else par.push_back(map(x - 1));
            std::sort(par.begin(), par.end());
            s.graph.push(par, map(x), map(y - 1) + 1);
        }
    }
    for (uint64_t v : version) s.version.push_back(map(v));
    std::sort(s.version.begin(), s.version.end());
    s.version.erase(std::unique(s.version.begin(), s.version.end()), s.version.end());
    if (s.n_lv != nn) return ErrCheckout;
    s.finish();
    return OK;
}

// TextInfo::merge_into's subgraph (src/listmerge/merge.rs:954-1054 via Graph::subgraph_raw and
// project_onto_subgraph_raw, src/causalgraph/graph/subgraph.rs:39-250): the ops of one text CRDT
// are the LV spans `T` of a shared causal graph; the text is checked out over the graph
// projected onto T, where a version's projection is the frontier of Hist(version) n T.  The
// sub-oplog is compacted like history_oplog (agents, seqs and positions kept: a text op's
// position is relative to that text alone), so the same device path checks it out.
static Status project_oplog(const HostOpLog &o, std::vector<std::pair<uint64_t, uint64_t>> spans, HostOpLog &s,
                            const std::vector<std::vector<uint64_t>> *extra = nullptr,
                            std::vector<std::vector<uint64_t>> *extra_out = nullptr) {
    std::sort(spans.begin(), spans.end());
    std::vector<std::pair<uint64_t, uint64_t>> t;   // merged, non-empty
    for (auto r : spans) {
        if (r.first > r.second || r.second > o.n_lv) return ErrArg;
        if (r.first == r.second) continue;
        if (!t.empty() && r.first <= t.back().second) t.back().second = std::max(t.back().second, r.second);
        else t.push_back(r);
    }
    std::vector<uint64_t> base(t.size());
    uint64_t nn = 0;
    for (size_t i = 0; i < t.size(); i++) { base[i] = nn; nn += t[i].second - t[i].first; }
    auto span_of = [&](uint64_t lv) -> int64_t {   // last span starting at or before lv
        return int64_t(std::upper_bound(t.begin(), t.end(), lv, [](uint64_t v, const std::pair<uint64_t, uint64_t> &r) {
                           return v < r.first; }) - t.begin()) - 1;
    };
    auto in_t = [&](uint64_t lv) { const int64_t i = span_of(lv); return i >= 0 && lv < t[size_t(i)].second; };
    auto map = [&](uint64_t lv) -> uint64_t { const int64_t i = span_of(lv); return base[size_t(i)] + (lv - t[size_t(i)].first); };
    s = HostOpLog();
    s.agent_names = o.agent_names;
    s.agent_seqs.assign(o.agent_names.size(), {});
    size_t oi = 0, ai = 0, ei = 0;
    for (const auto &r : t) {
        while (ai < o.agent_runs.size() && o.agent_runs[ai].lv + o.agent_runs[ai].len <= r.first) ai++;
        for (size_t k = ai; k < o.agent_runs.size() && o.agent_runs[k].lv < r.second; k++) {
            const AgentRun &a = o.agent_runs[k];
            const uint64_t x = std::max(a.lv, r.first), y = std::min(a.lv + a.len, r.second);
            if (x < y) s.assign(a.agent, a.seq + (x - a.lv), map(x), y - x);
        }
        while (oi < o.ops.size() && o.ops[oi].lv + o.ops[oi].len <= r.first) oi++;
        for (size_t k = oi; k < o.ops.size() && o.ops[k].lv < r.second; k++) {
            const OpRun &op = o.ops[k];
            const uint64_t x = std::max(op.lv, r.first), y = std::min(op.lv + op.len, r.second);
            if (x >= y) continue;
            if (op.kind == 0) {
                for (uint64_t u = x; u < y;) {
                    const bool known = o.ins_cbyte[u] != ~0u;
                    uint64_t w = u + 1;
                    while (w < y && (o.ins_cbyte[w] != ~0u) == known) w++;
                    size_t b0 = 0, b1 = 0;
                    if (known) {
                        b0 = o.ins_cbyte[u];
                        b1 = o.ins_cbyte[w - 1] + utf8_len(o.ins_content[o.ins_cbyte[w - 1]]);
                    }
                    s.push_ins(op.pos + (u - op.lv), known ? o.ins_content.data() + b0 : nullptr, b1 - b0, w - u, known);
                    u = w;
                }
            } else if (op.fwd) {
                s.push_del(op.pos, y - x, true);
            } else {
                s.push_del(op.pos + (op.lv + op.len - y), y - x, false);
            }
        }
    }
    (void)ei;
    // The graph, in one pass over the entries cut into runs inside / outside T.  A run outside T
    // gets its projected version P (constant along the run: the chain below it); a run inside T
    // is an entry of the projected graph whose parents are the projection of its own parents.  A
    // projection is the union of the parents' P (a T member projects to itself), reduced to its
    // frontier in the projected graph built so far (it holds every earlier T member).
    // Projected versions can be wide antichains (a text whose ops hang off another's), so runs
    // share them and a union is reduced by one walk down the projected graph, newest entry first,
    // that stops below the union's lowest member (the reference's find_dominators heap walk,
    // src/causalgraph/graph/tools.rs:545-578).
    using Set = std::shared_ptr<const std::vector<uint64_t>>;
    struct Piece { uint64_t start, end; Set proj; };
    std::vector<Piece> outside;   // ascending
    std::vector<uint64_t> seen_to(1, 0);   // per projected entry: 1 + highest LV walked
    auto frontier_of = [&](std::vector<uint64_t> u) -> std::vector<uint64_t> {
        std::sort(u.begin(), u.end());
        u.erase(std::unique(u.begin(), u.end()), u.end());
        if (u.size() < 2) return u;
        const uint64_t lo = u.front();
        std::vector<uint8_t> dominated(u.size(), 0);
        std::priority_queue<uint64_t> heap;
        std::vector<size_t> touched;
        seen_to.resize(s.graph.entries.size(), 0);
        auto push_parents = [&](uint64_t x) {   // parents of LV x in the projected graph
            const int64_t ei = s.graph.find_idx(x);
            const GraphEntry &e = s.graph.entries[size_t(ei)];
            if (x > e.start) heap.push(x - 1);
            else for (uint64_t p : e.parents) heap.push(p);
        };
        for (uint64_t c : u) push_parents(c);
        while (!heap.empty()) {
            const uint64_t v = heap.top();
            heap.pop();
            if (v < lo) break;
            const size_t ei = size_t(s.graph.find_idx(v));
            if (seen_to[ei] > v) continue;
            const GraphEntry &e = s.graph.entries[ei];
            const uint64_t from = std::max(e.start, seen_to[ei]);   // [from, v] is new history
            if (!seen_to[ei]) touched.push_back(ei);
            seen_to[ei] = v + 1;
            for (auto it = std::lower_bound(u.begin(), u.end(), from); it != u.end() && *it <= v; ++it)
                dominated[size_t(it - u.begin())] = 1;
            if (from == e.start) for (uint64_t p : e.parents) heap.push(p);
        }
        for (size_t ei : touched) seen_to[ei] = 0;
        std::vector<uint64_t> dom;
        for (size_t i = 0; i < u.size(); i++) if (!dominated[i]) dom.push_back(u[i]);
        return dom;
    };
    auto project_set = [&](const std::vector<uint64_t> &ver) -> Set {
        std::vector<uint64_t> u;
        Set only;
        size_t sources = 0;
        for (uint64_t p : ver) {
            sources++;
            if (in_t(p)) { u.push_back(map(p)); continue; }
            auto it = std::upper_bound(outside.begin(), outside.end(), p,
                                       [](uint64_t v, const Piece &q) { return v < q.start; });
            if (it == outside.begin() || p >= (--it)->end) continue;   // cannot happen: parents precede
            only = it->proj;
            u.insert(u.end(), it->proj->begin(), it->proj->end());
        }
        if (sources == 1 && only) return only;   // one parent outside T: its run's projection
        return std::make_shared<const std::vector<uint64_t>>(frontier_of(std::move(u)));
    };
    auto project = [&](const std::vector<uint64_t> &ver) -> std::vector<uint64_t> { return *project_set(ver); };
    for (const GraphEntry &e : o.graph.entries) {
        for (uint64_t x = e.start; x < e.end;) {
            const bool inside = in_t(x);
            uint64_t y = x + 1;
            if (inside) {
                y = std::min(e.end, t[size_t(span_of(x))].second);
            } else {
                const int64_t i = span_of(x);   // next T span starts after x
                const size_t nx = size_t(i + 1);
                y = nx < t.size() ? std::min(e.end, t[nx].first) : e.end;
            }
            Set par = project_set(x == e.start ? e.parents : std::vector<uint64_t>{x - 1});
            if (inside) s.graph.push(*par, map(x), map(y - 1) + 1);
            else outside.push_back(Piece{x, y, std::move(par)});
            x = y;
        }
    }
    s.version = project(o.version);
    if (extra && extra_out) {   // further versions of the shared graph, projected the same way
        extra_out->clear();
        for (const auto &v : *extra) {
            for (uint64_t x : v) if (x >= o.n_lv) return ErrArg;
            extra_out->push_back(project(v));
        }
    }
    if (s.n_lv != nn) return ErrCheckout;
    s.finish();
    return OK;
}

dtgpu_status dtgpu_oplog_project(const dtgpu_oplog *h, const uint64_t *spans, size_t n_spans, dtgpu_oplog **out) {
    if (!h || !out || (n_spans && !spans)) return DTGPU_ERR_ARG;
    *out = nullptr;
    std::vector<std::pair<uint64_t, uint64_t>> t(n_spans);
    for (size_t i = 0; i < n_spans; i++) t[i] = {spans[2 * i], spans[2 * i + 1]};
    HostOpLog log = h->o;
    log.finish();   // op runs split at graph entries
    auto *sub = new dtgpu_oplog;
    const Status st = project_oplog(log, t, sub->o);
    if (st != OK) { delete sub; return dtgpu_status(st); }
    *out = sub;
    return DTGPU_OK;
}

int64_t dtgpu_oplog_project_version(const dtgpu_oplog *h, const uint64_t *spans, size_t n_spans, const uint64_t *version,
                                    size_t n_version, uint64_t *out, size_t cap) {
    if (!h || (n_spans && !spans) || (n_version && !version) || (cap && !out)) return -1;
    std::vector<std::pair<uint64_t, uint64_t>> t(n_spans);
    for (size_t i = 0; i < n_spans; i++) t[i] = {spans[2 * i], spans[2 * i + 1]};
    HostOpLog log = h->o;
    log.finish();
    HostOpLog sub;
    const std::vector<std::vector<uint64_t>> vs{std::vector<uint64_t>(version, version + n_version)};
    std::vector<std::vector<uint64_t>> pv;
    if (project_oplog(log, t, sub, &vs, &pv) != OK || pv.size() != 1) return -1;
    for (size_t i = 0; i < pv[0].size() && i < cap; i++) out[i] = pv[0][i];
    return int64_t(pv[0].size());
}

// AgentAssignment::local_to_agent_version (src/causalgraph/agent_assignment/mod.rs): the agent
// run holding lv, by binary search over the LV-ordered runs.
dtgpu_status dtgpu_oplog_local_to_remote(const dtgpu_oplog *h, uint64_t lv, uint32_t *agent, uint64_t *seq) {
    if (!h || !agent || !seq || lv >= h->o.n_lv) return DTGPU_ERR_ARG;
    const auto &r = h->o.agent_runs;
    auto it = std::upper_bound(r.begin(), r.end(), lv, [](uint64_t v, const AgentRun &a) { return v < a.lv; });
    if (it == r.begin()) return DTGPU_ERR_ARG;
    --it;
    if (lv >= it->lv + it->len) return DTGPU_ERR_ARG;
    *agent = it->agent;
    *seq = it->seq + (lv - it->lv);
    return DTGPU_OK;
}

// The local LV spans of the remote span (agent, seq .. seq + n), in seq order
// (AgentAssignment::remote_to_local_version over a span): binary search over the agent's runs,
// which are seq-ordered whenever the agent's ops arrived in seq order (a linear pass otherwise).
// Returns the span count, or -1 when part of the span is not in the oplog.
int64_t dtgpu_oplog_remote_to_local(const dtgpu_oplog *h, uint32_t agent, uint64_t seq, uint64_t n, uint64_t *spans,
                                    size_t cap) {
    if (!h || agent >= h->o.agent_seqs.size() || (cap && !spans)) return -1;
    const auto &v = h->o.agent_seqs[agent];
    const auto by_seq = [](const SeqRun &a, const SeqRun &b) { return a.seq < b.seq; };
    std::vector<SeqRun> hit;
    const uint64_t end = seq + n;
    if (std::is_sorted(v.begin(), v.end(), by_seq)) {
        auto it = std::upper_bound(v.begin(), v.end(), seq, [](uint64_t x, const SeqRun &r) { return x < r.seq; });
        if (it != v.begin()) --it;
        for (; it != v.end() && it->seq < end; ++it)
            if (it->seq + it->len > seq) hit.push_back(*it);
    } else {
        for (const SeqRun &r : v)
            if (r.seq < end && r.seq + r.len > seq) hit.push_back(r);
        std::sort(hit.begin(), hit.end(), by_seq);
    }
    size_t k = 0;
    uint64_t at = seq;
    for (const SeqRun &r : hit) {
        if (r.seq + r.len <= at) continue;
        if (r.seq > at) return -1;   // a gap: that seq is not known here
        const uint64_t hi = std::min(end, r.seq + r.len);
        if (k < cap) { spans[2 * k] = r.lv + (at - r.seq); spans[2 * k + 1] = r.lv + (hi - r.seq); }
        k++;
        at = hi;
    }
    return at == end ? int64_t(k) : -1;
}

dtgpu_status dtgpu_oplog_history(const dtgpu_oplog *h, const uint64_t *version, size_t n_version, dtgpu_oplog **out) {
    if (!h || !out || (n_version && !version)) return DTGPU_ERR_ARG;
    *out = nullptr;
    std::vector<uint64_t> v(n_version + 1);
    const int64_t nv = dtgpu_oplog_dominators(h, version, n_version, nullptr, 0, v.data(), v.size());
    if (nv < 0) return DTGPU_ERR_ARG;
    v.resize(size_t(nv));
    auto *sub = new dtgpu_oplog;
    const Status st = history_oplog(h->o, v, sub->o);
    if (st != OK) { delete sub; return dtgpu_status(st); }
    *out = sub;
    return DTGPU_OK;
}
dtgpu_status dtgpu_checkout(const dtgpu_oplog *h, const uint64_t *version, size_t n_version, uint8_t *out, size_t cap,
                            size_t *out_len) {
    if (!h || (n_version && !version)) return DTGPU_ERR_ARG;
    std::vector<uint64_t> v(n_version + 1);   // reduce to a frontier (Frontier::from_unsorted)
    const int64_t nv = dtgpu_oplog_dominators(h, version, n_version, nullptr, 0, v.data(), v.size());
    if (nv < 0) return DTGPU_ERR_CHECKOUT;
    v.resize(size_t(nv));
    dtgpu_oplog sub;
    const Status st = history_oplog(h->o, v, sub.o);
    if (st != OK) return dtgpu_status(st);
    return dtgpu_checkout_tip(&sub, out, cap, out_len);
}

dtgpu_status dtgpu_xf_operations_from(const dtgpu_oplog *h, const uint64_t *from, size_t n_from, const uint64_t *merge,
                                      size_t n_merge, uint32_t *out, size_t cap, size_t *n_out) {
    if (!h || (n_from && !from) || (n_merge && !merge)) return DTGPU_ERR_ARG;
    std::vector<Prepared> prep(1);
    Prepared &p = prep[0];
    p.log = h->o;
    p.log.finish();
    for (auto [v, n, dst] : {std::make_tuple(from, n_from, &p.xf_from), std::make_tuple(merge, n_merge, &p.xf_merge)}) {
        dst->resize(n + 1);   // reduce to frontiers (Frontier::from_unsorted)
        const int64_t k = dtgpu_oplog_dominators(h, v, n, nullptr, 0, dst->data(), dst->size());
        if (k < 0) return DTGPU_ERR_ARG;
        dst->resize(size_t(k));
    }
    {   // the reported LV count comes from the host plan (no GPU needed for a size query)
        Plan plan;
        size_t first = 0;
        const Status st = build_xf_plan_from(p.log, p.xf_from, p.xf_merge, plan, first);
        if (st != OK) return dtgpu_status(st);
        size_t k = 0;
        for (size_t i = first; i < plan.cmds.size(); i++) if ((plan.cmds[i].op & 15u) != CMD_TOG) k += plan.cmds[i].len;
        if (n_out) *n_out = k;
        if (!out) return DTGPU_OK;
        if (cap < k) return DTGPU_ERR_ARG;
        if (k == 0) return DTGPU_OK;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return DTGPU_ERR_NO_DEVICE;
    prepare_input(p);
    dtgpu_batch *B = nullptr;
    dtgpu_status st = stage(prep, nullptr, &B, true);
    if (st) return st;
    std::unique_ptr<dtgpu_batch> hold(B);
    if (B->host_status[0] != OK) return dtgpu_status(B->host_status[0]);
    if (launch_replay_xf(B->large, B->stream) != OK) return DTGPU_ERR_HIP;
    DocResult r;
    std::vector<uint32_t> xfv(p.log.n_lv);
    if (hipMemcpyAsync(&r, B->d_results.p, sizeof r, hipMemcpyDeviceToHost, B->stream) != hipSuccess ||
        hipMemcpyAsync(xfv.data(), B->d_xf.p, xfv.size() * 4, hipMemcpyDeviceToHost, B->stream) != hipSuccess ||
        hipStreamSynchronize(B->stream) != hipSuccess)
        return DTGPU_ERR_HIP;
    if (r.status != OK) return dtgpu_status(r.status);
    // application order = the plan's reported INS / DEL commands in order
    size_t k = 0;
    for (size_t i = p.xf_first; i < p.plan.cmds.size(); i++) {
        const Cmd &c = p.plan.cmds[i];
        if ((c.op & 15u) == CMD_TOG) continue;
        for (uint32_t j = 0; j < c.len && k < cap; j++, k++) {
            out[2 * k] = c.lv + j;
            out[2 * k + 1] = xfv[c.lv + j];
        }
    }
    return DTGPU_OK;
}
dtgpu_status dtgpu_xf_operations(const dtgpu_oplog *h, uint32_t *out, size_t cap, size_t *n_out) {
    if (!h) return DTGPU_ERR_ARG;
    return dtgpu_xf_operations_from(h, nullptr, 0, h->o.version.data(), h->o.version.size(), out, cap, n_out);
}

dtgpu_status dtgpu_checkout_tip(const dtgpu_oplog *h, uint8_t *out, size_t cap, size_t *out_len) {
    if (!h) return DTGPU_ERR_ARG;
    dtgpu_batch *B = nullptr;
    dtgpu_status s = dtgpu_batch_create_from_oplogs(&h, 1, nullptr, &B);
    if (s) return s;
    s = dtgpu_batch_run(B, nullptr);
    size_t len = 0;
    if (!s) s = dtgpu_batch_text(B, 0, nullptr, 0, &len);
    if (!s) {
        if (out_len) *out_len = len;
        if (out) s = cap < len ? DTGPU_ERR_ARG : dtgpu_batch_text(B, 0, out, cap, &len);
    }
    dtgpu_batch_free(B);
    return s;
}

uint64_t dtgpu_text_hash(const uint8_t *t, size_t n) { return text_hash(t, n); }
int dtgpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}
const char *dtgpu_status_str(dtgpu_status s) {
    static const char *names[] = {"OK", "InvalidMagic", "UnsupportedProtocolVersion", "DocIdMismatch",
                                  "BaseVersionUnknown", "UnknownChunk", "LZ4DecoderNeeded", "LZ4DecompressionError",
                                  "CompressedDataMissing", "InvalidChunkHeader", "MissingChunk", "InvalidLength",
                                  "UnexpectedEOF", "InvalidUTF8", "InvalidRemoteID", "InvalidVarInt", "InvalidContent",
                                  "GenericInvalidData", "ChecksumFailed", "DataMissing"};
    if (int(s) >= 0 && int(s) < 20) return names[s];
    switch (s) {
        case DTGPU_ERR_CHECKOUT: return "ErrCheckout";
        case DTGPU_ERR_CAPACITY: return "ErrCapacity";
        case DTGPU_ERR_HIP: return "ErrHip";
        case DTGPU_ERR_ARG: return "ErrArg";
        case DTGPU_ERR_NO_DEVICE: return "ErrNoDevice";
        default: return "Unknown";
    }
}

}  // extern "C"
