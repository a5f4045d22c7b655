// dtgpu_decode.cpp -- C ABI of the batched GPU `.dt` decoder (include/dtgpu.h, dtgpu_decode_*).
//
// Staging: the documents are packed into one HBM arena (256-B aligned, 256 B of padding each so
// the decoder's register windows never read past the allocation), a sizing pass of the decode
// kernel reads the chunk directory and the OpVersions stream, and the output arenas are
// allocated from its counts.  dtgpu_decode_run is then the full decode, entirely on the device.
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <atomic>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/dtgpu.h"
#include "dt_decoded.hpp"
#include "dt_host.hpp"

using namespace dtgpu;

namespace {

uint32_t multmodp_host(uint32_t a, uint32_t b) {
    if (!a) return 0;
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1u) ? (b >> 1) ^ 0x82F63B78u : b >> 1;
    }
    return p;
}

uint64_t align256(uint64_t x) { return (x + 255) & ~uint64_t(255); }

// Process-wide pinned staging chunks for document uploads (allocated once, reused by every batch;
// each upload ends with its stream synchronised, so the next one finds both chunks idle).
struct Staging {
    std::mutex mu;
    uint8_t *buf[2] = {nullptr, nullptr};
};
Staging &staging() {
    static Staging *st = new Staging();   // (never destroyed: pinned memory outlives static teardown)
    return *st;
}
constexpr uint64_t kStageChunk = 64ull << 20;

// The documents into dst (their DecodeDesc offsets, zero padding up to the next document) on
// stream s: packed on nt host threads into a pinned chunk, one async copy per chunk, two chunks
// alternating.  A document larger than a chunk is copied from the caller's buffer directly.
Status upload_packed(uint8_t *dst, uint64_t total, const uint8_t *const *docs, const size_t *lens, size_t n,
                     const std::vector<DecodeDesc> &desc, int nt, hipStream_t s) {
    if (!total) return OK;
    Staging &st = staging();
    std::lock_guard<std::mutex> lock(st.mu);
    for (int k = 0; k < 2; k++)
        if (!st.buf[k] && DTGPU_HIP_FAILED(hipHostMalloc(reinterpret_cast<void **>(&st.buf[k]), kStageChunk, hipHostMallocPortable)))
            return ErrHip;
    struct Ev {   // this upload's copy-done events, one per chunk
        hipEvent_t e[2] = {nullptr, nullptr};
        bool rec[2] = {false, false};
        ~Ev() { for (hipEvent_t x : e) if (x) (void)hipEventDestroy(x); }
    } ev;
    for (int k = 0; k < 2; k++)
        if (DTGPU_HIP_FAILED(hipEventCreateWithFlags(&ev.e[k], hipEventDisableTiming))) return ErrHip;
    auto end_of = [&](size_t i) { return i + 1 < n ? desc[i + 1].in_off : total; };
    size_t i = 0;
    int k = 0;
    while (i < n) {
        const uint64_t base = desc[i].in_off;
        size_t j = i;
        while (j < n && end_of(j) - base <= kStageChunk) j++;
        if (j == i) {   // one document larger than a chunk: straight from the caller's memory
            if ((lens[i] && DTGPU_HIP_FAILED(hipMemcpyAsync(dst + base, docs[i], lens[i], hipMemcpyHostToDevice, s))) ||
                DTGPU_HIP_FAILED(hipMemsetAsync(dst + base + lens[i], 0, end_of(i) - base - lens[i], s)) ||
                DTGPU_HIP_FAILED(hipStreamSynchronize(s)))
                return ErrHip;
            i++;
            continue;
        }
        if (ev.rec[k] && DTGPU_HIP_FAILED(hipEventSynchronize(ev.e[k]))) return ErrHip;   // the chunk's last copy is done
        uint8_t *chunk = st.buf[k];
        std::atomic<size_t> next{i};
        auto work = [&] {
            for (size_t q; (q = next.fetch_add(1)) < j;) {
                uint8_t *p = chunk + (desc[q].in_off - base);
                if (lens[q]) std::memcpy(p, docs[q], lens[q]);
                std::memset(p + lens[q], 0, end_of(q) - desc[q].in_off - lens[q]);
            }
        };
        const int w = int(std::min<size_t>(size_t(nt), (j - i) / 16 + 1));
        std::vector<std::thread> pool;
        for (int t = 1; t < w; t++) pool.emplace_back(work);
        work();
        for (auto &th : pool) th.join();
        if (DTGPU_HIP_FAILED(hipMemcpyAsync(dst + base, chunk, end_of(j - 1) - base, hipMemcpyHostToDevice, s)) ||
            DTGPU_HIP_FAILED(hipEventRecord(ev.e[k], s)))
            return ErrHip;
        ev.rec[k] = true;
        k ^= 1;
        i = j;
    }
    return DTGPU_HIP_FAILED(hipStreamSynchronize(s)) ? ErrHip : OK;
}

}  // namespace

extern "C" {

dtgpu_status dtgpu_decode_create(const uint8_t *const *docs, const size_t *lens, size_t n,
                                 const dtgpu_batch_opts *opts, dtgpu_decoded **out) {
    if (!out || (n && (!docs || !lens))) return DTGPU_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return DTGPU_ERR_NO_DEVICE;
    stage_prof(nullptr);
    auto D = new dtgpu_decoded();
    std::unique_ptr<dtgpu_decoded> guard(D);
    D->device = opts ? opts->device : 0;
#define CK(x) do { if (DTGPU_HIP_FAILED(x)) return DTGPU_ERR_HIP; } while (0)
    CK(hipSetDevice(D->device));
    CK(hipStreamCreateWithFlags(&D->stream, hipStreamNonBlocking));
    CK(hipEventCreate(&D->ev0));
    CK(hipEventCreate(&D->ev1));
    hipStream_t s = D->stream;
    D->n = n;
    D->desc.assign(n, DecodeDesc{});
    D->res.assign(n, DecodeResult{});
    // documents into one arena
    uint64_t total = 0;
    for (size_t i = 0; i < n; i++) {
        if (lens[i] >= (1ull << 31)) return DTGPU_ERR_ARG;
        D->desc[i].in_off = total;
        D->desc[i].in_len = uint32_t(lens[i]);
        D->desc[i].ignore_crc = opts && opts->ignore_crc ? 1u : 0u;
        total = align256(total + lens[i] + 256);
        D->in_bytes += lens[i];
    }
    {   // one device arena: the documents are packed into pinned staging chunks on host threads
        // (only each document's padding is zeroed) and each chunk is copied while the next one is
        // packed -- no transient host copy of the whole batch (at 10k friendsforever documents a
        // 360 MB buffer spent ~100 ms in page faults and unmapping alone)
        CK(D->in.alloc(total));
        int nt = opts && opts->host_threads > 0 ? opts->host_threads : int(std::thread::hardware_concurrency());
        nt = int(std::max<size_t>(1, std::min<size_t>({size_t(std::max(nt, 1)), size_t(16), n / 64 + 1})));
        if (Status e = upload_packed(D->in.p, total, docs, lens, n, D->desc, nt, s)) return dtgpu_status(e);
        stage_prof("decode: upload documents");
    }
    CK(D->d_desc.upload(D->desc, s));
    CK(D->d_res.alloc(n));
    DecodeParams &P = D->P;
    P.in = D->in.p;
    P.docs = D->d_desc.p;
    P.results = D->d_res.p;
    P.n_docs = uint32_t(n);
    P.x2n[0] = 1u << 30;
    for (int k = 1; k < 32; k++) P.x2n[k] = multmodp_host(P.x2n[k - 1], P.x2n[k - 1]);
    // sizing pass
    P.size_only = 1;
    P.max_file_agents = 0;
    P.lz_ring = 0;
    if (launch_decode(P, s)) return DTGPU_ERR_HIP;
    CK(hipMemcpyAsync(D->res.data(), D->d_res.p, n * sizeof(DecodeResult), hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    stage_prof("decode: sizing pass");
    if (getenv("DTGPU_STAGE_PROF") && n) {   // core cycles per sizing phase: header + LZ4 claim, chunks, OpVersions
        double a[3] = {0, 0, 0}, m[3] = {0, 0, 0};
        for (size_t i = 0; i < n; i++)
            for (int k = 0; k < 3; k++) { a[k] += D->res[i].prof[k]; m[k] = std::max<double>(m[k], D->res[i].prof[k]); }
        fprintf(stderr, "[stage] sizing cycles/doc avg %.0f %.0f %.0f max %.0f %.0f %.0f\n", a[0] / n, a[1] / n, a[2] / n, m[0], m[1], m[2]);
    }
    // arenas from the sizing pass
    uint64_t lz = 0, ar = 0, pre = 0, ops = 0, ent = 0, poff = 0, par = 0, content = 0, lv = 0, ag = 0, ver = 0;
    uint32_t max_f = 0;
    uint64_t max_lz = 0;
    // LVs from which a document defers its per-LV offsets (DTGPU_FILL_MIN overrides)
    const uint64_t FILL_BIG = getenv("DTGPU_FILL_MIN") ? strtoull(getenv("DTGPU_FILL_MIN"), nullptr, 10) : 131072;
    uint64_t fill_words = 0;
    std::vector<uint32_t> fill_doc;
    for (size_t i = 0; i < n; i++) {
        DecodeDesc &d = D->desc[i];
        const DecodeResult &r = D->res[i];
        if (r.status == DECODE_DEFER || r.n_file_agents > DECODE_MAX_FILE_AGENTS) d.skip = 1;
        d.lz_off = lz;
        d.lz_cap = r.lz_len;
        lz = align256(lz + r.lz_len + 256);
        d.arun_off = ar;
        d.arun_cap = r.raw_aruns;
        ar += r.raw_aruns;
        d.pre_off = pre;
        d.pre_cap = r.tp_bytes + r.cik_bytes + r.raw_aruns + 1;
        pre += d.pre_cap;
        d.ent_off = ent;
        d.ent_cap = r.hist_bytes / 2 + 1;
        ent += d.ent_cap;
        d.poff_off = poff;
        poff += d.ent_cap + 1;
        d.op_off = ops;
        d.op_cap = d.pre_cap + d.ent_cap;
        ops += d.op_cap;
        d.par_off = par;
        d.par_cap = r.hist_bytes;
        par += r.hist_bytes;
        d.content_off = content;
        d.content_cap = uint32_t(std::min<uint64_t>(uint64_t(d.in_len) + r.lz_len, 0xFFFFFFFFull));
        content += d.content_cap;
        d.lv_off = lv;
        d.lv_cap = uint32_t(r.n_lv);
        lv += r.n_lv;
        d.agent_off = ag;
        d.agent_cap = r.n_file_agents;
        ag += r.n_file_agents;
        d.ver_off = ver;
        ver += DECODE_MAX_FRONTIER;
        if (!d.skip) max_f = std::max(max_f, r.n_file_agents);
        if (!d.skip) max_lz = std::max<uint64_t>(max_lz, r.lz_len);
        // a long document hands its per-LV offsets to fill_kernel: about one job per 64-varint
        // batch of op records (a document that needs more fills the rest inline)
        d.fill_off = 0; d.fill_job0 = 0; d.fill_cap = 0; d.fill_copy = 0;
        if (!d.skip && r.n_lv >= FILL_BIG && !getenv("DTGPU_NO_FILL_DEFER")) {
            d.fill_off = fill_words;
            d.fill_job0 = uint32_t(fill_doc.size());
            d.fill_cap = r.tp_bytes / 32 + 64;
            d.fill_copy = d.content_cap / 4096 + 1;   // the insert text, 4 KB per slot
            fill_words += 68 + uint64_t(d.fill_cap) * 132;
            fill_doc.insert(fill_doc.end(), size_t(d.fill_cap) + d.fill_copy, uint32_t(i));
        }
    }
    if (!fill_doc.empty()) {
        CK(D->fill.alloc(fill_words));
        CK(D->fill_n.alloc(n));
        CK(D->fill_doc.alloc(fill_doc.size()));
        CK(hipMemcpyAsync(D->fill_doc.p, fill_doc.data(), fill_doc.size() * 4, hipMemcpyHostToDevice, s));
    }
    CK(D->lz.alloc(lz));
    CK(D->aruns.alloc(4 * ar));
    CK(D->alist.alloc(4 * ar));
    CK(D->pre.alloc(4 * pre));
    CK(D->ops.alloc(4 * ops));
    CK(D->ent.alloc(2 * ent));
    CK(D->poff.alloc(poff));
    CK(D->par.alloc(par));
    CK(D->content.alloc(content));
    CK(D->cbyte.alloc(lv));
    CK(D->agents.alloc(2 * ag));
    CK(D->ver.alloc(ver));
    CK(D->d_desc.upload(D->desc, s));
    P.docs = D->d_desc.p;
    P.lz = D->lz.p;
    P.aruns = D->aruns.p; P.alist = D->alist.p; P.pre = D->pre.p; P.ops = D->ops.p;
    P.ent = D->ent.p; P.poff = D->poff.p; P.par = D->par.p; P.cbyte = D->cbyte.p;
    P.agents = D->agents.p; P.ver = D->ver.p; P.content = D->content.p;
    P.size_only = 0;
    P.max_file_agents = std::max<uint32_t>(max_f, 1);
    // a long LZ4 block bounds the batch's decode: lz4_kernel decompresses those first, two waves
    // per document (its resolved-source ring included); decode_kernel then needs no ring, whose
    // 4 KB of LDS per wave would cost the small documents occupancy
    // decode_kernel dispatches the longest documents first (a batch with long ones only: they
    // bound it, and a late start would add to the tail)
    P.order = nullptr;
    if (n > 1 && (max_lz >= 65536 || !fill_doc.empty())) {
        std::vector<uint32_t> ord(n);
        for (size_t i = 0; i < n; i++) ord[i] = uint32_t(i);
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) {
            return uint64_t(D->desc[a].in_len) + D->res[a].lz_len > uint64_t(D->desc[b].in_len) + D->res[b].lz_len;
        });
        CK(D->order.alloc(n));
        CK(hipMemcpyAsync(D->order.p, ord.data(), n * 4, hipMemcpyHostToDevice, s));
        P.order = D->order.p;
    }
    P.fill = fill_doc.empty() ? nullptr : D->fill.p;
    P.fill_n = fill_doc.empty() ? nullptr : D->fill_n.p;
    P.fill_doc = fill_doc.empty() ? nullptr : D->fill_doc.p;
    P.fill_blocks = uint32_t(fill_doc.size());
    P.lz_ring = 0;
    P.n_big = 0;
    P.lz_big = nullptr;
    P.lz_pre = nullptr;
    // a block this long gets lz4_kernel (DTGPU_LZ_PRE_MIN overrides; DTGPU_NO_LZ_PRE: never)
    const uint64_t LZ_BIG = getenv("DTGPU_LZ_PRE_MIN") ? strtoull(getenv("DTGPU_LZ_PRE_MIN"), nullptr, 10) : 65536;
    if (max_lz >= LZ_BIG && !getenv("DTGPU_NO_LZ_PRE")) {
        std::vector<uint32_t> big;
        for (size_t i = 0; i < n; i++)
            if (!D->desc[i].skip && D->res[i].lz_len >= LZ_BIG) big.push_back(uint32_t(i));
        // longest blocks first: they are dispatched first, each to a CU of its own
        std::stable_sort(big.begin(), big.end(), [&](uint32_t a, uint32_t b) { return D->res[a].lz_len > D->res[b].lz_len; });
        CK(D->lz_big.alloc(big.size()));
        CK(hipMemcpyAsync(D->lz_big.p, big.data(), big.size() * 4, hipMemcpyHostToDevice, s));
        CK(D->lz_pre.alloc(n));
        CK(hipMemsetAsync(D->lz_pre.p, 0, n * 4, s));
        P.lz_big = D->lz_big.p;
        P.lz_pre = D->lz_pre.p;
        P.n_big = uint32_t(big.size());
        // three waves per block up to this many blocks (DTGPU_LZ3_MAX overrides): with the longest
        // first, 1,600 linear blocks decode in 11.4 ms on three (12.4 on two) while 10,000
        // git-makefile blocks take 55.6 ms on three (47.4 on two)
        P.lz3_max = getenv("DTGPU_LZ3_MAX") ? uint32_t(strtoul(getenv("DTGPU_LZ3_MAX"), nullptr, 10)) : 4096u;
    }
    CK(hipStreamSynchronize(s));
    stage_prof("decode: arenas");
#undef CK
    *out = guard.release();
    return DTGPU_OK;
}

dtgpu_status dtgpu_decode_run(dtgpu_decoded *D, float *ms) {
    if (!D || D->merged) return DTGPU_ERR_ARG;
    if (hipSetDevice(D->device) != hipSuccess) return DTGPU_ERR_HIP;
    if (hipEventRecord(D->ev0, D->stream) != hipSuccess) return DTGPU_ERR_HIP;
    if (launch_decode(D->P, D->stream)) return DTGPU_ERR_HIP;
    if (hipEventRecord(D->ev1, D->stream) != hipSuccess) return DTGPU_ERR_HIP;
    if (hipMemcpyAsync(D->res.data(), D->d_res.p, D->n * sizeof(DecodeResult), hipMemcpyDeviceToHost, D->stream) !=
        hipSuccess)
        return DTGPU_ERR_HIP;
    if (hipStreamSynchronize(D->stream) != hipSuccess) return DTGPU_ERR_HIP;
    float t = 0;
    if (hipEventElapsedTime(&t, D->ev0, D->ev1) != hipSuccess) return DTGPU_ERR_HIP;
    D->last_ms = t;
    if (ms) *ms = t;
    return DTGPU_OK;
}

// ListOpLog::decode_and_add_opts for a batch (decode_oplog.rs:476-583): patch i merged into
// document i of `base` on the device (dt_decode.hip decode_add_kernel).  Staging: the patches go to
// HBM, the decoder's sizing pass reads their chunk directories (a StartBranch version is not an
// error there), and the merged arenas are sized from the resident counts plus the patch counts.
dtgpu_status dtgpu_decode_add(const dtgpu_decoded *B, const uint8_t *const *patches, const size_t *lens, size_t n,
                              int ignore_crc, float *ms, dtgpu_decoded **out) {
    if (!B || !out || n != B->n || (n && (!patches || !lens))) return DTGPU_ERR_ARG;
    auto M = new dtgpu_decoded();
    std::unique_ptr<dtgpu_decoded> guard(M);
    M->device = B->device;
    M->merged = true;
#define CK(x) do { if (DTGPU_HIP_FAILED(x)) return DTGPU_ERR_HIP; } while (0)
    CK(hipSetDevice(M->device));
    CK(hipStreamCreateWithFlags(&M->stream, hipStreamNonBlocking));
    CK(hipEventCreate(&M->ev0));
    CK(hipEventCreate(&M->ev1));
    hipStream_t s = M->stream;
    M->n = n;
    // the patches, packed like dtgpu_decode_create's documents
    std::vector<DecodeDesc> pd(n, DecodeDesc{});
    uint64_t ptotal = 0;
    for (size_t i = 0; i < n; i++) {
        if (lens[i] >= (1ull << 31)) return DTGPU_ERR_ARG;
        pd[i].in_off = ptotal;
        pd[i].in_len = uint32_t(lens[i]);
        pd[i].patch = 1;
        ptotal = align256(ptotal + lens[i] + 256);
        M->in_bytes += lens[i];
    }
    DevBuf<uint8_t> pin;
    {
        std::vector<uint8_t> host(ptotal, 0);
        for (size_t i = 0; i < n; i++)
            if (lens[i]) std::memcpy(host.data() + pd[i].in_off, patches[i], lens[i]);
        CK(pin.upload(host, s));
    }
    DevBuf<DecodeDesc> d_pd;
    DevBuf<DecodeResult> d_pr;
    CK(d_pd.upload(pd, s));
    CK(d_pr.alloc(n));
    std::vector<DecodeResult> pr(n);
    {   // sizing pass over the patches
        DecodeParams P{};
        P.in = pin.p;
        P.docs = d_pd.p;
        P.results = d_pr.p;
        P.n_docs = uint32_t(n);
        P.size_only = 1;
        if (launch_decode(P, s)) return DTGPU_ERR_HIP;
        CK(hipMemcpyAsync(pr.data(), d_pr.p, n * sizeof(DecodeResult), hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
    }
    // merged arenas
    std::vector<AddDesc> ad(n, AddDesc{});
    M->desc.assign(n, DecodeDesc{});
    uint64_t in = 0, lz = 0, ar = 0, ops = 0, ent = 0, poff = 0, par = 0, content = 0, lv = 0, ag = 0, ver = 0, scr = 0;
    uint32_t max_f = 1, max_a = 1;
    constexpr uint32_t kAddMaxAgents = (160 * 1024 / 4 - 512 - 2 * DECODE_MAX_FILE_AGENTS) / 3;
    for (size_t i = 0; i < n; i++) {
        const DecodeDesc &bd = B->desc[i];
        const DecodeResult &br = B->res[i];
        const DecodeResult &r = pr[i];
        AddDesc &a = ad[i];
        DecodeDesc &md = M->desc[i];
        a.skip = br.status != 0 || r.status == DECODE_DEFER || r.n_file_agents > DECODE_MAX_FILE_AGENTS;
        a.ignore_crc = ignore_crc ? 1u : 0u;
        a.b_in = bd.in_off; a.b_arun = bd.arun_off; a.b_op = bd.op_off; a.b_ent = bd.ent_off; a.b_poff = bd.poff_off;
        a.b_par = bd.par_off; a.b_content = bd.content_off; a.b_lv = bd.lv_off; a.b_agent = bd.agent_off; a.b_ver = bd.ver_off;
        a.b_in_len = bd.in_len;
        const bool bok = br.status == 0;
        a.b_n_aruns = bok ? br.n_aruns : 0; a.b_n_ops = bok ? br.n_ops : 0; a.b_n_ent = bok ? br.n_entries : 0;
        a.b_n_par = bok ? br.n_parents : 0; a.b_n_content = bok ? br.n_content : 0; a.b_n_agents = bok ? br.n_agents : 0;
        a.b_n_ver = bok ? br.n_version : 0; a.b_n_lv = bok ? uint32_t(br.n_lv) : 0;
        a.b_complete = bok ? br.content_complete : 1; a.b_ascii = bok ? br.ascii : 1;
        a.b_doc_id_off = br.doc_id_off; a.b_doc_id_len = bok ? br.doc_id_len : 0xFFFFFFFFu;
        a.p_off = pd[i].in_off;
        a.p_len = uint32_t(lens[i]);
        a.p_rel = uint32_t(align256(uint64_t(bd.in_len) + 256));
        a.m_in = in;
        in = align256(in + a.p_rel + a.p_len + 256);
        a.lz_off = lz; a.lz_cap = r.lz_len;
        lz = align256(lz + r.lz_len + 256);
        // pieces: records split at the resident's run boundaries
        const uint64_t pieces = uint64_t(r.raw_aruns) + 2ull * a.b_n_aruns + 1;
        a.c_vm = uint32_t(pieces);
        a.c_pre = uint32_t(1 + r.tp_bytes + r.cik_bytes + pieces);
        a.c_arun = uint32_t(a.b_n_aruns + pieces);
        a.c_ent = uint32_t(a.b_n_ent + r.hist_bytes / 2 + 1 + pieces);
        a.c_par = uint32_t(a.b_n_par + r.hist_bytes + pieces);
        a.c_op = uint32_t(a.b_n_ops + a.c_pre + a.c_ent);
        a.c_content = uint32_t(std::min<uint64_t>(uint64_t(a.b_n_content) + a.p_len + r.lz_len, 0xFFFFFFFFull));
        a.c_lv = uint32_t(std::min<uint64_t>(uint64_t(a.b_n_lv) + r.n_lv, 0xFFFFFFFFull));
        a.c_agent = a.b_n_agents + r.n_file_agents;
        // the kernel's per-agent LDS tables (launch_decode_add: 512 + 2 max_file_agents + 3
        // max_agents words) must fit the CU's 160 KiB for the batch's largest document: with
        // n_file_agents <= DECODE_MAX_FILE_AGENTS that holds for every merged agent count up to
        // kAddMaxAgents, and a document past it is deferred to the host alone (never failing the batch)
        if (a.c_agent > kAddMaxAgents) a.skip = 1;
        a.m_arun = ar; ar += a.c_arun;
        a.m_op = ops; ops += a.c_op;
        a.m_ent = ent; ent += a.c_ent;
        a.m_poff = poff; poff += a.c_ent + 1;
        a.m_par = par; par += a.c_par;
        a.m_content = content; content += a.c_content;
        a.m_lv = lv; lv += a.c_lv;
        a.m_agent = ag; ag += a.c_agent;
        a.m_ver = ver; ver += DECODE_MAX_FRONTIER;
        a.m_scr = scr; scr += uint64_t(a.c_pre) + a.c_vm;
        if (!a.skip) { max_f = std::max(max_f, r.n_file_agents); max_a = std::max(max_a, a.c_agent); }
        md.in_off = a.m_in; md.in_len = a.p_rel + a.p_len;
        md.arun_off = a.m_arun; md.op_off = a.m_op; md.ent_off = a.m_ent; md.poff_off = a.m_poff; md.par_off = a.m_par;
        md.content_off = a.m_content; md.lv_off = a.m_lv; md.agent_off = a.m_agent; md.ver_off = a.m_ver;
        md.arun_cap = a.c_arun; md.op_cap = a.c_op; md.ent_cap = a.c_ent; md.par_cap = a.c_par;
        md.content_cap = a.c_content; md.lv_cap = a.c_lv; md.agent_cap = a.c_agent;
    }
    CK(M->in.alloc(in)); CK(M->lz.alloc(lz)); CK(M->aruns.alloc(4 * ar)); CK(M->ops.alloc(4 * ops));
    CK(M->ent.alloc(2 * ent)); CK(M->poff.alloc(poff)); CK(M->par.alloc(par)); CK(M->content.alloc(content));
    CK(M->cbyte.alloc(lv)); CK(M->agents.alloc(2 * ag)); CK(M->ver.alloc(ver)); CK(M->ffr.alloc(ver));
    DevBuf<uint32_t> d_scr;
    CK(d_scr.alloc(4 * scr));
    DevBuf<AddDesc> d_ad;
    CK(d_ad.upload(ad, s));
    CK(M->d_res.alloc(n));
    AddParams A{};
    A.b_in = B->in.p; A.b_content = B->content.p; A.p_in = pin.p;
    A.b_aruns = B->aruns.p; A.b_ops = B->ops.p; A.b_ent = B->ent.p; A.b_poff = B->poff.p; A.b_par = B->par.p;
    A.b_cbyte = B->cbyte.p; A.b_agents = B->agents.p; A.b_ver = B->ver.p;
    A.m_in = M->in.p; A.lz = M->lz.p; A.m_content = M->content.p;
    A.m_aruns = M->aruns.p; A.m_ops = M->ops.p; A.m_ent = M->ent.p; A.m_poff = M->poff.p; A.m_par = M->par.p;
    A.m_cbyte = M->cbyte.p; A.m_agents = M->agents.p; A.m_ver = M->ver.p; A.m_ffr = M->ffr.p; A.scr = d_scr.p;
    A.docs = d_ad.p; A.results = M->d_res.p; A.n_docs = uint32_t(n); A.max_file_agents = max_f; A.max_agents = max_a;
    A.x2n[0] = 1u << 30;
    for (int k = 1; k < 32; k++) A.x2n[k] = multmodp_host(A.x2n[k - 1], A.x2n[k - 1]);
    CK(hipEventRecord(M->ev0, s));
    if (launch_decode_add(A, s)) return DTGPU_ERR_HIP;
    CK(hipEventRecord(M->ev1, s));
    M->res.assign(n, DecodeResult{});
    CK(hipMemcpyAsync(M->res.data(), M->d_res.p, n * sizeof(DecodeResult), hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    float t = 0;
    CK(hipEventElapsedTime(&t, M->ev0, M->ev1));
    M->last_ms = t;
    if (ms) *ms = t;
#undef CK
    // each merged document is valid (the resident one again after a failed merge); the merge's
    // own status is kept apart
    M->add_status.assign(n, 0);
    for (size_t i = 0; i < n; i++) {
        M->add_status[i] = M->res[i].status;
        M->res[i].status = B->res[i].status;
    }
    *out = guard.release();
    return DTGPU_OK;
}

dtgpu_status dtgpu_decode_add_result(const dtgpu_decoded *M, size_t i, uint64_t *frontier, size_t cap,
                                     size_t *n_frontier) {
    if (!M || !M->merged || i >= M->n || (!frontier && cap)) return DTGPU_ERR_ARG;
    const uint32_t st = M->add_status[i];
    const size_t k = st == 0 ? M->res[i].n_file_frontier : 0;
    if (n_frontier) *n_frontier = k;
    if (k && cap) {
        std::vector<uint32_t> f(k);
        if (hipMemcpy(f.data(), M->ffr.p + M->desc[i].ver_off, k * 4, hipMemcpyDeviceToHost) != hipSuccess)
            return DTGPU_ERR_HIP;
        for (size_t j = 0; j < k && j < cap; j++) frontier[j] = f[j];
    }
    return dtgpu_status(st);
}

size_t dtgpu_decode_size(const dtgpu_decoded *D) { return D ? D->n : 0; }

dtgpu_status dtgpu_decode_status(const dtgpu_decoded *D, size_t i, uint64_t out[12]) {
    if (!D || i >= D->n || !out) return DTGPU_ERR_ARG;
    const DecodeResult &r = D->res[i];
    out[0] = r.status; out[1] = r.n_lv; out[2] = r.n_ops; out[3] = r.n_aruns; out[4] = r.n_entries;
    out[5] = r.n_parents; out[6] = r.n_content; out[7] = r.n_version; out[8] = r.n_agents;
    out[9] = r.content_complete; out[10] = r.ascii; out[11] = r.n_file_agents;
    return DTGPU_OK;
}

size_t dtgpu_decode_export(const dtgpu_decoded *D, size_t i, int what, void *out, size_t cap) {
    if (!D || i >= D->n) return 0;
    const DecodeDesc &d = D->desc[i];
    const DecodeResult &r = D->res[i];
    if (r.status != 0) return 0;
    const void *src = nullptr;
    size_t count = 0, elem = 4;
    switch (what) {
        case DTGPU_EXPORT_OPS: src = D->ops.p + 4 * d.op_off; count = r.n_ops; elem = 16; break;
        case DTGPU_EXPORT_AGENT_RUNS: src = D->aruns.p + 4 * d.arun_off; count = r.n_aruns; elem = 16; break;
        case DTGPU_EXPORT_ENTRIES: src = D->ent.p + 2 * d.ent_off; count = r.n_entries; elem = 8; break;
        case DTGPU_EXPORT_PARENT_OFFSETS: src = D->poff.p + d.poff_off; count = r.n_entries + 1; break;
        case DTGPU_EXPORT_PARENTS: src = D->par.p + d.par_off; count = r.n_parents; break;
        case DTGPU_EXPORT_CONTENT: src = D->content.p + d.content_off; count = r.n_content; elem = 1; break;
        case DTGPU_EXPORT_CHAR_OFFSETS: src = D->cbyte.p + d.lv_off; count = size_t(r.n_lv); break;
        case DTGPU_EXPORT_VERSION: src = D->ver.p + d.ver_off; count = r.n_version; break;
        case DTGPU_EXPORT_AGENT_NAMES: {   // u8 length + bytes per agent, in agent-id order
            std::vector<uint32_t> pairs(2 * size_t(r.n_agents));
            if (!pairs.empty() &&
                hipMemcpy(pairs.data(), D->agents.p + 2 * d.agent_off, pairs.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
                return 0;
            std::vector<uint8_t> doc(d.in_len);
            if (d.in_len && hipMemcpy(doc.data(), D->in.p + d.in_off, d.in_len, hipMemcpyDeviceToHost) != hipSuccess)
                return 0;
            std::vector<uint8_t> blob;
            for (uint32_t a = 0; a < r.n_agents; a++) {
                blob.push_back(uint8_t(pairs[2 * a + 1]));
                blob.insert(blob.end(), doc.begin() + pairs[2 * a], doc.begin() + pairs[2 * a] + pairs[2 * a + 1]);
            }
            if (out) std::memcpy(out, blob.data(), std::min(cap, blob.size()));
            return blob.size();
        }
        case DTGPU_EXPORT_DOC_ID: {
            std::vector<uint8_t> blob(1, 0);
            if (r.doc_id_len != 0xFFFFFFFFu) {
                blob[0] = 1;
                blob.resize(1 + r.doc_id_len);
                if (r.doc_id_len &&
                    hipMemcpy(blob.data() + 1, D->in.p + d.in_off + r.doc_id_off, r.doc_id_len, hipMemcpyDeviceToHost) != hipSuccess)
                    return 0;
            }
            if (out) std::memcpy(out, blob.data(), std::min(cap, blob.size()));
            return blob.size();
        }
        default: return 0;
    }
    if (out && count) {
        const size_t k = std::min(cap, count);
        if (hipMemcpy(out, src, k * elem, hipMemcpyDeviceToHost) != hipSuccess) return 0;
    }
    return count;
}

uint64_t dtgpu_decode_bytes(const dtgpu_decoded *D, int which) {
    if (!D) return 0;
    if (which == 0) return D->in_bytes;
    // SoA written: 16 B per op run and agent run, 8 per entry (+4 per CSR slot), 4 per parent,
    // the inserted bytes and 4 per LV of content offsets
    uint64_t b = 0;
    for (size_t i = 0; i < D->n; i++) {
        const DecodeResult &r = D->res[i];
        if (r.status) continue;
        b += 16ull * (r.n_ops + r.n_aruns) + 12ull * r.n_entries + 4 + 4ull * r.n_parents + r.n_content + 4ull * r.n_lv;
    }
    return b;
}

dtgpu_status dtgpu_decode_profile(const dtgpu_decoded *D, size_t i, uint32_t out[8]) {
    if (!D || i >= D->n || !out) return DTGPU_ERR_ARG;
    for (int k = 0; k < 8; k++) out[k] = D->res[i].prof[k];
    return DTGPU_OK;
}

float dtgpu_decode_last_ms(const dtgpu_decoded *D) { return D ? D->last_ms : 0.f; }

void dtgpu_decode_free(dtgpu_decoded *D) { delete D; }

}  // extern "C"
