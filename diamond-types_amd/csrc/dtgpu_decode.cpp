// dtgpu_decode.cpp -- C ABI of the batched GPU `.dt` decoder (include/dtgpu.h, dtgpu_decode_*).
//
// Staging: the documents are packed into one HBM arena (256-B aligned, 256 B of padding each so
// the decoder's register windows never read past the allocation), a sizing pass of the decode
// kernel reads the chunk directory and the OpVersions stream, and the output arenas are
// allocated from its counts.  dtgpu_decode_run is then the full decode, entirely on the device.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>
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

}  // namespace

extern "C" {

dtgpu_status dtgpu_decode_create(const uint8_t *const *docs, const size_t *lens, size_t n,
                                 const dtgpu_batch_opts *opts, dtgpu_decoded **out) {
    if (!out || (n && (!docs || !lens))) return DTGPU_ERR_ARG;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return DTGPU_ERR_NO_DEVICE;
    auto D = new dtgpu_decoded();
    std::unique_ptr<dtgpu_decoded> guard(D);
    D->device = opts ? opts->device : 0;
#define CK(x) do { if ((x) != hipSuccess) return DTGPU_ERR_HIP; } while (0)
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
    {
        std::vector<uint8_t> host(total, 0);
        for (size_t i = 0; i < n; i++)
            if (lens[i]) std::memcpy(host.data() + D->desc[i].in_off, docs[i], lens[i]);
        CK(D->in.upload(host, s));
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
    if (launch_decode(P, s)) return DTGPU_ERR_HIP;
    CK(hipMemcpyAsync(D->res.data(), D->d_res.p, n * sizeof(DecodeResult), hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    // arenas from the sizing pass
    uint64_t lz = 0, ar = 0, pre = 0, ops = 0, ent = 0, poff = 0, par = 0, content = 0, lv = 0, ag = 0, ver = 0;
    uint32_t max_f = 0;
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
    CK(hipStreamSynchronize(s));
#undef CK
    *out = guard.release();
    return DTGPU_OK;
}

dtgpu_status dtgpu_decode_run(dtgpu_decoded *D, float *ms) {
    if (!D) return DTGPU_ERR_ARG;
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
