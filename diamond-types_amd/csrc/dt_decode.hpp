// dt_decode.hpp -- host/device layout of the batched `.dt` decoder (dt_decode.hip).
//
// One 64-lane wavefront decodes one document (ListOpLog::load_from,
// src/list/encoding/decode_oplog.rs:447-960) into the same SoA runs the host decoder builds
// (dt_host.hpp HostOpLog): op runs split at graph-entry boundaries, agent runs, graph entries with
// sorted parents, inserted content with a per-LV byte offset, and the frontier.  A sizing pass
// (size_only) reads the chunk directory and the OpVersions stream to size every arena; the full
// pass then decodes with exact or upper-bound capacities.
#pragma once
#include <stdint.h>

namespace dtgpu {

// Arena capacities / offsets of one document.  Offsets are in elements of each arena.
struct DecodeDesc {
    uint64_t in_off;        // bytes; 256-B aligned with >= 256 B of readable padding after the doc
    uint64_t lz_off;        // bytes; the decompressed LZ4 buffer (same alignment / padding)
    uint64_t arun_off;      // quads (lv, len, agent, seq) -- also the per-agent lookup lists
    uint64_t pre_off;       // quads: op runs before the entry split
    uint64_t op_off;        // quads (lv, len, pos, kind | fwd << 1): the final op runs
    uint64_t ent_off;       // pairs (start, end)
    uint64_t poff_off;      // ent_cap + 1 words: parents CSR
    uint64_t par_off;       // words
    uint64_t content_off;   // bytes: inserted UTF-8 in LV order
    uint64_t lv_off;        // words: per-LV byte offset of an inserted char (~0 otherwise)
    uint64_t agent_off;     // pairs (name offset in the document, name length), by agent id
    uint64_t ver_off;       // words: the frontier (cg.version), <= 64 LVs
    uint32_t in_len, lz_cap, arun_cap, pre_cap, op_cap, ent_cap, par_cap, content_cap, lv_cap, agent_cap;
    uint32_t ignore_crc, skip;
    uint32_t patch, pad;    // sizing a patch for decode_and_add: a StartBranch version is not an error
    // a long document's deferred per-LV offsets (fill_kernel): its area in DecodeParams::fill
    // (words), its first job slot in the fill grid and its job capacity (0: filled inline)
    uint64_t fill_off;
    uint32_t fill_job0, fill_cap;
    uint32_t fill_copy, pad4;   // its fill-grid slots after the jobs: the insert text copied 4 KB each
};

struct DecodeResult {
    uint32_t status;        // dtgpu_status codes; DECODE_DEFER = decode this document on the host
    uint32_t n_file_agents, n_agents, n_aruns, n_pre, n_ops, n_entries, n_parents;
    uint32_t n_content, n_version, content_complete, ascii;
    uint64_t n_lv;
    // sizing pass (size_only): what the full pass needs
    uint32_t lz_len, tp_bytes, cik_bytes, hist_bytes, raw_aruns;
    uint32_t n_file_frontier;   // decode_and_add: the patch's version (decode_and_add's return value)
    uint32_t prof[8];       // core-clock cycles per decode phase (full pass)
    uint32_t doc_id_off, doc_id_len;   // the DocId bytes in the document (len ~0: none)
};

constexpr uint32_t DECODE_DEFER = 80;           // a case the device decoder hands to the host
constexpr uint32_t DECODE_MAX_FILE_AGENTS = 2048;
constexpr uint32_t DECODE_MAX_FRONTIER = 64;
constexpr uint32_t DECODE_MAX_PARENTS = 64;

struct DecodeParams {
    const uint8_t *in;
    uint8_t *lz;
    uint32_t *aruns, *alist, *pre, *ops, *ent, *poff, *par, *cbyte, *agents, *ver;
    uint8_t *content;
    const DecodeDesc *docs;
    DecodeResult *results;
    uint32_t n_docs, size_only, max_file_agents;
    uint32_t lz_ring;       // entries of the LZ4 copy's resolved-source ring in dynamic LDS (0: none)
    // documents with a long LZ4 block, decompressed first by lz4_kernel (two waves each: one
    // parses the next 64 sequences while the other copies the current ones); lz_pre[doc]:
    // 1 decompressed, 2 malformed (LZ4DecompressionError), 0 left to decode_kernel
    const uint32_t *lz_big;
    uint32_t *lz_pre;
    uint32_t n_big, lz3_max;   // lz3_max: three waves per block while n_big <= lz3_max
    // deferred per-LV offsets of long documents: job arena, each document's job count (written by
    // decode_kernel when its fast path succeeds), the document of each fill-grid slot, grid size
    uint32_t *fill;
    uint32_t *fill_n;
    const uint32_t *fill_doc;
    uint32_t fill_blocks, pad3;
    const uint32_t *order;  // decode_kernel's block -> document (longest first), or null
    uint32_t x2n[32];       // x^(2^k) mod the CRC-32C polynomial (crc32 combine tables)
};

int launch_decode(const DecodeParams &p, void *stream);

// decode_and_add (ListOpLog::decode_and_add_opts, decode_oplog.rs:476-583 and the overlap filter of
// decode_internal :670-913) on the device: one wavefront per (resident oplog, patch) pair.  The
// merged oplog goes to a new set of arenas: the resident arrays are copied, then the patch's new
// operations appended with the reference's RLE rules (agent runs, op runs, Graph::push); on an
// error the merged document is the resident one again (the reference's unwind).
struct AddDesc {
    // the resident oplog (a decoded handle's document)
    uint64_t b_in, b_arun, b_op, b_ent, b_poff, b_par, b_content, b_lv, b_agent, b_ver;
    uint32_t b_in_len, b_n_aruns, b_n_ops, b_n_ent, b_n_par, b_n_content, b_n_agents, b_n_ver, b_n_lv;
    uint32_t b_complete, b_ascii, b_doc_id_off, b_doc_id_len;
    // the patch: its bytes in the merged `in` region at p_rel, its LZ4 buffer
    uint32_t p_rel, p_len, lz_cap, pad0;
    uint64_t p_off, lz_off;   // the patch in the patch arena (copied to m_in + p_rel first)
    // merged arenas (offsets in elements) and capacities; scr: op-run pieces, then the version map
    uint64_t m_in, m_arun, m_op, m_ent, m_poff, m_par, m_content, m_lv, m_agent, m_ver, m_scr;
    uint32_t c_arun, c_op, c_ent, c_par, c_content, c_lv, c_agent, c_pre, c_vm;
    uint32_t ignore_crc, skip, pad1;
};

struct AddParams {
    const uint8_t *b_in, *b_content, *p_in;
    const uint32_t *b_aruns, *b_ops, *b_ent, *b_poff, *b_par, *b_cbyte, *b_agents, *b_ver;
    uint8_t *m_in, *lz, *m_content;
    uint32_t *m_aruns, *m_ops, *m_ent, *m_poff, *m_par, *m_cbyte, *m_agents, *m_ver, *m_ffr, *scr;
    const AddDesc *docs;
    DecodeResult *results;
    uint32_t n_docs, max_file_agents, max_agents, pad;   // max_agents: merged agents of any document
    uint32_t x2n[32];
};

int launch_decode_add(const AddParams &p, void *stream);

}  // namespace dtgpu
