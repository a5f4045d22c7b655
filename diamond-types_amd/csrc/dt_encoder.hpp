// dt_encoder.hpp -- host/device layout of the batched `.dt` encoder (dt_encoder.hip):
// ListOpLog::encode(opts) (src/list/encoding/encode_oplog.rs:404-747) from ROOT for every
// document of a device-staged batch, reading the decoded oplog in the decoder's arenas and the
// walk order in the planner's commands.  The bytes equal dt_encode.cpp's (the host encoder) for
// the same options.
#pragma once
#include <stdint.h>

#include "dt_host.hpp"

namespace dtgpu {

struct EncDesc {
    // decoder / planner arenas (offsets in each arena's units)
    uint64_t in_off;        // bytes: the document (agent names, doc id)
    uint64_t arun_off;      // quads (lv, len, agent, seq)
    uint64_t ent_off;       // pairs (start, end)
    uint64_t poff_off;      // words (ne + 1)
    uint64_t par_off;       // words
    uint64_t content_off;   // bytes: inserted UTF-8 in LV order
    uint64_t lv_off;        // words: per-LV byte offset into content
    uint64_t agent_off;     // pairs (name offset in the document, length)
    uint64_t cmd_off;       // Cmd units: the walk (INS / DEL commands in walk order, TOG between)
    uint32_t ncmd, n_aruns, ne, n_agents, n_lv, n_content, doc_id_off, doc_id_len;   // doc_id_len ~0: none
    // scratch and output
    uint64_t w_off;         // words: worder[ne], outpos[ne], op records (8 words), agent records (4),
                            //        txn heads (ne), agent map (n_agents)
    uint64_t b_off;         // bytes: walk-order text (n_content), then the LZ4 block (lz4_bound)
    uint64_t out_off;       // bytes
    uint32_t out_cap, skip;
};

struct EncResult {
    uint32_t status, len;
    uint32_t n_op_runs, n_agent_runs, n_txns, text_len, lz_len, stage;
    uint32_t n_mapped, aa_bytes, op_bytes, tx_bytes, nm_bytes, n_ins;   // kernel 1 -> kernel 2
    uint64_t prof[8];       // cycles: walk, records (ops), sizes, text + LZ4, write, CRC, txn heads, agent runs
    uint64_t lzcyc[3];      // LZ4 cycles: probing, extending, emitting
    uint32_t lzst[4];       // LZ4 counts: probe steps, steps with shared hashes, sequences, -
};

struct EncParams {
    const uint8_t *in, *content;
    const uint32_t *aruns, *ent, *poff, *par, *cbyte, *agents;
    const Cmd *cmds;
    uint32_t *w;
    uint8_t *b, *out;
    const EncDesc *docs;
    EncResult *results;
    uint32_t n_docs, flags, max_agents, prof;
    uint32_t lds_text, pad;   // text bytes kernel 2 stages in LDS (LZ4 input)
    uint32_t x2n[32];       // x^(2^k) mod the CRC-32C polynomial
};

inline uint64_t lz4_bound(uint64_t n) { return n + n / 255 + 16; }
inline uint64_t enc_words(uint32_t ne, uint32_t ncmd, uint32_t n_aruns, uint32_t n_agents) {
    return 2ull * ne + 8ull * ncmd + 4ull * (uint64_t(n_aruns) + ne) + ne + n_agents + 8;
}

int launch_encode(const EncParams &p, void *stream);

}  // namespace dtgpu
