// dt_encode.cpp -- `.dt` encoder: ListOpLog::encode / encode_from
// (src/list/encoding/encode_oplog.rs:404-747).
//
// The history is written in the reference's order, Graph::optimized_txns_between(from, tip)
// (a SpanningTreeWalker over the new spans, txn_trace.rs:356-360), through the same run mergers
// the reference uses, so the output is byte-identical to the reference encoder's whenever the
// same options are set (EncodeOptions, encode_oplog.rs:88-130):
//   agent assignment  AgentAssignmentRun (agent, seq jump, len), merged on same agent + no jump
//                     (encode_oplog.rs:142-189)
//   ops               ListOpMetrics runs merged by can_append_ops / append_ops
//                     (op_metrics.rs:235-293), written by write_op (encode_oplog.rs:20-92)
//   parents           GraphEntrySimple runs (graph/mod.rs:239-254): local parents as output-order
//                     deltas, foreign parents as (mapped agent, seq) (encode_oplog.rs:476-541)
//   content           PatchContent: Content + ContentIsKnown bit runs (encode_oplog.rs:347-399);
//                     with compress_content, every content field of >= 20 bytes goes into one
//                     LZ4 block written first as CompressedFieldsLZ4 (encode_oplog.rs:270-343,
//                     661-677), start-branch content before inserted content (:606-660)
//   CRC-32C           over everything before the CRC chunk (encode_oplog.rs:731-734)
#include "dt_host.hpp"

#include <algorithm>
#include <cstring>
#include <map>

namespace dtgpu {

namespace {

void leb(std::vector<uint8_t> &o, uint64_t v) {
    while (v >= 0x80) { o.push_back(uint8_t(v | 0x80)); v >>= 7; }
    o.push_back(uint8_t(v));
}
uint64_t mix(uint64_t v, bool b) { return v * 2 + (b ? 1 : 0); }
uint64_t zigzag_old(int64_t v) { return (uint64_t(v < 0 ? -v : v) << 1) | (v < 0 ? 1u : 0u); }   // leb.rs:305-316
void chunk(std::vector<uint8_t> &o, uint32_t type, const std::vector<uint8_t> &data) {
    leb(o, type);
    leb(o, data.size());
    o.insert(o.end(), data.begin(), data.end());
}
enum : uint32_t {
    C_FileInfo = 1, C_DocId = 2, C_AgentNames = 3, C_CompressedFieldsLZ4 = 5, C_StartBranch = 10, C_Version = 12,
    C_Content = 13, C_ContentCompressed = 14,
    C_Patches = 20, C_OpVersions = 21, C_OpTypeAndPosition = 22, C_OpParents = 23, C_PatchContent = 24,
    C_ContentIsKnown = 25, C_Crc = 100,
};
constexpr uint32_t PLAIN_TEXT = 4;   // DataType::PlainText

struct Op {                  // ListOpMetrics: loc (RangeRev) + kind + content_pos
    uint64_t start, end;     // span
    bool fwd;
    uint8_t kind;            // 0 Ins, 1 Del
    bool has_content;
    uint64_t c0, c1;         // content byte range (Ins with known content)
    uint64_t len() const { return end - start; }
};
bool can_append(const Op &a, const Op &b) {
    if (a.kind != b.kind) return false;
    if (a.has_content != b.has_content) return false;
    if (a.has_content && a.c1 != b.c0) return false;
    const bool af = a.len() == 1 || a.fwd, bf = b.len() == 1 || b.fwd;
    if (af && bf && ((a.kind == 0 && b.start == a.end) || (a.kind == 1 && b.start == a.start))) return true;
    const bool ar = a.len() == 1 || !a.fwd, br = b.len() == 1 || !b.fwd;
    if (a.kind == 1 && ar && br && b.end == a.start) return true;
    return false;
}
void append(Op &a, const Op &b) {
    a.fwd = b.start >= a.start && (b.start != a.start || a.kind == 1);
    if (a.kind == 1 && !a.fwd) a.start = b.start;
    else a.end += b.len();
    if (a.has_content) a.c1 = b.c1;
}
void write_op(std::vector<uint8_t> &dest, const Op &op, uint64_t &cursor) {
    const bool fwd = op.fwd || op.len() == 1;
    const uint64_t op_start = (op.kind == 1 && !fwd) ? op.end : op.start;
    const uint64_t op_end = (op.kind == 0 && fwd) ? op.end : op.start;
    const int64_t diff = int64_t(op_start) - int64_t(cursor);
    cursor = op_end;
    const uint64_t len = op.len();
    uint64_t n;
    if (len != 1) { n = len; if (op.kind == 1) n = mix(n, fwd); }
    else if (diff != 0) n = zigzag_old(diff);
    else n = 0;
    n = mix(n, op.kind == 1);
    n = mix(n, diff != 0);
    n = mix(n, len != 1);
    leb(dest, n);
    if (len != 1 && diff != 0) leb(dest, zigzag_old(diff));
}

struct AgentMap {            // AgentMapping (encode_oplog.rs:191-240)
    const HostOpLog &o;
    std::vector<int64_t> mapped;     // file agent id (1-based) or -1
    std::vector<uint64_t> last_seq;  // end of the last seq range written per agent
    uint32_t next = 1;
    std::vector<uint8_t> names;
    explicit AgentMap(const HostOpLog &log) : o(log), mapped(log.agent_names.size(), -1), last_seq(log.agent_names.size(), 0) {}
    uint32_t map(uint32_t agent) {
        if (mapped[agent] < 0) {
            mapped[agent] = next++;
            const std::string &nm = o.agent_names[agent];
            leb(names, nm.size());
            names.insert(names.end(), nm.begin(), nm.end());
        }
        return uint32_t(mapped[agent]);
    }
    int64_t seq_delta(uint32_t agent, uint64_t s0, uint64_t s1) {
        const int64_t d = int64_t(s0) - int64_t(last_seq[agent]);
        last_seq[agent] = s1;
        return d;
    }
};

// LV -> (agent, seq) (lv_to_agent_version)
std::pair<uint32_t, uint64_t> agent_version(const HostOpLog &o, uint64_t lv) {
    auto it = std::upper_bound(o.agent_runs.begin(), o.agent_runs.end(), lv,
                               [](uint64_t v, const AgentRun &r) { return v < r.lv; });
    const AgentRun &r = *(it - 1);
    return {r.agent, r.seq + (lv - r.lv)};
}

void write_version(std::vector<uint8_t> &dest, const std::vector<uint64_t> &v, AgentMap &am, const HostOpLog &o) {
    if (v.empty()) return;   // ROOT: no Version chunk
    std::vector<uint8_t> buf;
    for (size_t i = 0; i < v.size(); i++) {
        const auto av = agent_version(o, v[i]);
        leb(buf, mix(am.map(av.first), i + 1 < v.size()));
        leb(buf, av.second);
    }
    chunk(dest, C_Version, buf);
}

}  // namespace

// lz4_flex 0.10 block compressor (`lz4_flex::compress_into`, called at encode_oplog.rs:326).
// lz4_flex is a third-party crate absent from the reference tree; this restates its published
// greedy parse, and the parameters below are pinned by the reference's own files: the LZ4 blocks
// inside friendsforever.dt (U16 table), git-makefile.dt and node_nodecc.dt (U32 table) are
// reproduced byte for byte from their decompressed content (tests/test_encoder.py).
//   * inputs < 65,535 B: 8,192-entry table of u16 positions, hash = (u32 LE * 2654435761) >> 19;
//     larger inputs: 4,096-entry table, hash = ((u64 LE << 24) * 889523592379) >> 52;
//   * position 0 is hashed first and the search starts at 1; positions past len - 12 (MFLIMIT)
//     are never searched; a search run of k misses steps by 1 + (k >> 5) bytes;
//   * a candidate is taken when its first four bytes equal the current ones and it lies within
//     65,535 bytes; the match is extended backwards over the pending literals, forwards up to
//     len - 6, and position (match end - 2) is hashed;
//   * sequences are token (literal length, match length - 4), 255-run length extensions, the
//     literals, the 16-bit LE offset; the tail is one literal-only sequence.
void lz4_block_compress(const uint8_t *in, size_t n, std::vector<uint8_t> &out) {
    auto u32at = [&](size_t p) { uint32_t v; std::memcpy(&v, in + p, 4); return v; };
    auto ext = [&](size_t v) {
        while (v >= 255) { out.push_back(255); v -= 255; }
        out.push_back(uint8_t(v));
    };
    auto emit = [&](size_t l0, size_t l1, size_t off, size_t mlen) {
        const size_t ll = l1 - l0;
        out.push_back(uint8_t((std::min<size_t>(ll, 15) << 4) | (off ? std::min<size_t>(mlen - 4, 15) : 0)));
        if (ll >= 15) ext(ll - 15);
        out.insert(out.end(), in + l0, in + l1);
        if (!off) return;
        out.push_back(uint8_t(off));
        out.push_back(uint8_t(off >> 8));
        if (mlen - 4 >= 15) ext(mlen - 4 - 15);
    };
    if (n < 13) { emit(0, n, 0, 0); return; }
    const bool small = n < 65535;
    std::vector<uint32_t> table(small ? 8192 : 4096, 0);
    auto hash = [&](size_t p) -> size_t {
        if (small) return size_t((u32at(p) * 2654435761u) >> 19);
        uint64_t v;
        std::memcpy(&v, in + p, 8);
        return size_t(((v << 24) * 889523592379ull) >> 52);
    };
    const size_t end_check = n - 12, match_lim = n - 6;
    size_t lit = 0, cur = 1;
    table[hash(0)] = 0;
    for (;;) {
        size_t cand, nmc = 32, next = cur;
        for (;;) {
            const size_t step = nmc >> 5;
            nmc++;
            cur = next;
            next += step;
            if (cur > end_check) { emit(lit, n, 0, 0); return; }
            const size_t h = hash(cur);
            cand = table[h];
            table[h] = uint32_t(cur);
            if (cur - cand > 65535) continue;
            if (u32at(cand) == u32at(cur)) break;
        }
        while (cur > lit && cand > 0 && in[cur - 1] == in[cand - 1]) { cur--; cand--; }
        const size_t m0 = cur, off = cur - cand;
        cur += 4;
        cand += 4;
        while (cur < match_lim && in[cur] == in[cand]) { cur++; cand++; }
        table[hash(cur - 2)] = uint32_t(cur - 2);
        emit(lit, m0, off, cur - m0);
        lit = cur;
    }
}

Status encode_dt(const HostOpLog &o, const std::vector<uint64_t> &from, bool store_inserted_content,
                 bool compress_content, const std::vector<uint8_t> *start_content, std::vector<uint8_t> &result) {
    result.clear();
    for (uint64_t v : from) if (v >= o.n_lv) return ErrArg;
    AgentMap am(o);
    // ---- agent assignment (merged runs) ----
    std::vector<uint8_t> aa_chunk;
    bool aa_have = false;
    uint32_t aa_agent = 0;
    int64_t aa_delta = 0;
    uint64_t aa_len = 0;
    auto aa_flush = [&]() {
        if (!aa_have) return;
        const bool jump = aa_delta != 0;
        leb(aa_chunk, mix(aa_agent, jump));
        leb(aa_chunk, aa_len);
        if (jump) leb(aa_chunk, zigzag_old(aa_delta));
    };
    auto aa_push = [&](uint32_t agent, int64_t delta, uint64_t len) {
        if (aa_have && aa_agent == agent && delta == 0) { aa_len += len; return; }
        aa_flush();
        aa_have = true; aa_agent = agent; aa_delta = delta; aa_len = len;
    };
    // ---- ops ----
    std::vector<uint8_t> ops_chunk;
    uint64_t cursor = 0;
    bool op_have = false;
    Op op_last{};
    auto op_push = [&](const Op &op) {
        if (op_have && can_append(op_last, op)) { append(op_last, op); return; }
        if (op_have) write_op(ops_chunk, op_last, cursor);
        op_have = true;
        op_last = op;
    };
    // ---- inserted content ----
    std::vector<uint8_t> ins_text, known_out;
    bool kr_have = false, kr_val = false;
    uint64_t kr_len = 0;
    auto known_push = [&](bool val, uint64_t len) {
        if (kr_have && (kr_val == val || kr_len == 0)) { kr_len += len; kr_val = val; return; }
        if (kr_have) leb(known_out, mix(kr_len, kr_val));
        kr_have = true; kr_val = val; kr_len = len;
    };
    // ---- parents ----
    struct TxnMap { uint64_t end, out; };
    std::map<uint64_t, TxnMap> txn_map;   // written txns: LV start -> (end, output start)
    std::vector<uint8_t> txns_chunk;
    uint64_t next_out = 0;
    bool tx_have = false;
    uint64_t tx_s = 0, tx_e = 0;
    std::vector<uint64_t> tx_par;
    auto find_local = [&](uint64_t p, uint64_t &mapped) -> bool {
        auto it = txn_map.upper_bound(p);
        if (it == txn_map.begin()) return false;
        --it;
        if (p >= it->second.end) return false;
        mapped = it->second.out + (p - it->first);
        return true;
    };
    auto tx_write = [&]() {
        const uint64_t len = tx_e - tx_s, out0 = next_out;
        txn_map.emplace(tx_s, TxnMap{tx_e, out0});
        next_out += len;
        leb(txns_chunk, len);
        if (tx_par.empty()) { leb(txns_chunk, 1); return; }   // ROOT: foreign agent 0
        for (size_t i = 0; i < tx_par.size(); i++) {
            const bool more = i + 1 < tx_par.size();
            uint64_t mp = 0;
            if (find_local(tx_par[i], mp)) {
                leb(txns_chunk, mix(mix(out0 - mp, more), false));
            } else {
                const auto av = agent_version(o, tx_par[i]);
                leb(txns_chunk, mix(mix(am.map(av.first), more), true));
                leb(txns_chunk, av.second);
            }
        }
    };
    auto tx_push = [&](uint64_t s, uint64_t e, const std::vector<uint64_t> &par) {
        if (tx_have && s == tx_e && par.size() == 1 && par[0] == tx_e - 1) { tx_e = e; return; }
        if (tx_have) tx_write();
        tx_have = true; tx_s = s; tx_e = e; tx_par = par;
    };

    // ---- the walk: optimized_txns_between(from, tip) ----
    std::vector<std::pair<uint64_t, uint64_t>> only_from, spans;
    o.graph.diff_rev(from, o.version, only_from, spans);
    std::reverse(spans.begin(), spans.end());
    Status err = OK;
    spanning_walk(o, spans, [&](uint64_t s, uint64_t e, const std::vector<uint64_t> &parents) {
        // 1. agent assignment (client_with_localtime.iter_range_ctx)
        auto it = std::upper_bound(o.agent_runs.begin(), o.agent_runs.end(), s,
                                   [](uint64_t v, const AgentRun &r) { return v < r.lv; });
        for (size_t k = size_t(it - o.agent_runs.begin()) - 1; k < o.agent_runs.size() && o.agent_runs[k].lv < e; k++) {
            const AgentRun &r = o.agent_runs[k];
            const uint64_t x = std::max(r.lv, s), y = std::min(r.lv + r.len, e);
            if (x >= y) continue;
            const uint32_t mapped = am.map(r.agent);
            const uint64_t s0 = r.seq + (x - r.lv);
            const int64_t d = am.seq_delta(r.agent, s0, s0 + (y - x));
            aa_push(mapped, d, y - x);
        }
        // 2. operations (iter_range_simple: op runs clipped to the span)
        auto ot = std::upper_bound(o.ops.begin(), o.ops.end(), s, [](uint64_t v, const OpRun &r) { return v < r.lv + r.len; });
        for (; ot != o.ops.end() && ot->lv < e; ++ot) {
          const OpRun &r = *ot;
          const uint64_t x0 = std::max(r.lv, s), y0 = std::min(r.lv + r.len, e);
          for (uint64_t x = x0, y; x < y0; x = y) {
            y = y0;   // inserts: pieces of uniform ContentIsKnown (a ListOpMetrics run never mixes)
            if (r.kind == 0) {
                const bool kn = o.ins_cbyte[x] != ~0u;
                for (y = x + 1; y < y0 && (o.ins_cbyte[y] != ~0u) == kn; y++) {}
            }
            const uint64_t k = x - r.lv, m = y - x;
            Op op{};
            op.kind = r.kind;
            if (r.kind == 0) { op.start = r.pos + k; op.end = op.start + m; op.fwd = true; }
            else if (r.fwd || r.len == 1) { op.start = r.pos; op.end = r.pos + m; op.fwd = true; }
            else { op.start = r.pos + (r.len - k - m); op.end = op.start + m; op.fwd = false; }
            if (r.kind == 0) {
                const bool known = o.ins_cbyte[x] != ~0u;
                if (known) {
                    op.has_content = true;
                    op.c0 = o.ins_cbyte[x];
                    op.c1 = o.ins_cbyte[y - 1] + utf8_len(o.ins_content[o.ins_cbyte[y - 1]]);
                    if (store_inserted_content) ins_text.insert(ins_text.end(), o.ins_content.begin() + ptrdiff_t(op.c0),
                                                                o.ins_content.begin() + ptrdiff_t(op.c1));
                } else if (store_inserted_content) {
                    err = ErrCheckout;   // the reference asserts content.is_some() for inserts
                }
                if (store_inserted_content) known_push(known, m);
            }
            op_push(op);
          }
        }
        // 3. parents
        tx_push(s, e, parents);
    });
    if (err != OK) return err;
    aa_flush();
    if (op_have) write_op(ops_chunk, op_last, cursor);
    if (tx_have) tx_write();
    if (kr_have) leb(known_out, mix(kr_len, kr_val));

    // ---- content fields: write_content (encode_oplog.rs:270-305).  A field of >= 20 bytes goes
    // into the shared LZ4 buffer when compressing (ContentCompressed holds its length in situ).
    std::vector<uint8_t> lz;
    auto write_content = [&](std::vector<uint8_t> &dest, const uint8_t *b, size_t n) {
        std::vector<uint8_t> buf;
        leb(buf, PLAIN_TEXT);
        if (compress_content && n >= 20) {
            leb(buf, n);
            lz.insert(lz.end(), b, b + n);
            chunk(dest, C_ContentCompressed, buf);
        } else {
            buf.insert(buf.end(), b, b + n);
            chunk(dest, C_Content, buf);
        }
    };
    // ---- start branch (encode_oplog.rs:606-618): the version, then the checkout at `from`
    // (the caller runs it on the device) when store_start_branch_content ----
    std::vector<uint8_t> start_branch;
    if (!from.empty()) {
        write_version(start_branch, from, am, o);
        if (start_content) write_content(start_branch, start_content->data(), start_content->size());
    }
    // ---- file info ----
    std::vector<uint8_t> fileinfo;
    if (o.has_doc_id) {   // write_chunk_str (encode_oplog.rs:311-318, 639-641)
        std::vector<uint8_t> d;
        leb(d, PLAIN_TEXT);
        d.insert(d.end(), o.doc_id.begin(), o.doc_id.end());
        chunk(fileinfo, C_DocId, d);
    }
    chunk(fileinfo, C_AgentNames, am.names);
    // ---- patches ----
    std::vector<uint8_t> patches;
    if (store_inserted_content && !ins_text.empty()) {   // ContentChunk::flush (encode_oplog.rs:381-398)
        std::vector<uint8_t> pc;
        leb(pc, 0);   // Ins
        write_content(pc, ins_text.data(), ins_text.size());
        chunk(pc, C_ContentIsKnown, known_out);
        chunk(patches, C_PatchContent, pc);
    }
    chunk(patches, C_OpVersions, aa_chunk);
    chunk(patches, C_OpTypeAndPosition, ops_chunk);
    chunk(patches, C_OpParents, txns_chunk);
    static const uint8_t magic[8] = {'D', 'M', 'N', 'D', 'T', 'Y', 'P', 'S'};
    result.assign(magic, magic + 8);
    leb(result, 0);   // PROTOCOL_VERSION
    if (!lz.empty()) {   // write_compressed_chunk (encode_oplog.rs:320-343), the first chunk
        std::vector<uint8_t> c;
        leb(c, lz.size());
        lz4_block_compress(lz.data(), lz.size(), c);
        chunk(result, C_CompressedFieldsLZ4, c);
    }
    chunk(result, C_FileInfo, fileinfo);
    chunk(result, C_StartBranch, start_branch);
    chunk(result, C_Patches, patches);
    const uint32_t crc = crc32c(result.data(), result.size());
    std::vector<uint8_t> c(4);
    std::memcpy(c.data(), &crc, 4);   // little endian (push_u32_le)
    chunk(result, C_Crc, c);
    return OK;
}

}  // namespace dtgpu
