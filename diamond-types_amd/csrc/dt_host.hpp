// dt_host.hpp -- host-side model of a diamond-types list oplog for the MI355X engine:
// the `.dt` decoder and the causal-graph walk planner that feed the device replay.
//
// The oplog is kept as SoA runs (not the reference's RleVec<KVPair<..>> trees):
//   OpRun     <- ListOpMetrics runs   (src/list/op_metrics.rs:22-42), split at graph-entry
//                boundaries so that every run is a linear chain of LVs
//   AgentRun  <- client_with_localtime (src/causalgraph/agent_assignment/mod.rs:29-45)
//   GraphEntry<- GraphEntryInternal   (src/causalgraph/graph/mod.rs:25-53)
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace dtgpu {

enum Status : int {
    OK = 0, InvalidMagic = 1, UnsupportedProtocolVersion = 2, DocIdMismatch = 3, BaseVersionUnknown = 4,
    UnknownChunk = 5, LZ4DecoderNeeded = 6, LZ4DecompressionError = 7, CompressedDataMissing = 8,
    InvalidChunkHeader = 9, MissingChunk = 10, InvalidLength = 11, UnexpectedEOF = 12, InvalidUTF8 = 13,
    InvalidRemoteID = 14, InvalidVarInt = 15, InvalidContent = 16, GenericInvalidData = 17,
    ChecksumFailed = 18, DataMissing = 19,
    ErrCheckout = 64, ErrCapacity = 65, ErrHip = 66, ErrArg = 67, ErrNoDevice = 68,
};

struct OpRun {            // a run of LVs [lv, lv+len) of one kind inside one graph entry
    uint64_t lv, len;
    uint64_t pos;         // Ins: position of the first char. Del fwd: start. Del rev: span start
    uint8_t kind;         // 0 Ins, 1 Del
    uint8_t fwd;          // Del only: 1 forward, 0 reversed (backspace)
};

struct AgentRun { uint64_t lv, len; uint32_t agent; uint64_t seq; };
struct SeqRun { uint64_t seq, lv, len; };

struct GraphEntry {
    uint64_t start, end, shadow;
    std::vector<uint64_t> parents;   // sorted
};

struct Graph {
    std::vector<GraphEntry> entries;
    int64_t find_idx(uint64_t lv) const;
    void push(const std::vector<uint64_t> &parents, uint64_t start, uint64_t end);
    // Graph::diff_rev (src/causalgraph/graph/tools.rs:176-292); spans descending.
    void diff_rev(const std::vector<uint64_t> &a, const std::vector<uint64_t> &b,
                  std::vector<std::pair<uint64_t, uint64_t>> &only_a,
                  std::vector<std::pair<uint64_t, uint64_t>> &only_b) const;
};

struct HostOpLog {
    std::vector<std::string> agent_names;
    std::vector<std::vector<SeqRun>> agent_seqs;   // per agent, seq -> LV
    std::vector<AgentRun> agent_runs;              // LV order
    std::vector<OpRun> ops;                        // LV order, contiguous, split at entries
    std::vector<uint8_t> ins_content;              // UTF-8 of inserted chars in LV order
    std::vector<uint32_t> ins_cbyte;               // per LV: byte offset of its char (Ins), else ~0
    bool content_complete = true;                  // every insert has known content
    Graph graph;
    std::vector<uint64_t> version;                 // cg.version (frontier)
    uint64_t n_lv = 0;
    std::string doc_id;                            // ListOpLog::doc_id (src/list/mod.rs:109)
    bool has_doc_id = false;

    int32_t agent_id(const char *name, size_t len);          // get_or_create_agent_id
    uint64_t next_seq(uint32_t agent) const;
    int64_t seq_to_lv(uint32_t agent, uint64_t seq) const;
    void assign(uint32_t agent, uint64_t seq, uint64_t lv, uint64_t len);
    void push_ins(uint64_t pos, const uint8_t *utf8, size_t nbytes, uint64_t nchars, bool known);
    void push_del(uint64_t pos, uint64_t len, bool fwd);
    void add_span(uint32_t agent, std::vector<uint64_t> parents, uint64_t start, uint64_t end);
    void finish();                                 // split op runs at graph-entry boundaries
};

// ListOpLog::load_from (src/list/encoding/decode_oplog.rs:447-960)
Status decode_dt(const uint8_t *data, size_t len, bool ignore_crc, HostOpLog &out);
// ListOpLog::decode_and_add_opts (decode_oplog.rs:476-583): merge a `.dt` patch into `o`, skipping
// the operations it already has; `file_frontier` = the version of the loaded data.  On error `o`
// is unchanged.
Status decode_and_add(const uint8_t *data, size_t len, bool ignore_crc, HostOpLog &o,
                      std::vector<uint64_t> &file_frontier);
uint32_t crc32c(const uint8_t *d, size_t n);
// ListOpLog::encode_from (src/list/encoding/encode_oplog.rs:404-747).  compress_content: LZ4 for
// content fields of >= 20 bytes; start_content: the StartBranch content (the checkout at `from`,
// store_start_branch_content) or null.
Status encode_dt(const HostOpLog &o, const std::vector<uint64_t> &from, bool store_inserted_content,
                 bool compress_content, const std::vector<uint8_t> *start_content, std::vector<uint8_t> &result);
// lz4_flex::compress_into (lz4_flex 0.10 block format, no length prefix)
void lz4_block_compress(const uint8_t *in, size_t n, std::vector<uint8_t> &out);
bool lz4_block_decompress(const uint8_t *src, size_t n, uint8_t *dst, size_t out_len);
bool utf8_valid(const uint8_t *s, size_t n);
inline uint32_t utf8_len(uint8_t c) { return c < 0x80 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : 4; }

// Device command stream (consumed by dt_replay.hip).  One command = 16 bytes.
//   INS {lv, len, pos}          apply an insert run at visible position pos
//   DEL {lv, len, pos} (+fwd)   apply a delete run (op bit 4: forward; clear: backspace run)
//   TOG {off, n}                one walk step's retreat + advance set: n tlist entries from off
enum CmdOp : uint32_t { CMD_INS = 0, CMD_DEL = 1, CMD_TOG = 2 };
struct Cmd { uint32_t op; uint32_t lv; uint32_t len; uint32_t pos; };   // op: bits 0-3 opcode, bit 4 fwd
// tlist entry: LV | is_del << 30 | advance << 31
constexpr uint32_t TL_DEL = 1u << 30, TL_ADV = 1u << 31;
constexpr uint64_t MAX_PLAN_LV = 1ull << 30;

struct Plan {
    std::vector<Cmd> cmds;
    std::vector<uint32_t> tlist;
    std::vector<uint32_t> agent_runs;   // quads (lv_start, name_rank, seq_start, agent) for YjsMod tie-breaks
    uint64_t n_steps = 0, n_retreat = 0, n_advance = 0, n_tip_advance = 0;
};

// SpanningTreeWalker over the whole graph from ROOT (src/listmerge/txn_trace.rs:114-333) turned
// into the device command stream (retreat / advance / apply, src/listmerge/merge.rs:564-581).
Status build_plan(const HostOpLog &o, Plan &plan);
// The order TransformedOpsIter applies ops in for iter_xf_operations (src/list/merge.rs:24-48;
// src/listmerge/merge.rs:788-940): the fast-forward prefix, then the walker from its frontier.
// SpanningTreeWalker over ascending spans (txn_trace.rs:114-333): visit(start, end, parents) per
// consumed span in walk order (Graph::optimized_txns_between when spans = diff from a version).
void spanning_walk(const HostOpLog &o, const std::vector<std::pair<uint64_t, uint64_t>> &spans,
                   const std::function<void(uint64_t, uint64_t, const std::vector<uint64_t> &)> &visit);
std::vector<uint64_t> parents_at(const HostOpLog &o, uint64_t lv);
Status build_xf_plan(const HostOpLog &o, Plan &plan);
// iter_xf_operations_from(from, merge) (src/list/merge.rs:24-38): the walk that rebuilds the
// branch at `from` (not reported), then the new ops Hist(merge) - Hist(from) in
// TransformedOpsIter order; ends at the merged version.  first_emitted = index of the first
// command whose ops are reported.
Status build_xf_plan_from(const HostOpLog &o, const std::vector<uint64_t> &from, const std::vector<uint64_t> &merge,
                          Plan &plan, size_t &first_emitted);

// The decoded oplog as flat arrays for the device planner (dt_plan.hip): the same information
// the reference's ListOpLog holds (Graph entries with parents and child indexes, the agent
// assignment in both directions, op runs), laid out for coalesced loads.
struct PlanInput {
    uint32_t n_agents = 0;
    std::vector<uint32_t> est;      // per entry: start, end
    std::vector<uint32_t> poff;     // parents CSR (n_entries + 1)
    std::vector<uint32_t> par;      // parent LV
    std::vector<uint32_t> pent;     // entry index of that parent
    std::vector<uint32_t> coff;     // children CSR (n_entries + 1), children in index order
    std::vector<uint32_t> child;
    std::vector<uint32_t> eop;      // first op run of each entry (n_entries + 1)
    std::vector<uint32_t> ear;      // first agent run overlapping each entry
    std::vector<Cmd> opc;           // op runs as INS / DEL commands (runs never cross entries)
    std::vector<uint32_t> aruns;    // quads (lv_start, name_rank, seq_start, agent), LV order
    std::vector<uint32_t> aoff;     // per agent: offset into aseq (n_agents + 1)
    std::vector<uint32_t> aseq;     // triples (seq, lv, len) sorted by seq within each agent
    std::vector<uint32_t> isdel;    // bit per LV: 1 = delete op
    std::vector<uint32_t> tip;      // pairs (LV, entry) of cg.version
    // per entry, EREC_WORDS words: start, end, parents offset, parent count, first op run, op
    // runs, chain, first seq in the chain (the head: EREC_HEAD words), then children offset,
    // child count, first parent LV, for the first two parents (entry, chain, ops of that chain up
    // to the parent), last child, first child (the tail).  Stored split: every entry's head
    // (entry e at e * EREC_HEAD), then every entry's tail (at ne * EREC_HEAD + e * EREC_TAIL) --
    // the planner's per-step loads and the checkout pass's prep touch only the heads
    std::vector<uint32_t> erec;
    std::vector<uint32_t> pch, pcnt;  // per parent slot: its chain and that chain's ops up to it
    uint32_t n_chains = 0;          // causal chains the entries are partitioned into
    std::vector<uint32_t> prow;     // per entry: parent version vector over chains (n_chains words)
    std::vector<uint32_t> doff;     // per chain: offset of its dense seq table (n_chains + 1)
    std::vector<uint32_t> dense;    // per chain, by seq: LV | is_del << 30
    bool device_ok = true;
};
constexpr uint32_t EREC_WORDS = 20, EREC_HEAD = 8, EREC_TAIL = EREC_WORDS - EREC_HEAD;
// word k of entry e's record among ne entries
constexpr size_t erec_word(size_t ne, size_t e, uint32_t k) {
    return k < EREC_HEAD ? e * EREC_HEAD + k : ne * EREC_HEAD + e * EREC_TAIL + (k - EREC_HEAD);
}
constexpr uint32_t PLAN_CHAIN_LIMIT = 512;   // = PLAN_MAX_AGENTS of the device planner
Status build_plan_input(const HostOpLog &o, PlanInput &pi);

uint64_t text_hash(const uint8_t *t, size_t n);

}  // namespace dtgpu
