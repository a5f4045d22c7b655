/*
 * dtgpu.h -- C ABI of the MI355X-native batch checkout engine for diamond-types oplogs.
 *
 * Drop-in boundary for the reference's `ListOpLog` -> `checkout_tip()` / `ListBranch::merge()`
 * path.  Every entry point names the reference interface it replaces
 * (paths under jarrodhroberson/diamond-types).  Plain pointers and sizes only; no torch or HIP
 * types appear in the signatures (streams are passed as `void*` = hipStream_t).
 *
 * Ownership: an oplog handle is immutable once loaded except through the add_* calls; the
 * caller owns every output buffer.  Batch handles own their device memory.  No call aborts the
 * process: conditions on which the reference panics become DTGPU_ERR_CHECKOUT.
 */
#ifndef DTGPU_H
#define DTGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes.  1..19 mirror `ParseError` in declaration order
 * (src/encoding/parseerror.rs:14-48); the rest are engine statuses. */
typedef enum dtgpu_status {
    DTGPU_OK = 0,
    DTGPU_INVALID_MAGIC = 1,
    DTGPU_UNSUPPORTED_PROTOCOL_VERSION = 2,
    DTGPU_DOC_ID_MISMATCH = 3,
    DTGPU_BASE_VERSION_UNKNOWN = 4,
    DTGPU_UNKNOWN_CHUNK = 5,
    DTGPU_LZ4_DECODER_NEEDED = 6,
    DTGPU_LZ4_DECOMPRESSION_ERROR = 7,
    DTGPU_COMPRESSED_DATA_MISSING = 8,
    DTGPU_INVALID_CHUNK_HEADER = 9,
    DTGPU_MISSING_CHUNK = 10,
    DTGPU_INVALID_LENGTH = 11,
    DTGPU_UNEXPECTED_EOF = 12,
    DTGPU_INVALID_UTF8 = 13,
    DTGPU_INVALID_REMOTE_ID = 14,
    DTGPU_INVALID_VARINT = 15,
    DTGPU_INVALID_CONTENT = 16,
    DTGPU_GENERIC_INVALID_DATA = 17,
    DTGPU_CHECKSUM_FAILED = 18,
    DTGPU_DATA_MISSING = 19,
    DTGPU_ERR_CHECKOUT = 64,    /* the reference would panic (merge.rs:384,489; yjsspan.rs:49-90) */
    DTGPU_ERR_CAPACITY = 65,    /* a device-side structure overflowed its reservation */
    DTGPU_ERR_HIP = 66,         /* HIP runtime error (no GPU, OOM, launch failure) */
    DTGPU_ERR_ARG = 67,         /* invalid argument / buffer too small */
    DTGPU_ERR_NO_DEVICE = 68,   /* no HIP device: the engine has no CPU fallback */
} dtgpu_status;

typedef struct dtgpu_oplog dtgpu_oplog;
typedef struct dtgpu_batch dtgpu_batch;

/* ---- ListOpLog construction -------------------------------------------------------------- */

/* ListOpLog::load_from(&[u8]) -> Result<ListOpLog, ParseError>
 * (src/list/encoding/decode_oplog.rs:447-451).  CRC-32C is verified unless ignore_crc
 * (DecodeOptions::ignore_crc, decode_oplog.rs:428-444). */
dtgpu_status dtgpu_oplog_load(const uint8_t *bytes, size_t len, int ignore_crc, dtgpu_oplog **out);

/* ListOpLog::new() (src/list/oplog.rs:22-30) */
dtgpu_oplog *dtgpu_oplog_new(void);
void dtgpu_oplog_free(dtgpu_oplog *oplog);

/* ListOpLog::decode_and_add_opts(&[u8], DecodeOptions) -> Result<Frontier, ParseError>
 * (src/list/encoding/decode_oplog.rs:476-583): merge a `.dt` file or patch into the oplog,
 * skipping the operations it already has (the overlap filter, :780-850).  On success writes the
 * file's version (min(len, cap) LVs, ascending) and its length in *n_frontier.  On error the
 * oplog is unchanged (the reference unwinds the partial merge) and the ParseError is returned.
 * Not safe to call while another thread reads the same oplog. */
dtgpu_status dtgpu_oplog_decode_and_add(dtgpu_oplog *oplog, const uint8_t *bytes, size_t len, int ignore_crc,
                                        uint64_t *frontier, size_t cap, size_t *n_frontier);
/* The whole frontier the last successful dtgpu_oplog_decode_and_add reported (for a caller whose
 * buffer was too small): copies min(len, cap) LVs, returns len.  Reads only; adds nothing. */
size_t dtgpu_oplog_last_added_frontier(const dtgpu_oplog *oplog, uint64_t *out, size_t cap);
/* ListOpLog::doc_id (src/list/mod.rs:109): returns the id's byte length (copying min(len, cap)
 * bytes), or -1 when the oplog has none.  set_doc_id with id == NULL clears it. */
int64_t dtgpu_oplog_doc_id(const dtgpu_oplog *oplog, char *out, size_t cap);
dtgpu_status dtgpu_oplog_set_doc_id(dtgpu_oplog *oplog, const char *id, size_t len);

/* ListOpLog::get_or_create_agent_id (src/list/oplog.rs:44-46).  Returns -1 on a reserved or
 * over-long name (the reference panics: agent_assignment/mod.rs:88-91). */
int32_t dtgpu_oplog_get_or_create_agent_id(dtgpu_oplog *oplog, const char *name, size_t name_len);

/* ListOpLog::add_insert_at / add_delete_at (src/list/oplog.rs:221-246).  Return the last LV
 * of the new span (`end - 1`), or -1 on an invalid argument. */
int64_t dtgpu_oplog_add_insert_at(dtgpu_oplog *oplog, int32_t agent, const uint64_t *parents, size_t n_parents,
                                  uint64_t pos, const char *utf8, size_t n_bytes);
int64_t dtgpu_oplog_add_delete_at(dtgpu_oplog *oplog, int32_t agent, const uint64_t *parents, size_t n_parents,
                                  uint64_t del_start, uint64_t del_end);
/* ListOpLog::add_insert / add_delete_without_content at the current version (oplog.rs:273-300) */
int64_t dtgpu_oplog_add_insert(dtgpu_oplog *oplog, int32_t agent, uint64_t pos, const char *utf8, size_t n_bytes);
int64_t dtgpu_oplog_add_delete_without_content(dtgpu_oplog *oplog, int32_t agent, uint64_t del_start, uint64_t del_end);

/* ListOpLog::encode(opts) / encode_from(opts, from) (src/list/encoding/encode_oplog.rs:404-747):
 * the `.dt` bytes of the ops after `from` (an empty `from` is ROOT: the whole oplog).  Written in
 * the reference's order (Graph::optimized_txns_between) through the reference's run mergers, with
 * content fields of >= 20 bytes LZ4-compressed by a restatement of lz4_flex 0.10's block
 * compressor (encode_oplog.rs:270-343).  Byte parity with the reference encoder is pinned on the
 * reference's own vectors (compat_simple_doc, compat_empty_doc, the LZ4 blocks of the three
 * benchmark files); for concurrent (multi-agent) histories it is unpinned: no reference-produced
 * encoding of one exists, so those are checked by round trip only.  flags mirror EncodeOptions
 * (encode_oplog.rs:88-130):
 *   DTGPU_ENCODE_STORE_INSERTED_CONTENT      store_inserted_content
 *   DTGPU_ENCODE_COMPRESS_CONTENT            compress_content
 *   DTGPU_ENCODE_STORE_START_BRANCH_CONTENT  store_start_branch_content: with a non-ROOT `from`
 *                                            the StartBranch holds the checkout at `from`, which
 *                                            runs on the GPU (DTGPU_ERR_NO_DEVICE without one)
 * DTGPU_ENCODE_FULL / DTGPU_ENCODE_PATCH are the reference's ENCODE_FULL / ENCODE_PATCH.
 * out == NULL returns the size in *out_len. */
#define DTGPU_ENCODE_STORE_INSERTED_CONTENT 1u
#define DTGPU_ENCODE_COMPRESS_CONTENT 2u
#define DTGPU_ENCODE_STORE_START_BRANCH_CONTENT 4u
#define DTGPU_ENCODE_FULL 7u
#define DTGPU_ENCODE_PATCH 3u
dtgpu_status dtgpu_oplog_encode(const dtgpu_oplog *oplog, const uint64_t *from, size_t n_from, uint32_t flags,
                                uint8_t *out, size_t cap, size_t *out_len);

/* ListOpLog::len() (src/list/oplog.rs:89-91) */
size_t dtgpu_oplog_len(const dtgpu_oplog *oplog);
/* Cut points of the causal graph: LVs v such that the ops below v form the single version
 * {v-1} and every later op has v-1 in its history -- where the reference's merge can
 * fast-forward (src/listmerge/merge.rs:811-840) and where a batch's cut replay may split a
 * document.  Returns the number of maximal ranges and writes up to `cap` of them as
 * {first, last} pairs (both ends are cuts). */
size_t dtgpu_oplog_cut_ranges(const dtgpu_oplog *oplog, uint64_t *out, size_t cap);
/* ListOpLog::local_frontier() (src/list/oplog.rs:329-331).  Returns the frontier length;
 * writes min(len, cap) LVs. */
size_t dtgpu_oplog_local_frontier(const dtgpu_oplog *oplog, uint64_t *out, size_t cap);

/* Graph::find_dominators_2 (src/causalgraph/graph/tools.rs:545-578): the frontier of the union
 * of versions a and b (ascending LVs), the version ListBranch::merge ends at
 * (src/list/merge.rs:63-95, iter.into_frontier()).  Returns its length (writes min(len, cap)),
 * or -1 on an LV outside the oplog. */
int64_t dtgpu_oplog_dominators(const dtgpu_oplog *oplog, const uint64_t *a, size_t na, const uint64_t *b,
                               size_t nb, uint64_t *out, size_t cap);

/* Host-side walk plan of checkout_tip for this oplog (SpanningTreeWalker over all LVs,
 * src/listmerge/txn_trace.rs:114-333): out[0] walk steps, out[1] retreated LVs, out[2]
 * advanced LVs, out[3] device commands.  Pure host code; usable without a GPU. */
dtgpu_status dtgpu_oplog_plan_stats(const dtgpu_oplog *oplog, uint64_t out[4]);

/* The device command stream of the host plan (16 B per command: op | fwd<<4, lv, len, pos;
 * op 0 INS, 1 DEL, 2 TOG {tlist offset, count}).  Returns the command count; writes at most
 * cap commands.  Introspection for tests and tools (the device planner, dt_plan.hip, must
 * produce the same stream). */
size_t dtgpu_oplog_plan_commands(const dtgpu_oplog *oplog, uint32_t *cmds, size_t cap);
/* Retreat / advance entries of the host plan (LV | is_del << 30 | advance << 31). */
size_t dtgpu_oplog_plan_tlist(const dtgpu_oplog *oplog, uint32_t *out, size_t cap);

/* Inserted-content arena (UTF-8, LV order; the text every checkout draws from) and the byte
 * offset of each LV's char (~0 for deletes).  Return the full sizes; copy at most cap. */
size_t dtgpu_oplog_ins_content(const dtgpu_oplog *oplog, uint8_t *out, size_t cap);
size_t dtgpu_oplog_char_offsets(const dtgpu_oplog *oplog, uint32_t *out, size_t cap);
/* Tie-break agent runs of the plan: triples (first LV, agent-name rank, first seq). */
size_t dtgpu_oplog_agent_runs(const dtgpu_oplog *oplog, uint32_t *out, size_t cap);

/* ---- checkout ------------------------------------------------------------------------------ */

/* ListOpLog::checkout_tip() -> ListBranch, then ListBranch::content().to_string()
 * (src/list/oplog.rs:38-42, src/list/merge.rs:63-95, src/list/branch.rs:38-63).
 * Runs on the GPU.  out == NULL (or cap too small) returns the required length in *out_len
 * (with DTGPU_ERR_ARG when a non-NULL buffer was too small). */
/* ListOpLog::checkout(&[LV]) (src/list/oplog.rs:32-36): the text at `version` (any frontier of
 * the oplog; an empty version is ROOT).  Same buffer protocol as dtgpu_checkout_tip. */
dtgpu_status dtgpu_checkout(const dtgpu_oplog *oplog, const uint64_t *version, size_t n_version, uint8_t *out,
                            size_t cap, size_t *out_len);
dtgpu_status dtgpu_checkout_tip(const dtgpu_oplog *oplog, uint8_t *out, size_t cap, size_t *out_len);
/* lz4_flex::compress_into (the raw block the encoder writes, encode_oplog.rs:320-343; no length
 * prefix).  out == NULL returns the size in *out_len. */
dtgpu_status dtgpu_lz4_compress(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len);

/* ListOpLog::iter_xf_operations() (src/list/merge.rs:24-48): the transformed operations that
 * bring an empty document to the tip, in the order TransformedOpsIter yields them
 * (src/listmerge/merge.rs:788-940: fast-forward prefix, then a SpanningTreeWalker from its
 * frontier).  Runs on the GPU.  Writes n_lv records of two u32 {lv, pos} in application order:
 * pos = the BaseMoved position of that LV applied on its own (an insert lands at pos; a delete
 * removes the char at pos), 0xFFFFFFFF = DeleteAlreadyHappened.  out == NULL returns the record
 * count in *n_out; cap counts records. */
dtgpu_status dtgpu_xf_operations(const dtgpu_oplog *oplog, uint32_t *out, size_t cap, size_t *n_out);
/* ListOpLog::iter_xf_operations_from(from, merging) (src/list/merge.rs:24-38): the transformed
 * operations that take a branch at version `from` to find_dominators_2(from, merging) -- exactly
 * what ListBranch::merge applies to its content (src/list/merge.rs:63-95).  Same record format;
 * only the new ops Hist(merging) - Hist(from) are reported. */
dtgpu_status dtgpu_xf_operations_from(const dtgpu_oplog *oplog, const uint64_t *from, size_t n_from,
                                      const uint64_t *merging, size_t n_merging, uint32_t *out, size_t cap,
                                      size_t *n_out);
/* The LV order dtgpu_xf_operations_from reports (host plan only; usable without a GPU).
 * Returns the LV count (0 on an invalid version); writes at most cap LVs. */
size_t dtgpu_oplog_xf_order(const dtgpu_oplog *oplog, const uint64_t *from, size_t n_from, const uint64_t *merging,
                            size_t n_merging, uint32_t *out, size_t cap);
/* One text CRDT of a shared causal graph (OpLog::checkout_text, src/oplog.rs:388-394, via
 * TextInfo::merge_into, src/listmerge/merge.rs:954-1054): the ops in the LV spans
 * [spans[2i], spans[2i+1]) with the causal graph projected onto them (Graph::subgraph_raw /
 * project_onto_subgraph_raw, src/causalgraph/graph/subgraph.rs:39-250: a version's projection is
 * the frontier of its history restricted to the spans), LVs compacted in order, agents / seqs /
 * positions unchanged.  Its tip checkout (dtgpu_checkout_tip, on the device) is the text. */
dtgpu_status dtgpu_oplog_project(const dtgpu_oplog *oplog, const uint64_t *spans, size_t n_spans, dtgpu_oplog **out);
/* The projection of a version of the shared graph onto the sub-oplog of `spans`
 * (Graph::project_onto_subgraph_raw, src/causalgraph/graph/subgraph.rs; used by
 * TextInfo::with_xf_iter, src/listmerge/merge.rs:954-985): the frontier of Hist(version) n spans
 * in the sub-oplog's LVs (the numbering dtgpu_oplog_project gives).  Writes up to cap LVs and
 * returns the frontier's size, or -1 on bad arguments. */
int64_t dtgpu_oplog_project_version(const dtgpu_oplog *oplog, const uint64_t *spans, size_t n_spans,
                                    const uint64_t *version, size_t n_version, uint64_t *out, size_t cap);
/* AgentAssignment::local_to_agent_version (src/causalgraph/agent_assignment/mod.rs): the
 * (agent, seq) of a local LV. */
dtgpu_status dtgpu_oplog_local_to_remote(const dtgpu_oplog *oplog, uint64_t lv, uint32_t *agent, uint64_t *seq);
/* The local LV spans [start, end) of the remote span (agent, seq .. seq + n), in seq order
 * (AgentAssignment::remote_to_local_version, span form).  Writes up to cap pairs and returns
 * their count, or -1 when part of the span is unknown to this oplog. */
int64_t dtgpu_oplog_remote_to_local(const dtgpu_oplog *oplog, uint32_t agent, uint64_t seq, uint64_t n,
                                    uint64_t *spans, size_t cap);
/* The history of `version` as an oplog of its own (what ListOpLog::checkout(&[LV]) replays:
 * diff_rev(version, ROOT), src/causalgraph/graph/tools.rs:176-292), LVs compacted in order,
 * agents / seqs / positions unchanged; its tip checkout is the checkout at `version`. */
dtgpu_status dtgpu_oplog_history(const dtgpu_oplog *oplog, const uint64_t *version, size_t n_version,
                                 dtgpu_oplog **out);


/* ---- batch checkout (SURVEY.md §8b "batch entry") ------------------------------------------ */

typedef struct dtgpu_batch_opts {
    int ignore_crc;          /* DecodeOptions::ignore_crc */
    int host_threads;        /* decode/plan worker threads, 0 = hardware concurrency */
    int device;              /* HIP device ordinal */
    /* How the batch checks out (0 everywhere = the defaults).  The DTGPU_* environment variables
     * of the same names override these at batch creation, for experiments and A/B runs only. */
    uint32_t flags;          /* DTGPU_OPT_* below */
    uint32_t seg_ops;        /* cut replay: op runs per segment (0: 500, raised to the batch's fair share) */
    uint32_t seg_max;        /* cut replay: segments per document, <= 64 (0: 32) */
    uint32_t lds_fill;       /* expected chars per 64-slot block when sizing LDS indexes (0: 40) */
} dtgpu_batch_opts;
#define DTGPU_OPT_NO_FAST_FORWARD 1u   /* linear histories on the tracker, not dt_ff.hip (DTGPU_FF=0) */
#define DTGPU_OPT_NO_SEGMENTS 2u       /* no cut replay: long documents on one wave (DTGPU_SEG=0) */
#define DTGPU_OPT_HOST_PLAN 4u         /* walk plans built on the host (DTGPU_HOST_PLAN) */
#define DTGPU_OPT_NO_SPLIT 8u          /* no split pass for skewed batches (DTGPU_NO_SPLIT) */
#define DTGPU_OPT_NO_CRITICAL 16u      /* no critical-replay priority (DTGPU_CRITICAL=0) */
#define DTGPU_OPT_DEBUG 32u            /* invariant checks after every replay command (DTGPU_DEBUG=1) */
#define DTGPU_OPT_PASS_MARK 64u        /* every pass opens with a marker kernel (DTGPU_PASS_MARK) */

typedef struct dtgpu_doc_result {
    uint32_t status;         /* dtgpu_status of this document */
    uint32_t reserved;
    uint64_t text_len;       /* bytes of checkout_tip().content() */
    uint64_t text_hash;      /* dtgpu_text_hash of the content (see below) */
    uint64_t n_lv;           /* ListOpLog::len() = merged ops of this document */
} dtgpu_doc_result;

/* Decode + plan every document on host threads and stage the batch in HBM.  Documents are
 * `.dt` byte buffers (decode_oplog.rs:447).  Per-document failures are reported in the
 * results, never abort the batch. */
dtgpu_status dtgpu_batch_create(const uint8_t *const *docs, const size_t *lens, size_t n_docs,
                                const dtgpu_batch_opts *opts, dtgpu_batch **out);
/* Same, from already-built oplog handles (e.g. JSON traces built with add_*). */
dtgpu_status dtgpu_batch_create_from_oplogs(const dtgpu_oplog *const *oplogs, size_t n_docs,
                                            const dtgpu_batch_opts *opts, dtgpu_batch **out);
/* Enqueue the device checkout of the whole batch on `stream` (hipStream_t, NULL = the batch's
 * own stream).  Asynchronous; inputs are already resident in HBM. */
dtgpu_status dtgpu_batch_run(dtgpu_batch *batch, void *stream);
/* Run once, synchronously, and report the device time of one whole checkout pass (hipEvents on
 * the launch stream) in *kernel_ms: for device-staged batches the walker-input kernel
 * (dt_prep.hip: parent entries, children CSR, chain decomposition -- SpanningTreeWalker::new,
 * src/listmerge/txn_trace.rs:114-188), then the walk planner and the replay. */
dtgpu_status dtgpu_batch_run_timed(dtgpu_batch *batch, float *kernel_ms);
dtgpu_status dtgpu_batch_sync(dtgpu_batch *batch);
size_t dtgpu_batch_size(const dtgpu_batch *batch);
/* Device time of the last dtgpu_batch_run_timed split into out[0] = walk planning (dt_plan.hip),
 * out[1] = replay + materialisation (dt_replay.hip) and out[2] = walker inputs (dt_prep.hip; 0 for
 * host-staged batches), milliseconds.  In a split pass (a skewed device-staged batch whose
 * biggest LDS tier runs its own prep -> plan -> replay on a side stream) out[2] and out[0] are
 * the main pipeline's prep and plan; the big tier's prep and plan overlap them and are counted
 * inside out[1]. */
dtgpu_status dtgpu_batch_last_times(const dtgpu_batch *batch, float out[3]);
/* Documents planned on the host because the device planner declined them: returns their count
 * and, when flags is not NULL, one code per document: 0 device-planned, 1 DTGPU_HOST_PLAN set,
 * 2 outside the planner's limits (> 512 agents, > 16384 graph entries, sparse agent seq
 * numbering), 16 + k the device planner stopped with status k (17: an agent whose ops are not
 * one causal chain, e.g. one author committing on concurrent branches). */
size_t dtgpu_batch_host_planned(const dtgpu_batch *batch, uint8_t *flags, size_t cap);
/* Documents checked out on the fast-forward path (dt_ff.hip): a history of one graph entry, which
 * the reference's merge fast-forwards through op by op (src/listmerge/merge.rs:811-840) -- on
 * the device a piece table of segment replays composed pairwise, not the per-item tracker.
 * flags[i] = 1 for those documents (up to cap); returns how many there are. */
size_t dtgpu_batch_fast_forwarded(const dtgpu_batch *batch, uint8_t *flags, size_t cap);
/* The command stream of document `doc` as last planned (16-byte commands as uint32 quads
 * {op, lv, len, pos}; TOG commands index the retreat/advance entries copied to tlist).
 * NULL buffers query the sizes.  A fast-forwarded document (dtgpu_batch_fast_forwarded) has no
 * walk plan in a checkout pass: 0 commands. */
dtgpu_status dtgpu_batch_plan(dtgpu_batch *batch, size_t doc, uint32_t *cmds, size_t cmd_cap, uint32_t *tlist,
                              size_t tlist_cap, size_t *n_cmds, size_t *n_tlist);
/* Copy per-document results (n_docs entries) to host. */
dtgpu_status dtgpu_batch_results(dtgpu_batch *batch, dtgpu_doc_result *results);
/* Copy one document's merged text to host. */
dtgpu_status dtgpu_batch_text(dtgpu_batch *batch, size_t doc, uint8_t *out, size_t cap, size_t *out_len);
/* Compulsory bytes of one run (the roofline numerator, SURVEY.md §8d merge-only formula):
 * 16 per op run + (8 + 4 per parent) per graph entry + 12 per agent run + inserted bytes, plus
 * the text written.  Reads the results of the last run. */
uint64_t dtgpu_batch_algorithmic_bytes(dtgpu_batch *batch);
/* Diagnostics of one document from the last run: out[0] items, [1] blocks used, [2] failing
 * command, [3] failing site, [4] commands, [5] block capacity, [6..21] profile / debug words
 * (DTGPU_DEBUG=2: cycles/16 in insert, delete, retreat+advance, materialise, YjsMod scans,
 * splits, and the insert phases find / block load / origin_right / run; scan and split
 * counts; total cycles/16), [22] superblocks, [23] 1 if the index was in LDS, [24..26] the
 * retreat/advance pass split, [27] block loads that rebuilt stale masks, [28] block loads.
 * doc < the batch size addresses a document (its first segment when it was cut); past it, the
 * cut documents' later segments in staging order, up to the first index that returns
 * DTGPU_ERR_ARG. */
dtgpu_status dtgpu_batch_doc_stats(dtgpu_batch *batch, size_t doc, uint32_t out[29]);
/* Cut replay: the LV segments document `doc` replays as, each on its own wave -- cut where the
 * whole history below the cut is one version that every later op has seen, the boundary the
 * reference fast-forwards across (src/listmerge/merge.rs:811-840), each later segment starting
 * from placeholders for the text at its cut.  Returns the segment count (0 for a document
 * replayed whole) and writes up to `cap` records of 12 words: {first LV, end LV (~0: the end),
 * placeholders -- as the last pass's cut planning (cut_kernel) wrote them on the device --,
 * status, visible items, cycles/16 (DTGPU_DEBUG=2), 1 if its index was in LDS, blocks used,
 * 1 if the device planning declined and the host plan's ranges were used, then the host
 * plan's first LV, end LV and placeholders} from the last run.
 * DTGPU_SEG=0 disables segmenting; DTGPU_SEG_OPS (op runs per segment, default 500, raised
 * to the batch's fair share per wave slot) and DTGPU_SEG_MAX (default 32) size it; read at
 * batch creation. */
size_t dtgpu_batch_segments(dtgpu_batch *batch, size_t doc, uint32_t *out, size_t cap);
/* Device planner cycle profile of one document (DTGPU_PLAN_PROF set at batch creation):
 * out[0..5] cycles waiting for entry records, computing parent vectors, children + next pick,
 * emitting retreat/advance entries, copying op runs, initialising; out[6] commands, out[7]
 * retreat/advance entries. */
dtgpu_status dtgpu_batch_plan_profile(dtgpu_batch *batch, size_t doc, uint64_t out[8]);
/* Total merged ops (sum of ListOpLog::len()) in the batch. */
uint64_t dtgpu_batch_total_lv(const dtgpu_batch *batch);
void dtgpu_batch_free(dtgpu_batch *batch);

/* One-shot batch checkout: create + run + sync + results. */
dtgpu_status dtgpu_batch_checkout(const uint8_t *const *docs, const size_t *lens, size_t n_docs,
                                  const dtgpu_batch_opts *opts, dtgpu_doc_result *results);

/* Order-sensitive 64-bit hash of a text: sum over byte i of splitmix64((i << 8) | byte_i),
 * wrapping.  Computed on device for the RCCL length/hash gather; exported for checking. */
uint64_t dtgpu_text_hash(const uint8_t *text, size_t len);

/* Transformed-ops batch: every document's iter_xf_operations() (src/list/merge.rs:40-48) on the
 * GPU, host-planned in TransformedOpsIter order.  dtgpu_batch_run / run_timed replay it (the
 * merged text is materialised too: dtgpu_batch_text works); dtgpu_batch_xf_positions copies one
 * document's per-LV BaseMoved positions (indexed by LV, 0xFFFFFFFF = DeleteAlreadyHappened). */
dtgpu_status dtgpu_batch_create_xf(const dtgpu_oplog *const *oplogs, size_t n_docs, const dtgpu_batch_opts *opts,
                                   dtgpu_batch **out);
dtgpu_status dtgpu_batch_xf_positions(dtgpu_batch *batch, size_t doc, uint32_t *out, size_t cap, size_t *n_out);

/* ---- synthetic concurrent documents (BASELINE.json configs[3]) ---------------------------- */

/* Deterministic synthetic document `doc` (seed 0xD1A00000 + doc, 4..16 agents, epochs of
 * concurrent edits merged at their ends, >= target_ops LVs; dt_synth.cpp).  The op list is
 * written as variable-length uint32 records {agent, kind (0 ins, 1 del), pos, len, char0,
 * char1, n_parents, parents...}; returns the words needed (writes only when they fit in cap). */
size_t dtgpu_synth_ops(uint64_t doc, uint32_t target_ops, uint32_t *n_agents, uint32_t *out, size_t cap);
/* The same document built as an oplog (agents "a0".."a15"). */
dtgpu_status dtgpu_synth_oplog(uint64_t doc, uint32_t target_ops, dtgpu_oplog **out);
/* The SURVEY.md 8(d)4 generator (BASELINE configs[3]): every step one agent, with p = 0.1 a
 * pairwise merge of another agent's frontier (find_dominators_2), then one make_random_change
 * edit at a position of its own branch text.  n_agents = 0: U{4..16}; otherwise that many (the
 * wide variant: more concurrent causal chains than the device prep handles). */
dtgpu_status dtgpu_synth_merge_oplog(uint64_t doc, uint32_t target_ops, uint32_t n_agents, dtgpu_oplog **out);

/* Number of HIP devices visible (0 when there is no GPU). */
int dtgpu_device_count(void);
const char *dtgpu_status_str(dtgpu_status status);


/* Device-staged batch: the `.dt` bytes go to HBM and everything after runs on the device --
 * decode (dt_decode.hip), planner inputs (dt_prep.hip: parents, children, causal chains, entry
 * records), walk planning and replay; the host only sizes arenas from per-document counts.
 * Documents outside the device path's limits (see dtgpu_decode_*, and histories wider than 64
 * causal chains) report status DTGPU_DECODE_DEFER: check them out with dtgpu_batch_create.
 * dtgpu_batch_run / run_timed then re-run prep + plan + replay; run_e2e_timed re-runs decode + prep +
 * plan + replay and returns the four kernel times (ms). */
dtgpu_status dtgpu_batch_create_device(const uint8_t *const *docs, const size_t *lens, size_t n,
                                       const dtgpu_batch_opts *opts, dtgpu_batch **out);
dtgpu_status dtgpu_batch_run_e2e_timed(dtgpu_batch *batch, float ms[4]);
/* Batched ListOpLog::encode(opts) from ROOT (src/list/encoding/encode_oplog.rs:404-747) for every
 * document of a device-staged batch, on the GPU (dt_encoder.hip): the decoded oplogs and the
 * planner's walk order (Graph::optimized_txns_between) are read in place, the `.dt` bytes --
 * LZ4-compressed content, CRC-32C -- are written per document in HBM.  flags: DTGPU_ENCODE_FULL /
 * DTGPU_ENCODE_PATCH / their bits (the StartBranch is ROOT, so the two presets agree).
 * *kernel_ms = the encode kernel's time (HIP events).  The bytes equal dtgpu_oplog_encode's. */
dtgpu_status dtgpu_batch_encode(dtgpu_batch *batch, uint32_t flags, float *kernel_ms);
/* Document `doc`'s encoded bytes (out == NULL: size in *out_len); the document's status when the
 * batch did not stage it on the device (e.g. DTGPU_DECODE_DEFER).  prof (may be NULL), when
 * DTGPU_ENC_PROF is set: cycles per phase (walk, records, sizes, text + LZ4, write, CRC), LZ4
 * cycles (probing, extending, emitting), counts (probe steps, steps with shared hashes,
 * sequences), cycles of the txn-head and agent-run passes (the records figure is the op runs). */
dtgpu_status dtgpu_batch_encoded(const dtgpu_batch *batch, size_t doc, uint8_t *out, size_t cap, size_t *out_len,
                                 uint64_t prof[14]);
/* which = 0: encoded bytes written by the last dtgpu_batch_encode; 1: decoded SoA bytes it read */
uint64_t dtgpu_batch_encoded_bytes(const dtgpu_batch *batch, int which);

/* ---- batched `.dt` decode on the GPU ---------------------------
 * ListOpLog::load_from (src/list/encoding/decode_oplog.rs:447-960) for many documents at once:
 * one wavefront per document (dt_decode.hip).  dtgpu_decode_create uploads the documents and
 * runs a sizing pass; dtgpu_decode_run is the full decode (device only) and returns its kernel
 * time.  Per document the status is a dtgpu_status, or DTGPU_DECODE_DEFER when the document
 * uses something the device decoder hands to the host decoder (more than 2048 agents, 64
 * parents on one entry, a frontier wider than 64, overlapping seq ranges of one agent, LVs or
 * positions >= 2^31). */
typedef struct dtgpu_decoded dtgpu_decoded;
#define DTGPU_DECODE_DEFER 80
dtgpu_status dtgpu_decode_create(const uint8_t *const *docs, const size_t *lens, size_t n,
                                 const dtgpu_batch_opts *opts, dtgpu_decoded **out);
dtgpu_status dtgpu_decode_run(dtgpu_decoded *dec, float *ms);
size_t dtgpu_decode_size(const dtgpu_decoded *dec);
/* out: status, n_lv, op runs, agent runs, graph entries, parents, content bytes, frontier size,
 * agents, content_complete, ascii, file agents */
dtgpu_status dtgpu_decode_status(const dtgpu_decoded *dec, size_t i, uint64_t out[12]);
float dtgpu_decode_last_ms(const dtgpu_decoded *dec);
/* core-clock cycles of document i's last decode by phase: LZ4, chunk directory, op/agent runs,
 * seq lookup lists, parents, checks + CRC, content copy + entry split */
dtgpu_status dtgpu_decode_profile(const dtgpu_decoded *dec, size_t i, uint32_t out[8]);
/* which = 0: encoded bytes read; 1: SoA bytes written by the last run */
uint64_t dtgpu_decode_bytes(const dtgpu_decoded *dec, int which);
void dtgpu_decode_free(dtgpu_decoded *dec);

/* ListOpLog::decode_and_add_opts (src/list/encoding/decode_oplog.rs:476-583, with decode_internal's
 * overlap filter :670-913) for a batch on the GPU: patch i (any `.dt` file or encode_from patch) is
 * merged into decoded document i of `base` (after dtgpu_decode_run, or a previous dtgpu_decode_add)
 * by one wavefront per document (dt_decode.hip decode_add_kernel).  The merged oplogs form a new
 * handle (base is unchanged): its arrays equal what dtgpu_oplog_decode_and_add leaves in a host
 * oplog, element for element; a document whose merge fails is the resident document again (the
 * reference's unwind).  *ms = the merge kernel's time.  Per-document outcome and the patch's
 * version (decode_and_add's return value): dtgpu_decode_add_result, which returns the document's
 * status (DTGPU_DECODE_DEFER: a case for the host's dtgpu_oplog_decode_and_add, as in
 * dtgpu_decode_create).  A merged handle checks out on the device with dtgpu_batch_create_decoded;
 * it cannot be re-decoded (dtgpu_decode_run returns DTGPU_ERR_ARG). */
dtgpu_status dtgpu_decode_add(const dtgpu_decoded *base, const uint8_t *const *patches, const size_t *lens,
                              size_t n, int ignore_crc, float *ms, dtgpu_decoded **out);
dtgpu_status dtgpu_decode_add_result(const dtgpu_decoded *merged, size_t i, uint64_t *frontier, size_t cap,
                                     size_t *n_frontier);
/* A device-staged checkout batch over a decoded handle (consumed, also on failure): decoded here
 * unless it already holds merged oplogs; then as dtgpu_batch_create_device. */
dtgpu_status dtgpu_batch_create_decoded(dtgpu_decoded *dec, dtgpu_batch **out);

/* Decoded-oplog arrays, the same layouts from the device decoder and from a host oplog.
 * Returns the element count (bytes for CONTENT / AGENT_NAMES) and copies min(cap, count). */
typedef enum dtgpu_export {
    DTGPU_EXPORT_OPS = 0,            /* u32 x4: lv, len, pos, kind | fwd << 1 (split at entries) */
    DTGPU_EXPORT_AGENT_RUNS = 1,     /* u32 x4: lv, len, agent, seq */
    DTGPU_EXPORT_ENTRIES = 2,        /* u32 x2: start, end */
    DTGPU_EXPORT_PARENT_OFFSETS = 3, /* u32: CSR offsets into PARENTS (entries + 1) */
    DTGPU_EXPORT_PARENTS = 4,        /* u32: parent LVs, sorted per entry */
    DTGPU_EXPORT_CONTENT = 5,        /* bytes: inserted UTF-8 in LV order */
    DTGPU_EXPORT_CHAR_OFFSETS = 6,   /* u32 per LV: byte offset of an inserted char, else ~0 */
    DTGPU_EXPORT_VERSION = 7,        /* u32: the frontier */
    DTGPU_EXPORT_AGENT_NAMES = 8,    /* per agent id: u8 length + name bytes */
    DTGPU_EXPORT_DOC_ID = 9,         /* bytes: 1 + the doc id, or 0 when there is none */
} dtgpu_export;
size_t dtgpu_decode_export(const dtgpu_decoded *dec, size_t i, int what, void *out, size_t cap);
size_t dtgpu_oplog_export(const dtgpu_oplog *oplog, int what, void *out, size_t cap);


/* ---- batched causal-graph queries ------------------------------
 * One wavefront per query (dt_graph.hip).  Graphs are GraphEntrySimple lists flattened as
 * (start, end, n_parents, parents...) int64 runs; graph g spans hist[hist_off[g], hist_off[g+1]).
 *   DTGPU_GQ_DIFF      Graph::diff (tools.rs:158-292): spans only in a, then only in b, newest
 *                      first (flag 0 = a, 1 = b)
 *   DTGPU_GQ_CONFLICT  Graph::find_conflicting (tools.rs:296-484): visited spans newest first with
 *                      flag 0 OnlyA / 1 OnlyB / 2 Shared, and the common frontier
 *   DTGPU_GQ_CONTAINS  Graph::frontier_contains_version (tools.rs:88-146): n_a = 1 if a contains
 *                      target (-1 = ROOT)
 *   DTGPU_GQ_DOMINATORS Graph::find_dominators_2 (tools.rs:545-578; a, b sorted dominator sets):
 *                      common[0, n_common) = the union's dominators, ascending (ListBranch::merge's
 *                      end version)
 *   DTGPU_GQ_DIFF_LEVEL Graph::diff as DTGPU_GQ_DIFF, computed level-synchronously: the graph's
 *                      entries are levelled (Kahn, one level per round) and the two versions'
 *                      marks propagate down the levels over the CSR parent arrays (dt_level.hip);
 *                      every per-entry array in HBM (graphs of any size)
 *   DTGPU_GQ_CONFLICT_LEVEL Graph::find_conflicting as DTGPU_GQ_CONFLICT: the level-synchronous
 *                      marks give each span's OnlyA / OnlyB / Shared flag (membership); the span
 *                      cuts and the common frontier come from a sweep over the entries in
 *                      descending order with each entry's pending time points in a bucket (the
 *                      reference's heap walk without the heap, dt_level.hip)
 * spans: span_cap (start, end, flag) triples per query; common: common_cap LVs per query (the
 * common frontier of CONFLICT, the dominators of DOMINATORS).  Frontiers and the walks' queues have
 * no size limit: a heap walk whose queue outgrows LDS is answered again with its queue in HBM
 * scratch sized from its graph.  answer.status: 0 ok, 1 capacity (span_cap or common_cap too
 * small for the answer), 2 bad input (a version outside the graph). */
#define DTGPU_GQ_DIFF 0
#define DTGPU_GQ_CONFLICT 1
#define DTGPU_GQ_CONTAINS 2
#define DTGPU_GQ_DOMINATORS 3
#define DTGPU_GQ_DIFF_LEVEL 4
#define DTGPU_GQ_CONFLICT_LEVEL 5
typedef struct dtgpu_graph_query {
    uint32_t kind, graph;
    size_t na, nb;                  /* frontier sizes: any (SmallVec frontiers in the reference) */
    const int64_t *a, *b;           /* ascending LVs; b unused for CONTAINS */
    int64_t target;
} dtgpu_graph_query;
typedef struct dtgpu_graph_answer {
    uint32_t status, n_a, n_b, n_common;
} dtgpu_graph_answer;
dtgpu_status dtgpu_graph_queries(const int64_t *hist, const size_t *hist_off, size_t n_graphs,
                                 const dtgpu_graph_query *queries, size_t n_queries, int64_t *spans,
                                 size_t span_cap, int64_t *common, size_t common_cap,
                                 dtgpu_graph_answer *answers, float *ms);

#ifdef __cplusplus
}
#endif
#endif /* DTGPU_H */
