// dt_ff.hpp -- host/device layout of the linear-history checkout (dt_ff.hip).
//
// The reference's merge fast-forwards while the next graph entry's parents are the current
// frontier (src/listmerge/merge.rs:811-840): ops are then applied as plain positional edits, with
// no origin search, no YjsMod scan and no retreat / advance.  A document whose whole history is
// one graph entry (Graph::push extends the last entry whenever the new span continues it,
// src/causalgraph/graph/mod.rs) is checked out entirely on that path, and such a history is a
// splice sequence.  The device checks it out as a piece table instead of per-item replay:
//
//   1. segments of FF_RUNS op runs each replay on one wave, in registers (two pieces per lane),
//      on top of one placeholder piece standing for the text at the segment's start (its length
//      is the prefix sum of the earlier segments' inserts - deletes);
//   2. adjacent segments' piece lists are composed pairwise, log2(segments) levels: a
//      placeholder piece of the later list is replaced by the earlier list's pieces over its range
//      (splices never reorder surviving characters, so the result has at most |A| + |B| - 1
//      pieces and fits the pair's slots);
//   3. the final list (LV ranges only) gives each piece's byte offset, and the text is copied out
//      of the inserted content with the hash materialise computes.
//
// A piece is (src, len, pos): src = first LV of a run of consecutive inserted LVs, or FF_PH |
// offset into the text at the segment's (group's) start; len in chars; pos = its char offset in
// the list's text.  Op runs come straight from the decoder (quads lv, len, pos, kind | fwd << 1):
// an insert run puts LVs [lv, lv+len) at pos..pos+len-1, a delete run (either direction) removes
// the chars [pos, pos+len).
#pragma once
#include <stdint.h>

#include "dt_device.hpp"

namespace dtgpu {

constexpr uint32_t FF_RUNS = 63;        // op runs per segment (one wave)
constexpr uint32_t FF_PIECES = 128;     // piece slots per segment: 1 + 2 * FF_RUNS fit
constexpr uint32_t FF_PH = 0x80000000u; // placeholder piece flag
constexpr uint32_t FF_NONE = 0xFFFFFFFFu;
constexpr uint32_t FF_CHUNK = 4096;     // output bytes per copy workgroup (256 threads x 16)

struct FFDoc {
    uint64_t op_off;        // quads into ops
    uint64_t lv_off;        // into cbyte
    uint64_t content_off;   // into content (bytes)
    uint64_t out_off;       // into out (bytes)
    uint64_t piece_off;     // into the piece buffers: FF_PIECES * first_seg
    uint32_t n_ops, first_seg, n_seg, levels;
    uint32_t out_cap, result;   // result: the batch's document index (results[], out arena)
    uint32_t ascii, pad;
};
struct FFSeg { uint32_t doc, run0, nrun, pad; };           // doc: index into FFDoc
struct FFPair { uint32_t doc, a, b, pad; };                // local segment indexes of the two groups
                                                           // (b = FF_NONE: a lone group, copied)
struct FFChunk { uint32_t doc, start; };                   // one copy workgroup: output bytes from start

struct FFParams {
    const uint32_t *ops;
    const uint32_t *cbyte;
    const uint8_t *content;
    uint8_t *out;
    DocResult *results;
    const FFDoc *docs;
    const FFSeg *segs;
    const FFPair *pairs;
    const FFChunk *chunks;
    uint32_t n_docs, n_segs, n_chunks, n_levels;
    uint32_t level_off[33];   // pairs of level k: [level_off[k], level_off[k + 1])
    int32_t *delta;           // per segment: inserted - deleted chars
    uint32_t *bad;            // per FFDoc: nonzero = an op outside the text / a malformed list
    uint32_t *pa, *pb;        // piece buffers (uint4 per slot), ping-pong between levels
    uint32_t *ca, *cb;        // per segment: pieces of the group starting there
    uint32_t *boff;           // per slot of the final lists: byte offset (non-ASCII documents)
};

// Every kernel of one linear-history checkout pass on `stream`.
int launch_ff(const FFParams &p, void *stream);

}  // namespace dtgpu
