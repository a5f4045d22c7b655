// dt_decode.hip -- batched `.dt` decode on MI355X.
//
// One 64-lane wavefront decodes one document.  The `.dt` grammar is a sequential byte stream
// (chunk headers, LEB128 varints, run records whose cursor depends on the previous record), so
// the parse itself runs wave-uniformly: bytes come out of a 256-byte register window (lane i
// holds bytes 4i..4i+3, one coalesced load per refill, `v_readlane` to extract), and every
// parse variable lives in scalar registers.  Everything with data parallelism runs across the
// 64 lanes: LZ4 literal and match copies (a match with offset < length is periodic, so lane k
// copies byte `k mod offset`), UTF-8 validation (lead / continuation checks per byte, ASCII
// chunks by one ballot), character counting inside content runs (ballot + popcount),
// per-LV content offsets, CRC-32C (64 segment CRCs merged with the x^(8n) mod P combine), the
// per-agent seq -> LV lookup lists and the output records (buffered one per lane, flushed as
// coalesced 16-byte stores).
//
// Reference behaviour followed, by function:
//   header / chunk reader      src/list/encoding/decode_oplog.rs:590-615, decode_tools.rs:185-268
//   varints / zigzag           src/list/encoding/leb.rs:113-178, 305-323
//   LZ4 block                  decode_oplog.rs:621-633 (lz4_flex::decompress, raw block)
//   FileInfo / agent names     decode_oplog.rs:197-227, agent_assignment/mod.rs:80-100
//   StartBranch                decode_oplog.rs:652-664, read_version :70-93
//   PatchContent / runs        decode_oplog.rs:383-425, decode_tools.rs:133-195
//   OpVersions                 read_next_agent_assignment, decode_oplog.rs:29-68
//   OpTypeAndPosition          ReadPatchesIter::next_internal, decode_oplog.rs:289-337, 731-778
//   RLE op-run append          src/list/op_metrics.rs:235-293 (push_op_internal, oplog.rs:159-175)
//   OpParents / graph push     decode_oplog.rs:95-148, 856-913; graph/mod.rs:85-128
//   frontier advance           src/frontier.rs:251-279
//   CRC-32C                    decode_oplog.rs:940-955, src/encoding/tools.rs:111-115
// The host decoder (dt_host.cpp decode_dt) is the same algorithm in sequential C++; the parity
// tests compare the two array by array, and status by status on corrupted inputs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dt_decode.hpp"
#include "dt_device.hpp"

namespace dtgpu {
namespace ddec {

enum : int {
    S_OK = 0, InvalidMagic = 1, UnsupportedProtocolVersion = 2, DocIdMismatch = 3, BaseVersionUnknown = 4, UnknownChunk = 5,
    LZ4DecompressionError = 7, CompressedDataMissing = 8, MissingChunk = 10, InvalidLength = 11,
    UnexpectedEOF = 12, InvalidUTF8 = 13, InvalidVarInt = 15, InvalidContent = 16, ChecksumFailed = 18,
    ErrCheckout = 64, ErrCapacity = 65, Defer = int(DECODE_DEFER),
};

#define TRY(x) do { const int s_ = (x); if (s_) return s_; } while (0)

constexpr uint32_t CRC_POLY = 0x82F63B78u;
constexpr uint64_t LIM31 = 1ull << 31;

__device__ __forceinline__ uint32_t lane() { return __lane_id(); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) {
    return uint32_t(__builtin_amdgcn_readlane(int(v), int(l)));
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint64_t lt_mask() { return (1ull << lane()) - 1ull; }
__device__ __forceinline__ uint32_t popc(uint64_t m) { return uint32_t(__popcll(m)); }
__device__ __forceinline__ uint32_t ctz(uint64_t m) { return uint32_t(__ffsll((unsigned long long)m) - 1); }
// Inclusive prefix sum over the wave (all lanes active): row_shr 1, 2, 4, 8 scan each row of 16
// lanes, row_bcast 15 adds row 0's total to row 1 and row 2's to row 3, row_bcast 31 adds rows
// 0-1's total to rows 2 and 3 -- six DPP adds instead of six dependent LDS permutes.
__device__ __forceinline__ uint32_t scan_incl(uint32_t v) {
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xf, 0xf, false));   // row_shr:1
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xf, 0xf, false));   // row_shr:2
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xf, 0xf, false));   // row_shr:4
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xf, 0xf, false));   // row_shr:8
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false));   // row_bcast:15
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false));   // row_bcast:31
    return v;
}
// Prefix composition of boolean functions f_l: {0,1} -> {0,1} along the wave (all lanes
// active), each packed as f(0) | !f(1) << 1 so that the identity is 0 (what a DPP lane without a
// source reads): lane l gets f_l o ... o f_0, by the same row scan and row broadcasts as scan_incl.
__device__ __forceinline__ uint32_t fn_pack(bool f0, bool f1) { return uint32_t(f0) | (uint32_t(!f1) << 1); }
__device__ __forceinline__ uint32_t compose_scan(uint32_t v) {
    auto step = [&](uint32_t p) {   // v := v o p
        const uint32_t m0 = v & 1u, m1 = ((v >> 1) & 1u) ^ 1u;
        const uint32_t p0 = p & 1u, p1 = ((p >> 1) & 1u) ^ 1u;
        v = (p0 ? m1 : m0) | (((p1 ? m1 : m0) ^ 1u) << 1);
    };
    step(uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xf, 0xf, false)));   // row_shr:1
    step(uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xf, 0xf, false)));   // row_shr:2
    step(uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xf, 0xf, false)));   // row_shr:4
    step(uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xf, 0xf, false)));   // row_shr:8
    step(uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false)));   // row_bcast:15
    step(uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false)));   // row_bcast:31
    return v;
}
// LDS stores of this wave become visible to its lanes' later LDS loads (a wave's LDS operations
// complete in order; this only keeps the compiler from reordering them).
__device__ __forceinline__ void wave_lds_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
// Stores of this wave become visible to its later loads (same CU; workgroup scope).
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// ---------------------------------------------------------------------------------------------
// byte windows and readers
// ---------------------------------------------------------------------------------------------
struct Win {
    const uint8_t *base;   // 4-B aligned, readable for 256 B past any valid offset
    uint32_t wpos;         // window start (uniform)
    uint32_t w;            // lane i: bytes wpos + 4i .. + 3
};
__device__ __forceinline__ uint32_t wbyte(Win &W, uint32_t off) {
    uint32_t d = off - W.wpos;
    if (d >= 256u) {
        W.wpos = off & ~3u;
        W.w = *reinterpret_cast<const uint32_t *>(W.base + W.wpos + 4u * lane());
        d = off - W.wpos;
    }
    return (rdl(W.w, d >> 2) >> ((d & 3u) << 3)) & 0xFFu;
}

// A reader over one byte stream: source s selects the register window, 0 document (chunk
// headers), 1 LZ4 buffer.  The varint-only streams the main loop interleaves use queues (VQ).
struct Rd { uint32_t s, p, n; };
enum : uint32_t { SRC_DOC = 0, SRC_LZ = 1 };

struct Ctx {
    Win w0, w1;
    const uint8_t *in;   // the document
    uint8_t *lz;         // its decompressed LZ4 buffer
    __device__ __forceinline__ uint32_t byte(uint32_t s, uint32_t off) { return s ? wbyte(w1, off) : wbyte(w0, off); }
    __device__ __forceinline__ const uint8_t *ptr(uint32_t s) const { return s == SRC_LZ ? lz : in; }

    // unsigned LEB128 (leb.rs:113-178)
    __device__ __forceinline__ int varint_at(const Rd &r, uint64_t &v, uint32_t &used) {
        uint64_t x = 0;
        for (uint32_t i = 0; i < r.n; i++) {
            if (i == 10) return InvalidVarInt;
            const uint32_t b = byte(r.s, r.p + i);
            if (i == 9 && (b & 0x7fu) > 1u) return InvalidVarInt;
            x |= uint64_t(b & 0x7fu) << (7 * i);
            if (b < 0x80u) { v = x; used = i + 1; return S_OK; }
        }
        return r.n >= 10 ? InvalidVarInt : UnexpectedEOF;
    }
    __device__ __forceinline__ int u64v(Rd &r, uint64_t &v) {
        if (!r.n) return UnexpectedEOF;
        uint32_t used;
        TRY(varint_at(r, v, used));
        r.p += used; r.n -= used;
        return S_OK;
    }
    __device__ __forceinline__ int u32v(Rd &r, uint64_t &v) {
        TRY(u64v(r, v));
        return v >= 0xFFFFFFFFull ? InvalidVarInt : S_OK;
    }
    __device__ __forceinline__ int peek_u32(const Rd &r, bool &has, uint64_t &v) {
        has = false;
        if (!r.n) return S_OK;
        uint32_t used;
        TRY(varint_at(r, v, used));
        if (v >= 0xFFFFFFFFull) return InvalidVarInt;
        has = true;
        return S_OK;
    }
    __device__ __forceinline__ int zigzag(Rd &r, int64_t &v) {   // "old" sign-magnitude zigzag (leb.rs:305-323)
        uint64_t u;
        TRY(u64v(r, u));
        v = int64_t(u >> 1) * ((u & 1) ? -1 : 1);
        return S_OK;
    }
    // ChunkReader (decode_tools.rs:185-268)
    __device__ __forceinline__ static bool known_chunk(uint64_t t) {
        return t == 1 || t == 2 || t == 3 || t == 4 || t == 5 || t == 10 || t == 11 || t == 12 || t == 13 ||
               t == 14 || t == 20 || t == 21 || t == 22 || t == 23 || t == 24 || t == 25 || t == 27 || t == 100;
    }
    __device__ __forceinline__ int next_chunk(Rd &r, uint64_t &type, Rd &body) {
        for (;;) {
            uint64_t t, len;
            TRY(u32v(r, t));
            TRY(u64v(r, len));
            if (len > r.n) return InvalidLength;
            body = Rd{r.s, r.p, uint32_t(len)};
            r.p += uint32_t(len); r.n -= uint32_t(len);
            if (known_chunk(t)) { type = t; return S_OK; }
        }
    }
    __device__ __forceinline__ int chunk_if(Rd &r, uint64_t want, bool &found, Rd &body) {
        found = false;
        bool has; uint64_t t;
        TRY(peek_u32(r, has, t));
        if (!has || t != want) return S_OK;
        uint64_t tt;
        TRY(next_chunk(r, tt, body));
        found = true;
        return S_OK;
    }
    __device__ __forceinline__ int expect_chunk(Rd &r, uint64_t want, Rd &body) {
        uint64_t t;
        TRY(next_chunk(r, t, body));
        return t == want ? S_OK : MissingChunk;
    }
};

// ---------------------------------------------------------------------------------------------
// varint queues
// ---------------------------------------------------------------------------------------------
// A varint-only stream (OpVersions, OpTypeAndPosition, ContentIsKnown, OpParents) is decoded 64
// bytes at a time: lane i holds byte i, a ballot finds the terminator bytes, each terminator lane
// assembles its varint from up to 10 preceding bytes with lane shuffles, and the values are
// compacted into lanes in stream order.  The parser pops them with readlane.  Error entries
// carry the status the byte-serial reader (leb.rs:113-178) would return at that varint.
struct VQ {
    const uint8_t *base;   // stream start
    uint32_t len;          // stream bytes
    uint32_t at;           // bytes consumed by popped varints
    uint32_t wpos;         // end of the last queued varint
    uint32_t head, cnt;    // queue cursor / size (uniform)
    uint32_t lo, hi, end;  // lane k: varint k (end = ~0: error entry, lo = its status)
    __device__ __forceinline__ uint32_t left() const { return len - at; }
};

__device__ __forceinline__ VQ vq_make(const uint8_t *doc, const Rd &r) {
    VQ q;
    q.base = doc + r.p; q.len = r.n; q.at = 0; q.wpos = 0; q.head = 0; q.cnt = 0;
    q.lo = q.hi = q.end = 0;
    return q;
}

__device__ __forceinline__ void vq_refill(VQ &q, uint32_t *scratch) {
    const uint32_t i = lane();
    const uint32_t rem = q.len - q.wpos;
    const uint32_t b = i < rem ? q.base[q.wpos + i] : 0x80u;
    const uint64_t T = ballot(i < rem && b < 0x80u);
    q.head = 0;
    if (!T) {   // no varint ends within the window (or the stream): the reader's verdict
        q.cnt = 1;
        q.lo = rem >= 10 ? uint32_t(InvalidVarInt) : uint32_t(UnexpectedEOF);
        q.end = 0xFFFFFFFFu;
        return;
    }
    const bool term = (T >> i) & 1;
    const uint64_t below = T & lt_mask();
    const uint32_t start = below ? uint32_t(64 - __clzll((long long)below)) : 0u;
    const uint32_t L = i - start + 1;
    uint64_t v = 0;
#pragma unroll
    for (uint32_t j = 0; j < 10; j++) {
        const uint32_t bj = uint32_t(__shfl(int(b), int(i >= j ? i - j : 0)));
        if (j < L) v |= uint64_t(bj & 0x7fu) << (7 * (L - 1 - j));
    }
    const bool err = L > 10 || (L == 10 && (b & 0x7fu) > 1u);
    if (term) {
        const uint32_t k = popc(below);
        scratch[3 * k] = err ? uint32_t(InvalidVarInt) : uint32_t(v);
        scratch[3 * k + 1] = uint32_t(v >> 32);
        scratch[3 * k + 2] = err ? 0xFFFFFFFFu : q.wpos + i + 1;
    }
    __syncthreads();
    q.cnt = popc(T);
    if (i < q.cnt) { q.lo = scratch[3 * i]; q.hi = scratch[3 * i + 1]; q.end = scratch[3 * i + 2]; }
    __syncthreads();
    q.wpos += uint32_t(64 - __clzll((long long)T));
}

// Reader::u64v on a queue
// Top a queue up before it runs dry: the r < 64 entries left move to lanes 0 .. r-1 and the
// varints of the next window follow, as many as fit (the batched record loop then never sees a
// queue of a few varints, which it would take one record at a time).  A window without a
// terminator leaves the queue as it is; the refill once it is empty reports it.
__device__ __forceinline__ void vq_topup(VQ &q, uint32_t *scratch) {
    const uint32_t i = lane();
    const uint32_t r = q.cnt - q.head;
    const uint32_t olo = uint32_t(__shfl(int(q.lo), int(min(q.head + i, 63u))));
    const uint32_t ohi = uint32_t(__shfl(int(q.hi), int(min(q.head + i, 63u))));
    const uint32_t oend = uint32_t(__shfl(int(q.end), int(min(q.head + i, 63u))));
    const uint32_t rem = q.len - q.wpos;
    const uint32_t b = i < rem ? q.base[q.wpos + i] : 0x80u;
    const uint64_t T = ballot(i < rem && b < 0x80u);
    if (!T) return;
    const bool term = (T >> i) & 1;
    const uint64_t below = T & lt_mask();
    const uint32_t start = below ? uint32_t(64 - __clzll((long long)below)) : 0u;
    const uint32_t L = i - start + 1;
    uint64_t v = 0;
#pragma unroll
    for (uint32_t j = 0; j < 10; j++) {
        const uint32_t bj = uint32_t(__shfl(int(b), int(i >= j ? i - j : 0)));
        if (j < L) v |= uint64_t(bj & 0x7fu) << (7 * (L - 1 - j));
    }
    const bool err = L > 10 || (L == 10 && (b & 0x7fu) > 1u);
    const uint32_t nk = min(popc(T), 64u - r);   // new entries that fit
    const uint32_t k = popc(below);
    if (i < r) { scratch[3 * i] = olo; scratch[3 * i + 1] = ohi; scratch[3 * i + 2] = oend; }
    if (term && k < nk) {
        scratch[3 * (r + k)] = err ? uint32_t(InvalidVarInt) : uint32_t(v);
        scratch[3 * (r + k) + 1] = uint32_t(v >> 32);
        scratch[3 * (r + k) + 2] = err ? 0xFFFFFFFFu : q.wpos + i + 1;
    }
    const uint32_t lastk = ctz(ballot(term && k == nk - 1u));   // the window lane of the last kept one
    __syncthreads();
    q.cnt = r + nk;
    q.head = 0;
    if (i < q.cnt) { q.lo = scratch[3 * i]; q.hi = scratch[3 * i + 1]; q.end = scratch[3 * i + 2]; }
    __syncthreads();
    q.wpos += lastk + 1u;
}

__device__ __forceinline__ int vq_pop(VQ &q, uint64_t &v, uint32_t *scratch) {
    if (q.at >= q.len) return UnexpectedEOF;
    if (q.head == q.cnt) vq_refill(q, scratch);
    const uint32_t e = rdl(q.end, q.head);
    if (e == 0xFFFFFFFFu) return int(rdl(q.lo, q.head));
    v = uint64_t(rdl(q.lo, q.head)) | (uint64_t(rdl(q.hi, q.head)) << 32);
    q.at = e;
    q.head++;
    return S_OK;
}
__device__ __forceinline__ int vq_zigzag(VQ &q, int64_t &v, uint32_t *scratch) {
    uint64_t u;
    TRY(vq_pop(q, u, scratch));
    v = int64_t(u >> 1) * ((u & 1) ? -1 : 1);
    return S_OK;
}

// ---------------------------------------------------------------------------------------------
// lane-parallel helpers
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool utf8_ok_bytes(const uint8_t *s, uint32_t n, uint32_t t0, uint32_t t1, bool &ascii);
// UTF-8 validity (std::str::from_utf8): every lead byte carries exactly its continuation bytes,
// no overlong forms, no surrogates, <= U+10FFFF; every continuation byte lies inside the span
// of the nearest preceding lead.  ASCII windows are cleared by one ballot.
__device__ __forceinline__ bool utf8_ok(const uint8_t *s, uint32_t n, bool &ascii) {
    ascii = true;
    // 1 KB at a time, 16 bytes per lane from aligned blocks (each holds a text byte, so the load
    // stays inside the text's page): a kilobyte without a byte >= 0x80 is cleared by one ballot,
    // one with some takes the byte-wise check below
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(s) & ~uintptr_t(15);
    const uint32_t head = uint32_t(reinterpret_cast<uintptr_t>(s) - a0), span = head + n;
    for (uint32_t b = 0; b < span; b += 1024) {
        const uint32_t o = b + 16u * lane();
        uint4 w = make_uint4(0u, 0u, 0u, 0u);
        if (o < span) w = *reinterpret_cast<const uint4 *>(a0 + o);
        uint32_t hi = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            uint32_t m = (q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w) & 0x80808080u;
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {
                const uint32_t off = o + 4u * q + k;
                if (off < head || off >= span) m &= ~(0x80u << (8u * k));
            }
            hi |= m;
        }
        if (!ballot(hi != 0)) continue;
        const uint32_t t0 = b > head ? b - head : 0u, t1 = min(b + 1024u, span) - head;
        if (!utf8_ok_bytes(s, n, t0, t1, ascii)) return false;
    }
    return true;
}
// the byte-wise check of text bytes [t0, t1) (continuations look back, leads forward, over the
// whole text)
__device__ __forceinline__ bool utf8_ok_bytes(const uint8_t *s, uint32_t n, uint32_t t0, uint32_t t1, bool &ascii) {
    for (uint32_t i = t0; i < t1; i += 64) {
        const uint32_t j = i + lane();
        const uint32_t c = j < n ? s[j] : 0u;
        if (!ballot(c >= 0x80u)) continue;
        ascii = false;
        bool bad = false;
        if (j < n && c >= 0x80u) {
            if ((c & 0xC0u) == 0x80u) {   // continuation: covered by the nearest lead?
                bool covered = false, found = false;
                for (uint32_t k = 1; k <= 3 && k <= j && !found; k++) {
                    const uint32_t b = s[j - k];
                    if ((b & 0xC0u) == 0x80u) continue;
                    found = true;
                    const uint32_t L = (b & 0xE0u) == 0xC0u ? 2u : (b & 0xF0u) == 0xE0u ? 3u : (b & 0xF8u) == 0xF0u ? 4u : 0u;
                    covered = L > k;
                }
                bad = !covered;
            } else {
                uint32_t L, cp;
                if ((c & 0xE0u) == 0xC0u) { L = 2; cp = c & 0x1Fu; }
                else if ((c & 0xF0u) == 0xE0u) { L = 3; cp = c & 0x0Fu; }
                else if ((c & 0xF8u) == 0xF0u) { L = 4; cp = c & 0x07u; }
                else { L = 0; cp = 0; bad = true; }
                if (!bad && j + L > n) bad = true;
                for (uint32_t k = 1; !bad && k < L; k++) {
                    const uint32_t b = s[j + k];
                    if ((b & 0xC0u) != 0x80u) bad = true;
                    cp = (cp << 6) | (b & 0x3Fu);
                }
                if (!bad && ((L == 2 && cp < 0x80u) || (L == 3 && cp < 0x800u) || (L == 4 && cp < 0x10000u))) bad = true;
                if (!bad && (cp > 0x10FFFFu || (cp >= 0xD800u && cp <= 0xDFFFu))) bad = true;
            }
        }
        if (ballot(bad)) return false;
    }
    return true;
}

// Byte length of the first `want` chars of validated UTF-8 text (ContentRuns::next's walk):
// chars = min(want, chars in text).
__device__ __forceinline__ void walk_chars(const uint8_t *s, uint32_t n, uint64_t want, bool ascii, uint32_t &bytes, uint64_t &chars) {
    if (ascii) {
        chars = want < n ? want : n;
        bytes = uint32_t(chars);
        return;
    }
    uint64_t c = 0;
    for (uint32_t i = 0; i < n; i += 64) {
        const uint32_t j = i + lane();
        const bool st = j < n && (s[j] & 0xC0u) != 0x80u;
        uint64_t m = ballot(st);
        const uint32_t k = popc(m);
        if (c + k > want) {   // the char after the `want`-th starts in this window
            for (uint64_t skip = want - c; skip; skip--) m &= m - 1;
            bytes = i + ctz(m);
            chars = want;
            return;
        }
        c += k;
    }
    bytes = n;
    chars = c;
}

// One output record per lane, flushed as a coalesced quad store per 64 records.
struct Quads {
    uint32_t a, b, c, d;   // lane k: record k of the current group
    uint32_t n;            // records buffered (uniform)
    uint64_t at;           // records already flushed (uniform)
    __device__ __forceinline__ void init() { a = b = c = d = 0; n = 0; at = 0; }
    __device__ __forceinline__ void push(uint32_t x, uint32_t y, uint32_t z, uint32_t w, uint4 *dst) {
        const bool me = lane() == n;
        a = me ? x : a; b = me ? y : b; c = me ? z : c; d = me ? w : d;
        if (++n == 64) flush(dst);
    }
    __device__ __forceinline__ void flush(uint4 *dst) {
        if (lane() < n) dst[at + lane()] = make_uint4(a, b, c, d);
        at += n;
        n = 0;
    }
    __device__ uint64_t count() const { return at + n; }
};

// CRC-32C combine (zlib's crc32_combine scheme over the reflected polynomial)
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {
    if (!a) return 0;
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1u) ? (b >> 1) ^ CRC_POLY : b >> 1;
    }
    return p;
}
__device__ __forceinline__ uint32_t x2nmodp(const uint32_t *x2n, uint64_t n, uint32_t k) {
    uint32_t p = 1u << 31;
    while (n) {
        if (n & 1) p = multmodp(x2n[k & 31], p);
        n >>= 1;
        k++;
    }
    return p;
}
// CRC-32C of s[0, n): 64 lane segments (4-B aligned), merged in order.
__device__ __forceinline__ uint32_t crc32c_par(const uint8_t *s, uint32_t n, const uint32_t *T, const uint32_t *x2n) {
    // segments of a multiple of 16 bytes (s is 256-B aligned): 16-byte loads, a quarter of the
    // dependent load round trips of 4-byte ones
    const uint32_t S = (((n + 63) / 64) + 15) & ~15u;
    const uint32_t b0 = lane() * S;
    const uint32_t e0 = b0 < n ? (b0 + S < n ? b0 + S : n) : b0;
    uint32_t c = ~0u;
    uint32_t i = b0;
    for (; i + 16 <= e0; i += 16) {
        const uint4 w = *reinterpret_cast<const uint4 *>(s + i);
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            c ^= q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
            c = T[c & 0xFFu] ^ (c >> 8);
            c = T[c & 0xFFu] ^ (c >> 8);
            c = T[c & 0xFFu] ^ (c >> 8);
            c = T[c & 0xFFu] ^ (c >> 8);
        }
    }
    for (; i + 4 <= e0; i += 4) {
        c ^= *reinterpret_cast<const uint32_t *>(s + i);
        c = T[c & 0xFFu] ^ (c >> 8);
        c = T[c & 0xFFu] ^ (c >> 8);
        c = T[c & 0xFFu] ^ (c >> 8);
        c = T[c & 0xFFu] ^ (c >> 8);
    }
    for (; i < e0; i++) c = T[(c ^ s[i]) & 0xFFu] ^ (c >> 8);
    c = ~c;
    if (e0 <= b0) c = 0;   // empty segment
    const uint32_t op_full = x2nmodp(x2n, S, 3);
    uint32_t crc = rdl(c, 0);
    for (uint32_t l = 1; l < 64; l++) {
        const uint32_t sb = l * S;
        if (sb >= n) break;
        const uint32_t len = sb + S <= n ? S : n - sb;
        crc = multmodp(len == S ? op_full : x2nmodp(x2n, len, 3), crc) ^ rdl(c, l);
    }
    return crc;
}

// LZ4 raw block (lz4_flex::decompress; decode_oplog.rs:621-633) from the document into dst, up to
// 64 sequences at a time.  The sequence headers are parsed serially from the register window
// into lanes (sequence j: output start, literal length and source, match offset and length),
// with the reader's checks.  Then every output byte of the batch is resolved to where its value
// already lies -- an input literal byte, or an output byte written before the batch -- by
// following match offsets back through the batch's sequences (an overlapping match is periodic:
// its byte k repeats byte k mod offset, so one hop leaves the match; every hop lands in an
// earlier sequence, so at most 64 hops), and the bytes are copied wave-wide, one gather load and
// one store per lane per 64 bytes, instead of a dependent load round trip per sequence.
template <bool TWO = false, bool THREE = false>
__device__ __forceinline__ bool lz4_block(Ctx &C, const Rd &src, uint8_t *dst, uint32_t out_len, uint4 *lzm,
                                          uint32_t *lzr, uint32_t ring_n,
                                          uint32_t *parse_cycles = nullptr,   // DT_LZPROF: DecodeResult::prof
                                          uint32_t *xb = nullptr) {            // TWO: the batch exchange (LDS)
    const uint8_t *sp = C.in + src.p;
    const uint32_t n = src.n;
    uint32_t ip = 0, op = 0;
    uint32_t steps = 0, step_at = 1u;   // the token-step table and the window it was built for
    bool end = n == 0;
    // ---- parse up to 64 sequences into lanes (uniform); false: a malformed block ----
    auto parse_batch = [&](uint32_t &so, uint32_t &slit, uint32_t &ssrc, uint32_t &soff, uint32_t &sml,
                           uint32_t &ns) -> bool {
        so = 0xFFFFFFFFu; slit = 0; ssrc = 0; soff = 0; sml = 0;   // lane j: sequence j
        ns = 0;
        while (ns < 64 && !end) {
            {   // sequences whose lengths take at most one extension byte each, found by walking
                // a per-window table of token steps: lane l holds, for the window's bytes
                // 4l .. 4l+3 read as tokens, the distance to the next token (0 where that sequence
                // would have a longer length, no match, or cross the window or the block end).
                // The walk records each token's window offset in the next free lane; those lanes
                // then decode their sequences at once, and the reader's checks cut the run at the
                // first sequence failing one (the exact path below re-reads it).
                const uint32_t pos = src.p + ip;
                Win &W = C.w0;
                if (pos - W.wpos + 20u > 256u) {
                    W.wpos = pos & ~3u;
                    W.w = *reinterpret_cast<const uint32_t *>(W.base + W.wpos + 4u * lane());
                }
                if (step_at != W.wpos) {
                    step_at = W.wpos;
                    const uint32_t lim = src.p + n - W.wpos;   // the block end, window-relative
                    const uint32_t wn = uint32_t(__shfl(int(W.w), int(min(lane() + 1u, 63u))));
                    const uint64_t w2 = uint64_t(W.w) | (uint64_t(wn) << 32);
                    steps = 0;
#pragma unroll
                    for (uint32_t j = 0; j < 4; j++) {
                        const uint32_t c = 4u * lane() + j;
                        const uint32_t tok = uint32_t(w2 >> (8u * j)) & 0xFFu, b1 = uint32_t(w2 >> (8u * j + 8u)) & 0xFFu;
                        const uint32_t le = (tok >> 4) == 15u, me = (tok & 15u) == 15u;
                        const uint32_t lit = le ? 15u + b1 : tok >> 4;
                        const uint32_t mp = c + 3u + le + lit;   // the match length's extension byte
                        const uint32_t b2 = (uint32_t(__shfl(int(W.w), int(min(mp >> 2, 63u)))) >> ((mp & 3u) << 3)) & 0xFFu;
                        const uint32_t st = 3u + le + lit + me;
                        const bool ok = (!le || b1 < 255u) && (!me || b2 < 255u) && c + st <= 255u && c + st <= lim;
                        steps |= (ok ? st : 0u) << (8u * j);
                    }
                }
                uint32_t d = pos - W.wpos, cnt = 0, at = 0;
                const uint32_t cap = 64u - ns;
                while (cnt < cap) {   // uniform
                    const uint32_t st = (rdl(steps, d >> 2) >> ((d & 3u) << 3)) & 0xFFu;
                    if (!st) break;
                    at = lane() == ns + cnt ? d : at;
                    cnt++;
                    d += st;
                }
                if (cnt) {
                    const bool mine = lane() - ns < cnt;   // lanes ns .. ns + cnt - 1
                    const uint32_t t0 = uint32_t(__shfl(int(W.w), int(at >> 2)));
                    const uint32_t t1 = uint32_t(__shfl(int(W.w), int(min((at >> 2) + 1u, 63u))));
                    const uint32_t x = uint32_t((uint64_t(t0) | (uint64_t(t1) << 32)) >> ((at & 3u) << 3));
                    const uint32_t tok = x & 0xFFu;
                    const uint32_t le = (tok >> 4) == 15u, me = (tok & 15u) == 15u;
                    const uint32_t lit = le ? 15u + ((x >> 8) & 0xFFu) : tok >> 4;
                    const uint32_t e = at + 1u + le + lit;   // the offset's two bytes, then the extension
                    const uint32_t e0 = uint32_t(__shfl(int(W.w), int(e >> 2)));
                    const uint32_t e1 = uint32_t(__shfl(int(W.w), int(min((e >> 2) + 1u, 63u))));
                    const uint32_t y = uint32_t((uint64_t(e0) | (uint64_t(e1) << 32)) >> ((e & 3u) << 3));
                    const uint32_t off = y & 0xFFFFu;
                    const uint32_t ml = me ? 19u + ((y >> 16) & 0xFFu) : (tok & 15u) + 4u;
                    const uint32_t len = mine ? lit + ml : 0u;
                    const uint32_t incl = scan_incl(len);
                    const uint32_t o0 = op + incl - len, ms = o0 + lit;   // output start, match start
                    const uint64_t bm = ballot(mine && (off == 0 || off > ms || uint64_t(ms) + ml > out_len));
                    if (bm) cnt = ctz(bm) - ns;
                    if (cnt) {
                        const bool take = lane() - ns < cnt;
                        so = take ? o0 : so; slit = take ? lit : slit;
                        ssrc = take ? W.wpos + at - src.p + 1u + le : ssrc;
                        soff = take ? off : soff; sml = take ? ml : sml;
                        const uint32_t last = ns + cnt - 1u;
                        ip = W.wpos + rdl(e, last) - src.p + 2u + rdl(me, last);
                        op += rdl(incl, last);
                        ns += cnt;
                        end = ip >= n;
                        continue;
                    }
                }
            }
            const uint32_t tok = C.byte(0, src.p + ip++);
            uint32_t lit = tok >> 4;
            if (lit == 15) {
                uint32_t b;
                do {
                    if (ip >= n) return false;
                    b = C.byte(0, src.p + ip++);
                    lit += b;
                } while (b == 255 && lit < 0x80000000u);
            }
            if (uint64_t(ip) + lit > n || uint64_t(op) + lit > out_len) return false;
            const uint32_t lsrc = ip, o0 = op;
            ip += lit;
            op += lit;
            uint32_t off = 0, ml = 0;
            if (ip >= n) {
                end = true;
            } else {
                if (ip + 2 > n) return false;
                off = C.byte(0, src.p + ip) | (C.byte(0, src.p + ip + 1) << 8);
                ip += 2;
                if (off == 0 || off > op) return false;
                ml = tok & 15u;
                if (ml == 15) {
                    uint32_t b;
                    do {
                        if (ip >= n) return false;
                        b = C.byte(0, src.p + ip++);
                        ml += b;
                    } while (b == 255 && ml < 0x80000000u);
                }
                ml += 4;
                if (uint64_t(op) + ml > out_len) return false;
                op += ml;
                end = ip >= n;
            }
            const bool me = lane() == ns;
            so = me ? o0 : so; slit = me ? lit : slit; ssrc = me ? lsrc : ssrc;
            soff = me ? off : soff; sml = me ? ml : sml;
            ns++;
        }
        return true;
    };
    bool waited_out = false;   // THREE: a wait for the other copier gave up (the caller redoes the block)
    auto copy_batch = [&](const uint32_t bs, const uint32_t op, const uint32_t ns, const uint32_t so,
                          const uint32_t slit, const uint32_t ssrc, const uint32_t soff, const uint32_t sml,
                          uint4 *lzm, uint32_t *lzr, const volatile uint32_t *wflag, uint32_t wval) {
        // ---- resolve and copy the batch's output bytes [bs, op), CU rounds of 64 at a time ----
        // (every source lies in the input or before bs, so a group's loads all issue before its
        // stores: one memory round trip per group, not per round).  A batch of at most 4 KB of
        // output finds the sequence holding a byte in one LDS read: word w of lzm holds the
        // sequence starts among bytes bs + 64w .. + 63 as a bit mask and the starts before them;
        // a larger batch bisects the lanes' starts.
        const uint32_t nw = (op - bs + 63u) >> 6;
        const bool mapped = nw <= 64u;   // uniform
        if (mapped) {
            if (lane() < nw) lzm[lane()] = make_uint4(0u, 0u, 0u, 0u);
            wave_lds_fence();
            const uint32_t rel = so - bs;
            if (lane() < ns && rel < op - bs)
                atomicOr(reinterpret_cast<uint32_t *>(&lzm[rel >> 6]) + ((rel >> 5) & 1u), 1u << (rel & 31u));
            wave_lds_fence();
            const uint4 wv = lzm[lane()];
            const uint32_t c = lane() < nw ? uint32_t(__popc(wv.x) + __popc(wv.y)) : 0u;
            const uint32_t inc = scan_incl(c);
            if (lane() < nw) lzm[lane()].z = inc - c;
            wave_lds_fence();
        }
        constexpr uint32_t CU = THREE ? 16 : 8;
        bool waited = wflag == nullptr;   // THREE, odd batches: wait for the even batch's stores
        // Resolved sources of this batch's bytes, round by round, in an LDS ring (bit 31: an input
        // byte): a match byte whose source lies in an earlier round of the batch takes that
        // byte's source from the ring instead of hopping on (about half the resolution steps).
        const bool ring = ring_n && out_len < 0x80000000u;   // offsets leave bit 31 free (input too)
        for (uint32_t g0 = bs; g0 < op; g0 += 64u * CU) {   // uniform
            uint32_t fr[CU], inm = 0;   // per round: the source offset; bit u: it is an input byte
#pragma unroll
            for (uint32_t u = 0; u < CU; u++) {
                const uint32_t gu = g0 + 64u * u, p = gu + lane();
                uint32_t cur = p, from = 0;
                bool inp = false, done = p >= op;
                while (ballot(!done)) {
                    uint32_t r = 0;
                    if (mapped) {
                        const uint32_t rl = cur - bs;
                        const uint4 m = lzm[min(rl >> 6, 63u)];
                        const uint64_t bits = ((uint64_t(m.y) << 32) | m.x) & (~0ull >> (63u - (rl & 63u)));
                        r = m.z + popc(bits) - 1u;
                    } else {
#pragma unroll
                        for (uint32_t st = 32; st >= 1; st >>= 1)
                            if (uint32_t(__shfl(int(so), int(r + st))) <= cur) r += st;
                    }
                    const uint32_t o0 = uint32_t(__shfl(int(so), int(r))), lit = uint32_t(__shfl(int(slit), int(r)));
                    const uint32_t ls = uint32_t(__shfl(int(ssrc), int(r))), off = uint32_t(__shfl(int(soff), int(r)));
                    const uint32_t ml = uint32_t(__shfl(int(sml), int(r)));
                    if (!done) {
                        const uint32_t k = cur - o0;
                        if (k < lit) {
                            from = ls + k; inp = true; done = true;
                        } else {
                            const uint32_t m = k - lit;
                            const uint32_t q = o0 + lit - off + (off < ml ? m % off : m);
                            if (q < bs) {
                                from = q; done = true;
                            } else if (ring && q < gu && q + ring_n >= gu) {
                                const uint32_t x = lzr[q & (ring_n - 1u)];
                                from = x & 0x7FFFFFFFu; inp = x >> 31; done = true;
                            } else {
                                cur = q;
                            }
                        }
                    }
                }
                fr[u] = from;
                inm |= uint32_t(inp) << u;
                if (ring && p < op) lzr[p & (ring_n - 1u)] = from | (uint32_t(inp) << 31);
                wave_lds_fence();
            }
            if (!waited) {   // (the first group's sources are resolved while the other copier works)
                for (uint32_t it = 0; *wflag < wval; it++) {
                    if (it > (1u << 22)) { waited_out = true; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                waited = true;
            }
            uint32_t v[CU];
#pragma unroll
            for (uint32_t u = 0; u < CU; u++)
                v[u] = g0 + 64u * u + lane() >= op ? 0u : ((inm >> u) & 1u) ? sp[fr[u]] : dst[fr[u]];
#pragma unroll
            for (uint32_t u = 0; u < CU; u++)
                if (g0 + 64u * u + lane() < op) dst[g0 + 64u * u + lane()] = uint8_t(v[u]);
        }
        wave_fence();   // the next batch reads these bytes
    };
    if (!TWO) {
        while (!end) {
            uint32_t so, slit, ssrc, soff, sml, ns;
            const uint32_t bs = op;
#ifdef DT_LZPROF
            const uint64_t t_parse = __builtin_amdgcn_s_memtime();
#endif
            if (!parse_batch(so, slit, ssrc, soff, sml, ns)) return false;
#ifdef DT_LZPROF
            if (parse_cycles) parse_cycles[7] += uint32_t(__builtin_amdgcn_s_memtime() - t_parse);
#endif
            copy_batch(bs, op, ns, so, slit, ssrc, soff, sml, lzm, lzr, nullptr, 0u);
        }
        return op == out_len;
    }
    constexpr uint32_t XS = 5 * 64 + 4;
    if (THREE) {
        // Three waves: wave 0 parses batches 2t + 2 and 2t + 3 while wave 1 copies batch 2t and
        // wave 2 batch 2t + 1; wave 2 resolves its sources at once and waits for wave 1's stores
        // (a count in LDS) before its loads.  Four slots; flags bit 2: no such batch.  Each copier
        // has its own start map and ring (lzm, lzr: 256 + ring_n words each).
        const uint32_t w = threadIdx.x >> 6;
        volatile uint32_t *done = xb + 4 * XS;
        auto parse_slot = [&](uint32_t slot) {
            uint32_t so, slit, ssrc, soff, sml, ns;
            const uint32_t bs = op;
            const bool good = parse_batch(so, slit, ssrc, soff, sml, ns);
            uint32_t *b = xb + slot * XS;
            b[lane()] = so; b[64 + lane()] = slit; b[128 + lane()] = ssrc; b[192 + lane()] = soff; b[256 + lane()] = sml;
            const bool last = good && end;
            if (lane() == 0) {
                b[320] = bs; b[321] = op; b[322] = ns;
                b[323] = (last ? 1u : 0u) | ((!good || (last && op != out_len)) ? 2u : 0u);
            }
            return good && !last;
        };
        auto none_slot = [&](uint32_t slot) { if (lane() == 0) xb[slot * XS + 323] = 4u; };
        if (w == 0) {
            if (lane() == 0) { done[0] = 0; done[1] = 0; done[2] = 0; }
            if (parse_slot(0)) parse_slot(1); else none_slot(1);
        }
        __syncthreads();
        uint4 *mz = reinterpret_cast<uint4 *>(reinterpret_cast<uint32_t *>(lzm) + (w == 2 ? 256u + ring_n : 0u));
        uint32_t *rz = lzr + (w == 2 ? 256u + ring_n : 0u);
        for (uint32_t t = 0;; t++) {
            const uint32_t *c0 = xb + ((2u * t) & 3u) * XS, *c1 = xb + ((2u * t + 1u) & 3u) * XS;
            const uint32_t f0 = c0[323], f1 = c1[323];
            if ((f0 | f1) & 2u) return false;
            const bool fin = (f0 & 1u) || (f1 & 5u);
            if (w == 0) {
                if (!fin) {
                    if (parse_slot((2u * t + 2u) & 3u)) parse_slot((2u * t + 3u) & 3u);
                    else none_slot((2u * t + 3u) & 3u);
                }
            } else if (w == 1) {
                copy_batch(c0[320], c0[321], c0[322], c0[lane()], c0[64 + lane()], c0[128 + lane()],
                           c0[192 + lane()], c0[256 + lane()], mz, rz, nullptr, 0u);
                if (lane() == 0) done[0] = t + 1u;
            } else if (!(f1 & 4u)) {
                copy_batch(c1[320], c1[321], c1[322], c1[lane()], c1[64 + lane()], c1[128 + lane()],
                           c1[192 + lane()], c1[256 + lane()], mz, rz, done, t + 1u);
            }
            __syncthreads();
            if (fin) {
                done[1 + (w == 2 ? 1u : 0u)] = waited_out ? 1u : 0u;   // (lane writes; read after the barrier)
                __syncthreads();
                return !(done[1] | done[2]);
            }
        }
    }
    // Two waves (lz4_kernel): wave 0 parses batch k + 1 while wave 1 copies batch k.  A batch passes
    // through one of two slots of xb: the five lane arrays, then bs, the batch's end, its sequence
    // count and flags (bit 0: the block's last batch, bit 1: malformed); both waves read the same
    // flags after each barrier, so they leave together.
    const bool parser = threadIdx.x < 64;
    auto parse_into = [&](uint32_t slot) {
        uint32_t so, slit, ssrc, soff, sml, ns;
        const uint32_t bs = op;
        const bool good = parse_batch(so, slit, ssrc, soff, sml, ns);
        uint32_t *b = xb + slot * XS;
        b[lane()] = so; b[64 + lane()] = slit; b[128 + lane()] = ssrc; b[192 + lane()] = soff; b[256 + lane()] = sml;
        const bool last = good && end;
        if (lane() == 0) {
            b[320] = bs; b[321] = op; b[322] = ns;
            b[323] = (last ? 1u : 0u) | ((!good || (last && op != out_len)) ? 2u : 0u);
        }
    };
    if (parser) parse_into(0);
    __syncthreads();
    for (uint32_t k = 0;; k++) {
        const uint32_t *cur = xb + (k & 1u) * XS;
        const uint32_t fl = cur[323];
        if (fl & 2u) return false;
        if (parser) {
            if (!(fl & 1u)) parse_into((k + 1u) & 1u);
        } else {
            copy_batch(cur[320], cur[321], cur[322], cur[lane()], cur[64 + lane()], cur[128 + lane()],
                       cur[192 + lane()], cur[256 + lane()], lzm, lzr, nullptr, 0u);
        }
        __syncthreads();
        if (fl & 1u) return true;
    }
}

// ---------------------------------------------------------------------------------------------
// the document decoder
// ---------------------------------------------------------------------------------------------
struct Lds {                 // per-wave tables, F = max file agents of the batch
    uint32_t *fmap;          // file agent -> agent id
    uint32_t *fseq;          // file agent -> next seq (the assignment cursor)
    uint32_t *noff, *nlen;   // agent id -> name bytes in the document
    uint32_t *acnt, *aoff;   // agent id -> lookup list (count, offset)
    uint32_t *acur;          // agent id -> last lookup hit
    uint32_t *amono;         // agent id -> 1 if its runs' seq ranges increase in LV order
    uint32_t *crc;           // CRC-32C table (256)
    uint32_t *fr;            // frontier compaction scratch (64)
    uint32_t *vq;            // varint queue compaction scratch (192); fr + vq: the LZ4 byte map (1 KB)
    uint32_t *lzr;           // the LZ4 copy's resolved-source ring (DecodeParams::lz_ring entries)
};

struct CRuns {               // ContentIsKnown run iterator (ReadPatchContentIter)
    uint32_t present, ascii;
    VQ runs;
    Rd text;
    uint32_t t0;                 // where the text started
    uint32_t pb, pb_known;
    uint64_t pb_len;
    Rd pb_s;
};

template <bool SIZE>
__device__ __forceinline__ int content_str(Ctx &C, Rd &chunks, Rd &comp, bool has_comp, Rd &text, uint32_t &ascii) {
    uint64_t t; Rd c;
    TRY(C.next_chunk(chunks, t, c));
    if (t != 13 && t != 14) return MissingChunk;
    uint64_t dt;
    TRY(C.u32v(c, dt));
    if (dt != 4) return UnknownChunk;
    bool asc = true;
    if (t == 13) {
        if (!SIZE && !utf8_ok(C.in + c.p, c.n, asc)) return InvalidUTF8;
        text = c;
        ascii = asc;
        return S_OK;
    }
    uint64_t len;
    TRY(C.u64v(c, len));
    if (!has_comp) return CompressedDataMissing;
    if (len > comp.n) return UnexpectedEOF;
    text = Rd{comp.s, comp.p, uint32_t(len)};
    comp.p += uint32_t(len); comp.n -= uint32_t(len);
    if (!SIZE && !utf8_ok(C.lz + text.p, text.n, asc)) return InvalidUTF8;
    ascii = asc;
    return S_OK;
}

__device__ __forceinline__ int cruns_next(Ctx &C, CRuns &R, bool &has, uint64_t &len, bool &known, Rd &s,
                                          uint32_t *scratch) {
    if (R.pb) {
        R.pb = 0; has = true; len = R.pb_len; known = R.pb_known; s = R.pb_s;
        return S_OK;
    }
    if (!R.runs.left()) {
        if (!R.text.n) { has = false; return S_OK; }
        return UnexpectedEOF;
    }
    uint64_t x;
    TRY(vq_pop(R.runs, x, scratch));
    len = x >> 1;
    known = x & 1;
    s = Rd{R.text.s, R.text.p, 0};
    if (known) {
        uint32_t b; uint64_t c;
        walk_chars(C.ptr(R.text.s) + R.text.p, R.text.n, len, R.ascii, b, c);
        if (c != len) return UnexpectedEOF;
        s.n = b;
        R.text.p += b; R.text.n -= b;
    }
    has = true;
    return S_OK;
}

struct Out {                 // this document's output arenas
    uint4 *aruns, *pre, *ops;
    uint32_t *alist;         // triples (seq, lv, len) per agent, as quads
    uint2 *ent;
    uint32_t *poff, *par, *cbyte, *ver;
    uint2 *agents;
    uint8_t *content;
};

// Per-agent seq -> LV lookup lists from the agent runs (agent_assignment seq_to_lv): a stable
// counting sort by agent, so each list is in insertion order like the host's agent_seqs.  An
// agent whose seq ranges increase along the list is marked monotone (any hit is the only one).
__device__ __forceinline__ int build_lookup(const Out &O, const Lds &L, uint32_t n_agents, uint32_t n_aruns) {
    for (uint32_t a = lane(); a < n_agents; a += 64) { L.acnt[a] = 0; L.acur[a] = 0; L.amono[a] = 1; }
    __syncthreads();
    for (uint32_t i = lane(); i < n_aruns; i += 64) {
        const uint4 r = O.aruns[i];
        if (r.y) atomicAdd(&L.acnt[r.z], 1u);
    }
    __syncthreads();
    if (lane() == 0) {
        uint32_t s = 0;
        for (uint32_t a = 0; a < n_agents; a++) { L.aoff[a] = s; s += L.acnt[a]; L.acnt[a] = 0; }
    }
    __syncthreads();
    for (uint32_t i0 = 0; i0 < n_aruns; i0 += 64) {
        const uint32_t i = i0 + lane();
        uint4 r = make_uint4(0, 0, 0xFFFFFFFFu, 0);
        if (i < n_aruns) r = O.aruns[i];
        bool todo = i < n_aruns && r.y != 0;
        while (ballot(todo)) {   // one agent per round, lanes keep their LV order
            const uint32_t lead = rdl(todo ? r.z : 0xFFFFFFFFu, ctz(ballot(todo)));
            const uint64_t m = ballot(todo && r.z == lead);
            if (todo && r.z == lead) {
                const uint32_t k = L.aoff[lead] + L.acnt[lead] + popc(m & lt_mask());
                reinterpret_cast<uint4 *>(O.alist)[k] = make_uint4(r.w, r.x, r.y, 0);
                todo = false;
            }
            __syncthreads();
            if (lane() == 0) L.acnt[lead] += popc(m);
            __syncthreads();
        }
    }
    wave_fence();
    // an entry below its predecessor's end clears its agent's monotone flag
    for (uint32_t a = 0; a < n_agents; a++) {
        const uint32_t off = L.aoff[a], cnt = L.acnt[a];
        bool bad = false;
        for (uint32_t k = 1 + lane(); k < cnt; k += 64) {
            const uint4 p = reinterpret_cast<const uint4 *>(O.alist)[off + k - 1];
            const uint4 q = reinterpret_cast<const uint4 *>(O.alist)[off + k];
            if (uint64_t(q.x) < uint64_t(p.x) + p.z) bad = true;
        }
        if (ballot(bad) && lane() == 0) L.amono[a] = 0;
    }
    __syncthreads();
    return S_OK;
}

// seq -> LV in agent a's list (seq_to_lv: the first run in insertion order that holds seq).
// Monotone lists: a 64-entry window from the last hit, else binary search.  Others: scan in
// insertion order, 64 runs at a time.
__device__ __forceinline__ int64_t lookup_lv(const Out &O, const Lds &L, uint32_t a, uint64_t seq) {
    const uint32_t off = L.aoff[a], cnt = L.acnt[a];
    if (!cnt || seq >= LIM31) return -1;
    const uint4 *lst = reinterpret_cast<const uint4 *>(O.alist) + off;
    if (!L.amono[a]) {
        for (uint32_t k0 = 0; k0 < cnt; k0 += 64) {
            const uint32_t k = k0 + lane();
            uint4 e = make_uint4(0, 0, 0, 0);
            if (k < cnt) e = lst[k];
            const uint64_t m = ballot(k < cnt && seq >= e.x && seq < uint64_t(e.x) + e.z);
            if (m) {
                const uint32_t l = ctz(m);
                return int64_t(rdl(e.y, l)) + int64_t(seq - rdl(e.x, l));
            }
        }
        return -1;
    }
    uint32_t start = L.acur[a];
    start = start >= 4 ? start - 4 : 0;
    const uint32_t k = start + lane();
    uint4 e = make_uint4(0, 0, 0, 0);
    if (k < cnt) e = lst[k];
    const bool hit = k < cnt && seq >= e.x && seq < uint64_t(e.x) + e.z;
    const uint64_t m = ballot(hit);
    if (m) {
        const uint32_t l = ctz(m);
        if (lane() == 0) L.acur[a] = start + l;
        return int64_t(rdl(e.y, l)) + int64_t(seq - rdl(e.x, l));
    }
    uint32_t lo = 0, hi = cnt;   // first entry with seq start > seq
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint32_t s = rdl(lst[mid].x, 0);
        if (s <= seq) lo = mid + 1; else hi = mid;
    }
    if (!lo) return -1;
    const uint4 f = lst[lo - 1];
    const uint32_t fs = rdl(f.x, 0), fl = rdl(f.y, 0), fn = rdl(f.z, 0);
    if (seq >= uint64_t(fs) + fn) return -1;
    if (lane() == 0) L.acur[a] = lo - 1;
    return int64_t(fl) + int64_t(seq - fs);
}

// ---- UTF-8 insert text with few multi-byte chars ------------------------------------------------
// The byte offset of char k of a text is k plus the continuation bytes before the char's start.
// With at most 64 continuation bytes in the text they fit one register: lane e holds, for the e-th
// continuation byte (at byte p, e of them before it), t_e = p - e, the index of the first char
// starting after it -- so char k's offset is k + |{e : t_e <= k}|.  The fast path writes byte
// offsets straight away with it (no per-LV pass afterwards); a text with more continuation bytes
// takes utf8_offsets below.
struct Utf8Tab { uint32_t t, n; };   // lane e: t_e (n <= 64 entries, uniform)

// One pass over the text, 16 B per lane (aligned blocks: each holds a text byte, so the load
// stays inside the text's page).  Returns false with more than 64 continuation bytes.
__device__ __forceinline__ bool utf8_table(const uint8_t *txt, uint32_t n, Utf8Tab &tab, uint32_t &n_chars) {
    __shared__ uint32_t ent[64];
    const uintptr_t a0 = reinterpret_cast<uintptr_t>(txt) & ~uintptr_t(15);
    const uint32_t head = uint32_t(reinterpret_cast<uintptr_t>(txt) - a0), span = head + n;
    uint32_t conts = 0;   // uniform: continuation bytes before the current stride
    for (uint32_t b = 0; b < span; b += 1024) {
        const uint32_t o = b + 16u * lane();   // block offset from a0
        uint4 w = make_uint4(0u, 0u, 0u, 0u);
        if (o < span) w = *reinterpret_cast<const uint4 *>(a0 + o);
        uint32_t cm[4];
        uint32_t nc = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const uint32_t x = q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
            uint32_t m = x & ~(x << 1) & 0x80808080u;   // bytes 10xxxxxx
#pragma unroll
            for (uint32_t k = 0; k < 4; k++) {   // keep the text's own bytes only
                const uint32_t off = o + 4u * q + k;
                if (off < head || off >= span) m &= ~(0x80u << (8u * k));
            }
            cm[q] = m;
            nc += uint32_t(__popc(m));
        }
        const uint32_t incl = scan_incl(nc);
        const uint32_t tot = rdl(incl, 63);
        if (conts + tot > 64u) return false;
        if (nc) {   // rare: record this block's continuation bytes at their ranks
            uint32_t e = conts + incl - nc;
            for (uint32_t q = 0; q < 4; q++)
                for (uint32_t m = cm[q]; m; m &= m - 1) {
                    const uint32_t p = o + 4u * q + (uint32_t(__ffs(int(m)) - 1) >> 3) - head;
                    ent[e] = p - e;
                    e++;
                }
        }
        conts += tot;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    tab.n = conts;
    tab.t = lane() < conts ? ent[lane()] : 0xFFFFFFFFu;
    n_chars = n - conts;
    return true;
}
// byte offsets of the lanes' char indices k, all within [kmin, kmax] (uniform; all lanes active)
__device__ __forceinline__ uint32_t utf8_xlat(const Utf8Tab &tab, uint32_t k, uint32_t kmin, uint32_t kmax) {
    uint32_t v = k + popc(ballot(lane() < tab.n && tab.t <= kmin));
    for (uint64_t m = ballot(lane() < tab.n && tab.t > kmin && tab.t <= kmax); m; m &= m - 1)
        if (k >= rdl(tab.t, ctz(m))) v++;
    return v;
}

// ---- decode fast path ---------------------------------------------------------------------------
// The common case: the insert text is ASCII and covered by known runs, there is no deleted
// content (every benchmark file).  Pieces are then the op records split at agent-run boundaries
// (content-run splits never change an insert run), so one pass over the agent runs records their
// ends and one pass over the op records does the RLE appends (op_metrics.rs:235-293) and the
// per-LV offsets.
// Anything unusual -- including any error -- returns status 1 and decode_doc re-decodes along the
// exact piecewise path, which yields the reference's status.

// Up to 64 OpTypeAndPosition records at once (the fast path's common case): the queued varints'
// roles (record head or a head's diff) by a prefix composition, each record's cursor and LV by
// prefix sums, its agent run by a lane-permute search of 64 boundaries, the RLE merge of the op
// runs (op_metrics.rs:235-293) as in the encoder -- "record i extends the run" is a boolean
// function of "record i-1 extended it" -- and each run written at its last record.  Returns
// false without consuming anything when the batch is not the plain case (an error entry, a
// record crossing an agent-run boundary or the end of the assigned LVs, an incomplete record
// at the queue's end, a position out of range): the caller then takes one record the exact way.
#ifndef DTGPU_REC_FILL
#define DTGPU_REC_FILL 16u   // mean LVs per record from which the per-LV offsets are filled record by record
#endif
constexpr uint32_t FILL_JOB = 132;   // words of a deferred fill job: lv, tot, lincl[64], vk[64], dk mask
constexpr uint32_t FILL_HDR = 68;    // words before a document's jobs: the UTF-8 table (n, t[64])
// The per-LV content offsets of one batch of op records (batch_records, fill_kernel): LV j of
// the batch (lv + j) holds its record's vk + j for an insert, ~0 for a delete; lane i holds record
// i's inclusive LV prefix lincl, its length L (0: no record), vk and the delete flag dk.
__device__ __forceinline__ void fill_lvs(uint32_t *cbyte, uint32_t lv, uint32_t tot, uint32_t lincl, uint32_t L,
                                         uint32_t vk, bool dk, uint64_t hm, const Utf8Tab &tab) {
    const uint32_t l = lane();
    if (tot >= DTGPU_REC_FILL * popc(hm)) {   // long records: one wave-wide fill per record
        for (uint64_t m = hm; m; m &= m - 1) {   // uniform
            const uint32_t i = ctz(m);
            const uint32_t li = rdl(L, i), j0 = rdl(lincl, i) - li, vi = rdl(vk, i) + j0;
            const bool di = rdl(uint32_t(dk), i) != 0;
            if (di || !tab.n) {
                for (uint32_t k = l; k < li; k += 64) cbyte[lv + j0 + k] = di ? 0xFFFFFFFFu : vi + k;
            } else {
                for (uint32_t k0 = 0; k0 < li; k0 += 64) {   // uniform
                    const uint32_t v = utf8_xlat(tab, vi + k0 + l, vi + k0, vi + min(k0 + 63u, li - 1u));
                    if (k0 + l < li) cbyte[lv + j0 + k0 + l] = v;
                }
            }
        }
    } else for (uint32_t b = 0; b < tot; b += 64) {   // uniform: every lane runs the shuffles
        const uint32_t j = b + l;
        uint32_t r = 0;
#pragma unroll
        for (uint32_t s = 32; s >= 1; s >>= 1)
            if (uint32_t(__shfl(int(lincl), int(r + s - 1))) <= j) r += s;
        uint32_t v = uint32_t(__shfl(int(vk), int(r))) + j;
        const bool d = __shfl(int(dk), int(r)) != 0;
        if (tab.n) {   // the inserted chars of these LVs are numbered consecutively
            const uint64_t im = ballot(j < tot && !d);
            if (im) v = utf8_xlat(tab, v, rdl(v, ctz(im)), rdl(v, 63u - uint32_t(__clzll((long long)im))));
        }
        if (j < tot) cbyte[lv + j] = d ? 0xFFFFFFFFu : v;
    }
}

__device__ __forceinline__ bool batch_records(VQ &q, const uint32_t *bnd, uint32_t nb, uint32_t &bi, uint32_t &lv,
                                              uint32_t total, uint32_t &ins_size, int64_t &last_cursor,
                                              uint32_t &cr_valid, uint32_t &cr_lv, uint32_t &cr_len, uint32_t &cr_pos,
                                              uint32_t &cr_kind, uint32_t &cr_fwd, Quads &qp, uint4 *pre_out,
                                              uint32_t pre_cap, uint32_t *cbyte, const Utf8Tab &tab, uint32_t *job) {
    const uint32_t l = lane();
    const uint32_t h0 = q.head, cnt = q.cnt;
    const bool inq = l >= h0 && l < cnt;
    if (ballot(inq && q.end == 0xFFFFFFFFu)) return false;
    const uint64_t x = uint64_t(q.lo) | (uint64_t(q.hi) << 32);
    // roles: a head with has_length and diff_nz is followed by its diff varint
    const bool needs = (x & 1) && ((x >> 1) & 1);
    // successor's role given mine (head 0 / diff 1): (needs, false) in the queue, identity outside
    const uint32_t gf = compose_scan(inq ? fn_pack(needs, false) : fn_pack(false, true));
    const bool role_after = gf & 1u;                 // role of lane l + 1 (the head lane starts as a head)
    const bool role_here = __shfl_up(int(role_after), 1) != 0;   // (every lane runs the permute)
    const bool is_diff = l > h0 && role_here;
    const bool head = inq && !is_diff;
    const uint64_t x2 = uint64_t(uint32_t(__shfl(int(q.lo), int(min(l + 1, 63u))))) |
                        (uint64_t(uint32_t(__shfl(int(q.hi), int(min(l + 1, 63u))))) << 32);
    bool complete = head && (!needs || l + 1 < cnt);
    const uint64_t hm_all = ballot(head);
    const uint64_t inc = ballot(head && !complete);   // at most the last head
    uint64_t hm = hm_all & ~inc;
    if (!hm) return false;
    // record fields (head lanes)
    const bool has_length = x & 1, is_del = (x >> 2) & 1;
    uint64_t rest = x >> 3;
    bool fwd = true;
    uint64_t len;
    int64_t diff = 0;
    if (has_length) {
        if (is_del) { fwd = rest & 1; rest >>= 1; }
        len = rest;
        if (needs) diff = int64_t(x2 >> 1) * ((x2 & 1) ? -1 : 1);
    } else {
        len = 1;
        diff = int64_t(rest >> 1) * ((rest & 1) ? -1 : 1);
    }
    bool rec = (hm >> l) & 1;
    bool bad = rec && (len == 0 || len >= LIM31);
    const uint32_t L = rec && !bad ? uint32_t(len) : 0u;
    // LVs and cursors (64-bit cursor prefix over the records)
    const uint32_t lincl = scan_incl(L);
    const uint32_t lv_r = lv + lincl - L;
    const int64_t adj = !is_del ? int64_t(len) : (fwd ? 0 : -int64_t(len));
    const int64_t step = rec ? diff + adj : 0;
    // the cursor prefix in 32-bit wrapping arithmetic: record k's prefix is the previous record's
    // end cursor minus last_cursor, exact as an int32 while every earlier record's cursors lie in
    // [0, 2^31) -- which the checks below demand of each record (any failure rejects the batch)
    if (ballot(rec && (step != int64_t(int32_t(step)) || diff != int64_t(int32_t(diff))))) return false;
    const uint32_t cincl = scan_incl(uint32_t(step));
    const int64_t raw = last_cursor + int64_t(int32_t(cincl - uint32_t(step))) + diff;
    const int64_t st = (is_del && !fwd) ? raw - int64_t(len) : raw;
    bad = bad || (rec && (raw < 0 || st < 0 || uint64_t(st) + len >= LIM31 || uint64_t(raw) >= LIM31));
    bad = bad || (rec && uint64_t(lv_r) + len > total);
    // the agent run of each record: boundaries bnd[bi ..] (ascending ends of agent runs)
    const uint32_t bw = bi + l < nb ? bnd[bi + l] : 0xFFFFFFFFu;
    uint32_t c = 0;
#pragma unroll
    for (uint32_t sstep = 32; sstep >= 1; sstep >>= 1)
        if (uint32_t(__shfl(int(bw), int(c + sstep - 1))) <= lv_r) c += sstep;
    if (c == 63 && rdl(bw, 63) <= lv_r) c = 64;
    const uint32_t be = uint32_t(__shfl(int(bw), int(min(c, 63u))));
    bad = bad || (rec && (c >= 64 || uint64_t(lv_r) + len > be));
    if (const uint64_t bm = ballot(bad)) {   // the records before the first bad one still go as a batch
        hm &= (1ull << ctz(bm)) - 1ull;      // (every value below is a prefix over the records)
        if (!hm) return false;               // the first record itself: the caller takes it exactly
        rec = (hm >> l) & 1;
    }
    // content offsets per LV
    const uint32_t ilen = rec && !is_del ? L : 0u;
    const uint32_t iincl = scan_incl(ilen);
    {   // every LV of the batch, wave-strided: its record is the first lane whose lincl exceeds it
        const uint32_t tot = rdl(lincl, 63u - uint32_t(__clzll((long long)hm)));
        const uint32_t vk = ins_size + iincl - ilen - (lincl - L);   // content byte = vk + LV offset
        const bool dk = rec && is_del;
        if (job) {   // deferred: fill_kernel writes them once the document is decoded
            job[2 + l] = (hm >> l) ? lincl : tot;   // (no records past the batch's last one)
            job[66 + l] = vk;
            const uint64_t dm = ballot(dk);
            if (l == 0) { job[0] = lv; job[1] = tot; job[130] = uint32_t(dm); job[131] = uint32_t(dm >> 32); }
        } else {
            fill_lvs(cbyte, lv, tot, lincl, L, vk, dk, hm, tab);
        }
    }
    // RLE merge of the records into op runs
    const uint32_t pos = uint32_t(st), kind = is_del ? 1u : 0u, ofw = (!is_del || fwd) ? 1u : 0u;
    const uint64_t below = hm & lt_mask();
    const int pi = below ? int(63 - __clzll((long long)below)) : -1;
    const int psrc = pi >= 0 ? pi : int(l);
    uint32_t Pk = uint32_t(__shfl(int(kind), psrc)), Ppos = uint32_t(__shfl(int(pos), psrc));
    uint32_t PL = uint32_t(__shfl(int(L), psrc)), Plv = uint32_t(__shfl(int(lv_r), psrc));
    uint32_t Pf = uint32_t(__shfl(int(ofw), psrc));
    const int ppi = __shfl(pi, psrc);
    uint32_t PPpos = uint32_t(__shfl(int(pos), ppi >= 0 ? ppi : int(l)));
    bool pex = true, first = false;
    if (pi < 0) {   // the previous record is the open run's last one (the carry)
        first = true;
        pex = cr_valid != 0;
    } else if (ppi < 0) {
        PPpos = cr_pos;
    }
    bool g_0 = false, g_1 = true;   // identity on non-record lanes
    if (rec) {
        if (first) {   // the run state is known exactly: (cr_len == 1, cr_fwd)
            bool m = false;
            if (pex && cr_kind == kind && cr_lv + cr_len == lv_r) {
                if (!is_del) m = cr_pos + cr_len == pos;
                else m = ((cr_len == 1 || cr_fwd) && (L == 1 || fwd) && pos == cr_pos) ||
                         ((cr_len == 1 || !cr_fwd) && (L == 1 || !fwd) && pos + L == cr_pos);
            }
            g_0 = g_1 = m;
        } else {
            const bool base = Pk == kind && Plv + PL == lv_r;
            if (!is_del) {
                g_0 = g_1 = base && Ppos + PL == pos;
            } else {
                const bool f1 = Ppos == PPpos;   // P was appended: forwards iff it kept the run's position
                g_0 = base && (((PL == 1 || Pf) && (L == 1 || fwd) && pos == Ppos) ||
                               ((PL == 1 || !Pf) && (L == 1 || !fwd) && pos + L == Ppos));
                g_1 = base && ((f1 && (L == 1 || fwd) && pos == Ppos) || (!f1 && (L == 1 || !fwd) && pos + L == Ppos));
            }
        }
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const bool b0 = __shfl_up(int(g_0), d) != 0, b1 = __shfl_up(int(g_1), d) != 0;
        if (l >= uint32_t(d)) {
            const bool n0 = b0 ? g_1 : g_0, n1 = b1 ? g_1 : g_0;
            g_0 = n0; g_1 = n1;
        }
    }
    const bool merged = rec && g_0;   // the first record's function is constant: any start works
    const bool rhead = rec && !merged;
    const uint64_t rh = ballot(rhead);
    // runs that close in this batch: the open one (at slot qp.at) as soon as any record heads a
    // new run, and every run headed here except the last (it stays open, in cr_*)
    qp.flush(pre_out);
    const uint32_t n_heads = popc(rh);
    const uint32_t n_close = (n_heads && cr_valid ? 1u : 0u) + (n_heads ? n_heads - 1 : 0u);
    if (qp.at + n_close > pre_cap) return false;
    const uint64_t base_at = qp.at + (cr_valid ? 1u : 0u);   // slot of the first run headed here
    // run fields at each record: its head's, the length so far, the current pos / direction
    const uint64_t hle = rh & (lt_mask() | (1ull << l));
    const int hh = hle ? int(63 - __clzll((long long)hle)) : -1;
    const int hs = hh >= 0 ? hh : int(l);
    const uint32_t Hlv = uint32_t(__shfl(int(lv_r), hs)), Hpos = uint32_t(__shfl(int(pos), hs));
    const uint32_t Hk = uint32_t(__shfl(int(kind), hs));
    const uint32_t Hpre = uint32_t(__shfl(int(lincl - L), hs));
    const uint32_t rank = uint32_t(__shfl(int(popc(rh & lt_mask())), hs));
    uint32_t rlv, rlen, rpos, rk, rf;
    if (hh >= 0) {
        rlv = Hlv; rlen = lincl - Hpre; rk = Hk;
        if (!merged) { rpos = pos; rf = ofw; }
        else if (!Hk) { rpos = Hpos; rf = 1; }
        else { rf = pos == Ppos ? 1u : 0u; rpos = rf ? Hpos : pos; }
    } else {   // still the open run
        rlv = cr_lv; rlen = cr_len + lincl; rk = cr_kind;
        if (!cr_kind) { rpos = cr_pos; rf = 1; }
        else { rf = (first ? pos == cr_pos : pos == Ppos) ? 1u : 0u; rpos = rf ? cr_pos : pos; }
    }
    // the open run closes where the first run head appears: written from the carry when that
    // head is the batch's first record, else by the record before that head
    const uint32_t f0 = ctz(hm);
    if (cr_valid && ((rh >> f0) & 1) && l == 0) pre_out[qp.at] = make_uint4(cr_lv, cr_len, cr_pos, cr_kind | (cr_fwd << 1));
    const uint64_t above = hm & ~(lt_mask() | (1ull << l));
    const bool last = rec && above && ((rh >> ctz(above)) & 1);
    if (last) pre_out[hh >= 0 ? base_at + rank : qp.at] = make_uint4(rlv, rlen, rpos, rk | (rf << 1));
    qp.at += n_close;
    // the batch's last record carries the open run
    const uint32_t t = 63 - uint32_t(__clzll((long long)hm));
    cr_valid = 1;
    cr_lv = rdl(rlv, t); cr_len = rdl(rlen, t); cr_pos = rdl(rpos, t); cr_kind = rdl(rk, t); cr_fwd = rdl(rf, t);
    // consume the records' varints
    const uint32_t vlast = t + rdl(needs ? 1u : 0u, t);
    q.at = rdl(q.end, vlast);
    q.head = vlast + 1;
    lv += rdl(lincl, t);
    ins_size += rdl(iincl, t);
    last_cursor += int64_t(int32_t(rdl(cincl, t)));
    bi += rdl(c, t);
    return true;
}

// Up to 64 queued OpParents varints at once (decode_oplog.rs:856-913): each record is its span
// length and a parent list; the varints' roles (span length or parent) come from a prefix
// composition (a parent continues the list iff it is local with "more" set), span starts from a
// prefix sum, Graph::push's extension test (one parent, the span just before) is pairwise, and
// the entries closed here, their parent offsets and sorted parents are written by rank.  The
// frontier after the batch is (frontier before + every span's last LV) minus every parent named
// in it: a parent is always below its record's start, so it names an element present at that
// point, and elements are never re-added.  Returns false without consuming anything when the
// batch is not the plain case (a foreign parent other than ROOT, more than 8 parents, an error
// entry, an out-of-range length or parent, capacity, a frontier that could reach 64): the caller
// then takes one record the exact way, which yields the reference's status.
__device__ __forceinline__ bool batch_parents(VQ &q, uint32_t &next_file, uint32_t next_assign, uint32_t &pe_valid,
                                              uint32_t &pe_start, uint32_t &pe_end, uint32_t &pe_poff, uint32_t &n_ent,
                                              uint32_t &n_par, uint32_t &fr, uint32_t &fn, const DecodeDesc &D,
                                              const Out &O) {
    const uint32_t l = lane();
    const uint32_t h0 = q.head, cnt = q.cnt;
    const bool inq = l >= h0 && l < cnt;
    if (ballot(inq && q.end == 0xFFFFFFFFu)) return false;
    const uint32_t x = q.lo;
    const bool foreign = x & 1u, more = (x >> 1) & 1u;
    const uint64_t nn64 = (uint64_t(q.lo) | (uint64_t(q.hi) << 32)) >> 2;
    // roles: state 1 = a parent varint; a span length is always followed by a parent
    bool g0 = inq, g1 = inq ? (!foreign && more) : true;   // successor's state given mine (0 / 1)
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const bool b0 = __shfl_up(int(g0), d) != 0, b1 = __shfl_up(int(g1), d) != 0;
        if (l >= uint32_t(d)) {
            const bool n0 = b0 ? g1 : g0, n1 = b1 ? g1 : g0;
            g0 = n0; g1 = n1;
        }
    }
    const bool role_here = __shfl_up(int(g0), 1) != 0;   // (every lane runs the permute)
    const bool isP = inq && l > h0 && role_here;
    const bool isH = inq && !isP;
    const uint64_t fb = ballot(isP && foreign && nn64 != 0);
    const uint32_t first_bad = fb ? ctz(fb) : 64u;
    const uint64_t tm = ballot(isP && (foreign || !more));   // list terminators
    const uint64_t after = tm & ~(lt_mask() | (1ull << l));
    const uint32_t e = after ? ctz(after) : 64u;              // this span's terminator
    const bool root_e = __shfl(int(foreign), int(min(e, 63u))) != 0;
    const uint32_t np = e - l - (root_e ? 1u : 0u);
    const bool ok = e < cnt && e < first_bad && np <= 8u;
    const uint64_t nk_ = ballot(isH && !ok);
    const uint32_t first_notok = nk_ ? ctz(nk_) : 64u;
    const bool rec = isH && l < first_notok;
    const uint64_t hm = ballot(rec);
    if (!hm) return false;
    const uint32_t nrec = popc(hm);
    if (fn + nrec > DECODE_MAX_FRONTIER) return false;
    // spans
    bool bad = rec && (q.hi != 0 || x == 0 || x >= (1u << 25));
    const uint32_t L = rec && !bad ? x : 0u;
    const uint32_t incl = scan_incl(L);
    const uint32_t start = next_file + incl - L;
    bad = bad || (rec && uint64_t(start) + L > next_assign);
    // parents: a parent varint reads its span's start from the nearest span lane below it
    const uint64_t hall = ballot(isH) & (lt_mask() | (1ull << l));
    const int hsrc = hall ? int(63 - __clzll((long long)hall)) : int(l);
    const uint32_t pstart = uint32_t(__shfl(int(start), hsrc));
    const bool prec = __shfl(int(rec), hsrc) != 0;
    const bool pl = isP && prec && !foreign;
    const uint32_t nn = uint32_t(nn64);
    bad = bad || (pl && (nn64 == 0 || nn64 > pstart));
    if (ballot(bad)) return false;
    const uint32_t pv = pstart - nn;
    const uint32_t p0 = uint32_t(__shfl(int(pv), int(min(l + 1, 63u))));
    // Graph::push: one parent, the span just before (the pending entry always ends at `start`)
    const bool ext = rec && np == 1u && p0 + 1u == start && (l != h0 || pe_valid);
    const bool eh = rec && !ext;
    const uint64_t em = ballot(eh);
    const uint32_t npe = eh ? np : 0u;
    const uint32_t pincl = scan_incl(npe);
    const uint32_t poff = n_par + pincl - npe;
    const uint32_t t = 63 - uint32_t(__clzll((long long)hm));
    const uint32_t n_close = em ? popc(em) - 1u + pe_valid : 0u;
    if (n_ent + n_close > D.ent_cap || n_par + rdl(pincl, t) > D.par_cap) return false;
    // entries closed here: each entry head closes the one before it
    const uint32_t k = popc(em & lt_mask());
    const uint64_t pem = em & lt_mask();
    const int psrc = pem ? int(63 - __clzll((long long)pem)) : int(l);
    const uint32_t prev_start = uint32_t(__shfl(int(start), psrc)), prev_poff = uint32_t(__shfl(int(poff), psrc));
    if (eh && (k || pe_valid)) {
        const uint32_t idx = n_ent + pe_valid + k - 1u;
        O.ent[idx] = make_uint2(k ? prev_start : pe_start, start);
        O.poff[idx] = k ? prev_poff : pe_poff;
    }
    // each parent at its rank in its list: smaller values, then equal values at lower lanes
    const int gk = pl ? hsrc : -1;
    uint32_t prank = 0;
    for (int d = 1; d < 8; d++) {
        if (!ballot(rec && np > uint32_t(d))) break;   // lists no longer than d are ranked
        const uint32_t pd = uint32_t(__shfl_up(int(pv), d)), pu = uint32_t(__shfl_down(int(pv), d));
        const int gd = __shfl_up(gk, d), gu = __shfl_down(gk, d);
        prank += (l >= uint32_t(d) && gd == gk && pd <= pv) ? 1u : 0u;
        prank += (l + d < 64u && gu == gk && pu < pv) ? 1u : 0u;
    }
    const bool peh = __shfl(int(eh), hsrc) != 0;
    const uint32_t ppoff = uint32_t(__shfl(int(poff), hsrc));
    if (pl && peh) O.par[ppoff + prank] = pv;
    // frontier: the old elements, then each span's last LV, minus every parent named here
    const uint32_t ridx = popc(hm & lt_mask());
    const uint32_t dst = rec ? fn + ridx : (fn + nrec + popc(~hm & lt_mask())) & 63u;
    const uint32_t ev = uint32_t(__builtin_amdgcn_ds_permute(int(dst << 2), int(start + L - 1u)));
    const uint32_t cand = l < fn ? fr : ev;
    bool rm = false;
    for (uint64_t pm = ballot(pl); pm; pm &= pm - 1) rm |= cand == rdl(pv, ctz(pm));
    const bool keep = l < fn + nrec && !rm;
    const uint64_t km = ballot(keep);
    const uint32_t nk = popc(km);
    const uint32_t to = keep ? popc(km & lt_mask()) : nk + popc(~km & lt_mask());
    const uint32_t moved = uint32_t(__builtin_amdgcn_ds_permute(int(to << 2), int(cand)));
    fn = nk;
    fr = l < fn ? moved : 0u;
    // state after the batch
    const uint32_t last_e = rdl(e, t);
    q.at = rdl(q.end, last_e);
    q.head = last_e + 1;
    next_file += rdl(incl, t);
    pe_end = rdl(start + L, t);
    if (em) {
        const uint32_t le = 63 - uint32_t(__clzll((long long)em));
        pe_start = rdl(start, le);
        pe_poff = rdl(poff, le);
    }
    pe_valid = 1;
    n_ent += n_close;
    n_par += rdl(pincl, t);
    return true;
}

// Up to 64 queued OpVersions varints at once (decode_oplog.rs:764-800): each record is (file agent
// + jump flag, length[, jump]); the roles come from a prefix composition of 4-state functions
// (agent / length, no jump follows / length, a jump follows / jump), each record's seq start
// from its file agent's cursor plus a prefix sum over the records of that agent, the RLE merge
// of agent runs (same agent, seq contiguous) is pairwise, and the runs closed here are written
// by rank, as are the run-end boundaries the op records are split at.  Returns false without
// consuming anything when the batch is not the plain case (an error entry, an unknown agent, a
// seq or LV out of range, capacity): the caller then takes one record the exact way.
__device__ __forceinline__ uint32_t compose4(uint32_t g, uint32_t f) {   // (g after f)[s] = g[f[s]]
    uint32_t r = 0;
#pragma unroll
    for (uint32_t s = 0; s < 4; s++) r |= ((g >> (2u * ((f >> (2u * s)) & 3u))) & 3u) << (2u * s);
    return r;
}

__device__ __forceinline__ bool batch_agents(VQ &q, uint32_t n_file, uint32_t *fseq, const uint32_t *fmap,
                                             uint64_t &next_assign, uint32_t &ca_valid, uint32_t &ca_lv,
                                             uint32_t &ca_len, uint32_t &ca_agent, uint32_t &ca_seq, Quads &qa,
                                             uint4 *aruns_out, uint32_t arun_cap, uint32_t &nb, uint32_t &bbuf,
                                             uint32_t *bnd) {
    const uint32_t l = lane();
    const uint32_t h0 = q.head, cnt = q.cnt;
    const bool inq = l >= h0 && l < cnt;
    if (ballot(inq && q.end == 0xFFFFFFFFu)) return false;
    const uint32_t x = q.lo;
    // successor's state given mine: agent -> length (kind by my jump flag); length -> agent or
    // jump; jump -> agent.  Identity (0xE4) outside the queue.
    uint32_t f = inq ? (((x & 1u) ? 2u : 1u) | (3u << 4)) : 0xE4u;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = uint32_t(__shfl_up(int(f), d));
        if (l >= uint32_t(d)) f = compose4(f, o);
    }
    const uint32_t fb = uint32_t(__shfl_up(int(f), 1));   // every lane runs the permute (no inactive sources)
    const uint32_t st = l > h0 ? (fb & 3u) : 0u;
    const bool head = inq && st == 0u;
    const bool hj = x & 1u;
    const uint32_t x1 = uint32_t(__shfl(int(q.lo), int(min(l + 1, 63u))));
    const uint32_t x1h = uint32_t(__shfl(int(q.hi), int(min(l + 1, 63u))));
    const uint32_t x2 = uint32_t(__shfl(int(q.lo), int(min(l + 2, 63u))));
    const uint32_t x2h = uint32_t(__shfl(int(q.hi), int(min(l + 2, 63u))));
    const bool ok = l + 1u + (hj ? 1u : 0u) < cnt;
    const uint64_t nk_ = ballot(head && !ok);
    const uint32_t first_nk = nk_ ? ctz(nk_) : 64u;
    const bool rec = head && l < first_nk;
    const uint64_t hm = ballot(rec);
    if (!hm) return false;
    const uint32_t fa1 = x >> 1;
    bool bad = rec && (q.hi != 0 || fa1 == 0 || fa1 - 1u >= n_file || x1h != 0 || x1 >= (1u << 25));
    const uint32_t fa = rec && !bad ? fa1 - 1u : 0u;
    const uint32_t alen = rec && !bad ? x1 : 0u;
    const uint64_t jz = uint64_t(x2) | (uint64_t(x2h) << 32);
    const int64_t jump = (rec && hj) ? int64_t(jz >> 1) * ((jz & 1) ? -1 : 1) : 0;
    const int64_t delta = jump + int64_t(alen);
    const uint32_t base = rec ? fseq[fa] : 0u;
    // each record's cursor: its file agent's cursor plus the deltas of that agent's earlier records
    int64_t cb = 0;
    bool last_of_agent = false;
    for (uint64_t rem = hm; rem;) {
        const uint32_t f0 = rdl(fa, ctz(rem));
        const uint64_t same = ballot(rec && fa == f0);
        const bool me = (same >> l) & 1;
        const int64_t v = me ? delta : 0;
        int64_t inc = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int64_t o = __shfl_up(inc, d);
            if (l >= uint32_t(d)) inc += o;
        }
        if (me) { cb = inc - v; last_of_agent = l == 63u - uint32_t(__clzll((long long)same)); }
        rem &= ~same;
    }
    const int64_t sstart = int64_t(base) + cb + jump;
    bad = bad || (rec && (sstart < 0 || uint64_t(sstart) + alen >= LIM31));
    const uint32_t lincl = scan_incl(alen);
    bad = bad || (rec && next_assign + lincl >= LIM31);
    const uint32_t t = 63 - uint32_t(__clzll((long long)hm));
    const uint32_t total = rdl(lincl, t);
    if (ballot(bad)) return false;
    const uint32_t s32 = uint32_t(sstart), lv_r = uint32_t(next_assign) + lincl - alen;
    const uint32_t agent = rec ? fmap[fa] : 0u;
    // agent runs (AgentAssignment RLE): same agent and seq contiguous with the previous record
    const uint64_t below = hm & lt_mask();
    const int psrc = below ? int(63 - __clzll((long long)below)) : int(l);
    const uint32_t Pa = uint32_t(__shfl(int(agent), psrc)), Pe = uint32_t(__shfl(int(s32 + alen), psrc));
    const bool merged = rec && (below ? (Pa == agent && Pe == s32)
                                      : (ca_valid && ca_agent == agent && ca_seq + ca_len == s32));
    const uint64_t rh = ballot(rec && !merged);
    const uint32_t n_heads = popc(rh);
    const uint32_t n_close = (n_heads && ca_valid ? 1u : 0u) + (n_heads ? n_heads - 1u : 0u);
    const uint64_t nzm = ballot(rec && alen != 0);
    const uint32_t nzc = popc(nzm);
    if (qa.count() + n_close > arun_cap || nb + nzc > 4 * arun_cap) return false;
    // file agent cursors
    __syncthreads();
    if (rec && last_of_agent) fseq[fa] = s32 + alen;
    __syncthreads();
    // runs closed here: the open one (if a record heads a new run), every head but the last
    qa.flush(aruns_out);
    const uint32_t lv_f0 = uint32_t(__shfl(int(lv_r), int(rh ? ctz(rh) : 0u)));
    if (rh && ca_valid && l == 0)
        aruns_out[qa.at] = make_uint4(ca_lv, ca_len + (lv_f0 - uint32_t(next_assign)), ca_agent, ca_seq);
    const uint64_t hab = rh & ~(lt_mask() | (1ull << l));
    const uint32_t lvn = uint32_t(__shfl(int(lv_r), int(hab ? ctz(hab) : l)));
    const bool hd = (rh >> l) & 1;
    if (hd && hab) aruns_out[qa.at + (ca_valid ? 1u : 0u) + popc(rh & lt_mask())] = make_uint4(lv_r, lvn - lv_r, agent, s32);
    qa.at += n_close;
    if (rh) {
        const uint32_t th = 63 - uint32_t(__clzll((long long)rh));
        ca_lv = rdl(lv_r, th); ca_agent = rdl(agent, th); ca_seq = rdl(s32, th);
        ca_len = uint32_t(next_assign) + total - ca_lv;
    } else {
        ca_len += total;
    }
    ca_valid = 1;
    // run-end boundaries of the non-empty records; the partial block stays in bbuf
    const bool nz = (nzm >> l) & 1;
    const uint32_t rk = popc(nzm & lt_mask());
    const uint32_t endv = lv_r + alen;
    if (nz) bnd[nb + rk] = endv;
    if (l < (nb & 63u)) bnd[(nb & ~63u) + l] = bbuf;
    const uint32_t dst = nz ? rk : nzc + popc(~nzm & lt_mask());
    const uint32_t cmp = uint32_t(__builtin_amdgcn_ds_permute(int(dst << 2), int(endv)));
    const uint32_t nb2 = nb + nzc;
    const uint32_t idx = (nb2 & ~63u) + l;
    const uint32_t pulled = uint32_t(__builtin_amdgcn_ds_bpermute(int(((idx - nb) & 63u) << 2), int(cmp)));
    bbuf = idx < nb ? bbuf : pulled;
    nb = nb2;
    next_assign += total;
    const uint32_t vlast = t + 1u + rdl(hj ? 1u : 0u, t);
    q.at = rdl(q.end, vlast);
    q.head = vlast + 1;
    return true;
}

struct FastOut { uint32_t status, n_aruns, n_pre, n_lv, ins_size, n_jobs; uint64_t t_mid; };

// Non-ASCII insert text on the batched path: fast_runs numbers the inserted chars (cbyte = the
// char's index), then this pass puts each char's byte offset in place, 64 LVs at a time: the
// chunk's inserted chars are the next ones of the text, so their starts are the next char-start
// bytes from a running byte cursor (one ballot per 64 text bytes, a rank into LDS).  Returns
// false (the caller takes the exact path) when the numbering does not run 0, 1, 2, ... along
// the LVs or the text ends early.
__device__ __forceinline__ uint32_t count_char_starts(const uint8_t *t, uint32_t n) {
    uint32_t c = 0;
    for (uint32_t i = 0; i < n; i += 64) {
        const uint32_t j = i + lane();
        c += popc(ballot(j < n && (t[j] & 0xC0u) != 0x80u));
    }
    return c;
}
__device__ __forceinline__ bool utf8_offsets(const uint8_t *t, uint32_t n, uint32_t *cbyte, uint32_t n_lv, uint32_t n_chars) {
    __shared__ uint32_t slot[64];
    const uint32_t l = lane();
    uint32_t cur = 0, kbase = 0;
    for (uint32_t lv0 = 0; lv0 < n_lv; lv0 += 64) {
        const uint32_t lv = lv0 + l;
        const uint32_t k = lv < n_lv ? cbyte[lv] : 0xFFFFFFFFu;
        const bool ins = k != 0xFFFFFFFFu;
        const uint64_t m = ballot(ins);
        if (!m) continue;
        const uint32_t need = popc(m), r = popc(m & lt_mask());
        if (ballot(ins && k != kbase + r)) return false;
        uint32_t got = 0, lastb = 0, lastc = 0;
        for (uint32_t w = cur; got < need; w += 64) {
            if (w >= n) return false;
            const uint32_t j = w + l;
            const uint32_t c = j < n ? t[j] : 0x80u;
            const bool st = (c & 0xC0u) != 0x80u;
            const uint64_t sm = ballot(st);
            const uint32_t rk = got + popc(sm & lt_mask());
            if (st && rk < need) slot[rk] = j;
            // the chunk's last char start and its lead byte, straight from the window's lanes
            // (no read back of the slot and no dependent byte load before the next chunk)
            const uint64_t lm = ballot(st && rk == need - 1);
            if (lm) { lastb = rdl(j, ctz(lm)); lastc = rdl(c, ctz(lm)); }
            got += popc(sm);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (ins) cbyte[lv] = slot[r];
        __builtin_amdgcn_wave_barrier();   // (slot is rewritten by the next chunk: reads first, in order within the wave)
        cur = lastb + (lastc < 0x80 ? 1u : (lastc & 0xE0u) == 0xC0u ? 2u : (lastc & 0xF0u) == 0xE0u ? 3u : 4u);
        kbase += need;
    }
    return kbase == n_chars;
}

__device__ __forceinline__ FastOut fast_runs(VQ qav, VQ qtp, VQ runs, uint32_t text_n, uint32_t n_file, uint32_t *fseq,
                                          const uint32_t *fmap, uint32_t *vs, uint4 *aruns_out, uint4 *pre_out,
                                          uint32_t *cbyte, uint32_t *bnd, uint32_t arun_cap, uint32_t pre_cap,
                                          uint32_t lv_cap, const Utf8Tab &tab, uint32_t *jobs, uint32_t job_cap) {
    FastOut fo{1, 0, 0, 0, 0, 0, 0};
    uint32_t nj = 0;   // deferred fill jobs written (jobs: DecodeParams::fill slots, job_cap of them)
    uint64_t ins_total = 0;
    while (runs.left()) {
        uint64_t x;
        if (vq_pop(runs, x, vs) || !(x & 1) || !(x >> 1)) return fo;
        ins_total += x >> 1;
    }
    if (ins_total != text_n) return fo;
    Quads qa, qp;
    qa.init(); qp.init();
    uint32_t ca_valid = 0, ca_lv = 0, ca_len = 0, ca_agent = 0, ca_seq = 0;
    uint32_t cr_valid = 0, cr_lv = 0, cr_len = 0, cr_pos = 0, cr_kind = 0, cr_fwd = 0;
    uint64_t next_assign = 0;
    uint32_t nb = 0, bbuf = 0;
    while (qav.left()) {
        if (qav.head == qav.cnt) vq_refill(qav, vs);
        else if (qav.cnt - qav.head < 6 && qav.wpos < qav.len) vq_topup(qav, vs);
        if (qav.cnt - qav.head >= 6 && batch_agents(qav, n_file, fseq, fmap, next_assign, ca_valid, ca_lv, ca_len, ca_agent,
                                                    ca_seq, qa, aruns_out, arun_cap, nb, bbuf, bnd))
            continue;
        uint64_t n, alen;
        int64_t jump = 0;
        if (vq_pop(qav, n, vs)) return fo;
        const bool has_jump = n & 1;
        n >>= 1;
        if (vq_pop(qav, alen, vs)) return fo;
        if (has_jump && vq_zigzag(qav, jump, vs)) return fo;
        if (n == 0 || n - 1 >= n_file) return fo;
        const uint32_t fa = uint32_t(n - 1);
        const int64_t sstart = int64_t(fseq[fa]) + jump;
        if (sstart < 0 || uint64_t(sstart) + alen >= LIM31 || next_assign + alen >= LIM31) return fo;
        __syncthreads();
        if (lane() == 0) fseq[fa] = uint32_t(sstart + int64_t(alen));
        __syncthreads();
        const uint32_t agent = fmap[fa];
        if (ca_valid && ca_agent == agent && ca_lv + ca_len == next_assign && uint64_t(ca_seq) + ca_len == uint64_t(sstart)) {
            ca_len += uint32_t(alen);
        } else {
            if (ca_valid) {
                if (qa.count() >= arun_cap) return fo;
                qa.push(ca_lv, ca_len, ca_agent, ca_seq, aruns_out);
            }
            ca_valid = 1; ca_lv = uint32_t(next_assign); ca_len = uint32_t(alen); ca_agent = agent; ca_seq = uint32_t(sstart);
        }
        next_assign += alen;
        if (alen) {
            if (nb >= 4 * arun_cap) return fo;
            bbuf = lane() == (nb & 63u) ? uint32_t(next_assign) : bbuf;
            if ((++nb & 63u) == 0) bnd[nb - 64 + lane()] = bbuf;
        }
    }
    if ((nb & 63u) && lane() < (nb & 63u)) bnd[(nb & ~63u) + lane()] = bbuf;
    wave_fence();
    fo.t_mid = __builtin_amdgcn_s_memtime();
    uint32_t bblk = 0xFFFFFFFFu, bcache = 0, bi = 0;
    const uint32_t total = uint32_t(next_assign);
    if (total > lv_cap) return fo;
    uint32_t lv = 0, ins_size = 0;
    int64_t last_cursor = 0;
    while (lv < total) {
        if (!qtp.left()) return fo;
        if (qtp.head == qtp.cnt) vq_refill(qtp, vs);
        else if (qtp.cnt - qtp.head < 8 && qtp.wpos < qtp.len) vq_topup(qtp, vs);
        uint32_t *job = jobs && nj < job_cap ? jobs + nj * FILL_JOB : nullptr;
        if (qtp.cnt - qtp.head >= 8 && batch_records(qtp, bnd, nb, bi, lv, total, ins_size, last_cursor, cr_valid, cr_lv,
                                                     cr_len, cr_pos, cr_kind, cr_fwd, qp, pre_out, pre_cap, cbyte, tab, job)) {
            if (job) nj++;
            bblk = 0xFFFFFFFFu;   // bi moved: the cached boundary window is stale
            continue;
        }
        uint64_t x;
        if (vq_pop(qtp, x, vs)) return fo;
        const bool has_length = x & 1; x >>= 1;
        const bool diff_nz = x & 1; x >>= 1;
        const bool is_del = x & 1; x >>= 1;
        int64_t diff = 0;
        bool fwd = true;
        uint64_t l;
        if (has_length) {
            if (is_del) { fwd = x & 1; x >>= 1; }
            if (diff_nz && vq_zigzag(qtp, diff, vs)) return fo;
            l = x;
        } else {
            l = 1;
            diff = int64_t(x >> 1) * ((x & 1) ? -1 : 1);
        }
        const int64_t raw = int64_t(uint64_t(last_cursor) + uint64_t(diff));
        int64_t st;
        if (!is_del) { st = raw; last_cursor = raw + int64_t(l); }
        else if (fwd) { st = raw; last_cursor = raw; }
        else { st = raw - int64_t(l); last_cursor = raw - int64_t(l); }
        if (l == 0 || l >= LIM31) return fo;
        uint32_t rem = uint32_t(l);
        while (rem && lv < total) {
            uint32_t be;
            for (;;) {   // end of the agent run holding lv
                if ((bi & ~63u) != bblk) {
                    bblk = bi & ~63u;
                    bcache = bblk + lane() < nb ? bnd[bblk + lane()] : 0xFFFFFFFFu;
                }
                be = rdl(bcache, bi & 63u);
                if (be > lv) break;
                bi++;
            }
            const uint32_t take = min(rem, be - lv);
            const int64_t ppos = (!is_del || fwd) ? st : st + int64_t(rem) - int64_t(take);
            if (ppos < 0 || uint64_t(ppos) >= LIM31) return fo;
            const uint32_t pos = uint32_t(ppos);
            bool merged = false;
            if (!is_del) {
                if (!tab.n) {
                    for (uint32_t i = lane(); i < take; i += 64) cbyte[lv + i] = ins_size + i;
                } else {
                    for (uint32_t i0 = 0; i0 < take; i0 += 64) {   // uniform
                        const uint32_t v = utf8_xlat(tab, ins_size + i0 + lane(), ins_size + i0,
                                                     ins_size + min(i0 + 63u, take - 1u));
                        if (i0 + lane() < take) cbyte[lv + i0 + lane()] = v;
                    }
                }
                ins_size += take;
                if (cr_valid && cr_kind == 0 && cr_lv + cr_len == lv && cr_pos + cr_len == pos) { cr_len += take; merged = true; }
                st += int64_t(take);
            } else {
                for (uint32_t i = lane(); i < take; i += 64) cbyte[lv + i] = 0xFFFFFFFFu;
                if (cr_valid && cr_kind == 1 && cr_lv + cr_len == lv) {
                    if ((cr_len == 1 || cr_fwd) && (take == 1 || fwd) && pos == cr_pos) {
                        cr_len += take; cr_fwd = 1; merged = true;
                    } else if ((cr_len == 1 || !cr_fwd) && (take == 1 || !fwd) && uint64_t(pos) + take == cr_pos) {
                        cr_pos = pos; cr_len += take; cr_fwd = 0; merged = true;
                    }
                }
            }
            if (!merged) {
                if (cr_valid) {
                    if (qp.count() >= pre_cap) return fo;
                    qp.push(cr_lv, cr_len, cr_pos, cr_kind | (cr_fwd << 1), pre_out);
                }
                cr_valid = 1; cr_lv = lv; cr_len = take; cr_pos = pos; cr_kind = is_del ? 1u : 0u;
                cr_fwd = (!is_del || fwd) ? 1u : 0u;
            }
            lv += take;
            rem -= take;
        }
    }
    if (ins_size != ins_total) return fo;
    if (ca_valid) {
        if (qa.count() >= arun_cap) return fo;
        qa.push(ca_lv, ca_len, ca_agent, ca_seq, aruns_out);
    }
    if (cr_valid) {
        if (qp.count() >= pre_cap) return fo;
        qp.push(cr_lv, cr_len, cr_pos, cr_kind | (cr_fwd << 1), pre_out);
    }
    qa.flush(aruns_out);
    qp.flush(pre_out);
    fo.status = 0;
    fo.n_jobs = nj;
    fo.n_aruns = uint32_t(qa.at);
    fo.n_pre = uint32_t(qp.at);
    fo.n_lv = lv;
    fo.ins_size = ins_size;
    return fo;
}

template <bool SIZE>
__device__ __forceinline__ int decode_doc(const DecodeParams &P, const DecodeDesc &D, DecodeResult &R, const Lds &L,
                                          uint32_t doc) {
    Ctx C;
    C.in = P.in + D.in_off;
    C.lz = P.lz + D.lz_off;
    C.w0 = Win{C.in, 0x80000000u, 0};
    C.w1 = Win{C.lz, 0x80000000u, 0};
    const uint32_t len = D.in_len;
    Out O;
    O.aruns = reinterpret_cast<uint4 *>(P.aruns) + D.arun_off;
    O.alist = P.alist + 4 * D.arun_off;
    O.pre = reinterpret_cast<uint4 *>(P.pre) + D.pre_off;
    O.ops = reinterpret_cast<uint4 *>(P.ops) + D.op_off;
    O.ent = reinterpret_cast<uint2 *>(P.ent) + D.ent_off;
    O.poff = P.poff + D.poff_off;
    O.par = P.par + D.par_off;
    O.cbyte = P.cbyte + D.lv_off;
    O.ver = P.ver + D.ver_off;
    O.agents = reinterpret_cast<uint2 *>(P.agents) + D.agent_off;
    O.content = P.content + D.content_off;

    uint64_t t_prev = __builtin_amdgcn_s_memtime();
    auto prof_mark = [&](int k) {   // core-clock cycles per phase (DecodeResult::prof)
        const uint64_t t = __builtin_amdgcn_s_memtime();
        R.prof[k] += uint32_t(t - t_prev);
        t_prev = t;
    };
    if (len < 8) return UnexpectedEOF;
    {
        const char *magic = "DMNDTYPS";
        for (uint32_t i = 0; i < 8; i++)
            if (C.byte(0, i) != uint32_t(uint8_t(magic[i]))) return InvalidMagic;
    }
    Rd r{0, 8, len - 8};
    uint64_t pv;
    TRY(C.u64v(r, pv));
    if (pv != 0) return UnsupportedProtocolVersion;

    Rd comp{SRC_LZ, 0, 0};
    bool has_comp = false;
    {
        bool found; Rd c;
        TRY(C.chunk_if(r, 5, found, c));
        if (found) {
            uint64_t ulen;
            TRY(C.u64v(c, ulen));
            if (ulen > (uint64_t(1) << 34)) return LZ4DecompressionError;
            // an LZ4 block expands at most ~255x: a larger claim cannot decompress exactly
            if (ulen > 255ull * c.n + 64) return LZ4DecompressionError;
            if (SIZE) {
                R.lz_len = uint32_t(ulen);
            } else {
                if (ulen > D.lz_cap) return ErrCapacity;
                const uint32_t pre = P.lz_pre ? P.lz_pre[doc] : 0u;   // lz4_kernel's verdict
                if (pre == 2u) return LZ4DecompressionError;
                if (pre != 1u) {
#ifdef DT_LZPROF
                    if (!lz4_block(C, c, C.lz, uint32_t(ulen), reinterpret_cast<uint4 *>(L.fr), L.lzr, P.lz_ring, R.prof))
                        return LZ4DecompressionError;
#else
                    if (!lz4_block(C, c, C.lz, uint32_t(ulen), reinterpret_cast<uint4 *>(L.fr), L.lzr, P.lz_ring))
                        return LZ4DecompressionError;
#endif
                }
            }
            comp.n = uint32_t(ulen);
            has_comp = true;
        }
    }

    prof_mark(0);
    uint32_t n_file = 0, n_agents = 0;
    {   // FileInfo (decode_oplog.rs:197-227)
        Rd fi, an, tmp;
        bool found;
        TRY(C.expect_chunk(r, 1, fi));
        TRY(C.chunk_if(fi, 2, found, tmp));
        R.doc_id_len = 0xFFFFFFFFu;
        if (found) {
            uint64_t dt;
            TRY(C.u32v(tmp, dt));
            if (dt != 4) return UnknownChunk;
            R.doc_id_off = tmp.p;
            R.doc_id_len = tmp.n;
            bool asc;
            if (!SIZE && !utf8_ok(C.in + tmp.p, tmp.n, asc)) return InvalidUTF8;
        }
        TRY(C.expect_chunk(fi, 3, an));
        TRY(C.chunk_if(fi, 4, found, tmp));
        while (an.n) {
            uint64_t nl;
            TRY(C.u64v(an, nl));
            if (nl > an.n) return InvalidLength;
            const uint32_t noff = an.p, nlen = uint32_t(nl);
            an.p += nlen; an.n -= nlen;
            if (SIZE) { R.n_file_agents = ++n_file; continue; }
            if (n_file >= P.max_file_agents) return Defer;
            bool asc;
            if (!utf8_ok(C.in + noff, nlen, asc)) return InvalidUTF8;
            // get_or_create_agent_id: an existing name maps to its id
            uint32_t id = 0xFFFFFFFFu;
            for (uint32_t j0 = 0; j0 < n_agents && id == 0xFFFFFFFFu; j0 += 64) {
                const uint32_t j = j0 + lane();
                bool eq = false;
                if (j < n_agents && L.nlen[j] == nlen) {
                    eq = true;
                    const uint32_t o2 = L.noff[j];
                    for (uint32_t k = 0; k < nlen && eq; k++) eq = C.in[o2 + k] == C.in[noff + k];
                }
                const uint64_t m = ballot(eq);
                if (m) id = j0 + ctz(m);
            }
            if (id == 0xFFFFFFFFu) {
                bool root = nlen == 4 && C.byte(0, noff) == 'R' && C.byte(0, noff + 1) == 'O' &&
                            C.byte(0, noff + 2) == 'O' && C.byte(0, noff + 3) == 'T';
                if (root || nlen >= 50) return ErrCheckout;   // mod.rs:88-91
                id = n_agents++;
                if (lane() == 0) { L.noff[id] = noff; L.nlen[id] = nlen; }
            }
            if (lane() == 0) { L.fmap[n_file] = id; L.fseq[n_file] = 0; }
            n_file++;
            __syncthreads();
        }
    }
    R.n_file_agents = n_file;
    {   // StartBranch (decode_oplog.rs:652-664)
        Rd sb, ver;
        bool found;
        TRY(C.expect_chunk(r, 10, sb));
        TRY(C.chunk_if(sb, 12, found, ver));
        if (found) {   // read_version: any named version is unknown to a fresh oplog
            for (;;) {
                uint64_t n, seq;
                TRY(C.u64v(ver, n));
                TRY(C.u64v(ver, seq));
                if ((n >> 1) == 0) break;
                if ((n >> 1) - 1 >= n_file) return InvalidLength;
                if (!(SIZE && D.patch)) return BaseVersionUnknown;   // sizing a patch: resolved later
                if (!(n & 1)) break;
            }
            if (ver.n) return InvalidLength;
        }
        if (sb.n) {
            Rd s; uint32_t asc;
            TRY(content_str<SIZE>(C, sb, comp, has_comp, s, asc));
        }
    }
    Rd pc;
    TRY(C.expect_chunk(r, 20, pc));
    CRuns ins{}, del{};
    uint32_t cik_bytes = 0;
    for (;;) {
        bool found; Rd ch;
        TRY(C.chunk_if(pc, 24, found, ch));
        if (!found) break;
        uint64_t tag;
        TRY(C.u32v(ch, tag));
        if (tag > 1) return InvalidContent;
        CRuns it{};
        it.present = 1;
        TRY(content_str<SIZE>(C, ch, comp, has_comp, it.text, it.ascii));
        Rd runs;
        TRY(C.expect_chunk(ch, 25, runs));
        it.runs = vq_make(C.in, runs);
        it.t0 = it.text.p;
        cik_bytes += runs.n;
        if (tag == 0) ins = it; else del = it;
    }
    Rd av, tp, hist;
    TRY(C.expect_chunk(pc, 21, av));
    TRY(C.expect_chunk(pc, 22, tp));
    TRY(C.expect_chunk(pc, 23, hist));
    VQ qav = vq_make(C.in, av), qtp = vq_make(C.in, tp), qhist = vq_make(C.in, hist);
    uint32_t *vs = L.vq;
    prof_mark(1);

    if (SIZE) {   // OpVersions: LV count and agent runs
        uint64_t lv = 0;
        uint32_t runs = 0;
        R.tp_bytes = tp.n;
        R.cik_bytes = cik_bytes;
        R.hist_bytes = hist.n;
        while (qav.left()) {
            uint64_t n, alen;
            int64_t jump = 0;
            TRY(vq_pop(qav, n, vs));
            const bool hj = n & 1;
            TRY(vq_pop(qav, alen, vs));
            if (hj) TRY(vq_zigzag(qav, jump, vs));
            lv += alen;
            runs++;
            R.raw_aruns = runs;   // partial counts size a pass that fails later
            R.n_lv = lv;
            if (lv >= LIM31) return Defer;
        }
        R.raw_aruns = runs;
        R.n_lv = lv;
        prof_mark(2);
        return S_OK;
    }

    // ---- OpVersions + OpTypeAndPosition + content runs (decode_oplog.rs:29-68, 289-337, 731-778)
    Quads qa, qp;
    qa.init(); qp.init();
    uint32_t ca_valid = 0, ca_lv = 0, ca_len = 0, ca_agent = 0, ca_seq = 0;   // pending agent run
    uint32_t cr_valid = 0, cr_lv = 0, cr_len = 0, cr_pos = 0, cr_kind = 0, cr_fwd = 0;   // pending op run
    uint64_t n_lv = 0, next_assign = 0;
    uint32_t ins_size = 0, complete = 1, all_ascii = 1;
    int64_t last_cursor = 0;
    bool have_op = false;
    uint64_t op_len = 0;
    int64_t op_start = 0;
    bool op_del = false, op_fwd = true;

    auto flush_arun = [&]() -> int {
        if (!ca_valid) return S_OK;
        if (qa.count() >= D.arun_cap) return int(ErrCapacity);
        qa.push(ca_lv, ca_len, ca_agent, ca_seq, O.aruns);
        return S_OK;
    };
    auto flush_op = [&]() -> int {
        if (!cr_valid) return S_OK;
        if (qp.count() >= D.pre_cap) return int(ErrCapacity);
        qp.push(cr_lv, cr_len, cr_pos, cr_kind | (cr_fwd << 1), O.pre);
        return S_OK;
    };
    auto fill_cbyte = [&](uint64_t lv0, uint64_t k, uint32_t v) {
        for (uint64_t i = lane(); i < k; i += 64) O.cbyte[lv0 + i] = v;
    };

    uint32_t fill_jobs = 0;   // deferred fill jobs of a long document (fill_kernel)
    if (ins.present && !del.present) {
        const uint64_t t_runs = __builtin_amdgcn_s_memtime();
        // a non-ASCII text: with at most 64 continuation bytes the batched path writes byte offsets
        // through utf8_table; otherwise it numbers chars and utf8_offsets then places their bytes
        const uint8_t *txt = C.ptr(ins.text.s) + ins.text.p;
        Utf8Tab tab{0xFFFFFFFFu, 0u};
        uint32_t n_chars = ins.text.n;
        const bool tabled = !ins.ascii && ins.text.n && utf8_table(txt, ins.text.n, tab, n_chars);
        if (!ins.ascii && !tabled) {
            tab.n = 0;
            n_chars = count_char_starts(txt, ins.text.n);
        }
        uint32_t *jobs = nullptr;   // a long document defers its per-LV offsets to fill_kernel
        if (P.fill && D.fill_cap && (ins.ascii || tabled)) {
            uint32_t *hdr = P.fill + D.fill_off;
            hdr[1 + lane()] = tab.t;
            if (lane() == 0) hdr[0] = tab.n;
            jobs = hdr + FILL_HDR;
        }
        FastOut fo = fast_runs(qav, qtp, ins.runs, n_chars, n_file, L.fseq, L.fmap, vs, O.aruns, O.pre,
                               O.cbyte, O.alist, D.arun_cap, D.pre_cap, D.lv_cap, tab, jobs, D.fill_cap);
        if (fo.status == 0 && jobs) {
            fill_jobs = fo.n_jobs;
            if (lane() == 0) P.fill_n[doc] = fill_jobs;   // (bit 31 set with the text copy below)
        }
        if (fo.status == 0 && tabled) {   // the offsets are bytes already
            fo.ins_size = ins.text.n;
            all_ascii = 0;
        } else if (fo.status == 0 && !ins.ascii) {
            if (utf8_offsets(txt, ins.text.n, O.cbyte, fo.n_lv, n_chars)) {
                fo.ins_size = ins.text.n;   // bytes from here on
                all_ascii = 0;
            } else {
                fo.status = 1;
            }
        }
        if (fo.status == 0) {
#ifndef DT_LZPROF
            R.prof[7] += uint32_t(fo.t_mid - t_runs);   // the agent-assignment half of the fast path
#endif
            qa.at = fo.n_aruns;
            qp.at = fo.n_pre;
            n_lv = next_assign = fo.n_lv;
            ins_size = fo.ins_size;
            qav.at = qav.len;             // consumed
            ins.runs.at = ins.runs.len;   // the insert content is consumed exactly
            ins.text.p += ins.text.n;
            ins.text.n = 0;
        } else {                          // back to the exact path
            __syncthreads();
            for (uint32_t a = lane(); a < n_file; a += 64) L.fseq[a] = 0;
            __syncthreads();
        }
    }

    while (qav.left()) {
        uint64_t n, alen;
        int64_t jump = 0;
        TRY(vq_pop(qav, n, vs));
        const bool has_jump = n & 1;
        n >>= 1;
        TRY(vq_pop(qav, alen, vs));
        if (has_jump) TRY(vq_zigzag(qav, jump, vs));
        if (n == 0 || n - 1 >= n_file) return InvalidLength;
        const uint32_t fa = uint32_t(n - 1);
        const int64_t sstart = int64_t(L.fseq[fa]) + jump;
        if (sstart < 0 || uint64_t(sstart) + alen >= LIM31 || next_assign + alen >= LIM31) return Defer;
        __syncthreads();
        if (lane() == 0) L.fseq[fa] = uint32_t(sstart + int64_t(alen));
        __syncthreads();
        const uint32_t agent = L.fmap[fa];
        // assign (agent_runs RLE)
        if (ca_valid && ca_agent == agent && ca_lv + ca_len == next_assign && uint64_t(ca_seq) + ca_len == uint64_t(sstart)) {
            ca_len += uint32_t(alen);
        } else {
            TRY(flush_arun());
            ca_valid = 1; ca_lv = uint32_t(next_assign); ca_len = uint32_t(alen); ca_agent = agent; ca_seq = uint32_t(sstart);
        }
        next_assign += alen;

        uint64_t want = alen;
        while (want) {
            if (!have_op) {
                if (!qtp.left()) return InvalidLength;
                uint64_t x;
                TRY(vq_pop(qtp, x, vs));
                const bool has_length = x & 1; x >>= 1;
                const bool diff_nz = x & 1; x >>= 1;
                const bool is_del = x & 1; x >>= 1;
                int64_t diff = 0;
                bool fwd = true;
                uint64_t l;
                if (has_length) {
                    if (is_del) { fwd = x & 1; x >>= 1; }
                    if (diff_nz) TRY(vq_zigzag(qtp, diff, vs));
                    l = x;
                } else {
                    l = 1;
                    diff = int64_t(x >> 1) * ((x & 1) ? -1 : 1);
                }
                const int64_t raw = int64_t(uint64_t(last_cursor) + uint64_t(diff));
                int64_t st, raw_end;
                if (!is_del) { st = raw; raw_end = raw + int64_t(l); }
                else if (fwd) { st = raw; raw_end = raw; }
                else { st = raw - int64_t(l); raw_end = raw - int64_t(l); }
                last_cursor = raw_end;
                if (l == 0) return ErrCheckout;   // assert!(max_len > 0)
                op_len = l; op_start = st; op_del = is_del; op_fwd = fwd; have_op = true;
            }
            uint64_t take = want < op_len ? want : op_len;
            CRuns ci = op_del ? del : ins;   // by value: no dynamically indexed private memory
            bool known = false;
            Rd cs{0, 0, 0};
            if (ci.present) {
                bool has, cknown; uint64_t clen;
                TRY(cruns_next(C, ci, has, clen, cknown, cs, vs));
                if (!has) return InvalidLength;
                if (clen < take) take = clen;
                if (clen > take) {   // push the remainder back
                    uint32_t b = 0;
                    if (cknown) {
                        uint64_t c2;
                        walk_chars(C.ptr(cs.s) + cs.p, cs.n, take, ci.ascii, b, c2);
                    }
                    ci.pb = 1;
                    ci.pb_len = clen - take; ci.pb_known = cknown;
                    ci.pb_s = cknown ? Rd{cs.s, cs.p + b, cs.n - b} : Rd{cs.s, cs.p, 0};
                    cs.n = b;
                }
                known = cknown;
            }
            if (op_del) del = ci; else ins = ci;
            if (!take) return ErrCheckout;
            // the piece's position; out-of-range positions are left to the host decoder
            int64_t ppos;
            bool pfwd = true;
            if (!op_del) ppos = op_start;
            else if (op_fwd) ppos = op_start;
            else { ppos = op_start + int64_t(op_len) - int64_t(take); pfwd = false; }
            if (ppos < 0 || uint64_t(ppos) >= LIM31) return Defer;
            const uint32_t lv = uint32_t(n_lv);
            if (n_lv + take > D.lv_cap) return ErrCapacity;
            if (!op_del) {   // push_ins
                if (known) {
                    // the known pieces tile the insert text in order: the text is copied whole
                    // once at the end, pieces only place their per-LV offsets
                    const uint8_t *src = C.ptr(cs.s) + cs.p;
                    if (ci.ascii) {
                        for (uint64_t i = lane(); i < take; i += 64) O.cbyte[lv + i] = ins_size + uint32_t(i);
                    } else {
                        all_ascii = 0;
                        uint32_t cnt = 0;
                        for (uint32_t i = 0; i < cs.n; i += 64) {
                            const uint32_t j = i + lane();
                            const bool st = j < cs.n && (src[j] & 0xC0u) != 0x80u;
                            const uint64_t m = ballot(st);
                            if (st) O.cbyte[lv + cnt + popc(m & lt_mask())] = ins_size + j;
                            cnt += popc(m);
                        }
                    }
                    ins_size += cs.n;
                } else {
                    fill_cbyte(lv, take, 0xFFFFFFFFu);
                    complete = 0;
                }
                n_lv += take;
                if (cr_valid && cr_kind == 0 && cr_lv + cr_len == lv && uint64_t(cr_pos) + cr_len == uint64_t(ppos)) {
                    cr_len += uint32_t(take);
                } else {
                    TRY(flush_op());
                    cr_valid = 1; cr_lv = lv; cr_len = uint32_t(take); cr_pos = uint32_t(ppos); cr_kind = 0; cr_fwd = 1;
                }
                op_start += int64_t(take);
            } else {         // push_del
                fill_cbyte(lv, take, 0xFFFFFFFFu);
                n_lv += take;
                const uint32_t pos = uint32_t(ppos), ln = uint32_t(take);
                bool merged = false;
                if (cr_valid && cr_kind == 1 && cr_lv + cr_len == lv) {
                    if ((cr_len == 1 || cr_fwd) && (ln == 1 || pfwd) && pos == cr_pos) {
                        cr_len += ln; cr_fwd = 1; merged = true;
                    } else if ((cr_len == 1 || !cr_fwd) && (ln == 1 || !pfwd) && uint64_t(pos) + ln == cr_pos) {
                        cr_pos = pos; cr_len += ln; cr_fwd = 0; merged = true;
                    }
                }
                if (!merged) {
                    TRY(flush_op());
                    cr_valid = 1; cr_lv = lv; cr_len = ln; cr_pos = pos; cr_kind = 1; cr_fwd = pfwd ? 1 : 0;
                }
            }
            op_len -= take;
            if (!op_len) have_op = false;
            want -= take;
        }
    }
    if (n_lv != next_assign) return InvalidLength;
    TRY(flush_arun());
    TRY(flush_op());
    qa.flush(O.aruns);
    qp.flush(O.pre);
    const uint32_t n_aruns = uint32_t(qa.at), n_pre = uint32_t(qp.at);
    wave_fence();
    prof_mark(2);
    TRY(build_lookup(O, L, n_agents, n_aruns));
    prof_mark(3);

    // ---- OpParents (decode_oplog.rs:95-148, 856-913) -----------------------------------------
    uint64_t next_file = 0;
    uint32_t pe_valid = 0, pe_start = 0, pe_end = 0, pe_poff = 0;   // pending graph entry
    uint32_t n_ent = 0, n_par = 0;
    uint32_t fr = 0, fn = 0;   // frontier: lane k holds element k (sorted)
    while (qhist.left()) {
        if (qhist.head == qhist.cnt) vq_refill(qhist, vs);
        else if (qhist.cnt - qhist.head < 4 && qhist.wpos < qhist.len) vq_topup(qhist, vs);
        if (qhist.cnt - qhist.head >= 4) {   // next_assign < 2^31 (checked with the agent runs)
            uint32_t nf = uint32_t(next_file);
            if (batch_parents(qhist, nf, uint32_t(next_assign), pe_valid, pe_start, pe_end, pe_poff, n_ent, n_par,
                              fr, fn, D, O)) {
                next_file = nf;
                continue;
            }
        }
        uint64_t hl;
        TRY(vq_pop(qhist, hl, vs));
        uint32_t parv = 0, np = 0;
        bool par_bad = false;   // next_time - n underflowed (fails the range check below)
        for (;;) {
            uint64_t n;
            TRY(vq_pop(qhist, n, vs));
            const bool foreign = n & 1; n >>= 1;
            const bool more = n & 1; n >>= 1;
            uint64_t p;
            if (foreign) {
                if (n == 0) break;
                if (n - 1 >= n_file) return InvalidLength;
                uint64_t seq;
                TRY(vq_pop(qhist, seq, vs));
                const int64_t lv = lookup_lv(O, L, L.fmap[n - 1], seq);
                if (lv < 0) return InvalidLength;
                p = uint64_t(lv);
            } else {
                par_bad |= n > next_file;
                p = next_file - n;
            }
            if (np == DECODE_MAX_PARENTS) return Defer;
            parv = lane() == np ? uint32_t(p) : parv;
            np++;
            if (!more) break;
        }
        if (hl == 0 || next_file + hl > next_assign) return InvalidLength;
        if (par_bad || ballot(lane() < np && parv >= next_file)) return InvalidLength;
        // sort the parents: rank = smaller values + equal values at lower lanes
        uint32_t rank = 0;
        for (uint32_t j = 0; j < np; j++) {
            const uint32_t pj = rdl(parv, j);
            rank += (pj < parv || (pj == parv && j < lane())) ? 1u : 0u;
        }
        const uint32_t start = uint32_t(next_file), end = uint32_t(next_file + hl);
        if (np == 1 && pe_valid && rdl(parv, 0) == pe_end - 1 && pe_end == start) {   // Graph::push extends
            pe_end = end;
        } else {
            if (pe_valid) {
                if (n_ent >= D.ent_cap) return ErrCapacity;
                if (lane() == 0) { O.ent[n_ent] = make_uint2(pe_start, pe_end); O.poff[n_ent] = pe_poff; }
                n_ent++;
            }
            if (n_par + np > D.par_cap) return ErrCapacity;
            if (lane() < np) O.par[n_par + rank] = parv;
            pe_valid = 1; pe_start = start; pe_end = end; pe_poff = n_par;
            n_par += np;
        }
        // frontier advance (frontier.rs:251-279): drop the parents, append the span's last LV
        bool in_par = false;
        for (uint32_t j = 0; j < np; j++) in_par |= rdl(parv, j) == fr;
        const bool keep = lane() < fn && !in_par;
        const uint64_t km = ballot(keep);
        // compaction by a lane permute: kept lanes to the front in order, the others behind them
        const uint32_t nk = popc(km);
        const uint32_t to = keep ? popc(km & lt_mask()) : nk + popc(~km & lt_mask());
        const uint32_t moved = uint32_t(__builtin_amdgcn_ds_permute(int(to << 2), int(fr)));
        fn = nk;
        if (fn >= DECODE_MAX_FRONTIER) return Defer;
        fr = lane() < fn ? moved : 0u;
        fr = lane() == fn ? end - 1 : fr;
        fn++;
        next_file += hl;
    }
    if (next_file != next_assign) return InvalidLength;
    if (pe_valid) {
        if (n_ent >= D.ent_cap) return ErrCapacity;
        if (lane() == 0) { O.ent[n_ent] = make_uint2(pe_start, pe_end); O.poff[n_ent] = pe_poff; }
        n_ent++;
    }
    if (lane() == 0) O.poff[n_ent] = n_par;
    prof_mark(4);
    if (pc.n) return InvalidLength;
    if (ins.present) {   // the content iterators must be exhausted
        bool has, kn; uint64_t l; Rd s;
        const int e = cruns_next(C, ins, has, l, kn, s, vs);
        if (e || has) return InvalidContent;
    }
    if (del.present) {
        bool has, kn; uint64_t l; Rd s;
        const int e = cruns_next(C, del, has, l, kn, s, vs);
        if (e || has) return InvalidContent;
    }
    {   // CRC (decode_oplog.rs:940-955)
        const uint32_t reader_len = r.n;
        bool found; Rd c;
        TRY(C.chunk_if(r, 100, found, c));
        if (found && !D.ignore_crc) {
            if (c.n < 4) return UnexpectedEOF;
            const uint32_t want = C.byte(0, c.p) | (C.byte(0, c.p + 1) << 8) | (C.byte(0, c.p + 2) << 16) |
                                  (C.byte(0, c.p + 3) << 24);
            if (crc32c_par(C.in, len - reader_len, L.crc, P.x2n) != want) return ChecksumFailed;
        }
    }
    wave_fence();
    prof_mark(5);

    // ---- the insert text (every known piece, in order) ------------------------------------------
    if (ins.present && ins_size && P.fill && D.fill_cap) {   // a long document: fill_kernel copies it
        if (ins_size > D.content_cap) return ErrCapacity;
        uint32_t *hdr = P.fill + D.fill_off;
        if (lane() == 0) {
            hdr[65] = ins.text.s;
            hdr[66] = ins.t0;
            hdr[67] = ins_size;
            P.fill_n[doc] = fill_jobs | 0x80000000u;
        }
    } else if (ins.present && ins_size) {
        if (ins_size > D.content_cap) return ErrCapacity;
        const uint8_t *src = C.ptr(ins.text.s) + ins.t0;
        for (uint32_t i = 0; i < ins_size; i += 256) {
            uint8_t b[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t j = i + 64 * u + lane();
                b[u] = j < ins_size ? src[j] : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t j = i + 64 * u + lane();
                if (j < ins_size) O.content[j] = b[u];
            }
        }
    }

    // ---- split op runs at graph-entry boundaries (HostOpLog::finish) --------------------------
    // one run per lane: its first entry by bisection, its pieces (one per entry it touches) at a
    // prefix-sum offset; a run rarely spans entries, so the per-lane loops are short
    wave_fence();   // the entries were written by lane 0 above
    {
        uint32_t nout = 0, ebase = 0;   // ebase: the entry of the previous chunk's last run
        for (uint32_t b0 = 0; b0 < n_pre; b0 += 64) {
            const uint32_t i = b0 + lane();
            const bool live = i < n_pre;
            const uint4 q = live ? O.pre[i] : make_uint4(0, 0, 0, 0);
            // runs and entries are both in LV order, so a run's first entry is at or after ebase:
            // search the 64 entries from there in registers, HBM only past that window
            const uint32_t we = ebase + lane() < n_ent ? O.ent[ebase + lane()].y : 0xFFFFFFFFu;
            uint32_t c = 0;
#pragma unroll
            for (uint32_t st = 32; st >= 1; st >>= 1)
                if (uint32_t(__shfl(int(we), int(c + st - 1))) <= q.x) c += st;
            if (c == 63 && rdl(we, 63) <= q.x) c = 64;
            uint32_t lo = ebase + c, hi = live && c == 64 ? n_ent : lo;
            while (lo < hi) {
                const uint32_t m = (lo + hi) >> 1;
                if (O.ent[m].y <= q.x) lo = m + 1; else hi = m;
            }
            uint32_t npc = 0;
            if (live) {
                npc = 1;
                const uint32_t end = q.x + q.y;
                for (uint32_t e = lo; e < n_ent && O.ent[e].y < end; e++) npc++;
            }
            const uint32_t incl = scan_incl(npc);
            const uint32_t tot = rdl(incl, 63);
            if (uint64_t(nout) + tot > D.op_cap) return ErrCapacity;
            if (live) {
                uint32_t rlv = q.x, rlen = q.y, rpos = q.z, e = lo, k = nout + incl - npc;
                const uint32_t kf = q.w, kind = kf & 1u, fwd = kf >> 1;
                while (rlen) {
                    const uint32_t cut = e < n_ent ? O.ent[e].y : rlv + rlen;
                    const uint32_t mm = rlen < cut - rlv ? rlen : cut - rlv;
                    uint32_t apos = rpos;
                    if (kind == 0) rpos += mm;
                    else if (!fwd) apos = rpos + rlen - mm;
                    O.ops[k++] = make_uint4(rlv, mm, apos, kf);
                    rlv += mm;
                    rlen -= mm;
                    if (rlv >= cut) e++;
                }
            }
            nout += tot;
            ebase = rdl(lo, min(n_pre - 1 - b0, 63u));
        }
        R.n_ops = nout;
    }
    prof_mark(6);
    if (lane() < fn) O.ver[lane()] = fr;
    for (uint32_t a = lane(); a < n_agents; a += 64) O.agents[a] = make_uint2(L.noff[a], L.nlen[a]);

    R.n_agents = n_agents;
    R.n_aruns = n_aruns;
    R.n_pre = n_pre;
    R.n_entries = n_ent;
    R.n_parents = n_par;
    R.n_content = ins_size;
    R.n_version = fn;
    R.content_complete = complete;
    R.ascii = all_ascii;
    R.n_lv = n_lv;
    return S_OK;
}

// The LZ4 block of a document in P.lz_big, before decode_kernel: its header read as decode_doc
// reads it (anything unusual leaves the document to decode_kernel, which then reports it), the
// block decompressed by two waves (lz4_block<true>), the verdict in P.lz_pre.
constexpr uint32_t LZ_PRE_RING = 1024;
// waves per long block: 2 (parse | copy) or 3 (parse | copy even batches | copy odd batches)
template <int W>
constexpr size_t lz_pre_lds() {
    return W == 3 ? (2 * (256 + LZ_PRE_RING) + 4 * (5 * 64 + 4) + 4) * 4 : (256 + LZ_PRE_RING + 2 * (5 * 64 + 4)) * 4;
}
template <int DTGPU_LZ_WAVES>
__global__ __launch_bounds__(64 * DTGPU_LZ_WAVES) void lz4_kernel(DecodeParams P) {
    extern __shared__ uint32_t lds[];
    const uint32_t doc = P.lz_big[blockIdx.x];
    const DecodeDesc D = P.docs[doc];
    Ctx C;
    C.in = P.in + D.in_off;
    C.lz = P.lz + D.lz_off;
    C.w0 = Win{C.in, 0x80000000u, 0};
    C.w1 = Win{C.lz, 0x80000000u, 0};
    const uint32_t len = D.in_len;
    uint32_t verdict = 0;
    do {   // both waves read the header alike (wave-uniform), so they agree on what follows
        if (len < 8) break;
        bool bad = false;
        const char *magic = "DMNDTYPS";
        for (uint32_t i = 0; i < 8; i++)
            if (C.byte(0, i) != uint32_t(uint8_t(magic[i]))) bad = true;
        if (bad) break;
        Rd r{0, 8, len - 8};
        uint64_t pv;
        if (C.u64v(r, pv) || pv != 0) break;
        bool found;
        Rd c;
        if (C.chunk_if(r, 5, found, c) || !found) break;
        uint64_t ulen;
        if (C.u64v(c, ulen)) break;
        if (ulen > (uint64_t(1) << 34) || ulen > 255ull * c.n + 64 || ulen > D.lz_cap) break;
        if (DTGPU_LZ_WAVES == 3) {   // waves 1 and 2 each: start map (256) + ring; then the slots
            const bool ok = lz4_block<true, true>(C, c, C.lz, uint32_t(ulen), reinterpret_cast<uint4 *>(lds),
                                                  lds + 256, LZ_PRE_RING, nullptr, lds + 2 * (256 + LZ_PRE_RING));
            // a copier that gave up waiting leaves the block to decode_kernel (verdict 0)
            const volatile uint32_t *done = lds + 2 * (256 + LZ_PRE_RING) + 4 * (5 * 64 + 4);
            verdict = ok ? 1u : (done[1] | done[2]) ? 0u : 2u;
        } else {
            verdict = lz4_block<true>(C, c, C.lz, uint32_t(ulen), reinterpret_cast<uint4 *>(lds), lds + 256,
                                      LZ_PRE_RING, nullptr, lds + 256 + LZ_PRE_RING) ? 1u : 2u;
        }
    } while (false);
    if (threadIdx.x == 0) P.lz_pre[doc] = verdict;
}

// The per-LV content offsets that long documents deferred (fill_lvs on each job): one wave per
// job slot; slots past the document's job count (its fast path failed: 0) leave at once.
__global__ __launch_bounds__(64) void fill_kernel(DecodeParams P) {
    const uint32_t b = blockIdx.x;
    const uint32_t doc = P.fill_doc[b];
    const DecodeDesc D = P.docs[doc];
    const uint32_t j = b - D.fill_job0;
    const uint32_t fn = P.fill_n[doc];
    const uint32_t *hdr = P.fill + D.fill_off;
    if (j >= D.fill_cap) {   // 4 KB of the insert text (bit 31 of fill_n: decode_kernel left it here)
        if (!(fn >> 31)) return;
        const uint8_t *src = (hdr[65] == SRC_LZ ? P.lz + D.lz_off : P.in + D.in_off) + hdr[66];
        uint8_t *dst = P.content + D.content_off;
        const uint32_t n = hdr[67], k0 = (j - D.fill_cap) * 4096u;
        uint8_t v[16];
        for (uint32_t q = 0; q < 4; q++) {   // 16 loads in flight per lane, then their stores
#pragma unroll
            for (uint32_t u = 0; u < 16; u++) {
                const uint32_t i = k0 + 1024u * q + 64u * u + lane();
                v[u] = i < n ? src[i] : 0;
            }
#pragma unroll
            for (uint32_t u = 0; u < 16; u++) {
                const uint32_t i = k0 + 1024u * q + 64u * u + lane();
                if (i < n) dst[i] = v[u];
            }
        }
        return;
    }
    if (j >= (fn & 0x7FFFFFFFu)) return;
    const uint32_t *job = hdr + FILL_HDR + size_t(j) * FILL_JOB;
    Utf8Tab tab;
    tab.n = hdr[0];
    tab.t = hdr[1 + lane()];
    const uint32_t lincl = job[2 + lane()], vk = job[66 + lane()];
    const uint64_t dm = uint64_t(job[130]) | (uint64_t(job[131]) << 32);
    const uint32_t prev = uint32_t(__shfl_up(int(lincl), 1));
    const uint32_t L = lincl - (lane() ? prev : 0u);
    fill_lvs(P.cbyte + D.lv_off, job[0], job[1], lincl, L, vk, (dm >> lane()) & 1u, ballot(L > 0), tab);
}

template <bool SIZE>
#ifndef DTGPU_DECODE_WAVES
#define DTGPU_DECODE_WAVES 5   // occupancy target (tuning knob; the register budget follows from it):
                               // 5 (96 VGPRs) beat 6 (80, VGPR spills) once long documents moved work out (r6_w5)
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DTGPU_DECODE_WAVES))) void decode_kernel(DecodeParams P) {
    extern __shared__ uint32_t lds[];
    if (blockIdx.x >= P.n_docs) return;
    const uint32_t doc = !SIZE && P.order ? P.order[blockIdx.x] : blockIdx.x;   // longest documents first
    const DecodeDesc D = P.docs[doc];
    Lds L;
    const uint32_t F = P.max_file_agents;
    L.crc = lds;
    L.fr = lds + 256;
    L.vq = lds + 320;
    L.fmap = lds + 512;
    L.fseq = L.fmap + F;
    L.noff = L.fseq + F;
    L.nlen = L.noff + F;
    L.acnt = L.nlen + F;
    L.aoff = L.acnt + F;
    L.acur = L.aoff + F;
    L.amono = L.acur + F;
    L.lzr = L.amono + F;
    if (!SIZE) {
        for (uint32_t i = lane(); i < 256; i += 64) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ CRC_POLY : c >> 1;
            L.crc[i] = c;
        }
        __syncthreads();
    }
    DecodeResult R{};
    int st = S_OK;
    if (D.skip) st = Defer;
    else st = decode_doc<SIZE>(P, D, R, L, doc);
    R.status = uint32_t(st);
    if (lane() == 0) P.results[doc] = R;
}


// =============================================================================================
// decode_and_add (ListOpLog::decode_and_add_opts, decode_oplog.rs:476-583; decode_internal's
// overlap filter :670-913).  One wavefront per (resident oplog, patch) pair; the parse is the
// decoder's exact path (wave-uniform, varint queues), each step restating dt_host.cpp decode_into
// so the error order is the host's.  The resident arrays are copied to the merged arenas first
// (lane-parallel); agent runs, op runs, entries and the frontier then grow with the reference's
// RLE rules, so the merged arrays equal the host decode_and_add's element for element.
// =============================================================================================
constexpr uint64_t UNDERWATER = ~uint64_t(0) / 4;   // UNDERWATER_START (src/dtrange.rs:197)

struct Merged {              // this document's merged arenas
    uint8_t *in, *content;
    uint4 *aruns, *ops, *pre, *vm;
    uint2 *ent, *agents;
    uint32_t *poff, *par, *cbyte, *ver, *ffr;
};

// Frontier::advance_by_known_run (frontier.rs:251-279) on a lane-array frontier (lane k = element
// k, sorted): false where the reference asserts.
__device__ __forceinline__ int advance_known(uint32_t &fv, uint32_t &fn, uint32_t par, uint32_t np, uint32_t start,
                                             uint32_t end, uint32_t *scratch) {
    const uint32_t last = end - 1;
    if (np == 1 && fn == 1 && rdl(par, 0) == rdl(fv, 0)) { fv = lane() == 0 ? last : 0u; return S_OK; }
    if (np == fn && !ballot(lane() < fn && fv != par)) { fv = lane() == 0 ? last : 0u; fn = 1; return S_OK; }
    if (ballot(lane() < fn && fv == start)) return InvalidLength;
    bool in_par = false;
    for (uint32_t j = 0; j < np; j++) in_par |= rdl(par, j) == fv;
    const bool keep = lane() < fn && !in_par;
    const uint64_t km = ballot(keep);
    const uint32_t nk = popc(km);
    if (nk + 1 > DECODE_MAX_FRONTIER) return Defer;
    // kept elements in order, `last` at its upper bound
    const uint32_t below = popc(ballot(keep && fv <= last));
    const uint32_t to = keep ? popc(km & lt_mask()) + (fv <= last ? 0u : 1u) : 64u;
    if (keep) scratch[to] = fv;
    if (lane() == 0) scratch[below] = last;
    __syncthreads();
    fn = nk + 1;
    fv = lane() < fn ? scratch[lane()] : 0u;
    __syncthreads();
    return S_OK;
}

// ascending sort of lanes [0, n) of a lane array (rank = smaller values + equal values at lower lanes)
__device__ __forceinline__ uint32_t lane_sort(uint32_t v, uint32_t n, uint32_t *scratch) {
    uint32_t rank = 0;
    for (uint32_t j = 0; j < n; j++) {
        const uint32_t pj = rdl(v, j);
        rank += (pj < v || (pj == v && j < lane())) ? 1u : 0u;
    }
    if (lane() < n) scratch[rank] = v;
    __syncthreads();
    const uint32_t out = lane() < n ? scratch[lane()] : 0u;
    __syncthreads();
    return out;
}

__device__ __forceinline__ int add_doc(const AddParams &P, const AddDesc &D, DecodeResult &R, const Lds &L,
                                       const Merged &M) {
    Ctx C;
    C.in = M.in + D.p_rel;
    C.lz = P.lz + D.lz_off;
    C.w0 = Win{C.in, 0x80000000u, 0};
    C.w1 = Win{C.lz, 0x80000000u, 0};
    const uint32_t len = D.p_len;
    uint32_t *vs = L.vq;

    // ---- merged state (uniform), starting as the resident oplog -----------------------------
    uint32_t n_agents = D.b_n_agents, n_aruns = D.b_n_aruns, n_ent = D.b_n_ent, n_par = D.b_n_par;
    uint32_t n_content = D.b_n_content, complete = D.b_complete, all_ascii = D.b_ascii;
    uint64_t n_lv = D.b_n_lv;
    uint32_t vf = lane() < D.b_n_ver ? M.ver[lane()] : 0u, vn = D.b_n_ver;   // cg.version
    uint32_t la_lv = 0, la_len = 0, la_agent = 0xFFFFFFFFu, la_seq = 0;    // last agent run
    if (n_aruns) { const uint4 a = M.aruns[n_aruns - 1]; la_lv = a.x; la_len = a.y; la_agent = a.z; la_seq = a.w; }
    uint32_t last_end = n_ent ? M.ent[n_ent - 1].y : 0u;                 // last graph entry's end
    uint32_t cr_valid = 0, cr_lv = 0, cr_len = 0, cr_pos = 0, cr_kind = 0, cr_fwd = 0;   // pending op run
    if (D.b_n_ops) {
        const uint4 o = M.ops[D.b_n_ops - 1];
        cr_valid = 1; cr_lv = o.x; cr_len = o.y; cr_pos = o.z; cr_kind = o.w & 1u; cr_fwd = (o.w >> 1) & 1u;
    }
    uint32_t n_pre = 0, n_vm = 0;
    uint32_t vm_file = 0, vm_local = 0, vm_len = 0;   // last version-map run (file offset from new_op_start)
    bool dirty = false;   // lane-0 stores the next lane-parallel scan must see (fenced lazily)

    // AgentAssignment::local_to_agent_version's inverse over the merged agent runs (LV order =
    // each agent's insertion order): the first run holding seq; gap = the next run start above it
    // Per merged agent (LDS): the end of its seq ranges so far, whether its runs' seq ranges
    // increase along LV order (then a run holding seq is the only one), and its last hit.  An
    // agent whose runs increase answers a seq at or past its end without a scan (the overlap
    // filter's new pieces), and a known one usually from the 64 runs around its last hit.
    uint32_t *A_end = L.acnt, *A_mono = L.amono, *A_cur = L.acur;
    auto seq_find = [&](uint32_t a, uint64_t seq, uint64_t &lv, uint64_t &gap) -> bool {
        if (dirty) { wave_fence(); dirty = false; }
        gap = ~uint64_t(0);
        const bool mono = A_mono[a] != 0;
        if (mono) {
            if (seq >= A_end[a]) return false;
            const uint32_t c = A_cur[a], w0 = c >= 16 ? c - 16 : 0;
            const uint32_t k = w0 + lane();
            const uint4 r = k < n_aruns ? M.aruns[k] : make_uint4(0, 0, 0xFFFFFFFFu, 0);
            const uint64_t hm = ballot(r.z == a && r.y != 0 && seq >= r.w && seq < uint64_t(r.w) + r.y);
            if (hm) {
                const uint32_t l = ctz(hm);
                lv = uint64_t(rdl(r.x, l)) + (seq - rdl(r.w, l));
                gap = uint64_t(rdl(r.w, l)) + rdl(r.y, l);
                if (lane() == 0) A_cur[a] = w0 + l;
                return true;
            }
        }
        for (uint32_t k0 = 0; k0 < n_aruns; k0 += 64) {
            const uint32_t k = k0 + lane();
            const uint4 r = k < n_aruns ? M.aruns[k] : make_uint4(0, 0, 0xFFFFFFFFu, 0);
            const bool mine = r.z == a && r.y != 0;
            const uint64_t hm = ballot(mine && seq >= r.w && seq < uint64_t(r.w) + r.y);
            if (hm) {
                const uint32_t l = ctz(hm);
                lv = uint64_t(rdl(r.x, l)) + (seq - rdl(r.w, l));
                gap = uint64_t(rdl(r.w, l)) + rdl(r.y, l);   // the run's end (seq)
                if (mono && lane() == 0) A_cur[a] = k0 + l;
                return true;
            }
            uint64_t g = mine && r.w > seq ? uint64_t(r.w) : ~uint64_t(0);
            for (int d = 32; d >= 1; d >>= 1) {
                const uint64_t o = uint64_t(uint32_t(__shfl_xor(int(uint32_t(g)), d))) |
                                   (uint64_t(uint32_t(__shfl_xor(int(uint32_t(g >> 32)), d))) << 32);
                g = o < g ? o : g;
            }
            gap = g < gap ? g : gap;
        }
        return false;
    };
    auto seq_to_lv = [&](uint32_t a, uint64_t seq) -> int64_t {
        uint64_t lv, gap;
        return seq_find(a, seq, lv, gap) ? int64_t(lv) : -1;
    };
    // cg.assign (agent_runs RLE, agent_assignment/mod.rs)
    auto assign = [&](uint32_t agent, uint32_t seq, uint32_t lv, uint32_t ln) -> int {
        if (lane() == 0) {
            const uint32_t e = A_end[agent];
            if (seq < e) A_mono[agent] = 0;
            A_end[agent] = max(e, seq + ln);
        }
        if (n_aruns && la_agent == agent && la_lv + la_len == lv && la_seq + la_len == seq) {
            la_len += ln;
            if (lane() == 0) M.aruns[n_aruns - 1].y = la_len;
        } else {
            if (n_aruns >= D.c_arun) return int(ErrCapacity);
            if (lane() == 0) M.aruns[n_aruns] = make_uint4(lv, ln, agent, seq);
            n_aruns++;
            la_lv = lv; la_len = ln; la_agent = agent; la_seq = seq;
        }
        dirty = true;
        return S_OK;
    };
    auto vmap_push = [&](uint32_t file, uint32_t local, uint32_t ln) -> int {
        if (n_vm && vm_file + vm_len == file && vm_local + vm_len == local) {
            vm_len += ln;
            if (lane() == 0) M.vm[n_vm - 1].z = vm_len;
        } else {
            if (n_vm >= D.c_vm) return int(ErrCapacity);
            if (lane() == 0) M.vm[n_vm] = make_uint4(file, local, ln, 0);
            n_vm++;
            vm_file = file; vm_local = local; vm_len = ln;
        }
        dirty = true;
        return S_OK;
    };
    // find_packed_with_offset: the version-map run holding file offset f (per lane)
    auto vmap_find = [&](uint32_t f, uint32_t &local, uint32_t &rem) -> bool {
        uint32_t lo = 0, hi = n_vm;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (M.vm[mid].x <= f) lo = mid + 1; else hi = mid;
        }
        if (!lo) return false;
        const uint4 m = M.vm[lo - 1];
        if (f >= m.x + m.z) return false;
        local = m.y + (f - m.x);
        rem = m.z - (f - m.x);
        return true;
    };
    auto flush_op = [&]() -> int {
        if (!cr_valid) return S_OK;
        if (n_pre >= D.c_pre) return int(ErrCapacity);
        if (lane() == 0) M.pre[n_pre] = make_uint4(cr_lv, cr_len, cr_pos, cr_kind | (cr_fwd << 1));
        n_pre++;
        cr_valid = 0;
        return S_OK;
    };

    // the per-agent tables from the resident's runs: agents one round at a time per 64 runs
    // (runs of one agent in LV order), each run checked against the end of the agent's previous
    for (uint32_t a = lane(); a < D.c_agent; a += 64) { A_end[a] = 0; A_mono[a] = 1; A_cur[a] = 0; }
    __syncthreads();
    for (uint32_t k0 = 0; k0 < n_aruns; k0 += 64) {
        const uint32_t k = k0 + lane();
        const uint4 r = k < n_aruns ? M.aruns[k] : make_uint4(0, 0, 0xFFFFFFFFu, 0);
        const uint32_t end = r.w + r.y;
        bool todo = k < n_aruns && r.y != 0;
        while (ballot(todo)) {
            const uint32_t lead = rdl(todo ? r.z : 0xFFFFFFFFu, ctz(ballot(todo)));
            const bool mine = todo && r.z == lead;
            const uint64_t m = ballot(mine);
            const uint64_t below = m & lt_mask();
            const uint32_t src = below ? 63u - uint32_t(__clzll((long long)below)) : lane();
            const uint32_t prev_end = uint32_t(__shfl(int(end), int(src)));
            const uint32_t first_end = A_end[lead];
            const bool bad = mine && r.w < (below ? prev_end : first_end);
            const uint32_t last = 63u - uint32_t(__clzll((long long)m));
            const uint32_t last_end = rdl(end, last);
            const uint64_t anybad = ballot(bad);
            __syncthreads();
            if (lane() == 0) {
                if (anybad) A_mono[lead] = 0;
                A_end[lead] = max(first_end, last_end);   // increasing runs: the last ends highest
            }
            __syncthreads();
            if (mine) todo = false;
        }
    }
    __syncthreads();

    // ---- header, LZ4 --------------------------------------------------------------------------
    if (len < 8) return UnexpectedEOF;
    {
        const char *magic = "DMNDTYPS";
        for (uint32_t i = 0; i < 8; i++)
            if (C.byte(0, i) != uint32_t(uint8_t(magic[i]))) return InvalidMagic;
    }
    Rd r{0, 8, len - 8};
    uint64_t pv;
    TRY(C.u64v(r, pv));
    if (pv != 0) return UnsupportedProtocolVersion;
    Rd comp{SRC_LZ, 0, 0};
    bool has_comp = false;
    {
        bool found; Rd c;
        TRY(C.chunk_if(r, 5, found, c));
        if (found) {
            uint64_t ulen;
            TRY(C.u64v(c, ulen));
            if (ulen > (uint64_t(1) << 34)) return LZ4DecompressionError;
            if (ulen > 255ull * c.n + 64) return LZ4DecompressionError;
            if (ulen > D.lz_cap) return ErrCapacity;
            if (!lz4_block(C, c, C.lz, uint32_t(ulen), reinterpret_cast<uint4 *>(L.fr), nullptr, 0u)) return LZ4DecompressionError;
            comp.n = uint32_t(ulen);
            has_comp = true;
        }
    }

    // ---- FileInfo: doc id, agent names (get_or_create_agent_id on the merged agents) ----------
    uint32_t n_file = 0;
    uint32_t did_off = D.b_doc_id_off, did_len = D.b_doc_id_len;
    {
        Rd fi, an, tmp, did;
        bool found;
        TRY(C.expect_chunk(r, 1, fi));
        TRY(C.chunk_if(fi, 2, found, did));
        if (found) {
            uint64_t dt;
            TRY(C.u32v(did, dt));
            if (dt != 4) return UnknownChunk;
            bool asc;
            if (!utf8_ok(C.in + did.p, did.n, asc)) return InvalidUTF8;
        }
        const bool has_did = found;
        TRY(C.expect_chunk(fi, 3, an));
        TRY(C.chunk_if(fi, 4, found, tmp));
        while (an.n) {
            uint64_t nl;
            TRY(C.u64v(an, nl));
            if (nl > an.n) return InvalidLength;
            const uint32_t noff = an.p, nlen = uint32_t(nl);
            an.p += nlen; an.n -= nlen;
            bool asc;
            if (!utf8_ok(C.in + noff, nlen, asc)) return InvalidUTF8;
            if (n_file >= P.max_file_agents) return Defer;
            uint32_t id = 0xFFFFFFFFu;
            for (uint32_t j0 = 0; j0 < n_agents && id == 0xFFFFFFFFu; j0 += 64) {
                const uint32_t j = j0 + lane();
                bool eq = false;
                if (j < n_agents) {
                    const uint2 a = M.agents[j];
                    eq = a.y == nlen;
                    for (uint32_t k = 0; k < nlen && eq; k++) eq = M.in[a.x + k] == C.in[noff + k];
                }
                const uint64_t m = ballot(eq);
                if (m) id = j0 + ctz(m);
            }
            if (id == 0xFFFFFFFFu) {
                const bool root = nlen == 4 && C.byte(0, noff) == 'R' && C.byte(0, noff + 1) == 'O' &&
                                  C.byte(0, noff + 2) == 'O' && C.byte(0, noff + 3) == 'T';
                if (root || nlen >= 50) return ErrCheckout;   // mod.rs:88-91
                if (n_agents >= D.c_agent) return ErrCapacity;
                id = n_agents++;
                if (lane() == 0) M.agents[id] = make_uint2(D.p_rel + noff, nlen);
                wave_fence();
            }
            if (lane() == 0) { L.fmap[n_file] = id; L.fseq[n_file] = 0; }
            n_file++;
            __syncthreads();
        }
        if (has_did) {   // a doc id must match a non-empty oplog's (decode_oplog.rs:520-530)
            if (D.b_doc_id_len != 0xFFFFFFFFu && D.b_n_lv != 0) {
                bool same = D.b_doc_id_len == did.n;
                for (uint32_t i = lane(); same && i < did.n; i += 64)
                    same = M.in[D.b_doc_id_off + i] == C.in[did.p + i];
                if (ballot(D.b_doc_id_len == did.n && !same) || D.b_doc_id_len != did.n) return DocIdMismatch;
            }
            did_off = D.p_rel + did.p;
            did_len = did.n;
        }
    }
    R.doc_id_off = did_off;
    R.doc_id_len = did_len;

    // ---- StartBranch: the version the patch starts from, in merged LVs -------------------------
    uint32_t sv = 0, svn = 0;   // lane k: element k
    {
        Rd sb, ver;
        bool found;
        TRY(C.expect_chunk(r, 10, sb));
        TRY(C.chunk_if(sb, 12, found, ver));
        if (found) {
            for (;;) {
                uint64_t n, seq;
                TRY(C.u64v(ver, n));
                TRY(C.u64v(ver, seq));
                if ((n >> 1) == 0) break;
                if ((n >> 1) - 1 >= n_file) return InvalidLength;
                const int64_t lv = seq_to_lv(L.fmap[(n >> 1) - 1], seq);
                if (lv < 0) return BaseVersionUnknown;
                if (svn == DECODE_MAX_FRONTIER) return Defer;
                sv = lane() == svn ? uint32_t(lv) : sv;
                svn++;
                if (!(n & 1)) break;
            }
            if (ver.n) return InvalidLength;
            sv = lane_sort(sv, svn, L.fr);
        }
        if (sb.n) {
            Rd s; uint32_t asc;
            TRY(content_str<false>(C, sb, comp, has_comp, s, asc));
        }
    }
    Rd pc;
    TRY(C.expect_chunk(r, 20, pc));
    CRuns ins{}, del{};
    for (;;) {
        bool found; Rd ch;
        TRY(C.chunk_if(pc, 24, found, ch));
        if (!found) break;
        uint64_t tag;
        TRY(C.u32v(ch, tag));
        if (tag > 1) return InvalidContent;
        CRuns it{};
        it.present = 1;
        TRY(content_str<false>(C, ch, comp, has_comp, it.text, it.ascii));
        Rd runs;
        TRY(C.expect_chunk(ch, 25, runs));
        it.runs = vq_make(C.in, runs);
        it.t0 = it.text.p;
        if (tag == 0) ins = it; else del = it;
    }
    Rd av, tp, hist;
    TRY(C.expect_chunk(pc, 21, av));
    TRY(C.expect_chunk(pc, 22, tp));
    TRY(C.expect_chunk(pc, 23, hist));
    VQ qav = vq_make(C.in, av), qtp = vq_make(C.in, tp), qhist = vq_make(C.in, hist);

    // The file continues the resident version, or its operations are filtered against what the
    // oplog already has (patches_overlap, decode_oplog.rs:670; file times go underwater).
    const bool overlap = svn != vn || ballot(lane() < vn && sv != vf);
    const uint64_t first_new = n_lv;
    const uint64_t new_op_start = overlap ? UNDERWATER : first_new;
    uint64_t next_assign = first_new, next_file = new_op_start;

    // ---- OpVersions + OpTypeAndPosition + content runs (decode_oplog.rs:29-68, 731-850) -------
    int64_t last_cursor = 0;
    bool have_op = false;
    uint64_t op_len = 0;
    int64_t op_start = 0;
    bool op_del = false, op_fwd = true;
    while (qav.left()) {
        uint64_t n, alen;
        int64_t jump = 0;
        TRY(vq_pop(qav, n, vs));
        const bool has_jump = n & 1;
        n >>= 1;
        TRY(vq_pop(qav, alen, vs));
        if (has_jump) TRY(vq_zigzag(qav, jump, vs));
        if (n == 0 || n - 1 >= n_file) return InvalidLength;
        const uint32_t fa = uint32_t(n - 1);
        const uint32_t agent = L.fmap[fa];
        int64_t sstart = int64_t(L.fseq[fa]) + jump;
        const int64_t send = sstart + int64_t(alen);
        if (sstart < 0 || uint64_t(send) >= LIM31 || next_assign + alen >= LIM31) return Defer;
        __syncthreads();
        if (lane() == 0) L.fseq[fa] = uint32_t(send);
        __syncthreads();
        while (sstart < send) {
            uint64_t known_lv = 0, run_end = uint64_t(send);
            bool keep = true;
            if (overlap) {
                uint64_t gap;
                keep = !seq_find(agent, uint64_t(sstart), known_lv, gap);
                run_end = gap;
            }
            const uint64_t l = (uint64_t(send) < run_end ? uint64_t(send) : run_end) - uint64_t(sstart);
            const uint32_t frel = uint32_t(next_file - new_op_start);
            if (keep) {
                TRY(assign(agent, uint32_t(sstart), uint32_t(next_assign), uint32_t(l)));
                TRY(vmap_push(frel, uint32_t(next_assign), uint32_t(l)));
                next_assign += l;
            } else {   // already here: map the file's items onto the local ones
                TRY(vmap_push(frel, uint32_t(known_lv), uint32_t(l)));
            }
            next_file += l;
            sstart += int64_t(l);

            uint64_t want = l;   // parse_next_patches (decode_oplog.rs:731-778)
            while (want) {
                if (!have_op) {
                    if (!qtp.left()) return InvalidLength;
                    uint64_t x;
                    TRY(vq_pop(qtp, x, vs));
                    const bool has_length = x & 1; x >>= 1;
                    const bool diff_nz = x & 1; x >>= 1;
                    const bool is_del = x & 1; x >>= 1;
                    int64_t diff = 0;
                    bool fwd = true;
                    uint64_t ol;
                    if (has_length) {
                        if (is_del) { fwd = x & 1; x >>= 1; }
                        if (diff_nz) TRY(vq_zigzag(qtp, diff, vs));
                        ol = x;
                    } else {
                        ol = 1;
                        diff = int64_t(x >> 1) * ((x & 1) ? -1 : 1);
                    }
                    const int64_t raw = int64_t(uint64_t(last_cursor) + uint64_t(diff));
                    int64_t st, raw_end;
                    if (!is_del) { st = raw; raw_end = raw + int64_t(ol); }
                    else if (fwd) { st = raw; raw_end = raw; }
                    else { st = raw - int64_t(ol); raw_end = raw - int64_t(ol); }
                    last_cursor = raw_end;
                    if (ol == 0) return ErrCheckout;   // assert!(max_len > 0)
                    op_len = ol; op_start = st; op_del = is_del; op_fwd = fwd; have_op = true;
                }
                uint64_t take = want < op_len ? want : op_len;
                CRuns ci = op_del ? del : ins;
                bool known = false;
                Rd cs{0, 0, 0};
                if (ci.present) {
                    bool has, cknown; uint64_t clen;
                    TRY(cruns_next(C, ci, has, clen, cknown, cs, vs));
                    if (!has) return InvalidLength;
                    if (clen < take) take = clen;
                    if (clen > take) {   // push the remainder back (SplitableSpan truncate)
                        uint32_t b = 0;
                        if (cknown) {
                            uint64_t c2;
                            walk_chars(C.ptr(cs.s) + cs.p, cs.n, take, ci.ascii, b, c2);
                        }
                        ci.pb = 1;
                        ci.pb_len = clen - take; ci.pb_known = cknown;
                        ci.pb_s = cknown ? Rd{cs.s, cs.p + b, cs.n - b} : Rd{cs.s, cs.p, 0};
                        cs.n = b;
                    }
                    known = cknown;
                }
                if (op_del) del = ci; else ins = ci;
                if (!take) return ErrCheckout;
                if (keep) {
                    int64_t ppos;
                    bool pfwd = true;
                    if (!op_del) ppos = op_start;
                    else if (op_fwd) ppos = op_start;
                    else { ppos = op_start + int64_t(op_len) - int64_t(take); pfwd = false; }
                    if (ppos < 0 || uint64_t(ppos) >= LIM31) return Defer;
                    const uint32_t lv = uint32_t(n_lv);
                    if (n_lv + take > D.c_lv) return ErrCapacity;
                    if (!op_del) {   // push_ins
                        if (known) {
                            if (n_content + cs.n > D.c_content) return ErrCapacity;
                            const uint8_t *src = C.ptr(cs.s) + cs.p;
                            // a catch-up patch keeps every piece: the known pieces tile the insert
                            // text in order, copied whole at the end
                            if (overlap)
                                for (uint32_t i = lane(); i < cs.n; i += 64) M.content[n_content + i] = src[i];
                            if (ci.ascii) {
                                for (uint64_t i = lane(); i < take; i += 64) M.cbyte[lv + i] = n_content + uint32_t(i);
                            } else {
                                all_ascii = 0;
                                uint32_t cnt = 0;
                                for (uint32_t i = 0; i < cs.n; i += 64) {
                                    const uint32_t j = i + lane();
                                    const bool s0 = j < cs.n && (src[j] & 0xC0u) != 0x80u;
                                    const uint64_t m = ballot(s0);
                                    if (s0) M.cbyte[lv + cnt + popc(m & lt_mask())] = n_content + j;
                                    cnt += popc(m);
                                }
                            }
                            n_content += cs.n;
                        } else {
                            for (uint64_t i = lane(); i < take; i += 64) M.cbyte[lv + i] = 0xFFFFFFFFu;
                            complete = 0;
                        }
                        n_lv += take;
                        if (cr_valid && cr_kind == 0 && cr_lv + cr_len == lv && uint64_t(cr_pos) + cr_len == uint64_t(ppos)) {
                            cr_len += uint32_t(take);
                        } else {
                            TRY(flush_op());
                            cr_valid = 1; cr_lv = lv; cr_len = uint32_t(take); cr_pos = uint32_t(ppos); cr_kind = 0; cr_fwd = 1;
                        }
                    } else {         // push_del
                        for (uint64_t i = lane(); i < take; i += 64) M.cbyte[lv + i] = 0xFFFFFFFFu;
                        n_lv += take;
                        const uint32_t pos = uint32_t(ppos), ln = uint32_t(take);
                        bool merged = false;
                        if (cr_valid && cr_kind == 1 && cr_lv + cr_len == lv) {
                            if ((cr_len == 1 || cr_fwd) && (ln == 1 || pfwd) && pos == cr_pos) {
                                cr_len += ln; cr_fwd = 1; merged = true;
                            } else if ((cr_len == 1 || !cr_fwd) && (ln == 1 || !pfwd) && uint64_t(pos) + ln == cr_pos) {
                                cr_pos = pos; cr_len += ln; cr_fwd = 0; merged = true;
                            }
                        }
                        if (!merged) {
                            TRY(flush_op());
                            cr_valid = 1; cr_lv = lv; cr_len = ln; cr_pos = pos; cr_kind = 1; cr_fwd = pfwd ? 1 : 0;
                        }
                    }
                }
                if (!op_del) op_start += int64_t(take);
                op_len -= take;
                if (!op_len) have_op = false;
                want -= take;
            }
        }
    }
    if (n_lv != next_assign) return InvalidLength;
    TRY(flush_op());
    const uint64_t file_end = next_file;
    if (!overlap && n_content > D.b_n_content) {
        const uint8_t *src = C.ptr(ins.text.s) + ins.t0;
        for (uint32_t i = lane(); i < n_content - D.b_n_content; i += 64) M.content[D.b_n_content + i] = src[i];
    }
    wave_fence();   // the agent runs and the version map, read lane-parallel from here on
    dirty = false;

    // ---- OpParents (decode_oplog.rs:95-148, 856-913) -----------------------------------------
    next_file = new_op_start;
    uint64_t next_hist = first_new;
    uint32_t ff = sv, ffn = svn;   // the file's version, advanced run by run
    while (qhist.left()) {
        uint64_t hl;
        TRY(vq_pop(qhist, hl, vs));
        uint64_t pv64 = 0;   // lane k: parent k (a merged LV, or a file time >= UNDERWATER)
        uint32_t np = 0;
        bool under = false;  // next_time - n below zero (fails the range check)
        for (;;) {
            uint64_t n;
            TRY(vq_pop(qhist, n, vs));
            const bool foreign = n & 1; n >>= 1;
            const bool more = n & 1; n >>= 1;
            uint64_t p;
            if (foreign) {
                if (n == 0) break;
                if (n - 1 >= n_file) return InvalidLength;
                uint64_t seq;
                TRY(vq_pop(qhist, seq, vs));
                const int64_t lv = seq_to_lv(L.fmap[n - 1], seq);
                if (lv < 0) return InvalidLength;
                p = uint64_t(lv);
            } else {
                if (overlap && n > next_file - new_op_start) return InvalidLength;   // would surface from underwater
                under |= n > next_file;
                p = next_file - n;
            }
            if (np == DECODE_MAX_PARENTS) return Defer;
            pv64 = lane() == np ? p : pv64;
            np++;
            if (!more) break;
        }
        if (hl == 0 || next_file + hl > file_end) return InvalidLength;
        if (under || ballot(lane() < np && pv64 >= next_file)) return InvalidLength;
        // history_entry_map_and_truncate (decode_oplog.rs:241-269), one mapped piece at a time
        uint64_t es = next_file;
        const uint64_t ee = next_file + hl;
        next_file = ee;
        for (;;) {
            uint32_t ms, mrem;
            if (!vmap_find(uint32_t(es - new_op_start), ms, mrem)) return InvalidLength;
            const uint32_t take = uint32_t(ee - es < uint64_t(mrem) ? ee - es : uint64_t(mrem));
            uint32_t me = ms + take;
            uint32_t mp = 0;
            bool bad = false;
            if (lane() < np) {
                if (pv64 >= UNDERWATER) {
                    uint32_t loc, rem;
                    if (vmap_find(uint32_t(pv64 - new_op_start), loc, rem)) mp = loc; else bad = true;
                } else {
                    mp = uint32_t(pv64);
                }
            }
            if (ballot(bad)) return InvalidLength;
            mp = lane_sort(mp, np, L.fr);
            TRY(advance_known(ff, ffn, mp, np, ms, me, L.fr));
            if (me > next_hist) {   // new here: graph.push + cg.version.advance_by_known_run
                uint32_t mpn = np;
                if (ms > next_hist) return InvalidLength;   // assert!(mapped.span.start <= next_history_time)
                if (ms < next_hist) { mp = lane() == 0 ? uint32_t(next_hist - 1) : 0u; mpn = 1; ms = uint32_t(next_hist); }
                if (ballot(lane() < mpn && mp >= ms)) return InvalidLength;
                if (mpn == 1 && n_ent && rdl(mp, 0) == last_end - 1 && last_end == ms) {   // Graph::push extends
                    last_end = me;
                    if (lane() == 0) M.ent[n_ent - 1].y = me;
                } else {
                    if (n_ent >= D.c_ent || n_par + mpn > D.c_par) return ErrCapacity;
                    if (lane() == 0) { M.ent[n_ent] = make_uint2(ms, me); M.poff[n_ent] = n_par; }
                    if (lane() < mpn) M.par[n_par + lane()] = mp;
                    n_ent++;
                    n_par += mpn;
                    last_end = me;
                }
                TRY(advance_known(vf, vn, mp, mpn, ms, me, L.fr));
                next_hist = me;
            }
            es += take;
            if (es == ee) break;
            pv64 = lane() == 0 ? es - 1 : 0;   // GraphEntrySimple::trim: the remainder's parent, unmapped
            np = 1;
        }
    }
    if (next_file != file_end || next_hist != next_assign) return InvalidLength;
    if (pc.n) return InvalidLength;
    if (ins.present) {
        bool has, kn; uint64_t l; Rd s;
        const int e = cruns_next(C, ins, has, l, kn, s, vs);
        if (e || has) return InvalidContent;
    }
    if (del.present) {
        bool has, kn; uint64_t l; Rd s;
        const int e = cruns_next(C, del, has, l, kn, s, vs);
        if (e || has) return InvalidContent;
    }
    {   // CRC (decode_oplog.rs:940-955)
        const uint32_t reader_len = r.n;
        bool found; Rd c;
        TRY(C.chunk_if(r, 100, found, c));
        if (found && !D.ignore_crc) {
            if (c.n < 4) return UnexpectedEOF;
            const uint32_t want = C.byte(0, c.p) | (C.byte(0, c.p + 1) << 8) | (C.byte(0, c.p + 2) << 16) |
                                  (C.byte(0, c.p + 3) << 24);
            if (crc32c_par(C.in, len - reader_len, L.crc, P.x2n) != want) return ChecksumFailed;
        }
    }
    wave_fence();

    // ---- HostOpLog::finish: the new op runs (and the resident's last) split at entry ends ------
    {
        const uint32_t o0 = D.b_n_ops ? D.b_n_ops - 1 : 0;
        uint32_t nout = o0;
        for (uint32_t b0 = 0; b0 < n_pre; b0 += 64) {
            const uint32_t i = b0 + lane();
            const bool live = i < n_pre;
            const uint4 q = live ? M.pre[i] : make_uint4(0, 0, 0, 0);
            uint32_t lo = 0, hi = live ? n_ent : 0;   // first entry ending above the run's first LV
            while (lo < hi) {
                const uint32_t m = (lo + hi) >> 1;
                if (M.ent[m].y <= q.x) lo = m + 1; else hi = m;
            }
            uint32_t npc = 0;
            if (live) {
                npc = 1;
                const uint32_t end = q.x + q.y;
                for (uint32_t e = lo; e < n_ent && M.ent[e].y < end; e++) npc++;
            }
            const uint32_t incl = scan_incl(npc);
            const uint32_t tot = rdl(incl, 63);
            if (uint64_t(nout) + tot > D.c_op) return ErrCapacity;
            if (live) {
                uint32_t rlv = q.x, rlen = q.y, rpos = q.z, e = lo, k = nout + incl - npc;
                const uint32_t kf = q.w, kind = kf & 1u, fwd = kf >> 1;
                while (rlen) {
                    const uint32_t cut = e < n_ent ? M.ent[e].y : rlv + rlen;
                    const uint32_t mm = rlen < cut - rlv ? rlen : cut - rlv;
                    uint32_t apos = rpos;
                    if (kind == 0) rpos += mm;
                    else if (!fwd) apos = rpos + rlen - mm;
                    M.ops[k++] = make_uint4(rlv, mm, apos, kf);
                    rlv += mm;
                    rlen -= mm;
                    if (rlv >= cut) e++;
                }
            }
            nout += tot;
        }
        R.n_ops = n_pre ? nout : D.b_n_ops;
    }
    if (lane() == 0) M.poff[n_ent] = n_par;
    if (lane() < vn) M.ver[lane()] = vf;
    if (lane() < ffn) M.ffr[lane()] = ff;
    R.n_agents = n_agents;
    R.n_aruns = n_aruns;
    R.n_entries = n_ent;
    R.n_parents = n_par;
    R.n_content = n_content;
    R.n_version = vn;
    R.n_file_frontier = ffn;
    R.content_complete = complete;
    R.ascii = all_ascii;
    R.n_lv = n_lv;
    R.n_file_agents = n_file;
    return S_OK;
}

// copies of the resident arrays (lane-parallel), and their restoration after an error
__device__ __forceinline__ void add_copy_base(const AddParams &P, const AddDesc &D, const Merged &M) {
    {   // the resident's bytes (agent names, doc id), then the patch after them
        const uint4 *s = reinterpret_cast<const uint4 *>(P.b_in + D.b_in);
        uint4 *d = reinterpret_cast<uint4 *>(M.in);
        for (uint32_t i = lane(); i < (D.b_in_len + 15) / 16; i += 64) d[i] = s[i];
        const uint4 *ps = reinterpret_cast<const uint4 *>(P.p_in + D.p_off);
        uint4 *pd = reinterpret_cast<uint4 *>(M.in + D.p_rel);
        for (uint32_t i = lane(); i < (D.p_len + 15) / 16; i += 64) pd[i] = ps[i];
    }
    const uint4 *ba = reinterpret_cast<const uint4 *>(P.b_aruns) + D.b_arun;
    for (uint32_t i = lane(); i < D.b_n_aruns; i += 64) M.aruns[i] = ba[i];
    const uint4 *bo = reinterpret_cast<const uint4 *>(P.b_ops) + D.b_op;
    for (uint32_t i = lane(); i < D.b_n_ops; i += 64) M.ops[i] = bo[i];
    const uint2 *be = reinterpret_cast<const uint2 *>(P.b_ent) + D.b_ent;
    for (uint32_t i = lane(); i < D.b_n_ent; i += 64) M.ent[i] = be[i];
    for (uint32_t i = lane(); i <= D.b_n_ent; i += 64) M.poff[i] = P.b_poff[D.b_poff + i];
    for (uint32_t i = lane(); i < D.b_n_par; i += 64) M.par[i] = P.b_par[D.b_par + i];
    for (uint32_t i = lane(); i < D.b_n_content; i += 64) M.content[i] = P.b_content[D.b_content + i];
    for (uint32_t i = lane(); i < D.b_n_lv; i += 64) M.cbyte[i] = P.b_cbyte[D.b_lv + i];
    const uint2 *bg = reinterpret_cast<const uint2 *>(P.b_agents) + D.b_agent;
    for (uint32_t i = lane(); i < D.b_n_agents; i += 64) M.agents[i] = bg[i];
    if (lane() < D.b_n_ver) M.ver[lane()] = P.b_ver[D.b_ver + lane()];
    wave_fence();
}

#ifndef DTGPU_ADD_WAVES
#define DTGPU_ADD_WAVES 2   // 231 VGPRs, no VGPR spills (4: 218 spilled, 1.5x slower)
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DTGPU_ADD_WAVES))) void decode_add_kernel(AddParams P) {
    extern __shared__ uint32_t lds[];
    const uint32_t doc = blockIdx.x;
    if (doc >= P.n_docs) return;
    const AddDesc D = P.docs[doc];
    Lds L{};
    const uint32_t F = P.max_file_agents;
    L.crc = lds;
    L.fr = lds + 256;
    L.vq = lds + 320;
    L.fmap = lds + 512;
    L.fseq = L.fmap + F;
    L.acnt = L.fseq + F;            // per merged agent: seq end,
    L.amono = L.acnt + P.max_agents;   // runs increase,
    L.acur = L.amono + P.max_agents;   // last hit
    for (uint32_t i = lane(); i < 256; i += 64) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ CRC_POLY : c >> 1;
        L.crc[i] = c;
    }
    __syncthreads();
    Merged M;
    M.in = P.m_in + D.m_in;
    M.content = P.m_content + D.m_content;
    M.aruns = reinterpret_cast<uint4 *>(P.m_aruns) + D.m_arun;
    M.ops = reinterpret_cast<uint4 *>(P.m_ops) + D.m_op;
    M.pre = reinterpret_cast<uint4 *>(P.scr) + D.m_scr;
    M.vm = M.pre + D.c_pre;
    M.ent = reinterpret_cast<uint2 *>(P.m_ent) + D.m_ent;
    M.agents = reinterpret_cast<uint2 *>(P.m_agents) + D.m_agent;
    M.poff = P.m_poff + D.m_poff;
    M.par = P.m_par + D.m_par;
    M.cbyte = P.m_cbyte + D.m_lv;
    M.ver = P.m_ver + D.m_ver;
    M.ffr = P.m_ffr + D.m_ver;
    DecodeResult R{};
    int st = Defer;
    add_copy_base(P, D, M);   // (a resident document that failed its own decode has no arrays)
    if (!D.skip) st = add_doc(P, D, R, L, M);
    if (st != S_OK) {   // the unwind: the merged document is the resident one
        const uint4 *ba = reinterpret_cast<const uint4 *>(P.b_aruns) + D.b_arun;
        const uint2 *be = reinterpret_cast<const uint2 *>(P.b_ent) + D.b_ent;
        if (lane() == 0 && D.b_n_aruns) M.aruns[D.b_n_aruns - 1] = ba[D.b_n_aruns - 1];
        if (lane() == 0 && D.b_n_ent) M.ent[D.b_n_ent - 1] = be[D.b_n_ent - 1];
        if (lane() == 0) M.poff[D.b_n_ent] = D.b_n_par;
        if (lane() < D.b_n_ver) M.ver[lane()] = P.b_ver[D.b_ver + lane()];
        R = DecodeResult{};
        R.n_agents = D.b_n_agents; R.n_aruns = D.b_n_aruns; R.n_ops = D.b_n_ops; R.n_entries = D.b_n_ent;
        R.n_parents = D.b_n_par; R.n_content = D.b_n_content; R.n_version = D.b_n_ver; R.n_lv = D.b_n_lv;
        R.content_complete = D.b_complete; R.ascii = D.b_ascii;
        R.doc_id_off = D.b_doc_id_off; R.doc_id_len = D.b_doc_id_len;
    }
    R.status = uint32_t(st);
    if (lane() == 0) P.results[doc] = R;
}

}  // namespace ddec

int launch_decode(const DecodeParams &p, void *stream) {
    if (!p.n_docs) return 0;
    const size_t lds = (512 + 8 * size_t(p.max_file_agents) + (p.size_only ? 0u : p.lz_ring)) * 4;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (!p.size_only && p.n_big)
    {   // three waves while the long blocks are not too many (P.lz3_max; the mixed batch's 300:
        // node_nodecc 13.6 -> 13.0 ms), two past that (git-makefile x 10,000: 47 vs 56 ms)
        if (p.n_big <= p.lz3_max)
            hipLaunchKernelGGL(ddec::lz4_kernel<3>, dim3(p.n_big), dim3(192), ddec::lz_pre_lds<3>(), s, p);
        else
            hipLaunchKernelGGL(ddec::lz4_kernel<2>, dim3(p.n_big), dim3(128), ddec::lz_pre_lds<2>(), s, p);
    }
    if (!p.size_only && p.fill_blocks && hipMemsetAsync(p.fill_n, 0, size_t(p.n_docs) * 4, s) != hipSuccess) return 66;
    if (p.size_only)
        hipLaunchKernelGGL(ddec::decode_kernel<true>, dim3(p.n_docs), dim3(64), lds, s, p);
    else
        hipLaunchKernelGGL(ddec::decode_kernel<false>, dim3(p.n_docs), dim3(64), lds, s, p);
    if (!p.size_only && p.fill_blocks)
        hipLaunchKernelGGL(ddec::fill_kernel, dim3(p.fill_blocks), dim3(64), 0, s, p);
    return launch_error() == hipSuccess ? 0 : 66;
}

int launch_decode_add(const AddParams &p, void *stream) {
    if (!p.n_docs) return 0;
    const size_t lds = (512 + 2 * size_t(p.max_file_agents) + 3 * size_t(p.max_agents)) * 4;
    if (lds > 160 * 1024) return 65;   // ErrCapacity: more agents than the LDS tables hold
    if (lds > 64 * 1024 &&
        hipFuncSetAttribute(reinterpret_cast<const void *>(&ddec::decode_add_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
        return 66;
    hipLaunchKernelGGL(ddec::decode_add_kernel, dim3(p.n_docs), dim3(64), lds, reinterpret_cast<hipStream_t>(stream), p);
    return launch_error() == hipSuccess ? 0 : 66;
}

}  // namespace dtgpu
