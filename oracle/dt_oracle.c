/*
 * dt_oracle.c -- CPU restatement of diamond-types' `ListOpLog::load_from` + `checkout_tip`
 * hot path.  TEST INFRASTRUCTURE ONLY: this file is the parity checker for the MI355X engine
 * (libdtgpu).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * it.  The product never links or calls it.
 *
 * Parity is pinned by the reference's own fixtures (tests/golden/): friendsforever.dt vs
 * friendsforever_flat.json.gz endContent, the five JSON traces' endContent, the
 * compat_simple_doc / compat_empty_doc byte vectors (src/list/encoding/tests.rs:374-424),
 * test_data/causal_graph/{diff,conflicting,version_contains}.json and the merge KATs of
 * src/listmerge/merge.rs:1109-1325.
 *
 * Restated from (all paths under /root/reference):
 *   varint / zigzag ............ src/list/encoding/leb.rs:113-178, 305-323
 *   chunk reader ............... src/list/encoding/decode_tools.rs:28-268
 *   .dt decode ................. src/list/encoding/decode_oplog.rs:29-337, 383-425, 590-960
 *   CRC-32C .................... src/encoding/tools.rs:111-115 (crc 3.0, CRC_32_ISCSI)
 *   LZ4 raw block .............. lz4_flex 0.10 `decompress` (published LZ4 block format)
 *   graph push / shadow ........ src/causalgraph/graph/mod.rs:85-128
 *   diff / conflicts / contains  src/causalgraph/graph/tools.rs:52-484
 *   frontier advance ........... src/frontier.rs:251-279
 *   spanning tree walk ......... src/listmerge/txn_trace.rs:114-333
 *   tracker semantics .......... src/listmerge/merge.rs:154-558, advance_retreat.rs:58-153,
 *                                yjsspan.rs:13-228 (per-item formulation)
 *   text materialisation ....... src/list/merge.rs:63-95
 *
 * The tracker is the checkout-from-ROOT per-item formulation (every LV replayed by the
 * spanning-tree walk, as `ListOpLog::dbg_items` does, src/listmerge/to_old.rs:171-191).  The
 * document-order list is an implicit treap (order statistics by total and by visible count) --
 * deliberately a different data structure from the GPU engine's blocked arrays.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>

#define EXPORT __attribute__((visibility("default")))

/* ParseError (src/encoding/parseerror.rs:14-48), numbered in declaration order from 1. */
enum {
    E_OK = 0, E_InvalidMagic, E_UnsupportedProtocolVersion, E_DocIdMismatch, E_BaseVersionUnknown,
    E_UnknownChunk, E_LZ4DecoderNeeded, E_LZ4DecompressionError, E_CompressedDataMissing,
    E_InvalidChunkHeader, E_MissingChunk, E_InvalidLength, E_UnexpectedEOF, E_InvalidUTF8,
    E_InvalidRemoteID, E_InvalidVarInt, E_InvalidContent, E_GenericInvalidData, E_ChecksumFailed,
    E_DataMissing,
    E_CheckoutPanic = 64,   /* the reference panics (merge.rs:384/489, yjsspan.rs:49-90) */
};

typedef int64_t i64;
typedef uint64_t u64;
typedef uint32_t u32;
typedef uint8_t u8;

#define ROOT_LV (-1)

/* ------------------------------------------------------------------------------------------ */
/* small growable vectors                                                                      */
/* ------------------------------------------------------------------------------------------ */
#define VEC(T) struct { T *v; i64 n, cap; }
#define VPUSH(vec, x) do { if ((vec).n == (vec).cap) { (vec).cap = (vec).cap ? (vec).cap * 2 : 16; \
    (vec).v = realloc((vec).v, sizeof(*(vec).v) * (size_t)(vec).cap); } (vec).v[(vec).n++] = (x); } while (0)
#define VFREE(vec) do { free((vec).v); (vec).v = NULL; (vec).n = (vec).cap = 0; } while (0)

typedef struct { i64 start, end; } Range;
typedef VEC(i64) VecI64;
typedef VEC(Range) VecRange;

/* ------------------------------------------------------------------------------------------ */
/* byte reader: leb.rs:113-178, decode_tools.rs:10-160                                          */
/* ------------------------------------------------------------------------------------------ */
typedef struct { const u8 *p; size_t n; } Buf;

static int leb_decode(const u8 *buf, size_t n, u64 *out, size_t *used) {
    u64 r = 0;
    for (size_t i = 0; i < n; i++) {
        if (i == 10) return E_InvalidVarInt;
        u8 b = buf[i];
        if (i == 9 && (b & 0x7f) > 1) return E_InvalidVarInt;
        r |= ((u64)(b & 0x7f)) << (i * 7);
        if (b < 0x80) { *out = r; *used = i + 1; return E_OK; }
    }
    return n >= 10 ? E_InvalidVarInt : E_UnexpectedEOF;
}
static int rd_usize(Buf *b, u64 *out) {
    if (b->n == 0) return E_UnexpectedEOF;
    size_t used; int e = leb_decode(b->p, b->n, out, &used);
    if (e) return e;
    b->p += used; b->n -= used; return E_OK;
}
static int rd_u32(Buf *b, u64 *out) {
    int e = rd_usize(b, out);
    if (e) return e;
    if (*out >= 0xFFFFFFFFull) return E_InvalidVarInt;   /* decode_leb_u32: val >= u32::MAX */
    return E_OK;
}
static int peek_u32(const Buf *b, int *has, u64 *out) {
    if (b->n == 0) { *has = 0; return E_OK; }
    size_t used; int e = leb_decode(b->p, b->n, out, &used);
    if (e) return e;
    if (*out >= 0xFFFFFFFFull) return E_InvalidVarInt;
    *has = 1; return E_OK;
}
static i64 zigzag_old(u64 n) { return (i64)(n >> 1) * ((n & 1) ? -1 : 1); }  /* leb.rs:318-321 */
static int rd_zigzag(Buf *b, i64 *out) { u64 n; int e = rd_usize(b, &n); if (e) return e; *out = zigzag_old(n); return E_OK; }
static int rd_bytes(Buf *b, size_t k, const u8 **out) {
    if (k > b->n) return E_UnexpectedEOF;
    *out = b->p; b->p += k; b->n -= k; return E_OK;
}

static int utf8_valid(const u8 *s, size_t n) {
    size_t i = 0;
    while (i < n) {
        u8 c = s[i];
        if (c < 0x80) { i++; continue; }
        size_t len; u32 cp;
        if ((c & 0xE0) == 0xC0) { len = 2; cp = c & 0x1F; }
        else if ((c & 0xF0) == 0xE0) { len = 3; cp = c & 0x0F; }
        else if ((c & 0xF8) == 0xF0) { len = 4; cp = c & 0x07; }
        else return 0;
        if (i + len > n) return 0;
        for (size_t k = 1; k < len; k++) { if ((s[i + k] & 0xC0) != 0x80) return 0; cp = (cp << 6) | (s[i + k] & 0x3F); }
        if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && cp < 0x10000)) return 0;
        if (cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return 0;
        i += len;
    }
    return 1;
}
static size_t utf8_char_len(u8 c) { return c < 0x80 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : 4; }

/* chunk types (src/list/encoding/mod.rs:26-58) */
enum { CT_FileInfo = 1, CT_DocId = 2, CT_AgentNames = 3, CT_UserData = 4, CT_LZ4 = 5, CT_StartBranch = 10,
       CT_EndBranch = 11, CT_Version = 12, CT_Content = 13, CT_ContentCompressed = 14, CT_Patches = 20,
       CT_OpVersions = 21, CT_OpTypeAndPosition = 22, CT_OpParents = 23, CT_PatchContent = 24,
       CT_ContentIsKnown = 25, CT_TransformedPositions = 27, CT_Crc = 100 };
static int chunk_known(u64 t) {
    switch (t) { case 1: case 2: case 3: case 4: case 5: case 10: case 11: case 12: case 13: case 14:
        case 20: case 21: case 22: case 23: case 24: case 25: case 27: case 100: return 1; }
    return 0;
}
/* ChunkReader::next_chunk (decode_tools.rs:208-236): skips unknown chunk types. */
static int next_chunk(Buf *r, u64 *type, Buf *out) {
    for (;;) {
        u64 t, len; int e = rd_u32(r, &t); if (e) return e;
        e = rd_usize(r, &len); if (e) return e;
        if (len > r->n) return E_InvalidLength;
        out->p = r->p; out->n = (size_t)len; r->p += len; r->n -= len;
        if (chunk_known(t)) { *type = t; return E_OK; }
    }
}
static int read_chunk_if_eq(Buf *r, u64 want, int *found, Buf *out) {
    int has; u64 t; int e = peek_u32(r, &has, &t); if (e) return e;
    *found = 0;
    if (!has || t != want) return E_OK;
    u64 tt; e = next_chunk(r, &tt, out); if (e) return e;
    *found = 1; return E_OK;
}
static int expect_chunk(Buf *r, u64 want, Buf *out) {
    u64 t; int e = next_chunk(r, &t, out); if (e) return e;
    return t == want ? E_OK : E_MissingChunk;
}

/* ------------------------------------------------------------------------------------------ */
/* CRC-32C (crc crate CRC_32_ISCSI: refin/refout, poly 0x1EDC6F41, init/xorout 0xFFFFFFFF)      */
/* ------------------------------------------------------------------------------------------ */
static u32 crc_tab[256]; static int crc_init;
EXPORT u32 dto_crc32c(const u8 *d, size_t n) {
    if (!crc_init) {
        for (u32 i = 0; i < 256; i++) { u32 c = i; for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1; crc_tab[i] = c; }
        crc_init = 1;
    }
    u32 c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; i++) c = crc_tab[(c ^ d[i]) & 0xFF] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}

/* ------------------------------------------------------------------------------------------ */
/* LZ4 raw block decompression (lz4_flex::decompress(input, uncompressed_len))                 */
/* ------------------------------------------------------------------------------------------ */
EXPORT int dto_lz4_decompress(const u8 *src, size_t n, u8 *dst, size_t out_len) {
    size_t ip = 0, op = 0;
    while (ip < n) {
        u8 tok = src[ip++];
        size_t lit = tok >> 4;
        if (lit == 15) { u8 b; do { if (ip >= n) return -1; b = src[ip++]; lit += b; } while (b == 255); }
        if (ip + lit > n || op + lit > out_len) return -1;
        memcpy(dst + op, src + ip, lit); ip += lit; op += lit;
        if (ip >= n) break;                           /* last sequence: literals only */
        if (ip + 2 > n) return -1;
        size_t off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8); ip += 2;
        if (off == 0 || off > op) return -1;
        size_t ml = (tok & 15);
        if (ml == 15) { u8 b; do { if (ip >= n) return -1; b = src[ip++]; ml += b; } while (b == 255); }
        ml += 4;
        if (op + ml > out_len) return -1;
        for (size_t k = 0; k < ml; k++) { dst[op] = dst[op - off]; op++; }   /* overlapping copy */
    }
    return op == out_len ? 0 : -1;
}

/* ------------------------------------------------------------------------------------------ */
/* causal graph (src/causalgraph/graph/mod.rs:25-128)                                         */
/* ------------------------------------------------------------------------------------------ */
typedef struct { i64 start, end, shadow; int np; i64 *parents; } GEntry;
typedef struct { VEC(GEntry) e; } Graph;

static i64 graph_find_idx(const Graph *g, i64 lv) {
    i64 lo = 0, hi = g->e.n - 1;
    while (lo <= hi) {
        i64 mid = (lo + hi) / 2; const GEntry *e = &g->e.v[mid];
        if (lv < e->start) hi = mid - 1; else if (lv >= e->end) lo = mid + 1; else return mid;
    }
    return -1;
}
static const GEntry *graph_find(const Graph *g, i64 lv) { i64 i = graph_find_idx(g, lv); return i < 0 ? NULL : &g->e.v[i]; }
static int contains_i64(const i64 *a, int n, i64 x) { for (int i = 0; i < n; i++) if (a[i] == x) return 1; return 0; }

static void graph_push(Graph *g, const i64 *parents, int np, i64 start, i64 end) {
    if (g->e.n) {   /* fast path: linear append extends the last entry */
        GEntry *last = &g->e.v[g->e.n - 1];
        if (np == 1 && parents[0] == last->end - 1 && last->end == start) { last->end = end; return; }
    }
    i64 shadow = start;
    while (shadow >= 1 && contains_i64(parents, np, shadow - 1)) shadow = graph_find(g, shadow - 1)->shadow;
    GEntry ne = { start, end, shadow, np, NULL };
    if (np) { ne.parents = malloc(sizeof(i64) * (size_t)np); memcpy(ne.parents, parents, sizeof(i64) * (size_t)np); }
    VPUSH(g->e, ne);
}
static void graph_free(Graph *g) { for (i64 i = 0; i < g->e.n; i++) free(g->e.v[i].parents); VFREE(g->e); }

static int cmp_i64(const void *a, const void *b) { i64 x = *(const i64 *)a, y = *(const i64 *)b; return x < y ? -1 : x > y; }
static void sort_frontier(i64 *f, int n) { qsort(f, (size_t)n, sizeof(i64), cmp_i64); }

/* ---- binary max-heap of (key, aux) pairs ---- */
typedef struct { i64 k; int f; } HItem;
typedef VEC(HItem) Heap;
static int hi_gt(HItem a, HItem b) { return a.k != b.k ? a.k > b.k : a.f > b.f; }
static void heap_push(Heap *h, i64 k, int f) {
    HItem x = { k, f }; VPUSH(*h, x);
    i64 i = h->n - 1;
    while (i > 0) { i64 p = (i - 1) / 2; if (!hi_gt(h->v[i], h->v[p])) break; HItem t = h->v[i]; h->v[i] = h->v[p]; h->v[p] = t; i = p; }
}
static HItem heap_pop(Heap *h) {
    HItem top = h->v[0]; h->v[0] = h->v[--h->n];
    i64 i = 0;
    for (;;) {
        i64 l = 2 * i + 1, r = l + 1, m = i;
        if (l < h->n && hi_gt(h->v[l], h->v[m])) m = l;
        if (r < h->n && hi_gt(h->v[r], h->v[m])) m = r;
        if (m == i) break;
        HItem t = h->v[i]; h->v[i] = h->v[m]; h->v[m] = t; i = m;
    }
    return top;
}

/* frontier_contains_version (tools.rs:88-146) */
static int frontier_contains_version(const Graph *g, const i64 *f, int n, i64 target) {
    if (contains_i64(f, n, target)) return 1;
    if (n == 0) return 0;
    for (int i = 0; i < n; i++) if (f[i] > target) { const GEntry *e = graph_find(g, f[i]); if (target >= e->shadow) return 1; }
    Heap q = {0};
    for (int i = 0; i < n; i++) if (f[i] > target) heap_push(&q, f[i], 0);
    int found = 0;
    while (q.n) {
        i64 ord = heap_pop(&q).k;
        const GEntry *e = graph_find(g, ord);
        if (target >= e->shadow) { found = 1; break; }
        while (q.n && q.v[0].k >= e->start) heap_pop(&q);
        for (int i = 0; i < e->np; i++) {
            i64 p = e->parents[i];
            if (p == target) { found = 1; goto done; }
            else if (p > target) heap_push(&q, p, 0);
        }
    }
done:
    VFREE(q);
    return found;
}

/* push_reversed_rle: spans arrive in descending order; merge when contiguous. */
static void push_rev(VecRange *v, i64 s, i64 e) {
    if (v->n && v->v[v->n - 1].start == e) { v->v[v->n - 1].start = s; return; }
    Range r = { s, e }; VPUSH(*v, r);
}

enum { F_OnlyA = 0, F_OnlyB = 1, F_Shared = 2 };

/* diff_rev / diff_slow_internal (tools.rs:176-292). Outputs in descending order. */
static void graph_diff_rev(const Graph *g, const i64 *a, int na, const i64 *b, int nb, VecRange *oa, VecRange *ob) {
    oa->n = ob->n = 0;
    if (na == nb && (na == 0 || memcmp(a, b, sizeof(i64) * (size_t)na) == 0)) return;
    if (na == 1 && nb == 1) {
        i64 x = a[0], y = b[0];
        const GEntry *ex = graph_find(g, x), *ey = graph_find(g, y);
        if (x > y && y >= ex->start) { push_rev(oa, y + 1, x + 1); return; }   /* is_direct_descendant_coarse */
        if (y > x && x >= ey->start) { push_rev(ob, x + 1, y + 1); return; }
    }
    Heap q = {0};
    for (int i = 0; i < na; i++) heap_push(&q, a[i], F_OnlyA);
    for (int i = 0; i < nb; i++) heap_push(&q, b[i], F_OnlyB);
    i64 num_shared = 0;
    while (q.n) {
        HItem it = heap_pop(&q);
        i64 ord = it.k; int flag = it.f;
        if (flag == F_Shared) num_shared--;
        while (q.n && q.v[0].k == ord) {
            HItem pk = q.v[0];
            if (pk.f != flag) flag = F_Shared;
            if (pk.f == F_Shared) num_shared--;
            heap_pop(&q);
        }
        const GEntry *e = graph_find(g, ord);
        while (q.n && q.v[0].k >= e->start) {
            HItem pk = q.v[0];
            if (pk.f != flag) {
                if (flag == F_OnlyA) push_rev(oa, pk.k + 1, ord + 1);
                else if (flag == F_OnlyB) push_rev(ob, pk.k + 1, ord + 1);
                ord = pk.k; flag = F_Shared;
            }
            if (pk.f == F_Shared) num_shared--;
            heap_pop(&q);
        }
        if (flag == F_OnlyA) push_rev(oa, e->start, ord + 1);
        else if (flag == F_OnlyB) push_rev(ob, e->start, ord + 1);
        for (int i = 0; i < e->np; i++) { heap_push(&q, e->parents[i], flag); if (flag == F_Shared) num_shared++; }
        if (q.n == num_shared) break;
    }
    VFREE(q);
}

/* ---- find_conflicting (tools.rs:296-484) ---- */
/* TimePoint + flag; merged_with is a SmallVec in the reference: OR_TP_M bounds it here (a wider
 * frontier or merge aborts the oracle rather than answer wrongly) */
#define OR_TP_M 255
typedef struct { i64 last; int nm; i64 m[OR_TP_M]; int flag; } TP;
typedef VEC(TP) TPHeap;
/* Ord for (TimePoint, DiffFlag): last.wrapping_add(1) asc, then fewer merged_with is greater,
 * then (Rust tuple / derived Ord) merged_with lexicographic is irrelevant once lens differ... */
static int tp_cmp(const TP *a, const TP *b) {
    u64 la = (u64)a->last + 1, lb = (u64)b->last + 1;      /* ROOT (-1) -> 0 */
    if (la != lb) return la < lb ? -1 : 1;
    if (a->nm != b->nm) return a->nm > b->nm ? -1 : 1;      /* other.len().cmp(self.len()) */
    /* TimePoint's Ord ignores merged_with content; the tuple then compares the flag. */
    if (a->flag != b->flag) return a->flag < b->flag ? -1 : 1;
    return 0;
}
static int tp_eq_time(const TP *a, const TP *b) {   /* PartialEq derives on (last, merged_with) */
    if (a->last != b->last || a->nm != b->nm) return 0;
    for (int i = 0; i < a->nm; i++) if (a->m[i] != b->m[i]) return 0;
    return 1;
}
static void tph_push(TPHeap *h, TP x) {
    VPUSH(*h, x); i64 i = h->n - 1;
    while (i > 0) { i64 p = (i - 1) / 2; if (tp_cmp(&h->v[i], &h->v[p]) <= 0) break; TP t = h->v[i]; h->v[i] = h->v[p]; h->v[p] = t; i = p; }
}
static TP tph_pop(TPHeap *h) {
    TP top = h->v[0]; h->v[0] = h->v[--h->n]; i64 i = 0;
    for (;;) {
        i64 l = 2 * i + 1, r = l + 1, m = i;
        if (l < h->n && tp_cmp(&h->v[l], &h->v[m]) > 0) m = l;
        if (r < h->n && tp_cmp(&h->v[r], &h->v[m]) > 0) m = r;
        if (m == i) break;
        TP t = h->v[i]; h->v[i] = h->v[m]; h->v[m] = t; i = m;
    }
    return top;
}
static TP tp_from_frontier(const i64 *f, int n, int flag) {
    if (n - 1 > OR_TP_M) abort();
    TP t; t.flag = flag; t.nm = 0;
    t.last = n ? f[n - 1] : ROOT_LV;
    if (n > 1) { t.nm = n - 1; for (int i = 0; i < n - 1; i++) t.m[i] = f[i]; }
    return t;
}
typedef void (*visit_fn)(void *ctx, i64 s, i64 e, int flag);

/* returns common-ancestor frontier size, writes into common[] (cap OR_TP_M + 1) */
static int find_conflicting_slow(const Graph *g, const i64 *a, int na, const i64 *b, int nb, visit_fn visit, void *ctx, i64 *common) {
    TPHeap q = {0};
    tph_push(&q, tp_from_frontier(a, na, F_OnlyA));
    tph_push(&q, tp_from_frontier(b, nb, F_OnlyB));
    int nc = 0;
    for (;;) {
        TP time = tph_pop(&q);
        int flag = time.flag;
        i64 t = time.last;
        if (t == ROOT_LV) { nc = 0; break; }
        while (q.n && tp_eq_time(&q.v[0], &time)) { if (q.v[0].flag != flag) flag = F_Shared; tph_pop(&q); }
        if (q.n == 0) {
            for (int i = 0; i < time.nm; i++) common[nc++] = time.m[i];
            common[nc++] = t;
            break;
        }
        for (int i = 0; i < time.nm; i++) { TP x = tp_from_frontier(&time.m[i], 1, flag); tph_push(&q, x); }
        const GEntry *e = graph_find(g, t);
        i64 rs = e->start, re = t + 1;
        for (;;) {
            if (q.n) {
                TP *pk = &q.v[0];
                if (pk->last != ROOT_LV && pk->last >= e->start) {
                    TP tm = tph_pop(&q);
                    int next_flag = tm.flag;
                    if (tm.last + 1 < re) {
                        i64 off = tm.last + 1 - e->start;
                        /* range.truncate(offset): keeps [rs, rs+off), returns remainder [rs+off, re) */
                        i64 rem_s = rs + off, rem_e = re;
                        re = rs + off;
                        visit(ctx, rem_s, rem_e, flag);
                    }
                    for (int i = 0; i < tm.nm; i++) { TP x = tp_from_frontier(&tm.m[i], 1, next_flag); tph_push(&q, x); }
                    if (next_flag != flag) flag = F_Shared;
                } else {
                    visit(ctx, rs, re, flag);
                    tph_push(&q, tp_from_frontier(e->parents, e->np, flag));
                    break;
                }
            } else {
                common[nc++] = re - 1;
                goto out;
            }
        }
    }
out:
    VFREE(q);
    return nc;
}
static int find_conflicting(const Graph *g, const i64 *a, int na, const i64 *b, int nb, visit_fn visit, void *ctx, i64 *common) {
    if (na == nb && (na == 0 || memcmp(a, b, sizeof(i64) * (size_t)na) == 0)) { for (int i = 0; i < na; i++) common[i] = a[i]; return na; }
    if (na == 1 && nb == 1) {
        i64 x = a[0], y = b[0];
        const GEntry *ex = graph_find(g, x), *ey = graph_find(g, y);
        if (x == y || (x > y && y >= ex->start)) { visit(ctx, y + 1, x + 1, F_OnlyA); common[0] = y; return 1; }
        if (y > x && x >= ey->start) { visit(ctx, x + 1, y + 1, F_OnlyB); common[0] = x; return 1; }
    }
    return find_conflicting_slow(g, a, na, b, nb, visit, ctx, common);
}

/* ------------------------------------------------------------------------------------------ */
/* oplog                                                                                       */
/* ------------------------------------------------------------------------------------------ */
typedef struct { i64 lv_start, len, agent, seq_start; } AgentRun;     /* client_with_localtime */
typedef struct { i64 seq_start, lv_start, len; } SeqRun;             /* ClientData::item_times */
typedef struct { char *name; int name_len; VEC(SeqRun) seqs; } Agent;

typedef struct dto_oplog {
    VEC(Agent) agents;
    VEC(AgentRun) aruns;
    /* per-LV op metrics (the RLE runs of ListOpMetrics expanded to per-LV semantics) */
    VEC(u8) kind;          /* 0 ins, 1 del */
    VEC(i64) pos;          /* ins: position of this char; del: position deleted by this LV */
    VEC(i64) cbyte;        /* ins: byte offset into ins_content, or -1 if content unknown */
    VEC(u8) ins_content;
    Graph g;
    VecI64 version;        /* cg.version */
} dto_oplog;

EXPORT dto_oplog *dto_new(void) { return calloc(1, sizeof(dto_oplog)); }
EXPORT void dto_free(dto_oplog *o) {
    if (!o) return;
    for (i64 i = 0; i < o->agents.n; i++) { free(o->agents.v[i].name); VFREE(o->agents.v[i].seqs); }
    VFREE(o->agents); VFREE(o->aruns); VFREE(o->kind); VFREE(o->pos); VFREE(o->cbyte); VFREE(o->ins_content);
    graph_free(&o->g); VFREE(o->version); free(o);
}
EXPORT i64 dto_len(const dto_oplog *o) { return o->kind.n; }

EXPORT int dto_get_or_create_agent(dto_oplog *o, const char *name, int len) {
    for (i64 i = 0; i < o->agents.n; i++)
        if (o->agents.v[i].name_len == len && memcmp(o->agents.v[i].name, name, (size_t)len) == 0) return (int)i;
    Agent a; memset(&a, 0, sizeof a);
    a.name = malloc((size_t)len + 1); memcpy(a.name, name, (size_t)len); a.name[len] = 0; a.name_len = len;
    VPUSH(o->agents, a);
    return (int)(o->agents.n - 1);
}
static i64 agent_next_seq(const Agent *a) {
    i64 m = 0;
    for (i64 i = 0; i < a->seqs.n; i++) { i64 e = a->seqs.v[i].seq_start + a->seqs.v[i].len; if (e > m) m = e; }
    return m;
}
/* ClientData::try_seq_to_lv (agent_assignment/mod.rs:55-58) */
static i64 seq_to_lv(const Agent *a, i64 seq) {
    for (i64 i = 0; i < a->seqs.n; i++) {
        const SeqRun *r = &a->seqs.v[i];
        if (seq >= r->seq_start && seq < r->seq_start + r->len) return r->lv_start + (seq - r->seq_start);
    }
    return -1;
}
static void assign_span(dto_oplog *o, int agent, i64 seq_start, i64 lv_start, i64 len) {
    Agent *a = &o->agents.v[agent];
    SeqRun s = { seq_start, lv_start, len };
    if (a->seqs.n) { SeqRun *l = &a->seqs.v[a->seqs.n - 1];
        if (l->seq_start + l->len == seq_start && l->lv_start + l->len == lv_start) { l->len += len; goto ar; } }
    VPUSH(a->seqs, s);
ar:;
    if (o->aruns.n) { AgentRun *l = &o->aruns.v[o->aruns.n - 1];
        if (l->agent == agent && l->lv_start + l->len == lv_start && l->seq_start + l->len == seq_start) { l->len += len; return; } }
    AgentRun r = { lv_start, len, agent, seq_start };
    VPUSH(o->aruns, r);
}
static const AgentRun *arun_find(const dto_oplog *o, i64 lv) {
    i64 lo = 0, hi = o->aruns.n - 1;
    while (lo <= hi) { i64 m = (lo + hi) / 2; const AgentRun *r = &o->aruns.v[m];
        if (lv < r->lv_start) hi = m - 1; else if (lv >= r->lv_start + r->len) lo = m + 1; else return r; }
    return NULL;
}

/* Frontier::advance_by_known_run (frontier.rs:251-279) */
static void frontier_advance_known(VecI64 *f, const i64 *parents, int np, i64 last) {
    if (np == 1 && f->n == 1 && parents[0] == f->v[0]) { f->v[0] = last; return; }
    if (f->n == np && (np == 0 || memcmp(f->v, parents, sizeof(i64) * (size_t)np) == 0)) { f->n = 0; VPUSH(*f, last); return; }
    i64 w = 0;
    for (i64 i = 0; i < f->n; i++) if (!contains_i64(parents, np, f->v[i])) f->v[w++] = f->v[i];
    f->n = w; VPUSH(*f, last); sort_frontier(f->v, (int)f->n);
}

/* push one per-LV op (Ins: content chars; Del: positional semantics of truncate_tagged_span) */
static void push_ins_lv(dto_oplog *o, i64 pos, i64 cbyte) { VPUSH(o->kind, 0); VPUSH(o->pos, pos); VPUSH(o->cbyte, cbyte); }
static void push_del_lv(dto_oplog *o, i64 pos) { VPUSH(o->kind, 1); VPUSH(o->pos, pos); VPUSH(o->cbyte, -1); }

/* ListOpLog::add_insert_at / add_delete_at (src/list/oplog.rs:221-246) with cg.assign_span. */
static void add_span_common(dto_oplog *o, int agent, const i64 *parents_in, int np, i64 start, i64 end) {
    i64 *par = malloc(sizeof(i64) * (size_t)(np ? np : 1));
    memcpy(par, parents_in, sizeof(i64) * (size_t)np); sort_frontier(par, np);
    assign_span(o, agent, agent_next_seq(&o->agents.v[agent]), start, end - start);
    graph_push(&o->g, par, np, start, end);
    frontier_advance_known(&o->version, par, np, end - 1);
    free(par);
}
EXPORT i64 dto_add_insert_at(dto_oplog *o, int agent, const i64 *parents, int np, i64 pos, const char *s, i64 nbytes) {
    i64 start = o->kind.n, k = 0;
    i64 base = o->ins_content.n;
    for (i64 i = 0; i < nbytes; i++) VPUSH(o->ins_content, (u8)s[i]);
    for (i64 i = 0; i < nbytes; i += (i64)utf8_char_len((u8)s[i]), k++) push_ins_lv(o, pos + k, base + i);
    if (k == 0) return start - 1;
    add_span_common(o, agent, parents, np, start, start + k);
    return start + k - 1;
}
EXPORT i64 dto_add_delete_at(dto_oplog *o, int agent, const i64 *parents, int np, i64 del_start, i64 del_end) {
    i64 start = o->kind.n;
    for (i64 i = del_start; i < del_end; i++) push_del_lv(o, del_start);   /* fwd delete: every LV at start */
    if (del_end <= del_start) return start - 1;
    add_span_common(o, agent, parents, np, start, start + (del_end - del_start));
    return start + (del_end - del_start) - 1;
}
EXPORT i64 dto_add_insert(dto_oplog *o, int agent, i64 pos, const char *s, i64 nbytes) {
    VecI64 v = o->version; return dto_add_insert_at(o, agent, v.v, (int)v.n, pos, s, nbytes);
}
EXPORT i64 dto_add_delete(dto_oplog *o, int agent, i64 s, i64 e) {
    VecI64 v = o->version; return dto_add_delete_at(o, agent, v.v, (int)v.n, s, e);
}
EXPORT int dto_frontier(const dto_oplog *o, i64 *out, int cap) {
    for (int i = 0; i < o->version.n && i < cap; i++) out[i] = o->version.v[i];
    return (int)o->version.n;
}
EXPORT int dto_num_agents(const dto_oplog *o) { return (int)o->agents.n; }
EXPORT i64 dto_num_graph_entries(const dto_oplog *o) { return o->g.e.n; }
EXPORT i64 dto_num_agent_runs(const dto_oplog *o) { return o->aruns.n; }
EXPORT i64 dto_ins_content_len(const dto_oplog *o) { return o->ins_content.n; }

/* ------------------------------------------------------------------------------------------ */
/* .dt decode: ListOpLog::load_from -> decode_internal (decode_oplog.rs:447-960)              */
/* ------------------------------------------------------------------------------------------ */
typedef struct { i64 len; int known; const u8 *s; size_t sn; } CItem;   /* ContentItem */
typedef struct { int present; Buf runs; const u8 *content; size_t cn; int has_pb; CItem pb; } CIter;

static int citer_next(CIter *it, int *has, CItem *out) {
    if (it->has_pb) { *out = it->pb; it->has_pb = 0; *has = 1; return E_OK; }
    if (it->runs.n == 0) {
        if (it->cn == 0) { *has = 0; return E_OK; }
        return E_UnexpectedEOF;
    }
    u64 n; int e = rd_usize(&it->runs, &n); if (e) return e;
    out->len = (i64)(n >> 1); out->known = (int)(n & 1); out->s = NULL; out->sn = 0;
    if (out->known) {   /* consume_chars(len) + count check (decode_oplog.rs:402-407) */
        size_t b = 0; i64 c = 0;
        while (c < out->len && b < it->cn) { b += utf8_char_len(it->content[b]); c++; }
        if (b > it->cn) b = it->cn;
        if (c != out->len) return E_UnexpectedEOF;
        out->s = it->content; out->sn = b; it->content += b; it->cn -= b;
    }
    *has = 1; return E_OK;
}
/* split a content item after `at` chars; remainder goes back to the iterator */
static CItem citem_trim(CItem *c, i64 at) {
    CItem r = *c; r.len = c->len - at;
    if (c->known) { size_t b = 0; for (i64 k = 0; k < at; k++) b += utf8_char_len(c->s[b]); r.s = c->s + b; r.sn = c->sn - b; c->sn = b; }
    c->len = at; return r;
}

static int read_content_str(Buf *chunks, Buf *compressed, int has_comp, const u8 **s, size_t *sn) {
    u64 t; Buf c; int e = next_chunk(chunks, &t, &c); if (e) return e;
    if (t != CT_Content && t != CT_ContentCompressed) return E_MissingChunk;
    u64 dt; e = rd_u32(&c, &dt); if (e) return e;
    if (dt != 4) return E_UnknownChunk;
    if (t == CT_Content) { if (!utf8_valid(c.p, c.n)) return E_InvalidUTF8; *s = c.p; *sn = c.n; return E_OK; }
    u64 len; e = rd_usize(&c, &len); if (e) return e;
    if (!has_comp) return E_CompressedDataMissing;
    const u8 *b; e = rd_bytes(compressed, (size_t)len, &b); if (e) return e;
    if (!utf8_valid(b, (size_t)len)) return E_InvalidUTF8;
    *s = b; *sn = (size_t)len; return E_OK;
}

typedef struct { int agent; i64 seq; } AMap;   /* agent_map entries: (AgentId, next seq) */

static int decode_internal(dto_oplog *o, const u8 *data, size_t len, int ignore_crc) {
    int e; Buf r = { data, len };
    u8 *lz = NULL; Buf comp = {0}; int has_comp = 0;
    VEC(AMap) amap = {0};
    if (r.n < 8) { e = E_UnexpectedEOF; goto fail; }
    if (memcmp(r.p, "DMNDTYPS", 8) != 0) { e = E_InvalidMagic; goto fail; }
    r.p += 8; r.n -= 8;
    { u64 pv; if ((e = rd_usize(&r, &pv))) goto fail; if (pv != 0) { e = E_UnsupportedProtocolVersion; goto fail; } }

    {   /* CompressedFieldsLZ4 */
        int found; Buf c;
        if ((e = read_chunk_if_eq(&r, CT_LZ4, &found, &c))) goto fail;
        if (found) {
            u64 ulen; if ((e = rd_usize(&c, &ulen))) goto fail;
            lz = malloc(ulen ? (size_t)ulen : 1);
            if (dto_lz4_decompress(c.p, c.n, lz, (size_t)ulen) != 0) { e = E_LZ4DecompressionError; goto fail; }
            comp.p = lz; comp.n = (size_t)ulen; has_comp = 1;
        }
    }
    {   /* FileInfo (decode_oplog.rs:197-227) */
        Buf fi, an, tmp; int found;
        if ((e = expect_chunk(&r, CT_FileInfo, &fi))) goto fail;
        if ((e = read_chunk_if_eq(&fi, CT_DocId, &found, &tmp))) goto fail;
        if (found) { u64 dt; if ((e = rd_u32(&tmp, &dt))) goto fail; if (dt != 4) { e = E_UnknownChunk; goto fail; }
                     if (!utf8_valid(tmp.p, tmp.n)) { e = E_InvalidUTF8; goto fail; } }
        if ((e = expect_chunk(&fi, CT_AgentNames, &an))) goto fail;
        if ((e = read_chunk_if_eq(&fi, CT_UserData, &found, &tmp))) goto fail;
        while (an.n) {
            u64 nl; if ((e = rd_usize(&an, &nl))) goto fail;
            if (nl > an.n) { e = E_InvalidLength; goto fail; }
            const u8 *nm; if ((e = rd_bytes(&an, (size_t)nl, &nm))) goto fail;
            if (!utf8_valid(nm, (size_t)nl)) { e = E_InvalidUTF8; goto fail; }
            if ((nl == 4 && memcmp(nm, "ROOT", 4) == 0) || nl >= 50) { e = E_CheckoutPanic; goto fail; }
            AMap m = { dto_get_or_create_agent(o, (const char *)nm, (int)nl), 0 };
            VPUSH(amap, m);
        }
    }
    {   /* StartBranch */
        Buf sb, ver; int found;
        if ((e = expect_chunk(&r, CT_StartBranch, &sb))) goto fail;
        if ((e = read_chunk_if_eq(&sb, CT_Version, &found, &ver))) goto fail;
        if (found) {   /* read_version (decode_oplog.rs:70-93): nothing is known in a fresh oplog */
            for (;;) {
                u64 n, seq; if ((e = rd_usize(&ver, &n))) goto fail; if ((e = rd_usize(&ver, &seq))) goto fail;
                if ((n >> 1) == 0) break;
                if ((n >> 1) - 1 >= (u64)amap.n) { e = E_InvalidLength; goto fail; }
                if (seq_to_lv(&o->agents.v[amap.v[(n >> 1) - 1].agent], (i64)seq) < 0) { e = E_BaseVersionUnknown; goto fail; }
                if (!(n & 1)) break;
            }
            if (ver.n) { e = E_InvalidLength; goto fail; }
        }
        if (sb.n) { const u8 *s; size_t sn; if ((e = read_content_str(&sb, &comp, has_comp, &s, &sn))) goto fail; }
    }
    {   /* Patches */
        Buf pc, ch; int found;
        CIter ins = {0}, del = {0};
        if ((e = expect_chunk(&r, CT_Patches, &pc))) goto fail;
        for (;;) {
            if ((e = read_chunk_if_eq(&pc, CT_PatchContent, &found, &ch))) goto fail;
            if (!found) break;
            u64 tag; if ((e = rd_u32(&ch, &tag))) goto fail;
            if (tag > 1) { e = E_InvalidContent; goto fail; }
            CIter it = {0}; it.present = 1;
            if ((e = read_content_str(&ch, &comp, has_comp, &it.content, &it.cn))) goto fail;
            if ((e = expect_chunk(&ch, CT_ContentIsKnown, &it.runs))) goto fail;
            if (tag == 0) ins = it; else del = it;
        }
        /* the ins content arena is the concatenation of known insert content in LV order */
        Buf av, tp, hist;
        if ((e = expect_chunk(&pc, CT_OpVersions, &av))) goto fail;
        if ((e = expect_chunk(&pc, CT_OpTypeAndPosition, &tp))) goto fail;
        if ((e = expect_chunk(&pc, CT_OpParents, &hist))) goto fail;

        /* ReadPatchesIter state */
        i64 last_cursor = 0;
        int has_op_pb = 0; i64 op_len = 0, op_start = 0; int op_kind = 0, op_fwd = 1;
        i64 next_patch = 0, next_assign = 0;

        while (av.n) {   /* read_next_agent_assignment (decode_oplog.rs:29-68) */
            u64 n, alen; i64 jump = 0;
            if ((e = rd_usize(&av, &n))) goto fail;
            int has_jump = (int)(n & 1); n >>= 1;
            if ((e = rd_usize(&av, &alen))) goto fail;
            if (has_jump) { if ((e = rd_zigzag(&av, &jump))) goto fail; }
            if (n == 0 || n - 1 >= (u64)amap.n) { e = E_InvalidLength; goto fail; }
            AMap *m = &amap.v[n - 1];
            i64 sstart = m->seq + jump;
            m->seq = sstart + (i64)alen;
            assign_span(o, m->agent, sstart, next_assign, (i64)alen);
            next_assign += (i64)alen;

            i64 want = (i64)alen;   /* parse_next_patches (decode_oplog.rs:731-778) */
            while (want > 0) {
                if (!has_op_pb) {
                    if (tp.n == 0) { e = E_InvalidLength; goto fail; }
                    u64 x; if ((e = rd_usize(&tp, &x))) goto fail;
                    int has_length = (int)(x & 1); x >>= 1;
                    int diff_nz = (int)(x & 1); x >>= 1;
                    int is_del = (int)(x & 1); x >>= 1;
                    i64 diff; int fwd = 1; i64 l;
                    if (has_length) {
                        if (is_del) { fwd = (int)(x & 1); x >>= 1; }
                        diff = 0; if (diff_nz) { if ((e = rd_zigzag(&tp, &diff))) goto fail; }
                        l = (i64)x;
                    } else { l = 1; diff = zigzag_old(x); }
                    i64 raw = (i64)((u64)last_cursor + (u64)diff);
                    i64 st, raw_end;
                    if (!is_del) { st = raw; raw_end = raw + l; }
                    else if (fwd) { st = raw; raw_end = raw; }
                    else { st = raw - l; raw_end = raw - l; }
                    last_cursor = raw_end;
                    op_len = l; op_start = st; op_kind = is_del; op_fwd = fwd; has_op_pb = 1;
                    if (l == 0) { e = E_CheckoutPanic; goto fail; }   /* assert!(max_len > 0) */
                }
                i64 max_len = want < op_len ? want : op_len;
                CIter *ci = op_kind ? &del : &ins;
                CItem citem; int have_c = 0;
                if (ci->present) {
                    int has; if ((e = citer_next(ci, &has, &citem))) goto fail;
                    if (!has) { e = E_InvalidLength; goto fail; }
                    if (citem.len < max_len) max_len = citem.len;
                    if (citem.len > max_len) { ci->pb = citem_trim(&citem, max_len); ci->has_pb = 1; }
                    have_c = 1;
                }
                if (max_len <= 0) { e = E_CheckoutPanic; goto fail; }
                /* emit max_len LVs of this op (per-LV semantics of truncate_tagged_span) */
                if (op_kind == 0) {
                    i64 b0 = -1;
                    if (have_c && citem.known) { b0 = o->ins_content.n; for (size_t k = 0; k < citem.sn; k++) VPUSH(o->ins_content, citem.s[k]); }
                    size_t bo = 0;
                    for (i64 k = 0; k < max_len; k++) {
                        push_ins_lv(o, op_start + k, b0 >= 0 ? b0 + (i64)bo : -1);
                        if (b0 >= 0) bo += utf8_char_len(citem.s[bo]);
                    }
                    op_start += max_len;
                } else if (op_fwd) {
                    for (i64 k = 0; k < max_len; k++) push_del_lv(o, op_start);
                } else {
                    i64 end = op_start + op_len;
                    for (i64 k = 0; k < max_len; k++) push_del_lv(o, end - 1 - k);
                }
                op_len -= max_len;
                if (op_len == 0) has_op_pb = 0;
                next_patch += max_len; want -= max_len;
            }
        }
        /* history (decode_oplog.rs:856-913); fresh load => identity version map */
        i64 next_file = 0, next_hist = 0;
        VecI64 par = {0};
        while (hist.n) {
            u64 hl; if ((e = rd_usize(&hist, &hl))) goto fail_par;
            par.n = 0;
            for (;;) {   /* read_parents (decode_oplog.rs:95-137) */
                u64 n; if ((e = rd_usize(&hist, &n))) goto fail_par;
                int foreign = (int)(n & 1); n >>= 1;
                int more = (int)(n & 1); n >>= 1;
                i64 p;
                if (foreign) {
                    if (n == 0) break;
                    if (n - 1 >= (u64)amap.n) { e = E_InvalidLength; goto fail_par; }
                    u64 seq; if ((e = rd_usize(&hist, &seq))) goto fail_par;
                    p = seq_to_lv(&o->agents.v[amap.v[n - 1].agent], (i64)seq);
                    if (p < 0) { e = E_InvalidLength; goto fail_par; }
                } else p = next_file - (i64)n;
                VPUSH(par, p);
                if (!more) break;
            }
            sort_frontier(par.v, (int)par.n);
            if (hl == 0 || next_file + (i64)hl > next_assign) { e = E_InvalidLength; goto fail_par; }
            for (i64 i = 0; i < par.n; i++) if (par.v[i] < 0 || par.v[i] >= next_file) { e = E_InvalidLength; goto fail_par; }
            graph_push(&o->g, par.v, (int)par.n, next_file, next_file + (i64)hl);
            frontier_advance_known(&o->version, par.v, (int)par.n, next_file + (i64)hl - 1);
            next_file += (i64)hl; next_hist += (i64)hl;
        }
        VFREE(par);
        if (next_patch != next_assign || next_patch != next_hist) { e = E_InvalidLength; goto fail; }
        if (pc.n) { e = E_InvalidLength; goto fail; }
        if (ins.present) { int has; CItem c; int ee = citer_next(&ins, &has, &c); if (ee || has) { e = E_InvalidContent; goto fail; } }
        if (del.present) { int has; CItem c; int ee = citer_next(&del, &has, &c); if (ee || has) { e = E_InvalidContent; goto fail; } }
        if (0) { fail_par: VFREE(par); goto fail; }
    }
    {   /* CRC (decode_oplog.rs:940-955) */
        size_t reader_len = r.n; int found; Buf c;
        if ((e = read_chunk_if_eq(&r, CT_Crc, &found, &c))) goto fail;
        if (found && !ignore_crc) {
            if (c.n < 4) { e = E_UnexpectedEOF; goto fail; }
            u32 want = (u32)c.p[0] | ((u32)c.p[1] << 8) | ((u32)c.p[2] << 16) | ((u32)c.p[3] << 24);
            if (dto_crc32c(data, len - reader_len) != want) { e = E_ChecksumFailed; goto fail; }
        }
    }
    free(lz); VFREE(amap);
    return E_OK;
fail:
    free(lz); VFREE(amap);
    return e;
}

EXPORT int dto_load(const u8 *bytes, size_t len, int ignore_crc, dto_oplog **out) {
    dto_oplog *o = dto_new();
    int e = decode_internal(o, bytes, len, ignore_crc);
    if (e) { dto_free(o); *out = NULL; return e; }
    *out = o; return E_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* SpanningTreeWalker (txn_trace.rs:114-333), full walk from ROOT                              */
/* ------------------------------------------------------------------------------------------ */
typedef struct { i64 start, end; int np; const i64 *parents; i64 p1; int own_p1; VecI64 pidx, cidx; int visited; } VisitEntry;
typedef struct { VecRange retreat, advance_rev; Range consume; } WalkStep;

typedef struct {
    const Graph *g; VEC(VisitEntry) in; VecI64 todo; VecI64 frontier;
} Walker;

static i64 find_input(const Walker *w, i64 t) {
    i64 lo = 0, hi = w->in.n - 1;
    while (lo <= hi) { i64 m = (lo + hi) / 2; const VisitEntry *e = &w->in.v[m];
        if (t < e->start) hi = m - 1; else if (t >= e->end) lo = m + 1; else return m; }
    return -1;
}
/* SpanningTreeWalker::new (txn_trace.rs:114-182): ascending input spans split per graph entry;
 * parents outside the input are ignored. */
static void walker_init(Walker *w, const Graph *g, const Range *spans, i64 nspans) {
    memset(w, 0, sizeof *w); w->g = g;
    for (i64 si = 0; si < nspans; si++) {
        i64 s = spans[si].start, e = spans[si].end;
        i64 gi = graph_find_idx(g, s);
        while (s < e) {
            const GEntry *ge = &g->e.v[gi];
            i64 pe = ge->end < e ? ge->end : e;
            VisitEntry ve; memset(&ve, 0, sizeof ve);
            ve.start = s; ve.end = pe;
            if (s > ge->start) { ve.p1 = s - 1; ve.own_p1 = 1; ve.np = 1; }   /* clone_parents_at_version */
            else { ve.np = ge->np; ve.parents = ge->parents; }
            VPUSH(w->in, ve);
            s = pe; gi++;
        }
    }
    for (i64 i = 0; i < w->in.n; i++) {
        VisitEntry *ve = &w->in.v[i];
        if (ve->own_p1) ve->parents = &ve->p1;   /* stable now that the vector is built */
        for (int k = 0; k < ve->np; k++) { i64 pi = find_input(w, ve->parents[k]); if (pi >= 0) VPUSH(ve->pidx, pi); }
        if (ve->pidx.n == 0) VPUSH(w->todo, i);
    }
    for (i64 i = 0; i < w->in.n; i++)
        for (i64 k = 0; k < w->in.v[i].pidx.n; k++) VPUSH(w->in.v[w->in.v[i].pidx.v[k]].cidx, i);
    for (i64 i = 0, j = w->todo.n - 1; i < j; i++, j--) { i64 t = w->todo.v[i]; w->todo.v[i] = w->todo.v[j]; w->todo.v[j] = t; }
}
static void walker_free(Walker *w) {
    for (i64 i = 0; i < w->in.n; i++) { VFREE(w->in.v[i].pidx); VFREE(w->in.v[i].cidx); }
    VFREE(w->in); VFREE(w->todo); VFREE(w->frontier);
}
static int walker_next(Walker *w, WalkStep *st) {
    if (w->todo.n == 0) return 0;
    i64 idx = w->todo.v[w->todo.n - 1];
    if (w->in.v[idx].np >= 2) {
        i64 found = -1;
        for (i64 ii = w->todo.n - 1; ii >= 0; ii--) if (w->in.v[w->todo.v[ii]].np < 2) { found = ii; break; }
        if (found >= 0) { idx = w->todo.v[found]; w->todo.v[found] = w->todo.v[w->todo.n - 1]; w->todo.n--; }
        else w->todo.n--;
    } else w->todo.n--;
    VisitEntry *e = &w->in.v[idx];
    e->visited = 1;
    graph_diff_rev(w->g, w->frontier.v, (int)w->frontier.n, e->parents, e->np, &st->retreat, &st->advance_rev);
    /* after retreat+advance the walker frontier equals the txn parents; consuming the span
     * makes it [span.last] (Frontier::advance_by_known_run, frontier.rs:251-263). */
    w->frontier.n = 0; VPUSH(w->frontier, e->end - 1);
    st->consume.start = e->start; st->consume.end = e->end;
    for (i64 k = 0; k < e->cidx.n; k++) {
        i64 c = e->cidx.v[k]; VisitEntry *ce = &w->in.v[c];
        if (ce->visited) continue;
        int ok = 1; for (i64 q = 0; q < ce->pidx.n; q++) if (!w->in.v[ce->pidx.v[q]].visited) { ok = 0; break; }
        if (ok) VPUSH(w->todo, c);
    }
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
/* per-item tracker on an implicit treap                                                      */
/* ------------------------------------------------------------------------------------------ */
typedef struct { int l, r, p; u32 prio; int cnt, vis, up; } TNode;   /* up: items never deleted */
typedef struct {
    const dto_oplog *o;
    TNode *t; int root;
    u32 *state;          /* per LV (insert items): 0 NIY, 1 inserted, k>=2 deleted k-1 times */
    u8 *ever_deleted;
    i64 *ol, *orr;       /* origin_left / origin_right per insert LV (ROOT=-1, END=-2) */
    i64 *del_target;     /* per delete LV */
    i64 n_items;
    i64 xf;              /* transformed position of the last applied LV (-1: DeleteAlreadyHappened) */
    u64 rng;
    int err;
    /* stats */
    i64 n_retreat, n_advance, n_steps, n_scans;
} Tracker;

#define END_LV (-2)
static inline int tcnt(Tracker *T, int x) { return x < 0 ? 0 : T->t[x].cnt; }
static inline int tvis(Tracker *T, int x) { return x < 0 ? 0 : T->t[x].vis; }
static inline int isvis(Tracker *T, int x) { return T->state[x] == 1; }
static inline int tup(Tracker *T, int x) { return x < 0 ? 0 : T->t[x].up; }
static void tupd(Tracker *T, int x) {
    TNode *n = &T->t[x];
    n->cnt = 1 + tcnt(T, n->l) + tcnt(T, n->r);
    n->vis = isvis(T, x) + tvis(T, n->l) + tvis(T, n->r);
    n->up = !T->ever_deleted[x] + tup(T, n->l) + tup(T, n->r);
    if (n->l >= 0) T->t[n->l].p = x;
    if (n->r >= 0) T->t[n->r].p = x;
}
static int tmerge(Tracker *T, int a, int b) {
    if (a < 0) return b;
    if (b < 0) return a;
    if (T->t[a].prio > T->t[b].prio) { T->t[a].r = tmerge(T, T->t[a].r, b); tupd(T, a); return a; }
    T->t[b].l = tmerge(T, a, T->t[b].l); tupd(T, b); return b;
}
static void tsplit(Tracker *T, int x, int k, int *L, int *R) {   /* first k items -> L */
    if (x < 0) { *L = *R = -1; return; }
    if (tcnt(T, T->t[x].l) >= k) { int a, b; tsplit(T, T->t[x].l, k, &a, &b); T->t[x].l = b; tupd(T, x); *L = a; *R = x; }
    else { int a, b; tsplit(T, T->t[x].r, k - tcnt(T, T->t[x].l) - 1, &a, &b); T->t[x].r = a; tupd(T, x); *L = x; *R = b; }
}
static int trank(Tracker *T, int x) {   /* index of x in document order */
    int r = tcnt(T, T->t[x].l);
    while (T->t[x].p >= 0) { int p = T->t[x].p; if (T->t[p].r == x) r += tcnt(T, T->t[p].l) + 1; x = p; }
    return r;
}
/* upstream position of x: never-deleted items before it (MarkerMetrics upstream_len,
 * metrics.rs:18-66; upstream_cursor_pos) */
static int tuprank(Tracker *T, int x) {
    int r = tup(T, T->t[x].l);
    while (T->t[x].p >= 0) { int p = T->t[x].p; if (T->t[p].r == x) r += tup(T, T->t[p].l) + !T->ever_deleted[p]; x = p; }
    return r;
}
static int tfind_vis(Tracker *T, i64 p) {   /* the item holding visible index p */
    int x = T->root;
    while (x >= 0) {
        int lv = tvis(T, T->t[x].l);
        if (p < lv) x = T->t[x].l;
        else if (p == lv && isvis(T, x)) return x;
        else { p -= lv + isvis(T, x); x = T->t[x].r; }
    }
    return -1;
}
static int tat(Tracker *T, int k) {   /* item at document index k */
    int x = T->root;
    while (x >= 0) {
        int lc = tcnt(T, T->t[x].l);
        if (k < lc) x = T->t[x].l; else if (k == lc) return x; else { k -= lc + 1; x = T->t[x].r; }
    }
    return -1;
}
static void tfix_up(Tracker *T, int x) { while (x >= 0) { tupd(T, x); x = T->t[x].p; } }
static u32 xrand(Tracker *T) { T->rng ^= T->rng << 13; T->rng ^= T->rng >> 7; T->rng ^= T->rng << 17; return (u32)(T->rng >> 11); }

/* agent name compare then seq (merge.rs:199-218) */
static int tie_new_first(Tracker *T, i64 new_lv, i64 other_lv) {
    const AgentRun *a = arun_find(T->o, new_lv), *b = arun_find(T->o, other_lv);
    const Agent *an = &T->o->agents.v[a->agent], *bn = &T->o->agents.v[b->agent];
    int ml = an->name_len < bn->name_len ? an->name_len : bn->name_len;
    int c = memcmp(an->name, bn->name, (size_t)ml);
    if (c == 0) c = an->name_len < bn->name_len ? -1 : an->name_len > bn->name_len;
    if (c < 0) return 1;
    if (c > 0) return 0;
    i64 sa = a->seq_start + (new_lv - a->lv_start), sb = b->seq_start + (other_lv - b->lv_start);
    return sa < sb;
}
static i64 rank_left(Tracker *T, i64 ol) { return ol == ROOT_LV ? -1 : trank(T, (int)ol); }
static i64 rank_right(Tracker *T, i64 orr) { return orr == END_LV ? T->n_items : trank(T, (int)orr); }

/* M2Tracker::apply for one insert LV (merge.rs:383-455) + integrate (merge.rs:154-278) */
static void apply_ins(Tracker *T, i64 lv, i64 pos) {
    i64 origin_left; int cur;   /* cur = document index of the cursor */
    if (pos == 0) { origin_left = ROOT_LV; cur = 0; }
    else {
        int x = tfind_vis(T, pos - 1);
        if (x < 0) { T->err = E_CheckoutPanic; return; }
        origin_left = x; cur = trank(T, x) + 1;
    }
    /* origin_right: first item at/after cursor not in NIY state (may be deleted) */
    i64 origin_right = END_LV; int k = cur, total = tcnt(T, T->root);
    for (; k < total; k++) { int x = tat(T, k); if (T->state[x] != 0) { origin_right = x; break; } }
    int ins_at = cur;
    if (k > cur) {   /* NIY items between cursor and origin_right: YjsMod integrate */
        T->n_scans++;
        i64 my_left = rank_left(T, origin_left), my_right = rank_right(T, origin_right);
        int scanning = 0, scan_start = cur, c = cur;
        for (; c < total; c++) {
            int o = tat(T, c);
            if ((i64)o == origin_right) break;
            i64 ol = rank_left(T, T->ol[o]);
            if (ol < my_left) break;
            if (ol == my_left) {
                if (T->orr[o] == origin_right) {
                    if (tie_new_first(T, lv, o)) break;
                    scanning = 0;
                } else {
                    if (rank_right(T, T->orr[o]) < my_right) { if (!scanning) { scanning = 1; scan_start = c; } }
                    else scanning = 0;
                }
            }
        }
        ins_at = scanning ? scan_start : c;
    }
    T->state[lv] = 1; T->ol[lv] = origin_left; T->orr[lv] = origin_right;
    TNode *n = &T->t[lv]; n->l = n->r = n->p = -1; n->prio = xrand(T); n->cnt = 1; n->vis = 1; n->up = 1;
    int L, R; tsplit(T, T->root, ins_at, &L, &R);
    T->root = tmerge(T, tmerge(T, L, (int)lv), R);
    T->t[T->root].p = -1;
    T->n_items++;
    T->xf = tuprank(T, (int)lv);   /* integrate's ins_pos (merge.rs:154-278) */
}
/* M2Tracker::apply for one delete LV (merge.rs:457-556) */
static void apply_del(Tracker *T, i64 lv, i64 pos) {
    int x = tfind_vis(T, pos);
    if (x < 0 || T->state[x] != 1) { T->err = E_CheckoutPanic; return; }
    T->xf = T->ever_deleted[x] ? -1 : tuprank(T, x);   /* BaseMoved(del_start_xf) / DeleteAlreadyHappened */
    T->state[x] = 2; T->ever_deleted[x] = 1; T->del_target[lv] = x;
    tfix_up(T, x);
}
/* advance_by_range / retreat_by_range per LV (advance_retreat.rs:58-153, yjsspan.rs:49-90) */
static void advance_lv(Tracker *T, i64 lv) {
    T->n_advance++;
    if (T->o->kind.v[lv] == 0) { if (T->state[lv] != 0) { T->err = E_CheckoutPanic; return; } T->state[lv] = 1; tfix_up(T, (int)lv); }
    else { i64 x = T->del_target[lv]; if (T->state[x] == 0) { T->err = E_CheckoutPanic; return; }
           T->state[x]++; T->ever_deleted[x] = 1; tfix_up(T, (int)x); }
}
static void retreat_lv(Tracker *T, i64 lv) {
    T->n_retreat++;
    if (T->o->kind.v[lv] == 0) { if (T->state[lv] != 1) { T->err = E_CheckoutPanic; return; } T->state[lv] = 0; tfix_up(T, (int)lv); }
    else { i64 x = T->del_target[lv]; if (T->state[x] < 2) { T->err = E_CheckoutPanic; return; }
           T->state[x]--; tfix_up(T, (int)x); }
}

typedef struct { i64 n_steps, n_retreat, n_advance, n_scans, n_items; } dto_stats;

static void inorder(Tracker *T, int x, const dto_oplog *o, u8 *out, size_t *n) {
    /* iterative in-order traversal */
    int *stack = malloc(sizeof(int) * (size_t)(T->n_items + 1)); int sp = 0;
    while (x >= 0 || sp) {
        while (x >= 0) { stack[sp++] = x; x = T->t[x].l; }
        x = stack[--sp];
        if (!T->ever_deleted[x]) {
            i64 b = o->cbyte.v[x]; size_t cl = utf8_char_len(o->ins_content.v[b]);
            memcpy(out + *n, &o->ins_content.v[b], cl); *n += cl;
        }
        x = T->t[x].r;
    }
    free(stack);
}

/* ListOpLog::checkout(version) -> text (src/list/oplog.rs:32-36; checkout_tip = version
 * cg.version).  order: 0 = spanning-tree walk (the reference's), 1 = plain LV order (a second
 * topological order, for the convergence check of SURVEY.md §8c). */
EXPORT int dto_checkout(const dto_oplog *o, const i64 *version, int nv, int order, u8 **out, size_t *out_len, dto_stats *stats) {
    i64 n = o->kind.n;
    VecRange hist = {0}, none = {0};
    graph_diff_rev(&o->g, version, nv, NULL, 0, &hist, &none);   /* Hist(version), descending */
    for (i64 i = 0, j = hist.n - 1; i < j; i++, j--) { Range t = hist.v[i]; hist.v[i] = hist.v[j]; hist.v[j] = t; }
    for (i64 i = 0; i < hist.n; i++)
        for (i64 v = hist.v[i].start; v < hist.v[i].end; v++)
            if (o->kind.v[v] == 0 && o->cbyte.v[v] < 0) { VFREE(hist); VFREE(none); return E_CheckoutPanic; }  /* content.unwrap() */
    Tracker T; memset(&T, 0, sizeof T);
    T.o = o; T.root = -1; T.rng = 0x9E3779B97F4A7C15ull;
    T.t = malloc(sizeof(TNode) * (size_t)(n + 1));
    T.state = calloc((size_t)n + 1, sizeof(u32));
    T.ever_deleted = calloc((size_t)n + 1, 1);
    T.ol = malloc(sizeof(i64) * (size_t)(n + 1)); T.orr = malloc(sizeof(i64) * (size_t)(n + 1));
    T.del_target = malloc(sizeof(i64) * (size_t)(n + 1));
    Walker w; WalkStep st; memset(&st, 0, sizeof st);
    walker_init(&w, &o->g, hist.v, hist.n);
    VecI64 cur = {0};       /* for order 1 */
    i64 next_entry = 0;
    for (;;) {
        Range consume;
        if (order == 0) {
            if (!walker_next(&w, &st)) break;
            consume = st.consume;
        } else {
            if (next_entry >= w.in.n) break;
            const VisitEntry *ve = &w.in.v[next_entry++];
            graph_diff_rev(&o->g, cur.v, (int)cur.n, ve->parents, ve->np, &st.retreat, &st.advance_rev);
            consume.start = ve->start; consume.end = ve->end;
            cur.n = 0; VPUSH(cur, ve->end - 1);
        }
        T.n_steps++;
        for (i64 i = 0; i < st.retreat.n && !T.err; i++)
            for (i64 v = st.retreat.v[i].end - 1; v >= st.retreat.v[i].start && !T.err; v--) retreat_lv(&T, v);
        for (i64 i = st.advance_rev.n - 1; i >= 0 && !T.err; i--)
            for (i64 v = st.advance_rev.v[i].start; v < st.advance_rev.v[i].end && !T.err; v++) advance_lv(&T, v);
        for (i64 v = consume.start; v < consume.end && !T.err; v++) {
            if (o->kind.v[v] == 0) apply_ins(&T, v, o->pos.v[v]); else apply_del(&T, v, o->pos.v[v]);
        }
        if (T.err) break;
    }
    int err = T.err;
    if (!err) {
        size_t cap = (size_t)o->ins_content.n + 1, len = 0;
        u8 *buf = malloc(cap);
        inorder(&T, T.root, o, buf, &len);
        *out = buf; *out_len = len;
    }
    if (stats) { stats->n_steps = T.n_steps; stats->n_retreat = T.n_retreat; stats->n_advance = T.n_advance;
                 stats->n_scans = T.n_scans; stats->n_items = T.n_items; }
    walker_free(&w);
    VFREE(st.retreat); VFREE(st.advance_rev); VFREE(cur); VFREE(hist); VFREE(none);
    free(T.t); free(T.state); free(T.ever_deleted); free(T.ol); free(T.orr); free(T.del_target);
    return err;
}
EXPORT int dto_checkout_tip(const dto_oplog *o, int order, u8 **out, size_t *out_len, dto_stats *stats) {
    return dto_checkout(o, o->version.v, (int)o->version.n, order, out, out_len, stats);
}
EXPORT void dto_free_buf(u8 *p) { free(p); }
/* The reference's fast-forward path for a linear history (TransformedOpsIter::next while
 * `can_ff`, src/listmerge/merge.rs:811-840; ListBranch::merge applies each op at its original
 * position to the rope, src/list/merge.rs:68-89): when every graph entry's parents are the LV
 * just before it, checkout_tip needs no tracker -- the ops are applied in LV order to a gap
 * buffer of code points.  Any other history takes the per-item tracker (dto_checkout_tip).
 * Used as the CPU baseline for linear traces (BASELINE configs[0], automerge-paper); parity
 * against dto_checkout_tip is tested on every linear fixture.  *ff = 1 when the FF path ran. */
static u32 utf8_decode(const u8 *s) {
    if (s[0] < 0x80) return s[0];
    if ((s[0] & 0xE0) == 0xC0) return ((u32)(s[0] & 0x1F) << 6) | (s[1] & 0x3F);
    if ((s[0] & 0xF0) == 0xE0) return ((u32)(s[0] & 0x0F) << 12) | ((u32)(s[1] & 0x3F) << 6) | (s[2] & 0x3F);
    return ((u32)(s[0] & 0x07) << 18) | ((u32)(s[1] & 0x3F) << 12) | ((u32)(s[2] & 0x3F) << 6) | (s[3] & 0x3F);
}
static size_t utf8_encode(u32 c, u8 *o) {
    if (c < 0x80) { o[0] = (u8)c; return 1; }
    if (c < 0x800) { o[0] = (u8)(0xC0 | (c >> 6)); o[1] = (u8)(0x80 | (c & 0x3F)); return 2; }
    if (c < 0x10000) { o[0] = (u8)(0xE0 | (c >> 12)); o[1] = (u8)(0x80 | ((c >> 6) & 0x3F)); o[2] = (u8)(0x80 | (c & 0x3F)); return 3; }
    o[0] = (u8)(0xF0 | (c >> 18)); o[1] = (u8)(0x80 | ((c >> 12) & 0x3F)); o[2] = (u8)(0x80 | ((c >> 6) & 0x3F)); o[3] = (u8)(0x80 | (c & 0x3F));
    return 4;
}
EXPORT int dto_checkout_tip_ff(const dto_oplog *o, u8 **out, size_t *out_len, int *ff) {
    const i64 n = o->kind.n;
    int linear = o->version.n == (n ? 1 : 0) && (n == 0 || o->version.v[0] == n - 1);
    for (i64 i = 0; i < o->g.e.n && linear; i++) {
        const GEntry *e = &o->g.e.v[i];
        if (e->start == 0 ? e->np != 0 : (e->np != 1 || e->parents[0] != e->start - 1)) linear = 0;
    }
    for (i64 v = 0; v < n && linear; v++) if (o->kind.v[v] == 0 && o->cbyte.v[v] < 0) linear = 0;
    *ff = linear;
    if (!linear) return dto_checkout_tip(o, 0, out, out_len, NULL);
    /* gap buffer: [0, gs) text before the gap, [ge, cap) text after it */
    i64 cap = 16;
    for (i64 v = 0; v < n; v++) cap += o->kind.v[v] == 0;
    u32 *buf = malloc(sizeof(u32) * (size_t)cap);
    i64 gs = 0, ge = cap;
    for (i64 v = 0; v < n; v++) {
        const i64 p = o->pos.v[v], len = gs + (cap - ge);
        if (p < 0 || p > len || (o->kind.v[v] == 1 && p >= len)) { free(buf); return E_CheckoutPanic; }
        if (p < gs) { memmove(buf + ge - (gs - p), buf + p, sizeof(u32) * (size_t)(gs - p)); ge -= gs - p; gs = p; }
        else if (p > gs) { memmove(buf + gs, buf + ge, sizeof(u32) * (size_t)(p - gs)); ge += p - gs; gs = p; }
        if (o->kind.v[v] == 0) buf[gs++] = utf8_decode(&o->ins_content.v[o->cbyte.v[v]]);
        else ge++;
    }
    u8 *t = malloc((size_t)(4 * (gs + cap - ge) + 1));
    size_t k = 0;
    for (i64 i = 0; i < gs; i++) k += utf8_encode(buf[i], t + k);
    for (i64 i = ge; i < cap; i++) k += utf8_encode(buf[i], t + k);
    free(buf);
    *out = t; *out_len = k;
    return E_OK;
}

/* ListOpLog::iter_xf_operations_from(from, merging) (src/list/merge.rs:24-38) restated per LV,
 * in the TransformedOpsIter order (src/listmerge/merge.rs:618-940): the new ops are
 * Hist(merging) - Hist(from); fast-forward through them while the next op's parents are the
 * current frontier (whole graph entries, :792-835), then a SpanningTreeWalker over the rest
 * starting at that frontier.  The tracker first replays Hist(from) (not emitted), so every item
 * the branch at `from` holds is in it; a transformed position is the upstream position of the
 * inserted item / of the deleted item (-1: the delete already happened).  out receives
 * (lv, xf) pairs in application order; *n_out their count. */
static void walk_apply(Tracker *T, const Graph *g, const Range *spans, i64 nspans, VecI64 *front, i64 *out, i64 *k) {
    Walker w; WalkStep st; memset(&st, 0, sizeof st);
    walker_init(&w, g, spans, nspans);
    for (i64 q = 0; q < front->n; q++) VPUSH(w.frontier, front->v[q]);   /* SpanningTreeWalker::new(.., start_at) */
    while (!T->err && walker_next(&w, &st)) {
        for (i64 i = 0; i < st.retreat.n && !T->err; i++)
            for (i64 v = st.retreat.v[i].end - 1; v >= st.retreat.v[i].start && !T->err; v--) retreat_lv(T, v);
        for (i64 i = st.advance_rev.n - 1; i >= 0 && !T->err; i--)
            for (i64 v = st.advance_rev.v[i].start; v < st.advance_rev.v[i].end && !T->err; v++) advance_lv(T, v);
        for (i64 v = st.consume.start; v < st.consume.end && !T->err; v++) {
            if (T->o->kind.v[v] == 0) apply_ins(T, v, T->o->pos.v[v]); else apply_del(T, v, T->o->pos.v[v]);
            if (out) { out[2 * *k] = v; out[2 * *k + 1] = T->xf; }
            (*k)++;
        }
    }
    front->n = 0;
    for (i64 q = 0; q < w.frontier.n; q++) VPUSH(*front, w.frontier.v[q]);
    walker_free(&w);
    VFREE(st.retreat); VFREE(st.advance_rev);
}
static void ascending(VecRange *r) {
    for (i64 i = 0, j = r->n - 1; i < j; i++, j--) { Range t = r->v[i]; r->v[i] = r->v[j]; r->v[j] = t; }
}
EXPORT int dto_xf_operations_from(const dto_oplog *o, const i64 *from, int nf, const i64 *merge, int nm,
                                  i64 *out, i64 *n_out) {
    i64 n = o->kind.n;
    *n_out = 0;
    for (int i = 0; i < nf; i++) if (from[i] < 0 || from[i] >= n) return E_CheckoutPanic;
    for (int i = 0; i < nm; i++) if (merge[i] < 0 || merge[i] >= n) return E_CheckoutPanic;
    Tracker T; memset(&T, 0, sizeof T);
    T.o = o; T.root = -1; T.rng = 0x9E3779B97F4A7C15ull;
    T.t = malloc(sizeof(TNode) * (size_t)(n + 1));
    T.state = calloc((size_t)n + 1, sizeof(u32));
    T.ever_deleted = calloc((size_t)n + 1, 1);
    T.ol = malloc(sizeof(i64) * (size_t)(n + 1)); T.orr = malloc(sizeof(i64) * (size_t)(n + 1));
    T.del_target = malloc(sizeof(i64) * (size_t)(n + 1));
    VecRange hist = {0}, newr = {0}, none = {0}, ra = {0}, rb = {0};
    VecI64 front = {0};
    i64 k = 0, warm = 0;
    graph_diff_rev(&o->g, from, nf, NULL, 0, &hist, &none);       /* Hist(from) */
    graph_diff_rev(&o->g, merge, nm, from, nf, &newr, &none);     /* new ops: Hist(merge) - Hist(from) */
    ascending(&hist); ascending(&newr);
    for (i64 i = 0; i < hist.n; i++) for (i64 v = hist.v[i].start; v < hist.v[i].end; v++)
        if (o->kind.v[v] == 0 && o->cbyte.v[v] < 0) T.err = E_CheckoutPanic;
    for (i64 i = 0; i < newr.n; i++) for (i64 v = newr.v[i].start; v < newr.v[i].end; v++)
        if (o->kind.v[v] == 0 && o->cbyte.v[v] < 0) T.err = E_CheckoutPanic;
    /* the branch at `from`: replay its history, then sit exactly at `from` */
    if (!T.err && hist.n) walk_apply(&T, &o->g, hist.v, hist.n, &front, NULL, &warm);
    if (!T.err) {
        graph_diff_rev(&o->g, front.v, (int)front.n, from, nf, &ra, &rb);
        for (i64 i = 0; i < ra.n && !T.err; i++)
            for (i64 v = ra.v[i].end - 1; v >= ra.v[i].start && !T.err; v--) retreat_lv(&T, v);
        for (i64 i = rb.n - 1; i >= 0 && !T.err; i--)
            for (i64 v = rb.v[i].start; v < rb.v[i].end && !T.err; v++) advance_lv(&T, v);
        front.n = 0;
        for (int i = 0; i < nf; i++) VPUSH(front, from[i]);
    }
    /* fast-forward: consume up to the end of the entry while its parents are the frontier */
    i64 si = 0;
    while (!T.err && si < newr.n) {
        i64 s0 = newr.v[si].start;
        i64 gi = graph_find_idx(&o->g, s0);
        const GEntry *e = &o->g.e.v[gi];
        i64 p1 = s0 - 1; const i64 *par = &p1; int np = 1;    /* clone_parents_at_version */
        if (s0 == e->start) { par = e->parents; np = e->np; }
        if (np != front.n) break;
        int same = 1; for (int q = 0; q < np; q++) if (par[q] != front.v[q]) same = 0;
        if (!same) break;
        i64 s1 = e->end < newr.v[si].end ? e->end : newr.v[si].end;
        for (i64 v = s0; v < s1 && !T.err; v++) {
            if (o->kind.v[v] == 0) apply_ins(&T, v, o->pos.v[v]); else apply_del(&T, v, o->pos.v[v]);
            out[2 * k] = v; out[2 * k + 1] = T.xf; k++;
        }
        front.n = 0; VPUSH(front, s1 - 1);
        newr.v[si].start = s1;
        if (s1 == newr.v[si].end) si++;
    }
    if (!T.err && si < newr.n) walk_apply(&T, &o->g, newr.v + si, newr.n - si, &front, out, &k);
    int err = T.err;
    *n_out = k;
    VFREE(front); VFREE(hist); VFREE(newr); VFREE(none); VFREE(ra); VFREE(rb);
    free(T.t); free(T.state); free(T.ever_deleted); free(T.ol); free(T.orr); free(T.del_target);
    return err;
}
/* ListOpLog::iter_xf_operations() (src/list/merge.rs:40-48): from ROOT to the tip. */
EXPORT int dto_xf_operations(const dto_oplog *o, i64 *out) {
    i64 k = 0;
    int err = dto_xf_operations_from(o, NULL, 0, o->version.v, (int)o->version.n, out, &k);
    if (!err && k != o->kind.n) err = E_CheckoutPanic;
    return err;
}

/* Decoded arrays, for the element-by-element check of the product's decoders against this
 * independent restatement (tests/test_decode_parity.py).  Each returns the element count and
 * copies min(count, cap) elements.
 *   dto_export_lv:      3 x i64 per LV: kind (0 ins, 1 del), position, content byte offset (-1)
 *   dto_export_aruns:   4 x i64 per agent run: lv_start, len, agent, seq_start
 *   dto_export_entries: 3 x i64 per graph entry: start, end, parent count; parents in *par
 *   dto_export_version: the frontier
 *   dto_agent_name:     bytes of agent i's name */
EXPORT i64 dto_export_lv(const dto_oplog *o, i64 *out, i64 cap) {
    for (i64 v = 0; v < o->kind.n && v < cap; v++) {
        out[3 * v] = o->kind.v[v]; out[3 * v + 1] = o->pos.v[v]; out[3 * v + 2] = o->cbyte.v[v];
    }
    return o->kind.n;
}
EXPORT i64 dto_export_aruns(const dto_oplog *o, i64 *out, i64 cap) {
    for (i64 i = 0; i < o->aruns.n && i < cap; i++) {
        const AgentRun *r = &o->aruns.v[i];
        out[4 * i] = r->lv_start; out[4 * i + 1] = r->len; out[4 * i + 2] = r->agent; out[4 * i + 3] = r->seq_start;
    }
    return o->aruns.n;
}
EXPORT i64 dto_export_entries(const dto_oplog *o, i64 *out, i64 cap, i64 *par, i64 par_cap) {
    i64 k = 0;
    for (i64 i = 0; i < o->g.e.n; i++) {
        const GEntry *e = &o->g.e.v[i];
        if (i < cap) { out[3 * i] = e->start; out[3 * i + 1] = e->end; out[3 * i + 2] = e->np; }
        for (int j = 0; j < e->np; j++, k++) if (k < par_cap) par[k] = e->parents[j];
    }
    return o->g.e.n;
}
EXPORT i64 dto_export_version(const dto_oplog *o, i64 *out, i64 cap) {
    for (i64 i = 0; i < o->version.n && i < cap; i++) out[i] = o->version.v[i];
    return o->version.n;
}
EXPORT int dto_agent_name(const dto_oplog *o, int i, char *out, int cap) {
    if (i < 0 || i >= o->agents.n) return -1;
    const Agent *a = &o->agents.v[i];
    memcpy(out, a->name, (size_t)(a->name_len < cap ? a->name_len : cap));
    return a->name_len;
}
EXPORT const u8 *dto_ins_content(const dto_oplog *o) { return o->ins_content.v; }

/* ------------------------------------------------------------------------------------------ */
/* graph-tool entry points for the causal_graph fixtures                                      */
/* ------------------------------------------------------------------------------------------ */
EXPORT Graph *dto_graph_new(void) { return calloc(1, sizeof(Graph)); }
EXPORT void dto_graph_free(Graph *g) { graph_free(g); free(g); }
EXPORT void dto_graph_push(Graph *g, const i64 *parents, int np, i64 start, i64 end) {
    i64 *p = malloc(sizeof(i64) * (size_t)(np ? np : 1));
    memcpy(p, parents, sizeof(i64) * (size_t)np); sort_frontier(p, np);
    graph_push(g, p, np, start, end);
    free(p);
}
EXPORT int dto_graph_num_entries(const Graph *g) { return (int)g->e.n; }
EXPORT void dto_graph_entry(const Graph *g, int i, i64 *start, i64 *end, i64 *shadow) {
    *start = g->e.v[i].start; *end = g->e.v[i].end; *shadow = g->e.v[i].shadow;
}
/* diff (ascending ranges, Graph::diff tools.rs:158-163). out_a/out_b: pairs; returns counts */
EXPORT void dto_graph_diff(const Graph *g, const i64 *a, int na, const i64 *b, int nb,
                           i64 *out_a, int *n_a, i64 *out_b, int *n_b) {
    VecRange ra = {0}, rb = {0};
    graph_diff_rev(g, a, na, b, nb, &ra, &rb);
    *n_a = (int)ra.n; *n_b = (int)rb.n;
    for (i64 i = 0; i < ra.n; i++) { out_a[2 * i] = ra.v[ra.n - 1 - i].start; out_a[2 * i + 1] = ra.v[ra.n - 1 - i].end; }
    for (i64 i = 0; i < rb.n; i++) { out_b[2 * i] = rb.v[rb.n - 1 - i].start; out_b[2 * i + 1] = rb.v[rb.n - 1 - i].end; }
    VFREE(ra); VFREE(rb);
}
EXPORT int dto_graph_contains(const Graph *g, const i64 *f, int n, i64 target) {
    if (target == ROOT_LV) return 1;   /* version_contains_time: ROOT is in every version */
    return frontier_contains_version(g, f, n, target);
}
/* Graph::find_dominators_2 / find_dominators (tools.rs:505-578) restated by its definition, not
 * its heap walk: the members of a u b that are in the history of no other member, ascending.
 * Returns the count; out holds them. */
EXPORT int dto_graph_dominators(const Graph *g, const i64 *a, int na, const i64 *b, int nb, i64 *out) {
    i64 u[128];
    int n = 0;
    for (int i = 0; i < na && n < 128; i++) u[n++] = a[i];
    for (int i = 0; i < nb && n < 128; i++) u[n++] = b[i];
    sort_frontier(u, n);
    int m = 0;
    for (int i = 0; i < n; i++) if (!m || u[m - 1] != u[i]) u[m++] = u[i];
    int k = 0;
    for (int i = 0; i < m; i++) {
        int dominated = 0;
        for (int j = i + 1; j < m && !dominated; j++) dominated = frontier_contains_version(g, &u[j], 1, u[i]);
        if (!dominated) out[k++] = u[i];
    }
    return k;
}
typedef struct { i64 *spans; int n; } ConfCtx;
static void conf_visit(void *ctx, i64 s, i64 e, int flag) {
    ConfCtx *c = ctx;   /* push_rev_rle of the test harness (tools.rs:745-752) */
    if (c->n && c->spans[3 * (c->n - 1) + 2] == flag && c->spans[3 * (c->n - 1)] == e) { c->spans[3 * (c->n - 1)] = s; return; }
    c->spans[3 * c->n] = s; c->spans[3 * c->n + 1] = e; c->spans[3 * c->n + 2] = flag; c->n++;
}
/* returns the number of (start,end,flag) triples in descending order; common frontier out */
EXPORT int dto_graph_find_conflicting(const Graph *g, const i64 *a, int na, const i64 *b, int nb,
                                      i64 *spans, i64 *common, int *n_common) {
    ConfCtx c = { spans, 0 };
    *n_common = find_conflicting(g, a, na, b, nb, conf_visit, &c, common);
    return c.n;
}
