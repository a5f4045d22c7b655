// dt_encoder.hip -- batched `.dt` encoder: ListOpLog::encode(ENCODE_FULL / ENCODE_PATCH) from ROOT
// (src/list/encoding/encode_oplog.rs:404-747), one 64-lane wavefront per document.
//
// Inputs stay where the device-staged batch left them: the decoded oplog in the decoder's arenas
// (agent runs, entries + parents, content + per-LV byte offsets, agent names in the document
// bytes) and the walk -- Graph::optimized_txns_between(ROOT, tip), the SpanningTreeWalker order the
// planner already produced for the checkout: its INS / DEL commands are the op runs of each entry
// in walk order.  Output bytes equal dt_encode.cpp's (the host encoder) for the same options.
//
//   A  walk       lane-parallel: each command's entry (bisection), entry starts in walk order,
//                 every entry's output position (prefix sums)
//   B  records    the reference's run mergers, which are sequential state machines: agent
//                 assignment (encode_oplog.rs:142-189), ops (op_metrics.rs:235-293) and txns
//                 (graph/mod.rs:239-254) -- the gathers are lane-parallel per 64 items, the merge
//                 decisions a wave-uniform loop over registers (readlane), one record store per run
//   C  sizes      lane-parallel: each record's varint bytes, prefix sums -> every chunk's length
//   D  text       the inserted content in walk order (one lane per op run)
//   E  LZ4        lz4_flex 0.10's greedy parse (see dt_encode.cpp lz4_block_compress) with 64
//                 probe positions per step: a probe's candidate is the last earlier probe of the
//                 same hash in the step, else the table (LDS); the first matching probe ends the
//                 step and only probes up to it enter the table; backtrack / extend 64 bytes at a time
//   F  write      chunk headers (one lane), records serialised lane-parallel at final offsets
//   G  CRC-32C    64 lane segments combined (as in dt_decode.hip)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dt_encoder.hpp"
#include "dt_device.hpp"

namespace dtgpu {
namespace enc {

#define DEV __device__ __forceinline__

DEV uint32_t lane() { return __lane_id(); }
DEV uint32_t rdl(uint32_t v, uint32_t l) { return uint32_t(__builtin_amdgcn_readlane(int(v), int(l))); }
DEV uint64_t ballot(bool p) { return __ballot(p); }
DEV uint64_t lt_mask() { return (1ull << lane()) - 1ull; }
DEV uint32_t popc(uint64_t m) { return uint32_t(__popcll(m)); }
DEV uint32_t ctz(uint64_t m) { return uint32_t(__ffsll((unsigned long long)m) - 1); }
DEV void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }
// inclusive prefix sum over the wave (all lanes active): DPP row scans, then row_bcast 15 / 31
DEV uint32_t scan_incl(uint32_t v) {
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xf, 0xf, false));   // row_shr:1
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xf, 0xf, false));   // row_shr:2
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xf, 0xf, false));   // row_shr:4
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xf, 0xf, false));   // row_shr:8
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false));   // row_bcast:15
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false));   // row_bcast:31
    return v;
}
DEV uint32_t wave_sum(uint32_t v) { return uint32_t(__builtin_amdgcn_readlane(int(scan_incl(v)), 63)); }

// wave-wide byte copy, eight loads in flight per lane before their stores
DEV void copy_bytes(uint8_t *dst, const uint8_t *src, uint32_t n) {
    uint32_t i = lane();
    for (; i + 7 * 64 < n; i += 8 * 64) {
        uint8_t v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = src[i + 64 * k];
#pragma unroll
        for (int k = 0; k < 8; k++) dst[i + 64 * k] = v[k];
    }
    for (; i < n; i += 64) dst[i] = src[i];
}

// ---- varints (leb.rs) ---------------------------------------------------------------------------
DEV uint32_t leb_len(uint64_t v) {
    uint32_t n = 1;
    while (v >= 0x80) { v >>= 7; n++; }
    return n;
}
DEV uint32_t put_leb(uint8_t *d, uint64_t v) {
    uint32_t n = 0;
    while (v >= 0x80) { d[n++] = uint8_t(v | 0x80); v >>= 7; }
    d[n++] = uint8_t(v);
    return n;
}
DEV uint64_t zz_old(int64_t v) { return (uint64_t(v < 0 ? -v : v) << 1) | (v < 0 ? 1u : 0u); }
DEV uint32_t utf8_len(uint8_t c) { return c < 0x80 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : 4; }

constexpr uint32_t CRC_POLY = 0x82F63B78u;
constexpr uint32_t ST_OK = 0, ST_CHECKOUT = 64, ST_CAPACITY = 65;
constexpr uint32_t C_LZ4 = 5, C_FILEINFO = 1, C_DOCID = 2, C_AGENTNAMES = 3, C_STARTBRANCH = 10, C_CONTENT = 13,
                   C_CONTENTCOMP = 14, C_PATCHES = 20, C_OPVERSIONS = 21, C_OPTYPEPOS = 22, C_OPPARENTS = 23,
                   C_PATCHCONTENT = 24, C_CONTENTKNOWN = 25, C_CRC = 100;

DEV uint32_t entry_of(const uint2 *ent, uint32_t ne, uint32_t lv) {   // Graph::find_packed
    uint32_t lo = 0, hi = ne;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (ent[m].y <= lv) lo = m + 1; else hi = m;
    }
    return lo;
}
DEV uint32_t arun_of(const uint4 *ar, uint32_t n, uint32_t lv) {   // last run with ar.lv <= lv
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (ar[m].x <= lv) lo = m + 1; else hi = m;
    }
    return lo ? lo - 1 : 0;
}

// ---- CRC-32C (zlib's crc32_combine scheme over the reflected polynomial) ------------------------
DEV uint32_t multmodp(uint32_t a, uint32_t b) {
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
DEV uint32_t x2nmodp(const uint32_t *x2n, uint64_t n, uint32_t k) {
    uint32_t p = 1u << 31;
    while (n) {
        if (n & 1) p = multmodp(x2n[k & 31], p);
        n >>= 1;
        k++;
    }
    return p;
}
// s must be 16-byte aligned: each lane's segment is a multiple of 16 bytes, read as uint4 words
// with the next word in flight while the current one goes through the table
DEV uint32_t crc_word(uint32_t c, uint32_t w, const uint32_t *T) {
    c ^= w;
    c = T[c & 0xFFu] ^ (c >> 8);
    c = T[c & 0xFFu] ^ (c >> 8);
    c = T[c & 0xFFu] ^ (c >> 8);
    return T[c & 0xFFu] ^ (c >> 8);
}
DEV uint32_t crc32c_par(const uint8_t *s, uint32_t n, const uint32_t *T, const uint32_t *x2n) {
    const uint32_t S = ((n + 63) / 64 + 15) & ~15u;
    const uint32_t b0 = lane() * S;
    const uint32_t e0 = b0 < n ? min(b0 + S, n) : b0;
    uint32_t c = ~0u;
    uint32_t i = b0;
    if (i + 16 <= e0) {
        const uint4 *w = reinterpret_cast<const uint4 *>(s + i);
        uint4 cur = w[0];
        for (uint32_t k = 1;; k++) {
            const bool more = i + 32 <= e0;
            const uint4 nxt = more ? w[k] : cur;
            c = crc_word(c, cur.x, T);
            c = crc_word(c, cur.y, T);
            c = crc_word(c, cur.z, T);
            c = crc_word(c, cur.w, T);
            i += 16;
            if (!more) break;
            cur = nxt;
        }
    }
    for (; i < e0; i++) c = T[(c ^ s[i]) & 0xFFu] ^ (c >> 8);
    c = ~c;
    if (e0 <= b0) c = 0;
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

// ---- LZ4 (lz4_flex 0.10 compress_into, restated in dt_encode.cpp) -----------------------------
DEV uint32_t ld32(const uint8_t *p) {
    return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}
DEV uint64_t ld64(const uint8_t *p) { return uint64_t(ld32(p)) | (uint64_t(ld32(p + 4)) << 32); }

// sum_{i < x} (i >> 5): the miss loop's probe offsets in closed form (step = nmc >> 5, nmc += 1)
DEV uint64_t probe_sum(uint64_t x) {
    const uint64_t q = x >> 5, r = x & 31;
    return 16 * q * (q - (q ? 1 : 0)) + r * q;
}

typedef __attribute__((address_space(3))) uint16_t LDS16;
typedef __attribute__((address_space(3))) uint32_t LDS32;

constexpr uint32_t LZ_RING = 512;   // LDS staging of the compressed bytes (flushed to HBM)

struct Lz {
    const uint8_t *in;   // the text: LDS or HBM (one address space per instantiation site)
    uint8_t *out;        // HBM
    uint8_t *ring;       // LDS, LZ_RING bytes
    uint32_t n, o, f;    // text length, bytes emitted, bytes flushed
    bool small, prof;
    uint32_t st[4];      // profile: probe steps, steps with shared hashes, sequences, -
    uint64_t cyc[3];     // profile: cycles in probing, extending, emitting
    uint32_t *tab;   // LDS: 8,192 u16 (small) or 4,096 u32
    DEV uint32_t hash(uint32_t p) const {
        if (small) return (ld32(in + p) * 2654435761u) >> 19;
        return uint32_t(((ld64(in + p) << 24) * 889523592379ull) >> 52);
    }
    // volatile LDS (address space 3) accesses: ds ops that are never forwarded or merged
    DEV uint32_t vget(uint32_t h) const {
        return small ? uint32_t(((volatile LDS16 *)tab)[h]) : ((volatile LDS32 *)tab)[h];
    }
    DEV void vput(uint32_t h, uint32_t v) {
        if (small) ((volatile LDS16 *)tab)[h] = uint16_t(v);
        else ((volatile LDS32 *)tab)[h] = v;
    }
    // the output goes through the LDS ring, so the parse never waits on HBM stores (vmcnt)
    DEV void flush() {
        for (uint32_t i = f + lane(); i < o; i += 64) out[i] = ring[i & (LZ_RING - 1)];
        f = o;
    }
    DEV void reserve(uint32_t k) {   // k <= 128
        if (o + k - f > LZ_RING) flush();
    }
    DEV void put1(uint8_t v) {
        reserve(1);
        if (lane() == 0) ring[o & (LZ_RING - 1)] = v;
        o++;
    }
    DEV void ext(uint32_t v) {   // 255-run length extension
        const uint32_t nb = v / 255 + 1;
        for (uint32_t x = 0; x < nb; x += 64) {
            const uint32_t k = min(64u, nb - x);
            reserve(k);
            if (lane() < k) ring[(o + lane()) & (LZ_RING - 1)] = x + lane() + 1 < nb ? 255 : uint8_t(v - 255 * (nb - 1));
            o += k;
        }
    }
    // emit() with the (<= 64) literals already in registers: lane j holds in[l0 + j]
    DEV void emit_lits(uint32_t l0, uint32_t l1, uint32_t lb, uint32_t off, uint32_t mlen) {
        const uint32_t ll = l1 - l0;
        put1(uint8_t((min(ll, 15u) << 4) | min(mlen - 4, 15u)));
        if (ll >= 15) ext(ll - 15);
        reserve(ll);
        if (lane() < ll) ring[(o + lane()) & (LZ_RING - 1)] = uint8_t(lb);
        o += ll;
        put1(uint8_t(off));
        put1(uint8_t(off >> 8));
        if (mlen - 4 >= 15) ext(mlen - 19);
    }
    DEV void emit(uint32_t l0, uint32_t l1, uint32_t off, uint32_t mlen) {
        const uint32_t ll = l1 - l0;
        put1(uint8_t((min(ll, 15u) << 4) | (off ? min(mlen - 4, 15u) : 0u)));
        if (ll >= 15) ext(ll - 15);
        for (uint32_t x = 0; x < ll; x += 64) {
            const uint32_t k = min(64u, ll - x);
            reserve(k);
            if (lane() < k) ring[(o + lane()) & (LZ_RING - 1)] = in[l0 + x + lane()];
            o += k;
        }
        if (!off) return;
        put1(uint8_t(off));
        put1(uint8_t(off >> 8));
        if (mlen - 4 >= 15) ext(mlen - 19);
    }
    DEV uint32_t run() {
        o = f = 0;
        small = n < 65535;
        st[0] = st[1] = st[2] = st[3] = 0;
        cyc[0] = cyc[1] = cyc[2] = 0;
        uint64_t tc = prof ? clock64() : 0;
        auto tick = [&](int k) {
            if (prof) { const uint64_t t = clock64(); cyc[k] += t - tc; tc = t; }
        };
        for (uint32_t i = lane(); i < 4096; i += 64) tab[i] = 0;
        if (n < 13) { emit(0, n, 0, 0); flush(); return o; }
        const uint32_t end_check = n - 12, match_lim = n - 6;
        uint32_t lit = 0, cur = 1;   // position 0 is hashed first: its entry is the table's zero
        const uint32_t l = lane();
        for (;;) {
            uint32_t nmc = 32, pos = cur, cand = 0;
            bool found = false;
            // probes of the miss loop: 16 in the first step (a match is usually a few bytes
            // away: fewer shared hashes to resolve), 64 in later ones
            for (uint32_t width = 16;; width = 64) {
                const uint64_t base = probe_sum(nmc);
                const uint32_t p = pos + uint32_t(probe_sum(nmc + l) - base);
                const bool valid = l < width && p <= end_check;
                const uint32_t nv = popc(ballot(valid));   // valid probes form a prefix
                const uint32_t h = valid ? hash(p) : 0xFFFFFFFFu;
                const uint32_t w32 = valid ? ld32(in + p) : 0u;
                // every probe writes its position into its slot and reads the slot back: when
                // each probe won its own slot, no two probes share a hash and the table held
                // every candidate (volatile: the read-back must see the other lanes' writes)
                const uint32_t old = valid ? vget(h) : 0u;
                const uint32_t cw = valid ? ld32(in + old) : 0u;   // in flight across the slot check
                if (valid) vput(h, p);
                const bool won = !valid || vget(h) == p;
                uint32_t c, lim;
                uint64_t m;
                st[0]++;
                if (!ballot(!won)) {
                    c = old;
                    const bool ok = valid && p - c <= 65535u && cw == w32;
                    m = ballot(ok);
                    lim = m ? ctz(m) + 1 : nv;
                    if (valid && l >= lim) vput(h, old);   // probes past the match never ran
                } else {   // shared hashes: a probe's candidate is the last earlier probe of its hash
                    st[1]++;
                    if (valid) vput(h, old);
                    // one ballot per contested hash: each group lost at least one slot write
                    uint64_t lost = ballot(!won);
                    int prevj = -1;
                    uint32_t nextj = 64;
                    while (lost) {
                        const uint32_t hj = rdl(h, ctz(lost));
                        const bool mine = valid && h == hj;
                        const uint64_t g = ballot(mine);
                        if (mine) {
                            const uint64_t below = g & lt_mask(), above = g & ~lt_mask() & ~(1ull << l);
                            prevj = below ? int(63 - __clzll((long long)below)) : -1;
                            nextj = above ? ctz(above) : 64;
                        }
                        lost &= ~g;
                    }
                    const uint32_t pp = uint32_t(__shfl(int(p), prevj < 0 ? int(l) : prevj));
                    c = prevj >= 0 ? pp : old;
                    const bool ok = valid && p - c <= 65535u && (prevj >= 0 ? ld32(in + c) : cw) == w32;
                    m = ballot(ok);
                    lim = m ? ctz(m) + 1 : nv;
                    if (l < lim && nextj >= lim) vput(h, p);   // the last probe of each hash wins
                }
                if (m) {
                    cur = rdl(p, lim - 1);
                    cand = rdl(c, lim - 1);
                    found = true;
                    break;
                }
                if (nv < width) break;   // past len - 12: the tail is literals
                pos += uint32_t(probe_sum(nmc + width) - base);
                nmc += width;
            }
            tick(0);
            if (!found) { emit(lit, n, 0, 0); flush(); return o; }
            st[2]++;
            // one round of loads serves the usual sequence: 64 bytes before the match (backwards
            // extension), 64 after its first four (forwards extension: independent of how far
            // the backwards one goes, since the backtracked bytes match) and the pending literals
            const uint32_t cur0 = cur, cand0 = cand;
            const uint32_t mb0 = min(cur - lit, cand);
            const bool bok = l < mb0, fok = cur + 4 + l < match_lim, lok = lit + l < cur;
            const uint32_t bx = bok ? in[cur - 1 - l] : 0u, by = bok ? in[cand - 1 - l] : 1u;
            const uint32_t fx = fok ? in[cur + 4 + l] : 0u, fy = fok ? in[cand + 4 + l] : 1u;
            const uint32_t lb = lok ? in[lit + l] : 0u;
            {
                const uint64_t x = ballot(bx != by);
                uint32_t b = x ? ctz(x) : 64;
                cur -= b;
                cand -= b;
                while (b == 64) {   // extend backwards over the pending literals
                    const uint32_t mb = min(cur - lit, cand);
                    const bool eq = l < mb && in[cur - 1 - l] == in[cand - 1 - l];
                    const uint64_t y = ballot(!eq);
                    b = y ? ctz(y) : 64;
                    cur -= b;
                    cand -= b;
                }
            }
            const uint32_t m0 = cur, off = cur - cand;
            {
                const uint64_t x = ballot(fx != fy);
                uint32_t b = x ? ctz(x) : 64;
                cur = cur0 + 4 + b;
                cand = cand0 + 4 + b;
                while (b == 64) {   // extend forwards up to len - 6
                    const bool eq = cur + l < match_lim && in[cur + l] == in[cand + l];
                    const uint64_t y = ballot(!eq);
                    b = y ? ctz(y) : 64;
                    cur += b;
                    cand += b;
                }
            }
            const uint32_t h2 = hash(cur - 2);
            if (l == 0) vput(h2, cur - 2);
            tick(1);
            if (m0 - lit <= 64) emit_lits(lit, m0, lb, off, cur - m0);
            else emit(lit, m0, off, cur - m0);
            lit = cur;
            tick(2);
        }
    }
};

// ---- op runs: write_op (encode_oplog.rs:20-92); the ListOpMetrics merge (op_metrics.rs:235-293)
// is in encode_records_kernel
// the varint head of a written op run and its optional diff; op_end is the next cursor
DEV void op_code(uint4 r, uint32_t cursor, uint64_t &n, int64_t &diff, bool &has_diff, uint32_t &op_end) {
    const uint32_t start = r.x, end = r.y, len = end - start;
    const bool del = r.z & 1u, fwd = (r.z & 2u) || len == 1;
    const uint32_t op_start = (del && !fwd) ? end : start;
    op_end = (!del && fwd) ? end : start;
    diff = int64_t(op_start) - int64_t(cursor);
    uint64_t v;
    if (len != 1) v = del ? (uint64_t(len) * 2 + (fwd ? 1 : 0)) : len;
    else v = diff != 0 ? zz_old(diff) : 0;
    v = v * 2 + (del ? 1 : 0);
    v = v * 2 + (diff != 0 ? 1 : 0);
    v = v * 2 + (len != 1 ? 1 : 0);
    n = v;
    has_diff = len != 1 && diff != 0;
}

struct Layout {   // byte offsets of the streams in the output
    uint32_t aa, ops, tx, names, text, known, lz, total;
};

// tx_record(t, dst): txn t's bytes (len, then parents as output-order distances, all local from
// ROOT); dst == nullptr counts them
#define ENC_TX_RECORD \
    auto tx_record = [&](uint32_t t, uint32_t ntx_, uint8_t *dst) -> uint32_t { \
        const uint32_t e = worder[heads[t]]; \
        const uint32_t out0 = outpos[e]; \
        const uint32_t nxt = t + 1 < ntx_ ? outpos[worder[heads[t + 1]]] : D.n_lv; \
        uint32_t nb = dst ? put_leb(dst, nxt - out0) : leb_len(nxt - out0); \
        const uint32_t p0 = poff[e], np = poff[e + 1] - p0; \
        if (np == 0) { \
            if (dst) dst[nb] = 1; \
            return nb + 1; \
        } \
        for (uint32_t j = 0; j < np; j++) { \
            const uint32_t p = par[p0 + j]; \
            const uint32_t pe = min(entry_of(ent, ne, p), ne - 1); \
            const uint32_t mp = outpos[pe] + (p - ent[pe].x); \
            const uint64_t v = (uint64_t(out0 - mp) * 2 + (j + 1 < np ? 1 : 0)) * 2; \
            nb += dst ? put_leb(dst + nb, v) : leb_len(v); \
        } \
        return nb; \
    }; \
    do {} while (0);

// Kernel 1: A walk, B records, C sizes, D text -- small LDS (the agent map), high occupancy.
__global__ __launch_bounds__(64) void encode_records_kernel(EncParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t doc = blockIdx.x;
    if (doc >= P.n_docs) return;
    const EncDesc D = P.docs[doc];
    EncResult R{};
    if (D.skip) return;
    const uint32_t l = lane();
    uint64_t t_prev = P.prof ? clock64() : 0;
    auto mark = [&](int i) {
        if (P.prof) { const uint64_t t = clock64(); R.prof[i] = t - t_prev; t_prev = t; }
    };
    uint32_t *amap = lds;                    // agent -> mapped id (0: not yet), max_agents
    uint32_t *alast = amap + P.max_agents;   // agent -> end of its last seq range written
    for (uint32_t i = l; i < D.n_agents; i += 64) { amap[i] = 0; alast[i] = 0; }
#define ENC_UNUSED (void)in; (void)lzb; (void)out; (void)compress; (void)store_text;
    const uint8_t *in = P.in + D.in_off;
    const uint4 *ar = reinterpret_cast<const uint4 *>(P.aruns) + D.arun_off;
    const uint2 *ent = reinterpret_cast<const uint2 *>(P.ent) + D.ent_off;
    const uint32_t *poff = P.poff + D.poff_off, *par = P.par + D.par_off;
    const uint8_t *content = P.content + D.content_off;
    const uint32_t *cbyte = P.cbyte + D.lv_off;
    const uint2 *names = reinterpret_cast<const uint2 *>(P.agents) + D.agent_off;
    const Cmd *cmds = P.cmds + D.cmd_off;
    const uint32_t ne = D.ne, ncmd = D.ncmd;
    uint32_t *worder = P.w + D.w_off, *outpos = worder + ne;
    uint32_t *oprec = outpos + ne;                          // 8 words per op run
    uint32_t *aarec = oprec + 8ull * ncmd;                  // 4 words per agent run
    uint32_t *heads = aarec + 4ull * (D.n_aruns + ne);      // walk index of each txn head
    uint32_t *ainv = heads + ne;                            // mapped id - 1 -> agent
    uint8_t *text = P.b + D.b_off, *lzb = text + D.n_content;
    uint8_t *out = P.out + D.out_off;
    const bool store_text = P.flags & 1u, compress = P.flags & 2u;
    ENC_TX_RECORD
    ENC_UNUSED
    // ---- A: the walk ---------------------------------------------------------------------------
    uint32_t nw = 0, opos = 0;
    for (uint32_t c0 = 0; c0 < ncmd; c0 += 64) {
        const uint32_t c = c0 + l;
        uint32_t e = 0, len = 0;
        bool starts = false;
        if (c < ncmd) {
            const Cmd cm = cmds[c];
            if ((cm.op & 15u) != CMD_TOG) {
                e = entry_of(ent, ne, cm.lv);
                if (e < ne) {
                    const uint2 se = ent[e];
                    starts = se.x == cm.lv;
                    len = se.y - se.x;
                }
            }
        }
        const uint64_t m = ballot(starts);
        if (!starts) len = 0;
        const uint32_t incl = scan_incl(len);
        if (starts && nw + popc(m & lt_mask()) < ne) {
            worder[nw + popc(m & lt_mask())] = e;
            outpos[e] = opos + incl - len;
        }
        nw += popc(m);
        opos += rdl(incl, 63);
    }
    if (nw != ne || opos != D.n_lv) {
        if (l == 0) { R.status = ST_CHECKOUT; P.results[doc] = R; }
        return;
    }
    wave_fence();
    mark(0);

    // ---- B: records ------------------------------------------------------------------------------
    // txn heads: an entry continues the previous txn when it follows it directly with that txn's
    // last LV as its only parent (tx_push; GraphEntrySimple::can_append)
    uint32_t ntx = 0, carry_end = 0xFFFFFFFFu;
    for (uint32_t k0 = 0; k0 < ne; k0 += 64) {
        const uint32_t k = k0 + l;
        uint2 se = make_uint2(0, 0);
        uint32_t np = 0, p0v = 0;
        if (k < ne) {
            const uint32_t e = worder[k];
            se = ent[e];
            const uint32_t p0 = poff[e];
            np = poff[e + 1] - p0;
            if (np == 1) p0v = par[p0];
        }
        const uint32_t prev_end_l = uint32_t(__shfl_up(int(se.y), 1));
        const uint32_t prev_end = l == 0 ? carry_end : prev_end_l;
        const bool merge = k > 0 && se.x == prev_end && np == 1 && p0v + 1 == se.x;
        const bool head = k < ne && !merge;
        const uint64_t m = ballot(head);
        if (head) heads[ntx + popc(m & lt_mask())] = k;
        ntx += popc(m);
        carry_end = rdl(se.y, 63);
    }
    mark(6);
    // agent assignment runs (encode_oplog.rs:142-189, AgentMapping :191-240).  A piece is an agent
    // run clipped to a walk entry; it continues the previous piece's run when it has the same
    // (file) agent and no seq jump -- a pairwise test once each piece knows its agent's mapped id
    // and the end of that agent's previous piece.  Those come from one ballot per distinct agent
    // among 64 pieces (first use assigns the next id, as AgentMapping::map does).  An entry
    // spanning more than four agent runs sends its 64 entries down the sequential path.
    uint32_t n_mapped = 0, naa = 0;    // naa: runs started so far (the open run is naa - 1)
    bool ay = false;                   // an open run: agent, seq jump, length
    uint32_t aA = 0, aL = 0;
    int32_t aJ = 0;
    auto aa_store = [&](uint32_t idx, uint32_t a, int32_t d, uint32_t len) {
        uint32_t *w = aarec + 4 * idx;
        w[0] = a; w[1] = uint32_t(d); w[2] = len;
    };
    uint32_t *pb = alast + P.max_agents;   // LDS: up to 256 pieces (agent, seq, len) of 64 entries
    for (uint32_t k0 = 0; k0 < ne; k0 += 64) {
        const uint32_t k = k0 + l;
        // each lane gathers its entry's first four agent runs
        uint32_t s = 0, e_end = 0, ai = 0;
        uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0, q2 = q0, q3 = q0;
        const uint32_t na = D.n_aruns;
        uint32_t npk = 0;
        bool over = false;
        if (k < ne) {
            const uint2 se = ent[worder[k]];
            s = se.x; e_end = se.y;
            ai = arun_of(ar, na, s);
            q0 = ar[ai];
            if (ai + 1 < na) q1 = ar[ai + 1];
            if (ai + 2 < na) q2 = ar[ai + 2];
            if (ai + 3 < na) q3 = ar[ai + 3];
            npk = 1;
            if (q0.x + q0.y < e_end && ai + 1 < na) npk = 2;
            if (npk == 2 && q1.x + q1.y < e_end && ai + 2 < na) npk = 3;
            if (npk == 3 && q2.x + q2.y < e_end && ai + 3 < na) npk = 4;
            over = npk == 4 && q3.x + q3.y < e_end && ai + 4 < na;
        }
        if (ballot(over)) {   // the sequential path for these 64 entries
            uint32_t cur_agent = 0xFFFFFFFFu, cur_mapped = 0, cur_last = 0;
            const uint32_t nk = min(64u, ne - k0);
            for (uint32_t j = 0; j < nk; j++) {
                const uint32_t js = rdl(s, j), je = rdl(e_end, j);
                uint32_t i = rdl(ai, j);
                uint4 r = make_uint4(rdl(q0.x, j), rdl(q0.y, j), rdl(q0.z, j), rdl(q0.w, j));
                for (uint32_t u = 1;; u++) {
                    const uint32_t x = max(r.x, js), y = min(r.x + r.y, je);
                    if (x < y) {
                        const uint32_t agent = r.z;
                        if (agent != cur_agent) {
                            if (cur_agent != 0xFFFFFFFFu && l == 0) alast[cur_agent] = cur_last;
                            cur_agent = agent;
                            cur_mapped = amap[agent];
                            cur_last = alast[agent];
                            if (!cur_mapped) {
                                cur_mapped = ++n_mapped;
                                if (l == 0) { amap[agent] = cur_mapped; ainv[cur_mapped - 1] = agent; }
                            }
                        }
                        const uint32_t s0 = r.w + (x - r.x);
                        const int32_t d = int32_t(s0 - cur_last);
                        cur_last = s0 + (y - x);
                        if (ay && aA == cur_mapped && d == 0) {
                            aL += y - x;
                        } else {
                            if (ay && l == 0) aa_store(naa - 1, aA, aJ, aL);
                            naa++;
                            ay = true; aA = cur_mapped; aJ = d; aL = y - x;
                        }
                    }
                    if (r.x + r.y >= je || ++i >= na) break;
                    if (u < 4) {
                        const uint4 v = u == 1 ? q1 : u == 2 ? q2 : q3;
                        r = make_uint4(rdl(v.x, j), rdl(v.y, j), rdl(v.z, j), rdl(v.w, j));
                    } else {
                        r = ar[i];
                    }
                }
            }
            if (cur_agent != 0xFFFFFFFFu && l == 0) alast[cur_agent] = cur_last;
            continue;
        }
        // pieces in walk order into LDS
        const uint32_t pincl = scan_incl(npk);
        const uint32_t np = rdl(pincl, 63);
        {
            uint32_t at = pincl - npk;
            for (uint32_t u = 0; u < npk; u++, at++) {
                const uint4 r = u == 0 ? q0 : u == 1 ? q1 : u == 2 ? q2 : q3;
                const uint32_t x = max(r.x, s), y = min(r.x + r.y, e_end);
                pb[3 * at] = r.z; pb[3 * at + 1] = r.w + (x - r.x); pb[3 * at + 2] = y - x;
            }
        }
        wave_fence();
        for (uint32_t j0 = 0; j0 < np; j0 += 64) {
            const uint32_t j = j0 + l;
            const bool valid = j < np;
            const uint32_t A = valid ? pb[3 * j] : 0xFFFFFFFFu, S0 = valid ? pb[3 * j + 1] : 0;
            const uint32_t LN = valid ? pb[3 * j + 2] : 0, endv = S0 + LN;
            uint32_t MA = 0, PE = 0;
            for (uint64_t todo = ballot(valid); todo;) {   // one round per distinct agent
                const uint32_t lead = rdl(A, ctz(todo));
                const bool mine = valid && A == lead;
                const uint64_t g = ballot(mine);
                uint32_t m = amap[lead];
                const uint32_t last = alast[lead];
                if (!m) {
                    m = ++n_mapped;
                    if (l == 0) { amap[lead] = m; ainv[m - 1] = lead; }
                }
                const uint64_t gb = g & lt_mask();
                const int pe = gb ? int(63 - __clzll((long long)gb)) : int(l);
                const uint32_t pv = uint32_t(__shfl(int(endv), pe));
                if (mine) { MA = m; PE = gb ? pv : last; }
                const uint32_t newlast = rdl(endv, 63 - uint32_t(__clzll((long long)g)));
                if (l == 0) alast[lead] = newlast;
                todo &= ~g;
            }
            const int32_t d = int32_t(S0 - PE);
            const uint32_t prevA = uint32_t(__shfl_up(int(MA), 1));
            const bool pexist = l > 0 ? true : ay;
            const uint32_t pA = l > 0 ? prevA : aA;
            const bool head = valid && !(pexist && pA == MA && d == 0);
            const uint64_t hm = ballot(head);
            const uint64_t vm = ballot(valid);
            if ((hm & 1ull) && ay && l == 0) aa_store(naa - 1, aA, aJ, aL);   // the open run ends here
            // run of each piece: index, head fields, length so far
            const uint32_t lincl = scan_incl(valid ? LN : 0u);
            const uint64_t hle = hm & (lt_mask() | (1ull << l));
            const int h = hle ? int(63 - __clzll((long long)hle)) : -1;
            const int hsrc = h >= 0 ? h : int(l);
            const uint32_t HA = uint32_t(__shfl(int(MA), hsrc)), Hpre = uint32_t(__shfl(int(lincl - LN), hsrc));
            const int32_t HJ = __shfl(d, hsrc);
            const uint32_t Hidx = naa + uint32_t(__shfl(int(popc(hm & lt_mask())), hsrc));
            const bool last_in_run = valid && (l == 63 ? false : ((vm >> (l + 1)) & 1) && ((hm >> (l + 1)) & 1));
            if (last_in_run) {
                if (h >= 0) aa_store(Hidx, HA, HJ, lincl - Hpre);
                else aa_store(naa - 1, aA, aJ, aL + lincl);
            }
            // carry the open run: the last piece's run
            const uint32_t t = 63 - uint32_t(__clzll((long long)vm));
            const int ht = __shfl(h, int(t));
            if (ht >= 0) {
                aA = rdl(HA, t); aJ = int32_t(rdl(uint32_t(HJ), t)); aL = rdl(lincl - Hpre, t);
            } else {
                aL += rdl(lincl, t);
            }
            ay = true;
            naa += popc(hm);
        }
    }
    if (ay && l == 0) aa_store(naa - 1, aA, aJ, aL);
    mark(7);
    // op runs in walk order (the INS / DEL commands), merged lane-parallel.  can_append /
    // append (op_metrics.rs:235-293) depend on the run so far only through three facts about its
    // last piece P: whether P started the run, P's own (start, end, fwd), and -- when P was
    // appended -- the direction the append gave the run (P.start >= the piece before P's start,
    // for deletes; always forwards for inserts).  So "piece i is appended" is a boolean function of
    // "piece i-1 was appended", one of {0, 1, id, not}: the flags are a prefix composition of those
    // functions (six shuffles per 64 commands), and each run's record is built at its last piece.
    uint32_t nop = 0, n_ins = 0;
    bool cy = false, cM = false;                          // the last piece so far: exists, appended
    uint32_t cS = 0, cE = 0, cF = 0, cD = 0, cC = 0, cC1 = 0, cPS = 0;
    bool oy = false;                                      // the open run (continues into the next chunk)
    uint32_t oS = 0, oD = 0, oC = 0, oC0 = 0, oLen = 0, oIdx = 0;
    auto close_open = [&]() {   // record of the open run, whose last piece is the carried one
        uint32_t st, en, dl, fw, cc = oC;
        if (!cM) { st = cS; en = cE; dl = cD; fw = cF; cc = cC; }
        else if (!oD) { st = oS; en = oS + oLen; dl = 0; fw = 1; }
        else if (cS >= cPS) { st = oS; en = oS + oLen; dl = 1; fw = 1; }
        else { st = cS; en = cS + oLen; dl = 1; fw = 0; }
        if (l == 0) {
            uint32_t *w = oprec + 8ull * oIdx;
            w[0] = st; w[1] = en; w[2] = dl | (fw << 1) | (cc << 2); w[3] = oC0; w[4] = cC1;
        }
        oy = false;
    };
    for (uint32_t c0 = 0; c0 < ncmd; c0 += 64) {
        const uint32_t c = c0 + l;
        bool valid = false;
        uint32_t S = 0, E = 0, D = 0, F = 0, C = 0, C0 = 0, C1 = 0;
        if (c < ncmd) {
            const Cmd cm = cmds[c];
            const uint32_t opc = cm.op & 15u;
            if (opc != CMD_TOG) {
                valid = true;
                S = cm.pos; E = cm.pos + cm.len;
                D = opc == CMD_DEL ? 1u : 0u;
                F = (!D || (cm.op & 16u)) ? 1u : 0u;
                if (!D) {
                    C0 = cbyte[cm.lv];
                    const uint32_t lb = cbyte[cm.lv + cm.len - 1];
                    C1 = lb != 0xFFFFFFFFu ? lb + utf8_len(content[lb]) : 0xFFFFFFFFu;
                    C = C0 != 0xFFFFFFFFu ? 1u : 0u;
                }
            }
        }
        const uint32_t L = E - S;
        if (valid && !D) n_ins += L;
        const uint64_t vm = ballot(valid);
        const uint64_t below = vm & lt_mask();
        const int pi = below ? int(63 - __clzll((long long)below)) : -1;
        const int psrc = pi >= 0 ? pi : int(l);
        uint32_t PS = uint32_t(__shfl(int(S), psrc)), PE = uint32_t(__shfl(int(E), psrc));
        uint32_t PD = uint32_t(__shfl(int(D), psrc)), PF = uint32_t(__shfl(int(F), psrc));
        uint32_t PC = uint32_t(__shfl(int(C), psrc)), PC1 = uint32_t(__shfl(int(C1), psrc));
        const int ppi = __shfl(pi, psrc);
        uint32_t PPS = uint32_t(__shfl(int(S), ppi >= 0 ? ppi : int(l)));
        bool pex = true;
        if (pi < 0) {
            pex = cy;
            PS = cS; PE = cE; PD = cD; PF = cF; PC = cC; PC1 = cC1; PPS = cPS;
        } else if (ppi < 0) {
            PPS = cS;
        }
        const uint32_t PL = PE - PS;
        bool g0 = false, g1 = true;   // identity for TOG lanes
        if (valid) {
            const bool base = pex && PD == D && PC == C && (!C || PC1 == C0);
            if (!D) {
                g0 = g1 = base && S == PE;
            } else {
                const bool bf = L == 1 || F, br = L == 1 || !F;
                const bool af0 = PL == 1 || PF, ar0 = PL == 1 || !PF, fw1 = PS >= PPS;
                g0 = base && ((af0 && bf && S == PS) || (ar0 && br && E == PS));
                g1 = base && ((fw1 && bf && S == PS) || (!fw1 && br && E == PS));
            }
        }
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {   // prefix composition: f_i o ... o f_0
            const bool b0 = __shfl_up(int(g0), d) != 0, b1 = __shfl_up(int(g1), d) != 0;
            if (l >= uint32_t(d)) {
                const bool n0 = b0 ? g1 : g0, n1 = b1 ? g1 : g0;
                g0 = n0; g1 = n1;
            }
        }
        const bool merged = valid && (cy && cM ? g1 : g0);
        const bool head = valid && !merged;
        const uint64_t hm = ballot(head);
        if (vm && oy && ((hm >> ctz(vm)) & 1)) close_open();
        const uint32_t myidx = nop + popc(hm & lt_mask());
        const uint32_t pref = scan_incl(valid ? L : 0u);
        const uint64_t hle = hm & (lt_mask() | (1ull << l));
        const int h = hle ? int(63 - __clzll((long long)hle)) : -1;
        const int hsrc = h >= 0 ? h : int(l);
        const uint32_t HS = uint32_t(__shfl(int(S), hsrc)), HD = uint32_t(__shfl(int(D), hsrc));
        const uint32_t HC = uint32_t(__shfl(int(C), hsrc)), HC0 = uint32_t(__shfl(int(C0), hsrc));
        const uint32_t Hpre = uint32_t(__shfl(int(pref - L), hsrc)), Hidx = uint32_t(__shfl(int(myidx), hsrc));
        const uint64_t above = vm & ~(lt_mask() | (1ull << l));
        const bool last = valid && above && ((hm >> ctz(above)) & 1);
        if (last) {   // this piece ends a run whose next piece heads a new one
            const bool hin = h >= 0;
            const uint32_t total = hin ? pref - Hpre : oLen + pref;
            const uint32_t rS = hin ? HS : oS, rD = hin ? HD : oD, rC = hin ? HC : oC, rC0 = hin ? HC0 : oC0;
            const uint32_t idx = hin ? Hidx : oIdx;
            uint32_t st, en, dl, fw, cc = rC;
            if (!merged) { st = S; en = E; dl = D; fw = F; cc = C; }
            else if (!rD) { st = rS; en = rS + total; dl = 0; fw = 1; }
            else if (S >= PS) { st = rS; en = rS + total; dl = 1; fw = 1; }
            else { st = S; en = S + total; dl = 1; fw = 0; }
            uint32_t *w = oprec + 8ull * idx;
            w[0] = st; w[1] = en; w[2] = dl | (fw << 1) | (cc << 2); w[3] = rC0; w[4] = C1;
        }
        if (vm) {   // carry the chunk's last piece and its open run
            const uint32_t t = 63 - uint32_t(__clzll((long long)vm));
            const int ht = __shfl(h, int(t));
            if (ht >= 0) {
                oy = true;
                oS = rdl(HS, t); oD = rdl(HD, t); oC = rdl(HC, t); oC0 = rdl(HC0, t);
                oLen = rdl(pref - Hpre, t); oIdx = rdl(Hidx, t);
            } else {
                oLen += rdl(pref, t);
            }
            cy = true;
            cS = rdl(S, t); cE = rdl(E, t); cF = rdl(F, t); cD = rdl(D, t); cC = rdl(C, t); cC1 = rdl(C1, t);
            cPS = rdl(PS, t);
            cM = rdl(merged ? 1u : 0u, t) != 0;
        }
        nop += popc(hm);
    }
    if (oy) close_open();
    n_ins = wave_sum(n_ins);
    wave_fence();
    mark(1);

    // ---- C: sizes ----------------------------------------------------------------------------------
    uint32_t aa_bytes = 0, op_bytes = 0, tx_bytes = 0, nm_bytes = 0, text_len = 0;
    for (uint32_t i0 = 0; i0 < naa; i0 += 64) {
        const uint32_t i = i0 + l;
        if (i < naa) {
            const uint32_t *w = aarec + 4 * i;
            const int32_t d = int32_t(w[1]);
            aa_bytes += leb_len(uint64_t(w[0]) * 2 + (d != 0 ? 1 : 0)) + leb_len(w[2]) + (d != 0 ? leb_len(zz_old(d)) : 0);
        }
    }
    aa_bytes = wave_sum(aa_bytes);
    for (uint32_t i0 = 0; i0 < nop; i0 += 64) {
        const uint32_t i = i0 + l;
        if (i < nop) {
            const uint32_t *w = oprec + 8ull * i;
            uint32_t cursor = 0;
            if (i > 0) {
                const uint32_t *pw = w - 8;
                uint64_t n2; int64_t d2; bool h2; op_code(make_uint4(pw[0], pw[1], pw[2], 0), 0, n2, d2, h2, cursor);
            }
            uint64_t n; int64_t d; bool hd; uint32_t oe;
            op_code(make_uint4(w[0], w[1], w[2], 0), cursor, n, d, hd, oe);
            op_bytes += leb_len(n) + (hd ? leb_len(zz_old(d)) : 0);
            if (!(w[2] & 1u) && (w[2] & 4u)) text_len += w[4] - w[3];
        }
    }
    op_bytes = wave_sum(op_bytes);
    text_len = store_text ? wave_sum(text_len) : 0;
    for (uint32_t t0 = 0; t0 < ntx; t0 += 64)
        if (t0 + l < ntx) tx_bytes += tx_record(t0 + l, ntx, nullptr);
    tx_bytes = wave_sum(tx_bytes);
    for (uint32_t i = l; i < n_mapped; i += 64) {
        const uint32_t nl = names[ainv[i]].y;
        nm_bytes += leb_len(nl) + nl;
    }
    nm_bytes = wave_sum(nm_bytes);
    mark(2);

    // ---- D + E: walk-order text, LZ4 ---------------------------------------------------------------
    if (text_len > D.n_content) {
        if (l == 0) { R.status = ST_CHECKOUT; P.results[doc] = R; }
        return;
    }
    if (text_len) {
        uint32_t tpos = 0;
        for (uint32_t i0 = 0; i0 < nop; i0 += 64) {
            const uint32_t i = i0 + l;
            uint32_t tl = 0, c0b = 0;
            if (i < nop) {
                const uint32_t *w = oprec + 8ull * i;
                if (!(w[2] & 1u) && (w[2] & 4u)) { c0b = w[3]; tl = w[4] - w[3]; }
            }
            const uint32_t incl = scan_incl(tl);
            uint8_t *d = text + tpos + incl - tl;
            for (uint32_t x = 0; x < tl; x++) d[x] = content[c0b + x];
            tpos += rdl(incl, 63);
        }
        if (tpos != text_len) {
            if (l == 0) { R.status = ST_CHECKOUT; P.results[doc] = R; }
            return;
        }
    }
    R.status = ST_OK;
    R.n_op_runs = nop;
    R.n_agent_runs = naa;
    R.n_txns = ntx;
    R.text_len = text_len;
    R.n_mapped = n_mapped;
    R.aa_bytes = aa_bytes;
    R.op_bytes = op_bytes;
    R.tx_bytes = tx_bytes;
    R.nm_bytes = nm_bytes;
    R.n_ins = n_ins;
    R.stage = 1;
    if (l == 0) P.results[doc] = R;
}

// Kernel 2: E LZ4 (the text staged in LDS when it fits), F write, G CRC.
__global__ __launch_bounds__(64) void encode_write_kernel(EncParams P) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t doc = blockIdx.x;
    if (doc >= P.n_docs) return;
    const EncDesc D = P.docs[doc];
    if (D.skip) return;
    EncResult R = P.results[doc];
    if (R.status != ST_OK || R.stage != 1) return;
    const uint32_t l = lane();
    uint64_t t_prev = P.prof ? clock64() : 0;
    auto mark = [&](int i) {
        if (P.prof) { const uint64_t t = clock64(); R.prof[i] = t - t_prev; t_prev = t; }
    };
    uint32_t *tab = lds;                     // LZ4 hash table (4,096 words), then the CRC table
    uint8_t *lring = reinterpret_cast<uint8_t *>(lds + 4096);                 // LZ4 output staging
    uint8_t *ltext = reinterpret_cast<uint8_t *>(lds + 4096 + LZ_RING / 4);   // the text, when it fits
    const uint8_t *in = P.in + D.in_off;
    const uint4 *ar = reinterpret_cast<const uint4 *>(P.aruns) + D.arun_off;
    const uint2 *ent = reinterpret_cast<const uint2 *>(P.ent) + D.ent_off;
    const uint32_t *poff = P.poff + D.poff_off, *par = P.par + D.par_off;
    const uint8_t *content = P.content + D.content_off;
    const uint32_t *cbyte = P.cbyte + D.lv_off;
    const uint2 *names = reinterpret_cast<const uint2 *>(P.agents) + D.agent_off;
    const Cmd *cmds = P.cmds + D.cmd_off;
    const uint32_t ne = D.ne, ncmd = D.ncmd;
    uint32_t *worder = P.w + D.w_off, *outpos = worder + ne;
    uint32_t *oprec = outpos + ne;                          // 8 words per op run
    uint32_t *aarec = oprec + 8ull * ncmd;                  // 4 words per agent run
    uint32_t *heads = aarec + 4ull * (D.n_aruns + ne);      // walk index of each txn head
    uint32_t *ainv = heads + ne;                            // mapped id - 1 -> agent
    uint8_t *text = P.b + D.b_off, *lzb = text + D.n_content;
    uint8_t *out = P.out + D.out_off;
    const bool store_text = P.flags & 1u, compress = P.flags & 2u;
    ENC_TX_RECORD
    const uint32_t nop = R.n_op_runs, naa = R.n_agent_runs, ntx = R.n_txns, text_len = R.text_len;
    const uint32_t n_mapped = R.n_mapped, aa_bytes = R.aa_bytes, op_bytes = R.op_bytes, tx_bytes = R.tx_bytes;
    const uint32_t nm_bytes = R.nm_bytes, n_ins = R.n_ins;
    (void)cmds; (void)cbyte; (void)content; (void)ar;
    ENC_UNUSED
    const bool use_lz = compress && text_len >= 20;
    uint32_t lz_len = 0;
    if (use_lz) {
        wave_fence();
        Lz z;
        z.prof = P.prof;
        z.out = lzb;
        z.ring = lring;
        z.n = text_len;
        z.tab = tab;
        if (text_len <= P.lds_text) {   // stage the text in LDS (16-byte copies); ds reads from here on
            const uint4 *g = reinterpret_cast<const uint4 *>(text);
            uint4 *d = reinterpret_cast<uint4 *>(ltext);
            for (uint32_t i = l; i < (text_len + 15) / 16; i += 64) d[i] = g[i];
            z.in = ltext;
            lz_len = z.run();
        } else {
            z.in = text;
            lz_len = z.run();
        }
        if (P.prof) {
            for (int k = 0; k < 3; k++) R.lzcyc[k] = z.cyc[k];
            for (int k = 0; k < 3; k++) R.lzst[k] = z.st[k];
        }
    }
    wave_fence();
    R.lz_len = lz_len;
    mark(3);

    // ---- F: layout and write -----------------------------------------------------------------------
    const bool has_doc_id = D.doc_id_len != 0xFFFFFFFFu;
    const uint32_t lz_body = use_lz ? leb_len(text_len) + lz_len : 0;
    const uint32_t lz_chunk = use_lz ? 1 + leb_len(lz_body) + lz_body : 0;
    const uint32_t docid_body = has_doc_id ? 1 + D.doc_id_len : 0;
    const uint32_t fi_body = (has_doc_id ? 1 + leb_len(docid_body) + docid_body : 0) + 1 + leb_len(nm_bytes) + nm_bytes;
    const uint32_t content_body = use_lz ? 1 + leb_len(text_len) : 1 + text_len;
    const uint64_t known_v = uint64_t(n_ins) * 2 + 1;
    const uint32_t known_body = leb_len(known_v);
    const uint32_t pc_body = 1 + (1 + leb_len(content_body) + content_body) + (1 + leb_len(known_body) + known_body);
    const uint32_t pc_chunk = text_len ? 1 + leb_len(pc_body) + pc_body : 0;
    const uint32_t patches_body = pc_chunk + (1 + leb_len(aa_bytes) + aa_bytes) + (1 + leb_len(op_bytes) + op_bytes) +
                                  (1 + leb_len(tx_bytes) + tx_bytes);
    const uint32_t total = 9 + lz_chunk + (1 + leb_len(fi_body) + fi_body) + 2 + (1 + leb_len(patches_body) + patches_body) + 6;
    if (total > D.out_cap) {
        if (l == 0) { R.status = ST_CAPACITY; P.results[doc] = R; }
        return;
    }
    Layout L;
    uint32_t at = 0;
    if (l == 0) {
        const uint8_t magic[8] = {'D', 'M', 'N', 'D', 'T', 'Y', 'P', 'S'};
        for (int i = 0; i < 8; i++) out[i] = magic[i];
        out[8] = 0;
        at = 9;
        if (use_lz) {
            out[at++] = C_LZ4;
            at += put_leb(out + at, lz_body);
            at += put_leb(out + at, text_len);
        }
    }
    at = 9 + (use_lz ? 1 + leb_len(lz_body) + leb_len(text_len) : 0);
    L.lz = at;
    at += lz_len;
    if (l == 0) {
        uint32_t p = at;
        out[p++] = C_FILEINFO;
        p += put_leb(out + p, fi_body);
        if (has_doc_id) {
            out[p++] = C_DOCID;
            p += put_leb(out + p, docid_body);
            out[p++] = 4;   // DataType::PlainText
        }
    }
    at += 1 + leb_len(fi_body) + (has_doc_id ? 1 + leb_len(docid_body) + 1 : 0);
    const uint32_t docid_at = at;
    at += has_doc_id ? D.doc_id_len : 0;
    if (l == 0) {
        out[at] = C_AGENTNAMES;
        put_leb(out + at + 1, nm_bytes);
    }
    at += 1 + leb_len(nm_bytes);
    L.names = at;
    at += nm_bytes;
    if (l == 0) {
        uint32_t p = at;
        out[p++] = C_STARTBRANCH;
        out[p++] = 0;
        out[p++] = C_PATCHES;
        p += put_leb(out + p, patches_body);
        if (text_len) {
            out[p++] = C_PATCHCONTENT;
            p += put_leb(out + p, pc_body);
            out[p++] = 0;   // Ins
            out[p++] = use_lz ? C_CONTENTCOMP : C_CONTENT;
            p += put_leb(out + p, content_body);
            out[p++] = 4;
            if (use_lz) p += put_leb(out + p, text_len);
        }
    }
    at += 2 + 1 + leb_len(patches_body);
    if (text_len) at += 1 + leb_len(pc_body) + 1 + 1 + leb_len(content_body) + 1 + (use_lz ? leb_len(text_len) : 0);
    L.text = at;
    if (text_len && !use_lz) at += text_len;
    if (text_len) {
        if (l == 0) {
            out[at] = C_CONTENTKNOWN;
            put_leb(out + at + 1, known_body);
            put_leb(out + at + 2, known_v);   // known_body < 128
        }
        at += 2 + known_body;
    }
    if (l == 0) { out[at] = C_OPVERSIONS; put_leb(out + at + 1, aa_bytes); }
    at += 1 + leb_len(aa_bytes);
    L.aa = at;
    at += aa_bytes;
    if (l == 0) { out[at] = C_OPTYPEPOS; put_leb(out + at + 1, op_bytes); }
    at += 1 + leb_len(op_bytes);
    L.ops = at;
    at += op_bytes;
    if (l == 0) { out[at] = C_OPPARENTS; put_leb(out + at + 1, tx_bytes); }
    at += 1 + leb_len(tx_bytes);
    L.tx = at;
    at += tx_bytes;
    L.total = at + 6;
    if (L.total != total) {
        if (l == 0) { R.status = ST_CAPACITY; P.results[doc] = R; }
        return;
    }
    // doc id, LZ4 block or text
    if (has_doc_id)
        for (uint32_t i = l; i < D.doc_id_len; i += 64) out[docid_at + i] = in[D.doc_id_off + i];
    if (use_lz)
        copy_bytes(out + L.lz, lzb, lz_len);
    else if (text_len)
        copy_bytes(out + L.text, text, text_len);
    // names
    {
        uint32_t base = L.names;
        for (uint32_t i0 = 0; i0 < n_mapped; i0 += 64) {
            const uint32_t i = i0 + l;
            uint32_t nb = 0;
            uint2 nmv = make_uint2(0, 0);
            if (i < n_mapped) { nmv = names[ainv[i]]; nb = leb_len(nmv.y) + nmv.y; }
            const uint32_t incl = scan_incl(nb);
            if (i < n_mapped) {
                uint8_t *d = out + base + incl - nb;
                const uint32_t h = put_leb(d, nmv.y);
                for (uint32_t x = 0; x < nmv.y; x++) d[h + x] = in[nmv.x + x];
            }
            base += rdl(incl, 63);
        }
    }
    // agent assignment runs
    {
        uint32_t base = L.aa;
        for (uint32_t i0 = 0; i0 < naa; i0 += 64) {
            const uint32_t i = i0 + l;
            uint32_t nb = 0, ag = 0, ln = 0;
            int32_t d = 0;
            if (i < naa) {
                const uint32_t *w = aarec + 4 * i;
                ag = w[0]; d = int32_t(w[1]); ln = w[2];
                nb = leb_len(uint64_t(ag) * 2 + (d != 0 ? 1 : 0)) + leb_len(ln) + (d != 0 ? leb_len(zz_old(d)) : 0);
            }
            const uint32_t incl = scan_incl(nb);
            if (i < naa) {
                uint8_t *p = out + base + incl - nb;
                uint32_t k = put_leb(p, uint64_t(ag) * 2 + (d != 0 ? 1 : 0));
                k += put_leb(p + k, ln);
                if (d != 0) put_leb(p + k, zz_old(d));
            }
            base += rdl(incl, 63);
        }
    }
    // op runs
    {
        uint32_t base = L.ops;
        for (uint32_t i0 = 0; i0 < nop; i0 += 64) {
            const uint32_t i = i0 + l;
            uint32_t nb = 0;
            uint64_t n = 0;
            int64_t d = 0;
            bool hd = false;
            if (i < nop) {
                const uint32_t *w = oprec + 8ull * i;
                uint32_t cursor = 0, oe;
                if (i > 0) {
                    const uint32_t *pw = w - 8;
                    uint64_t n2; int64_t d2; bool h2; op_code(make_uint4(pw[0], pw[1], pw[2], 0), 0, n2, d2, h2, cursor);
                }
                op_code(make_uint4(w[0], w[1], w[2], 0), cursor, n, d, hd, oe);
                nb = leb_len(n) + (hd ? leb_len(zz_old(d)) : 0);
            }
            const uint32_t incl = scan_incl(nb);
            if (i < nop) {
                uint8_t *p = out + base + incl - nb;
                const uint32_t k = put_leb(p, n);
                if (hd) put_leb(p + k, zz_old(d));
            }
            base += rdl(incl, 63);
        }
    }
    // txns
    {
        uint32_t base = L.tx;
        for (uint32_t t0 = 0; t0 < ntx; t0 += 64) {
            const uint32_t t = t0 + l;
            const uint32_t nb = t < ntx ? tx_record(t, ntx, nullptr) : 0;
            const uint32_t incl = scan_incl(nb);
            if (t < ntx) tx_record(t, ntx, out + base + incl - nb);
            base += rdl(incl, 63);
        }
    }
    wave_fence();
    mark(4);

    // ---- G: CRC chunk --------------------------------------------------------------------------------
    uint32_t *T = tab;
    for (uint32_t i = l; i < 256; i += 64) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ CRC_POLY : c >> 1;
        T[i] = c;
    }
    const uint32_t crc = crc32c_par(out, L.total - 6, T, P.x2n);
    if (l == 0) {
        uint8_t *p = out + L.total - 6;
        p[0] = C_CRC; p[1] = 4;
        p[2] = uint8_t(crc); p[3] = uint8_t(crc >> 8); p[4] = uint8_t(crc >> 16); p[5] = uint8_t(crc >> 24);
    }
    mark(5);
    if (l == 0) {
        R.status = ST_OK;
        R.len = L.total;
        R.n_op_runs = nop;
        R.n_agent_runs = naa;
        R.n_txns = ntx;
        R.text_len = text_len;
        P.results[doc] = R;
    }
}

}  // namespace enc

int launch_encode(const EncParams &p, void *stream) {
    if (!p.n_docs) return OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(enc::encode_records_kernel, dim3(p.n_docs), dim3(64), (2 * size_t(p.max_agents) + 3 * 256) * 4, s, p);
    if (launch_error() != hipSuccess) return ErrHip;
    hipLaunchKernelGGL(enc::encode_write_kernel, dim3(p.n_docs), dim3(64), 4096 * 4 + enc::LZ_RING + size_t(p.lds_text + 15) / 16 * 16, s, p);
    return launch_error() == hipSuccess ? OK : ErrHip;
}

}  // namespace dtgpu
