// dt_host.cpp -- `.dt` decoder, causal graph and walk planner (host side of libdtgpu).
// See dt_host.hpp for the data model.  Reference files are cited per function.
#include "dt_host.hpp"

#include <algorithm>
#include <functional>
#include <cstring>
#include <queue>

namespace dtgpu {

// ------------------------------------------------------------------------------------------
// byte-level primitives
// ------------------------------------------------------------------------------------------
namespace {

// Unsigned LEB128, at most 10 bytes, 10th byte <= 1 (src/list/encoding/leb.rs:113-178).
struct Reader {
    const uint8_t *p = nullptr;
    size_t n = 0;
    bool empty() const { return n == 0; }
    Status varint_at(uint64_t &v, size_t &used) const {
        uint64_t r = 0;
        for (size_t i = 0; i < n; i++) {
            if (i == 10) return InvalidVarInt;
            uint8_t b = p[i];
            if (i == 9 && (b & 0x7f) > 1) return InvalidVarInt;
            r |= uint64_t(b & 0x7f) << (7 * i);
            if (b < 0x80) { v = r; used = i + 1; return OK; }
        }
        return n >= 10 ? InvalidVarInt : UnexpectedEOF;
    }
    Status u64v(uint64_t &v) {
        if (!n) return UnexpectedEOF;
        size_t used;
        Status s = varint_at(v, used);
        if (s) return s;
        p += used; n -= used;
        return OK;
    }
    Status u32v(uint64_t &v) {
        Status s = u64v(v);
        if (s) return s;
        return v >= 0xFFFFFFFFull ? InvalidVarInt : OK;
    }
    Status peek_u32(bool &has, uint64_t &v) const {
        has = false;
        if (!n) return OK;
        size_t used;
        Status s = varint_at(v, used);
        if (s) return s;
        if (v >= 0xFFFFFFFFull) return InvalidVarInt;
        has = true;
        return OK;
    }
    // "old" sign-magnitude zigzag (leb.rs:305-323)
    Status zigzag(int64_t &v) {
        uint64_t u;
        Status s = u64v(u);
        if (s) return s;
        v = int64_t(u >> 1) * ((u & 1) ? -1 : 1);
        return OK;
    }
    Status bytes(size_t k, const uint8_t *&out) {
        if (k > n) return UnexpectedEOF;
        out = p; p += k; n -= k;
        return OK;
    }
};

inline int64_t zigzag_of(uint64_t u) { return int64_t(u >> 1) * ((u & 1) ? -1 : 1); }

enum Chunk : uint64_t {
    C_FileInfo = 1, C_DocId = 2, C_AgentNames = 3, C_UserData = 4, C_LZ4 = 5, C_StartBranch = 10,
    C_Version = 12, C_Content = 13, C_ContentCompressed = 14, C_Patches = 20, C_OpVersions = 21,
    C_OpTypeAndPosition = 22, C_OpParents = 23, C_PatchContent = 24, C_ContentIsKnown = 25, C_Crc = 100,
};
bool chunk_is_known(uint64_t t) {   // ListChunkType (src/list/encoding/mod.rs:26-58)
    switch (t) {
        case 1: case 2: case 3: case 4: case 5: case 10: case 11: case 12: case 13: case 14:
        case 20: case 21: case 22: case 23: case 24: case 25: case 27: case 100: return true;
        default: return false;
    }
}
// ChunkReader (src/list/encoding/decode_tools.rs:185-268)
Status next_chunk(Reader &r, uint64_t &type, Reader &body) {
    for (;;) {
        uint64_t t, len;
        if (Status s = r.u32v(t)) return s;
        if (Status s = r.u64v(len)) return s;
        if (len > r.n) return InvalidLength;
        body.p = r.p; body.n = size_t(len);
        r.p += len; r.n -= len;
        if (chunk_is_known(t)) { type = t; return OK; }
    }
}
Status chunk_if(Reader &r, uint64_t want, bool &found, Reader &body) {
    found = false;
    bool has; uint64_t t;
    if (Status s = r.peek_u32(has, t)) return s;
    if (!has || t != want) return OK;
    uint64_t tt;
    if (Status s = next_chunk(r, tt, body)) return s;
    found = true;
    return OK;
}
Status expect_chunk(Reader &r, uint64_t want, Reader &body) {
    uint64_t t;
    if (Status s = next_chunk(r, t, body)) return s;
    return t == want ? OK : MissingChunk;
}
// expect_content_str (decode_oplog.rs:176-195 / decode_tools.rs:133-144)
Status content_str(Reader &chunks, Reader *comp, const uint8_t *&s, size_t &sn) {
    uint64_t t; Reader c;
    if (Status e = next_chunk(chunks, t, c)) return e;
    if (t != C_Content && t != C_ContentCompressed) return MissingChunk;
    uint64_t dt;
    if (Status e = c.u32v(dt)) return e;
    if (dt != 4) return UnknownChunk;
    if (t == C_Content) {
        if (!utf8_valid(c.p, c.n)) return InvalidUTF8;
        s = c.p; sn = c.n;
        return OK;
    }
    uint64_t len;
    if (Status e = c.u64v(len)) return e;
    if (!comp) return CompressedDataMissing;
    if (Status e = comp->bytes(size_t(len), s)) return e;
    if (!utf8_valid(s, size_t(len))) return InvalidUTF8;
    sn = size_t(len);
    return OK;
}

// ContentIsKnown run iterator (ReadPatchContentIter, decode_oplog.rs:383-425)
struct ContentRuns {
    bool present = false;
    Reader runs;
    const uint8_t *text = nullptr;
    size_t tn = 0;
    // pushed-back remainder
    bool pb = false;
    uint64_t pb_len = 0; bool pb_known = false; const uint8_t *pb_s = nullptr; size_t pb_n = 0;

    Status next(bool &has, uint64_t &len, bool &known, const uint8_t *&s, size_t &sn) {
        if (pb) { pb = false; has = true; len = pb_len; known = pb_known; s = pb_s; sn = pb_n; return OK; }
        if (runs.empty()) {
            if (tn == 0) { has = false; return OK; }
            return UnexpectedEOF;
        }
        uint64_t x;
        if (Status e = runs.u64v(x)) return e;
        len = x >> 1; known = x & 1; s = nullptr; sn = 0;
        if (known) {
            size_t b = 0; uint64_t c = 0;
            while (c < len && b < tn) { b += utf8_len(text[b]); c++; }
            if (b > tn) b = tn;
            if (c != len) return UnexpectedEOF;
            s = text; sn = b; text += b; tn -= b;
        }
        has = true;
        return OK;
    }
};

}  // namespace

bool utf8_valid(const uint8_t *s, size_t n) {
    size_t i = 0;
    while (i < n) {
        uint8_t c = s[i];
        if (c < 0x80) { i++; continue; }
        size_t len; uint32_t cp;
        if ((c & 0xE0) == 0xC0) { len = 2; cp = c & 0x1F; }
        else if ((c & 0xF0) == 0xE0) { len = 3; cp = c & 0x0F; }
        else if ((c & 0xF8) == 0xF0) { len = 4; cp = c & 0x07; }
        else return false;
        if (i + len > n) return false;
        for (size_t k = 1; k < len; k++) {
            if ((s[i + k] & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (s[i + k] & 0x3F);
        }
        if ((len == 2 && cp < 0x80) || (len == 3 && cp < 0x800) || (len == 4 && cp < 0x10000)) return false;
        if (cp > 0x10FFFF || (cp >= 0xD800 && cp <= 0xDFFF)) return false;
        i += len;
    }
    return true;
}

// CRC-32/ISCSI, slicing-by-8 (crc crate CRC_32_ISCSI; src/encoding/tools.rs:111-115)
uint32_t crc32c(const uint8_t *d, size_t n) {
    static uint32_t T[8][256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
            T[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; i++)
            for (int t = 1; t < 8; t++) T[t][i] = (T[t - 1][i] >> 8) ^ T[0][T[t - 1][i] & 0xFF];
        init = true;
    }
    uint32_t c = 0xFFFFFFFFu;
    while (n >= 8) {
        uint64_t w;
        std::memcpy(&w, d, 8);
        w ^= c;
        c = T[7][w & 0xFF] ^ T[6][(w >> 8) & 0xFF] ^ T[5][(w >> 16) & 0xFF] ^ T[4][(w >> 24) & 0xFF] ^
            T[3][(w >> 32) & 0xFF] ^ T[2][(w >> 40) & 0xFF] ^ T[1][(w >> 48) & 0xFF] ^ T[0][w >> 56];
        d += 8; n -= 8;
    }
    while (n--) c = T[0][(c ^ *d++) & 0xFF] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}

// LZ4 raw block (the format lz4_flex::decompress reads; decode_oplog.rs:621-633)
bool lz4_block_decompress(const uint8_t *src, size_t n, uint8_t *dst, size_t out_len) {
    size_t ip = 0, op = 0;
    while (ip < n) {
        const uint8_t tok = src[ip++];
        size_t lit = tok >> 4;
        if (lit == 15) {
            uint8_t b;
            do { if (ip >= n) return false; b = src[ip++]; lit += b; } while (b == 255);
        }
        if (ip + lit > n || op + lit > out_len) return false;
        std::memcpy(dst + op, src + ip, lit);
        ip += lit; op += lit;
        if (ip >= n) break;
        if (ip + 2 > n) return false;
        const size_t off = size_t(src[ip]) | (size_t(src[ip + 1]) << 8);
        ip += 2;
        if (off == 0 || off > op) return false;
        size_t ml = tok & 15;
        if (ml == 15) {
            uint8_t b;
            do { if (ip >= n) return false; b = src[ip++]; ml += b; } while (b == 255);
        }
        ml += 4;
        if (op + ml > out_len) return false;
        if (off >= ml) { std::memcpy(dst + op, dst + op - off, ml); op += ml; }
        else for (size_t k = 0; k < ml; k++, op++) dst[op] = dst[op - off];
    }
    return op == out_len;
}

uint64_t text_hash(const uint8_t *t, size_t n) {
    uint64_t h = 0;
    for (size_t i = 0; i < n; i++) {
        uint64_t z = (uint64_t(i) << 8) | t[i];
        z += 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        h += z ^ (z >> 31);
    }
    return h;
}

// ------------------------------------------------------------------------------------------
// graph (src/causalgraph/graph/mod.rs:85-128, tools.rs:52-292)
// ------------------------------------------------------------------------------------------
int64_t Graph::find_idx(uint64_t lv) const {
    auto it = std::upper_bound(entries.begin(), entries.end(), lv,
                               [](uint64_t v, const GraphEntry &e) { return v < e.end; });
    if (it == entries.end() || lv < it->start) return -1;
    return it - entries.begin();
}

void Graph::push(const std::vector<uint64_t> &parents, uint64_t start, uint64_t end) {
    if (!entries.empty()) {
        GraphEntry &last = entries.back();
        if (parents.size() == 1 && parents[0] == last.end - 1 && last.end == start) { last.end = end; return; }
    }
    uint64_t shadow = start;
    while (shadow >= 1 && std::find(parents.begin(), parents.end(), shadow - 1) != parents.end())
        shadow = entries[size_t(find_idx(shadow - 1))].shadow;
    entries.push_back(GraphEntry{start, end, shadow, parents});
}

namespace {
inline void push_rev(std::vector<std::pair<uint64_t, uint64_t>> &v, uint64_t s, uint64_t e) {
    if (!v.empty() && v.back().first == e) { v.back().first = s; return; }
    v.emplace_back(s, e);
}
}  // namespace

void Graph::diff_rev(const std::vector<uint64_t> &a, const std::vector<uint64_t> &b,
                     std::vector<std::pair<uint64_t, uint64_t>> &oa,
                     std::vector<std::pair<uint64_t, uint64_t>> &ob) const {
    oa.clear(); ob.clear();
    if (a == b) return;
    if (a.size() == 1 && b.size() == 1) {   // is_direct_descendant_coarse fast paths
        const uint64_t x = a[0], y = b[0];
        if (x > y && y >= entries[size_t(find_idx(x))].start) { push_rev(oa, y + 1, x + 1); return; }
        if (y > x && x >= entries[size_t(find_idx(y))].start) { push_rev(ob, x + 1, y + 1); return; }
    }
    enum : uint8_t { A = 0, B = 1, S = 2 };
    // max-heap on (lv, flag) as BinaryHeap<(LV, DiffFlag)>
    std::priority_queue<std::pair<uint64_t, uint8_t>> q;
    for (uint64_t v : a) q.emplace(v, A);
    for (uint64_t v : b) q.emplace(v, B);
    int64_t shared = 0;
    auto mark = [&](uint64_t s, uint64_t e_incl, uint8_t f) {
        if (f == A) push_rev(oa, s, e_incl + 1);
        else if (f == B) push_rev(ob, s, e_incl + 1);
    };
    while (!q.empty()) {
        auto [ord, flag] = q.top();
        q.pop();
        if (flag == S) shared--;
        while (!q.empty() && q.top().first == ord) {
            if (q.top().second != flag) flag = S;
            if (q.top().second == S) shared--;
            q.pop();
        }
        const GraphEntry &e = entries[size_t(find_idx(ord))];
        while (!q.empty() && q.top().first >= e.start) {
            auto pk = q.top();
            if (pk.second != flag) {
                mark(pk.first + 1, ord, flag);
                ord = pk.first;
                flag = S;
            }
            if (pk.second == S) shared--;
            q.pop();
        }
        mark(e.start, ord, flag);
        for (uint64_t p : e.parents) { q.emplace(p, flag); if (flag == S) shared++; }
        if (int64_t(q.size()) == shared) break;
    }
}

// ------------------------------------------------------------------------------------------
// oplog model
// ------------------------------------------------------------------------------------------
int32_t HostOpLog::agent_id(const char *name, size_t len) {
    for (size_t i = 0; i < agent_names.size(); i++)
        if (agent_names[i].size() == len && std::memcmp(agent_names[i].data(), name, len) == 0) return int32_t(i);
    if ((len == 4 && std::memcmp(name, "ROOT", 4) == 0) || len >= 50) return -1;   // mod.rs:88-91
    agent_names.emplace_back(name, len);
    agent_seqs.emplace_back();
    return int32_t(agent_names.size() - 1);
}
uint64_t HostOpLog::next_seq(uint32_t agent) const {
    uint64_t m = 0;
    for (const SeqRun &r : agent_seqs[agent]) m = std::max(m, r.seq + r.len);
    return m;
}
int64_t HostOpLog::seq_to_lv(uint32_t agent, uint64_t seq) const {
    for (const SeqRun &r : agent_seqs[agent])
        if (seq >= r.seq && seq < r.seq + r.len) return int64_t(r.lv + (seq - r.seq));
    return -1;
}
void HostOpLog::assign(uint32_t agent, uint64_t seq, uint64_t lv, uint64_t len) {
    auto &v = agent_seqs[agent];
    if (!v.empty() && v.back().seq + v.back().len == seq && v.back().lv + v.back().len == lv) v.back().len += len;
    else v.push_back(SeqRun{seq, lv, len});
    if (!agent_runs.empty()) {
        AgentRun &l = agent_runs.back();
        if (l.agent == agent && l.lv + l.len == lv && l.seq + l.len == seq) { l.len += len; return; }
    }
    agent_runs.push_back(AgentRun{lv, len, agent, seq});
}
// push_op_internal + RLE append rules (src/list/oplog.rs:159-175, op_metrics.rs:235-293)
void HostOpLog::push_ins(uint64_t pos, const uint8_t *utf8, size_t nbytes, uint64_t nchars, bool known) {
    const uint64_t lv = n_lv;
    if (known) {
        size_t b = 0;
        for (uint64_t k = 0; k < nchars; k++) {
            ins_cbyte.push_back(uint32_t(ins_content.size() + b));
            b += utf8_len(utf8[b]);
        }
        ins_content.insert(ins_content.end(), utf8, utf8 + nbytes);
    } else {
        content_complete = false;
        ins_cbyte.insert(ins_cbyte.end(), nchars, ~0u);
    }
    n_lv += nchars;
    if (!ops.empty()) {
        OpRun &l = ops.back();
        if (l.kind == 0 && l.lv + l.len == lv && l.pos + l.len == pos) { l.len += nchars; return; }
    }
    ops.push_back(OpRun{lv, nchars, pos, 0, 1});
}
void HostOpLog::push_del(uint64_t pos, uint64_t len, bool fwd) {
    const uint64_t lv = n_lv;
    ins_cbyte.insert(ins_cbyte.end(), len, ~0u);
    n_lv += len;
    if (!ops.empty()) {
        OpRun &l = ops.back();
        if (l.kind == 1 && l.lv + l.len == lv) {
            if ((l.len == 1 || l.fwd) && (len == 1 || fwd) && pos == l.pos) { l.len += len; l.fwd = 1; return; }
            if ((l.len == 1 || !l.fwd) && (len == 1 || !fwd) && pos + len == l.pos) {
                l.pos = pos; l.len += len; l.fwd = 0; return;
            }
        }
    }
    ops.push_back(OpRun{lv, len, pos, 1, uint8_t(fwd ? 1 : 0)});
}
// cg.assign_span + Frontier::advance_by_known_run (frontier.rs:251-279)
void HostOpLog::add_span(uint32_t agent, std::vector<uint64_t> parents, uint64_t start, uint64_t end) {
    std::sort(parents.begin(), parents.end());
    assign(agent, next_seq(agent), start, end - start);
    graph.push(parents, start, end);
    const uint64_t last = end - 1;
    if (parents.size() == 1 && version.size() == 1 && parents[0] == version[0]) { version[0] = last; return; }
    if (version == parents) { version.assign(1, last); return; }
    std::vector<uint64_t> nv;
    for (uint64_t v : version) if (std::find(parents.begin(), parents.end(), v) == parents.end()) nv.push_back(v);
    nv.push_back(last);
    std::sort(nv.begin(), nv.end());
    version.swap(nv);
}
// Split op runs at graph-entry boundaries so every run is a linear chain (distinct targets).
void HostOpLog::finish() {
    std::vector<OpRun> out;
    out.reserve(ops.size() + graph.entries.size());
    size_t gi = 0;
    for (OpRun r : ops) {
        while (r.len) {
            while (gi < graph.entries.size() && graph.entries[gi].end <= r.lv) gi++;
            const uint64_t cut = gi < graph.entries.size() ? graph.entries[gi].end : r.lv + r.len;
            const uint64_t m = std::min(r.len, cut - r.lv);
            OpRun a = r;
            a.len = m;
            if (r.kind == 0) { r.pos += m; }
            else if (!r.fwd) { a.pos = r.pos + r.len - m; }   // truncate_tagged_span, rev Del
            r.lv += m;
            r.len -= m;
            out.push_back(a);
        }
    }
    ops.swap(out);
}

// ------------------------------------------------------------------------------------------
// .dt decode (src/list/encoding/decode_oplog.rs:476-960)
// ------------------------------------------------------------------------------------------
namespace {

constexpr uint64_t UNDERWATER = ~uint64_t(0) / 4;   // UNDERWATER_START (src/dtrange.rs:197)

// Frontier::advance_by_known_run (src/frontier.rs:251-279); false where the reference asserts.
bool advance_known_run(std::vector<uint64_t> &ver, const std::vector<uint64_t> &par, uint64_t start, uint64_t end) {
    const uint64_t last = end - 1;
    if (par.size() == 1 && ver.size() == 1 && par[0] == ver[0]) { ver[0] = last; return true; }
    if (ver == par) { ver.assign(1, last); return true; }
    if (std::find(ver.begin(), ver.end(), start) != ver.end()) return false;
    std::vector<uint64_t> nv;
    for (uint64_t v : ver) if (std::find(par.begin(), par.end(), v) == par.end()) nv.push_back(v);
    nv.insert(std::upper_bound(nv.begin(), nv.end(), last), last);
    ver.swap(nv);
    return true;
}

// version_map of decode_internal (decode_oplog.rs:717-727): file time -> local LV, RLE
struct VMap { uint64_t file, local, len; };
void vmap_push(std::vector<VMap> &vm, uint64_t file, uint64_t local, uint64_t len) {
    if (!vm.empty()) {
        VMap &l = vm.back();
        if (l.file + l.len == file && l.local + l.len == local) { l.len += len; return; }
    }
    vm.push_back(VMap{file, local, len});
}
const VMap *vmap_find(const std::vector<VMap> &vm, uint64_t file) {   // find_packed_with_offset
    auto it = std::upper_bound(vm.begin(), vm.end(), file, [](uint64_t f, const VMap &m) { return f < m.file; });
    if (it == vm.begin()) return nullptr;
    --it;
    return file < it->file + it->len ? &*it : nullptr;
}

// ClientData::item_times.find_sparse (decode_oplog.rs:811-819): the known run holding `seq`
// (its LV), or the end of the unknown gap starting at `seq`.
bool seq_find_sparse(const HostOpLog &o, uint32_t agent, uint64_t seq, uint64_t &lv, uint64_t &run_end) {
    uint64_t gap_end = ~uint64_t(0);
    for (const SeqRun &r : o.agent_seqs[agent]) {
        if (seq >= r.seq && seq < r.seq + r.len) { lv = r.lv + (seq - r.seq); run_end = r.seq + r.len; return true; }
        if (r.seq > seq) gap_end = std::min(gap_end, r.seq);
    }
    run_end = gap_end;
    return false;
}

// decode_internal (decode_oplog.rs:590-960) into `o`, which may already hold operations: the
// overlap filter (:706-850) drops what `o` already has; `file_frontier` gets the file's version.
// On error `o` is left partially modified: decode_and_add unwinds it.
Status decode_into(const uint8_t *data, size_t len, bool ignore_crc, HostOpLog &o,
                   std::vector<uint64_t> &file_frontier) {
    Reader r{data, len};
    if (r.n < 8) return UnexpectedEOF;
    if (std::memcmp(r.p, "DMNDTYPS", 8) != 0) return InvalidMagic;
    r.p += 8; r.n -= 8;
    uint64_t pv;
    if (Status s = r.u64v(pv)) return s;
    if (pv != 0) return UnsupportedProtocolVersion;

    std::vector<uint8_t> lz;
    Reader comp;
    bool has_comp = false;
    {
        bool found; Reader c;
        if (Status s = chunk_if(r, C_LZ4, found, c)) return s;
        if (found) {
            uint64_t ulen;
            if (Status s = c.u64v(ulen)) return s;
            if (ulen > (uint64_t(1) << 34)) return LZ4DecompressionError;
            lz.resize(size_t(ulen));
            if (!lz4_block_decompress(c.p, c.n, lz.data(), lz.size())) return LZ4DecompressionError;
            comp.p = lz.data(); comp.n = lz.size();
            has_comp = true;
        }
    }
    Reader *compp = has_comp ? &comp : nullptr;

    struct AMap { uint32_t agent; uint64_t seq; };
    std::vector<AMap> amap;
    {   // FileInfo (decode_oplog.rs:197-227, 638-649)
        Reader fi, an, tmp, did;
        bool found;
        if (Status s = expect_chunk(r, C_FileInfo, fi)) return s;
        if (Status s = chunk_if(fi, C_DocId, found, did)) return s;
        if (found) {   // into_content_str (decode_tools.rs:133-144)
            uint64_t dt;
            if (Status s = did.u32v(dt)) return s;
            if (dt != 4) return UnknownChunk;
            if (!utf8_valid(did.p, did.n)) return InvalidUTF8;
        }
        const bool has_did = found;
        if (Status s = expect_chunk(fi, C_AgentNames, an)) return s;
        if (Status s = chunk_if(fi, C_UserData, found, tmp)) return s;
        while (!an.empty()) {
            uint64_t nl;
            if (Status s = an.u64v(nl)) return s;
            if (nl > an.n) return InvalidLength;
            const uint8_t *nm;
            if (Status s = an.bytes(size_t(nl), nm)) return s;
            if (!utf8_valid(nm, size_t(nl))) return InvalidUTF8;
            const int32_t id = o.agent_id(reinterpret_cast<const char *>(nm), size_t(nl));
            if (id < 0) return ErrCheckout;
            amap.push_back(AMap{uint32_t(id), 0});
        }
        if (has_did) {   // a doc id must match a non-empty oplog's
            std::string id(reinterpret_cast<const char *>(did.p), did.n);
            if (o.has_doc_id && id != o.doc_id && o.n_lv != 0) return DocIdMismatch;
            o.doc_id.swap(id);
            o.has_doc_id = true;
        }
    }
    std::vector<uint64_t> start_version;
    {   // StartBranch (decode_oplog.rs:652-664), read_version (:70-93)
        Reader sb, ver;
        bool found;
        if (Status s = expect_chunk(r, C_StartBranch, sb)) return s;
        if (Status s = chunk_if(sb, C_Version, found, ver)) return s;
        if (found) {
            for (;;) {
                uint64_t n, seq;
                if (Status s = ver.u64v(n)) return s;
                if (Status s = ver.u64v(seq)) return s;
                if ((n >> 1) == 0) break;
                if ((n >> 1) - 1 >= amap.size()) return InvalidLength;
                const int64_t lv = o.seq_to_lv(amap[size_t((n >> 1) - 1)].agent, seq);
                if (lv < 0) return BaseVersionUnknown;
                start_version.push_back(uint64_t(lv));
                if (!(n & 1)) break;
            }
            if (!ver.empty()) return InvalidLength;
            std::sort(start_version.begin(), start_version.end());
        }
        if (!sb.empty()) {
            const uint8_t *s; size_t sn;
            if (Status e = content_str(sb, compp, s, sn)) return e;
        }
    }
    Reader pc;
    if (Status s = expect_chunk(r, C_Patches, pc)) return s;
    ContentRuns ins, del;
    for (;;) {
        bool found; Reader ch;
        if (Status s = chunk_if(pc, C_PatchContent, found, ch)) return s;
        if (!found) break;
        uint64_t tag;
        if (Status s = ch.u32v(tag)) return s;
        if (tag > 1) return InvalidContent;
        ContentRuns it;
        it.present = true;
        if (Status s = content_str(ch, compp, it.text, it.tn)) return s;
        if (Status s = expect_chunk(ch, C_ContentIsKnown, it.runs)) return s;
        (tag == 0 ? ins : del) = it;
    }
    Reader av, tp, hist;
    if (Status s = expect_chunk(pc, C_OpVersions, av)) return s;
    if (Status s = expect_chunk(pc, C_OpTypeAndPosition, tp)) return s;
    if (Status s = expect_chunk(pc, C_OpParents, hist)) return s;

    // ReadPatchesIter (decode_oplog.rs:289-337) with one pushed-back remainder
    int64_t last_cursor = 0;
    bool have_op = false;
    uint64_t op_len = 0;
    int64_t op_start = 0;
    bool op_del = false, op_fwd = true;
    // The file continues this oplog's version, or its operations must be filtered against what
    // the oplog already has (patches_overlap, decode_oplog.rs:670; file times go underwater).
    const bool overlap = start_version != o.version;
    const uint64_t first_new = o.n_lv;
    const uint64_t new_op_start = overlap ? UNDERWATER : first_new;
    uint64_t next_assign = first_new, next_file = new_op_start;
    std::vector<VMap> vm;

    while (!av.empty()) {   // read_next_agent_assignment (decode_oplog.rs:29-68, 780-850)
        uint64_t n, alen;
        int64_t jump = 0;
        if (Status s = av.u64v(n)) return s;
        const bool has_jump = n & 1;
        n >>= 1;
        if (Status s = av.u64v(alen)) return s;
        if (has_jump) { if (Status s = av.zigzag(jump)) return s; }
        if (n == 0 || n - 1 >= amap.size()) return InvalidLength;
        AMap &m = amap[size_t(n - 1)];
        uint64_t sstart = uint64_t(int64_t(m.seq) + jump);
        const uint64_t send = sstart + alen;
        m.seq = send;
      while (sstart < send) {
        uint64_t known_lv = 0, run_end = send;
        const bool keep = !overlap || !seq_find_sparse(o, m.agent, sstart, known_lv, run_end);
        const uint64_t l = std::min(send, run_end) - sstart;
        if (keep) {
            o.assign(m.agent, sstart, next_assign, l);
            vmap_push(vm, next_file, next_assign, l);
            next_assign += l;
        } else {   // already here: map the file's items onto the local ones
            vmap_push(vm, next_file, known_lv, l);
        }
        next_file += l;
        sstart += l;

        uint64_t want = l;   // parse_next_patches (decode_oplog.rs:731-778)
        while (want) {
            if (!have_op) {
                if (tp.empty()) return InvalidLength;
                uint64_t x;
                if (Status s = tp.u64v(x)) return s;
                const bool has_length = x & 1; x >>= 1;
                const bool diff_nz = x & 1; x >>= 1;
                const bool is_del = x & 1; x >>= 1;
                int64_t diff = 0;
                bool fwd = true;
                uint64_t l;
                if (has_length) {
                    if (is_del) { fwd = x & 1; x >>= 1; }
                    if (diff_nz) { if (Status s = tp.zigzag(diff)) return s; }
                    l = x;
                } else {
                    l = 1;
                    diff = zigzag_of(x);
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
            uint64_t take = std::min(want, op_len);
            ContentRuns &ci = op_del ? del : ins;
            bool known = false;
            const uint8_t *cs = nullptr;
            size_t csn = 0;
            if (ci.present) {
                bool has; uint64_t clen; bool cknown;
                if (Status s = ci.next(has, clen, cknown, cs, csn)) return s;
                if (!has) return InvalidLength;
                if (clen < take) take = clen;
                if (clen > take) {   // push the remainder back (SplitableSpan truncate)
                    size_t b = 0;
                    if (cknown) for (uint64_t k = 0; k < take; k++) b += utf8_len(cs[b]);
                    ci.pb = true;
                    ci.pb_len = clen - take; ci.pb_known = cknown;
                    ci.pb_s = cknown ? cs + b : nullptr; ci.pb_n = cknown ? csn - b : 0;
                    csn = b;
                }
                known = cknown;
            }
            if (!take) return ErrCheckout;
            if (!op_del) {
                if (keep) o.push_ins(uint64_t(op_start), cs, csn, take, known);
                op_start += int64_t(take);
            } else if (!keep) {
            } else if (op_fwd) {
                o.push_del(uint64_t(op_start), take, true);
            } else {
                o.push_del(uint64_t(op_start + int64_t(op_len) - int64_t(take)), take, false);
            }
            op_len -= take;
            if (!op_len) have_op = false;
            want -= take;
        }
      }
    }
    if (o.n_lv != next_assign) return InvalidLength;
    const uint64_t file_end = next_file;

    // OpParents (decode_oplog.rs:95-148, 856-913)
    next_file = new_op_start;
    uint64_t next_hist = first_new;
    file_frontier = start_version;
    std::vector<uint64_t> par, mp;
    while (!hist.empty()) {
        uint64_t hl;
        if (Status s = hist.u64v(hl)) return s;
        par.clear();
        for (;;) {
            uint64_t n;
            if (Status s = hist.u64v(n)) return s;
            const bool foreign = n & 1; n >>= 1;
            const bool more = n & 1; n >>= 1;
            uint64_t p;
            if (foreign) {
                if (n == 0) break;
                if (n - 1 >= amap.size()) return InvalidLength;
                uint64_t seq;
                if (Status s = hist.u64v(seq)) return s;
                const int64_t lv = o.seq_to_lv(amap[size_t(n - 1)].agent, seq);
                if (lv < 0) return InvalidLength;
                p = uint64_t(lv);
            } else {   // next_time - n: an out-of-range value fails the range check below
                if (overlap && n > next_file - new_op_start) return InvalidLength;   // would surface from underwater
                p = next_file - n;
            }
            par.push_back(p);
            if (!more) break;
        }
        std::sort(par.begin(), par.end());
        if (hl == 0 || next_file + hl > file_end) return InvalidLength;
        for (uint64_t p : par) if (p >= next_file) return InvalidLength;
        // history_entry_map_and_truncate (decode_oplog.rs:241-269), one mapped piece at a time
        uint64_t es = next_file;
        const uint64_t ee = next_file + hl;
        next_file = ee;
        for (;;) {
            const VMap *m = vmap_find(vm, es);
            if (!m) return InvalidLength;
            const uint64_t take = std::min(ee - es, m->len - (es - m->file));
            uint64_t ms = m->local + (es - m->file);
            const uint64_t me = ms + take;
            mp.clear();
            for (uint64_t p : par) {
                if (p >= UNDERWATER) {
                    const VMap *pm = vmap_find(vm, p);
                    if (!pm) return InvalidLength;
                    p = pm->local + (p - pm->file);
                }
                mp.push_back(p);
            }
            std::sort(mp.begin(), mp.end());
            if (!advance_known_run(file_frontier, mp, ms, me)) return InvalidLength;
            if (me > next_hist) {   // new here: graph.push + cg.version.advance_by_known_run
                if (ms > next_hist) return InvalidLength;   // assert!(mapped.span.start <= next_history_time)
                if (ms < next_hist) { mp.assign(1, next_hist - 1); ms = next_hist; }   // truncate_keeping_right
                for (uint64_t p : mp) if (p >= ms) return InvalidLength;
                o.graph.push(mp, ms, me);
                if (!advance_known_run(o.version, mp, ms, me)) return InvalidLength;
                next_hist = me;
            }
            es += take;
            if (es == ee) break;
            par.assign(1, es - 1);   // GraphEntrySimple::trim: the remainder's parent, unmapped
        }
    }
    if (next_file != file_end || next_hist != next_assign) return InvalidLength;
    if (!pc.empty()) return InvalidLength;
    if (ins.present) {
        bool has; uint64_t l; bool k; const uint8_t *s; size_t sn;
        Status e = ins.next(has, l, k, s, sn);
        if (e || has) return InvalidContent;
    }
    if (del.present) {
        bool has; uint64_t l; bool k; const uint8_t *s; size_t sn;
        Status e = del.next(has, l, k, s, sn);
        if (e || has) return InvalidContent;
    }
    {   // CRC (decode_oplog.rs:940-955)
        const size_t reader_len = r.n;
        bool found; Reader c;
        if (Status s = chunk_if(r, C_Crc, found, c)) return s;
        if (found && !ignore_crc) {
            if (c.n < 4) return UnexpectedEOF;
            const uint32_t want = uint32_t(c.p[0]) | (uint32_t(c.p[1]) << 8) | (uint32_t(c.p[2]) << 16) |
                                  (uint32_t(c.p[3]) << 24);
            if (crc32c(data, len - reader_len) != want) return ChecksumFailed;
        }
    }
    o.finish();
    return OK;
}

}  // namespace

Status decode_dt(const uint8_t *data, size_t len, bool ignore_crc, HostOpLog &o) {
    std::vector<uint64_t> frontier;
    return decode_into(data, len, ignore_crc, o, frontier);
}

// ListOpLog::decode_and_add_opts (decode_oplog.rs:476-583): on error the oplog is unwound to
// what it was before the call.  Like the reference, each structure is truncated back to its old
// length; the RLE appends may have extended the last run of a structure in place, so that run is
// recorded and restored too.  O(agents + version) to record, no copy of the oplog.
namespace {
struct OpLogMark {
    size_t n_agents, n_agent_runs, n_ops, n_content, n_cbyte, n_entries;
    std::vector<std::pair<size_t, uint64_t>> seqs;   // per agent: runs, len of the last run
    AgentRun last_agent_run{};
    OpRun last_op{};
    uint64_t last_entry_end = 0;
    std::vector<uint64_t> version;
    uint64_t n_lv;
    bool content_complete, has_doc_id;
    std::string doc_id;

    explicit OpLogMark(const HostOpLog &o)
        : n_agents(o.agent_names.size()), n_agent_runs(o.agent_runs.size()), n_ops(o.ops.size()),
          n_content(o.ins_content.size()), n_cbyte(o.ins_cbyte.size()), n_entries(o.graph.entries.size()),
          version(o.version), n_lv(o.n_lv), content_complete(o.content_complete),
          has_doc_id(o.has_doc_id), doc_id(o.doc_id) {
        seqs.reserve(o.agent_seqs.size());
        for (const auto &v : o.agent_seqs) seqs.emplace_back(v.size(), v.empty() ? 0 : v.back().len);
        if (n_agent_runs) last_agent_run = o.agent_runs.back();
        if (n_ops) last_op = o.ops.back();
        if (n_entries) last_entry_end = o.graph.entries.back().end;
    }
    void unwind(HostOpLog &o) const {
        o.agent_names.resize(n_agents);
        o.agent_seqs.resize(seqs.size());
        for (size_t a = 0; a < seqs.size(); a++) {
            auto &v = o.agent_seqs[a];
            v.resize(seqs[a].first);
            if (!v.empty()) v.back().len = seqs[a].second;
        }
        o.agent_runs.resize(n_agent_runs);
        if (n_agent_runs) o.agent_runs.back() = last_agent_run;
        o.ops.resize(n_ops);
        if (n_ops) o.ops.back() = last_op;
        o.ins_content.resize(n_content);
        o.ins_cbyte.resize(n_cbyte);
        o.graph.entries.resize(n_entries);
        if (n_entries) o.graph.entries.back().end = last_entry_end;
        o.version = version;
        o.n_lv = n_lv;
        o.content_complete = content_complete;
        o.has_doc_id = has_doc_id;
        o.doc_id = doc_id;
    }
};
}  // namespace

Status decode_and_add(const uint8_t *data, size_t len, bool ignore_crc, HostOpLog &o,
                      std::vector<uint64_t> &file_frontier) {
    const OpLogMark mark(o);
    const Status s = decode_into(data, len, ignore_crc, o, file_frontier);
    if (s != OK) { mark.unwind(o); file_frontier.clear(); }
    return s;
}

// ------------------------------------------------------------------------------------------
// walk plan (src/listmerge/txn_trace.rs:114-333 + merge.rs:564-581)
// ------------------------------------------------------------------------------------------
// Agent-name ranks for the YjsMod tie-break (byte-wise name order, merge.rs:199-218) as the
// device's (first LV, rank, first seq, agent) quads.
static void plan_agent_runs(const HostOpLog &o, Plan &plan) {
    plan.agent_runs.clear();
    std::vector<uint32_t> order(o.agent_names.size()), rank(o.agent_names.size());
    for (uint32_t i = 0; i < order.size(); i++) order[i] = i;
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return o.agent_names[a] < o.agent_names[b]; });
    for (uint32_t i = 0; i < order.size(); i++) rank[order[i]] = i;
    for (const AgentRun &r : o.agent_runs) {
        plan.agent_runs.push_back(uint32_t(r.lv));
        plan.agent_runs.push_back(rank[r.agent]);
        plan.agent_runs.push_back(uint32_t(r.seq));
        plan.agent_runs.push_back(r.agent);
    }
}

// SpanningTreeWalker over every graph entry from ROOT.
Status build_plan(const HostOpLog &o, Plan &plan) {
    plan.cmds.clear();
    plan.tlist.clear();
    plan.agent_runs.clear();
    if (o.n_lv >= MAX_PLAN_LV) return ErrCapacity;
    if (!o.content_complete) return ErrCheckout;   // content.unwrap() in apply_to (merge.rs:329)

    plan_agent_runs(o, plan);

    const auto &E = o.graph.entries;
    const size_t ne = E.size();
    // VisitEntry table: parent / child indexes inside the (whole-graph) input
    std::vector<std::vector<uint32_t>> pidx(ne), cidx(ne);
    std::vector<uint32_t> todo;
    for (size_t i = 0; i < ne; i++) {
        for (uint64_t p : E[i].parents) pidx[i].push_back(uint32_t(o.graph.find_idx(p)));
        if (pidx[i].empty()) todo.push_back(uint32_t(i));
    }
    for (size_t i = 0; i < ne; i++) for (uint32_t p : pidx[i]) cidx[p].push_back(uint32_t(i));
    std::reverse(todo.begin(), todo.end());
    std::vector<uint8_t> visited(ne, 0);

    // op-run lookup
    const auto &ops = o.ops;
    auto run_of = [&](uint64_t lv) -> size_t {
        auto it = std::upper_bound(ops.begin(), ops.end(), lv, [](uint64_t v, const OpRun &r) { return v < r.lv + r.len; });
        return size_t(it - ops.begin());
    };
    // retreat / advance entries of one walk step, labelled Ins/Del per op run
    auto emit_state = [&](uint64_t s, uint64_t e, bool retreat) {
        if (s >= e) return;
        size_t ri = run_of(s);
        for (uint64_t lo = s; lo < e; ri++) {
            const OpRun &r = ops[ri];
            const uint64_t hi = std::min(e, r.lv + r.len);
            const uint32_t tag = (r.kind ? TL_DEL : 0u) | (retreat ? 0u : TL_ADV);
            for (uint64_t v = lo; v < hi; v++) plan.tlist.push_back(uint32_t(v) | tag);
            lo = hi;
        }
    };
    auto flush_step = [&](size_t from) {
        if (plan.tlist.size() > from)
            plan.cmds.push_back(Cmd{CMD_TOG, uint32_t(from), uint32_t(plan.tlist.size() - from), 0});
    };
    auto emit_apply = [&](uint64_t s, uint64_t e) {
        size_t ri = run_of(s);
        uint64_t lo = s;
        while (lo < e) {
            const OpRun &r = ops[ri];
            const uint64_t hi = std::min(e, r.lv + r.len);
            const uint64_t k = lo - r.lv, m = hi - lo;
            if (r.kind == 0) plan.cmds.push_back(Cmd{CMD_INS, uint32_t(lo), uint32_t(m), uint32_t(r.pos + k)});
            else if (r.fwd) plan.cmds.push_back(Cmd{CMD_DEL | 16u, uint32_t(lo), uint32_t(m), uint32_t(r.pos)});
            else plan.cmds.push_back(Cmd{CMD_DEL, uint32_t(lo), uint32_t(m), uint32_t(r.pos + r.len - k - m)});
            lo = hi;
            ri++;
        }
    };

    std::vector<uint64_t> frontier;
    std::vector<std::pair<uint64_t, uint64_t>> only_a, only_b;
    while (!todo.empty()) {
        uint32_t idx = todo.back();
        if (E[idx].parents.size() >= 2) {   // prefer non-merge entries (txn_trace.rs:249-266)
            int64_t found = -1;
            for (int64_t ii = int64_t(todo.size()) - 1; ii >= 0; ii--)
                if (E[todo[size_t(ii)]].parents.size() < 2) { found = ii; break; }
            if (found >= 0) { idx = todo[size_t(found)]; todo[size_t(found)] = todo.back(); todo.pop_back(); }
            else todo.pop_back();
        } else todo.pop_back();
        visited[idx] = 1;
        const GraphEntry &e = E[idx];
        o.graph.diff_rev(frontier, e.parents, only_a, only_b);
        const size_t t0 = plan.tlist.size();
        for (auto &rg : only_a) { emit_state(rg.first, rg.second, true); plan.n_retreat += rg.second - rg.first; }
        for (auto &rg : only_b) { emit_state(rg.first, rg.second, false); plan.n_advance += rg.second - rg.first; }
        flush_step(t0);
        emit_apply(e.start, e.end);
        frontier.assign(1, e.end - 1);
        plan.n_steps++;
        for (uint32_t c : cidx[idx]) {
            if (visited[c]) continue;
            bool ok = true;
            for (uint32_t p : pidx[c]) if (!visited[p]) { ok = false; break; }
            if (ok) todo.push_back(c);
        }
    }
    // advance to the tip: the tracker's visible set is then the checkout (list/merge.rs:63-95)
    o.graph.diff_rev(frontier, o.version, only_a, only_b);
    if (!only_a.empty()) return ErrCheckout;   // the tip contains every LV
    const size_t t0 = plan.tlist.size();
    for (auto &rg : only_b) { emit_state(rg.first, rg.second, false); plan.n_tip_advance += rg.second - rg.first; }
    flush_step(t0);
    if (plan.tlist.size() >= 0xFFFFFFFFull) return ErrCapacity;
    return OK;
}

// ---- transformed-ops plans ----------------------------------------------------------------
std::vector<uint64_t> parents_at(const HostOpLog &o, uint64_t lv) {   // clone_parents_at_version
    const GraphEntry &e = o.graph.entries[size_t(o.graph.find_idx(lv))];
    return lv > e.start ? std::vector<uint64_t>{lv - 1} : e.parents;
}

// SpanningTreeWalker::new(graph, spans, frontier) + its iteration (txn_trace.rs:114-333):
// ascending spans split per graph entry; parents outside the input are ignored.  visit(start,
// end, parents) is called per consumed span in walk order.
void spanning_walk(const HostOpLog &o, const std::vector<std::pair<uint64_t, uint64_t>> &spans,
                   const std::function<void(uint64_t, uint64_t, const std::vector<uint64_t> &)> &visit) {
    struct In { uint64_t start, end; std::vector<uint64_t> parents; std::vector<uint32_t> pidx, cidx; };
    std::vector<In> in;
    for (auto sp : spans) {
        for (uint64_t s = sp.first; s < sp.second;) {
            const GraphEntry &e = o.graph.entries[size_t(o.graph.find_idx(s))];
            const uint64_t t = std::min(e.end, sp.second);
            in.push_back(In{s, t, parents_at(o, s), {}, {}});
            s = t;
        }
    }
    auto find_in = [&](uint64_t lv) -> int64_t {
        auto it = std::upper_bound(in.begin(), in.end(), lv, [](uint64_t v, const In &x) { return v < x.end; });
        return it != in.end() && it->start <= lv ? int64_t(it - in.begin()) : -1;
    };
    std::vector<uint32_t> todo;
    for (size_t i = 0; i < in.size(); i++) {
        for (uint64_t p : in[i].parents) { const int64_t j = find_in(p); if (j >= 0) in[i].pidx.push_back(uint32_t(j)); }
        if (in[i].pidx.empty()) todo.push_back(uint32_t(i));
    }
    for (size_t i = 0; i < in.size(); i++) for (uint32_t p : in[i].pidx) in[p].cidx.push_back(uint32_t(i));
    std::reverse(todo.begin(), todo.end());
    std::vector<uint8_t> visited(in.size(), 0);
    while (!todo.empty()) {
        uint32_t idx = todo.back();
        if (in[idx].parents.size() >= 2) {   // prefer non-merge entries (txn_trace.rs:243-265)
            int64_t found = -1;
            for (int64_t ii = int64_t(todo.size()) - 1; ii >= 0; ii--)
                if (in[todo[size_t(ii)]].parents.size() < 2) { found = ii; break; }
            if (found >= 0) { idx = todo[size_t(found)]; todo[size_t(found)] = todo.back(); todo.pop_back(); }
            else todo.pop_back();
        } else todo.pop_back();
        visited[idx] = 1;
        visit(in[idx].start, in[idx].end, in[idx].parents);
        for (uint32_t c : in[idx].cidx) {
            if (visited[c]) continue;
            bool ok = true;
            for (uint32_t p : in[c].pidx) if (!visited[p]) { ok = false; break; }
            if (ok) todo.push_back(c);
        }
    }
}

namespace {
struct XfPlanner {
    const HostOpLog &o;
    Plan &plan;
    size_t run_of(uint64_t lv) const {
        auto it = std::upper_bound(o.ops.begin(), o.ops.end(), lv, [](uint64_t v, const OpRun &r) { return v < r.lv + r.len; });
        return size_t(it - o.ops.begin());
    }
    void state(uint64_t s, uint64_t e, bool retreat) {   // retreat / advance entries, tagged Ins/Del
        for (size_t ri = run_of(s); s < e; ri++) {
            const OpRun &r = o.ops[ri];
            const uint64_t hi = std::min(e, r.lv + r.len);
            const uint32_t tag = (r.kind ? TL_DEL : 0u) | (retreat ? 0u : TL_ADV);
            for (uint64_t v = s; v < hi; v++) plan.tlist.push_back(uint32_t(v) | tag);
            s = hi;
        }
    }
    // retreat / advance from `cur` to `to` as one TOG command (Graph::diff_rev)
    void move(const std::vector<uint64_t> &cur, const std::vector<uint64_t> &to) {
        std::vector<std::pair<uint64_t, uint64_t>> a, b;
        o.graph.diff_rev(cur, to, a, b);
        const size_t t0 = plan.tlist.size();
        for (auto &rg : a) { state(rg.first, rg.second, true); plan.n_retreat += rg.second - rg.first; }
        for (auto &rg : b) { state(rg.first, rg.second, false); plan.n_advance += rg.second - rg.first; }
        if (plan.tlist.size() > t0) plan.cmds.push_back(Cmd{CMD_TOG, uint32_t(t0), uint32_t(plan.tlist.size() - t0), 0});
    }
    void apply(uint64_t s, uint64_t e) {   // op runs clipped to [s, e) (truncate_tagged_span)
        for (size_t ri = run_of(s); s < e; ri++) {
            const OpRun &r = o.ops[ri];
            const uint64_t hi = std::min(e, r.lv + r.len);
            const uint64_t k = s - r.lv, m = hi - s;
            if (r.kind == 0) plan.cmds.push_back(Cmd{CMD_INS, uint32_t(s), uint32_t(m), uint32_t(r.pos + k)});
            else if (r.fwd) plan.cmds.push_back(Cmd{CMD_DEL | 16u, uint32_t(s), uint32_t(m), uint32_t(r.pos)});
            else plan.cmds.push_back(Cmd{CMD_DEL, uint32_t(s), uint32_t(m), uint32_t(r.pos + r.len - k - m)});
            s = hi;
        }
    }
    void walk(const std::vector<std::pair<uint64_t, uint64_t>> &spans, std::vector<uint64_t> &frontier) {
        spanning_walk(o, spans, [&](uint64_t s, uint64_t e, const std::vector<uint64_t> &parents) {
            move(frontier, parents);
            apply(s, e);
            frontier.assign(1, e - 1);
            plan.n_steps++;
        });
    }
};
std::vector<std::pair<uint64_t, uint64_t>> ascending(std::vector<std::pair<uint64_t, uint64_t>> v) {
    std::reverse(v.begin(), v.end());
    return v;
}
}  // namespace

Status build_xf_plan_from(const HostOpLog &o, const std::vector<uint64_t> &from, const std::vector<uint64_t> &merge,
                          Plan &plan, size_t &first_emitted) {
    plan = Plan();
    first_emitted = 0;
    if (o.n_lv >= MAX_PLAN_LV) return ErrCapacity;
    if (!o.content_complete) return ErrCheckout;
    for (uint64_t v : from) if (v >= o.n_lv) return ErrArg;
    for (uint64_t v : merge) if (v >= o.n_lv) return ErrArg;
    plan_agent_runs(o, plan);
    XfPlanner P{o, plan};
    std::vector<std::pair<uint64_t, uint64_t>> hist, newr, none;
    o.graph.diff_rev(from, {}, hist, none);      // Hist(from): the branch's content
    o.graph.diff_rev(merge, from, newr, none);   // new ops: Hist(merge) - Hist(from)
    hist = ascending(hist);
    newr = ascending(newr);
    std::vector<uint64_t> frontier;
    if (!hist.empty()) P.walk(hist, frontier);
    P.move(frontier, from);
    frontier = from;
    first_emitted = plan.cmds.size();
    // fast-forward (merge.rs:792-835): up to the entry's end while its parents are the frontier
    size_t si = 0;
    while (si < newr.size()) {
        const uint64_t s0 = newr[si].first;
        if (parents_at(o, s0) != frontier) break;
        const GraphEntry &e = o.graph.entries[size_t(o.graph.find_idx(s0))];
        const uint64_t s1 = std::min(e.end, newr[si].second);
        P.apply(s0, s1);
        frontier.assign(1, s1 - 1);
        newr[si].first = s1;
        if (s1 == newr[si].second) si++;
    }
    newr.erase(newr.begin(), newr.begin() + ptrdiff_t(si));
    if (!newr.empty()) P.walk(newr, frontier);
    // end at the merged version (ListBranch::merge's frontier, find_dominators_2)
    std::vector<uint64_t> u(from);
    u.insert(u.end(), merge.begin(), merge.end());
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    std::vector<uint64_t> fin;
    std::vector<std::pair<uint64_t, uint64_t>> a, b;
    for (uint64_t v : u) {
        bool dom = false;
        for (uint64_t w : u) if (w > v) { o.graph.diff_rev({v}, {w}, a, b); if (a.empty()) { dom = true; break; } }
        if (!dom) fin.push_back(v);
    }
    P.move(frontier, fin);
    if (plan.tlist.size() >= 0xFFFFFFFFull) return ErrCapacity;
    return OK;
}
Status build_xf_plan(const HostOpLog &o, Plan &plan) {
    size_t first = 0;
    return build_xf_plan_from(o, {}, o.version, plan, first);
}

Status build_plan_input(const HostOpLog &o, PlanInput &pi) {
    if (o.n_lv >= MAX_PLAN_LV) return ErrCapacity;
    if (!o.content_complete) return ErrCheckout;
    const auto &E = o.graph.entries;
    const size_t ne = E.size();
    pi = PlanInput();
    pi.n_agents = uint32_t(o.agent_names.size());
    pi.est.reserve(2 * ne);
    pi.poff.assign(1, 0);
    std::vector<uint32_t> ccount(ne + 1, 0);
    for (size_t i = 0; i < ne; i++) {
        pi.est.push_back(uint32_t(E[i].start));
        pi.est.push_back(uint32_t(E[i].end));
        for (uint64_t p : E[i].parents) {
            const int64_t pe = o.graph.find_idx(p);
            if (pe < 0) return ErrCheckout;
            pi.par.push_back(uint32_t(p));
            pi.pent.push_back(uint32_t(pe));
            ccount[size_t(pe)]++;
        }
        pi.poff.push_back(uint32_t(pi.par.size()));
    }
    pi.coff.assign(ne + 1, 0);
    for (size_t i = 0; i < ne; i++) pi.coff[i + 1] = pi.coff[i] + ccount[i];
    pi.child.assign(pi.coff[ne], 0);
    {
        std::vector<uint32_t> fill(pi.coff.begin(), pi.coff.end() - 1);
        for (size_t i = 0; i < ne; i++)
            for (uint32_t k = pi.poff[i]; k < pi.poff[i + 1]; k++) pi.child[fill[pi.pent[k]]++] = uint32_t(i);
    }
    // op runs (already split at entry boundaries by finish()) as apply commands
    pi.eop.assign(ne + 1, 0);
    {
        size_t ri = 0;
        for (size_t i = 0; i < ne; i++) {
            while (ri < o.ops.size() && o.ops[ri].lv < E[i].start) ri++;
            pi.eop[i] = uint32_t(ri);
        }
        pi.eop[ne] = uint32_t(o.ops.size());
    }
    for (const OpRun &r : o.ops) {
        if (r.kind == 0) pi.opc.push_back(Cmd{CMD_INS, uint32_t(r.lv), uint32_t(r.len), uint32_t(r.pos)});
        else pi.opc.push_back(Cmd{r.fwd ? (CMD_DEL | 16u) : uint32_t(CMD_DEL), uint32_t(r.lv), uint32_t(r.len), uint32_t(r.pos)});
    }
    // agent assignment, both directions
    std::vector<uint32_t> order(o.agent_names.size()), rank(o.agent_names.size());
    for (uint32_t i = 0; i < order.size(); i++) order[i] = i;
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return o.agent_names[a] < o.agent_names[b]; });
    for (uint32_t i = 0; i < order.size(); i++) rank[order[i]] = i;
    for (const AgentRun &r : o.agent_runs) {
        pi.aruns.push_back(uint32_t(r.lv));
        pi.aruns.push_back(rank[r.agent]);
        pi.aruns.push_back(uint32_t(r.seq));
        pi.aruns.push_back(r.agent);
    }
    pi.ear.assign(ne, 0);
    {
        size_t ai = 0;
        const auto &R = o.agent_runs;
        for (size_t i = 0; i < ne; i++) {
            while (ai < R.size() && R[ai].lv + R[ai].len <= E[i].start) ai++;
            pi.ear[i] = uint32_t(ai);
        }
    }
    pi.aoff.assign(1, 0);
    for (uint32_t a = 0; a < pi.n_agents; a++) {
        std::vector<SeqRun> v = o.agent_seqs[a];
        std::sort(v.begin(), v.end(), [](const SeqRun &x, const SeqRun &y) { return x.seq < y.seq; });
        for (const SeqRun &r : v) {
            pi.aseq.push_back(uint32_t(r.seq));
            pi.aseq.push_back(uint32_t(r.lv));
            pi.aseq.push_back(uint32_t(r.len));
        }
        pi.aoff.push_back(uint32_t(pi.aseq.size() / 3));
    }
    pi.isdel.assign((o.n_lv + 31) / 32, 0);
    for (const OpRun &r : o.ops)
        if (r.kind)
            for (uint64_t v = r.lv; v < r.lv + r.len; v++) pi.isdel[v >> 5] |= 1u << (v & 31);
    for (uint64_t t : o.version) {
        const int64_t te = o.graph.find_idx(t);
        if (te < 0) return ErrCheckout;
        pi.tip.push_back(uint32_t(t));
        pi.tip.push_back(uint32_t(te));
    }
    // Chain decomposition of the graph, in LV order: an entry joins a chain whose every op is
    // already in the entry's history (the chain's length equals the entry's parent version
    // vector at that chain), preferring its first parent's chain; with none such it opens a
    // new chain.  Every chain is then a causal chain, so a version's ancestor set is a prefix
    // of every chain and a version vector over chains describes it exactly (the device planner
    // diffs those vectors).  The chain count stays near the history's concurrency width.
    std::vector<uint32_t> chain_of(ne), seq0(ne);
    std::vector<uint64_t> clen;                    // per chain: ops so far
    std::vector<std::vector<uint32_t>> prow(ne);   // per entry: parent vector over chains
    for (size_t i = 0; i < ne; i++) {
        std::vector<uint32_t> &row = prow[i];
        row.assign(clen.size(), 0);
        for (uint32_t k = pi.poff[i]; k < pi.poff[i + 1]; k++) {
            const uint32_t pe = pi.pent[k];
            const std::vector<uint32_t> &pr = prow[pe];
            for (size_t c = 0; c < pr.size(); c++) row[c] = std::max(row[c], pr[c]);
            const uint32_t pc = chain_of[pe];
            row[pc] = std::max<uint32_t>(row[pc], seq0[pe] + uint32_t(pi.par[k] - E[pe].start) + 1);
        }
        uint32_t c = 0xFFFFFFFFu;
        if (pi.poff[i + 1] > pi.poff[i]) {
            const uint32_t pc = chain_of[pi.pent[pi.poff[i]]];
            if (row[pc] == clen[pc]) c = pc;
        }
        for (size_t k = 0; k < clen.size() && c == 0xFFFFFFFFu; k++)
            if (row[k] == clen[k]) c = uint32_t(k);
        if (c == 0xFFFFFFFFu) {
            c = uint32_t(clen.size());
            clen.push_back(0);
            if (clen.size() > PLAN_CHAIN_LIMIT) {   // too wide for the device planner
                pi.device_ok = false;
                return OK;
            }
            row.push_back(0);
        }
        chain_of[i] = c;
        seq0[i] = uint32_t(clen[c]);
        clen[c] += E[i].end - E[i].start;
    }
    pi.n_chains = uint32_t(clen.size());
    // the parent vectors, n_chains words per entry (chains opened later are 0): the device
    // planner reads each consumed entry's vector instead of rebuilding it from its parents'
    if (pi.n_chains <= 64) {
        pi.prow.assign(ne * pi.n_chains, 0);
        for (size_t i = 0; i < ne; i++)
            for (size_t c = 0; c < prow[i].size(); c++) pi.prow[i * pi.n_chains + c] = prow[i][c];
    }
    pi.pch.resize(pi.par.size());
    pi.pcnt.resize(pi.par.size());
    for (size_t k = 0; k < pi.par.size(); k++) {
        const uint32_t pe = pi.pent[k];
        pi.pch[k] = chain_of[pe];
        pi.pcnt[k] = seq0[pe] + (pi.par[k] - uint32_t(E[pe].start)) + 1;
    }
    // entry records
    pi.erec.assign(ne * EREC_WORDS, 0);
    for (size_t i = 0; i < ne; i++) {
        uint32_t r[EREC_WORDS] = {};
        r[0] = uint32_t(E[i].start);
        r[1] = uint32_t(E[i].end);
        r[2] = pi.poff[i];
        r[3] = pi.poff[i + 1] - pi.poff[i];
        r[4] = pi.eop[i];
        r[5] = pi.eop[i + 1] - pi.eop[i];
        r[6] = chain_of[i];
        r[7] = seq0[i];
        r[8] = pi.coff[i];
        r[9] = pi.coff[i + 1] - pi.coff[i];
        r[10] = r[3] ? pi.par[pi.poff[i]] : 0xFFFFFFFFu;
        for (uint32_t j = 0; j < 2; j++) {
            const bool has = r[3] > j;
            const uint32_t k = pi.poff[i] + j;
            r[11 + 3 * j] = has ? pi.pent[k] : 0xFFFFFFFFu;
            r[12 + 3 * j] = has ? pi.pch[k] : 0;
            r[13 + 3 * j] = has ? pi.pcnt[k] : 0;
        }
        r[17] = r[9] ? pi.child[pi.coff[i + 1] - 1] : 0xFFFFFFFFu;
        r[18] = r[9] ? pi.child[pi.coff[i]] : 0xFFFFFFFFu;
        for (uint32_t k = 0; k < EREC_WORDS; k++) pi.erec[erec_word(ne, i, k)] = r[k];
    }
    // dense chain seq -> LV | is_del tables (the planner copies retreat/advance ranges out)
    pi.doff.assign(pi.n_chains + 1, 0);
    for (uint32_t c = 0; c < pi.n_chains; c++) pi.doff[c + 1] = pi.doff[c] + uint32_t(clen[c]);
    pi.dense.assign(o.n_lv, 0);
    for (size_t i = 0; i < ne; i++)
        for (uint64_t lv = E[i].start; lv < E[i].end; lv++)
            pi.dense[pi.doff[chain_of[i]] + seq0[i] + (lv - E[i].start)] =
                uint32_t(lv) | (((pi.isdel[lv >> 5] >> (lv & 31)) & 1u) ? TL_DEL : 0u);
    return OK;
}

}  // namespace dtgpu
