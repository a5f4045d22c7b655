// dt_ff.hip -- linear-history checkout on MI355X (gfx950): the reference's fast-forward path
// (src/listmerge/merge.rs:811-840: while the next entry's parents are the frontier, ops apply as
// plain positional edits; src/list/merge.rs:63-95 writes them into the branch's rope) for
// documents whose whole history is one graph entry.  See dt_ff.hpp for the piece-table layout.
//
// Kernels of one pass (launch_ff), all integer and memory-latency work, no MFMA:
//   ff_delta_kernel    thread per segment: its inserted - deleted chars
//   ff_seg_kernel      wave per segment: FF_RUNS op runs applied to <= 128 pieces held two per
//                      lane; a splice = one DPP prefix scan over the lanes' piece lengths, a ballot
//                      for the piece holding the position, and an LDS round trip that re-packs
//                      the pieces (shift for an insert, compaction for a delete)
//   ff_compose_kernel  one workgroup per pair of adjacent groups per level: the later group's
//                      placeholder pieces expanded into the earlier group's pieces (two binary
//                      searches per placeholder, a block scan for output slots, load-balanced
//                      writes)
//   ff_text_kernel     workgroup per document: byte offset of every final piece (UTF-8)
//   ff_copy_kernel     workgroup per 4 KiB of output: the text bytes and their hash terms
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "dt_ff.hpp"
#include "dt_host.hpp"

namespace dtgpu {
namespace ff {

typedef unsigned long long u64;
#define DEV __device__ __forceinline__

DEV uint32_t lane_id() { return __lane_id(); }
DEV void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); }
DEV uint32_t bcast(uint32_t v, uint32_t l) { return uint32_t(__builtin_amdgcn_readlane(int(v), int(l))); }
DEV uint32_t first_lane(u64 m) { return uint32_t(__ffsll((long long)m) - 1); }
// inclusive 64-lane prefix sum (DPP row shifts, then row_bcast 15 / 31), as dt_replay.hip
DEV uint32_t wave_scan(uint32_t x) {
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xF, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x142, 0xA, 0xF, false));
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x143, 0xC, 0xF, false));
    return x;
}
DEV uint32_t wave_sum(uint32_t v) { return bcast(wave_scan(v), 63); }
DEV u64 splitmix(u64 z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
DEV uint32_t utf8_len(uint8_t c) { return c < 0x80 ? 1 : (c & 0xE0) == 0xC0 ? 2 : (c & 0xF0) == 0xE0 ? 3 : 4; }

// Exclusive prefix sum over a workgroup of NT threads (wave scans + one LDS round for the wave
// totals); *total = the sum.  s_w holds NT / 64 + 1 words.  Ends with a barrier.
template <uint32_t NT>
DEV uint32_t block_scan(uint32_t x, uint32_t *s_w, uint32_t &total) {
    const uint32_t l = lane_id(), w = threadIdx.x / 64;
    const uint32_t inc = wave_scan(x);
    if (l == 63) s_w[w] = inc;
    __syncthreads();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < NT / 64; k++) {
        const uint32_t v = s_w[k];
        base += k < w ? v : 0;
        tot += v;
    }
    total = tot;
    __syncthreads();
    return base + inc - x;
}

// ---- 1. per-segment length deltas ----------------------------------------------------------------
__global__ __launch_bounds__(256) void ff_delta_kernel(FFParams P) {
    const uint32_t s = blockIdx.x * 256 + threadIdx.x;
    if (s >= P.n_segs) return;
    const FFSeg g = P.segs[s];
    const FFDoc &D = P.docs[g.doc];
    const uint4 *ops = reinterpret_cast<const uint4 *>(P.ops) + D.op_off + g.run0;
    uint32_t d = 0;
    for (uint32_t k = 0; k < g.nrun; k++) {
        const uint4 r = ops[k];
        d += (r.w & 1u) ? 0u - r.y : r.y;
    }
    P.delta[s] = int32_t(d);
    if (s == D.first_seg) P.bad[g.doc] = 0;
}

// ---- 2. segment replay (one wave, pieces in registers) -------------------------------------------
__global__ __launch_bounds__(64) void ff_seg_kernel(FFParams P) {
    __shared__ uint4 sv[FF_PIECES / 2 + 1];   // re-pack area: piece j at uint2 slot j
    uint2 *sp = reinterpret_cast<uint2 *>(sv);
    const uint32_t l = lane_id();
    const uint32_t gs = blockIdx.x;
    const FFSeg g = P.segs[gs];
    const FFDoc &D = P.docs[g.doc];
    const uint32_t first = D.first_seg, li = gs - first;
    // the text length at the segment's start: every earlier segment's inserts - deletes
    uint32_t acc = 0;
    for (uint32_t k = l; k < li; k += 64) acc += uint32_t(P.delta[first + k]);
    const uint32_t lin = wave_sum(acc);
    uint4 run = make_uint4(0, 0, 0, 0);
    if (l < g.nrun) run = reinterpret_cast<const uint4 *>(P.ops)[D.op_off + g.run0 + l];
    uint32_t s0 = 0, l0 = 0, s1 = 0, l1 = 0;   // pieces 2l and 2l + 1
    uint32_t n = 0;
    if (lin) {
        n = 1;
        if (l == 0) { s0 = FF_PH; l0 = lin; }
    }
    uint32_t bad = int32_t(lin) < 0 ? 1u : 0u;   // more deleted than inserted before this segment
    const uint32_t j0 = 2 * l, j1 = 2 * l + 1;
    for (uint32_t r = 0; r < g.nrun && !bad; r++) {
        const uint32_t lv = bcast(run.x, r), len = bcast(run.y, r), pos = bcast(run.z, r);
        const bool del = (bcast(run.w, r) & 1u) != 0;
        const uint32_t pair = l0 + l1;
        const uint32_t inc = wave_scan(pair);
        const uint32_t total = bcast(inc, 63);
        const uint32_t e0 = inc - pair, e1 = e0 + l0;
        if (!del) {
            if (pos > total || len == 0) { bad = 1; break; }
            // the piece holding pos (none: pos is the end of the text)
            const bool c0 = pos - e0 < l0, c1 = pos - e1 < l1;   // (unsigned: e <= pos < e + len)
            const u64 m = __ballot(c0 || c1);
            uint32_t k = n, off = 0;
            if (m) {
                const uint32_t kl = first_lane(m);
                const uint32_t in0 = bcast(c0 ? 1u : 0u, kl);
                k = 2 * kl + (in0 ? 0u : 1u);
                off = pos - bcast(in0 ? e0 : e1, kl);
            }
            if (off == 0 && k > 0) {   // the run continues the piece before it (typing)
                const uint32_t pl = (k - 1) >> 1, ph = (k - 1) & 1u;
                const uint32_t ps = bcast(ph ? s1 : s0, pl), pn = bcast(ph ? l1 : l0, pl);
                if (!(ps & FF_PH) && ps + pn == lv) {
                    if (l == pl) { if (ph) l1 += len; else l0 += len; }
                    continue;
                }
            }
            if (n + (off ? 2u : 1u) > FF_PIECES) { bad = 1; break; }   // (FF_RUNS bounds it)
            const uint32_t sh = off ? 2u : 1u;
            if (j0 < n) {
                if (j0 < k) sp[j0] = make_uint2(s0, l0);
                else if (j0 > k || off == 0) sp[j0 + sh] = make_uint2(s0, l0);
                else { sp[j0] = make_uint2(s0, off); sp[j0 + 2] = make_uint2(s0 + off, l0 - off); }
            }
            if (j1 < n) {
                if (j1 < k) sp[j1] = make_uint2(s1, l1);
                else if (j1 > k || off == 0) sp[j1 + sh] = make_uint2(s1, l1);
                else { sp[j1] = make_uint2(s1, off); sp[j1 + 2] = make_uint2(s1 + off, l1 - off); }
            }
            if (l == 0) sp[k + (off ? 1u : 0u)] = make_uint2(lv, len);
            n += sh;
        } else {
            const uint32_t de = pos + len;
            if (de > total || de < pos || len == 0) { bad = 1; break; }
            // what survives of each piece [a, b): its part left of pos and its part right of de
            const uint32_t a0 = e0, b0 = e0 + l0, a1 = e1, b1 = e1 + l1;
            const uint32_t L0 = a0 < pos ? min(b0, pos) - a0 : 0u, R0 = b0 > de ? b0 - max(a0, de) : 0u;
            const uint32_t L1 = a1 < pos ? min(b1, pos) - a1 : 0u, R1 = b1 > de ? b1 - max(a1, de) : 0u;
            const uint32_t c = (L0 ? 1u : 0u) + (R0 ? 1u : 0u) + (L1 ? 1u : 0u) + (R1 ? 1u : 0u);
            const uint32_t ci = wave_scan(c);
            uint32_t o = ci - c;
            if (L0) sp[o++] = make_uint2(s0, L0);
            if (R0) sp[o++] = make_uint2(s0 + (max(a0, de) - a0), R0);
            if (L1) sp[o++] = make_uint2(s1, L1);
            if (R1) sp[o++] = make_uint2(s1 + (max(a1, de) - a1), R1);
            n = bcast(ci, 63);
        }
        wave_fence();
        const uint4 v = sv[l];
        s0 = j0 < n ? v.x : 0u; l0 = j0 < n ? v.y : 0u;
        s1 = j1 < n ? v.z : 0u; l1 = j1 < n ? v.w : 0u;
        wave_fence();
    }
    if (bad && l == 0) P.bad[g.doc] = 1;
    const uint32_t pair = l0 + l1;
    const uint32_t e0 = wave_scan(pair) - pair;
    uint4 *out = reinterpret_cast<uint4 *>(P.pa) + D.piece_off + size_t(FF_PIECES) * li;
    if (j0 < n) out[j0] = make_uint4(s0, l0, e0, 0);
    if (j1 < n) out[j1] = make_uint4(s1, l1, e0 + l0, 0);
    if (l == 0) P.ca[gs] = n;
}

// ---- 3. pairwise composition ----------------------------------------------------------------------
// The last piece of A (n pieces, ascending pos) whose pos is <= x (0 if none).
DEV uint32_t last_at_or_before(const uint4 *A, uint32_t n, uint32_t x) {
    uint32_t lo = 0, hi = n;   // answer in [lo, hi)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (A[mid].z <= x) lo = mid; else hi = mid;
    }
    return lo;
}

// CT threads per pair: one wave for the low levels (a pair of <= 4 segments' pieces is one or
// a few rounds), four for the rest
template <uint32_t CT>
__global__ __launch_bounds__(CT) void ff_compose_kernel(FFParams P, uint32_t level, const uint4 *in, uint4 *out,
                                                        const uint32_t *cin, uint32_t *cout) {
    __shared__ uint32_t s_ex[CT + 1], s_i0[CT], s_w[CT / 64 + 1];
    __shared__ uint4 s_b[CT];
    const uint32_t t = threadIdx.x;
    const FFPair pr = P.pairs[P.level_off[level] + blockIdx.x];
    const FFDoc &D = P.docs[pr.doc];
    const size_t abase = D.piece_off + size_t(FF_PIECES) * pr.a;
    const uint32_t na = cin[D.first_seg + pr.a];
    if (pr.b == FF_NONE) {   // a lone group: carried to the next level's buffer as it is
        for (uint32_t i = t; i < na; i += CT) out[abase + i] = in[abase + i];
        if (t == 0) cout[D.first_seg + pr.a] = na;
        return;
    }
    const size_t bbase = D.piece_off + size_t(FF_PIECES) * pr.b;
    const uint32_t nb = cin[D.first_seg + pr.b];
    const uint32_t b_end = min(pr.b + (1u << level), D.n_seg);
    const uint32_t cap = FF_PIECES * (b_end - pr.a);
    const uint4 *A = in + abase;
    if (t == 0) s_w[CT / 64] = 0;   // error flag of the rounds below (ordered by block_scan's barrier)
    const uint32_t a_total = na ? A[na - 1].z + A[na - 1].y : 0u;
    uint32_t carry = 0, bad = 0;
    for (uint32_t r0 = 0; r0 < nb; r0 += CT) {
        const uint32_t j = r0 + t, m = min(CT, nb - r0);
        uint4 bp = make_uint4(0, 0, 0, 0);
        uint32_t cnt = 0, i0 = 0, err = 0;
        if (j < nb) {
            bp = in[bbase + j];
            if (bp.x & FF_PH) {
                const uint32_t p = bp.x & ~FF_PH, q = p + bp.y - 1;
                if (bp.y == 0 || q >= a_total || q < p) {
                    err = 1;
                } else {
                    i0 = last_at_or_before(A, na, p);
                    cnt = last_at_or_before(A, na, q) - i0 + 1;
                }
            } else {
                cnt = 1;
            }
        }
        uint32_t tot = 0;
        const uint32_t ex = block_scan<CT>(cnt, s_w, tot);
        s_ex[t] = ex;
        s_i0[t] = i0;
        s_b[t] = bp;
        if (err) s_w[CT / 64] = 1;
        __syncthreads();
        if (s_w[CT / 64] || carry + tot > cap) { bad = 1; break; }
        for (uint32_t o = t; o < tot; o += CT) {
            uint32_t lo = 0, hi = m;   // the B piece of output o: last k with s_ex[k] <= o
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) / 2;
                if (s_ex[mid] <= o) lo = mid; else hi = mid;
            }
            const uint4 b = s_b[lo];
            uint4 res = b;
            if (b.x & FF_PH) {
                const uint4 a = A[s_i0[lo] + (o - s_ex[lo])];
                const uint32_t p = b.x & ~FF_PH;
                const uint32_t x0 = max(a.z, p), x1 = min(a.z + a.y, p + b.y);
                res = make_uint4(a.x + (x0 - a.z), x1 - x0, b.z + (x0 - p), 0);
            }
            out[abase + carry + o] = res;
        }
        carry += tot;
        __syncthreads();
    }
    if (t == 0) {
        cout[D.first_seg + pr.a] = bad ? 0u : carry;
        if (bad) P.bad[pr.doc] = 1;
    }
}

// ---- 4. byte offsets of the final pieces, the document's result -----------------------------------
constexpr uint32_t TT = 1024;
__global__ __launch_bounds__(TT) void ff_text_kernel(FFParams P) {
    __shared__ uint32_t s_w[TT / 64 + 1];
    const uint32_t t = threadIdx.x;
    const uint32_t d = blockIdx.x;
    const FFDoc &D = P.docs[d];
    const uint4 *F = reinterpret_cast<const uint4 *>((D.levels & 1u) ? P.pb : P.pa) + D.piece_off;
    const uint32_t nf = ((D.levels & 1u) ? P.cb : P.ca)[D.first_seg];
    const uint32_t *cbyte = P.cbyte + D.lv_off;
    const uint8_t *content = P.content + D.content_off;
    uint32_t *boff = P.boff + D.piece_off;
    uint32_t carry = 0, ph = 0;
    if (D.ascii) {
        if (nf) carry = F[nf - 1].z + F[nf - 1].y;
        for (uint32_t i = t; i < nf; i += TT) ph |= F[i].x & FF_PH;
    } else {
        for (uint32_t r0 = 0; r0 < nf; r0 += TT) {
            const uint32_t i = r0 + t;
            uint32_t bytes = 0;
            if (i < nf) {
                const uint4 p = F[i];
                ph |= p.x & FF_PH;
                if (!(p.x & FF_PH) && p.y) {
                    const uint32_t c0 = cbyte[p.x], cl = cbyte[p.x + p.y - 1];
                    bytes = cl + utf8_len(content[cl]) - c0;
                }
            }
            uint32_t tot = 0;
            const uint32_t ex = block_scan<TT>(bytes, s_w, tot);
            if (i < nf) boff[i] = carry + ex;
            carry += tot;
        }
    }
    if (t == 0) s_w[TT / 64] = 0;
    __syncthreads();
    if (ph) s_w[TT / 64] = 1;   // a placeholder survived into the final list: malformed
    __syncthreads();
    if (t == 0) {
        DocResult &R = P.results[D.result];
        const uint32_t bad = P.bad[d] | s_w[TT / 64];
        R.status = bad ? uint32_t(ErrCheckout) : carry > D.out_cap ? uint32_t(ErrCapacity) : 0u;
        R.out_len = R.status ? 0u : carry;
        R.hash = 0;
        R.n_items = nf;   // pieces of the final list
        R.n_blocks = D.n_seg;
        R.fail_cmd = 0;
        R.fail_site = bad ? 40u : 0u;
        R.n_sb = 0;
        R.lds = 0;
    }
}

// ---- 5. text bytes and hash ----------------------------------------------------------------------
constexpr uint32_t XT = 256, XB = FF_CHUNK / XT;   // threads, bytes per thread
__global__ __launch_bounds__(XT) void ff_copy_kernel(FFParams P) {
    __shared__ uint32_t s_off[FF_CHUNK + 2], s_cb[FF_CHUNK + 1], s_rng[2];
    __shared__ u64 s_h[XT / 64];
    const uint32_t t = threadIdx.x;
    const FFChunk ch = P.chunks[blockIdx.x];
    const FFDoc &D = P.docs[ch.doc];
    DocResult &R = P.results[D.result];
    const uint32_t len = R.out_len;
    if (R.status || ch.start >= len) return;
    const uint32_t c0 = ch.start, c1 = min(c0 + FF_CHUNK, len);
    const uint4 *F = reinterpret_cast<const uint4 *>((D.levels & 1u) ? P.pb : P.pa) + D.piece_off;
    const uint32_t nf = ((D.levels & 1u) ? P.cb : P.ca)[D.first_seg];
    const uint32_t *boff = P.boff + D.piece_off;
    const bool ascii = D.ascii != 0;
    auto off_of = [&](uint32_t i) { return ascii ? F[i].z : boff[i]; };
    // pieces overlapping [c0, c1): the last one starting at or before c0 through the last one
    // starting before c1 (at most FF_CHUNK + 1 of them: pieces are never empty)
    if (t < 2) {
        const uint32_t x = t ? c1 - 1 : c0;
        uint32_t lo = 0, hi = nf;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) / 2;
            if (off_of(mid) <= x) lo = mid; else hi = mid;
        }
        s_rng[t] = lo;
    }
    __syncthreads();
    const uint32_t p0 = s_rng[0], m = s_rng[1] - p0 + 1;
    const uint32_t *cbyte = P.cbyte + D.lv_off;
    for (uint32_t k = t; k <= m; k += XT) {
        const uint32_t i = p0 + k;
        s_off[k] = i < nf ? off_of(i) : len;
        if (k < m) s_cb[k] = cbyte[F[i].x];
    }
    __syncthreads();
    const uint8_t *content = P.content + D.content_off;
    uint8_t *out = P.out + D.out_off;
    u64 h = 0;
    const uint32_t b0 = c0 + XB * t;
    if (b0 < c1) {
        uint32_t lo = 0, hi = m;   // the piece holding b0
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) / 2;
            if (s_off[mid] <= b0) lo = mid; else hi = mid;
        }
        const uint32_t b1 = min(b0 + XB, c1);
        for (uint32_t b = b0; b < b1; b++) {
            while (b >= s_off[lo + 1]) lo++;
            const uint8_t byte = content[s_cb[lo] + (b - s_off[lo])];
            out[b] = byte;
            h += splitmix((u64(b) << 8) | byte);
        }
    }
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) h += __shfl_xor(h, k, 64);
    if (lane_id() == 0) s_h[t / 64] = h;
    __syncthreads();
    if (t == 0) {
        u64 sum = 0;
        for (uint32_t w = 0; w < XT / 64; w++) sum += s_h[w];
        atomicAdd(reinterpret_cast<unsigned long long *>(&R.hash), sum);
    }
}

}  // namespace ff

int launch_ff(const FFParams &p, void *stream) {
    if (!p.n_docs) return 0;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(ff::ff_delta_kernel, dim3((p.n_segs + 255) / 256), dim3(256), 0, s, p);
    hipLaunchKernelGGL(ff::ff_seg_kernel, dim3(p.n_segs), dim3(64), 0, s, p);
    uint4 *a = reinterpret_cast<uint4 *>(p.pa), *b = reinterpret_cast<uint4 *>(p.pb);
    uint32_t *ca = p.ca, *cb = p.cb;
    for (uint32_t k = 0; k < p.n_levels; k++) {
        const uint32_t np = p.level_off[k + 1] - p.level_off[k];
        if (np && k < 2) hipLaunchKernelGGL(ff::ff_compose_kernel<64>, dim3(np), dim3(64), 0, s, p, k, a, b, ca, cb);
        else if (np) hipLaunchKernelGGL(ff::ff_compose_kernel<256>, dim3(np), dim3(256), 0, s, p, k, a, b, ca, cb);
        std::swap(a, b);
        std::swap(ca, cb);
    }
    hipLaunchKernelGGL(ff::ff_text_kernel, dim3(p.n_docs), dim3(ff::TT), 0, s, p);
    if (p.n_chunks) hipLaunchKernelGGL(ff::ff_copy_kernel, dim3(p.n_chunks), dim3(ff::XT), 0, s, p);
    return launch_error() == hipSuccess ? 0 : int(ErrHip);
}

}  // namespace dtgpu
