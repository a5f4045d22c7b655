// dt_prep.hip -- planner inputs from the device-decoded oplog (the device half of
// dt_host.cpp build_plan_input), one 64-lane wavefront per document.
//
//   parents -> entry index (Graph::find_packed, graph/mod.rs), children CSR in child-index order
//   op runs -> apply commands and each entry's first op run (ops never cross entries)
//   agent runs -> (lv, name rank, seq, agent) quads; ranks order agent names byte-wise, the
//                 YjsMod tie-break of listmerge/merge.rs:199-218
//   causal-chain decomposition (see dt_host.cpp build_plan_input): an entry joins a chain whose
//                 every op is in its history (its parent vector over chains equals the chain's
//                 length), preferring its first parent's chain, else opens a chain.  Sequential
//                 over entries; the parent vector is one VGPR (lane = chain), vectors of earlier
//                 entries come back from HBM (or from registers for the previous entry, the usual
//                 parent), so a linear stretch of history costs no memory round trip.
//   entry records, per-chain dense seq -> (LV | is_del) tables, tips with their entries.
// Everything but the decomposition is lane-parallel.  Documents with more than 64 chains are
// reported PREP_WIDE and prepared on the host.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dt_prep.hpp"

namespace dtgpu {
namespace prep {

__device__ __forceinline__ uint32_t lane() { return __lane_id(); }
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) {
    return uint32_t(__builtin_amdgcn_readlane(int(v), int(l)));
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint64_t lt_mask() { return (1ull << lane()) - 1ull; }
__device__ __forceinline__ uint32_t popc(uint64_t m) { return uint32_t(__popcll(m)); }
__device__ __forceinline__ uint32_t ctz(uint64_t m) { return uint32_t(__ffsll((unsigned long long)m) - 1); }
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }
__device__ __forceinline__ uint32_t scan_incl(uint32_t v) {   // inclusive prefix sum over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = uint32_t(__shfl_up(int(v), d));
        if (lane() >= uint32_t(d)) v += o;
    }
    return v;
}

// A refill waits for its load inside the refill branch: the compiler's counter analysis then
// sees nothing pending where the paths meet, instead of a vmcnt(0) at every use -- which would
// also wait for each entry's row store (vmcnt counts stores).  s_waitcnt vmcnt(0), the other
// counters left alone.
__device__ __forceinline__ void wait_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// 64 consecutive words / pairs cached in one VGPR, addressed by a uniform index
struct Chunk {
    uint32_t blk, v;
    __device__ __forceinline__ void init() { blk = 0xFFFFFFFFu; v = 0; }
    template <typename F>
    __device__ __forceinline__ uint32_t get(uint32_t i, uint32_t n, F load) {
        if ((i & ~63u) != blk) {
            blk = i & ~63u;
            const uint32_t k = blk + lane();
            v = k < n ? load(k) : 0xFFFFFFFFu;
            wait_vm();
        }
        return rdl(v, i & 63u);
    }
};

// two such words per index, refilled by one load issue (one round trip, not two)
struct Chunk2 {
    uint32_t blk, a, b;
    __device__ __forceinline__ void init() { blk = 0xFFFFFFFFu; a = b = 0; }
    template <typename F>
    __device__ __forceinline__ uint2 get(uint32_t i, uint32_t n, F load) {
        if ((i & ~63u) != blk) {
            blk = i & ~63u;
            const uint32_t k = blk + lane();
            const uint2 v = k < n ? load(k) : make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
            a = v.x; b = v.y;
            wait_vm();
        }
        return make_uint2(rdl(a, i & 63u), rdl(b, i & 63u));
    }
};

// entry of `lv` among entries [0, hi) (sorted, contiguous): the previous entry first
__device__ __forceinline__ uint32_t entry_of(const uint2 *ent, uint32_t hi, uint32_t lv) {
    if (hi && lv >= ent[hi - 1].x && lv < ent[hi - 1].y) return hi - 1;
    // gallop back from hi (a merge's other parent is usually a few entries back), then bisect
    uint32_t lo = 0, h = hi;
    for (uint32_t step = 1; step < h; step <<= 1) {
        const uint32_t m = h - step;
        if (ent[m].x <= lv) { lo = m; break; }
        h = m;
    }
    while (lo < h) {
        const uint32_t mid = (lo + h) >> 1;
        if (lv >= ent[mid].y) lo = mid + 1; else h = mid;
    }
    return lo < hi && lv >= ent[lo].x ? lo : 0xFFFFFFFFu;
}

#ifndef DTGPU_PREP_WAVES
#define DTGPU_PREP_WAVES 8   // occupancy target (tuning knob; the register budget follows from it)
#endif
// CHECK (debug mode, DTGPU_DEBUG): every computed table index -- child slots, parent-vector rows,
// chain pairs, chain offsets, dense chain slots, the parents and entries records read through
// computed indexes -- is asserted inside the document's arena before it is used; a failure skips
// the access and reports PREP_BOUNDS with the table (the host then fails the document), so a
// layout bug shows up as a status instead of a stray store.  The release kernel is unchanged.
#define PREP_ASSERT(cond, table)                                  \
    do {                                                          \
        if (CHECK && !(cond)) { oob = oob ? oob : (table); }      \
    } while (0)
template <bool CHECK>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(DTGPU_PREP_WAVES))) void prep_kernel(PrepParams P) {
    // per entry (u16, two per LDS word): child count, then the next free slot of its children
    // list relative to coff -- half the LDS of absolute u32 slots, so more documents share a CU
    extern __shared__ uint32_t lfw[];
    uint16_t *lfill = reinterpret_cast<uint16_t *>(lfw);
    if (blockIdx.x >= P.n_docs) return;
    const uint32_t doc = P.doc_list ? P.doc_list[blockIdx.x] : blockIdx.x;
    uint32_t flag = 0;
    if (P.mode == 1 && lane() == 0) P.chain_flag[doc] = 0;
    if (P.mode == 2) {
        flag = P.chain_flag[doc];
        if (flag == 0) return;   // the first half ended the document (its status is written)
    }
    const PrepDesc D = P.docs[doc];
    PrepResult R{};
    if (D.skip) {
        if (lane() == 0) { R.status = PREP_SKIP; P.results[doc] = R; }
        return;
    }
    const uint32_t l = lane();
    const uint32_t ne = D.ne, npar = D.n_par, nops = D.n_ops;
    const uint2 *ent = reinterpret_cast<const uint2 *>(P.d_ent) + D.d_ent;
    const uint32_t *poff = P.d_poff + D.d_poff;
    const uint32_t *par_in = P.d_par + D.d_par;
    const uint4 *ops = reinterpret_cast<const uint4 *>(P.d_ops) + D.d_op;
    const uint4 *ar = reinterpret_cast<const uint4 *>(P.d_aruns) + D.d_arun;
    uint32_t *par = P.par + D.o_par, *pent = P.pent + D.o_par, *pch = P.pch + D.o_par, *pcnt = P.pcnt + D.o_par;
    uint32_t *child = P.child + D.o_child;
    uint32_t *erec = P.erec + D.o_erec;
    uint32_t *doff = P.doff + D.o_doff;
    uint32_t *dense = P.dense + D.o_dense;
    uint32_t *rows = P.rows + D.o_rows;
    const uint32_t rs = D.row_stride;   // <= PREP_MAX_CHAINS
    uint32_t *owner = P.scr + D.o_scr;
    // per entry {chain, seq0 - start (mod 2^32)}: one 8-byte load gives a parent's chain and the
    // offset that turns its parent LV into a chain length (dt_prep.hpp prep_scratch_words)
    uint2 *cs = reinterpret_cast<uint2 *>(owner + ((npar + 1) & ~1u));
    uint32_t *coff = reinterpret_cast<uint32_t *>(cs + ne), *eop = coff + ne + 1;
    uint32_t *kids = eop + ne + 1;   // walk kernel: per entry {children | first slot, first | last child}
    Cmd *opc = P.opc + D.o_op;
    if (ne > P.max_entries || D.n_lv >= (1u << 30)) {
        if (l == 0) { R.status = PREP_BAD; P.results[doc] = R; }
        return;
    }
    if (npar >= 0xFFFFu) {   // a child count could overflow its u16: prepared on the host
        if (l == 0) { R.status = PREP_WIDE; P.results[doc] = R; }
        return;
    }
    uint32_t oob = 0;   // CHECK: the first table whose bounds assert failed (per lane)
    auto report_oob = [&]() -> bool {   // wave-uniform: true when a bounds assert failed anywhere
        if (!CHECK) return false;
        const uint64_t m = ballot(oob != 0);
        if (!m) return false;
        if (l == 0) { R.status = PREP_BOUNDS; R.pad = rdl(oob, ctz(m)); P.results[doc] = R; }
        return true;
    };

#ifdef DTGPU_PREP_PROF
    const uint64_t T0 = wall_clock64();
    uint64_t T1 = T0, T2 = T0;
#endif
    if (P.mode != 2) {
    // ---- 1. parents: entry of each parent, child counts ------------------------------------------
    for (uint32_t i = l; i < (ne + 1) / 2; i += 64) lfw[i] = 0;
    __syncthreads();
    bool bad = false;
    for (uint32_t i0 = 0; i0 < ne; i0 += 64) {
        const uint32_t i = i0 + l;
        if (i < ne) {
            const uint32_t k1 = poff[i + 1];
            for (uint32_t k = poff[i]; k < k1; k++) {
                const uint32_t p = par_in[k];
                const uint32_t pe = entry_of(ent, i, p);
                if (pe == 0xFFFFFFFFu) { bad = true; break; }
                PREP_ASSERT(pe < i, PREP_T_ENTRY);
                owner[k] = i;
                if (!P.short_rec) par[k] = p;   // (read by the records' tails and the one-phase planner)
                pent[k] = pe;
                atomicAdd(&lfw[pe >> 1], 1u << (16 * (pe & 1u)));
            }
        }
    }
    if (ballot(bad)) {
        if (l == 0) { R.status = PREP_BAD; P.results[doc] = R; }
        return;
    }
    __syncthreads();
    // children CSR offsets (exclusive scan); lfill becomes each entry's next free child slot
    // (relative to its offset)
    {
        uint32_t carry = 0;
        for (uint32_t i0 = 0; i0 < ne; i0 += 64) {
            const uint32_t i = i0 + l;
            const uint32_t c = i < ne ? lfill[i] : 0;
            const uint32_t inc = scan_incl(c);
            if (i < ne) { coff[i] = carry + inc - c; lfill[i] = 0; }
            carry += rdl(inc, 63);
        }
        if (l == 0) coff[ne] = carry;
    }
    __syncthreads();
    wave_fence();
    // children in child-index order (slots are in (child, parent) order): a stable scatter,
#ifdef DTGPU_PREP_PROF
    T1 = wall_clock64();
#endif
    // 64 slots at a time: each lane gathers its key's CSR offset and fill once, register-only
    // rounds (one key each) rank the lanes sharing a key, then one parallel store places them and
    // the last lane of each key advances its fill
    for (uint32_t k0 = 0; k0 < npar; k0 += 64) {
        const uint32_t k = k0 + l;
        const bool live = k < npar;
        const uint32_t key = live ? pent[k] : 0xFFFFFFFFu;
        const uint32_t own = live ? owner[k] : 0;
        const uint32_t kco = live ? coff[key] : 0;
        const uint32_t krel = live ? uint32_t(lfill[key]) : 0;
        uint32_t rank = 0, cnt = 0;
        bool todo = live;
        for (uint64_t m = ballot(todo); m; m = ballot(todo)) {
            const uint32_t lead = rdl(key, ctz(m));
            const bool mine = todo && key == lead;
            const uint64_t mm = ballot(mine);
            if (mine) {
                rank = popc(mm & lt_mask());
                cnt = popc(mm);
                todo = false;
            }
        }
        PREP_ASSERT(!live || (key < ne && kco + krel + rank < npar), PREP_T_CHILD);
        if (live && (!CHECK || !oob)) {
            child[kco + krel + rank] = own;
            if (rank + 1 == cnt) lfill[key] = uint16_t(krel + cnt);
        }
        __syncthreads();
    }
    if (report_oob()) return;

#ifdef DTGPU_PREP_PROF
    T2 = wall_clock64();
#endif
    // ---- 2. each entry's first op run (ops are split at entry boundaries) ------------------------
    // eop[i] = lower bound of the entry's first LV among the op runs' first LVs (strictly
    // increasing): 64 entries at a time, each lane binary-searches 64-op windows by lane permute;
    // a batch starts at the previous batch's last bound
    {
        const uint32_t *opx = reinterpret_cast<const uint32_t *>(ops);   // ops[k].x = opx[4 k]
        uint32_t j0 = 0;
        for (uint32_t i0 = 0; i0 < ne; i0 += 64) {
            const uint32_t i = i0 + l;
            const bool live = i < ne;
            const uint32_t s = live ? ent[i].x : 0u;
            uint32_t res = 0xFFFFFFFFu;
            for (uint32_t jb = j0;; jb += 64) {
                const uint32_t k = jb + l;
                const uint32_t ox = k < nops ? opx[4 * size_t(k)] : 0xFFFFFFFFu;
                uint32_t c = 0;   // ops of this window below s
#pragma unroll
                for (uint32_t step = 32; step >= 1; step >>= 1)
                    if (uint32_t(__shfl(int(ox), int(c + step - 1))) < s) c += step;
                if (c == 63 && rdl(ox, 63) < s) c = 64;   // (a permute here would run divergent)
                if (res == 0xFFFFFFFFu && c < 64) res = jb + c;
                if (!ballot(live && res == 0xFFFFFFFFu) || jb >= nops) break;
            }
            if (live) eop[i] = res;
            j0 = rdl(res, min(ne - 1 - i0, 63u));
        }
        if (l == 0) eop[ne] = nops;
    }
    wave_fence();
    }   // P.mode != 2
    if (P.mode == 1) {   // first half done: chain_kernel (or the second half) goes on from HBM
        // each entry's children for the walk kernel, which starts now: {children | first slot
        // << 16, first child | last child << 16} (slots < n_par < 0xFFFF; the walk takes documents
        // of at most PLAN_MAX_LDS_ENTRIES entries)
        uint2 *k2 = reinterpret_cast<uint2 *>(kids);
        for (uint32_t i = l; i < ne; i += 64) {
            const uint32_t c0 = coff[i], nc = coff[i + 1] - c0;
            k2[i] = make_uint2(nc | (c0 << 16), nc ? (child[c0] & 0xFFFFu) | (child[c0 + nc - 1] << 16) : 0u);
        }
        if (l == 0) P.chain_flag[doc] = 1;
        return;
    }

#ifdef DTGPU_PREP_PROF
    const uint64_t T3 = wall_clock64();
#endif
    // ---- 3. causal-chain decomposition (sequential over entries) ---------------------------------
    uint32_t clen = 0, nch = 0;      // lane c: ops in chain c so far
    if (flag == 2) nch = doff[PREP_MAX_CHAINS];   // chain_kernel decomposed it (<= CHAIN_GROUP chains)
    uint32_t prev_row = 0;           // parent vector of entry i - 1
    uint32_t prev_chain = 0, prev_sd = 0;   // chain, seq0 - start of entry i - 1
    if (flag != 2) {
        Chunk2 cpp;   // parent slot (LV, entry)
        cpp.init();
        // the current 64 entries' parent-slot ranges and LV spans, lane = entry mod 64, loaded at
        // each 64-entry boundary (no per-entry refill test)
        uint32_t bk0 = 0, bk1 = 0, bs = 0, be = 0;
        uint32_t bch = 0, bsd = 0;   // chain / seq0 - start of the current 64 entries, flushed per 64
        constexpr uint32_t RING = 8;
        uint64_t keep = 0;   // entries of the current 64 whose row a child beyond the ring reads
        // the last RING entries' parent vectors with their chain and seq offset, in LDS (the
        // child-count table's space, free after the scatter), slot = entry mod RING: a merge's
        // other parent is almost always a few entries back (friendsforever: all within 7,
        // git-makefile 63 % within 8), so its row is one LDS read, not an HBM round trip (a
        // register ring costs a compare-and-select chain over every slot per entry)
        uint32_t *ring_row = lfw;                  // RING x 64 words
        uint32_t *ring_meta = lfw + RING * 64;     // RING x {entry, chain, seq0 - start}
        if (l < RING) ring_meta[3 * l] = 0xFFFFFFFFu;
        __syncthreads();
#ifdef DTGPU_PREP_PROF
        uint64_t pa = 0, pb = 0, pc_ = 0, pk = 0;
#endif
        for (uint32_t i = 0; i < ne; i++) {
#ifdef DTGPU_PREP_PROF
            uint64_t tq = __builtin_amdgcn_s_memtime();
#endif
            if ((i & 63u) == 0) {
                const uint32_t j = min(i + l, ne - 1);
                bk0 = poff[j];
                bk1 = poff[j + 1];
                const uint2 se = ent[j];
                bs = se.x;
                be = se.y;
                wait_vm();
            }
            if ((i & 63u) == 0) {   // a row is stored only for a child more than RING entries on
                // (children are in index order: the last is the farthest; nearer ones read the
                // row from the ring or, for the next entry, from prev_row)
                const uint32_t j = i + l;
                bool need = false;
                if (j < ne) {
                    const uint32_t c0 = coff[j], nc = coff[j + 1] - c0;
                    need = nc > 0 && child[c0 + nc - 1] > j + RING;
                }
                keep = ballot(need);
            }
#ifdef DTGPU_PREP_PROF
            { const uint64_t t = __builtin_amdgcn_s_memtime(); pk += t - tq; tq = t; }
#endif
            const uint32_t k0 = rdl(bk0, i & 63u), k1 = rdl(bk1, i & 63u);
            uint32_t row = 0;
            uint32_t first_chain = 0xFFFFFFFFu;
            for (uint32_t k = k0; k < k1; k++) {
                const uint2 pp = cpp.get(k, npar, [&](uint32_t x) { return make_uint2(par_in[x], pent[x]); });
                const uint32_t p = pp.x, pe = pp.y;
                uint32_t prow, pc, psd;
                if (pe + 1 == i) {
                    prow = prev_row; pc = prev_chain; psd = prev_sd;
                } else {
                    const uint32_t slot = pe & (RING - 1);
                    const bool hit = ring_meta[3 * slot] == pe;
                    prow = pc = psd = 0;
                    if (hit) { prow = ring_row[slot * 64 + l]; pc = ring_meta[3 * slot + 1]; psd = ring_meta[3 * slot + 2]; }
                    if (!hit) {
                        PREP_ASSERT(pe < i, PREP_T_ROWS);
                        prow = l < rs && (!CHECK || pe < i) ? rows[size_t(pe) * rs + l] : 0u;
                        if (pe >= (i & ~63u)) {   // not flushed yet: from the registers
                            pc = rdl(bch, pe & 63u); psd = rdl(bsd, pe & 63u);
                        } else {
                            PREP_ASSERT(pe < ne, PREP_T_PAIRS);
                            const uint2 q = (!CHECK || pe < ne) ? cs[pe] : make_uint2(0, 0);
                            pc = q.x; psd = q.y;
                        }
                    }
                }
                row = max(row, prow);
                if (l == pc) row = max(row, psd + p + 1);   // seq0 + (p - start) + 1
                if (k == k0) first_chain = pc;
            }
            // every entry's parent vector (the planner reads it) goes out with its ring: the
            // rows of 8 entries stored together when the ring wraps, so the store's completion
            // (vmcnt counts stores) is waited for once per 8 entries, not at every entry
#ifdef DTGPU_PREP_PROF
            { const uint64_t t = __builtin_amdgcn_s_memtime(); pa += t - tq; tq = t; }
#endif
            uint32_t c = 0xFFFFFFFFu;
            if (first_chain != 0xFFFFFFFFu && rdl(row, first_chain) == rdl(clen, first_chain)) c = first_chain;
            if (c == 0xFFFFFFFFu) {
                const uint64_t m = ballot(l < nch && row == clen);
                if (m) c = ctz(m);
            }
            if (c == 0xFFFFFFFFu) {
                if (nch == rs) {   // (rs = PREP_MAX_CHAINS until staging counted the chains)
                    if (l == 0) { R.status = PREP_WIDE; R.n_chains = nch + 1; P.results[doc] = R; }
                    return;
                }
                c = nch++;
            }
#ifdef DTGPU_PREP_PROF
            { const uint64_t t = __builtin_amdgcn_s_memtime(); pb += t - tq; tq = t; }
#endif
            const uint32_t s = rdl(bs, i & 63u), e = rdl(be, i & 63u);
            const uint32_t s0 = rdl(clen, c);
            if (l == c) clen += e - s;
            bch = (i & 63u) == l ? c : bch;
            bsd = (i & 63u) == l ? s0 - s : bsd;
            if ((i & 63u) == 63u || i + 1 == ne) {
                const uint32_t at = i & ~63u;
                if (at + l <= i) cs[at + l] = make_uint2(bch, bsd);
                wave_fence();   // later entries read these pairs back from other lanes
            }
            prev_row = row; prev_chain = c; prev_sd = s0 - s;
            {
                const uint32_t slot = i & (RING - 1);
                ring_row[slot * 64 + l] = row;
                if (l == 0) { ring_meta[3 * slot] = i; ring_meta[3 * slot + 1] = c; ring_meta[3 * slot + 2] = s0 - s; }
                if (slot == RING - 1 || i + 1 == ne) {
                    for (uint32_t r = i & ~(RING - 1); r <= i; r++) {
                        // a row a child more than RING entries on reads back is stored whole
                        // (chains opened later read as zero); the planner reads chains < nch.
                        // A compact stride stores every row whole (one short contiguous piece)
                        if (l < rs && (rs < PREP_MAX_CHAINS || l < nch || ((keep >> (r & 63u)) & 1u)))
                            rows[size_t(r) * rs + l] = ring_row[(r & (RING - 1)) * 64 + l];
                    }
                }
            }
#ifdef DTGPU_PREP_PROF
            pc_ += __builtin_amdgcn_s_memtime() - tq;
#endif
        }
#ifdef DTGPU_PREP_PROF
        if (l == 0 && (doc == 0 || doc == P.n_docs / 2))
            printf("PREPCHAIN doc %u ne %u keep %llu parents %llu select %llu rest %llu (cycles)\n", doc, ne,
                   (unsigned long long)pk, (unsigned long long)pa, (unsigned long long)pb, (unsigned long long)pc_);
#endif
    }
    wave_fence();
    if (report_oob()) return;
#ifdef DTGPU_PREP_PROF
    const uint64_t T4 = wall_clock64();
#endif
    // per chain: offset of its dense table (also kept in a register, lane = chain)
    uint32_t doff_l;
    if (flag == 2) {
        doff_l = l < nch ? doff[l] : 0u;   // (doff[PREP_MAX_CHAINS] holds the chain count)
    } else {
        const uint32_t c = l < nch ? clen : 0;
        const uint32_t inc = scan_incl(c);
        doff_l = inc - c;
        PREP_ASSERT(rdl(inc, 63) == D.n_lv, PREP_T_DOFF);   // the chains partition the LVs
        if (l < nch) doff[l] = doff_l;
        if (l == 0) doff[nch] = rdl(inc, 63);
    }

    // ---- 4. lane-parallel outputs -----------------------------------------------------------------
    // parent slots: chain and ops of that chain up to it; four 64-slot rounds per iteration so
    // their dependent loads (slot -> entry -> chain pair) are in flight together.  (Read by the
    // records' tails and the one-phase planner only: a heads-only pass skips them.)
    for (uint32_t k0 = 0; k0 < npar && !P.short_rec; k0 += 256) {
        uint32_t pe[4], pv[4];
        uint2 q[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint32_t k = k0 + 64 * uint32_t(r) + l;
            pe[r] = k < npar ? pent[k] : 0u;
            pv[r] = k < npar ? par[k] : 0u;
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint32_t k = k0 + 64 * uint32_t(r) + l;
            PREP_ASSERT(k >= npar || pe[r] < ne, PREP_T_PAIRS);
            q[r] = k < npar && (!CHECK || pe[r] < ne) ? cs[pe[r]] : make_uint2(0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint32_t k = k0 + 64 * uint32_t(r) + l;
            if (k < npar) {
                pch[k] = q[r].x;
                pcnt[k] = q[r].y + pv[r] + 1;
            }
        }
    }
    wave_fence();
    // entry records (dt_host.hpp PlanInput::erec), one per lane: a lane's head (32 bytes) and
    // tail (48) are contiguous and next to its neighbours', so the stores coalesce as they are
    // (the 80-byte records of round 4 went through LDS, with a fence per 32 records).
    // P.short_rec: the pass's walk reads the CSR and its planner only the heads, so the tails are
    // neither built nor stored (their gathers of parent and child slots skipped with them)
    {
        static_assert(EREC_WORDS == 20 && EREC_HEAD == 8, "erec layout");
        uint4 *eh = reinterpret_cast<uint4 *>(erec);
        uint4 *et = reinterpret_cast<uint4 *>(erec + size_t(ne) * EREC_HEAD);
        for (uint32_t i = l; i < ne; i += 64) {
            // head: 0-3 start, end, parents offset / count; 4-7 first op run, op runs, chain, seq0.
            // tail: 8-10 children offset / count, first parent LV; 11-13 and 14-16 the first two
            // parents' entry, chain, count; 17 last child, 18 first child
            const uint2 e = ent[i];
            const uint32_t p0 = poff[i], np = poff[i + 1] - p0;
            const uint32_t c0 = coff[i], nc = coff[i + 1] - c0;
            const uint32_t o0 = eop[i], o1 = eop[i + 1];
            const uint2 q = cs[i];
            PREP_ASSERT(p0 + np <= npar && c0 + nc <= npar && o0 <= o1 && o1 <= nops, PREP_T_ERECP);
            if (CHECK && oob) continue;   // no reads through a bad index (the document fails with PREP_BOUNDS)
            eh[2 * size_t(i)] = make_uint4(e.x, e.y, p0, np);
            eh[2 * size_t(i) + 1] = make_uint4(o0, o1 - o0, q.x, q.y + e.x);
            if (!P.short_rec) {
                const bool h0 = np > 0, h1 = np > 1;
                et[3 * size_t(i)] = make_uint4(c0, nc, h0 ? par[p0] : 0xFFFFFFFFu, h0 ? pent[p0] : 0xFFFFFFFFu);
                et[3 * size_t(i) + 1] = make_uint4(h0 ? pch[p0] : 0u, h0 ? pcnt[p0] : 0u, h1 ? pent[p0 + 1] : 0xFFFFFFFFu,
                                                   h1 ? pch[p0 + 1] : 0u);
                et[3 * size_t(i) + 2] = make_uint4(h1 ? pcnt[p0 + 1] : 0u, nc ? child[c0 + nc - 1] : 0xFFFFFFFFu,
                                                   nc ? child[c0] : 0xFFFFFFFFu, 0u);
            }
        }
    }
    // op runs: apply commands and the dense chain tables (LV | is_del per chain seq), one op run
    // per lane -- per entry, a history of few long entries (node_nodecc: 91 entries, 53k runs)
    // would leave most lanes idle behind one entry's runs.  A run's entry is the last entry whose
    // first run is at or below it: searched among the 64 entries from the previous chunk's last
    // run's entry in registers, by bisection past that window.  The window's chain pairs are
    // loaded with it and the runs themselves, one round trip per 64 runs, and a chain's table
    // offset comes from a register (lane = chain), not a dependent load.
    uint32_t n_ins = 0;
    {
        // software-pipelined: chunk j0 + 64's window and runs are requested before chunk j0's
        // stores (gfx9 counts stores in vmcnt: loads issued after them would wait for them)
        auto fetch = [&](uint32_t j0, uint32_t eb, uint32_t &we, uint2 &wq, uint4 &o) {
            const uint32_t wi = eb + l;
            const bool wv = wi < ne;
            we = wv ? eop[wi + 1] : 0xFFFFFFFFu;   // end of entry eb + l
            wq = wv ? cs[wi] : make_uint2(0, 0);
            o = j0 + l < nops ? ops[j0 + l] : make_uint4(0, 0, 0, 0);   // lv, len, pos, kind | fwd << 1
        };
        uint32_t ebase = 0, we = 0;
        uint2 wq = make_uint2(0, 0);
        uint4 o = make_uint4(0, 0, 0, 0);
        if (nops) fetch(0, 0, we, wq, o);
        for (uint32_t j0 = 0; j0 < nops; j0 += 64) {
            const uint32_t j = j0 + l;
            const bool live = j < nops;
            uint32_t c = 0;
#pragma unroll
            for (uint32_t st = 32; st >= 1; st >>= 1)
                if (uint32_t(__shfl(int(we), int(c + st - 1))) <= j) c += st;
            if (c == 63 && rdl(we, 63) <= j) c = 64;
            uint32_t lo = ebase + c, hi = live && c == 64 ? ne : lo;
            while (lo < hi) {   // past the window: first entry whose end is above j
                const uint32_t mid = (lo + hi) >> 1;
                if (eop[mid + 1] <= j) lo = mid + 1; else hi = mid;
            }
            const uint32_t i = lo;
            const uint32_t src = min(i - ebase, 63u);
            uint32_t qx = uint32_t(__shfl(int(wq.x), int(src))), qy = uint32_t(__shfl(int(wq.y), int(src)));
            if (live && i - ebase >= 64) {   // past the window
                const uint2 q = cs[i];
                qx = q.x; qy = q.y;
            }
            const uint32_t dch = uint32_t(__shfl(int(doff_l), int(qx & 63u)));
            const uint4 oc = o;
            ebase = rdl(i, min(nops - 1 - j0, 63u));
            if (j0 + 64 < nops) fetch(j0 + 64, ebase, we, wq, o);
            // the run's dense slots [dch + qy + lv, + len) lie inside the chain tables
            PREP_ASSERT(!live || (qx < nch && uint64_t(uint32_t(dch + qy + oc.x)) + oc.y <= D.n_lv), PREP_T_DENSE);
            const bool ok = live && (!CHECK || !oob);
            const uint32_t flag = (oc.w & 1u) ? TL_DEL : 0u;
            const uint32_t dst = dch + qy + oc.x;   // the run's first dense slot
            constexpr uint32_t LONG_RUN = 64;      // longer runs are filled by the whole wave
            if (ok) {
                const bool del = oc.w & 1u;
                opc[j] = Cmd{del ? (CMD_DEL | ((oc.w & 2u) ? 16u : 0u)) : uint32_t(CMD_INS), oc.x, oc.y, oc.z};
                if (!del) n_ins += oc.y;
            }
            if (ok && oc.y <= LONG_RUN) {
                // the run's dense slots (chain offset + seq0 - start + LV): 16-byte stores between
                // a scalar head and tail.  (Filling the chunk LV by LV across the lanes instead
                // measured no faster.)
                uint32_t *dp = dense + dst;
                uint32_t v = 0;
                for (; v < oc.y && (reinterpret_cast<uintptr_t>(dp + v) & 15u); v++) dp[v] = (oc.x + v) | flag;
                for (; v + 4 <= oc.y; v += 4) {
                    const uint32_t b = oc.x + v;
                    *reinterpret_cast<uint4 *>(dp + v) = make_uint4(b | flag, (b + 1) | flag, (b + 2) | flag, (b + 3) | flag);
                }
                for (; v < oc.y; v++) dp[v] = (oc.x + v) | flag;
            }
            // a long run (node_nodecc's pastes: thousands of LVs) by every lane, 256 bytes per
            // store instead of one lane's serial stores setting the chunk's time
            for (uint64_t m = ballot(ok && oc.y > LONG_RUN); m; m &= m - 1) {
                const uint32_t k = ctz(m);
                const uint32_t d0 = rdl(dst, k), lv0 = rdl(oc.x, k), len = rdl(oc.y, k), fl = rdl(flag, k);
                for (uint32_t v = l; v < len; v += 64) dense[d0 + v] = (lv0 + v) | fl;
            }
        }
    }
    if (report_oob()) return;
#ifdef DTGPU_PREP_PROF
    const uint64_t T5 = wall_clock64();
#endif
    bool tip_miss = false;
    for (uint32_t t = l; t < D.n_ver; t += 64) {   // tips and their entries
        const uint32_t v = P.d_ver[D.d_ver + t];
        const uint32_t e = entry_of(ent, ne, v);
        if (e >= ne || v < ent[e].x || v >= ent[e].y) tip_miss = true;   // host path: ErrCheckout
        *reinterpret_cast<uint2 *>(P.tip + 2 * (D.o_tip + t)) = make_uint2(v, e);
    }
    if (ballot(tip_miss)) {
        if (l == 0) { R.status = PREP_BAD; P.results[doc] = R; }
        return;
    }
    // agent runs with name ranks (byte-wise name order; names are distinct): each agent's rank
    // once (lane per agent), into the scatter's owner scratch (free by now) when it fits, then
    // one lookup per run; otherwise ranked per run
    const uint2 *names = reinterpret_cast<const uint2 *>(P.d_agents) + D.d_agent;
    const uint8_t *in = P.in + D.d_in;
    // (the LDS is free by now: the ranks go there when they fit -- it is at least the erec
    // staging's 32 records -- else into the owner scratch)
    const uint32_t lds_words = max((P.max_entries + 1) / 2, 32u * EREC_WORDS);
    uint32_t *rk = D.n_agents <= lds_words ? lfw : owner;
    if (D.n_agents <= lds_words || D.n_agents <= ((npar + 1) & ~1u)) {
        for (uint32_t a = l; a < D.n_agents; a += 64) {
            const uint2 me = names[a];
            uint32_t rank = 0;
            for (uint32_t b = 0; b < D.n_agents; b++) {
                const uint2 o = names[b];
                const uint32_t n = min(o.y, me.y);
                int cmp = 0;
                for (uint32_t x = 0; x < n && !cmp; x++) {
                    const uint32_t cb = in[o.x + x], cm = in[me.x + x];
                    cmp = cb < cm ? -1 : cb > cm ? 1 : 0;
                }
                if (!cmp) cmp = o.y < me.y ? -1 : o.y > me.y ? 1 : 0;
                rank += cmp < 0 ? 1u : 0u;
            }
            rk[a] = rank;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        for (uint32_t k = l; k < D.n_aruns; k += 64) {
            const uint4 a = ar[k];   // lv, len, agent, seq
            *reinterpret_cast<uint4 *>(P.aruns + 4 * (D.o_arun + k)) = make_uint4(a.x, rk[a.z], a.w, a.z);
        }
    } else {
        for (uint32_t k = l; k < D.n_aruns; k += 64) {
            const uint4 a = ar[k];   // lv, len, agent, seq
            const uint2 me = names[a.z];
            uint32_t rank = 0;
            for (uint32_t b = 0; b < D.n_agents; b++) {
                const uint2 o = names[b];
                const uint32_t n = min(o.y, me.y);
                int cmp = 0;
                for (uint32_t x = 0; x < n && !cmp; x++) {
                    const uint32_t cb = in[o.x + x], cm = in[me.x + x];
                    cmp = cb < cm ? -1 : cb > cm ? 1 : 0;
                }
                if (!cmp) cmp = o.y < me.y ? -1 : o.y > me.y ? 1 : 0;
                rank += cmp < 0 ? 1u : 0u;
            }
            *reinterpret_cast<uint4 *>(P.aruns + 4 * (D.o_arun + k)) = make_uint4(a.x, rank, a.w, a.z);
        }
    }
    for (int d = 32; d >= 1; d >>= 1) n_ins += uint32_t(__shfl_xor(int(n_ins), d));
    R.status = PREP_OK;
    R.n_chains = nch;
    R.n_ins = n_ins;
    if (l == 0) P.results[doc] = R;
#ifdef DTGPU_PREP_PROF   // phase split (100 MHz wall clock) of two documents: profiles/r1_v19
    const uint64_t T6 = wall_clock64();
    if (l == 0 && (doc == 0 || doc == P.n_docs / 2))
        printf("PREPPROF doc %u ne %u npar %u parents %llu scatter %llu firstop %llu chains %llu outputs %llu tail %llu\n", doc, ne, npar,
               (unsigned long long)(T1 - T0), (unsigned long long)(T2 - T1), (unsigned long long)(T3 - T2),
               (unsigned long long)(T4 - T3), (unsigned long long)(T5 - T4), (unsigned long long)(T6 - T5));
#endif
}


// ---- chain_kernel: the causal-chain decomposition of CHAIN_DOCS documents per wave ---------------
// Phase 3 of prep_kernel (see there) for documents of at most CHAIN_GROUP chains, each document on
// its own 16-lane group (lane = chain): the decomposition is one sequential walk over the
// entries, so a wave per document spent most of its issue slots on one document's scalar chain
// of steps; four documents now share every instruction.  Group-uniform values live in VGPRs,
// reads across a group's lanes are permutes within the group.  A document that opens a 17th
// chain is left to the second half of prep_kernel (its flag stays 1).  Rows are stored whole
// (min(CHAIN_GROUP, row stride) words: the planner reads chains < its count), so no keep-list is needed.
__device__ __forceinline__ uint32_t gsh(uint32_t v, uint32_t src) { return uint32_t(__shfl(int(v), int(src))); }

__global__ __launch_bounds__(64) void chain_kernel(PrepParams P) {
    // RING: the last 2 G entries' rows and {entry, chain, sd} in LDS.  A block of G entries goes
    // out to HBM (rows, chain pairs) in the middle of the next block, and the fence that makes it
    // readable waits at the start of the block after that: by then the stores are done, so
    // neither the fence nor the next block's loads (vmcnt counts stores) wait on a store in
    // flight.  Parents up to 2 G entries back come from the ring and the block registers.
    constexpr uint32_t G = CHAIN_GROUP, RING = 2 * G, FLUSH_AT = G / 2 - 1;
    // per group: RING rows x W words, RING x {entry, chain, sd}.  W: the batch's widest row
    // stride up to G (every document here has fewer chains than its stride, so a row's words
    // past W are zero)
    extern __shared__ uint32_t csh[];
    const uint32_t W = chain_ring_width(P.chain_w);
    const uint32_t l = lane(), g = l / G, c = l % G, base = g * G;
    uint32_t *rr = csh + g * (RING * W + 3 * RING), *rm = rr + RING * W;
    const uint32_t li = blockIdx.x * CHAIN_DOCS + g;
    bool live = li < P.n_docs;
    const uint32_t doc = live ? (P.doc_list ? P.doc_list[li] : li) : 0u;
    live = live && P.chain_flag[doc] == 1;
    const PrepDesc D = P.docs[doc];
    const uint32_t ne = live ? D.ne : 0u, npar = D.n_par;
    const uint2 *ent = reinterpret_cast<const uint2 *>(P.d_ent) + D.d_ent;
    const uint32_t *poff = P.d_poff + D.d_poff;
    const uint32_t *par_in = P.d_par + D.d_par;
    const uint32_t *pent = P.pent + D.o_par;
    uint32_t *rows = P.rows + D.o_rows;
    const uint32_t rs = D.row_stride;
    uint32_t *doff = P.doff + D.o_doff;
    uint2 *cs = reinterpret_cast<uint2 *>(P.scr + D.o_scr + ((npar + 1) & ~1u));
    for (uint32_t r = c; r < RING; r += G) rm[3 * r] = 0xFFFFFFFFu;
    __builtin_amdgcn_wave_barrier();
    uint32_t maxne = ne;
    for (int d = 32; d >= 1; d >>= 1) maxne = max(maxne, uint32_t(__shfl_xor(int(maxne), d)));
    // prev_sd: seq0 - start of entry i - 1, held by the lane of its chain (the one lane that
    // reads it); the ring's {entry, chain, sd} are written by that lane too, so no lane of the
    // group waits for a permute of the chain's length
    uint32_t clen = 0, nch = 0, prev_row = 0, prev_chain = 0, prev_sd = 0;
    uint32_t bk0 = 0, bk1 = 0, bs = 0, be = 0;                     // lane c: entry (i & ~15) + c
    uint32_t pblk = 0xFFFFFFFFu, ppa = 0, ppe = 0;                 // lane c: parent slot pblk + c
    bool ok = live;
    // entries [at, end) out: rows and chain pairs from the ring
    auto flush = [&](uint32_t at, uint32_t end) {
        if (c < rs)
            for (uint32_t r = at; r < end; r++) rows[size_t(r) * rs + c] = c < W ? rr[(r & (RING - 1)) * W + c] : 0u;
        if (at + c < end) {
            const uint32_t sl = (at + c) & (RING - 1);
            cs[at + c] = make_uint2(rm[3 * sl + 1], rm[3 * sl + 2]);
        }
    };
    for (uint32_t i = 0; i < maxne; i++) {
        const bool on = ok && i < ne;
        const uint32_t ib = i & (G - 1), at = i & ~(G - 1);
        if (ib == 0) {
            wave_fence();   // the block flushed in the middle of the last one is readable
            if (on) {
                const uint32_t j = min(i + c, ne - 1);
                bk0 = poff[j];
                bk1 = poff[j + 1];
                const uint2 se = ent[j];
                bs = se.x;
                be = se.y;
                wait_vm();
            }
        }
        if (on && ib == FLUSH_AT && at) flush(at - G, at);
        if (on) {
            const uint32_t k0 = gsh(bk0, base + ib), k1 = gsh(bk1, base + ib);
            uint32_t row = 0, first_chain = 0xFFFFFFFFu;
            for (uint32_t k = k0; k < k1; k++) {
                if ((k & ~(G - 1)) != pblk) {
                    pblk = k & ~(G - 1);
                    const uint32_t x = min(pblk + c, npar - 1);
                    ppa = par_in[x];
                    ppe = pent[x];
                    wait_vm();
                }
                const uint32_t p = gsh(ppa, base + (k & (G - 1))), pe = gsh(ppe, base + (k & (G - 1)));
                uint32_t prow, pc, psd;
                if (pe + 1 == i) {
                    prow = prev_row; pc = prev_chain; psd = prev_sd;
                } else {
                    const uint32_t slot = pe & (RING - 1);
                    if (rm[3 * slot] == pe) {
                        prow = c < W ? rr[slot * W + c] : 0u; pc = rm[3 * slot + 1]; psd = rm[3 * slot + 2];
                    } else {   // more than RING entries back: flushed and fenced
                        prow = c < rs ? rows[size_t(pe) * rs + c] : 0u;
                        const uint2 q = cs[pe];
                        wait_vm();
                        pc = q.x; psd = q.y;
                    }
                }
                row = max(row, prow);
                if (c == pc) row = max(row, psd + p + 1);
                if (k == k0) first_chain = pc;
            }
            uint32_t ch = 0xFFFFFFFFu;
            const uint64_t eqm = ballot(row == clen);   // (a ballot, not two lane permutes)
            if (first_chain != 0xFFFFFFFFu && ((eqm >> (base + first_chain)) & 1ull)) ch = first_chain;
            if (ch == 0xFFFFFFFFu) {
                const uint32_t m = uint32_t(ballot(c < nch && row == clen) >> base) & 0xFFFFu;
                if (m) ch = uint32_t(__ffs(int(m)) - 1);
            }
            if (ch == 0xFFFFFFFFu) {
                if (nch == G || nch == rs) ok = false;   // a 17th chain: prep_kernel's second half redoes it
                else ch = nch++;
            }
            if (ok) {
                const uint32_t s = gsh(bs, base + ib), e = gsh(be, base + ib);
                const uint32_t slot = i & (RING - 1);
                if (c == ch) {   // seq0 - start = the chain's length so far - start
                    prev_sd = clen - s;
                    rm[3 * slot] = i; rm[3 * slot + 1] = ch; rm[3 * slot + 2] = clen - s;
                    clen += e - s;
                }
                prev_row = row; prev_chain = ch;
                if (c < W) rr[slot * W + c] = row;
            }
        }
    }
    if (ok && ne) {   // the blocks not out yet: the last one, and the one before unless flushed
        const uint32_t at = (ne - 1) & ~(G - 1);
        if (at && ((ne - 1) & (G - 1)) < FLUSH_AT) flush(at - G, at);
        flush(at, ne);
        wave_fence();
    }
    if (ok) {   // the chain tables' offsets: exclusive prefix of the chain lengths
        uint32_t v = c < nch ? clen : 0u;
        for (uint32_t d = 1; d < G; d <<= 1) {
            const uint32_t o = uint32_t(__shfl_up(int(v), d, int(G)));
            if (c >= d) v += o;
        }
        const uint32_t ex = v - (c < nch ? clen : 0u);
        if (c < nch) doff[c] = ex;
        if (c == G - 1) doff[nch] = v;
        if (c == 0) doff[PREP_MAX_CHAINS] = nch;
        if (c == 0) P.chain_flag[doc] = 2;
    }
}


// ---- cut_kernel: the cut planning of one cut document per wave (dt_prep.hpp CutParams) -----------
// The same decisions as dtgpu_api.cpp cut_ranges / plan_segments, lane-parallel:
//   entry k is a cut range's entry when the prefix's frontier is empty there -- every earlier
//   entry's last LV is named as a parent by some entry up to k: max over j < k of nxt(j) <= k,
//   nxt(j) = the first entry naming j's last LV -- and the range is [start + 1, min(end, 1 + the
//   smallest parent of every later entry)];
//   the cuts are the op-run starts inside a range nearest to the op runs where the cost (SegPlan::w_op,
//   dt_prep.hpp) reaches each equal share (nearest first, the earlier of two at the same
//   distance), a later one only a quarter share of the cost past the previous one, none a
//   quarter share from the end;
//   a segment's placeholders bound the text at its start: min(inserts, inserts - deletes + the
//   deletes not inside one range).
// (the cut kernel's scratch is written by stores and memory-side atomics and read back by other
// lanes: an agent-scope fence also drops the CU's L1 lines, so no read meets a stale one)
__device__ __forceinline__ void agent_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent"); }
__device__ __forceinline__ uint32_t scan_max_excl(uint32_t v) {   // exclusive prefix max
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = uint32_t(__shfl_up(int(v), d));
        if (lane() >= uint32_t(d)) v = max(v, o);
    }
    const uint32_t e = uint32_t(__shfl_up(int(v), 1));
    return lane() ? e : 0u;
}
__device__ __forceinline__ int32_t scan_min_suffix(int32_t v) {   // inclusive suffix min
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int32_t o = __shfl_down(v, d);
        if (lane() + uint32_t(d) < 64u) v = min(v, o);
    }
    return v;
}
// the last range whose first cut is <= v (ranges ascending), or nr
__device__ __forceinline__ uint32_t range_of(const uint2 *rng, uint32_t nr, uint32_t v) {
    uint32_t lo = 0, hi = nr;   // first range with .x > v
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rng[mid].x <= v) lo = mid + 1; else hi = mid;
    }
    return lo ? lo - 1 : nr;
}

constexpr uint32_t CUT_WAVES = 4;   // the op-run pass (step 5) on four waves: a long document's 53k runs
__global__ __launch_bounds__(64 * CUT_WAVES) void cut_kernel(CutParams P) {
    if (blockIdx.x >= P.n_groups) return;
    const uint32_t l = lane(), w = threadIdx.x / 64;
    __shared__ uint32_t s_pick[64], s_np, s_nr, s_at[3][64], s_tot[CUT_WAVES][3], s_ok;
    const SegGroup G = P.groups[blockIdx.x];
    const SegPlan SP = P.plans[blockIdx.x];
    const uint32_t d = P.seg_docs[G.first];
    const PrepDesc D = P.pdocs[d];
    const uint32_t ne = D.ne, nop = D.n_ops, S = G.count, T = SP.n_targets;   // segments; equal-share targets
    // declined: the host plan's ranges (staging reserved the arenas from it; DOC_CUT_HOST marks it)
    uint32_t *sized = P.sized ? P.sized + size_t(blockIdx.x) * CUT_SIZED_WORDS : nullptr;
    auto host_ranges = [&]() {
        if (sized) { if (threadIdx.x == 0) sized[0] = 0; return; }   // sizing: not cut
        if (w != 0 || l >= S || l >= 64) return;
        const SegCap cap = P.caps[G.first + l];
        DocDesc *dd = P.docs + P.seg_docs[G.first + l];
        dd->seg_lo = cap.lo;
        dd->seg_hi = cap.hi;
        dd->seg_u = cap.u;
        dd->flags |= DOC_CUT_HOST;
    };
    if (S < 2 || S > 64 || T < S || ne == 0 || nop == 0 || ne > P.max_ne) { host_ranges(); return; }   // (staging makes none such)
    // short documents: the op-run pass on one wave (the other waves take empty parts: every wave
    // stays to the workgroup's barriers)
    const uint32_t NW = nop >= 4096 ? CUT_WAVES : 1u;
    const uint2 *ent = reinterpret_cast<const uint2 *>(P.d_ent) + D.d_ent;
    const uint32_t *poff = P.d_poff + D.d_poff, *par = P.d_par + D.d_par;
    const uint4 *ops = reinterpret_cast<const uint4 *>(P.d_ops) + D.d_op;   // lv, len, pos, kind (bit 0: delete)
    extern __shared__ uint32_t nxt[];   // per entry: the first entry naming its last LV as a parent
    const uint32_t *pent = P.pent ? P.pent + D.o_par : nullptr;   // prep's first half: each parent's entry (or searched)
    int32_t *suf = reinterpret_cast<int32_t *>(P.scr + SP.scr_off);        // ne + 1
    uint2 *rng = reinterpret_cast<uint2 *>(P.scr + SP.scr_off + ((uint64_t(ne) + 2) & ~1ull));   // <= ne ranges

    if (threadIdx.x == 0) s_ok = 0;
    __syncthreads();
    if (w == 0) {
    // 1. nxt (LDS atomics) and each entry's smallest parent (-1: ROOT)
    for (uint32_t j = l; j < ne; j += 64) nxt[j] = 0xFFFFFFFFu;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (uint32_t e = l; e < ne; e += 64) {
        const uint32_t k0 = poff[e], k1 = poff[e + 1];
        int32_t mp = k0 == k1 ? -1 : 0x7FFFFFFF;
        for (uint32_t k = k0; k < k1; k++) {
            const uint32_t p = par[k], j = pent ? pent[k] : entry_of(ent, e, p);
            mp = min(mp, int32_t(p));
            if (j < e && p + 1 == ent[j].y) atomicMin(&nxt[j], e);
        }
        suf[e] = mp;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    agent_fence();
    // 2. suffix minima of the smallest parents (suf[k] = over entries >= k; suf[ne] = none)
    {
        int32_t carry = 0x7FFFFFFF;
        for (int32_t c0 = int32_t((ne - 1) & ~63u); c0 >= 0; c0 -= 64) {
            const uint32_t k = uint32_t(c0) + l;
            const int32_t v = scan_min_suffix(k < ne ? suf[k] : 0x7FFFFFFF);
            if (k < ne) suf[k] = min(v, carry);
            carry = min(carry, __shfl(v, 0));
        }
        if (l == 0) suf[ne] = 0x7FFFFFFF;
    }
    agent_fence();
    // 3. the cut ranges, compacted in entry order
    uint32_t nr = 0;
    {
        uint32_t carry = 0;   // max nxt over the entries before the chunk
        for (uint32_t c0 = 0; c0 < ne; c0 += 64) {
            const uint32_t k = c0 + l;
            const bool live = k < ne;
            const uint2 se = live ? ent[k] : make_uint2(0, 1);
            const uint32_t v = live ? nxt[k] : 0u;
            const uint32_t before = max(carry, scan_max_excl(v));
            bool ok = false;
            uint2 r = make_uint2(0, 0);
            if (live && before <= k) {
                const int32_t sn = suf[k + 1];
                const int64_t lim = sn == 0x7FFFFFFF ? int64_t(se.y) : min(int64_t(se.y), int64_t(sn) + 1);
                ok = lim >= int64_t(se.x) + 1;
                r = make_uint2(se.x + 1, uint32_t(lim));
            }
            const uint64_t m = ballot(ok);
            if (ok) rng[nr + popc(m & lt_mask())] = r;
            nr += popc(m);
            uint32_t cm = live ? v : 0u;
#pragma unroll
            for (int dd = 32; dd >= 1; dd >>= 1) cm = max(cm, uint32_t(__shfl_xor(int(cm), dd)));
            carry = max(carry, cm);
        }
    }
    agent_fence();
    if (nr != 0) {
    auto in_cut = [&](uint32_t v) {
        const uint32_t i = range_of(rng, nr, v);
        return i < nr && v <= rng[i].y;
    };
    // 4. the cuts: op-run starts in a range, nearest to where the cost reaches k / T of the total
    const uint4 lastop = ops[nop - 1];
    const uint64_t total = uint64_t(SP.w_op) * nop + lastop.x + lastop.y, q4c = total / (4ull * T);
    auto cost = [&](uint32_t j) { return uint64_t(SP.w_op) * j + ops[j].x; };
    uint32_t tj = 0;   // lane k: the first op run whose cost reaches k * total / T (a bisection each)
    if (l >= 1 && l < T) {
        const uint64_t tc = uint64_t(l) * total / T;
        uint32_t lo = 0, hi = nop;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (cost(mid) < tc) lo = mid + 1; else hi = mid;
        }
        tj = lo;
    }
    uint32_t picks = 0, npick = 0;   // lane i of picks: the i-th cut's op run
    uint64_t lastc = 0;
    for (uint32_t k = 1; k < T; k++) {
        const uint32_t target = rdl(tj, k);
        const uint32_t dmax = nop / (2 * T) + 1;
        uint32_t best = 0xFFFFFFFFu;
        for (uint32_t d0 = 0; d0 <= dmax && d0 < nop && best == 0xFFFFFFFFu; d0 += 32) {
            const uint32_t dd = d0 + (l >> 1);
            const uint32_t j = (l & 1u) ? target + dd : target - min(target, dd);
            const bool ok = dd <= dmax && dd < nop && j > 0 && j < nop && in_cut(ops[j].x);
            const uint64_t m = ballot(ok);
            if (m) best = rdl(j, ctz(m));
        }
        if (best != 0xFFFFFFFFu) {
            const uint64_t bc = cost(best);
            if (npick == 0 || bc > lastc + q4c) {
                picks = l == npick ? best : picks;
                npick++;
                lastc = bc;
            }
        }
    }
    while (npick && total - cost(rdl(picks, npick - 1)) < q4c) npick--;
    if (sized ? npick >= 1 : npick + 1 == S) {   // else not the staged segments (the host plan's ranges then)
        if (l < npick) s_pick[l] = picks;
        if (l == 0) { s_np = npick; s_nr = nr; s_ok = 1; }
    }
    }   // nr != 0
    }
    __syncthreads();
    if (!s_ok) { host_ranges(); return; }
    // 5. inserts, deletes and concurrent deletes before each cut (exclusive prefix sums), the op
    //    runs split in four contiguous parts, one per wave; each part's sums are offset by the
    //    parts before it afterwards
    const uint32_t npick = s_np, nr = s_nr;
    const uint32_t picks = l < npick ? s_pick[l] : 0u;
    uint32_t at_ins = 0, at_del = 0, at_dc = 0;   // lane i: before the i-th cut
    uint32_t tot_ins = 0;
    {
        // a delete run is inside one range or concurrent: the runs' LVs ascend, so each chunk
        // looks its runs up among the 64 ranges from the previous chunk's last one (one load,
        // a search by lane permutes), a global bisection only past that window
        const uint32_t part = ((nop + NW - 1) / NW + 63) & ~63u;
        const uint32_t b0 = w < NW ? min(nop, w * part) : nop, b1 = min(nop, b0 + part);
        uint32_t ci = 0, cd = 0, cc = 0, pi = 0;
        const uint32_t last_pick = rdl(picks, npick - 1);   // past it only the inserts are summed
        uint32_t rc = b0 < b1 ? range_of(rng, nr, ops[b0].x) : 0u;
        if (rc >= nr) rc = 0;
        while (pi < npick && rdl(picks, pi) < b0) pi++;
        for (uint32_t c0 = b0; c0 < b1; c0 += 64) {
            const uint32_t j = c0 + l;
            const uint4 o = j < b1 ? ops[j] : make_uint4(0xFFFFFFFFu, 0, 0, 0);
            const bool look = c0 <= last_pick;
            const uint2 wr = look && rc + l < nr ? rng[rc + l] : make_uint2(0xFFFFFFFFu, 0);
            uint32_t c = 0;   // window ranges whose first cut is <= the run's LV
#pragma unroll
            for (uint32_t st = 32; st >= 1; st >>= 1)
                if (uint32_t(__shfl(int(wr.x), int(c + st - 1))) <= o.x) c += st;
            if (c == 63 && rdl(wr.x, 63) <= o.x) c = 64;
            uint32_t ri = c ? rc + c - 1 : nr, rhi = uint32_t(__shfl(int(wr.y), int(c ? c - 1 : 0)));
            if (look && j < b1 && ((c == 64 && rc + 64 < nr) || (c == 0 && rc > 0))) {   // outside the window
                ri = range_of(rng, nr, o.x);
                rhi = ri < nr ? rng[ri].y : 0u;
            }
            uint32_t vi = 0, vd = 0, vc = 0;
            if (j < b1) {
                if (o.w & 1u) {
                    vd = o.y;
                    if (!(ri < nr && uint64_t(o.x) + o.y <= rhi)) vc = o.y;
                } else {
                    vi = o.y;
                }
            }
            const uint32_t rl = rdl(ri, min(b1 - 1 - c0, 63u));
            if (rl < nr) rc = rl;
            const uint32_t si = scan_incl(vi), sd = scan_incl(vd), sc = scan_incl(vc);
            while (pi < npick) {
                const uint32_t pj = rdl(picks, pi);
                if (pj >= c0 + 64 || pj >= b1) break;
                const uint32_t t = pj - c0;   // exclusive prefix (within the part) at lane t
                if (l == 0) {
                    s_at[0][pi] = ci + rdl(si, t) - rdl(vi, t);
                    s_at[1][pi] = cd + rdl(sd, t) - rdl(vd, t);
                    s_at[2][pi] = cc + rdl(sc, t) - rdl(vc, t);
                }
                pi++;
            }
            ci += rdl(si, 63); cd += rdl(sd, 63); cc += rdl(sc, 63);
        }
        if (l == 0) { s_tot[w][0] = ci; s_tot[w][1] = cd; s_tot[w][2] = cc; }
        __syncthreads();
        if (w) return;
        // offsets: every part before the cut's own
        uint32_t oi = 0, od = 0, oc = 0, pw = 0;
        const uint32_t pk = picks;
        for (uint32_t v = 0; v < NW; v++) {
            const uint32_t vb0 = min(nop, v * part);
            if (l < npick && pk >= vb0 + part) { oi += s_tot[v][0]; od += s_tot[v][1]; oc += s_tot[v][2]; }
            (void)pw;
        }
        if (l < npick) { at_ins = oi + s_at[0][l]; at_del = od + s_at[1][l]; at_dc = oc + s_at[2][l]; }
        for (uint32_t v = 0; v < NW; v++) tot_ins += s_tot[v][0];
    }
    // 6. each segment's range and placeholder bound, against what staging reserved (sizing:
    //    written out for staging to reserve)
    if (sized) {
        const uint32_t Sr = npick + 1, k = l;
        const uint32_t pprev = uint32_t(__shfl(int(picks), int(k ? k - 1 : 0)));
        const uint32_t ai = uint32_t(__shfl(int(at_ins), int(k ? k - 1 : 0)));
        const uint32_t ad = uint32_t(__shfl(int(at_del), int(k ? k - 1 : 0)));
        const uint32_t ac = uint32_t(__shfl(int(at_dc), int(k ? k - 1 : 0)));
        const uint32_t ins_lo = k ? ai : 0u;
        const uint32_t ins_hi = k + 1 < Sr ? at_ins : tot_ins;
        if (k < Sr) {
            sized[1 + 4 * k] = k ? ops[pprev].x : 0u;
            sized[2 + 4 * k] = k + 1 < Sr ? ops[picks].x : 0xFFFFFFFFu;
            sized[3 + 4 * k] = k ? uint32_t(max<int64_t>(0, min(int64_t(ai), int64_t(ai) - int64_t(ad) + int64_t(ac)))) : 0u;
            sized[4 + 4 * k] = ins_hi - ins_lo;
        }
        if (l == 0) sized[0] = Sr;
        return;
    }
    bool fits = true;
    for (uint32_t k = 0; k < S; k++) {
        const uint32_t ins_lo = k ? rdl(at_ins, k - 1) : 0u;
        const uint32_t ins_hi = k + 1 < S ? rdl(at_ins, k) : tot_ins;
        const int64_t ai = k ? int64_t(rdl(at_ins, k - 1)) : 0, ad = k ? int64_t(rdl(at_del, k - 1)) : 0,
                      ac = k ? int64_t(rdl(at_dc, k - 1)) : 0;
        const uint32_t u = k ? uint32_t(max<int64_t>(0, min(ai, ai - ad + ac))) : 0u;
        const SegCap cap = P.caps[G.first + k];
        fits = fits && u <= cap.u && ins_hi - ins_lo <= cap.ins;
    }
    if (!fits) { host_ranges(); return; }
    {   // lane k writes segment k's descriptor fields
        const uint32_t k = l;
        const uint32_t pprev = uint32_t(__shfl(int(picks), int(k ? k - 1 : 0)));   // cut before segment k
        const uint32_t ai = uint32_t(__shfl(int(at_ins), int(k ? k - 1 : 0)));
        const uint32_t ad = uint32_t(__shfl(int(at_del), int(k ? k - 1 : 0)));
        const uint32_t ac = uint32_t(__shfl(int(at_dc), int(k ? k - 1 : 0)));
        if (k < S) {
            const uint32_t lo = k ? ops[pprev].x : 0u;
            const uint32_t hi = k + 1 < S ? ops[picks].x : 0xFFFFFFFFu;
            const uint32_t u = k ? uint32_t(max<int64_t>(0, min(int64_t(ai), int64_t(ai) - int64_t(ad) + int64_t(ac)))) : 0u;
            DocDesc *dd = P.docs + P.seg_docs[G.first + k];
            dd->seg_lo = lo;
            dd->seg_hi = hi;
            dd->seg_u = u;
            dd->flags &= ~DOC_CUT_HOST;
        }
    }
}


}  // namespace prep

int launch_cut(const CutParams &p, void *stream) {
    if (!p.n_groups) return 0;
    const size_t lds = size_t(p.max_ne) * 4;
    // the entry table beside ~1.1 KB of static LDS: past the default 64 KiB of dynamic LDS the
    // per-function limit is raised (staging cuts documents of at most PLAN_MAX_LDS_ENTRIES entries)
    if (lds + 2048 > 160 * 1024) return 66;
    if (lds + 2048 > 64 * 1024 &&
        hipFuncSetAttribute(reinterpret_cast<const void *>(&prep::cut_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int(lds)) != hipSuccess)
        return 66;
    hipLaunchKernelGGL(prep::cut_kernel, dim3(p.n_groups), dim3(64 * prep::CUT_WAVES), lds, reinterpret_cast<hipStream_t>(stream), p);
    return launch_error() == hipSuccess ? 0 : 66;
}

namespace prep {
__global__ void pass_mark_kernel() {}
}  // namespace prep
int launch_pass_mark(void *stream) {
    hipLaunchKernelGGL(prep::pass_mark_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream));
    return launch_error() == hipSuccess ? 0 : 66;
}

int launch_prep_stage(const PrepParams &p, void *stream, int stage) {
    if (!p.n_docs) return 0;
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const size_t cw = (size_t(p.max_entries) + 1) / 2, rw = 32 * EREC_WORDS;   // >= the ring (8 x 64 + 24)
    const size_t lds = (cw > rw ? cw : rw) * 4;
    PrepParams q = p;
    if (stage == 2) {
        const size_t clds = size_t(CHAIN_DOCS) * chain_lds_words(p.chain_w) * 4;
        hipLaunchKernelGGL(prep::chain_kernel, dim3((p.n_docs + CHAIN_DOCS - 1) / CHAIN_DOCS), dim3(64), clds, st, q);
    } else {
        q.mode = stage == 1 ? 1u : 2u;
        hipLaunchKernelGGL(prep::prep_kernel<false>, dim3(p.n_docs), dim3(64), lds, st, q);
    }
    return launch_error() == hipSuccess ? 0 : 66;
}

int launch_prep(const PrepParams &p, void *stream) {
    if (!p.n_docs) return 0;
    // LDS: the child counts (u16 per entry), later the chain decomposition's ring (8 rows + meta)
    const size_t cw = (size_t(p.max_entries) + 1) / 2, rw = 32 * EREC_WORDS;   // >= the ring (8 x 64 + 24)
    const size_t lds = (cw > rw ? cw : rw) * 4;
    const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    PrepParams q = p;
    if (p.check || !p.chain_flag) {   // one launch (the debug kernel always)
        q.mode = 0;
        if (p.check) hipLaunchKernelGGL(prep::prep_kernel<true>, dim3(p.n_docs), dim3(64), lds, st, q);
        else hipLaunchKernelGGL(prep::prep_kernel<false>, dim3(p.n_docs), dim3(64), lds, st, q);
        return launch_error() == hipSuccess ? 0 : 66;
    }
    // first half, the chain decomposition four documents per wave, second half
    q.mode = 1;
    hipLaunchKernelGGL(prep::prep_kernel<false>, dim3(p.n_docs), dim3(64), lds, st, q);
    const size_t clds = size_t(CHAIN_DOCS) * chain_lds_words(p.chain_w) * 4;
    hipLaunchKernelGGL(prep::chain_kernel, dim3((p.n_docs + CHAIN_DOCS - 1) / CHAIN_DOCS), dim3(64), clds, st, q);
    q.mode = 2;
    hipLaunchKernelGGL(prep::prep_kernel<false>, dim3(p.n_docs), dim3(64), lds, st, q);
    return launch_error() == hipSuccess ? 0 : 66;
}

}  // namespace dtgpu
