//! `dtgpu-sys`: Rust FFI to libdtgpu, the MI355X (gfx950) batch checkout engine for
//! diamond-types oplogs.  Raw `extern "C"` declarations of include/dtgpu.h (checked against the
//! header by tests/test_ffi_crate.py) plus safe wrappers shaped like the reference's
//! `ListOpLog` API (src/list/oplog.rs, src/list/merge.rs).  Linked statically by build.rs.
#![allow(non_camel_case_types)]
use std::os::raw::{c_char, c_int, c_void};

#[repr(C)]
pub struct dtgpu_oplog {
    _p: [u8; 0],
}
#[repr(C)]
pub struct dtgpu_batch {
    _p: [u8; 0],
}
#[repr(C)]
pub struct dtgpu_decoded {
    _p: [u8; 0],
}
#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct dtgpu_doc_result {
    pub status: u32,
    pub reserved: u32,
    pub text_len: u64,
    pub text_hash: u64,
    pub n_lv: u64,
}
#[repr(C)]
#[derive(Default, Clone, Copy, Debug)]
pub struct dtgpu_batch_opts {
    pub ignore_crc: c_int,
    pub host_threads: c_int,
    pub device: c_int,
    pub flags: u32,      // DTGPU_OPT_*
    pub seg_ops: u32,    // 0: default
    pub seg_max: u32,    // 0: default
    pub lds_fill: u32,   // 0: default
}
pub const DTGPU_OPT_NO_FAST_FORWARD: u32 = 1;
pub const DTGPU_OPT_NO_SEGMENTS: u32 = 2;
pub const DTGPU_OPT_HOST_PLAN: u32 = 4;
pub const DTGPU_OPT_NO_SPLIT: u32 = 8;
pub const DTGPU_OPT_NO_CRITICAL: u32 = 16;
pub const DTGPU_OPT_DEBUG: u32 = 32;
pub const DTGPU_OPT_PASS_MARK: u32 = 64;
pub type dtgpu_status = c_int;
pub const DTGPU_OK: dtgpu_status = 0;
// EncodeOptions (src/list/encoding/encode_oplog.rs:88-130) as dtgpu_oplog_encode flags
pub const DTGPU_ENCODE_STORE_INSERTED_CONTENT: u32 = 1;
pub const DTGPU_ENCODE_COMPRESS_CONTENT: u32 = 2;
pub const DTGPU_ENCODE_STORE_START_BRANCH_CONTENT: u32 = 4;
pub const DTGPU_ENCODE_FULL: u32 = 7;
pub const DTGPU_ENCODE_PATCH: u32 = 3;

extern "C" {
    // ListOpLog (src/list/oplog.rs, src/list/encoding/decode_oplog.rs:447)
    pub fn dtgpu_oplog_load(bytes: *const u8, len: usize, ignore_crc: c_int, out: *mut *mut dtgpu_oplog) -> dtgpu_status;
    pub fn dtgpu_oplog_new() -> *mut dtgpu_oplog;
    pub fn dtgpu_oplog_free(oplog: *mut dtgpu_oplog);
    pub fn dtgpu_oplog_decode_and_add(oplog: *mut dtgpu_oplog, bytes: *const u8, len: usize, ignore_crc: c_int,
                                      frontier: *mut u64, cap: usize, n_frontier: *mut usize) -> dtgpu_status;
    pub fn dtgpu_oplog_get_or_create_agent_id(oplog: *mut dtgpu_oplog, name: *const c_char, name_len: usize) -> i32;
    pub fn dtgpu_oplog_add_insert_at(oplog: *mut dtgpu_oplog, agent: i32, parents: *const u64, n_parents: usize,
                                     pos: u64, utf8: *const c_char, n_bytes: usize) -> i64;
    pub fn dtgpu_oplog_add_delete_at(oplog: *mut dtgpu_oplog, agent: i32, parents: *const u64, n_parents: usize,
                                     del_start: u64, del_end: u64) -> i64;
    pub fn dtgpu_oplog_add_insert(oplog: *mut dtgpu_oplog, agent: i32, pos: u64, utf8: *const c_char, n_bytes: usize) -> i64;
    pub fn dtgpu_oplog_add_delete_without_content(oplog: *mut dtgpu_oplog, agent: i32, del_start: u64, del_end: u64) -> i64;
    pub fn dtgpu_oplog_encode(oplog: *const dtgpu_oplog, from: *const u64, n_from: usize, flags: u32, out: *mut u8,
                              cap: usize, out_len: *mut usize) -> dtgpu_status;
    pub fn dtgpu_lz4_compress(input: *const u8, n: usize, out: *mut u8, cap: usize, out_len: *mut usize) -> dtgpu_status;
    pub fn dtgpu_oplog_len(oplog: *const dtgpu_oplog) -> usize;
    pub fn dtgpu_oplog_local_frontier(oplog: *const dtgpu_oplog, out: *mut u64, cap: usize) -> usize;
    pub fn dtgpu_oplog_last_added_frontier(oplog: *const dtgpu_oplog, out: *mut u64, cap: usize) -> usize;
    pub fn dtgpu_oplog_dominators(oplog: *const dtgpu_oplog, a: *const u64, na: usize, b: *const u64, nb: usize,
                                  out: *mut u64, cap: usize) -> i64;
    // multi-CRDT OpLog support (src/oplog.rs, src/branch.rs:180-232): a text's ops projected out of
    // the shared graph, versions projected the same way, remote ids <-> LVs
    pub fn dtgpu_oplog_project(oplog: *const dtgpu_oplog, spans: *const u64, n_spans: usize,
                               out: *mut *mut dtgpu_oplog) -> dtgpu_status;
    pub fn dtgpu_oplog_project_version(oplog: *const dtgpu_oplog, spans: *const u64, n_spans: usize,
                                       version: *const u64, n_version: usize, out: *mut u64, cap: usize) -> i64;
    pub fn dtgpu_oplog_local_to_remote(oplog: *const dtgpu_oplog, lv: u64, agent: *mut u32, seq: *mut u64) -> dtgpu_status;
    pub fn dtgpu_oplog_remote_to_local(oplog: *const dtgpu_oplog, agent: u32, seq: u64, n: u64, spans: *mut u64,
                                       cap: usize) -> i64;
    // checkout (src/list/oplog.rs:32-42) and transformed ops (src/list/merge.rs:24-48)
    pub fn dtgpu_checkout(oplog: *const dtgpu_oplog, version: *const u64, n_version: usize, out: *mut u8, cap: usize,
                          out_len: *mut usize) -> dtgpu_status;
    pub fn dtgpu_checkout_tip(oplog: *const dtgpu_oplog, out: *mut u8, cap: usize, out_len: *mut usize) -> dtgpu_status;
    pub fn dtgpu_xf_operations(oplog: *const dtgpu_oplog, out: *mut u32, cap: usize, n_out: *mut usize) -> dtgpu_status;
    pub fn dtgpu_xf_operations_from(oplog: *const dtgpu_oplog, from: *const u64, n_from: usize, merging: *const u64,
                                    n_merging: usize, out: *mut u32, cap: usize, n_out: *mut usize) -> dtgpu_status;
    // batches (SURVEY.md 8b "batch entry")
    pub fn dtgpu_batch_create(docs: *const *const u8, lens: *const usize, n_docs: usize, opts: *const dtgpu_batch_opts,
                              out: *mut *mut dtgpu_batch) -> dtgpu_status;
    pub fn dtgpu_batch_create_device(docs: *const *const u8, lens: *const usize, n: usize, opts: *const dtgpu_batch_opts,
                                     out: *mut *mut dtgpu_batch) -> dtgpu_status;
    pub fn dtgpu_batch_run(batch: *mut dtgpu_batch, stream: *mut c_void) -> dtgpu_status;
    pub fn dtgpu_batch_sync(batch: *mut dtgpu_batch) -> dtgpu_status;
    pub fn dtgpu_batch_size(batch: *const dtgpu_batch) -> usize;
    pub fn dtgpu_batch_results(batch: *mut dtgpu_batch, results: *mut dtgpu_doc_result) -> dtgpu_status;
    pub fn dtgpu_batch_text(batch: *mut dtgpu_batch, doc: usize, out: *mut u8, cap: usize, out_len: *mut usize) -> dtgpu_status;
    pub fn dtgpu_batch_free(batch: *mut dtgpu_batch);
    // many ListOpLog::encode(opts) at once on the GPU (device-staged batches)
    pub fn dtgpu_batch_encode(batch: *mut dtgpu_batch, flags: u32, kernel_ms: *mut f32) -> dtgpu_status;
    pub fn dtgpu_batch_encoded(batch: *const dtgpu_batch, doc: usize, out: *mut u8, cap: usize, out_len: *mut usize,
                               prof: *mut u64) -> dtgpu_status;
    pub fn dtgpu_batch_checkout(docs: *const *const u8, lens: *const usize, n_docs: usize, opts: *const dtgpu_batch_opts,
                                results: *mut dtgpu_doc_result) -> dtgpu_status;
    pub fn dtgpu_text_hash(text: *const u8, len: usize) -> u64;
    // batched load_from / decode_and_add on the GPU (decode_oplog.rs:447-960, 476-583)
    pub fn dtgpu_decode_create(docs: *const *const u8, lens: *const usize, n: usize, opts: *const dtgpu_batch_opts,
                               out: *mut *mut dtgpu_decoded) -> dtgpu_status;
    pub fn dtgpu_decode_run(dec: *mut dtgpu_decoded, ms: *mut f32) -> dtgpu_status;
    pub fn dtgpu_decode_free(dec: *mut dtgpu_decoded);
    pub fn dtgpu_decode_add(base: *const dtgpu_decoded, patches: *const *const u8, lens: *const usize, n: usize,
                            ignore_crc: c_int, ms: *mut f32, out: *mut *mut dtgpu_decoded) -> dtgpu_status;
    pub fn dtgpu_decode_add_result(merged: *const dtgpu_decoded, i: usize, frontier: *mut u64, cap: usize,
                                   n_frontier: *mut usize) -> dtgpu_status;
    pub fn dtgpu_batch_create_decoded(dec: *mut dtgpu_decoded, out: *mut *mut dtgpu_batch) -> dtgpu_status;
    pub fn dtgpu_device_count() -> c_int;
    // the decoded oplog's arrays (op runs, inserted content, per-LV byte offsets, ...)
    pub fn dtgpu_oplog_export(oplog: *const dtgpu_oplog, what: c_int, out: *mut c_void, cap: usize) -> usize;
    // which documents of a batch took the fast-forward path (linear histories, merge.rs:811-840)
    pub fn dtgpu_batch_fast_forwarded(batch: *const dtgpu_batch, flags: *mut u8, cap: usize) -> usize;
}
pub const DTGPU_EXPORT_OPS: c_int = 0;
pub const DTGPU_EXPORT_CONTENT: c_int = 5;
pub const DTGPU_EXPORT_CHAR_OFFSETS: c_int = 6;

/// A decoded oplog (`ListOpLog`), owned.
pub struct ListOpLog {
    h: *mut dtgpu_oplog,
}

impl ListOpLog {
    /// `ListOpLog::load_from(bytes)` (src/list/encoding/decode_oplog.rs:447); Err = ParseError code.
    pub fn load_from(bytes: &[u8]) -> Result<Self, i32> {
        let mut h = std::ptr::null_mut();
        let s = unsafe { dtgpu_oplog_load(bytes.as_ptr(), bytes.len(), 0, &mut h) };
        if s != DTGPU_OK { Err(s) } else { Ok(ListOpLog { h }) }
    }
    /// `ListOpLog::len()` (src/list/oplog.rs:89).
    pub fn len(&self) -> usize { unsafe { dtgpu_oplog_len(self.h) } }
    pub fn is_empty(&self) -> bool { self.len() == 0 }
    /// `ListOpLog::local_frontier()` (src/list/oplog.rs:329).
    pub fn local_frontier(&self) -> Vec<u64> {
        unsafe {
            let n = dtgpu_oplog_local_frontier(self.h, std::ptr::null_mut(), 0);
            let mut v = vec![0u64; n];
            dtgpu_oplog_local_frontier(self.h, v.as_mut_ptr(), n);
            v
        }
    }
    /// `checkout_tip().content().to_string()` (src/list/oplog.rs:38-42), replayed on the GPU.
    pub fn checkout_tip_text(&self) -> Result<String, i32> {
        unsafe {
            let mut n = 0usize;
            let s = dtgpu_checkout_tip(self.h, std::ptr::null_mut(), 0, &mut n);
            if s != DTGPU_OK { return Err(s); }
            let mut buf = vec![0u8; n];
            let s = dtgpu_checkout_tip(self.h, buf.as_mut_ptr(), n, &mut n);
            if s != DTGPU_OK { return Err(s); }
            buf.truncate(n);
            Ok(String::from_utf8(buf).expect("the engine emits UTF-8"))
        }
    }
    /// `checkout(version).content().to_string()` (src/list/oplog.rs:32-36).
    pub fn checkout_text(&self, version: &[u64]) -> Result<String, i32> {
        unsafe {
            let mut n = 0usize;
            let s = dtgpu_checkout(self.h, version.as_ptr(), version.len(), std::ptr::null_mut(), 0, &mut n);
            if s != DTGPU_OK { return Err(s); }
            let mut buf = vec![0u8; n];
            let s = dtgpu_checkout(self.h, version.as_ptr(), version.len(), buf.as_mut_ptr(), n, &mut n);
            if s != DTGPU_OK { return Err(s); }
            buf.truncate(n);
            Ok(String::from_utf8(buf).expect("the engine emits UTF-8"))
        }
    }
    /// `decode_and_add(data) -> Result<Frontier, ParseError>` (decode_oplog.rs:465); the oplog is
    /// unchanged on error.
    pub fn decode_and_add(&mut self, data: &[u8]) -> Result<Vec<u64>, i32> {
        unsafe {
            let mut f = vec![0u64; 64];
            let mut n = 0usize;
            let s = dtgpu_oplog_decode_and_add(self.h, data.as_ptr(), data.len(), 0, f.as_mut_ptr(), f.len(), &mut n);
            if s != DTGPU_OK { return Err(s); }
            if n > f.len() {   // the buffer was short: read the whole reported frontier back
                f.resize(n, 0);
                n = dtgpu_oplog_last_added_frontier(self.h, f.as_mut_ptr(), n);
            }
            f.truncate(n);
            Ok(f)
        }
    }
    /// The transformed ops `ListBranch::merge` applies to move a branch from `from` to `merging`
    /// (`iter_xf_operations_from`, src/list/merge.rs:24-38): (lv, Some(pos) | None for
    /// DeleteAlreadyHappened), in TransformedOpsIter order.
    pub fn xf_operations_from(&self, from: &[u64], merging: &[u64]) -> Result<Vec<(u32, Option<u32>)>, i32> {
        unsafe {
            let mut n = 0usize;
            let s = dtgpu_xf_operations_from(self.h, from.as_ptr(), from.len(), merging.as_ptr(), merging.len(),
                                             std::ptr::null_mut(), 0, &mut n);
            if s != DTGPU_OK { return Err(s); }
            let mut buf = vec![0u32; 2 * n];
            let s = dtgpu_xf_operations_from(self.h, from.as_ptr(), from.len(), merging.as_ptr(), merging.len(),
                                             buf.as_mut_ptr(), n, &mut n);
            if s != DTGPU_OK { return Err(s); }
            Ok(buf.chunks(2).take(n).map(|r| (r[0], if r[1] == u32::MAX { None } else { Some(r[1]) })).collect())
        }
    }
}

impl ListOpLog {
    /// `ListOpLog::checkout_tip()` (src/list/oplog.rs:38-42): the branch at the oplog's version.
    pub fn checkout_tip(&self) -> Result<ListBranch, i32> {
        Ok(ListBranch { content: self.checkout_tip_text()?, version: self.local_frontier() })
    }
    /// `ListOpLog::checkout(version)` (src/list/oplog.rs:32-36).
    pub fn checkout(&self, version: &[u64]) -> Result<ListBranch, i32> {
        let mut v = version.to_vec();
        v.sort_unstable();
        Ok(ListBranch { content: self.checkout_text(&v)?, version: v })
    }
    /// `find_dominators_2(a, b)` (src/causalgraph/graph/tools.rs:545-578): the frontier of a and b together.
    pub fn dominators(&self, a: &[u64], b: &[u64]) -> Result<Vec<u64>, i32> {
        unsafe {
            let n = dtgpu_oplog_dominators(self.h, a.as_ptr(), a.len(), b.as_ptr(), b.len(), std::ptr::null_mut(), 0);
            if n < 0 { return Err(-1); }
            let mut v = vec![0u64; n as usize];
            dtgpu_oplog_dominators(self.h, a.as_ptr(), a.len(), b.as_ptr(), b.len(), v.as_mut_ptr(), v.len());
            Ok(v)
        }
    }
    fn export_u32(&self, what: c_int) -> Vec<u32> {
        unsafe {
            let n = dtgpu_oplog_export(self.h, what, std::ptr::null_mut(), 0);
            let mut v = vec![0u32; n / 4];
            dtgpu_oplog_export(self.h, what, v.as_mut_ptr() as *mut c_void, n);
            v
        }
    }
    fn export_bytes(&self, what: c_int) -> Vec<u8> {
        unsafe {
            let n = dtgpu_oplog_export(self.h, what, std::ptr::null_mut(), 0);
            let mut v = vec![0u8; n];
            dtgpu_oplog_export(self.h, what, v.as_mut_ptr() as *mut c_void, n);
            v
        }
    }
}

impl Drop for ListOpLog {
    fn drop(&mut self) { unsafe { dtgpu_oplog_free(self.h) } }
}

/// `ListBranch` (src/list/mod.rs:65-76, src/list/branch.rs): a document's text at a version.
/// Checkouts and the transformed ops a merge applies are computed on the GPU.
#[derive(Clone, Debug, Default, PartialEq, Eq)]
pub struct ListBranch {
    content: String,
    version: Vec<u64>,
}

impl ListBranch {
    /// `ListBranch::new()` (src/list/branch.rs:12-20): empty, at ROOT.
    pub fn new() -> Self { ListBranch::default() }
    /// `ListBranch::new_at_tip(oplog)` (src/list/branch.rs:30-32).
    pub fn new_at_tip(oplog: &ListOpLog) -> Result<Self, i32> { oplog.checkout_tip() }
    /// `ListBranch::new_at_local_version(oplog, version)` (src/list/branch.rs:22-26).
    pub fn new_at_local_version(oplog: &ListOpLog, version: &[u64]) -> Result<Self, i32> { oplog.checkout(version) }
    /// `ListBranch::content()` (src/list/branch.rs:38-41).
    pub fn content(&self) -> &str { &self.content }
    /// `ListBranch::len()` (src/list/branch.rs:49-52): characters, not bytes.
    pub fn len(&self) -> usize { self.content.chars().count() }
    pub fn is_empty(&self) -> bool { self.content.is_empty() }
    /// `ListBranch::local_frontier()` (src/list/branch.rs:43-46).
    pub fn local_frontier(&self) -> Vec<u64> { self.version.clone() }
    pub fn local_frontier_ref(&self) -> &[u64] { &self.version }
    /// `ListBranch::merge(&oplog, merge_frontier)` (src/list/merge.rs:63-95): apply the
    /// transformed operations between the branch's version and `merge_frontier`
    /// (iter_xf_operations_from, replayed on the GPU) to the content, then move to the dominators
    /// of both versions.
    pub fn merge(&mut self, oplog: &ListOpLog, merge_frontier: &[u64]) -> Result<(), i32> {
        let target = oplog.dominators(&self.version, merge_frontier)?;
        if target == self.version { return Ok(()); }
        let xf = oplog.xf_operations_from(&self.version, merge_frontier)?;
        let ops = oplog.export_u32(DTGPU_EXPORT_OPS);          // lv, len, pos, kind | fwd << 1
        let content = oplog.export_bytes(DTGPU_EXPORT_CONTENT);
        let cbyte = oplog.export_u32(DTGPU_EXPORT_CHAR_OFFSETS);
        let mut text: Vec<char> = self.content.chars().collect();
        for (lv, pos) in xf {
            let pos = match pos { Some(p) => p as usize, None => continue };   // DeleteAlreadyHappened
            // the op run holding lv (runs are in LV order)
            let runs = ops.len() / 4;
            let (mut lo, mut hi) = (0usize, runs);
            while hi - lo > 1 {
                let mid = (lo + hi) / 2;
                if ops[4 * mid] <= lv { lo = mid; } else { hi = mid; }
            }
            if runs == 0 || lv < ops[4 * lo] || lv >= ops[4 * lo] + ops[4 * lo + 1] || pos > text.len() {
                return Err(64);   // DTGPU_ERR_CHECKOUT
            }
            if ops[4 * lo + 3] & 1 == 0 {
                let at = cbyte[lv as usize] as usize;
                if at >= content.len() { return Err(64); }
                let ch = std::str::from_utf8(&content[at..]).ok().and_then(|t| t.chars().next()).ok_or(64)?;
                text.insert(pos, ch);
            } else {
                if pos >= text.len() { return Err(64); }
                text.remove(pos);
            }
        }
        self.content = text.into_iter().collect();
        self.version = target;
        Ok(())
    }
}

/// Many `ListOpLog::load_from(doc)?.checkout_tip()` at once on one GPU: per document its status,
/// text length, text hash (dtgpu_text_hash) and merged ops.
pub fn batch_checkout(docs: &[&[u8]], device: i32) -> Result<Vec<dtgpu_doc_result>, i32> {
    let ptrs: Vec<*const u8> = docs.iter().map(|d| d.as_ptr()).collect();
    let lens: Vec<usize> = docs.iter().map(|d| d.len()).collect();
    let opts = dtgpu_batch_opts { device, ..Default::default() };
    let mut res = vec![dtgpu_doc_result::default(); docs.len()];
    let s = unsafe { dtgpu_batch_checkout(ptrs.as_ptr(), lens.as_ptr(), docs.len(), &opts, res.as_mut_ptr()) };
    if s != DTGPU_OK { Err(s) } else { Ok(res) }
}

/// Many `ListOpLog::load_from(doc)` at once, decoded into HBM (dtgpu_decode_*); `add` merges one
/// patch per document on the GPU (`decode_and_add`), `checkout` checks the oplogs out in place.
pub struct DecodedBatch {
    h: *mut dtgpu_decoded,
    n: usize,
}

impl DecodedBatch {
    pub fn load(docs: &[&[u8]], device: i32) -> Result<DecodedBatch, i32> {
        let ptrs: Vec<*const u8> = docs.iter().map(|d| d.as_ptr()).collect();
        let lens: Vec<usize> = docs.iter().map(|d| d.len()).collect();
        let opts = dtgpu_batch_opts { device, ..Default::default() };
        let mut h = std::ptr::null_mut();
        let s = unsafe { dtgpu_decode_create(ptrs.as_ptr(), lens.as_ptr(), docs.len(), &opts, &mut h) };
        if s != DTGPU_OK { return Err(s); }
        let b = DecodedBatch { h, n: docs.len() };
        let s = unsafe { dtgpu_decode_run(b.h, std::ptr::null_mut()) };
        if s != DTGPU_OK { Err(s) } else { Ok(b) }
    }
    /// `decode_and_add(patches[i])` into document i; per document `Result<Frontier, ParseError>`.
    pub fn add(&self, patches: &[&[u8]]) -> Result<(DecodedBatch, Vec<Result<Vec<u64>, i32>>), i32> {
        let ptrs: Vec<*const u8> = patches.iter().map(|d| d.as_ptr()).collect();
        let lens: Vec<usize> = patches.iter().map(|d| d.len()).collect();
        let mut h = std::ptr::null_mut();
        let s = unsafe { dtgpu_decode_add(self.h, ptrs.as_ptr(), lens.as_ptr(), patches.len(), 0, std::ptr::null_mut(), &mut h) };
        if s != DTGPU_OK { return Err(s); }
        let m = DecodedBatch { h, n: self.n };
        let mut out = Vec::with_capacity(m.n);
        for i in 0..m.n {
            let mut f = vec![0u64; 64];
            let mut k = 0usize;
            let s = unsafe { dtgpu_decode_add_result(m.h, i, f.as_mut_ptr(), f.len(), &mut k) };
            f.truncate(k);
            out.push(if s == DTGPU_OK { Ok(f) } else { Err(s) });
        }
        Ok((m, out))
    }
    /// checkout_tip of every document on the GPU (consumes the decoded oplogs).
    pub fn checkout(mut self) -> Result<Vec<dtgpu_doc_result>, i32> {
        let mut b = std::ptr::null_mut();
        let s = unsafe { dtgpu_batch_create_decoded(self.h, &mut b) };
        self.h = std::ptr::null_mut();
        if s != DTGPU_OK { return Err(s); }
        let mut res = vec![dtgpu_doc_result::default(); self.n];
        let s = unsafe {
            let s = dtgpu_batch_run(b, std::ptr::null_mut());
            let s = if s == DTGPU_OK { dtgpu_batch_sync(b) } else { s };
            let s = if s == DTGPU_OK { dtgpu_batch_results(b, res.as_mut_ptr()) } else { s };
            dtgpu_batch_free(b);
            s
        };
        if s != DTGPU_OK { Err(s) } else { Ok(res) }
    }
}

impl Drop for DecodedBatch {
    fn drop(&mut self) {
        if !self.h.is_null() { unsafe { dtgpu_decode_free(self.h) } }
    }
}
