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
}
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
}

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

impl Drop for ListOpLog {
    fn drop(&mut self) { unsafe { dtgpu_oplog_free(self.h) } }
}

/// Many `ListOpLog::load_from(doc)?.checkout_tip()` at once on one GPU: per document its status,
/// text length, text hash (dtgpu_text_hash) and merged ops.
pub fn batch_checkout(docs: &[&[u8]], device: i32) -> Result<Vec<dtgpu_doc_result>, i32> {
    let ptrs: Vec<*const u8> = docs.iter().map(|d| d.as_ptr()).collect();
    let lens: Vec<usize> = docs.iter().map(|d| d.len()).collect();
    let opts = dtgpu_batch_opts { ignore_crc: 0, host_threads: 0, device };
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
        let opts = dtgpu_batch_opts { ignore_crc: 0, host_threads: 0, device };
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
