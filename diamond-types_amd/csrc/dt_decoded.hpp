// dt_decoded.hpp -- the decoder handle (dtgpu_decoded): device arenas of a decoded batch,
// shared by the decode API (dtgpu_decode.cpp) and the device-staged checkout batches
// (dtgpu_api.cpp), which read the decoded oplogs in place.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

#include "dt_decode.hpp"
#include "dt_devbuf.hpp"

using dtgpu::DecodeDesc;
using dtgpu::DecodeParams;
using dtgpu::DecodeResult;
using dtgpu::DevBuf;

struct dtgpu_decoded {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    size_t n = 0;
    uint64_t in_bytes = 0;
    float last_ms = 0;
    std::vector<DecodeDesc> desc;
    std::vector<DecodeResult> res;
    DevBuf<uint8_t> in, lz, content;
    DevBuf<uint32_t> aruns, alist, pre, ops, ent, poff, par, cbyte, agents, ver;
    DevBuf<uint32_t> lz_big, lz_pre;   // documents whose LZ4 block lz4_kernel decompresses, its verdicts
    DevBuf<uint32_t> fill, fill_n, fill_doc;   // deferred per-LV offsets (DecodeParams::fill)
    DevBuf<uint32_t> order;                    // decode_kernel's dispatch order (DecodeParams::order)
    // dtgpu_decode_add results: the merged oplogs (not re-decodable), each merge's status and the
    // patch's version
    bool merged = false;
    std::vector<uint32_t> add_status;
    DevBuf<uint32_t> ffr;
    DevBuf<DecodeDesc> d_desc;
    DevBuf<DecodeResult> d_res;
    DecodeParams P{};
    ~dtgpu_decoded() {
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (stream) (void)hipStreamDestroy(stream);
    }
};
