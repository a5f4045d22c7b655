// dt_devbuf.hpp -- owning device buffer used by the host staging code.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace dtgpu {

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t alloc(size_t count) {
        if (p) { (void)hipFree(p); p = nullptr; }
        n = count;
        return hipMalloc(reinterpret_cast<void **>(&p), std::max<size_t>(count, 1) * sizeof(T));
    }
    hipError_t upload(const std::vector<T> &v, hipStream_t s) {
        hipError_t e = alloc(v.size());
        if (e != hipSuccess || v.empty()) return e;
        return hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
    }
};

// A failed HIP call on a staging path: named on stderr (file:line and the runtime's message)
// before the caller returns DTGPU_ERR_HIP, so a failure is never anonymous.
inline bool hip_failed(hipError_t e, const char *file, int line) {
    if (e == hipSuccess) return false;
    fprintf(stderr, "[dtgpu] HIP error at %s:%d: %s\n", file, line, hipGetErrorString(e));
    return true;
}
#define DTGPU_HIP_FAILED(x) ::dtgpu::hip_failed((x), __FILE__, __LINE__)

// Staging phase clock (DTGPU_STAGE_PROF=1): stage_prof("name") prints the wall milliseconds since
// the previous call on this thread to stderr; stage_prof(nullptr) restarts the clock.
inline void stage_prof(const char *phase) {
    static const bool on = getenv("DTGPU_STAGE_PROF") != nullptr;
    thread_local std::chrono::steady_clock::time_point last = std::chrono::steady_clock::now();
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    if (phase) fprintf(stderr, "[stage] %-28s %9.2f ms\n", phase, std::chrono::duration<double, std::milli>(now - last).count());
    last = now;
}

}  // namespace dtgpu
