// Dependent-load latency probe (one wave): pointer chase through a buffer of `n` words with a
// fixed stride pattern, reporting s_memtime cycles per hop.  Calibrates the per-round-trip cost
// the replay / planner kernels pay (MI355X_MICROARCH.md quotes one-lane idle-chip latencies).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void chase(const unsigned *buf, unsigned start, int hops, unsigned long long *out, int wide) {
    unsigned idx = start;
    const unsigned l = __lane_id();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < hops; i++) {
        unsigned v = buf[idx + (wide ? l : 0)];
        idx = __builtin_amdgcn_readfirstlane(v);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) { out[0] = t1 - t0; out[1] = idx; }
}
__global__ void chase_store(unsigned *buf, unsigned start, int hops, unsigned long long *out, unsigned *sink) {
    unsigned idx = start;
    const unsigned l = __lane_id();
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < hops; i++) {
        sink[(i * 64 + l) & 0xFFFFF] = idx;   // a store per hop, then the dependent load
        unsigned v = buf[idx + l];
        idx = __builtin_amdgcn_readfirstlane(v);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) { out[0] = t1 - t0; out[1] = idx; }
}

int main() {
    for (size_t n : {size_t(1) << 14, size_t(1) << 20, size_t(1) << 26}) {
        std::vector<unsigned> h(n + 64);
        const size_t step = 4099 * 16;   // jump across lines / pages
        size_t cur = 0;
        for (size_t i = 0; i < n; i++) { size_t nx = (cur + step) % n; h[cur] = unsigned(nx); cur = nx; }
        unsigned *d; unsigned long long *o; unsigned *sink;
        hipMalloc(&d, (n + 64) * 4); hipMalloc(&o, 16); hipMalloc(&sink, (1 << 20) * 4 + 256);
        hipMemcpy(d, h.data(), (n + 64) * 4, hipMemcpyHostToDevice);
        const int hops = 2000;
        for (int wide = 0; wide < 2; wide++) {
            unsigned long long r[2];
            for (int rep = 0; rep < 2; rep++) {
                hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, 0, d, 0u, hops, o, wide);
                hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
            }
            printf("n=%zu words wide=%d: %.0f cycles/hop\n", n, wide, double(r[0]) / hops);
        }
        unsigned long long r[2];
        for (int rep = 0; rep < 2; rep++) {
            hipLaunchKernelGGL(chase_store, dim3(1), dim3(64), 0, 0, d, 0u, hops, o, sink);
            hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
        }
        printf("n=%zu words wide+store: %.0f cycles/hop\n", n, double(r[0]) / hops);
        hipFree(d); hipFree(o); hipFree(sink);
    }
    return 0;
}
