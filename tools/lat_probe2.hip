// One-wave latency calibration for the replay kernels' building blocks (s_memtime ticks per
// dependent step, and the tick rate against hipEvent wall time):
//   gload   dependent 64-lane global load (L2-resident 1 MiB window)
//   gload+st  the same with a 64-lane store issued before each load (gfx9 vmcnt counts both)
//   lds     dependent ds_read_b32 chain
//   bperm   dependent ds_bpermute chain
//   scan    dependent DPP wave prefix sum (6 DPP adds) + readlane
//   rlane   dependent v_readlane / readfirstlane round trip through an SGPR
//   ldsatom returnless LDS add then a dependent LDS read of another word
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/lat_probe2 tools/lat_probe2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define DEV __device__ __forceinline__
DEV unsigned U(unsigned v) { return unsigned(__builtin_amdgcn_readfirstlane(int(v))); }
DEV unsigned wave_scan(unsigned x) {
    x += unsigned(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xF, 0xF, false));
    x += unsigned(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xF, 0xF, false));
    x += unsigned(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xF, 0xF, false));
    x += unsigned(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xF, 0xF, false));
    x += unsigned(__builtin_amdgcn_update_dpp(0, int(x), 0x142, 0xA, 0xF, false));
    x += unsigned(__builtin_amdgcn_update_dpp(0, int(x), 0x143, 0xC, 0xF, false));
    return x;
}

__global__ __launch_bounds__(64) void probe(const unsigned *buf, unsigned *sink, int mode, int hops, unsigned long long *out) {
    __shared__ unsigned s[4096];
    const unsigned l = __lane_id();
    for (unsigned i = l; i < 4096; i += 64) s[i] = (i * 97u + 13u) & 4095u;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    unsigned idx = U(buf[0]) & 0x3FFFu;
    unsigned x = l;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    switch (mode) {
        case 0:
            for (int i = 0; i < hops; i++) idx = U(buf[(idx << 6) + l]) & 0x3FFFu;
            break;
        case 1:
            for (int i = 0; i < hops; i++) {
                sink[((i & 1023) << 6) + l] = idx;
                idx = U(buf[(idx << 6) + l]) & 0x3FFFu;
            }
            break;
        case 2:
            for (int i = 0; i < hops; i++) idx = U(s[(idx + l) & 4095u]);
            break;
        case 3:
            for (int i = 0; i < hops; i++) x = unsigned(__builtin_amdgcn_ds_bpermute(int(((x + 1) & 63u) << 2), int(x)));
            idx = U(x);
            break;
        case 4:
            for (int i = 0; i < hops; i++) x = unsigned(__builtin_amdgcn_readlane(int(wave_scan(x)), 63)) + l;
            idx = U(x);
            break;
        case 5:
            for (int i = 0; i < hops; i++) x = U(x * 3u + l) + 1u;
            idx = x;
            break;
        case 6:
            for (int i = 0; i < hops; i++) {
                __hip_atomic_fetch_add(&s[idx & 4095u], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                idx = U(s[(idx + 64) & 4095u]);
            }
            break;
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) { out[0] = t1 - t0; out[1] = idx + x; }
}

int main() {
    const size_t n = (1u << 14) * 64;   // 16k rows of 64 words = 4 MiB
    std::vector<unsigned> h(n);
    unsigned r = 12345;
    for (size_t i = 0; i < n; i++) { r = r * 1664525u + 1013904223u; h[i] = r >> 8; }
    unsigned *buf, *sink;
    unsigned long long *out;
    (void)hipMalloc(&buf, n * 4);
    (void)hipMalloc(&sink, 1024 * 64 * 4);
    (void)hipMalloc(&out, 16);
    (void)hipMemcpy(buf, h.data(), n * 4, hipMemcpyHostToDevice);
    const char *names[] = {"gload(L2, 4MiB window)", "gload+store", "lds read", "ds_bpermute", "dpp scan+readlane", "readfirstlane", "lds atomic+read"};
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int mode = 0; mode < 7; mode++) {
        const int hops = mode <= 1 ? 20000 : 200000;
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, buf, sink, mode, 1000, out);   // warm
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, buf, sink, mode, hops, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        unsigned long long o[2];
        (void)hipMemcpy(o, out, 16, hipMemcpyDeviceToHost);
        printf("%-24s %8.1f ticks/step  %8.2f ns/step  tick rate %.3f GHz\n", names[mode], double(o[0]) / hops,
               ms * 1e6 / hops, double(o[0]) / (ms * 1e6));
    }
    return 0;
}
