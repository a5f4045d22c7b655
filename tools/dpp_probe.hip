#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
__device__ __forceinline__ uint32_t compose_scan(uint32_t v) {
    auto step = [&](uint32_t p) {
        const uint32_t m0 = v & 1u, m1 = ((v >> 1) & 1u) ^ 1u;
        const uint32_t p0 = p & 1u, p1 = ((p >> 1) & 1u) ^ 1u;
        v = (p0 ? m1 : m0) | (((p1 ? m1 : m0) ^ 1u) << 1);
    };
    step(uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xf, 0xf, false)));
    step(uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xf, 0xf, false)));
    step(uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xf, 0xf, false)));
    step(uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xf, 0xf, false)));
    step(uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false)));
    step(uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false)));
    return v;
}
__device__ __forceinline__ uint32_t scan_sum(uint32_t v) {
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xf, 0xf, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xf, 0xf, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xf, 0xf, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xf, 0xf, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false));
    v += uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false));
    return v;
}
__global__ void k(const uint32_t *in, uint32_t *out, uint32_t *out2) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    out[i] = compose_scan(in[i]);
    out2[i] = scan_sum(in[i]);
}
int main() {
    const int B = 256, N = B * 64;
    uint32_t *h = (uint32_t *)malloc(N * 4), *o = (uint32_t *)malloc(N * 4), *o2 = (uint32_t *)malloc(N * 4);
    srand(1);
    for (int i = 0; i < N; i++) h[i] = rand() & 3;
    uint32_t *d, *dout, *dout2;
    hipMalloc(&d, N * 4); hipMalloc(&dout, N * 4); hipMalloc(&dout2, N * 4);
    hipMemcpy(d, h, N * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(B), dim3(64), 0, 0, d, dout, dout2);
    hipMemcpy(o, dout, N * 4, hipMemcpyDeviceToHost);
    hipMemcpy(o2, dout2, N * 4, hipMemcpyDeviceToHost);
    int bad = 0, bad2 = 0;
    for (int b = 0; b < B; b++) {
        int a0 = 0, a1 = 1; uint32_t s = 0;
        for (int l = 0; l < 64; l++) {
            const uint32_t v = h[b * 64 + l];
            const int f0 = v & 1, f1 = ((v >> 1) & 1) ^ 1;
            const int n0 = a0 ? f1 : f0, n1 = a1 ? f1 : f0;
            a0 = n0; a1 = n1;
            const uint32_t want = uint32_t(a0) | (uint32_t(a1 ^ 1) << 1);
            s += v;
            if (o[b * 64 + l] != want) { if (bad < 10) printf("compose blk %d lane %d got %u want %u\n", b, l, o[b*64+l], want); bad++; }
            if (o2[b * 64 + l] != s) { if (bad2 < 10) printf("sum blk %d lane %d got %u want %u\n", b, l, o2[b*64+l], s); bad2++; }
        }
    }
    printf("compose bad %d, sum bad %d\n", bad, bad2);
    return 0;
}
