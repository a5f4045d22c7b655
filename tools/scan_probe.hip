// Validate the DPP wave-scan used by dt_replay.hip against a sequential prefix sum (gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ uint32_t dpp_scan(uint32_t x) {
    // Hillis-Steele inside each 16-lane row, then row_bcast:15 / row_bcast:31 across rows.
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);   // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);   // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);   // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);   // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);   // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);   // row_bcast:31
    return x;
}

__global__ __launch_bounds__(64) void k(const uint32_t *in, uint32_t *out, int n) {
    for (int r = 0; r < n; r++) out[r * 64 + threadIdx.x] = dpp_scan(in[r * 64 + threadIdx.x]);
}

int main() {
    const int R = 1000;
    std::vector<uint32_t> h(64 * R), o(64 * R);
    srand(1);
    for (auto &x : h) x = rand() % 1000;
    uint32_t *di, *dout;
    (void)hipMalloc(&di, h.size() * 4);
    (void)hipMalloc(&dout, h.size() * 4);
    (void)hipMemcpy(di, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, di, dout, R);
    (void)hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int r = 0; r < R; r++) {
        uint32_t acc = 0;
        for (int l = 0; l < 64; l++) { acc += h[r * 64 + l]; if (o[r * 64 + l] != acc) bad++; }
    }
    printf("dpp scan mismatches: %d of %d\n", bad, 64 * R);
    return bad != 0;
}
