// Probe: global-memory store -> load hand-off between lanes of one wavefront (gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int MODE>
__global__ __launch_bounds__(64) void k(int *items, int *out, int rounds) {
    const int l = threadIdx.x;
    for (int r = 0; r < rounds; r++) {
        int *it = items + r * 64;
        const int v = l < 6 ? it[l] : 0;            // warm the line in L1
        if (MODE == 0) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (MODE == 1) __syncthreads();
        if (MODE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (l >= 5 && l < 6) it[l + 28] = v;
        if (l >= 5 && l < 33) it[l] = 1000 + l;
        if (MODE == 0) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (MODE == 1) __syncthreads();
        if (MODE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (MODE == 3) asm volatile("s_waitcnt vmcnt(0)\n\tbuffer_inv sc0" ::: "memory");
        out[r * 64 + l] = it[l];
    }
}

template <int MODE>
int run(int rounds) {
    std::vector<int> h(64 * rounds);
    for (int r = 0; r < rounds; r++) for (int l = 0; l < 64; l++) h[r * 64 + l] = l < 6 ? l : 0;
    int *d_items, *d_out;
    hipMalloc(&d_items, h.size() * 4);
    hipMalloc(&d_out, h.size() * 4);
    hipMemcpy(d_items, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k<MODE>, dim3(1), dim3(64), 0, 0, d_items, d_out, rounds);
    std::vector<int> o(h.size());
    hipMemcpy(o.data(), d_out, o.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int r = 0; r < rounds; r++)
        for (int l = 0; l < 64; l++) {
            int want = l < 5 ? l : l < 33 ? 1000 + l : l == 33 ? 5 : 0;
            if (o[r * 64 + l] != want) bad++;
        }
    hipFree(d_items); hipFree(d_out);
    return bad;
}

int main() {
    const int R = 4096;
    printf("mode0 wavefront-fence bad=%d\n", run<0>(R));
    printf("mode1 syncthreads      bad=%d\n", run<1>(R));
    printf("mode2 waitcnt          bad=%d\n", run<2>(R));
    printf("mode3 waitcnt+inv      bad=%d\n", run<3>(R));
    return 0;
}
