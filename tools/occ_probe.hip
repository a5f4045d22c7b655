// occ_probe.hip -- residency census: how many single-wave workgroups one CU holds at once for a
// given dynamic LDS size and SGPR count (gfx950).  Each workgroup counts itself in on its CU
// (hardware ids), records the running maximum, spins ~50 us (100 MHz clock), counts itself out.
//   hipcc --offload-arch=gfx950 -O2 tools/occ_probe.hip -o tools/occ_probe && ./tools/occ_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int SLOTS = 8 * 128;

__device__ __forceinline__ unsigned cu_slot() {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID
    return (xcc & 7) * 128 + ((hw >> 8) & 127);                       // CU, SH, SE ids
}

template <int SG>
__global__ __launch_bounds__(64) void occ(unsigned *cur, unsigned *mx, unsigned long long spin) {
    extern __shared__ unsigned smem[];
    // TotalSGPRs = the highest SGPR used + 7 (VCC and the reserved ones): 78 / 94 / 106
    if (SG == 78) asm volatile("s_mov_b32 s71, 0" ::: "s71");
    if (SG == 94) asm volatile("s_mov_b32 s87, 0" ::: "s87");
    if (SG == 106) asm volatile("s_mov_b32 s99, 0" ::: "s99");
    const unsigned s = cu_slot();
    if (threadIdx.x == 0) {
        const unsigned old = atomicAdd(cur + s, 1u);
        atomicMax(mx + s, old + 1);
    }
    smem[threadIdx.x] = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) atomicSub(cur + s, 1u);
}

template <int SG>
void run(size_t lds, unsigned *cur, unsigned *mx) {
    hipMemset(cur, 0, SLOTS * 4);
    hipMemset(mx, 0, SLOTS * 4);
    if (lds > 64 * 1024) hipFuncSetAttribute(reinterpret_cast<const void *>(&occ<SG>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(occ<SG>, dim3(256 * 48), dim3(64), lds, 0, cur, mx, 5000ull);
    hipDeviceSynchronize();
    std::vector<unsigned> h(SLOTS);
    hipMemcpy(h.data(), mx, SLOTS * 4, hipMemcpyDeviceToHost);
    unsigned cus = 0, lo = ~0u, hi = 0;
    for (unsigned v : h) if (v) { cus++; lo = std::min(lo, v); hi = std::max(hi, v); }
    printf("sgpr_req=%3d lds=%6zu  CUs=%u  max resident per CU: min %u max %u\n", SG, lds, cus, lo, hi);
}

int main() {
    unsigned *cur, *mx;
    hipMalloc(&cur, SLOTS * 4);
    hipMalloc(&mx, SLOTS * 4);
    for (size_t lds : {256, 4096, 4864, 5120, 5121, 5632, 6144, 6200, 6400, 6656, 8192})
        run<0>(lds, cur, mx);
    for (size_t lds : {4864, 6200}) { run<78>(lds, cur, mx); run<94>(lds, cur, mx); run<106>(lds, cur, mx); }
    return 0;
}
