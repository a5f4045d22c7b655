// WRITE_SIZE / FETCH_SIZE calibration for the replay kernel's access widths.
// Each kernel moves a known number of bytes in one of the shapes dt_replay.hip issues; run it
// under `rocprofv3 --pmc WRITE_SIZE` (and FETCH_SIZE, TCC_EA0_WRREQ_sum, ...) and divide the
// counter by the printed algorithmic bytes.  Also prints each kernel's time (hipEvents).
//   scatter4     one 4-byte store per lane, every lane in a different random 128-B line
//   row256       64 lanes x 4 B contiguous (a block's items row)
//   atom_ret     workgroup-scope returning atomic add (cv_add), random lines
//   atom_nr_x2   workgroup-scope non-returning 8-byte atomic xor (mask toggles), random lines
//   atom_ret_l2  returning atomic add confined to a 1 MiB window (L2-resident)
//   store_l2     4-byte scattered stores confined to a 1 MiB window, repeated
//   gather4      one 4-byte load per lane, every lane in a different random 128-B line
//   rowload256   64 lanes x 4 B contiguous loads of random 256-B rows
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { if ((x) != hipSuccess) { printf("hip error %s line %d\n", #x, __LINE__); return 1; } } while (0)

__device__ __forceinline__ uint32_t hsh(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

// n_wave_instr wave-instructions per wave; words = buffer size in 4-byte words (power of two)
__global__ void scatter4(uint32_t *buf, uint32_t mask_lines, int iters) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    for (int i = 0; i < iters; i++) {
        const uint32_t line = hsh(g * 977u + uint32_t(i) * 0x9E3779B9u) & mask_lines;
        buf[line * 32u] = g + uint32_t(i);
    }
}
__global__ void row256(uint32_t *buf, uint32_t mask_rows, int iters) {
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, l = threadIdx.x & 63u;
    for (int i = 0; i < iters; i++) {
        const uint32_t row = hsh(w * 131u + uint32_t(i) * 0x9E3779B9u) & mask_rows;
        buf[row * 64u + l] = w + uint32_t(i);
    }
}
__global__ void gather4(const uint32_t *buf, uint32_t mask_lines, int iters, uint32_t *sink) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (int i = 0; i < iters; i++) {
        const uint32_t line = hsh(g * 977u + uint32_t(i) * 0x9E3779B9u) & mask_lines;
        acc += buf[line * 32u];
    }
    if (acc == 0xFFFFFFFFu) sink[0] = acc;
}
__global__ void rowload256(const uint32_t *buf, uint32_t mask_rows, int iters, uint32_t *sink) {
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, l = threadIdx.x & 63u;
    uint32_t acc = 0;
    for (int i = 0; i < iters; i++) {
        const uint32_t row = hsh(w * 131u + uint32_t(i) * 0x9E3779B9u) & mask_rows;
        acc += buf[row * 64u + l];
    }
    if (acc == 0xFFFFFFFFu) sink[0] = acc;
}
__global__ void atom_ret(uint32_t *buf, uint32_t mask_lines, int iters, uint32_t *sink) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (int i = 0; i < iters; i++) {
        const uint32_t line = hsh(g * 977u + uint32_t(i) * 0x9E3779B9u) & mask_lines;
        acc += __hip_atomic_fetch_add(buf + line * 32u, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (acc == 0xFFFFFFFFu) sink[0] = acc;
}
__global__ void atom_nr_x2(unsigned long long *buf, uint32_t mask_lines, int iters) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    for (int i = 0; i < iters; i++) {
        const uint32_t line = hsh(g * 977u + uint32_t(i) * 0x9E3779B9u) & mask_lines;
        __hip_atomic_fetch_xor(buf + line * 16u, 1ull << (g & 63u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

int main() {
    const size_t bytes = size_t(1) << 31;   // 2 GiB: far beyond L2 + Infinity Cache
    uint32_t *buf, *sink;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&sink, 256));
    CHECK(hipMemset(buf, 0, bytes));
    const uint32_t lines_all = uint32_t(bytes / 128) - 1;       // 2^24 - 1
    const uint32_t lines_l2 = (1u << 20) / 128 - 1;              // 1 MiB window
    const int grid = 2048, block = 256, iters = 64;
    const double lanes = double(grid) * block * iters;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    auto run = [&](const char *name, double alg_bytes, auto launch) {
        launch();                                     // warm (page tables)
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a));
        launch();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        printf("%-12s alg_bytes_per_dispatch=%.0f ms=%.3f (each kernel is dispatched twice; divide the "
               "per-dispatch counter by alg_bytes)\n", name, alg_bytes, ms);
        return 0;
    };
    run("scatter4", lanes * 4, [&] { hipLaunchKernelGGL(scatter4, dim3(grid), dim3(block), 0, 0, buf, lines_all, iters); });
    run("row256", lanes * 4, [&] { hipLaunchKernelGGL(row256, dim3(grid), dim3(block), 0, 0, buf, uint32_t(bytes / 256) - 1, iters); });
    run("atom_ret", lanes * 4, [&] { hipLaunchKernelGGL(atom_ret, dim3(grid), dim3(block), 0, 0, buf, lines_all, iters, sink); });
    run("atom_nr_x2", lanes * 8, [&] { hipLaunchKernelGGL(atom_nr_x2, dim3(grid), dim3(block), 0, 0, (unsigned long long *)buf, lines_all, iters); });
    run("atom_ret_l2", lanes * 4, [&] { hipLaunchKernelGGL(atom_ret, dim3(grid), dim3(block), 0, 0, buf, lines_l2, iters, sink); });
    run("gather4", lanes * 4, [&] { hipLaunchKernelGGL(gather4, dim3(grid), dim3(block), 0, 0, buf, lines_all, iters, sink); });
    run("rowload256", lanes * 4, [&] { hipLaunchKernelGGL(rowload256, dim3(grid), dim3(block), 0, 0, buf, uint32_t(bytes / 256) - 1, iters, sink); });
    run("store_l2", lanes * 4, [&] { hipLaunchKernelGGL(scatter4, dim3(grid), dim3(block), 0, 0, buf, lines_l2, iters); });
    return 0;
}
