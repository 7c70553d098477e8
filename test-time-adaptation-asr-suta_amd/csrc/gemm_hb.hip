// bf16 GEMM on bf16 operand planes (LDS-DMA staging, 64-deep K-steps) + the fp32 -> bf16 plane conversion.
#include "gemm_kernels.h"
#include <cstdlib>

// ns: 2 (default) | 3 = three LDS stages | 4 = 128-deep bf16 K-steps, two stages (benchmark variants,
// tools/hb_bench); tile 4 = 256x128, 5 = 128x256 (benchmark only)
void gemm_run_hb(int tile, int ns, const GemmParams& p, dim3 grid, hipStream_t st) {
    if (tile == 6) {  // 256 x 256 ping-pong (K % 32 == 0, no split-K)
        const char* e = std::getenv("SUTA_HB8_PF");  // 1: fragments read one phase ahead
        launch_hb8(p, grid, st, e && atoi(e) == 1);
        return;
    }
    if (tile == 4) {
        launch_hb<256, 128, 2>(p, grid, st);
        return;
    }
    if (tile == 5) {
        launch_hb<128, 256, 2>(p, grid, st);
        return;
    }

    if (ns == 5 || ns == 6) {  // 32-deep bf16 K-steps: 4 (ns 5) or 3 (ns 6) LDS stages of 16 KB at 128 x 128
        if (ns == 5) launch_hb<128, 128, 4, 16>(p, grid, st);
        else launch_hb<128, 128, 3, 16>(p, grid, st);
        return;
    }
    if (ns == 4) {
        if (tile == 0) launch_hb<128, 128, 2, 64>(p, grid, st);
        else if (tile == 1) launch_hb<128, 64, 2, 64>(p, grid, st);
        else if (tile == 2) launch_hb<64, 128, 2, 64>(p, grid, st);
        else launch_hb<64, 64, 2, 64>(p, grid, st);
        return;
    }
    if (ns == 3) {
        if (tile == 0) launch_hb<128, 128, 3>(p, grid, st);
        else if (tile == 1) launch_hb<128, 64, 3>(p, grid, st);
        else if (tile == 2) launch_hb<64, 128, 3>(p, grid, st);
        else launch_hb<64, 64, 3>(p, grid, st);
        return;
    }
    if (tile == 0) launch_hb<128, 128, 2>(p, grid, st);
    else if (tile == 1) launch_hb<128, 64, 2>(p, grid, st);
    else if (tile == 2) launch_hb<64, 128, 2>(p, grid, st);
    else launch_hb<64, 64, 2>(p, grid, st);
}

namespace {
// one thread per 8 elements: two 16-B loads, one 16-B store
__global__ __launch_bounds__(256) void to_bf16_kernel(const float* __restrict__ src, long lds, long rows, int K,
                                                      bf16x8* __restrict__ dst) {
    const int k8 = K / 8;
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= rows * k8) return;
    const long r = i / k8;
    const int c = (int)(i % k8) * 8;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(src + r * lds + c);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(src + r * lds + c + 4);
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        v[e] = (__bf16)lo[e];
        v[4 + e] = (__bf16)hi[e];
    }
    dst[i] = v;
}
}  // namespace

void launch_to_bf16(const float* src, long lds, long rows, int K, void* dst, hipStream_t st) {
    const long n = rows * (K / 8);
    if (n <= 0) return;
    hipLaunchKernelGGL(to_bf16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, lds, rows, K,
                       reinterpret_cast<bf16x8*>(dst));
}
