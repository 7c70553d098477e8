// bf16 GEMM on bf16 operand planes (LDS-DMA staging, 64-deep K-steps) + the fp32 -> bf16 plane conversion.
#include "gemm_kernels.h"
#include <cstdlib>

// ns: 2 (default) | 3 = three LDS stages | 4 = 128-deep bf16 K-steps, two stages (benchmark variants,
// tools/hb_bench); tile 4 = 256x128, 5 = 128x256 (benchmark only)
void gemm_run_hb(int tile, int ns, const GemmParams& p, dim3 grid, hipStream_t st) {
    if (p.segK > 0) {  // conv input gradient on bf16 planes (128 x 128, conv-A rows, per-tap B segments)
        if (p.segB) launch_hb<128, 128, 2, 32, 4, true, true>(p, grid, st);
        else launch_hb<128, 128, 2, 32, 4, true, false>(p, grid, st);
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
    if (tile == 0 && gemm_run_hb_class(p, grid, st)) return;
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

// Per-slot transposed bf16 copy of a trainable [K][N] fp32 matrix (conv weights [tap][C_in][C_out] of every
// utterance slot): dst[z][n][k] = bf16(src[z * zs + k * N + n]), 64 x 64 tiles through LDS (coalesced both
// ways).  The B operand of the bf16-plane conv GEMMs ([N][K], k-contiguous), rebuilt after every AdamW step.
// dstn (optional): the same values in the source layout, dstn[z][k][n] (the conv input gradient's B operand),
// from the same read.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const float* __restrict__ src, long zs, int K, int N,
                                                             __bf16* __restrict__ dst, __bf16* __restrict__ dstn) {
    __shared__ float t[64][65];
    const int z = blockIdx.z, k0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
    const float* s = src + (long)z * zs;
    __bf16* d = dst + (long)z * N * K;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int k = k0 + r, n = n0 + tx;
        const float v = (k < K && n < N) ? s[(long)k * N + n] : 0.f;
        t[r][tx] = v;
        if (dstn && k < K && n < N) dstn[(long)z * N * K + (long)k * N + n] = (__bf16)v;
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int n = n0 + r, k = k0 + tx;
        if (n < N && k < K) d[(long)n * K + k] = (__bf16)t[tx][r];
    }
}

void launch_transpose_bf16(const float* src, long zs, int Z, int K, int N, void* dst, hipStream_t st, void* dstn) {
    hipLaunchKernelGGL(transpose_bf16_kernel, dim3((N + 63) / 64, (K + 63) / 64, Z), dim3(256), 0, st, src, zs, K, N,
                       reinterpret_cast<__bf16*>(dst), reinterpret_cast<__bf16*>(dstn));
}

void gemm_run_hbt(const GemmParams& p, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL((gemm_hbt_kernel<128, 128>), grid, dim3(256), 0, st, p);
}
