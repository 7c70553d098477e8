// Flash attention microbenchmark on the bench shapes (config C4: B = 164, T = 399, 16 heads of 64, bf16 planes;
// config C2: 12 heads, exact fp32): times launch_flash_fwd / launch_flash_bwd (HIP events, `reps` calls each) and
// prints a checksum of dQ / dK / dV so two library builds (or switch settings) can be compared.
// Build: C=test-time-adaptation-asr-suta_amd/csrc
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I $C -c tools/attn_bench.hip -o /tmp/ab.o
//   hipcc --offload-arch=gfx950 /tmp/ab.o $(ls $C/*.o | grep -v engine.o) -o tools/attn_bench
// Run:   tools/attn_bench <bf16 0|1> [B] [T] [NH] [reps]
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"
#include "ops.h"

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__);                        \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

__global__ void fill(float* x, long n, unsigned seed, float amp) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned h = (unsigned)(i * 2654435761u) ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995;
    h ^= h >> 15;
    x[i] = amp * ((h & 0xffffff) / 16777216.0f - 0.5f);
}
__global__ void to_bf(const float* x, __bf16* y, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = (__bf16)x[i];
}
// delta[b][h][t] = sum_d dctx[b t][h d] ctx[b t][h d]
__global__ void delta_k(const float* dctx, const float* ctx, float* delta, int B, int T, int NH) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)B * NH * T) return;
    const int t = (int)(i % T), hd = (int)((i / T) % NH), b = (int)(i / ((long)T * NH));
    const long o = ((long)b * T + t) * NH * 64 + hd * 64;
    float s = 0.f;
    for (int d = 0; d < 64; ++d) s += dctx[o + d] * ctx[o + d];
    delta[i] = s;
}
// deterministic checksum: one block, fixed per-thread strides, fixed-order final sum
__global__ void absum(const float* x, long n, double* out) {
    __shared__ double part[256];
    double s = 0;
    for (long i = threadIdx.x; i < n; i += 256) s += fabs(x[i]) * ((i % 7) + 1);
    part[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0;
        for (int k = 0; k < 256; ++k) t += part[k];
        *out = t;
    }
}
__global__ void bf_to_f(const __bf16* x, float* y, long n) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = (float)x[i];
}

int main(int argc, char** argv) {
    const bool bf16 = argc > 1 ? atoi(argv[1]) != 0 : true;
    const int B = argc > 2 ? atoi(argv[2]) : 164, T = argc > 3 ? atoi(argv[3]) : 399;
    const int NH = argc > 4 ? atoi(argv[4]) : (bf16 ? 16 : 12), reps = argc > 5 ? atoi(argv[5]) : 20;
    const int H = NH * 64;
    const long rows = (long)B * T;
    suta_latch_switches();
    float *qkv, *ctx, *dctx, *lse, *delta, *dqkv, *dqp, *tmp;
    __bf16 *qkvb, *ctxb, *dctxb, *dqkvb;
    CK(hipMalloc(&qkv, rows * 3 * H * 4));
    CK(hipMalloc(&ctx, rows * H * 4));
    CK(hipMalloc(&dctx, rows * H * 4));
    CK(hipMalloc(&lse, rows * NH * 4));
    CK(hipMalloc(&delta, rows * NH * 4));
    CK(hipMalloc(&dqkv, rows * 3 * H * 4));
    CK(hipMalloc(&tmp, rows * 3 * H * 4));
    CK(hipMalloc(&dqp, flash_dq_scratch_floats(B, T, NH) * 4));
    CK(hipMalloc(&qkvb, rows * 3 * H * 2));
    CK(hipMalloc(&ctxb, rows * H * 2));
    CK(hipMalloc(&dctxb, rows * H * 2));
    CK(hipMalloc(&dqkvb, rows * 3 * H * 2));
    auto grid = [](long n) { return dim3((unsigned)((n + 255) / 256)); };
    hipLaunchKernelGGL(fill, grid(rows * 3 * H), dim3(256), 0, 0, qkv, rows * 3 * H, 1u, 4.0f);
    hipLaunchKernelGGL(fill, grid(rows * H), dim3(256), 0, 0, dctx, rows * H, 2u, 0.02f);
    hipLaunchKernelGGL(to_bf, grid(rows * 3 * H), dim3(256), 0, 0, qkv, qkvb, rows * 3 * H);
    hipLaunchKernelGGL(to_bf, grid(rows * H), dim3(256), 0, 0, dctx, dctxb, rows * H);
    const float scale = 0.125f;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    auto fwd = [&] {
        launch_flash_fwd(bf16 ? nullptr : qkv, ctx, lse, B, T, NH, H, 64, scale, nullptr, bf16, st,
                         bf16 ? ctxb : nullptr, bf16 ? qkvb : nullptr);
    };
    auto bwd = [&] {
        // bf16 mode as the engine runs it: dQ / dK / dV only as the bf16 plane (the fp32 dqkv is not written)
        launch_flash_bwd(bf16 ? nullptr : qkv, dctx, lse, delta, bf16 ? nullptr : dqkv, dqp, B, T, NH, H, 64, scale,
                         nullptr, bf16, st,
                         bf16 ? dqkvb : nullptr, bf16 ? qkvb : nullptr, bf16 ? dctxb : nullptr);
    };
    fwd();
    hipLaunchKernelGGL(delta_k, grid(rows * NH), dim3(256), 0, st, dctx, ctx, delta, B, T, NH);
    CK(hipMemsetAsync(dqkv, 0, rows * 3 * H * 4, st));
    bwd();
    CK(hipStreamSynchronize(st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time_it = [&](auto f) {
        float best = 1e30f, tot = 0.f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, st));
            f();
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = std::min(best, ms);
            tot += ms;
        }
        return std::make_pair(best, tot / reps);
    };
    const auto tf = time_it(fwd);
    const auto tb = time_it(bwd);
    const double unit = 2.0 * T * T * 64.0 * NH * B;
    // checksums of dQ, dK, dV (fp32 columns; in bf16 mode the bf16 plane widened)
    const float* src = dqkv;
    if (bf16) {
        hipLaunchKernelGGL(bf_to_f, grid(rows * 3 * H), dim3(256), 0, st, dqkvb, tmp, rows * 3 * H);
        src = tmp;
    }
    double* dsum;
    CK(hipMalloc(&dsum, 8));
    CK(hipMemsetAsync(dsum, 0, 8, st));
    hipLaunchKernelGGL(absum, dim3(1), dim3(256), 0, st, src, rows * 3 * H, dsum);
    double h = 0;
    CK(hipMemcpy(&h, dsum, 8, hipMemcpyDeviceToHost));
    printf("%s B=%d T=%d NH=%d  fwd %.3f ms (avg %.3f) %.1f TF   bwd %.3f ms (avg %.3f) %.1f TF  checksum %.9e\n",
           bf16 ? "bf16" : "fp32", B, T, NH, tf.first, tf.second, 2 * unit / (tf.first * 1e-3) / 1e12, tb.first,
           tb.second, 4 * unit / (tb.first * 1e-3) / 1e12, h);
    return 0;
}
