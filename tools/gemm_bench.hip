// Standalone fp32-MFMA GEMM microbenchmark + correctness check for the SUTA shapes.
// Build (after make in csrc): hipcc -O3 --offload-arch=gfx950 -I test-time-adaptation-asr-suta_amd/csrc -c tools/gemm_bench.hip -o gb.o
//        && hipcc --offload-arch=gfx950 gb.o test-time-adaptation-asr-suta_amd/csrc/gemm*.o -o tools/gemm_bench
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "common.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void ref_gemm(GemmParams p, float* out) {
    // out[z][m][n] = sum_k A(m,k) B(k,n)   (no epilogue), one thread per output
    long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
    long MN = (long)p.M * p.N;
    if (idx >= MN * p.Z) return;
    int z = idx / MN; long r = idx % MN; int m = r / p.N, n = r % p.N;
    int z1 = z / p.zdiv, z0 = z % p.zdiv;
    const float* A = p.A + z1 * p.sA1 + z0 * p.sA0;
    const float* B = p.B + z1 * p.sB1 + z0 * p.sB0;
    double s = 0;
    for (int k = 0; k < p.K; ++k) {
        float a;
        if (p.segK > 0) {
            int seg = k / p.segK, rr = k % p.segK, srow = m + seg - p.pad;
            a = (srow >= 0 && srow < p.Mvalid) ? A[(long)srow * p.lda + rr] : 0.f;
        } else a = p.ta ? A[(long)k * p.lda + m] : A[(long)m * p.lda + k];
        float b = p.tb ? B[(long)n * p.ldb + k] : B[(long)k * p.ldb + n];
        s += (double)a * b;
    }
    out[idx] = (float)s;
}

__global__ void fill(float* x, long n, unsigned seed) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { unsigned h = (unsigned)(i * 2654435761u) ^ seed; h ^= h >> 13; h *= 0x5bd1e995; h ^= h >> 15;
                 x[i] = ((h & 0xffffff) / 16777216.0f - 0.5f); }
}

// register-only MFMA loop: the practical fp32 MFMA ceiling (and clock) under load
__global__ __launch_bounds__(256) void mfma_peak(float* out, int iters, float seed) {
    f32x16 acc[4];
    for (int j = 0; j < 4; ++j) for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    float a = seed * (threadIdx.x + 1), b = seed * (blockIdx.x + 3);
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
        a += 1e-7f; b -= 1e-7f;
    }
    float s = 0; for (int j = 0; j < 4; ++j) for (int r = 0; r < 16; ++r) s += acc[j][r];
    if (s == 12345.f) out[0] = s;
}

struct Shape { const char* name; int M, N, K, Z, zdiv; int ta, tb; long lda, ldb, ldc, sA0, sA1, sB0, sB1, sC0, sC1;
               long Asz, Bsz, Csz; int segK, pad, Mvalid; double flops_scale; };

int main(int argc, char** argv) {
    const int Bu = 64, T = 399, Tp = 400, H = 768, F = 3072, L1 = 12799, L0 = 25599, NH = 12;
    std::vector<Shape> S = {
        {"ffn1_fwd NT", Bu*T, F, H, 1, 1, 0, 1, H, H, F, 0,0,0,0,0,0, (long)Bu*T*H, (long)F*H, (long)Bu*T*F, 0,0,0, 1},
        {"qkv_fwd NT", Bu*T, 3*H, H, 1, 1, 0, 1, H, H, 3*H, 0,0,0,0,0,0, (long)Bu*T*H, 3L*H*H, (long)Bu*T*3*H, 0,0,0, 1},
        {"ffn2_fwd NT", Bu*T, H, F, 1, 1, 0, 1, F, F, H, 0,0,0,0,0,0, (long)Bu*T*F, (long)F*H, (long)Bu*T*H, 0,0,0, 1},
        {"oproj_fwd NT", Bu*T, H, H, 1, 1, 0, 1, H, H, H, 0,0,0,0,0,0, (long)Bu*T*H, (long)H*H, (long)Bu*T*H, 0,0,0, 1},
        {"dh1 NN", Bu*T, H, F, 1, 1, 0, 0, F, H, H, 0,0,0,0,0,0, (long)Bu*T*F, (long)F*H, (long)Bu*T*H, 0,0,0, 1},
        {"du NN", Bu*T, F, H, 1, 1, 0, 0, H, F, F, 0,0,0,0,0,0, (long)Bu*T*H, (long)F*H, (long)Bu*T*F, 0,0,0, 1},
        {"dqkv->dx NN", Bu*T, H, 3*H, 1, 1, 0, 0, 3*H, H, H, 0,0,0,0,0,0, (long)Bu*T*3*H, 3L*H*H, (long)Bu*T*H, 0,0,0, 1},
        {"conv1_fwd NN", L1, 512, 1536, Bu, 1, 0, 0, 1024, 512, 512, 0,(long)L0*512, 0,1536L*512, 0,(long)L1*512,
            (long)Bu*L0*512, (long)Bu*1536*512, (long)Bu*L1*512, 0,0,0, 1},
        {"conv1_dcol NT", L1, 1536, 512, Bu, 1, 0, 1, 512, 512, 1536, 0,(long)L1*512, 0,1536L*512, 0,(long)L1*1536,
            (long)Bu*L1*512, (long)Bu*1536*512, (long)Bu*L1*1536, 0,0,0, 1},
        {"conv1_dW TN", 1536, 512, L1, Bu, 1, 1, 0, 1024, 512, 512, 0,(long)L0*512, 0,(long)L1*512, 0,1536L*512,
            (long)Bu*L0*512, (long)Bu*L1*512, (long)Bu*1536*512, 0,0,0, 1},
        {"attn_S NT", T, T, 64, Bu*NH, NH, 0, 1, 3*H, 3*H, Tp, 64,(long)T*3*H, 64,(long)T*3*H, (long)T*Tp,(long)NH*T*Tp,
            (long)Bu*T*3*H, (long)Bu*T*3*H, (long)Bu*NH*T*Tp, 0,0,0, 1},
        {"attn_PV NN", T, 64, T, Bu*NH, NH, 0, 0, Tp, 3*H, H, (long)T*Tp,(long)NH*T*Tp, 64,(long)T*3*H, 64,(long)T*H,
            (long)Bu*NH*T*Tp, (long)Bu*T*3*H, (long)Bu*T*H, 0,0,0, 1},
        {"attn_dK TN", T, 64, T, Bu*NH, NH, 1, 0, Tp, 3*H, 3*H, (long)T*Tp,(long)NH*T*Tp, 64,(long)T*3*H, 64,(long)T*3*H,
            (long)Bu*NH*T*Tp, (long)Bu*T*3*H, (long)Bu*T*3*H, 0,0,0, 1},
        {"posconv conv-A", T, 48, 128*48, Bu*16, 16, 0, 0, H, 48, H, 48,(long)T*H, 128L*48*48,0, 48,(long)T*H,
            (long)Bu*T*H, 16L*128*48*48, (long)Bu*T*H, 48, 64, T, 1},
    };
    float *A, *B, *C, *R;
    long maxA = 0, maxB = 0, maxC = 0;
    for (auto& s : S) { maxA = std::max(maxA, s.Asz); maxB = std::max(maxB, s.Bsz); maxC = std::max(maxC, s.Csz); }
    CK(hipMalloc(&A, maxA * 4)); CK(hipMalloc(&B, maxB * 4)); CK(hipMalloc(&C, maxC * 4)); CK(hipMalloc(&R, maxC * 4));
    float* ws; long wsf = 32L << 20; CK(hipMalloc(&ws, wsf * 4));
    hipLaunchKernelGGL(fill, dim3((maxA + 255) / 256), dim3(256), 0, 0, A, maxA, 1u);
    hipLaunchKernelGGL(fill, dim3((maxB + 255) / 256), dim3(256), 0, 0, B, maxB, 2u);
    hipStream_t st; CK(hipStreamCreate(&st));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int variants[][2] = {{-1, 1}, {-1, 3}, {0, 3}, {0, 7}, {0, 5}, {0, 6}, {1, 3}, {1, 7},
                               {3, 3}, {3, 7}, {2, 3}, {2, 7}, {0, 1}, {3, 1}, {-1, 7}, {-1, 8}, {-1, 9}, {-1, 10}, {0, 11}, {4, 11}, {5, 11}};
    const char* vname[] = {"auto/1buf", "auto/g32x2", "128/g32x2", "128/g64x2", "128/g16x3", "128/g32x3",
                           "128x64/g32x2", "128x64/g64x2", "64/g32x2", "64/g64x2", "64x128/g32", "64x128/g64",
                           "128/1buf", "64/1buf", "auto/g64x2", "auto/v8", "auto/v9", "auto/v10",
                           "x1-128", "x1-256x128", "x1-128x256"};
    const int NV = 21;
    bool check = argc < 2 || atoi(argv[1]) != 0;
    int only_v = argc >= 3 ? atoi(argv[2]) : -1;
    int only_s = argc >= 4 ? atoi(argv[3]) : -1;
    int mode = argc >= 5 ? atoi(argv[4]) : 0;
    gemm_set_mode(mode);
    printf("GEMM mode %d (%s)\n", mode, mode == 2 ? "bf16" : mode ? "x6 bf16-split" : "exact fp32 MFMA");
    {
        const int iters = 20000, blocks = 256 * 4;
        hipLaunchKernelGGL(mfma_peak, dim3(blocks), dim3(256), 0, st, C, 100, 0.001f);
        CK(hipEventRecord(e0, st));
        hipLaunchKernelGGL(mfma_peak, dim3(blocks), dim3(256), 0, st, C, iters, 0.001f);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        double fl = 2.0 * 32 * 32 * 2 * 4.0 * iters * blocks * 4;
        printf("mfma_f32_32x32x2 register loop: %.1f TF (%.3f ms)\n", fl / (ms * 1e-3) / 1e12, ms);
    }
    for (size_t si = 0; si < S.size(); ++si) {
        auto& s = S[si];
        if (only_s >= 0 && (int)si != only_s) continue;
        GemmParams p; gemm_init(p);
        p.A = A; p.B = B; p.C = C; p.M = s.M; p.N = s.N; p.K = s.K; p.Z = s.Z; p.zdiv = s.zdiv; p.ta = s.ta; p.tb = s.tb;
        p.lda = s.lda; p.ldb = s.ldb; p.ldc = s.ldc; p.sA0 = s.sA0; p.sA1 = s.sA1; p.sB0 = s.sB0; p.sB1 = s.sB1;
        p.sC0 = s.sC0; p.sC1 = s.sC1; p.segK = s.segK; p.pad = s.pad; p.Mvalid = s.Mvalid;
        double flops = 2.0 * s.M * s.N * (double)s.K * s.Z;
        if (s.segK) flops = 2.0 * s.M * s.N * (double)s.K * s.Z;
        printf("%-16s M=%d N=%d K=%d Z=%d  %.1f GF\n", s.name, s.M, s.N, s.K, s.Z, flops / 1e9);
        float* ref = nullptr;
        if (check) {
            CK(hipMalloc(&ref, (long)s.M * s.N * s.Z * 4));
            long n = (long)s.M * s.N * s.Z;
            hipLaunchKernelGGL(ref_gemm, dim3((n + 255) / 256), dim3(256), 0, st, p, ref);
        }
        for (int v = 0; v < NV; ++v) {
            if (only_v >= 0 && v != only_v) continue;
            gemm_set_variant(variants[v][0], variants[v][1]);
            CK(hipMemsetAsync(C, 0, s.Csz * 4, st));
            gemm_launch(p, st, ws, wsf);
            CK(hipStreamSynchronize(st));
            double maxerr = 0;
            if (check) {
                // compare (C may have a stride): copy both to host
                std::vector<float> hc(s.Csz), hr((long)s.M * s.N * s.Z);
                CK(hipMemcpy(hc.data(), C, s.Csz * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hr.data(), ref, hr.size() * 4, hipMemcpyDeviceToHost));
                for (int z = 0; z < s.Z; z += std::max(1, s.Z / 4))
                    for (int m = 0; m < s.M; m += 7)
                        for (int n = 0; n < s.N; ++n) {
                            long ci = (z / s.zdiv) * s.sC1 + (z % s.zdiv) * s.sC0 + (long)m * s.ldc + n;
                            double d = fabs(hc[ci] - hr[((long)z * s.M + m) * s.N + n]);
                            maxerr = std::max(maxerr, d);
                        }
            }
            const int it = 10;
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < it; ++i) gemm_launch(p, st, ws, wsf);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            printf("   %-10s %8.3f ms  %6.1f TF  maxerr %.2e\n", vname[v], ms / it, flops / (ms / it * 1e-3) / 1e12, maxerr);
        }
        if (ref) CK(hipFree(ref));
    }
    return 0;
}
