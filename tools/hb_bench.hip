// bf16-plane GEMM (gemm_hb_kernel) microbenchmark + check on the C4 (w2v2-large, 64 x 8 s) linear shapes.
// Build: hipcc -O3 --offload-arch=gfx950 -I test-time-adaptation-asr-suta_amd/csrc -c tools/hb_bench.hip -o /tmp/hb.o
//        && hipcc --offload-arch=gfx950 /tmp/hb.o test-time-adaptation-asr-suta_amd/csrc/gemm*.o -o tools/hb_bench
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "common.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void fillb(__bf16* x, long n, unsigned seed) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { unsigned h = (unsigned)(i * 2654435761u) ^ seed; h ^= h >> 13; h *= 0x5bd1e995; h ^= h >> 15;
                 x[i] = (__bf16)((h & 0xffffff) / 16777216.0f - 0.5f); }
}
// C[m][n] = sum_k A[m][k] B[n][k] for a sample of rows
__global__ void ref(const __bf16* A, const __bf16* B, int M, int N, int K, int rstep, float* out) {
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    int rows = (M + rstep - 1) / rstep;
    if (i >= (long)rows * N) return;
    int m = (int)(i / N) * rstep, n = (int)(i % N);
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += (float)A[(long)m * K + k] * (float)B[(long)n * K + k];
    out[i] = s;
}

int main(int argc, char** argv) {
    const int M = 25536;
    struct S { const char* name; int N, K; } shapes[] = {
        {"qkv  N3072 K1024", 3072, 1024}, {"out  N1024 K1024", 1024, 1024}, {"ffn1 N4096 K1024", 4096, 1024},
        {"ffn2 N1024 K4096", 1024, 4096}, {"dqkv N1024 K3072", 1024, 3072}, {"edge N1000 K1024", 1000, 1024}};
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    __bf16 *A, *B;
    float *C, *R;
    CK(hipMalloc(&A, (size_t)M * 4096 * 2));
    CK(hipMalloc(&B, (size_t)4096 * 4096 * 2));
    CK(hipMalloc(&C, (size_t)M * 4096 * 4));
    CK(hipMalloc(&R, (size_t)M * 4096 * 4));
    hipLaunchKernelGGL(fillb, dim3((M * 4096L + 255) / 256), dim3(256), 0, 0, A, (long)M * 4096, 1u);
    hipLaunchKernelGGL(fillb, dim3((4096L * 4096 + 255) / 256), dim3(256), 0, 0, B, 4096L * 4096, 2u);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // (tile, ns, pf) -- gemm_run_hb (6: 256x256 ping-pong; pf: SUTA_HB8_PF, fragments read one phase ahead)
    const int variants[][3] = {{0, 2, 0}, {0, 5, 0}, {0, 6, 0}, {6, 2, 0}, {0, 2, 0}, {0, 5, 0}, {0, 6, 0}, {6, 2, 0}};
    __bf16* Cb;
    CK(hipMalloc(&Cb, (size_t)M * 4096 * 2));
    for (auto& s : shapes) {
        for (auto& vt : variants) {
            const int ti = vt[0], ns = vt[1];
            setenv("SUTA_HB8_PF", vt[2] ? "1" : "0", 1);
            {
                GemmParams p;
                gemm_init(p);
                p.mode = 2;
                p.A = reinterpret_cast<const float*>(A);  // unused by the plane kernel (alignment only)
                p.B = reinterpret_cast<const float*>(B);
                p.M = M; p.N = s.N; p.K = s.K;
                p.lda = s.K; p.ldb = s.K; p.tb = 1;
                p.C = C; p.ldc = s.N;
                p.Ab = A; p.Bb = B; p.ldab = s.K; p.ldbb = s.K;
                gemm_set_variant(ti, ns);
                for (int w = 0; w < 3; ++w) gemm_launch(p, 0, nullptr, 0);
                CK(hipEventRecord(e0, 0));
                for (int r = 0; r < reps; ++r) gemm_launch(p, 0, nullptr, 0);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                ms /= reps;
                const double tf = 2.0 * M * s.N * (double)s.K / (ms * 1e-3) / 1e12;
                // check a row sample
                const int rstep = 97, rows = (M + rstep - 1) / rstep;
                hipLaunchKernelGGL(ref, dim3(((long)rows * s.N + 255) / 256), dim3(256), 0, 0, A, B, M, s.N, s.K, rstep, R);
                std::vector<float> hc((size_t)M * s.N), hr((size_t)rows * s.N);
                CK(hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost));
                double err = 0, errb = 0;
                {   // the bf16 copy of C (epilogue CB path): one extra launch with the plane on
                    GemmParams q = p;
                    q.Cb = Cb; q.ldcb = s.N;
                    gemm_launch(q, 0, nullptr, 0);
                    CK(hipDeviceSynchronize());
                    std::vector<__bf16> hb((size_t)M * s.N);
                    CK(hipMemcpy(hb.data(), Cb, hb.size() * 2, hipMemcpyDeviceToHost));
                    for (size_t i = 0; i < hb.size(); i += 13) errb = fmax(errb, fabs((float)hb[i] - hc[i]) / (fabs(hc[i]) + 1.0));
                }
                for (int r = 0; r < rows; ++r)
                    for (int n = 0; n < s.N; ++n)
                        err = fmax(err, fabs(hc[(size_t)r * rstep * s.N + n] - hr[(size_t)r * s.N + n]));
                printf("%s tile %d ns %d pf %d: %.4f ms %.1f TF maxerr %.2e bf16-copy relerr %.2e\n", s.name, ti, ns, vt[2], ms, tf, err, errb);
                fflush(stdout);
            }
    }
    }
    return 0;
}
