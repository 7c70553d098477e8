// bf16-plane GEMM microbenchmark + check on the C4 linear shapes (w2v2-large, M = 164 x 399 rows: bench.py's layout):
// gemm_hb_kernel (128 x 128), gemm_hbx_kernel (256 x 256 slice ring) with its two epilogue forms (column-per-lane
// accumulators, and C^T accumulators with 16-B row-per-lane stores).  Variants run interleaved, `rounds` times each (median reported).
// Build (the SUTA_HBX_DBG diagnostic forms exist only in this tools build of gemm_hbx.hip, -DSUTA_HBX_DIAG):
//   C=test-time-adaptation-asr-suta_amd/csrc
//   hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DSUTA_HBX_DIAG -c $C/gemm_hbx.hip -o /tmp/gemm_hbx_diag.o
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I $C -c tools/hb_bench.hip -o /tmp/hb.o
//   hipcc --offload-arch=gfx950 /tmp/hb.o /tmp/gemm_hbx_diag.o $(ls $C/gemm*.o | grep -v gemm_hbx.o) $C/ops.o \
//         -o tools/hb_bench
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
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
    const int M = 164 * 399;
    struct S { const char* name; int N, K; } shapes[] = {
        {"qkv  N3072 K1024", 3072, 1024}, {"out  N1024 K1024", 1024, 1024}, {"ffn1 N4096 K1024", 4096, 1024},
        {"ffn2 N1024 K4096", 1024, 4096}, {"dqkv N1024 K3072", 1024, 3072}, {"edge N1000 K1024", 1000, 1024}};
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    const int rounds = argc > 2 ? atoi(argv[2]) : 3;
    __bf16 *A, *B;
    float *C, *R;
    CK(hipMalloc(&A, (size_t)M * 4096 * 2));
    CK(hipMalloc(&B, (size_t)4096 * 4096 * 2));
    // HB_PAD: extra elements per row of every output / epilogue-operand plane (leading dimension N + pad)
    const int pad = getenv("HB_PAD") ? atoi(getenv("HB_PAD")) : 0;
    CK(hipMalloc(&C, (size_t)M * (4096 + pad) * 4));
    CK(hipMalloc(&R, (size_t)M * 4096 * 4));
    hipLaunchKernelGGL(fillb, dim3((M * 4096L + 255) / 256), dim3(256), 0, 0, A, (long)M * 4096, 1u);
    hipLaunchKernelGGL(fillb, dim3((4096L * 4096 + 255) / 256), dim3(256), 0, 0, B, 4096L * 4096, 2u);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // (tile, ns, cb-capable, SUTA_HBX_T): 0 = hb 128 x 128, 8 = hbx (32x32x16) with the column-per-lane epilogue
    // and with C^T accumulators + the row-per-lane epilogue (hbxT)
    // (tile, ns, cb-capable, SUTA_HBX_T, SUTA_HBX_DBG): the DBG forms are diagnostics (wrong results): 1 no B DMA,
    // 2 no B fragment reads, 3 no DMA, 4 no fragment reads
    // + SUTA_HBX_FORM (6th): 1 the four-phase K-tile schedule (gemm_hbp_kernel), 2 the same with staggered wave groups
    // 3: the four-phase schedule with three half-tiles of DMA in flight and one counted wait per K-tile; 4: form 3 on
    // 16x16x32 MFMAs
    // SUTA_HBX_FORM 5: form 4 persistent; SUTA_HBX_DBG 11 / 12 / 13 / 14 / 15 (HB_DIAG=1 only): form 4 without its epilogue / K loop / both / epilogue
    // global stores / accumulator remap (profiles/r6/hbp_diag*.txt)
    // SUTA_HBX_DBG 16: form 4 with the accumulators remapped to the 32x32 layout and epilogue_t (the first form 4);
    // HB_DIAG=1: + SUTA_HBX_DBG 11 .. 15 on that form (tools build only; wrong results): without its epilogue / K loop /
    // both / the epilogue's global stores / the accumulator remap (profiles/r6/hbp_diag*.txt)
    const int variants[][6] = {{8, 2, 1, 2, 0, 3}, {8, 2, 1, 2, 0, 4}, {8, 2, 1, 2, 16, 4}, {8, 2, 1, 2, 11, 4},
                               {8, 2, 1, 2, 12, 4}, {8, 2, 1, 2, 13, 4}, {8, 2, 1, 2, 14, 4}, {8, 2, 1, 2, 15, 4}};
    const char* vname[] = {"hbpD ", "hbp16", "16-remap", "16-noepi", "16-noloop", "16-neither", "16-nostore",
                           "16-noremap"};
    int NV = getenv("HB_DIAG") ? 8 : 3;
    // HB_NT=1: form 4 (default epilogues) against the same with nontemporal epilogue stores (SUTA_HBX_DBG 17)
    int vmap[8] = {0, 1, 2, 3, 4, 5, 6, 7};
    static const int vnt[2][6] = {{8, 2, 1, 2, 0, 4}, {8, 2, 1, 2, 17, 4}};
    const char* vnt_name[2] = {"hbp16", "16-NT"};
    const bool ntmode = getenv("HB_NT") != nullptr;
    if (ntmode) NV = 2;
    (void)vmap;
    auto vrow = [&](int v) -> const int* { return ntmode ? vnt[v] : variants[v]; };
    auto set_variant = [&](int v) {
        const char* tv[] = {"0", "1", "2", "3", "4", "5", "6", "7", "8", "9", "10", "11", "12", "13", "14", "15", "16", "17"};
        setenv("SUTA_HBX_T", tv[vrow(v)[3]], 1);
        setenv("SUTA_HBX_DBG", tv[vrow(v)[4]], 1);
        setenv("SUTA_HBX_FORM", tv[vrow(v)[5]], 1);
        suta_latch_switches();
        gemm_set_variant(vrow(v)[0], vrow(v)[1]);
    };
    __bf16* Cb;
    CK(hipMalloc(&Cb, (size_t)M * (4096 + pad) * 2));
    for (auto& s : shapes) {
        GemmParams p;
        gemm_init(p);
        p.mode = 2;
        p.A = reinterpret_cast<const float*>(A);  // unused by the plane kernels (alignment only)
        p.B = reinterpret_cast<const float*>(B);
        p.M = M; p.N = s.N; p.K = s.K;
        p.lda = s.K; p.ldb = s.K; p.tb = 1;
        p.C = C; p.ldc = s.N + pad;
        p.Ab = A; p.Bb = B; p.ldab = s.K; p.ldbb = s.K;
        std::vector<float> ms[8];
        for (int rd = 0; rd < rounds; ++rd)
            for (int v = 0; v < NV; ++v) {
                set_variant(v);
                for (int w = 0; w < 2; ++w) gemm_launch(p, 0, nullptr, 0);
                CK(hipEventRecord(e0, 0));
                for (int r = 0; r < reps; ++r) gemm_launch(p, 0, nullptr, 0);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t = 0;
                CK(hipEventElapsedTime(&t, e0, e1));
                ms[v].push_back(t / reps);
            }
        for (int v = 0; v < NV; ++v) {
            set_variant(v);
            CK(hipMemset(C, 0, (size_t)M * s.N * 4));
            gemm_launch(p, 0, nullptr, 0);
            const int rstep = 97, rows = (M + rstep - 1) / rstep;
            hipLaunchKernelGGL(ref, dim3(((long)rows * s.N + 255) / 256), dim3(256), 0, 0, A, B, M, s.N, s.K, rstep, R);
            std::vector<float> hc((size_t)M * s.N), hr((size_t)rows * s.N);
            CK(hipMemcpy(hc.data(), C, hc.size() * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost));
            double err = 0, errb = -1;
            for (int r = 0; r < rows; ++r)
                for (int n = 0; n < s.N; ++n)
                    err = fmax(err, fabs(hc[(size_t)r * rstep * s.N + n] - hr[(size_t)r * s.N + n]));
            if (vrow(v)[2]) {   // the bf16 copy of C (epilogue CB path)
                GemmParams q = p;
                q.Cb = Cb; q.ldcb = s.N + pad;
                gemm_launch(q, 0, nullptr, 0);
                CK(hipDeviceSynchronize());
                std::vector<__bf16> hb((size_t)M * s.N);
                CK(hipMemcpy(hb.data(), Cb, hb.size() * 2, hipMemcpyDeviceToHost));
                errb = 0;
                for (size_t i = 0; i < hb.size(); i += 13) errb = fmax(errb, fabs((float)hb[i] - hc[i]) / (fabs(hc[i]) + 1.0));
            }
            std::vector<float> m = ms[v];
            std::sort(m.begin(), m.end());
            const float med = m[m.size() / 2], mn = m[0];
            const double tf = 2.0 * M * s.N * (double)s.K / (med * 1e-3) / 1e12;
            const double tfb = 2.0 * M * s.N * (double)s.K / (mn * 1e-3) / 1e12;
            printf("%s %s: median %.4f ms %.1f TF (best %.1f) maxerr %.2e bf16-copy relerr %.2e\n", s.name, (ntmode ? vnt_name[v] : vname[v]), med, tf,
                   tfb, err, errb);
            fflush(stdout);
        }
    }
    // HB_RESID: the residual linears (out-projection and FFN2 forward: bias + residual, fp32 C; with and without the
    // bf16 C plane)
    if (getenv("HB_RESID")) {
        float* bias;
        CK(hipMalloc(&bias, 4096 * 4));
        CK(hipMemset(bias, 0, 4096 * 4));
        struct RS { const char* name; int K; bool cb; } rs[] = {{"outR  K1024 fp32", 1024, false}, {"outR  K1024 +Cb ", 1024, true},
                                                               {"ffn2R K4096 fp32", 4096, false}};
        for (auto& r : rs) {
            GemmParams p;
            gemm_init(p);
            p.mode = 2;
            p.A = reinterpret_cast<const float*>(A);
            p.B = reinterpret_cast<const float*>(B);
            p.M = M; p.N = 1024; p.K = r.K;
            p.lda = r.K; p.ldb = r.K; p.tb = 1;
            p.C = C; p.ldc = 1024;
            p.Ab = A; p.Bb = B; p.ldab = r.K; p.ldbb = r.K;
            p.epi = EPI_BIAS | EPI_RESID;
            p.bias = bias;
            p.R = R; p.ldr = 1024;
            if (r.cb) { p.Cb = Cb; p.ldcb = 1024; }
            std::vector<float> ms[8];
            for (int rd = 0; rd < rounds; ++rd)
                for (int v = 0; v < NV; ++v) {
                    set_variant(v);
                    for (int w = 0; w < 2; ++w) gemm_launch(p, 0, nullptr, 0);
                    CK(hipEventRecord(e0, 0));
                    for (int q = 0; q < reps; ++q) gemm_launch(p, 0, nullptr, 0);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float tt = 0;
                    CK(hipEventElapsedTime(&tt, e0, e1));
                    ms[v].push_back(tt / reps);
                }
            for (int v = 0; v < NV; ++v) {
                std::vector<float> m = ms[v];
                std::sort(m.begin(), m.end());
                printf("%s %s: median %.4f ms %.1f TF  per tile round %.2f us\n", r.name, (ntmode ? vnt_name[v] : vname[v]),
                       m[m.size() / 2], 2.0 * M * 1024.0 * r.K / (m[m.size() / 2] * 1e-3) / 1e12, m[m.size() / 2] * 1e3 / 4.0);
                fflush(stdout);
            }
        }
        return 0;
    }
    // K sweep (N = 4096, bf16 C plane only): time = fixed per-tile cost (prologue + epilogue) + K x loop rate
    if (getenv("HB_KSWEEP")) {
        for (int K : {128, 256, 512, 1024, 2048, 4096}) {
            GemmParams p;
            gemm_init(p);
            p.mode = 2;
            p.A = reinterpret_cast<const float*>(A);
            p.B = reinterpret_cast<const float*>(B);
            p.M = M; p.N = 4096; p.K = K;
            p.lda = K; p.ldb = K; p.tb = 1;
            p.C = nullptr; p.ldc = 4096;
            p.Ab = A; p.Bb = B; p.ldab = K; p.ldbb = K;
            p.Cb = Cb; p.ldcb = 4096 + pad;
            std::vector<float> ms[8];
            for (int rd = 0; rd < rounds; ++rd)
                for (int v = 0; v < NV; ++v) {
                    set_variant(v);
                    for (int w = 0; w < 2; ++w) gemm_launch(p, 0, nullptr, 0);
                    CK(hipEventRecord(e0, 0));
                    for (int r = 0; r < reps; ++r) gemm_launch(p, 0, nullptr, 0);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float tt = 0;
                    CK(hipEventElapsedTime(&tt, e0, e1));
                    ms[v].push_back(tt / reps);
                }
            for (int v = 0; v < NV; ++v) {
                std::vector<float> m = ms[v];
                std::sort(m.begin(), m.end());
                const double tf = 2.0 * M * 4096.0 * K / (m[m.size() / 2] * 1e-3) / 1e12;
                printf("ksweep K%5d %s: median %.4f ms %.1f TF  per tile round %.2f us\n", K, (ntmode ? vnt_name[v] : vname[v]), m[m.size() / 2], tf,
                       m[m.size() / 2] * 1e3 / 16.0);
                fflush(stdout);
            }
        }
        return 0;
    }
    // epilogue-heavy C4 shapes (bf16 C plane only, bf16 pre-activation operand): FFN1 forward (bias + GELU +
    // pre-activation store) and the FFN2 input gradient (x GELU'(u)); variants compared on their Cb outputs
    {
        float* bias;
        __bf16 *U, *Cref;
        CK(hipMalloc(&bias, 4096 * 4));
        CK(hipMalloc(&U, (size_t)M * (4096 + pad) * 2));
        CK(hipMalloc(&Cref, (size_t)M * (4096 + pad) * 2));
        hipLaunchKernelGGL(fillb, dim3((M * 4096L + 255) / 256), dim3(256), 0, 0, U, (long)M * 4096, 3u);
        std::vector<float> hbias(4096);
        for (int i = 0; i < 4096; ++i) hbias[i] = 0.01f * (i % 17) - 0.08f;
        CK(hipMemcpy(bias, hbias.data(), 4096 * 4, hipMemcpyHostToDevice));
        // forms: 0 FFN1 (bias + GELU + bf16 pre), 1 FFN2 input gradient (x GELU'(u)), 2 FFN1 without the GELU
        // (bias + bf16 pre: the GELU's own cost), 3 no epilogue, bf16 C plane only (C dead: the QKV / FFN1 form)
        const char* fname[] = {"ffn1 epi=bias+gelu+pre", "ffn2dx epi=dgelu    ", "ffn1 epi=bias+pre    ",
                               "ffn1 epi=none Cb only "};
        for (int form = 0; form < 4; ++form) {
            GemmParams p;
            gemm_init(p);
            p.mode = 2;
            p.A = reinterpret_cast<const float*>(A);
            p.B = reinterpret_cast<const float*>(B);
            p.M = M; p.N = 4096; p.K = 1024;
            p.lda = 1024; p.ldb = 1024; p.tb = 1;
            p.C = nullptr; p.ldc = 4096;
            p.Ab = A; p.Bb = B; p.ldab = 1024; p.ldbb = 1024;
            p.Cb = Cb; p.ldcb = 4096 + pad; p.preb = 1;
            if (form == 0 || form == 2) {
                p.epi = EPI_BIAS | EPI_STORE_PRE | (form == 0 ? EPI_GELU : 0);
                p.bias = bias;
                p.C2 = reinterpret_cast<float*>(U); p.ldc2 = 4096 + pad;
            } else if (form == 1) {
                p.epi = EPI_DGELU;
                p.aux = reinterpret_cast<const float*>(U); p.ldaux = 4096 + pad;
            } else {
                p.epi = 0;
                p.preb = 0;
            }
            const int evs[] = {0, 1, 2};
            std::vector<float> ms[8];
            for (int rd = 0; rd < rounds; ++rd)
                for (int v : evs) {
                    set_variant(v);
                    if (form == 0 || form == 2) hipLaunchKernelGGL(fillb, dim3((M * 4096L + 255) / 256), dim3(256), 0, 0, U, (long)M * 4096, 3u);
                    for (int w = 0; w < 2; ++w) gemm_launch(p, 0, nullptr, 0);
                    CK(hipEventRecord(e0, 0));
                    for (int r = 0; r < reps; ++r) gemm_launch(p, 0, nullptr, 0);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float tt = 0;
                    CK(hipEventElapsedTime(&tt, e0, e1));
                    ms[v].push_back(tt / reps);
                }
            for (int v : evs) {
                set_variant(v);
                hipLaunchKernelGGL(fillb, dim3((M * 4096L + 255) / 256), dim3(256), 0, 0, U, (long)M * 4096, 3u);
                gemm_launch(p, 0, nullptr, 0);
                CK(hipDeviceSynchronize());
                double dmax = 0;
                if (v == 0) CK(hipMemcpy(Cref, Cb, (size_t)M * 4096 * 2, hipMemcpyDeviceToDevice));
                else {
                    std::vector<__bf16> a((size_t)M * 4096), b((size_t)M * 4096);
                    CK(hipMemcpy(a.data(), Cb, a.size() * 2, hipMemcpyDeviceToHost));
                    CK(hipMemcpy(b.data(), Cref, b.size() * 2, hipMemcpyDeviceToHost));
                    for (size_t i = 0; i < a.size(); i += 7) dmax = fmax(dmax, fabs((float)a[i] - (float)b[i]) / (fabs((float)b[i]) + 1.0));
                }
                std::vector<float> m = ms[v];
                std::sort(m.begin(), m.end());
                const double tf = 2.0 * M * 4096.0 * 1024.0 / (m[m.size() / 2] * 1e-3) / 1e12;
                printf("%s %s: median %.4f ms %.1f TF (best %.1f) vs hb128 Cb relerr %.2e\n",
                       fname[form], (ntmode ? vnt_name[v] : vname[v]), m[m.size() / 2], tf,
                       2.0 * M * 4096.0 * 1024.0 / (m[0] * 1e-3) / 1e12, dmax);
                fflush(stdout);
            }
        }
    }
    return 0;
}
