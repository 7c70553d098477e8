// fp32 MFMA GEMM for gfx950 (v_mfma_f32_32x32x2_f32: exact f32 products, f32 accumulate).
//
// One kernel template serves every contraction of the SUTA step: encoder linears (NT),
// their input-gradients (NN), attention QK^T / PV and their backward (NT / NN / TN),
// feature-encoder convs as strided-row GEMMs (time-major activations make the im2col
// matrix a plain matrix with lda = stride*C), their weight gradients (TN, split-K over
// time), and the grouped positional conv through the conv-A (segmented K) loader.
//
// Block = 256 threads = 4 waves (WM x WN), block tile BM x BN, K-step 16 staged through
// LDS in a k-contiguous layout [row][16 + 4 pad] so every MFMA operand is read with
// ds_read_b128 (row stride 20 dwords: conflict-free over the b128 lane groups).
// The MFMA k-pair (lane half h) takes tile-k h*8 + 4q + e, q<2, e<4, so each lane's four
// consecutive k come from one 16-B LDS read.  Global->register prefetch of stage s+1
// overlaps the MFMAs of stage s.
#include "common.h"
#include <algorithm>

namespace {

constexpr int BK = 16;
constexpr int LDK = BK + 4;

template <int ROWS>
struct Stage {
    static constexpr int LOADS = ROWS * BK / 4 / 256;  // float4 per thread
};

// Load one BK-deep stage of an operand into registers.
//   KC = true : source is k-contiguous (A with ta=0, B with tb=1): element (row, k) at row*ld + k
//   KC = false: source is row-contiguous (A with ta=1, B with tb=0): element (row, k) at k*ld + row
template <int ROWS, bool KC, bool CONV>
__device__ __forceinline__ void load_stage(f32x4 (&r)[Stage<ROWS>::LOADS], const float* __restrict__ src,
                                           long ld, int row0, int nrows, int k0, int kend, bool vec,
                                           int segK, int pad, int Mvalid) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < Stage<ROWS>::LOADS; ++i) {
        const int f = tid + i * 256;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (KC) {
            const int row = f >> 2;
            const int kq = (f & 3) * 4;
            const int gr = row0 + row;
            const int gk = k0 + kq;
            if (gr < nrows) {
                if (CONV) {
                    const int seg = gk / segK;
                    const int rr = gk - seg * segK;
                    const int srow = gr + seg - pad;
                    if (gk < kend && srow >= 0 && srow < Mvalid) {
                        // segK % 4 == 0 and gk % 4 == 0: the 4 elements stay in one segment
                        const float* s = src + (long)srow * ld + rr;
                        if (vec && gk + 3 < kend) {
                            v = *reinterpret_cast<const f32x4*>(s);
                        } else {
#pragma unroll
                            for (int e = 0; e < 4; ++e)
                                if (gk + e < kend) v[e] = s[e];
                        }
                    }
                } else {
                    const float* s = src + (long)gr * ld + gk;
                    if (vec && gk + 3 < kend) {
                        v = *reinterpret_cast<const f32x4*>(s);
                    } else {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (gk + e < kend) v[e] = s[e];
                    }
                }
            }
        } else {
            constexpr int RQ = ROWS / 4;
            const int k = f / RQ;
            const int rq = (f % RQ) * 4;
            const int gk = k0 + k;
            const int gr = row0 + rq;
            if (gk < kend) {
                const float* s = src + (long)gk * ld + gr;
                if (vec && gr + 3 < nrows) {
                    v = *reinterpret_cast<const f32x4*>(s);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (gr + e < nrows) v[e] = s[e];
                }
            }
        }
        r[i] = v;
    }
}

template <int ROWS, bool KC>
__device__ __forceinline__ void store_stage(float* __restrict__ lds, const f32x4 (&r)[Stage<ROWS>::LOADS]) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < Stage<ROWS>::LOADS; ++i) {
        const int f = tid + i * 256;
        if (KC) {
            const int row = f >> 2;
            const int kq = (f & 3) * 4;
            *reinterpret_cast<f32x4*>(lds + row * LDK + kq) = r[i];
        } else {
            constexpr int RQ = ROWS / 4;
            const int k = f / RQ;
            const int rq = (f % RQ) * 4;
#pragma unroll
            for (int e = 0; e < 4; ++e) lds[(rq + e) * LDK + k] = r[i][e];
        }
    }
}

__device__ __forceinline__ float epi_value(const GemmParams& p, float acc, long row, long col, const float* bias,
                                           const float* R, const float* aux, float* C2, const float* Cold) {
    float v = acc * p.alpha;
    if (p.epi & EPI_BIAS) v += bias[col];
    if (p.epi & EPI_ACCUM) v += Cold[row * p.ldc + col];
    if (p.epi & EPI_STORE_PRE) C2[row * p.ldc2 + col] = v;
    if (p.epi & EPI_GELU) v = gelu_f(v);
    if (p.epi & EPI_DGELU) v *= dgelu_f(aux[row * p.ldaux + col]);
    if (p.epi & EPI_RESID) v += R[row * p.ldr + col];
    return v;
}

template <int BM, int BN, int WM, int WN, bool TA, bool TB, bool CONV>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmParams p) {
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int RM = WTM / 32, RN = WTN / 32;
    static_assert(WM * WN == 4, "4 waves");
    static_assert(RM >= 1 && RN >= 1, "wave tile >= 32x32");
    __shared__ __attribute__((aligned(16))) float As[BM * LDK];
    __shared__ __attribute__((aligned(16))) float Bs[BN * LDK];

    int zz = blockIdx.z;
    int split = 0;
    if (p.splits > 1) {
        split = zz % p.splits;
        zz /= p.splits;
    }
    const int z1 = zz / p.zdiv, z0 = zz % p.zdiv;
    const float* A = p.A + z1 * p.sA1 + z0 * p.sA0;
    const float* B = p.B + z1 * p.sB1 + z0 * p.sB0;

    const int m0 = blockIdx.y * BM;
    const int n0 = blockIdx.x * BN;
    const int kbeg = split * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);

    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int h = lane >> 5, l32 = lane & 31;

    f32x16 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    f32x4 ra[Stage<BM>::LOADS];
    f32x4 rb[Stage<BN>::LOADS];
    const bool va = p.va != 0, vb = p.vb != 0;

    load_stage<BM, !TA, CONV>(ra, A, p.lda, m0, p.M, kbeg, kend, va, p.segK, p.pad, p.Mvalid);
    load_stage<BN, TB, false>(rb, B, p.ldb, n0, p.N, kbeg, kend, vb, 0, 0, 0);

    for (int k0 = kbeg; k0 < kend; k0 += BK) {
        __syncthreads();
        store_stage<BM, !TA>(As, ra);
        store_stage<BN, TB>(Bs, rb);
        __syncthreads();
        if (k0 + BK < kend) {
            load_stage<BM, !TA, CONV>(ra, A, p.lda, m0, p.M, k0 + BK, kend, va, p.segK, p.pad, p.Mvalid);
            load_stage<BN, TB, false>(rb, B, p.ldb, n0, p.N, k0 + BK, kend, vb, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            f32x4 af[RM], bf[RN];
#pragma unroll
            for (int i = 0; i < RM; ++i)
                af[i] = *reinterpret_cast<const f32x4*>(As + (wm * WTM + i * 32 + l32) * LDK + h * 8 + q * 4);
#pragma unroll
            for (int j = 0; j < RN; ++j)
                bf[j] = *reinterpret_cast<const f32x4*>(Bs + (wn * WTN + j * 32 + l32) * LDK + h * 8 + q * 4);
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < RM; ++i)
#pragma unroll
                    for (int j = 0; j < RN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][e], bf[j][e], acc[i][j], 0, 0, 0);
        }
    }

    // ---- epilogue ----
    if (p.splits > 1) {
        float* W = p.ws + ((long)blockIdx.z) * p.M * (long)p.N;
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int j = 0; j < RN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const int col = n0 + wn * WTN + j * 32 + l32;
                    if (row < p.M && col < p.N) W[(long)row * p.N + col] = acc[i][j][r];
                }
        return;
    }
    float* C = p.C + z1 * p.sC1 + z0 * p.sC0;
    const float* bias = p.bias ? p.bias + z1 * p.sBias1 + z0 * p.sBias0 : nullptr;
    const float* R = p.R ? p.R + z1 * p.sR1 + z0 * p.sR0 : nullptr;
    const float* aux = p.aux ? p.aux + z1 * p.sAux1 + z0 * p.sAux0 : nullptr;
    float* C2 = p.C2 ? p.C2 + z1 * p.sC21 + z0 * p.sC20 : nullptr;
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m0 + wm * WTM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const int col = n0 + wn * WTN + j * 32 + l32;
                if (row < p.M && col < p.N)
                    C[(long)row * p.ldc + col] = epi_value(p, acc[i][j][r], row, col, bias, R, aux, C2, C);
            }
}

// Sum split-K partials in split order (deterministic) and apply the epilogue.
__global__ __launch_bounds__(256) void gemm_splitk_reduce(GemmParams p) {
    const long MN = (long)p.M * p.N;
    const int zz = blockIdx.y;
    const int z1 = zz / p.zdiv, z0 = zz % p.zdiv;
    float* C = p.C + z1 * p.sC1 + z0 * p.sC0;
    const float* bias = p.bias ? p.bias + z1 * p.sBias1 + z0 * p.sBias0 : nullptr;
    const float* R = p.R ? p.R + z1 * p.sR1 + z0 * p.sR0 : nullptr;
    const float* aux = p.aux ? p.aux + z1 * p.sAux1 + z0 * p.sAux0 : nullptr;
    float* C2 = p.C2 ? p.C2 + z1 * p.sC21 + z0 * p.sC20 : nullptr;
    const float* W = p.ws + (long)zz * p.splits * MN;
    for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < MN; idx += (long)gridDim.x * blockDim.x) {
        float s = 0.f;
        for (int sp = 0; sp < p.splits; ++sp) s += W[sp * MN + idx];
        const long row = idx / p.N, col = idx % p.N;
        C[row * p.ldc + col] = epi_value(p, s, row, col, bias, R, aux, C2, C);
    }
}

template <int BM, int BN, int WM, int WN>
void launch_tile(const GemmParams& p, dim3 grid, hipStream_t st) {
    if (p.segK > 0) {
        hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, false, false, true>), grid, dim3(256), 0, st, p);
        return;
    }
    if (!p.ta && !p.tb)
        hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, false, false, false>), grid, dim3(256), 0, st, p);
    else if (!p.ta && p.tb)
        hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, false, true, false>), grid, dim3(256), 0, st, p);
    else if (p.ta && !p.tb)
        hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, true, false, false>), grid, dim3(256), 0, st, p);
    else
        hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, WM, WN, true, true, false>), grid, dim3(256), 0, st, p);
}

bool aligned16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

}  // namespace

void gemm_init(GemmParams& p) {
    p = GemmParams{};
    p.Z = 1;
    p.zdiv = 1;
    p.alpha = 1.f;
    p.splits = 1;
}

void gemm_launch(GemmParams p, hipStream_t st, float* ws, long ws_floats) {
    if (p.M <= 0 || p.N <= 0 || p.Z <= 0) return;
    // vector loads need 16-B aligned rows (and batch strides) along the contiguous axis
    auto vec_ok = [](const float* base, long ld, long s0, long s1) {
        return aligned16(base) && (ld % 4 == 0) && (s0 % 4 == 0) && (s1 % 4 == 0);
    };
    p.va = vec_ok(p.A, p.lda, p.sA0, p.sA1) && (p.segK == 0 || p.segK % 4 == 0);
    p.vb = vec_ok(p.B, p.ldb, p.sB0, p.sB1);

    int BM = p.M > 64 ? 128 : 64;
    int BN = p.N > 64 ? 128 : 64;
    // small grids: prefer 64-row tiles to raise the block count
    const long tiles128 = (long)((p.M + 127) / 128) * ((p.N + BN - 1) / BN) * p.Z;
    if (BM == 128 && tiles128 < 512) BM = 64;
    const int gx = (p.N + BN - 1) / BN, gy = (p.M + BM - 1) / BM;
    const long blocks = (long)gx * gy * p.Z;

    // split-K when the grid is too small to fill 256 CUs and K is long
    int splits = 1;
    if (ws && p.K >= 1024 && blocks < 256) {
        splits = (int)std::min<long>(16, (512 + blocks - 1) / blocks);
        while (splits > 1 && (long)splits * p.Z * p.M * (long)p.N > ws_floats) --splits;
        const int maxs = (p.K + 255) / 256;  // keep >= 256 K per split
        splits = std::min(splits, std::max(1, maxs));
    }
    p.splits = splits;
    p.kchunk = splits > 1 ? (((p.K + splits - 1) / splits + BK - 1) / BK) * BK : p.K;
    if (splits > 1) splits = (p.K + p.kchunk - 1) / p.kchunk;
    p.splits = splits;
    p.ws = ws;
    dim3 grid(gx, gy, p.Z * splits);
    if (BM == 128 && BN == 128) launch_tile<128, 128, 2, 2>(p, grid, st);
    else if (BM == 128 && BN == 64) launch_tile<128, 64, 2, 2>(p, grid, st);
    else if (BM == 64 && BN == 128) launch_tile<64, 128, 2, 2>(p, grid, st);
    else launch_tile<64, 64, 2, 2>(p, grid, st);
    if (splits > 1) {
        const long MN = (long)p.M * p.N;
        const int gxr = (int)std::min<long>(1024, (MN + 255) / 256);
        hipLaunchKernelGGL(gemm_splitk_reduce, dim3(gxr, p.Z), dim3(256), 0, st, p);
    }
}
