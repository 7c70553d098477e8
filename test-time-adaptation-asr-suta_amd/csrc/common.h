// Shared device helpers and kernel launcher declarations for libsuta (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#define SUTA_WAVE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float gelu_f(float x) {
    return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}
__device__ __forceinline__ float dgelu_f(float x) {
    // d/dx [x Phi(x)] = Phi(x) + x phi(x)
    const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752f));
    const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
    return cdf + x * pdf;
}

// Branch-free erf for the bf16-plane GEMM epilogues and the conv front-end (conv0_gn_kernel, every mode): erfc(z),
// z = |x|, as t exp(-z^2 + P(t)), t = 1 / (1 + z / 2), with the 9-term Chebyshev fit of Numerical Recipes 2nd ed.
// section 6.2 (fractional error < 1.2e-7 for every z >= 0: fp32-accurate).  ~18 VALU operations against ~40 for the
// two-range erff; SUTA_FAST_GELU=0 restores erff for A/B runs.  (The fp32 GEMM epilogues keep erff: a second GELU
// form in every fp32 GEMM instantiation grew libsuta.so by 11 MB.)
__device__ __forceinline__ float erfc_t(float z, float t, float ez2) {  // ez2 = exp(-z^2)
    float p = 0.17087277f;
    p = fmaf(p, t, -0.82215223f);
    p = fmaf(p, t, 1.48851587f);
    p = fmaf(p, t, -1.13520398f);
    p = fmaf(p, t, 0.27886807f);
    p = fmaf(p, t, -0.18628806f);
    p = fmaf(p, t, 0.09678418f);
    p = fmaf(p, t, 0.37409196f);
    p = fmaf(p, t, 1.00002368f);
    p = fmaf(p, t, -1.26551223f);
    return t * ez2 * __expf(p);
}
__device__ __forceinline__ float gelu_fast(float x) {
    const float z = fabsf(x) * 0.70710678118654752f;
    const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
    const float erfc = erfc_t(z, t, __expf(-z * z));
    // x Phi(x) = x (1 + erf(x / sqrt 2)) / 2, erf = sign(x) (1 - erfc)
    return 0.5f * x * (x >= 0.f ? 2.0f - erfc : erfc);
}
__device__ __forceinline__ float dgelu_fast(float x) {
    const float z = fabsf(x) * 0.70710678118654752f;
    const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, z, 1.0f));
    const float e = __expf(-z * z);  // exp(-x^2 / 2): the normal density's exponential too
    const float erfc = erfc_t(z, t, e);
    const float cdf = 0.5f * (x >= 0.f ? 2.0f - erfc : erfc);
    return cdf + x * (0.39894228040143268f * e);
}

// A/B switches read from the environment (SUTA_* = 0 selects the path a round replaced).  They decide which
// buffers a forward writes in which format (fp32 or a bf16 plane) and which the backward reads, so one snapshot is
// taken per engine call (suta_latch_switches, at the start of suta_forward / suta_step / suta_adapt*) and every
// launcher and engine predicate of that call reads the snapshot: a switch flipped between a forward and its
// backward, or between graph capture and replay, cannot mismatch formats.  The snapshot is part of the engine's
// graph key.  Launchers used without an engine (tools/) take a snapshot on first use.  The snapshot is per host
// thread: an engine call latches and launches on its calling thread, so engines driven from different threads (one
// per device in one process) never see each other's snapshot.
struct SutaSwitches {
    int latched;
    int fast_gelu;        // SUTA_FAST_GELU: branch-free GELU / GELU' (front-end and bf16-plane epilogues)
    int flash_fwd_plane;  // SUTA_FLASH_FWD_PLANE: flash forward on the bf16 qkv plane
    int flash_bwd_plane;  // SUTA_FLASH_BWD_PLANE: flash backward on the bf16 qkv / dctx planes
    int flash_bf16_img;   // SUTA_FLASH_BF16_IMG: bf16 LDS images in the fp32-row bf16 flash kernels
    int conv_planes;      // SUTA_CONV_PLANES
    int pre_bf16;         // SUTA_PRE_BF16
    int conv_z_bf16;      // SUTA_CONV_Z_BF16
    int dy_planes;        // SUTA_DY_PLANES
    int conv_dx_planes;   // SUTA_CONV_DX_PLANES
    int fused_conv_ln;    // SUTA_FUSED_CONV_LN
    int flash_fwd_nw;     // SUTA_FLASH_FWD_NW (default 4): waves per block of the bf16-plane flash forward
    int hbx;              // SUTA_HBX (default 1): the 256 x 256 slice-ring bf16-plane GEMM for plain-epilogue linears
                          // on full grids; 2: on every eligible bf16-plane linear (tests: small grids, edge tiles)
    int splitk;           // SUTA_SPLITK (default 1): split-K for small grids; 0 = never (tests comparing kernels
                          // bitwise: a split changes the k summation order)
    int hbx_form;         // SUTA_HBX_FORM (default 4): the 256 x 256 kernel's main loop with the C^T staged epilogue
                          // (SUTA_HBX_T=2) and K % 64 == 0: 2 four-phase 64-deep K-tiles with two wave groups one
                          // barrier apart + s_setprio (gemm_hbp_kernel), 1 the same in lockstep, 0 the 32-deep slice
                          // ring, 3 form 2 with three half-tiles in flight, 4 form 3 on 16x16x32 MFMAs
    int ln_rpw;           // SUTA_LN_RPW (default 2): rows per wave of the bf16-input (conv stack) LayerNorm forward; 1 = one
    int hbx_dbg;          // SUTA_HBX_DBG (tools/hb_bench diagnostics; wrong results): gemm_hbx with parts of its loop removed;
                          // honoured only by the tools build of gemm_hbx.hip (-DSUTA_HBX_DIAG), ignored by libsuta.so
    int fused_delta;      // SUTA_FUSED_DELTA (default 1): the flash backward's delta in the dctx GEMM's epilogue
    int hbx_t;            // SUTA_HBX_T (default 2): gemm_hbx accumulates C^T fragments with a row-per-lane epilogue whose
                          // outputs are staged through LDS into whole-line stores; 1 = direct 16-B row-per-lane stores,
                          // 0 = the column-per-lane form shared with the 128 x 128 kernel
    int hbp_conv;         // SUTA_HBP_CONV (default 1): the conv stack's conv-seg input gradients on the four-phase 256 x 256
                          // kernel (gemm.hip use_hbp_conv); 0 = the 128 x 128 kernel
    int hbt4;             // SUTA_HBT4 (default 1): the conv weight gradients (MN-contiguous bf16 planes) on the four-phase
                          // 256 x 256 kernel's TN form (gemm_hbp_kernel) on grids of >= 256 tiles; 2 on every grid
                          // (tests); 0 = gemm_hbt_kernel (128 x 128, two stages, split-K on small grids)
    int epi_fast;         // SUTA_EPI_FAST (default 1): 32-bit-offset GEMM epilogue where every operand fits 4 GiB (p.off32);
                          // 0 = the general epilogue everywhere
};
void suta_latch_switches();
// hipFuncSetAttribute(fn, MaxDynamicSharedMemorySize, bytes) once per kernel, thread-safe (ops.hip)
void set_max_lds_once(const void* fn, size_t bytes, const char* name);
const SutaSwitches& suta_switches();  // the snapshot (taken now if none was)

// GELU / GELU' of the bf16-plane GEMM epilogues (config C4: the result is rounded to a bf16 plane), two elements per
// call on packed fp32 arithmetic (v_pk_mul_f32 / v_pk_fma_f32: half the VALU instructions of two scalar calls).
// erf by Abramowitz & Stegun 7.1.28, erf(z) = 1 - (1 + a1 z + ... + a6 z^6)^-16 for z >= 0, |error| <= 3e-7 (the
// bf16 output's own rounding step is 4e-3 relative): Phi(x) = 0.5 q for x < 0 and 1 - 0.5 q for x >= 0, q = p^-16
// evaluated without cancellation.  About 9 VALU operations per element against ~22 for gelu_fast.
typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2v phi_as2(f32x2v x, f32x2v& q) {
    const f32x2v z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
    f32x2v p = z * 0.0000430638f + 0.0002765672f;
    p = p * z + 0.0001520143f;
    p = p * z + 0.0092705272f;
    p = p * z + 0.0422820123f;
    p = p * z + 0.0705230784f;
    p = p * z + 1.0f;
    p = p * p;
    p = p * p;
    p = p * p;
    p = p * p;
    q = f32x2v{__builtin_amdgcn_rcpf(p.x), __builtin_amdgcn_rcpf(p.y)};
    const f32x2v h = 0.5f * q;
    return f32x2v{x.x >= 0.f ? 1.0f - h.x : h.x, x.y >= 0.f ? 1.0f - h.y : h.y};
}
__device__ __forceinline__ f32x2v gelu2_bf16ep(f32x2v x) {
    f32x2v q;
    return x * phi_as2(x, q);
}
__device__ __forceinline__ f32x2v dgelu2_bf16ep(f32x2v x) {
    f32x2v q;
    const f32x2v cdf = phi_as2(x, q);
    const f32x2v a = x * x * (-0.5f * 1.4426950408889634f);  // log2 of exp(-x^2 / 2)
    const f32x2v e = f32x2v{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
    return cdf + (x * 0.39894228040143268f) * e;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// ------------------------------------------------------------------------------------------
// GEMM:  C[z](m,n) = epi( sum_k A[z](m,k) * B[z](k,n) )         (fp32 in, fp32 MFMA accumulate)
//   A(m,k) = A[m*lda + k]   (ta = 0)   or A[k*lda + m]   (ta = 1)
//   conv A mode (ta = 0, segK > 0): k = seg*segK + r, A(m,k) = A[(m + seg - pad)*lda + r],
//        zero unless 0 <= m + seg - pad < Mvalid   (implicit grouped/positional conv, conv dX)
//   segmented B (segB, tb = 1): B(k,n) = B[n*ldb + seg*sBseg + r]   (per-tap weight slices)
//   B(k,n) = B[k*ldb + n]   (tb = 0)   or B[n*ldb + k]   (tb = 1)
//   batch z in [0, Z): pointer += (z / zdiv) * s?1 + (z % zdiv) * s?0
// epilogue flags, applied in this order:  v = alpha*acc; +bias[n]; +C(acc) ; C2 = v (store pre);
//   GELU; *gelu'(aux(m,n)); +R(m,n); C = v
// ------------------------------------------------------------------------------------------
enum {
    EPI_BIAS = 1,
    EPI_GELU = 2,
    EPI_RESID = 4,
    EPI_STORE_PRE = 8,
    EPI_DGELU = 16,
    EPI_ACCUM = 32,
    EPI_SMBWD = 64,  // softmax backward: v = alpha * aux(m,n) * (acc - rowv[m])  (dS from dP, P, delta)
    EPI_ROWMASK = 128,  // ragged batch: rows >= zrows[z / zdiv] are stored as 0
    EPI_DELTA = 256,    // flash-backward row term from the dctx GEMM (gemm_hbx C^T epilogue only): see GemmParams.dlt_o
};

struct GemmParams {
    const float* A;
    const float* B;
    float* C;
    int M, N, K;
    long lda, ldb, ldc;
    int Z, zdiv;
    long sA0, sA1, sB0, sB1, sC0, sC1;
    int ta, tb;
    int segK, pad, Mvalid;  // conv-A mode when segK > 0
    int segB;               // with segK > 0 and tb: B(k, n) = B[n*ldb + (k/segK)*sBseg + k%segK]
    long sBseg;
    const float* bias;
    long sBias0, sBias1;
    const float* R;
    long ldr, sR0, sR1;
    const float* aux;
    long ldaux, sAux0, sAux1;
    float* C2;
    long ldc2, sC20, sC21;
    const float* rowv;  // per-row vector (EPI_SMBWD), batch strides as the others
    long sRow0, sRow1;
    // ragged batch (per utterance z1 = z / zdiv): valid output rows (EPI_ROWMASK) and the conv-A
    // Mvalid (rows outside [0, zmvalid[z1]) read as zero); null = uniform
    const int* zrows;
    const int* zmvalid;
    float alpha;
    int epi;
    // internal
    int splits, kchunk;
    float* ws;  // split-K workspace
    int va, vb; // vector (16 B) loads legal
    int mode;   // 0 exact fp32 MFMA, 1 x6 (fp32-accurate bf16 split), 2 bf16 products; gemm_init takes the default
    int order;  // LDS-DMA kernel tile order within an XCD's range: 0 n fastest (A panel reuse), 1 m fastest (B band reuse)
    // bf16 mode with bf16 operand planes (Z == 1, both k-contiguous): A(m,k) = Ab[m*ldab + k],
    // B(k,n) = Bb[n*ldbb + k] (16-B aligned, ldab % 8 == ldbb % 8 == K % 8 == 0) -> gemm_hb_kernel
    const void* Ab;
    const void* Bb;
    long ldab, ldbb;
    void* Cb;   // optional bf16 copy of the stored C: the A plane of the next bf16-plane GEMM
    long ldcb;
    long sCb1;  // Cb's stride per z1 (bf16 elements; Z-batched conv-stack planes)
    int off32;  // internal: every epilogue operand (rows x ld) within 4 GiB -> 32-bit offset epilogue
    // bf16-plane GEMMs (Cb given, gemm_hb_kernel, no split-K): C2 (EPI_STORE_PRE) and aux (EPI_DGELU) hold bf16
    // elements (ld and batch strides in elements; ldc2 even) -- the FFN pre-activation u of config C4
    int preb;
    // internal: bf16-plane epilogues (Cb given) evaluate GELU / GELU' with gelu_fast / dgelu_fast (SUTA_FAST_GELU=0:
    // erff, for A/B runs)
    int fgelu;
    // EPI_DELTA: delta[(b * dNH + head) * dT + t] = sum_d C(row, 64 head + d) * O(row, 64 head + d), row = b * dT + t,
    // O = dlt_o (fp32 [M][ldo], the attention forward's ctx), C = the epilogue's final value (dctx): the softmax
    // backward's row term, summed in the order of ops.hip attn_delta_kernel (bitwise the same delta)
    const float* dlt_o;
    long ldo;
    float* delta;
    int dT, dNH;
};

void gemm_init(GemmParams& p);
// whether gemm_launch(p) takes the 256 x 256 bf16-plane kernel with its C^T epilogue (the one that carries EPI_DELTA);
// p as it will be launched (planes routed)
bool gemm_hbx_t_selected(const GemmParams& p);
// Launch; ws/ws_floats: scratch for split-K (may be null -> no split).
void gemm_launch(GemmParams p, hipStream_t st, float* ws, long ws_floats);
// Benchmark/test override: tile (-1 auto, 0 128x128, 1 128x64, 2 64x128, 3 64x64), LDS buffers (1|2).
void gemm_set_variant(int tile, int nbuf);
// 0 = exact fp32 MFMA (v_mfma_f32_32x32x2_f32); 1 = fp32-accurate 3-way bf16 split (6 bf16 MFMA products);
// 2 = bf16 GEMM (operands rounded to bf16 once, one bf16 MFMA product, fp32 accumulate).
void gemm_set_mode(int mode);
// dst[r][0:K] = bf16(src[r * lds + 0:K]) (RNE) for r < rows; K % 8 == 0, src/lds 16-B aligned, dst 16-B aligned
// with row stride K: the A plane of a bf16-plane GEMM.
// the 128 x 128 bf16-plane GEMM specialised on its epilogue class (false: no class covers p.epi)
bool gemm_run_hb_class(const GemmParams& p, dim3 grid, hipStream_t st);
void launch_to_bf16(const float* src, long lds, long rows, int K, void* dst, hipStream_t st);
// dst[z][n][k] = bf16(src[z * zs + k * N + n]) (per-slot transposed bf16 weights)
void launch_transpose_bf16(const float* src, long zs, int Z, int K, int N, void* dst, hipStream_t st,
                          void* dstn = nullptr);
int gemm_get_mode();
// launch census per (kernel, tile, Z, splits, operand form): suta_set_census / suta_get_census
void gemm_census_enable(bool on);
std::string gemm_census_text();
bool gemm_census_is_on();
void gemm_census_time(const std::string& shape, double ms);
