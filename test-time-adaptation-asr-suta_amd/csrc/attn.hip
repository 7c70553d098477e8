// Flash-style fused attention for head dim 64 and any T (reference: the HF Wav2Vec2Attention the
// SUTA loop runs, modeling_wav2vec2.py Wav2Vec2Attention.forward: softmax(q k^T * d^-1/2) v, and its
// autograd backward).  No T x T matrix is stored: the forward keeps the per-row log-sum-exp, the
// backward recomputes the probabilities from it.
//
//   flash_fwd_kernel  block = NW waves of one (utterance, head); wave = 32 queries.  Key tiles of 32
//                     stream through LDS (double-buffered, one barrier per tile): K row-major, V
//                     transposed.  S^T = K Q^T (key in the accumulator rows, query on the lane), online
//                     softmax in registers, O^T += V^T P^T with the lane's own probabilities as the B
//                     operand (no LDS round trip for P); the rescale is lane-local because the query
//                     is the lane.  Writes ctx and LSE[q] = max + log(sum).
//   flash_bwd_kernel  block = NW waves = a block of key groups of one (utterance, head); wave = 32
//                     keys whose K and V rows stay in registers.  Query tiles of 32 stream through
//                     LDS (Q, dO, LSE, delta; double-buffered).  S = Q K^T and dP = dO V^T (key on the
//                     lane), P = exp(scale S - LSE), dS = scale P (dP - delta); dV^T += dO^T P and
//                     dK^T += Q^T dS accumulate in registers over all query tiles (written once, no
//                     cross-block sum).  dS crosses LDS once: the block's dQ partial over its keys,
//                     dQ_kb = dS K, is written to scratch per key block.
//   flash_dq_reduce   dQ = sum over key blocks in fixed order -> dqkv's Q columns (bitwise
//                     deterministic: no float atomics).
//
// Contractions: exact fp32 v_mfma_f32_32x32x2_f32 (and 16x16x4 for dQ), or in bf16 mode (config C4)
// the operands rounded to bf16 (RNE) on v_mfma_f32_32x32x16_bf16 / 16x16x32 with fp32 accumulation;
// softmax, LSE, delta and every stored value are fp32.
// Ragged batches: keys >= the utterance's length get probability 0; query tiles past it are skipped in
// the backward (their dO rows are exactly 0, so they contribute nothing).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

#include "common.h"
#include "ops.h"

namespace {

typedef __bf16 fbf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 fbf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// [row][64] tiles padded to 68 floats (17 16-B slots): the row reads of prod_rows (ds_read_b128, lane l32 -> row
// l32) put row r in slot r mod 16, so each of gfx950's four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}
// and the upper half's) reads 16 distinct 4-bank slots (72 = 18 slots put rows r and r + 8 on one slot: 2-way
// conflicts); the column reads of apply_rows stay conflict-free (32 consecutive floats per 32-lane group)
constexpr int FA_LD = 68;
constexpr int FA_LDT = 36;  // [64][32] transposed tiles

__device__ __forceinline__ fbf16x8 cvt8(f32x4 lo, f32x4 hi) {
    fbf16x8 v;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[j] = (__bf16)lo[j];
        v[4 + j] = (__bf16)hi[j];
    }
    return v;
}

// accumulator register v of a 32x32 MFMA tile holds row r8(v, h) of column (lane & 31)
__device__ __forceinline__ int r8(int v, int h) { return 8 * (v >> 2) + 4 * h + (v & 3); }

// 1-D XCD-aware renumbering (cdna_hip_programming.md T1, bijective): consecutive logical blocks (the
// query or key blocks of one head) run on one XCD and share its L2.
__device__ __forceinline__ int xcd_block() {
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// The lane's 64-wide register row (the B operand of prod_rows): fp32 X[row][32h + 4m + e], m < 8;
// bf16 X[row][16s + 8h + j], s < 4.
template <bool BF16>
struct RowReg;
template <>
struct RowReg<false> {
    f32x4 v[8];
    __device__ __forceinline__ void load(const float* __restrict__ row, int h) {
#pragma unroll
        for (int m = 0; m < 8; ++m) v[m] = *reinterpret_cast<const f32x4*>(row + 32 * h + 4 * m);
    }
};
template <>
struct RowReg<true> {
    fbf16x8 v[4];
    __device__ __forceinline__ void load(const float* __restrict__ row, int h) {
#pragma unroll
        for (int s = 0; s < 4; ++s)
            v[s] = cvt8(*reinterpret_cast<const f32x4*>(row + 16 * s + 8 * h),
                        *reinterpret_cast<const f32x4*>(row + 16 * s + 8 * h + 4));
    }
};

// acc[r8(v,h)][l32] += sum_d L[r8-row i = l32 of the A operand][d] * X[l32][d]:
//   C[i][j] = sum_d L[i][d] X[j][d], L = 32 LDS rows of stride FA_LD (row i read by lane i), X the
//   lane's register row.  Output: row i in the accumulator registers, column j on the lane.
template <bool BF16>
__device__ __forceinline__ void prod_rows(f32x16& acc, const float* __restrict__ L, const RowReg<BF16>& x, int l32,
                                          int h) {
    const float* lr = L + l32 * FA_LD;
    if constexpr (!BF16) {
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const f32x4 a = *reinterpret_cast<const f32x4*>(lr + 32 * h + 4 * m);
#pragma unroll
            for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[e], x.v[m][e], acc, 0, 0, 0);
        }
    } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const fbf16x8 a = cvt8(*reinterpret_cast<const f32x4*>(lr + 16 * s + 8 * h),
                                   *reinterpret_cast<const f32x4*>(lr + 16 * s + 8 * h + 4));
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, x.v[s], acc, 0, 0, 0);
        }
    }
}

// o[t][n = 32t + r8(v,h)][l32] += sum_r L[r][32t + n'] pv_r, the contraction index r being the
// accumulator row of pv (pv[v] holds row r8(v,h) of column l32): A operand = L rows read by column
// (L row-major [r][FA_LD], one float per lane), B operand = the lane's own pv registers.
template <bool BF16>
__device__ __forceinline__ void apply_rows(f32x16 (&o)[2], const float* __restrict__ L, const f32x16& pv, int l32,
                                           int h) {
    if constexpr (!BF16) {
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const float* lr = L + r8(v, h) * FA_LD + l32;
            const float a0 = lr[0], a1 = lr[32];
            o[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, pv[v], o[0], 0, 0, 0);
            o[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, pv[v], o[1], 0, 0, 0);
        }
    } else {
        // MFMA c takes k-slot 8h + j <-> accumulator register v = 8c + j (row r8(8c + j, h))
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            fbf16x8 b;
#pragma unroll
            for (int j = 0; j < 8; ++j) b[j] = (__bf16)pv[8 * c + j];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                fbf16x8 a;
#pragma unroll
                for (int j = 0; j < 8; ++j) a[j] = (__bf16)L[r8(8 * c + j, h) * FA_LD + 32 * t + l32];
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, o[t], 0, 0, 0);
            }
        }
    }
}

// Same contraction with L stored transposed (Lt[n][LDT], n the output row; contraction rows from
// column c0): 16-B reads of four consecutive contraction rows r8(4a + 0..3, h) = 8a + 4h + 0..3.
template <bool BF16, int LDT>
__device__ __forceinline__ void apply_cols(f32x16 (&o)[2], const float* __restrict__ Lt, const f32x16& pv, int l32,
                                           int h) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const float* lr = Lt + (32 * t + l32) * LDT + 4 * h;
        if constexpr (!BF16) {
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const f32x4 x = *reinterpret_cast<const f32x4*>(lr + 8 * a);
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    o[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(x[b], pv[4 * a + b], o[t], 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                fbf16x8 b;
#pragma unroll
                for (int j = 0; j < 8; ++j) b[j] = (__bf16)pv[8 * c + j];
                const fbf16x8 a = cvt8(*reinterpret_cast<const f32x4*>(lr + 16 * c),
                                       *reinterpret_cast<const f32x4*>(lr + 16 * c + 8));
                o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, o[t], 0, 0, 0);
            }
        }
    }
}

// max / sum with the other half-wave's value (lane l and l ^ 32) through v_permlane32_swap (no LDS round trip, as
// __shfl_xor's ds_bpermute is): swapping two copies of x leaves {x[l], x[l + 32]} in the lower half's pair and
// {x[l - 32], x[l]} in the upper's, so one op of the pair is op(x[l], x[l ^ 32]) -- bitwise the shuffle form (fmax
// and a two-term sum are commutative)
__device__ __forceinline__ float half_swap_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float half_swap_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

constexpr float LOG2E = 1.4426950408889634f;

// ------------------------------------------------------------------------------------------------
// forward: key tiles of FK = 64 (two 32-key sub-tiles: two independent S^T chains, one softmax
// update, one O rescale and one barrier per 64 keys).  Probabilities via v_exp_f32 on log2-domain
// scores (scale * log2 e folded into one multiply).
// ------------------------------------------------------------------------------------------------
constexpr int FK = 64;
constexpr int FK_LDT = FK + 4;  // transposed V tile row stride
constexpr int FF_NW_BF = 4;     // waves per block of the bf16 forward

// An utterance with no valid key (tl <= 0) has no softmax: its rows get ctx = 0 and LSE = -inf, and the kernel
// returns before any LDS image is filled (the peeled last tile would otherwise run tile -1 on stale LDS).  The host
// rejects zero-frame utterances (engine set_lengths: "utterance too short"), so this is a guard, not a path.
__device__ __forceinline__ void flash_fwd_no_keys(float* ctx, __bf16* ctxb, float* lse, long row0, long bhT, int T,
                                                  int H, int hd, int q0, int l32, int h) {
    const int q = q0 + l32;
    if (q0 >= T || q >= T) return;
    float* cr = ctx + (row0 + q) * H + hd * 64 + 32 * h;
#pragma unroll
    for (int c = 0; c < 32; ++c) cr[c] = 0.f;
    if (ctxb) {
        __bf16* br = ctxb + (row0 + q) * H + hd * 64 + 32 * h;
#pragma unroll
        for (int c = 0; c < 32; ++c) br[c] = (__bf16)0.f;
    }
    if (h == 0) lse[bhT + q] = -INFINITY;
}

template <int NW, bool BF16>
__global__ __launch_bounds__(NW * 64) void flash_fwd_kernel(const float* __restrict__ qkv, float* __restrict__ ctx,
                                                            float* __restrict__ lse, int T, int NH, int H, float scale,
                                                            const int* __restrict__ tlen, int nqb,
                                                            __bf16* __restrict__ ctxb) {
    constexpr int NT = NW * 64;
    constexpr int ITEMS = FK * 16, NPT = (ITEMS + NT - 1) / NT;  // float4 of a FK x 64 tile per thread
    __shared__ __attribute__((aligned(16))) float Ks[2][FK * FA_LD];
    __shared__ __attribute__((aligned(16))) float Vt[2][64 * FK_LDT];
    const int id = xcd_block();
    const int qb = id % nqb, bh = id / nqb, hd = bh % NH, u = bh / NH;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
    const int tl = tlen ? tlen[u] : T;
    const long ld = 3L * H;
    const float* Qb = qkv + (long)u * T * ld + hd * 64;
    const float* Kb = Qb + H;
    const float* Vb = Qb + 2 * H;
    const int q0 = (qb * NW + w) * 32;
    if (tl <= 0) {  // (block-uniform: one utterance per block)
        flash_fwd_no_keys(ctx, ctxb, lse, (long)u * T, (long)bh * T, T, H, hd, q0, l32, h);
        return;
    }
    const bool active = q0 < T;
    const float sl2 = scale * LOG2E;
    RowReg<BF16> qv;
    qv.load(Qb + (long)min(q0 + l32, T - 1) * ld, h);

    // K: 16 lanes per row (coalesced, row-major image).  V: a wave-instruction covers 16 keys x 4 column
    // chunks, so the transposed 4-byte writes (c4 + e) * FK_LDT + key hit 64 distinct banks
    // (FK_LDT = 68 = 4 mod 64) -- the row-per-16-lanes map was a 4-way conflict on every V write
    auto vmap = [](int it, int& key, int& c4) {
        const int l = it & 63, wi = it >> 6;
        key = (l & 15) + 16 * (wi & 3);
        c4 = 4 * ((l >> 4) + 4 * (wi >> 2));
    };
    f32x4 kr[NPT], vr[NPT];
    auto fetch = [&](int kt) {
#pragma unroll
        for (int n = 0; n < NPT; ++n) {
            const int it = threadIdx.x + n * NT, row = it >> 4, c4 = (it & 15) * 4, key = kt * FK + row;
            int vk, vc;
            vmap(it, vk, vc);
            kr[n] = vr[n] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (it < ITEMS && key < T) kr[n] = *reinterpret_cast<const f32x4*>(Kb + (long)key * ld + c4);
            if (it < ITEMS && kt * FK + vk < T) vr[n] = *reinterpret_cast<const f32x4*>(Vb + (long)(kt * FK + vk) * ld + vc);
        }
    };
    auto put = [&](int buf) {
#pragma unroll
        for (int n = 0; n < NPT; ++n) {
            const int it = threadIdx.x + n * NT, row = it >> 4, c4 = (it & 15) * 4;
            int vk, vc;
            vmap(it, vk, vc);
            if (it < ITEMS) {
                *reinterpret_cast<f32x4*>(&Ks[buf][row * FA_LD + c4]) = kr[n];
#pragma unroll
                for (int e = 0; e < 4; ++e) Vt[buf][(vc + e) * FK_LDT + vk] = vr[n][e];
            }
        }
    };

    const int nkt = (tl + FK - 1) / FK;  // key tiles holding a valid key (later ones have probability 0)
    f32x16 o[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) o[t][v] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;  // log2-domain running maximum; this lane's half of the sum
    fetch(0);
    put(0);
    __syncthreads();
    // full tiles (every key valid, both 32-key halves) run a body without masks or branches; the utterance's
    // last tile, with the masks and the skipped empty half, is peeled (same arithmetic per element: bitwise the
    // single-body loop)
    auto tile = [&](int kt, auto last_tag) {
        constexpr bool LAST = decltype(last_tag)::value;
        const int buf = kt & 1;
        if (!LAST) fetch(kt + 1);
        if (active) {
            // the second 32-key half of a tile holding no valid key (the tail of the last tile) is skipped:
            // its probabilities are exactly 0
            const bool two = !LAST || kt * FK + 32 < tl;
            f32x16 s[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int v = 0; v < 16; ++v) s[j][v] = 0.f;
                if (j == 0 || two) prod_rows<BF16>(s[j], Ks[buf] + 32 * j * FA_LD, qv, l32, h);  // S^T: key r8(v,h), query l32
            }
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const bool ok = !LAST || kt * FK + 32 * j + r8(v, h) < tl;
                    s[j][v] = ok ? sl2 * s[j][v] : -INFINITY;
                    mx = fmaxf(mx, s[j][v]);
                }
            mx = half_swap_max(mx);
            const float m_new = fmaxf(m_run, mx);
            float ls = 0.f;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    s[j][v] = __builtin_amdgcn_exp2f(s[j][v] - m_new);
                    ls += s[j][v];
                }
            if (m_new != m_run) {  // rescale only when the maximum moved (exact: alpha = 1 otherwise)
                const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);  // 0 on the first tile
                l_run *= alpha;
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int v = 0; v < 16; ++v) o[t][v] *= alpha;
                m_run = m_new;
            }
            l_run += ls;
            apply_cols<BF16, FK_LDT>(o, Vt[buf], s[0], l32, h);  // O^T[n][q] += sum_key V[key][n] P[q][key]
            if (two) apply_cols<BF16, FK_LDT>(o, Vt[buf] + 32, s[1], l32, h);
        }
        if (!LAST) put(buf ^ 1);
        __syncthreads();
    };
    for (int kt = 0; kt + 1 < nkt; ++kt) tile(kt, std::false_type{});
    tile(nkt - 1, std::true_type{});
    if (!active) return;
    const float l_tot = half_swap_sum(l_run);
    const int q = q0 + l32;
    if (q >= T) return;
    const float inv = 1.0f / l_tot;
    float* cr = ctx + ((long)u * T + q) * H + hd * 64 + 4 * h;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            f32x4 r;
#pragma unroll
            for (int b = 0; b < 4; ++b) r[b] = o[t][4 * a + b] * inv;
            *reinterpret_cast<f32x4*>(cr + 32 * t + 8 * a) = r;
            if (ctxb) {  // bf16 plane of the out-projection's A operand
                fbf16x4 b;
#pragma unroll
                for (int e = 0; e < 4; ++e) b[e] = (__bf16)r[e];
                *reinterpret_cast<fbf16x4*>(ctxb + ((long)u * T + q) * H + hd * 64 + 4 * h + 32 * t + 8 * a) = b;
            }
        }
    if (h == 0) lse[(long)bh * T + q] = (m_run + log2f(l_tot)) * (1.0f / LOG2E);  // natural-log LSE
}


// ------------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------------
// NW waves per block = NW key groups of 32.  Query tiles are double-buffered: the next tile's Q / dO /
// LSE / delta are loaded into registers while the current tile computes and written to the other LDS
// image after the dQ product (two barriers per tile).  LDS: K^T [64][32 NW + 4] + dS [32][32 NW + 4]
// + 2 x (Q, dO [32][72]): NW = 8 -> 136 KB, NW = 4 -> 86 KB.  (A single-buffered form staged right after
// the dS barrier measured equal in fp32 but spilled 132 B in the bf16 instantiation: 1.6x slower.)
template <int NW>
constexpr int fb_kbp() { return NW * 32 + 4; }
template <int NW>
constexpr size_t fb_lds_bytes() { return sizeof(float) * ((size_t)(64 + 32) * fb_kbp<NW>() + 4 * 32 * FA_LD + 128); }

template <int NW, bool BF16>
__global__ __launch_bounds__(NW * 64, NW == 4 ? 2 : 1) void flash_bwd_kernel(
    const float* __restrict__ qkv, const float* __restrict__ dctx, const float* __restrict__ lse,
    const float* __restrict__ delta, float* __restrict__ dqkv, float* __restrict__ dqp, int T, int NH, int H,
    float scale, const int* __restrict__ tlen, int nkb, int gpb, int B, __bf16* __restrict__ dqkvb) {
    constexpr int NT = NW * 64;
    constexpr int KBP = fb_kbp<NW>();
    constexpr int QPT = 512 / NT;       // float4 of a 32 x 64 tile per thread
    constexpr int SUB = 8 / NW;         // 16 x 16 dQ subtiles per wave
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* Kt = smem;                   // [64][KBP]: K of the block's keys, transposed
    float* Ss = Kt + 64 * KBP;          // [32][KBP]: dS of the current query tile
    float* Qs = Ss + 32 * KBP;          // [2][32][FA_LD]
    float* Ds = Qs + 2 * 32 * FA_LD;    // [2][32][FA_LD]  (dO = dctx rows)
    float* Ls = Ds + 2 * 32 * FA_LD;    // [2][32] LSE
    float* Dl = Ls + 64;                // [2][32] delta
    const int id = xcd_block();
    const int kb = id % nkb, bh = id / nkb, hd = bh % NH, u = bh / NH;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
    const int tl = tlen ? tlen[u] : T;
    const int ng = (T + 31) >> 5;
    const int g0 = kb * gpb, ngb = min(gpb, ng - g0);  // key groups of this block
    const int kbase = g0 * 32;
    const long ld = 3L * H;
    const float* Qb = qkv + (long)u * T * ld + hd * 64;
    const float* Kb = Qb + H;
    const float* Vb = Qb + 2 * H;
    const float* Ob = dctx + (long)u * T * H + hd * 64;
    const float* lb = lse + (long)bh * T;
    const float* db = delta + (long)bh * T;
    const bool active = w < ngb && kbase + 32 * w < tl;
    const int key = kbase + 32 * w + l32;
    const float sl2 = scale * LOG2E;
    RowReg<BF16> kv, vv;
    kv.load(Kb + (long)min(key, T - 1) * ld, h);
    vv.load(Vb + (long)min(key, T - 1) * ld, h);

    // the block's keys transposed into LDS (zero past T) for the dQ product
    for (int it = threadIdx.x; it < ngb * 32 * 16; it += NT) {
        const int row = it >> 4, c4 = (it & 15) * 4, k = kbase + row;
        f32x4 x = {0.f, 0.f, 0.f, 0.f};
        if (k < T) x = *reinterpret_cast<const f32x4*>(Kb + (long)k * ld + c4);
#pragma unroll
        for (int e = 0; e < 4; ++e) Kt[(c4 + e) * KBP + row] = x[e];
    }
    // query tiles: Q and dO rows, LSE and delta, in two register stages (loads of tile qt+2 issued at the start of
    // tile qt, written to LDS at the end of tile qt+1: two tiles of compute cover a load's latency)
    struct Stg {
        f32x4 qr[QPT], orr[QPT];
        float lr;
    };
    auto fetch = [&](int qt, Stg& sg) {
#pragma unroll
        for (int n = 0; n < QPT; ++n) {
            const int it = threadIdx.x + n * NT, row = it >> 4, c4 = (it & 15) * 4, q = qt * 32 + row;
            sg.qr[n] = sg.orr[n] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (q < T) {
                sg.qr[n] = *reinterpret_cast<const f32x4*>(Qb + (long)q * ld + c4);
                sg.orr[n] = *reinterpret_cast<const f32x4*>(Ob + (long)q * H + c4);
            }
        }
        sg.lr = 0.f;
        const int qq = qt * 32 + (threadIdx.x & 31);
        if (threadIdx.x < 64 && qq < T) sg.lr = threadIdx.x < 32 ? lb[qq] : db[qq];
    };
    auto put = [&](int buf, const Stg& sg) {
#pragma unroll
        for (int n = 0; n < QPT; ++n) {
            const int it = threadIdx.x + n * NT, row = it >> 4, c4 = (it & 15) * 4;
            *reinterpret_cast<f32x4*>(Qs + (buf * 32 + row) * FA_LD + c4) = sg.qr[n];
            *reinterpret_cast<f32x4*>(Ds + (buf * 32 + row) * FA_LD + c4) = sg.orr[n];
        }
        if (threadIdx.x < 32) Ls[buf * 32 + threadIdx.x] = sg.lr;
        else if (threadIdx.x < 64) Dl[buf * 32 + threadIdx.x - 32] = sg.lr;
    };

    f32x16 dv[2], dk[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) dv[t][v] = dk[t][v] = 0.f;
    const int g = lane >> 4, l16 = lane & 15;
    const int kq = ngb * 32;  // contraction length of the dQ product
    const int NQT = (T + 31) >> 5;                     // query tiles of the layout
    const long dq_stride = (long)B * NH * NQT * 2048;  // one key block's partials: [B * NH][NQT][8 sub-tiles][64][4]
    float* dqb = dqp + kb * dq_stride + (long)bh * NQT * 2048;

    const int nqt = (tl + 31) >> 5;  // query tiles past the length: dO rows are 0, nothing to add
    if (!active && w < ngb)         // keys past the length: their dS columns stay 0 for the dQ product
        for (int r = 0; r < 32; ++r)
            if (h == 0) Ss[r * KBP + 32 * w + l32] = 0.f;
    // AHEAD = 2 (the exact fp32 instantiation of the headline): two register stages; 1 (the A/B-only instantiations,
    // which the second stage would push into scratch): fetch tile qt+1 at the start of tile qt, as before
    constexpr int AHEAD = (!BF16 && NW == 8) ? 2 : 1;
    Stg sa, sb;
    fetch(0, sa);
    put(0, sa);
    __syncthreads();
    if (AHEAD == 2 && nqt > 1) fetch(1, sb);
    // tile qt: fetch tile qt+AHEAD into fx (its previous content is in LDS), put tile qt+1 from py
    auto tile = [&](int qt, Stg& fx, const Stg& py) {
        const int q0 = qt * 32, buf = qt & 1;
        if (qt + AHEAD < nqt) fetch(qt + AHEAD, fx);
        const float* Qt = Qs + buf * 32 * FA_LD;
        const float* Dt = Ds + buf * 32 * FA_LD;
        const float* Lt = Ls + buf * 32;
        const float* Dlt = Dl + buf * 32;
        if (active) {
            f32x16 s, dp;
#pragma unroll
            for (int v = 0; v < 16; ++v) s[v] = dp[v] = 0.f;
            prod_rows<BF16>(s, Qt, kv, l32, h);   // S[q][key]: query r8(v,h), key on the lane
            prod_rows<BF16>(dp, Dt, vv, l32, h);  // dP[q][key]
            const bool kok = key < tl;
            // LSE / delta of the lane's rows r8(v, h): 4 runs of 4 consecutive rows, one run live at a time
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                const f32x4 lq = *reinterpret_cast<const f32x4*>(Lt + 8 * a + 4 * h);
                const f32x4 dq = *reinterpret_cast<const f32x4*>(Dlt + 8 * a + 4 * h);
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int v = 4 * a + b, r = r8(v, h);
                    const bool ok = kok && q0 + r < T;
                    const float p = ok ? __builtin_amdgcn_exp2f(sl2 * s[v] - LOG2E * lq[b]) : 0.f;
                    s[v] = p;
                    dp[v] = scale * (p * (dp[v] - dq[b]));
                }
            }
            apply_rows<BF16>(dv, Dt, s, l32, h);   // dV^T[n][key] += sum_q dO[q][n] P[q][key]
            apply_rows<BF16>(dk, Qt, dp, l32, h);  // dK^T[d][key] += sum_q Q[q][d] dS[q][key]
            // dS pairs (as in flash_bwd_bf16_kernel): lanes 2i / 2i + 1 swap one value, 8-B writes
            const bool odd = lane & 1;
#pragma unroll
            for (int v = 0; v < 16; v += 2) {
                const float a = dp[v], b = dp[v + 1];
                const float recv = __int_as_float(
                    __builtin_amdgcn_mov_dpp(__float_as_int(odd ? a : b), 0xB1, 0xF, 0xF, false));
                f32x2 pr;
                pr[0] = odd ? recv : a;
                pr[1] = odd ? b : recv;
                *reinterpret_cast<f32x2*>(Ss + (r8(v, h) + (odd ? 1 : 0)) * KBP + 32 * w + (l32 & ~1)) = pr;
            }
        }
        __syncthreads();  // dS tile complete
#pragma unroll
        for (int j = 0; j < SUB; ++j) {  // dQ partial of this key block: dQ[q][d] = sum_key dS[q][key] K[key][d]
            const int st = w * SUB + j, qi = st & 1, di = st >> 1;
            const float* ar = Ss + (16 * qi + l16) * KBP;
            const float* br = Kt + (16 * di + l16) * KBP;
            f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0;
            if constexpr (!BF16) {
                for (int kc = 0; kc < kq; kc += 32) {
                    const f32x4 a0 = *reinterpret_cast<const f32x4*>(ar + kc + 4 * g);
                    const f32x4 b0 = *reinterpret_cast<const f32x4*>(br + kc + 4 * g);
                    const f32x4 a1 = *reinterpret_cast<const f32x4*>(ar + kc + 16 + 4 * g);
                    const f32x4 b1 = *reinterpret_cast<const f32x4*>(br + kc + 16 + 4 * g);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[e], b0[e], c0, 0, 0, 0);
                        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[e], b1[e], c1, 0, 0, 0);
                    }
                }
            } else {
                for (int kc = 0; kc < kq; kc += 32) {
                    const fbf16x8 a = cvt8(*reinterpret_cast<const f32x4*>(ar + kc + 8 * g),
                                           *reinterpret_cast<const f32x4*>(ar + kc + 8 * g + 4));
                    const fbf16x8 b = cvt8(*reinterpret_cast<const f32x4*>(br + kc + 8 * g),
                                           *reinterpret_cast<const f32x4*>(br + kc + 8 * g + 4));
                    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c0, 0, 0, 0);
                }
            }
            // the block's dQ partial of sub-tile st in fragment order (flash_dq_reduce_frag transposes): one 16-B
            // store per lane, 1 KB contiguous per wave
            *reinterpret_cast<f32x4*>(dqb + ((long)qt * 8 + st) * 256 + lane * 4) = c0 + c1;
        }
        if (qt + 1 < nqt) put(buf ^ 1, py);
        __syncthreads();  // next tile visible; dS tile free
    };
    if constexpr (AHEAD == 2) {
        int qt = 0;
        for (; qt + 1 < nqt; qt += 2) {
            tile(qt, sa, sb);
            tile(qt + 1, sb, sa);
        }
        if (qt < nqt) tile(qt, sa, sb);
    } else {
        for (int qt = 0; qt < nqt; ++qt) tile(qt, sa, sa);
    }
    // dK, dV rows of this wave's keys (0 past the length): lane = key, registers = 4 consecutive columns
    if (w < ngb && key < T) {  // dK, dV rows of this wave's keys
        float* dkr = dqkv + ((long)u * T + key) * ld + H + hd * 64 + 4 * h;
        float* dvr = dkr + H;
    #pragma unroll
        for (int t = 0; t < 2; ++t)
    #pragma unroll
            for (int a = 0; a < 4; ++a) {
                f32x4 x, y;
    #pragma unroll
                for (int b = 0; b < 4; ++b) {
                    x[b] = dk[t][4 * a + b];
                    y[b] = dv[t][4 * a + b];
                }
                if (dqkv) {
                    *reinterpret_cast<f32x4*>(dkr + 32 * t + 8 * a) = x;
                    *reinterpret_cast<f32x4*>(dvr + 32 * t + 8 * a) = y;
                }
                if (dqkvb) {
                    fbf16x4 bx, by;
    #pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        bx[e] = (__bf16)x[e];
                        by[e] = (__bf16)y[e];
                    }
                    __bf16* kb = dqkvb + ((long)u * T + key) * ld + H + hd * 64 + 4 * h + 32 * t + 8 * a;
                    *reinterpret_cast<fbf16x4*>(kb) = bx;
                    *reinterpret_cast<fbf16x4*>(kb + H) = by;
                }
            }
    }
}

// ------------------------------------------------------------------------------------------------
// bf16 mode (config C4): the same two kernels with every LDS image in bf16.  The bf16 MFMAs are 16x the
// fp32 rate, so the fp32-image forms were bound by LDS bytes and the per-element conversions (each
// product read fp32 rows and converted them in registers, the transposed contractions 8 scalar reads per
// MFMA).  Here the staging pass rounds once (RNE, the same rounding the MFMA operands had), row images
// feed 16-B fragment reads and transposed images 8-B reads of 4 consecutive contraction rows.
// ------------------------------------------------------------------------------------------------
typedef __bf16 fbf16x2 __attribute__((ext_vector_type(2)));
constexpr int FB_RS = 72;  // bf16 row image [row][64 + 8]: 144-B rows, 8 consecutive rows on distinct banks

__device__ __forceinline__ fbf16x4 cvt4(f32x4 v) {
    fbf16x4 b;
#pragma unroll
    for (int e = 0; e < 4; ++e) b[e] = (__bf16)v[e];
    return b;
}

// acc[r8(v,h)][l32] += sum_d L[i][d] X[l32][d], L a bf16 row image (stride FB_RS), X the lane's bf16 row
__device__ __forceinline__ void prod_rows_b(f32x16& acc, const __bf16* __restrict__ L, const RowReg<true>& x, int l32,
                                            int h) {
    const __bf16* lr = L + l32 * FB_RS + 8 * h;
#pragma unroll
    for (int s = 0; s < 4; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const fbf16x8*>(lr + 16 * s), x.v[s], acc, 0,
                                                      0, 0);
}

// o[t][32t + r8(v,h)][l32] += sum_r L[r][n] pv[r], L given transposed (Lt[n][r], stride LDT bf16): MFMA c
// takes rows 16c + 4h + 0..3 and 16c + 8 + 4h + 0..3 (accumulator registers 8c .. 8c + 7)
template <int LDT>
__device__ __forceinline__ void apply_cols_b(f32x16 (&o)[2], const __bf16* __restrict__ Lt, const f32x16& pv, int l32,
                                             int h) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        fbf16x8 b;
#pragma unroll
        for (int j = 0; j < 8; ++j) b[j] = (__bf16)pv[8 * c + j];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const __bf16* lr = Lt + (32 * t + l32) * LDT + 16 * c + 4 * h;
            const fbf16x4 lo = *reinterpret_cast<const fbf16x4*>(lr), hi = *reinterpret_cast<const fbf16x4*>(lr + 8);
            fbf16x8 a;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                a[j] = lo[j];
                a[4 + j] = hi[j];
            }
            o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, o[t], 0, 0, 0);
        }
    }
}

constexpr int FBK_LDT = FK + 8;  // transposed bf16 V image [64][64 keys + 8]

__global__ __launch_bounds__(FF_NW_BF * 64) void flash_fwd_bf16_kernel(
    const float* __restrict__ qkv, float* __restrict__ ctx, float* __restrict__ lse, int T, int NH, int H, float scale,
    const int* __restrict__ tlen, int nqb, __bf16* __restrict__ ctxb) {
    constexpr int NW = FF_NW_BF, NT = NW * 64;
    constexpr int ITEMS = FK * 16, NPT = (ITEMS + NT - 1) / NT;
    __shared__ __attribute__((aligned(16))) __bf16 Ks[2][FK * FB_RS];
    __shared__ __attribute__((aligned(16))) __bf16 Vt[2][64 * FBK_LDT];
    const int id = xcd_block();
    const int qb = id % nqb, bh = id / nqb, hd = bh % NH, u = bh / NH;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
    const int tl = tlen ? tlen[u] : T;
    const long ld = 3L * H;
    const float* Qb = qkv + (long)u * T * ld + hd * 64;
    const float* Kb = Qb + H;
    const float* Vb = Qb + 2 * H;
    const int q0 = (qb * NW + w) * 32;
    if (tl <= 0) {  // (block-uniform: one utterance per block)
        flash_fwd_no_keys(ctx, ctxb, lse, (long)u * T, (long)bh * T, T, H, hd, q0, l32, h);
        return;
    }
    const bool active = q0 < T;
    const float sl2 = scale * LOG2E;
    RowReg<true> qv;
    qv.load(Qb + (long)min(q0 + l32, T - 1) * ld, h);
    auto vmap = [](int it, int& key, int& c4) {
        const int l = it & 63, wi = it >> 6;
        key = (l & 15) + 16 * (wi & 3);
        c4 = 4 * ((l >> 4) + 4 * (wi >> 2));
    };
    f32x4 kr[NPT], vr[NPT];
    auto fetch = [&](int kt) {
#pragma unroll
        for (int n = 0; n < NPT; ++n) {
            const int it = threadIdx.x + n * NT, row = it >> 4, c4 = (it & 15) * 4, key = kt * FK + row;
            int vk, vc;
            vmap(it, vk, vc);
            kr[n] = vr[n] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (it < ITEMS && key < T) kr[n] = *reinterpret_cast<const f32x4*>(Kb + (long)key * ld + c4);
            if (it < ITEMS && kt * FK + vk < T) vr[n] = *reinterpret_cast<const f32x4*>(Vb + (long)(kt * FK + vk) * ld + vc);
        }
    };
    auto put = [&](int buf) {
#pragma unroll
        for (int n = 0; n < NPT; ++n) {
            const int it = threadIdx.x + n * NT, row = it >> 4, c4 = (it & 15) * 4;
            int vk, vc;
            vmap(it, vk, vc);
            if (it < ITEMS) {
                *reinterpret_cast<fbf16x4*>(&Ks[buf][row * FB_RS + c4]) = cvt4(kr[n]);
                // V^T as key pairs: lanes 2i / 2i + 1 hold keys k / k + 1 of the same 4 columns; each swaps two
                // values (DPP quad_perm [1,0,3,2]) so the even lane writes columns 0-1 and the odd lane columns
                // 2-3 as (k, k+1) words: 2 writes per lane instead of 4
                const bool odd = threadIdx.x & 1;
                const float s0 = odd ? vr[n][0] : vr[n][2], s1 = odd ? vr[n][1] : vr[n][3];
                const float q0 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s0), 0xB1, 0xF, 0xF, false));
                const float q1 = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(s1), 0xB1, 0xF, 0xF, false));
                fbf16x2 w0, w1;
                w0[0] = (__bf16)(odd ? q0 : vr[n][0]);
                w0[1] = (__bf16)(odd ? vr[n][2] : q0);
                w1[0] = (__bf16)(odd ? q1 : vr[n][1]);
                w1[1] = (__bf16)(odd ? vr[n][3] : q1);
                const int e0 = odd ? 2 : 0;
                *reinterpret_cast<fbf16x2*>(&Vt[buf][(vc + e0) * FBK_LDT + (vk & ~1)]) = w0;
                *reinterpret_cast<fbf16x2*>(&Vt[buf][(vc + e0 + 1) * FBK_LDT + (vk & ~1)]) = w1;
            }
        }
    };
    const int nkt = (tl + FK - 1) / FK;
    f32x16 o[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) o[t][v] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;
    fetch(0);
    put(0);
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nkt) fetch(kt + 1);
        if (active) {
            const bool two = kt * FK + 32 < tl;  // as in flash_fwd_kernel
            f32x16 s[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int v = 0; v < 16; ++v) s[j][v] = 0.f;
                if (j == 0 || two) prod_rows_b(s[j], Ks[buf] + 32 * j * FB_RS, qv, l32, h);
            }
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const bool ok = kt * FK + 32 * j + r8(v, h) < tl;
                    s[j][v] = ok ? sl2 * s[j][v] : -INFINITY;
                    mx = fmaxf(mx, s[j][v]);
                }
            mx = half_swap_max(mx);
            const float m_new = fmaxf(m_run, mx);
            float ls = 0.f;
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    s[j][v] = __builtin_amdgcn_exp2f(s[j][v] - m_new);
                    ls += s[j][v];
                }
            if (m_new != m_run) {
                const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
                l_run *= alpha;
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int v = 0; v < 16; ++v) o[t][v] *= alpha;
                m_run = m_new;
            }
            l_run += ls;
            apply_cols_b<FBK_LDT>(o, Vt[buf], s[0], l32, h);
            if (two) apply_cols_b<FBK_LDT>(o, Vt[buf] + 32, s[1], l32, h);
        }
        if (kt + 1 < nkt) put(buf ^ 1);
        __syncthreads();
    }
    if (!active) return;
    const float l_tot = half_swap_sum(l_run);
    const int q = q0 + l32;
    if (q >= T) return;
    const float inv = 1.0f / l_tot;
    float* cr = ctx + ((long)u * T + q) * H + hd * 64 + 4 * h;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            f32x4 r;
#pragma unroll
            for (int b = 0; b < 4; ++b) r[b] = o[t][4 * a + b] * inv;
            *reinterpret_cast<f32x4*>(cr + 32 * t + 8 * a) = r;
            if (ctxb)
                *reinterpret_cast<fbf16x4*>(ctxb + ((long)u * T + q) * H + hd * 64 + 4 * h + 32 * t + 8 * a) = cvt4(r);
        }
    if (h == 0) lse[(long)bh * T + q] = (m_run + log2f(l_tot)) * (1.0f / LOG2E);
}

// ------------------------------------------------------------------------------------------------
// forward, bf16 operand plane (config C4 with bf16 planes): Q, K and V come from the bf16 plane of qkv
// that the QKV GEMM writes beside its fp32 output, so the kernel converts nothing.  Per 64-key tile the
// block copies the K and V rows as 16-B chunks into row-major LDS images; S^T = K Q^T with the K rows read
// by row (prod_rows_b), and the PV product's V^T operand is read from the ROW-major V image with
// ds_read_b64_tr_b16 (gfx950 transposed read: per 16-lane group, lane 4q + p addresses row q, columns
// 4p..4p+3 of a 4 x 16 block and receives column (lane & 15) of the 4 rows), so the staging writes no
// transposed image.  Masks and address arithmetic only where they are needed: keys past the utterance's
// length exist only in its last tile, and the per-thread copy addresses advance by one constant per tile.
// The exponent argument is one fma (scores scaled to the log2 domain, the row maximum taken on raw
// scores: scaling by a positive constant commutes with max under round-to-nearest).
// ------------------------------------------------------------------------------------------------
constexpr int FP_KS = 72;  // K image row stride (bf16): 144 B
constexpr int FP_VS = 96;  // V image row stride (bf16): 192 B -> the 4 rows x 64 B of a 32-lane tr read hit 64 banks

typedef __attribute__((address_space(3))) fbf16x4* lds_b4p;

// o[t] += V^T(rows 32t..32t+31 = head dims, contraction over 16 keys from kb) P^T: the A operand by two
// transposed reads of the row-major V image (keys kb + 4h + 0..3 and kb + 8 + 4h + 0..3, as apply_cols_b)
template <int RS = FP_VS>
__device__ __forceinline__ void pv_tr(f32x16 (&o)[2], const __bf16* __restrict__ V, int kb, const fbf16x8& b,
                                      int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int k0 = kb + 4 * (g >> 1) + q;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const __bf16* a0 = V + k0 * RS + 32 * t + 16 * (g & 1) + 4 * pp;
        const fbf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4p)(a0));
        const fbf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4p)(a0 + 8 * RS));
        fbf16x8 a;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            a[j] = lo[j];
            a[4 + j] = hi[j];
        }
        o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, o[t], 0, 0, 0);
    }
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void flash_fwd_bf16p_kernel(
    const __bf16* __restrict__ qkvb, float* __restrict__ ctx, float* __restrict__ lse, int T, int NH, int H,
    float scale, const int* __restrict__ tlen, int nqb, __bf16* __restrict__ ctxb) {
    constexpr int NT = NW * 64;
    constexpr int NPT = 512 / NT;  // 16-B chunks of a 64 x 64 bf16 tile per thread (each of K and V)
    __shared__ __attribute__((aligned(16))) __bf16 Ks[2][FK * FP_KS];
    __shared__ __attribute__((aligned(16))) __bf16 Vs[2][FK * FP_VS];
    const int id = xcd_block();
    const int qb = id % nqb, bh = id / nqb, hd = bh % NH, u = bh / NH;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
    const int tl = tlen ? tlen[u] : T;
    const long ld = 3L * H;
    const __bf16* Qb = qkvb + (long)u * T * ld + hd * 64;
    const int q0 = (qb * NW + w) * 32;
    if (tl <= 0) {  // (block-uniform: one utterance per block)
        flash_fwd_no_keys(ctx, ctxb, lse, (long)u * T, (long)bh * T, T, H, hd, q0, l32, h);
        return;
    }
    const bool active = q0 < T;
    const float sl2 = scale * LOG2E;
    RowReg<true> qv;
    {
        const __bf16* qr = Qb + (long)min(q0 + l32, T - 1) * ld + 8 * h;
#pragma unroll
        for (int s = 0; s < 4; ++s) qv.v[s] = *reinterpret_cast<const fbf16x8*>(qr + 16 * s);
    }
    // copy map: chunk c = threadIdx.x + n NT of a tile, row c >> 3, columns 8 (c & 7) .. + 7
    const int crow = threadIdx.x >> 3, ccol = (threadIdx.x & 7) * 8;
    fbf16x8 kr[NPT], vr[NPT];
    auto fetch = [&](int kt) {
#pragma unroll
        for (int n = 0; n < NPT; ++n) {
            const int key = min(kt * FK + crow + n * (NT / 8), T - 1);  // rows past T: any finite row (P = 0)
            const __bf16* src = Qb + (long)key * ld + ccol;
            kr[n] = *reinterpret_cast<const fbf16x8*>(src + H);
            vr[n] = *reinterpret_cast<const fbf16x8*>(src + 2 * H);
        }
    };
    auto put = [&](int buf) {
#pragma unroll
        for (int n = 0; n < NPT; ++n) {
            const int row = crow + n * (NT / 8);
            *reinterpret_cast<fbf16x8*>(&Ks[buf][row * FP_KS + ccol]) = kr[n];
            *reinterpret_cast<fbf16x8*>(&Vs[buf][row * FP_VS + ccol]) = vr[n];
        }
    };
    const int nkt = (tl + FK - 1) / FK;
    f32x16 o[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) o[t][v] = 0.f;
    float m_run = -INFINITY, l_run = 0.f;
    fetch(0);
    put(0);
    __syncthreads();
    // full tiles run a body without masks; the utterance's last tile (masks, the empty second half skipped) is
    // peeled, so neither costs the full tiles a branch-merged register copy
    auto tile = [&](int kt, auto last_tag) {
        constexpr bool LAST = decltype(last_tag)::value;
        const int buf = kt & 1;
        if (!LAST) fetch(kt + 1);
        if (active) {
            const bool two = !LAST || kt * FK + 32 < tl;
            f32x16 s[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
                for (int v = 0; v < 16; ++v) s[j][v] = LAST ? -INFINITY : 0.f;
                if (j == 0 || two) {
                    if (LAST)
#pragma unroll
                        for (int v = 0; v < 16; ++v) s[j][v] = 0.f;
                    prod_rows_b(s[j], Ks[buf] + 32 * j * FP_KS, qv, l32, h);
                }
            }
            if (LAST) {  // keys >= tl get probability 0
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int v = 0; v < 16; ++v)
                        if (kt * FK + 32 * j + r8(v, h) >= tl) s[j][v] = -INFINITY;
            }
            float mx = s[0][0];
#pragma unroll
            for (int v = 1; v < 16; ++v) mx = fmaxf(mx, s[0][v]);
            if (two)
#pragma unroll
                for (int v = 0; v < 16; ++v) mx = fmaxf(mx, s[1][v]);
            mx = half_swap_max(mx);
            const float m_new = fmaxf(m_run, sl2 * mx);
            float ls = 0.f;
            fbf16x8 pb[2][2];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int v = 0; v < 16; ++v) {
                    const float pr = __builtin_amdgcn_exp2f(fmaf(s[j][v], sl2, -m_new));
                    ls += pr;
                    pb[j][v >> 3][v & 7] = (__bf16)pr;
                }
            if (m_new != m_run) {
                const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
                l_run *= alpha;
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int v = 0; v < 16; ++v) o[t][v] *= alpha;
                m_run = m_new;
            }
            l_run += ls;
#pragma unroll
            for (int c = 0; c < 2; ++c) pv_tr(o, Vs[buf], 16 * c, pb[0][c], lane);
            if (two)
#pragma unroll
                for (int c = 0; c < 2; ++c) pv_tr(o, Vs[buf], 32 + 16 * c, pb[1][c], lane);
        }
        if (!LAST) put(buf ^ 1);
        __syncthreads();
    };
    for (int kt = 0; kt + 1 < nkt; ++kt) tile(kt, std::false_type{});
    tile(nkt - 1, std::true_type{});
    if (!active) return;
    const float l_tot = half_swap_sum(l_run);
    const int q = q0 + l32;
    if (q >= T) return;
    const float inv = 1.0f / l_tot;
    float* cr = ctx + ((long)u * T + q) * H + hd * 64 + 4 * h;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            f32x4 r;
#pragma unroll
            for (int b = 0; b < 4; ++b) r[b] = o[t][4 * a + b] * inv;
            *reinterpret_cast<f32x4*>(cr + 32 * t + 8 * a) = r;
            if (ctxb)
                *reinterpret_cast<fbf16x4*>(ctxb + ((long)u * T + q) * H + hd * 64 + 4 * h + 32 * t + 8 * a) = cvt4(r);
        }
    if (h == 0) lse[(long)bh * T + q] = (m_run + log2f(l_tot)) * (1.0f / LOG2E);
}

// backward, bf16 images: Q / dO tiles row-major (S, dP) and transposed (dV, dK), dS and K^T in bf16
constexpr int FBB_NW = 8;
constexpr int FBB_KB = FBB_NW * 32 + 8;   // bf16 row stride of the dS tile and the K^T image
constexpr int FBB_QT = 32 + 8;            // bf16 row stride of the transposed Q / dO tiles
constexpr size_t fbb_lds_bytes() {
    return 2 * ((size_t)(64 + 32) * FBB_KB + 2 * (2 * 32 * FB_RS + 2 * 64 * FBB_QT)) + 4 * 128;
}

__global__ __launch_bounds__(FBB_NW * 64, 1) void flash_bwd_bf16_kernel(
    const float* __restrict__ qkv, const float* __restrict__ dctx, const float* __restrict__ lse,
    const float* __restrict__ delta, float* __restrict__ dqkv, float* __restrict__ dqp, int T, int NH, int H,
    float scale, const int* __restrict__ tlen, int nkb, int gpb, int B, __bf16* __restrict__ dqkvb) {
    constexpr int NW = FBB_NW, NT = NW * 64;
    constexpr int QPT = 512 / NT;
    extern __shared__ __attribute__((aligned(16))) __bf16 sm16[];
    __bf16* Kt = sm16;                            // [64][FBB_KB]
    __bf16* Ss = Kt + 64 * FBB_KB;                // [32][FBB_KB]
    __bf16* Qr = Ss + 32 * FBB_KB;                // [2][32][FB_RS]   Q rows
    __bf16* Dr = Qr + 2 * 32 * FB_RS;             // [2][32][FB_RS]   dO rows
    __bf16* Qc = Dr + 2 * 32 * FB_RS;             // [2][64][FBB_QT]  Q transposed
    __bf16* Dc = Qc + 2 * 64 * FBB_QT;            // [2][64][FBB_QT]  dO transposed
    float* Ls = reinterpret_cast<float*>(Dc + 2 * 64 * FBB_QT);  // [2][32]
    float* Dl = Ls + 64;                          // [2][32]
    const int id = xcd_block();
    const int kb = id % nkb, bh = id / nkb, hd = bh % NH, u = bh / NH;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, l32 = lane & 31, h = lane >> 5;
    const int tl = tlen ? tlen[u] : T;
    const int ng = (T + 31) >> 5;
    const int g0 = kb * gpb, ngb = min(gpb, ng - g0);
    const int kbase = g0 * 32;
    const long ld = 3L * H;
    const float* Qb = qkv + (long)u * T * ld + hd * 64;
    const float* Kb = Qb + H;
    const float* Vb = Qb + 2 * H;
    const float* Ob = dctx + (long)u * T * H + hd * 64;
    const float* lb = lse + (long)bh * T;
    const float* db = delta + (long)bh * T;
    const bool active = w < ngb && kbase + 32 * w < tl;
    const int key = kbase + 32 * w + l32;
    const float sl2 = scale * LOG2E;
    RowReg<true> kv, vv;
    kv.load(Kb + (long)min(key, T - 1) * ld, h);
    vv.load(Vb + (long)min(key, T - 1) * ld, h);
    for (int it = threadIdx.x; it < ngb * 32 * 16; it += NT) {
        const int row = it >> 4, c4 = (it & 15) * 4, k = kbase + row;
        f32x4 x = {0.f, 0.f, 0.f, 0.f};
        if (k < T) x = *reinterpret_cast<const f32x4*>(Kb + (long)k * ld + c4);
#pragma unroll
        for (int e = 0; e < 4; ++e) Kt[(c4 + e) * FBB_KB + row] = (__bf16)x[e];
    }
    f32x4 qr[QPT], orr[QPT];
    float lr = 0.f;
    auto fetch = [&](int qt) {
#pragma unroll
        for (int n = 0; n < QPT; ++n) {
            const int it = threadIdx.x + n * NT, row = it >> 4, c4 = (it & 15) * 4, q = qt * 32 + row;
            qr[n] = orr[n] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (q < T) {
                qr[n] = *reinterpret_cast<const f32x4*>(Qb + (long)q * ld + c4);
                orr[n] = *reinterpret_cast<const f32x4*>(Ob + (long)q * H + c4);
            }
        }
        lr = 0.f;
        const int qq = qt * 32 + (threadIdx.x & 31);
        if (threadIdx.x < 64 && qq < T) lr = threadIdx.x < 32 ? lb[qq] : db[qq];
    };
    auto put = [&](int buf) {
#pragma unroll
        for (int n = 0; n < QPT; ++n) {
            const int it = threadIdx.x + n * NT, row = it >> 4, c4 = (it & 15) * 4;
            *reinterpret_cast<fbf16x4*>(Qr + (buf * 32 + row) * FB_RS + c4) = cvt4(qr[n]);
            *reinterpret_cast<fbf16x4*>(Dr + (buf * 32 + row) * FB_RS + c4) = cvt4(orr[n]);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                Qc[(buf * 64 + c4 + e) * FBB_QT + row] = (__bf16)qr[n][e];
                Dc[(buf * 64 + c4 + e) * FBB_QT + row] = (__bf16)orr[n][e];
            }
        }
        if (threadIdx.x < 32) Ls[buf * 32 + threadIdx.x] = lr;
        else if (threadIdx.x < 64) Dl[buf * 32 + threadIdx.x - 32] = lr;
    };
    f32x16 dv[2], dk[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) dv[t][v] = dk[t][v] = 0.f;
    const int g = lane >> 4, l16 = lane & 15;
    const int qi = w & 1, di = w >> 1;
    const int kq = ngb * 32;
    const long dq_stride = (long)B * NH * T * 64;
    float* dqb = dqp + kb * dq_stride + (long)bh * T * 64;
    const int nqt = (tl + 31) >> 5;
    if (!active && w < ngb)
        for (int r = 0; r < 32; ++r)
            if (h == 0) Ss[r * FBB_KB + 32 * w + l32] = (__bf16)0.f;
    fetch(0);
    put(0);
    __syncthreads();
    // the wave's dQ B operand (K^T rows 16 di + l16 over the block's keys) is the same for every query
    // tile: held in registers (kq <= 256 keys = 8 fragments) instead of re-read from LDS per tile
    fbf16x8 kfr[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        if (32 * j < kq) kfr[j] = *reinterpret_cast<const fbf16x8*>(Kt + (16 * di + l16) * FBB_KB + 32 * j + 8 * g);
    const bool odd = lane & 1;
    for (int qt = 0; qt < nqt; ++qt) {
        const int q0 = qt * 32, buf = qt & 1;
        if (qt + 1 < nqt) fetch(qt + 1);
        const float* Lt = Ls + buf * 32;
        const float* Dlt = Dl + buf * 32;
        if (active) {
            f32x16 s, dp;
#pragma unroll
            for (int v = 0; v < 16; ++v) s[v] = dp[v] = 0.f;
            prod_rows_b(s, Qr + buf * 32 * FB_RS, kv, l32, h);
            prod_rows_b(dp, Dr + buf * 32 * FB_RS, vv, l32, h);
            // the lane's 16 rows r8(v, h) are 4 runs of 4 consecutive rows: 16-B reads of LSE and delta
            f32x4 lq[4], dq[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                lq[a] = *reinterpret_cast<const f32x4*>(Lt + 8 * a + 4 * h);
                dq[a] = *reinterpret_cast<const f32x4*>(Dlt + 8 * a + 4 * h);
            }
            const bool kok = key < tl;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int r = r8(v, h);
                const bool ok = kok && q0 + r < T;
                const float p = ok ? __builtin_amdgcn_exp2f(sl2 * s[v] - LOG2E * lq[v >> 2][v & 3]) : 0.f;
                s[v] = p;
                dp[v] = scale * (p * (dp[v] - dq[v >> 2][v & 3]));
            }
            apply_cols_b<FBB_QT>(dv, Dc + buf * 64 * FBB_QT, s, l32, h);   // dV^T += dO^T P
            apply_cols_b<FBB_QT>(dk, Qc + buf * 64 * FBB_QT, dp, l32, h);  // dK^T += Q^T dS
            // dS into LDS as bf16 pairs: lanes 2i / 2i + 1 (keys k, k + 1) swap one value (DPP quad_perm
            // [1,0,3,2]) so the even lane writes row r keys (k, k+1) and the odd lane row r + 1 (rows r8(v, h)
            // and r8(v + 1, h) = r + 1 for even v): 8 four-byte writes per lane instead of 16 two-byte ones
#pragma unroll
            for (int v = 0; v < 16; v += 2) {
                const float a = dp[v], b = dp[v + 1];
                const float recv = __int_as_float(
                    __builtin_amdgcn_mov_dpp(__float_as_int(odd ? a : b), 0xB1, 0xF, 0xF, false));
                fbf16x2 pr;
                pr[0] = (__bf16)(odd ? recv : a);
                pr[1] = (__bf16)(odd ? b : recv);
                *reinterpret_cast<fbf16x2*>(Ss + (r8(v, h) + (odd ? 1 : 0)) * FBB_KB + 32 * w + (l32 & ~1)) = pr;
            }
        }
        __syncthreads();  // dS tile complete
        {
            const __bf16* ar = Ss + (16 * qi + l16) * FBB_KB + 8 * g;
            f32x4 c[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int j = 0; j < 8; ++j)  // same split of the key chunks over two chains as before (j even / odd)
                if (32 * j < kq)
                    c[j & 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        *reinterpret_cast<const fbf16x8*>(ar + 32 * j), kfr[j], c[j & 1], 0, 0, 0);
            const f32x4 c0 = c[0], c1 = c[1];
            float* dr = dqb + (long)(q0 + 16 * qi + 4 * g) * 64 + 16 * di + l16;
#pragma unroll
            for (int r = 0; r < 4; ++r)
                if (q0 + 16 * qi + 4 * g + r < T) dr[r * 64] = c0[r] + c1[r];
        }
        if (qt + 1 < nqt) put(buf ^ 1);
        __syncthreads();
    }
    if (w < ngb && key < T) {  // dK, dV rows of this wave's keys
        float* dkr = dqkv + ((long)u * T + key) * ld + H + hd * 64 + 4 * h;
        float* dvr = dkr + H;
    #pragma unroll
        for (int t = 0; t < 2; ++t)
    #pragma unroll
            for (int a = 0; a < 4; ++a) {
                f32x4 x, y;
    #pragma unroll
                for (int b = 0; b < 4; ++b) {
                    x[b] = dk[t][4 * a + b];
                    y[b] = dv[t][4 * a + b];
                }
                if (dqkv) {  // null in bf16 mode when only the bf16 plane is read (the QKV input-gradient GEMM)
                    *reinterpret_cast<f32x4*>(dkr + 32 * t + 8 * a) = x;
                    *reinterpret_cast<f32x4*>(dvr + 32 * t + 8 * a) = y;
                }
                if (dqkvb) {
                    __bf16* kb2 = dqkvb + ((long)u * T + key) * ld + H + hd * 64 + 4 * h + 32 * t + 8 * a;
                    *reinterpret_cast<fbf16x4*>(kb2) = cvt4(x);
                    *reinterpret_cast<fbf16x4*>(kb2 + H) = cvt4(y);
                }
            }
    }
}

// backward on bf16 operand planes (config C4 with bf16 planes): K and V rows of the wave's keys, the
// block's K^T image, and the Q / dO query tiles all come from bf16 planes (qkv's, written by the QKV GEMM
// in the forward; dctx's, written by the out-projection's input-gradient GEMM), so nothing is converted.
// One row image per query tile serves the S / dP products (row reads) and the dV^T / dK^T products
// (ds_read_b64_tr_b16 transposed reads, as the forward's PV): no transposed tiles are written.  Masks only
// on a wave whose keys pass the utterance's length or on a query tile past T.
//
// One barrier per query tile (round 5; the two-barrier form was removed in round 6).  The dS image is double-buffered (tile qt
// writes Ss[qt & 1]) and tile qt + 1's Q / dO rows are put into their image BEFORE tile qt's barrier, so that one
// barrier both completes tile qt's dS image (RAW for its dQ) and publishes tile qt + 1 (RAW for its S / dP).  WAR:
// the Q / dO image tile qt + 1 overwrites held tile qt - 1, whose last reads (its S / dP / dV / dK products) every
// wave finished before tile qt - 1's barrier; Ss[qt & 1] is rewritten by tile qt + 2 after tile qt + 1's barrier,
// which every wave reaches only after its dQ reads of tile qt.  Per element the same operations in the same order:
// bitwise equal to the two-barrier form.
//
// The dS image is KEY-major (round 6; cdna_hip_programming.md section 3, "an accumulator tile whose column index a
// later product sums over"): the lane holds dS for its key (the lane) and 16 query rows (registers 4a .. 4a + 3 =
// rows 8a + 4h + 0..3, four consecutive rows), so it stores 4 packed 8-byte words at [its key][8a + 4h] -- 4
// ds_write_b64 per lane and tile instead of 16 two-byte stores (the former query-major image: 1.87 bank-conflict
// cycles per LDS instruction).  The dQ product's A operand (16 queries x 32 keys of the 16x16x32 MFMA)
// is read back with ds_read_b64_tr_b16 (T10: per 16-lane group 4 key rows x 16 query columns delivered column-
// major).  Rows of 72 B (FBS_RS = 36 bf16): the 16 consecutive keys of a store's lane group land on 16 distinct
// 2-dword bank pairs (18 k mod 32), and a transposed read's 32-lane half takes the 8 keys {4m + c} of a 32-key
// chunk (72 m mod 64 = 8 m: 8 disjoint 8-dword windows).  The MFMA's k-slot 8 gg + jj (gg = lane >> 4) therefore
// holds key fbs_key(gg, jj) of the chunk, and the K^T image stores each chunk's keys in that order (fbs_pos), so the
// B operand stays one contiguous 16-B read.
constexpr int FBS_RS = 36;
__device__ __forceinline__ int fbs_key(int gg, int jj) { return 16 * (gg & 1) + 4 * (jj & 3) + 2 * (gg >> 1) + (jj >> 2); }
__device__ __forceinline__ int fbs_pos(int kl) {  // inverse of fbs_key within a 32-key chunk
    const int gg = ((kl >> 4) & 1) | (((kl >> 1) & 1) << 1), jj = ((kl >> 2) & 3) | ((kl & 1) << 2);
    return 8 * gg + jj;
}

// The Q / dO row images of the bf16-plane backward (round 6): query row q of a tile at image row fq_row(q) (a
// permutation of the 5 row bits: image bits 0, 1, 2, 3 = row bits 2, 3, 0, 1), rows padded to FB_RS = 72 bf16.  With
// rows in natural order the transposed reads were 2-way conflicted (36 r mod 64 puts rows r and r + 2 of a read's four
// rows on overlapping 16-bank windows); with this order both reads of the tile body are conflict-free (searched over
// every bit permutation and padded stride):
//   row reads (prod_rows_q: ds_read_b128, lane l32 -> query l32, 16 B at column 8h + 16s) -- each 16-lane group's 16
//     rows cover the 64 banks once;
//   transposed reads (pv_tr_q: ds_read_b64_tr_b16 of queries R0 .. R0 + 3, R0 = 0 mod 4, 16 columns per 32-lane half)
//     -- the four image rows' 16-dword windows are disjoint mod 64.
// Rows R0 + 8 and R0 + 16 are image rows fq_row(R0) + 2 and + 16, and a column step is a constant too, so every read
// is one address register plus an immediate offset.
__device__ __forceinline__ int fq_row(int q) {
    return ((q >> 2) & 1) | (((q >> 3) & 1) << 1) | ((q & 1) << 2) | (((q >> 1) & 1) << 3) | (q & 16);
}

// prod_rows_b on a permuted image
__device__ __forceinline__ void prod_rows_q(f32x16& acc, const __bf16* __restrict__ L, const RowReg<true>& x, int l32,
                                            int h) {
    const __bf16* lr = L + fq_row(l32) * FB_RS + 8 * h;
#pragma unroll
    for (int s = 0; s < 4; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const fbf16x8*>(lr + 16 * s), x.v[s], acc, 0,
                                                      0, 0);
}

// pv_tr on a permuted image: o[t] += L^T(rows 32t.. = columns of L, contraction over 16 queries from kb) b
__device__ __forceinline__ void pv_tr_q(f32x16 (&o)[2], const __bf16* __restrict__ L, int kb, const fbf16x8& b,
                                        int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const int k0 = kb + 4 * (g >> 1) + q;  // (bit 3 clear: query k0 + 8 is image row fq_row(k0) + 2)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const __bf16* a0 = L + fq_row(k0) * FB_RS + 32 * t + 16 * (g & 1) + 4 * pp;
        const fbf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4p)(a0));
        const fbf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4p)(a0 + 2 * FB_RS));
        fbf16x8 a;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            a[j] = lo[j];
            a[4 + j] = hi[j];
        }
        o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, o[t], 0, 0, 0);
    }
}

constexpr size_t fbbp_lds_bytes() {
    return 2 * ((size_t)64 * FBB_KB + 2 * FBB_NW * 32 * FBS_RS + 2 * 2 * 32 * FB_RS) + 4 * 128;
}
constexpr int FBB_DKS = 72;  // bf16 row stride of the dK / dV staging images at the end of the kernel

// DG (tools build only, SUTA_FB_DIAG; wrong results): parts of the tile body removed to locate its time -- 1 the dQ
// product, 2 the softmax / dS arithmetic, 4 the dV / dK products, 8 the S / dP products, 16 the query-tile prefetch,
// 32 the dS stores, 64 the K^T image, 128 the dK / dV stores.  libsuta.so instantiates DG = 0 only.
template <int DG = 0>
__global__ __launch_bounds__(FBB_NW * 64, 1) void flash_bwd_bf16p_kernel(
    const __bf16* __restrict__ qkvb, const __bf16* __restrict__ dob, const float* __restrict__ lse,
    const float* __restrict__ delta, float* __restrict__ dqkv, float* __restrict__ dqp, int T, int NH, int H,
    float scale, const int* __restrict__ tlen, int nkb, int gpb, int B, __bf16* __restrict__ dqkvb) {
    constexpr int NW = FBB_NW, NT = NW * 64;
    constexpr int NSS = 2;                        // dS images (one barrier per query tile)
    extern __shared__ __attribute__((aligned(16))) __bf16 sm16[];
    __bf16* Kt = sm16;                            // [64][FBB_KB]   K^T of the block's keys (fbs_pos order per chunk)
    __bf16* Ss = Kt + 64 * FBB_KB;                // [NSS][NW * 32][FBS_RS] dS of the query tile, key-major
    __bf16* Qr = Ss + NSS * NW * 32 * FBS_RS;     // [2][32][FB_RS] Q rows (query q at image row fq_row(q))
    __bf16* Dr = Qr + 2 * 32 * FB_RS;             // [2][32][FB_RS] dO rows (likewise)
    float* Ls = reinterpret_cast<float*>(Dr + 2 * 32 * FB_RS);  // [2][32]
    float* Dl = Ls + 64;                          // [2][32]
    const int id = xcd_block();
    const int kb = id % nkb, bh = id / nkb, hd = bh % NH, u = bh / NH;
    // the wave index as a scalar: every per-wave condition below (active, kall) is then a scalar branch
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, l32 = lane & 31,
              h = lane >> 5;
    const int tl = tlen ? tlen[u] : T;
    const int ng = (T + 31) >> 5;
    const int g0 = kb * gpb, ngb = min(gpb, ng - g0);
    const int kbase = g0 * 32;
    const long ld = 3L * H;
    const __bf16* Qb = qkvb + (long)u * T * ld + hd * 64;
    const __bf16* Kb = Qb + H;
    const __bf16* Vb = Qb + 2 * H;
    const __bf16* Ob = dob + (long)u * T * H + hd * 64;
    const float* lb = lse + (long)bh * T;
    const float* db = delta + (long)bh * T;
    const bool active = w < ngb && kbase + 32 * w < tl;
    const bool kall = kbase + 32 * w + 32 <= tl;  // every key of the wave inside the length (wave-uniform)
    const int key = kbase + 32 * w + l32;
    const float sl2 = scale * LOG2E;
    RowReg<true> kv, vv;
    {
        const long kr = (long)min(key, T - 1) * ld + 8 * h;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            kv.v[s] = *reinterpret_cast<const fbf16x8*>(Kb + kr + 16 * s);
            vv.v[s] = *reinterpret_cast<const fbf16x8*>(Vb + kr + 16 * s);
        }
    }
    for (int it = threadIdx.x; it < ((DG & 64) ? 0 : ngb * 32 * 8); it += NT) {  // K^T image of the block's keys
        const int row = it >> 3, c8 = (it & 7) * 8, k = kbase + row;
        fbf16x8 x = {};
        if (k < T) x = *reinterpret_cast<const fbf16x8*>(Kb + (long)k * ld + c8);
        const int pos = (row & ~31) | fbs_pos(row & 31);
#pragma unroll
        for (int e = 0; e < 8; ++e) Kt[(c8 + e) * FBB_KB + pos] = x[e];
    }
    // query-tile copy: threads 0..255 one 16-B chunk of the Q rows, 256..511 one of the dO rows.  Two register
    // stages: the loads of tile qt+2 are issued at the start of tile qt and written to LDS at the end of tile qt+1,
    // so a global load has two tiles of compute to land (one tile was shorter than its latency: parked waves)
    const bool isq = threadIdx.x < 256;
    const int crow = (threadIdx.x & 255) >> 3, ccol = (threadIdx.x & 7) * 8;
    struct Stg {
        fbf16x8 xr;
        float lr;
    };
    auto fetch = [&](int qt, Stg& sg) {
        const int q = qt * 32 + crow;
        sg.xr = fbf16x8{};
        if (q < T) sg.xr = *reinterpret_cast<const fbf16x8*>(isq ? Qb + (long)q * ld + ccol : Ob + (long)q * H + ccol);
        sg.lr = 0.f;
        const int qq = qt * 32 + (threadIdx.x & 31);
        if (threadIdx.x < 64 && qq < T) sg.lr = threadIdx.x < 32 ? lb[qq] : db[qq];
    };
    auto put = [&](int buf, const Stg& sg) {
        *reinterpret_cast<fbf16x8*>((isq ? Qr : Dr) + (buf * 32 + fq_row(crow)) * FB_RS + ccol) = sg.xr;
        if (threadIdx.x < 32) Ls[buf * 32 + threadIdx.x] = sg.lr;
        else if (threadIdx.x < 64) Dl[buf * 32 + threadIdx.x - 32] = sg.lr;
    };
    f32x16 dv[2], dk[2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int v = 0; v < 16; ++v) dv[t][v] = dk[t][v] = 0.f;
    const int g = lane >> 4, l16 = lane & 15;
    const int qi = w & 1, di = w >> 1;
    const int kq = ngb * 32;
    const int NQT = (T + 31) >> 5;                     // query tiles of the layout
    const long dq_stride = (long)B * NH * NQT * 2048;  // one key block's partials: [B * NH][NQT][NW][64 lanes][4]
    float* dqb = dqp + kb * dq_stride + (long)bh * NQT * 2048;
    const int nqt = (tl + 31) >> 5;
    if (!active && w < ngb)  // keys past the length: zero dS rows in every image
        for (int i = 0; i < NSS; ++i)
#pragma unroll
            for (int c = 0; c < 32; c += 8)
                *reinterpret_cast<fbf16x4*>(Ss + (i * NW * 32 + 32 * w + l32) * FBS_RS + c + 4 * h) = fbf16x4{};
    Stg sa, sb;
    fetch(0, sa);
    put(0, sa);
    __syncthreads();
    if (nqt > 1) fetch(1, sb);
    // (the dQ product's K^T fragments are read from the K^T image per tile: holding them in registers, 32 VGPRs,
    // made the two-stage prefetch spill)
    const __bf16* kfrow = Kt + (16 * di + l16) * FBB_KB + 8 * g;
    // the dQ A operand's transposed reads: lane 4 q' + p of 16-lane group g reads key rows fbs_key(g, q') and
    // fbs_key(g, 4 + q') of each 32-key chunk, query columns 16 qi + 4 p .. + 3
    const int trq = (lane >> 2) & 3, trp = lane & 3;
    const int tr_off0 = fbs_key(g, trq) * FBS_RS + 16 * qi + 4 * trp;
    const int tr_off1 = fbs_key(g, 4 + trq) * FBS_RS + 16 * qi + 4 * trp;
    // tile qt: fetch tile qt+2 into fx (its previous content, tile qt, is in LDS), put tile qt+1 from py; BUF = qt & 1
    // as a constant (the two unrolled instances), so the LDS image addresses fold
    auto tile = [&](int qt, Stg& fx, const Stg& py, auto buf_tag) {
        constexpr int buf = decltype(buf_tag)::value;
        __bf16* const Sb = Ss + buf * NW * 32 * FBS_RS;  // this tile's dS image (key-major)
        __bf16* const srow = Sb + (32 * w + l32) * FBS_RS + 4 * h;       // the lane's key row, its half's columns
        const int q0 = qt * 32;
        if (!(DG & 16) && qt + 2 < nqt) fetch(qt + 2, fx);
        const float* Lt = Ls + buf * 32;
        const float* Dlt = Dl + buf * 32;
        if (active) {
            const __bf16* Qt = Qr + buf * 32 * FB_RS;
            const __bf16* Dt = Dr + buf * 32 * FB_RS;
            f32x16 s, dp;
#pragma unroll
            for (int v = 0; v < 16; ++v) s[v] = dp[v] = 0.f;
            if constexpr (!(DG & 8)) {
                prod_rows_q(s, Qt, kv, l32, h);
                prod_rows_q(dp, Dt, vv, l32, h);
            }
            f32x4 lq[4], dq[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                lq[a] = *reinterpret_cast<const f32x4*>(Lt + 8 * a + 4 * h);
                dq[a] = *reinterpret_cast<const f32x4*>(Dlt + 8 * a + 4 * h);
            }
            if constexpr (!(DG & 2)) {
#pragma unroll
            for (int v = 0; v < 16; ++v) s[v] = __builtin_amdgcn_exp2f(fmaf(s[v], sl2, -LOG2E * lq[v >> 2][v & 3]));
            if (!kall || q0 + 32 > T) {  // keys past the length, query rows past T: probability 0
                const bool kok = key < tl;
#pragma unroll
                for (int v = 0; v < 16; ++v)
                    if (!(kok && q0 + r8(v, h) < T)) s[v] = 0.f;
            }
#pragma unroll
            for (int v = 0; v < 16; ++v) dp[v] = scale * (s[v] * (dp[v] - dq[v >> 2][v & 3]));
            }
            fbf16x8 pb[2], sb[2];
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                pb[v >> 3][v & 7] = (__bf16)s[v];
                sb[v >> 3][v & 7] = (__bf16)dp[v];
            }
            if constexpr (!(DG & 4)) {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                pv_tr_q(dv, Dt, 16 * c, pb[c], lane);  // dV^T += dO^T P
                pv_tr_q(dk, Qt, 16 * c, sb[c], lane);  // dK^T += Q^T dS
            }
            }
            // dS into the key-major image: registers 4a .. 4a + 3 (query rows 8a + 4h + 0..3) as one 8-byte store each
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                if constexpr (DG & 32) break;
                fbf16x4 w4;
#pragma unroll
                for (int e = 0; e < 4; ++e) w4[e] = sb[a >> 1][4 * (a & 1) + e];
                *reinterpret_cast<fbf16x4*>(srow + 8 * a) = w4;
            }
        }
        if (qt + 1 < nqt) put(buf ^ 1, py);  // published by the barrier below
        __syncthreads();  // dS tile complete
        if constexpr (!(DG & 1)) {
            f32x4 c[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (32 * j < kq) {  // (wave-uniform: EXEC stays all ones for the transposed reads)
                    const __bf16* a0 = Sb + 32 * j * FBS_RS;
                    const fbf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4p)(a0 + tr_off0));
                    const fbf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4p)(a0 + tr_off1));
                    fbf16x8 a;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        a[e] = lo[e];
                        a[4 + e] = hi[e];
                    }
                    c[j & 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        a, *reinterpret_cast<const fbf16x8*>(kfrow + 32 * j), c[j & 1], 0, 0, 0);
                }
            // the block's dQ partial of this tile in fragment order (flash_dq_reduce_frag transposes): one 16-B store
            // per lane, the wave's 1 KB contiguous (the row layout took four stores of 64-B pieces)
            *reinterpret_cast<f32x4*>(dqb + ((long)qt * NW + w) * 256 + lane * 4) = c[0] + c[1];
        }
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    int qt = 0;
    for (; qt + 1 < nqt; qt += 2) {
        tile(qt, sa, sb, B0{});
        tile(qt + 1, sb, sa, B1{});
    }
    if (qt < nqt) tile(qt, sa, sb, B0{});
    // dK, dV rows of this wave's keys.  fp32 (when requested; in bf16 mode null when only the bf16 plane is read, the
    // QKV input-gradient GEMM): direct 16-B stores
    if (!(DG & 128) && dqkv && w < ngb && key < T) {
        float* dkr = dqkv + ((long)u * T + key) * ld + H + hd * 64 + 4 * h;
        float* dvr = dkr + H;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                f32x4 x, y;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    x[b] = dk[t][4 * a + b];
                    y[b] = dv[t][4 * a + b];
                }
                *reinterpret_cast<f32x4*>(dkr + 32 * t + 8 * a) = x;
                *reinterpret_cast<f32x4*>(dvr + 32 * t + 8 * a) = y;
            }
    }
    // the bf16 plane: each wave's 32 x 64 dK and dV tiles staged through LDS (rows of FBB_DKS; the K^T / dS / Q / dO
    // images are free once every wave is past the last tile's dQ reads) and stored as whole 128-B rows, 16 B per lane
    // (the accumulator layout gave 8-byte stores one 6-KB row apart: ~0.1 ms of a 0.8-ms C4 layer backward,
    // tools/attn_bench SUTA_FB_DIAG=128)
    if (!(DG & 128) && dqkvb) {
        static_assert(FBB_NW * 2 * 32 * FBB_DKS <= 64 * FBB_KB + 2 * FBB_NW * 32 * FBS_RS + 4 * 32 * FB_RS,
                      "dK / dV staging must fit the K^T, dS and Q / dO images");
        __syncthreads();
        __bf16* const stk = sm16 + w * 2 * 32 * FBB_DKS;  // this wave's dK image [32][FBB_DKS], then its dV image
        __bf16* const stv = stk + 32 * FBB_DKS;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                fbf16x4 x, y;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    x[b] = (__bf16)dk[t][4 * a + b];
                    y[b] = (__bf16)dv[t][4 * a + b];
                }
                *reinterpret_cast<fbf16x4*>(stk + l32 * FBB_DKS + 32 * t + 8 * a + 4 * h) = x;
                *reinterpret_cast<fbf16x4*>(stv + l32 * FBB_DKS + 32 * t + 8 * a + 4 * h) = y;
            }
        __syncthreads();
        if (w < ngb) {
            __bf16* const ob = dqkvb + (long)u * T * ld + H + hd * 64;
#pragma unroll
            for (int it = 0; it < 4; ++it) {  // 8 rows x 8 chunks of 16 B per instruction
                const int r = 8 * it + (lane >> 3), c8 = (lane & 7) * 8, k2 = kbase + 32 * w + r;
                const fbf16x8 x = *reinterpret_cast<const fbf16x8*>(stk + r * FBB_DKS + c8);
                const fbf16x8 y = *reinterpret_cast<const fbf16x8*>(stv + r * FBB_DKS + c8);
                if (k2 < T) {
                    *reinterpret_cast<fbf16x8*>(ob + ((unsigned)k2 * (unsigned)ld + c8)) = x;
                    *reinterpret_cast<fbf16x8*>(ob + ((unsigned)k2 * (unsigned)ld + H + c8)) = y;
                }
            }
        }
    }
}

// dQ = sum over key blocks in order (query rows < tl; rows past it get 0, as their dS is 0).  Row-layout partials
// (flash_bwd_kernel, flash_bwd_bf16_kernel): one thread per 4 columns of a row.
__global__ __launch_bounds__(256) void flash_dq_reduce(const float* __restrict__ dqp, float* __restrict__ dqkv, int B,
                                                       int T, int NH, int H, int nkb, const int* __restrict__ tlen,
                                                       __bf16* __restrict__ dqkvb) {
    const long n4 = (long)B * NH * T * 16;
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const int c4 = (int)(i & 15) * 4;
    const long row = i >> 4;  // (u * NH + hd) * T + q
    const int q = (int)(row % T);
    const long bh = row / T;
    const int hd = (int)(bh % NH), u = (int)(bh / NH);
    const int tl = tlen ? tlen[u] : T;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    if (q < tl) {
        const long stride = (long)B * NH * T * 64;
        const f32x4* p = reinterpret_cast<const f32x4*>(dqp + row * 64 + c4);
        for (int k = 0; k < nkb; ++k) s += p[k * (stride / 4)];
    }
    if (dqkv) *reinterpret_cast<f32x4*>(dqkv + ((long)u * T + q) * 3 * H + hd * 64 + c4) = s;
    if (dqkvb) {
        fbf16x4 b;
#pragma unroll
        for (int e = 0; e < 4; ++e) b[e] = (__bf16)s[e];
        *reinterpret_cast<fbf16x4*>(dqkvb + ((long)u * T + q) * 3 * H + hd * 64 + c4) = b;
    }
}

// The same for the fragment-order partials of flash_bwd_bf16p_kernel ([kb][B * NH][NQT][8 waves][64 lanes][4]: lane
// (g, l16) of wave w = qi + 2 di holds rows 16 qi + 4 g + 0..3, column 16 di + l16 of its 32 x 64 tile): one block per
// (head, query tile) sums the key blocks' 8-KB tiles in key-block order (per element the row-layout pass's order, so
// the results are bitwise the same), transposes them through LDS and writes the tile's dQ rows whole.
__global__ __launch_bounds__(256) void flash_dq_reduce_frag(const float* __restrict__ dqp, float* __restrict__ dqkv,
                                                            int B, int T, int NH, int H, int nkb,
                                                            const int* __restrict__ tlen, __bf16* __restrict__ dqkvb) {
    __shared__ __attribute__((aligned(16))) float tile[32][64 + 4];
    const int NQT = (T + 31) >> 5;
    const long bt = blockIdx.x;  // bh * NQT + qt
    const int qt = (int)(bt % NQT);
    const long bh = bt / NQT;
    const int hd = (int)(bh % NH), u = (int)(bh / NH);
    const int tl = tlen ? tlen[u] : T;
    const int q0 = qt * 32;
    if (q0 < tl) {  // (block-uniform)
        const long stride = (long)B * NH * NQT * 2048;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            const int f = half * 256 + threadIdx.x;  // fragment = wave * 64 + lane
            const f32x4* p = reinterpret_cast<const f32x4*>(dqp + bt * 2048) + f;
            f32x4 s = {0.f, 0.f, 0.f, 0.f};
            for (int k = 0; k < nkb; ++k) s += p[k * (stride / 4)];
            const int wv = f >> 6, ln = f & 63, qi = wv & 1, di = wv >> 1, g = ln >> 4, l16 = ln & 15;
#pragma unroll
            for (int r = 0; r < 4; ++r) tile[16 * qi + 4 * g + r][16 * di + l16] = s[r];
        }
    }
    __syncthreads();
    // 32 rows x 64 columns: thread -> row threadIdx / 8, columns (threadIdx % 8) * 8 .. + 7
    const int r = threadIdx.x >> 3, c8 = (threadIdx.x & 7) * 8, q = q0 + r;
    if (q >= T) return;
    f32x4 lo = {0.f, 0.f, 0.f, 0.f}, hi = {0.f, 0.f, 0.f, 0.f};
    if (q < tl) {
        lo = *reinterpret_cast<const f32x4*>(&tile[r][c8]);
        hi = *reinterpret_cast<const f32x4*>(&tile[r][c8 + 4]);
    }
    const long o = ((long)u * T + q) * 3 * H + hd * 64 + c8;
    if (dqkv) {
        *reinterpret_cast<f32x4*>(dqkv + o) = lo;
        *reinterpret_cast<f32x4*>(dqkv + o + 4) = hi;
    }
    if (dqkvb) *reinterpret_cast<fbf16x8*>(dqkvb + o) = cvt8(lo, hi);
}

}  // namespace

constexpr int FF_NW = 4;

// backward block width: 4 or 8 waves (env SUTA_FLASH_BWD_NW, default 8), read once (thread-safe initialisation)
static int fb_nw() {
    static const int nw = [] {
        const char* e = std::getenv("SUTA_FLASH_BWD_NW");
        return (e && atoi(e) == 4) ? 4 : 8;
    }();
    return nw;
}

// bf16 mode: LDS images in bf16 (flash_*_bf16_kernel; env SUTA_FLASH_BF16_IMG=0 selects the fp32-image
// instantiations for A/B runs; from the call's switch snapshot, common.h SutaSwitches)
static bool fb_img() { return suta_switches().flash_bf16_img != 0; }

long flash_dq_scratch_floats(int B, int T, int NH) {
    const int ng = (T + 31) / 32, nkb = (ng + fb_nw() - 1) / fb_nw();
    // the per-key-block dQ partials (row layout: T rows per head; fragment layout of the bf16-plane kernel: whole
    // 32-row query tiles)
    return (long)nkb * B * NH * ((T + 31) / 32) * 32 * 64 + 64;
}

// bf16 mode, bf16 qkv plane given: flash_fwd_bf16p_kernel (env SUTA_FLASH_FWD_PLANE=0 keeps the fp32-row
// kernels for A/B runs; from the call's switch snapshot)
static bool ff_plane() { return suta_switches().flash_fwd_plane != 0; }

bool flash_fwd_reads_plane(bool bf16, const void* qkvb, int H) { return bf16 && qkvb && H % 8 == 0 && ff_plane(); }

bool launch_flash_fwd(const float* qkv, float* ctx, float* lse, int B, int T, int NH, int H, int dh, float scale,
                      const int* tlen, bool bf16, hipStream_t st, void* ctxb_, const void* qkvb) {
    __bf16* ctxb = reinterpret_cast<__bf16*>(ctxb_);
    if (dh != 64 || T < 1 || H % 4) return false;
    const int ng = (T + 31) / 32, nqb = (ng + FF_NW - 1) / FF_NW;
    const dim3 grid((unsigned)((long)B * NH * nqb));
    const bool on_plane = flash_fwd_reads_plane(bf16, qkvb, H);
    if (!qkv && !on_plane) throw std::invalid_argument("flash_fwd: fp32 qkv not written and the plane kernel not taken");
    if (on_plane) {
        if (reinterpret_cast<uintptr_t>(qkvb) & 15) throw std::invalid_argument("flash_fwd: bf16 qkv plane not 16-B aligned");
        // SUTA_FLASH_FWD_NW=8: 8-wave blocks (256 queries share each K / V tile copy); switch snapshot
        if (suta_switches().flash_fwd_nw == 8) {
            const int nqb8 = (ng + 7) / 8;
            hipLaunchKernelGGL(flash_fwd_bf16p_kernel<8>, dim3((unsigned)((long)B * NH * nqb8)), dim3(512), 0, st,
                               reinterpret_cast<const __bf16*>(qkvb), ctx, lse, T, NH, H, scale, tlen, nqb8, ctxb);
        } else {
            hipLaunchKernelGGL(flash_fwd_bf16p_kernel<FF_NW>, grid, dim3(FF_NW * 64), 0, st,
                               reinterpret_cast<const __bf16*>(qkvb), ctx, lse, T, NH, H, scale, tlen, nqb, ctxb);
        }
    } else if (bf16 && fb_img()) {
        static_assert(FF_NW_BF == FF_NW, "the bf16 forward shares the query-block grid");
        hipLaunchKernelGGL(flash_fwd_bf16_kernel, grid, dim3(FF_NW_BF * 64), 0, st, qkv, ctx, lse, T, NH, H, scale,
                           tlen, nqb, ctxb);
    } else if (bf16)
        hipLaunchKernelGGL((flash_fwd_kernel<FF_NW, true>), grid, dim3(FF_NW * 64), 0, st, qkv, ctx, lse, T, NH, H,
                           scale, tlen, nqb, ctxb);
    else
        hipLaunchKernelGGL((flash_fwd_kernel<FF_NW, false>), grid, dim3(FF_NW * 64), 0, st, qkv, ctx, lse, T, NH, H,
                           scale, tlen, nqb, ctxb);
    return true;
}

template <int NW, bool BF16>
static void flash_bwd_go(dim3 grid, hipStream_t st, const float* qkv, const float* dctx, const float* lse,
                         const float* delta, float* dqkv, float* dqp, int T, int NH, int H, float scale,
                         const int* tlen, int nkb, int gpb, int B, __bf16* dqkvb) {
    constexpr size_t lds = fb_lds_bytes<NW>();
    set_max_lds_once(reinterpret_cast<const void*>(&flash_bwd_kernel<NW, BF16>), lds, "flash_bwd_kernel");
    hipLaunchKernelGGL((flash_bwd_kernel<NW, BF16>), grid, dim3(NW * 64), lds, st, qkv, dctx, lse, delta, dqkv, dqp,
                       T, NH, H, scale, tlen, nkb, gpb, B, dqkvb);
}

template <int DG = 0>
static void flash_bwd_bf16p_go(dim3 grid, hipStream_t st, const void* qkvb, const void* dctxb, const float* lse,
                               const float* delta, float* dqkv, float* dqp, int T, int NH, int H, float scale,
                               const int* tlen, int nkb, int gpb, int B, __bf16* dqkvb) {
#ifdef SUTA_FB_DIAG
    if constexpr (DG == 0) {  // tools build: SUTA_FB_DIAG=<bits> selects a diagnostic form (wrong results)
        const char* e = std::getenv("SUTA_FB_DIAG");
        const int dg = e ? atoi(e) : 0;
#define FBD(D_) if (dg == D_) return flash_bwd_bf16p_go<D_>(grid, st, qkvb, dctxb, lse, delta, dqkv, dqp, T, NH, H, scale, tlen, nkb, gpb, B, dqkvb)
        FBD(1); FBD(2); FBD(4); FBD(8); FBD(16); FBD(32); FBD(3); FBD(7); FBD(15); FBD(31); FBD(63); FBD(14); FBD(6);
        FBD(64); FBD(128); FBD(127); FBD(191); FBD(255);
#undef FBD
    }
#endif
    constexpr size_t lds = fbbp_lds_bytes();
    set_max_lds_once(reinterpret_cast<const void*>(&flash_bwd_bf16p_kernel<DG>), lds, "flash_bwd_bf16p_kernel");
    hipLaunchKernelGGL((flash_bwd_bf16p_kernel<DG>), grid, dim3(FBB_NW * 64), lds, st,
                       reinterpret_cast<const __bf16*>(qkvb), reinterpret_cast<const __bf16*>(dctxb), lse, delta, dqkv,
                       dqp, T, NH, H, scale, tlen, nkb, gpb, B, dqkvb);
}

// bf16 mode, bf16 planes of qkv and dctx given: flash_bwd_bf16p_kernel (env SUTA_FLASH_BWD_PLANE=0 keeps the
// fp32-row kernels for A/B runs; from the call's switch snapshot)
static bool fb_plane() { return suta_switches().flash_bwd_plane != 0; }

bool flash_bwd_reads_planes(bool bf16, const void* qkvb, const void* dctxb, int H) {
    return bf16 && fb_nw() == FBB_NW && qkvb && dctxb && H % 8 == 0 && fb_plane();
}

bool launch_flash_bwd(const float* qkv, const float* dctx, const float* lse, const float* delta, float* dqkv,
                      float* dqp, int B, int T, int NH, int H, int dh, float scale, const int* tlen, bool bf16,
                      hipStream_t st, void* dqkvb_, const void* qkvb, const void* dctxb) {
    __bf16* dqkvb = reinterpret_cast<__bf16*>(dqkvb_);
    if (dh != 64 || T < 1 || H % 4) return false;
    const int nw = fb_nw();
    const int ng = (T + 31) / 32;
    const int nkb = (ng + nw - 1) / nw;   // key blocks per head
    const int gpb = (ng + nkb - 1) / nkb;  // key groups per block (balanced)
    const dim3 grid((unsigned)((long)B * NH * nkb));
    const bool on_planes = flash_bwd_reads_planes(bf16, qkvb, dctxb, H);
    if (!qkv && !on_planes) throw std::invalid_argument("flash_bwd: fp32 qkv not written and the plane kernel not taken");
    if (on_planes) {
        if ((reinterpret_cast<uintptr_t>(qkvb) | reinterpret_cast<uintptr_t>(dctxb)) & 15)
            throw std::invalid_argument("flash_bwd: bf16 planes not 16-B aligned");
        flash_bwd_bf16p_go(grid, st, qkvb, dctxb, lse, delta, dqkv, dqp, T, NH, H, scale, tlen, nkb, gpb, B, dqkvb);
        hipLaunchKernelGGL(flash_dq_reduce_frag, dim3((unsigned)((long)B * NH * ((T + 31) / 32))), dim3(256), 0, st, dqp,
                           dqkv, B, T, NH, H, nkb, tlen, dqkvb);
        return true;
    } else if (bf16 && nw == FBB_NW && fb_img()) {
        constexpr size_t lds = fbb_lds_bytes();
        set_max_lds_once(reinterpret_cast<const void*>(&flash_bwd_bf16_kernel), lds, "flash_bwd_bf16_kernel");
        hipLaunchKernelGGL(flash_bwd_bf16_kernel, grid, dim3(FBB_NW * 64), lds, st, qkv, dctx, lse, delta, dqkv, dqp,
                           T, NH, H, scale, tlen, nkb, gpb, B, dqkvb);
    } else {
        // flash_bwd_kernel: dQ partials in fragment order, as the bf16-plane kernel's
        if (nw == 4) {
            if (bf16) flash_bwd_go<4, true>(grid, st, qkv, dctx, lse, delta, dqkv, dqp, T, NH, H, scale, tlen, nkb, gpb, B, dqkvb);
            else flash_bwd_go<4, false>(grid, st, qkv, dctx, lse, delta, dqkv, dqp, T, NH, H, scale, tlen, nkb, gpb, B, dqkvb);
        } else {
            if (bf16) flash_bwd_go<8, true>(grid, st, qkv, dctx, lse, delta, dqkv, dqp, T, NH, H, scale, tlen, nkb, gpb, B, dqkvb);
            else flash_bwd_go<8, false>(grid, st, qkv, dctx, lse, delta, dqkv, dqp, T, NH, H, scale, tlen, nkb, gpb, B, dqkvb);
        }
        hipLaunchKernelGGL(flash_dq_reduce_frag, dim3((unsigned)((long)B * NH * ((T + 31) / 32))), dim3(256), 0, st, dqp,
                           dqkv, B, T, NH, H, nkb, tlen, dqkvb);
        return true;
    }
    const long n4 = (long)B * NH * T * 16;
    hipLaunchKernelGGL(flash_dq_reduce, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, dqp, dqkv, B, T, NH, H,
                       nkb, tlen, dqkvb);
    return true;
}
