// 256 x 256 bf16-plane GEMM with a slice ring and reads one slice ahead ("hbx"; SUTA_PRECISION_BF16 linears).
//
// Same operands and epilogue as gemm_hb_kernel (A [M][K], B [N][K] bf16 planes, k-contiguous; fp32 accumulation;
// the shared fp32 / bf16-C epilogue), different main loop:
//   * one block of 8 waves per CU (2 along M x 4 along N), wave tile 128 x 64: 2x the MFMA work per LDS byte of
//     the 128 x 128 tile (the bf16 operand stream through L2 -> LDS is what bounds the 128 x 128 kernel);
//   * 32-deep K slices in a ring of NR = 4 LDS slots (32 KB each: A 256 x 32 + B 256 x 32 bf16), filled by LDS-DMA
//     three slices ahead of the one being consumed, retired by a counted vmcnt that leaves the newest slice in
//     flight across the barrier (never vmcnt(0) in the loop);
//   * ONE barrier per slice, and the fragments of slice s+1 are read into a second register set while the MFMAs of
//     slice s run (the reads, the DMA issue and the MFMAs interleaved by sched_group_barrier), so no MFMA waits on
//     an LDS read issued in its own slice.
// Hazards (slice s in ring slot s % 4):
//   RAW -- a wave reads slice s+1 only after barrier B_s, which every wave passes after its own counted wait for
//          its DMA share of slice s+1;
//   WAR -- slice s+3 is DMA'd into slot (s+3) % 4 = (s-1) % 4 right after B_s; slice s-1's fragments were read
//          during iteration s-2 and consumed by the MFMAs of iteration s-1, which every wave finished before B_s.
// LDS image: rows of 64 B (32 bf16 = four 16-B chunks); chunk c of row r sits in slot c ^ g((r >> 2) & 3),
// g = {0, 2, 3, 1}, applied to the per-lane DMA SOURCE address (LDS-DMA writes are lane-linear).  Conflict-free
// for the ds_read_b128 lane groups of both MFMA shapes (32x32x16: lane -> row l & 31, chunk 2 kc + (l >> 5);
// 16x16x32: row l & 15, chunk l >> 4): the 16 lanes of a group land on 16 distinct 16-B bank slots.
// MS: MFMA shape, 32 (v_mfma_f32_32x32x16_bf16, the epilogue's fragment form) or 16 (v_mfma_f32_16x16x32_bf16).
// Requires K % 32 == 0 and K >= 128, no split-K, no conv-A rows, and Z == 1 except on the four-phase form
// (gemm_hbp_kernel below, K % 64 == 0), which rebases its operands per batch (the dispatcher's conditions).
#include "gemm_kernels.h"
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <type_traits>

namespace {

constexpr int X_BM = 256, X_BN = 256, X_KS = 16;  // slice depth in 4-byte units (32 bf16)
constexpr int X_NR = 4;                           // ring slots
constexpr int X_NWV = 8;
constexpr int X_SLOT = (X_BM + X_BN) * X_KS;      // 4-byte units per slot (32 KB)
constexpr int X_NPW = (X_BM + X_BN) * X_KS / (256 * X_NWV);  // DMA instructions per wave per slice (4)

__device__ __forceinline__ int hbx_swz(int row) {
    const int q = (row >> 2) & 3;
    return (0x1320 >> (4 * q)) & 3;  // g = {0, 2, 3, 1}
}

// per-lane DMA sources of one operand (ROWS rows of the tile): NI = ROWS * KS / (256 * NWV) pieces per wave
template <int ROWS>
struct XStream {
    static constexpr int NI = ROWS * X_KS / (256 * X_NWV);
    const float* ptr[NI];
    int inc[NI];
    __device__ __forceinline__ void init(const float* __restrict__ src, long ld, int row0, int nrows, int w, int lane) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int ci = i * X_NWV + w;  // 1-KiB piece of the operand's slice image = 16 rows
            const int row = ci * 16 + lane / 4;
            const int c = (lane & 3) ^ hbx_swz(row);
            const bool ok = row0 + row < nrows;
            ptr[i] = ok ? src + (long)(row0 + row) * ld + c * 4 : g_zero16;
            inc[i] = ok ? X_KS : 0;
        }
    }
};

template <int ROWS>
__device__ __forceinline__ void xstream_issue(XStream<ROWS>& sm, float* dst, int w) {
#pragma unroll
    for (int i = 0; i < XStream<ROWS>::NI; ++i) {
        const float* g = sm.ptr[i];
        __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)(dst + (i * X_NWV + w) * 256), 16, 0, 0);
        sm.ptr[i] = g + sm.inc[i];
    }
}

// 16 B of row `row`, chunk c (8 bf16 at k = 8c..8c+7 of the slice)
__device__ __forceinline__ bf16x8 xfrag(const float* lds, int row, int c) {
    return *reinterpret_cast<const bf16x8*>(lds + row * X_KS + ((c ^ hbx_swz(row)) * 4));
}

// one 16-deep k-chunk of a slice (MS 32: A 4 row blocks, B 2; MS 16: one 32-deep slice's half -- A 4 row blocks of
// 16, B 4 column blocks of 16, the m-half `hm` of the wave tile)
template <int MS>
struct XFr;
template <>
struct XFr<32> {
    bf16x8 a[4], b[2];
};
template <>
struct XFr<16> {
    bf16x8 a[4], b[4];
};

// Epilogue of 16x16 accumulator fragments (v_mfma_f32_16x16x32_bf16: register r of acc[i][j] is row 16 i + 4 (lane >> 4)
// + r, column 16 j + (lane & 15) of the wave tile).  The flags of the bf16 linears (bias, residual, bias + GELU +
// pre-activation store, GELU', ragged row mask; fp32 C and / or the bf16 C plane; bf16 pre-activation operands) with
// the same operations in the same order as gemm_epilogue; interior tiles with 32-bit offsets (scalar row bases +
// one lane offset per fragment), edge tiles element by element with bounds checks.  No split-K, ACCUM or SMBWD
// (gemm_run_hbx checks).
template <int FM, int FN, bool CB, int EM>
__device__ __forceinline__ void epilogue16(const GemmParams& p, const f32x4 (&acc)[FM][FN], int rbase, int cbase,
                                           int lane, bool interior) {
    const int e = p.epi & EM;
    const int q4 = lane >> 4, l16 = lane & 15;
    float* C = p.C;
    const float* bias = p.bias;
    const float* R = p.R;
    const int rlim = (e & EPI_ROWMASK) ? p.zrows[0] : 0x7fffffff;
    const bool preb = CB && p.preb;
    const float alpha = p.alpha;
    typedef __bf16 cb2 __attribute__((ext_vector_type(2)));
    const bool odd = lane & 1;
    __bf16* Cb = CB ? reinterpret_cast<__bf16*>(p.Cb) : nullptr;
    const bool fast = interior && p.off32 && (!CB || (p.ldcb & 1) == 0) && (!preb || (p.ldc2 & 1) == 0);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            const int rb = rbase + 16 * i + 4 * q4;
            const int col = cbase + 16 * j + l16;
            float v[4], xa[4], xr[4];
            if (fast) {
                const unsigned uc = (unsigned)col;
                if (e & EPI_DGELU) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        xa[r] = preb ? (float)*byte_at(reinterpret_cast<const __bf16*>(p.aux) + (long)(rb + r) * p.ldaux, 2u * uc)
                                     : *byte_at(p.aux + (long)(rb + r) * p.ldaux, 4u * uc);
                }
                if (e & EPI_RESID) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) xr[r] = *byte_at(R + (long)(rb + r) * p.ldr, 4u * uc);
                }
            } else {
                const int cc = min(col, p.N - 1);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const long row = min(rb + r, p.M - 1);
                    if (e & EPI_DGELU)
                        xa[r] = preb ? (float)reinterpret_cast<const __bf16*>(p.aux)[row * p.ldaux + cc] : p.aux[row * p.ldaux + cc];
                    if (e & EPI_RESID) xr[r] = R[row * p.ldr + cc];
                }
            }
            const float bj = (e & EPI_BIAS) ? bias[min(col, p.N - 1)] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                v[r] = acc[i][j][r] * alpha;
                if (e & EPI_BIAS) v[r] += bj;
            }
            if (e & EPI_STORE_PRE) {
                if (preb && fast) {  // (column, column + 1) bf16 pairs: lanes 2i / 2i + 1 swap one value
#pragma unroll
                    for (int r = 0; r < 4; r += 2) {
                        const float a = v[r], b = v[r + 1];
                        const float q = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(odd ? a : b), 0xB1, 0xF, 0xF, false));
                        cb2 pr;
                        pr[0] = (__bf16)(odd ? q : a);
                        pr[1] = (__bf16)(odd ? b : q);
                        *reinterpret_cast<cb2*>(byte_at(reinterpret_cast<__bf16*>(p.C2) + (long)(rb + r + (odd ? 1 : 0)) * p.ldc2,
                                                        2u * (unsigned)(col & ~1))) = pr;
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (interior || (rb + r < p.M && col < p.N)) {
                            if (preb) reinterpret_cast<__bf16*>(p.C2)[(long)(rb + r) * p.ldc2 + col] = (__bf16)v[r];
                            else p.C2[(long)(rb + r) * p.ldc2 + col] = v[r];
                        }
                }
            }
            if ((e & EPI_GELU) && CB && p.fgelu) {  // (uniform choice hoisted out of the element loop)
#pragma unroll
                for (int r = 0; r < 4; r += 2) {
                    const f32x2v g = gelu2_bf16ep(f32x2v{v[r], v[r + 1]});
                    v[r] = g.x;
                    v[r + 1] = g.y;
                }
            } else if (e & EPI_GELU) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = gelu_f(v[r]);
            }
            if ((e & EPI_DGELU) && CB && p.fgelu) {
#pragma unroll
                for (int r = 0; r < 4; r += 2) {
                    const f32x2v g = dgelu2_bf16ep(f32x2v{xa[r], xa[r + 1]});
                    v[r] *= g.x;
                    v[r + 1] *= g.y;
                }
            } else if (e & EPI_DGELU) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] *= dgelu_f(xa[r]);
            }
            if (e & EPI_RESID) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] += xr[r];
            }
            if (e & EPI_ROWMASK) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (rb + r >= rlim) v[r] = 0.f;
            }
            if (C) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if (fast) *byte_at(C + (long)(rb + r) * p.ldc, 4u * (unsigned)col) = v[r];
                    else if (rb + r < p.M && col < p.N) C[(long)(rb + r) * p.ldc + col] = v[r];
                }
            }
            if (CB) {
                if (fast) {
#pragma unroll
                    for (int r = 0; r < 4; r += 2) {
                        const float a = v[r], b = v[r + 1];
                        const float q = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(odd ? a : b), 0xB1, 0xF, 0xF, false));
                        cb2 pr;
                        pr[0] = (__bf16)(odd ? q : a);
                        pr[1] = (__bf16)(odd ? b : q);
                        *reinterpret_cast<cb2*>(byte_at(Cb + (long)(rb + r + (odd ? 1 : 0)) * p.ldcb, 2u * (unsigned)(col & ~1))) = pr;
                    }
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (rb + r < p.M && col < p.N) Cb[(long)(rb + r) * p.ldcb + col] = (__bf16)v[r];
                }
            }
        }
}

// Row-per-lane epilogue of the transposed accumulators (TR: the MFMAs take B as their first operand, so acc[i][j]
// holds C^T: lane l carries row 32 i + (l & 31) of the wave tile, register r = 4 g + k its column 32 j + 8 g +
// 4 (l >> 5) + k).  Each lane holds runs of 4 consecutive columns; v_permlane32_swap pairs the half-waves' runs of
// column groups (g, g + 1) into 16 contiguous bytes per lane (cdna_hip_programming.md T21), so every bf16 plane
// (C plane, pre-activation store, GELU' operand) moves in 16-B accesses and fp32 operands in float4s: 16 store
// instructions per bf16 plane per wave instead of 128 two-lane-pair dword stores.  Same operations in the same order
// as gemm_epilogue (elementwise; packed GELU pairs are lane-independent).  Rows past M are predicated per lane;
// column tiles past N take the element-wise path.  gemm_run_hbx checks alignment (16-B bases, ld % 8 for the bf16
// planes, % 4 for the fp32 ones) and off32 before choosing this form.
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
    bf16x2v t;
    t[0] = (__bf16)a;
    t[1] = (__bf16)b;
    return __builtin_bit_cast(unsigned, t);
}
__device__ __forceinline__ float bf16_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

// runs (g0, g0 + 1) of 4 bf16 each (x0 = cols 0-1, y0 = cols 2-3 of run g0; x1, y1 of run g0 + 1) <-> one 16-B chunk
// per lane (lower half-wave: cols 8 g0 .. 8 g0 + 7, upper: 8 g0 + 8 .. 8 g0 + 15); the exchange is its own inverse
__device__ __forceinline__ void swap_runs(unsigned& x0, unsigned& y0, unsigned& x1, unsigned& y1) {
    auto rx = __builtin_amdgcn_permlane32_swap(x0, x1, false, false);
    auto ry = __builtin_amdgcn_permlane32_swap(y0, y1, false, false);
    x0 = rx[0];
    x1 = rx[1];
    y0 = ry[0];
    y1 = ry[1];
}

// column tiles past N: element by element (same arithmetic, bounds-checked stores)
template <bool CB, int EM>
__device__ __forceinline__ void epilogue_t_edge(const GemmParams& p, const f32x16 (&acc)[4][2], int rbase, int cbase,
                                                int lane) {
    const int e = p.epi & EM;
    const int h = lane >> 5, l32 = lane & 31;
    const int rlim = (e & EPI_ROWMASK) ? p.zrows[0] : 0x7fffffff;
    const bool preb = CB && p.preb;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = rbase + 32 * i + l32;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int col = cbase + 32 * j + 8 * (r >> 2) + 4 * h + (r & 3);
                if (row >= p.M || col >= p.N) continue;
                float v = acc[i][j][r] * p.alpha;
                if (e & EPI_BIAS) v += p.bias[col];
                if (e & EPI_STORE_PRE) {
                    if (preb) reinterpret_cast<__bf16*>(p.C2)[(long)row * p.ldc2 + col] = (__bf16)v;
                    else p.C2[(long)row * p.ldc2 + col] = v;
                }
                if (e & EPI_GELU) v = (CB && p.fgelu) ? gelu2_bf16ep(f32x2v{v, v}).x : gelu_f(v);
                if (e & EPI_DGELU) {
                    const float xa = preb ? (float)reinterpret_cast<const __bf16*>(p.aux)[(long)row * p.ldaux + col]
                                          : p.aux[(long)row * p.ldaux + col];
                    v *= (CB && p.fgelu) ? dgelu2_bf16ep(f32x2v{xa, xa}).x : dgelu_f(xa);
                }
                if (e & EPI_RESID) v += p.R[(long)row * p.ldr + col];
                if (row >= rlim) v = 0.f;
                if (!CB || p.C) p.C[(long)row * p.ldc + col] = v;
                if (CB) reinterpret_cast<__bf16*>(p.Cb)[(long)row * p.ldcb + col] = (__bf16)v;
            }
    }
}

// ST (staged): the 32-row band i of each output plane goes through a wave-private LDS image (the slice ring, free
// after the main loop) and leaves in full 128-B lines: 16-B chunks written per lane as the fragments hold them
// (chunk c of row r in slot c ^ (r & 7): conflict-free ds_write_b128 / ds_read_b128), read back row-contiguous
// (8 lanes = one 128-B bf16 row of the wave tile, 16 lanes = one 256-B fp32 row) and stored with every lane of an
// instruction in 8 whole lines.  Without ST a store instruction touches 32 rows.
template <bool CB, int EM, bool ST, int NOST = 0, bool NT = false>
__device__ __forceinline__ void epilogue_t(const GemmParams& p, const f32x16 (&acc)[4][2], int rbase, int cbase,
                                           int lane, char* stage) {
    if (cbase + 64 > p.N) {
        epilogue_t_edge<CB, EM>(p, acc, rbase, cbase, lane);
        return;
    }
    // staging images per wave (bytes): bf16 pre-activation 4 KB, fp32 C 8 KB, bf16 C plane 4 KB
    char* const s_pre = stage;
    char* const s_c32 = stage + 4096;
    char* const s_cb = stage + 12288;
    const bool st_pre = ST && (p.epi & EM & EPI_STORE_PRE) && CB && p.preb;
    const bool st_c32 = ST && (!CB || p.C);
    const int e = p.epi & EM;
    const int h = lane >> 5, l32 = lane & 31;
    const float alpha = p.alpha;
    const int rlim = (e & EPI_ROWMASK) ? p.zrows[0] : 0x7fffffff;
    const bool preb = CB && p.preb;
    // one bf16 plane's 8 values of runs (2q, 2q + 1) as one 16-B chunk per lane: to global (d) or to the staging
    // image (img, chunk c of row l32)
    auto store_bf16 = [&](__bf16* d, const float* v, bool rok, char* img, int c) {
        unsigned x0 = pack_bf16x2(v[0], v[1]), y0 = pack_bf16x2(v[2], v[3]);
        unsigned x1 = pack_bf16x2(v[4], v[5]), y1 = pack_bf16x2(v[6], v[7]);
        swap_runs(x0, y0, x1, y1);
        if (img) *reinterpret_cast<u32x4v*>(img + l32 * 128 + ((c ^ (l32 & 7)) << 4)) = u32x4v{x0, y0, x1, y1};
        else if (rok) *reinterpret_cast<u32x4v*>(d) = u32x4v{x0, y0, x1, y1};
    };
    // staged band i -> global: bf16 images 4 rows... 8 rows x 128 B per instruction, fp32 4 rows x 256 B
    auto flush_bf16 = [&](const char* img, __bf16* base, long ld, int row0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int r = 8 * k + (lane >> 3), c = lane & 7;
            const u32x4v w = *reinterpret_cast<const u32x4v*>(img + r * 128 + ((c ^ (r & 7)) << 4));
            if constexpr (NOST != 0) asm volatile("" ::"v"(w));  // (tools diagnostics: no global store)
            else if (row0 + r < p.M) {
                u32x4v* d = reinterpret_cast<u32x4v*>(base + (long)(row0 + r) * ld + cbase + 8 * c);
                if constexpr (NT) __builtin_nontemporal_store(w, d);
                else *d = w;
            }
        }
    };
    auto flush_f32 = [&](const char* img, float* base, long ld, int row0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int r = 4 * k + (lane >> 4), c = lane & 15;
            const f32x4 w = *reinterpret_cast<const f32x4*>(img + r * 256 + ((c ^ (r & 7)) << 4));
            if (row0 + r < p.M) {
                f32x4* d = reinterpret_cast<f32x4*>(base + (long)(row0 + r) * ld + cbase + 4 * c);
                if constexpr (NT) __builtin_nontemporal_store(w, d);
                else *d = w;
            }
        }
    };
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // GELU' / residual operands one band ahead (issued once band i has consumed its own, before band i's stores: a wait
    // for them never covers those stores; as epilogue16t)
    struct OpsT {
        u32x4v a[2][2];    // GELU' operand of the bf16 pre-activation plane (the 16 B of the run pair; an fp32
                           // operand is loaded where it is used)
        f32x4 r[2][2][2];  // residual [j][q][t]
    };
    auto load_ops = [&](int i, OpsT& o) {
        const long rowc = min(rbase + 32 * i + l32, p.M - 1);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int nb = cbase + 32 * j + 16 * q;
                if ((e & EPI_DGELU) && preb)
                    o.a[j][q] = *reinterpret_cast<const u32x4v*>(reinterpret_cast<const __bf16*>(p.aux) + rowc * p.ldaux +
                                                                 nb + 8 * h);
                if (e & EPI_RESID) {
#pragma unroll
                    for (int t = 0; t < 2; ++t)
                        o.r[j][q][t] = *reinterpret_cast<const f32x4*>(p.R + rowc * p.ldr + nb + 8 * t + 4 * h);
                }
            }
    };
    OpsT o;
    if (e & (EPI_DGELU | EPI_RESID)) load_ops(0, o);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = rbase + 32 * i + l32;
        const long rowc = min(row, p.M - 1);
        const bool rok = row < p.M;
        const bool zero = (e & EPI_ROWMASK) && row >= rlim;
        float sg[4];  // EPI_DELTA: the lane's 4-column dot products, summed over j (attn_delta_kernel's first level)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 2; ++q) {  // runs 2q, 2q + 1: columns nb .. nb + 15 of the block
                const int nb = cbase + 32 * j + 16 * q;
                float v[8], xa[8], xr[8];
                if (e & EPI_DGELU) {
                    if (preb) {
                        const u32x4v w = o.a[j][q];
                        unsigned x0 = w[0], y0 = w[1], x1 = w[2], y1 = w[3];
                        swap_runs(x0, y0, x1, y1);
                        xa[0] = bf16_lo(x0); xa[1] = bf16_hi(x0); xa[2] = bf16_lo(y0); xa[3] = bf16_hi(y0);
                        xa[4] = bf16_lo(x1); xa[5] = bf16_hi(x1); xa[6] = bf16_lo(y1); xa[7] = bf16_hi(y1);
                    } else {
#pragma unroll
                        for (int t = 0; t < 2; ++t) {
                            const f32x4 w = *reinterpret_cast<const f32x4*>(p.aux + rowc * p.ldaux + nb + 8 * t + 4 * h);
#pragma unroll
                            for (int k = 0; k < 4; ++k) xa[4 * t + k] = w[k];
                        }
                    }
                }
                if (e & EPI_RESID) {
#pragma unroll
                    for (int t = 0; t < 2; ++t)
#pragma unroll
                        for (int k = 0; k < 4; ++k) xr[4 * t + k] = o.r[j][q][t][k];
                }
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    f32x4 bj = {0.f, 0.f, 0.f, 0.f};
                    if (e & EPI_BIAS) bj = *reinterpret_cast<const f32x4*>(p.bias + nb + 8 * t + 4 * h);
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        v[4 * t + k] = acc[i][j][8 * q + 4 * t + k] * alpha;
                        if (e & EPI_BIAS) v[4 * t + k] += bj[k];
                    }
                }
                if (e & EPI_STORE_PRE) {
                    if (preb)
                        store_bf16(reinterpret_cast<__bf16*>(p.C2) + (long)row * p.ldc2 + nb + 8 * h, v, rok,
                                   st_pre ? s_pre : nullptr, 4 * j + 2 * q + h);
                    else if (rok)
#pragma unroll
                        for (int t = 0; t < 2; ++t)
                            *reinterpret_cast<f32x4*>(p.C2 + (long)row * p.ldc2 + nb + 8 * t + 4 * h) =
                                f32x4{v[4 * t], v[4 * t + 1], v[4 * t + 2], v[4 * t + 3]};
                }
                if ((e & EPI_GELU) && CB && p.fgelu) {
#pragma unroll
                    for (int r = 0; r < 8; r += 2) {
                        const f32x2v g2 = gelu2_bf16ep(f32x2v{v[r], v[r + 1]});
                        v[r] = g2.x;
                        v[r + 1] = g2.y;
                    }
                } else if (e & EPI_GELU) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[r] = gelu_f(v[r]);
                }
                if ((e & EPI_DGELU) && CB && p.fgelu) {
#pragma unroll
                    for (int r = 0; r < 8; r += 2) {
                        const f32x2v g2 = dgelu2_bf16ep(f32x2v{xa[r], xa[r + 1]});
                        v[r] *= g2.x;
                        v[r + 1] *= g2.y;
                    }
                } else if (e & EPI_DGELU) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[r] *= dgelu_f(xa[r]);
                }
                if (e & EPI_RESID) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[r] += xr[r];
                }
                if (zero) {
#pragma unroll
                    for (int r = 0; r < 8; ++r) v[r] = 0.f;
                }
                if (e & EPI_DELTA) {
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const f32x4 od = *reinterpret_cast<const f32x4*>(p.dlt_o + rowc * p.ldo + nb + 8 * t + 4 * h);
                        const float d4 = fmaf(v[4 * t + 3], od[3], fmaf(v[4 * t + 2], od[2], fmaf(v[4 * t + 1], od[1], v[4 * t] * od[0])));
                        sg[2 * q + t] = j == 0 ? d4 : sg[2 * q + t] + d4;
                    }
                }
                if (st_c32) {
#pragma unroll
                    for (int t = 0; t < 2; ++t) {
                        const int c = 8 * j + 4 * q + 2 * t + h;  // 16-B chunk of the 256-B fp32 row
                        *reinterpret_cast<f32x4*>(s_c32 + l32 * 256 + ((c ^ (l32 & 7)) << 4)) =
                            f32x4{v[4 * t], v[4 * t + 1], v[4 * t + 2], v[4 * t + 3]};
                    }
                } else if ((!CB || p.C) && rok) {
#pragma unroll
                    for (int t = 0; t < 2; ++t)
                        *reinterpret_cast<f32x4*>(p.C + (long)row * p.ldc + nb + 8 * t + 4 * h) =
                            f32x4{v[4 * t], v[4 * t + 1], v[4 * t + 2], v[4 * t + 3]};
                }
                if (CB)
                    store_bf16(reinterpret_cast<__bf16*>(p.Cb) + (long)row * p.ldcb + nb + 8 * h, v, rok,
                               ST ? s_cb : nullptr, 4 * j + 2 * q + h);
            }
        if ((e & (EPI_DGELU | EPI_RESID)) && i + 1 < 4) load_ops(i + 1, o);
        if constexpr (ST) {
            wave_sync();
            const int row0 = rbase + 32 * i;
            if (st_pre) flush_bf16(s_pre, reinterpret_cast<__bf16*>(p.C2), p.ldc2, row0);
            if (st_c32) flush_f32(s_c32, p.C, p.ldc, row0);
            if (CB) flush_bf16(s_cb, reinterpret_cast<__bf16*>(p.Cb), p.ldcb, row0);
            wave_sync();
        }
        if (e & EPI_DELTA) {
            // the head is the wave's 64 columns; attn_delta_kernel's xor tree over its 16 four-column groups
            // (d / 4 = 8 j + 2 g + h: levels j, g >> 1, g & 1, then the half-wave h)
            const float l2 = (sg[0] + sg[2]) + (sg[1] + sg[3]);
            const float other = __shfl_xor(l2, 32, 64);
            if (h == 0 && rok) {
                const int b = row / p.dT, t = row - b * p.dT;
                p.delta[((long)b * p.dNH + cbase / 64) * p.dT + t] = l2 + other;
            }
        }
    }
}

// Epilogue of the 16x16x32 accumulators in their own C^T layout (round 6; gemm_hbp_kernel form 4): acc[bm][bn] lane l
// holds row 16 bm + (l & 15) of the wave tile and its 4 consecutive columns 16 bn + 4 (l >> 4) .. + 3, so bias, residual
// and fp32 operands load as 16-B vectors and bf16 operands as 8-B vectors per lane, and the outputs enter the staging
// images as 8-B (bf16) or 16-B (fp32) pieces straight from the registers -- no remap of the accumulators to the 32x32
// layout (which cost 1.6 us of a 33-us K = 1024 tile: profiles/r6/hbp_diag2.txt) and no v_permlane32_swap.  Same
// operations in the same order as epilogue_t per element.  Used for the bias / residual class (see NATIVE16 in
// hbp_tile); every flag is implemented so the A/B forms (tools DBG builds) stay comparable.  Images per 32-row band and wave (the buffers are free after
// the main loop): bf16 [32][128 B] with 16-B chunk c of row r at slot c ^ ((r >> 1) & 7) (the 8-B writes of 16 rows x 2
// halves and the 16-B flush reads both conflict-free), fp32 [32][256 B] with chunk c at c ^ (r & 15).  Classes without
// EPI_DELTA (the delta epilogue's summation tree is the 32x32 layout's: its kernels keep the remap).
template <bool CB, int EM, bool NT = false>
__device__ __forceinline__ void epilogue16t(const GemmParams& p, const f32x4 (&acc)[8][4], int rbase, int cbase,
                                            int lane, char* stage) {
    const int e = p.epi & EM;
    const int l16 = lane & 15, g = lane >> 4;
    const float alpha = p.alpha;
    const int rlim = (e & EPI_ROWMASK) ? p.zrows[0] : 0x7fffffff;
    const bool preb = CB && p.preb;
    if (cbase + 64 > p.N) {  // column tiles past N: element by element (same arithmetic, bounds-checked stores)
#pragma unroll
        for (int bm = 0; bm < 8; ++bm) {
            const int row = rbase + 16 * bm + l16;
#pragma unroll
            for (int bn = 0; bn < 4; ++bn)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int col = cbase + 16 * bn + 4 * g + k;
                    if (row >= p.M || col >= p.N) continue;
                    float v = acc[bm][bn][k] * alpha;
                    if (e & EPI_BIAS) v += p.bias[col];
                    if (e & EPI_STORE_PRE) {
                        if (preb) reinterpret_cast<__bf16*>(p.C2)[(long)row * p.ldc2 + col] = (__bf16)v;
                        else p.C2[(long)row * p.ldc2 + col] = v;
                    }
                    if (e & EPI_GELU) v = (CB && p.fgelu) ? gelu2_bf16ep(f32x2v{v, v}).x : gelu_f(v);
                    if (e & EPI_DGELU) {
                        const float xa = preb ? (float)reinterpret_cast<const __bf16*>(p.aux)[(long)row * p.ldaux + col]
                                              : p.aux[(long)row * p.ldaux + col];
                        v *= (CB && p.fgelu) ? dgelu2_bf16ep(f32x2v{xa, xa}).x : dgelu_f(xa);
                    }
                    if (e & EPI_RESID) v += p.R[(long)row * p.ldr + col];
                    if (row >= rlim) v = 0.f;
                    if (!CB || p.C) p.C[(long)row * p.ldc + col] = v;
                    if (CB) reinterpret_cast<__bf16*>(p.Cb)[(long)row * p.ldcb + col] = (__bf16)v;
                }
        }
        return;
    }
    char* const s_pre = stage;          // bf16 pre-activation image
    char* const s_c32 = stage + 4096;   // fp32 C image
    char* const s_cb = stage + 12288;   // bf16 C plane image
    const bool st_pre = (e & EPI_STORE_PRE) && preb;
    const bool c32 = !CB || p.C;
    auto bimg = [](char* img, int r, int c0) {  // 8-B piece of columns c0 .. c0 + 3 (c0 % 4 == 0) of image row r
        const int ch = c0 >> 3;
        return img + r * 128 + ((ch ^ ((r >> 1) & 7)) << 4) + 2 * (c0 & 7);
    };
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto flush_bf16 = [&](const char* img, __bf16* base, long ld, int row0) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int r = 8 * k + (lane >> 3), c = lane & 7;
            const u32x4v w = *reinterpret_cast<const u32x4v*>(img + r * 128 + ((c ^ ((r >> 1) & 7)) << 4));
            if (row0 + r < p.M) {
                u32x4v* d = reinterpret_cast<u32x4v*>(base + (long)(row0 + r) * ld + cbase + 8 * c);
                if constexpr (NT) __builtin_nontemporal_store(w, d);
                else *d = w;
            }
        }
    };
    auto flush_f32 = [&](const char* img, float* base, long ld, int row0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int r = 4 * k + (lane >> 4), c = lane & 15;
            const f32x4 w = *reinterpret_cast<const f32x4*>(img + r * 256 + ((c ^ (r & 15)) << 4));
            if (row0 + r < p.M) {
                f32x4* d = reinterpret_cast<f32x4*>(base + (long)(row0 + r) * ld + cbase + 4 * c);
                if constexpr (NT) __builtin_nontemporal_store(w, d);
                else *d = w;
            }
        }
    };
    typedef __bf16 bf16x4v __attribute__((ext_vector_type(4)));
    // Epilogue operands one 32-row band ahead: band i + 1's residual / GELU'-operand loads are issued as soon as band i
    // has consumed its own (before band i's stores), so the wait for them never covers those stores (a counted vmcnt
    // retires in order: loading right before use made every band wait for the previous band's stores and for each
    // load's latency -- profiles/r6/hbp_resid*.txt).  The bias (the same for every band) is loaded once.
    typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
    struct Ops {
        f32x4 r[2][4];   // residual, [b2][bn]
        u32x4v a[2][4];  // GELU' operand: 4 bf16 in words 0-1 (bf16 pre-activation plane) or 4 fp32
    };
    auto load_ops = [&](int i, Ops& o) {
#pragma unroll
        for (int b2 = 0; b2 < 2; ++b2) {
            const long rowc = min(rbase + 32 * i + 16 * b2 + l16, p.M - 1);
#pragma unroll
            for (int bn = 0; bn < 4; ++bn) {
                const int col = cbase + 16 * bn + 4 * g;
                if (e & EPI_RESID) o.r[b2][bn] = *reinterpret_cast<const f32x4*>(p.R + rowc * p.ldr + col);
                if (e & EPI_DGELU) {
                    if (preb) {
                        const u32x2v w = *reinterpret_cast<const u32x2v*>(reinterpret_cast<const __bf16*>(p.aux) +
                                                                          rowc * p.ldaux + col);
                        o.a[b2][bn] = u32x4v{w[0], w[1], 0u, 0u};
                    } else {
                        o.a[b2][bn] = *reinterpret_cast<const u32x4v*>(p.aux + rowc * p.ldaux + col);
                    }
                }
            }
        }
    };
    f32x4 bjv[4];
    if (e & EPI_BIAS) {
#pragma unroll
        for (int bn = 0; bn < 4; ++bn) bjv[bn] = *reinterpret_cast<const f32x4*>(p.bias + cbase + 16 * bn + 4 * g);
    }
    Ops o;
    load_ops(0, o);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int b2 = 0; b2 < 2; ++b2) {
            const int rl = 16 * b2 + l16;  // row within the band
            const int row = rbase + 32 * i + rl;
            const bool rok = row < p.M;
            const bool zero = (e & EPI_ROWMASK) && row >= rlim;
#pragma unroll
            for (int bn = 0; bn < 4; ++bn) {
                const int cl = 16 * bn + 4 * g;  // column within the wave tile
                const int col = cbase + cl;
                float v[4], xa[4], xr[4];
                if (e & EPI_DGELU) {
                    const u32x4v w = o.a[b2][bn];
                    if (preb) {
                        xa[0] = bf16_lo(w[0]);
                        xa[1] = bf16_hi(w[0]);
                        xa[2] = bf16_lo(w[1]);
                        xa[3] = bf16_hi(w[1]);
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; ++k) xa[k] = __uint_as_float(w[k]);
                    }
                }
                if (e & EPI_RESID) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) xr[k] = o.r[b2][bn][k];
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    v[k] = acc[2 * i + b2][bn][k] * alpha;
                    if (e & EPI_BIAS) v[k] += bjv[bn][k];
                }
                if (e & EPI_STORE_PRE) {
                    if (preb) {
                        const bf16x4v w = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
                        *reinterpret_cast<bf16x4v*>(bimg(s_pre, rl, cl)) = w;
                    } else if (rok) {
                        *reinterpret_cast<f32x4*>(p.C2 + (long)row * p.ldc2 + col) = f32x4{v[0], v[1], v[2], v[3]};
                    }
                }
                if ((e & EPI_GELU) && CB && p.fgelu) {
#pragma unroll
                    for (int r = 0; r < 4; r += 2) {
                        const f32x2v g2 = gelu2_bf16ep(f32x2v{v[r], v[r + 1]});
                        v[r] = g2.x;
                        v[r + 1] = g2.y;
                    }
                } else if (e & EPI_GELU) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = gelu_f(v[r]);
                }
                if ((e & EPI_DGELU) && CB && p.fgelu) {
#pragma unroll
                    for (int r = 0; r < 4; r += 2) {
                        const f32x2v g2 = dgelu2_bf16ep(f32x2v{xa[r], xa[r + 1]});
                        v[r] *= g2.x;
                        v[r + 1] *= g2.y;
                    }
                } else if (e & EPI_DGELU) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] *= dgelu_f(xa[r]);
                }
                if (e & EPI_RESID) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] += xr[r];
                }
                if (zero) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] = 0.f;
                }
                if (c32) {
                    const int ch = cl >> 2;
                    *reinterpret_cast<f32x4*>(s_c32 + rl * 256 + ((ch ^ (rl & 15)) << 4)) = f32x4{v[0], v[1], v[2], v[3]};
                }
                if (CB) {
                    const bf16x4v w = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
                    *reinterpret_cast<bf16x4v*>(bimg(s_cb, rl, cl)) = w;
                }
            }
        }
        if (i + 1 < 4) load_ops(i + 1, o);  // (band i's operands are dead: issued before band i's stores)
        wave_sync();
        const int row0 = rbase + 32 * i;
        if (st_pre) flush_bf16(s_pre, reinterpret_cast<__bf16*>(p.C2), p.ldc2, row0);
        if (c32) flush_f32(s_c32, p.C, p.ldc, row0);
        if (CB) flush_bf16(s_cb, reinterpret_cast<__bf16*>(p.Cb), p.ldcb, row0);
        wave_sync();
    }
}

// DBG (tools/hb_bench diagnostics only; the results are garbage): 1 no B-operand DMA, 2 no B-fragment reads after
// the first, 3 no DMA at all, 4 no fragment reads after the first slice; 5 (correct results) s_setprio(1) around
// the MFMA halves
template <int MS, bool CB, int EM, int TR, int DBG = 0>
__global__ __launch_bounds__(512, 1) void gemm_hbx_kernel(GemmParams p) {
    __shared__ __attribute__((aligned(16))) float smem[X_NR * X_SLOT];
    const TileId tid = xcd_tile(p.order);
    const float* A = reinterpret_cast<const float*>(p.Ab);
    const float* B = reinterpret_cast<const float*>(p.Bb);
    const long lda = p.ldab / 2, ldb = p.ldbb / 2;  // in 4-byte units
    const int m0 = tid.y * X_BM, n0 = tid.x * X_BN;
    const int nst = p.K / 32;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wid >> 2, wc = wid & 3;
    const int h = lane >> 5, l32 = lane & 31, l16 = lane & 15, q4 = lane >> 4;

    constexpr int AM = MS == 32 ? 4 : 8, AN = MS == 32 ? 2 : 4;  // fragments of the 128 x 64 wave tile
    typedef typename std::conditional<MS == 32, f32x16, f32x4>::type Acc;
    Acc acc[AM][AN];
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
            for (int r = 0; r < (MS == 32 ? 16 : 4); ++r) acc[i][j][r] = 0.f;

    XStream<X_BM> sa;
    XStream<X_BN> sb;
    sa.init(A, lda, m0, p.M, wid, lane);
    sb.init(B, ldb, n0, p.N, wid, lane);
    auto issue = [&](int s) {
        float* st = smem + (s % X_NR) * X_SLOT;
        if constexpr (DBG != 3) xstream_issue(sa, st, wid);
        if constexpr (DBG != 1 && DBG != 3) xstream_issue(sb, st + X_BM * X_KS, wid);
    };
    // part c of slice s: MS 32 -> k-chunk c (k 16c..16c+15); MS 16 -> the wave tile's m-half c (k 0..31)
    auto read = [&](int s, int c, XFr<MS>& f) {
        const float* As = smem + (s % X_NR) * X_SLOT;
        const float* Bs = As + X_BM * X_KS;
        if constexpr (MS == 32) {
            if (DBG == 4 && s > 0) return;
            if (DBG != 2 || s == 0) {
#pragma unroll
                for (int j = 0; j < 2; ++j) f.b[j] = xfrag(Bs, wc * 64 + j * 32 + l32, 2 * c + h);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) f.a[i] = xfrag(As, wr * 128 + i * 32 + l32, 2 * c + h);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) f.b[j] = xfrag(Bs, wc * 64 + j * 16 + l16, q4);
#pragma unroll
            for (int i = 0; i < 4; ++i) f.a[i] = xfrag(As, wr * 128 + (4 * c + i) * 16 + l16, q4);
        }
    };
    auto mfma = [&](int c, const XFr<MS>& f) {
        if constexpr (MS == 32) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = TR ? __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.b[j], f.a[i], acc[i][j], 0, 0, 0)
                                   : __builtin_amdgcn_mfma_f32_32x32x16_bf16(f.a[i], f.b[j], acc[i][j], 0, 0, 0);
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[4 * c + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.a[i], f.b[j], acc[4 * c + i][j], 0, 0, 0);
        }
    };
    constexpr int NMF = 16;  // MFMAs per half-slice part (MS 32: 8 of 32x32x16 = 16 cycles-equivalents... see below)
    (void)NMF;
    // one slice step.  On entry X holds part 0 of slice s.  [counted wait + barrier B_s] -> DMA of slice s+3;
    // read part 1 of slice s into Y; MFMAs of part 0 (X); read part 0 of slice s+1 into X (after B_s: landed);
    // MFMAs of part 1 (Y).  Each read batch overlaps the other part's MFMAs.
    auto step = [&](int s, XFr<MS>& X, XFr<MS>& Y, auto dma_tag, auto rd_tag) {
        constexpr bool DMA = decltype(dma_tag)::value, RD = decltype(rd_tag)::value;
        if (s + 2 < nst) wait_vm<X_NPW>();  // slice s+1 landed; s+2 may stay in flight
        else wait_vm<0>();
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (DBG == 5) {  // s_setprio(1) over the MFMA halves (cdna_hip_programming.md T5)
            if constexpr (DMA) issue(s + 3);
            read(s, 1, Y);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
            mfma(0, X);
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (RD) read(s + 1, 0, X);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_setprio(1);
            mfma(1, Y);
            __builtin_amdgcn_s_setprio(0);
            __builtin_amdgcn_sched_barrier(0);
            return;
        }
        if constexpr (DMA) issue(s + 3);
        read(s, 1, Y);
        mfma(0, X);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (RD) read(s + 1, 0, X);
        mfma(1, Y);
        __builtin_amdgcn_sched_barrier(0);
    };
    using T1 = std::true_type;
    using T0 = std::false_type;

    // prologue: slices 0, 1, 2 in flight; slice 0 landed; its part 0 read (nst >= 4: the dispatcher's K >= 128)
    issue(0);
    issue(1);
    issue(2);
    wait_vm<2 * X_NPW>();
    __builtin_amdgcn_s_barrier();
    XFr<MS> fx{}, fy{};
    read(0, 0, fx);
    if constexpr (DBG == 2 || DBG == 4) read(0, 1, fy);
    int s = 0;
    for (; s + 3 < nst; ++s) step(s, fx, fy, T1{}, T1{});
    if (s + 1 < nst) step(s++, fx, fy, T0{}, T1{});
    if (s + 1 < nst) step(s++, fx, fy, T0{}, T1{});
    step(s, fx, fy, T0{}, T0{});
    wait_vm<0>();

    const bool interior = m0 + X_BM <= p.M && n0 + X_BN <= p.N;
    if constexpr (TR == 2) {
        __syncthreads();  // every wave is done with the ring: wave-private 16-KB staging images
        epilogue_t<CB, EM, true>(p, reinterpret_cast<const f32x16(&)[4][2]>(acc[0]), m0 + wr * 128, n0 + wc * 64, lane,
                                 reinterpret_cast<char*>(smem) + wid * 16384);
    } else if constexpr (TR == 1) {
        epilogue_t<CB, EM, false>(p, reinterpret_cast<const f32x16(&)[4][2]>(acc[0]), m0 + wr * 128, n0 + wc * 64, lane,
                                  nullptr);
    } else if constexpr (MS == 32) {
        gemm_epilogue<2, 2, CB, EM>(p, reinterpret_cast<const f32x16(&)[2][2]>(acc[0]), 0, 0, m0 + wr * 128,
                                    n0 + wc * 64, h, l32, interior, tid.z);
        gemm_epilogue<2, 2, CB, EM>(p, reinterpret_cast<const f32x16(&)[2][2]>(acc[2]), 0, 0, m0 + wr * 128 + 64,
                                    n0 + wc * 64, h, l32, interior, tid.z);
    } else {
        // two 64-row halves (bounds the epilogue's live temporaries beside the accumulators)
        epilogue16<4, 4, CB, EM>(p, reinterpret_cast<const f32x4(&)[4][4]>(acc[0]), m0 + wr * 128, n0 + wc * 64, lane,
                                 interior);
        epilogue16<4, 4, CB, EM>(p, reinterpret_cast<const f32x4(&)[4][4]>(acc[4]), m0 + wr * 128 + 64, n0 + wc * 64,
                                 lane, interior);
    }
}

// ---------------------------------------------------------------------------------------------------------------
// "hbp": the same 256 x 256 tile, C^T accumulators and staged epilogue, with the four-phase K-tile schedule of
// cdna_hip_programming.md's 256^2 8-phase template (BK = 64, two LDS buffers of four 16-KB half-tiles, one half-tile
// of DMA issued per phase, counted vmcnt every phase, two barriers per phase, optionally two wave groups one
// barrier apart with s_setprio(1) over each MFMA cluster).
// Half-tiles of a K-tile: A0 / A1 = A rows {128 wr + 64 qm + r : wr in 0..1, r < 64} for qm = 0 / 1, B0 / B1 = B rows
// {64 wc + 32 qn + r : wc in 0..3, r < 32} for qn = 0 / 1 -- so wave (wr, wc)'s quadrant (qm, qn) reads 64 rows of
// A half qm and 32 of B half qn and the four quadrants cover its contiguous 128 x 64 output (epilogue_t unchanged).
// LDS rows of 128 B (64 bf16 of K), chunk c of row r in slot c ^ ((r >> 1) & 7): conflict-free ds_read_b128 for
// 32 consecutive rows at one chunk (both 16-lane group patterns), swizzle on the DMA source address.
// Phases of K-tile t (buffer t & 1): 1 quadrant (0,0) reads A(qm 0) + B(qn 0); 2 (0,1) reads B(qn 1); 3 (1,1) reads
// A(qm 1); 4 (1,0) no reads (B(qn 0) kept in registers).  Phase p also issues half-tile p - 1 (A0, B0, B1, A1) of
// K-tile t + 1 into the other buffer, whose last reads (phase 3 of K-tile t - 1) are two phases back (WAR).  The
// wait at phase p retires every half issued before phase p - 1 (vmcnt(4)); a half issued at phase q is read at
// phase q + 3 or later, after that wait and a barrier every wave has passed (RAW; with the wave-group stagger the
// lagging group's wait still precedes the leading group's read by one barrier).
constexpr int P_HALF = 16384;  // bytes per half-tile image (128 rows x 128 B)

__device__ __forceinline__ int hbp_swz(int r) { return (r >> 1) & 7; }

// FORM 1: lockstep; 2: wave groups one barrier apart (STAG); 3: STAG with three half-tiles of DMA in flight and one
// counted wait per K-tile (below); 4: form 3's schedule on v_mfma_f32_16x16x32_bf16 (16 MFMAs per phase instead of 8
// of 32x32x16, the guide's 256^2 template shape), accumulators remapped through LDS to the 32x32 C^T layout of
// epilogue_t after the main loop (round 6).
// CONV: conv-A rows with per-tap weight segments (the conv stack's input gradients, gemm.hip use_hbp_conv): A(m, k) =
// Ab[(m + seg - pad) ldab + k - seg segK], zero unless 0 <= m + seg - pad < Mvalid (per utterance: zmvalid), B(k, n) =
// Bb[n ldbb + k - seg segK + seg sBseg], seg = k / segK.  With ldab == segK the A address is linear in k (a segment
// step is one row down and back to column 0), so only the row's validity changes per segment; the B address jumps by
// sBseg - segK at each segment boundary.  Both are evaluated per DMA issue (segK % 64 == 0: a K-tile lies in one
// segment), so the shifts live in the DMA pointers, not in per-element VALU work.
// DBG (tools/hb_bench diagnostics only, -DSUTA_HBX_DIAG; wrong results): 1 no epilogue (accumulators kept live), 2 no
// K loop (prologue DMA and epilogue only), 3 neither, 4 no global stores of the staged epilogue (with the remap), 8 no
// LDS remap of the 16x16 accumulators (into epilogue_t), 16 the remap + epilogue_t instead of epilogue16t, 32
// nontemporal global stores in the epilogue
// one 256 x 256 output tile (a persistent kernel looping this body over its XCD's tiles, one block per CU with the next
// tile's first K-tiles fetched while the epilogue's stores drain, measured 1-2 us per tile slower than one block per
// tile: DESIGN.md section 8)
// TN (round 6, form 4 only): MN-contiguous operands (A(m, k) = Ab[k ldab + m], B(k, n) = Bb[k ldbb + n]: the conv
// stack's weight gradients, im2col(a)^T dz, formerly gemm_hbt_kernel's 128 x 128 two-stage loop).  A half-tile image is
// [64 k][128 columns] bf16 (256-B rows; columns = the half's 128 m or n in the same order as the k-contiguous form), its
// 16-B chunk c of row r in slot c ^ tn_swz(r) (on the DMA source); a fragment's 8 consecutive k of one column are two
// ds_read_b64_tr_b16 reads (per 16-lane group 4 rows x 16 columns delivered column-major: lane i gets column i), the
// 8 rows a 32-lane half reads land on 8 disjoint 32-B slot pairs (conflict-free).  K need not be a multiple of 64: rows
// past K read the zero page.  The quadrants, phases, waits and epilogue are form 4's.
__device__ __forceinline__ int tn_swz(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

template <bool CB, int EM, int FORM, bool CONV, int DBG, bool TN = false>
__device__ __forceinline__ void hbp_tile(const GemmParams& p, const TileId tid, char* const lds) {
    static_assert(!TN || (FORM == 4 && !CONV), "TN: form 4, no conv-A rows");
    // batch z (Z-batched GEMMs, the conv stack's per-utterance forward): operand planes offset in bf16 elements, the
    // epilogue's operands through a rebased copy of the parameters (batch z of a Z = 1 view)
    const int z1 = tid.z / p.zdiv, z0 = tid.z % p.zdiv;
    const __bf16* A = reinterpret_cast<const __bf16*>(p.Ab) + z1 * p.sA1 + z0 * p.sA0;
    const __bf16* B = reinterpret_cast<const __bf16*>(p.Bb) + z1 * p.sB1 + z0 * p.sB0;
    const int m0 = tid.y * 256, n0 = tid.x * 256;
    const int nk = TN ? (p.K + 63) / 64 : p.K / 64;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wid >> 2, wc = wid & 3;
    constexpr bool STAG = FORM >= 2;

    // DMA sources: half h (0 A0, 1 B0, 2 B1, 3 A1 -- the issue order), pieces wid and wid + 8 (8 LDS rows each)
    const __bf16* src[4][2];
    int inc[4][2];
    int arow[2][2];  // CONV: source row m - pad of the A halves' pieces (segment 0)
    const int mv = CONV ? (p.zmvalid ? p.zmvalid[z1] : p.Mvalid) : 0;
    int krow[2];  // TN: the k row (within a K-tile) of the lane's 16-B piece, per piece
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if constexpr (TN) {  // piece = 4 image rows of 256 B; lane j: row 4 pc + j / 16, slot j % 16
                const int pc = wid + 8 * i, kr = 4 * pc + (lane >> 4);
                const int ch = (lane & 15) ^ tn_swz(kr);
                const bool isa = h == 0 || h == 3;
                const int q = h == 3 ? 1 : h == 2 ? 1 : 0;
                const int gc = isa ? m0 + 128 * (ch >> 3) + 64 * q + 8 * (ch & 7) : n0 + 64 * (ch >> 2) + 32 * q + 8 * (ch & 3);
                const bool ok = gc < (isa ? p.M : p.N);
                const long ld = isa ? p.ldab : p.ldbb;
                krow[i] = kr;
                src[h][i] = ok ? (isa ? A : B) + (long)kr * ld + gc : reinterpret_cast<const __bf16*>(g_zero16);
                inc[h][i] = ok ? (int)(64 * ld) : 0;
                continue;
            }
            const int pc = wid + 8 * i, lr = 8 * pc + (lane >> 3);
            const int c = (lane & 7) ^ hbp_swz(lr);
            const bool isa = h == 0 || h == 3;
            const int q = h == 3 ? 1 : h == 2 ? 1 : 0;  // qm for A halves, qn for B halves
            const int grow = isa ? m0 + (lr >> 6) * 128 + q * 64 + (lr & 63) : n0 + (lr >> 5) * 64 + q * 32 + (lr & 31);
            if (CONV && isa) {  // linear address of row grow - pad (validity decided per issue)
                arow[h == 3 ? 1 : 0][i] = grow - p.pad;
                src[h][i] = A + (long)(grow - p.pad) * p.ldab + 8 * c;
                inc[h][i] = 64;
                continue;
            }
            const bool ok = grow < (isa ? p.M : p.N);
            const long ld = isa ? p.ldab : p.ldbb;
            src[h][i] = ok ? (isa ? A : B) + (long)grow * ld + 8 * c : reinterpret_cast<const __bf16*>(g_zero16);
            inc[h][i] = ok ? 64 : 0;
        }
    const int spt = CONV ? p.segK / 64 : 1;          // K-tiles per segment
    const long bjump = CONV ? p.sBseg - p.segK : 0;  // B address step at a segment boundary (bf16 elements)
    // LDS image of half h in buffer b (images in the order A0, A1, B0, B1)
    auto himg = [&](int b, int h) -> char* {
        const int slot = h == 0 ? 0 : h == 3 ? 1 : h == 1 ? 2 : 3;
        return lds + (b * 4 + slot) * P_HALF;
    };
    auto issue = [&](int t, int h) {  // half h of K-tile t into buffer t & 1
        char* dst = himg(t & 1, h);
        if constexpr (CONV) {
            const int seg = t / spt;
            const bool isa = h == 0 || h == 3;
            if (!isa && t > 0 && t == seg * spt) {  // the next tap's weight slice
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    if (inc[h][i]) src[h][i] += bjump;
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const __bf16* g = src[h][i];
                if (isa && (unsigned)(arow[h == 3 ? 1 : 0][i] + seg) >= (unsigned)mv)
                    g = reinterpret_cast<const __bf16*>(g_zero16);  // conv padding row: zeros
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const float*>(g),
                                                 (lds_ptr_t)(dst + (wid + 8 * i) * 1024), 16, 0, 0);
                src[h][i] += inc[h][i];
            }
            return;
        }
        if constexpr (TN) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const __bf16* g = t * 64 + krow[i] < p.K ? src[h][i] : reinterpret_cast<const __bf16*>(g_zero16);
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const float*>(g),
                                                 (lds_ptr_t)(dst + (wid + 8 * i) * 1024), 16, 0, 0);
                src[h][i] += inc[h][i];
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const float*>(src[h][i]),
                                             (lds_ptr_t)(dst + (wid + 8 * i) * 1024), 16, 0, 0);
            src[h][i] += inc[h][i];
        }
    };
    auto frag = [&](const char* img, int lr, int kk) {
        const int c = 2 * kk + (lane >> 5);
        return *reinterpret_cast<const bf16x8*>(img + lr * 128 + ((c ^ hbp_swz(lr)) << 4));
    };
    constexpr bool M16 = FORM == 4;
    f32x16 acc[4][2];
    f32x4 acc16[8][4];  // M16: acc16[bm][bn] = C^T fragment of rows 16 bm .. of the wave tile, columns 16 bn ..
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    if constexpr (M16) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc16[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    bf16x8 fa[2][4], fb0[4], fb1[4];
    // M16 fragments (16x16x32: lane -> row lane & 15 of a 16-row block, 8 k at 32 kk2 + 8 (lane >> 4) = chunk
    // 4 kk2 + (lane >> 4); the same registers as the 32x32 form: fa[bi][kk] = 16-row block bi, kk2 = kk & 1 for
    // bi < 4 ... stored as fa[bm >> 1][2 (bm & 1) + kk2], fb[2 bn + kk2])
    auto frag16 = [&](const char* img, int lr, int kk2) {
        const int c = 4 * kk2 + (lane >> 4);
        return *reinterpret_cast<const bf16x8*>(img + lr * 128 + ((c ^ hbp_swz(lr)) << 4));
    };
    // TN: 8 consecutive k (32 kk2 + 8 (lane >> 4) ..) of column 16 j + (lane & 15) of a [64][128] image
    auto tr8 = [&](const char* img, int j, int kk2) {
        typedef __attribute__((address_space(3))) fbf16x4_t* lp4;
        const int gq = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
        bf16x8 v;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const int r = 32 * kk2 + 8 * gq + 4 * s2 + q;
            const int slot = (2 * j + (pp >> 1)) ^ tn_swz(r);
            const fbf16x4_t x = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp4)(img + r * 256 + slot * 16 + 8 * (pp & 1)));
#pragma unroll
            for (int e = 0; e < 4; ++e) v[4 * s2 + e] = x[e];
        }
        return v;
    };
    auto read_a = [&](int b, int qm) {
        const char* img = lds + (b * 4 + qm) * P_HALF;
        if constexpr (TN) {
#pragma unroll
            for (int bm = 0; bm < 4; ++bm)
#pragma unroll
                for (int kk2 = 0; kk2 < 2; ++kk2) fa[bm >> 1][2 * (bm & 1) + kk2] = tr8(img, 4 * wr + bm, kk2);
        } else if constexpr (M16) {
#pragma unroll
            for (int bm = 0; bm < 4; ++bm)
#pragma unroll
                for (int kk2 = 0; kk2 < 2; ++kk2)
                    fa[bm >> 1][2 * (bm & 1) + kk2] = frag16(img, wr * 64 + 16 * bm + (lane & 15), kk2);
        } else {
#pragma unroll
            for (int bi = 0; bi < 2; ++bi)
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) fa[bi][kk] = frag(img, wr * 64 + 32 * bi + (lane & 31), kk);
        }
    };
    auto read_b = [&](int b, int qn, bf16x8 (&fb)[4]) {
        const char* img = lds + (b * 4 + 2 + qn) * P_HALF;
        if constexpr (TN) {
#pragma unroll
            for (int bn = 0; bn < 2; ++bn)
#pragma unroll
                for (int kk2 = 0; kk2 < 2; ++kk2) fb[2 * bn + kk2] = tr8(img, 2 * wc + bn, kk2);
        } else if constexpr (M16) {
#pragma unroll
            for (int bn = 0; bn < 2; ++bn)
#pragma unroll
                for (int kk2 = 0; kk2 < 2; ++kk2) fb[2 * bn + kk2] = frag16(img, wc * 32 + 16 * bn + (lane & 15), kk2);
        } else {
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) fb[kk] = frag(img, wc * 32 + (lane & 31), kk);
        }
    };
    auto mfma_q = [&](int qm, int qn, const bf16x8 (&fb)[4]) {
        if constexpr (M16) {
#pragma unroll
            for (int bm = 0; bm < 4; ++bm)
#pragma unroll
                for (int bn = 0; bn < 2; ++bn)
#pragma unroll
                    for (int kk2 = 0; kk2 < 2; ++kk2)
                        acc16[4 * qm + bm][2 * qn + bn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            fb[2 * bn + kk2], fa[bm >> 1][2 * (bm & 1) + kk2], acc16[4 * qm + bm][2 * qn + bn], 0, 0, 0);
        } else {
#pragma unroll
            for (int bi = 0; bi < 2; ++bi)
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
                    acc[2 * qm + bi][qn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[kk], fa[bi][kk], acc[2 * qm + bi][qn], 0, 0, 0);
        }
    };
    // counted wait of phase p: the halves issued at phases p - 1 and p (if any) may stay in flight
    auto wait_phase = [&](int n_out) {
        __builtin_amdgcn_sched_barrier(0);
        if (n_out >= 3) wait_vm<6>();
        else if (n_out >= 2) wait_vm<4>();
        else if (n_out == 1) wait_vm<2>();
        else wait_vm<0>();
    };
    auto barrier = [] {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
    };
    auto mfma_phase = [&](int qm, int qn, const bf16x8 (&fb)[4]) {
        barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) (vmcnt 63, expcnt 7): this phase's fragment reads
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (STAG) __builtin_amdgcn_s_setprio(1);
        mfma_q(qm, qn, fb);
        if constexpr (STAG) __builtin_amdgcn_s_setprio(0);
        barrier();
    };

    if constexpr (FORM >= 3) {
        // Deep form (cdna_hip_programming.md's 256^2 template schedule): the halves of K-tile t + 2 go into buffer t & 1
        // as soon as K-tile t is done with them, so three halves stay in flight and the wave waits once per K-tile.
        //   phase 1  reads B0, A0 of t  (B first)  | issues A1 of t + 1 (last read: phase 3 of t - 1, two phases back)
        //                                          | lgkmcnt(0) BEFORE the barrier: A0 / B0 of buffer t & 1 are free
        //   phase 2  reads B1                      | issues A0 of t + 2 (read in phase 1, retired before its barrier)
        //   phase 3  reads A1                      | issues B0 of t + 2 (read in phase 1)
        //   phase 4  --                            | issues B1 of t + 2 (read in phase 2); vmcnt(6): all but the three
        //                                          | halves of t + 2 retired -> K-tile t + 1 complete, read from phase 5
        // With the groups one barrier apart a read of the lagging group still follows the other group's wait by a
        // barrier, and an issue of the leading group follows the lagging group's retired reads by one (the phase
        // bodies are placed so: reads and issues before the first barrier, the wait before it in phase 4).
#pragma unroll
        for (int h = 0; h < 4; ++h) issue(0, h);
        if (nk > 1) {
            issue(1, 0);
            issue(1, 1);
            issue(1, 2);
            wait_vm<6>();
        } else {
            wait_vm<0>();
        }
        if (wr == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind group 0
        __builtin_amdgcn_s_barrier();
        for (int t = 0; t < ((DBG & 2) ? 0 : nk); ++t) {
            const int b = t & 1;
            const bool n1 = t + 1 < nk, n2 = t + 2 < nk;
            // phase 1: quadrant (0,0)
            read_b(b, 0, fb0);
            __builtin_amdgcn_sched_barrier(0);
            read_a(b, 0);
            if (n1) issue(t + 1, 3);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) before the barrier (WAR of phase 2's issue)
            __builtin_amdgcn_sched_barrier(0);
            barrier();
            __builtin_amdgcn_s_setprio(1);
            mfma_q(0, 0, fb0);
            __builtin_amdgcn_s_setprio(0);
            barrier();
            // phase 2: quadrant (0,1)
            read_b(b, 1, fb1);
            if (n2) issue(t + 2, 0);
            mfma_phase(0, 1, fb1);
            // phase 3: quadrant (1,1)
            read_a(b, 1);
            if (n2) issue(t + 2, 1);
            mfma_phase(1, 1, fb1);
            // phase 4: quadrant (1,0)
            if (n2) issue(t + 2, 2);
            wait_phase(n2 ? 3 : 0);
            mfma_phase(1, 0, fb0);
        }
    } else {
    // prologue: K-tile 0's four halves; A0 and B0 (phase 1's) retired
#pragma unroll
    for (int h = 0; h < 4; ++h) issue(0, h);
    wait_vm<4>();
    if constexpr (STAG) {
        if (wr == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind group 0
    }
    __builtin_amdgcn_s_barrier();
    for (int t = 0; t < nk; ++t) {
        const int b = t & 1;
        const bool nxt = t + 1 < nk;  // halves of K-tile t + 1 issued in this K-tile's phases
        // phase 1: quadrant (0,0)
        read_a(b, 0);
        read_b(b, 0, fb0);
        if (nxt) issue(t + 1, 0);
        wait_phase(1 + (nxt ? 1 : 0));  // (phase 4 of the previous K-tile, or the prologue's last half, issued one)
        mfma_phase(0, 0, fb0);
        // phase 2: quadrant (0,1)
        read_b(b, 1, fb1);
        if (nxt) issue(t + 1, 1);
        wait_phase(nxt ? 2 : 0);
        mfma_phase(0, 1, fb1);
        // phase 3: quadrant (1,1)
        read_a(b, 1);
        if (nxt) issue(t + 1, 2);
        wait_phase(nxt ? 2 : 0);
        mfma_phase(1, 1, fb1);
        // phase 4: quadrant (1,0)
        if (nxt) issue(t + 1, 3);
        wait_phase(nxt ? 2 : 0);
        mfma_phase(1, 0, fb0);
    }
    }
    wait_vm<0>();
    if constexpr (STAG) {
        if (wr == 0) __builtin_amdgcn_s_barrier();  // the leading group's matching barrier
    }
    __syncthreads();  // every wave is done with the buffers: wave-private 16-KB staging images
    // the native 16x16 epilogue on the class where the C4 loop measured it faster than the remap + epilogue_t: the bias /
    // residual linears, conv GEMMs and conv weight gradients (profiles/r6/trace_ab/nat2_*: fp32-output residual linears
    // -7 %, QKV -7 %, bf16-plane residual linears -2 %, with the band-ahead operand loads); the GELU / GELU' classes
    // measured 2 % slower with it in the loop (though faster in tools/hb_bench) and keep the remap
    constexpr bool NATIVE16 = EM == (EPI_BIAS | EPI_RESID | EPI_ROWMASK) && (DBG & 16) == 0;
    // nontemporal epilogue stores (round 6 default: the outputs stream past the caches on their way out; C4 +0.6 %,
    // GEMM family -0.9 %, profiles/r6/ntab/summary.txt; -DSUTA_EPI_NT=0 builds the cached stores for A/B runs)
#ifndef SUTA_EPI_NT
#define SUTA_EPI_NT 1
#endif
    constexpr bool NTST = (DBG & 32) != 0 || SUTA_EPI_NT != 0;
    if constexpr ((DBG & 1) != 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc16[i][j]));
        return;
    }
    if constexpr (M16 && (DBG & 8) != 0) {  // (tools diagnostics: no remap, wrong results)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int g = 0; g < 4; ++g)
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[i][j][4 * g + k] = acc16[2 * i + (g >> 1)][2 * j + (g & 1)][k];
    } else if constexpr (M16 && NATIVE16) {
        // (the native 16x16 epilogue below)
    } else if constexpr (M16) {
        // 16x16 C^T fragments -> the 32x32 C^T layout (lane l: row 32 i + (l & 31), register 4 g + k: column 32 j + 8 g +
        // 4 (l >> 5) + k), one 32-row band at a time through the wave's staging image: fp32 [32][64], 16-B chunk c of
        // row r at slot c ^ (r & 15) (conflict-free 16-B writes and reads)
        char* const tb = lds + wid * 16384;
        const int l16 = lane & 15, g4 = lane >> 4, l32 = lane & 31, hh = lane >> 5;
        auto wave_sync = [] {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
                for (int bn = 0; bn < 4; ++bn) {
                    const int r = 16 * b2 + l16, c = 4 * bn + g4;
                    *reinterpret_cast<f32x4*>(tb + r * 256 + ((c ^ (r & 15)) << 4)) = acc16[2 * i + b2][bn];
                }
            wave_sync();
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int c = 8 * j + 2 * g + hh;
                    const f32x4 v = *reinterpret_cast<const f32x4*>(tb + l32 * 256 + ((c ^ (l32 & 15)) << 4));
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[i][j][4 * g + k] = v[k];
                }
            wave_sync();
        }
    }
    {  // (one epilogue instantiation: for Z = 1 the rebase adds zero)
        GemmParams q = p;
        const bool preb = CB && p.preb;
        if (p.C) q.C = p.C + z1 * p.sC1 + z0 * p.sC0;
        if (p.Cb) q.Cb = reinterpret_cast<__bf16*>(p.Cb) + z1 * p.sCb1;
        if (p.bias) q.bias = p.bias + z1 * p.sBias1 + z0 * p.sBias0;
        if (p.R) q.R = p.R + z1 * p.sR1 + z0 * p.sR0;
        if (p.aux)
            q.aux = preb ? reinterpret_cast<const float*>(reinterpret_cast<const __bf16*>(p.aux) + z1 * p.sAux1 + z0 * p.sAux0)
                         : p.aux + z1 * p.sAux1 + z0 * p.sAux0;
        if (p.C2)
            q.C2 = preb ? reinterpret_cast<float*>(reinterpret_cast<__bf16*>(p.C2) + z1 * p.sC21 + z0 * p.sC20)
                        : p.C2 + z1 * p.sC21 + z0 * p.sC20;
        if (p.zrows) q.zrows = p.zrows + z1;
        if constexpr (M16 && NATIVE16 && (DBG & 8) == 0)
            epilogue16t<CB, EM, NTST>(q, acc16, m0 + wr * 128, n0 + wc * 64, lane, lds + wid * 16384);
        else
            epilogue_t<CB, EM, true, (DBG & 4), NTST>(q, acc, m0 + wr * 128, n0 + wc * 64, lane, lds + wid * 16384);
    }
}

template <bool CB, int EM, int FORM, bool CONV = false, int DBG = 0, bool TN = false>
__global__ __launch_bounds__(512, 1) void gemm_hbp_kernel(GemmParams p) {
    __shared__ __attribute__((aligned(16))) float smem[8 * P_HALF / 4];
    hbp_tile<CB, EM, FORM, CONV, DBG, TN>(p, xcd_tile(p.order), reinterpret_cast<char*>(smem));
}

template <int MS, int EM, int TR = 0>
void launch_hbx_em(const GemmParams& p, dim3 grid, hipStream_t st) {
    if (p.Cb) hipLaunchKernelGGL((gemm_hbx_kernel<MS, true, EM, TR>), grid, dim3(512), 0, st, p);
    else hipLaunchKernelGGL((gemm_hbx_kernel<MS, false, EM, TR>), grid, dim3(512), 0, st, p);
}

// operands of the row-per-lane epilogue: 16-B bases, leading dimensions in whole 16-B chunks
}  // namespace

bool hbx_t_ok(const GemmParams& p, bool check_off32) {
    auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    const int e = p.epi;
    if (check_off32 && !p.off32) return false;
    if ((!p.Cb || p.C) && !(a16(p.C) && p.ldc % 4 == 0)) return false;
    if (p.Cb && !(a16(p.Cb) && p.ldcb % 8 == 0)) return false;
    if ((e & EPI_BIAS) && !a16(p.bias)) return false;
    if ((e & EPI_RESID) && !(a16(p.R) && p.ldr % 4 == 0)) return false;
    const bool preb = p.Cb && p.preb;
    if ((e & EPI_DGELU) && !(a16(p.aux) && p.ldaux % (preb ? 8 : 4) == 0)) return false;
    if ((e & EPI_STORE_PRE) && !(a16(p.C2) && p.ldc2 % (preb ? 8 : 4) == 0)) return false;
    if (p.Z > 1) {  // batch strides keep every row base 16-B aligned (planes in bf16 elements, fp32 operands in floats)
        if (((p.sA0 | p.sA1 | p.sB0 | p.sB1) % 8) || (p.Cb && (p.sCb1 % 8 || p.zdiv != 1)) ||
            ((!p.Cb || p.C) && ((p.sC0 | p.sC1) % 4)) || ((e & EPI_BIAS) && ((p.sBias0 | p.sBias1) % 4)) ||
            ((e & EPI_RESID) && ((p.sR0 | p.sR1) % 4)) || (e & EPI_DELTA))
            return false;
        const long sa = preb ? 8 : 4;
        if (((e & EPI_DGELU) && ((p.sAux0 | p.sAux1) % sa)) || ((e & EPI_STORE_PRE) && ((p.sC20 | p.sC21) % sa)))
            return false;
    }
    if ((e & EPI_DELTA) && !(e == EPI_DELTA && a16(p.dlt_o) && p.ldo % 4 == 0 && p.delta && p.dT > 0 &&
                             (long)p.dNH * 64 == p.N && p.M % p.dT == 0))
        return false;
    return true;
}

// the conv stack's input-gradient GEMMs (conv-A rows, per-tap bf16 weight segments) on the four-phase 256 x 256 kernel:
// k-contiguous planes whose A rows are the segments (ldab == segK, segK % 64 == 0, segmented B, no batch split inside a
// plane), the staggered main loop (SUTA_HBX_FORM 2 / 3) with the staged C^T epilogue, the plain epilogue class
// SUTA_HBX_DBG: gemm_hbx_kernel with parts of its main loop removed (wrong results; tools/hb_bench diagnostics of
// where the loop's time goes).  Compiled only into the tools build (-DSUTA_HBX_DIAG), never into libsuta.so.
static int hbx_diag() {
#ifdef SUTA_HBX_DIAG
    return suta_switches().hbx_dbg;
#else
    return 0;
#endif
}

bool hbp_conv_ok(const GemmParams& p) {
    const SutaSwitches& sw = suta_switches();
    return p.segK > 0 && p.segB && p.segK % 64 == 0 && p.ldab == p.segK && p.pad >= 0 && p.K % 64 == 0 && p.K >= 128 &&
           p.zdiv == 1 && !p.ta && p.Ab && p.Bb && sw.hbx_form >= 2 && sw.hbx_t == 2 && !hbx_diag() &&
           (p.epi & ~(EPI_BIAS | EPI_RESID | EPI_ROWMASK)) == 0 && !p.preb && p.splits <= 1 && hbx_t_ok(p, true);
}

namespace {

// epilogue classes of the bf16 linears (as gemm_hb_ep.hip): bias / residual, bias + GELU + pre-activation store,
// GELU'; ragged row masks in each
constexpr int XEM_A = EPI_BIAS | EPI_RESID | EPI_ROWMASK;
constexpr int XEM_G = EPI_BIAS | EPI_GELU | EPI_STORE_PRE | EPI_ROWMASK;
constexpr int XEM_D = EPI_DGELU | EPI_ROWMASK;
constexpr int XEM_L = EPI_DELTA;  // the attention out-projection's input gradient with the flash backward's delta

}  // namespace

// the conv stack's weight gradients (MN-contiguous bf16 planes, gemm.hip use_hbt4) on the four-phase 256 x 256 kernel's
// TN form: fp32 C only, the plain / bias / residual class, no split-K, the staged C^T epilogue's operand conditions
bool hbt4_ok(const GemmParams& p) {
    return suta_switches().hbt4 && p.ta && !p.tb && p.Ab && p.Bb && !p.Cb && p.segK == 0 && p.zdiv == 1 &&
           p.splits <= 1 && (p.epi & ~(EPI_BIAS | EPI_RESID | EPI_ROWMASK)) == 0 && hbx_t_ok(p, true);
}
void gemm_run_hbt4(const GemmParams& p, dim3 grid, hipStream_t st) {
    if (!hbt4_ok(p)) throw std::invalid_argument("hbt4: outside the TN form's conditions");
    hipLaunchKernelGGL((gemm_hbp_kernel<false, EPI_BIAS | EPI_RESID | EPI_ROWMASK, 4, false, 0, true>), grid, dim3(512),
                       0, st, p);
}

// variant 1: v_mfma_f32_32x32x16_bf16 with the shared epilogue (class-specialised kernels for the linears' epilogue
// classes, the generic one otherwise); 2: v_mfma_f32_16x16x32_bf16 with epilogue16 (the linears' classes only)
void gemm_run_hbx(int variant, const GemmParams& p, dim3 grid, hipStream_t st) {
    const int e = p.epi;
    if (p.splits > 1 || (e & (EPI_ACCUM | EPI_SMBWD)))
        throw std::invalid_argument("hbx: no split-K, ACCUM or SMBWD");
    if (p.Z != 1 && !(variant == 1 && suta_switches().hbx_form && suta_switches().hbx_t == 2 && p.K % 64 == 0 &&
                      hbx_t_ok(p, true) && !hbx_diag()))
        throw std::invalid_argument("hbx: batched GEMMs only on the four-phase form with the staged C^T epilogue");
    if (p.segK > 0) {  // conv-A rows: the four-phase form's CONV instantiation (gemm.hip hbp_conv_ok)
        if (!hbp_conv_ok(p)) throw std::invalid_argument("hbx: conv-A GEMM outside the four-phase CONV form's conditions");
        if (suta_switches().hbx_form >= 4) {
            if (p.Cb) hipLaunchKernelGGL((gemm_hbp_kernel<true, XEM_A, 4, true>), grid, dim3(512), 0, st, p);
            else hipLaunchKernelGGL((gemm_hbp_kernel<false, XEM_A, 4, true>), grid, dim3(512), 0, st, p);
        } else if (suta_switches().hbx_form == 3) {
            if (p.Cb) hipLaunchKernelGGL((gemm_hbp_kernel<true, XEM_A, 3, true>), grid, dim3(512), 0, st, p);
            else hipLaunchKernelGGL((gemm_hbp_kernel<false, XEM_A, 3, true>), grid, dim3(512), 0, st, p);
        } else {
            if (p.Cb) hipLaunchKernelGGL((gemm_hbp_kernel<true, XEM_A, 2, true>), grid, dim3(512), 0, st, p);
            else hipLaunchKernelGGL((gemm_hbp_kernel<false, XEM_A, 2, true>), grid, dim3(512), 0, st, p);
        }
        return;
    }
    if ((e & EPI_DELTA) && !(variant == 1 && suta_switches().hbx_t && hbx_t_ok(p, true)))
        throw std::invalid_argument("hbx: EPI_DELTA needs the C^T epilogue and its operand conditions");
    if (variant == 2) {
        if ((e & ~XEM_A) == 0) launch_hbx_em<16, XEM_A>(p, grid, st);
        else if ((e & ~XEM_G) == 0) launch_hbx_em<16, XEM_G>(p, grid, st);
        else if ((e & ~XEM_D) == 0) launch_hbx_em<16, XEM_D>(p, grid, st);
        else throw std::invalid_argument("hbx 16x16: epilogue flags outside the linears' classes");
        return;
    }
    const int tr = suta_switches().hbx_t;
    const int dbg = hbx_diag();
    // SUTA_HBX_FORM 4 (default): the 16x16x32 form on every shape (tools/hb_bench, profiles/r6/hb16.txt: +8-14 % on
    // the QKV, FFN1, FFN2 and dQKV shapes, the N = K = 1024 out-projection -4 % alone; in the C4 loop every shape on
    // form 4 measured +0.3 % over keeping form 3 for that one, profiles/r6/conv16)
    const int form = suta_switches().hbx_form;
    if (form && tr == 2 && p.K % 64 == 0 && hbx_t_ok(p, true) && !dbg) {  // the four-phase K-tile schedule
        const bool cb = p.Cb != nullptr;
#define HBP(EM_)                                                                                                   \
        do {                                                                                                       \
            if (form == 4) {                                                                                       \
                if (cb) hipLaunchKernelGGL((gemm_hbp_kernel<true, EM_, 4>), grid, dim3(512), 0, st, p);            \
                else hipLaunchKernelGGL((gemm_hbp_kernel<false, EM_, 4>), grid, dim3(512), 0, st, p);              \
            } else if (form == 3) {                                                                                \
                if (cb) hipLaunchKernelGGL((gemm_hbp_kernel<true, EM_, 3>), grid, dim3(512), 0, st, p);            \
                else hipLaunchKernelGGL((gemm_hbp_kernel<false, EM_, 3>), grid, dim3(512), 0, st, p);              \
            } else if (form == 2) {                                                                                \
                if (cb) hipLaunchKernelGGL((gemm_hbp_kernel<true, EM_, 2>), grid, dim3(512), 0, st, p);            \
                else hipLaunchKernelGGL((gemm_hbp_kernel<false, EM_, 2>), grid, dim3(512), 0, st, p);              \
            } else {                                                                                               \
                if (cb) hipLaunchKernelGGL((gemm_hbp_kernel<true, EM_, 1>), grid, dim3(512), 0, st, p);            \
                else hipLaunchKernelGGL((gemm_hbp_kernel<false, EM_, 1>), grid, dim3(512), 0, st, p);              \
            }                                                                                                      \
            return;                                                                                                \
        } while (0)
        if (e == XEM_L) HBP(XEM_L);
        if ((e & ~XEM_A) == 0) HBP(XEM_A);
        if ((e & ~XEM_G) == 0) HBP(XEM_G);
        if ((e & ~XEM_D) == 0) HBP(XEM_D);
#undef HBP
    }
#ifdef SUTA_HBX_DIAG
    if (dbg >= 11 && dbg <= 17 && (e & ~XEM_A) == 0) {  // tools/hb_bench: gemm_hbp_kernel form 4 diagnostics
        const bool cb = p.Cb != nullptr;
#define HBP_DBG(D)                                                                                                 \
        do {                                                                                                       \
            if (cb) hipLaunchKernelGGL((gemm_hbp_kernel<true, XEM_A, 4, false, D>), grid, dim3(512), 0, st, p);    \
            else hipLaunchKernelGGL((gemm_hbp_kernel<false, XEM_A, 4, false, D>), grid, dim3(512), 0, st, p);      \
        } while (0)
        if (dbg == 11) HBP_DBG(1);
        else if (dbg == 12) HBP_DBG(2);
        else if (dbg == 13) HBP_DBG(3);
        else if (dbg == 14) HBP_DBG(20);
        else if (dbg == 15) HBP_DBG(8);
        else if (dbg == 16) HBP_DBG(16);
        else HBP_DBG(32);
#undef HBP_DBG
        return;
    }
    if (dbg && tr == 2 && hbx_t_ok(p, true) && (e & ~XEM_A) == 0) {  // tools/hb_bench diagnostics
        const bool cb = p.Cb != nullptr;
#define HBX_DBG(D)                                                                                                 \
        do {                                                                                                       \
            if (cb) hipLaunchKernelGGL((gemm_hbx_kernel<32, true, XEM_A, 2, D>), grid, dim3(512), 0, st, p);       \
            else hipLaunchKernelGGL((gemm_hbx_kernel<32, false, XEM_A, 2, D>), grid, dim3(512), 0, st, p);         \
        } while (0)
        if (dbg == 1) HBX_DBG(1);
        else if (dbg == 2) HBX_DBG(2);
        else if (dbg == 3) HBX_DBG(3);
        else if (dbg == 4) HBX_DBG(4);
        else HBX_DBG(5);
#undef HBX_DBG
        return;
    }
#endif
    if (tr && hbx_t_ok(p, true)) {  // C^T accumulators, row-per-lane epilogue (2: LDS-staged whole-line stores)
        if (tr == 2) {
            if (e == XEM_L) return launch_hbx_em<32, XEM_L, 2>(p, grid, st);
            if ((e & ~XEM_A) == 0) return launch_hbx_em<32, XEM_A, 2>(p, grid, st);
            if ((e & ~XEM_G) == 0) return launch_hbx_em<32, XEM_G, 2>(p, grid, st);
            if ((e & ~XEM_D) == 0) return launch_hbx_em<32, XEM_D, 2>(p, grid, st);
        }
        if (e == XEM_L) return launch_hbx_em<32, XEM_L, 1>(p, grid, st);
        if ((e & ~XEM_A) == 0) return launch_hbx_em<32, XEM_A, 1>(p, grid, st);
        if ((e & ~XEM_G) == 0) return launch_hbx_em<32, XEM_G, 1>(p, grid, st);
        if ((e & ~XEM_D) == 0) return launch_hbx_em<32, XEM_D, 1>(p, grid, st);
    }
    if ((e & ~XEM_A) == 0) launch_hbx_em<32, XEM_A>(p, grid, st);
    else if ((e & ~XEM_G) == 0) launch_hbx_em<32, XEM_G>(p, grid, st);
    else if ((e & ~XEM_D) == 0) launch_hbx_em<32, XEM_D>(p, grid, st);
    else launch_hbx_em<32, -1>(p, grid, st);
}
