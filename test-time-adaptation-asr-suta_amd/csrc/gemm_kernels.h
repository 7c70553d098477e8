// GEMM kernel templates shared by the gemm*.hip translation units (one TU per kernel family, so
// the families compile in parallel).  Included only by gemm*.hip.
// fp32 MFMA GEMM for gfx950 (v_mfma_f32_32x32x2_f32: exact f32 products, f32 accumulate).
//
// One kernel template serves every contraction of the SUTA step: encoder linears (NT),
// their input-gradients (NN), attention QK^T / PV and their backward (NT / NN / TN),
// feature-encoder convs as strided-row GEMMs (time-major activations make the im2col
// matrix a plain matrix with lda = stride*C), their weight gradients (TN, split-K over
// time), and the grouped positional conv through the conv-A (segmented K) loader.
//
// Block = 256 threads = 4 waves (2 x 2), block tile BM x BN, K-step 32.  Each operand is
// staged through LDS in the layout its global source makes conflict-free:
//   k-contiguous source  -> LDS [row][32 + 4]  (16-B writes; 16-B fragment reads, row stride
//                           36 dwords: conflict-free over the ds_read_b128 lane groups)
//   row-contiguous source -> LDS [k][ROWS]    (16-B writes; 4-B fragment reads by 32
//                           consecutive rows: conflict-free)
// The MFMA k-pair (lane half h) takes tile-k h*16 + 4q + e, so a k-contiguous fragment is
// one 16-B read per 4 MFMA k-steps.  Global->register prefetch of stage s+1 overlaps the
// MFMAs of stage s; with two LDS buffers there is one barrier per K-step.
#include "common.h"
#include <algorithm>
#include <stdexcept>

#pragma once

namespace {


constexpr int BK = 32;
constexpr int LDK = BK + 4;

template <int ROWS>
struct Op {
    static constexpr int LOADS = ROWS * BK / 4 / 256;  // float4 per thread per stage
    static constexpr int KC_FLOATS = ROWS * LDK;
    static constexpr int MN_FLOATS = BK * ROWS;
};

template <int ROWS, bool KC>
constexpr int lds_floats() {
    return KC ? Op<ROWS>::KC_FLOATS : Op<ROWS>::MN_FLOATS;
}

// Load one BK-deep stage of an operand into registers.
//   KC = true : element (row, k) at row*ld + k   (A with ta=0, B with tb=1)
//   KC = false: element (row, k) at k*ld + row   (A with ta=1, B with tb=0)
// MODE 0: plain; 1: conv-A (segment shifts the source row by seg - pad, rows outside
// [0, Mvalid) read as zero); 2: segmented B (segment offsets the source by seg * sseg).
template <int ROWS, bool KC, int MODE>
__device__ __forceinline__ void load_stage(f32x4 (&r)[Op<ROWS>::LOADS], const float* __restrict__ src, long ld,
                                           int row0, int nrows, int k0, int kend, bool vec, int segK, int pad,
                                           int Mvalid, long sseg) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < Op<ROWS>::LOADS; ++i) {
        const int f = tid + i * 256;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (KC) {
            const int row = f >> 3;
            const int kq = (f & 7) * 4;
            const int gr = row0 + row;
            const int gk = k0 + kq;
            if (gr < nrows && gk < kend) {
                const float* s;
                bool ok = true;
                if (MODE == 1) {
                    const int seg = gk / segK;
                    const int srow = gr + seg - pad;
                    ok = srow >= 0 && srow < Mvalid;
                    s = src + (long)srow * ld + (gk - seg * segK);  // segK % 4 == 0: one segment
                } else if (MODE == 2) {
                    const int seg = gk / segK;
                    s = src + (long)gr * ld + seg * sseg + (gk - seg * segK);
                } else {
                    s = src + (long)gr * ld + gk;
                }
                if (ok) {
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
            if (gk < kend && gr < nrows) {
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

// Interior fast path: the whole ROWS x BK stage is in bounds and 16-B aligned (no predicates).
template <int ROWS, bool KC>
__device__ __forceinline__ void load_stage_full(f32x4 (&r)[Op<ROWS>::LOADS], const float* __restrict__ src, long ld,
                                                int row0, int k0) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < Op<ROWS>::LOADS; ++i) {
        const int f = tid + i * 256;
        if (KC) {
            r[i] = *reinterpret_cast<const f32x4*>(src + (long)(row0 + (f >> 3)) * ld + k0 + (f & 7) * 4);
        } else {
            constexpr int RQ = ROWS / 4;
            r[i] = *reinterpret_cast<const f32x4*>(src + (long)(k0 + f / RQ) * ld + row0 + (f % RQ) * 4);
        }
    }
}

template <int ROWS, bool KC>
__device__ __forceinline__ void store_stage(float* __restrict__ lds, const f32x4 (&r)[Op<ROWS>::LOADS]) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < Op<ROWS>::LOADS; ++i) {
        const int f = tid + i * 256;
        if (KC) {
            *reinterpret_cast<f32x4*>(lds + (f >> 3) * LDK + (f & 7) * 4) = r[i];
        } else {
            constexpr int RQ = ROWS / 4;
            *reinterpret_cast<f32x4*>(lds + (f / RQ) * ROWS + (f % RQ) * 4) = r[i];
        }
    }
}

// fragment of 4 consecutive MFMA k-steps (tile k = h*16 + 4q + e, e < 4) for MFMA row `row`
template <int ROWS, bool KC>
__device__ __forceinline__ f32x4 read_frag(const float* __restrict__ lds, int row, int h, int q) {
    if (KC) return *reinterpret_cast<const f32x4*>(lds + row * LDK + h * 16 + q * 4);
    f32x4 v;
    const int k = h * 16 + q * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = lds[(k + e) * ROWS + row];
    return v;
}

// Epilogue arithmetic on operands already in registers (xa = aux, xr = R, xc = old C, xw = rowv).
__device__ __forceinline__ float epi_apply(int epi, float alpha, float acc, float bj, float xa, float xr, float xc,
                                           float xw, float* c2) {
    if (epi & EPI_SMBWD) return alpha * (xa * (acc - xw));
    float v = acc * alpha;
    if (epi & EPI_BIAS) v += bj;
    if (epi & EPI_ACCUM) v += xc;
    if (epi & EPI_STORE_PRE) *c2 = v;
    if (epi & EPI_GELU) v = gelu_f(v);
    if (epi & EPI_DGELU) v *= dgelu_f(xa);
    if (epi & EPI_RESID) v += xr;
    return v;
}

__device__ __forceinline__ float epi_value(const GemmParams& p, float acc, long row, long col, const float* bias,
                                           const float* R, const float* aux, float* C2, const float* Cold,
                                           const float* rowv) {
    const int e = p.epi;
    return epi_apply(e, p.alpha, acc, (e & EPI_BIAS) ? bias[col] : 0.f,
                     (e & (EPI_DGELU | EPI_SMBWD)) ? aux[row * p.ldaux + col] : 0.f,
                     (e & EPI_RESID) ? R[row * p.ldr + col] : 0.f, (e & EPI_ACCUM) ? Cold[row * p.ldc + col] : 0.f,
                     (e & EPI_SMBWD) ? rowv[row] : 0.f, C2 ? C2 + row * p.ldc2 + col : nullptr);
}

// XCD-aware tile order (cdna_hip_programming.md T1, bijective form): blocks are dealt round-robin over
// the 8 XCDs, so block b is renumbered to give every XCD one contiguous range of tiles (n fastest, then
// m, then batch/split) -- the tiles that share an A row panel run on one L2.  Speed only.
struct TileId {
    int x, y, z;
};
// tile of remapped id `id` in a gx x gy (x Z) grid, in the tile order `order`
__device__ __forceinline__ TileId tile_of_id(int id, int gx, int gy, int order) {
    if (order == 1) return TileId{(id / gy) % gx, id % gy, id / (gx * gy)};  // m fastest: an XCD keeps a B band
    if (order >= 2) {  // grouped: bands of `order` tile rows walked column by column (A and B panels both reused)
        const int zid = id / (gx * gy), i2 = id % (gx * gy);
        const int per = order * gx, fm = (i2 / per) * order, gsz = min(gy - fm, order), loc = i2 % per;
        return TileId{loc / gsz, fm + loc % gsz, zid};
    }
    return TileId{id % gx, (id / gx) % gy, id / (gx * gy)};
}
__device__ __forceinline__ TileId xcd_tile(int order = 0) {
    const int gx = gridDim.x, gy = gridDim.y;
    const int nwg = gx * gy * gridDim.z;
    const int orig = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
    return tile_of_id(id, gx, gy, order);
}

// Interior-tile epilogue with 32-bit offsets (p.off32: every operand's rows x leading dimension fits 4 GiB):
// element r of a fragment sits at row rb + ro(r), ro(r) = (r & 3) + 8 (r >> 2) the same for every lane, so its
// address is a wave-uniform base (operand + ro(r) x ld, scalar arithmetic) plus the lane's 32-bit byte offset of
// row rb (one multiply per fragment): the stores and operand loads take the scalar-base + vector-offset form
// and cost no per-element address arithmetic (the general epilogue below spends ~15 VALU per element on
// 64-bit addresses).  Same operations in the same order as the general epilogue.
template <typename T>
__device__ __forceinline__ T* byte_at(T* base, unsigned off) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off);
}
template <typename T>
__device__ __forceinline__ const T* byte_at(const T* base, unsigned off) {
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + off);
}

// EM: the epilogue flags a kernel instantiation can see (p.epi & EM; -1 = all): class-specialised kernels carry
// only their own epilogue code
template <int RM, int RN, bool CB, int EM = -1>
__device__ __forceinline__ void gemm_epilogue_fast(const GemmParams& p, const f32x16 (&acc)[RM][RN], int z1, int z0,
                                                   int rbase, int cbase, int h, int l32) {
    const int e = p.epi & EM;
    float* C = p.C ? p.C + z1 * p.sC1 + z0 * p.sC0 : nullptr;
    const float* bias = p.bias ? p.bias + z1 * p.sBias1 + z0 * p.sBias0 : nullptr;
    const float* aux = p.aux ? p.aux + z1 * p.sAux1 + z0 * p.sAux0 : nullptr;
    const int rlim = (e & EPI_ROWMASK) ? p.zrows[z1] : 0x7fffffff;
    float* C2 = p.C2 ? p.C2 + z1 * p.sC21 + z0 * p.sC20 : nullptr;
    const float* Q = nullptr;
    long ldq = 0;
    if (e & EPI_RESID) {
        Q = p.R + z1 * p.sR1 + z0 * p.sR0;
        ldq = p.ldr;
    } else if (e & EPI_ACCUM) {
        Q = C;
        ldq = p.ldc;
    } else if (e & EPI_SMBWD) {
        Q = p.rowv + z1 * p.sRow1 + z0 * p.sRow0;
    }
    const float alpha = p.alpha;
    const bool cbpair = CB && (p.ldcb & 1) == 0;
    const bool odd = l32 & 1;
    const bool preb = CB && p.preb;  // bf16 pre-activation store / DGELU operand
    const __bf16* auxh = preb && p.aux ? reinterpret_cast<const __bf16*>(p.aux) + z1 * p.sAux1 + z0 * p.sAux0 : nullptr;
    __bf16* C2h = preb && p.C2 ? reinterpret_cast<__bf16*>(p.C2) + z1 * p.sC21 + z0 * p.sC20 : nullptr;
    typedef __bf16 cb2 __attribute__((ext_vector_type(2)));
    constexpr int CH = 8;
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) {
            const unsigned rb = rbase + i * 32 + 4 * h;
            const unsigned col = cbase + j * 32 + l32;
            const unsigned oc = 4u * (rb * (unsigned)p.ldc + col);
            const unsigned oq = (e & EPI_SMBWD) ? 4u * rb : 4u * (rb * (unsigned)ldq + col);
            const unsigned oa = 4u * (rb * (unsigned)p.ldaux + col);
            const unsigned o2 = 4u * (rb * (unsigned)p.ldc2 + col);
            const unsigned ob = 2u * ((rb + (odd ? 1u : 0u)) * (unsigned)p.ldcb + (col & ~1u));
            const unsigned oah = 2u * (rb * (unsigned)p.ldaux + col);
            const unsigned o2h = 2u * ((rb + (odd ? 1u : 0u)) * (unsigned)p.ldc2 + (col & ~1u));
            const float bj = (e & EPI_BIAS) ? bias[col] : 0.f;
#pragma unroll
            for (int r0 = 0; r0 < 16; r0 += CH) {
                float v[CH], xa[CH], xq[CH];
                // (the bf16 / fp32 choice is hoisted out of the element loop: a per-element select branches around
                // every load and waits for each one)
                if ((e & EPI_DGELU) && preb) {
#pragma unroll
                    for (int r = 0; r < CH; ++r) {
                        const int ro = ((r0 + r) & 3) + 8 * ((r0 + r) >> 2);
                        xa[r] = (float)*byte_at(auxh + ro * p.ldaux, oah);
                    }
                } else if (e & (EPI_DGELU | EPI_SMBWD)) {
#pragma unroll
                    for (int r = 0; r < CH; ++r) {
                        const int ro = ((r0 + r) & 3) + 8 * ((r0 + r) >> 2);
                        xa[r] = *byte_at(aux + ro * p.ldaux, oa);
                    }
                }
                if (Q) {
#pragma unroll
                    for (int r = 0; r < CH; ++r) {
                        const int ro = ((r0 + r) & 3) + 8 * ((r0 + r) >> 2);
                        xq[r] = (e & EPI_SMBWD) ? *byte_at(Q + ro, oq) : *byte_at(Q + ro * ldq, oq);
                    }
                }
                if (e & EPI_SMBWD) {
#pragma unroll
                    for (int r = 0; r < CH; ++r) v[r] = alpha * (xa[r] * (acc[i][j][r0 + r] - xq[r]));
                } else {
#pragma unroll
                    for (int r = 0; r < CH; ++r) v[r] = acc[i][j][r0 + r] * alpha;
                    if (e & EPI_BIAS) {
#pragma unroll
                        for (int r = 0; r < CH; ++r) v[r] += bj;
                    }
                    if (e & EPI_ACCUM) {
#pragma unroll
                        for (int r = 0; r < CH; ++r) v[r] += xq[r];
                    }
                    if ((e & EPI_STORE_PRE) && preb) {
                        // (column, column + 1) bf16 pairs, as the Cb store below
#pragma unroll
                        for (int r = 0; r < CH; r += 2) {
                            const int ro = ((r0 + r) & 3) + 8 * ((r0 + r) >> 2);
                            const float a = v[r], b = v[r + 1];
                            const float q = __int_as_float(
                                __builtin_amdgcn_mov_dpp(__float_as_int(odd ? a : b), 0xB1, 0xF, 0xF, false));
                            cb2 pr;
                            pr[0] = (__bf16)(odd ? q : a);
                            pr[1] = (__bf16)(odd ? b : q);
                            *reinterpret_cast<cb2*>(byte_at(C2h + ro * p.ldc2, o2h)) = pr;
                        }
                    } else if (e & EPI_STORE_PRE) {
#pragma unroll
                        for (int r = 0; r < CH; ++r) {
                            const int ro = ((r0 + r) & 3) + 8 * ((r0 + r) >> 2);
                            *byte_at(C2 + ro * p.ldc2, o2) = v[r];
                        }
                    }
                    if ((e & EPI_GELU) && CB && p.fgelu) {  // (uniform choice hoisted out of the element loop)
#pragma unroll
                        for (int r = 0; r < CH; r += 2) {
                            const f32x2v g = gelu2_bf16ep(f32x2v{v[r], v[r + 1]});
                            v[r] = g.x;
                            v[r + 1] = g.y;
                        }
                    } else if (e & EPI_GELU) {
#pragma unroll
                        for (int r = 0; r < CH; ++r) v[r] = gelu_f(v[r]);
                    }
                    if ((e & EPI_DGELU) && CB && p.fgelu) {  // (uniform choice hoisted out of the element loop)
#pragma unroll
                        for (int r = 0; r < CH; r += 2) {
                            const f32x2v g = dgelu2_bf16ep(f32x2v{xa[r], xa[r + 1]});
                            v[r] *= g.x;
                            v[r + 1] *= g.y;
                        }
                    } else if (e & EPI_DGELU) {
#pragma unroll
                        for (int r = 0; r < CH; ++r) v[r] *= dgelu_f(xa[r]);
                    }
                    if (e & EPI_RESID) {
#pragma unroll
                        for (int r = 0; r < CH; ++r) v[r] += xq[r];
                    }
                }
                if (e & EPI_ROWMASK) {
#pragma unroll
                    for (int r = 0; r < CH; ++r) {
                        const int ro = ((r0 + r) & 3) + 8 * ((r0 + r) >> 2);
                        if ((int)rb + ro >= rlim) v[r] = 0.f;
                    }
                }
                if (!CB || C) {
#pragma unroll
                    for (int r = 0; r < CH; ++r) {
                        const int ro = ((r0 + r) & 3) + 8 * ((r0 + r) >> 2);
                        *byte_at(C + ro * p.ldc, oc) = v[r];
                    }
                }
                if (CB) {
                    __bf16* Cb = reinterpret_cast<__bf16*>(p.Cb) + z1 * p.sCb1;
                    if (cbpair) {
                        // (column, column + 1) pairs: lanes 2i / 2i + 1 swap one value (DPP quad_perm [1,0,3,2]);
                        // the even lane writes row r, the odd lane row r + 1 (registers r, r + 1: consecutive rows)
#pragma unroll
                        for (int r = 0; r < CH; r += 2) {
                            const int ro = ((r0 + r) & 3) + 8 * ((r0 + r) >> 2);
                            const float a = v[r], b = v[r + 1];
                            const float q = __int_as_float(
                                __builtin_amdgcn_mov_dpp(__float_as_int(odd ? a : b), 0xB1, 0xF, 0xF, false));
                            cb2 pr;
                            pr[0] = (__bf16)(odd ? q : a);
                            pr[1] = (__bf16)(odd ? b : q);
                            *reinterpret_cast<cb2*>(byte_at(Cb + ro * p.ldcb, ob)) = pr;
                        }
                    } else {
#pragma unroll
                        for (int r = 0; r < CH; ++r) {
                            const int ro = ((r0 + r) & 3) + 8 * ((r0 + r) >> 2);
                            Cb[(long)(rb + ro) * p.ldcb + col] = (__bf16)v[r];
                        }
                    }
                }
            }
        }
}

// Store the wave's RM x RN 32x32 accumulator fragments (MFMA 32x32 output layout: lane -> column,
// register r -> row (r&3) + 8(r>>2) + 4h).  Flags are block-uniform, so each epilogue step is one
// uniform branch per fragment rather than per element; operand loads use clamped (always valid)
// indices so they are unpredicated, and every operand of a fragment is in registers before its first
// store (C may alias aux / R in place).  Only the stores are predicated, and only on edge tiles.
// gemm_launch guarantees RESID, ACCUM and SMBWD are mutually exclusive (they share xq).
template <int RM, int RN, bool CB = false, int EM = -1>
__device__ __forceinline__ void gemm_epilogue(const GemmParams& p, const f32x16 (&acc)[RM][RN], int z1, int z0,
                                              int rbase, int cbase, int h, int l32, bool interior, int tz) {
    if (p.splits > 1) {
        float* W = p.ws + ((long)tz) * p.M * (long)p.N;
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int j = 0; j < RN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = rbase + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const int col = cbase + j * 32 + l32;
                    if (interior || (row < p.M && col < p.N)) W[(long)row * p.N + col] = acc[i][j][r];
                }
        return;
    }
    if (interior && p.off32) {
        gemm_epilogue_fast<RM, RN, CB, EM>(p, acc, z1, z0, rbase, cbase, h, l32);
        return;
    }
    const int e = p.epi & EM;
    float* C = p.C + z1 * p.sC1 + z0 * p.sC0;
    const float* bias = p.bias ? p.bias + z1 * p.sBias1 + z0 * p.sBias0 : nullptr;
    const float* aux = p.aux ? p.aux + z1 * p.sAux1 + z0 * p.sAux0 : nullptr;
    const int rlim = (e & EPI_ROWMASK) ? p.zrows[z1] : p.M;
    float* C2 = p.C2 ? p.C2 + z1 * p.sC21 + z0 * p.sC20 : nullptr;
    const bool preb = CB && p.preb;  // bf16 pre-activation store / DGELU operand
    const __bf16* auxh = preb && p.aux ? reinterpret_cast<const __bf16*>(p.aux) + z1 * p.sAux1 + z0 * p.sAux0 : nullptr;
    __bf16* C2h = preb && p.C2 ? reinterpret_cast<__bf16*>(p.C2) + z1 * p.sC21 + z0 * p.sC20 : nullptr;
    // second operand: R (RESID), old C (ACCUM) or the row vector (SMBWD)
    const float* Q = nullptr;
    long ldq = 0, colq = 1;
    if (e & EPI_RESID) {
        Q = p.R + z1 * p.sR1 + z0 * p.sR0;
        ldq = p.ldr;
    } else if (e & EPI_ACCUM) {
        Q = C;
        ldq = p.ldc;
    } else if (e & EPI_SMBWD) {
        Q = p.rowv + z1 * p.sRow1 + z0 * p.sRow0;
        ldq = 1;
        colq = 0;
    }
    const float alpha = p.alpha;
#ifndef GEMM_EPI_CH
#define GEMM_EPI_CH 8
#endif
    constexpr int CH = GEMM_EPI_CH;  // elements per epilogue chunk (bounds the extra live registers to 3 x CH)
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int r0 = 0; r0 < 16; r0 += CH) {
                const int col = cbase + j * 32 + l32;
                const long colc = min(col, p.N - 1);
                float v[CH], xa[CH], xq[CH];
                if ((e & EPI_DGELU) && preb) {
#pragma unroll
                    for (int r = 0; r < CH; ++r) {
                        const int rr = r0 + r;
                        const long row = min(rbase + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * h, p.M - 1);
                        xa[r] = (float)auxh[row * p.ldaux + colc];
                    }
                } else if (e & (EPI_DGELU | EPI_SMBWD)) {
#pragma unroll
                    for (int r = 0; r < CH; ++r) {
                        const int rr = r0 + r;
                        const long row = min(rbase + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * h, p.M - 1);
                        xa[r] = aux[row * p.ldaux + colc];
                    }
                }
                if (Q) {
#pragma unroll
                    for (int r = 0; r < CH; ++r) {
                        const int rr = r0 + r;
                        const long row = min(rbase + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * h, p.M - 1);
                        xq[r] = Q[row * ldq + colc * colq];
                    }
                }
                if (e & EPI_SMBWD) {
#pragma unroll
                    for (int r = 0; r < CH; ++r) v[r] = alpha * (xa[r] * (acc[i][j][r0 + r] - xq[r]));
                } else {
#pragma unroll
                    for (int r = 0; r < CH; ++r) v[r] = acc[i][j][r0 + r] * alpha;
                    if (e & EPI_BIAS) {
                        const float bj = bias[colc];
#pragma unroll
                        for (int r = 0; r < CH; ++r) v[r] += bj;
                    }
                    if (e & EPI_ACCUM) {
#pragma unroll
                        for (int r = 0; r < CH; ++r) v[r] += xq[r];
                    }
                    if (e & EPI_STORE_PRE) {
#pragma unroll
                        for (int r = 0; r < CH; ++r) {
                            const int rr = r0 + r;
                            const int row = rbase + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * h;
                            if (interior || (row < p.M && col < p.N)) {
                                if (preb) C2h[(long)row * p.ldc2 + col] = (__bf16)v[r];
                                else C2[(long)row * p.ldc2 + col] = v[r];
                            }
                        }
                    }
                    if ((e & EPI_GELU) && CB && p.fgelu) {  // (uniform choice hoisted out of the element loop)
#pragma unroll
                        for (int r = 0; r < CH; r += 2) {
                            const f32x2v g = gelu2_bf16ep(f32x2v{v[r], v[r + 1]});
                            v[r] = g.x;
                            v[r + 1] = g.y;
                        }
                    } else if (e & EPI_GELU) {
#pragma unroll
                        for (int r = 0; r < CH; ++r) v[r] = gelu_f(v[r]);
                    }
                    if ((e & EPI_DGELU) && CB && p.fgelu) {  // (uniform choice hoisted out of the element loop)
#pragma unroll
                        for (int r = 0; r < CH; r += 2) {
                            const f32x2v g = dgelu2_bf16ep(f32x2v{xa[r], xa[r + 1]});
                            v[r] *= g.x;
                            v[r + 1] *= g.y;
                        }
                    } else if (e & EPI_DGELU) {
#pragma unroll
                        for (int r = 0; r < CH; ++r) v[r] *= dgelu_f(xa[r]);
                    }
                    if (e & EPI_RESID) {
#pragma unroll
                        for (int r = 0; r < CH; ++r) v[r] += xq[r];
                    }
                }
#pragma unroll
                for (int r = 0; r < CH; ++r) {
                    const int rr = r0 + r;
                    const int row = rbase + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * h;
                    if (interior || (row < p.M && col < p.N)) {
                        const float o = row < rlim ? v[r] : 0.f;
                        if (!CB || p.C) C[(long)row * p.ldc + col] = o;  // bf16-plane GEMMs: C may be dead
                        if (CB && !(interior && (p.ldcb & 1) == 0))
                            (reinterpret_cast<__bf16*>(p.Cb) + z1 * p.sCb1)[(long)row * p.ldcb + col] = (__bf16)o;
                    }
                }
                if (CB && interior && (p.ldcb & 1) == 0) {
                    // bf16 copy as (column, column + 1) pairs: lanes 2i / 2i + 1 swap one value (DPP quad_perm
                    // [1,0,3,2]); the even lane writes row r, the odd lane row r + 1 (registers rr, rr + 1 hold
                    // consecutive rows): half the store instructions of one 2-byte store per element
                    typedef __bf16 cb2 __attribute__((ext_vector_type(2)));
                    const bool odd = l32 & 1;
#pragma unroll
                    for (int r = 0; r < CH; r += 2) {
                        const int rr = r0 + r;
                        const int row = rbase + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * h;
                        const float a = row < rlim ? v[r] : 0.f, b = row + 1 < rlim ? v[r + 1] : 0.f;
                        const float q = __int_as_float(
                            __builtin_amdgcn_mov_dpp(__float_as_int(odd ? a : b), 0xB1, 0xF, 0xF, false));
                        cb2 pr;
                        pr[0] = (__bf16)(odd ? q : a);
                        pr[1] = (__bf16)(odd ? b : q);
                        *reinterpret_cast<cb2*>(reinterpret_cast<__bf16*>(p.Cb) + z1 * p.sCb1 +
                                                (long)(row + (odd ? 1 : 0)) * p.ldcb + (col & ~1)) = pr;
                    }
                }
            }
}

template <int BM, int BN, bool TA, bool TB, bool CONV, bool SEGB, int NBUF>
#ifndef GEMM_ABL
#define GEMM_ABL 0  // benchmark-only ablations (wrong results): 1 no global loads, 2 1/4 LDS reads, 4 no barriers
#endif
#ifndef GEMM_F32_MINB
#define GEMM_F32_MINB 3
#endif
__global__ __launch_bounds__(256, GEMM_F32_MINB) void gemm_f32_kernel(GemmParams p) {
    constexpr int WTM = BM / 2, WTN = BN / 2;
    constexpr int RM = WTM / 32, RN = WTN / 32;
    constexpr bool AKC = !TA, BKC = TB;
    constexpr int A_FL = lds_floats<BM, AKC>(), B_FL = lds_floats<BN, BKC>();
    static_assert(RM >= 1 && RN >= 1, "wave tile >= 32x32");
    __shared__ __attribute__((aligned(16))) float smem[NBUF * (A_FL + B_FL)];

    const TileId tid = xcd_tile();
    int zz = tid.z;
    int split = 0;
    if (p.splits > 1) {
        split = zz % p.splits;
        zz /= p.splits;
    }
    const int z1 = zz / p.zdiv, z0 = zz % p.zdiv;
    const int Mv = p.zmvalid ? p.zmvalid[z1] : p.Mvalid;  // conv-A valid source rows
    const float* A = p.A + z1 * p.sA1 + z0 * p.sA0;
    const float* B = p.B + z1 * p.sB1 + z0 * p.sB0;

    const int m0 = tid.y * BM;
    const int n0 = tid.x * BN;
    const int kbeg = split * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);

    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int h = lane >> 5, l32 = lane & 31;

    f32x16 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    f32x4 ra[Op<BM>::LOADS];
    f32x4 rb[Op<BN>::LOADS];
    const bool va = p.va != 0, vb = p.vb != 0;

    // block-uniform: interior tiles take the unpredicated 16-B loader for every full K-step;
    // segmented operands qualify when a K-step stays inside one segment (segK % BK == 0)
    const bool segAligned = p.segK > 0 && p.segK % BK == 0;
    auto stageA = [&](int k) {
        bool full = va && m0 + BM <= p.M && k + BK <= kend;
        const float* base = A;
        int kk = k;
        if (CONV) {
            const int seg = segAligned ? k / p.segK : 0;
            const int sh = seg - p.pad;
            full = full && segAligned && m0 + sh >= 0 && m0 + BM + sh <= Mv;
            base = A + (long)sh * p.lda;
            kk = k - seg * p.segK;
        }
        if (full) load_stage_full<BM, AKC>(ra, base, p.lda, m0, kk);
        else load_stage<BM, AKC, CONV ? 1 : 0>(ra, A, p.lda, m0, p.M, k, kend, va, p.segK, p.pad, Mv, 0);
    };
    auto stageB = [&](int k) {
        bool full = vb && n0 + BN <= p.N && k + BK <= kend;
        const float* base = B;
        int kk = k;
        if (SEGB) {
            const int seg = segAligned ? k / p.segK : 0;
            full = full && segAligned;
            base = B + seg * p.sBseg;
            kk = k - seg * p.segK;
        }
        if (full) load_stage_full<BN, BKC>(rb, base, p.ldb, n0, kk);
        else load_stage<BN, BKC, SEGB ? 2 : 0>(rb, B, p.ldb, n0, p.N, k, kend, vb, p.segK, 0, 0, p.sBseg);
    };
    stageA(kbeg);
    stageB(kbeg);

    int buf = 0;
    if (NBUF == 2) {
        store_stage<BM, AKC>(smem, ra);
        store_stage<BN, BKC>(smem + A_FL, rb);
        __syncthreads();
    }
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
        const bool more = k0 + BK < kend;
        if (NBUF == 1 && !(GEMM_ABL & 4)) {
            __syncthreads();
            store_stage<BM, AKC>(smem, ra);
            store_stage<BN, BKC>(smem + A_FL, rb);
            __syncthreads();
        }
        if (more && !(GEMM_ABL & 1)) {
            stageA(k0 + BK);
            stageB(k0 + BK);
        }
        const float* As = smem + buf * (A_FL + B_FL);
        const float* Bs = As + A_FL;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f32x4 af[RM], bf[RN];
            const int qq = (GEMM_ABL & 2) ? 0 : q;  // benchmark ablation: one fragment read per K-step
#pragma unroll
            for (int i = 0; i < RM; ++i) af[i] = read_frag<BM, AKC>(As, wm * WTM + i * 32 + l32, h, qq);
#pragma unroll
            for (int j = 0; j < RN; ++j) bf[j] = read_frag<BN, BKC>(Bs, wn * WTN + j * 32 + l32, h, qq);
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < RM; ++i)
#pragma unroll
                    for (int j = 0; j < RN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][e], bf[j][e], acc[i][j], 0, 0, 0);
        }
        if (NBUF == 2 && more) {
            // the other buffer was last read before the previous barrier
            float* nxt = smem + (buf ^ 1) * (A_FL + B_FL);
            store_stage<BM, AKC>(nxt, ra);
            store_stage<BN, BKC>(nxt + A_FL, rb);
            __syncthreads();
            buf ^= 1;
        }
    }

    gemm_epilogue<RM, RN>(p, acc, z1, z0, m0 + wm * WTM, n0 + wn * WTN, h, l32, m0 + BM <= p.M && n0 + BN <= p.N, tid.z);
}

// ============================================================================================
// fp32-accurate GEMM on the bf16 matrix cores ("x6"): every fp32 operand is split exactly into
// three bf16 terms x = x_h + x_m + x_l (24 = 3 x 8 significand bits, each residual exact in fp32),
// and A*B is accumulated in fp32 from the six products whose order is <= 2 (h*h, h*m, m*h, h*l,
// m*m, l*h); the dropped terms are <= 2^-24 |a b|, the size of one fp32 rounding, so the result
// carries the error of an fp32 GEMM (tools/split_accuracy + tests) at 16/6 = 2.7x the fp32-MFMA
// rate.  The split happens once per element when the stage is written to LDS: three bf16 planes
// per operand, rows of 32 k (64 B) with the 16-B chunk XOR-swizzled by (row >> 2) & 3 so the
// ds_read_b128 fragment reads are conflict-free without padding.
// ============================================================================================
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 fbf16x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

template <int ROWS, int BKX>
struct X6 {
    static constexpr int LOADS = ROWS * BKX / 4 / 256;  // float4 per thread per stage
    static constexpr int PLANE = ROWS * BKX;            // bf16 per plane
    static constexpr int KPT = LOADS;                   // MN mapping: k per thread (4 rows each)
    static constexpr int JN = BKX / KPT;                // MN mapping: threads along k
    static constexpr int KQ = BKX / 4;                  // KC mapping: float4 per row
};

// swizzled bf16 index inside a plane: rows of BKX bf16, 16-B chunks XORed so that the
// ds_read_b128 lane groups (rows {0-3,12-15,20-27}+...) hit distinct bank slots
template <int BKX>
__device__ __forceinline__ int x6_idx(int row, int k) {
    if (BKX == 32) return row * 32 + ((((k >> 3) ^ (row >> 2)) & 3) << 3) + (k & 7);
    return row * 16 + ((((k >> 3) ^ (row >> 3)) & 1) << 3) + (k & 7);
}

#ifndef X6_ABLATE
#define X6_ABLATE 0  // benchmark-only ablations: 1 = no split VALU, 2 = one MFMA product instead of six
#endif
__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
#if X6_ABLATE == 1
    m = h;
    l = h;
#else
    const float r = x - (float)h;
    m = (__bf16)r;
    l = (__bf16)(r - (float)m);
#endif
}

// KC (k-contiguous) source: thread -> float4 (row idx / KQ, k 4*(idx % KQ)); MODE as load_stage.
template <int ROWS, int BKX, int MODE, bool FULL>
__device__ __forceinline__ void x6_load_kc(f32x4 (&r)[(X6<ROWS, BKX>::LOADS)], const float* __restrict__ src, long ld,
                                           int row0, int nrows, int k0, int kend, bool vec, int segK, int pad,
                                           int Mvalid, long sseg) {
    constexpr int KQ = X6<ROWS, BKX>::KQ;
#pragma unroll
    for (int i = 0; i < X6<ROWS, BKX>::LOADS; ++i) {
        const int f = threadIdx.x + i * 256;
        const int row = f / KQ, kq = (f % KQ) * 4;
        if (FULL) {
            r[i] = *reinterpret_cast<const f32x4*>(src + (long)(row0 + row) * ld + k0 + kq);
            continue;
        }
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        const int gr = row0 + row, gk = k0 + kq;
        if (gr < nrows && gk < kend) {
            const float* sp;
            bool ok = true;
            if (MODE == 1) {
                const int seg = gk / segK;
                const int srow = gr + seg - pad;
                ok = srow >= 0 && srow < Mvalid;
                sp = src + (long)srow * ld + (gk - seg * segK);
            } else if (MODE == 2) {
                const int seg = gk / segK;
                sp = src + (long)gr * ld + seg * sseg + (gk - seg * segK);
            } else {
                sp = src + (long)gr * ld + gk;
            }
            if (ok) {
                if (vec && gk + 3 < kend) {
                    v = *reinterpret_cast<const f32x4*>(sp);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (gk + e < kend) v[e] = sp[e];
                }
            }
        }
        r[i] = v;
    }
}

// MN (row-contiguous) source, block mapping: thread -> rows 4i..4i+3, k = KPT*j + c.
template <int ROWS, int BKX, bool FULL>
__device__ __forceinline__ void x6_load_mn(f32x4 (&r)[(X6<ROWS, BKX>::LOADS)], const float* __restrict__ src, long ld,
                                           int row0, int nrows, int k0, int kend, bool vec) {
    const int f = threadIdx.x;
    const int i = f / X6<ROWS, BKX>::JN, j = f % X6<ROWS, BKX>::JN;
#pragma unroll
    for (int c = 0; c < X6<ROWS, BKX>::KPT; ++c) {
        const int gk = k0 + X6<ROWS, BKX>::KPT * j + c;
        const int gr = row0 + 4 * i;
        const float* sp = src + (long)gk * ld + gr;
        if (FULL) {
            r[c] = *reinterpret_cast<const f32x4*>(sp);
        } else {
            f32x4 v = {0.f, 0.f, 0.f, 0.f};
            if (gk < kend && gr < nrows) {
                if (vec && gr + 3 < nrows) {
                    v = *reinterpret_cast<const f32x4*>(sp);
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (gr + e < nrows) v[e] = sp[e];
                }
            }
            r[c] = v;
        }
    }
}

template <int N>
struct bfvec;
template <>
struct bfvec<4> {
    typedef bf16x4 T;
};
template <>
struct bfvec<2> {
    typedef bf16x2 T;
};
template <>
struct bfvec<8> {
    typedef bf16x8 T;
};

template <int ROWS, int BKX, bool KC, int NPL>
__device__ __forceinline__ void x6_store(__bf16* __restrict__ lds, const f32x4 (&r)[(X6<ROWS, BKX>::LOADS)]) {
    constexpr int PL = X6<ROWS, BKX>::PLANE;
    const int f = threadIdx.x;
    if (KC) {
        constexpr int KQ = X6<ROWS, BKX>::KQ;
#pragma unroll
        for (int i = 0; i < X6<ROWS, BKX>::LOADS; ++i) {
            const int idx = f + i * 256;
            const int row = idx / KQ, kq = (idx % KQ) * 4;
            bf16x4 hh, mm, ll;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                __bf16 a, b, c;
                split3(r[i][e], a, b, c);
                hh[e] = a;
                mm[e] = b;
                ll[e] = c;
            }
            const int o = x6_idx<BKX>(row, kq);
            *reinterpret_cast<bf16x4*>(lds + o) = hh;
            if (NPL == 3) {
                *reinterpret_cast<bf16x4*>(lds + PL + o) = mm;
                *reinterpret_cast<bf16x4*>(lds + 2 * PL + o) = ll;
            }
        }
    } else if (X6<ROWS, BKX>::KPT == 1) {
        const int i = f / X6<ROWS, BKX>::JN, j = f % X6<ROWS, BKX>::JN;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int o = x6_idx<BKX>(4 * i + rr, j);
            __bf16 a, b, cc;
            split3(r[0][rr], a, b, cc);
            lds[o] = a;
            if (NPL == 3) {
                lds[PL + o] = b;
                lds[2 * PL + o] = cc;
            }
        }
    } else {
        constexpr int KPT = X6<ROWS, BKX>::KPT > 1 ? X6<ROWS, BKX>::KPT : 2;  // 2, 4 or 8
        typedef typename bfvec<KPT>::T V;
        const int i = f / X6<ROWS, BKX>::JN, j = f % X6<ROWS, BKX>::JN;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int o = x6_idx<BKX>(4 * i + rr, KPT * j);
            V hh, mm, ll;
#pragma unroll
            for (int c = 0; c < KPT; ++c) {
                __bf16 a, b, cc;
                split3(r[c][rr], a, b, cc);
                hh[c] = a;
                mm[c] = b;
                ll[c] = cc;
            }
            *reinterpret_cast<V*>(lds + o) = hh;
            if (NPL == 3) {
                *reinterpret_cast<V*>(lds + PL + o) = mm;
                *reinterpret_cast<V*>(lds + 2 * PL + o) = ll;
            }
        }
    }
}

template <int BM, int BN, bool TA, bool TB, bool CONV, bool SEGB, int BKX, int NBUF, int NPL>
__global__ __launch_bounds__(256, (BM * BN > 128 * 128) ? 2 : 3) void gemm_x6_kernel(GemmParams p) {
    constexpr int WTM = BM / 2, WTN = BN / 2;
    constexpr int RM = WTM / 32, RN = WTN / 32;
    constexpr bool AKC = !TA, BKC = TB;
    constexpr int PA = X6<BM, BKX>::PLANE, PB = X6<BN, BKX>::PLANE;
    constexpr int STAGE = NPL * (PA + PB);  // NPL = 3 planes (x6) or 1 (bf16: the one product h*h)
    static_assert(RM >= 1 && RN >= 1, "wave tile >= 32x32");
    __shared__ __attribute__((aligned(16))) __bf16 smem[NBUF * STAGE];

    const TileId tid = xcd_tile();
    int zz = tid.z;
    int split = 0;
    if (p.splits > 1) {
        split = zz % p.splits;
        zz /= p.splits;
    }
    const int z1 = zz / p.zdiv, z0 = zz % p.zdiv;
    const int Mv = p.zmvalid ? p.zmvalid[z1] : p.Mvalid;  // conv-A valid source rows
    const float* A = p.A + z1 * p.sA1 + z0 * p.sA0;
    const float* B = p.B + z1 * p.sB1 + z0 * p.sB0;
    const int m0 = tid.y * BM;
    const int n0 = tid.x * BN;
    const int kbeg = split * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int h = lane >> 5, l32 = lane & 31;

    f32x16 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    f32x4 ra[X6<BM, BKX>::LOADS];
    f32x4 rb[X6<BN, BKX>::LOADS];
    const bool va = p.va != 0, vb = p.vb != 0;
    const bool segAligned = p.segK > 0 && p.segK % BKX == 0;
    auto stageA = [&](int k) {
        bool full = va && m0 + BM <= p.M && k + BKX <= kend;
        const float* base = A;
        int kk = k;
        if (CONV) {
            const int seg = segAligned ? k / p.segK : 0;
            const int sh = seg - p.pad;
            full = full && segAligned && m0 + sh >= 0 && m0 + BM + sh <= Mv;
            base = A + (long)sh * p.lda;
            kk = k - seg * p.segK;
        }
        if (AKC) {
            if (full) x6_load_kc<BM, BKX, 0, true>(ra, base, p.lda, m0, p.M, kk, kend, va, 0, 0, 0, 0);
            else x6_load_kc<BM, BKX, CONV ? 1 : 0, false>(ra, A, p.lda, m0, p.M, k, kend, va, p.segK, p.pad, Mv, 0);
        } else {
            if (full) x6_load_mn<BM, BKX, true>(ra, A, p.lda, m0, p.M, k, kend, va);
            else x6_load_mn<BM, BKX, false>(ra, A, p.lda, m0, p.M, k, kend, va);
        }
    };
    auto stageB = [&](int k) {
        bool full = vb && n0 + BN <= p.N && k + BKX <= kend;
        const float* base = B;
        int kk = k;
        if (SEGB) {
            const int seg = segAligned ? k / p.segK : 0;
            full = full && segAligned;
            base = B + seg * p.sBseg;
            kk = k - seg * p.segK;
        }
        if (BKC) {
            if (full) x6_load_kc<BN, BKX, 0, true>(rb, base, p.ldb, n0, p.N, kk, kend, vb, 0, 0, 0, 0);
            else x6_load_kc<BN, BKX, SEGB ? 2 : 0, false>(rb, B, p.ldb, n0, p.N, k, kend, vb, p.segK, 0, 0, p.sBseg);
        } else {
            if (full) x6_load_mn<BN, BKX, true>(rb, B, p.ldb, n0, p.N, k, kend, vb);
            else x6_load_mn<BN, BKX, false>(rb, B, p.ldb, n0, p.N, k, kend, vb);
        }
    };
    auto mfma_stage = [&](const __bf16* As, const __bf16* Bs) {
#pragma unroll
        for (int kc = 0; kc < BKX / 16; ++kc) {
            bf16x8 af[RM][NPL], bf[RN][NPL];
            const int k = kc * 16 + h * 8;
#pragma unroll
            for (int i = 0; i < RM; ++i) {
                const int o = x6_idx<BKX>(wm * WTM + i * 32 + l32, k);
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl) af[i][pl] = *reinterpret_cast<const bf16x8*>(As + pl * PA + o);
            }
#pragma unroll
            for (int j = 0; j < RN; ++j) {
                const int o = x6_idx<BKX>(wn * WTN + j * 32 + l32, k);
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl) bf[j][pl] = *reinterpret_cast<const bf16x8*>(Bs + pl * PB + o);
            }
            // small terms first, the h*h product last
#pragma unroll
            for (int t = (X6_ABLATE == 2 || NPL == 1 ? 5 : 0); t < 6; ++t) {
                constexpr int pa[6] = {0, 1, 2, 0, 1, 0};
                constexpr int pb[6] = {2, 1, 0, 1, 0, 0};
                const int ia = NPL == 1 ? 0 : pa[t], ib = NPL == 1 ? 0 : pb[t];
#pragma unroll
                for (int i = 0; i < RM; ++i)
#pragma unroll
                    for (int j = 0; j < RN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][ia], bf[j][ib], acc[i][j], 0, 0, 0);
            }
        }
    };

    stageA(kbeg);
    stageB(kbeg);
    if (NBUF == 1) {
        for (int k0 = kbeg; k0 < kend; k0 += BKX) {
            __syncthreads();
            x6_store<BM, BKX, AKC, NPL>(smem, ra);
            x6_store<BN, BKX, BKC, NPL>(smem + NPL * PA, rb);
            __syncthreads();
            if (k0 + BKX < kend) {
                stageA(k0 + BKX);
                stageB(k0 + BKX);
            }
            mfma_stage(smem, smem + NPL * PA);
        }
    } else {
        // two LDS stages: while the MFMAs read stage s, the registers holding stage s+1 are split
        // into the other buffer (last read before the previous barrier) and stage s+2 is loaded
        x6_store<BM, BKX, AKC, NPL>(smem, ra);
        x6_store<BN, BKX, BKC, NPL>(smem + NPL * PA, rb);
        if (kbeg + BKX < kend) {
            stageA(kbeg + BKX);
            stageB(kbeg + BKX);
        }
        __syncthreads();
        int buf = 0;
        for (int k0 = kbeg; k0 < kend; k0 += BKX) {
            const __bf16* As = smem + buf * STAGE;
            mfma_stage(As, As + NPL * PA);
            if (k0 + BKX < kend) {
                __bf16* nxt = smem + (buf ^ 1) * STAGE;
                x6_store<BM, BKX, AKC, NPL>(nxt, ra);
                x6_store<BN, BKX, BKC, NPL>(nxt + NPL * PA, rb);
                if (k0 + 2 * BKX < kend) {
                    stageA(k0 + 2 * BKX);
                    stageB(k0 + 2 * BKX);
                }
                __syncthreads();
                buf ^= 1;
            }
        }
    }


    gemm_epilogue<RM, RN>(p, acc, z1, z0, m0 + wm * WTM, n0 + wn * WTN, h, l32, m0 + BM <= p.M && n0 + BN <= p.N, tid.z);
}

template <int BM, int BN, int BKX, int NB, int NPL = 3>
void launch_x6(const GemmParams& p, dim3 grid, hipStream_t st) {
#define X6K(TA_, TB_, CV_, SB_) gemm_x6_kernel<BM, BN, TA_, TB_, CV_, SB_, BKX, NB, NPL>
    if (p.segK > 0) {
        if (p.segB) hipLaunchKernelGGL((X6K(false, true, true, true)), grid, dim3(256), 0, st, p);
        else hipLaunchKernelGGL((X6K(false, false, true, false)), grid, dim3(256), 0, st, p);
        return;
    }
    if (!p.ta && !p.tb) hipLaunchKernelGGL((X6K(false, false, false, false)), grid, dim3(256), 0, st, p);
    else if (!p.ta && p.tb) hipLaunchKernelGGL((X6K(false, true, false, false)), grid, dim3(256), 0, st, p);
    else if (p.ta && !p.tb) hipLaunchKernelGGL((X6K(true, false, false, false)), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((X6K(true, true, false, false)), grid, dim3(256), 0, st, p);
#undef X6K
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
    const float* rowv = p.rowv ? p.rowv + z1 * p.sRow1 + z0 * p.sRow0 : nullptr;
    const float* W = p.ws + (long)zz * p.splits * MN;
    for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < MN; idx += (long)gridDim.x * blockDim.x) {
        float s = 0.f;
        for (int sp = 0; sp < p.splits; ++sp) s += W[sp * MN + idx];
        const long row = idx / p.N, col = idx % p.N;
        const float v = epi_value(p, s, row, col, bias, R, aux, C2, C, rowv);
        const float o = ((p.epi & EPI_ROWMASK) && row >= p.zrows[z1]) ? 0.f : v;
        if (p.C) C[row * p.ldc + col] = o;  // null: a bf16-plane GEMM whose fp32 output is dead
        if (p.Cb) reinterpret_cast<__bf16*>(p.Cb)[row * p.ldcb + col] = (__bf16)o;
    }
}

// ============================================================================================
// fp32 GEMM with LDS-DMA staging ("glds"): global_load_lds_dwordx4 moves each K-step of both
// operands straight into LDS (no VGPR staging, no ds_write), two LDS stages, ONE barrier per K-step:
//   wait(stage s landed) + barrier -> issue DMA of stage s+1 into the other buffer -> MFMAs on stage s
// so the next stage's loads are in flight for the whole compute phase.  LDS-DMA writes are
// lane-linear (1 KiB per wave-instruction), so:
//   k-contiguous operand: LDS [row][32] (128-B rows) with the 16-B chunk c of row r stored in slot
//       c ^ ((r >> 1) & 7) -- the swizzle is applied to the per-lane SOURCE address; fragment reads
//       (16 lanes = 16 consecutive rows, same chunk) hit 16 distinct 4-bank groups: conflict-free
//   row-contiguous operand: LDS [k][ROWS] linear; 4-B fragment reads by consecutive rows.
// Lanes outside the operand (M/N edge rows, K tail, conv padding rows) read a zero page, so no
// predicates reach LDS.  Preconditions (checked by the dispatcher): 16-B aligned operands, leading
// dimensions and batch strides multiples of 4, K % 4 == 0 for k-contiguous operands.
// ============================================================================================
__device__ __attribute__((aligned(16))) float g_zero16[4];

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// k-contiguous stage image: rows of BKS floats, CPR = BKS/4 16-B chunks per row, RPB = rows per
// 256-B bank row; chunk c of row r lives in slot c ^ ((r / RPB) % CPR).
template <int BKS>
__device__ __forceinline__ int glds_swz(int row) {
    constexpr int CPR = BKS / 4, RPB = 64 / BKS;
    return (row / RPB) % CPR;
}

// Issue the LDS-DMA of one BKS-deep stage of an operand tile (ROWS rows) into `dst` (wave-uniform).
//   KC = true : element (row, k) at src[row*ld + k]     (MODE 1: conv-A row shift, MODE 2: segmented)
//   KC = false: element (row, k) at src[k*ld + row]
// dummy: load the zero page (keeps the per-wave DMA count uniform past the last K-step).
template <int ROWS, int BKS, bool KC, int MODE, int NWV = 4>
__device__ __forceinline__ void glds_stage(float* dst, const float* __restrict__ src, long ld, int row0, int nrows,
                                           int k0, int kend, int segK, int pad, int Mvalid, long sseg, int w,
                                           int lane, bool dummy) {
    constexpr int NI = ROWS * BKS / (256 * NWV);  // wave-instructions per wave (1 KiB each, NWV waves)
    static_assert(NI >= 1, "stage too small for the block's waves");
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const int ci = i * NWV + w;  // 1-KiB piece of the stage image
        const float* g = g_zero16;
        if (!dummy) {
            if (KC) {
                constexpr int CPR = BKS / 4;
                const int row = ci * (256 / BKS) + lane / CPR;
                const int c = (lane % CPR) ^ glds_swz<BKS>(row);
                const int gr = row0 + row, gk = k0 + c * 4;
                if (gr < nrows && gk < kend) {
                    if (MODE == 1) {
                        const int seg = gk / segK;
                        const int srow = gr + seg - pad;
                        if (srow >= 0 && srow < Mvalid) g = src + (long)srow * ld + (gk - seg * segK);
                    } else if (MODE == 2) {
                        const int seg = gk / segK;
                        g = src + (long)gr * ld + seg * sseg + (gk - seg * segK);
                    } else {
                        g = src + (long)gr * ld + gk;
                    }
                }
            } else {
                const int f = ci * 256 + lane * 4;
                const int k = f / ROWS, m = f % ROWS;
                const int gk = k0 + k, gm = row0 + m;
                if (gk < kend && gm < nrows) g = src + (long)gk * ld + gm;
            }
        }
        __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)(dst + ci * 256), 16, 0, 0);
    }
}

// Plain-operand (MODE 0) DMA sources, set up once per block and advanced by one K-step per stage: the
// K-loop issues NI global_load_lds per operand with no address arithmetic beyond one add.  Lanes
// outside the operand point at the zero page and never move.  Valid for full stages (k + BKS <= kend);
// a partial last stage goes through glds_stage.
template <int ROWS, int BKS, bool KC, int NWV = 4>
struct GldsStream {
    static constexpr int NI = ROWS * BKS / (256 * NWV);
    const float* ptr[NI];
    int inc[NI];  // floats per K-step (0 on zero-page lanes)
    __device__ __forceinline__ void init(const float* __restrict__ src, long ld, int row0, int nrows, int k0, int w,
                                         int lane) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int ci = i * NWV + w;
            bool ok;
            const float* g;
            if (KC) {
                constexpr int CPR = BKS / 4;
                const int row = ci * (256 / BKS) + lane / CPR;
                const int c = (lane % CPR) ^ glds_swz<BKS>(row);
                ok = row0 + row < nrows;
                g = src + (long)(row0 + row) * ld + k0 + c * 4;
            } else {
                const int f = ci * 256 + lane * 4;
                const int k = f / ROWS, m = f % ROWS;
                ok = row0 + m < nrows;
                g = src + (long)(k0 + k) * ld + row0 + m;
            }
            ptr[i] = ok ? g : g_zero16;
            inc[i] = ok ? (KC ? BKS : (int)(BKS * ld)) : 0;
        }
    }
};

// one full stage of a GldsStream operand (free function: a member-function form of this builtin call
// made hipcc's host pass drop the kernels' launch stubs)
template <int ROWS, int BKS, bool KC, int NWV>
__device__ __forceinline__ void glds_stream_issue(GldsStream<ROWS, BKS, KC, NWV>& sm, float* dst, int w) {
#pragma unroll
    for (int i = 0; i < GldsStream<ROWS, BKS, KC, NWV>::NI; ++i) {
        const float* g = sm.ptr[i];
        __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)(dst + (i * NWV + w) * 256), 16, 0, 0);
        sm.ptr[i] = g + sm.inc[i];
    }
}

// fragment of 4 consecutive MFMA k-steps: tile k = h * BKS/2 + 4q + e  (q < BKS/8)
template <int ROWS, int BKS, bool KC>
__device__ __forceinline__ f32x4 glds_frag(const float* __restrict__ lds, int row, int h, int q) {
    if (KC) {
        const int c = h * (BKS / 8) + q;
        return *reinterpret_cast<const f32x4*>(lds + row * BKS + ((c ^ glds_swz<BKS>(row)) * 4));
    }
    f32x4 v;
    const int k = h * (BKS / 2) + q * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = lds[(k + e) * ROWS + row];
    return v;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    // s_waitcnt: vmcnt[3:0] | expcnt[6:4] (7 = no wait) | lgkmcnt[11:8] (15 = no wait) | vmcnt[5:4] << 14
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// BKS-deep K-steps through NS LDS stages: NS-1 stages of DMA in flight while a stage is consumed;
// one barrier per K-step, preceded by a counted vmcnt that retires exactly the stage about to be
// read (never vmcnt(0) inside the loop).
template <int BM, int BN, bool TA, bool TB, bool CONV, bool SEGB, int BKS, int NS>
__global__ __launch_bounds__(256, 2) void gemm_glds_kernel(GemmParams p) {
    // waves 2 x 2 (wave tile BM/2 x BN/2), or 1 x 4 when BM is not a multiple of 64 (the 160-row tile:
    // wave tile 160 x BN/4, five A fragments against one B fragment)
    constexpr int WGM = (BM % 64 == 0) ? 2 : 1, WGN = 4 / WGM;
    constexpr int WTM = BM / WGM, WTN = BN / WGN;
    constexpr int RM = WTM / 32, RN = WTN / 32;
    static_assert(RM * 32 == WTM && RN * 32 == WTN, "wave tile must be whole 32x32 fragments");
    constexpr bool AKC = !TA, BKC = TB;
    constexpr int STAGE = (BM + BN) * BKS;  // floats per LDS stage
    constexpr int NPW = (BM + BN) * BKS / 1024;  // DMA instructions per wave per stage
    __shared__ __attribute__((aligned(16))) float smem[NS * STAGE];

    const TileId tid = xcd_tile(p.order);
    int zz = tid.z;
    int split = 0;
    if (p.splits > 1) {
        split = zz % p.splits;
        zz /= p.splits;
    }
    const int z1 = zz / p.zdiv, z0 = zz % p.zdiv;
    const int Mv = p.zmvalid ? p.zmvalid[z1] : p.Mvalid;  // conv-A valid source rows
    const float* A = p.A + z1 * p.sA1 + z0 * p.sA0;
    const float* B = p.B + z1 * p.sB1 + z0 * p.sB0;
    const int m0 = tid.y * BM;
    const int n0 = tid.x * BN;
    const int kbeg = split * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);
    const int nst = (kend - kbeg + BKS - 1) / BKS;

    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid / WGN, wn = wid % WGN;
    const int h = lane >> 5, l32 = lane & 31;

    f32x16 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // plain operands stream from precomputed per-lane pointers (GldsStream); conv / segmented operands
    // and the partial last stage recompute addresses (glds_stage)
    constexpr bool STREAM = !CONV && !SEGB;
    GldsStream<BM, BKS, AKC> sa;
    GldsStream<BN, BKS, BKC> sb;
    if (STREAM) {
        sa.init(A, p.lda, m0, p.M, kbeg, wid, lane);
        sb.init(B, p.ldb, n0, p.N, kbeg, wid, lane);
    }
    auto issue = [&](int s) {
        float* st = smem + (s % NS) * STAGE;
        const int k = kbeg + s * BKS;
        const bool dummy = s >= nst;
        if (NS == 2 && dummy) {
            // vmcnt(0) waits: nothing to keep in step past the last stage
        } else if (STREAM && k + BKS <= kend) {
            glds_stream_issue(sa, st, wid);
            glds_stream_issue(sb, st + BM * BKS, wid);
        } else {
            glds_stage<BM, BKS, AKC, CONV ? 1 : 0>(st, A, p.lda, m0, p.M, k, kend, p.segK, p.pad, Mv, 0, wid,
                                                    lane, dummy);
            glds_stage<BN, BKS, BKC, SEGB ? 2 : 0>(st + BM * BKS, B, p.ldb, n0, p.N, k, kend, p.segK, 0, 0,
                                                    p.sBseg, wid, lane, dummy);
        }
    };
    auto compute = [&](int s) {
        const float* As = smem + (s % NS) * STAGE;
        const float* Bs = As + BM * BKS;
#pragma unroll
        for (int q = 0; q < BKS / 8; ++q) {
            f32x4 af[RM], bf[RN];
#pragma unroll
            for (int i = 0; i < RM; ++i) af[i] = glds_frag<BM, BKS, AKC>(As, wm * WTM + i * 32 + l32, h, q);
#pragma unroll
            for (int j = 0; j < RN; ++j) bf[j] = glds_frag<BN, BKS, BKC>(Bs, wn * WTN + j * 32 + l32, h, q);
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < RM; ++i)
#pragma unroll
                    for (int j = 0; j < RN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][e], bf[j][e], acc[i][j], 0, 0, 0);
        }
    };

#pragma unroll
    for (int s = 0; s < NS - 1; ++s) issue(s);
    for (int s = 0; s < nst; ++s) {
        wait_vm<(NS - 2) * NPW>();  // stage s landed (this wave's share); later stages may be in flight
        __builtin_amdgcn_s_barrier();  // every wave's share landed; stage s-1's buffer is free
        issue(s + NS - 1);
        compute(s);
    }
    wait_vm<0>();  // no LDS-DMA may outlive the block
    gemm_epilogue<RM, RN>(p, acc, z1, z0, m0 + wm * WTM, n0 + wn * WTN, h, l32, m0 + BM <= p.M && n0 + BN <= p.N,
                          tid.z);
}

// ============================================================================================
// bf16 matrix cores fed from the same LDS-DMA fp32 stages ("gbf"): operands stay fp32 in HBM and
// LDS; each wave converts its own fragments to bf16 in registers right before the MFMAs
// (v_cvt_pk_bf16_f32, round-to-nearest-even), so the staging is the glds kernel's unchanged.
//   NPROD = 1: bf16 GEMM (x -> bf16(x)), fp32 accumulate -- SUTA_PRECISION_BF16 (config C4)
//   NPROD = 6: fp32-accurate split (x = h + m + l, the six products of order <= 2, small terms
//              first) -- the register-split alternative to gemm_x6_kernel's LDS planes
// v_mfma_f32_32x32x16_bf16 lane l takes row l % 32 and k = 16 kc + 8 (l / 32) + [0, 8): a
// k-contiguous fragment is two adjacent 16-B chunks of the swizzled [row][BKS] image.
// ============================================================================================
typedef float f32x8 __attribute__((ext_vector_type(8)));

template <int ROWS, int BKS, bool KC>
__device__ __forceinline__ f32x8 gbf_frag(const float* __restrict__ lds, int row, int kc, int h) {
    f32x8 v;
    if (KC) {
        const int c = kc * 4 + h * 2;
        const int sw = glds_swz<BKS>(row);
        const f32x4 lo = *reinterpret_cast<const f32x4*>(lds + row * BKS + ((c ^ sw) * 4));
        const f32x4 hi = *reinterpret_cast<const f32x4*>(lds + row * BKS + (((c + 1) ^ sw) * 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            v[e] = lo[e];
            v[4 + e] = hi[e];
        }
        return v;
    }
    const int k = kc * 16 + h * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = lds[(k + e) * ROWS + row];
    return v;
}

template <int NPL>
__device__ __forceinline__ void gbf_split(const f32x8& x, bf16x8 (&o)[NPL]) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const __bf16 hh = (__bf16)x[e];
        o[0][e] = hh;
        if (NPL == 3) {
            const float r = x[e] - (float)hh;
            const __bf16 mm = (__bf16)r;
            o[1][e] = mm;
            o[2][e] = (__bf16)(r - (float)mm);
        }
    }
}

template <int BM, int BN, bool TA, bool TB, bool CONV, bool SEGB, int BKS, int NS, int NPROD>
__global__ __launch_bounds__(256, 2) void gemm_gbf_kernel(GemmParams p) {
    constexpr int WTM = BM / 2, WTN = BN / 2;
    constexpr int RM = WTM / 32, RN = WTN / 32;
    constexpr bool AKC = !TA, BKC = TB;
    constexpr int STAGE = (BM + BN) * BKS;
    constexpr int NPW = (BM + BN) * BKS / 1024;
    constexpr int NPL = NPROD == 1 ? 1 : 3;
    static_assert(BKS % 16 == 0, "bf16 MFMA k-step is 16");
    __shared__ __attribute__((aligned(16))) float smem[NS * STAGE];

    const TileId tid = xcd_tile();
    int zz = tid.z;
    int split = 0;
    if (p.splits > 1) {
        split = zz % p.splits;
        zz /= p.splits;
    }
    const int z1 = zz / p.zdiv, z0 = zz % p.zdiv;
    const int Mv = p.zmvalid ? p.zmvalid[z1] : p.Mvalid;
    const float* A = p.A + z1 * p.sA1 + z0 * p.sA0;
    const float* B = p.B + z1 * p.sB1 + z0 * p.sB0;
    const int m0 = tid.y * BM;
    const int n0 = tid.x * BN;
    const int kbeg = split * p.kchunk;
    const int kend = min(p.K, kbeg + p.kchunk);
    const int nst = (kend - kbeg + BKS - 1) / BKS;

    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid >> 1, wn = wid & 1;
    const int h = lane >> 5, l32 = lane & 31;

    f32x16 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    constexpr bool STREAM = !CONV && !SEGB;  // plain operands: per-block DMA source setup (GldsStream)
    GldsStream<BM, BKS, AKC> sa;
    GldsStream<BN, BKS, BKC> sb;
    if (STREAM) {
        sa.init(A, p.lda, m0, p.M, kbeg, wid, lane);
        sb.init(B, p.ldb, n0, p.N, kbeg, wid, lane);
    }
    auto issue = [&](int s) {
        float* st = smem + (s % NS) * STAGE;
        const int k = kbeg + s * BKS;
        const bool dummy = s >= nst;
        if (NS == 2 && dummy) {
            // vmcnt(0) waits: nothing to keep in step past the last stage
        } else if (STREAM && k + BKS <= kend) {
            glds_stream_issue(sa, st, wid);
            glds_stream_issue(sb, st + BM * BKS, wid);
        } else {
            glds_stage<BM, BKS, AKC, CONV ? 1 : 0>(st, A, p.lda, m0, p.M, k, kend, p.segK, p.pad, Mv, 0, wid,
                                                    lane, dummy);
            glds_stage<BN, BKS, BKC, SEGB ? 2 : 0>(st + BM * BKS, B, p.ldb, n0, p.N, k, kend, p.segK, 0, 0,
                                                    p.sBseg, wid, lane, dummy);
        }
    };
    auto compute = [&](int s) {
        const float* As = smem + (s % NS) * STAGE;
        const float* Bs = As + BM * BKS;
#pragma unroll
        for (int kc = 0; kc < BKS / 16; ++kc) {
            bf16x8 af[RM][NPL], bf[RN][NPL];
#pragma unroll
            for (int i = 0; i < RM; ++i) gbf_split<NPL>(gbf_frag<BM, BKS, AKC>(As, wm * WTM + i * 32 + l32, kc, h), af[i]);
#pragma unroll
            for (int j = 0; j < RN; ++j) gbf_split<NPL>(gbf_frag<BN, BKS, BKC>(Bs, wn * WTN + j * 32 + l32, kc, h), bf[j]);
#pragma unroll
            for (int t = 0; t < NPROD; ++t) {
                constexpr int pa6[6] = {0, 1, 2, 0, 1, 0};
                constexpr int pb6[6] = {2, 1, 0, 1, 0, 0};
                const int ia = NPROD == 1 ? 0 : pa6[t], ib = NPROD == 1 ? 0 : pb6[t];
#pragma unroll
                for (int i = 0; i < RM; ++i)
#pragma unroll
                    for (int j = 0; j < RN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i][ia], bf[j][ib], acc[i][j], 0, 0, 0);
            }
        }
    };

#pragma unroll
    for (int s = 0; s < NS - 1; ++s) issue(s);
    for (int s = 0; s < nst; ++s) {
        wait_vm<(NS - 2) * NPW>();
        __builtin_amdgcn_s_barrier();
        issue(s + NS - 1);
        compute(s);
    }
    wait_vm<0>();
    gemm_epilogue<RM, RN>(p, acc, z1, z0, m0 + wm * WTM, n0 + wn * WTN, h, l32, m0 + BM <= p.M && n0 + BN <= p.N,
                          tid.z);
}

template <int BM, int BN, int BKS, int NS, int NPROD>
void launch_gbf(const GemmParams& p, dim3 grid, hipStream_t st) {
#define GB(TA_, TB_, CV_, SB_) gemm_gbf_kernel<BM, BN, TA_, TB_, CV_, SB_, BKS, NS, NPROD>
    if (p.segK > 0) {
        if (p.segB) hipLaunchKernelGGL((GB(false, true, true, true)), grid, dim3(256), 0, st, p);
        else hipLaunchKernelGGL((GB(false, false, true, false)), grid, dim3(256), 0, st, p);
        return;
    }
    if (!p.ta && !p.tb) hipLaunchKernelGGL((GB(false, false, false, false)), grid, dim3(256), 0, st, p);
    else if (!p.ta && p.tb) hipLaunchKernelGGL((GB(false, true, false, false)), grid, dim3(256), 0, st, p);
    else if (p.ta && !p.tb) hipLaunchKernelGGL((GB(true, false, false, false)), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((GB(true, true, false, false)), grid, dim3(256), 0, st, p);
#undef GB
}

template <int BKS, int NS, int NPROD>
void launch_gbf_tile(int tile, const GemmParams& p, dim3 grid, hipStream_t st) {
    if (tile == 0) launch_gbf<128, 128, BKS, NS, NPROD>(p, grid, st);
    else if (tile == 1) launch_gbf<128, 64, BKS, NS, NPROD>(p, grid, st);
    else if (tile == 2) launch_gbf<64, 128, BKS, NS, NPROD>(p, grid, st);
    else launch_gbf<64, 64, BKS, NS, NPROD>(p, grid, st);
}

template <int BM, int BN, int BKS, int NS>
void launch_glds(const GemmParams& p, dim3 grid, hipStream_t st) {
#define GK(TA_, TB_, CV_, SB_) gemm_glds_kernel<BM, BN, TA_, TB_, CV_, SB_, BKS, NS>
    if (p.segK > 0) {
        if (p.segB) hipLaunchKernelGGL((GK(false, true, true, true)), grid, dim3(256), 0, st, p);
        else hipLaunchKernelGGL((GK(false, false, true, false)), grid, dim3(256), 0, st, p);
        return;
    }
    if (!p.ta && !p.tb) hipLaunchKernelGGL((GK(false, false, false, false)), grid, dim3(256), 0, st, p);
    else if (!p.ta && p.tb) hipLaunchKernelGGL((GK(false, true, false, false)), grid, dim3(256), 0, st, p);
    else if (p.ta && !p.tb) hipLaunchKernelGGL((GK(true, false, false, false)), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((GK(true, true, false, false)), grid, dim3(256), 0, st, p);
#undef GK
}

template <int BKS, int NS>
void launch_glds_tile(int tile, const GemmParams& p, dim3 grid, hipStream_t st) {
    if (tile == 0) launch_glds<128, 128, BKS, NS>(p, grid, st);
    else if (tile == 1) launch_glds<128, 64, BKS, NS>(p, grid, st);
    else if (tile == 2) launch_glds<64, 128, BKS, NS>(p, grid, st);
    else launch_glds<64, 64, BKS, NS>(p, grid, st);
}

template <int BM, int BN, int NBUF>
void launch_tile(const GemmParams& p, dim3 grid, hipStream_t st) {
    if (p.segK > 0) {
        if (p.segB)
            hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, false, true, true, true, NBUF>), grid, dim3(256), 0, st, p);
        else
            hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, false, false, true, false, NBUF>), grid, dim3(256), 0, st, p);
        return;
    }
    if (!p.ta && !p.tb)
        hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, false, false, false, false, NBUF>), grid, dim3(256), 0, st, p);
    else if (!p.ta && p.tb)
        hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, false, true, false, false, NBUF>), grid, dim3(256), 0, st, p);
    else if (p.ta && !p.tb)
        hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, true, false, false, false, NBUF>), grid, dim3(256), 0, st, p);
    else
        hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, true, true, false, false, NBUF>), grid, dim3(256), 0, st, p);
}


// ============================================================================================
// bf16 GEMM on bf16 operand planes ("hb", SUTA_PRECISION_BF16 with planes): both operands bf16 and
// k-contiguous in HBM (A [M][K] activations converted once, B [N][K] frozen weights or their
// transposes converted at engine setup), staged by the glds LDS-DMA machinery in 4-byte units (a
// 64-deep bf16 K-step is a 32-float-wide stage image: 128-B rows, 16-B chunks XOR-swizzled by
// (row / 2) % 8, conflict-free fragment reads), fp32 accumulation on v_mfma_f32_32x32x16_bf16 (lane l:
// row l % 32, k = 16 kc + 8 (l / 32) + [0, 8) = one 16-B chunk), the fp32 epilogue of every kernel.
// Half the operand bytes of the fp32-staged bf16 kernels, no conversion in the K-loop.
// ============================================================================================
// NWV = 4 waves (2 x 2) or 8 waves (2 x 4, the 256 x 256 tile: 128 x 64 per wave, 128 KB of LDS)
// CONV / SEGB: the conv input-gradient form (conv-A rows of A, per-tap B segments; glds_stage modes 1 / 2 in
// 4-byte units: segK, pad, sBseg given in bf16 elements, even)
// CBT: -1 = the bf16 C plane chosen at run time (p.Cb), 0 / 1 = fixed; EM: epilogue flag class (gemm_epilogue)
template <int BM, int BN, int NS, int BKS = 32, int NWV = 4, bool CONV = false, bool SEGB = false, int CBT = -1,
          int EM = -1>  // BKS: 4-byte units
__global__ __launch_bounds__(64 * NWV, (BM * BN > 128 * 128 || BKS > 32) ? 1 : 2) void gemm_hb_kernel(GemmParams p) {
    constexpr int WNW = NWV / 2;                 // waves along N
    constexpr int WTM = BM / 2, WTN = BN / WNW;
    constexpr int RM = WTM / 32, RN = WTN / 32;
    constexpr int STAGE = (BM + BN) * BKS;       // 4-byte units per LDS stage
    constexpr int NPW = (BM + BN) * BKS / (256 * NWV);  // DMA instructions per wave per stage
    __shared__ __attribute__((aligned(16))) float smem[NS * STAGE];

    const TileId tid = xcd_tile(p.order);
    // grid z = batch x split (Z-batched planes: batch strides in bf16 elements, even)
    const int split = p.splits > 1 ? tid.z % p.splits : 0;
    const int zz = p.splits > 1 ? tid.z / p.splits : tid.z;
    const int z1 = zz / p.zdiv, z0 = zz % p.zdiv;
    const float* A = reinterpret_cast<const float*>(p.Ab) + (z1 * p.sA1 + z0 * p.sA0) / 2;
    const float* B = reinterpret_cast<const float*>(p.Bb) + (z1 * p.sB1 + z0 * p.sB0) / 2;
    const long lda = p.ldab / 2, ldb = p.ldbb / 2;  // in 4-byte units
    const int m0 = tid.y * BM;
    const int n0 = tid.x * BN;
    const int kbeg = split * p.kchunk / 2;
    const int kend = min(p.K, split * p.kchunk + p.kchunk) / 2;
    const int nst = (kend - kbeg + BKS - 1) / BKS;

    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid / WNW, wn = wid % WNW;
    const int h = lane >> 5, l32 = lane & 31;

    f32x16 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    GldsStream<BM, BKS, true, NWV> sa;
    GldsStream<BN, BKS, true, NWV> sb;
    sa.init(A, lda, m0, p.M, kbeg, wid, lane);
    sb.init(B, ldb, n0, p.N, kbeg, wid, lane);
    const int segK2 = p.segK / 2, pad = p.pad;
    const int Mv = p.zmvalid ? p.zmvalid[z1] : p.Mvalid;
    const long sseg2 = p.sBseg / 2;
    auto issue = [&](int s) {
        float* st = smem + (s % NS) * STAGE;
        const int k = kbeg + s * BKS;
        if (s >= nst) {
            if (NS > 2) {  // keep the per-wave DMA count uniform past the last stage
                glds_stage<BM, BKS, true, 0, NWV>(st, A, lda, m0, p.M, k, kend, 0, 0, 0, 0, wid, lane, true);
                glds_stage<BN, BKS, true, 0, NWV>(st + BM * BKS, B, ldb, n0, p.N, k, kend, 0, 0, 0, 0, wid, lane, true);
            }
        } else if (CONV || SEGB) {  // conv input gradient: per-lane addresses from the row / segment maps
            glds_stage<BM, BKS, true, CONV ? 1 : 0, NWV>(st, A, lda, m0, p.M, k, kend, segK2, pad, Mv, 0, wid, lane,
                                                          false);
            glds_stage<BN, BKS, true, SEGB ? 2 : 0, NWV>(st + BM * BKS, B, ldb, n0, p.N, k, kend, segK2, 0, 0, sseg2,
                                                          wid, lane, false);
        } else if (k + BKS <= kend) {
            glds_stream_issue(sa, st, wid);
            glds_stream_issue(sb, st + BM * BKS, wid);
        } else {
            glds_stage<BM, BKS, true, 0, NWV>(st, A, lda, m0, p.M, k, kend, 0, 0, 0, 0, wid, lane, false);
            glds_stage<BN, BKS, true, 0, NWV>(st + BM * BKS, B, ldb, n0, p.N, k, kend, 0, 0, 0, 0, wid, lane, false);
        }
    };
    auto frag = [&](const float* lds, int row, int kc) {
        const int c = 2 * kc + h;
        return *reinterpret_cast<const bf16x8*>(lds + row * BKS + ((c ^ glds_swz<BKS>(row)) * 4));
    };
    auto compute = [&](int s) {
        const float* As = smem + (s % NS) * STAGE;
        const float* Bs = As + BM * BKS;
#pragma unroll
        for (int kc = 0; kc < BKS / 8; ++kc) {
            bf16x8 af[RM], bf[RN];
#pragma unroll
            for (int i = 0; i < RM; ++i) af[i] = frag(As, wm * WTM + i * 32 + l32, kc);
#pragma unroll
            for (int j = 0; j < RN; ++j) bf[j] = frag(Bs, wn * WTN + j * 32 + l32, kc);
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int j = 0; j < RN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
            if (RM * RN > 4) __builtin_amdgcn_sched_barrier(0);  // big tiles: bound the fragment reads hoisted ahead
        }
    };

#pragma unroll
    for (int s = 0; s < NS - 1; ++s) issue(s);
    for (int s = 0; s < nst; ++s) {
        wait_vm<(NS - 2) * NPW>();  // stage s landed (this wave's share); later stages may be in flight
        __builtin_amdgcn_s_barrier();
        issue(s + NS - 1);
        compute(s);
    }
    wait_vm<0>();
    // only the bf16-plane GEMMs write a bf16 copy of C (the template keeps the other kernels' epilogue as it was)
    if (CBT == 1 || (CBT < 0 && p.Cb))
        gemm_epilogue<RM, RN, true, EM>(p, acc, z1, z0, m0 + wm * WTM, n0 + wn * WTN, h, l32,
                                        m0 + BM <= p.M && n0 + BN <= p.N, tid.z);
    else
        gemm_epilogue<RM, RN, false, EM>(p, acc, z1, z0, m0 + wm * WTM, n0 + wn * WTN, h, l32,
                                         m0 + BM <= p.M && n0 + BN <= p.N, tid.z);
}

template <int BM, int BN, int NS, int BKS = 32, int NWV = 4, bool CONV = false, bool SEGB = false, int CBT = -1,
          int EM = -1>
void launch_hb(const GemmParams& p, dim3 grid, hipStream_t st) {
    hipLaunchKernelGGL((gemm_hb_kernel<BM, BN, NS, BKS, NWV, CONV, SEGB, CBT, EM>), grid, dim3(64 * NWV), 0, st, p);
}

}  // namespace

// Per-family launch wrappers (each defined in its own TU).
void gemm_run_f32(int tile, int nbuf, const GemmParams& p, dim3 grid, hipStream_t st);      // gemm_f32.hip
void gemm_run_x6(int tile, int bk16, int npl, const GemmParams& p, dim3 grid, hipStream_t st);  // gemm_x6.hip
void gemm_run_glds(int variant, int tile, const GemmParams& p, dim3 grid, hipStream_t st);  // gemm_glds.hip
// ============================================================================================
// bf16 GEMM on MN-contiguous bf16 planes ("hbt"; the conv weight gradients of config C4):
//   A(m, k) = Ab[k * ldab + m], B(k, n) = Bb[k * ldbb + n]   (both row-major over k: im2col(a)^T and dz)
// Stages of 64 k-rows of both operands arrive by LDS-DMA as [k][BM] / [k][BN] bf16 images (one 256-B row per k at
// 128 columns); the MFMA operands (8 consecutive k of one column) come from two ds_read_b64_tr_b16 transposed reads
// per fragment.  Conflict-free: the 16-B chunk c of image row r sits in slot c ^ 4 (r & 3) (applied to the DMA
// SOURCE, as the glds swizzle), so the 4 rows x 64 B a 32-lane half reads land in 64 distinct banks.  Two stages,
// one barrier per stage; the general epilogues (fast 32-bit path on interior tiles).  M % 8 == N % 8 == 0.
// ============================================================================================
template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void gemm_hbt_kernel(GemmParams p) {
    constexpr int BKR = 64;                    // k rows per stage
    constexpr int ASZ = BKR * BM * 2, BSZ = BKR * BN * 2;  // bytes per stage
    constexpr int STAGE = ASZ + BSZ;
    constexpr int APC = ASZ / 1024 / 4, BPC = BSZ / 1024 / 4;  // 1-KiB DMA pieces per wave per stage
    constexpr int ACPR = BM / 8, BCPR = BN / 8;  // 16-B chunks per image row
    constexpr int WTM = BM / 2, WTN = BN / 2, RM = WTM / 32, RN = WTN / 32;
    static_assert(ACPR == 16 && BCPR == 16, "hbt: 128-column images (the swizzle assumes 16 chunks per row)");
    __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

    const TileId tid = xcd_tile(p.order);
    const int split = p.splits > 1 ? tid.z % p.splits : 0;
    const int zz = p.splits > 1 ? tid.z / p.splits : tid.z;
    const int z1 = zz / p.zdiv, z0 = zz % p.zdiv;
    const __bf16* A = reinterpret_cast<const __bf16*>(p.Ab) + z1 * p.sA1 + z0 * p.sA0;
    const __bf16* B = reinterpret_cast<const __bf16*>(p.Bb) + z1 * p.sB1 + z0 * p.sB0;
    const int m0 = tid.y * BM, n0 = tid.x * BN;
    const int kbeg = split * p.kchunk, kend = min(p.K, kbeg + p.kchunk);
    const int nst = (kend - kbeg + BKR - 1) / BKR;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid >> 1, wn = wid & 1;
    const int h = lane >> 5, l32 = lane & 31;

    f32x16 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // DMA sources: piece c (wave-uniform) covers image rows 4c .. 4c + 3; lane j: row 4c + j / 16, slot j % 16
    // holding global chunk (j % 16) ^ 4 (row & 3)
    const __bf16* asrc[APC];
    const __bf16* bsrc[BPC];
    int arow[APC], brow[BPC];
    bool aok[APC], bok[BPC];
#pragma unroll
    for (int i = 0; i < APC; ++i) {
        const int c = i * 4 + wid, r = 4 * c + lane / 16, gc = (lane % 16) ^ (4 * (r & 3));
        arow[i] = r;
        aok[i] = m0 + 8 * gc < p.M;
        asrc[i] = A + (long)(kbeg + r) * p.ldab + m0 + 8 * gc;
    }
#pragma unroll
    for (int i = 0; i < BPC; ++i) {
        const int c = i * 4 + wid, r = 4 * c + lane / 16, gc = (lane % 16) ^ (4 * (r & 3));
        brow[i] = r;
        bok[i] = n0 + 8 * gc < p.N;
        bsrc[i] = B + (long)(kbeg + r) * p.ldbb + n0 + 8 * gc;
    }
    auto issue = [&](int s) {
        if (s >= nst) return;
        char* st = smem + (s & 1) * STAGE;
        const int kb = kbeg + s * BKR;
#pragma unroll
        for (int i = 0; i < APC; ++i) {
            const void* g = (aok[i] && kb + arow[i] < kend) ? (const void*)(asrc[i] + (long)s * BKR * p.ldab)
                                                            : (const void*)g_zero16;
            __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)(st + (i * 4 + wid) * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < BPC; ++i) {
            const void* g = (bok[i] && kb + brow[i] < kend) ? (const void*)(bsrc[i] + (long)s * BKR * p.ldbb)
                                                            : (const void*)g_zero16;
            __builtin_amdgcn_global_load_lds(g, (lds_ptr_t)(st + ASZ + (i * 4 + wid) * 1024), 16, 0, 0);
        }
    };
    // fragment of 8 consecutive k (16 ks + 8 h + 0..7) of column col0 + lane-column: two transposed reads
    const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    auto frag = [&](const char* img, int col0, int ks) {
        const int c = col0 + 16 * (g & 1) + 4 * pp;   // the column block this lane addresses (4 columns)
        const int gc = c >> 3, half = (c & 7) * 2;
        const int r0 = 16 * ks + 8 * (g >> 1) + q;    // rows r0 and r0 + 4: row & 3 == q for both
        const int off = (gc ^ (4 * q)) * 16 + half;
        typedef __attribute__((address_space(3))) fbf16x4_t* lp4;
        const fbf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp4)(img + r0 * 256 + off));
        const fbf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lp4)(img + (r0 + 4) * 256 + off));
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            v[e] = lo[e];
            v[4 + e] = hi[e];
        }
        return v;
    };
    auto compute = [&](int s) {
        const char* As = smem + (s & 1) * STAGE;
        const char* Bs = As + ASZ;
#pragma unroll
        for (int ks = 0; ks < BKR / 16; ++ks) {
            bf16x8 af[RM], bfr[RN];
#pragma unroll
            for (int i = 0; i < RM; ++i) af[i] = frag(As, wm * WTM + i * 32, ks);
#pragma unroll
            for (int j = 0; j < RN; ++j) bfr[j] = frag(Bs, wn * WTN + j * 32, ks);
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int j = 0; j < RN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    };
    issue(0);
    for (int s = 0; s < nst; ++s) {
        wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        issue(s + 1);
        compute(s);
    }
    wait_vm<0>();
    gemm_epilogue<RM, RN, false>(p, acc, z1, z0, m0 + wm * WTM, n0 + wn * WTN, h, l32,
                                 m0 + BM <= p.M && n0 + BN <= p.N, tid.z);
}

void gemm_run_gbf(int bk64, int nprod, int tile, const GemmParams& p, dim3 grid, hipStream_t st);  // gemm_gbf.hip
void gemm_run_hb(int tile, int ns, const GemmParams& p, dim3 grid, hipStream_t st);                         // gemm_hb.hip
void gemm_run_hbt(const GemmParams& p, dim3 grid, hipStream_t st);                                          // gemm_hb.hip
void gemm_run_hbx(int variant, const GemmParams& p, dim3 grid, hipStream_t st);                             // gemm_hbx.hip
void gemm_run_hbt4(const GemmParams& p, dim3 grid, hipStream_t st);                                         // gemm_hbx.hip
bool hbt4_ok(const GemmParams& p);  // the conv weight gradients on the four-phase kernel's TN form (gemm_hbx.hip)
// the row-per-lane (C^T accumulator) epilogue's operand conditions (gemm_hbx.hip)
bool hbx_t_ok(const GemmParams& p, bool check_off32);
// conv-A GEMM (segK > 0) eligible for the four-phase 256 x 256 kernel's CONV form (gemm_hbx.hip; p.off32 set)
bool hbp_conv_ok(const GemmParams& p);
