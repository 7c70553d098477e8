// Launchers for the non-GEMM kernels of the SUTA step (ops.hip).  All tensors are fp32,
// time-major ([frame][channel]) and packed over the utterances of a batch.
#pragma once
#include "common.h"

// HF feature-extractor normalisation (feature_extraction_wav2vec2.py:78-97), per utterance:
// y = (x - mean) / sqrt(var + 1e-7), population variance.  lens (device, may be null): ragged batch,
// utterance b has lens[b] <= N samples at stride N; its padding samples are written as 0.
void launch_wave_normalize(const float* x, float* y, int B, long N, const int* lens, hipStream_t st);

// conv0: z[b][t][c] = sum_k x[b][s*t + k] * W[b][k][c] (+ bias[b][c]);  W stored [k][c] per utterance.
void launch_conv0(const float* x, long N, const float* W, const float* bias, long wstride, float* z, int B, int L0,
                  int C, int K, int S, hipStream_t st, void* zb = nullptr);  // zb: bf16 output instead of z

// Fused conv0 + GroupNorm + GELU (group mode): conv0 is recomputed from the waveform in each pass.
// fwd: mean/rstd per (utterance, channel) and a = gelu(GN(conv0(x))).  dpart: >= B*ceil(L0/128)*2*C + B*C doubles.
// L0s (device, may be null): ragged batch, utterance b has L0s[b] <= L0 valid frames (statistics and
// gradients over those only).
void launch_front_gn_fwd(const float* x, long N, const float* W, const float* bias, long wstride, int B, int L0, int C,
                         int K, int S, const float* g, const float* beta, float* mean, float* rstd, float* a,
                         double* dpart, const int* L0s, hipStream_t st);
// bwd: da (overwritten with dg) -> dgamma, dbeta and the conv0 weight gradient dW[k][c] (gstride per
// utterance).  fpart: >= B*ceil(L0/128)*K*C floats.
void launch_front_gn_bwd(const float* x, long N, const float* W, const float* bias, long wstride, int B, int L0, int C,
                         int K, int S, const float* g, const float* beta, const float* mean, const float* rstd,
                         float* da, float* dgamma, float* dbeta, float* dW, long gstride, double* dpart, float* fpart,
                         const int* L0s, hipStream_t st);

// LayerNorm over the last dim D of `rows` rows; gamma/beta of utterance (row / rows_per_utt)
// at pstride.  Stores y, xhat, rstd.  gelu_out: y = gelu(LN(x)) (feature-encoder "layer" mode).
void launch_layernorm_fwd(const float* x, const float* g, const float* beta, long pstride, int rows_per_utt,
                          float* y, float* xhat, float* rstd, int rows, int D, float eps, int gelu_out,
                          hipStream_t st, void* yb = nullptr, float* mean = nullptr, const void* xb = nullptr);
// yb: optional bf16 copy of y (bf16-plane GEMMs); xhat may be null when `mean` is given: the row means
// are stored instead and the backward recomputes x-hat from the (stored) input; xb: the input as a bf16 plane
// (x null; vectorised widths)
// LayerNorm backward.  gin = dy (times gelu'(xhat*g+beta) when gelu_in); dx = LN-bwd(gin)
// (times gelu'(post_aux) when post_aux) (+ resid).  dgamma/dbeta (may be null) summed per
// utterance into the grad buffer (gstride per utterance).  part: >= B*ceil(rows_per_utt/16)*2*D floats.
void launch_layernorm_bwd(const float* dy, const float* xhat, const float* rstd, const float* g, const float* beta,
                          long pstride, int rows_per_utt, int B, int D, int gelu_in, const float* post_aux,
                          const float* resid, float* dx, float* dgamma, float* dbeta, long gstride, float* part,
                          hipStream_t st, void* dxb = nullptr, const float* x = nullptr, const float* mean = nullptr,
                          const void* dyb = nullptr);
// dxb: optional bf16 copy of dx; xhat null: x-hat = (x - mean) * rstd recomputed from the LayerNorm input;
// dyb: dy given as a bf16 plane instead (dy must be null; vectorised widths 512 / 768 / 1024 only)

// Layer-mode conv stack (D = 512, GELU after the LayerNorm, x-hat recomputed from the stored conv output x and
// its row means): the LayerNorm backward that also sums the conv bias gradient (dbias, may be null) and, with
// ktaps = 10 (conv0), the weight gradient dw[k][c] = sum_t xw[xs t + k] dx[t][c] (xw: the waveform, xws per
// utterance) -- dgamma / dbeta / dbias / dw per utterance at gstride.  Returns false when the shape is not
// covered (the caller then runs launch_layernorm_bwd + launch_colsum + its GEMM).  part: >=
// layernorm_bwd_conv_part_floats(...) floats.
long layernorm_bwd_conv_part_floats(int B, int rows_per_utt, int D, int ktaps);
bool launch_layernorm_bwd_conv(const float* dy, const float* rstd, const float* g, const float* beta, long pstride,
                               int rows_per_utt, int B, int D, float* dx, float* dgamma, float* dbeta, float* dbias,
                               float* dw, long gstride, float* part, hipStream_t st, const float* x, const float* mean,
                               const float* xw, long xws, int xs, int ktaps, void* dxb = nullptr, int bf16_in = 0);
// bf16_in: bit 0 dy, bit 1 x given as bf16 planes (the pointers reinterpreted; conv stack on bf16 planes)
// Column sums per utterance: out[b][c] = sum_{t < rows} x[b][t][c]   (bias gradients).
void launch_colsum(const float* x, int B, int rows, int C, float* out, long ostride, float* part, hipStream_t st);

// Flash-style fused attention (attn.hip), head dim 64, any T: forward writes ctx and the per-row
// log-sum-exp lse[b][head][t] (no T x T matrix); backward recomputes P from lse and writes dQ, dK, dV
// into dqkv's Q/K/V columns (dqp: flash_dq_scratch_floats floats of per-key-block dQ partials).
// delta[b][head][t] = rowsum(dctx * ctx) (launch_attn_delta).  bf16: operands rounded to bf16 on the bf16
// MFMAs (config C4).  false (nothing launched) when dh != 64.
long flash_dq_scratch_floats(int B, int T, int NH);
// ctxb / dqkvb (may be null): bf16 copies of ctx / dqkv for the bf16-plane GEMMs that consume them.
// qkv may be null when the launch takes the bf16-plane kernel (flash_*_reads_plane[s]: the engine's test for
// leaving the fp32 qkv unwritten); the launch throws otherwise.
bool flash_fwd_reads_plane(bool bf16, const void* qkvb, int H);
bool flash_bwd_reads_planes(bool bf16, const void* qkvb, const void* dctxb, int H);
bool launch_flash_fwd(const float* qkv, float* ctx, float* lse, int B, int T, int NH, int H, int dh, float scale,
                      const int* tlen, bool bf16, hipStream_t st, void* ctxb = nullptr, const void* qkvb = nullptr);
bool launch_flash_bwd(const float* qkv, const float* dctx, const float* lse, const float* delta, float* dqkv,
                      float* dqp, int B, int T, int NH, int H, int dh, float scale, const int* tlen, bool bf16,
                      hipStream_t st, void* dqkvb = nullptr, const void* qkvb = nullptr,
                      const void* dctxb = nullptr);
// grouped positional conv (group width 48 or 64, exact fp32 MFMA); fwd: C = R + gelu(conv + bias), C2 = conv + bias;
// bwd: C = conv + R (rows >= tlen -> 0).  false (nothing launched) outside the supported shapes
bool launch_posconv(bool fwd, const float* x, const float* W, const float* bias, const float* R, float* C, float* C2,
                    int B, int T, int H, int G, int K, int pad, const int* tlen, hipStream_t st);
// bf16 mode, group width 64: Wt = bf16 weights [G][K][n][k] (n = output channel, k = input channel)
bool launch_posconv_bf16(bool fwd, const float* x, const void* Wt, const float* bias, const float* R, float* C,
                         float* C2, int B, int T, int H, int G, int K, int pad, const int* tlen, hipStream_t st);
// In-place row softmax of `nrows` rows of length T (row stride ld).  tlen (device, may be null):
// ragged batch, rows of utterance row / rows_per_utt use their first tlen[u] keys; the rest get 0.
// (GEMM attention path: head dims other than 64)
void launch_softmax_rows(float* s, long nrows, int T, long ld, const int* tlen, long rows_per_utt, hipStream_t st);

// delta[b][h][t] = dot(dO[b][t][head h], O[b][t][head h]): the softmax-backward row term sum_j P_ij dP_ij.
void launch_attn_delta(const float* dO, const float* O, float* delta, int B, int T, int NH, int dh, hipStream_t st);

// out = g * gelu'(z), n elements.
void launch_dgelu_mul(const float* g, const float* z, float* out, long n, hipStream_t st);

// SUTA loss + dL/dlogits for each utterance (reference main.py:26-60, 181-203).
struct LossHP {
    float temp, em_coef, div_coef;
    int reweight, non_blank;
};
// tlen (device, may be null): ragged batch, utterance b has tlen[b] <= T frames at stride T; the
// gradient of its padding frames is written as 0.
void launch_suta_loss(const float* logits, int B, int T, int V, LossHP hp, const int* tlen, float* dlogits, float* loss,
                      float* scratch, hipStream_t st);

// SDPL pseudo-label CTC objective (main_SDPL.py:143-209; sdpl.hip): mixes pl_coef * L_ctc into the
// SUTA loss / gradient already in loss / dlogits (V <= 32).  scratch: B * sdpl_scratch_floats(T)
// floats; *err |= 1 when a pseudo-label transcript holds a special token (the reference raises).
long sdpl_scratch_floats(int T);
void launch_sdpl_loss(const float* logits, int B, int T, int V, float pl_coef, const int* tlen, float* dlogits,
                      float* loss, float* scratch, int* err, hipStream_t st);

// Argmax ids per frame (first max, like torch.argmax), optional copy of logits.
void launch_argmax(const float* logits, long rows, int V, int* ids, hipStream_t st);

// AdamW single-tensor semantics with per-run multiplicity k (k sub-steps with the same gradient).
struct AdamRun {
    long start, len;
    int k;
};
#define SUTA_MAX_RUNS 24
#define ADAM_TAB 52  // floats per optimizer step in the device step table
struct AdamArgs {
    int nruns;
    AdamRun runs[SUTA_MAX_RUNS];
    int blk0[SUTA_MAX_RUNS];  // first block of each run (filled by launch_adam)
    float beta1, beta2, omb1, omb2, eps, lr_wd;  // omb = (1 - beta) rounded from double; lr_wd = lr * wd
    int sgd;  // SUTA_OPT_SGD: p = fma(g, -lr, p) per sub-step (no moments); the step table's [51] holds -lr
    // per sub-step j (1-based t = step0*k + j): step_size and sqrt(bias_correction2), indexed [k-1][j-1]
    float step_size[5][5];
    float bc2_sqrt[5][5];
    // device-resident alternative (graph-replayable): tab[step0 * ADAM_TAB + {0|25} + (k-1) * 5 + j-1] =
    // step_size | bc2_sqrt, tab[.. + 50] = the weight-decay factor 1 - lr_i wd, tab[.. + 51] = -lr_i (SGD), lr_i
    // the scheduled lr of step step0; step0 read from *step (advanced by launch_step_advance); used when tab !=
    // null.  At *step == 0 the moments are taken as zero (not read): every reset of the slots sets the step
    // counter to 0
    const float* tab;
    const int* step;
};
// dst[b][0:n] = src[0:n] for b in [0, B) (n a multiple of 4, 16-B aligned): the episodic slot reset.
void launch_broadcast(float* dst, const float* src, long n, int B, hipStream_t st);
// *step += 1 (one thread): the Adam step counter of graph-replayed SUTA steps.
void launch_step_advance(int* step, hipStream_t st);
void launch_adam(float* P, const float* G, float* M, float* V, long pstride, int B, const AdamArgs& a,
                 hipStream_t st);
