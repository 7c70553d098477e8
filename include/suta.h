/*
 * suta.h — C ABI of libsuta.so, the MI355X-native SUTA adapt-loop engine.
 *
 * The reference has no FFI for this path: it is Python calling HF transformers and
 * torch.optim.  Each entry point below replaces one reference
 * interface, cited as file:line:
 *
 *   suta_create          Wav2Vec2ForCTC.from_pretrained(...).eval() + configure_model +
 *                        collect_params + setup_optimizer + copy_model_and_optimizer
 *                        (reference main.py:302-311, 8-23, 62-103, 137-145, 167-170)
 *   suta_reset           load_model_and_optimizer — episodic restore (main.py:147-155, 327-328)
 *   suta_forward         `model(input_values).logits` under no_grad (main.py:331-332)
 *   suta_step            forward_and_adapt(...) — one SUTA step, reference schedule
 *                        (main.py:172-215)
 *   suta_step_ex         the same with forward_and_adapt's repeat_inference argument (main.py:211-215)
 *   suta_adapt           the per-utterance loop: vanilla forward + `steps` x forward_and_adapt
 *                        with recorded checkpoints (main.py:327-398), minimal schedule
 *                        ((S+1) forwards + S backwards), batched over utterances
 *   suta_adapt_varlen    the same over utterances of different lengths in one batch
 *   suta_loss_grad       softmax_entropy + mcc_loss (+ div_loss) and loss.backward() w.r.t. the
 *                        logits (main.py:26-60, 181-205): the fused loss kernel alone
 *   suta_get_param       model.state_dict()[name] of an adapted slot (main.py:139)
 *   suta_param_info      collect_params' entry multiplicity per trainable tensor
 *                        (main.py:79-94; duplicates => k Adam sub-steps per step)
 *   suta_num_frames      Wav2Vec2Model._get_feat_extract_output_lengths (HF modeling_wav2vec2.py)
 *
 * Conventions: plain pointers and sizes, float32 data, int32 status codes (0 = OK),
 * a thread-local message via suta_last_error().  No exceptions cross the ABI.
 * One engine per GPU per process; calls on one engine must be serialised by the caller.
 * A "slot" is one utterance's private state (trainable tensors + Adam moments);
 * an engine holds `max_batch` slots.  Batched calls process slots 0..batch-1 in lockstep
 * and are equivalent to `batch` independent batch-1 reference runs.
 */
#ifndef SUTA_H
#define SUTA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SUTA_OK 0
#define SUTA_ERR_ARG 1         /* invalid argument / shape / missing tensor            */
#define SUTA_ERR_HIP 2         /* HIP runtime failure                                   */
#define SUTA_ERR_UNSUPPORTED 3 /* configuration the engine does not implement           */
#define SUTA_ERR_OOM 4         /* device allocation failed                               */

#define SUTA_MAX_CONV 8

typedef struct suta_engine suta_engine;

/* HF Wav2Vec2Config fields that determine the arithmetic (configuration_wav2vec2.py:165-219). */
typedef struct suta_model_config {
    int32_t hidden_size;                   /* 768 base, 1024 large */
    int32_t num_hidden_layers;             /* 12 / 24 */
    int32_t num_attention_heads;           /* 12 / 16 */
    int32_t intermediate_size;             /* 3072 / 4096 */
    int32_t vocab_size;                    /* 32 */
    int32_t num_conv_layers;               /* 7 */
    int32_t conv_dim[SUTA_MAX_CONV];
    int32_t conv_kernel[SUTA_MAX_CONV];
    int32_t conv_stride[SUTA_MAX_CONV];
    int32_t conv_bias;                     /* 0 base, 1 large */
    int32_t feat_extract_norm_layer;       /* 0 = "group" (base), 1 = "layer" (large) */
    int32_t do_stable_layer_norm;          /* 0 post-LN (base), 1 pre-LN (large) */
    int32_t num_conv_pos_embeddings;       /* 128 */
    int32_t num_conv_pos_embedding_groups; /* 16 */
    float layer_norm_eps;                  /* 1e-5 */
} suta_model_config;

/* forward_and_adapt / setup_optimizer / collect_params arguments (main.py:8-23, 62-103, 172-173)
 * and the CLI flags of main.py:221-241. */
typedef struct suta_hparams {
    float lr;             /* --lr (AdamW lr) */
    float temp;           /* --temp */
    float em_coef;        /* --em_coef */
    float div_coef;       /* --div_coef */
    float beta1, beta2;   /* AdamW betas (0.9, 0.999) */
    float adam_eps;       /* 1e-8 */
    float weight_decay;   /* setup_optimizer passes 0 */
    int32_t reweight;     /* --reweight */
    int32_t non_blank;    /* --non_blank */
    int32_t train_feature;/* --train_feature */
    int32_t bias_only;    /* --bias_only */
    int32_t episodic;     /* --episodic: reset every slot before adapting */
    float pl_coef;        /* SDPL (main_SDPL.py:143-209): loss = (1 - pl_coef) * SUTA + pl_coef *
                             pseudo-label CTC; 0 = SUTA only (main.py); main_SDPL's driver passes 1 */
    int32_t optimizer;    /* --opt (main.py:9-18): SUTA_OPT_ADAMW (AdamW, or Adam: identical at weight decay 0)
                             or SUTA_OPT_SGD (torch.optim.SGD(lr, weight_decay=0): p -= lr * g once per
                             collect_params entry, the single-tensor order) */
    int32_t lr_step_size; /* --scheduler torch.optim.lr_scheduler.StepLR (main.py:20-21: step_size 1, gamma
                             0.7), stepped after every optimizer step (main.py:207-208) and restored with the
                             episodic reset (main.py:147-152): optimizer step i (counted from the last reset)
                             uses lr * gamma^floor(i / lr_step_size), the products taken in double as torch
                             does; 0 = no scheduler */
    float lr_gamma;
} suta_hparams;

#define SUTA_OPT_ADAMW 0
#define SUTA_OPT_SGD 1

/* Weights: `n` tensors named by their HF state_dict key (e.g.
 * "wav2vec2.encoder.layers.0.attention.q_proj.weight"), float32, host memory, HF layout.
 * max_samples: longest utterance any later call may pass (the reference truncates to 600000,
 * data.py); longer inputs return SUTA_ERR_ARG; <= 0 means no limit beyond T <= 2048 frames. */
int32_t suta_create(const suta_model_config* cfg, const char* const* names, const float* const* data,
                    const int64_t* numels, int32_t n, int32_t device, int32_t max_batch,
                    int64_t max_samples, suta_engine** out);

int32_t suta_destroy(suta_engine* e);

/* Restore every slot's trainable tensors to the pristine copy and clear Adam state. */
int32_t suta_reset(suta_engine* e);

/* Frames T produced for an utterance of n_samples (conv length recursion). */
int32_t suta_num_frames(const suta_model_config* cfg, int64_t n_samples, int64_t* frames_out);

/* Vanilla no-grad forward of slots 0..batch-1 on `batch` utterances of n_samples each.
 * wav: batch x n_samples float32 (host if wav_on_device == 0, else device pointer).
 * normalize != 0 applies the HF processor's zero-mean/unit-variance normalisation first.
 * logits_out: batch x T x vocab float32 host buffer. */
int32_t suta_forward(suta_engine* e, const float* wav, int32_t wav_on_device, int32_t normalize,
                     int32_t batch, int64_t n_samples, float* logits_out);

/* One forward_and_adapt step per slot with the reference schedule (grad forward, loss,
 * backward, AdamW, no-grad re-forward).  logits_out (host, batch x T x vocab) receives the
 * re-inference logits; loss_out (host, batch floats, may be NULL) the SUTA loss value. */
int32_t suta_step(suta_engine* e, const float* wav, int32_t wav_on_device, int32_t normalize,
                  int32_t batch, int64_t n_samples, const suta_hparams* hp, float* logits_out,
                  float* loss_out);

/* suta_step with forward_and_adapt's `repeat_inference` argument (main.py:172-173, 211-215): != 0 returns the
 * no-grad re-inference logits after the update (suta_step), 0 returns the grad forward's logits -- the ones the
 * loss was taken on -- and skips the re-forward.  logits_out is a device pointer when logits_on_device != 0.
 * The forward_and_adapt-compatible Python shim (suta_amd/suta.py) calls this entry. */
int32_t suta_step_ex(suta_engine* e, const float* wav, int32_t wav_on_device, int32_t normalize,
                     int32_t batch, int64_t n_samples, const suta_hparams* hp, int32_t repeat_inference,
                     float* logits_out, int32_t logits_on_device, float* loss_out);

/* Episodic SUTA on `batch` utterances: (reset if hp->episodic), vanilla forward, `steps`
 * adaptation steps.  record_steps[0..n_record) are step counts r in [0, steps] (0 = vanilla);
 * for each, logits after r updates go to logits_out[(i*batch + b)*T*vocab ...] (host or device
 * per logits_on_device; may be NULL) and greedy ids to ids_out[(i*batch + b)*T ...] (host,
 * may be NULL).  frames_out receives T.  With hp->episodic == 0 the slots continue from
 * their current state (reference non-episodic mode; use batch 1). */
int32_t suta_adapt(suta_engine* e, const float* wav, int32_t wav_on_device, int32_t normalize,
                   int32_t batch, int64_t n_samples, int32_t steps, const suta_hparams* hp,
                   const int32_t* record_steps, int32_t n_record, float* logits_out,
                   int32_t logits_on_device, int32_t* ids_out, int64_t* frames_out);

/* suta_adapt over a ragged batch: utterance b has n_samples[b] samples at wav + b*stride
 * (stride >= max n_samples; stride is also the layout length, so a caller can quantise it to
 * let repeated layouts replay the captured SUTA step), and is adapted exactly as if it were run alone (the reference
 * processes one utterance per forward_and_adapt, main.py:327-398; no padding enters any
 * statistic, softmax or gradient).  frames_out receives `batch` frame counts T_b.  logits_out /
 * ids_out use the layout: [n_record][batch][Tl][vocab] / [..][Tl], Tl = suta_num_frames(stride);
 * rows t >= T_b of utterance b are padding. */
int32_t suta_adapt_varlen(suta_engine* e, const float* wav, int32_t wav_on_device, int32_t normalize,
                          int32_t batch, const int64_t* n_samples, int64_t stride, int32_t steps,
                          const suta_hparams* hp, const int32_t* record_steps, int32_t n_record,
                          float* logits_out, int32_t logits_on_device, int32_t* ids_out,
                          int64_t* frames_out);

/* The fused entropy+MCC loss-and-gradient kernel alone (softmax_entropy / mcc_loss / div_loss and
 * the loss assembly of main.py:26-60, 181-203) on `batch` host logit blocks of T x vocab.
 * dlogits_out: batch x T x vocab (host); loss_out: batch floats (host). */
int32_t suta_loss_grad(suta_engine* e, const float* logits, int32_t batch, int64_t frames,
                       const suta_hparams* hp, float* dlogits_out, float* loss_out);

/* Copy slot `slot`'s current value of trainable tensor `name` (HF layout) to host `out`. */
int32_t suta_get_param(suta_engine* e, int32_t slot, const char* name, float* out, int64_t numel);

/* Multiplicity k (number of collect_params entries, 0 = frozen) for trainable tensor `name`
 * under the given flags. */
int32_t suta_param_info(suta_engine* e, const char* name, int32_t train_feature, int32_t bias_only,
                        int32_t* multiplicity_out, int64_t* numel_out);

/* Wait for all work of the engine's stream. */
int32_t suta_sync(suta_engine* e);

/* hipStream_t the engine launches on (as void*), for callers that time with HIP events. */
void* suta_stream(suta_engine* e);

/* Per-kernel-family device time (ms) accumulated with HIP events while timing is enabled
 * (family 0 = MFMA GEMM, 1 = attention softmax, 2 = norm, 3 = elementwise/other,
 * 4 = loss, 5 = adam); counts = launches.  enable != 0 also clears the counters. */
int32_t suta_set_timing(suta_engine* e, int32_t enable);
int32_t suta_get_timing(suta_engine* e, double* ms_out /*[6]*/, int64_t* launches_out /*[6]*/);

/* The same counters over SUTA_TIMING_FAMILIES finer families (the first nfam are written): 0 = MFMA
 * GEMMs and the positional-conv kernel, 1 = softmax-backward row term, 2 = norm, 3 = elementwise,
 * 4 = loss, 5 = adam, 6 = conv feature-encoder front-end (conv0 + GroupNorm / conv0), 7 = fused
 * attention kernels; alg_bytes_out (may be null) = algorithmic HBM bytes of the timed launches (each
 * operand touched once; GEMM families only, 0 elsewhere).  (bench.py roofline; no reference
 * counterpart: the reference has no kernel timing.) */
#define SUTA_TIMING_FAMILIES 8
int32_t suta_get_timing_ex(suta_engine* e, int32_t nfam, double* ms_out, int64_t* launches_out,
                           double* alg_bytes_out);

/* GEMM launch census (process-wide; not in the reference, test/bench instrumentation): while enabled,
 * every GEMM launch the engine issues (eagerly or while capturing a graph; replays issue none) is
 * counted per "<kernel> <BMxBN> z=<batch> split=<k> <A/B form>" key.  suta_set_census(1) clears and
 * starts it, suta_get_census copies "key count\n" lines (needed = bytes incl. the NUL).  Used by
 * tests/test_gpu_bench_scale.py to assert which tile and weight-gradient schedule a layout reaches. */
int32_t suta_set_census(int32_t enable);
int32_t suta_get_census(char* buf, int64_t cap, int64_t* needed);

/* GEMM arithmetic.  The first two are fp32-accurate; results agree to fp32 rounding
 * (tests/test_gpu_parity.py):
 *   SUTA_PRECISION_FP32_MFMA        v_mfma_f32_32x32x2_f32: exact fp32 products, fp32 accumulation
 *   SUTA_PRECISION_FP32_SPLIT_BF16  each fp32 operand split exactly into 3 bf16 terms; the 6 products
 *                                   of order <= 2 on v_mfma_f32_32x32x16_bf16, fp32 accumulation
 *                                   (dropped terms <= 2^-24 |ab|: the size of one fp32 rounding)
 *   SUTA_PRECISION_BF16             bf16 GEMMs (config C4, the reference has no bf16 path): every GEMM
 *                                   operand rounded to bf16 (RNE) as it enters the MFMA, fp32
 *                                   accumulation; activations, norms, softmax, loss, AdamW and the
 *                                   trainable master tensors stay fp32 (torch.autocast(bf16)
 *                                   semantics for the matmuls) -- tests/parity.py (assert_bf16_close) states the
 *                                   tolerance, tests/test_gpu_large_bf16.py applies it */
#define SUTA_PRECISION_FP32_MFMA 0
#define SUTA_PRECISION_FP32_SPLIT_BF16 1
#define SUTA_PRECISION_BF16 2
int32_t suta_set_precision(suta_engine* e, int32_t mode);

/* Use hipGraph capture/replay for suta_adapt (default on): when a call repeats the previous call's
 * key (batch, layout, ragged, precision, hparams, steps, record set, requested outputs), the call's
 * whole loop -- episodic slot reset, vanilla forward, steps x (backward + AdamW + forward), recorded
 * logits and greedy ids into device staging -- is captured once as one graph and replayed per call;
 * a call with a new key runs eagerly.  Per-kernel timing (suta_set_timing) disables it. */
int32_t suta_set_graphs(suta_engine* e, int32_t enable);

/* How the last suta_adapt / suta_adapt_varlen call ran its loop, and totals over the engine's life
 * (instrumentation, no reference counterpart; tests pin that the bench's timed mode -- graph replay --
 * is the one checked against the oracle): last_mode_out = 0 eager, 1 captured then launched, 2 replayed
 * an earlier capture; captures_out / launches_out = graphs captured / graph launches so far. */
#define SUTA_LOOP_EAGER 0
#define SUTA_LOOP_CAPTURED 1
#define SUTA_LOOP_REPLAYED 2
int32_t suta_get_graph_stats(suta_engine* e, int32_t* last_mode_out, int64_t* captures_out, int64_t* launches_out);

const char* suta_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SUTA_H */
