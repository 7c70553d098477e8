// libsuta engine: the SUTA adapt loop (reference main.py:172-215, 327-398) on gfx950.
//
// Per batch of utterances (same length, one slot each) the engine runs, per step:
//   forward with saved activations -> fused entropy+MCC loss-and-grad -> hand-written backward
//   (dX through every frozen op, dW only for collect_params' tensors) -> AdamW with the
//   duplicate-entry multiplicity -> next step's forward doubles as this step's re-inference.
// Layout: every activation is time-major [utterance][frame][channel] in HBM; trainable tensors
// of slot b live in one flat buffer P[b][Pn] (conv weights stored [k][c_in][c_out] so every
// conv layer is a strided-row GEMM); frozen encoder weights are shared by all slots.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/suta.h"
#include "common.h"
#include "ops.h"

namespace {

thread_local std::string g_err;

struct SutaError : std::runtime_error {
    int code;
    SutaError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIPCHK(x)                                                                                        \
    do {                                                                                                 \
        hipError_t _e = (x);                                                                             \
        if (_e != hipSuccess)                                                                            \
            throw SutaError(_e == hipErrorOutOfMemory ? SUTA_ERR_OOM : SUTA_ERR_HIP,                      \
                            std::string(#x) + ": " + hipGetErrorString(_e));                             \
    } while (0)

inline long rup(long a, long b) { return (a + b - 1) / b * b; }

// shortest decimal of a float, read back as a double (0.9f -> 0.9)
inline double py_double(float f) {
    char buf[48];
    snprintf(buf, sizeof buf, "%.9g", (double)f);
    double best = atof(buf);
    for (int prec = 1; prec <= 9; ++prec) {
        snprintf(buf, sizeof buf, "%.*g", prec, (double)f);
        const double d = atof(buf);
        if ((float)d == f) {
            best = d;
            break;
        }
    }
    return best;
}

struct Cfg {
    int H, L, NH, F, V, nconv;
    int C[SUTA_MAX_CONV], K[SUTA_MAX_CONV], S[SUTA_MAX_CONV];
    int conv_bias, layer_mode, stable, posK, posG;
    float eps;
};

// trainable tensor descriptor
struct TP {
    std::string name;
    std::vector<long> shape;  // HF shape
    long off = 0, numel = 0;
    bool conv_w = false;      // stored permuted [k][cin][cout]
    bool ln_member = false;   // belongs to an nn.LayerNorm module
    bool is_bias = false;
    int feat_depth = 0;       // feature-branch module count containing it (train_feature)
};

// kernel families of the per-launch timing (suta_get_timing_ex); the legacy 6-family view folds
// F_ATTN into F_GEMM and F_FRONT into F_NORM
enum Fam { F_GEMM = 0, F_SOFTMAX = 1, F_NORM = 2, F_EW = 3, F_LOSS = 4, F_ADAM = 5, F_FRONT = 6, F_ATTN = 7, NFAM = 8 };

struct DevBuf {
    float* p = nullptr;
    size_t bytes = 0;
    // returns true when (re)allocated
    bool alloc(size_t b) {
        if (b <= bytes) return false;
        if (p) HIPCHK(hipFree(p));
        p = nullptr;
        bytes = 0;
        HIPCHK(hipMalloc(&p, b));
        bytes = b;
        return true;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// SUTA_FUSED_CONV_LN=0: the layer-mode conv stack's LayerNorm backward without the fused bias / conv0 weight
// gradient sums (separate column-sum pass and GEMM), for A/B runs; from the call's switch snapshot
static bool fused_conv_ln() { return suta_switches().fused_conv_ln != 0; }

struct Arena {
    char* base = nullptr;
    size_t off = 0, cap = 0;
    bool dry = true;
    template <typename T>
    T* take(size_t n) {
        off = rup(off, 256);
        T* r = dry ? nullptr : reinterpret_cast<T*>(base + off);
        off += n * sizeof(T);
        return r;
    }
};

// Algorithmic (compulsory) HBM bytes of one GEMM launch: every operand element touched once — A's unique
// rows (overlapping strided conv rows and conv-A windows counted once), B once per distinct batch slice
// (shared weights once), C written (read too when accumulating), and the epilogue's stored
// pre-activation, residual and auxiliary operands.  Split-K partials and tile re-reads are not counted.
// Element sizes follow what the launch reads and writes: 2 B for a bf16 operand plane (Ab, Bb), the bf16 C
// plane (Cb) and the bf16 pre-activation operands (preb: C2 / aux), 4 B for fp32 operands; an fp32 C that is
// not written (p.C null: the bf16 plane is the only output) costs nothing.  a_fp32: A is read as fp32 even
// though p.Ab is set (the to_bf16 conversion inside the same timed launch reads the fp32 source once).
double gemm_alg_bytes(const GemmParams& p, bool a_fp32 = false) {
    auto zeff = [&](long s0, long s1) -> double {
        if (s0 == 0 && s1 == 0) return 1.0;
        if (s0 == 0) return (double)((p.Z + p.zdiv - 1) / std::max(1, p.zdiv));
        return (double)p.Z;
    };
    const bool bf = p.mode == SUTA_PRECISION_BF16;
    const double ea = (bf && p.Ab && !a_fp32) ? 2.0 : 4.0;
    const double eb = (bf && p.Bb) ? 2.0 : 4.0;
    const double epre = p.preb ? 2.0 : 4.0;
    double a;
    if (p.segK > 0) {
        const long rows = std::min<long>((long)p.M + p.K / p.segK - 1, p.Mvalid > 0 ? p.Mvalid : p.M);
        a = (double)rows * p.segK;
    } else if (!p.ta) {
        const long lda = (bf && p.Ab && !a_fp32) ? p.ldab : p.lda;
        a = lda < p.K ? (double)(p.M - 1) * lda + p.K : (double)p.M * p.K;
    } else {
        const long lda = (bf && p.Ab && !a_fp32) ? p.ldab : p.lda;
        a = lda < p.M ? (double)(p.K - 1) * lda + p.M : (double)p.M * p.K;
    }
    const double mn = (double)p.M * p.N;
    double bytes = ea * a * zeff(p.sA0, p.sA1) + eb * (double)p.K * p.N * zeff(p.sB0, p.sB1);
    double c = 0.0;
    if (p.C) c += 4.0 * mn * ((p.epi & EPI_ACCUM) ? 2 : 1);
    if (p.Cb && bf) c += 2.0 * mn;
    if (p.epi & EPI_STORE_PRE) c += epre * mn;
    if (p.epi & EPI_RESID) c += 4.0 * mn;
    if (p.epi & EPI_DGELU) c += epre * mn;
    if (p.epi & EPI_SMBWD) c += 4.0 * mn;
    if (p.epi & EPI_DELTA) c += 4.0 * mn + 4.0 * (double)p.M * p.dNH;  // O read, delta written
    bytes += c * p.Z;
    return bytes;
}

struct LayerBufs {
    float *x_in, *xhat1, *rstd1, *y1, *qkv, *P, *lse, *ctx, *hmid, *xhat2, *rstd2, *y2, *u, *x_out;
    float *mean1, *mean2;  // row means when x-hat is recomputed from the stored LayerNorm input (xhat null)
};

struct Plan {
    int B = 0;
    long N = 0;
    int Lc[SUTA_MAX_CONV];
    int T = 0, Tp = 0;
    // ragged batch: utterance b has n[b] <= N samples, L0[b] conv0 frames and T[b] <= T frames
    // (device copies); the layout (strides) stays that of the longest utterance, N
    bool ragged = false;
    int *len_n = nullptr, *len_L0 = nullptr, *len_T = nullptr;
    std::vector<int> h_n, h_T;
    // forward
    float *xraw, *x;
    float *z[SUTA_MAX_CONV], *a[SUTA_MAX_CONV], *cxhat[SUTA_MAX_CONV], *crstd[SUTA_MAX_CONV], *cmean[SUTA_MAX_CONV];
    float *gn_mean, *gn_rstd;
    float *fp_xhat, *fp_rstd, *fp_y, *h0, *pz, *e, *enc_xhat, *enc_rstd, *enc_y;
    float *fp_mean, *enc_mean;
    // LayerNorms whose input stays stored keep only the row means (x-hat recomputed in the backward):
    // the conv LNs of layer mode, the feature-projection LN, the encoder LN, and every LN of stable
    // (pre-LN) layers; post-LN layers' LN inputs are transient and keep x-hat
    std::vector<LayerBufs> lay;
    long lnpart_floats = 0;
    float *ctx, *gu, *rtmp, *logits;
    // backward
    float *dlogits, *d1, *d2, *d3, *dqkv, *dP, *dqp, *du, *dzc, *dzc2, *lnpart, *loss, *loss_scratch, *c0part, *delta;
    bool flash = false;  // flash attention kernels (head dim 64): no T x T matrices, per-row LSE
    double* dpart;
    int* ids;
    float* splitws;
    long splitws_floats;
    size_t bytes;
};

}  // namespace

struct suta_engine {
    Cfg c;
    int device = 0;
    hipStream_t st = nullptr;
    int max_batch = 0;
    long max_samples = 0;
    bool attn_fused = true;  // fused attention fwd/bwd kernels where their shape holds; env SUTA_ATTN_FUSED=0 off
    bool posconv_kernel = true;  // dedicated positional-conv kernel (exact fp32 mode); env SUTA_POSCONV=0 off
    bool bf16_planes = true;     // bf16 mode: linears on bf16 operand planes; env SUTA_BF16_PLANES=0 off
    // frozen weights
    std::vector<float*> wqkv, bqkv, wo, bo, w1, b1, w2, b2;
    float *wpos_f = nullptr, *wpos_b = nullptr, *bpos = nullptr, *wlm = nullptr, *blm = nullptr;
    // bf16 positional-conv weights [G][K][n][k] (fwd: n = c_out, k = c_in; bwd: taps flipped, n = c_in, k = c_out)
    // for posconv_bf16_kernel (group width 64); null otherwise
    void *wpos_bf_f = nullptr, *wpos_bf_b = nullptr;
    // trainable
    std::vector<TP> tps;
    std::map<std::string, int> tpi;
    long Pn = 0;
    float *P0 = nullptr, *P = nullptr, *G = nullptr, *Mo = nullptr, *Vo = nullptr;
    long opt_steps = 0;
    // offsets of trainable pieces
    long o_cw[SUTA_MAX_CONV], o_cb[SUTA_MAX_CONV], o_cg[SUTA_MAX_CONV], o_cbeta[SUTA_MAX_CONV];
    long o_fpg, o_fpb, o_pw, o_pb, o_eg, o_eb;
    std::vector<long> o_l1g, o_l1b, o_l2g, o_l2b;
    // workspace
    DevBuf ws;
    Plan plan;
    DevBuf sdpl_ws;  // SDPL CTC scratch (+ error flag), allocated on first use
    bool sdpl_used = false;
    int* sdpl_err = nullptr;
    // after a call that ran the SDPL objective: a pseudo-label transcript held <s>, </s> or <unk>
    void check_sdpl() {
        if (!sdpl_used) return;
        int e = 0;
        HIPCHK(hipMemcpy(&e, sdpl_err, sizeof(int), hipMemcpyDeviceToHost));
        HIPCHK(hipMemset(sdpl_err, 0, sizeof(int)));
        sdpl_used = false;
        if (e)
            throw SutaError(SUTA_ERR_UNSUPPORTED,
                            "SDPL pseudo label contains a special token (<s>, </s>, <unk>): the reference's "
                            "vocab lookup raises KeyError (main_SDPL.py:196-200)");
    }
    // timing
    bool timing = false;
    double fam_ms[NFAM] = {0};
    long fam_n[NFAM] = {0};
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
    std::vector<hipEvent_t> evpool;
    bool use_graphs = true;
    int gemm_mode = 0;  // SUTA_PRECISION_*
    // Adam step tables on the device (tab[step0][step_size | bc2_sqrt][k-1][j-1]) and the step counter the
    // kernel reads: a captured SUTA step replays with the right bias corrections
    float* d_adam_tab = nullptr;
    long adam_tab_cap = 0;
    int* d_step = nullptr;
    int h_step = 0;
    // host rows [0, h_lr.size()) of the table for the optimizer scalars in tab_hp (h_lr = each step's scheduled lr,
    // the StepLR chained product carried row to row); rows [0, dev_rows) are on the device.  A non-episodic run
    // grows them by `steps` rows per call instead of rebuilding every row since its start (advisor r5)
    std::vector<float> h_tab;
    std::vector<double> h_lr;
    long dev_rows = 0;
    suta_hparams tab_hp{};
    double lr_at(const suta_hparams& hp, long i);
    // the whole S-step loop of one suta_adapt call (slot reset, forward, S x (backward + Adam + forward),
    // recorded argmax ids and logits into device staging) captured as one graph per key
    struct GraphKey {
        int B = 0;
        long N = 0;
        int ragged = 0, mode = 0, steps = 0, want_logits = 0, want_ids = 0;
        suta_hparams hp{};
        std::vector<int> rec;
        SutaSwitches sw{};  // the call's A/B switch snapshot (buffer formats and kernel choices captured)
    };
    hipGraphExec_t loop_graph = nullptr;
    int last_loop_mode = SUTA_LOOP_EAGER;  // suta_get_graph_stats
    long graph_captures = 0, graph_launches = 0;
    GraphKey gkey;
    bool gkey_seen = false;  // key of the previous suta_adapt call (its lazy allocations are done)
    DevBuf recbuf;           // recorded logits [nrec][B*T*V] then ids [nrec][B*T]
    void prepare_adam(const suta_hparams& hp, int steps);
    bool graph_key_repeats(const GraphKey& k);
    void adapt_loop(int B, const suta_hparams& hp, int steps, const int* rec, int nrec, float* rec_logits,
                    int* rec_ids);
    void run_adapt_loop(int B, const suta_hparams& hp, int steps, const int* rec, int nrec, float* rec_logits,
                        int* rec_ids, bool graph_ok);
    void drop_graph() {
        if (loop_graph) (void)hipGraphExecDestroy(loop_graph);
        loop_graph = nullptr;
        gkey_seen = false;
    }
    std::vector<float*> owned;

    ~suta_engine();

    // ---------------- helpers ----------------
    float* dalloc(long n) {
        float* p = nullptr;
        HIPCHK(hipMalloc(&p, std::max<long>(n, 1) * sizeof(float)));
        owned.push_back(p);
        return p;
    }
    hipEvent_t ev() {
        if (!evpool.empty()) {
            hipEvent_t e = evpool.back();
            evpool.pop_back();
            return e;
        }
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        return e;
    }
    double fam_bytes[NFAM] = {0};  // algorithmic HBM bytes of the timed launches (each operand touched once)
    template <typename Fn>
    void timed(int fam, Fn&& fn, double alg_bytes = 0.0) {
        if (!timing) {
            fn();
            return;
        }
        fam_bytes[fam] += alg_bytes;
        hipEvent_t a = ev(), b = ev();
        HIPCHK(hipEventRecord(a, st));
        fn();
        HIPCHK(hipEventRecord(b, st));
        pending.push_back({fam, {a, b}});
        pending_shape.push_back(fam == F_GEMM ? gemm_shape : std::string());
    }
    std::vector<std::string> pending_shape;  // per pending pair: the GEMM shape (census on), else empty
    std::string gemm_shape;
    void collect_timing() {
        for (size_t i = 0; i < pending.size(); ++i) {
            auto& pe = pending[i];
            float ms = 0.f;
            HIPCHK(hipEventSynchronize(pe.second.second));
            HIPCHK(hipEventElapsedTime(&ms, pe.second.first, pe.second.second));
            fam_ms[pe.first] += ms;
            fam_n[pe.first] += 1;
            if (i < pending_shape.size() && !pending_shape[i].empty()) gemm_census_time(pending_shape[i], ms);
            evpool.push_back(pe.second.first);
            evpool.push_back(pe.second.second);
        }
        pending.clear();
        pending_shape.clear();
    }
    // bf16 mode: bf16 planes of the frozen linear weights, {[N][K] for x W^T, [in][out] for dY W}, keyed by
    // the fp32 weight pointer (built once when the mode is selected), and the A plane of the current GEMM
    std::map<const float*, std::pair<void*, void*>> wplanes;
    DevBuf abuf;
    // two bf16 activation planes [B*T][<= max(3H, F)] (ping-pong): written by the producer of a linear's A
    // operand (LayerNorm, flash attention, GEMM epilogue), read by the linear right after
    DevBuf planebuf;
    bool use_planes() const { return gemm_mode == SUTA_PRECISION_BF16 && !wplanes.empty(); }
    // planes 0 / 1: the ping-pong A planes; plane 2: dctx's plane (the flash backward's dO operand)
    void* plane(int i) {
        if (!use_planes()) return nullptr;
        const size_t half = rup((long)plan.B * plan.T * std::max(3 * c.H, c.F) * 2, 256);
        if (planebuf.alloc(3 * half)) drop_graph();
        return reinterpret_cast<char*>(planebuf.p) + i * half;
    }
    // layer-mode conv stack on bf16 planes (bf16 mode): the conv LayerNorm forwards write bf16 activation planes
    // (ping-pong) that the next conv GEMM reads as its A operand, and the per-slot conv weights are re-laid
    // [C_out][tap * C_in] in bf16 (the B operand) at the start of every forward; SUTA_CONV_PLANES=0 keeps the
    // fp32-staged one-plane kernels
    DevBuf convact, convwt;
    bool conv_planes() const {
        if (!use_planes() || !c.layer_mode) return false;
        if (!suta_switches().conv_planes) return false;
        for (int i = 0; i < c.nconv; ++i)
            if (c.C[i] != 512 || (i > 0 && ((long)c.K[i] * c.C[i - 1] % 8 || (long)c.S[i] * c.C[i - 1] % 8))) return false;
        return true;
    }
    void* conv_act_plane(int i) {  // layer i < nconv - 1: [B][L_i][C_i] bf16, kept for the weight gradients
        size_t off = 0, tot = 0;
        for (int j = 0; j + 1 < c.nconv; ++j) {
            const size_t n = rup((long)plan.B * plan.Lc[j] * c.C[j] * 2, 256);
            if (j < i) off += n;
            tot += n;
        }
        if (convact.alloc(tot)) drop_graph();
        return reinterpret_cast<char*>(convact.p) + off;
    }
    DevBuf convdz;
    // bf16 plane of the current conv layer's dz (the weight gradient's B operand)
    void* conv_dz_plane() {
        size_t n = 0;
        for (int j = 1; j < c.nconv; ++j) n = std::max(n, (size_t)rup((long)plan.B * plan.Lc[j] * c.C[j] * 2, 256));
        if (convdz.alloc(n)) drop_graph();
        return convdz.p;
    }
    // layer i >= 1, native = 0: [B][C_i][K_i * C_{i-1}] bf16 (forward B operand); native = 1: the source layout
    // [B][K_i][C_{i-1}][C_i] (the input gradient's per-tap B segments)
    void* conv_wt_plane(int i, int native = 0) {
        size_t off = 0, tot = 0;
        for (int j = 1; j < c.nconv; ++j) {
            const size_t n = rup((long)plan.B * c.C[j] * c.K[j] * c.C[j - 1] * 2, 256);
            if (j < i) off += n;
            tot += n;
        }
        if (convwt.alloc(2 * tot)) drop_graph();
        return reinterpret_cast<char*>(convwt.p) + native * tot + off;
    }
    // with bf16 planes, fp32 activations read only as a frozen linear's A operand are not written (the linear
    // reads the plane; no weight gradient reads them): stable-LN outputs, gelu(FFN1), dU.  Only where every
    // producer and consumer takes its plane path (the vectorised LayerNorm widths, K % 8 == 0).  One predicate
    // for the forward and the backward.
    bool fp32_acts_dead() const {
        return use_planes() && (c.H == 512 || c.H == 768 || c.H == 1024) && c.F % 8 == 0;
    }
    // bf16 mode with planes: the FFN pre-activation u (stored by FFN1, read by the FFN2 input gradient's gelu')
    // kept in bf16 (SUTA_PRE_BF16=0: fp32, for A/B runs)
    bool pre_bf16() const {
        return use_planes() && suta_switches().pre_bf16;
    }
    // layer-mode conv stack on bf16 planes: the conv outputs z_i (conv0's by conv0_vec, the others by the conv GEMMs'
    // epilogues) and the activation gradients da_i (the conv input-gradient GEMMs) stored in bf16 only, in place in
    // their fp32 buffers; the conv LayerNorms read them widened -- torch autocast's bf16 conv outputs and gradients,
    // about half the conv stack's LayerNorm bytes (SUTA_CONV_Z_BF16=0: fp32 storage, for A/B runs)
    bool conv_z_bf16() const {
        if (!conv_planes() || !conv_dx_planes() || !fused_conv_ln() || c.K[0] != 10 || c.S[0] != 5) return false;
        return suta_switches().conv_z_bf16 != 0;
    }
    // stable-LN layers: the input gradients of QKV and FFN1 (the dy of LN1 / LN2 backward) written by their GEMMs as a
    // bf16 plane only (plane 2) and read so by the LayerNorm backward -- torch autocast's bf16 matmul gradient; 104 MB
    // less written and read per LayerNorm backward on C4 (SUTA_DY_PLANES=0: fp32 dy, for A/B runs)
    bool dy_planes() const {
        return fp32_acts_dead() && c.stable && suta_switches().dy_planes;
    }
    // conv input gradients on the bf16 planes too (SUTA_CONV_DX_PLANES=0: fp32-staged x6 kernels, for A/B runs)
    bool conv_dx_planes() const {
        return conv_planes() && suta_switches().conv_dx_planes;
    }
    // bf16 plane of layer l's qkv [B*T][3H]: written by the QKV GEMM, read by the flash forward and, in the
    // backward, by the flash backward (kept for every layer, like the fp32 qkv)
    DevBuf qkvplanes;
    void* qkv_plane(int l) {
        if (!use_planes() || c.H % 8) return nullptr;
        const size_t per = rup((long)plan.B * plan.T * 3 * c.H * 2, 256);
        if (qkvplanes.alloc(per * c.L)) drop_graph();
        return reinterpret_cast<char*>(qkvplanes.p) + l * per;
    }
    void build_weight_planes();
    // whether gemm(p0) takes the 256 x 256 bf16-plane kernel's C^T epilogue (the producer's A plane given, B a frozen
    // weight with planes): the condition for fusing EPI_DELTA into it
    bool routes_to_hbx_t(const GemmParams& p0) {
        if (gemm_mode != SUTA_PRECISION_BF16 || !p0.Ab || p0.segK != 0 || p0.ta || p0.Z != 1 || p0.K % 8) return false;
        auto it = wplanes.find(p0.B);
        if (it == wplanes.end() || !(p0.tb ? p0.ldb == p0.K : p0.ldb == p0.N)) return false;
        GemmParams p = p0;
        p.mode = gemm_mode;
        p.Bb = p.tb ? it->second.first : it->second.second;
        p.ldbb = p.K;
        return gemm_hbx_t_selected(p);
    }
    void gemm(const GemmParams& p0) {
        GemmParams p = p0;
        p.mode = gemm_mode;
        gemm_shape.clear();
        if (timing && gemm_census_is_on()) {  // per-shape time table (census + timing: tools/gemm_shapes.py)
            char key[200];
            snprintf(key, sizeof key, "M=%d N=%d K=%d z=%d %s%s epi=%d%s%s%s%s", p.M, p.N, p.K, p.Z, p.ta ? "T" : "N",
                     p.tb ? "T" : "N", p.epi, p.segK > 0 ? " conv" : "", p.Ab ? " Ab" : "", p.C ? " C" : "",
                     p.Cb ? " Cb" : "");
            gemm_shape = key;
        }
        if (gemm_mode == SUTA_PRECISION_BF16 && p.Ab && p.Bb) {  // both planes given by the caller (conv stack)
            timed(F_GEMM, [&] { gemm_launch(p, st, plan.splitws, plan.splitws_floats); }, timing ? gemm_alg_bytes(p) : 0.0);
            return;
        }
        if (gemm_mode == SUTA_PRECISION_BF16 && p.segK == 0 && !p.ta && p.Z == 1 && p.K % 8 == 0 && p.lda % 4 == 0 &&
            (reinterpret_cast<uintptr_t>(p.A) & 15) == 0) {
            auto it = wplanes.find(p.B);
            const bool fits = it != wplanes.end() && (p.tb ? p.ldb == p.K : p.ldb == p.N);
            if (fits) {  // linear with a frozen weight: the bf16-plane GEMM
                p.Bb = p.tb ? it->second.first : it->second.second;
                p.ldbb = p.K;
                if (p.Ab) {  // the producer of A wrote its bf16 plane
                    timed(F_GEMM, [&] { gemm_launch(p, st, plan.splitws, plan.splitws_floats); },
                          timing ? gemm_alg_bytes(p) : 0.0);
                    return;
                }
                if (!p.A) throw SutaError(SUTA_ERR_UNSUPPORTED, "gemm: neither an fp32 A nor its bf16 plane");
                if (abuf.alloc((size_t)p.M * p.K * 2 + 256)) drop_graph();
                p.Ab = abuf.p;
                p.ldab = p.K;
                timed(F_GEMM, [&] {
                    launch_to_bf16(p.A, p.lda, p.M, p.K, abuf.p, st);
                    gemm_launch(p, st, plan.splitws, plan.splitws_floats);
                }, timing ? gemm_alg_bytes(p, true) : 0.0);
                return;
            }
        }
        if (!p.C) throw SutaError(SUTA_ERR_UNSUPPORTED, "gemm: fp32 output skipped on a plane-less GEMM");
        if (!p.A) throw SutaError(SUTA_ERR_UNSUPPORTED, "gemm: fp32 A not written (bf16-plane producer) on a plane-less GEMM");
        if (p.Cb) throw SutaError(SUTA_ERR_UNSUPPORTED, "gemm: a bf16 C plane (read by the next kernel) requested on a plane-less GEMM");
        p.Ab = nullptr;  // (plane-less GEMM: a plane given for a non-frozen B is ignored)
        p.Cb = nullptr;
        timed(F_GEMM, [&] { gemm_launch(p, st, plan.splitws, plan.splitws_floats); }, timing ? gemm_alg_bytes(p) : 0.0);
    }

    int multiplicity(const TP& t, int train_feature, int bias_only) const {
        int k = 0;
        if (t.ln_member && (!bias_only || t.is_bias)) k += 1;
        if (train_feature) k += t.feat_depth;
        return k;
    }

    void build_plan(int B, long N);
    void set_lengths(int B, const int64_t* ns);
    const int* rN() const { return plan.ragged ? plan.len_n : nullptr; }
    const int* rL0() const { return plan.ragged ? plan.len_L0 : nullptr; }
    const int* rT() const { return plan.ragged ? plan.len_T : nullptr; }
    void forward(int B);
    void backward(int B, const suta_hparams& hp);
    void adam(int B, const suta_hparams& hp);
    void reset_slots(int B, bool zero_moments);
    void stage_input(const float* wav, int on_dev, int norm, int B, long N, long stride = 0);
};

suta_engine::~suta_engine() {
    if (loop_graph) (void)hipGraphExecDestroy(loop_graph);
    if (d_adam_tab) (void)hipFree(d_adam_tab);
    for (float* p : owned) (void)hipFree(p);
    for (auto& pe : pending) {
        (void)hipEventDestroy(pe.second.first);
        (void)hipEventDestroy(pe.second.second);
    }
    for (auto e : evpool) (void)hipEventDestroy(e);
    if (st) (void)hipStreamDestroy(st);
}

// ----------------------------------------------------------------------------------------------
// workspace plan
// ----------------------------------------------------------------------------------------------
void suta_engine::build_plan(int B, long N) {
    if (plan.B == B && plan.N == N) return;
    drop_graph();
    const Cfg& k = c;
    Plan pl;
    pl.B = B;
    pl.N = N;
    long L = N;
    for (int i = 0; i < k.nconv; ++i) {
        // (a conv input shorter than its kernel has no output frame: torch's Conv1d raises; C division would
        // round (L - K) / S toward zero and report one frame)
        if (L < k.K[i]) throw SutaError(SUTA_ERR_ARG, "utterance too short for the conv feature encoder");
        L = (L - k.K[i]) / k.S[i] + 1;
        pl.Lc[i] = (int)L;
    }
    pl.T = pl.Lc[k.nconv - 1];
    pl.Tp = (int)rup(pl.T, 4);
    if (pl.T > 2048) throw SutaError(SUTA_ERR_UNSUPPORTED, "T > 2048 frames (max 600000 samples in the reference)");
    const long T = pl.T, H = k.H, BT = (long)B * T;
    long maxLC = 0;
    for (int i = 0; i < k.nconv; ++i) maxLC = std::max(maxLC, (long)pl.Lc[i] * k.C[i]);
    for (int pass = 0; pass < 2; ++pass) {
        Arena ar;
        ar.dry = pass == 0;
        ar.base = reinterpret_cast<char*>(ws.p);
        pl.xraw = ar.take<float>((size_t)B * N);
        pl.x = ar.take<float>((size_t)B * N);
        for (int i = 0; i < k.nconv; ++i) {
            const long n = (long)B * pl.Lc[i] * k.C[i];
            pl.z[i] = (i == 0 && !k.layer_mode) ? nullptr : ar.take<float>(n);  // group-mode conv0 is recomputed
            pl.a[i] = ar.take<float>(n);
            pl.cxhat[i] = nullptr;
            if (k.layer_mode) {
                pl.crstd[i] = ar.take<float>((size_t)B * pl.Lc[i]);
                pl.cmean[i] = ar.take<float>((size_t)B * pl.Lc[i]);
            } else {
                pl.crstd[i] = pl.cmean[i] = nullptr;
            }
        }
        pl.gn_mean = ar.take<float>((size_t)B * k.C[0]);
        pl.gn_rstd = ar.take<float>((size_t)B * k.C[0]);
        const long C6 = k.C[k.nconv - 1];
        pl.fp_xhat = nullptr;
        pl.fp_mean = ar.take<float>(BT);
        pl.fp_rstd = ar.take<float>(BT);
        pl.fp_y = ar.take<float>(BT * C6);
        pl.h0 = ar.take<float>(BT * H);
        pl.pz = ar.take<float>(BT * H);
        pl.e = ar.take<float>(BT * H);
        pl.enc_xhat = nullptr;
        pl.enc_mean = ar.take<float>(BT);
        pl.enc_rstd = ar.take<float>(BT);
        pl.enc_y = ar.take<float>(BT * H);
        pl.lay.assign(k.L, LayerBufs{});
        pl.flash = attn_fused && k.H / k.NH == 64;
        const long Psz = pl.flash ? 0 : (long)B * k.NH * T * pl.Tp;
        for (int l = 0; l < k.L; ++l) {
            LayerBufs& lb = pl.lay[l];
            lb.xhat1 = k.stable ? nullptr : ar.take<float>(BT * H);
            lb.mean1 = k.stable ? ar.take<float>(BT) : nullptr;
            lb.rstd1 = ar.take<float>(BT);
            lb.y1 = ar.take<float>(BT * H);
            lb.qkv = ar.take<float>(BT * 3 * H);
            lb.P = pl.flash ? nullptr : ar.take<float>(Psz);
            lb.lse = pl.flash ? ar.take<float>((size_t)B * k.NH * T) : nullptr;
            lb.ctx = ar.take<float>(BT * H);
            lb.hmid = k.stable ? ar.take<float>(BT * H) : nullptr;
            lb.xhat2 = k.stable ? nullptr : ar.take<float>(BT * H);
            lb.mean2 = k.stable ? ar.take<float>(BT) : nullptr;
            lb.rstd2 = ar.take<float>(BT);
            lb.y2 = k.stable ? ar.take<float>(BT * H) : nullptr;
            lb.u = ar.take<float>(BT * k.F);
            lb.x_out = ar.take<float>(BT * H);
        }
        for (int l = 0; l < k.L; ++l) {
            pl.lay[l].x_in = l == 0 ? (k.stable ? pl.e : pl.enc_y) : pl.lay[l - 1].x_out;
            if (!k.stable) pl.lay[l].y2 = pl.lay[l].x_out;
        }
        pl.ctx = ar.take<float>(BT * H);
        pl.gu = ar.take<float>(BT * k.F);
        pl.rtmp = ar.take<float>(BT * H);
        pl.logits = ar.take<float>(BT * k.V);
        pl.dlogits = ar.take<float>(BT * k.V);
        pl.d1 = ar.take<float>(BT * H);
        pl.d2 = ar.take<float>(BT * H);
        pl.d3 = ar.take<float>(BT * H);
        pl.dqkv = ar.take<float>(BT * 3 * H);
        pl.dP = pl.flash ? nullptr : ar.take<float>(Psz);
        pl.dqp = pl.flash ? ar.take<float>(flash_dq_scratch_floats(B, pl.T, k.NH)) : nullptr;
        pl.delta = ar.take<float>((size_t)B * k.NH * T);
        pl.du = ar.take<float>(BT * k.F);
        pl.dzc = ar.take<float>((size_t)B * maxLC);
        pl.dzc2 = ar.take<float>((size_t)B * maxLC);
        const long lnrows = std::max<long>(pl.Lc[0], T);
        pl.lnpart_floats = (long)B * ((lnrows + 15) / 16) * 2 * std::max<long>(H, maxLC / pl.Lc[0] + 1) + 64;
        if (k.layer_mode && k.C[0] == 512)  // the fused conv LayerNorm backwards' partial slabs (short inputs too)
            for (int i = 0; i < k.nconv; ++i)
                pl.lnpart_floats = std::max(pl.lnpart_floats,
                                            layernorm_bwd_conv_part_floats(B, pl.Lc[i], k.C[i], i == 0 ? 10 : 0));
        pl.lnpart = ar.take<float>((size_t)pl.lnpart_floats);
        pl.dpart = ar.take<double>((size_t)B * ((pl.Lc[0] + 127) / 128 + 2) * 2 * k.C[0] + (size_t)B * k.C[0] * 2);
        pl.c0part = ar.take<float>((size_t)B * ((pl.Lc[0] + 127) / 128) * k.K[0] * k.C[0] + 64);
        pl.loss = ar.take<float>(B);
        pl.loss_scratch = ar.take<float>((size_t)B * T * 66 + 64);
        pl.ids = ar.take<int>((size_t)BT);
        pl.len_n = ar.take<int>((size_t)B);
        pl.len_L0 = ar.take<int>((size_t)B);
        pl.len_T = ar.take<int>((size_t)B);
        pl.splitws_floats = 32L << 20;
        pl.splitws = ar.take<float>(pl.splitws_floats);
        pl.bytes = ar.off;
        // a fresh workspace starts zeroed (on the engine stream, ordered before any use): the padding
        // frames of ragged batches must hold finite values
        if (pass == 0 && ws.alloc(ar.off + 256)) HIPCHK(hipMemsetAsync(ws.p, 0, ws.bytes, st));
    }
    plan = pl;
}

// Per-utterance lengths of a ragged batch (null: every utterance has the layout length plan.N).
void suta_engine::set_lengths(int B, const int64_t* ns) {
    Plan& pl = plan;
    pl.ragged = false;
    pl.h_n.assign(B, (int)pl.N);
    pl.h_T.assign(B, pl.T);
    if (!ns) return;
    std::vector<int> l0(B);
    for (int b = 0; b < B; ++b) {
        if (ns[b] < 1 || ns[b] > pl.N) throw SutaError(SUTA_ERR_ARG, "n_samples[b] outside [1, layout length]");
        long L = ns[b];
        for (int i = 0; i < c.nconv; ++i) {
            if (L < c.K[i]) throw SutaError(SUTA_ERR_ARG, "utterance too short for the conv feature encoder");
            L = (L - c.K[i]) / c.S[i] + 1;
            if (i == 0) l0[b] = (int)L;
        }
        pl.h_n[b] = (int)ns[b];
        pl.h_T[b] = (int)L;
        if (ns[b] != pl.N) pl.ragged = true;
    }
    if (!pl.ragged) return;
    HIPCHK(hipMemcpyAsync(pl.len_n, pl.h_n.data(), B * sizeof(int), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(pl.len_L0, l0.data(), B * sizeof(int), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(pl.len_T, pl.h_T.data(), B * sizeof(int), hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));  // host vectors are pageable and reused
}

// ----------------------------------------------------------------------------------------------
// forward (saves everything the backward needs)
// ----------------------------------------------------------------------------------------------
void suta_engine::forward(int B) {
    const Cfg& k = c;
    Plan& pl = plan;
    const int T = pl.T, H = k.H, NH = k.NH, d = H / NH;
    const long BT = (long)B * T;
    if (!k.layer_mode) {
        // conv0 + GroupNorm + GELU, conv0 recomputed in each pass (never stored)
        timed(F_FRONT, [&] {
            launch_front_gn_fwd(pl.x, pl.N, P + o_cw[0], k.conv_bias ? P + o_cb[0] : nullptr, Pn, B, pl.Lc[0], k.C[0],
                                k.K[0], k.S[0], P + o_cg[0], P + o_cbeta[0], pl.gn_mean, pl.gn_rstd, pl.a[0],
                                pl.dpart, rL0(), st);
        }, 4.0 * B * ((double)pl.N + (double)pl.Lc[0] * k.C[0]));  // waveform read, activation written
    }
    const bool zbf = k.layer_mode && conv_z_bf16();  // z_i in bf16, in place in the fp32 buffers
    if (k.layer_mode) {
        timed(F_FRONT, [&] {
            launch_conv0(pl.x, pl.N, P + o_cw[0], k.conv_bias ? P + o_cb[0] : nullptr, Pn, pl.z[0], B, pl.Lc[0],
                         k.C[0], k.K[0], k.S[0], st, zbf ? pl.z[0] : nullptr);
        }, (zbf ? 2.0 : 4.0) * B * ((double)pl.N + (double)pl.Lc[0] * k.C[0]));
    }
    const bool cpl = conv_planes();
    if (k.layer_mode) {
        timed(F_NORM, [&] {
            // with conv planes only the bf16 activation is read (the next conv GEMM and its weight gradient)
            launch_layernorm_fwd(zbf ? nullptr : pl.z[0], P + o_cg[0], P + o_cbeta[0], Pn, pl.Lc[0],
                                 cpl ? nullptr : pl.a[0], pl.cxhat[0], pl.crstd[0], B * pl.Lc[0], k.C[0], 1e-5f, 1, st,
                                 cpl ? conv_act_plane(0) : nullptr, pl.cmean[0], zbf ? pl.z[0] : nullptr);
        });
    }
    for (int i = 1; i < k.nconv; ++i) {
        GemmParams g;
        gemm_init(g);
        g.A = pl.a[i - 1];
        g.lda = (long)k.S[i] * k.C[i - 1];
        g.M = pl.Lc[i];
        g.K = k.K[i] * k.C[i - 1];
        g.N = k.C[i];
        g.B = P + o_cw[i];
        g.ldb = k.C[i];
        g.Z = B;
        g.sA1 = (long)pl.Lc[i - 1] * k.C[i - 1];
        g.sB1 = Pn;
        g.sC1 = (long)pl.Lc[i] * k.C[i];
        if (cpl) {  // bf16 planes: activations written by the previous LayerNorm, weights re-laid per slot
            void* wt = conv_wt_plane(i);
            timed(F_EW, [&] {
                launch_transpose_bf16(P + o_cw[i], Pn, B, g.K, g.N, wt, st, conv_dx_planes() ? conv_wt_plane(i, 1) : nullptr);
            });
            g.Ab = conv_act_plane(i - 1);
            g.ldab = g.lda;
            g.Bb = wt;
            g.ldbb = g.K;
            g.sB1 = (long)g.N * g.K;
            // (g.sA1: the same element stride in the bf16 plane)
        }
        if (k.conv_bias) {
            g.epi |= EPI_BIAS;
            g.bias = P + o_cb[i];
            g.sBias1 = Pn;
        }
        if (!k.layer_mode) {
            g.C = pl.a[i];
            g.ldc = k.C[i];
            g.epi |= EPI_STORE_PRE | EPI_GELU;
            g.C2 = pl.z[i];
            g.ldc2 = k.C[i];
            g.sC21 = g.sC1;
            gemm(g);
        } else {
            g.C = zbf ? nullptr : pl.z[i];
            g.ldc = k.C[i];
            if (zbf) {  // bf16 z_i only (the LayerNorm forward and backward read it widened)
                g.Cb = pl.z[i];
                g.ldcb = k.C[i];
                g.sCb1 = (long)pl.Lc[i] * k.C[i];
            }
            gemm(g);
            timed(F_NORM, [&] {
                const bool pln = cpl && i + 1 < k.nconv;
                launch_layernorm_fwd(zbf ? nullptr : pl.z[i], P + o_cg[i], P + o_cbeta[i], Pn, pl.Lc[i],
                                     pln ? nullptr : pl.a[i], pl.cxhat[i], pl.crstd[i], B * pl.Lc[i], k.C[i], 1e-5f, 1, st,
                                     pln ? conv_act_plane(i) : nullptr, pl.cmean[i], zbf ? pl.z[i] : nullptr);
            });
        }
    }
    const int C6 = k.C[k.nconv - 1];
    const float* feat = pl.a[k.nconv - 1];
    timed(F_NORM, [&] {
        launch_layernorm_fwd(feat, P + o_fpg, P + o_fpb, Pn, T, pl.fp_y, pl.fp_xhat, pl.fp_rstd, (int)BT, C6, k.eps, 0,
                             st, nullptr, pl.fp_mean);
    });
    {  // projection (per-utterance trainable W, b)
        GemmParams g;
        gemm_init(g);
        g.A = pl.fp_y;
        g.lda = C6;
        g.B = P + o_pw;
        g.tb = 1;
        g.ldb = C6;
        g.C = pl.h0;
        g.ldc = H;
        g.M = T;
        g.N = H;
        g.K = C6;
        g.Z = B;
        g.sA1 = (long)T * C6;
        g.sB1 = Pn;
        g.sC1 = (long)T * H;
        g.epi = EPI_BIAS;
        g.bias = P + o_pb;
        g.sBias1 = Pn;
        gemm(g);
    }
    // dedicated kernel in exact fp32 mode for group widths 48 / 64 (timed with the MFMA contractions)
    const bool pc_ok = posconv_kernel && gemm_mode == SUTA_PRECISION_FP32_MFMA && (H / k.posG == 48 || H / k.posG == 64) &&
                       k.posK % 2 == 0;
    if (pc_ok)
        timed(F_GEMM, [&] {
            if (!launch_posconv(true, pl.h0, wpos_f, bpos, pl.h0, pl.e, pl.pz, B, T, H, k.posG, k.posK, k.posK / 2,
                                rT(), st))
                throw SutaError(SUTA_ERR_UNSUPPORTED, "positional conv shape");
        });
    // bf16 mode, group width 64 (config C4): posconv_bf16_kernel
    const bool pcb16 = posconv_kernel && gemm_mode == SUTA_PRECISION_BF16 && wpos_bf_f && k.posK % 4 == 0;
    if (pcb16)
        timed(F_GEMM, [&] {
            if (!launch_posconv_bf16(true, pl.h0, wpos_bf_f, bpos, pl.h0, pl.e, pl.pz, B, T, H, k.posG, k.posK,
                                     k.posK / 2, rT(), st))
                throw SutaError(SUTA_ERR_UNSUPPORTED, "positional conv shape");
        });
    if (!pc_ok && !pcb16) {  // positional conv: e = h0 + gelu(posconv(h0)); pz = pre-activation
        const int Cg = H / k.posG;
        GemmParams g;
        gemm_init(g);
        g.A = pl.h0;
        g.lda = H;
        g.segK = Cg;
        g.pad = k.posK / 2;
        g.Mvalid = T;
        g.zmvalid = rT();  // zero padding at each utterance's own end
        g.M = T;
        g.N = Cg;
        g.K = k.posK * Cg;
        g.Z = B * k.posG;
        g.zdiv = k.posG;
        g.sA0 = Cg;
        g.sA1 = (long)T * H;
        g.B = wpos_f;
        g.ldb = Cg;
        g.sB0 = (long)k.posK * Cg * Cg;
        g.C = pl.e;
        g.ldc = H;
        g.sC0 = Cg;
        g.sC1 = (long)T * H;
        g.epi = EPI_BIAS | EPI_STORE_PRE | EPI_GELU | EPI_RESID;
        g.bias = bpos;
        g.sBias0 = Cg;
        g.C2 = pl.pz;
        g.ldc2 = H;
        g.sC20 = Cg;
        g.sC21 = (long)T * H;
        g.R = pl.h0;
        g.ldr = H;
        g.sR0 = Cg;
        g.sR1 = (long)T * H;
        gemm(g);
    }
    if (!k.stable) {
        timed(F_NORM, [&] {
            launch_layernorm_fwd(pl.e, P + o_eg, P + o_eb, Pn, T, pl.enc_y, pl.enc_xhat, pl.enc_rstd, (int)BT, H,
                                 k.eps, 0, st, plane(0), pl.enc_mean);
        });
    }
    const float scale = 1.0f / std::sqrt((float)d);
    // bf16 mode: producers of the linears' A operands also write bf16 planes (P0 / P1, ping-pong)
    void* P0 = plane(0);
    void* P1 = plane(1);
    const bool dead = fp32_acts_dead();  // (P0 non-null exactly then)
    for (int l = 0; l < k.L; ++l) {
        LayerBufs& lb = pl.lay[l];
        const float* attn_in = lb.x_in;
        if (k.stable) {
            timed(F_NORM, [&] {
                launch_layernorm_fwd(lb.x_in, P + o_l1g[l], P + o_l1b[l], Pn, T, dead ? nullptr : lb.y1, lb.xhat1,
                                     lb.rstd1, (int)BT, H, k.eps, 0, st, P0, lb.mean1);
            });
            attn_in = dead ? nullptr : lb.y1;  // (dead: the QKV GEMM reads the LN1 plane only)
        }
        void* qkvp = pl.flash ? qkv_plane(l) : nullptr;
        // both flash kernels read qkv's bf16 plane only (the backward's dO plane is plane 2): no fp32 qkv
        const bool bf = gemm_mode == SUTA_PRECISION_BF16;
        const bool qkv_dead = qkvp && P0 && flash_fwd_reads_plane(bf, qkvp, H) && flash_bwd_reads_planes(bf, qkvp, plane(2), H);
        {  // fused QKV
            GemmParams g;
            gemm_init(g);
            g.A = attn_in;
            g.lda = H;
            g.Ab = P0;  // LN output plane (stable: LN1; post-LN: the previous LayerNorm)
            g.ldab = H;
            g.B = wqkv[l];
            g.tb = 1;
            g.ldb = H;
            g.C = qkv_dead ? nullptr : lb.qkv;
            g.ldc = 3 * H;
            g.M = (int)BT;
            g.N = 3 * H;
            g.K = H;
            g.epi = EPI_BIAS;
            g.bias = bqkv[l];
            if (qkvp) {  // bf16 plane of qkv: the flash kernels' operands
                g.Cb = qkvp;
                g.ldcb = 3 * H;
            }
            gemm(g);
        }
        // flash attention (head dim 64, any T): ctx and the per-row LSE, no T x T matrix
        const bool fused = pl.flash;
        if (fused)
            timed(F_ATTN, [&] {
                if (!launch_flash_fwd(qkv_dead ? nullptr : lb.qkv, lb.ctx, lb.lse, B, T, NH, H, d, scale, rT(),
                                      gemm_mode == SUTA_PRECISION_BF16, st, P0, qkvp))
                    throw SutaError(SUTA_ERR_UNSUPPORTED, "flash attention shape");
            }, (double)BT * ((qkv_dead || (bf && qkvp && flash_fwd_reads_plane(bf, qkvp, H)) ? 2.0 : 4.0) * 3.0 * H +
                            4.0 * H + (P0 && bf ? 2.0 * H : 0.0) + 4.0 * NH));  // Q, K, V read; ctx (+ plane), LSE written
        if (!fused) {
            {  // S = Q K^T * scale
                GemmParams g;
                gemm_init(g);
                g.A = lb.qkv;
                g.lda = 3 * H;
                g.B = lb.qkv + H;
                g.tb = 1;
                g.ldb = 3 * H;
                g.C = lb.P;
                g.ldc = pl.Tp;
                g.M = T;
                g.N = T;
                g.K = d;
                g.Z = B * NH;
                g.zdiv = NH;
                g.sA0 = d;
                g.sA1 = (long)T * 3 * H;
                g.sB0 = d;
                g.sB1 = (long)T * 3 * H;
                g.sC0 = (long)T * pl.Tp;
                g.sC1 = (long)NH * T * pl.Tp;
                g.alpha = scale;
                gemm(g);
            }
            timed(F_SOFTMAX, [&] { launch_softmax_rows(lb.P, (long)B * NH * T, T, pl.Tp, rT(), (long)NH * T, st); });
            {  // ctx = P V
                GemmParams g;
                gemm_init(g);
                g.A = lb.P;
                g.lda = pl.Tp;
                g.B = lb.qkv + 2 * H;
                g.ldb = 3 * H;
                g.C = lb.ctx;
                g.ldc = H;
                g.M = T;
                g.N = d;
                g.K = T;
                g.Z = B * NH;
                g.zdiv = NH;
                g.sA0 = (long)T * pl.Tp;
                g.sA1 = (long)NH * T * pl.Tp;
                g.sB0 = d;
                g.sB1 = (long)T * 3 * H;
                g.sC0 = d;
                g.sC1 = (long)T * H;
                gemm(g);
            }
        }
        {  // out projection + residual
            GemmParams g;
            gemm_init(g);
            g.A = lb.ctx;
            g.lda = H;
            if (fused) {
                g.Ab = P0;
                g.ldab = H;
            }
            g.B = wo[l];
            g.tb = 1;
            g.ldb = H;
            g.C = k.stable ? lb.hmid : pl.rtmp;
            g.ldc = H;
            g.M = (int)BT;
            g.N = H;
            g.K = H;
            g.epi = EPI_BIAS | EPI_RESID;
            g.bias = bo[l];
            g.R = lb.x_in;
            g.ldr = H;
            gemm(g);
        }
        const float* ffn_in;
        const float* ffn_res;
        float* ffn_out;
        if (k.stable) {
            timed(F_NORM, [&] {
                launch_layernorm_fwd(lb.hmid, P + o_l2g[l], P + o_l2b[l], Pn, T, dead ? nullptr : lb.y2, lb.xhat2,
                                     lb.rstd2, (int)BT, H, k.eps, 0, st, P0, lb.mean2);
            });
            ffn_in = dead ? nullptr : lb.y2;
            ffn_res = lb.hmid;
            ffn_out = lb.x_out;
        } else {
            timed(F_NORM, [&] {
                launch_layernorm_fwd(pl.rtmp, P + o_l1g[l], P + o_l1b[l], Pn, T, lb.y1, lb.xhat1, lb.rstd1, (int)BT, H,
                                     k.eps, 0, st, P0);
            });
            ffn_in = lb.y1;
            ffn_res = lb.y1;
            ffn_out = pl.rtmp;
        }
        {  // u = in W1^T + b1 (stored), gu = gelu(u)
            GemmParams g;
            gemm_init(g);
            g.A = ffn_in;
            g.lda = H;
            g.Ab = P0;
            g.ldab = H;
            g.Cb = P1;  // gelu(u) plane for FFN2
            g.ldcb = k.F;
            g.B = w1[l];
            g.tb = 1;
            g.ldb = H;
            g.C = dead ? nullptr : pl.gu;  // with planes FFN2 reads only the bf16 plane (no weight gradient)
            g.ldc = k.F;
            g.M = (int)BT;
            g.N = k.F;
            g.K = H;
            g.epi = EPI_BIAS | EPI_STORE_PRE | EPI_GELU;
            g.bias = b1[l];
            g.C2 = lb.u;  // (dead: bf16 elements, the first half of the fp32 buffer)
            g.ldc2 = k.F;
            g.preb = dead && pre_bf16();
            gemm(g);
        }
        {  // out = gu W2^T + b2 + residual
            GemmParams g;
            gemm_init(g);
            g.A = dead ? nullptr : pl.gu;
            g.lda = k.F;
            g.Ab = P1;
            g.ldab = k.F;
            g.B = w2[l];
            g.tb = 1;
            g.ldb = k.F;
            g.C = ffn_out;
            g.ldc = H;
            g.M = (int)BT;
            g.N = H;
            g.K = k.F;
            g.epi = EPI_BIAS | EPI_RESID;
            g.bias = b2[l];
            g.R = ffn_res;
            g.ldr = H;
            gemm(g);
        }
        if (!k.stable) {
            timed(F_NORM, [&] {
                launch_layernorm_fwd(pl.rtmp, P + o_l2g[l], P + o_l2b[l], Pn, T, lb.x_out, lb.xhat2, lb.rstd2, (int)BT,
                                     H, k.eps, 0, st, P0);
            });
        }
    }
    const float* hfin = pl.lay[k.L - 1].x_out;
    if (k.stable) {
        timed(F_NORM, [&] {
            launch_layernorm_fwd(hfin, P + o_eg, P + o_eb, Pn, T, dead ? nullptr : pl.enc_y, pl.enc_xhat, pl.enc_rstd,
                                 (int)BT, H, k.eps, 0, st, P0, pl.enc_mean);
        });
        hfin = dead ? nullptr : pl.enc_y;
    }
    {  // lm_head
        GemmParams g;
        gemm_init(g);
        g.A = hfin;
        g.lda = H;
        g.Ab = P0;  // final LayerNorm output plane (stable: enc LN; post-LN: the last layer's LN2)
        g.ldab = H;
        g.B = wlm;
        g.tb = 1;
        g.ldb = H;
        g.C = pl.logits;
        g.ldc = k.V;
        g.M = (int)BT;
        g.N = k.V;
        g.K = H;
        g.epi = EPI_BIAS;
        g.bias = blm;
        gemm(g);
    }
}

// ----------------------------------------------------------------------------------------------
// backward: grads of the trainable tensors into G[b] (fully overwritten for every k > 0 tensor)
// ----------------------------------------------------------------------------------------------
void suta_engine::backward(int B, const suta_hparams& hp) {
    const Cfg& k = c;
    Plan& pl = plan;
    const int T = pl.T, H = k.H, NH = k.NH, d = H / NH;
    const long BT = (long)B * T;
    const float scale = 1.0f / std::sqrt((float)d);
    LossHP lh{hp.temp, hp.em_coef, hp.div_coef, hp.reweight, hp.non_blank};
    timed(F_LOSS,
          [&] { launch_suta_loss(pl.logits, B, T, k.V, lh, rT(), pl.dlogits, pl.loss, pl.loss_scratch, st); });
    if (hp.pl_coef > 0.f) {  // SDPL: (1 - pl) * SUTA + pl * pseudo-label CTC (main_SDPL.py:143-209)
        if (k.V > 32) throw SutaError(SUTA_ERR_UNSUPPORTED, "SDPL objective needs vocab_size <= 32");
        const long per = sdpl_scratch_floats(T);
        // [error flag | 63 pad | B x per-utterance scratch]: the flag stays at a fixed offset
        if (sdpl_ws.alloc(((size_t)B * per + 64) * sizeof(float)))
            HIPCHK(hipMemsetAsync(sdpl_ws.p, 0, sdpl_ws.bytes, st));
        int* err = reinterpret_cast<int*>(sdpl_ws.p);
        timed(F_LOSS, [&] {
            launch_sdpl_loss(pl.logits, B, T, k.V, hp.pl_coef, rT(), pl.dlogits, pl.loss, sdpl_ws.p + 64, err, st);
        });
        sdpl_used = true;
        sdpl_err = err;
    }

    // Ab: bf16 plane of A written by its producer; Cb: bf16 plane of C for the next linear (bf16 mode)
    auto nn_gemm = [&](const float* A, int lda, const float* Bm, int ldb, float* C, int ldc, int M, int N, int K,
                       int epi, const float* R, int ldr, const float* aux, int ldaux, const void* Ab = nullptr,
                       void* Cb = nullptr, int preb = 0) {
        GemmParams g;
        gemm_init(g);
        g.preb = preb;
        g.A = A;
        g.lda = lda;
        g.Ab = Ab;
        g.ldab = K;
        g.Cb = Cb;
        g.ldcb = N;
        g.B = Bm;
        g.ldb = ldb;
        g.C = C;
        g.ldc = ldc;
        g.M = M;
        g.N = N;
        g.K = K;
        g.epi = epi;
        g.R = R;
        g.ldr = ldr;
        g.aux = aux;
        g.ldaux = ldaux;
        gemm(g);
    };
    void* P0 = plane(0);  // bf16 planes of the linears' A operands (ping-pong), null outside bf16 mode
    void* P1 = plane(1);
    // with bf16 planes (the forward's condition) dU = dH W2 * gelu'(u) is read only through its plane by the
    // FFN1 input-gradient GEMM (no weight gradient): its fp32 copy is not written
    const bool dead = fp32_acts_dead();
    float* du32 = dead ? nullptr : pl.du;
    // d hfin = dlogits @ Wlm
    nn_gemm(pl.dlogits, k.V, wlm, H, pl.d1, H, (int)BT, H, k.V, 0, nullptr, 0, nullptr, 0);
    float* dx = pl.d1;  // grad wrt current residual stream
    float* t1 = pl.d2;
    float* t2 = pl.d3;
    if (k.stable) {
        timed(F_NORM, [&] {
            launch_layernorm_bwd(dx, pl.enc_xhat, pl.enc_rstd, P + o_eg, P + o_eb, Pn, T, B, H, 0, nullptr, nullptr, t1,
                                 G + o_eg, G + o_eb, Pn, pl.lnpart, st, P0, pl.lay[k.L - 1].x_out, pl.enc_mean);
        });
        std::swap(dx, t1);
    }
    for (int l = k.L - 1; l >= 0; --l) {
        LayerBufs& lb = pl.lay[l];
        float* dhres;  // grad flowing into the attention-block output (residual point)
        if (!k.stable) {
            // dr2 = LN2 bwd(dx)
            timed(F_NORM, [&] {
                launch_layernorm_bwd(dx, lb.xhat2, lb.rstd2, P + o_l2g[l], P + o_l2b[l], Pn, T, B, H, 0, nullptr,
                                     nullptr, t1, G + o_l2g[l], G + o_l2b[l], Pn, pl.lnpart, st, P0);
            });
            // du = (dr2 @ W2) * gelu'(u)
            nn_gemm(t1, H, w2[l], k.F, du32, k.F, (int)BT, k.F, H, EPI_DGELU, nullptr, 0, lb.u, k.F, P0, P1,
                    dead && pre_bf16());
            // dh1 = du @ W1 + dr2
            nn_gemm(du32, k.F, w1[l], H, t2, H, (int)BT, H, k.F, EPI_RESID, t1, H, nullptr, 0, P1);
            // dr1 = LN1 bwd(dh1)
            timed(F_NORM, [&] {
                launch_layernorm_bwd(t2, lb.xhat1, lb.rstd1, P + o_l1g[l], P + o_l1b[l], Pn, T, B, H, 0, nullptr,
                                     nullptr, t1, G + o_l1g[l], G + o_l1b[l], Pn, pl.lnpart, st, P0);
            });
            dhres = t1;  // dr1
        } else {
            // du = (dx @ W2) * gelu'(u); dy2 = du @ W1; dhmid = LN2 bwd(dy2) + dx
            nn_gemm(dx, H, w2[l], k.F, du32, k.F, (int)BT, k.F, H, EPI_DGELU, nullptr, 0, lb.u, k.F, P0, P1,
                    dead && pre_bf16());
            void* dyp = dy_planes() ? plane(2) : nullptr;  // (plane 2's dctx of the layer above is consumed)
            nn_gemm(du32, k.F, w1[l], H, dyp ? nullptr : t2, H, (int)BT, H, k.F, 0, nullptr, 0, nullptr, 0, P1, dyp);
            timed(F_NORM, [&] {
                launch_layernorm_bwd(dyp ? nullptr : t2, lb.xhat2, lb.rstd2, P + o_l2g[l], P + o_l2b[l], Pn, T, B, H, 0,
                                     nullptr, dx, t1, G + o_l2g[l], G + o_l2b[l], Pn, pl.lnpart, st, P0, lb.hmid,
                                     lb.mean2, dyp);
            });
            dhres = t1;  // dhmid
        }
        // dctx = dhres @ Wo
        void* dctxp = (pl.flash && P0) ? plane(2) : nullptr;   // dO plane of the flash backward
        void* qkvp = (pl.flash && P0) ? qkv_plane(l) : nullptr;
        if (!qkvp) dctxp = nullptr;
        // softmax-backward row term delta = rowsum(dctx * ctx) per head: in the dctx GEMM's epilogue when it takes the
        // C^T-epilogue kernel and the flash backward reads the dctx plane (the fp32 dctx is then not written), else a
        // separate pass over the fp32 dctx
        bool delta_fused = false;
        if (pl.flash && dctxp && d == 64 && suta_switches().fused_delta &&
            flash_bwd_reads_planes(gemm_mode == SUTA_PRECISION_BF16, qkvp, dctxp, H)) {
            GemmParams g;
            gemm_init(g);
            g.A = dhres;
            g.lda = H;
            g.Ab = P0;
            g.ldab = H;
            g.Cb = dctxp;
            g.ldcb = H;
            g.B = wo[l];
            g.ldb = H;
            g.C = nullptr;
            g.ldc = H;
            g.M = (int)BT;
            g.N = H;
            g.K = H;
            g.epi = EPI_DELTA;
            g.dlt_o = lb.ctx;
            g.ldo = H;
            g.delta = pl.delta;
            g.dT = T;
            g.dNH = NH;
            if (routes_to_hbx_t(g)) {
                gemm(g);
                delta_fused = true;
            }
        }
        if (!delta_fused) {
            nn_gemm(dhres, H, wo[l], H, pl.ctx, H, (int)BT, H, H, 0, nullptr, 0, nullptr, 0, P0, dctxp);
            timed(F_SOFTMAX, [&] { launch_attn_delta(pl.ctx, lb.ctx, pl.delta, B, T, NH, d, st); });
        }
        // flash backward: P recomputed from the LSE, dQ, dK, dV into dqkv (else the GEMM path below)
        const bool fused_bwd = pl.flash;
        // with bf16 planes the QKV input-gradient GEMM reads only dqkv's bf16 plane: the fp32 copy is not written
        const bool dqkv_dead = fused_bwd && P1 && dead;
        if (fused_bwd)
            timed(F_ATTN, [&] {
                // (the forward's test: the fp32 qkv was not written when both flash kernels read its plane)
                const bool bf = gemm_mode == SUTA_PRECISION_BF16;
                const bool qkv_dead = qkvp && flash_fwd_reads_plane(bf, qkvp, H) && flash_bwd_reads_planes(bf, qkvp, dctxp, H);
                if (!launch_flash_bwd(qkv_dead ? nullptr : lb.qkv, pl.ctx, lb.lse, pl.delta, dqkv_dead ? nullptr : pl.dqkv, pl.dqp, B, T,
                                      NH, H, d, scale, rT(), gemm_mode == SUTA_PRECISION_BF16, st, P1, qkvp, dctxp))
                    throw SutaError(SUTA_ERR_UNSUPPORTED, "flash attention shape");
            }, [&] {  // Q, K, V, dO, LSE, delta read; dQ, dK, dV written (fp32 and / or the bf16 plane)
                const bool bf = gemm_mode == SUTA_PRECISION_BF16;
                const bool planes = bf && qkvp && dctxp && flash_bwd_reads_planes(bf, qkvp, dctxp, H);
                return (double)BT * ((planes ? 2.0 : 4.0) * 4.0 * H + 4.0 * 2.0 * NH + (dqkv_dead ? 0.0 : 12.0 * H) +
                                     (P1 && bf ? 6.0 * H : 0.0));
            }());
        if (!fused_bwd) {
            {  // dS = scale * P * (dctx_h @ V_h^T - delta)
                GemmParams g;
                gemm_init(g);
                g.A = pl.ctx;
                g.lda = H;
                g.B = lb.qkv + 2 * H;
                g.tb = 1;
                g.ldb = 3 * H;
                g.C = pl.dP;
                g.ldc = pl.Tp;
                g.M = T;
                g.N = T;
                g.K = d;
                g.Z = B * NH;
                g.zdiv = NH;
                g.sA0 = d;
                g.sA1 = (long)T * H;
                g.sB0 = d;
                g.sB1 = (long)T * 3 * H;
                g.sC0 = (long)T * pl.Tp;
                g.sC1 = (long)NH * T * pl.Tp;
                g.epi = EPI_SMBWD;
                g.alpha = scale;
                g.aux = lb.P;
                g.ldaux = pl.Tp;
                g.sAux0 = (long)T * pl.Tp;
                g.sAux1 = (long)NH * T * pl.Tp;
                g.rowv = pl.delta;
                g.sRow0 = T;
                g.sRow1 = (long)NH * T;
                gemm(g);
            }
            {  // dQ = dS K_h
                GemmParams g;
                gemm_init(g);
                g.A = pl.dP;
                g.lda = pl.Tp;
                g.B = lb.qkv + H;
                g.ldb = 3 * H;
                g.C = pl.dqkv;
                g.ldc = 3 * H;
                g.M = T;
                g.N = d;
                g.K = T;
                g.Z = B * NH;
                g.zdiv = NH;
                g.sA0 = (long)T * pl.Tp;
                g.sA1 = (long)NH * T * pl.Tp;
                g.sB0 = d;
                g.sB1 = (long)T * 3 * H;
                g.sC0 = d;
                g.sC1 = (long)T * 3 * H;
                gemm(g);
            }
        }
        if (!fused_bwd) {  // dK = dS^T Q_h
            GemmParams g;
            gemm_init(g);
            g.A = pl.dP;
            g.ta = 1;
            g.lda = pl.Tp;
            g.B = lb.qkv;
            g.ldb = 3 * H;
            g.C = pl.dqkv + H;
            g.ldc = 3 * H;
            g.M = T;
            g.N = d;
            g.K = T;
            g.Z = B * NH;
            g.zdiv = NH;
            g.sA0 = (long)T * pl.Tp;
            g.sA1 = (long)NH * T * pl.Tp;
            g.sB0 = d;
            g.sB1 = (long)T * 3 * H;
            g.sC0 = d;
            g.sC1 = (long)T * 3 * H;
            gemm(g);
        }
        if (!fused_bwd) {  // dV = P^T dctx_h
            GemmParams g;
            gemm_init(g);
            g.A = lb.P;
            g.ta = 1;
            g.lda = pl.Tp;
            g.B = pl.ctx;
            g.ldb = H;
            g.C = pl.dqkv + 2 * H;
            g.ldc = 3 * H;
            g.M = T;
            g.N = d;
            g.K = T;
            g.Z = B * NH;
            g.zdiv = NH;
            g.sA0 = (long)T * pl.Tp;
            g.sA1 = (long)NH * T * pl.Tp;
            g.sB0 = d;
            g.sB1 = (long)T * H;
            g.sC0 = d;
            g.sC1 = (long)T * 3 * H;
            gemm(g);
        }
        if (!k.stable) {
            // dx_in = dqkv @ Wqkv + dr1
            nn_gemm(dqkv_dead ? nullptr : pl.dqkv, 3 * H, wqkv[l], H, t2, H, (int)BT, H, 3 * H, EPI_RESID, dhres, H,
                    nullptr, 0,
                    fused_bwd ? P1 : nullptr);
            std::swap(dx, t2);
        } else {
            // dy1 = dqkv @ Wqkv ; dx_in = LN1 bwd(dy1) + dhmid
            // (plane 2 held dctx, consumed by the flash backward above)
            void* dyp = (dy_planes() && fused_bwd && P1) ? plane(2) : nullptr;
            nn_gemm(dqkv_dead ? nullptr : pl.dqkv, 3 * H, wqkv[l], H, dyp ? nullptr : t2, H, (int)BT, H, 3 * H, 0, nullptr,
                    0, nullptr, 0, fused_bwd ? P1 : nullptr, dyp);
            timed(F_NORM, [&] {
                launch_layernorm_bwd(dyp ? nullptr : t2, lb.xhat1, lb.rstd1, P + o_l1g[l], P + o_l1b[l], Pn, T, B, H, 0,
                                     nullptr, dhres, dx, G + o_l1g[l], G + o_l1b[l], Pn, pl.lnpart, st, P0, lb.x_in,
                                     lb.mean1, dyp);
            });
            // dx now holds grad wrt x_in; t1/t2 free
        }
    }
    // encoder input
    float* de = dx;
    if (!k.stable) {
        timed(F_NORM, [&] {
            launch_layernorm_bwd(dx, pl.enc_xhat, pl.enc_rstd, P + o_eg, P + o_eb, Pn, T, B, H, 0, nullptr, nullptr, t1,
                                 G + o_eg, G + o_eb, Pn, pl.lnpart, st, nullptr, pl.e, pl.enc_mean);
        });
        de = t1;
    }
    float* dpz = (de == pl.d1) ? pl.d2 : (de == pl.d2 ? pl.d3 : pl.d1);
    float* dh0 = (dpz == pl.d1 || de == pl.d1) ? ((dpz == pl.d2 || de == pl.d2) ? pl.d3 : pl.d2) : pl.d1;
    timed(F_EW, [&] { launch_dgelu_mul(de, pl.pz, dpz, BT * H, st); });
    const bool pcb_ok = posconv_kernel && gemm_mode == SUTA_PRECISION_FP32_MFMA && (H / k.posG == 48 || H / k.posG == 64) &&
                        k.posK % 2 == 0;
    if (pcb_ok)
        timed(F_GEMM, [&] {
            if (!launch_posconv(false, dpz, wpos_b, nullptr, de, dh0, nullptr, B, T, H, k.posG, k.posK,
                                k.posK - 1 - k.posK / 2, rT(), st))
                throw SutaError(SUTA_ERR_UNSUPPORTED, "positional conv shape");
        });
    const bool pcb16 = posconv_kernel && gemm_mode == SUTA_PRECISION_BF16 && wpos_bf_b && k.posK % 4 == 0;
    if (pcb16)
        timed(F_GEMM, [&] {
            if (!launch_posconv_bf16(false, dpz, wpos_bf_b, nullptr, de, dh0, nullptr, B, T, H, k.posG, k.posK,
                                     k.posK - 1 - k.posK / 2, rT(), st))
                throw SutaError(SUTA_ERR_UNSUPPORTED, "positional conv shape");
        });
    if (!pcb_ok && !pcb16) {  // dh0 = posconv^T(dpz) + de
        const int Cg = H / k.posG;
        GemmParams g;
        gemm_init(g);
        g.A = dpz;
        g.lda = H;
        g.segK = Cg;
        g.pad = k.posK - 1 - k.posK / 2;
        g.Mvalid = T;
        g.zmvalid = rT();
        g.M = T;
        g.N = Cg;
        g.K = k.posK * Cg;
        g.Z = B * k.posG;
        g.zdiv = k.posG;
        g.sA0 = Cg;
        g.sA1 = (long)T * H;
        g.B = wpos_b;
        g.ldb = Cg;
        g.sB0 = (long)k.posK * Cg * Cg;
        g.C = dh0;
        g.ldc = H;
        g.sC0 = Cg;
        g.sC1 = (long)T * H;
        g.epi = EPI_RESID;
        g.R = de;
        g.ldr = H;
        g.sR0 = Cg;
        g.sR1 = (long)T * H;
        if (plan.ragged) {  // padding frames receive conv gradient from valid ones: keep them at 0
            g.epi |= EPI_ROWMASK;
            g.zrows = rT();
        }
        gemm(g);
    }
    const int C6 = k.C[k.nconv - 1];
    if (hp.train_feature) {
        {  // dWproj = dh0^T fp_y  (per utterance)
            GemmParams g;
            gemm_init(g);
            g.A = dh0;
            g.ta = 1;
            g.lda = H;
            g.B = pl.fp_y;
            g.ldb = C6;
            g.C = G + o_pw;
            g.ldc = C6;
            g.M = H;
            g.N = C6;
            g.K = T;
            g.Z = B;
            g.sA1 = (long)T * H;
            g.sB1 = (long)T * C6;
            g.sC1 = Pn;
            gemm(g);
        }
        timed(F_NORM, [&] { launch_colsum(dh0, B, T, H, G + o_pb, Pn, pl.lnpart, st); });
    }
    {  // d fp_y = dh0 @ Wproj  (per utterance W)
        GemmParams g;
        gemm_init(g);
        g.A = dh0;
        g.lda = H;
        g.B = P + o_pw;
        g.ldb = C6;
        g.C = pl.dzc;
        g.ldc = C6;
        g.M = T;
        g.N = C6;
        g.K = H;
        g.Z = B;
        g.sA1 = (long)T * H;
        g.sB1 = Pn;
        g.sC1 = (long)T * C6;
        gemm(g);
    }
    const int last = k.nconv - 1;
    // feature-projection LN bwd; in group mode also * gelu'(z_last) => dz_last
    float* cur = pl.dzc2;
    timed(F_NORM, [&] {
        launch_layernorm_bwd(pl.dzc, pl.fp_xhat, pl.fp_rstd, P + o_fpg, P + o_fpb, Pn, T, B, C6, 0,
                             (!k.layer_mode && hp.train_feature) ? pl.z[last] : nullptr, nullptr, cur, G + o_fpg,
                             G + o_fpb, Pn, pl.lnpart, st, nullptr, pl.a[last], pl.fp_mean);
    });
    if (!hp.train_feature) return;
    float* other = pl.dzc;
    // bf16 conv storage: z_i and (below the last layer) da_i are bf16 planes in place in their fp32 buffers
    const bool zbf = k.layer_mode && conv_z_bf16();
    for (int i = last; i >= 1; --i) {
        // cur: group mode -> dz_i ; layer mode -> da_i
        bool bias_done = false;
        const bool cpl = conv_planes();
        if (k.layer_mode) {
            timed(F_NORM, [&] {
                // fused: the LayerNorm backward also sums the conv bias gradient (one read of dz_i)
                const int bfin = zbf ? (2 | (i < last ? 1 : 0)) : 0;
                if (!pl.cxhat[i] && (fused_conv_ln() || cpl) &&
                    layernorm_bwd_conv_part_floats(B, pl.Lc[i], k.C[i], 0) <= pl.lnpart_floats &&
                    launch_layernorm_bwd_conv(cur, pl.crstd[i], P + o_cg[i], P + o_cbeta[i], Pn, pl.Lc[i], B, k.C[i],
                                              // both conv GEMMs read dz_i from its plane: no fp32 copy
                                              cpl && conv_dx_planes() ? nullptr : other, G + o_cg[i], G + o_cbeta[i],
                                              k.conv_bias ? G + o_cb[i] : nullptr,
                                              nullptr, Pn, pl.lnpart, st, pl.z[i], pl.cmean[i], nullptr, 0, 0, 0,
                                              cpl ? conv_dz_plane() : nullptr, bfin)) {
                    bias_done = true;
                } else if (zbf) {
                    throw SutaError(SUTA_ERR_UNSUPPORTED, "conv stack in bf16: the fused LayerNorm backward is required");
                } else {
                    launch_layernorm_bwd(cur, pl.cxhat[i], pl.crstd[i], P + o_cg[i], P + o_cbeta[i], Pn, pl.Lc[i], B,
                                         k.C[i], 1, nullptr, nullptr, other, G + o_cg[i], G + o_cbeta[i], Pn, pl.lnpart,
                                         st, nullptr, pl.z[i], pl.cmean[i]);
                }
            });
            std::swap(cur, other);
        }
        if (k.conv_bias && !bias_done)
            timed(F_NORM, [&] { launch_colsum(cur, B, pl.Lc[i], k.C[i], G + o_cb[i], Pn, pl.lnpart, st); });
        {  // dW_i = im2col(a_{i-1})^T dz_i
            GemmParams g;
            gemm_init(g);
            g.A = pl.a[i - 1];
            g.ta = 1;
            g.lda = (long)k.S[i] * k.C[i - 1];
            g.M = k.K[i] * k.C[i - 1];
            g.K = pl.Lc[i];
            g.B = cur;
            g.ldb = k.C[i];
            g.N = k.C[i];
            g.C = G + o_cw[i];
            g.ldc = k.C[i];
            g.Z = B;
            g.sA1 = (long)pl.Lc[i - 1] * k.C[i - 1];
            g.sB1 = (long)pl.Lc[i] * k.C[i];
            g.sC1 = Pn;
            if (cpl) {  // bf16 planes: the forward's activation plane and the LayerNorm-written dz plane (the fp32
                        // activation was not stored)
                if (!bias_done) throw SutaError(SUTA_ERR_UNSUPPORTED, "conv planes: dz plane not written");
                g.A = nullptr;
                g.Ab = conv_act_plane(i - 1);
                g.ldab = g.lda;
                g.Bb = conv_dz_plane();
                g.ldbb = g.ldb;
            }
            gemm(g);
        }
        {  // da_{i-1} = conv_i^T(dz_i): one GEMM per output-row residue rho (rows S*m + rho), whose K
           // runs over the taps k = rho + S*j (segment seg = nj-1-j reads dz row m - j and weight tap k)
            const int S_ = k.S[i], Kt = k.K[i], Cin = k.C[i - 1], Cout = k.C[i];
            const int Lin = pl.Lc[i - 1], Lout = pl.Lc[i];
            const float* zprev = (!k.layer_mode && i - 1 >= 1) ? pl.z[i - 1] : nullptr;
            for (int rho = 0; rho < S_; ++rho) {
                const int Mrows = (Lin - rho + S_ - 1) / S_;
                const int nj = (Kt - rho + S_ - 1) / S_;
                if (Mrows <= 0) continue;
                if (nj <= 0) throw SutaError(SUTA_ERR_UNSUPPORTED, "conv stride > kernel");
                GemmParams g;
                gemm_init(g);
                g.A = cur;
                g.lda = Cout;
                g.segK = Cout;
                g.pad = nj - 1;
                g.Mvalid = Lout;
                g.M = Mrows;
                g.K = nj * Cout;
                g.N = Cin;
                g.B = P + o_cw[i] + (long)(rho + S_ * (nj - 1)) * Cin * Cout;
                g.tb = 1;
                g.ldb = Cout;
                g.segB = 1;
                g.sBseg = -(long)S_ * Cin * Cout;
                g.C = other + (long)rho * Cin;
                g.ldc = (long)S_ * Cin;
                g.Z = B;
                g.sA1 = (long)Lout * Cout;
                g.sB1 = Pn;
                g.sC1 = (long)Lin * Cin;
                if (zprev) {
                    g.epi = EPI_DGELU;
                    g.aux = zprev + (long)rho * Cin;
                    g.ldaux = (long)S_ * Cin;
                    g.sAux1 = (long)Lin * Cin;
                }
                if (cpl && conv_dx_planes()) {  // bf16 planes: the LayerNorm-written dz plane and the forward's
                                                // source-layout bf16 weights (strides in bf16 elements)
                    if (!bias_done) throw SutaError(SUTA_ERR_UNSUPPORTED, "conv planes: dz plane not written");
                    g.A = nullptr;
                    g.B = nullptr;
                    g.Ab = conv_dz_plane();
                    g.ldab = Cout;
                    g.Bb = static_cast<char*>(conv_wt_plane(i, 1)) + (long)(rho + S_ * (nj - 1)) * Cin * Cout * 2;
                    g.ldbb = Cout;
                    g.tb = 0;
                    g.sB1 = (long)Kt * Cin * Cout;
                    if (zbf) {  // da_{i-1} in bf16 only (the next LayerNorm backward reads it widened)
                        g.C = nullptr;
                        g.Cb = reinterpret_cast<__bf16*>(other) + (long)rho * Cin;
                        g.ldcb = (long)S_ * Cin;
                        g.sCb1 = (long)Lin * Cin;
                    }
                }
                gemm(g);
            }
        }
        std::swap(cur, other);
    }
    // conv0: cur = da0
    if (!k.layer_mode) {
        timed(F_FRONT, [&] {
            launch_front_gn_bwd(pl.x, pl.N, P + o_cw[0], k.conv_bias ? P + o_cb[0] : nullptr, Pn, B, pl.Lc[0], k.C[0],
                                k.K[0], k.S[0], P + o_cg[0], P + o_cbeta[0], pl.gn_mean, pl.gn_rstd, cur, G + o_cg[0],
                                G + o_cbeta[0], G + o_cw[0], Pn, pl.dpart, pl.c0part, rL0(), st);
        }, 4.0 * B * ((double)pl.N + (double)pl.Lc[0] * k.C[0]));  // waveform and activation gradient read
        return;
    }
    bool fused0 = false;
    timed(F_NORM, [&] {
        // fused: the LayerNorm backward also sums the conv0 bias and weight gradients (dz0 read once)
        if (!pl.cxhat[0] && (fused_conv_ln() || zbf) && k.K[0] == 10 &&
            layernorm_bwd_conv_part_floats(B, pl.Lc[0], k.C[0], 10) <= pl.lnpart_floats &&
            // dz0 itself is consumed in registers (conv0's bias and weight gradients): not stored
            launch_layernorm_bwd_conv(cur, pl.crstd[0], P + o_cg[0], P + o_cbeta[0], Pn, pl.Lc[0], B, k.C[0], nullptr,
                                      G + o_cg[0], G + o_cbeta[0], k.conv_bias ? G + o_cb[0] : nullptr, G + o_cw[0], Pn,
                                      pl.lnpart, st, pl.z[0], pl.cmean[0], pl.x, pl.N, k.S[0], 10, nullptr,
                                      zbf ? (2 | (last > 0 ? 1 : 0)) : 0)) {
            fused0 = true;
        } else if (zbf) {
            throw SutaError(SUTA_ERR_UNSUPPORTED, "conv stack in bf16: the fused conv0 LayerNorm backward is required");
        } else {
            launch_layernorm_bwd(cur, pl.cxhat[0], pl.crstd[0], P + o_cg[0], P + o_cbeta[0], Pn, pl.Lc[0], B, k.C[0], 1,
                                 nullptr, nullptr, other, G + o_cg[0], G + o_cbeta[0], Pn, pl.lnpart, st, nullptr,
                                 pl.z[0], pl.cmean[0]);
        }
    });
    if (fused0) return;
    if (k.conv_bias)
        timed(F_NORM, [&] { launch_colsum(other, B, pl.Lc[0], k.C[0], G + o_cb[0], Pn, pl.lnpart, st); });
    {  // dW0[k][c] = sum_t x[S0 t + k] dz0[t][c]
        GemmParams g;
        gemm_init(g);
        g.A = pl.x;
        g.ta = 1;
        g.lda = k.S[0];
        g.M = k.K[0];
        g.K = pl.Lc[0];
        g.B = other;
        g.ldb = k.C[0];
        g.N = k.C[0];
        g.C = G + o_cw[0];
        g.ldc = k.C[0];
        g.Z = B;
        g.sA1 = pl.N;
        g.sB1 = (long)pl.Lc[0] * k.C[0];
        g.sC1 = Pn;
        gemm(g);
    }
}

// The optimizer scalars a table row depends on (the rest of suta_hparams only shapes the loss)
static bool same_opt_scalars(const suta_hparams& a, const suta_hparams& b) {
    return a.lr == b.lr && a.beta1 == b.beta1 && a.beta2 == b.beta2 && a.weight_decay == b.weight_decay &&
           a.optimizer == b.optimizer && a.lr_step_size == b.lr_step_size && a.lr_gamma == b.lr_gamma;
}

// lr of optimizer step i counted from the last reset: torch.optim.lr_scheduler.StepLR (main.py:20-21, step_size 1 and
// gamma 0.7 there) multiplies the group's lr by gamma, in double, each time its step count (advanced after every
// optimizer step, main.py:207-208) reaches a multiple of step_size (StepLR.get_lr, the chained form); the episodic
// reset restores it (main.py:147-152).  Carried as a running product over h_lr (rows are only ever appended while
// the scalars stay the same), so step i costs O(1) amortised and equals the chained loop bitwise.
double suta_engine::lr_at(const suta_hparams& hp, long i) {
    if (h_lr.empty() || !same_opt_scalars(hp, tab_hp)) {
        h_lr.clear();
        h_tab.clear();
        dev_rows = 0;
        tab_hp = hp;
        h_lr.push_back(py_double(hp.lr));
    }
    const double g = py_double(hp.lr_gamma);
    while ((long)h_lr.size() <= i) {
        const long e = (long)h_lr.size();
        const double prev = h_lr.back();
        h_lr.push_back(hp.lr_step_size > 0 && e % hp.lr_step_size == 0 ? prev * g : prev);
    }
    return h_lr[i];
}

static void check_optimizer(const suta_hparams& hp) {
    if (hp.optimizer != SUTA_OPT_ADAMW && hp.optimizer != SUTA_OPT_SGD)
        throw SutaError(SUTA_ERR_UNSUPPORTED, "optimizer: SUTA_OPT_ADAMW or SUTA_OPT_SGD");
    if (hp.lr_step_size < 0) throw SutaError(SUTA_ERR_ARG, "lr_step_size < 0");
}

void suta_engine::adam(int B, const suta_hparams& hp) {
    AdamArgs a{};
    check_optimizer(hp);
    // Python floats are doubles: recover the decimal the caller meant (0.9f -> 0.9) so the
    // scalars match torch's double-precision host arithmetic (adam.py:495-510)
    const double lr = lr_at(hp, opt_steps), b1 = py_double(hp.beta1), b2 = py_double(hp.beta2);
    a.beta1 = (float)b1;
    a.beta2 = (float)b2;
    a.omb1 = (float)(1.0 - b1);
    a.omb2 = (float)(1.0 - b2);
    a.eps = (float)py_double(hp.adam_eps);
    a.lr_wd = (float)(py_double(hp.lr) * py_double(hp.weight_decay));  // (a flag: the per-step factor is in the table)
    a.sgd = hp.optimizer == SUTA_OPT_SGD;
    // runs of equal multiplicity over the flat layout
    a.nruns = 0;
    int kmax = 0;
    for (const TP& t : tps) {
        const int m = multiplicity(t, hp.train_feature, hp.bias_only);
        kmax = std::max(kmax, m);
        if (m == 0) continue;
        if (a.nruns > 0 && a.runs[a.nruns - 1].k == m && a.runs[a.nruns - 1].start + a.runs[a.nruns - 1].len == t.off) {
            a.runs[a.nruns - 1].len += t.numel;
        } else {
            if (a.nruns >= SUTA_MAX_RUNS) throw SutaError(SUTA_ERR_UNSUPPORTED, "too many Adam runs");
            a.runs[a.nruns++] = AdamRun{t.off, t.numel, m};
        }
    }
    if (kmax > 5) throw SutaError(SUTA_ERR_UNSUPPORTED, "multiplicity > 5");
    for (int kk = 1; kk <= 5; ++kk)
        for (int j = 1; j <= kk; ++j) {
            const double t = (double)(opt_steps * kk + j);
            const double bc1 = 1.0 - std::pow(b1, t);
            const double bc2 = 1.0 - std::pow(b2, t);
            a.step_size[kk - 1][j - 1] = (float)(a.sgd ? lr : lr / bc1);
            a.bc2_sqrt[kk - 1][j - 1] = (float)std::sqrt(bc2);
        }
    a.tab = d_adam_tab;
    a.step = d_step;
    timed(F_ADAM, [&] {
        launch_adam(P, G, Mo, Vo, Pn, B, a, st);
        launch_step_advance(d_step, st);
    });
    opt_steps += 1;
}

// Device optimizer tables for steps [0, opt_steps + steps) and the device step counter = opt_steps.
void suta_engine::prepare_adam(const suta_hparams& hp, int steps) {
    check_optimizer(hp);
    const long need = opt_steps + std::max(steps, 1);
    (void)lr_at(hp, need - 1);  // (re)starts the host rows when the optimizer scalars changed
    if (need > adam_tab_cap) {
        const long cap = std::max<long>(need, 2 * adam_tab_cap);
        if (d_adam_tab) HIPCHK(hipFree(d_adam_tab));
        HIPCHK(hipMalloc(&d_adam_tab, cap * ADAM_TAB * sizeof(float)));
        adam_tab_cap = cap;
        dev_rows = 0;
        drop_graph();  // captured steps point at the old table
    }
    const double b1 = py_double(hp.beta1), b2 = py_double(hp.beta2), wd = py_double(hp.weight_decay);
    const long have = (long)(h_tab.size() / ADAM_TAB);
    if (need > have) h_tab.resize(need * ADAM_TAB, 0.f);
    for (long s0 = have; s0 < need; ++s0) {
        const double lr = h_lr[s0];
        float* row = h_tab.data() + s0 * ADAM_TAB;
        for (int kk = 1; kk <= 5; ++kk)
            for (int j = 1; j <= kk; ++j) {
                const double t = (double)(s0 * kk + j);
                row[(kk - 1) * 5 + (j - 1)] = (float)(lr / (1.0 - std::pow(b1, t)));
                row[25 + (kk - 1) * 5 + (j - 1)] = (float)std::sqrt(1.0 - std::pow(b2, t));
            }
        row[50] = (float)(1.0 - lr * wd);
        row[51] = (float)(-lr);
    }
    h_step = (int)opt_steps;
    if (need > dev_rows) {  // rows already on the device hold the same values: only the new ones go up
        HIPCHK(hipMemcpyAsync(d_adam_tab + dev_rows * ADAM_TAB, h_tab.data() + dev_rows * ADAM_TAB,
                              (need - dev_rows) * ADAM_TAB * sizeof(float), hipMemcpyHostToDevice, st));
        dev_rows = need;
    }
    HIPCHK(hipMemcpyAsync(d_step, &h_step, sizeof(int), hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));  // pageable sources
}

// The device work of one suta_adapt call after its input is staged: episodic slot reset (pristine
// tensors broadcast into the slots; the moments are implicit zeros at Adam step 0), the vanilla forward,
// then S x (backward, Adam, forward); at each recorded step the logits are copied and the greedy ids
// computed into device staging.  Ordered on the engine stream only, so it captures as one graph.
void suta_engine::adapt_loop(int B, const suta_hparams& hp, int steps, const int* rec, int nrec, float* rec_logits,
                             int* rec_ids) {
    const long rows = (long)B * plan.T;
    if (hp.episodic) launch_broadcast(P, P0, Pn, B, st);
    for (int s = 0; s <= steps; ++s) {
        if (s > 0) {
            backward(B, hp);
            adam(B, hp);
        }
        forward(B);
        for (int i = 0; i < nrec; ++i) {
            if (rec[i] != s) continue;
            if (rec_logits)
                HIPCHK(hipMemcpyAsync(rec_logits + i * rows * c.V, plan.logits, rows * c.V * sizeof(float),
                                      hipMemcpyDeviceToDevice, st));
            if (rec_ids) launch_argmax(plan.logits, rows, c.V, rec_ids + i * rows, st);
        }
    }
}

// With graphs on, per-kernel timing off and `graph_ok` (this call repeats the previous call's key: batch,
// layout, ragged, precision, hparams, steps, record set, outputs), the whole loop is captured once and
// replayed per call; a one-off key runs eagerly (no capture cost).  Replay == eager bitwise (GPU test).
void suta_engine::run_adapt_loop(int B, const suta_hparams& hp, int steps, const int* rec, int nrec,
                                 float* rec_logits, int* rec_ids, bool graph_ok) {
    if (!use_graphs || timing || !graph_ok) {
        adapt_loop(B, hp, steps, rec, nrec, rec_logits, rec_ids);
        last_loop_mode = SUTA_LOOP_EAGER;
        return;
    }
    last_loop_mode = loop_graph ? SUTA_LOOP_REPLAYED : SUTA_LOOP_CAPTURED;
    if (!loop_graph) {
        const long steps0 = opt_steps;
        hipGraph_t g = nullptr;
        HIPCHK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
        try {
            adapt_loop(B, hp, steps, rec, nrec, rec_logits, rec_ids);
        } catch (...) {
            (void)hipStreamEndCapture(st, &g);
            if (g) (void)hipGraphDestroy(g);
            opt_steps = steps0;
            throw;
        }
        HIPCHK(hipStreamEndCapture(st, &g));
        opt_steps = steps0;  // the capture recorded the Adam steps without running them
        HIPCHK(hipGraphInstantiate(&loop_graph, g, nullptr, nullptr, 0));
        HIPCHK(hipGraphDestroy(g));
        ++graph_captures;
    }
    HIPCHK(hipGraphLaunch(loop_graph, st));
    ++graph_launches;
    opt_steps += steps;
    if (hp.pl_coef > 0.f && steps > 0) sdpl_used = true;  // the replayed SDPL kernels may raise the error flag
}

// Key of this call; true when it equals the previous call's (graph capture pays off from the 2nd call)
bool suta_engine::graph_key_repeats(const GraphKey& k) {
    const bool same = gkey_seen && gkey.B == k.B && gkey.N == k.N && gkey.ragged == k.ragged &&
                      gkey.mode == k.mode && gkey.steps == k.steps && gkey.want_logits == k.want_logits &&
                      gkey.want_ids == k.want_ids && gkey.rec == k.rec &&
                      std::memcmp(&gkey.hp, &k.hp, sizeof(suta_hparams)) == 0 &&
                      std::memcmp(&gkey.sw, &k.sw, sizeof(SutaSwitches)) == 0;
    if (!same) {
        drop_graph();
        gkey = k;
        gkey_seen = true;
    }
    return same;
}

// bf16 planes of the frozen linear weights (RNE, as the bf16 GEMMs round every operand): W [N][K] for the
// forward x W^T and W^T [in][out] for the input gradient dY W, so both GEMMs read k-contiguous planes.
void suta_engine::build_weight_planes() {
    if (!wplanes.empty()) return;
    auto add = [&](const float* w, long rows, long cols) {  // w: [rows = out][cols = in]
        std::vector<float> hw((size_t)rows * cols);
        HIPCHK(hipMemcpy(hw.data(), w, hw.size() * 4, hipMemcpyDeviceToHost));
        std::vector<__bf16> a(hw.size()), t(hw.size());
        for (long r = 0; r < rows; ++r)
            for (long c2 = 0; c2 < cols; ++c2) {
                const __bf16 v = (__bf16)hw[(size_t)r * cols + c2];
                a[(size_t)r * cols + c2] = v;
                t[(size_t)c2 * rows + r] = v;
            }
        float* pa = dalloc((long)(a.size() + 1) / 2 + 4);
        float* pt = dalloc((long)(t.size() + 1) / 2 + 4);
        HIPCHK(hipMemcpy(pa, a.data(), a.size() * 2, hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(pt, t.data(), t.size() * 2, hipMemcpyHostToDevice));
        wplanes[w] = {pa, pt};
    };
    const long H = c.H, F = c.F;
    for (int l = 0; l < c.L; ++l) {
        add(wqkv[l], 3 * H, H);
        add(wo[l], H, H);
        add(w1[l], F, H);
        add(w2[l], H, F);
    }
    add(wlm, c.V, H);
}

// Pristine tensors into slots [0, B) and the Adam step counter to 0.  The moments need no clearing: the
// Adam kernel takes them as zero at step 0 (zero_moments only keeps unused slots deterministic).
void suta_engine::reset_slots(int B, bool zero_moments) {
    launch_broadcast(P, P0, Pn, B, st);
    if (zero_moments) {
        HIPCHK(hipMemsetAsync(Mo, 0, (size_t)B * Pn * sizeof(float), st));
        HIPCHK(hipMemsetAsync(Vo, 0, (size_t)B * Pn * sizeof(float), st));
    }
    opt_steps = 0;
    h_step = 0;
    HIPCHK(hipMemcpyAsync(d_step, &h_step, sizeof(int), hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
}

void suta_engine::stage_input(const float* wav, int on_dev, int norm, int B, long N, long stride) {
    const hipMemcpyKind kind = on_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (!plan.ragged) {
        HIPCHK(hipMemcpyAsync(plan.xraw, wav, (size_t)B * N * sizeof(float), kind, st));
    } else {  // utterance b: n[b] samples at wav + b * stride -> slot b of the N-stride layout, zero padded
        HIPCHK(hipMemsetAsync(plan.xraw, 0, (size_t)B * N * sizeof(float), st));
        for (int b = 0; b < B; ++b)
            HIPCHK(hipMemcpyAsync(plan.xraw + (long)b * N, wav + (long)b * stride, (size_t)plan.h_n[b] * sizeof(float),
                                  kind, st));
    }
    if (norm) timed(F_EW, [&] { launch_wave_normalize(plan.xraw, plan.x, B, N, rN(), st); });
    else HIPCHK(hipMemcpyAsync(plan.x, plan.xraw, (size_t)B * N * sizeof(float), hipMemcpyDeviceToDevice, st));
}

// ==============================================================================================
// C ABI
// ==============================================================================================
namespace {

template <typename Fn>
int32_t guard(Fn&& fn) {
    try {
        fn();
        return SUTA_OK;
    } catch (const SutaError& e) {
        g_err = e.what();
        return e.code;
    } catch (const std::exception& e) {
        g_err = e.what();
        return SUTA_ERR_ARG;
    }
}

Cfg make_cfg(const suta_model_config* m) {
    Cfg c{};
    c.H = m->hidden_size;
    c.L = m->num_hidden_layers;
    c.NH = m->num_attention_heads;
    c.F = m->intermediate_size;
    c.V = m->vocab_size;
    c.nconv = m->num_conv_layers;
    if (c.nconv < 2 || c.nconv > SUTA_MAX_CONV) throw SutaError(SUTA_ERR_ARG, "num_conv_layers out of range");
    for (int i = 0; i < c.nconv; ++i) {
        c.C[i] = m->conv_dim[i];
        c.K[i] = m->conv_kernel[i];
        c.S[i] = m->conv_stride[i];
        if (c.C[i] % 4 || c.C[i] <= 0) throw SutaError(SUTA_ERR_UNSUPPORTED, "conv_dim must be a multiple of 4");
    }
    if (c.K[0] > 16) throw SutaError(SUTA_ERR_UNSUPPORTED, "conv0 kernel > 16");
    c.conv_bias = m->conv_bias;
    c.layer_mode = m->feat_extract_norm_layer;
    c.stable = m->do_stable_layer_norm;
    c.posK = m->num_conv_pos_embeddings;
    c.posG = m->num_conv_pos_embedding_groups;
    c.eps = m->layer_norm_eps;
    if (c.H % c.NH || c.H % c.posG) throw SutaError(SUTA_ERR_ARG, "hidden_size not divisible by heads/groups");
    if ((c.H / c.posG) % 16) throw SutaError(SUTA_ERR_UNSUPPORTED, "pos-conv group width must be a multiple of 16");
    if (c.V > 64) throw SutaError(SUTA_ERR_UNSUPPORTED, "vocab_size > 64");
    if (c.H > 1024 || c.C[c.nconv - 1] > 1024) throw SutaError(SUTA_ERR_UNSUPPORTED, "hidden > 1024");
    return c;
}

}  // namespace

extern "C" {

const char* suta_last_error(void) { return g_err.c_str(); }

int32_t suta_num_frames(const suta_model_config* cfg, int64_t n, int64_t* out) {
    return guard([&] {
        long L = n;
        for (int i = 0; i < cfg->num_conv_layers; ++i)  // 0 frames once a layer's input is shorter than its kernel
            L = L < cfg->conv_kernel[i] ? 0 : (L - cfg->conv_kernel[i]) / cfg->conv_stride[i] + 1;
        *out = L;
    });
}

int32_t suta_create(const suta_model_config* cfg, const char* const* names, const float* const* data,
                    const int64_t* numels, int32_t n, int32_t device, int32_t max_batch, int64_t max_samples,
                    suta_engine** out) {
    return guard([&] {
        if (!cfg || !out || max_batch < 1) throw SutaError(SUTA_ERR_ARG, "null argument");
        std::unique_ptr<suta_engine> e(new suta_engine());
        e->c = make_cfg(cfg);
        const Cfg& c = e->c;
        e->device = device;
        e->max_batch = max_batch;
        e->max_samples = max_samples;
        if (const char* af = std::getenv("SUTA_ATTN_FUSED")) e->attn_fused = af[0] != '0';
        if (const char* pc = std::getenv("SUTA_POSCONV")) e->posconv_kernel = pc[0] != '0';
        if (const char* bp = std::getenv("SUTA_BF16_PLANES")) e->bf16_planes = bp[0] != '0';
        // SUTA_GRAPHS=0: no graph capture (as suta_set_graphs(e, 0)); profiling runs under rocprofv3 --pmc, which
        // crashes (SIGSEGV in a profiler thread) once a captured graph is launched -- the kernels are the same
        if (const char* gr = std::getenv("SUTA_GRAPHS")) e->use_graphs = gr[0] != '0';
        HIPCHK(hipSetDevice(device));
        HIPCHK(hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking));
        e->d_step = reinterpret_cast<int*>(e->dalloc(1));
        HIPCHK(hipMemset(e->d_step, 0, sizeof(int)));
        std::map<std::string, std::pair<const float*, long>> w;
        for (int i = 0; i < n; ++i) w[names[i]] = {data[i], numels[i]};
        auto get = [&](const std::string& nm, long numel) -> const float* {
            auto it = w.find(nm);
            if (it == w.end()) throw SutaError(SUTA_ERR_ARG, "missing weight " + nm);
            if (it->second.second != numel)
                throw SutaError(SUTA_ERR_ARG, "size mismatch for " + nm + ": got " + std::to_string(it->second.second) +
                                                  " expected " + std::to_string(numel));
            return it->second.first;
        };
        auto up = [&](const std::string& nm, long numel) {
            const float* h = get(nm, numel);
            float* dptr = e->dalloc(numel);
            HIPCHK(hipMemcpy(dptr, h, numel * sizeof(float), hipMemcpyHostToDevice));
            return dptr;
        };
        const std::string pfx = "wav2vec2.";
        const int H = c.H;
        // ---- trainable layout ----
        auto add = [&](const std::string& nm, std::vector<long> shape, bool conv_w, bool ln, bool bias, int depth) {
            TP t;
            t.name = nm;
            t.shape = shape;
            t.numel = 1;
            for (long s : shape) t.numel *= s;
            t.conv_w = conv_w;
            t.ln_member = ln;
            t.is_bias = bias;
            t.feat_depth = depth;
            t.off = rup(e->Pn, 4);
            e->Pn = t.off + t.numel;
            e->tpi[nm] = (int)e->tps.size();
            e->tps.push_back(t);
            return t.off;
        };
        for (int i = 0; i < c.nconv; ++i) {  // conv-layer norms first (layer mode: k = 5)
            const std::string b = pfx + "feature_extractor.conv_layers." + std::to_string(i) + ".layer_norm.";
            if (c.layer_mode) {
                e->o_cg[i] = add(b + "weight", {c.C[i]}, false, true, false, 4);
                e->o_cbeta[i] = add(b + "bias", {c.C[i]}, false, true, true, 4);
            } else if (i == 0) {
                e->o_cg[i] = add(b + "weight", {c.C[i]}, false, false, false, 4);
                e->o_cbeta[i] = add(b + "bias", {c.C[i]}, false, false, true, 4);
            } else {
                e->o_cg[i] = e->o_cbeta[i] = -1;
            }
        }
        for (int i = 0; i < c.nconv; ++i) {
            const std::string b = pfx + "feature_extractor.conv_layers." + std::to_string(i) + ".conv.";
            const long cin = i == 0 ? 1 : c.C[i - 1];
            e->o_cw[i] = add(b + "weight", {c.C[i], cin, c.K[i]}, true, false, false, 4);
            e->o_cb[i] = c.conv_bias ? add(b + "bias", {c.C[i]}, false, false, true, 4) : -1;
        }
        const int C6 = c.C[c.nconv - 1];
        e->o_fpg = add(pfx + "feature_projection.layer_norm.weight", {C6}, false, true, false, 2);
        e->o_fpb = add(pfx + "feature_projection.layer_norm.bias", {C6}, false, true, true, 2);
        e->o_pw = add(pfx + "feature_projection.projection.weight", {H, C6}, false, false, false, 2);
        e->o_pb = add(pfx + "feature_projection.projection.bias", {H}, false, false, true, 2);
        e->o_eg = add(pfx + "encoder.layer_norm.weight", {H}, false, true, false, 0);
        e->o_eb = add(pfx + "encoder.layer_norm.bias", {H}, false, true, true, 0);
        for (int l = 0; l < c.L; ++l) {
            const std::string b = pfx + "encoder.layers." + std::to_string(l) + ".";
            e->o_l1g.push_back(add(b + "layer_norm.weight", {H}, false, true, false, 0));
            e->o_l1b.push_back(add(b + "layer_norm.bias", {H}, false, true, true, 0));
            e->o_l2g.push_back(add(b + "final_layer_norm.weight", {H}, false, true, false, 0));
            e->o_l2b.push_back(add(b + "final_layer_norm.bias", {H}, false, true, true, 0));
        }
        e->Pn = rup(e->Pn, 64);
        std::vector<float> hp0(e->Pn, 0.f);
        for (const TP& t : e->tps) {
            const float* src = get(t.name, t.numel);
            if (t.conv_w) {  // [co][ci][k] -> [k][ci][co]
                const long co = t.shape[0], ci = t.shape[1], kk = t.shape[2];
                for (long o = 0; o < co; ++o)
                    for (long i2 = 0; i2 < ci; ++i2)
                        for (long q = 0; q < kk; ++q) hp0[t.off + (q * ci + i2) * co + o] = src[(o * ci + i2) * kk + q];
            } else {
                std::memcpy(&hp0[t.off], src, t.numel * sizeof(float));
            }
        }
        e->P0 = e->dalloc(e->Pn);
        HIPCHK(hipMemcpy(e->P0, hp0.data(), e->Pn * sizeof(float), hipMemcpyHostToDevice));
        e->P = e->dalloc((long)max_batch * e->Pn);
        e->G = e->dalloc((long)max_batch * e->Pn);
        e->Mo = e->dalloc((long)max_batch * e->Pn);
        e->Vo = e->dalloc((long)max_batch * e->Pn);
        HIPCHK(hipMemset(e->G, 0, (size_t)max_batch * e->Pn * sizeof(float)));
        // ---- frozen encoder weights ----
        for (int l = 0; l < c.L; ++l) {
            const std::string b = pfx + "encoder.layers." + std::to_string(l) + ".";
            std::vector<float> qkv((size_t)3 * H * H), bq((size_t)3 * H);
            const char* parts[3] = {"q_proj", "k_proj", "v_proj"};
            for (int j = 0; j < 3; ++j) {
                std::memcpy(&qkv[(size_t)j * H * H], get(b + "attention." + parts[j] + ".weight", (long)H * H),
                            sizeof(float) * H * H);
                std::memcpy(&bq[(size_t)j * H], get(b + "attention." + parts[j] + ".bias", H), sizeof(float) * H);
            }
            float* dq = e->dalloc(3L * H * H);
            HIPCHK(hipMemcpy(dq, qkv.data(), qkv.size() * 4, hipMemcpyHostToDevice));
            float* dbq = e->dalloc(3L * H);
            HIPCHK(hipMemcpy(dbq, bq.data(), bq.size() * 4, hipMemcpyHostToDevice));
            e->wqkv.push_back(dq);
            e->bqkv.push_back(dbq);
            e->wo.push_back(up(b + "attention.out_proj.weight", (long)H * H));
            e->bo.push_back(up(b + "attention.out_proj.bias", H));
            e->w1.push_back(up(b + "feed_forward.intermediate_dense.weight", (long)c.F * H));
            e->b1.push_back(up(b + "feed_forward.intermediate_dense.bias", c.F));
            e->w2.push_back(up(b + "feed_forward.output_dense.weight", (long)c.F * H));
            e->b2.push_back(up(b + "feed_forward.output_dense.bias", H));
        }
        e->wlm = up("lm_head.weight", (long)c.V * H);
        e->blm = up("lm_head.bias", c.V);
        // ---- positional conv: weight norm (dim=2) precomputed, regrouped for the conv-A GEMM ----
        {
            const int K = c.posK, G = c.posG, Cg = H / G;
            const std::string b = pfx + "encoder.pos_conv_embed.conv.";
            const float* g = get(b + "parametrizations.weight.original0", K);
            const float* v = get(b + "parametrizations.weight.original1", (long)H * Cg * K);
            std::vector<double> nrm(K, 0.0);
            for (long o = 0; o < H; ++o)
                for (long i2 = 0; i2 < Cg; ++i2)
                    for (int q = 0; q < K; ++q) {
                        const double x = v[(o * Cg + i2) * K + q];
                        nrm[q] += x * x;
                    }
            // ATen _weight_norm: w = v * (g / ||v||) in fp32
            std::vector<float> nf(K);
            for (int q = 0; q < K; ++q) nf[q] = (float)std::sqrt(nrm[q]);
            std::vector<float> wf((size_t)G * K * Cg * Cg), wb((size_t)G * K * Cg * Cg);
            const bool bfw = Cg == 64;  // bf16-mode kernel weights (group width 64)
            std::vector<uint16_t> bf_f(bfw ? wf.size() : 0), bf_b(bfw ? wf.size() : 0);
            auto rne = [](float f) {  // fp32 -> bf16 bits, round to nearest even (finite values), as (__bf16)f
                uint32_t u;
                std::memcpy(&u, &f, 4);
                return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
            };
            for (int gi = 0; gi < G; ++gi)
                for (int co = 0; co < Cg; ++co)
                    for (int ci = 0; ci < Cg; ++ci)
                        for (int q = 0; q < K; ++q) {
                            const long o = (long)gi * Cg + co;
                            const float wv = v[(o * Cg + ci) * K + q] * (g[q] / nf[q]);  // ATen _weight_norm
                            // fwd B[(q, ci)][co] ; bwd B[(q', co)][ci] with q' = K-1-q
                            wf[(((size_t)gi * K + q) * Cg + ci) * Cg + co] = wv;
                            wb[(((size_t)gi * K + (K - 1 - q)) * Cg + co) * Cg + ci] = wv;
                            if (bfw) {  // [g][q][n][k]: fwd n = co, k = ci; bwd (q' = K-1-q) n = ci, k = co
                                bf_f[(((size_t)gi * K + q) * Cg + co) * Cg + ci] = rne(wv);
                                bf_b[(((size_t)gi * K + (K - 1 - q)) * Cg + ci) * Cg + co] = rne(wv);
                            }
                        }
            e->wpos_f = e->dalloc((long)wf.size());
            e->wpos_b = e->dalloc((long)wb.size());
            HIPCHK(hipMemcpy(e->wpos_f, wf.data(), wf.size() * 4, hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(e->wpos_b, wb.data(), wb.size() * 4, hipMemcpyHostToDevice));
            if (bfw) {
                e->wpos_bf_f = e->dalloc((long)(bf_f.size() + 1) / 2);
                e->wpos_bf_b = e->dalloc((long)(bf_b.size() + 1) / 2);
                HIPCHK(hipMemcpy(e->wpos_bf_f, bf_f.data(), bf_f.size() * 2, hipMemcpyHostToDevice));
                HIPCHK(hipMemcpy(e->wpos_bf_b, bf_b.data(), bf_b.size() * 2, hipMemcpyHostToDevice));
            }
            e->bpos = up(b + "bias", H);
        }
        e->reset_slots(max_batch, true);
        HIPCHK(hipStreamSynchronize(e->st));
        *out = e.release();
    });
}

int32_t suta_destroy(suta_engine* e) {
    return guard([&] {
        if (!e) return;
        (void)hipStreamSynchronize(e->st);
        delete e;
    });
}

int32_t suta_reset(suta_engine* e) {
    return guard([&] {
        e->reset_slots(e->max_batch, true);
        HIPCHK(hipStreamSynchronize(e->st));
    });
}

static void check_batch(suta_engine* e, int32_t batch, int64_t n) {
    if (batch < 1 || batch > e->max_batch) throw SutaError(SUTA_ERR_ARG, "batch outside [1, max_batch]");
    if (n < 1) throw SutaError(SUTA_ERR_ARG, "n_samples < 1");
    if (e->max_samples > 0 && n > e->max_samples)
        throw SutaError(SUTA_ERR_ARG, "n_samples > max_samples given to suta_create");
}

int32_t suta_forward(suta_engine* e, const float* wav, int32_t on_dev, int32_t norm, int32_t batch, int64_t n,
                     float* logits_out) {
    return guard([&] {
        check_batch(e, batch, n);
        HIPCHK(hipSetDevice(e->device));
        suta_latch_switches();
        e->build_plan(batch, n);
        e->set_lengths(batch, nullptr);
        e->stage_input(wav, on_dev, norm, batch, n);
        e->forward(batch);
        HIPCHK(hipMemcpyAsync(logits_out, e->plan.logits, (size_t)batch * e->plan.T * e->c.V * 4, hipMemcpyDeviceToHost,
                              e->st));
        HIPCHK(hipStreamSynchronize(e->st));
        if (e->timing) e->collect_timing();
        e->check_sdpl();
    });
}

int32_t suta_step_ex(suta_engine* e, const float* wav, int32_t on_dev, int32_t norm, int32_t batch, int64_t n,
                     const suta_hparams* hp, int32_t repeat_inference, float* logits_out, int32_t logits_on_dev,
                     float* loss_out) {
    return guard([&] {
        check_batch(e, batch, n);
        if (!logits_out) throw SutaError(SUTA_ERR_ARG, "logits_out is null");
        HIPCHK(hipSetDevice(e->device));
        suta_latch_switches();
        e->build_plan(batch, n);
        e->set_lengths(batch, nullptr);
        e->stage_input(wav, on_dev, norm, batch, n);
        e->prepare_adam(*hp, 1);
        const size_t lbytes = (size_t)batch * e->plan.T * e->c.V * 4;
        const hipMemcpyKind lk = logits_on_dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        e->forward(batch);
        // repeat_inference == False (main.py:212-215): the caller gets the grad forward's logits, taken before the
        // backward reuses any buffer
        if (!repeat_inference) HIPCHK(hipMemcpyAsync(logits_out, e->plan.logits, lbytes, lk, e->st));
        e->backward(batch, *hp);
        e->adam(batch, *hp);
        if (repeat_inference) {
            e->forward(batch);
            HIPCHK(hipMemcpyAsync(logits_out, e->plan.logits, lbytes, lk, e->st));
        }
        if (loss_out)
            HIPCHK(hipMemcpyAsync(loss_out, e->plan.loss, (size_t)batch * 4, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipStreamSynchronize(e->st));
        if (e->timing) e->collect_timing();
        e->check_sdpl();
    });
}

int32_t suta_step(suta_engine* e, const float* wav, int32_t on_dev, int32_t norm, int32_t batch, int64_t n,
                  const suta_hparams* hp, float* logits_out, float* loss_out) {
    return suta_step_ex(e, wav, on_dev, norm, batch, n, hp, 1, logits_out, 0, loss_out);
}

}  // extern "C"

// suta_adapt / suta_adapt_varlen body: ns == null -> every utterance has n samples (stride n)
static void adapt_impl(suta_engine* e, const float* wav, int32_t on_dev, int32_t norm, int32_t batch, int64_t n,
                       const int64_t* ns, int64_t stride, int32_t steps, const suta_hparams* hp, const int32_t* rec,
                       int32_t nrec, float* logits_out, int32_t logits_on_dev, int32_t* ids_out, int64_t* frames_out) {
    check_batch(e, batch, n);
    if (steps < 0) throw SutaError(SUTA_ERR_ARG, "steps < 0");
    suta_latch_switches();
    for (int i = 0; i < nrec; ++i)
        if (rec[i] < 0 || rec[i] > steps) throw SutaError(SUTA_ERR_ARG, "record step outside [0, steps]");
    HIPCHK(hipSetDevice(e->device));
    e->build_plan(batch, n);
    e->set_lengths(batch, ns);
    const int T = e->plan.T, V = e->c.V;
    if (frames_out) {
        if (ns) for (int b = 0; b < batch; ++b) frames_out[b] = e->plan.h_T[b];
        else *frames_out = T;
    }
    const size_t per = (size_t)batch * T * V;
    e->stage_input(wav, on_dev, norm, batch, n, stride);
    if (hp->episodic) e->opt_steps = 0;  // slots are reset inside the loop (adapt_loop)
    e->prepare_adam(*hp, steps);
    // device staging of the recorded outputs (the loop is graph-captured; it never touches host memory)
    const size_t rl = logits_out ? (size_t)nrec * per : 0, ri = ids_out ? (size_t)nrec * batch * T : 0;
    if (e->recbuf.alloc((rl + ri) * sizeof(float) + 256)) e->drop_graph();
    float* rec_logits = logits_out ? e->recbuf.p : nullptr;
    int* rec_ids = ids_out ? reinterpret_cast<int*>(e->recbuf.p + rl) : nullptr;
    suta_engine::GraphKey key;
    key.B = batch;
    key.N = e->plan.N;
    key.ragged = e->plan.ragged;
    key.mode = e->gemm_mode;
    key.steps = steps;
    key.want_logits = logits_out != nullptr;
    key.want_ids = ids_out != nullptr;
    key.hp = *hp;
    key.rec.assign(rec, rec + nrec);
    key.sw = suta_switches();
    const bool graph_ok = e->graph_key_repeats(key);
    e->run_adapt_loop(batch, *hp, steps, rec, nrec, rec_logits, rec_ids, graph_ok);
    // the loop ran to completion with this key, so every buffer it needs is allocated now: a lazy allocation during
    // it (drop_graph) must not cost the next call of the key its capture (config C4 allocated its bf16 conversion
    // buffer in the first call, which pushed the capture to the third)
    e->gkey_seen = true;
    if (logits_out && nrec)
        HIPCHK(hipMemcpyAsync(logits_out, rec_logits, rl * 4, logits_on_dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                              e->st));
    if (ids_out && nrec) HIPCHK(hipMemcpyAsync(ids_out, rec_ids, ri * 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(hipStreamSynchronize(e->st));
    if (e->timing) e->collect_timing();
    e->check_sdpl();
}

extern "C" {

int32_t suta_adapt(suta_engine* e, const float* wav, int32_t on_dev, int32_t norm, int32_t batch, int64_t n,
                   int32_t steps, const suta_hparams* hp, const int32_t* rec, int32_t nrec, float* logits_out,
                   int32_t logits_on_dev, int32_t* ids_out, int64_t* frames_out) {
    return guard([&] {
        adapt_impl(e, wav, on_dev, norm, batch, n, nullptr, n, steps, hp, rec, nrec, logits_out, logits_on_dev,
                   ids_out, frames_out);
    });
}

int32_t suta_adapt_varlen(suta_engine* e, const float* wav, int32_t on_dev, int32_t norm, int32_t batch,
                          const int64_t* n_samples, int64_t stride, int32_t steps, const suta_hparams* hp,
                          const int32_t* rec, int32_t nrec, float* logits_out, int32_t logits_on_dev, int32_t* ids_out,
                          int64_t* frames_out) {
    return guard([&] {
        if (!n_samples || batch < 1) throw SutaError(SUTA_ERR_ARG, "n_samples is null or batch < 1");
        int64_t nmax = 0;
        for (int b = 0; b < batch; ++b) nmax = std::max<int64_t>(nmax, n_samples[b]);
        if (stride < nmax) throw SutaError(SUTA_ERR_ARG, "stride < max(n_samples)");
        if (e->max_samples > 0 && nmax > e->max_samples)
            throw SutaError(SUTA_ERR_ARG, "n_samples > max_samples given to suta_create");
        // the layout length is `stride`: callers quantise it so repeated layouts reuse the captured step
        adapt_impl(e, wav, on_dev, norm, batch, stride, n_samples, stride, steps, hp, rec, nrec, logits_out,
                   logits_on_dev, ids_out, frames_out);
    });
}

int32_t suta_loss_grad(suta_engine* e, const float* logits, int32_t batch, int64_t frames, const suta_hparams* hp,
                       float* dlogits_out, float* loss_out) {
    return guard([&] {
        if (batch < 1 || frames < 1) throw SutaError(SUTA_ERR_ARG, "empty logits");
        HIPCHK(hipSetDevice(e->device));
        const int V = e->c.V;
        const size_t n = (size_t)batch * frames * V;
        DevBuf buf;
        buf.alloc((2 * n + (size_t)batch * frames * 66 + 64 + batch) * sizeof(float));
        float* dl = buf.p;
        float* dd = dl + n;
        float* scr = dd + n;
        float* ls = scr + (size_t)batch * frames * 66 + 64;
        HIPCHK(hipMemcpyAsync(dl, logits, n * 4, hipMemcpyHostToDevice, e->st));
        LossHP lh{hp->temp, hp->em_coef, hp->div_coef, hp->reweight, hp->non_blank};
        launch_suta_loss(dl, batch, (int)frames, V, lh, nullptr, dd, ls, scr, e->st);
        DevBuf sbuf;
        if (hp->pl_coef > 0.f) {
            if (V > 32) throw SutaError(SUTA_ERR_UNSUPPORTED, "SDPL objective needs vocab_size <= 32");
            if (frames > 2048) throw SutaError(SUTA_ERR_UNSUPPORTED, "T > 2048 frames");
            const long per = sdpl_scratch_floats((int)frames);
            sbuf.alloc(((size_t)batch * per + 64) * sizeof(float));
            HIPCHK(hipMemsetAsync(sbuf.p, 0, sbuf.bytes, e->st));
            int* err = reinterpret_cast<int*>(sbuf.p);
            launch_sdpl_loss(dl, batch, (int)frames, V, hp->pl_coef, nullptr, dd, ls, sbuf.p + 64, err, e->st);
            e->sdpl_used = true;
            e->sdpl_err = err;
        }
        HIPCHK(hipMemcpyAsync(dlogits_out, dd, n * 4, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipMemcpyAsync(loss_out, ls, (size_t)batch * 4, hipMemcpyDeviceToHost, e->st));
        HIPCHK(hipStreamSynchronize(e->st));
        e->check_sdpl();
    });
}

int32_t suta_get_param(suta_engine* e, int32_t slot, const char* name, float* out, int64_t numel) {
    return guard([&] {
        auto it = e->tpi.find(name);
        if (it == e->tpi.end()) throw SutaError(SUTA_ERR_ARG, std::string("not a trainable tensor: ") + name);
        if (slot < 0 || slot >= e->max_batch) throw SutaError(SUTA_ERR_ARG, "slot out of range");
        const TP& t = e->tps[it->second];
        if (numel != t.numel) throw SutaError(SUTA_ERR_ARG, "numel mismatch");
        std::vector<float> h(t.numel);
        HIPCHK(hipStreamSynchronize(e->st));
        HIPCHK(hipMemcpy(h.data(), e->P + (long)slot * e->Pn + t.off, t.numel * 4, hipMemcpyDeviceToHost));
        if (t.conv_w) {
            const long co = t.shape[0], ci = t.shape[1], kk = t.shape[2];
            for (long o = 0; o < co; ++o)
                for (long i2 = 0; i2 < ci; ++i2)
                    for (long q = 0; q < kk; ++q) out[(o * ci + i2) * kk + q] = h[(q * ci + i2) * co + o];
        } else {
            std::memcpy(out, h.data(), t.numel * 4);
        }
    });
}

int32_t suta_param_info(suta_engine* e, const char* name, int32_t train_feature, int32_t bias_only, int32_t* k,
                        int64_t* numel) {
    return guard([&] {
        auto it = e->tpi.find(name);
        if (it == e->tpi.end()) {
            *k = 0;
            *numel = 0;
            return;
        }
        const TP& t = e->tps[it->second];
        *k = e->multiplicity(t, train_feature, bias_only);
        *numel = t.numel;
    });
}

int32_t suta_sync(suta_engine* e) { return guard([&] { HIPCHK(hipStreamSynchronize(e->st)); }); }

void* suta_stream(suta_engine* e) { return (void*)e->st; }

int32_t suta_set_timing(suta_engine* e, int32_t enable) {
    return guard([&] {
        e->timing = enable != 0;
        for (int i = 0; i < NFAM; ++i) {
            e->fam_ms[i] = 0;
            e->fam_n[i] = 0;
            e->fam_bytes[i] = 0;
        }
    });
}

int32_t suta_get_timing(suta_engine* e, double* ms, int64_t* n) {
    return guard([&] {
        e->collect_timing();
        for (int i = 0; i < 6; ++i) {
            ms[i] = e->fam_ms[i];
            n[i] = e->fam_n[i];
        }
        ms[F_GEMM] += e->fam_ms[F_ATTN];
        n[F_GEMM] += e->fam_n[F_ATTN];
        ms[F_NORM] += e->fam_ms[F_FRONT];
        n[F_NORM] += e->fam_n[F_FRONT];
    });
}

int32_t suta_get_timing_ex(suta_engine* e, int32_t nfam, double* ms, int64_t* n, double* alg_bytes) {
    return guard([&] {
        if (nfam < 1 || nfam > NFAM) throw SutaError(SUTA_ERR_ARG, "nfam outside [1, SUTA_TIMING_FAMILIES]");
        e->collect_timing();
        for (int i = 0; i < nfam; ++i) {
            ms[i] = e->fam_ms[i];
            n[i] = e->fam_n[i];
            if (alg_bytes) alg_bytes[i] = e->fam_bytes[i];
        }
    });
}

int32_t suta_set_precision(suta_engine* e, int32_t mode) {
    return guard([&] {
        if (mode != SUTA_PRECISION_FP32_MFMA && mode != SUTA_PRECISION_FP32_SPLIT_BF16 && mode != SUTA_PRECISION_BF16)
            throw SutaError(SUTA_ERR_ARG, "unknown precision mode");
        HIPCHK(hipSetDevice(e->device));
        if (mode == SUTA_PRECISION_BF16 && e->bf16_planes) e->build_weight_planes();
        e->gemm_mode = mode;
    });
}

int32_t suta_set_graphs(suta_engine* e, int32_t enable) {
    return guard([&] { e->use_graphs = enable != 0; });
}

int32_t suta_get_graph_stats(suta_engine* e, int32_t* last_mode, int64_t* captures, int64_t* launches) {
    return guard([&] {
        if (last_mode) *last_mode = e->last_loop_mode;
        if (captures) *captures = e->graph_captures;
        if (launches) *launches = e->graph_launches;
    });
}

int32_t suta_set_census(int32_t enable) {
    return guard([&] { gemm_census_enable(enable != 0); });
}

int32_t suta_get_census(char* buf, int64_t cap, int64_t* needed) {
    return guard([&] {
        const std::string t = gemm_census_text();
        if (needed) *needed = (int64_t)t.size() + 1;
        if (!buf || cap < (int64_t)t.size() + 1) throw SutaError(SUTA_ERR_ARG, "census buffer too small");
        memcpy(buf, t.c_str(), t.size() + 1);
    });
}

}  // extern "C"
