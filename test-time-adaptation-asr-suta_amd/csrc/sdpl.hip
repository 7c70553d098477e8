// SDPL objective (reference main_SDPL.py:143-209): pseudo-label CTC loss on the
// model's own greedy transcript, mixed with the SUTA loss:  L = (1 - pl) * L_suta + pl * L_ctc.
//
// pseudo_labeling_loss (main_SDPL.py:192-209), restated:
//   target  = vocab ids of processor.batch_decode(argmax ids): collapse repeats, drop blank 0, the
//             word delimiter '|' (4) decodes to a space and the transcript is strip()ped, so leading
//             and trailing delimiters vanish; every character maps back through vocab.json (a
//             special token <s>, </s>, <unk> decodes to several characters and the reference raises
//             KeyError: flagged here, reported by the engine)
//   lp      = outputs.log_softmax(1): log-softmax over TIME (dim 1 of (1, T, V)), per class
//   L_ctc   = nn.CTCLoss(blank=0, reduction='mean')(lp, target) = nll / max(U, 1)
//   dL/dlp  = torch's CTC backward (LossCTC.cpp): exp(lp) - exp(lcab + nll - lp), lcab = log sum over
//             the extended-target states s with label c of alpha_t(s) beta_t(s); the exp(lp) term
//             assumes lp is normalised over classes, which it is not here -- reproduced as is
//   dL/dz   = through the time log-softmax: g - softmax_t(z)[t,c] * sum_t' g[t',c]
// Kernels: (1) per utterance (one block): greedy ids, target, time log-softmax, the alpha and beta
// recursions in log space (fp32, torch's 3-term max-shifted log-sum-exp); (2) one thread per
// (frame, class): posterior occupancy and dL/dlp; (3) per utterance: the time-softmax backward and
// the (1 - pl, pl) mix into the SUTA gradient and loss already in dlogits / loss.  Fixed-order sums
// throughout (bitwise reproducible).
#include "ops.h"

namespace {

constexpr int SD_MAXT = 2048;

__device__ __forceinline__ float lse2(float a, float b) {
    const float m = fmaxf(a, b);
    if (m == -INFINITY) return -INFINITY;
    return logf(expf(a - m) + expf(b - m)) + m;
}
__device__ __forceinline__ float lse3(float a, float b, float c) {
    float m = fmaxf(a, fmaxf(b, c));
    if (m == -INFINITY) return -INFINITY;
    return logf(expf(a - m) + expf(b - m) + expf(c - m)) + m;
}

struct SdplScratch {
    float* lp;     // [Tl][32]
    float* g;      // [Tl][32]
    float* alpha;  // [Tl][S]
    float* beta;   // [Tl][S]
    int* tgt;      // [Tl]
    int* meta;     // [4]: U, error flag, T
    float* nll;    // [1]
};

__device__ __forceinline__ SdplScratch sdpl_scratch(float* base, int Tl) {
    const long S = 2L * Tl + 1;
    SdplScratch s;
    s.lp = base;
    s.g = s.lp + (long)Tl * 32;
    s.alpha = s.g + (long)Tl * 32;
    s.beta = s.alpha + (long)Tl * S;
    s.tgt = reinterpret_cast<int*>(s.beta + (long)Tl * S);
    s.meta = s.tgt + Tl;
    s.nll = reinterpret_cast<float*>(s.meta + 4);
    return s;
}

__global__ __launch_bounds__(256) void sdpl_prep_kernel(const float* __restrict__ logits, int Tl, int V,
                                                        const int* __restrict__ tlen, float* __restrict__ scratch,
                                                        long sstride) {
    __shared__ int ids[SD_MAXT];
    __shared__ int tg[SD_MAXT];
    __shared__ float rowa[2 * SD_MAXT + 1], rowb[2 * SD_MAXT + 1];
    __shared__ int sU;
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int T = tlen ? tlen[b] : Tl;
    const float* L = logits + (long)b * Tl * V;
    SdplScratch sc = sdpl_scratch(scratch + (long)b * sstride, Tl);

    // greedy ids (first max, torch.argmax)
    for (int t = tid; t < T; t += 256) {
        const float* l = L + (long)t * V;
        float bv = l[0];
        int bi = 0;
        for (int j = 1; j < V; ++j)
            if (l[j] > bv) {
                bv = l[j];
                bi = j;
            }
        ids[t] = bi;
    }
    __syncthreads();
    if (tid == 0) {  // transcript -> target ids (HF decode + strip + vocab lookup)
        int U = 0, prev = -1, err = 0;
        for (int t = 0; t < T; ++t) {
            const int i = ids[t];
            if (i == prev) continue;
            prev = i;
            if (i == 0) continue;
            tg[U++] = i;
        }
        int lo = 0, hi = U;
        while (lo < hi && tg[lo] == 4) ++lo;
        while (hi > lo && tg[hi - 1] == 4) --hi;
        U = hi - lo;
        for (int j = 0; j < U; ++j) {
            tg[j] = tg[lo + j];
            if (tg[j] >= 1 && tg[j] <= 3) err = 1;
        }
        sU = U;
        sc.meta[0] = U;
        sc.meta[1] = err;
        sc.meta[2] = T;
    }
    __syncthreads();
    const int U = sU, S = 2 * U + 1;
    for (int j = tid; j < U; j += 256) sc.tgt[j] = tg[j];

    // lp = log_softmax over time, per class (one wave per class, fixed-order reductions)
    for (int c = w; c < V; c += 4) {
        float m = -INFINITY;
        for (int t = lane; t < T; t += 64) m = fmaxf(m, L[(long)t * V + c]);
        m = wave_max(m);
        float s = 0.f;
        for (int t = lane; t < T; t += 64) s += expf(L[(long)t * V + c] - m);
        s = wave_sum(s);
        const float lz = m + logf(s);
        for (int t = lane; t < T; t += 64) sc.lp[(long)t * 32 + c] = L[(long)t * V + c] - lz;
    }
    __syncthreads();

    auto lab = [&](int s) { return (s & 1) ? tg[s >> 1] : 0; };
    // alpha (Graves eq. 6-7, torch LossCTC.cpp): alpha_0(0) = lp[0][0], alpha_0(1) = lp[0][l1]
    for (int s = tid; s < S; s += 256) {
        float v = -INFINITY;
        if (s == 0) v = sc.lp[0];
        else if (s == 1) v = sc.lp[lab(1)];
        rowa[s] = v;
        sc.alpha[s] = v;
    }
    __syncthreads();
    float* prev = rowa;
    float* cur = rowb;
    for (int t = 1; t < T; ++t) {
        for (int s = tid; s < S; s += 256) {
            const int l = lab(s);
            const float a1 = prev[s];
            const float a2 = s > 0 ? prev[s - 1] : -INFINITY;
            const float a3 = (s > 1 && l != 0 && l != lab(s - 2)) ? prev[s - 2] : -INFINITY;
            const float v = lse3(a1, a2, a3) + sc.lp[(long)t * 32 + l];
            cur[s] = v;
            sc.alpha[(long)t * S + s] = v;
        }
        __syncthreads();
        float* tmp = prev;
        prev = cur;
        cur = tmp;
    }
    if (tid == 0) {
        const float l1 = prev[S - 1];
        const float l2 = S > 1 ? prev[S - 2] : -INFINITY;
        sc.nll[0] = -lse2(l1, l2);
    }
    __syncthreads();
    // beta: beta_{T-1}(S-1) = lp[T-1][l'(S-1)], beta_{T-1}(S-2) = lp[T-1][l'(S-2)]
    for (int s = tid; s < S; s += 256) {
        float v = -INFINITY;
        if (s == S - 1 || s == S - 2) v = sc.lp[(long)(T - 1) * 32 + lab(s)];
        rowa[s] = v;
        sc.beta[(long)(T - 1) * S + s] = v;
    }
    __syncthreads();
    prev = rowa;
    cur = rowb;
    for (int t = T - 2; t >= 0; --t) {
        for (int s = tid; s < S; s += 256) {
            const int l = lab(s);
            const float b1 = prev[s];
            const float b2 = s < S - 1 ? prev[s + 1] : -INFINITY;
            const float b3 = (s < S - 2 && l != 0 && l != lab(s + 2)) ? prev[s + 2] : -INFINITY;
            const float v = lse3(b1, b2, b3) + sc.lp[(long)t * 32 + l];
            cur[s] = v;
            sc.beta[(long)t * S + s] = v;
        }
        __syncthreads();
        float* tmp = prev;
        prev = cur;
        cur = tmp;
    }
}

// g[t][c] = (exp(lp) - sum_{s: l'(s) = c} exp(alpha + beta + nll - lp)) / max(U, 1)
__global__ __launch_bounds__(256) void sdpl_grad_kernel(int Tl, float* __restrict__ scratch, long sstride) {
    const int b = blockIdx.y;
    SdplScratch sc = sdpl_scratch(scratch + (long)b * sstride, Tl);
    const int U = sc.meta[0], T = sc.meta[2], S = 2 * U + 1;
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)Tl * 32) return;
    const int t = (int)(i >> 5), c = (int)(i & 31);
    if (t >= T) {
        sc.g[i] = 0.f;
        return;
    }
    const float lp = sc.lp[i], nll = sc.nll[0];
    const float* al = sc.alpha + (long)t * S;
    const float* be = sc.beta + (long)t * S;
    float occ = 0.f;
    if (c == 0) {
        for (int s = 0; s < S; s += 2) occ += expf(al[s] + be[s] + nll - lp);
    } else {
        for (int j = 0; j < U; ++j)
            if (sc.tgt[j] == c) occ += expf(al[2 * j + 1] + be[2 * j + 1] + nll - lp);
    }
    sc.g[i] = (expf(lp) - occ) / (float)max(U, 1);
}

// dz[t][c] = g[t][c] - exp(lp[t][c]) * sum_t g[t][c];  dlogits = (1 - pl) dlogits + pl dz;
// loss = (1 - pl) loss + pl nll / max(U, 1)
__global__ __launch_bounds__(256) void sdpl_combine_kernel(int Tl, int V, float pl, float* __restrict__ dlogits,
                                                           float* __restrict__ loss, float* __restrict__ scratch,
                                                           long sstride, int* __restrict__ err) {
    __shared__ float Gc[32];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    SdplScratch sc = sdpl_scratch(scratch + (long)b * sstride, Tl);
    const int U = sc.meta[0], T = sc.meta[2];
    for (int c = w; c < 32; c += 4) {
        float s = 0.f;
        for (int t = lane; t < T; t += 64) s += sc.g[(long)t * 32 + c];
        s = wave_sum(s);
        if (lane == 0) Gc[c] = s;
    }
    __syncthreads();
    float* dL = dlogits + (long)b * Tl * V;
    const float keep = 1.0f - pl;
    for (long i = tid; i < (long)T * V; i += 256) {
        const int t = (int)(i / V), c = (int)(i % V);
        const long k = (long)t * 32 + c;
        const float dz = sc.g[k] - expf(sc.lp[k]) * Gc[c];
        dL[i] = keep * dL[i] + pl * dz;
    }
    if (tid == 0) {
        loss[b] = keep * loss[b] + pl * (sc.nll[0] / (float)max(U, 1));
        if (sc.meta[1]) atomicOr(err, 1);
    }
}

}  // namespace

long sdpl_scratch_floats(int Tl) {
    const long S = 2L * Tl + 1;
    return 64L * Tl + 2L * Tl * S + Tl + 4 + 1 + 16;
}

void launch_sdpl_loss(const float* logits, int B, int Tl, int V, float pl_coef, const int* tlen, float* dlogits,
                      float* loss, float* scratch, int* err, hipStream_t st) {
    const long ss = sdpl_scratch_floats(Tl);
    hipLaunchKernelGGL(sdpl_prep_kernel, dim3(B), dim3(256), 0, st, logits, Tl, V, tlen, scratch, ss);
    hipLaunchKernelGGL(sdpl_grad_kernel, dim3((unsigned)((Tl * 32L + 255) / 256), B), dim3(256), 0, st, Tl, scratch,
                       ss);
    hipLaunchKernelGGL(sdpl_combine_kernel, dim3(B), dim3(256), 0, st, Tl, V, pl_coef, dlogits, loss, scratch, ss,
                       err);
}
