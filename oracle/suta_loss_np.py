"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Float64 NumPy closed form of the SUTA loss and its gradient w.r.t. the logits,
for ONE utterance (the reference's mcc_loss is batch-1 only, main.py:32).

Restates reference main.py:26-60 (softmax_entropy, mcc_loss, div_loss) and the
loss assembly of forward_and_adapt main.py:181-203; the gradient is the
analytic one of SURVEY.md Appendix A (pinned against autograd through the
reference's own code by tests/golden G1).
"""
import numpy as np


def _softmax(z, axis=-1):
    m = z.max(axis=axis, keepdims=True)
    e = np.exp(z - m)
    return e / e.sum(axis=axis, keepdims=True)


def _log_softmax(z, axis=-1):
    m = z.max(axis=axis, keepdims=True)
    return z - m - np.log(np.exp(z - m).sum(axis=axis, keepdims=True))


def suta_loss_and_grad(logits, temp=2.5, em_coef=0.3, reweight=True, non_blank=True, div_coef=0.0):
    """logits: (T, V) array.  Returns (loss: float, dlogits: (T, V) float64)."""
    l = np.asarray(logits, dtype=np.float64)
    T, V = l.shape
    z = l / temp
    p = _softmax(z)
    lp = _log_softmax(z)
    H = -(p * lp).sum(-1)                                   # main.py:28
    dH = -p * (lp + H[:, None])                             # dH_t/dz_tj
    loss = 0.0
    dz = np.zeros_like(z)
    if em_coef > 0:
        if non_blank:
            m = (l.argmax(-1) != 0)                         # main.py:183-184 (first max wins, as torch)
            K = int(m.sum())
            if K == 0:
                loss += float("nan")                        # mean of an empty selection
            else:
                loss += em_coef * H[m].mean()
                dz += em_coef * (m[:, None] / K) * dH
        else:
            loss += em_coef * H.mean()
            dz += em_coef * dH / T
    if 1 - em_coef > 0:
        if reweight:                                        # main.py:33-37 (weights detached)
            w = 1 + np.exp(-H)
            w = T * w / w.sum()
        else:
            w = np.ones(T)
        C = (p * w[:, None]).T @ p                          # (V, V)
        s = C.sum(1)                                        # main.py:41 torch.sum(C, dim=1)
        Nn = C / s[None, :]
        G = (1.0 - np.eye(V)) / V
        mcc = (Nn.sum() - np.trace(Nn)) / V                 # main.py:42
        loss += (1 - em_coef) * mcc
        rho = (G * C).sum(0) / s ** 2                       # rho_a = sum_i G_ia C_ia / s_a^2
        dC = G / s[None, :] - rho[:, None]
        dP = w[:, None] * (p @ (dC + dC.T))
        dz += (1 - em_coef) * p * (dP - (dP * p).sum(-1, keepdims=True))
    dl = dz / temp
    if div_coef > 0:                                        # main.py:46-60: raw logits, blank dropped
        cls = l.mean(0)[1:]
        q = _softmax(cls)
        lq = _log_softmax(cls)
        Hq = -(q * lq).sum()
        loss += div_coef * (-Hq)
        dcls = q * (lq + Hq)
        dl[:, 1:] += div_coef * dcls[None, :] / T
    return loss, dl
