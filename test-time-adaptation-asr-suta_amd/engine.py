"""ctypes binding of libsuta.so (C ABI: include/suta.h).

There is no CPU fallback: if the HIP library is missing or fails to load, every entry
point raises.  Build it with `__graft_entry__.build()` (or `make -C csrc`).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence

import numpy as np

from .config import param_shapes

LIB_PATH = os.environ.get("SUTA_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsuta.so")
MAX_CONV = 8

# exported symbols (kept in sync with include/suta.h; tests/test_abi.py checks both)
EXPORTS = ("suta_create", "suta_destroy", "suta_reset", "suta_num_frames", "suta_forward", "suta_step", "suta_step_ex",
           "suta_adapt", "suta_adapt_varlen", "suta_loss_grad", "suta_get_param", "suta_param_info", "suta_sync", "suta_stream", "suta_set_timing",
           "suta_get_timing", "suta_get_timing_ex", "suta_set_precision", "suta_set_graphs", "suta_set_census",
           "suta_get_census", "suta_get_graph_stats", "suta_last_error")


class ModelConfigC(C.Structure):
    _fields_ = [("hidden_size", C.c_int32), ("num_hidden_layers", C.c_int32), ("num_attention_heads", C.c_int32),
                ("intermediate_size", C.c_int32), ("vocab_size", C.c_int32), ("num_conv_layers", C.c_int32),
                ("conv_dim", C.c_int32 * MAX_CONV), ("conv_kernel", C.c_int32 * MAX_CONV),
                ("conv_stride", C.c_int32 * MAX_CONV), ("conv_bias", C.c_int32),
                ("feat_extract_norm_layer", C.c_int32), ("do_stable_layer_norm", C.c_int32),
                ("num_conv_pos_embeddings", C.c_int32), ("num_conv_pos_embedding_groups", C.c_int32),
                ("layer_norm_eps", C.c_float)]


class HParamsC(C.Structure):
    _fields_ = [("lr", C.c_float), ("temp", C.c_float), ("em_coef", C.c_float), ("div_coef", C.c_float),
                ("beta1", C.c_float), ("beta2", C.c_float), ("adam_eps", C.c_float), ("weight_decay", C.c_float),
                ("reweight", C.c_int32), ("non_blank", C.c_int32), ("train_feature", C.c_int32),
                ("bias_only", C.c_int32), ("episodic", C.c_int32), ("pl_coef", C.c_float),
                ("optimizer", C.c_int32), ("lr_step_size", C.c_int32), ("lr_gamma", C.c_float)]

OPTIMIZERS = {"AdamW": 0, "Adam": 0, "SGD": 1}  # SUTA_OPT_*: Adam == AdamW at the reference's weight decay 0


@dataclass
class SutaHParams:
    """forward_and_adapt / setup_optimizer arguments; defaults = scripts/LS.sh flags."""
    lr: float = 2e-5
    temp: float = 2.5
    em_coef: float = 0.3
    div_coef: float = 0.0
    reweight: bool = True
    non_blank: bool = True
    train_feature: bool = True
    bias_only: bool = False
    episodic: bool = True
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.0
    pl_coef: float = 0.0  # SDPL mix (main_SDPL.py:143-209); 0 = SUTA
    optimizer: str = "AdamW"  # --opt (main.py:9-18): AdamW / Adam / SGD
    lr_step_size: int = 0     # StepLR (main.py:20-21: step_size 1, gamma 0.7); 0 = no scheduler
    lr_gamma: float = 0.7

    def to_c(self) -> HParamsC:
        if self.optimizer not in OPTIMIZERS:
            raise ValueError(f"optimizer {self.optimizer!r}: the engine implements {sorted(OPTIMIZERS)}")
        if self.optimizer == "Adam" and self.weight_decay != 0:
            raise ValueError("Adam with weight decay (L2 in the gradient) is not AdamW; the reference passes 0")
        if self.optimizer == "SGD" and self.weight_decay != 0:
            raise ValueError("SGD with weight decay (wd * p added to the gradient) is not implemented; the reference "
                             "passes 0 (main.py:18)")
        return HParamsC(self.lr, self.temp, self.em_coef, self.div_coef, self.betas[0], self.betas[1], self.eps,
                        self.weight_decay, int(self.reweight), int(self.non_blank), int(self.train_feature),
                        int(self.bias_only), int(self.episodic), float(self.pl_coef), OPTIMIZERS[self.optimizer],
                        int(self.lr_step_size), float(self.lr_gamma))


_lib = None


def load_library(path: str = LIB_PATH):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libsuta.so not found at {path}: build it with __graft_entry__.build() "
                           "(there is no CPU fallback)")
    lib = C.CDLL(path)
    P = C.POINTER
    f32p, i64p, i32p = P(C.c_float), P(C.c_int64), P(C.c_int32)
    lib.suta_create.argtypes = [P(ModelConfigC), P(C.c_char_p), P(f32p), i64p, C.c_int32, C.c_int32, C.c_int32,
                                C.c_int64, P(C.c_void_p)]
    lib.suta_destroy.argtypes = [C.c_void_p]
    lib.suta_reset.argtypes = [C.c_void_p]
    lib.suta_num_frames.argtypes = [P(ModelConfigC), C.c_int64, i64p]
    lib.suta_forward.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int64, C.c_void_p]
    lib.suta_step.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int64, P(HParamsC),
                              C.c_void_p, C.c_void_p]
    lib.suta_step_ex.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int64, P(HParamsC),
                                 C.c_int32, C.c_void_p, C.c_int32, C.c_void_p]
    lib.suta_adapt.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int64, C.c_int32,
                               P(HParamsC), i32p, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p, i64p]
    lib.suta_loss_grad.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int64, P(HParamsC), C.c_void_p,
                                   C.c_void_p]
    lib.suta_get_param.argtypes = [C.c_void_p, C.c_int32, C.c_char_p, f32p, C.c_int64]
    lib.suta_param_info.argtypes = [C.c_void_p, C.c_char_p, C.c_int32, C.c_int32, i32p, i64p]
    lib.suta_sync.argtypes = [C.c_void_p]
    lib.suta_stream.argtypes = [C.c_void_p]
    lib.suta_stream.restype = C.c_void_p
    if hasattr(lib, "suta_adapt_varlen"):  # (tools may load an older library build for A/B runs)
        lib.suta_adapt_varlen.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, i64p, C.c_int64,
                                          C.c_int32, P(HParamsC), i32p, C.c_int32, C.c_void_p, C.c_int32,
                                          C.c_void_p, i64p]
    lib.suta_set_timing.argtypes = [C.c_void_p, C.c_int32]
    lib.suta_get_timing.argtypes = [C.c_void_p, P(C.c_double), i64p]
    if hasattr(lib, "suta_get_timing_ex"):
        lib.suta_get_timing_ex.argtypes = [C.c_void_p, C.c_int32, P(C.c_double), i64p, P(C.c_double)]
    lib.suta_set_graphs.argtypes = [C.c_void_p, C.c_int32]
    if hasattr(lib, "suta_set_census"):
        lib.suta_set_census.argtypes = [C.c_int32]
        lib.suta_get_census.argtypes = [C.c_char_p, C.c_int64, i64p]
    lib.suta_set_precision.argtypes = [C.c_void_p, C.c_int32]
    if hasattr(lib, "suta_get_graph_stats"):
        lib.suta_get_graph_stats.argtypes = [C.c_void_p, i32p, i64p, i64p]
    lib.suta_last_error.restype = C.c_char_p
    for name in EXPORTS:
        if name != "suta_stream" and name != "suta_last_error" and hasattr(lib, name):
            getattr(lib, name).restype = C.c_int32
    _lib = lib
    return lib


def _check(status: int):
    if status != 0:
        msg = _lib.suta_last_error().decode(errors="replace")
        raise RuntimeError(f"libsuta error {status}: {msg}")


def config_to_c(cfg: dict) -> ModelConfigC:
    m = ModelConfigC()
    m.hidden_size = cfg["hidden_size"]
    m.num_hidden_layers = cfg["num_hidden_layers"]
    m.num_attention_heads = cfg["num_attention_heads"]
    m.intermediate_size = cfg["intermediate_size"]
    m.vocab_size = cfg["vocab_size"]
    n = len(cfg["conv_dim"])
    m.num_conv_layers = n
    for i in range(n):
        m.conv_dim[i] = cfg["conv_dim"][i]
        m.conv_kernel[i] = cfg["conv_kernel"][i]
        m.conv_stride[i] = cfg["conv_stride"][i]
    m.conv_bias = int(bool(cfg["conv_bias"]))
    m.feat_extract_norm_layer = int(cfg["feat_extract_norm"] == "layer")
    m.do_stable_layer_norm = int(bool(cfg["do_stable_layer_norm"]))
    m.num_conv_pos_embeddings = cfg["num_conv_pos_embeddings"]
    m.num_conv_pos_embedding_groups = cfg["num_conv_pos_embedding_groups"]
    m.layer_norm_eps = cfg.get("layer_norm_eps", 1e-5)
    return m


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class SutaEngine:
    """One libsuta engine on one GPU: `max_batch` utterance slots sharing the frozen encoder."""

    def __init__(self, cfg: dict, weights: Dict[str, np.ndarray], device: int = 0, max_batch: int = 1,
                 max_samples: int = 600000):
        self.lib = load_library()
        self.cfg = cfg
        self.shapes = dict(param_shapes(cfg))
        names = [k for k in weights if k in self.shapes]
        arrs = [np.ascontiguousarray(weights[k], dtype=np.float32) for k in names]
        cnames = (C.c_char_p * len(names))(*[n.encode() for n in names])
        cdata = (C.POINTER(C.c_float) * len(names))(*[a.ctypes.data_as(C.POINTER(C.c_float)) for a in arrs])
        cnum = (C.c_int64 * len(names))(*[a.size for a in arrs])
        self._c_cfg = config_to_c(cfg)
        h = C.c_void_p()
        _check(self.lib.suta_create(C.byref(self._c_cfg), cnames, cdata, cnum, len(names), device, max_batch,
                                    max_samples, C.byref(h)))
        self.handle = h
        self.max_batch = max_batch
        self.V = cfg["vocab_size"]

    def close(self):
        if getattr(self, "handle", None):
            self.lib.suta_destroy(self.handle)
            self.handle = None

    __del__ = close

    def num_frames(self, n_samples: int) -> int:
        out = C.c_int64()
        _check(self.lib.suta_num_frames(C.byref(self._c_cfg), n_samples, C.byref(out)))
        return out.value

    @staticmethod
    def _wav(wav):
        """(ptr, on_device, batch, n, keepalive) for a numpy array or a torch tensor (cpu or cuda)."""
        if hasattr(wav, "data_ptr"):  # torch tensor
            t = wav.detach()
            if t.dim() == 1:
                t = t[None]
            t = t.contiguous().float()
            on_dev = int(t.is_cuda)
            if not on_dev:
                a = t.numpy()
                return _ptr(a), 0, a.shape[0], a.shape[1], a
            return C.c_void_p(t.data_ptr()), 1, t.shape[0], t.shape[1], t
        a = np.ascontiguousarray(wav, dtype=np.float32)
        if a.ndim == 1:
            a = a[None]
        return _ptr(a), 0, a.shape[0], a.shape[1], a

    def reset(self):
        _check(self.lib.suta_reset(self.handle))

    def forward(self, wav, normalize: bool = False) -> np.ndarray:
        p, dev, B, N, keep = self._wav(wav)
        T = self.num_frames(N)
        out = np.empty((B, T, self.V), np.float32)
        _check(self.lib.suta_forward(self.handle, p, dev, int(normalize), B, N, _ptr(out)))
        return out

    def step(self, wav, hp: SutaHParams, normalize: bool = False):
        p, dev, B, N, keep = self._wav(wav)
        T = self.num_frames(N)
        out = np.empty((B, T, self.V), np.float32)
        loss = np.empty((B,), np.float32)
        _check(self.lib.suta_step(self.handle, p, dev, int(normalize), B, N, C.byref(hp.to_c()), _ptr(out),
                                  _ptr(loss)))
        return out, loss

    def step_ex(self, wav, hp: SutaHParams, repeat_inference: bool = True, normalize: bool = False,
                logits_device_ptr: Optional[int] = None):
        """suta_step_ex: one forward_and_adapt step; returns (logits (B,T,V) numpy or None when written to
        `logits_device_ptr`, loss (B,)).  repeat_inference=False returns the grad forward's logits."""
        p, dev, B, N, keep = self._wav(wav)
        T = self.num_frames(N)
        loss = np.empty((B,), np.float32)
        if logits_device_ptr is not None:
            out, lp, ldev = None, C.c_void_p(logits_device_ptr), 1
        else:
            out = np.empty((B, T, self.V), np.float32)
            lp, ldev = _ptr(out), 0
        _check(self.lib.suta_step_ex(self.handle, p, dev, int(normalize), B, N, C.byref(hp.to_c()),
                                     int(bool(repeat_inference)), lp, ldev, _ptr(loss)))
        return out, loss

    def adapt(self, wav, steps: int, hp: SutaHParams, record: Sequence[int] = (), normalize: bool = False,
              want_logits: bool = True, logits_device_ptr: Optional[int] = None):
        """Returns (logits {r: (B,T,V)} or None, ids {r: (B,T)}, T)."""
        p, dev, B, N, keep = self._wav(wav)
        T = self.num_frames(N)
        rec = list(record)
        crec = (C.c_int32 * max(1, len(rec)))(*rec)
        ids = np.empty((max(1, len(rec)), B, T), np.int32)
        frames = C.c_int64()
        if logits_device_ptr is not None:
            lp, ldev, logits = C.c_void_p(logits_device_ptr), 1, None
        elif want_logits and rec:
            logits = np.empty((len(rec), B, T, self.V), np.float32)
            lp, ldev = _ptr(logits), 0
        else:
            lp, ldev, logits = None, 0, None
        _check(self.lib.suta_adapt(self.handle, p, dev, int(normalize), B, N, steps, C.byref(hp.to_c()), crec,
                                   len(rec), lp, ldev, _ptr(ids) if rec else None, C.byref(frames)))
        lg = {r: logits[i] for i, r in enumerate(rec)} if logits is not None else None
        return lg, {r: ids[i] for i, r in enumerate(rec)}, frames.value

    def adapt_varlen(self, wavs, steps: int, hp: SutaHParams, record: Sequence[int] = (), normalize: bool = False,
                     want_logits: bool = True, lengths: Optional[Sequence[int]] = None, quantum: int = 1):
        """Ragged batch (suta_adapt_varlen): `wavs` is a list of 1-D waveforms, or a padded (B, stride)
        array / tensor with `lengths`.  Each utterance is adapted as if alone.  The layout length is the
        padded width (for a list: max length rounded up to `quantum` samples, so that batches of
        similar lengths share a layout and replay one captured step).  Returns
        (logits {r: [ (T_b, V) ]} or None, ids {r: [ (T_b,) ]}, [T_b])."""
        if lengths is None:
            arrs = [np.ascontiguousarray(w.detach().cpu().numpy() if hasattr(w, "detach") else w,
                                         dtype=np.float32).reshape(-1) for w in wavs]
            lengths = [a.size for a in arrs]
            width = -(-max(lengths) // max(1, quantum)) * max(1, quantum)
            pad = np.zeros((len(arrs), width), np.float32)
            for b, a in enumerate(arrs):
                pad[b, :a.size] = a
            wavs = pad
        p, dev, B, stride, keep = self._wav(wavs)
        ns = (C.c_int64 * B)(*[int(n) for n in lengths])
        T = self.num_frames(stride)
        rec = list(record)
        crec = (C.c_int32 * max(1, len(rec)))(*rec)
        ids = np.empty((max(1, len(rec)), B, T), np.int32)
        frames = (C.c_int64 * B)()
        logits = np.empty((len(rec), B, T, self.V), np.float32) if (want_logits and rec) else None
        _check(self.lib.suta_adapt_varlen(self.handle, p, dev, int(normalize), B, ns, stride, steps,
                                          C.byref(hp.to_c()), crec, len(rec),
                                          _ptr(logits) if logits is not None else None, 0,
                                          _ptr(ids) if rec else None, frames))
        tb = [int(frames[b]) for b in range(B)]
        lg = ({r: [logits[i, b, :tb[b]] for b in range(B)] for i, r in enumerate(rec)}
              if logits is not None else None)
        return lg, {r: [ids[i, b, :tb[b]] for b in range(B)] for i, r in enumerate(rec)}, tb

    def loss_grad(self, logits: np.ndarray, hp: SutaHParams):
        """Fused loss-and-grad kernel on logits of shape (B, T, V): returns (dlogits, loss)."""
        a = np.ascontiguousarray(logits, dtype=np.float32)
        if a.ndim == 2:
            a = a[None]
        d = np.empty_like(a)
        loss = np.empty((a.shape[0],), np.float32)
        _check(self.lib.suta_loss_grad(self.handle, _ptr(a), a.shape[0], a.shape[1], C.byref(hp.to_c()), _ptr(d),
                                       _ptr(loss)))
        return d, loss

    def get_param(self, slot: int, name: str) -> np.ndarray:
        shape = self.shapes[name]
        out = np.empty(shape, np.float32)
        _check(self.lib.suta_get_param(self.handle, slot, name.encode(), out.ctypes.data_as(C.POINTER(C.c_float)),
                                       out.size))
        return out

    def param_info(self, name: str, train_feature=True, bias_only=False):
        k, n = C.c_int32(), C.c_int64()
        _check(self.lib.suta_param_info(self.handle, name.encode(), int(train_feature), int(bias_only), C.byref(k),
                                        C.byref(n)))
        return k.value, n.value

    def trainable_names(self) -> List[str]:
        return [n for n in self.shapes if self.param_info(n)[1] > 0]

    def stream(self) -> int:
        return self.lib.suta_stream(self.handle) or 0

    def sync(self):
        _check(self.lib.suta_sync(self.handle))

    def set_timing(self, enable: bool):
        _check(self.lib.suta_set_timing(self.handle, int(enable)))

    def get_timing(self):
        ms = (C.c_double * 6)()
        n = (C.c_int64 * 6)()
        _check(self.lib.suta_get_timing(self.handle, ms, n))
        fams = ("gemm", "softmax", "norm", "elementwise", "loss", "adam")
        return {f: (ms[i], n[i]) for i, f in enumerate(fams)}

    TIMING_FAMILIES = ("gemm", "softmax", "norm", "elementwise", "loss", "adam", "frontend", "attention")

    def get_timing_ex(self):
        """Finer families (suta_get_timing_ex): {family: (ms, launches, algorithmic HBM bytes)};
        'gemm' here excludes the fused attention kernels ('attention') and 'norm' the conv front-end."""
        k = len(self.TIMING_FAMILIES)
        ms, n, by = (C.c_double * k)(), (C.c_int64 * k)(), (C.c_double * k)()
        _check(self.lib.suta_get_timing_ex(self.handle, k, ms, n, by))
        return {f: (ms[i], n[i], by[i]) for i, f in enumerate(self.TIMING_FAMILIES)}

    PRECISIONS = {"fp32": 0, "fp32-split-bf16": 1, "bf16": 2}

    def set_precision(self, mode: str):
        """'fp32' (exact fp32 MFMA) or 'fp32-split-bf16' (fp32-accurate 3-way bf16 split)."""
        _check(self.lib.suta_set_precision(self.handle, self.PRECISIONS[mode]))

    def set_graphs(self, enable: bool):
        _check(self.lib.suta_set_graphs(self.handle, int(enable)))

    LOOP_MODES = ("eager", "captured", "replayed")

    def graph_stats(self) -> dict:
        """How the last adapt call ran its loop ('eager' | 'captured' | 'replayed') and the engine's graph
        captures / launches so far (suta_get_graph_stats)."""
        m, c, n = C.c_int32(), C.c_int64(), C.c_int64()
        _check(self.lib.suta_get_graph_stats(self.handle, C.byref(m), C.byref(c), C.byref(n)))
        return {"last": self.LOOP_MODES[m.value], "captures": c.value, "launches": n.value}

    def set_census(self, enable: bool):
        """Start (clear) or stop the process-wide GEMM launch census (suta_set_census)."""
        _check(self.lib.suta_set_census(int(enable)))

    def get_census(self) -> Dict[str, int]:
        """{"<kernel> <BMxBN> z=<Z> split=<k> <form>": launches} since set_census(True) (and, with timing on,
        "ms|<shape>|n=<launches>": microseconds entries: get_gemm_shape_times)."""
        need = C.c_int64()
        self.lib.suta_get_census(None, 0, C.byref(need))
        buf = C.create_string_buffer(int(need.value))
        _check(self.lib.suta_get_census(buf, need.value, C.byref(need)))
        out = {}
        for ln in buf.value.decode().splitlines():
            key, n = ln.rsplit(" ", 1)
            out[key] = int(n)
        return out

    def get_gemm_shape_times(self) -> Dict[str, tuple]:
        """With the census and timing both on: {"M=.. N=.. K=.. z=.. <form> epi=..": (launches, total ms)}."""
        out = {}
        for k, v in self.get_census().items():
            if k.startswith("ms|"):
                _, shape, n = k.split("|")
                out[shape] = (int(n[2:]), v / 1000.0)
        return out
