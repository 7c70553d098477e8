"""Algorithmic work per adapted utterance.

FLOPs_alg(N, S) = (S+1) * F(N) + S * B(N): the minimal schedule, 2 flops per MAC, GEMM-shaped
ops only (convs, linears, attention products).  Redundant re-forwards of the reference
schedule are not credited.
"""
from .config import frame_lengths


def forward_flops(cfg: dict, n_samples: int) -> float:
    L = frame_lengths(cfg, n_samples)
    T = L[-1]
    H, F, NL, V = cfg["hidden_size"], cfg["intermediate_size"], cfg["num_hidden_layers"], cfg["vocab_size"]
    C = cfg["conv_dim"]
    conv = 0.0
    for i, (c, k) in enumerate(zip(C, cfg["conv_kernel"])):
        cin = 1 if i == 0 else C[i - 1]
        conv += 2.0 * c * cin * k * L[i]
    proj = 2.0 * T * C[-1] * H
    G, K = cfg["num_conv_pos_embedding_groups"], cfg["num_conv_pos_embeddings"]
    pos = 2.0 * T * (H // G) ** 2 * K * G
    lin = NL * T * (8.0 * H * H + 4.0 * H * F)
    att = NL * 4.0 * T * T * H
    head = 2.0 * T * H * V
    return conv + proj + pos + lin + att + head


def backward_flops(cfg: dict, n_samples: int) -> float:
    L = frame_lengths(cfg, n_samples)
    T = L[-1]
    H, F, NL, V = cfg["hidden_size"], cfg["intermediate_size"], cfg["num_hidden_layers"], cfg["vocab_size"]
    C = cfg["conv_dim"]
    head = 2.0 * T * H * V                           # dX only
    lin = NL * T * (8.0 * H * H + 4.0 * H * F)       # dX only (frozen weights)
    att = 2.0 * NL * 4.0 * T * T * H                 # dS, dQ, dK, dV
    G, K = cfg["num_conv_pos_embedding_groups"], cfg["num_conv_pos_embeddings"]
    pos = 2.0 * T * (H // G) ** 2 * K * G            # dX only
    proj = 2.0 * (2.0 * T * C[-1] * H)               # dW + dX
    conv = 0.0
    for i, (c, k) in enumerate(zip(C, cfg["conv_kernel"])):
        cin = 1 if i == 0 else C[i - 1]
        f = 2.0 * c * cin * k * L[i]
        conv += f if i == 0 else 2.0 * f             # conv0: dW only; conv1..: dW + dX
    return head + lin + att + pos + proj + conv


def suta_flops(cfg: dict, n_samples: int, steps: int) -> float:
    return (steps + 1) * forward_flops(cfg, n_samples) + steps * backward_flops(cfg, n_samples)


def reference_schedule_flops(cfg: dict, n_samples: int, steps: int) -> float:
    """What the reference loop executes per utterance: a vanilla forward, then per step a grad forward,
    a backward and a no-grad re-inference forward (main.py:172-215, 330-348): (2S+1) F + S B."""
    return (2 * steps + 1) * forward_flops(cfg, n_samples) + steps * backward_flops(cfg, n_samples)


def kernel_base(name: str) -> str:
    """Base name of a kernel as rocprofv3 tables spell it, mangled or demangled, template arguments dropped:
    '_ZN12_GLOBAL__N_122flash_fwd_bf16p_kernelILi4EEEvPKDF16b...' and
    'void (anonymous namespace)::flash_fwd_bf16p_kernel<4>(...)' -> 'flash_fwd_bf16p_kernel' (the PMC / trace
    reductions key kernel families by this name)."""
    if name.startswith("_Z"):
        i = 3 if name.startswith("_ZN") else 2
        idents = []
        while i < len(name) and name[i].isdigit():
            j = i
            while j < len(name) and name[j].isdigit():
                j += 1
            n = int(name[i:j])
            idents.append(name[j:j + n])
            i = j + n
        return idents[-1] if idents else name
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].strip()
