"""Calibration: vendor BLAS (torch.mm -> hipBLASLt/rocBLAS) fp32 throughput on the SUTA GEMM shapes."""
import time
import torch

SHAPES = {  # name: (M, N, K)
    "ffn1_fwd": (25536, 3072, 768), "qkv_fwd": (25536, 2304, 768), "ffn2_fwd": (25536, 768, 3072),
    "oproj_fwd": (25536, 768, 768), "conv1_fwd_per_utt_x16": (16 * 12800, 512, 1536),
}


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    for name, (M, N, K) in SHAPES.items():
        a = torch.randn(M, K, device="cuda")
        b = torch.randn(K, N, device="cuda")
        for _ in range(3):
            torch.mm(a, b)
        torch.cuda.synchronize()
        it = 20
        t0 = time.perf_counter()
        for _ in range(it):
            torch.mm(a, b)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / it
        print(f"{name:24s} M={M} N={N} K={K}  {dt*1e3:.3f} ms  {2*M*N*K/dt/1e12:.1f} TF", flush=True)


if __name__ == "__main__":
    main()
