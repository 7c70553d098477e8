// Register-staged fp32 MFMA GEMM family (operands that are not 16-B aligned / k-contiguous with K % 4).
#include "gemm_kernels.h"

void gemm_run_f32(int tile, int nbuf, const GemmParams& p, dim3 grid, hipStream_t st) {
    if (nbuf == 2) {
        if (tile == 0) launch_tile<128, 128, 2>(p, grid, st);
        else if (tile == 1) launch_tile<128, 64, 2>(p, grid, st);
        else if (tile == 2) launch_tile<64, 128, 2>(p, grid, st);
        else launch_tile<64, 64, 2>(p, grid, st);
        return;
    }
    if (tile == 0) launch_tile<128, 128, 1>(p, grid, st);
    else if (tile == 1) launch_tile<128, 64, 1>(p, grid, st);
    else if (tile == 2) launch_tile<64, 128, 1>(p, grid, st);
    else launch_tile<64, 64, 1>(p, grid, st);
}
