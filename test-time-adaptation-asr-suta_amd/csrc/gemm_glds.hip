// LDS-DMA fp32 MFMA GEMM family (the default exact path).
#include "gemm_kernels.h"

void gemm_run_glds(int variant, int tile, const GemmParams& p, dim3 grid, hipStream_t st) {
    if (variant == 7) launch_glds_tile<64, 2>(tile, p, grid, st);
    else if (variant == 4) launch_glds_tile<16, 4>(tile, p, grid, st);
    else if (variant == 5) launch_glds_tile<16, 3>(tile, p, grid, st);
    else if (variant == 6) launch_glds_tile<32, 3>(tile, p, grid, st);
    else launch_glds_tile<32, 2>(tile, p, grid, st);
}
