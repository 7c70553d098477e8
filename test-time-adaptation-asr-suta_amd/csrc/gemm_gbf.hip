// LDS-DMA stages + register bf16 conversion: bf16 GEMM (1 product) and the register-split x6 (6 products).
#include "gemm_kernels.h"

void gemm_run_gbf(int bk64, int nprod, int tile, const GemmParams& p, dim3 grid, hipStream_t st) {
    if (nprod == 1) {
        if (bk64) launch_gbf_tile<64, 2, 1>(tile, p, grid, st);
        else launch_gbf_tile<32, 2, 1>(tile, p, grid, st);
    } else {
        if (bk64) launch_gbf_tile<64, 2, 6>(tile, p, grid, st);
        else launch_gbf_tile<32, 2, 6>(tile, p, grid, st);
    }
}
