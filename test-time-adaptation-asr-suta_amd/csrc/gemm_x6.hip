// Register-staged bf16-plane GEMM family: x6 (3 planes, 6 products) and its one-plane bf16 form.
#include "gemm_kernels.h"

void gemm_run_x6(int tile, int bk16, int npl, const GemmParams& p, dim3 grid, hipStream_t st) {
    if (npl == 1) {
        // bf16 big tiles (4 = 256x128, 5 = 128x256; wave tile 128x64 / 64x128): 1.3x fewer L2 bytes per flop
        if (tile == 4) launch_x6<256, 128, 32, 1, 1>(p, grid, st);
        else if (tile == 5) launch_x6<128, 256, 32, 1, 1>(p, grid, st);
        else if (tile == 0) launch_x6<128, 128, 32, 1, 1>(p, grid, st);
        else if (tile == 1) launch_x6<128, 64, 32, 1, 1>(p, grid, st);
        else if (tile == 2) launch_x6<64, 128, 32, 1, 1>(p, grid, st);
        else launch_x6<64, 64, 32, 1, 1>(p, grid, st);
    } else if (bk16) {
        if (tile == 0) launch_x6<128, 128, 16, 2>(p, grid, st);
        else if (tile == 1) launch_x6<128, 64, 16, 2>(p, grid, st);
        else if (tile == 2) launch_x6<64, 128, 16, 2>(p, grid, st);
        else launch_x6<64, 64, 16, 2>(p, grid, st);
    } else {
        if (tile == 0) launch_x6<128, 128, 32, 1>(p, grid, st);
        else if (tile == 1) launch_x6<128, 64, 32, 1>(p, grid, st);
        else if (tile == 2) launch_x6<64, 128, 32, 1>(p, grid, st);
        else launch_x6<64, 64, 32, 1>(p, grid, st);
    }
}
