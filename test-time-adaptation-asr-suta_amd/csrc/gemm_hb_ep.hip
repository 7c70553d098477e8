// Epilogue-class instantiations of the default 128 x 128 bf16-plane GEMM (gemm_hb_kernel): the generic kernel
// carries every epilogue flag combination and both bf16-C forms (~360 KB of code); a class kernel carries only
// its own flags and one C form.  Classes cover the linears of the bf16 path: bias / residual (QKV, out
// projection, FFN2, lm_head and the input gradients), bias + GELU + pre-activation store (FFN1), GELU' (the
// FFN2 input gradient); ragged row masks in each.
#include "gemm_kernels.h"
#include <cstdlib>

namespace {
constexpr int EM_A = EPI_BIAS | EPI_RESID | EPI_ROWMASK;
constexpr int EM_G = EPI_BIAS | EPI_GELU | EPI_STORE_PRE | EPI_ROWMASK;
constexpr int EM_D = EPI_DGELU | EPI_ROWMASK;

template <int EM>
void launch_class(const GemmParams& p, dim3 grid, hipStream_t st) {
    if (p.Cb) launch_hb<128, 128, 2, 32, 4, false, false, 1, EM>(p, grid, st);
    else launch_hb<128, 128, 2, 32, 4, false, false, 0, EM>(p, grid, st);
}
}  // namespace

bool gemm_run_hb_class(const GemmParams& p, dim3 grid, hipStream_t st) {
    static const int on = [] {  // SUTA_HB_EPI_CLASS=0: the generic kernel for every epilogue (A/B runs); read once
        const char* e = std::getenv("SUTA_HB_EPI_CLASS");
        return (e && atoi(e) == 0) ? 0 : 1;
    }();
    if (!on || p.segK > 0) return false;
    const int e = p.epi;
    if ((e & ~EM_A) == 0) launch_class<EM_A>(p, grid, st);
    else if ((e & ~EM_G) == 0) launch_class<EM_G>(p, grid, st);
    else if ((e & ~EM_D) == 0) launch_class<EM_D>(p, grid, st);
    else return false;
    return true;
}
