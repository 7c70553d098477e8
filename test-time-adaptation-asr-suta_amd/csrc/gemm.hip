// GEMM dispatcher: tile choice, split-K, precision mode -> kernel family (gemm_kernels.h).
#include "gemm_kernels.h"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>

namespace {

bool aligned16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

int g_force_tile = -1;  // test/bench override: 0=128x128 1=128x64 2=64x128 3=64x64
int g_nbuf = 3;  // 3 = LDS-DMA kernel where its preconditions hold (else the register-staged one)
int g_mode = 0;  // 0 = exact fp32 MFMA, 1 = x6 (fp32-accurate bf16 split), 2 = bf16 products

}  // namespace

void gemm_set_variant(int tile, int nbuf) {
    g_force_tile = tile;
    g_nbuf = nbuf;
}

// Kernel census (suta_set_census / suta_get_census): host-side count of GEMM launches per
// (kernel, tile, batch count, split count, operand form), so a test can assert which instantiation a
// layout reaches.  Counted when a launch is issued (eager or while a graph is captured), not on replay.
static std::mutex g_census_mu;
static std::map<std::string, long> g_census;
static std::atomic<bool> g_census_on{false};
// with engine timing on as well: per GEMM shape, the summed HIP-event time of its launches ("ms|<shape>|n=<n>"
// entries, value in microseconds)
static std::map<std::string, std::pair<double, long>> g_census_ms;

void gemm_census_enable(bool on) {
    std::lock_guard<std::mutex> lk(g_census_mu);
    g_census_on = on;
    g_census.clear();
    g_census_ms.clear();
}

bool gemm_census_is_on() { return g_census_on; }

void gemm_census_time(const std::string& shape, double ms) {
    std::lock_guard<std::mutex> lk(g_census_mu);
    auto& e = g_census_ms[shape];
    e.first += ms;
    e.second += 1;
}

std::string gemm_census_text() {
    std::lock_guard<std::mutex> lk(g_census_mu);
    std::string out;
    for (const auto& kv : g_census) out += kv.first + " " + std::to_string(kv.second) + "\n";
    for (const auto& kv : g_census_ms)
        out += "ms|" + kv.first + "|n=" + std::to_string(kv.second.second) + " " +
               std::to_string((long)(kv.second.first * 1000.0)) + "\n";
    return out;
}

// Each launch also counts one "grid <kernel> <BMxBN> gx=<column tiles> gy=<row tiles> z=<Z> split=<k>" entry, so
// a test can assert the tile grid a layout reaches (e.g. the 512 row tiles of 164 x 399 frames).
// and one "epi <kernel> <BMxBN> <epilogue flags>" entry (e.g. EPI_DELTA = 256 on hbx: the fused flash-backward delta ran).
static void census(const char* kernel, int BM, int BN, const GemmParams& p, int splits) {
    if (!g_census_on) return;
    char key[160], gkey[160], ekey[96];
    snprintf(key, sizeof key, "%s %dx%d z=%ld split=%d %s%s%s", kernel, BM, BN, (long)p.Z, splits, p.ta ? "T" : "N",
             p.tb ? "T" : "N", p.segK > 0 ? (p.segB ? " conv-seg" : " conv") : "");
    snprintf(gkey, sizeof gkey, "grid %s %dx%d gx=%d gy=%d z=%ld split=%d", kernel, BM, BN, (p.N + BN - 1) / BN,
             (p.M + BM - 1) / BM, (long)p.Z, splits);
    snprintf(ekey, sizeof ekey, "epi %s %dx%d %d", kernel, BM, BN, p.epi);
    std::lock_guard<std::mutex> lk(g_census_mu);
    ++g_census[key];
    ++g_census[gkey];
    ++g_census[ekey];
}

void gemm_set_mode(int mode) { g_mode = mode; }
int gemm_get_mode() { return g_mode; }

void gemm_init(GemmParams& p) {
    p = GemmParams{};
    p.Z = 1;
    p.zdiv = 1;
    p.alpha = 1.f;
    p.splits = 1;
    p.mode = g_mode;
}

// Tile choice: time ~ padded output area / eff, where eff is the tile's relative MFMA efficiency
// (measured with tools/gemm_bench on the SUTA shapes at 64 utterances: 128x128 wins every large
// GEMM despite its coarser tail; smaller tiles win where M or N is below ~128, e.g. attention and
// the 48-channel positional-conv groups); a grid with fewer tiles than CUs is charged as one full
// round of its tiles.
static int choose_tile(long M, long N, long Z, long K, int mode) {
    struct Cand {
        int bm, bn;
        double eff;
    };
    static const Cand glds[4] = {{128, 128, 1.0}, {128, 64, 0.93}, {64, 128, 0.92}, {64, 64, 0.85}};
    static const Cand x6[4] = {{128, 128, 1.0}, {128, 64, 0.9}, {64, 128, 0.9}, {64, 64, 0.75}};
    const Cand* cands = mode == 0 ? glds : x6;
    int best = 0;
    double bt = 1e300;
    for (int c = 0; c < 4; ++c) {
        const long tiles = ((M + cands[c].bm - 1) / cands[c].bm) * ((N + cands[c].bn - 1) / cands[c].bn) * Z;
        const double area = (double)cands[c].bm * cands[c].bn;
        const double t = std::max((double)tiles, 256.0) * area / cands[c].eff;
        if (t < bt * 0.999) {
            bt = t;
            best = c;
        }
    }
    (void)K;
    return best;
}

// bf16 mode (tools/gemm_bench, 64 utterances): the register-staged one-plane kernel beats the LDS-DMA
// fp32-staged one on every operand layout except transposed A (weight gradients, TN), and its
// 256x128 tile (wave tile 128x64: 1.3x fewer L2 bytes per flop) wins wherever the grid still fills
// whole rounds of 512 resident blocks (2 per CU): 420-430 TF on FFN1 / QKV / conv1 vs 360-390.
// Cost = rounds of 512 blocks x tile area / eff.
static int choose_tile_bf16(long M, long N, long Z, bool big) {
    struct Cand {
        int id, bm, bn;
        double eff;
    };
    static const Cand c[5] = {{0, 128, 128, 1.0}, {4, 256, 128, 1.12}, {1, 128, 64, 0.85}, {2, 64, 128, 0.85},
                              {3, 64, 64, 0.6}};
    int best = 0;
    double bt = 1e300;
    for (int i = 0; i < 5; ++i) {
        if (c[i].id == 4 && !big) continue;
        const long tiles = ((M + c[i].bm - 1) / c[i].bm) * ((N + c[i].bn - 1) / c[i].bn) * Z;
        const double t = (double)((tiles + 511) / 512) * c[i].bm * c[i].bn / c[i].eff;
        if (t < bt * 0.999) {
            bt = t;
            best = c[i].id;
        }
    }
    return best;
}

// bf16-plane GEMMs (tools/hb_bench, C4 linears at M = 25536): 128x128 with two LDS stages wins every
// shape (460-660 TF vs 370-570 for 256x128 at one block per CU); smaller tiles only for small grids.
static int choose_tile_hb(long M, long N, long Z) {
    struct Cand {
        int id, bm, bn;
        double eff;
    };
    static const Cand c[4] = {{0, 128, 128, 1.0}, {1, 128, 64, 0.85}, {2, 64, 128, 0.85}, {3, 64, 64, 0.6}};
    int best = 0;
    double bt = 1e300;
    for (int i = 0; i < 4; ++i) {
        const long tiles = ((M + c[i].bm - 1) / c[i].bm) * ((N + c[i].bn - 1) / c[i].bn) * Z;
        const double t = (double)((tiles + 511) / 512) * c[i].bm * c[i].bn / c[i].eff;
        if (t < bt * 0.999) {
            bt = t;
            best = c[i].id;
        }
    }
    return best;
}

// 256 x 256 slice-ring bf16-plane kernel (gemm_hbx.hip, v_mfma_f32_32x32x16_bf16; bitwise the 128 x 128 kernel's
// results: same MFMA products, same k order) for the linears on grids of at least one full round of 256 tiles.
// tools/hb_bench (C4 shapes at M = 164 x 399, same box; profiles/r4/hbx_epilogue_hb_bench.log): qkv 729 -> 875 TF,
// out-proj 597 -> 770, FFN1 759 -> 854, FFN2 866 -> 1065, dQKV 819 -> 1003.  The GELU / GELU' linears need its C^T
// epilogue with LDS-staged whole-line stores (SUTA_HBX_T=2): FFN1 (bias + GELU + bf16 pre) 603 -> 737 TF, FFN2 input
// gradient 611 -> 719; the column-per-lane epilogue (two-lane-pair dword stores, 2 rows per instruction) measured
// 595 / 627 and direct row-per-lane 16-B stores (32 rows per instruction) 515 / 625, so without the staged form
// they keep the 128 x 128 kernel.
// SUTA_HBX=0: off (A/B runs); 2: every eligible linear, any epilogue and grid (tests).
// batched (Z > 1) GEMMs -- the conv stack's per-utterance forward -- only on the four-phase form with the staged C^T
// epilogue (gemm_hbp_kernel rebases its operands per batch)
// (p.off32 already set: gemm_run_hbx refuses a batched GEMM without the 32-bit-offset epilogue, so one without it -- an
// operand over 4 GiB, or SUTA_EPI_FAST=0 -- must stay on the 128 x 128 kernel)
static bool hbx_batch_ok(const GemmParams& p) {
    const SutaSwitches& sw = suta_switches();
    return p.Z == 1 || (sw.hbx_form && sw.hbx_t == 2 && p.K % 64 == 0 && hbx_t_ok(p, true));
}

static bool use_hbx(const GemmParams& p) {
    const int mode = suta_switches().hbx;
    if (!mode || p.segK > 0 || p.K % 32 || p.K < 128 || (p.epi & (EPI_ACCUM | EPI_SMBWD)) || !hbx_batch_ok(p)) return false;
    if (mode == 2) return true;  // SUTA_HBX=2: every eligible linear (tests)
    if ((p.epi & (EPI_GELU | EPI_DGELU | EPI_STORE_PRE)) && !(suta_switches().hbx_t == 2 && hbx_t_ok(p, false)))
        return false;
    return (long)((p.M + 255) / 256) * ((p.N + 255) / 256) * p.Z >= 256;
}

// the conv stack's input gradients (conv-A rows, per-tap weight segments: config C4's conv-seg GEMMs, Z = B) on the
// four-phase 256 x 256 kernel's CONV form (gemm_hbx.hip hbp_conv_ok) on grids of at least one round of 256 tiles;
// SUTA_HBP_CONV=0 keeps them on the 128 x 128 kernel (A/B runs), SUTA_HBX=2 forces them on every eligible grid
static bool use_hbp_conv(const GemmParams& p) {
    const SutaSwitches& sw = suta_switches();
    if (!sw.hbx || !sw.hbp_conv || !hbp_conv_ok(p)) return false;
    if (sw.hbx == 2) return true;
    return (long)((p.M + 255) / 256) * ((p.N + 255) / 256) * p.Z >= 256;
}

// 32-bit epilogue offsets: M x ld elements of every operand the epilogue touches within 4 GiB
// (SUTA_EPI_FAST=0 in the call's switch snapshot: the general epilogue everywhere, for A/B runs)
static int epilogue_off32(const GemmParams& p) {
    const int fast = suta_switches().epi_fast;
    const double lim = 4294967295.0 - 1024.0;
    auto fits = [&](long ld, double esz) { return (double)p.M * (double)std::max(ld, (long)p.N) * esz < lim; };
    return fits(p.ldc, 4) && (!(p.epi & EPI_RESID) || fits(p.ldr, 4)) &&
           (!(p.epi & (EPI_DGELU | EPI_SMBWD)) || fits(p.ldaux, 4)) && (!(p.epi & EPI_STORE_PRE) || fits(p.ldc2, 4)) &&
           (!(p.epi & EPI_DELTA) || fits(p.ldo, 4)) && (!p.Cb || fits(p.ldcb, 2)) && p.ldc >= 0 && p.ldr >= 0 &&
           p.ldaux >= 0 && p.ldc2 >= 0 && p.ldcb >= 0 && p.ldo >= 0 && fast;
}

bool gemm_hbx_t_selected(const GemmParams& p0) {
    GemmParams p = p0;
    p.off32 = epilogue_off32(p);
    const bool hb = p.mode == 2 && p.Ab && p.Bb && !p.ta && p.segK == 0;
    return hb && g_force_tile < 0 && use_hbx(p) && suta_switches().hbx_t && hbx_t_ok(p, true);
}

void gemm_launch(GemmParams p, hipStream_t st, float* ws, long ws_floats) {
    if (p.M <= 0 || p.N <= 0 || p.Z <= 0) return;
    const int second = ((p.epi & EPI_RESID) != 0) + ((p.epi & EPI_ACCUM) != 0) + ((p.epi & EPI_SMBWD) != 0);
    if (second > 1 || ((p.epi & EPI_SMBWD) && p.epi != EPI_SMBWD))
        throw std::invalid_argument("gemm epilogue: RESID / ACCUM / SMBWD are mutually exclusive");
    auto vec_ok = [](const float* base, long ld, long s0, long s1) {
        return aligned16(base) && (ld % 4 == 0) && (s0 % 4 == 0) && (s1 % 4 == 0);
    };
    p.va = vec_ok(p.A, p.lda, p.sA0, p.sA1) && (p.segK == 0 || p.segK % 4 == 0);
    p.vb = vec_ok(p.B, p.ldb, p.sB0, p.sB1) && (!p.segB || (p.sBseg % 4 == 0 && p.segK % 4 == 0));

    const bool glds_ok = p.va && p.vb && (p.ta || p.K % 4 == 0) && (!p.tb || p.K % 4 == 0);
    const bool hbt = p.mode == 2 && p.Ab && p.Bb && p.ta && !p.tb;  // MN-contiguous bf16 planes (gemm_hbt_kernel)
    const bool hb = p.mode == 2 && p.Ab && p.Bb && !p.ta;            // k-contiguous bf16 planes (gemm_hb_kernel)
    if (p.mode == 2 && p.Ab && p.Bb && !hb && !hbt)
        throw std::invalid_argument("gemm: bf16 planes: A and B both k-contiguous ([M][K], [N][K]) or both MN-contiguous");
    if (hbt && (p.M % 8 || p.N % 8 || p.ldab % 8 || p.ldbb % 8 || !aligned16(p.Ab) || !aligned16(p.Bb) || p.Cb ||
                ((p.sA0 | p.sA1 | p.sB0 | p.sB1) % 8)))
        throw std::invalid_argument("gemm: MN-contiguous bf16 planes need M, N, ld, batch strides % 8 == 0, 16-B alignment");
    if (p.Cb && (!hb || (p.Z != 1 && (p.sCb1 % 4 || p.zdiv != 1)) || (reinterpret_cast<uintptr_t>(p.Cb) & 7)))
        throw std::invalid_argument("gemm: a bf16 output plane needs the bf16-plane kernel, 8-B alignment (Z > 1: sCb1 % 4 == 0)");
    if (hb && (p.K % 8 || p.ldab % 8 || p.ldbb % 8 || !aligned16(p.Ab) || !aligned16(p.Bb) ||
               (p.Z > 1 && ((p.sA0 | p.sA1 | p.sB0 | p.sB1) % 8))))
        throw std::invalid_argument("gemm: bf16 planes need K, ld and batch strides % 8 == 0 and 16-B alignment");
    const bool bf16_gbf = p.mode == 2 && glds_ok && p.ta;  // bf16 weight gradients: LDS-DMA fp32 stages
    p.off32 = epilogue_off32(p);  // before the tile choice: the 256 x 256 kernel's batched form needs it
    p.fgelu = suta_switches().fast_gelu;  // (the engine call's switch snapshot)
    if (p.preb && (!hb || !p.Cb || (p.ldc2 & 1)))
        throw std::invalid_argument("gemm: bf16 pre-activation operands need the bf16-plane kernel with a Cb plane, ldc2 even");
    if (hb && p.segK > 0 && (p.segK % 8 || p.pad < 0 || (p.segB && (p.sBseg % 8))))
        throw std::invalid_argument("gemm: conv-A bf16 planes need segK and the tap stride % 8 == 0");
    // conv weight gradients: the four-phase 256 x 256 TN form on grids that fill the chip (>= 256 tiles of 256^2; a
    // smaller grid keeps the 128 x 128 kernel with its split-K)
    const bool hbt4 = hbt && g_force_tile < 0 && hbt4_ok(p) &&
                      (suta_switches().hbt4 == 2 || (long)((p.M + 255) / 256) * ((p.N + 255) / 256) * p.Z >= 256);
    int tile = hbt ? (hbt4 ? 8 : 0)
               : (hb && p.segK > 0) ? (g_force_tile < 0 && use_hbp_conv(p) ? 8 : 0)
               : g_force_tile >= 0 ? g_force_tile
               : hb            ? (use_hbx(p) ? 8 : choose_tile_hb(p.M, p.N, p.Z))
               : p.mode == 2   ? choose_tile_bf16(p.M, p.N, p.Z, !bf16_gbf)
                               : choose_tile(p.M, p.N, p.Z, p.K, p.mode);
    if ((tile == 8 || tile == 9) && !(hb && p.K % 32 == 0 && p.K >= 128 && p.segK == 0 && (p.Z == 1 || (tile == 8 && hbx_batch_ok(p)))) &&
        !(tile == 8 && hb && p.segK > 0 && hbp_conv_ok(p)) && !(tile == 8 && hbt))
        tile = 0;
    if (tile == 6 || tile == 7) tile = 0;  // (the removed 256 x 256 ping-pong and 160 x 128 tiles: DESIGN.md 8)
    // tiles 0 = 128x128, 1 = 128x64, 2 = 64x128, 3 = 64x64; bf16 mode also 4 = 256x128, 5 = 128x256
    // 8 / 9: the 256 x 256 slice-ring bf16-plane kernel (gemm_hbx.hip) on v_mfma_f32_32x32x16_bf16 / 16x16x32
    const bool big = tile == 4 || tile == 8 || tile == 9;
    const int BM = big ? 256 : (tile == 0 || tile == 1 || tile == 5) ? 128 : 64;
    const int BN = (tile == 5 || tile == 8 || tile == 9) ? 256 : (tile == 0 || tile == 2 || tile == 4) ? 128 : 64;
    const int gx = (p.N + BN - 1) / BN, gy = (p.M + BM - 1) / BM;
    const long blocks = (long)gx * gy * p.Z;

    // split-K when the grid cannot fill 256 CUs and K is long
    int splits = 1;
    // (the split-K reduce has no bf16 pre store and no batched bf16 C plane)
    if (ws && suta_switches().splitk && p.K >= 1024 && blocks < 256 && tile != 8 && tile != 9 && !p.preb &&
        !(p.Cb && p.Z > 1)) {
        splits = (int)std::min<long>(16, (512 + blocks - 1) / blocks);
        while (splits > 1 && (long)splits * p.Z * p.M * (long)p.N > ws_floats) --splits;
        splits = std::min(splits, std::max(1, (p.K + 255) / 256));  // >= 256 K per split
    }
    p.kchunk = splits > 1 ? (((p.K + splits - 1) / splits + BK - 1) / BK) * BK : p.K;
    if (splits > 1) splits = (p.K + p.kchunk - 1) / p.kchunk;
    p.splits = splits;
    p.ws = ws;
    if ((p.epi & EPI_DELTA) && !(tile == 8 && suta_switches().hbx_t && hbx_t_ok(p, true)))
        throw std::invalid_argument("gemm: EPI_DELTA needs the 256 x 256 bf16-plane kernel's C^T epilogue (gemm_hbx_t_selected)");
    {
        // tile order (xcd_tile): n-fastest by default (m-fastest and other band widths measured 1-4 % slower on the
        // fp32 linears).  bf16-plane GEMMs: bands of 8 tile rows (N >= 2048) or 4 walked column by column keep both operand
        // panels L2-resident (tools/hb_bench, M = 25 536: qkv 543 -> 598 TF, ffn1 525 -> 590, the N = 1024
        // shapes within +-2 %); the fp32 kernels measured neutral and keep the n-fastest order
        p.order = 0;
        if (hb && splits == 1) p.order = gx >= 16 ? 8 : 4;
        // fp32 linears with >= 16 column tiles (QKV, FFN1 and their input-gradient GEMMs): their weight panels do
        // not stay in an XCD's 4 MB L2 across a band of rows in n-fastest order; bands of 8 tile rows walked
        // column by column halve their HBM reads (FFN1 forward 1.43 -> 0.72 GB per launch, PMC) at equal time
        // (37.05 vs 37.13 utt/s, within noise); narrow GEMMs (6 column tiles) keep the n-fastest order, which
        // reads less for them
        if (!hb && p.mode == 0 && splits == 1 && p.Z == 1 && gx >= 16) p.order = 8;
    }
    dim3 grid(gx, gy, p.Z * splits);
    if (hbt && tile == 8) {
        census("hbt4", BM, BN, p, splits);
        gemm_run_hbt4(p, grid, st);
    } else if (hbt) {
        census("hbt", BM, BN, p, splits);
        gemm_run_hbt(p, grid, st);
    } else if (hb) {
        // SUTA_HB_NS: stage variant of the 128 x 128 bf16-plane kernel (A/B runs; 2 default), read once (thread-safe)
        static const int hbns = [] {
            const char* ev = std::getenv("SUTA_HB_NS");
            return ev ? std::max(2, atoi(ev)) : 2;
        }();
        const int ns = g_force_tile >= 0 ? g_nbuf : (tile == 0 ? hbns : 2);
        if (tile == 8 || tile == 9) {
            census(tile == 8 ? "hbx" : "hbx16", BM, BN, p, splits);
            gemm_run_hbx(tile == 8 ? 1 : 2, p, grid, st);
        } else {
            census("hb", BM, BN, p, splits);
            gemm_run_hb(tile, ns, p, grid, st);
        }
    } else if (p.mode == 2) {
        // bf16: register-staged one-plane kernel; weight gradients (and benchmark variants 3 / 8) on
        // register-converted LDS-DMA stages (8 = BK64 x 2)
        const bool gbf = glds_ok && tile < 4 && (g_force_tile >= 0 ? (g_nbuf == 3 || g_nbuf == 8) : bf16_gbf);
        census(gbf ? "gbf" : "x6_1plane", BM, BN, p, splits);
        if (gbf) gemm_run_gbf(g_nbuf == 8, 1, tile, p, grid, st);
        else gemm_run_x6(tile, 0, 1, p, grid, st);
    } else if (p.mode == 1 && glds_ok && g_nbuf >= 9) {
        // x6 with register splits on LDS-DMA stages (benchmark variants 9 = BK32 x 2, 10 = BK64 x 2)
        census("gbf_x6", BM, BN, p, splits);
        gemm_run_gbf(g_nbuf == 10, 6, tile, p, grid, st);
    } else if (p.mode == 1) {
        // x6 planes: g_nbuf 2 -> BK 16 double-buffered; else BK 32 single LDS stage
        census("x6", BM, BN, p, splits);
        gemm_run_x6(tile, g_nbuf == 2, 3, p, grid, st);
    } else if (g_nbuf >= 3 && glds_ok) {
        // LDS-DMA variants: 3 = BK32 x 2 stages, 4 = BK16 x 4, 5 = BK16 x 3, 6 = BK32 x 3, 7 = BK64 x 2
        census("glds", BM, BN, p, splits);
        gemm_run_glds(g_nbuf, tile, p, grid, st);
    } else {
        census("f32", BM, BN, p, splits);
        gemm_run_f32(tile, g_nbuf == 2 ? 2 : 1, p, grid, st);
    }
    if (splits > 1) {
        const long MN = (long)p.M * p.N;
        const int gxr = (int)std::min<long>(1024, (MN + 255) / 256);
        hipLaunchKernelGGL(gemm_splitk_reduce, dim3(gxr, p.Z), dim3(256), 0, st, p);
    }
}
