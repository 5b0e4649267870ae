// gemm.hip — GEMM entry points (alignn_gemm_f32 / _workspace / _path): plan, routing to the tiled, bf16
// row-streaming (gemm_rows.hip) and bf16 weight-gradient (gemm_wgrad.hip) kernels, split-K reduce and
// the column sums.  The tiled kernels live in gemm_tile.h, instantiated per
// arithmetic in gemm_tile_p0/1.hip.
#include <cstring>

#include "gemm_tile.h"

namespace alignn {

__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmParams p) {
  const int64_t total = (p.reduce_batch ? 1 : p.batch) * p.M * p.N;
  const int64_t all = total + (p.rsum ? p.M : 0);   // then the row sums' partials (batch 1)
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < all; i += (int64_t)gridDim.x * blockDim.x) {
    if (i >= total) {   // rowsum[m]: the split partials in the same eight-chain order
      const int64_t m = i - total;
      const float* w = p.ws + (int64_t)p.split_k * total + m;
      float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      int k = 0;
      for (; k + 7 < p.split_k; k += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += w[(int64_t)(k + j) * p.M];
      }
      for (int j = 0; k < p.split_k; ++k, ++j) s[j] += w[(int64_t)k * p.M];
      p.rsum[m] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
      continue;
    }
    const int64_t col = i % p.N;
    const int64_t row = (i / p.N) % p.M;
    const int64_t b = i / (p.N * p.M);
    // eight independent chains (partial k goes to chain k % 8), combined in a fixed tree
    store_c(p, b, row, col, epilogue_value(p, b, row, col, splitk_sum(p, b, row, col)), p.cbf != 0);
  }
}


static bool aligned16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15u) == 0; }
static bool aligned8(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 7u) == 0; }

static int g_cus = 0;
static int device_cus() {
  if (g_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    g_cus = n;
  }
  return g_cus;
}

struct GemmPlan {
  int bm, bn, split, bk;
  int64_t kchunk;
};

// Automatic plan, fitted to a sweep of every product of the training step on MI355X
// (tools/gemm_bench.py, profiles/r01/v11_gemm_sweep.log; all tiles x stage depths x splits):
//  * tile 64x64 — it was the fastest tile for every one of the 52 shapes (these products are
//    latency-bound at 1-20 us; more, smaller workgroups hide more of it);
//  * split-K toward one workgroup per CU (tiles x split ~ CUs) when the product is long (K >= 512)
//    on fewer than 160 tiles, or its grid tiny (< 32 tiles); details at the rule below;
//  * 64-deep stages (a quarter of the global round trips) when a split is >= 512 deep on at most
//    one workgroup per CU; 16-deep otherwise (large grids keep more workgroups resident with them).
// Explicit tile / stage bits (tuning) override the choice.
static GemmPlan make_plan(int64_t M, int64_t N, int64_t Ktot, int64_t nb, int requested, int tile) {
  const int cus = device_cus();
  static const int cand[4][2] = {{128, 128}, {128, 64}, {64, 128}, {64, 64}};
  GemmPlan pl{64, 64, 1, 16, 0};
  const int shape = tile & 15;  // bits 16/32/128: stage depth, bit 64: bf16 compute
  if (shape >= 1 && shape <= 4) {
    pl.bm = cand[shape - 1][0];
    pl.bn = cand[shape - 1][1];
  }
  // bf16 long-K products (weight gradients over every row, M >= 128): 128 x 64 tiles, 32-deep
  // stages, two workgroups per CU (B = 256 bf16 sweep, profiles/r02/v20_gemm_sweep_b256_bf16.json:
  // M768 N256 K16020 38.7 vs 64.6 us, M256 N256 K184320 115 vs 129 us)
  const bool bf_long = (tile & ALIGNN_GEMM_BF16) && shape == 0 && !(tile & (ALIGNN_GEMM_BK16 | ALIGNN_GEMM_BK32 |
                       ALIGNN_GEMM_BK64)) && Ktot >= 4096 && M >= 128 && requested <= 0;
  if (bf_long) {
    pl.bm = 128;
    pl.bn = 64;
  }
  // bf16 products over many rows with a deep K (C3's dX += dQKVR Wb, M 15,360 x 256 x 1,024, and the
  // line graph's row-scattered M 16,020 x 256 x 768): 128 x 64 tiles, 32-deep stages — 44.3 vs 50.5 us
  // and 44.8 vs 46.0 us, the best of every tile x depth x split (profiles/r06/gemm_c3_big.log)
  const bool bf_deep = (tile & ALIGNN_GEMM_BF16) && shape == 0 && !bf_long && !(tile & (ALIGNN_GEMM_BK16 |
                       ALIGNN_GEMM_BK32 | ALIGNN_GEMM_BK64)) && requested <= 0 && M >= 8192 && N <= 256 && Ktot >= 512;
  if (bf_deep) {
    pl.bm = 128;
    pl.bn = 64;
  }
  const int64_t tiles = ((M + pl.bm - 1) / pl.bm) * ((N + pl.bn - 1) / pl.bn) * nb;
  int split = requested;
  if (bf_long) {
    split = (int)std::max<int64_t>(1, std::min<int64_t>((2 * cus + tiles / 2) / std::max<int64_t>(tiles, 1),
                                                         Ktot / 256));
  } else if (split <= 0) {
    split = 1;
    // round-2 sweep of every product of the B = 32 step (profiles/r02/v15_gemm_sweep.json): a grid
    // of >= 160 tiles is not split (M2580 N256 K768: 25.8 vs 29.9 us in two); long-K splits keep
    // >= 240-deep chunks (M64 N256 K1920 b4: 8 splits, not 16) and go to two workgroups per CU when
    // the chunks would be >= 1024 deep (M256 N256 K23040: 32 splits, 40 vs 51 us)
    if ((Ktot >= 512 && tiles < 160) || tiles < 32) {
      int64_t want = std::max<int64_t>(1, (cus + tiles / 2) / std::max<int64_t>(tiles, 1));
      if (Ktot >= 512 && Ktot / want >= 1024) want *= 2;
      // a grid of at most 4 tiles splits down to 16-deep chunks (round-4 sweep, gpurun_out r4g
      // gemm_sweep_c2.json: the heads' M32 N256 K545 24.6 -> 10.6 us in 32, M256 N36 K23040 30.9 -> 27.3)
      const int64_t maxs = std::max<int64_t>(1, Ktot / (tiles <= 4 ? 16 : (Ktot >= 512 ? 240 : 32)));
      split = (int)std::min(want, maxs);
    }
  }
  if (Ktot == 0) split = 1;
  int64_t kchunk = (Ktot + split - 1) / split;
  kchunk = (kchunk + BK - 1) / BK * BK;
  if (kchunk == 0) kchunk = BK;
  split = (int)((Ktot + kchunk - 1) / kchunk);
  if (split < 1) split = 1;
  pl.split = split;
  pl.kchunk = kchunk;
  if (bf_long || bf_deep) pl.bk = 32;
  else if (tile & ALIGNN_GEMM_BK64) pl.bk = 64;
  else if (tile & ALIGNN_GEMM_BK32) pl.bk = 32;
  else if (tile & ALIGNN_GEMM_BK16) pl.bk = 16;
  // 64-deep stages only for long chunks on at most one workgroup per CU (short-K products and
  // two-per-CU splits run faster 16-deep: M2580 N768 K256 18.3 vs 20.6 us, M1024 N256 K1920 23.3 vs 26.0)
  else pl.bk = ((kchunk >= 512 || (tiles <= 4 && kchunk >= 128)) && tiles * split <= (int64_t)cus) ? 64 : 16;
  return pl;
}

static bool plan_args(const AlignnGemmArgs* a, GemmPlan& pl, int64_t& ktot, int64_t& nb_out) {
  if (!a || a->M < 0 || a->N < 0 || a->K < 0 || a->batch < 1) return false;
  const bool rb = a->reduce_batch && a->batch > 1;
  ktot = rb ? a->K * a->batch : a->K;
  nb_out = rb ? 1 : a->batch;
  pl = make_plan(a->M, a->N, ktot, nb_out, a->split_k, a->tile);
  // a stage must not straddle two batch entries of a batch-reduced product, nor a split chunk
  if (rb && pl.bk > 64) pl.bk = 64;
  if (rb && (a->K % pl.bk != 0 || (pl.split > 1 && pl.kchunk % pl.bk != 0))) pl.bk = 16;
  return true;
}



// bf16 arithmetic through bf16 LDS images (gemm_tile.h arithmetic 2, bitwise equal to 1): forced on /
// off by ALIGNN_GEMM_LDS16 / ALIGNN_GEMM_NOLDS16; otherwise taken when A is k-contiguous.  C3 sweep
// (profiles/r04/v3_lds16_*): the products over rows (X·Wᵀ, dX) run 7-28 % faster, e.g. M 16,020 x 768 x
// 256 60.6 -> 44.6 us, M 15,360 x 1,024 x 256 70.2 -> 51.6; the weight gradients, whose A is
// row-contiguous and transposed into the image by 2-byte stores, 15-50 % slower (M 256 x 256 x 184,320
// 108.7 -> 138.1).  ALIGNN_GEMM_LDS16=0 in the environment (read once) turns the default off (A/B).
static bool lds16(const AlignnGemmArgs* a, bool akc) {
  static const bool env_off = [] {
    const char* e = std::getenv("ALIGNN_GEMM_LDS16");
    return e && std::atoi(e) == 0;
  }();
  if (a->rowsum) return false;   // the row sums read the fp32 stage images
  if (a->tile & ALIGNN_GEMM_NOLDS16) return false;
  if (a->tile & ALIGNN_GEMM_LDS16) return true;
  return akc && !env_off;
}

// The row-streaming kernel (gemm_rows.hip): bf16 arithmetic, K <= 256 (K % 4, % 8 for bf16 A), N a
// multiple of 256, batched without batch reduction (and then no mask), no split / row scatter / rowscale / rowsum, A k-contiguous 16-byte rows,
// fp32 W, row-major C / mask with 32-bit byte offsets; taken from ALIGNN_GEMM_ROWS_MIN_M rows up
// (read once; default 4096), at any M on request (ALIGNN_GEMM_ROWS), never with ALIGNN_GEMM_NOROWS.
// C3 step, same box (profiles/r05/v5_ab_gemm_rows.txt): 20,658 / 20,742 graphs/s without it,
// 21,720 / 21,598 from 32768 rows, 21,722 / 21,808 from 4096 (the 16k-row Q/K/V projections too).
void gemm_rows_launch(const GemmParams& p, int cus, hipStream_t s);
static int64_t rows_min_m() {
  static const int64_t v = [] {
    const char* e = std::getenv("ALIGNN_GEMM_ROWS_MIN_M");
    return e ? std::max<int64_t>(32, std::atoll(e)) : int64_t(4096);
  }();
  return v;
}
static bool rows_ok(const AlignnGemmArgs* a, int split) {
  if (a->rowsum || a->c_rows || a->rowscale) return false;
  if (!(a->tile & ALIGNN_GEMM_BF16) || (a->tile & ALIGNN_GEMM_NOROWS) || (a->tile & 15) != 0) return false;
  if (a->reduce_batch || split != 1 || (a->batch > 1 && a->mask)) return false;
  const bool abf = (a->tile & ALIGNN_GEMM_A_BF16) != 0, cbf = (a->tile & ALIGNN_GEMM_C_BF16) != 0;
  if (a->tile & ALIGNN_GEMM_B_BF16) return false;
  if (a->batch > 1 && (a->sab % (abf ? 8 : 4) || a->scb % 4)) return false;   // 16-byte aligned batch entries
  if (a->K < 1 || a->K > 256 || a->K % (abf ? 8 : 4) != 0) return false;
  if (a->N % 256 != 0 || a->M < ((a->tile & ALIGNN_GEMM_ROWS) ? 1 : rows_min_m())) return false;
  if (a->sak != 1 || a->sam % (abf ? 8 : 4) || (reinterpret_cast<uintptr_t>(a->A) & 15)) return false;
  if (a->scn != 1 || a->scm < a->N || a->scm % 4 || (reinterpret_cast<uintptr_t>(a->C) & (cbf ? 7 : 15))) return false;
  if (cbf && (a->beta != 0.f || a->mask)) return false;
  if (a->mask && (a->smk_n != 1 || a->smk_m < a->N || a->smk_m % 4 || (reinterpret_cast<uintptr_t>(a->mask) & 15)))
    return false;
  if ((a->M + 32) * std::max(a->scm, a->mask ? a->smk_m : 0) * 4 >= ((int64_t)1 << 31)) return false;
  return true;
}

// The per-head form of the row kernel (gemm_rows.hip gemm_heads_kernel): the S_h M_h^T / Sz_h M_h^T
// products (batch = 4 heads, N = 64 each, K = 256, rowscale x bias2, beta); same row floor and
// ALIGNN_GEMM_ROWS / _NOROWS switches as the row kernel.
void gemm_heads_launch(const GemmParams& p, int cus, hipStream_t s);
static bool heads_ok(const AlignnGemmArgs* a, int split, bool vecB) {
  if (!(a->tile & ALIGNN_GEMM_BF16) || (a->tile & ALIGNN_GEMM_NOROWS) || (a->tile & 15) != 0) return false;
  if (a->rowsum || a->c_rows || a->mask || a->reduce_batch || split != 1) return false;
  if (a->batch != 4 || a->N != 64 || a->K < 8 || a->K > 256 || a->K % 8) return false;
  if (a->M < ((a->tile & ALIGNN_GEMM_ROWS) ? 1 : rows_min_m())) return false;
  const bool abf = (a->tile & ALIGNN_GEMM_A_BF16) != 0;
  if ((a->tile & (ALIGNN_GEMM_B_BF16 | ALIGNN_GEMM_C_BF16)) || !vecB || a->sbk != 1) return false;
  if (a->sak != 1 || a->sam % (abf ? 8 : 4) || a->sab % (abf ? 8 : 4) || (reinterpret_cast<uintptr_t>(a->A) & 15)) return false;
  if (a->scn != 1 || a->scm % 4 || a->scb % 4 || (reinterpret_cast<uintptr_t>(a->C) & 15)) return false;
  if (a->rowscale && !a->bias2) return false;
  if ((a->M + 32) * a->scm * 4 >= ((int64_t)1 << 31)) return false;
  return true;
}

// The weight-gradient kernel (gemm_wgrad.hip): bf16 arithmetic, A = dY^T and B = X both stored
// row-major over the long K axis (sam == 1, sbn == 1; 16-byte rows), K >= 4096, batched or not (no
// batch reduction), no split
// request / row scatter / rowscale, M and N multiples of 4 (8 for bf16 storage) and >= 8; its partials
// go through the split-K workspace and reduce.  ALIGNN_GEMM_NOWGRAD turns it off (tests, A/B).
int64_t gemm_wgrad_split(int64_t M, int64_t N, int64_t K, int64_t batch, int cus, int64_t* rows_per);
void gemm_wgrad_launch(const GemmParams& p, int64_t S, int64_t rows_per, hipStream_t s);
static bool wgrad_ok(const AlignnGemmArgs* a) {
  static const bool env_off = [] {   // ALIGNN_GEMM_WGRAD=0 in the environment (read once): off (A/B)
    const char* e = std::getenv("ALIGNN_GEMM_WGRAD");
    return e && std::atoi(e) == 0;
  }();
  if (env_off || !(a->tile & ALIGNN_GEMM_BF16) || (a->tile & ALIGNN_GEMM_NOWGRAD) || (a->tile & 15) != 0) return false;
  if (a->tile & (ALIGNN_GEMM_BK16 | ALIGNN_GEMM_BK32 | ALIGNN_GEMM_BK64)) return false;
  if (a->reduce_batch || a->split_k > 0 || a->c_rows || a->rowscale || a->mask) return false;
  const bool abf = (a->tile & ALIGNN_GEMM_A_BF16) != 0, bbf = (a->tile & ALIGNN_GEMM_B_BF16) != 0;
  if (a->batch > 1 && (a->sab % (abf ? 8 : 4) || a->sbb % (bbf ? 8 : 4))) return false;   // 16-byte aligned entries
  // M >= 128: the per-head dM products (M = 64, batch 4) ran slower here than tiled (45-50 vs 38 us,
  // profiles/r05/v10_ab_gemm_batched.txt) — a 256-row output tile three-quarters empty
  if (a->K < 4096 || a->M < 128 || a->N < 8 || a->M % (abf ? 8 : 4) || a->N % (bbf ? 8 : 4)) return false;
  if (a->sam != 1 || a->sak < a->M || a->sak % (abf ? 8 : 4) || (reinterpret_cast<uintptr_t>(a->A) & 15)) return false;
  if (a->sbn != 1 || a->sbk < a->N || a->sbk % (bbf ? 8 : 4) || (reinterpret_cast<uintptr_t>(a->B) & 15)) return false;
  return true;
}


}  // namespace alignn

using namespace alignn;

extern "C" int64_t alignn_gemm_workspace(const AlignnGemmArgs* a) {
  GemmPlan pl;
  int64_t ktot, nb;
  if (!plan_args(a, pl, ktot, nb)) return -1;
  if (wgrad_ok(a)) {
    int64_t rp;
    const int64_t S = gemm_wgrad_split(a->M, a->N, a->K, a->batch, device_cus(), &rp);
    return S * a->batch * a->M * a->N + (a->rowsum ? S * a->M : 0);
  }
  return pl.split > 1 ? (int64_t)pl.split * nb * a->M * a->N + (a->rowsum ? (int64_t)pl.split * a->M : 0) : 0;
}

extern "C" int alignn_gemm_path(const AlignnGemmArgs* a) {
  GemmPlan pl;
  int64_t ktot, nb;
  if (!plan_args(a, pl, ktot, nb)) return -1;
  const bool vecB = a->sbk == 1 && a->sbn % 4 == 0 && a->sbb % 4 == 0 && (reinterpret_cast<uintptr_t>(a->B) & 15) == 0;
  return wgrad_ok(a) ? 3 : (rows_ok(a, pl.split) || heads_ok(a, pl.split, vecB)) ? 2 : 0;
}

extern "C" int alignn_gemm_f32(const AlignnGemmArgs* a, void* stream) {
  if (!a || a->M < 0 || a->N < 0 || a->K < 0 || a->batch < 1) {
    set_error("gemm: bad shape");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (a->M == 0 || a->N == 0) return ALIGNN_OK;
  if (a->rowscale && !a->bias2) {
    set_error("gemm: rowscale without bias2");
    return ALIGNN_E_BAD_SHAPE;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  GemmParams p;
  std::memset(&p, 0, sizeof p);  // defined padding bytes (plan.hip scans recorded struct words)
  p.M = a->M; p.N = a->N; p.K = a->K; p.batch = a->batch;
  p.A = a->A; p.sam = a->sam; p.sak = a->sak; p.sab = a->sab;
  p.B = a->B; p.sbk = a->sbk; p.sbn = a->sbn; p.sbb = a->sbb;
  p.C = a->C; p.scm = a->scm; p.scn = a->scn; p.scb = a->scb;
  p.bias = a->bias; p.sbias_b = a->sbias_b;
  p.rowscale = a->rowscale; p.srs_m = a->srs_m; p.srs_b = a->srs_b;
  p.bias2 = a->bias2; p.sb2_b = a->sb2_b;
  p.mask = a->mask; p.smk_m = a->smk_m; p.smk_n = a->smk_n;
  p.alpha = a->alpha; p.beta = a->beta; p.relu = a->relu;
  p.reduce_batch = a->reduce_batch && a->batch > 1;
  p.c_rows = a->c_rows;
  p.rsum = a->rowsum;
  if (a->rowsum && (a->batch != 1 || a->reduce_batch)) {
    set_error("gemm: rowsum needs batch == 1 without reduce_batch");
    return ALIGNN_E_UNSUPPORTED;
  }
  p.abf = (a->tile & ALIGNN_GEMM_A_BF16) ? 1 : 0;
  p.bbf = (a->tile & ALIGNN_GEMM_B_BF16) ? 1 : 0;
  p.cbf = (a->tile & ALIGNN_GEMM_C_BF16) ? 1 : 0;
  if (p.cbf && (a->beta != 0.f || a->mask)) {
    set_error("gemm: a bf16 C is write-only (no beta, no mask)");
    return ALIGNN_E_UNSUPPORTED;
  }
  if (p.reduce_batch && a->K % BK != 0) {
    set_error("gemm: reduce_batch needs K %% %d == 0 (K=%lld)", BK, (long long)a->K);
    return ALIGNN_E_UNSUPPORTED;
  }
  GemmPlan pl;
  int64_t Ktot, nbatch_out;
  plan_args(a, pl, Ktot, nbatch_out);
  // A is "k-contiguous" unless it is contiguous along m only.
  const bool akc = !(a->sam == 1 && a->sak != 1);
  const bool bkc = !(a->sbn == 1 && a->sbk != 1);
  // vector loads: four elements per load (16 bytes fp32, 8 bytes bf16), aligned
  const bool alA = p.abf ? aligned8(a->A) : aligned16(a->A), alB = p.bbf ? aligned8(a->B) : aligned16(a->B);
  p.vecA = akc ? (a->sak == 1 && a->sam % 4 == 0 && a->sab % 4 == 0 && alA)
               : (a->sak % 4 == 0 && a->sab % 4 == 0 && alA);
  p.vecB = bkc ? (a->sbk == 1 && a->sbn % 4 == 0 && a->sbb % 4 == 0 && alB)
               : (a->sbk % 4 == 0 && a->sbb % 4 == 0 && alB);
  p.kchunk = pl.kchunk;
  p.split_k = pl.split;
  p.ws = a->workspace;
  const int64_t ws_need = (int64_t)pl.split * nbatch_out * a->M * a->N + (a->rowsum ? (int64_t)pl.split * a->M : 0);
  if (pl.split > 1 && (!a->workspace || a->workspace_elems < ws_need)) {
    set_error("gemm: split_k=%d needs %lld workspace floats", pl.split, (long long)ws_need);
    return ALIGNN_E_WORKSPACE;
  }
  if (wgrad_ok(a)) {
    int64_t rp;
    const int64_t S = gemm_wgrad_split(a->M, a->N, a->K, a->batch, device_cus(), &rp);
    const int64_t need = S * a->batch * a->M * a->N + (a->rowsum ? S * a->M : 0);
    if (!a->workspace || a->workspace_elems < need) {
      set_error("gemm: the weight-gradient kernel needs %lld workspace floats", (long long)need);
      return ALIGNN_E_WORKSPACE;
    }
    p.split_k = (int)S;
    gemm_wgrad_launch(p, S, rp, s);
    ALIGNN_LAUNCH_CHECK("wgrad_kernel");
    const int64_t total = a->batch * a->M * a->N + (a->rowsum ? a->M : 0);
    launch(splitk_reduce_kernel, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 4096)), dim3(256), 0, s, p);
    ALIGNN_LAUNCH_CHECK("splitk_reduce_kernel");
    return ALIGNN_OK;
  }
  if (heads_ok(a, pl.split, p.vecB)) {
    gemm_heads_launch(p, device_cus(), s);
    ALIGNN_LAUNCH_CHECK("gemm_heads_kernel");
    return ALIGNN_OK;
  }
  if (rows_ok(a, pl.split)) {
    gemm_rows_launch(p, device_cus(), s);
    ALIGNN_LAUNCH_CHECK("gemm_rows_kernel");
    return ALIGNN_OK;
  }
  const int64_t tiles = ((a->M + pl.bm - 1) / pl.bm) * ((a->N + pl.bn - 1) / pl.bn);
  dim3 grid((unsigned)tiles, 1, (unsigned)(nbatch_out * pl.split));
  const bool np = (a->tile & ALIGNN_GEMM_NOPIPE) != 0;
  if ((a->tile & ALIGNN_GEMM_BF16) && lds16(a, akc)) gemm_tiled_launch<2>(p, pl.bm, pl.bn, akc, bkc, grid, pl.bk, np, s);
  else if (a->tile & ALIGNN_GEMM_BF16) gemm_tiled_launch<1>(p, pl.bm, pl.bn, akc, bkc, grid, pl.bk, np, s);
  else gemm_tiled_launch<0>(p, pl.bm, pl.bn, akc, bkc, grid, pl.bk, np, s);
  ALIGNN_LAUNCH_CHECK("gemm_f32_kernel");
  if (pl.split > 1) {
    int64_t total = nbatch_out * a->M * a->N + (a->rowsum ? a->M : 0);
    int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
    launch(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, s, p);
    ALIGNN_LAUNCH_CHECK("splitk_reduce_kernel");
  }
  return ALIGNN_OK;
}

// -------------------------------------------------------------------------------------------
// Column sums (bias gradients), two fixed-order stages.
//   stage 1: block (R, strip) = 4 row-lanes x 64 columns; each thread sums rows r0+ty, r0+ty+4, ...
//            of its row chunk (4 independent loads in flight), LDS-reduces the 4 row-lanes and
//            writes one partial per (chunk, column).
//   stage 2: one block per 64-column strip sums the R partials the same way.
// -------------------------------------------------------------------------------------------
namespace alignn {
// BF: X holds bf16 elements (the bias gradient of a Linear whose output gradient is stored in bf16)
template <bool BF = false>
__global__ __launch_bounds__(256) void colsum_stage1(const float* __restrict__ X, int64_t M, int64_t N, int64_t ldx,
                                                     int64_t rows_per, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.y * 64 + tx;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per, r1 = min(M, r0 + rows_per);
  auto at = [&](int64_t i) { return BF ? bf_at(X, i) : X[i]; };
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (col < N) {
    int64_t r = r0 + ty;
    for (; r + 12 < r1; r += 16) {
      s0 += at(r * ldx + col);
      s1 += at((r + 4) * ldx + col);
      s2 += at((r + 8) * ldx + col);
      s3 += at((r + 12) * ldx + col);
    }
    for (; r < r1; r += 4) s0 += at(r * ldx + col);
  }
  red[ty][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty == 0 && col < N) part[(int64_t)blockIdx.x * N + col] = (red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]);
}

// Weighted column sums of two row-strided matrices, per-row weights per column group of width C:
//   out[j] (+)= sum_r W1[r, j / C] X1[r, j] + W2[r, j / C] X2[r, j]
// (the w-bar gradient of a TransformerConv with a folded edge projection: per head h,
// sum_n Q_nh sigz_nh + dout_nh sumA_nh).  Same two fixed-order stages as colsum.
__global__ __launch_bounds__(256) void wcolsum2_stage1(const float* __restrict__ X1, int64_t ld1,
                                                       const float* __restrict__ W1, int64_t lw1,
                                                       const float* __restrict__ X2, int64_t ld2,
                                                       const float* __restrict__ W2, int64_t lw2, int64_t M,
                                                       int64_t N, int C, int64_t rows_per, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t col = (int64_t)blockIdx.y * 64 + tx;
  const int64_t h = col / C;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per, r1 = min(M, r0 + rows_per);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (col < N) {
    int64_t r = r0 + ty;
    for (; r + 12 < r1; r += 16) {
      s0 = fmaf(W1[r * lw1 + h], X1[r * ld1 + col], fmaf(W2[r * lw2 + h], X2[r * ld2 + col], s0));
      s1 = fmaf(W1[(r + 4) * lw1 + h], X1[(r + 4) * ld1 + col], fmaf(W2[(r + 4) * lw2 + h], X2[(r + 4) * ld2 + col], s1));
      s2 = fmaf(W1[(r + 8) * lw1 + h], X1[(r + 8) * ld1 + col], fmaf(W2[(r + 8) * lw2 + h], X2[(r + 8) * ld2 + col], s2));
      s3 = fmaf(W1[(r + 12) * lw1 + h], X1[(r + 12) * ld1 + col],
                fmaf(W2[(r + 12) * lw2 + h], X2[(r + 12) * ld2 + col], s3));
    }
    for (; r < r1; r += 4) s0 = fmaf(W1[r * lw1 + h], X1[r * ld1 + col], fmaf(W2[r * lw2 + h], X2[r * ld2 + col], s0));
  }
  red[ty][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty == 0 && col < N) part[(int64_t)blockIdx.x * N + col] = (red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]);
}
}  // namespace alignn

static int colsum(const float* X, int64_t M, int64_t N, int64_t ldx, float* out, int32_t accumulate,
                  float* workspace, bool bf, void* stream) {
  if (M < 0 || N < 0) return ALIGNN_E_BAD_SHAPE;
  if (N == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const unsigned strips = (unsigned)((N + 63) / 64);
  // ~2 blocks per CU in stage 1, at least 64 rows per chunk, at most 256 chunks
  int64_t want = std::max<int64_t>(1, 512 / (int64_t)strips);
  int nparts = (int)std::min<int64_t>({256, want, std::max<int64_t>(1, (M + 63) / 64)});
  int64_t rows_per = (M + nparts - 1) / nparts;
  if (rows_per == 0) rows_per = 1;
  nparts = (int)((M + rows_per - 1) / rows_per);
  if (nparts < 1) nparts = 1;
  if (M == 0) {
    launch(colsum_stage2<0>, dim3(colsum_blocks(N)), dim3(kColsumThreads), 0, s, workspace, 0, N, out, accumulate);
    ALIGNN_LAUNCH_CHECK("colsum_stage2");
    return ALIGNN_OK;
  }
  if (bf) launch(colsum_stage1<true>, dim3(nparts, strips), dim3(256), 0, s, X, M, N, ldx, rows_per, workspace);
  else launch(colsum_stage1<false>, dim3(nparts, strips), dim3(256), 0, s, X, M, N, ldx, rows_per, workspace);
  ALIGNN_LAUNCH_CHECK("colsum_stage1");
  launch(colsum_stage2<0>, dim3(colsum_blocks(N)), dim3(kColsumThreads), 0, s, workspace, nparts, N, out, accumulate);
  ALIGNN_LAUNCH_CHECK("colsum_stage2");
  return ALIGNN_OK;
}

extern "C" int alignn_colsum_f32(const float* X, int64_t M, int64_t N, int64_t ldx, float* out, int32_t accumulate,
                                 float* workspace, void* stream) {
  return colsum(X, M, N, ldx, out, accumulate, workspace, false, stream);
}

extern "C" int alignn_colsum_bf16(const uint16_t* X, int64_t M, int64_t N, int64_t ldx, float* out, int32_t accumulate,
                                  float* workspace, void* stream) {
  return colsum(reinterpret_cast<const float*>(X), M, N, ldx, out, accumulate, workspace, true, stream);
}

extern "C" int alignn_wcolsum2_f32(int64_t M, int64_t N, int32_t C, const float* X1, int64_t ld1, const float* W1,
                                   int64_t lw1, const float* X2, int64_t ld2, const float* W2, int64_t lw2, float* out,
                                   int32_t accumulate, float* workspace, void* stream) {
  if (M < 0 || N < 0 || C <= 0 || N % C != 0) return ALIGNN_E_BAD_SHAPE;
  if (N == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const unsigned strips = (unsigned)((N + 63) / 64);
  // as alignn_colsum_f32: ~2 blocks per CU, >= 64 rows per chunk, <= 256 chunks
  int64_t want = std::max<int64_t>(1, 512 / (int64_t)strips);
  int nparts = (int)std::min<int64_t>({256, want, std::max<int64_t>(1, (M + 63) / 64)});
  int64_t rows_per = std::max<int64_t>(1, (M + nparts - 1) / nparts);
  nparts = (int)std::max<int64_t>(1, (M + rows_per - 1) / rows_per);
  if (M == 0) {
    launch(colsum_stage2<0>, dim3(colsum_blocks(N)), dim3(kColsumThreads), 0, s, workspace, 0, N, out, accumulate);
    ALIGNN_LAUNCH_CHECK("colsum_stage2");
    return ALIGNN_OK;
  }
  launch(wcolsum2_stage1, dim3(nparts, strips), dim3(256), 0, s, X1, ld1, W1, lw1, X2, ld2, W2, lw2, M, N, (int)C,
         rows_per, workspace);
  ALIGNN_LAUNCH_CHECK("wcolsum2_stage1");
  launch(colsum_stage2<0>, dim3(colsum_blocks(N)), dim3(kColsumThreads), 0, s, workspace, nparts, N, out, accumulate);
  ALIGNN_LAUNCH_CHECK("colsum_stage2");
  return ALIGNN_OK;
}
