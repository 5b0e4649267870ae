// gemm_wgrad.hip — bf16 weight-gradient GEMM over every row: dW[M, N] = sum_r dY[r, m] X[r, n] (A = dY^T,
// B = X, both stored row-major over the long K = rows axis), config C3's long-K products (the skip
// projections and edge MLP over 184,320 bonds, the Q/K/V(R) projections over 15,360 atoms / 16,020
// active bonds), with the bias gradient sum_r dY[r, m] (AlignnGemmArgs.rowsum) from the same launch.
//
// The tiled kernel runs these as 128 x 64 tiles with split-K (bf_long plan): every tile re-reads its
// 128 rows of dY^T and 64 of X per split, with 4-byte transposing LDS stores (both operands are
// row-contiguous, the MFMA wants them k-contiguous) — 131 us for 256 x 256 x 184,320 (0.19-0.36 of
// HBM; 65.5 us here with bf16 operands, 90 / 120 us with one / both fp32, standalone on all CUs;
// profiles/r05/v8_ab_gemm_wgrad.txt).  Here one 8-wave workgroup per CU computes a whole 256 x 256 output tile over a contiguous
// chunk of rows: the chunk's rows are staged as they lie in memory (16-byte loads, one read of each
// operand byte per tile) into bf16 [32][288] LDS images, and the MFMA operands come out of them with
// the gfx950 transpose read ds_read_b64_tr_b16 (two per 32x32x16 operand: four k-rows of 16 columns
// per 16-lane group, column-major into the lanes).  The 576-byte image row puts the four rows of
// a 16-lane group and the two groups of a 32-lane half on distinct banks.  Each wave owns 64 x 128
// of the output (8 accumulators); a chunk's partial tile goes to the split-K workspace and the
// library's fixed-order split-K reduce (gemm.hip) forms dW = epilogue(sum of partials) and the bias
// gradient from the per-chunk row sums (each thread sums its fixed columns of the staged dY rows in
// row order; the chunk's threads combine in a fixed order) — deterministic, no atomics.
//
// Operand rounding: bf16 RNE as every bf16-arithmetic path here (fp32 operands are rounded as they are
// staged); accumulation fp32 in 16-row k-steps.  The row sums add the operand values as stored (fp32
// or bf16), not rounded.
#include "gemm_tile.h"

namespace alignn {
namespace wgk {

typedef float gf4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef short s4 __attribute__((ext_vector_type(4)));
constexpr int NT = 512;     // 8 waves
constexpr int TM = 256;     // output tile rows (m) per workgroup
constexpr int TN = 256;     // output tile columns (n)
constexpr int ROWS = 32;    // k-rows per staged band
constexpr int LDR = 288;    // image row stride (bf16): 576 B, 144 dwords = 16 banks mod 64

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)bf_rne(a) | ((uint32_t)bf_rne(b) << 16);
}

// One band (ROWS k-rows x 256 columns) of one operand in registers: 16-byte chunks.
template <bool BF>
struct Stage {
  static constexpr int CPR = BF ? 32 : 64;            // chunks per row (8 bf16 or 4 fp32 values)
  static constexpr int PER = ROWS * CPR / NT;          // chunks per thread: bf16 2, fp32 4
  gf4 r[PER];
  // row r of the operand starts at P + r * srow; columns c0 .. c0 + 255 (clamped to < ncol, zeroed)
  __device__ __forceinline__ void load(const float* __restrict__ P, int64_t srow, int64_t r0, int64_t rend,
                                       int64_t c0, int64_t ncol) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = threadIdx.x + NT * i;
      const int64_t row = min(r0 + idx / CPR, rend - 1);
      const int64_t col = min(c0 + (idx % CPR) * (BF ? 8 : 4), ncol - (BF ? 8 : 4));
      r[i] = *reinterpret_cast<const gf4*>(eoff(P, row * srow + col, BF));
    }
    asm volatile("" ::: "memory");
  }
  // live: the band row exists (< rend) and the columns are < ncol; else zeros
  __device__ __forceinline__ void store(__bf16* __restrict__ img, int64_t r0, int64_t rend, int64_t c0,
                                        int64_t ncol, float (&rs)[BF ? 8 : 4], bool sum) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int idx = threadIdx.x + NT * i;
      const int rr = idx / CPR, cc = (idx % CPR) * (BF ? 8 : 4);
      const bool live = r0 + rr < rend && c0 + cc < ncol;
      if constexpr (BF) {
        u32x4 u = __builtin_bit_cast(u32x4, r[i]);
        if (!live) u = u32x4{0u, 0u, 0u, 0u};
        *reinterpret_cast<u32x4*>(img + rr * LDR + cc) = u;
        if (sum) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            rs[2 * e] += bf_lo(u[e]);
            rs[2 * e + 1] += bf_hi(u[e]);
          }
        }
      } else {
        const gf4 v = live ? r[i] : gf4{0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<u32x2*>(img + rr * LDR + cc) = u32x2{pack2(v.x, v.y), pack2(v.z, v.w)};
        if (sum) {
          rs[0] += v.x; rs[1] += v.y; rs[2] += v.z; rs[3] += v.w;
        }
      }
    }
  }
};

// The MFMA operand of a 32-column block at image column c, k-step ks (16 rows): lane l receives
// column c + (l & 31), rows 16 ks + 8 (l >> 5) + 0..7 (two transposed reads of four rows).
__device__ __forceinline__ bf16x8 tr_operand(const __bf16* img, int c, int ks, int lane) {
  typedef __attribute__((address_space(3))) s4 lds_s4;
  typedef short s8 __attribute__((ext_vector_type(8)));
  const int g = lane >> 4, li = lane & 15;
  const int row = 16 * ks + 8 * (g >> 1) + (li >> 2), col = c + 16 * (g & 1) + 4 * (li & 3);
  const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + row * LDR + col));
  const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + (row + 4) * LDR + col));
  const s8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// grid (tiles_m * tiles_n, S): workgroup (t, s) owns output tile t and rows [s * rows_per, ...).
template <bool ABF, bool BBF>
__global__ __launch_bounds__(NT, 1) void wgrad_kernel(GemmParams p, int64_t rows_per) {
  __shared__ __attribute__((aligned(16))) __bf16 Ai[2][ROWS * LDR];
  __shared__ __attribute__((aligned(16))) __bf16 Bi[2][ROWS * LDR];
  const int64_t tiles_n = (p.N + TN - 1) / TN;
  const int64_t m0 = (blockIdx.x / tiles_n) * TM, n0 = (blockIdx.x % tiles_n) * TN;
  const int s = blockIdx.y;
  const int64_t bz = blockIdx.z;   // batch entry (the per-head dM products: batch = heads)
  if (bz > 0) {
    p.A = eoff(p.A, bz * p.sab, ABF);
    p.B = eoff(p.B, bz * p.sbb, BBF);
  }
  const int64_t r0 = (int64_t)s * rows_per, rend = min(p.K, r0 + rows_per);
  const int lane = threadIdx.x & 63, wave = wave_id();
  const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, l32 = lane & 31;
  const bool sum = p.rsum != nullptr && n0 == 0;   // workgroup-uniform: the first column tile sums dY

  floatx16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float rs[ABF ? 8 : 4] = {}, rsb[BBF ? 8 : 4];   // dY's row sums (rsb: unused, B is not summed)

  // A = dY^T: k-row r of A is dY row r, its m-columns contiguous (stride sak between rows);
  // B = X: k-row r is X row r (stride sbk), n-columns contiguous
  Stage<ABF> sa;
  Stage<BBF> sb;
  const int nb = (int)((rend - r0 + ROWS - 1) / ROWS);   // >= 1 (host check)
  sa.load(p.A, p.sak, r0, rend, m0, p.M);
  sb.load(p.B, p.sbk, r0, rend, n0, p.N);
  for (int b = 0; b < nb; ++b) {
    const int cur = b & 1;
    const int64_t rb = r0 + (int64_t)b * ROWS;
    sa.store(Ai[cur], rb, rend, m0, p.M, rs, sum);
    sb.store(Bi[cur], rb, rend, n0, p.N, rsb, false);
    if (b + 1 < nb) {   // workgroup-uniform: the next band in flight during this one's MFMAs
      sa.load(p.A, p.sak, rb + ROWS, rend, m0, p.M);
      sb.load(p.B, p.sbk, rb + ROWS, rend, n0, p.N);
    }
    __syncthreads();   // this band's images complete (and the other buffer's readers done, below)
#pragma unroll
    for (int ks = 0; ks < ROWS / 16; ++ks) {
      bf16x8 fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = tr_operand(Ai[cur], 64 * wm + 32 * i, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = tr_operand(Bi[cur], 128 * wn + 32 * j, ks, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    // the next iteration writes the other buffer, last read two iterations ago: the barrier above
    // (every wave past this band's store) orders it after those reads
  }

  // partial tile -> split-K workspace [s][M][N] (rows and columns past M / N dropped)
  float* W = p.ws + ((int64_t)s * p.batch + bz) * p.M * p.N;   // the split-K workspace layout [s][b][M][N]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t col = n0 + 128 * wn + 32 * j + l32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + 64 * wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < p.M && col < p.N) W[row * p.N + col] = acc[i][j][r];
      }
    }
  if (sum) {   // the chunk's row sums: threads with the same columns combined in thread order
    constexpr int CW = ABF ? 8 : 4, CPR = Stage<ABF>::CPR, G = NT / CPR;   // columns per thread, threads per column
    __shared__ float Lrs[NT][CW];
#pragma unroll
    for (int e = 0; e < CW; ++e) Lrs[threadIdx.x][e] = rs[e];
    __syncthreads();
    if ((int)threadIdx.x < CPR) {
      float t[CW];
#pragma unroll
      for (int e = 0; e < CW; ++e) t[e] = 0.f;
      for (int gi = 0; gi < G; ++gi)
#pragma unroll
        for (int e = 0; e < CW; ++e) t[e] += Lrs[threadIdx.x + CPR * gi][e];
      float* R = p.ws + (int64_t)p.split_k * p.M * p.N + (int64_t)s * p.M;
#pragma unroll
      for (int e = 0; e < CW; ++e) {
        const int64_t m = m0 + threadIdx.x * CW + e;
        if (m < p.M) R[m] = t[e];
      }
    }
  }
}

}  // namespace wgk

// Plan (host): S chunks of rows_per rows (a multiple of 32) so that tiles x S ~ one workgroup per two
// CUs (ALIGNN_WGRAD_WGS overrides the target, read once).  These products run on the side stream beside
// the critical path's attention and dX products, so half the CUs is the better share: C3 step, same
// box (profiles/r05/v8_ab_gemm_wgrad.txt), 256 workgroups 21,702 / 21,907 graphs/s, 128 22,164 /
// 22,424, 64 22,231 / 22,272, the tiled kernel instead 22,054 / 21,718.
int64_t gemm_wgrad_split(int64_t M, int64_t N, int64_t K, int64_t batch, int cus, int64_t* rows_per) {
  static const int64_t target_env = [] {
    const char* e = std::getenv("ALIGNN_WGRAD_WGS");
    return e ? std::max<int64_t>(1, std::atoll(e)) : int64_t(0);
  }();
  const int64_t tiles = ((M + wgk::TM - 1) / wgk::TM) * ((N + wgk::TN - 1) / wgk::TN) * batch;
  const int64_t target = target_env ? target_env : std::max<int64_t>(1, cus / 2);
  int64_t S = std::max<int64_t>(1, target / tiles);
  int64_t rp = (K + S - 1) / S;
  rp = (rp + wgk::ROWS - 1) / wgk::ROWS * wgk::ROWS;
  S = (K + rp - 1) / rp;
  *rows_per = rp;
  return S;
}

void gemm_wgrad_launch(const GemmParams& p, int64_t S, int64_t rows_per, hipStream_t s) {
  const int64_t tiles = ((p.M + wgk::TM - 1) / wgk::TM) * ((p.N + wgk::TN - 1) / wgk::TN);
  const dim3 grid((unsigned)tiles, (unsigned)S, (unsigned)p.batch);
  if (p.abf && p.bbf) launch(wgk::wgrad_kernel<true, true>, grid, dim3(wgk::NT), 0, s, p, rows_per);
  else if (p.abf) launch(wgk::wgrad_kernel<true, false>, grid, dim3(wgk::NT), 0, s, p, rows_per);
  else if (p.bbf) launch(wgk::wgrad_kernel<false, true>, grid, dim3(wgk::NT), 0, s, p, rows_per);
  else launch(wgk::wgrad_kernel<false, false>, grid, dim3(wgk::NT), 0, s, p, rows_per);
}

}  // namespace alignn
