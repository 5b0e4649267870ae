// gemm_reg.hip — fp32 GEMM with register-direct operands, for the large-M products whose operands are
// both k-contiguous (X·Wᵀ: every nn.Linear forward of the reference's step over bonds / line-graph
// rows; and the dX products through K-contiguous weight copies).
//
// The tiled kernels (gemm_tile.h) stage 16-deep slices through LDS behind a workgroup barrier per
// stage; on the M 23,040 x 256 x 256 products of config C2 they keep the f32 matrix cores ~45 % busy
// (profiles/r04/c2_pmc_mfma.txt).  For a k-contiguous operand the MFMA fragment of a lane is already
// contiguous in memory: v_mfma_f32_32x32x2_f32 takes, on lane half h of a 16-deep slice, k = 8h + s
// (s = 0..7) of row l32 — two 16-byte loads per 32-row block.  So here one wave is one workgroup,
// owns a (32 MI) x (32 NI) output tile, and loads its fragments straight into VGPRs, PD slices in
// flight (a ring of register sets, fully unrolled), with no LDS and no barrier.  Row reuse across the
// waves of a row band comes from L2/L1 (the XCD-contiguous tile order puts a band's column tiles on
// one XCD).
//
// Same k-slot assignment, same MFMA order per accumulator (slice by slice, s = 0..7) and the same
// epilogue function as the tiled kernels: results are bitwise equal to theirs.
#include "gemm_tile.h"

namespace alignn {

typedef float rf4 __attribute__((ext_vector_type(4)));

template <int MI, int NI, int PD>
__global__ __launch_bounds__(64) void gemm_reg_kernel(GemmParams p) {
  constexpr int TM = 32 * MI, TN = 32 * NI;
  const int64_t tiles_n = (p.N + TN - 1) / TN;
  const int64_t nlin = (int64_t)gridDim.x * gridDim.z;   // XCD-contiguous order, as gemm_f32_kernel
  const int64_t lin = (int64_t)blockIdx.z * gridDim.x + blockIdx.x;
  const int64_t xq = nlin / 8, xr = nlin % 8, xcd = lin % 8;
  const int64_t item = xcd * xq + min(xcd, xr) + lin / 8;
  const int64_t tile = item % gridDim.x, b = item / gridDim.x;
  const int64_t m0 = (tile / tiles_n) * TM, n0 = (tile % tiles_n) * TN;
  const int lane = threadIdx.x, h = lane >> 5, l32 = lane & 31;

  // rows past the end are clamped to the last row: they only feed outputs that are never stored
  const float* pa[MI];
  const float* pb[NI];
#pragma unroll
  for (int i = 0; i < MI; ++i) pa[i] = p.A + b * p.sab + min(m0 + 32 * i + l32, p.M - 1) * p.sam + 8 * h;
#pragma unroll
  for (int j = 0; j < NI; ++j) pb[j] = p.B + b * p.sbb + min(n0 + 32 * j + l32, p.N - 1) * p.sbn + 8 * h;
  const int ns = (int)(p.K / 16);   // a multiple of PD (host check)

  floatx16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  rf4 ra[PD][MI][2], rb[PD][NI][2];
  auto load = [&](rf4 (&xa)[MI][2], rf4 (&xb)[NI][2], int s) {
    const int64_t ko = 16 * (int64_t)s;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      xa[i][0] = *reinterpret_cast<const rf4*>(pa[i] + ko);
      xa[i][1] = *reinterpret_cast<const rf4*>(pa[i] + ko + 4);
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      xb[j][0] = *reinterpret_cast<const rf4*>(pb[j] + ko);
      xb[j][1] = *reinterpret_cast<const rf4*>(pb[j] + ko + 4);
    }
    asm volatile("" ::: "memory");   // keep the loads here (not sunk to their first use)
  };
  auto mma = [&](const rf4 (&xa)[MI][2], const rf4 (&xb)[NI][2]) {
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[i][s >> 2][s & 3], xb[j][s >> 2][s & 3], acc[i][j], 0, 0, 0);
  };

#pragma unroll
  for (int d = 0; d < PD; ++d) load(ra[d], rb[d], d);
  for (int base = 0; base + PD < ns; base += PD) {
#pragma unroll
    for (int d = 0; d < PD; ++d) {
      mma(ra[d], rb[d]);
      load(ra[d], rb[d], base + PD + d);
    }
  }
#pragma unroll
  for (int d = 0; d < PD; ++d) mma(ra[d], rb[d]);

  // epilogue: store_tile's element map and epilogue_value (C/D map of 32x32: col = lane & 31,
  // row = (r & 3) + 8 (r >> 2) + 4 h)
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int64_t col = n0 + 32 * j + l32;
      if (col >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row >= p.M) continue;
        store_c(p, b, row, col, epilogue_value(p, b, row, col, acc[i][j][r]), false);
      }
    }
}

constexpr int REG_PD = 4;   // slices in flight; the host requires K % (16 REG_PD) == 0

// mode 1: 64 x 32 per wave, 2: 64 x 64, 3: 32 x 64
void gemm_reg_launch(const GemmParams& p, int mode, int64_t nbatch, hipStream_t s) {
  const int tm = mode == 3 ? 32 : 64, tn = mode == 1 ? 32 : 64;
  const int64_t tiles = ((p.M + tm - 1) / tm) * ((p.N + tn - 1) / tn);
  const dim3 grid((unsigned)tiles, 1, (unsigned)nbatch);
  if (mode == 2) launch(gemm_reg_kernel<2, 2, REG_PD>, grid, dim3(64), 0, s, p);
  else if (mode == 3) launch(gemm_reg_kernel<1, 2, REG_PD>, grid, dim3(64), 0, s, p);
  else launch(gemm_reg_kernel<2, 1, REG_PD>, grid, dim3(64), 0, s, p);
}

int gemm_reg_depth() { return REG_PD; }

}  // namespace alignn
