// gemm_tile.h — fp32 GEMM on gfx950 MFMA (v_mfma_f32_32x32x2_f32: exact f32 fma chain, 64 cyc/SIMD).
//
// Replaces the cuBLAS addmm/mm behind every nn.Linear / PyG Linear of the reference's hot path
// (SURVEY §2 implicit-kernel table) and their autograd backward products.
//
// Tiling: BM x BN block (64 or 128 each), K stage BKT = 16, 32 or 64 (16-deep slices), 256 threads
// = 4 waves in a 2x2 grid, each wave owns (BM/2)x(BN/2) = MI x NI subtiles of 32x32.  One stage per
// iteration, double-buffered LDS with register prefetch of the next stage (issue global loads
// before the MFMAs, write LDS after); a 32-deep stage halves the barriers per MFMA, a 64-deep one
// quarters the stages of a small-grid long-K product (latency-bound: one global round trip each).
//
// k-slot assignment: an MFMA 32x32x2 sums over two k-slots, lane half h = lane>>5 supplying slot h.
// Over the 8 MFMAs of a 16-deep slice, step s uses k = 8h + s for lane half h, so a lane's eight
// k-values are contiguous: one pair of ds_read_b128 per subtile when the LDS image is [row][k],
// eight ds_read_b32 when it is [k][row].  Both operands use the same assignment, so the sum over
// k is complete (in a permuted order — still an exact per-product-rounded fp32 chain).
//
// bf16 compute (ALIGNN_GEMM_BF16): v_mfma_f32_32x32x16_bf16 takes, on lane half h, k = 8h + j
// (j = 0..7) of a 16-deep slice — the same eight k-values the f32 path feeds to its 8 MFMAs — so
// the tiles and LDS images are unchanged: the fragments are rounded to bf16 (v_cvt_pk_bf16_f32,
// RNE) after the LDS read and one MFMA replaces eight.
//
// LDS images follow global contiguity (no transposes while staging):
//   operand contiguous along k   -> [row][BKT+4]
//   operand contiguous along row -> [BKT][ROWS+4]
#pragma once

#include "common.h"

namespace alignn {


typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int BK = 16;  // split-K chunk granularity

struct GemmParams {
  int64_t M, N, K, batch;
  const float* A; int64_t sam, sak, sab;
  const float* B; int64_t sbk, sbn, sbb;
  float* C; int64_t scm, scn, scb;
  const float* bias; int64_t sbias_b;
  const float* rowscale; int64_t srs_m, srs_b;
  const float* bias2; int64_t sb2_b;
  const float* mask; int64_t smk_m, smk_n;
  float alpha, beta;
  int relu;
  int split_k;
  int64_t kchunk;
  float* ws;
  int vecA, vecB;
  int reduce_batch;  // sum the batch into one output: K loop runs over (batch, k), K % BK == 0
  int pad_;
  const int32_t* c_rows;  // optional scatter of C rows
  // bf16 storage (ALIGNN_GEMM_A_BF16 / _B_BF16 / _C_BF16): the pointer holds bf16 elements (strides
  // still in elements); A / B are widened to fp32 exactly as they are staged, C is rounded (RNE)
  int abf, bbf, cbf, pad3_;
  // row sums of A (AlignnGemmArgs.rowsum): the first column tile's workgroups sum their A stages;
  // with split-K the partials go to ws after the C partials, [split][M]
  float* rsum;
};

// Element pointer arithmetic for an operand that holds fp32 or (bf) bf16 elements.
__device__ __forceinline__ const float* eoff(const float* p, int64_t off, int bf) {
  return reinterpret_cast<const float*>(reinterpret_cast<const char*>(p) + off * (bf ? 2 : 4));
}
__device__ __forceinline__ float bf_lo(uint32_t u) { return __builtin_bit_cast(float, u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __builtin_bit_cast(float, u & 0xffff0000u); }
__device__ __forceinline__ float bf_at(const float* p, int64_t i) {
  return __builtin_bit_cast(float, (uint32_t)reinterpret_cast<const uint16_t*>(p)[i] << 16);
}
__device__ __forceinline__ uint16_t bf_rne(float v) { return __builtin_bit_cast(uint16_t, (__bf16)v); }

// Loads one operand tile (ROWS x BKT) into registers.  KC: load along k (general strides,
// float4 when stride_k==1 and aligned); !KC: load along rows (stride_row == 1).
template <int ROWS, bool KC, int BKT, bool L16 = false, int NT = 256>
struct TileLoader {
  static constexpr int F4 = ROWS * BKT / 4 / NT;   // float4 per thread
  static constexpr int KP = BKT + 4;               // padded k-row of the [row][k] image
  static constexpr int KP16 = BKT + 8;             // L16: bf16 [row][k] image for both layouts (16-byte rows)
  // !KC thread -> (k, first of four rows) map.  L16 walks k fastest, so a wave's 2-byte transposing
  // LDS stores land on consecutive halfwords (rows fastest would put 16 lanes on two banks); global
  // loads then still read 64-byte row pieces (four lanes per k).
  __device__ __forceinline__ static int nk(int idx) { return L16 ? idx % BKT : idx / (ROWS / 4); }
  __device__ __forceinline__ static int nr(int idx) { return L16 ? (idx / BKT) * 4 : (idx % (ROWS / 4)) * 4; }
  float4 r[F4];
  const float* base[F4];                           // fast path: this thread's float4 at k = kb
  bool raw = false;                                // r[] holds 4 bf16 values in .x/.y (widened by store)

  // Fast path (vectorisable operand, full stage): per-thread addresses are formed once; a stage
  // is F4 plain float4 loads, no bounds branches.  KC: rows past the end are clamped to the last
  // row (they only feed output rows that are never stored).  !KC: only for interior tiles
  // (row0 + ROWS <= rows), the caller checks.
  __device__ __forceinline__ void setup_fast(const float* __restrict__ P, int64_t srow, int64_t sk, int64_t row0,
                                             int64_t rows, int64_t kb, int bf = 0) {
#pragma unroll
    for (int i = 0; i < F4; ++i) {
      const int idx = threadIdx.x + NT * i;
      if (KC) {
        const int64_t gr = min(row0 + idx / (BKT / 4), rows - 1);
        base[i] = eoff(P, gr * srow + kb + (idx % (BKT / 4)) * 4, bf);
      } else {
        base[i] = eoff(P, (kb + nk(idx)) * sk + row0 + nr(idx), bf);
      }
    }
  }
  // k0 - kb = koff; KC operands have sk == 1 on the fast path.  bf: 8-byte loads of four bf16
  // values kept raw until store() (a conversion here would wait for the load: no prefetch)
  __device__ __forceinline__ void load_fast(int64_t koff, int64_t sk, int bf = 0) {
    if (bf) {
#pragma unroll
      for (int i = 0; i < F4; ++i) {
        const uint2 u = *reinterpret_cast<const uint2*>(eoff(base[i], KC ? koff : koff * sk, 1));
        r[i] = make_float4(__builtin_bit_cast(float, u.x), __builtin_bit_cast(float, u.y), 0.f, 0.f);
      }
      raw = true;
      return;
    }
#pragma unroll
    for (int i = 0; i < F4; ++i) r[i] = *reinterpret_cast<const float4*>(base[i] + (KC ? koff : koff * sk));
    raw = false;
  }

  __device__ __forceinline__ void load(const float* __restrict__ P, int64_t srow, int64_t sk, int64_t row0,
                                       int64_t rows, int64_t k0, int64_t kend, int vec, int bf = 0) {
    raw = false;
    if (bf) {   // bf16 edge tiles: element loads, widened here
#pragma unroll
      for (int i = 0; i < F4; ++i) {
        const int idx = threadIdx.x + NT * i;
        float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          int64_t gr, gk;
          if (KC) {
            gr = row0 + (idx / (BKT / 4));
            gk = k0 + (idx % (BKT / 4)) * 4 + j;
          } else {
            gk = k0 + nk(idx);
            gr = row0 + nr(idx) + j;
          }
          if (gr < rows && gk < kend) v[j] = bf_at(P, KC ? gr * srow + gk * sk : gk * sk + gr);
        }
        r[i] = make_float4(v[0], v[1], v[2], v[3]);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < F4; ++i) {
      int idx = threadIdx.x + NT * i;
      int64_t gr, gk;
      if (KC) {
        gr = row0 + (idx / (BKT / 4));
        gk = k0 + (idx % (BKT / 4)) * 4;
      } else {
        gk = k0 + nk(idx);
        gr = row0 + nr(idx);
      }
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (KC) {
        if (gr < rows) {
          if (vec && gk + 3 < kend) {
            float4 t = *reinterpret_cast<const float4*>(P + gr * srow + gk);
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (gk + j < kend) v[j] = P[gr * srow + (gk + j) * sk];
          }
        }
      } else {
        if (gk < kend) {
          if (vec && gr + 3 < rows) {
            float4 t = *reinterpret_cast<const float4*>(P + gk * sk + gr);
            v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (gr + j < rows) v[j] = P[gk * sk + gr + j];
          }
        }
      }
      r[i] = make_float4(v[0], v[1], v[2], v[3]);
    }
  }

  __device__ __forceinline__ void store(float* __restrict__ lds) {
    if constexpr (L16) {
      // bf16 LDS image [row][KP16] for either global layout: values rounded (RNE) once here instead
      // of per fragment read, raw bf16 operands stored as they are.  KC: one 8-byte store of four k;
      // !KC (four rows at one k): four 2-byte stores, transposing into the [row][k] image.
      uint16_t* L = reinterpret_cast<uint16_t*>(lds);
#pragma unroll
      for (int i = 0; i < F4; ++i) {
        const int idx = threadIdx.x + NT * i;
        uint32_t w0, w1;
        if (raw) {
          w0 = __builtin_bit_cast(uint32_t, r[i].x);
          w1 = __builtin_bit_cast(uint32_t, r[i].y);
        } else {
          w0 = (uint32_t)bf_rne(r[i].x) | ((uint32_t)bf_rne(r[i].y) << 16);
          w1 = (uint32_t)bf_rne(r[i].z) | ((uint32_t)bf_rne(r[i].w) << 16);
        }
        if (KC) {
          const int rr = idx / (BKT / 4), kk = (idx % (BKT / 4)) * 4;
          *reinterpret_cast<uint2*>(L + rr * KP16 + kk) = make_uint2(w0, w1);
        } else {
          const int kk = nk(idx), rr = nr(idx);
          L[(rr + 0) * KP16 + kk] = (uint16_t)w0;
          L[(rr + 1) * KP16 + kk] = (uint16_t)(w0 >> 16);
          L[(rr + 2) * KP16 + kk] = (uint16_t)w1;
          L[(rr + 3) * KP16 + kk] = (uint16_t)(w1 >> 16);
        }
      }
      raw = false;
      return;
    }
    if (raw) {
#pragma unroll
      for (int i = 0; i < F4; ++i) {
        const uint32_t a = __builtin_bit_cast(uint32_t, r[i].x), b = __builtin_bit_cast(uint32_t, r[i].y);
        r[i] = make_float4(bf_lo(a), bf_hi(a), bf_lo(b), bf_hi(b));
      }
      raw = false;
    }
#pragma unroll
    for (int i = 0; i < F4; ++i) {
      int idx = threadIdx.x + NT * i;
      if (KC) {
        int rr = idx / (BKT / 4), kk = (idx % (BKT / 4)) * 4;
        *reinterpret_cast<float4*>(lds + rr * KP + kk) = r[i];
      } else {
        int kk = idx / (ROWS / 4), rr = (idx % (ROWS / 4)) * 4;
        *reinterpret_cast<float4*>(lds + kk * (ROWS + 4) + rr) = r[i];
      }
    }
  }
};

template <int ROWS, bool KC, int BKT, bool L16 = false>
constexpr int lds_floats() {
  return L16 ? ROWS * (BKT + 8) / 2 : KC ? ROWS * (BKT + 4) : BKT * (ROWS + 4);
}

// Reads the 8 k-values of lane half h in 16-deep slice `sub` for subtile row `row`:
// k = 16*sub + 8*h + s, s = 0..7 (the MFMA k-slot assignment, identical for A and B).
template <int ROWS, bool KC, int BKT>
__device__ __forceinline__ void read_frag(const float* __restrict__ lds, int row, int h, int sub, float (&f)[8]) {
  if (KC) {
    const float* q = lds + row * (BKT + 4) + 16 * sub + 8 * h;
    float4 a = *reinterpret_cast<const float4*>(q);
    float4 b = *reinterpret_cast<const float4*>(q + 4);
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
    f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  } else {
#pragma unroll
    for (int s = 0; s < 8; ++s) f[s] = lds[(16 * sub + 8 * h + s) * (ROWS + 4) + row];
  }
}

__device__ __forceinline__ int64_t c_row(const GemmParams& p, int64_t row) {
  return p.c_rows ? (int64_t)p.c_rows[row] : row;
}

// Epilogue arithmetic, in one explicit order shared by every GEMM path (the bf16 streaming kernel's
// band_store too): v = alpha acc; v = fma(beta, C, v); v = v + bias; v = fma(rowscale, bias2, v).
// Written with explicit roundings so that no path's compiler contraction changes the bits.
__device__ __forceinline__ float epilogue_value(const GemmParams& p, int64_t b, int64_t row, int64_t col, float acc) {
  float v = __fmul_rn(p.alpha, acc);
  float* Cb = p.C + b * p.scb;
  if (p.beta != 0.f) v = fmaf(p.beta, Cb[c_row(p, row) * p.scm + col * p.scn], v);
  if (p.bias) v = __fadd_rn(v, p.bias[b * p.sbias_b + col]);
  if (p.rowscale) v = fmaf(p.rowscale[b * p.srs_b + row * p.srs_m], p.bias2[b * p.sb2_b + col], v);
  if (p.relu) v = fmaxf(v, 0.f);
  if (p.mask) v = p.mask[row * p.smk_m + col * p.smk_n] > 0.f ? v : 0.f;
  return v;
}

// One LDS stage of MFMAs: BKT/16 slices of the wave's (BM/2) x (BN/2) subtile, from an LDS image of
// depth LD (>= BKT: the wave-group K-split kernel reads its group's slices `sub0..` of a deeper stage).
template <int BM, int BN, bool A_KC, bool B_KC, int BKT, int BF, int LD = BKT>
__device__ __forceinline__ void mma_stage(floatx16 (&acc)[BM / 64][BN / 64], const float* __restrict__ As,
                                          const float* __restrict__ Bs, int wm, int wn, int h, int l32,
                                          int sub0 = 0) {
  constexpr int MI = BM / 64, NI = BN / 64;
#pragma unroll
  for (int s16 = 0; s16 < BKT / 16; ++s16) {
    const int sub = sub0 + s16;
    if constexpr (BF == 2) {   // bf16 images [row][LD + 8]: a lane's eight k are one 16-byte read
      const uint16_t* A16 = reinterpret_cast<const uint16_t*>(As);
      const uint16_t* B16 = reinterpret_cast<const uint16_t*>(Bs);
      bf16x8 ha[MI], hb[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        ha[i] = *reinterpret_cast<const bf16x8*>(A16 + (wm * (BM / 2) + i * 32 + l32) * (LD + 8) + 16 * sub + 8 * h);
#pragma unroll
      for (int j = 0; j < NI; ++j)
        hb[j] = *reinterpret_cast<const bf16x8*>(B16 + (wn * (BN / 2) + j * 32 + l32) * (LD + 8) + 16 * sub + 8 * h);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha[i], hb[j], acc[i][j], 0, 0, 0);
      continue;
    }
    float fa[MI][8], fb[NI][8];
#pragma unroll
    for (int i = 0; i < MI; ++i) read_frag<BM, A_KC, LD>(As, wm * (BM / 2) + i * 32 + l32, h, sub, fa[i]);
#pragma unroll
    for (int j = 0; j < NI; ++j) read_frag<BN, B_KC, LD>(Bs, wn * (BN / 2) + j * 32 + l32, h, sub, fb[j]);
    if constexpr (BF == 1) {
      bf16x8 ha[MI], hb[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int s = 0; s < 8; ++s) ha[i][s] = (__bf16)fa[i][s];
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int s = 0; s < 8; ++s) hb[j][s] = (__bf16)fb[j][s];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha[i], hb[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][s], fb[j][s], acc[i][j], 0, 0, 0);
    }
  }
}

// Row sums of the A image of one LDS stage (fp32 images only: arithmetic 0 / 1), thread t < ROWS owns
// row t: its BKT values added in k order (zero-filled past the operand's end).
template <int ROWS, bool KC, int BKT>
__device__ __forceinline__ float stage_rowsum(const float* __restrict__ lds, int t, float acc) {
#pragma unroll
  for (int k = 0; k < BKT; ++k) acc += KC ? lds[t * (BKT + 4) + k] : lds[k * (ROWS + 4) + t];
  return acc;
}
template <int BM>
__device__ __forceinline__ void store_rowsum(const GemmParams& p, int64_t m0, int sidx, float acc) {
  const int t = threadIdx.x;
  if (t < BM && m0 + t < p.M) {
    if (p.split_k > 1) p.ws[(int64_t)p.split_k * p.batch * p.M * p.N + (int64_t)sidx * p.M + m0 + t] = acc;
    else p.rsum[m0 + t] = acc;
  }
}

// cbf: C holds bf16 (the caller passes a compile-time false for the fp32-arithmetic kernels, whose
// operands and output are always fp32, so their loops carry no storage-type branches)
__device__ __forceinline__ void store_c(const GemmParams& p, int64_t b, int64_t row, int64_t col, float v, bool cbf) {
  const int64_t i = b * p.scb + c_row(p, row) * p.scm + col * p.scn;
  if (cbf) reinterpret_cast<uint16_t*>(p.C)[i] = bf_rne(v);
  else p.C[i] = v;
}

// Epilogue. C/D map of 32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
// Every operand the epilogue reads (the C rows' scatter targets, beta's C values, the column's bias
// and bias2, the rows' rowscale, the mask) is loaded for four elements of a 32x32 block before their
// stores (register rows r = 4q..4q+3 are four consecutive output rows): element by element, each
// load waited behind the previous element's store (the compiler cannot move a load of possibly
// aliasing memory past a store) — up to 16 dependent global round trips per block, now 4 (+1 for
// the column's bias).  Same arithmetic as epilogue_value, in the same order: bitwise equal.
template <int BM, int BN>
__device__ __forceinline__ void store_tile(const GemmParams& p, const floatx16 (&acc)[BM / 64][BN / 64], int64_t m0,
                                           int64_t n0, int64_t b, int sidx, int wm, int wn, int h, int l32, bool cbf) {
  constexpr int MI = BM / 64, NI = BN / 64;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int64_t col = n0 + wn * (BN / 2) + j * 32 + l32;
      if (col >= p.N) continue;
      const int64_t row0 = m0 + wm * (BM / 2) + i * 32 + 4 * h;   // + (r & 3) + 8 (r >> 2)
      if (p.split_k > 1) {
        float* w = p.ws + ((int64_t)sidx * (p.reduce_batch ? 1 : p.batch) + b) * p.M * p.N + col;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int64_t row = row0 + (r & 3) + 8 * (r >> 2);
          if (row < p.M) w[row * p.N] = acc[i][j][r];
        }
        continue;
      }
      // four rows at a time (registers: the loop's occupancy, not the epilogue's, is what matters)
      const float bv = p.bias ? p.bias[b * p.sbias_b + col] : 0.f;
      const float b2 = p.rowscale ? p.bias2[b * p.sb2_b + col] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float cv[4], rs[4], mk[4];
        int64_t ci[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t row = min(row0 + 8 * q + u, p.M - 1);   // clamped: loads stay in range
          ci[u] = b * p.scb + c_row(p, row) * p.scm + col * p.scn;
          rs[u] = p.rowscale ? p.rowscale[b * p.srs_b + row * p.srs_m] : 0.f;
          mk[u] = p.mask ? p.mask[row * p.smk_m + col * p.smk_n] : 1.f;
          cv[u] = p.beta != 0.f ? (cbf ? bf_at(p.C, ci[u]) : p.C[ci[u]]) : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          float x = __fmul_rn(p.alpha, acc[i][j][4 * q + u]);
          if (p.beta != 0.f) x = fmaf(p.beta, cv[u], x);
          if (p.bias) x = __fadd_rn(x, bv);
          if (p.rowscale) x = fmaf(rs[u], b2, x);
          if (p.relu) x = fmaxf(x, 0.f);
          if (p.mask) x = mk[u] > 0.f ? x : 0.f;
          if (row0 + 8 * q + u >= p.M) continue;
          if (cbf) reinterpret_cast<uint16_t*>(p.C)[ci[u]] = bf_rne(x);
          else p.C[ci[u]] = x;
        }
      }
    }
}

// Sum of one output element's split-K partials (eight chains, partial s into chain s % 8, combined as
// a fixed tree).  An in-launch combine by each tile's last workgroup was measured slower than this
// separate reduce launch (profiles/r02/v9_ab_splitk_combine.log) and removed in round 3.
__device__ __forceinline__ float splitk_sum(const GemmParams& p, int64_t b, int64_t row, int64_t col) {
  const int64_t nb = p.reduce_batch ? 1 : p.batch;
  const int64_t stride = nb * p.M * p.N;
  const float* w = p.ws + (b * p.M + row) * p.N + col;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int k = 0;
  for (; k + 7 < p.split_k; k += 8) {
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += w[(int64_t)(k + j) * stride];
  }
  for (int j = 0; k < p.split_k; ++k, ++j) s[j] += w[(int64_t)k * stride];
  return ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

template <int BM, int BN, bool A_KC, bool B_KC, int BKT, int BF, bool RB>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmParams p) {
  constexpr int MI = BM / 64, NI = BN / 64;
  constexpr bool L16 = BF == 2;
  constexpr int LA = lds_floats<BM, A_KC, BKT, L16>(), LB = lds_floats<BN, B_KC, BKT, L16>();
  __shared__ __attribute__((aligned(16))) float smem[2 * (LA + LB)];

  const int64_t tiles_n = (p.N + BN - 1) / BN;
  // XCD-contiguous work order (same-box A/B +1.5 % step, profiles/r01/v30_ab_gemm_xcd.log; split-K
  // grids too: v33_ab_gemm_xcd_nosplit.log): workgroups are dispatched round-robin over the 8 XCDs,
  // so the linear id lin lands on XCD lin % 8.  Give XCD x the contiguous range of (z, tile) items
  // [x*q + min(x, r), ...) so the column tiles of one A row band share that XCD's L2.
  const int64_t nlin = (int64_t)gridDim.x * gridDim.z;
  const int64_t lin = (int64_t)blockIdx.z * gridDim.x + blockIdx.x;
  const int64_t xq = nlin / 8, xr = nlin % 8, xcd = lin % 8;
  const int64_t item = xcd * xq + min(xcd, xr) + lin / 8;
  const int64_t tile = item % gridDim.x, zid = item / gridDim.x;
  const int64_t m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int64_t b = RB ? 0 : zid / p.split_k;
  const int sidx = zid % p.split_k;
  const int64_t Ktot = RB ? p.K * p.batch : p.K;
  const int64_t kb = (int64_t)sidx * p.kchunk;
  const int64_t ke = min(Ktot, kb + p.kchunk);

  // bf16 storage exists only with bf16 arithmetic (host check): compile-time fp32 otherwise
  const int abf = BF >= 1 ? p.abf : 0, bbf = BF >= 1 ? p.bbf : 0;
  const float* A = eoff(p.A, b * p.sab, abf);
  const float* B = eoff(p.B, b * p.sbb, bbf);
  // (batch, local k) of a global k index; identity unless the batch is reduced (RB)
  auto tileA = [&](int64_t k0) { return RB ? eoff(p.A, (k0 / p.K) * p.sab, abf) : A; };
  auto tileB = [&](int64_t k0) { return RB ? eoff(p.B, (k0 / p.K) * p.sbb, bbf) : B; };
  auto kloc = [&](int64_t k0) { return RB ? k0 % p.K : k0; };
  auto kend = [&](int64_t k0) { return RB ? p.K : ke; };
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, l32 = lane & 31;

  floatx16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  TileLoader<BM, A_KC, BKT, L16> la;
  TileLoader<BN, B_KC, BKT, L16> lb;
  // fast loads (block-uniform): vectorisable operand, not batch-reduced, interior tile for a
  // row-contiguous operand; then every full stage [k0, k0 + BKT) <= ke takes them
  const bool fastA = !RB && p.vecA && (A_KC || m0 + BM <= p.M);
  const bool fastB = !RB && p.vecB && (B_KC || n0 + BN <= p.N);
  if (fastA) la.setup_fast(A, p.sam, p.sak, m0, p.M, kb, abf);
  if (fastB) lb.setup_fast(B, p.sbn, p.sbk, n0, p.N, kb, bbf);
  auto load_stage = [&](int64_t k0) {
    const bool full = k0 + BKT <= ke;
    // A(m,k): rows along m. For A_KC srow = sam, sk = sak; for !A_KC the loader uses (sk = sak).
    if (fastA && full) la.load_fast(k0 - kb, p.sak, abf);
    else la.load(tileA(k0), p.sam, p.sak, m0, p.M, kloc(k0), kend(k0), p.vecA, abf);
    if (fastB && full) lb.load_fast(k0 - kb, p.sbk, bbf);
    else lb.load(tileB(k0), p.sbn, p.sbk, n0, p.N, kloc(k0), kend(k0), p.vecB, bbf);
  };
  load_stage(kb);
  la.store(smem);
  lb.store(smem + LA);
  __syncthreads();

  int cur = 0;
  const bool rs = !L16 && !RB && p.rsum != nullptr && n0 == 0;   // block-uniform
  float rsacc = 0.f;
  for (int64_t k0 = kb; k0 < ke; k0 += BKT) {
    const bool more = k0 + BKT < ke;
    if (more) load_stage(k0 + BKT);
    const float* As = smem + cur * (LA + LB);
    mma_stage<BM, BN, A_KC, B_KC, BKT, BF>(acc, As, As + LA, wm, wn, h, l32);
    if (rs && (int)threadIdx.x < BM) rsacc = stage_rowsum<BM, A_KC, BKT>(As, threadIdx.x, rsacc);
    if (more) {
      float* nxt = smem + (cur ^ 1) * (LA + LB);
      la.store(nxt);
      lb.store(nxt + LA);
    }
    __syncthreads();
    cur ^= 1;
  }

  if (rs) store_rowsum<BM>(p, m0, sidx, rsacc);
  store_tile<BM, BN>(p, acc, m0, n0, b, sidx, wm, wn, h, l32, BF >= 1 && p.cbf);
}

// Pipelined variant: two register sets of global loads in flight, so a stage's
// loads are covered by two stages of MFMAs instead of one (a 16-deep stage is 512 cycles of MFMA per
// wave against a loaded global round trip of several thousand: the one-stage loop above is latency
// bound).  Used when every stage of every workgroup is full and both operands take the vector fast
// path (host check, gemm_pipe_ok), so the loop has no bounds logic.  Loads are unconditional, their
// stage index clamped to the last (a load under a condition becomes a phi whose register copy waits
// for it); the loop covers pairs of stages with one exit, the odd last stage's MFMAs under a
// wave-uniform branch.  Same MFMA order and epilogue as gemm_f32_kernel: bitwise equal results.
typedef float gf4 __attribute__((ext_vector_type(4)));
template <int BM, int BN, bool A_KC, bool B_KC, int BKT, int BF>
__global__ __launch_bounds__(256) void gemm_pipe_kernel(GemmParams p) {
  constexpr int MI = BM / 64, NI = BN / 64;
  constexpr bool L16 = BF == 2;
  constexpr int LA = lds_floats<BM, A_KC, BKT, L16>(), LB = lds_floats<BN, B_KC, BKT, L16>();
  constexpr int FA = TileLoader<BM, A_KC, BKT, L16>::F4, FB = TileLoader<BN, B_KC, BKT, L16>::F4;
  __shared__ __attribute__((aligned(16))) float smem[2 * (LA + LB)];

  const int64_t tiles_n = (p.N + BN - 1) / BN;
  const int64_t nlin = (int64_t)gridDim.x * gridDim.z;   // XCD-contiguous order, as gemm_f32_kernel
  const int64_t lin = (int64_t)blockIdx.z * gridDim.x + blockIdx.x;
  const int64_t xq = nlin / 8, xr = nlin % 8, xcd = lin % 8;
  const int64_t item = xcd * xq + min(xcd, xr) + lin / 8;
  const int64_t tile = item % gridDim.x, zid = item / gridDim.x;
  const int64_t m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;
  const int64_t b = zid / p.split_k;
  const int sidx = zid % p.split_k;
  const int64_t kb = (int64_t)sidx * p.kchunk;
  const int64_t ke = min(p.K, kb + p.kchunk);
  const int nst = (int)((ke - kb) / BKT);  // >= 1 full stages (host check)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, l32 = lane & 31;

  floatx16 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  TileLoader<BM, A_KC, BKT, L16> la;
  TileLoader<BN, B_KC, BKT, L16> lb;
  const bool abf = BF >= 1 && p.abf != 0, bbf = BF >= 1 && p.bbf != 0;   // compile-time false for fp32
  la.setup_fast(eoff(p.A, b * p.sab, abf), p.sam, p.sak, m0, p.M, kb, abf);
  lb.setup_fast(eoff(p.B, b * p.sbb, bbf), p.sbn, p.sbk, n0, p.N, kb, bbf);
  gf4 pa[FA], pb[FB], qa[FA], qb[FB];
  // bf16 operands: 8-byte loads into the first two words, widened when the stage is stored
  auto ld = [](const float* ptr, bool bf) -> gf4 {
    if (bf) {
      const uint2 u = *reinterpret_cast<const uint2*>(ptr);
      return gf4{__builtin_bit_cast(float, u.x), __builtin_bit_cast(float, u.y), 0.f, 0.f};
    }
    return *reinterpret_cast<const gf4*>(ptr);
  };
  auto load = [&](gf4 (&ra)[FA], gf4 (&rb)[FB], int st) {
    const int64_t koff = (int64_t)min(st, nst - 1) * BKT;
#pragma unroll
    for (int i = 0; i < FA; ++i) ra[i] = ld(eoff(la.base[i], A_KC ? koff : koff * p.sak, abf), abf);
#pragma unroll
    for (int i = 0; i < FB; ++i) rb[i] = ld(eoff(lb.base[i], B_KC ? koff : koff * p.sbk, bbf), bbf);
    asm volatile("" ::: "memory");  // keep the loads here (not sunk to their first use)
  };
  auto store = [&](const gf4 (&ra)[FA], const gf4 (&rb)[FB], float* buf) {
#pragma unroll
    for (int i = 0; i < FA; ++i) la.r[i] = make_float4(ra[i].x, ra[i].y, ra[i].z, ra[i].w);
#pragma unroll
    for (int i = 0; i < FB; ++i) lb.r[i] = make_float4(rb[i].x, rb[i].y, rb[i].z, rb[i].w);
    la.raw = abf;
    lb.raw = bbf;
    la.store(buf);
    lb.store(buf + LA);
  };
  float* L0 = smem;
  float* L1 = smem + (LA + LB);
  load(pa, pb, 0);
  store(pa, pb, L0);
  load(pa, pb, 1);
  load(qa, qb, 2);
  __syncthreads();
  const int npairs = (nst + 1) / 2;
  const bool rs = !L16 && p.rsum != nullptr && n0 == 0;   // block-uniform
  float rsacc = 0.f;
  for (int it = 0; it < npairs; ++it) {
    const int s0 = 2 * it;
    mma_stage<BM, BN, A_KC, B_KC, BKT, BF>(acc, L0, L0 + LA, wm, wn, h, l32);   // stage s0
    if (rs && (int)threadIdx.x < BM) rsacc = stage_rowsum<BM, A_KC, BKT>(L0, threadIdx.x, rsacc);
    store(pa, pb, L1);                                                          // stage s0 + 1
    load(pa, pb, s0 + 3);
    __syncthreads();
    if (s0 + 1 < nst) {
      mma_stage<BM, BN, A_KC, B_KC, BKT, BF>(acc, L1, L1 + LA, wm, wn, h, l32);
      if (rs && (int)threadIdx.x < BM) rsacc = stage_rowsum<BM, A_KC, BKT>(L1, threadIdx.x, rsacc);
    }
    store(qa, qb, L0);                                                          // stage s0 + 2
    load(qa, qb, s0 + 4);
    __syncthreads();
  }
  if (rs) store_rowsum<BM>(p, m0, sidx, rsacc);
  store_tile<BM, BN>(p, acc, m0, n0, b, sidx, wm, wn, h, l32, BF >= 1 && p.cbf);
}

template <int BM, int BN, bool A_KC, bool B_KC, int PR>
static void launch_pipe_p(const GemmParams& p, dim3 grid, int bk, hipStream_t s) {
  if (bk >= 64) launch((gemm_pipe_kernel<BM, BN, A_KC, B_KC, 64, PR>), grid, dim3(256), 0, s, p);
  else if (bk == 32) launch((gemm_pipe_kernel<BM, BN, A_KC, B_KC, 32, PR>), grid, dim3(256), 0, s, p);
  else launch((gemm_pipe_kernel<BM, BN, A_KC, B_KC, 16, PR>), grid, dim3(256), 0, s, p);
}


template <int BM, int BN, bool A_KC, bool B_KC, bool RB, int PR>
static void launch_rb_p(const GemmParams& p, dim3 grid, int bk, hipStream_t s) {
  if (bk >= 64) launch((gemm_f32_kernel<BM, BN, A_KC, B_KC, 64, PR, RB>), grid, dim3(256), 0, s, p);
  else if (bk == 32) launch((gemm_f32_kernel<BM, BN, A_KC, B_KC, 32, PR, RB>), grid, dim3(256), 0, s, p);
  else launch((gemm_f32_kernel<BM, BN, A_KC, B_KC, 16, PR, RB>), grid, dim3(256), 0, s, p);
}


// Every workgroup of the pipelined kernel must have only full stages and fast-path operands.
template <int BM, int BN, bool A_KC, bool B_KC>
static bool gemm_pipe_ok(const GemmParams& p, int bk) {
  if (p.reduce_batch || !p.vecA || !p.vecB || bk > 64 || p.K <= 0) return false;
  if (p.kchunk % bk != 0 || p.K % bk != 0) return false;   // every split chunk a whole number of stages
  if (!A_KC && p.M % BM != 0) return false;                 // row-contiguous operands: interior tiles only
  if (!B_KC && p.N % BN != 0) return false;
  if (A_KC && p.sak != 1) return false;
  if (B_KC && p.sbk != 1) return false;
  return true;
}

template <int BM, int BN, bool A_KC, bool B_KC, int PR>
static void launch_tile(const GemmParams& p, dim3 grid, int bk, bool nopipe, hipStream_t s) {
  if (!nopipe && gemm_pipe_ok<BM, BN, A_KC, B_KC>(p, bk)) {
    launch_pipe_p<BM, BN, A_KC, B_KC, PR>(p, grid, bk, s);
    return;
  }
  if (p.reduce_batch) launch_rb_p<BM, BN, A_KC, B_KC, true, PR>(p, grid, bk, s);
  else launch_rb_p<BM, BN, A_KC, B_KC, false, PR>(p, grid, bk, s);
}

template <int BM, int BN, int PR>
static void dispatch_layout(const GemmParams& p, bool akc, bool bkc, dim3 grid, int bk, bool nopipe, hipStream_t s) {
  if (akc && bkc) launch_tile<BM, BN, true, true, PR>(p, grid, bk, nopipe, s);
  else if (akc && !bkc) launch_tile<BM, BN, true, false, PR>(p, grid, bk, nopipe, s);
  else if (!akc && bkc) launch_tile<BM, BN, false, true, PR>(p, grid, bk, nopipe, s);
  else launch_tile<BM, BN, false, false, PR>(p, grid, bk, nopipe, s);
}

// The tiled kernels of one arithmetic (PR: 0 exact fp32 on v_mfma_f32_32x32x2_f32, 1 bf16 inputs,
// 2 bf16 inputs rounded as they are staged into bf16 LDS images — bitwise equal to 1), instantiated
// in gemm_tile_p<PR>.hip (one translation unit each).
template <int PR>
void gemm_tiled_launch(const GemmParams& p, int bm, int bn, bool akc, bool bkc, dim3 grid, int bk, bool nopipe,
                       hipStream_t s) {
  if (bm == 128 && bn == 128) dispatch_layout<128, 128, PR>(p, akc, bkc, grid, bk, nopipe, s);
  else if (bm == 128) dispatch_layout<128, 64, PR>(p, akc, bkc, grid, bk, nopipe, s);
  else if (bn == 128) dispatch_layout<64, 128, PR>(p, akc, bkc, grid, bk, nopipe, s);
  else dispatch_layout<64, 64, PR>(p, akc, bkc, grid, bk, nopipe, s);
}

extern template void gemm_tiled_launch<0>(const GemmParams&, int, int, bool, bool, dim3, int, bool, hipStream_t);
extern template void gemm_tiled_launch<1>(const GemmParams&, int, int, bool, bool, dim3, int, bool, hipStream_t);
extern template void gemm_tiled_launch<2>(const GemmParams&, int, int, bool, bool, dim3, int, bool, hipStream_t);

}  // namespace alignn
