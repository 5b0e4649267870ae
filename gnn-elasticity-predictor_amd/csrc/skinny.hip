// skinny.hip — products with a tiny inner or outer dimension, streamed at HBM rate instead of
// through the MFMA tiles (which would spend a full 16-deep K stage and a 64-wide tile on them).
//
// Replaces, for the angle encoder's first Linear (train.py:358-364, `lg_edge_attr [T, 11]`):
//   forward   h1 = relu(x W1^T + b1)        [T, 11] x [11, D] -> [T, D]    (alignn_linear_smallk_f32)
//   backward  dW1 = dh1^T x, db1 = sum dh1   [D, T] x [T, 11]              (alignn_gemm_tn_smalln_f32)
// At B = 32 (T = 253,440, D = 256) both move the 259 MB [T, D] array once; nothing else is large.
//
// linear_smallk: block = 256 threads = 4 row-lanes x 64 column quads; 64 rows of x staged in LDS
// (every wave reads the same row: LDS broadcast), W's 4 columns x K in registers, float4 stores
// of whole 1 KB output rows.
// tn_smalln: two fixed-order stages (deterministic).  Stage 1: block (row chunk, 256-wide column
// strip of A): 4 row-lanes x 64 threads, each thread 4 consecutive columns of A (float4 loads,
// four rows in flight) and N+1 accumulators per column (the +1 is the column sum); row-lanes
// combined in LDS in lane order; one partial per (chunk, column, n).  Stage 2: per output, the
// chunk partials summed in chunk order (four chains, fixed combine).
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace alignn {

#ifndef ALIGNN_SK_ROWS
#define ALIGNN_SK_ROWS 256  // measured +0.5 % step vs 64 (profiles/r01/v22_ab_sk_rows.log)
#endif
constexpr int SK_ROWS = ALIGNN_SK_ROWS;  // rows of x per workgroup (W's 4 x K columns loaded once per workgroup)
constexpr int SK_KMAX = 16;   // linear_smallk: K <= 16
constexpr int SN_NMAX = 16;   // tn_smalln: N <= 16
constexpr int SN_SLOTS = SN_NMAX + 1;

template <typename OutT>
__global__ __launch_bounds__(256) void linear_smallk_kernel(const float* __restrict__ X, int64_t ldx, int64_t M,
                                                            int K, const float* __restrict__ W, int64_t ldw,
                                                            const float* __restrict__ bias, int64_t N, int relu,
                                                            OutT* __restrict__ out, int64_t ldo) {
  __shared__ float xs[SK_ROWS][SK_KMAX + 1];
  const int tid = threadIdx.x, rl = tid >> 6, cq = tid & 63;
  const int64_t r0 = (int64_t)blockIdx.x * SK_ROWS;
  for (int i = tid; i < SK_ROWS * SK_KMAX; i += 256) {
    const int r = i / SK_KMAX, k = i % SK_KMAX;
    xs[r][k] = (r0 + r < M && k < K) ? X[(r0 + r) * ldx + k] : 0.f;
  }
  __syncthreads();
  const int rows = (int)(M - r0 < SK_ROWS ? M - r0 : SK_ROWS);
  for (int64_t c0 = (int64_t)cq * 4; c0 < N; c0 += 256) {
    float w[4][SK_KMAX], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int k = 0; k < SK_KMAX; ++k) w[j][k] = k < K ? W[(c0 + j) * ldw + k] : 0.f;
      b[j] = bias ? bias[c0 + j] : 0.f;
    }
    for (int r = rl; r < rows; r += 4) {
      float a[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < SK_KMAX; ++k) {
        const float x = xs[r][k];
#pragma unroll
        for (int j = 0; j < 4; ++j) a[j] = fmaf(x, w[j][k], a[j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] += b[j];
        if (relu) a[j] = fmaxf(a[j], 0.f);
      }
      if constexpr (sizeof(OutT) == 4) {
        *reinterpret_cast<float4*>(out + (r0 + r) * ldo + c0) = make_float4(a[0], a[1], a[2], a[3]);
      } else {
        typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
        bf4 h;
        h.x = (__bf16)a[0]; h.y = (__bf16)a[1]; h.z = (__bf16)a[2]; h.w = (__bf16)a[3];
        *reinterpret_cast<bf4*>(out + (r0 + r) * ldo + c0) = h;
      }
    }
  }
}

__global__ __launch_bounds__(256) void tn_smalln_stage1(const float* __restrict__ A, int64_t lda, int64_t K,
                                                        int64_t M, const float* __restrict__ X, int64_t ldx, int N,
                                                        int64_t rows_per, int vec, float* __restrict__ part) {
  __shared__ float xs[SK_ROWS][SN_NMAX + 1];
  __shared__ float red[256 * SN_SLOTS];
  const int tid = threadIdx.x, rl = tid >> 6, cq = tid & 63;
  const int64_t m0 = (int64_t)blockIdx.y * 256 + cq * 4;
  const int64_t kb = (int64_t)blockIdx.x * rows_per;
  const int64_t ke = kb + rows_per < K ? kb + rows_per : K;
  float acc[4][SN_SLOTS];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int n = 0; n < SN_SLOTS; ++n) acc[j][n] = 0.f;

  auto load4 = [&](int64_t k) -> float4 {
    if (k >= ke || m0 >= M) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float* p = A + k * lda + m0;
    if (vec) return *reinterpret_cast<const float4*>(p);
    float v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = m0 + j < M ? p[j] : 0.f;
    return make_float4(v[0], v[1], v[2], v[3]);
  };

  for (int64_t t0 = kb; t0 < ke; t0 += SK_ROWS) {
    for (int i = tid; i < SK_ROWS * SN_NMAX; i += 256) {
      const int r = i / SN_NMAX, n = i % SN_NMAX;
      xs[r][n] = (t0 + r < ke && n < N) ? X[(t0 + r) * ldx + n] : 0.f;
    }
    __syncthreads();
    // rows rl, rl+4, ..., 16 per row-lane per tile, four loads in flight
    for (int r = rl; r < SK_ROWS; r += 16) {
      float4 a4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) a4[u] = load4(t0 + r + 4 * u);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float av[4] = {a4[u].x, a4[u].y, a4[u].z, a4[u].w};
#pragma unroll
        for (int n = 0; n < SN_NMAX; ++n) {
          const float x = xs[r + 4 * u][n];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j][n] = fmaf(av[j], x, acc[j][n]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j][SN_NMAX] += av[j];
      }
    }
    __syncthreads();
  }
  // row-lanes combined in lane order: 0 + 1 + 2 + 3
  for (int l = 1; l < 4; ++l) {
    if (rl == l) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int n = 0; n < SN_SLOTS; ++n) red[(cq * 4 + j) * SN_SLOTS + n] = acc[j][n];
    }
    __syncthreads();
    if (rl == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int n = 0; n < SN_SLOTS; ++n) acc[j][n] += red[(cq * 4 + j) * SN_SLOTS + n];
    }
    __syncthreads();
  }
  if (rl == 0) {
    float* dst = part + (int64_t)blockIdx.x * M * SN_SLOTS;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (m0 + j < M)
#pragma unroll
        for (int n = 0; n < SN_SLOTS; ++n) dst[(m0 + j) * SN_SLOTS + n] = acc[j][n];
  }
}

__global__ __launch_bounds__(256) void tn_smalln_stage2(const float* __restrict__ part, int chunks, int64_t M, int N,
                                                        float* __restrict__ C, int64_t ldc,
                                                        float* __restrict__ colsum, int acc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * SN_SLOTS) return;
  const int64_t m = i / SN_SLOTS;
  const int n = (int)(i % SN_SLOTS);
  if (n < SN_NMAX && n >= N) return;
  if (n == SN_NMAX && !colsum) return;
  const int64_t stride = M * SN_SLOTS;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int c = 0;
  for (; c + 3 < chunks; c += 4) {
    s0 += part[(int64_t)c * stride + i];
    s1 += part[(int64_t)(c + 1) * stride + i];
    s2 += part[(int64_t)(c + 2) * stride + i];
    s3 += part[(int64_t)(c + 3) * stride + i];
  }
  for (; c < chunks; ++c) s0 += part[(int64_t)c * stride + i];
  const float t = (s0 + s1) + (s2 + s3);
  float* dst = n == SN_NMAX ? colsum + m : C + m * ldc + n;
  *dst = acc ? *dst + t : t;
}

static void smalln_plan(int64_t K, int64_t M, int64_t& chunks, int64_t& rows_per) {
  const int64_t strips = (M + 255) / 256;
  int64_t want = 512 / (strips > 0 ? strips : 1);
  if (want < 1) want = 1;
  int64_t maxc = (K + 255) / 256;
  chunks = want < maxc ? want : maxc;
  if (chunks < 1) chunks = 1;
  rows_per = (K + chunks - 1) / chunks;
  rows_per = (rows_per + SK_ROWS - 1) / SK_ROWS * SK_ROWS;
  if (rows_per < SK_ROWS) rows_per = SK_ROWS;
  chunks = (K + rows_per - 1) / rows_per;
  if (chunks < 1) chunks = 1;
}

static bool aligned16p(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// ---------------------------------------------------------------------------------------------
// bf16 output: autocast's arithmetic (train.py:554 under :636) — x, W and b rounded to bf16, the
// products accumulated in fp32 on the matrix cores, the sum rounded to bf16, then ReLU on the bf16
// value.  One v_mfma_f32_32x32x16_bf16 per 32 output columns x 32 rows with the operands of the
// deferred encoder backward's mask recompute (encbwd.hip, enc_bwd_bf16_kernel<H, true>): the same
// [W | b] fragment (lane (hh, r): column r, inputs 8 hh .. 8 hh + 7, b at k = K) and the same [x | 1]
// fragment (row r), in swapped operand roles — D^T instead of D, each element the same 16 products
// in the same k slots — so the stored layer's ReLU mask is the recompute's bit for bit and that
// backward may take either.  Workgroup: 4 waves; per 32-row chunk and 256-column slab each wave
// computes two 32-column tiles (w, w + 4) into an LDS image (lane (hh, r): row r, columns
// 8 q + 4 hh .. + 3 of the tile for register group q), then the workgroup stores the slab's rows as
// whole 16-byte pieces (a wave instruction writes two full 512-byte rows; nontemporal: the layer is
// written once and read back by the next kernel from HBM).  Grid-stride over chunks, the next chunk's
// raw inputs loaded before the current one is computed.
typedef __bf16 skh8 __attribute__((ext_vector_type(8)));
typedef __bf16 skh4 __attribute__((ext_vector_type(4)));
typedef float skx16 __attribute__((ext_vector_type(16)));
typedef uint32_t sku4 __attribute__((ext_vector_type(4)));
constexpr int SKM_KMAX = 15;        // inputs + the ones column within one 16-deep k step
constexpr int SKM_SLABS = 4;        // 256-column slabs (N <= 1024)
constexpr int SKM_LDT = 256 + 8;    // LDS image row (bf16), padded
__device__ __forceinline__ float sk_keep(float v, bool keep) {
  return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, v) & (keep ? 0xffffffffu : 0u));
}
template <int SLABS>
__global__ __launch_bounds__(256) void linear_smallk_bf16_mx_kernel(const float* __restrict__ X, int64_t ldx,
                                                                   int64_t M, int K, const float* __restrict__ W,
                                                                   int64_t ldw, const float* __restrict__ bias,
                                                                   int N, int relu, uint16_t* __restrict__ out,
                                                                   int64_t ldo) {
  __shared__ __attribute__((aligned(16))) uint16_t img[32 * SKM_LDT];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int nt = N / 32, slabs = (N + 255) / 256;
  skh8 WB[2 * SLABS];   // tile 8 s + w + 4 j -> WB[2 s + j]
#pragma unroll
  for (int t = 0; t < 2 * SLABS; ++t) {
    const int tile = 8 * (t >> 1) + w + 4 * (t & 1);
    const int col = 32 * min(tile, nt - 1) + r;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * hh + j;
      const float v = W[(int64_t)col * ldw + min(k, K - 1)];
      const float b = bias ? bias[col] : 0.f;
      WB[t][j] = (__bf16)(k < K ? v : (k == K ? b : 0.f));
    }
  }
  // this lane's 8 raw inputs of row r of a chunk (unconditional loads, row clamped into X), one chunk ahead
  auto load_x = [&](int64_t c0, float (&v)[8]) {
    const float* xr = X + min(c0 + r, M - 1) * ldx;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = xr[min(8 * hh + j, K - 1)];
  };
  const int64_t step = 32 * (int64_t)gridDim.x;
  float xv[8];
  load_x(32 * (int64_t)blockIdx.x, xv);
  for (int64_t r0 = 32 * (int64_t)blockIdx.x; r0 < M; r0 += step) {
    skh8 XB;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * hh + j;
      XB[j] = (__bf16)(k == K ? 1.f : sk_keep(xv[j], k < K));
    }
    load_x(r0 + step, xv);
#pragma unroll
    for (int s = 0; s < SLABS; ++s) {
      if (s >= slabs) break;   // uniform
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int tl = w + 4 * j;   // tile within the slab
        if (8 * s + tl >= nt) break;   // wave-uniform
        const skx16 pre = __builtin_amdgcn_mfma_f32_32x32x16_bf16(WB[2 * s + j], XB, skx16{}, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          skh4 h;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const __bf16 b = (__bf16)pre[4 * q + i];
            h[i] = (relu && !((float)b > 0.f)) ? (__bf16)0.f : b;
          }
          *reinterpret_cast<skh4*>(img + r * SKM_LDT + 32 * tl + 8 * q + 4 * hh) = h;
        }
      }
      __syncthreads();
      const int ncol = min(256, N - 256 * s);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int piece = threadIdx.x + 256 * u, row = piece >> 5, c8 = 8 * (piece & 31);
        if (r0 + row < M && c8 < ncol) {
          sku4* dst = reinterpret_cast<sku4*>(out + (r0 + row) * ldo + 256 * s + c8);
          const sku4 v = *reinterpret_cast<const sku4*>(img + row * SKM_LDT + c8);
          __builtin_nontemporal_store(v, dst);   // streamed once (1 GB at B = 256): 336 -> 216 us
        }
      }
      __syncthreads();
    }
  }
}

}  // namespace alignn

using namespace alignn;

extern "C" int alignn_linear_smallk_f32(const float* X, int64_t ldx, int64_t M, int32_t K, const float* W,
                                        int64_t ldw, const float* bias, int64_t N, int32_t relu, float* out,
                                        int64_t ldo, void* stream) {
  if (M < 0 || K < 0 || N < 0 || (M > 0 && (!X || !out)) || (N > 0 && K > 0 && !W)) {
    set_error("linear_smallk: bad arguments");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (K > SK_KMAX || N % 4 != 0 || ldo % 4 != 0 || !aligned16p(out) || ldx < K || ldw < K || ldo < N) {
    set_error("linear_smallk: needs K <= %d, N %% 4 == 0, 16-byte aligned output rows (K=%d N=%lld ldo=%lld)",
              SK_KMAX, (int)K, (long long)N, (long long)ldo);
    return ALIGNN_E_UNSUPPORTED;
  }
  if (M == 0 || N == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const unsigned blocks = (unsigned)((M + SK_ROWS - 1) / SK_ROWS);
  launch(linear_smallk_kernel<float>, dim3(blocks), dim3(256), 0, s, X, ldx, M, (int)K, W, ldw, bias, N,
                     (int)relu, out, ldo);
  ALIGNN_LAUNCH_CHECK("linear_smallk_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_linear_smallk_bf16out(const float* X, int64_t ldx, int64_t M, int32_t K, const float* W,
                                            int64_t ldw, const float* bias, int64_t N, int32_t relu, uint16_t* out,
                                            int64_t ldo, void* stream) {
  if (M < 0 || K < 0 || N < 0 || (M > 0 && (!X || !out)) || (N > 0 && K > 0 && !W)) {
    set_error("linear_smallk_bf16out: bad arguments");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (K < 1 || K > SKM_KMAX || N % 32 != 0 || N > 256 * SKM_SLABS || ldo % 8 != 0 ||
      (reinterpret_cast<uintptr_t>(out) & 15u) || ldx < K || ldw < K || ldo < N) {
    set_error("linear_smallk_bf16out: needs 1 <= K <= %d, N %% 32 == 0, N <= %d, 16-byte aligned output rows "
              "(K=%d N=%lld ldo=%lld)", SKM_KMAX, 256 * SKM_SLABS, (int)K, (long long)N, (long long)ldo);
    return ALIGNN_E_UNSUPPORTED;
  }
  if (M == 0 || N == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // 8 workgroups per CU (measured 216 us at B = 256 against 234-237 with 2 or 4, profiles/r06/ab_linear_bf16.txt)
  const unsigned blocks = (unsigned)std::min<int64_t>((M + 31) / 32, 256 * 8);
  if (N <= 256)
    launch(linear_smallk_bf16_mx_kernel<1>, dim3(blocks), dim3(256), 0, s, X, ldx, M, (int)K, W, ldw, bias, (int)N,
           (int)relu, out, ldo);
  else
    launch(linear_smallk_bf16_mx_kernel<SKM_SLABS>, dim3(blocks), dim3(256), 0, s, X, ldx, M, (int)K, W, ldw, bias,
           (int)N, (int)relu, out, ldo);
  ALIGNN_LAUNCH_CHECK("linear_smallk_bf16_mx_kernel");
  return ALIGNN_OK;
}

extern "C" int64_t alignn_gemm_tn_smalln_workspace(int64_t K, int64_t M, int32_t N) {
  if (K < 0 || M < 0 || N < 0 || N > SN_NMAX) return -1;
  int64_t chunks, rows_per;
  smalln_plan(K, M, chunks, rows_per);
  return chunks * M * SN_SLOTS;
}

extern "C" int alignn_gemm_tn_smalln_f32(const float* A, int64_t lda, int64_t K, int64_t M, const float* X,
                                         int64_t ldx, int32_t N, float* C, int64_t ldc, float* colsum,
                                         int32_t accumulate, float* workspace, int64_t workspace_elems,
                                         void* stream) {
  if (K < 0 || M < 0 || N < 0 || lda < M || ldx < N || ldc < N) {
    set_error("gemm_tn_smalln: bad shape");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (N > SN_NMAX) {
    set_error("gemm_tn_smalln: N=%d > %d", (int)N, SN_NMAX);
    return ALIGNN_E_UNSUPPORTED;
  }
  if (M == 0 || (N == 0 && !colsum)) return ALIGNN_OK;
  int64_t chunks, rows_per;
  smalln_plan(K, M, chunks, rows_per);
  if (!workspace || workspace_elems < chunks * M * SN_SLOTS) {
    set_error("gemm_tn_smalln: needs %lld workspace floats", (long long)(chunks * M * SN_SLOTS));
    return ALIGNN_E_WORKSPACE;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int vec = (lda % 4 == 0 && M % 4 == 0 && aligned16p(A)) ? 1 : 0;
  if (K > 0) {
    launch(tn_smalln_stage1, dim3((unsigned)chunks, (unsigned)((M + 255) / 256)), dim3(256), 0, s, A, lda,
                       K, M, X, ldx, (int)N, rows_per, vec, workspace);
    ALIGNN_LAUNCH_CHECK("tn_smalln_stage1");
  } else {
    const hipError_t e = hipMemsetAsync(workspace, 0, sizeof(float) * M * SN_SLOTS, s);
    if (e != hipSuccess) return hip_status(e, "tn_smalln memset");
    chunks = 1;
  }
  const int64_t total = M * SN_SLOTS;
  launch(tn_smalln_stage2, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, workspace, (int)chunks,
                     M, (int)N, C, ldc, colsum, (int)accumulate);
  ALIGNN_LAUNCH_CHECK("tn_smalln_stage2");
  return ALIGNN_OK;
}
