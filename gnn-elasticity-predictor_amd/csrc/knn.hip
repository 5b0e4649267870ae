// knn.hip — KNN density weights over graph embeddings (reference
// compute_global_knn_weights, scripts/train.py:930-1010, which uses sklearn on the host).
//
// Z [n, D] embeddings -> column standardization (two-pass, population std, floor 1e-8) -> squared
// distances from the Gram matrix G = Zs Zs^T (an MFMA GEMM outside) and row norms r:
//   d2_ij = r_i + r_j - 2 G_ij.  Per row, the k nearest j != i are selected in (distance, index)
// order by k passes of a wave-wide lexicographic argmin (deterministic ties), then
//   rho = k / (sum_k sqrt(d2) + eps), w = rho^-alpha, w /= 1 + beta * mean_t var_k(Y[nbr, t]).
// Clipping and the final normalisation by the mean are left to the caller (host, as the reference).
#include "common.h"

namespace alignn {

__global__ void col_center_sq_kernel(const float* __restrict__ Z, int64_t n, int D, const float* __restrict__ colsum,
                                     float* __restrict__ out) {
  const int64_t total = n * D;
  const float invn = 1.0f / (float)n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const float c = Z[i] - colsum[i % D] * invn;
    out[i] = c * c;
  }
}

// Zs = (Z - mean) / max(sqrt(ssq / n), 1e-8); mean and ssq arrive as column SUMS.
__global__ void standardize_kernel(const float* __restrict__ Z, int64_t n, int D, const float* __restrict__ colsum,
                                   const float* __restrict__ ssq, float* __restrict__ out) {
  const int64_t total = n * D;
  const float invn = 1.0f / (float)n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % D);
    const float sd = fmaxf(sqrtf(ssq[c] * invn), 1e-8f);
    out[i] = (Z[i] - colsum[c] * invn) / sd;
  }
}

__global__ void row_sqnorm_kernel(const float* __restrict__ Zs, int64_t n, int D, float* __restrict__ r) {
  const int64_t row = (int64_t)blockIdx.x * 4 + wave_id();
  if (row >= n) return;
  float s = 0.f;
  for (int c = threadIdx.x & 63; c < D; c += 64) {
    const float v = Zs[row * D + c];
    s = fmaf(v, v, s);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) r[row] = s;
}

// (d, j) < (d', j') lexicographically
__device__ __forceinline__ bool lex_less(float d, int64_t j, float d2, int64_t j2) {
  return d < d2 || (d == d2 && j < j2);
}

// One wave per query row (rows row0 .. row0+rows-1 of the full set; G holds those rows).
__global__ __launch_bounds__(256) void knn_select_kernel(const float* __restrict__ G, int64_t ldg,
                                                         const float* __restrict__ r, int64_t n, int64_t row0,
                                                         int64_t rows, int k, const float* __restrict__ Y, int T,
                                                         float eps, float alpha, float beta,
                                                         int64_t* __restrict__ nbr, float* __restrict__ w_raw) {
  const int lane = threadIdx.x & 63;
  const int64_t q = (int64_t)blockIdx.x * 4 + wave_id();
  if (q >= rows) return;
  const int64_t i = row0 + q;
  const float ri = r[i];
  const float* g = G + q * ldg;
  float prev_d = -INFINITY;
  int64_t prev_j = -1;
  float dsum = 0.f;
  int64_t my_nbr = -1;  // lane t < k keeps the t-th neighbour
  for (int t = 0; t < k; ++t) {
    float best_d = INFINITY;
    int64_t best_j = INT64_MAX;
    for (int64_t j = lane; j < n; j += 64) {
      if (j == i) continue;
      const float d2 = fmaxf(ri + r[j] - 2.0f * g[j], 0.0f);
      if (lex_less(prev_d, prev_j, d2, j) && lex_less(d2, j, best_d, best_j)) {
        best_d = d2;
        best_j = j;
      }
    }
    // wave-wide lexicographic argmin
    for (int o = 32; o > 0; o >>= 1) {
      const float od = __shfl_xor(best_d, o, 64);
      const int64_t oj = __shfl_xor(best_j, o, 64);
      if (lex_less(od, oj, best_d, best_j)) {
        best_d = od;
        best_j = oj;
      }
    }
    prev_d = best_d;
    prev_j = best_j;
    dsum += sqrtf(best_d);
    if (lane == t) my_nbr = best_j;
    if (nbr && lane == 0) nbr[q * k + t] = best_j;
  }
  // local target variance over the k neighbours (population), averaged over targets
  float vsum = 0.f;
  for (int tt = 0; tt < T; ++tt) {
    const float y = (lane < k) ? Y[my_nbr * T + tt] : 0.f;
    const float mean = wave_sum(y) / (float)k;
    const float dv = (lane < k) ? (y - mean) : 0.f;
    vsum += wave_sum(dv * dv) / (float)k;
  }
  if (lane == 0) {
    const float rho = (float)k / (dsum + eps);
    float w = powf(rho, -alpha);
    w = w / (1.0f + beta * (vsum / (float)T));
    w_raw[i] = w;
  }
}

}  // namespace alignn

using namespace alignn;

static int knn_grid(int64_t work) {
  int64_t g = (work + 255) / 256;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 8192));
}

extern "C" int alignn_col_center_sq_f32(const float* Z, int64_t n, int32_t D, const float* colsum, float* out,
                                        void* stream) {
  if (n < 0 || D <= 0) return ALIGNN_E_BAD_SHAPE;
  if (n == 0) return ALIGNN_OK;
  launch(col_center_sq_kernel, dim3(knn_grid(n * D)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     Z, n, D, colsum, out);
  ALIGNN_LAUNCH_CHECK("col_center_sq_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_standardize_f32(const float* Z, int64_t n, int32_t D, const float* colsum, const float* ssq,
                                      float* out, void* stream) {
  if (n < 0 || D <= 0) return ALIGNN_E_BAD_SHAPE;
  if (n == 0) return ALIGNN_OK;
  launch(standardize_kernel, dim3(knn_grid(n * D)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     Z, n, D, colsum, ssq, out);
  ALIGNN_LAUNCH_CHECK("standardize_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_row_sqnorm_f32(const float* Zs, int64_t n, int32_t D, float* r, void* stream) {
  if (n < 0 || D <= 0) return ALIGNN_E_BAD_SHAPE;
  if (n == 0) return ALIGNN_OK;
  launch(row_sqnorm_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), Zs, n, D, r);
  ALIGNN_LAUNCH_CHECK("row_sqnorm_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_knn_select_weights(const float* G, int64_t ldg, const float* r, int64_t n, int64_t row0,
                                         int64_t rows, int32_t k, const float* Y, int32_t T, float eps, float alpha,
                                         float beta, int64_t* nbr, float* w_raw, void* stream) {
  if (n < 2 || k < 1 || k > 64 || k > n - 1 || T < 1 || row0 < 0 || rows < 0 || row0 + rows > n || ldg < n) {
    set_error("knn_select: need 2 <= n, 1 <= k <= min(64, n-1), T >= 1, rows within n, ldg >= n");
    return ALIGNN_E_BAD_SHAPE;
  }
  if (rows == 0) return ALIGNN_OK;
  launch(knn_select_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), G, ldg, r, n, row0, rows, k, Y, T, eps, alpha, beta, nbr,
                     w_raw);
  ALIGNN_LAUNCH_CHECK("knn_select_kernel");
  return ALIGNN_OK;
}
