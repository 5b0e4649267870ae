// ensemble.hip — deep-ensemble inference reductions.
//
// ensemble_collect (train.py:849-904) and predict.ensemble_predict (predict.py:582-653) combine M
// heteroscedastic members per graph and target:
//   var_j = exp(max(logvar_j, floor)),  mean = E_j[mu_j],  var = E_j[var_j] + E_j[mu_j^2] - mean^2
//   std_z = sqrt(max(var, 1e-12))
// and predict.py converts to the target scale (log-normal moments):
//   log_mean = mean * s + m, log_std = std_z * s, mean_orig = exp(log_mean)
//   std_lin = sqrt(max((exp(log_std^2) - 1) exp(2 log_mean + log_std^2), 0))
//   ci90 = mean_orig -/+ 1.6448536269514722 std_lin, lower clipped at 0 (predict.py:63, :631-640).
// One thread per (graph, target); members summed in index order.
#include "common.h"

namespace alignn {

__global__ void ensemble_moments_kernel(int M, int64_t B, int T, const float* __restrict__ heads, int64_t sm,
                                        int64_t ldh, float floor_lv, const float* __restrict__ log_means,
                                        const float* __restrict__ log_stds, float* mean_z, float* std_z,
                                        float* mean_orig, float* std_lin, float* lo90, float* hi90) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= B * T) return;
  const int64_t b = i / T;
  const int t = (int)(i - b * T);
  float smu = 0.f, smu2 = 0.f, svar = 0.f;
  for (int j = 0; j < M; ++j) {
    const float* h = heads + j * sm + b * ldh;
    const float mu = h[t];
    const float lv = fmaxf(h[T + t], floor_lv);
    smu += mu;
    smu2 += mu * mu;
    svar += expf(lv);
  }
  const float inv = 1.0f / (float)M;
  const float mean = smu * inv;
  const float var = svar * inv + smu2 * inv - mean * mean;
  const float sd = sqrtf(fmaxf(var, 1e-12f));
  if (mean_z) mean_z[i] = mean;
  if (std_z) std_z[i] = sd;
  if (log_means && log_stds) {
    const float s = log_stds[t];
    const float lm = mean * s + log_means[t];
    const float ls = sd * s;
    const float mo = expf(lm);
    const float vl = (expf(ls * ls) - 1.0f) * expf(2.0f * lm + ls * ls);
    const float sl = sqrtf(fmaxf(vl, 0.0f));
    if (mean_orig) mean_orig[i] = mo;
    if (std_lin) std_lin[i] = sl;
    const float z90 = 1.6448536269514722f;
    if (lo90) lo90[i] = fmaxf(mo - z90 * sl, 0.0f);
    if (hi90) hi90[i] = mo + z90 * sl;
  }
}

// out[i] = (1/M) sum_j x[j*sm + i] (ensemble_collect_embeddings, train.py:907-927)
__global__ void member_mean_kernel(int M, int64_t n, const float* __restrict__ x, int64_t sm, float* __restrict__ out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int j = 0; j < M; ++j) s += x[j * sm + i];
  out[i] = s / (float)M;
}

}  // namespace alignn

using namespace alignn;

extern "C" int alignn_ensemble_moments(int32_t M, int64_t B, int32_t T, const float* heads, int64_t member_stride,
                                       int64_t ldh, float min_logvar_floor, const float* log_means,
                                       const float* log_stds, float* mean_z, float* std_z, float* mean_orig,
                                       float* std_lin, float* lo90, float* hi90, void* stream) {
  if (M < 1 || B < 0 || T < 1 || ldh < 2 * (int64_t)T) {
    set_error("ensemble_moments: need M >= 1, T >= 1, ldh >= 2T (M=%d T=%d ldh=%lld)", M, T, (long long)ldh);
    return ALIGNN_E_BAD_SHAPE;
  }
  if (B == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = B * T;
  launch(ensemble_moments_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, M, B, T, heads,
                     member_stride, ldh, min_logvar_floor, log_means, log_stds, mean_z, std_z, mean_orig, std_lin,
                     lo90, hi90);
  ALIGNN_LAUNCH_CHECK("ensemble_moments_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_member_mean_f32(int32_t M, int64_t n, const float* x, int64_t member_stride, float* out,
                                      void* stream) {
  if (M < 1 || n < 0) return ALIGNN_E_BAD_SHAPE;
  if (n == 0) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  launch(member_mean_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, M, n, x, member_stride,
                     out);
  ALIGNN_LAUNCH_CHECK("member_mean_kernel");
  return ALIGNN_OK;
}
