// optim.hip — gradient clipping + AdamW over the flat parameter buffer.
//
// Reference (scripts/train.py:693-699, :1532-1542): torch.nn.utils.clip_grad_norm_(params, 5.0)
// then torch.optim.AdamW (fused, betas (0.9, 0.999), eps 1e-8, decoupled weight decay) over two
// param groups — base + mean heads | logvar heads — which the flat layout keeps as two contiguous
// segments [0, split) and [split, n) with their own learning rates.
//   clip:  norm = ||g||_2 ;  c = min(max_norm / (norm + 1e-6), 1) ;  g *= c
//   AdamW: step += 1 ; p *= 1 - lr*wd ; m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2 ;
//          p -= (lr / (1 - b1^step)) * m / (sqrt(v) / sqrt(1 - b2^step) + eps)
// The norm is a fixed-order two-stage reduction (deterministic); the step counter and the norm live
// in device memory, so the update can sit inside a captured HIP graph.
#include "common.h"

namespace alignn {

constexpr int kNormBlocks = 1024;

__global__ __launch_bounds__(256) void sumsq_stage1(const float* __restrict__ g, int64_t n, float* __restrict__ part) {
  __shared__ float red[4];
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t b0 = (int64_t)blockIdx.x * per, b1 = min(n, b0 + per);
  float s0 = 0.f, s1 = 0.f;
  int64_t i = b0 + threadIdx.x;
  for (; i + 256 < b1; i += 512) {
    const float x = g[i], y = g[i + 256];
    s0 = fmaf(x, x, s0);
    s1 = fmaf(y, y, s1);
  }
  for (; i < b1; i += 256) s0 = fmaf(g[i], g[i], s0);
  float s = wave_sum(s0 + s1);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void sumsq_stage2(const float* __restrict__ part, int nparts, float* __restrict__ norm) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *norm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
}

__global__ void step_inc_kernel(float* step) { *step += 1.0f; }

__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                    float* __restrict__ v, int64_t n, int64_t split, float lr0,
                                                    float lr1, float wd, float b1, float b2, float eps,
                                                    const float* __restrict__ norm, float max_norm,
                                                    const float* __restrict__ step) {
  const float t = *step;
  const float bc1 = 1.0f - powf(b1, t);
  const float bc2s = sqrtf(1.0f - powf(b2, t));
  float c = 1.0f;
  if (norm) c = fminf(max_norm / (*norm + 1e-6f), 1.0f);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float lr = i < split ? lr0 : lr1;
    const float gi = g[i] * c;
    g[i] = gi;  // clip_grad_norm_ scales the gradients in place
    float pi = p[i] * (1.0f - lr * wd);
    const float mi = b1 * m[i] + (1.0f - b1) * gi;
    const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    pi -= (lr / bc1) * mi / (sqrtf(vi) / bc2s + eps);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

}  // namespace alignn

using namespace alignn;

extern "C" int alignn_grad_norm_f32(const float* g, int64_t n, float* norm, float* workspace, void* stream) {
  if (n < 0 || !norm || !workspace) return ALIGNN_E_BAD_SHAPE;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int parts = (int)std::max<int64_t>(1, std::min<int64_t>(kNormBlocks, (n + 4095) / 4096));
  hipLaunchKernelGGL(sumsq_stage1, dim3(parts), dim3(256), 0, s, g, n, workspace);
  hipLaunchKernelGGL(sumsq_stage2, dim3(1), dim3(256), 0, s, workspace, parts, norm);
  ALIGNN_LAUNCH_CHECK("grad norm");
  return ALIGNN_OK;
}

extern "C" int alignn_adamw_f32(float* p, float* g, float* m, float* v, int64_t n, int64_t split, float lr0,
                                float lr1, float weight_decay, float beta1, float beta2, float eps,
                                const float* norm, float max_norm, float* step, void* stream) {
  if (n < 0 || split < 0 || split > n || !step) return ALIGNN_E_BAD_SHAPE;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, s, step);
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  if (n > 0)
    hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, g, m, v, n, split, lr0, lr1,
                       weight_decay, beta1, beta2, eps, norm, max_norm, step);
  ALIGNN_LAUNCH_CHECK("adamw_kernel");
  return ALIGNN_OK;
}
