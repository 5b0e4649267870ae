// optim.hip — gradient clipping + AdamW over the flat parameter buffer.
//
// Reference (scripts/train.py:693-699, :1532-1542): torch.nn.utils.clip_grad_norm_(params, 5.0)
// then torch.optim.AdamW (betas (0.9, 0.999), eps 1e-8, decoupled weight decay; fused on a GPU,
// the single-tensor loop on the CPU path this engine is held to) over two param groups — base +
// mean heads | logvar heads — which the flat layout keeps as two contiguous segments [0, split)
// and [split, n) with their own learning rates.
//   clip:  norm = ||g||_2 ;  c = min(max_norm / (norm + 1e-6), 1) ;  g *= c
//   AdamW: step += 1 ; p *= 1 - lr*wd ; m = lerp(m, g, 1-b1) ; v = b2 v + (1-b2) g^2 ;
//          p -= (lr / (1 - b1^step)) * m / (sqrt(v) / sqrt(1 - b2^step) + eps)
// The norm is a fixed-order two-stage reduction (deterministic); the step counter and the norm live
// in device memory, so the update can sit inside a captured HIP graph.
#include "common.h"

namespace alignn {

constexpr int kNormBlocks = 1024;

// AMP: the same sums, plus GradScaler's found-inf test of each element (flag[blockIdx] = 1 when some
// g * scale is inf / NaN: the reference's backward runs on the scaled loss, torch.amp.GradScaler,
// train.py:690-695, and unscale_ flags a step whose scaled gradients overflowed or were non-finite)
template <bool AMP>
__global__ __launch_bounds__(256) void sumsq_stage1(const float* __restrict__ g, int64_t n, float* __restrict__ part,
                                                    const float* __restrict__ scaler, float* __restrict__ flag) {
  __shared__ float red[4];
  __shared__ int bad[4];
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t b0 = (int64_t)blockIdx.x * per, b1 = min(n, b0 + per);
  const float scale = AMP ? scaler[0] : 1.0f;
  float s0 = 0.f, s1 = 0.f;
  bool nf = false;
  int64_t i = b0 + threadIdx.x;
  // four iterations' loads in flight before any is summed, summed in the one-iteration order below
  // (bitwise the same norm; a block's ~4k elements were 8 dependent round trips per lane)
  for (; i + 1792 < b1; i += 2048) {
    float x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = g[i + 256 * k];
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
      s0 = fmaf(x[k], x[k], s0);
      s1 = fmaf(x[k + 1], x[k + 1], s1);
      if (AMP) nf |= !__builtin_isfinite(x[k] * scale) || !__builtin_isfinite(x[k + 1] * scale);
    }
  }
  for (; i + 256 < b1; i += 512) {
    const float x = g[i], y = g[i + 256];
    s0 = fmaf(x, x, s0);
    s1 = fmaf(y, y, s1);
    if (AMP) nf |= !__builtin_isfinite(x * scale) || !__builtin_isfinite(y * scale);
  }
  for (; i < b1; i += 256) {
    const float x = g[i];
    s0 = fmaf(x, x, s0);
    if (AMP) nf |= !__builtin_isfinite(x * scale);
  }
  float s = wave_sum(s0 + s1);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  if (AMP) {
    const bool any = __any(nf);
    if ((threadIdx.x & 63) == 0) bad[threadIdx.x >> 6] = any ? 1 : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
    if (AMP) flag[blockIdx.x] = (bad[0] | bad[1] | bad[2] | bad[3]) ? 1.0f : 0.0f;
  }
}

template <bool AMP>
__global__ __launch_bounds__(256) void sumsq_stage2(const float* __restrict__ part, int nparts, float* __restrict__ norm,
                                                    const float* __restrict__ flag, float* __restrict__ scaler) {
  __shared__ float red[4];
  __shared__ float bad[4];
  float s = 0.f, f = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) {
    s += part[i];
    if (AMP) f = fmaxf(f, flag[i]);
  }
  s = wave_sum(s);
  if (AMP) f = wave_max(f);
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = s;
    if (AMP) bad[threadIdx.x >> 6] = f;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    *norm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    if (AMP) scaler[2] = fmaxf(fmaxf(bad[0], bad[1]), fmaxf(bad[2], bad[3]));   // found_inf
  }
}

__global__ void step_inc_kernel(float* step) { *step += 1.0f; }

// GradScaler.step + update (torch.amp, defaults: growth 2, backoff 0.5): a step whose gradients were
// flagged is skipped (no AdamW update, the step count stays) and the scale halves; otherwise the step
// counts and after growth_interval clean steps in a row the scale doubles.
// scaler: [scale, growth_tracker, found_inf, skipped steps]
__global__ void step_amp_kernel(float* step, float* scaler, int growth_interval) {
  if (scaler[2] != 0.0f) {
    scaler[0] *= 0.5f;
    scaler[1] = 0.0f;
    scaler[3] += 1.0f;
    return;
  }
  *step += 1.0f;
  const float t = scaler[1] + 1.0f;
  if (t >= (float)growth_interval) {
    const float grown = scaler[0] * 2.0f;
    if (__builtin_isfinite(grown)) scaler[0] = grown;
    scaler[1] = 0.0f;
  } else {
    scaler[1] = t;
  }
}

__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                    float* __restrict__ v, int64_t n, int64_t split, double lr0,
                                                    double lr1, double wd, double b1, double b2, float eps,
                                                    const float* __restrict__ norm, float max_norm,
                                                    const float* __restrict__ step, const double* __restrict__ lr_dev,
                                                    const float* __restrict__ scaler) {
  if (scaler && scaler[2] != 0.0f) return;   // GradScaler skipped this step: parameters and moments stay
  // The reference's CPU AdamW (torch _single_tensor_adam, decoupled decay) forms its scalars as
  // Python doubles and rounds each to fp32 once where a tensor op consumes it: 1 - lr*wd, 1 - b1
  // (lerp weight), 1 - b2 (addcmul value), lr / (1 - b1^t), sqrt(1 - b2^t).  Same here.
  const double t = (double)*step;
  if (lr_dev) {  // device-resident learning rates (a recorded plan follows the schedule)
    lr0 = lr_dev[0];
    lr1 = lr_dev[1];
  }
  const float omb1 = (float)(1.0 - b1), omb2 = (float)(1.0 - b2), fb2 = (float)b2;
  const float bc2s = (float)sqrt(1.0 - pow(b2, t));
  const double bc1 = 1.0 - pow(b1, t);
  const float ss0 = (float)(lr0 / bc1), ss1 = (float)(lr1 / bc1);
  const float dec0 = (float)(1.0 - lr0 * wd), dec1 = (float)(1.0 - lr1 * wd);
  float c = 1.0f;
  if (norm) c = fminf(max_norm / (*norm + 1e-6f), 1.0f);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool g0 = i < split;
    const float gi = g[i] * c;
    g[i] = gi;  // clip_grad_norm_ scales the gradients in place
    const float pi = p[i] * (g0 ? dec0 : dec1);
    const float m0 = m[i];
    const float mi = m0 + omb1 * (gi - m0);            // lerp_(g, 1 - b1), weight < 0.5 branch
    const float vi = v[i] * fb2 + omb2 * gi * gi;       // mul_(b2).addcmul_(g, g, value=1 - b2)
    const float den = sqrtf(vi) / bc2s + eps;
    p[i] = pi + (-(g0 ? ss0 : ss1)) * mi / den;        // addcdiv_(m, denom, value=-step_size)
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
  launch(sumsq_stage1<false>, dim3(parts), dim3(256), 0, s, g, n, workspace, nullptr, nullptr);
  launch(sumsq_stage2<false>, dim3(1), dim3(256), 0, s, workspace, parts, norm, nullptr, nullptr);
  ALIGNN_LAUNCH_CHECK("grad norm");
  return ALIGNN_OK;
}

extern "C" int alignn_grad_norm_amp_f32(const float* g, int64_t n, float* norm, float* scaler, float* workspace,
                                        void* stream) {
  if (n < 0 || !norm || !workspace || !scaler) return ALIGNN_E_BAD_SHAPE;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int parts = (int)std::max<int64_t>(1, std::min<int64_t>(kNormBlocks, (n + 4095) / 4096));
  launch(sumsq_stage1<true>, dim3(parts), dim3(256), 0, s, g, n, workspace, scaler, workspace + kNormBlocks);
  launch(sumsq_stage2<true>, dim3(1), dim3(256), 0, s, workspace, parts, norm, workspace + kNormBlocks, scaler);
  ALIGNN_LAUNCH_CHECK("grad norm (amp)");
  return ALIGNN_OK;
}

static int adamw(float* p, float* g, float* m, float* v, int64_t n, int64_t split, double lr0, double lr1,
                 const double* lr_dev, double weight_decay, double beta1, double beta2, double eps, const float* norm,
                 float max_norm, float* step, float* scaler, int growth_interval, void* stream) {
  if (n < 0 || split < 0 || split > n || !step || (scaler && growth_interval < 1)) return ALIGNN_E_BAD_SHAPE;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (scaler)
    launch(step_amp_kernel, dim3(1), dim3(1), 0, s, step, scaler, growth_interval);
  else
    launch(step_inc_kernel, dim3(1), dim3(1), 0, s, step);
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
  if (n > 0)
    launch(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, g, m, v, n, split, lr0, lr1,
                       weight_decay, beta1, beta2, (float)eps, norm, max_norm, step, lr_dev, scaler);
  ALIGNN_LAUNCH_CHECK("adamw_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_adamw_f32(float* p, float* g, float* m, float* v, int64_t n, int64_t split, double lr0,
                                double lr1, double weight_decay, double beta1, double beta2, double eps,
                                const float* norm, float max_norm, float* step, void* stream) {
  return adamw(p, g, m, v, n, split, lr0, lr1, nullptr, weight_decay, beta1, beta2, eps, norm, max_norm, step, nullptr,
               0, stream);
}

extern "C" int alignn_adamw_f32_dev(float* p, float* g, float* m, float* v, int64_t n, int64_t split,
                                    const double* lr, double weight_decay, double beta1, double beta2, double eps,
                                    const float* norm, float max_norm, float* step, void* stream) {
  if (!lr) return ALIGNN_E_BAD_SHAPE;
  return adamw(p, g, m, v, n, split, 0.0, 0.0, lr, weight_decay, beta1, beta2, eps, norm, max_norm, step, nullptr, 0,
               stream);
}

extern "C" int alignn_adamw_amp_f32_dev(float* p, float* g, float* m, float* v, int64_t n, int64_t split,
                                        const double* lr, double weight_decay, double beta1, double beta2, double eps,
                                        const float* norm, float max_norm, float* step, float* scaler,
                                        int32_t growth_interval, void* stream) {
  if (!lr || !scaler) return ALIGNN_E_BAD_SHAPE;
  return adamw(p, g, m, v, n, split, 0.0, 0.0, lr, weight_decay, beta1, beta2, eps, norm, max_norm, step, scaler,
               growth_interval, stream);
}
