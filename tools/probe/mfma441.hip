// Probe: v_mfma_f32_4x4x1f32 (16 blocks) as a k-chain of fused multiply-adds, against an fmaf chain.
// Lane l: A = x[l & 3][k], B = W[4 * l + m][k]; expects D[l][r] = sum_k x[r][k] W[4l+m][k] if the
// output register index is the A row.  Prints mismatch counts for both operand orders.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int K = 11;
__global__ void probe(const float* x, const float* W, float* out_mfma_ab, float* out_mfma_ba, float* out_fma) {
  const int l = threadIdx.x;
  for (int m = 0; m < 4; ++m) {
    v4f c = {0.f, 0.f, 0.f, 0.f}, c2 = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) {
      const float a = x[(l & 3) * K + k];
      const float b = W[(4 * l + m) * K + k];
      c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(b, a, c2, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) {
      out_mfma_ab[(l * 4 + m) * 4 + r] = c[r];
      out_mfma_ba[(l * 4 + m) * 4 + r] = c2[r];
      float acc = 0.f;
      for (int k = 0; k < K; ++k) acc = fmaf(x[r * K + k], W[(4 * l + m) * K + k], acc);
      out_fma[(l * 4 + m) * 4 + r] = acc;
    }
  }
}
int main() {
  srand(1);
  float hx[4 * K], hW[256 * K];
  int bad_ab = 0, bad_ba = 0, bad_ab_close = 0;
  float *dx, *dW, *d1, *d2, *d3;
  hipMalloc(&dx, sizeof hx); hipMalloc(&dW, sizeof hW);
  hipMalloc(&d1, 1024 * 4); hipMalloc(&d2, 1024 * 4); hipMalloc(&d3, 1024 * 4);
  float o1[1024], o2[1024], o3[1024];
  for (int trial = 0; trial < 200; ++trial) {
    for (auto& v : hx) v = (rand() / (float)RAND_MAX - 0.5f) * 4.f;
    for (auto& v : hW) v = (rand() / (float)RAND_MAX - 0.5f) * 0.6f;
    hipMemcpy(dx, hx, sizeof hx, hipMemcpyHostToDevice);
    hipMemcpy(dW, hW, sizeof hW, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dx, dW, d1, d2, d3);
    hipMemcpy(o1, d1, sizeof o1, hipMemcpyDeviceToHost);
    hipMemcpy(o2, d2, sizeof o2, hipMemcpyDeviceToHost);
    hipMemcpy(o3, d3, sizeof o3, hipMemcpyDeviceToHost);
    for (int i = 0; i < 1024; ++i) {
      bad_ab += memcmp(&o1[i], &o3[i], 4) != 0;
      bad_ba += memcmp(&o2[i], &o3[i], 4) != 0;
      bad_ab_close += fabsf(o1[i] - o3[i]) > 1e-5f * (1.f + fabsf(o3[i]));
    }
  }
  printf("mfma(a=x,b=W) bitwise mismatches %d / %d (not close: %d); mfma(a=W,b=x) mismatches %d\n", bad_ab,
         200 * 1024, bad_ab_close, bad_ba);
  return 0;
}
