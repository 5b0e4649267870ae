// Layout probe for v_mfma_f32_4x4x4_16b_bf16 (gfx950): which accumulator (lane, reg) entries an A or
// B operand element (lane, element) reaches.  Prints one JSON object.  Build: see tools/job_r3_h.sh.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void probe(float* out, int which) {
  // which < 256: A one-hot at (lane which/4, element which%4), B all ones;
  // else B one-hot at ((which-256)/4, (which-256)%4), A all ones.
  const int l = threadIdx.x;
  bf4 a, b;
  for (int j = 0; j < 4; ++j) {
    const bool hitA = which < 256 && l == which / 4 && j == which % 4;
    const bool hitB = which >= 256 && l == (which - 256) / 4 && j == (which - 256) % 4;
    a[j] = (__bf16)(which < 256 ? (hitA ? 1.f : 0.f) : 1.f);
    b[j] = (__bf16)(which >= 256 ? (hitB ? 1.f : 0.f) : 1.f);
  }
  f4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(__builtin_bit_cast(s4, a), __builtin_bit_cast(s4, b), c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}

int main() {
  float* d;
  hipMalloc(&d, 256 * sizeof(float));
  float h[256];
  printf("{");
  for (int w = 0; w < 512; ++w) {
    probe<<<1, 64>>>(d, w);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("%s\"%d\": [", w ? ", " : "", w);
    bool first = true;
    for (int i = 0; i < 256; ++i)
      if (h[i] != 0.f) { printf("%s[%d, %d, %g]", first ? "" : ", ", i / 4, i % 4, h[i]); first = false; }
    printf("]");
  }
  printf("}\n");
  hipFree(d);
  return 0;
}
