// vec.h — VPL-wide register vectors (VPL fp32 values per lane, contiguous in memory).
#pragma once
#include <hip/hip_runtime.h>

namespace alignn {

template <int VPL>
__device__ __forceinline__ void vload(const float* __restrict__ p, float (&v)[VPL]) {
  if constexpr (VPL == 4) {
    float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else if constexpr (VPL == 2) {
    float2 t = *reinterpret_cast<const float2*>(p);
    v[0] = t.x; v[1] = t.y;
  } else if constexpr (VPL == 8) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int i = 0; i < VPL; ++i) v[i] = p[i];
  }
}

template <int VPL>
__device__ __forceinline__ void vstore(float* __restrict__ p, const float (&v)[VPL]) {
  if constexpr (VPL == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else if constexpr (VPL == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
  } else if constexpr (VPL == 8) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
#pragma unroll
    for (int i = 0; i < VPL; ++i) p[i] = v[i];
  }
}

// VPL bf16 values (contiguous) widened to fp32 (exact); VPL % 4 == 0 loads 8 bytes per four
template <int VPL>
__device__ __forceinline__ void vload_bf(const uint16_t* __restrict__ p, float (&v)[VPL]) {
  if constexpr (VPL % 4 == 0) {
#pragma unroll
    for (int q = 0; q < VPL / 4; ++q) {
      const uint2 u = *reinterpret_cast<const uint2*>(p + 4 * q);
      v[4 * q] = __builtin_bit_cast(float, u.x << 16);
      v[4 * q + 1] = __builtin_bit_cast(float, u.x & 0xffff0000u);
      v[4 * q + 2] = __builtin_bit_cast(float, u.y << 16);
      v[4 * q + 3] = __builtin_bit_cast(float, u.y & 0xffff0000u);
    }
  } else {
#pragma unroll
    for (int i = 0; i < VPL; ++i) v[i] = __builtin_bit_cast(float, (uint32_t)p[i] << 16);
  }
}

// VPL fp32 values rounded to bf16 (RNE) and stored contiguously
template <int VPL>
__device__ __forceinline__ void vstore_bf(uint16_t* __restrict__ p, const float (&v)[VPL]) {
  auto rne = [](float x) { return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)x); };
  if constexpr (VPL % 4 == 0) {
#pragma unroll
    for (int q = 0; q < VPL / 4; ++q) {
      uint2 u;
      u.x = rne(v[4 * q]) | (rne(v[4 * q + 1]) << 16);
      u.y = rne(v[4 * q + 2]) | (rne(v[4 * q + 3]) << 16);
      *reinterpret_cast<uint2*>(p + 4 * q) = u;
    }
  } else {
#pragma unroll
    for (int i = 0; i < VPL; ++i) p[i] = (uint16_t)rne(v[i]);
  }
}

template <int VPL>
__device__ __forceinline__ void vzero(float (&v)[VPL]) {
#pragma unroll
  for (int i = 0; i < VPL; ++i) v[i] = 0.f;
}

template <int VPL>
__device__ __forceinline__ float vdot(const float (&a)[VPL], const float (&b)[VPL]) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) s = fmaf(a[i], b[i], s);
  return s;
}

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}

// Wave-uniform value (index loaded from memory at a uniform address) moved to an SGPR, so the
// addresses derived from it are scalar (global_load with SGPR base + one shared VGPR offset).
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ float f_bits(unsigned u) { return __builtin_bit_cast(float, u); }
__device__ __forceinline__ unsigned u_bits(float f) { return __builtin_bit_cast(unsigned, f); }

// x summed over its 16-lane row (every lane of the row gets the sum): DPP quad_perm xor1, xor2,
// row_half_mirror, row_mirror — each fused into a v_add_f32_dpp.
__device__ __forceinline__ float row_sum16(float x) {
  x += f_bits((unsigned)__builtin_amdgcn_update_dpp(0, (int)u_bits(x), 0xB1, 0xF, 0xF, true));   // quad_perm [1,0,3,2]
  x += f_bits((unsigned)__builtin_amdgcn_update_dpp(0, (int)u_bits(x), 0x4E, 0xF, 0xF, true));   // quad_perm [2,3,0,1]
  x += f_bits((unsigned)__builtin_amdgcn_update_dpp(0, (int)u_bits(x), 0x141, 0xF, 0xF, true));  // row_half_mirror
  x += f_bits((unsigned)__builtin_amdgcn_update_dpp(0, (int)u_bits(x), 0x140, 0xF, 0xF, true));  // row_mirror
  return x;
}

// All-reduce N per-lane partials over the 64 lanes and broadcast: afterwards every lane holds all
// N sums (wave-uniform).  Select-free transpose-reduction: v_permlane32_swap pairs value i with
// value i+P/2 across the two wave halves (lanes < 32 keep the first half of the values, lanes >= 32
// the second), v_permlane16_swap does the same across rows of 16, then each remaining value is
// summed within its row by DPP and row r's values are read out with v_readlane.
// N = 16: 12 swaps + 12 adds + 16 DPP adds + 16 readlanes (vs 96 shuffles for 16 butterflies).
template <int N>
__device__ __forceinline__ void reduce_bcast(float (&v)[N], int lane) {
  (void)lane;
  constexpr int P = (N + 3) / 4 * 4;
  float a[P / 2];
#pragma unroll
  for (int i = 0; i < P / 2; ++i) {
    const float x = i < N ? v[i] : 0.f;
    const float y = (i + P / 2) < N ? v[i + P / 2] : 0.f;
    const auto r = __builtin_amdgcn_permlane32_swap(u_bits(x), u_bits(y), false, false);
    a[i] = f_bits(r[0]) + f_bits(r[1]);
  }
  float b[P / 4];
#pragma unroll
  for (int i = 0; i < P / 4; ++i) {
    const auto r = __builtin_amdgcn_permlane16_swap(u_bits(a[i]), u_bits(a[i + P / 4]), false, false);
    b[i] = row_sum16(f_bits(r[0]) + f_bits(r[1]));
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int i = 0; i < P / 4; ++i)
      if (r * (P / 4) + i < N) v[r * (P / 4) + i] = readlane_f(b[i], 16 * r);
}

template <int H>
__device__ __forceinline__ void reduce_heads(float (&p)[H], int lane) {
  reduce_bcast<H>(p, lane);
}

// Branch-free select of element `idx` (runtime, per lane) of a small register array.
template <int H>
__device__ __forceinline__ float pick(const float (&a)[H], int idx) {
  float r = a[0];
#pragma unroll
  for (int h = 1; h < H; ++h) r = (idx == h) ? a[h] : r;
  return r;
}

// pick<H> with every candidate laundered through an empty asm: the optimizer otherwise folds the
// select chain into a dynamically indexed load of the array, which forces the array into scratch
// memory (private segment) — observed on the attention kernels' per-head state arrays.
__device__ __forceinline__ float launder(float v) {
  asm volatile("" : "+v"(v));
  return v;
}

template <int H>
__device__ __forceinline__ float pick_r(const float (&a)[H], int idx) {
  float r = launder(a[0]);
#pragma unroll
  for (int h = 1; h < H; ++h) r = (idx == h) ? launder(a[h]) : r;
  return r;
}

}  // namespace alignn
