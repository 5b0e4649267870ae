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

// All-reduce H per-lane partials over the 64 lanes; every lane receives all H sums.
// H == 4: transpose-reduce (2 + 1 exchanges halve the live values, then 4 plain butterfly steps)
// and 4 readlanes — 7 shuffles instead of 24.
template <int H>
__device__ __forceinline__ void reduce_heads(float (&p)[H], int lane) {
  if constexpr (H == 4) {
    const bool hi = lane >= 32;
    // step xor 32: keep heads {0,1} (lo) or {2,3} (hi)
    float send0 = hi ? p[0] : p[2];
    float send1 = hi ? p[1] : p[3];
    float keep0 = hi ? p[2] : p[0];
    float keep1 = hi ? p[3] : p[1];
    keep0 += __shfl_xor(send0, 32, 64);
    keep1 += __shfl_xor(send1, 32, 64);
    // step xor 16: keep one head
    const bool b4 = (lane >> 4) & 1;
    float send = b4 ? keep0 : keep1;
    float v = b4 ? keep1 : keep0;
    v += __shfl_xor(send, 16, 64);
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    // lane groups: 0-15 head 0, 16-31 head 1, 32-47 head 2, 48-63 head 3
    p[0] = readlane_f(v, 0);
    p[1] = readlane_f(v, 16);
    p[2] = readlane_f(v, 32);
    p[3] = readlane_f(v, 48);
  } else if constexpr (H == 2) {
    const bool hi = lane >= 32;
    float send = hi ? p[0] : p[1];
    float v = hi ? p[1] : p[0];
    v += __shfl_xor(send, 32, 64);
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    p[0] = readlane_f(v, 0);
    p[1] = readlane_f(v, 32);
  } else if constexpr (H == 1) {
    float v = p[0];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    p[0] = readlane_f(v, 0);
  } else {
#pragma unroll
    for (int h = 0; h < H; ++h) {
      float v = p[h];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      p[h] = readlane_f(v, 0);
    }
  }
}

// Branch-free select of element `idx` (runtime, per lane) of a small register array.
template <int H>
__device__ __forceinline__ float pick(const float (&a)[H], int idx) {
  float r = a[0];
#pragma unroll
  for (int h = 1; h < H; ++h) r = (idx == h) ? a[h] : r;
  return r;
}

}  // namespace alignn
