// common.h — shared device helpers for libalignn_hip (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <tuple>
#include <type_traits>
#include <utility>

#include "../../include/alignn_hip.h"

#define ALIGNN_WAVE 64

namespace alignn {

// Index of this thread's wavefront in its workgroup, as a wave-uniform (SGPR) value.  Plain
// threadIdx.x >> 6 is uniform per wave64 too, but the compiler's divergence analysis cannot see
// it: every address derived from it then stays in VGPRs, index loads become vector loads, and the
// s_waitcnt vmcnt(0) that guards each dependent load also waits for every prefetch in flight
// (measured in the attention kernels' ISA: one full memory round trip per edge).
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

// Load of a kernel-invariant value at a wave-uniform address through the constant address space,
// so it is a scalar (s_load) load: its s_waitcnt lgkmcnt does not wait for the vector loads in
// flight.  Only for arrays no kernel thread writes (CSR offsets, index lists).
template <typename T>
__device__ __forceinline__ T sld(const T* p, int64_t i) {
  return ((const __attribute__((address_space(4))) T*)p)[i];
}

// ---------------------------------------------------------------------------------------------
// Error handling (no exceptions cross the ABI)
// ---------------------------------------------------------------------------------------------
void set_error(const char* fmt, ...);
int hip_status(hipError_t e, const char* what);

#define ALIGNN_LAUNCH_CHECK(what)                                 \
  do {                                                            \
    hipError_t _e = hipGetLastError();                            \
    if (_e != hipSuccess) return ::alignn::hip_status(_e, what);  \
  } while (0)

// ---------------------------------------------------------------------------------------------
// Kernel launches.  Every kernel of the library goes through launch(): the arguments are
// converted to the kernel's parameter types and passed by address to hipLaunchKernel.  While a
// launch plan is being recorded (plan.hip, alignn_plan_begin), the launch is also appended to it —
// kernel, grid, block, LDS bytes, stream and a copy of the argument bytes — so the plan can issue
// the same step again from C++ (alignn_plan_replay) without any per-launch host work above HIP.
// ---------------------------------------------------------------------------------------------
// Recording state is per host thread (a plan records the launches its own thread issues), so
// independent callers on other threads neither see nor disturb it.
extern thread_local bool g_recording;
void record_launch(const void* func, dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, void* const* args,
                   const size_t* sizes, const size_t* aligns, const unsigned char* kinds, int nargs);

// Argument kinds kept with a recorded launch, for the plan's pointer-ownership check
// (alignn_plan_check_ptrs): 1 = device pointer, 2 = struct (its 8-byte words are scanned), 0 = scalar.
template <typename T>
constexpr unsigned char arg_kind() {
  return std::is_pointer<T>::value ? 1 : (std::is_class<T>::value ? 2 : 0);
}

template <typename... P, typename... A>
inline void launch(void (*kernel)(P...), dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, A&&... a) {
  static_assert(sizeof...(P) == sizeof...(A), "launch: argument count differs from the kernel's");
  std::tuple<std::decay_t<P>...> vals(static_cast<std::decay_t<P>>(a)...);
  void* ptrs[sizeof...(P) + 1];
  std::apply([&](auto&... v) { int i = 0; ((ptrs[i++] = (void*)&v), ...); }, vals);
  if (g_recording) {
    const size_t sizes[sizeof...(P) + 1] = {sizeof(std::decay_t<P>)..., 0};
    const size_t aligns[sizeof...(P) + 1] = {alignof(std::decay_t<P>)..., 1};
    const unsigned char kinds[sizeof...(P) + 1] = {arg_kind<std::decay_t<P>>()..., 0};
    record_launch(reinterpret_cast<const void*>(kernel), grid, block, shmem, s, ptrs, sizes, aligns, kinds,
                  (int)sizeof...(P));
  }
  // a failure is left in hipGetLastError for the caller's ALIGNN_LAUNCH_CHECK
  (void)hipLaunchKernel(reinterpret_cast<const void*>(kernel), grid, block, ptrs, shmem, s);
}

// ---------------------------------------------------------------------------------------------
// Wave-level reductions (64 lanes).  __shfl_xor lowers to DPP/ds_swizzle/bpermute as the
// compiler sees fit; the 32-lane stage crosses the two halves.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// Sum within aligned groups of `width` lanes (width power of two <= 64).
__device__ __forceinline__ float group_sum(float v, int width) {
  for (int o = width >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------------------------------------
// Counter-based random numbers (dropout masks / jitter).  Each call site gets its own 64-bit
// seed from the host; the element counter makes the mask reproducible in the backward pass.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  uint64_t x = seed ^ (idx * 0x9E3779B97F4A7C15ULL);
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)(x >> 32);
}
// keep-probability (1-p) Bernoulli, returns the dropout multiplier (0 or 1/(1-p)).
__device__ __forceinline__ float dropout_mul(uint64_t seed, uint64_t idx, uint32_t thresh, float inv_keep) {
  return hash_u32(seed, idx) >= thresh ? inv_keep : 0.0f;
}

// Device-resident step seed registered by alignn_set_step_seed (NULL: host seeds only).  Per host
// thread: the registering caller's launches (and the plans they record) carry its pointer.
extern thread_local const uint64_t* g_step_seed;

__device__ __forceinline__ uint64_t mix_seed(uint64_t site, const uint64_t* sptr) {
  if (!sptr) return site;
  uint64_t x = (*sptr + 0x632BE59BD9B4E019ULL) * 0x9E3779B97F4A7C15ULL;
  x ^= x >> 31;
  return site ^ x;
}

struct DropParams {
  uint64_t seed;
  uint32_t thresh;   // p * 2^32
  float inv_keep;    // 1/(1-p)
  int active;
  int pad_;              // explicit: kernel-argument structs have no undefined bytes (plan.hip)
  const uint64_t* sptr;  // step seed (mixed in once per thread: resolve_drop)
};
// Call once at kernel entry: folds the device step seed into d.seed.
__device__ __forceinline__ void resolve_drop(DropParams& d) {
  d.seed = mix_seed(d.seed, d.sptr);
  d.sptr = nullptr;
}
inline DropParams make_drop(float p, uint64_t seed) {
  DropParams d;
  d.seed = seed;
  d.sptr = g_step_seed;
  d.active = p > 0.0f ? 1 : 0;
  d.pad_ = 0;
  double t = (double)p * 4294967296.0;
  d.thresh = p > 0.0f ? (uint32_t)(t >= 4294967295.0 ? 4294967295.0 : t) : 0u;
  d.inv_keep = p < 1.0f ? 1.0f / (1.0f - p) : 0.0f;
  return d;
}

// Fixed-order column reduction of a [rows, N] partial buffer: out[c] (+)= sum_r part[r*N + c].
// Grid: ceil(N/16) blocks of 256 threads (16 row-lanes x 16 columns); each thread keeps four
// independent partial sums (rows ty, ty+16, ty+32, ty+48 of every 64-row stride) so 16 x 4 loads
// per column are in flight; the 16 row-lanes are combined in lane order.  Blocks of 256 threads
// (not 1024) find room on a CU beside a side-stream kernel that fills it (a 1024-thread block
// waited up to 80 us on the critical path, profiles/r01/v15_kernel_stats.csv).
constexpr int kColsumThreads = 256;
constexpr int kColsumCols = 16;
template <int kUnused = 0>
__global__ __launch_bounds__(256) void colsum_stage2(const float* __restrict__ part, int rows, int64_t N,
                                                     float* __restrict__ out, int acc) {
  __shared__ float red[16][kColsumCols];
  const int tx = threadIdx.x % kColsumCols, ty = threadIdx.x / kColsumCols;
  const int64_t col = (int64_t)blockIdx.x * kColsumCols + tx;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (col < N) {
    int r = ty;
    // Four iterations' loads issued before any is summed (16 requests in flight per thread instead
    // of 4: the pass is latency-bound at ~1,000 partial rows over 80 workgroups); the sums are taken
    // in the one-iteration order, so the result is bitwise the same as the loop below.
    for (; r + 240 < rows; r += 256) {
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = part[(int64_t)(r + 16 * i) * N + col];
#pragma unroll
      for (int i = 0; i < 16; i += 4) {
        s0 += v[i];
        s1 += v[i + 1];
        s2 += v[i + 2];
        s3 += v[i + 3];
      }
    }
    for (; r + 48 < rows; r += 64) {
      s0 += part[(int64_t)r * N + col];
      s1 += part[(int64_t)(r + 16) * N + col];
      s2 += part[(int64_t)(r + 32) * N + col];
      s3 += part[(int64_t)(r + 48) * N + col];
    }
    for (; r < rows; r += 16) s0 += part[(int64_t)r * N + col];
  }
  red[ty][tx] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (ty == 0 && col < N) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][tx];
    out[col] = acc ? out[col] + t : t;
  }
}
static inline unsigned colsum_blocks(int64_t N) { return (unsigned)((N + kColsumCols - 1) / kColsumCols); }

}  // namespace alignn
