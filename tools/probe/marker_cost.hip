// Cost of a cross-stream event edge on the SOURCE stream: a stream runs N pairs of short kernels;
// variant 0 nothing in between, 1 hipEventRecord on the stream between them (another stream waits
// on the event), 2 the same with a stream-ordered write of a flag instead (hipStreamWriteValue32) and
// hipStreamWaitValue32 on the other stream.  Prints the source stream's time per pair.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void spin(float* x, int iters) {
  float v = x[threadIdx.x + blockIdx.x * blockDim.x];
  for (int i = 0; i < iters; ++i) v = v * 0.999f + 0.001f;
  x[threadIdx.x + blockIdx.x * blockDim.x] = v;
}

__global__ void signal(uint32_t* flag, uint32_t v) {
  __threadfence();
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

#define CK(x) do { hipError_t rc_ = (x); if (rc_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(rc_)); return 1; } } while (0)

int main() {
  float *a, *b;
  CK(hipMalloc(&a, 1 << 24));
  CK(hipMalloc(&b, 1 << 24));
  uint32_t* flag;
  CK(hipMalloc(&flag, 4096));
  CK(hipMemset(flag, 0, 4096));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  const int N = 400;
  std::vector<hipEvent_t> ev(N), evf(N), evd(N);
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : evf) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
  for (auto& e : evd) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventReleaseToDevice));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  for (int variant = 0; variant < 6; ++variant) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(t0, s0));
      for (int i = 0; i < N; ++i) {
        spin<<<1024, 256, 0, s0>>>(a, 200);
        if (variant == 1) {
          CK(hipEventRecord(ev[i], s0));
          CK(hipStreamWaitEvent(s1, ev[i], 0));
          spin<<<8, 64, 0, s1>>>(b, 10);
        } else if (variant == 3 || variant == 4) {
          hipEvent_t e = variant == 3 ? evf[i] : evd[i];
          CK(hipEventRecord(e, s0));
          CK(hipStreamWaitEvent(s1, e, 0));
          spin<<<8, 64, 0, s1>>>(b, 10);
        } else if (variant == 5) {
          const uint32_t v = (uint32_t)(rep * N + i + 1 + variant * 100000);
          signal<<<1, 64, 0, s0>>>(flag, v);
          CK(hipStreamWaitValue32(s1, flag, v, hipStreamWaitValueGte, 0xffffffffu));
          spin<<<8, 64, 0, s1>>>(b, 10);
        } else if (variant == 2) {
          CK(hipStreamWriteValue32(s0, flag, (uint32_t)(rep * N + i + 1 + variant * 100000), 0));
          CK(hipStreamWaitValue32(s1, flag, (uint32_t)(rep * N + i + 1 + variant * 100000), hipStreamWaitValueGte, 0xffffffffu));
          spin<<<8, 64, 0, s1>>>(b, 10);
        }
      }
      CK(hipEventRecord(t1, s0));
      CK(hipDeviceSynchronize());
      float ms = 0;
      CK(hipEventElapsedTime(&ms, t0, t1));
      std::printf("variant %d rep %d: %.2f us per kernel on the source stream\n", variant, rep, 1e3f * ms / N);
    }
  }
  return 0;
}
