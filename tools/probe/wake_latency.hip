// Cross-stream wake-up latency: stream B runs kernel A, records edge event E (no system fence) and
// a timing event TA, then (variant 1) a long kernel X; stream S waits on E, records timing event TW
// and runs a short kernel.  Prints TW - TA: how long after A's completion the waiting stream moves,
// with the source stream idle (variant 0) or busy with X (1), and with a third stream busy (2).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(float* x, int iters) {
  float v = x[threadIdx.x + blockIdx.x * blockDim.x];
  for (int i = 0; i < iters; ++i) v = v * 0.999f + 0.001f;
  x[threadIdx.x + blockIdx.x * blockDim.x] = v;
}
#define CK(x) do { hipError_t rc_ = (x); if (rc_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(rc_)); return 1; } } while (0)

int main() {
  float *a, *b, *c;
  CK(hipMalloc(&a, 1 << 24)); CK(hipMalloc(&b, 1 << 24)); CK(hipMalloc(&c, 1 << 24));
  hipStream_t sb, sw, so;
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sw, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&so, hipStreamNonBlocking));
  hipEvent_t E, TA, TW;
  CK(hipEventCreateWithFlags(&E, hipEventDisableTiming | hipEventDisableSystemFence));
  CK(hipEventCreate(&TA)); CK(hipEventCreate(&TW));
  for (int variant = 0; variant < 4; ++variant) {
    float tot = 0.f, mx = 0.f;
    const int R = 50;
    for (int r = 0; r < R; ++r) {
      CK(hipDeviceSynchronize());
      if (variant >= 2) spin<<<2048, 256, 0, so>>>(c, 20000);     // a third stream keeps the CUs busy
      spin<<<512, 256, 0, sb>>>(a, 2000);                          // A
      CK(hipEventRecord(E, sb));
      CK(hipEventRecord(TA, sb));
      if (variant == 1 || variant == 3) spin<<<4096, 256, 0, sb>>>(a, 20000);   // X after the marker
      CK(hipStreamWaitEvent(sw, E, 0));
      CK(hipEventRecord(TW, sw));
      spin<<<8, 64, 0, sw>>>(b, 10);
      CK(hipDeviceSynchronize());
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, TA, TW));
      tot += ms; mx = ms > mx ? ms : mx;
    }
    std::printf("variant %d: wake-up %.1f us mean, %.1f us max\n", variant, 1e3f * tot / R, 1e3f * mx);
  }
  return 0;
}
