// Micro-test: is fine-grained device memory host-writable here (large BAR), and how long do a
// host write of a P(t) request and a kernel read of it take, against pinned host memory?
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void touch(const double* src, double* dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i] * 2.0;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const int n = 1022 * 2;
  std::vector<double> h(n, 1.5);
  double *fg = nullptr, *pin = nullptr, *pin_dev = nullptr, *out = nullptr;
  hipError_t e = hipExtMallocWithFlags((void**)&fg, n * sizeof(double), hipDeviceMallocFinegrained);
  printf("fine-grained alloc: %s\n", hipGetErrorString(e));
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, fg) == hipSuccess)
    printf("attr: type %d hostPointer %p devicePointer %p\n", (int)attr.type, attr.hostPointer, attr.devicePointer);
  hipHostMalloc((void**)&pin, n * sizeof(double), hipHostMallocMapped);
  hipHostGetDevicePointer((void**)&pin_dev, pin, 0);
  hipMalloc((void**)&out, n * sizeof(double));
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int mode = 0; mode < 2; ++mode) {
    double* src = mode == 0 ? pin_dev : fg;
    double* hw = mode == 0 ? pin : fg;  // host writes through this pointer
    double tw = 0, tk = 0;
    for (int it = 0; it < 60; ++it) {
      const double t0 = now_us();
      std::memcpy(hw, h.data(), n * sizeof(double));
      const double t1 = now_us();
      hipEventRecord(a, s);
      touch<<<(n + 255) / 256, 256, 0, s>>>(src, out, n);
      hipEventRecord(b, s);
      hipStreamSynchronize(s);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (it >= 10) {
        tw += t1 - t0;
        tk += ms * 1000.0;
      }
    }
    printf("%s: host write %.2f us, kernel read+write %.2f us\n", mode == 0 ? "pinned host" : "fine-grained VRAM",
           tw / 50, tk / 50);
  }
  return 0;
}
