// fp64 VALU / MFMA peak microbenchmark (gfx950): achievable fp64 FMA rate, to put the
// fused kernels' fraction of the 78.6 TF/s spec into context.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(256) void fma_kernel(double* out, int iters, double a, double b) {
  double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      x0 = __builtin_fma(x0, a, b); x1 = __builtin_fma(x1, a, b); x2 = __builtin_fma(x2, a, b);
      x3 = __builtin_fma(x3, a, b); x4 = __builtin_fma(x4, a, b); x5 = __builtin_fma(x5, a, b);
      x6 = __builtin_fma(x6, a, b); x7 = __builtin_fma(x7, a, b);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

typedef double f64x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void mfma_kernel(double* out, int iters, double a, double b) {
  f64x4 d0 = {0, 0, 0, 0}, d1 = d0, d2 = d0, d3 = d0;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      d0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d3, 0, 0, 0);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = d0[0] + d1[1] + d2[2] + d3[3];
}

// v_mfma_f64_4x4x4_4b_f64: 4 blocks of 4x4x4 per wave (512 flops per instruction, one
// f64 result per lane).  20 states tile as 5 x 4 rows with no padding, where the 16x16x4
// form runs 32-row tiles (37.5 % padding): worth it only if its flop rate is close.
__global__ __launch_bounds__(256) void mfma4_kernel(double* out, int iters, double a, double b) {
  double d0 = 0, d1 = 0, d2 = 0, d3 = 0, d4 = 0, d5 = 0, d6 = 0, d7 = 0;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      d0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d3, 0, 0, 0);
      d4 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d4, 0, 0, 0);
      d5 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d5, 0, 0, 0);
      d6 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d6, 0, 0, 0);
      d7 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d7, 0, 0, 0);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7;
}

// Do the fp64 VALU and the fp64 matrix pipe overlap?  Per iteration a wave issues 64
// v_fma_f64 (V) and/or 16 v_mfma_f64_4x4x4_4b (M) -- about equal times alone.  If the two
// pipes run side by side, V+M in one wave (or in alternate waves) takes ~max(V, M), else ~V + M.
// mode 0: V, 1: M, 2: V and M interleaved in every wave, 3: even waves V, odd waves M (2x iters).
template <int MODE>
__global__ __launch_bounds__(256) void mix_kernel(double* out, int iters, double a, double b) {
  double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  double d0 = 0, d1 = 0, d2 = 0, d3 = 0, d4 = 0, d5 = 0, d6 = 0, d7 = 0;
  const int wave = threadIdx.x >> 6;
  const bool do_v = MODE == 0 || MODE == 2 || (MODE == 3 && (wave & 1) == 0);
  const bool do_m = MODE == 1 || MODE == 2 || (MODE == 3 && (wave & 1) == 1);
  const int n = MODE == 3 ? 2 * iters : iters;
  if (do_v && do_m) {
    for (int i = 0; i < n; ++i) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        d0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d0, 0, 0, 0);
        x0 = __builtin_fma(x0, a, b); x1 = __builtin_fma(x1, a, b); x2 = __builtin_fma(x2, a, b); x3 = __builtin_fma(x3, a, b);
        d1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d1, 0, 0, 0);
        x4 = __builtin_fma(x4, a, b); x5 = __builtin_fma(x5, a, b); x6 = __builtin_fma(x6, a, b); x7 = __builtin_fma(x7, a, b);
        d2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d2, 0, 0, 0);
        x0 = __builtin_fma(x0, a, b); x1 = __builtin_fma(x1, a, b); x2 = __builtin_fma(x2, a, b); x3 = __builtin_fma(x3, a, b);
        d3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d3, 0, 0, 0);
        x4 = __builtin_fma(x4, a, b); x5 = __builtin_fma(x5, a, b); x6 = __builtin_fma(x6, a, b); x7 = __builtin_fma(x7, a, b);
        d4 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d4, 0, 0, 0);
        x0 = __builtin_fma(x0, a, b); x1 = __builtin_fma(x1, a, b); x2 = __builtin_fma(x2, a, b); x3 = __builtin_fma(x3, a, b);
        d5 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d5, 0, 0, 0);
        x4 = __builtin_fma(x4, a, b); x5 = __builtin_fma(x5, a, b); x6 = __builtin_fma(x6, a, b); x7 = __builtin_fma(x7, a, b);
        d6 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d6, 0, 0, 0);
        x0 = __builtin_fma(x0, a, b); x1 = __builtin_fma(x1, a, b); x2 = __builtin_fma(x2, a, b); x3 = __builtin_fma(x3, a, b);
        d7 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d7, 0, 0, 0);
        x4 = __builtin_fma(x4, a, b); x5 = __builtin_fma(x5, a, b); x6 = __builtin_fma(x6, a, b); x7 = __builtin_fma(x7, a, b);
      }
    }
  } else if (do_v) {
    for (int i = 0; i < n; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        x0 = __builtin_fma(x0, a, b); x1 = __builtin_fma(x1, a, b); x2 = __builtin_fma(x2, a, b); x3 = __builtin_fma(x3, a, b);
        x4 = __builtin_fma(x4, a, b); x5 = __builtin_fma(x5, a, b); x6 = __builtin_fma(x6, a, b); x7 = __builtin_fma(x7, a, b);
      }
    }
  } else {
    for (int i = 0; i < n; ++i) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        d0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d0, 0, 0, 0);
        d1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d1, 0, 0, 0);
        d2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d2, 0, 0, 0);
        d3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d3, 0, 0, 0);
        d4 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d4, 0, 0, 0);
        d5 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d5, 0, 0, 0);
        d6 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d6, 0, 0, 0);
        d7 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d7, 0, 0, 0);
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7 + d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7;
}

template <int MODE>
static void run_mix(double* out, int blocks, int threads, int iters, hipEvent_t e0, hipEvent_t e1) {
  static const char* names[] = {"64 v_fma_f64 / iter", "16 v_mfma_f64_4x4x4_4b / iter", "both in every wave",
                                "alternate waves (2x iters each)"};
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    mix_kernel<MODE><<<blocks, threads>>>(out, iters, 0.999999, 1e-7);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("mix mode %d (%s): %.3f ms\n", MODE, names[MODE], ms);
  }
}

int main() {
  const int blocks = 256 * 8, threads = 256, iters = 4096;
  double* out;
  hipMalloc(&out, (size_t)blocks * threads * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    fma_kernel<<<blocks, threads>>>(out, iters, 0.999999, 1e-7);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 8 * 8 * (double)iters * blocks * threads;
    printf("VALU v_fma_f64: %.1f TF/s (%.3f ms)\n", flops / ms / 1e9, ms);
  }
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    mfma_kernel<<<blocks, threads>>>(out, iters / 4, 0.999999, 1e-7);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 16 * 16 * 4 * 8 * 4 * (double)(iters / 4) * blocks * (threads / 64);
    printf("MFMA v_mfma_f64_16x16x4: %.1f TF/s (%.3f ms)\n", flops / ms / 1e9, ms);
  }
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    mfma4_kernel<<<blocks, threads>>>(out, iters / 4, 0.999999, 1e-7);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double flops = 2.0 * 4 * 4 * 4 * 4 * 8 * 8 * (double)(iters / 4) * blocks * (threads / 64);
    printf("MFMA v_mfma_f64_4x4x4_4b: %.1f TF/s (%.3f ms)\n", flops / ms / 1e9, ms);
  }
  run_mix<0>(out, blocks, threads, iters / 4, e0, e1);
  run_mix<1>(out, blocks, threads, iters / 4, e0, e1);
  run_mix<2>(out, blocks, threads, iters / 4, e0, e1);
  run_mix<3>(out, blocks, threads, iters / 4, e0, e1);
  return 0;
}
