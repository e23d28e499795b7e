// Micro-benchmark of the class-sum root reduction of the one-class-per-workgroup 4-state
// traversal (plk_kernels.hpp cls_blocks_kernel): C = 4 class terms per pattern -> log, site
// lnL, weighted sums, 4096-pattern block sums, at 1M patterns.  Variants:
//   0: cls_blocks_kernel's shape (1024 threads per block, 4 pattern-waves per wave)
//   1: 0 without the log (memory floor of the same access pattern)
//   2: 0 without the site lnL stores
//   3: 256-thread blocks, one pattern-wave per wave, wave sums to HBM (no block sums)
//   4: pure streaming read of the class terms (sum only)
//   5: 0 with the block chain read from LDS (broadcast reads, then the 64 adds)
//   6: 0 without the block chain (wave sums left in LDS)
//   7-10: red_pipe<waves per block, batch>: <8,4>, <4,4>, <4,2>, <16,2> (next batch's loads
//         issued before the current batch's log and reduction)
//   11, 12: 5 with the class terms interleaved per 64-pattern group ([group][C][64]); 12 with the
//         weights as a fifth row of each group
//   13: the product's loads alone (no log, no stores, no reduction)
// hipcc -O3 --offload-arch=gfx950 -o cls_reduce cls_reduce.hip; ./cls_reduce [patterns]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));               \
      return 1;                                                                \
    }                                                                          \
  } while (0)

constexpr int kBlock = 4096;

template <int V>
__global__ __launch_bounds__(1024) void red1024(const double* __restrict__ cls, int64_t n_pad, const double* __restrict__ w,
                                                double* __restrict__ site, double* __restrict__ blocks, int64_t n) {
  constexpr int kW = kBlock / 64, kPer = kW / 16, C = 4;
  __shared__ double ws[kW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, b = blockIdx.x;
  double t[kPer][C], wt[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t p = ((int64_t)b * kW + wv + 16 * j) * 64 + lane;
#pragma unroll
    for (int c = 0; c < C; ++c) t[j][c] = cls[(int64_t)c * n_pad + p];
    wt[j] = w[p];
  }
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int k = wv + 16 * j;
    const int64_t p = ((int64_t)b * kW + k) * 64 + lane;
    double l = 0.0;
#pragma unroll
    for (int c = 0; c < C; ++c)
      if (t[j][c] > 0.0) l += t[j][c];
    const double r = V == 1 ? l : log(l);
    if (V != 2 && p < n) site[p] = r;
    double wr = wt[j] * r;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) wr += __shfl_xor(wr, off, 64);
    if (lane == 0) ws[k] = wr;
  }
  __syncthreads();
  if (V == 6) return;
  if (V == 5) {  // the chain from LDS: broadcast reads, then the 64 dependent adds
    if (wv == 0) {
      double x[kW];
#pragma unroll
      for (int k = 0; k < kW; ++k) x[k] = ws[k];
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < kW; ++k) s += x[k];
      if (lane == 0) blocks[b] = s;
    }
    return;
  }
  if (wv == 0) {
    const double v = ws[lane];
    double s = 0.0;
    for (int k = 0; k < kW; ++k) s += __shfl(v, k, 64);
    if (lane == 0) blocks[b] = s;
  }
}


// Pipelined: NWV waves per 4096-pattern block, each wave 64 / NWV pattern-waves in batches of B,
// the next batch's loads issued before the current batch's log / reduction (double buffer);
// the block chain from LDS.
template <int NWV, int B>
__global__ __launch_bounds__(64 * NWV) void red_pipe(const double* __restrict__ cls, int64_t n_pad,
                                                     const double* __restrict__ w, double* __restrict__ site,
                                                     double* __restrict__ blocks, int64_t n) {
  constexpr int kW = kBlock / 64, KPW = kW / NWV, NB = KPW / B, C = 4;
  __shared__ double ws[kW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, b = blockIdx.x;
  double t[2][B][C + 1];
  auto load = [&](int buf, int bi) {
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const int k = wv + NWV * (bi * B + j);
      const int64_t p = ((int64_t)b * kW + k) * 64 + lane;
#pragma unroll
      for (int c = 0; c < C; ++c) t[buf][j][c] = cls[(int64_t)c * n_pad + p];
      t[buf][j][C] = w[p];
    }
  };
  load(0, 0);
#pragma unroll
  for (int bi = 0; bi < NB; ++bi) {
    if (bi + 1 < NB) load((bi + 1) & 1, bi + 1);
#pragma unroll
    for (int j = 0; j < B; ++j) {
      const int k = wv + NWV * (bi * B + j);
      const int64_t p = ((int64_t)b * kW + k) * 64 + lane;
      double l = 0.0;
#pragma unroll
      for (int c = 0; c < C; ++c)
        if (t[bi & 1][j][c] > 0.0) l += t[bi & 1][j][c];
      const double r = log(l);
      if (p < n) site[p] = r;
      double wr = t[bi & 1][j][C] * r;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) wr += __shfl_xor(wr, off, 64);
      if (lane == 0) ws[k] = wr;
    }
  }
  __syncthreads();
  if (wv == 0) {
    double x[kW];
#pragma unroll
    for (int k = 0; k < kW; ++k) x[k] = ws[k];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kW; ++k) s += x[k];
    if (lane == 0) blocks[b] = s;
  }
}


// Interleaved layout: per 64-pattern group the class terms (and with W the weights too) as
// consecutive 512-byte rows, [group][C (+1)][64] -- one contiguous chunk per pattern-wave
template <bool W>
__global__ __launch_bounds__(1024) void red_il(const double* __restrict__ cls, const double* __restrict__ w,
                                               double* __restrict__ site, double* __restrict__ blocks, int64_t n) {
  constexpr int kW = kBlock / 64, kPer = kW / 16, C = 4, R = W ? C + 1 : C;
  __shared__ double ws[kW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, b = blockIdx.x;
  double t[kPer][C], wt[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t g = (int64_t)b * kW + wv + 16 * j, p = g * 64 + lane;
#pragma unroll
    for (int c = 0; c < C; ++c) t[j][c] = cls[(g * R + c) * 64 + lane];
    wt[j] = W ? cls[(g * R + C) * 64 + lane] : w[p];
  }
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int k = wv + 16 * j;
    const int64_t p = ((int64_t)b * kW + k) * 64 + lane;
    double l = 0.0;
#pragma unroll
    for (int c = 0; c < C; ++c)
      if (t[j][c] > 0.0) l += t[j][c];
    const double r = log(l);
    if (p < n) site[p] = r;
    double wr = wt[j] * r;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) wr += __shfl_xor(wr, off, 64);
    if (lane == 0) ws[k] = wr;
  }
  __syncthreads();
  if (wv == 0) {
    double x[kW];
#pragma unroll
    for (int k = 0; k < kW; ++k) x[k] = ws[k];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kW; ++k) s += x[k];
    if (lane == 0) blocks[b] = s;
  }
}


// The product's access pattern with no arithmetic beyond one sum per lane (memory floor of
// the shape): every load issued first, then one store per block
__global__ __launch_bounds__(1024) void red_loads(const double* __restrict__ cls, int64_t n_pad,
                                                  const double* __restrict__ w, double* __restrict__ blocks) {
  constexpr int kW = kBlock / 64, kPer = kW / 16, C = 4;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, b = blockIdx.x;
  double t[kPer][C + 1];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t p = ((int64_t)b * kW + wv + 16 * j) * 64 + lane;
#pragma unroll
    for (int c = 0; c < C; ++c) t[j][c] = cls[(int64_t)c * n_pad + p];
    t[j][C] = w[p];
  }
  double s = 0.0;
#pragma unroll
  for (int j = 0; j < kPer; ++j)
#pragma unroll
    for (int c = 0; c <= C; ++c) s += t[j][c];
  if (s == 12345.0) blocks[b] = s;
}

__global__ __launch_bounds__(256) void red256(const double* __restrict__ cls, int64_t n_pad, const double* __restrict__ w,
                                              double* __restrict__ site, double* __restrict__ wsums, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t p0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64, p = p0 + lane;
  double l = 0.0;
  double t[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) t[c] = cls[(int64_t)c * n_pad + p];
  const double wt = w[p];
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (t[c] > 0.0) l += t[c];
  const double r = log(l);
  if (p < n) site[p] = r;
  double wr = wt * r;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) wr += __shfl_xor(wr, off, 64);
  if (lane == 0) wsums[p0 >> 6] = wr;
}

__global__ __launch_bounds__(256) void stream(const double* __restrict__ cls, int64_t total, double* __restrict__ out) {
  double s = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
    s += cls[i];
  if (s == 12345.0) out[0] = s;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 1000000, n_pad = (n + kBlock - 1) / kBlock * kBlock;
  const int nb = (int)(n_pad / kBlock);
  double *cls, *w, *site, *blocks, *wsums;
  CK(hipMalloc(&cls, 5 * n_pad * 8));  // (variant 12 reads a fifth row per group)
  CK(hipMalloc(&w, n_pad * 8));
  CK(hipMalloc(&site, n_pad * 8));
  CK(hipMalloc(&blocks, nb * 8));
  CK(hipMalloc(&wsums, n_pad / 64 * 8));
  std::vector<double> h(4 * n_pad, 0.1);
  CK(hipMemcpy(cls, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, h.data(), n_pad * 8, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int v = 0; v < 14; ++v) {
    auto run = [&]() {
      if (v == 0) red1024<0><<<nb, 1024>>>(cls, n_pad, w, site, blocks, n);
      if (v == 1) red1024<1><<<nb, 1024>>>(cls, n_pad, w, site, blocks, n);
      if (v == 2) red1024<2><<<nb, 1024>>>(cls, n_pad, w, site, blocks, n);
      if (v == 3) red256<<<(unsigned)(n_pad / 256), 256>>>(cls, n_pad, w, site, wsums, n);
      if (v == 5) red1024<5><<<nb, 1024>>>(cls, n_pad, w, site, blocks, n);
      if (v == 6) red1024<6><<<nb, 1024>>>(cls, n_pad, w, site, blocks, n);
      if (v == 7) red_pipe<8, 4><<<nb, 512>>>(cls, n_pad, w, site, blocks, n);
      if (v == 8) red_pipe<4, 4><<<nb, 256>>>(cls, n_pad, w, site, blocks, n);
      if (v == 9) red_pipe<4, 2><<<nb, 256>>>(cls, n_pad, w, site, blocks, n);
      if (v == 10) red_pipe<16, 2><<<nb, 1024>>>(cls, n_pad, w, site, blocks, n);
      if (v == 11) red_il<false><<<nb, 1024>>>(cls, w, site, blocks, n);
      if (v == 12) red_il<true><<<nb, 1024>>>(cls, w, site, blocks, n);
      if (v == 13) red_loads<<<nb, 1024>>>(cls, n_pad, w, blocks);
      if (v == 4) stream<<<1024, 256>>>(cls, 4 * n_pad, site);  // the class terms only (4 * n_pad doubles)
    };
    for (int i = 0; i < 20; ++i) run();
    CK(hipEventRecord(a));
    const int reps = 200;
    for (int i = 0; i < reps; ++i) run();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("n %lld variant %d: %.2f us per launch\n", (long long)n, v, ms * 1000.0 / reps);
  }
  return 0;
}
