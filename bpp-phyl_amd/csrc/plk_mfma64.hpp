// plk_mfma64.hpp -- K3: 64-state (codon) partials on fp64 matrix cores (gfx950).
//
// For a child with transition matrix P (64 x 64, stop codons are null states) the
// contribution to a tile of patterns is the dense product
//     D[x][p] = sum_y P[x][y] * L[y][p]
// (RHomogeneousTreeLikelihood.cpp:839-861 with the site loop as the N dimension).
// The partial layout [c*S + s][128 patterns] is exactly L^T row-major, so D = P . L^T
// runs on v_mfma_f64_16x16x4f64 with
//   A = P       (16 x 4 fragments from LDS: P^T staged with an 80-double row stride),
//   B = L^T     (4 x 16 fragments straight from HBM: 4 rows x 128 contiguous bytes),
//   C/D         (lane l holds D[x0 + (l>>4) + 4r][p0 + (l&15)], r = 0..3),
// so both the loads and the stores are 128-byte row segments.  The product over
// children happens in registers.  A workgroup = 8 waves = one 128-pattern tile; wave
// w owns patterns [16w, 16w + 16): 16 accumulators + 16 result registers per lane, and
// the 16 B fragments of a child are all issued before the P^T staging barrier, so the
// HBM latency of the child tile overlaps the staging and the MFMA chain (~64 cycles
// per fp64 16x16x4) drains them in order.  Low register use keeps 4 waves per SIMD.
//
// fp64 MFMA and fp64 FMA have the same peak on MI355X (78.6 TF); the matrix core buys
// operand reuse and leaves the VALU free for the tip lookups and the product.
#pragma once

#include "plk_treeM.hpp"  // f64x4 helpers, transpose_pmats

namespace plk {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kM64Ld = 80;      // LDS row stride (doubles) of P^T
constexpr int kM64Threads = 512;

template <bool SCALE>
__global__ __launch_bounds__(kM64Threads) void partials_mfma64_kernel(const KOp* __restrict__ ops, PartialsArgs a,
                                                                      const double* __restrict__ pmatsT, int C) {
  constexpr int S = 64;
  extern __shared__ __attribute__((aligned(16))) double lds[];  // P^T [64][80] or tip table [n_codes][64]
  const KOp& op = ops[blockIdx.y];
  const int n = op.n;
  const int nc = a.n_codes;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = blockIdx.x;
  const int lr = lane >> 4;   // 0..3
  const int lc = lane & 15;   // 0..15
  const int pw = w * 16;      // first pattern of this wave inside the tile
  const size_t tbase = (size_t)tile * ((size_t)C * S * kTile);
  double* outp = a.partials + (size_t)op.parent * a.slot_stride + tbase + pw + lc;
  const size_t pidx = (size_t)tile * kTile + pw + lc;

  int cnt = 0;
  if (SCALE) {
    cnt = (op.flags & 1) ? a.scale[(size_t)op.parent * a.n_pad + pidx] : 0;
    for (int k = 0; k < n; ++k)
      if (!op.is_tip[k]) cnt += a.scale[(size_t)op.child[k] * a.n_pad + pidx];
  }
  double m = 0.0;

  for (int c = 0; c < C; ++c) {
    f64x4 acc[4];
    if (op.flags & 1) {
#pragma unroll
      for (int xt = 0; xt < 4; ++xt)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[xt][r] = outp[(size_t)(c * S + 16 * xt + lr + 4 * r) * kTile];
    } else {
#pragma unroll
      for (int xt = 0; xt < 4; ++xt) acc[xt] = (f64x4){1.0, 1.0, 1.0, 1.0};
    }
    for (int k = 0; k < n; ++k) {
      if (op.is_tip[k]) {
        const int code = a.codes[(size_t)op.child[k] * a.n_pad + pidx];
        __syncthreads();  // previous users of the LDS image are done
        const double* src = a.tipP + ((size_t)op.child[k] * C + c) * nc * S;
        for (int i = threadIdx.x; i < nc * S; i += kM64Threads) lds[i] = src[i];
        __syncthreads();
        // D[x][p] = tipP[code(p)][x]
        const double* t = lds + code * S;
#pragma unroll
        for (int xt = 0; xt < 4; ++xt)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[xt][r] *= t[16 * xt + lr + 4 * r];
      } else {
        // the child's 64 x 16 slab of this wave: all 16 B fragments in flight first
        const double* L = a.partials + (size_t)op.child[k] * a.slot_stride + tbase + (size_t)c * S * kTile + pw + lc;
        double bf[16];
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) bf[ks] = L[(size_t)(4 * ks + lr) * kTile];
        __syncthreads();
        const double* src = pmatsT + ((size_t)op.branch[k] * C + c) * S * S;  // P^T[y][x]
        for (int i = threadIdx.x; i < S * S; i += kM64Threads) lds[(i >> 6) * kM64Ld + (i & 63)] = src[i];
        __syncthreads();
        f64x4 d[4];
#pragma unroll
        for (int xt = 0; xt < 4; ++xt) d[xt] = (f64x4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) {
          const int y = 4 * ks + lr;
          double af[4];
#pragma unroll
          for (int xt = 0; xt < 4; ++xt) af[xt] = lds[y * kM64Ld + 16 * xt + lc];
#pragma unroll
          for (int xt = 0; xt < 4; ++xt) d[xt] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[xt], bf[ks], d[xt], 0, 0, 0);
        }
#pragma unroll
        for (int xt = 0; xt < 4; ++xt) acc[xt] *= d[xt];
      }
    }
#pragma unroll
    for (int xt = 0; xt < 4; ++xt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (SCALE) m = fmax(m, acc[xt][r]);
        outp[(size_t)(c * S + 16 * xt + lr + 4 * r) * kTile] = acc[xt][r];
      }
  }
  if (SCALE) {
    // a pattern's 64 states are spread over the 4 lane rows (lr): combine the maxima
    double v = m;
    v = fmax(v, __shfl_xor(v, 16, 64));
    v = fmax(v, __shfl_xor(v, 32, 64));
    const bool rs = v > 0.0 && v < kScaleThr;
    if (rs) {
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int xt = 0; xt < 4; ++xt)
#pragma unroll
          for (int r = 0; r < 4; ++r) outp[(size_t)(c * S + 16 * xt + lr + 4 * r) * kTile] *= kScaleUp;
    }
    if (lr == 0) a.scale[(size_t)op.parent * a.n_pad + pidx] = cnt + (rs ? 1 : 0);
  }
}

}  // namespace plk
