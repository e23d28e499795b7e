// plk_mfma64.hpp -- K3: 64-state (codon) partials on fp64 matrix cores (gfx950).
//
// For a child with transition matrix P (64 x 64, stop codons are null states) the
// contribution to a tile of patterns is the dense product
//     D[x][p] = sum_y P[x][y] * L[y][p]
// (RHomogeneousTreeLikelihood.cpp:839-861 with the site loop as the N dimension).
// The partial layout [c*S + s][128 patterns] is exactly L^T row-major, so D = P . L^T
// runs on v_mfma_f64_16x16x4f64 with
//   A = P       (16 x 4 fragments from LDS, P^T staged with a 80-double row stride:
//                conflict-free ds_read_b64 for the 16x4 lane map),
//   B = L^T     (4 x 16 fragments straight from HBM: 4 rows x 128 contiguous bytes),
//   C/D         (lane l holds D[x0 + (l>>4) + 4r][p0 + (l&15)], r = 0..3),
// so both the loads and the stores are 128-byte row segments.  The product over
// children happens in registers.  A workgroup = 4 waves = one 128-pattern tile;
// wave w owns patterns [32w, 32w + 32) (two 16-pattern column tiles).
//
// fp64 MFMA and fp64 FMA have the same peak on MI355X; the matrix core buys operand
// reuse (one LDS read of P feeds 2 MFMAs = 4096 flops) and leaves the VALU free.
#pragma once

#include "plk_kernels.hpp"

namespace plk {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kM64Ld = 80;  // LDS row stride (doubles) of P^T: 2*80 = 32 mod 64 banks

template <bool SCALE>
__global__ __launch_bounds__(256) void partials_mfma64_kernel(const KOp* __restrict__ ops, PartialsArgs a,
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
  const int pw = w * 32;      // first pattern of this wave inside the tile
  const size_t tbase = (size_t)tile * ((size_t)C * S * kTile);
  double* outp = a.partials + (size_t)op.parent * a.slot_stride + tbase;
  const size_t pidx0 = (size_t)tile * kTile + pw;

  int cnt[2] = {0, 0};
  if (SCALE) {
    for (int pt = 0; pt < 2; ++pt) {
      const size_t pi = pidx0 + 16 * pt + lc;
      int s = (op.flags & 1) ? a.scale[(size_t)op.parent * a.n_pad + pi] : 0;
      for (int k = 0; k < n; ++k)
        if (!op.is_tip[k]) s += a.scale[(size_t)op.child[k] * a.n_pad + pi];
      cnt[pt] = s;
    }
  }
  double m[2] = {0.0, 0.0};

  for (int c = 0; c < C; ++c) {
    f64x4 acc[4][2];
    if (op.flags & 1) {
#pragma unroll
      for (int xt = 0; xt < 4; ++xt)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc[xt][pt][r] = outp[(size_t)(c * S + 16 * xt + lr + 4 * r) * kTile + pw + 16 * pt + lc];
    } else {
#pragma unroll
      for (int xt = 0; xt < 4; ++xt)
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) acc[xt][pt] = (f64x4){1.0, 1.0, 1.0, 1.0};
    }
    for (int k = 0; k < n; ++k) {
      __syncthreads();  // previous users of the LDS image are done
      if (op.is_tip[k]) {
        const double* src = a.tipP + ((size_t)op.child[k] * C + c) * nc * S;
        for (int i = threadIdx.x; i < nc * S; i += blockDim.x) lds[i] = src[i];
        __syncthreads();
        // D[x][p] = tipP[code(p)][x]
#pragma unroll
        for (int pt = 0; pt < 2; ++pt) {
          const int code = a.codes[(size_t)op.child[k] * a.n_pad + pidx0 + 16 * pt + lc];
          const double* t = lds + code * S;
#pragma unroll
          for (int xt = 0; xt < 4; ++xt)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[xt][pt][r] *= t[16 * xt + lr + 4 * r];
        }
      } else {
        const double* src = pmatsT + ((size_t)op.branch[k] * C + c) * S * S;  // P^T[y][x]
        for (int i = threadIdx.x; i < S * S; i += blockDim.x) lds[(i >> 6) * kM64Ld + (i & 63)] = src[i];
        __syncthreads();
        const double* L = a.partials + (size_t)op.child[k] * a.slot_stride + tbase + (size_t)c * S * kTile + pw + lc;
        f64x4 d[4][2];
#pragma unroll
        for (int xt = 0; xt < 4; ++xt)
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) d[xt][pt] = (f64x4){0.0, 0.0, 0.0, 0.0};
#pragma unroll 2
        for (int ks = 0; ks < 16; ++ks) {
          const int y = 4 * ks + lr;
          double bf[2];
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) bf[pt] = L[(size_t)y * kTile + 16 * pt];
          double af[4];
#pragma unroll
          for (int xt = 0; xt < 4; ++xt) af[xt] = lds[y * kM64Ld + 16 * xt + lc];
#pragma unroll
          for (int xt = 0; xt < 4; ++xt)
#pragma unroll
            for (int pt = 0; pt < 2; ++pt)
              d[xt][pt] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[xt], bf[pt], d[xt][pt], 0, 0, 0);
        }
#pragma unroll
        for (int xt = 0; xt < 4; ++xt)
#pragma unroll
          for (int pt = 0; pt < 2; ++pt) acc[xt][pt] *= d[xt][pt];
      }
    }
#pragma unroll
    for (int xt = 0; xt < 4; ++xt)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (SCALE) m[pt] = fmax(m[pt], acc[xt][pt][r]);
          outp[(size_t)(c * S + 16 * xt + lr + 4 * r) * kTile + pw + 16 * pt + lc] = acc[xt][pt][r];
        }
  }
  if (SCALE) {
    // a pattern's values are spread over the 4 lane rows (lr): combine the maxima
#pragma unroll
    for (int pt = 0; pt < 2; ++pt) {
      double v = m[pt];
      v = fmax(v, __shfl_xor(v, 16, 64));
      v = fmax(v, __shfl_xor(v, 32, 64));
      const bool rs = v > 0.0 && v < kScaleThr;
      if (rs) {
        for (int c = 0; c < C; ++c)
          for (int xt = 0; xt < 4; ++xt)
            for (int r = 0; r < 4; ++r)
              outp[(size_t)(c * S + 16 * xt + lr + 4 * r) * kTile + pw + 16 * pt + lc] *= kScaleUp;
      }
      if (lr == 0) a.scale[(size_t)op.parent * a.n_pad + pidx0 + 16 * pt + lc] = cnt[pt] + (rs ? 1 : 0);
    }
  }
}

// P^T copy for the MFMA path: PT[b][c][y][x] = P[b][c][x][y]  (grid: nodes x classes)
__global__ void transpose_pmats64(const double* __restrict__ P, double* __restrict__ PT, int C) {
  const int b = blockIdx.x;
  const int c = blockIdx.y;
  const size_t off = ((size_t)b * C + c) * 64 * 64;
  for (int e = threadIdx.x; e < 64 * 64; e += blockDim.x) {
    const int y = e >> 6, x = e & 63;
    PT[off + e] = P[off + (size_t)x * 64 + y];
  }
}

}  // namespace plk
