// plk_tree4.hpp -- fused postorder traversal for 4-state models (gfx950).
//
// One lane = one site pattern, one wave = 64 consecutive patterns.  A wave walks a
// small "tree program" (postorder events, wave-uniform, read with scalar loads) and
// keeps the pending product of every open ancestor in registers: level d of the
// current root-to-node path owns acc[d][C*4].  All register indices are compile
// time constants (the runtime level selects a template instance through a switch),
// so nothing spills.  A child's contribution is multiplied into its parent's level
// as soon as the child completes, in the reference's son order:
//     L_node[c][x] = prod_son sum_y P_son[c][x][y] L_son[c][y]
// (Likelihood/RHomogeneousTreeLikelihood.cpp:839-861).
//
// Compared with one launch per tree level (partials_s4_kernel), child partials are
// never re-read from HBM: a materialising traversal only WRITES each internal
// partial once (half the HBM traffic), and an lnL-only traversal writes nothing but
// the fragment roots.  Tips enter as uint8 codes through the getInitValue table
// (n_codes x 4 in LDS), which covers ambiguity codes exactly like the reference's
// dense leaf vectors.  The root reduction (RHomogeneousTreeLikelihood.cpp:162-216)
// is fused into the program's ROOT event.
#pragma once

#include "plk_kernels.hpp"

namespace plk {

enum TreeOp : int32_t { T_ENTER = 0, T_TIP = 1, T_LOAD = 2, T_EXIT = 3, T_ROOT = 4, T_END = 5 };

// 16-byte program word: wave-uniform, fetched with s_load_dwordx4.
struct TInstr {
  int32_t op;
  int32_t d;  // level of the accumulator the event writes
  int32_t a;  // TIP: tip index; LOAD: internal slot; EXIT/ROOT: store slot or -1
  int32_t b;  // TIP/LOAD/EXIT: branch (child node index); ROOT: 1 = reduce lnL
};

struct TreeArgs {
  const TInstr* prog;
  const int32_t* frag_start;  // program offset of each fragment (blockIdx.y)
  double* partials;           // [n_internal][slot_stride]
  int32_t* scale;             // [n_internal][n_pad] (SCALE only)
  const uint8_t* codes;       // [n_tips][n_pad]
  const double* pmats;        // [n_nodes][C][4][4]
  const double* init;         // [n_codes][4]
  const double* weights;      // [n_pad]
  const double* pi;           // [4]
  const double* probs;        // [C]
  double* site_lnl;           // [n_pad]
  double* wave_sums;          // [n_pad / 64]
  int64_t slot_stride;
  int64_t n_pad;
  int64_t n_patterns;
  int32_t n_codes;
  int32_t guard;
};

template <int C>
struct Acc {
  double v[C * 4];
};

// acc[D][c][x] *= sum_y P[c][x][y] * src[c][y]
template <int C>
__device__ __forceinline__ void contribute(double (&dst)[C * 4], const double (&src)[C * 4],
                                           const double* __restrict__ P) {
#pragma unroll
  for (int c = 0; c < C; ++c) {
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const double* Px = P + (c * 4 + x) * 4;
      double s = Px[0] * src[c * 4 + 0];
      s = __builtin_fma(Px[1], src[c * 4 + 1], s);
      s = __builtin_fma(Px[2], src[c * 4 + 2], s);
      s = __builtin_fma(Px[3], src[c * 4 + 3], s);
      dst[c * 4 + x] *= s;
    }
  }
}

// Exact power-of-two rescaling of one pattern's partial (max < 2^-256 -> x 2^256).
template <int C>
__device__ __forceinline__ void rescale(double (&v)[C * 4], int& cnt) {
  double m = 0.0;
#pragma unroll
  for (int i = 0; i < C * 4; ++i) m = fmax(m, v[i]);
  if (m > 0.0 && m < kScaleThr) {
#pragma unroll
    for (int i = 0; i < C * 4; ++i) v[i] *= kScaleUp;
    cnt += 1;
  }
}

template <int C, bool SCALE>
__device__ __forceinline__ void store_partial(const TreeArgs& a, int slot, int64_t p, const double (&v)[C * 4],
                                              int cnt) {
  const int64_t tile = p >> 7, q = p & (kTile - 1);
  double* dst = a.partials + (size_t)slot * a.slot_stride + tile * (C * 4 * kTile) + q;
#pragma unroll
  for (int i = 0; i < C * 4; ++i) __builtin_nontemporal_store(v[i], dst + (size_t)i * kTile);
  if (SCALE) a.scale[(size_t)slot * a.n_pad + p] = cnt;
}

template <int C, int DM, bool SCALE>
__global__ __launch_bounds__(256) void tree4_kernel(TreeArgs a) {
  extern __shared__ __attribute__((aligned(16))) double init_lds[];  // [n_codes][4]
  for (int i = threadIdx.x; i < a.n_codes * 4; i += blockDim.x) init_lds[i] = a.init[i];
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // pattern (< n_pad always)
  double acc[DM][C * 4];
  int cnt[DM];
#pragma unroll
  for (int d = 0; d < DM; ++d) cnt[d] = 0;
  const TInstr* pc = a.prog + a.frag_start[blockIdx.y];

  for (;;) {
    const TInstr in = *pc++;
    if (in.op == T_END) break;
    switch (in.op) {
      case T_ENTER:
        switch (in.d) {
#define PLK_ENTER(D)                                          \
  case D:                                                     \
    _Pragma("unroll") for (int i = 0; i < C * 4; ++i) acc[D][i] = 1.0; \
    cnt[D] = 0;                                               \
    break;
          PLK_ENTER(0) PLK_ENTER(1) PLK_ENTER(2) PLK_ENTER(3) PLK_ENTER(4) PLK_ENTER(5) PLK_ENTER(6) PLK_ENTER(7)
#undef PLK_ENTER
        }
        break;
      case T_TIP: {
        const int code = a.codes[(size_t)in.a * a.n_pad + p];
        double src[C * 4];
        const double* iv = init_lds + code * 4;
        const double i0 = iv[0], i1 = iv[1], i2 = iv[2], i3 = iv[3];
#pragma unroll
        for (int c = 0; c < C; ++c) {
          src[c * 4 + 0] = i0;
          src[c * 4 + 1] = i1;
          src[c * 4 + 2] = i2;
          src[c * 4 + 3] = i3;
        }
        const double* __restrict__ P = a.pmats + (size_t)in.b * (C * 16);
        switch (in.d) {
#define PLK_TIP(D) \
  case D:          \
    if (D < DM) contribute<C>(acc[D < DM ? D : 0], src, P); \
    break;
          PLK_TIP(0) PLK_TIP(1) PLK_TIP(2) PLK_TIP(3) PLK_TIP(4) PLK_TIP(5) PLK_TIP(6) PLK_TIP(7)
#undef PLK_TIP
        }
        break;
      }
      case T_LOAD: {
        const int64_t tile = p >> 7, q = p & (kTile - 1);
        const double* L = a.partials + (size_t)in.a * a.slot_stride + tile * (C * 4 * kTile) + q;
        double src[C * 4];
#pragma unroll
        for (int i = 0; i < C * 4; ++i) src[i] = L[(size_t)i * kTile];
        int sc = SCALE ? a.scale[(size_t)in.a * a.n_pad + p] : 0;
        const double* __restrict__ P = a.pmats + (size_t)in.b * (C * 16);
        switch (in.d) {
#define PLK_LOAD(D)                                            \
  case D:                                                      \
    if (D < DM) {                                              \
      contribute<C>(acc[D < DM ? D : 0], src, P);              \
      if (SCALE) cnt[D < DM ? D : 0] += sc;                    \
    }                                                          \
    break;
          PLK_LOAD(0) PLK_LOAD(1) PLK_LOAD(2) PLK_LOAD(3) PLK_LOAD(4) PLK_LOAD(5) PLK_LOAD(6) PLK_LOAD(7)
#undef PLK_LOAD
        }
        break;
      }
      case T_EXIT: {
        // child complete at level d+1: rescale, optionally store, multiply into level d
        const double* __restrict__ P = a.pmats + (size_t)in.b * (C * 16);
        switch (in.d) {
#define PLK_EXIT(D)                                                                  \
  case D:                                                                            \
    if (D + 1 < DM) {                                                                \
      constexpr int K = (D + 1 < DM) ? D + 1 : 0;                                    \
      constexpr int J = (D + 1 < DM) ? D : 0;                                        \
      if (SCALE) rescale<C>(acc[K], cnt[K]);                                         \
      if (in.a >= 0) store_partial<C, SCALE>(a, in.a, p, acc[K], cnt[K]);            \
      contribute<C>(acc[J], acc[K], P);                                              \
      if (SCALE) cnt[J] += cnt[K];                                                   \
    }                                                                                \
    break;
          PLK_EXIT(0) PLK_EXIT(1) PLK_EXIT(2) PLK_EXIT(3) PLK_EXIT(4) PLK_EXIT(5) PLK_EXIT(6)
#undef PLK_EXIT
        }
        break;
      }
      case T_ROOT: {
        // fragment root at level 0: rescale, optionally store, optionally reduce lnL
        if (SCALE) rescale<C>(acc[0], cnt[0]);
        if (in.a >= 0) store_partial<C, SCALE>(a, in.a, p, acc[0], cnt[0]);
        if (in.b) {
          double l = 0.0;
#pragma unroll
          for (int c = 0; c < C; ++c) {
            double lc = 0.0;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              const double li = acc[0][c * 4 + s] * a.pi[s];
              if (a.guard) {
                if (li > 0.0) lc += li;
              } else {
                lc += li;
              }
            }
            const double li = lc * a.probs[c];
            if (a.guard) {
              if (li > 0.0) l += li;
            } else {
              l += li;
            }
          }
          if (!a.guard && l < 0.0) l = 0.0;
          double r = log(l);
          if (SCALE) r -= (double)cnt[0] * kLn2x256;
          const bool valid = p < a.n_patterns;
          double wr = 0.0;
          if (valid) {
            a.site_lnl[p] = r;
            wr = a.weights[p] * r;
          }
          // fixed-order wave reduction (xor butterfly, same order for every wave)
#pragma unroll
          for (int off = 32; off > 0; off >>= 1) wr += __shfl_xor(wr, off, 64);
          if ((threadIdx.x & 63) == 0) a.wave_sums[p >> 6] = wr;
        }
        break;
      }
    }
  }
}

// block_sums[b] = sum of the 64 wave sums of patterns [b*4096, (b+1)*4096), in order.
__global__ void wave_sums_to_blocks(const double* __restrict__ wave_sums, double* __restrict__ block_sums,
                                    int n_waves, int n_blocks) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= n_blocks) return;
  double s = 0.0;
  const int w0 = b * (kRootBlock / 64);
  for (int w = w0; w < w0 + kRootBlock / 64 && w < n_waves; ++w) s += wave_sums[w];
  block_sums[b] = s;
}

}  // namespace plk
