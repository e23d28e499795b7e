// plk_deriv.hpp -- analytic branch-length derivatives of lnL (gfx950).
//
// Reference: RHomogeneousTreeLikelihood::computeTreeDLikelihood / computeDownSubtreeDLikelihood
// and the D2 twins (Likelihood/RHomogeneousTreeLikelihood.cpp:365-541, 615-791):
//   at the father of the branch   dL = prod_{other sons} (P L_son) * (dP L_branch)
//   on every ancestor up the path dL = prod_{other sons} (P L_son) * (P dL_child)
//   at the root                   dl = sum_c p_c sum_x pi_x dL[c][x],
//   d lnL / dt = sum_sites dl / l,  d2 lnL / dt2 = sum_sites (d2l / l - (dl / l)^2)
// with dP = r_c dP/dt and d2P = r_c^2 d2P/dt2 from K4 (AbstractHomogeneousTreeLikelihood.cpp:375-413).
//
// One lane = one pattern, all classes in registers.  L, dL and d2L travel up the
// path together in registers (nothing is written to HBM); siblings are read from the
// materialised partials (or tip codes).  L is recomputed along the path from the same
// inputs as dL, so dl / l is exact even with power-of-two rescaling (L, dL, d2L are
// rescaled jointly by L's maximum).
#pragma once

#include "plk_kernels.hpp"

namespace plk {

enum DerivOp : int32_t { D_TIP = 1, D_LOAD = 2, D_PATH = 3, D_STEP = 4, D_END = 5 };

// Per path step: one word per son of the node (TIP / LOAD / PATH), then STEP.
// The first step's PATH son is the branch itself (a = tip index or slot, d = 1 if tip).
struct DInstr {
  int32_t op;
  int32_t d;  // PATH of the first step: 1 = branch is a tip, 0 = internal
  int32_t a;  // TIP: tip index; LOAD: slot; PATH (first step): tip index or slot
  int32_t b;  // branch (son node index)
};

struct DerivArgs {
  const double* partials;
  const uint8_t* codes;
  const double* init;   // [n_codes][S]
  const double* pi;
  const double* probs;
  const double* weights;
  double* d1_sums;      // [n_pad / 64] wave sums of w * dl / l
  double* d2_sums;      // [n_pad / 64] wave sums of w * (d2l / l - (dl / l)^2)
  int64_t slot_stride;
  int64_t n_pad;
  int64_t n_patterns;
  int32_t n_codes;
};

template <int S, int C>
__device__ __forceinline__ void load_son(const DerivArgs& a, int is_tip, int idx, int64_t p, double (&v)[C * S]) {
  if (is_tip) {
    const int code = a.codes[(size_t)idx * a.n_pad + p];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int y = 0; y < S; ++y) v[c * S + y] = a.init[code * S + y];
  } else {
    const int64_t tile = p >> 7, q = p & (kTile - 1);
    const double* L = a.partials + (size_t)idx * a.slot_stride + tile * ((int64_t)C * S * kTile) + q;
#pragma unroll
    for (int i = 0; i < C * S; ++i) v[i] = L[(size_t)i * kTile];
  }
}

// out[c][x] = sum_y M[c][x][y] v[c][y]
template <int S, int C>
__device__ __forceinline__ void matvec(const double* __restrict__ M, const double (&v)[C * S], double (&out)[C * S]) {
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int x = 0; x < S; ++x) {
      const double* Mx = M + (c * S + x) * S;
      double s = Mx[0] * v[c * S];
#pragma unroll
      for (int y = 1; y < S; ++y) s = __builtin_fma(Mx[y], v[c * S + y], s);
      out[c * S + x] = s;
    }
}

template <int S, int C>
__global__ __launch_bounds__(256) void deriv_kernel(DerivArgs a, const DInstr* __restrict__ prog,
                                                    const double* __restrict__ pmats,
                                                    const double* __restrict__ dpmats,
                                                    const double* __restrict__ d2pmats, int guard) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // < n_pad
  double L[C * S], dL[C * S], d2L[C * S];
  double nL[C * S], ndL[C * S], nd2L[C * S];
  bool first = true;
#pragma unroll
  for (int i = 0; i < C * S; ++i) nL[i] = ndL[i] = nd2L[i] = 1.0;
  const DInstr* __restrict__ pc = prog;
  for (;;) {
    const DInstr in = *pc++;
    if (in.op == D_END) break;
    const size_t moff = (size_t)in.b * C * S * S;
    if (in.op == D_STEP) {
      // node complete: joint rescale by L's maximum (keeps dl / l exact)
      double m = 0.0;
#pragma unroll
      for (int i = 0; i < C * S; ++i) m = fmax(m, nL[i]);
      const double f = (m > 0.0 && m < kScaleThr) ? kScaleUp : 1.0;
#pragma unroll
      for (int i = 0; i < C * S; ++i) {
        L[i] = nL[i] * f;
        dL[i] = ndL[i] * f;
        d2L[i] = nd2L[i] * f;
        nL[i] = ndL[i] = nd2L[i] = 1.0;
      }
      first = false;
      continue;
    }
    double v[C * S], s[C * S];
    if (in.op == D_PATH && !first) {
      matvec<S, C>(pmats + moff, L, s);
#pragma unroll
      for (int i = 0; i < C * S; ++i) nL[i] *= s[i];
      matvec<S, C>(pmats + moff, dL, s);
#pragma unroll
      for (int i = 0; i < C * S; ++i) ndL[i] *= s[i];
      matvec<S, C>(pmats + moff, d2L, s);
#pragma unroll
      for (int i = 0; i < C * S; ++i) nd2L[i] *= s[i];
    } else if (in.op == D_PATH) {
      load_son<S, C>(a, in.d, in.a, p, v);
      matvec<S, C>(pmats + moff, v, s);
#pragma unroll
      for (int i = 0; i < C * S; ++i) nL[i] *= s[i];
      matvec<S, C>(dpmats + moff, v, s);
#pragma unroll
      for (int i = 0; i < C * S; ++i) ndL[i] *= s[i];
      matvec<S, C>(d2pmats + moff, v, s);
#pragma unroll
      for (int i = 0; i < C * S; ++i) nd2L[i] *= s[i];
    } else {
      load_son<S, C>(a, in.op == D_TIP, in.a, p, v);
      matvec<S, C>(pmats + moff, v, s);
#pragma unroll
      for (int i = 0; i < C * S; ++i) {
        nL[i] *= s[i];
        ndL[i] *= s[i];
        nd2L[i] *= s[i];
      }
    }
  }
  // root: l (with the reference's per-class guards), dl, d2l
  double l = 0.0, dl = 0.0, d2l = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    double lc = 0.0, dlc = 0.0, d2lc = 0.0;
#pragma unroll
    for (int x = 0; x < S; ++x) {
      const double li = L[c * S + x] * a.pi[x];
      if (!guard || li > 0.0) lc += li;
      dlc += dL[c * S + x] * a.pi[x];
      d2lc += d2L[c * S + x] * a.pi[x];
    }
    l += lc * a.probs[c];
    dl += dlc * a.probs[c];
    d2l += d2lc * a.probs[c];
  }
  double r1 = 0.0, r2 = 0.0;
  if (p < a.n_patterns) {
    const double g = dl / l;
    r1 = a.weights[p] * g;
    r2 = a.weights[p] * (d2l / l - g * g);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    r1 += __shfl_xor(r1, off, 64);
    r2 += __shfl_xor(r2, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    a.d1_sums[p >> 6] = r1;
    a.d2_sums[p >> 6] = r2;
  }
}

// ---------------------------------------------------------------------------
// Any S, C: derivatives from the path partials of plk_branch_derivatives' levelwise
// path (dL and d2L of the root computed by the partials kernels with the branch's P
// replaced by r_c dP/dt and r_c^2 d2P/dt2 -- lnL is linear in P of one branch).  Each
// root vector carries its own power-of-two scale count, so per pattern
//   dl / l = (dl' / l') 2^(256 (k - k1)),   d2l / l = (d2l'' / l') 2^(256 (k - k2))
// with the same guards as deriv_kernel (per-term <= 0 dropped in l only).
// ---------------------------------------------------------------------------
struct DRArgs {
  const double* L;    // root slot
  const double* dL;   // root dL (scratch slot)
  const double* d2L;  // root d2L (scratch slot)
  const int32_t* k0;  // scale rows (null without scaling)
  const int32_t* k1;
  const int32_t* k2;
  const double* pi;
  const double* probs;
  const double* weights;
  double* d1_sums;
  double* d2_sums;
  int64_t n_patterns;
  int S, C, guard;
};

__global__ __launch_bounds__(256) void deriv_reduce_kernel(DRArgs a) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tile = p >> 7, q = p & (kTile - 1);
  const int CS = a.C * a.S;
  double r1 = 0.0, r2 = 0.0;
  if (p < a.n_patterns) {
    const size_t off = (size_t)tile * CS * kTile + q;
    double l = 0.0, dl = 0.0, d2l = 0.0;
    for (int c = 0; c < a.C; ++c) {
      double lc = 0.0, dlc = 0.0, d2lc = 0.0;
      for (int x = 0; x < a.S; ++x) {
        const size_t i = off + (size_t)(c * a.S + x) * kTile;
        const double li = a.L[i] * a.pi[x];
        if (!a.guard || li > 0.0) lc += li;
        dlc += a.dL[i] * a.pi[x];
        d2lc += a.d2L[i] * a.pi[x];
      }
      l += lc * a.probs[c];
      dl += dlc * a.probs[c];
      d2l += d2lc * a.probs[c];
    }
    double g = dl / l, hh = d2l / l;
    if (a.k0) {
      g = ldexp(g, 256 * (a.k0[p] - a.k1[p]));
      hh = ldexp(hh, 256 * (a.k0[p] - a.k2[p]));
    }
    r1 = a.weights[p] * g;
    r2 = a.weights[p] * (hh - g * g);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    r1 += __shfl_xor(r1, off, 64);
    r2 += __shfl_xor(r2, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    a.d1_sums[p >> 6] = r1;
    a.d2_sums[p >> 6] = r2;
  }
}

// ---------------------------------------------------------------------------
// Root-pair derivatives (plk_root_pair_derivatives): the lengths of two sons a, b of the
// root move together, t_a + alpha s and t_b + beta s -- the reference's BrLenRoot
// (alpha = RootPosition, beta = 1 - RootPosition) and RootPosition (alpha = -beta =
// BrLenRoot), RNonHomogeneousTreeLikelihood.cpp:391-560 and 862-1100.  The root vector is
// bilinear in (P_a, P_b), so per pattern
//   l'  = alpha l_a + beta l_b,   l'' = alpha^2 l_aa + 2 alpha beta l_ab + beta^2 l_bb
// with l_x the root reduction of the root product whose a / b factors carry dP / d2P
// (X[0..4] = a, b, aa, bb, ab).  Each product has its own power-of-two scale count.
// ---------------------------------------------------------------------------
struct PairArgs {
  const double* L;        // root slot
  const double* X[5];     // substituted root products
  const int32_t* k0;      // scale rows (null without scaling)
  const int32_t* kx[5];
  const double* pi;
  const double* probs;
  const double* weights;
  double* d1_sums;
  double* d2_sums;
  int64_t n_patterns;
  double alpha, beta;
  int S, C, guard;
};

__global__ __launch_bounds__(256) void pair_reduce_kernel(PairArgs a) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t tile = p >> 7, q = p & (kTile - 1);
  const int CS = a.C * a.S;
  double r1 = 0.0, r2 = 0.0;
  if (p < a.n_patterns) {
    const size_t off = (size_t)tile * CS * kTile + q;
    double l = 0.0, lx[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    for (int c = 0; c < a.C; ++c) {
      double lc = 0.0, lxc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
      for (int x = 0; x < a.S; ++x) {
        const size_t i = off + (size_t)(c * a.S + x) * kTile;
        const double li = a.L[i] * a.pi[x];
        if (!a.guard || li > 0.0) lc += li;
#pragma unroll
        for (int v = 0; v < 5; ++v) lxc[v] += a.X[v][i] * a.pi[x];
      }
      l += lc * a.probs[c];
#pragma unroll
      for (int v = 0; v < 5; ++v) lx[v] += lxc[v] * a.probs[c];
    }
    double g[5];
#pragma unroll
    for (int v = 0; v < 5; ++v) g[v] = a.k0 ? ldexp(lx[v] / l, 256 * (a.k0[p] - a.kx[v][p])) : lx[v] / l;
    const double g1 = a.alpha * g[0] + a.beta * g[1];
    const double g2 = a.alpha * a.alpha * g[2] + a.beta * a.beta * g[3] + 2.0 * a.alpha * a.beta * g[4];
    r1 = a.weights[p] * g1;
    r2 = a.weights[p] * (g2 - g1 * g1);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    r1 += __shfl_xor(r1, off, 64);
    r2 += __shfl_xor(r2, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    a.d1_sums[p >> 6] = r1;
    a.d2_sums[p >> 6] = r2;
  }
}

}  // namespace plk
