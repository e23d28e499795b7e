// plk_treeS.hpp -- fused postorder traversal for S-state models with S > 4 (protein,
// S = 20) on gfx950.
//
// Same tree programs (TInstr words, fragments, tiers) as the 4-state kernel in
// plk_tree4.hpp, with one wave per rate class: a workgroup owns 64 consecutive site
// patterns (one per lane) and C waves.  Level d of the current root-to-node path
// keeps the pending product of an open ancestor in S registers per lane; the
// child's contribution
//     acc[x] *= sum_y P_son[c][x][y] L_son[c][y]      (RHomogeneousTreeLikelihood.cpp:839-861)
// is an S x S matvec with P(t) streamed from the scalar cache (wave-uniform rows,
// s_load into SGPRs) and the child vector in VGPRs, so the partials of the nodes
// inside a fragment never touch HBM.  The register depth DM is small (S doubles per
// level), so a fragment is a subtree of height <= DM; fragment roots are
// materialised and LOADed by the next tier.  Leaves use the per-branch tip tables
// tipP[tip][c][code][x] = sum_y P[x][y] init[code][y] (tip_table_kernel): one
// 160-byte row per lane instead of a matvec.  Rescaling and the fused root
// reduction follow plk_tree4.hpp exactly (joint max over classes through LDS; the
// same fixed-order wave butterfly), so the block sums have the same structure.
#pragma once

#include "plk_tree4.hpp"

namespace plk {

// dst[x] *= sum_y P[x][y] * src[y]
template <int S>
__device__ __forceinline__ void contribute_s(double (&dst)[S], const double (&src)[S],
                                             const double* __restrict__ P) {
#pragma unroll
  for (int x = 0; x < S; ++x) {
    const double* Px = P + x * S;
    double s = Px[0] * src[0];
#pragma unroll
    for (int y = 1; y < S; ++y) s = __builtin_fma(Px[y], src[y], s);
    dst[x] *= s;
  }
}

template <int S>
__device__ __forceinline__ void rescale_s(double (&v)[S], int& cnt, double* xmax, int nw) {
  double m = 0.0;
#pragma unroll
  for (int i = 0; i < S; ++i) m = fmax(m, v[i]);
  if (nw > 1) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    xmax[w * 64 + lane] = m;
    __syncthreads();
    m = 0.0;
    for (int k = 0; k < nw; ++k) m = fmax(m, xmax[k * 64 + lane]);
    __syncthreads();
  }
  if (m > 0.0 && m < kScaleThr) {
#pragma unroll
    for (int i = 0; i < S; ++i) v[i] *= kScaleUp;
    cnt += 1;
  }
}

template <int S, bool SCALE>
__device__ __forceinline__ void store_partial_s(const TreeArgs& a, int slot, int64_t p, int c0, const double (&v)[S],
                                                int cnt) {
  const int64_t tile = p >> 7, q = p & (kTile - 1);
  double* dst = a.partials + (size_t)slot * a.slot_stride + tile * ((int64_t)a.C * S * kTile) + (size_t)c0 * S * kTile + q;
#pragma unroll
  for (int i = 0; i < S; ++i) __builtin_nontemporal_store(v[i], dst + (size_t)i * kTile);
  if (SCALE && c0 == 0) a.scale[(size_t)slot * a.n_pad + p] = cnt;
}

template <int S, int D, int DM, bool SCALE>
__device__ __forceinline__ void eval_node_s(const TreeArgs& a, const TInstr* __restrict__& pc,
                                            const double* __restrict__ pmats, double* xch, int nw, int c0, int64_t p,
                                            double (&acc)[S], int& cnt) {
#pragma unroll
  for (int i = 0; i < S; ++i) acc[i] = 1.0;
  cnt = 0;
  for (;;) {
    const TInstr in = fetch_instr(pc++);
    if (in.op == T_ASCEND) {
      if (in.b >= 0) {
        if (SCALE) rescale_s<S>(acc, cnt, xch, nw);
        if (in.a >= 0) store_partial_s<S, SCALE>(a, in.a, p, c0, acc, cnt);
      }
      return;
    }
    if (in.op == T_TIP) {
      const int code = a.codes[(size_t)in.a * a.n_pad + p];
      const double2* t =
          reinterpret_cast<const double2*>(a.tipP + (((size_t)in.a * a.C + c0) * a.n_codes + code) * S);
#pragma unroll
      for (int i = 0; i < S / 2; ++i) {
        const double2 v = t[i];
        acc[2 * i] *= v.x;
        acc[2 * i + 1] *= v.y;
      }
    } else if (in.op == T_LOAD) {
      const int64_t tile = p >> 7, q = p & (kTile - 1);
      const double* L = a.partials + (size_t)in.a * a.slot_stride + tile * ((int64_t)a.C * S * kTile) +
                        (size_t)c0 * S * kTile + q;
      double src[S];
#pragma unroll
      for (int i = 0; i < S; ++i) src[i] = L[(size_t)i * kTile];
      if (SCALE) cnt += a.scale[(size_t)in.a * a.n_pad + p];
      contribute_s<S>(acc, src, pmats + ((size_t)in.b * a.C + c0) * S * S);
    } else {  // T_DESCEND
      if constexpr (D + 1 < DM) {
        double child[S];
        int ccnt;
        eval_node_s<S, D + 1, DM, SCALE>(a, pc, pmats, xch, nw, c0, p, child, ccnt);
        const TInstr up = fetch_instr(pc - 1);
        contribute_s<S>(acc, child, pmats + ((size_t)up.b * a.C + c0) * S * S);
        if (SCALE) cnt += ccnt;
      }
    }
  }
}

template <int S, int DM, bool SCALE>
__global__ __launch_bounds__(256) void treeS_kernel(TreeArgs a, const TInstr* __restrict__ prog,
                                                    const int32_t* __restrict__ frag_start,
                                                    const double* __restrict__ pmats) {
  __shared__ double xch[kTreeMaxWaves * 64];
  const int nw = blockDim.x >> 6;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c0 = w;  // one class per wave
  const int64_t p0 = (int64_t)blockIdx.x * 64;
  const int64_t p = p0 + lane;
  const TInstr* __restrict__ pc = prog + frag_start[blockIdx.y];
  double acc[S];
  int cnt;
  eval_node_s<S, 0, DM, SCALE>(a, pc, pmats, xch, nw, c0, p, acc, cnt);
  const TInstr in = fetch_instr(pc);  // T_ROOT
  if (SCALE) rescale_s<S>(acc, cnt, xch, nw);
  if (in.a >= 0) store_partial_s<S, SCALE>(a, in.a, p, c0, acc, cnt);
  if (in.b) {
    double lc = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const double li = acc[s] * a.pi[s];
      if (a.guard) {
        if (li > 0.0) lc += li;
      } else {
        lc += li;
      }
    }
    const double t = lc * a.probs[c0];
    __syncthreads();
    xch[c0 * 64 + lane] = t;
    __syncthreads();
    if (w == 0) {
      double l = 0.0;
      for (int c = 0; c < a.C; ++c) {
        const double li = xch[c * 64 + lane];
        if (a.guard) {
          if (li > 0.0) l += li;
        } else {
          l += li;
        }
      }
      if (!a.guard && l < 0.0) l = 0.0;
      double r = log(l);
      if (SCALE) r -= (double)cnt * kLn2x256;
      double wr = 0.0;
      if (p < a.n_patterns) {
        a.site_lnl[p] = r;
        wr = a.weights[p] * r;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) wr += __shfl_xor(wr, off, 64);
      if (lane == 0) a.wave_sums[p0 >> 6] = wr;
    }
  }
}

}  // namespace plk
