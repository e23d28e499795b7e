// plk_kernels.hpp -- CDNA4 (gfx950) device code of libplk.
//
// Hot path: the per-node partial-likelihood update of
// RHomogeneousTreeLikelihood::computeSubtreeLikelihood
// (/root/reference/src/Bpp/Phyl/Likelihood/RHomogeneousTreeLikelihood.cpp:802-863):
//     L_node[i][c][x] = prod_son sum_y P_son[c][x][y] * L_son[i][c][y]
// plus the batched transition-matrix exponential behind getPij_t
// (Model/AbstractSubstitutionModel.cpp:426-641) and the root reduction
// (Likelihood/RHomogeneousTreeLikelihood.cpp:162-216).
//
// HBM layout (site-pattern-major, tiled): a partial vector of one internal node
// is [tile][c*S + s][kTile] fp64 with kTile = 128 patterns per tile.  One
// wave-instruction of the 4-state kernel loads 64 lanes x 16 B (two adjacent
// patterns per lane) = 1 KiB contiguous; the generic kernel loads 64 x 8 B.
// Tips are stored as one uint8 state code per pattern and resolved through a
// per-branch table tipP[c][code][x] = sum_y P[c][x][y] * init[code][y], which
// replaces the reference's dense one-hot leaf matvec.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace plk {

constexpr int kTile = 128;          // patterns per tile (layout granule)
constexpr int kRootBlock = 4096;    // patterns per fixed-order reduction block
constexpr int kMaxCodes4 = 32;      // code-table rows the 4-state kernel stages in LDS
constexpr double kScaleUp = 115792089237316195423570985008687907853269984665640564039457584007913129639936.0;  // 2^256
constexpr double kScaleThr = 1.0 / kScaleUp;                                                                 // 2^-256
constexpr double kLn2x256 = 177.44567822334599921;                                                           // 256 ln 2

// Device-side description of one partial update (children already resolved
// into tip indices or internal slots).
struct KOp {
  int32_t parent;    // internal slot
  int32_t n;         // number of children (1..3)
  int32_t child[3];  // tip index (is_tip) or internal slot
  int32_t branch[3]; // node index of the child = transition-matrix index
  int32_t is_tip[3];
  int32_t flags;     // PLK_OP_ACCUMULATE
};

struct PartialsArgs {
  double* partials;          // [n_internal][slot_stride]
  int32_t* scale;            // [n_internal][n_pad] (SCALE only)
  const uint8_t* codes;      // [n_tips][n_pad]
  const double* tipP;        // [n_tips][C][n_codes][S]
  const double* pmats;       // [n_nodes][C][S][S]
  int64_t slot_stride;       // doubles per internal slot = n_tiles * C*S * kTile
  int64_t n_pad;             // padded pattern count
  int32_t n_tiles;
  int32_t n_codes;
};

// ---------------------------------------------------------------------------
// 4-state kernel: one lane = two adjacent patterns (double2 loads/stores),
// one wave = one 128-pattern tile, 4 waves per workgroup.  P(t) of the branch
// is wave-uniform and lives in scalar registers (s_load), tip tables in LDS.
// HBM-bound: per internal child 16*C B/pattern read, 8*C*S B/pattern written.
// ---------------------------------------------------------------------------
template <int C, bool SCALE>
__global__ __launch_bounds__(256) void partials_s4_kernel(const KOp* __restrict__ ops, PartialsArgs a) {
  constexpr int S = 4;
  constexpr int CS = C * S;
  __shared__ double tipT[3][C * kMaxCodes4 * S];
  const KOp& op = ops[blockIdx.y];
  const int n = op.n;
  const int nc = a.n_codes;
  // Stage the tip tables of tip children.
  for (int k = 0; k < n; ++k) {
    if (op.is_tip[k]) {
      const double* src = a.tipP + (size_t)op.child[k] * (C * nc * S);
      for (int i = threadIdx.x; i < C * nc * S; i += blockDim.x) tipT[k][i] = src[i];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tile >= a.n_tiles) return;
  const size_t toff = (size_t)tile * (CS * kTile);
  double2* outp = reinterpret_cast<double2*>(a.partials + (size_t)op.parent * a.slot_stride + toff) + lane;

  double2 acc[C][S];
  int2 cnt = make_int2(0, 0);
  if (op.flags & 1) {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int x = 0; x < S; ++x) acc[c][x] = outp[(c * S + x) * (kTile / 2)];
    if (SCALE) cnt = reinterpret_cast<const int2*>(a.scale + (size_t)op.parent * a.n_pad + (size_t)tile * kTile)[lane];
  } else {
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int x = 0; x < S; ++x) acc[c][x] = make_double2(1.0, 1.0);
  }

  for (int k = 0; k < n; ++k) {
    const int child = op.child[k];
    if (op.is_tip[k]) {
      const uint16_t cc =
          reinterpret_cast<const uint16_t*>(a.codes + (size_t)child * a.n_pad + (size_t)tile * kTile)[lane];
      const int c0 = cc & 0xff, c1 = cc >> 8;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const double* t0 = &tipT[k][(c * nc + c0) * S];
        const double* t1 = &tipT[k][(c * nc + c1) * S];
#pragma unroll
        for (int x = 0; x < S; ++x) {
          acc[c][x].x *= t0[x];
          acc[c][x].y *= t1[x];
        }
      }
    } else {
      const double* __restrict__ P = a.pmats + (size_t)op.branch[k] * (C * S * S);
      const double2* L = reinterpret_cast<const double2*>(a.partials + (size_t)child * a.slot_stride + toff) + lane;
      double2 l[C][S];
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int y = 0; y < S; ++y) l[c][y] = L[(c * S + y) * (kTile / 2)];
#pragma unroll
      for (int c = 0; c < C; ++c) {
#pragma unroll
        for (int x = 0; x < S; ++x) {
          const double* Px = P + (c * S + x) * S;
          double s0 = Px[0] * l[c][0].x, s1 = Px[0] * l[c][0].y;
#pragma unroll
          for (int y = 1; y < S; ++y) {
            s0 = __builtin_fma(Px[y], l[c][y].x, s0);
            s1 = __builtin_fma(Px[y], l[c][y].y, s1);
          }
          acc[c][x].x *= s0;
          acc[c][x].y *= s1;
        }
      }
      if (SCALE) {
        const int2 sc = reinterpret_cast<const int2*>(a.scale + (size_t)child * a.n_pad + (size_t)tile * kTile)[lane];
        cnt.x += sc.x;
        cnt.y += sc.y;
      }
    }
  }

  if (SCALE) {
    double m0 = 0.0, m1 = 0.0;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int x = 0; x < S; ++x) {
        m0 = fmax(m0, acc[c][x].x);
        m1 = fmax(m1, acc[c][x].y);
      }
    const bool r0 = (m0 > 0.0 && m0 < kScaleThr), r1 = (m1 > 0.0 && m1 < kScaleThr);
    if (r0 || r1) {
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int x = 0; x < S; ++x) {
          if (r0) acc[c][x].x *= kScaleUp;
          if (r1) acc[c][x].y *= kScaleUp;
        }
      cnt.x += r0;
      cnt.y += r1;
    }
    reinterpret_cast<int2*>(a.scale + (size_t)op.parent * a.n_pad + (size_t)tile * kTile)[lane] = cnt;
  }
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int x = 0; x < S; ++x) outp[(c * S + x) * (kTile / 2)] = acc[c][x];
}

// ---------------------------------------------------------------------------
// Per-subtree site-pattern compression (reference usePatterns = true,
// Likelihood/DRASRTreeLikelihoodData.cpp:218-332): a node's partial is computed once
// per DISTINCT pattern of its subtree's tips (D of them, D <= n_patterns; the first D
// entries of its slot, same tile layout) and each child is read through a pattern
// link -- the child's distinct pattern (or, for a tip, its compact code) of parent
// pattern j, the reference's patternLinks_[node][son].  One lane = one parent
// pattern; the arithmetic per pattern is partials_s4_kernel's, so the values are
// bitwise those of the uncompressed traversal.
// ---------------------------------------------------------------------------
struct KOpL {
  int32_t parent;    // internal slot
  int32_t n;         // children (any number: a polytomy's whole list)
  int32_t D;         // distinct patterns of the parent's subtree
  int32_t k0;        // its first child record (KKid)
};
struct KKid {
  int32_t child;     // tip index or internal slot
  int32_t branch;    // node index of the child = transition-matrix index
  int32_t is_tip;
  int32_t pad_;
  int64_t link;      // offset of the child's link array (D uint32) in the link pool
};
// The links kernels stage the tables of three children at a time in LDS; a node with more
// (a polytomy) takes them three by three, its product in the children's order.
constexpr int kLinkGroup = 3;

template <int C, bool SCALE>
__global__ __launch_bounds__(256) void partials_links_s4_kernel(const KOpL* __restrict__ ops, const KKid* __restrict__ kids,
                                                                PartialsArgs a, const uint32_t* __restrict__ links) {
  constexpr int S = 4;
  constexpr int CS = C * S;
  __shared__ double tipT[kLinkGroup][C * kMaxCodes4 * S];
  const KOpL& op = ops[blockIdx.y];
  const int n = op.n;
  const int nc = a.n_codes;
  if ((int)(blockIdx.x * blockDim.x) >= op.D) return;  // whole workgroup past this op's patterns
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double acc[C][S];
  int cnt = 0;
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int x = 0; x < S; ++x) acc[c][x] = 1.0;
  for (int g0 = 0; g0 < n; g0 += kLinkGroup) {
    const int gn = n - g0 < kLinkGroup ? n - g0 : kLinkGroup;
    if (g0 > 0) __syncthreads();  // the previous group's tables are read
    for (int k = 0; k < gn; ++k) {
      const KKid& kd = kids[op.k0 + g0 + k];
      if (kd.is_tip) {
        const double* src = a.tipP + (size_t)kd.child * (C * nc * S);
        for (int i = threadIdx.x; i < C * nc * S; i += blockDim.x) tipT[k][i] = src[i];
      }
    }
    __syncthreads();
    if (j < op.D)
      for (int k = 0; k < gn; ++k) {
        const KKid& kd = kids[op.k0 + g0 + k];
        const uint32_t l = links[kd.link + j];
        if (kd.is_tip) {
#pragma unroll
          for (int c = 0; c < C; ++c) {
            const double* t = &tipT[k][(c * nc + (int)l) * S];
#pragma unroll
            for (int x = 0; x < S; ++x) acc[c][x] *= t[x];
          }
        } else {
          const double* __restrict__ P = a.pmats + (size_t)kd.branch * (C * S * S);
          const double* L = a.partials + (size_t)kd.child * a.slot_stride + (size_t)(l >> 7) * (CS * kTile) + (l & 127);
          double v[C][S];
#pragma unroll
          for (int c = 0; c < C; ++c)
#pragma unroll
            for (int y = 0; y < S; ++y) v[c][y] = L[(c * S + y) * kTile];
#pragma unroll
          for (int c = 0; c < C; ++c)
#pragma unroll
            for (int x = 0; x < S; ++x) {
              const double* Px = P + (c * S + x) * S;
              double s = Px[0] * v[c][0];
#pragma unroll
              for (int y = 1; y < S; ++y) s = __builtin_fma(Px[y], v[c][y], s);
              acc[c][x] *= s;
            }
          if (SCALE) cnt += a.scale[(size_t)kd.child * a.n_pad + l];
        }
      }
    // the joint rescale after every group of three, as the uncompressed traversal's
    // ACCUMULATE ops do (a wide polytomy's running product never drifts below 2^-256)
    if (SCALE && j < op.D) {
      double m = 0.0;
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int x = 0; x < S; ++x) m = fmax(m, acc[c][x]);
      if (m > 0.0 && m < kScaleThr) {
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
          for (int x = 0; x < S; ++x) acc[c][x] *= kScaleUp;
        cnt += 1;
      }
    }
  }
  if (j >= op.D) return;
  if (SCALE) a.scale[(size_t)op.parent * a.n_pad + j] = cnt;
  double* out = a.partials + (size_t)op.parent * a.slot_stride + (size_t)(j >> 7) * (CS * kTile) + (j & 127);
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int x = 0; x < S; ++x) out[(c * S + x) * kTile] = acc[c][x];
}

// Any state count: partials_generic_kernel's arithmetic (P and tip tables staged in LDS,
// XB states per chunk, the same product and FMA order) with the children read through
// their pattern links (the levelwise 20 / 64-state traversal runs K2 / K3, which sum in
// another order: 1e-12 apart).  One lane = one distinct pattern j of the parent (its slot
// entry j).
template <int S, int XB, bool SCALE>
__global__ __launch_bounds__(256) void partials_links_generic_kernel(const KOpL* __restrict__ ops,
                                                                     const KKid* __restrict__ kids, PartialsArgs a,
                                                                     const uint32_t* __restrict__ links, int C) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const KOpL& op = ops[blockIdx.y];
  const int n = op.n;
  const int nc = a.n_codes;
  const int CS = C * S;
  if ((int)(blockIdx.x * blockDim.x) >= op.D) return;  // whole workgroup past this op's patterns
  const int per = C * S * ((S > nc) ? S : nc);
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double* outp = a.partials + (size_t)op.parent * a.slot_stride + (size_t)(j >> 7) * ((size_t)CS * kTile) + (j & 127);
  int cnt = 0;
  // children three at a time (their tables in LDS); after the first group the product so
  // far is read back from the parent's slot and extended in the children's order, and
  // each group ends with the joint rescale, as the uncompressed traversal's ACCUMULATE ops
  for (int g0 = 0; g0 < n; g0 += kLinkGroup) {
    const int gn = n - g0 < kLinkGroup ? n - g0 : kLinkGroup;
    double m = 0.0;
    if (g0 > 0) __syncthreads();  // the previous group's tables are read
    for (int k = 0; k < gn; ++k) {
      const KKid& kd = kids[op.k0 + g0 + k];
      const double* src = kd.is_tip ? a.tipP + (size_t)kd.child * (C * nc * S) : a.pmats + (size_t)kd.branch * (C * S * S);
      const int nel = kd.is_tip ? C * nc * S : C * S * S;
      for (int i = threadIdx.x; i < nel; i += blockDim.x) lds[k * per + i] = src[i];
    }
    __syncthreads();
    if (j >= op.D) continue;
    uint32_t l[kLinkGroup] = {0u, 0u, 0u};
    for (int k = 0; k < gn; ++k) l[k] = links[kids[op.k0 + g0 + k].link + j];
    if (SCALE)
      for (int k = 0; k < gn; ++k) {
        const KKid& kd = kids[op.k0 + g0 + k];
        if (!kd.is_tip) cnt += a.scale[(size_t)kd.child * a.n_pad + l[k]];
      }
    for (int c = 0; c < C; ++c) {
      for (int x0 = 0; x0 < S; x0 += XB) {
        double acc[XB];
#pragma unroll
        for (int xb = 0; xb < XB; ++xb) acc[xb] = g0 == 0 ? 1.0 : outp[(size_t)(c * S + x0 + xb) * kTile];
        for (int k = 0; k < gn; ++k) {
          const KKid& kd = kids[op.k0 + g0 + k];
          if (kd.is_tip) {
            const double* t = &lds[k * per + (c * nc + (int)l[k]) * S + x0];
#pragma unroll
            for (int xb = 0; xb < XB; ++xb) acc[xb] *= t[xb];
          } else {
            const double* L = a.partials + (size_t)kd.child * a.slot_stride +
                              (size_t)(l[k] >> 7) * ((size_t)CS * kTile) + (l[k] & 127) + (size_t)c * S * kTile;
            const double* Pc = &lds[k * per + (c * S + x0) * S];
            double s[XB];
            {
              const double l0 = L[0];
#pragma unroll
              for (int xb = 0; xb < XB; ++xb) s[xb] = Pc[xb * S] * l0;
            }
#pragma unroll 4
            for (int y = 1; y < S; ++y) {
              const double ly = L[(size_t)y * kTile];
#pragma unroll
              for (int xb = 0; xb < XB; ++xb) s[xb] = __builtin_fma(Pc[xb * S + y], ly, s[xb]);
            }
#pragma unroll
            for (int xb = 0; xb < XB; ++xb) acc[xb] *= s[xb];
          }
        }
#pragma unroll
        for (int xb = 0; xb < XB; ++xb) {
          if (SCALE) m = fmax(m, acc[xb]);
          outp[(size_t)(c * S + x0 + xb) * kTile] = acc[xb];
        }
      }
    }
    if (SCALE && m > 0.0 && m < kScaleThr) {
      for (int i = 0; i < CS; ++i) outp[(size_t)i * kTile] *= kScaleUp;
      cnt += 1;
    }
  }
  if (j >= op.D) return;
  if (SCALE) a.scale[(size_t)op.parent * a.n_pad + j] = cnt;
}

// ---------------------------------------------------------------------------
// Generic-S kernel (S up to 64): one lane = one pattern, 2 tiles per 256-thread
// workgroup.  The children's P(t) (C x S x S each) and tip tables are staged in
// LDS once per workgroup; inner products read P by wave-uniform LDS address
// (broadcast).  Outputs are produced in chunks of XB states per class.
// ---------------------------------------------------------------------------
template <int S, int XB, bool SCALE>
__global__ __launch_bounds__(256) void partials_generic_kernel(const KOp* __restrict__ ops, PartialsArgs a, int C) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const KOp& op = ops[blockIdx.y];
  const int n = op.n;
  const int nc = a.n_codes;
  const int CS = C * S;
  // LDS image: per child k, either P (C*S*S) or tipP (C*nc*S); offset k*per.
  const int per = C * S * ((S > nc) ? S : nc);
  for (int k = 0; k < n; ++k) {
    const double* src = op.is_tip[k] ? a.tipP + (size_t)op.child[k] * (C * nc * S)
                                     : a.pmats + (size_t)op.branch[k] * (C * S * S);
    const int cnt = op.is_tip[k] ? C * nc * S : C * S * S;
    for (int i = threadIdx.x; i < cnt; i += blockDim.x) lds[k * per + i] = src[i];
  }
  __syncthreads();
  const int q = threadIdx.x & (kTile - 1);
  const int tile = blockIdx.x * 2 + (threadIdx.x >> 7);
  if (tile >= a.n_tiles) return;
  const size_t toff = (size_t)tile * ((size_t)CS * kTile) + q;
  double* outp = a.partials + (size_t)op.parent * a.slot_stride + toff;
  const size_t pidx = (size_t)tile * kTile + q;

  int cnt = 0;
  if (SCALE) {
    if (op.flags & 1) cnt = a.scale[(size_t)op.parent * a.n_pad + pidx];
    for (int k = 0; k < n; ++k)
      if (!op.is_tip[k]) cnt += a.scale[(size_t)op.child[k] * a.n_pad + pidx];
  }
  int code[3] = {0, 0, 0};
  for (int k = 0; k < n; ++k)
    if (op.is_tip[k]) code[k] = a.codes[(size_t)op.child[k] * a.n_pad + pidx];

  double m = 0.0;
  for (int c = 0; c < C; ++c) {
    for (int x0 = 0; x0 < S; x0 += XB) {
      double acc[XB];
      if (op.flags & 1) {
#pragma unroll
        for (int xb = 0; xb < XB; ++xb) acc[xb] = outp[(size_t)(c * S + x0 + xb) * kTile];
      } else {
#pragma unroll
        for (int xb = 0; xb < XB; ++xb) acc[xb] = 1.0;
      }
      for (int k = 0; k < n; ++k) {
        if (op.is_tip[k]) {
          const double* t = &lds[k * per + (c * nc + code[k]) * S + x0];
#pragma unroll
          for (int xb = 0; xb < XB; ++xb) acc[xb] *= t[xb];
        } else {
          const double* L = a.partials + (size_t)op.child[k] * a.slot_stride + toff + (size_t)c * S * kTile;
          const double* Pc = &lds[k * per + (c * S + x0) * S];
          double s[XB];
          {
            const double l0 = L[0];
#pragma unroll
            for (int xb = 0; xb < XB; ++xb) s[xb] = Pc[xb * S] * l0;
          }
#pragma unroll 4
          for (int y = 1; y < S; ++y) {
            const double ly = L[(size_t)y * kTile];
#pragma unroll
            for (int xb = 0; xb < XB; ++xb) s[xb] = __builtin_fma(Pc[xb * S + y], ly, s[xb]);
          }
#pragma unroll
          for (int xb = 0; xb < XB; ++xb) acc[xb] *= s[xb];
        }
      }
#pragma unroll
      for (int xb = 0; xb < XB; ++xb) {
        if (SCALE) m = fmax(m, acc[xb]);
        outp[(size_t)(c * S + x0 + xb) * kTile] = acc[xb];
      }
    }
  }
  if (SCALE) {
    if (m > 0.0 && m < kScaleThr) {
      for (int i = 0; i < CS; ++i) outp[(size_t)i * kTile] *= kScaleUp;
      cnt += 1;
    }
    a.scale[(size_t)op.parent * a.n_pad + pidx] = cnt;
  }
}

// ---------------------------------------------------------------------------
// K2: medium state counts (S = 20 amino acids).  One lane = one pattern; classes
// outer.  P(t) rows are wave-uniform and come from scalar loads straight into SGPRs
// (pmats is a separate __restrict__ argument so the compiler may use s_load), so each
// v_fma_f64 takes its P operand from an SGPR pair: no LDS traffic per FMA.  Tip
// children use the per-branch tip tables staged in LDS.  Child partials are read
// once per (class, child) into VGPRs (20 coalesced 512-B loads per wave).
// ---------------------------------------------------------------------------
template <int S, bool SCALE>
__global__ __launch_bounds__(256) void partials_sgpr_kernel(const KOp* __restrict__ ops, PartialsArgs a,
                                                            const double* __restrict__ pmats, int C) {
  extern __shared__ __attribute__((aligned(16))) double tipT[];  // [3][C][n_codes][S]
  const KOp& op = ops[blockIdx.y];
  const int n = op.n;
  const int nc = a.n_codes;
  const int per = C * nc * S;
  for (int k = 0; k < n; ++k)
    if (op.is_tip[k]) {
      const double* src = a.tipP + (size_t)op.child[k] * per;
      for (int i = threadIdx.x; i < per; i += blockDim.x) tipT[k * per + i] = src[i];
    }
  __syncthreads();
  const int q = threadIdx.x & (kTile - 1);
  const int tile = blockIdx.x * 2 + (threadIdx.x >> 7);
  if (tile >= a.n_tiles) return;
  const int CS = C * S;
  const size_t toff = (size_t)tile * ((size_t)CS * kTile) + q;
  double* outp = a.partials + (size_t)op.parent * a.slot_stride + toff;
  const size_t pidx = (size_t)tile * kTile + q;
  int code[3] = {0, 0, 0};
  for (int k = 0; k < n; ++k)
    if (op.is_tip[k]) code[k] = a.codes[(size_t)op.child[k] * a.n_pad + pidx];
  int cnt = 0;
  if (SCALE) {
    if (op.flags & 1) cnt = a.scale[(size_t)op.parent * a.n_pad + pidx];
    for (int k = 0; k < n; ++k)
      if (!op.is_tip[k]) cnt += a.scale[(size_t)op.child[k] * a.n_pad + pidx];
  }
  double m = 0.0;
  for (int c = 0; c < C; ++c) {
    double acc[S];
    if (op.flags & 1) {
#pragma unroll
      for (int x = 0; x < S; ++x) acc[x] = outp[(size_t)(c * S + x) * kTile];
    } else {
#pragma unroll
      for (int x = 0; x < S; ++x) acc[x] = 1.0;
    }
    for (int k = 0; k < n; ++k) {
      if (op.is_tip[k]) {
        const double* t = &tipT[k * per + (c * nc + code[k]) * S];
#pragma unroll
        for (int x = 0; x < S; ++x) acc[x] *= t[x];
      } else {
        const double* L = a.partials + (size_t)op.child[k] * a.slot_stride + toff + (size_t)c * S * kTile;
        double l[S];
#pragma unroll
        for (int y = 0; y < S; ++y) l[y] = __builtin_nontemporal_load(L + (size_t)y * kTile);
        const double* __restrict__ P = pmats + ((size_t)op.branch[k] * C + c) * S * S;
#pragma unroll
        for (int x = 0; x < S; ++x) {
          double s = P[x * S] * l[0];
#pragma unroll
          for (int y = 1; y < S; ++y) s = __builtin_fma(P[x * S + y], l[y], s);
          acc[x] *= s;
        }
      }
    }
#pragma unroll
    for (int x = 0; x < S; ++x) {
      if (SCALE) m = fmax(m, acc[x]);
      outp[(size_t)(c * S + x) * kTile] = acc[x];
    }
  }
  if (SCALE) {
    if (m > 0.0 && m < kScaleThr) {
      for (int i = 0; i < CS; ++i) outp[(size_t)i * kTile] *= kScaleUp;
      cnt += 1;
    }
    a.scale[(size_t)op.parent * a.n_pad + pidx] = cnt;
  }
}

// ---------------------------------------------------------------------------
// K4: batched transition matrices.  One workgroup per (branch i, class c):
//   P = V diag(exp(lambda * r_c * t_i)) Vinv                (getPij_t :426-438)
//   dP = r_c * V diag(lambda e) Vinv, d2P = r_c^2 V diag(lambda^2 e) Vinv
//   (AbstractHomogeneousTreeLikelihood.cpp:375-413, AbstractSubstitutionModel.cpp:499-641)
// ---------------------------------------------------------------------------
struct PmatArgs {
  const int32_t* branch;   // [n]
  const int32_t* model;    // [n] or null
  const double* t;         // [n]
  const double* rates;     // [C]
  const double* V;         // [n_models][S][S]
  const double* Vinv;      // [n_models][S][S]
  const double* lambda;    // [n_models][S]
  double* P;               // [n_nodes][C][S][S]
  double* PT;              // P transposed, [n_nodes][C][y][x] (pmat64s_kernel; null: not written)
  double* dP;
  double* d2P;
  const double* init;      // [n_codes][S] code table (null: no tip tables)
  double* tipP;            // [n_tips][C][n_codes][S]
  int n_tips, n_codes;
  int S, C;
  unsigned mask;
  int n_req;               // branches in the request
  int uni_model;           // every entry of the request uses this model (-1: mixed or unknown)
};

// Requests of up to kPmatInline branches travel in the kernel arguments (no staging
// copy, no dependent launch in front of the kernel).
constexpr int kPmatInline = 160;
struct PmatInline {
  double t[kPmatInline];
  int32_t branch[kPmatInline];
  int32_t model[kPmatInline];
  int32_t n;  // 0: use PmatArgs' device arrays
};
// the same for requests of up to 64 branches (cfg2: 62): a 1 KB argument block instead of
// 2.5 KB -- the launch copies every argument byte into the kernel-argument buffer
constexpr int kPmatInlineSmall = 64;
struct PmatInlineSmall {
  double t[kPmatInlineSmall];
  int32_t branch[kPmatInlineSmall];
  int32_t model[kPmatInlineSmall];
  int32_t n;
};

// n doubles global -> LDS, the first NE * blockDim.x of them with every thread's loads
// issued before its first store (a load -> store loop pays one L2 round trip per element and
// thread); any remainder (n beyond NE * blockDim.x, e.g. more codes than a launch sized for)
// element by element
template <int NE>
__device__ __forceinline__ void stage_lds(double* __restrict__ dst, const double* __restrict__ src, int n) {
  double r[NE];
#pragma unroll
  for (int q = 0; q < NE; ++q) {
    const int k = (int)threadIdx.x + (int)blockDim.x * q;
    r[q] = src[k < n ? k : 0];
  }
#pragma unroll
  for (int q = 0; q < NE; ++q) {
    const int k = (int)threadIdx.x + (int)blockDim.x * q;
    if (k < n) dst[k] = r[q];
  }
  for (int k = (int)threadIdx.x + (int)blockDim.x * NE; k < n; k += (int)blockDim.x) dst[k] = src[k];
}

// NE: S * S / blockDim.x rounded up (the staging loads per thread)
template <int NE>
__global__ __launch_bounds__(256) void pmat_kernel(PmatArgs a, const PmatInline inl) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int i = blockIdx.x, c = blockIdx.y, S = a.S;
  const int b = inl.n ? inl.branch[i] : a.branch[i];
  const int m = inl.n ? inl.model[i] : (a.model ? a.model[i] : 0);
  const double rc = a.rates[c];
  const double tt = (inl.n ? inl.t[i] : a.t[i]) * rc;
  double* e = sm;           // exp(lambda t)
  double* Vm = sm + S;      // V
  double* Vi = Vm + S * S;  // Vinv
  const double* V = a.V + (size_t)m * S * S;
  const double* lam = a.lambda + (size_t)m * S;
  for (int k = threadIdx.x; k < S; k += blockDim.x) e[k] = exp(lam[k] * tt);
  stage_lds<NE>(Vm, V, S * S);
  stage_lds<NE>(Vi, a.Vinv + (size_t)m * S * S, S * S);
  __syncthreads();
  const size_t off = ((size_t)b * a.C + c) * S * S;
  for (int idx = threadIdx.x; idx < S * S; idx += blockDim.x) {
    const int x = idx / S, y = idx % S;
    double p = 0.0, dp = 0.0, d2p = 0.0;
    for (int k = 0; k < S; ++k) {
      const double w = Vm[x * S + k] * Vi[k * S + y];
      const double ek = e[k];
      p = __builtin_fma(w, ek, p);
      if (a.mask & 6u) {
        const double le = lam[k] * ek;
        dp = __builtin_fma(w, le, dp);
        d2p = __builtin_fma(w, lam[k] * le, d2p);
      }
    }
    if (tt == 0.0) p = (x == y) ? 1.0 : 0.0;  // getPij_t: t == 0 -> identity (:428-431)
    if (a.mask & 1u) a.P[off + idx] = p;
    if (a.PT && (a.mask & 1u)) a.PT[off + (size_t)y * S + x] = p;  // transposed copy (transpose_pmats' layout)
    if (a.mask & 2u) a.dP[off + idx] = rc * dp;
    if (a.mask & 4u) a.d2P[off + idx] = rc * rc * d2p;
    if (a.init && b < a.n_tips) Vi[S * S + idx] = p;
  }
  // tip branch: its table row tipP[b][c][code][x] = sum_y P[x][y] init[code][y], with
  // tip_table_kernel's arithmetic (the fused kernels read tips through it)
  if (a.init && b < a.n_tips && (a.mask & 1u)) {
    __syncthreads();
    const double* Pl = Vi + S * S;
    double* out = a.tipP + ((size_t)b * a.C + c) * a.n_codes * S;
    for (int idx = threadIdx.x; idx < a.n_codes * S; idx += blockDim.x) {
      const int code = idx / S, x = idx % S;
      double t = 0.0;
      for (int y = 0; y < S; ++y) t = __builtin_fma(Pl[x * S + y], a.init[code * S + y], t);
      out[idx] = t;
    }
  }
}

// K4 for 4 states: one thread per (branch, class, row x) -- its row of P (and dP, d2P) and
// the row's entries of the tip table -- with pmat_kernel's operations in the same order
// (bitwise its results).  pmat_kernel's workgroup per (branch, class) ran a chain of
// dependent loads, LDS staging and barriers for 16 outputs; here each thread issues its
// loads at once and the launch is n * C * 4 threads.
template <class Inl>
__global__ __launch_bounds__(64) void pmat4_kernel(PmatArgs a, const Inl inl) {
  constexpr int S = 4;
  const int gid = blockIdx.x * 64 + threadIdx.x;
  if (gid >= a.n_req * a.C * S) return;
  const int x = gid & 3, ic = gid >> 2, i = ic / a.C, c = ic - i * a.C;
  const int b = inl.n ? inl.branch[i] : a.branch[i];
  const int m = inl.n ? inl.model[i] : (a.model ? a.model[i] : 0);
  const double rc = a.rates[c];
  const double tt = (inl.n ? inl.t[i] : a.t[i]) * rc;
  const double* V = a.V + (size_t)m * S * S;
  const double* Vi = a.Vinv + (size_t)m * S * S;
  const double* lam = a.lambda + (size_t)m * S;
  double e[S], l[S], vx[S], vi[S * S];
#pragma unroll
  for (int k = 0; k < S; ++k) {
    l[k] = lam[k];
    vx[k] = V[x * S + k];
  }
#pragma unroll
  for (int k = 0; k < S * S; ++k) vi[k] = Vi[k];
#pragma unroll
  for (int k = 0; k < S; ++k) e[k] = exp(l[k] * tt);
  double p[S], dp[S], d2p[S];
#pragma unroll
  for (int y = 0; y < S; ++y) {
    p[y] = 0.0;
    dp[y] = 0.0;
    d2p[y] = 0.0;
#pragma unroll
    for (int k = 0; k < S; ++k) {
      const double w = vx[k] * vi[k * S + y];
      p[y] = __builtin_fma(w, e[k], p[y]);
      if (a.mask & 6u) {
        const double le = l[k] * e[k];
        dp[y] = __builtin_fma(w, le, dp[y]);
        d2p[y] = __builtin_fma(w, l[k] * le, d2p[y]);
      }
    }
    if (tt == 0.0) p[y] = (x == y) ? 1.0 : 0.0;  // getPij_t: t == 0 -> identity (:428-431)
  }
  const size_t off = ((size_t)b * a.C + c) * S * S + x * S;
#pragma unroll
  for (int y = 0; y < S; ++y) {
    if (a.mask & 1u) a.P[off + y] = p[y];
    if (a.mask & 2u) a.dP[off + y] = rc * dp[y];
    if (a.mask & 4u) a.d2P[off + y] = rc * rc * d2p[y];
  }
  // tip branch: entries x of its table rows, tipP[b][c][code][x] = sum_y P[x][y] init[code][y]
  if (a.init && b < a.n_tips && (a.mask & 1u)) {
    double* out = a.tipP + ((size_t)b * a.C + c) * a.n_codes * S + x;
    for (int code = 0; code < a.n_codes; ++code) {
      double t = 0.0;
#pragma unroll
      for (int y = 0; y < S; ++y) t = __builtin_fma(p[y], a.init[code * S + y], t);
      out[code * S] = t;
    }
  }
}

// K4 for 64 states (codon models), P only: the same sums as pmat_kernel in the same order
// (k ascending, w = V[x][k] Vinv[k][y], fma(w, e_k, p)), so bitwise its results, but with
// V, Vinv and e staged in LDS and a register block of outputs per thread (independent FMA
// chains over LDS reads instead of one chain over two reads, one of them from L2), split
// over four 16-row slabs of P (blockIdx.z): 4x the workgroups, so a tree's few hundred
// branches fill the device several deep instead of one workgroup per CU.
__global__ __launch_bounds__(256) void pmat64s_kernel(PmatArgs a, const PmatInline inl) {
  constexpr int S = 64, R = 16;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int i = blockIdx.x, c = blockIdx.y, x0 = R * blockIdx.z;
  const int b = inl.n ? inl.branch[i] : a.branch[i];
  const int m = inl.n ? inl.model[i] : (a.model ? a.model[i] : 0);
  const double tt = (inl.n ? inl.t[i] : a.t[i]) * a.rates[c];
  double* e = sm;
  double* Vm = sm + S;      // rows x0 .. x0 + R - 1 of V
  double* Vi = Vm + R * S;  // all of Vinv
  const double* V = a.V + (size_t)m * S * S;
  const double* VI = a.Vinv + (size_t)m * S * S;
  const double* lam = a.lambda + (size_t)m * S;
  for (int k = threadIdx.x; k < S; k += blockDim.x) e[k] = exp(lam[k] * tt);
  stage_lds<R * S / 256>(Vm, V + x0 * S, R * S);
  stage_lds<S * S / 256>(Vi, VI, S * S);
  __syncthreads();
  const int xr = threadIdx.x >> 4, yb = threadIdx.x & 15;
  double p[4] = {0.0, 0.0, 0.0, 0.0};
  for (int k = 0; k < S; ++k) {
    const double ek = e[k];
    const double vx = Vm[xr * S + k];
    double vy[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) vy[v] = Vi[k * S + yb + 16 * v];
#pragma unroll
    for (int v = 0; v < 4; ++v) p[v] = __builtin_fma(vx * vy[v], ek, p[v]);
  }
  double* out = a.P + ((size_t)b * a.C + c) * S * S;
  const int x = x0 + xr;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int y = yb + 16 * v;
    p[v] = tt == 0.0 ? (x == y ? 1.0 : 0.0) : p[v];  // getPij_t: t == 0 -> identity
    out[x * S + y] = p[v];
  }
  // the transposed copy the 64-state matrix-core kernels read (transpose_pmats' layout),
  // written here so that an evaluation needs no transpose launch
  if (a.PT) {
    double* outT = a.PT + ((size_t)b * a.C + c) * S * S;
#pragma unroll
    for (int v = 0; v < 4; ++v) outT[(yb + 16 * v) * S + x] = p[v];
  }
  if (a.init && b < a.n_tips) {
    __syncthreads();  // done with Vm / Vi
    double* Pl = Vm;  // [R][y]
    double* In = Vi;  // [code][y], n_codes <= 64 (launch guarantees)
#pragma unroll
    for (int v = 0; v < 4; ++v) Pl[xr * S + yb + 16 * v] = p[v];
    stage_lds<S * S / 256>(In, a.init, a.n_codes * S);
    __syncthreads();
    double* tout = a.tipP + ((size_t)b * a.C + c) * a.n_codes * S;
    const int xl = threadIdx.x & 15, cb = 4 * (threadIdx.x >> 4);
    double t[4] = {0.0, 0.0, 0.0, 0.0};
    for (int y = 0; y < S; ++y) {
      const double px = Pl[xl * S + y];
#pragma unroll
      for (int u = 0; u < 4; ++u) t[u] = __builtin_fma(px, cb + u < a.n_codes ? In[(cb + u) * S + y] : 0.0, t[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (cb + u < a.n_codes) tout[(cb + u) * S + x0 + xl] = t[u];
  }
}

// K4 for 64 states, several matrices per workgroup, one P row per wave register: lane y of
// a wave holds P[x][y] of its rows x.  w = V[x][k] Vinv[k][y] does not depend on the branch
// length or the rate class, so the NB matrices of a workgroup (request entry i, class c, in
// i-major order) that share a model share every w: per (x, y, k) one multiply and NB FMAs.
// Per k a lane reads Vinv[k][y] from LDS (consecutive, no conflicts); V[x][k] and
// e_q[k] = exp(lambda_k r_c t_i) come by v_readlane from lane k of a register.  The sums
// are pmat_kernel's in its order (k ascending, fma(w, e_k, p)), so the results are bitwise
// pmat64s_kernel's.  A workgroup covers rows x0 .. x0 + 4 RX - 1 (blockIdx.y, RX per wave);
// its matrices form runs of one model (a non-homogeneous request can change model inside the
// group), each staged and computed in turn; a request of one model (a.uni_model >= 0, known
// to the host) stages Vinv while the request entries -- in pinned host memory for requests
// over kPmatInline branches, a bus round trip -- are on their way.  cfg4 (254 branches):
// 31 us against pmat64s_kernel's 36-37; in-kernel stamps put ~4.7 us in the prologue
// (request, staging), ~6 us in the k loop and ~10 us in the P / P^T stores
// (profiles/r05/ab_runs.md).
constexpr int kP64Pad = 65;
__device__ __forceinline__ double readlane_f64(double v, int k) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, k), hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int RX, int NB>
__global__ __launch_bounds__(256) void pmat64w_kernel(PmatArgs a, const PmatInline inl) {
  constexpr int S = 64, R = 4 * RX;
  static_assert(NB * S <= 256 && R <= 64, "NB exponential rows over 256 threads; R rows");
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* Vi = sm;               // [S][S] Vinv; tip phase: the code table [code][kP64Pad]
  double* e = Vi + S * kP64Pad;  // [NB][S]
  double* Pl = e + NB * S;       // [NB][R][kP64Pad]: the workgroup's P rows
  __shared__ int s_b[NB], s_m[NB];
  __shared__ double s_t[NB];
  const int n_mat = a.n_req * a.C;
  const int j0 = blockIdx.x * NB, jn = min(n_mat, j0 + NB), x0 = R * blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63;
  const int xw = x0 + RX * __builtin_amdgcn_readfirstlane(tid >> 6);  // the wave's first row
  if (tid < NB && j0 + tid < jn) {
    const int j = j0 + tid, i = j / a.C;
    s_b[tid] = inl.n ? inl.branch[i] : a.branch[i];
    s_m[tid] = inl.n ? inl.model[i] : (a.model ? a.model[i] : 0);
    s_t[tid] = (inl.n ? inl.t[i] : a.t[i]) * a.rates[j - i * a.C];
  }
  int staged = -1;
  if (a.uni_model >= 0) {
    stage_lds<S * S / 256>(Vi, a.Vinv + (size_t)a.uni_model * S * S, S * S);
    staged = a.uni_model;
  }
  __syncthreads();
  for (int r0 = j0; r0 < jn;) {
    const int m = __builtin_amdgcn_readfirstlane(s_m[r0 - j0]);
    int r1 = r0 + 1;
    while (r1 < jn && s_m[r1 - j0] == m) ++r1;
    if (staged != m) {
      if (staged >= 0) __syncthreads();  // the previous run is done with Vi
      stage_lds<S * S / 256>(Vi, a.Vinv + (size_t)m * S * S, S * S);
      staged = m;
    }
    const double* lam = a.lambda + (size_t)m * S;
    if (tid < NB * S) {
      const int q = tid / S;
      e[tid] = r0 + q < r1 ? exp(lam[tid % S] * s_t[r0 + q - j0]) : 0.0;
    }
    __syncthreads();
    double ek[NB], vxl[RX];
#pragma unroll
    for (int q = 0; q < NB; ++q) ek[q] = e[q * S + lane];  // lane k holds e_q[k]
#pragma unroll
    for (int r = 0; r < RX; ++r) vxl[r] = a.V[((size_t)m * S + xw + r) * S + lane];  // lane k holds V[x][k]
    double p[RX][NB];
#pragma unroll
    for (int r = 0; r < RX; ++r)
#pragma unroll
      for (int q = 0; q < NB; ++q) p[r][q] = 0.0;
#pragma unroll 4
    for (int k = 0; k < S; ++k) {
      const double vi = Vi[k * S + lane];
      double w[RX];
#pragma unroll
      for (int r = 0; r < RX; ++r) w[r] = readlane_f64(vxl[r], k) * vi;
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const double eq = readlane_f64(ek[q], k);
#pragma unroll
        for (int r = 0; r < RX; ++r) p[r][q] = __builtin_fma(w[r], eq, p[r][q]);
      }
    }
    // P rows straight from the registers (lane y: 512-byte rows); the workgroup's rows of
    // every matrix also go to LDS, from where P^T leaves as whole 128-byte lines of R
    // consecutive x per y (a store of column y from the registers scatters 64 lanes over
    // 64 lines -- 16 K such stores per cfg4 request ran ~20 us)
    bool any_tip = false;
#pragma unroll
    for (int q = 0; q < NB; ++q) {
      const int j = r0 + q;
      if (j >= r1) break;
      const int b = s_b[j - j0], c = j % a.C;
      const bool ident = s_t[j - j0] == 0.0;  // getPij_t: t == 0 -> identity
      double* out = a.P + ((size_t)b * a.C + c) * S * S;
#pragma unroll
      for (int r = 0; r < RX; ++r) {
        const int x = xw + r;
        p[r][q] = ident ? (x == lane ? 1.0 : 0.0) : p[r][q];
        out[x * S + lane] = p[r][q];
        Pl[(q * R + xw - x0 + r) * kP64Pad + lane] = p[r][q];
      }
      any_tip |= a.init && b < a.n_tips;
    }
    __syncthreads();
    if (a.PT) {
      const int y = tid >> 2, xq = (tid & 3) * RX;  // 4 threads per y, RX consecutive x each
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const int j = r0 + q;
        if (j >= r1) break;
        const int b = s_b[j - j0], c = j % a.C;
        double* outT = a.PT + ((size_t)b * a.C + c) * S * S + (size_t)y * S + x0 + xq;
#pragma unroll
        for (int u = 0; u < RX; ++u) outT[u] = Pl[(q * R + xq + u) * kP64Pad + y];
      }
    }
    if (any_tip) {
      // tip rows tipP[b][c][code][x0 + xl] = sum_y P[x][y] init[code][y] (tip_table64_kernel's
      // sums, y ascending) from the P rows in LDS
      constexpr int NC = R / 4;  // codes per thread
      const int xl = tid % R, cb = NC * (tid / R);
      for (int k = tid; k < a.n_codes * S; k += 256) Vi[(k / S) * kP64Pad + k % S] = a.init[k];
      staged = -1;
      __syncthreads();
#pragma unroll
      for (int q = 0; q < NB; ++q) {
        const int j = r0 + q;
        if (j >= r1) break;
        const int b = s_b[j - j0], c = j % a.C;
        if (b >= a.n_tips) continue;
        double t[NC];
#pragma unroll
        for (int u = 0; u < NC; ++u) t[u] = 0.0;
#pragma unroll 4
        for (int y = 0; y < S; ++y) {
          const double px = Pl[(q * R + xl) * kP64Pad + y];
#pragma unroll
          for (int u = 0; u < NC; ++u)
            t[u] = __builtin_fma(px, cb + u < a.n_codes ? Vi[(cb + u) * kP64Pad + y] : 0.0, t[u]);
        }
        double* tout = a.tipP + ((size_t)b * a.C + c) * a.n_codes * S;
#pragma unroll
        for (int u = 0; u < NC; ++u)
          if (cb + u < a.n_codes) tout[(cb + u) * S + x0 + xl] = t[u];
      }
    }
    r0 = r1;
    if (r0 < jn) __syncthreads();  // the next run rewrites e
  }
}

// tip tables for 64 states: tip_table_kernel's sums (y ascending) with P and the code
// table staged in LDS and 4 codes x 4 states per thread
__global__ __launch_bounds__(256) void tip_table64_kernel(const double* __restrict__ P, const double* __restrict__ init,
                                                          double* __restrict__ tipP, int n_tips, int C,
                                                          int n_codes) {
  constexpr int S = 64;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int tip = blockIdx.x, c = blockIdx.y;
  double* Pl = sm;           // [x][y]
  double* In = sm + S * S;   // [code][y]
  const double* Pc = P + ((size_t)tip * C + c) * S * S;
  stage_lds<S * S / 256>(Pl, Pc, S * S);
  stage_lds<S * S / 256>(In, init, n_codes * S);
  __syncthreads();
  double* out = tipP + ((size_t)tip * C + c) * n_codes * S;
  const int xb = 4 * (threadIdx.x & 15);
  for (int cb = 4 * (threadIdx.x >> 4); cb < n_codes; cb += 64) {
    double t[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int v = 0; v < 4; ++v) t[u][v] = 0.0;
    for (int y = 0; y < S; ++y) {
      double px[4], iv[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) px[v] = Pl[(xb + v) * S + y];
#pragma unroll
      for (int u = 0; u < 4; ++u) iv[u] = cb + u < n_codes ? In[(cb + u) * S + y] : 0.0;
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) t[u][v] = __builtin_fma(px[v], iv[u], t[u][v]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (cb + u < n_codes)
#pragma unroll
        for (int v = 0; v < 4; ++v) out[(cb + u) * S + xb + v] = t[u][v];
  }
}

// tipP[tip][c][code][x] = sum_y P[tip][c][x][y] * init[code][y]
__global__ __launch_bounds__(256) void tip_table_kernel(const double* __restrict__ P, const double* __restrict__ init,
                                                        double* __restrict__ tipP, int n_tips, int C, int S,
                                                        int n_codes) {
  const int tip = blockIdx.x, c = blockIdx.y;
  if (tip >= n_tips) return;
  const double* Pc = P + ((size_t)tip * C + c) * S * S;
  double* out = tipP + ((size_t)tip * C + c) * n_codes * S;
  for (int idx = threadIdx.x; idx < n_codes * S; idx += blockDim.x) {
    const int code = idx / S, x = idx % S;
    double s = 0.0;
    for (int y = 0; y < S; ++y) s = __builtin_fma(Pc[x * S + y], init[code * S + y], s);
    out[idx] = s;
  }
}

// Code rows of the tree-specialised kernel's table units (plk_jit.hpp: JitUnit): unit u
// reads codes[ta] (tb < 0) or the combined code codes[ta] * U + codes[tb] of a cherry's
// product table.  Rebuilt when tip codes or the unit list change, not per evaluation.
// Bytes are combined four to a word: a byte times U plus a byte < U stays below 256.
// units[k] = (ta, tb, tc, td): a tip (tb < 0), a cherry (ca U + cb) or a quad
// (((ca U + cb) U + cc) U + cd, plk_jit.hpp JitUnit); 4 codes per 32-bit word, bytes stay < 256
// Position of row r (combined code ((ca 4 + cb) 4 + cc) 4 + cd) in a quad table of 256 rows:
// each 16-row block is rotated by 7 (ca + cb), so that the 16-byte half-rows that one
// ds_read_b128 lane group gathers land on distinct bank slots more often -- sibling tips tend to
// share a code, which the plain order (slot = 4 cc + cd) maps onto 4 of the 16 slots (cfg2's
// data: 2.29 -> 1.47 LDS cycles per 16-lane group, tools/lds_conflict_sim.py).  The generated
// kernel's quad build places rows the same way (plk_jit.hpp QROW_).
__host__ __device__ inline int quad_row(int r) {
  return (r & ~15) | ((r + 7 * ((r >> 6) & 3) + 7 * ((r >> 4) & 3)) & 15);
}

__global__ __launch_bounds__(256) void unit_codes_kernel(const uint8_t* __restrict__ codes, int64_t n_pad,
                                                         const int4* __restrict__ units, int U,
                                                         uint8_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // uint4 index in the row
  if (i * 16 >= n_pad) return;
  const int4 u = units[blockIdx.y];
  uint4 v = reinterpret_cast<const uint4*>(codes + (int64_t)u.x * n_pad)[i];
  const int more[3] = {u.y, u.z, u.w};
  for (int k = 0; k < 3; ++k) {
    if (more[k] < 0) break;
    const uint4 b = reinterpret_cast<const uint4*>(codes + (int64_t)more[k] * n_pad)[i];
    v.x = v.x * U + b.x;
    v.y = v.y * U + b.y;
    v.z = v.z * U + b.z;
    v.w = v.w * U + b.w;
  }
  if (u.w >= 0 && U == 4) {
    // quad rows are placed by quad_row (one class per workgroup's tables), so the code is the
    // row's position
    unsigned* wv = &v.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      unsigned o = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) o |= (unsigned)quad_row((int)((wv[j] >> (8 * b)) & 255u)) << (8 * b);
      wv[j] = o;
    }
  }
  reinterpret_cast<uint4*>(out + (int64_t)blockIdx.y * n_pad)[i] = v;
}

// ---------------------------------------------------------------------------
// K5: root reduction.  Per pattern p: l_c = sum_s L[c][s] pi_s, l = sum_c l_c w_c
// with the reference's "<= 0 terms dropped" guards (HOMOG) or NH clamp;
// lnl_p = log(l) - nscale * 256 ln 2.  One wave per 64 patterns (a grid of n_pad/64
// single-wave blocks fills the chip even at 50k patterns); each wave sums w_p * lnl_p
// with the same fixed butterfly as the fused traversal's root (plk_tree4.hpp), and
// wave_sums_to_blocks then forms the fixed-order 4096-pattern block sums, so both
// paths give bit-identical lnL from bit-identical root partials.
// ---------------------------------------------------------------------------
struct RootArgs {
  const double* partials;  // root slot base
  const int32_t* scale;    // root scale row or null
  const double* weights;   // [n_pad]
  const double* pi;        // [S]
  const double* probs;     // [C]
  double* site_lnl;        // [n_pad]
  double* wave_sums;       // [n_pad / 64]
  int64_t n_patterns;
  int S, C;
  int guard;               // 1: homogeneous guards, 0: NH clamp
  int32_t* uflow;          // unscaled handles: set to 1 when a site likelihood is < 2^-255 (or null)
};

// Direct-code layout of the generated 4-state kernel (plk_jit.hpp JitShape::dc): fragment f's
// unit codes of pattern p as dw 16-byte words, byte k = unit k (at most 16 dw units), from the
// per-unit rows of unit_codes_kernel.  units_start: CSR of the fragments' units (n_frag + 1 entries).
__global__ __launch_bounds__(256) void unit_codes_dc_kernel(const uint8_t* __restrict__ rows, int64_t n_pad,
                                                            const int32_t* __restrict__ units_start, int dw,
                                                            uint4* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pad) return;
  const int f = blockIdx.y, u0 = units_start[f], nu = units_start[f + 1] - u0;
  unsigned w[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  for (int k = 0; k < nu && k < 16 * dw && k < 32; ++k)
    w[k >> 2] |= (unsigned)rows[(int64_t)(u0 + k) * n_pad + p] << (8 * (k & 3));
  for (int j = 0; j < dw && j < 2; ++j)
    out[((int64_t)f * n_pad + p) * dw + j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
}

// The root reduction of a traversal run with one class per workgroup (plk_jit.hpp, JitShape::cls):
// cls_sum[c][p] holds each class's term t_c = l_c prob_c (the per-state guards applied); the
// classes are added in class order with the class-level guard or the NH clamp, then log, the
// underflow flag, site lnL, the 64-pattern wave sums (the same butterfly) and the 4096-pattern
// block sum (the same chain of adds as wave_sums_to_blocks) -- reduce_root's and
// wave_sums_to_blocks' operations in their order, so the block sums are bitwise those of the
// classes-in-one-workgroup kernel.  One workgroup of 16 waves per block, each wave four of its
// 64-pattern waves with every load issued before the first log (one memory round trip).
// (C a template parameter: every class's load of every pattern issued before the first add --
// with a runtime class loop each wave waited for one load at a time, 15.5 us at 1M patterns)
template <int C>
__global__ __launch_bounds__(1024) void cls_blocks_kernel(const double* __restrict__ cls_sum, int64_t n_pad,
                                                          const double* __restrict__ weights,
                                                          double* __restrict__ site_lnl, double* __restrict__ block_sums,
                                                          int64_t n_patterns, int n_waves, int guard, int32_t* uflow) {
  constexpr int kW = kRootBlock / 64;  // 64-pattern waves per block
  constexpr int kPer = kW / 16;        // per hardware wave
  __shared__ double ws[kW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int b = blockIdx.x;
  double l[kPer], wt[kPer], t[kPer][C];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t p = ((int64_t)b * kW + wv + 16 * j) * 64 + lane;
    const int64_t pc = p < n_pad ? p : 0;
#pragma unroll
    for (int c = 0; c < C; ++c) t[j][c] = cls_sum[(int64_t)c * n_pad + pc];
    wt[j] = p < n_patterns ? weights[p] : 0.0;
  }
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    l[j] = 0.0;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const double li = t[j][c];
      if (guard) {
        if (li > 0.0) l[j] += li;
      } else {
        l[j] += li;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int k = wv + 16 * j;
    const int64_t p0 = ((int64_t)b * kW + k) * 64, p = p0 + lane;
    double wr = 0.0;
    if (p0 < n_pad) {
      double lj = l[j];
      if (!guard && lj < 0.0) lj = 0.0;
      const double r = log(lj);
      if (p < n_patterns) {
        if (uflow && !(lj >= 2.0 * kScaleThr)) *uflow = 1;  // plk_root_underflow
        if (site_lnl) site_lnl[p] = r;
        wr = wt[j] * r;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) wr += __shfl_xor(wr, off, 64);
    }
    if (lane == 0) ws[k] = wr;
  }
  __syncthreads();
  if (wv == 0) {
    // the chain of adds in wave order, its operands read from LDS (broadcast reads, issued ahead
    // of the adds; a shuffle per operand put a cross-lane round trip before every add)
    double x[kW];
#pragma unroll
    for (int k = 0; k < kW; ++k) x[k] = ws[k];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kW; ++k)
      if (b * kW + k < n_waves) s += x[k];
    if (lane == 0) block_sums[b] = s;
  }
}

// Under a communicator: the underflow flag into this rank's exchange record once every block of
// cls_blocks_kernel has set it (plk_exchange.hpp layout; wave_sums_to_blocks does this itself).
__global__ void flag_slot_kernel(const int32_t* uflow, double* __restrict__ slot) {
  *slot = __hip_atomic_load(uflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ? 1.0 : 0.0;
}

__global__ __launch_bounds__(64) void root_kernel(RootArgs a) {
  const int lane = threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.x * 64;
  const int64_t p = p0 + lane;
  const int64_t tile = p / kTile, q = p % kTile;
  const double* L = a.partials + tile * ((int64_t)a.C * a.S * kTile) + q;
  double l = 0.0;
  for (int c = 0; c < a.C; ++c) {
    double lc = 0.0;
    for (int s = 0; s < a.S; ++s) {
      const double li = L[(int64_t)(c * a.S + s) * kTile] * a.pi[s];
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
  if (a.scale) r -= (double)a.scale[p] * kLn2x256;
  double wr = 0.0;
  if (p < a.n_patterns) {
    if (a.uflow && !(l >= 2.0 * kScaleThr)) *a.uflow = 1;  // plk_root_underflow
    a.site_lnl[p] = r;
    wr = a.weights[p] * r;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) wr += __shfl_xor(wr, off, 64);
  if (lane == 0) a.wave_sums[p0 >> 6] = wr;
}

}  // namespace plk
