// plk_dr.hpp -- double-recursive (DR) branch derivatives: every branch of the tree
// from one preorder pass (row f4 of SURVEY 8(f)).
//
// The reference's DRHomogeneousTreeLikelihood keeps, for every node, the likelihood
// arrays of each neighbour direction (computeSubtreeLikelihoodPostfix / Prefix,
// Likelihood/DRHomogeneousTreeLikelihood.cpp:483-651) and forms the derivative of a
// branch from the two arrays on either side of it (computeTreeDLikelihoodAtNode
// :287-328, computeTreeD2LikelihoodAtNode :373-413).  Here the father-side array of
// branch v is the "upper" vector
//     U_v[c][y] = (M_f U_f)[c][y] * prod_{siblings s of v} (P_s L_s)[c][y]
// at v's father f (y = state at f), with M_f = P_f^T for an ordinary father and
// M_f = P_f^T diag(pi) for a child of the root (whose own upper vector leaves pi out;
// pi enters the branch reduction instead).  U_v is produced by the ordinary partial
// kernels (plk_kernels.hpp et al.): it is a product of children, U_f being a child
// whose "transition matrix" is M_f -- so the preorder pass reuses the levelwise S=4,
// S=20 (SGPR) and S=64 (MFMA) paths as they are, rescaling included.
//
// 4 states without rescaling take the fused form instead (dr_pre_s4_kernel below): the
// father-side vectors stay in registers within a father's op and the branch terms are
// reduced where they are formed.
//
// Per branch and pattern the reduction below forms
//     l = sum_c p_c sum_y u[c][y] (P_v L_v)[c][y],   u = U_v (x pi at the root's children)
// and l', l'' with r_c dP_v and r_c^2 d2P_v in place of P_v (lnL is linear in P_v), then
// d1 += w l'/l and d2 += w (l''/l - (l'/l)^2).  Power-of-two scale counts of U_v and
// L_v multiply l, l', l'' alike, so the ratios need no scale bookkeeping.
#pragma once

#include "plk_kernels.hpp"
#include "plk_treeM.hpp"

namespace plk {

// M_f of one father f and class c: dst[f][c][y][w] = P_f[c][w][y] * (use_pi ? pi_w : 1),
// and its transpose (the P^T copy the MFMA kernels read) when dstT is given.
__global__ __launch_bounds__(256) void dr_matrix_kernel(const double* __restrict__ pmats, double* __restrict__ dst,
                                                        double* __restrict__ dstT, const double* __restrict__ pi,
                                                        const int2* __restrict__ list, int dst_base, int C, int S) {
  const int2 e = list[blockIdx.x];
  const int c = blockIdx.y;
  const int SS = S * S;
  const double* P = pmats + ((size_t)e.x * C + c) * SS;
  const size_t o = ((size_t)(dst_base + e.x) * C + c) * SS;
  for (int i = threadIdx.x; i < SS; i += blockDim.x) {
    const int y = i / S, w = i - y * S;
    const double v = e.y ? P[w * S + y] * pi[w] : P[w * S + y];
    dst[o + i] = v;
    if (dstT) dstT[o + (size_t)w * S + y] = v;
  }
}

struct DrBranch {
  int32_t node;    // branch = child node index (P, dP, d2P index)
  int32_t is_tip;  // L_v from the tip's codes
  int32_t child;   // tip index or internal slot of v
  int32_t uslot;   // slot of U_v
  int32_t use_pi;  // v is a child of the root
  // fuse = 1 (a tip whose father f has exactly one other son s and a father of its own):
  // U_v = (M_f U_f) (*) (P_s L_s) is formed here instead of being written by the preorder
  // pass and read back -- the upper vectors of such tips are never stored
  int32_t fuse;
  int32_t uf_slot;     // slot of U_f
  int32_t mf;          // matrix index of M_f
  int32_t sib_tip;     // s is a tip (row of its tip table) or internal (P_s L_s)
  int32_t sib;         // tip index or internal slot of s
  int32_t sib_branch;  // node index of s (its P)
  int32_t pad_;
};

struct DrArgs {
  const double* partials;
  const uint8_t* codes;       // compact codes [tip][n_pad]
  const double* code_table;   // compact table [n_codes][S]
  const double* pmats;
  const double* dpmats;
  const double* d2pmats;
  const double* pi;
  const double* probs;
  const double* weights;
  const double* tipP;         // [n_tips][C][n_codes][S] (fused tips' siblings)
  double* blk1;               // [branch][n_blk] block sums of w l'/l
  double* blk2;               // [branch][n_blk] block sums of w (l''/l - (l'/l)^2)
  double* uout;               // partial slots receiving U (fused preorder)
  int64_t slot_stride;
  int64_t n_pad;
  int64_t n_patterns;
  int32_t C;
  int32_t n_blk;
  int32_t G;                  // classes staged in LDS at a time
  int32_t n_codes;
};

constexpr int kDrThreads = 256;

// One workgroup = 256 patterns of one branch.  P_v, dP_v, d2P_v of G classes are
// staged in LDS (3 G S^2 doubles, read as wave-wide broadcasts); L_v of the lane's
// pattern sits in registers; U_v is read once per (class, state), coalesced.
template <int S>
__global__ __launch_bounds__(kDrThreads) void dr_branch_kernel(const DrBranch* __restrict__ branches, DrArgs a) {
  extern __shared__ double lds[];
  __shared__ double red[2][kDrThreads / 64];
  const DrBranch b = branches[blockIdx.y];
  const int64_t p = (int64_t)blockIdx.x * kDrThreads + threadIdx.x;
  const bool live = p < a.n_patterns;
  const int64_t tile = p >> 7, q = p & (kTile - 1);
  const int CS = a.C * S;
  double l0 = 0.0, l1 = 0.0, l2 = 0.0;
  // classes staged G at a time (G = C when 3 C S^2 doubles fit the LDS budget of the
  // launch, else 1): no barrier inside a group
  for (int c0 = 0; c0 < a.C; c0 += a.G) {
    const int g = min(a.G, a.C - c0);
    const int SS = S * S;
    __syncthreads();
    for (int i = threadIdx.x; i < g * SS; i += kDrThreads) {
      const size_t mo = ((size_t)b.node * a.C + c0) * SS + i;
      lds[i] = a.pmats[mo];
      lds[g * SS + i] = a.dpmats[mo];
      lds[2 * g * SS + i] = a.d2pmats[mo];
    }
    __syncthreads();
    if (live) {
      for (int cc = 0; cc < g; ++cc) {
        const int c = c0 + cc;
        const double* sP = lds + cc * SS;
        const double* sD = lds + (g + cc) * SS;
        const double* sD2 = lds + (2 * g + cc) * SS;
        double L[S];
        if (b.is_tip) {
          const double* row = a.code_table + (size_t)a.codes[(size_t)b.child * a.n_pad + p] * S;
#pragma unroll
          for (int z = 0; z < S; ++z) L[z] = row[z];
        } else {
          const double* src = a.partials + (size_t)b.child * a.slot_stride + ((size_t)tile * CS + c * S) * kTile + q;
#pragma unroll
          for (int z = 0; z < S; ++z) L[z] = src[(size_t)z * kTile];
        }
        double s0 = 0.0, s1 = 0.0, s2 = 0.0;
        if constexpr (S <= 4) {
        double uu[S];
        if (b.fuse) {
          const size_t co = ((size_t)tile * CS + c * S) * kTile + q;
          const double* Uf = a.partials + (size_t)b.uf_slot * a.slot_stride + co;
          const double* Mf = a.pmats + ((size_t)b.mf * a.C + c) * S * S;
          double uf[S], sv[S];
#pragma unroll
          for (int w = 0; w < S; ++w) uf[w] = Uf[(size_t)w * kTile];
          if (b.sib_tip) {
            const double* row =
                a.tipP + (((size_t)b.sib * a.C + c) * a.n_codes + a.codes[(size_t)b.sib * a.n_pad + p]) * S;
#pragma unroll
            for (int y = 0; y < S; ++y) sv[y] = row[y];
          } else {
            const double* Ls = a.partials + (size_t)b.sib * a.slot_stride + co;
            const double* Ps = a.pmats + ((size_t)b.sib_branch * a.C + c) * S * S;
            double ls[S];
#pragma unroll
            for (int z = 0; z < S; ++z) ls[z] = Ls[(size_t)z * kTile];
#pragma unroll
            for (int y = 0; y < S; ++y) {
              double t = 0.0;
#pragma unroll
              for (int z = 0; z < S; ++z) t = fma(Ps[y * S + z], ls[z], t);
              sv[y] = t;
            }
          }
#pragma unroll
          for (int y = 0; y < S; ++y) {
            double t = 0.0;
#pragma unroll
            for (int w = 0; w < S; ++w) t = fma(Mf[y * S + w], uf[w], t);
            uu[y] = t * sv[y];
          }
        } else {
          const double* U = a.partials + (size_t)b.uslot * a.slot_stride + ((size_t)tile * CS + c * S) * kTile + q;
#pragma unroll
          for (int y = 0; y < S; ++y) uu[y] = b.use_pi ? U[(size_t)y * kTile] * a.pi[y] : U[(size_t)y * kTile];
        }
#pragma unroll
        for (int y = 0; y < S; ++y) {
          double t0 = 0.0, t1 = 0.0, t2 = 0.0;
#pragma unroll
          for (int z = 0; z < S; ++z) {
            t0 = fma(sP[y * S + z], L[z], t0);
            t1 = fma(sD[y * S + z], L[z], t1);
            t2 = fma(sD2[y * S + z], L[z], t2);
          }
          const double u = uu[y];
          s0 = fma(u, t0, s0);
          s1 = fma(u, t1, s1);
          s2 = fma(u, t2, s2);
        }
        } else {
        const double* U = a.partials + (size_t)b.uslot * a.slot_stride + ((size_t)tile * CS + c * S) * kTile + q;
        for (int y = 0; y < S; ++y) {
          double t0 = 0.0, t1 = 0.0, t2 = 0.0;
#pragma unroll
          for (int z = 0; z < S; ++z) {
            t0 = fma(sP[y * S + z], L[z], t0);
            t1 = fma(sD[y * S + z], L[z], t1);
            t2 = fma(sD2[y * S + z], L[z], t2);
          }
          const double u = b.use_pi ? U[(size_t)y * kTile] * a.pi[y] : U[(size_t)y * kTile];
          s0 = fma(u, t0, s0);
          s1 = fma(u, t1, s1);
          s2 = fma(u, t2, s2);
        }
        }
        l0 = fma(a.probs[c], s0, l0);
        l1 = fma(a.probs[c], s1, l1);
        l2 = fma(a.probs[c], s2, l2);
      }
    }
  }
  double r1 = 0.0, r2 = 0.0;
  if (live) {
    const double g = l1 / l0, hh = l2 / l0;
    r1 = a.weights[p] * g;
    r2 = a.weights[p] * (hh - g * g);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    r1 += __shfl_xor(r1, off, 64);
    r2 += __shfl_xor(r2, off, 64);
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wv] = r1;
    red[1][wv] = r2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t1 = 0.0, t2 = 0.0;
    for (int k = 0; k < kDrThreads / 64; ++k) {  // fixed order
      t1 += red[0][k];
      t2 += red[1][k];
    }
    a.blk1[(size_t)blockIdx.y * a.n_blk + blockIdx.x] = t1;
    a.blk2[(size_t)blockIdx.y * a.n_blk + blockIdx.x] = t2;
  }
}

// S = 20 / 64: the same reduction on fp64 matrix cores.  A wave owns 16 patterns; L_v of
// the wave's patterns is the B operand of v_mfma_f64_16x16x4f64 in treeM's C/D layout
// (plk_treeM.hpp: lane l holds states 16 xt + (l >> 4) + 4 r of pattern l & 15), and
// (P_v L_v), (dP_v L_v), (d2P_v L_v) come out of matvec_m in that same layout, so the
// dot with U_v is lane-local plus two cross-lane adds.  P^T, dP^T, d2P^T of one class are
// staged transposed in LDS (3 S^2 doubles).  Block sums cover 64 patterns.
constexpr int kDrmThreads = 256;

template <int S>
__global__ __launch_bounds__(kDrmThreads) void dr_branch_mfma_kernel(const DrBranch* __restrict__ branches, DrArgs a) {
  constexpr int XT = MShape<S>::XT;
  extern __shared__ double lds[];
  __shared__ double red[2][kDrmThreads / 64];
  const DrBranch b = branches[blockIdx.y];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int lr = lane >> 4, lc = lane & 15;
  // persistent over the branch's 64-pattern blocks: the matrices are staged once per
  // workgroup (not once per block) when all classes fit
  bool staged = false;
  for (int64_t blk = blockIdx.x; blk < a.n_blk; blk += gridDim.x) {
  const int64_t p = blk * 64 + 16 * g + lc;
  const bool live = p < a.n_patterns;
  const int64_t tile = p >> 7, q = p & (kTile - 1);
  const int CS = a.C * S;
  double l0 = 0.0, l1 = 0.0, l2 = 0.0;
  // classes staged G at a time (all of them when 3 C S^2 doubles fit the launch's LDS)
  for (int c = 0; c < a.C; ++c) {
    const int cc = c % a.G;
    if (cc == 0 && !(staged && a.G == a.C)) {
      const int g = min(a.G, a.C - c);
      staged = true;
      __syncthreads();
      for (int i = threadIdx.x; i < g * S * S; i += kDrmThreads) {
        const int k = i / (S * S), e = i - k * S * S;
        const int x = e / S, y = e - x * S;  // source [x][y] -> LDS [y][x]
        const size_t mo = ((size_t)b.node * a.C + c + k) * S * S + e;
        lds[(3 * k) * S * S + y * S + x] = a.pmats[mo];
        lds[(3 * k + 1) * S * S + y * S + x] = a.dpmats[mo];
        lds[(3 * k + 2) * S * S + y * S + x] = a.d2pmats[mo];
      }
      __syncthreads();
    }
    const double* sP = lds + (3 * cc) * S * S;
    const double* sD = lds + (3 * cc + 1) * S * S;
    const double* sD2 = lds + (3 * cc + 2) * S * S;
    MAcc<S> src;
    if (b.is_tip) {
      const double* row = a.code_table + (size_t)a.codes[(size_t)b.child * a.n_pad + p] * S;
#pragma unroll
      for (int xt = 0; xt < XT; ++xt)
#pragma unroll
        for (int r = 0; r < 4; ++r) src[xt][r] = m_valid<S>(xt, r, lr) ? row[16 * xt + lr + 4 * r] : 0.0;
    } else {
      const double* L = a.partials + (size_t)b.child * a.slot_stride + ((size_t)tile * CS + c * S) * kTile + q;
#pragma unroll
      for (int xt = 0; xt < XT; ++xt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          src[xt][r] = m_valid<S>(xt, r, lr) ? L[(size_t)(16 * xt + lr + 4 * r) * kTile] : 0.0;
    }
    f64x4m d0[XT], d1[XT], d2[XT];
    matvec_m<S>(d0, src, sP, lr, lc);
    matvec_m<S>(d1, src, sD, lr, lc);
    matvec_m<S>(d2, src, sD2, lr, lc);
    const double* U = a.partials + (size_t)b.uslot * a.slot_stride + ((size_t)tile * CS + c * S) * kTile + q;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int xt = 0; xt < XT; ++xt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (m_valid<S>(xt, r, lr)) {
          const int x = 16 * xt + lr + 4 * r;
          const double u = b.use_pi ? U[(size_t)x * kTile] * a.pi[x] : U[(size_t)x * kTile];
          s0 = fma(u, d0[xt][r], s0);
          s1 = fma(u, d1[xt][r], s1);
          s2 = fma(u, d2[xt][r], s2);
        }
    s0 += __shfl_xor(s0, 16, 64);
    s1 += __shfl_xor(s1, 16, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s0 += __shfl_xor(s0, 32, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    l0 = fma(a.probs[c], s0, l0);
    l1 = fma(a.probs[c], s1, l1);
    l2 = fma(a.probs[c], s2, l2);
  }
  double r1 = 0.0, r2 = 0.0;
  if (live && lr == 0) {
    const double gg = l1 / l0, hh = l2 / l0;
    r1 = a.weights[p] * gg;
    r2 = a.weights[p] * (hh - gg * gg);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    r1 += __shfl_xor(r1, off, 64);
    r2 += __shfl_xor(r2, off, 64);
  }
  if (lane == 0) {
    red[0][g] = r1;
    red[1][g] = r2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t1 = 0.0, t2 = 0.0;
    for (int k = 0; k < kDrmThreads / 64; ++k) {  // fixed order
      t1 += red[0][k];
      t2 += red[1][k];
    }
    a.blk1[(size_t)blockIdx.y * a.n_blk + blk] = t1;
    a.blk2[(size_t)blockIdx.y * a.n_blk + blk] = t2;
  }
  __syncthreads();  // red[] and (G < C) the staged matrices are reused by the next block
  }  // blocks
}

// Per branch: the fixed-order sum of its block sums (strided partial sums, then a
// fixed LDS tree), written to out1/out2[node].
// ---------------------------------------------------------------------------
// Fused preorder for 4 states without rescaling: one launch per preorder level, one
// workgroup = 256 patterns of one father f.  Per class the father-side vector of f's sons
// is formed in registers,
//     MU = pi (f the root) or P_f^T U_f,   Q_j = P_j L_j,   U_i = MU (*) prod_{j != i} Q_j,
// U_i is stored only for an internal son (its own sons read it at the next level), and
// son i's branch terms l, l', l'' (Q_i, dP_i L_i, d2P_i L_i against U_i) are reduced right
// there -- the separate reduction pass, which re-read every U_v and L_v, disappears
// (cfg2: 64.7 -> ~23.5 KB of HBM traffic per pattern).  pi sits in the root sons' U
// instead of in M_f, so results equal dr_branch_kernel's to rounding, not bitwise.
struct DrPreOp {      // (field order is read as 18 int32 by dr_pre_s4_kernel)
  int32_t f;          // father node (its P for P_f^T)
  int32_t uf_slot;    // slot of U_f; -1: f is the root
  int32_t n;          // sons (2 or 3)
  int32_t son[3];     // son node (P, dP, d2P index)
  int32_t is_tip[3];
  int32_t idx[3];     // tip index or internal slot of the son's L
  int32_t uslot[3];   // slot receiving U_son (internal sons), -1: not stored
  int32_t bidx[3];    // the son's branch row in blk1 / blk2
};

// (the op and the wave-uniform matrices are read through the constant address space:
// scalar loads into SGPRs -- through plain pointers the U stores would make every later
// matrix read a per-lane vector load, as the compiler cannot rule out aliasing)
typedef __attribute__((address_space(4))) const double* DrCPd;
// With rescaling (SCALE) the stored U of an internal son is rescaled jointly over its
// states and classes (x 2^256 when that maximum is below 2^-256, the traversal's rule)
// after the class loop, in place: the lane rewrites its own stores.  The branch terms need
// no scale bookkeeping: l, l', l'' share U's and L's factors, and only their ratios enter.
template <int C, bool SCALE = false>
// (part / uout: the partial slots read (L, U_f) and written (U of internal sons) -- never
// the same slot within a launch, so both are restrict and the next class's loads may be
// scheduled above this class's stores)
__global__ __launch_bounds__(kDrThreads) void dr_pre_s4_kernel(const DrPreOp* __restrict__ ops, DrArgs a,
                                                               const double* __restrict__ part,
                                                               double* __restrict__ uout) {
  constexpr int S = 4;
  __shared__ double red[2][3][kDrThreads / 64];
  typedef __attribute__((address_space(4))) const int32_t* DrCI;
  const DrCI w = (DrCI)(ops + blockIdx.y);
  DrPreOp op;
  op.f = w[0];
  op.uf_slot = w[1];
  op.n = w[2];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    op.son[j] = w[3 + j];
    op.is_tip[j] = w[6 + j];
    op.idx[j] = w[9 + j];
    op.uslot[j] = w[12 + j];
    op.bidx[j] = w[15 + j];
  }
  const int64_t p = (int64_t)blockIdx.x * kDrThreads + threadIdx.x;
  const bool live = p < a.n_patterns;
  const int64_t tile = p >> 7, q = p & (kTile - 1);
  double l0[3] = {0.0, 0.0, 0.0}, l1[3] = {0.0, 0.0, 0.0}, l2[3] = {0.0, 0.0, 0.0};
  double umax[3] = {0.0, 0.0, 0.0};  // SCALE: joint max of each stored U
  // operand sources per son: a tip's code-table row (the same for every class) or the
  // internal son's partial; a missing third son aliases son 0 (loaded, never used).  The
  // next class's operands are loaded before this class's arithmetic and stores.
  const int64_t tb = (int64_t)tile * C * S * kTile + q;
  const double* sb[3];
  int64_t sst[3], scs[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int jj = j < op.n ? j : 0;
    if (op.is_tip[jj]) {
      sb[j] = a.code_table + (int64_t)a.codes[(int64_t)op.idx[jj] * a.n_pad + p] * S;
      sst[j] = 1;
      scs[j] = 0;
    } else {
      sb[j] = part + (int64_t)op.idx[jj] * a.slot_stride + tb;
      sst[j] = kTile;
      scs[j] = S * kTile;
    }
  }
  const bool root = op.uf_slot < 0;
  const double* ub = part + (int64_t)(root ? 0 : op.uf_slot) * a.slot_stride + tb;
  double Lb[2][3][S], Ub[2][S];
  auto load = [&](int c, int bf) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int z = 0; z < S; ++z) Lb[bf][j][z] = sb[j][c * scs[j] + z * sst[j]];
    if (!root)
#pragma unroll
      for (int y = 0; y < S; ++y) Ub[bf][y] = ub[(int64_t)c * S * kTile + (int64_t)y * kTile];
  };
  load(0, 0);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int bf = c & 1;
    if (c + 1 < C) load(c + 1, bf ^ 1);
    const int64_t co = tb + (int64_t)c * S * kTile;
    double mu[S];
    if (root) {
#pragma unroll
      for (int x = 0; x < S; ++x) mu[x] = ((DrCPd)a.pi)[x];
    } else {
      const DrCPd Pf = (DrCPd)(a.pmats + ((int64_t)op.f * C + c) * S * S);
#pragma unroll
      for (int x = 0; x < S; ++x) {
        double t = 0.0;
#pragma unroll
        for (int y = 0; y < S; ++y) t = fma(Pf[y * S + x], Ub[bf][y], t);
        mu[x] = t;
      }
    }
    double Q[3][S];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j >= op.n) continue;
      const DrCPd P = (DrCPd)(a.pmats + ((int64_t)op.son[j] * C + c) * S * S);
#pragma unroll
      for (int x = 0; x < S; ++x) {
        double t = 0.0;
#pragma unroll
        for (int z = 0; z < S; ++z) t = fma(P[x * S + z], Lb[bf][j][z], t);
        Q[j][x] = t;
      }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i >= op.n) continue;
      double u[S];
#pragma unroll
      for (int x = 0; x < S; ++x) {
        double t = mu[x];
#pragma unroll
        for (int j = 0; j < 3; ++j)
          if (j != i && j < op.n) t *= Q[j][x];
        u[x] = t;
      }
      if (op.uslot[i] >= 0) {
        double* dst = uout + (int64_t)op.uslot[i] * a.slot_stride + co;
#pragma unroll
        for (int x = 0; x < S; ++x) dst[(int64_t)x * kTile] = u[x];
        if (SCALE)
#pragma unroll
          for (int x = 0; x < S; ++x) umax[i] = fmax(umax[i], u[x]);
      }
      const DrCPd D1 = (DrCPd)(a.dpmats + ((int64_t)op.son[i] * C + c) * S * S);
      const DrCPd D2 = (DrCPd)(a.d2pmats + ((int64_t)op.son[i] * C + c) * S * S);
      double s0 = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll
      for (int x = 0; x < S; ++x) {
        double t1 = 0.0, t2 = 0.0;
#pragma unroll
        for (int z = 0; z < S; ++z) {
          t1 = fma(D1[x * S + z], Lb[bf][i][z], t1);
          t2 = fma(D2[x * S + z], Lb[bf][i][z], t2);
        }
        s0 = fma(u[x], Q[i][x], s0);
        s1 = fma(u[x], t1, s1);
        s2 = fma(u[x], t2, s2);
      }
      const double pc = ((DrCPd)a.probs)[c];
      l0[i] = fma(pc, s0, l0[i]);
      l1[i] = fma(pc, s1, l1[i]);
      l2[i] = fma(pc, s2, l2[i]);
    }
  }
  if (SCALE)
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (i < op.n && op.uslot[i] >= 0 && umax[i] > 0.0 && umax[i] < kScaleThr) {
        double* dst = uout + (int64_t)op.uslot[i] * a.slot_stride + tb;
#pragma unroll
        for (int e = 0; e < C * S; ++e) dst[(int64_t)e * kTile] *= kScaleUp;
      }
  const int wv = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (i >= op.n) continue;
    double r1 = 0.0, r2 = 0.0;
    if (live) {
      const double g = l1[i] / l0[i], hh = l2[i] / l0[i];
      r1 = a.weights[p] * g;
      r2 = a.weights[p] * (hh - g * g);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      r1 += __shfl_xor(r1, off, 64);
      r2 += __shfl_xor(r2, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
      red[0][i][wv] = r1;
      red[1][i][wv] = r2;
    }
  }
  __syncthreads();
  if (threadIdx.x < 3 && (int)threadIdx.x < op.n) {
    const int i = threadIdx.x;
    double t1 = 0.0, t2 = 0.0;
    for (int k = 0; k < kDrThreads / 64; ++k) {  // fixed order
      t1 += red[0][i][k];
      t2 += red[1][i][k];
    }
    a.blk1[(size_t)op.bidx[i] * a.n_blk + blockIdx.x] = t1;
    a.blk2[(size_t)op.bidx[i] * a.n_blk + blockIdx.x] = t2;
  }
}

// ---------------------------------------------------------------------------
// Fused preorder for 20 states on v_mfma_f64_4x4x4_4b (plk_jitm.hpp's layout): 20 states
// tile as 5 x 4 with no padding, where 16x16x4 tiles would pad 20 to 32 in both
// dimensions (39 % useful flops).  Lane l = 16 hi + 4 b + lo of wave w holds states
// 4X + hi (X = 0..4) of pattern 16 w + 4 b + lo; a matvec D = M v is, per X, five MFMAs
// over Y with A(X, Y)[lo][hi] = M[4X + lo][4Y + hi] read from LDS, and v's register Y as
// the B operand (D comes out in the same layout, so products chain in registers).  Per
// class the workgroup stages the matrices of the op -- P_f (read transposed for
// M_f = P_f^T) and each son's P, dP, d2P, as stored -- in LDS; the products, rescaling
// and per-block branch terms as dr_pre_s4_kernel's, on 64-pattern blocks: per class
//     MU = pi (f the root) or P_f^T U_f,   Q_j = P_j L_j,
//     U_i = MU (*) prod_{j != i} Q_j   (stored for internal sons),
//     l += p_c U_i . Q_i,  l' += p_c U_i . (dP_i L_i),  l'' += p_c U_i . (d2P_i L_i),
// stored U rescaled jointly over states and classes after the class loop.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double dr_mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

template <int C, bool SCALE, int NS>
__global__ __launch_bounds__(256) void dr_pre_m20_kernel(const DrPreOp* __restrict__ ops, DrArgs a) {
  constexpr int S = 20, XB = 5, SS = S * S, CS = C * S;
  __shared__ __attribute__((aligned(16))) double mats[10 * SS];  // [P_f | P_j, dP_j, d2P_j for j < 3] of one class
  __shared__ double red[2][3][4];
  const DrPreOp op = ops[blockIdx.y];
  const int nsn = NS == 2 ? min(2, op.n) : op.n;  // (the two-son build)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int hi = lane >> 4, lo = lane & 3;
  const int64_t p = (int64_t)blockIdx.x * 64 + 16 * w + (lane & 15);
  const bool live = p < a.n_patterns;
  const int64_t tb = (p >> 7) * CS * kTile + (p & (kTile - 1)) + (int64_t)hi * kTile;
  const bool root = op.uf_slot < 0;
  const int nm = 1 + 3 * nsn;
  double l0[3] = {0.0, 0.0, 0.0}, l1[3] = {0.0, 0.0, 0.0}, l2[3] = {0.0, 0.0, 0.0};
  double umax[3] = {0.0, 0.0, 0.0};
  // D = M v for M at LDS matrix m (as stored, or transposed)
  auto matvec = [&](double (&d)[XB], const double (&v)[XB], int m, bool transposed) {
    const double* M = mats + m * SS;
#pragma unroll
    for (int X = 0; X < XB; ++X) {
      double acc = 0.0;
#pragma unroll
      for (int Y = 0; Y < XB; ++Y)
        acc = dr_mfma4(transposed ? M[(4 * Y + hi) * S + 4 * X + lo] : M[(4 * X + lo) * S + 4 * Y + hi], v[Y], acc);
      d[X] = acc;
    }
  };
  auto loadL = [&](int j, int c, double (&v)[XB]) {
    if (op.is_tip[j]) {
      const double* row = a.code_table + (int64_t)a.codes[(int64_t)op.idx[j] * a.n_pad + p] * S + hi;
#pragma unroll
      for (int X = 0; X < XB; ++X) v[X] = row[4 * X];
    } else {
      const double* L = a.partials + (int64_t)op.idx[j] * a.slot_stride + tb + (int64_t)c * S * kTile;
#pragma unroll
      for (int X = 0; X < XB; ++X) v[X] = L[(int64_t)(4 * X) * kTile];
    }
  };
  auto dot = [&](const double (&u)[XB], const double (&t)[XB]) {
    double s = 0.0;
#pragma unroll
    for (int X = 0; X < XB; ++X) s = fma(u[X], t[X], s);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    return s;
  };
#pragma unroll 1
  for (int c = 0; c < C; ++c) {
    // this class's matrices: every thread's 16-byte loads issued before the first store (a
    // loop of load -> store paid one L2 round trip per element, ~11 per thread and class);
    // out-of-range lanes load element 0 and store nothing (matrices are 400 doubles, so no
    // pair straddles two of them)
    constexpr int NE2 = ((1 + 3 * NS) * SS / 2 + 255) / 256;
    double2 mv[NE2];
    int tq = tid;
    asm volatile("" : "+v"(tq));  // (opaque per class: the element addresses are not hoisted out of the class loop)
#pragma unroll
    for (int q = 0; q < NE2; ++q) {
      const int e0 = 2 * (tq + 256 * q), e = e0 < nm * SS ? e0 : 0;
      const int m = e / SS, k = e - m * SS;
      const int j = (m - 1) / 3, kind = (m - 1) - 3 * j;
      // (selects, not op.son[j]: a runtime index would put the op in scratch memory)
      const int son = j == 0 ? op.son[0] : j == 1 ? op.son[1] : op.son[2];
      const double* src = m == 0 ? a.pmats + ((size_t)op.f * C + c) * SS
                                 : (kind == 0 ? a.pmats : kind == 1 ? a.dpmats : a.d2pmats) +
                                       ((size_t)son * C + c) * SS;
      mv[q] = *reinterpret_cast<const double2*>(src + k);
    }
    __syncthreads();  // the previous class is done with mats
#pragma unroll
    for (int q = 0; q < NE2; ++q) {
      const int e = 2 * (tid + 256 * q);
      if (e < nm * SS) *reinterpret_cast<double2*>(mats + e) = (e < SS && root) ? make_double2(0.0, 0.0) : mv[q];
    }
    __syncthreads();
    double mu[XB];
    if (root) {
#pragma unroll
      for (int X = 0; X < XB; ++X) mu[X] = a.pi[4 * X + hi];
    } else {
      const double* U = a.partials + (int64_t)op.uf_slot * a.slot_stride + tb + (int64_t)c * S * kTile;
      double uf[XB];
#pragma unroll
      for (int X = 0; X < XB; ++X) uf[X] = U[(int64_t)(4 * X) * kTile];
      matvec(mu, uf, 0, true);  // M_f U_f = P_f^T U_f
    }
    double Q[3][XB];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (j >= nsn) continue;
      double L[XB];
      loadL(j, c, L);
      matvec(Q[j], L, 1 + 3 * j, false);
    }
    const double pc = a.probs[c];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i >= nsn) continue;
      double u[XB];
#pragma unroll
      for (int X = 0; X < XB; ++X) {
        u[X] = mu[X];
#pragma unroll
        for (int j = 0; j < 3; ++j)
          if (j != i && j < nsn) u[X] *= Q[j][X];
      }
      if (op.uslot[i] >= 0) {
        double* dst = a.uout + (int64_t)op.uslot[i] * a.slot_stride + tb + (int64_t)c * S * kTile;
#pragma unroll
        for (int X = 0; X < XB; ++X) {
          dst[(int64_t)(4 * X) * kTile] = u[X];
          if (SCALE) umax[i] = fmax(umax[i], u[X]);
        }
      }
      const double s0 = dot(u, Q[i]);
      double L[XB], t[XB];
      loadL(i, c, L);
      matvec(t, L, 2 + 3 * i, false);
      const double s1 = dot(u, t);
      matvec(t, L, 3 + 3 * i, false);
      const double s2 = dot(u, t);
      l0[i] = fma(pc, s0, l0[i]);
      l1[i] = fma(pc, s1, l1[i]);
      l2[i] = fma(pc, s2, l2[i]);
    }
  }
  if (SCALE)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i >= nsn || op.uslot[i] < 0) continue;
      double m = umax[i];
      m = fmax(m, __shfl_xor(m, 16, 64));
      m = fmax(m, __shfl_xor(m, 32, 64));
      if (m > 0.0 && m < kScaleThr) {
        double* dst = a.uout + (int64_t)op.uslot[i] * a.slot_stride + tb;
        for (int c = 0; c < C; ++c)
#pragma unroll
          for (int X = 0; X < XB; ++X) dst[(int64_t)(c * S + 4 * X) * kTile] *= kScaleUp;
      }
    }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (i >= nsn) continue;
    double r1 = 0.0, r2 = 0.0;
    if (live && hi == 0) {
      const double g = l1[i] / l0[i], hh = l2[i] / l0[i];
      r1 = a.weights[p] * g;
      r2 = a.weights[p] * (hh - g * g);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      r1 += __shfl_xor(r1, off, 64);
      r2 += __shfl_xor(r2, off, 64);
    }
    if (lane == 0) {
      red[0][i][w] = r1;
      red[1][i][w] = r2;
    }
  }
  __syncthreads();
  if (tid < 3 && tid < nsn) {
    double t1 = 0.0, t2 = 0.0;
    for (int k = 0; k < 4; ++k) {  // fixed order
      t1 += red[0][tid][k];
      t2 += red[1][tid][k];
    }
    const int b = tid == 0 ? op.bidx[0] : tid == 1 ? op.bidx[1] : op.bidx[2];
    a.blk1[(size_t)b * a.n_blk + blockIdx.x] = t1;
    a.blk2[(size_t)b * a.n_blk + blockIdx.x] = t2;
  }
}

__global__ __launch_bounds__(256) void dr_sum_kernel(const DrBranch* __restrict__ branches, const double* __restrict__ blk1,
                                                     const double* __restrict__ blk2, int n_blk, double* __restrict__ out1,
                                                     double* __restrict__ out2) {
  __shared__ double s1[256], s2[256];
  const size_t o = (size_t)blockIdx.x * n_blk;
  double t1 = 0.0, t2 = 0.0;
  for (int i = threadIdx.x; i < n_blk; i += 256) {
    t1 += blk1[o + i];
    t2 += blk2[o + i];
  }
  s1[threadIdx.x] = t1;
  s2[threadIdx.x] = t2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      s1[threadIdx.x] += s1[threadIdx.x + w];
      s2[threadIdx.x] += s2[threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out1[branches[blockIdx.x].node] = s1[0];
    out2[branches[blockIdx.x].node] = s2[0];
  }
}

}  // namespace plk
