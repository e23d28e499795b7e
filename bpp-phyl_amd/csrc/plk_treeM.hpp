// plk_treeM.hpp -- fused postorder traversal on fp64 matrix cores for S = 20 (protein)
// and S = 64 (codon) models (gfx950).
//
// Same tree programs as plk_tree4.hpp (TInstr words, fragments, tiers).  A wave owns
// 16 consecutive site patterns of ONE rate class; a workgroup is C x 4 waves = 64
// patterns x all classes.  The partial of a node lives in the C/D register layout of
// v_mfma_f64_16x16x4f64: lane l holds states x = 16*xt + (l>>4) + 4*r (r = 0..3) of
// pattern l&15, for the XT = ceil(S/16) row tiles.  A child's contribution
//     D[x][p] = sum_y P[x][y] L[y][p]       (RHomogeneousTreeLikelihood.cpp:839-861)
// is a chain of KS = S/4 MFMAs per row tile, and that layout is also exactly the B
// operand layout of the next level: B for k-step ks is the register (xt, r) =
// (ks/4, ks%4) of the same lane.  So a DESCEND child feeds its parent straight from
// registers, with no shuffle and no LDS round trip; LOAD children come from HBM as
// 128-byte row segments.  Padding rows x >= S (S = 20: 12 of the 32 rows) have zero
// A rows, so they stay zero through the product.
//
// LDS-staged tables, double-buffered: every event that needs a table -- TIP (the tip
// table tipP[tip][c][code][x] of all classes) and LOAD / child ASCEND (P^T of the
// branch, all classes) -- finds it already in LDS buffer `cur`.  While it computes,
// each thread holds its slice of the NEXT event's table in registers (the builder
// chains the tables through TInstr.d), writes it to buffer cur^1 afterwards, and one
// workgroup barrier hands the buffers over.  The L2 latency of the tables thus hides
// behind the MFMA chains, the A operands come from LDS (conflict-light 64-bit reads),
// and the tip codes of the workgroup's 64 patterns are staged once at the start.
//
// Rescaling is the joint (all states, all classes) exact power-of-two rule of the
// other kernels; the fused root reduction writes per-pattern lnL and the same
// fixed-order 64-pattern wave sums as root_kernel (plk_kernels.hpp).
#pragma once

#include "plk_tree4.hpp"

namespace plk {

constexpr int kTreeMGroups = 4;  // 16-pattern groups per workgroup (64 patterns)

template <int S>
struct MShape {
  static constexpr int XT = (S + 15) / 16;  // 16-row tiles of the state dimension
  static constexpr int KS = S / 4;          // k-steps (S % 4 == 0)
};

typedef double f64x4m __attribute__((ext_vector_type(4)));

template <int S>
using MAcc = f64x4m[MShape<S>::XT];

template <int S>
__device__ __forceinline__ bool m_valid(int xt, int r, int lr) {
  return S % 16 == 0 || 16 * xt + lr + 4 * r < S;
}

// d[x] = sum_y P[x][y] src[y]  for the lane's 16-pattern column; PT = P^T of the child's
// branch and this wave's class ([y][x], row stride S; LDS or global)
template <int S>
__device__ __forceinline__ void matvec_m(f64x4m (&d)[MShape<S>::XT], const MAcc<S>& src, const double* PT, int lr,
                                         int lc) {
  constexpr int XT = MShape<S>::XT, KS = MShape<S>::KS;
#pragma unroll
  for (int xt = 0; xt < XT; ++xt) d[xt] = (f64x4m){0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const double b = src[ks >> 2][ks & 3];
#pragma unroll
    for (int xt = 0; xt < XT; ++xt) {
      const int x = 16 * xt + lc;
      const double av = (S % 16 == 0 || x < S) ? PT[(4 * ks + lr) * S + x] : 0.0;
      d[xt] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b, d[xt], 0, 0, 0);
    }
  }
}

// acc[x] *= sum_y P[x][y] src[y]
template <int S>
__device__ __forceinline__ void contribute_m(MAcc<S>& acc, const MAcc<S>& src, const double* PT, int lr, int lc) {
  constexpr int XT = MShape<S>::XT;
  f64x4m d[XT];
  matvec_m<S>(d, src, PT, lr, lc);
#pragma unroll
  for (int xt = 0; xt < XT; ++xt) acc[xt] *= d[xt];
}

// Cherry contribution tables.  A cherry (a node whose only children are two tips) that
// is not stored contributes to its parent  D = P_cherry . (row_a (*) row_b)  -- a function
// of its tips' two codes only.  cherry_table_kernel forms D for every code pair (U^2
// rows) with the same operations as the traversal (tip products from 1, the joint
// rescale of rescale_m, matvec_m), so a T_CHERRY event is one row gather, bitwise equal to
// the DESCEND / TIP / TIP / ASCEND it replaces, with no table staging and no barrier.
// Per cherry, at a.cherry + k * stride: table [C][U^2][S] fp64 | counts [U^2] u8 (padded
// to 8) | combined codes ca * U + cb [n_pad] u16.
struct CherryLayout {
  size_t table_bytes, count_bytes, stride;
  __host__ __device__ CherryLayout(int C, int U, int S, int64_t n_pad) {
    table_bytes = (size_t)C * U * U * S * sizeof(double);
    count_bytes = ((size_t)U * U + 7) & ~(size_t)7;
    stride = table_bytes + count_bytes + (size_t)n_pad * sizeof(uint16_t);
  }
};

// codes of cherry k = blockIdx.y (tips cherry_tips[2k], [2k+1])
__global__ __launch_bounds__(256) void cherry_codes_kernel(const uint8_t* __restrict__ codes, int64_t n_pad,
                                                           const int32_t* __restrict__ cherry_tips, int U,
                                                           CherryLayout lay, uint8_t* __restrict__ cherry) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_pad) return;
  const int k = blockIdx.y;
  const int ca = codes[(int64_t)cherry_tips[2 * k] * n_pad + i], cb = codes[(int64_t)cherry_tips[2 * k + 1] * n_pad + i];
  uint16_t* out = reinterpret_cast<uint16_t*>(cherry + (size_t)k * lay.stride + lay.table_bytes + lay.count_bytes);
  out[i] = (uint16_t)(ca * U + cb);
}

// mark[k][ca * U + cb] = 1 for every code pair cherry k = blockIdx.y meets (padding included)
__global__ __launch_bounds__(256) void cherry_mark_kernel(int64_t n_pad, int U, CherryLayout lay,
                                                          const uint8_t* __restrict__ cherry, uint8_t* __restrict__ mark) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_pad) return;
  const int k = blockIdx.y;
  const uint16_t* cc = reinterpret_cast<const uint16_t*>(cherry + (size_t)k * lay.stride + lay.table_bytes + lay.count_bytes);
  mark[(size_t)k * U * U + cc[i]] = 1;
}

// Four waves per block, one per 16 code pairs (rows) of one cherry and class: blockIdx.x =
// 64-row block, blockIdx.y = cherry * C + class; P^T of the cherry branch is staged in LDS.
// cherry3[3k .. 3k+2] = tip a, tip b, cherry node.  Only the code pairs the cherry's tips
// meet are formed (row_list[row_start[k] ..], row_start[k + 1]): the traversal reads no other
// row (cfg4: ~1/3 of the 61^2 codon pairs occur under the model).
template <int S, bool SCALE>
__global__ __launch_bounds__(256) void cherry_table_kernel(const double* __restrict__ tipP,
                                                           const double* __restrict__ pmatsT,
                                                           const int32_t* __restrict__ cherry3, int C, int U,
                                                           CherryLayout lay, uint8_t* __restrict__ cherry,
                                                           int rows_per_wg, const int32_t* __restrict__ row_start,
                                                           const int32_t* __restrict__ row_list) {
  constexpr int XT = MShape<S>::XT;
  __shared__ double PTl[S * S];
  const int lane = threadIdx.x & 63, lr = lane >> 4, lc = lane & 15;
  const int k = blockIdx.y / C, c = blockIdx.y % C, U2 = U * U;
  {
    const double* PT = pmatsT + ((size_t)cherry3[3 * k + 2] * C + c) * S * S;
    stage_lds<(S * S + 255) / 256>(PTl, PT, S * S);
    __syncthreads();
  }
  // each workgroup stages P^T once and covers rows_per_wg code pairs, 64 per pass
  const int rs = row_start[k], nr = row_start[k + 1] - rs;
  for (int r0 = blockIdx.x * rows_per_wg; r0 < min(nr, (int)(blockIdx.x + 1) * rows_per_wg); r0 += 64) {
  const int pos = r0 + (threadIdx.x >> 6) * 16 + lc;  // this lane's entry of the row list
  const bool rv = pos < nr;
  const int r = rv ? row_list[rs + pos] : 0;  // its row (code pair)
  const int ca = rv ? r / U : 0, cb = rv ? r % U : 0;
  const int ta = cherry3[3 * k], tb = cherry3[3 * k + 1], node = cherry3[3 * k + 2];
  // the cherry's partial for every class (the joint check needs all of them), own class kept
  MAcc<S> acc;
  double m = 0.0;
  for (int cc = 0; cc < C; ++cc) {
    const double* rowa = tipP + (((size_t)ta * C + cc) * U + ca) * S;
    const double* rowb = tipP + (((size_t)tb * C + cc) * U + cb) * S;
#pragma unroll
    for (int xt = 0; xt < XT; ++xt)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int x = 16 * xt + lr + 4 * q;
        double v = 1.0;
        v *= m_valid<S>(xt, q, lr) ? rowa[x] : 0.0;
        v *= m_valid<S>(xt, q, lr) ? rowb[x] : 0.0;
        if (m_valid<S>(xt, q, lr)) m = fmax(m, v);
        if (cc == c) acc[xt][q] = v;
      }
  }
  m = fmax(m, __shfl_xor(m, 16, 64));
  m = fmax(m, __shfl_xor(m, 32, 64));
  int cnt = 0;
  if (SCALE && m > 0.0 && m < kScaleThr) {
#pragma unroll
    for (int xt = 0; xt < XT; ++xt) acc[xt] *= kScaleUp;
    cnt = 1;
  }
  f64x4m d[XT];
  (void)node;
  matvec_m<S>(d, acc, PTl, lr, lc);
  uint8_t* base = cherry + (size_t)k * lay.stride;
  if (rv) {
    double* row = reinterpret_cast<double*>(base) + ((size_t)c * U2 + r) * S;
#pragma unroll
    for (int xt = 0; xt < XT; ++xt)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (m_valid<S>(xt, q, lr)) row[16 * xt + lr + 4 * q] = d[xt][q];
    if (c == 0 && lr == 0) base[lay.table_bytes + r] = (uint8_t)cnt;
  }
  }  // row passes
}

template <int S>
__device__ __forceinline__ void rescale_m(MAcc<S>& v, int& cnt, double* xch, int C, int c, int g, int lr, int lc) {
  constexpr int XT = MShape<S>::XT;
  double m = 0.0;
#pragma unroll
  for (int xt = 0; xt < XT; ++xt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (m_valid<S>(xt, r, lr)) m = fmax(m, v[xt][r]);
  m = fmax(m, __shfl_xor(m, 16, 64));
  m = fmax(m, __shfl_xor(m, 32, 64));
  if (C > 1) {
    if (lr == 0) xch[(c * kTreeMGroups + g) * 16 + lc] = m;
    __syncthreads();
    m = 0.0;
    for (int k = 0; k < C; ++k) m = fmax(m, xch[(k * kTreeMGroups + g) * 16 + lc]);
    __syncthreads();
  }
  if (m > 0.0 && m < kScaleThr) {
#pragma unroll
    for (int xt = 0; xt < XT; ++xt) v[xt] *= kScaleUp;
    cnt += 1;
  }
}

template <int S, bool SCALE>
__device__ __forceinline__ void store_partial_m(const TreeArgs& a, int slot, int64_t p, int c, const MAcc<S>& v,
                                                int cnt, int lr) {
  constexpr int XT = MShape<S>::XT;
  const int64_t tile = p >> 7, q = p & (kTile - 1);
  double* dst = a.partials + (size_t)slot * a.slot_stride + tile * ((int64_t)a.C * S * kTile) + (size_t)c * S * kTile + q;
#pragma unroll
  for (int xt = 0; xt < XT; ++xt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (m_valid<S>(xt, r, lr)) __builtin_nontemporal_store(v[xt][r], dst + (size_t)(16 * xt + lr + 4 * r) * kTile);
  if (SCALE && c == 0 && lr == 0) a.scale[(size_t)slot * a.n_pad + p] = cnt;
}

// ---- table staging (see the header): res >= 0 -> P^T of branch res, res <= -2 -> tip
// table of tip -2-res, -1 -> nothing
template <int S>
__device__ __forceinline__ int table_size(const TreeArgs& a, int res) {
  return res >= 0 ? a.C * S * S : (res <= -2 ? a.C * a.n_codes * S : 0);
}

// Every thread moves exactly PF doubles per table: loads clamp to the table (no
// divergent predicates, no phis); a buffer holds at least (PF-1) x blockDim doubles,
// so only the last store is predicated (the tail beyond the table is never read).
template <int S, int PF>
__device__ __forceinline__ void stage_load(const TreeArgs& a, const double* __restrict__ pmatsT, int res,
                                           double (&pf)[PF]) {
  const int n = table_size<S>(a, res);
  const double* src = res >= 0 ? pmatsT + (size_t)res * a.C * S * S
                               : (res <= -2 ? a.tipP + (size_t)(-2 - res) * a.C * a.n_codes * S : pmatsT);
  const int last = n > 0 ? n - 1 : 0;
#pragma unroll
  for (int j = 0; j < PF; ++j) pf[j] = src[min((int)threadIdx.x + j * (int)blockDim.x, last)];
}

template <int S, int PF>
__device__ __forceinline__ void stage_store(const TreeArgs& a, int res, const double (&pf)[PF], double* buf) {
#pragma unroll
  for (int j = 0; j < PF - 1; ++j) buf[threadIdx.x + j * blockDim.x] = pf[j];
  const int i = threadIdx.x + (PF - 1) * blockDim.x;
  if (i < a.buf_doubles) buf[i] = pf[PF - 1];
}

struct MCtx {
  double* buf;            // two table buffers of a.buf_doubles each
  const uint8_t* codes;   // staged codes [n_tips][64] or null
  const uint16_t* ccodes; // staged cherry codes [n_cherry_staged][64] or null
  double* xch;
  int cur;
};

template <int S, int PF>
__device__ __forceinline__ void handover(const TreeArgs& a, MCtx& m, int next, const double (&pf)[PF]) {
  stage_store<S, PF>(a, next, pf, m.buf + (m.cur ^ 1) * a.buf_doubles);
  __syncthreads();
  m.cur ^= 1;
}

template <int S, int PF, int D, int DM, bool SCALE, bool DIRECT>
__device__ __forceinline__ void eval_node_m(const TreeArgs& a, const TInstr* __restrict__& pc,
                                            const double* __restrict__ pmatsT, MCtx& m, int c, int g, int lr,
                                            int lc, int64_t p, MAcc<S>& acc, int& cnt) {
  constexpr int XT = MShape<S>::XT;
#pragma unroll
  for (int xt = 0; xt < XT; ++xt) acc[xt] = (f64x4m){1.0, 1.0, 1.0, 1.0};
  cnt = 0;
  for (;;) {
    const TInstr in = fetch_instr(pc++);
    if (in.op == T_ASCEND) {
      if (in.b >= 0) {
        if (SCALE) rescale_m<S>(acc, cnt, m.xch, a.C, c, g, lr, lc);
        if (in.a >= 0) store_partial_m<S, SCALE>(a, in.a, p, c, acc, cnt, lr);
      }
      return;
    }
    if (in.op == T_TIP) {
      const int code = m.codes ? m.codes[in.a * 64 + 16 * g + lc] : a.codes[(size_t)in.a * a.n_pad + p];
      if constexpr (DIRECT) {
        // the tip table row straight from L2 (a per-lane gather by code)
        const double* t = a.tipP + ((size_t)in.a * a.C * a.n_codes + (size_t)c * a.n_codes + code) * S;
#pragma unroll
        for (int xt = 0; xt < XT; ++xt)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[xt][r] *= m_valid<S>(xt, r, lr) ? t[16 * xt + lr + 4 * r] : 0.0;
      } else {
        double pf[PF];
        stage_load<S, PF>(a, pmatsT, in.d, pf);
        const double* t = m.buf + m.cur * a.buf_doubles + (c * a.n_codes + code) * S;
#pragma unroll
        for (int xt = 0; xt < XT; ++xt)
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[xt][r] *= m_valid<S>(xt, r, lr) ? t[16 * xt + lr + 4 * r] : 0.0;
        handover<S, PF>(a, m, in.d, pf);
      }
    } else if (in.op == T_CHERRY) {
      // one row of the cherry's contribution table; no table staging, no barrier
      const CherryLayout lay(a.C, a.n_codes, S, a.n_pad);
      const uint8_t* base = a.cherry + (size_t)in.a * lay.stride;
      const int code = m.ccodes ? m.ccodes[in.a * 64 + 16 * g + lc]
                                : reinterpret_cast<const uint16_t*>(base + lay.table_bytes + lay.count_bytes)[p];
      const double* t = reinterpret_cast<const double*>(base) + ((size_t)c * a.n_codes * a.n_codes + code) * S;
      if (a.cherry_pairs) {
        const TInstr nx = fetch_instr(pc);
        if (nx.op == T_CHERRY) {
          // a sibling cherry follows: both rows' gathers in flight at once (their L2 / MALL
          // latencies overlap); multiplied in event order, so bitwise the same
          const uint8_t* base2 = a.cherry + (size_t)nx.a * lay.stride;
          const int code2 = m.ccodes ? m.ccodes[nx.a * 64 + 16 * g + lc]
                                     : reinterpret_cast<const uint16_t*>(base2 + lay.table_bytes + lay.count_bytes)[p];
          const double* t2 =
              reinterpret_cast<const double*>(base2) + ((size_t)c * a.n_codes * a.n_codes + code2) * S;
          double r1[XT][4], r2[XT][4];
#pragma unroll
          for (int xt = 0; xt < XT; ++xt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              r1[xt][r] = m_valid<S>(xt, r, lr) ? t[16 * xt + lr + 4 * r] : 0.0;
              r2[xt][r] = m_valid<S>(xt, r, lr) ? t2[16 * xt + lr + 4 * r] : 0.0;
            }
#pragma unroll
          for (int xt = 0; xt < XT; ++xt)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[xt][r] *= r1[xt][r];
#pragma unroll
          for (int xt = 0; xt < XT; ++xt)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[xt][r] *= r2[xt][r];
          if (SCALE) {
            cnt += base[lay.table_bytes + code];
            cnt += base2[lay.table_bytes + code2];
          }
          ++pc;
          continue;
        }
      }
#pragma unroll
      for (int xt = 0; xt < XT; ++xt)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[xt][r] *= m_valid<S>(xt, r, lr) ? t[16 * xt + lr + 4 * r] : 0.0;
      if (SCALE) cnt += base[lay.table_bytes + code];
    } else if (in.op == T_LOAD) {
      const int64_t tile = p >> 7, q = p & (kTile - 1);
      const double* L = a.partials + (size_t)in.a * a.slot_stride + tile * ((int64_t)a.C * S * kTile) +
                        (size_t)c * S * kTile + q;
      MAcc<S> src;
#pragma unroll
      for (int xt = 0; xt < XT; ++xt)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          src[xt][r] = m_valid<S>(xt, r, lr) ? L[(size_t)(16 * xt + lr + 4 * r) * kTile] : 0.0;
      if (SCALE) cnt += a.scale[(size_t)in.a * a.n_pad + p];
      if constexpr (DIRECT) {
        contribute_m<S>(acc, src, pmatsT + ((size_t)in.b * a.C + c) * S * S, lr, lc);
      } else {
        double pf[PF];
        stage_load<S, PF>(a, pmatsT, in.d, pf);
        contribute_m<S>(acc, src, m.buf + m.cur * a.buf_doubles + c * S * S, lr, lc);
        handover<S, PF>(a, m, in.d, pf);
      }
    } else {  // T_DESCEND
      if constexpr (D + 1 < DM) {
        MAcc<S> child;
        int ccnt;
        eval_node_m<S, PF, D + 1, DM, SCALE, DIRECT>(a, pc, pmatsT, m, c, g, lr, lc, p, child, ccnt);
        const TInstr up = fetch_instr(pc - 1);
        if constexpr (DIRECT) {
          contribute_m<S>(acc, child, pmatsT + ((size_t)up.b * a.C + c) * S * S, lr, lc);
        } else {
          double pf[PF];
          stage_load<S, PF>(a, pmatsT, up.d, pf);
          contribute_m<S>(acc, child, m.buf + m.cur * a.buf_doubles + c * S * S, lr, lc);
          handover<S, PF>(a, m, up.d, pf);
        }
        if (SCALE) cnt += ccnt;
      }
    }
  }
}

// Workgroup = C x kTreeMGroups waves; wave w: class c = w / 4, pattern group g = w % 4.
// S = 64 runs with one class (4 waves, up to 256 VGPRs); S = 20 with up to 4 classes
// (16 waves, 128 VGPRs = 4 waves per SIMD).  PF = table doubles per thread.
template <int S, int G>
constexpr int treeM_threads() { return S == 64 ? 64 * G : 64 * G * kTreeMaxWaves; }
template <int S, int G = 4>
constexpr int treeM_pf() { return S == 64 ? (G == 8 ? 9 : 17) : 3; }

// DIRECT: no LDS staging and no per-event barrier -- MFMA A operands (P^T) and tip
// table rows are read by each wave straight from L1/L2 (same values, same order).
// G = 16-pattern groups per workgroup (4: 64 patterns; 2: 32 patterns, two workgroups per
// CU for S = 20 -- the root's fixed-order 64-pattern wave sums are then formed from
// site_lnl by site_wave_sums_kernel, same butterfly, same bits).
template <int S, int DM, bool SCALE, bool DIRECT, int G>
__global__ __launch_bounds__((treeM_threads<S, G>()), (S == 64 ? 1 : 4)) void treeM_kernel(TreeArgs a, const TInstr* __restrict__ prog,
                                                                   const int32_t* __restrict__ frag_start,
                                                                   const double* __restrict__ pmatsT) {
  constexpr int XT = MShape<S>::XT;
  constexpr int PF = treeM_pf<S, G>();
  extern __shared__ __attribute__((aligned(16))) double lds[];  // 2 table buffers | codes
  __shared__ double xch[kTreeMaxWaves * kTreeMGroups * 16];
  __shared__ double red[16 * (G > kTreeMGroups ? G : kTreeMGroups)];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = w / G, g = w % G;
  const int lr = lane >> 4, lc = lane & 15;
  const int64_t p0 = (int64_t)blockIdx.x * (16 * G);
  const int64_t p = p0 + 16 * g + lc;
  MCtx m;
  m.buf = lds;
  m.xch = xch;
  m.cur = 0;
  m.codes = nullptr;
  if (a.stage_codes) {
    uint8_t* cl = reinterpret_cast<uint8_t*>(lds + 2 * a.buf_doubles);
    for (int i = threadIdx.x; i < a.n_tips * 4; i += blockDim.x) {
      const int t = i >> 2, j = i & 3;
      reinterpret_cast<uint4*>(cl)[i] = *reinterpret_cast<const uint4*>(a.codes + (size_t)t * a.n_pad + p0 + 16 * j);
    }
    m.codes = cl;
  }
  m.ccodes = nullptr;
  if constexpr (DIRECT) {
    if (a.n_cherry_staged) {
      // the cherries' combined codes of the workgroup's 64 patterns (read by every T_CHERRY
      // of every wave; one latency here instead of one per event)
      uint16_t* cc = reinterpret_cast<uint16_t*>(lds + 2 * a.buf_doubles) + (a.stage_codes ? a.n_tips * 32 : 0);
      const CherryLayout lay(a.C, a.n_codes, S, a.n_pad);
      for (int i = threadIdx.x; i < a.n_cherry_staged * 16; i += blockDim.x) {
        const int k = i >> 4, j = i & 15;
        const uint16_t* src = reinterpret_cast<const uint16_t*>(a.cherry + (size_t)k * lay.stride + lay.table_bytes +
                                                                lay.count_bytes) + p0 + 4 * j;
        reinterpret_cast<uint2*>(cc)[i] = *reinterpret_cast<const uint2*>(src);
      }
      m.ccodes = cc;
    }
  }
  if constexpr (!DIRECT) {
    const int first = frag_start[a.n_frags + blockIdx.y];
    double pf[PF];
    stage_load<S, PF>(a, pmatsT, first, pf);
    stage_store<S, PF>(a, first, pf, m.buf);
    __syncthreads();
  } else if (a.stage_codes || a.n_cherry_staged) {
    __syncthreads();
  }
  const TInstr* __restrict__ pc = prog + frag_start[blockIdx.y];
  MAcc<S> acc;
  int cnt;
  eval_node_m<S, PF, 0, DM, SCALE, DIRECT>(a, pc, pmatsT, m, c, g, lr, lc, p, acc, cnt);
  const TInstr in = fetch_instr(pc);  // T_ROOT
  if (SCALE) rescale_m<S>(acc, cnt, xch, a.C, c, g, lr, lc);
  if (in.a >= 0) store_partial_m<S, SCALE>(a, in.a, p, c, acc, cnt, lr);
  if (in.b) {
    // l_c = sum_x L[c][x] pi_x over the lane's states, then over the 4 lanes of the pattern
    double s = 0.0;
#pragma unroll
    for (int xt = 0; xt < XT; ++xt)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (m_valid<S>(xt, r, lr)) {
          const double li = acc[xt][r] * a.pi[16 * xt + lr + 4 * r];
          if (a.guard) {
            if (li > 0.0) s += li;
          } else {
            s += li;
          }
        }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    const double t = s * a.probs[c];
    __syncthreads();
    if (lr == 0) xch[(c * kTreeMGroups + g) * 16 + lc] = t;
    __syncthreads();
    if (c == 0 && lr == 0) {
      double l = 0.0;
      for (int k = 0; k < a.C; ++k) {
        const double li = xch[(k * kTreeMGroups + g) * 16 + lc];
        if (a.guard) {
          if (li > 0.0) l += li;
        } else {
          l += li;
        }
      }
      if (!a.guard && l < 0.0) l = 0.0;
      double rr = log(l);
      if (SCALE) rr -= (double)cnt * kLn2x256;
      double wr = 0.0;
      if (p < a.n_patterns) {
        if (a.uflow && !(l >= 2.0 * kScaleThr)) *a.uflow = 1;  // plk_root_underflow
        a.site_lnl[p] = rr;
        wr = a.weights[p] * rr;
      }
      red[16 * g + lc] = wr;
    }
    __syncthreads();
    if (G == kTreeMGroups && w == 0) {
      // the 64 patterns of the workgroup in root_kernel's butterfly order
      double wr = red[lane];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) wr += __shfl_xor(wr, off, 64);
      if (lane == 0) a.wave_sums[p0 >> 6] = wr;
    }
  }
}

// wave_sums[k] = fixed butterfly over patterns 64k .. 64k + 63 of weights[p] * site_lnl[p]
// (0 beyond n_patterns): what treeM_kernel<.., 4> forms in its root fragment.
__global__ __launch_bounds__(256) void site_wave_sums_kernel(const double* __restrict__ site_lnl,
                                                             const double* __restrict__ weights, double* __restrict__ wave_sums,
                                                             int64_t n_patterns, int64_t n_pad) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pad) return;  // n_pad is a multiple of 256: whole waves only
  double wr = p < n_patterns ? weights[p] * site_lnl[p] : 0.0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) wr += __shfl_xor(wr, off, 64);
  if ((threadIdx.x & 63) == 0) wave_sums[p >> 6] = wr;
}

// P^T copy: PT[b][c][y][x] = P[b][c][x][y]  (grid: nodes x classes)
template <int S>
__global__ void transpose_pmats(const double* __restrict__ P, double* __restrict__ PT, int C) {
  const int b = blockIdx.x;
  const int c = blockIdx.y;
  const size_t off = ((size_t)b * C + c) * S * S;
  for (int e = threadIdx.x; e < S * S; e += blockDim.x) {
    const int y = e / S, x = e % S;
    PT[off + e] = P[off + (size_t)x * S + y];
  }
}

}  // namespace plk
