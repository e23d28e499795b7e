// plk_tree4.hpp -- fused postorder traversal for 4-state models (gfx950).
//
// A workgroup owns 64 consecutive site patterns (one per lane) and C/CW waves: wave
// w evaluates rate classes [w*CW, (w+1)*CW) for those patterns.  Every wave walks
// the same small "tree program" (postorder events, wave-uniform, fetched one word
// ahead with scalar loads) and keeps the pending product of every open ancestor in
// registers: level d of the current root-to-node path owns acc[d][CW*4].  Register
// indices are compile-time constants (the runtime level selects a template instance
// through a switch), so nothing spills, and the per-wave footprint is small enough
// for several waves per SIMD to hide the scalar-load and LDS latencies.  A child's
// contribution is multiplied into its parent's level as soon as the child completes,
// in the reference's son order:
//     L_node[c][x] = prod_son sum_y P_son[c][x][y] L_son[c][y]
// (Likelihood/RHomogeneousTreeLikelihood.cpp:839-861).
//
// Compared with one launch per tree level (partials_s4_kernel) child partials are
// never re-read from HBM: a materialising traversal only WRITES each internal
// partial once, an lnL-only traversal writes nothing but fragment roots.  Tips enter
// as uint8 codes (staged in LDS) through the getInitValue table, which covers
// ambiguity codes exactly like the reference's dense leaf vectors.  Power-of-two
// rescaling uses the max over ALL classes of a pattern (waves exchange their maxima
// through LDS), i.e. the same rule as the levelwise kernels and the oracle.  The
// root reduction (RHomogeneousTreeLikelihood.cpp:162-216) is fused into ROOT.
#pragma once

#include "plk_kernels.hpp"

namespace plk {

enum TreeOp : int32_t { T_TIP = 1, T_LOAD = 2, T_DESCEND = 3, T_ASCEND = 4, T_ROOT = 5, T_CHERRY = 6 };

// 16-byte program word: wave-uniform, fetched with s_load_dwordx4.
// Per node: its child events in son order -- TIP / LOAD / DESCEND (followed by the
// child's own events) -- then ASCEND.  A fragment ends with ROOT.
struct TInstr {
  int32_t op;
  int32_t d;  // register level (informational)
  int32_t a;  // TIP: tip index; LOAD: internal slot; ASCEND/ROOT: store slot or -1; CHERRY: cherry index
  int32_t b;  // TIP/LOAD/ASCEND/CHERRY: branch (node index of the child; -1 for a fragment root); ROOT: 1 = reduce lnL
};
// T_CHERRY (treeM only): an unstored cherry contributes one row of its precomputed
// contribution table (plk_treeM.hpp: cherry_table_kernel), selected by its tips' codes.

struct TreeArgs {
  const TInstr* prog;
  const int32_t* frag_start;  // program offset of each fragment (blockIdx.y)
  double* partials;           // [n_internal][slot_stride]
  int32_t* scale;             // [n_internal][n_pad] (SCALE only)
  const uint8_t* codes;       // [n_tips][n_pad]
  const double* pmats;        // [n_nodes][C][4][4]
  const double* init;         // [n_codes][4]
  const double* tipP;         // [n_tips][C][n_codes][S] (S > 4 kernels)
  const double* weights;      // [n_pad]
  const double* pi;           // [4]
  const double* probs;        // [C]
  double* site_lnl;           // [n_pad]
  double* wave_sums;          // [n_pad / 64]
  int64_t slot_stride;
  int64_t n_pad;
  int64_t n_patterns;
  int32_t n_codes;
  int32_t n_tips;
  int32_t C;
  int32_t guard;
  int32_t stage_codes;        // 1: tip codes staged in LDS
  int32_t n_frags;            // fragments of the program (frag_start[n_frags + f] = first table, treeM)
  int32_t buf_doubles;        // treeM: doubles per LDS table buffer
  int32_t bmask;              // -1 (timing experiments: 0 = every branch reads P of node 0)
  const uint8_t* cherry;      // treeM: per cherry [table | counts | codes] (plk_treeM.hpp: CherryLayout)
  int32_t cherry_pairs;       // treeM: two consecutive T_CHERRY rows gathered together
  int32_t n_cherry_staged;    // treeM: cherries whose combined codes are staged in LDS (0: none)
  int32_t* uflow;             // unscaled handles: set to 1 when a site likelihood is < 2^-255 (or null)
};

constexpr int kTreeMaxWaves = 4;

// Program words are wave-uniform and read-only for the whole launch: read them through
// the constant address space so that they always come in with s_load (scalar cache,
// SGPR result).  Through a generic pointer the compiler may pick a vector load for a
// field it then branches on, which puts a full vector-memory round trip (and a
// vmcnt(0) drain of every outstanding partial load) on every tree event.
// The address itself is made provably uniform with readfirstlane (a no-op when the
// pointer already lives in SGPRs): the nested per-level loops otherwise let the
// divergence analysis treat the program counter as divergent.
typedef __attribute__((address_space(4))) const TInstr* ConstProg;
__device__ __forceinline__ TInstr fetch_instr(const TInstr* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  const ConstProg q = reinterpret_cast<ConstProg>(((uint64_t)hi << 32) | lo);
  TInstr r;
  r.op = q->op;
  r.d = q->d;
  r.a = q->a;
  r.b = q->b;
  return r;
}

// dst[c][x] *= sum_y P[c][x][y] * src[c][y]   (P = this wave's classes, 16 doubles each)
template <int CW>
__device__ __forceinline__ void contribute(double (&dst)[CW * 4], const double (&src)[CW * 4],
                                           const double* __restrict__ P) {
#pragma unroll
  for (int c = 0; c < CW; ++c) {
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

// Joint (all-class) exact power-of-two rescaling of one pattern's partial.
template <int CW>
__device__ __forceinline__ void rescale(double (&v)[CW * 4], int& cnt, double* xmax, int nw) {
  double m = 0.0;
#pragma unroll
  for (int i = 0; i < CW * 4; ++i) m = fmax(m, v[i]);
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
    for (int i = 0; i < CW * 4; ++i) v[i] *= kScaleUp;
    cnt += 1;
  }
}

template <int CW, bool SCALE>
__device__ __forceinline__ void store_partial(const TreeArgs& a, int slot, int64_t p, int c0,
                                              const double (&v)[CW * 4], int cnt) {
  const int64_t tile = p >> 7, q = p & (kTile - 1);
  double* dst = a.partials + (size_t)slot * a.slot_stride + tile * ((int64_t)a.C * 4 * kTile) + (size_t)c0 * 4 * kTile + q;
#pragma unroll
  for (int i = 0; i < CW * 4; ++i) __builtin_nontemporal_store(v[i], dst + (size_t)i * kTile);
  if (SCALE && c0 == 0) a.scale[(size_t)slot * a.n_pad + p] = cnt;
}

// Evaluate one node at register level D: consume its child events until ASCEND.
// Each level is its own inlined loop with its own accumulator, so the ancestors'
// products stay in fixed registers without any phi copies.
template <int CW, int D, int DM, bool SCALE>
__device__ __forceinline__ void eval_node(const TreeArgs& a, const TInstr* __restrict__& pc,
                                          const double* __restrict__ pmats, const double* init_lds,
                                          const uint8_t* code_lds, double* xch, int nw, int c0, int64_t p,
                                          double (&acc)[CW * 4], int& cnt) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < CW * 4; ++i) acc[i] = 1.0;
  cnt = 0;
  for (;;) {
    const TInstr in = fetch_instr(pc++);
    if (in.op == T_ASCEND) {
      // node complete: rescale, optionally store (its parent contributes it)
      if (in.b >= 0) {
        if (SCALE) rescale<CW>(acc, cnt, xch, nw);
        if (in.a >= 0) store_partial<CW, SCALE>(a, in.a, p, c0, acc, cnt);
      }
      return;
    }
    const double* __restrict__ P = pmats + ((size_t)(in.b & a.bmask) * a.C + c0) * 16;
    if (in.op == T_TIP) {
      const int code = a.stage_codes ? code_lds[in.a * 64 + lane] : a.codes[(size_t)in.a * a.n_pad + p];
      const double2* iv = reinterpret_cast<const double2*>(init_lds + code * 4);
      const double2 i01 = iv[0], i23 = iv[1];
      double src[CW * 4];
#pragma unroll
      for (int c = 0; c < CW; ++c) {
        src[c * 4 + 0] = i01.x;
        src[c * 4 + 1] = i01.y;
        src[c * 4 + 2] = i23.x;
        src[c * 4 + 3] = i23.y;
      }
      contribute<CW>(acc, src, P);
    } else if (in.op == T_LOAD) {
      const int64_t tile = p >> 7, q = p & (kTile - 1);
      const double* L = a.partials + (size_t)in.a * a.slot_stride + tile * ((int64_t)a.C * 4 * kTile) +
                        (size_t)c0 * 4 * kTile + q;
      double src[CW * 4];
#pragma unroll
      for (int i = 0; i < CW * 4; ++i) src[i] = L[(size_t)i * kTile];
      if (SCALE) cnt += a.scale[(size_t)in.a * a.n_pad + p];
      contribute<CW>(acc, src, P);
    } else {  // T_DESCEND: an internal child evaluated one register level down
      if constexpr (D + 1 < DM) {
        double child[CW * 4];
        int ccnt;
        eval_node<CW, D + 1, DM, SCALE>(a, pc, pmats, init_lds, code_lds, xch, nw, c0, p, child, ccnt);
        // the child's ASCEND word carried its branch; re-read it (uniform, cached)
        const TInstr up = fetch_instr(pc - 1);
        const double* __restrict__ Pc = pmats + ((size_t)(up.b & a.bmask) * a.C + c0) * 16;
        contribute<CW>(acc, child, Pc);
        if (SCALE) cnt += ccnt;
      }
    }
  }
}

// prog / frag_start / pmats are separate __restrict__ kernel arguments: the compiler
// can then prove they are never written in the kernel and fetches the wave-uniform
// program words and P(t) entries with scalar loads into SGPRs.
template <int CW, int DM, bool SCALE>
__global__ __launch_bounds__(256) void tree4_kernel(TreeArgs a, const TInstr* __restrict__ prog,
                                                    const int32_t* __restrict__ frag_start,
                                                    const double* __restrict__ pmats) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  // LDS: init table [n_codes][4] | class exchange [4][64] | codes [n_tips][64] (if staged)
  double* init_lds = lds;
  double* xch = lds + ((a.n_codes * 4 + 1) & ~1);
  uint8_t* code_lds = reinterpret_cast<uint8_t*>(xch + kTreeMaxWaves * 64);
  const int nw = blockDim.x >> 6;
  const int lane = threadIdx.x & 63;
  // wave index as a scalar: keeps P(t) addresses uniform -> s_load into SGPRs
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c0 = w * CW;
  const int64_t p0 = (int64_t)blockIdx.x * 64;
  const int64_t p = p0 + lane;
  for (int i = threadIdx.x; i < a.n_codes * 4; i += blockDim.x) init_lds[i] = a.init[i];
  if (a.stage_codes) {
    // 16 B per thread: tip t, bytes [16*j, 16*j + 16) of the 64-pattern row
    for (int i = threadIdx.x; i < a.n_tips * 4; i += blockDim.x) {
      const int t = i >> 2, j = i & 3;
      reinterpret_cast<uint4*>(code_lds)[i] =
          *reinterpret_cast<const uint4*>(a.codes + (size_t)t * a.n_pad + p0 + 16 * j);
    }
  }
  __syncthreads();

  const TInstr* __restrict__ pc = prog + frag_start[blockIdx.y];
  double acc[CW * 4];
  int cnt;
  eval_node<CW, 0, DM, SCALE>(a, pc, pmats, init_lds, code_lds, xch, nw, c0, p, acc, cnt);
  const TInstr in = fetch_instr(pc);  // T_ROOT
  // fragment root: rescale, optionally store, optionally reduce lnL
  if (SCALE) rescale<CW>(acc, cnt, xch, nw);
  if (in.a >= 0) store_partial<CW, SCALE>(a, in.a, p, c0, acc, cnt);
  if (in.b) {
    // per class: l_c = sum_s L[c][s] pi_s, t_c = l_c * prob_c  (guards: drop <= 0)
    double t[CW];
#pragma unroll
    for (int c = 0; c < CW; ++c) {
      double lc = 0.0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const double li = acc[c * 4 + s] * a.pi[s];
        if (a.guard) {
          if (li > 0.0) lc += li;
        } else {
          lc += li;
        }
      }
      t[c] = lc * a.probs[c0 + c];
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < CW; ++c) xch[(c0 + c) * 64 + lane] = t[c];  // C <= 4 classes fit in xch
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
        if (a.uflow && !(l >= 2.0 * kScaleThr)) *a.uflow = 1;  // plk_root_underflow
        a.site_lnl[p] = r;
        wr = a.weights[p] * r;
      }
      // fixed-order butterfly: the same summation order for every wave
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) wr += __shfl_xor(wr, off, 64);
      if (lane == 0) a.wave_sums[p0 >> 6] = wr;
    }
  }
}

// block_sums[b] = sum of the 64 wave sums of patterns [b*4096, (b+1)*4096), added in
// wave order.  One wave per block: the 64 loads are issued together (one per lane),
// then lane 0 adds them in order through shuffles, so the result is the plain
// sequential sum without 64 dependent memory round trips.
// Under a communicator flag_out is the underflow slot of this rank's exchange record
// (plk_exchange.hpp): the root reduction's flag travels in the same all-gather.
__global__ __launch_bounds__(256) void wave_sums_to_blocks(const double* __restrict__ wave_sums,
                                                           double* __restrict__ block_sums, int n_waves,
                                                           int n_blocks, const int32_t* uflow,
                                                           double* __restrict__ flag_out) {
  const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (flag_out && b == 0 && lane == 0)
    *flag_out = __hip_atomic_load(uflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ? 1.0 : 0.0;
  if (b >= n_blocks) return;
  const int w = b * (kRootBlock / 64) + lane;
  const double v = w < n_waves ? wave_sums[w] : 0.0;
  // the chain of adds in wave order (operands by shuffle; a v_readlane form measured slower:
  // 5.4-5.9 vs 4.2-4.4 us, its SGPR results need wait states before every add)
  double s = 0.0;
  for (int k = 0; k < kRootBlock / 64; ++k) {
    const double x = __shfl(v, k, 64);
    if (b * (kRootBlock / 64) + k < n_waves) s += x;
  }
  if (lane == 0) block_sums[b] = s;
}

}  // namespace plk
