// plk_jitm.hpp -- tree-specialised fused traversal for 20-state (protein) models on
// v_mfma_f64_4x4x4_4b (gfx950).
//
// Why a second matrix-core layout.  treeM_kernel (plk_treeM.hpp) runs the contraction
//     D[x][p] = sum_y P[x][y] L[y][p]          (RHomogeneousTreeLikelihood.cpp:839-861)
// on v_mfma_f64_16x16x4: 20 states occupy two 16-row tiles, so 12 of every 32 rows are
// padding (37.5 % of the issued flops), and the instruction itself peaks at 72.9 TF/s.
// v_mfma_f64_4x4x4_4b -- four independent 4x4x4 blocks per instruction -- peaks at 77.9 TF/s
// on this part (99 % of the fp64 spec, profiles/r02/fp64_mfma_peak.txt) and tiles 20 states
// as 5 x 4 rows with no padding: 1.7x less matrix-pipe time per contraction.
//
// Layout (decoded on the device, profiles/r02/mfma_f64_4x4x4_layout.txt): lane
// l = 16*hi + 4*b + lo holds A_b[lo][hi], B_b[hi][lo] and D_b[hi][lo].  A wave owns 16
// site patterns -- pattern 4b + lo of its group -- and EVERY rate class; lane l keeps the
// states x = 4X + hi (X = 0..4) of its pattern for each class, i.e. D of x-block X.  That
// register is exactly the B operand of y-block Y = X of the parent's contraction, so a
// child feeds its parent straight from registers.  The A operand of block (X, Y) is
// P[4X + lo][4Y + hi] -- pattern-independent, one 16-double tile per (class, X, Y) in LDS,
// read with ds_read_b64 at a constant offset from one lane base (the 4 blocks of a lane
// group broadcast).  P(t) is staged in LDS as stored, [c][x][y]: lane (hi, lo) reads row
// 4X + lo, column 4Y + hi, so a 32-lane group reads rows lo = 0..3 at columns hi = 0, 1 --
// 8 distinct doubles on 8 distinct bank pairs (conflict-free) -- and the staging is a
// plain copy whose ds_write_b64 groups store 16 consecutive doubles (conflict-free).
// SQ_LDS_BANK_CONFLICT on cfg3: 0 (round 2's 16-double tile image [c][X][Y][hi][lo]: 4-way
// conflicted stores, 43 M conflict cycles per launch, 3.60 vs 3.43 ms; profiles/r03).
//
// All classes in one wave: the joint (all states, all classes) exact power-of-two
// rescale of the other kernels is an in-register max plus two shuffles -- no LDS exchange
// and no barrier per node (treeM_kernel's one-class-per-wave layout needs two per node).
//
// Per tree: the fragment programs of build_tree4_program (cherries as T_CHERRY rows of
// the contribution tables built by cherry_table_kernel) are emitted as straight-line HIP
// -- constant branch / cherry / slot offsets, no program decode -- and compiled once per
// (program, shape) with hiprtc.  The P(t) of the next contributing branch is loaded into
// registers while the current contraction runs and written to the other LDS buffer
// behind one workgroup barrier; operands of later events (cherry rows, tip rows, child
// partials from HBM) are fetched L events ahead.
//
// Results are not bitwise those of treeM_kernel (the dot products group their terms in
// 4-term MFMA blocks instead of 16x16 tiles); the traversal is checked against the oracle
// at 1e-12 per pattern, and lnL-only vs materialising runs of this kernel are bitwise
// identical (same program, same operations).
#pragma once

#include <algorithm>
#include <string>
#include <vector>

#include "plk_tree4.hpp"
#include "plk_treeM.hpp"

namespace plk {

static const char* kJitMPrelude = R"PLKJITM(
typedef unsigned char u8;
typedef unsigned short u16;
typedef long long i64;
typedef int i32;
#define kTile 128
#define kLn2x256 177.44567822334599921
#define kScaleUp 115792089237316195423570985008687907853269984665640564039457584007913129639936.0
#define kScaleThr (1.0 / kScaleUp)

struct JMArgs {
  double* partials; i32* scale; const u8* codes; const double* tipP; const u8* cherry; const double* pmats;
  const double* weights; const double* pi; const double* probs; double* site_lnl; double* wave_sums;
  i64 slot_stride; i64 n_pad; i64 n_patterns; i64 cherry_stride; i64 cherry_table_bytes; i64 cherry_count_bytes;
  i32 guard; i32* uflow;
};

__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
typedef double f64x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f64x4 mfma16(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
__device__ __attribute__((noinline)) double jitm_log(double x) { return log(x); }
// rescale decision from the doubles' high words (see plk_jit.hpp hiw / hi_decides)
#define kThrHi 0x2FF00000
__device__ __forceinline__ int hiw(double x) { return (int)(__double_as_longlong(x) >> 32); }
__device__ __forceinline__ bool hi_decides(int mh) { return mh > 0 && mh < 0x7FF00000; }
)PLKJITM";

// Host mirror of JMArgs (field order and types must match the prelude).
struct JMArgs {
  double* partials;
  int32_t* scale;
  const uint8_t* codes;
  const double* tipP;
  const uint8_t* cherry;
  const double* pmats;
  const double* weights;
  const double* pi;
  const double* probs;
  double* site_lnl;
  double* wave_sums;
  int64_t slot_stride;
  int64_t n_pad;
  int64_t n_patterns;
  int64_t cherry_stride;
  int64_t cherry_table_bytes;
  int64_t cherry_count_bytes;
  int32_t guard;
  int32_t* uflow;  // unscaled handles: set to 1 when a site likelihood is < 2^-255 (or null)
};

struct JitMShape {
  int S = 20;
  int C = 1;
  int U = 1;         // codes in use (rows of a tip table; cherry tables have U * U)
  bool scale = false;
  int L = 1;         // operand fetch lookahead (events)
  int minw = 2;      // __launch_bounds__ min waves per SIMD
  int pd = 1;        // P(t) staging prefetch distance (contractions ahead)
  int G = 4;         // waves (16-pattern groups) per workgroup: 64 patterns (4) or 128 (8)
  int lc = 3;        // two-stage fetch: codes lc events ahead, rows L ahead (0: one stage)
  int pipe = 1;      // contraction order: 0 = per output block, 1 = Y-outer with A read ahead,
                     // 2 = 1 with the read / MFMA groups pinned (sched_group_barrier)
  int pb() const { return C * S * S; }  // doubles of P(t) per branch (every class)
  // LDS buffer stride: pb() rounded up to whole staging rounds, so that every thread stores
  // unconditionally (a guarded last store is a divergent branch, and the wait-count pass
  // then drains every outstanding load, the operand prefetches included, before it)
  int pbs() const { const int nth = 64 * G; return (pb() + nth - 1) / nth * nth; }
  size_t lds_bytes() const { return (size_t)(2 * pbs() + 16 * G) * sizeof(double); }
  bool operator==(const JitMShape& o) const {
    return S == o.S && C == o.C && U == o.U && scale == o.scale && L == o.L && minw == o.minw && pd == o.pd &&
           G == o.G && pipe == o.pipe && lc == o.lc;
  }
};

// Emit the kernel for build_tree4_program's words `prog` and fragment start offsets
// `starts` (tier order; fragment id = frag_base + blockIdx.y).
inline std::string jit_treeM4_source(const std::vector<TInstr>& prog, const std::vector<int32_t>& starts,
                                     const JitMShape& sh) {
  const int S = sh.S, C = sh.C, XB = S / 4, L = std::max(sh.L, 1);
  std::string s;
  s.reserve(65536 * std::max<size_t>(starts.size(), 1));
  s += kJitMPrelude;
  const size_t pre_pos = s.size();  // per-fragment base tables go here (global scope)
  std::string pre_;
  char buf[512];
  const int NTH = 64 * sh.G, PB = sh.pb(), PF = (PB + NTH - 1) / NTH;
  snprintf(buf, sizeof(buf),
           "#define S_ %d\n#define C_ %d\n#define XB_ %d\n#define U_ %d\n#define U2_ %d\n#define G_ %d\n"
           "#define NTH_ %d\n#define PB_ %d\n#define PBS_ %d\n#define PF_ %d\n#define SC_ %s\n#define PIPE_ %d\n",
           S, C, XB, sh.U, sh.U * sh.U, sh.G, NTH, PB, sh.pbs(), PF, sh.scale ? "true" : "false", sh.pipe);
  s += buf;
  s += R"PLKJITM(
// P(t) of branch b (all classes, [c][x][y]) -> registers -> LDS buffer bf, as stored
#define PSTAGE_LOAD(R, b) { const double* s_ = a.pmats + (i64)(b) * PB_; \
  _Pragma("unroll") for (int j_ = 0; j_ < PF_; ++j_) { const int e_ = tid + j_ * NTH_; R[j_] = s_[e_ < PB_ ? e_ : PB_ - 1]; } }
#define PSTAGE_STORE(R, bf) { double* d_ = lds + (bf) * PBS_; \
  _Pragma("unroll") for (int j_ = 0; j_ < PF_; ++j_) d_[tid + j_ * NTH_] = R[j_]; }
// D[c][X] (*)= sum_Y A(c, X, Y) . SRC[c][Y]   (SET: D was 1); lane (hi, lo) reads
// A(c, X, Y)[lo][hi] = P_c[4X + lo][4Y + hi] at a constant offset from its lane base PA
#if PIPE_ == 0
#define CONTRIB(D, SRC, bf, SET) { \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) { \
    double d_ = 0.0; \
    _Pragma("unroll") for (int Y_ = 0; Y_ < XB_; ++Y_) \
      d_ = mfma4(PA[(bf) * PBS_ + (c_ * S_ + 4 * X_) * S_ + 4 * Y_], SRC[c_][Y_], d_); \
    if (SET) D[c_][X_] = d_; else D[c_][X_] *= d_; } }
#else
// the same sums (each output block accumulates Y = 0..4 in order, so results are bitwise
// those of PIPE_ 0), issued Y-outer: the five output blocks' MFMAs are independent of each
// other, and the A operands of step Y + 1 are read from LDS while step Y's MFMAs run
#define CONTRIB(D, SRC, bf, SET) { \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) { \
    const double* pa_ = PA + (bf) * PBS_ + c_ * S_ * S_; \
    double acc_[XB_], an_[XB_]; \
    _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) an_[X_] = pa_[4 * X_ * S_]; \
    _Pragma("unroll") for (int Y_ = 0; Y_ < XB_; ++Y_) { \
      double ac_[XB_]; \
      _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) ac_[X_] = an_[X_]; \
      if (Y_ + 1 < XB_) { _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) an_[X_] = pa_[4 * X_ * S_ + 4 * (Y_ + 1)]; } \
      _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) acc_[X_] = mfma4(ac_[X_], SRC[c_][Y_], Y_ ? acc_[X_] : 0.0); \
      PIPE_GROUPS(Y_) \
    } \
    _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) { if (SET) D[c_][X_] = acc_[X_]; else D[c_][X_] *= acc_[X_]; } } }
#if PIPE_ == 2
#define PIPE_GROUPS(Y) { if ((Y) + 1 < XB_) __builtin_amdgcn_sched_group_barrier(0x100, XB_, 0); \
  __builtin_amdgcn_sched_group_barrier(0x008, XB_, 0); }
#else
#define PIPE_GROUPS(Y)
#endif
#endif
#define ROWMUL(D, F, SET) { _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") \
  for (int X_ = 0; X_ < XB_; ++X_) { if (SET) D[c_][X_] = F[c_][X_]; else D[c_][X_] *= F[c_][X_]; } }
// one row of cherry k's contribution table (combined code of the pattern's two tips)
#define CHERRY_FETCH(F, FK, k) { const u8* base_ = a.cherry + (i64)(k) * a.cherry_stride; \
  const int code_ = reinterpret_cast<const u16*>(base_ + a.cherry_table_bytes + a.cherry_count_bytes)[p]; \
  const double* r_ = reinterpret_cast<const double*>(base_) + (i64)code_ * S_ + hi; \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) \
    F[c_][X_] = r_[(i64)c_ * (U2_ * S_) + 4 * X_]; \
  if (SC_) FK = (int)base_[a.cherry_table_bytes + code_]; }
// two-stage operand fetch (JitMShape::lc > 0): a table row's code is loaded lc events
// ahead (CHERRY_CODE / TIP_CODE, one VGPR), its row L events ahead from that code -- so no
// row load waits on a code load issued just before it (vmcnt counts in issue order: such a
// wait also drains every load issued earlier, the P(t) staging of the contraction included)
#define CHERRY_CODE(Q, k) { Q = reinterpret_cast<const u16*>(a.cherry + (i64)(k) * a.cherry_stride + \
  a.cherry_table_bytes + a.cherry_count_bytes)[p]; }
#define CHERRY_ROW(F, FK, k, Q) { const u8* base_ = a.cherry + (i64)(k) * a.cherry_stride; \
  const double* r_ = reinterpret_cast<const double*>(base_) + (i64)(Q) * S_ + hi; \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) \
    F[c_][X_] = r_[(i64)c_ * (U2_ * S_) + 4 * X_]; \
  if (SC_) FK = (int)base_[a.cherry_table_bytes + (Q)]; }
#define TIP_CODE(Q, t) { Q = a.codes[(i64)(t) * a.n_pad + p]; }
#define TIP_ROW(F, t, Q) { const double* r_ = a.tipP + ((i64)(t) * (C_ * U_) + (Q)) * S_ + hi; \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) \
    F[c_][X_] = r_[(i64)c_ * (U_ * S_) + 4 * X_]; }
#define TIP_FETCH(F, t) { const int code_ = a.codes[(i64)(t) * a.n_pad + p]; \
  const double* r_ = a.tipP + ((i64)(t) * (C_ * U_) + code_) * S_ + hi; \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) \
    F[c_][X_] = r_[(i64)c_ * (U_ * S_) + 4 * X_]; }
#define LOAD_FETCH(F, FK, slot) { const double* L_ = a.partials + (i64)(slot) * a.slot_stride + toff; \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) \
    F[c_][X_] = L_[(i64)(c_ * S_ + 4 * X_) * kTile]; \
  if (SC_) FK = a.scale[(i64)(slot) * a.n_pad + p]; }
#define STORE(V, K, slot) { double* D_ = a.partials + (i64)(slot) * a.slot_stride + toff; \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) \
    __builtin_nontemporal_store(V[c_][X_], D_ + (i64)(c_ * S_ + 4 * X_) * kTile); \
  if (SC_ && hi == 0) a.scale[(i64)(slot) * a.n_pad + p] = K; }
// joint exact power-of-two rescale of the pattern (its states sit in lanes hi = 0..3)
// (the hi-word max is the same in the four lanes of a pattern, so a fallback to the f64
// max runs with all four active)
#define RESCALE(V, K) { int mh_ = 0; bool up_; \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) mh_ = max(mh_, hiw(V[c_][X_])); \
  mh_ = max(mh_, __shfl_xor(mh_, 16, 64)); mh_ = max(mh_, __shfl_xor(mh_, 32, 64)); \
  if (__builtin_expect(hi_decides(mh_), 1)) { up_ = mh_ < kThrHi; } else { double m_ = 0.0; \
    _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) m_ = fmax(m_, V[c_][X_]); \
    m_ = fmax(m_, __shfl_xor(m_, 16, 64)); m_ = fmax(m_, __shfl_xor(m_, 32, 64)); \
    up_ = m_ > 0.0 && m_ < kScaleThr; } \
  if (up_) { \
    _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) V[c_][X_] *= kScaleUp; \
    K += 1; } }
// root reduction (RHomogeneousTreeLikelihood.cpp:162-216 / NH :168-233) and the fixed
// butterfly over each 64 patterns of the workgroup (root_kernel's order)
#define REDUCE_ROOT(V, K) { double l_ = 0.0; \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) { double s_ = 0.0; \
    _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) { const double li_ = V[c_][X_] * a.pi[4 * X_ + hi]; \
      if (a.guard) { if (li_ > 0.0) s_ += li_; } else { s_ += li_; } } \
    s_ += __shfl_xor(s_, 16, 64); s_ += __shfl_xor(s_, 32, 64); \
    const double t_ = s_ * a.probs[c_]; \
    if (a.guard) { if (t_ > 0.0) l_ += t_; } else { l_ += t_; } } \
  if (!a.guard && l_ < 0.0) l_ = 0.0; \
  double rr_ = jitm_log(l_); \
  if (SC_) rr_ -= (double)K * kLn2x256; \
  double wr_ = 0.0; \
  if (p < a.n_patterns) { if (hi == 0) a.site_lnl[p] = rr_; wr_ = a.weights[p] * rr_; \
    if (a.uflow && hi == 0 && !(l_ >= 2.0 * kScaleThr)) *a.uflow = 1; } \
  if (hi == 0) red[16 * w + pl] = wr_; \
  __syncthreads(); \
  if (w < G_ / 4) { double v_ = red[64 * w + lane]; \
    _Pragma("unroll") for (int off_ = 32; off_ > 0; off_ >>= 1) v_ += __shfl_xor(v_, off_, 64); \
    if (lane == 0) a.wave_sums[(p0 >> 6) + w] = v_; } }
#define SB __builtin_amdgcn_sched_barrier(0);
)PLKJITM";
  snprintf(buf, sizeof(buf),
           "extern \"C\" __global__ __launch_bounds__(%d, %d) void plk_jit_treeM(JMArgs a, int frag_base) {\n", NTH,
           std::max(sh.minw, 1));
  s += buf;
  s += R"PLKJITM(  extern __shared__ __attribute__((aligned(16))) double lds[];  // [2][PBS_] P(t) | red[16 G_]
  double* red = lds + 2 * PBS_;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 4, pl = lane & 15;
  const i64 p0 = (i64)blockIdx.x * (16 * G_);
  const i64 p = p0 + 16 * w + pl;
  const i64 toff = (p >> 7) * (i64)(C_ * S_ * kTile) + (p & (kTile - 1)) + (i64)hi * kTile;
  // A-operand lane base: lane 16 hi + 4 b + lo reads row lo, column hi of a 4x4 block
  const double* PA = lds + (lane & 3) * S_ + hi;
  double R0[PF_] = {}, R1[PF_] = {}, R2[PF_] = {};
  (void)red; (void)PA; (void)R0; (void)R1; (void)R2; (void)toff;
  const int frag = frag_base + (int)blockIdx.y;
)PLKJITM";
  // accumulators per register level and the operand ring
  int max_level = 0;
  for (size_t f = 0; f < starts.size(); ++f) {
    int d = 0;
    for (size_t i = (size_t)starts[f]; prog[i].op != T_ROOT; ++i) {
      if (prog[i].op == T_DESCEND) max_level = std::max(max_level, ++d);
      if (prog[i].op == T_ASCEND) --d;
    }
  }
  for (int d = 0; d <= max_level; ++d) {
    snprintf(buf, sizeof(buf), "  double A%d[C_][XB_]; int K%d = 0; (void)K%d;\n", d, d, d);
    s += buf;
  }
  for (int r = 0; r <= L; ++r) {
    snprintf(buf, sizeof(buf), "  double F%d[C_][XB_]; int FK%d = 0; (void)FK%d;\n", r, r, r);
    s += buf;
  }
  // code lookahead and code ring: the prologue loads the codes of fetchers 0 .. LC - 1
  // before the first row, so the ring needs LC slots (LC - L + 1 suffice in steady state)
  const int LC = sh.lc > L ? sh.lc : 0, NQ = LC;
  for (int q = 0; q < NQ; ++q) {
    snprintf(buf, sizeof(buf), "  int QC%d = 0; (void)QC%d;\n", q, q);
    s += buf;
  }
  // Fragments of one shape share one case (a balanced tree's subtrees): per fragment a node
  // base (P(t) of its branches), a slot base (loads / stores), a tip base and a cherry base,
  // and the shared code's offsets relative to them (plk_jit.hpp does the same).
  const size_t NFR = starts.size();
  std::vector<int> nbase(NFR, 0), sbase(NFR, 0), tbase(NFR, 0), kbase(NFR, 0), leader(NFR, -1);
  {
    std::vector<std::string> sig(NFR);
    for (size_t f = 0; f < NFR; ++f) {
      int nb = 1 << 30, sb = 1 << 30, tb = 1 << 30, kb = 1 << 30;
      for (size_t i = (size_t)starts[f];; ++i) {
        const TInstr& e = prog[i];
        if ((e.op == T_LOAD || e.op == T_ASCEND) && e.b >= 0) nb = std::min(nb, (int)e.b);
        if ((e.op == T_LOAD || e.op == T_ASCEND || e.op == T_ROOT) && e.a >= 0) sb = std::min(sb, (int)e.a);
        if (e.op == T_TIP) tb = std::min(tb, (int)e.a);
        if (e.op == T_CHERRY) kb = std::min(kb, (int)e.a);
        if (e.op == T_ROOT) break;
      }
      nbase[f] = nb == (1 << 30) ? 0 : nb;
      sbase[f] = sb == (1 << 30) ? 0 : sb;
      tbase[f] = tb == (1 << 30) ? 0 : tb;
      kbase[f] = kb == (1 << 30) ? 0 : kb;
      std::string& g = sig[f];
      for (size_t i = (size_t)starts[f];; ++i) {
        const TInstr& e = prog[i];
        int ra = -1, rb = -1;
        if (e.op == T_TIP) ra = e.a - tbase[f];
        if (e.op == T_CHERRY) ra = e.a - kbase[f];
        if ((e.op == T_LOAD || e.op == T_ASCEND || e.op == T_ROOT) && e.a >= 0) ra = e.a - sbase[f];
        if ((e.op == T_LOAD || e.op == T_ASCEND) && e.b >= 0) rb = e.b - nbase[f];
        if (e.op == T_ROOT) rb = e.b;
        snprintf(buf, sizeof(buf), "%d,%d,%d;", (int)e.op, ra, rb);
        g += buf;
        if (e.op == T_ROOT) break;
      }
      for (size_t q = 0; q < f && leader[f] < 0; ++q)
        if (leader[q] == (int)q && sig[q] == g) leader[f] = (int)q;
      if (leader[f] < 0) leader[f] = (int)f;
    }
    const char* names[4] = {"kFragNB", "kFragSB", "kFragTB", "kFragKB"};
    const std::vector<int>* vals[4] = {&nbase, &sbase, &tbase, &kbase};
    for (int t = 0; t < 4; ++t) {
      std::string arr = std::string("__device__ const int ") + names[t] + "[] = {0";
      for (size_t f = 0; f < NFR; ++f) {
        snprintf(buf, sizeof(buf), ",%d", (*vals[t])[f]);
        arr += buf;
      }
      pre_ += arr + "};\n";
    }
  }
  s += "  switch (frag) {\n";
  for (size_t f = 0; f < starts.size(); ++f) {
    if (leader[f] != (int)f) continue;
    std::vector<TInstr> ev;
    for (size_t i = (size_t)starts[f];; ++i) {
      ev.push_back(prog[i]);
      if (prog[i].op == T_ROOT) break;
    }
    auto rel = [&](const char* base, int v, int b0) -> std::string {
      return std::string(base) + " + " + std::to_string(v - b0);
    };
    // operand fetchers (ring slots) and the P chain (events that contract through a branch)
    std::vector<int> slot(ev.size(), -1), fetchers, pchain;
    for (size_t i = 0; i < ev.size(); ++i) {
      const int op = ev[i].op;
      if (op == T_CHERRY || op == T_TIP || op == T_LOAD) {
        slot[i] = (int)(fetchers.size() % (size_t)(L + 1));
        fetchers.push_back((int)i);
      }
      if (op == T_LOAD || (op == T_ASCEND && ev[i].b >= 0)) pchain.push_back((int)i);
    }
    // two-stage: fetcher m's code at fetcher m - LC's event, its row at fetcher m - L's
    auto emit_code = [&](size_t m) {
      if (!LC || m >= fetchers.size()) return;
      const TInstr& e = ev[(size_t)fetchers[m]];
      const int q = (int)(m % (size_t)NQ);
      if (e.op == T_CHERRY)
        snprintf(buf, sizeof(buf), "    CHERRY_CODE(QC%d, %s)\n", q, rel("kb_", e.a, kbase[f]).c_str());
      else if (e.op == T_TIP)
        snprintf(buf, sizeof(buf), "    TIP_CODE(QC%d, %s)\n", q, rel("tb_", e.a, tbase[f]).c_str());
      else
        return;
      s += buf;
    };
    auto emit_row = [&](size_t m) {
      if (m >= fetchers.size()) return;
      const TInstr& e = ev[(size_t)fetchers[m]];
      const int sl = slot[(size_t)fetchers[m]], q = (int)(m % (size_t)NQ);
      if (e.op == T_CHERRY)
        snprintf(buf, sizeof(buf), "    CHERRY_ROW(F%d, FK%d, %s, QC%d)\n", sl, sl, rel("kb_", e.a, kbase[f]).c_str(), q);
      else if (e.op == T_TIP)
        snprintf(buf, sizeof(buf), "    TIP_ROW(F%d, %s, QC%d)\n", sl, rel("tb_", e.a, tbase[f]).c_str(), q);
      else
        snprintf(buf, sizeof(buf), "    LOAD_FETCH(F%d, FK%d, %s)\n", sl, sl, rel("sb_", e.a, sbase[f]).c_str());
      s += buf;
    };
    auto emit_fetch = [&](int i) {
      const TInstr& e = ev[(size_t)i];
      const int sl = slot[(size_t)i];
      if (e.op == T_CHERRY)
        snprintf(buf, sizeof(buf), "    CHERRY_FETCH(F%d, FK%d, %s)\n", sl, sl, rel("kb_", e.a, kbase[f]).c_str());
      else if (e.op == T_TIP)
        snprintf(buf, sizeof(buf), "    TIP_FETCH(F%d, %s)\n", sl, rel("tb_", e.a, tbase[f]).c_str());
      else
        snprintf(buf, sizeof(buf), "    LOAD_FETCH(F%d, FK%d, %s)\n", sl, sl, rel("sb_", e.a, sbase[f]).c_str());
      s += buf;
    };
    for (size_t q = f; q < NFR; ++q)
      if (leader[q] == (int)f) {
        snprintf(buf, sizeof(buf), "  case %zu:\n", q);
        s += buf;
      }
    s += "  {\n    const int nb_ = __builtin_amdgcn_readfirstlane(kFragNB[frag + 1]), sb_ = "
         "__builtin_amdgcn_readfirstlane(kFragSB[frag + 1]);\n    const int tb_ = "
         "__builtin_amdgcn_readfirstlane(kFragTB[frag + 1]), kb_ = __builtin_amdgcn_readfirstlane(kFragKB[frag + 1]);\n"
         "    (void)nb_; (void)sb_; (void)tb_; (void)kb_;\n";
    size_t nf = 0;
    if (LC) {
      for (size_t m = 0; m < (size_t)LC; ++m) emit_code(m);
      for (size_t m = 0; m < (size_t)L; ++m) emit_row(m);
    } else {
      for (; nf < fetchers.size() && nf < (size_t)L; ++nf) emit_fetch(fetchers[nf]);
    }
    size_t nfetch = 0;  // fetchers consumed (two-stage)
    int cur = 0;
    size_t np = 0;  // P-chain events consumed
    const int PD = std::min(std::max(sh.pd, 1), 3);
    // chain event j is staged from register set j % PD: loaded PD contractions ahead, stored
    // to the other LDS buffer (and a barrier) at the end of the contraction before its own
    const char* bar = " __syncthreads();";
    auto pload = [&](size_t j) {
      if (j < pchain.size()) {
        snprintf(buf, sizeof(buf), "    PSTAGE_LOAD(R%zu, %s)\n", j % (size_t)PD,
                 rel("nb_", ev[(size_t)pchain[j]].b, nbase[f]).c_str());
        s += buf;
      }
    };
    if (!pchain.empty()) {
      pload(0);
      s += "    PSTAGE_STORE(R0, 0) __syncthreads();\n";
      for (size_t j = 1; j <= (size_t)PD; ++j) pload(j);
    }
    // after chain event np's contraction: hand the next one's P(t) over, refill the set
    auto pnext = [&]() {
      if (np + 1 < pchain.size()) {
        snprintf(buf, sizeof(buf), "    PSTAGE_STORE(R%zu, %d)%s\n", (np + 1) % (size_t)PD, cur ^ 1, bar);
        s += buf;
        cur ^= 1;
        pload(np + 1 + (size_t)PD);
      }
      ++np;
    };
    s += "    SB\n";
    std::vector<char> fresh((size_t)max_level + 2, 0);
    fresh[0] = 1;
    int d = 0;
    for (size_t i = 0; i < ev.size(); ++i) {
      const TInstr& e = ev[i];
      if (e.op == T_CHERRY || e.op == T_TIP || e.op == T_LOAD) {
        if (LC) {
          emit_code(nfetch + (size_t)LC);
          emit_row(nfetch + (size_t)L);
          ++nfetch;
        } else if (nf < fetchers.size()) {
          emit_fetch(fetchers[nf++]);
        }
        const int sl = slot[i];
        if (e.op == T_LOAD) {
          snprintf(buf, sizeof(buf), "    CONTRIB(A%d, F%d, %d, %s)\n", d, sl, cur, fresh[(size_t)d] ? "true" : "false");
          s += buf;
          pnext();
          if (sh.scale) {
            snprintf(buf, sizeof(buf), "    K%d += FK%d;\n", d, sl);
            s += buf;
          }
        } else {
          snprintf(buf, sizeof(buf), "    ROWMUL(A%d, F%d, %s)\n", d, sl, fresh[(size_t)d] ? "true" : "false");
          s += buf;
          if (e.op == T_CHERRY && sh.scale) {
            snprintf(buf, sizeof(buf), "    K%d += FK%d;\n", d, sl);
            s += buf;
          }
        }
        fresh[(size_t)d] = 0;
        s += "    SB\n";
      } else if (e.op == T_DESCEND) {
        ++d;
        fresh[(size_t)d] = 1;
        snprintf(buf, sizeof(buf), "    K%d = 0;\n", d);
        s += buf;
      } else if (e.op == T_ASCEND) {
        if (e.b < 0) continue;  // the fragment root: finished by ROOT
        if (sh.scale) {
          snprintf(buf, sizeof(buf), "    RESCALE(A%d, K%d)\n", d, d);
          s += buf;
        }
        if (e.a >= 0) {
          snprintf(buf, sizeof(buf), "    STORE(A%d, K%d, %s)\n", d, d, rel("sb_", e.a, sbase[f]).c_str());
          s += buf;
        }
        snprintf(buf, sizeof(buf), "    CONTRIB(A%d, A%d, %d, %s)\n", d - 1, d, cur, fresh[(size_t)d - 1] ? "true" : "false");
        s += buf;
        pnext();
        if (sh.scale) {
          snprintf(buf, sizeof(buf), "    K%d += K%d;\n", d - 1, d);
          s += buf;
        }
        fresh[(size_t)d - 1] = 0;
        --d;
        s += "    SB\n";
      } else {  // T_ROOT
        if (sh.scale) s += "    RESCALE(A0, K0)\n";
        if (e.a >= 0) {
          snprintf(buf, sizeof(buf), "    STORE(A0, K0, %s)\n", rel("sb_", e.a, sbase[f]).c_str());
          s += buf;
        }
        if (e.b) s += "    REDUCE_ROOT(A0, K0)\n";
      }
    }
    s += "  } break;\n";
  }
  s += "  default: break;\n  }\n}\n";
  s.insert(pre_pos, pre_);
  return s;
}

}  // namespace plk
