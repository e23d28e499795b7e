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
// read with ds_read_b64 at a constant offset (the 4 blocks of a lane group broadcast).
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
  i32 guard; i64 p_base;  // p_base: first pattern of the launch (pattern chunks)
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
  int64_t p_base;
};

struct JitMShape {
  int S = 20;
  int C = 1;
  int U = 1;         // codes in use (rows of a tip table; cherry tables have U * U)
  bool scale = false;
  int L = 1;         // operand fetch lookahead (events)
  int minw = 2;      // __launch_bounds__ min waves per SIMD
  bool direct = false;  // A operands straight from P(t) in L1/L2 (no LDS staging, no barriers)
  int pd = 1;           // P(t) staging prefetch distance (contractions ahead)
  bool hoist = false;   // cherry codes of the whole fragment loaded at its start
  bool youter = false;  // contraction order: independent chains interleaved block by block
  bool padstage = false; // P staging: padded LDS stride, unconditional stores (cfg3 3.93 vs 3.51 ms: off)
  int debug = 0;        // timing experiments only (wrong results): bit 1 no P(t) staging barrier, bit 2 no
                        // P(t) loads, bit 4 one A operand read per class and contraction
  bool hyb = false;     // 16-state tiles on 16x16x4, the rest on 4x4x4 (CONTRIB, HYB_; 20 and 64
                        // states; cfg3 4.37 vs 3.56 ms all-4x4x4, so off)
  bool hybrid() const { return hyb && (S == 20 || S == 64) && !direct; }
  int G = 4;  // waves (16-pattern groups) per workgroup: 64 patterns (4) or 128 (8)
  int pb() const { return C * S * S; }  // doubles of P(t) per branch (every class)
  // LDS stride of a P buffer: every staging element of the workgroup has a slot (the
  // elements past pb() land in the padding), so the staging stores need no condition
  int pbs() const { return padstage ? (pb() + 64 * G - 1) / (64 * G) * (64 * G) : pb(); }
  size_t lds_bytes() const { return (size_t)((direct ? 0 : 2 * pbs()) + 16 * G) * sizeof(double); }
  bool operator==(const JitMShape& o) const {
    return S == o.S && C == o.C && U == o.U && scale == o.scale && L == o.L && minw == o.minw && direct == o.direct &&
           pd == o.pd && hoist == o.hoist && youter == o.youter && padstage == o.padstage && hyb == o.hyb &&
           debug == o.debug && G == o.G;
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
  char buf[512];
  const int NTH = 64 * sh.G, PB = sh.pb(), PF = (PB + NTH - 1) / NTH, PBS = sh.pbs();
  snprintf(buf, sizeof(buf),
           "#define S_ %d\n#define C_ %d\n#define XB_ %d\n#define U_ %d\n#define U2_ %d\n#define G_ %d\n"
           "#define NTH_ %d\n#define PB_ %d\n#define PBS_ %d\n#define PF_ %d\n#define SC_ %s\n#define DIRECT_ %d\n#define YOUTER_ %d\n"
           "#define HYB_ %d\n#define DBGA_ %d\n",
           S, C, XB, sh.U, sh.U * sh.U, sh.G, NTH, PB, PBS, PF, sh.scale ? "true" : "false", sh.direct ? 1 : 0,
           sh.youter ? 1 : 0, sh.hybrid() ? 1 : 0, (sh.debug & 4) ? 1 : 0);
  s += buf;
  s += R"PLKJITM(
// P(t) of branch b (all classes, [c][x][y]) -> registers -> the LDS tile image
// [c][X][Y][hi][lo] with tile element (hi, lo) = P[4X + lo][4Y + hi]
#define PSTAGE_LOAD(R, b) { const double* s_ = a.pmats + (i64)(b) * PB_; \
  _Pragma("unroll") for (int j_ = 0; j_ < PF_; ++j_) { const int e_ = tid + j_ * NTH_; R[j_] = s_[e_ < PB_ ? e_ : PB_ - 1]; } }
#define PSTAGE_STORE(R, bf) { double* d_ = lds + (bf) * PBS_; \
  _Pragma("unroll") for (int j_ = 0; j_ < PF_; ++j_) if (PBS_ > PB_ || sidx[j_] >= 0) d_[sidx[j_]] = R[j_]; }
// D[c][X] (*)= sum_Y A(c, X, Y) . SRC[c][Y]   (SET: D was 1)
// (YOUTER_: the C * XB independent chains advance one block at a time, so consecutive MFMAs
// never depend on each other; the same sums in the same order either way)
// HYB_: the output's 16-state tiles on v_mfma_f64_16x16x4 (A = the 16 x 4 tile
// P[16 t + i][4Y + k], lane l holding i = l % 16, k = l / 16: 64 distinct values per 2048
// flops) and the remaining S % 16 states (20 states: 16..19) on v_mfma_f64_4x4x4_4b -- 4x
// fewer A operands per flop than all-4x4x4.  The 16x16 D registers q = 0..3 of tile t hold
// states 16 t + 4q + hi, exactly the layout of blocks X = 4t + q, and the 4x4x4 D the
// layout of the last block.  Image per class: NT16_ * XB_ tiles of 64, then XB_ of 16.
#define NT16_ (S_ / 16)
#define R4_ ((S_ % 16) / 4)
#define CONTRIB(D, SRC, bf, SET) { const double* P_ = PA + (bf) * PBS_; \
  if (HYB_) { const double* Q_ = PA16 + (bf) * PBS_; f64x4 h_[C_][NT16_]; double l_[C_]; \
    _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) { l_[c_] = 0.0; \
      _Pragma("unroll") for (int t_ = 0; t_ < NT16_; ++t_) h_[c_][t_] = (f64x4){0.0, 0.0, 0.0, 0.0}; } \
    _Pragma("unroll") for (int Y_ = 0; Y_ < XB_; ++Y_) _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) { \
      _Pragma("unroll") for (int t_ = 0; t_ < NT16_; ++t_) \
        h_[c_][t_] = mfma16(Q_[c_ * (S_ * S_) + (t_ * XB_ + Y_) * 64], SRC[c_][Y_], h_[c_][t_]); \
      if (R4_) l_[c_] = mfma4(P_[c_ * (S_ * S_) + NT16_ * XB_ * 64 + Y_ * 16], SRC[c_][Y_], l_[c_]); } \
    _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) { \
      _Pragma("unroll") for (int t_ = 0; t_ < NT16_; ++t_) _Pragma("unroll") for (int q_ = 0; q_ < 4; ++q_) { \
        if (SET) D[c_][4 * t_ + q_] = h_[c_][t_][q_]; else D[c_][4 * t_ + q_] *= h_[c_][t_][q_]; } \
      if (R4_) { if (SET) D[c_][4 * NT16_] = l_[c_]; else D[c_][4 * NT16_] *= l_[c_]; } } \
  } else if (YOUTER_) { double d_[C_][XB_]; \
    _Pragma("unroll") for (int Y_ = 0; Y_ < XB_; ++Y_) _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) \
      _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) \
        d_[c_][X_] = mfma4(P_[((c_ * XB_ + X_) * XB_ + Y_) * 16], SRC[c_][Y_], Y_ == 0 ? 0.0 : d_[c_][X_]); \
    _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) { \
      if (SET) D[c_][X_] = d_[c_][X_]; else D[c_][X_] *= d_[c_][X_]; } \
  } else { \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) { \
    double d_ = 0.0; \
    _Pragma("unroll") for (int Y_ = 0; Y_ < XB_; ++Y_) \
      d_ = mfma4(P_[DBGA_ ? c_ * (XB_ * XB_ * 16) : ((c_ * XB_ + X_) * XB_ + Y_) * 16], SRC[c_][Y_], d_); \
    if (SET) D[c_][X_] = d_; else D[c_][X_] *= d_; } } }
// direct: A(c, X, Y) = P[c][4X + lo][4Y + hi] read from the branch's P(t) in global memory
#define CONTRIB_G(D, SRC, b, SET) { const double* P_ = PG + (i64)(b) * PB_; \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) { \
    double d_ = 0.0; \
    _Pragma("unroll") for (int Y_ = 0; Y_ < XB_; ++Y_) d_ = mfma4(P_[(c_ * S_ + 4 * X_) * S_ + 4 * Y_], SRC[c_][Y_], d_); \
    if (SET) D[c_][X_] = d_; else D[c_][X_] *= d_; } }
#define ROWMUL(D, F, SET) { _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") \
  for (int X_ = 0; X_ < XB_; ++X_) { if (SET) D[c_][X_] = F[c_][X_]; else D[c_][X_] *= F[c_][X_]; } }
// one row of cherry k's contribution table (combined code of the pattern's two tips)
#define CHERRY_FETCH(F, FK, k) { const u8* base_ = a.cherry + (i64)(k) * a.cherry_stride; \
  const int code_ = reinterpret_cast<const u16*>(base_ + a.cherry_table_bytes + a.cherry_count_bytes)[p]; \
  const double* r_ = reinterpret_cast<const double*>(base_) + (i64)code_ * S_ + hi; \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) \
    F[c_][X_] = r_[(i64)c_ * (U2_ * S_) + 4 * X_]; \
  if (SC_) FK = (int)base_[a.cherry_table_bytes + code_]; }
// the same with the combined code already in a register (hoisted to the fragment start)
#define CHERRY_CODE(CC, k) const int CC = reinterpret_cast<const u16*>(a.cherry + (i64)(k) * a.cherry_stride + \
  a.cherry_table_bytes + a.cherry_count_bytes)[p];
#define CHERRY_FETCH_C(F, FK, k, CC) { const u8* base_ = a.cherry + (i64)(k) * a.cherry_stride; \
  const double* r_ = reinterpret_cast<const double*>(base_) + (i64)(CC) * S_ + hi; \
  _Pragma("unroll") for (int c_ = 0; c_ < C_; ++c_) _Pragma("unroll") for (int X_ = 0; X_ < XB_; ++X_) \
    F[c_][X_] = r_[(i64)c_ * (U2_ * S_) + 4 * X_]; \
  if (SC_) FK = (int)base_[a.cherry_table_bytes + (CC)]; }
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
  if (p < a.n_patterns) { if (hi == 0) a.site_lnl[p] = rr_; wr_ = a.weights[p] * rr_; } \
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
  s += R"PLKJITM(  extern __shared__ __attribute__((aligned(16))) double lds[];  // [2][PBS_] P tiles | red[16 G_]
  double* red = lds + (DIRECT_ ? 0 : 2 * PBS_);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 4, pl = lane & 15;
  const i64 p0 = a.p_base + (i64)blockIdx.x * (16 * G_);
  const i64 p = p0 + 16 * w + pl;
  const i64 toff = (p >> 7) * (i64)(C_ * S_ * kTile) + (p & (kTile - 1)) + (i64)hi * kTile;
  const double* PA = lds + ((hi << 2) | (lane & 3));
  const double* PA16 = lds + lane;  // HYB_: 16x16x4 A tiles, one element per lane
  const double* PG = a.pmats + (lane & 3) * S_ + hi;   // direct A operands: P[..][4X + lo][4Y + hi]
  int sidx[PF_];   // this thread's staging elements -> tile slots (past the table: padding)
  _Pragma("unroll") for (int j = 0; j < PF_; ++j) {
    const int e = tid + j * NTH_;
    const int c = e / (S_ * S_), r = e - c * (S_ * S_), x = r / S_, y = r - x * S_;
    const int t_ = HYB_ ? c * (S_ * S_) + (x < 16 * NT16_ ? ((x >> 4) * XB_ + (y >> 2)) * 64 + (y & 3) * 16 + (x & 15)
                                                        : NT16_ * XB_ * 64 + (y >> 2) * 16 + (y & 3) * 4 + (x - 16 * NT16_))
                        : ((c * XB_ + (x >> 2)) * XB_ + (y >> 2)) * 16 + ((y & 3) << 2) + (x & 3);
    sidx[j] = e < PB_ ? t_ : PBS_ > PB_ ? e : -1;
  }
  double R0[PF_] = {}, R1[PF_] = {}, R2[PF_] = {};
  (void)red; (void)PA; (void)PA16; (void)PG; (void)R0; (void)R1; (void)R2; (void)toff; (void)sidx;
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
  s += "  switch (frag) {\n";
  for (size_t f = 0; f < starts.size(); ++f) {
    std::vector<TInstr> ev;
    for (size_t i = (size_t)starts[f];; ++i) {
      ev.push_back(prog[i]);
      if (prog[i].op == T_ROOT) break;
    }
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
    auto emit_fetch = [&](int i) {
      const TInstr& e = ev[(size_t)i];
      const int sl = slot[(size_t)i];
      if (e.op == T_CHERRY && sh.hoist)
        snprintf(buf, sizeof(buf), "    CHERRY_FETCH_C(F%d, FK%d, %d, CC%d)\n", sl, sl, e.a, e.a);
      else if (e.op == T_CHERRY)
        snprintf(buf, sizeof(buf), "    CHERRY_FETCH(F%d, FK%d, %d)\n", sl, sl, e.a);
      else if (e.op == T_TIP)
        snprintf(buf, sizeof(buf), "    TIP_FETCH(F%d, %d)\n", sl, e.a);
      else
        snprintf(buf, sizeof(buf), "    LOAD_FETCH(F%d, FK%d, %d)\n", sl, sl, e.a);
      s += buf;
    };
    snprintf(buf, sizeof(buf), "  case %zu: {\n", f);
    s += buf;
    if (sh.hoist)
      for (const TInstr& e : ev)
        if (e.op == T_CHERRY) {
          snprintf(buf, sizeof(buf), "    CHERRY_CODE(CC%d, %d)\n", e.a, e.a);
          s += buf;
        }
    size_t nf = 0;
    for (; nf < fetchers.size() && nf < (size_t)L; ++nf) emit_fetch(fetchers[nf]);
    int cur = 0;
    size_t np = 0;  // P-chain events consumed
    if (sh.direct) pchain.clear();  // no staging chain: every contraction reads P(t) directly
    const int PD = std::min(std::max(sh.pd, 1), 3);
    // chain event j is staged from register set j % PD: loaded PD contractions ahead, stored
    // to the other LDS buffer (and a barrier) at the end of the contraction before its own
    const char* bar = (sh.debug & 1) ? "" : " __syncthreads();";
    auto pload = [&](size_t j) {
      if (j < pchain.size() && !(sh.debug & 2)) {
        snprintf(buf, sizeof(buf), "    PSTAGE_LOAD(R%zu, %d)\n", j % (size_t)PD, ev[(size_t)pchain[j]].b);
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
        if (nf < fetchers.size()) emit_fetch(fetchers[nf++]);
        const int sl = slot[i];
        if (e.op == T_LOAD && sh.direct) {
          snprintf(buf, sizeof(buf), "    CONTRIB_G(A%d, F%d, %d, %s)\n", d, sl, e.b, fresh[(size_t)d] ? "true" : "false");
          s += buf;
          if (sh.scale) {
            snprintf(buf, sizeof(buf), "    K%d += FK%d;\n", d, sl);
            s += buf;
          }
        } else if (e.op == T_LOAD) {
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
          snprintf(buf, sizeof(buf), "    STORE(A%d, K%d, %d)\n", d, d, e.a);
          s += buf;
        }
        if (sh.direct)
          snprintf(buf, sizeof(buf), "    CONTRIB_G(A%d, A%d, %d, %s)\n", d - 1, d, e.b, fresh[(size_t)d - 1] ? "true" : "false");
        else
          snprintf(buf, sizeof(buf), "    CONTRIB(A%d, A%d, %d, %s)\n", d - 1, d, cur, fresh[(size_t)d - 1] ? "true" : "false");
        s += buf;
        if (!sh.direct) pnext();
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
          snprintf(buf, sizeof(buf), "    STORE(A0, K0, %d)\n", e.a);
          s += buf;
        }
        if (e.b) s += "    REDUCE_ROOT(A0, K0)\n";
      }
    }
    s += "  } break;\n";
  }
  s += "  default: break;\n  }\n}\n";
  return s;
}

}  // namespace plk
