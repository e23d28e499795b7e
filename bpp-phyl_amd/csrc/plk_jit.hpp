// plk_jit.hpp -- tree-specialised fused traversal for 4-state models (gfx950).
//
// The interpreter in plk_tree4.hpp walks a tree program one event at a time: every
// event costs a scalar load of its program word, a compare-and-branch decode, 64-bit
// address arithmetic on the scalar unit and a dependent scalar load of P(t) -- all on
// the critical path of a wave that then issues only ~20 fp64 VALU instructions.
// Counters on cfg2 (64 taxa, GTR+G4): per wave ~4.7k SALU + 1.4k branches next to
// ~4.7k VALU, 42 % of wave cycles parked in s_waitcnt, VALU busy ~14 %.
//
// Here the same fragment programs (build_tree4_program: fragments and tiers) are
// emitted as straight-line HIP source -- one `case` per fragment -- and compiled once
// per (topology, C, codes in use, flags) with hiprtc for gfx950:
//   * every P(t) address is a constant offset from one wave-uniform base, so P lives
//     in SGPRs (s_load) and there is no decode, no program fetch and no branch;
//   * a tip contributes through its table row tipP[tip][c][code][x] =
//     sum_y P[c][x][y] init[code][y] (tip_table_kernel), staged in LDS once per
//     workgroup for the fragment's tips: one 32-byte LDS read and 4 multiplies
//     instead of a 4x4 matvec (16 FMAs) per tip;
//   * the first contribution into a node's accumulator is an assignment (1 * s == s
//     exactly), not a multiply;
//   * workgroups are persistent over pattern super-blocks (64 * G patterns), so the
//     tables are staged once per workgroup, not once per 64 patterns;
//   * the operands of event i + L (tip row, or a materialised child partial) are
//     fetched next to the compute of event i inside one scheduling region (closed by
//     sched_barrier), which hides their latency while bounding registers.
// Every arithmetic operation is the interpreter's, in the same order, so the results
// are bitwise those of tree4_kernel<1, DM, SCALE>.  Modules are compiled and cached
// per process by source (plk.hip: jit_function).
#pragma once

#include <algorithm>
#include <string>
#include <vector>

#include "plk_tree4.hpp"

namespace plk {

// Device helpers of the generated kernels.  They restate rescale / store_partial /
// the fused root reduction of plk_tree4.hpp for one class per wave and G pattern
// groups per workgroup (wave w: class w % C, group w / C).
static const char* kJitPrelude = R"PLKJIT(
typedef unsigned char u8;
typedef long long i64;
typedef int i32;
typedef __attribute__((address_space(4))) const double* CPd;
#define kTile 128
#define kLn2x256 177.44567822334599921
#define kScaleUp 115792089237316195423570985008687907853269984665640564039457584007913129639936.0
#define kScaleThr (1.0 / kScaleUp)

struct JArgs {  // codes: one row per table unit (unit_codes_kernel)
  double* partials; i32* scale; const u8* codes; const double* tipP; const double* weights;
  const double* pi; const double* probs; double* site_lnl; double* wave_sums;
  i64 slot_stride; i64 n_pad; i64 n_patterns; i32 n_sblocks; i32 guard;
  unsigned* sb_ctr; i32 dyn; unsigned* exit_ctr; i32* uflow;
  double* cls_sum;  // workgroups of one class (CLS_): per class and pattern, its root term [C][n_pad]
};

// Register vectors hold 4 * CW * PW doubles: vector v = pw * CW + cw is class c0 + cw of
// the lane's pattern pw (patterns p and p + 64 of a 128-pattern tile when PW = 2).

// dst[v][x] (*)= sum_y P_cw[x][y] src[v][y] (P_cw at P + 16 cw, row-major; one P read
// serves every pattern of the lane); SET: dst was 1
template <int PW, bool SET, int CW>
__device__ __forceinline__ void contrib_cls(double (&dst)[4 * CW * PW], const double (&src)[4 * CW * PW],
                                            const double (&p)[16], int cw) {
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int pw = 0; pw < PW; ++pw) {
      const int v = 4 * (pw * CW + cw);
      double s = p[4 * x + 0] * src[v + 0];
      s = __builtin_fma(p[4 * x + 1], src[v + 1], s);
      s = __builtin_fma(p[4 * x + 2], src[v + 2], s);
      s = __builtin_fma(p[4 * x + 3], src[v + 3], s);
      if (SET) dst[v + x] = s; else dst[v + x] *= s;
    }
}
// P(t) of one class (16 doubles, wave-uniform: scalar loads into SGPRs), and an empty use
// of it that places the wait for those loads
__device__ __forceinline__ void pload(double (&r)[16], CPd P) {
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = P[i];
}
__device__ __forceinline__ void ptouch(const double (&r)[16]) {
  asm volatile("" ::"s"(r[0]), "s"(r[1]), "s"(r[2]), "s"(r[3]), "s"(r[4]), "s"(r[5]), "s"(r[6]), "s"(r[7]));
  asm volatile("" ::"s"(r[8]), "s"(r[9]), "s"(r[10]), "s"(r[11]), "s"(r[12]), "s"(r[13]), "s"(r[14]), "s"(r[15]));
}
template <int CW, int PW, bool SET>
__device__ __forceinline__ void contrib(double (&dst)[4 * CW * PW], const double (&src)[4 * CW * PW], CPd P) {
  if (CW == 1 || !PPIPE_) {
#pragma unroll
    for (int cw = 0; cw < CW; ++cw) {
      double p[16];
      pload(p, P + 16 * cw);
      contrib_cls<PW, SET, CW>(dst, src, p, cw);
    }
    return;
  }
  // classes in the wave (PPIPE_): class cw + 1's loads are issued before class cw's
  // arithmetic and waited for after it.  Scalar loads complete out of order, so every
  // wait is for all of them: left to itself the compiler loads each class right before
  // its use and exposes the whole scalar-load latency once per class (cfg5: P loads
  // ~23 % of the kernel at two waves per SIMD)
  double pa[16], pb[16];
  pload(pa, P);
  ptouch(pa);
#pragma unroll
  for (int cw = 0; cw < CW; cw += 2) {
    if (cw + 1 < CW) pload(pb, P + 16 * (cw + 1));
    __builtin_amdgcn_sched_barrier(0);
    contrib_cls<PW, SET, CW>(dst, src, pa, cw);
    __builtin_amdgcn_sched_barrier(0);
    if (cw + 1 < CW) {
      ptouch(pb);
      if (cw + 2 < CW) pload(pa, P + 16 * (cw + 2));
      __builtin_amdgcn_sched_barrier(0);
      contrib_cls<PW, SET, CW>(dst, src, pb, cw + 1);
      __builtin_amdgcn_sched_barrier(0);
      if (cw + 2 < CW) ptouch(pa);
    }
  }
}

// Stream form of the pipelined contrib across a fragment's contributions: pbuf[B0] holds
// this contribution's class 0 (loaded and waited); each class's arithmetic runs while the
// next class's P(t) -- after the last class, class 0 of the next contribution (Pn, NEXT) --
// is loading into the other buffer, waited for after the arithmetic.  One exposed wait per
// fragment instead of one per contribution.
template <int CW, int PW, bool SET, int B0, bool NEXT>
__device__ __forceinline__ void contrib_s(double (&dst)[4 * CW * PW], const double (&src)[4 * CW * PW], CPd P,
                                          CPd Pn, double (&pbuf)[2][16]) {
#pragma unroll
  for (int cw = 0; cw < CW; ++cw) {
    double(&cur)[16] = pbuf[(B0 + cw) & 1];
    double(&nxt)[16] = pbuf[(B0 + cw + 1) & 1];
    if (cw + 1 < CW)
      pload(nxt, P + 16 * (cw + 1));
    else if (NEXT)
      pload(nxt, Pn);
    __builtin_amdgcn_sched_barrier(0);
    contrib_cls<PW, SET, CW>(dst, src, cur, cw);
    __builtin_amdgcn_sched_barrier(0);
    if (cw + 1 < CW || NEXT) ptouch(nxt);
  }
}

template <int N, bool SET>
__device__ __forceinline__ void tipmul(double (&dst)[N], const double (&row)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (SET) dst[i] = row[i]; else dst[i] *= row[i];
  }
}

// Keep a freshly computed accumulator where the program put it: sched_barrier only binds
// the machine scheduler, and IR-level sinking would otherwise delay multiplies of one
// pattern to their next use (their operands then stay live and spill).  No code.
template <int N>
__device__ __forceinline__ void pin(double (&v)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}

template <int PW>
__device__ __forceinline__ void kzero(int (&k)[PW]) {
#pragma unroll
  for (int i = 0; i < PW; ++i) k[i] = 0;
}
template <int PW>
__device__ __forceinline__ void kadd(int (&k)[PW], const int (&d)[PW]) {
#pragma unroll
  for (int i = 0; i < PW; ++i) k[i] += d[i];
}

// opaque copies (no code): values the optimiser cannot prove equal to their source
__device__ __forceinline__ unsigned long long launder_s(unsigned long long x) {
  asm volatile("" : "+s"(x));
  return x;
}
// component j of a uint4 (j a constant)
__device__ __forceinline__ unsigned cvw(const uint4& v, int j) { return j == 0 ? v.x : j == 1 ? v.y : j == 2 ? v.z : v.w; }
// Table element x of row r (R rows per class block): [row][4] or, with SOA_, [half][row][2]
#define TABIX(R, r, x) (SOA_ ? ((x) >> 1) * ((R) * 2) + (r) * 2 + ((x) & 1) : (r) * 4 + (x))
// a quad table's row position (plk_kernels.hpp quad_row: unit_codes_kernel stores it as the code)
#define QROW_(r) (U_ == 4 ? (((r) & ~15) | (((r) + 7 * (((r) >> 6) & 3) + 7 * (((r) >> 4) & 3)) & 15)) : (r))
__device__ __forceinline__ unsigned long long launder_v(unsigned long long x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Rescale decisions from the high words of the doubles.  For x >= 0, x < 2^-256 iff
// hi(x) < kThrHi (2^-256 has a zero low word), and negative values have negative (signed)
// high words, so mh = max(0, hi(v)...) decides "0 < max(0, v...) < 2^-256" whenever
// 0 < mh < 0x7FF00000: one 32-bit max3 per two values instead of an f64 max per value
// plus the NaN canonicalisation of its operand.  Otherwise (every value <= 0, positive
// values only denormals with a zero high word, an Inf or a NaN) the f64 path decides.
#define kThrHi 0x2FF00000
__device__ __forceinline__ int hiw(double x) { return (int)(__double_as_longlong(x) >> 32); }
__device__ __forceinline__ bool hi_decides(int mh) { return mh > 0 && mh < 0x7FF00000; }

// own-class max below the rescale threshold (or zero / NaN): the joint check of the
// exact pass could fire here
// (the flag is pinned with an empty asm right away: otherwise the compares sink to the
// vote at the end of the fragment and keep every node's accumulator alive until then)
// (hi-word max as in rescale(): not risky iff some value is finite and >= the threshold)
template <int N>
__device__ __forceinline__ void flag_risky(int& dng, const double (&v)[N]) {
  int mh = hiw(v[0]);
#pragma unroll
  for (int i = 1; i < N; ++i) mh = max(mh, hiw(v[i]));
  dng |= !(mh >= kThrHi && mh < 0x7FF00000);
  asm volatile("" : "+v"(dng));
}

// Joint (all-class) exact power-of-two rescale of each of the lane's patterns.  NW =
// C / CW waves hold the classes of one pattern group (NWT waves in the workgroup);
// with NW = 1 the joint max is all in registers.
template <int C, int CW, int PW, int NWT>
__device__ __forceinline__ void rescale(double (&v)[4 * CW * PW], int (&cnt)[PW], double* xch, int w, int g) {
  constexpr int NW = C / CW;
  if (NW == 1) {
#pragma unroll
    for (int pw = 0; pw < PW; ++pw) {
      int mh = 0;
#pragma unroll
      for (int i = 0; i < 4 * CW; ++i) mh = max(mh, hiw(v[4 * CW * pw + i]));
      bool up;
      if (__builtin_expect(hi_decides(mh), 1)) {
        up = mh < kThrHi;
      } else {
        double m = 0.0;
#pragma unroll
        for (int i = 0; i < 4 * CW; ++i) m = fmax(m, v[4 * CW * pw + i]);
        up = m > 0.0 && m < kScaleThr;
      }
      if (up) {
#pragma unroll
        for (int i = 0; i < 4 * CW; ++i) v[4 * CW * pw + i] *= kScaleUp;
        cnt[pw] += 1;
      }
    }
    return;
  }
  double m[PW];
#pragma unroll
  for (int pw = 0; pw < PW; ++pw) {
    m[pw] = 0.0;
#pragma unroll
    for (int i = 0; i < 4 * CW; ++i) m[pw] = fmax(m[pw], v[4 * CW * pw + i]);
  }
  {
    // one barrier: consecutive rescales alternate between two exchange buffers, so a
    // wave can only overwrite this buffer after every wave has passed the next
    // rescale's barrier, i.e. after every wave has read it here
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int pw = 0; pw < PW; ++pw) xch[(pw * NWT + w) * 64 + lane] = m[pw];
    __syncthreads();
#pragma unroll
    for (int pw = 0; pw < PW; ++pw) {
      m[pw] = 0.0;
      for (int k = 0; k < NW; ++k) m[pw] = fmax(m[pw], xch[(pw * NWT + g * NW + k) * 64 + lane]);
    }
  }
#pragma unroll
  for (int pw = 0; pw < PW; ++pw)
    if (m[pw] > 0.0 && m[pw] < kScaleThr) {
#pragma unroll
      for (int i = 0; i < 4 * CW; ++i) v[4 * CW * pw + i] *= kScaleUp;
      cnt[pw] += 1;
    }
}

// One class per workgroup (JitShape::cls): this class's root term of each of the lane's patterns,
// t_c = (sum_s L[c][s] pi_s, terms <= 0 dropped under the guards) * prob_c -- reduce_root's
// t[pw][0] -- goes to cls_sum[c][p]; class_sums_to_blocks adds the classes in class order with
// the guard or clamp, takes the log and forms the block sums as reduce_root + wave_sums_to_blocks.
template <int PW>
__device__ __forceinline__ void reduce_root_cls(const JArgs& a, const double (&acc)[4 * PW], int c0, i64 p, bool gv) {
  if (!gv) return;
#pragma unroll
  for (int pw = 0; pw < PW; ++pw) {
    double lc = 0.0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const double li = acc[4 * pw + s] * a.pi[s];
      if (a.guard) {
        if (li > 0.0) lc += li;
      } else {
        lc += li;
      }
    }
    __builtin_nontemporal_store(lc * a.probs[c0], a.cls_sum + (i64)c0 * a.n_pad + p + 64 * pw);
  }
}

// off: the lane's first pattern in the slot (tile layout); pattern pw is 64 further
template <int CW, int PW, bool SCALE>
__device__ __forceinline__ void store(const JArgs& a, int slot, i64 off, i64 p, int c0,
                                      const double (&v)[4 * CW * PW], const int (&cnt)[PW], bool gv) {
  if (!gv) return;  // a group past the last pattern (ragged last super-block) recomputes group 0
  slot = (int)launder_s(slot);  // (as in LOADF)
  double* dst = a.partials + (i64)slot * a.slot_stride + off;
#pragma unroll
  for (int pw = 0; pw < PW; ++pw)
#pragma unroll
    for (int i = 0; i < 4 * CW; ++i) __builtin_nontemporal_store(v[4 * CW * pw + i], dst + 64 * pw + (i64)i * kTile);
  if (SCALE && c0 == 0)
#pragma unroll
    for (int pw = 0; pw < PW; ++pw) a.scale[(i64)slot * a.n_pad + p + 64 * pw] = cnt[pw];
}

// log() out of line: inlined into the persistent loop, its polynomial constants are
// hoisted out of the loop into registers (and spilled with two patterns per lane)
__device__ __attribute__((noinline)) double jit_log(double x) { return log(x); }

template <int C, int CW, int PW, int NWT, bool SCALE>
__device__ __forceinline__ void reduce_root(const JArgs& a, const double (&acc)[4 * CW * PW], const int (&cnt)[PW],
                                            double* xch, int w, int g, int c0, i64 p0, i64 p, bool gv) {
  constexpr int NW = C / CW;
  const int lane = threadIdx.x & 63;
  double t[PW][CW];
#pragma unroll
  for (int pw = 0; pw < PW; ++pw)
#pragma unroll
    for (int cw = 0; cw < CW; ++cw) {
      double lc = 0.0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const double li = acc[4 * (pw * CW + cw) + s] * a.pi[s];
        if (a.guard) {
          if (li > 0.0) lc += li;
        } else {
          lc += li;
        }
      }
      t[pw][cw] = lc * a.probs[c0 + cw];
    }
  if (NW > 1) {
    __syncthreads();
#pragma unroll
    for (int pw = 0; pw < PW; ++pw) xch[(pw * NWT + w) * 64 + lane] = t[pw][0];
    __syncthreads();
  }
  if (c0 == 0) {
#pragma unroll
    for (int pw = 0; pw < PW; ++pw) {
      double l = 0.0;
      for (int c = 0; c < C; ++c) {
        const double li = NW > 1 ? xch[(pw * NWT + g * NW + c) * 64 + lane] : t[pw][c < CW ? c : 0];
        if (a.guard) {
          if (li > 0.0) l += li;
        } else {
          l += li;
        }
      }
      if (!a.guard && l < 0.0) l = 0.0;
      double r = jit_log(l);
      if (SCALE) r -= (double)cnt[pw] * kLn2x256;
      double wr = 0.0;
      const i64 pp = p + 64 * pw;
      if (gv && pp < a.n_patterns) {
        if (a.uflow && !(l >= 2.0 * kScaleThr)) *a.uflow = 1;  // plk_root_underflow
        a.site_lnl[pp] = r;
        wr = a.weights[pp] * r;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) wr += __shfl_xor(wr, off, 64);
      if (gv && lane == 0) a.wave_sums[(p0 + 64 * pw) >> 6] = wr;
    }
  }
}
)PLKJIT";

// Host mirror of JArgs (field order and types must match the prelude).
struct JArgs {
  double* partials;
  int32_t* scale;
  const uint8_t* codes;
  const double* tipP;
  const double* weights;
  const double* pi;
  const double* probs;
  double* site_lnl;
  double* wave_sums;
  int64_t slot_stride;
  int64_t n_pad;
  int64_t n_patterns;
  int32_t n_sblocks;
  int32_t guard;
  // dynamic super-blocks (dyn != 0): after its first super-block (blockIdx.x) a workgroup
  // takes the next one from sb_ctr[frag], which is 0 when the launch starts (the last
  // workgroup to exit resets it)
  unsigned* sb_ctr;
  int32_t dyn;
  // exit ticket (with dyn): every workgroup takes one ticket as it exits; the last one resets
  // the launch's super-block counters and the ticket counter to 0
  unsigned* exit_ctr;
  int32_t* uflow;  // unscaled handles: set to 1 when a site likelihood is < 2^-255 (or null)
  double* cls_sum;  // JitShape::cls: every class's root term per pattern, [C][n_pad] (class_sums_to_blocks)
};

struct JitShape {
  int C = 1;        // rate classes
  int CW = 1;       // classes per wave (1, or C: a wave holds every class of its patterns)
  int PW = 1;       // patterns per lane (1 or 2: p and p + 64 share every P(t) read)
  bool pin = false; // pin accumulators after every event (see pin())
  int G = 1;        // 64-pattern groups per workgroup
  int U = 1;        // codes in use (rows of a tip table)
  int NT = 0;       // most table units (tips or tip pairs) of any fragment: code rows in LDS
  int TD = 0;       // most table doubles of any fragment (JitPlan::tab_doubles)
  bool scale = false;
  int L = 1;        // operand fetch lookahead (events)
  int RD = 1;       // two-stage fetch: table rows RD fetchers ahead (codes L ahead; RD <= L)
  int minw = 0;     // __launch_bounds__ min waves per SIMD (0: compiler default)
  bool ppipe = true;        // classes in the wave: P(t) of the next class loaded during this one (contrib)
  int clk = 0;              // PLK_DEBUG_CLOCK: per-workgroup shader-clock / constant-clock stamps (diagnostic; 2: prologue only)
  // one class per workgroup (grid.z = class): the tables hold that class only (C x smaller, so
  // a fragment's cherries fit as quad units, JitUnit), and the root terms of the classes meet
  // in HBM (class_sums_to_blocks) instead of an LDS exchange.  One class per wave, no scaling.
  bool cls = false;
  int QT = 0;       // quad build scratch doubles (JitPlan::quad_tmp), in the code rows' LDS
  // table rows as two planes of 16-byte halves ([half][row] per class) instead of 32-byte rows:
  // a ds_read_b128 of random rows then spreads over all 16 four-bank windows, not 8
  bool soa = false;
  bool ps1 = false;  // one class per wave: the P(t) stream (contrib_s) too
  // direct codes (cls, at most 16 units per fragment): every wave loads its own patterns' unit
  // codes, 16 bytes per pattern ([fragment][pattern][16], unit_codes_dc_kernel), into
  // registers one super-block ahead -- no code rows in LDS and one barrier per super-block
  bool dc = false;
  int dcw = 1;       // direct codes: 16-byte words per pattern (16 units each; 2 for up to 32 units)
  int nw() const { return cls ? 1 : C / CW; }  // waves per pattern group
  size_t lds_bytes() const {
    const size_t nt = (size_t)std::max(NT, 1);
    // the class exchange (root reduction, per-node rescale; the second buffer only serves the
    // rescale) -- none with one class per workgroup
    const size_t xch = cls ? 0 : (scale ? 2 : 1) * (size_t)PW * G * nw() * 64 * sizeof(double);
    // the code rows' space also holds the quad build's cherry rows before the first super-block
    return (size_t)std::max(TD, 4) * sizeof(double) + xch +
           std::max(dc ? (size_t)0 : (size_t)G * nt * 64 * PW, (size_t)QT * sizeof(double));
  }
};

// The generated kernel's name: one class per workgroup is plk_jit_tree4c, so that kernel-trace
// statistics keep it apart from the classes-in-the-wave kernel (plk_jit_tree4) of other configs
inline const char* jit_tree4_name(const JitShape& sh) { return sh.cls ? "plk_jit_tree4c" : "plk_jit_tree4"; }

// Pattern groups per workgroup with the most waves resident per CU: LDS (160 KiB per CU)
// against the tables every workgroup stages once, and VGPRs at the ~72 registers these
// kernels take (7 waves per SIMD); ties go to fewer groups.
inline int jit_auto_groups(const JitShape& base) {
  int best_g = 1, best_w = 0;
  for (int g = 1; g <= 4; ++g) {
    JitShape t = base;
    t.G = g;
    const int waves_wg = t.nw() * g;
    const int by_lds = (int)((160 * 1024) / std::max<size_t>(t.lds_bytes(), 1));
    const int by_vgpr = (4 * 7) / waves_wg;
    const int waves = std::min(by_lds, by_vgpr) * waves_wg;
    if (waves > best_w) {
      best_w = waves;
      best_g = g;
    }
  }
  return best_g;
}

struct JitEvent {
  int op;     // T_TIP (a = fragment-local table unit), T_LOAD, T_DESCEND, T_ASCEND (level >= 1), T_ROOT
  int level;  // accumulator level the event works on
  int a, b;   // program word fields
};

// One LDS table of a fragment: a tip's rows tipP[tip][c][code][x] (tb < 0), or -- for two
// tips that are the first two contributions of one node (a cherry) -- their product
// rows pair[c][ca * U + cb][x] = tipP[ta][c][ca][x] * tipP[tb][c][cb][x], read with one
// combined code (ca * U + cb, formed while staging the codes).  The interpreter forms the
// same product (A = row_a, then A *= row_b), so the results stay bitwise identical while
// a cherry costs one table read instead of two and no multiply.  Layout in LDS at `off`
// (doubles): [C][rows][4].
// A cherry whose partial is not stored goes one step further: its unit holds the
// cherry's contribution to its parent, cont[c][ca * U + cb][x] =
// sum_y P_br[c][x][y] pair[c][ca * U + cb][y] (br = the cherry node), formed in the
// interpreter's operation order (contrib), and the cherry's branch costs no FMA either.
// With rescaling, the cherry's joint check depends on its row alone: the row is rescaled
// before the product exactly as the kernel would, and its count (0 / 1) is kept in U * U
// bytes at koff, added to the parent's count with the contribution.
// A quad (one class per workgroup, no scaling) goes one level further: a node Q whose two
// children are unstored cherries (a, b) and (c, d), itself not stored, is one unit whose rows
// hold Q's contribution to its parent, quad[((ca U + cb) U + cc) U + cd][x] =
// sum_y P_Q[x][y] (contA[ca U + cb][y] * contB[cc U + cd][y]) with contA / contB the cherries'
// contribution rows -- the operations of the interpreter in its order (Q's accumulator is
// contA, then *= contB; then contrib), read with one combined code (U^4 <= 256).  A 4-tip
// subtree then costs one LDS row read instead of two reads, 4 multiplies and a 4x4 matvec.
struct JitUnit {
  int ta, tb;
  int off;
  int br = -1;    // >= 0: contribution unit through P of node br
  int koff = -1;  // rescaling contribution unit: doubles offset of its count bytes
  int tc = -1, td = -1;    // quad: tips of the second cherry (ta, tb: the first)
  int brA = -1, brB = -1;  // quad: the two cherry nodes (br: the quad node Q)
};

struct JitPlan {
  std::vector<std::vector<JitEvent> > events;  // per fragment (tier order)
  std::vector<std::vector<JitUnit> > units;    // per fragment: its tables, in event order
  int NU = 0;           // most units of any fragment
  int tab_doubles = 0;  // most table doubles of any fragment
  int quad_tmp = 0;     // most doubles of any fragment's quad build scratch (its cherries' rows)
};

// Per fragment: its events with TIP events renumbered to fragment-local table units.
// Cherries become pair units while the fragment's tables stay within pair_budget
// doubles (0: no pairs; pairs need U * U <= 256 so that a combined code is one byte).
// cls: one class per workgroup (tables of one class); quad_budget > 0 (doubles, cls only): pairs
// of unstored cherries under an unstored node become quad units while the tables fit.
inline JitPlan jit_plan(const std::vector<TInstr>& prog, const std::vector<int32_t>& starts, int C, int U,
                        int pair_budget, bool scale, bool cls = false, int quad_budget = 0) {
  JitPlan plan;
  plan.events.assign(starts.size(), {});
  plan.units.assign(starts.size(), {});
  const int CT = cls ? 1 : C;  // classes in the tables
  const bool pairs = pair_budget > 0 && U * U <= 256;
  const bool quads = cls && !scale && pairs && quad_budget > 0 && U * U * U * U <= 256;
  const int single = CT * U * 4, grow = CT * U * 4 * (U - 1), pair = CT * U * U * 4, quad = CT * U * U * U * U * 4;
  for (size_t f = 0; f < starts.size(); ++f) {
    std::vector<JitEvent>& ev = plan.events[f];
    std::vector<JitUnit>& un = plan.units[f];
    int d = 0, total = 0;
    for (size_t i = (size_t)starts[f];; ++i) {
      const TInstr& w = prog[i];
      if (w.op == T_TIP) {
        // the previous event is this node's first contribution, a tip not yet paired
        const size_t n = ev.size();
        const bool first_tip = n >= 1 && ev[n - 1].op == T_TIP && ev[n - 1].level == d &&
                               un[(size_t)ev[n - 1].a].tb < 0 &&
                               (n == 1 ? d == 0 : ev[n - 2].op == T_DESCEND && ev[n - 2].level == d);
        if (pairs && first_tip && total + grow <= pair_budget) {
          un[(size_t)ev[n - 1].a].tb = w.a;
          total += grow;
        } else {
          ev.push_back({T_TIP, d, (int)un.size(), w.b});
          un.push_back({w.a, -1, 0});
          total += single;
        }
      } else if (w.op == T_LOAD) {
        ev.push_back({T_LOAD, d, w.a, w.b});
      } else if (w.op == T_DESCEND) {
        ++d;
        ev.push_back({T_DESCEND, d, 0, 0});
      } else if (w.op == T_ASCEND) {
        if (d == 0) continue;  // fragment root: finished by ROOT
        const size_t n = ev.size();
        if (w.a < 0 && w.b >= 0 && n >= 2 && ev[n - 1].op == T_TIP && ev[n - 1].level == d &&
            un[(size_t)ev[n - 1].a].tb >= 0 && ev[n - 2].op == T_DESCEND && ev[n - 2].level == d) {
          // a cherry (two tips, nothing else) that is not stored: its contribution unit is
          // a tip-like operand of the parent
          const int k = ev[n - 1].a;
          un[(size_t)k].br = w.b;
          if (scale) un[(size_t)k].koff = 0;  // placed below
          ev.resize(n - 2);
          --d;
          ev.push_back({T_TIP, d, k, w.b});
          continue;
        }
        auto cherry_unit = [&](size_t i) {  // event i: a contribution unit of an unstored cherry at level d
          if (ev[i].op != T_TIP || ev[i].level != d) return false;
          const JitUnit& u = un[(size_t)ev[i].a];
          return u.tb >= 0 && u.br >= 0 && u.tc < 0 && u.koff < 0;
        };
        if (quads && w.a < 0 && w.b >= 0 && n >= 3 && cherry_unit(n - 1) && cherry_unit(n - 2) &&
            ev[n - 3].op == T_DESCEND && ev[n - 3].level == d && ev[n - 1].a == (int)un.size() - 1 &&
            total + quad - 2 * pair <= quad_budget) {
          // a quad: the node's two children are unstored cherries, the node is not stored
          const int k1 = ev[n - 2].a, k2 = ev[n - 1].a;
          JitUnit& q = un[(size_t)k1];
          q.tc = un[(size_t)k2].ta;
          q.td = un[(size_t)k2].tb;
          q.brA = q.br;
          q.brB = un[(size_t)k2].br;
          q.br = w.b;
          un.pop_back();
          total += quad - 2 * pair;
          ev.resize(n - 3);
          --d;
          ev.push_back({T_TIP, d, k1, w.b});
          continue;
        }
        ev.push_back({T_ASCEND, d, w.a, w.b});
        --d;
      } else if (w.op == T_ROOT) {
        ev.push_back({T_ROOT, 0, w.a, w.b});
        break;
      }
    }
    int off = 0;
    for (JitUnit& u : un) {
      u.off = off;
      off += u.tb < 0 ? single : u.tc >= 0 ? quad : pair;
      if (u.koff >= 0) {
        u.koff = off;
        off += (U * U + 31) / 32 * 4;  // count bytes, whole 32-byte rows
      }
    }
    plan.NU = std::max(plan.NU, (int)un.size());
    plan.tab_doubles = std::max(plan.tab_doubles, off);
    int nq = 0;
    for (const JitUnit& u : un) nq += u.tc >= 0;
    plan.quad_tmp = std::max(plan.quad_tmp, 2 * nq * U * U * 4);
  }
  return plan;
}

// Emit the kernel for a fragment plan (jit_plan over build_tree4_program's words and
// fragment start offsets in tier order; fragment id = frag_base + blockIdx.y).
inline std::string jit_tree4_source(const JitPlan& plan, const JitShape& sh) {
  const std::vector<std::vector<JitEvent> >& events = plan.events;
  const int C = sh.C, L = std::max(sh.L, 1), U = sh.U;
  std::string s;
  s.reserve(4096 * events.size() + 16384);
  s += sh.ppipe ? "#define PPIPE_ 1\n" : "#define PPIPE_ 0\n";  // read by the prelude's contrib
  s += kJitPrelude;
  char buf[400];
  const std::string minw_s = sh.minw > 0 ? ", " + std::to_string(sh.minw) : std::string();
  // fragment table units (CSR) as constant data of the module: unit k of fragment f is
  // entry kFragUnitStart[f] + k of kUnitD, one 32-byte record (ta, tb (-1: single tip), off,
  // br, koff) read with ONE scalar load -- five separate arrays cost a chain of dependent
  // scalar loads per unit (the branch on tb placed a wait before the next load), ~2.8 us
  // per staging round at the start of every launch (profiles/r03/r3d sweep)
  std::string ud = "};\nstruct __attribute__((aligned(32))) UnitD { int ta, tb, off, br, koff, p0, p1, p2; };\n"
                   "__device__ const UnitD kUnitD[] = {{0, 0, 0, 0, 0, 0, 0, 0}";
  // With rescaling, a fragment's rescaling contribution units (koff >= 0) are listed apart
  // (kScUnit, CSR kFragScStart) and staged with one (unit, row) per thread of the whole
  // workgroup -- such a unit has only U * U rows (16 for DNA), so one unit per wave left 48
  // of 64 lanes idle and cost one dependent load round per unit and wave; the other units
  // (kOtherD: their records in that order, CSR kFragOtherStart) keep one unit per wave.
  std::string sc = "};\n__device__ const int kFragScStart[] = {0", scu = "};\n__device__ const int kScUnit[] = {0",
              ot = "};\n__device__ const int kFragOtherStart[] = {0",
              otu = "};\n__device__ const UnitD kOtherD[] = {{0, 0, 0, 0, 0, 0, 0, 0}";
  // quad units (JitUnit): their own list (kQuadD, CSR kFragQuadStart), staged one row per thread
  std::string qs = "};\nstruct QuadD { int ta, tb, tc, td, brA, brB, brQ, off; };\n"
                   "__device__ const int kFragQuadStart[] = {0",
              qd = "};\n__device__ const QuadD kQuadD[] = {{0, 0, 0, 0, 0, 0, 0, 0}";
  {
    // the P(t) matrices each fragment reads (CSR kFragPStart / kFragPBr), touched at launch
    std::string st = "\n__device__ const int kFragPStart[] = {0", br = "};\n__device__ const int kFragPBr[] = {0";
    int acc = 0;
    for (size_t f = 0; f < events.size(); ++f) {
      std::vector<int> b;
      for (const JitEvent& e : events[f])
        if ((e.op == T_LOAD || e.op == T_ASCEND) && e.b >= 0) b.push_back(e.b);
      for (const JitUnit& u : plan.units[f])
        if (u.br >= 0) b.push_back(u.br);
      std::sort(b.begin(), b.end());
      b.erase(std::unique(b.begin(), b.end()), b.end());
      for (int x : b) {
        snprintf(buf, sizeof(buf), ",%d", x);
        br += buf;
      }
      acc += (int)b.size();
      snprintf(buf, sizeof(buf), ",%d", acc);
      st += buf;
    }
    s += st + br + "};\n";
  }
  // Fragments of one shape share their code (a balanced tree's eight 64-tip subtrees: one
  // case instead of eight -- 8x less generated code to compile and to fetch).  The code
  // differs between such fragments only in the P(t) offsets of their branches and the slots
  // they load and store; those become a per-fragment base (kFragNB: node, kFragSB: slot) plus
  // the shared relative offset.  Shape = the event list with node / slot fields relative to
  // the bases, and the table units' layout (tips and cherry branches are runtime data).
  std::vector<int> nbase(events.size(), 0), sbase(events.size(), 0), leader(events.size(), -1);
  {
    std::vector<std::string> sig(events.size());
    for (size_t f = 0; f < events.size(); ++f) {
      int nb = 1 << 30, sb = 1 << 30;
      for (const JitEvent& e : events[f]) {
        if ((e.op == T_LOAD || e.op == T_ASCEND) && e.b >= 0) nb = std::min(nb, e.b);
        if ((e.op == T_LOAD || e.op == T_ASCEND || e.op == T_ROOT) && e.a >= 0) sb = std::min(sb, e.a);
      }
      nbase[f] = nb == (1 << 30) ? 0 : nb;
      sbase[f] = sb == (1 << 30) ? 0 : sb;
      std::string& g = sig[f];
      for (const JitEvent& e : events[f]) {
        const bool node = (e.op == T_LOAD || e.op == T_ASCEND) && e.b >= 0;
        const bool slt = (e.op == T_LOAD || e.op == T_ASCEND || e.op == T_ROOT) && e.a >= 0;
        snprintf(buf, sizeof(buf), "%d,%d,%d,%d;", e.op, e.level,
                 slt ? e.a - sbase[f] : (e.op == T_TIP ? e.a : -1),
                 node ? e.b - nbase[f] : (e.op == T_ROOT ? e.b : -1));
        g += buf;
      }
      g += "|";
      for (const JitUnit& u : plan.units[f]) {
        snprintf(buf, sizeof(buf), "%d,%d,%d,%d;", u.tb < 0 ? 0 : 1, u.br >= 0 ? 1 : 0, u.off, u.koff);
        g += buf;
      }
      for (size_t q = 0; q < f && leader[f] < 0; ++q)
        if (leader[q] == (int)q && sig[q] == g) leader[f] = (int)q;
      if (leader[f] < 0) leader[f] = (int)f;
    }
    std::string nbs = "\n__device__ const int kFragNB[] = {0", sbs = "};\n__device__ const int kFragSB[] = {0";
    for (size_t f = 0; f < events.size(); ++f) {
      snprintf(buf, sizeof(buf), ",%d", nbase[f]);
      nbs += buf;
      snprintf(buf, sizeof(buf), ",%d", sbase[f]);
      sbs += buf;
    }
    s += nbs + sbs + "};\n";
  }
  s += "\n__device__ const int kFragUnitStart[] = {0";
  {
    int acc = 0, nsc = 0, not_ = 0, nq = 0;
    for (const auto& un : plan.units) {
      acc += (int)un.size();
      snprintf(buf, sizeof(buf), ",%d", acc);
      s += buf;
      for (size_t k = 0; k < un.size(); ++k) {
        const JitUnit& u = un[k];
        snprintf(buf, sizeof(buf), ",{%d,%d,%d,%d,%d,0,0,0}", u.ta, u.tb, u.off, u.br, u.koff);
        ud += buf;
        snprintf(buf, sizeof(buf), ",%zu", k);
        if (u.tc >= 0) {
          snprintf(buf, sizeof(buf), ",{%d,%d,%d,%d,%d,%d,%d,%d}", u.ta, u.tb, u.tc, u.td, u.brA, u.brB, u.br, u.off);
          qd += buf;
          ++nq;
        } else if (sh.scale && u.tb >= 0 && u.koff >= 0) {
          scu += buf;
          ++nsc;
        } else {
          snprintf(buf, sizeof(buf), ",{%d,%d,%d,%d,%d,0,0,0}", u.ta, u.tb, u.off, u.br, u.koff);
          otu += buf;
          ++not_;
        }
      }
      snprintf(buf, sizeof(buf), ",%d", nsc);
      sc += buf;
      snprintf(buf, sizeof(buf), ",%d", not_);
      ot += buf;
      snprintf(buf, sizeof(buf), ",%d", nq);
      qs += buf;
    }
  }
  s += ud + sc + scu + ot + otu + qs + qd + "};\n";
  const int CW = sh.CW, NW = sh.nw(), PW = sh.PW;
  snprintf(buf, sizeof(buf), "#define CLS_ %d\n#define CT_ %d\n#define SOA_ %d\n#define DC_ %d\n#define DCW_ %d\n",
           sh.cls ? 1 : 0, sh.cls ? 1 : C, sh.soa ? 1 : 0, sh.dc ? 1 : 0, sh.dc ? sh.dcw : 1);
  s += buf;
  snprintf(buf, sizeof(buf),
           "#define C_ %d\n#define CW_ %d\n#define NW_ %d\n#define PW_ %d\n#define G_ %d\n#define NWT_ %d\n"
           "#define U_ %d\n#define NT_ %d\n#define TD_ %d\n#define SC_ %s\n#define V_ (4 * CW_ * PW_)\n"
           "extern \"C\" __global__ __launch_bounds__(%d%s) void %s(JArgs a, const double* __restrict__ "
           "pmats, int frag_base%s) {\n",
           C, CW, NW, PW, sh.G, NW * sh.G, U, std::max(sh.NT, 1), std::max(sh.TD, 4), sh.scale ? "true" : "false",
           64 * NW * sh.G, minw_s.c_str(), jit_tree4_name(sh), sh.clk ? ", unsigned long long* __restrict__ clk_" : "");
  s += buf;
  // PLK_DEBUG_CLOCK (diagnostic build of the same program): thread 0 of every workgroup records
  // the shader clock counter (clock64) and the constant 100 MHz counter (wall_clock64) at its
  // start and end, so the host can tell the shader clock the launch ran at
  if (sh.clk) s += "  const unsigned long long clk_c0_ = clock64(), clk_w0_ = wall_clock64();\n";
  s += R"PLKJIT(  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* tab = lds;                                          // units: [C_][U_ or U_ * U_][4] each
  double* xch = tab + TD_;                                    // [2][PW_][NWT_][64] (rescale alternates)
  double* xch2 = xch + PW_ * NWT_ * 64;
  u8* code_lds = reinterpret_cast<u8*>(xch + (CLS_ ? 0 : (SC_ ? 2 : 1) * PW_ * NWT_ * 64)); // [G_][NT_][64 * PW_]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // (CLS_: the workgroup's class is blockIdx.z; TC0_ = the class of table class 0)
  const int c0 = CLS_ ? (int)blockIdx.z : (w % NW_) * CW_, g = w / NW_;
  const int TC0_ = CLS_ ? c0 : 0;
  const int frag = frag_base + (int)blockIdx.y;
  // dynamic super-block counter of this fragment (and class)
  unsigned* const sbc_ = a.sb_ctr + frag * (int)gridDim.z + (int)blockIdx.z;
  const int u0 = 1 + kFragUnitStart[frag], nu = kFragUnitStart[frag + 1] - kFragUnitStart[frag];
  // code staging: this thread's items (uint4 column j of group gg in unit k's code row;
  // JArgs::codes holds one row per unit, unit_codes_kernel), fixed over the super-blocks.
  // The codes of the next super-block are loaded into registers while this one computes.
  constexpr int NI_ = (G_ * NT_ * 4 * PW_ + 64 * NWT_ - 1) / (64 * NWT_);
  const uint4* ucodes = reinterpret_cast<const uint4*>(a.codes);
  const i64 row16 = a.n_pad / 16;
  i64 iu_[NI_]; int ic_[NI_], il_[NI_]; uint4 va_[NI_];
  _Pragma("unroll") for (int m = 0; m < NI_; ++m) {
    const int i = threadIdx.x + m * (64 * NWT_);
    const int gg = i / (nu * 4 * PW_), r = i - gg * (nu * 4 * PW_), k = r / (4 * PW_), j = r - k * (4 * PW_);
    const bool ok = i < G_ * nu * 4 * PW_;
    ic_[m] = ok ? gg * (64 * PW_) + 16 * j : 0x7fffffff;  // column in the super-block (none: past n_pad)
    iu_[m] = (i64)(u0 - 1 + k) * row16 + (ic_[m] >> 4);
    il_[m] = (gg * NT_ + k) * 4 * PW_ + j;
  }
  auto fetch_codes = [&](int sb_) {
    const i64 q0_ = (i64)sb_ * (64 * PW_ * G_);
    _Pragma("unroll") for (int m = 0; m < NI_; ++m)
      if (q0_ + ic_[m] < a.n_pad) va_[m] = ucodes[iu_[m] + (q0_ >> 4)];
  };
  // DC_: this wave's own patterns' codes (DCW_ 16-byte words per pattern: unit k is byte k),
  // next super-block's
  uint4 cv_[PW_][DCW_], cvn_[PW_][DCW_];
  const uint4* dcodes = reinterpret_cast<const uint4*>(a.codes) + (i64)frag * a.n_pad * DCW_;
  auto fetch_dc = [&](int sb_) {
    const i64 q0_ = (i64)sb_ * (64 * PW_ * G_);
    const i64 pp_ = (q0_ + g * (64 * PW_) < a.n_pad ? q0_ + g * (64 * PW_) : q0_) + lane;
    if (sb_ < a.n_sblocks)
      _Pragma("unroll") for (int pw = 0; pw < PW_; ++pw)
        _Pragma("unroll") for (int w_ = 0; w_ < DCW_; ++w_) cvn_[pw][w_] = dcodes[(pp_ + 64 * pw) * DCW_ + w_];
  };
  (void)cv_; (void)cvn_; (void)dcodes;
  // (issued before the table staging below: its loads overlap it)
  if (DC_) fetch_dc(blockIdx.x); else fetch_codes(blockIdx.x);
  // The fragment's P(t) matrices, touched with wide loads while the tables stage: the
  // traversal reads P(t) through scalar loads one contribution ahead, and their first touch
  // (the P(t) launch wrote them through another XCD's L2) made the first super-block ~12 us
  // slower on cfg5 (34 vs 22 us; steady state 19 us)
  // (with one class per wave (cfg2) the first super-block shows no such penalty and the
  // touch only lengthened the staging, so there it is left out)
  double ptouch_ = 0.0;
  if (CW_ > 1) {
    const int pb0 = 1 + kFragPStart[frag], npb = kFragPStart[frag + 1] - kFragPStart[frag];
    const double2* pp_ = reinterpret_cast<const double2*>(pmats);
    for (int i = threadIdx.x; i < npb * C_ * 8; i += 64 * NWT_) {
      const int k_ = i / (C_ * 8);
      ptouch_ += pp_[(i64)kFragPBr[pb0 + k_] * (C_ * 8) + (i - k_ * (C_ * 8))].x;
    }
  }
  if (SC_) {
    // rescaling contribution units: one (unit, row) per thread; each row all classes, the
    // cherry's joint check as rescale() makes it, then contrib<.., true>
    const int sc0 = 1 + kFragScStart[frag], nsc = kFragScStart[frag + 1] - kFragScStart[frag];
    for (int t = threadIdx.x; t < nsc * (U_ * U_); t += 64 * NWT_) {
      const int kk = t / (U_ * U_), r = t - kk * (U_ * U_);
      const UnitD ud = kUnitD[u0 + kScUnit[sc0 + kk]];
      double* dst = tab + ud.off;
      const double* ra = a.tipP + (i64)ud.ta * (C_ * U_ * 4);
      const double* rb = a.tipP + (i64)ud.tb * (C_ * U_ * 4);
      const int ca = r / U_, cb = r - ca * U_;
      double v[C_][4], m = 0.0;
      for (int c = 0; c < C_; ++c)
        for (int y = 0; y < 4; ++y) {
          v[c][y] = ra[(c * U_ + ca) * 4 + y] * rb[(c * U_ + cb) * 4 + y];
          m = fmax(m, v[c][y]);
        }
      const bool up = m > 0.0 && m < kScaleThr;
      for (int c = 0; c < C_; ++c) {
        if (up)
          for (int y = 0; y < 4; ++y) v[c][y] *= kScaleUp;
        for (int x = 0; x < 4; ++x) {
          const double* P = pmats + ((i64)ud.br * C_ + c) * 16 + 4 * x;
          double t2 = P[0] * v[c][0];
          t2 = __builtin_fma(P[1], v[c][1], t2);
          t2 = __builtin_fma(P[2], v[c][2], t2);
          t2 = __builtin_fma(P[3], v[c][3], t2);
          dst[c * (U_ * U_ * 4) + TABIX(U_ * U_, r, x)] = t2;
        }
      }
      reinterpret_cast<u8*>(tab + ud.koff)[r] = up ? 1 : 0;
    }
  }
  // the other tables: wave w stages units w, w + NWT_, ... of the fragment's other-unit list
  // (one dependent chain per unit and wave, the waves' chains overlap)
  const int ot0 = 1 + kFragOtherStart[frag], not_ = kFragOtherStart[frag + 1] - kFragOtherStart[frag];
  // (the next unit's record is loaded while this one's rows load and compute)
  UnitD ud_nx = kOtherD[w < not_ ? ot0 + w : 0];
  for (int ko = w; ko < not_; ko += NWT_) {
    const UnitD ud = ud_nx;
    // every field materialised here: one wait before the branches on them
    asm volatile("" ::"s"(ud.ta), "s"(ud.tb), "s"(ud.off), "s"(ud.br), "s"(ud.koff));
    if (ko + NWT_ < not_) ud_nx = kOtherD[ot0 + ko + NWT_];
    const int ta = ud.ta, tb = ud.tb;
    double* dst = tab + ud.off;
    const double* ra = a.tipP + (i64)ta * (C_ * U_ * 4) + TC0_ * (U_ * 4);
    if (tb < 0) {
      for (int i = lane; i < CT_ * U_ * 4; i += 64) {
        const int c = i / (U_ * 4), q = i - c * (U_ * 4);
        dst[c * (U_ * 4) + TABIX(U_, q >> 2, q & 3)] = ra[i];
      }
    } else {
      const double* rb = a.tipP + (i64)tb * (C_ * U_ * 4) + TC0_ * (U_ * 4);
      const int br = ud.br;  // (rescaling contribution units were staged above)
      // one row (class c, code pair ca, cb: 4 doubles) per lane, its operands loaded
      // together (16-byte loads), so a unit costs one load latency, not one per double
      for (int r = lane; r < CT_ * U_ * U_; r += 64) {
        const int c = r / (U_ * U_), q = r - c * (U_ * U_), ca = q / U_, cb = q - ca * U_;
        const double2* pa = reinterpret_cast<const double2*>(ra + (c * U_ + ca) * 4);
        const double2* pb = reinterpret_cast<const double2*>(rb + (c * U_ + cb) * 4);
        const double2 a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
        double v[4] = {a0.x * b0.x, a0.y * b0.y, a1.x * b1.x, a1.y * b1.y};
        double2* o0 = reinterpret_cast<double2*>(dst + c * (U_ * U_ * 4) + TABIX(U_ * U_, q, 0));
        double2* o1 = reinterpret_cast<double2*>(dst + c * (U_ * U_ * 4) + TABIX(U_ * U_, q, 2));
        if (br < 0) {
          *o0 = make_double2(v[0], v[1]);
          *o1 = make_double2(v[2], v[3]);
        } else {  // contrib<.., true>: the same operations in the same order
          const double2* P2 = reinterpret_cast<const double2*>(pmats + ((i64)br * C_ + TC0_ + c) * 16);
          double P[16];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const double2 pj = P2[j];
            P[2 * j] = pj.x;
            P[2 * j + 1] = pj.y;
          }
          double t[4];
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            t[x] = P[4 * x] * v[0];
            t[x] = __builtin_fma(P[4 * x + 1], v[1], t[x]);
            t[x] = __builtin_fma(P[4 * x + 2], v[2], t[x]);
            t[x] = __builtin_fma(P[4 * x + 3], v[3], t[x]);
          }
          *o0 = make_double2(t[0], t[1]);
          *o1 = make_double2(t[2], t[3]);
        }
      }
    }
  }
  if (CLS_) {
    // quad units: one (unit, row) per thread of the workgroup.  The interpreter's operations
    // in its order: each cherry's pair product and contrib<.., true> through the cherry's P,
    // Q's accumulator = contA, *= contB, then contrib<.., true> through P_Q.
    constexpr int U4_ = U_ * U_ * U_ * U_;
    const int q0_ = 1 + kFragQuadStart[frag], nq_ = kFragQuadStart[frag + 1] - kFragQuadStart[frag];
    auto pcon = [&](const double (&P)[16], const double (&v_)[4], double (&t_)[4]) {
      _Pragma("unroll") for (int x = 0; x < 4; ++x) {
        t_[x] = P[4 * x] * v_[0];
        t_[x] = __builtin_fma(P[4 * x + 1], v_[1], t_[x]);
        t_[x] = __builtin_fma(P[4 * x + 2], v_[2], t_[x]);
        t_[x] = __builtin_fma(P[4 * x + 3], v_[3], t_[x]);
      }
    };
    auto pload = [&](int br_, double (&P)[16]) {  // (br_ wave-uniform: scalar loads)
      const double* P1 = pmats + ((i64)br_ * C_ + c0) * 16;
      _Pragma("unroll") for (int j = 0; j < 16; ++j) P[j] = P1[j];
    };
    // One wave per quad (quads w, w + NWT_, ...), every load of the quad issued before its
    // arithmetic: the quad's record and its three P(t) (the two cherries', Q's) wave-uniform.
    // Phase 1: lanes [0, 2 U^2) form the two cherries' contribution rows (U^2 rows each) in the
    // code rows' LDS space (staged only at the first super-block); phase 2: the wave's lanes
    // form the quad rows from them.  The same operations per row as before (the interpreter's
    // order: each cherry's pair product and contrib<.., true> through the cherry's P, Q's
    // accumulator = contA, *= contB, then contrib<.., true> through P_Q).
    double* qtmp = reinterpret_cast<double*>(code_lds);
    for (int kk = w; kk < nq_; kk += NWT_) {
      const QuadD qd_ = kQuadD[q0_ + kk];
      double PA[16], PB[16], PQ[16];
      pload(qd_.brA, PA);
      pload(qd_.brB, PB);
      pload(qd_.brQ, PQ);
      for (int hr = lane; hr < 2 * U_ * U_; hr += 64) {
        const int which = hr / (U_ * U_), r = hr - which * (U_ * U_), ca = r / U_, cb = r - ca * U_;
        const int t1 = which ? qd_.tc : qd_.ta, t2 = which ? qd_.td : qd_.tb;
        const double2* pa = reinterpret_cast<const double2*>(a.tipP + ((i64)t1 * C_ + c0) * (U_ * 4) + ca * 4);
        const double2* pb = reinterpret_cast<const double2*>(a.tipP + ((i64)t2 * C_ + c0) * (U_ * 4) + cb * 4);
        const double2 a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
        const double v[4] = {a0.x * b0.x, a0.y * b0.y, a1.x * b1.x, a1.y * b1.y};
        double P[16], o[4];
        _Pragma("unroll") for (int j = 0; j < 16; ++j) P[j] = which ? PB[j] : PA[j];
        pcon(P, v, o);
        double2* od = reinterpret_cast<double2*>(qtmp + ((i64)(2 * kk) * (U_ * U_) + hr) * 4);
        od[0] = make_double2(o[0], o[1]);
        od[1] = make_double2(o[2], o[3]);
      }
      // (the rows just written are read by other lanes of this wave)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      _Pragma("unroll") for (int r = lane; r < U4_; r += 64) {
        const int ab = r / (U_ * U_), cd = r - ab * (U_ * U_);
        const double2* pa = reinterpret_cast<const double2*>(qtmp + ((i64)(2 * kk) * (U_ * U_) + ab) * 4);
        const double2* pb = reinterpret_cast<const double2*>(qtmp + ((i64)(2 * kk + 1) * (U_ * U_) + cd) * 4);
        const double2 a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
        double acc[4] = {a0.x, a0.y, a1.x, a1.y}, o[4];
        acc[0] *= b0.x; acc[1] *= b0.y; acc[2] *= b1.x; acc[3] *= b1.y;
        pcon(PQ, acc, o);
        *reinterpret_cast<double2*>(tab + qd_.off + TABIX(U4_, QROW_(r), 0)) = make_double2(o[0], o[1]);
        *reinterpret_cast<double2*>(tab + qd_.off + TABIX(U4_, QROW_(r), 2)) = make_double2(o[2], o[3]);
      }
    }
  }
  const CPd pm = (CPd)(pmats + c0 * 16);
  const double* trow = tab + (CLS_ ? 0 : c0 * (U_ * 4));         // single-tip units
  const double* trow2 = tab + (CLS_ ? 0 : c0 * (U_ * U_ * 4));   // pair units
  const double* trow4 = tab;                                      // quad units (CLS_ only)
  (void)xch; (void)xch2; (void)trow; (void)trow2; (void)trow4;
// unit k: codes of the lane's patterns (4 per int), then their table rows (R rows per
// class at OFF doubles from the class base TB)
#define CODEF(Q, k) { Q = 0; _Pragma("unroll") for (int pw_ = 0; pw_ < PW_; ++pw_) \
    Q |= (DC_ ? (int)((cvw(cv_[pw_][(k) >> 4], ((k) >> 2) & 3) >> (8 * ((k) & 3))) & 255) : (int)crow[(k) * (64 * PW_) + 64 * pw_]) << (8 * pw_); }
#define ROWF(F, TB, OFF, R, Q) { _Pragma("unroll") for (int pw_ = 0; pw_ < PW_; ++pw_) { \
    const double* r0_ = TB + (OFF) + TABIX(R, ((Q) >> (8 * pw_)) & 255, 0); \
    _Pragma("unroll") for (int cw_ = 0; cw_ < CW_; ++cw_) { \
      const double2* r_ = reinterpret_cast<const double2*>(r0_ + cw_ * ((R) * 4)); \
      const double2 x_ = r_[0], y_ = r_[SOA_ ? (R) : 1]; const int v_ = 4 * (pw_ * CW_ + cw_); \
      F[v_] = x_.x; F[v_ + 1] = x_.y; F[v_ + 2] = y_.x; F[v_ + 3] = y_.y; } } }
#define TIPF(F, Q, k, TB, OFF, R) { CODEF(Q, k) ROWF(F, TB, OFF, R, Q) }
// count bytes of a rescaling contribution unit
#define KTF(K, KOFF, Q) { _Pragma("unroll") for (int pw_ = 0; pw_ < PW_; ++pw_) \
    K[pw_] += (int)reinterpret_cast<const u8*>(tab + (KOFF))[((Q) >> (8 * pw_)) & 255]; }
// (slot numbers are laundered: otherwise every slot's base address is hoisted out of the
// super-block loop into its own SGPR pair, and they spill)
#define LOADF(F, FK, slot) { const i64 sl_ = (i64)launder_s(slot); \
    const double* L_ = a.partials + sl_ * a.slot_stride + toff; \
    _Pragma("unroll") for (int pw_ = 0; pw_ < PW_; ++pw_) { \
      _Pragma("unroll") for (int i_ = 0; i_ < 4 * CW_; ++i_) F[4 * CW_ * pw_ + i_] = L_[64 * pw_ + (i64)i_ * kTile]; \
      if (SC_) FK[pw_] = a.scale[sl_ * a.n_pad + p + 64 * pw_]; } }
#define SB __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::"v"(ptouch_));  // (keeps the touch loads)
  // Super-block order.  Static: blockIdx.x, + gridDim.x, ...  Dynamic (a.dyn): the first is
  // blockIdx.x, every later one comes from the fragment's counter -- thread 0 takes the index
  // of the super-block after the next one while this one computes, so the atomic's latency is
  // hidden; a workgroup stops taking after its first index past the end.  The counter starts
  // the launch at 0 (the exit ticket below resets it).  Which workgroup computes a
  // super-block does not change its results.
  __shared__ int sb_next_lds[2];  // (DC_: alternating, one barrier per super-block)
  unsigned sb_pend = 0;
  int it_ = 0;
  if (a.dyn && threadIdx.x == 0)
    sb_pend = __hip_atomic_fetch_add(sbc_, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int sb = blockIdx.x, sb_nx = 0; sb < a.n_sblocks; sb = sb_nx) {
    const i64 q0 = (i64)sb * (64 * PW_ * G_);
    // super-blocks of G_ groups; in a ragged last one, groups past n_pad recompute group 0
    // (in bounds everywhere) and store nothing
    const bool gv = q0 + g * (64 * PW_) < a.n_pad;
    const i64 p0 = gv ? q0 + g * (64 * PW_) : q0, p = p0 + lane;
    const u8* crow = code_lds + (gv ? g : 0) * (NT_ * 64 * PW_) + lane;
    (void)crow;
    const i64 toff = (p >> 7) * (C_ * 4 * kTile) + (i64)c0 * 4 * kTile + (p & (kTile - 1));
    (void)toff;
    const int sl_ = DC_ ? (it_ & 1) : 0;
    if (DC_) {
      _Pragma("unroll") for (int pw = 0; pw < PW_; ++pw)
        _Pragma("unroll") for (int w_ = 0; w_ < DCW_; ++w_) cv_[pw][w_] = cvn_[pw][w_];
    } else {
      __syncthreads();  // the previous super-block is done with code_lds / xch (and tab is staged)
      _Pragma("unroll") for (int m = 0; m < NI_; ++m)
        if (q0 + ic_[m] < a.n_pad) reinterpret_cast<uint4*>(code_lds)[il_[m]] = va_[m];
    }
    if (a.dyn && threadIdx.x == 0) {  // (an index outside this launch's range ends the loop)
      const unsigned d_ = sb_pend;
      sb_next_lds[sl_] = d_ < (unsigned)(a.n_sblocks - (int)gridDim.x) ? (int)gridDim.x + (int)d_ : a.n_sblocks;
    }
    __syncthreads();  // (DC_: also the tables' staging before the first super-block)
    sb_nx = a.dyn ? __builtin_amdgcn_readfirstlane(sb_next_lds[sl_]) : sb + (int)gridDim.x;
    ++it_;
    if (a.dyn && threadIdx.x == 0 && sb_nx < a.n_sblocks)
      sb_pend = __hip_atomic_fetch_add(sbc_, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (DC_) fetch_dc(sb_nx); else fetch_codes(sb_nx);
)PLKJIT";
  int max_level = 0;
  for (const auto& ev : events)
    for (const JitEvent& e : ev) max_level = std::max(max_level, e.level);
  for (int d = 0; d <= max_level; ++d) {
    snprintf(buf, sizeof(buf), "    double A%d[V_]; int K%d[PW_] = {}; (void)K%d;\n", d, d, d);
    s += buf;
  }
  for (int r = 0; r <= L; ++r) {
    snprintf(buf, sizeof(buf), "    double F%d[V_]; int FK%d[PW_] = {}; (void)FK%d; int Q%d = 0; (void)Q%d;\n", r, r,
             r, r, r);
    s += buf;
  }
  s += "    switch (frag) {\n";
  for (size_t f = 0; f < events.size(); ++f) {
    if (leader[f] != (int)f) continue;
    const std::vector<JitEvent>& ev = events[f];
    std::vector<int> slot(ev.size(), -1), fetchers;
    for (size_t i = 0; i < ev.size(); ++i)
      if (ev[i].op == T_TIP || ev[i].op == T_LOAD) {
        slot[i] = (int)(fetchers.size() % (size_t)(L + 1));
        fetchers.push_back((int)i);
      }
    auto pref = [&](size_t i) -> std::string {  // P operand of event i (relative to the node base)
      snprintf(buf, sizeof(buf), "pmf_ + %lld", (long long)(ev[i].b - nbase[f]) * C * 16);
      return buf;
    };
    auto sref = [&](int a) -> std::string {  // a slot (relative to the slot base)
      return "sb_ + " + std::to_string(a - sbase[f]);
    };
    // Two-stage operand pipeline (L >= 2): a tip's code is read L fetchers ahead (and a
    // materialised child partial is loaded from HBM L ahead), its table row one ahead, so
    // neither the code -> row dependency nor HBM latency sits in front of the FMAs.
    auto emit_stage1 = [&](int i) {
      const JitEvent& e = ev[(size_t)i];
      if (e.op == T_TIP)
        snprintf(buf, sizeof(buf), "      CODEF(Q%d, %d)\n", slot[(size_t)i], e.a);
      else
        snprintf(buf, sizeof(buf), "      LOADF(F%d, FK%d, %s)\n", slot[(size_t)i], slot[(size_t)i], sref(e.a).c_str());
      s += buf;
    };
    auto unit_args = [&](const JitEvent& e) -> std::string {  // TB, OFF, R of a unit
      const JitUnit& u = plan.units[f][(size_t)e.a];
      char ubuf[96];
      snprintf(ubuf, sizeof(ubuf), "%s, %d, %d", u.tb < 0 ? "trow" : u.tc >= 0 ? "trow4" : "trow2", u.off,
               u.tb < 0 ? U : u.tc >= 0 ? U * U * U * U : U * U);
      return ubuf;
    };
    auto emit_stage2 = [&](int i) {
      const JitEvent& e = ev[(size_t)i];
      if (e.op != T_TIP) return;
      snprintf(buf, sizeof(buf), "      ROWF(F%d, %s, Q%d)\n", slot[(size_t)i], unit_args(e).c_str(), slot[(size_t)i]);
      s += buf;
    };
    auto emit_fetch = [&](int i) {
      const JitEvent& e = ev[(size_t)i];
      if (e.op == T_TIP)
        snprintf(buf, sizeof(buf), "      TIPF(F%d, Q%d, %d, %s)\n", slot[(size_t)i], slot[(size_t)i], e.a,
                 unit_args(e).c_str());
      else
        snprintf(buf, sizeof(buf), "      LOADF(F%d, FK%d, %s)\n", slot[(size_t)i], slot[(size_t)i], sref(e.a).c_str());
      s += buf;
    };
    // One pass over the fragment.  exact: the per-node joint rescale of the other
    // kernels.  !exact (scaling only): no rescale, but every node the exact pass would
    // check raises `dng` when its own-class max is below the threshold -- the joint
    // max can then be below it too; otherwise the joint max is >= the threshold at
    // every check, no rescale would happen, and this pass IS the exact result.
    // classes in the wave with pipelined P(t): the fragment's contributions form one
    // stream of class loads (contrib_s), the first loaded ahead of the body
    const bool pstream = sh.ppipe && (CW > 1 || sh.ps1);
    std::vector<size_t> cev;  // events with a contribution, in order
    for (size_t i = 0; i < ev.size(); ++i)
      if (ev[i].op == T_LOAD || ev[i].op == T_ASCEND) cev.push_back(i);
    auto emit_body = [&](bool exact) {
      s += "      kzero(K0);\n";
      size_t kc = 0;   // contributions emitted
      int pbase = 0;   // buffer of the next contribution's class 0
      if (pstream && !cev.empty()) {
        snprintf(buf, sizeof(buf), "      double pbuf[2][16]; pload(pbuf[0], %s); ptouch(pbuf[0]);\n",
                 pref(cev[0]).c_str());
        s += buf;
      }
      auto contrib_line = [&](size_t i, const char* set, const std::string& dst, const std::string& src) {
        const std::string pr = pref(i);
        if (!pstream) {
          snprintf(buf, sizeof(buf), "      contrib<CW_, PW_, %s>(%s, %s, %s);\n", set, dst.c_str(), src.c_str(),
                   pr.c_str());
        } else {
          const bool next = kc + 1 < cev.size();
          const std::string pn = next ? pref(cev[kc + 1]) : pr;
          snprintf(buf, sizeof(buf), "      contrib_s<CW_, PW_, %s, %d, %s>(%s, %s, %s, %s, pbuf);\n", set, pbase,
                   next ? "true" : "false", dst.c_str(), src.c_str(), pr.c_str(), pn.c_str());
          pbase = (pbase + CW) & 1;
        }
        ++kc;
        s += buf;
      };
      std::vector<char> fresh((size_t)max_level + 1, 0);
      fresh[0] = 1;
      size_t nf = 0;
      size_t n1 = 0, n2 = 0;  // two-stage pipeline: stage-1 / stage-2 fetches emitted
      if (L >= 2) {
        for (; n1 < fetchers.size() && n1 < (size_t)L; ++n1) emit_stage1(fetchers[n1]);
        const size_t rd = (size_t)std::max(1, std::min(sh.RD, L));  // (a slot's row is used before its reuse)
        for (; n2 < fetchers.size() && n2 < rd; ++n2) emit_stage2(fetchers[n2]);
      } else {
        for (; nf < fetchers.size() && nf < (size_t)L; ++nf) emit_fetch(fetchers[nf]);
      }
      s += "      SB\n";
      int n_rescale = 0;  // rescales alternate exchange buffers (the superblock barrier resets)
      auto check_line = [&](int d) {
        if (exact)
          snprintf(buf, sizeof(buf), "      rescale<C_, CW_, PW_, NWT_>(A%d, K%d, %s, w, g);\n", d, d,
                   (n_rescale++ & 1) ? "xch2" : "xch");
        else
          snprintf(buf, sizeof(buf), "      flag_risky(dng, A%d);\n", d);
        s += buf;
      };
      for (size_t i = 0; i < ev.size(); ++i) {
        const JitEvent& e = ev[i];
        if (e.op == T_TIP || e.op == T_LOAD) {
          if (L >= 2) {
            if (n1 < fetchers.size()) emit_stage1(fetchers[n1++]);
            if (n2 < fetchers.size()) emit_stage2(fetchers[n2++]);
          } else if (nf < fetchers.size()) {
            emit_fetch(fetchers[nf++]);
          }
          const char* set = fresh[(size_t)e.level] ? "true" : "false";
          if (e.op == T_TIP) {
            snprintf(buf, sizeof(buf), "      tipmul<V_, %s>(A%d, F%d);\n", set, e.level, slot[i]);
            const JitUnit& u = plan.units[f][(size_t)e.a];
            if (u.koff >= 0) {
              s += buf;
              snprintf(buf, sizeof(buf), "      KTF(K%d, %d, Q%d)\n", e.level, u.koff, slot[i]);
            }
            s += buf;
          } else {
            contrib_line(i, set, "A" + std::to_string(e.level), "F" + std::to_string(slot[i]));
          }
          if (sh.pin) {
            snprintf(buf, sizeof(buf), "      pin(A%d);\n", e.level);
            s += buf;
          }
          fresh[(size_t)e.level] = 0;
          if (e.op == T_LOAD && sh.scale) {
            snprintf(buf, sizeof(buf), "      kadd(K%d, FK%d);\n", e.level, slot[i]);
            s += buf;
          }
          s += "      SB\n";
        } else if (e.op == T_DESCEND) {
          fresh[(size_t)e.level] = 1;
          snprintf(buf, sizeof(buf), "      kzero(K%d);\n", e.level);
          s += buf;
        } else if (e.op == T_ASCEND) {
          const int dd = e.level;
          if (e.b >= 0) {
            if (sh.scale) check_line(dd);
            if (e.a >= 0) {
              snprintf(buf, sizeof(buf), "      store<CW_, PW_, SC_>(a, %s, toff, p, c0, A%d, K%d, gv);\n",
                       sref(e.a).c_str(), dd, dd);
              s += buf;
            }
          }
          contrib_line(i, fresh[(size_t)dd - 1] ? "true" : "false", "A" + std::to_string(dd - 1),
                       "A" + std::to_string(dd));
          if (sh.pin) {
            snprintf(buf, sizeof(buf), "      pin(A%d);\n", dd - 1);
            s += buf;
          }
          fresh[(size_t)dd - 1] = 0;
          if (sh.scale) {
            snprintf(buf, sizeof(buf), "      kadd(K%d, K%d);\n", dd - 1, dd);
            s += buf;
          }
          s += "      SB\n";
        } else {  // T_ROOT
          if (sh.scale) check_line(0);
          if (e.a >= 0) {
            snprintf(buf, sizeof(buf), "      store<CW_, PW_, SC_>(a, %s, toff, p, c0, A0, K0, gv);\n",
                     sref(e.a).c_str());
            s += buf;
          }
          if (e.b)
            s += sh.cls ? "      reduce_root_cls<PW_>(a, A0, c0, p, gv);\n"
                        : "      reduce_root<C_, CW_, PW_, NWT_, SC_>(a, A0, K0, xch, w, g, c0, p0, p, gv);\n";
        }
      }
    };
    for (size_t q = f; q < events.size(); ++q)
      if (leader[q] == (int)f) {
        snprintf(buf, sizeof(buf), "    case %zu:\n", q);
        s += buf;
      }
    s += "    {\n      const CPd pmf_ = pm + (i64)kFragNB[frag + 1] * (C_ * 16);\n"
         "      const int sb_ = __builtin_amdgcn_readfirstlane(kFragSB[frag + 1]); (void)pmf_; (void)sb_;\n";
    emit_body(true);
    s += "    } break;\n";
  }
  s += "    default: break;\n    }\n  }\n";
  if (sh.clk == 1)
    s += "  if (threadIdx.x == 0) {\n"
         "    unsigned long long* q_ = clk_ + 4 * (((unsigned long long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + "
         "blockIdx.x);\n"
         "    const unsigned long long c1_ = clock64(), w1_ = wall_clock64();\n"
         "    q_[0] = clk_c0_; q_[1] = clk_w0_; q_[2] = c1_; q_[3] = w1_;\n  }\n";
  // Exit ticket (dynamic super-blocks): thread 0 of every workgroup takes one ticket after its
  // last super-block -- its own counter atomics have returned by then -- and the last one
  // leaves the launch's counters and the ticket counter at 0 for the next launch, so the host
  // keeps no copy of them.  (Forming the block sums in the last workgroup as well was measured
  // 8 us slower per cfg2 traversal than wave_sums_to_blocks: the wave sums must then cross the
  // XCDs' L2s, as sc1 stores and loads or behind L2 write-backs -- profiles/r05/ab_runs.md.)
  s += R"PLKJIT(  if (a.exit_ctr && threadIdx.x == 0) {
    const unsigned t_ = __hip_atomic_fetch_add(a.exit_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t_ == gridDim.x * gridDim.y * gridDim.z - 1u) {
      for (unsigned f_ = 0; f_ < gridDim.y * gridDim.z; ++f_)
        __hip_atomic_store(a.sb_ctr + frag_base * gridDim.z + f_, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.exit_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
)PLKJIT";
  if (sh.clk == 2) {
    // PLK_DEBUG_CLOCK=2: the end stamp is taken where the super-block loop starts (the prologue:
    // code fetch, table staging, quad build), not at the kernel's end.  (Inserted into the
    // generated text, so that the ordinary programs' sources -- and their cached code -- do not change.)
    const std::string anchor = "  for (int sb = blockIdx.x, sb_nx = 0; sb < a.n_sblocks; sb = sb_nx) {";
    const size_t at = s.find(anchor);
    if (at != std::string::npos)
      s.insert(at, "  if (threadIdx.x == 0) { unsigned long long* q_ = clk_ + 4 * (((unsigned long long)blockIdx.z * "
                   "gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x); const unsigned long long c1_ = clock64(), w1_ = "
                   "wall_clock64(); q_[0] = clk_c0_; q_[1] = clk_w0_; q_[2] = c1_; q_[3] = w1_; }\n");
  }
  return s;
}

}  // namespace plk
