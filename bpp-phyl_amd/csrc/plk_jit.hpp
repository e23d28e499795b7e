// plk_jit.hpp -- tree-specialised fused traversal for 4-state models (gfx950).
//
// The interpreter in plk_tree4.hpp walks a tree program one event at a time: every
// event costs a scalar load of its program word, a compare-and-branch decode, 64-bit
// address arithmetic on the scalar unit and a dependent scalar load of P(t) -- all on
// the critical path of a wave that then issues only ~20 fp64 VALU instructions.
// Counters on cfg2 (64 taxa, GTR+G4): per wave ~4.7k SALU + 1.4k branches next to
// ~4.7k VALU, 42 % of wave cycles parked in s_waitcnt, VALU busy ~14 %.
//
// Here the same program (fragments and tiers from build_tree4_program) is emitted as
// straight-line HIP source -- one `case` per fragment -- and compiled once per
// (topology, C, flags) with hiprtc for gfx950.  Every P(t) address becomes a constant
// offset from one wave-uniform base, so the compiler issues the s_loads early and
// overlaps them with the previous events' FMAs; there is no decode, no program fetch
// and no branch in a fragment.  The arithmetic of every event is exactly the
// interpreter's (same helpers, same operation order), so results are bitwise those
// of tree4_kernel<1, DM, SCALE>.  Compiled modules are cached per process, keyed by
// the generated source (plk.hip: jit_function).
#pragma once

#include <string>
#include <vector>

#include "plk_tree4.hpp"

namespace plk {

// Device helpers of the generated kernels (hiprtc compiles them with the program).
// They restate contribute / rescale / store_partial / the fused root reduction of
// plk_tree4.hpp for one class per wave.
static const char* kJitPrelude = R"PLKJIT(
typedef unsigned char u8;
typedef long long i64;
typedef int i32;
typedef __attribute__((address_space(4))) const double* CPd;
#define kTile 128
__device__ const double kScaleUp = 115792089237316195423570985008687907853269984665640564039457584007913129639936.0;
__device__ const double kScaleThr = 1.0 / 115792089237316195423570985008687907853269984665640564039457584007913129639936.0;
#define kLn2x256 177.44567822334599921

struct JArgs {
  double* partials; i32* scale; const u8* codes; const double* init; const double* weights;
  const double* pi; const double* probs; double* site_lnl; double* wave_sums;
  i64 slot_stride; i64 n_pad; i64 n_patterns; i32 n_codes; i32 n_tips; i32 guard; i32 pad_;
};

__device__ __forceinline__ void one(double (&v)[4]) { v[0] = 1.0; v[1] = 1.0; v[2] = 1.0; v[3] = 1.0; }

// dst[x] *= sum_y P[x][y] src[y]   (P row-major, this wave's class)
__device__ __forceinline__ void contrib(double (&dst)[4], const double (&src)[4], CPd P) {
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    double s = P[4 * x + 0] * src[0];
    s = __builtin_fma(P[4 * x + 1], src[1], s);
    s = __builtin_fma(P[4 * x + 2], src[2], s);
    s = __builtin_fma(P[4 * x + 3], src[3], s);
    dst[x] *= s;
  }
}

__device__ __forceinline__ void rescale(double (&v)[4], int& cnt, double* xmax, int nw) {
  double m = 0.0;
#pragma unroll
  for (int i = 0; i < 4; ++i) m = fmax(m, v[i]);
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
    for (int i = 0; i < 4; ++i) v[i] *= kScaleUp;
    cnt += 1;
  }
}

template <int C, bool SCALE>
__device__ __forceinline__ void store(const JArgs& a, int slot, i64 p, int c0, const double (&v)[4], int cnt) {
  const i64 tile = p >> 7, q = p & (kTile - 1);
  double* dst = a.partials + (i64)slot * a.slot_stride + tile * (C * 4 * kTile) + (i64)c0 * 4 * kTile + q;
#pragma unroll
  for (int i = 0; i < 4; ++i) __builtin_nontemporal_store(v[i], dst + (i64)i * kTile);
  if (SCALE && c0 == 0) a.scale[(i64)slot * a.n_pad + p] = cnt;
}

template <int C, bool SCALE>
__device__ __forceinline__ void reduce_root(const JArgs& a, const double (&acc)[4], int cnt, double* xch, int c0, i64 p0,
                                            i64 p) {
  const int lane = threadIdx.x & 63;
  double lc = 0.0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
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
  if (c0 == 0) {
    double l = 0.0;
    for (int c = 0; c < C; ++c) {
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
)PLKJIT";

// Host mirror of JArgs (field order and types must match the prelude).
struct JArgs {
  double* partials;
  int32_t* scale;
  const uint8_t* codes;
  const double* init;
  const double* weights;
  const double* pi;
  const double* probs;
  double* site_lnl;
  double* wave_sums;
  int64_t slot_stride;
  int64_t n_pad;
  int64_t n_patterns;
  int32_t n_codes;
  int32_t n_tips;
  int32_t guard;
  int32_t pad_;
};

// Emit the kernel for a tree program.  `prog` / `starts` are build_tree4_program's
// words and fragment start offsets in tier order (fragment id = blockIdx.y + base).
//
// Each fragment is a list of events; an event has a FETCH part (tip code -> init row
// from LDS, or a materialised child partial from HBM) and a COMPUTE part (the
// contribution into its level).  The fetch of event i + L is emitted next to the
// compute of event i, inside one scheduling region (regions are closed with
// sched_barrier), so the LDS / HBM latency of the operands hides behind L events of
// FMAs while the register footprint stays bounded (a ring of L + 1 operand vectors).
// Without the regions the scheduler hoists every fetch of the fragment to its start
// and spills.
struct JitEvent {
  int op;     // T_TIP, T_LOAD, T_DESCEND, T_ASCEND (level >= 1), T_ROOT
  int level;  // accumulator level the event works on
  int a, b;   // program word fields
};

inline std::string jit_tree4_source(const std::vector<TInstr>& prog, const std::vector<int32_t>& starts, int C,
                                    bool scale, bool stage_codes, int L) {
  std::string s;
  s.reserve(96 * prog.size() + 8192);
  s += kJitPrelude;
  char buf[320];
  snprintf(buf, sizeof(buf),
           "\nextern \"C\" __global__ __launch_bounds__(256) void plk_jit_tree4(JArgs a, const double* __restrict__ "
           "pmats, int frag_base) {\n#define C_ %d\n#define SC_ %s\n#define STG_ %d\n",
           C, scale ? "true" : "false", stage_codes ? 1 : 0);
  s += buf;
  s += R"PLKJIT(  extern __shared__ __attribute__((aligned(16))) double lds[];
  double* init_lds = lds;
  double* xch = lds + ((a.n_codes * 4 + 1) & ~1);
  u8* code_lds = reinterpret_cast<u8*>(xch + 4 * 64);
  const int nw = C_;
  const int lane = threadIdx.x & 63;
  const int c0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const i64 p0 = (i64)blockIdx.x * 64;
  const i64 p = p0 + lane;
  for (int i = threadIdx.x; i < a.n_codes * 4; i += blockDim.x) init_lds[i] = a.init[i];
  if (STG_) {
    for (int i = threadIdx.x; i < a.n_tips * 4; i += blockDim.x) {
      const int t = i >> 2, j = i & 3;
      reinterpret_cast<uint4*>(code_lds)[i] = *reinterpret_cast<const uint4*>(a.codes + (i64)t * a.n_pad + p0 + 16 * j);
    }
  }
  __syncthreads();
  const CPd pm = (CPd)(pmats + c0 * 16);
  const i64 tile_off = (p >> 7) * (C_ * 4 * kTile) + (i64)c0 * 4 * kTile + (p & (kTile - 1));
  (void)nw; (void)xch; (void)tile_off;
#define TIPF(F, t) { const int code_ = STG_ ? code_lds[(t) * 64 + lane] : a.codes[(i64)(t) * a.n_pad + p]; \
    const double2* iv_ = reinterpret_cast<const double2*>(init_lds + code_ * 4); const double2 x_ = iv_[0], y_ = iv_[1]; \
    F[0] = x_.x; F[1] = x_.y; F[2] = y_.x; F[3] = y_.y; }
#define LOADF(F, FK, slot) { const double* L_ = a.partials + (i64)(slot) * a.slot_stride + tile_off; \
    F[0] = L_[0]; F[1] = L_[kTile]; F[2] = L_[2 * kTile]; F[3] = L_[3 * kTile]; \
    if (SC_) FK = a.scale[(i64)(slot) * a.n_pad + p]; }
#define SB __builtin_amdgcn_sched_barrier(0);
)PLKJIT";
  int max_level = 0;
  {
    int lvl = 0;
    for (const TInstr& w : prog) {
      if (w.op == T_DESCEND) max_level = std::max(max_level, ++lvl);
      else if (w.op == T_ASCEND && lvl > 0) --lvl;
      else if (w.op == T_ROOT) lvl = 0;
    }
  }
  for (int d = 0; d <= max_level; ++d) {
    snprintf(buf, sizeof(buf), "  double A%d[4]; int K%d = 0; (void)K%d;\n", d, d, d);
    s += buf;
  }
  for (int r = 0; r <= L; ++r) {
    snprintf(buf, sizeof(buf), "  double F%d[4]; int FK%d = 0; (void)FK%d;\n", r, r, r);
    s += buf;
  }
  s += "  switch (frag_base + (int)blockIdx.y) {\n";
  std::vector<JitEvent> ev;
  for (size_t f = 0; f < starts.size(); ++f) {
    ev.clear();
    int d = 0;
    for (size_t i = (size_t)starts[f];; ++i) {
      const TInstr& w = prog[i];
      if (w.op == T_TIP || w.op == T_LOAD) {
        ev.push_back({w.op, d, w.a, w.b});
      } else if (w.op == T_DESCEND) {
        ++d;
        ev.push_back({T_DESCEND, d, 0, 0});
      } else if (w.op == T_ASCEND) {
        if (d == 0) continue;  // fragment root: finished by ROOT
        ev.push_back({T_ASCEND, d, w.a, w.b});
        --d;
      } else if (w.op == T_ROOT) {
        ev.push_back({T_ROOT, 0, w.a, w.b});
        break;
      }
    }
    // fetching events (TIP / LOAD) get ring slots in order
    std::vector<int> slot(ev.size(), -1), fetchers;
    for (size_t i = 0; i < ev.size(); ++i)
      if (ev[i].op == T_TIP || ev[i].op == T_LOAD) {
        slot[i] = (int)(fetchers.size() % (size_t)(L + 1));
        fetchers.push_back((int)i);
      }
    auto emit_fetch = [&](int i) {
      const JitEvent& e = ev[(size_t)i];
      if (e.op == T_TIP)
        snprintf(buf, sizeof(buf), "    TIPF(F%d, %d)\n", slot[(size_t)i], e.a);
      else
        snprintf(buf, sizeof(buf), "    LOADF(F%d, FK%d, %d)\n", slot[(size_t)i], slot[(size_t)i], e.a);
      s += buf;
    };
    snprintf(buf, sizeof(buf), "  case %zu: {\n    one(A0); K0 = 0;\n", f);
    s += buf;
    size_t nf = 0;  // fetches emitted
    for (; nf < fetchers.size() && nf < (size_t)L; ++nf) emit_fetch(fetchers[nf]);
    s += "    SB\n";
    size_t done_fetchers = 0;
    for (size_t i = 0; i < ev.size(); ++i) {
      const JitEvent& e = ev[i];
      const long long off = (long long)e.b * C * 16;
      if (e.op == T_TIP || e.op == T_LOAD) {
        // keep L fetches in flight: issue the one L events ahead of this fetcher
        if (nf < fetchers.size()) emit_fetch(fetchers[nf++]);
        snprintf(buf, sizeof(buf), "    contrib(A%d, F%d, pm + %lld);\n", e.level, slot[i], off);
        s += buf;
        if (e.op == T_LOAD && scale) {
          snprintf(buf, sizeof(buf), "    K%d += FK%d;\n", e.level, slot[i]);
          s += buf;
        }
        ++done_fetchers;
        s += "    SB\n";
      } else if (e.op == T_DESCEND) {
        snprintf(buf, sizeof(buf), "    one(A%d); K%d = 0;\n", e.level, e.level);
        s += buf;
      } else if (e.op == T_ASCEND) {
        const int dd = e.level;
        if (e.b >= 0) {
          if (scale) {
            snprintf(buf, sizeof(buf), "    rescale(A%d, K%d, xch, nw);\n", dd, dd);
            s += buf;
          }
          if (e.a >= 0) {
            snprintf(buf, sizeof(buf), "    store<C_, SC_>(a, %d, p, c0, A%d, K%d);\n", e.a, dd, dd);
            s += buf;
          }
        }
        snprintf(buf, sizeof(buf), "    contrib(A%d, A%d, pm + %lld);\n", dd - 1, dd, off);
        s += buf;
        if (scale) {
          snprintf(buf, sizeof(buf), "    K%d += K%d;\n", dd - 1, dd);
          s += buf;
        }
        s += "    SB\n";
      } else {  // T_ROOT
        if (scale) s += "    rescale(A0, K0, xch, nw);\n";
        if (e.a >= 0) {
          snprintf(buf, sizeof(buf), "    store<C_, SC_>(a, %d, p, c0, A0, K0);\n", e.a);
          s += buf;
        }
        if (e.b) s += "    reduce_root<C_, SC_>(a, A0, K0, xch, c0, p0, p);\n";
      }
    }
    s += "  } break;\n";
  }
  s += "  default: break;\n  }\n#undef C_\n#undef SC_\n#undef STG_\n}\n";
  return s;
}

}  // namespace plk
