// plk_exchange.hpp -- host-side bookkeeping of the multi-rank lnL exchange.
//
// Under a communicator (plk_comm_init) every rank holds a contiguous, 4096-aligned range of
// the site patterns; the lnL they share is the sum the reference forms over all sites
// (RNonHomogeneousTreeLikelihood::getLogLikelihood, L/RNonHomogeneousTreeLikelihood.cpp:
// 168-182; RHomogeneousTreeLikelihood.cpp:162-176).  One fixed-size all-gather per
// evaluation moves every rank's record:
//
//   record of rank r = [ block sums 0 .. counts[r)  |  zeros up to cmax  |  underflow flag ]
//                       stride = cmax + 1 doubles,  cmax = max_r counts[r]
//
// (the device writes it: wave_sums_to_blocks fills the block sums and the flag slot, the
// padding is zeroed once at plk_comm_init).  After the gather every rank runs the same
// chain of adds -- rank 0's blocks in block order, then rank 1's, ... -- which is the
// one-process fixed-order sum over all blocks, so the total is bitwise the same for any
// rank count, and ORs the ranks' underflow flags (plk_root_underflow is global).
// Derivative sums (n doubles per rank) are added in rank order the same way.
//
// Pure host code, no HIP: libplk's communicator path calls these, and they are exported
// through the C-ABI (plk_exchange_*) so that the CPU suite drives the same code over gloo
// ranks with uneven block counts (tests/test_distributed_cpu.py).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>

namespace plk {
namespace xchg {

// Record stride (doubles per rank) for the given per-rank block counts; 0 if invalid.
inline int64_t stride(const int64_t* counts, int n_ranks) {
  if (!counts || n_ranks < 1) return 0;
  int64_t cmax = 0;
  for (int r = 0; r < n_ranks; ++r) {
    if (counts[r] < 0) return 0;
    if (counts[r] > cmax) cmax = counts[r];
  }
  return cmax + 1;
}

// This rank's record: its block sums, zero padding, the flag (1.0 set, 0.0 clear).
inline void pack(const double* blocks, int64_t n_blocks, int uflow, int64_t stride, double* rec) {
  for (int64_t i = 0; i < stride - 1; ++i) rec[i] = i < n_blocks ? blocks[i] : 0.0;
  rec[stride - 1] = uflow ? 1.0 : 0.0;
}

// Global lnL (rank order, block order: one chain of adds) and the OR of the flags.
inline double reduce(const double* gathered, const int64_t* counts, int n_ranks, int64_t stride, int* uflow) {
  double s = 0.0;
  int f = 0;
  for (int r = 0; r < n_ranks; ++r) {
    const double* b = gathered + (size_t)r * (size_t)stride;
    for (int64_t i = 0; i < counts[r]; ++i) s += b[i];
    f |= b[stride - 1] != 0.0;
  }
  if (uflow) *uflow = f;
  return s;
}

// v[i] = sum over ranks, in rank order, of gathered[r * n + i].
inline void rank_sums(const double* gathered, int n_ranks, size_t n, double* v) {
  for (size_t i = 0; i < n; ++i) {
    double s = 0.0;
    for (int r = 0; r < n_ranks; ++r) s += gathered[(size_t)r * n + i];
    v[i] = s;
  }
}

}  // namespace xchg
}  // namespace plk
