// Micro-test for the round-4 wrong-result (a fresh shard handle's P(t) kernel read other data
// than the host had written into its request staging, device memory written over the BAR).
// Hypothesis: dirty L2 lines of a freed device allocation, written by an earlier kernel, stay
// in L2 after the allocation is freed; the pages come back as the staging of a new handle, the
// host writes the request into HBM over the BAR (bypassing L2), and a later eviction writes the
// old lines back over it -- or a read hits the stale lines.
//
// Per trial: a coarse-grained buffer X is filled with OLD by a kernel (lines left in L2),
// freed; a host-writable buffer F of the same size is allocated (fine-grained or uncached);
// the host writes NEW into F through its pointer; optionally an L2-thrashing kernel runs; a
// kernel copies F into a result buffer; the host counts words that are not NEW.
// Modes: 0 read right away, 1 thrash L2 first, 2 flush (system-scope fence in every CU's
// workgroup) after the free and before the host write, then thrash, then read.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));                       \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

__global__ void fill(unsigned long long* p, size_t n, unsigned long long v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void copy(const unsigned long long* src, unsigned long long* dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
// reads and writes a large buffer: evicts whatever else the L2s hold
__global__ void thrash(double* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = p[i] * 1.0000001 + 1.0;
}
// system-scope release + acquire in every workgroup: write back and invalidate the L2s
__global__ void flush_l2() {
  __atomic_thread_fence(__ATOMIC_SEQ_CST);  // (HIP default scope: system)
}

int main() {
  const unsigned long long OLD = 0x0dd0dd0dd0dd0dd0ull, NEW = 0x1234567812345678ull;
  const size_t big = (size_t)1 << 28;  // 256 MB thrash buffer (L2 4 MB per XCD, MALL 256 MB)
  double* thr = nullptr;
  CK(hipMalloc(&thr, big));
  CK(hipMemset(thr, 0, big));
  unsigned long long* out = nullptr;
  const size_t max_n = (size_t)1 << 20;
  CK(hipMalloc(&out, max_n * 8));
  std::vector<unsigned long long> h(max_n);
  const unsigned flags[2] = {hipDeviceMallocFinegrained, hipDeviceMallocUncached};
  for (int fl = 0; fl < 2; ++fl)
    for (int mode = 0; mode < 3; ++mode) {
      long long bad = 0, reused = 0, trials = 0;
      for (int t = 0; t < 24; ++t) {
        const size_t n = ((size_t)4096 << (t % 6)) + (t / 6) * 512;  // 32 KB .. 1 MB
        unsigned long long* x = nullptr;
        CK(hipMalloc(&x, n * 8));
        fill<<<256, 256>>>(x, n, OLD);
        CK(hipDeviceSynchronize());
        CK(hipFree(x));
        if (mode == 2) {
          flush_l2<<<2048, 64>>>();
          CK(hipDeviceSynchronize());
        }
        unsigned long long* f = nullptr;
        CK(hipExtMallocWithFlags((void**)&f, n * 8, flags[fl]));
        reused += f == x;
        for (size_t i = 0; i < n; ++i) f[i] = NEW;  // host stores over the BAR
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        if (mode >= 1) {
          thrash<<<2048, 256>>>(thr, big / 8);
          CK(hipDeviceSynchronize());
        }
        copy<<<256, 256>>>(f, out, n);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), out, n * 8, hipMemcpyDeviceToHost));
        long long b = 0;
        for (size_t i = 0; i < n; ++i) b += h[i] != NEW;
        // also what the host reads back through its pointer
        long long hb = 0;
        for (size_t i = 0; i < n; ++i) hb += f[i] != NEW;
        bad += b + hb;
        ++trials;
        CK(hipFree(f));
      }
      std::printf("%s mode %d (%s): %lld trials, %lld same address as the freed buffer, %lld words not NEW\n",
                  fl == 0 ? "fine-grained" : "uncached", mode,
                  mode == 0 ? "read at once" : mode == 1 ? "L2 thrashed before the read" : "L2 flushed after free",
                  trials, reused, bad);
    }
  // Bulk reuse: the round-4 staging was a small fine-grained allocation made after many other
  // buffers were freed.  Free 64 coarse 256 KB buffers a kernel filled with OLD, then make 512
  // small (16 KB) fine-grained / uncached allocations, write NEW into each from the host,
  // thrash the L2s (or not), and read them all back in one kernel per buffer.
  // (mode 2: the fix -- a system-scope release in workgroups on every XCD writes the freed
  // buffers' dirty lines back before the host writes, then the L2s are thrashed)
  for (int fl = 0; fl < 2; ++fl)
    for (int thr_first = 0; thr_first < 3; ++thr_first) {
      const size_t big_n = 32768, small_n = 2048;  // 256 KB, 16 KB
      std::vector<unsigned long long*> xs(64), fs(512);
      for (auto& x : xs) {
        CK(hipMalloc(&x, big_n * 8));
        fill<<<64, 256>>>(x, big_n, OLD);
      }
      CK(hipDeviceSynchronize());
      for (auto& x : xs) CK(hipFree(x));
      if (thr_first == 2) {
        flush_l2<<<2048, 64>>>();
        CK(hipDeviceSynchronize());
      }
      for (auto& f : fs) {
        CK(hipExtMallocWithFlags((void**)&f, small_n * 8, flags[fl]));
        for (size_t i = 0; i < small_n; ++i) f[i] = NEW;
      }
      __atomic_thread_fence(__ATOMIC_SEQ_CST);
      if (thr_first) {
        thrash<<<2048, 256>>>(thr, big / 8);
        CK(hipDeviceSynchronize());
      }
      long long bad = 0, overlap = 0;
      for (auto& f : fs) {
        copy<<<8, 256>>>(f, out, small_n);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h.data(), out, small_n * 8, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < small_n; ++i) bad += h[i] != NEW;
        for (auto& x : xs) overlap += (char*)f >= (char*)x && (char*)f < (char*)x + big_n * 8;
      }
      std::printf("bulk %s, %s: 512 x 16 KB after 64 x 256 KB freed, %lld inside a freed range, %lld words not NEW\n",
                  fl == 0 ? "fine-grained" : "uncached",
                  thr_first == 2 ? "L2 written back after the free, then thrashed" : thr_first ? "L2 thrashed" : "read at once",
                  overlap, bad);
      for (auto& f : fs) CK(hipFree(f));
    }
  return 0;
}
