// Operand / result lane layout of v_mfma_f64_4x4x4_4b_f64 on gfx950 (not in the guides).
// For each lane L0 the B operand is one-hot at L0 and A holds (lane id + 1); then
//   D[lane] = sum_k A[i][k] B[k][j] = (A lane id of element (i, k0)) + 1  where B[k0][j] sits
// in lane L0, and 0 elsewhere.  Prints "L0: lane=value ..." for the nonzero D lanes.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(double* out, int l0) {
  const int lane = threadIdx.x;
  const double a = lane + 1.0, b = lane == l0 ? 1.0 : 0.0;
  double d = 0.0;
  d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d, 0, 0, 0);
  out[lane] = d;
}

int main() {
  double* out;
  if (hipMalloc(&out, 64 * sizeof(double)) != hipSuccess) return 1;
  double h[64];
  for (int l0 = 0; l0 < 64; ++l0) {
    probe<<<1, 64>>>(out, l0);
    if (hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("B lane %2d:", l0);
    for (int l = 0; l < 64; ++l)
      if (h[l] != 0.0) printf(" D%d=A%d", l, (int)h[l] - 1);
    printf("\n");
  }
  return 0;
}
