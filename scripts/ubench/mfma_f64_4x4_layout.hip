// Lane layout probe of v_mfma_f64_4x4x4f64 (4 blocks) on gfx950.  For each source lane s, A is
// one-hot at lane s and B holds 1000 * (lane + 1); output lane o then reads
// D = sum_k A[i][k] B[k][j] = B value of the lane that pairs with lane s, or 0.
// Prints, per source lane s, the output lanes that received a non-zero value and from which
// B lane: enough to fix the (block, row, k) / (block, k, col) / (block, row, col) lane maps.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(double* out) {
  const int l = threadIdx.x;
  for (int s = 0; s < 64; ++s) {
    const double a = l == s ? 1.0 : 0.0;
    const double b = 1000.0 * (l + 1);
    const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    out[s * 64 + l] = d;
  }
}

int main() {
  double* d;
  if (hipMalloc(&d, 64 * 64 * sizeof(double)) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  double h[64 * 64];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int s = 0; s < 64; ++s) {
    printf("A lane %2d ->", s);
    for (int o = 0; o < 64; ++o)
      if (h[s * 64 + o] != 0.0) printf(" out%d<-B%d", o, (int)(h[s * 64 + o] / 1000.0) - 1);
    printf("\n");
  }
  (void)hipFree(d);
  return 0;
}
