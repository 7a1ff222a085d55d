// mfma_f64.hip — issue rate of v_mfma_f64_16x16x4_f64 on gfx950 (pins the FP64 matrix peak
// the dense kernels are priced against).  Each wave runs NACC independent accumulator chains
// of ITERS MFMAs; waves per SIMD set by the block size (one block per CU).
//   hipcc --offload-arch=gfx950 -O3 mfma_f64.hip -o mfma_f64 && ./mfma_f64
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void k_mfma(double* out, int iters, double a0, double b0) {
  d4 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
  double a = a0 + threadIdx.x * 1e-9, b = b0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
void run(int cus, int waves_per_cu, int iters) {
  double* out;
  (void)hipMalloc(&out, (size_t)cus * waves_per_cu * 64 * sizeof(double));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_mfma<NACC><<<cus, 64 * waves_per_cu>>>(out, iters, 1.0, 1e-3);
  (void)hipEventRecord(e0);
  k_mfma<NACC><<<cus, 64 * waves_per_cu>>>(out, iters, 1.0, 1e-3);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double n_mfma = (double)cus * waves_per_cu * iters * NACC;
  const double flops = n_mfma * 16 * 16 * 4 * 2;
  printf("NACC=%d waves/CU=%2d: %.3f ms, %.1f TFLOP/s, %.2f ns per MFMA per SIMD\n", NACC, waves_per_cu, ms,
         flops / (ms * 1e-3) / 1e12, (ms * 1e6) / (n_mfma / (cus * 4.0)));
  (void)hipFree(out);
}

int main() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  printf("CUs: %d\n", cus);
  const int iters = 20000;
  for (int w : {4, 8, 16}) {
    run<1>(cus, w, iters);
    run<4>(cus, w, iters);
    run<7>(cus, w, iters);
  }
  return 0;
}
