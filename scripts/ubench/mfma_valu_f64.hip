// mfma_valu_f64.hip — does FP64 VALU work of one wave overlap the f64 MFMAs of another wave on the
// same SIMD (gfx950)?  Decides whether a NUTS step can hide its VALU/memory phases behind a partner
// wave's gradient (two waves per SIMD) or whether they serialise on the FP64 hardware.
//   hipcc --offload-arch=gfx950 -O3 mfma_valu_f64.hip -o mfma_valu_f64 && ./mfma_valu_f64
// One 512-thread block per CU: waves 0-3 (one per SIMD) run f64 MFMA chains, waves 4-7 (the
// partners on the same SIMDs) run f64 FMA chains, a dependent global-load chain, or nothing.
// Mode 'same' runs both streams interleaved inside ONE wave per SIMD (256-thread blocks).
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef double d4 __attribute__((ext_vector_type(4)));

enum { M_MFMA = 0, M_VALU = 1, M_BOTH = 2, M_SAME = 3, M_LOADS = 4, M_MFMA_LOADS = 5, M_VALU_ALONE8 = 6 };

__device__ __forceinline__ void mfma_part(int iters, double a, double b, d4 (&acc)[4]) {
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
}

__device__ __forceinline__ void valu_part(int iters, double (&x)[8], double y) {
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = __builtin_fma(x[i], y, 1e-7);
  }
}

__global__ __launch_bounds__(512) void k_mix(int mode, int it_m, int it_v, const unsigned* __restrict__ chain,
                                             int it_l, double* out, unsigned long long* cyc) {
  const int w = threadIdx.x / 64;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  double s = 0.0;
  d4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
  double x[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3 + i;
  const double a = 1.0 + threadIdx.x * 1e-9, b = 0.999;
  bool mf = false, vl = false, ld = false;
  if (mode == M_MFMA) mf = w < 4;
  if (mode == M_VALU) vl = w >= 4;
  if (mode == M_VALU_ALONE8) vl = true;
  if (mode == M_BOTH) { mf = w < 4; vl = w >= 4; }
  if (mode == M_LOADS) ld = w >= 4;
  if (mode == M_MFMA_LOADS) { mf = w < 4; ld = w >= 4; }
  if (mode == M_SAME) {
    // one wave per SIMD: blocks of 256; interleave 1 MFMA iteration (4 MFMAs) with the VALU share
    const int ratio = it_v / it_m;
    for (int it = 0; it < it_m; ++it) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
      for (int r = 0; r < ratio; ++r) {
#pragma unroll
        for (int i = 0; i < 8; ++i) x[i] = __builtin_fma(x[i], b, 1e-7);
      }
    }
  } else {
    if (mf) mfma_part(it_m, a, b, acc);
    if (vl) valu_part(it_v, x, b);
    if (ld) {
      unsigned j = threadIdx.x & 63;
      for (int it = 0; it < it_l; ++it) j = __builtin_nontemporal_load(chain + j);
      s += j;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
#pragma unroll
  for (int i = 0; i < 8; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

int main() {
  int dev = 0, cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int it_m = 4000, it_v = 32000, it_l = 2000;
  double* out;
  unsigned long long* cyc;
  unsigned* chain;
  const size_t nchain = 1 << 26;   // 256 MB pointer chase table (beyond L2)
  (void)hipMalloc(&out, (size_t)cus * 512 * sizeof(double));
  (void)hipMalloc(&cyc, (size_t)cus * 8 * sizeof(unsigned long long));
  (void)hipMalloc(&chain, nchain * sizeof(unsigned));
  {
    unsigned* h = (unsigned*)malloc(nchain * sizeof(unsigned));
    unsigned long long st = 12345;
    for (size_t i = 0; i < nchain; ++i) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      h[i] = (unsigned)((st >> 20) % nchain);
    }
    (void)hipMemcpy(chain, h, nchain * sizeof(unsigned), hipMemcpyHostToDevice);
    free(h);
  }
  const char* names[] = {"mfma only (w0-3)", "valu only (w4-7)", "mfma w0-3 + valu w4-7", "same wave mfma+valu",
                         "loads only (w4-7)", "mfma w0-3 + loads w4-7", "valu all 8 waves"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  unsigned long long* hc = (unsigned long long*)malloc((size_t)cus * 8 * sizeof(unsigned long long));
  for (int mode = 0; mode <= 6; ++mode) {
    const int threads = mode == M_SAME ? 256 : 512;
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipMemset(cyc, 0, (size_t)cus * 8 * sizeof(unsigned long long));
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k_mix, dim3(cus), dim3(threads), 0, 0, mode, it_m, it_v, chain, it_l, out, cyc);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      (void)hipMemcpy(hc, cyc, (size_t)cus * 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
      double lo = 0, hi = 0;
      int nlo = 0, nhi = 0;
      for (int b = 0; b < cus; ++b)
        for (int w = 0; w < 8; ++w) {
          if (!hc[b * 8 + w]) continue;
          if (w < 4) { lo += hc[b * 8 + w]; ++nlo; } else { hi += hc[b * 8 + w]; ++nhi; }
        }
      if (rep == 1)
        printf("%-28s  %8.3f ms   waves0-3 %10.0f clk   waves4-7 %10.0f clk   (mfma %d x4, valu %d x8 fma, loads %d)\n",
               names[mode], ms, nlo ? lo / nlo : 0.0, nhi ? hi / nhi : 0.0, it_m, it_v, it_l);
    }
  }
  return 0;
}
