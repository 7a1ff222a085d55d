// Microbenchmark: issue cost (cycles per wave-instruction) of the instruction mixes the RNG, the
// integrator and the reductions use, 8 waves per SIMD, 4 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>

#define BODY_LOOP(ASM)                                                                      \
  for (int k = 0; k < n; ++k) {                                                             \
    ASM                                                                                     \
  }

__global__ void k_mad64(unsigned* out, int n) {
  unsigned a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
  unsigned long long r0 = a, r1 = b, r2 = c, r3 = d;
  BODY_LOOP(asm volatile(
      "v_mad_u64_u32 %0, s[0:1], %4, %8, 0\n v_mad_u64_u32 %1, s[0:1], %5, %8, 0\n"
      "v_mad_u64_u32 %2, s[0:1], %6, %8, 0\n v_mad_u64_u32 %3, s[0:1], %7, %8, 0\n"
      : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3)
      : "v"(a), "v"(b), "v"(c), "v"(d), "s"(0xD2511F53u)
      : "s0", "s1");)
  out[blockIdx.x * blockDim.x + threadIdx.x] = (unsigned)(r0 + r1 + r2 + r3);
}
__global__ void k_mulhi(unsigned* out, int n) {
  unsigned a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
  BODY_LOOP(asm volatile(
      "v_mul_hi_u32 %0, %0, %4\n v_mul_hi_u32 %1, %1, %4\n v_mul_hi_u32 %2, %2, %4\n v_mul_hi_u32 %3, %3, %4\n"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
      : "s"(0xD2511F53u));)
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}
__global__ void k_mullo(unsigned* out, int n) {
  unsigned a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
  BODY_LOOP(asm volatile(
      "v_mul_lo_u32 %0, %0, %4\n v_mul_lo_u32 %1, %1, %4\n v_mul_lo_u32 %2, %2, %4\n v_mul_lo_u32 %3, %3, %4\n"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
      : "s"(0xD2511F53u));)
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}
__global__ void k_xor(unsigned* out, int n) {
  unsigned a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
  BODY_LOOP(asm volatile(
      "v_xor_b32 %0, %4, %0\n v_xor_b32 %1, %4, %1\n v_xor_b32 %2, %4, %2\n v_xor_b32 %3, %4, %3\n"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
      : "s"(0xD2511F53u));)
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}
__global__ void k_fma64(double* out, int n) {
  double a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
  BODY_LOOP(asm volatile(
      "v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4\n"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d)
      : "v"(0.5));)
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}
__global__ void k_dppmov(unsigned* out, int n) {
  unsigned a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
  BODY_LOOP(asm volatile(
      "v_mov_b32_dpp %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_mov_b32_dpp %2, %3 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_mov_b32_dpp %1, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      "v_mov_b32_dpp %3, %2 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}
__global__ void k_cvt(double* out, int n) {
  double a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
  unsigned u = threadIdx.x;
  BODY_LOOP(asm volatile(
      "v_cvt_f64_u32 %0, %4\n v_cvt_f64_u32 %1, %4\n v_cvt_f64_u32 %2, %4\n v_cvt_f64_u32 %3, %4\n"
      : "=v"(a), "=v"(b), "=v"(c), "=v"(d)
      : "v"(u));)
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}
__global__ void k_rcp64(double* out, int n) {
  double a = threadIdx.x + 1.0, b = a + 1, c = a + 2, d = a + 3;
  BODY_LOOP(asm volatile(
      "v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3\n"
      : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c + d;
}

template <typename K, typename T>
float timeit(K k, T* out, int n, dim3 grid) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<<<grid, 256>>>(out, n);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  k<<<grid, 256>>>(out, n);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  void* out;
  hipMalloc(&out, 1 << 26);
  const int n = 1 << 14;
  const int wps = 8;   // waves per SIMD
  dim3 grid(256 * wps);
  const double instr_per_wave = 4.0 * n;
  const double waves_per_simd = wps;
#define RUN(K, T)                                                                            \
  {                                                                                          \
    float ms = timeit(K, (T*)out, n, grid);                                                  \
    printf("%-10s %.3f ms  %.2f cyc/wave-instr @2.4GHz\n", #K, ms,                            \
           ms * 1e-3 * 2.4e9 / (instr_per_wave * waves_per_simd));                           \
  }
  RUN(k_mad64, unsigned)
  RUN(k_mulhi, unsigned)
  RUN(k_mullo, unsigned)
  RUN(k_xor, unsigned)
  RUN(k_fma64, double)
  RUN(k_dppmov, unsigned)
  RUN(k_cvt, double)
  RUN(k_rcp64, double)
  return 0;
}
