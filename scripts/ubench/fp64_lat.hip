// Microbenchmark: fp64 FMA dependent-chain latency and throughput on gfx950 (measure, don't guess).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int ILP>
__global__ void chain(double* out, int n, double a, double b) {
  double x[ILP];
#pragma unroll
  for (int i = 0; i < ILP; ++i) x[i] = threadIdx.x * 1e-3 + i;
  for (int k = 0; k < n; ++k) {
#pragma unroll
    for (int i = 0; i < ILP; ++i) x[i] = __builtin_fma(x[i], a, b);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < ILP; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// dependent chain with a data-dependent loop trip count per lane (divergent loop like the leapfrog)
__global__ void chain_divloop(double* out, const int* trips, int outer, double a, double b) {
  double x = threadIdx.x * 1e-3, y = x + 1;
  int L = trips[threadIdx.x & 63];
  for (int o = 0; o < outer; ++o) {
    for (int l = 0; l < L; ++l) {
      x = __builtin_fma(-a, y, x);
      y = __builtin_fma(b, x, y);
      x = __builtin_fma(-a, y, x);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x + y;
}

template <typename F>
float timeit(F f) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  f();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  double* out; hipMalloc(&out, 1 << 26);
  int* trips; hipMalloc(&trips, 64 * sizeof(int));
  int h[64]; for (int i = 0; i < 64; ++i) h[i] = 12; hipMemcpy(trips, h, sizeof(h), hipMemcpyHostToDevice);
  const int n = 1 << 16;
  for (int wps : {1, 2, 4, 8}) {   // waves per SIMD: blocks of 256 threads, 256*wps blocks
    dim3 grid(256 * wps);
    float t1 = timeit([&] { chain<1><<<grid, 256>>>(out, n, 0.999999, 1e-7); });
    float t4 = timeit([&] { chain<4><<<grid, 256>>>(out, n, 0.999999, 1e-7); });
    double fmas1 = (double)n * 1;      // per lane
    double fmas4 = (double)n * 4;
    // cycles per FMA per wave at 2.4 GHz (upper bound clock)
    printf("waves/SIMD=%d  ILP1: %.2f ms -> %.1f cyc/FMA/wave   ILP4: %.2f ms -> %.1f cyc/FMA/wave ; chip %.2f TFLOP/s(ILP4)\n",
           wps, t1, t1 * 1e-3 * 2.4e9 / fmas1, t4, t4 * 1e-3 * 2.4e9 / fmas4,
           2.0 * fmas4 * 256 * wps * 256 / (t4 * 1e-3) / 1e12);
  }
  for (int wps : {1, 6}) {
    dim3 grid(256 * wps);
    float t = timeit([&] { chain_divloop<<<grid, 256>>>(out, trips, 4096, 0.05, 0.1); });
    printf("divloop waves/SIMD=%d: %.2f ms -> %.1f cyc per step per wave\n", wps, t, t * 1e-3 * 2.4e9 / (4096.0 * 12));
  }
  return 0;
}
