// Bisect why one leapfrog step costs ~6K SIMD-cycles in k_wave_iters (diagnostic microbenchmark).
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../understanding-hmc_amd/csrc/hmc_device.hpp"
using namespace hmc;

struct Args { double* out; int n_chains; int iters; int L; double h, dt; uint32_t k0, k1; int cap; };

template <bool RNG, bool RED, bool STORE, bool CAPBR, bool READL>
__global__ __launch_bounds__(256) void mimic(Args a) {
  const int lane = threadIdx.x & 63;
  const int c = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + threadIdx.x / 64);
  if (c >= a.n_chains) return;
  double q0 = lane * 1e-3, q1 = lane * 2e-3, p0 = 0.3, p1 = -0.2;
  double E = 0;
  int drawL = a.L + (lane & 0);
  const bool cap = (c == 0) && a.cap;
  for (int it = 0; it < a.iters; ++it) {
    if (RNG) normal_pair(draw_block(lane, it, c, a.k0, a.k1), p0, p1);
    if (RED) E += wave_sum_dpp(q0 * q0 + p0 * p0);
    int L = READL ? __builtin_amdgcn_readlane(drawL, it & 63) : a.L;
    L = __builtin_amdgcn_readfirstlane(L);
    for (int l = 0; l < L; ++l) {
      double ph0 = __builtin_fma(-a.h, q0, p0), ph1 = __builtin_fma(-a.h, q1, p1);
      q0 = __builtin_fma(a.dt, ph0, q0); q1 = __builtin_fma(a.dt, ph1, q1);
      if (CAPBR && cap && lane == 0) a.out[l] = q0;
      p0 = __builtin_fma(-a.h, q0, ph0); p1 = __builtin_fma(-a.h, q1, ph1);
    }
    if (RED) E += wave_sum_dpp(q1 * q1 + p1 * p1);
    if (STORE) *reinterpret_cast<double2*>(a.out + ((int64_t)c * a.iters + it) * 128 + 2 * lane) = make_double2(q0, q1);
  }
  if (lane == 0) a.out[(int64_t)a.n_chains * a.iters * 128 + c] = E + q0 + p1;
}

template <typename F> float timeit(F f) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  f(); (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0); f(); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1); return ms;
}

#define RUN(name, ...) do { \
  for (int L : {0, 1, 12}) { Args b = a; b.L = L; \
    float t = timeit([&] { mimic<__VA_ARGS__><<<grid, 256>>>(b); }); \
    printf("%-28s L=%2d %.3f ms\n", name, L, t); } } while (0)

int main() {
  Args a{};
  a.n_chains = 32768; a.iters = 10; a.h = 0.05; a.dt = 0.1; a.k0 = 1; a.k1 = 2; a.cap = 0;
  (void)hipMalloc(&a.out, ((size_t)a.n_chains * a.iters * 128 + a.n_chains + 64) * 8);
  dim3 grid((a.n_chains + 3) / 4);
  RUN("full", true, true, true, true, true);
  RUN("no rng", false, true, true, true, true);
  RUN("no reductions", true, false, true, true, true);
  RUN("no store", true, true, false, true, true);
  RUN("no cap branch", true, true, true, false, true);
  RUN("no readlane L", true, true, true, true, false);
  RUN("loop only", false, false, false, false, false);
  return 0;
}
