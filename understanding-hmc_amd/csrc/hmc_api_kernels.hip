// hmc_api_kernels.hip — the non-hot entry points of the C ABI:
//   * batched single leap_frog  (HMC_sampler.leap_frog, samplers.py:831-839)
//   * batched energy E(q,p)     (HMC_sampler.E / K, samplers.py:811-823; V of utils.py:213-218)
//   * Philox blocks and the Philox-mode momentum normals (verification of the in-kernel RNG)
// One thread per row; these run at parity-test sizes, not in the timed path.
#include "hmc_device.hpp"
#include "hmc_internal.hpp"

namespace hmc {


// g_d = (P (q - q0))_d in ascending-j order (dense) or P_dd (q_d - q0_d) (diagonal).
template <bool EXACT>
__device__ __forceinline__ double grad_d(const RowArgs& a, const double* q, int d) {
  if (a.dense) {
    const double* Pr = a.prec + (int64_t)d * a.D;
    double acc = 0.0;
    for (int j = 0; j < a.D; ++j) {
      const double x = q[j] - (a.q0 ? a.q0[j] : 0.0);
      acc = EXACT ? acc + Pr[j] * x : __builtin_fma(Pr[j], x, acc);
    }
    return acc;
  }
  const double x = q[d] - (a.q0 ? a.q0[d] : 0.0);
  return a.prec ? a.prec[d] * x : x;
}

// (inv(cov_p) dVdq(q))_d: the diagonal mass scales g_d; a dense one (minvf) takes the row
// product with every g_j, recomputed on the fly (O(D^3) per row: these are parity-size calls).
template <bool EXACT>
__device__ __forceinline__ double kick_d(const RowArgs& a, const double* q, int d) {
  if (a.minvf) {
    const double* Mr = a.minvf + (int64_t)d * a.D;
    double acc = 0.0;
    for (int j = 0; j < a.D; ++j) {
      const double g = grad_d<EXACT>(a, q, j);
      acc = EXACT ? acc + Mr[j] * g : __builtin_fma(Mr[j], g, acc);
    }
    return acc;
  }
  return a.minv ? a.minv[d] * grad_d<EXACT>(a, q, d) : grad_d<EXACT>(a, q, d);
}

template <bool EXACT>
__global__ __launch_bounds__(256) void k_leapfrog_rows(RowArgs a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.n) return;
  const double* p = a.p + r * a.D;
  const double* q = a.q + r * a.D;
  double* po = a.po + r * a.D;
  double* qo = a.qo + r * a.D;
  for (int d = 0; d < a.D; ++d) {       // p_half = p_old - dt*(Minv dVdq(q_old))/2
    const double dt = a.dtv ? a.dtv[d] : a.dt;
    po[d] = p[d] - (dt * kick_d<EXACT>(a, q, d)) * 0.5;
  }
  for (int d = 0; d < a.D; ++d) {       // q_new = q_old + dt*p_half
    const double dt = a.dtv ? a.dtv[d] : a.dt;
    qo[d] = q[d] + dt * po[d];
  }
  for (int d = 0; d < a.D; ++d) {       // p_new = p_half - dt*(Minv dVdq(q_new))/2
    const double dt = a.dtv ? a.dtv[d] : a.dt;
    po[d] = po[d] - (dt * kick_d<EXACT>(a, qo, d)) * 0.5;
  }
}

__global__ __launch_bounds__(256) void k_energy_rows(RowArgs a) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.n) return;
  const double* p = a.p + r * a.D;
  const double* q = a.q + r * a.D;
  double maha = 0.0, kin = 0.0;
  for (int d = 0; d < a.D; ++d) {
    const double x = q[d] - (a.q0 ? a.q0[d] : 0.0);
    maha += x * grad_d<true>(a, q, d);
    if (a.minvf) {
      const double* Mr = a.minvf + (int64_t)d * a.D;
      double mp = 0.0;
      for (int j = 0; j < a.D; ++j) mp += Mr[j] * p[j];
      kin += p[d] * mp;
    } else {
      kin += p[d] * (a.minv ? a.minv[d] * p[d] : p[d]);
    }
  }
  a.E[r] = 0.5 * (a.logc + maha) + kin / 2.0;
}

__global__ __launch_bounds__(256) void k_philox(uint4 c, uint32_t k0, uint32_t k1, int64_t n, uint32_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 r = philox4x32_10(make_uint4(c.x + (uint32_t)i, c.y, c.z, c.w), k0, k1);
  reinterpret_cast<uint4*>(out)[i] = r;
}

__global__ __launch_bounds__(256) void k_rng_normals(uint32_t k0, uint32_t k1, int64_t chain0, int64_t n,
                                                     int it, int npairs, double* out) {
  __shared__ double tab[kNormalTableDoubles];
  init_normal_tables(tab);
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * npairs) return;
  const int64_t row = i / npairs;
  const int k = (int)(i - row * npairs);
  double z0, z1;   // the wave kernel's (table-driven) momentum transform
  normal_pair_tab(draw_block((uint32_t)k, (uint32_t)it, (uint64_t)(chain0 + row), k0, k1), tab, z0, z1);
  out[2 * i] = z0;
  out[2 * i + 1] = z1;
}

static dim3 rows_grid(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

hipError_t launch_leapfrog_rows(const RowArgs& a, bool exact, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  if (exact) k_leapfrog_rows<true><<<rows_grid(a.n), 256, 0, s>>>(a);
  else k_leapfrog_rows<false><<<rows_grid(a.n), 256, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_energy_rows(const RowArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  k_energy_rows<<<rows_grid(a.n), 256, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_philox(uint4 c, uint32_t k0, uint32_t k1, int64_t n, uint32_t* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  k_philox<<<rows_grid(n), 256, 0, s>>>(c, k0, k1, n, out);
  return hipGetLastError();
}

hipError_t launch_rng_normals(uint32_t k0, uint32_t k1, int64_t chain0, int64_t n, int it, int npairs,
                              double* out, hipStream_t s) {
  if (n == 0 || npairs == 0) return hipSuccess;
  k_rng_normals<<<rows_grid(n * npairs), 256, 0, s>>>(k0, k1, chain0, n, it, npairs, out);
  return hipGetLastError();
}

}  // namespace hmc
