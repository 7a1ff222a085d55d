// hmc_target_ops.hpp — per-coordinate arithmetic of the diagonal-precision MVN target, in the
// reference's operation order (shared by the group and wave-per-chain kernels).
#pragma once
#include "hmc_device.hpp"
#include "hmc_internal.hpp"

namespace hmc {

// Per-dimension constants of the general diagonal target (loaded through L1/L2; tiny).
struct DimConst {
  double q0, prec, minv, dt, hd;
};

template <bool GEN>
__device__ __forceinline__ DimConst dim_const(const RandArgs& a, int d) {
  DimConst c{0.0, 1.0, 1.0, a.dt, a.h};
  if constexpr (GEN) {
    if (a.q0) c.q0 = a.q0[d];
    if (a.prec) c.prec = a.prec[d];
    if (a.minv) c.minv = a.minv[d];
    if (a.dtv) {
      c.dt = a.dtv[d];
      c.hd = c.dt * 0.5;
    }
  }
  return c;
}

// Constants of coordinate slot (pair k, half h); padding slots get neutral constants and never
// touch the per-dimension arrays.
template <bool GEN>
__device__ __forceinline__ DimConst slot_const(const RandArgs& a, int k, int h, bool pair_valid) {
  const int d = 2 * k + h;
  if (GEN && pair_valid && d < a.D) return dim_const<GEN>(a, d);
  return DimConst{0.0, 1.0, 1.0, a.dt, a.h};
}

// Kick term (dt * (Minv * (P (q - q0)))) / 2 in the reference's operation order
// (samplers.py:835/:837 with dVdq of case1-script.py:49).  (dt*x)/2 == (dt/2)*x exactly.
template <bool GEN>
__device__ __forceinline__ double kick(const DimConst& c, double q) {
  if constexpr (GEN) {
    return c.hd * (c.minv * (c.prec * (q - c.q0)));
  } else {
    return c.hd * q;
  }
}

template <bool GEN>
__device__ __forceinline__ void energy_terms(const DimConst& c, double q, double p, double& maha,
                                             double& kin) {
  if constexpr (GEN) {
    const double x = q - c.q0;
    maha += c.prec * x * x;
    kin += p * (c.minv * p);
  } else {
    maha += q * q;
    kin += p * p;
  }
}

}  // namespace hmc
