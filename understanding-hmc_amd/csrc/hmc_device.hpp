// hmc_device.hpp — device-side building blocks shared by the HMC kernels (gfx950).
//
//  * Philox4x32-10 counter-based generator (Salmon et al., SC'11), keyed by
//    (seed) with counter (slot, iteration, global chain id): every draw is a pure
//    function of (seed, chain, iteration, slot), so results do not depend on the
//    launch geometry or on how chains are sharded over GPUs.
//  * fp64 Box–Muller from 53-bit uniforms (momentum draws, replaces
//    np.random.multivariate_normal at samplers.py:829).
//  * Lane-group layout: a chain's D coordinates live in one "group" of LPC
//    consecutive lanes of a wave64; lane s of the group owns coordinate pairs
//    k = s + LPC*j (j < K).  CPW = 64/LPC chains share a wave.  Group sums use
//    ds_bpermute shuffles (no LDS, no barriers).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hmc {

constexpr int kWave = 64;
constexpr uint32_t kDrawSlot = 0x80000000u;  // counter.x for non-momentum draws (L, u, NUTS draws)

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ uint4 draw_block(uint32_t slot, uint32_t iter, uint64_t gchain, uint32_t k0,
                                            uint32_t k1) {
  return philox4x32_10(make_uint4(slot, iter, (uint32_t)gchain, (uint32_t)(gchain >> 32)), k0, k1);
}

// 53-bit uniform in [0, 1) from two words.
__device__ __forceinline__ double u53(uint32_t lo, uint32_t hi) {
  return (double)((((uint64_t)hi) << 21) | (lo >> 11)) * 0x1p-53;
}
// 53-bit uniform in (0, 1].
__device__ __forceinline__ double u53_open0(uint32_t lo, uint32_t hi) {
  return ((double)((((uint64_t)hi) << 21) | (lo >> 11)) + 1.0) * 0x1p-53;
}

// Two independent N(0,1) from one Philox block (fp64 Box–Muller).
__device__ __forceinline__ void normal_pair(uint4 r, double& z0, double& z1) {
  const double u1 = u53_open0(r.x, r.y);
  const double u2 = u53(r.z, r.w);
  const double rad = sqrt(-2.0 * log(u1));
  double s, c;
  sincospi(2.0 * u2, &s, &c);
  z0 = rad * c;
  z1 = rad * s;
}

// Uniform integer in [lo, hi) from one word (multiply-shift; bias <= (hi-lo)/2^32).
__device__ __forceinline__ int uniform_int(uint32_t w, int lo, int hi) {
  return lo + (int)(((uint64_t)w * (uint32_t)(hi - lo)) >> 32);
}

// Sum over the LPC lanes of a group; every lane of the group receives the total.
// `s` = lane index inside the group, `base` = wave lane of the group's first lane.
__device__ __forceinline__ double group_sum(double v, int s, int lpc, int base) {
  for (int off = 1; off < lpc; off <<= 1) {
    const double o = __shfl_down(v, off, kWave);
    if (s + off < lpc) v += o;
  }
  return __shfl(v, base, kWave);
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Load / store coordinate pair k of a row (16-B vector access when D is even).
__device__ __forceinline__ void load_pair(const double* __restrict__ row, int k, bool even, bool v1,
                                          double& a, double& b) {
  if (even) {
    const double2 x = *reinterpret_cast<const double2*>(row + 2 * k);
    a = x.x;
    b = x.y;
  } else {
    a = row[2 * k];
    b = v1 ? row[2 * k + 1] : 0.0;
  }
}

__device__ __forceinline__ void store_pair(double* __restrict__ row, int k, bool even, bool v1, double a,
                                           double b) {
  if (even) {
    *reinterpret_cast<double2*>(row + 2 * k) = make_double2(a, b);
  } else {
    row[2 * k] = a;
    if (v1) row[2 * k + 1] = b;
  }
}

}  // namespace hmc
